// hg_encode.hip — device-resident SSTable encode (record packing) for gfx950.
//
// Replaces InternalPair::serialize / serialize_flatten (reference
// src/format.rs:23-42): every record becomes
//     [u64 LE klen][u64 LE vlen][key][value]      (vlen == 0: no value bytes)
// concatenated in the given order, and Index::new's second encode that only
// learns block positions/lengths (src/sstable/index.rs:55-67).
//
// Three launches on one stream:
//  1. encode_sums_kernel: one 256-thread workgroup per tile of 256 records
//     sums 16 + klen + vlen (reads only the descriptors) -> tile sums, and
//     adds them into per-group sums (16 tiles per group).
//  2. encode_bases_kernel: one workgroup scans the group sums -> group output
//     offsets, and writes the call's result (total bytes, capacity check).
//     (A single-pass decoupled look-back over tile statuses measured 0.21 ms
//     slower on BASELINE cfg 3: every tile's copy waited for it.)
//  3. encode_kernel: a workgroup per tile loads its descriptors, scans sizes
//     and 16-byte piece counts in LDS, adds the preceding tile sums of its
//     group to the group offset, and copies consecutive 16-byte output pieces
//     per lane (coalesced 1 KiB per wave instruction; unaligned 16-byte loads
//     and stores are native on gfx950).  Piece 0 of a record is its header,
//     synthesised in registers; body pieces are 16-byte loads from the key or
//     value source; a piece straddling key|value or ending mid-record is
//     assembled in registers from two in-bounds 16-byte windows and stored as
//     16 B or 8/4/2/1-byte parts, so no byte outside a record's own output
//     range is ever stored.  The loop is software-pipelined (loads of step i+1
//     issued before the stores of step i).  Tiles of equal-size records
//     resolve a piece's record by division instead of a search.
// Block index entries come from a fourth, tiny kernel over record offsets.
#include "hg_device.hpp"

namespace hgk {

#ifndef HG_ENC_RPT
#define HG_ENC_RPT 1
#endif
constexpr uint32_t ENC_THREADS = 256;
constexpr uint32_t ENC_RPT = HG_ENC_RPT;                 // records per thread
constexpr uint32_t ENC_TILE = ENC_THREADS * ENC_RPT;     // records per tile (workgroup)
#ifndef HG_ENC_U
#define HG_ENC_U 6  // cfg 3: 6 -> 1.12 ms, 4 -> 1.145 (a shuffled mixed-size pair order prefers 4: 0.66 vs 0.72 ms)
#endif
constexpr uint32_t ENC_U = HG_ENC_U;  // 16-byte pieces in flight per lane
#ifndef HG_ENC_U_GATHER
#define HG_ENC_U_GATHER 1
#endif
constexpr uint32_t ENC_U_GATHER = HG_ENC_U_GATHER;  // the same for gathered pairs
#ifndef HG_ENC_PRE
#define HG_ENC_PRE 1
#endif
constexpr uint32_t ENC_PRE = HG_ENC_PRE;  // pieces per lane loaded before the look-back
#ifndef HG_ENC_NT
#define HG_ENC_NT 1
#endif
typedef uint32_t enc_u32x4 __attribute__((ext_vector_type(4)));
// Output bytes are written once: nontemporal stores (HG_ENC_NT=0: default
// policy, for A/B runs).  Arena bytes are read once when the pairs walk the
// arena in order (a table's own records): nontemporal loads.  Pairs that
// gather records from several tables (a compaction's merged order) read each
// source line in two or more visits (a 132-byte record spans two lines, the
// neighbouring records of its table come a few pieces later): default-policy
// loads keep those lines in L2 (cfg 5 leg: encode 552 -> 420 us).
template <bool NTL>
__device__ __forceinline__ uint4 ld_stream16(const uint8_t* p) {
    if (HG_ENC_NT && NTL) {
        const enc_u32x4 x = __builtin_nontemporal_load(reinterpret_cast<const enc_u32x4*>(p));
        return make_uint4(x.x, x.y, x.z, x.w);
    }
    return *reinterpret_cast<const uint4*>(p);
}
__device__ __forceinline__ void st_stream16(uint8_t* p, uint4 v) {
    if (HG_ENC_NT) {
        enc_u32x4 x = {v.x, v.y, v.z, v.w};
        __builtin_nontemporal_store(x, reinterpret_cast<enc_u32x4*>(p));
    } else {
        *reinterpret_cast<uint4*>(p) = v;
    }
}
constexpr uint32_t ENC_NW = ENC_THREADS / 64;
constexpr uint32_t ENC_GROUP = 16;  // tiles per group sum (two-level output offsets)

struct EncodeArgs {
    const uint8_t* arena;
    const hg_pair* pairs;
    uint64_t n;
    uint8_t* out;
    uint64_t cap;
    uint64_t* rec_off;  // may be null
    uint64_t rec_base;  // added to every record offset (chunked host encode)
    hg_encode_result* result;
    const uint64_t* tile_sum;    // output bytes of every tile (encode_sums_kernel)
    const uint64_t* group_base;  // output offset of every ENC_GROUP tiles (encode_bases_kernel)
    const uint64_t* n_dev;       // optional: records = min(n, *n_dev) (a merge's device count)
};

__device__ __forceinline__ uint64_t enc_count(uint64_t n, const uint64_t* n_dev) {
    return n_dev ? min(n, *n_dev) : n;
}

struct EncodeSmem {
    uint64_t key_off[ENC_TILE], val_off[ENC_TILE], off[ENC_TILE + 1];
    uint32_t klen[ENC_TILE], vlen[ENC_TILE], piece[ENC_TILE + 1];
    uint32_t scan_tmp[ENC_NW];
    uint64_t scan_tmp64[ENC_NW];
    uint64_t tile_base;
    uint64_t wsize[ENC_NW];  // per wave: the (klen, vlen) all its records share
    uint32_t wflag[ENC_NW];  // per wave: 0 no records, 1 all share wsize, 2 mixed
};

__device__ __forceinline__ uint64_t block_excl_scan64(uint64_t v, uint64_t* s_tmp,
                                                      uint64_t& total) {
    const uint32_t lane = threadIdx.x & 63u, wid = threadIdx.x >> 6;
    uint64_t x = v;
#pragma unroll
    for (uint32_t d = 1; d < 64; d <<= 1) {
        uint64_t y = __shfl_up(x, d, 64);
        if (lane >= d) x += y;
    }
    if (lane == 63) s_tmp[wid] = x;
    __syncthreads();
    uint64_t pre = 0, tot = 0;
#pragma unroll
    for (uint32_t w = 0; w < ENC_NW; ++w) {
        uint64_t t = s_tmp[w];
        pre += (w < wid) ? t : 0ull;
        tot += t;
    }
    __syncthreads();
    total = tot;
    return pre + x - v;
}

__device__ __forceinline__ void store_bytes(uint8_t* dst, const uint8_t* src_k, uint32_t klen,
                                            const uint8_t* src_v, uint64_t body0,
                                            uint32_t nbytes, uint64_t lim) {
    // Bytes [body0, body0 + nbytes) of key||value to dst[0..nbytes), skipping
    // anything at or beyond `lim` (capacity).
    for (uint32_t i = 0; i < nbytes; ++i) {
        if ((uint64_t)i >= lim) break;
        const uint64_t b = body0 + i;
        dst[i] = b < klen ? src_k[b] : src_v[b - klen];
    }
}

// Bytes [off, ...) of a source region of len >= 16 bytes, shifted to byte 0,
// read through the 16-byte window [min(off, len - 16), +16) -- never outside
// the region.  Callers use only the bytes that lie in the region.
__device__ __forceinline__ unsigned __int128 window_bytes(const uint8_t* base, uint64_t len,
                                                          uint64_t off) {
    const uint64_t w = min(off, len - 16);
    const uint4 x = *reinterpret_cast<const uint4*>(base + w);
    unsigned __int128 v = ((unsigned __int128)(((uint64_t)x.w << 32) | x.z) << 64) |
                          (((uint64_t)x.y << 32) | x.x);
    return v >> (8 * (uint32_t)(off - w));
}

// The low n (<= 16) bytes of v to dst: one 16-byte store, or 8/4/2/1-byte parts.
__device__ __forceinline__ void store_part(uint8_t* dst, unsigned __int128 v, uint32_t n) {
    if (n >= 16) {
        *reinterpret_cast<uint4*>(dst) =
            make_uint4((uint32_t)v, (uint32_t)(v >> 32), (uint32_t)(v >> 64), (uint32_t)(v >> 96));
        return;
    }
    uint32_t o = 0;
    if (n & 8) {
        *reinterpret_cast<uint64_t*>(dst) = (uint64_t)v;
        o = 8;
    }
    if (n & 4) {
        *reinterpret_cast<uint32_t*>(dst + o) = (uint32_t)(v >> (8 * o));
        o += 4;
    }
    if (n & 2) {
        *reinterpret_cast<uint16_t*>(dst + o) = (uint16_t)(v >> (8 * o));
        o += 2;
    }
    if (n & 1) dst[o] = (uint8_t)(v >> (8 * o));
}

// One 16-byte output piece of the tile, resolved from the LDS tables.
struct EncPiece {
    const uint8_t* src;  // kind 2: 16 contiguous source bytes
    uint64_t lo;         // output offset within the tile
    uint32_t kind;       // 0 none, 1 header, 2 16-byte copy, 3 assembled (straddle / tail)
    uint32_t rec;        // record within the tile
};

// A tile whose records all share one (klen, vlen) -- fixed-size records,
// BASELINE cfg 2/3/5 -- resolves a piece by one division instead of a search.
struct EncUniform {
    uint32_t on, c;  // c = 16-byte pieces per record
    uint64_t R;      // record bytes
};

__device__ __forceinline__ EncPiece enc_resolve(const EncodeSmem& s, const EncodeArgs& a,
                                                uint32_t p, uint32_t ptot, uint32_t nrec,
                                                float pscale, const EncUniform& un) {
    EncPiece e;
    e.src = nullptr;
    e.lo = 0;
    e.kind = 0;
    e.rec = 0;
    if (p >= ptot) return e;
    uint32_t rec, q;
    if (un.on) {
        rec = p / un.c;
        q = p - rec * un.c;
        e.lo = (uint64_t)rec * un.R + 16ull * q;
    } else {
        // record owning piece p (last rec with piece[rec] <= p): interpolate,
        // then walk
        rec = (uint32_t)((float)p * pscale);
        if (rec >= nrec) rec = nrec - 1;
        while (s.piece[rec] > p) --rec;
        while (rec + 1 < nrec && s.piece[rec + 1] <= p) ++rec;
        q = p - s.piece[rec];  // piece within the record
        e.lo = s.off[rec] + 16ull * q;
    }
    e.rec = rec;
    if (q == 0) {
        e.kind = 1;
        return e;
    }
    const uint64_t kl = s.klen[rec], vl = s.vlen[rec];
    const uint64_t b0 = 16ull * (q - 1);  // body offset
    if (b0 + 16 <= kl) {
        e.src = a.arena + s.key_off[rec] + b0;
        e.kind = 2;
    } else if (b0 >= kl && b0 + 16 <= kl + vl) {
        e.src = a.arena + s.val_off[rec] + (b0 - kl);
        e.kind = 2;
    } else {
        e.kind = 3;
    }
    return e;
}

__device__ __forceinline__ void enc_store(const EncodeSmem& s, const EncodeArgs& a,
                                          const EncPiece& e, uint4 v, uint64_t tb) {
    if (e.kind == 0) return;
    const uint64_t o = tb + e.lo;
    if (o >= a.cap) return;
    const uint64_t room = a.cap - o;
    uint8_t* dst = a.out + o;
    const uint32_t kl = s.klen[e.rec], vl = s.vlen[e.rec];
    if (e.kind == 1) v = make_uint4(kl, 0u, vl, 0u);
    if (e.kind <= 2 && room >= 16) {
        st_stream16(dst, v);
        return;
    }
    if (e.kind <= 2) {  // clipped by the capacity
        const unsigned __int128 w = ((unsigned __int128)(((uint64_t)v.w << 32) | v.z) << 64) |
                                    (((uint64_t)v.y << 32) | v.x);
        store_part(dst, w, (uint32_t)room);
        return;
    }
    // straddle (key tail | value head) and/or record tail: the piece's nb
    // bytes are assembled in registers from at most two in-bounds 16-byte
    // windows, then stored whole (16 B) or as 8/4/2/1-byte parts, so no byte
    // outside the record is written
    const uint64_t b0 = e.lo - s.off[e.rec] - 16;
    const uint32_t nb = (uint32_t)min((uint64_t)16, (uint64_t)kl + vl - b0);
    const uint8_t* kp = a.arena + s.key_off[e.rec];
    const uint8_t* vp = a.arena + s.val_off[e.rec];
    const uint32_t m1 = b0 < kl ? (uint32_t)min((uint64_t)nb, kl - b0) : 0u;  // key bytes
    const uint32_t m2 = nb - m1;                                               // value bytes
    const uint64_t vo = b0 + m1 - kl;  // value offset of the first value byte (if m2)
    if ((m1 && kl < 16) || (m2 && vl < 16)) {  // a source shorter than one window
        store_bytes(dst, kp, kl, vp, b0, nb, room);
        return;
    }
    unsigned __int128 w = 0;
    if (m1) w = window_bytes(kp, kl, b0);
    if (m2) w |= window_bytes(vp, vl, vo) << (8 * m1);
    store_part(dst, w, (uint32_t)min((uint64_t)nb, room));
}

template <bool NTL>
__global__ __launch_bounds__(ENC_THREADS) void encode_kernel(EncodeArgs a) {
    // pieces in flight per lane: streaming sources want several; gathered
    // ones (a compaction's merged order) run faster with one and more
    // resident waves (cfg 5 leg: 450 -> 424 us; ENC_U 2: 428, 3: 451)
    constexpr uint32_t U = NTL ? ENC_U : ENC_U_GATHER;
    __shared__ EncodeSmem s;
    const uint32_t tid = threadIdx.x;
    a.n = enc_count(a.n, a.n_dev);
    const uint32_t t = blockIdx.x;
    if ((uint64_t)t * ENC_TILE >= a.n) return;  // grid sized for the upper bound
    const uint64_t r0 = (uint64_t)t * ENC_TILE + (uint64_t)tid * ENC_RPT;  // this thread's records

    // ---- 1. descriptors, sizes, piece counts ----------------------------------
    uint64_t sz = 0;
    uint32_t pc = 0;
    uint64_t rsz[ENC_RPT];
    uint32_t rpc[ENC_RPT];
#pragma unroll
    for (uint32_t i = 0; i < ENC_RPT; ++i) {
        const uint64_t r = r0 + i;
        const uint32_t li = tid * ENC_RPT + i;
        rsz[i] = 0;
        rpc[i] = 0;
        if (r < a.n) {
            const hg_pair p = a.pairs[r];
            s.key_off[li] = p.key_off;
            s.val_off[li] = p.val_off;
            s.klen[li] = p.klen;
            s.vlen[li] = p.vlen;
            rsz[i] = 16ull + p.klen + p.vlen;
            rpc[i] = (uint32_t)((rsz[i] + 15) >> 4);
        }
        sz += rsz[i];
        pc += rpc[i];
    }
    {  // uniform-tile test: every valid record's (klen, vlen) equal
        uint64_t key = 0;
        bool have = false, same = true;
#pragma unroll
        for (uint32_t i = 0; i < ENC_RPT; ++i) {
            if (!rpc[i]) continue;
            const uint32_t li = tid * ENC_RPT + i;
            const uint64_t k = ((uint64_t)s.klen[li] << 32) | s.vlen[li];
            same = same && (!have || key == k);
            key = k;
            have = true;
        }
        const unsigned long long hv = __ballot(have);
        const uint64_t m = hv ? (uint64_t)__shfl(key, __ffsll((long long)hv) - 1, 64) : 0ull;
        const bool ok = __all(same && (!have || key == m));
        if ((tid & 63u) == 0) {
            s.wsize[tid >> 6] = m;
            s.wflag[tid >> 6] = hv ? (ok ? 1u : 2u) : 0u;
        }
    }
    uint64_t tot;
    uint64_t loff = block_excl_scan64(sz, s.scan_tmp64, tot);
    uint32_t ptot;
    uint32_t lpc = block_excl_scan<ENC_NW>(pc, s.scan_tmp, ptot);
#pragma unroll
    for (uint32_t i = 0; i < ENC_RPT; ++i) {
        s.off[tid * ENC_RPT + i] = loff;
        s.piece[tid * ENC_RPT + i] = lpc;
        loff += rsz[i];
        lpc += rpc[i];
    }
    if (tid == 0) {
        s.off[ENC_TILE] = tot;
        s.piece[ENC_TILE] = ptot;
    }
    __syncthreads();

    // ---- 2. first pieces in flight, then the look-back ----------------------------
    // Sources do not depend on the tile's output offset, so the first U
    // pieces per lane are loaded before the look-back and land while it runs.
    // The copy loop is software-pipelined: the loads of step i+1 are issued
    // before the stores of step i (vmcnt counts loads and stores together, in
    // issue order, so a load issued after a store would also wait for it).
    const uint32_t nrec = (uint32_t)min((uint64_t)ENC_TILE, a.n - (uint64_t)t * ENC_TILE);
    const float pscale = (float)nrec / (float)ptot;
    EncUniform un;
    {
        uint64_t k = 0;
        bool ok = true, have = false;
#pragma unroll
        for (uint32_t w = 0; w < ENC_NW; ++w) {
            const uint32_t f = s.wflag[w];
            if (f == 0) continue;  // wave without records
            ok = ok && f == 1 && (!have || k == s.wsize[w]);
            k = s.wsize[w];
            have = true;
        }
        un.on = ok && have;
        un.R = 16ull + (k >> 32) + (k & 0xFFFFFFFFull);
        un.c = un.on ? (uint32_t)((un.R + 15) >> 4) : 1u;
    }
    // a piece without a 16-byte source loads the descriptors' first 16 bytes
    // (branch-free, so all U loads are in flight together)
    const uint8_t* safe = reinterpret_cast<const uint8_t*>(a.pairs);
    // ENC_PRE steps of pieces are loaded first; the tile's output offset is
    // read meanwhile: its group's base plus the sums of the tiles before it
    // in the group.
    EncPiece pre[ENC_PRE];
    uint4 vpre[ENC_PRE];
#pragma unroll
    for (uint32_t k = 0; k < ENC_PRE; ++k) {
        pre[k] = enc_resolve(s, a, tid + k * ENC_THREADS, ptot, nrec, pscale, un);
        vpre[k] = ld_stream16<NTL>(pre[k].kind == 2 ? pre[k].src : safe);
    }
    if (tid < 64) {
        const uint32_t g = t / ENC_GROUP, j = t % ENC_GROUP;
        const uint64_t v = tid < j ? a.tile_sum[(uint64_t)g * ENC_GROUP + tid] : 0ull;
        const uint64_t b = wave_sum<uint64_t>(v) + a.group_base[g];
        if (tid == 0) s.tile_base = b;
    }
    __syncthreads();
    const uint64_t tb = s.tile_base;
    if (a.rec_off)
#pragma unroll
        for (uint32_t i = 0; i < ENC_RPT; ++i)
            if (r0 + i < a.n) a.rec_off[r0 + i] = a.rec_base + tb + s.off[tid * ENC_RPT + i];

    // ---- 3. piece copy ----------------------------------------------------------
    // Unrolled by two with swapped roles, so the in-flight loads are never
    // moved between registers (a move would wait for them).
    constexpr uint32_t STEP = ENC_THREADS * U;
    const uint32_t p0 = tid + ENC_PRE * ENC_THREADS;  // first piece of the pipelined loop
    EncPiece cur[U], nx[U];
    uint4 vc[U], vn[U];
#pragma unroll
    for (uint32_t u = 0; u < U; ++u) {
        cur[u] = enc_resolve(s, a, p0 + u * ENC_THREADS, ptot, nrec, pscale, un);
        vc[u] = ld_stream16<NTL>(cur[u].kind == 2 ? cur[u].src : safe);
    }
#pragma unroll
    for (uint32_t k = 0; k < ENC_PRE; ++k) enc_store(s, a, pre[k], vpre[k], tb);
    auto step = [&](EncPiece* c, uint4* vcur, EncPiece* n, uint4* vnext, uint32_t pb) {
#pragma unroll
        for (uint32_t u = 0; u < U; ++u) {
            n[u] = enc_resolve(s, a, pb + STEP + u * ENC_THREADS, ptot, nrec, pscale, un);
            vnext[u] = ld_stream16<NTL>(n[u].kind == 2 ? n[u].src : safe);
        }
#pragma unroll
        for (uint32_t u = 0; u < U; ++u) enc_store(s, a, c[u], vcur[u], tb);
    };
    for (uint32_t pb = p0; pb < ptot; pb += 2 * STEP) {
        step(cur, vc, nx, vn, pb);
        if (pb + STEP >= ptot) break;
        step(nx, vn, cur, vc, pb + STEP);
    }
}

// ---- whole-record gather (compaction) ------------------------------------------------
// When every pair is a whole source record -- its header the 16 bytes before
// key_off, val_off == key_off + klen: pairs emitted by the merge of decoded
// tables -- the output is those records' bytes verbatim, in pair order (the
// header a record carries is the one encode_kernel would write: the decoder
// took klen / vlen from it and rejects high words).  Output pieces are then
// 16 bytes aligned in the OUTPUT: a piece takes the bytes of the record it
// starts in and, where a record boundary falls inside it, of the next record,
// whose window is read from n1 bytes before that record's start so its bytes
// land in place and one v_bfi per dword merges the two.  encode_kernel's
// record-relative pieces had paid header synthesis, key|value straddles and
// tail parts (4-byte stores) on every record: ~190 VALU per wave-piece on the
// cfg 5 leg, a VALU-bound gather.  A tile owns the pieces that START in its
// byte range; the last one may finish with the next tile's first record.
#ifndef HG_ENC_REC_U
#define HG_ENC_REC_U 1  // cfg 5 leg, round 4 same box: 1 -> 1.254-1.257 ms, 2: 1.268-1.279, 4: 1.285-1.336
#endif
constexpr uint32_t REC_U = HG_ENC_REC_U;  // pieces per lane per step (their loads overlap)

struct RecSmem {
    uint64_t src[ENC_TILE + 1];  // arena offset of each record's header (+ the next tile's first)
    uint64_t off[ENC_TILE + 2];  // tile-relative output offsets (off[nrec] = tile bytes)
    uint64_t scan_tmp64[ENC_NW];
    uint64_t tile_base;
};

// 16 bytes of the arena from p, never outside [0, len): a window past either
// end is read in bounds and shifted (rare: records at the arena's edges).
__device__ __forceinline__ uint4 arena16(const uint8_t* arena, uint64_t len, int64_t p) {
    if (p >= 0 && (uint64_t)p + 16 <= len) return *reinterpret_cast<const uint4*>(arena + p);
    uint8_t b[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        const int64_t q = p + i;
        b[i] = (q >= 0 && (uint64_t)q < len) ? arena[q] : 0;
    }
    uint4 v;
    v.x = b[0] | (b[1] << 8) | (b[2] << 16) | ((uint32_t)b[3] << 24);
    v.y = b[4] | (b[5] << 8) | (b[6] << 16) | ((uint32_t)b[7] << 24);
    v.z = b[8] | (b[9] << 8) | (b[10] << 16) | ((uint32_t)b[11] << 24);
    v.w = b[12] | (b[13] << 8) | (b[14] << 16) | ((uint32_t)b[15] << 24);
    return v;
}

// Byte mask of dword i for the bytes of a 16-byte piece below n (n in [0, 16]).
__device__ __forceinline__ uint32_t lowbytes_mask(uint32_t n, uint32_t i) {
    const int32_t k = (int32_t)n - 4 * (int32_t)i;  // bytes of dword i below n
    return k >= 4 ? ~0u : (k <= 0 ? 0u : (1u << (8 * k)) - 1u);
}

__global__ __launch_bounds__(ENC_THREADS) void encode_records_kernel(EncodeArgs a,
                                                                     uint64_t arena_len) {
    __shared__ RecSmem s;
    const uint32_t tid = threadIdx.x;
    a.n = enc_count(a.n, a.n_dev);
    const uint32_t t = blockIdx.x;
    if ((uint64_t)t * ENC_TILE >= a.n) return;  // grid sized for the upper bound
    const uint64_t r0 = (uint64_t)t * ENC_TILE;
    const uint32_t nrec = (uint32_t)min((uint64_t)ENC_TILE, a.n - r0);
    // ---- descriptors -> record sources and sizes, next tile's first record
    uint64_t sz = 0;
    if (tid < nrec) {
        const hg_pair p = a.pairs[r0 + tid];
        s.src[tid] = p.key_off - 16;
        sz = 16ull + p.klen + p.vlen;
    }
    if (tid == 0) s.src[nrec] = r0 + nrec < a.n ? a.pairs[r0 + nrec].key_off - 16 : 0ull;
    uint64_t tot;
    const uint64_t loff = block_excl_scan64(sz, s.scan_tmp64, tot);
    if (tid < nrec) s.off[tid] = loff;
    if (tid == 0) s.off[nrec] = tot;
    if (tid < 64) {  // the tile's output offset: its group's base + the tiles before it there
        const uint32_t g = t / ENC_GROUP, j = t % ENC_GROUP;
        const uint64_t v = tid < j ? a.tile_sum[(uint64_t)g * ENC_GROUP + tid] : 0ull;
        const uint64_t b = wave_sum<uint64_t>(v) + a.group_base[g];
        if (tid == 0) s.tile_base = b;
    }
    __syncthreads();
    const uint64_t tb = s.tile_base;
    if (a.rec_off && tid < nrec) a.rec_off[r0 + tid] = a.rec_base + tb + loff;
    const bool has_next = r0 + nrec < a.n;  // a piece may run into the next tile's first record
    // pieces starting in [tb, tb + tot): P in [ceil(tb / 16), ceil((tb + tot) / 16))
    const uint64_t pa = (tb + 15) >> 4, pe = (tb + tot + 15) >> 4;
    const uint32_t np = (uint32_t)(pe - pa);
    const float scale = tot ? (float)nrec / (float)tot : 0.f;
    for (uint32_t i0 = 0; i0 < np; i0 += ENC_THREADS * REC_U) {
        uint4 w1[REC_U], w2[REC_U];
        uint32_t n1[REC_U];
        uint64_t o[REC_U];
        bool live[REC_U], two[REC_U];
#pragma unroll
        for (uint32_t u = 0; u < REC_U; ++u) {
            const uint32_t i = i0 + u * ENC_THREADS + tid;
            live[u] = i < np;
            const uint64_t ob = 16 * (pa + (live[u] ? i : 0)) - tb;  // tile-relative piece start
            o[u] = ob;
            uint32_t r = min((uint32_t)((float)ob * scale), nrec - 1);  // interpolate, then walk
            while (r > 0 && s.off[r] > ob) --r;
            while (r + 1 < nrec && s.off[r + 1] <= ob) ++r;
            const uint64_t rem = s.off[r + 1] - ob;  // record r's bytes from the piece start
            n1[u] = rem < 16 ? (uint32_t)rem : 16u;
            two[u] = n1[u] < 16 && (r + 1 < nrec || has_next);
            w1[u] = arena16(a.arena, arena_len, (int64_t)(s.src[r] + (ob - s.off[r])));
            w2[u] = two[u] ? arena16(a.arena, arena_len, (int64_t)s.src[r + 1] - (int64_t)n1[u])
                           : make_uint4(0, 0, 0, 0);
        }
#pragma unroll
        for (uint32_t u = 0; u < REC_U; ++u) {
            if (!live[u]) continue;
            uint4 v = w1[u];
            if (n1[u] < 16) {
                v.x = (v.x & lowbytes_mask(n1[u], 0)) | (w2[u].x & ~lowbytes_mask(n1[u], 0));
                v.y = (v.y & lowbytes_mask(n1[u], 1)) | (w2[u].y & ~lowbytes_mask(n1[u], 1));
                v.z = (v.z & lowbytes_mask(n1[u], 2)) | (w2[u].z & ~lowbytes_mask(n1[u], 2));
                v.w = (v.w & lowbytes_mask(n1[u], 3)) | (w2[u].w & ~lowbytes_mask(n1[u], 3));
            }
            const uint64_t O = tb + o[u];  // absolute output offset of the piece
            // bytes of the piece that exist: the output ends after the last
            // record (no next record), and nothing at or past cap is written
            uint64_t lim = two[u] || n1[u] == 16 ? 16ull : n1[u];
            if (O >= a.cap) continue;
            if (a.cap - O < lim) lim = a.cap - O;
            uint8_t* dst = a.out + O;
            if (lim == 16) {
                st_stream16(dst, v);
            } else {
                const unsigned __int128 wv = ((unsigned __int128)(((uint64_t)v.w << 32) | v.z) << 64) |
                                             (((uint64_t)v.y << 32) | v.x);
                store_part(dst, wv, (uint32_t)lim);
            }
        }
    }
}

// Output bytes per tile and per group of ENC_GROUP tiles: tsum[t] = sum over
// the tile's records of 16 + klen + vlen; gsum[t / ENC_GROUP] += tsum[t]
// (gsum zeroed before launch).
__global__ __launch_bounds__(ENC_THREADS) void encode_sums_kernel(const hg_pair* pairs,
                                                                  uint64_t n, uint64_t* tsum,
                                                                  unsigned long long* gsum,
                                                                  const uint64_t* n_dev) {
    __shared__ uint64_t part[ENC_NW];
    const uint32_t tid = threadIdx.x, t = blockIdx.x;
    n = enc_count(n, n_dev);
    uint64_t sz = 0;
#pragma unroll
    for (uint32_t i = 0; i < ENC_RPT; ++i) {
        const uint64_t r = (uint64_t)t * ENC_TILE + (uint64_t)i * ENC_THREADS + tid;
        if (r < n) sz += 16ull + pairs[r].klen + pairs[r].vlen;
    }
    sz = wave_sum<uint64_t>(sz);
    if ((tid & 63u) == 0) part[tid >> 6] = sz;
    __syncthreads();
    if (tid == 0) {
        uint64_t tot = 0;
#pragma unroll
        for (uint32_t w = 0; w < ENC_NW; ++w) tot += part[w];
        tsum[t] = tot;
        atomicAdd(&gsum[t / ENC_GROUP], (unsigned long long)tot);
    }
}

// In-place exclusive scan of the group sums (one workgroup; each thread owns
// a contiguous chunk, loaded 8 at a time so the loads overlap) and the call's
// result: out_len = total bytes, HG_ERR_CAPACITY if they exceed cap.
constexpr uint32_t BASES_THREADS = 1024;
// zero_next / zero_words (nullable): the next call's group sums (the other
// half of a double buffer, hgk_encode_launch_ctl), cleared here.
__global__ __launch_bounds__(BASES_THREADS) void encode_bases_kernel(uint64_t* gsum, uint64_t ng,
                                                                     uint64_t cap,
                                                                     hg_encode_result* result,
                                                                     uint64_t* zero_next,
                                                                     uint64_t zero_words) {
    __shared__ uint64_t part[BASES_THREADS / 64];
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wid = tid >> 6;
    for (uint64_t i = tid; i < zero_words; i += BASES_THREADS) zero_next[i] = 0;
    const uint64_t chunk = (ng + BASES_THREADS - 1) / BASES_THREADS;
    const uint64_t lo = min(ng, (uint64_t)tid * chunk), hi = min(ng, lo + chunk);
    uint64_t sum = 0;
    for (uint64_t i = lo; i < hi; i += 8) {
        uint64_t v[8];
#pragma unroll
        for (uint32_t k = 0; k < 8; ++k) v[k] = i + k < hi ? gsum[i + k] : 0ull;
#pragma unroll
        for (uint32_t k = 0; k < 8; ++k) sum += v[k];
    }
    uint64_t x = sum;  // block exclusive scan of the chunk sums
#pragma unroll
    for (uint32_t d = 1; d < 64; d <<= 1) {
        const uint64_t y = __shfl_up(x, d, 64);
        if (lane >= d) x += y;
    }
    if (lane == 63) part[wid] = x;
    __syncthreads();
    uint64_t pre = 0, tot = 0;
#pragma unroll
    for (uint32_t w = 0; w < BASES_THREADS / 64; ++w) {
        pre += w < wid ? part[w] : 0ull;
        tot += part[w];
    }
    uint64_t run = pre + x - sum;
    for (uint64_t i = lo; i < hi; i += 8) {
        uint64_t v[8];
#pragma unroll
        for (uint32_t k = 0; k < 8; ++k) v[k] = i + k < hi ? gsum[i + k] : 0ull;
#pragma unroll
        for (uint32_t k = 0; k < 8; ++k)
            if (i + k < hi) {
                gsum[i + k] = run;
                run += v[k];
            }
    }
    if (tid == 0) {
        hg_encode_result res;
        res.out_len = tot;
        res.kind = tot <= cap ? HG_OK : HG_ERR_CAPACITY;
        res.reserved = 0;
        *result = res;
    }
}

// blocks[b] = {b*stride, rec_off[b*stride], rec_off[min((b+1)*stride, n)] - pos}
// The table's total length comes from `res` (device) or, with res null, `total`.
__global__ void blocks_kernel(const uint64_t* rec_off, uint64_t n, uint32_t stride,
                              const hg_encode_result* res, uint64_t total, hg_block* blocks,
                              uint64_t nb, const uint64_t* n_dev) {
    const uint64_t b = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    n = enc_count(n, n_dev);
    if (b >= nb || b * stride >= n) return;
    const uint64_t first = b * stride;
    const uint64_t nxt = first + stride;
    const uint64_t pos = rec_off[first];
    const uint64_t end = nxt < n ? rec_off[nxt] : (res ? res->out_len : total);
    hg_block blk;
    blk.first_rec = first;
    blk.position = pos;
    blk.length = end - pos;
    blocks[b] = blk;
}

}  // namespace hgk

extern "C" uint64_t hgk_encode_workspace_bytes(uint64_t n) {
    const uint64_t nt = (n + hgk::ENC_TILE - 1) / hgk::ENC_TILE;
    const uint64_t ng = (nt + hgk::ENC_GROUP - 1) / hgk::ENC_GROUP;
    return (nt + ng + 2) * sizeof(unsigned long long);
}

// d_status: hgk_encode_workspace_bytes(n) bytes (the tile sums / bases).
// d_rec_off may be null unless d_blocks is requested (the runtime then passes
// workspace).  Three launches: tile sums, their scan (+ the result), copy.
// rec_base is added to every record offset written (0 for a whole table; the
// chunk's output offset when a host encode runs the table in chunks).
// d_n (optional): the record count is min(n, *d_n), read on the device -- a
// merge's output count, so merge and encode run without a host round trip
// (grids are sized for n).  gather: pairs point into several tables (merged
// order), sources are read with the default cache policy.
namespace {
// mode 0: streaming sources (a table's own pairs), 1: gathered pairs, 2:
// whole records gathered (encode_records_kernel; rec_arena_len = arena bytes)
int encode_launch_mode(const uint8_t* d_arena, const hg_pair* d_pairs, uint64_t n,
                       const uint64_t* d_n, int mode, uint64_t rec_arena_len, uint8_t* d_out,
                       uint64_t cap, uint64_t* d_rec_off, uint64_t rec_base,
                       uint32_t block_stride, hg_block* d_blocks, hg_encode_result* d_result,
                       unsigned long long* d_status, hipStream_t stream, bool gsum_zeroed = false,
                       uint64_t* gsum_ext = nullptr, uint64_t* zero_next = nullptr,
                       uint64_t zero_words = 0, bool sums_ready = false) {
    using namespace hgk;
    const uint64_t nt = (n + ENC_TILE - 1) / ENC_TILE;
    const uint64_t ng = (nt + ENC_GROUP - 1) / ENC_GROUP;
    uint64_t* tsum = reinterpret_cast<uint64_t*>(d_status);
    uint64_t* gsum = gsum_ext ? gsum_ext : tsum + nt;  // (gsum_ext: a double-buffered half)
    if (nt == 0) {
        if (hipMemsetAsync(d_result, 0, sizeof(hg_encode_result), stream) != hipSuccess)
            return HG_HIP_FAIL;
        return HG_OK;
    }
    // sums_ready: the merge's last round accumulated tsum / gsum (no pass here)
    if (!sums_ready && !gsum_zeroed && hipMemsetAsync(gsum, 0, ng * sizeof(uint64_t), stream) != hipSuccess)
        return HG_HIP_FAIL;
    if (!sums_ready) {
        hipLaunchKernelGGL(encode_sums_kernel, dim3((uint32_t)nt), dim3(ENC_THREADS), 0, stream,
                           d_pairs, n, tsum, reinterpret_cast<unsigned long long*>(gsum), d_n);
        if (HG_LAUNCH_STATUS() != HG_OK) return HG_ERR_HIP;
    }
    hipLaunchKernelGGL(encode_bases_kernel, dim3(1), dim3(BASES_THREADS), 0, stream, gsum, ng, cap,
                       d_result, zero_next, zero_words);
    if (HG_LAUNCH_STATUS() != HG_OK) return HG_ERR_HIP;
    EncodeArgs a;
    a.arena = d_arena;
    a.pairs = d_pairs;
    a.n = n;
    a.out = d_out;
    a.cap = cap;
    a.rec_off = d_rec_off;
    a.rec_base = rec_base;
    a.result = d_result;
    a.tile_sum = tsum;
    a.group_base = gsum;
    a.n_dev = d_n;
    if (mode == 2)
        hipLaunchKernelGGL(encode_records_kernel, dim3((uint32_t)nt), dim3(ENC_THREADS), 0, stream, a,
                           rec_arena_len);
    else if (mode == 1)
        hipLaunchKernelGGL(encode_kernel<false>, dim3((uint32_t)nt), dim3(ENC_THREADS), 0, stream, a);
    else
        hipLaunchKernelGGL(encode_kernel<true>, dim3((uint32_t)nt), dim3(ENC_THREADS), 0, stream, a);
    if (HG_LAUNCH_STATUS() != HG_OK) return HG_ERR_HIP;
    if (d_blocks) {
        const uint64_t nb = (n + block_stride - 1) / block_stride;
        const uint32_t grid = (uint32_t)((nb + 255) / 256);
        hipLaunchKernelGGL(blocks_kernel, dim3(grid), dim3(256), 0, stream, d_rec_off, n,
                           block_stride, (const hg_encode_result*)d_result, (uint64_t)0, d_blocks,
                           nb, d_n);
        if (HG_LAUNCH_STATUS() != HG_OK) return HG_ERR_HIP;
    }
    return HG_OK;
}

}  // namespace

extern "C" int hgk_encode_launch_ex(const uint8_t* d_arena, const hg_pair* d_pairs, uint64_t n,
                                    const uint64_t* d_n, bool gather, uint8_t* d_out, uint64_t cap,
                                    uint64_t* d_rec_off, uint64_t rec_base, uint32_t block_stride,
                                    hg_block* d_blocks, hg_encode_result* d_result,
                                    unsigned long long* d_status, hipStream_t stream) {
    return encode_launch_mode(d_arena, d_pairs, n, d_n, gather ? 1 : 0, 0, d_out, cap, d_rec_off,
                              rec_base, block_stride, d_blocks, d_result, d_status, stream);
}

// Pairs that are whole source records in an arena of arena_len bytes (the
// compaction's merged pairs): encode_records_kernel gathers the records.
extern "C" int hgk_encode_launch_records(const uint8_t* d_arena, uint64_t arena_len,
                                         const hg_pair* d_pairs, uint64_t n, const uint64_t* d_n,
                                         uint8_t* d_out, uint64_t cap, uint64_t* d_rec_off,
                                         uint32_t block_stride, hg_block* d_blocks,
                                         hg_encode_result* d_result, unsigned long long* d_status,
                                         hipStream_t stream, int gsum_zeroed, int sums_ready) {
    return encode_launch_mode(d_arena, d_pairs, n, d_n, 2, arena_len, d_out, cap, d_rec_off, 0,
                              block_stride, d_blocks, d_result, d_status, stream, gsum_zeroed != 0,
                              nullptr, nullptr, 0, sums_ready != 0);
}

// hgk_encode_launch_ex with its group sums in gs_cur (clean: words of it
// known to be zero; no memset launch when they cover the call's) and the
// next call's in gs_next (next_words of room), cleared by encode_bases_kernel;
// *zeroed = the words cleared.
extern "C" int hgk_encode_launch_ctl(const uint8_t* d_arena, const hg_pair* d_pairs, uint64_t n,
                                     uint8_t* d_out, uint64_t cap, uint64_t* d_rec_off,
                                     uint32_t block_stride, hg_block* d_blocks,
                                     hg_encode_result* d_result, unsigned long long* d_status,
                                     uint64_t* gs_cur, uint64_t clean, uint64_t* gs_next,
                                     uint64_t next_words, uint64_t* zeroed, hipStream_t stream) {
    using namespace hgk;
    const uint64_t nt = (n + ENC_TILE - 1) / ENC_TILE;
    const uint64_t ng = (nt + ENC_GROUP - 1) / ENC_GROUP;
    const uint64_t z = ng < next_words ? ng : next_words;
    *zeroed = nt ? z : 0;
    return encode_launch_mode(d_arena, d_pairs, n, nullptr, 0, 0, d_out, cap, d_rec_off, 0,
                              block_stride, d_blocks, d_result, d_status, stream, clean >= ng,
                              gs_cur, gs_next, z);
}

// The group sums an encode of n pairs accumulates into (words from d_status):
// cleared by the launch unless its caller had them cleared earlier on the
// stream (gsum_zeroed; the compaction's merge flag kernel does).
extern "C" void hgk_encode_tile_geometry(uint32_t* tile_log2, uint32_t* group_log2) {
    using namespace hgk;
    static_assert((ENC_TILE & (ENC_TILE - 1)) == 0 && (ENC_GROUP & (ENC_GROUP - 1)) == 0,
                  "encode tiles and groups are powers of two");
    *tile_log2 = (uint32_t)__builtin_ctz(ENC_TILE);
    *group_log2 = (uint32_t)__builtin_ctz(ENC_GROUP);
}

extern "C" void hgk_encode_group_sums(uint64_t n, uint64_t* first_word, uint64_t* words) {
    using namespace hgk;
    const uint64_t nt = (n + ENC_TILE - 1) / ENC_TILE;
    *first_word = nt;
    *words = (nt + ENC_GROUP - 1) / ENC_GROUP;
}

extern "C" int hgk_encode_launch_at(const uint8_t* d_arena, const hg_pair* d_pairs, uint64_t n,
                                    uint8_t* d_out, uint64_t cap, uint64_t* d_rec_off,
                                    uint64_t rec_base, uint32_t block_stride, hg_block* d_blocks,
                                    hg_encode_result* d_result, unsigned long long* d_status,
                                    hipStream_t stream) {
    return hgk_encode_launch_ex(d_arena, d_pairs, n, nullptr, false, d_out, cap, d_rec_off,
                                rec_base, block_stride, d_blocks, d_result, d_status, stream);
}

extern "C" int hgk_encode_launch(const uint8_t* d_arena, const hg_pair* d_pairs, uint64_t n,
                                 uint8_t* d_out, uint64_t cap, uint64_t* d_rec_off,
                                 uint32_t block_stride, hg_block* d_blocks,
                                 hg_encode_result* d_result, unsigned long long* d_status,
                                 hipStream_t stream) {
    return hgk_encode_launch_at(d_arena, d_pairs, n, d_out, cap, d_rec_off, 0, block_stride,
                                d_blocks, d_result, d_status, stream);
}

// Block entries of a whole table from its (global) record offsets and total
// length (host known): the chunked host encode runs this once at the end.
extern "C" int hgk_encode_blocks_launch(const uint64_t* d_rec_off, uint64_t n,
                                        uint32_t block_stride, uint64_t total, hg_block* d_blocks,
                                        hipStream_t stream) {
    using namespace hgk;
    if (n == 0 || block_stride == 0) return HG_OK;
    const uint64_t nb = (n + block_stride - 1) / block_stride;
    const uint32_t grid = (uint32_t)((nb + 255) / 256);
    hipLaunchKernelGGL(blocks_kernel, dim3(grid), dim3(256), 0, stream, d_rec_off, n, block_stride,
                       (const hg_encode_result*)nullptr, total, d_blocks, nb,
                       (const uint64_t*)nullptr);
    return HG_LAUNCH_STATUS();
}

// Block entries of a compaction written by the merge's records mode: the
// record count (*d_n, at most n_ub) and the total length (d_res->out_len)
// are on the device; grid sized for n_ub.
extern "C" int hgk_encode_blocks_launch_dev(const uint64_t* d_rec_off, uint64_t n_ub,
                                            const uint64_t* d_n, const hg_encode_result* d_res,
                                            uint32_t block_stride, hg_block* d_blocks,
                                            hipStream_t stream) {
    using namespace hgk;
    if (n_ub == 0 || block_stride == 0) return HG_OK;
    const uint64_t nb = (n_ub + block_stride - 1) / block_stride;
    const uint32_t grid = (uint32_t)((nb + 255) / 256);
    hipLaunchKernelGGL(blocks_kernel, dim3(grid), dim3(256), 0, stream, d_rec_off, n_ub, block_stride,
                       d_res, (uint64_t)0, d_blocks, nb, d_n);
    return HG_LAUNCH_STATUS();
}

// Encoded size only (hg_encoded_size on device pairs): the tile sums and
// their scan, no copy -- d_result->out_len = sum(16 + klen + vlen).
extern "C" int hgk_encode_size_launch(const hg_pair* d_pairs, uint64_t n,
                                      hg_encode_result* d_result, unsigned long long* d_status,
                                      hipStream_t stream) {
    using namespace hgk;
    const uint64_t nt = (n + ENC_TILE - 1) / ENC_TILE;
    const uint64_t ng = (nt + ENC_GROUP - 1) / ENC_GROUP;
    uint64_t* tsum = reinterpret_cast<uint64_t*>(d_status);
    uint64_t* gsum = tsum + nt;
    if (nt == 0)
        return hipMemsetAsync(d_result, 0, sizeof(hg_encode_result), stream) == hipSuccess
                   ? HG_OK
                   : HG_HIP_FAIL;
    if (hipMemsetAsync(gsum, 0, ng * sizeof(uint64_t), stream) != hipSuccess) return HG_HIP_FAIL;
    hipLaunchKernelGGL(encode_sums_kernel, dim3((uint32_t)nt), dim3(ENC_THREADS), 0, stream,
                       d_pairs, n, tsum, reinterpret_cast<unsigned long long*>(gsum),
                       (const uint64_t*)nullptr);
    hipLaunchKernelGGL(encode_bases_kernel, dim3(1), dim3(BASES_THREADS), 0, stream, gsum, ng,
                       ~0ull, d_result, (uint64_t*)nullptr, (uint64_t)0);
    return HG_LAUNCH_STATUS();
}

namespace hgk {
// out[j] = v[first + j * stride] for first + j * stride < n: the record
// offsets a key-range slice of a compaction contributes to the block index.
__global__ void gather_stride_kernel(const uint64_t* v, uint64_t n, uint64_t first,
                                     uint64_t stride, uint64_t* out) {
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t i = first + j * stride;
    if (i < n) out[j] = v[i];
}
}  // namespace hgk

extern "C" int hgk_gather_stride_launch(const uint64_t* d_v, uint64_t n, uint64_t first,
                                        uint64_t stride, uint64_t* d_out, hipStream_t stream) {
    if (first >= n || stride == 0) return HG_OK;
    const uint64_t m = (n - first + stride - 1) / stride;
    hipLaunchKernelGGL(hgk::gather_stride_kernel, dim3((uint32_t)((m + 255) / 256)), dim3(256), 0,
                       stream, d_v, n, first, stride, d_out);
    return HG_LAUNCH_STATUS();
}
