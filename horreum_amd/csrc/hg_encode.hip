// hg_encode.hip — device-resident SSTable encode (record packing) for gfx950.
//
// Replaces InternalPair::serialize / serialize_flatten (reference
// src/format.rs:23-42): every record becomes
//     [u64 LE klen][u64 LE vlen][key][value]      (vlen == 0: no value bytes)
// concatenated in the given order, and Index::new's second encode that only
// learns block positions/lengths (src/sstable/index.rs:55-67).
//
// One pass:
//  1. A 256-thread workgroup takes a tile of 256 records by atomic ticket,
//     loads their descriptors and scans record sizes (16 + klen + vlen) and
//     16-byte piece counts in LDS.
//  2. The tile's output offset comes from a decoupled look-back over the
//     tiles before it (CUB-style: one wave reads 63 predecessor statuses per
//     step; AGG = tile bytes, INCL = inclusive prefix).
//  3. Lanes copy consecutive 16-byte output pieces (coalesced 1 KiB per wave
//     instruction): piece 0 of a record is its header, synthesised in
//     registers; body pieces are unaligned 16-byte loads from the key/value
//     source; pieces that straddle key|value or end mid-record go bytewise,
//     so no byte outside a record's own output range is ever stored.
// Block index entries come from a second, tiny kernel over record offsets.
#include "hg_device.hpp"

namespace hgk {

constexpr uint32_t ENC_TILE = 256;
constexpr uint32_t ENC_NW = ENC_TILE / 64;
constexpr uint64_t EF_AGG = 1ull << 62, EF_INCL = 2ull << 62;
constexpr uint64_t EV_MASK = (1ull << 62) - 1;

struct EncodeArgs {
    const uint8_t* arena;
    const hg_pair* pairs;
    uint64_t n;
    uint8_t* out;
    uint64_t cap;
    uint64_t* rec_off;  // may be null
    hg_encode_result* result;
    unsigned long long* status;  // 1 word per tile, zeroed before launch
    uint32_t* ticket;
    uint32_t ntiles;
};

struct EncodeSmem {
    uint64_t key_off[ENC_TILE], val_off[ENC_TILE], off[ENC_TILE + 1];
    uint32_t klen[ENC_TILE], vlen[ENC_TILE], piece[ENC_TILE + 1];
    uint32_t scan_tmp[ENC_NW];
    uint64_t scan_tmp64[ENC_NW];
    uint32_t tile;
    uint64_t tile_base;
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

// Exclusive prefix of tile sums before tile `t` (wave 0, all lanes).
__device__ uint64_t enc_lookback(const EncodeArgs& a, uint32_t t, bool& timeout) {
    const uint32_t lane = threadIdx.x & 63u;
    uint64_t acc = 0;
    int64_t j0 = (int64_t)t - 1;
    uint32_t spins = 0;
    timeout = false;
    while (j0 >= 0) {
        const int64_t j = j0 - (int64_t)lane;
        unsigned long long w;
        int fi;
        for (;;) {
            w = j >= 0 ? ld_agent(&a.status[j]) : (EF_INCL | 0ull);
            const uint64_t f = w >> 62;
            unsigned long long incl = __ballot(f == 2);
            unsigned long long notready = __ballot(f == 0);
            fi = incl ? __ffsll((long long)incl) - 1 : 64;
            unsigned long long relevant = fi >= 63 ? ~0ull : ((1ull << (fi + 1)) - 1ull);
            if (!(notready & relevant)) break;
            if (++spins > (1u << 22)) {
                timeout = true;
                return 0;
            }
            __builtin_amdgcn_s_sleep(2);
        }
        const uint64_t v = (int)lane <= fi ? (w & EV_MASK) : 0ull;  // AGGs + first INCL
        acc += wave_sum<uint64_t>(v);
        if (fi < 64) return acc;
        j0 -= 64;
    }
    return acc;
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

__global__ __launch_bounds__(ENC_TILE) void encode_kernel(EncodeArgs a) {
    __shared__ EncodeSmem s;
    const uint32_t tid = threadIdx.x;
    if (tid == 0) s.tile = atomicAdd(a.ticket, 1u);
    __syncthreads();
    const uint32_t t = s.tile;
    const uint64_t r = (uint64_t)t * ENC_TILE + tid;

    // ---- 1. descriptors, sizes, piece counts ----------------------------------
    uint64_t sz = 0;
    uint32_t pc = 0;
    if (r < a.n) {
        const hg_pair p = a.pairs[r];
        s.key_off[tid] = p.key_off;
        s.val_off[tid] = p.val_off;
        s.klen[tid] = p.klen;
        s.vlen[tid] = p.vlen;
        sz = 16ull + p.klen + p.vlen;
        pc = (uint32_t)((sz + 15) >> 4);
    }
    uint64_t tot;
    const uint64_t loff = block_excl_scan64(sz, s.scan_tmp64, tot);
    uint32_t ptot;
    const uint32_t lpc = block_excl_scan<ENC_NW>(pc, s.scan_tmp, ptot);
    s.off[tid] = loff;
    s.piece[tid] = lpc;
    if (tid == 0) {
        s.off[ENC_TILE] = tot;
        s.piece[ENC_TILE] = ptot;
    }

    // ---- 2. look-back for the tile's output offset ----------------------------
    if (tid < 64) {
        if (tid == 0) st_agent(&a.status[t], (t == 0 ? EF_INCL : EF_AGG) | tot);
        uint64_t base = 0;
        bool timeout = false;
        if (t > 0) {
            base = enc_lookback(a, t, timeout);
            if (tid == 0) st_agent(&a.status[t], EF_INCL | ((base + tot) & EV_MASK));
        }
        if (tid == 0) s.tile_base = base;
        if (timeout && tid == 0) {
            hg_encode_result res;
            res.out_len = 0;
            res.kind = HG_ERR_INTERNAL;
            res.reserved = 0;
            *a.result = res;
        }
    }
    __syncthreads();
    const uint64_t tb = s.tile_base;
    if (r < a.n && a.rec_off) a.rec_off[r] = tb + loff;

    // ---- 3. piece copy ----------------------------------------------------------
    const uint32_t nrec = (uint32_t)min((uint64_t)ENC_TILE, a.n - (uint64_t)t * ENC_TILE);
    for (uint32_t p = tid; p < ptot; p += ENC_TILE) {
        // record owning piece p (last rec with piece[rec] <= p): interpolate,
        // then walk -- exact at once for equal-size records, a few steps
        // otherwise (replaces an 8-step LDS binary search per piece)
        uint32_t rec = (uint32_t)(((uint64_t)p * nrec) / ptot);
        if (rec >= nrec) rec = nrec - 1;
        while (s.piece[rec] > p) --rec;
        while (rec + 1 < nrec && s.piece[rec + 1] <= p) ++rec;
        const uint32_t q = p - s.piece[rec];  // piece within record
        const uint32_t kl = s.klen[rec], vl = s.vlen[rec];
        const uint64_t rsz = 16ull + kl + vl;
        const uint64_t o = tb + s.off[rec] + 16ull * q;  // absolute output byte
        if (o >= a.cap) continue;
        const uint64_t room = a.cap - o;
        uint8_t* dst = a.out + o;
        if (q == 0) {
            uint4 h = make_uint4(kl, 0u, vl, 0u);
            if (room >= 16) {
                *reinterpret_cast<uint4*>(dst) = h;
            } else {
                const uint8_t* hb = reinterpret_cast<const uint8_t*>(&h);
                for (uint32_t i = 0; i < room; ++i) dst[i] = hb[i];
            }
            continue;
        }
        const uint64_t b0 = 16ull * (q - 1);  // body offset
        const uint32_t nb = (uint32_t)min((uint64_t)16, rsz - 16 - b0);
        const uint8_t* sk = a.arena + s.key_off[rec];
        const uint8_t* sv = a.arena + s.val_off[rec];
        if (nb == 16 && room >= 16) {
            if (b0 + 16 <= kl) {
                *reinterpret_cast<uint4*>(dst) = *reinterpret_cast<const uint4*>(sk + b0);
                continue;
            }
            if (b0 >= kl) {
                *reinterpret_cast<uint4*>(dst) = *reinterpret_cast<const uint4*>(sv + (b0 - kl));
                continue;
            }
        }
        store_bytes(dst, sk, kl, sv, b0, nb, room);
    }

    // ---- 4. the last tile to finish its look-back reports the total ------------
    if (tid == 0 && t == a.ntiles - 1) {
        hg_encode_result res;
        res.out_len = tb + tot;
        res.kind = (tb + tot) <= a.cap ? HG_OK : HG_ERR_CAPACITY;
        res.reserved = 0;
        if (a.result->kind != HG_ERR_INTERNAL) *a.result = res;
    }
}

// blocks[b] = {b*stride, rec_off[b*stride], rec_off[min((b+1)*stride, n)] - pos}
__global__ void blocks_kernel(const uint64_t* rec_off, uint64_t n, uint32_t stride,
                              const hg_encode_result* res, hg_block* blocks, uint64_t nb) {
    const uint64_t b = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= nb) return;
    const uint64_t first = b * stride;
    const uint64_t nxt = first + stride;
    const uint64_t pos = rec_off[first];
    const uint64_t end = nxt < n ? rec_off[nxt] : res->out_len;
    hg_block blk;
    blk.first_rec = first;
    blk.position = pos;
    blk.length = end - pos;
    blocks[b] = blk;
}

}  // namespace hgk

extern "C" uint64_t hgk_encode_workspace_bytes(uint64_t n) {
    const uint64_t nt = (n + hgk::ENC_TILE - 1) / hgk::ENC_TILE;
    return (nt + 2) * sizeof(unsigned long long);
}

// d_status: hgk_encode_workspace_bytes(n) bytes.  d_rec_off may be null unless
// d_blocks is requested (the runtime then passes workspace).
extern "C" int hgk_encode_launch(const uint8_t* d_arena, const hg_pair* d_pairs, uint64_t n,
                                 uint8_t* d_out, uint64_t cap, uint64_t* d_rec_off,
                                 uint32_t block_stride, hg_block* d_blocks,
                                 hg_encode_result* d_result, unsigned long long* d_status,
                                 hipStream_t stream) {
    using namespace hgk;
    const uint64_t nt = (n + ENC_TILE - 1) / ENC_TILE;
    if (hipMemsetAsync(d_status, 0, (size_t)(nt + 2) * sizeof(unsigned long long), stream) !=
        hipSuccess)
        return HG_ERR_HIP;
    if (hipMemsetAsync(d_result, 0, sizeof(hg_encode_result), stream) != hipSuccess)
        return HG_ERR_HIP;
    EncodeArgs a;
    a.arena = d_arena;
    a.pairs = d_pairs;
    a.n = n;
    a.out = d_out;
    a.cap = cap;
    a.rec_off = d_rec_off;
    a.result = d_result;
    a.status = d_status;
    a.ticket = reinterpret_cast<uint32_t*>(d_status + nt);
    a.ntiles = (uint32_t)nt;
    hipLaunchKernelGGL(encode_kernel, dim3((uint32_t)nt), dim3(ENC_TILE), 0, stream, a);
    if (hipGetLastError() != hipSuccess) return HG_ERR_HIP;
    if (d_blocks) {
        const uint64_t nb = (n + block_stride - 1) / block_stride;
        const uint32_t grid = (uint32_t)((nb + 255) / 256);
        hipLaunchKernelGGL(blocks_kernel, dim3(grid), dim3(256), 0, stream, d_rec_off, n,
                           block_stride, d_result, d_blocks, nb);
        if (hipGetLastError() != hipSuccess) return HG_ERR_HIP;
    }
    return HG_OK;
}
