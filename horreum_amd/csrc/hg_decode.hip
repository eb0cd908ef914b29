// hg_decode.hip — device-resident SSTable decode (record boundary discovery
// + span emission) for gfx950.
//
// Replaces the serial cursor walk of InternalPair::deserialize_from_bytes
// (reference src/format.rs:50-59) and deserialize_inner (:63-77):
//     off[i+1] = off[i] + 16 + klen[i] + vlen[i]
// is one long dependency chain with no sync points on disk
// (src/sstable/storage.rs:31-32).  Here it becomes a single pass over HBM.
//
// Chunk (16 KiB, one 256-thread workgroup, taken by atomic ticket so chunk
// k-1 is always already running and the look-back cannot deadlock):
//  1. Stage the chunk (+16 B halo) in LDS with 16-byte loads; per-granule
//     zero-byte masks give a bit-parallel header filter (a genuine length
//     field has `hz` zero high bytes, since every record fits in `len`).
//  2. Speculative segmented walk: lane t owns bytes [64t, 64t+64).  It guesses
//     its first record start (first position passing the filter, a full
//     bound check and one step of look-ahead) and walks from it to its
//     segment end: <= 4 records, kept in registers.
//  3. Relaxation: given an entry X, each lane's true entry is its left
//     neighbour's exit; lanes whose guess disagrees re-walk.  Rounds of
//     (read neighbour exit from LDS, barrier) until nothing changes; the
//     fixed point is exact.  Typically 1-2 rounds.
//  4. The chunk entry is speculated (predecessor's published exit if it is
//     already out, else the earliest lane whose guessed chain agrees with
//     the most following lanes) and the chunk publishes AGG(count, entry,
//     exit).  A decoupled look-back (one wave, 63 predecessors per step)
//     yields the exact entry X_k and record base G_k: the nearest INCL
//     predecessor plus the AGGs after it, provided each AGG's guessed entry
//     equals its predecessor's exit (checked with one ballot); a mismatch
//     waits for that chunk's self-corrected INCL.
//  5. If X_k differs from the guess, relax again from X_k (lane walks are
//     reused), publish INCL(G_k + count, exit) and emit spans[G_k + ...]
//     straight from the lane walks.  Format errors and pathological chunks
//     (too many relaxation rounds) fall back to an exact serial walk in LDS.
#include <stdlib.h>

#include "hg_device.hpp"

namespace hgk {

// Chunk geometry is a template parameter (DEC_CHUNK bytes per workgroup of
// DEC_THREADS threads; each lane owns a 64-byte segment).
#define HG_DEC_GEOM                                                               \
    constexpr uint32_t DEC_THREADS = DEC_CHUNK / 64;                             \
    constexpr uint32_t DEC_NW = DEC_THREADS / 64;                                \
    constexpr uint32_t DEC_SEG = 64;                                             \
    constexpr uint32_t DEC_NGRAN = DEC_CHUNK / 16;                               \
    constexpr uint32_t DEC_GPT = DEC_NGRAN / DEC_THREADS;                        \
    constexpr uint32_t DEC_LOG = DEC_CHUNK / 16;                                 \
    (void)DEC_NW; (void)DEC_SEG; (void)DEC_NGRAN; (void)DEC_GPT; (void)DEC_LOG;
constexpr uint32_t DEC_CHUNK_MIN = 4096;
constexpr uint32_t DEC_MAX_ROUNDS = 24;
constexpr uint32_t DEC_CAND_CAP = 16;                   // strong candidates examined per lane
constexpr uint32_t NONE_REL = 0x3FFFFFu;                // "no record starts here"
constexpr uint32_t NO_GUESS = 0xFFFFFFFFu;

enum : uint32_t { ST_NONE = 0, ST_AGG = 1, ST_INCL = 2, ST_ERR = 3 };

struct DecodeArgs {
    const uint8_t* sst;
    uint64_t len;
    hg_span* spans;
    uint64_t cap;
    hg_decode_result* result;
    unsigned long long* status;  // 2 words per chunk, zeroed before launch
    uint32_t* ticket;            // zeroed before launch
    uint32_t nchunks;
    uint32_t hz;                 // zero high bytes required in klen/vlen
    uint32_t* diag;              // DIAG builds only: DIAG_WORDS per chunk
};

// Diagnostic record per chunk (tools/decode_diag.py): phase end stamps
// (s_memtime, relative to the chunk's start) and path facts.
constexpr uint32_t DIAG_WORDS = 12;
enum : uint32_t {
    D_T_LOAD = 0, D_T_SPEC, D_T_RES, D_T_AGG, D_T_LB, D_T_END,
    D_ROUNDS, D_ROUNDS2, D_GUESS, D_SPINS, D_COUNT, D_FLAGS
};

template <uint32_t DEC_CHUNK>
struct DecodeSmem {
    static constexpr uint32_t DEC_THREADS = DEC_CHUNK / 64;
    static constexpr uint32_t DEC_NW = DEC_THREADS / 64;
    uint64_t data64[(DEC_CHUNK + 64) / 8];  // chunk bytes + 16 B halo + read slack
    uint16_t pc[DEC_CHUNK / 16 + 8];        // header-filter masks; later the serial-walk log
    uint64_t sx[2][DEC_THREADS];            // per-lane exits, double-buffered by round
    uint32_t sg[DEC_THREADS];               // per-lane guesses
    uint8_t tgt[DEC_THREADS];               // lane is the target of another lane's exit
    uint32_t bk[DEC_CHUNK / 32];            // "backed": some strong candidate's next lands here
    uint32_t scan_tmp[DEC_NW];
    unsigned long long best, best2;         // entry-heuristic reductions
    uint32_t chunk, walk_n, walk_done, x_count, pred_ok;
    uint64_t pred_exit;
    uint64_t xk, gk, exitk;
    int32_t err_kind;
    uint64_t err_pos;
};

// ---- lane walk --------------------------------------------------------------
// Records starting in [x, segend) (chunk-relative), validated exactly as the
// reference would read them.  dead = a record that cannot be read (the
// reference would fail there).  Exit = first start at or after segend.
struct Walk {
    uint64_t exit;  // absolute
    uint32_t p0, p1, p2, p3;
    uint32_t cnt;
    bool dead;
};

__device__ __forceinline__ void lane_walk(const uint8_t* data, uint64_t base, uint64_t len,
                                          uint32_t x, uint32_t segend, Walk& w) {
    w.cnt = 0;
    w.dead = false;
    uint64_t cur = x;
#pragma unroll
    for (int it = 0; it < 4; ++it) {
        if (cur >= segend) break;
        const uint64_t abs = base + cur;
        if (abs + 16 > len) {
            w.dead = true;
            break;
        }
        uint64_t kl, vl;
        lds_header(data, (uint32_t)cur, kl, vl);
        if (kl > ~0ull - vl || kl + vl > len - abs - 16 || ((kl >> 32) | (vl >> 32))) {
            w.dead = true;
            break;
        }
        if (it == 0) w.p0 = (uint32_t)cur;
        if (it == 1) w.p1 = (uint32_t)cur;
        if (it == 2) w.p2 = (uint32_t)cur;
        if (it == 3) w.p3 = (uint32_t)cur;
        ++w.cnt;
        cur += 16 + kl + vl;
    }
    w.exit = base + cur;
}

// ---- relaxation ---------------------------------------------------------------
// Exact per-lane state for chunk entry X (absolute).  All threads call it.
// Each lane caches one walk (from guess g).  A lane is a pass-through when
// its true entry lies at or past its segment end (a record spans it).
// Seeding: a lane is "on the chain" if it is the entry lane or another
// lane's cached exit lands exactly on its guess; every lane starts from the
// cached exit of the nearest chain lane at or before it (block max-scan), so
// with correct guesses one verification round suffices.  Rounds then re-walk
// lanes whose true entry differs from their guess until nothing changes;
// that fixed point is exact.  Returns false if it did not converge (the
// caller falls back to a serial walk).  On return cnt = this lane's records,
// any_dead says whether the true path hits an unreadable record, and s.exitk
// is the chunk exit.
template <uint32_t DEC_CHUNK>
__device__ bool relax(DecodeSmem<DEC_CHUNK>& s, const uint8_t* data, uint64_t base, uint64_t len,
                      uint32_t clen, uint64_t X, uint32_t& g, Walk& w, uint32_t& cnt,
                      bool& any_dead, uint32_t& rounds) {
    HG_DEC_GEOM
    const uint32_t t = threadIdx.x;
    const uint32_t lane = t & 63u, wid = t >> 6;
    const uint32_t segend = min((t + 1) * DEC_SEG, clen);
    const uint64_t seg_end_abs = base + segend;
    const uint32_t je = (X >= base + clen) ? DEC_THREADS : (uint32_t)((X - base) / DEC_SEG);
    const bool active = t >= je;
    if (t == je && (g == NO_GUESS || base + g != X)) {
        g = (uint32_t)(X - base);
        lane_walk(data, base, len, g, segend, w);
    }
    const bool valid = g != NO_GUESS && !w.dead;
    s.sg[t] = valid ? g : NO_GUESS;
    s.sx[0][t] = valid ? w.exit : ~0ull;
    s.tgt[t] = 0;
    __syncthreads();
    if (active && valid && w.exit < base + clen) {  // link into the lane holding our exit
        const uint32_t u = (uint32_t)((w.exit - base) / DEC_SEG);
        if (s.sg[u] == (uint32_t)(w.exit - base)) s.tgt[u] = 1;
    }
    __syncthreads();
    // nearest chain lane at or before t (inclusive max-scan of lane ids)
    int c = (active && (t == je || (valid && s.tgt[t]))) ? (int)t : -1;
#pragma unroll
    for (uint32_t d = 1; d < 64; d <<= 1) {
        const int o = __shfl_up(c, d, 64);
        if (lane >= d) c = max(c, o);
    }
    if (lane == 63) s.scan_tmp[wid] = (uint32_t)(c + 1);
    __syncthreads();
    for (uint32_t q = 0; q < wid; ++q) c = max(c, (int)s.scan_tmp[q] - 1);
    const uint64_t seed = active ? (c >= 0 ? s.sx[0][c] : ~0ull) : 0;
    __syncthreads();
    s.sx[1][t] = seed;
    __syncthreads();
    bool ok = false, pass = false;
    uint32_t r = 1;
    for (; r <= DEC_MAX_ROUNDS; ++r) {
        const uint64_t* cur = s.sx[r & 1];
        uint64_t* nxt = s.sx[(r + 1) & 1];
        int changed = 0;
        if (active) {
            const uint64_t ein = (t == je) ? X : cur[t - 1];
            uint64_t val;
            if (ein >= seg_end_abs) {  // a record (or the chunk exit) spans this segment
                pass = true;
                val = ein;
            } else {
                pass = false;
                if (g == NO_GUESS || ein != base + g) {  // guess was wrong: walk from the true entry
                    g = (uint32_t)(ein - base);
                    lane_walk(data, base, len, g, segend, w);
                }
                val = w.dead ? ~0ull : w.exit;
            }
            changed = val != cur[t];
            nxt[t] = val;
        } else {
            nxt[t] = 0;
        }
        changed = __syncthreads_or(changed);
        if (!changed) {
            ok = true;
            break;
        }
    }
    rounds = r;
    cnt = (active && !pass) ? w.cnt : 0;
    any_dead = __syncthreads_or(active && !pass && w.dead);
    if (t == DEC_THREADS - 1) s.exitk = s.sx[(r + 1) & 1][t];
    __syncthreads();
    return ok;
}

// ---- look-back ------------------------------------------------------------
struct LookbackOut {
    uint64_t x, g, errpos;
    int32_t err;  // HG_OK or error kind to propagate
};

// Called by all 64 lanes of wave 0.
template <uint32_t DEC_CHUNK>
__device__ LookbackOut lookback(const DecodeArgs& a, uint32_t k, uint32_t& spins_out) {
    const uint32_t lane = threadIdx.x & 63u;
    LookbackOut r{0, 0, 0, HG_OK};
    uint32_t spins = 0;
    const uint32_t SPIN_LIMIT = 1u << 22;
restart:
    int64_t j0 = (int64_t)k - 1;
    uint64_t acc = 0, xk = 0;
    bool first = true;
    for (;;) {
        const int64_t j = j0 - (int64_t)lane;
        unsigned long long w0, w1;
        uint32_t f;
        int fi;
        for (;;) {
            if (j < 0) {  // virtual chunk -1: exact exit 0, 0 records
                w0 = pack_status(ST_INCL, 0, 0);
                w1 = pack_status(ST_INCL, NONE_REL, 0);
            } else {
                w0 = ld_agent(&a.status[2 * j]);
                w1 = ld_agent(&a.status[2 * j + 1]);
            }
            f = st_flag(w0) == st_flag(w1) ? st_flag(w0) : ST_NONE;
            unsigned long long incl = __ballot(f >= ST_INCL);
            unsigned long long notready = __ballot(f == ST_NONE);
            fi = incl ? __ffsll((long long)incl) - 1 : 64;
            unsigned long long relevant = fi >= 63 ? ~0ull : ((1ull << (fi + 1)) - 1ull);
            if (!(notready & relevant)) break;
            if (++spins > SPIN_LIMIT) {
                r.err = HG_ERR_INTERNAL;
                spins_out = spins;
                return r;
            }
            __builtin_amdgcn_s_sleep(1);
        }
        const uint64_t E = st_val(w0);
        if (first) xk = __shfl(E, 0, 64);
        if (fi < 64) {
            const uint32_t fflag = __shfl(f, fi, 64);
            if (fflag == ST_ERR) {  // propagate the first error downstream
                r.err = (int32_t)__shfl(st_aux(w0), fi, 64) - 16;
                r.errpos = __shfl(E, fi, 64);
                r.g = __shfl(st_val(w1), fi, 64);
                spins_out = spins;
                return r;
            }
        }
        // AGG lanes: predicted incoming exit must equal the older neighbour's exit.
        const uint32_t xrel = st_aux(w1);
        const uint64_t P = (xrel != NONE_REL) ? (uint64_t)j * DEC_CHUNK + xrel : E;
        const uint64_t Eolder = __shfl_down(E, 1, 64);
        const int lim = fi < 64 ? fi : 63;  // lanes [0, lim) are checked
        const bool bad = (int)lane < lim && P != Eolder;
        const unsigned long long badm = __ballot(bad);
        if (badm) {
            // The oldest mismatch is a chunk whose guess was wrong; it
            // corrects itself after its own look-back.  Wait for its INCL.
            const int m = 63 - __clzll((long long)badm);
            const int64_t jm = j0 - m;
            for (;;) {
                unsigned long long v0 = ld_agent(&a.status[2 * jm]);
                unsigned long long v1 = ld_agent(&a.status[2 * jm + 1]);
                if (st_flag(v0) == st_flag(v1) && st_flag(v0) >= ST_INCL) break;
                if (++spins > SPIN_LIMIT) {
                    r.err = HG_ERR_INTERNAL;
                    spins_out = spins;
                    return r;
                }
                __builtin_amdgcn_s_sleep(1);
            }
            goto restart;
        }
        const uint32_t c = ((int)lane < lim) ? st_aux(w0) : 0u;
        acc += wave_sum<uint64_t>(c);
        if (fi < 64) {
            r.g = __shfl(st_val(w1), fi, 64) + acc;
            r.x = xk;
            spins_out = spins;
            return r;
        }
        first = false;
        j0 -= 63;  // lane 63 becomes the next window's lane 0
    }
}

// ---- serial count (AGG for chunks the relaxation cannot settle) -------------
// Thread 0 walks the guessed path from absolute x to the chunk end without
// emitting; all threads get (count, exit, dead) through LDS.
template <uint32_t DEC_CHUNK>
__device__ void serial_count(DecodeSmem<DEC_CHUNK>& s, const DecodeArgs& a, uint64_t base, uint32_t clen,
                             uint64_t x, uint64_t& count, uint64_t& exit, bool& dead) {
    HG_DEC_GEOM
    const uint8_t* data = reinterpret_cast<const uint8_t*>(s.data64);
    if (threadIdx.x == 0) {
        uint64_t cur = x, n = 0;
        bool bad = false;
        while (cur < base + clen) {
            if (cur + 16 > a.len) { bad = true; break; }
            uint64_t kl, vl;
            lds_header(data, (uint32_t)(cur - base), kl, vl);
            if (kl > ~0ull - vl || kl + vl > a.len - cur - 16 || ((kl >> 32) | (vl >> 32))) {
                bad = true;
                break;
            }
            ++n;
            cur += 16 + kl + vl;
        }
        s.walk_n = (uint32_t)n;
        s.walk_done = bad;
        s.exitk = cur;
    }
    __syncthreads();
    count = s.walk_n;
    dead = s.walk_done;
    exit = s.exitk;
    __syncthreads();
}

// ---- serial walk (exact; errors and pathological chunks) -------------------
// Thread 0 walks from absolute x, logging up to DEC_LOG starts into s.pc; the
// whole block then emits the batch.
template <uint32_t DEC_CHUNK>
__device__ void serial_walk_emit(DecodeSmem<DEC_CHUNK>& s, const DecodeArgs& a, uint64_t base,
                                 uint32_t clen, uint64_t x, uint64_t g) {
    HG_DEC_GEOM
    const uint8_t* data = reinterpret_cast<const uint8_t*>(s.data64);
    uint64_t emitted = 0;
    if (threadIdx.x == 0) {
        s.err_kind = HG_OK;
        s.exitk = x;
    }
    for (;;) {
        __syncthreads();
        if (threadIdx.x == 0) {
            uint32_t n = 0;
            uint64_t cur = s.exitk;
            bool done = false;
            while (n < DEC_LOG) {
                if (cur >= base + clen) {
                    done = true;
                    break;
                }
                if (cur + 16 > a.len) {
                    s.err_kind = HG_ERR_TRUNCATED_HEADER;
                    done = true;
                    break;
                }
                uint64_t kl, vl;
                lds_header(data, (uint32_t)(cur - base), kl, vl);
                if (kl > ~0ull - vl) {
                    s.err_kind = HG_ERR_LEN_OVERFLOW;
                    done = true;
                    break;
                }
                if (kl + vl > a.len - cur - 16) {
                    s.err_kind = HG_ERR_TRUNCATED_BODY;
                    done = true;
                    break;
                }
                if ((kl >> 32) | (vl >> 32)) {
                    s.err_kind = HG_ERR_SPAN_RANGE;
                    done = true;
                    break;
                }
                s.pc[n++] = (uint16_t)(cur - base);
                cur += 16 + kl + vl;
            }
            s.walk_n = n;
            s.walk_done = done;
            s.exitk = cur;  // next start, or the failing record's start
        }
        __syncthreads();
        const uint32_t n = s.walk_n;
        for (uint32_t t = threadIdx.x; t < n; t += DEC_THREADS) {
            uint32_t p = s.pc[t];
            uint64_t kl, vl;
            lds_header(data, p, kl, vl);
            uint64_t gi = g + emitted + t;
            if (gi < a.cap) {
                uint4 sp;
                uint64_t off = base + p;
                sp.x = (uint32_t)off;
                sp.y = (uint32_t)(off >> 32);
                sp.z = (uint32_t)kl;
                sp.w = (uint32_t)vl;
                *reinterpret_cast<uint4*>(a.spans + gi) = sp;
            }
        }
        emitted += n;
        const bool done = s.walk_done;
        if (done) break;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        s.x_count = (uint32_t)emitted;
        if (s.err_kind != HG_OK) s.err_pos = s.exitk;
    }
    __syncthreads();
}

__device__ __forceinline__ void store_span(hg_span* spans, uint64_t cap, uint64_t gi,
                                           const uint8_t* data, uint64_t base, uint32_t p) {
    if (gi >= cap) return;
    uint64_t kl, vl;
    lds_header(data, p, kl, vl);
    const uint64_t off = base + p;
    uint4 sp;
    sp.x = (uint32_t)off;
    sp.y = (uint32_t)(off >> 32);
    sp.z = (uint32_t)kl;
    sp.w = (uint32_t)vl;
    *reinterpret_cast<uint4*>(spans + gi) = sp;
}


// ---- stride fast path ---------------------------------------------------------
// Header (klen, vlen) at chunk-relative p.
__device__ __forceinline__ bool hdr_eq(const uint8_t* data, uint32_t p, uint64_t kl, uint64_t vl) {
    uint64_t a, b;
    lds_header(data, p, a, b);
    return a == kl && b == vl;
}

// Starts in [X, chunk end) if every record there repeats the header at X:
// record t starts at X + t*R.  All threads call it; one parallel compare per
// record.  Exact: if all headers match, each record's next is the following
// one.  Returns false (not an error) when the run breaks or X cannot be read.
template <uint32_t DEC_CHUNK>
__device__ bool stride_run(DecodeSmem<DEC_CHUNK>& s, const uint8_t* data, uint64_t base, uint64_t len,
                           uint32_t clen, uint64_t X, uint64_t& count, uint64_t& exit,
                           uint64_t& R, uint32_t& rk, uint32_t& rv) {
    HG_DEC_GEOM
    if (X >= base + clen) {  // no record starts in this chunk
        count = 0;
        exit = X;
        R = 0;
        return true;
    }
    const uint32_t xr = (uint32_t)(X - base);
    if (X + 16 > len) return false;
    uint64_t kl, vl;
    lds_header(data, xr, kl, vl);
    if (kl > ~0ull - vl || kl + vl > len - X - 16 || ((kl >> 32) | (vl >> 32))) return false;
    R = 16 + kl + vl;
    const uint64_t m = (clen - xr + R - 1) / R;  // records starting in [xr, clen)
    if (X + m * R > len) return false;          // the last one would not fit
    int bad = 0;
    for (uint64_t t = 1 + threadIdx.x; t < m; t += DEC_THREADS)
        bad |= !hdr_eq(data, xr + (uint32_t)(t * R), kl, vl);
    bad = __syncthreads_or(bad);
    if (bad) return false;
    count = m;
    exit = X + m * R;
    rk = (uint32_t)kl;
    rv = (uint32_t)vl;
    return true;
}

// Header filter bits for the 16 positions of granule gi (from LDS zero masks).
__device__ __forceinline__ uint32_t filter_bits(const uint8_t* data, uint32_t gi, uint32_t hz,
                                                uint32_t clen, uint32_t plim, bool any_valid) {
    const uint4 a = *reinterpret_cast<const uint4*>(data + gi * 16);
    const uint4 b = *reinterpret_cast<const uint4*>(data + gi * 16 + 16);
    const uint32_t m = zmask16(a) | (zmask16(b) << 16);
    uint32_t r = m;
    for (uint32_t sh = 1; sh < hz; ++sh) r &= m >> sh;
    uint32_t c = (r >> (8 - hz)) & (r >> (16 - hz)) & 0xFFFFu;
    const uint32_t p0 = gi * 16;
    if (!any_valid || p0 >= clen || p0 > plim) return 0;
    const uint32_t hi = min(min(plim, clen - 1), p0 + 15);  // last valid p
    const uint32_t nbits = hi - p0 + 1;
    if (nbits < 16) c &= (1u << nbits) - 1u;
    return c;
}

// Wave 0: the first position in the chunk's first KiB whose header repeats
// 3 strides ahead (inside the chunk), or NO_GUESS.
template <uint32_t DEC_CHUNK>
__device__ uint32_t stride_guess(const DecodeSmem<DEC_CHUNK>& s, const uint8_t* data, uint64_t rem,
                                 uint32_t clen, uint32_t hz) {
    HG_DEC_GEOM
    const uint32_t lane = threadIdx.x & 63u;
    const bool any_valid = rem >= 16;
    const uint64_t plim64 = any_valid ? rem - 16 : 0;
    const uint32_t plim = plim64 < 0xFFFFFFFFull ? (uint32_t)plim64 : 0xFFFFFFFFu;
    uint32_t c = filter_bits(data, lane, hz, clen, plim, any_valid);
    uint32_t found = NO_GUESS;
    while (c) {
        const uint32_t b = __ffs(c) - 1;
        c &= c - 1;
        const uint32_t p = lane * 16 + b;
        uint64_t kl, vl;
        lds_header(data, p, kl, vl);
        if ((kl >> 32) | (vl >> 32)) continue;
        const uint64_t R = 16 + kl + vl;
        if (R > rem - p || p + 3 * R >= clen) continue;
        const uint32_t r = (uint32_t)R;
        if (hdr_eq(data, p + r, kl, vl) && hdr_eq(data, p + 2 * r, kl, vl) &&
            hdr_eq(data, p + 3 * r, kl, vl)) {
            found = p;
            break;
        }
    }
    for (int d = 32; d >= 1; d >>= 1) found = min(found, (uint32_t)__shfl_xor((int)found, d, 64));
    return found;
}

// ---- general engine -------------------------------------------------------------
// Header filter, strong candidates, "backed" marks, lane guess and the lane's
// speculative walk (see the file comment).  All threads call it.
template <uint32_t DEC_CHUNK>
__device__ void general_prepare(DecodeSmem<DEC_CHUNK>& s, const uint8_t* data, uint64_t base, uint64_t len,
                                uint64_t rem, uint32_t clen, uint32_t hz, uint32_t& g, Walk& w) {
    HG_DEC_GEOM
    const uint32_t tid = threadIdx.x;
    const bool any_valid = rem >= 16;
    const uint64_t plim64 = any_valid ? rem - 16 : 0;
    const uint32_t plim = plim64 < 0xFFFFFFFFull ? (uint32_t)plim64 : 0xFFFFFFFFu;
#pragma unroll
    for (uint32_t i = 0; i < DEC_GPT; ++i) {
        const uint32_t gi = i * DEC_THREADS + tid;
        s.pc[gi] = (uint16_t)filter_bits(data, gi, hz, clen, plim, any_valid);
    }
    for (uint32_t i = tid; i < DEC_CHUNK / 32; i += DEC_THREADS) s.bk[i] = 0;
    __syncthreads();
    // strong = passes the filter, the exact bound check and one step of
    // look-ahead (next start passes the filter or leaves the chunk).  A true
    // record start is "backed": its predecessor's next lands on it.  Shifted
    // reads of a header (hdr-1, hdr-2, hdr+6 ...) pass the filter too but are
    // almost never backed.
    const uint32_t seg0 = tid * DEC_SEG;
    const uint32_t segend = min(seg0 + DEC_SEG, clen);
    uint64_t strong = 0;
    uint32_t seen = 0;
    for (uint32_t j = 0; j < DEC_GPT && seen < DEC_CAND_CAP; ++j) {
        uint32_t c = s.pc[tid * DEC_GPT + j];
        while (c && seen < DEC_CAND_CAP) {
            const uint32_t b = __ffs(c) - 1;
            c &= c - 1;
            ++seen;
            const uint32_t p = seg0 + j * 16 + b;
            uint64_t kl, vl;
            lds_header(data, p, kl, vl);
            if (((kl >> 32) | (vl >> 32)) || kl + vl > rem - p - 16) continue;
            const uint64_t nx = (uint64_t)p + 16 + kl + vl;
            if (nx < clen) {
                if (!((s.pc[nx >> 4] >> (nx & 15)) & 1u)) continue;  // look-ahead
                atomicOr(&s.bk[nx >> 5], 1u << (nx & 31));
            }
            strong |= 1ull << (j * 16 + b);
        }
    }
    __syncthreads();
    const uint64_t backed = (uint64_t)s.bk[seg0 >> 5] | ((uint64_t)s.bk[(seg0 >> 5) + 1] << 32);
    const uint64_t gm = strong & backed;
    g = gm ? seg0 + (uint32_t)(__ffsll((long long)gm) - 1) : NO_GUESS;
    w.exit = 0;
    w.cnt = 0;
    w.dead = true;
    if (g != NO_GUESS) lane_walk(data, base, len, g, segend, w);
    s.sg[tid] = (g != NO_GUESS && !w.dead) ? g : NO_GUESS;
    // keep the strong mask for the entry guess
    s.sx[0][tid] = strong;
    __syncthreads();
}

// Chunk entry guess from the general engine: the first strong candidate whose
// next start is another lane's guess (the chunk's first record backs its
// second); else the strong candidate with the shortest record (shifted reads
// of a header decode as huge lengths).  ~0 if the chunk has no candidate.
template <uint32_t DEC_CHUNK>
__device__ uint64_t general_entry_guess(DecodeSmem<DEC_CHUNK>& s, const uint8_t* data, uint64_t base,
                                        uint32_t clen, uint32_t /*g*/) {
    HG_DEC_GEOM
    const uint32_t tid = threadIdx.x;
    const uint32_t seg0 = tid * DEC_SEG;
    if (tid == 0) {
        s.best = ~0ull;
        s.best2 = ~0ull;
    }
    uint64_t m = s.sx[0][tid];
    __syncthreads();
    unsigned long long first_link = ~0ull, shortest = ~0ull;
    for (uint32_t it = 0; m && it < DEC_CAND_CAP; ++it) {
        const uint32_t b = __ffsll((long long)m) - 1;
        m &= m - 1;
        const uint32_t p = seg0 + b;
        uint64_t kl, vl;
        lds_header(data, p, kl, vl);
        const uint64_t nx = (uint64_t)p + 16 + kl + vl;
        if (nx < clen && s.sg[nx / DEC_SEG] == (uint32_t)nx) {
            first_link = p;
            break;
        }
        const unsigned long long key = ((16 + kl + vl) << 16) | p;
        shortest = key < shortest ? key : shortest;
    }
    for (int d = 32; d >= 1; d >>= 1) {
        const unsigned long long o1 = __shfl_xor(first_link, d, 64);
        const unsigned long long o2 = __shfl_xor(shortest, d, 64);
        first_link = o1 < first_link ? o1 : first_link;
        shortest = o2 < shortest ? o2 : shortest;
    }
    if ((tid & 63) == 0) {
        atomicMin(&s.best, first_link);
        atomicMin(&s.best2, shortest);
    }
    __syncthreads();
    const unsigned long long b1 = s.best, b2 = s.best2;
    __syncthreads();
    if (b1 != ~0ull) return base + b1;
    if (b2 != ~0ull) return base + (b2 & 0xFFFFu);
    return ~0ull;
}

template <uint32_t DEC_CHUNK, bool DIAG>
__global__ __launch_bounds__(DEC_CHUNK / 64) void decode_kernel(DecodeArgs a) {
    HG_DEC_GEOM
    __shared__ DecodeSmem<DEC_CHUNK> s;
    const uint32_t tid = threadIdx.x;
    uint8_t* data = reinterpret_cast<uint8_t*>(s.data64);
    uint64_t t_start = 0;
    uint32_t* dg = nullptr;
#define HG_STAMP(slot)                                                                      \
    do {                                                                                    \
        if (DIAG && tid == 0) dg[slot] = (uint32_t)(__builtin_amdgcn_s_memtime() - t_start); \
    } while (0)

    if (tid == 0) s.chunk = atomicAdd(a.ticket, 1u);
    __syncthreads();
    const uint32_t k = s.chunk;
    if (DIAG) {
        t_start = __builtin_amdgcn_s_memtime();
        dg = a.diag + (size_t)k * DIAG_WORDS;
    }
    const uint64_t base = (uint64_t)k * DEC_CHUNK;
    const uint64_t rem = a.len - base;  // bytes from chunk start to end of input
    const uint32_t clen = rem < DEC_CHUNK ? (uint32_t)rem : DEC_CHUNK;

    // ---- 1. stage chunk (+16 B halo) in LDS ------------------------------------
    const bool full = rem >= (uint64_t)DEC_CHUNK + 16;
    uint4 v[DEC_GPT];
#pragma unroll
    for (uint32_t i = 0; i < DEC_GPT; ++i) {
        const uint32_t off = (i * DEC_THREADS + tid) * 16;
        if (full || off + 16 <= rem) {
            v[i] = *reinterpret_cast<const uint4*>(a.sst + base + off);
        } else {
            uint8_t tmp[16];
#pragma unroll
            for (int b = 0; b < 16; ++b) tmp[b] = (off + b < rem) ? a.sst[base + off + b] : 0;
            v[i] = *reinterpret_cast<uint4*>(tmp);
        }
    }
#pragma unroll
    for (uint32_t i = 0; i < DEC_GPT; ++i)
        *reinterpret_cast<uint4*>(data + (i * DEC_THREADS + tid) * 16) = v[i];
    if (tid < 4) {  // halo granule (16 B) + zeroed read slack
        const uint32_t off = DEC_CHUNK + tid * 16;
        uint4 h = make_uint4(0, 0, 0, 0);
        if (tid == 0) {
            if (full) {
                h = *reinterpret_cast<const uint4*>(a.sst + base + off);
            } else {
                uint8_t tmp[16];
#pragma unroll
                for (int b = 0; b < 16; ++b)
                    tmp[b] = ((uint64_t)off + b < rem) ? a.sst[base + off + b] : 0;
                h = *reinterpret_cast<uint4*>(tmp);
            }
        }
        *reinterpret_cast<uint4*>(data + off) = h;
    }
    if (tid == 0) {  // is the predecessor's exit already published?
        s.pred_ok = k == 0;
        s.pred_exit = 0;
        if (k > 0) {
            unsigned long long v0 = ld_agent(&a.status[2 * (k - 1)]);
            unsigned long long v1 = ld_agent(&a.status[2 * (k - 1) + 1]);
            if (st_flag(v0) == st_flag(v1) && (st_flag(v0) == ST_AGG || st_flag(v0) == ST_INCL)) {
                s.pred_ok = 1;
                s.pred_exit = st_val(v0);
            }
        }
    }
    __syncthreads();
    HG_STAMP(D_T_LOAD);

    const uint32_t hz = a.hz;

    // ---- 2. entry guess: predecessor's exit, else a stride-consistent head record
    uint64_t X = ~0ull;
    bool have = false;
    if (s.pred_ok) {
        X = s.pred_exit;
        have = true;
    } else {
        if (tid < 64) {
            const uint32_t f = stride_guess(s, data, rem, clen, hz);
            if (tid == 0) s.walk_n = f;
        }
        __syncthreads();
        if (s.walk_n != NO_GUESS) {
            X = base + s.walk_n;
            have = true;
        }
    }

    // ---- 3. path for the guess: one stride run, else the general engine -------
    uint64_t gcount = 0, gexit = 0;
    uint32_t rk = 0, rv = 0;  // stride run's key/value lengths
    uint64_t rlen = 0;        // stride run's record length
    bool stride_ok = false, conv = false, any_dead = false, gen_ready = false;
    uint32_t g = NO_GUESS, cnt = 0, prefix = 0, rounds = 0, rounds2 = 0, mode = 0;
    Walk w;
    w.exit = 0;
    w.cnt = 0;
    w.dead = true;
    w.p0 = w.p1 = w.p2 = w.p3 = 0;
    if (have) stride_ok = stride_run(s, data, base, a.len, clen, X, gcount, gexit, rlen, rk, rv);
    if (!stride_ok) {
        general_prepare(s, data, base, a.len, rem, clen, hz, g, w);
        gen_ready = true;
        if (!have) {
            X = general_entry_guess(s, data, base, clen, g);
            have = X != ~0ull;
        }
        if (have) {
            conv = relax(s, data, base, a.len, clen, X, g, w, cnt, any_dead, rounds);
            uint32_t tot;
            prefix = block_excl_scan<DEC_NW>(cnt, s.scan_tmp, tot);
            gcount = tot;
            gexit = X >= base + clen ? X : s.exitk;
            if (!conv) {  // still publish an AGG so successors are not serialised behind us
                bool dead = false;
                serial_count(s, a, base, clen, X, gcount, gexit, dead);
                any_dead = dead;
            }
            if (any_dead) have = false;
        }
    }
    HG_STAMP(D_T_RES);
    if (have && tid == 0) {
        const uint32_t xrel = X < base + clen ? (uint32_t)(X - base) : NONE_REL;
        st_agent(&a.status[2 * k + 1], pack_status(ST_AGG, xrel, 0));
        st_agent(&a.status[2 * k], pack_status(ST_AGG, (uint32_t)gcount, gexit));
    }
    HG_STAMP(D_T_AGG);

    // ---- 4. look-back (wave 0) ----------------------------------------------------
    if (tid < 64) {
        uint32_t spins = 0;
        LookbackOut lb = lookback<DEC_CHUNK>(a, k, spins);
        if (tid == 0) {
            s.xk = lb.x;
            s.gk = lb.g;
            s.err_kind = lb.err;
            s.err_pos = lb.errpos;
            if (DIAG) dg[D_SPINS] = spins;
        }
    }
    __syncthreads();
    HG_STAMP(D_T_LB);

    const int32_t perr = s.err_kind;
    const uint64_t xk = s.xk, gk = s.gk;
    int32_t kind = HG_OK;
    uint64_t errpos = 0, count = 0, exitk = 0;
    if (perr != HG_OK) {  // an earlier chunk failed: propagate, emit nothing
        kind = perr;
        errpos = s.err_pos;
    } else {
        // ---- 5. exact path from X_k -------------------------------------------------
        // mode 1: stride run, 2: relaxed lanes, 3: serial walk
        if (have && xk == X && stride_ok) {
            mode = 1;
        } else if (have && xk == X && conv) {
            mode = 2;
        } else {
            stride_ok = stride_run(s, data, base, a.len, clen, xk, gcount, gexit, rlen, rk, rv);
            if (stride_ok) {
                mode = 1;
            } else {
                if (!gen_ready) general_prepare(s, data, base, a.len, rem, clen, hz, g, w);
                any_dead = false;
                conv = relax(s, data, base, a.len, clen, xk, g, w, cnt, any_dead, rounds2);
                uint32_t tot;
                prefix = block_excl_scan<DEC_NW>(cnt, s.scan_tmp, tot);
                gcount = tot;
                gexit = xk >= base + clen ? xk : s.exitk;
                mode = (conv && !any_dead) ? 2 : 3;
            }
        }
        if (mode != 3) {
            count = gcount;
            exitk = gexit;
            if (tid == 0) {
                st_agent(&a.status[2 * k + 1],
                         pack_status(ST_INCL, xk < base + clen ? (uint32_t)(xk - base) : NONE_REL,
                                     gk + count));
                st_agent(&a.status[2 * k], pack_status(ST_INCL, (uint32_t)count, exitk));
            }
        }
        // ---- 6. emission ------------------------------------------------------------
        if (mode == 1) {  // arithmetic: record t starts at X_k + t*R
            for (uint32_t t = tid; t < count; t += DEC_THREADS) {
                const uint64_t gi = gk + t;
                if (gi < a.cap) {
                    const uint64_t off = xk + (uint64_t)t * rlen;
                    uint4 sp;
                    sp.x = (uint32_t)off;
                    sp.y = (uint32_t)(off >> 32);
                    sp.z = rk;
                    sp.w = rv;
                    *reinterpret_cast<uint4*>(a.spans + gi) = sp;
                }
            }
        } else if (mode == 2) {  // straight from the lane walks
            const uint64_t gi = gk + prefix;
            if (cnt > 0) store_span(a.spans, a.cap, gi, data, base, w.p0);
            if (cnt > 1) store_span(a.spans, a.cap, gi + 1, data, base, w.p1);
            if (cnt > 2) store_span(a.spans, a.cap, gi + 2, data, base, w.p2);
            if (cnt > 3) store_span(a.spans, a.cap, gi + 3, data, base, w.p3);
        } else {
            serial_walk_emit(s, a, base, clen, xk, gk);
            count = s.x_count;
            kind = s.err_kind;
            errpos = s.err_pos;
            exitk = s.exitk;
            if (tid == 0) {
                if (kind == HG_OK) {
                    st_agent(&a.status[2 * k + 1],
                             pack_status(ST_INCL,
                                         xk < base + clen ? (uint32_t)(xk - base) : NONE_REL,
                                         gk + count));
                    st_agent(&a.status[2 * k], pack_status(ST_INCL, (uint32_t)count, exitk));
                } else {
                    st_agent(&a.status[2 * k + 1], pack_status(ST_ERR, 0, gk + count));
                    st_agent(&a.status[2 * k],
                             pack_status(ST_ERR, (uint32_t)(kind + 16), errpos));
                }
            }
        }
    }
    if (perr != HG_OK && tid == 0) {
        st_agent(&a.status[2 * k + 1], pack_status(ST_ERR, 0, gk));
        st_agent(&a.status[2 * k], pack_status(ST_ERR, (uint32_t)(kind + 16), errpos));
    }
    HG_STAMP(D_T_END);
    if (DIAG && tid == 0) {
        dg[D_T_SPEC] = mode;
        dg[D_ROUNDS] = rounds;
        dg[D_ROUNDS2] = rounds2;
        dg[D_GUESS] = (have ? 1u : 0u) | (s.pred_ok ? 2u : 0u) | ((have && xk == X) ? 4u : 0u);
        dg[D_COUNT] = (uint32_t)count;
        dg[D_FLAGS] = (perr != HG_OK ? 2u : 0u) | (kind != HG_OK ? 4u : 0u) |
                      (gen_ready ? 8u : 0u);
    }
#undef HG_STAMP
    // ---- 7. the last chunk reports the whole-file result ----------------------
    if (tid == 0 && k == a.nchunks - 1) {
        hg_decode_result r;
        r.n_records = gk + count;
        r.kind = kind;
        r.reserved = 0;
        r.err_offset = kind != HG_OK ? errpos : 0;
        *a.result = r;
    }
}

}  // namespace hgk

// d_status must hold hgk_decode_workspace_bytes(len) bytes; the launcher
// zeroes the statuses and the ticket word that follows them.  chunk selects
// the geometry (4096, 8192 or 16384 bytes per workgroup).
extern "C" int hgk_decode_launch_variant(const uint8_t* d_sst, uint64_t len, hg_span* d_spans,
                                         uint64_t cap, hg_decode_result* d_result,
                                         unsigned long long* d_status, uint32_t* d_diag,
                                         uint32_t chunk, hipStream_t stream) {
    using namespace hgk;
    if (chunk != 4096 && chunk != 8192 && chunk != 16384) return HG_ERR_INVALID_ARG;
    const uint64_t nch = (len + chunk - 1) / chunk;
    // Zero high bytes every genuine length field must have: any record fits
    // in len bytes, so klen, vlen < 2^(8*nb) with nb = bytes needed for len.
    uint32_t nb = 0;
    for (uint64_t x = len; x; x >>= 8) ++nb;
    DecodeArgs a;
    a.sst = d_sst;
    a.len = len;
    a.spans = d_spans;
    a.cap = cap;
    a.result = d_result;
    a.status = d_status;
    a.ticket = reinterpret_cast<uint32_t*>(d_status + 2 * nch);
    a.nchunks = (uint32_t)nch;
    a.hz = 8 - nb;
    a.diag = d_diag;
    hipError_t e = hipMemsetAsync(d_status, 0, (size_t)(2 * nch + 2) * sizeof(unsigned long long),
                                  stream);
    if (e != hipSuccess) return HG_ERR_HIP;
    const dim3 grid((uint32_t)nch);
#define HG_LAUNCH(C)                                                                          \
    if (chunk == C) {                                                                         \
        if (d_diag)                                                                           \
            hipLaunchKernelGGL((decode_kernel<C, true>), grid, dim3(C / 64), 0, stream, a);   \
        else                                                                                  \
            hipLaunchKernelGGL((decode_kernel<C, false>), grid, dim3(C / 64), 0, stream, a);  \
    }
    HG_LAUNCH(4096)
    HG_LAUNCH(8192)
    HG_LAUNCH(16384)
#undef HG_LAUNCH
    return hipGetLastError() == hipSuccess ? HG_OK : HG_ERR_HIP;
}

static uint32_t default_chunk() {
    static uint32_t c = 0;
    if (!c) {
        const char* e = getenv("HG_DECODE_CHUNK");
        c = e ? (uint32_t)atoi(e) : 16384u;
        if (c != 4096 && c != 8192 && c != 16384) c = 16384;
    }
    return c;
}

extern "C" int hgk_decode_launch_diag(const uint8_t* d_sst, uint64_t len, hg_span* d_spans,
                                      uint64_t cap, hg_decode_result* d_result,
                                      unsigned long long* d_status, uint32_t* d_diag,
                                      hipStream_t stream) {
    return hgk_decode_launch_variant(d_sst, len, d_spans, cap, d_result, d_status, d_diag,
                                     default_chunk(), stream);
}

extern "C" int hgk_decode_launch(const uint8_t* d_sst, uint64_t len, hg_span* d_spans,
                                 uint64_t cap, hg_decode_result* d_result,
                                 unsigned long long* d_status, hipStream_t stream) {
    return hgk_decode_launch_diag(d_sst, len, d_spans, cap, d_result, d_status, nullptr, stream);
}

extern "C" uint64_t hgk_decode_workspace_bytes(uint64_t len) {
    const uint64_t nch = (len + hgk::DEC_CHUNK_MIN - 1) / hgk::DEC_CHUNK_MIN;
    return (2 * nch + 2) * sizeof(unsigned long long);
}
