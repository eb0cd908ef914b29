// hg_decode.hip — device-resident SSTable decode (record boundary discovery
// + span emission) for gfx950.
//
// Replaces the serial cursor walk of InternalPair::deserialize_from_bytes
// (reference src/format.rs:50-59) and deserialize_inner (:63-77):
//     off[i+1] = off[i] + 16 + klen[i] + vlen[i]
// is one long dependency chain with no sync points on disk
// (src/sstable/storage.rs:31-32).  Here it becomes a single pass over HBM:
//
//  1. Each 256-thread workgroup takes a 16 KiB chunk by atomic ticket (so
//     chunk k-1 is always already running: the look-back below cannot
//     deadlock) and stages it in LDS with 16-byte loads.
//  2. Candidate headers: a bit-parallel zero-byte filter (a header's length
//     fields must have `hz` zero high bytes for any record that fits in
//     `len` bytes), then a full bound check, then one level of pruning
//     (next(p) must itself pass the filter or leave the chunk).  Survivors are
//     compacted in position order by a block prefix scan of per-granule
//     popcounts (ballot-free: each lane owns 16-bit granule masks).
//  3. Binary lifting over survivor next-pointers in LDS: J_k = J_{k-1}∘J_{k-1},
//     saturating at terminal nodes (EXIT = next leaves the chunk, DEAD = next
//     is not a survivor).  Any path's length/last node is O(log) lookups and
//     the t-th node of a path is O(log) lookups, so a lane per record can emit.
//  4. Speculative entry: the predecessor's published exit if it is already
//     out, else the head survivor with the longest EXIT-terminated path.  The
//     chunk publishes AGG(count, guessed entry, exit).
//  5. Decoupled look-back (one wave, 63 predecessors per step): the exact
//     entry X_k and record base G_k follow from the nearest INCL predecessor
//     and the chain of AGG statuses after it, provided each AGG's guessed
//     entry equals its predecessor's exit (checked in parallel); a mismatch
//     waits for that chunk's self-corrected INCL.
//  6. With X_k exact: recompute the path if the guess was wrong, publish
//     INCL(G_k + count, exit), and emit spans[G_k + t] (16 B per lane,
//     coalesced).  Errors, over-dense chunks and over-long paths fall back
//     to an exact serial walk in LDS with batched emission.
#include "hg_device.hpp"

namespace hgk {

constexpr uint32_t DEC_CHUNK = 16384;
constexpr uint32_t DEC_THREADS = 256;
constexpr uint32_t DEC_NW = DEC_THREADS / 64;
constexpr uint32_t DEC_NGRAN = DEC_CHUNK / 16;          // 1024 granules of 16 B
constexpr uint32_t DEC_GPT = DEC_NGRAN / DEC_THREADS;   // 4 granules per thread
constexpr uint32_t DEC_CAP = 1024;                      // survivors for the lifting path
constexpr uint32_t DEC_KMAX = 10;                       // lifting levels
constexpr uint32_t NONE_REL = 0x3FFFFFu;                // "no record starts here"

enum : uint32_t { ST_NONE = 0, ST_AGG = 1, ST_INCL = 2, ST_ERR = 3 };
enum : uint8_t { T_INNER = 0, T_EXIT = 1, T_DEAD = 2 };

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
    D_T_LOAD = 0, D_T_SURV, D_T_LIFT, D_T_AGG, D_T_LB, D_T_END,
    D_NSURV, D_NLEV, D_GUESS, D_SPINS, D_COUNT, D_FLAGS
};

struct DecodeSmem {
    uint64_t data64[(DEC_CHUNK + 64) / 8];  // chunk bytes + 16 B halo + read slack
    uint16_t zm[DEC_NGRAN + 8];             // zero masks, later survivor masks
    uint16_t pc[DEC_NGRAN + 8];             // pre-candidate masks
    uint16_t pre[DEC_NGRAN + 8];            // exclusive survivor prefix per granule
    uint16_t pos[DEC_CAP];                  // survivor positions (also the serial-walk log)
    uint16_t J[DEC_KMAX][DEC_CAP];          // lifting tables
    uint8_t term[DEC_CAP];
    uint32_t scan_tmp[DEC_NW];
    uint32_t chunk, nsurv, nlev, slow;
    uint32_t x_idx, x_count, x_last;  // resolved path (lifting mode)
    uint32_t walk_n, walk_done;
    uint64_t xk, gk, exitk;
    uint32_t err_kind;
    uint64_t err_pos;
};

// ---- lifting queries (any thread) ----------------------------------------
// Number of nodes on the path from survivor x to its terminal, and the
// terminal itself.
__device__ __forceinline__ void path_len(const DecodeSmem& s, uint32_t x, uint32_t& count,
                                         uint32_t& last) {
    if (s.term[x] != T_INNER) {
        count = 1;
        last = x;
        return;
    }
    uint32_t y = x, steps = 0;
    for (int k = (int)s.nlev - 1; k >= 0; --k) {
        uint32_t z = s.J[k][y];
        if (s.term[z] == T_INNER) {
            y = z;
            steps += 1u << k;
        }
    }
    last = s.J[0][y];
    count = steps + 2;
}

__device__ __forceinline__ uint32_t path_node(const DecodeSmem& s, uint32_t x, uint32_t t) {
    uint32_t y = x;
    for (uint32_t k = 0; t; ++k, t >>= 1)
        if (t & 1u) y = s.J[k][y];
    return y;
}

// Exit position (absolute) of an EXIT terminal: next record start.
__device__ __forceinline__ uint64_t node_next_abs(const DecodeSmem& s, uint64_t base,
                                                  uint32_t node) {
    uint64_t k, v;
    uint32_t p = s.pos[node];
    lds_header(reinterpret_cast<const uint8_t*>(s.data64), p, k, v);
    return base + p + 16 + k + v;
}

// Survivor index of chunk-relative position p, or UINT32_MAX.
__device__ __forceinline__ uint32_t surv_index(const DecodeSmem& s, uint32_t p) {
    uint32_t g = p >> 4, b = p & 15u;
    uint32_t m = s.zm[g];
    if (!((m >> b) & 1u)) return 0xFFFFFFFFu;
    return s.pre[g] + __popc(m & ((1u << b) - 1u));
}

// ---- look-back ------------------------------------------------------------
struct LookbackOut {
    uint64_t x, g, errpos;
    uint32_t err;  // HG_OK or error kind to propagate
};

// Called by all 64 lanes of wave 0.
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
                { spins_out = spins; return r; }
            }
            __builtin_amdgcn_s_sleep(2);
        }
        const uint64_t E = st_val(w0);
        if (first) xk = __shfl(E, 0, 64);
        if (fi < 64) {
            const uint32_t fflag = __shfl(f, fi, 64);
            if (fflag == ST_ERR) {  // propagate the first error downstream
                r.err = __shfl(st_aux(w0), fi, 64);
                r.errpos = __shfl(E, fi, 64);
                r.g = __shfl(st_val(w1), fi, 64);
                { spins_out = spins; return r; }
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
                    { spins_out = spins; return r; }
                }
                __builtin_amdgcn_s_sleep(2);
            }
            goto restart;
        }
        const uint32_t c = ((int)lane < lim) ? st_aux(w0) : 0u;
        acc += wave_sum<uint64_t>(c);
        if (fi < 64) {
            r.g = __shfl(st_val(w1), fi, 64) + acc;
            r.x = xk;
            { spins_out = spins; return r; }
        }
        first = false;
        j0 -= 63;  // lane 63 becomes the next window's lane 0
    }
}

// ---- serial walk (exact; errors, dense chunks, long paths) -----------------
// Thread 0 walks from absolute x, logging up to DEC_CAP starts into s.pos;
// the whole block then emits the batch.  Returns via s.* fields.
__device__ void serial_walk_emit(DecodeSmem& s, const DecodeArgs& a, uint64_t base,
                                 uint32_t clen, uint64_t x, uint64_t g) {
    const uint8_t* data = reinterpret_cast<const uint8_t*>(s.data64);
    uint64_t emitted = 0;
    if (threadIdx.x == 0) {
        s.err_kind = HG_OK;
        s.exitk = x;
    }
    for (;;) {
        if (threadIdx.x == 0) {
            uint32_t n = 0;
            uint64_t cur = s.exitk;
            bool done = false;
            while (n < DEC_CAP) {
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
                s.pos[n++] = (uint16_t)(cur - base);
                cur += 16 + kl + vl;
            }
            s.walk_n = n;
            s.walk_done = done;
            s.exitk = cur;  // next start, or the failing record's start
        }
        __syncthreads();
        const uint32_t n = s.walk_n;
        for (uint32_t t = threadIdx.x; t < n; t += DEC_THREADS) {
            uint32_t p = s.pos[t];
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
        __syncthreads();
        if (done) break;
    }
    if (threadIdx.x == 0) {
        s.x_count = (uint32_t)emitted;
        if (s.err_kind != HG_OK) s.err_pos = s.exitk;
    }
    __syncthreads();
}

template <bool DIAG>
__global__ __launch_bounds__(DEC_THREADS) void decode_kernel(DecodeArgs a) {
    __shared__ DecodeSmem s;
    const uint32_t tid = threadIdx.x;
    uint8_t* data = reinterpret_cast<uint8_t*>(s.data64);
    uint64_t t_start = 0;
    uint32_t* dg = nullptr;
#define HG_STAMP(slot)                                                              \
    do {                                                                            \
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

    // ---- 1. stage chunk (+16 B halo) in LDS, zero masks from registers -----
    const bool full = rem >= (uint64_t)DEC_CHUNK + 16;
#pragma unroll
    for (uint32_t i = 0; i < DEC_GPT; ++i) {
        const uint32_t g = i * DEC_THREADS + tid;
        const uint32_t off = g * 16;
        uint4 v;
        if (full || off + 16 <= rem) {
            v = *reinterpret_cast<const uint4*>(a.sst + base + off);
        } else {
            uint8_t tmp[16];
#pragma unroll
            for (int b = 0; b < 16; ++b) tmp[b] = (off + b < rem) ? a.sst[base + off + b] : 0;
            v = *reinterpret_cast<uint4*>(tmp);
        }
        *reinterpret_cast<uint4*>(data + off) = v;
        s.zm[g] = (uint16_t)zmask16(v);
    }
    if (tid < 4) {  // halo granule (16 B) + zeroed read slack
        const uint32_t off = DEC_CHUNK + tid * 16;
        uint4 v = make_uint4(0, 0, 0, 0);
        if (tid == 0) {
            if (full) {
                v = *reinterpret_cast<const uint4*>(a.sst + base + off);
            } else {
                uint8_t tmp[16];
#pragma unroll
                for (int b = 0; b < 16; ++b)
                    tmp[b] = ((uint64_t)off + b < rem) ? a.sst[base + off + b] : 0;
                v = *reinterpret_cast<uint4*>(tmp);
            }
            s.zm[DEC_NGRAN] = (uint16_t)zmask16(v);
        }
        *reinterpret_cast<uint4*>(data + off) = v;
    }
    __syncthreads();
    HG_STAMP(D_T_LOAD);

    // ---- 2a. pre-candidate masks (zero-pattern filter) ----------------------
    // Positions p with base+p+16 > len can never start a record.
    const uint64_t plim64 = rem >= 16 ? rem - 16 : 0;  // valid p <= plim (if rem >= 16)
    const uint32_t plim = plim64 < 0xFFFFFFFFull ? (uint32_t)plim64 : 0xFFFFFFFFu;
    const bool any_valid = rem >= 16;
    const uint32_t hz = a.hz;
#pragma unroll
    for (uint32_t j = 0; j < DEC_GPT; ++j) {
        const uint32_t g = tid * DEC_GPT + j;
        const uint32_t m = (uint32_t)s.zm[g] | ((uint32_t)s.zm[g + 1] << 16);
        uint32_t r = m;
        for (uint32_t sh = 1; sh < hz; ++sh) r &= m >> sh;
        uint32_t c = hz ? ((r >> (8 - hz)) & (r >> (16 - hz)) & 0xFFFFu) : 0xFFFFu;
        const uint32_t p0 = g * 16;
        if (!any_valid || p0 >= clen || p0 > plim) {
            c = 0;
        } else {
            const uint32_t hi = min(min(plim, clen - 1), p0 + 15);  // last valid p
            const uint32_t nb = hi - p0 + 1;
            if (nb < 16) c &= (1u << nb) - 1u;
        }
        s.pc[g] = (uint16_t)c;
    }
    if (tid == 0) s.pc[DEC_NGRAN] = 0;
    __syncthreads();

    // ---- 2b. bound check + one-level pruning -> survivor masks --------------
    uint32_t cnt = 0;
    uint32_t svm[DEC_GPT];
#pragma unroll
    for (uint32_t j = 0; j < DEC_GPT; ++j) {
        const uint32_t g = tid * DEC_GPT + j;
        uint32_t c = s.pc[g], sv = 0;
        while (c) {
            const uint32_t b = __ffs(c) - 1;
            c &= c - 1;
            const uint32_t p = g * 16 + b;
            uint64_t kl, vl;
            lds_header(data, p, kl, vl);
            // klen, vlen < 2^40 here (filter), so no overflow below.
            bool ok = ((kl >> 32) | (vl >> 32)) == 0 && kl + vl <= rem - p - 16;
            if (ok) {
                const uint64_t nx = (uint64_t)p + 16 + kl + vl;
                if (nx < clen) ok = (s.pc[nx >> 4] >> (nx & 15)) & 1u;
            }
            sv |= (uint32_t)ok << b;
        }
        svm[j] = sv;
        cnt += __popc(sv);
    }
    __syncthreads();  // all reads of zm done before it is reused for survivors
#pragma unroll
    for (uint32_t j = 0; j < DEC_GPT; ++j) s.zm[tid * DEC_GPT + j] = (uint16_t)svm[j];
    uint32_t total;
    uint32_t ex = block_excl_scan<DEC_NW>(cnt, s.scan_tmp, total);
#pragma unroll
    for (uint32_t j = 0; j < DEC_GPT; ++j) {
        s.pre[tid * DEC_GPT + j] = (uint16_t)ex;
        ex += __popc(svm[j]);
    }
    if (tid == 0) {
        s.nsurv = total;
        s.slow = total > DEC_CAP;
        s.zm[DEC_NGRAN] = 0;
    }
    __syncthreads();
    HG_STAMP(D_T_SURV);
    const uint32_t N = s.nsurv;
    bool lifting = !s.slow;

    // ---- 3. survivor table + level-0 next pointers --------------------------
    if (lifting) {
#pragma unroll
        for (uint32_t j = 0; j < DEC_GPT; ++j) {
            const uint32_t g = tid * DEC_GPT + j;
            uint32_t c = svm[j];
            uint32_t idx = s.pre[g];
            while (c) {
                const uint32_t b = __ffs(c) - 1;
                c &= c - 1;
                const uint32_t p = g * 16 + b;
                uint64_t kl, vl;
                lds_header(data, p, kl, vl);
                const uint64_t nx = (uint64_t)p + 16 + kl + vl;
                uint32_t nxt = idx;
                uint8_t t = T_EXIT;
                if (nx < clen) {
                    const uint32_t ni = surv_index(s, (uint32_t)nx);
                    if (ni != 0xFFFFFFFFu) {
                        nxt = ni;
                        t = T_INNER;
                    } else {
                        t = T_DEAD;
                    }
                }
                s.pos[idx] = (uint16_t)p;
                s.J[0][idx] = (uint16_t)nxt;
                s.term[idx] = t;
                ++idx;
            }
        }
        __syncthreads();
        // ---- 4. binary lifting until every J_{K-1} is terminal ---------------
        uint32_t K = 1;
        for (;;) {
            int any = 0;
            for (uint32_t i = tid; i < N; i += DEC_THREADS) any |= s.term[s.J[K - 1][i]] == T_INNER;
            any = __syncthreads_or(any);
            if (!any) break;
            if (K == DEC_KMAX) {
                lifting = false;
                break;
            }
            for (uint32_t i = tid; i < N; i += DEC_THREADS) s.J[K][i] = s.J[K - 1][s.J[K - 1][i]];
            __syncthreads();
            ++K;
        }
        if (tid == 0) s.nlev = K;
        __syncthreads();
    }
    HG_STAMP(D_T_LIFT);
    if (DIAG && tid == 0) {
        dg[D_NSURV] = N;
        dg[D_NLEV] = lifting ? s.nlev : 0;
    }

    // ---- 5. speculative entry + AGG publish (wave 0) ---------------------------
    if (tid < 64) {
        const uint32_t lane = tid;
        uint64_t gexit = 0;
        uint32_t gcount = 0, gxrel = NONE_REL;
        bool have = false;
        if (lifting) {
            uint64_t pe = 0;
            bool pred = false;
            if (k == 0) {
                pred = true;
            } else {
                unsigned long long v0 = ld_agent(&a.status[2 * (k - 1)]);
                unsigned long long v1 = ld_agent(&a.status[2 * (k - 1) + 1]);
                if (st_flag(v0) == st_flag(v1) &&
                    (st_flag(v0) == ST_AGG || st_flag(v0) == ST_INCL)) {
                    pred = true;
                    pe = st_val(v0);
                }
            }
            if (pred) {
                if (pe >= base + clen) {  // a record spans this whole chunk
                    have = true;
                    gexit = pe;
                    gcount = 0;
                    gxrel = NONE_REL;
                } else {
                    const uint32_t xi = surv_index(s, (uint32_t)(pe - base));
                    if (xi != 0xFFFFFFFFu) {
                        uint32_t c, last;
                        path_len(s, xi, c, last);
                        if (s.term[last] == T_EXIT) {
                            have = true;
                            gcount = c;
                            gxrel = (uint32_t)(pe - base);
                            gexit = node_next_abs(s, base, last);
                        }
                    }
                }
            }
            if (!have) {  // heuristic: longest EXIT-terminated path among the first 64
                uint64_t key = 0;
                uint32_t c = 0, last = 0;
                if (lane < N) {
                    path_len(s, lane, c, last);
                    if (s.term[last] == T_EXIT) key = ((uint64_t)c << 16) | (0xFFFFu - lane);
                }
                for (int d = 32; d >= 1; d >>= 1) {
                    uint64_t o = __shfl_xor(key, d, 64);
                    key = o > key ? o : key;
                }
                if (key) {
                    const uint32_t wl = 0xFFFFu - (uint32_t)(key & 0xFFFFu);
                    uint32_t cc, ll;
                    path_len(s, wl, cc, ll);
                    have = true;
                    gcount = cc;
                    gxrel = s.pos[wl];
                    gexit = node_next_abs(s, base, ll);
                }
            }
        }
        if (have && lane == 0) {
            st_agent(&a.status[2 * k + 1], pack_status(ST_AGG, gxrel, 0));
            st_agent(&a.status[2 * k], pack_status(ST_AGG, gcount, gexit));
        }
        HG_STAMP(D_T_AGG);
        // ---- 6. look-back ----------------------------------------------------
        uint32_t spins = 0;
        LookbackOut lb = lookback(a, k, spins);
        HG_STAMP(D_T_LB);
        if (DIAG && lane == 0) {
            dg[D_SPINS] = spins;
            dg[D_GUESS] = (have ? 1u : 0u) | (gxrel != NONE_REL ? 2u : 0u) |
                          ((lb.x == (gxrel != NONE_REL ? base + gxrel : gexit)) ? 4u : 0u);
        }
        if (lane == 0) {
            s.xk = lb.x;
            s.gk = lb.g;
            s.err_kind = lb.err;
            s.err_pos = lb.errpos;
        }
    }
    __syncthreads();

    const uint32_t perr = s.err_kind;
    uint64_t xk = s.xk, gk = s.gk;
    uint32_t kind = HG_OK;
    uint64_t errpos = 0, count = 0, exitk = 0;
    if (perr != HG_OK) {  // an earlier chunk failed: propagate, emit nothing
        kind = perr;
        errpos = s.err_pos;
        count = 0;
    } else {
        // ---- 7. resolve the exact path --------------------------------------
        bool fast = false;
        if (xk >= base + clen) {  // no record starts in this chunk
            fast = true;
            if (tid == 0) {
                s.x_count = 0;
                s.exitk = xk;
            }
        } else if (lifting) {
            const uint32_t xi = surv_index(s, (uint32_t)(xk - base));
            if (xi != 0xFFFFFFFFu) {
                uint32_t c, last;
                path_len(s, xi, c, last);
                if (s.term[last] == T_EXIT) {
                    fast = true;
                    if (tid == 0) {
                        s.x_idx = xi;
                        s.x_count = c;
                        s.exitk = node_next_abs(s, base, last);
                    }
                }
            }
        }
        __syncthreads();
        if (fast) {
            count = s.x_count;
            exitk = s.exitk;
            if (tid == 0) {
                st_agent(&a.status[2 * k + 1],
                         pack_status(ST_INCL, (xk < base + clen) ? (uint32_t)(xk - base) : NONE_REL,
                                     gk + count));
                st_agent(&a.status[2 * k], pack_status(ST_INCL, (uint32_t)count, exitk));
            }
            // ---- 8. emission: lane t writes record t of the path ------------
            const uint32_t xi = s.x_idx;
            for (uint32_t t = tid; t < count; t += DEC_THREADS) {
                const uint32_t node = path_node(s, xi, t);
                const uint32_t p = s.pos[node];
                uint64_t kl, vl;
                lds_header(data, p, kl, vl);
                const uint64_t gi = gk + t;
                if (gi < a.cap) {
                    const uint64_t off = base + p;
                    uint4 sp;
                    sp.x = (uint32_t)off;
                    sp.y = (uint32_t)(off >> 32);
                    sp.z = (uint32_t)kl;
                    sp.w = (uint32_t)vl;
                    *reinterpret_cast<uint4*>(a.spans + gi) = sp;
                }
            }
        } else {
            serial_walk_emit(s, a, base, clen, xk, gk);
            count = s.x_count;
            kind = s.err_kind;
            errpos = s.err_pos;
            exitk = s.exitk;
            if (tid == 0) {
                if (kind == HG_OK) {
                    st_agent(&a.status[2 * k + 1],
                             pack_status(ST_INCL, (uint32_t)(xk - base), gk + count));
                    st_agent(&a.status[2 * k], pack_status(ST_INCL, (uint32_t)count, exitk));
                } else {
                    st_agent(&a.status[2 * k + 1], pack_status(ST_ERR, 0, gk + count));
                    st_agent(&a.status[2 * k], pack_status(ST_ERR, kind, errpos));
                }
            }
        }
    }
    if (perr != HG_OK && tid == 0) {
        st_agent(&a.status[2 * k + 1], pack_status(ST_ERR, 0, gk));
        st_agent(&a.status[2 * k], pack_status(ST_ERR, kind, errpos));
    }
    HG_STAMP(D_T_END);
    if (DIAG && tid == 0) {
        dg[D_COUNT] = (uint32_t)count;
        dg[D_FLAGS] = (lifting ? 1u : 0u) | (perr != HG_OK ? 2u : 0u) | (kind != HG_OK ? 4u : 0u);
    }
#undef HG_STAMP
    // ---- 9. the last chunk reports the whole-file result ----------------------
    if (tid == 0 && k == a.nchunks - 1) {
        hg_decode_result r;
        r.n_records = gk + count;
        r.kind = (int32_t)kind;
        r.reserved = 0;
        r.err_offset = kind != HG_OK ? errpos : 0;
        *a.result = r;
    }
}

}  // namespace hgk

// Host-side launcher (called by the runtime; stream-ordered, no sync).
// d_status must hold hgk_decode_workspace_bytes(len) bytes; the launcher
// zeroes the statuses and the ticket word that follows them.
extern "C" int hgk_decode_launch_diag(const uint8_t* d_sst, uint64_t len, hg_span* d_spans,
                                      uint64_t cap, hg_decode_result* d_result,
                                      unsigned long long* d_status, uint32_t* d_diag,
                                      hipStream_t stream) {
    using namespace hgk;
    const uint64_t nch = (len + DEC_CHUNK - 1) / DEC_CHUNK;
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
    if (d_diag)
        hipLaunchKernelGGL(decode_kernel<true>, dim3((uint32_t)nch), dim3(DEC_THREADS), 0, stream,
                           a);
    else
        hipLaunchKernelGGL(decode_kernel<false>, dim3((uint32_t)nch), dim3(DEC_THREADS), 0,
                           stream, a);
    return hipGetLastError() == hipSuccess ? HG_OK : HG_ERR_HIP;
}

extern "C" int hgk_decode_launch(const uint8_t* d_sst, uint64_t len, hg_span* d_spans,
                                 uint64_t cap, hg_decode_result* d_result,
                                 unsigned long long* d_status, hipStream_t stream) {
    return hgk_decode_launch_diag(d_sst, len, d_spans, cap, d_result, d_status, nullptr, stream);
}

extern "C" uint64_t hgk_decode_workspace_bytes(uint64_t len) {
    const uint64_t nch = (len + hgk::DEC_CHUNK - 1) / hgk::DEC_CHUNK;
    return (2 * nch + 2) * sizeof(unsigned long long);
}
