// hg_merge.hip — device k-way merge for SSTable compaction (gfx950).
//
// Replaces SSTableManager::compact_inner (reference src/sstable/manager.rs:
// 199-234): tables are given in priority order (index 0 wins ties; compact()
// passes them newest first, manager.rs:146-149).  The output is the sorted
// union of the keys, each taken from the highest-priority table holding it;
// tombstones are kept (no filtering, :216-217).  For tables that are sorted
// with unique keys -- every table horreum writes (memtable BTreeMap flush,
// compaction output) -- that is exactly the reference loop's result, and the
// parallel merge-path rounds below build it.  Any other input (duplicate or
// unordered keys in a table) runs the reference loop itself (step 5).
//
// Design (MI355X): keys are compared through 24-byte merge entries: a 16-byte
// big-endian key prefix (one 128-bit compare decides almost every pair), the
// key length and the record's global entry index (its table by a search over
// the run offsets; < 2^31 entries per merge); only keys that agree on their
// first 16 bytes and are both longer fetch the rest from HBM.
//   1. merge_prep_kernel: one entry per record (runs laid out table by table),
//   2. and in the same pass: each table strictly increasing (else step 5).
//   3. log2(k) rounds of merge_level_kernel: adjacent runs (A = higher
//      priority, B = lower) merge by merge path: a workgroup owns TILE output
//      positions, takes its A/B split from merge_split_kernel (an 8-ary
//      search per tile boundary, all boundaries at once), stages
//      both segments in LDS, and each thread finds its 4 outputs' split by one
//      binary search on its diagonal and merges them sequentially (ties: A
//      first; coalesced stores).  A B element whose key also occurs in A is
//      marked dead (newest wins).  Output runs occupy the same index
//      ranges as their two inputs.
//   4. merge_count / merge_scan / merge_emit kernels: the live entries, in
//      order, become hg_pair records pointing into the arena -- the input of
//      hg_encode_*, so compaction is decode -> merge -> encode on device.
//   5. merge_exact_kernel: only when step 2 found a table that is not
//      strictly increasing (every round above then skips its work): the
//      reference loop, step by step, by one wave.
#include <stdlib.h>

#include "hg_device.hpp"

namespace hgm {

constexpr uint32_t THREADS = 256;
#ifndef HG_MERGE_TILE
#define HG_MERGE_TILE 1024
#endif
constexpr uint32_t TILE = HG_MERGE_TILE;  // merged positions per workgroup
constexpr uint32_t EPT = TILE / THREADS;
constexpr uint32_t WPT = 3 * TILE / THREADS;  // 8-byte words of a tile's entries per thread
constexpr uint32_t FIN_LDS_TABLES = 64;
constexpr uint32_t DEAD = 0x80000000u;
constexpr uint32_t MAX_TABLES = 1u << 16;

struct MEnt {          // 24 bytes
    uint64_t p0, p1;   // key bytes [0,8) and [8,16), big-endian, zero padded
    uint32_t klen;
    uint32_t gd;       // global entry index g (runs laid out table by table) | DEAD
};
constexpr uint64_t MAX_ENTRIES = DEAD;  // g must fit below the DEAD bit

struct MergeArgs {
    const uint8_t* arena;
    uint64_t arena_len;
    const uint64_t* table_off;   // [ntables] byte offset of each table in the arena
    const hg_span* const* spans; // [ntables] device pointers
    const uint64_t* run_off;     // [ntables + 1] entry offsets of the tables' runs
    uint32_t ntables;
    uint64_t n;                  // total entries
};


__device__ __forceinline__ uint64_t bswap64(uint64_t x) { return __builtin_bswap64(x); }

__device__ __forceinline__ uint32_t run_of(const MergeArgs& a, uint64_t g);

// The record behind entry e: its table t and span.
__device__ __forceinline__ hg_span ent_span(const MergeArgs& a, const MEnt& e, uint32_t& t) {
    const uint64_t g = e.gd & ~DEAD;
    t = run_of(a, g);
    return a.spans[t][g - a.run_off[t]];
}

__device__ __forceinline__ const uint8_t* key_ptr(const MergeArgs& a, const MEnt& e) {
    uint32_t t;
    const hg_span sp = ent_span(a, e, t);
    return a.arena + a.table_off[t] + sp.off + 16;
}

// Bytes [from, to) of two keys that agree on their first `from` bytes.
__device__ int tail_cmp(const MergeArgs& a, const MEnt& x, const MEnt& y) {
    const uint8_t* kx = key_ptr(a, x);
    const uint8_t* ky = key_ptr(a, y);
    const uint32_t m = min(x.klen, y.klen);
    for (uint32_t i = 16; i < m; ++i) {
        const uint8_t bx = kx[i], by = ky[i];
        if (bx != by) return bx < by ? -1 : 1;
    }
    return x.klen < y.klen ? -1 : x.klen > y.klen ? 1 : 0;
}

// Lexicographic byte order, a shorter key first when it is a prefix
// (Vec<u8> Ord, src/format.rs:5).
__device__ __forceinline__ int key_cmp(const MergeArgs& a, const MEnt& x, const MEnt& y) {
    if (x.p0 != y.p0) return x.p0 < y.p0 ? -1 : 1;
    if (x.p1 != y.p1) return x.p1 < y.p1 ? -1 : 1;
    if (x.klen <= 16 || y.klen <= 16) return x.klen < y.klen ? -1 : x.klen > y.klen ? 1 : 0;
    return tail_cmp(a, x, y);
}

// ---- 1. entries ---------------------------------------------------------------------
__device__ __forceinline__ uint32_t run_of(const MergeArgs& a, uint64_t g) {
    uint32_t lo = 0, hi = a.ntables;  // last run with run_off[r] <= g
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (a.run_off[mid] <= g) lo = mid;
        else hi = mid;
    }
    return lo;
}

__device__ __forceinline__ MEnt make_ent(const MergeArgs& a, uint64_t g, uint32_t t) {
    const uint64_t rec = g - a.run_off[t];
    // spans and key bytes are read once: nontemporal 16-byte loads
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    const u32x4 spv = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(a.spans[t] + rec));
    hg_span sp;
    sp.off = ((uint64_t)spv.y << 32) | spv.x;
    sp.klen = spv.z;
    sp.vlen = spv.w;
    const uint64_t kofs = a.table_off[t] + sp.off + 16;
    const uint8_t* k = a.arena + kofs;
    uint64_t w0 = 0, w1 = 0;
    if (kofs + 16 <= a.arena_len) {
        // one unaligned 16-byte load (native on gfx950), then mask past klen
        const u32x4 kv = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(k));
        uint64_t r0 = ((uint64_t)kv.y << 32) | kv.x, r1 = ((uint64_t)kv.w << 32) | kv.z;
        const uint32_t kl = sp.klen;
        if (kl < 8) r0 &= kl ? (~0ull >> (64 - 8 * kl)) : 0ull;
        if (kl < 16) r1 &= kl <= 8 ? 0ull : (~0ull >> (64 - 8 * (kl - 8)));
        w0 = bswap64(r0);
        w1 = bswap64(r1);
    } else {
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const uint64_t byte = (uint32_t)i < sp.klen ? k[i] : 0;
            if (i < 8) w0 = (w0 << 8) | byte;
            else w1 = (w1 << 8) | byte;
        }
    }
    MEnt m;
    m.p0 = w0;
    m.p1 = w1;
    m.klen = sp.klen;
    m.gd = (uint32_t)g;
    return m;
}

// One entry per record, and (step 2, fused) each table strictly increasing:
// an entry is compared with its predecessor in the same table -- the
// neighbouring thread's entry through LDS, or for the workgroup's first
// entry the predecessor rebuilt.  err[0] = lowest offending global entry
// index (initialised to ~0).
__global__ __launch_bounds__(THREADS) void merge_prep_kernel(MergeArgs a, MEnt* e,
                                                             unsigned long long* err) {
    __shared__ MEnt sh[THREADS];
    const uint32_t tid = threadIdx.x;
    const uint64_t g = (uint64_t)blockIdx.x * THREADS + tid;
    const bool ok = g < a.n;
    // the workgroup's first run by a uniform search (scalar loads), then the
    // rare lane past a run boundary steps forward
    uint32_t t = run_of(a, (uint64_t)blockIdx.x * THREADS);
    while (t + 1 < a.ntables && a.run_off[t + 1] <= g) ++t;
    MEnt m;
    if (ok) {
        m = make_ent(a, g, t);
        e[g] = m;
        sh[tid] = m;
    }
    __syncthreads();
    if (!ok || g == 0) return;
    if (g == a.run_off[t]) return;  // first record of its table
    const MEnt prev = tid ? sh[tid - 1] : make_ent(a, g - 1, t);
    if (key_cmp(a, prev, m) >= 0) atomicMin(err, (unsigned long long)g);
}

// ---- 3. one merge round ---------------------------------------------------------------
struct LevelArgs {
    const uint64_t* roff;  // [nruns + 1] run offsets of this round's input
    uint32_t nruns;
};

struct LevelSmem {
    alignas(16) MEnt seg[TILE + 2];  // A segment then B segment (then the merged output)
    MEnt aprev;              // A element just before the tile's A segment
    uint64_t i0, i1;         // A split at the tile's start / end
    uint32_t has_prev;
};

// Lower bound of x in s[0, n) (first element >= x); upper = first > x.
__device__ __forceinline__ uint32_t lds_bound(const MergeArgs& a, const MEnt* s, uint32_t n,
                                              const MEnt& x, bool upper) {
    uint32_t lo = 0, hi = n;
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        const int c = key_cmp(a, s[mid], x);
        if (c < 0 || (upper && c == 0)) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

// Pair of runs holding output position d of a round: A run index pa, the
// pair's start o, A/B boundary amid and end oend.
__device__ __forceinline__ void pair_of(const LevelArgs& l, uint64_t d, uint32_t& pa, uint64_t& o,
                                        uint64_t& amid, uint64_t& oend) {
    uint32_t lo = 0, hi = l.nruns;
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (l.roff[mid] <= d) lo = mid;
        else hi = mid;
    }
    pa = lo & ~1u;
    o = l.roff[pa];
    amid = l.roff[min(pa + 1, l.nruns)];
    oend = l.roff[min(pa + 2, l.nruns)];
}

// A split (A elements among the merged positions before it) for every tile
// start of a round, all boundaries at once: the merge-path searches'
// dependent HBM probes overlap across the grid instead of sitting at the head
// of every tile of the round.  SPLIT_G lanes per boundary run a SPLIT_G-ary
// search (~log8(run) dependent rounds of SPLIT_G probes of two entries):
// one lane per boundary (a binary search, ~20 dependent probes) was bound by
// the probes' latency, one wave per boundary (64-ary) by the bytes it moved.
#ifndef HG_SPLIT_G
#define HG_SPLIT_G 8  // cfg5 leg: 8-ary 21 us per round, 4-ary 25, 16-ary 29
#endif
constexpr uint32_t SPLIT_G = HG_SPLIT_G;
__global__ __launch_bounds__(THREADS) void merge_split_kernel(MergeArgs a, LevelArgs l,
                                                              const MEnt* in, uint64_t* split,
                                                              uint64_t nb_tiles,
                                                              const unsigned long long* err) {
    const uint32_t lane = threadIdx.x & 63u, j = lane % SPLIT_G, gsh = lane - j;
    const uint64_t t = ((uint64_t)blockIdx.x * THREADS + threadIdx.x) / SPLIT_G;
    if (t > nb_tiles) return;  // the whole group
    uint64_t i = 0;
    if (*err == ~0ull) {
        const uint64_t d = min(t * TILE, a.n);
        uint32_t pa;
        uint64_t o, amid, oend;
        pair_of(l, d, pa, o, amid, oend);
        const uint64_t na = amid - o, nb = oend - amid, dd = d - o;
        if (nb == 0) {
            i = dd;
        } else {  // first c in [lo, hi] with A[c] > B[dd-c-1] (A[c] not among the first dd)
            const MEnt* A = in + o;
            const MEnt* B = in + amid;
            uint64_t lo = dd > nb ? dd - nb : 0, hi = dd < na ? dd : na;
            while (lo < hi) {  // uniform within the group
                const uint64_t span = hi - lo;
                const uint64_t c = lo + span * j / SPLIT_G;  // < hi
                const bool after = key_cmp(a, A[c], B[dd - c - 1]) > 0;
                const uint32_t m =
                    (uint32_t)((__ballot(after) >> gsh) & ((2ull << (SPLIT_G - 1)) - 1ull));
                if (!m) {
                    lo = lo + span * (SPLIT_G - 1) / SPLIT_G + 1;
                } else {
                    const uint32_t f = (uint32_t)__ffs(m) - 1;
                    const uint64_t cf = lo + span * f / SPLIT_G;
                    lo = f ? lo + span * (f - 1) / SPLIT_G + 1 : lo;
                    hi = cf;
                }
            }
            i = lo;
        }
    }
    if (j == 0) split[t] = i;
}

// The last round (two runs -> one) emits the hg_pairs itself (step 4 fused):
// each tile counts its live entries, takes the live entries of the tiles
// before it by a decoupled look-back over per-tile status words, and writes
// its pairs at their final positions; the last tile writes the result.
struct FinalArgs {
    unsigned long long* st;  // [ntiles] look-back status (zeroed): flag << 62 | live count
    hg_pair* out;
    uint64_t cap;
    hg_merge_result* result;
    uint32_t ntiles;
};
constexpr unsigned long long LB_AGG = 1ull << 62, LB_INCL = 2ull << 62;
constexpr unsigned long long LB_VAL = (1ull << 62) - 1;

// Live entries of the tiles before tile t (wave 0; every lane gets it) and
// publication of this tile's inclusive count.  A wait that exceeds its budget
// flags the merge (err) so the exact loop redoes it: never an endless spin.
__device__ uint64_t final_lookback(const FinalArgs& f, uint32_t t, uint64_t agg,
                                   unsigned long long* err) {
    const uint32_t lane = threadIdx.x & 63u;
    if (t == 0) {
        if (lane == 0) hgk::st_agent(&f.st[0], LB_INCL | agg);
        return 0;
    }
    if (lane == 0) hgk::st_agent(&f.st[t], LB_AGG | agg);
    uint64_t acc = 0;
    int64_t j0 = (int64_t)t - 1;
    uint32_t spins = 0;
    for (;;) {
        const int64_t j = j0 - (int64_t)lane;
        unsigned long long w = j >= 0 ? hgk::ld_agent(&f.st[j]) : LB_INCL;
        unsigned long long incl, rel;
        for (;;) {
            incl = __ballot((w >> 62) == 2);
            const int fi = incl ? __ffsll((long long)incl) - 1 : 63;
            rel = fi >= 63 ? ~0ull : ((1ull << (fi + 1)) - 1ull);
            if (!(__ballot((w >> 62) == 0) & rel)) break;
            if (++spins > (1u << 22)) {
                if (lane == 0) {
                    atomicMin(err, 0ull);
                    hgk::st_agent(&f.st[t], LB_INCL | agg);
                }
                return 0;
            }
            __builtin_amdgcn_s_sleep(1);
            if (j >= 0 && (w >> 62) == 0) w = hgk::ld_agent(&f.st[j]);
        }
        acc += hgk::wave_sum<uint64_t>(((rel >> lane) & 1ull) ? (w & LB_VAL) : 0ull);
        if (incl) break;
        j0 -= 64;
    }
    if (lane == 0) hgk::st_agent(&f.st[t], LB_INCL | (acc + agg));
    return acc;
}

// err: the order check's result; merging unsorted runs is meaningless (and
// their merge paths are not monotone), so every round skips work once set.
// FINAL: the last round, emitting pairs (f) instead of entries (out unused).
template <bool FINAL>
// Occupancy over registers: bounded to 5 (6 for the last round) waves/SIMD
// the rounds run faster despite a few spilled registers (cfg 5 leg: 96 -> 92
// and 185 -> 167 us against 4 waves/SIMD unbounded).
__global__ __launch_bounds__(THREADS, FINAL ? 6 : 5) void merge_level_kernel(MergeArgs a, LevelArgs l,
                                                              const MEnt* in, MEnt* out,
                                                              const uint64_t* split,
                                                              unsigned long long* err,
                                                              FinalArgs f) {
    __shared__ LevelSmem s;
    __shared__ uint32_t fin_tmp[THREADS / 64];
    __shared__ uint64_t fin_base;
    // FINAL: the tables' run offsets, span arrays and arena offsets in LDS
    // (up to FIN_LDS_TABLES tables), so a live record's span lookup is one
    // HBM load after an LDS search instead of a chain of dependent loads
    __shared__ uint64_t fin_roff[FIN_LDS_TABLES + 1], fin_sp[FIN_LDS_TABLES],
        fin_toff[FIN_LDS_TABLES];
    const uint32_t tid = threadIdx.x;
    const uint64_t t0 = (uint64_t)blockIdx.x * TILE;
    if (t0 >= a.n) return;
    const bool fin_lds = FINAL && a.ntables <= FIN_LDS_TABLES;
    if (fin_lds) {  // read after the segment staging's barrier
        if (tid <= a.ntables) fin_roff[tid] = a.run_off[tid];
        if (tid < a.ntables) {
            fin_sp[tid] = reinterpret_cast<uint64_t>(a.spans[tid]);
            fin_toff[tid] = a.table_off[tid];
        }
    }
    // A FINAL tile that stops early still publishes its status (count 0), so
    // no later tile waits on it; the exact loop then redoes the merge.
    auto fin_abort = [&]() {
        if (FINAL && tid < 64) final_lookback(f, blockIdx.x, 0, err);
    };
    // The error word is loaded with the splits (one round trip) and tested
    // before anything is staged: once the order check failed the splits are
    // all 0 and the segments they imply run past the runs' ends.
    const unsigned long long err0 = *err;
    const uint64_t t1 = min(t0 + TILE, a.n);
    // The tile may span several output runs (pairs); handle each piece.
    uint64_t d0 = t0;
    while (d0 < t1) {
        // pair containing output position d0
        uint32_t pa;
        uint64_t o, amid, oend;
        pair_of(l, d0, pa, o, amid, oend);
        const uint64_t d1 = min(t1, oend);
        const MEnt* A = in + o;
        const MEnt* B = in + amid;
        const uint64_t na = amid - o, nb = oend - amid;
        if (nb == 0) {  // odd run out: copied as is (never in the FINAL round)
            if (err0 != ~0ull) {
                fin_abort();
                return;
            }
            for (uint64_t d = d0 + tid; d < d1; d += THREADS) out[d] = in[d];
            d0 = d1;
            __syncthreads();
            continue;
        }
        // splits from merge_split_kernel (pair edges are 0 / na), read by every
        // thread (uniform addresses); the A element before the tile's A segment
        // is fetched with the segments
        const uint64_t i0 = d0 == t0 ? split[blockIdx.x] : 0;
        const uint64_t i1 = d1 == oend ? na : split[blockIdx.x + 1];
        if (err0 != ~0ull) {  // an earlier check or round found unsorted input
            fin_abort();
            return;
        }
        if (i1 < i0 || i0 > d0 - o || i1 > d1 - o || (d1 - o) - i1 < (d0 - o) - i0) {
            // splits of sorted runs are monotone; anything else means the
            // input was not sorted: flag it (the exact loop takes over) and stop
            if (tid == 0) atomicMin(err, (unsigned long long)o);
            fin_abort();
            return;
        }
        const uint64_t j0 = (d0 - o) - i0, j1 = (d1 - o) - i1;
        const uint32_t nA = (uint32_t)(i1 - i0), nB = (uint32_t)(j1 - j0);
        {  // both segments as 8-byte words, contiguous per lane (entries are 24 B);
           // every load of a thread is issued before its first LDS write (a
           // load / wait / write loop paid one HBM round trip per word, 12 per
           // thread per tile); a word past the segments re-reads the last one
            const uint64_t* wa = reinterpret_cast<const uint64_t*>(A + i0);
            const uint64_t* wb = reinterpret_cast<const uint64_t*>(B + j0);
            uint64_t* ws = reinterpret_cast<uint64_t*>(s.seg);
            const uint32_t wA = 3 * nA, wT = 3 * (nA + nB);  // wT >= 3: d1 > d0
            uint64_t v[WPT];
#pragma unroll
            for (uint32_t i = 0; i < WPT; ++i) {
                const uint32_t q = min(tid + i * THREADS, wT - 1);
                v[i] = *(q < wA ? wa + q : wb + (q - wA));
            }
#pragma unroll
            for (uint32_t i = 0; i < WPT; ++i)
                if (tid + i * THREADS < wT) ws[tid + i * THREADS] = v[i];
        }
        if (tid == THREADS - 1) {
            s.has_prev = i0 > 0;
            if (i0 > 0 && i0 <= na) s.aprev = A[i0 - 1];
        }
        __syncthreads();
        const MEnt* SA = s.seg;
        const MEnt* SB = s.seg + nA;
        MEnt* dst = out + d0;
        // Merge path inside the tile: thread tid owns outputs [tid*EPT, +EPT),
        // finds how many of them come from A by one binary search on its
        // diagonal (A first on equal keys, as merge_split_kernel) and merges
        // them sequentially into registers.  The merged entries (or, in the
        // FINAL round, the live records' pairs) then go back into LDS in
        // output order and out with contiguous 16- / 8-byte stores per lane:
        // per-thread stores of 32-byte entries at a 128-byte lane stride cost
        // 20 % extra HBM writes, of 24-byte pairs 2x (rocprofv3 WRITE_SIZE).
        {
            const uint32_t nt = nA + nB;
            const uint32_t d = tid * EPT;
            const uint32_t e = d < nt ? min(d + EPT, nt) : d;
            MEnt fx[EPT];
            uint32_t fcnt = 0;
            if (d < nt) {
                uint32_t lo = d > nB ? d - nB : 0, hi = d < nA ? d : nA;
                while (lo < hi) {
                    const uint32_t mid = (lo + hi) >> 1;
                    if (key_cmp(a, SA[mid], SB[d - 1 - mid]) <= 0) lo = mid + 1;
                    else hi = mid;
                }
                uint32_t ai = lo, bj = d - lo;
#pragma unroll
                for (uint32_t k = 0; k < EPT; ++k) {  // constant indices: fx stays in VGPRs
                    if (d + k >= e) break;
                    MEnt x;
                    if (bj >= nB || (ai < nA && key_cmp(a, SA[ai], SB[bj]) <= 0)) {
                        x = SA[ai++];
                    } else {
                        x = SB[bj++];
                        // newest wins: the last A element at or before it (inside
                        // the tile, or the one just before the tile) kills an equal key
                        const bool eq = ai > 0 ? key_cmp(a, SA[ai - 1], x) == 0
                                               : (s.has_prev && key_cmp(a, s.aprev, x) == 0);
                        if (eq) x.gd |= DEAD;
                    }
                    fx[k] = x;
                    fcnt += (x.gd & DEAD) ? 0u : 1u;
                }
            }
            __syncthreads();  // every thread is done reading the segments
            if (!FINAL) {
#pragma unroll
                for (uint32_t k = 0; k < EPT; ++k)
                    if (d + k < e) s.seg[d + k] = fx[k];
                __syncthreads();
                const uint64_t* src = reinterpret_cast<const uint64_t*>(s.seg);
                uint64_t* o8 = reinterpret_cast<uint64_t*>(dst);
                for (uint32_t i = tid; i < 3 * nt; i += THREADS) o8[i] = src[i];
            } else {
                // live entries before this thread's in the tile, the tiles'
                // before it (look-back), then the pairs at their positions
                uint32_t ftot;
                const uint32_t fpre = hgk::block_excl_scan<THREADS / 64>(fcnt, fin_tmp, ftot);
                if (tid < 64) {
                    const uint64_t b = final_lookback(f, blockIdx.x, ftot, err);
                    if (tid == 0) {
                        fin_base = b;
                        if (blockIdx.x + 1 == f.ntiles) {
                            hg_merge_result r;
                            r.n_out = b + ftot;
                            r.kind = HG_OK;
                            r.table = 0;
                            r.index = 0;
                            *f.result = r;
                        }
                    }
                }
                hg_pair* lp = reinterpret_cast<hg_pair*>(s.seg);
                uint32_t r = fpre;
                // the spans of this thread's outputs, every load issued
                // before the first is used (branch-free: an output past the
                // tile or dead looks up entry 0 and is dropped below)
                uint32_t tk[EPT];
                hg_span spk[EPT];
                uint64_t tof[EPT];
#pragma unroll
                for (uint32_t k = 0; k < EPT; ++k) {
                    const uint64_t g = d + k < e ? (uint64_t)(fx[k].gd & ~DEAD) : 0ull;
                    if (fin_lds) {
                        uint32_t lo = 0, hi = a.ntables;  // last run with fin_roff[r] <= g
                        while (hi - lo > 1) {
                            const uint32_t mid = (lo + hi) >> 1;
                            if (fin_roff[mid] <= g) lo = mid;
                            else hi = mid;
                        }
                        tk[k] = lo;
                        tof[k] = fin_toff[lo];
                        spk[k] = reinterpret_cast<const hg_span*>(fin_sp[lo])[g - fin_roff[lo]];
                    } else {
                        tk[k] = run_of(a, g);
                        tof[k] = a.table_off[tk[k]];
                        spk[k] = a.spans[tk[k]][g - a.run_off[tk[k]]];
                    }
                }
#pragma unroll
                for (uint32_t k = 0; k < EPT; ++k) {
                    if (d + k >= e || (fx[k].gd & DEAD)) continue;
                    const hg_span sp = spk[k];
                    hg_pair p;
                    p.key_off = tof[k] + sp.off + 16;
                    p.val_off = p.key_off + sp.klen;
                    p.klen = sp.klen;
                    p.vlen = sp.vlen;
                    lp[r++] = p;
                }
                __syncthreads();  // also publishes fin_base
                // the tile's pairs are words [3 base, 3 (base + ftot)) of out
                const uint64_t w0 = 3 * fin_base, wcap = 3 * f.cap;
                const uint64_t* s8 = reinterpret_cast<const uint64_t*>(s.seg);
                uint64_t* o8 = reinterpret_cast<uint64_t*>(f.out);
                for (uint32_t i = tid; i < 3 * ftot; i += THREADS)
                    if (w0 + i < wcap) o8[w0 + i] = s8[i];
            }
        }
        d0 = d1;
        __syncthreads();
    }
}

// ---- 4. live entries -> hg_pair ---------------------------------------------------------
__global__ __launch_bounds__(THREADS) void merge_count_kernel(MergeArgs a, const MEnt* e,
                                                              uint32_t* tile_live) {
    const uint64_t t0 = (uint64_t)blockIdx.x * TILE;
    uint32_t c = 0;
    for (uint32_t q = threadIdx.x; q < TILE; q += THREADS) {
        const uint64_t g = t0 + q;
        if (g < a.n && !(e[g].gd & DEAD)) ++c;
    }
    __shared__ uint32_t ws[THREADS / 64];
    c = hgk::wave_sum<uint32_t>(c);
    if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t s = 0;
        for (uint32_t w = 0; w < THREADS / 64; ++w) s += ws[w];
        tile_live[blockIdx.x] = s;
    }
}

// Exclusive scan of the tile counts by one workgroup (ntiles = n / TILE).
__global__ __launch_bounds__(1024) void merge_scan_kernel(const uint32_t* tile_live, uint32_t ntiles,
                                                          uint64_t* tile_base,
                                                          hg_merge_result* result) {
    __shared__ uint64_t wt[16];
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wid = tid >> 6;
    uint64_t carry = 0;
    for (uint32_t c0 = 0; c0 < ntiles; c0 += 1024) {
        const uint32_t j = c0 + tid;
        const uint64_t v = j < ntiles ? tile_live[j] : 0;
        uint64_t incl = v;
        for (uint32_t d = 1; d < 64; d <<= 1) {
            const uint64_t o = __shfl_up(incl, d, 64);
            if (lane >= d) incl += o;
        }
        if (lane == 63) wt[wid] = incl;
        __syncthreads();
        uint64_t base = carry + incl - v, tot = 0;
        for (uint32_t w = 0; w < 16; ++w) {
            if (w < wid) base += wt[w];
            tot += wt[w];
        }
        if (j < ntiles) tile_base[j] = base;
        carry += tot;
        __syncthreads();
    }
    if (tid == 0) {
        result->n_out = carry;
        result->kind = HG_OK;
        result->table = 0;
        result->index = 0;
    }
}

__global__ __launch_bounds__(THREADS) void merge_emit_kernel(MergeArgs a, const MEnt* e,
                                                             const uint64_t* tile_base,
                                                             hg_pair* out, uint64_t cap,
                                                             const unsigned long long* err) {
    // Row-major over the tile (entry t0 + k * THREADS + tid), so every load of
    // entries and most stores of pairs are contiguous across the wave; a
    // live entry's rank = live entries of the rows before + its wave's prefix
    // in the row (ballot) + the lanes before it (popcount).
    __shared__ uint32_t wc[EPT][THREADS / 64];
    if (*err != ~0ull) return;
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wid = tid >> 6;
    const uint64_t t0 = (uint64_t)blockIdx.x * TILE;
    MEnt x[EPT];
    uint32_t pre[EPT];
    bool lv[EPT];
#pragma unroll
    for (uint32_t k = 0; k < EPT; ++k) {
        const uint64_t g = t0 + (uint64_t)k * THREADS + tid;
        lv[k] = false;
        if (g < a.n) {
            x[k] = e[g];
            lv[k] = !(x[k].gd & DEAD);
        }
    }
    const unsigned long long below = (1ull << lane) - 1ull;
#pragma unroll
    for (uint32_t k = 0; k < EPT; ++k) {
        const unsigned long long m = __ballot(lv[k]);
        pre[k] = (uint32_t)__popcll(m & below);
        if (lane == 0) wc[k][wid] = (uint32_t)__popcll(m);
    }
    __syncthreads();
    uint64_t run = tile_base[blockIdx.x];
#pragma unroll
    for (uint32_t k = 0; k < EPT; ++k) {
        uint32_t row = 0, woff = 0;
#pragma unroll
        for (uint32_t w = 0; w < THREADS / 64; ++w) {
            row += wc[k][w];
            woff += w < wid ? wc[k][w] : 0u;
        }
        const uint64_t pos = run + woff + pre[k];
        if (lv[k] && pos < cap) {
            uint32_t t;
            const hg_span sp = ent_span(a, x[k], t);
            hg_pair p;
            p.key_off = a.table_off[t] + sp.off + 16;
            p.val_off = p.key_off + sp.klen;
            p.klen = sp.klen;
            p.vlen = sp.vlen;
            out[pos] = p;
        }
        run += row;
    }
}

// ---- 5. exact reference loop for tables that are not strictly increasing ----------------
// SSTableManager::compact_inner (src/sstable/manager.rs:199-234) step by step:
// the smallest head key wins, the FIRST table holding it in priority order is
// emitted (min_by_key keeps the first minimum, :209-216), and every table
// whose head key equals it advances (:218-227), until every table is
// exhausted (:228-230).  On strictly increasing tables this is the newest-wins
// union the merge-path rounds build; on tables with duplicate or unordered
// keys (legal: SSTable::new accepts any pair list, src/sstable/table.rs:93-108)
// only the loop itself defines the output, so one wave runs it: lane l owns
// tables l, l + 64, ...; their head entries live in a per-table state array;
// a butterfly over (key, table) picks the winner in every lane.  Runs only
// when merge_prep_kernel found a table that is not strictly increasing.
struct ExactHead {  // 40 bytes per table
    MEnt e;         // current head entry (valid when idx < cnt)
    uint64_t idx, cnt;
};

__device__ __forceinline__ bool ent_before(const MergeArgs& a, const MEnt& x, const MEnt& y) {
    const int c = key_cmp(a, x, y);
    // equal keys: the lower table first -- runs are laid out table by table
    return c < 0 || (c == 0 && (x.gd & ~DEAD) < (y.gd & ~DEAD));
}

__device__ __forceinline__ MEnt shfl_ent(const MEnt& m, int src) {
    MEnt o;
    o.p0 = __shfl(m.p0, src, 64);
    o.p1 = __shfl(m.p1, src, 64);
    o.klen = __shfl(m.klen, src, 64);
    o.gd = __shfl(m.gd, src, 64);
    return o;
}

__global__ __launch_bounds__(64) void merge_exact_kernel(MergeArgs a, const MEnt* e,
                                                         const unsigned long long* err,
                                                         ExactHead* hs, hg_pair* out, uint64_t cap,
                                                         hg_merge_result* result) {
    if (*err == ~0ull) return;  // every table strictly increasing: the rounds did the merge
    const uint32_t lane = threadIdx.x;
    bool any = false;
    for (uint32_t t = lane; t < a.ntables; t += 64) {
        ExactHead h;
        h.idx = 0;
        h.cnt = a.run_off[t + 1] - a.run_off[t];
        if (h.cnt) h.e = e[a.run_off[t]];
        any |= h.cnt != 0;
        hs[t] = h;
    }
    uint64_t n = 0;
    if (__ballot(any)) {
        for (;;) {
            // :209-216 the first minimum head over the tables in priority order
            bool have = false;
            MEnt best;
            best.p0 = best.p1 = 0;
            best.klen = best.gd = 0;
            for (uint32_t t = lane; t < a.ntables; t += 64) {
                const ExactHead h = hs[t];
                if (h.idx < h.cnt && (!have || ent_before(a, h.e, best))) {
                    best = h.e;
                    have = true;
                }
            }
#pragma unroll 1
            for (int d = 1; d < 64; d <<= 1) {
                const MEnt o = shfl_ent(best, (int)(lane ^ (uint32_t)d));
                const bool oh = __shfl((int)have, (int)(lane ^ (uint32_t)d), 64) != 0;
                if (oh && (!have || ent_before(a, o, best))) {
                    best = o;
                    have = true;
                }
            }
            // :216-217 push the winner
            if (lane == 0 && n < cap) {
                uint32_t t;
                const hg_span sp = ent_span(a, best, t);
                hg_pair p;
                p.key_off = a.table_off[t] + sp.off + 16;
                p.val_off = p.key_off + sp.klen;
                p.klen = sp.klen;
                p.vlen = sp.vlen;
                out[n] = p;
            }
            ++n;
            // :218-227 advance every table whose head key equals the winner's
            bool left = false;
            for (uint32_t t = lane; t < a.ntables; t += 64) {
                ExactHead h = hs[t];
                if (h.idx < h.cnt && key_cmp(a, h.e, best) == 0) {
                    ++h.idx;
                    if (h.idx < h.cnt) h.e = e[a.run_off[t] + h.idx];
                    hs[t] = h;
                }
                left |= h.idx < h.cnt;
            }
            // :228-230 stop when every candidate is None
            if (!__ballot(left)) break;
        }
    }
    if (lane == 0) {
        hg_merge_result r;
        r.n_out = n;
        r.kind = HG_OK;
        r.table = 1;  // on success: 1 = the serial reference loop produced the output
        r.index = 0;
        *result = r;
    }
}

}  // namespace hgm

// ---- launcher ----------------------------------------------------------------------------
// Workspace (device): two entry buffers, tile counts/bases, run offsets for
// every round, table offsets and span pointers, the error word.
extern "C" uint64_t hgk_merge_workspace_bytes(uint32_t ntables, uint64_t n) {
    using namespace hgm;
    const uint64_t ntiles = (n + TILE - 1) / TILE + 1;
    uint64_t b = 2 * ((n * sizeof(MEnt) + 255) & ~255ull);
    b += ((ntiles * 4 + 255) & ~255ull) + 2 * ((ntiles * 8 + 255) & ~255ull);
    b += ((5 * (uint64_t)ntables + 72) * 8 + 255) & ~255ull;  // device copy of the staging
    b += 256;                                                  // error word
    b += ((uint64_t)ntables * sizeof(ExactHead) + 255) & ~255ull;  // exact-loop heads
    return b;
}

// Host arrays: table_off[ntables], spans[ntables] (device pointers),
// counts[ntables].  `staging` is pinned host memory of at least
// hgk_merge_staging_bytes(ntables) bytes (copied to the device on `stream`).
// [table_off | span ptrs | run offsets of every round]: the rounds' offset
// lists total at most 2 * ntables + 2 * ceil(log2 ntables) + 2 words.
extern "C" uint64_t hgk_merge_staging_bytes(uint32_t ntables) {
    return (5 * (uint64_t)ntables + 72) * 8;
}

extern "C" int hgk_merge_launch(const uint8_t* d_arena, uint64_t arena_len, uint32_t ntables,
                                const uint64_t* table_off, const hg_span* const* spans,
                                const uint64_t* counts, hg_pair* d_out, uint64_t cap,
                                hg_merge_result* d_result, void* d_ws, void* staging,
                                hipStream_t stream) {
    using namespace hgm;
    if (ntables == 0 || ntables > MAX_TABLES) return HG_ERR_INVALID_ARG;
    uint64_t n = 0;
    for (uint32_t t = 0; t < ntables; ++t) n += counts[t];
    if (n >= MAX_ENTRIES) return HG_ERR_TOO_LARGE;  // entries carry a 31-bit global index
    // host staging: [table_off | span ptrs | run offsets of every round]
    uint64_t* h = static_cast<uint64_t*>(staging);
    uint64_t* h_toff = h;
    uint64_t* h_sp = h + ntables;
    uint64_t* h_roff = h + 2 * (uint64_t)ntables;  // table run offsets, then every round's
    uint64_t nr = 0, total_roff = 0, nruns0 = 0;
    for (uint32_t t = 0; t < ntables; ++t) {
        h_toff[t] = table_off[t];
        h_sp[t] = reinterpret_cast<uint64_t>(spans[t]);
    }
    {  // [ntables + 1] run offsets of the tables (entry layout; empty runs
       // included), then per round r its nr runs (nr + 1 offsets).  Round 0
       // merges the NON-EMPTY runs only: an empty run as the last round's B
       // side would have sent that round down the odd-run copy path, which
       // emits no pairs (and publishes no look-back status).
        uint64_t* r = h_roff;
        r[0] = 0;
        for (uint32_t t = 0; t < ntables; ++t) r[t + 1] = r[t] + counts[t];
        uint64_t* r0 = r + ntables + 1;
        r0[0] = 0;
        for (uint32_t t = 0; t < ntables; ++t)
            if (counts[t]) r0[++nr] = r[t + 1];
        total_roff = (uint64_t)ntables + 1 + nr + 1;
        nruns0 = nr;  // non-empty runs (round 0)
        r = r0;
        while (nr > 1) {
            uint64_t* nxt = r + (nr + 1);
            const uint64_t m = (nr + 1) / 2;
            for (uint64_t i = 0; i <= m; ++i) nxt[i] = r[min(2 * i, nr)];
            total_roff += m + 1;
            r = nxt;
            nr = m;
        }
    }
    const uint64_t stage_words = 2 * (uint64_t)ntables + total_roff;
    if (stage_words * 8 > hgk_merge_staging_bytes(ntables)) return HG_ERR_INTERNAL;
    char* ws = static_cast<char*>(d_ws);
    const uint64_t ntiles = (n + TILE - 1) / TILE;
    MEnt* e0 = reinterpret_cast<MEnt*>(ws);
    MEnt* e1 = reinterpret_cast<MEnt*>(ws + ((n * sizeof(MEnt) + 255) & ~255ull));
    char* p = ws + 2 * ((n * sizeof(MEnt) + 255) & ~255ull);
    uint32_t* tile_live = reinterpret_cast<uint32_t*>(p);
    p += ((ntiles + 1) * 4 + 255) & ~255ull;
    uint64_t* tile_base = reinterpret_cast<uint64_t*>(p);
    p += ((ntiles + 1) * 8 + 255) & ~255ull;
    unsigned long long* lb_status = reinterpret_cast<unsigned long long*>(p);
    p += ((ntiles + 1) * 8 + 255) & ~255ull;
    uint64_t* d_stage = reinterpret_cast<uint64_t*>(p);
    p += (stage_words * 8 + 255) & ~255ull;
    unsigned long long* err = reinterpret_cast<unsigned long long*>(p);
    p += 256;
    ExactHead* heads = reinterpret_cast<ExactHead*>(p);
    if (hipMemcpyAsync(d_stage, h, stage_words * 8, hipMemcpyHostToDevice, stream) != hipSuccess)
        return HG_HIP_FAIL;
    if (hipMemsetAsync(err, 0xFF, 8, stream) != hipSuccess) return HG_HIP_FAIL;

    MergeArgs a;
    a.arena = d_arena;
    a.arena_len = arena_len;
    a.table_off = d_stage;
    a.spans = reinterpret_cast<const hg_span* const*>(d_stage + ntables);
    a.run_off = d_stage + 2 * (uint64_t)ntables;
    a.ntables = ntables;
    a.n = n;
    if (n == 0) {
        // every table empty: the reference's unwrap on None (manager.rs:213)
        hg_merge_result r{0, HG_ERR_EMPTY_MERGE, 0, 0};
        return hipMemcpyAsync(d_result, &r, sizeof r, hipMemcpyHostToDevice, stream) == hipSuccess
                   ? HG_OK
                   : HG_HIP_FAIL;
    }
    const uint32_t g1 = (uint32_t)((n + THREADS - 1) / THREADS);
    hipLaunchKernelGGL(merge_prep_kernel, dim3(g1), dim3(THREADS), 0, stream, a, e0, err);
    MEnt* cur = e0;
    MEnt* nxt = e1;
    const uint64_t* roff = a.run_off + ntables + 1;  // round 0: the non-empty runs
    uint64_t nruns = nruns0;
    FinalArgs fa;
    fa.st = lb_status;
    fa.out = d_out;
    fa.cap = cap;
    fa.result = d_result;
    fa.ntiles = (uint32_t)ntiles;
    if (nruns0 >= 2 && hipMemsetAsync(lb_status, 0, ntiles * 8, stream) != hipSuccess)
        return HG_HIP_FAIL;
    while (nruns > 1) {
        LevelArgs l;
        l.roff = roff;
        l.nruns = (uint32_t)nruns;
        // tile_base is free until the final count/scan: the round's splits
        const uint32_t gs = (uint32_t)(((ntiles + 1) * SPLIT_G + THREADS - 1) / THREADS);
        hipLaunchKernelGGL(merge_split_kernel, dim3(gs), dim3(THREADS), 0, stream, a, l,
                           (const MEnt*)cur, tile_base, ntiles, (const unsigned long long*)err);
        if (nruns == 2)  // the last round emits the pairs
            hipLaunchKernelGGL(merge_level_kernel<true>, dim3((uint32_t)ntiles), dim3(THREADS), 0,
                               stream, a, l, (const MEnt*)cur, nxt, (const uint64_t*)tile_base,
                               err, fa);
        else
            hipLaunchKernelGGL(merge_level_kernel<false>, dim3((uint32_t)ntiles), dim3(THREADS), 0,
                               stream, a, l, (const MEnt*)cur, nxt, (const uint64_t*)tile_base,
                               err, fa);
        roff += nruns + 1;
        nruns = (nruns + 1) / 2;
        MEnt* t = cur;
        cur = nxt;
        nxt = t;
    }
    if (nruns0 >= 2) {  // pairs and result written by the last round
        hipLaunchKernelGGL(merge_exact_kernel, dim3(1), dim3(64), 0, stream, a, (const MEnt*)e0,
                           (const unsigned long long*)err, heads, d_out, cap, d_result);
        return HG_LAUNCH_STATUS();
    }
    hipLaunchKernelGGL(merge_count_kernel, dim3((uint32_t)ntiles), dim3(THREADS), 0, stream, a,
                       (const MEnt*)cur, tile_live);
    hipLaunchKernelGGL(merge_scan_kernel, dim3(1), dim3(1024), 0, stream, (const uint32_t*)tile_live,
                       (uint32_t)ntiles, tile_base, d_result);
    hipLaunchKernelGGL(merge_emit_kernel, dim3((uint32_t)ntiles), dim3(THREADS), 0, stream, a,
                       (const MEnt*)cur, (const uint64_t*)tile_base, d_out, cap,
                       (const unsigned long long*)err);
    hipLaunchKernelGGL(merge_exact_kernel, dim3(1), dim3(64), 0, stream, a, (const MEnt*)e0,
                       (const unsigned long long*)err, heads, d_out, cap, d_result);
    return HG_LAUNCH_STATUS();
}
