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
//      Compaction (hg_compact_*): both come from the decode's workspace
//      instead, one workgroup per pre-pass batch (hg_decode.hip,
//      decode_entries_multi: the pre-pass left the key prefixes).
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
#include <string.h>

#include <algorithm>
#include <vector>

#include "hg_device.hpp"
#include "hg_knobs.hpp"

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
    // compaction mode (kp_tag != 0): per table, the decode workspace's span
    // scratch, piece records and piece tags, where the decode pre-pass left the
    // key prefixes of stride pieces (hg_decode.hip, DecodeArgs::kpre_tag)
    const uint64_t* kp_scratch;
    const uint64_t* kp_spiece;
    const uint64_t* kp_ptag;
    uint32_t kp_tag;
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
    if (a.kp_tag) {  // the decode pre-pass's key prefix, if its piece was a current stride run
        // the tag and the piece record are loaded together (one round trip,
        // both L2-resident), then the prefix: span -> piece -> prefix
        const uint64_t piece = sp.off / hgk::PIECE_BYTES;
        const uint32_t tag = reinterpret_cast<const uint32_t*>(a.kp_ptag[t])[piece];
        const hgk::SpecPiece q = reinterpret_cast<const hgk::SpecPiece*>(a.kp_spiece[t])[piece];
        if (tag == a.kp_tag) {
            // the prefix was masked with the piece's key length: it is this
            // record's only if the record has that length (a piece past a
            // header mismatch keeps its lattice but not its records)
            if (q.pad == hgk::SP_STRIDE && sp.off >= q.x && q.R && sp.klen == q.kl) {
                const uint64_t d = sp.off - q.x, j = d / q.R;
                if (j * q.R == d && j < q.count) {
                    const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(
                        reinterpret_cast<const hg_span*>(a.kp_scratch[t]) + piece * hgk::PIECE_RECS + j));
                    MEnt m;
                    m.p0 = ((uint64_t)v.y << 32) | v.x;
                    m.p1 = ((uint64_t)v.w << 32) | v.z;
                    m.klen = sp.klen;
                    m.gd = (uint32_t)g;
                    return m;
                }
            }
        }
    }
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
// neighbouring entry through LDS, or for the workgroup's first entry the
// predecessor rebuilt.  err[0] = lowest offending global entry index
// (initialised to ~0).  PREP_U entries per thread (g = workgroup base + u *
// THREADS + tid), built in stages so the PREP_U dependent load chains of
// make_ent (span -> piece tag and record -> prefix) overlap: one entry per
// thread left each thread three HBM round trips deep with nothing else in flight.
#ifndef HG_PREP_U
#define HG_PREP_U 2
#endif
constexpr uint32_t PREP_U = HG_PREP_U;

__global__ __launch_bounds__(THREADS) void merge_prep_kernel(MergeArgs a, MEnt* e,
                                                             unsigned long long* err) {
    __shared__ MEnt sh[THREADS * PREP_U];
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    const uint32_t tid = threadIdx.x;
    const uint64_t gb = (uint64_t)blockIdx.x * THREADS * PREP_U;
    // the workgroup's first run by a uniform search (scalar loads), then the
    // rare entry past a run boundary steps forward
    uint32_t t = run_of(a, gb);
    uint32_t tt[PREP_U];
    hg_span sp[PREP_U];
    bool ok[PREP_U];
#pragma unroll
    for (uint32_t u = 0; u < PREP_U; ++u) {  // stage 1: spans
        const uint64_t g = gb + u * THREADS + tid;
        ok[u] = g < a.n;
        while (t + 1 < a.ntables && a.run_off[t + 1] <= g) ++t;
        tt[u] = t;
        if (ok[u]) {
            const u32x4 v = __builtin_nontemporal_load(
                reinterpret_cast<const u32x4*>(a.spans[t] + (g - a.run_off[t])));
            sp[u].off = ((uint64_t)v.y << 32) | v.x;
            sp[u].klen = v.z;
            sp[u].vlen = v.w;
        }
    }
    int64_t pj[PREP_U];  // stage 2: the prefix slot of a current stride piece, else -1
#pragma unroll
    for (uint32_t u = 0; u < PREP_U; ++u) {
        pj[u] = -1;
        if (!ok[u] || !a.kp_tag) continue;
        const uint64_t piece = sp[u].off / hgk::PIECE_BYTES;
        const uint32_t tag = reinterpret_cast<const uint32_t*>(a.kp_ptag[tt[u]])[piece];
        const hgk::SpecPiece q = reinterpret_cast<const hgk::SpecPiece*>(a.kp_spiece[tt[u]])[piece];
        if (tag == a.kp_tag && q.pad == hgk::SP_STRIDE && sp[u].off >= q.x && q.R &&
            sp[u].klen == q.kl) {  // (a prefix masked with the piece's key length: make_ent)
            const uint64_t d = sp[u].off - q.x, j = d / q.R;
            if (j * q.R == d && j < q.count) pj[u] = (int64_t)(piece * hgk::PIECE_RECS + j);
        }
    }
    u32x4 kv[PREP_U];  // stage 3: the prefix, or the key's first 16 bytes
#pragma unroll
    for (uint32_t u = 0; u < PREP_U; ++u) {
        kv[u] = u32x4{0, 0, 0, 0};
        if (!ok[u]) continue;
        if (pj[u] >= 0) {
            kv[u] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(
                reinterpret_cast<const hg_span*>(a.kp_scratch[tt[u]]) + pj[u]));
        } else {
            const uint64_t kofs = a.table_off[tt[u]] + sp[u].off + 16;
            if (kofs + 16 <= a.arena_len)
                kv[u] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(a.arena + kofs));
        }
    }
#pragma unroll
    for (uint32_t u = 0; u < PREP_U; ++u) {  // stage 4: entries
        if (!ok[u]) continue;
        const uint64_t g = gb + u * THREADS + tid;
        MEnt m;
        if (pj[u] >= 0) {
            m.p0 = ((uint64_t)kv[u].y << 32) | kv[u].x;
            m.p1 = ((uint64_t)kv[u].w << 32) | kv[u].z;
            m.klen = sp[u].klen;
            m.gd = (uint32_t)g;
        } else if (a.table_off[tt[u]] + sp[u].off + 32 <= a.arena_len) {
            uint64_t r0 = ((uint64_t)kv[u].y << 32) | kv[u].x, r1 = ((uint64_t)kv[u].w << 32) | kv[u].z;
            const uint32_t kl = sp[u].klen;
            if (kl < 8) r0 &= kl ? (~0ull >> (64 - 8 * kl)) : 0ull;
            if (kl < 16) r1 &= kl <= 8 ? 0ull : (~0ull >> (64 - 8 * (kl - 8)));
            m.p0 = bswap64(r0);
            m.p1 = bswap64(r1);
            m.klen = kl;
            m.gd = (uint32_t)g;
        } else {
            m = make_ent(a, g, tt[u]);  // the key's 16 bytes run past the arena
        }
        e[g] = m;
        sh[u * THREADS + tid] = m;
    }
    __syncthreads();
#pragma unroll
    for (uint32_t u = 0; u < PREP_U; ++u) {
        const uint64_t g = gb + u * THREADS + tid;
        if (!ok[u] || g == 0 || g == a.run_off[tt[u]]) continue;  // first record of its table
        const uint32_t l = u * THREADS + tid;
        const MEnt prev = l ? sh[l - 1] : make_ent(a, g - 1, tt[u]);
        if (key_cmp(a, prev, sh[l]) >= 0) atomicMin(err, (unsigned long long)g);
    }
}

// ---- 3. one merge round ---------------------------------------------------------------
struct LevelArgs {
    const uint64_t* roff;  // [nruns + 1] run offsets of this round's input; nullptr:
    uint32_t nruns;        // runs of uw entries each (the last one short) over un entries
    uint64_t uw, un;       // (the rank path's sort rounds, section 7)
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
    if (!l.roff) {  // uniform runs (scalar arithmetic, no search)
        pa = (uint32_t)(d / l.uw) & ~1u;
        o = (uint64_t)pa * l.uw;
        amid = min(o + l.uw, l.un);
        oend = min(o + 2 * l.uw, l.un);
        return;
    }
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
// zst (nullable): the FINAL round's look-back status words, zeroed here by
// a merge's first round (one launch fewer than a memset: ~10 us of gap).
__global__ __launch_bounds__(THREADS) void merge_split_kernel(MergeArgs a, LevelArgs l,
                                                              const MEnt* in, uint64_t* split,
                                                              uint64_t nb_tiles,
                                                              const unsigned long long* err,
                                                              unsigned long long* zst,
                                                              unsigned long long* zsum = nullptr,
                                                              uint64_t zsum_words = 0) {
    const uint32_t lane = threadIdx.x & 63u, j = lane % SPLIT_G, gsh = lane - j;
    const uint64_t gt = (uint64_t)blockIdx.x * THREADS + threadIdx.x;
    if (gt < zsum_words) zsum[gt] = 0;  // the last round's encode sums (FinalArgs::enc_sums)
    const uint64_t t = gt / SPLIT_G;
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
    if (j == 0) {
        split[t] = i;
        if (zst && t < nb_tiles) {  // (both status words of a tile: records mode uses two)
            zst[t] = 0;
            zst[nb_tiles + t] = 0;
        }
        if (zst && t == nb_tiles) zst[2 * nb_tiles] = 0;  // the FINAL round's tile ticket
    }
}

// The last round (two runs -> one) emits the hg_pairs itself (step 4 fused):
// each tile counts its live entries, takes the live entries of the tiles
// before it by a decoupled look-back over per-tile status words, and writes
// its pairs at their final positions; the last tile writes the result.
struct FinalArgs {
    unsigned long long* st;  // [ntiles] look-back status (zeroed): flag << 62 | live count
                             // (records mode: then [ntiles] of output bytes, same flags;
                             // st[2 ntiles]: the tile ticket, zeroed with them)
    hg_pair* out;
    uint64_t cap;
    hg_merge_result* result;
    uint32_t ntiles;
    // records mode (merge_level_kernel<2>, compaction): the live records
    // themselves, gathered from the arena into rec_out (rec_cap bytes) at
    // their output offsets -- no hg_pair array, no encode pass
    uint8_t* rec_out;
    uint64_t rec_cap;
    uint64_t* rec_off;             // nullable: each record's output offset (block index)
    hg_encode_result* enc_result;  // out_len, HG_ERR_CAPACITY past rec_cap
    // pairs mode (MODE 1), nullable: the encode's tile sums [enc_nt] and group
    // sums after them, accumulated here (zeroed by the round's split kernel)
    unsigned long long* enc_sums;
    uint64_t enc_nt, enc_words;  // tile sums; all words (tile + group sums)
    uint32_t enc_tile_log2, enc_group_log2;
    // test hook (knob HG_MERGE_TEST_LB_EXPIRE): this tile's look-back acts
    // as if its wait ran over the budget (~0u: none)
    uint32_t test_expire = ~0u;
};
constexpr uint32_t FIN_ENC_SLOTS = 17;  // encode tiles one merge tile's pairs can touch (>= 64 records each)
constexpr unsigned long long LB_AGG = 1ull << 62, LB_INCL = 2ull << 62;
constexpr unsigned long long LB_VAL = (1ull << 62) - 1;

// Live entries of the tiles before tile t (wave 0; every lane gets it) and
// publication of this tile's inclusive count.  The spin budget counts polls
// in which none of the awaited status words changed (a predecessor publishing
// its aggregate or inclusive count restarts it), so a busy or shared GPU only
// makes waits long; a wait over the budget means a stalled grid and flags the
// merge (err) for a redo: never an endless spin.  (A grid-wide progress
// counter bumped by every tile measured 16-22 % slower on the cfg 5 legs:
// thousands of tiles contending for one atomic.)
__device__ __forceinline__ void final_publish(const FinalArgs& f, uint32_t t, unsigned long long v) {
    hgk::st_agent(&f.st[t], v);
}

__device__ uint64_t final_lookback(const FinalArgs& f, uint32_t t, uint64_t agg,
                                   unsigned long long* err) {
    const uint32_t lane = threadIdx.x & 63u;
    if (t == 0) {
        if (lane == 0) final_publish(f, 0, LB_INCL | agg);
        return 0;
    }
    if (t == f.test_expire) {  // test hook: a wait over the budget
        if (lane == 0) {
            atomicMin(err, 0ull);
            final_publish(f, t, LB_INCL | agg);
        }
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
                    final_publish(f, t, LB_INCL | agg);
                }
                return 0;
            }
            __builtin_amdgcn_s_sleep(1);
            bool moved = false;
            if (j >= 0 && (w >> 62) == 0) {
                const unsigned long long w2 = hgk::ld_agent(&f.st[j]);
                moved = w2 != w;
                w = w2;
            }
            if (__ballot(moved)) spins = 0;
        }
        acc += hgk::wave_sum<uint64_t>(((rel >> lane) & 1ull) ? (w & LB_VAL) : 0ull);
        if (incl) break;
        j0 -= 64;
    }
    if (lane == 0) final_publish(f, t, LB_INCL | (acc + agg));
    return acc;
}

// Records mode: the look-back over (live records, output bytes) of the tiles
// before tile t -- two status words per tile, st[t] and st[ntiles + t], each
// written whole with the same flag (AGG, then INCL); a predecessor whose two
// words do not show the same flag yet (caught between its two stores) reads
// as not ready.  Wave 0; every lane gets (base_c, base_b).
__device__ void final_lookback2(const FinalArgs& f, uint32_t t, uint64_t agg_c, uint64_t agg_b,
                                unsigned long long* err, uint64_t& base_c, uint64_t& base_b) {
    const uint32_t lane = threadIdx.x & 63u;
    unsigned long long* stb = f.st + f.ntiles;
    base_c = base_b = 0;
    if (t == 0) {
        if (lane == 0) {
            hgk::st_agent(&f.st[0], LB_INCL | agg_c);
            hgk::st_agent(&stb[0], LB_INCL | agg_b);
        }
        return;
    }
    if (lane == 0 && t != f.test_expire) {
        hgk::st_agent(&f.st[t], LB_AGG | agg_c);
        hgk::st_agent(&stb[t], LB_AGG | agg_b);
    }
    if (t == f.test_expire) {  // test hook: a wait over the budget
        if (lane == 0) {
            atomicMin(err, 0ull);
            hgk::st_agent(&f.st[t], LB_INCL | agg_c);
            hgk::st_agent(&stb[t], LB_INCL | agg_b);
        }
        return;
    }
    uint64_t acc_c = 0, acc_b = 0;
    int64_t j0 = (int64_t)t - 1;
    uint32_t spins = 0;
    for (;;) {
        const int64_t j = j0 - (int64_t)lane;
        unsigned long long w = j >= 0 ? hgk::ld_agent(&f.st[j]) : LB_INCL;
        unsigned long long wb = j >= 0 ? hgk::ld_agent(&stb[j]) : LB_INCL;
        unsigned long long incl, rel;
        for (;;) {
            const uint32_t fl = (w >> 62) == (wb >> 62) ? (uint32_t)(w >> 62) : 0u;
            incl = __ballot(fl == 2);
            const int fi = incl ? __ffsll((long long)incl) - 1 : 63;
            rel = fi >= 63 ? ~0ull : ((1ull << (fi + 1)) - 1ull);
            if (!(__ballot(fl == 0) & rel)) break;
            if (++spins > (1u << 22)) {
                if (lane == 0) {
                    atomicMin(err, 0ull);
                    hgk::st_agent(&f.st[t], LB_INCL | agg_c);
                    hgk::st_agent(&stb[t], LB_INCL | agg_b);
                }
                return;
            }
            __builtin_amdgcn_s_sleep(1);
            bool moved = false;
            if (j >= 0 && fl == 0) {
                const unsigned long long w2 = hgk::ld_agent(&f.st[j]);
                const unsigned long long wb2 = hgk::ld_agent(&stb[j]);
                moved = w2 != w || wb2 != wb;
                w = w2;
                wb = wb2;
            }
            if (__ballot(moved)) spins = 0;
        }
        const bool in = (rel >> lane) & 1ull;
        acc_c += hgk::wave_sum<uint64_t>(in ? (w & LB_VAL) : 0ull);
        acc_b += hgk::wave_sum<uint64_t>(in ? (wb & LB_VAL) : 0ull);
        if (incl) break;
        j0 -= 64;
    }
    if (lane == 0) {
        hgk::st_agent(&f.st[t], LB_INCL | (acc_c + agg_c));
        hgk::st_agent(&stb[t], LB_INCL | (acc_b + agg_b));
    }
    base_c = acc_c;
    base_b = acc_b;
}

// 16 bytes of the arena from p, never outside [0, len) (a window past either
// end is assembled byte by byte: records at the arena's edges).
__device__ __forceinline__ uint4 arena16(const uint8_t* arena, uint64_t len, int64_t p) {
    if (p >= 0 && (uint64_t)p + 16 <= len) return *reinterpret_cast<const uint4*>(arena + p);
    uint8_t b[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        const int64_t q = p + i;
        b[i] = (q >= 0 && (uint64_t)q < len) ? arena[q] : 0;
    }
    return make_uint4(b[0] | (b[1] << 8) | (b[2] << 16) | ((uint32_t)b[3] << 24),
                      b[4] | (b[5] << 8) | (b[6] << 16) | ((uint32_t)b[7] << 24),
                      b[8] | (b[9] << 8) | (b[10] << 16) | ((uint32_t)b[11] << 24),
                      b[12] | (b[13] << 8) | (b[14] << 16) | ((uint32_t)b[15] << 24));
}
// Byte mask of dword i for the bytes of a 16-byte window below n (n in [0, 16]).
__device__ __forceinline__ uint32_t low_mask(uint32_t n, uint32_t i) {
    const int32_t k = (int32_t)n - 4 * (int32_t)i;
    return k >= 4 ? ~0u : (k <= 0 ? 0u : (1u << (8 * k)) - 1u);
}
// The low n (< 16) bytes of v to dst by 8 / 4 / 2 / 1-byte stores.
__device__ __forceinline__ void store_low(uint8_t* dst, uint4 v, uint32_t n) {
    const uint64_t lo = ((uint64_t)v.y << 32) | v.x, hi = ((uint64_t)v.w << 32) | v.z;
    uint32_t o = 0;
    uint64_t cur = lo;
    if (n & 8) {
        *reinterpret_cast<uint64_t*>(dst) = lo;
        o = 8;
        cur = hi;
    }
    if (n & 4) {
        *reinterpret_cast<uint32_t*>(dst + o) = (uint32_t)cur;
        cur >>= 32;
        o += 4;
    }
    if (n & 2) {
        *reinterpret_cast<uint16_t*>(dst + o) = (uint16_t)cur;
        cur >>= 16;
        o += 2;
    }
    if (n & 1) dst[o] = (uint8_t)cur;
}
typedef uint32_t m_u32x4 __attribute__((ext_vector_type(4)));
// Records mode: 16-byte output pieces per lane per step of the gather (their
// loads in flight together) and the kernel's waves per SIMD.
#ifndef HG_REC_GU
#define HG_REC_GU 1  // cfg 5 leg: 1 595 us, 2 630 us (more spills)
#endif
constexpr uint32_t REC_GU = HG_REC_GU;
#ifndef HG_REC_WAVES
#define HG_REC_WAVES 5
#endif

// err: the order check's result; merging unsorted runs is meaningless (and
// their merge paths are not monotone), so every round skips work once set.
// MODE 0: a round writing entries; 1 (FINAL): the last round, emitting pairs
// (f) instead of entries (out unused); 2 (FINAL, records mode): the last
// round of a compaction, writing the live records' bytes themselves.
template <int MODE>
// Occupancy over registers: bounded to 5 (6 for the last round) waves/SIMD
// the rounds run faster despite a few spilled registers (cfg 5 leg: 96 -> 92
// and 185 -> 167 us against 4 waves/SIMD unbounded).
__global__ __launch_bounds__(THREADS, MODE == 1 ? 6 : MODE == 2 ? HG_REC_WAVES : 5) void merge_level_kernel(MergeArgs a, LevelArgs l,
                                                              const MEnt* in, MEnt* out,
                                                              const uint64_t* split,
                                                              unsigned long long* err,
                                                              FinalArgs f) {
    constexpr bool FINAL = MODE != 0;
    __shared__ LevelSmem s;
    __shared__ uint32_t fin_tmp[THREADS / 64];
    __shared__ uint64_t fin_base, fin_bbase, fin_tmp64[THREADS / 64];
    __shared__ unsigned long long fin_esum[FIN_ENC_SLOTS];  // MODE 1: this tile's bytes per encode tile
    // FINAL: the tables' run offsets, span arrays and arena offsets in LDS
    // (up to FIN_LDS_TABLES tables), so a live record's span lookup is one
    // HBM load after an LDS search instead of a chain of dependent loads
    __shared__ uint64_t fin_roff[FIN_LDS_TABLES + 1], fin_sp[FIN_LDS_TABLES],
        fin_toff[FIN_LDS_TABLES];
    const uint32_t tid = threadIdx.x;
    // (tiles in blockIdx order: an XCD-contiguous deal of the tiles, measured
    // round 4, made the non-final rounds 87 -> 94 us and the record gather
    // 368 -> 376 us on the cfg 5 leg)
    // The FINAL round's look-back waits on the tiles before it, so its tile
    // index is a ticket drawn when the workgroup starts: every tile it waits
    // on is then already resident and running.  By blockIdx a later tile
    // could occupy a CU while an earlier one still waits for dispatch -- on
    // a GPU shared with another process (whose waves hold the earlier
    // tile's XCD) that wait ran out the spin budget and the merge went to a
    // redo, 4-125 s per compaction (profiles/r5_bench_n2_shared_gpu_rehearsal.json).
    __shared__ uint32_t fin_ticket;
    if (FINAL) {
        if (tid == 0) fin_ticket = atomicAdd(reinterpret_cast<unsigned int*>(f.st + 2 * (uint64_t)f.ntiles), 1u);
        __syncthreads();
    }
    const uint32_t bx = FINAL ? fin_ticket : blockIdx.x;
    const uint64_t t0 = (uint64_t)bx * TILE;
    if (t0 >= a.n) return;
    const bool fin_lds = FINAL && a.ntables <= FIN_LDS_TABLES;
    if (MODE == 1 && tid < FIN_ENC_SLOTS) fin_esum[tid] = 0;  // read after later barriers
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
        if (MODE == 1 && tid < 64) final_lookback(f, bx, 0, err);
        if (MODE == 2 && tid < 64) {
            uint64_t bc, bb;
            final_lookback2(f, bx, 0, 0, err, bc, bb);
        }
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
        const uint64_t i0 = d0 == t0 ? split[bx] : 0;
        const uint64_t i1 = d1 == oend ? na : split[bx + 1];
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
                // before it (look-back), then the pairs (MODE 1) or the
                // records' bytes (MODE 2) at their positions
                uint32_t ftot;
                const uint32_t fpre = hgk::block_excl_scan<THREADS / 64>(fcnt, fin_tmp, ftot);
                // the spans of this thread's outputs, every load issued
                // before the first is used (branch-free: an output past the
                // tile or dead looks up entry 0 and is dropped below).  MODE
                // 1 looks them up after the look-back (their registers are
                // not live across it: no spills), MODE 2 before (it needs
                // the record sizes for the byte look-back)
                uint32_t tk[EPT];
                hg_span spk[EPT];
                uint64_t tof[EPT];
                auto lookups = [&]() {
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
                };
                if (MODE == 1) {
                    if (tid < 64) {
                        const uint64_t b = final_lookback(f, bx, ftot, err);
                        if (tid == 0) {
                            fin_base = b;
                            if (bx + 1 == f.ntiles) {
                                hg_merge_result r;
                                r.n_out = b + ftot;
                                r.kind = HG_OK;
                                r.table = 0;
                                r.index = 0;
                                *f.result = r;
                            }
                        }
                    }
                    lookups();
                    hg_pair* lp = reinterpret_cast<hg_pair*>(s.seg);
                    uint32_t r = fpre;
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
                    if (f.enc_sums) {
                        // the encode's record sizes per tile of its output
                        // (pair q in encode tile q >> tile_log2): into LDS,
                        // then one atomic per touched tile and group
                        const uint64_t T0 = fin_base >> f.enc_tile_log2;
                        for (uint32_t i = tid; i < ftot; i += THREADS) {
                            const hg_pair& p = lp[i];
                            atomicAdd(&fin_esum[((fin_base + i) >> f.enc_tile_log2) - T0],
                                      16ull + p.klen + p.vlen);
                        }
                        __syncthreads();
                        if (tid < FIN_ENC_SLOTS && fin_esum[tid]) {
                            const uint64_t T = T0 + tid;
                            atomicAdd(f.enc_sums + T, fin_esum[tid]);
                            atomicAdd(f.enc_sums + f.enc_nt + (T >> f.enc_group_log2), fin_esum[tid]);
                        }
                    }
                } else {
                    // records mode: each live record's source (its header in
                    // the arena) and output offset in the tile go to LDS --
                    // src[0, ftot), off[0, ftot], in place of the segments --
                    // then the tile's output bytes [B, B + btot) are written
                    // as 16-byte pieces aligned in the OUTPUT (a piece takes
                    // the bytes of the record it starts in and, across a record
                    // boundary, the next one's; the pieces at the tile's two
                    // edges only the tile's own bytes)
                    lookups();
                    uint64_t bsz = 0;
#pragma unroll
                    for (uint32_t k = 0; k < EPT; ++k)
                        if (d + k < e && !(fx[k].gd & DEAD)) bsz += 16ull + spk[k].klen + spk[k].vlen;
                    uint64_t bx64 = bsz;  // block exclusive scan (u64)
#pragma unroll
                    for (uint32_t dd = 1; dd < 64; dd <<= 1) {
                        const uint64_t y = __shfl_up(bx64, dd, 64);
                        if ((tid & 63u) >= dd) bx64 += y;
                    }
                    if ((tid & 63u) == 63u) fin_tmp64[tid >> 6] = bx64;
                    __syncthreads();
                    uint64_t bpre = bx64 - bsz, btot = 0;
#pragma unroll
                    for (uint32_t w = 0; w < THREADS / 64; ++w) {
                        bpre += w < (tid >> 6) ? fin_tmp64[w] : 0ull;
                        btot += fin_tmp64[w];
                    }
                    if (tid < 64) {
                        uint64_t bc, bb;
                        final_lookback2(f, bx, ftot, btot, err, bc, bb);
                        if (tid == 0) {
                            fin_base = bc;
                            fin_bbase = bb;
                            if (bx + 1 == f.ntiles) {
                                hg_merge_result r;
                                r.n_out = bc + ftot;
                                r.kind = HG_OK;
                                r.table = 0;
                                r.index = 0;
                                *f.result = r;
                                hg_encode_result er;
                                er.out_len = bb + btot;
                                er.kind = bb + btot <= f.rec_cap ? HG_OK : HG_ERR_CAPACITY;
                                er.reserved = 0;
                                *f.enc_result = er;
                            }
                        }
                    }
                    uint64_t* lsrc = reinterpret_cast<uint64_t*>(s.seg);
                    uint64_t* loff = lsrc + TILE;
                    uint32_t r = fpre;
                    uint64_t o = bpre;
#pragma unroll
                    for (uint32_t k = 0; k < EPT; ++k) {
                        if (d + k >= e || (fx[k].gd & DEAD)) continue;
                        lsrc[r] = tof[k] + spk[k].off;
                        loff[r] = o;
                        o += 16ull + spk[k].klen + spk[k].vlen;
                        ++r;
                    }
                    if (tid == 0) loff[ftot] = btot;
                    __syncthreads();  // also publishes fin_base / fin_bbase
                    const uint64_t B = fin_bbase, bc = fin_base;
                    if (f.rec_off)
                        for (uint32_t i = tid; i < ftot; i += THREADS) f.rec_off[bc + i] = B + loff[i];
                    const uint64_t P0 = B >> 4, np = ((B + btot + 15) >> 4) - P0;
                    const float scale = btot ? (float)ftot / (float)btot : 0.f;
                    for (uint64_t i0 = 0; btot && i0 < np; i0 += (uint64_t)THREADS * REC_GU) {
                        uint4 v[REC_GU], w2[REC_GU];
                        uint32_t n1[REC_GU], need[REC_GU];
                        uint64_t lo[REC_GU];
#pragma unroll
                        for (uint32_t u = 0; u < REC_GU; ++u) {  // every load before any store
                            const uint64_t i = min(i0 + (uint64_t)u * THREADS + tid, np - 1);
                            const uint64_t A = (P0 + i) << 4;
                            lo[u] = (A > B ? A : B) - B;  // tile-relative
                            need[u] = (uint32_t)(min(A + 16, B + btot) - B - lo[u]);
                            uint32_t rr = min((uint32_t)((float)lo[u] * scale), ftot - 1);  // interpolate, walk
                            while (rr > 0 && loff[rr] > lo[u]) --rr;
                            while (rr + 1 < ftot && loff[rr + 1] <= lo[u]) ++rr;
                            const uint64_t rem = loff[rr + 1] - lo[u];  // record rr's bytes from lo
                            n1[u] = rem < 16 ? (uint32_t)rem : 16u;
                            v[u] = arena16(a.arena, a.arena_len, (int64_t)(lsrc[rr] + (lo[u] - loff[rr])));
                            w2[u] = n1[u] < need[u]  // the next record supplies bytes [n1, need)
                                        ? arena16(a.arena, a.arena_len, (int64_t)lsrc[rr + 1] - (int64_t)n1[u])
                                        : make_uint4(0, 0, 0, 0);
                        }
#pragma unroll
                        for (uint32_t u = 0; u < REC_GU; ++u) {
                            if (i0 + (uint64_t)u * THREADS + tid >= np) continue;
                            uint4 x = v[u];
                            if (n1[u] < need[u]) {
                                x.x = (x.x & low_mask(n1[u], 0)) | (w2[u].x & ~low_mask(n1[u], 0));
                                x.y = (x.y & low_mask(n1[u], 1)) | (w2[u].y & ~low_mask(n1[u], 1));
                                x.z = (x.z & low_mask(n1[u], 2)) | (w2[u].z & ~low_mask(n1[u], 2));
                                x.w = (x.w & low_mask(n1[u], 3)) | (w2[u].w & ~low_mask(n1[u], 3));
                            }
                            const uint64_t O = B + lo[u];  // absolute output offset
                            if (O >= f.rec_cap) continue;
                            const uint32_t lim = (uint32_t)min((uint64_t)need[u], f.rec_cap - O);
                            if (lim == 16) {
                                m_u32x4 xv = {x.x, x.y, x.z, x.w};
                                __builtin_nontemporal_store(xv, reinterpret_cast<m_u32x4*>(f.rec_out + O));
                            } else {
                                store_low(f.rec_out + O, x, lim);
                            }
                        }
                    }
                }
            }
        }
        d0 = d1;
        __syncthreads();
    }
}

// ---- 3b. one-pass k-way merge (K <= KW_MAX runs) -----------------------------------------
// The 3 rounds of 2-way merges above move every entry through HBM three times
// (8 runs: 2 x 86 + 156 us, plus 3 x 23 us of split searches on the cfg 5
// leg).  Here one pass does it: tiles are cut at sampled splitters instead of
// fixed output positions, so a tile's share of every run is known from K
// searches and the tile merges its K segments inside LDS.
//   kw_sample_kernel: every KW_S-th entry of each run (a sample), in run
//     order, into a compact array (L2-resident for the searches below).
//   kw_split_kernel: each sample's rank among all samples in the strict total
//     order (key, run) -- K - 1 searches over the other runs' samples, one
//     lane each -- and for every KW_M-th rank (a splitter) its exact position
//     in every run: the search narrowed to the KW_S entries between two
//     samples.  Tile k = the entries from splitter k to splitter k + 1: in run
//     i at most KW_S x (samples of run i in between + 1) - 1 entries, so
//     <= KW_S KW_M + K (KW_S - 1) <= KW_CAP in all.
//   kw_merge_kernel: a tile's K segments into LDS, log2(K) pairwise merge
//     passes in place (merge path per thread, ties: the lower run first; a
//     B element equal to the last A element before it is dead -- newest
//     wins, as the rounds), then the FINAL round's emission (look-back over
//     the tiles' live counts, pairs).  An entry equal to one of a higher
//     priority run in an earlier tile can only be its segment's first and
//     that run's entry just before the tile: checked when staging.
// Measured (cfg 5 leg, 8 x 1 M, same box, profiles/r4_ab_spec_emit.log): one
// pass is slower than the rounds -- kw_merge_kernel 425 us + 43 us of splits
// against 2 x 93 + 161 us + 3 x 22 us; without its LDS passes it still takes
// 258 us (the FINAL emission's span lookups and look-back dominate, at 4
// workgroups per CU), and the three in-LDS passes cost another 167 us of
// dependent LDS compares.  Kept behind HG_MERGE_KWAY=1 (tests compare it with
// the oracle and the rounds), not the default.
constexpr uint32_t KW_S = 64;
constexpr uint32_t KW_M = 16;
constexpr uint32_t KW_MAX = 8;
constexpr uint32_t KW_CAP = 1536;  // >= KW_S KW_M + KW_MAX (KW_S - 1) = 1528
constexpr uint32_t KW_THREADS = 384;
constexpr uint32_t KW_EPT = KW_CAP / KW_THREADS;  // 4
constexpr uint32_t KW_WPT = 3 * KW_EPT;           // 8-byte words per thread when staging
static_assert(KW_S * KW_M + KW_MAX * (KW_S - 1) <= KW_CAP, "tile bound");

struct KwArgs {
    uint64_t roff[KW_MAX + 1];  // the runs' entry offsets in `in`
    uint32_t soff[KW_MAX + 1];  // their samples' offsets (ceil(len / KW_S) each)
    uint32_t K, ns, ntiles;     // runs, samples, tiles (ceil(ns / KW_M))
};

__device__ __forceinline__ uint32_t kw_run_of_sample(const KwArgs& k, uint32_t s) {
    uint32_t j = 0;
#pragma unroll
    for (uint32_t i = 1; i < KW_MAX; ++i)
        if (i < k.K && k.soff[i] <= s) j = i;
    return j;
}

// Samples, and the FINAL look-back statuses zeroed (one launch fewer).
__global__ __launch_bounds__(THREADS) void kw_sample_kernel(KwArgs k, const MEnt* in, MEnt* samp,
                                                            unsigned long long* zst) {
    const uint32_t s = blockIdx.x * THREADS + threadIdx.x;
    if (s < k.ntiles) zst[s] = 0;
    if (s >= k.ns) return;
    const uint32_t j = kw_run_of_sample(k, s);
    samp[s] = in[k.roff[j] + (uint64_t)(s - k.soff[j]) * KW_S];
}

// y (run i) before x (run j) in the order (key, run).
__device__ __forceinline__ bool kw_before(const MergeArgs& a, const MEnt& y, uint32_t i, const MEnt& x,
                                          uint32_t j) {
    const int c = key_cmp(a, y, x);
    return c < 0 || (c == 0 && i < j);
}

// Eight lanes per sample (lane i: run i).  split[t * K + i] = tile t's first
// entry of run i (run-relative), t = 0 .. ntiles (the last row: the run ends).
__global__ __launch_bounds__(THREADS) void kw_split_kernel(MergeArgs a, KwArgs k, const MEnt* in,
                                                           const MEnt* samp, uint64_t* split,
                                                           const unsigned long long* err) {
    const uint32_t gt = blockIdx.x * THREADS + threadIdx.x;
    const uint32_t s = gt / KW_MAX, i = gt % KW_MAX;
    if (s >= k.ns || *err != ~0ull) return;  // (the merge kernel aborts on err)
    const uint32_t j = kw_run_of_sample(k, s);
    const uint32_t u = s - k.soff[j];
    const MEnt x = samp[s];
    // q: samples of run i before x
    uint32_t q = 0;
    if (i == j) {
        q = u;
    } else if (i < k.K) {
        uint32_t lo = 0, hi = k.soff[i + 1] - k.soff[i];
        const MEnt* si = samp + k.soff[i];
        while (lo < hi) {
            const uint32_t mid = (lo + hi) >> 1;
            if (kw_before(a, si[mid], i, x, j)) lo = mid + 1;
            else hi = mid;
        }
        q = lo;
    }
    uint32_t rank = q;  // sum over the sample's eight lanes
#pragma unroll
    for (uint32_t d = 1; d < KW_MAX; d <<= 1) rank += __shfl_xor(rank, d, 64);
    if (s == 0 && i < k.K) split[(uint64_t)k.ntiles * k.K + i] = k.roff[i + 1] - k.roff[i];
    if (rank % KW_M || i >= k.K) return;
    const uint64_t t = rank / KW_M;
    uint64_t pos;
    if (i == j) {
        pos = (uint64_t)u * KW_S;
    } else {
        // entries of run i before x: in [KW_S (q - 1) + 1, KW_S q] (q > 0), else 0
        const uint64_t len = k.roff[i + 1] - k.roff[i];
        uint64_t lo = q ? (uint64_t)KW_S * (q - 1) + 1 : 0, hi = min((uint64_t)KW_S * q, len);
        const MEnt* ri = in + k.roff[i];
        while (lo < hi) {
            const uint64_t mid = (lo + hi) >> 1;  // entry mid before x <=> more than mid entries are
            if (kw_before(a, ri[mid], i, x, j)) lo = mid + 1;
            else hi = mid;
        }
        pos = lo;
    }
    split[t * k.K + i] = pos;
}

struct KwSmem {
    alignas(16) MEnt seg[KW_CAP];
    MEnt prev[KW_MAX];
    uint32_t so[KW_MAX + 1];  // segment offsets in seg (so[i] = N for i >= K)
    uint64_t c0[KW_MAX];      // the tile's first entry of each run (run-relative)
    uint32_t has_prev[KW_MAX];
    uint32_t bad;
};

__global__ __launch_bounds__(KW_THREADS, 2) void kw_merge_kernel(MergeArgs a, KwArgs k, const MEnt* in,
                                                                  const uint64_t* split,
                                                                  unsigned long long* err, FinalArgs f) {
    __shared__ KwSmem s;
    __shared__ uint32_t fin_tmp[KW_THREADS / 64];
    __shared__ uint64_t fin_base;
    __shared__ uint64_t fin_roff[FIN_LDS_TABLES + 1], fin_sp[FIN_LDS_TABLES], fin_toff[FIN_LDS_TABLES];
    const uint32_t tid = threadIdx.x;
    const uint32_t bx = blockIdx.x;
    const uint32_t K = k.K;
    const bool fin_lds = a.ntables <= FIN_LDS_TABLES;
    if (fin_lds) {
        if (tid <= a.ntables) fin_roff[tid] = a.run_off[tid];
        if (tid < a.ntables) {
            fin_sp[tid] = reinterpret_cast<uint64_t>(a.spans[tid]);
            fin_toff[tid] = a.table_off[tid];
        }
    }
    if (tid == 0) s.bad = 0;
    if (tid < KW_MAX) {
        // once the order check failed the split kernel wrote nothing: no
        // split is read then, and none is used unless it lies in its run
        const bool errset = *err != ~0ull;
        uint64_t c0 = 0, c1 = 0;
        if (tid < K && !errset) {
            c0 = split[(uint64_t)bx * K + tid];
            c1 = split[(uint64_t)(bx + 1) * K + tid];
        }
        const uint64_t rl = tid < K ? k.roff[tid + 1] - k.roff[tid] : 0;
        const bool okc = c0 <= c1 && c1 <= rl && c1 - c0 <= KW_CAP;
        if (!okc) c0 = c1 = 0;
        s.c0[tid] = c0;
        // segment lengths -> offsets (eight lanes of wave 0)
        const uint32_t len = okc ? (uint32_t)(c1 - c0) : KW_CAP + 1;
        uint32_t incl = len;
#pragma unroll
        for (uint32_t d = 1; d < KW_MAX; d <<= 1) {
            const uint32_t o = __shfl_up(incl, d, 64);
            if (tid >= d) incl += o;
        }
        s.so[tid + 1] = incl;
        if (tid == 0) s.so[0] = 0;
        s.has_prev[tid] = tid < K && c0 > 0;
        if (tid < K && c0 > 0) s.prev[tid] = in[k.roff[tid] + c0 - 1];
        if (tid == KW_MAX - 1 && (incl > KW_CAP || errset)) s.bad = 1;
    }
    __syncthreads();
    if (s.bad) {  // unsorted input (err) or splits no sorted input gives
        if (*err == ~0ull && tid == 0) atomicMin(err, 0ull);
        if (tid < 64) final_lookback(f, bx, 0, err);
        return;
    }
    const uint32_t N = s.so[KW_MAX];
    {  // the segments as 8-byte words, every load before the first LDS write
        uint64_t v[KW_WPT];
        uint64_t* ws = reinterpret_cast<uint64_t*>(s.seg);
#pragma unroll
        for (uint32_t r = 0; r < KW_WPT; ++r) {
            const uint32_t w = tid + r * KW_THREADS;
            v[r] = 0;
            if (w < 3 * N) {
                const uint32_t e = w / 3;
                uint32_t i = 0;
#pragma unroll
                for (uint32_t q = 1; q < KW_MAX; ++q)
                    if (s.so[q] <= e) i = q;
                const uint64_t* src = reinterpret_cast<const uint64_t*>(in + k.roff[i] + s.c0[i]);
                v[r] = src[w - 3 * s.so[i]];
            }
        }
#pragma unroll
        for (uint32_t r = 0; r < KW_WPT; ++r) {
            const uint32_t w = tid + r * KW_THREADS;
            if (w < 3 * N) ws[w] = v[r];
        }
    }
    __syncthreads();
    // a segment's first entry equal to a higher-priority run's entry just
    // before the tile: dead (newest wins across the tile edge)
    if (tid < K && s.so[tid + 1] > s.so[tid]) {
        MEnt& x = s.seg[s.so[tid]];
        bool eq = false;
        for (uint32_t i = 0; i < tid; ++i)
            if (s.has_prev[i] && key_cmp(a, s.prev[i], x) == 0) eq = true;
        if (eq) x.gd |= DEAD;
    }
    __syncthreads();
    MEnt fx[KW_EPT];
    const uint32_t d0 = tid * KW_EPT;
    for (uint32_t w = 1; w < K; w <<= 1) {
        // pass: runs [2 p w, (2 p + 1) w) (A) and [(2 p + 1) w, (2 p + 2) w) (B) merge
        uint32_t pend = 0, ai = 0, bj = 0, A0 = 0, Am = 0, B1 = 0;
#pragma unroll
        for (uint32_t e = 0; e < KW_EPT; ++e) {
            const uint32_t pos = d0 + e;
            if (pos >= N) break;
            if (pos >= pend) {  // the pair holding pos, and its merge-path split there
                uint32_t p = 0;
                for (uint32_t q = 2 * w; q < KW_MAX; q += 2 * w)
                    if (s.so[q] <= pos) p = q;
                A0 = s.so[p];
                Am = s.so[p + w];
                B1 = s.so[min(p + 2 * w, KW_MAX)];
                pend = B1;
                const uint32_t na = Am - A0, nb = B1 - Am, dd = pos - A0;
                uint32_t lo = dd > nb ? dd - nb : 0, hi = dd < na ? dd : na;
                while (lo < hi) {
                    const uint32_t mid = (lo + hi) >> 1;
                    if (key_cmp(a, s.seg[A0 + mid], s.seg[Am + dd - 1 - mid]) <= 0) lo = mid + 1;
                    else hi = mid;
                }
                ai = lo;
                bj = dd - lo;
            }
            const uint32_t na = Am - A0, nb = B1 - Am;
            const MEnt* SA = s.seg + A0;
            const MEnt* SB = s.seg + Am;
            MEnt x;
            if (bj >= nb || (ai < na && key_cmp(a, SA[ai], SB[bj]) <= 0)) {
                x = SA[ai++];
            } else {
                x = SB[bj++];
                if (ai > 0 && key_cmp(a, SA[ai - 1], x) == 0) x.gd |= DEAD;
            }
            fx[e] = x;
        }
        __syncthreads();  // every thread is done reading this pass's input
        if (2 * w < K) {  // another pass follows
#pragma unroll
            for (uint32_t e = 0; e < KW_EPT; ++e)
                if (d0 + e < N) s.seg[d0 + e] = fx[e];
            __syncthreads();
        }
    }
    // FINAL emission (as merge_level_kernel<true>)
    const uint32_t ne = d0 < N ? min(KW_EPT, N - d0) : 0u;
    uint32_t fcnt = 0;
#pragma unroll
    for (uint32_t e = 0; e < KW_EPT; ++e) fcnt += e < ne && !(fx[e].gd & DEAD) ? 1u : 0u;
    uint32_t ftot;
    const uint32_t fpre = hgk::block_excl_scan<KW_THREADS / 64>(fcnt, fin_tmp, ftot);
    if (tid < 64) {
        const uint64_t b = final_lookback(f, bx, ftot, err);
        if (tid == 0) {
            fin_base = b;
            if (bx + 1 == f.ntiles) {
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
    uint32_t tk[KW_EPT];
    hg_span spk[KW_EPT];
    uint64_t tof[KW_EPT];
#pragma unroll
    for (uint32_t e = 0; e < KW_EPT; ++e) {
        const uint64_t g = e < ne ? (uint64_t)(fx[e].gd & ~DEAD) : 0ull;
        if (fin_lds) {
            uint32_t lo = 0, hi = a.ntables;
            while (hi - lo > 1) {
                const uint32_t mid = (lo + hi) >> 1;
                if (fin_roff[mid] <= g) lo = mid;
                else hi = mid;
            }
            tk[e] = lo;
            tof[e] = fin_toff[lo];
            spk[e] = reinterpret_cast<const hg_span*>(fin_sp[lo])[g - fin_roff[lo]];
        } else {
            tk[e] = run_of(a, g);
            tof[e] = a.table_off[tk[e]];
            spk[e] = a.spans[tk[e]][g - a.run_off[tk[e]]];
        }
    }
#pragma unroll
    for (uint32_t e = 0; e < KW_EPT; ++e) {
        if (e >= ne || (fx[e].gd & DEAD)) continue;
        const hg_span sp = spk[e];
        hg_pair p;
        p.key_off = tof[e] + sp.off + 16;
        p.val_off = p.key_off + sp.klen;
        p.klen = sp.klen;
        p.vlen = sp.vlen;
        lp[r++] = p;
    }
    __syncthreads();  // also publishes fin_base
    const uint64_t w0 = 3 * fin_base, wcap = 3 * f.cap;
    const uint64_t* s8 = reinterpret_cast<const uint64_t*>(s.seg);
    uint64_t* o8 = reinterpret_cast<uint64_t*>(f.out);
    for (uint32_t i = tid; i < 3 * ftot; i += KW_THREADS)
        if (w0 + i < wcap) o8[w0 + i] = s8[i];
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

// start (nullable): heads to begin from (table-local indices), n0: records
// already emitted before them (the epochs below hand over to this loop).
__global__ __launch_bounds__(64) void merge_exact_kernel(MergeArgs a, const MEnt* e,
                                                         const unsigned long long* err,
                                                         ExactHead* hs, hg_pair* out, uint64_t cap,
                                                         hg_merge_result* result,
                                                         const uint64_t* start, uint64_t n0) {
    // err nullptr (the epochs' hand-over): run the loop unconditionally
    if (err && *err == ~0ull) return;  // every table strictly increasing: the rounds did the merge
    const uint32_t lane = threadIdx.x;
    bool any = false;
    for (uint32_t t = lane; t < a.ntables; t += 64) {
        ExactHead h;
        h.idx = start ? start[t] : 0;
        h.cnt = a.run_off[t + 1] - a.run_off[t];
        if (h.idx < h.cnt) h.e = e[a.run_off[t] + h.idx];
        any |= h.idx < h.cnt;
        hs[t] = h;
    }
    uint64_t n = n0;
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

// ---- 6. epochs: the reference loop on tables that are not strictly increasing --------
// The loop (manager.rs:199-234) is a newest-wins merge of the tables' heads for
// as long as every table's remaining sequence is strictly increasing.  Cut
// each table at its DISORDER points (entries whose key is not greater than
// the one before): from heads h_t the loop equals the merge of the stretches
// [h_t, f_t) (f_t = the next disorder point) up to and including the key
// M = min over the tables with a disorder left of K_t[f_t - 1]; right after
// emitting M the first table reaches its disorder point.  So an epoch merges
// the sub-runs [h_t, u_t) (u_t = upper bound of M in the stretch; all of it
// when no disorder is left) with the parallel rounds, appends the pairs, and
// moves every head to u_t.  Each epoch consumes at least one disorder point.

// Disorder points: entries g (not the first of their table) with key[g] <=
// key[g - 1], appended to list (count; at most cap kept).
__global__ __launch_bounds__(THREADS) void merge_disorder_kernel(MergeArgs a, const MEnt* e,
                                                                 uint64_t* list,
                                                                 unsigned long long* count,
                                                                 uint64_t cap) {
    const uint64_t g = (uint64_t)blockIdx.x * THREADS + threadIdx.x;
    if (g >= a.n || g == 0) return;
    const uint32_t t = run_of(a, g);
    if (g == a.run_off[t]) return;
    if (key_cmp(a, e[g - 1], e[g]) >= 0) {
        const unsigned long long i = atomicAdd(count, 1ull);
        if (i < cap) list[i] = g;
    }
}

// One workgroup: M = the smallest key among the candidate entries cand[0, nc)
// (wave 0), then for every table t the upper bound u[t] of M in its stretch
// [lo[t], hi[t]) (table-local; entries strictly increasing there).  nc == 0:
// u = hi.
__global__ __launch_bounds__(THREADS) void merge_bound_kernel(MergeArgs a, const MEnt* e,
                                                              const uint64_t* cand, uint32_t nc,
                                                              const uint64_t* lo, const uint64_t* hi,
                                                              uint64_t* u) {
    __shared__ MEnt m;
    const uint32_t tid = threadIdx.x;
    if (tid < 64) {
        bool have = false;
        MEnt best;
        best.p0 = best.p1 = 0;
        best.klen = best.gd = 0;
        for (uint32_t i = tid; i < nc; i += 64) {
            const MEnt x = e[cand[i]];
            if (!have || key_cmp(a, x, best) < 0) {
                best = x;
                have = true;
            }
        }
#pragma unroll 1
        for (int d = 1; d < 64; d <<= 1) {
            const MEnt o = shfl_ent(best, (int)(tid ^ (uint32_t)d));
            const bool oh = __shfl((int)have, (int)(tid ^ (uint32_t)d), 64) != 0;
            if (oh && (!have || key_cmp(a, o, best) < 0)) {
                best = o;
                have = true;
            }
        }
        if (tid == 0) m = best;
    }
    __syncthreads();
    for (uint32_t t = tid; t < a.ntables; t += THREADS) {
        uint64_t l = lo[t], h = hi[t];
        if (nc) {  // first entry of [l, h) whose key is > M
            const MEnt* r = e + a.run_off[t];
            while (l < h) {
                const uint64_t mid = l + (h - l) / 2;
                if (key_cmp(a, r[mid], m) <= 0) l = mid + 1;
                else h = mid;
            }
        } else {
            l = h;
        }
        u[t] = l;
    }
}

// defer mode: the merge found input that is not strictly increasing and
// leaves it to the host's epoch driver (no pairs, n_out 0)
// zero/zero_words: a buffer the next kernel on the stream accumulates into
// (the compaction's encode block sums), cleared here instead of by a memset
__global__ void merge_flag_kernel(const unsigned long long* err, hg_merge_result* result,
                                  uint64_t* zero, uint64_t zero_words) {
    for (uint64_t i = threadIdx.x; i < zero_words; i += blockDim.x) zero[i] = 0;
    if (threadIdx.x != 0 || *err == ~0ull) return;
    hg_merge_result r;
    r.n_out = 0;
    r.kind = HG_ERR_UNSORTED;
    r.table = 0;
    r.index = 0;
    *result = r;
}

// ---- 7. rank path: the reference loop on heavily disordered tables ------------------------
// The loop's only operations on keys are "smallest head" and "equal to it"
// (manager.rs:209-227), so any order-preserving integer image of the keys runs
// it exactly.  Dense ranks (the number of distinct keys below a key) are built
// in parallel -- every entry sorted (tiles of TILE in LDS, then merge-path
// rounds over uniform runs), equal neighbours sharing a rank -- and the loop
// itself then runs in ONE wave on 4-byte ranks: lane t holds table t's head
// and next rank in registers, the smallest head is a DPP min over the lanes,
// the first table holding it is the lowest set bit of a ballot (min_by_key keeps
// the first minimum, :209-216), every lane whose head equals it advances
// (:218-227).  Each table's next ranks stream through an LDS ring of two
// halves refilled by LDS-DMA with counted waits, so no step waits on HBM; the
// winners' entry indices go out 64 at a time and a parallel kernel turns them
// into hg_pairs.  (The round-2 loop, merge_exact_kernel, compared 24-byte
// entries and chased a global load per step: ~1-2 us per record.)
constexpr uint32_t RANK_INF = 0xFFFFFFFFu;
constexpr uint32_t RANK_MAX_TABLES = 64;  // one lane per table
constexpr uint32_t RANK_LDS = 65536;      // the loop's LDS ring bytes
constexpr uint32_t RANK_PAD = 4096;       // ranks readable past n (ring fills run up to 2 H + 2 past a table's end)

__device__ __forceinline__ bool ent_is_pad(const MEnt& x) { return x.gd == 0xFFFFFFFFu; }

// x < y in key order; the padding of a short last tile sorts after everything
__device__ __forceinline__ bool sort_lt(const MergeArgs& a, const MEnt& x, const MEnt& y) {
    if (ent_is_pad(y)) return !ent_is_pad(x);
    if (ent_is_pad(x)) return false;
    return key_cmp(a, x, y) < 0;
}

// Every TILE entries of `in` sorted by key (bitonic network in LDS; equal keys
// in any order -- ranks do not depend on it) into `out`.
__global__ __launch_bounds__(THREADS) void sort_tile_kernel(MergeArgs a, const MEnt* in, MEnt* out) {
    __shared__ MEnt s[TILE];
    const uint32_t tid = threadIdx.x;
    const uint64_t t0 = (uint64_t)blockIdx.x * TILE;
    for (uint32_t i = tid; i < TILE; i += THREADS) {
        MEnt m;
        if (t0 + i < a.n) {
            m = in[t0 + i];
        } else {
            m.p0 = m.p1 = ~0ull;
            m.klen = m.gd = 0xFFFFFFFFu;
        }
        s[i] = m;
    }
    __syncthreads();
    for (uint32_t k = 2; k <= TILE; k <<= 1) {
        for (uint32_t j = k >> 1; j > 0; j >>= 1) {
            for (uint32_t q = tid; q < TILE / 2; q += THREADS) {
                const uint32_t i = ((q & ~(j - 1)) << 1) | (q & (j - 1)), l = i + j;
                const MEnt x = s[i], y = s[l];
                const bool up = (i & k) == 0;
                if (up ? sort_lt(a, y, x) : sort_lt(a, x, y)) {
                    s[i] = y;
                    s[l] = x;
                }
            }
            __syncthreads();
        }
    }
    for (uint32_t i = tid; i < TILE && t0 + i < a.n; i += THREADS) out[t0 + i] = s[i];
}

// Key-change flags of the sorted entries: f = 1 where a key differs from the
// one before it (the first entry: 1).  Thread tid of a tile owns 4
// consecutive entries.
__device__ __forceinline__ uint32_t rank_flags(const MergeArgs& a, const MEnt* srt, uint64_t i0,
                                               uint32_t f[EPT]) {
    uint32_t c = 0;
    MEnt prev;
    if (i0 > 0 && i0 < a.n) prev = srt[i0 - 1];
#pragma unroll
    for (uint32_t u = 0; u < EPT; ++u) {
        const uint64_t i = i0 + u;
        f[u] = 0;
        if (i < a.n) {
            const MEnt x = srt[i];
            f[u] = (i == 0 || key_cmp(a, prev, x) != 0) ? 1u : 0u;
            prev = x;
        }
        c += f[u];
    }
    return c;
}

__global__ __launch_bounds__(THREADS) void rank_count_kernel(MergeArgs a, const MEnt* srt,
                                                             uint32_t* tile_cnt) {
    __shared__ uint32_t ws[THREADS / 64];
    uint32_t f[EPT];
    uint32_t c = rank_flags(a, srt, (uint64_t)blockIdx.x * TILE + threadIdx.x * EPT, f);
    c = hgk::wave_sum<uint32_t>(c);
    if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t s = 0;
        for (uint32_t w = 0; w < THREADS / 64; ++w) s += ws[w];
        tile_cnt[blockIdx.x] = s;
    }
}

// rank[g] = distinct keys below entry g's key (g = the entry's index in the
// tables' layout), from the flags' prefix sums (tile bases from merge_scan_kernel).
// pack (every rank < 2^26, <= 64 tables): the value stored is rank << 6 |
// the entry's table, the loop's reduction key (rank_loop).
__global__ __launch_bounds__(THREADS) void rank_scatter_kernel(MergeArgs a, const MEnt* srt,
                                                               const uint64_t* tile_base,
                                                               uint32_t* rank, uint32_t pack) {
    __shared__ uint32_t tmp[THREADS / 64];
    const uint64_t i0 = (uint64_t)blockIdx.x * TILE + threadIdx.x * EPT;
    uint32_t f[EPT];
    const uint32_t c = rank_flags(a, srt, i0, f);
    uint32_t tot;
    uint64_t r = tile_base[blockIdx.x] + hgk::block_excl_scan<THREADS / 64>(c, tmp, tot);
#pragma unroll
    for (uint32_t u = 0; u < EPT; ++u) {
        if (i0 + u >= a.n) break;
        r += f[u];
        const uint32_t g = srt[i0 + u].gd & ~DEAD;
        rank[g] = pack ? ((uint32_t)(r - 1) << 6) | run_of(a, g) : (uint32_t)(r - 1);
    }
}

// Wave-wide inclusive min by DPP (lane 63 holds the wave's minimum); lanes
// without a source keep ~0 as the identity.
__device__ __forceinline__ uint32_t dpp_min_incl(uint32_t v) {
#define HG_DPP_MIN(ctrl, rmask) \
    v = min(v, (uint32_t)__builtin_amdgcn_update_dpp((int)RANK_INF, (int)v, ctrl, rmask, 0xf, false))
    HG_DPP_MIN(0x111, 0xf);
    HG_DPP_MIN(0x112, 0xf);
    HG_DPP_MIN(0x114, 0xf);
    HG_DPP_MIN(0x118, 0xf);
    HG_DPP_MIN(0x142, 0xa);
    HG_DPP_MIN(0x143, 0xc);
#undef HG_DPP_MIN
    return v;
}

// s_waitcnt vmcnt(min(n, 8)): this wave's vector memory operations retire in
// issue order, so "at most n outstanding" covers every one issued n or more
// operations ago (fewer allowed is merely conservative).
__device__ __forceinline__ void rank_wait_vm(uint32_t n) {
    switch (n) {
        case 0: __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
        case 1: __asm__ volatile("s_waitcnt vmcnt(1)" ::: "memory"); break;
        case 2: __asm__ volatile("s_waitcnt vmcnt(2)" ::: "memory"); break;
        case 3: __asm__ volatile("s_waitcnt vmcnt(3)" ::: "memory"); break;
        case 4: __asm__ volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
        case 5: __asm__ volatile("s_waitcnt vmcnt(5)" ::: "memory"); break;
        case 6: __asm__ volatile("s_waitcnt vmcnt(6)" ::: "memory"); break;
        case 7: __asm__ volatile("s_waitcnt vmcnt(7)" ::: "memory"); break;
        default: __asm__ volatile("s_waitcnt vmcnt(8)" ::: "memory"); break;
    }
}

__device__ __forceinline__ uint64_t readlane64(uint64_t v, uint32_t l) {
    return ((uint64_t)__builtin_amdgcn_readlane((uint32_t)(v >> 32), l) << 32) |
           __builtin_amdgcn_readlane((uint32_t)v, l);
}

struct RankArgs {
    const uint32_t* rank;     // dense rank per entry (tables' layout), RANK_PAD readable past n
    const uint64_t* run_off;  // [ntables + 1]
    uint32_t ntables;         // <= RANK_MAX_TABLES
    uint32_t H;               // ranks per ring half: a power of two >= 128, 2 H ntables 4 B <= RANK_LDS
    const uint64_t* start;    // [ntables] heads to start from (table-local)
    uint32_t* win_idx;        // out: the winners' entry indices, in output order
    uint64_t* steps;          // out: the number of winners
    uint32_t pack;            // rank entries are rank << 6 | table (rank_scatter_kernel)
};

// One half of table t's ring (ranks [q, q + H) of the table) by LDS-DMA; the
// whole wave issues it (wave-uniform LDS base, one 16-byte piece per lane).
// Returns the vector memory instructions issued.
__device__ __forceinline__ uint32_t rank_fill(const RankArgs& r, uint32_t* ring_half,
                                              const uint32_t* src) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t lanes = min(64u, r.H / 4), nins = max(1u, r.H / 256);
    for (uint32_t q = 0; q < nins; ++q)
        if (lane < lanes)
            __builtin_amdgcn_global_load_lds(static_cast<const void*>(src + q * 256 + lane * 4),
                                             (__attribute__((address_space(3))) void*)(ring_half + q * 256),
                                             16, 0, 0);
    return nins;
}

// Wave-wide min over the first 8 << (NL - 3) lanes by NL DPP steps (lanes
// without a source keep ~0): lane (8 << (NL - 3)) - 1 holds it.
template <int NL>
__device__ __forceinline__ uint32_t dpp_min_lanes(uint32_t v) {
#define HG_DPP_MIN(ctrl, rmask) \
    v = min(v, (uint32_t)__builtin_amdgcn_update_dpp((int)RANK_INF, (int)v, ctrl, rmask, 0xf, false))
    HG_DPP_MIN(0x111, 0xf);
    HG_DPP_MIN(0x112, 0xf);
    HG_DPP_MIN(0x114, 0xf);
    if (NL > 3) HG_DPP_MIN(0x118, 0xf);
    if (NL > 4) HG_DPP_MIN(0x142, 0xa);
    if (NL > 5) HG_DPP_MIN(0x143, 0xc);
#undef HG_DPP_MIN
    return __builtin_amdgcn_readlane(v, (8u << (NL - 3)) - 1u);
}

struct RankState {
    uint32_t idx, gidx, hk, pv, ob, tk0, tk1, vm;
};

// The loop proper (manager.rs:205-231), NL DPP steps over the tables' lanes.
// Lane t holds its head's key hk (PACK: rank << 6 | t, so the min also names
// the winner -- the lowest table holding the smallest key, min_by_key's first
// minimum -- without a ballot and a bit scan; else the rank) and pv, the ring
// slot of its next record, read one step ahead.
template <int NL, bool PACK>
__device__ __forceinline__ uint32_t rank_loop(const RankArgs& r, uint32_t* ring, const uint32_t* my,
                                              uint32_t base, uint32_t cnt, RankState& st) {
    const uint32_t lane = threadIdx.x;
    const uint32_t H = r.H, hs = (uint32_t)__builtin_ctz(H), RM = 2 * H - 1;
    uint32_t idx = st.idx, gidx = st.gidx, hk = st.hk, pv = st.pv;
    uint32_t ob = st.ob, tk0 = st.tk0, tk1 = st.tk1, vm = st.vm;
    uint32_t j = 0;
    for (;;) {
        const uint32_t key = dpp_min_lanes<NL>(hk);
        if (key == RANK_INF) break;  // every table exhausted (:228-230)
        const uint32_t w = PACK ? (key & 63u) : (uint32_t)__builtin_ctzll(__ballot(hk == key));
        const uint32_t gw = __builtin_amdgcn_readlane(gidx, w);
        ob = lane == (j & 63u) ? gw : ob;
        if ((j & 63u) == 63u) {
            r.win_idx[j - 63 + lane] = ob;
            ++vm;
        }
        ++j;
        // every table whose head equals the winner's key advances (:218-227)
        const bool adv = PACK ? (hk ^ key) < 64u : hk == key;
        if (adv) {
            ++idx;
            ++gidx;
            hk = idx < cnt ? pv : RANK_INF;
        }
        const uint32_t p = idx + 1;  // the next record's position
        const uint64_t cm = __ballot(adv && (p & (H - 1)) == 0);
        if (cm) {  // lanes entering a new half: it must have landed; refill the one left
            const uint32_t h = (p >> hs) & 1u;
            const uint32_t tkh = h ? tk1 : tk0;
            uint32_t allowed = RANK_INF;
            for (uint64_t c = cm; c; c &= c - 1)
                allowed = min(allowed, vm - __builtin_amdgcn_readlane(tkh, (uint32_t)__builtin_ctzll(c)));
            rank_wait_vm(allowed);
            for (uint64_t c = cm; c; c &= c - 1) {
                const uint32_t t = (uint32_t)__builtin_ctzll(c);
                const uint32_t bt = __builtin_amdgcn_readlane(base, t), pt = __builtin_amdgcn_readlane(p, t);
                const uint32_t th = (pt >> hs) & 1u;
                vm += rank_fill(r, ring + t * 2 * H + (th ^ 1u) * H, r.rank + bt + pt + H);
                if (lane == t) {
                    if (th) tk0 = vm;
                    else tk1 = vm;
                }
            }
        }
        // every lane reads its next record's slot (a lane that did not advance
        // reads the same one again: its half is refilled only once it has left
        // it), so the read lands in pv's own register, waited for one step later
        pv = my[p & RM];
    }
    st.ob = ob;
    st.vm = vm;
    return j;
}

__global__ __launch_bounds__(64) void rank_merge_kernel(RankArgs r) {
    extern __shared__ uint32_t ring[];  // [ntables][2][H]
    const uint32_t lane = threadIdx.x;
    const uint32_t H = r.H, hs = (uint32_t)__builtin_ctz(H), RM = 2 * H - 1;
    const bool mine = lane < r.ntables;
    // positions are table-local u32 (a merge holds < 2^31 entries)
    const uint32_t base = mine ? (uint32_t)r.run_off[lane] : 0u;
    const uint32_t cnt = mine ? (uint32_t)r.run_off[lane + 1] - base : 0u;
    RankState st;
    st.idx = mine ? (uint32_t)min(r.start[lane], (uint64_t)cnt) : 0u;
    st.hk = st.idx < cnt ? r.rank[base + st.idx] : RANK_INF;
    // the ring holds the table's ranks [b H, (b + 2) H) around the next
    // record's position idx + 1 (slot = position mod 2H); both halves now,
    // waited for
    for (uint32_t t = 0; t < r.ntables; ++t) {
        const uint32_t bt = __builtin_amdgcn_readlane(base, t), it = __builtin_amdgcn_readlane(st.idx, t);
        const uint32_t b = (it + 1) >> hs;
        uint32_t* rt = ring + t * 2 * H;
        rank_fill(r, rt + (b & 1u) * H, r.rank + bt + ((uint64_t)b << hs));
        rank_fill(r, rt + ((b + 1) & 1u) * H, r.rank + bt + ((uint64_t)(b + 1) << hs));
    }
    __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const uint32_t* my = ring + lane * 2 * H;
    st.pv = my[(st.idx + 1) & RM];
    st.vm = 0;            // vector memory instructions issued since (wave-uniform)
    st.tk0 = st.tk1 = 0;  // per half: vm right after its last refill was issued
    st.gidx = base + st.idx;
    st.ob = 0;
    uint32_t j;
    if (r.pack) {
        if (r.ntables <= 8) j = rank_loop<3, true>(r, ring, my, base, cnt, st);
        else if (r.ntables <= 16) j = rank_loop<4, true>(r, ring, my, base, cnt, st);
        else if (r.ntables <= 32) j = rank_loop<5, true>(r, ring, my, base, cnt, st);
        else j = rank_loop<6, true>(r, ring, my, base, cnt, st);
    } else {
        if (r.ntables <= 8) j = rank_loop<3, false>(r, ring, my, base, cnt, st);
        else if (r.ntables <= 16) j = rank_loop<4, false>(r, ring, my, base, cnt, st);
        else if (r.ntables <= 32) j = rank_loop<5, false>(r, ring, my, base, cnt, st);
        else j = rank_loop<6, false>(r, ring, my, base, cnt, st);
    }
    const uint32_t jl = j & 63u;
    if (jl && lane < jl) r.win_idx[j - jl + lane] = st.ob;
    if (lane == 0) *r.steps = j;
}

// The winners (entry indices in output order) -> hg_pairs at out[i], i <
// *steps and i < cap; the last thread of the grid's first workgroup writes the result.
__global__ __launch_bounds__(THREADS) void rank_emit_kernel(MergeArgs a, const uint32_t* win_idx,
                                                            const uint64_t* steps, hg_pair* out,
                                                            uint64_t cap, uint64_t n0,
                                                            hg_merge_result* result) {
    const uint64_t ns = *steps;
    const uint64_t i = (uint64_t)blockIdx.x * THREADS + threadIdx.x;
    if (i == 0) {
        hg_merge_result res;
        res.n_out = n0 + ns;
        res.kind = HG_OK;
        res.table = 1;  // on success: 1 = the serial reference loop produced the output
        res.index = 0;
        *result = res;
    }
    if (i >= ns || n0 + i >= cap) return;
    MEnt e;
    e.gd = win_idx[i];
    uint32_t t;
    const hg_span sp = ent_span(a, e, t);
    hg_pair p;
    p.key_off = a.table_off[t] + sp.off + 16;
    p.val_off = p.key_off + sp.klen;
    p.klen = sp.klen;
    p.vlen = sp.vlen;
    out[n0 + i] = p;
}

}  // namespace hgm

// ---- launcher ----------------------------------------------------------------------------
// Workspace (device): three entry buffers (the entries, then two ping-pong
// buffers for the rounds: the epochs keep the entries and gather into the
// other two), tile counts / bases / look-back words, the staging copy (table
// offsets, span pointers, run offsets of the tables and of every round), the
// error word, the exact loop's heads, and the epochs' scratch.
namespace {
extern "C" uint64_t hgk_merge_staging_bytes(uint32_t ntables);
extern "C" int hgk_decode_entries_launch(const void* d_stage, uint32_t ntab, uint32_t nspec_total,
                                         const uint64_t* d_run_off, void* d_ent,
                                         unsigned long long* d_err, hipStream_t stream);
constexpr uint64_t EPOCH_MAX_DISORDER = 4096;  // more disorder points: the serial loop
inline uint64_t al256(uint64_t b) { return (b + 255) & ~255ull; }
struct MergeWs {
    hgm::MEnt *e0, *e1, *e2;
    uint32_t* tile_live;
    uint64_t* tile_base;
    unsigned long long* lb_status;
    uint64_t* d_stage;
    unsigned long long* err;
    hgm::ExactHead* heads;
    uint64_t* dis_list;             // disorder points (EPOCH_MAX_DISORDER)
    unsigned long long* dis_count;  // [0] count, [1] an epoch's error word
    uint64_t* ep;                   // 4 * ntables: candidates, lo, hi, u
    uint64_t* ep_roff;              // an epoch's round offsets
    hg_merge_result* ep_res;
    uint32_t* rank;                 // the rank path: a dense rank per entry (+ RANK_PAD)
    uint32_t* win_idx;              // its winners' entry indices
    uint64_t* rank_steps;           // its winner count
    uint64_t bytes;
};
MergeWs merge_ws(void* d_ws, uint32_t ntables, uint64_t n) {
    using namespace hgm;
    const uint64_t ntiles = (n + TILE - 1) / TILE + 1;
    const uint64_t stage = hgk_merge_staging_bytes(ntables);
    char* base = static_cast<char*>(d_ws);
    char* p = base;
    MergeWs w;
    w.e0 = reinterpret_cast<MEnt*>(p);
    p += al256(n * sizeof(MEnt));
    w.e1 = reinterpret_cast<MEnt*>(p);
    p += al256(n * sizeof(MEnt));
    w.e2 = reinterpret_cast<MEnt*>(p);
    p += al256(n * sizeof(MEnt));
    w.tile_live = reinterpret_cast<uint32_t*>(p);
    p += al256(ntiles * 4);
    w.tile_base = reinterpret_cast<uint64_t*>(p);
    p += al256(ntiles * 8);
    w.lb_status = reinterpret_cast<unsigned long long*>(p);
    p += al256(2 * ntiles * 8);
    w.d_stage = reinterpret_cast<uint64_t*>(p);
    p += al256(stage);
    w.err = reinterpret_cast<unsigned long long*>(p);
    p += 256;
    w.heads = reinterpret_cast<ExactHead*>(p);
    p += al256((uint64_t)ntables * sizeof(ExactHead));
    w.dis_list = reinterpret_cast<uint64_t*>(p);
    p += al256(EPOCH_MAX_DISORDER * 8);
    w.dis_count = reinterpret_cast<unsigned long long*>(p);
    p += 256;
    w.ep = reinterpret_cast<uint64_t*>(p);
    p += al256(4 * (uint64_t)ntables * 8);
    w.ep_roff = reinterpret_cast<uint64_t*>(p);
    p += al256(stage);
    w.ep_res = reinterpret_cast<hg_merge_result*>(p);
    p += 256;
    w.rank = reinterpret_cast<uint32_t*>(p);
    p += al256((n + RANK_PAD) * 4);
    w.win_idx = reinterpret_cast<uint32_t*>(p);
    p += al256(n * 4 + 256);
    w.rank_steps = reinterpret_cast<uint64_t*>(p);
    p += 256;
    w.bytes = (uint64_t)(p - base);
    return w;
}

// Round structure of nr sorted runs with round-0 offsets r[0..nr]: the
// offsets of every later round follow in place (round r + 1 pairs up the runs
// of round r).  Returns the words written.
uint64_t round_offsets(uint64_t* r, uint64_t nr) {
    uint64_t words = nr + 1;
    while (nr > 1) {
        uint64_t* nxt = r + (nr + 1);
        const uint64_t m = (nr + 1) / 2;
        for (uint64_t i = 0; i <= m; ++i) nxt[i] = r[std::min(2 * i, nr)];
        words += m + 1;
        r = nxt;
        nr = m;
    }
    return words;
}

// The merge of nr >= 1 sorted runs of `in` (a.n entries; round offsets at
// roff on the device): log2(nr) rounds, the last emitting the pairs to
// fa.out / fa.result; one run: its live entries become pairs directly.  The
// first round reads `in` and writes b1; later rounds alternate b2, b1 (so
// `in` is never written unless it is b2).
int launch_rounds(const hgm::MergeArgs& a, const uint64_t* roff, uint64_t nr, hgm::MEnt* in,
                  hgm::MEnt* b1, hgm::MEnt* b2, const MergeWs& w, unsigned long long* err,
                  hgm::FinalArgs fa, hipStream_t stream, const uint64_t* h_roff = nullptr,
                  int* done = nullptr) {
    using namespace hgm;
    const uint64_t ntiles = (a.n + TILE - 1) / TILE;
    fa.st = w.lb_status;
    fa.ntiles = (uint32_t)ntiles;
    // 3..KW_MAX runs with their offsets on the host and HG_MERGE_KWAY=1: the
    // one-pass k-way merge (section 3b; not the default: slower, see there)
    if (h_roff && nr >= 3 && nr <= KW_MAX && hgk_knob("HG_MERGE_KWAY", 0) == 1) {
        KwArgs k{};
        k.K = (uint32_t)nr;
        uint64_t ns = 0;
        for (uint32_t i = 0; i <= KW_MAX; ++i) {
            const uint64_t o = h_roff[std::min<uint64_t>(i, nr)];
            k.roff[i] = o;
            k.soff[i] = (uint32_t)ns;
            if (i < nr) ns += (h_roff[i + 1] - o + KW_S - 1) / KW_S;
        }
        k.ns = (uint32_t)ns;
        k.ntiles = (uint32_t)((ns + KW_M - 1) / KW_M);
        fa.ntiles = k.ntiles;
        MEnt* samp = b1;
        uint64_t* split = reinterpret_cast<uint64_t*>(b2);
        hipLaunchKernelGGL(kw_sample_kernel, dim3((uint32_t)((ns + THREADS - 1) / THREADS)), dim3(THREADS), 0,
                           stream, k, (const MEnt*)in, samp, w.lb_status);
        hipLaunchKernelGGL(kw_split_kernel, dim3((uint32_t)((ns * KW_MAX + THREADS - 1) / THREADS)),
                           dim3(THREADS), 0, stream, a, k, (const MEnt*)in, (const MEnt*)samp, split,
                           (const unsigned long long*)err);
        hipLaunchKernelGGL(kw_merge_kernel, dim3(k.ntiles), dim3(KW_THREADS), 0, stream, a, k,
                           (const MEnt*)in, (const uint64_t*)split, err, fa);
        return HG_LAUNCH_STATUS();
    }
    if (nr >= 2) {
        bool first = true;  // the first round's split kernel zeroes the look-back statuses
        MEnt* cur = in;
        MEnt* nxt = b1;
        while (nr > 1) {
            LevelArgs l;
            l.roff = roff;
            l.nruns = (uint32_t)nr;
            l.uw = l.un = 0;
            // tile_base is free in the rounds: the round's splits
            const uint32_t gs = (uint32_t)(((ntiles + 1) * SPLIT_G + THREADS - 1) / THREADS);
            // the last round's split kernel also clears the encode sums that
            // round accumulates (when its grid covers them)
            const bool sums = nr == 2 && !fa.rec_out && fa.enc_sums &&
                              fa.enc_words <= (uint64_t)gs * THREADS;
            hipLaunchKernelGGL(merge_split_kernel, dim3(gs), dim3(THREADS), 0, stream, a, l,
                               (const MEnt*)cur, w.tile_base, ntiles, (const unsigned long long*)err,
                               first ? w.lb_status : (unsigned long long*)nullptr,
                               sums ? fa.enc_sums : (unsigned long long*)nullptr,
                               sums ? fa.enc_words : (uint64_t)0);
            first = false;
            if (nr == 2 && !sums) fa.enc_sums = nullptr;
            if (sums && done) *done |= HGK_MERGE_SUMS;
            if (nr == 2)  // the last round emits the pairs
                if (fa.rec_out) {  // compaction: the records themselves
                    hipLaunchKernelGGL(merge_level_kernel<2>, dim3((uint32_t)ntiles), dim3(THREADS), 0,
                                       stream, a, l, (const MEnt*)cur, nxt, (const uint64_t*)w.tile_base,
                                       err, fa);
                    if (done) *done |= HGK_MERGE_EMITTED;
                } else
                    hipLaunchKernelGGL(merge_level_kernel<1>, dim3((uint32_t)ntiles), dim3(THREADS), 0,
                                       stream, a, l, (const MEnt*)cur, nxt, (const uint64_t*)w.tile_base,
                                       err, fa);
            else
                hipLaunchKernelGGL(merge_level_kernel<0>, dim3((uint32_t)ntiles), dim3(THREADS), 0,
                                   stream, a, l, (const MEnt*)cur, nxt, (const uint64_t*)w.tile_base,
                                   err, fa);
            roff += nr + 1;
            nr = (nr + 1) / 2;
            cur = nxt;
            nxt = nxt == b1 ? b2 : b1;
        }
        return HG_LAUNCH_STATUS();
    }
    const MEnt* cur = in;
    hipLaunchKernelGGL(merge_count_kernel, dim3((uint32_t)ntiles), dim3(THREADS), 0, stream, a,
                       (const MEnt*)cur, w.tile_live);
    hipLaunchKernelGGL(merge_scan_kernel, dim3(1), dim3(1024), 0, stream, (const uint32_t*)w.tile_live,
                       (uint32_t)ntiles, w.tile_base, fa.result);
    hipLaunchKernelGGL(merge_emit_kernel, dim3((uint32_t)ntiles), dim3(THREADS), 0, stream, a,
                       (const MEnt*)cur, (const uint64_t*)w.tile_base, fa.out, fa.cap,
                       (const unsigned long long*)err);
    return HG_LAUNCH_STATUS();
}

int sync_copy(void* dst, const void* src, size_t n, hipMemcpyKind k, hipStream_t s) {
    if (!n) return HG_OK;
    if (hipMemcpyAsync(dst, src, n, k, s) != hipSuccess || hipStreamSynchronize(s) != hipSuccess)
        return HG_HIP_FAIL;
    return HG_OK;
}

// The rank path (section 7) over the entries in w.e0: dense ranks (tiles
// sorted in LDS, merge rounds over uniform runs, key-change flags scanned),
// then the reference loop in one wave from the heads `start` (host,
// table-local; nullptr: every table from its first record) with n0 records
// already emitted, the pairs to d_out[n0, cap).  ntables <= RANK_MAX_TABLES.
// Synchronous; the result goes to d_result and *h_result.
int rank_path(const hgm::MergeArgs& a, const MergeWs& w, const uint64_t* start, uint64_t n0,
              hg_pair* d_out, uint64_t cap, hg_merge_result* d_result, hg_merge_result* h_result,
              uint64_t* h, hipStream_t stream) {
    using namespace hgm;
    const uint32_t k = a.ntables;
    const uint64_t n = a.n;
    if (k > RANK_MAX_TABLES || n == 0) return HG_ERR_INTERNAL;
    const uint64_t ntiles = (n + TILE - 1) / TILE;
    unsigned long long* serr = w.dis_count + 1;  // the sort rounds' order word (sorted runs: stays ~0)
    if (hipMemsetAsync(serr, 0xFF, 8, stream) != hipSuccess) return HG_HIP_FAIL;
    hipLaunchKernelGGL(sort_tile_kernel, dim3((uint32_t)ntiles), dim3(THREADS), 0, stream, a,
                       (const MEnt*)w.e0, w.e1);
    MEnt* cur = w.e1;
    MEnt* nxt = w.e2;
    FinalArgs fa{};
    for (uint64_t uw = TILE; uw < n; uw *= 2) {
        LevelArgs l;
        l.roff = nullptr;
        l.nruns = (uint32_t)((n + uw - 1) / uw);
        l.uw = uw;
        l.un = n;
        const uint32_t gs = (uint32_t)(((ntiles + 1) * SPLIT_G + THREADS - 1) / THREADS);
        hipLaunchKernelGGL(merge_split_kernel, dim3(gs), dim3(THREADS), 0, stream, a, l,
                           (const MEnt*)cur, w.tile_base, ntiles, (const unsigned long long*)serr,
                           (unsigned long long*)nullptr);
        hipLaunchKernelGGL(merge_level_kernel<0>, dim3((uint32_t)ntiles), dim3(THREADS), 0, stream,
                           a, l, (const MEnt*)cur, nxt, (const uint64_t*)w.tile_base, serr, fa);
        std::swap(cur, nxt);
    }
    hipLaunchKernelGGL(rank_count_kernel, dim3((uint32_t)ntiles), dim3(THREADS), 0, stream, a,
                       (const MEnt*)cur, w.tile_live);
    hipLaunchKernelGGL(merge_scan_kernel, dim3(1), dim3(1024), 0, stream, (const uint32_t*)w.tile_live,
                       (uint32_t)ntiles, w.tile_base, w.ep_res);
    // ranks < n; HG_RANK_NOPACK: plain ranks at any size (tests the > 2^26 form)
    const uint32_t pack = n < (1ull << 26) && !hgk_knob("HG_RANK_NOPACK", 0) ? 1u : 0u;
    hipLaunchKernelGGL(rank_scatter_kernel, dim3((uint32_t)ntiles), dim3(THREADS), 0, stream, a,
                       (const MEnt*)cur, (const uint64_t*)w.tile_base, w.rank, pack);
    int rc = HG_LAUNCH_STATUS();
    if (rc != HG_OK) return rc;
    uint64_t done = 0;
    for (uint32_t t = 0; t < k; ++t) {
        h[t] = start ? start[t] : 0;
        done += h[t];
    }
    if (hipMemcpyAsync(w.ep, h, (uint64_t)k * 8, hipMemcpyHostToDevice, stream) != hipSuccess)
        return HG_HIP_FAIL;
    uint32_t H = 1024;  // ranks per ring half: both halves of every table in RANK_LDS
    while (H > 128 && (uint64_t)k * 2 * H * 4 > RANK_LDS) H >>= 1;
    RankArgs ra;
    ra.rank = w.rank;
    ra.run_off = a.run_off;
    ra.ntables = k;
    ra.H = H;
    ra.start = w.ep;
    ra.win_idx = w.win_idx;
    ra.steps = w.rank_steps;
    ra.pack = pack;
    hipLaunchKernelGGL(rank_merge_kernel, dim3(1), dim3(64), (size_t)k * 2 * H * 4, stream, ra);
    const uint64_t left = n > done ? n - done : 1;
    hipLaunchKernelGGL(rank_emit_kernel, dim3((uint32_t)((left + THREADS - 1) / THREADS)), dim3(THREADS),
                       0, stream, a, (const uint32_t*)w.win_idx, (const uint64_t*)w.rank_steps, d_out,
                       cap, n0, d_result);
    if ((rc = HG_LAUNCH_STATUS()) != HG_OK) return rc;
    unsigned long long e = 0;
    if ((rc = sync_copy(&e, serr, 8, hipMemcpyDeviceToHost, stream)) != HG_OK ||
        (rc = sync_copy(h_result, d_result, sizeof(hg_merge_result), hipMemcpyDeviceToHost, stream)) !=
            HG_OK)
        return rc;
    return e == ~0ull ? HG_OK : HG_ERR_INTERNAL;
}
}  // namespace

extern "C" uint64_t hgk_merge_workspace_bytes(uint32_t ntables, uint64_t n) {
    return merge_ws(nullptr, ntables, n).bytes;
}

// Host arrays: table_off[ntables], spans[ntables] (device pointers),
// counts[ntables].  `staging` is pinned host memory of at least
// hgk_merge_staging_bytes(ntables) bytes (copied to the device on `stream`):
// [table_off | span ptrs | run offsets of the tables | of every round].
extern "C" uint64_t hgk_merge_staging_bytes(uint32_t ntables) {
    return (12 * (uint64_t)ntables + 80) * 8;
}

// Compaction: the merge entries built before the host has the record counts
// (hg_runtime.hip compact_core).  kent_runoff_kernel turns the decode results
// into the tables' run offsets on the device (a table whose decode failed
// counts 0: the call then fails on the host and the entries are unused) and
// resets the order-check word; decode_entries_multi then fills the entries
// at the start of the merge workspace (w.e0, laid out independently of n).
__global__ void kent_runoff_kernel(const hg_decode_result* res, uint32_t ntables, uint64_t* run_off,
                                   unsigned long long* err) {
    if (threadIdx.x != 0) return;
    uint64_t o = 0;
    for (uint32_t t = 0; t < ntables; ++t) {
        run_off[t] = o;
        o += res[t].kind == HG_OK ? res[t].n_records : 0;
    }
    run_off[ntables] = o;
    *err = ~0ull;
}

extern "C" int hgk_merge_prebuild(const uint64_t* kp, uint32_t ntables,
                                  const hg_decode_result* d_results, uint64_t* d_run_off,
                                  unsigned long long* d_err, void* d_ws, hipStream_t stream) {
    using namespace hgm;
    if (!kp || !ntables) return HG_ERR_INVALID_ARG;
    hipLaunchKernelGGL(kent_runoff_kernel, dim3(1), dim3(64), 0, stream, d_results, ntables, d_run_off,
                       d_err);
    const int rc = HG_LAUNCH_STATUS();
    if (rc != HG_OK) return rc;
    return hgk_decode_entries_launch(reinterpret_cast<const void*>(kp[3 * (uint64_t)ntables]), ntables,
                                     (uint32_t)kp[3 * (uint64_t)ntables + 1], d_run_off,
                                     merge_ws(d_ws, ntables, 0).e0, d_err, stream);
}

// defer: on input that is not strictly increasing, leave the result as
// HG_ERR_UNSORTED (n_out 0, no pairs) for hgk_merge_epochs instead of running
// the serial reference loop on the device.
// kp (nullable): [3 * ntables] device pointers -- per table the decode
// workspace's span scratch, piece records, piece tags -- and kp_tag, the
// decode's compaction-mode tag: merge entries take the key prefixes the
// decode pre-pass left there (merge_prep_kernel, make_ent).
extern "C" int hgk_merge_launch(const uint8_t* d_arena, uint64_t arena_len, uint32_t ntables,
                                const uint64_t* table_off, const hg_span* const* spans,
                                const uint64_t* counts, hg_pair* d_out, uint64_t cap,
                                hg_merge_result* d_result, void* d_ws, void* staging,
                                hipStream_t stream, int defer, const uint64_t* kp,
                                uint32_t kp_tag, const unsigned long long* d_err_pre,
                                const hgk_merge_records* rec, int* done) {
    using namespace hgm;
    if (done) *done = 0;
    if (ntables == 0 || ntables > MAX_TABLES) return HG_ERR_INVALID_ARG;
    uint64_t n = 0;
    for (uint32_t t = 0; t < ntables; ++t) n += counts[t];
    if (n >= MAX_ENTRIES) return HG_ERR_TOO_LARGE;  // entries carry a 31-bit global index
    uint64_t* h = static_cast<uint64_t*>(staging);
    uint64_t* h_toff = h;
    uint64_t* h_sp = h + ntables;
    uint64_t* r = h + 2 * (uint64_t)ntables;  // run offsets of the tables (entry layout)
    for (uint32_t t = 0; t < ntables; ++t) {
        h_toff[t] = table_off[t];
        h_sp[t] = reinterpret_cast<uint64_t>(spans[t]);
    }
    r[0] = 0;
    for (uint32_t t = 0; t < ntables; ++t) r[t + 1] = r[t] + counts[t];
    // Round 0 merges the NON-EMPTY runs only: an empty run as the last round's
    // B side would send that round down the odd-run copy path, which emits no
    // pairs (and publishes no look-back status).
    uint64_t* r0 = r + ntables + 1;
    uint64_t nruns0 = 0;
    r0[0] = 0;
    for (uint32_t t = 0; t < ntables; ++t)
        if (counts[t]) r0[++nruns0] = r[t + 1];
    const uint64_t rwords = 3 * (uint64_t)ntables + 1 + round_offsets(r0, nruns0);
    // kp: 3 groups of per-table pointers (then the decode's staging and grid)
    const uint64_t stage_words = rwords + (kp ? 3 * (uint64_t)ntables : 0);
    if (stage_words * 8 > hgk_merge_staging_bytes(ntables)) return HG_ERR_INTERNAL;
    const uint32_t kent_grid = kp ? (uint32_t)kp[3 * (uint64_t)ntables + 1] : 0u;
    if (kp)
        for (uint64_t i = 0; i < 3 * (uint64_t)ntables; ++i) h[rwords + i] = kp[i];
    const MergeWs w = merge_ws(d_ws, ntables, n);
    // the error word (~0: no order violation yet) follows the staging in the
    // workspace: one copy sets both (a memset launch fewer)
    const uint64_t err_word = (uint64_t)(reinterpret_cast<uint64_t*>(w.err) - w.d_stage);
    h[err_word] = ~0ull;
    if (hipMemcpyAsync(w.d_stage, h, (err_word + 1) * 8, hipMemcpyHostToDevice, stream) != hipSuccess)
        return HG_HIP_FAIL;
    MergeArgs a;
    a.arena = d_arena;
    a.arena_len = arena_len;
    a.table_off = w.d_stage;
    a.spans = reinterpret_cast<const hg_span* const*>(w.d_stage + ntables);
    a.run_off = w.d_stage + 2 * (uint64_t)ntables;
    a.ntables = ntables;
    a.n = n;
    a.kp_scratch = kp ? w.d_stage + rwords : nullptr;
    a.kp_spiece = kp ? w.d_stage + rwords + ntables : nullptr;
    a.kp_ptag = kp ? w.d_stage + rwords + 2 * (uint64_t)ntables : nullptr;
    a.kp_tag = kp ? kp_tag : 0;
    if (n == 0) {
        // every table empty: the reference's unwrap on None (manager.rs:213)
        hg_merge_result res{0, HG_ERR_EMPTY_MERGE, 0, 0};
        return hipMemcpyAsync(d_result, &res, sizeof res, hipMemcpyHostToDevice, stream) == hipSuccess
                   ? HG_OK
                   : HG_HIP_FAIL;
    }
    // compaction mode: the entries come from the decode's workspace, one
    // workgroup per pre-pass batch (hg_decode.hip, decode_entries_multi;
    // kp[3 ntables] = the batched decode's device staging, kp[3 ntables + 1]
    // its pre-pass grid) instead of merge_prep_kernel's per-record chains
    const bool kent_on = hgk_knob("HG_MERGE_KENT", 1) != 0;  // 0: merge_prep_kernel (A/B runs)
    // the entries were built into w.e0 by hgk_merge_prebuild while the host
    // waited for the counts: its order-check word is the one the rounds and
    // the flag read (w.err, set by the staging copy, stays unused)
    unsigned long long* const err =
        d_err_pre ? const_cast<unsigned long long*>(d_err_pre) : w.err;
    if (d_err_pre) {
        // entries in place (hgk_merge_prebuild)
    } else if (kent_grid && kent_on) {
        const int rk = hgk_decode_entries_launch(
            reinterpret_cast<const void*>(kp[3 * (uint64_t)ntables]), ntables, kent_grid, a.run_off,
            w.e0, w.err, stream);
        if (rk != HG_OK) return rk;
    } else {
        const uint32_t g1 = (uint32_t)((n + THREADS * PREP_U - 1) / (THREADS * PREP_U));
        hipLaunchKernelGGL(merge_prep_kernel, dim3(g1), dim3(THREADS), 0, stream, a, w.e0, w.err);
    }
    FinalArgs fa{};
    fa.out = d_out;
    fa.cap = cap;
    fa.result = d_result;
    fa.test_expire = (uint32_t)hgk_knob("HG_MERGE_TEST_LB_EXPIRE", -1);  // test hook (unset: ~0u)
    if (rec && rec->out) {  // records mode: the last round writes the records (no pairs)
        fa.rec_out = rec->out;
        fa.rec_cap = rec->cap;
        fa.rec_off = rec->rec_off;
        fa.enc_result = rec->enc_result;
    } else if (rec && rec->enc_sums && defer) {
        // pairs mode: the last round also sums the encode's tiles (defer only:
        // otherwise the exact loop may rewrite the pairs after it)
        fa.enc_sums = reinterpret_cast<unsigned long long*>(rec->enc_sums);
        fa.enc_nt = rec->enc_nt;
        fa.enc_words = rec->enc_words;
        fa.enc_tile_log2 = rec->enc_tile_log2;
        fa.enc_group_log2 = rec->enc_group_log2;
    }
    // the rounds ping-pong between e1 and e2, so e0 keeps the entries for the
    // exact loop / the epochs (the first round reads e0)
    int dl = 0;
    int rc = launch_rounds(a, a.run_off + ntables + 1, nruns0, w.e0, w.e1, w.e2, w, err, fa,
                           stream, r0, &dl);
    if (done) *done |= dl;
    if (rc != HG_OK) return rc;
    if (defer) {
        // (not the group sums the last round accumulated)
        uint64_t* const zero = rec && !(dl & HGK_MERGE_SUMS) ? rec->zero : nullptr;
        const uint64_t zero_words = zero ? rec->zero_words : 0;
        hipLaunchKernelGGL(merge_flag_kernel, dim3(1), dim3(THREADS), 0, stream,
                           (const unsigned long long*)err, d_result, zero, zero_words);
        if (zero && done) *done |= HGK_MERGE_ZEROED;
    } else
        hipLaunchKernelGGL(merge_exact_kernel, dim3(1), dim3(64), 0, stream, a, (const MEnt*)w.e0,
                           (const unsigned long long*)err, w.heads, d_out, cap, d_result,
                           (const uint64_t*)nullptr, (uint64_t)0);
    return HG_LAUNCH_STATUS();
}

// After hgk_merge_launch(defer) reported HG_ERR_UNSORTED (same arguments and
// workspace, stream synchronized): the reference loop by epochs (see
// merge_bound_kernel): disorder points listed on the device, then per epoch
// the bound of M and every table's cut (one small kernel, one sync), the
// sub-runs gathered (device copies) and merged by the parallel rounds, the
// pairs appended.  More than EPOCH_MAX_DISORDER disorder points: the serial
// loop.  Synchronous; the result goes to d_result and *h_result.
extern "C" int hgk_merge_epochs(const uint8_t* d_arena, uint64_t arena_len, uint32_t ntables,
                                const uint64_t* table_off, const hg_span* const* spans,
                                const uint64_t* counts, hg_pair* d_out, uint64_t cap,
                                hg_merge_result* d_result, hg_merge_result* h_result, void* d_ws,
                                void* staging, hipStream_t stream) {
    using namespace hgm;
    (void)table_off;
    (void)spans;
    uint64_t n = 0;
    std::vector<uint64_t> ro(ntables + 1, 0);
    for (uint32_t t = 0; t < ntables; ++t) ro[t + 1] = ro[t] + counts[t];
    n = ro[ntables];
    const MergeWs w = merge_ws(d_ws, ntables, n);
    MergeArgs a;  // as hgk_merge_launch staged it (its staging copy is still in place)
    a.arena = d_arena;
    a.arena_len = arena_len;
    a.table_off = w.d_stage;
    a.spans = reinterpret_cast<const hg_span* const*>(w.d_stage + ntables);
    a.run_off = w.d_stage + 2 * (uint64_t)ntables;
    a.ntables = ntables;
    a.n = n;
    a.kp_scratch = a.kp_spiece = a.kp_ptag = nullptr;  // the entries exist (e0)
    a.kp_tag = 0;
    uint64_t* h = static_cast<uint64_t*>(staging);  // free: the stream is synchronized
    // 1. disorder points
    if (hipMemsetAsync(w.dis_count, 0, 8, stream) != hipSuccess) return HG_HIP_FAIL;
    hipLaunchKernelGGL(merge_disorder_kernel, dim3((uint32_t)((n + THREADS - 1) / THREADS)),
                       dim3(THREADS), 0, stream, a, (const MEnt*)w.e0, w.dis_list, w.dis_count,
                       EPOCH_MAX_DISORDER);
    int rc = HG_LAUNCH_STATUS();
    if (rc == HG_OK) rc = sync_copy(h, w.dis_count, 8, hipMemcpyDeviceToHost, stream);
    if (rc != HG_OK) return rc;
    const uint64_t D = h[0];
    auto finish = [&](hg_merge_result res) -> int {
        *h_result = res;
        return sync_copy(d_result, h_result, sizeof res, hipMemcpyHostToDevice, stream);
    };
    // The reference loop itself from heads hd (host, table-local; nullptr:
    // the tables' first records) with n0 records emitted: the rank path (one
    // wave over dense ranks) for up to RANK_MAX_TABLES tables, else the
    // round-2 loop over entries.  Knob HG_MERGE_SERIAL 2 forces the latter (A/B).
    const int64_t serial_knob = hgk_knob("HG_MERGE_SERIAL", 0);
    const bool exact_loop = serial_knob == 2;
    auto serial = [&](const uint64_t* hd0, uint64_t n0) -> int {
        if (ntables <= RANK_MAX_TABLES && !exact_loop)
            return rank_path(a, w, hd0, n0, d_out, cap, d_result, h_result, h, stream);
        const uint64_t* dstart = nullptr;
        if (hd0) {
            for (uint32_t t = 0; t < ntables; ++t) h[t] = hd0[t];
            if (hipMemcpyAsync(w.ep, h, (uint64_t)ntables * 8, hipMemcpyHostToDevice, stream) !=
                hipSuccess)
                return HG_HIP_FAIL;
            dstart = w.ep;
        }
        // the epochs run only after an order violation: the loop runs unconditionally
        hipLaunchKernelGGL(merge_exact_kernel, dim3(1), dim3(64), 0, stream, a, (const MEnt*)w.e0,
                           (const unsigned long long*)nullptr, w.heads, d_out, cap, d_result, dstart,
                           n0);
        int r2 = HG_LAUNCH_STATUS();
        if (r2 != HG_OK) return r2;
        return sync_copy(h_result, d_result, sizeof(hg_merge_result), hipMemcpyDeviceToHost, stream);
    };
    // D == 0: the tables are strictly increasing after all -- the error word
    // came from a look-back wait over its budget (contention), not from the
    // order check -- and the one epoch below is the whole merge again, by
    // the parallel rounds (result table 3, index = the redos).
    // an epoch costs a few launches and host round trips (~0.1-0.2 ms): many
    // disorder points -> the serial loop
    if (D > EPOCH_MAX_DISORDER || D > n / 128 + 1 || serial_knob) return serial(nullptr, 0);
    // test hook: epoch number HG_MERGE_TEST_EPOCH_FAIL reports a failure after
    // it ran (as a look-back wait over its budget would), so the hand-over to
    // the serial loop from the epochs' heads is exercised
    const long fail_at = (long)hgk_knob("HG_MERGE_TEST_EPOCH_FAIL", -1);
    std::vector<uint64_t> dl(D);
    if ((rc = sync_copy(dl.data(), w.dis_list, D * 8, hipMemcpyDeviceToHost, stream)) != HG_OK)
        return rc;
    std::sort(dl.begin(), dl.end());
    std::vector<std::vector<uint64_t>> dis(ntables);  // table-local disorder points, ascending
    for (uint64_t g : dl) {
        const uint32_t t = (uint32_t)(std::upper_bound(ro.begin(), ro.end(), g) - ro.begin()) - 1;
        dis[t].push_back(g - ro[t]);
    }
    // 2. epochs
    std::vector<uint64_t> hd(ntables, 0), f(ntables), u(ntables);
    uint64_t N = 0, epochs = 0;
    uint64_t* dcand = w.ep;
    uint64_t* dlo = w.ep + ntables;
    uint64_t* dhi = w.ep + 2 * (uint64_t)ntables;
    uint64_t* du = w.ep + 3 * (uint64_t)ntables;
    unsigned long long* ep_err = w.dis_count + 1;
    // An epoch's sub-runs are strictly increasing, so its error word can only
    // come from a look-back wait over the budget: the epoch is merged again
    // by the parallel rounds (up to EPOCH_REDOS times in all) before the
    // serial loop takes over -- a serial loop over millions of records is
    // thousands of times slower than a redo.
    constexpr uint32_t EPOCH_REDOS = 4;
    uint32_t redos = 0;
    for (;;) {
        uint32_t nc = 0;
        bool left = false;
        for (uint32_t t = 0; t < ntables; ++t) {
            const uint64_t cnt = counts[t];
            auto it = std::upper_bound(dis[t].begin(), dis[t].end(), hd[t]);
            f[t] = it == dis[t].end() ? cnt : *it;
            left |= hd[t] < cnt;
            if (f[t] < cnt) h[nc++] = ro[t] + f[t] - 1;  // candidates for M
        }
        if (!left) break;
        for (uint32_t t = 0; t < ntables; ++t) {
            h[ntables + t] = hd[t];
            h[2 * (uint64_t)ntables + t] = f[t];
        }
        if (hipMemcpyAsync(w.ep, h, 3 * (uint64_t)ntables * 8, hipMemcpyHostToDevice, stream) !=
            hipSuccess)
            return HG_HIP_FAIL;
        hipLaunchKernelGGL(merge_bound_kernel, dim3(1), dim3(THREADS), 0, stream, a,
                           (const MEnt*)w.e0, (const uint64_t*)dcand, nc, (const uint64_t*)dlo,
                           (const uint64_t*)dhi, du);
        if ((rc = HG_LAUNCH_STATUS()) != HG_OK) return rc;
        if ((rc = sync_copy(u.data(), du, (uint64_t)ntables * 8, hipMemcpyDeviceToHost, stream)) !=
            HG_OK)
            return rc;
        // the epoch's sub-runs [hd, u), gathered in priority order
        uint64_t ne = 0, nre = 0;
        h[0] = 0;
        for (uint32_t t = 0; t < ntables; ++t) {
            const uint64_t len = u[t] - hd[t];
            if (u[t] < hd[t] || u[t] > f[t]) return serial(hd.data(), N);  // (never on a sound bound)
            if (!len) continue;
            if (hipMemcpyAsync(w.e1 + ne, w.e0 + ro[t] + hd[t], len * sizeof(MEnt),
                               hipMemcpyDeviceToDevice, stream) != hipSuccess)
                return HG_HIP_FAIL;
            ne += len;
            h[++nre] = ne;
        }
        if (!ne) return serial(hd.data(), N);  // every epoch consumes a disorder point
        const uint64_t words = round_offsets(h, nre);
        if (words * 8 > hgk_merge_staging_bytes(ntables)) return HG_ERR_INTERNAL;
        if (hipMemcpyAsync(w.ep_roff, h, words * 8, hipMemcpyHostToDevice, stream) != hipSuccess ||
            hipMemsetAsync(ep_err, 0xFF, 8, stream) != hipSuccess)
            return HG_HIP_FAIL;
        MergeArgs ae = a;
        ae.n = ne;
        FinalArgs fa{};
        fa.out = d_out + std::min(N, cap);
        fa.cap = cap > N ? cap - N : 0;
        fa.result = w.ep_res;
        if ((rc = launch_rounds(ae, w.ep_roff, nre, w.e1, w.e2, w.e1, w, ep_err, fa, stream)) !=
            HG_OK)
            return rc;
        struct {
            hg_merge_result r;
            unsigned long long e;
        } er;
        if ((rc = sync_copy(&er.r, w.ep_res, sizeof er.r, hipMemcpyDeviceToHost, stream)) != HG_OK ||
            (rc = sync_copy(&er.e, ep_err, 8, hipMemcpyDeviceToHost, stream)) != HG_OK)
            return rc;
        // a look-back wait over its budget (a stalled or shared GPU): the
        // epoch again; any other failure of the epoch (or too many redos):
        // the serial loop takes over from its heads, overwriting whatever
        // pairs the epoch left past N
        if ((long)epochs == fail_at) return serial(hd.data(), N);
        if (er.e == 0 && er.r.kind == HG_OK && redos < EPOCH_REDOS) {
            ++redos;
            continue;  // hd unchanged: the same cuts, merged again
        }
        if (er.e != ~0ull || er.r.kind != HG_OK) return serial(hd.data(), N);
        N += er.r.n_out;
        for (uint32_t t = 0; t < ntables; ++t) hd[t] = u[t];
        ++epochs;
    }
    // table = 2: the epochs produced the output (index = their number); D == 0
    // (a look-back over its budget, sorted input): the one epoch was a plain
    // redo of the parallel merge (table 3, index = the redos, >= 1)
    return finish(hg_merge_result{N, HG_OK, D ? 2u : 3u, D ? epochs : (uint64_t)redos + 1});
}
