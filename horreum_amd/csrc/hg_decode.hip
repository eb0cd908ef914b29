// hg_decode.hip — device-resident SSTable decode (record boundary discovery
// + span emission) for gfx950.
//
// Replaces the serial cursor walk of InternalPair::deserialize_from_bytes
// (reference src/format.rs:50-59) and deserialize_inner (:63-77):
//     off[i+1] = off[i] + 16 + klen[i] + vlen[i]
// is one long dependency chain with no sync points on disk
// (src/sstable/storage.rs:31-32).  Here it becomes a single pass over HBM.
//
// Work unit = a BATCH of PIECES (16..64 x 16 KiB), one 256-thread workgroup, taken
// by one atomic ticket (so batch b-1 is always already running: the look-back
// cannot deadlock; one returning atomic per >= 256 KiB keeps the ticket far from
// its ~88/us limit).  Per batch:
//  1. Entry guess for piece 0: the predecessor batch's published exit if it is
//     out, else a record whose 16-byte header repeats 3 lengths ahead, else
//     the general engine's guess (below).
//  2. Pieces are staged in LDS one at a time (the next piece's 16-byte loads
//     are in flight in registers meanwhile) and walked from the exact exit of
//     the previous piece — speculation happens once per batch:
//     - stride run: if the header at X repeats at X+R, X+2R ... to the piece
//       end (one compare per lane), the records are that progression; kept as
//       a 32-byte summary and emitted arithmetically later;
//     - general engine otherwise: bit-parallel header filter over zero-byte
//       masks (a genuine length field has `hz` zero high bytes), exact bound
//       check and one look-ahead step give "strong" candidates; a candidate
//       is "backed" if another candidate's next lands on it (true records are
//       backed by their predecessor; shifted reads of a header are not).  Each
//       lane owns 64 bytes, guesses its first backed candidate, walks <= 4
//       records, and a relaxation (entry := left neighbour's exit, re-walk on
//       disagreement, seeded by a block max-scan over chain lanes) reaches the
//       exact fixed point; spans go to a scratch area until the batch's record
//       base is known.  Pathological pieces use an exact serial walk.
//  3. Publish AGG(count, guessed entry, exit); decoupled look-back (one wave,
//     63 predecessors per step): the nearest INCL plus the AGGs after it give
//     the exact entry X_b and record base G_b, provided every AGG's guessed
//     entry equals its predecessor's exit (one ballot); a mismatch waits for
//     that batch's self-corrected INCL.
//  4. Guess right: emit stride pieces arithmetically and copy scratch spans to
//     spans[G_b + ...], publish INCL.  Guess wrong or a format error: redo the
//     batch exactly from X_b (pieces re-read), emitting directly.
#include <stdlib.h>
#include <string.h>

#include <algorithm>

#include "hg_device.hpp"
#include "hg_knobs.hpp"

namespace hgk {

constexpr uint32_t PIECE = 16384;                 // bytes staged in LDS at a time
constexpr uint32_t THREADS = 256;                 // one 64-byte segment per lane
constexpr uint32_t NW = THREADS / 64;
constexpr uint32_t SEG = PIECE / THREADS;         // 64
constexpr uint32_t NGRAN = PIECE / 16;            // 1024 granules of 16 B
constexpr uint32_t GPT = NGRAN / THREADS;         // 4 granules per thread
// Pieces per batch (ticket / look-back status) are chosen per launch: enough
// that the batches fill the resident grid in about one round (each batch pays
// one look-back and emission tail, during which its workgroup has no loads in
// flight), between BATCH_MIN and BATCH (the LDS arrays' size).
constexpr uint32_t BATCH = 64;
// Floor 16: with 4-piece batches a 64 MiB table has 1024 batches whose
// speculative passes all end together, and each look-back then walks ~16
// windows to the nearest INCL (cfg 4 measured 8.2 ms vs 4.7 ms at 16).
#ifndef HG_BATCH_MIN
#define HG_BATCH_MIN 16
#endif
constexpr uint32_t BATCH_MIN = HG_BATCH_MIN;
constexpr uint32_t MAX_REC_PIECE = PIECE / 16;    // records per piece (>= 16 B each)
constexpr uint32_t WALK_LOG = PIECE / 16;         // serial-walk batch
constexpr uint32_t MAX_ROUNDS = 24;
constexpr uint32_t CAND_CAP = 16;                 // strong candidates examined per lane
#ifndef HG_SHORT_WALK
#define HG_SHORT_WALK 16
#endif
// serial pre-walk budget (24 -> 64: medium records 0.76 -> 0.69 ms in round 1;
// with the lean engine 64 -> 16: medium 0.465 -> 0.39 ms, the parallel engine
// beats one thread walking 48 records)
constexpr uint32_t SHORT_WALK = HG_SHORT_WALK;
constexpr uint32_t NONE_REL = 0x3FFFFFu;          // "no record starts here"
#ifndef HG_FAR_CAND
#define HG_FAR_CAND 8192ull  // candidate records this long are guesses only as a fallback
#endif
#ifndef HG_EMPTY_SPEC
#define HG_EMPTY_SPEC 1  // a piece without a guess is speculated empty (records > a piece)
#endif
#ifndef HG_LEADIN
#define HG_LEADIN 1  // general batches guess their entry from a walked lead-in piece
#endif
constexpr uint32_t NO_GUESS = 0xFFFFFFFFu;
#ifndef HG_SPLICE
#define HG_SPLICE 1  // 0: a pre-pass batch entered off its predecessor's exit is decoded again (A/B)
#endif
#ifndef HG_LEAN
#define HG_LEAN 1  // lean lane guesses for pieces entered at a known position (0: candidate
                   // evaluation + backing everywhere; 2: lean entry guesses too)
#endif

enum : uint32_t { ST_NONE = 0, ST_AGG = 1, ST_INCL = 2, ST_ERR = 3 };
enum : uint32_t { PK_EMPTY = 0, PK_STRIDE = 1, PK_SCRATCH = 2 };

struct DecodeArgs {
    const uint8_t* sst;          // first byte of the decoded range
    uint64_t len;                // bytes of the table from sst (records must fit in them)
    uint64_t rlen;               // bytes present at sst (>= min(len, stop + 16); == len for a whole table)
    uint64_t stop;               // records START in [entry, stop) (== len for a whole table)
    uint64_t entry;              // exact start of the first record (0 for a whole table)
    uint64_t obase;              // added to every span offset written to `spans`
    uint32_t range;              // a range decode: the result's err_offset on success = exit
    hg_span* spans;
    uint64_t cap;
    hg_decode_result* result;
    unsigned long long* status;  // 2 words per batch, zeroed before launch
    uint32_t* ticket;            // zeroed before launch
    hg_span* scratch;            // MAX_REC_PIECE spans per piece (speculative general pieces)
    uint32_t nbatches;
    uint32_t npieces;
    uint32_t hz;                 // zero high bytes required in klen/vlen
    uint32_t bp;                 // pieces per batch (BATCH_MIN..BATCH)
    uint32_t* diag;              // DIAG builds only: DIAG_WORDS per batch
    uint32_t* sdiag;             // diagnostics: LW_PROF words per pre-pass batch (or null)
    // Stride pre-pass results (decode_spec_kernel): batches of SPEC_BP
    // pieces [0, first_bad) are resolved; decode_kernel writes their spans.
    struct SpecBatch* sbatch;
    const struct SpecPiece* spiece;
    struct SpecPiece* spiece_rw;     // the same records (splice_repair rewrites its batch's)
    // compaction mode (kpre_tag != 0): stride pieces of the pre-pass leave the
    // key prefix of each record (key_prefix_be) in their unused span-scratch
    // slot and set their piece tag (piece_tags) to kpre_tag; the general
    // engine clears the tags of the pieces whose scratch it takes (hg_merge.hip's
    // entry builder reads a prefix only under a current tag, else the key)
    uint32_t kpre_tag;
    struct DecodeCtl* ctl;
    unsigned long long* gsum;    // records per group of SPEC_GROUP pre-pass batches
    unsigned long long* link;    // per adjacent pre-pass batch pair: arrivals | exit - x0
    uint32_t nspec;              // stride pre-pass batches
    uint32_t sbp;                // pieces per pre-pass batch (SPEC_BP_MIN..SPEC_BP)
    uint32_t q;                  // pre-pass batches per general batch (bp / sbp)
    uint32_t hop_wide;           // hop batches with at most this many piece-0 run ends walk
                                 // wide segments (HOP_WIDE_CAND, or 0: see hop_wide_cand)
    // the NEXT call's control region (hgk_decode_launch_ctl; null otherwise):
    // decode_spec_kernel zeroes its first zero_next_n16 x 16 bytes
    uint4* zero_next;
    uint32_t zero_next_n16;
};

// The piece tags (decode_layout: right after the piece records).
__device__ __forceinline__ uint32_t* piece_tags(const DecodeArgs& a);

// Bytes of the piece at `base` where records may start: up to `stop` (the
// piece's bytes up to `len` are still staged and readable).
__device__ __forceinline__ uint32_t piece_clen(const DecodeArgs& a, uint64_t base) {
    const uint64_t r = a.stop - base;
    return r < PIECE ? (uint32_t)r : PIECE;
}

// ---- stride pre-pass records --------------------------------------------------------
constexpr uint32_t SPEC_BP = 64;      // most pieces per pre-pass batch (LDS halo array)
constexpr uint32_t SPEC_BP_MIN = 4;
struct SpecBatch {                // one per pre-pass batch
    uint64_t x0;                  // guessed entry (absolute)
    uint64_t exit;                // first record start at or after the batch end
    uint32_t count;               // records starting in the batch
    uint32_t ok;                  // every piece verified as a stride run from x0
    uint64_t pad;
};

// Spans are written by decode_kernel, after the pre-pass, never by the
// pre-pass itself: span stores that share HBM with the table stream cost
// more than a store pass of their own.  Measured on cfg 2 (same box, A/B):
// spans written while the pieces stream (round 4, HG_SPEC_EMIT) 0.213 ->
// 0.274 ms; each pre-pass workgroup writing its batch's spans once its own
// stream is done, the others still streaming (round 5, "tail emission", all
// of a lattice table's spans then known from x0 and R) 0.203 -> 0.255 ms,
// nontemporal stores 0.254 ms (profiles/r5_ab_tail_emit.log); a first form
// of the latter that handed out span tickets from one counter 0.59 ms.
// Control words of a decode call (zero at launch, with the statuses: cleared
// by the previous call's pre-pass or by a memset, launch_decode).
struct DecodeCtl {
    uint32_t ticket;              // decode_kernel batch tickets
    uint32_t bad_rev;             // max over unresolved pre-pass batches b of nspec - b
    uint32_t progress;            // general batches published (INCL / ERR): the look-back's
                                  // waits restart their budget whenever it moves
    uint32_t repairs;             // pre-pass batches spliced onto their predecessor's exit
};
// (the group sums follow it: 8-byte atomics, which fault when misaligned)
static_assert(sizeof(DecodeCtl) % 8 == 0, "DecodeCtl keeps the group sums 8-byte aligned");
constexpr uint32_t SPEC_GROUP = 64;  // pre-pass batches per group sum
__device__ __forceinline__ uint32_t first_bad(const DecodeCtl* c, uint32_t nspec) {
    return nspec - c->bad_rev;       // bad_rev 0 (nothing bad) -> nspec
}
static_assert(PIECE_BYTES == 16384 && PIECE_RECS == 1024, "piece geometry (hg_device.hpp)");
__device__ __forceinline__ uint32_t* piece_tags(const DecodeArgs& a) {
    return reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(a.spiece_rw) +
                                       (((uint64_t)a.npieces * sizeof(SpecPiece) + 255) & ~255ull));
}
// SpecBatch.pad (diagnostics, tools/spec_diag.py): how the pre-pass batch went
enum : uint32_t { SB_STRIDE = 1, SB_STRIDE_BROKE = 2, SB_HOP_SMALL = 3, SB_HOP_DEAD = 4, SB_HOP = 5,
                  SB_LW = 6, SB_LW_DEAD = 7 };

// Diagnostic record per batch (tools/decode_diag.py).
constexpr uint32_t DIAG_WORDS = 24;
constexpr uint32_t NPROF = 8;  // DIAG phase cycle counters, words 16..23
enum : uint32_t {
    D_T_SPEC = 0, D_T_AGG, D_T_LB, D_T_END, D_NSTRIDE, D_NGEN, D_NSERIAL,
    D_GUESS, D_SPINS, D_COUNT, D_FLAGS, D_REDO, D_C_PREP, D_C_RELAX, D_ROUNDS, D_NSHORT
};

struct PieceSum {
    uint64_t x;     // entry (absolute)
    uint64_t exit;  // first start at or after the piece end (absolute)
    uint64_t R;     // stride run record length
    uint32_t kl, vl;
    uint32_t count;
    uint32_t kind;  // PK_*
};

struct DecodeSmem {
    uint64_t data64[(PIECE + 64) / 8];  // piece bytes + 16 B halo + read slack
    uint16_t pc[NGRAN + 8];             // header-filter masks; later the serial-walk log
    uint64_t sx[2][THREADS];            // per-lane exits, double-buffered by round
    uint32_t sg[THREADS];               // per-lane guesses
    uint8_t tgt[THREADS];               // lane is the target of another lane's exit
    uint32_t bk[PIECE / 32];            // "backed": some strong candidate's next lands here
    uint4 halo[BATCH];                  // first 16 bytes after each piece of the batch
    uint4 lead_halo;                    // first 16 bytes of the batch (lead-in piece's halo)
    PieceSum sum[BATCH];
    uint32_t scan_tmp[NW];
    unsigned long long best, best2;     // entry-heuristic reductions
    uint32_t batch, walk_n, walk_done, pred_ok;
    uint64_t pred_exit;
    uint64_t xk, gk, exitk;
    uint32_t rounds;                    // relaxation rounds of the last relax()
    uint32_t prof[NPROF];               // DIAG: cycles per phase (see HG_PROF)
    uint64_t plast;                     // DIAG: last phase stamp
    int32_t err_kind;
    uint64_t err_pos;
};

// Block-uniform values read from LDS: keep them in SGPRs.
__device__ __forceinline__ uint32_t uni(uint32_t x) { return __builtin_amdgcn_readfirstlane(x); }
__device__ __forceinline__ int32_t uni(int32_t x) { return __builtin_amdgcn_readfirstlane(x); }
__device__ __forceinline__ uint64_t uni(uint64_t x) {
    return (uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)x) |
           ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(x >> 32)) << 32);
}

// DIAG phase accounting: cycles since the last stamp go to counter `slot`
// (0 filter, 1 candidates, 2 lane walks, 3 relax seeding, 4 relax rounds,
// 5 scan+emit, 6 staging, 7 stride attempt).
#define HG_PROF(slot)                                                \
    do {                                                             \
        if (DIAG && threadIdx.x == 0) {                              \
            const uint64_t now_ = __builtin_amdgcn_s_memtime();      \
            s.prof[slot] += (uint32_t)(now_ - s.plast);              \
            s.plast = now_;                                          \
        }                                                            \
    } while (0)

// ---- lane walk --------------------------------------------------------------
// Records starting in [x, segend) (piece-relative), validated exactly as the
// reference would read them.  dead = a record that cannot be read (the
// reference would fail there).  Exit = first start at or after segend.
struct Walk {
    uint64_t exit;      // absolute
    uint32_t p01, p23;  // up to four 16-bit positions
    uint32_t cnt;
    bool dead;
};

__device__ __forceinline__ uint32_t walk_pos(const Walk& w, uint32_t i) {
    const uint32_t v = i < 2 ? w.p01 : w.p23;
    return (i & 1) ? (v >> 16) : (v & 0xFFFFu);
}

__device__ __forceinline__ void lane_walk(const uint8_t* data, uint64_t base, uint64_t len,
                                          uint32_t x, uint32_t segend, Walk& w) {
    w.cnt = 0;
    w.dead = false;
    w.p01 = w.p23 = 0;
    uint64_t cur = x;
#pragma unroll
    for (int it = 0; it < 4; ++it) {
        if (cur >= segend) break;
        const uint64_t abs = base + cur;
        if (abs + 16 > len) {
            w.dead = true;
            break;
        }
        uint32_t k0, k1, v0, v1;
        lds_header32(data, (uint32_t)cur, k0, k1, v0, v1);
        const uint64_t body = (uint64_t)k0 + v0;
        if ((k1 | v1) || body > len - abs - 16) {
            w.dead = true;
            break;
        }
        if (it == 0) w.p01 = (uint32_t)cur;
        if (it == 1) w.p01 |= (uint32_t)cur << 16;
        if (it == 2) w.p23 = (uint32_t)cur;
        if (it == 3) w.p23 |= (uint32_t)cur << 16;
        ++w.cnt;
        cur += 16 + body;
    }
    w.exit = base + cur;
}

__device__ __forceinline__ void write_span(hg_span* out, uint64_t gi, uint64_t off, uint64_t kl,
                                           uint64_t vl) {
    uint4 sp;
    sp.x = (uint32_t)off;
    sp.y = (uint32_t)(off >> 32);
    sp.z = (uint32_t)kl;
    sp.w = (uint32_t)vl;
    *reinterpret_cast<uint4*>(out + gi) = sp;
}

__device__ __forceinline__ void store_span(hg_span* out, uint64_t cap, uint64_t gi,
                                           const uint8_t* data, uint64_t base, uint32_t p) {
    if (gi >= cap) return;
    uint64_t kl, vl;
    lds_header(data, p, kl, vl);
    write_span(out, gi, base + p, kl, vl);
}

// A span from scratch (offset relative to the range) to its final slot.
__device__ __forceinline__ void copy_span(hg_span* dst, const hg_span* src, uint64_t obase) {
    uint4 v = *reinterpret_cast<const uint4*>(src);
    const uint64_t off = (((uint64_t)v.y << 32) | v.x) + obase;
    v.x = (uint32_t)off;
    v.y = (uint32_t)(off >> 32);
    *reinterpret_cast<uint4*>(dst) = v;
}

// store_span for headers whose high words are known zero (the lane walks
// checked them): two 32-bit halves by byte funnel shifts from dword reads
// instead of 64-bit shifts.
#ifndef HG_LW_ST32
#define HG_LW_ST32 1
#endif
__device__ __forceinline__ void lw_store_span(hg_span* out, uint64_t gi, const uint8_t* data,
                                              uint64_t base, uint32_t p) {
    if (!HG_LW_ST32) {
        store_span(out, ~0ull, gi, data, base, p);
        return;
    }
    const uint32_t* w = reinterpret_cast<const uint32_t*>(data + (p & ~3u));
    const uint32_t sh = p & 3u;
    write_span(out, gi, base + p, __builtin_amdgcn_alignbyte(w[1], w[0], sh),
               __builtin_amdgcn_alignbyte(w[3], w[2], sh));
}

// ---- relaxation ---------------------------------------------------------------
// Exact per-lane state for piece entry X (absolute).  All threads call it.
// Each lane caches one walk (from guess g).  A lane is a pass-through when
// its true entry lies at or past its segment end (a record spans it).
// Seeding: a lane is "on the chain" if it is the entry lane or another
// lane's cached exit lands exactly on its guess; every lane starts from the
// cached exit of the nearest chain lane at or before it (block max-scan), so
// with correct guesses one verification round suffices.  Rounds then re-walk
// lanes whose true entry differs from their guess until nothing changes;
// that fixed point is exact.  Returns false if it did not converge.  On
// return cnt = this lane's records, any_dead says whether the true path hits
// an unreadable record, and s.exitk is the piece exit.
template <bool DIAG, typename Smem>
__device__ bool relax(Smem& s, const uint8_t* data, uint64_t base, uint64_t len,
                      uint32_t clen, uint64_t X, uint32_t& g, Walk& w, uint32_t& cnt,
                      bool& any_dead) {
    const uint32_t t = threadIdx.x;
    const uint32_t lane = t & 63u, wid = t >> 6;
    const uint32_t segend = min((t + 1) * SEG, clen);
    const uint64_t seg_end_abs = base + segend;
    const uint32_t je = (X >= base + clen) ? THREADS : (uint32_t)((X - base) / SEG);
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
        const uint32_t u = (uint32_t)((w.exit - base) / SEG);
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
    HG_PROF(3);
    bool ok = false, pass = false;
    uint32_t r = 1;
    for (; r <= MAX_ROUNDS; ++r) {
        const uint64_t* cur = s.sx[r & 1];
        uint64_t* nxt = s.sx[(r + 1) & 1];
        int changed = 0;
        if (active) {
            const uint64_t ein = (t == je) ? X : cur[t - 1];
            uint64_t val;
            if (ein >= seg_end_abs) {  // a record (or the piece exit) spans this segment
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
    cnt = (active && !pass) ? w.cnt : 0;
    any_dead = __syncthreads_or(active && !pass && w.dead);
    if (t == THREADS - 1) {
        s.exitk = s.sx[(r + 1) & 1][t];
        s.rounds = r;
    }
    __syncthreads();
    HG_PROF(4);
    return ok;
}

// ---- look-back ------------------------------------------------------------
struct LookbackOut {
    uint64_t x, g, errpos;
    int32_t err;  // HG_OK or error kind to propagate
};

// Exact entry and record base of batch k.  Called by all 64 lanes of wave 0.
__device__ LookbackOut lookback(const DecodeArgs& a, uint32_t k, uint32_t& spins_out) {
    const uint32_t lane = threadIdx.x & 63u;
    LookbackOut r{0, 0, 0, HG_OK};
    // The budget bounds each wait (a restart waits for a newer batch, so a
    // legitimately long chain of restarts does not add up to a false error);
    // spins_out reports the total.
    // A wait can legitimately outlast any fixed budget: when every batch
    // guessed wrong, each INCL is the end of a serial chain of redos below
    // it.  So the budget counts spins without progress anywhere in the grid
    // (DecodeCtl::progress unchanged), and only a stalled grid is an error.
    uint32_t spins = 0, spins_done = 0;
    const uint32_t SPIN_LIMIT = 1u << 22;
    uint32_t seen = __hip_atomic_load(&a.ctl->progress, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    auto stalled = [&]() -> bool {
        const uint32_t now =
            __hip_atomic_load(&a.ctl->progress, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (now != seen) {
            seen = now;
            spins_done += spins;
            spins = 0;
            return false;
        }
        return ++spins > SPIN_LIMIT;
    };
restart:
    spins_done += spins;
    spins = 0;
    int64_t j0 = (int64_t)k - 1;
    uint64_t acc = 0, xk = 0;
    bool first = true;
    for (;;) {
        const int64_t j = j0 - (int64_t)lane;
        unsigned long long w0, w1;
        uint32_t f;
        int fi;
        for (;;) {
            if (j < 0) {  // virtual batch -1: exact exit = the entry, 0 records
                w0 = pack_status(ST_INCL, 0, a.entry);
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
            if (stalled()) {
                r.err = HG_ERR_INTERNAL;
                spins_out = spins_done + spins;
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
                spins_out = spins_done + spins;
                return r;
            }
        }
        // AGG lanes: predicted incoming exit must equal the older neighbour's exit.
        const uint32_t xrel = st_aux(w1);
        const uint64_t P = (xrel != NONE_REL) ? (uint64_t)j * a.bp * PIECE + xrel : E;
        const uint64_t Eolder = __shfl_down(E, 1, 64);
        const int lim = fi < 64 ? fi : 63;  // lanes [0, lim) are checked
        const bool bad = (int)lane < lim && P != Eolder;
        const unsigned long long badm = __ballot(bad);
        if (badm) {
            // The oldest mismatch is a batch whose guess was wrong; it
            // corrects itself after its own look-back.  Wait for its INCL.
            const int m = 63 - __clzll((long long)badm);
            const int64_t jm = j0 - m;
            for (;;) {
                unsigned long long v0 = ld_agent(&a.status[2 * jm]);
                unsigned long long v1 = ld_agent(&a.status[2 * jm + 1]);
                if (st_flag(v0) == st_flag(v1) && st_flag(v0) >= ST_INCL) break;
                if (stalled()) {
                    r.err = HG_ERR_INTERNAL;
                    spins_out = spins_done + spins;
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
            spins_out = spins_done + spins;
            return r;
        }
        first = false;
        j0 -= 63;  // lane 63 becomes the next window's lane 0
    }
}

// ---- serial walk (exact; errors and pathological pieces) ---------------------
// Thread 0 walks from absolute x, logging up to WALK_LOG starts into s.pc;
// the whole block then writes the batch to out[gbase + i] (i < cap - gbase).
// Returns the count; s.err_kind / s.err_pos / s.exitk describe the end.
__device__ uint64_t serial_walk_emit(DecodeSmem& s, uint64_t len, uint64_t base, uint32_t clen,
                                     uint64_t x, hg_span* out, uint64_t cap, uint64_t gbase,
                                     uint64_t ob) {
    const uint8_t* data = reinterpret_cast<const uint8_t*>(s.data64);
    uint64_t emitted = 0;
    __syncthreads();
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
            while (n < WALK_LOG) {
                if (cur >= base + clen) {
                    done = true;
                    break;
                }
                if (cur + 16 > len) {
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
                if (kl + vl > len - cur - 16) {
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
        for (uint32_t t = threadIdx.x; t < n; t += THREADS)
            store_span(out, cap, gbase + emitted + t, data, base + ob, s.pc[t]);
        emitted += n;
        const bool done = s.walk_done;
        if (done) break;
    }
    __syncthreads();
    if (threadIdx.x == 0 && s.err_kind != HG_OK) s.err_pos = s.exitk;
    __syncthreads();
    return emitted;
}

// ---- stride fast path ---------------------------------------------------------
__device__ __forceinline__ bool hdr_eq(const uint8_t* data, uint32_t p, uint64_t kl, uint64_t vl) {
    uint64_t a, b;
    lds_header(data, p, a, b);
    return a == kl && b == vl;
}

// Starts in [X, piece end) if every record there repeats the header at X:
// record t starts at X + t*R.  All threads call it; one parallel compare per
// record.  Exact: if all headers match, each record's next is the following
// one.  Returns false (not an error) when the run breaks or X cannot be read.
__device__ bool stride_run(const uint8_t* data, uint64_t base, uint64_t len, uint32_t clen,
                           uint64_t X, PieceSum& ps) {
    ps.x = X;
    if (X >= base + clen) {  // no record starts in this piece
        ps.count = 0;
        ps.R = 0;
        ps.kl = ps.vl = 0;
        ps.kind = PK_EMPTY;
        return true;
    }
    const uint32_t xr = (uint32_t)(X - base);
    if (X + 16 > len) return false;
    uint64_t kl, vl;
    lds_header(data, xr, kl, vl);
    kl = uni(kl);
    vl = uni(vl);
    if (kl > ~0ull - vl || kl + vl > len - X - 16 || ((kl >> 32) | (vl >> 32))) return false;
    const uint64_t R = 16 + kl + vl;
    const uint32_t m = (uint32_t)((clen - xr + R - 1) / R);  // records starting in [xr, clen)
    if (X + m * R > len) return false;                       // the last one would not fit
    // fail fast without a barrier: the second record's header (block-uniform)
    if (m > 1) {
        uint64_t k2, v2;
        lds_header(data, xr + (uint32_t)R, k2, v2);
        if (uni(k2) != kl || uni(v2) != vl) return false;
    }
    int bad = 0;
    for (uint32_t t = 1 + threadIdx.x; t < m; t += THREADS)
        bad |= !hdr_eq(data, xr + (uint32_t)(t * R), kl, vl);
    bad = __syncthreads_or(bad);
    if (bad) return false;
    ps.count = m;
    ps.R = R;
    ps.kl = (uint32_t)kl;
    ps.vl = (uint32_t)vl;
    ps.kind = PK_STRIDE;
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

// Wave 0: the first position in the piece's first KiB whose header repeats
// 3 lengths ahead (inside the piece), or NO_GUESS.
__device__ uint32_t stride_guess(const uint8_t* data, uint64_t rem, uint32_t clen, uint32_t hz) {
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
template <bool DIAG>
__device__ void general_prepare(DecodeSmem& s, const uint8_t* data, uint64_t base, uint64_t len,
                                uint64_t rem, uint32_t clen, uint32_t hz, uint32_t& g, Walk& w,
                                uint64_t far = HG_FAR_CAND) {
    const uint32_t tid = threadIdx.x;
    const bool any_valid = rem >= 16;
    const uint64_t plim64 = any_valid ? rem - 16 : 0;
    const uint32_t plim = plim64 < 0xFFFFFFFFull ? (uint32_t)plim64 : 0xFFFFFFFFu;
    __syncthreads();
#pragma unroll
    for (uint32_t i = 0; i < GPT; ++i) {
        const uint32_t gi = i * THREADS + tid;
        s.pc[gi] = (uint16_t)filter_bits(data, gi, hz, clen, plim, any_valid);
    }
    for (uint32_t i = tid; i < PIECE / 32; i += THREADS) s.bk[i] = 0;
    __syncthreads();
    HG_PROF(0);
    const uint32_t seg0 = tid * SEG;
    const uint32_t segend = min(seg0 + SEG, clen);
    uint64_t strong = 0;
    uint32_t seen = 0;
    for (uint32_t j = 0; j < GPT && seen < CAND_CAP; ++j) {
        uint32_t c = s.pc[tid * GPT + j];
        while (c && seen < CAND_CAP) {
            const uint32_t b = __ffs(c) - 1;
            c &= c - 1;
            ++seen;
            const uint32_t p = seg0 + j * 16 + b;
            uint64_t kl, vl;
            lds_header(data, p, kl, vl);
            // far candidates (a record of >= HG_FAR_CAND bytes) are not used
            // for guesses: shifted reads of a small header decode as records
            // 256x or 65536x longer, and genuine huge records are walked
            // exactly anyway (speed only; every path is exact from its entry)
            if (((kl >> 32) | (vl >> 32)) || kl + vl > rem - p - 16 || kl + vl >= far) continue;
            const uint64_t nx = (uint64_t)p + 16 + kl + vl;
            if (nx < clen) {
                if (!((s.pc[nx >> 4] >> (nx & 15)) & 1u)) continue;  // look-ahead
                atomicOr(&s.bk[nx >> 5], 1u << (nx & 31));
            }
            strong |= 1ull << (j * 16 + b);
        }
    }
    __syncthreads();
    HG_PROF(1);
    const uint64_t backed = (uint64_t)s.bk[seg0 >> 5] | ((uint64_t)s.bk[(seg0 >> 5) + 1] << 32);
    const uint64_t gm = strong & backed;
    g = gm ? seg0 + (uint32_t)(__ffsll((long long)gm) - 1) : NO_GUESS;
    w.exit = 0;
    w.cnt = 0;
    w.dead = true;
    w.p01 = w.p23 = 0;
    if (g != NO_GUESS) lane_walk(data, base, len, g, segend, w);
    s.sg[tid] = (g != NO_GUESS && !w.dead) ? g : NO_GUESS;
    s.sx[0][tid] = strong;  // the strong mask, for the entry guess
    __syncthreads();
    HG_PROF(2);
}

// Lean preparation (HG_LEAN, the default): each lane's guess is the first
// candidate of its 64 bytes that reads as a record shorter than HG_FAR_CAND
// and fits the file (a shifted read of a small header decodes as a record
// 256x or 65536x longer), then the lane walks <= 4 records from it.  No
// candidate evaluation beyond the guess and no "backed" marks: relax() makes
// the result exact from the piece entry either way, and with these guesses
// it verifies in one round on random data (profiles/r2_pmc_small.json: the
// evaluation of every candidate was ~40 % of the engine's time).
// Candidate positions of the 64-byte segment at seg0 (n <= 64 positions,
// p <= plim): bit j <=> bytes [j+8-hz, j+8) and [j+16-hz, j+16) are zero.
__device__ __forceinline__ uint64_t cand_mask(const uint8_t* data, uint32_t seg0, uint32_t n,
                                              uint64_t plim, uint32_t hz) {
    const uint4* q = reinterpret_cast<const uint4*>(data + seg0);
    const uint64_t z0 = (uint64_t)zmask16(q[0]) | ((uint64_t)zmask16(q[1]) << 16) |
                        ((uint64_t)zmask16(q[2]) << 32) | ((uint64_t)zmask16(q[3]) << 48);
    const uint64_t z1 = zmask16(q[4]);
    const unsigned __int128 Z = ((unsigned __int128)z1 << 64) | z0;
    unsigned __int128 A = Z;  // bit j: bytes j .. j+hz-1 are zero
    for (uint32_t sh = 1; sh < hz; ++sh) A &= Z >> sh;
    uint64_t c = (uint64_t)(A >> (8 - hz)) & (uint64_t)(A >> (16 - hz));
    if (n < 64) c &= (1ull << n) - 1ull;
    if (plim < seg0) return 0;
    const uint64_t lim = plim - seg0;  // j <= lim
    if (lim < 63) c &= (2ull << lim) - 1ull;
    return c;
}

// Each lane publishes its candidate mask (s.sx[1], free until relax()), then
// takes the first candidate that (a) ENDS a run of consecutive candidates, (b)
// reads as a record shorter than `far` that fits the file, and (c) whose next
// record start is again a candidate or lies past the piece.  (a) is the key
// rule: a genuine header with small lengths also passes the zero-byte filter
// 1-3 bytes to its left (those reads see the length bytes shifted up, i.e.
// 256x / 65536x longer records whose next start usually lies past the piece,
// so (c) cannot reject them); the genuine start is the last position of that
// run (tools/lean_sim.py: ~28 of 256 lanes guessed wrong on small records
// without (a), ~0.1 with it).  Lanes whose run ends hold no usable guess fall
// back to any candidate.  All threads call it.
template <bool DIAG>
__device__ void lean_prepare(DecodeSmem& s, const uint8_t* data, uint64_t base, uint64_t len,
                             uint64_t rem, uint32_t clen, uint32_t hz, uint32_t& g, Walk& w,
                             uint64_t far = HG_FAR_CAND) {
    const uint32_t tid = threadIdx.x;
    const uint32_t seg0 = tid * SEG;
    const uint32_t segend = min(seg0 + SEG, clen);
    g = NO_GUESS;
    w.exit = 0;
    w.cnt = 0;
    w.dead = true;
    w.p01 = w.p23 = 0;
    const uint64_t cm0 =
        (seg0 < clen && rem >= 16) ? cand_mask(data, seg0, segend - seg0, rem - 16, hz) : 0;
    __syncthreads();  // the previous user of s.sx is done
    s.sx[1][tid] = cm0;
    __syncthreads();
    HG_PROF(0);
    const uint64_t nextbit = tid + 1 < THREADS ? (s.sx[1][tid + 1] & 1ull) : 0ull;
    const uint64_t runend = cm0 & ~((cm0 >> 1) | (nextbit << 63));
    uint64_t cm = runend;
#pragma nounroll
    for (uint32_t pass = 0; pass < 2 && g == NO_GUESS; ++pass) {
        if (pass) cm = cm0 & ~runend;
        while (cm) {
            const uint32_t p = seg0 + (uint32_t)(__ffsll((long long)cm) - 1);
            cm &= cm - 1;
            uint32_t k0, k1, v0, v1;
            lds_header32(data, p, k0, k1, v0, v1);
            const uint64_t body = (uint64_t)k0 + v0;
            if ((k1 | v1) || body >= far || body > rem - p - 16) continue;
            const uint64_t nx = (uint64_t)p + 16 + body;
            if (nx < clen && !((s.sx[1][nx / SEG] >> (nx % SEG)) & 1ull)) continue;  // look-ahead
            g = p;
            break;
        }
    }
    if (g != NO_GUESS) lane_walk(data, base, len, g, segend, w);
    HG_PROF(1);
}

// Entry guess of a piece whose entry is unknown (lean mode): the first lane
// guess that is LINKED (its walk exits exactly on another lane's guess), else
// the first lane guess, else -- a piece of nothing but records longer than
// HG_FAR_CAND -- the same with every candidate.  ~0 if the piece has none.
// Leaves g / w as lean_prepare made them for relax().  All threads call it.
template <bool DIAG>
__device__ uint64_t lean_entry_guess(DecodeSmem& s, const uint8_t* data, uint64_t base,
                                     uint64_t len, uint64_t rem, uint32_t clen, uint32_t hz,
                                     uint32_t& g, Walk& w) {
    const uint32_t tid = threadIdx.x;
#pragma nounroll
    for (uint32_t attempt = 0; attempt < 2; ++attempt) {
        lean_prepare<DIAG>(s, data, base, len, rem, clen, hz, g, w,
                           attempt ? ~0ull : (uint64_t)HG_FAR_CAND);
        const bool valid = g != NO_GUESS && !w.dead;
        s.sg[tid] = valid ? g : NO_GUESS;
        if (tid == 0) {
            s.best = ~0ull;
            s.best2 = ~0ull;
        }
        __syncthreads();
        bool linked = false;
        if (valid && w.exit < base + clen) {
            const uint32_t u = (uint32_t)(w.exit - base);
            linked = s.sg[u / SEG] == u;
        }
        if (linked) atomicMin(&s.best, (unsigned long long)(base + g));
        if (valid) atomicMin(&s.best2, (unsigned long long)(base + g));
        __syncthreads();
        const uint64_t b1 = uni((uint64_t)s.best), b2 = uni((uint64_t)s.best2);
        __syncthreads();
        if (b1 != ~0ull) return b1;
        if (b2 != ~0ull) return b2;
    }
    return ~0ull;
}

// Piece entry guess from the general engine.  p1 = the first strong
// candidate whose next start is another lane's guess ("links": the first
// record backs the second).  The true entry is in [p1, next(p1)) and links
// too; a shifted read of a small header also links sometimes, but decodes
// as a ~256x longer record — so the guess is the linking candidate with the
// shortest record in that window.  With no link at all: the strong candidate
// with the shortest record.  ~0 if the piece has no candidate.
__device__ uint64_t general_entry_guess(DecodeSmem& s, const uint8_t* data, uint64_t base,
                                        uint32_t clen) {
    const uint32_t tid = threadIdx.x;
    const uint32_t seg0 = tid * SEG;
    if (tid == 0) {
        s.best = ~0ull;
        s.best2 = ~0ull;
    }
    const uint64_t m0 = s.sx[0][tid];
    __syncthreads();
    uint64_t m = m0;
    unsigned long long first_link = ~0ull, shortest = ~0ull;
    for (uint32_t it = 0; m && it < CAND_CAP; ++it) {
        const uint32_t b = __ffsll((long long)m) - 1;
        m &= m - 1;
        const uint32_t p = seg0 + b;
        uint64_t kl, vl;
        lds_header(data, p, kl, vl);
        const uint64_t nx = (uint64_t)p + 16 + kl + vl;
        if (nx < clen && s.sg[nx / SEG] == (uint32_t)nx) {
            first_link = ((unsigned long long)p << 32) | (uint32_t)nx;
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
    if (b1 == ~0ull) return b2 != ~0ull ? base + (b2 & 0xFFFFu) : ~0ull;
    const uint32_t p1 = (uint32_t)(b1 >> 32), n1 = (uint32_t)b1;
    // shortest linking candidate in [p1, n1)
    unsigned long long best = ~0ull;
    if (seg0 < n1 && seg0 + SEG > p1) {
        m = m0;
        for (uint32_t it = 0; m && it < CAND_CAP; ++it) {
            const uint32_t b = __ffsll((long long)m) - 1;
            m &= m - 1;
            const uint32_t p = seg0 + b;
            if (p < p1 || p >= n1) continue;
            uint64_t kl, vl;
            lds_header(data, p, kl, vl);
            const uint64_t nx = (uint64_t)p + 16 + kl + vl;
            if (nx < clen && s.sg[nx / SEG] == (uint32_t)nx) {
                const unsigned long long key = ((16 + kl + vl) << 16) | p;
                best = key < best ? key : best;
            }
        }
    }
    for (int d = 32; d >= 1; d >>= 1) {
        const unsigned long long o = __shfl_xor(best, d, 64);
        best = o < best ? o : best;
    }
    if (tid == 0) s.best = ~0ull;
    __syncthreads();
    if ((tid & 63) == 0) atomicMin(&s.best, best);
    __syncthreads();
    const unsigned long long bb = s.best;
    __syncthreads();
    return base + (bb != ~0ull ? (uint32_t)(bb & 0xFFFFu) : p1);
}

// ---- piece staging ------------------------------------------------------------
// 16 bytes at off (absolute), zero past len; register-only byte assembly at
// the file tail.
__device__ __forceinline__ uint4 load16(const DecodeArgs& a, uint64_t off) {
    if (off + 16 <= a.rlen) return *reinterpret_cast<const uint4*>(a.sst + off);
    uint32_t w[4] = {0, 0, 0, 0};
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int b = 0; b < 4; ++b) {
            const uint64_t o = off + q * 4 + b;
            if (o < a.rlen) w[q] |= (uint32_t)a.sst[o] << (8 * b);
        }
    return make_uint4(w[0], w[1], w[2], w[3]);
}

// Table bytes are read once per call: nontemporal loads (tools/probes/
// read_probe.hip: a 1 GiB sweep reads at 7.0 TB/s nt vs 6.3 TB/s default).
#ifndef HG_NT_LOADS
#define HG_NT_LOADS 1
#endif
__device__ __forceinline__ void load_piece(const DecodeArgs& a, uint32_t p, uint4 (&v)[GPT]) {
    const uint64_t base = (uint64_t)p * PIECE;
    if (base + PIECE <= a.rlen) {  // uniform: plain 16-byte loads, no per-lane branch
        const uint4* src = reinterpret_cast<const uint4*>(a.sst + base) + threadIdx.x;
#pragma unroll
        for (uint32_t i = 0; i < GPT; ++i) {
            if (HG_NT_LOADS) {
                typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
                const u32x4 x = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(src + i * THREADS));
                v[i] = make_uint4(x.x, x.y, x.z, x.w);
            } else {
                v[i] = src[i * THREADS];
            }
        }
    } else {
#pragma unroll
        for (uint32_t i = 0; i < GPT; ++i) v[i] = load16(a, base + (i * THREADS + threadIdx.x) * 16);
    }
}

// All threads: v -> LDS (after the previous piece is done with it), halo, slack.
// lead: the batch's lead-in piece (its halo is s.lead_halo).
__device__ __forceinline__ void stage_piece(DecodeSmem& s, const uint4 (&v)[GPT], uint32_t i,
                                            bool lead = false) {
    uint8_t* data = reinterpret_cast<uint8_t*>(s.data64);
    __syncthreads();
#pragma unroll
    for (uint32_t q = 0; q < GPT; ++q)
        *reinterpret_cast<uint4*>(data + (q * THREADS + threadIdx.x) * 16) = v[q];
    if (threadIdx.x < 4)
        *reinterpret_cast<uint4*>(data + PIECE + threadIdx.x * 16) =
            threadIdx.x == 0 ? (lead ? s.lead_halo : s.halo[i]) : make_uint4(0, 0, 0, 0);
    __syncthreads();
}

// Thread 0 walks at most SHORT_WALK records from X.  True if the piece ends
// within that budget with every record readable: the starts are then in
// s.pc[0, s.walk_n) and s.exitk is the exit.  Pieces of a few large records
// skip the general engine this way.
__device__ bool short_walk(DecodeSmem& s, const uint8_t* data, uint64_t len, uint64_t base,
                           uint32_t clen, uint64_t X) {
    if (threadIdx.x == 0) {
        uint32_t n = 0;
        uint64_t cur = X;
        bool ok = false;
        for (;;) {
            if (cur >= base + clen) {
                ok = true;
                break;
            }
            if (n == SHORT_WALK || cur + 16 > len) break;
            const uint32_t p = (uint32_t)(cur - base);
            uint32_t k0, k1, v0, v1;
            lds_header32(data, p, k0, k1, v0, v1);
            const uint64_t body = (uint64_t)k0 + v0;
            if ((k1 | v1) || body > len - cur - 16) break;
            s.pc[n++] = (uint16_t)p;
            cur += 16 + body;
        }
        s.walk_n = n;
        s.walk_done = ok;
        s.exitk = cur;
    }
    __syncthreads();
    return s.walk_done;
}

constexpr uint64_t X_UNKNOWN = ~0ull;
constexpr int32_t E_NO_GUESS = 100;  // speculative entry guess found nothing

// ---- one piece ------------------------------------------------------------------
// Path of the piece starting at X (absolute; X_UNKNOWN = guess it first: a
// record whose header repeats 3 lengths ahead, else the general engine's
// entry guess).  Stride pieces are summarised (emit_now: also emitted at
// out[gbase + t]); other pieces are emitted at out[gbase + ...] (the scratch
// area while the record base is unknown).  Returns HG_OK, E_NO_GUESS, or an
// error kind with s.err_pos (the failing record) — the records before it are
// emitted and counted in ps.count.  X is updated to the entry used.
template <bool DIAG>
__device__ int32_t piece_path(DecodeSmem& s, const DecodeArgs& a, uint32_t p, uint64_t& X,
                              bool emit_now, bool try_short, hg_span* out, uint64_t cap,
                              uint64_t gbase, PieceSum& ps, uint64_t& exit, uint32_t& mode,
                              bool try_stride = true) {
    const uint8_t* data = reinterpret_cast<const uint8_t*>(s.data64);
    const uint64_t base = (uint64_t)p * PIECE;
    const uint64_t rem = a.len - base;                       // readable (record validity)
    const uint32_t clen = piece_clen(a, base);               // where records may start
    const uint64_t ob = emit_now ? a.obase : 0;              // span offsets into `spans`
    uint32_t g = NO_GUESS, cnt = 0;
    Walk w;
    w.exit = 0;
    w.cnt = 0;
    w.dead = true;
    w.p01 = w.p23 = 0;
    bool prepared = false;
    if (X == X_UNKNOWN) {
        if (threadIdx.x < 64) {
            const uint32_t f = stride_guess(data, rem, clen, a.hz);
            if (threadIdx.x == 0) s.walk_n = f;
        }
        __syncthreads();
        const uint32_t f = uni(s.walk_n);
        if (f != NO_GUESS) {
            X = base + f;
        } else if (HG_LEAN == 2) {
            X = lean_entry_guess<DIAG>(s, data, base, a.len, rem, clen, a.hz, g, w);
            prepared = true;
            if (X == ~0ull) {
                X = X_UNKNOWN;
                mode = 0;
                return E_NO_GUESS;
            }
        } else {
            // first with far candidates left out of the guesses, then (a piece
            // of nothing but far records) with every candidate
#pragma nounroll
            for (uint32_t attempt = 0; attempt < 2; ++attempt) {
                general_prepare<DIAG>(s, data, base, a.len, rem, clen, a.hz, g, w,
                                      attempt ? ~0ull : (uint64_t)HG_FAR_CAND);
                // Park the lane walk in LDS that is free until relax() (keeps
                // the guess's registers off the walk's): exit -> sx[1],
                // positions -> bk, count|dead -> tgt; g is s.sg (NO_GUESS when
                // dead).
                const uint32_t t = threadIdx.x;
                s.sx[1][t] = w.exit;
                s.bk[t] = w.p01;
                s.bk[THREADS + t] = w.p23;
                s.tgt[t] = (uint8_t)(w.cnt | (w.dead ? 16u : 0u));
                X = uni(general_entry_guess(s, data, base, clen));
                g = s.sg[t];
                w.exit = s.sx[1][t];
                w.p01 = s.bk[t];
                w.p23 = s.bk[THREADS + t];
                w.cnt = s.tgt[t] & 15u;
                w.dead = (s.tgt[t] & 16u) != 0;
                if (X != ~0ull || HG_FAR_CAND >= (1ull << 62)) break;
            }
            prepared = true;
            if (X == ~0ull) {
                X = X_UNKNOWN;
                mode = 0;
                return E_NO_GUESS;
            }
        }
    }
    HG_PROF(6);
    if (!prepared && try_stride && stride_run(data, base, a.len, clen, X, ps)) {
        mode = 1;
        exit = ps.kind == PK_EMPTY ? X : X + ps.count * ps.R;
        ps.exit = exit;
        if (emit_now && ps.kind == PK_STRIDE)
            for (uint32_t t = threadIdx.x; t < ps.count; t += THREADS)
                if (gbase + t < cap) write_span(out, gbase + t, ob + X + t * ps.R, ps.kl, ps.vl);
        return HG_OK;
    }
    HG_PROF(7);
    ps.x = X;
    ps.R = 0;
    ps.kl = ps.vl = 0;
    ps.kind = PK_SCRATCH;
    if (!prepared && try_short && short_walk(s, data, a.len, base, clen, X)) {
        mode = 4;
        const uint32_t n = uni(s.walk_n);
        for (uint32_t t = threadIdx.x; t < n; t += THREADS)
            store_span(out, cap, gbase + t, data, base + ob, s.pc[t]);
        ps.count = n;
        exit = ps.exit = uni(s.exitk);
        return HG_OK;
    }
    if (!prepared) {
        if (HG_LEAN)
            lean_prepare<DIAG>(s, data, base, a.len, rem, clen, a.hz, g, w);
        else
            general_prepare<DIAG>(s, data, base, a.len, rem, clen, a.hz, g, w);
    }
    bool dead = false;
    const bool conv = relax<DIAG>(s, data, base, a.len, clen, X, g, w, cnt, dead);
    if (conv && !dead) {
        mode = 2;
        uint32_t tot;
        const uint32_t pre = block_excl_scan<NW>(cnt, s.scan_tmp, tot);
        for (uint32_t i = 0; i < cnt; ++i)
            store_span(out, cap, gbase + pre + i, data, base + ob, walk_pos(w, i));
        ps.count = uni(tot);
        exit = ps.exit = uni(s.exitk);
        __syncthreads();
        HG_PROF(5);
        return HG_OK;
    }
    mode = 3;
    ps.count = uni((uint32_t)serial_walk_emit(s, a.len, base, clen, X, out, cap, gbase, ob));
    exit = ps.exit = uni(s.exitk);
    return uni(s.err_kind);
}

// ---- kernel ------------------------------------------------------------------------
// The pre-pass batch's link check: batch j is good iff it verified and its
// guessed entry is its predecessor's exit (batch 0: entry 0).  Both batches of
// a pair add into one 64-bit word -- an arrival in the top byte, exit resp.
// -x0 mod 2^48 below -- so whichever arrives second sees the whole sum in the
// value its atomic returns.  No fences: an agent-scope release on gfx950
// writes back and invalidates the XCD's L2, which stalls the streaming
// workgroups around it (measured: 205 -> 755 us for the pre-pass).  Offsets
// are < 2^40 (HG_ERR_TOO_LARGE), so the 48-bit sum is exact.
constexpr uint64_t LINK_ONE = 1ull << 56, LINK_MASK = (1ull << 48) - 1;
__device__ __forceinline__ void mark_bad(DecodeCtl* c, uint32_t nspec, uint32_t j) {
    atomicMax(&c->bad_rev, nspec - j);
}
__device__ __forceinline__ void link_arrive(const DecodeArgs& a, uint32_t j, uint64_t v) {
    const unsigned long long add = LINK_ONE | (v & LINK_MASK);
    const unsigned long long old = atomicAdd(&a.link[j], add);
    if ((old >> 56) == 1 && ((old + add) & LINK_MASK) != 0) mark_bad(a.ctl, a.nspec, j);
}

// Record base of pre-pass batch e (all batches below e resolved): the group
// sums before e's group plus the counts before e inside it.  One wave, one
// round of independent loads (plus one per 64 further groups).
__device__ uint64_t spec_base(const DecodeArgs& a, uint32_t e) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t g = e / SPEC_GROUP;
    uint64_t v = 0;
    for (uint32_t k = lane; k < g; k += 64) v += a.gsum[k];
    const uint32_t j = g * SPEC_GROUP + lane;
    if (j < e) v += a.sbatch[j].count;
    return wave_sum<uint64_t>(v);
}

#ifndef HG_EMIT_U
#define HG_EMIT_U 4
#endif
constexpr uint32_t EMIT_U = HG_EMIT_U;  // scratch spans in flight per thread (emit_spec_range)

// Wave 0 (all 64 lanes): piece record p of lane (< n) into LDS with its
// record base g0 + the counts before it (one DPP scan; a serial loop of
// thread 0 over 64 pieces was ~3 us of dependent LDS reads per workgroup,
// with no span store in flight meanwhile), then the batch's end and whether
// any piece was hop-walked.
__device__ __forceinline__ void stage_pieces(SpecPiece* pc, uint64_t* pbase, const SpecPiece& p,
                                             uint32_t n, uint64_t g0) {
    const uint32_t lane = threadIdx.x;
    const uint32_t cnt = lane < n ? p.count : 0u;
    const uint32_t incl = dpp_sum_incl(cnt);  // n <= SPEC_BP = 64 counts of <= PIECE_RECS
    const bool hop = lane < n && p.pad == SP_HOP;
    if (lane < n) {
        pc[lane] = p;
        pbase[lane] = g0 + incl - cnt;
    }
    const uint32_t tot = __builtin_amdgcn_readlane(incl, 63);
    const uint64_t hb = __ballot(hop);
    if (lane == 0) {
        pbase[SPEC_BP] = g0 + tot;
        pbase[SPEC_BP + 1] = hb != 0;
    }
}

__device__ uint64_t emit_staged(DecodeSmem& s, const DecodeArgs& a, uint32_t q0, uint32_t n,
                                uint64_t g0);

// Spans of pieces [q0, q0 + n) (n <= SPEC_BP) from their pre-pass summaries
// (stride arithmetic, or the hop walk's scratch), record base g0.  All
// threads; returns the record index after the last piece.
__device__ uint64_t emit_spec_range(DecodeSmem& s, const DecodeArgs& a, uint32_t q0, uint32_t n,
                                    uint64_t g0) {
    const uint32_t tid = threadIdx.x;
    SpecPiece* pc = reinterpret_cast<SpecPiece*>(s.data64);  // LDS scratch
    uint64_t* pbase = reinterpret_cast<uint64_t*>(pc + SPEC_BP);
    __syncthreads();
    if (tid < 64) {
        SpecPiece p{};
        if (tid < n) p = a.spiece[q0 + tid];
        stage_pieces(pc, pbase, p, n, g0);
    }
    __syncthreads();
    return emit_staged(s, a, q0, n, g0);
}

__device__ uint64_t spec_base(const DecodeArgs& a, uint32_t e);

// The same for pre-pass batch e (pieces [q0, q0 + n)) of the resolved prefix
// at the start of decode_kernel: its record base (spec_base) is loaded by
// wave 0 together with the piece records (one round of loads, one barrier).
__device__ uint64_t emit_spec_batch(DecodeSmem& s, const DecodeArgs& a, uint32_t e, uint32_t q0,
                                    uint32_t n) {
    const uint32_t tid = threadIdx.x;
    SpecPiece* pc = reinterpret_cast<SpecPiece*>(s.data64);
    uint64_t* pbase = reinterpret_cast<uint64_t*>(pc + SPEC_BP);
    if (tid < 64) {
        SpecPiece p{};
        if (tid < n) p = a.spiece[q0 + tid];
        const uint64_t g0 = spec_base(a, e);
        stage_pieces(pc, pbase, p, n, g0);
        if (tid == 0) s.xk = g0;
    }
    __syncthreads();
    return emit_staged(s, a, q0, n, uni(s.xk));
}

// emit_spec_range after the pieces were staged (all threads).
__device__ uint64_t emit_staged(DecodeSmem& s, const DecodeArgs& a, uint32_t q0, uint32_t n,
                                uint64_t g0) {
    const uint32_t tid = threadIdx.x;
    const SpecPiece* pc = reinterpret_cast<const SpecPiece*>(s.data64);
    const uint64_t* pbase = reinterpret_cast<const uint64_t*>(pc + SPEC_BP);
    if (uni(pbase[SPEC_BP + 1])) {
        // Batches with walked pieces (hop / lane-walk spans in scratch): the
        // copies run over the batch's records flattened, EMIT_U per thread
        // with every load issued before the first store (per piece, one
        // load / wait / store round per 256 records had made this a chain
        // of ~2 HBM round trips per piece).
        const uint64_t total = uni(pbase[SPEC_BP]) - g0;
        for (uint64_t j0 = 0; j0 < total; j0 += (uint64_t)THREADS * EMIT_U) {
            uint4 v[EMIT_U];
            uint32_t pi[EMIT_U];
            uint64_t tt[EMIT_U];
    #pragma unroll
            for (uint32_t u = 0; u < EMIT_U; ++u) {
                const uint64_t j = min(j0 + u * THREADS + tid, total - 1);
                const uint64_t gp = g0 + j;
                uint32_t lo = 0, hi = n;  // the piece holding record gp: last pbase <= gp
                while (hi - lo > 1) {
                    const uint32_t mid = (lo + hi) >> 1;
                    if (pbase[mid] <= gp) lo = mid;
                    else hi = mid;
                }
                pi[u] = lo;
                tt[u] = gp - pbase[lo];
                const hg_span* src = a.scratch + (size_t)(q0 + lo) * MAX_REC_PIECE + tt[u];
                v[u] = pc[lo].pad == SP_HOP ? *reinterpret_cast<const uint4*>(src)
                                            : make_uint4(0, 0, 0, 0);
            }
    #pragma unroll
            for (uint32_t u = 0; u < EMIT_U; ++u) {
                const uint64_t j = j0 + u * THREADS + tid;
                const uint64_t gp = g0 + j;
                if (j >= total || gp >= a.cap) continue;
                const SpecPiece& q = pc[pi[u]];
                if (q.pad == SP_HOP) {
                    const uint64_t off = (((uint64_t)v[u].y << 32) | v[u].x) + a.obase;
                    v[u].x = (uint32_t)off;
                    v[u].y = (uint32_t)(off >> 32);
                    *reinterpret_cast<uint4*>(a.spans + gp) = v[u];
                } else {
                    write_span(a.spans, gp, a.obase + q.x + tt[u] * q.R, q.kl, q.vl);
                }
            }
        }
        const uint64_t end = uni(pbase[SPEC_BP]);
        __syncthreads();
        return end;
    }
    for (uint32_t i = 0; i < n; ++i) {
        const uint64_t g = uni(pbase[i]);
        const uint64_t x = uni(pc[i].x), R = uni(pc[i].R);
        const uint32_t kl = uni(pc[i].kl), vl = uni(pc[i].vl), cnt = uni(pc[i].count);
        if (uni(pc[i].pad) == SP_HOP) {  // hop segment: spans were walked into scratch
            const hg_span* src = a.scratch + (size_t)(q0 + i) * MAX_REC_PIECE;
            for (uint32_t t = tid; t < cnt; t += THREADS)
                if (g + t < a.cap) copy_span(a.spans + g + t, src + t, a.obase);
        } else {
            for (uint32_t t = tid; t < cnt; t += THREADS)
                if (g + t < a.cap) write_span(a.spans, g + t, a.obase + x + t * R, kl, vl);
        }
    }
    const uint64_t end = uni(pbase[SPEC_BP]);
    __syncthreads();
    return end;
}

__device__ __forceinline__ bool rec_ok(uint64_t q, uint64_t len, uint64_t kl, uint64_t vl) {
    return kl <= ~0ull - vl && kl + vl <= len - q - 16 && !((kl >> 32) | (vl >> 32));
}

// Header at absolute q (q + 16 <= len) straight from HBM.
__device__ __forceinline__ void hbm_header(const DecodeArgs& a, uint64_t q, uint64_t& kl,
                                           uint64_t& vl) {
    const uint64_t* p = reinterpret_cast<const uint64_t*>(a.sst + q);
    kl = p[0];
    vl = p[1];
}

// ---- splice repair of a pre-pass batch entered off its predecessor's exit -------
// Pre-pass batch e (pieces [q0, q0 + n)) was resolved from a guessed entry x0
// that is not the exit X of batch e - 1 (both resolved).  Exits are usually
// right even then: a wrong guess follows a self-consistent path (inside a
// zero-byte value every position reads as an empty record; a shifted header
// read can decode as one long record) that joins the true path at some true
// header, after which the two paths are the same walk.  So instead of
// decoding the batch again, wave 0 walks the exact path from X through HBM
// headers (one dependent 16-byte read per record) until it lands on a start of
// the speculative path -- found by a two-pointer sweep over the speculative
// starts, 64 per step (stride pieces arithmetically, walked pieces from their
// scratch spans) -- or on the batch exit.  The exact records before that point
// replace the speculative ones: they go in front of the speculative spans of
// the piece holding the join point (its scratch slot shifted in place; a
// stride piece is written out as spans), the pieces before it are emptied.
// Only this general batch reads these pieces' records (the resolved prefix
// stops before e), so rewriting them needs no cross-workgroup ordering.
// Returns (wave 0) the batch's exact record count; ~0u if the path cannot be
// read, does not join within SPLICE_MAX records, or the joined piece would
// overflow its slot -- the look-back and the general engine then take the
// batch as before.
constexpr uint32_t SPLICE_MAX = 512;  // exact records before the join (LDS: 8 KiB)
struct SpliceArgs {  // what splice_repair needs of DecodeArgs (by value: it is not inlined)
    const uint8_t* sst;
    uint64_t len, stop;
    hg_span* scratch;
    SpecPiece* spiece;
    DecodeCtl* ctl;
    uint32_t sbp, npieces;
};
__device__ __noinline__ uint32_t splice_repair(SpliceArgs a, uint4* ebuf, uint32_t e, uint64_t X,
                                               uint64_t exit_e, uint32_t count_e) {
    // ebuf: SPLICE_MAX exact spans in LDS; returns the new count, or ~0u
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t q0 = e * a.sbp;
    const uint32_t n = min(a.sbp, a.npieces - q0);
    const uint64_t bend = min((uint64_t)(q0 + n) * PIECE, a.stop);
    // piece records: lane i holds piece i's
    SpecPiece pr{};
    if (lane < n) pr = a.spiece[q0 + lane];
    const uint32_t pcnt = lane < n ? pr.count : 0u;
    auto piece_pos = [&](uint32_t pi, uint32_t j) -> uint64_t {  // start of record j of piece pi
        const uint64_t x = __shfl(pr.x, (int)pi, 64), R = __shfl(pr.R, (int)pi, 64);
        const uint32_t kind = __shfl(pr.pad, (int)pi, 64);
        if (kind == SP_HOP) return a.scratch[(size_t)(q0 + pi) * MAX_REC_PIECE + j].off;
        return x + (uint64_t)j * R;
    };
    // speculative sweep: chunk = records [lo, lo + 64) of piece pi
    uint32_t pi = 0, lo = 0;
    auto next_nonempty = [&](uint32_t from) -> uint32_t {
        const unsigned long long m = __ballot(lane >= from && lane < n && pcnt > 0);
        return m ? (uint32_t)(__ffsll((long long)m) - 1) : n;
    };
    pi = next_nonempty(0);
    uint64_t pos = ~0ull, cmax = ~0ull;
    auto load_chunk = [&]() {
        if (pi >= n) {
            pos = ~0ull;
            cmax = ~0ull;
            return;
        }
        const uint32_t c = __shfl(pcnt, (int)pi, 64);
        pos = lo + lane < c ? piece_pos(pi, lo + lane) : ~0ull;
        const uint32_t last = min(lo + 63u, c - 1u);
        cmax = __shfl(pos, (int)(last - lo), 64);
    };
    load_chunk();
    uint64_t p = X;
    uint32_t E = 0, jpi = n, jlo = 0;  // join: piece jpi, record jlo (jpi == n: at the exit)
    for (;;) {
        if (p >= bend) {
            if (p != exit_e) return ~0u;
            jpi = n;
            break;
        }
        while (pi < n && cmax < p) {  // every start in the chunk is before p
            lo += 64;
            if (lo >= __shfl(pcnt, (int)pi, 64)) {
                pi = next_nonempty(pi + 1);
                lo = 0;
            }
            load_chunk();
        }
        const unsigned long long m = __ballot(pos == p);
        if (m) {
            jpi = pi;
            jlo = lo + (uint32_t)(__ffsll((long long)m) - 1);
            break;
        }
        if (E == SPLICE_MAX || p + 16 > a.len) return ~0u;
        uint64_t kl = 0, vl = 0;
        if (lane == 0) {
            const uint64_t* hp = reinterpret_cast<const uint64_t*>(a.sst + p);
            kl = hp[0];
            vl = hp[1];
        }
        kl = __shfl(kl, 0, 64);
        vl = __shfl(vl, 0, 64);
        if (kl > ~0ull - vl || kl + vl > a.len - p - 16 || ((kl >> 32) | (vl >> 32))) return ~0u;
        if (lane == 0) ebuf[E] = make_uint4((uint32_t)p, (uint32_t)(p >> 32), (uint32_t)kl, (uint32_t)vl);
        ++E;
        p += 16 + kl + vl;
    }
    // the join piece: exact spans, then its speculative spans from jlo on
    const uint32_t tp = jpi < n ? jpi : n - 1;           // piece that takes the exact spans
    const uint32_t tc = __shfl(pcnt, (int)tp, 64);
    const uint32_t keep0 = jpi < n ? jlo : tc;           // its speculative spans kept: [keep0, tc)
    const uint32_t keep = tc - keep0;
    if (E + keep > MAX_REC_PIECE) return ~0u;
    uint32_t before = 0;                                 // speculative records dropped
    {
        const uint32_t c = lane < tp ? pcnt : 0u;
        before = wave_sum<uint32_t>(c) + keep0;
    }
    hg_span* slot = a.scratch + (size_t)(q0 + tp) * MAX_REC_PIECE;
    const uint32_t tkind = __shfl(pr.pad, (int)tp, 64);
    if (keep && tkind != SP_HOP) {  // a stride piece: write its kept records out as spans
        const uint64_t x = __shfl(pr.x, (int)tp, 64), R = __shfl(pr.R, (int)tp, 64);
        const uint32_t kl = __shfl(pr.kl, (int)tp, 64), vl = __shfl(pr.vl, (int)tp, 64);
        for (uint32_t j = lane; j < keep; j += 64)
            write_span(slot, E + j, x + (uint64_t)(keep0 + j) * R, kl, vl);
    } else if (keep && E < keep0) {  // shift down, ascending (no chunk reads what an earlier one wrote)
        for (uint32_t j0 = 0; j0 < keep; j0 += 64) {
            uint4 v = make_uint4(0, 0, 0, 0);
            if (j0 + lane < keep) v = *reinterpret_cast<const uint4*>(slot + keep0 + j0 + lane);
            if (j0 + lane < keep) *reinterpret_cast<uint4*>(slot + E + j0 + lane) = v;
        }
    } else if (keep && E > keep0) {  // shift up, descending
        for (uint32_t j1 = keep; j1 > 0;) {
            const uint32_t j0 = j1 > 64 ? j1 - 64 : 0;
            uint4 v = make_uint4(0, 0, 0, 0);
            if (j0 + lane < j1) v = *reinterpret_cast<const uint4*>(slot + keep0 + j0 + lane);
            if (j0 + lane < j1) *reinterpret_cast<uint4*>(slot + E + j0 + lane) = v;
            j1 = j0;
        }
    }
    for (uint32_t j = lane; j < E; j += 64) *reinterpret_cast<uint4*>(slot + j) = ebuf[j];
    if (lane <= tp) {  // pieces before the join piece hold nothing now
        SpecPiece o = pr;
        o.count = lane == tp ? E + keep : 0u;
        o.pad = SP_HOP;
        a.spiece[q0 + lane] = o;
    }
    if (lane == 0) atomicAdd(&a.ctl->repairs, 1u);
    return count_e - before + E;
}

template <bool DIAG>
__device__ void decode_body(const DecodeArgs& a, uint32_t blk) {
    __shared__ DecodeSmem s;
    const uint32_t tid = threadIdx.x;
    uint64_t t_start = 0;
    uint32_t* dg = nullptr;
#define HG_STAMP(slot)                                                                      \
    do {                                                                                    \
        if (DIAG && tid == 0) dg[slot] = (uint32_t)(__builtin_amdgcn_s_memtime() - t_start); \
    } while (0)

    // ---- spans of the pre-pass's resolved prefix (workgroup e = batch e) ----------
    const uint32_t fb = first_bad(a.ctl, a.nspec);
    // Only batches whose whole general batch is resolved: the general engine
    // redoes a general batch that holds an unresolved pre-pass batch (and
    // reuses the scratch spans of its pieces meanwhile).
    if (blk < fb && min((blk / a.q + 1) * a.q, a.nspec) <= fb) {
        const uint32_t e = blk;
        const uint32_t ep0 = e * a.sbp;
        const uint32_t enp = min(a.sbp, a.npieces - ep0);
        const uint64_t g = emit_spec_batch(s, a, e, ep0, enp);
        if (tid == 0 && e == a.nspec - 1) {  // the whole file resolved: report it
            hg_decode_result r;
            r.n_records = g;
            r.kind = HG_OK;
            r.reserved = 0;
            r.err_offset = a.range ? a.obase + a.sbatch[e].exit : 0;
            *a.result = r;
        }
    }
    if (fb >= a.nspec || blk >= a.nbatches) return;  // nothing left for the general engine
    if (tid == 0) s.batch = atomicAdd(a.ticket, 1u);
    __syncthreads();
    if (min((s.batch + 1) * a.q, a.nspec) <= fb) {
        // Resolved by the pre-pass (spans written above): publish its INCL.
        if (tid < 64) {
            const uint32_t b0 = s.batch;
            const uint32_t e1 = min((b0 + 1) * a.q, a.nspec);  // first batch after it
            const uint64_t gend = spec_base(a, e1);
            const uint64_t g0 = spec_base(a, b0 * a.q);
            if (tid == 0) {
                const uint64_t ex = a.sbatch[e1 - 1].exit;
                st_agent(&a.status[2 * b0 + 1], pack_status(ST_INCL, 0, gend));
                st_agent(&a.status[2 * b0], pack_status(ST_INCL, (uint32_t)(gend - g0), ex));
                __hip_atomic_fetch_add(&a.ctl->progress, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
        return;
    }
    const uint32_t b = s.batch;
    const uint32_t p0 = b * a.bp;
    const uint32_t np = min(a.bp, a.npieces - p0);
    if (DIAG) {
        t_start = __builtin_amdgcn_s_memtime();
        dg = a.diag + (size_t)b * DIAG_WORDS;
    }
    // Pre-resolved: every pre-pass batch in this general batch verified and
    // chained to its neighbour (the pre-pass resolves batches past the first
    // unresolved one too).  Publish that result at once, look back, and if the
    // looked-back entry is the pre-pass entry emit from the summaries -- no
    // table bytes are read.  Otherwise the general engine below runs from the
    // exact entry.
    uint64_t x_exact = X_UNKNOWN;
    {
        const uint32_t e0 = b * a.q, e1 = min((b + 1) * a.q, a.nspec);
        if (tid < 64) {
            // Each pre-pass batch must be resolved and entered at its
            // predecessor's exit; one entered elsewhere is spliced onto that
            // exit (splice_repair).  The first one's predecessor belongs to the
            // previous general batch: its exit is only a better guess of our
            // entry (the look-back below checks it).
            bool good = true;
            uint64_t cnt = 0, P0 = a.sbatch[e0].x0;
            for (uint32_t e = e0; e < e1 && good; ++e) {
                const SpecBatch sbe = a.sbatch[e];
                uint32_t c = sbe.count;
                good = sbe.ok != 0;
                if (good && e > 0) {
                    const SpecBatch sbp = a.sbatch[e - 1];
                    if (sbe.x0 != sbp.exit && (sbp.ok || e > e0)) {
                        const SpliceArgs sa{a.sst, a.len, a.stop, a.scratch, a.spiece_rw, a.ctl, a.sbp,
                                            a.npieces};
                        const uint32_t cr =
                            HG_SPLICE && sbp.ok
                                ? splice_repair(sa, reinterpret_cast<uint4*>(s.data64), e, sbp.exit,
                                                sbe.exit, c)
                                : ~0u;
                        if (cr != ~0u) {
                            c = cr;
                            if (e == e0) P0 = sbp.exit;
                        } else if (e > e0) {
                            good = false;
                        }
                    }
                }
                cnt += c;
            }
            if (tid == 0) {
                s.pred_ok = good;
                s.gk = cnt;
                s.xk = P0;
                s.exitk = a.sbatch[e1 - 1].exit;
            }
        }
        __syncthreads();
        if (uni(s.pred_ok)) {
            const uint64_t P0 = uni(s.xk), ptot = uni(s.gk), pex = uni(s.exitk);
            const uint64_t bb = (uint64_t)p0 * PIECE;
            if (tid == 0) {
                const uint32_t xrel = P0 < bb + (uint64_t)np * PIECE ? (uint32_t)(P0 - bb) : NONE_REL;
                st_agent(&a.status[2 * b + 1], pack_status(ST_AGG, xrel, 0));
                st_agent(&a.status[2 * b], pack_status(ST_AGG, (uint32_t)ptot, pex));
            }
            __syncthreads();
            if (tid < 64) {
                uint32_t spins = 0;
                LookbackOut lb = lookback(a, b, spins);
                if (tid == 0) {
                    s.xk = lb.x;
                    s.gk = lb.g;
                    s.err_kind = lb.err;
                }
            }
            __syncthreads();
            const uint64_t xk0 = uni(s.xk), gk0 = uni(s.gk);
            if (uni(s.err_kind) == HG_OK && xk0 == P0) {
                if (tid == 0) {
                    st_agent(&a.status[2 * b + 1], pack_status(ST_INCL, 0, gk0 + ptot));
                    st_agent(&a.status[2 * b], pack_status(ST_INCL, (uint32_t)ptot, pex));
                    __hip_atomic_fetch_add(&a.ctl->progress, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    if (b == a.nbatches - 1) {
                        hg_decode_result r;
                        r.n_records = gk0 + ptot;
                        r.kind = HG_OK;
                        r.reserved = 0;
                        r.err_offset = a.range ? a.obase + pex : 0;
                        *a.result = r;
                    }
                }
                emit_spec_range(s, a, p0, np, gk0);
                return;
            }
            if (uni(s.err_kind) == HG_OK) x_exact = xk0;  // wrong entry: decode from the exact one
        }
        __syncthreads();  // s.pred_ok / s.xk are reused below
    }
    if (tid < np) {
        s.halo[tid] = load16(a, (uint64_t)(p0 + tid + 1) * PIECE);
        piece_tags(a)[p0 + tid] = 0;  // the general engine takes these pieces' scratch slots
    }
    if (tid == 0) {  // is the predecessor batch's exit already published?
        s.pred_ok = b == 0;
        s.pred_exit = a.entry;
        if (b > 0) {
            unsigned long long v0 = ld_agent(&a.status[2 * (b - 1)]);
            unsigned long long v1 = ld_agent(&a.status[2 * (b - 1) + 1]);
            if (st_flag(v0) == st_flag(v1) && (st_flag(v0) == ST_AGG || st_flag(v0) == ST_INCL)) {
                s.pred_ok = 1;
                s.pred_exit = st_val(v0);
            }
        }
    }
    hg_span* const scratch = a.scratch + (size_t)p0 * MAX_REC_PIECE;
    const uint64_t bbase = (uint64_t)p0 * PIECE;

    // Pass 0 is speculative (entry guessed, spans to scratch, stride pieces
    // summarised).  Pass 1 runs only when the guess was wrong or the guessed
    // path fails: exactly from the looked-back entry, emitting directly, until
    // a piece's exact exit equals its speculative exit — from there on the
    // speculative pieces are exact (a piece's path depends only on its entry)
    // and only their record base moves.
    uint64_t X0 = X_UNKNOWN, x = X_UNKNOWN, total = 0, gk = 0, xk = 0, errpos = 0, gi = 0;
    uint64_t gres = 0;  // record index of piece `resume`
    int32_t kind = HG_OK, perr = HG_OK;
    bool spec_ok = true, redo = false;
    uint32_t nstride = 0, ngen = 0, nserial = 0, nshort = 0, resume = 0, nredo = 0;
    if (DIAG && tid == 0) {
        for (uint32_t q = 0; q < NPROF; ++q) s.prof[q] = 0;
        s.plast = __builtin_amdgcn_s_memtime();
    }
    uint32_t rounds_acc = 0;
    __syncthreads();
    if (uni(s.pred_ok)) x = uni(s.pred_exit);
    if (x_exact != X_UNKNOWN) x = x_exact;
    // Lead-in: with no published entry, pass 0 first walks the piece before
    // the batch (its own entry guessed, spans to this batch's scratch slot 0,
    // rewritten by piece 0) and takes its exit as the batch's guessed entry.
    // A wrong guess there has almost always re-joined the true path by the
    // piece end, so the batch's AGG chains and its successors need not wait
    // for an exact redo (each redo is one serial hop of the look-back chain).
    // Same call site as the batch's pieces: no second copy of the engine.
    const bool lead0 = HG_LEADIN && x == X_UNKNOWN && p0 > 0;
    if (lead0 && tid == 0) s.lead_halo = load16(a, (uint64_t)p0 * PIECE);
    uint4 v[GPT];
    load_piece(a, lead0 ? p0 - 1 : p0, v);
#pragma nounroll
    for (uint32_t pass = 0;; ++pass) {
        gi = gk;
        uint32_t prev_count = 0;
        uint32_t prev_mode = 0;  // the previous piece's mode (stride attempts while it is <= 1)
        uint32_t i = 0;
        bool lead = pass == 0 && lead0;
#pragma nounroll
        for (; i < np;) {
            const uint32_t pi = lead ? p0 - 1 : p0 + i;
            if (pass == 1) load_piece(a, pi, v);  // (rare pass: no prefetch, fewer VGPRs)
            stage_piece(s, v, i, lead);
            if (pass == 0 && (lead || i + 1 < np)) load_piece(a, pi + 1, v);  // in flight meanwhile
            PieceSum ps;
            uint64_t ex;
            uint32_t mode = 0;
            hg_span* out = pass ? a.spans : scratch + (size_t)i * MAX_REC_PIECE;
            const int32_t e = piece_path<DIAG>(s, a, pi, x, pass == 1, prev_count <= SHORT_WALK,
                                               out, pass ? a.cap : ~0ull, pass ? gi : 0, ps, ex, mode,
                                               prev_mode <= 1);
            if (lead) {  // the lead-in only supplies the guessed entry
                lead = false;
                x = e == HG_OK ? ex : X_UNKNOWN;
                continue;
            }
            if (HG_EMPTY_SPEC && pass == 0 && e == E_NO_GUESS) {
                // No record start found in this piece and no entry known yet:
                // speculate that it holds none (records longer than a piece
                // leave many pieces without a start).  The batch's guessed
                // entry becomes the first guess found in a later piece; the
                // look-back verifies it like any other guess, and the exact
                // pass never re-joins on these pieces (their exit is unknown).
                ps.x = X_UNKNOWN;
                ps.exit = X_UNKNOWN;
                ps.R = 0;
                ps.kl = ps.vl = 0;
                ps.count = 0;
                ps.kind = PK_EMPTY;
                if (tid == 0) s.sum[i] = ps;
                prev_count = 0;
                ++i;
                continue;
            }
            if (pass == 0 && X0 == X_UNKNOWN) X0 = x;
            nstride += mode == 1;
            ngen += mode == 2;
            nserial += mode == 3;
            nshort += mode == 4;
            if (DIAG && mode == 2) rounds_acc += s.rounds;
            nredo += pass;
            prev_count = ps.count;
            prev_mode = mode;
            if (e != HG_OK) {
                if (pass == 0) {  // the guessed path fails: the exact pass reports it
                    spec_ok = false;
                } else {
                    kind = e;
                    errpos = s.err_pos;
                    gi += ps.count;
                }
                break;
            }
            if (pass == 0 && tid == 0) s.sum[i] = ps;
            gi += ps.count;
            x = ex;
            if (pass == 1 && spec_ok && ex == uni(s.sum[i].exit)) {  // re-joined the speculative path
                ++i;
                break;
            }
            ++i;
        }
        resume = pass == 0 ? 0 : i;
        gres = gi;
        if (pass == 1) {
            if (kind == HG_OK && spec_ok && resume < np) {
                for (uint32_t j = resume; j < np; ++j) gi += uni(s.sum[j].count);
                x = uni(s.sum[np - 1].exit);
            }
            total = gi - gk;
            break;
        }
        total = gi;  // gk == 0 in pass 0
        HG_STAMP(D_T_SPEC);
        if (spec_ok && tid == 0) {
            const uint32_t xrel =
                X0 < bbase + (uint64_t)np * PIECE ? (uint32_t)(X0 - bbase) : NONE_REL;
            st_agent(&a.status[2 * b + 1], pack_status(ST_AGG, xrel, 0));
            st_agent(&a.status[2 * b], pack_status(ST_AGG, (uint32_t)total, x));
        }
        HG_STAMP(D_T_AGG);
        if (tid < 64) {  // look-back (wave 0)
            uint32_t spins = 0;
            LookbackOut lb = lookback(a, b, spins);
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
        perr = uni(s.err_kind);
        xk = uni(s.xk);
        gk = uni(s.gk);
        if (perr != HG_OK) {  // an earlier batch failed: propagate, emit nothing
            kind = perr;
            errpos = s.err_pos;
            total = 0;
            resume = np;
            break;
        }
        if (spec_ok && xk == X0) {
            gres = gk;
            break;
        }
        redo = true;
        x = xk;
    }
    // ---- publish, then emit the speculative pieces from `resume` on -------------------
    if (tid == 0) {
        if (kind == HG_OK) {
            st_agent(&a.status[2 * b + 1], pack_status(ST_INCL, 0, gk + total));
            st_agent(&a.status[2 * b], pack_status(ST_INCL, (uint32_t)total, x));
        } else {
            st_agent(&a.status[2 * b + 1], pack_status(ST_ERR, 0, gk + total));
            st_agent(&a.status[2 * b], pack_status(ST_ERR, (uint32_t)(kind + 16), errpos));
        }
        __hip_atomic_fetch_add(&a.ctl->progress, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (kind == HG_OK && spec_ok) {
        uint64_t go = gres;
        for (uint32_t i = resume; i < np; ++i) {
            PieceSum ps = s.sum[i];
            ps.x = uni(ps.x);
            ps.R = uni(ps.R);
            ps.kl = uni(ps.kl);
            ps.vl = uni(ps.vl);
            ps.count = uni(ps.count);
            ps.kind = uni(ps.kind);
            if (ps.kind == PK_STRIDE) {
                for (uint32_t t = tid; t < ps.count; t += THREADS)
                    if (go + t < a.cap)
                        write_span(a.spans, go + t, a.obase + ps.x + t * ps.R, ps.kl, ps.vl);
            } else if (ps.kind == PK_SCRATCH) {
                const hg_span* src = scratch + (size_t)i * MAX_REC_PIECE;
                for (uint32_t t = tid; t < ps.count; t += THREADS)
                    if (go + t < a.cap) copy_span(a.spans + go + t, src + t, a.obase);
            }
            go += ps.count;
        }
    }
    HG_STAMP(D_T_END);
    if (DIAG && tid == 0) {
        dg[D_NSTRIDE] = nstride;
        dg[D_NGEN] = ngen;
        dg[D_NSERIAL] = nserial;
        dg[D_GUESS] = (X0 != X_UNKNOWN ? 1u : 0u) | (s.pred_ok ? 2u : 0u) | ((xk == X0) ? 4u : 0u);
        dg[D_COUNT] = (uint32_t)total;
        dg[D_FLAGS] = (perr != HG_OK ? 2u : 0u) | (kind != HG_OK ? 4u : 0u) | (spec_ok ? 8u : 0u);
        dg[D_REDO] = redo ? 1u + nredo : 0u;
        dg[D_C_PREP] = s.prof[0] + s.prof[1] + s.prof[2];
        dg[D_C_RELAX] = s.prof[3] + s.prof[4];
        for (uint32_t q = 0; q < NPROF; ++q) dg[16 + q] = s.prof[q];
        dg[D_ROUNDS] = rounds_acc;
        dg[D_NSHORT] = nshort;
    }
#undef HG_STAMP
    // ---- the last batch reports the whole-file result --------------------------------
    if (tid == 0 && b == a.nbatches - 1) {
        hg_decode_result r;
        r.n_records = gk + total;
        r.kind = kind;
        r.reserved = 0;
        r.err_offset = kind != HG_OK ? a.obase + errpos : (a.range ? a.obase + x : 0);
        *a.result = r;
    }
}

// Speculative entry of a range that starts inside a table (a single huge
// table split over devices): the first record start at or after
// `stop`, found by walking the piece [begin, stop) (one piece, begin = stop -
// 16 KiB, or 0) from a guessed entry -- the general engine's lead-in.  The
// caller verifies the guess against the exact exit of the previous range and
// redoes the range from that exit when they differ.  ~0 if nothing was found.
__global__ __launch_bounds__(THREADS, 4) void decode_guess_kernel(DecodeArgs a, uint64_t* out) {
    __shared__ DecodeSmem s;
    uint4 v[GPT];
    load_piece(a, 0, v);
    if (threadIdx.x == 0) s.lead_halo = load16(a, PIECE);
    stage_piece(s, v, 0, true);
    PieceSum ps;
    uint64_t ex = 0, X = a.obase == 0 ? 0 : X_UNKNOWN;  // a table's first byte is a record start
    uint32_t mode = 0;
    const int32_t e = piece_path<false>(s, a, 0, X, false, true, a.scratch, ~0ull, 0, ps, ex, mode);
    if (threadIdx.x == 0) *out = e == HG_OK ? a.obase + ex : ~0ull;
}

template <bool DIAG>
#ifndef HG_DEC_WAVES
#define HG_DEC_WAVES 4
#endif
__global__ __launch_bounds__(THREADS, HG_DEC_WAVES) void decode_kernel(DecodeArgs a) {
    decode_body<DIAG>(a, blockIdx.x);
}

// ---- stride pre-pass ---------------------------------------------------------------
// decode_spec_kernel: one workgroup per SPEC_BP pieces, no inter-workgroup
// communication: guesses the batch entry (stride_guess), verifies every piece
// as a stride run from the previous piece's exit and records per-piece
// summaries.  Pure streaming (register prefetch of the next piece).  A batch
// that is not one verified chain of stride runs is left to decode_kernel.
// ---- hop mode (large records): read headers, not tables ---------------------------
// A batch whose first piece has no stride run but whose records are large
// (few header candidates in the first piece: HOP_MAX_CAND) is
// decoded by hopping from header to header in HBM: decode output depends on
// the 16-byte headers alone, so with ~2 KiB records (BASELINE cfg 4) only
// ~1 cache line per record is touched instead of the whole table
// (tools/probes/read_probe.hip: header-only reads of 1 KiB records take
// 1/8 of the full sweep).  The batch is cut into 64 KiB segments:
//   A. one wave per segment stages a HOP_WIN-byte window at the segment start,
//      finds header candidates (zero-mask filter) and takes the first one whose
//      next HOP_CHECK headers (read from HBM) are readable records;
//   B. one lane per segment walks from its guess to the segment end, writing
//      spans to the segment's scratch (one dependent 16-byte load per record);
//   C. thread 0 stitches: a segment whose guess is not its predecessor's exit
//      (a wrong guess, or no record starts in its window) is re-walked from
//      that exit.  So the batch's spans are exact given its entry, like a
//      stride batch's, and the pre-pass links check the entries as usual.
#ifndef HG_HOP_SEG
#define HG_HOP_SEG 4
#endif
constexpr uint32_t HOP_SEG_PIECES = HG_HOP_SEG;           // 64 KiB segments
constexpr uint32_t HOP_SEGS = SPEC_BP / HOP_SEG_PIECES;   // per pre-pass batch, at most
// (Round 5: only when the pre-pass grid fits the resident workgroups -- see
// hop_wide_cand.)  Batches whose piece 0 shows at most HOP_WIDE_CAND candidate run ends walk
// HOP_WIDE-piece (128 KiB) segments: half the guesses for chains twice as
// long (a walk takes up to HOP_MAX_RECS records per 4 pieces).  Shorter
// segments measured slower on every hop shape (cfg 4, 32 x 64 MiB: 32 KiB
// 0.665 -> 0.75 ms, 16 KiB 1.27 ms); 128 KiB ones for every hop batch with the
// record limit unscaled cost 400-1200 B records 3.7x (their walks gave up).
// Thresholds, same box, 2 rounds (tools/multi_table.py, decode_variants.py):
// 64 KiB always: cfg 4 0.662 ms, 8 B-4 KiB 0.091, 0-16 KiB 0.210, 0-64 KiB
// 0.214, 400-1200 B 0.166; <= 12: 0.507-0.582 / 0.084 / 0.199 / 0.204 / 0.162;
// <= 16: 0.501-0.523 / 0.084 / 0.198 / 0.201 / 0.165; <= 24: 0.489 / 0.085-
// 0.088 / 0.198 / 0.202 / 0.156.
#ifndef HG_HOP_WIDE_CAND
#define HG_HOP_WIDE_CAND 24
#endif
#ifndef HG_HOP_WIDE
#define HG_HOP_WIDE 8
#endif
constexpr uint32_t HOP_WIDE_CAND = HG_HOP_WIDE_CAND;
constexpr uint32_t HOP_WIDE = HG_HOP_WIDE;
static_assert(HOP_WIDE % HOP_SEG_PIECES == 0 && HOP_WIDE <= SPEC_BP, "hop segment geometry");
constexpr uint32_t HOP_WIN = 4096;                        // guess window (bytes)
constexpr uint32_t HOP_CHECK = 3;                         // hops a guess must survive
#ifndef HG_HOP_MAX_CAND
#define HG_HOP_MAX_CAND 32  // candidate run ends in piece 0 (~1-2 per record): hop >= ~0.5-1 KiB records
#endif
constexpr uint32_t HOP_MAX_CAND = HG_HOP_MAX_CAND;        // large-record test on piece 0
constexpr uint32_t HOP_MAX_RECS = 128;  // a segment walk gives up past this (small records)
constexpr uint32_t HOP_MAX_REDO = 2;    // stitch re-walks per batch before giving up
constexpr uint32_t HOP_TRIES = 8;                         // candidates tried per lane
constexpr uint64_t NO_HOP = ~0ull;

constexpr uint32_t LW_ZM_WORDS = 64 * 64 / 16 + 8;  // granule masks per lane-walk chunk (+ halo)
struct SpecSmem {
    uint64_t data64[(PIECE + 512) / 8];  // a piece, four HOP_WIN + 16 byte windows, or lane-walk chunk buffers
    uint4 halo[SPEC_BP];
    uint32_t guess;
    uint64_t hg[HOP_SEGS];    // guessed segment entries (NO_HOP: none)
    uint64_t hd[HOP_SEGS];    // HOP_CHECK-record span of the guess
    uint64_t hexit[HOP_SEGS];
    uint32_t hcnt[HOP_SEGS];
    uint32_t hdead[HOP_SEGS];
    uint32_t hok;
    uint64_t hx, ht;          // batch exit and records after stitching
    uint32_t hcode;           // SpecBatch.pad: how the batch went (SB_*)
    // lane-walk mode (lw_batch): per-wave chunk masks and guess / chain
    // scratch, quarter summaries of the last two stitching rounds
    alignas(8) uint16_t lw_zm[NW][LW_ZM_WORDS];
    uint32_t lw_sg[THREADS];
    uint8_t lw_tg[THREADS];
    uint64_t lw_wx[2][NW];
    uint64_t lw_wexit[2][NW];
    uint32_t lw_wcnt[2][NW];
    uint32_t lw_wbad[2][NW];
    uint64_t lw_px[NW][SPEC_BP / NW];  // per wave: entries / records of its quarter's pieces
    uint32_t lw_pc[NW][SPEC_BP / NW];
    uint32_t lw_prof[8];      // diagnostics (a.sdiag): cycles per lane-walk phase, see LW_STAMP
    uint64_t lw_last;
};

// Span of the HOP_CHECK records after the (valid) record at p, or 0 if one
// of them cannot be read.  Reaching the end of the file exactly passes.
__device__ uint64_t hop_check(const DecodeArgs& a, uint64_t p, uint64_t kl, uint64_t vl) {
    uint64_t q = p + 16 + kl + vl;
    for (uint32_t h = 0; h < HOP_CHECK; ++h) {
        if (q == a.len) return q - p;
        if (q + 16 > a.len || q + 16 > a.rlen) return 0;
        hbm_header(a, q, kl, vl);
        if (!rec_ok(q, a.len, kl, vl)) return 0;
        q += 16 + kl + vl;
    }
    return q - p;
}

// Exact walk of [x, end) through HBM headers: spans to out[0..), count,
// exit (first start >= end) and whether a record cannot be read or the
// segment holds more than maxr records (dead: the batch is left to the
// general engine, which reads the table instead).
__device__ void hop_walk(const DecodeArgs& a, uint64_t x, uint64_t end, hg_span* out,
                         uint32_t maxr, uint32_t& cnt, uint64_t& exit, uint32_t& dead) {
    uint32_t n = 0;
    uint64_t cur = x;
    dead = 0;
    while (cur < end) {
        if (n == maxr) {
            dead = 1;
            break;
        }
        uint64_t kl, vl;
        if (cur + 16 > a.len || cur + 16 > a.rlen) {
            dead = 1;
            break;
        }
        hbm_header(a, cur, kl, vl);
        if (!rec_ok(cur, a.len, kl, vl)) {
            dead = 1;
            break;
        }
        write_span(out, n, cur, kl, vl);
        ++n;
        cur += 16 + kl + vl;
    }
    cnt = n;
    exit = cur;
}

// Phase A for segment starting at S (absolute), by one wave, window staged in
// w (HOP_WIN + 16 bytes).  Returns (guess, span) in every lane.  Each lane
// tries the candidates of its 64 bytes that END a run of candidates first (a
// genuine header with short lengths also passes the filter 1-3 bytes to its
// left; a record read from such a shifted position can still chain into a
// true header far ahead and pass the check, which made a batch's entry
// wrong), then the others; all-zero headers are skipped (inside zero-byte
// values every position reads as an empty record and chains on).
#ifndef HG_HOP_Z16
#define HG_HOP_Z16 1  // 0: run ends over every candidate (round-3 rule, A/B)
#endif
__device__ void hop_guess(const DecodeArgs& a, const uint8_t* w, uint64_t S, uint64_t& guess,
                          uint64_t& span) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t rem = a.len - S;
    const bool any_valid = rem >= 16;
    const uint64_t plim64 = any_valid ? rem - 16 : 0;
    const uint32_t plim = plim64 < 0xFFFFFFFFull ? (uint32_t)plim64 : 0xFFFFFFFFu;
    const uint32_t clen = rem < HOP_WIN ? (uint32_t)rem : HOP_WIN;
    unsigned long long best = ~0ull;  // (position << 40) | span
    uint64_t cm = 0;
#pragma unroll
    for (uint32_t j = 0; j < 4; ++j)
        cm |= (uint64_t)filter_bits(w, lane * 4 + j, a.hz, clen, plim, any_valid) << (16 * j);
    uint64_t nb = filter_bits(w, lane * 4 + 4, a.hz, clen, plim, any_valid) & 1u;
    // Positions where 16 zero bytes start are dropped before the run ends are
    // taken: a header followed by zero bytes -- a tombstone (vlen 0) whose key
    // starts with zero bytes -- merges with them into one run whose end reads
    // as an all-zero header (skipped), so the tombstone was never tried and the
    // guess landed on the record after it (one record lost per such batch
    // entry, repaired later at the cost of a look-back chain: cfg 4 0.27 ->
    // 0.48 ms in round 3).
    if (HG_HOP_Z16) {
        uint64_t zl = 0;
        uint32_t zh = 0;
#pragma unroll
        for (uint32_t j = 0; j < 4; ++j)
            zl |= (uint64_t)zmask16(*reinterpret_cast<const uint4*>(w + (lane * 4 + j) * 16)) << (16 * j);
        zh = zmask16(*reinterpret_cast<const uint4*>(w + (lane * 4 + 4) * 16));
#pragma unroll
        for (uint32_t pw = 1; pw < 16; pw *= 2) {  // bit j <=> bytes j .. j+15 are zero
            zl &= (zl >> pw) | ((uint64_t)zh << (64 - pw));
            zh &= zh >> pw;
        }
        cm &= ~zl;
        nb &= ~(uint64_t)(zh & 1u);
    }
    const uint64_t runend = cm & ~((cm >> 1) | (nb << 63));
    uint64_t c = runend;
    uint32_t tries = 0;
#pragma unroll 1
    for (uint32_t pass = 0; pass < 2 && best == ~0ull; ++pass) {
        if (pass) c = cm & ~runend;
        while (c && tries < HOP_TRIES) {
            const uint32_t p = lane * 64 + (uint32_t)(__ffsll((long long)c) - 1);
            c &= c - 1;
            ++tries;
            uint64_t kl, vl;
            lds_header(w, p, kl, vl);
            if ((kl | vl) == 0 || !rec_ok(S + p, a.len, kl, vl)) continue;
            const uint64_t d = hop_check(a, S + p, kl, vl);
            if (d) {
                best = ((unsigned long long)p << 40) | (d < V40 ? d : V40);
                break;
            }
        }
    }
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
        const unsigned long long o = __shfl_xor(best, d, 64);
        best = o < best ? o : best;
    }
    guess = best == ~0ull ? NO_HOP : S + (best >> 40);
    span = best == ~0ull ? 0 : (best & V40);
}

// The hop-mode batch [p0, p0 + np): all threads call it.  On success fills
// sp[] (SP_HOP pieces: segment entry and count on its first piece) and
// returns true with X0 = entry, X = exit, total = records.
__device__ bool hop_batch(SpecSmem& s, const DecodeArgs& a, uint32_t p0, uint32_t np,
                          SpecPiece* sp, uint64_t& X0, uint64_t& X, uint64_t& total) {
    const uint32_t tid = threadIdx.x, wid = tid >> 6, lane = tid & 63u;
    const uint64_t bend = min((uint64_t)(p0 + np) * PIECE, a.stop);
    // Large records?  Piece 0 is still staged: count its header candidates
    // (a record start and its shifts pass the zero-byte filter, ~4 per record
    // for short keys/values).  At most HOP_MAX_CAND (~512 B per record) -> hop.
    {
        const uint64_t base = (uint64_t)p0 * PIECE;
        const uint64_t rem = a.len - base;
        const bool any_valid = rem >= 16;
        const uint64_t plim64 = any_valid ? rem - 16 : 0;
        const uint32_t plim = plim64 < 0xFFFFFFFFull ? (uint32_t)plim64 : 0xFFFFFFFFu;
        const uint32_t clen = piece_clen(a, base);
        const uint8_t* data = reinterpret_cast<const uint8_t*>(s.data64);
        // count RUN ENDS of candidates: a genuine header with small lengths
        // also passes the filter 1-3 bytes to its left, zero key bytes add
        // runs of their own; the last position of each run is ~one per record
        uint32_t nc = 0;
        uint32_t c = filter_bits(data, tid * GPT, a.hz, clen, plim, any_valid);
#pragma unroll
        for (uint32_t j = 0; j < GPT; ++j) {
            const uint32_t nxt = (j + 1 < GPT || tid + 1 < THREADS)
                                     ? filter_bits(data, tid * GPT + j + 1, a.hz, clen, plim, any_valid)
                                     : 0u;
            nc += __popc(c & ~((c >> 1) | ((nxt & 1u) << 15)));
            c = nxt;
        }
        nc = wave_sum<uint32_t>(nc);
        if (tid == 0) s.hcnt[0] = 0;
        __syncthreads();
        if (lane == 0) atomicAdd(&s.hcnt[0], nc);
        __syncthreads();
        if (s.hcnt[0] > HOP_MAX_CAND) {
            s.hcode = SB_HOP_SMALL;
            return false;
        }
    }
    // pieces per segment (uniform): wide segments for sparse candidates
    const uint32_t hsp = uni(s.hcnt[0]) <= a.hop_wide ? HOP_WIDE : HOP_SEG_PIECES;
    const uint32_t maxr = HOP_MAX_RECS / HOP_SEG_PIECES * hsp;
    const uint32_t nseg = (np + hsp - 1) / hsp;
    uint8_t* w = reinterpret_cast<uint8_t*>(s.data64) + wid * (HOP_WIN + 16);
    // A: guesses, four segments per round (one per wave)
    for (uint32_t r = 0; r * NW < nseg; ++r) {
        const uint32_t k = r * NW + wid;
        const uint64_t S = (uint64_t)(p0 + k * hsp) * PIECE;
        __syncthreads();
        if (k < nseg) {
#pragma unroll
            for (uint32_t j = 0; j < 4; ++j)
                *reinterpret_cast<uint4*>(w + (j * 64 + lane) * 16) =
                    load16(a, S + (j * 64 + lane) * 16);
            if (lane == 0) *reinterpret_cast<uint4*>(w + HOP_WIN) = load16(a, S + HOP_WIN);
        }
        __syncthreads();
        if (k < nseg) {
            uint64_t g, d;
            hop_guess(a, w, S, g, d);
            if (lane == 0) {
                s.hg[k] = g;
                s.hd[k] = d;
            }
        }
    }
    if (p0 == 0 && tid == 0) {  // the first batch's entry is known exactly
        s.hg[0] = a.entry;
        s.hd[0] = 0;
    }
    __syncthreads();
    if (s.hg[0] == NO_HOP) {  // no entry for the batch: the general engine takes it
        s.hcode = SB_HOP_DEAD | (1u << 8);
        return false;
    }
    // B: one lane per segment walks it into scratch
    if (tid < nseg && s.hg[tid] != NO_HOP) {
        const uint64_t S1 = (uint64_t)(p0 + (tid + 1) * hsp) * PIECE;
        uint32_t c, dd;
        uint64_t ex;
        hop_walk(a, s.hg[tid], min(S1, bend), a.scratch + (size_t)(p0 + tid * hsp) * MAX_REC_PIECE,
                 maxr, c, ex, dd);
        s.hcnt[tid] = c;
        s.hexit[tid] = ex;
        s.hdead[tid] = dd;
    }
    __syncthreads();
    // C: stitch in segment order (re-walk a segment entered off its guess)
    if (tid == 0) {
        uint32_t ok = s.hdead[0] == 0, redo = 0, why = ok ? 0u : 3u;
        uint64_t x = s.hexit[0], t = s.hcnt[0];
        for (uint32_t k = 1; k < nseg && ok; ++k) {
            if (s.hg[k] != x) {
                if (++redo > HOP_MAX_REDO) {
                    ok = 0;
                    why = 2;
                    break;
                }
                const uint64_t S1 = (uint64_t)(p0 + (k + 1) * hsp) * PIECE;
                uint32_t c, dd;
                uint64_t ex;
                hop_walk(a, x, min(S1, bend), a.scratch + (size_t)(p0 + k * hsp) * MAX_REC_PIECE,
                         maxr, c, ex, dd);
                s.hg[k] = x;
                s.hcnt[k] = c;
                s.hexit[k] = ex;
                s.hdead[k] = dd;
            }
            ok = s.hdead[k] == 0;
            if (!ok) why = 3;
            x = s.hexit[k];
            t += s.hcnt[k];
        }
        s.hok = ok;
        s.hx = x;
        s.ht = t;
        // SpecBatch.pad bits 8..15: why a hop batch failed (1 no entry guess, 2 too
        // many re-walks, 3 a walk hit an unreadable record or HOP_MAX_RECS)
        s.hcode = ok ? SB_HOP : (SB_HOP_DEAD | (why << 8));
    }
    __syncthreads();
    if (!s.hok) return false;
    if (tid < np) {
        const uint32_t k = tid / hsp;
        const bool first = tid % hsp == 0;
        SpecPiece o;
        o.x = first ? s.hg[k] : 0;
        o.R = 0;
        o.kl = o.vl = 0;
        o.count = first ? s.hcnt[k] : 0;
        o.pad = SP_HOP;
        sp[p0 + tid] = o;
    }
    X0 = s.hg[0];
    X = s.hx;
    total = s.ht;
    return true;
}

// ---- lane-walk mode (small and medium records) ----------------------------------
// A pre-pass batch whose records are too small to hop (hop_batch: more than
// HOP_MAX_CAND candidate run ends in piece 0) is resolved here.  Each of the
// four waves owns a quarter of the batch's pieces and streams it on its own,
// 4 KiB CHUNK by chunk, with no workgroup barrier until the end: chunk k + 1
// is DMA'd global -> LDS (wave-private double buffer, no registers) while
// chunk k is walked, and a chunk's entry is the exact exit of the one before.
// A chunk entered at X:
//   - zero masks: one 16-bit mask per 16-byte granule, computed by the wave
//     from LDS in a conflict-free pattern; every lane owns 64 bytes and takes
//     its candidate bits from 80 mask bits (one aligned 8-byte LDS read);
//   - the lane holding X starts there, every later lane guesses its first
//     record start: the first candidate that ENDS a run of zero-mask
//     candidates (a short header also passes the filter 1-3 bytes to its
//     left), reads as a record shorter than HG_FAR_CAND that fits the file and
//     whose next header (if inside the chunk) is readable; it walks <= 4
//     records to its segment end;
//   - relaxation (DPP max-scans, wave-local): a lane's entry is the largest
//     exit of the CHAIN lanes before it (the entry lane, or a lane whose guess
//     another lane's walk exits on -- a wrong guess in a segment without a
//     record start rarely lies on another lane's exit, so it cannot push the
//     lanes after it past their true entries), a segment that entry jumps over
//     is passed through, a lane entered off its guess walks again; rounds
//     repeat until no exit changes -- that fixed point is exact from X by
//     induction over the lanes; no convergence: lane 0 walks the chunk;
//   - spans go to the piece's scratch slot (decode_kernel copies them, as for
//     hop segments), counts and entries to the piece records.
// A wave's first chunk is entered at the exit of a LEAD-IN chunk (the 4 KiB
// before its quarter, entered at its first lane guess whose walk lands on
// another guess): a wrong lead-in guess has re-joined the true path by the
// quarter's start almost always.  The quarters are stitched once at the end;
// a quarter entered off its predecessor's exit is streamed again from it.
// Any unreadable record on the exact path leaves the batch to decode_kernel's
// engine, which reports errors exactly.
#ifndef HG_LW
#define HG_LW 1  // 0: no lane-walk pre-pass mode (A/B builds)
#endif
constexpr uint32_t LW_CHUNK = 64 * SEG;         // bytes per chunk: one wave, 64 x 64 B
constexpr uint32_t LW_CBUF = LW_CHUNK + 128;    // chunk + halo + read slack
constexpr uint32_t LW_CPP = PIECE / LW_CHUNK;   // chunks per piece
static_assert(LW_ZM_WORDS == LW_CHUNK / 16 + 8, "lane-walk mask rows");
static_assert(4 * LW_CBUF <= PIECE + 512, "two waves' chunk buffers per piece buffer");
constexpr uint32_t LW_WROUNDS = 64;             // relaxation rounds before lane 0 walks it
constexpr uint32_t LW_ENTRY_RETRIES = 4;        // guessed entries tried after one whose path dies
#ifndef HG_LW_LOOKAHEAD
#define HG_LW_LOOKAHEAD 0  // 1: a guess must also read a valid next header (small/medium 2.5 % slower; zero-byte values no better)
#endif
#ifndef HG_LW_ZERO
#define HG_LW_ZERO 1  // 0: lane guesses may take all-zero headers (A/B builds; see lw_guess_nz)
#endif
#ifndef HG_LW_TRIES
#define HG_LW_TRIES 1  // 2: small and medium 1.3 % slower (the second try rarely pays for its reads)
#endif
constexpr uint32_t LW_TRIES = HG_LW_TRIES;      // candidates a lane examines for its guess
constexpr uint32_t LW_PROF = 8;
constexpr uint64_t LW_GUESS = ~0ull;            // "enter at the first linked lane guess"
// Diagnostics (a build with -DHG_LW_DIAG=1 and a.sdiag != null,
// tools/lw_diag.py): lane 0 of wave 0 charges the cycles since the last
// stamp to phase k (0 waiting for a chunk + its masks,
// 1 guesses + walks, 2 chain marks, 3 relaxation, 4 span stores, 5 stitching,
// 6 lead-in chunks, 7 relaxation rounds run).
#ifndef HG_LW_DIAG
#define HG_LW_DIAG 0  // 1: the lane-walk phase clock (a.sdiag) is compiled in
#endif
#define LW_STAMP(k)                                                   \
    do {                                                              \
        if (HG_LW_DIAG && a.sdiag && threadIdx.x == 0) {              \
            const uint64_t now_ = __builtin_amdgcn_s_memtime();       \
            s.lw_prof[k] += (uint32_t)(now_ - s.lw_last);             \
            s.lw_last = now_;                                         \
        }                                                             \
    } while (0)

// LDS written by some lanes of this wave, read by others: DS operations of one
// wave execute in order; this keeps the compiler from reordering them.
__device__ __forceinline__ void lw_wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
}

// s_waitcnt vmcnt(min(n, 12)): the wave's vector memory operations complete in
// issue order, so with the chunk DMA issued before n span stores this waits
// for the DMA only (fewer than n allowed outstanding is merely conservative).
__device__ __forceinline__ void lw_wait_vm(uint32_t n) {
    switch (n) {
        case 0: __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
        case 1: __asm__ volatile("s_waitcnt vmcnt(1)" ::: "memory"); break;
        case 2: __asm__ volatile("s_waitcnt vmcnt(2)" ::: "memory"); break;
        case 3: __asm__ volatile("s_waitcnt vmcnt(3)" ::: "memory"); break;
        case 4: __asm__ volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
        case 5: __asm__ volatile("s_waitcnt vmcnt(5)" ::: "memory"); break;
        case 6: __asm__ volatile("s_waitcnt vmcnt(6)" ::: "memory"); break;
        case 7: __asm__ volatile("s_waitcnt vmcnt(7)" ::: "memory"); break;
        case 8: __asm__ volatile("s_waitcnt vmcnt(8)" ::: "memory"); break;
        case 9: __asm__ volatile("s_waitcnt vmcnt(9)" ::: "memory"); break;
        case 10: __asm__ volatile("s_waitcnt vmcnt(10)" ::: "memory"); break;
        case 11: __asm__ volatile("s_waitcnt vmcnt(11)" ::: "memory"); break;
        default: __asm__ volatile("s_waitcnt vmcnt(12)" ::: "memory"); break;
    }
}

// Chunk at cb (relative to a.sst) into the wave buffer dst: bytes [cb, cb +
// LW_CHUNK + 64).  In bounds: five global_load_lds instructions (4 x 1 KiB,
// lane-linear, + the halo by lanes 0-3); near the end of the bytes present:
// plain 16-byte loads with zero fill (returns after they landed).  Returns the
// vector memory instructions left in flight.
// Cache policy of the chunk DMA: nontemporal (aux 2) -- the table is read
// once.  Same box, 2 rounds (tools/decode_variants.py): small 0.1517 ->
// 0.1476 ms, medium 0.2065 -> 0.2009, 16 B / 8 B-4 KiB 0.0915 -> 0.0893,
// zero-valued small unchanged.
#ifndef HG_LW_DMA_AUX
#define HG_LW_DMA_AUX 2
#endif
// The DMA as inline asm (HG_DMA_ASM): the compiler's wait insertion treats
// every LDS access behind a global_load_lds builtin as possibly reading the
// bytes in flight and puts an s_waitcnt vmcnt(0) before it, so the chunk /
// piece prefetched for the next iteration was waited for at the first LDS
// read of the current one (no overlap at all).  Issued from asm the DMA is
// invisible to it: the kernels' own counted waits (lw_wait_vm) order every
// read of a DMA'd buffer after its DMA, and the compiler's waits for its own
// loads only become stricter (it does not count these).  s_nop 0: the M0
// write -> LDS-DMA hazard (one wait state).
#ifndef HG_DMA_ASM
#define HG_DMA_ASM 1
#endif
__device__ __forceinline__ void dma16(const void* src, uint8_t* dst) {
    if (HG_DMA_ASM) {
        // the low half of a flat LDS address is the LDS offset (the aperture
        // is the high half): no null check as in an address-space cast
        const uint32_t l = __builtin_amdgcn_readfirstlane((uint32_t)(size_t)dst);
        if (HG_LW_DMA_AUX == 2)
            __asm__ volatile("s_nop 0\n\tglobal_load_lds_dwordx4 %0, off nt" :: "v"(src), "{m0}"(l) : "memory");
        else
            __asm__ volatile("s_nop 0\n\tglobal_load_lds_dwordx4 %0, off" :: "v"(src), "{m0}"(l) : "memory");
    } else {
        __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)dst, 16, 0,
                                         HG_LW_DMA_AUX);
    }
}
__device__ __forceinline__ uint32_t lw_fetch_chunk(const DecodeArgs& a, uint64_t cb, uint8_t* dst) {
    const uint32_t lane = threadIdx.x & 63u;
    if (cb + LW_CHUNK + 64 <= a.rlen) {
#pragma unroll
        for (uint32_t q = 0; q < 4; ++q)
            dma16(static_cast<const void*>(a.sst + cb + (uint64_t)(q * 64 + lane) * 16), dst + q * 1024);
        if (lane < 4) dma16(static_cast<const void*>(a.sst + cb + LW_CHUNK + lane * 16), dst + LW_CHUNK);
        return 5;
    }
#pragma unroll 1
    for (uint32_t q = 0; q < 4; ++q)
        *reinterpret_cast<uint4*>(dst + (q * 64 + lane) * 16) = load16(a, cb + (q * 64 + lane) * 16);
    if (lane < 4)
        *reinterpret_cast<uint4*>(dst + LW_CHUNK + lane * 16) = load16(a, cb + LW_CHUNK + lane * 16);
    return 0;
}

// Granule zero masks of the staged chunk into zm (conflict-free: lane l reads
// granules l, l+64, l+128, l+192 and the halo's).  These masks are a large
// share of the mode's VALU work (zmask4: one multiply gathers the flags).
#ifndef HG_LW_MASK_LOADS_FIRST
#define HG_LW_MASK_LOADS_FIRST 1
#endif
__device__ __forceinline__ void lw_chunk_masks(const uint8_t* buf, uint16_t* zm) {
    const uint32_t lane = threadIdx.x & 63u;
#if HG_LW_MASK_LOADS_FIRST
    uint4 g[5];  // every read issued before the first mask store (one LDS round trip, not five)
#pragma unroll
    for (uint32_t q = 0; q < 4; ++q) g[q] = *reinterpret_cast<const uint4*>(buf + (q * 64 + lane) * 16);
    g[4] = *reinterpret_cast<const uint4*>(buf + LW_CHUNK + (lane & 3u) * 16);
    uint32_t m[5];
#pragma unroll
    for (uint32_t q = 0; q < 5; ++q) m[q] = zmask16(g[q]);
#pragma unroll
    for (uint32_t q = 0; q < 4; ++q) zm[q * 64 + lane] = (uint16_t)m[q];
    if (lane < 4) zm[256 + lane] = (uint16_t)m[4];
#else
#pragma unroll
    for (uint32_t q = 0; q < 4; ++q)
        zm[q * 64 + lane] = (uint16_t)zmask16(*reinterpret_cast<const uint4*>(buf + (q * 64 + lane) * 16));
    if (lane < 4)
        zm[256 + lane] = (uint16_t)zmask16(*reinterpret_cast<const uint4*>(buf + LW_CHUNK + lane * 16));
#endif
    lw_wave_sync();
}

// Candidate mask of this lane's segment and the next lane's first bit from
// the granule masks: bit j of the 80 zero-mask bits z1:z0 <=> byte j is zero,
// candidate j <=> bytes [j+8-hz, j+8) and [j+16-hz, j+16) are zero.
// HG_LW_LEAN: the lane-walk mode filters candidates with 4 high zero bytes
// (hz' = 4) whatever the table's hz: a lane walk runs in 32-bit arithmetic,
// where a record whose klen or vlen needs more than 32 bits is dead anyway, so
// no position on a live path is dropped (and for hz > 4 the extra candidates
// are positions a walk reads as records longer than the file).  Then a
// position's mask bit says exactly "header readable, klen and vlen < 2^32":
// walks test that bit instead of reading and checking the high words, and the
// masks need two fixed doubling steps in 32-bit funnel shifts.
#ifndef HG_LW_LEAN
#define HG_LW_LEAN 1
#endif
__device__ __forceinline__ void lw_masks4(const uint16_t* zm, uint32_t seg0, uint32_t clen,
                                          uint64_t rem, uint64_t& cm0, uint64_t& nextbit,
                                          uint64_t& zb, uint64_t* nb_raw = nullptr) {
    cm0 = 0;
    nextbit = 0;
    zb = 0;
    if (nb_raw) *nb_raw = 0;
    if (seg0 >= clen || rem < 16) return;
    const uint32_t gi = seg0 / 16;  // zero-byte bits of bytes seg0 .. seg0 + 79: d0, d1, d2 (16)
    const uint2 z = *reinterpret_cast<const uint2*>(&zm[gi]);
    zb = ((uint64_t)z.y << 32) | z.x;  // the segment's zero bytes (lw_guess)
    uint32_t d0 = z.x, d1 = z.y, d2 = zm[gi + 4];
    d0 &= __builtin_amdgcn_alignbit(d1, d0, 1);  // bit j: bytes j, j+1 zero
    d1 &= __builtin_amdgcn_alignbit(d2, d1, 1);
    d2 &= d2 >> 1;
    d0 &= __builtin_amdgcn_alignbit(d1, d0, 2);  // bit j: bytes j .. j+3 zero
    d1 &= __builtin_amdgcn_alignbit(d2, d1, 2);
    d2 &= d2 >> 2;
    // candidate j <=> bytes [j+4, j+8) and [j+12, j+16) zero
    uint64_t c = ((uint64_t)(__builtin_amdgcn_alignbit(d2, d1, 4) & __builtin_amdgcn_alignbit(d2, d1, 12)) << 32) |
                 (__builtin_amdgcn_alignbit(d1, d0, 4) & __builtin_amdgcn_alignbit(d1, d0, 12));
    const uint64_t c64 = (d2 >> 4) & (d2 >> 12) & 1u;
    const uint32_t n = min(seg0 + SEG, clen) - seg0;
    if (n < 64) c &= (1ull << n) - 1ull;
    const uint64_t plim = rem - 16;
    if (plim < seg0) {
        c = 0;
    } else if (plim - seg0 < 63) {
        c &= (2ull << (plim - seg0)) - 1ull;
    }
    const uint32_t q = seg0 + SEG;
    nextbit = (q < clen && (uint64_t)q <= plim) ? c64 : 0ull;
    // (past the chunk's last position: the halo's mask bits, for run ends)
    if (nb_raw) *nb_raw = (uint64_t)q <= plim ? c64 : 0ull;
    cm0 = c;
}

__device__ __forceinline__ void lw_masks(const uint16_t* zm, uint32_t seg0, uint32_t clen,
                                         uint64_t rem, uint32_t hz, uint64_t& cm0,
                                         uint64_t& nextbit, uint64_t& zb, uint64_t* nb_raw = nullptr) {
    if (HG_LW_LEAN) {
        lw_masks4(zm, seg0, clen, rem, cm0, nextbit, zb, nb_raw);
        return;
    }
    cm0 = 0;
    nextbit = 0;
    zb = 0;
    if (seg0 >= clen || rem < 16) return;
    const uint32_t gi = seg0 / 16;
    const uint64_t z0 = *reinterpret_cast<const uint64_t*>(&zm[gi]);
    zb = z0;
    const uint32_t z1 = zm[gi + 4];
    uint64_t c, c64;
    if (hz == 0) {
        c = ~0ull;
        c64 = 1;
    } else {  // 80-bit shifts as 64 + 16 bits
        const uint32_t hi = z1 & 0xFFFFu;
        uint64_t alo = z0;  // bit i of A: bytes i .. i+hz-1 are zero, by doubling:
        uint32_t ahi = hi;  // A_2p = A_p & (A_p >> p), then one overlapping step
        uint32_t pw = 1;
        while (2 * pw <= hz) {
            alo &= (alo >> pw) | ((uint64_t)ahi << (64 - pw));
            ahi &= ahi >> pw;
            pw *= 2;
        }
        if (pw < hz) {
            const uint32_t r = hz - pw;
            alo &= (alo >> r) | ((uint64_t)ahi << (64 - r));
            ahi &= ahi >> r;
        }
        const uint32_t s1 = 8 - hz, s2 = 16 - hz;  // s1 in [0, 7], s2 in [8, 15]
        const uint64_t a1 = s1 ? ((alo >> s1) | ((uint64_t)ahi << (64 - s1))) : alo;
        const uint64_t a2 = (alo >> s2) | ((uint64_t)ahi << (64 - s2));
        c = a1 & a2;
        c64 = ((ahi >> s1) & (ahi >> s2)) & 1u;
    }
    const uint32_t n = min(seg0 + SEG, clen) - seg0;  // positions where records may start
    if (n < 64) c &= (1ull << n) - 1ull;
    const uint64_t plim = rem - 16;  // last readable header position
    if (plim < seg0) {
        c = 0;
    } else if (plim - seg0 < 63) {
        c &= (2ull << (plim - seg0)) - 1ull;
    }
    const uint32_t q = seg0 + SEG;
    nextbit = (q < clen && (uint64_t)q <= plim) ? c64 : 0ull;
    cm0 = c;
}

// lw_guess when the lane's guess reads as an all-zero header followed by 16
// more zero bytes (a genuine empty record -- InternalPair::default, 16 zero
// bytes -- is followed by a header, not by zeros): the lane is inside a run
// of zero bytes (a zero-byte value), where every
// position reads as an empty 16-byte record and a walk chains on through the
// zeros -- a guess there is self-consistent but usually off the true path, so
// the chunk's entry and the lanes after it would follow it.  The candidates
// at which 16 zero bytes start are dropped (doubling over the zero-byte
// masks), run ends recomputed, and up to LW_ZTRIES candidates tried with a
// look-ahead (a shifted read of a header next to a zero run decodes as a
// short record that lands inside a key).  Only lanes that meet a zero header
// pay for this.
constexpr uint32_t LW_ZTRIES = 4;
constexpr uint32_t LW_ZERO_HDR = 1u << 30;  // lw_guess: the guess reads as an all-zero header
__device__ __noinline__ uint32_t lw_guess_nz(const uint8_t* data, const uint16_t* zm,
                                             uint32_t seg0, uint32_t clen, uint64_t rem,
                                             uint64_t cm0, uint64_t nextbit) {
    const uint32_t gi = seg0 / 16;
    uint64_t alo = *reinterpret_cast<const uint64_t*>(&zm[gi]);
    uint32_t ahi = zm[gi + 4] & 0xFFFFu;
#pragma unroll
    for (uint32_t pw = 1; pw < 16; pw *= 2) {  // bit j <=> bytes j .. j+15 are zero
        alo &= (alo >> pw) | ((uint64_t)ahi << (64 - pw));
        ahi &= ahi >> pw;
    }
    const uint64_t cm = cm0 & ~alo;
    const uint64_t nb = nextbit & ~(uint64_t)(ahi & 1u);
    const uint64_t runend = cm & ~((cm >> 1) | (nb << 63));
    uint64_t c = runend;
    uint32_t tries = 0;
    for (uint32_t pass = 0; pass < 2; ++pass) {
        if (pass) c = cm & ~runend;
        while (c && tries++ < LW_ZTRIES) {
            const uint32_t p = seg0 + (uint32_t)(__ffsll((long long)c) - 1);
            c &= c - 1;
            uint32_t k0, k1, v0, v1;
            lds_header32(data, p, k0, k1, v0, v1);
            const uint64_t body = (uint64_t)k0 + v0;
            if ((k1 | v1) || body == 0 || body >= HG_FAR_CAND || body > rem - p - 16) continue;
            const uint64_t nx = (uint64_t)p + 16 + body;
            if (nx < clen) {
                if (nx + 16 > rem) continue;
                lds_header32(data, (uint32_t)nx, k0, k1, v0, v1);
                if ((k1 | v1) || (uint64_t)k0 + v0 > rem - nx - 16) continue;
            }
            return p;
        }
    }
    return NO_GUESS;
}

#ifndef HG_LW_WSHR
#define HG_LW_WSHR 1  // 0: the relaxation's lane shift by __shfl_up (A/B)
#endif
#ifndef HG_LW_NZ1
#define HG_LW_NZ1 1  // 0: run ends in position order (round-3 rule, A/B)
#endif
// This lane's guess in [seg0, segend) (piece-relative) or NO_GUESS; cm0 / the
// next lane's first candidate bit as in lean_prepare.
__device__ __forceinline__ uint32_t lw_guess(const uint8_t* data, const uint16_t* zm,
                                             uint32_t seg0, uint32_t segend, uint32_t clen,
                                             uint64_t rem, uint32_t hz, uint64_t cm0,
                                             uint64_t nextbit, uint64_t zb) {
    uint64_t runend = cm0 & ~((cm0 >> 1) | (nextbit << 63));
    // Inside zero-byte values runs of candidates end 16 and 8 bytes before
    // the true header (those positions read as the headers (0, 0) and
    // (0, klen): klen's low byte lands in the vlen) -- reads inside the value
    // that chain into the next record.  So a run end whose first byte is zero
    // is passed over when a run end with a non-zero first byte follows 8 or 16
    // bytes later; a true header of an empty key (first byte zero too) has no
    // such partner (passing every zero-first-byte run end over cost small
    // records 5 %).
    if (HG_LW_NZ1) {  // (zb: the segment's zero-byte bits, from lw_masks)
        const uint64_t nzr = runend & ~zb;
        runend &= ~(zb & ((nzr >> 8) | (nzr >> 16)));
    }
    uint64_t cm = runend;
    uint32_t tries = 0;  // a lane left without a guess is entered by the relaxation
#pragma nounroll
    for (uint32_t pass = 0; pass < 2; ++pass) {
        if (pass) cm = cm0 & ~runend;
        while (cm && tries++ < LW_TRIES) {
            const uint32_t p = seg0 + (uint32_t)(__ffsll((long long)cm) - 1);
            cm &= cm - 1;
            uint32_t k0, k1 = 0, v0, v1 = 0;
            if (HG_LW_LEAN) lds_kv32(data, p, k0, v0);  // high words zero by the mask
            else lds_header32(data, p, k0, k1, v0, v1);
            const uint64_t body = (uint64_t)k0 + v0;
            if ((k1 | v1) || body >= HG_FAR_CAND || body > rem - p - 16) continue;
            const uint64_t nx = (uint64_t)p + 16 + body;
            if (HG_LW_LOOKAHEAD && nx < clen) {  // look-ahead: the next header must be a readable record
                if (nx + 16 > rem) continue;
                lds_header32(data, (uint32_t)nx, k0, k1, v0, v1);
                if ((k1 | v1) || (uint64_t)k0 + v0 > rem - nx - 16) continue;
            }
            if (HG_LW_ZERO && body == 0) {  // (0, 0): inside a run of >= 32 zero bytes?
                lds_header32(data, p + 16, k0, k1, v0, v1);  // (in the chunk buffer's halo)
                if ((k0 | k1 | v0 | v1) == 0) return p | LW_ZERO_HDR;  // see lw_guess_nz
            }
            return p;
        }
    }
    (void)segend;
    return NO_GUESS;
}

// lane_walk in 32-bit chunk-relative arithmetic (the lane-walk mode's hot
// loop): records starting in [x, segend), lim = bytes from the chunk start to
// the end of the file, clamped to 2^31 (a record reaching past a clamped
// limit reads as dead, and the chunk then takes the exact serial walk).
struct LWalk {
    uint32_t exit;      // chunk-relative
    uint32_t p01, p23;  // up to four 16-bit positions
    uint32_t cnt;
    bool dead;
};

__device__ __forceinline__ uint32_t walk_pos(const LWalk& w, uint32_t i) {
    const uint32_t v = i < 2 ? w.p01 : w.p23;
    return (i & 1) ? (v >> 16) : (v & 0xFFFFu);
}

__device__ __forceinline__ void lw_walk(const uint8_t* data, uint32_t lim, uint32_t x,
                                        uint32_t segend, uint32_t seg0, uint64_t cm, LWalk& w) {
    w.cnt = 0;
    w.dead = false;
    w.p01 = w.p23 = 0;
    uint32_t cur = x;
    if (HG_LW_LEAN) {  // positions in [seg0, segend): the mask bit is "readable, high words zero"
        const uint32_t lim16 = lim - 16;
#pragma unroll
        for (int it = 0; it < 4; ++it) {
            if (cur >= segend) break;
            if (!((cm >> (cur - seg0)) & 1u)) {
                w.dead = true;
                break;
            }
            uint32_t k0, v0;
            lds_kv32(data, cur, k0, v0);
            const uint32_t room = lim16 - cur;
            if (k0 > room || v0 > room - k0) {
                w.dead = true;
                break;
            }
            if (it == 0) w.p01 = cur;
            if (it == 1) w.p01 |= cur << 16;
            if (it == 2) w.p23 = cur;
            if (it == 3) w.p23 |= cur << 16;
            ++w.cnt;
            cur += 16 + k0 + v0;
        }
        w.exit = cur;
        return;
    }
#pragma unroll
    for (int it = 0; it < 4; ++it) {
        if (cur >= segend) break;
        if (cur + 16 > lim) {
            w.dead = true;
            break;
        }
        uint32_t k0, k1, v0, v1;
        lds_header32(data, cur, k0, k1, v0, v1);
        const uint32_t room = lim - cur - 16;
        if ((k1 | v1) || k0 > room || v0 > room - k0) {
            w.dead = true;
            break;
        }
        if (it == 0) w.p01 = cur;
        if (it == 1) w.p01 |= cur << 16;
        if (it == 2) w.p23 = cur;
        if (it == 3) w.p23 |= cur << 16;
        ++w.cnt;
        cur += 16 + k0 + v0;
    }
    w.exit = cur;
}

// Lane 0 walks the staged chunk exactly from X (the relaxation did not
// converge: rare, e.g. a wrong guess that links and pushes a long run of
// lanes past their entries): spans to out (if any).  False if a record on
// the path cannot be read.  Wave-level; every lane returns the same values.
__device__ __forceinline__ bool lw_chunk_serial(const DecodeArgs& a, const uint8_t* data,
                                                uint64_t cb, uint32_t clen, uint64_t X,
                                                hg_span* out, uint32_t& count, uint64_t& exit,
                                                uint32_t& nstores) {
    uint32_t n = 0, ok = 1;
    uint64_t cur = X;
    if ((threadIdx.x & 63u) == 0) {
        while (cur < cb + clen) {
            if (cur + 16 > a.len) {
                ok = 0;
                break;
            }
            uint32_t k0, k1, v0, v1;
            lds_header32(data, (uint32_t)(cur - cb), k0, k1, v0, v1);
            const uint64_t body = (uint64_t)k0 + v0;
            if ((k1 | v1) || body > a.len - cur - 16) {
                ok = 0;
                break;
            }
            if (out) write_span(out, n, cur, k0, v0);
            ++n;
            cur += 16 + body;
        }
    }
    count = __shfl(n, 0, 64);
    exit = __shfl(cur, 0, 64);
    nstores = out ? count : 0u;
    return __shfl(ok, 0, 64) != 0;
}

// Round 6: a chunk entered at an exact X is first tried
// by per-chunk discovery with no walks and no relaxation.  Take every
// candidate that ENDS a run of header candidates (the masks' filter: a
// short header also passes 1-3 bytes to its left) at or after X as a record
// start, read each one's header (independent LDS reads, no chain), and
// verify the whole set at once: inside a lane each candidate's successor
// must be the lane's next candidate; a lane's first candidate must be the
// largest successor of all earlier lanes' last candidates (one DPP max-scan)
// -- lane je's first must be X -- and the chunk's largest successor must
// reach its end.  By induction from X the verified set is exactly the
// record chain (a record start that is not a run end, a false run end, an
// unreadable record or more than 4 starts in a lane fail the check).  Then a
// DPP sum-scan places the spans.  A failing chunk takes the lane walks
// below, which are exact on any input.  Same contract as lw_chunk.
// Same box, 3 rounds (profiles/r6_ab_lw_verify.log; every run bit-exact
// against the oracle): small records 0.1366 -> 0.1264 ms, medium 0.1806 ->
// 0.1637, zero-valued small 0.1465 -> 0.1511 (its chunks skip the try, the
// gate costs ~3 %), the stride and hop shapes unchanged.  Variants measured
// on the way: every run end taken (no spacing filter) fails on 2/3 of the
// small-record chunks (a tiny record's value read 8 bytes in also ends a
// run): small 0.147; always trying on every chunk: zero-valued small 0.179;
// a per-stream back-off instead of the zero-byte gate: streams are only 16
// chunks long, small 0.135.
#ifndef HG_LW_VSTORE
#define HG_LW_VSTORE 1
#endif
#ifndef HG_LW_VERIFY
#define HG_LW_VERIFY 1
#endif
__device__ __forceinline__ bool lw_chunk_verify(const uint8_t* data, uint64_t cb, uint32_t xw,
                                                uint32_t je, uint32_t seg0, uint32_t clen,
                                                uint32_t lim, uint64_t cm0, uint64_t nb,
                                                hg_span* out, uint32_t& count, uint64_t& exit,
                                                uint32_t& nstores) {
    const uint32_t lane = threadIdx.x & 63u;
    uint64_t re = cm0 & ~((cm0 >> 1) | (nb << 63));  // run ends of this lane's segment
    if (lane < je) re = 0;
    else if (lane == je) re &= ~0ull << (xw - seg0);  // starts at or after X (xw - seg0 < 64)
    // Records are >= 16 bytes apart, so of run ends closer than that at most
    // one is a start: keep them greedily in position order (the earlier one
    // -- a tiny record's value / next header read 8 bytes in also ends a
    // run).  Within the lane, then again from the previous lane's last kept
    // run end (its first pass; a cascade over a whole lane of run ends
    // spaced < 16 apart is left to the verification).
    auto greedy = [&](int32_t last, int32_t& lastk) -> uint64_t {
        uint64_t kept = 0, t = re;
        while (t) {
            const int32_t q = __ffsll((long long)t) - 1;
            t &= t - 1;
            if (q - last >= 16) {
                kept |= 1ull << q;
                last = q;
            }
        }
        lastk = last;
        return kept;
    };
    int32_t l1 = -64;
    (void)greedy(-64, l1);
    const int32_t prevl = __builtin_amdgcn_update_dpp(-1000, l1, 0x138, 0xf, 0xf, false) - 64;
    int32_t l2 = 0;
    uint64_t r = greedy(lane == je ? -64 : prevl, l2);  // (lane je: the entry X is exact)
    const uint32_t n = (uint32_t)__popcll(r);
    bool ok = n <= 4;
    const uint32_t lim16 = lim - 16;
    // HG_LW_VSTORE: each candidate's span is stored as soon as its header is
    // read (placed by the candidates' prefix count); a chunk that fails the
    // check is stored again, exactly, by the walks (after these stores have
    // completed), and candidates beyond its true count land inside the
    // piece's scratch slot (<= 256 per chunk) where nothing reads them.
    const uint32_t incl = dpp_sum_incl(n);
    const uint32_t pre = incl - n;
    uint32_t first = 0, nx = 0, p01 = 0, p23 = 0;
#pragma unroll
    for (uint32_t it = 0; it < 4; ++it) {
        if (!r) break;
        const uint32_t p = seg0 + (uint32_t)(__ffsll((long long)r) - 1);
        r &= r - 1;
        uint32_t k0, v0;  // (the mask bit says: readable, high words zero)
        lds_kv32(data, p, k0, v0);
        const uint32_t room = lim16 - p;
        if (k0 > room || v0 > room - k0) ok = false;  // unreadable: the walks report it exactly
        if (it == 0) first = p;
        else if (nx != p) ok = false;
        nx = p + 16 + k0 + v0;
        if (HG_LW_VSTORE) {
            if (out) write_span(out, pre + it, cb + p, k0, v0);
        } else {
            if (it == 0) p01 = p;
            if (it == 1) p01 |= p << 16;
            if (it == 2) p23 = p;
            if (it == 3) p23 |= p << 16;
        }
    }
    const uint32_t m = dpp_max_incl(n ? nx : 0u);
    // the previous lanes' largest successor (gfx9 wave_shr:1, lane 0 gets 0)
    const uint32_t before = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)m, 0x138, 0xf, 0xf, false);
    if (lane == je) ok = ok && n && first == xw;
    else if (n) ok = ok && before == first;
    const uint32_t E = (uint32_t)__builtin_amdgcn_readlane((int)m, 63);
    if (__ballot(!ok) || E < clen) {  // (E < clen: a record starts after the last run end)
        if (HG_LW_VSTORE && out) lw_wait_vm(0);  // the walks' stores land after these
        return false;
    }
    count = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
    exit = cb + E;
    nstores = 0;
    if (out && HG_LW_VSTORE) {
        nstores = (uint32_t)__builtin_amdgcn_readlane((int)dpp_max_incl(n), 63);
    } else if (out) {
        const uint32_t cmax = (uint32_t)__builtin_amdgcn_readlane((int)dpp_max_incl(n), 63);
        for (uint32_t i = 0; i < cmax; ++i) {  // one store instruction per step
            if (i < n) {
                const uint32_t v = i < 2 ? p01 : p23;
                lw_store_span(out, pre + i, data, cb, (i & 1) ? (v >> 16) : (v & 0xFFFFu));
            }
        }
        nstores = cmax;
    }
    return true;
}

// The staged chunk at cb (records start in [cb, cb + clen)) entered at X
// (exact; LW_GUESS: at its first lane guess whose walk lands on another
// lane's guess): spans to out[0, count) (nullptr: none), entry = the entry
// used, exit = the first start at or after cb + clen, nstores = span store
// instructions issued.  Wave-level; every lane returns the same values.
// vs: reserved for a stream-level verification state (unused).
template <bool VER>
__device__ __forceinline__ bool lw_chunk(SpecSmem& s, const DecodeArgs& a, const uint8_t* data,
                                         const uint16_t* zm, uint32_t* sg, uint8_t* tg,
                                         uint64_t cb, uint32_t clen, uint64_t X, hg_span* out,
                                         uint64_t& entry, uint32_t& count, uint64_t& exit,
                                         uint32_t& nstores, uint32_t& vs) {
    const uint32_t lane = threadIdx.x & 63u;
    const bool guess = X == LW_GUESS;
    nstores = 0;
    count = 0;
    if (!guess && (clen == 0 || X >= cb + clen)) {  // past stop, or a record spans the chunk
        entry = exit = X;
        return true;
    }
    const uint64_t rem = a.len - cb;
    const uint32_t seg0 = lane * SEG, segend = min(seg0 + SEG, clen);
    const uint32_t je = guess ? 0u : (uint32_t)((X - cb) / SEG);
    const bool in_chunk = seg0 < clen && lane >= je;
    uint64_t cm0, nb, zb, nbr = 0;
    lw_masks(zm, seg0, clen, rem, a.hz, cm0, nb, zb, &nbr);
    const uint32_t lim = (uint32_t)min(rem, (uint64_t)1 << 31);
    // (a chunk whose bytes are mostly zero -- zero-byte values -- is full of
    // false run ends: the verification would fail, so it is not tried when a
    // quarter of its lanes hold >= 40 zero bytes of their 64)
    if (VER && HG_LW_VERIFY && HG_LW_LEAN && !guess &&
        __popcll(__ballot(in_chunk && __popcll(zb) >= 40)) < 16 &&
        lw_chunk_verify(data, cb, (uint32_t)(X - cb), je, seg0, clen, lim, cm0, nbr, out, count, exit,
                        nstores)) {
        entry = X;
        LW_STAMP(4);
        return true;
    }
    (void)vs;
    uint32_t g = NO_GUESS;
    LWalk w;
    w.dead = true;
    w.exit = 0;
    w.cnt = 0;
    w.p01 = w.p23 = 0;
    if (!guess && lane == je) g = (uint32_t)(X - cb);
    else if (in_chunk) g = lw_guess(data, zm, seg0, segend, clen, rem, a.hz, cm0, nb, zb);
    if (HG_LW_ZERO && g != NO_GUESS && (g & LW_ZERO_HDR))  // rare: a lane inside zero bytes
        g = lw_guess_nz(data, zm, seg0, clen, rem, cm0, nb);
    if (in_chunk && g != NO_GUESS) lw_walk(data, lim, g, segend, seg0, cm0, w);
    LW_STAMP(1);
    // chain marks: which lane guesses some lane's walk exits on
    const bool valid0 = in_chunk && g != NO_GUESS && !w.dead;
    sg[lane] = valid0 ? g : NO_GUESS;
    tg[lane] = 0;
    lw_wave_sync();
    bool links = false;
    if (valid0) {
        const uint32_t u = w.exit;
        if (u < clen && sg[u / SEG] == u) {
            tg[u / SEG] = 1;
            links = true;
        }
    }
    lw_wave_sync();
    const bool chain = tg[lane] != 0;
    uint32_t jl = je, xw = 0;
    unsigned long long vm = 0;
    if (guess) {
        const unsigned long long lm = __ballot(valid0 && links);
        vm = __ballot(valid0);
        if (!vm) return false;  // nothing that reads as a record: no entry
        jl = (uint32_t)__ffsll((long long)(lm ? lm : vm)) - 1;
        xw = __shfl(g, (int)jl, 64);
        X = cb + xw;
    } else {
        xw = (uint32_t)(X - cb);
    }
    entry = X;
    LW_STAMP(2);
    // ---- relaxation from (jl, xw) ----
    const bool act = in_chunk && lane >= jl;
    uint32_t ev = (act && valid0 && (lane == jl || chain)) ? w.exit : 0u;
    uint32_t st = act ? 0u : 3u;  // 0 walking from g, 1 passed through, 2 waiting, 3 not on the path
    bool conv = false;
    for (uint32_t r = 0; r < LW_WROUNDS; ++r) {
        if (HG_LW_DIAG && a.sdiag && threadIdx.x == 0) ++s.lw_prof[7];
        const uint32_t m = dpp_max_incl(ev);
        // the previous lane's inclusive max: a DPP wave shift (gfx9 wave_shr:1,
        // lane 0 gets 0) instead of __shfl_up's LDS permute round trip
        uint32_t excl;
        if (HG_LW_WSHR) {
            excl = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)m, 0x138, 0xf, 0xf, false);
        } else {
            excl = __shfl_up(m, 1, 64);
            if (lane == 0) excl = 0;
        }
        const uint32_t seed = lane == jl ? xw : excl;
        uint32_t nev = ev;
        if (act) {
            if (lane != jl && seed >= segend) {  // jumped over by a record / the exit
                st = 1;
                nev = 0;
            } else if (lane != jl && seed < seg0) {  // not resolved yet: keep the exit
                st = 2;                              // (resetting it would cost the lanes
            } else {                                 // after it one round each)
                if (st != 0 || g == NO_GUESS || seed != g) {
                    g = seed;
                    lw_walk(data, lim, g, segend, seg0, cm0, w);
                }
                st = 0;
                nev = w.dead ? 0u : w.exit;
            }
        }
        const bool changed = nev != ev;
        ev = nev;
        if (!__ballot(changed)) {
            conv = true;
            break;
        }
    }
    LW_STAMP(3);
    const bool walking = act && st == 0;
    if (!conv || __ballot(act && (st == 2 || (st == 0 && w.dead)))) {
        const bool sok = lw_chunk_serial(a, data, cb, clen, X, out, count, exit, nstores);
        if (sok || !guess) return sok;
        // A guessed entry whose path cannot be read (e.g. a shifted read next to
        // a run of zero bytes that still looked like a record): walk from the
        // next lanes' original guesses (sg) in order until one path reaches
        // the chunk end.  Guess mode writes no spans (lead-in chunks).
        unsigned long long cand = vm & ~((2ull << jl) - 1ull);
        for (uint32_t t = 0; t < LW_ENTRY_RETRIES && cand; ++t) {
            const uint32_t l2 = (uint32_t)(__ffsll((long long)cand) - 1);
            cand &= cand - 1;
            const uint64_t X2 = cb + sg[l2];
            if (lw_chunk_serial(a, data, cb, clen, X2, out, count, exit, nstores)) {
                entry = X2;
                return true;
            }
        }
        return false;
    }
    const uint32_t c = walking ? w.cnt : 0u;
    const uint32_t incl = dpp_sum_incl(c);
    count = __builtin_amdgcn_readlane((int)incl, 63);
    const unsigned long long wm = __ballot(walking);  // the chain's last lane holds the exit
    const uint32_t ll = 63u - (uint32_t)__clzll((long long)wm);
    exit = cb + (uint32_t)__builtin_amdgcn_readlane((int)w.exit, ll);
    if (out) {
        const uint32_t cmax = __builtin_amdgcn_readlane((int)dpp_max_incl(c), 63);
        const uint32_t pre = incl - c;
        for (uint32_t i = 0; i < cmax; ++i)  // one store instruction per step
            if (i < c) lw_store_span(out, pre + i, data, cb, walk_pos(w, i));
        nstores = cmax;
    }
    LW_STAMP(4);
    return true;
}

// One lane's exact walk of the staged chunk from X (records of a few hundred
// bytes: a dozen dependent LDS header reads per 4 KiB cost less than the
// lanes' masks, guesses and relaxation): the positions go to pos (the chunk's
// mask rows, unused in this mode), then the wave stores the spans, one
// instruction per 64 records.  A record this 32-bit walk cannot read takes
// lw_chunk_serial (exact 64-bit walk).  Same contract as lw_chunk with X exact.
// After a full chunk of at most HG_LW_SER records, the stream walks its next
// chunk by one lane (0: never).  Measured (tools/decode_variants.py, same box,
// 2 rounds): 400-1200 B records with zero-byte values 0.745 -> 0.390 ms (their
// lanes' guesses fall into the zero runs), 0-16 KiB values 0.212 -> 0.209;
// small, 8 B-4 KiB and 400-1200 B random values unchanged; a threshold of 12
// made medium records (8-64 B keys, 64-512 B values) 2.5 % slower.
#ifndef HG_LW_SER
#define HG_LW_SER 8
#endif
__device__ __forceinline__ bool lw_chunk_walk(const DecodeArgs& a, const uint8_t* data,
                                              uint16_t* pos, uint64_t cb, uint32_t clen, uint64_t X,
                                              hg_span* out, uint64_t& entry, uint32_t& count,
                                              uint64_t& exit, uint32_t& nstores) {
    const uint32_t lane = threadIdx.x & 63u;
    nstores = 0;
    count = 0;
    entry = X;
    if (clen == 0 || X >= cb + clen) {
        exit = X;
        return true;
    }
    const uint32_t lim = (uint32_t)min(a.len - cb, (uint64_t)1 << 31);
    uint32_t n = 0, ok = 1, cur = (uint32_t)(X - cb);
    if (lane == 0) {
        while (cur < clen) {
            if (cur + 16 > lim) {
                ok = 0;
                break;
            }
            uint32_t k0, k1, v0, v1;
            lds_header32(data, cur, k0, k1, v0, v1);
            const uint32_t room = lim - cur - 16;
            if ((k1 | v1) || k0 > room || v0 > room - k0) {
                ok = 0;
                break;
            }
            pos[n++] = (uint16_t)cur;
            cur += 16 + k0 + v0;
        }
    }
    if (!__shfl(ok, 0, 64)) return lw_chunk_serial(a, data, cb, clen, X, out, count, exit, nstores);
    count = __shfl(n, 0, 64);
    exit = cb + __shfl(cur, 0, 64);
    lw_wave_sync();
    if (out) {
        for (uint32_t i = lane; i < count; i += 64) lw_store_span(out, i, data, cb, pos[i]);
        nstores = (count + 63) / 64;
    }
    return true;
}

// This wave's quarter [pb, pe) of the batch's pieces, entered at X (exact;
// LW_GUESS: through the lead-in chunk before pb), streamed chunk by chunk
// through the wave's two LDS chunk buffers: piece records into sp[], spans
// into the pieces' scratch slots.  Wave-level; returns ok with the entry
// used, the exit and the records.
template <bool VER>
__device__ __forceinline__ bool lw_stream(SpecSmem& s, const DecodeArgs& a, uint8_t* bufs,
                                          uint16_t* zm, uint32_t* sg, uint8_t* tg, uint32_t pb,
                                          uint32_t pe, uint64_t X, SpecPiece* sp, uint64_t& entry,
                                          uint64_t& exit, uint64_t& total, uint32_t nlead) {
    const uint32_t lane = threadIdx.x & 63u;
    // piece records of the quarter, kept in LDS until the stream ends so the
    // chunk loop issues no vector memory operations besides its span stores
    uint64_t* const px = s.lw_px[threadIdx.x >> 6];
    uint32_t* const pc = s.lw_pc[threadIdx.x >> 6];
    const bool lead = X == LW_GUESS;
    // nlead lead-in chunks: the first entered at a guess, the others exactly
    const uint64_t nl = lead ? min((uint64_t)nlead, (uint64_t)pb * LW_CPP) : 0u;
    const uint64_t k0 = (uint64_t)pb * LW_CPP - nl;
    const uint64_t k1 = (uint64_t)pe * LW_CPP;
    lw_fetch_chunk(a, k0 * LW_CHUNK, bufs);
    lw_wait_vm(0);
    uint64_t x = X, pentry = X;
    uint32_t pcount = 0;
    bool ok = true;
    total = 0;
    entry = X;
    bool ser = false;  // HG_LW_SER: the last chunk's records were few, walk this one by one lane
    uint32_t vs = 0;   // HG_LW_VERIFY back-off (lw_chunk)
    for (uint64_t k = k0; k < k1; ++k) {
        uint8_t* const cur = bufs + ((k - k0) & 1u) * LW_CBUF;
        uint8_t* const nxt = bufs + ((k - k0 + 1) & 1u) * LW_CBUF;
        if (k + 1 < k1) lw_fetch_chunk(a, (k + 1) * LW_CHUNK, nxt);  // in flight meanwhile
        const bool walk1 = HG_LW_SER && ser && x != LW_GUESS;
        if (!walk1) lw_chunk_masks(cur, zm);
        LW_STAMP(0);
        const uint64_t cb = k * LW_CHUNK;
        const uint32_t clen = a.stop > cb ? (uint32_t)min((uint64_t)LW_CHUNK, a.stop - cb) : 0u;
        const bool is_lead = k < k0 + nl;
        const uint64_t piece = k / LW_CPP;
        hg_span* out = is_lead ? nullptr : a.scratch + (size_t)piece * MAX_REC_PIECE + pcount;
        uint64_t en = 0, ex = 0;
        uint32_t cnt = 0, nst = 0;
        const bool okc = walk1 ? lw_chunk_walk(a, cur, zm, cb, clen, x, out, en, cnt, ex, nst)
                               : lw_chunk<VER>(s, a, cur, zm, sg, tg, cb, clen, x, out, en, cnt, ex, nst, vs);
        if (!okc) {
            ok = false;
            break;
        }
        if (HG_LW_SER && clen == LW_CHUNK) ser = cnt <= HG_LW_SER;
        if (is_lead) {
            entry = ex;
            x = ex;
            LW_STAMP(6);
        } else {
            if (k % LW_CPP == 0) pentry = x;
            pcount += cnt;
            total += cnt;
            if (k % LW_CPP == LW_CPP - 1 || k + 1 == k1) {  // piece record: written at the end
                if (lane == 0) {
                    px[piece - pb] = pentry;
                    pc[piece - pb] = pcount;
                }
                pcount = 0;
            }
            x = ex;
        }
        lw_wait_vm(nst);  // chunk k + 1 landed: its DMA was issued before the nst span stores
    }
    lw_wait_vm(0);  // no DMA may land after the stream is done with its buffers
    if (ok) {
        lw_wave_sync();
        for (uint32_t i = lane; i < pe - pb; i += 64) {
            SpecPiece o;
            o.x = px[i];
            o.R = 0;
            o.kl = o.vl = 0;
            o.count = pc[i];
            o.pad = SP_HOP;
            sp[pb + i] = o;
        }
    }
    exit = x;
    return ok;
}

// Stage piece i of the batch (held in v) into LDS with its halo.
__device__ __forceinline__ void spec_stage(SpecSmem& s, const uint4 (&v)[GPT], uint32_t i) {
    uint8_t* data = reinterpret_cast<uint8_t*>(s.data64);
#pragma unroll
    for (uint32_t q = 0; q < GPT; ++q)
        *reinterpret_cast<uint4*>(data + (q * THREADS + threadIdx.x) * 16) = v[q];
    if (threadIdx.x < 4)  // thread 0 reads back its own halo write when i == 0
        *reinterpret_cast<uint4*>(data + PIECE + threadIdx.x * 16) =
            threadIdx.x == 0 ? s.halo[i] : make_uint4(0, 0, 0, 0);
}

// The lane-walk batch [p0, p0 + np): wave w streams pieces [p0 + w*q, +q)
// (q = ceil(np / 4)); the first wave enters at the batch's entry (the table's
// for the first batch, else through its lead-in), the others through their
// lead-ins; then the quarters are stitched (a quarter entered off its
// predecessor's exit is streamed again from it).  On success X0 = entry, X =
// exit, total = records.  All threads call it (the pieces staged by the
// caller are not used: every chunk is fetched again, L2-warm).
// VER: the per-chunk verification (HG_LW_VERIFY) is compiled in -- not in
// compaction mode, whose kernel it pushed from 114 VGPRs into scratch spills.
template <bool VER = true>
__device__ __forceinline__ bool lw_batch(SpecSmem& s, uint64_t* alt, const DecodeArgs& a,
                                         uint32_t p0, uint32_t np, SpecPiece* sp, uint64_t& X0,
                                         uint64_t& X, uint64_t& total, uint32_t& why) {
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wid = tid >> 6;
    why = 0;
    uint8_t* const bufs = wid < 2 ? reinterpret_cast<uint8_t*>(s.data64) + wid * 2 * LW_CBUF
                                  : reinterpret_cast<uint8_t*>(alt) + (wid - 2) * 2 * LW_CBUF;
    uint16_t* const zm = s.lw_zm[wid];
    uint32_t* const sg = s.lw_sg + wid * 64;
    uint8_t* const tg = s.lw_tg + wid * 64;
    if (tid == 0) {
        for (uint32_t k = 0; k < LW_PROF; ++k) s.lw_prof[k] = 0;
        s.lw_last = __builtin_amdgcn_s_memtime();
    }
    __syncthreads();  // the caller is done with the staged piece (data64)
    const uint32_t q = (np + NW - 1) / NW;
    const uint32_t pb = p0 + min(wid * q, np), pe = p0 + min((wid + 1) * q, np);
    uint64_t xin = (wid == 0 && p0 == 0) ? a.entry : LW_GUESS;
    bool exact = xin != LW_GUESS;
    uint64_t en = 0, ex = 0, tot = 0;
    bool okw = true, run = pb < pe;
    bool ok = true, long_lead = false;
    uint32_t nlead = 1;
    uint64_t x = 0;
    uint32_t flast = 0;
    for (uint32_t att = 0;; ++att) {  // one call site of lw_stream (first pass and re-streams)
        if (run) okw = lw_stream<VER>(s, a, bufs, zm, sg, tg, pb, pe, xin, sp, en, ex, tot, nlead);
        run = false;
        const uint32_t f = att & 1u;
        flast = f;
        if (lane == 0) {
            s.lw_wx[f][wid] = en;
            s.lw_wexit[f][wid] = ex;
            s.lw_wcnt[f][wid] = (uint32_t)tot;
            s.lw_wbad[f][wid] = (okw ? 0u : 1u) | (exact ? 2u : 0u) | (pb < pe ? 4u : 0u);
        }
        __syncthreads();
        // stitch in order (uniform in every wave)
        uint32_t fix = NW;
        total = 0;
        for (uint32_t v = 0; v < NW; ++v) {
            const uint32_t fl = s.lw_wbad[f][v];
            if (!(fl & 4u)) continue;  // no pieces
            const bool entered = v == 0 || s.lw_wx[f][v] == x;
            if ((fl & 1u) || !entered) {  // unresolved, or entered off the exact exit
                if (v == 0 && !(fl & 2u) && !long_lead) {
                    // the first quarter's guessed entry led nowhere (a path that
                    // survived the 4 KiB lead-in inside zero-byte values): stream
                    // it again behind a whole piece of lead-in chunks
                    fix = 0;
                    long_lead = true;
                } else if (v == 0 || (fl & 2u)) {  // exact entry and still unresolved
                    ok = false;
                    why = (fl & 2u) ? 2u : 1u;
                } else {
                    fix = v;
                }
                break;
            }
            x = s.lw_wexit[f][v];
            total += s.lw_wcnt[f][v];
        }
        if (!ok || fix == NW || att == NW) {
            if (fix != NW) {
                ok = false;
                why = 3;
            }
            break;
        }
        if (wid == fix) {  // stream the quarter again from the exact entry
            exact = fix != 0 || (p0 == 0);
            xin = fix == 0 ? (p0 == 0 ? a.entry : LW_GUESS) : x;
            nlead = fix == 0 ? LW_CPP : 1u;
            run = true;
        }
        x = 0;
    }
    LW_STAMP(5);
    X0 = s.lw_wx[flast][0];
    X = x;
    if (ok && a.sdiag && tid == 0)
        for (uint32_t k = 0; k < LW_PROF; ++k) a.sdiag[(size_t)(p0 / a.sbp) * LW_PROF + k] = s.lw_prof[k];
    return ok;
}

// Stride check of one staged piece without a barrier: the run's geometry
// (entry, R, count) follows from the uniform header at X alone, so the exit
// is known at once; the per-lane compares only decide whether the batch is
// resolved and are OR-reduced by the caller (after piece 0, so a non-stride
// table leaves after one piece, then once per batch).  Returns false when X
// itself cannot start a run.
__device__ __forceinline__ bool stride_geom(const uint8_t* data, uint64_t base, uint64_t len,
                                           uint32_t clen, uint64_t X, PieceSum& ps, int& bad) {
    ps.x = X;
    if (X >= base + clen) {  // no record starts in this piece
        ps.count = 0;
        ps.R = 0;
        ps.kl = ps.vl = 0;
        ps.kind = PK_EMPTY;
        return true;
    }
    const uint32_t xr = (uint32_t)(X - base);
    if (X + 16 > len) return false;
    uint64_t kl, vl;
    lds_header(data, xr, kl, vl);
    kl = uni(kl);
    vl = uni(vl);
    if (kl > ~0ull - vl || kl + vl > len - X - 16 || ((kl >> 32) | (vl >> 32))) return false;
    const uint64_t R = 16 + kl + vl;
    const uint32_t m = (uint32_t)((clen - xr + R - 1) / R);  // records starting in [xr, clen)
    if (X + m * R > len) return false;                       // the last one would not fit
    for (uint32_t t = 1 + threadIdx.x; t < m; t += THREADS)
        bad |= !hdr_eq(data, xr + (uint32_t)(t * R), kl, vl);
    ps.count = m;
    ps.R = R;
    ps.kl = (uint32_t)kl;
    ps.vl = (uint32_t)vl;
    ps.kind = PK_STRIDE;
    return true;
}

// Thread 0: publish batch b (read by decode_kernel after the kernel boundary),
// count its records per group, then settle the two links it is part of.
__device__ __forceinline__ void spec_publish(const DecodeArgs& a, SpecBatch* sb, uint32_t b,
                                             uint64_t X0, uint64_t X, uint64_t total, bool ok,
                                             uint32_t code) {
    SpecBatch o;
    o.x0 = X0;
    o.exit = X;
    o.count = (uint32_t)total;
    o.ok = ok ? 1u : 0u;
    o.pad = code;
    sb[b] = o;
    atomicAdd(&a.gsum[b / SPEC_GROUP], (unsigned long long)total);
    if (!ok || (b == 0 && X0 != a.entry)) mark_bad(a.ctl, a.nspec, b);
    if (b > 0) link_arrive(a, b, 0 - X0);
    if (b + 1 < a.nspec) link_arrive(a, b + 1, X);
}

// KPRE (compaction mode, a.kpre_tag != 0): stride pieces also leave their
// records' key prefixes in their span-scratch slots.  The prefixes of piece i
// are computed from LDS into registers after it is verified and stored during
// the next iteration, before the next piece's loads are issued: stores issued
// behind the loads would make the wait for those loads (vmcnt counts both, in
// order) wait for the stores too (measured: the pre-pass 173 -> 221 us with
// the stores right after the verification).
//
// Piece staging (HG_SPEC_GLDS): the pieces stream into two LDS buffers by
// global_load_lds (nontemporal, 4 x 1 KiB per wave per piece), piece i + 1 in
// flight while piece i is checked, with counted vmcnt waits and raw
// s_barriers (a __syncthreads() would wait for the DMA in flight too).  The
// register-staged form (loads into v, ds_write after barrier (A)) streams at
// ~6.4 TB/s, the LDS-DMA form at ~7.0 (tools/probes/sweep_probe.hip,
// profiles/r4_sweep_glds.log).  The table's tail piece is staged from
// registers (load16 zero-fills past the bytes present).
#ifndef HG_SPEC_GLDS
#define HG_SPEC_GLDS 1
#endif
// HG_LW_FUSE: the lane walks of SB_HOP_SMALL batches run in the pre-pass
// workgroup itself (no decode_lw_kernel launch); the second piece buffer is
// then also lw_batch's chunk buffer of waves 2 and 3.  With the pieces
// staged by LDS-DMA the pre-pass already needs the lane walks' LDS (4
// workgroups per CU either way), so the fused kernel costs the stride path
// nothing: same box, 3 rounds (profiles/r4_ab_fuse.log): cfg 2 0.2034 ->
// 0.2028 ms, small 0.1471 -> 0.1407, medium 0.191 -> 0.185, zero-valued
// small 0.1565 -> 0.1505, zero-valued 400-1200 B 0.276 -> 0.271, 400-1200 B
// 0.150 -> 0.152.
#ifndef HG_LW_FUSE
#define HG_LW_FUSE 1
#endif
#if HG_LW_FUSE && !HG_SPEC_GLDS
#error "HG_LW_FUSE needs HG_SPEC_GLDS (the second buffer)"
#endif
constexpr uint32_t SPEC_ALT_BYTES = HG_LW_FUSE ? PIECE + 512 : PIECE + 64;  // a piece + halo and zeros
// HG_SPEC_STWAIT: the wait for piece i's DMA lets the stores the wave issued
// after the previous wait (thread 0's piece record) stay in flight: they sit
// between piece i's DMA and piece i + 1's in the wave's in-order vmcnt queue,
// so a plain vmcnt(GPT) also waited for their write acknowledgement every
// piece.  Same box, 3 rounds each (profiles/r6_ab_store_wait.log): cfg 2
// 0.2025 / 0.1971 / 0.1987 -> 0.2005 / 0.1953 / 0.1974 ms, small and medium
// records ~1 % faster.  Not in compaction mode (KPRE): counting its prefix
// stores out too took that kernel from 114 to 122 VGPRs and the cfg 5 legs
// 9.0 -> 10.4 ms and 1.22 -> 1.45 ms.
#ifndef HG_SPEC_STWAIT
#define HG_SPEC_STWAIT 1
#endif

__device__ __forceinline__ bool spec_dma(const DecodeArgs& a, uint32_t p, uint8_t* dst) {
    const uint64_t base = (uint64_t)p * PIECE;
    if (base + PIECE > a.rlen) return false;
    const uint32_t lane = threadIdx.x & 63u, wid = threadIdx.x >> 6;
#pragma unroll
    for (uint32_t q = 0; q < GPT; ++q) {
        const uint32_t g0 = q * THREADS + wid * 64;  // granule layout as spec_stage's
        dma16(static_cast<const void*>(a.sst + base + (uint64_t)(g0 + lane) * 16), dst + g0 * 16);
    }
    return true;
}
__device__ __forceinline__ void raw_barrier() {
    __asm__ volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}


template <bool KPRE>
__device__ void spec_body(const DecodeArgs& a, SpecBatch* sb, SpecPiece* sp, uint32_t blk) {
    __shared__ SpecSmem s;
    const uint32_t tid = threadIdx.x;
    const uint8_t* data = reinterpret_cast<const uint8_t*>(s.data64);
    const uint32_t b = blk;
    const uint32_t p0 = b * a.sbp;
    const uint32_t np = min(a.sbp, a.npieces - p0);
#ifdef HG_SPEC_TIMELINE  // diagnostics build (tools/spec_timeline.py): realtime stamps
    uint64_t* const tl = reinterpret_cast<uint64_t*>(a.scratch + (size_t)p0 * MAX_REC_PIECE);
    if (tid == 0) tl[0] = __builtin_amdgcn_s_memrealtime();
#endif
#if HG_SPEC_GLDS
    __shared__ uint64_t spec_alt[SPEC_ALT_BYTES / 8];
    uint8_t* const buf0 = reinterpret_cast<uint8_t*>(s.data64);
    uint8_t* const buf1 = reinterpret_cast<uint8_t*>(spec_alt);
    bool dma_cur = spec_dma(a, p0, buf0);
#else
    uint4 v[GPT];
    load_piece(a, p0, v);
#endif
    uint4 h = make_uint4(0, 0, 0, 0);
    // (the halos by DMA behind piece 0's, so that piece 0's halo store no
    // longer waits for the next piece's DMA, measured no faster: cfg 2
    // 0.2037 vs 0.1999 ms, same box, profiles/r4_ab_first_piece.log)
    if (tid < np) h = load16(a, (uint64_t)(p0 + tid + 1) * PIECE);
    uint64_t X = 0, X0 = 0, total = 0;
    bool ok = true, hop = false;
    int bad = 0;
    constexpr uint32_t KPT = KPRE ? MAX_REC_PIECE / THREADS : 1;  // prefixes per thread
    uint4 pf[KPT];
    uint32_t pf_n = 0, pf_piece = 0;  // the pending prefixes (KPRE)
    // The flushes return a lower bound of the store instructions this wave
    // issued (one per 16-byte store; a wave issues one when its first lane
    // does), for the counted waits of the LDS-DMA staging.
    const uint32_t w64 = tid & ~63u;  // the wave's first thread
    uint32_t nst = 0;  // store instructions the wave issued since its last wait (lower bound)
    auto flush_prefixes = [&]() -> uint32_t {
        if (!KPRE || !pf_n) return 0u;
        hg_span* slot = a.scratch + (size_t)pf_piece * MAX_REC_PIECE;
        uint32_t n = 0;
#pragma unroll
        for (uint32_t k = 0; k < KPT; ++k) {
            if (tid + k * THREADS < pf_n) *reinterpret_cast<uint4*>(slot + tid + k * THREADS) = pf[k];
            n += w64 + k * THREADS < pf_n ? 1u : 0u;
        }
        if (tid == 0) piece_tags(a)[pf_piece] = a.kpre_tag;
        pf_n = 0;
        return n + (w64 == 0 ? 1u : 0u);
    };
    // Two barriers per piece: (A) the previous piece is done with LDS; stage
    // v and the halo and put the next piece's loads in flight before (B).
    for (uint32_t i = 0; i < np; ++i) {
        const uint32_t p = p0 + i;
        const uint64_t base = (uint64_t)p * PIECE;
        const uint64_t rem = a.len - base;
        const uint32_t clen = piece_clen(a, base);
#if HG_SPEC_GLDS
        uint8_t* const cur = (i & 1) ? buf1 : buf0;
        data = cur;
        raw_barrier();  // (A) every wave is done with the other buffer (piece i - 1)
        const bool dma_next = i + 1 < np && spec_dma(a, p + 1, (i & 1) ? buf0 : buf1);
        // (and every store before the DMA, unless HG_SPEC_STWAIT counts them out)
        lw_wait_vm(dma_next ? GPT + (HG_SPEC_STWAIT && !KPRE ? nst : 0u) : 0);
        nst = flush_prefixes();  // (a lower bound of the wave's store instructions)
#ifdef HG_SPEC_TIMELINE
        if (i == 0 && tid == 0) tl[3] = __builtin_amdgcn_s_memrealtime();
#endif
        if (!dma_cur) {                  // the tail piece
#pragma unroll
            for (uint32_t q = 0; q < GPT; ++q)
                *reinterpret_cast<uint4*>(cur + (q * THREADS + tid) * 16) =
                    load16(a, base + (q * THREADS + tid) * 16);
        }
        if (i == 0 && tid < np) s.halo[tid] = h;
        if (tid < 4)  // thread 0 reads back its own halo write when i == 0
            *reinterpret_cast<uint4*>(cur + PIECE + tid * 16) = tid == 0 ? s.halo[i] : make_uint4(0, 0, 0, 0);
        raw_barrier();     // (B)
        dma_cur = dma_next;
#else
        __syncthreads();  // (A)
        if (i == 0 && tid < np) s.halo[tid] = h;
        spec_stage(s, v, i);
        flush_prefixes();  // the previous piece's prefixes, ahead of the next loads
        if (i + 1 < np) load_piece(a, p + 1, v);  // in flight while this piece is verified
        __syncthreads();  // (B)
#endif
        if (i == 0 && b == 0) {
            X = X0 = a.entry;  // the first batch's entry is known exactly
        } else if (i == 0) {
            if (tid < 64) {
                const uint32_t f = stride_guess(data, rem, clen, a.hz);
                if (tid == 0) s.guess = f;
            }
            __syncthreads();
            const uint32_t f = uni(s.guess);
#ifdef HG_SPEC_TIMELINE
            if (tid == 0) tl[4] = __builtin_amdgcn_s_memrealtime();
#endif
            if (f == NO_GUESS) {  // no stride run: large records are hopped, others left
                hop = true;
                break;
            }
            X = X0 = base + f;
        }
        PieceSum ps;
        if (!stride_geom(data, base, a.len, clen, X, ps, bad)) {
            ok = false;
            break;
        }
        if (i == 0 && __syncthreads_or(bad)) {  // not a stride table: leave after one piece
            hop = true;
            break;
        }
#ifdef HG_SPEC_TIMELINE
        if (i == 0 && tid == 0) tl[1] = __builtin_amdgcn_s_memrealtime();
#endif
        if (tid == 0) {
            SpecPiece o;
            o.x = ps.x;
            o.R = ps.R;
            o.kl = ps.kl;
            o.vl = ps.vl;
            o.count = ps.count;
            o.pad = 0;
            sp[p] = o;
        }
        if (HG_SPEC_STWAIT && !KPRE && w64 == 0) ++nst;  // thread 0's piece record: wave 0 only
        if (KPRE && ps.kind == PK_STRIDE) {  // compaction mode: key prefixes from LDS
            const uint32_t xr = (uint32_t)(X - base), R = (uint32_t)ps.R;
#pragma unroll
            for (uint32_t k = 0; k < KPT; ++k) {
                const uint32_t t = tid + k * THREADS;
                if (t >= ps.count) continue;
                const uint32_t kp = xr + t * R + 16;  // key start, piece-relative
                uint64_t lo, hi;
                if (kp + 16 <= PIECE + 16) {           // staged (the halo holds 16 more bytes)
                    lds_header(data, kp, lo, hi);
                } else {
                    const uint4 w = load16(a, base + kp);
                    lo = ((uint64_t)w.y << 32) | w.x;
                    hi = ((uint64_t)w.w << 32) | w.z;
                }
                pf[k] = key_prefix_be(lo, hi, ps.kl);
            }
            pf_n = ps.count;
            pf_piece = p;
        }
        total += ps.count;
        X = ps.kind == PK_EMPTY ? X : X + (uint64_t)ps.count * ps.R;
    }
#if HG_SPEC_GLDS
    lw_wait_vm(0);  // a break leaves the next piece's DMA in flight
#endif
    flush_prefixes();
    if (hop) {
        bad = 0;
        ok = hop_batch(s, a, p0, np, sp, X0, X, total);
    }
    if (__syncthreads_or(bad)) ok = false;  // some piece's run broke: not resolved here
#ifdef HG_SPEC_TIMELINE
    if (tid == 0) tl[2] = __builtin_amdgcn_s_memrealtime();
#endif

#if HG_LW_FUSE
    if (HG_LW && !ok && hop && __builtin_amdgcn_readfirstlane(s.hcode) == SB_HOP_SMALL) {
        uint32_t why = 0;
        const bool lok = lw_batch<!KPRE>(s, spec_alt, a, p0, np, sp, X0, X, total, why);
        if (tid == 0) spec_publish(a, sb, b, X0, X, total, lok, lok ? SB_LW : (SB_LW_DEAD | (why << 8)));
        return;
    }
#endif
    if (tid == 0) {
        const uint32_t code = hop ? s.hcode : (ok ? SB_STRIDE : SB_STRIDE_BROKE);
        if (HG_LW && !HG_LW_FUSE && !ok && code == SB_HOP_SMALL) {
            // small records: left to decode_lw_kernel, which publishes the
            // batch (its counts and links) once its lane walks are done
            SpecBatch o;
            o.x0 = o.exit = 0;
            o.count = 0;
            o.ok = 0;
            o.pad = SB_HOP_SMALL;
            sb[b] = o;
        } else {
            spec_publish(a, sb, b, X0, X, total, ok, code);
        }
    }
}

// The lane-walk mode as its own launch between the pre-pass and decode_kernel:
// only batches the pre-pass left as SB_HOP_SMALL do work (every other
// workgroup returns at once), so the stride / hop pre-pass keeps its own
// register and LDS budget (81 VGPRs, 5 waves/SIMD, 23 KB; the lane walks need
// 108 and 40 KB, which cost the fixed-stride headline 2 %).
__device__ void lw_body(const DecodeArgs& a, SpecBatch* sb, SpecPiece* sp, uint32_t b) {
    __shared__ SpecSmem s;
    __shared__ uint64_t lw_alt[(PIECE + 512) / 8];  // lane-walk chunk buffers of waves 2 and 3
#ifdef HG_LW_PAD  // occupancy experiments (A/B builds): extra LDS per workgroup
    __shared__ uint8_t lw_pad[HG_LW_PAD];
    if (a.len == 3) {
        lw_pad[threadIdx.x] = (uint8_t)threadIdx.x;
        __syncthreads();
        if (a.sdiag) a.sdiag[0] = lw_pad[(threadIdx.x + 1) & 255u];
    }
#endif
    if (__builtin_amdgcn_readfirstlane(sb[b].pad) != SB_HOP_SMALL) return;
    const uint32_t p0 = b * a.sbp;
    const uint32_t np = min(a.sbp, a.npieces - p0);
    uint64_t X0 = 0, X = 0, total = 0;
    uint32_t why = 0;
    const bool ok = lw_batch(s, lw_alt, a, p0, np, sp, X0, X, total, why);
    // SpecBatch.pad bits 8..15 of a failed batch: 1 the first quarter's guessed
    // entry, 2 a quarter entered exactly, 3 too many re-streams
    if (threadIdx.x == 0) spec_publish(a, sb, b, X0, X, total, ok, ok ? SB_LW : (SB_LW_DEAD | (why << 8)));
}

__global__ __launch_bounds__(THREADS, 4) void decode_spec_kernel(DecodeArgs a, SpecBatch* sb,
                                                              SpecPiece* sp) {
    // the other half of a double-buffered control region, cleared for the
    // next call (no workgroup of this call reads it): that call then needs no
    // memset launch ahead of its pre-pass (hgk_decode_launch_ctl)
    if (a.zero_next)
        for (uint32_t i = blockIdx.x * THREADS + threadIdx.x; i < a.zero_next_n16;
             i += gridDim.x * THREADS)
            a.zero_next[i] = make_uint4(0u, 0u, 0u, 0u);
#ifdef HG_SPEC_SWAP_PAIRS  // diagnostics: workgroup b takes batch b ^ 1 (XCD vs address)
    spec_body<false>(a, sb, sp, (blockIdx.x ^ 1u) < a.nspec ? blockIdx.x ^ 1u : blockIdx.x);
#else
    spec_body<false>(a, sb, sp, blockIdx.x);
#endif
}

__global__ __launch_bounds__(THREADS, 4) void decode_lw_kernel(DecodeArgs a, SpecBatch* sb,
                                                            SpecPiece* sp) {
    lw_body(a, sb, sp, blockIdx.x);
}

// ---- many tables in one launch ---------------------------------------------------
// hg_decode_batch_dev_async: every table keeps its own DecodeArgs (own
// workspace slice: controls, statuses, scratch, pre-pass records) and the
// single-table code runs unchanged on it; a workgroup finds its table from
// the prefix sums of the per-table grids (binary search over <= ntab + 1
// words).  Tickets and look-backs are per table, so the ordering argument of
// the single-table decode holds inside each table.
__device__ __forceinline__ uint32_t find_table(const uint32_t* pre, uint32_t ntab, uint32_t blk) {
    uint32_t lo = 0, hi = ntab;  // pre[lo] <= blk < pre[hi]
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (pre[mid] <= blk) lo = mid; else hi = mid;
    }
    return uni(lo);
}

// Zero every table's control region; empty tables get their (empty) result.
__global__ __launch_bounds__(THREADS) void decode_zero_multi(const DecodeArgs* tabs,
                                                             const uint64_t* zero_bytes,
                                                             uint32_t ntab) {
    const uint32_t t = blockIdx.x;
    if (t >= ntab) return;
    unsigned long long* w = reinterpret_cast<unsigned long long*>(tabs[t].ctl);
    const uint64_t n = zero_bytes[t] / 8;
    for (uint64_t i = threadIdx.x; i < n; i += THREADS) w[i] = 0;
    if (tabs[t].len == 0 && threadIdx.x == 0) {
        hg_decode_result r;
        r.n_records = 0;
        r.kind = HG_OK;
        r.reserved = 0;
        r.err_offset = 0;
        *tabs[t].result = r;
    }
}

template <bool KPRE>
__global__ __launch_bounds__(THREADS, 4) void decode_spec_multi(const DecodeArgs* tabs,
                                                             const uint32_t* pre, uint32_t ntab) {
    const uint32_t t = __builtin_amdgcn_readfirstlane(find_table(pre, ntab, blockIdx.x));
    const DecodeArgs a = tabs[t];
    const uint32_t blk = blockIdx.x - __builtin_amdgcn_readfirstlane(pre[t]);
    // the table's region of the next call's control half (hgk_multi_ctl).
    // Not in compaction mode: there the loop took the kernel from 114 to 122
    // VGPRs and 223 to 438 us on the cfg 5 leg (its piece staging is that
    // sensitive, see the round-4 notes); those calls keep the zero kernel.
    if (!KPRE && a.zero_next)
        for (uint32_t i = blk * THREADS + threadIdx.x; i < a.zero_next_n16; i += a.nspec * THREADS)
            a.zero_next[i] = make_uint4(0u, 0u, 0u, 0u);
    spec_body<KPRE>(a, a.sbatch, const_cast<SpecPiece*>(a.spiece), blk);
}

__global__ __launch_bounds__(THREADS, 4) void decode_lw_multi(const DecodeArgs* tabs,
                                                           const uint32_t* pre, uint32_t ntab) {
    const uint32_t t = __builtin_amdgcn_readfirstlane(find_table(pre, ntab, blockIdx.x));
    const DecodeArgs a = tabs[t];
    lw_body(a, a.sbatch, const_cast<SpecPiece*>(a.spiece),
            blockIdx.x - __builtin_amdgcn_readfirstlane(pre[t]));
}

// Same register bound as decode_kernel (4 waves/SIMD); the table index is
// block-uniform, so its arguments are fetched with scalar loads into a copy.
__global__ __launch_bounds__(THREADS, HG_DEC_WAVES) void decode_multi(const DecodeArgs* tabs,
                                                           const uint32_t* pre, uint32_t ntab) {
    const uint32_t t = __builtin_amdgcn_readfirstlane(find_table(pre, ntab, blockIdx.x));
    const DecodeArgs a = tabs[t];
    decode_body<false>(a, blockIdx.x - __builtin_amdgcn_readfirstlane(pre[t]));
}

// ---- compaction mode: merge entries ------------------------------------------------
// The merge's entries (hg_merge.hip MEnt: the key's bytes [0, 16) big-endian,
// klen, entry index g = run_off[t] + record) with its order check fused (each
// entry against its predecessor in the table), one workgroup per pre-pass
// batch of the batched decode -- instead of merge_prep_kernel's per-record
// span -> piece tag -> prefix load chains (124 us on the cfg 5 leg).  A batch
// the resolved prefix emitted (its general batch wholly before the first
// unresolved pre-pass batch) whose pieces are all stride runs with the key
// prefixes the pre-pass left (current tag) takes its records' indices from the
// pre-pass counts (spec_base) and its prefixes from the pieces' scratch slots:
// contiguous loads and stores.  Any other batch finds the records starting in
// its bytes by a search over the table's spans and reads each key through its
// span.  Every record starts in exactly one batch, so the tables are covered.
struct KEnt {  // hg_merge.hip MEnt
    uint64_t p0, p1;
    uint32_t klen, gd;
};
static_assert(sizeof(KEnt) == 24, "merge entry layout");

// Entry of record i of the table (its key's first 16 bytes through its span).
__device__ __forceinline__ KEnt kent_of(const DecodeArgs& a, uint64_t i, uint64_t g) {
    const hg_span sp = a.spans[i];
    const uint64_t ko = sp.off - a.obase + 16;
    uint64_t lo = 0, hi = 0;
    if (ko + 16 <= a.len) {
        const uint4 w = *reinterpret_cast<const uint4*>(a.sst + ko);
        lo = ((uint64_t)w.y << 32) | w.x;
        hi = ((uint64_t)w.w << 32) | w.z;
    } else {
        for (uint32_t k = 0; k < 16 && ko + k < a.len; ++k) {
            const uint64_t b = a.sst[ko + k];
            if (k < 8) lo |= b << (8 * k);
            else hi |= b << (8 * (k - 8));
        }
    }
    const uint4 v = key_prefix_be(lo, hi, sp.klen);
    KEnt e;
    e.p0 = ((uint64_t)v.y << 32) | v.x;
    e.p1 = ((uint64_t)v.w << 32) | v.z;
    e.klen = sp.klen;
    e.gd = (uint32_t)g;
    return e;
}

// Key order of records xi, yi of the table (Vec<u8> Ord, src/format.rs:5).
__device__ int kent_cmp(const DecodeArgs& a, const KEnt& x, uint64_t xi, const KEnt& y, uint64_t yi) {
    if (x.p0 != y.p0) return x.p0 < y.p0 ? -1 : 1;
    if (x.p1 != y.p1) return x.p1 < y.p1 ? -1 : 1;
    if (x.klen <= 16 || y.klen <= 16) return x.klen < y.klen ? -1 : x.klen > y.klen ? 1 : 0;
    const uint8_t* kx = a.sst + (a.spans[xi].off - a.obase) + 16;
    const uint8_t* ky = a.sst + (a.spans[yi].off - a.obase) + 16;
    const uint32_t m = min(x.klen, y.klen);
    for (uint32_t i = 16; i < m; ++i)
        if (kx[i] != ky[i]) return kx[i] < ky[i] ? -1 : 1;
    return x.klen < y.klen ? -1 : x.klen > y.klen ? 1 : 0;
}

// First record of the table (n records) whose span starts at or after `off`
// (spans ascend): a 64-ary search by one wave, every lane gets it.
__device__ uint64_t span_lower_bound(const DecodeArgs& a, uint64_t n, uint64_t off) {
    const uint32_t lane = threadIdx.x & 63u;
    uint64_t lo = 0, hi = n;  // answer in [lo, hi]
    while (hi - lo > 64) {
        const uint64_t step = (hi - lo) / 64;
        const uint64_t probe = lo + (uint64_t)(lane + 1) * step;  // <= lo + 64 step <= hi
        const bool below = probe < hi && a.spans[probe].off < off;
        const unsigned long long m = __ballot(below);
        const uint32_t k = m ? 64u - (uint32_t)__clzll((long long)m) : 0u;  // lanes 0..k-1 below
        const uint64_t nlo = k ? lo + (uint64_t)k * step + 1 : lo;
        hi = k < 64 ? min(hi, lo + (uint64_t)(k + 1) * step) : hi;
        lo = nlo;
    }
    const bool below = lo + lane < hi && a.spans[lo + lane].off < off;
    return lo + (uint64_t)__popcll(__ballot(below));
}

constexpr uint32_t KE_U = 4;  // records per thread per step (their loads overlap)
__global__ __launch_bounds__(THREADS) void decode_entries_multi(const DecodeArgs* tabs, uint32_t ntab,
                                                                const uint32_t* pre,
                                                                const uint64_t* run_off, KEnt* ent,
                                                                unsigned long long* err) {
    __shared__ KEnt st[THREADS * KE_U];
    __shared__ uint64_t pb[SPEC_BP + 1];  // fast: batch-relative index of each piece's first record
    __shared__ uint32_t pkl[SPEC_BP];
    __shared__ KEnt last;                 // the record before the step's first
    __shared__ uint64_t srange[2];
    const uint32_t tid = threadIdx.x;
    const uint32_t t = __builtin_amdgcn_readfirstlane(find_table(pre, ntab, blockIdx.x));
    const DecodeArgs& a = tabs[t];
    const uint32_t e = blockIdx.x - __builtin_amdgcn_readfirstlane(pre[t]);
    if (e >= a.nspec) return;
    const uint32_t q0 = e * a.sbp, n = min(a.sbp, a.npieces - q0);
    const uint64_t nrec = run_off[t + 1] - run_off[t];
    bool ok = a.kpre_tag != 0 && min((e / a.q + 1) * a.q, a.nspec) <= first_bad(a.ctl, a.nspec);
    uint32_t cnt = 0;
    if (ok && tid < n) {
        const SpecPiece q = a.spiece[q0 + tid];
        cnt = q.count;
        ok = cnt == 0 || (q.pad == SP_STRIDE && piece_tags(a)[q0 + tid] == a.kpre_tag);
        pkl[tid] = q.kl;
    }
    const bool fast = !__syncthreads_or(!ok);
    if (tid < 64) {
        uint64_t r_lo, r_hi;
        if (fast) {
            const uint32_t incl = dpp_sum_incl(cnt);  // n <= SPEC_BP = 64: wave 0 holds them
            if (tid < n) pb[tid + 1] = incl;
            r_lo = spec_base(a, e);
            r_hi = r_lo + __builtin_amdgcn_readlane((int)incl, 63);
        } else {  // the records starting in the batch's bytes
            r_lo = span_lower_bound(a, nrec, a.obase + (uint64_t)q0 * PIECE);
            r_hi = q0 + n >= a.npieces ? nrec
                                       : span_lower_bound(a, nrec, a.obase + (uint64_t)(q0 + n) * PIECE);
        }
        if (tid == 0) {
            pb[0] = 0;
            srange[0] = r_lo;
            srange[1] = r_hi;
            if (r_lo > 0 && r_lo < r_hi) last = kent_of(a, r_lo - 1, run_off[t] + r_lo - 1);
        }
    }
    __syncthreads();
    const uint64_t r_lo = srange[0], total = srange[1] - r_lo, g0 = run_off[t] + r_lo;
    for (uint64_t r0 = 0; r0 < total; r0 += THREADS * KE_U) {
        KEnt m[KE_U];
#pragma unroll
        for (uint32_t u = 0; u < KE_U; ++u) {
            const uint64_t r = r0 + u * THREADS + tid;
            m[u] = KEnt{};
            if (r >= total) continue;
            if (fast) {
                uint32_t lo = 0, hi = n;  // the piece: last i with pb[i] <= r (empty pieces
                while (hi - lo > 1) {     // share their successor's base: the search passes them)
                    const uint32_t mid = (lo + hi) >> 1;
                    if (pb[mid] <= r) lo = mid;
                    else hi = mid;
                }
                typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
                const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(
                    a.scratch + (size_t)(q0 + lo) * MAX_REC_PIECE + (r - pb[lo])));
                m[u].p0 = ((uint64_t)v.y << 32) | v.x;
                m[u].p1 = ((uint64_t)v.w << 32) | v.z;
                m[u].klen = pkl[lo];
                m[u].gd = (uint32_t)(g0 + r);
            } else {
                m[u] = kent_of(a, r_lo + r, g0 + r);
            }
        }
#pragma unroll
        for (uint32_t u = 0; u < KE_U; ++u) st[u * THREADS + tid] = m[u];
        __syncthreads();
        const uint32_t nv = (uint32_t)min((uint64_t)THREADS * KE_U, total - r0);
#pragma unroll
        for (uint32_t u = 0; u < KE_U; ++u) {  // order check against the predecessor
            const uint32_t l = u * THREADS + tid;
            const uint64_t r = r_lo + r0 + l;  // the record
            if (l >= nv || r == 0) continue;
            const KEnt pv = l ? st[l - 1] : last;
            if (kent_cmp(a, pv, r - 1, m[u], r) >= 0) atomicMin(err, (unsigned long long)(run_off[t] + r));
        }
        const uint64_t* s8 = reinterpret_cast<const uint64_t*>(st);
        uint64_t* o8 = reinterpret_cast<uint64_t*>(ent + g0 + r0);
        for (uint32_t w = tid; w < 3 * nv; w += THREADS) o8[w] = s8[w];
        __syncthreads();
        if (tid == 0) last = st[nv - 1];
        __syncthreads();
    }
}

}  // namespace hgk

namespace {
struct DecodeLayout {
    uint64_t npieces, nbatches, status_words, scratch_off, nspec, sbatch_off, spiece_off, bytes;
    uint64_t gsum_off, link_off, status_off, ptag_off;
};
DecodeLayout decode_layout(uint64_t len) {
    using namespace hgk;
    DecodeLayout l;
    l.npieces = (len + PIECE - 1) / PIECE;
    l.nbatches = (l.npieces + BATCH_MIN - 1) / BATCH_MIN;  // most batches any launch uses
    // [DecodeCtl | group sums | pair links | statuses] are zeroed per call
    // (up to the statuses in use), then the scratch and pre-pass records.
    l.nspec = (l.npieces + SPEC_BP_MIN - 1) / SPEC_BP_MIN;  // most pre-pass batches
    l.gsum_off = sizeof(DecodeCtl);
    l.link_off = l.gsum_off + ((l.nspec + SPEC_GROUP - 1) / SPEC_GROUP) * 8;
    l.status_off = (l.link_off + l.nspec * 8 + 255) & ~255ull;
    l.status_words = 2 * l.nbatches;
    l.scratch_off = (l.status_off + l.status_words * 8 + 255) & ~255ull;
    l.sbatch_off = l.scratch_off + l.npieces * MAX_REC_PIECE * sizeof(hg_span);
    l.spiece_off = l.sbatch_off + ((l.nspec * sizeof(SpecBatch) + 255) & ~255ull);
    l.ptag_off = l.spiece_off + ((l.npieces * sizeof(SpecPiece) + 255) & ~255ull);
    l.bytes = l.ptag_off + ((l.npieces * 4 + 255) & ~255ull);
    return l;
}
}  // namespace

extern "C" uint64_t hgk_decode_workspace_bytes(uint64_t len) { return decode_layout(len).bytes; }

// Where a table's workspace keeps its span scratch, piece records and piece
// tags (compaction mode: the merge's entry builder reads key prefixes there).
extern "C" void hgk_decode_ws_layout(uint64_t len, uint64_t* scratch_off, uint64_t* spiece_off,
                                     uint64_t* ptag_off) {
    const DecodeLayout l = decode_layout(len);
    *scratch_off = l.scratch_off;
    *spiece_off = l.spiece_off;
    *ptag_off = l.ptag_off;
}

// Diagnostics (tools/spec_diag.py): geometry of the last launch.
static uint64_t g_last_launch[8];
extern "C" void hgk_decode_last_layout(uint64_t* out) {
    for (int i = 0; i < 8; ++i) out[i] = g_last_launch[i];
}

namespace {
// Workgroups of `kernel` (256 threads) resident at once on the current device.
template <typename K>
uint32_t resident_workgroups(K kernel, int slot) {
    static int cached[8][64] = {{0}};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) dev = 0;
    if (!cached[slot][dev]) {
        int per_cu = 0, cus = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, hgk::THREADS, 0) !=
                hipSuccess ||
            per_cu <= 0)
            per_cu = 1;
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
            cus <= 0)
            cus = 1;
        cached[slot][dev] = per_cu * cus;
    }
    return (uint32_t)cached[slot][dev];
}

uint64_t knob_or(const char* name, uint64_t dflt) {
    const int64_t v = hgk_knob(name, 0);
    return v > 0 ? (uint64_t)v : dflt;
}

// Pieces per general batch: about one round of batches over decode_kernel's
// resident grid (each batch pays one look-back + emission tail), a power of
// two in [BATCH_MIN, BATCH] (HG_DECODE_BP overrides).  Pieces per pre-pass
// batch: long-lived streams win -- enough pieces that the pre-pass grid is
// about 4 workgroups per CU, in [SPEC_BP_MIN, SPEC_BP] and at most the general
// batch (a general batch is whole pre-pass batches).  Measured on cfg2 (1 GiB,
// nontemporal loads, tools/sweep_spec.sh): 8 pieces 0.223 ms, 16: 0.218,
// 32: 0.207, 64 (1024 workgroups): 0.197-0.200 ms.  HG_DECODE_SBP overrides.
uint32_t pow2_in(uint64_t want, uint32_t lo, uint32_t hi) {
    uint32_t v = lo;
    while (v < hi && v < want) v <<= 1;
    return v;
}
uint32_t general_pieces(uint64_t npieces, uint32_t resident) {
    using namespace hgk;
    return pow2_in(knob_or("HG_DECODE_BP", (npieces + resident - 1) / resident), BATCH_MIN, BATCH);
}
uint32_t spec_pieces(uint32_t bp, uint64_t npieces, uint32_t cus) {
    using namespace hgk;
    const uint64_t want = (npieces + 4ull * cus - 1) / (4ull * cus);
    const uint32_t s = pow2_in(knob_or("HG_DECODE_SBP", want), SPEC_BP_MIN, SPEC_BP);
    return s < bp ? s : bp;
}
// Wide hop segments (half the guess rounds, chains twice as long) pay off
// while the pre-pass grid fits the resident workgroups at once; a grid of
// more batches than resident slots (cfg 4's 32 tables: 2,048 pre-pass
// workgroups over ~1,024 slots) runs faster on 64 KiB segments throughout
// (same box, 2 rounds, profiles/r5_ab_hop_geometry.log: cfg 4 0.227-0.228 ->
// 0.2145-0.2151 ms; one 793 MB table of 8 B-4 KiB values, 757 workgroups,
// 0.0857 -> 0.0907 ms the other way).
uint32_t hop_wide_cand(uint64_t grid, uint32_t resident) {
    return grid > resident ? 0u : hgk::HOP_WIDE_CAND;
}
uint32_t device_cus() {
    static int cached[64] = {0};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) dev = 0;
    if (!cached[dev]) {
        int cus = 0;
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
            cus <= 0)
            cus = 1;
        cached[dev] = cus;
    }
    return (uint32_t)cached[dev];
}
}  // namespace

namespace {
// DecodeArgs of one table with the given batch geometry (bp pieces per
// general batch, sbp per pre-pass batch); zero_bytes = control region to zero.
// Range form (hgk_decode_range_launch): bytes [begin, len) readable, records
// starting in [entry, stop) decoded, entry an exact record start; the
// workspace is laid out for stop - begin bytes.
hgk::DecodeArgs make_args(const uint8_t* d_sst, uint64_t len, hg_span* d_spans, uint64_t cap,
                          hg_decode_result* d_result, void* d_ws, uint32_t* d_diag, uint32_t bp,
                          uint32_t sbp, uint64_t& zero_bytes, uint64_t begin = 0,
                          uint64_t stop = ~0ull, uint64_t entry = 0, bool range = false,
                          uint64_t rlen = ~0ull, uint32_t kpre_tag = 0, void* d_ctl = nullptr) {
    using namespace hgk;
    if (stop > len) stop = len;
    if (rlen > len) rlen = len;
    d_sst += begin;
    len -= begin;
    stop -= begin;
    rlen -= begin;
    const DecodeLayout l = decode_layout(stop);
    // Zero high bytes every genuine length field must have: any record fits
    // in len bytes, so klen, vlen < 2^(8*nb) with nb = bytes needed for len.
    uint32_t nb = 0;
    for (uint64_t x = len; x; x >>= 8) ++nb;
    DecodeArgs a;
    a.sst = d_sst;
    a.len = len;
    a.rlen = rlen;
    a.stop = stop;
    a.entry = entry - begin;
    a.obase = begin;
    a.range = range ? 1u : 0u;
    a.spans = d_spans;
    a.cap = cap;
    a.result = d_result;
    char* ws = static_cast<char*>(d_ws);
    // the control region [0, scratch_off) lives at the workspace start, or in
    // a separate buffer (d_ctl, hgk_decode_launch_ctl)
    char* cr = d_ctl ? static_cast<char*>(d_ctl) : ws;
    DecodeCtl* ctl = reinterpret_cast<DecodeCtl*>(cr);
    a.ctl = ctl;
    a.gsum = reinterpret_cast<unsigned long long*>(cr + l.gsum_off);
    a.link = reinterpret_cast<unsigned long long*>(cr + l.link_off);
    a.status = reinterpret_cast<unsigned long long*>(cr + l.status_off);
    a.ticket = &ctl->ticket;
    a.scratch = reinterpret_cast<hg_span*>(ws + l.scratch_off);
    a.bp = bp;
    a.sbp = sbp < bp ? sbp : bp;
    a.nbatches = (uint32_t)((l.npieces + a.bp - 1) / a.bp);
    a.npieces = (uint32_t)l.npieces;
    a.hz = 8 - nb;
    a.diag = d_diag;
    a.sdiag = d_diag ? d_diag + (size_t)l.nbatches * DIAG_WORDS : nullptr;
    a.sbatch = reinterpret_cast<SpecBatch*>(ws + l.sbatch_off);
    a.spiece = reinterpret_cast<SpecPiece*>(ws + l.spiece_off);
    a.spiece_rw = reinterpret_cast<SpecPiece*>(ws + l.spiece_off);
    a.kpre_tag = kpre_tag;
    a.nspec = (uint32_t)((l.npieces + a.sbp - 1) / a.sbp);
    a.q = a.bp / a.sbp;
    a.hop_wide = HOP_WIDE_CAND;
    a.zero_next = nullptr;
    a.zero_next_n16 = 0;
    zero_bytes = (l.status_off + 2 * (uint64_t)a.nbatches * 8 + 7) & ~7ull;
    const uint64_t ll[8] = {l.sbatch_off, l.spiece_off, a.nspec, a.sbp, a.bp, a.nbatches,
                            l.status_off, 0};
    for (int i = 0; i < 8; ++i) g_last_launch[i] = ll[i];
    return a;
}
}  // namespace

// d_ws must hold hgk_decode_workspace_bytes(len) bytes.  The launcher zeroes
// the statuses and the ticket (the scratch area needs no initialisation).
// len == 0 is handled by the caller (no launch).
namespace {
__global__ void decode_const_result(hg_decode_result* r, uint64_t off) {
    hg_decode_result v;
    v.n_records = 0;
    v.kind = HG_OK;
    v.reserved = 0;
    v.err_offset = off;
    *r = v;
}

// ctl (nullable): the double-buffered control region of hgk_decode_launch_ctl.
struct CtlPair {
    void* cur;            // this call's control region
    uint64_t cur_clean;   // bytes of it known to be zero
    void* next;           // the next call's, cleared by the pre-pass
    uint64_t next_bytes;  // room in it
    uint64_t* zeroed;     // out: bytes of `next` cleared
};
int launch_decode(const uint8_t* d_sst, uint64_t len, hg_span* d_spans, uint64_t cap,
                  hg_decode_result* d_result, void* d_ws, uint32_t* d_diag, hipStream_t stream,
                  uint64_t begin, uint64_t stop, uint64_t entry, bool range, uint64_t rlen,
                  const CtlPair* ctl = nullptr) {
    using namespace hgk;
    if (stop > len) stop = len;
    if (entry >= stop) {  // no record starts in the range: 0 records, exit = entry
        hipLaunchKernelGGL(decode_const_result, dim3(1), dim3(1), 0, stream, d_result,
                           range ? entry : 0ull);
        return HG_LAUNCH_STATUS();
    }
    const uint64_t npieces = (stop - begin + PIECE - 1) / PIECE;
    const uint32_t res_gen = d_diag ? resident_workgroups(decode_kernel<true>, 1)
                                    : resident_workgroups(decode_kernel<false>, 2);
    const uint32_t bp = general_pieces(npieces, res_gen);
    const uint32_t sbp = spec_pieces(bp, npieces, device_cus());
    uint64_t zero_bytes = 0;
    DecodeArgs a = make_args(d_sst, len, d_spans, cap, d_result, d_ws, d_diag, bp, sbp,
                             zero_bytes, begin, stop, entry, range, rlen, 0u,
                             ctl ? ctl->cur : nullptr);
    a.hop_wide = hop_wide_cand(a.nspec, resident_workgroups(decode_spec_kernel, 3));
    if (!ctl || ctl->cur_clean < zero_bytes) {
        if (hipMemsetAsync(ctl ? ctl->cur : d_ws, 0, zero_bytes, stream) != hipSuccess)
            return HG_HIP_FAIL;
    }
    if (ctl) {
        // the next call of the same geometry finds its region clear (one of
        // this size or smaller; another pays the memset)
        const uint64_t z16 = std::min((zero_bytes + 15) / 16, ctl->next_bytes / 16);
        a.zero_next = static_cast<uint4*>(ctl->next);
        a.zero_next_n16 = (uint32_t)z16;
        *ctl->zeroed = z16 * 16;
    }
    // 1. pre-pass (stride runs, hop walks): verifies, links neighbours, sums records per group
    // 2. decode_kernel: spans of the resolved prefix, then the general engine
    //    from the first unresolved batch on (exits at once if there is none)
    hipLaunchKernelGGL(decode_spec_kernel, dim3(a.nspec), dim3(THREADS), 0, stream, a,
                       a.sbatch, const_cast<SpecPiece*>(a.spiece));
    if (HG_LW && !HG_LW_FUSE)
        hipLaunchKernelGGL(decode_lw_kernel, dim3(a.nspec), dim3(THREADS), 0, stream, a, a.sbatch,
                           const_cast<SpecPiece*>(a.spiece));
    const uint32_t grid = a.nbatches > a.nspec ? a.nbatches : a.nspec;
    if (d_diag)
        hipLaunchKernelGGL(decode_kernel<true>, dim3(grid), dim3(THREADS), 0, stream, a);
    else
        hipLaunchKernelGGL(decode_kernel<false>, dim3(grid), dim3(THREADS), 0, stream, a);
    return HG_LAUNCH_STATUS();
}
}  // namespace

extern "C" int hgk_decode_launch_diag(const uint8_t* d_sst, uint64_t len, hg_span* d_spans,
                                      uint64_t cap, hg_decode_result* d_result, void* d_ws,
                                      uint32_t* d_diag, hipStream_t stream) {
    return launch_decode(d_sst, len, d_spans, cap, d_result, d_ws, d_diag, stream, 0, len, 0,
                         false, len);
}

// Range decode of a table of `len` bytes whose bytes [begin, rlen) are
// present at d_sst + begin (rlen >= min(len, stop + 16)): the records starting
// in [entry, stop) (entry an exact record start, begin <= entry) are decoded
// with absolute offsets; the result's err_offset on success is the exit (the
// first record start at or after stop).  d_ws holds
// hgk_decode_workspace_bytes(stop - begin) bytes.
extern "C" int hgk_decode_range_launch(const uint8_t* d_sst, uint64_t len, uint64_t rlen,
                                       uint64_t begin, uint64_t stop, uint64_t entry,
                                       hg_span* d_spans, uint64_t cap,
                                       hg_decode_result* d_result, void* d_ws,
                                       hipStream_t stream) {
    return launch_decode(d_sst, len, d_spans, cap, d_result, d_ws, nullptr, stream, begin, stop,
                         entry, true, rlen);
}

// Guess of the first record start at or after `stop` (see decode_guess_kernel)
// into *d_out (device).  Bytes [stop - 16 KiB (or 0), min(len, stop + 16)) must
// be present at d_sst (absolute addressing, as hgk_decode_range_launch).
// d_ws: hgk_decode_workspace_bytes(16384) bytes.
extern "C" int hgk_decode_guess_launch(const uint8_t* d_sst, uint64_t len, uint64_t rlen,
                                       uint64_t stop, uint64_t* d_out, void* d_ws,
                                       hipStream_t stream) {
    using namespace hgk;
    if (stop > len) stop = len;
    const uint64_t begin = stop > PIECE ? stop - PIECE : 0;
    uint64_t zb = 0;
    const DecodeArgs a = make_args(d_sst, len, nullptr, 0, nullptr, d_ws, nullptr, BATCH_MIN,
                                   SPEC_BP_MIN, zb, begin, stop, begin, true, rlen);
    hipLaunchKernelGGL(decode_guess_kernel, dim3(1), dim3(THREADS), 0, stream, a, d_out);
    return HG_LAUNCH_STATUS();
}

extern "C" int hgk_decode_launch(const uint8_t* d_sst, uint64_t len, hg_span* d_spans,
                                 uint64_t cap, hg_decode_result* d_result, void* d_ws,
                                 hipStream_t stream) {
    return hgk_decode_launch_diag(d_sst, len, d_spans, cap, d_result, d_ws, nullptr, stream);
}

// Bytes of a table's control region (statuses, links, group sums, ticket):
// the part of the workspace zeroed before every call.
extern "C" uint64_t hgk_decode_ctl_bytes(uint64_t len) { return decode_layout(len).scratch_off; }

// hgk_decode_launch with the control region in d_ctl (hgk_decode_ctl_bytes(len)
// bytes) instead of the workspace start, `clean` bytes of it known to be zero
// (no memset launch when that covers this call's), and d_next (next_bytes) the
// next call's region: the pre-pass clears it; *zeroed = the bytes cleared.
extern "C" int hgk_decode_launch_ctl(const uint8_t* d_sst, uint64_t len, hg_span* d_spans,
                                     uint64_t cap, hg_decode_result* d_result, void* d_ws,
                                     void* d_ctl, uint64_t clean, void* d_next,
                                     uint64_t next_bytes, uint64_t* zeroed, hipStream_t stream) {
    *zeroed = 0;
    const CtlPair cp{d_ctl, clean, d_next, next_bytes, zeroed};
    return launch_decode(d_sst, len, d_spans, cap, d_result, d_ws, nullptr, stream, 0, len, 0,
                         false, len, &cp);
}

// Many tables, three launches in all (zero, pre-pass, decode).  Batch
// geometry comes from the total size (the tables share the chip), so a
// batch of small tables gets the long pre-pass batches one big table would.
// Table i's workspace is d_ws + ws_off[i] (hgk_decode_workspace_bytes(lens[i])
// bytes).  h_stage: pinned host memory of at least hgk_decode_multi_stage_bytes(ntab)
// bytes, d_stage: device memory of the same size; the caller keeps h_stage
// untouched until the stream has passed this call (the arguments are copied
// from it asynchronously).
namespace {
// The staging of a batched decode (host copy and device copy alike): the
// tables' DecodeArgs, their control-region sizes, the prefix sums of their
// pre-pass grids and of their decode grids.
struct MultiStage {
    uint64_t zb, pre_s, pre_d, bytes;  // byte offsets (DecodeArgs at 0) and size
};
MultiStage multi_stage(uint32_t ntab) {
    auto al = [](uint64_t b) { return (b + 255) / 256 * 256; };
    MultiStage m;
    m.zb = al((uint64_t)ntab * sizeof(hgk::DecodeArgs));
    m.pre_s = m.zb + al((uint64_t)ntab * 8);
    m.pre_d = m.pre_s + al(((uint64_t)ntab + 1) * 4);
    m.bytes = m.pre_d + al(((uint64_t)ntab + 1) * 4);
    return m;
}
}  // namespace

extern "C" uint64_t hgk_decode_multi_stage_bytes(uint32_t ntab) { return multi_stage(ntab).bytes; }

// mc (nullable): control regions and staging reuse across calls (hgk_multi_ctl).
extern "C" int hgk_decode_launch_multi(uint32_t ntab, const uint8_t* const* d_tables,
                                       const uint64_t* lens, hg_span* const* d_spans,
                                       const uint64_t* caps, hg_decode_result* d_results,
                                       void* d_ws, const uint64_t* ws_off, void* h_stage,
                                       void* d_stage, hipStream_t stream, uint32_t kpre_tag,
                                       const hgk_multi_ctl* mc) {
    using namespace hgk;
    if (ntab == 0) return HG_OK;
    uint64_t total_pieces = 0;
    for (uint32_t i = 0; i < ntab; ++i) total_pieces += (lens[i] + PIECE - 1) / PIECE;
    const uint32_t res_gen = resident_workgroups(decode_kernel<false>, 2);
    const uint32_t bp = general_pieces(total_pieces, res_gen);
    const uint32_t sbp = spec_pieces(bp, total_pieces, device_cus());
    char* hs = static_cast<char*>(h_stage);
    const MultiStage ms = multi_stage(ntab);
    DecodeArgs* args = reinterpret_cast<DecodeArgs*>(hs);
    uint64_t* zb = reinterpret_cast<uint64_t*>(hs + ms.zb);
    uint32_t* pre_s = reinterpret_cast<uint32_t*>(hs + ms.pre_s);
    uint32_t* pre_d = reinterpret_cast<uint32_t*>(hs + ms.pre_d);
    pre_s[0] = pre_d[0] = 0;
    uint64_t nspec_all = 0;
    bool clean = mc && mc->cur_zero, empty = false;
    for (uint32_t i = 0; i < ntab; ++i) {
        args[i] = make_args(d_tables[i], lens[i], d_spans[i], caps[i], d_results + i,
                            static_cast<char*>(d_ws) + ws_off[i], nullptr, bp, sbp, zb[i], 0,
                            ~0ull, 0, false, ~0ull, kpre_tag, mc ? mc->cur + mc->off[i] : nullptr);
        empty |= lens[i] == 0;
        if (clean && lens[i] && mc->cur_zero[i] < zb[i]) clean = false;
        if (mc) {  // the pre-pass of a non-empty table clears its region of `next`
            const uint64_t z16 = lens[i] && !kpre_tag ? (zb[i] + 15) / 16 : 0;
            args[i].zero_next = reinterpret_cast<uint4*>(mc->next + mc->off[i]);
            args[i].zero_next_n16 = (uint32_t)z16;
            mc->next_zero[i] = z16 * 16;
        }
        const uint32_t gs = lens[i] ? args[i].nspec : 0;
        nspec_all += gs;
        const uint32_t gd = lens[i] ? (args[i].nbatches > args[i].nspec ? args[i].nbatches
                                                                          : args[i].nspec)
                                    : 0;
        pre_s[i + 1] = pre_s[i] + gs;
        pre_d[i + 1] = pre_d[i] + gd;
    }
    {
        const uint32_t hw = hop_wide_cand(nspec_all, kpre_tag ? resident_workgroups(decode_spec_multi<true>, 4)
                                                             : resident_workgroups(decode_spec_multi<false>, 5));
        for (uint32_t i = 0; i < ntab; ++i) args[i].hop_wide = hw;
    }
    const uint64_t bytes = hgk_decode_multi_stage_bytes(ntab);
    // the device staging already holds these argument bytes (same tables,
    // buffers and geometry as the call that staged them): no copy
    const bool same = mc && mc->shadow && mc->shadow_bytes == bytes &&
                      memcmp(mc->shadow, h_stage, bytes) == 0;
    if (mc) *mc->copied = same ? 0 : 1;
    if (!same && hipMemcpyAsync(d_stage, h_stage, bytes, hipMemcpyHostToDevice, stream) != hipSuccess)
        return HG_HIP_FAIL;
    if (!same && mc && mc->stage_ev && hipEventRecord(mc->stage_ev, stream) != hipSuccess)
        return HG_HIP_FAIL;
    char* ds = static_cast<char*>(d_stage);
    const DecodeArgs* dargs = reinterpret_cast<const DecodeArgs*>(ds);
    const uint64_t* dzb = reinterpret_cast<const uint64_t*>(ds + ms.zb);
    const uint32_t* dpre_s = reinterpret_cast<const uint32_t*>(ds + ms.pre_s);
    const uint32_t* dpre_d = reinterpret_cast<const uint32_t*>(ds + ms.pre_d);
    // control regions: zeroed here unless the previous call's pre-pass
    // cleared them (empty tables' results are written here too)
    if (!clean || empty)
        hipLaunchKernelGGL(decode_zero_multi, dim3(ntab), dim3(THREADS), 0, stream, dargs, dzb, ntab);
    if (pre_s[ntab]) {
        if (kpre_tag)
            hipLaunchKernelGGL(decode_spec_multi<true>, dim3(pre_s[ntab]), dim3(THREADS), 0, stream,
                               dargs, dpre_s, ntab);
        else
            hipLaunchKernelGGL(decode_spec_multi<false>, dim3(pre_s[ntab]), dim3(THREADS), 0, stream,
                               dargs, dpre_s, ntab);
        if (HG_LW && !HG_LW_FUSE)
            hipLaunchKernelGGL(decode_lw_multi, dim3(pre_s[ntab]), dim3(THREADS), 0, stream, dargs,
                               dpre_s, ntab);
    }
    if (pre_d[ntab])
        hipLaunchKernelGGL(decode_multi, dim3(pre_d[ntab]), dim3(THREADS), 0, stream, dargs, dpre_d,
                           ntab);
    return HG_LAUNCH_STATUS();
}

// Compaction mode, after hgk_decode_launch_multi(kpre_tag) of ntab tables:
// the merge entries of every table (decode_entries_multi) into d_ent at
// d_run_off[t] + record, order violations into *d_err (atomicMin of the entry
// index).  d_stage: that call's device staging; nspec_total: its pre-pass grid
// (hgk_decode_multi_geometry).
extern "C" int hgk_decode_entries_launch(const void* d_stage, uint32_t ntab, uint32_t nspec_total,
                                         const uint64_t* d_run_off, void* d_ent,
                                         unsigned long long* d_err, hipStream_t stream) {
    using namespace hgk;
    if (!nspec_total) return HG_OK;
    const char* ds = static_cast<const char*>(d_stage);
    hipLaunchKernelGGL(decode_entries_multi, dim3(nspec_total), dim3(THREADS), 0, stream,
                       reinterpret_cast<const DecodeArgs*>(ds), ntab,
                       reinterpret_cast<const uint32_t*>(ds + multi_stage(ntab).pre_s), d_run_off,
                       static_cast<KEnt*>(d_ent), d_err);
    return HG_LAUNCH_STATUS();
}

// The pre-pass grid of the last hgk_decode_launch_multi whose host staging is
// h_stage (read back from it: the caller keeps it until the entries launch).
extern "C" uint32_t hgk_decode_multi_geometry(const void* h_stage, uint32_t ntab) {
    using namespace hgk;
    return reinterpret_cast<const uint32_t*>(static_cast<const char*>(h_stage) +
                                             multi_stage(ntab).pre_s)[ntab];
}
