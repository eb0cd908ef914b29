// hg_multi.hip — host driver over several contexts (devices): one host thread
// per context, no collectives.  Three ways to split the work:
//   - many tables (cold open of a table directory, SSTableManager::new,
//     src/sstable/manager.rs:47-55; BASELINE config 4): tables round-robin
//     over the contexts, each context decodes its share in one batched launch
//     chain;
//   - one huge table: cut into byte ranges; context c guesses the first record
//     start of its range (decode_guess_kernel), decodes its range from that
//     guess, and the host hands the exact entry over in order (the exit of
//     range c-1); a range whose guess differs is decoded again from the exact
//     entry.  One u64 per split crosses between devices, nothing else;
//   - compaction (SSTableManager::compact, manager.rs:137-159; config 5): G-1
//     splitter keys chosen from sampled record keys of every table (the
//     reference's block first keys, index.rs:55-67, are every block_stride-th
//     key); each context decodes, merges (newest wins) and encodes the slice
//     of EVERY table inside its key range; the compacted table is the
//     concatenation of the slices in key order, byte-identical to the
//     single-device compaction.  The reference loop on tables that are not
//     strictly increasing is not range-separable, so such input (found by the
//     slices' merges or at a split boundary) falls back to one context.
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

#include "hg_internal.hpp"
#include "hg_knobs.hpp"
#include "hg_knobs.hpp"

using namespace hgi;

namespace {

constexpr uint64_t kPiece = 16384;  // hg_decode.hip PIECE

// Persistent host workers for fan_out: a split compaction runs four steps
// over every context, and spawning and joining a thread per context per step
// cost more than a context's share of the work on eight GPUs.  One fan_out
// uses the pool at a time (busy); a second, concurrent one (another host
// thread's call) spawns its own threads as before.
class FanPool {
  public:
    ~FanPool() {
        {
            std::lock_guard<std::mutex> lk(m_);
            stop_ = true;
        }
        cv_.notify_all();
        for (std::thread& t : workers_) t.join();
    }
    std::mutex busy;
    // fn(i) for i in [0, n) on the workers (the caller only waits: its
    // current HIP device stays its own); returns when all ran
    void run(uint32_t n, const std::function<void(uint32_t)>& fn) {
        {
            std::lock_guard<std::mutex> lk(m_);
            // (a new worker starts from the generation before this job's)
            while (workers_.size() < n && workers_.size() < 64)
                workers_.emplace_back([this, g = gen_] { work(g); });
            job_ = &fn;
            njobs_ = n;
            next_ = 0;
            pending_ = n;
            ++gen_;
        }
        cv_.notify_all();
        std::unique_lock<std::mutex> lk(m_);
        done_.wait(lk, [this] { return pending_ == 0; });
        job_ = nullptr;
    }

  private:
    void take(std::unique_lock<std::mutex>& lk) {  // run indices until none is left
        while (next_ < njobs_) {
            const uint32_t i = next_++;
            const std::function<void(uint32_t)>* f = job_;
            lk.unlock();
            (*f)(i);
            lk.lock();
            if (--pending_ == 0) done_.notify_all();
        }
    }
    void work(uint64_t seen) {
        std::unique_lock<std::mutex> lk(m_);
        while (true) {
            cv_.wait(lk, [&] { return stop_ || gen_ != seen; });
            if (stop_) return;
            seen = gen_;
            take(lk);
        }
    }
    std::mutex m_;
    std::condition_variable cv_, done_;
    std::vector<std::thread> workers_;
    const std::function<void(uint32_t)>* job_ = nullptr;
    uint32_t njobs_ = 0, next_ = 0, pending_ = 0;
    uint64_t gen_ = 0;
    bool stop_ = false;
};
FanPool g_pool;

// Run fn(i) for i in [0, n) on host threads (a worker per index while the
// pool has room; more than 64 share them); the first failing code.
template <typename F>
int fan_out(uint32_t n, F fn) {
    std::vector<int> rc(n, HG_OK);
    if (n == 1) {
        rc[0] = fn(0u);
    } else if (g_pool.busy.try_lock()) {
        const std::function<void(uint32_t)> job = [&rc, &fn](uint32_t i) { rc[i] = fn(i); };
        g_pool.run(n, job);
        g_pool.busy.unlock();
    } else {
        std::vector<std::thread> th;
        th.reserve(n);
        for (uint32_t i = 0; i < n; ++i) th.emplace_back([&rc, &fn, i] { rc[i] = fn(i); });
        for (auto& t : th) t.join();
    }
    for (int r : rc)
        if (r != HG_OK) return r;
    return HG_OK;
}

// Phase times of the last hg_multi_compact_dev (diagnostics for the bench's
// cross-GPU leg, hgk_multi_last_phases): per context, ms of [0] its decode of
// the tables it owns (host wall clock, the decode synchronises), [1] the
// sample / splitter / cut steps (wall clock, all contexts together), and of
// its key range [2] the slice copies, [3] the merge, [4] the encode (HIP
// events on the context's stream).
constexpr uint32_t kPhases = 5, kPhaseCtx = 64;
struct Phases {
    std::mutex mu;
    uint32_t nctx = 0;
    double ms[kPhaseCtx][kPhases] = {};
} g_phases;
double wall_ms() {
    return std::chrono::duration<double, std::milli>(
               std::chrono::steady_clock::now().time_since_epoch()).count();
}

int sync_d2h(hg_ctx* c, void* dst, const void* src, size_t n) {
    if (!n) return HG_OK;
    if (hipMemcpyAsync(dst, src, n, hipMemcpyDeviceToHost, c->stream) != hipSuccess ||
        hipStreamSynchronize(c->stream) != hipSuccess)
        return HG_HIP_FAIL;
    return HG_OK;
}

// Tables of one context uploaded into one arena (256-byte aligned starts) and
// decoded by one batched launch chain; spans (capacity len / 16 each) stay in
// c->mspans, results are copied to the host.
struct Share {
    std::vector<uint32_t> ids;
    std::vector<uint64_t> aoff, soff;
    std::vector<hg_decode_result> res;
};

// Tables already on c's device (d_tables[ids[j]]): one batched decode, spans
// into c->mspans at soff[j], results to the host.
int decode_share_dev(hg_ctx* c, Share& sh, const uint8_t* const* d_tables, const uint64_t* lens) {
    const uint32_t k = (uint32_t)sh.ids.size();
    sh.soff.resize(k);
    sh.res.assign(k, hg_decode_result{0, HG_OK, 0, 0});
    if (!k) return HG_OK;
    if (set_dev(c) != HG_OK) return HG_HIP_FAIL;
    uint64_t sb = 0;
    for (uint32_t j = 0; j < k; ++j) {
        sh.soff[j] = sb;
        sb += lens[sh.ids[j]] / 16;
    }
    int r = ensure(c, c->mspans, (sb ? sb : 1) * sizeof(hg_span));
    if (r == HG_OK) r = ensure(c, c->x_res, k * sizeof(hg_decode_result) + 64);
    if (r != HG_OK) return r;
    hg_span* spans = static_cast<hg_span*>(c->mspans.p);
    std::vector<const uint8_t*> dt(k);
    std::vector<hg_span*> ds(k);
    std::vector<uint64_t> ln(k), caps(k);
    for (uint32_t j = 0; j < k; ++j) {
        const uint32_t t = sh.ids[j];
        dt[j] = d_tables[t];
        ds[j] = spans + sh.soff[j];
        ln[j] = lens[t];
        caps[j] = lens[t] / 16;
    }
    hg_decode_result* dr = static_cast<hg_decode_result*>(c->x_res.p);
    r = hg_decode_batch_dev_async(c, k, dt.data(), ln.data(), ds.data(), caps.data(), dr);
    if (r != HG_OK) return r;
    return sync_d2h(c, sh.res.data(), dr, k * sizeof(hg_decode_result));
}

int decode_share(hg_ctx* c, Share& sh, const uint8_t* const* h_tables, const uint64_t* lens) {
    const uint32_t k = (uint32_t)sh.ids.size();
    sh.aoff.resize(k);
    sh.soff.resize(k);
    sh.res.assign(k, hg_decode_result{0, HG_OK, 0, 0});
    if (!k) return HG_OK;
    if (set_dev(c) != HG_OK) return HG_HIP_FAIL;
    uint64_t ab = 0, sb = 0;
    for (uint32_t j = 0; j < k; ++j) {
        const uint64_t L = lens[sh.ids[j]];
        if (L >= kMaxLen) return HG_ERR_TOO_LARGE;
        sh.aoff[j] = ab;
        sh.soff[j] = sb;
        ab += (L + 255) & ~255ull;
        sb += L / 16;
    }
    int r = ensure(c, c->d_in, ab ? ab : 1);
    if (r == HG_OK) r = ensure(c, c->mspans, (sb ? sb : 1) * sizeof(hg_span));
    if (r == HG_OK) r = ensure(c, c->x_res, k * sizeof(hg_decode_result) + 64);
    if (r != HG_OK) return r;
    char* arena = static_cast<char*>(c->d_in.p);
    hg_span* spans = static_cast<hg_span*>(c->mspans.p);
    std::vector<const uint8_t*> dt(k);
    std::vector<hg_span*> ds(k);
    std::vector<uint64_t> ln(k), caps(k);
    for (uint32_t j = 0; j < k; ++j) {
        const uint32_t t = sh.ids[j];
        if (lens[t] && (r = h2d_pipelined(c, arena + sh.aoff[j], h_tables[t], lens[t])) != HG_OK)
            return r;
        dt[j] = reinterpret_cast<const uint8_t*>(arena + sh.aoff[j]);
        ds[j] = spans + sh.soff[j];
        ln[j] = lens[t];
        caps[j] = lens[t] / 16;
    }
    hg_decode_result* dr = static_cast<hg_decode_result*>(c->x_res.p);
    r = hg_decode_batch_dev_async(c, k, dt.data(), ln.data(), ds.data(), caps.data(), dr);
    if (r != HG_OK) return r;
    return sync_d2h(c, sh.res.data(), dr, k * sizeof(hg_decode_result));
}

// Device bytes one decode_share of these tables takes: the arena (256-byte
// aligned starts) and the spans (capacity len / 16 each).
uint64_t share_bytes(uint64_t len) { return ((len + 255) & ~255ull) + (len / 16) * sizeof(hg_span); }

// Byte budget of one batched decode of many tables (SSTableManager's cold open
// of a whole directory): HG_DECODE_GROUP_BYTES, else 40 % of the device memory
// free now.  A share larger than this is decoded in groups of tables, one
// group after another; a table larger than the budget is a group of its own.
uint64_t group_budget() {
    if (const int64_t v = hgk_knob("HG_DECODE_GROUP_BYTES", 0); v > 0) return (uint64_t)v;
    size_t fr = 0, tot = 0;
    if (hipMemGetInfo(&fr, &tot) != hipSuccess || fr == 0) return 4ull << 30;
    return (uint64_t)(fr / 10 * 4);
}

std::vector<std::vector<uint32_t>> groups_of(const std::vector<uint32_t>& ids, const uint64_t* lens,
                                              uint64_t budget) {
    std::vector<std::vector<uint32_t>> g;
    uint64_t acc = 0;
    for (uint32_t t : ids) {
        const uint64_t b = share_bytes(lens[t]);
        if (g.empty() || (acc + b > budget && !g.back().empty())) {
            g.emplace_back();
            acc = 0;
        }
        g.back().push_back(t);
        acc += b;
    }
    return g;
}

std::vector<Share> round_robin(uint32_t nctx, uint32_t ntables) {
    std::vector<Share> sh(nctx);
    for (uint32_t t = 0; t < ntables; ++t) sh[t % nctx].ids.push_back(t);
    return sh;
}

// ---- device helpers for the key-range split -----------------------------------
struct KeyRef {      // a sampled key: 16-byte big-endian prefix, length, where it is
    uint64_t p0, p1;
    uint32_t klen, table;
    uint64_t rec;
};

__device__ __forceinline__ void key_prefix(const uint8_t* k, uint32_t kl, uint64_t& p0,
                                           uint64_t& p1) {
    p0 = p1 = 0;
    for (uint32_t i = 0; i < 16; ++i) {
        const uint64_t b = i < kl ? k[i] : 0;
        if (i < 8) p0 = (p0 << 8) | b;
        else p1 = (p1 << 8) | b;
    }
}

// Up to kSampleTabs tables' samples in one launch (by value: no upload);
// block y = table, m <= blockDim.x samples each.
constexpr uint32_t kSampleTabs = 32;
struct SampleArgs {
    struct Tab {
        const uint8_t* table;
        const hg_span* spans;
        uint64_t n, step, at;
        uint32_t m, id;
    } t[kSampleTabs];
};

__global__ void sample_keys_kernel(SampleArgs sa, KeyRef* out) {
    const SampleArgs::Tab& tb = sa.t[blockIdx.x];
    const uint32_t j = threadIdx.x;
    if (j >= tb.m) return;
    const uint64_t rec = j * tb.step < tb.n ? j * tb.step : tb.n - 1;
    const hg_span sp = tb.spans[rec];
    KeyRef r;
    key_prefix(tb.table + sp.off + 16, sp.klen, r.p0, r.p1);
    r.klen = sp.klen;
    r.table = tb.id;
    r.rec = rec;
    out[tb.at + j] = r;
}

// Vec<u8> Ord (shorter first on a common prefix).
__device__ int dkey_cmp(const uint8_t* a, uint32_t al, const uint8_t* b, uint32_t bl) {
    const uint32_t m = al < bl ? al : bl;
    for (uint32_t i = 0; i < m; ++i)
        if (a[i] != b[i]) return a[i] < b[i] ? -1 : 1;
    return al < bl ? -1 : (al > bl ? 1 : 0);
}

// A key's first 16 bytes as two big-endian words (zero past klen): two
// unaligned 8-byte reads for keys of 16 bytes or more (no byte loop of
// dependent reads), the key's own bytes otherwise.
__device__ __forceinline__ void key_prefix16(const uint8_t* k, uint32_t kl, uint64_t& p0,
                                             uint64_t& p1) {
    uint64_t lo = 0, hi = 0;
    if (kl >= 16) {
        lo = *reinterpret_cast<const uint64_t*>(k);
        hi = *reinterpret_cast<const uint64_t*>(k + 8);
    } else {
        for (uint32_t i = 0; i < kl; ++i) {
            const uint64_t b = k[i];
            if (i < 8) lo |= b << (8 * i);
            else hi |= b << (8 * (i - 8));
        }
    }
    p0 = __builtin_bswap64(lo);
    p1 = __builtin_bswap64(hi);
}

// Vec<u8> Ord of a table key against splitter s (prefix words sp0 / sp1):
// the prefixes decide unless they are equal; then both keys' bytes from 16 on.
__device__ __forceinline__ int split_cmp(const uint8_t* k, uint32_t kl, uint64_t p0, uint64_t p1,
                                         const uint8_t* sk, uint32_t sl, uint64_t sp0,
                                         uint64_t sp1) {
    if (p0 != sp0) return p0 < sp0 ? -1 : 1;
    if (p1 != sp1) return p1 < sp1 ? -1 : 1;
    if (kl <= 16 || sl <= 16) return kl < sl ? -1 : (kl > sl ? 1 : 0);
    return dkey_cmp(k + 16, kl - 16, sk + 16, sl - 16);
}

struct SplitTab {  // one table of a context's cut search
    const uint8_t* table;
    const hg_span* spans;
    uint64_t len, n;
};

// For splitter s of table t (one wave per pair, grid = tables x splitters):
// the first record with key >= s (lower bound), its byte offset (the table
// length past the end), and whether the two records around the cut are
// strictly increasing (a cut inside a run of equal or unordered keys cannot
// be merged slice by slice).  A 64-ary search: each step the 64 lanes probe
// 64 evenly spaced records at once (about four dependent steps for a million
// records, against ~20 for a binary search, each step one span read and one
// key read).  On sorted input this is the exact lower bound; on unsorted input
// it is some index, and the ok flag or the slice merges find the disorder.
__global__ __launch_bounds__(256) void split_points_kernel(const SplitTab* tabs, uint32_t ntab,
                                                           const uint8_t* keys,
                                                           const uint64_t* koff,
                                                           const uint32_t* klen,
                                                           const uint64_t* kpre, uint32_t nsplit,
                                                           uint64_t* out) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t w = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (w >= ntab * nsplit) return;
    const uint32_t t = w / nsplit, s = w % nsplit;
    const SplitTab tb = tabs[t];
    const uint8_t* key = keys + koff[s];
    const uint32_t kl = klen[s];
    const uint64_t sp0 = kpre[2 * s], sp1 = kpre[2 * s + 1];
    auto less = [&](uint64_t r) -> bool {  // key of record r < splitter
        const hg_span sp = tb.spans[r];
        uint64_t p0, p1;
        key_prefix16(tb.table + sp.off + 16, sp.klen, p0, p1);
        return split_cmp(tb.table + sp.off + 16, sp.klen, p0, p1, key, kl, sp0, sp1) < 0;
    };
    uint64_t lo = 0, hi = tb.n;  // the answer lies in [lo, hi]
    while (hi - lo > 64) {
        const uint64_t span = hi - lo;
        const uint64_t pr = lo + span * (lane + 1) / 65;  // strictly increasing, in [lo, hi)
        const uint64_t m = __ballot(less(pr));
        const uint32_t c = (uint32_t)__popcll(m);
        const uint64_t nlo = c ? lo + span * c / 65 + 1 : lo;
        const uint64_t nhi = c < 64 ? lo + span * (c + 1) / 65 : hi;
        lo = nlo;
        hi = nhi;
    }
    const uint64_t pr = lo + lane;
    lo += (uint64_t)__popcll(__ballot(pr < hi && less(pr)));
    if (lane != 0) return;
    uint64_t ok = 1;
    if (lo > 0 && lo < tb.n) {
        const hg_span a = tb.spans[lo - 1], b = tb.spans[lo];
        uint64_t a0, a1, b0, b1;
        key_prefix16(tb.table + a.off + 16, a.klen, a0, a1);
        key_prefix16(tb.table + b.off + 16, b.klen, b0, b1);
        ok = split_cmp(tb.table + a.off + 16, a.klen, a0, a1, tb.table + b.off + 16, b.klen, b0, b1) < 0;
    }
    uint64_t* o = out + 3 * ((size_t)t * nsplit + s);
    o[0] = lo;
    o[1] = lo < tb.n ? tb.spans[lo].off : tb.len;
    o[2] = ok;
}

int host_key_cmp(const std::vector<uint8_t>& a, const std::vector<uint8_t>& b) {
    const size_t m = std::min(a.size(), b.size());
    const int c = m ? memcmp(a.data(), b.data(), m) : 0;
    if (c) return c < 0 ? -1 : 1;
    return a.size() < b.size() ? -1 : (a.size() > b.size() ? 1 : 0);
}

}  // namespace

extern "C" {

// ---- many tables ------------------------------------------------------------------
int hg_multi_decode_host(hg_ctx* const* ctxs, uint32_t nctx, uint32_t ntables,
                         const uint8_t* const* h_tables, const uint64_t* lens,
                         hg_span* const* h_spans, const uint64_t* caps, uint64_t* n_out,
                         hg_err* errs) {
    DeviceGuard keep;  // every device switch below is undone on return
    if (!ctxs || !nctx || (ntables && (!h_tables || !lens || !h_spans || !caps || !n_out)))
        return HG_ERR_INVALID_ARG;
    for (uint32_t i = 0; i < nctx; ++i)
        if (!ctxs[i]) return HG_ERR_INVALID_ARG;
    for (uint32_t t = 0; t < ntables; ++t)
        if ((lens[t] && !h_tables[t]) || (caps[t] && !h_spans[t])) return HG_ERR_INVALID_ARG;
    std::vector<Share> sh = round_robin(nctx, ntables);
    return fan_out(nctx, [&](uint32_t ci) {
        hg_ctx* c = ctxs[ci];
        if (set_dev(c) != HG_OK) return (int)HG_HIP_FAIL;
        // groups under the byte budget (a directory larger than HBM opens too)
        for (const std::vector<uint32_t>& grp : groups_of(sh[ci].ids, lens, group_budget())) {
            Share s;
            s.ids = grp;
            int r = decode_share(c, s, h_tables, lens);
            if (r != HG_OK) return r;
            const hg_span* spans = static_cast<const hg_span*>(c->mspans.p);
            for (size_t j = 0; j < s.ids.size(); ++j) {
                const uint32_t t = s.ids[j];
                const hg_decode_result& res = s.res[j];
                n_out[t] = res.n_records;
                if (errs) {
                    errs[t].kind = res.kind;
                    errs[t].reserved = 0;
                    errs[t].offset = res.kind != HG_OK ? res.err_offset : 0;
                }
                const uint64_t nc = std::min(std::min(res.n_records, caps[t]), lens[t] / 16);
                if (nc && (r = d2h_pipelined(c, h_spans[t], spans + s.soff[j],
                                             nc * sizeof(hg_span))) != HG_OK)
                    return r;
            }
        }
        return (int)HG_OK;
    });
}

// ---- one table split into byte ranges ------------------------------------------------
int hg_multi_decode_file_host(hg_ctx* const* ctxs, uint32_t nctx, const uint8_t* h_sst,
                              uint64_t len, hg_span* h_spans, uint64_t cap, uint64_t* n_out,
                              hg_err* err) {
    DeviceGuard keep;  // every device switch below is undone on return
    if (!ctxs || !nctx || (len && !h_sst) || (cap && !h_spans)) return HG_ERR_INVALID_ARG;
    if (len >= kMaxLen) return HG_ERR_TOO_LARGE;
    for (uint32_t i = 0; i < nctx; ++i)
        if (!ctxs[i]) return HG_ERR_INVALID_ARG;
    // range c = [B[c], B[c+1]), cuts 16 KiB-aligned, no empty range
    std::vector<uint64_t> B;
    B.push_back(0);
    for (uint32_t c = 1; c < nctx; ++c) {
        const uint64_t b = (len / nctx * c) & ~(kPiece - 1);
        if (b > B.back() && b < len) B.push_back(b);
    }
    B.push_back(len);
    const uint32_t nr = (uint32_t)B.size() - 1;
    struct Part {
        uint64_t lo = 0, hi = 0;   // bytes on the device: [lo, hi)
        uint64_t guess = 0, n = 0, exit = 0, err_off = 0;
        int32_t kind = HG_OK;
    };
    std::vector<Part> P(nr);
    auto decode_range = [&](uint32_t c, uint64_t entry) {
        hg_ctx* x = ctxs[c];
        Part& p = P[c];
        const uint64_t cap_c = (B[c + 1] - B[c]) / 16 + 2;
        int r = ensure(x, x->mspans, cap_c * sizeof(hg_span));
        if (r == HG_OK) r = ensure(x, x->ws, hgk_decode_workspace_bytes(B[c + 1] - B[c]));
        if (r == HG_OK) r = ensure(x, x->x_res, 64);
        if (r != HG_OK) return r;
        const uint8_t* base = static_cast<const uint8_t*>(x->d_in.p) - p.lo;  // absolute view
        hg_decode_result* dr = static_cast<hg_decode_result*>(x->x_res.p);
        r = hgk_decode_range_launch(base, len, p.hi, B[c], B[c + 1], entry,
                                    static_cast<hg_span*>(x->mspans.p), cap_c, dr, x->ws.p,
                                    x->stream);
        hg_decode_result res{};
        if (r == HG_OK) r = sync_d2h(x, &res, dr, sizeof res);
        if (r != HG_OK) return r;
        p.n = res.n_records;
        p.kind = res.kind;
        p.exit = res.kind == HG_OK ? res.err_offset : 0;
        p.err_off = res.kind == HG_OK ? 0 : res.err_offset;
        return (int)HG_OK;
    };
    // 1. every range at once: upload, guess the entry, decode from the guess
    int r = fan_out(nr, [&](uint32_t c) {
        hg_ctx* x = ctxs[c];
        Part& p = P[c];
        if (set_dev(x) != HG_OK) return (int)HG_HIP_FAIL;
        p.lo = c ? B[c] - std::min(B[c], kPiece) : 0;
        p.hi = std::min(len, B[c + 1] + 16);
        int rr = ensure(x, x->d_in, p.hi - p.lo ? p.hi - p.lo : 1);
        if (rr == HG_OK && p.hi > p.lo)
            rr = h2d_pipelined(x, x->d_in.p, h_sst + p.lo, p.hi - p.lo);
        if (rr != HG_OK) return rr;
        p.guess = 0;
        if (c) {
            if ((rr = ensure(x, x->ws, hgk_decode_workspace_bytes(kPiece))) != HG_OK ||
                (rr = ensure(x, x->x_aux, 64)) != HG_OK)
                return rr;
            const uint8_t* base = static_cast<const uint8_t*>(x->d_in.p) - p.lo;
            uint64_t* d_g = static_cast<uint64_t*>(x->x_aux.p);
            rr = hgk_decode_guess_launch(base, len, p.hi, B[c], d_g, x->ws.p, x->stream);
            if (rr == HG_OK) rr = sync_d2h(x, &p.guess, d_g, 8);
            if (rr != HG_OK) return rr;
        }
        if (p.guess == ~0ull) return (int)HG_OK;  // no guess: decoded after the handoff
        return decode_range(c, std::max(p.guess, B[c]));
    });
    if (r != HG_OK) return r;
    // 2. entry handoff in order; a range entered off its guess is decoded again
    uint32_t last = nr - 1;
    for (uint32_t c = 1; c < nr; ++c) {
        if (P[c - 1].kind != HG_OK) {  // the first error ends the table (the reference stops there)
            last = c - 1;
            break;
        }
        if (P[c].guess != P[c - 1].exit) {
            if (set_dev(ctxs[c]) != HG_OK) return HG_HIP_FAIL;
            P[c].guess = P[c - 1].exit;
            if ((r = decode_range(c, P[c].guess)) != HG_OK) return r;
        }
    }
    uint64_t total = 0;
    std::vector<uint64_t> G(nr + 1, 0);
    for (uint32_t c = 0; c <= last; ++c) {
        G[c] = total;
        total += P[c].n;
    }
    if (n_out) *n_out = total;
    if (err) {
        err->kind = P[last].kind;
        err->reserved = 0;
        err->offset = P[last].err_off;
    }
    // 3. spans into place
    r = fan_out(last + 1, [&](uint32_t c) {
        hg_ctx* x = ctxs[c];
        if (set_dev(x) != HG_OK) return (int)HG_HIP_FAIL;
        if (G[c] >= cap) return (int)HG_OK;
        const uint64_t nc = std::min(P[c].n, cap - G[c]);
        return nc ? d2h_pipelined(x, h_spans + G[c], x->mspans.p, nc * sizeof(hg_span))
                  : (int)HG_OK;
    });
    if (r != HG_OK) return r;
    if (P[last].kind != HG_OK) return P[last].kind;
    return total > cap ? HG_ERR_CAPACITY : HG_OK;
}

// ---- compaction split by key range -----------------------------------------------------
// Diagnostics only (not in include/horreum_gpu.h; bench.py's cross-GPU leg):
// the phase times of the last hg_multi_compact_dev that split by key range
// (see Phases), kPhases doubles per context into out[0 .. 5 * max_ctx);
// returns the contexts recorded.
uint32_t hgk_multi_last_phases(double* out, uint32_t max_ctx) {
    std::lock_guard<std::mutex> g(g_phases.mu);
    const uint32_t n = g_phases.nctx < max_ctx ? g_phases.nctx : max_ctx;
    for (uint32_t ci = 0; ci < n; ++ci)
        for (uint32_t k = 0; k < kPhases; ++k) out[ci * kPhases + k] = g_phases.ms[ci][k];
    return n;
}

}  // extern "C"

namespace {

// n bytes from device memory of device src_dev to c's device, on c's stream
// (a device-to-device copy, or a peer copy over xGMI: a copy, not a collective).
int copy_dev(hg_ctx* c, void* dst, int src_dev, const void* src, size_t n) {
    if (!n) return HG_OK;
    // (HG_MULTI_TEST_PEER_COPY: the peer-copy call on one device too, so a
    // one-GPU box runs the branch the cross-GPU split takes)
    const hipError_t e = src_dev == c->device && hgk_knob("HG_MULTI_TEST_PEER_COPY", 0) != 1
                             ? hipMemcpyAsync(dst, src, n, hipMemcpyDeviceToDevice, c->stream)
                             : hipMemcpyPeerAsync(dst, c->device, src, src_dev, n, c->stream);
    return e == hipSuccess ? HG_OK : HG_HIP_FAIL;
}

// Direct peer access between every pair of the contexts' devices where the
// hardware allows it (xGMI); copies work without it too (staged by the runtime).
void enable_peers(hg_ctx* const* ctxs, uint32_t nctx) {
    // hipSetDevice below is per thread: the caller's device comes back on return
    DeviceGuard keep;
    for (uint32_t i = 0; i < nctx; ++i)
        for (uint32_t j = 0; j < nctx; ++j) {
            const int a = ctxs[i]->device, b = ctxs[j]->device;
            if (a == b) continue;
            int can = 0;
            if (hipDeviceCanAccessPeer(&can, a, b) != hipSuccess || !can) continue;
            if (hipSetDevice(a) == hipSuccess) (void)hipDeviceEnablePeerAccess(b, 0);  // may already be on
        }
    (void)hipGetLastError();
}

// Decoded tables of every context (owner[t]: the context holding table t at
// dptr[t]; sh[owner[t]].soff[slot[t]]: its spans in that context's mspans).
struct Owned {
    std::vector<Share> sh;
    std::vector<uint32_t> owner, slot;
    std::vector<const uint8_t*> dptr;
};

struct RangeOut {
    uint64_t n = 0, bytes = 0;
    uint32_t exact = 0;  // the slice's merge followed the reference loop (unsorted input)
    uint64_t redos = 0;  // merges redone after a look-back wait over its budget (table 3)
};

// The merge path of a split compaction for hg_merge_result: 0, or 3 with the
// redos of every range summed (the output is the same either way).
hg_merge_result split_result(const std::vector<RangeOut>& O, uint64_t nrec) {
    uint64_t redos = 0;
    for (const RangeOut& o : O) redos += o.redos;
    return hg_merge_result{nrec, HG_OK, redos ? 3u : 0u, redos};
}

// Steps 2-5 of a split compaction over decoded tables: samples -> splitters ->
// cut points -> every range on its context (slices gathered by device copies,
// merged, encoded into dsts[g] or, when dsts is null, c->d_out).  separable =
// false: the input is not range-separable (keys not strictly increasing at a
// cut or inside a slice); nothing usable was produced.
int split_compact(hg_ctx* const* ctxs, uint32_t nctx, uint32_t ntables, const uint64_t* lens,
                  Owned& ow, uint8_t* const* dsts, const uint64_t* caps, std::vector<RangeOut>& O,
                  bool& separable, double (*ph)[kPhases] = nullptr) {
    separable = true;
    const double t_cut0 = wall_ms();
    // 2. samples of every table's keys (on its owner), then nctx - 1 splitters
    std::vector<std::vector<KeyRef>> samples(nctx);
    constexpr uint64_t kSamples = 256;  // per table
    int r = fan_out(nctx, [&](uint32_t ci) {
        hg_ctx* c = ctxs[ci];
        Share& s = ow.sh[ci];
        if (s.ids.empty()) return (int)HG_OK;
        if (set_dev(c) != HG_OK) return (int)HG_HIP_FAIL;
        uint64_t m_tot = 0;
        for (size_t j = 0; j < s.ids.size(); ++j)
            if (s.res[j].n_records) m_tot += std::min<uint64_t>(kSamples, s.res[j].n_records);
        if (!m_tot) return (int)HG_OK;
        int rr = ensure(c, c->x_aux, m_tot * sizeof(KeyRef));
        if (rr != HG_OK) return rr;
        KeyRef* d = static_cast<KeyRef*>(c->x_aux.p);
        uint64_t at = 0;
        SampleArgs sa{};
        uint32_t k = 0;
        auto launch = [&]() -> int {  // the tables gathered so far, one launch
            if (!k) return (int)HG_OK;
            hipLaunchKernelGGL(sample_keys_kernel, dim3(k), dim3(kSamples), 0, c->stream, sa, d);
            k = 0;
            return HG_LAUNCH_STATUS();
        };
        for (size_t j = 0; j < s.ids.size(); ++j) {
            const uint64_t n = s.res[j].n_records;
            if (!n) continue;
            const uint64_t m = std::min<uint64_t>(kSamples, n);
            sa.t[k++] = SampleArgs::Tab{ow.dptr[s.ids[j]],
                                        static_cast<const hg_span*>(c->mspans.p) + s.soff[j], n,
                                        (n + m - 1) / m, at, (uint32_t)m, s.ids[j]};
            at += m;
            if (k == kSampleTabs && (rr = launch()) != HG_OK) return rr;
        }
        if ((rr = launch()) != HG_OK) return rr;
        samples[ci].resize(m_tot);
        return sync_d2h(c, samples[ci].data(), d, m_tot * sizeof(KeyRef));
    });
    if (r != HG_OK) return r;
    std::vector<KeyRef> all;
    for (auto& v : samples) all.insert(all.end(), v.begin(), v.end());
    std::vector<std::vector<uint8_t>> keys;
    if (!all.empty()) {
        std::sort(all.begin(), all.end(), [](const KeyRef& a, const KeyRef& b) {
            if (a.p0 != b.p0) return a.p0 < b.p0;
            if (a.p1 != b.p1) return a.p1 < b.p1;
            return a.klen < b.klen;
        });
        for (uint32_t g = 1; g < nctx; ++g) {  // the splitter's exact bytes
            const KeyRef& kr = all[all.size() * g / nctx];
            if (kr.klen <= 16) {  // the sampled prefix holds the whole key (no round trip)
                std::vector<uint8_t> k(kr.klen);
                for (uint32_t i = 0; i < kr.klen; ++i)
                    k[i] = (uint8_t)((i < 8 ? kr.p0 >> (56 - 8 * i) : kr.p1 >> (56 - 8 * (i - 8))) & 0xFF);
                keys.push_back(std::move(k));
                continue;
            }
            const uint32_t o = ow.owner[kr.table];  // longer keys: from the table's owner
            hg_ctx* c = ctxs[o];
            if (set_dev(c) != HG_OK) return HG_HIP_FAIL;
            hg_span sp;
            const hg_span* dsp = static_cast<const hg_span*>(c->mspans.p) + ow.sh[o].soff[ow.slot[kr.table]];
            if ((r = sync_d2h(c, &sp, dsp + kr.rec, sizeof sp)) != HG_OK) return r;
            std::vector<uint8_t> k(sp.klen);
            if (sp.klen && (r = sync_d2h(c, k.data(), ow.dptr[kr.table] + sp.off + 16, sp.klen)) != HG_OK)
                return r;
            keys.push_back(std::move(k));
        }
    }
    std::sort(keys.begin(), keys.end(),
              [](const std::vector<uint8_t>& a, const std::vector<uint8_t>& b) {
                  return host_key_cmp(a, b) < 0;
              });
    keys.erase(std::unique(keys.begin(), keys.end(),
                           [](const std::vector<uint8_t>& a, const std::vector<uint8_t>& b) {
                               return host_key_cmp(a, b) == 0;
                           }),
               keys.end());
    const uint32_t nsplit = (uint32_t)keys.size();
    const uint32_t nrange = nsplit + 1;
    // 3. cut points of every table (lower bound of each splitter) on its owner
    std::vector<uint64_t> kofs(nsplit + 1, 0);
    std::vector<uint32_t> kls(nsplit + 1, 0);
    std::vector<uint8_t> kbytes;
    for (uint32_t s = 0; s < nsplit; ++s) {
        kofs[s] = kbytes.size();
        kls[s] = (uint32_t)keys[s].size();
        kbytes.insert(kbytes.end(), keys[s].begin(), keys[s].end());
    }
    std::vector<std::vector<uint64_t>> cut_rec(ntables, std::vector<uint64_t>(nrange + 1, 0)),
        cut_off(ntables, std::vector<uint64_t>(nrange + 1, 0));
    std::vector<int> cut_ok(ntables, 1);
    r = fan_out(nctx, [&](uint32_t ci) {
        hg_ctx* c = ctxs[ci];
        const Share& s = ow.sh[ci];
        if (s.ids.empty()) return (int)HG_OK;
        if (set_dev(c) != HG_OK) return (int)HG_HIP_FAIL;
        for (size_t j = 0; j < s.ids.size(); ++j) {  // defaults: one range holds the table
            const uint32_t t = s.ids[j];
            for (uint32_t g = 1; g <= nrange; ++g) {
                cut_rec[t][g] = s.res[j].n_records;
                cut_off[t][g] = lens[t];
            }
        }
        if (!nsplit) return (int)HG_OK;
        // one stream-ordered upload from a pageable host blob laid out as on
        // the device: splitter bytes, offsets, lengths, 16-byte big-endian
        // prefixes, then this context's tables; one launch for all of them
        const uint32_t nt = (uint32_t)s.ids.size();
        const size_t kb = (kbytes.size() + 255) & ~(size_t)255;
        const size_t o_ko = kb, o_kl = o_ko + 8 * (nsplit + 1), o_kp = (o_kl + 4 * nsplit + 15) & ~(size_t)15;
        const size_t o_tb = (o_kp + 16 * (size_t)nsplit + 255) & ~(size_t)255;
        const size_t o_out = (o_tb + sizeof(SplitTab) * nt + 255) & ~(size_t)255;
        int rr = ensure(c, c->x_aux, o_out + 24 * (size_t)nsplit * nt);
        if (rr != HG_OK) return rr;
        char* d = static_cast<char*>(c->x_aux.p);
        std::vector<uint8_t> blob(o_out, 0);
        if (!kbytes.empty()) memcpy(blob.data(), kbytes.data(), kbytes.size());
        memcpy(blob.data() + o_ko, kofs.data(), 8 * (nsplit + 1));
        memcpy(blob.data() + o_kl, kls.data(), 4 * (size_t)nsplit);
        uint64_t* kp = reinterpret_cast<uint64_t*>(blob.data() + o_kp);
        for (uint32_t q = 0; q < nsplit; ++q) {  // prefix words as split_cmp compares them
            uint64_t w0 = 0, w1 = 0;
            for (uint32_t i = 0; i < 16; ++i) {
                const uint64_t b = i < kls[q] ? kbytes[kofs[q] + i] : 0;
                if (i < 8) w0 = (w0 << 8) | b;
                else w1 = (w1 << 8) | b;
            }
            kp[2 * q] = w0;
            kp[2 * q + 1] = w1;
        }
        SplitTab* tb = reinterpret_cast<SplitTab*>(blob.data() + o_tb);
        for (uint32_t j = 0; j < nt; ++j)
            tb[j] = SplitTab{ow.dptr[s.ids[j]], static_cast<const hg_span*>(c->mspans.p) + s.soff[j],
                             lens[s.ids[j]], s.res[j].n_records};
        if (hipMemcpyAsync(d, blob.data(), blob.size(), hipMemcpyHostToDevice, c->stream) != hipSuccess)
            return (int)HG_HIP_FAIL;
        uint64_t* dout = reinterpret_cast<uint64_t*>(d + o_out);
        const uint32_t waves = nt * nsplit;
        hipLaunchKernelGGL(split_points_kernel, dim3((waves + 3) / 4), dim3(256), 0, c->stream,
                           reinterpret_cast<const SplitTab*>(d + o_tb), nt,
                           reinterpret_cast<const uint8_t*>(d), reinterpret_cast<const uint64_t*>(d + o_ko),
                           reinterpret_cast<const uint32_t*>(d + o_kl),
                           reinterpret_cast<const uint64_t*>(d + o_kp), nsplit, dout);
        if ((rr = HG_LAUNCH_STATUS()) != HG_OK) return rr;
        std::vector<uint64_t> h(3 * (size_t)nsplit * s.ids.size());
        if ((rr = sync_d2h(c, h.data(), dout, 8 * h.size())) != HG_OK) return rr;
        for (size_t j = 0; j < s.ids.size(); ++j) {
            const uint32_t t = s.ids[j];
            for (uint32_t g = 0; g < nsplit; ++g) {
                cut_rec[t][g + 1] = h[3 * (nsplit * j + g)];
                cut_off[t][g + 1] = h[3 * (nsplit * j + g) + 1];
                if (!h[3 * (nsplit * j + g) + 2]) cut_ok[t] = 0;
            }
        }
        return (int)HG_OK;
    });
    if (r != HG_OK) return r;
    for (uint32_t t = 0; t < ntables; ++t) {
        for (uint32_t g = 0; g < nrange && cut_ok[t]; ++g)  // lower bounds of unordered keys
            if (cut_rec[t][g] > cut_rec[t][g + 1] || cut_off[t][g] > cut_off[t][g + 1])
                cut_ok[t] = 0;
        if (!cut_ok[t]) {
            separable = false;
            return HG_OK;
        }
    }
    if (ph)
        for (uint32_t ci = 0; ci < nctx && ci < kPhaseCtx; ++ci) ph[ci][1] = wall_ms() - t_cut0;
    // 4. range g on context g: its slice of every table copied from the
    //    table's owner (bytes and decoded spans, device to device: each byte
    //    crosses once, nothing is uploaded or decoded again), merged, encoded
    O.assign(nrange, RangeOut{});
    // (ph: timing events per range -- start, copies done, merged, encoded)
    struct TEvents {
        std::vector<hipEvent_t> ev;
        ~TEvents() {
            for (hipEvent_t e : ev)
                if (e) (void)hipEventDestroy(e);
        }
    } tev;
    if (ph) tev.ev.assign(4 * (size_t)nrange, nullptr);
    auto stamp = [&](uint32_t g, uint32_t k) {
        if (!ph || g >= kPhaseCtx) return;
        hipEvent_t& e = tev.ev[4 * (size_t)g + k];
        if (hipEventCreate(&e) != hipSuccess || hipEventRecord(e, ctxs[g]->stream) != hipSuccess) {
            (void)hipGetLastError();
            e = nullptr;
        }
    };
    // every owner's decode (and sample / cut work) is ordered before the copies
    // out of it by an event on its stream -- not only by the host having
    // synchronised it (decode_share's D2H), which an asynchronous decode would drop
    struct Events {
        std::vector<hipEvent_t> ev;
        ~Events() {
            for (hipEvent_t e : ev)
                if (e) (void)hipEventDestroy(e);
        }
    } evs;
    evs.ev.assign(nctx, nullptr);
    for (uint32_t ci = 0; ci < nctx; ++ci) {
        if (set_dev(ctxs[ci]) != HG_OK ||
            hipEventCreateWithFlags(&evs.ev[ci], hipEventDisableTiming) != hipSuccess ||
            hipEventRecord(evs.ev[ci], ctxs[ci]->stream) != hipSuccess)
            return HG_HIP_FAIL;
    }
    r = fan_out(nrange, [&](uint32_t g) {
        hg_ctx* c = ctxs[g];
        if (set_dev(c) != HG_OK) return (int)HG_HIP_FAIL;
        for (uint32_t ci = 0; ci < nctx; ++ci)
            if (ci != g && hipStreamWaitEvent(c->stream, evs.ev[ci], 0) != hipSuccess)
                return (int)HG_HIP_FAIL;
        stamp(g, 0);
        std::vector<uint64_t> pos(ntables), toff(ntables), cnt(ntables), sps(ntables);
        uint64_t ab = 0, nb = 0;
        for (uint32_t t = 0; t < ntables; ++t) {
            pos[t] = ab;
            ab += (cut_off[t][g + 1] - cut_off[t][g] + 255) & ~255ull;
            cnt[t] = cut_rec[t][g + 1] - cut_rec[t][g];
            sps[t] = nb;
            nb += cnt[t];
        }
        if (nb == 0) return (int)HG_OK;
        int rr = ensure(c, c->x_arena, ab + 256);
        if (rr == HG_OK) rr = ensure(c, c->x_spans, nb * sizeof(hg_span));
        if (rr == HG_OK) rr = ensure(c, c->mpairs, nb * sizeof(hg_pair));
        if (rr != HG_OK) return rr;
        uint8_t* arena = static_cast<uint8_t*>(c->x_arena.p);
        hg_span* spans = static_cast<hg_span*>(c->x_spans.p);
        std::vector<const hg_span*> sp(ntables);
        for (uint32_t t = 0; t < ntables; ++t) {
            const uint32_t o = ow.owner[t];
            const hg_span* osp = static_cast<const hg_span*>(ctxs[o]->mspans.p) + ow.sh[o].soff[ow.slot[t]];
            if ((rr = copy_dev(c, arena + pos[t], ctxs[o]->device, ow.dptr[t] + cut_off[t][g],
                               cut_off[t][g + 1] - cut_off[t][g])) != HG_OK ||
                (rr = copy_dev(c, spans + sps[t], ctxs[o]->device, osp + cut_rec[t][g],
                               cnt[t] * sizeof(hg_span))) != HG_OK)
                return rr;
            // spans keep their table-relative offsets: the slice's table offset
            // absorbs the cut (mod 2^64), so key and value addresses come out right
            toff[t] = pos[t] - cut_off[t][g];
            sp[t] = spans + sps[t];
        }
        stamp(g, 1);
        hg_merge_result mr{};
        rr = hg_merge_dev(c, ntables, arena, ab, toff.data(), sp.data(), cnt.data(),
                          static_cast<hg_pair*>(c->mpairs.p), nb, &mr);
        if (rr != HG_OK) return rr;
        O[g].n = mr.n_out;
        // table 3: sorted input, the parallel merge redone after a look-back
        // wait over its budget -- the slice is good
        O[g].exact = mr.table == 1 || mr.table == 2;
        O[g].redos = mr.table == 3 ? mr.index : 0;
        stamp(g, 2);
        if (O[g].exact) return (int)HG_OK;  // not range-separable: decided after the join
        uint8_t* dst = dsts ? dsts[g] : nullptr;
        uint64_t cap = dsts ? caps[g] : ab;
        if (!dsts) {
            if ((rr = ensure(c, c->d_out, ab ? ab : 1)) != HG_OK) return rr;
            dst = static_cast<uint8_t*>(c->d_out.p);
        }
        if ((rr = ensure(c, c->d_aux, (mr.n_out ? mr.n_out : 1) * sizeof(uint64_t))) != HG_OK)
            return rr;
        uint64_t enc = 0;
        rr = rt_encode_dev(c, arena, static_cast<const hg_pair*>(c->mpairs.p), mr.n_out, dst, cap,
                           static_cast<uint64_t*>(c->d_aux.p), 0, nullptr, &enc, true);
        // the slice's size also on HG_ERR_CAPACITY, so the caller can resize and retry
        O[g].bytes = enc;
        stamp(g, 3);
        return rr;
    });
    if (r != HG_OK) return r;
    for (uint32_t g = 0; ph && g < nrange && g < kPhaseCtx; ++g) {
        hipEvent_t* e = &tev.ev[4 * (size_t)g];
        for (uint32_t k = 0; k < 3; ++k) {
            float ms = 0.f;
            ph[g][2 + k] = (e[k] && e[k + 1] && hipEventSynchronize(e[k + 1]) == hipSuccess &&
                            hipEventElapsedTime(&ms, e[k], e[k + 1]) == hipSuccess)
                               ? (double)ms
                               : -1.0;
        }
    }
    (void)hipGetLastError();
    for (const RangeOut& o : O)
        if (o.exact) separable = false;
    return HG_OK;
}

}  // namespace

extern "C" {

int hg_multi_compact_host(hg_ctx* const* ctxs, uint32_t nctx, uint32_t ntables,
                          const uint8_t* const* h_tables, const uint64_t* lens, uint8_t* h_out,
                          uint64_t cap, uint64_t* out_len, uint32_t block_stride,
                          hg_block* h_blocks, hg_merge_result* result) {
    DeviceGuard keep;  // every device switch below is undone on return
    if (!ctxs || !nctx || (ntables && (!h_tables || !lens)) || (cap && !h_out))
        return HG_ERR_INVALID_ARG;
    if (h_blocks && block_stride == 0) return HG_ERR_INVALID_ARG;
    for (uint32_t i = 0; i < nctx; ++i)
        if (!ctxs[i]) return HG_ERR_INVALID_ARG;
    auto single = [&] {
        return hg_compact_host(ctxs[0], ntables, h_tables, lens, h_out, cap, out_len,
                               block_stride, h_blocks, result);
    };
    if (nctx == 1 || ntables == 0) return single();
    if (out_len) *out_len = 0;
    enable_peers(ctxs, nctx);
    // 1. every table uploaded once to its context (round-robin) and decoded there
    Owned ow;
    ow.sh = round_robin(nctx, ntables);
    ow.owner.resize(ntables);
    ow.slot.resize(ntables);
    ow.dptr.resize(ntables);
    int r = fan_out(nctx, [&](uint32_t ci) { return decode_share(ctxs[ci], ow.sh[ci], h_tables, lens); });
    if (r != HG_OK) return r;
    for (uint32_t ci = 0; ci < nctx; ++ci)
        for (size_t j = 0; j < ow.sh[ci].ids.size(); ++j) {
            const uint32_t t = ow.sh[ci].ids[j];
            if (ow.sh[ci].res[j].kind != HG_OK) return single();  // one context reports it
            ow.owner[t] = ci;
            ow.slot[t] = (uint32_t)j;
            ow.dptr[t] = static_cast<const uint8_t*>(ctxs[ci]->d_in.p) + ow.sh[ci].aoff[j];
        }
    std::vector<RangeOut> O;
    bool separable = true;
    if ((r = split_compact(ctxs, nctx, ntables, lens, ow, nullptr, nullptr, O, separable)) != HG_OK)
        return r;
    if (!separable) return single();
    const uint32_t nrange = (uint32_t)O.size();
    // 5. concatenate in key order (output offsets from the slice sizes)
    std::vector<uint64_t> OB(nrange + 1, 0), RB(nrange + 1, 0);
    for (uint32_t g = 0; g < nrange; ++g) {
        OB[g + 1] = OB[g] + O[g].bytes;
        RB[g + 1] = RB[g] + O[g].n;
    }
    const uint64_t total = OB[nrange], nrec = RB[nrange];
    if (out_len) *out_len = total;
    if (result) *result = split_result(O, nrec);
    if (total > cap) return HG_ERR_CAPACITY;
    const uint64_t nb = h_blocks ? (nrec + block_stride - 1) / block_stride : 0;
    std::vector<uint64_t> bpos(nb + 1, 0);
    r = fan_out(nrange, [&](uint32_t g) {
        hg_ctx* c = ctxs[g];
        if (set_dev(c) != HG_OK) return (int)HG_HIP_FAIL;
        int rr = O[g].bytes ? d2h_pipelined(c, h_out + OB[g], c->d_out.p, O[g].bytes) : HG_OK;
        if (rr != HG_OK || !nb || !O[g].n) return rr;
        // block starts inside this slice: global record b * stride
        const uint64_t first = (block_stride - RB[g] % block_stride) % block_stride;
        if (first >= O[g].n) return (int)HG_OK;
        const uint64_t m = (O[g].n - first + block_stride - 1) / block_stride;
        if ((rr = ensure(c, c->x_aux, m * 8)) != HG_OK) return rr;
        rr = hgk_gather_stride_launch(static_cast<const uint64_t*>(c->d_aux.p), O[g].n, first,
                                      block_stride, static_cast<uint64_t*>(c->x_aux.p), c->stream);
        std::vector<uint64_t> h(m);
        if (rr == HG_OK) rr = sync_d2h(c, h.data(), c->x_aux.p, m * 8);
        if (rr != HG_OK) return rr;
        const uint64_t b0 = (RB[g] + first) / block_stride;
        for (uint64_t j = 0; j < m; ++j) bpos[b0 + j] = OB[g] + h[j];
        return (int)HG_OK;
    });
    if (r != HG_OK) return r;
    for (uint64_t b = 0; b < nb; ++b) {
        h_blocks[b].first_rec = b * block_stride;
        h_blocks[b].position = bpos[b];
        h_blocks[b].length = (b + 1 < nb ? bpos[b + 1] : total) - bpos[b];
    }
    return HG_OK;
}

int hg_multi_compact_dev(hg_ctx* const* ctxs, uint32_t nctx, uint32_t ntables,
                         const uint32_t* owner, const uint8_t* const* d_tables,
                         const uint64_t* lens, uint8_t* const* d_outs, const uint64_t* caps,
                         uint64_t* out_lens, uint64_t* out_recs, hg_merge_result* result) {
    DeviceGuard keep;  // every device switch below is undone on return
    if (!ctxs || !nctx || !d_outs || !caps || !out_lens || !out_recs ||
        (ntables && (!owner || !d_tables || !lens)))
        return HG_ERR_INVALID_ARG;
    for (uint32_t i = 0; i < nctx; ++i)
        if (!ctxs[i]) return HG_ERR_INVALID_ARG;
    for (uint32_t t = 0; t < ntables; ++t) {
        if (owner[t] >= nctx || (lens[t] && !d_tables[t])) return HG_ERR_INVALID_ARG;
        if (lens[t] >= kMaxLen) return HG_ERR_TOO_LARGE;
    }
    for (uint32_t g = 0; g < nctx; ++g) out_lens[g] = out_recs[g] = 0;
    enable_peers(ctxs, nctx);
    // everything on context 0: the tables gathered there (device copies), one
    // hg_compact_dev -- the reference loop for input that is not range-separable
    auto single = [&]() -> int {
        hg_ctx* c = ctxs[0];
        if (set_dev(c) != HG_OK) return HG_HIP_FAIL;
        std::vector<uint64_t> pos(ntables);
        uint64_t ab = 0;
        for (uint32_t t = 0; t < ntables; ++t) {
            pos[t] = ab;
            ab += (lens[t] + 255) & ~255ull;
        }
        int rr = ensure(c, c->x_arena, ab + 256);
        if (rr != HG_OK) return rr;
        uint8_t* arena = static_cast<uint8_t*>(c->x_arena.p);
        for (uint32_t t = 0; t < ntables; ++t)
            if ((rr = copy_dev(c, arena + pos[t], ctxs[owner[t]]->device, d_tables[t], lens[t])) != HG_OK)
                return rr;
        hg_merge_result res{};
        uint64_t ol = 0;
        rr = hg_compact_dev(c, ntables, arena, ab, pos.data(), lens, d_outs[0], caps[0], &ol, 0,
                            nullptr, &res);
        out_lens[0] = ol;
        out_recs[0] = res.n_out;
        if (result) *result = res;
        return rr;
    };
    if (nctx == 1 || ntables == 0) return single();
    // 1. every context decodes the tables it holds, in place
    Owned ow;
    ow.sh.resize(nctx);
    ow.owner.assign(owner, owner + ntables);
    ow.slot.resize(ntables);
    ow.dptr.assign(d_tables, d_tables + ntables);
    for (uint32_t t = 0; t < ntables; ++t) {
        ow.slot[t] = (uint32_t)ow.sh[owner[t]].ids.size();
        ow.sh[owner[t]].ids.push_back(t);
    }
    double ph[kPhaseCtx][kPhases] = {};
    int r = fan_out(nctx, [&](uint32_t ci) {
        const double t0 = wall_ms();
        const int rr = decode_share_dev(ctxs[ci], ow.sh[ci], d_tables, lens);
        if (ci < kPhaseCtx) ph[ci][0] = wall_ms() - t0;
        return rr;
    });
    if (r != HG_OK) return r;
    for (uint32_t ci = 0; ci < nctx; ++ci)
        for (const hg_decode_result& res : ow.sh[ci].res)
            if (res.kind != HG_OK) return single();  // reports the table's error
    std::vector<RangeOut> O;
    bool separable = true;
    r = split_compact(ctxs, nctx, ntables, lens, ow, d_outs, caps, O, separable, ph);
    {
        std::lock_guard<std::mutex> g(g_phases.mu);
        g_phases.nctx = nctx < kPhaseCtx ? nctx : kPhaseCtx;
        for (uint32_t ci = 0; ci < g_phases.nctx; ++ci)
            for (uint32_t k = 0; k < kPhases; ++k) g_phases.ms[ci][k] = ph[ci][k];
    }
    if (r != HG_OK) {
        if (r == HG_ERR_CAPACITY)  // a slice did not fit its caller buffer
            for (uint32_t g = 0; g < O.size(); ++g) out_lens[g] = O[g].bytes;
        return r;
    }
    if (!separable) return single();
    uint64_t nrec = 0;
    for (uint32_t g = 0; g < O.size(); ++g) {
        out_lens[g] = O[g].bytes;
        out_recs[g] = O[g].n;
        nrec += O[g].n;
    }
    if (result) *result = split_result(O, nrec);
    return HG_OK;
}

}  // extern "C"
