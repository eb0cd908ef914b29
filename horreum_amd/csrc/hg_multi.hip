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
#include <thread>
#include <vector>

#include "hg_internal.hpp"

using namespace hgi;

namespace {

constexpr uint64_t kPiece = 16384;  // hg_decode.hip PIECE

// Run fn(i) for i in [0, n) on one host thread each; the first failing code.
template <typename F>
int fan_out(uint32_t n, F fn) {
    std::vector<int> rc(n, HG_OK);
    if (n == 1) {
        rc[0] = fn(0u);
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
    if (const char* e = getenv("HG_DECODE_GROUP_BYTES")) {
        const long long v = atoll(e);
        if (v > 0) return (uint64_t)v;
    }
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

__global__ void sample_keys_kernel(const uint8_t* table, const hg_span* spans, uint64_t n,
                                   uint64_t step, uint32_t tid, KeyRef* out, uint64_t m) {
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= m) return;
    const uint64_t rec = j * step < n ? j * step : n - 1;
    const hg_span sp = spans[rec];
    KeyRef r;
    key_prefix(table + sp.off + 16, sp.klen, r.p0, r.p1);
    r.klen = sp.klen;
    r.table = tid;
    r.rec = rec;
    out[j] = r;
}

// Vec<u8> Ord (shorter first on a common prefix).
__device__ int dkey_cmp(const uint8_t* a, uint32_t al, const uint8_t* b, uint32_t bl) {
    const uint32_t m = al < bl ? al : bl;
    for (uint32_t i = 0; i < m; ++i)
        if (a[i] != b[i]) return a[i] < b[i] ? -1 : 1;
    return al < bl ? -1 : (al > bl ? 1 : 0);
}

// For splitter key s: the first record with key >= s (lower bound), its byte
// offset (the table length past the end), and whether the two records around
// the cut are strictly increasing (a cut inside a run of equal or unordered
// keys cannot be merged slice by slice).
__global__ void split_points_kernel(const uint8_t* table, uint64_t len, const hg_span* spans,
                                    uint64_t n, const uint8_t* keys, const uint64_t* koff,
                                    const uint32_t* klen, uint32_t nsplit, uint64_t* out) {
    const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= nsplit) return;
    const uint8_t* key = keys + koff[s];
    const uint32_t kl = klen[s];
    uint64_t lo = 0, hi = n;
    while (lo < hi) {
        const uint64_t mid = lo + (hi - lo) / 2;
        const hg_span sp = spans[mid];
        if (dkey_cmp(table + sp.off + 16, sp.klen, key, kl) < 0) lo = mid + 1;
        else hi = mid;
    }
    uint64_t ok = 1;
    if (lo > 0 && lo < n) {
        const hg_span a = spans[lo - 1], b = spans[lo];
        ok = dkey_cmp(table + a.off + 16, a.klen, table + b.off + 16, b.klen) < 0;
    }
    out[3 * s] = lo;
    out[3 * s + 1] = lo < n ? spans[lo].off : len;
    out[3 * s + 2] = ok;
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
int hg_multi_compact_host(hg_ctx* const* ctxs, uint32_t nctx, uint32_t ntables,
                          const uint8_t* const* h_tables, const uint64_t* lens, uint8_t* h_out,
                          uint64_t cap, uint64_t* out_len, uint32_t block_stride,
                          hg_block* h_blocks, hg_merge_result* result) {
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
    // 1. decode every table on its context (round-robin), sample its keys
    std::vector<Share> sh = round_robin(nctx, ntables);
    std::vector<std::vector<KeyRef>> samples(nctx);
    constexpr uint64_t kSamples = 256;  // per table
    int r = fan_out(nctx, [&](uint32_t ci) {
        hg_ctx* c = ctxs[ci];
        Share& s = sh[ci];
        int rr = decode_share(c, s, h_tables, lens);
        if (rr != HG_OK) return rr;
        uint64_t m_tot = 0;
        for (size_t j = 0; j < s.ids.size(); ++j)
            if (s.res[j].kind == HG_OK && s.res[j].n_records)
                m_tot += std::min<uint64_t>(kSamples, s.res[j].n_records);
        if (!m_tot) return (int)HG_OK;
        if ((rr = ensure(c, c->x_aux, m_tot * sizeof(KeyRef))) != HG_OK) return rr;
        KeyRef* d = static_cast<KeyRef*>(c->x_aux.p);
        uint64_t at = 0;
        for (size_t j = 0; j < s.ids.size(); ++j) {
            const uint64_t n = s.res[j].n_records;
            if (s.res[j].kind != HG_OK || !n) continue;
            const uint64_t m = std::min<uint64_t>(kSamples, n);
            const uint64_t step = (n + m - 1) / m;
            hipLaunchKernelGGL(sample_keys_kernel, dim3((uint32_t)((m + 255) / 256)), dim3(256), 0,
                               c->stream, static_cast<const uint8_t*>(c->d_in.p) + s.aoff[j],
                               static_cast<const hg_span*>(c->mspans.p) + s.soff[j], n, step,
                               s.ids[j], d + at, m);
            at += m;
        }
        samples[ci].resize(m_tot);
        return sync_d2h(c, samples[ci].data(), d, m_tot * sizeof(KeyRef));
    });
    if (r != HG_OK) return r;
    for (uint32_t ci = 0; ci < nctx; ++ci)  // a table that does not decode: one context reports it
        for (const hg_decode_result& res : sh[ci].res)
            if (res.kind != HG_OK) return single();
    // 2. splitters: quantiles of the sampled keys (16-byte prefix order), then
    //    their exact bytes, sorted exactly and de-duplicated
    std::vector<KeyRef> all;
    for (auto& v : samples) all.insert(all.end(), v.begin(), v.end());
    if (all.empty()) return single();
    std::sort(all.begin(), all.end(), [](const KeyRef& a, const KeyRef& b) {
        if (a.p0 != b.p0) return a.p0 < b.p0;
        if (a.p1 != b.p1) return a.p1 < b.p1;
        return a.klen < b.klen;
    });
    std::vector<uint32_t> owner(ntables), slot(ntables);
    for (uint32_t ci = 0; ci < nctx; ++ci)
        for (size_t j = 0; j < sh[ci].ids.size(); ++j) {
            owner[sh[ci].ids[j]] = ci;
            slot[sh[ci].ids[j]] = (uint32_t)j;
        }
    std::vector<std::vector<uint8_t>> keys;
    for (uint32_t g = 1; g < nctx; ++g) {
        const KeyRef& kr = all[all.size() * g / nctx];
        hg_ctx* c = ctxs[owner[kr.table]];
        const Share& s = sh[owner[kr.table]];
        if (set_dev(c) != HG_OK) return HG_HIP_FAIL;
        hg_span sp;
        const hg_span* dsp = static_cast<const hg_span*>(c->mspans.p) + s.soff[slot[kr.table]];
        if ((r = sync_d2h(c, &sp, dsp + kr.rec, sizeof sp)) != HG_OK) return r;
        std::vector<uint8_t> k(sp.klen);
        if (sp.klen) memcpy(k.data(), h_tables[kr.table] + sp.off + 16, sp.klen);
        keys.push_back(std::move(k));
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
    // 3. cut points of every table (lower bound of each splitter), on the
    //    context holding the table; a cut between records that are not
    //    strictly increasing sends the whole compaction to one context
    std::vector<uint64_t> kofs(nsplit + 1, 0);
    std::vector<uint32_t> kls(nsplit);
    std::vector<uint8_t> kbytes;
    for (uint32_t s = 0; s < nsplit; ++s) {
        kofs[s] = kbytes.size();
        kls[s] = (uint32_t)keys[s].size();
        kbytes.insert(kbytes.end(), keys[s].begin(), keys[s].end());
    }
    // cut[t][g]: record index and byte offset where range g of table t starts
    std::vector<std::vector<uint64_t>> cut_rec(ntables, std::vector<uint64_t>(nrange + 1, 0)),
        cut_off(ntables, std::vector<uint64_t>(nrange + 1, 0));
    std::vector<int> cut_ok(ntables, 1);
    r = fan_out(nctx, [&](uint32_t ci) {
        hg_ctx* c = ctxs[ci];
        const Share& s = sh[ci];
        if (s.ids.empty()) return (int)HG_OK;
        if (set_dev(c) != HG_OK) return (int)HG_HIP_FAIL;
        const size_t kb = (kbytes.size() + 255) & ~(size_t)255;
        const size_t need = kb + 16 * (nsplit + 1) + 256 + 24 * (size_t)(nsplit + 1) * s.ids.size();
        int rr = ensure(c, c->x_aux, need);
        if (rr != HG_OK) return rr;
        char* d = static_cast<char*>(c->x_aux.p);
        uint8_t* dk = reinterpret_cast<uint8_t*>(d);
        uint64_t* dko = reinterpret_cast<uint64_t*>(d + kb);
        uint32_t* dkl = reinterpret_cast<uint32_t*>(d + kb + 8 * (nsplit + 1));
        uint64_t* dout = reinterpret_cast<uint64_t*>(d + kb + 16 * (nsplit + 1) + 256);
        if ((!kbytes.empty() && hipMemcpy(dk, kbytes.data(), kbytes.size(),
                                          hipMemcpyHostToDevice) != hipSuccess) ||
            hipMemcpy(dko, kofs.data(), 8 * (nsplit + 1), hipMemcpyHostToDevice) != hipSuccess ||
            (nsplit && hipMemcpy(dkl, kls.data(), 4 * nsplit, hipMemcpyHostToDevice) != hipSuccess))
            return (int)HG_HIP_FAIL;
        for (size_t j = 0; j < s.ids.size(); ++j)
            hipLaunchKernelGGL(split_points_kernel, dim3((nsplit + 63) / 64), dim3(64), 0, c->stream,
                               static_cast<const uint8_t*>(c->d_in.p) + s.aoff[j],
                               lens[s.ids[j]], static_cast<const hg_span*>(c->mspans.p) + s.soff[j],
                               s.res[j].n_records, (const uint8_t*)dk, (const uint64_t*)dko,
                               (const uint32_t*)dkl, nsplit, dout + 3 * (size_t)nsplit * j);
        std::vector<uint64_t> h(3 * (size_t)nsplit * s.ids.size());
        if ((rr = sync_d2h(c, h.data(), dout, 8 * h.size())) != HG_OK) return rr;
        for (size_t j = 0; j < s.ids.size(); ++j) {
            const uint32_t t = s.ids[j];
            cut_rec[t][nrange] = s.res[j].n_records;
            cut_off[t][nrange] = lens[t];
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
        // lower bounds over unordered keys need not be monotone either
        for (uint32_t g = 0; g < nrange && cut_ok[t]; ++g)
            if (cut_rec[t][g] > cut_rec[t][g + 1] || cut_off[t][g] > cut_off[t][g + 1])
                cut_ok[t] = 0;
        if (!cut_ok[t]) return single();
    }
    // 4. every range on its context: its slice of every table -> decode ->
    //    merge -> encode (+ record offsets for the block index)
    struct Out {
        uint64_t n = 0, bytes = 0;
        uint32_t exact = 0;
        int32_t kind = HG_OK;
    };
    std::vector<Out> O(nrange);
    const uint32_t nwork = std::min(nctx, nrange);
    r = fan_out(nwork, [&](uint32_t w) {
        for (uint32_t g = w; g < nrange; g += nwork) {  // nrange <= nctx: one range each
            hg_ctx* c = ctxs[w];
            std::vector<const uint8_t*> pt(ntables);
            std::vector<uint64_t> pl(ntables);
            for (uint32_t t = 0; t < ntables; ++t) {
                pt[t] = h_tables[t] + cut_off[t][g];
                pl[t] = cut_off[t][g + 1] - cut_off[t][g];
            }
            // reuse hg_compact_host's device pipeline, keeping the output on the
            // device: decode + merge + encode of the slices
            Share s;
            for (uint32_t t = 0; t < ntables; ++t) s.ids.push_back(t);
            int rr = decode_share(c, s, pt.data(), pl.data());
            if (rr != HG_OK) return rr;
            uint64_t nm = 0;
            std::vector<uint64_t> toff(ntables), counts(ntables);
            std::vector<const hg_span*> sp(ntables);
            for (uint32_t t = 0; t < ntables; ++t) {
                if (s.res[t].kind != HG_OK) return (int)HG_ERR_INTERNAL;  // cut off a boundary
                toff[t] = s.aoff[t];
                counts[t] = s.res[t].n_records;
                sp[t] = static_cast<const hg_span*>(c->mspans.p) + s.soff[t];
                nm += counts[t];
            }
            if ((rr = ensure(c, c->mpairs, (nm ? nm : 1) * sizeof(hg_pair))) != HG_OK) return rr;
            hg_merge_result mr{};
            uint64_t arena_len = 0;
            for (uint32_t t = 0; t < ntables; ++t) arena_len = std::max(arena_len, toff[t] + pl[t]);
            if (nm == 0) {
                O[g].n = 0;
                O[g].bytes = 0;
                continue;
            }
            rr = hg_merge_dev(c, ntables, static_cast<const uint8_t*>(c->d_in.p), arena_len,
                              toff.data(), sp.data(), counts.data(),
                              static_cast<hg_pair*>(c->mpairs.p), nm, &mr);
            if (rr != HG_OK) return rr;
            O[g].n = mr.n_out;
            O[g].exact = mr.table;
            if (mr.table) continue;  // not range-separable: decided after the join
            uint64_t enc = 0;
            if ((rr = ensure(c, c->d_out, arena_len ? arena_len : 1)) != HG_OK ||
                (rr = ensure(c, c->d_aux, (mr.n_out ? mr.n_out : 1) * sizeof(uint64_t))) != HG_OK)
                return rr;
            rr = rt_encode_dev(c, static_cast<const uint8_t*>(c->d_in.p),
                               static_cast<const hg_pair*>(c->mpairs.p), mr.n_out,
                               static_cast<uint8_t*>(c->d_out.p), arena_len,
                               static_cast<uint64_t*>(c->d_aux.p), 0, nullptr, &enc, true);
            if (rr != HG_OK) return rr;
            O[g].bytes = enc;
        }
        return (int)HG_OK;
    });
    if (r != HG_OK) return r;
    for (uint32_t g = 0; g < nrange; ++g)
        if (O[g].exact) return single();
    // 5. concatenate in key order (output offsets from the slice sizes)
    std::vector<uint64_t> OB(nrange + 1, 0), RB(nrange + 1, 0);
    for (uint32_t g = 0; g < nrange; ++g) {
        OB[g + 1] = OB[g] + O[g].bytes;
        RB[g + 1] = RB[g] + O[g].n;
    }
    const uint64_t total = OB[nrange], nrec = RB[nrange];
    if (out_len) *out_len = total;
    if (result) *result = hg_merge_result{nrec, HG_OK, 0, 0};
    if (total > cap) return HG_ERR_CAPACITY;
    const uint64_t nb = h_blocks ? (nrec + block_stride - 1) / block_stride : 0;
    std::vector<uint64_t> bpos(nb + 1, 0);
    r = fan_out(nwork, [&](uint32_t w) {
        for (uint32_t g = w; g < nrange; g += nwork) {
            hg_ctx* c = ctxs[w];
            if (set_dev(c) != HG_OK) return (int)HG_HIP_FAIL;
            int rr = O[g].bytes ? d2h_pipelined(c, h_out + OB[g], c->d_out.p, O[g].bytes) : HG_OK;
            if (rr != HG_OK || !nb || !O[g].n) return rr;
            // block starts inside this slice: global record b * stride
            const uint64_t first = (block_stride - RB[g] % block_stride) % block_stride;
            if (first >= O[g].n) continue;
            const uint64_t m = (O[g].n - first + block_stride - 1) / block_stride;
            if ((rr = ensure(c, c->x_aux, m * 8)) != HG_OK) return rr;
            rr = hgk_gather_stride_launch(static_cast<const uint64_t*>(c->d_aux.p), O[g].n, first,
                                          block_stride, static_cast<uint64_t*>(c->x_aux.p),
                                          c->stream);
            std::vector<uint64_t> h(m);
            if (rr == HG_OK) rr = sync_d2h(c, h.data(), c->x_aux.p, m * 8);
            if (rr != HG_OK) return rr;
            const uint64_t b0 = (RB[g] + first) / block_stride;
            for (uint64_t j = 0; j < m; ++j) bpos[b0 + j] = OB[g] + h[j];
        }
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

}  // extern "C"
