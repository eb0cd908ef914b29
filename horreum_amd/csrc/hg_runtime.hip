// hg_runtime.hip — host runtime behind include/horreum_gpu.h: contexts
// (device + stream + workspace), argument checking, sync/async entry points
// and the pinned host staging pipeline.  Kernels: hg_decode.hip,
// hg_encode.hip.
#include <hip/hip_runtime.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <mutex>
#include <new>
#include <thread>
#include <utility>
#include <vector>


#include "hg_internal.hpp"
#include "hg_knobs.hpp"

using namespace hgi;

namespace hgi {

}  // namespace hgi

// ---- HIP failure sites (hg_err.hpp) ----------------------------------------------
namespace hgerr {
static std::mutex g_mu;
static char g_msg[256];

static void record(const char* file, int line, hipError_t e) {
    const char* base = strrchr(file, '/');
    std::lock_guard<std::mutex> lk(g_mu);
    snprintf(g_msg, sizeof g_msg, "%s:%d: %s (%d)", base ? base + 1 : file, line,
             hipGetErrorName(e), (int)e);
}

void note(const char* file, int line) { record(file, line, hipPeekAtLastError()); }

int launch_status(const char* file, int line) {
    const hipError_t e = hipGetLastError();
    if (e == hipSuccess) return HG_OK;
    record(file, line, e);
    return HG_ERR_HIP;
}
}  // namespace hgerr

extern "C" const char* hg_last_hip_error(void) {
    static thread_local char copy[256];
    std::lock_guard<std::mutex> lk(hgerr::g_mu);
    memcpy(copy, hgerr::g_msg, sizeof copy);
    return copy;
}

namespace hgi {
// Every ABI entry starts here: besides selecting the device it drops a stale
// per-thread launch error left by earlier, unrelated runtime calls (a query
// that reported "not ready", a failed allocation already returned as
// HG_ERR_HIP), so the hipGetLastError() after this entry's own launches
// reports only those launches.
int set_dev(hg_ctx* c) {
    (void)hipGetLastError();
    return hipSetDevice(c->device) == hipSuccess ? HG_OK : HG_HIP_FAIL;
}

// Grow a device buffer; only ever called outside stream-ordered hot loops
// (hg_ctx_reserve pre-sizes everything the bench touches).
int ensure(hg_ctx* c, DevBuf& b, size_t bytes) {
    if (b.bytes >= bytes) return HG_OK;
    if (hipStreamSynchronize(c->stream) != hipSuccess) return HG_HIP_FAIL;
    if (b.p) hipFree(b.p);
    b.p = nullptr;
    b.bytes = 0;
    size_t want = std::max(bytes, (size_t)256);
    if (hipMalloc(&b.p, want) != hipSuccess) return HG_HIP_FAIL;
    b.bytes = want;
    // diagnostics knob: new buffers hold 0xA5 bytes, so a read of memory no
    // call wrote shows up whatever the allocator hands back
    if (hgk_knob("HG_DEBUG_POISON", 0) == 1 && hipMemsetAsync(b.p, 0xA5, want, c->stream) != hipSuccess)
        return HG_HIP_FAIL;
    return HG_OK;
}

// Grow b to `bytes` if that allocation succeeds (the old buffer is kept
// otherwise, and the HIP error cleared): false when it does not.
bool try_grow(hg_ctx* c, DevBuf& b, size_t bytes) {
    if (b.bytes >= bytes) return true;
    void* p = nullptr;
    if (hipMalloc(&p, bytes) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    if (hipStreamSynchronize(c->stream) != hipSuccess) {  // work queued on the old buffer
        (void)hipFree(p);
        return false;
    }
    if (b.p) (void)hipFree(b.p);
    b.p = p;
    b.bytes = bytes;
    if (hgk_knob("HG_DEBUG_POISON", 0) == 1) (void)hipMemsetAsync(b.p, 0xA5, bytes, c->stream);
    return true;
}

int ensure_pin(PinBuf& b, size_t bytes) {
    if (b.bytes >= bytes) return HG_OK;
    if (b.p) hipHostFree(b.p);
    b.p = nullptr;
    b.bytes = 0;
    if (hipHostMalloc(&b.p, bytes, hipHostMallocDefault) != hipSuccess) return HG_HIP_FAIL;
    b.bytes = bytes;
    return HG_OK;
}

}  // namespace hgi

namespace {

hg_decode_result* dres(hg_ctx* c) { return reinterpret_cast<hg_decode_result*>(c->results.p); }
hg_encode_result* eres(hg_ctx* c) {
    return reinterpret_cast<hg_encode_result*>(reinterpret_cast<char*>(c->results.p) + 64);
}

}  // namespace

extern "C" {

// Diagnostics only (not in include/horreum_gpu.h): the decode workspace and a
// blocking device->host copy, for tools/spec_diag.py.
void* hgk_ctx_workspace(hg_ctx* c) { return c ? c->ws.p : nullptr; }
// the control region (DecodeCtl, group sums, links, statuses) of the last
// single-table decode (hg_decode_dev_async: two regions used in turn)
void* hgk_ctx_decode_ctl(hg_ctx* c) {
    if (!c || !c->dctl.p) return nullptr;
    const uint64_t half = c->dctl.bytes / 2 & ~(uint64_t)255;
    return static_cast<char*>(c->dctl.p) + (1 - c->dctl_cur) * half;
}
// Diagnostics: device bytes the context's work buffers hold (tests check
// that hg_ctx_reserve leaves nothing for the first calls to grow).
uint64_t hgk_ctx_device_bytes(hg_ctx* c) {
    if (!c) return 0;
    uint64_t t = 0;
    for (const DevBuf* b : {&c->ws, &c->dctl, &c->bctl, &c->egs, &c->recoff, &c->results, &c->d_in, &c->d_out,
                            &c->d_aux, &c->d_blk, &c->mws, &c->mres, &c->mspans, &c->mpairs, &c->lk_index,
                            &c->lk_keys, &c->lk_res, &c->bws, &c->bstage_d, &c->x_res, &c->x_aux, &c->x_arena,
                            &c->x_spans})
        t += b->bytes;
    for (int i = 0; i < c->naux; ++i) t += c->aux_ws[i].bytes;
    return t;
}
int hgk_debug_d2h(void* dst, const void* src, uint64_t n) {
    return hipMemcpy(dst, src, n, hipMemcpyDeviceToHost) == hipSuccess ? HG_OK : HG_HIP_FAIL;
}

int hg_abi_version(void) { return HG_ABI_VERSION; }

// ---- knobs (hg_set_knob): the only run-time switches of the library --------
namespace {
struct Knob {
    const char* name;
    int64_t value;
    bool set;
};
Knob g_knobs[] = {
    {"HG_DECODE_BP", 0, false},          // pieces per general decode batch (power of two)
    {"HG_DECODE_SBP", 0, false},         // pieces per pre-pass batch
    {"HG_DECODE_BATCH", 0, false},       // 1: batched decode on auxiliary streams
    {"HG_DECODE_STREAMS", 0, false},     // auxiliary streams of that mode
    {"HG_DECODE_GROUP_BYTES", 0, false}, // device byte budget of a multi-context decode group
    {"HG_DECODE_HOST_SERIAL", 0, false}, // 1: host decode without the overlapped chunks
    {"HG_DEC_CHUNK_MB", 0, false},       // host decode chunk (MiB)
    {"HG_ENCODE_HOST_SERIAL", 0, false}, // 1: host encode without the overlapped chunks
    {"HG_ENC_CHUNK_MB", 0, false},       // host encode output chunk (MiB)
    {"HG_HOST_TIMING", 0, false},        // 1: host encode phase times on stderr
    {"HG_HOST_COPY_THREADS", 0, false},  // host staging copy threads
    {"HG_COMPACT_KPRE", 0, false},       // 0: no key prefixes from the compaction decode
    {"HG_COMPACT_PREBUILD", 0, false},   // 0: merge entries built after the host has the counts
    {"HG_COMPACT_ENCODE", 0, false},     // 1: compaction encode by the general pair gather
    {"HG_COMPACT_RECORDS", 0, false},    // 1: compaction merge writes the records (no pairs, no encode pass)
    {"HG_COMPACT_MERGE_SUMS", 0, false}, // 0: the records encode sums its tiles itself (not the merge)
    {"HG_MERGE_KENT", 0, false},         // 0: merge entries by merge_prep_kernel
    {"HG_MERGE_KWAY", 0, false},         // 1: the one-pass k-way merge (3..KW_MAX runs)
    {"HG_MERGE_SERIAL", 0, false},       // 1: the reference loop (rank path), 2: the round-2 loop
    {"HG_MERGE_TEST_EPOCH_FAIL", 0, false},  // test hook: epoch k reports a failure
    {"HG_MERGE_TEST_LB_EXPIRE", 0, false},   // test hook: the first merge's final-round tile k
                                             // acts as if its look-back wait ran over budget
    {"HG_RANK_NOPACK", 0, false},        // 1: rank path with plain ranks at any size
    {"HG_MULTI_TEST_PEER_COPY", 0, false},  // test hook: 1: same-device context copies also
                                             // take the peer-copy call (the cross-GPU branch)
    {"HG_DEBUG_POISON", 0, false},       // 1: new device buffers filled with 0xA5 (diagnostics)
};
std::mutex g_knob_mu;
Knob* find_knob(const char* name) {
    if (!name) return nullptr;
    for (Knob& k : g_knobs)
        if (strcmp(k.name, name) == 0) return &k;
    return nullptr;
}
}  // namespace

int64_t hgk_knob(const char* name, int64_t dflt) {
    std::lock_guard<std::mutex> g(g_knob_mu);
    const Knob* k = find_knob(name);
    return k && k->set ? k->value : dflt;
}

int hg_set_knob(const char* name, int64_t value) {
    std::lock_guard<std::mutex> g(g_knob_mu);
    Knob* k = find_knob(name);
    if (!k) return HG_ERR_INVALID_ARG;
    k->set = value >= 0;
    k->value = value >= 0 ? value : 0;
    return HG_OK;
}

int hg_get_knob(const char* name, int64_t* value) {
    std::lock_guard<std::mutex> g(g_knob_mu);
    const Knob* k = find_knob(name);
    if (!k || !value) return HG_ERR_INVALID_ARG;
    *value = k->set ? k->value : -1;
    return HG_OK;
}

const char* hg_status_string(int s) {
    switch (s) {
        case HG_OK: return "ok";
        case HG_ERR_TRUNCATED_HEADER: return "truncated record header (UnexpectedEof)";
        case HG_ERR_TRUNCATED_BODY: return "truncated record body (UnexpectedEof)";
        case HG_ERR_LEN_OVERFLOW: return "key_len + value_len overflows u64";
        case HG_ERR_SPAN_RANGE: return "key or value length >= 2^32 (span limit)";
        case HG_ERR_CAPACITY: return "output buffer too small";
        case HG_ERR_INVALID_ARG: return "invalid argument";
        case HG_ERR_HIP: return "HIP runtime error";
        case HG_ERR_TOO_LARGE: return "input too large (>= 2^40 bytes)";
        case HG_ERR_INTERNAL: return "internal error (device spin timeout)";
        case HG_ERR_EMPTY_MERGE: return "merge of zero records";
        case HG_ERR_UNSORTED: return "retired status (merge input not strictly increasing, ABI <= 3)";
        default: return "unknown status";
    }
}

int hg_ctx_create(int device, hg_ctx** out) {
    if (!out) return HG_ERR_INVALID_ARG;
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev)
        return HG_ERR_INVALID_ARG;
    hg_ctx* c = new (std::nothrow) hg_ctx();
    if (!c) return HG_ERR_INTERNAL;
    c->device = device;
    if (set_dev(c) != HG_OK || hipStreamCreateWithFlags(&c->own, hipStreamNonBlocking) != hipSuccess) {
        delete c;
        return HG_HIP_FAIL;
    }
    c->stream = c->own;
    if (ensure(c, c->results, 256) != HG_OK || ensure_pin(c->hres, 256) != HG_OK) {
        hg_ctx_destroy(c);
        return HG_HIP_FAIL;
    }
    *out = c;
    return HG_OK;
}

int hg_ctx_destroy(hg_ctx* c) {
    if (!c) return HG_ERR_INVALID_ARG;
    hipSetDevice(c->device);
    if (c->stream) hipStreamSynchronize(c->stream);
    for (DevBuf* b : {&c->ws, &c->dctl, &c->bctl, &c->egs, &c->recoff, &c->results, &c->d_in, &c->d_out, &c->d_aux, &c->d_blk, &c->mws,
                      &c->mres, &c->mspans, &c->mpairs, &c->lk_index, &c->lk_keys, &c->lk_res,
                      &c->bws, &c->bstage_d, &c->x_res, &c->x_aux, &c->x_arena, &c->x_spans})
        if (b->p) hipFree(b->p);
    for (PinBuf* b : {&c->hres, &c->h_stage[0], &c->h_stage[1], &c->mstage, &c->bstage, &c->kres})
        if (b->p) hipHostFree(b->p);
    if (c->mstage_ev) hipEventDestroy(c->mstage_ev);
    if (c->kres_ev) hipEventDestroy(c->kres_ev);
    if (c->bstage_ev) hipEventDestroy(c->bstage_ev);
    for (int i = 0; i < c->naux; ++i) {
        if (c->aux[i]) hipStreamDestroy(c->aux[i]);
        if (c->aux_ws[i].p) hipFree(c->aux_ws[i].p);
        if (c->join_ev[i]) hipEventDestroy(c->join_ev[i]);
    }
    if (c->fork_ev) hipEventDestroy(c->fork_ev);
    if (c->own) hipStreamDestroy(c->own);
    delete c;
    return HG_OK;
}

int hg_ctx_trim(hg_ctx* c) {
    if (!c) return HG_ERR_INVALID_ARG;
    if (set_dev(c) != HG_OK) return HG_HIP_FAIL;
    if (c->stream && hipStreamSynchronize(c->stream) != hipSuccess) return HG_HIP_FAIL;
    c->dctl_clean[0] = c->dctl_clean[1] = 0;
    c->egs_clean[0] = c->egs_clean[1] = 0;
    c->bctl_off[0].clear();
    c->bctl_off[1].clear();
    c->bstage_shadow[0].clear();
    c->bstage_shadow[1].clear();
    for (DevBuf* b : {&c->ws, &c->dctl, &c->bctl, &c->egs, &c->bstage_d, &c->recoff, &c->d_in, &c->d_out, &c->d_aux, &c->d_blk, &c->mws,
                      &c->mspans, &c->mpairs, &c->lk_index, &c->lk_keys, &c->lk_res, &c->bws,
                      &c->x_aux, &c->x_arena, &c->x_spans}) {
        if (b->p) hipFree(b->p);
        b->p = nullptr;
        b->bytes = 0;
    }
    for (int i = 0; i < c->naux; ++i) {
        if (c->aux[i] && hipStreamSynchronize(c->aux[i]) != hipSuccess) return HG_HIP_FAIL;
        if (c->aux_ws[i].p) hipFree(c->aux_ws[i].p);
        c->aux_ws[i].p = nullptr;
        c->aux_ws[i].bytes = 0;
    }
    return HG_OK;
}

int hg_ctx_set_stream(hg_ctx* c, void* s) {
    if (!c) return HG_ERR_INVALID_ARG;
    c->stream = reinterpret_cast<hipStream_t>(s);
    return HG_OK;
}

int hg_ctx_use_own_stream(hg_ctx* c) {
    if (!c) return HG_ERR_INVALID_ARG;
    c->stream = c->own;
    return HG_OK;
}

void* hg_ctx_stream(hg_ctx* c) { return c ? reinterpret_cast<void*>(c->stream) : nullptr; }

int hg_ctx_synchronize(hg_ctx* c) {
    if (!c) return HG_ERR_INVALID_ARG;
    return hipStreamSynchronize(c->stream) == hipSuccess ? HG_OK : HG_HIP_FAIL;
}

// A stream being captured into a graph: every stream-ordered entry point
// refuses it (HG_ERR_INVALID_ARG, nothing enqueued).  A context carries state
// from call to call -- which control half the previous call's kernels left
// clear, argument staging halves, pinned argument copies -- that a graph
// replay would not follow, and a captured single-table decode faulted the
// GPU on its first replay (round 6); capture is not supported.
static bool capturing(hipStream_t s) {
    hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(s, &st) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    return st != hipStreamCaptureStatusNone;
}

// The single-table decode's two control regions (hg_ctx::dctl) for a table
// of len bytes; a new allocation holds nothing known to be zero.
static int ensure_dctl(hg_ctx* c, uint64_t len) {
    const uint64_t need = 2 * ((hgk_decode_ctl_bytes(len) + 255) & ~(uint64_t)255);
    if (c->dctl.bytes >= need) return HG_OK;
    c->dctl_clean[0] = c->dctl_clean[1] = 0;
    return ensure(c, c->dctl, need);
}

int hg_ctx_reserve(hg_ctx* c, uint64_t max_sst_bytes, uint64_t max_pairs) {
    if (!c) return HG_ERR_INVALID_ARG;
    if (set_dev(c) != HG_OK) return HG_HIP_FAIL;
    size_t need = std::max(hgk_decode_workspace_bytes(max_sst_bytes),
                           hgk_encode_workspace_bytes(max_pairs));
    int r = ensure(c, c->ws, need);
    if (r == HG_OK && max_sst_bytes) r = ensure_dctl(c, max_sst_bytes);
    if (r == HG_OK && max_pairs) r = ensure(c, c->recoff, max_pairs * sizeof(uint64_t));
    if (r == HG_OK && max_pairs) {  // the encode's group-sum halves
        uint64_t first = 0, ng = 0;
        hgk_encode_group_sums(max_pairs, &first, &ng);
        const uint64_t gneed = 2 * ((ng * 8 + 255) & ~(uint64_t)255);
        if (c->egs.bytes < gneed) {
            c->egs_clean[0] = c->egs_clean[1] = 0;
            r = ensure(c, c->egs, gneed);
        }
    }
    if (r == HG_OK && max_sst_bytes) {  // a one-table batched decode's control + staging
        const uint64_t ctot = (hgk_decode_ctl_bytes(max_sst_bytes) + 255) & ~255ull;
        const uint64_t sbh = (hgk_decode_multi_stage_bytes(1) + 255) & ~(uint64_t)255;
        if (c->bctl.bytes < 2 * ctot) {
            c->bctl_off[0].clear();
            c->bctl_off[1].clear();
            r = ensure(c, c->bctl, 2 * ctot);
        }
        if (r == HG_OK && c->bstage_d.bytes < 2 * sbh) {
            c->bstage_shadow[0].clear();
            c->bstage_shadow[1].clear();
            r = ensure(c, c->bstage_d, 2 * sbh);
        }
        if (r == HG_OK && ensure_pin(c->bstage, hgk_decode_multi_stage_bytes(1)) != HG_OK)
            r = HG_HIP_FAIL;
        if (r == HG_OK && ensure(c, c->bws, (hgk_decode_workspace_bytes(max_sst_bytes) + 255) & ~255ull) != HG_OK)
            r = HG_HIP_FAIL;
    }
    return r;
}

uint64_t hg_block_count(uint64_t n, uint32_t stride) {
    return stride ? (n + stride - 1) / stride : 0;
}

// ---- decode ------------------------------------------------------------------
int hg_decode_dev_async(hg_ctx* c, const uint8_t* d_sst, uint64_t len, hg_span* d_spans,
                        uint64_t cap, hg_decode_result* d_result) {
    if (!c || !d_result || (len && !d_sst) || (cap && !d_spans)) return HG_ERR_INVALID_ARG;
    if (len >= kMaxLen) return HG_ERR_TOO_LARGE;
    if (set_dev(c) != HG_OK) return HG_HIP_FAIL;
    if (capturing(c->stream)) return HG_ERR_INVALID_ARG;
    if (len == 0)  // empty file: zero records (src/format.rs:54 loop never runs)
        return hipMemsetAsync(d_result, 0, sizeof(hg_decode_result), c->stream) == hipSuccess
                   ? HG_OK
                   : HG_HIP_FAIL;
    int r = ensure(c, c->ws, hgk_decode_workspace_bytes(len));
    if (r != HG_OK) return r;
    if ((r = ensure_dctl(c, len)) != HG_OK) return r;
    const uint64_t half = c->dctl.bytes / 2 & ~(uint64_t)255;
    char* base = static_cast<char*>(c->dctl.p);
    const int cur = c->dctl_cur;
    uint64_t zeroed = 0;
    r = hgk_decode_launch_ctl(d_sst, len, d_spans, cap, d_result, c->ws.p, base + cur * half,
                              c->dctl_clean[cur], base + (1 - cur) * half, half, &zeroed,
                              c->stream);
    c->dctl_clean[cur] = 0;  // this call's statuses
    c->dctl_clean[1 - cur] = r == HG_OK ? zeroed : 0;
    c->dctl_cur = 1 - cur;
    return r;
}

static int finish_decode(const hg_decode_result& res, uint64_t cap, uint64_t* n_out,
                         hg_err* err) {
    if (n_out) *n_out = res.n_records;
    if (err) {
        err->kind = res.kind;
        err->reserved = 0;
        err->offset = res.err_offset;
    }
    if (res.kind != HG_OK) return res.kind;
    return res.n_records > cap ? HG_ERR_CAPACITY : HG_OK;
}

int hg_decode_dev(hg_ctx* c, const uint8_t* d_sst, uint64_t len, hg_span* d_spans, uint64_t cap,
                  uint64_t* n_out, hg_err* err) {
    int r = hg_decode_dev_async(c, d_sst, len, d_spans, cap, c ? dres(c) : nullptr);
    if (r != HG_OK) return r;
    if (hipMemcpyAsync(c->hres.p, dres(c), sizeof(hg_decode_result), hipMemcpyDeviceToHost,
                       c->stream) != hipSuccess ||
        hipStreamSynchronize(c->stream) != hipSuccess)
        return HG_HIP_FAIL;
    return finish_decode(*reinterpret_cast<hg_decode_result*>(c->hres.p), cap, n_out, err);
}

// Batched decode (many independent tables, e.g. the 256 tables of BASELINE
// config 4).  Default: ONE launch chain for all tables (hgk_decode_launch_multi:
// every table's batches in one grid, per-table workspaces side by side), so
// small tables fill the chip together instead of queueing launch by launch.
// HG_DECODE_BATCH=streams selects the older fan-out: tables round-robin over
// auxiliary streams forked from and joined back into the context stream
// (HG_DECODE_STREAMS, 1..8, default 4).  Asynchronous; results land in
// d_results[i].
static int rt_ensure_aux(hg_ctx* c, int want) {
    if (!c->fork_ev && hipEventCreateWithFlags(&c->fork_ev, hipEventDisableTiming) != hipSuccess)
        return HG_HIP_FAIL;
    while (c->naux < want) {
        const int i = c->naux;
        if (hipStreamCreateWithFlags(&c->aux[i], hipStreamNonBlocking) != hipSuccess ||
            hipEventCreateWithFlags(&c->join_ev[i], hipEventDisableTiming) != hipSuccess)
            return HG_HIP_FAIL;
        ++c->naux;
    }
    return HG_OK;
}

// The one-launch batched decode.  kpre_tag != 0: compaction mode (stride
// pieces leave key prefixes for the merge, see hg_decode.hip); ws_off (if
// given) receives every table's workspace offset in c->bws.
static int batch_one_launch(hg_ctx* c, uint32_t ntables, const uint8_t* const* d_tables,
                            const uint64_t* lens, hg_span* const* d_spans, const uint64_t* caps,
                            hg_decode_result* d_results, uint32_t kpre_tag,
                            std::vector<uint64_t>* ws_off) {
    if (ntables == 0) return HG_OK;
    std::vector<uint64_t> off(ntables);
    uint64_t total = 0;
    for (uint32_t i = 0; i < ntables; ++i) {
        off[i] = total;
        total += (hgk_decode_workspace_bytes(lens[i]) + 255) & ~255ull;
    }
    const uint64_t sb = hgk_decode_multi_stage_bytes(ntables);
    // the tables' control regions, in each half of c->bctl
    std::vector<uint64_t> coff(ntables);
    uint64_t ctot = 0;
    for (uint32_t i = 0; i < ntables; ++i) {
        coff[i] = ctot;
        ctot += (hgk_decode_ctl_bytes(lens[i]) + 255) & ~255ull;
    }
    if (c->bctl.bytes < 2 * ctot) {  // a new allocation holds nothing known to be zero
        for (int h = 0; h < 2; ++h) c->bctl_off[h].clear();
    }
    const uint64_t sbh = (sb + 255) & ~(uint64_t)255;
    if (c->bstage_d.bytes < 2 * sbh) c->bstage_shadow[0].clear(), c->bstage_shadow[1].clear();
    int r = ensure(c, c->bws, total ? total : 256);
    if (r == HG_OK) r = ensure(c, c->bctl, 2 * (ctot ? ctot : 256));
    if (r == HG_OK) r = ensure(c, c->bstage_d, 2 * sbh);
    if (r == HG_OK && !c->bstage_ev &&
        hipEventCreateWithFlags(&c->bstage_ev, hipEventDisableTiming) != hipSuccess)
        r = HG_HIP_FAIL;
    // the previous call's arguments may still be in flight from the pinned stage
    if (r == HG_OK && c->bstage_busy && hipEventSynchronize(c->bstage_ev) != hipSuccess)
        r = HG_HIP_FAIL;
    if (r == HG_OK && ensure_pin(c->bstage, sb) != HG_OK) r = HG_HIP_FAIL;
    const uint64_t half = c->bctl.bytes / 2 & ~(uint64_t)255;
    const int cur = c->bctl_cur;
    char* base = static_cast<char*>(c->bctl.p);
    std::vector<uint64_t> next_zero(ntables, 0);
    int copied = 1;
    std::vector<uint8_t>& shadow = c->bstage_shadow[cur];
    // the staging halves split the buffer, not this call's size: a half's
    // place must not move with the table count, or a smaller call's second
    // half would land in the first half's bytes (whose shadow then lies)
    const uint64_t shalf = c->bstage_d.bytes / 2 & ~(uint64_t)255;
    void* const d_stage = static_cast<char*>(c->bstage_d.p) + cur * shalf;
    const hgk_multi_ctl mc{base + cur * half,
                           base + (1 - cur) * half,
                           coff.data(),
                           c->bctl_off[cur] == coff ? c->bctl_zero[cur].data() : nullptr,
                           next_zero.data(),
                           shadow.empty() ? nullptr : shadow.data(),
                           shadow.size(),
                           &copied,
                           c->bstage_ev};
    if (r == HG_OK)
        r = hgk_decode_launch_multi(ntables, d_tables, lens, d_spans, caps, d_results, c->bws.p,
                                    off.data(), c->bstage.p, d_stage, c->stream, kpre_tag, &mc);
    c->bstage_last = d_stage;
    // this call dirtied its half; the other is clear where its pre-pass ran
    c->bctl_off[cur].clear();
    if (r == HG_OK) {
        c->bctl_off[1 - cur] = coff;
        c->bctl_zero[1 - cur] = std::move(next_zero);
        if (copied) {
            const uint8_t* hs = static_cast<const uint8_t*>(c->bstage.p);
            shadow.assign(hs, hs + sb);
        }
    } else {
        c->bctl_off[1 - cur].clear();
        shadow.clear();
    }
    c->bctl_cur = 1 - cur;
    if (r != HG_OK) return r;
    // bstage_ev was recorded behind the argument copy (if one ran): the next
    // call's host staging waits for that copy only, not for this decode
    c->bstage_busy = copied != 0;
    if (ws_off) *ws_off = std::move(off);
    return HG_OK;
}

int hg_decode_batch_dev_async(hg_ctx* c, uint32_t ntables, const uint8_t* const* d_tables,
                              const uint64_t* lens, hg_span* const* d_spans,
                              const uint64_t* caps, hg_decode_result* d_results) {
    if (!c || (ntables && (!d_tables || !lens || !d_spans || !caps || !d_results)))
        return HG_ERR_INVALID_ARG;
    for (uint32_t i = 0; i < ntables; ++i) {
        if ((lens[i] && !d_tables[i]) || (caps[i] && !d_spans[i])) return HG_ERR_INVALID_ARG;
        if (lens[i] >= kMaxLen) return HG_ERR_TOO_LARGE;
    }
    if (set_dev(c) != HG_OK) return HG_HIP_FAIL;
    if (capturing(c->stream)) return HG_ERR_INVALID_ARG;
    if (hgk_knob("HG_DECODE_BATCH", 0) != 1)
        return batch_one_launch(c, ntables, d_tables, lens, d_spans, caps, d_results, 0, nullptr);
    int fan = (int)hgk_knob("HG_DECODE_STREAMS", 4);
    fan = std::max(1, std::min<int>(fan, hg_ctx::kAux));
    fan = std::min<int>(fan, std::max<uint32_t>(ntables, 1));
    int r = rt_ensure_aux(c, fan);
    if (r != HG_OK) return r;
    // size every auxiliary workspace first (growing synchronises that stream)
    for (int s = 0; s < fan; ++s) {
        uint64_t need = 0;
        for (uint32_t i = s; i < ntables; i += fan)
            need = std::max<uint64_t>(need, hgk_decode_workspace_bytes(lens[i]));
        DevBuf& b = c->aux_ws[s];
        if (need > b.bytes) {
            if (hipStreamSynchronize(c->aux[s]) != hipSuccess) return HG_HIP_FAIL;
            if (b.p) hipFree(b.p);
            b.p = nullptr;
            b.bytes = 0;
            if (hipMalloc(&b.p, need) != hipSuccess) return HG_HIP_FAIL;
            b.bytes = need;
        }
    }
    if (hipEventRecord(c->fork_ev, c->stream) != hipSuccess) return HG_HIP_FAIL;
    for (int s = 0; s < fan; ++s)
        if (hipStreamWaitEvent(c->aux[s], c->fork_ev, 0) != hipSuccess) return HG_HIP_FAIL;
    for (uint32_t i = 0; i < ntables; ++i) {
        const int s = (int)(i % (uint32_t)fan);
        if (lens[i] == 0) {
            if (hipMemsetAsync(d_results + i, 0, sizeof(hg_decode_result), c->aux[s]) != hipSuccess)
                return HG_HIP_FAIL;
            continue;
        }
        r = hgk_decode_launch(d_tables[i], lens[i], d_spans[i], caps[i], d_results + i,
                              c->aux_ws[s].p, c->aux[s]);
        if (r != HG_OK) return r;
    }
    for (int s = 0; s < fan; ++s)
        if (hipEventRecord(c->join_ev[s], c->aux[s]) != hipSuccess ||
            hipStreamWaitEvent(c->stream, c->join_ev[s], 0) != hipSuccess)
            return HG_HIP_FAIL;
    return HG_OK;
}

// Host bytes in, host spans out.  Host buffers move in 64 MiB pieces:
//  - pinned (hipHostMalloc'd, or registered with hg_host_register, e.g. an
//    mmap'd SSTable file kept registered by the caller): DMA straight from /
//    to the caller's pages, no CPU copy;
//  - pageable: two pinned staging buffers; the CPU copy of piece i+1 (split
//    over up to kCopyThreads host threads) overlaps the DMA of piece i.
// The decode runs on the device copy; the spans come back the same way.
static constexpr size_t kStage = 64ull << 20;
static constexpr unsigned kCopyThreads = 8;     // default (HG_HOST_COPY_THREADS overrides)
static constexpr unsigned kMaxCopyThreads = 32;

// True if `p` lies in page-locked host memory the DMA engines can address.
static bool rt_host_pinned(const void* p) {
    hipPointerAttribute_t a;
    const hipError_t e = hipPointerGetAttributes(&a, p);
    if (e != hipSuccess) {
        (void)hipGetLastError();  // pageable memory reports an error: not sticky for us
        return false;
    }
    return a.type == hipMemoryTypeHost;
}

static unsigned copy_threads() {
    unsigned t = kCopyThreads;
    t = (unsigned)std::max<int64_t>(1, hgk_knob("HG_HOST_COPY_THREADS", t));
    const unsigned hw = std::thread::hardware_concurrency();
    return std::max(1u, std::min({t, hw ? hw : 1u, kMaxCopyThreads}));
}

// memcpy split over host threads in 2 MiB-aligned slices (pageable <-> pinned).
static void rt_par_memcpy(void* dst, const void* src, size_t n) {
    const unsigned nt = copy_threads();
    const size_t grain = 2ull << 20;
    if (nt <= 1 || n < 2 * grain) {
        memcpy(dst, src, n);
        return;
    }
    const size_t slices = (n + grain - 1) / grain;
    const unsigned use = (unsigned)std::min<size_t>(nt, slices);
    const size_t per = (slices + use - 1) / use * grain;
    std::thread th[kMaxCopyThreads];
    unsigned started = 0;
    for (unsigned t = 1; t < use; ++t) {
        const size_t o = t * per;
        if (o >= n) break;
        const size_t m = std::min(per, n - o);
        th[started++] = std::thread([=] {
            memcpy(static_cast<char*>(dst) + o, static_cast<const char*>(src) + o, m);
        });
    }
    memcpy(dst, src, std::min(per, n));
    for (unsigned t = 0; t < started; ++t) th[t].join();
}

static int copy_direct(hg_ctx* c, void* dst, const void* src, size_t bytes, hipMemcpyKind kind) {
    for (size_t off = 0; off < bytes; off += kStage)
        if (hipMemcpyAsync(static_cast<char*>(dst) + off, static_cast<const char*>(src) + off,
                           std::min(kStage, bytes - off), kind, c->stream) != hipSuccess)
            return HG_HIP_FAIL;
    return hipStreamSynchronize(c->stream) == hipSuccess ? HG_OK : HG_HIP_FAIL;
}

static int rt_h2d_pipelined(hg_ctx* c, void* dst, const void* src, size_t bytes) {
    if (rt_host_pinned(src)) return copy_direct(c, dst, src, bytes, hipMemcpyHostToDevice);
    if (ensure_pin(c->h_stage[0], kStage) != HG_OK || ensure_pin(c->h_stage[1], kStage) != HG_OK)
        return HG_HIP_FAIL;
    hipEvent_t ev[2];
    hipEventCreateWithFlags(&ev[0], hipEventDisableTiming);
    hipEventCreateWithFlags(&ev[1], hipEventDisableTiming);
    bool used[2] = {false, false};
    int rc = HG_OK;
    for (size_t off = 0, i = 0; off < bytes; off += kStage, ++i) {
        const size_t n = std::min(kStage, bytes - off);
        const int b = (int)(i & 1);
        if (used[b] && hipEventSynchronize(ev[b]) != hipSuccess) { rc = HG_HIP_FAIL; break; }
        rt_par_memcpy(c->h_stage[b].p, static_cast<const char*>(src) + off, n);
        if (hipMemcpyAsync(static_cast<char*>(dst) + off, c->h_stage[b].p, n,
                           hipMemcpyHostToDevice, c->stream) != hipSuccess ||
            hipEventRecord(ev[b], c->stream) != hipSuccess) {
            rc = HG_HIP_FAIL;
            break;
        }
        used[b] = true;
    }
    hipStreamSynchronize(c->stream);
    hipEventDestroy(ev[0]);
    hipEventDestroy(ev[1]);
    return rc;
}

static int rt_d2h_pipelined(hg_ctx* c, void* dst, const void* src, size_t bytes) {
    if (rt_host_pinned(dst)) return copy_direct(c, dst, src, bytes, hipMemcpyDeviceToHost);
    if (ensure_pin(c->h_stage[0], kStage) != HG_OK || ensure_pin(c->h_stage[1], kStage) != HG_OK)
        return HG_HIP_FAIL;
    hipEvent_t ev[2];
    hipEventCreateWithFlags(&ev[0], hipEventDisableTiming);
    hipEventCreateWithFlags(&ev[1], hipEventDisableTiming);
    size_t pend_off[2] = {0, 0}, pend_n[2] = {0, 0};
    bool used[2] = {false, false};
    int rc = HG_OK;
    size_t i = 0;
    for (size_t off = 0; off < bytes; off += kStage, ++i) {
        const size_t n = std::min(kStage, bytes - off);
        const int b = (int)(i & 1);
        if (used[b]) {  // drain the previous use of this buffer
            if (hipEventSynchronize(ev[b]) != hipSuccess) { rc = HG_HIP_FAIL; break; }
            rt_par_memcpy(static_cast<char*>(dst) + pend_off[b], c->h_stage[b].p, pend_n[b]);
        }
        if (hipMemcpyAsync(c->h_stage[b].p, static_cast<const char*>(src) + off, n,
                           hipMemcpyDeviceToHost, c->stream) != hipSuccess ||
            hipEventRecord(ev[b], c->stream) != hipSuccess) {
            rc = HG_HIP_FAIL;
            break;
        }
        used[b] = true;
        pend_off[b] = off;
        pend_n[b] = n;
    }
    for (int k = 0; k < 2 && rc == HG_OK; ++k) {
        const int b = (int)((i + k) & 1);
        if (!used[b]) continue;
        if (hipEventSynchronize(ev[b]) != hipSuccess) { rc = HG_HIP_FAIL; break; }
        rt_par_memcpy(static_cast<char*>(dst) + pend_off[b], c->h_stage[b].p, pend_n[b]);
        used[b] = false;
    }
    hipStreamSynchronize(c->stream);
    hipEventDestroy(ev[0]);
    hipEventDestroy(ev[1]);
    return rc;
}

int hg_host_register(const void* h_ptr, uint64_t len) {
    if (!h_ptr || !len) return HG_ERR_INVALID_ARG;
    const hipError_t e = hipHostRegister(const_cast<void*>(h_ptr), len, hipHostRegisterDefault);
    if (e != hipSuccess) {
        (void)hipGetLastError();
        return HG_HIP_FAIL;
    }
    return HG_OK;
}

int hg_host_unregister(const void* h_ptr) {
    if (!h_ptr) return HG_ERR_INVALID_ARG;
    const hipError_t e = hipHostUnregister(const_cast<void*>(h_ptr));
    if (e != hipSuccess) {
        (void)hipGetLastError();
        return HG_HIP_FAIL;
    }
    return HG_OK;
}

int hg_host_is_pinned(const void* h_ptr) { return h_ptr && rt_host_pinned(h_ptr) ? 1 : 0; }

// Page-locked table and span buffers: the table goes up in chunks on one
// stream (each chunk carries 4 KiB of the next one, the bytes a range decode
// may read past its stop), chunk i is range-decoded on the context stream as
// soon as it has landed -- entered at the exit of chunk i-1, its spans written
// straight after chunk i-1's -- and its spans go down on a third stream while
// later chunks are still going up (PCIe is full duplex).  One host sync per
// chunk reads its exit and count.  HG_DEC_CHUNK_MB sets the chunk (default 128).
static int decode_host_overlapped(hg_ctx* c, const uint8_t* h_sst, uint64_t len, hg_span* h_spans,
                                  uint64_t cap, uint64_t* n_out, hg_err* err) {
    const uint64_t C = (uint64_t)std::max<int64_t>(1, hgk_knob("HG_DEC_CHUNK_MB", 128)) << 20;
    const uint64_t K = (len + C - 1) / C;
    int r = rt_ensure_aux(c, 2);
    if (r == HG_OK) r = ensure(c, c->d_in, len);
    if (r == HG_OK) r = ensure(c, c->d_out, (len / 16 + 2 * K + 2) * sizeof(hg_span));
    if (r == HG_OK) r = ensure(c, c->ws, hgk_decode_workspace_bytes(C));
    if (r != HG_OK) return r;
    hipStream_t up = c->aux[0], down = c->aux[1], cs = c->stream;
    std::vector<hipEvent_t> ev(2 * K, nullptr);
    for (auto& e : ev)
        if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) r = HG_HIP_FAIL;
    uint8_t* din = static_cast<uint8_t*>(c->d_in.p);
    hg_span* dsp = static_cast<hg_span*>(c->d_out.p);
    for (uint64_t i = 0; r == HG_OK && i < K; ++i) {
        const uint64_t b = i * C, hi = std::min(len, (i + 1) * C + 4096);
        if (hipMemcpyAsync(din + b, h_sst + b, hi - b, hipMemcpyHostToDevice, up) != hipSuccess ||
            hipEventRecord(ev[i], up) != hipSuccess)
            r = HG_HIP_FAIL;
    }
    uint64_t entry = 0, G = 0, errpos = 0;
    int32_t kind = HG_OK;
    for (uint64_t i = 0; r == HG_OK && i < K; ++i) {
        const uint64_t b = i * C, stop = std::min(len, (i + 1) * C);
        const uint64_t rlen = std::min(len, (i + 1) * C + 4096);
        if (hipStreamWaitEvent(cs, ev[i], 0) != hipSuccess) { r = HG_HIP_FAIL; break; }
        r = hgk_decode_range_launch(din, len, rlen, b, stop, entry, dsp + G, (stop - b) / 16 + 2,
                                    dres(c), c->ws.p, cs);
        if (r != HG_OK) break;
        if (hipMemcpyAsync(c->hres.p, dres(c), sizeof(hg_decode_result), hipMemcpyDeviceToHost,
                           cs) != hipSuccess ||
            hipStreamSynchronize(cs) != hipSuccess) {
            r = HG_HIP_FAIL;
            break;
        }
        const hg_decode_result res = *static_cast<hg_decode_result*>(c->hres.p);
        const uint64_t ncopy = G < cap ? std::min(res.n_records, cap - G) : 0;
        if (ncopy && (hipEventRecord(ev[K + i], cs) != hipSuccess ||
                      hipStreamWaitEvent(down, ev[K + i], 0) != hipSuccess ||
                      hipMemcpyAsync(h_spans + G, dsp + G, ncopy * sizeof(hg_span),
                                     hipMemcpyDeviceToHost, down) != hipSuccess)) {
            r = HG_HIP_FAIL;
            break;
        }
        G += res.n_records;
        if (res.kind != HG_OK) {  // the reference stops at the first unreadable record
            kind = res.kind;
            errpos = res.err_offset;
            break;
        }
        entry = res.err_offset;  // the exit: the next chunk's entry
    }
    if (hipStreamSynchronize(down) != hipSuccess || hipStreamSynchronize(up) != hipSuccess)
        r = r == HG_OK ? HG_HIP_FAIL : r;
    for (auto e : ev)
        if (e) (void)hipEventDestroy(e);
    if (r != HG_OK) return r;
    if (n_out) *n_out = G;
    if (err) {
        err->kind = kind;
        err->reserved = 0;
        err->offset = kind != HG_OK ? errpos : 0;
    }
    if (kind != HG_OK) return kind;
    return G > cap ? HG_ERR_CAPACITY : HG_OK;
}

int hg_decode_host(hg_ctx* c, const uint8_t* h_sst, uint64_t len, hg_span* h_spans, uint64_t cap,
                   uint64_t* n_out, hg_err* err) {
    if (!c || (len && !h_sst) || (cap && !h_spans)) return HG_ERR_INVALID_ARG;
    if (len >= kMaxLen) return HG_ERR_TOO_LARGE;
    if (set_dev(c) != HG_OK) return HG_HIP_FAIL;
    {
        const uint64_t C = (uint64_t)std::max<int64_t>(1, hgk_knob("HG_DEC_CHUNK_MB", 128)) << 20;
        if (len >= 2 * C && !hgk_knob("HG_DECODE_HOST_SERIAL", 0) && rt_host_pinned(h_sst) &&
            (!cap || rt_host_pinned(h_spans)))
            return decode_host_overlapped(c, h_sst, len, h_spans, cap, n_out, err);
    }
    // A file of L bytes holds at most L/16 records.
    const uint64_t dcap = std::min<uint64_t>(cap, len / 16);
    int r;
    if ((r = ensure(c, c->d_in, len ? len : 1)) != HG_OK) return r;
    if ((r = ensure(c, c->d_out, (dcap ? dcap : 1) * sizeof(hg_span))) != HG_OK) return r;
    if (len && (r = rt_h2d_pipelined(c, c->d_in.p, h_sst, len)) != HG_OK) return r;
    uint64_t n = 0;
    hg_err e{};
    r = hg_decode_dev(c, static_cast<const uint8_t*>(c->d_in.p), len,
                      static_cast<hg_span*>(c->d_out.p), dcap, &n, &e);
    if (r != HG_OK && r != HG_ERR_CAPACITY && e.kind == HG_OK) return r;  // runtime failure
    const uint64_t ncopy = std::min(n, dcap);
    if (ncopy && rt_d2h_pipelined(c, h_spans, c->d_out.p, ncopy * sizeof(hg_span)) != HG_OK)
        return HG_HIP_FAIL;
    if (n_out) *n_out = n;
    if (err) *err = e;
    if (e.kind != HG_OK) return e.kind;
    return n > cap ? HG_ERR_CAPACITY : HG_OK;
}

// ---- range decode (a table split over devices, or decoded in chunks) ----------
int hg_decode_range_dev_async(hg_ctx* c, const uint8_t* d_sst, uint64_t len, uint64_t begin,
                              uint64_t stop, uint64_t entry, hg_span* d_spans, uint64_t cap,
                              hg_decode_result* d_result) {
    if (!c || !d_result || (len && !d_sst) || (cap && !d_spans)) return HG_ERR_INVALID_ARG;
    if (len >= kMaxLen) return HG_ERR_TOO_LARGE;
    if (stop > len) stop = len;
    if (begin > entry || begin > len || entry > len) return HG_ERR_INVALID_ARG;
    if (set_dev(c) != HG_OK) return HG_HIP_FAIL;
    if (capturing(c->stream)) return HG_ERR_INVALID_ARG;
    const uint64_t span = stop > begin ? stop - begin : 0;
    int r = ensure(c, c->ws, hgk_decode_workspace_bytes(span ? span : 1));
    if (r != HG_OK) return r;
    return hgk_decode_range_launch(d_sst, len, std::min(len, stop + 16), begin, stop, entry,
                                   d_spans, cap, d_result, c->ws.p, c->stream);
}

int hg_decode_range_dev(hg_ctx* c, const uint8_t* d_sst, uint64_t len, uint64_t begin,
                        uint64_t stop, uint64_t entry, hg_span* d_spans, uint64_t cap,
                        uint64_t* n_out, uint64_t* exit, hg_err* err) {
    int r = hg_decode_range_dev_async(c, d_sst, len, begin, stop, entry, d_spans, cap,
                                      c ? dres(c) : nullptr);
    if (r != HG_OK) return r;
    if (hipMemcpyAsync(c->hres.p, dres(c), sizeof(hg_decode_result), hipMemcpyDeviceToHost,
                       c->stream) != hipSuccess ||
        hipStreamSynchronize(c->stream) != hipSuccess)
        return HG_HIP_FAIL;
    const hg_decode_result res = *reinterpret_cast<hg_decode_result*>(c->hres.p);
    if (exit) *exit = res.kind == HG_OK ? res.err_offset : 0;
    hg_decode_result rr = res;
    if (res.kind == HG_OK) rr.err_offset = 0;
    return finish_decode(rr, cap, n_out, err);
}

int hg_decode_guess_entry_dev(hg_ctx* c, const uint8_t* d_sst, uint64_t len, uint64_t stop,
                              uint64_t* entry) {
    if (!c || !entry || (len && !d_sst)) return HG_ERR_INVALID_ARG;
    if (len >= kMaxLen) return HG_ERR_TOO_LARGE;
    if (set_dev(c) != HG_OK) return HG_HIP_FAIL;
    if (stop >= len) {  // the exit of a range reaching the table's end is its length
        *entry = len;
        return HG_OK;
    }
    int r = ensure(c, c->ws, hgk_decode_workspace_bytes(16384));
    if (r == HG_OK) r = ensure(c, c->x_res, 64);
    if (r != HG_OK) return r;
    uint64_t* d_out = static_cast<uint64_t*>(c->x_res.p);
    r = hgk_decode_guess_launch(d_sst, len, std::min(len, stop + 16), stop, d_out, c->ws.p,
                                c->stream);
    if (r != HG_OK) return r;
    if (hipMemcpyAsync(c->hres.p, d_out, 8, hipMemcpyDeviceToHost, c->stream) != hipSuccess ||
        hipStreamSynchronize(c->stream) != hipSuccess)
        return HG_HIP_FAIL;
    *entry = *static_cast<uint64_t*>(c->hres.p);
    return HG_OK;
}

// ---- encoded size --------------------------------------------------------------
int hg_encoded_size(hg_ctx* c, const hg_pair* pairs, uint64_t n, uint64_t* bytes) {
    if (!c || !bytes || (n && !pairs)) return HG_ERR_INVALID_ARG;
    *bytes = 0;
    if (n == 0) return HG_OK;
    hipPointerAttribute_t at;
    const hipError_t e = hipPointerGetAttributes(&at, pairs);
    if (e != hipSuccess) (void)hipGetLastError();
    if (e != hipSuccess || at.type != hipMemoryTypeDevice) {  // host pairs: sum here
        uint64_t t = 0;
        for (uint64_t i = 0; i < n; ++i) t += 16ull + pairs[i].klen + pairs[i].vlen;
        *bytes = t;
        return HG_OK;
    }
    if (set_dev(c) != HG_OK) return HG_HIP_FAIL;
    int r = ensure(c, c->ws, hgk_encode_workspace_bytes(n));
    if (r != HG_OK) return r;
    r = hgk_encode_size_launch(pairs, n, eres(c), reinterpret_cast<unsigned long long*>(c->ws.p),
                               c->stream);
    if (r != HG_OK) return r;
    if (hipMemcpyAsync(c->hres.p, eres(c), sizeof(hg_encode_result), hipMemcpyDeviceToHost,
                       c->stream) != hipSuccess ||
        hipStreamSynchronize(c->stream) != hipSuccess)
        return HG_HIP_FAIL;
    *bytes = reinterpret_cast<hg_encode_result*>(c->hres.p)->out_len;
    return HG_OK;
}

// ---- encode ------------------------------------------------------------------
static int encode_dev_async_ex(hg_ctx* c, const uint8_t* d_arena, const hg_pair* d_pairs,
                               uint64_t n, uint8_t* d_out, uint64_t cap, uint64_t* d_rec_off,
                               uint32_t block_stride, hg_block* d_blocks,
                               hg_encode_result* d_result, bool gather) {
    if (!c || !d_result || (n && !d_pairs) || (cap && !d_out)) return HG_ERR_INVALID_ARG;
    if (d_blocks && block_stride == 0) return HG_ERR_INVALID_ARG;  // slice::chunks(0) panics
    if (set_dev(c) != HG_OK) return HG_HIP_FAIL;
    if (capturing(c->stream)) return HG_ERR_INVALID_ARG;
    if (n == 0)
        return hipMemsetAsync(d_result, 0, sizeof(hg_encode_result), c->stream) == hipSuccess
                   ? HG_OK
                   : HG_HIP_FAIL;
    int r = ensure(c, c->ws, hgk_encode_workspace_bytes(n));
    if (r != HG_OK) return r;
    if (d_blocks && !d_rec_off) {
        if ((r = ensure(c, c->recoff, n * sizeof(uint64_t))) != HG_OK) return r;
        d_rec_off = static_cast<uint64_t*>(c->recoff.p);
    }
    if (gather)
        return hgk_encode_launch_ex(d_arena, d_pairs, n, nullptr, gather, d_out, cap, d_rec_off, 0,
                                    block_stride, d_blocks, d_result,
                                    reinterpret_cast<unsigned long long*>(c->ws.p), c->stream);
    // group sums double-buffered: this call's were cleared by the previous
    // call's bases kernel when they are big enough (no memset launch)
    uint64_t first = 0, ng = 0;
    hgk_encode_group_sums(n, &first, &ng);
    const uint64_t need = 2 * ((ng * 8 + 255) & ~(uint64_t)255);
    if (c->egs.bytes < need) {
        c->egs_clean[0] = c->egs_clean[1] = 0;
        if ((r = ensure(c, c->egs, need)) != HG_OK) return r;
    }
    const uint64_t half = c->egs.bytes / 2 & ~(uint64_t)255;
    char* base = static_cast<char*>(c->egs.p);
    const int cur = c->egs_cur;
    uint64_t zeroed = 0;
    r = hgk_encode_launch_ctl(d_arena, d_pairs, n, d_out, cap, d_rec_off, block_stride, d_blocks,
                              d_result, reinterpret_cast<unsigned long long*>(c->ws.p),
                              reinterpret_cast<uint64_t*>(base + cur * half), c->egs_clean[cur],
                              reinterpret_cast<uint64_t*>(base + (1 - cur) * half), half / 8,
                              &zeroed, c->stream);
    c->egs_clean[cur] = 0;
    c->egs_clean[1 - cur] = r == HG_OK ? zeroed : 0;
    c->egs_cur = 1 - cur;
    return r;
}

int hg_encode_dev_async(hg_ctx* c, const uint8_t* d_arena, const hg_pair* d_pairs, uint64_t n,
                        uint8_t* d_out, uint64_t cap, uint64_t* d_rec_off, uint32_t block_stride,
                        hg_block* d_blocks, hg_encode_result* d_result) {
    return encode_dev_async_ex(c, d_arena, d_pairs, n, d_out, cap, d_rec_off, block_stride,
                               d_blocks, d_result, false);
}

}  // extern "C"

namespace hgi {
// hg_encode_dev; gather: the pairs are a merge's output (records of several
// tables in key order), read with the default cache policy.
int rt_encode_dev(hg_ctx* c, const uint8_t* d_arena, const hg_pair* d_pairs, uint64_t n,
                  uint8_t* d_out, uint64_t cap, uint64_t* d_rec_off, uint32_t block_stride,
                  hg_block* d_blocks, uint64_t* out_len, bool gather) {
    int r = encode_dev_async_ex(c, d_arena, d_pairs, n, d_out, cap, d_rec_off, block_stride,
                                d_blocks, c ? eres(c) : nullptr, gather);
    if (r != HG_OK) return r;
    if (hipMemcpyAsync(c->hres.p, eres(c), sizeof(hg_encode_result), hipMemcpyDeviceToHost,
                       c->stream) != hipSuccess ||
        hipStreamSynchronize(c->stream) != hipSuccess)
        return HG_HIP_FAIL;
    const hg_encode_result res = *reinterpret_cast<hg_encode_result*>(c->hres.p);
    if (out_len) *out_len = res.out_len;
    return res.kind;
}
}  // namespace hgi

extern "C" {

int hg_encode_dev(hg_ctx* c, const uint8_t* d_arena, const hg_pair* d_pairs, uint64_t n,
                  uint8_t* d_out, uint64_t cap, uint64_t* d_rec_off, uint32_t block_stride,
                  hg_block* d_blocks, uint64_t* out_len) {
    return hgi::rt_encode_dev(c, d_arena, d_pairs, n, d_out, cap, d_rec_off, block_stride,
                              d_blocks, out_len, false);
}

// Host encode with page-locked buffers, in chunks of ~256 MiB of output: the
// arena goes up in order only as far as the next chunk's sources reach
// (running max of the source ends), each chunk is encoded as soon as its
// bytes and pairs are up, and its output comes back on a second stream while
// the next chunk's input goes up (PCIe is full duplex).  For a memtable arena
// in pair order (a flush) upload and download overlap almost completely;
// scattered sources make the first chunk wait for most of the arena, which
// degrades gracefully to upload-then-download.  Record offsets are written
// global (rec_base = the chunk's output offset); block entries are built once
// at the end from them.
static int encode_host_overlapped(hg_ctx* c, const uint8_t* h_arena, uint64_t arena_len,
                                  const hg_pair* h_pairs, uint64_t n, uint8_t* h_out,
                                  uint64_t total, uint64_t* h_rec_off, uint32_t block_stride,
                                  hg_block* h_blocks) {
    // Chunk size: measured on MI355X with cfg 3 from pinned memory (tools/host_encode.py):
    // 64 MiB 183 ms, 128 MiB 142 ms, 192-256 MiB 76 ms, 512 MiB 82 ms, one
    // upload-then-download pass 118 ms (smaller copies behind cross-stream
    // waits fall off a cliff).  HG_ENC_CHUNK_MB overrides.
    const uint64_t kChunkOut = (uint64_t)std::max<int64_t>(1, hgk_knob("HG_ENC_CHUNK_MB", 256)) << 20;
    const bool tm = hgk_knob("HG_HOST_TIMING", 0) != 0;
    auto now = [] { return std::chrono::duration<double, std::milli>(
                        std::chrono::steady_clock::now().time_since_epoch()).count(); };
    const double t_start = now();
    int r = rt_ensure_aux(c, 1);
    if (r != HG_OK) return r;
    hipStream_t up = c->stream, down = c->aux[0];
    const size_t pairs_at = (arena_len + 63) & ~(size_t)63;
    const size_t in_bytes = pairs_at + n * sizeof(hg_pair);
    const uint64_t nb = h_blocks ? hg_block_count(n, block_stride) : 0;
    const bool want_rec = h_rec_off || h_blocks;
    if ((r = ensure(c, c->d_in, in_bytes)) != HG_OK) return r;
    if ((r = ensure(c, c->d_out, total)) != HG_OK) return r;
    if ((r = ensure(c, c->d_aux, n * sizeof(uint64_t) + nb * sizeof(hg_block) + 64)) != HG_OK)
        return r;
    if ((r = ensure(c, c->ws, hgk_encode_workspace_bytes(n))) != HG_OK) return r;
    char* din = static_cast<char*>(c->d_in.p);
    const uint8_t* darena = reinterpret_cast<const uint8_t*>(din);
    hg_pair* dpairs = reinterpret_cast<hg_pair*>(din + pairs_at);
    uint8_t* dout = static_cast<uint8_t*>(c->d_out.p);
    uint64_t* drec = static_cast<uint64_t*>(c->d_aux.p);
    hg_block* dblk =
        reinterpret_cast<hg_block*>(static_cast<char*>(c->d_aux.p) + n * sizeof(uint64_t));
    unsigned long long* ws = reinterpret_cast<unsigned long long*>(c->ws.p);
    std::vector<hipEvent_t> evs;
    uint64_t up_arena = 0, p_lo = 0, base = 0, srcmax = 0;
    while (r == HG_OK && p_lo < n) {
        uint64_t p_hi = p_lo, bytes = 0;
        while (p_hi < n && (bytes < kChunkOut || p_hi == p_lo)) {
            const hg_pair& q = h_pairs[p_hi];
            bytes += 16ull + q.klen + q.vlen;
            if (q.klen) srcmax = std::max(srcmax, q.key_off + q.klen);
            if (q.vlen) srcmax = std::max(srcmax, q.val_off + q.vlen);
            ++p_hi;
        }
        const uint64_t need = std::min(srcmax, arena_len);
        if (need > up_arena) {
            if (hipMemcpyAsync(din + up_arena, h_arena + up_arena, need - up_arena,
                               hipMemcpyHostToDevice, up) != hipSuccess)
                r = HG_HIP_FAIL;
            up_arena = need;
        }
        if (r == HG_OK && hipMemcpyAsync(dpairs + p_lo, h_pairs + p_lo,
                                         (p_hi - p_lo) * sizeof(hg_pair), hipMemcpyHostToDevice,
                                         up) != hipSuccess)
            r = HG_HIP_FAIL;
        if (r == HG_OK)
            r = hgk_encode_launch_at(darena, dpairs + p_lo, p_hi - p_lo, dout + base, bytes,
                                     want_rec ? drec + p_lo : nullptr, base, 0, nullptr, eres(c),
                                     ws, up);
        hipEvent_t ev = nullptr;
        if (r == HG_OK && (hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess ||
                           hipEventRecord(ev, up) != hipSuccess ||
                           hipStreamWaitEvent(down, ev, 0) != hipSuccess ||
                           hipMemcpyAsync(h_out + base, dout + base, bytes, hipMemcpyDeviceToHost,
                                          down) != hipSuccess))
            r = HG_HIP_FAIL;
        if (ev) evs.push_back(ev);
        base += bytes;
        p_lo = p_hi;
    }
    if (r == HG_OK && h_blocks)
        r = hgk_encode_blocks_launch(drec, n, block_stride, total, dblk, up);
    const double t_issued = now();
    if (hipStreamSynchronize(up) != hipSuccess || hipStreamSynchronize(down) != hipSuccess)
        r = r == HG_OK ? HG_HIP_FAIL : r;
    if (tm)
        fprintf(stderr, "[hg] encode_host_overlapped: issue %.2f ms, wait %.2f ms, %zu chunks\n",
                t_issued - t_start, now() - t_issued, evs.size());
    for (hipEvent_t e : evs) (void)hipEventDestroy(e);
    if (r == HG_OK && h_rec_off) r = rt_d2h_pipelined(c, h_rec_off, drec, n * sizeof(uint64_t));
    if (r == HG_OK && h_blocks && nb) r = rt_d2h_pipelined(c, h_blocks, dblk, nb * sizeof(hg_block));
    return r;
}

int hg_encode_host(hg_ctx* c, const uint8_t* h_arena, uint64_t arena_len, const hg_pair* h_pairs,
                   uint64_t n, uint8_t* h_out, uint64_t cap, uint64_t* h_rec_off,
                   uint32_t block_stride, hg_block* h_blocks, uint64_t* out_len) {
    if (!c || (n && !h_pairs) || (arena_len && !h_arena) || (cap && !h_out))
        return HG_ERR_INVALID_ARG;
    if (h_blocks && block_stride == 0) return HG_ERR_INVALID_ARG;
    if (set_dev(c) != HG_OK) return HG_HIP_FAIL;
    uint64_t total = 0;
    for (uint64_t i = 0; i < n; ++i) total += 16ull + h_pairs[i].klen + h_pairs[i].vlen;
    if (out_len) *out_len = total;
    if (total > cap) return HG_ERR_CAPACITY;
    if (n && total && arena_len && !hgk_knob("HG_ENCODE_HOST_SERIAL", 0) &&
        rt_host_pinned(h_arena) && rt_host_pinned(h_pairs) && rt_host_pinned(h_out))
        return encode_host_overlapped(c, h_arena, arena_len, h_pairs, n, h_out, total, h_rec_off,
                                      block_stride, h_blocks);
    const uint64_t nb = h_blocks ? hg_block_count(n, block_stride) : 0;
    // d_in: arena ++ pairs; d_out: encoded bytes; d_aux: rec_off ++ blocks
    const size_t pairs_at = (arena_len + 63) & ~(size_t)63;
    const size_t in_bytes = pairs_at + n * sizeof(hg_pair);
    const size_t blocks_at = n * sizeof(uint64_t);
    int r;
    if ((r = ensure(c, c->d_in, in_bytes ? in_bytes : 1)) != HG_OK) return r;
    if ((r = ensure(c, c->d_out, total ? total : 1)) != HG_OK) return r;
    if ((r = ensure(c, c->d_aux, blocks_at + nb * sizeof(hg_block) + 64)) != HG_OK) return r;
    char* din = static_cast<char*>(c->d_in.p);
    if (arena_len && (r = rt_h2d_pipelined(c, din, h_arena, arena_len)) != HG_OK) return r;
    if (n && (r = rt_h2d_pipelined(c, din + pairs_at, h_pairs, n * sizeof(hg_pair))) != HG_OK)
        return r;
    uint64_t* d_rec = static_cast<uint64_t*>(c->d_aux.p);
    hg_block* d_blk = h_blocks ? reinterpret_cast<hg_block*>(static_cast<char*>(c->d_aux.p) + blocks_at)
                               : nullptr;
    uint64_t got = 0;
    r = hg_encode_dev(c, reinterpret_cast<const uint8_t*>(din),
                      reinterpret_cast<const hg_pair*>(din + pairs_at), n,
                      static_cast<uint8_t*>(c->d_out.p), total, d_rec, block_stride, d_blk, &got);
    if (r != HG_OK) return r;
    if (total && (r = rt_d2h_pipelined(c, h_out, c->d_out.p, total)) != HG_OK) return r;
    if (h_rec_off && n && (r = rt_d2h_pipelined(c, h_rec_off, d_rec, n * sizeof(uint64_t))) != HG_OK)
        return r;
    if (h_blocks && nb && (r = rt_d2h_pipelined(c, h_blocks, d_blk, nb * sizeof(hg_block))) != HG_OK)
        return r;
    return HG_OK;
}

// ---- merge (compaction) ------------------------------------------------------------
}  // extern "C"

namespace {
// hg_merge_dev_async with the choice of what happens on input that is not
// strictly increasing: defer = 0 runs the serial reference loop on the device
// (the async API's contract); defer = 1 leaves HG_ERR_UNSORTED for
// merge_epochs (the synchronous paths).
int merge_async(hg_ctx* c, uint32_t ntables, const uint8_t* d_arena, uint64_t arena_len,
                const uint64_t* table_off, const hg_span* const* d_spans, const uint64_t* counts,
                hg_pair* d_out, uint64_t cap, hg_merge_result* d_result, int defer,
                const uint64_t* kp = nullptr, uint32_t kp_tag = 0,
                const unsigned long long* d_err_pre = nullptr,
                const hgk_merge_records* rec = nullptr, int* done = nullptr) {
    if (done) *done = 0;
    if (!c || !d_result || (ntables && (!table_off || !d_spans || !counts)) || (cap && !d_out))
        return HG_ERR_INVALID_ARG;
    if (set_dev(c) != HG_OK) return HG_HIP_FAIL;
    if (capturing(c->stream)) return HG_ERR_INVALID_ARG;
    if (!c->mstage_ev && hipEventCreateWithFlags(&c->mstage_ev, hipEventDisableTiming) != hipSuccess)
        return HG_HIP_FAIL;
    if (ntables == 0) {  // min_by_key over no candidates: the reference panics (:213)
        hg_merge_result r{0, HG_ERR_EMPTY_MERGE, 0, 0};
        if (ensure_pin(c->mstage, 4096) != HG_OK) return HG_HIP_FAIL;
        if (c->mstage_busy && hipEventSynchronize(c->mstage_ev) != hipSuccess) return HG_HIP_FAIL;
        memcpy(c->mstage.p, &r, sizeof r);
        if (hipMemcpyAsync(d_result, c->mstage.p, sizeof r, hipMemcpyHostToDevice, c->stream) !=
            hipSuccess)
            return HG_HIP_FAIL;
    } else {
        uint64_t n = 0;
        for (uint32_t t = 0; t < ntables; ++t) {
            if (counts[t] && !d_spans[t]) return HG_ERR_INVALID_ARG;
            n += counts[t];
        }
        int r = ensure(c, c->mws, hgk_merge_workspace_bytes(ntables, n) + 4096);
        if (r != HG_OK) return r;
        // the previous call's argument copy must have left the pinned staging
        if (c->mstage_busy && hipEventSynchronize(c->mstage_ev) != hipSuccess) return HG_HIP_FAIL;
        if (ensure_pin(c->mstage, hgk_merge_staging_bytes(ntables) + 4096) != HG_OK)
            return HG_HIP_FAIL;
        r = hgk_merge_launch(d_arena, arena_len, ntables, table_off, d_spans, counts, d_out, cap,
                             d_result, c->mws.p, c->mstage.p, c->stream, defer, kp, kp_tag, d_err_pre,
                             rec, done);
        if (r != HG_OK) return r;
    }
    if (hipEventRecord(c->mstage_ev, c->stream) != hipSuccess) return HG_HIP_FAIL;
    c->mstage_busy = true;
    return HG_OK;
}

// After merge_async(defer) reported HG_ERR_UNSORTED (stream synchronized):
// the reference loop by epochs (hgk_merge_epochs) on the same workspace.
int merge_epochs(hg_ctx* c, uint32_t ntables, const uint8_t* d_arena, uint64_t arena_len,
                 const uint64_t* table_off, const hg_span* const* d_spans, const uint64_t* counts,
                 hg_pair* d_out, uint64_t cap, hg_merge_result* d_result, hg_merge_result* res) {
    if (c->mstage_busy && hipEventSynchronize(c->mstage_ev) != hipSuccess) return HG_HIP_FAIL;
    c->mstage_busy = false;
    return hgk_merge_epochs(d_arena, arena_len, ntables, table_off, d_spans, counts, d_out, cap,
                            d_result, res, c->mws.p, c->mstage.p, c->stream);
}
}  // namespace

extern "C" {

int hg_merge_dev_async(hg_ctx* c, uint32_t ntables, const uint8_t* d_arena, uint64_t arena_len,
                       const uint64_t* table_off, const hg_span* const* d_spans,
                       const uint64_t* counts, hg_pair* d_out, uint64_t cap,
                       hg_merge_result* d_result) {
    return merge_async(c, ntables, d_arena, arena_len, table_off, d_spans, counts, d_out, cap,
                       d_result, 0);
}

int hg_merge_dev(hg_ctx* c, uint32_t ntables, const uint8_t* d_arena, uint64_t arena_len,
                 const uint64_t* table_off, const hg_span* const* d_spans, const uint64_t* counts,
                 hg_pair* d_out, uint64_t cap, hg_merge_result* result) {
    if (!c) return HG_ERR_INVALID_ARG;
    if (ensure(c, c->mres, 64) != HG_OK) return HG_HIP_FAIL;
    hg_merge_result* dres_m = static_cast<hg_merge_result*>(c->mres.p);
    int r = merge_async(c, ntables, d_arena, arena_len, table_off, d_spans, counts, d_out, cap,
                        dres_m, 1);
    if (r != HG_OK) return r;
    if (hipMemcpyAsync(c->hres.p, dres_m, sizeof(hg_merge_result), hipMemcpyDeviceToHost,
                       c->stream) != hipSuccess ||
        hipStreamSynchronize(c->stream) != hipSuccess)
        return HG_HIP_FAIL;
    hg_merge_result res = *static_cast<hg_merge_result*>(c->hres.p);
    if (res.kind == HG_ERR_UNSORTED &&
        (r = merge_epochs(c, ntables, d_arena, arena_len, table_off, d_spans, counts, d_out, cap,
                          dres_m, &res)) != HG_OK)
        return r;
    if (result) *result = res;
    if (res.kind != HG_OK) return res.kind;
    return res.n_out > cap ? HG_ERR_CAPACITY : HG_OK;
}

// Decode -> merge -> encode of tables already in one device arena.  One host
// sync for the record counts (the merge's launch geometry needs them); the
// encode reads the merge's output count on the device (grids sized for the
// input count), so merge and encode run back to back; one sync at the end for
// the results.  *enc = encoded bytes (0 unless the merge succeeded).
static int compact_core(hg_ctx* c, uint32_t ntables, const uint8_t* arena, uint64_t arena_len,
                        const uint64_t* toff, const uint64_t* lens, uint8_t* d_out, uint64_t cap,
                        uint64_t* enc, uint32_t block_stride, hg_block* d_blk,
                        hg_merge_result* res) {
    *enc = 0;
    *res = hg_merge_result{0, HG_OK, 0, 0};
    uint64_t span_cap = 0;
    for (uint32_t t = 0; t < ntables; ++t) {
        if (lens[t] >= kMaxLen) return HG_ERR_TOO_LARGE;
        if (toff[t] > arena_len || lens[t] > arena_len - toff[t]) return HG_ERR_INVALID_ARG;
        span_cap += lens[t] / 16;
    }
    std::vector<const uint8_t*> dt(ntables);
    std::vector<hg_span*> ds(ntables);
    std::vector<const hg_span*> sp(ntables);
    std::vector<uint64_t> caps(ntables), counts(ntables, 0);
    std::vector<hg_decode_result> hr(ntables);
    int r = ensure(c, c->mspans, (span_cap ? span_cap : 1) * sizeof(hg_span));
    // d_aux: the decode results, then (hgk_merge_prebuild) the run offsets and
    // an order-check word -- sized once here, so it never moves under them
    const size_t rbytes = ntables * sizeof(hg_decode_result);
    const size_t roff_at = (rbytes + 64 + 255) & ~(size_t)255;
    if (r == HG_OK) r = ensure(c, c->d_aux, roff_at + (ntables + 2) * sizeof(uint64_t) + 64);
    if (r != HG_OK) return r;
    hg_span* spans = static_cast<hg_span*>(c->mspans.p);
    for (uint32_t t = 0; t < ntables; ++t) {
        dt[t] = arena + toff[t];
        ds[t] = spans;
        sp[t] = spans;
        caps[t] = lens[t] / 16;
        spans += caps[t];
    }
    // 1. one batched decode chain for all tables, one sync for the counts; in
    //    compaction mode its stride pieces leave key prefixes for the merge
    //    entries (kp: per table the decode workspace's scratch, piece records
    //    and piece tags) -- the entry builder then reads spans, not key lines
    std::vector<uint64_t> kp;
    uint32_t kp_tag = 0;
    const unsigned long long* prebuilt_err = nullptr;  // the entries are built (hgk_merge_prebuild)
    const bool use_kp = hgk_knob("HG_COMPACT_KPRE", 1) != 0 && hgk_knob("HG_DECODE_BATCH", 0) != 1;
    // Merge entries built before the host has the record counts (below) need
    // a merge workspace for every record the tables could hold (lens / 16):
    // taken only when that bound is modest -- the workspace already has it,
    // or it fits 1/16 of the free device memory (at most 16 GiB) -- and
    // sized here, before the decode is queued, so that growing it (a stream
    // sync) does not sit between the decode and the entry builder.  If the
    // allocation fails the merge simply builds its entries after the counts.
    bool prebuild = false;
    if (use_kp && ntables && hgk_knob("HG_COMPACT_PREBUILD", 1) != 0 &&
        hgk_knob("HG_MERGE_KENT", 1) != 0 && span_cap < (1ull << 31)) {
        const uint64_t ws_ub = hgk_merge_workspace_bytes(ntables, span_cap) + 4096;
        if (c->mws.bytes >= ws_ub) {
            prebuild = true;
        } else if (ws_ub <= (16ull << 30)) {
            size_t fr = 0, tot = 0;
            if (hipMemGetInfo(&fr, &tot) == hipSuccess && ws_ub <= fr / 16) prebuild = try_grow(c, c->mws, ws_ub);
            else (void)hipGetLastError();
        }
    }
    if (ntables) {
        hg_decode_result* dr = static_cast<hg_decode_result*>(c->d_aux.p);
        if (use_kp) {
            if (++c->kpre_calls == 0) ++c->kpre_calls;  // 0 means "off"
            kp_tag = c->kpre_calls;
            std::vector<uint64_t> wso;
            r = batch_one_launch(c, ntables, dt.data(), lens, ds.data(), caps.data(), dr, kp_tag,
                                 &wso);
            if (r == HG_OK) {
                kp.resize(3 * (size_t)ntables + 2);
                for (uint32_t t = 0; t < ntables; ++t) {
                    uint64_t so, po, to;
                    hgk_decode_ws_layout(lens[t], &so, &po, &to);
                    const uint64_t b = reinterpret_cast<uint64_t>(c->bws.p) + wso[t];
                    kp[t] = b + so;
                    kp[ntables + t] = b + po;
                    kp[2 * (size_t)ntables + t] = b + to;
                }
                // the decode's device staging (its DecodeArgs and pre-pass grid)
                // for the per-batch entry builder (hgk_decode_entries_launch)
                kp[3 * (size_t)ntables] = reinterpret_cast<uint64_t>(c->bstage_last);
                kp[3 * (size_t)ntables + 1] = hgk_decode_multi_geometry(c->bstage.p, ntables);
            }
        } else {
            r = hg_decode_batch_dev_async(c, ntables, dt.data(), lens, ds.data(), caps.data(), dr);
        }
        if (r != HG_OK) return r;
        // The counts come back through a pinned copy and an event; meanwhile
        // (compaction mode, a merge workspace for every possible record of
        // at most 16 GiB) the merge entries are built on the device from the
        // device-side counts, so the host round trip overlaps the entry
        // builder instead of sitting between the kernels (HG_COMPACT_PREBUILD=0:
        // after it, as before).
        // With the prebuild the copy goes on an auxiliary stream forked
        // after the decode: the entry builder then follows the decode on the
        // context stream directly (a copy and a launch gap fewer, ~10 us).
        const bool side = prebuild && rt_ensure_aux(c, 1) == HG_OK;
        hipStream_t cs = side ? c->aux[0] : c->stream;
        if (ensure_pin(c->kres, rbytes + 64) != HG_OK ||
            (!c->kres_ev && hipEventCreateWithFlags(&c->kres_ev, hipEventDisableTiming) != hipSuccess) ||
            (side && (hipEventRecord(c->fork_ev, c->stream) != hipSuccess ||
                      hipStreamWaitEvent(cs, c->fork_ev, 0) != hipSuccess)) ||
            hipMemcpyAsync(c->kres.p, dr, rbytes, hipMemcpyDeviceToHost, cs) != hipSuccess ||
            hipEventRecord(c->kres_ev, cs) != hipSuccess)
            return HG_HIP_FAIL;
        // (kp[3 ntables + 1]: the pre-pass grid -- with none the entry
        // builder would launch nothing and the merge must build them itself)
        if (prebuild && !kp.empty() && kp[3 * (size_t)ntables + 1] != 0) {
            uint64_t* d_roff = reinterpret_cast<uint64_t*>(static_cast<char*>(c->d_aux.p) + roff_at);
            unsigned long long* d_perr = reinterpret_cast<unsigned long long*>(d_roff + ntables + 1);
            if ((r = hgk_merge_prebuild(kp.data(), ntables, dr, d_roff, d_perr, c->mws.p, c->stream)) !=
                HG_OK)
                return r;
            prebuilt_err = d_perr;
        }
        if (hipEventSynchronize(c->kres_ev) != hipSuccess) return HG_HIP_FAIL;
        memcpy(hr.data(), c->kres.p, rbytes);
        for (uint32_t t = 0; t < ntables; ++t) {
            if (hr[t].kind != HG_OK) {  // the reference's read_all unwrap (storage.rs:64-66)
                *res = hg_merge_result{0, hr[t].kind, t, hr[t].err_offset};
                return hr[t].kind;
            }
            counts[t] = hr[t].n_records;
        }
    }
    // 2. merge -> pairs; 3. encode (+ blocks) of the merge's device count
    uint64_t nm = 0;
    for (uint32_t t = 0; t < ntables; ++t) nm += counts[t];
    r = ensure(c, c->mpairs, (nm ? nm : 1) * sizeof(hg_pair));
    if (r == HG_OK) r = ensure(c, c->mres, 128);
    if (r == HG_OK) r = ensure(c, c->ws, hgk_encode_workspace_bytes(nm ? nm : 1));
    if (r == HG_OK && d_blk) r = ensure(c, c->recoff, (nm ? nm : 1) * sizeof(uint64_t));
    if (r != HG_OK) return r;
    hg_merge_result* dres_m = static_cast<hg_merge_result*>(c->mres.p);
    hg_encode_result* dres_e =
        reinterpret_cast<hg_encode_result*>(static_cast<char*>(c->mres.p) + 64);
    hg_pair* pairs = static_cast<hg_pair*>(c->mpairs.p);
    // tables that are not strictly increasing: the merge reports HG_ERR_UNSORTED
    // with no output (the encode then writes nothing) and the epochs below run
    // the reference loop; otherwise merge and encode run back to back
    // records mode (knob HG_COMPACT_RECORDS 1): the merge's last round writes
    // the live records' bytes itself (look-back over record and byte
    // counts) -- no hg_pair array, no encode pass; the encode below runs
    // whenever the merge did not take that path.  Off by default: measured
    // slower (same box, alternating; cfg 5 legs 8 x 1 M 1.201-1.209 ms with
    // pairs + encode vs 1.226-1.231, 8 x 1 GiB 8.95-9.01 vs 9.02-9.05 ms;
    // profiles/r5_ab_compact_records.log): the fused round's gather runs at 5
    // waves/SIMD behind a look-back per tile, the record gather at 8.
    const bool enc_records = hgk_knob("HG_COMPACT_ENCODE", 0) != 1;
    const bool rec_mode = hgk_knob("HG_COMPACT_RECORDS", 0) == 1 && enc_records;
    // the records encode's group sums are cleared by the merge's flag kernel
    // (c->ws holds them: sized for the encode of nm pairs above)
    uint64_t gs_first = 0, gs_words = 0;
    hgk_encode_group_sums(nm, &gs_first, &gs_words);
    // (pairs mode: the merge's last round also accumulates the records
    // encode's tile sums, c->ws [0, gs_first), and group sums after them)
    uint32_t tl2 = 0, gl2 = 0;
    hgk_encode_tile_geometry(&tl2, &gl2);
    const bool merge_sums = enc_records && !rec_mode && nm && hgk_knob("HG_COMPACT_MERGE_SUMS", 1) != 0;
    hgk_merge_records rec{rec_mode ? d_out : nullptr,
                          cap,
                          d_blk ? static_cast<uint64_t*>(c->recoff.p) : nullptr,
                          dres_e,
                          enc_records && nm ? static_cast<uint64_t*>(c->ws.p) + gs_first : nullptr,
                          gs_words,
                          merge_sums ? static_cast<uint64_t*>(c->ws.p) : nullptr,
                          gs_first,
                          gs_first + gs_words,
                          tl2,
                          gl2};
    int done = 0;
    r = merge_async(c, ntables, arena, arena_len, toff, sp.data(), counts.data(), pairs, nm, dres_m,
                    1, kp.empty() ? nullptr : kp.data(), kp_tag, prebuilt_err, &rec, &done);
    if (r != HG_OK) return r;
    const bool emitted = (done & HGK_MERGE_EMITTED) != 0;
    bool zeroed = (done & HGK_MERGE_ZEROED) != 0;  // for the first encode only
    bool sums = (done & HGK_MERGE_SUMS) != 0;      // (likewise)
    auto encode = [&]() -> int {
        if (nm == 0)
            return hipMemsetAsync(dres_e, 0, sizeof(hg_encode_result), c->stream) == hipSuccess
                       ? HG_OK
                       : HG_HIP_FAIL;
        // the merged pairs are whole records of the decoded tables: gathered as
        // records (HG_COMPACT_ENCODE=pairs: the general gather, for A/B runs)
        if (hgk_knob("HG_COMPACT_ENCODE", 0) == 1)
            return hgk_encode_launch_ex(arena, pairs, nm, &dres_m->n_out, true, d_out, cap,
                                        d_blk ? static_cast<uint64_t*>(c->recoff.p) : nullptr, 0,
                                        block_stride, d_blk, dres_e,
                                        reinterpret_cast<unsigned long long*>(c->ws.p), c->stream);
        return hgk_encode_launch_records(arena, arena_len, pairs, nm, &dres_m->n_out, d_out, cap,
                                         d_blk ? static_cast<uint64_t*>(c->recoff.p) : nullptr,
                                         block_stride, d_blk, dres_e,
                                         reinterpret_cast<unsigned long long*>(c->ws.p), c->stream,
                                         std::exchange(zeroed, false), std::exchange(sums, false));
    };
    if (!emitted) {
        if ((r = encode()) != HG_OK) return r;
    } else if (d_blk) {
        r = hgk_encode_blocks_launch_dev(static_cast<const uint64_t*>(c->recoff.p), nm, &dres_m->n_out,
                                         dres_e, block_stride, d_blk, c->stream);
        if (r != HG_OK) return r;
    }
    char* h = static_cast<char*>(c->hres.p);
    if (hipMemcpyAsync(h, c->mres.p, 128, hipMemcpyDeviceToHost, c->stream) != hipSuccess ||
        hipStreamSynchronize(c->stream) != hipSuccess)
        return HG_HIP_FAIL;
    *res = *reinterpret_cast<const hg_merge_result*>(h);
    if (res->kind == HG_ERR_UNSORTED) {
        hg_merge_result er2{};
        if ((r = merge_epochs(c, ntables, arena, arena_len, toff, sp.data(), counts.data(), pairs,
                              nm, dres_m, &er2)) != HG_OK ||
            (r = encode()) != HG_OK)
            return r;
        if (hipMemcpyAsync(h, c->mres.p, 128, hipMemcpyDeviceToHost, c->stream) != hipSuccess ||
            hipStreamSynchronize(c->stream) != hipSuccess)
            return HG_HIP_FAIL;
        *res = *reinterpret_cast<const hg_merge_result*>(h);
    }
    const hg_encode_result er = *reinterpret_cast<const hg_encode_result*>(h + 64);
    if (res->kind != HG_OK) return res->kind;
    if (res->n_out > nm) return HG_ERR_INTERNAL;  // the merge never grows the record count
    *enc = er.out_len;
    return er.kind;
}

int hg_compact_dev(hg_ctx* c, uint32_t ntables, const uint8_t* d_arena, uint64_t arena_len,
                   const uint64_t* table_off, const uint64_t* lens, uint8_t* d_out, uint64_t cap,
                   uint64_t* out_len, uint32_t block_stride, hg_block* d_blocks,
                   hg_merge_result* result) {
    if (!c || (ntables && (!d_arena || !table_off || !lens)) || (cap && !d_out))
        return HG_ERR_INVALID_ARG;
    if (d_blocks && block_stride == 0) return HG_ERR_INVALID_ARG;
    if (set_dev(c) != HG_OK) return HG_HIP_FAIL;
    if (out_len) *out_len = 0;
    uint64_t enc = 0;
    hg_merge_result res;
    const int r = compact_core(c, ntables, d_arena, arena_len, table_off, lens, d_out, cap, &enc,
                               block_stride, d_blocks, &res);
    if (out_len) *out_len = enc;
    if (result) *result = res;
    return r;
}

int hg_compact_host(hg_ctx* c, uint32_t ntables, const uint8_t* const* h_tables,
                    const uint64_t* lens, uint8_t* h_out, uint64_t cap, uint64_t* out_len,
                    uint32_t block_stride, hg_block* h_blocks, hg_merge_result* result) {
    if (!c || (ntables && (!h_tables || !lens)) || (cap && !h_out)) return HG_ERR_INVALID_ARG;
    if (h_blocks && block_stride == 0) return HG_ERR_INVALID_ARG;
    if (set_dev(c) != HG_OK) return HG_HIP_FAIL;
    hg_merge_result res{0, HG_OK, 0, 0};
    if (out_len) *out_len = 0;
    // 1. all tables into one device arena (8-byte aligned starts)
    uint64_t total = 0;
    std::vector<uint64_t> toff(ntables + 1);
    int r = HG_OK;
    for (uint32_t t = 0; r == HG_OK && t < ntables; ++t) {
        if (lens[t] && !h_tables[t]) r = HG_ERR_INVALID_ARG;
        if (lens[t] >= kMaxLen) r = HG_ERR_TOO_LARGE;
        toff[t] = total;
        total += (lens[t] + 7) & ~7ull;
    }
    if (r == HG_OK) r = ensure(c, c->d_in, total ? total : 1);
    if (r == HG_OK) r = ensure(c, c->d_out, total ? total : 1);  // output <= input bytes
    char* arena = static_cast<char*>(c->d_in.p);
    for (uint32_t t = 0; r == HG_OK && t < ntables; ++t)
        if (lens[t]) r = rt_h2d_pipelined(c, arena + toff[t], h_tables[t], lens[t]);
    // 2. decode, merge, encode on the device
    uint64_t enc = 0, nb = 0;
    hg_block* d_blk = nullptr;
    if (r == HG_OK && h_blocks) {
        uint64_t bound = 0;  // block entries: at most one per block_stride input records
        for (uint32_t t = 0; t < ntables; ++t) bound += lens[t] / 16;
        r = ensure(c, c->d_blk, (hg_block_count(bound, block_stride) + 1) * sizeof(hg_block));
        d_blk = static_cast<hg_block*>(c->d_blk.p);
    }
    if (r == HG_OK)
        r = compact_core(c, ntables, reinterpret_cast<const uint8_t*>(arena), total, toff.data(),
                         lens, static_cast<uint8_t*>(c->d_out.p), total, &enc, block_stride, d_blk,
                         &res);
    // 3. the compacted table (and its index blocks) back to the host
    if (r == HG_OK) {
        if (out_len) *out_len = enc;
        nb = h_blocks ? hg_block_count(res.n_out, block_stride) : 0;
        if (enc > cap) {
            r = HG_ERR_CAPACITY;
        } else {
            if (enc) r = rt_d2h_pipelined(c, h_out, c->d_out.p, enc);
            if (r == HG_OK && h_blocks && nb)
                r = rt_d2h_pipelined(c, h_blocks, d_blk, nb * sizeof(hg_block));
        }
    }
    if (result) *result = res;
    return r;
}

// ---- point lookups -----------------------------------------------------------------
uint64_t hg_keyindex_bytes(uint64_t n) { return hgk_keyindex_bytes(n); }

int hg_keyindex_build_dev_async(hg_ctx* c, const uint8_t* d_table, uint64_t len,
                                const hg_span* d_spans, uint64_t n, void* d_index) {
    if (!c || (n && (!d_table || !d_spans || !d_index))) return HG_ERR_INVALID_ARG;
    if (set_dev(c) != HG_OK) return HG_HIP_FAIL;
    if (capturing(c->stream)) return HG_ERR_INVALID_ARG;
    return hgk_keyindex_launch(d_table, len, d_spans, n, d_index, c->stream);
}

int hg_lookup_dev_async(hg_ctx* c, const uint8_t* d_table, const hg_span* d_spans,
                        const void* d_index, uint64_t n, uint32_t block_stride,
                        const uint8_t* d_keys, const hg_key* d_queries, uint64_t nq,
                        hg_lookup_result* d_results) {
    if (!c || (nq && (!d_queries || !d_results)) || (n && nq && (!d_table || !d_spans || !d_index)))
        return HG_ERR_INVALID_ARG;
    if (set_dev(c) != HG_OK) return HG_HIP_FAIL;
    if (capturing(c->stream)) return HG_ERR_INVALID_ARG;
    return hgk_lookup_launch(d_table, d_spans, d_index, n, block_stride, d_keys, d_queries, nq,
                             d_results, c->stream);
}

int hg_lookup_host(hg_ctx* c, const uint8_t* h_table, uint64_t len, uint32_t block_stride,
                   const uint8_t* h_keys, uint64_t keys_len, const hg_key* h_queries, uint64_t nq,
                   hg_lookup_result* h_results) {
    if (!c || (len && !h_table) || (nq && (!h_queries || !h_results)) || (keys_len && !h_keys))
        return HG_ERR_INVALID_ARG;
    if (len >= kMaxLen) return HG_ERR_TOO_LARGE;
    if (set_dev(c) != HG_OK) return HG_HIP_FAIL;
    for (uint64_t i = 0; i < nq; ++i)
        if (h_queries[i].off + h_queries[i].len > keys_len) return HG_ERR_INVALID_ARG;
    const uint64_t cap = len / 16;
    int r;
    if ((r = ensure(c, c->d_in, len ? len : 1)) != HG_OK) return r;
    if ((r = ensure(c, c->d_out, (cap ? cap : 1) * sizeof(hg_span))) != HG_OK) return r;
    if (len && (r = rt_h2d_pipelined(c, c->d_in.p, h_table, len)) != HG_OK) return r;
    uint64_t n = 0;
    hg_err e{};
    if (len) {
        r = hg_decode_dev(c, static_cast<const uint8_t*>(c->d_in.p), len,
                          static_cast<hg_span*>(c->d_out.p), cap, &n, &e);
        if (r != HG_OK) return r;  // a table that does not decode cannot be searched
    }
    const size_t qat = (keys_len + 63) & ~(size_t)63;
    if ((r = ensure(c, c->lk_index, (n ? n : 1) * 32)) != HG_OK) return r;
    if ((r = ensure(c, c->lk_keys, qat + (nq ? nq : 1) * sizeof(hg_key))) != HG_OK) return r;
    if ((r = ensure(c, c->lk_res, (nq ? nq : 1) * sizeof(hg_lookup_result))) != HG_OK) return r;
    char* kd = static_cast<char*>(c->lk_keys.p);
    if (keys_len && (r = rt_h2d_pipelined(c, kd, h_keys, keys_len)) != HG_OK) return r;
    if (nq && (r = rt_h2d_pipelined(c, kd + qat, h_queries, nq * sizeof(hg_key))) != HG_OK) return r;
    r = hg_keyindex_build_dev_async(c, static_cast<const uint8_t*>(c->d_in.p), len,
                                    static_cast<const hg_span*>(c->d_out.p), n, c->lk_index.p);
    if (r == HG_OK)
        r = hg_lookup_dev_async(c, static_cast<const uint8_t*>(c->d_in.p),
                                static_cast<const hg_span*>(c->d_out.p), c->lk_index.p, n,
                                block_stride, reinterpret_cast<const uint8_t*>(kd),
                                reinterpret_cast<const hg_key*>(kd + qat), nq,
                                static_cast<hg_lookup_result*>(c->lk_res.p));
    if (r != HG_OK) return r;
    if (nq && (r = rt_d2h_pipelined(c, h_results, c->lk_res.p, nq * sizeof(hg_lookup_result))) != HG_OK)
        return r;
    return HG_OK;
}

}  // extern "C"

// Internal entry points for hg_multi.hip (hg_internal.hpp).
namespace hgi {
int ensure_aux(hg_ctx* c, int want) { return rt_ensure_aux(c, want); }
bool host_pinned(const void* p) { return rt_host_pinned(p); }
int h2d_pipelined(hg_ctx* c, void* dst, const void* src, size_t bytes) {
    return rt_h2d_pipelined(c, dst, src, bytes);
}
int d2h_pipelined(hg_ctx* c, void* dst, const void* src, size_t bytes) {
    return rt_d2h_pipelined(c, dst, src, bytes);
}
void par_memcpy(void* dst, const void* src, size_t n) { rt_par_memcpy(dst, src, n); }
}  // namespace hgi
