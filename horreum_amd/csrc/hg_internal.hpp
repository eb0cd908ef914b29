// hg_internal.hpp — host-runtime internals shared by hg_runtime.hip and
// hg_multi.hip (not part of the C ABI): the context, its device / pinned
// buffers and the staging helpers.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include <vector>

#include "../../include/horreum_gpu.h"
#include "hg_device.hpp"  // hgk_multi_ctl, hgk_merge_records
#include "hg_err.hpp"

extern "C" uint64_t hgk_decode_ctl_bytes(uint64_t len);
extern "C" int hgk_decode_launch_ctl(const uint8_t*, uint64_t, hg_span*, uint64_t,
                                     hg_decode_result*, void* d_ws, void* d_ctl, uint64_t clean,
                                     void* d_next, uint64_t next_bytes, uint64_t* zeroed,
                                     hipStream_t);
extern "C" int hgk_decode_launch(const uint8_t*, uint64_t, hg_span*, uint64_t, hg_decode_result*,
                                 void*, hipStream_t);
extern "C" int hgk_decode_range_launch(const uint8_t*, uint64_t, uint64_t, uint64_t, uint64_t,
                                       uint64_t, hg_span*, uint64_t, hg_decode_result*, void*,
                                       hipStream_t);
extern "C" int hgk_decode_guess_launch(const uint8_t*, uint64_t, uint64_t, uint64_t, uint64_t*,
                                       void*, hipStream_t);
extern "C" uint64_t hgk_decode_workspace_bytes(uint64_t);
extern "C" uint64_t hgk_decode_multi_stage_bytes(uint32_t);
extern "C" int hgk_decode_launch_multi(uint32_t, const uint8_t* const*, const uint64_t*,
                                       hg_span* const*, const uint64_t*, hg_decode_result*, void*,
                                       const uint64_t*, void*, void*, hipStream_t, uint32_t,
                                       const hgk_multi_ctl* mc);
extern "C" int hgk_encode_launch(const uint8_t*, const hg_pair*, uint64_t, uint8_t*, uint64_t,
                                 uint64_t*, uint32_t, hg_block*, hg_encode_result*,
                                 unsigned long long*, hipStream_t);
extern "C" uint64_t hgk_encode_workspace_bytes(uint64_t);
extern "C" int hgk_encode_launch_at(const uint8_t*, const hg_pair*, uint64_t, uint8_t*, uint64_t,
                                    uint64_t*, uint64_t, uint32_t, hg_block*, hg_encode_result*,
                                    unsigned long long*, hipStream_t);
extern "C" int hgk_encode_launch_ex(const uint8_t*, const hg_pair*, uint64_t, const uint64_t*, bool,
                                    uint8_t*, uint64_t, uint64_t*, uint64_t, uint32_t, hg_block*,
                                    hg_encode_result*, unsigned long long*, hipStream_t);
extern "C" int hgk_encode_launch_records(const uint8_t*, uint64_t, const hg_pair*, uint64_t,
                                         const uint64_t*, uint8_t*, uint64_t, uint64_t*, uint32_t,
                                         hg_block*, hg_encode_result*, unsigned long long*,
                                         hipStream_t, int gsum_zeroed, int sums_ready);
extern "C" void hgk_encode_group_sums(uint64_t n, uint64_t* first_word, uint64_t* words);
extern "C" void hgk_encode_tile_geometry(uint32_t* tile_log2, uint32_t* group_log2);
extern "C" int hgk_encode_launch_ctl(const uint8_t*, const hg_pair*, uint64_t, uint8_t*, uint64_t,
                                     uint64_t*, uint32_t, hg_block*, hg_encode_result*,
                                     unsigned long long*, uint64_t* gs_cur, uint64_t clean,
                                     uint64_t* gs_next, uint64_t next_words, uint64_t* zeroed,
                                     hipStream_t);
extern "C" int hgk_encode_blocks_launch(const uint64_t*, uint64_t, uint32_t, uint64_t, hg_block*,
                                        hipStream_t);
extern "C" int hgk_encode_size_launch(const hg_pair*, uint64_t, hg_encode_result*, unsigned long long*,
                                      hipStream_t);
extern "C" int hgk_gather_stride_launch(const uint64_t*, uint64_t, uint64_t, uint64_t, uint64_t*,
                                        hipStream_t);
extern "C" uint64_t hgk_keyindex_bytes(uint64_t);
extern "C" int hgk_keyindex_launch(const uint8_t*, uint64_t, const hg_span*, uint64_t, void*,
                                   hipStream_t);
extern "C" int hgk_lookup_launch(const uint8_t*, const hg_span*, const void*, uint64_t,
                                 uint32_t, const uint8_t*, const hg_key*, uint64_t,
                                 hg_lookup_result*, hipStream_t);
extern "C" void hgk_decode_ws_layout(uint64_t, uint64_t*, uint64_t*, uint64_t*);
extern "C" int hgk_decode_entries_launch(const void* d_stage, uint32_t ntab, uint32_t nspec_total,
                                         const uint64_t* d_run_off, void* d_ent,
                                         unsigned long long* d_err, hipStream_t stream);
extern "C" uint32_t hgk_decode_multi_geometry(const void* h_stage, uint32_t ntab);
extern "C" uint64_t hgk_merge_workspace_bytes(uint32_t, uint64_t);
extern "C" uint64_t hgk_merge_staging_bytes(uint32_t);
extern "C" int hgk_merge_launch(const uint8_t*, uint64_t, uint32_t, const uint64_t*,
                                const hg_span* const*, const uint64_t*, hg_pair*, uint64_t,
                                hg_merge_result*, void*, void*, hipStream_t, int defer,
                                const uint64_t* kp, uint32_t kp_tag,
                                const unsigned long long* d_err_pre,
                                const hgk_merge_records* rec, int* done);
extern "C" int hgk_encode_blocks_launch_dev(const uint64_t* d_rec_off, uint64_t n_ub,
                                            const uint64_t* d_n, const hg_encode_result* d_res,
                                            uint32_t stride, hg_block* d_blocks, hipStream_t stream);
extern "C" int hgk_merge_prebuild(const uint64_t* kp, uint32_t ntables,
                                  const hg_decode_result* d_results, uint64_t* d_run_off,
                                  unsigned long long* d_err, void* d_ws, hipStream_t stream);
extern "C" int hgk_merge_epochs(const uint8_t*, uint64_t, uint32_t, const uint64_t*,
                                const hg_span* const*, const uint64_t*, hg_pair*, uint64_t,
                                hg_merge_result*, hg_merge_result*, void*, void*, hipStream_t);

namespace hgi {

constexpr uint64_t kMaxLen = 1ull << 40;  // 40-bit positions in decode statuses

struct DevBuf {
    void* p = nullptr;
    size_t bytes = 0;
};

struct PinBuf {
    void* p = nullptr;
    size_t bytes = 0;
};

}  // namespace hgi

struct hg_ctx {
    int device = 0;
    hipStream_t own = nullptr;
    hipStream_t stream = nullptr;
    hgi::DevBuf ws;        // decode statuses / encode tile statuses
    // single-table decode: two control regions used in turn, each call's
    // pre-pass clearing the other's (hgk_decode_launch_ctl); dctl_clean:
    // bytes of each known to be zero
    hgi::DevBuf dctl;
    uint64_t dctl_clean[2] = {0, 0};
    int dctl_cur = 0;
    // device-pair encode: its group sums in two halves used in turn, each
    // call's bases kernel clearing the other's (hgk_encode_launch_ctl)
    hgi::DevBuf egs;
    uint64_t egs_clean[2] = {0, 0};
    int egs_cur = 0;
    hgi::DevBuf recoff;    // encode record offsets when blocks are wanted w/o rec_off
    hgi::DevBuf results;   // hg_decode_result + hg_encode_result
    hgi::PinBuf hres;      // pinned mirror of `results`
    // host-path staging (device side)
    hgi::DevBuf d_in, d_out, d_aux, d_blk;
    hgi::PinBuf h_stage[2];
    // merge: workspace, result, pinned argument staging and its reuse event
    hgi::DevBuf mws, mres, mspans, mpairs;
    hgi::DevBuf lk_index, lk_keys, lk_res;  // host lookup path
    hgi::PinBuf mstage;
    hipEvent_t mstage_ev = nullptr;
    bool mstage_busy = false;
    // batched decode: auxiliary streams (fork/join on `stream`), one workspace each
    static constexpr int kAux = 8;
    int naux = 0;
    hipStream_t aux[kAux] = {};
    hgi::DevBuf aux_ws[kAux];
    hipEvent_t fork_ev = nullptr, join_ev[kAux] = {};
    // batched decode in one launch: all tables' workspaces, argument staging
    hgi::DevBuf bws, bstage_d;
    hgi::PinBuf bstage;
    // its control regions in two halves used in turn (hgk_multi_ctl): per half
    // the region offsets of the call that cleared it and the bytes cleared
    hgi::DevBuf bctl;
    int bctl_cur = 0;
    std::vector<uint64_t> bctl_off[2], bctl_zero[2];
    // bstage_d in two halves used with the control halves (the arguments
    // point at the call's control half, so a call's bytes repeat two calls
    // later); what each half holds (a host copy), and the last call's half
    std::vector<uint8_t> bstage_shadow[2];
    void* bstage_last = nullptr;
    hipEvent_t bstage_ev = nullptr;
    bool bstage_busy = false;
    // multi-context driver (hg_multi.hip): decode results, gathered offsets
    hgi::DevBuf x_res, x_aux;
    hgi::DevBuf x_arena, x_spans;  // split compaction: this context's key-range slices
    uint32_t kpre_calls = 0;       // compaction-mode decode tags (hg_decode.hip kpre_tag)
    // compaction: the decode results' pinned copy and its event (the merge
    // entries are built while the host waits on it)
    hgi::PinBuf kres;
    hipEvent_t kres_ev = nullptr;
};

namespace hgi {
// Restores the calling thread's current HIP device on scope exit: the
// multi-context entry points switch devices on the caller's thread (set_dev,
// peer enabling), and a caller that allocates next must stay on its own GPU.
struct DeviceGuard {
    int dev = -1;
    DeviceGuard() {
        if (hipGetDevice(&dev) != hipSuccess) dev = -1;
    }
    ~DeviceGuard() {
        if (dev >= 0) (void)hipSetDevice(dev);
    }
    DeviceGuard(const DeviceGuard&) = delete;
    DeviceGuard& operator=(const DeviceGuard&) = delete;
};
int set_dev(hg_ctx* c);
int ensure(hg_ctx* c, DevBuf& b, size_t bytes);
int ensure_pin(PinBuf& b, size_t bytes);
bool try_grow(hg_ctx* c, DevBuf& b, size_t bytes);
int rt_encode_dev(hg_ctx* c, const uint8_t* d_arena, const hg_pair* d_pairs, uint64_t n,
                  uint8_t* d_out, uint64_t cap, uint64_t* d_rec_off, uint32_t block_stride,
                  hg_block* d_blocks, uint64_t* out_len, bool gather);
int ensure_aux(hg_ctx* c, int want);
bool host_pinned(const void* p);
int h2d_pipelined(hg_ctx* c, void* dst, const void* src, size_t bytes);
int d2h_pipelined(hg_ctx* c, void* dst, const void* src, size_t bytes);
void par_memcpy(void* dst, const void* src, size_t n);
}  // namespace hgi
