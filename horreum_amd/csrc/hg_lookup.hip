// hg_lookup.hip — batched point lookups on a decoded SSTable (gfx950).
//
// Replaces SSTable::get (reference src/sstable/table.rs:54-70): Index::get
// (src/sstable/index.rs:72-78) binary-searches the block first keys, the
// block is read and decoded, and binary_search_by_key finds the key in it.
// Both searches are Rust's slice::binary_search_by (std 1.52-1.81: probe
// mid = left + (right - left) / 2, return the first probe that compares
// Equal), so on tables with duplicate or unordered keys (legal,
// table.rs:93-108) the record found is the one the reference finds, not
// merely some record with the key.  A batch of queries runs on the device in
// one launch:
//   keyindex_kernel: one 32-byte entry per record (16-byte big-endian key
//     prefix, key length, record index), built once per decoded table;
//   lookup_kernel: one thread per query; the block search probes entries
//     b * stride (block first keys), the in-block search the block's entries
//     (one 32-byte load per probe; the top levels are shared by all queries
//     and stay in L2); keys that agree on 16 bytes and are both longer finish
//     the compare on the table bytes.
#include "hg_device.hpp"

namespace hgl {

constexpr uint32_t THREADS = 256;

struct KEnt {        // 32 bytes (same layout as the merge entries)
    uint64_t p0, p1; // key bytes [0,8), [8,16) big-endian, zero padded
    uint32_t klen;
    uint32_t pad;
    uint64_t rec;
};

__device__ __forceinline__ void prefix16(const uint8_t* k, uint32_t kl, uint64_t avail,
                                         uint64_t& w0, uint64_t& w1) {
    w0 = w1 = 0;
    if (avail >= 16) {
        uint64_t r0, r1;
        __builtin_memcpy(&r0, k, 8);
        __builtin_memcpy(&r1, k + 8, 8);
        if (kl < 8) r0 &= kl ? (~0ull >> (64 - 8 * kl)) : 0ull;
        if (kl < 16) r1 &= kl <= 8 ? 0ull : (~0ull >> (64 - 8 * (kl - 8)));
        w0 = __builtin_bswap64(r0);
        w1 = __builtin_bswap64(r1);
    } else {
        for (uint32_t i = 0; i < 16; ++i) {
            const uint64_t b = (i < kl && i < avail) ? k[i] : 0;
            if (i < 8) w0 = (w0 << 8) | b;
            else w1 = (w1 << 8) | b;
        }
    }
}

__global__ __launch_bounds__(THREADS) void keyindex_kernel(const uint8_t* table, uint64_t len,
                                                           const hg_span* spans, uint64_t n,
                                                           KEnt* ents) {
    const uint64_t i = (uint64_t)blockIdx.x * THREADS + threadIdx.x;
    if (i >= n) return;
    const hg_span s = spans[i];
    const uint64_t ko = s.off + 16;
    KEnt e;
    prefix16(table + ko, s.klen, len - ko, e.p0, e.p1);
    e.klen = s.klen;
    e.pad = 0;
    e.rec = i;
    ents[i] = e;
}

// Order of (table key of entry e) vs the query (q bytes, prefix qp0/qp1, ql).
__device__ __forceinline__ int cmp_entry(const uint8_t* table, const hg_span* spans, const KEnt& e,
                                         const uint8_t* q, uint64_t qp0, uint64_t qp1,
                                         uint32_t ql) {
    if (e.p0 != qp0) return e.p0 < qp0 ? -1 : 1;
    if (e.p1 != qp1) return e.p1 < qp1 ? -1 : 1;
    if (e.klen <= 16 || ql <= 16) return e.klen < ql ? -1 : e.klen > ql ? 1 : 0;
    const uint8_t* k = table + spans[e.rec].off + 16;
    const uint32_t m = min(e.klen, ql);
    for (uint32_t i = 16; i < m; ++i)
        if (k[i] != q[i]) return k[i] < q[i] ? -1 : 1;
    return e.klen < ql ? -1 : e.klen > ql ? 1 : 0;
}

// Rust's binary_search_by over entries base + i * step, i in [0, size):
// Ok(i) -> (true, i); Err(i) -> (false, i).
__device__ __forceinline__ bool rust_search(const uint8_t* table, const hg_span* spans,
                                            const KEnt* ents, uint64_t base, uint64_t step,
                                            uint64_t size, const uint8_t* q, uint64_t qp0,
                                            uint64_t qp1, uint32_t ql, uint64_t& pos) {
    uint64_t left = 0, right = size;
    while (left < right) {
        const uint64_t mid = left + (right - left) / 2;
        const int c = cmp_entry(table, spans, ents[base + mid * step], q, qp0, qp1, ql);
        if (c == 0) {
            pos = mid;
            return true;
        }
        if (c < 0) left = mid + 1;
        else right = mid;
    }
    pos = left;
    return false;
}

__global__ __launch_bounds__(THREADS) void lookup_kernel(const uint8_t* table, const hg_span* spans,
                                                         const KEnt* ents, uint64_t n,
                                                         uint64_t stride, const uint8_t* keys,
                                                         const hg_key* queries, uint64_t nq,
                                                         hg_lookup_result* out) {
    const uint64_t i = (uint64_t)blockIdx.x * THREADS + threadIdx.x;
    if (i >= nq) return;
    const hg_key qk = queries[i];
    const uint8_t* q = keys + qk.off;
    uint64_t qp0, qp1;
    prefix16(q, qk.len, qk.len, qp0, qp1);
    hg_lookup_result r;
    r.rec = ~0ull;
    r.val_off = 0;
    r.vlen = 0;
    r.found = 0;
    // Index::get (index.rs:72-78): Ok(b) -> block b; Err(b) -> block b - 1, none if b == 0
    const uint64_t nb = n ? (n - 1) / stride + 1 : 0;
    uint64_t b = 0;
    bool hit = rust_search(table, spans, ents, 0, stride, nb, q, qp0, qp1, qk.len, b);
    if (hit || b > 0) {
        if (!hit) --b;
        const uint64_t r0 = b * stride;
        const uint64_t cnt = n - r0 < stride ? n - r0 : stride;
        uint64_t j = 0;
        if (rust_search(table, spans, ents, r0, 1, cnt, q, qp0, qp1, qk.len, j)) {  // table.rs:65-68
            const hg_span s = spans[r0 + j];
            r.rec = r0 + j;
            r.val_off = s.off + 16 + s.klen;
            r.vlen = s.vlen;
            r.found = 1;
        }
    }
    out[i] = r;
}

}  // namespace hgl

extern "C" uint64_t hgk_keyindex_bytes(uint64_t n) { return n * sizeof(hgl::KEnt); }

extern "C" int hgk_keyindex_launch(const uint8_t* d_table, uint64_t len, const hg_span* d_spans,
                                   uint64_t n, void* d_index, hipStream_t stream) {
    using namespace hgl;
    if (n == 0) return HG_OK;
    hipLaunchKernelGGL(keyindex_kernel, dim3((uint32_t)((n + THREADS - 1) / THREADS)),
                       dim3(THREADS), 0, stream, d_table, len, d_spans, n,
                       static_cast<KEnt*>(d_index));
    return HG_LAUNCH_STATUS();
}

// block_stride 0: the whole table is one block.
extern "C" int hgk_lookup_launch(const uint8_t* d_table, const hg_span* d_spans,
                                 const void* d_index, uint64_t n, uint32_t block_stride,
                                 const uint8_t* d_keys, const hg_key* d_queries, uint64_t nq,
                                 hg_lookup_result* d_results, hipStream_t stream) {
    using namespace hgl;
    if (nq == 0) return HG_OK;
    const uint64_t stride = block_stride ? block_stride : (n ? n : 1);
    hipLaunchKernelGGL(lookup_kernel, dim3((uint32_t)((nq + THREADS - 1) / THREADS)),
                       dim3(THREADS), 0, stream, d_table, d_spans,
                       static_cast<const KEnt*>(d_index), n, stride, d_keys, d_queries, nq,
                       d_results);
    return HG_LAUNCH_STATUS();
}
