// FETCH_SIZE calibration probe (not part of the product).  The microarch
// guide calibrates rocprofv3's FETCH_SIZE only for 16-byte-per-lane coalesced
// streaming reads (it reports half the bytes); the merge and encode kernels
// read in other widths.  Each kernel below reads a known number of distinct
// bytes of a 1 GiB buffer (well past the 256 MiB Infinity Cache) once, so
// FETCH_SIZE / known bytes is the factor for that access shape:
//   w16   16 B per lane, coalesced (the guide's case: expect 0.5)
//   w8    8 B per lane, coalesced (merge rounds' entry staging)
//   w4    4 B per lane, coalesced
//   rec   one unaligned 16-byte load at the start of every 132-byte record
//         (a key prefix per record: merge_prep's fallback pattern; bytes =
//         the distinct 128-byte lines touched)
//   gath  whole 132-byte records read as 16-byte unaligned pieces in a
//         shuffled record order, 8 tables interleaved (the compaction gather)
// Run under rocprofv3 --pmc FETCH_SIZE; prints each kernel's known bytes.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CHECK(x)                                                             \
    do {                                                                     \
        hipError_t e_ = (x);                                                 \
        if (e_ != hipSuccess) {                                              \
            printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); \
            exit(1);                                                         \
        }                                                                    \
    } while (0)

template <typename T>
__global__ __launch_bounds__(256) void wide(const T* src, uint64_t n, unsigned long long* out) {
    uint64_t acc = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) {
        const T v = src[i];
        acc ^= reinterpret_cast<const uint32_t*>(&v)[0];
    }
    if (acc == 0x1234567ull) out[0] = acc;
}

__global__ __launch_bounds__(256) void rec_prefix(const uint8_t* src, uint64_t nrec, unsigned long long* out) {
    uint64_t acc = 0;
    for (uint64_t r = (uint64_t)blockIdx.x * 256 + threadIdx.x; r < nrec; r += (uint64_t)gridDim.x * 256) {
        const uint4 v = *reinterpret_cast<const uint4*>(src + r * 132 + 16);
        acc ^= v.x ^ v.w;
    }
    if (acc == 0x1234567ull) out[0] = acc;
}

// record j of the merged order is perm[j] (a record index); 9 pieces of 16 B
// cover its 132 bytes (the last piece overlaps the next record: read anyway)
__global__ __launch_bounds__(256) void gather(const uint8_t* src, const uint32_t* perm, uint64_t nrec,
                                              unsigned long long* out) {
    uint64_t acc = 0;
    const uint64_t np = nrec * 9;
    for (uint64_t p = (uint64_t)blockIdx.x * 256 + threadIdx.x; p < np; p += (uint64_t)gridDim.x * 256) {
        const uint64_t j = p / 9, q = p % 9;
        const uint64_t r = perm[j];
        const uint64_t o = r * 132 + 16 * q;
        const uint4 v = *reinterpret_cast<const uint4*>(src + o);
        acc ^= v.x ^ v.w;
    }
    if (acc == 0x1234567ull) out[0] = acc;
}

int main() {
    const uint64_t bytes = 1ull << 30;
    uint8_t* d;
    unsigned long long* o;
    CHECK(hipMalloc(&d, bytes + 4096));
    CHECK(hipMalloc(&o, 64));
    CHECK(hipMemset(d, 1, bytes + 4096));
    const int grid = 8192;
    for (int rep = 0; rep < 2; ++rep) {
        hipLaunchKernelGGL(wide<uint4>, dim3(grid), dim3(256), 0, 0, (const uint4*)d, bytes / 16, o);
        hipLaunchKernelGGL(wide<uint2>, dim3(grid), dim3(256), 0, 0, (const uint2*)d, bytes / 8, o);
        hipLaunchKernelGGL(wide<uint32_t>, dim3(grid), dim3(256), 0, 0, (const uint32_t*)d, bytes / 4, o);
    }
    printf("wide<uint4> w16: %llu bytes\n", (unsigned long long)bytes);
    printf("wide<uint2> w8: %llu bytes\n", (unsigned long long)bytes);
    printf("wide<unsigned int> w4: %llu bytes\n", (unsigned long long)bytes);
    const uint64_t nrec = (bytes - 64) / 132;
    for (int rep = 0; rep < 2; ++rep)
        hipLaunchKernelGGL(rec_prefix, dim3(grid), dim3(256), 0, 0, (const uint8_t*)d, nrec, o);
    // lines touched by [r*132+16, +16): count on the host
    uint64_t lines = 0, last = ~0ull;
    for (uint64_t r = 0; r < nrec; ++r) {
        const uint64_t a = (r * 132 + 16) / 128, b = (r * 132 + 31) / 128;
        if (a != last) ++lines;
        if (b != a) ++lines;
        last = b;
    }
    printf("rec_prefix: %llu bytes (distinct 128-B lines)\n", (unsigned long long)(lines * 128));
    // gather order: 8 tables of nrec/8 records interleaved by a random merge
    const uint64_t per = nrec / 8, ng = per * 8;
    uint32_t* perm = (uint32_t*)malloc(ng * 4);
    uint64_t head[8] = {0};
    srand(5);
    for (uint64_t j = 0; j < ng; ++j) {
        int t;
        do t = rand() % 8; while (head[t] >= per);
        perm[j] = (uint32_t)(t * per + head[t]++);
    }
    uint32_t* dp;
    CHECK(hipMalloc(&dp, ng * 4));
    CHECK(hipMemcpy(dp, perm, ng * 4, hipMemcpyHostToDevice));
    for (int rep = 0; rep < 2; ++rep)
        hipLaunchKernelGGL(gather, dim3(grid), dim3(256), 0, 0, (const uint8_t*)d, (const uint32_t*)dp, ng, o);
    CHECK(hipDeviceSynchronize());
    printf("gather: %llu bytes of records (+ %llu perm bytes, 4 B per lane / 9 lanes)\n",
           (unsigned long long)(ng * 132), (unsigned long long)(ng * 4));
    free(perm);
    return 0;
}
