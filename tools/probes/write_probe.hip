// Store-only probe (not part of the product): what rate 16-byte-per-lane
// stores of 130 MB (the cfg 2 span array) reach, by layout of the writes over
// the grid, stores per lane per iteration and cache policy.  Sets the
// ceiling for decode_kernel's span emission.  Prints GB/s of bytes written.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

// Workgroup b writes its own contiguous share (like decode_kernel: one
// pre-pass batch's spans per workgroup), ROW x 16 B per pass over 256 lanes.
template <int U, bool NT>
__global__ __launch_bounds__(256) void write_share(u32x4* __restrict__ dst, uint64_t n16, uint64_t per) {
    const uint64_t b0 = (uint64_t)blockIdx.x * per;
    const uint64_t b1 = b0 + per < n16 ? b0 + per : n16;
    for (uint64_t i = b0 + threadIdx.x * U; i < b1; i += 256 * U) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t j = i + u;
            u32x4 v = {(uint32_t)j, (uint32_t)(j >> 32), 16u, 100u};
            if (j < b1) {
                if (NT) __builtin_nontemporal_store(v, dst + j);
                else dst[j] = v;
            }
        }
    }
}

// Same share, lanes interleaved: store u of a pass covers 256 consecutive
// 16-byte slots (the current emission's pattern).
template <int U, bool NT>
__global__ __launch_bounds__(256) void write_share_il(u32x4* __restrict__ dst, uint64_t n16, uint64_t per) {
    const uint64_t b0 = (uint64_t)blockIdx.x * per;
    const uint64_t b1 = b0 + per < n16 ? b0 + per : n16;
    for (uint64_t i = b0 + threadIdx.x; i < b1; i += 256 * U) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t j = i + (uint64_t)u * 256;
            u32x4 v = {(uint32_t)j, (uint32_t)(j >> 32), 16u, 100u};
            if (j < b1) {
                if (NT) __builtin_nontemporal_store(v, dst + j);
                else dst[j] = v;
            }
        }
    }
}

// 124 of 256 lanes per pass (one 16 KiB piece of 132-byte records per pass)
__global__ __launch_bounds__(256) void write_share_piece(u32x4* __restrict__ dst, uint64_t n16, uint64_t per) {
    const uint64_t b0 = (uint64_t)blockIdx.x * per;
    const uint64_t b1 = b0 + per < n16 ? b0 + per : n16;
    for (uint64_t i = b0; i < b1; i += 124) {
        const uint64_t j = i + threadIdx.x;
        u32x4 v = {(uint32_t)j, (uint32_t)(j >> 32), 16u, 100u};
        if (threadIdx.x < 124 && j < b1) dst[j] = v;
    }
}

template <typename F>
static float time_it(F f) {
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    f();
    CHECK(hipDeviceSynchronize());
    float tot = 0;
    const int reps = 20;
    CHECK(hipEventRecord(a));
    for (int r = 0; r < reps; ++r) f();
    CHECK(hipEventRecord(b));
    CHECK(hipEventSynchronize(b));
    CHECK(hipEventElapsedTime(&tot, a, b));
    return tot / reps;
}

int main() {
    const uint64_t n16 = 8134407ull;  // cfg 2 spans
    const uint64_t bytes = n16 * 16;
    u32x4* dst;
    CHECK(hipMalloc(&dst, bytes + 4096));
    auto rep = [&](const char* name, float ms) {
        printf("%-36s %8.2f us  %7.1f GB/s\n", name, ms * 1e3, bytes / (ms * 1e-3) / 1e9);
    };
    for (int grid : {1024, 2048, 4096}) {
        const uint64_t per = (n16 + grid - 1) / grid;
        char nm[96];
#define RUN(K, U, NT, label)                                                                   \
        snprintf(nm, sizeof nm, "grid %d %s", grid, label);                                    \
        rep(nm, time_it([&] { hipLaunchKernelGGL((K<U, NT>), dim3(grid), dim3(256), 0, 0, dst, n16, per); }));
        RUN(write_share_il, 1, false, "il U=1");
        RUN(write_share_il, 4, false, "il U=4");
        RUN(write_share_il, 4, true, "il U=4 nt");
        RUN(write_share, 2, false, "contig U=2");
        RUN(write_share, 4, false, "contig U=4");
        snprintf(nm, sizeof nm, "grid %d piece124", grid);
        rep(nm, time_it([&] { hipLaunchKernelGGL(write_share_piece, dim3(grid), dim3(256), 0, 0, dst, n16, per); }));
    }
    const float ms = time_it([&] { CHECK(hipMemsetAsync(dst, 0, bytes, 0)); });
    rep("hipMemsetAsync", ms);
    return 0;
}
