// Read-only probe (not part of the product): what reading only the 16-byte
// record headers of a fixed-stride table costs against streaming the whole
// table.  cfg 2's records are 132 bytes, so nearly every 128-byte line holds
// a header; the question is whether the memory side fetches whole lines or
// only the sectors a header touches.  Prints us and GB/s of table bytes.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

// Whole table, 16 B per lane per step, grid-stride; a sum keeps the loads live.
__global__ __launch_bounds__(256) void read_all(const uint4* __restrict__ src, uint64_t n16,
                                                uint32_t* __restrict__ sink) {
    uint32_t acc = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * 256) {
        const uint4 v = src[i];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

// One 16-byte header per record at stride R (lane per record), U loads in flight.
template <int U>
__global__ __launch_bounds__(256) void read_headers(const uint8_t* __restrict__ src, uint64_t nrec,
                                                    uint64_t R, uint32_t* __restrict__ sink) {
    uint32_t acc = 0;
    const uint64_t step = (uint64_t)gridDim.x * 256 * U;
    for (uint64_t i0 = (uint64_t)blockIdx.x * 256 * U + threadIdx.x; i0 < nrec; i0 += step) {
        uint4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t i = i0 + (uint64_t)u * 256;
            v[u] = make_uint4(0, 0, 0, 0);
            if (i < nrec) {
                const uint32_t* p = reinterpret_cast<const uint32_t*>(src + i * R);
                v[u] = make_uint4(p[0], p[1], p[2], p[3]);
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) acc ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
    }
    if (acc == 0x12345678u) sink[0] = acc;
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
    const uint64_t L = 1073741724ull;  // cfg 2 table bytes
    uint8_t* src;
    uint32_t* sink;
    CHECK(hipMalloc(&src, L + 4096));
    CHECK(hipMalloc(&sink, 64));
    CHECK(hipMemset(src, 1, L + 4096));
    auto rep = [&](const char* name, float ms) {
        printf("%-40s %8.2f us  %7.1f GB/s of table\n", name, ms * 1e3, L / (ms * 1e-3) / 1e9);
    };
    const uint64_t n16 = L / 16;
    for (int grid : {1024, 2048, 4096})
        for (int rep_i = 0; rep_i < 1; ++rep_i) {
            char nm[96];
            snprintf(nm, sizeof nm, "read_all grid %d", grid);
            rep(nm, time_it([&] { hipLaunchKernelGGL(read_all, dim3(grid), dim3(256), 0, 0,
                                                     reinterpret_cast<const uint4*>(src), n16, sink); }));
        }
    for (uint64_t R : {132ull, 128ull, 256ull, 512ull}) {
        const uint64_t nrec = L / R;
        for (int grid : {1024, 4096}) {
            char nm[96];
            snprintf(nm, sizeof nm, "headers R=%llu grid %d U=4", (unsigned long long)R, grid);
            rep(nm, time_it([&] { hipLaunchKernelGGL(read_headers<4>, dim3(grid), dim3(256), 0, 0, src,
                                                     nrec, R, sink); }));
        }
    }
    return 0;
}
