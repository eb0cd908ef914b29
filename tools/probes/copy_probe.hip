// Device-copy probe (not part of the product): what read+write rate a plain
// 16-byte-per-lane copy reaches on this GPU, by loads in flight per lane
// (U), cache policy and grid shape.  Sets the practical ceiling for encode
// (which reads and writes each byte once).  Prints GB/s (read + write bytes).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

template <int U, bool NT>
__global__ __launch_bounds__(256) void copy_grid(const u32x4* __restrict__ src, u32x4* __restrict__ dst,
                                                 uint64_t n16) {
    const uint64_t stride = (uint64_t)gridDim.x * 256 * U;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 * U + threadIdx.x; i < n16; i += stride) {
        u32x4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t j = i + (uint64_t)u * 256;
            if (j < n16) v[u] = NT ? __builtin_nontemporal_load(src + j) : src[j];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t j = i + (uint64_t)u * 256;
            if (j < n16) {
                if (NT) __builtin_nontemporal_store(v[u], dst + j);
                else dst[j] = v[u];
            }
        }
    }
}

// one tile of T x 16 B per workgroup (no grid-stride loop), like encode's tiles
template <int T, bool NT>
__global__ __launch_bounds__(256) void copy_tile(const u32x4* __restrict__ src, u32x4* __restrict__ dst,
                                                 uint64_t n16) {
    const uint64_t b = (uint64_t)blockIdx.x * 256 * T;
#pragma unroll 1
    for (int t = 0; t < T; ++t) {
        const uint64_t j = b + (uint64_t)t * 256 + threadIdx.x;
        if (j < n16) {
            u32x4 v = NT ? __builtin_nontemporal_load(src + j) : src[j];
            if (NT) __builtin_nontemporal_store(v, dst + j);
            else dst[j] = v;
        }
    }
}

// each workgroup copies one contiguous chunk (no grid stride), U loads in
// flight per lane, TH threads per workgroup
template <int U, int TH, bool NT>
__global__ __launch_bounds__(TH) void copy_chunk(const u32x4* __restrict__ src, u32x4* __restrict__ dst,
                                                 uint64_t n16, uint64_t per) {
    const uint64_t b = (uint64_t)blockIdx.x * per;
    const uint64_t e = b + per < n16 ? b + per : n16;
    for (uint64_t i = b + threadIdx.x; i < e; i += (uint64_t)TH * U) {
        u32x4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t j = i + (uint64_t)u * TH;
            if (j < e) v[u] = NT ? __builtin_nontemporal_load(src + j) : src[j];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t j = i + (uint64_t)u * TH;
            if (j < e) {
                if (NT) __builtin_nontemporal_store(v[u], dst + j);
                else dst[j] = v[u];
            }
        }
    }
}

// loads nontemporal, stores default (or the reverse): which side the policy helps
template <int U, bool NTL, bool NTS>
__global__ __launch_bounds__(256) void copy_mixed(const u32x4* __restrict__ src, u32x4* __restrict__ dst,
                                                  uint64_t n16) {
    const uint64_t stride = (uint64_t)gridDim.x * 256 * U;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 * U + threadIdx.x; i < n16; i += stride) {
        u32x4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t j = i + (uint64_t)u * 256;
            if (j < n16) v[u] = NTL ? __builtin_nontemporal_load(src + j) : src[j];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t j = i + (uint64_t)u * 256;
            if (j < n16) {
                if (NTS) __builtin_nontemporal_store(v[u], dst + j);
                else dst[j] = v[u];
            }
        }
    }
}

// Round 6: the read side by LDS-DMA (global_load_lds, the decode pre-pass's
// 7.1 TB/s read form) into NBUF 16 KiB LDS buffers, NBUF - 1 in flight, the
// write side by 16-byte nontemporal stores from LDS; each workgroup copies a
// contiguous span of PPB pieces.
template <int NBUF>
__global__ __launch_bounds__(256) void copy_glds(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst,
                                                 uint32_t ppb) {
    extern __shared__ u32x4 lbuf[];
    constexpr uint32_t PIECE = 16384;
    const uint32_t tid = threadIdx.x, wid = tid >> 6, lane = tid & 63u;
    const uint64_t base = (uint64_t)blockIdx.x * ppb * PIECE;
    auto issue = [&](uint32_t k) {
        const uint8_t* s = src + base + (uint64_t)k * PIECE;
        uint8_t* d = reinterpret_cast<uint8_t*>(lbuf) + (k % NBUF) * PIECE;
#pragma unroll
        for (uint32_t q = 0; q < 4; ++q) {
            const uint32_t g0 = q * 256 + wid * 64;
            __builtin_amdgcn_global_load_lds(static_cast<const void*>(s + (uint64_t)(g0 + lane) * 16),
                                             (__attribute__((address_space(3))) void*)(d + g0 * 16), 16, 0, 2);
        }
    };
    for (uint32_t k = 0; k + 1 < NBUF && k < ppb; ++k) issue(k);
    for (uint32_t k = 0; k < ppb; ++k) {
        if (k + NBUF - 1 < ppb) {
            issue(k + NBUF - 1);
            // stores of earlier pieces are older than these DMAs: counted waits
            // cover them too (conservative)
            if (NBUF == 2) __asm__ volatile("s_waitcnt vmcnt(4)" ::: "memory");
            else __asm__ volatile("s_waitcnt vmcnt(8)" ::: "memory");
        } else {
            __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        __asm__ volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        const u32x4* l = lbuf + (k % NBUF) * (PIECE / 16);
        u32x4* o = reinterpret_cast<u32x4*>(dst + base + (uint64_t)k * PIECE);
        u32x4 v[4];
#pragma unroll
        for (uint32_t q = 0; q < 4; ++q) v[q] = l[q * 256 + tid];
#pragma unroll
        for (uint32_t q = 0; q < 4; ++q) __builtin_nontemporal_store(v[q], o + q * 256 + tid);
        __asm__ volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    }
}

template <typename F>
static float time_it(F f) {
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    f();
    CHECK(hipDeviceSynchronize());
    float best = 1e30f, tot = 0;
    const int reps = 7;
    for (int r = 0; r < reps; ++r) {
        CHECK(hipEventRecord(a));
        f();
        CHECK(hipEventRecord(b));
        CHECK(hipEventSynchronize(b));
        float ms;
        CHECK(hipEventElapsedTime(&ms, a, b));
        tot += ms;
        if (ms < best) best = ms;
    }
    return tot / reps;
}

int main() {
    const uint64_t bytes = 3040000000ull;
    const uint64_t n16 = bytes / 16;
    u32x4 *src, *dst;
    CHECK(hipMalloc(&src, bytes));
    CHECK(hipMalloc(&dst, bytes));
    CHECK(hipMemset(src, 1, bytes));
    auto rep = [&](const char* name, float ms) {
        printf("%-34s %8.4f ms  %7.1f GB/s (r+w)\n", name, ms, 2.0 * bytes / ms / 1e6);
        fflush(stdout);
    };
    rep("hipMemcpyAsync d2d", time_it([&] { CHECK(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, 0)); }));
    for (int g : {2048, 4096, 8192}) {
        char nm[64];
#define G(U, NT)                                                                              \
        snprintf(nm, sizeof nm, "grid %d U=%d nt=%d", g, U, NT);                              \
        rep(nm, time_it([&] { copy_grid<U, NT><<<g, 256>>>(src, dst, n16); }));
        G(1, false) G(1, true) G(2, true) G(4, true) G(4, false) G(8, true)
#undef G
    }
    {
        const uint64_t nb19 = (n16 + 256 * 19 - 1) / (256 * 19);
        rep("tile 19x1KiB nt (encode-shaped)", time_it([&] { copy_tile<19, true><<<(uint32_t)nb19, 256>>>(src, dst, n16); }));
        rep("tile 19x1KiB default", time_it([&] { copy_tile<19, false><<<(uint32_t)nb19, 256>>>(src, dst, n16); }));
        const uint64_t nb76 = (n16 + 256 * 76 - 1) / (256 * 76);
        rep("tile 76x1KiB nt", time_it([&] { copy_tile<76, true><<<(uint32_t)nb76, 256>>>(src, dst, n16); }));
    }
    if (getenv("COPY_GLDS")) {
        const uint32_t npieces = (uint32_t)(bytes / 16384);
        for (uint32_t ppb : {16u, 32u, 64u, 128u}) {
            char nm[64];
            const uint32_t g = npieces / ppb;
            CHECK(hipFuncSetAttribute((const void*)copy_glds<2>, hipFuncAttributeMaxDynamicSharedMemorySize, 40960));
            CHECK(hipFuncSetAttribute((const void*)copy_glds<3>, hipFuncAttributeMaxDynamicSharedMemorySize, 49152));
            snprintf(nm, sizeof nm, "glds copy x2 ppb=%u grid %u", ppb, g);
            rep(nm, time_it([&] { copy_glds<2><<<g, 256, 40960>>>((const uint8_t*)src, (uint8_t*)dst, ppb); }));
            snprintf(nm, sizeof nm, "glds copy x3 ppb=%u grid %u", ppb, g);
            rep(nm, time_it([&] { copy_glds<3><<<g, 256, 49152>>>((const uint8_t*)src, (uint8_t*)dst, ppb); }));
        }
        for (int g : {4096, 8192, 16384}) {
            char nm[64];
            snprintf(nm, sizeof nm, "grid %d U=8 nt=1", g);
            rep(nm, time_it([&] { copy_grid<8, true><<<g, 256>>>(src, dst, n16); }));
        }
        CHECK(hipFree(src));
        CHECK(hipFree(dst));
        return 0;
    }
    for (int g : {256, 512, 1024, 2048}) {  // contiguous chunk per workgroup
        char nm[64];
        const uint64_t per = (n16 + g - 1) / g;
#define C(U, TH, NT)                                                                          \
        snprintf(nm, sizeof nm, "chunk %d U=%d th=%d nt=%d", g, U, TH, NT);                  \
        rep(nm, time_it([&] { copy_chunk<U, TH, NT><<<g, TH>>>(src, dst, n16, per); }));
        C(4, 256, true) C(8, 256, true) C(16, 256, true) C(4, 512, true) C(8, 512, true)
        C(4, 1024, true) C(8, 1024, false)
#undef C
    }
    for (int g : {4096, 8192}) {
        char nm[64];
#define M(U, L, S)                                                                            \
        snprintf(nm, sizeof nm, "grid %d U=%d ntl=%d nts=%d", g, U, L, S);                     \
        rep(nm, time_it([&] { copy_mixed<U, L, S><<<g, 256>>>(src, dst, n16); }));
        M(8, true, false) M(8, false, true) M(16, true, true)
#undef M
    }
    CHECK(hipFree(src));
    CHECK(hipFree(dst));
    return 0;
}
