// glds_probe: checks the lane-walk mode's global->LDS piece DMA pattern
// (16-byte global_load_lds, 1 KiB per wave instruction) against a plain copy.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

constexpr uint32_t PIECE = 16384, THREADS = 256, GPT = PIECE / 16 / THREADS;

__device__ __forceinline__ void dma_piece(const uint8_t* src, uint8_t* dst) {
    const uint32_t tid = threadIdx.x, wid = tid >> 6;
#pragma unroll
    for (uint32_t q = 0; q < GPT; ++q) {
        const uint32_t g0 = q * THREADS + wid * 64;
        __builtin_amdgcn_global_load_lds(static_cast<const void*>(src + (uint64_t)(g0 + (tid & 63u)) * 16),
                                         (__attribute__((address_space(3))) void*)(dst + g0 * 16), 16, 0, 0);
    }
}

__global__ __launch_bounds__(THREADS) void k(const uint8_t* in, uint8_t* out, int npieces) {
    __shared__ uint64_t a[PIECE / 8 + 8];
    __shared__ uint64_t b[PIECE / 8 + 8];
    uint8_t* bufs0 = reinterpret_cast<uint8_t*>(a);
    uint8_t* bufs1 = reinterpret_cast<uint8_t*>(b);
    dma_piece(in, bufs0);
    for (int p = 0; p < npieces; ++p) {
        __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __asm__ volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        uint8_t* cur = ((p & 1) ? bufs1 : bufs0);
        if (p + 1 < npieces) dma_piece(in + (uint64_t)(p + 1) * PIECE, (((p + 1) & 1) ? bufs1 : bufs0));
        for (uint32_t q = 0; q < GPT; ++q) {
            const uint32_t gi = q * THREADS + threadIdx.x;
            *reinterpret_cast<uint4*>(out + (uint64_t)p * PIECE + gi * 16) =
                *reinterpret_cast<const uint4*>(cur + gi * 16);
        }
        __asm__ volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    }
}

int main() {
    const int np = 64;
    const size_t n = (size_t)np * PIECE;
    uint8_t* h = (uint8_t*)malloc(n);
    for (size_t i = 0; i < n; ++i) h[i] = (uint8_t)(i * 131 + (i >> 9));
    uint8_t *din, *dout;
    hipMalloc(&din, n);
    hipMalloc(&dout, n);
    hipMemcpy(din, h, n, hipMemcpyHostToDevice);
    hipMemset(dout, 0, n);
    hipLaunchKernelGGL(k, dim3(1), dim3(THREADS), 0, 0, din, dout, np);
    uint8_t* r = (uint8_t*)malloc(n);
    hipMemcpy(r, dout, n, hipMemcpyDeviceToHost);
    size_t bad = 0, first = ~(size_t)0;
    for (size_t i = 0; i < n; ++i)
        if (r[i] != h[i]) {
            if (first == ~(size_t)0) first = i;
            ++bad;
        }
    printf("glds_probe: %zu bad bytes of %zu, first at %zd (err %s)\n", bad, n, (ssize_t)first,
           hipGetErrorString(hipGetLastError()));
    return bad ? 1 : 0;
}
