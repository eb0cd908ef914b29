// VALU issue cost per wave64 instruction of the integer operations the
// lane-walk masks and walks are built from (gfx950).  Each thread runs 8
// independent chains of one operation; the time per wave-instruction per SIMD
// is printed for each.  Build: hipcc --offload-arch=gfx950 -O3 valu_rate.hip -o valu_rate
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

constexpr int ITERS = 2048, CH = 8, BLOCKS = 4096, THREADS = 256;

#define KERNEL(name, expr)                                                                \
    __global__ __launch_bounds__(THREADS) void name(uint32_t* out, uint32_t s0, uint32_t s1) { \
        uint32_t v[CH];                                                                   \
        for (int c = 0; c < CH; ++c) v[c] = threadIdx.x * 0x9E3779B9u + c * 0x85EBCA6Bu + s0; \
        const uint32_t k = s1 + (threadIdx.x & 3);                                        \
        for (int i = 0; i < ITERS; ++i) {                                                 \
            _Pragma("unroll") for (int c = 0; c < CH; ++c) {                              \
                uint32_t x = v[c];                                                        \
                x = (expr);                                                               \
                __asm__ volatile("" : "+v"(x));                                           \
                v[c] = x;                                                                 \
            }                                                                             \
        }                                                                                 \
        uint32_t r = 0;                                                                   \
        for (int c = 0; c < CH; ++c) r ^= v[c];                                           \
        if (r == 0x12345678u) out[0] = r;                                                 \
    }

KERNEL(k_add, x + k)
KERNEL(k_mulhi, __umulhi(x, k))
KERNEL(k_udot4, __builtin_amdgcn_udot4(x, k, x, false))
KERNEL(k_alignbyte, __builtin_amdgcn_alignbyte(x, k, x & 3))
KERNEL(k_shr64, (uint32_t)((((uint64_t)k << 32) | x) >> (x & 63)))
KERNEL(k_bitop3, (~(x | k) & 0x80808080u))
KERNEL(k_ffs, (uint32_t)__builtin_ctz(x | 0x80000000u) + x)

int main() {
    uint32_t* out;
    hipMalloc(&out, 4);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    struct {
        const char* n;
        void (*f)(uint32_t*, uint32_t, uint32_t);
    } ks[] = {{"v_add_u32", k_add},         {"v_mul_hi_u32", k_mulhi},
              {"v_dot4_u32_u8", k_udot4},   {"v_alignbyte_b32", k_alignbyte},
              {"v_lshrrev_b64", k_shr64},   {"v_bitop3", k_bitop3},
              {"v_ffbl+add", k_ffs}};
    for (auto& k : ks) {
        for (int rep = 0; rep < 2; ++rep) {
            hipEventRecord(a);
            hipLaunchKernelGGL(k.f, dim3(BLOCKS), dim3(THREADS), 0, 0, out, 1u, 7u);
            hipEventRecord(b);
            hipEventSynchronize(b);
            float ms = 0;
            hipEventElapsedTime(&ms, a, b);
            const double winst = (double)BLOCKS * THREADS / 64 * ITERS * CH;  // wave-instructions
            const double per_simd = winst / (cus * 4.0);
            if (rep) printf("%-18s %.3f ms  %.2f ns per wave-instr per SIMD\n", k.n, ms, ms * 1e6 / per_simd);
        }
    }
    return 0;
}
