// Streaming-read probe for the decode access pattern (not part of the product).
// Each workgroup (256 threads) streams batches of PIECES x 16 KiB: register
// prefetch of the next piece, LDS staging of the current one, a trivial LDS
// pass; LDS padding sets workgroups per CU.  Prints GB/s per configuration.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <stdint.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

template <int GPT, int PAD_KB, bool LDS_STAGE>
__global__ __launch_bounds__(256) void stream_kernel(const uint8_t* src, uint64_t len, uint32_t pieces_per_batch,
                                                     uint32_t nbatches, uint32_t* ticket, unsigned long long* out) {
    constexpr uint32_t PIECE = GPT * 256 * 16;
    __shared__ u32x4 lds[PIECE / 16 + PAD_KB * 64];
    __shared__ uint32_t sb;
    const uint32_t tid = threadIdx.x;
    if (tid == 0) sb = atomicAdd(ticket, 1u);
    __syncthreads();
    const uint32_t b = sb;
    if (b >= nbatches) return;
    const uint64_t base = (uint64_t)b * pieces_per_batch * PIECE;
    u32x4 v[GPT];
    uint32_t acc = 0;
#pragma unroll
    for (int i = 0; i < GPT; ++i) v[i] = *reinterpret_cast<const u32x4*>(src + base + (i * 256 + tid) * 16);
    for (uint32_t p = 0; p < pieces_per_batch; ++p) {
        if (LDS_STAGE) {
            __syncthreads();
#pragma unroll
            for (int i = 0; i < GPT; ++i) lds[i * 256 + tid] = v[i];
            __syncthreads();
        } else {
#pragma unroll
            for (int i = 0; i < GPT; ++i) acc ^= v[i].x ^ v[i].y ^ v[i].z ^ v[i].w;
        }
        {  // unconditional (clamped) prefetch keeps v in registers
            const uint64_t nb = base + (uint64_t)min(p + 1, pieces_per_batch - 1) * PIECE;
#pragma unroll
            for (int i = 0; i < GPT; ++i) v[i] = *reinterpret_cast<const u32x4*>(src + nb + (i * 256 + tid) * 16);
        }
        if (LDS_STAGE) {
            const u32x4 a = lds[(tid * 7 + p) % (PIECE / 16)];
            acc ^= a.x ^ a.w;
        }
    }
    if (acc == 0x12345678u) out[0] = acc;  // keep the loads alive
}

template <int GPT, int PAD_KB, bool LDS_STAGE>
void run(const uint8_t* d, uint64_t len, uint32_t ppb, uint32_t* ticket, unsigned long long* out, const char* name) {
    constexpr uint32_t PIECE = GPT * 256 * 16;
    const uint64_t batch_bytes = (uint64_t)ppb * PIECE;
    const uint32_t nbatches = (uint32_t)(len / batch_bytes);
    int occ = 0;
    CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, stream_kernel<GPT, PAD_KB, LDS_STAGE>, 256, 0));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    float best = 1e9f;
    for (int r = 0; r < 6; ++r) {
        CHECK(hipMemset(ticket, 0, 4));
        CHECK(hipEventRecord(e0));
        stream_kernel<GPT, PAD_KB, LDS_STAGE><<<nbatches, 256>>>(d, len, ppb, nbatches, ticket, out);
        CHECK(hipEventRecord(e1));
        CHECK(hipEventSynchronize(e1));
        float ms;
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        if (r > 0 && ms < best) best = ms;
    }
    printf("%-28s piece=%6u KiB ppb=%3u occ/CU=%2d  %.4f ms  %.0f GB/s\n", name, PIECE / 1024, ppb, occ, best,
           (double)nbatches * batch_bytes / best / 1e6);
}

int main() {
    const uint64_t len = 1ull << 30;
    uint8_t* d;
    uint32_t* ticket;
    unsigned long long* out;
    CHECK(hipMalloc(&d, len));
    CHECK(hipMalloc(&ticket, 4));
    CHECK(hipMalloc(&out, 8));
    CHECK(hipMemset(d, 1, len));
    run<4, 0, true>(d, len, 16, ticket, out, "lds gpt4 pad0");
    run<4, 10, true>(d, len, 16, ticket, out, "lds gpt4 pad10 (~26KB)");
    run<4, 24, true>(d, len, 16, ticket, out, "lds gpt4 pad24 (~40KB)");
    run<4, 0, true>(d, len, 8, ticket, out, "lds gpt4 pad0");
    run<4, 0, true>(d, len, 64, ticket, out, "lds gpt4 pad0");
    run<8, 0, true>(d, len, 8, ticket, out, "lds gpt8 pad0");
    run<4, 0, false>(d, len, 16, ticket, out, "regs gpt4");
    run<8, 0, false>(d, len, 8, ticket, out, "regs gpt8");
    run<16, 0, false>(d, len, 4, ticket, out, "regs gpt16");
    return 0;
}
