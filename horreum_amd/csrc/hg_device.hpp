// hg_device.hpp — device helpers shared by the decode and encode kernels
// (gfx950 / CDNA4: 64-lane waves, 160 KiB LDS per CU).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/horreum_gpu.h"
#include "hg_err.hpp"

// Batched decode (hgk_decode_launch_multi) across calls on one context: the
// tables' control regions in two halves used in turn (cur / next, table i at
// off[i] in each), each call's pre-pass clearing next; cur_zero (nullable):
// bytes of each region of cur known to be zero (no zero kernel when they
// cover the call's); next_zero (out): bytes cleared per region of next.
// shadow (nullable): a host copy of what d_stage holds (shadow_bytes): the
// staging copy is skipped when the call's arguments are the same bytes;
// *copied (out) says whether it ran; stage_ev (nullable) is recorded right
// after it, so the host may reuse h_stage once the copy -- not the whole
// decode -- has passed.
struct hgk_multi_ctl {
    char* cur;
    char* next;
    const uint64_t* off;
    const uint64_t* cur_zero;
    uint64_t* next_zero;
    const void* shadow;
    uint64_t shadow_bytes;
    int* copied;
    hipEvent_t stage_ev;
};

// Compaction extras of a merge (hgk_merge_launch in hg_merge.hip).
// out non-null: records mode -- the last round writes the live records' bytes
// to out (cap bytes; rec_off, nullable: each record's output offset) and the
// encode result, no hg_pair array, no encode pass.  zero (nullable):
// zero_words words the defer-mode flag kernel clears for the encode that
// follows on the stream (its block sums; a memset launch fewer).
struct hgk_merge_records {
    uint8_t* out;
    uint64_t cap;
    uint64_t* rec_off;
    hg_encode_result* enc_result;
    uint64_t* zero;
    uint64_t zero_words;
    // (nullable) the encode's tile sums (enc_nt words) and group sums after
    // them, accumulated by the merge's last round: the encode then skips its
    // sums pass over the pairs.  Tiles of 2^enc_tile_log2 records, groups of
    // 2^enc_group_log2 tiles (hgk_encode_tile_geometry).
    uint64_t* enc_sums;
    uint64_t enc_nt, enc_words;
    uint32_t enc_tile_log2, enc_group_log2;
};
// hgk_merge_launch's done flags
constexpr int HGK_MERGE_EMITTED = 1;  // records mode wrote the records
constexpr int HGK_MERGE_ZEROED = 2;   // the flag kernel cleared rec->zero
constexpr int HGK_MERGE_SUMS = 4;     // the last round accumulated rec->enc_sums

namespace hgk {

constexpr uint64_t V40 = (1ull << 40) - 1;  // 40-bit positions/counts in status words


// Decode pieces and their pre-pass records (hg_decode.hip), shared with the
// merge's entry builder (hg_merge.hip), which takes key prefixes the decode
// pre-pass left in the span scratch of stride pieces (compaction mode).
constexpr uint32_t PIECE_BYTES = 16384;
constexpr uint32_t PIECE_RECS = PIECE_BYTES / 16;  // most records starting in a piece
struct SpecPiece {                // one per piece of an ok pre-pass batch
    uint64_t x, R;
    uint32_t kl, vl, count, pad;  // pad: SP_STRIDE, or SP_HOP (count spans in scratch)
};
enum : uint32_t { SP_STRIDE = 0, SP_HOP = 1 };

// Key prefix of a record as merge entries compare it: bytes [0, 16) of the
// key, big-endian, zero past klen; lo / hi = the key's first 16 bytes read
// little-endian (bytes past the key arbitrary).
__device__ __forceinline__ uint4 key_prefix_be(uint64_t lo, uint64_t hi, uint32_t kl) {
    if (kl < 8) lo &= kl ? (~0ull >> (64 - 8 * kl)) : 0ull;
    if (kl < 16) hi &= kl <= 8 ? 0ull : (~0ull >> (64 - 8 * (kl - 8)));
    const uint64_t p0 = __builtin_bswap64(lo), p1 = __builtin_bswap64(hi);
    return make_uint4((uint32_t)p0, (uint32_t)(p0 >> 32), (uint32_t)p1, (uint32_t)(p1 >> 32));
}

// Status word: [63:62] flag | [61:40] aux (22 bits) | [39:0] value (40 bits).
// Every word a look-back reads is written whole by ONE 8-byte agent-scope
// atomic store (a granule, cdna_hip_programming.md G16 R2), so a reader sees
// either the old or the new word, never a torn one.
__device__ __forceinline__ unsigned long long pack_status(uint32_t flag, uint32_t aux,
                                                          uint64_t val) {
    return ((unsigned long long)flag << 62) |
           ((unsigned long long)(aux & 0x3FFFFFu) << 40) | (val & V40);
}
__device__ __forceinline__ uint32_t st_flag(unsigned long long w) { return (uint32_t)(w >> 62); }
__device__ __forceinline__ uint32_t st_aux(unsigned long long w) {
    return (uint32_t)(w >> 40) & 0x3FFFFFu;
}
__device__ __forceinline__ uint64_t st_val(unsigned long long w) { return w & V40; }

__device__ __forceinline__ unsigned long long ld_agent(const unsigned long long* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_agent(unsigned long long* p, unsigned long long v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Per-byte zero mask of 16 bytes held as 4 dwords: bit i set <=> byte i == 0.
// The byte MSB flags of ~(((x & 0x7F..) + 0x7F..) | x) are gathered by one
// multiply: flags at bits 7, 15, 23, 31 times 2^25 + 2^18 + 2^11 + 2^4 land
// on bits 32..35 of the product and every other partial product on a
// distinct bit, so nothing carries (lane-walk decode: 5-8 % faster than
// shift-and-mask gathering, the masks being a large share of its VALU work).
// zflags: the 4 flags in bits 0..3, other partial products at bits 8-10, 16,
// 17 and 24 (left in place by zmask16: shifted by 8 or 12 they land at 16+).
__device__ __forceinline__ uint32_t zflags(uint32_t x) {
    const uint32_t t = ((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x;  // byte MSB set <=> byte != 0
    return __umulhi(~t & 0x80808080u, 0x02040810u);
}
__device__ __forceinline__ uint32_t zmask4(uint32_t x) { return zflags(x) & 0xFu; }
#ifndef HG_ZDOT
#define HG_ZDOT 1
#endif
// zmask16 by dot products (HG_ZDOT): the byte flags (0x80 or 0) of two dwords
// weighted 1, 2, 4, 8 and 16, 32, 64, 128 by two v_dot4_u32_u8 sum to 128 x the
// mask byte, so four dot products and two shifts replace four multiplies and
// their combining shifts.
__device__ __forceinline__ uint32_t zbyte_flags(uint32_t x) {
    return ~(((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x) & 0x80808080u;
}
#ifndef HG_ZADD64
#define HG_ZADD64 0  // A/B r6 (profiles/r6_ab_zmask_diag.log): mixed, within noise -- off
#endif
// zbyte_flags of two dwords with one 64-bit add (v_lshl_add_u64): the
// masked bytes are <= 0x7F, so no carry crosses a byte and the 64-bit sum is
// the two 32-bit ones.
__device__ __forceinline__ void zbyte_flags2(uint32_t x, uint32_t y, uint32_t& fx, uint32_t& fy) {
    const uint64_t w = ((uint64_t)y << 32) | x;
    const uint64_t t = (w & 0x7F7F7F7F7F7F7F7Full) + 0x7F7F7F7F7F7F7F7Full;
    // ~(t | x) & 0x80808080 as one v_bitop3 (truth table bit (t<<2 | x<<1 | c): only 0,0,1)
    fx = __builtin_amdgcn_bitop3_b32((uint32_t)t, x, 0x80808080u, 0x02);
    fy = __builtin_amdgcn_bitop3_b32((uint32_t)(t >> 32), y, 0x80808080u, 0x02);
}
__device__ __forceinline__ uint32_t zmask16(uint4 v) {
    if (HG_ZDOT && HG_ZADD64) {
        uint32_t fx, fy, fz, fw;
        zbyte_flags2(v.x, v.y, fx, fy);
        zbyte_flags2(v.z, v.w, fz, fw);
        const uint32_t lo = __builtin_amdgcn_udot4(
            fy, 0x80402010u, __builtin_amdgcn_udot4(fx, 0x08040201u, 0u, false), false);
        const uint32_t hi = __builtin_amdgcn_udot4(
            fw, 0x80402010u, __builtin_amdgcn_udot4(fz, 0x08040201u, 0u, false), false);
        return (lo >> 7) | (hi << 1);
    }
    if (HG_ZDOT) {
        const uint32_t lo = __builtin_amdgcn_udot4(
            zbyte_flags(v.y), 0x80402010u,
            __builtin_amdgcn_udot4(zbyte_flags(v.x), 0x08040201u, 0u, false), false);
        const uint32_t hi = __builtin_amdgcn_udot4(
            zbyte_flags(v.w), 0x80402010u,
            __builtin_amdgcn_udot4(zbyte_flags(v.z), 0x08040201u, 0u, false), false);
        return (lo >> 7) | (hi << 1);
    }
    return (((zflags(v.x) | (zflags(v.y) << 4)) & 0xFFu) | (zflags(v.z) << 8) |
            (zflags(v.w) << 12)) & 0xFFFFu;
}

// Unaligned little-endian u64 pair (klen, vlen) at byte offset p of an
// 8-byte-aligned LDS buffer; reads 24 bytes from p & ~7.
__device__ __forceinline__ void lds_header(const uint8_t* lds, uint32_t p, uint64_t& k,
                                           uint64_t& v) {
    const uint64_t* w = reinterpret_cast<const uint64_t*>(lds + (p & ~7u));
    uint64_t w0 = w[0], w1 = w[1], w2 = w[2];
    uint32_t s = (p & 7u) * 8u;
    if (s) {
        k = (w0 >> s) | (w1 << (64u - s));
        v = (w1 >> s) | (w2 << (64u - s));
    } else {
        k = w0;
        v = w1;
    }
}

// The same header as four 32-bit halves from five dword reads (always
// dword-aligned) and byte funnel shifts: fewer dependent operations on the
// serial walks' critical path than the 64-bit form (reads 20 bytes from p & ~3).
__device__ __forceinline__ void lds_header32(const uint8_t* lds, uint32_t p, uint32_t& k0,
                                             uint32_t& k1, uint32_t& v0, uint32_t& v1) {
    const uint32_t* w = reinterpret_cast<const uint32_t*>(lds + (p & ~3u));
    const uint32_t a0 = w[0], a1 = w[1], a2 = w[2], a3 = w[3], a4 = w[4];
    const uint32_t sh = p & 3u;
    k0 = __builtin_amdgcn_alignbyte(a1, a0, sh);
    k1 = __builtin_amdgcn_alignbyte(a2, a1, sh);
    v0 = __builtin_amdgcn_alignbyte(a3, a2, sh);
    v1 = __builtin_amdgcn_alignbyte(a4, a3, sh);
}

// The low halves of klen and vlen only (four dword reads): for positions whose
// high words are known to be zero.
__device__ __forceinline__ void lds_kv32(const uint8_t* lds, uint32_t p, uint32_t& k0,
                                         uint32_t& v0) {
    const uint32_t* w = reinterpret_cast<const uint32_t*>(lds + (p & ~3u));
    const uint32_t sh = p & 3u;
    k0 = __builtin_amdgcn_alignbyte(w[1], w[0], sh);
    v0 = __builtin_amdgcn_alignbyte(w[3], w[2], sh);
}

// Wave-level inclusive max / sum scans over u32 by DPP (row shifts 1, 2, 4, 8
// inside each 16-lane row, then the row totals by row_bcast 15 / 31): six
// VALU steps, no LDS round trips (a __shfl_up chain is six ds_bpermutes).
__device__ __forceinline__ uint32_t dpp_max_incl(uint32_t v) {
#define HG_DPP_MAX(ctrl, rmask) \
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, ctrl, rmask, 0xf, false))
    HG_DPP_MAX(0x111, 0xf);
    HG_DPP_MAX(0x112, 0xf);
    HG_DPP_MAX(0x114, 0xf);
    HG_DPP_MAX(0x118, 0xf);
    HG_DPP_MAX(0x142, 0xa);
    HG_DPP_MAX(0x143, 0xc);
#undef HG_DPP_MAX
    return v;
}
__device__ __forceinline__ uint32_t dpp_sum_incl(uint32_t v) {
#define HG_DPP_ADD(ctrl, rmask) \
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, ctrl, rmask, 0xf, false)
    HG_DPP_ADD(0x111, 0xf);
    HG_DPP_ADD(0x112, 0xf);
    HG_DPP_ADD(0x114, 0xf);
    HG_DPP_ADD(0x118, 0xf);
    HG_DPP_ADD(0x142, 0xa);
    HG_DPP_ADD(0x143, 0xc);
#undef HG_DPP_ADD
    return v;
}

// Wave-level inclusive scan (64 lanes).
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t x) {
    const uint32_t lane = threadIdx.x & 63u;
#pragma unroll
    for (uint32_t d = 1; d < 64; d <<= 1) {
        uint32_t y = __shfl_up(x, d, 64);
        if (lane >= d) x += y;
    }
    return x;
}

template <typename T>
__device__ __forceinline__ T wave_sum(T x) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) x += __shfl_xor(x, d, 64);
    return x;
}

// Block-wide exclusive scan over NW waves; s_tmp needs NW words.
template <uint32_t NW>
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t* s_tmp,
                                                    uint32_t& total) {
    const uint32_t lane = threadIdx.x & 63u, wid = threadIdx.x >> 6;
    uint32_t inc = wave_incl_scan(v);
    if (lane == 63) s_tmp[wid] = inc;
    __syncthreads();
    uint32_t pre = 0, tot = 0;
#pragma unroll
    for (uint32_t w = 0; w < NW; ++w) {
        uint32_t t = s_tmp[w];
        pre += (w < wid) ? t : 0u;
        tot += t;
    }
    __syncthreads();
    total = tot;
    return pre + inc - v;
}

}  // namespace hgk
