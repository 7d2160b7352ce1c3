// engine_device.hpp — device-side building blocks shared by every engine
// kernel (jlcrc_kernels.hip, stream_kernel.hip): LDS table addressing, the
// gap-table chain step, lane re-alignment, wave reductions and the scalar
// (SMEM) helpers.  Algebra and LDS layout: crc_math.hpp and DESIGN.md §3.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "jlcrc_kernels.hpp"

namespace jlk {

typedef uint32_t __attribute__((aligned(1))) u32u;  // unaligned dword (unaligned mode is on under KFD)

__device__ __forceinline__ uint32_t lds_at(const uint32_t *lds, uint32_t byte_addr) {
    return *(const uint32_t *)((const char *)lds + byte_addr);
}

// Per-lane constant bytes of the four G lookups (crc_math.hpp, region A):
// byte 0 = (t&1)<<7 | 4*(lane&31), byte 2 = t>>1; byte k of x is G_{3-k}.
struct GLanes {
    uint32_t l3, l2, l1, l0;
    __device__ __forceinline__ explicit GLanes(uint32_t lane) {
        const uint32_t l4 = (lane & 31u) << 2;
        l3 = 0x10000u | 0x80u | l4;  // G3: region 1, odd half
        l2 = 0x10000u | l4;          // G2: region 1, even half
        l1 = 0x80u | l4;             // G1: region 0, odd half
        l0 = l4;                     // G0: region 0, even half
    }
};

// v_perm_b32(S0 = lane constant, S1 = x): D.b0 = S0.b0, D.b1 = x.b[k], D.b2 = S0.b2, D.b3 = 0
#define JL_GADDR(L, x, k) __builtin_amdgcn_perm((L), (x), 0x0C060004u | ((k) << 8))

// One chain step: returns G3[x.b0] ^ G2[x.b1] ^ G1[x.b2] ^ G0[x.b3]
// (4 v_perm_b32 + 4 ds_read_b32, bank-conflict-free).
__device__ __forceinline__ uint32_t gstep(const uint32_t *lds, uint32_t x, const GLanes &g) {
    uint32_t v0 = lds_at(lds, JL_GADDR(g.l3, x, 0u));
    uint32_t v1 = lds_at(lds, JL_GADDR(g.l2, x, 1u));
    uint32_t v2 = lds_at(lds, JL_GADDR(g.l1, x, 2u));
    uint32_t v3 = lds_at(lds, JL_GADDR(g.l0, x, 3u));
    return (v0 ^ v1) ^ (v2 ^ v3);
}

// Re-alignment of lane l's chain by z^-(4l): 8 nibble lookups in region B.
// lc = 131072 | ((lane>>5) << 14) | 4*(lane&31).
__device__ __forceinline__ uint32_t realign(const uint32_t *lds, uint32_t r, uint32_t lc) {
    uint32_t c0 = lds_at(lds, (((r << 7) & 0x780u) | lc) + 0u * 2048u);
    uint32_t c1 = lds_at(lds, (((r << 3) & 0x780u) | lc) + 1u * 2048u);
    uint32_t c2 = lds_at(lds, (((r >> 1) & 0x780u) | lc) + 2u * 2048u);
    uint32_t c3 = lds_at(lds, (((r >> 5) & 0x780u) | lc) + 3u * 2048u);
    uint32_t c4 = lds_at(lds, (((r >> 9) & 0x780u) | lc) + 4u * 2048u);
    uint32_t c5 = lds_at(lds, (((r >> 13) & 0x780u) | lc) + 5u * 2048u);
    uint32_t c6 = lds_at(lds, (((r >> 17) & 0x780u) | lc) + 6u * 2048u);
    uint32_t c7 = lds_at(lds, (((r >> 21) & 0x780u) | lc) + 7u * 2048u);
    return ((c0 ^ c1) ^ (c2 ^ c3)) ^ ((c4 ^ c5) ^ (c6 ^ c7));
}

// XOR of all 64 lanes, returned as a wave-uniform (SGPR) value.
__device__ __forceinline__ uint32_t wave_xor(uint32_t v) {
    v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xf, 0xf, true);   // quad_perm [1,0,3,2]
    v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xf, 0xf, true);   // quad_perm [2,3,0,1]
    v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x124, 0xf, 0xf, true);  // row_ror:4
    v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x128, 0xf, 0xf, true);  // row_ror:8
    uint32_t a = (uint32_t)__builtin_amdgcn_readlane((int)v, 0);
    uint32_t b = (uint32_t)__builtin_amdgcn_readlane((int)v, 16);
    uint32_t c = (uint32_t)__builtin_amdgcn_readlane((int)v, 32);
    uint32_t d = (uint32_t)__builtin_amdgcn_readlane((int)v, 48);
    return (a ^ b) ^ (c ^ d);
}

__device__ __forceinline__ uint32_t uni(uint32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)v); }
__device__ __forceinline__ uint64_t uni64(uint64_t v) {
    uint32_t lo = uni((uint32_t)v), hi = uni((uint32_t)(v >> 32));
    return ((uint64_t)hi << 32) | lo;
}

__device__ __forceinline__ uint32_t mask_crc(uint32_t crc) { return ((crc >> 15) | (crc << 17)) + 0xa282ead8u; }
__device__ __forceinline__ uint32_t unmask_crc(uint32_t m) {  // J/util/Crc32C.java:72-75
    const uint32_t r = m - 0xa282ead8u;
    return (r >> 17) | (r << 15);
}

__device__ __forceinline__ void load_image(uint32_t *lds, const uint4 *__restrict__ img) {
    uint4 *d = (uint4 *)lds;
    for (uint32_t i = threadIdx.x; i < kImageBytes / 16; i += blockDim.x) d[i] = img[i];
    __syncthreads();
}

// 3-input XOR in one issue slot: gfx950's v_bitop3_b32 with truth table 0x96
// (the compiler does not form it on its own from a ^ b ^ c).
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

// Four G lookups of x, XOR-folded together with `w` (the next step's data word
// or 0): 4 v_perm_b32 + 4 ds_read_b32 + 2 v_bitop3_b32 per step instead of
// 1 + 4 + 3 separate XORs.
__device__ __forceinline__ uint32_t gstep_x3(const uint32_t *lds, uint32_t x, const GLanes &g, uint32_t w) {
    uint32_t v0 = lds_at(lds, JL_GADDR(g.l3, x, 0u));
    uint32_t v1 = lds_at(lds, JL_GADDR(g.l2, x, 1u));
    uint32_t v2 = lds_at(lds, JL_GADDR(g.l1, x, 2u));
    uint32_t v3 = lds_at(lds, JL_GADDR(g.l0, x, 3u));
    return xor3(xor3(v0, v1, v2), v3, w);
}

// Scalar (SMEM) load of a wave-uniform address: goes through the scalar cache
// and lgkmcnt, so it never perturbs the hand-counted vmcnt pipeline.
__device__ __forceinline__ uint32_t sload(const void *p) {
    uint32_t v;
    asm volatile("s_load_dword %0, %1, 0x0\n\ts_waitcnt lgkmcnt(0)" : "=s"(v) : "s"(p) : "memory");
    return v;
}
__device__ __forceinline__ uint32_t saux(const uint32_t *aux, uint32_t idx) { return sload(aux + uni(idx)); }

// byte i of a byte array through its aligned dword (scalar load)
__device__ __forceinline__ uint32_t sbyte(const uint8_t *__restrict__ a, uint64_t i) {
    const uint64_t addr = uni64((uint64_t)(uintptr_t)(a + i));
    const uint32_t wv = sload((const void *)(uintptr_t)(addr & ~(uint64_t)3));
    return (wv >> (8 * (addr & 3))) & 0xffu;
}

__device__ __forceinline__ uint64_t sload64(const void *p) {
    uint64_t v;
    asm volatile("s_load_dwordx2 %0, %1, 0x0\n\ts_waitcnt lgkmcnt(0)" : "=s"(v) : "s"(p) : "memory");
    return v;
}

// Uniform shift z^-d through 8 nibble tables at LDS byte `base` (16 dwords each).
__device__ __forceinline__ uint32_t ushift(const uint32_t *lds, uint32_t c, uint32_t base) {
    uint32_t a0 = lds_at(lds, base + 0 * 64 + ((c << 2) & 0x3cu));
    uint32_t a1 = lds_at(lds, base + 1 * 64 + ((c >> 2) & 0x3cu));
    uint32_t a2 = lds_at(lds, base + 2 * 64 + ((c >> 6) & 0x3cu));
    uint32_t a3 = lds_at(lds, base + 3 * 64 + ((c >> 10) & 0x3cu));
    uint32_t a4 = lds_at(lds, base + 4 * 64 + ((c >> 14) & 0x3cu));
    uint32_t a5 = lds_at(lds, base + 5 * 64 + ((c >> 18) & 0x3cu));
    uint32_t a6 = lds_at(lds, base + 6 * 64 + ((c >> 22) & 0x3cu));
    uint32_t a7 = lds_at(lds, base + 7 * 64 + ((c >> 26) & 0x3cu));
    return xor3(xor3(a0, a1, a2), xor3(a3, a4, a5), a6 ^ a7);
}

// XOR over each aligned group of LPB lanes (DPP, result in every lane of the group).
template <int LPB>
__device__ __forceinline__ uint32_t group_xor(uint32_t v) {
    v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xf, 0xf, true);  // quad_perm [1,0,3,2]
    v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xf, 0xf, true);  // quad_perm [2,3,0,1]
    if (LPB >= 8) v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x141, 0xf, 0xf, true);  // row_half_mirror
    if (LPB >= 16) v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x140, 0xf, 0xf, true);  // row_mirror
    return v;
}

}  // namespace jlk
