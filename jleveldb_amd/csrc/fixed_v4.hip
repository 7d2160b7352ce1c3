// fixed_v4.hip — "v4" fast path for contiguous 4 KiB blocks (configs C2/C4).
//
// Layout.  A wave processes R = 64/LPB blocks per "round": lanes
// L = LPB*q + l' (q = block of the round, l' = 0..LPB-1) read block q with one
// 16-byte buffer_load_dwordx4 per step, lane l' taking bytes
// [STEP*k + 16*l', +16) of step k (STEP = 16*LPB bytes; for LPB = 8 one full
// 128-B cache line per block and instruction, 1 KiB per wave-instruction).
// Dword j of a lane's 16 bytes feeds chain j (4 independent chains per lane):
// chain (l', j) sees 4 data bytes and then STEP-4 bytes that other chains own,
// so its step is a slicing-by-4 update through the gap tables
// G_t = z^(STEP-4+t)∘T0 (region A of the v4 image, same bank-conflict-free
// addressing as the 4 KiB kernel of jlcrc_kernels.hip).  After the last step
// chain (l', j) sits 16*l' + 4*j bytes past the end of the block; the four
// chains are folded with the wave-uniform maps z^-4, z^-8, z^-12 (nibble
// tables, 16 entries in 16 distinct banks: conflict-free without replication),
// the lane with z^-(16 l') (per-lane nibble tables, one copy per bank) and the
// LPB lanes of a block XOR-reduced with DPP.
//
// Compared with crc_fixed4k_x2_kernel (one 4-B dword per lane per step, one
// block per wave): 4x fewer load instructions, and the per-block epilogue
// (re-alignment, reduction, result) is shared by R blocks per instruction.
//
// Pipeline.  The loads are inline-asm buffer_load_dwordx4 … nt through a
// buffer resource per round (num_records = the bytes of the round that exist:
// reads past the last block return zeros, so ragged tails need no predication).
// A register ring of P slots keeps P KiB in flight per wave: step k consumes
// slot k % P after s_waitcnt vmcnt(P-2) and immediately refills it with step
// k + P (of this round or the next), so the HBM stream never drains, including
// across the epilogue and group boundaries.  The product instantiation is P = 8
// slots at 1024 threads (16 waves per CU: 128 KiB in flight per CU; shape 3
// below); the 16-slot ring at 512 threads survives as a study shape.  vmcnt is
// conservative by one so that the one result store per group (vmcnt counts
// stores on gfx9) can never be mistaken for a completed load.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <utility>

#include "engine_device.hpp"


namespace jlk {

constexpr int kFxRingSlack = 2;  // ring waits vmcnt(P - 2): see general_v4.hip's JL_RING_SLACK

typedef uint32_t v4u __attribute__((ext_vector_type(4)));
typedef int32_t v4i __attribute__((ext_vector_type(4)));

// gfx9 raw buffer resource: 48-bit base, stride 0, num_records in bytes
// (dword 3 as CK uses for gfx9: DATA_FORMAT 32, no swizzle).
__device__ __forceinline__ v4i make_rsrc(uint64_t base, uint32_t nbytes) {
    v4i r;
    r.x = (int32_t)(uint32_t)base;
    r.y = (int32_t)((uint32_t)(base >> 32) & 0xffffu);
    r.z = (int32_t)nbytes;
    r.w = 0x00020000;
    return r;
}

template <int LPB, int RING = 16>
struct V4Geom {
    static constexpr int STEP = 16 * LPB;   // bytes of one block-step
    static constexpr int S = 4096 / STEP;   // steps per block
    static constexpr int R = 64 / LPB;      // blocks per round
    static constexpr int P = RING;          // ring slots = prefetch distance in steps
    static_assert(S % P == 0 || P % S == 0, "ring must tile the round");
    static_assert(S >= P, "at least one ring of steps per round");
};

template <int LPB, bool NT, int RING>
struct V4Wave {
    using Gm = V4Geom<LPB, RING>;
    const uint32_t *lds;
    GLanes gl;
    uint32_t voff, lc, s_init, zero;
    v4u w[Gm::P];
    uint32_t x0, x1, x2, x3;  // chain states (x-form: state ^ pending data word)
    v4i cur, nxt;             // resources of this round and the next (prefetch side)

    __device__ __forceinline__ explicit V4Wave(const uint32_t *l, uint32_t lane) : lds(l), gl(lane) {
        asm volatile("v_mov_b32 %0, 0" : "=v"(zero));
    }

    template <int OFF>
    __device__ __forceinline__ void load(v4u &dst, const v4i &rs) {
        if (NT)
            asm volatile("buffer_load_dwordx4 %0, %1, %2, 0 offen offset:%3 nt"
                         : "+v"(dst) : "v"(voff), "s"(rs), "n"(OFF) : "memory");
        else
            asm volatile("buffer_load_dwordx4 %0, %1, %2, 0 offen offset:%3"
                         : "+v"(dst) : "v"(voff), "s"(rs), "n"(OFF) : "memory");
    }

    // the prologue: steps 0..P-1 of the first round
    template <int K>
    __device__ __forceinline__ void prime() {
        load<K * Gm::STEP>(w[K], cur);
    }
    template <int... K>
    __device__ __forceinline__ void prime_all(std::integer_sequence<int, K...>) {
        (prime<K>(), ...);
    }

    template <int K>
    __device__ __forceinline__ void step() {
        constexpr int SL = K % Gm::P;
        asm volatile("s_waitcnt vmcnt(%1)" : "+v"(w[SL]) : "n"(Gm::P - kFxRingSlack));
        if (K == 0) {  // real XORs (zero is opaque): a plain copy here lets RA copy the ring slot before its wait
            x0 = s_init ^ w[SL].x;
            x1 = zero ^ w[SL].y;
            x2 = zero ^ w[SL].z;
            x3 = zero ^ w[SL].w;
        } else {
            x0 = gstep_x3(lds, x0, gl, w[SL].x);
            x1 = gstep_x3(lds, x1, gl, w[SL].y);
            x2 = gstep_x3(lds, x2, gl, w[SL].z);
            x3 = gstep_x3(lds, x3, gl, w[SL].w);
        }
        if (K + Gm::P < Gm::S) load<(K + Gm::P) * Gm::STEP>(w[SL], cur);
        else load<(K + Gm::P - Gm::S) * Gm::STEP>(w[SL], nxt);
    }
    template <int... K>
    __device__ __forceinline__ void round(std::integer_sequence<int, K...>) {
        (step<K>(), ...);
    }

    // crc of this lane's block after the round (valid in every lane of the block)
    __device__ __forceinline__ uint32_t finish() {
        const uint32_t s0 = gstep_x3(lds, x0, gl, 0u), s1 = gstep_x3(lds, x1, gl, 0u);
        const uint32_t s2 = gstep_x3(lds, x2, gl, 0u), s3 = gstep_x3(lds, x3, gl, 0u);
        const uint32_t c = xor3(s0, ushift(lds, s1, kV4U4Byte), ushift(lds, s2, kV4U4Byte + 512u)) ^
                           ushift(lds, s3, kV4U4Byte + 1024u);
        return ~group_xor<LPB>(realign(lds, c, lc));
    }
};

template <int LPB, bool NT, int RING = 16, int THREADS = 1024>
__global__ __launch_bounds__(THREADS) void crc_fixed4k_v4_kernel(const uint4 *__restrict__ img,
                                                                 const uint8_t *__restrict__ data, uint64_t n_blocks,
                                                                 uint32_t flags, uint32_t *__restrict__ out) {
    using Gm = V4Geom<LPB, RING>;
    __shared__ uint32_t lds[kImageBytes / 4];
    load_image(lds, img);
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = threadIdx.x >> 6;
    const uint64_t waves = (uint64_t)gridDim.x * (blockDim.x >> 6);
    uint64_t g = uni64((uint64_t)blockIdx.x * (blockDim.x >> 6) + wave);  // group of 64 blocks
    if (g * 64u >= n_blocks) return;
    uint32_t *slot = lds + kV4SlotDword + wave * 64u;
    const uint64_t dbase = (uint64_t)(uintptr_t)data;
    const uint32_t do_mask = flags & 1u;

    V4Wave<LPB, NT, RING> W(lds, lane);
    W.voff = (lane / LPB) * 4096u + (lane % LPB) * 16u;
    W.lc = 131072u | ((lane & 31u) << 2);
    W.s_init = (lane % LPB == 0) ? 0xffffffffu : 0u;

    // prefetch cursor: group pg, round pr (first block pg*64 + pr*R)
    uint64_t pg = g;
    uint32_t pr = 0;
    auto rsrc = [&](uint64_t gg, uint32_t rr) -> v4i {
        const uint64_t b = gg * 64u + (uint64_t)rr * Gm::R;
        if (b >= n_blocks) return make_rsrc(dbase, 0u);
        const uint64_t nb = n_blocks - b < (uint64_t)Gm::R ? n_blocks - b : (uint64_t)Gm::R;
        return make_rsrc(dbase + b * 4096u, (uint32_t)(nb * 4096u));
    };
    auto adv = [&](uint64_t &gg, uint32_t &rr) {
        if (++rr == (uint32_t)LPB || gg * 64u + (uint64_t)rr * Gm::R >= n_blocks) {
            rr = 0;
            gg += waves;
        }
    };
    W.cur = rsrc(pg, pr);
    adv(pg, pr);
    W.nxt = rsrc(pg, pr);
    W.prime_all(std::make_integer_sequence<int, Gm::P>());

    uint32_t r = 0;  // round within the group
    for (;;) {
        W.round(std::make_integer_sequence<int, Gm::S>());
        // rotate the prefetch resources: the next round's loads already use nxt
        W.cur = W.nxt;
        adv(pg, pr);
        W.nxt = rsrc(pg, pr);
        uint32_t crc = W.finish();
        if (do_mask) crc = mask_crc(crc);
        if (lane % LPB == 0) slot[r * Gm::R + lane / LPB] = crc;
        const uint64_t g0 = g * 64u;
        if (++r == (uint32_t)LPB || g0 + (uint64_t)r * Gm::R >= n_blocks) {
            const uint32_t res = slot[lane];
            if (g0 + lane < n_blocks) out[g0 + lane] = res;
            r = 0;
            g += waves;
            if (g * 64u >= n_blocks) break;
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the ring's trailing (zero-range) loads
}

hipError_t launch_fixed4k_v4(const void *img, const uint8_t *data, uint64_t n_blocks, uint32_t flags, uint32_t *out,
                             int grid, hipStream_t st) {
    // the product kernel: 8 lanes per block, nt loads, 8-slot ring, 1024 threads
    // (r1 sustained A/B: 0.638 ms vs 0.643 for the 16-slot ring, 0.654 at 512 threads;
    // the other shapes live on the branch study-superseded-kernels)
    hipLaunchKernelGGL((crc_fixed4k_v4_kernel<8, true, 8, 1024>), dim3(grid), dim3(1024), 0, st,
                       (const uint4 *)img, data, n_blocks, flags, out);
    return hipGetLastError();
}

}  // namespace jlk

