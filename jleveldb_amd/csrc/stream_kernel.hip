// stream_kernel.hip — the general-path engine kernel (arbitrary block lengths,
// alignment, per-block init/suffix, and the caller-shim epilogues).  Compiled
// once per mode (-DJL_MODE=k, Makefile) so the instantiations build in parallel.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "engine_device.hpp"

#ifndef JL_MODE
#error "compile with -DJL_MODE=<jlk::MODE_*>"
#endif

namespace jlk {

// ---------------------------------------------------------------------------
// Stream kernel: arbitrary blocks (lengths, alignment, per-block init/suffix)
// and the caller-shim epilogues, with NO padding work.
//
// A wave owns a contiguous range of blocks [b_begin, b_end) (byte-balanced
// when the caller passes a partition) and turns it into a stream of "entries":
// every block of n bytes contributes K = ceil(n/256) 256-B steps of the
// end-aligned view (as in the fixed kernel: lane l holds the dword at virtual
// offset 256k + 4l, f = 256K - n zero bytes in front), preceded by one "extra"
// entry when the block needs bytes outside its steps (stored crc of a verify
// mode, or the bytes of a block shorter than 4 B).  Each entry is ONE
// wave-wide dword load into a P-deep register ring: the loop consumes ring slot
// u (s_waitcnt vmcnt(P-1)) and refills it with the entry P ahead, so exactly
// P-1 loads are always in flight behind the one being consumed, across block
// boundaries, whatever the block sizes.  Steps k >= 1 load through an SGPR base
// (no address VALU); the first step and extra entries use per-lane addresses.
//
// Seeding needs no state shift: W = slice4^-1(~init) (crc_math.hpp) is fed as
// the 4 data bytes just before the block, i.e. lane l0-1 gets W << 8r and the
// straddling lane l0 gets (first real bytes << 8r) | W >> (32-8r), with
// l0 = f>>2, r = f&3 (l0 == 0: lane 63 starts from one gap step of W << 8r).
// ---------------------------------------------------------------------------

struct SDesc {
    uint64_t ptr;  // first byte
    uint32_t n;    // bytes covered by the crc
    uint32_t K;    // 256-B steps
    uint32_t f;    // 256K - n
    uint32_t ex;   // 1: an extra entry precedes the steps
    uint32_t bad;  // 1: the block lies outside the caller's base_bytes (nothing read, result 0)
};

template <int MODE>
__device__ __forceinline__ SDesc stream_desc(const KParams &P, uint64_t i) {
    SDesc d;
    uint64_t off;
    uint32_t n;
    if (P.off) {
        off = sload64((const void *)(uintptr_t)uni64((uint64_t)(uintptr_t)(P.off + i)));
        n = sload((const void *)(uintptr_t)uni64((uint64_t)(uintptr_t)(P.len + i))) + P.len_add;
    } else {
        off = i * P.fixed_bytes;
        n = (uint32_t)P.fixed_bytes;
    }
    d.bad = block_in_range(P, off, n) ? 0u : 1u;
    if (d.bad) n = 0u;
    d.ptr = (uint64_t)(uintptr_t)P.base + off;
    d.n = n;
    d.K = (n + 255u) >> 8;
    d.f = (d.K << 8) - n;
    d.ex = (n > 0u && (n < 4u || MODE == MODE_TABLE_VERIFY || MODE == MODE_LOG_VERIFY)) ? 1u : 0u;
    return d;
}

// init of block i (Crc32C.extend's initCrc; 0 for value())
template <int MODE>
__device__ __forceinline__ uint32_t stream_init(const KParams &P, uint64_t i) {
    if (MODE == MODE_LOG_HEADER) return saux(P.aux, 512 + sbyte(P.type, i) % 5u);
    if (P.init) return sload((const void *)(uintptr_t)uni64((uint64_t)(uintptr_t)(P.init + i)));
    return 0u;
}

// seed word W = slice4^-1(~init) of block i
template <int MODE>
__device__ __forceinline__ uint32_t stream_seed(const KParams &P, uint64_t i) {
    if (MODE == MODE_LOG_HEADER) return saux(P.aux, 520 + sbyte(P.type, i) % 5u);
    if (P.init) {
        const uint32_t y = ~stream_init<MODE>(P, i);
        return saux(P.aux, 528 + (y & 0xffu)) ^ saux(P.aux, 784 + ((y >> 8) & 0xffu)) ^
               saux(P.aux, 1040 + ((y >> 16) & 0xffu)) ^ saux(P.aux, 1296 + (y >> 24));
    }
    return saux(P.aux, 525);
}

template <int MODE>
__device__ __forceinline__ uint32_t stream_suffix(const KParams &P, uint64_t i) {
    if (MODE == MODE_TRAILER) return 0x100u | (P.type ? sbyte(P.type, i) : 0u);
    if (P.suffix) return 0x100u | sbyte(P.suffix, i);
    return 0u;
}

__device__ __forceinline__ void ld_sbase(uint32_t &dst, uint64_t base, uint32_t voff) {
    // sb is usually produced by v_readfirstlane (a VALU SGPR write): a VMEM read of
    // that SGPR needs 5 wait states, and the compiler's hazard recognizer does not
    // look inside inline asm (r1: without the s_nop the load used a stale base)
    const uint64_t sb = uni64(base);
    asm volatile("s_nop 4\n\tglobal_load_dword %0, %1, %2" : "=v"(dst) : "v"(voff), "s"(sb) : "memory");
}
__device__ __forceinline__ void ld_vaddr(uint32_t &dst, uint64_t addr) {
    asm volatile("global_load_dword %0, %1, off" : "=v"(dst) : "v"(addr) : "memory");
}

// Prefetch cursor.  All state is wave-uniform (SGPRs).  The common case — a
// step k >= 1 of the current block — is "plain": bump the SGPR base by 256 and
// issue one SGPR-based load (a few SALU, no VALU, no branch but the counter
// test).  Everything else (extra entry, first step with per-lane addresses,
// moving to the next block and its descriptor) is the rare path, taken
// ex + 1 times per block.
template <int MODE, bool DBG>
struct StreamPF {
    uint64_t b, b_end;  // current block, range end
    SDesc d;            // descriptor of b
    uint64_t base;      // next plain step's base address - 256
    uint32_t plain;     // plain steps left in b
    uint32_t stage;     // 0: extra entry next, 1: first step next, 2: block done
    __device__ __forceinline__ void load_block(const KParams &P) {  // b -> next block with entries (or b_end)
        while (b < b_end) {
            d = stream_desc<MODE>(P, b);
            if (d.K + d.ex) {
                stage = d.ex ? 0u : 1u;
                return;
            }
            b++;
        }
    }
    __device__ __forceinline__ uint64_t check(const KParams &P, uint64_t a, uint32_t lane) const {
        const uint64_t zp = (uint64_t)(uintptr_t)P.zero;
        if ((a >= P.dbg_lo && a + 4 <= P.dbg_hi) || (a >= zp && a + 4 <= zp + 4096)) return a;
        const unsigned long long slot = atomicAdd(P.dbg, 1ull);
        if (slot < 256) {
            P.dbg[1 + 4 * slot] = b;
            P.dbg[2 + 4 * slot] = stage;
            P.dbg[3 + 4 * slot] = lane;
            P.dbg[4 + 4 * slot] = a;
        }
        return zp + 4u * lane;
    }
    __device__ __forceinline__ void rare(uint32_t &dst, const KParams &P, uint32_t lane) {
        const uint64_t zp = (uint64_t)(uintptr_t)P.zero;
        if (stage == 2u) {
            b++;
            load_block(P);
        }
        uint64_t a = zp + lane * 4u;
        if (b < b_end) {
            if (stage == 0u) {  // extra: lane 0 = stored crc, lanes 1-2 = aligned dwords of a block < 4 B
                if (lane == 0u && MODE == MODE_TABLE_VERIFY) a = d.ptr + d.n;  // trailer crc after block || type
                if (lane == 0u && MODE == MODE_LOG_VERIFY) a = d.ptr - 6u;      // header crc before type || payload
                const uint64_t al = d.ptr & ~(uint64_t)3;
                if (d.n < 4u) {
                    if (lane == 1u) a = al;
                    if (lane == 2u && al + 4u <= d.ptr + d.n - 1u) a = al + 4u;
                }
                stage = 1u;
            } else {  // first step: lanes before the block read the zero page
                const uint32_t l0 = d.f >> 2, r = d.f & 3u;
                a = d.ptr - d.f + lane * 4u;
                if (lane < l0) a = zp + lane * 4u;
                if (lane == l0 && r) a = d.n >= 4u ? d.ptr : zp + lane * 4u;
                base = uni64(d.ptr - d.f);
                plain = d.K - 1u;
                stage = 2u;
            }
        }
        ld_vaddr(dst, DBG ? check(P, a, lane) : a);
        // the lane-dependent selects above make the compiler treat this path's
        // results as divergent; pin the cursor back to SGPRs so the plain path
        // stays scalar
        b = uni64(b);
        base = uni64(base);
        plain = uni(plain);
        stage = uni(stage);
    }
    __device__ __forceinline__ void issue(uint32_t &dst, const KParams &P, uint32_t lane) {
        if (__builtin_expect(plain != 0u, 1)) {
            plain--;
            base += 256u;
            if (DBG) ld_vaddr(dst, check(P, base + lane * 4u, lane));
            else ld_sbase(dst, base, lane * 4u);
            return;
        }
        rare(dst, P, lane);
    }
};

// Results of finished blocks are collected lane-wise (lane j = j-th block
// finished since the last flush: a lane select of a wave-uniform value) and
// leave in one batch: a coalesced dword/byte store, or per-lane 5-byte trailers
// / 7-byte headers.  Blocks finish in index order, so lane j is block fin0 + j.
struct StreamFin {
    uint32_t res = 0;  // result / masked crc
    uint32_t aux = 0;  // MODE_TRAILER: type byte; MODE_LOG_HEADER: n | type << 16
    uint32_t hlo = 0, hhi = 0;  // MODE_LOG_HEADER: header offset
    uint64_t fin0 = 0;
    uint32_t nfin = 0;
};

template <int MODE>
__device__ __forceinline__ void stream_flush(const KParams &P, StreamFin &F, uint32_t lane) {
    if (F.nfin == 0) return;
    if (lane < F.nfin) {
        const uint64_t bi = F.fin0 + lane;
        if (MODE == MODE_CRC) P.out32[bi] = F.res;
        if (MODE == MODE_TABLE_VERIFY || MODE == MODE_LOG_VERIFY) P.out8[bi] = (uint8_t)F.res;
        if (MODE == MODE_TRAILER) {
            uint8_t *o = P.out8 + 5 * bi;
            o[0] = (uint8_t)F.aux;
            o[1] = (uint8_t)F.res;
            o[2] = (uint8_t)(F.res >> 8);
            o[3] = (uint8_t)(F.res >> 16);
            o[4] = (uint8_t)(F.res >> 24);
        }
        if (MODE == MODE_LOG_HEADER) {
            uint8_t *o = P.hdr_off ? P.out8 + (((uint64_t)F.hhi << 32) | F.hlo) : P.out8 + 7 * bi;
            o[0] = (uint8_t)F.res;
            o[1] = (uint8_t)(F.res >> 8);
            o[2] = (uint8_t)(F.res >> 16);
            o[3] = (uint8_t)(F.res >> 24);
            o[4] = (uint8_t)F.aux;
            o[5] = (uint8_t)(F.aux >> 8);
            o[6] = (uint8_t)(F.aux >> 16);
        }
    }
    F.fin0 += F.nfin;
    F.nfin = 0;
}

// wave-uniform result of block b whose crc state (before ~) is st
template <int MODE>
__device__ __forceinline__ void stream_result(const KParams &P, StreamFin &F, uint64_t b, const SDesc &d, uint32_t st,
                                              uint32_t stored, uint32_t lane) {
    const uint32_t sfx = stream_suffix<MODE>(P, b);
    if (sfx) st = (st >> 8) ^ saux(P.aux, (st ^ sfx) & 0xffu);
    const uint32_t crc = ~st, m = mask_crc(crc);
    uint32_t r = m, a = 0;
    if (MODE == MODE_CRC) r = (P.flags & 1u) ? m : crc;
    if (MODE == MODE_TABLE_VERIFY || MODE == MODE_LOG_VERIFY) r = (d.n == 0u || stored == m) ? 1u : 0u;
    if (MODE == MODE_TRAILER) a = sfx & 0xffu;
    if (MODE == MODE_LOG_HEADER) {
        a = (d.n & 0xffffu) | (sbyte(P.type, b) << 16);
        if (P.hdr_off) {
            const uint64_t h = sload64((const void *)(uintptr_t)uni64((uint64_t)(uintptr_t)(P.hdr_off + b)));
            F.hlo = lane == F.nfin ? (uint32_t)h : F.hlo;
            F.hhi = lane == F.nfin ? (uint32_t)(h >> 32) : F.hhi;
        }
    }
    if (d.bad) r = 0u;
    F.res = lane == F.nfin ? r : F.res;
    F.aux = lane == F.nfin ? a : F.aux;
    if (++F.nfin == 64u) stream_flush<MODE>(P, F, lane);
}

template <int MODE, int P_, bool DBG = false>
__global__ __launch_bounds__(1024) void crc_stream_kernel(const uint4 *__restrict__ img, KParams P,
                                                          const uint64_t *__restrict__ part) {
    static_assert(P_ >= 4 && P_ <= 48, "ring depth: vmcnt holds at most 63 outstanding loads");
    __shared__ uint32_t lds[kImageBytes / 4];
    load_image(lds, img);
    const uint32_t lane = threadIdx.x & 63u;
    const GLanes gl(lane);
    const uint32_t lc = 131072u | ((lane >> 5) << 14) | ((lane & 31u) << 2);
    const uint64_t waves = (uint64_t)gridDim.x * (blockDim.x >> 6);
    const uint64_t w = uni64((uint64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6));
    uint64_t b_begin, b_end;
    if (part) {
        b_begin = sload64((const void *)(uintptr_t)uni64((uint64_t)(uintptr_t)(part + w)));
        b_end = sload64((const void *)(uintptr_t)uni64((uint64_t)(uintptr_t)(part + w + 1)));
    } else {
        b_begin = P.n * w / waves;
        b_end = P.n * (w + 1) / waves;
    }
    if (b_begin >= b_end) return;

    StreamPF<MODE, DBG> pf;
    pf.b = b_begin;
    pf.b_end = b_end;
    pf.plain = 0;
    pf.base = 0;
    pf.stage = 1;
    pf.load_block(P);
    // The ring is indexed only with literal slot numbers (JL_PRE / JL_SLOT): a
    // ring register must never be copied between its asm load and its
    // s_waitcnt, so no loop the compiler might leave rolled may index it
    // (tests/test_asm.py).
    uint32_t ring[P_];
#define JL_PRE(u) \
    if constexpr ((u) < P_) pf.issue(ring[u], P, lane);
    JL_PRE(0) JL_PRE(1) JL_PRE(2) JL_PRE(3) JL_PRE(4) JL_PRE(5) JL_PRE(6) JL_PRE(7) JL_PRE(8) JL_PRE(9) JL_PRE(10)
    JL_PRE(11) JL_PRE(12) JL_PRE(13) JL_PRE(14) JL_PRE(15) JL_PRE(16) JL_PRE(17) JL_PRE(18) JL_PRE(19) JL_PRE(20)
    JL_PRE(21) JL_PRE(22) JL_PRE(23) JL_PRE(24) JL_PRE(25) JL_PRE(26) JL_PRE(27) JL_PRE(28) JL_PRE(29) JL_PRE(30)
    JL_PRE(31) JL_PRE(32) JL_PRE(33) JL_PRE(34) JL_PRE(35) JL_PRE(36) JL_PRE(37) JL_PRE(38) JL_PRE(39) JL_PRE(40)
    JL_PRE(41) JL_PRE(42) JL_PRE(43) JL_PRE(44) JL_PRE(45) JL_PRE(46) JL_PRE(47)
#undef JL_PRE

    // Compute cursor: plain = middle steps left in the current block; the rare
    // path handles the extra entry (stage 0), the first step with its seed
    // (stage 1) and the last step with the block's result (stage 2).
    uint64_t cb = b_begin;
    SDesc cd = stream_desc<MODE>(P, cb);
    uint32_t plain = 0, stage = cd.ex ? 0u : 1u;
    uint32_t t = 0, v3 = 0, stored = 0, tiny = 0;
    StreamFin F;
    F.fin0 = b_begin;

    // cb -> next block with entries, recording empty blocks on the way; false when done
    auto advance = [&]() -> bool {
        for (;;) {
            cb++;
            if (cb >= b_end) return false;
            cd = stream_desc<MODE>(P, cb);
            if (cd.K + cd.ex) {
                stage = cd.ex ? 0u : 1u;
                return true;
            }
            stream_result<MODE>(P, F, cb, cd, ~stream_init<MODE>(P, cb), 0u, lane);
        }
    };
    auto step = [&](uint32_t word) {
        const uint32_t x = xor3(t, v3, word);
        const uint32_t a0 = lds_at(lds, JL_GADDR(gl.l3, x, 0u));
        const uint32_t a1 = lds_at(lds, JL_GADDR(gl.l2, x, 1u));
        const uint32_t a2 = lds_at(lds, JL_GADDR(gl.l1, x, 2u));
        v3 = lds_at(lds, JL_GADDR(gl.l0, x, 3u));
        t = xor3(a0, a1, a2);
    };
    // rare entry of the compute cursor; false when the range is done
    auto rare = [&](uint32_t wv) -> bool {
        if (stage == 0u) {  // extra entry
            stored = uni(wv);
            if (cd.n < 4u) {
                const uint32_t d1 = (uint32_t)__builtin_amdgcn_readlane((int)wv, 1);
                const uint32_t d2 = (uint32_t)__builtin_amdgcn_readlane((int)wv, 2);
                tiny = __builtin_amdgcn_alignbyte(d2, d1, (uint32_t)(cd.ptr & 3u)) & (0xffffffffu >> (32 - 8 * cd.n));
            }
            stage = 1u;
            return true;
        }
        uint32_t word = wv;
        if (stage == 1u) {  // first step: seed word W fed as the 4 bytes before the block
            const uint32_t W = stream_seed<MODE>(P, cb);
            const uint32_t l0 = cd.f >> 2, r = cd.f & 3u, sh = 8u * r;
            if (r && lane == l0) word = ((cd.n >= 4u ? wv : tiny) << sh) | (W >> (32u - sh));
            if (l0 && lane == l0 - 1u) word = W << sh;
            t = 0;
            v3 = 0;
            if (l0 == 0u) {
                const uint32_t s63 = gstep(lds, W << sh, gl);
                t = lane == 63u ? s63 : 0u;
            }
            step(word);
            if (cd.K > 1u) {
                plain = cd.K - 2u;
                stage = 2u;
                return true;
            }
        } else {
            step(word);  // last step
        }
        stream_result<MODE>(P, F, cb, cd, wave_xor(realign(lds, t ^ v3, lc)), stored, lane);
        return advance();
    };
    auto rare_pinned = [&](uint32_t wv) -> bool {  // as in StreamPF::rare: keep the cursor in SGPRs
        const bool more = rare(wv);
        plain = uni(plain);
        stage = uni(stage);
        cb = uni64(cb);
        return more;
    };
    if (cd.K + cd.ex == 0) {
        stream_result<MODE>(P, F, cb, cd, ~stream_init<MODE>(P, cb), 0u, lane);
        if (!advance()) goto drain;
    }

    for (;;) {
#define JL_SLOT(u)                                                               \
    if constexpr ((u) < P_) {                                                    \
        asm volatile("s_waitcnt vmcnt(%1)" : "+v"(ring[u]) : "n"(P_ - 1));       \
        if (__builtin_expect(plain != 0u, 1)) {                                  \
            plain--;                                                             \
            step(ring[u]);                                                       \
        } else if (!rare_pinned(ring[u])) {                                      \
            goto drain;                                                          \
        }                                                                        \
        pf.issue(ring[u], P, lane);                                              \
    }
        JL_SLOT(0) JL_SLOT(1) JL_SLOT(2) JL_SLOT(3) JL_SLOT(4) JL_SLOT(5) JL_SLOT(6) JL_SLOT(7) JL_SLOT(8)
        JL_SLOT(9) JL_SLOT(10) JL_SLOT(11) JL_SLOT(12) JL_SLOT(13) JL_SLOT(14) JL_SLOT(15) JL_SLOT(16)
        JL_SLOT(17) JL_SLOT(18) JL_SLOT(19) JL_SLOT(20) JL_SLOT(21) JL_SLOT(22) JL_SLOT(23) JL_SLOT(24)
        JL_SLOT(25) JL_SLOT(26) JL_SLOT(27) JL_SLOT(28) JL_SLOT(29) JL_SLOT(30) JL_SLOT(31) JL_SLOT(32)
        JL_SLOT(33) JL_SLOT(34) JL_SLOT(35) JL_SLOT(36) JL_SLOT(37) JL_SLOT(38) JL_SLOT(39) JL_SLOT(40)
        JL_SLOT(41) JL_SLOT(42) JL_SLOT(43) JL_SLOT(44) JL_SLOT(45) JL_SLOT(46) JL_SLOT(47)
#undef JL_SLOT
    }
drain:
    stream_flush<MODE>(P, F, lane);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

template <>
hipError_t launch_stream_m<JL_MODE>(const void *img, const KParams &P, const uint64_t *part, int grid, int depth,
                                    hipStream_t st) {
    if (depth <= 16)
        hipLaunchKernelGGL((crc_stream_kernel<JL_MODE, 16>), dim3(grid), dim3(1024), 0, st, (const uint4 *)img, P, part);
    else if (depth <= 32)
        hipLaunchKernelGGL((crc_stream_kernel<JL_MODE, 32>), dim3(grid), dim3(1024), 0, st, (const uint4 *)img, P, part);
    else
        hipLaunchKernelGGL((crc_stream_kernel<JL_MODE, 48>), dim3(grid), dim3(1024), 0, st, (const uint4 *)img, P, part);
    return hipGetLastError();
}

}  // namespace jlk
