// jlcrc_kernels.hip — CDNA4 (gfx950) kernels of the masked-CRC32C engine.
//
// One wave (64 lanes) owns one block at a time.  A block of n bytes is viewed
// end-aligned as K = ceil(n/256) "steps" of 256 bytes (f = 256K - n virtual
// zero bytes in front); in step k lane l owns the 4-byte word at virtual offset
// 256k + 4l.  Every step is one coalesced 256-B wave load (global_load_dword)
// and, per lane, one slicing-by-4 update through the gap tables G (4 LDS
// lookups, bank-conflict-free by construction).  After K steps lane l is
// re-aligned with z^-(4l) (8 nibble lookups), the lanes are XOR-reduced with
// DPP, and the masked crc is stored by lane 0.  Algebra and LDS layout:
// crc_math.hpp and DESIGN.md §3.
//
// Persistent grid: one 1024-thread workgroup per CU (LDS = 160 KiB table image),
// 16 waves per CU; each wave walks its blocks with a one-chunk-ahead prefetch of
// the next 16 steps so the HBM stream never waits on the LDS chain.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "jlcrc_kernels.hpp"

namespace jlk {

typedef uint32_t __attribute__((aligned(1))) u32u;  // unaligned dword (unaligned mode is on under KFD)

__device__ __forceinline__ uint32_t lds_at(const uint32_t *lds, uint32_t byte_addr) {
    return *(const uint32_t *)((const char *)lds + byte_addr);
}

// One chain step: x = s ^ word; returns G3[x0] ^ G2[x1] ^ G1[x2] ^ G0[x3].
// l4lo = 4*(lane&31) (region A, tables G0/G1), l4hi = l4lo | 65536 (G2/G3).
__device__ __forceinline__ uint32_t gstep(const uint32_t *lds, uint32_t x, uint32_t l4lo, uint32_t l4hi) {
    uint32_t a0 = ((x << 7) & 0x7f80u) | l4hi;   // G3 @ 98304 = 65536 + 32768
    uint32_t a1 = ((x >> 1) & 0x7f80u) | l4hi;   // G2 @ 65536
    uint32_t a2 = ((x >> 9) & 0x7f80u) | l4lo;   // G1 @ 32768
    uint32_t a3 = ((x >> 17) & 0x7f80u) | l4lo;  // G0 @ 0
    uint32_t v0 = lds_at(lds, a0 + 32768u);
    uint32_t v1 = lds_at(lds, a1);
    uint32_t v2 = lds_at(lds, a2 + 32768u);
    uint32_t v3 = lds_at(lds, a3);
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

__device__ __forceinline__ void load_image(uint32_t *lds, const uint4 *__restrict__ img) {
    uint4 *d = (uint4 *)lds;
    for (uint32_t i = threadIdx.x; i < kImageBytes / 16; i += blockDim.x) d[i] = img[i];
    __syncthreads();
}

// ---------------------------------------------------------------------------
// Fast path: n_blocks contiguous 4 KiB blocks (one 16-step chunk each, f = 0).
// Ping-pong register buffers: the 16 loads of the wave's next block are issued
// (past the end: the zero page) before the current block's chain runs and are
// pinned there with a sched_barrier; the result store is issued by every lane
// to the same address (no divergent branch), so the loop body is one basic
// block and the waitcnt pass can leave the next block's loads in flight.
// ---------------------------------------------------------------------------
template <bool NT>
__device__ __forceinline__ void load16(uint32_t w[16], const uint32_t *p) {
#pragma unroll
    for (int k = 0; k < 16; k++) w[k] = NT ? __builtin_nontemporal_load(p + 64 * k) : p[64 * k];
}

__device__ __forceinline__ uint32_t chain16(uint32_t s, const uint32_t w[16], const uint32_t *lds, uint32_t l4lo,
                                            uint32_t l4hi) {
#pragma unroll
    for (int k = 0; k < 16; k++) s = gstep(lds, s ^ w[k], l4lo, l4hi);
    return s;
}

// 16 coalesced dword loads of one 4 KiB block, issued as inline asm so that the
// compiler cannot re-rotate them around the chain; the matching waits are
// wait16() below.  base is wave-uniform (SGPR pair), voff = 4*lane.
template <bool NT>
__device__ __forceinline__ void asm_load16(uint32_t w[16], const void *base, uint32_t voff) {
#define JL_LD(k, off)                                                                                    \
    if (NT) asm volatile("global_load_dword %0, %1, %2 offset:" #off " nt" : "=v"(w[k]) : "v"(voff), "s"(base) : "memory"); \
    else asm volatile("global_load_dword %0, %1, %2 offset:" #off : "=v"(w[k]) : "v"(voff), "s"(base) : "memory");
    JL_LD(0, 0) JL_LD(1, 256) JL_LD(2, 512) JL_LD(3, 768) JL_LD(4, 1024) JL_LD(5, 1280) JL_LD(6, 1536)
    JL_LD(7, 1792) JL_LD(8, 2048) JL_LD(9, 2304) JL_LD(10, 2560) JL_LD(11, 2816) JL_LD(12, 3072)
    JL_LD(13, 3328) JL_LD(14, 3584) JL_LD(15, 3840)
#undef JL_LD
}

// Chain over a block whose 16 loads were followed by the 16-load batches of D
// later blocks (plus at most D stores): word k is complete once at most
// 15-k + 16*D vector-memory operations are outstanding.
template <int D>
__device__ __forceinline__ uint32_t chain16_waited(uint32_t s, uint32_t w[16], const uint32_t *lds, uint32_t l4lo,
                                                   uint32_t l4hi) {
#define JL_STEP(k)                                                                    \
    asm volatile("s_waitcnt vmcnt(%1)" : "+v"(w[k]) : "n"(15 - k + 16 * D));         \
    s = gstep(lds, s ^ w[k], l4lo, l4hi);
    JL_STEP(0) JL_STEP(1) JL_STEP(2) JL_STEP(3) JL_STEP(4) JL_STEP(5) JL_STEP(6) JL_STEP(7)
    JL_STEP(8) JL_STEP(9) JL_STEP(10) JL_STEP(11) JL_STEP(12) JL_STEP(13) JL_STEP(14) JL_STEP(15)
#undef JL_STEP
    return s;
}

// D = prefetch depth in blocks (1..3): while block b's chain runs, the loads of
// blocks b+W .. b+D*W (W = waves in the grid) are in flight, i.e. up to
// 16 waves x D x 4 KiB per CU.  Buffers rotate statically (loop unrolled D+1).
template <bool NT, int D>
__global__ __launch_bounds__(1024) void crc_fixed4k_kernel(const uint4 *__restrict__ img,
                                                           const uint8_t *__restrict__ data,
                                                           const uint8_t *__restrict__ zero, uint64_t n_blocks,
                                                           uint32_t flags, uint32_t *__restrict__ out) {
    static_assert(D >= 1 && D <= 3, "vmcnt is 6 bits: at most 3 blocks ahead");
    __shared__ uint32_t lds[kImageBytes / 4];
    load_image(lds, img);
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t voff = lane * 4u;
    const uint32_t l4lo = (lane & 31u) << 2, l4hi = l4lo | 65536u;
    const uint32_t lc = 131072u | ((lane >> 5) << 14) | l4lo;
    const uint32_t s_init = (lane == 0) ? 0xffffffffu : 0u;
    const uint32_t do_mask = flags & 1u;
    const uint64_t waves = (uint64_t)gridDim.x * (blockDim.x >> 6);
    uint64_t b = uni64((uint64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6));
    if (b >= n_blocks) return;
    uint32_t w[D + 1][16];
#pragma unroll
    for (int j = 0; j < D; j++) {
        const uint64_t bj = b + (uint64_t)j * waves;
        asm_load16<NT>(w[j], bj < n_blocks ? data + bj * 4096u : zero, voff);
    }
    for (;;) {
#pragma unroll
        for (int j = 0; j <= D; j++) {
            const uint64_t bp = b + (uint64_t)D * waves;
            asm_load16<NT>(w[(j + D) % (D + 1)], bp < n_blocks ? data + bp * 4096u : zero, voff);
            const uint32_t crc = ~wave_xor(realign(lds, chain16_waited<D>(s_init, w[j], lds, l4lo, l4hi), lc));
            out[b] = do_mask ? mask_crc(crc) : crc;
            b += waves;
            if (b >= n_blocks) goto done;
        }
    }
done:
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // drain the zero-page prefetches
}

// ---------------------------------------------------------------------------
// General path: arbitrary lengths / alignment, per-block init & suffix and the
// epilogue modes of the caller shims (plain crc, table trailer, table verify,
// log header, log verify).  A block is end-aligned to whole 16-step chunks:
// f = 4096*chunks - n virtual zero bytes in front.  Zero words leave a zero
// chain state unchanged, so every chunk runs exactly 16 unconditional steps;
// the initial state z^-r(~init) is XORed into the word that holds real byte 0
// (step k0 = (f>>8)&15 of chunk f>>12, lane (f>>2)&63, r = f&3), together
// with that word's bytes when it straddles the block start.
// ---------------------------------------------------------------------------
struct BlockDesc {
    const uint8_t *ptr;  // first byte
    uint32_t n;          // bytes covered by the crc
    uint32_t init;       // extend() initial crc
    uint32_t suffix;     // 0x100 | byte, or 0
    uint32_t chunks;     // ceil(n/4096) (0 for n == 0)
    uint32_t f;          // 4096*chunks - n
};

__device__ __forceinline__ BlockDesc get_desc(const KParams &P, uint64_t i) {
    BlockDesc d;
    uint64_t off;
    uint32_t n;
    if (P.off) {
        off = uni64(P.off[i]);
        n = uni(P.len[i]) + P.len_add;
    } else {
        off = i * P.fixed_bytes;
        n = (uint32_t)P.fixed_bytes;
    }
    d.ptr = P.base + off;
    d.n = n;
    uint32_t init = 0;
    if (P.init) init = uni(P.init[i]);
    if (P.mode == MODE_LOG_HEADER) init = P.aux[512 + (uni(P.type[i]) & 0xffu) % 5u];
    d.init = init;
    uint32_t sfx = 0;
    if (P.mode == MODE_TRAILER) sfx = 0x100u | (P.type ? (uni(P.type[i]) & 0xffu) : 0u);
    else if (P.suffix) sfx = 0x100u | (uni(P.suffix[i]) & 0xffu);
    d.suffix = sfx;
    d.chunks = (uint32_t)(((uint64_t)n + 4095u) >> 12);
    d.f = (d.chunks << 12) - n;
    return d;
}

// Loads chunk `chunk` of block d for this lane (zero page outside the block).
__device__ __forceinline__ void load_chunk(uint32_t w[16], const BlockDesc &d, bool valid, uint32_t chunk,
                                           uint32_t lane, const uint8_t *zero) {
    const int64_t base_p = (int64_t)chunk * 4096 + 4 * (int64_t)lane - (int64_t)d.f;
    const uint8_t *zp = zero + 4 * lane;
#pragma unroll
    for (int k = 0; k < 16; k++) {
        int64_t p = base_p + 256 * k;
        const uint8_t *a = (valid && p >= 0) ? d.ptr + p : zp;
        w[k] = *(const u32u *)a;
    }
}

__device__ __forceinline__ void epilogue(const KParams &P, uint64_t i, const BlockDesc &d, uint32_t crc,
                                         uint32_t lane) {
    const uint32_t m = mask_crc(crc);
    switch (P.mode) {
    case MODE_CRC:
        P.out32[i] = (P.flags & 1u) ? m : crc;
        break;
    case MODE_TABLE_VERIFY:  // trailer crc stored LE32 right after the n = size+1 covered bytes
        if (lane == 0) P.out8[i] = (*(const u32u *)(d.ptr + d.n) == m) ? 1 : 0;
        break;
    case MODE_LOG_VERIFY:  // header crc 6 bytes before the covered range; n == 0: not an OK event
        if (lane == 0 && d.n) P.out8[i] = (*(const u32u *)(d.ptr - 6) == m) ? 1 : 0;
        break;
    case MODE_TRAILER:
        if (lane < 5) P.out8[5 * i + lane] = (lane == 0) ? (uint8_t)(d.suffix & 0xffu) : (uint8_t)(m >> (8 * (lane - 1)));
        break;
    case MODE_LOG_HEADER:
        if (lane < 7) {
            uint8_t b;
            if (lane < 4) b = (uint8_t)(m >> (8 * lane));
            else if (lane == 4) b = (uint8_t)(d.n & 0xffu);
            else if (lane == 5) b = (uint8_t)((d.n >> 8) & 0xffu);
            else b = (uint8_t)(uni(P.type[i]) & 0xffu);
            P.out8[7 * i + lane] = b;
        }
        break;
    default:
        break;
    }
}

struct GenState {
    uint64_t blk;
    uint32_t chunk;
    BlockDesc d;
    uint32_t s;
};

// Consumes `cur` (this wave's current chunk) after issuing the loads of its
// next chunk into `nxt`.  Returns false when the wave has no further chunk.
__device__ __forceinline__ bool general_item(const KParams &P, GenState &g, uint32_t cur[16], uint32_t nxt[16],
                                             const uint32_t *lds, uint32_t lane, uint32_t l4lo, uint32_t l4hi,
                                             uint32_t lc, uint64_t waves) {
    uint64_t nblk = g.blk;
    uint32_t nchunk = g.chunk + 1;
    BlockDesc nd = g.d;
    if (nchunk >= g.d.chunks) {
        nchunk = 0;
        nblk = g.blk + waves;
        if (nblk < P.n) nd = get_desc(P, nblk);
    }
    const bool more = nblk < P.n;
    load_chunk(nxt, nd, more && nchunk < nd.chunks, nchunk, lane, P.zero);
    __builtin_amdgcn_sched_barrier(0);

    const BlockDesc &d = g.d;
    if (d.chunks) {
        if (g.chunk == (d.f >> 12)) {
            // chunk holding real byte 0: XOR z^-r(~init) (and the straddling
            // bytes) into word k0 of lane l0; all earlier words are zero.
            uint32_t s0 = ~d.init;
            const uint32_t r = d.f & 3u, l0 = (d.f >> 2) & 63u, k0 = (d.f >> 8) & 15u;
            for (uint32_t q = 0; q < r; q++) {  // z^-1, wave-uniform
                uint32_t top = P.aux[256 + (s0 >> 24)];
                s0 = ((s0 ^ P.aux[top]) << 8) | top;
            }
            uint32_t x = 0;
            if (lane == l0) {
                x = s0;
                for (uint32_t j = 0; j < ((4u - r) & 3u); j++) x ^= (uint32_t)d.ptr[j] << (8 * (j + r));
            }
#pragma unroll
            for (int k = 0; k < 16; k++) cur[k] ^= ((uint32_t)k == k0) ? x : 0u;
        }
        g.s = chain16(g.chunk == 0 ? 0u : g.s, cur, lds, l4lo, l4hi);
    }
    if (g.chunk + 1 >= d.chunks) {
        uint32_t t = d.chunks ? wave_xor(realign(lds, g.s, lc)) : ~d.init;
        if (d.suffix) t = (t >> 8) ^ P.aux[(t ^ d.suffix) & 0xffu];
        epilogue(P, g.blk, d, ~t, lane);
    }
    g.blk = nblk;
    g.chunk = nchunk;
    g.d = nd;
    return more;
}

__global__ __launch_bounds__(1024) void crc_general_kernel(const uint4 *__restrict__ img, KParams P) {
    __shared__ uint32_t lds[kImageBytes / 4];
    load_image(lds, img);
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t l4lo = (lane & 31u) << 2, l4hi = l4lo | 65536u;
    const uint32_t lc = 131072u | ((lane >> 5) << 14) | l4lo;
    const uint64_t waves = (uint64_t)gridDim.x * (blockDim.x >> 6);
    GenState g;
    g.blk = uni64((uint64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6));
    if (g.blk >= P.n) return;
    g.d = get_desc(P, g.blk);
    g.chunk = 0;
    g.s = 0;
    uint32_t wa[16], wb[16];
    load_chunk(wa, g.d, g.d.chunks != 0, 0, lane, P.zero);
    for (;;) {
        if (!general_item(P, g, wa, wb, lds, lane, l4lo, l4hi, lc, waves)) break;
        if (!general_item(P, g, wb, wa, lds, lane, l4lo, l4hi, lc, waves)) break;
    }
}

// ---------------------------------------------------------------------------
// Log walk (LogReader.readPhysicalRecord header decisions per 32 KiB block,
// J/db/LogReader.java:297-383).  One thread per block; pass 0 counts events,
// pass 1 writes them (offsets from an exclusive scan of the counts).  CRC
// verification of the OK events is done by crc_general_kernel afterwards and
// applied by log_finalize_kernel.
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t rd16(const uint8_t *p) { return (uint32_t)p[0] | ((uint32_t)p[1] << 8); }

__global__ void log_walk_kernel(const uint8_t *__restrict__ log, uint64_t size, uint64_t n_blocks, int pass,
                                uint64_t *__restrict__ counts, const uint64_t *__restrict__ starts,
                                LogEvent *__restrict__ ev, uint64_t *__restrict__ d_off, uint32_t *__restrict__ d_len) {
    uint64_t b = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= n_blocks) return;
    const uint64_t bs = b * 32768u;
    const uint64_t be = (bs + 32768u < size) ? bs + 32768u : size;
    const bool eof = (be - bs) < 32768u;
    uint64_t p = bs, cnt = 0;
    uint64_t o = pass ? starts[b] : 0;
    for (;;) {
        const uint64_t rem = be - p;
        uint8_t kind = 0;
        uint32_t length = 0, type = 0;
        bool stop = false;
        if (rem < 7) {
            if (eof && rem > 0) { kind = 6; stop = true; }
            else break;
        } else {
            const uint8_t *h = log + p;
            length = rd16(h + 4);
            type = h[6];
            if (7u + (uint64_t)length > rem) { kind = eof ? 5 : 3; stop = true; }
            else if (type == 0 && length == 0) { kind = 4; stop = true; }
            else kind = 1;
        }
        if (pass) {
            LogEvent e;
            e.offset = p;
            e.length = length;
            e.type = (uint8_t)type;
            e.kind = kind;
            e.pad = 0;
            ev[o + cnt] = e;
            if (kind == 1) { d_off[o + cnt] = p + 6; d_len[o + cnt] = 1u + length; }
            else { d_off[o + cnt] = p; d_len[o + cnt] = 0; }
        }
        cnt++;
        if (stop) break;
        p += 7u + length;
    }
    if (!pass) counts[b] = cnt;
}

// Applies the per-record CRC results (ok[i] = 1 match) and truncates each block
// after its first mismatch (the reference clears its 32 KiB buffer, :359-367):
// the failing event becomes BAD_CRC, later events of the block become kind 0
// (not visible to the reader).
__global__ void log_finalize_kernel(uint64_t n_blocks, const uint64_t *__restrict__ starts,
                                    const uint64_t *__restrict__ counts, const uint8_t *__restrict__ ok,
                                    LogEvent *__restrict__ ev, int checksum) {
    uint64_t b = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= n_blocks || !checksum) return;
    const uint64_t s = starts[b], c = counts[b];
    bool dead = false;
    for (uint64_t i = s; i < s + c; i++) {
        if (dead) { ev[i].kind = 0; continue; }
        if (ev[i].kind == 1 && !ok[i]) { ev[i].kind = 2; dead = true; }
    }
}

__global__ void fill_random_kernel(uint64_t *__restrict__ dst, uint64_t words, uint64_t seed, uint64_t first_word) {
    uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < words; i += stride) {
        uint64_t z = seed + (first_word + i + 1) * 0x9E3779B97F4A7C15ull;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        z ^= z >> 31;
        dst[i] = z;
    }
}

__global__ void fill_random_tail_kernel(uint8_t *__restrict__ dst, uint64_t bytes, uint64_t seed, uint64_t first_word) {
    // tail bytes (bytes % 8) of the last word
    uint64_t w = bytes / 8;
    uint64_t z = seed + (first_word + w + 1) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    for (uint64_t i = w * 8, j = 0; i < bytes; i++, j++) dst[i] = (uint8_t)(z >> (8 * j));
}

// Read-only HBM stream (calibration for the roofline): every workgroup XOR-folds
// its grid-stride share of the buffer with 16-B loads and writes one word.
typedef uint32_t v4u __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void read_stream_kernel(const v4u *__restrict__ src, uint64_t n16,
                                                          uint32_t *__restrict__ sink) {
    v4u acc = {0, 0, 0, 0};
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (; i + 3 * stride < n16; i += 4 * stride) {
        v4u a = __builtin_nontemporal_load(src + i), b = __builtin_nontemporal_load(src + i + stride);
        v4u c = __builtin_nontemporal_load(src + i + 2 * stride), d = __builtin_nontemporal_load(src + i + 3 * stride);
        acc ^= a ^ b ^ c ^ d;
    }
    for (; i < n16; i += stride) acc ^= src[i];
    uint32_t v = wave_xor(acc.x ^ acc.y ^ acc.z ^ acc.w);
    if ((threadIdx.x & 63u) == 0) atomicXor(sink, v);
}

}  // namespace jlk

// ----------------------------------------------------------------- launchers
namespace jlk {

hipError_t launch_fixed4k(const void *img, const uint8_t *data, const uint8_t *zero, uint64_t n_blocks,
                          uint32_t flags, uint32_t *out, int grid, int nt, int depth, hipStream_t st) {
#define JL_L(NTV, DV)                                                                                          \
    hipLaunchKernelGGL((crc_fixed4k_kernel<NTV, DV>), dim3(grid), dim3(1024), 0, st, (const uint4 *)img, data, zero, \
                       n_blocks, flags, out)
    if (nt) {
        if (depth <= 1) JL_L(true, 1);
        else if (depth == 2) JL_L(true, 2);
        else JL_L(true, 3);
    } else {
        if (depth <= 1) JL_L(false, 1);
        else if (depth == 2) JL_L(false, 2);
        else JL_L(false, 3);
    }
#undef JL_L
    return hipGetLastError();
}

hipError_t launch_general(const void *img, const KParams &P, int grid, hipStream_t st) {
    hipLaunchKernelGGL(crc_general_kernel, dim3(grid), dim3(1024), 0, st, (const uint4 *)img, P);
    return hipGetLastError();
}

hipError_t launch_log_walk(const uint8_t *log, uint64_t size, uint64_t n_blocks, int pass, uint64_t *counts,
                           const uint64_t *starts, LogEvent *ev, uint64_t *d_off, uint32_t *d_len, hipStream_t st) {
    unsigned grid = (unsigned)((n_blocks + 255) / 256);
    hipLaunchKernelGGL(log_walk_kernel, dim3(grid), dim3(256), 0, st, log, size, n_blocks, pass, counts, starts, ev,
                       d_off, d_len);
    return hipGetLastError();
}

hipError_t launch_log_finalize(uint64_t n_blocks, const uint64_t *starts, const uint64_t *counts, const uint8_t *ok,
                               LogEvent *ev, int checksum, hipStream_t st) {
    unsigned grid = (unsigned)((n_blocks + 255) / 256);
    hipLaunchKernelGGL(log_finalize_kernel, dim3(grid), dim3(256), 0, st, n_blocks, starts, counts, ok, ev, checksum);
    return hipGetLastError();
}

hipError_t launch_read_stream(const void *src, uint64_t bytes, uint32_t *sink, int grid, hipStream_t st) {
    hipLaunchKernelGGL(read_stream_kernel, dim3(grid), dim3(256), 0, st, (const v4u *)src, bytes / 16, sink);
    return hipGetLastError();
}

hipError_t launch_fill_random(void *dst, uint64_t bytes, uint64_t seed, uint64_t first_word, hipStream_t st) {
    uint64_t words = bytes / 8;
    if (words) {
        uint64_t g = (words + 255) / 256;
        if (g > 65536) g = 65536;
        hipLaunchKernelGGL(fill_random_kernel, dim3((unsigned)g), dim3(256), 0, st, (uint64_t *)dst, words, seed,
                           first_word);
    }
    if (bytes % 8) hipLaunchKernelGGL(fill_random_tail_kernel, dim3(1), dim3(1), 0, st, (uint8_t *)dst, bytes, seed, first_word);
    return hipGetLastError();
}

}  // namespace jlk
