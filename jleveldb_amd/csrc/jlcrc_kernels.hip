// jlcrc_kernels.hip — CDNA4 (gfx950) helper kernels of the masked-CRC32C engine:
// the log-writer payload copy, the stream kernel's byte-balanced partition, the
// event rebase of chunked host log verification, and the fill and read-stream
// kernels of the benchmark (synthetic inputs, the HBM read ceiling).  The CRC
// kernels live in fixed_v4.hip (4 KiB blocks), general_v4.hip (offset/length
// batches, log record chunks), stream_kernel.hip (small batches, trailers,
// headers), log_chunks.hip and log_stream.hip (WAL verification).  The round-1
// kernels those superseded live on the git branch study-superseded-kernels.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "engine_device.hpp"

namespace jlk {

// Payload copies of a batched LogWriter (jl_log_emit_dev): one workgroup per
// fragment (grid-stride), byte-granular (arbitrary alignment on both sides);
// also records each payload's file offset for the header pass.
__global__ __launch_bounds__(256) void log_copy_kernel(const uint8_t *__restrict__ src,
                                                       const uint64_t *__restrict__ frag_src_off,
                                                       const uint64_t *__restrict__ frag_hdr_off,
                                                       const uint32_t *__restrict__ frag_len, uint64_t n_frags,
                                                       uint8_t *__restrict__ log, uint64_t *__restrict__ pay_off) {
    for (uint64_t f = blockIdx.x; f < n_frags; f += gridDim.x) {
        const uint64_t so = frag_src_off[f], d = frag_hdr_off[f] + 7u;
        const uint32_t n = frag_len[f];
        if (threadIdx.x == 0) pay_off[f] = d;
        for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) log[d + i] = src[so + i];
    }
}

// part[w] for every target T_w = ceil(total*w/W), w in [1, W): the first block
// whose exclusive prefix reaches T_w.  One thread per block sets the targets
// that fall inside it, (e_i, e_{i+1}] -> w in [floor(e_i W/total)+1, floor(e_{i+1} W/total)].
__global__ __launch_bounds__(256) void partition_kernel(const uint64_t *__restrict__ incl, uint64_t n, uint64_t W,
                                                        uint64_t *__restrict__ part) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t total = incl[n - 1];
    if (i == 0) {
        part[0] = 0;
        part[W] = n;
    }
    if (i >= n) return;
    const uint64_t e0 = i ? incl[i - 1] : 0, e1 = incl[i];
    uint64_t lo = e0 * W / total + 1, hi = e1 * W / total;
    if (hi > W - 1) hi = W - 1;
    for (uint64_t w = lo; w <= hi; w++) part[w] = i + 1;
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

// Read-only HBM stream (calibration for the roofline).  The fastest read shape
// measured on MI355X (tools/hbm_probe.hip, profiles/r1b_hbm_probe.log): LDS-DMA
// (global_load_lds_dwordx4 ... nt), each wave streaming 8 KiB pieces into its
// own 8 x 1 KiB LDS ring, 4 waves per workgroup, 8 workgroups per CU.  Bytes
// past the last whole 8 KiB piece are read with plain 16-B loads.
typedef uint32_t v4u __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void read_stream_kernel(const uint8_t *__restrict__ src, uint64_t bytes,
                                                          uint32_t *__restrict__ sink) {
    __shared__ __attribute__((aligned(16))) uint8_t ring[4][8][1024];
    const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
    const uint64_t waves = (uint64_t)gridDim.x * 4u;
    const uint64_t pieces = bytes / 8192u;
    uint32_t acc = 0;
    for (uint64_t c = (uint64_t)blockIdx.x * 4u + wv; c < pieces; c += waves) {
        const uint8_t *p = src + c * 8192u + lane * 16u;
#pragma unroll
        for (int k = 0; k < 8; k++)
            __builtin_amdgcn_global_load_lds((const void *)(p + k * 1024), (__attribute__((address_space(3))) void *)&ring[wv][k][0],
                                             16, 0, 2 /* nt */);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        acc ^= *(const uint32_t *)&ring[wv][lane & 7u][(lane >> 3) * 4u];
    }
    const uint64_t t0 = pieces * 8192u / 16u, n16 = bytes / 16u;
    for (uint64_t i = t0 + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * blockDim.x) {
        v4u v = ((const v4u *)src)[i];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    // one conditional store per wave (the loads must not be dead code): 8k
    // same-address atomics at the end of the grid cost ~75 us (r1 measurement)
    acc = wave_xor(acc);
    if (lane == 0 && acc == 0x6a4c4442u) *sink = acc;
}

}  // namespace jlk

// ----------------------------------------------------------------- launchers
namespace jlk {

hipError_t launch_stream(const void *img, const KParams &P, const uint64_t *part, int grid, int depth, hipStream_t st) {
    switch (P.mode) {
    case MODE_CRC: return launch_stream_m<MODE_CRC>(img, P, part, grid, depth, st);
    case MODE_TABLE_VERIFY: return launch_stream_m<MODE_TABLE_VERIFY>(img, P, part, grid, depth, st);
    case MODE_TRAILER: return launch_stream_m<MODE_TRAILER>(img, P, part, grid, depth, st);
    case MODE_LOG_HEADER: return launch_stream_m<MODE_LOG_HEADER>(img, P, part, grid, depth, st);
    default: return hipErrorInvalidValue;
    }
}

hipError_t launch_partition(const uint64_t *incl, uint64_t n, uint64_t parts, uint64_t *part, hipStream_t st) {
    hipLaunchKernelGGL(partition_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, incl, n, parts, part);
    return hipGetLastError();
}

hipError_t launch_log_copy(const uint8_t *src, const uint64_t *frag_src_off, const uint64_t *frag_hdr_off,
                           const uint32_t *frag_len, uint64_t n_frags, uint8_t *log, uint64_t *pay_off, hipStream_t st) {
    const unsigned grid = (unsigned)std::min<uint64_t>(n_frags, 65536);
    hipLaunchKernelGGL(log_copy_kernel, dim3(grid), dim3(256), 0, st, src, frag_src_off, frag_hdr_off, frag_len,
                       n_frags, log, pay_off);
    return hipGetLastError();
}

// Chunked host log verification (jl_log_verify): a chunk's events carry offsets
// relative to the chunk; this moves them to file offsets before the copy out.
__global__ void event_rebase_kernel(LogEvent *__restrict__ ev, uint64_t n, uint64_t base) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        ev[i].offset += base;
}

hipError_t launch_event_rebase(LogEvent *ev, uint64_t n, uint64_t base, hipStream_t st) {
    if (n == 0 || base == 0) return hipSuccess;
    const unsigned grid = (unsigned)std::min<uint64_t>((n + 255) / 256, 4096);
    hipLaunchKernelGGL(event_rebase_kernel, dim3(grid), dim3(256), 0, st, ev, n, base);
    return hipGetLastError();
}

hipError_t launch_read_stream(const void *src, uint64_t bytes, uint32_t *sink, int grid, hipStream_t st) {
    hipLaunchKernelGGL(read_stream_kernel, dim3(grid), dim3(256), 0, st, (const uint8_t *)src, bytes, sink);
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
