// hbm_probe.hip — standalone HBM read-bandwidth probe (tools only, not product).
// Measures which load shapes reach the highest read rate on this MI355X so the
// CRC kernel's load path can be chosen from measurements.
// Build: hipcc --offload-arch=gfx950 -O3 tools/hbm_probe.hip -o /tmp/hbm_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

typedef uint32_t v4u __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint32_t fold(v4u a) { return a.x ^ a.y ^ a.z ^ a.w; }

// A/B: grid-stride 16-B loads, U in flight per thread
template <int U, bool NT>
__global__ __launch_bounds__(256) void rd_v4(const v4u *__restrict__ s, uint64_t n16, uint32_t *sink) {
    v4u acc = {0, 0, 0, 0};
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (; i + (U - 1) * stride < n16; i += U * stride) {
        v4u t[U];
#pragma unroll
        for (int u = 0; u < U; u++) t[u] = NT ? __builtin_nontemporal_load(s + i + u * stride) : s[i + u * stride];
#pragma unroll
        for (int u = 0; u < U; u++) acc ^= t[u];
    }
    if (fold(acc) == 0x12345678u) atomicAdd(sink, 1u);
}

// C: per-wave contiguous chunks: each wave owns CH bytes, reads them with dword
// (W=4) or dwordx4 (W=16) loads, 16 loads in flight, persistent grid.
template <int W, bool NT>
__global__ __launch_bounds__(1024) void rd_chunk(const uint8_t *__restrict__ s, uint64_t bytes, uint32_t *sink) {
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t waves = (uint64_t)gridDim.x * (blockDim.x >> 6);
    uint64_t w = (uint64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    const uint64_t chunk = 64ull * W * 16;  // 16 wave-loads per chunk
    uint32_t acc = 0;
    for (uint64_t c = w; c * chunk < bytes; c += waves) {
        const uint8_t *p = s + c * chunk + lane * W;
        if (W == 4) {
            uint32_t t[16];
#pragma unroll
            for (int k = 0; k < 16; k++) t[k] = NT ? __builtin_nontemporal_load((const uint32_t *)(p + k * 256)) : *(const uint32_t *)(p + k * 256);
#pragma unroll
            for (int k = 0; k < 16; k++) acc ^= t[k];
        } else {
            v4u t[16];
#pragma unroll
            for (int k = 0; k < 16; k++) t[k] = NT ? __builtin_nontemporal_load((const v4u *)(p + k * 1024)) : *(const v4u *)(p + k * 1024);
#pragma unroll
            for (int k = 0; k < 16; k++) acc ^= fold(t[k]);
        }
    }
    if (acc == 0x12345678u) atomicAdd(sink, 1u);
}

// C2: chunk_dword_nt with optional 160 KiB LDS (1 WG/CU) and optional one-block prefetch
template <bool LDS, bool PF>
__global__ __launch_bounds__(1024) void rd_chunk2(const uint8_t *__restrict__ s, uint64_t bytes, uint32_t *sink) {
    __shared__ uint32_t big[LDS ? 40960 : 1];
    const uint32_t lane = threadIdx.x & 63;
    if (LDS) { big[threadIdx.x] = threadIdx.x; __syncthreads(); }
    const uint64_t waves = (uint64_t)gridDim.x * (blockDim.x >> 6);
    uint64_t w = (uint64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    const uint64_t nb = bytes / 4096;
    uint32_t acc = 0;
    if (!PF) {
        for (uint64_t c = w; c < nb; c += waves) {
            const uint32_t *p = (const uint32_t *)(s + c * 4096) + lane;
            uint32_t t[16];
#pragma unroll
            for (int k = 0; k < 16; k++) t[k] = __builtin_nontemporal_load(p + 64 * k);
#pragma unroll
            for (int k = 0; k < 16; k++) acc ^= t[k];
        }
    } else {
        uint32_t a[16], b[16];
        uint64_t c = w;
        const uint32_t *p = (const uint32_t *)(s + c * 4096) + lane;
#pragma unroll
        for (int k = 0; k < 16; k++) a[k] = __builtin_nontemporal_load(p + 64 * k);
        for (;;) {
            uint64_t c2 = c + waves < nb ? c + waves : c;
            const uint32_t *q = (const uint32_t *)(s + c2 * 4096) + lane;
#pragma unroll
            for (int k = 0; k < 16; k++) b[k] = __builtin_nontemporal_load(q + 64 * k);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int k = 0; k < 16; k++) acc ^= a[k] * (k + 1);
            c += waves;
            if (c >= nb) break;
#pragma unroll
            for (int k = 0; k < 16; k++) a[k] = b[k];
        }
    }
    if (LDS) acc ^= big[(threadIdx.x * 7) & 1023];
    if (acc == 0x12345678u) atomicAdd(sink, 1u);
}

// D: LDS-DMA (global_load_lds_dwordx4), ring of R x 1 KiB slots per wave, nt or not
template <bool NT>
__global__ __launch_bounds__(256) void rd_ldsdma(const uint8_t *__restrict__ s, uint64_t bytes, uint32_t *sink) {
    __shared__ __attribute__((aligned(16))) uint8_t ring[4][8][1024];  // 4 waves x 8 slots
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint64_t waves = (uint64_t)gridDim.x * 4;
    uint64_t w = (uint64_t)blockIdx.x * 4 + wv;
    uint32_t acc = 0;
    for (uint64_t c = w; c * 8192 < bytes; c += waves) {
        const uint8_t *p = s + c * 8192 + lane * 16;
#pragma unroll
        for (int k = 0; k < 8; k++)
            __builtin_amdgcn_global_load_lds((const void *)(p + k * 1024), (__attribute__((address_space(3))) void *)&ring[wv][k][0], 16, 0, NT ? 2 : 0);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        acc ^= *(const uint32_t *)&ring[wv][lane & 7][(lane >> 3) * 4];
    }
    if (acc == 0x12345678u) atomicAdd(sink, 1u);
}

__global__ void fill_rand(uint64_t *d, uint64_t words) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < words; i += (uint64_t)gridDim.x * blockDim.x) {
        uint64_t z = 0x4A4C4442ull + (i + 1) * 0x9E3779B97F4A7C15ull;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        d[i] = z ^ (z >> 31);
    }
}

int main(int argc, char **argv) {
    size_t bytes = (size_t)(argc > 3 ? atoi(argv[3]) : 4) << 30;  // GiB (argv[3]; default 4)
    uint8_t *d;
    uint32_t *sink;
    CK(hipMalloc(&d, bytes));
    CK(hipMalloc(&sink, 4));
    // random bytes: HBM read rates measured on constant data are higher than on
    // real data (profiles/r1b_*), so the probe reads what the engine reads
    fill_rand<<<4096, 256>>>((uint64_t *)d, bytes / 8);
    CK(hipDeviceSynchronize());
    hipDeviceProp_t p;
    CK(hipGetDeviceProperties(&p, 0));
    int cu = p.multiProcessorCount;
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    struct V { const char *name; int kind; int grid; };
    std::vector<V> vs = {
        {"v4_u4_plain_g2048", 0, cu * 8}, {"v4_u4_nt_g2048", 1, cu * 8}, {"v4_u8_plain_g2048", 2, cu * 8},
        {"v4_u8_nt_g2048", 3, cu * 8}, {"v4_u4_nt_g1024", 1, cu * 4}, {"v4_u4_nt_g8192", 1, cu * 32},
        {"v4_u8_nt_g512", 3, cu * 2},
        {"chunk_dword_nt_1wg", 4, cu}, {"chunk_dword_plain_1wg", 5, cu}, {"chunk_x4_nt_1wg", 6, cu},
        {"chunk_x4_plain_1wg", 7, cu}, {"chunk_dword_nt_2wg", 4, cu * 2},
        {"chunk2_nolds_nopf", 10, cu}, {"chunk2_lds_nopf", 11, cu}, {"chunk2_nolds_pf", 12, cu},
        {"chunk2_lds_pf", 13, cu},
        {"ldsdma_nt_g1024", 8, cu * 4}, {"ldsdma_plain_g1024", 9, cu * 4}, {"ldsdma_nt_g2048", 8, cu * 8},
    };
    const int rounds = argc > 1 ? atoi(argv[1]) : 5, reps = argc > 2 ? atoi(argv[2]) : 5;
    std::vector<std::vector<float>> t(vs.size());
    for (int r = 0; r < rounds; r++)
        for (size_t v = 0; v < vs.size(); v++) {
            auto launch = [&]() {
                int g = vs[v].grid;
                switch (vs[v].kind) {
                case 0: rd_v4<4, false><<<g, 256>>>((const v4u *)d, bytes / 16, sink); break;
                case 1: rd_v4<4, true><<<g, 256>>>((const v4u *)d, bytes / 16, sink); break;
                case 2: rd_v4<8, false><<<g, 256>>>((const v4u *)d, bytes / 16, sink); break;
                case 3: rd_v4<8, true><<<g, 256>>>((const v4u *)d, bytes / 16, sink); break;
                case 4: rd_chunk<4, true><<<g, 1024>>>(d, bytes, sink); break;
                case 5: rd_chunk<4, false><<<g, 1024>>>(d, bytes, sink); break;
                case 6: rd_chunk<16, true><<<g, 1024>>>(d, bytes, sink); break;
                case 7: rd_chunk<16, false><<<g, 1024>>>(d, bytes, sink); break;
                case 8: rd_ldsdma<true><<<g, 256>>>(d, bytes, sink); break;
                case 9: rd_ldsdma<false><<<g, 256>>>(d, bytes, sink); break;
                case 10: rd_chunk2<false, false><<<g, 1024>>>(d, bytes, sink); break;
                case 11: rd_chunk2<true, false><<<g, 1024>>>(d, bytes, sink); break;
                case 12: rd_chunk2<false, true><<<g, 1024>>>(d, bytes, sink); break;
                case 13: rd_chunk2<true, true><<<g, 1024>>>(d, bytes, sink); break;
                }
            };
            launch();
            CK(hipEventRecord(e0));
            for (int i = 0; i < reps; i++) launch();
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            t[v].push_back(ms / reps);
        }
    for (size_t v = 0; v < vs.size(); v++) {
        std::sort(t[v].begin(), t[v].end());
        float med = t[v][t[v].size() / 2], mn = t[v][0];
        printf("{\"variant\": \"%s\", \"GiB\": %zu, \"median_ms\": %.4f, \"GBps_median\": %.1f, \"GBps_best\": %.1f}\n", vs[v].name, bytes >> 30, med,
               bytes / (med * 1e-3) / 1e9, bytes / (mn * 1e-3) / 1e9);
    }
    return 0;
}
