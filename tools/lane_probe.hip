// lane_probe.hip — read-rate probe for the log-verify load shapes (tools only,
// not product).  A group of LPB lanes streams one 32 KiB log block, 16 B per
// lane and step (LPB*16 B of the block per wave-instruction), 64/LPB blocks per
// wave, 8 loads in flight per lane; optional per-group phase stagger (the
// group starts at step (g*STAG) mod S and wraps) to test address aliasing of
// blocks that sit 32 KiB apart.
// Build: hipcc --offload-arch=gfx950 -O3 tools/lane_probe.hip -o tools/lane_probe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                      \
    do {                                                                           \
        hipError_t e = (x);                                                        \
        if (e != hipSuccess) {                                                     \
            printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__);                \
            exit(1);                                                               \
        }                                                                          \
    } while (0)

typedef uint32_t v4u __attribute__((ext_vector_type(4)));

template <int LPB, int STAG, int THREADS>
__global__ __launch_bounds__(THREADS) void rd_groups(const uint8_t *__restrict__ s, uint64_t n_blocks, uint32_t *sink) {
    constexpr int STEP = 16 * LPB, S = 32768 / STEP, G = 64 / LPB;
    const uint32_t lane = threadIdx.x & 63, grp = lane / LPB, l = lane % LPB;
    const uint64_t waves = (uint64_t)gridDim.x * (THREADS / 64);
    const uint64_t w = (uint64_t)blockIdx.x * (THREADS / 64) + (threadIdx.x >> 6);
    v4u acc = {0, 0, 0, 0};
    for (uint64_t b0 = w * G; b0 < n_blocks; b0 += waves * G) {
        const uint64_t b = b0 + grp < n_blocks ? b0 + grp : b0;
        const uint8_t *p = s + b * 32768u + 16u * l;
        const uint32_t ph = (uint32_t)((grp * STAG) % S);
        v4u t[8];
#pragma unroll
        for (int k = 0; k < 8; k++) t[k] = __builtin_nontemporal_load((const v4u *)(p + ((k + ph) % S) * STEP));
        for (int s0 = 0; s0 < S; s0 += 8) {
#pragma unroll
            for (int k = 0; k < 8; k++) {
                acc ^= t[k];
                const int nx = s0 + 8 + k;
                if (nx < S) t[k] = __builtin_nontemporal_load((const v4u *)(p + ((nx + ph) % S) * STEP));
            }
        }
    }
    if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u) atomicAdd(sink, 1u);
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
    const size_t bytes = (size_t)4 << 30;
    const uint64_t nb = bytes / 32768;
    uint8_t *d;
    uint32_t *sink;
    CK(hipMalloc(&d, bytes));
    CK(hipMalloc(&sink, 4));
    fill_rand<<<4096, 256>>>((uint64_t *)d, bytes / 8);
    CK(hipDeviceSynchronize());
    hipDeviceProp_t p;
    CK(hipGetDeviceProperties(&p, 0));
    const int cu = p.multiProcessorCount;
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    struct V {
        const char *name;
        void (*launch)(const uint8_t *, uint64_t, uint32_t *, int);
    };
#define JL_V(L, ST, T)                                                                                    \
    V {                                                                                                   \
        "lpb" #L "_stag" #ST "_t" #T, [](const uint8_t *a, uint64_t n, uint32_t *k, int c) {               \
            rd_groups<L, ST, T><<<c, T>>>(a, n, k);                                                       \
        }                                                                                                 \
    }
    std::vector<V> vs = {JL_V(1, 0, 512),  JL_V(1, 0, 1024), JL_V(1, 37, 512), JL_V(1, 37, 1024),
                         JL_V(2, 0, 512),  JL_V(2, 0, 1024), JL_V(2, 37, 1024), JL_V(4, 0, 512),
                         JL_V(4, 0, 1024), JL_V(4, 37, 1024), JL_V(8, 0, 512),  JL_V(8, 0, 1024)};
    const int rounds = argc > 1 ? atoi(argv[1]) : 5, reps = argc > 2 ? atoi(argv[2]) : 5;
    std::vector<std::vector<float>> t(vs.size());
    for (int r = 0; r < rounds; r++)
        for (size_t v = 0; v < vs.size(); v++) {
            vs[v].launch(d, nb, sink, cu);
            CK(hipEventRecord(e0));
            for (int i = 0; i < reps; i++) vs[v].launch(d, nb, sink, cu);
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            t[v].push_back(ms / reps);
        }
    for (size_t v = 0; v < vs.size(); v++) {
        std::sort(t[v].begin(), t[v].end());
        const float med = t[v][t[v].size() / 2], mn = t[v][0];
        printf("{\"variant\": \"%s\", \"median_ms\": %.4f, \"GBps_median\": %.1f, \"GBps_best\": %.1f}\n", vs[v].name,
               med, bytes / (med * 1e-3) / 1e9, bytes / (mn * 1e-3) / 1e9);
    }
    return 0;
}
