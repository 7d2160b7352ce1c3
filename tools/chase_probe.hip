// chase_probe.hip — dependent random-line load rate (tools only, not product).
// lc_walk follows one chain of dependent 8-B header loads per 32 KiB block (one
// lane per block, two 256-lane workgroups per CU because of its LDS), ~4.17 M
// distinct lines in ~125 us on the C5 1 056-B set.  Is that the rate of random
// lines the chip gives, or the chains' memory-level parallelism?  Each lane runs
// C independent chains of H dependent loads (an address from a hash of the
// step, made to depend on the loaded value through an opaque zero), 8-B
// non-temporal loads at random places of a 4 GiB buffer, in workgroups of 256
// that hold `lds` KiB of LDS (80: two per CU, as lc_walk).
// Build: hipcc --offload-arch=gfx950 -O3 tools/chase_probe.hip -o /tmp/chase_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                  \
    do {                                                                       \
        hipError_t e = (x);                                                    \
        if (e != hipSuccess) {                                                 \
            printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__);           \
            exit(1);                                                           \
        }                                                                      \
    } while (0)

__device__ __forceinline__ uint64_t mix(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
__device__ __forceinline__ uint64_t hop(const uint8_t *p) {
    uint64_t v;
    asm volatile("global_load_dwordx2 %0, %1, off nt\n\ts_waitcnt vmcnt(0)" : "=v"(v) : "v"(p) : "memory");
    return v;
}
__device__ __forceinline__ uint64_t hop_nowait(const uint8_t *p) {
    uint64_t v;
    asm volatile("global_load_dwordx2 %0, %1, off nt" : "=v"(v) : "v"(p) : "memory");
    return v;
}
__device__ __forceinline__ uint32_t opaque_zero(uint64_t v) {
    uint32_t z;
    asm volatile("v_and_b32 %0, 0, %1" : "=v"(z) : "v"((uint32_t)v));
    return z;
}

template <int C>
__global__ __launch_bounds__(256) void chase(const uint8_t *__restrict__ buf, uint64_t bytes, int H, uint32_t *sink) {
    extern __shared__ uint32_t pad[];
    const uint64_t lane = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t z[C];
    uint64_t acc = 0;
#pragma unroll
    for (int c = 0; c < C; c++) z[c] = 0;
    for (int h = 0; h < H; h++) {
        uint64_t v[C];
#pragma unroll
        for (int c = 0; c < C; c++) {
            const uint64_t a = (mix(lane * 977 + (uint64_t)h * 131 + c * 7919) % (bytes - 16)) + z[c];
            v[c] = C == 1 ? hop(buf + a) : hop_nowait(buf + a);
        }
        if (C > 1) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
        for (int c = 0; c < C; c++) {
            z[c] = opaque_zero(v[c]);
            acc += v[c];
        }
    }
    if (acc == 0x1234567890abcdefull) sink[0] = (uint32_t)acc + pad[0];
}

int main() {
    const uint64_t bytes = 4ull << 30;
    uint8_t *buf;
    uint32_t *sink;
    CK(hipMalloc(&buf, bytes));
    CK(hipMalloc(&sink, 64));
    CK(hipMemset(buf, 3, bytes));
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, 0));
    const int cus = prop.multiProcessorCount;
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int H = 32;
    for (int lds_kib : {80, 40, 20})
        for (int C : {1, 2, 4}) {
            const int grid = 512;  // 131 072 lanes, as lc_walk on a 4 GiB log
            const size_t sh = (size_t)lds_kib * 1024;
            if (C == 1) CK(hipFuncSetAttribute((const void *)chase<1>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)sh));
            if (C == 2) CK(hipFuncSetAttribute((const void *)chase<2>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)sh));
            if (C == 4) CK(hipFuncSetAttribute((const void *)chase<4>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)sh));
            float best = 1e9f;
            for (int rep = 0; rep < 6; rep++) {
                CK(hipEventRecord(e0));
                if (C == 1) hipLaunchKernelGGL(chase<1>, dim3(grid), dim3(256), sh, 0, buf, bytes, H, sink);
                if (C == 2) hipLaunchKernelGGL(chase<2>, dim3(grid), dim3(256), sh, 0, buf, bytes, H / 2, sink);
                if (C == 4) hipLaunchKernelGGL(chase<4>, dim3(grid), dim3(256), sh, 0, buf, bytes, H / 4, sink);
                CK(hipGetLastError());
                CK(hipEventRecord(e1));
                CK(hipEventSynchronize(e1));
                float ms;
                CK(hipEventElapsedTime(&ms, e0, e1));
                if (rep >= 1) best = ms < best ? ms : best;
            }
            const double loads = (double)grid * 256 * H;  // the same loads in every mode
            printf("{\"lds_kib\": %d, \"chains_per_lane\": %d, \"lanes\": %d, \"loads\": %.0f, \"best_us\": %.1f, "
                   "\"G_lines_per_s\": %.2f, \"cus\": %d}\n",
                   lds_kib, C, grid * 256, loads, best * 1e3, loads / (best * 1e-3) / 1e9, cus);
        }
    return 0;
}
