// write_probe.hip — HBM write / copy bandwidth probe (tools only, not product).
// lc_build's run expansion writes the events of the dense blocks (16 B each,
// lane = event, a wave's stores one contiguous KiB) at ~4.3 TB/s of mixed
// traffic.  This probe measures what the chip gives
// to the same store shape with nothing else in the way:
//   mode 0  write-only, 16-B stores, grid-stride, default policy
//   mode 1  write-only, non-temporal stores
//   mode 2  copy (16-B load + 16-B store per lane), default policy
//   mode 3  write 16 B per lane, 8 B read per 8 lanes (lc_build's stash : event ratio of a run)
// Build: hipcc --offload-arch=gfx950 -O3 tools/write_probe.hip -o /tmp/write_probe
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

typedef uint32_t v4u __attribute__((ext_vector_type(4)));

template <int MODE>
__global__ __launch_bounds__(256) void wr(v4u *__restrict__ d, const v4u *__restrict__ s, uint64_t n16) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += stride) {
        v4u v = {(uint32_t)i, (uint32_t)(i >> 32), 7u, (uint32_t)i ^ 0x5a5a5a5au};
        if (MODE == 2) v = s[i];
        if (MODE == 3) {
            const uint64_t e = ((const uint64_t *)s)[i >> 3];
            v.z = (uint32_t)e;
        }
        if (MODE == 1) __builtin_nontemporal_store(v, d + i);
        else d[i] = v;
    }
}

int main() {
    const uint64_t bytes = 1ull << 30, n16 = bytes / 16;
    v4u *d, *s;
    CK(hipMalloc(&d, bytes));
    CK(hipMalloc(&s, bytes));
    CK(hipMemset(s, 1, bytes));
    CK(hipMemset(d, 0, bytes));
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, 0));
    const int cus = prop.multiProcessorCount;
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int mode = 0; mode < 4; mode++)
        for (int wpc : {8, 16, 32}) {  // workgroups of 256 per CU
            const int grid = cus * wpc;
            float best = 1e9f, sum = 0;
            for (int rep = 0; rep < 10; rep++) {
                CK(hipEventRecord(e0));
                if (mode == 0) hipLaunchKernelGGL(wr<0>, dim3(grid), dim3(256), 0, 0, d, s, n16);
                if (mode == 1) hipLaunchKernelGGL(wr<1>, dim3(grid), dim3(256), 0, 0, d, s, n16);
                if (mode == 2) hipLaunchKernelGGL(wr<2>, dim3(grid), dim3(256), 0, 0, d, s, n16);
                if (mode == 3) hipLaunchKernelGGL(wr<3>, dim3(grid), dim3(256), 0, 0, d, s, n16);
                CK(hipEventRecord(e1));
                CK(hipEventSynchronize(e1));
                float ms;
                CK(hipEventElapsedTime(&ms, e0, e1));
                if (rep >= 2) {
                    best = ms < best ? ms : best;
                    sum += ms;
                }
            }
            const double moved = (double)bytes * (mode == 2 ? 2.0 : mode == 3 ? 1.125 : 1.0);
            printf("{\"mode\": %d, \"wg_per_cu\": %d, \"best_ms\": %.4f, \"mean_ms\": %.4f, \"TBps_best\": %.3f}\n", mode,
                   wpc, best, sum / 8, moved / (best * 1e-3) / 1e12);
        }
    return 0;
}
