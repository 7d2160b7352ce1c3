// hwid_probe.hip — where a persistent 4-workgroups-per-CU grid's waves land
// (tools only, not product): every wave of a lc_dense-shaped launch (256
// threads, ~38 KiB of LDS) records HW_ID (s_getreg); the host prints, per
// (XCC, SE, CU), the workgroup slots (TG_ID) and each workgroup's SIMD of
// waves 0..3, and how often the four workgroups' wave 0 share a SIMD.
// Build: hipcc --offload-arch=gfx950 -O3 tools/hwid_probe.hip -o tools/hwid_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <map>
#include <tuple>
#include <vector>

#define CK(x)                                                       \
    do {                                                            \
        hipError_t e = (x);                                         \
        if (e != hipSuccess) {                                      \
            printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); \
            exit(1);                                                \
        }                                                           \
    } while (0)

__global__ __launch_bounds__(256) void probe(uint32_t *out, uint32_t *xcc) {
    __shared__ uint32_t pad[9600];
    const uint32_t t = threadIdx.x;
    pad[t] = t;
    __syncthreads();
    const uint32_t hw = __builtin_amdgcn_s_getreg((31 << 11) | (0 << 6) | 4);   // HW_REG_HW_ID
    const uint32_t xc = __builtin_amdgcn_s_getreg((31 << 11) | (0 << 6) | 20);  // HW_REG_XCC_ID
    // keep the workgroup resident a while so the grid's workgroups are co-resident
    uint64_t t0 = __builtin_amdgcn_s_memtime();
    while (__builtin_amdgcn_s_memtime() - t0 < 200000) __builtin_amdgcn_s_sleep(10);
    if ((t & 63) == 0) {
        out[blockIdx.x * 4 + t / 64] = hw + pad[(t + 1) & 255] * 0;
        xcc[blockIdx.x * 4 + t / 64] = xc;
    }
}

int main() {
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const int G = cus * 4;
    uint32_t *d, *x;
    CK(hipMalloc(&d, G * 16));
    CK(hipMalloc(&x, G * 16));
    hipLaunchKernelGGL(probe, dim3(G), dim3(256), 0, 0, d, x);
    CK(hipDeviceSynchronize());
    std::vector<uint32_t> h(G * 4), hx(G * 4);
    CK(hipMemcpy(h.data(), d, G * 16, hipMemcpyDeviceToHost));
    CK(hipMemcpy(hx.data(), x, G * 16, hipMemcpyDeviceToHost));
    // HW_ID (gfx9): wave 3:0, simd 5:4, pipe 7:6, cu 11:8, sh 12, se 15:13, tg 19:16
    std::map<std::tuple<int, int, int, int>, std::vector<int>> per_cu;
    int distinct_wave_simds = 0;
    for (int b = 0; b < G; b++) {
        const uint32_t w = h[b * 4];
        per_cu[{(int)(hx[b * 4] & 15), (int)((w >> 13) & 7), (int)((w >> 12) & 1), (int)((w >> 8) & 15)}].push_back(b);
        int m = 0;
        for (int k = 0; k < 4; k++) m |= 1 << ((h[b * 4 + k] >> 4) & 3);
        distinct_wave_simds += m == 15;
    }
    int shared0 = 0, tg_distinct = 0, n = 0;
    for (auto &kv : per_cu) {
        int m0 = 0, tgm = 0;
        bool same = false;
        for (int b : kv.second) {
            const int s0 = (h[b * 4] >> 4) & 3, tg = (h[b * 4] >> 16) & 15;
            if (m0 & (1 << s0)) same = true;
            m0 |= 1 << s0;
            tgm |= 1 << (tg & 3);
        }
        shared0 += same;
        tg_distinct += tgm == 15;
        if (n < 6) {
            printf("xcc %d se %d sh %d cu %d:", std::get<0>(kv.first), std::get<1>(kv.first), std::get<2>(kv.first),
                   std::get<3>(kv.first));
            for (int b : kv.second) {
                printf("  wg %d tg %d simd", b, (h[b * 4] >> 16) & 15);
                for (int k = 0; k < 4; k++) printf(" %d", (h[b * 4 + k] >> 4) & 3);
            }
            printf("\n");
        }
        n++;
    }
    printf("{\"cus_seen\": %d, \"wgs\": %d, \"wgs_waves_on_4_simds\": %d, \"cus_wave0_shared_simd\": %d, "
           "\"cus_tg_mod4_distinct\": %d}\n",
           n, G, distinct_wave_simds, shared0, tg_distinct);
    return 0;
}
