// dense_probe.hip — feasibility probe for dense WAL blocks (tools only, not product).
// lc_dense stages each 32 KiB block in LDS and checks one record per thread
// through 5-bit tables (7 lookups and ~19 VALU per dword: both the LDS and VALU
// pipes are busy).  This probe measures the other arrangement:
// no staged block, each thread reads its record's bytes with unaligned 16-B
// global loads (neighbouring records share lines through L2), and the LDS holds
// only the slicing-by-4 byte tables replicated per lane ([byte][lane & 31], 128
// KiB, conflict-free, one v_perm per lookup as in the 4 KiB kernel): 4 lookups
// and ~6 VALU per dword.
// Records: DBBench-shaped, one every 138 B (7-B header + 131-B payload), crc
// range 132 B from header + 6.  Checks the chains of the first records against
// the host, then times the whole 4 GiB.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/dense_probe.hip -o /tmp/dense_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                  \
    do {                                                                       \
        hipError_t e = (x);                                                    \
        if (e != hipSuccess) {                                                 \
            printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__);           \
            exit(1);                                                           \
        }                                                                      \
    } while (0)

typedef uint32_t v4u __attribute__((ext_vector_type(4)));
typedef v4u __attribute__((aligned(4))) v4u_a4;  // 4-B aligned 16-B loads

constexpr uint32_t kRec = 138, kOff = 6, kDw = 34;  // 132 B from a 4-B aligned start: 34 dwords
constexpr uint32_t kLds = 32768;                     // 128 KiB

__device__ __forceinline__ uint32_t gaddr(uint32_t L, uint32_t x, uint32_t k) {
    return __builtin_amdgcn_perm(L, x, 0x0C060004u | (k << 8));
}
__device__ __forceinline__ uint32_t lds_at(const uint32_t *lds, uint32_t byte_addr) {
    return *(const uint32_t *)((const char *)lds + byte_addr);
}
struct Lanes {
    uint32_t l3, l2, l1, l0;
    __device__ explicit Lanes(uint32_t lane) {
        const uint32_t l4 = (lane & 31u) << 2;
        l3 = 0x10000u | 0x80u | l4;
        l2 = 0x10000u | l4;
        l1 = 0x80u | l4;
        l0 = l4;
    }
};
// s' = T3[x.b0] ^ T2[x.b1] ^ T1[x.b2] ^ T0[x.b3], x = s ^ d
__device__ __forceinline__ uint32_t step(const uint32_t *lds, const Lanes &g, uint32_t s, uint32_t d) {
    const uint32_t x = s ^ d;
    const uint32_t v0 = lds_at(lds, gaddr(g.l3, x, 0u)), v1 = lds_at(lds, gaddr(g.l2, x, 1u));
    const uint32_t v2 = lds_at(lds, gaddr(g.l1, x, 2u)), v3 = lds_at(lds, gaddr(g.l0, x, 3u));
    return (v0 ^ v1) ^ (v2 ^ v3);
}

// MODE 0: one record at a time; 1: the next record's loads issued before this one's steps.
// wrap: records taken modulo `wrap` (a window that stays in L2: the load path alone)
template <int MODE>
__global__ __launch_bounds__(1024) void probe(const uint8_t *__restrict__ log, const uint32_t *__restrict__ img,
                                              uint64_t nrec, uint32_t *__restrict__ out, int write_all,
                                              uint64_t wrap = ~0ull) {
    __shared__ uint32_t lds[kLds];
    for (uint32_t i = threadIdx.x; i < kLds; i += blockDim.x) lds[i] = img[i];
    __syncthreads();
    const Lanes g(threadIdx.x & 63u);
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t acc = 0;
    auto ld = [&](uint64_t rr, v4u *w) {
        const uint8_t *a = log + (((rr % wrap) * kRec + kOff) & ~3ull);
#pragma unroll
        for (int j = 0; j < 9; j++) w[j] = *(const v4u_a4 *)(a + 16 * j);
    };
    auto run = [&](const v4u *w) {
        uint32_t s = 0xffffffffu;
#pragma unroll
        for (int j = 0; j < (int)kDw; j++) s = step(lds, g, s, w[j >> 2][j & 3]);
        return s;
    };
    if (MODE == 0) {
        for (; r < nrec; r += stride) {
            v4u w[9];
            ld(r, w);
            const uint32_t s = run(w);
            if (write_all) out[r] = s;
            acc ^= s;
        }
    } else {
        v4u w[9], n[9];
        if (r < nrec) ld(r, w);
        for (; r < nrec; r += stride) {
            if (r + stride < nrec) ld(r + stride, n);
            const uint32_t s = run(w);
            if (write_all) out[r] = s;
            acc ^= s;
#pragma unroll
            for (int j = 0; j < 9; j++) w[j] = n[j];
        }
    }
    if (!write_all && acc == 0x12345678u) out[0] = acc;
}

__global__ void fill(uint64_t *p, uint64_t n, uint64_t seed) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        uint64_t z = seed + (i + 1) * 0x9E3779B97F4A7C15ull;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        p[i] = z ^ (z >> 31);
    }
}

int main(int argc, char **argv) {
    const uint64_t bytes = 4ull << 30;
    const uint64_t nrec = (bytes - 64) / kRec;
    uint32_t T[4][256];
    for (uint32_t i = 0; i < 256; i++) {
        uint32_t c = i;
        for (int k = 0; k < 8; k++) c = (c >> 1) ^ (0x82F63B78u & (0u - (c & 1u)));
        T[0][i] = c;
    }
    for (int t = 1; t < 4; t++)
        for (uint32_t i = 0; i < 256; i++) T[t][i] = (T[t - 1][i] >> 8) ^ T[0][T[t - 1][i] & 0xffu];
    std::vector<uint32_t> img(kLds);
    for (int t = 0; t < 4; t++)  // table t at region t >> 1, half t & 1: [byte][lane]
        for (uint32_t b = 0; b < 256; b++)
            for (uint32_t l = 0; l < 32; l++) img[(t >> 1) * 16384 + b * 64 + (t & 1) * 32 + l] = T[t][b];
    uint8_t *log;
    uint32_t *dimg, *out;
    CK(hipMalloc(&log, bytes));
    CK(hipMalloc(&dimg, kLds * 4));
    CK(hipMalloc(&out, nrec * 4));
    CK(hipMemcpy(dimg, img.data(), kLds * 4, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, (uint64_t *)log, bytes / 8, 7ull);
    CK(hipDeviceSynchronize());
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, 0));
    const int cus = prop.multiProcessorCount;
    // check: the first 4096 records' chains against the host
    const uint64_t nchk = 4096;
    std::vector<uint8_t> hl(nchk * kRec + 64);
    CK(hipMemcpy(hl.data(), log, hl.size(), hipMemcpyDeviceToHost));
    for (int mode = 0; mode < 2; mode++) {
        CK(hipMemset(out, 0, nchk * 4));
        if (mode == 0)
            hipLaunchKernelGGL(probe<0>, dim3(4), dim3(1024), 0, 0, log, dimg, nchk, out, 1, ~0ull);
        else
            hipLaunchKernelGGL(probe<1>, dim3(4), dim3(1024), 0, 0, log, dimg, nchk, out, 1, ~0ull);
        CK(hipDeviceSynchronize());
        std::vector<uint32_t> got(nchk);
        CK(hipMemcpy(got.data(), out, nchk * 4, hipMemcpyDeviceToHost));
        uint64_t bad = 0;
        for (uint64_t r = 0; r < nchk; r++) {
            const uint8_t *a = hl.data() + ((r * kRec + kOff) & ~3ull);
            uint32_t s = 0xffffffffu;
            for (uint32_t j = 0; j < kDw; j++) {
                uint32_t d;
                memcpy(&d, a + 4 * j, 4);
                const uint32_t x = s ^ d;
                s = T[3][x & 0xff] ^ T[2][(x >> 8) & 0xff] ^ T[1][(x >> 16) & 0xff] ^ T[0][x >> 24];
            }
            bad += s != got[r];
        }
        printf("{\"check_mode\": %d, \"records\": %llu, \"mismatches\": %llu}\n", mode, (unsigned long long)nchk,
               (unsigned long long)bad);
    }
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int mode = 0; mode < 4; mode++)
        for (int wpc : {1}) {  // workgroups of 1024 threads per CU (128 KiB of LDS: one per CU)
            const int grid = cus * wpc;
            // modes 2 / 3: as 1, records modulo a 2 MiB / 32 MiB window (L2 / Infinity Cache resident)
            const uint64_t wrap = mode == 2 ? (2u << 20) / kRec : mode == 3 ? (32u << 20) / kRec : ~0ull;
            float best = 1e9f, sum = 0;
            for (int rep = 0; rep < 8; rep++) {
                CK(hipEventRecord(e0));
                if (mode == 0)
                    hipLaunchKernelGGL(probe<0>, dim3(grid), dim3(1024), 0, 0, log, dimg, nrec, out, 0, ~0ull);
                else
                    hipLaunchKernelGGL(probe<1>, dim3(grid), dim3(1024), 0, 0, log, dimg, nrec, out, 0, wrap);
                CK(hipEventRecord(e1));
                CK(hipEventSynchronize(e1));
                float ms;
                CK(hipEventElapsedTime(&ms, e0, e1));
                if (rep >= 2) {
                    best = ms < best ? ms : best;
                    sum += ms;
                }
            }
            printf("{\"mode\": %d, \"grid\": %d, \"records\": %llu, \"best_ms\": %.4f, \"mean_ms\": %.4f}\n", mode, grid,
                   (unsigned long long)nrec, best, sum / 6);
        }
    return 0;
}
