// pin_probe.hip — what a host-memory call of the dispatch sizes pays to get its
// bytes onto the device, per source kind (anonymous pageable memory, a read-only
// file mapping like EnvImpl's mmap'd tables), per size:
//   reg    hipHostRegister (read-only flag first) + H2D from the registration + unregister
//   stage1 memcpy into pinned staging on the calling thread + H2D
//   stageN the engine's copy pool (copy_pool.hpp, N threads) into pinned staging + H2D
//   direct hipMemcpy straight from pageable memory (the runtime's own staging)
// plus the pool's plain memcpy rate and the process's CPU share.  Medians of reps.
// Build: hipcc -O2 --offload-arch=gfx950 -std=c++17 -o tools/pin_probe tools/pin_probe.hip -lpthread
#include <hip/hip_runtime.h>
#include <fcntl.h>
#include <sched.h>
#include <sys/mman.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <string>
#include <vector>

#include "../jleveldb_amd/csrc/copy_pool.hpp"

#define CK(x)                                                                      \
    do {                                                                           \
        hipError_t e_ = (x);                                                       \
        if (e_ != hipSuccess) {                                                    \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                \
            exit(1);                                                               \
        }                                                                          \
    } while (0)

static double now_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
static double median(std::vector<double> v) {
    std::sort(v.begin(), v.end());
    return v[v.size() / 2];
}

int main(int argc, char **argv) {
    const int threads = argc > 1 ? atoi(argv[1]) : 8;
    const char *path = argc > 2 ? argv[2] : "gpurun_out/pin_probe.bin";
    cpu_set_t cs;
    sched_getaffinity(0, sizeof(cs), &cs);
    std::string quota = "?";
    {
        std::ifstream f("/sys/fs/cgroup/cpu.max");
        if (f) std::getline(f, quota);
    }
    printf("{\"affinity_cpus\": %d, \"cgroup_cpu_max\": \"%s\", \"threads\": %d}\n", CPU_COUNT(&cs), quota.c_str(), threads);
    const size_t maxb = 64u << 20;
    // sources
    uint8_t *anon = (uint8_t *)aligned_alloc(4096, maxb);
    for (size_t i = 0; i < maxb; i++) anon[i] = (uint8_t)(i * 131 + 7);
    {
        int fd = open(path, O_CREAT | O_TRUNC | O_WRONLY, 0644);
        if (fd < 0 || write(fd, anon, maxb) != (ssize_t)maxb) {
            perror("write file");
            return 1;
        }
        close(fd);
    }
    int fd = open(path, O_RDONLY);
    uint8_t *fmap = (uint8_t *)mmap(nullptr, maxb, PROT_READ, MAP_SHARED, fd, 0);
    if (fmap == MAP_FAILED) {
        perror("mmap");
        return 1;
    }
    volatile uint64_t sink = 0;
    for (size_t i = 0; i < maxb; i += 4096) sink += fmap[i];  // fault the mapping in
    CK(hipSetDevice(0));
    void *dev = nullptr, *pin = nullptr;
    CK(hipMalloc(&dev, maxb));
    CK(hipHostMalloc(&pin, maxb, hipHostMallocDefault));
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    jlhost::CopyPool pool;
    const size_t sizes[] = {256u << 10, 1u << 20, 2u << 20, 4u << 20, 8u << 20, 16u << 20, 64u << 20};
    for (int s = 0; s < 2; s++) {
        uint8_t *src = s ? fmap : anon;
        const char *kind = s ? "file_mmap" : "anon";
        for (size_t n : sizes) {
            const int reps = n <= (4u << 20) ? 30 : 10;
            std::vector<double> reg, reg_r, reg_c, reg_u, st1, stN, dir, cp1, cpN, rp[3];
            bool reg_ok = true;
            for (int r = 0; r < reps + 2; r++) {
                const bool keep = r >= 2;
                // reg
                double t0 = now_us();
                hipError_t e = hipHostRegister(src, n, hipHostRegisterReadOnly);
                if (e != hipSuccess) {
                    (void)hipGetLastError();
                    e = hipHostRegister(src, n, hipHostRegisterDefault);
                }
                if (e != hipSuccess) {
                    (void)hipGetLastError();
                    reg_ok = false;
                }
                double t1 = now_us();
                if (reg_ok) {
                    CK(hipMemcpyAsync(dev, src, n, hipMemcpyHostToDevice, st));
                    CK(hipStreamSynchronize(st));
                }
                double t2 = now_us();
                if (reg_ok) CK(hipHostUnregister(src));
                double t3 = now_us();
                if (keep && reg_ok) {
                    reg.push_back(t3 - t0);
                    reg_r.push_back(t1 - t0);
                    reg_c.push_back(t2 - t1);
                    reg_u.push_back(t3 - t2);
                }
                // stage1
                t0 = now_us();
                memcpy(pin, src, n);
                t1 = now_us();
                CK(hipMemcpyAsync(dev, pin, n, hipMemcpyHostToDevice, st));
                CK(hipStreamSynchronize(st));
                t2 = now_us();
                if (keep) {
                    st1.push_back(t2 - t0);
                    cp1.push_back(t1 - t0);
                }
                // stageN
                t0 = now_us();
                pool.copy(pin, src, n, threads);
                t1 = now_us();
                CK(hipMemcpyAsync(dev, pin, n, hipMemcpyHostToDevice, st));
                CK(hipStreamSynchronize(st));
                t2 = now_us();
                if (keep) {
                    stN.push_back(t2 - t0);
                    cpN.push_back(t1 - t0);
                }
                // registered in pieces of 256 KiB / 512 KiB / 1 MiB, each DMA'd once registered
                for (int k = 0; k < 3; k++) {
                    const size_t pc = (256u << 10) << k;
                    t0 = now_us();
                    bool ok = true;
                    for (size_t a = 0; a < n && ok; a += pc) {
                        const size_t m = std::min(pc, n - a);
                        hipError_t e2 = hipHostRegister(src + a, m, hipHostRegisterReadOnly);
                        if (e2 != hipSuccess) {
                            (void)hipGetLastError();
                            e2 = hipHostRegister(src + a, m, hipHostRegisterDefault);
                        }
                        if (e2 != hipSuccess) {
                            (void)hipGetLastError();
                            ok = false;
                            break;
                        }
                        CK(hipMemcpyAsync((char *)dev + a, src + a, m, hipMemcpyHostToDevice, st));
                    }
                    CK(hipStreamSynchronize(st));
                    for (size_t a = 0; a < n && ok; a += pc) CK(hipHostUnregister(src + a));
                    t1 = now_us();
                    if (keep) rp[k].push_back(ok ? t1 - t0 : -1.0);
                }
                // direct from pageable
                t0 = now_us();
                CK(hipMemcpy(dev, src, n, hipMemcpyHostToDevice));
                t1 = now_us();
                if (keep) dir.push_back(t1 - t0);
            }
            printf("{\"src\": \"%s\", \"MiB\": %.2f, \"reg_us\": %.1f, \"reg_register_us\": %.1f, \"reg_h2d_us\": %.1f, "
                   "\"reg_unregister_us\": %.1f, \"stage1_us\": %.1f, \"stageN_us\": %.1f, \"direct_us\": %.1f, "
                   "\"memcpy1_GBps\": %.1f, \"memcpyN_GBps\": %.1f, \"reg_ok\": %d, \"reg_pieces_256K_512K_1M_us\": [%.1f, %.1f, %.1f]}\n",
                   kind, n / 1048576.0, reg_ok ? median(reg) : -1, reg_ok ? median(reg_r) : -1, reg_ok ? median(reg_c) : -1,
                   reg_ok ? median(reg_u) : -1, median(st1), median(stN), median(dir), n / median(cp1) / 1e3,
                   n / median(cpN) / 1e3, (int)reg_ok, median(rp[0]), median(rp[1]), median(rp[2]));
            fflush(stdout);
        }
    }
    munmap(fmap, maxb);
    close(fd);
    unlink(path);
    return (int)(sink & 0);
}
