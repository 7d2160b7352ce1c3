// copy_pool_test.cpp — the staging copy pool (jleveldb_amd/csrc/copy_pool.hpp)
// under a sanitizer: concurrent callers with copies of every size class (below
// the split threshold, a few pieces, many pieces, ragged tails), each result
// compared byte for byte, callers' buffers on their own stacks / heaps and
// released right after the call (r4: a late worker's cursor update hit a
// returned caller's stack frame).  Test infrastructure only.
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#include "../../jleveldb_amd/csrc/copy_pool.hpp"

int main(int argc, char **argv) {
    const int iters = argc > 1 ? atoi(argv[1]) : 300;
    jlhost::CopyPool pool;
    std::atomic<int> bad{0};
    auto caller = [&](int id) {
        uint64_t rng = 0x9E3779B97F4A7C15ull * (id + 1);
        auto rnd = [&] {
            rng ^= rng << 13;
            rng ^= rng >> 7;
            rng ^= rng << 17;
            return rng;
        };
        for (int it = 0; it < iters; it++) {
            static const size_t sizes[] = {1, 4096, (256u << 10) - 1, 512u << 10, (1u << 20) + 17, 3u << 20};
            const size_t n = sizes[rnd() % 6] + rnd() % 4096;
            std::vector<uint8_t> src(n), dst(n, 0xee);
            for (size_t i = 0; i < n; i += 8) src[i] = (uint8_t)(rnd() >> 11);
            // the dispatch's hints around the copies: a host-path call ends the
            // workers' spinning, a device-path call wakes them ahead of its copy
            if (rnd() % 3 == 0) pool.quiesce();
            if (rnd() % 3 == 0) pool.prewake();
            pool.copy(dst.data(), src.data(), n, 1 + (int)(rnd() % 8));
            if (memcmp(dst.data(), src.data(), n) != 0) bad++;
        }
    };
    std::vector<std::thread> th;
    for (int t = 0; t < 4; t++) th.emplace_back(caller, t);
    for (auto &t : th) t.join();
    if (bad) {
        fprintf(stderr, "FAILED %d copies differ\n", bad.load());
        return 1;
    }
    printf("OK\n");
    return 0;
}
