// copy_pool.hpp — persistent host threads for the staging copies of the
// host-memory entry points (jlcrc_api.hip par_memcpy); header-only so the CPU
// tests can drive it under ThreadSanitizer (tests/cpp/copy_pool_test.cpp).
#pragma once
#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstddef>
#include <cstdint>
#include <cstring>
#include <deque>
#include <mutex>
#include <thread>
#include <vector>

namespace jlhost {

// Persistent staging workers for pageable -> pinned copies (one core copies at
// ~10-20 GB/s, well under PCIe's ~55): a copy is cut into one piece per thread
// (at least 256 KiB) that the caller and up to JL_OPT_STAGE_THREADS - 1 pool
// threads take from a shared cursor.  Persistent threads, because starting
// threads per call (r3) cost more than a one-table copy itself, so r3 copied
// anything under 4 MiB on one core.  Idle workers spin for kSpinUs before they
// sleep, so back-to-back calls do not pay a futex wake-up per copy.  Concurrent
// callers queue their copies; every caller also works on its own.
class CopyPool {
  public:
    static constexpr size_t kMinPiece = 256u << 10;
    static constexpr double kSpinUs = 300.0;
    void copy(void *dst, const void *src, size_t n, int threads) {
        if (n < 2 * kMinPiece || threads <= 1) {
            memcpy(dst, src, n);
            return;
        }
        const size_t piece = std::max<size_t>(kMinPiece, ((n + threads - 1) / threads + 4095) & ~(size_t)4095);
        Job j{(char *)dst, (const char *)src, n, piece};
        {
            std::unique_lock<std::mutex> lk(mu_);
            // a thread that cannot be started (rlimit, a container's pid limit) must
            // not throw through the C ABI: the copy goes on with the threads running
            // (the caller alone if there are none); the spawn is retried at most once
            // a second, and the failures are counted (JL_INFO_STAGE_SPAWN_FAILURES)
            const auto now = std::chrono::steady_clock::now();
            if (failures_ && now - last_fail_ < std::chrono::seconds(1)) threads = (int)th_.size() + 1;
            while ((int)th_.size() < threads - 1 && (int)th_.size() < 63) {
                try {
                    th_.emplace_back([this] { work(); });
                } catch (...) {
                    failures_++;
                    last_fail_ = now;
                    break;
                }
            }
            live_.store((int)th_.size());
            th_count_.store((int)th_.size(), std::memory_order_relaxed);
            q_.push_back(&j);
            queued_.fetch_add(1);
        }
        cv_.notify_all();
        run(j);  // the caller copies too, then waits for the pieces others took
        // and for every worker to have left the job: j lives on this stack
        std::unique_lock<std::mutex> lk(mu_);
        done_.wait(lk, [&] { return j.left.load() == 0 && j.active == 0; });
        auto it = std::find(q_.begin(), q_.end(), &j);
        if (it != q_.end()) {
            q_.erase(it);
            queued_.fetch_sub(1);
        }
    }
    // a caller about to run on the host (the SSE4.2 path) stops the idle workers'
    // spinning: spinners share the caller's cores (SMT siblings) and slowed the
    // host path right after a device call, which misled the auto dispatch's probes
    void quiesce() { epoch_.fetch_add(1, std::memory_order_relaxed); }
    // a caller about to stage for the device wakes the sleeping workers first: they
    // spin (kSpinUs) while the call sets up, instead of taking the futex wake-up on
    // the copy's path (a device call right after host calls staged 8 MiB at ~22 GB/s,
    // one core's rate, r6zc)
    void prewake() {
        if (th_count_.load(std::memory_order_relaxed) == 0) return;  // no workers yet
        {
            std::lock_guard<std::mutex> lk(mu_);
            wake_++;
        }
        cv_.notify_all();
    }
    int workers() const { return live_.load(); }  // threads running
    int spawn_failures() {
        std::lock_guard<std::mutex> lk(mu_);
        return failures_;
    }
    ~CopyPool() {
        {
            std::lock_guard<std::mutex> lk(mu_);
            stop_ = true;
        }
        cv_.notify_all();
        for (auto &t : th_) t.join();
    }

  private:
    struct Job {
        char *dst;
        const char *src;
        size_t n, piece, pieces;
        std::atomic<size_t> next{0}, left{0};
        int active = 0;  // pool workers inside run(): guarded by mu_
        Job(char *d, const char *s, size_t n_, size_t pc) : dst(d), src(s), n(n_), piece(pc), pieces((n_ + pc - 1) / pc) {
            left = pieces;
        }
    };
    void run(Job &j) {  // copies pieces of j until none is left to take
        for (size_t i; (i = j.next.fetch_add(1)) < j.pieces;) {
            const size_t a = i * j.piece, b = std::min(j.n, a + j.piece);
            memcpy(j.dst + a, j.src + a, b - a);
            j.left.fetch_sub(1);
        }
    }
    void work() {
        std::unique_lock<std::mutex> lk(mu_);
        uint64_t seen = wake_;  // prewake() calls seen (guarded by mu_)
        for (;;) {
            if (q_.empty() && !stop_) {  // spin a while (unlocked) before sleeping
                lk.unlock();
                const auto t0 = std::chrono::steady_clock::now();
                const uint64_t e = epoch_.load(std::memory_order_relaxed);
                while (queued_.load() == 0 && epoch_.load(std::memory_order_relaxed) == e &&
                       std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() < kSpinUs)
                    __builtin_ia32_pause();
                lk.lock();
            }
            cv_.wait(lk, [&] { return stop_ || !q_.empty() || wake_ != seen; });
            if (stop_) return;
            seen = wake_;
            if (q_.empty()) continue;  // woken ahead of a copy: spin for it
            Job *j = q_.front();
            if (j->next.load() >= j->pieces) {  // every piece taken: the job leaves the queue
                q_.pop_front();
                queued_.fetch_sub(1);
                continue;
            }
            j->active++;  // its caller returns only once this worker has left it
            lk.unlock();
            run(*j);
            lk.lock();
            j->active--;
            done_.notify_all();
        }
    }
    std::mutex mu_;
    std::condition_variable cv_, done_;
    std::deque<Job *> q_;
    std::atomic<int> queued_{0};  // jobs in q_ (read by spinning workers without the lock)
    std::atomic<uint64_t> epoch_{0};  // quiesce() calls: a change ends the workers' spinning
    uint64_t wake_ = 0;                 // prewake() calls (guarded by mu_)
    std::atomic<int> th_count_{0};      // th_.size() for prewake's quick check
    std::vector<std::thread> th_;
    bool stop_ = false;
    int failures_ = 0;                                // threads that could not start (guarded by mu_)
    std::chrono::steady_clock::time_point last_fail_;  // guarded by mu_
    std::atomic<int> live_{0};                        // th_.size(), readable without the lock
};
}  // namespace jlhost
