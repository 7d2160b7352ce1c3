// jlcrc_api.hip — C-ABI of the engine (include/jlcrc.h): device context,
// launches, host staging and the caller shims for the four reference call sites.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/jlcrc.h"
#include "crc_math.hpp"
#include "copy_pool.hpp"
#include "host_paths.hpp"
#include "jlcrc_kernels.hpp"

#ifndef JL_STUDY
#define JL_STUDY 0
#endif

static_assert(jlmath::kImageBytes == jlk::kImageBytes, "LDS image size mismatch");
static_assert(sizeof(jl_log_event) == sizeof(jlk::LogEvent), "event layout mismatch");
static_assert(jlmath::kLSMaskDword * 4 == jlk::kLSMaskByte && jlmath::kLSStageDword * 4 == jlk::kLSStageByte &&
                  jlmath::kLSLaneDword * 4 == jlk::kLSLaneByte && jlmath::kLSShiftDword * 4 == jlk::kLSShiftByte &&
                  jlmath::kLSEDword * 4 == jlk::kLSEByte,
              "log-stream image layout mismatch");
static_assert(jlmath::kG4SelDword * 4 == jlk::kG4SelByte && jlmath::kLCMDword * 4 == 16384 && jlmath::kLCSelDword * 4 == 30720,
              "gv4 image layout mismatch");
static_assert(jlmath::kAuxZW == 5648 && jlmath::kAuxZB == 5648 + 256 * 128, "aux layout mismatch (log_chunks.hip)");
static_assert(jlmath::kV4SlotDword == jlk::kV4SlotDword && jlmath::kV4UDword * 4 == jlk::kV4U4Byte, "v4 image layout mismatch");

namespace {

thread_local std::string g_err;

int fail(int code, const std::string &msg) {
    g_err = msg;
    return code;
}

#define JL_HIP(call)                                                                                   \
    do {                                                                                               \
        hipError_t e_ = (call);                                                                        \
        if (e_ != hipSuccess)                                                                          \
            return fail(JL_ERR_HIP, std::string(#call) + ": " + hipGetErrorString(e_));               \
    } while (0)

// Grow-only device buffer.
struct DevBuf {
    void *p = nullptr;
    size_t cap = 0;
    hipError_t ensure(size_t bytes) {
        if (bytes <= cap) return hipSuccess;
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
        size_t want = std::max<size_t>(bytes, 4096);
        hipError_t e = hipMalloc(&p, want);
        if (e == hipSuccess) cap = want;
        return e;
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
    }
};

// Grow-only pinned host buffer.
struct PinBuf {
    void *p = nullptr;
    size_t cap = 0;
    unsigned flags = hipHostMallocDefault;  // hipHostMallocCoherent: written by kernels, read by the host
    hipError_t ensure(size_t bytes) {
        if (bytes <= cap) return hipSuccess;
        if (p) (void)hipHostFree(p);
        p = nullptr;
        cap = 0;
        size_t want = std::max<size_t>(bytes, 4096);
        hipError_t e = hipHostMalloc(&p, want, flags);
        if (e == hipSuccess) cap = want;
        return e;
    }
    void release() {
        if (p) (void)hipHostFree(p);
        p = nullptr;
        cap = 0;
    }
};

// One half of a double-buffered host -> device pipeline: the device chunk and
// its descriptors, pinned staging for pageable sources, a copy stream and two
// events.  `copied`: the slot's H2D copies have landed; `used`: the compute and
// copy-out that read the slot are done (the next copy into it waits for that).
struct Slot {
    DevBuf d_in, d_desc, d_out;  // chunk bytes, packed descriptor arrays, results
    void *part[4] = {nullptr, nullptr, nullptr, nullptr};  // the descriptor arrays inside d_desc
    PinBuf h_data, h_desc, h_out;  // h_out: a log chunk's events on their way to the caller's array
    hipStream_t st = nullptr;
    hipEvent_t copied = nullptr, used = nullptr;
};

// Per-thread workspace of the entry points that stage host memory or keep
// scratch between launches (log verification).  Every calling thread has its
// own streams, staging and scratch, so concurrent callers neither share
// buffers nor serialise on a lock (r1 had one process-wide mutex).  Created on
// a thread's first call; released when the thread exits or by jl_shutdown.
struct Workspace {
    hipStream_t stream = nullptr;  // compute stream of the host-memory entry points
    DevBuf ws_lc, ws_slot, ws_desc, ws_big, ws_part, ws_tmp, ws_stash;  // chunked log verify (log_chunks.hip)
    DevBuf ws_ls, ws_lsev;  // fused log verify: per-block counts / first failures, event slots
    DevBuf ws_small;        // one-launch small-log verify (lc_small): ticket counter, look-back statuses
    // jl_log_verify of a small log: lc_small writes the events here (fine-grained
    // pinned memory: its stores reach host memory, none waits in the GPU's L2)
    PinBuf h_ev{nullptr, 0, hipHostMallocCoherent};
    uint32_t small_gen = 0;   // the last lc_small call's status tag
    bool small_dirty = true;  // ws_small not known to hold a zero ticket counter (new buffer, failed call)
    // the chunked log verify's result words: coherent host memory the last kernel
    // writes directly (no D2H copy of them, the host polls the stream)
    uint64_t *h_res = nullptr;
    // the last jl_log_verify_dev_async may still be in flight on async_st (NULL is
    // a valid stream, HIP's null stream: `async_pending` says whether there is one);
    // async_done is recorded on that stream after its launches
    bool async_pending = false;
    // the chunked log verification's four work counters (ws_lc's first 256 B) are
    // zeroed by the last kernel of each verification for the next one; a call that
    // stopped between its launches (or a new ws_lc) leaves them to a memset
    bool lc_dirty = true;
    uint32_t lc_gen = 0;  // the last chunked verification's tag (lc_dense's placement tiles)
    uint32_t *h_hint = nullptr;  // pinned: the last chunked verification's count of lc_dwalk's blocks
    hipStream_t async_st = nullptr;
    hipEvent_t async_done = nullptr;
    Slot slot[2];
    void release() {
        if (stream) (void)hipStreamSynchronize(stream);
        if (async_pending) (void)hipEventSynchronize(async_done);
        async_pending = false;
        if (async_done) (void)hipEventDestroy(async_done);
        async_done = nullptr;
        if (h_res) (void)hipHostFree(h_res);
        h_res = nullptr;
        if (h_hint) (void)hipHostFree(h_hint);
        h_hint = nullptr;
        for (DevBuf *b : {&ws_lc, &ws_slot, &ws_desc, &ws_big, &ws_part, &ws_tmp, &ws_stash, &ws_ls, &ws_lsev, &ws_small})
            b->release();
        small_dirty = true;
        h_ev.release();
        for (Slot &sl : slot) {
            if (sl.st) (void)hipStreamSynchronize(sl.st);
            for (DevBuf *b : {&sl.d_in, &sl.d_desc, &sl.d_out}) b->release();
            sl.h_data.release();
            sl.h_desc.release();
            sl.h_out.release();
            if (sl.copied) (void)hipEventDestroy(sl.copied);
            if (sl.used) (void)hipEventDestroy(sl.used);
            if (sl.st) (void)hipStreamDestroy(sl.st);
            sl = Slot();
        }
        if (stream) (void)hipStreamDestroy(stream);
        stream = nullptr;
    }
};

struct Context {
    std::mutex mu;  // guards init / shutdown and the workspace registry
    bool ready = false;
    int device = -1;
    int gen = 0;  // bumped by every jl_init: threads re-bind their HIP device
    int cus = 0;
    void *d_img = nullptr;   // 160 KiB LDS image
    void *d_img_v4[5] = {nullptr, nullptr, nullptr, nullptr, nullptr};  // v4 images for 4 / 8 / 16 lanes per block; [3] gv4; [4] gv4 log chunks
    void *d_img_log = nullptr;  // fused log-verify image (log_stream.hip)
    uint32_t *d_aux = nullptr;
    uint8_t *d_zero = nullptr;  // 4 KiB of zeros (read by predicated-off loads)
    uint32_t *d_scratch = nullptr;  // 4 KiB sink for stores of out-of-range pair members
    std::vector<Workspace *> live;  // every thread's workspace (jl_shutdown releases them)
};

Context &ctx() {
    static Context c;
    return c;
}

// Owner of the calling thread's workspace: releases it when the thread exits.
struct WsOwner {
    Workspace *w = nullptr;
    ~WsOwner() {
        if (!w) return;
        Context &c = ctx();
        std::lock_guard<std::mutex> lk(c.mu);
        c.live.erase(std::remove(c.live.begin(), c.live.end(), w), c.live.end());
        if (c.ready && hipSetDevice(c.device) == hipSuccess) w->release();
        delete w;
    }
};
thread_local WsOwner t_ws;
thread_local int t_gen = -1;  // the context generation this thread's HIP device is bound for

// The calling thread's workspace with its streams and events created.
int get_ws(Workspace **out) {
    if (!t_ws.w) {
        Workspace *w = new Workspace;
        Context &c = ctx();
        std::lock_guard<std::mutex> lk(c.mu);
        c.live.push_back(w);
        t_ws.w = w;
    }
    Workspace &w = *t_ws.w;
    if (!w.stream) JL_HIP(hipStreamCreateWithFlags(&w.stream, hipStreamNonBlocking));
    if (!w.async_done) JL_HIP(hipEventCreateWithFlags(&w.async_done, hipEventDisableTiming));
    for (Slot &sl : w.slot) {
        if (!sl.st) JL_HIP(hipStreamCreateWithFlags(&sl.st, hipStreamNonBlocking));
        if (!sl.copied) JL_HIP(hipEventCreateWithFlags(&sl.copied, hipEventDisableTiming));
        if (!sl.used) JL_HIP(hipEventCreateWithFlags(&sl.used, hipEventDisableTiming));
    }
    *out = &w;
    return JL_OK;
}

// Host-memory calls run either on the calling thread's SSE4.2 path
// (host_paths.cpp) or on the device; below a few MiB the device round trip
// (staging copy, DMA, launches, synchronisation) can cost more than the CRC
// itself.  Where the two cross depends on the box: the round-end driver's boxes
// staged pageable input at a third of our sessions' rate (BENCH_r05: a 16 MiB
// table 1 140 vs 505 us on the device, the same 1 180 vs 1 150 us on the host),
// so no fixed size is right everywhere.  The default (JL_HOST_THRESHOLD_AUTO)
// measures instead: per entry point and size class the first calls run on each
// path (three each, their median), then every call takes the faster one and the
// other is re-measured every 16 / 64 / 256 calls (Dispatch below).  A threshold
// >= 0 fixes the split.
constexpr int64_t kHostThresholdDefault = JL_HOST_THRESHOLD_AUTO, kLogHostThresholdDefault = JL_HOST_THRESHOLD_AUTO;
// Logs (and host-pipeline chunks of logs) up to this size take the one-launch path
// (lc_small_kernel: one workgroup per 32 KiB block); larger ones the chunked path.
constexpr int64_t kLogSmallMaxDefault = 16 << 20;

// Engine options (jl_set_option, include/jlcrc.h): which general-path kernel a
// batch takes and its tuning.  Defaults are the measured best; tests force the
// alternatives.
struct Options {
    int general_path = JL_PATH_AUTO;  // JL_OPT_GENERAL_PATH
    int stream_depth = 16;            // JL_OPT_STREAM_DEPTH: 16 / 32 / 48 ring entries
    int partition = 1;                // JL_OPT_STREAM_PARTITION: byte-balanced wave ranges
    int64_t split_cap = -1;           // JL_OPT_SPLIT_CAP: chunks of split blocks (-1: min(2^20, 2048 n))
    int host_register = 1;            // JL_OPT_HOST_REGISTER: pin pageable inputs >= 64 MiB for the call
    int stage_threads = 8;            // JL_OPT_STAGE_THREADS: host threads copying into pinned staging
    int64_t stage_piece = 16 << 20;   // JL_OPT_STAGE_PIECE: staged copy pieces of big chunks (0: whole chunk)
    int64_t host_threshold = kHostThresholdDefault;  // JL_OPT_HOST_THRESHOLD: smaller host-memory calls run on the host
    int64_t log_host_threshold = kLogHostThresholdDefault;  // JL_OPT_LOG_HOST_THRESHOLD: the same for jl_log_verify
    int failpoint = 0;                // JL_OPT_FAILPOINT (tests): bit 0 perturbs lc_dwalk's offsets
    int64_t log_small_max = kLogSmallMaxDefault;  // JL_OPT_LOG_SMALL_MAX: logs up to this size verify in one launch
};
Options &opt() {
    static Options o;
    return o;
}

// ------------------------------------------------------------ call dispatch
// Auto dispatch state: per kind of call (the entry point) and size class (2^17 ..
// 2^25 bytes), the two paths' cost per byte.  A class first runs kDispProbe calls
// on the device, then kDispProbe on the host (the median of each: a cold first call, page
// faults of a fresh buffer, do not decide it), then every call takes the cheaper
// path and feeds its average; the other path is measured again every 16 calls
// when the two are within 25 %, every 64 within 2x, else every 256 (a box whose
// costs drift, e.g. under host load, is followed; a clear loser costs < 1 %).
constexpr int kKindFixed = 0, kKindBatch = 1, kKindTable = 2, kKindTables = 3, kKindLog = 4, kDispKinds = 5;
constexpr int kDispBuckets = 9, kDispProbe = 3;
constexpr uint64_t kDispHostBelow = 128u << 10;   // auto: always the host below this
constexpr uint64_t kDispDeviceFrom = 64ull << 20;  // auto: always the device from this (host 3-4x slower)
struct Dispatch {
    struct Cell {
        double ns_per_byte[2] = {0.0, 0.0};  // [0] host path, [1] device path
        double probe[2][kDispProbe] = {};
        uint32_t n[2] = {0u, 0u};  // calls measured
        uint32_t since = 0;        // calls since the other path was last measured
    };
    std::mutex mu;
    Cell cell[kDispKinds][kDispBuckets];
};
Dispatch &dispatch() {
    static Dispatch d;
    return d;
}
// the calling thread's last host-memory call (JL_INFO_*)
thread_local int t_last_path = -1;
thread_local int64_t t_last_ns = 0, t_stage_ns = 0;

// The route of one host-memory call: its path (threshold >= 0: fixed; auto: the
// measured costs), its time recorded for the auto dispatch once it succeeded.
jlhost::CopyPool &copy_pool();
struct Route {
    int kind, bucket = -1;
    uint64_t bytes;
    bool host = false, ok = false;
    std::chrono::steady_clock::time_point t0;
    Route(int k, uint64_t b, int64_t threshold) : kind(k), bytes(b), t0(std::chrono::steady_clock::now()) {
        t_stage_ns = 0;
        if (threshold >= 0) {
            host = (int64_t)b < threshold;
        } else if (b < kDispHostBelow || b >= kDispDeviceFrom) {
            host = b < kDispHostBelow;
        } else {
            bucket = std::min(kDispBuckets - 1, 63 - __builtin_clzll(b) - 17);
            Dispatch &D = dispatch();
            std::lock_guard<std::mutex> lk(D.mu);
            Dispatch::Cell &c = D.cell[kind][bucket];
            if (c.n[0] < kDispProbe || c.n[1] < kDispProbe) {
                // the device's probes first, then the host's: alternated, a device call
                // after a host call (whose start ends the copy pool's spinning) paid
                // the workers' wake-up, and the probes chose the host for a 4 MiB table
                // that the device verifies in 204 against 287 us (r6zb)
                host = c.n[1] >= kDispProbe;
            } else {
                const bool h = c.ns_per_byte[0] <= c.ns_per_byte[1];
                const double r = h ? c.ns_per_byte[1] / c.ns_per_byte[0] : c.ns_per_byte[0] / c.ns_per_byte[1];
                const uint32_t every = r < 1.25 ? 16u : (r < 2.0 ? 64u : 256u);
                host = ++c.since >= every ? !h : h;
                if (host != h) c.since = 0;
            }
        }
        t_last_path = host ? 0 : 1;
        if (host) copy_pool().quiesce();
        else copy_pool().prewake();  // (the call's staging copies, if its input is pageable)
    }
    ~Route() {
        const int64_t ns =
            std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0).count();
        t_last_ns = ns;
        if (bucket < 0 || !ok || bytes == 0) return;
        Dispatch &D = dispatch();
        std::lock_guard<std::mutex> lk(D.mu);
        Dispatch::Cell &c = D.cell[kind][bucket];
        const int p = host ? 0 : 1;
        const double v = (double)ns / (double)bytes;
        if (c.n[p] < kDispProbe) {
            c.probe[p][c.n[p]] = v;
            if (c.n[p] + 1 == kDispProbe) {  // the median of the probe calls
                double *q = c.probe[p];
                c.ns_per_byte[p] = std::max(std::min(q[0], q[1]), std::min(std::max(q[0], q[1]), q[2]));
            }
        } else {
            c.ns_per_byte[p] = 0.75 * c.ns_per_byte[p] + 0.25 * v;
        }
        c.n[p]++;
    }
};

// Initialises the engine on device 0 if no jl_init came first, and binds the
// calling thread to the engine's device (HIP's current device is per thread).
int ensure_ready() {
    Context &c = ctx();
    if (!c.ready)
        if (int r = jl_init(0)) return r;
    if (t_gen != c.gen) {
        JL_HIP(hipSetDevice(c.device));
        t_gen = c.gen;
    }
    return JL_OK;
}

// ------------------------------------------------------- host input staging
constexpr uint64_t kRegisterMin = 64ull << 20;  // hipHostRegister only pays for large inputs

// The engine's own call-scoped hipHostRegister pins, shared by reference count:
// two threads verifying the same mmap'd file at once must not have the first
// one to finish unpin the range under the other's DMA (hipPointerGetAttributes
// reports the range as pinned to the second caller, which then copies straight
// from it).
struct PinRegistry {
    std::mutex mu;
    struct Pin {
        const void *p;
        uint64_t bytes;
        int refs;
    };
    std::vector<Pin> pins;
};
PinRegistry &pin_registry() {
    static PinRegistry r;
    return r;
}

// A host input range for one call: DMA'd directly when it is pinned
// (hipHostMalloc'ed or already registered) or could be registered for the call
// (JL_OPT_HOST_REGISTER), else copied through the slots' pinned staging.
struct HostSrc {
    const uint8_t *p = nullptr;
    uint64_t bytes = 0;
    bool direct = false, shared = false;  // shared: holds a reference on an engine pin
    HostSrc(const void *ptr, uint64_t n) : p((const uint8_t *)ptr), bytes(n) {
        PinRegistry &R = pin_registry();
        std::lock_guard<std::mutex> lk(R.mu);
        for (PinRegistry::Pin &q : R.pins) {
            const uint8_t *qa = (const uint8_t *)q.p, *qb = qa + q.bytes;
            if (qa <= p && p + bytes <= qb) {  // inside a range another call of the engine pinned
                q.refs++;
                direct = shared = true;
                return;
            }
            // overlapping an engine pin without lying inside it: the pin may be
            // dropped under this call's DMA (and hipPointerGetAttributes below
            // would report the whole range as pinned from its start alone), and a
            // second registration of the overlap fails: stage it
            if (p < qb && qa < p + bytes) return;
        }
        hipPointerAttribute_t attr;
        direct = hipPointerGetAttributes(&attr, ptr) == hipSuccess && attr.type == hipMemoryTypeHost;
        (void)hipGetLastError();  // pageable memory reports an error here; clear it
        if (!direct && opt().host_register && bytes >= kRegisterMin) {
            // read-only first: an mmap'd file opened O_RDONLY can only be pinned that way
            for (unsigned flags : {(unsigned)hipHostRegisterReadOnly, (unsigned)hipHostRegisterDefault}) {
                if (hipHostRegister((void *)ptr, bytes, flags) == hipSuccess) {
                    direct = shared = true;
                    R.pins.push_back({ptr, bytes, 1});
                    break;
                }
                (void)hipGetLastError();  // not registrable (e.g. some file mappings): staging
            }
        }
    }
    ~HostSrc() {
        if (!shared) return;
        PinRegistry &R = pin_registry();
        std::lock_guard<std::mutex> lk(R.mu);
        for (size_t i = 0; i < R.pins.size(); i++) {
            PinRegistry::Pin &q = R.pins[i];
            if ((const uint8_t *)q.p <= p && p + bytes <= (const uint8_t *)q.p + q.bytes) {
                if (--q.refs == 0) {
                    (void)hipHostUnregister((void *)q.p);
                    R.pins.erase(R.pins.begin() + (ptrdiff_t)i);
                }
                return;
            }
        }
    }
};

jlhost::CopyPool &copy_pool() {
    static jlhost::CopyPool *p = new jlhost::CopyPool;  // never destroyed: workers may outlive static destruction order
    return *p;
}
void par_memcpy(void *dst, const void *src, size_t n) {
    const auto t0 = std::chrono::steady_clock::now();
    copy_pool().copy(dst, src, n, std::max(1, opt().stage_threads));
    t_stage_ns += std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0).count();
}

// Enqueues the copy of src.p[off, off + bytes) into sl.d_in on the slot's copy
// stream, after the slot's previous use; staged through pinned memory when the
// source is pageable.
// A pageable source is staged in pieces of kStagePiece, each DMA'd as soon as it
// is in pinned memory, so the copy engine works on piece i while the host copies
// piece i + 1 (one call's latency is then about the host copy, not copy + DMA).
constexpr uint64_t kStagePiece = 4ull << 20;
int slot_put_data(Slot &sl, const HostSrc &src, uint64_t off, uint64_t bytes) {
    JL_HIP(hipStreamWaitEvent(sl.st, sl.used, 0));
    const uint8_t *p = src.p + off;
    if (src.direct) {
        if (bytes) JL_HIP(hipMemcpyAsync(sl.d_in.p, p, bytes, hipMemcpyHostToDevice, sl.st));
        return JL_OK;
    }
    JL_HIP(hipEventSynchronize(sl.copied));  // the staging buffer's previous copy is done
    JL_HIP(sl.h_data.ensure(bytes));
    // small chunks (one call's latency) in 4 MiB pieces; big ones in stage_piece
    // pieces: every piece is one job for the copy threads, and 16 jobs per 64 MiB
    // chunk cost the staged C2 stream ~1/3 of its rate (r4q 20.5 vs r3 ~30 GiB/s)
    const uint64_t sp = (uint64_t)opt().stage_piece;
    const uint64_t piece = bytes <= 4 * kStagePiece ? kStagePiece : (sp ? sp : bytes);
    for (uint64_t a = 0; a < bytes; a += piece) {
        const uint64_t m = std::min(piece, bytes - a);
        par_memcpy((uint8_t *)sl.h_data.p + a, p + a, m);
        JL_HIP(hipMemcpyAsync((uint8_t *)sl.d_in.p + a, (const uint8_t *)sl.h_data.p + a, m, hipMemcpyHostToDevice, sl.st));
    }
    return JL_OK;
}

// Enqueues the copy of a chunk's descriptor arrays (host arrays, null ones
// skipped) packed into sl.d_desc through the slot's pinned descriptor staging
// (256-B aligned parts, one H2D copy); sl.part[k] = the device address of part
// k (null for a null source).
struct Part {
    const void *src;
    size_t bytes;
};
constexpr size_t align256(size_t b) { return (b + 255) & ~(size_t)255; }
int slot_put_desc(Slot &sl, std::initializer_list<Part> parts) {
    void **dev = sl.part;
    size_t total = 0;
    for (const Part &p : parts) total += p.src ? align256(p.bytes) : 0;
    JL_HIP(hipStreamWaitEvent(sl.st, sl.used, 0));
    JL_HIP(hipEventSynchronize(sl.copied));  // the staging buffer's previous copy is done
    JL_HIP(sl.h_desc.ensure(total));
    JL_HIP(sl.d_desc.ensure(total));
    size_t at = 0;
    int k = 0;
    for (const Part &p : parts) {
        dev[k++] = p.src ? (char *)sl.d_desc.p + at : nullptr;
        if (!p.src) continue;
        memcpy((char *)sl.h_desc.p + at, p.src, p.bytes);
        at += align256(p.bytes);
    }
    if (total) JL_HIP(hipMemcpyAsync(sl.d_desc.p, sl.h_desc.p, total, hipMemcpyHostToDevice, sl.st));
    return JL_OK;
}

// Waits for the stream's work: polls it (hipStreamQuery) for up to kPollSpinUs,
// then polls yielding the core to other threads up to kPollYieldUs, then blocks.
// A log verification of a few MiB returns without the ~50 us wake-up of a
// blocking synchronise (r2: 0.93 -> 0.88 ms on C5), and concurrent callers do
// not each keep a host core spinning for long.
constexpr double kPollSpinUs = 200.0, kPollYieldUs = 5000.0;
hipError_t poll_stream(hipStream_t st) {
    const auto t0 = std::chrono::steady_clock::now();
    for (;;) {
        const hipError_t e = hipStreamQuery(st);
        if (e != hipErrorNotReady) return e;
        const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
        if (us > kPollYieldUs) return hipStreamSynchronize(st);
        if (us > kPollSpinUs) std::this_thread::yield();
    }
}

// Waits for both pipelines' work to finish and returns the first error of the
// call, if any.
int drain(Workspace &w, int rc) {
    hipError_t e = poll_stream(w.stream);  // a short call returns without a blocking wake-up
    for (Slot &sl : w.slot) {
        hipError_t f = poll_stream(sl.st);
        if (e == hipSuccess) e = f;
    }
    if (rc) return rc;
    if (e != hipSuccess) return fail(JL_ERR_HIP, std::string("pipeline: ") + hipGetErrorString(e));
    return JL_OK;
}

// Double-buffered host -> device pipeline over n_chunks chunks.  put(i, slot)
// enqueues chunk i's copies on the slot's copy stream; run(i, slot) enqueues
// its kernels and copy-out on the compute stream.  Chunk i+1's copy is enqueued
// before chunk i's compute, so the copy engine always has the next chunk queued
// and a copy-out that blocks the host (pageable destination) never starves it.
template <class Put, class Run>
int pipeline(Workspace &w, uint64_t n_chunks, Put put, Run run) {
    auto issue = [&](uint64_t i) -> int {
        Slot &sl = w.slot[i & 1];
        if (int r = put(i, sl)) return r;
        JL_HIP(hipEventRecord(sl.copied, sl.st));
        return JL_OK;
    };
    int rc = n_chunks ? issue(0) : JL_OK;
    for (uint64_t i = 0; i < n_chunks && !rc; i++) {
        if (i + 1 < n_chunks && (rc = issue(i + 1))) break;
        Slot &sl = w.slot[i & 1];
        hipError_t e = hipStreamWaitEvent(w.stream, sl.copied, 0);
        if (e != hipSuccess) {
            rc = fail(JL_ERR_HIP, std::string("pipeline: ") + hipGetErrorString(e));
            break;
        }
        if ((rc = run(i, sl))) break;
        e = hipEventRecord(sl.used, w.stream);
        if (e != hipSuccess) rc = fail(JL_ERR_HIP, std::string("pipeline: ") + hipGetErrorString(e));
    }
    return drain(w, rc);
}

constexpr uint64_t kSlack = 256;                // device bytes past a chunk (rounded-up tail reads)
constexpr uint64_t kChunkBlocks = 1ull << 20;   // descriptors per chunk

// Chunks of an offset/length batch: blocks [a, b) whose bytes (with `extra`
// trailing bytes each) lie in the host window [lo, hi).
struct Chunk {
    uint64_t a, b, lo, hi;
};
// When the offsets ascend (a table's handles, an arena of appended blocks) the
// blocks are cut into chunks whose windows span at most JL_STREAM_CHUNK_BYTES
// (a larger block is a chunk of its own); otherwise one chunk spans them all.
// Window starts are page-aligned (DMA).  Blocks were range-checked by the caller.
std::vector<Chunk> plan_chunks(const uint64_t *off, const uint32_t *len, uint32_t extra, uint64_t n) {
    std::vector<Chunk> ch;
    bool asc = true;
    for (uint64_t i = 1; i < n && asc; i++) asc = off[i] >= off[i - 1];
    auto page = [](uint64_t x) { return x & ~4095ull; };
    if (!asc) {
        uint64_t lo = ~0ull, hi = 0;
        for (uint64_t i = 0; i < n; i++) {
            lo = std::min(lo, off[i]);
            hi = std::max(hi, off[i] + len[i] + extra);
        }
        ch.push_back({0, n, page(lo), hi});
        return ch;
    }
    for (uint64_t a = 0; a < n;) {
        const uint64_t lo = page(off[a]);
        uint64_t hi = off[a] + len[a] + extra, b = a + 1;
        while (b < n && b - a < kChunkBlocks) {
            const uint64_t h = std::max(hi, off[b] + len[b] + extra);
            if (h - lo > JL_STREAM_CHUNK_BYTES) break;
            hi = h;
            b++;
        }
        ch.push_back({a, b, lo, hi});
        a = b;
    }
    return ch;
}

// Sizes both slots for the largest chunk: window bytes, results of out_bytes and
// descriptors of desc_bytes a block.
int ensure_chunk_bufs(Workspace &w, const std::vector<Chunk> &ch, size_t out_bytes, size_t desc_bytes) {
    uint64_t win = 0, m = 0;
    for (const Chunk &k : ch) {
        win = std::max(win, k.hi - k.lo);
        m = std::max(m, k.b - k.a);
    }
    for (Slot &sl : w.slot) {
        JL_HIP(sl.d_in.ensure(win + kSlack));
        JL_HIP(sl.d_out.ensure(m * out_bytes));
        JL_HIP(sl.d_desc.ensure(m * desc_bytes + 4 * 256));
    }
    return JL_OK;
}

// NULL is HIP's null (legacy default) stream, as everywhere in HIP, so device
// entry points order with the caller's default-stream work.
hipStream_t pick(void *stream) { return (hipStream_t)stream; }

// The device entry points refuse a stream that is being captured into a HIP
// graph: their per-thread scratch and the bookkeeping around it (the pending
// asynchronous call's event, scratch sizing, the host read-backs of the
// synchronous forms, stream-ordered scratch allocations) is done on the host
// at call time, so a replayed graph would run against state the host no longer
// tracks.  r5 replayed a captured jl_log_verify_dev_async and it faulted.
int no_capture(void *stream, const char *who) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    const hipError_t e = hipStreamIsCapturing(pick(stream), &cs);
    if (e != hipSuccess) {
        (void)hipGetLastError();
        // the null (legacy) stream while ANOTHER stream captures in global mode: the
        // given stream itself is not capturing, but work on it would join that capture
        if (e == hipErrorStreamCaptureImplicit)
            return fail(JL_ERR_INVALID, std::string(who) +
                                            ": the null stream cannot be used while another stream is being captured "
                                            "into a HIP graph (global capture mode); pass a stream of your own");
        return fail(JL_ERR_INVALID, std::string(who) + ": the stream's capture status cannot be queried (" +
                                        hipGetErrorString(e) + ")");
    }
    if (cs != hipStreamCaptureStatusNone)
        return fail(JL_ERR_INVALID, std::string(who) + ": stream capture (HIP graphs) is not supported");
    return JL_OK;
}

int grid_for(uint64_t blocks) {
    // one 1024-thread workgroup (16 waves) per CU; fewer when there is little work
    uint64_t wg = (blocks + 15) / 16;
    int cus = ctx().cus;
    return (int)std::max<uint64_t>(1, std::min<uint64_t>(wg, (uint64_t)cus));
}

jlk::KParams base_params(const void *d_base, uint64_t n, int mode) {
    jlk::KParams P;
    memset(&P, 0, sizeof(P));
    P.base = (const uint8_t *)d_base;
    P.aux = ctx().d_aux;
    P.zero = ctx().d_zero;
    P.n = n;
    P.mode = mode;
    P.base_bytes = ~0ull;
    return P;
}

struct U32ToU64 {
    __host__ __device__ uint64_t operator()(uint32_t v) const { return v; }
};

// weight of a block for the byte-balanced partition: its bytes plus the
// per-block fixed cost of the stream kernel (seed, re-alignment, result),
// roughly that of reading 256 B
struct BlockWeight {
    uint32_t add;
    __host__ __device__ uint64_t operator()(uint32_t len) const { return (uint64_t)len + add + 256u; }
};

// Byte-balanced wave ranges for the stream kernel (stream-ordered scratch:
// hipMallocAsync / hipFreeAsync on the caller's stream, so concurrent callers
// on different streams never share it).  Returns nullptr (count split) when the
// batch is too small to be worth a scan or the blocks have a fixed stride.
static uint64_t *make_partition(const jlk::KParams &P, uint64_t waves, hipStream_t st, int *rc) {
    *rc = JL_OK;
    if (!P.off || P.n < 16 * waves || !opt().partition) return nullptr;
    hipcub::TransformInputIterator<uint64_t, BlockWeight, const uint32_t *> it(P.len, BlockWeight{P.len_add});
    size_t tmp = 0;
    if (hipcub::DeviceScan::InclusiveSum(nullptr, tmp, it, (uint64_t *)nullptr, (int)P.n, st) != hipSuccess) {
        *rc = fail(JL_ERR_HIP, "partition scan sizing failed");
        return nullptr;
    }
    void *buf = nullptr;
    // every sub-buffer 256-B aligned: hipcub carves its temporaries out of
    // scan_tmp assuming that alignment (an unaligned one overran, r1)
    const size_t incl_bytes = (P.n * 8 + 255) & ~(size_t)255, part_bytes = ((waves + 1) * 8 + 255) & ~(size_t)255;
    if (hipMallocAsync(&buf, incl_bytes + part_bytes + tmp, st) != hipSuccess) {
        *rc = fail(JL_ERR_NOMEM, "partition scratch allocation failed");
        return nullptr;
    }
    uint64_t *incl = (uint64_t *)buf, *part = (uint64_t *)((char *)buf + incl_bytes);
    void *scan_tmp = (char *)buf + incl_bytes + part_bytes;
    if (hipcub::DeviceScan::InclusiveSum(scan_tmp, tmp, it, incl, (int)P.n, st) != hipSuccess ||
        jlk::launch_partition(incl, P.n, waves, part, st) != hipSuccess) {
        (void)hipFreeAsync(buf, st);
        *rc = fail(JL_ERR_HIP, "partition failed");
        return nullptr;
    }
    return part;  // == buf + incl_bytes; freed through free_partition
}

static void free_partition(const jlk::KParams &P, uint64_t *part, hipStream_t st) {
    if (part) (void)hipFreeAsync((char *)part - ((P.n * 8 + 255) & ~(size_t)255), st);
}

// General v4 path (general_v4.hip): 128-B aligned fixed strides run as implicit
// rounds; any other batch is sorted by step count K first (keys -> radix sort ->
// run starts -> round ids -> GDesc table), all stream-ordered on `st` with
// stream-ordered scratch.
static bool gv4_eligible(const jlk::KParams &P) {
    if (P.mode != jlk::MODE_CRC && P.mode != jlk::MODE_TABLE_VERIFY) return false;
    if (P.n >= (1ull << 31)) return false;  // hipcub sizes are int
    if (!P.off && (P.fixed_bytes == 0 || P.fixed_bytes > 0xffffffffull)) return false;
    return true;
}

static hipError_t gv4_launch(const jlk::GV4Args &A, hipStream_t st) {
    const void *img = ctx().d_img_v4[3];  // the general v4 image (crc_math.hpp)
    const int grid = ctx().cus;            // one 512-thread workgroup per CU (the LDS image)
    switch (A.P.mode) {
    case jlk::MODE_CRC: return jlk::launch_gv4_m<jlk::MODE_CRC>(img, A, ctx().d_zero, grid, st);
    case jlk::MODE_TABLE_VERIFY: return jlk::launch_gv4_m<jlk::MODE_TABLE_VERIFY>(img, A, ctx().d_zero, grid, st);
    case jlk::MODE_LOG_CHUNK: return jlk::launch_gv4_m<jlk::MODE_LOG_CHUNK>(ctx().d_img_v4[4], A, ctx().d_zero, grid, st);
    default: return hipErrorInvalidValue;
    }
}

static int run_gv4(const jlk::KParams &P, hipStream_t st) {
    jlk::GV4Args A;
    memset(&A, 0, sizeof(A));
    A.P = P;
    A.seed0 = jlmath::slice4_inv(0xffffffffu);
    // blocks above kGSplitMin (MODE_CRC) are split into chunks folded afterwards
    const bool can_split = P.mode == jlk::MODE_CRC;
    if (!P.off && ((uintptr_t)P.base & 127) == 0 && (P.fixed_bytes & 127) == 0 &&
        !(can_split && P.fixed_bytes > jlk::kGSplitMin)) {
        // every block starts on the 128-B grid: implicit rounds, no pads, no sort
        A.fixed_K = (uint32_t)(P.fixed_bytes / 128);
        JL_HIP(gv4_launch(A, st));
        return JL_OK;
    }
    const uint64_t n = P.n;
    // rounds: ceil(c/8) per bin of c blocks <= n/8 + one partial round per bin (2^17 bins),
    // plus one round per solo block (>= 16 MiB each: at most 18432 in 288 GiB)
    const uint64_t nb = (uint64_t)jlk::kGSoloKey + 1;
    // split blocks: up to part_cap chunks (JL_OPT_SPLIT_CAP), blocks beyond it stay whole
    const uint64_t part_cap =
        can_split ? (opt().split_cap >= 0 ? (uint64_t)opt().split_cap
                                          : std::min<uint64_t>(1ull << 20, 2048 * n))  // <= 2048 chunks a block
                  : 0;
    const uint64_t vn = n + part_cap;  // blocks and chunks
    const uint64_t max_rounds = vn / 8 + std::min<uint64_t>(vn, nb) + std::min<uint64_t>(n, 18432) + 1;
    auto al = [](size_t b) { return (b + 255) & ~(size_t)255; };
    const size_t ab = al((nb + 1) * 4), ad = al(max_rounds * sizeof(jlk::GDesc) * 8);  // hist[nb] = max bin
    const size_t a_bb = part_cap ? al(n * 4) : 0, a_big = al((part_cap / 2 + 1) * sizeof(jlk::GBig)),
                 a_parts = al(part_cap * 4);
    const size_t total = 3 * ab + ad + 256 + 256 + a_bb + a_big + a_parts;
    char *buf = nullptr;
    if (hipMallocAsync((void **)&buf, total, st) != hipSuccess) return fail(JL_ERR_NOMEM, "gv4 scratch allocation failed");
    uint32_t *hist = (uint32_t *)buf, *cursor = (uint32_t *)(buf + ab), *rstart = (uint32_t *)(buf + 2 * ab);
    jlk::GDesc *desc = (jlk::GDesc *)(buf + 3 * ab);
    uint32_t *n_rounds = (uint32_t *)(buf + 3 * ab + ad);
    char *sp = buf + 3 * ab + ad + 256;
    jlk::GSplit SP;
    // the split counters sit in the padding after hist[nb] (cleared with hist and cursor)
    static_assert(((((uint64_t)jlk::kGSoloKey + 2) * 4 + 7) & ~7ull) + 16 <= (((uint64_t)jlk::kGSoloKey + 2) * 4 + 255 & ~255ull),
                  "split counters must fit in hist's padding");
    SP.ctl = (unsigned long long *)(buf + ((((uint64_t)jlk::kGSoloKey + 2) * 4 + 7) & ~7ull));
    SP.bigbase = (uint32_t *)(sp + 256);
    SP.big = (jlk::GBig *)(sp + 256 + a_bb);
    SP.part_cap = (uint32_t)std::min<uint64_t>(part_cap, 0x7fffffffu);
    uint32_t *parts = (uint32_t *)(sp + 256 + a_bb + a_big);
    hipError_t e = hipMemsetAsync(buf, 0, 2 * ab, st);  // hist, cursor
    // (empty groups of partial rounds are marked by the scan kernel: no clearing)
    if (e == hipSuccess) e = jlk::launch_gv4_rounds(P, SP, hist, cursor, rstart, desc, n_rounds, st);
    A.parts = parts;
    A.desc = desc;
    A.n_rounds = n_rounds;
    A.deal = n_rounds + 1;  // zeroed by gv4_scan_kernel
    if (e == hipSuccess) e = gv4_launch(A, st);
    if (e == hipSuccess && SP.part_cap) e = jlk::launch_gv4_combine(P, SP, parts, st);
    (void)hipFreeAsync(buf, st);
    JL_HIP(e);
    return JL_OK;
}

int run_general(const jlk::KParams &P, hipStream_t st) {
    if (P.n == 0) return JL_OK;
    // general v4 (general_v4.hip) is the default for the crc / table-verify /
    // log-verify modes (r1 A/B: C3 2.38 vs 2.64 ms, C5 0.81 vs 0.93 ms, C2 through
    // offsets 0.95 vs 1.04 ms), except for small sorted verify batches, where its
    // ~12 pipeline launches cost more than the stream kernel's one; crc batches
    // always take gv4, which splits a few huge blocks across waves.
    // JL_OPT_GENERAL_PATH forces either.
    const Options &o = opt();
    const bool small = P.off && P.n < 4096 && P.mode != jlk::MODE_CRC;
    const bool want_gv4 = o.general_path == JL_PATH_GV4 || (o.general_path == JL_PATH_AUTO && !small);
    if (want_gv4 && gv4_eligible(P)) return run_gv4(P, st);
    const int grid = grid_for(P.n);
    int rc = JL_OK;
    uint64_t *part = make_partition(P, (uint64_t)grid * 16, st, &rc);
    if (rc) return rc;
    const hipError_t e = jlk::launch_stream(ctx().d_img, P, part, grid, o.stream_depth, st);
    free_partition(P, part, st);
    JL_HIP(e);
    return JL_OK;
}

}  // namespace

// host-side helpers in other translation units (table_walker.cpp) report through here
void jl_set_error(const std::string &msg) { g_err = msg; }

extern "C" {

const char *jl_last_error(void) { return g_err.c_str(); }

const char *jl_version(void) {
    return "jlcrc 0.2 gfx950 (v4: 8 lanes per block, 128-B steps, 4 chains per lane through LDS gap tables"
#if JL_STUDY
           "; study build"
#endif
           ")";
}

int jl_set_option(int option, int64_t value) {
    Options &o = opt();
    switch (option) {
    case JL_OPT_GENERAL_PATH:
        if (value < JL_PATH_AUTO || value > JL_PATH_GV4) break;
        o.general_path = (int)value;
        return JL_OK;
    case JL_OPT_STREAM_DEPTH:
        if (value != 16 && value != 32 && value != 48) break;
        o.stream_depth = (int)value;
        return JL_OK;
    case JL_OPT_STREAM_PARTITION:
        if (value != 0 && value != 1) break;
        o.partition = (int)value;
        return JL_OK;
    case JL_OPT_SPLIT_CAP:
        if (value < -1 || value > 0x7fffffff) break;
        o.split_cap = value;
        return JL_OK;
    case JL_OPT_HOST_REGISTER:
        if (value != 0 && value != 1) break;
        o.host_register = (int)value;
        return JL_OK;
    case JL_OPT_STAGE_THREADS:
        if (value < 1 || value > 64) break;
        o.stage_threads = (int)value;
        return JL_OK;
    case JL_OPT_HOST_THRESHOLD:
        if (value < JL_HOST_THRESHOLD_AUTO) break;
        o.host_threshold = value;
        return JL_OK;
    case JL_OPT_STAGE_PIECE:
        if (value < 0 || (value > 0 && value < (1 << 20))) break;
        o.stage_piece = value;
        return JL_OK;
    case JL_OPT_LOG_HOST_THRESHOLD:
        if (value < JL_HOST_THRESHOLD_AUTO) break;
        o.log_host_threshold = value;
        return JL_OK;
    case JL_OPT_FAILPOINT:
        if (value < 0 || value > 1) break;
        o.failpoint = (int)value;
        return JL_OK;
    case JL_OPT_LOG_SMALL_MAX:
        if (value < 0 || value > (int64_t)JL_STREAM_CHUNK_BYTES) break;
        o.log_small_max = value;
        return JL_OK;
    default:
        return fail(JL_ERR_INVALID, "jl_set_option: unknown option " + std::to_string(option));
    }
    return fail(JL_ERR_INVALID, "jl_set_option: value out of range for option " + std::to_string(option));
}

int64_t jl_get_option(int option) {
    const Options &o = opt();
    switch (option) {
    case JL_OPT_GENERAL_PATH: return o.general_path;
    case JL_OPT_STREAM_DEPTH: return o.stream_depth;
    case JL_OPT_STREAM_PARTITION: return o.partition;
    case JL_OPT_SPLIT_CAP: return o.split_cap;
    case JL_OPT_HOST_REGISTER: return o.host_register;
    case JL_OPT_STAGE_THREADS: return o.stage_threads;
    case JL_OPT_HOST_THRESHOLD: return o.host_threshold;
    case JL_OPT_LOG_HOST_THRESHOLD: return o.log_host_threshold;
    case JL_OPT_STAGE_PIECE: return o.stage_piece;
    case JL_OPT_FAILPOINT: return o.failpoint;
    case JL_OPT_LOG_SMALL_MAX: return o.log_small_max;
    case JL_INFO_STAGE_WORKERS: return copy_pool().workers();
    case JL_INFO_STAGE_SPAWN_FAILURES: return copy_pool().spawn_failures();
    case JL_INFO_LAST_PATH: return t_last_path;
    case JL_INFO_LAST_CALL_NS: return t_last_ns;
    case JL_INFO_LAST_STAGE_NS: return t_stage_ns;
    default: return fail(JL_ERR_INVALID, "jl_get_option: unknown option " + std::to_string(option));
    }
}

int jl_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

int jl_init(int device) {
    Context &c = ctx();
    std::lock_guard<std::mutex> lk(c.mu);
    if (c.ready) {
        if (c.device == device) return JL_OK;
        return fail(JL_ERR_INVALID, "jl_init: engine already bound to device " + std::to_string(c.device));
    }
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n == 0) return fail(JL_ERR_NO_DEVICE, "jl_init: no HIP device");
    if (device < 0 || device >= n) return fail(JL_ERR_INVALID, "jl_init: bad device ordinal");
    JL_HIP(hipSetDevice(device));
    hipDeviceProp_t prop;
    JL_HIP(hipGetDeviceProperties(&prop, device));
    if (std::string(prop.gcnArchName).find("gfx950") == std::string::npos)
        return fail(JL_ERR_NO_DEVICE, std::string("jl_init: engine is built for gfx950, device is ") + prop.gcnArchName);
    c.cus = prop.multiProcessorCount;
    {  // keep stream-ordered scratch (partition arrays) in the pool between calls
        hipMemPool_t pool;
        if (hipDeviceGetDefaultMemPool(&pool, device) == hipSuccess) {
            uint64_t keep = ~0ull;
            (void)hipMemPoolSetAttribute(pool, hipMemPoolAttrReleaseThreshold, &keep);
        }
        (void)hipGetLastError();
    }
    std::vector<uint32_t> img = jlmath::build_lds_image();
    std::vector<uint32_t> aux = jlmath::build_aux();
    JL_HIP(hipMalloc(&c.d_img, jlmath::kImageBytes));
    JL_HIP(hipMalloc((void **)&c.d_aux, aux.size() * 4));
    JL_HIP(hipMalloc((void **)&c.d_zero, 4096));
    JL_HIP(hipMalloc((void **)&c.d_scratch, 4096));
    JL_HIP(hipMemcpy(c.d_img, img.data(), jlmath::kImageBytes, hipMemcpyHostToDevice));
    for (int i = 0; i < 5; i++) {
        std::vector<uint32_t> v4 = i < 3    ? jlmath::build_lds_image_v4(4 << i)
                                   : i == 3 ? jlmath::build_lds_image_gv4_rotated()
                                            : jlmath::build_lds_image_logchunk();
        if (i >= 3) {  // the gv4 images: the round-dealing dwords must start zero (general_v4.hip)
            for (uint32_t d = jlk::kGvBatchDword; d < jlk::kGvDynEnd; d++)
                if ((d < jlk::kGvBatchDword + 32 || d >= jlk::kGvDynDword) && v4[d] != 0)
                    return fail(JL_ERR_HIP, "init: a gv4 LDS image overlaps the round-dealing dwords");
        }
        JL_HIP(hipMalloc(&c.d_img_v4[i], jlmath::kImageBytes));
        JL_HIP(hipMemcpy(c.d_img_v4[i], v4.data(), jlmath::kImageBytes, hipMemcpyHostToDevice));
    }
    {
        std::vector<uint32_t> li = jlmath::build_lds_image_logstream();
        JL_HIP(hipMalloc(&c.d_img_log, jlmath::kImageBytes));
        JL_HIP(hipMemcpy(c.d_img_log, li.data(), jlmath::kImageBytes, hipMemcpyHostToDevice));
    }
    JL_HIP(hipMemcpy(c.d_aux, aux.data(), aux.size() * 4, hipMemcpyHostToDevice));
    JL_HIP(hipMemset(c.d_zero, 0, 4096));
    c.device = device;
    c.gen++;
    t_gen = c.gen;
    c.ready = true;
    return JL_OK;
}

int jl_shutdown(void) {
    Context &c = ctx();
    std::lock_guard<std::mutex> lk(c.mu);
    if (!c.ready) return JL_OK;
    (void)hipSetDevice(c.device);
    (void)hipDeviceSynchronize();
    for (Workspace *w : c.live) w->release();  // their threads recreate them after the next jl_init
    (void)hipFree(c.d_img);
    (void)hipFree(c.d_img_log);
    c.d_img_log = nullptr;
    for (void *&p : c.d_img_v4) {
        (void)hipFree(p);
        p = nullptr;
    }
    (void)hipFree(c.d_aux);
    (void)hipFree(c.d_zero);
    (void)hipFree(c.d_scratch);
    c.d_scratch = nullptr;
    c.d_img = nullptr;
    c.d_aux = nullptr;
    c.d_zero = nullptr;
    c.ready = false;
    c.device = -1;
    return JL_OK;
}

// ----------------------------------------------------------- batch checksums
int jl_crc32c_fixed_dev(const void *d_data, uint64_t block_bytes, uint64_t n_blocks, uint32_t flags,
                        uint32_t *d_out, void *stream) {
    if (int r = ensure_ready()) return r;
    if (int r = no_capture(stream, "jl_crc32c_fixed_dev")) return r;
    if (n_blocks == 0) return JL_OK;
    if (!d_data || !d_out) return fail(JL_ERR_INVALID, "jl_crc32c_fixed_dev: null pointer");
    if (block_bytes > 0xffffffffull) return fail(JL_ERR_INVALID, "jl_crc32c_fixed_dev: block_bytes >= 4 GiB");
    hipStream_t st = pick(stream);
    if (block_bytes == 4096 && ((uintptr_t)d_data & 15) == 0) {  // the v4 kernel (fixed_v4.hip)
        JL_HIP(jlk::launch_fixed4k_v4(ctx().d_img_v4[1], (const uint8_t *)d_data, n_blocks, flags, d_out,
                                      grid_for(n_blocks), st));
        return JL_OK;
    }
    jlk::KParams P = base_params(d_data, n_blocks, jlk::MODE_CRC);
    P.fixed_bytes = block_bytes;
    P.flags = flags;
    P.out32 = d_out;
    return run_general(P, st);
}

int jl_crc32c_fixed(const uint8_t *host, uint64_t block_bytes, uint64_t n_blocks, uint32_t flags, uint32_t *out) {
    if (int r = ensure_ready()) return r;
    if (n_blocks == 0) return JL_OK;
    if (!host || !out || block_bytes == 0) return fail(JL_ERR_INVALID, "jl_crc32c_fixed: bad arguments");
    if (block_bytes > JL_STREAM_CHUNK_BYTES) return fail(JL_ERR_INVALID, "jl_crc32c_fixed: block larger than a chunk");
    Route rt(kKindFixed, n_blocks * block_bytes, opt().host_threshold);
    if (rt.host) {  // the host SSE4.2 path
        jlhost::fixed(host, block_bytes, n_blocks, flags, out);
        rt.ok = true;
        return JL_OK;
    }
    Workspace *w = nullptr;
    if (int r = get_ws(&w)) return r;
    const uint64_t per = JL_STREAM_CHUNK_BYTES / block_bytes;  // blocks per chunk
    const uint64_t first = std::min(per, n_blocks);
    for (Slot &sl : w->slot) {
        JL_HIP(sl.d_in.ensure(first * block_bytes + kSlack));
        JL_HIP(sl.d_out.ensure(first * 4));
    }
    HostSrc src(host, n_blocks * block_bytes);
    const uint64_t n_chunks = (n_blocks + per - 1) / per;
    const int rc = pipeline(
        *w, n_chunks,
        [&](uint64_t i, Slot &sl) {
            return slot_put_data(sl, src, i * per * block_bytes, std::min(per, n_blocks - i * per) * block_bytes);
        },
        [&](uint64_t i, Slot &sl) -> int {
            const uint64_t b0 = i * per, nb = std::min(per, n_blocks - b0);
            if (int r = jl_crc32c_fixed_dev(sl.d_in.p, block_bytes, nb, flags, (uint32_t *)sl.d_out.p, w->stream))
                return r;
            JL_HIP(hipMemcpyAsync(out + b0, sl.d_out.p, nb * 4, hipMemcpyDeviceToHost, w->stream));
            return JL_OK;
        });
    rt.ok = rc == JL_OK;
    return rc;
}

int jl_crc32c_batch_dev(const void *d_base, uint64_t base_bytes, const uint64_t *d_off, const uint32_t *d_len,
                        const uint32_t *d_init, const uint8_t *d_suffix, uint64_t n, uint32_t flags, uint32_t *d_out,
                        void *stream) {
    if (int r = ensure_ready()) return r;
    if (int r = no_capture(stream, "jl_crc32c_batch_dev")) return r;
    if (n == 0) return JL_OK;
    if (!d_base || !d_off || !d_len || !d_out) return fail(JL_ERR_INVALID, "jl_crc32c_batch_dev: null pointer");
    jlk::KParams P = base_params(d_base, n, jlk::MODE_CRC);
    P.base_bytes = base_bytes;
    P.off = d_off;
    P.len = d_len;
    P.init = d_init;
    P.suffix = d_suffix;
    P.flags = flags;
    P.out32 = d_out;
    return run_general(P, pick(stream));
}

int jl_crc32c_batch(const uint8_t *base, uint64_t base_bytes, const uint64_t *off, const uint32_t *len,
                    const uint32_t *init, const uint8_t *suffix, uint64_t n, uint32_t flags, uint32_t *out) {
    if (int r = ensure_ready()) return r;
    if (n == 0) return JL_OK;
    if (!base || !off || !len || !out) return fail(JL_ERR_INVALID, "jl_crc32c_batch: null pointer");
    uint64_t touched = 0;
    for (uint64_t i = 0; i < n; i++) {
        if (off[i] > base_bytes || len[i] > base_bytes - off[i])
            return fail(JL_ERR_INVALID, "jl_crc32c_batch: block out of range");
        touched += len[i];
    }
    Route rt(kKindBatch, touched, opt().host_threshold);
    if (rt.host) {  // the host SSE4.2 path
        jlhost::batch(base, off, len, init, suffix, n, flags, out);
        rt.ok = true;
        return JL_OK;
    }
    Workspace *w = nullptr;
    if (int r = get_ws(&w)) return r;
    const std::vector<Chunk> ch = plan_chunks(off, len, 0, n);
    if (int r = ensure_chunk_bufs(*w, ch, 4, 8 + 4 + 4 + 1)) return r;
    HostSrc src(base, base_bytes);
    const int rc = pipeline(
        *w, ch.size(),
        [&](uint64_t i, Slot &sl) -> int {
            const Chunk &k = ch[i];
            if (int r = slot_put_data(sl, src, k.lo, k.hi - k.lo)) return r;
            const uint64_t m = k.b - k.a;
            return slot_put_desc(sl, {{off + k.a, m * 8}, {len + k.a, m * 4}, {init ? init + k.a : nullptr, m * 4},
                                      {suffix ? suffix + k.a : nullptr, m}});
        },
        [&](uint64_t i, Slot &sl) -> int {
            const Chunk &k = ch[i];
            const uint64_t m = k.b - k.a;
            // the window [lo, hi) sits at d_in[0]: offsets stay arena offsets
            jlk::KParams P = base_params((const uint8_t *)sl.d_in.p - k.lo, m, jlk::MODE_CRC);
            P.base_bytes = k.hi;
            P.off = (const uint64_t *)sl.part[0];
            P.len = (const uint32_t *)sl.part[1];
            P.init = (const uint32_t *)sl.part[2];
            P.suffix = (const uint8_t *)sl.part[3];
            P.flags = flags;
            P.out32 = (uint32_t *)sl.d_out.p;
            if (int r = run_general(P, w->stream)) return r;
            JL_HIP(hipMemcpyAsync(out + k.a, sl.d_out.p, m * 4, hipMemcpyDeviceToHost, w->stream));
            return JL_OK;
        });
    rt.ok = rc == JL_OK;
    return rc;
}

// ------------------------------------------------------------- table shims
int jl_table_trailers_dev(const void *d_file, const uint64_t *d_off, const uint32_t *d_size, const uint8_t *d_type,
                          uint64_t n, uint8_t *d_trailer, void *stream) {
    if (int r = ensure_ready()) return r;
    if (int r = no_capture(stream, "jl_table_trailers_dev")) return r;
    if (n == 0) return JL_OK;
    if (!d_file || !d_off || !d_size || !d_trailer) return fail(JL_ERR_INVALID, "jl_table_trailers_dev: null pointer");
    jlk::KParams P = base_params(d_file, n, jlk::MODE_TRAILER);
    P.off = d_off;
    P.len = d_size;
    P.type = d_type;
    P.out8 = d_trailer;
    return run_general(P, pick(stream));
}

int jl_table_verify_dev(const void *d_file, uint64_t file_bytes, const uint64_t *d_off, const uint32_t *d_size,
                        uint64_t n, uint8_t *d_status, void *stream) {
    if (int r = ensure_ready()) return r;
    if (int r = no_capture(stream, "jl_table_verify_dev")) return r;
    if (n == 0) return JL_OK;
    if (!d_file || !d_off || !d_size || !d_status) return fail(JL_ERR_INVALID, "jl_table_verify_dev: null pointer");
    jlk::KParams P = base_params(d_file, n, jlk::MODE_TABLE_VERIFY);
    P.base_bytes = file_bytes;
    P.off = d_off;
    P.len = d_size;
    P.len_add = 1;  // block || type byte
    P.out8 = d_status;
    return run_general(P, pick(stream));
}

int jl_table_verify(const uint8_t *file, uint64_t file_bytes, const uint64_t *off, const uint32_t *size, uint64_t n,
                    uint8_t *status) {
    if (int r = ensure_ready()) return r;
    if (n == 0) return JL_OK;
    if (!file || !off || !size || !status) return fail(JL_ERR_INVALID, "jl_table_verify: null pointer");
    uint64_t touched = 0;
    for (uint64_t i = 0; i < n; i++) {
        if (off[i] > file_bytes || (uint64_t)size[i] + 5 > file_bytes - off[i])
            return fail(JL_ERR_INVALID, "jl_table_verify: truncated block read");  // TableFormat.java:203-206
        touched += (uint64_t)size[i] + 5;
    }
    Route rt(kKindTable, touched, opt().host_threshold);
    if (rt.host) {  // the host SSE4.2 path (one table)
        jlhost::table_verify(file, off, size, n, status);
        rt.ok = true;
        return JL_OK;
    }
    Workspace *w = nullptr;
    if (int r = get_ws(&w)) return r;
    const std::vector<Chunk> ch = plan_chunks(off, size, 5, n);  // block || 5-byte trailer
    if (int r = ensure_chunk_bufs(*w, ch, 1, 8 + 4)) return r;
    HostSrc src(file, file_bytes);
    const int rc = pipeline(
        *w, ch.size(),
        [&](uint64_t i, Slot &sl) -> int {
            const Chunk &k = ch[i];
            if (int r = slot_put_data(sl, src, k.lo, k.hi - k.lo)) return r;
            const uint64_t m = k.b - k.a;
            return slot_put_desc(sl, {{off + k.a, m * 8}, {size + k.a, m * 4}});
        },
        [&](uint64_t i, Slot &sl) -> int {
            const Chunk &k = ch[i];
            const uint64_t m = k.b - k.a;
            jlk::KParams P = base_params((const uint8_t *)sl.d_in.p - k.lo, m, jlk::MODE_TABLE_VERIFY);
            P.base_bytes = k.hi;
            P.off = (const uint64_t *)sl.part[0];
            P.len = (const uint32_t *)sl.part[1];
            P.len_add = 1;  // block || type byte
            P.out8 = (uint8_t *)sl.d_out.p;
            if (int r = run_general(P, w->stream)) return r;
            JL_HIP(hipMemcpyAsync(status + k.a, sl.d_out.p, m, hipMemcpyDeviceToHost, w->stream));
            return JL_OK;
        });
    rt.ok = rc == JL_OK;
    return rc;
}

// The input tables of a compaction verified together (VersionSet.makeInputIterator
// opens every input table with paranoidChecks, J/db/VersionSet.java:820-823): the
// tables are packed into 64 MiB groups, each group staged into one pinned buffer,
// copied with one H2D transfer and verified with one launch over all its handles
// (offsets moved by each table's place in the group), double-buffered like the
// single-table path.  Small batches take the host path (JL_OPT_HOST_THRESHOLD).
int jl_tables_verify(uint64_t n_tables, const uint8_t *const *files, const uint64_t *file_bytes, const uint64_t *first,
                     const uint64_t *off, const uint32_t *size, uint8_t *status) {
    if (int r = ensure_ready()) return r;
    if (n_tables == 0) return JL_OK;
    if (!files || !file_bytes || !first) return fail(JL_ERR_INVALID, "jl_tables_verify: null pointer");
    const uint64_t n = first[n_tables];
    if (first[0] != 0) return fail(JL_ERR_INVALID, "jl_tables_verify: first[0] must be 0");
    if (n && (!off || !size || !status)) return fail(JL_ERR_INVALID, "jl_tables_verify: null pointer");
    // every handle range inside [0, first[n_tables]) before any off[] / size[] access
    for (uint64_t t = 0; t < n_tables; t++)
        if (first[t + 1] < first[t] || first[t + 1] > n)
            return fail(JL_ERR_INVALID, "jl_tables_verify: handle ranges not ascending");
    uint64_t touched = 0;
    for (uint64_t t = 0; t < n_tables; t++) {
        if (first[t + 1] > first[t] && !files[t]) return fail(JL_ERR_INVALID, "jl_tables_verify: null table");
        for (uint64_t i = first[t]; i < first[t + 1]; i++) {
            if (off[i] > file_bytes[t] || (uint64_t)size[i] + 5 > file_bytes[t] - off[i])
                return fail(JL_ERR_INVALID, "jl_tables_verify: truncated block read");  // TableFormat.java:203-206
            touched += (uint64_t)size[i] + 5;
        }
    }
    if (n == 0) return JL_OK;
    Route rt(kKindTables, touched, opt().host_threshold);
    if (rt.host) {
        for (uint64_t t = 0; t < n_tables; t++)
            jlhost::table_verify(files[t], off + first[t], size + first[t], first[t + 1] - first[t], status + first[t]);
        rt.ok = true;
        return JL_OK;
    }
    // groups of whole tables (a table larger than a chunk is a group of its own)
    struct Group {
        uint64_t t0, t1, bytes;
    };
    std::vector<Group> groups;
    std::vector<uint64_t> place(n_tables);  // each table's offset in its group
    for (uint64_t t = 0; t < n_tables; t++) {
        const uint64_t sz = align256(file_bytes[t]);
        if (groups.empty() || (groups.back().bytes + sz > JL_STREAM_CHUNK_BYTES && groups.back().t1 > groups.back().t0))
            groups.push_back({t, t, 0});
        place[t] = groups.back().bytes;
        groups.back().t1 = t + 1;
        groups.back().bytes += sz;
    }
    Workspace *w = nullptr;
    if (int r = get_ws(&w)) return r;
    uint64_t max_bytes = 0, max_h = 0;
    for (const Group &g : groups) {
        max_bytes = std::max(max_bytes, g.bytes);
        max_h = std::max(max_h, first[g.t1] - first[g.t0]);
    }
    for (Slot &sl : w->slot) {
        JL_HIP(sl.d_in.ensure(max_bytes + kSlack));
        JL_HIP(sl.d_out.ensure(max_h));
        JL_HIP(sl.d_desc.ensure(max_h * 12 + 4 * 256));
    }
    std::vector<uint64_t> adj;
    const int rc = pipeline(
        *w, groups.size(),
        [&](uint64_t gi, Slot &sl) -> int {
            const Group &g = groups[gi];
            JL_HIP(hipStreamWaitEvent(sl.st, sl.used, 0));
            JL_HIP(hipEventSynchronize(sl.copied));  // the staging buffer's previous copy is done
            JL_HIP(sl.h_data.ensure(g.bytes));
            for (uint64_t t = g.t0; t < g.t1; t++)
                par_memcpy((uint8_t *)sl.h_data.p + place[t], files[t], file_bytes[t]);
            JL_HIP(hipMemcpyAsync(sl.d_in.p, sl.h_data.p, g.bytes, hipMemcpyHostToDevice, sl.st));
            const uint64_t h0 = first[g.t0], m = first[g.t1] - h0;
            adj.resize(m);
            for (uint64_t t = g.t0; t < g.t1; t++)
                for (uint64_t i = first[t]; i < first[t + 1]; i++) adj[i - h0] = off[i] + place[t];
            return slot_put_desc(sl, {{adj.data(), m * 8}, {size + h0, m * 4}});
        },
        [&](uint64_t gi, Slot &sl) -> int {
            const Group &g = groups[gi];
            const uint64_t h0 = first[g.t0], m = first[g.t1] - h0;
            if (m == 0) return JL_OK;
            jlk::KParams P = base_params(sl.d_in.p, m, jlk::MODE_TABLE_VERIFY);
            P.base_bytes = g.bytes;
            P.off = (const uint64_t *)sl.part[0];
            P.len = (const uint32_t *)sl.part[1];
            P.len_add = 1;  // block || type byte
            P.out8 = (uint8_t *)sl.d_out.p;
            if (int r = run_general(P, w->stream)) return r;
            JL_HIP(hipMemcpyAsync(status + h0, sl.d_out.p, m, hipMemcpyDeviceToHost, w->stream));
            return JL_OK;
        });
    rt.ok = rc == JL_OK;
    return rc;
}

// --------------------------------------------------------------- log shims
int jl_log_headers_dev(const void *d_base, const uint64_t *d_off, const uint32_t *d_len, const uint8_t *d_type,
                       uint64_t n, uint8_t *d_header, void *stream) {
    if (int r = ensure_ready()) return r;
    if (int r = no_capture(stream, "jl_log_headers_dev")) return r;
    if (n == 0) return JL_OK;
    if (!d_base || !d_off || !d_len || !d_type || !d_header)
        return fail(JL_ERR_INVALID, "jl_log_headers_dev: null pointer");
    jlk::KParams P = base_params(d_base, n, jlk::MODE_LOG_HEADER);
    P.off = d_off;
    P.len = d_len;
    P.type = d_type;
    P.out8 = d_header;
    return run_general(P, pick(stream));
}

int jl_log_emit_dev(const void *d_src, const uint64_t *d_frag_hdr_off, const uint64_t *d_frag_src_off,
                    const uint32_t *d_frag_len, const uint8_t *d_frag_type, uint64_t n_frags, uint64_t log_bytes,
                    uint8_t *d_log, void *stream) {
    if (int r = ensure_ready()) return r;
    if (int r = no_capture(stream, "jl_log_emit_dev")) return r;
    if (n_frags == 0 && log_bytes == 0) return JL_OK;
    if (!d_log || (n_frags && (!d_src || !d_frag_hdr_off || !d_frag_src_off || !d_frag_len || !d_frag_type)))
        return fail(JL_ERR_INVALID, "jl_log_emit_dev: null pointer");
    hipStream_t st = pick(stream);
    JL_HIP(hipMemsetAsync(d_log, 0, log_bytes, st));  // block trailers (J/db/LogWriter.java:101-107)
    if (n_frags == 0) return JL_OK;
    uint64_t *pay = nullptr;  // payload offsets: stream-ordered scratch, so the call stays asynchronous
    if (hipMallocAsync((void **)&pay, n_frags * 8, st) != hipSuccess)
        return fail(JL_ERR_NOMEM, "jl_log_emit_dev: scratch allocation failed");
    hipError_t e = jlk::launch_log_copy((const uint8_t *)d_src, d_frag_src_off, d_frag_hdr_off, d_frag_len, n_frags,
                                        d_log, pay, st);
    jlk::KParams P = base_params(d_log, n_frags, jlk::MODE_LOG_HEADER);
    P.off = pay;
    P.len = d_frag_len;
    P.type = d_frag_type;
    P.out8 = d_log;
    P.hdr_off = d_frag_hdr_off;
    const int r = e == hipSuccess ? run_general(P, st) : JL_OK;
    (void)hipFreeAsync(pay, st);
    JL_HIP(e);
    return r;
}

// Fused path (log_stream.hip): one streaming kernel walks and verifies every
// block, a scan of the per-block event counts places them, one compaction
// kernel writes them in file order; one synchronisation at the end.  Blocks
// with more than kLogStreamCap events (average record < 121 B) do not fit the
// per-block slots: *fallback is set and nothing is written.
constexpr uint32_t kLogStreamCap = 256;

static int log_verify_stream(Workspace &c, const void *d_log, uint64_t log_bytes, jl_log_event *d_events,
                             uint64_t cap, uint64_t *n_events, hipStream_t st, bool *fallback) {
    *fallback = false;
    const uint64_t nb = (log_bytes + 32767) / 32768;
    if (nb >= (1ull << 31)) {
        *fallback = true;
        return JL_OK;
    }
    // ws_ls: count[nb + 1] | first_bad[nb] | overflow | starts[nb + 1] (u64, 8-B aligned)
    const size_t cnt_b = (nb + 1) * 4, fb_b = nb * 4, flag_b = 4;
    const size_t st_off = (cnt_b + fb_b + flag_b + 7) & ~(size_t)7;
    JL_HIP(c.ws_ls.ensure(st_off + (nb + 1) * 8));
    JL_HIP(c.ws_lsev.ensure(nb * kLogStreamCap * sizeof(jlk::LogEvent)));
    char *ws = (char *)c.ws_ls.p;
    jlk::LogStreamArgs A;
    A.log = (const uint8_t *)d_log;
    A.size = log_bytes;
    A.n_blocks = (uint32_t)nb;
    A.cap = kLogStreamCap;
    A.slots = (jlk::LogEvent *)c.ws_lsev.p;
    A.count = (uint32_t *)ws;
    A.first_bad = (uint32_t *)(ws + cnt_b);
    A.overflow = (uint32_t *)(ws + cnt_b + fb_b);
    uint64_t *start = (uint64_t *)(ws + st_off);
    JL_HIP(hipMemsetAsync(A.count + nb, 0, 4, st));  // count[nb] = 0: start[nb] is the total
    JL_HIP(hipMemsetAsync(A.overflow, 0, 4, st));
    JL_HIP(jlk::launch_logstream(ctx().d_img_log, A, ctx().cus, st));
    hipcub::TransformInputIterator<uint64_t, U32ToU64, const uint32_t *> it(A.count, U32ToU64{});
    size_t tmp = 0;
    JL_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, tmp, it, start, (int)(nb + 1), st));
    JL_HIP(c.ws_tmp.ensure(tmp));
    JL_HIP(hipcub::DeviceScan::ExclusiveSum(c.ws_tmp.p, tmp, it, start, (int)(nb + 1), st));
    JL_HIP(jlk::launch_logstream_compact(A, start, (jlk::LogEvent *)d_events, cap, st));
    uint64_t total = 0;
    uint32_t over = 0;
    JL_HIP(hipMemcpyAsync(&total, start + nb, 8, hipMemcpyDeviceToHost, st));
    JL_HIP(hipMemcpyAsync(&over, A.overflow, 4, hipMemcpyDeviceToHost, st));
    JL_HIP(hipStreamSynchronize(st));
    if (over) {
        *fallback = true;
        return JL_OK;
    }
    *n_events = total;
    if (total > cap) return fail(JL_ERR_CAPACITY, "jl_log_verify: event array too small");
    return JL_OK;
}

// Chunked log verification (log_chunks.hip): walk -> scans -> dense blocks ->
// rounds setup -> build -> crc_gv4_kernel<MODE_LOG_CHUNK> -> combine -> apply,
// stream-ordered, one pass for any log: the round table is sized for at most
// kLCSlots events per 32 KiB block (records of ~500 B and up), and the blocks
// of more events (dense) are verified whole by lc_dense instead.
// d_result null: synchronous (the count read back); else asynchronous: the
// result words go to d_result on the stream and the call returns after the
// launches.
static int log_verify_chunks(Workspace &c, const void *d_log, uint64_t log_bytes, bool checksum,
                             jl_log_event *d_events, uint64_t cap, uint64_t *n_events, hipStream_t st,
                             uint64_t *d_result = nullptr) {
    if (log_bytes >= (1ull << 40)) return fail(JL_ERR_INVALID, "jl_log_verify: log larger than 1 TiB");
    const uint64_t nb = (log_bytes + 32767) / 32768, ng = (nb + jlk::kLCGroup - 1) / jlk::kLCGroup;
    auto al = [](size_t b) { return (b + 255) & ~(size_t)255; };
    const size_t hn = jlk::kLCCounters * ng + 1;
    const size_t o_cnt = 256, o_start = o_cnt + al((nb + 1) * 4), o_hist = o_start + al((nb + 1) * 8), o_hscan = o_hist + al(hn * 4),
                 o_rt = o_hscan + al(hn * 4), o_ts = o_rt + al(jlk::kLCCounters * 4),
                 o_ts0 = o_ts + al((nb / jlk::kLSTile + 1) * 8), o_pr = o_ts0 + al((nb / jlk::kLSTile + 1) * 8),
                 o_s0 = o_pr + al(nb * 4), o_rd = o_s0 + al((nb + 1) * 8), o_rs = o_rd + al((nb / jlk::kLSTile + 1) * 4), o_fb = o_rs + al((jlk::kLCBins + 1) * 4), o_do = o_fb + al(nb * 4),
                 o_flag = o_do + al(nb * 8), o_res = o_flag + 256, o_dl = o_res + 256, o_nl = o_dl + al(nb * 4),
                 o_di = o_nl + al(nb * 4), o_dw = o_di + al(nb * 4),
                 o_end = o_dw + al(nb * jlk::kDWMax * 2);
    const size_t lc_cap = c.ws_lc.cap;
    JL_HIP(c.ws_lc.ensure(o_end));
    if (c.ws_lc.cap != lc_cap) c.lc_dirty = true;  // a new buffer: its counters are not zero
    JL_HIP(c.ws_slot.ensure(nb * jlk::kLCSlots * 8));
    // The dense blocks' runs of events (lc_dense): no more runs than events, and
    // at most the caller's capacity of events (more fail the call anyway), plus one
    // link entry per pass after a block's first (a pass holds kLDRuns runs, so
    // links <= runs / kLDRuns).  With pools (>= 8 blocks per lc_dense workgroup) a
    // workgroup leaves less than a pool unused at the end and fewer than
    // kLDRuns + 1 entries per refill: refills <= entries / (pool - kLDRuns - 1) + grid.
    // A count-only call (no event array) stashes nothing: lc_dense skips the stores
    // of a pass that does not fit (stash_cap 0), and lc_build has no events to write.
    // (a block's first pass may hold lc_dwalk's kDWMax records: segments of <= kDWMax + 1)
    const uint64_t need0 = d_events ? std::min<uint64_t>(cap, nb * (uint64_t)jlk::kLDMaxEv) : 0;
    const uint64_t need = need0 + need0 / jlk::kLDRuns + (need0 ? nb : 0);
    const uint64_t grid = jlk::lc_dense_grid(ctx().cus);
    const uint64_t pool = need && nb >= 8 * grid ? jlk::kLDPool : 0;
    const uint64_t seg = std::max<uint64_t>(jlk::kLDRuns, jlk::kDWMax) + 1;
    const uint64_t stash_cap = pool ? need + (need / (pool - seg) + grid) * seg + grid * pool : need;
    JL_HIP(c.ws_stash.ensure(std::max<uint64_t>(stash_cap, 1) * 8));
    char *ws = (char *)c.ws_lc.p;
    jlk::LCArgs A;
    memset(&A, 0, sizeof(A));
    A.log = (const uint8_t *)d_log;
    A.size = log_bytes;
    A.n_blocks = (uint32_t)nb;
    A.n_grp = (uint32_t)ng;
    A.checksum = checksum ? 1 : 0;
    A.slots = (uint64_t *)c.ws_slot.p;
    A.count = (uint32_t *)(ws + o_cnt);
    A.start = (uint64_t *)(ws + o_start);
    A.hist = (uint32_t *)(ws + o_hist);
    A.hscan = (uint32_t *)(ws + o_hscan);
    A.rowtot = (uint32_t *)(ws + o_rt);
    A.tstat = (uint64_t *)(ws + o_ts);
    A.tstat0 = (uint64_t *)(ws + o_ts0);
    A.pred = (uint32_t *)(ws + o_pr);
    A.start0 = (uint64_t *)(ws + o_s0);
    A.ready0 = (uint32_t *)(ws + o_rd);
    if (++c.lc_gen == 0) c.lc_gen = 1;
    A.gen = c.lc_gen;
    A.rstart = (uint32_t *)(ws + o_rs);
    A.first_bad = (uint32_t *)(ws + o_fb);
    A.dense_off = (uint64_t *)(ws + o_do);
    A.cap_flag = (uint32_t *)(ws + o_flag);
    A.stash_ctr = (unsigned long long *)(ws + o_flag + 8);
    A.dense_ctr = (uint32_t *)ws;  // at a fixed place: the previous verification zeroed it
    A.nu_ctr = A.dense_ctr + 6;
    A.dense_list = (uint32_t *)(ws + o_dl);
    A.nlong = (uint32_t *)(ws + o_nl);
    A.dw_info = (uint32_t *)(ws + o_di);
    A.dw_off = (uint16_t *)(ws + o_dw);
    A.stash = (uint64_t *)c.ws_stash.p;
    A.stash_cap = stash_cap;
    A.stash_pool = pool;
    if (!c.h_res) JL_HIP(hipHostMalloc((void **)&c.h_res, 64, hipHostMallocCoherent));
    A.result = d_result ? d_result : c.h_res;
    A.ev = (jlk::LogEvent *)d_events;
    A.ev_cap = d_events ? cap : 0;
    A.aux = ctx().d_aux;
    A.seed0 = jlmath::slice4_inv(0xffffffffu);
    // walk (initialises count[nb], the hist tail, first_bad, cap_flag, the stash counter);
    // dense blocks: verified whole, exact counts, events stashed
    // [0] lc_walk's dense list, [1] lc_dense's chunk counter, [2] gv4 round batches, [3] lc_scan's work ids,
    // [6] lc_dwalk's blocks, [7] those whose events it did not predict
    // (lc_finish zeroes them again at the end; r5 dropped the memset here: a
    // 4.4 us fill dispatch plus a ~6 us gap before it in every verification)
    if (c.lc_dirty) JL_HIP(hipMemsetAsync(A.dense_ctr, 0, 32, st));
    c.lc_dirty = true;  // until the last launch of this verification is enqueued
    JL_HIP(jlk::launch_lc_walk(A, st));
    // the dense blocks' headers (lc_dwalk, one lane per block), then their crcs
    // (lc_dense).  r5 measured lc_dwalk of half the list on a second stream beside
    // lc_dense of the other half: random lengths 2.64 -> 2.47 ms, but every other
    // set 3-5 % slower (the cross-stream waits and the extra launches, ~40 us)
    // (r6: lc_dwalk on a second stream beside lc_dense, publishing each block to it,
    // ran the random set 3 % faster than its base but needed publication checks in
    // lc_dense that cost every dense set 2-3 %: branch study-r6-dwalk-lanes)
    JL_HIP(jlk::launch_lc_dwalk(A, st));
    if (opt().failpoint & 1) JL_HIP(jlk::launch_lc_failpoint(A, st));
    // the in-place kernel when the workspace's last verification had lc_dwalk's blocks
    // (a log verified again, or the next chunk of one: a guess, either kernel is right)
    if (!c.h_hint) {
        JL_HIP(hipHostMalloc((void **)&c.h_hint, 64, hipHostMallocCoherent));
        *c.h_hint = 0;
    }
    A.hint = c.h_hint;
    JL_HIP(jlk::launch_lc_dense(A, ctx().cus, *(volatile uint32_t *)c.h_hint != 0u, st));
    JL_HIP(jlk::launch_lc_scan(A, st));  // event starts per block; chunk ranks per (bin, group)
    // capacities of the round table, the multi-chunk records and their chunk states:
    // <= kLCSlots records in a block that is not dense, and a block's bytes bound its extra chunks
    A.round_cap = nb * (jlk::kLCSlots + 10) / 8 + jlk::kLCBins + 1;
    A.big_cap = nb * 8 + 1;
    A.part_cap = nb * 17 + 1;
    if (checksum) {
        JL_HIP(c.ws_desc.ensure(A.round_cap * 8 * sizeof(jlk::GDesc)));
        JL_HIP(c.ws_big.ensure(A.big_cap * sizeof(jlk::LCBig)));
        JL_HIP(c.ws_part.ensure(A.part_cap * 4));
        A.desc = (jlk::GDesc *)c.ws_desc.p;
        A.big = (jlk::LCBig *)c.ws_big.p;
        A.parts = (uint32_t *)c.ws_part.p;
        JL_HIP(jlk::launch_lc_setup(A, st));
    }
    JL_HIP(jlk::launch_lc_build(A, st));
    if (checksum) {
        jlk::GV4Args G;
        memset(&G, 0, sizeof(G));
        G.P = base_params(d_log, nb, jlk::MODE_LOG_CHUNK);
        G.P.out32 = A.first_bad;
        G.desc = A.desc;
        G.n_rounds = A.rstart + jlk::kLCBins;
        G.deal = A.dense_ctr + 2;  // zero when the verification starts (lc_finish of the one before)
        G.seed0 = jlmath::slice4_inv(0xffffffffu);
        G.parts = A.parts;
        JL_HIP(gv4_launch(G, st));
        JL_HIP(jlk::launch_lc_combine(A, st));
        JL_HIP(jlk::launch_lc_apply(A, st));
    }
    c.lc_dirty = false;  // lc_finish (lc_apply, or lc_build without checksums) zeroes the counters
    if (d_result) return JL_OK;  // asynchronous: the caller reads d_result in stream order
    // events, dense blocks, capacity flag (lc_finish, written to c.h_res by the
    // last kernel): wait by polling the stream (a blocking synchronise sleeps,
    // and a D2H copy of the words cost ~50 us between back-to-back calls)
    JL_HIP(poll_stream(st));
    const volatile uint64_t *hr = c.h_res;
    const uint64_t res[3] = {hr[0], hr[1], hr[2]};
    if (res[2]) {
        if (res[2] & jlk::kLCFlagStale) c.lc_dirty = true;  // the next call zeroes the counters itself
        return fail(JL_ERR_HIP, std::string("jl_log_verify: ") +
                                    (res[2] & jlk::kLCFlagStale ? "work counters not reset by the previous verification"
                                     : res[2] & jlk::kLCFlagInconsistent ? "records of a block overlap"
                                                                        : "internal capacity exceeded"));
    }
    *n_events = res[0];
    return JL_OK;
}

// One-launch verification of a small log (lc_small_kernel, log_chunks.hip):
// d_result null: synchronous (the count read back from the result words the
// kernel writes into coherent host memory); else asynchronous.
static int log_verify_small(Workspace &c, const void *d_log, uint64_t log_bytes, bool checksum, jl_log_event *d_events,
                            uint64_t cap, uint64_t *n_events, hipStream_t st, uint64_t *d_result = nullptr) {
    // (d_events may be pinned host memory: jl_log_verify's small-log path)
    const uint64_t nb = (log_bytes + 32767) / 32768;
    const size_t cap0 = c.ws_small.cap;
    JL_HIP(c.ws_small.ensure(256 + nb * 8));
    if (c.ws_small.cap != cap0) c.small_dirty = true;
    // a zero ticket counter and statuses that no tag matches: zero once per buffer
    // (the statuses then carry each call's tag, the last ticket re-zeroes the counter)
    if (c.small_dirty) JL_HIP(hipMemsetAsync(c.ws_small.p, 0, c.ws_small.cap, st));
    c.small_dirty = true;  // until the launch is enqueued
    if (++c.small_gen == 0) c.small_gen = 1;
    if (!c.h_res) JL_HIP(hipHostMalloc((void **)&c.h_res, 64, hipHostMallocCoherent));
    jlk::LSmallArgs A;
    memset(&A, 0, sizeof(A));
    A.log = (const uint8_t *)d_log;
    A.size = log_bytes;
    A.n_blocks = (uint32_t)nb;
    A.checksum = checksum ? 1 : 0;
    A.seed0 = jlmath::slice4_inv(0xffffffffu);
    A.gen = c.small_gen;
    A.aux = ctx().d_aux;
    A.ev = (jlk::LogEvent *)d_events;
    A.ev_cap = d_events ? cap : 0;
    A.ticket = (uint32_t *)c.ws_small.p;
    A.tstat = (uint64_t *)((char *)c.ws_small.p + 256);
    A.result = d_result ? d_result : c.h_res;
    JL_HIP(jlk::launch_lc_small(A, st));
    c.small_dirty = false;
    if (d_result) return JL_OK;
    JL_HIP(poll_stream(st));
    *n_events = ((const volatile uint64_t *)c.h_res)[0];
    return JL_OK;
}
static bool small_log(uint64_t log_bytes, int checksum) {
    return checksum != JL_LOG_CHECKSUM_FUSED && (int64_t)log_bytes <= opt().log_small_max;
}

// Verifies d_log[0, log_bytes) on `st` with the calling thread's scratch `c`;
// *n_events is known on return (the event count is read back) and the events
// are complete in stream order.
static int log_verify_impl(Workspace &c, const void *d_log, uint64_t log_bytes, int checksum, jl_log_event *d_events,
                           uint64_t cap, uint64_t *n_events, hipStream_t st) {
    if (checksum == JL_LOG_CHECKSUM_FUSED) {  // the single-pass kernel, unless a block overflows its slots
        bool fallback = false;
        *n_events = 0;
        if (log_bytes == 0) return JL_OK;
        if (int r = log_verify_stream(c, d_log, log_bytes, d_events, cap, n_events, st, &fallback)) return r;
        if (!fallback) return JL_OK;
    }
    *n_events = 0;
    if (log_bytes == 0) return JL_OK;
    if (small_log(log_bytes, checksum)) {
        if (int r = log_verify_small(c, d_log, log_bytes, checksum != JL_LOG_NO_CHECKSUM, d_events, cap, n_events, st))
            return r;
    } else if (int r = log_verify_chunks(c, d_log, log_bytes, checksum != JL_LOG_NO_CHECKSUM, d_events, cap, n_events,
                                         st)) {
        return r;
    }
    if (*n_events > cap) return fail(JL_ERR_CAPACITY, "jl_log_verify: event array too small");
    return JL_OK;
}

// The log-verify scratch of a workspace is reused by every call of its thread:
// a call on another stream than an asynchronous call still possibly in flight
// first makes its stream wait for that call's completion event (device-side,
// no host wait).  Synchronous calls finish their work before they return.
static int ws_order(Workspace &w, hipStream_t st) {
    if (w.async_pending && w.async_st != st) JL_HIP(hipStreamWaitEvent(st, w.async_done, 0));
    return JL_OK;
}
// A synchronous call does not always synchronise its stream (an empty log returns
// before any launch, and ws_order only made its stream wait on the device), so the
// pending asynchronous call is waited for on the host before it is forgotten: a
// completed event costs one query.
static int ws_after(Workspace &w, hipStream_t st, bool async, int rc) {
    if (!async || rc) {
        if (w.async_pending) (void)hipEventSynchronize(w.async_done);
        w.async_pending = false;
        return rc;
    }
    JL_HIP(hipEventRecord(w.async_done, st));
    w.async_pending = true;
    w.async_st = st;
    return JL_OK;
}

int jl_log_verify_dev(const void *d_log, uint64_t log_bytes, int checksum, jl_log_event *d_events, uint64_t cap,
                      uint64_t *n_events, void *stream) {
    if (int r = ensure_ready()) return r;
    if (int r = no_capture(stream, "jl_log_verify_dev")) return r;
    if (!n_events || (log_bytes && !d_log)) return fail(JL_ERR_INVALID, "jl_log_verify_dev: null pointer");
    if (checksum < 0 || checksum > JL_LOG_CHECKSUM_FUSED) return fail(JL_ERR_INVALID, "jl_log_verify_dev: bad checksum mode");
    Workspace *w = nullptr;
    if (int r = get_ws(&w)) return r;
    const hipStream_t st = pick(stream);
    if (int r = ws_order(*w, st)) return r;
    return ws_after(*w, st, false, log_verify_impl(*w, d_log, log_bytes, checksum, d_events, cap, n_events, st));
}

int jl_log_verify_dev_async(const void *d_log, uint64_t log_bytes, int checksum, jl_log_event *d_events, uint64_t cap,
                            uint64_t *d_result, void *stream) {
    if (int r = ensure_ready()) return r;
    if (int r = no_capture(stream, "jl_log_verify_dev_async")) return r;
    if (!d_result || (log_bytes && !d_log)) return fail(JL_ERR_INVALID, "jl_log_verify_dev_async: null pointer");
    if (checksum < 0 || checksum > JL_LOG_CHECKSUM_TWO_PASS)
        return fail(JL_ERR_INVALID, "jl_log_verify_dev_async: bad checksum mode");
    Workspace *w = nullptr;
    if (int r = get_ws(&w)) return r;
    const hipStream_t st = pick(stream);
    if (int r = ws_order(*w, st)) return r;
    if (log_bytes == 0) {
        JL_HIP(hipMemsetAsync(d_result, 0, 3 * sizeof(uint64_t), st));
        return JL_OK;
    }
    uint64_t n = 0;
    const bool cs = checksum != JL_LOG_NO_CHECKSUM;
    return ws_after(*w, st, true,
                    small_log(log_bytes, checksum) ? log_verify_small(*w, d_log, log_bytes, cs, d_events, cap, &n, st, d_result)
                                                   : log_verify_chunks(*w, d_log, log_bytes, cs, d_events, cap, &n, st, d_result));
}

// A small host-memory log (at most JL_OPT_LOG_SMALL_MAX): one H2D copy (staged in
// kStagePiece pieces, each DMA'd as soon as it is in pinned memory; 1 / 2 MiB
// pieces measured no better, same box, r6g), one lc_small launch that
// writes the events straight into pinned host memory, one wait, one host copy of
// the events into the caller's array.  The chunked pipeline below costs this
// call a second round trip (the event rebase and D2H after the count is known).
static int log_verify_small_host(Workspace &w, const uint8_t *log, uint64_t log_bytes, bool checksum, jl_log_event *events,
                                 uint64_t cap, uint64_t *n_events) {
    Slot &sl = w.slot[0];
    const uint64_t ev_max = log_bytes / 7 + 2;  // physical records of the log, at most
    JL_HIP(sl.d_in.ensure(log_bytes + kSlack));
    JL_HIP(w.h_ev.ensure(ev_max * sizeof(jl_log_event)));
    HostSrc src(log, log_bytes);
    if (src.direct) {
        JL_HIP(hipMemcpyAsync(sl.d_in.p, log, log_bytes, hipMemcpyHostToDevice, w.stream));
    } else {
        JL_HIP(sl.h_data.ensure(log_bytes));
        for (uint64_t a = 0; a < log_bytes; a += kStagePiece) {
            const uint64_t m = std::min(kStagePiece, log_bytes - a);
            par_memcpy((uint8_t *)sl.h_data.p + a, log + a, m);
            JL_HIP(hipMemcpyAsync((uint8_t *)sl.d_in.p + a, (const uint8_t *)sl.h_data.p + a, m, hipMemcpyHostToDevice,
                                  w.stream));
        }
    }
    uint64_t n = 0;
    if (int r = log_verify_small(w, sl.d_in.p, log_bytes, checksum, (jl_log_event *)w.h_ev.p, ev_max, &n, w.stream))
        return r;
    *n_events = n;
    if (n > cap) return fail(JL_ERR_CAPACITY, "jl_log_verify: event array too small");
    par_memcpy(events, w.h_ev.p, n * sizeof(jl_log_event));
    return JL_OK;
}

// Host-memory log verification: chunks of JL_STREAM_CHUNK_BYTES (whole 32 KiB
// blocks, so no record straddles a chunk and the final short block is the last
// chunk's) through the double-buffered pipeline; each chunk's events are moved
// to file offsets and copied out while the following chunks' bytes are in flight.
int jl_log_verify(const uint8_t *log, uint64_t log_bytes, int checksum, jl_log_event *events, uint64_t cap,
                  uint64_t *n_events) {
    if (int r = ensure_ready()) return r;
    if (!n_events || (log_bytes && !log)) return fail(JL_ERR_INVALID, "jl_log_verify: null pointer");
    if (checksum < 0 || checksum > JL_LOG_CHECKSUM_FUSED) return fail(JL_ERR_INVALID, "jl_log_verify: bad checksum mode");
    static_assert(JL_STREAM_CHUNK_BYTES % 32768 == 0, "log chunks must be whole blocks");
    *n_events = 0;
    if (log_bytes == 0) return JL_OK;
    Route rt(kKindLog, log_bytes, opt().log_host_threshold);
    if (rt.host) {  // the host SSE4.2 path (e.g. one WAL at recovery)
        jlhost::log_verify(log, log_bytes, checksum, events, cap, n_events);
        if (*n_events > cap) return fail(JL_ERR_CAPACITY, "jl_log_verify: event array too small");
        rt.ok = true;
        return JL_OK;
    }
    Workspace *w = nullptr;
    if (int r = get_ws(&w)) return r;
    if (int r = ws_order(*w, w->stream)) return r;
    if (small_log(log_bytes, checksum)) {
        const int rc = log_verify_small_host(*w, log, log_bytes, checksum != JL_LOG_NO_CHECKSUM, events, cap, n_events);
        if (rc) (void)hipStreamSynchronize(w->stream);  // nothing of the call left in flight
        w->async_pending = false;  // w->stream waited for any earlier asynchronous call, and it is done
        rt.ok = rc == JL_OK;
        return rc;
    }
    const uint64_t CH = JL_STREAM_CHUNK_BYTES, first = std::min(CH, log_bytes);
    const uint64_t ev_cap = first / 7 + 2;  // upper bound on a chunk's physical records
    for (Slot &sl : w->slot) {
        JL_HIP(sl.d_in.ensure(first + kSlack));
        JL_HIP(sl.d_out.ensure(ev_cap * sizeof(jl_log_event)));
    }
    HostSrc src(log, log_bytes);
    uint64_t total = 0;
    // A chunk's events leave by DMA into its slot's pinned h_out, and the host
    // copies them into the caller's array (the copy pool) one chunk later:
    // log_verify_impl returns chunk i's count only once chunk i's kernels are
    // done, so the copy of chunk i-1's events overlaps chunk i's rebase and D2H
    // and chunk i+1's H2D, not chunk i+1's kernels.  r4 copied them with one hipMemcpyAsync into the caller's pageable
    // array, which the runtime stages and the host waits for: on the DBBench set
    // (0.5 GB of events per 4 GiB) the call ran at 38 GiB/s from pinned input.
    struct Out {
        Slot *sl = nullptr;
        uint64_t at = 0, n = 0;
    } pend;
    auto flush = [&]() -> int {  // the pending chunk's events, once its D2H landed (`used`)
        if (!pend.n) return JL_OK;
        JL_HIP(hipEventSynchronize(pend.sl->used));
        par_memcpy(events + pend.at, pend.sl->h_out.p, pend.n * sizeof(jl_log_event));
        pend.n = 0;
        return JL_OK;
    };
    int rc = pipeline(
        *w, (log_bytes + CH - 1) / CH,
        [&](uint64_t i, Slot &sl) { return slot_put_data(sl, src, i * CH, std::min(CH, log_bytes - i * CH)); },
        [&](uint64_t i, Slot &sl) -> int {
            uint64_t n = 0;
            jl_log_event *ev = (jl_log_event *)sl.d_out.p;
            if (int r = log_verify_impl(*w, sl.d_in.p, std::min(CH, log_bytes - i * CH), checksum, ev, ev_cap, &n,
                                        w->stream))
                return r;
            if (n && total + n <= cap) {  // past cap: keep counting for *n_events, copy nothing
                JL_HIP(jlk::launch_event_rebase((jlk::LogEvent *)ev, n, i * CH, w->stream));
                JL_HIP(sl.h_out.ensure(n * sizeof(jl_log_event)));
                JL_HIP(hipMemcpyAsync(sl.h_out.p, ev, n * sizeof(jl_log_event), hipMemcpyDeviceToHost, w->stream));
            }
            // the previous chunk's events (its slot's h_out is next written by chunk i + 1)
            if (int r = flush()) return r;
            if (n && total + n <= cap) pend = Out{&sl, total, n};
            total += n;
            return JL_OK;
        });
    if (!rc) rc = flush();  // the pipeline drained: the last chunk's events landed
    *n_events = total;
    w->async_pending = false;  // the pipeline drained this thread's streams after any earlier async call
    if (rc) return rc;
    if (total > cap) return fail(JL_ERR_CAPACITY, "jl_log_verify: event array too small");
    rt.ok = true;
    return JL_OK;
}

// ------------------------------------------------------------------ helpers
int jl_fill_random_dev(void *d_dst, uint64_t bytes, uint64_t seed, uint64_t first_word, void *stream) {
    if (int r = ensure_ready()) return r;
    if (bytes == 0) return JL_OK;
    if (!d_dst) return fail(JL_ERR_INVALID, "jl_fill_random_dev: null pointer");
    JL_HIP(jlk::launch_fill_random(d_dst, bytes, seed, first_word, pick(stream)));
    return JL_OK;
}

int jl_read_stream_dev(const void *d_src, uint64_t bytes, uint32_t *d_sink, void *stream) {
    if (int r = ensure_ready()) return r;
    if (!d_src || !d_sink || bytes % 16) return fail(JL_ERR_INVALID, "jl_read_stream_dev: bad arguments");
    JL_HIP(jlk::launch_read_stream(d_src, bytes, d_sink, ctx().cus * 8, pick(stream)));
    return JL_OK;
}

}  // extern "C"
