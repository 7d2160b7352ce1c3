// jlcrc_api.hip — C-ABI of the engine (include/jlcrc.h): device context,
// launches, host staging and the caller shims for the four reference call sites.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/jlcrc.h"
#include "crc_math.hpp"
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

struct Context {
    std::mutex mu;  // guards init and the staging workspace of the host-memory entry points
    bool ready = false;
    int device = -1;
    int cus = 0;
    hipStream_t stream = nullptr;
    void *d_img = nullptr;   // 160 KiB LDS image
    void *d_img_v4[4] = {nullptr, nullptr, nullptr, nullptr};  // v4 images for 4 / 8 / 16 lanes per block; [3] gv4
    void *d_img_log = nullptr;  // fused log-verify image (log_stream.hip)
    uint32_t *d_aux = nullptr;
    uint8_t *d_zero = nullptr;  // 4 KiB of zeros (read by predicated-off loads)
    uint32_t *d_scratch = nullptr;  // 4 KiB sink for stores of out-of-range pair members
    // staging workspace (host-memory APIs, log verify)
    DevBuf ws_data, ws_off, ws_len, ws_init, ws_sfx, ws_out, ws_cnt, ws_start, ws_ev, ws_ok, ws_tmp, ws_slot;
    DevBuf ws_ls, ws_lsev;  // fused log verify: per-block counts / first failures, event slots
    // streaming pipeline (jl_crc32c_fixed): two slots, each a device chunk + result
    // buffer, a pinned staging buffer (pageable sources) and its own stream
    struct Slot {
        DevBuf d_in, d_out;
        void *h_stage = nullptr;
        size_t h_cap = 0;
        hipStream_t st = nullptr;
        hipEvent_t done = nullptr;
    } slot[2];
};

Context &ctx() {
    static Context c;
    return c;
}

// Engine options (jl_set_option, include/jlcrc.h): which general-path kernel a
// batch takes and its tuning.  Defaults are the measured best; tests force the
// alternatives.  The study options exist in the study build only (make STUDY=1).
struct Options {
    int general_path = JL_PATH_AUTO;  // JL_OPT_GENERAL_PATH
    int stream_depth = 16;            // JL_OPT_STREAM_DEPTH: 16 / 32 / 48 ring entries
    int partition = 1;                // JL_OPT_STREAM_PARTITION: byte-balanced wave ranges
    int64_t split_cap = -1;           // JL_OPT_SPLIT_CAP: chunks of split blocks (-1: min(2^20, 2048 n))
    int fixed_kernel = 7;             // study: JL_OPT_FIXED_KERNEL (7 = the v4 product kernel)
    int gv4_variant = 0;              // study: JL_OPT_GV4_VARIANT (0 = the product kernel)
};
Options &opt() {
    static Options o;
    return o;
}

int ensure_ready() {
    Context &c = ctx();
    if (c.ready) return JL_OK;
    int r = jl_init(0);
    return r;
}

// NULL is HIP's null (legacy default) stream, as everywhere in HIP, so device
// entry points order with the caller's default-stream work.
hipStream_t pick(void *stream) { return (hipStream_t)stream; }

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
#if JL_STUDY
    if (getenv("JL_PARTITION_DUMP")) {  // debugging: range sizes of the partition
        std::vector<uint64_t> h(waves + 1), hi(P.n);
        (void)hipMemcpyAsync(h.data(), part, (waves + 1) * 8, hipMemcpyDeviceToHost, st);
        (void)hipMemcpyAsync(hi.data(), incl, P.n * 8, hipMemcpyDeviceToHost, st);
        (void)hipStreamSynchronize(st);
        uint64_t mx = 0, mn = ~0ull, bad = 0;
        for (uint64_t w = 0; w < waves; w++) {
            if (h[w + 1] < h[w]) bad++;
            else { mx = std::max(mx, h[w + 1] - h[w]); mn = std::min(mn, h[w + 1] - h[w]); }
        }
        fprintf(stderr, "partition n=%llu waves=%llu min=%llu max=%llu bad=%llu\n", (unsigned long long)P.n,
                (unsigned long long)waves, (unsigned long long)mn, (unsigned long long)mx, (unsigned long long)bad);
    }
#endif
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
    if (P.mode != jlk::MODE_CRC && P.mode != jlk::MODE_TABLE_VERIFY && P.mode != jlk::MODE_LOG_VERIFY) return false;
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
    default: return jlk::launch_gv4_m<jlk::MODE_LOG_VERIFY>(img, A, ctx().d_zero, grid, st);
    }
}

static int run_gv4(const jlk::KParams &P, hipStream_t st) {
    jlk::GV4Args A;
    memset(&A, 0, sizeof(A));
    A.P = P;
    A.seed0 = jlmath::slice4_inv(0xffffffffu);
    A.study = (uint32_t)opt().gv4_variant;
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
#if JL_STUDY
    unsigned long long *d_dbg = nullptr, h_dbg[1 + 4 * 256];
    if (const char *dbg = getenv("JL_GV4_DEBUG")) {  // "lo:hi" valid load range (hex), debugging only
        A.P.dbg_lo = strtoull(dbg, nullptr, 16);
        const char *c = strchr(dbg, ':');
        A.P.dbg_hi = c ? strtoull(c + 1, nullptr, 16) : ~0ull;
        if (e == hipSuccess) e = hipMalloc((void **)&d_dbg, sizeof(h_dbg));
        if (e == hipSuccess) e = hipMemsetAsync(d_dbg, 0, sizeof(h_dbg), st);
        A.P.dbg = d_dbg;
        A.study = 4;
    }
#endif
    if (e == hipSuccess) e = gv4_launch(A, st);
    if (e == hipSuccess && SP.part_cap) e = jlk::launch_gv4_combine(P, SP, parts, st);
#if JL_STUDY
    if (d_dbg) {
        uint32_t hr = 0;
        if (e == hipSuccess) e = hipMemcpyAsync(h_dbg, d_dbg, sizeof(h_dbg), hipMemcpyDeviceToHost, st);
        if (e == hipSuccess) e = hipMemcpyAsync(&hr, n_rounds, 4, hipMemcpyDeviceToHost, st);
        if (e == hipSuccess) e = hipStreamSynchronize(st);
        (void)hipFree(d_dbg);
        fprintf(stderr, "JL_GV4_DEBUG mode=%d n=%llu rounds=%u bad=%llu\n", P.mode, (unsigned long long)P.n, hr, h_dbg[0]);
        for (unsigned long long i = 0; i < h_dbg[0] && i < 256; i++)
            fprintf(stderr, "  round %llu entry %llu lane %llu addr/idx %llx\n", h_dbg[1 + 4 * i], h_dbg[2 + 4 * i],
                    h_dbg[3 + 4 * i], h_dbg[4 + 4 * i]);
    }
#endif
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
#if JL_STUDY
    if (o.general_path == 3 && !getenv("JL_STREAM_DEBUG")) {  // the r1 chunked kernel
        JL_HIP(jlk::launch_general(ctx().d_img, P, grid_for(P.n), st));
        return JL_OK;
    }
    if (const char *dbg = getenv("JL_STREAM_DEBUG")) {  // "lo:hi" valid load range (hex), debugging only
        jlk::KParams Q = P;
        Q.dbg_lo = strtoull(dbg, nullptr, 16);
        const char *c = strchr(dbg, ':');
        Q.dbg_hi = c ? strtoull(c + 1, nullptr, 16) : ~0ull;
        unsigned long long *d_dbg = nullptr, h_dbg[1 + 4 * 256];
        JL_HIP(hipMalloc((void **)&d_dbg, sizeof(h_dbg)));
        JL_HIP(hipMemsetAsync(d_dbg, 0, sizeof(h_dbg), st));
        Q.dbg = d_dbg;
        JL_HIP(jlk::launch_stream(ctx().d_img, Q, nullptr, grid_for(P.n), o.stream_depth, st));
        JL_HIP(hipMemcpyAsync(h_dbg, d_dbg, sizeof(h_dbg), hipMemcpyDeviceToHost, st));
        JL_HIP(hipStreamSynchronize(st));
        (void)hipFree(d_dbg);
        fprintf(stderr, "JL_STREAM_DEBUG mode=%d n=%llu bad=%llu\n", P.mode, (unsigned long long)P.n, h_dbg[0]);
        return JL_OK;
    }
#endif
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
        if (value < JL_PATH_AUTO || value > (JL_STUDY ? 3 : JL_PATH_GV4)) break;
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
#if JL_STUDY
    case JL_OPT_FIXED_KERNEL:
        o.fixed_kernel = (int)value;
        return JL_OK;
    case JL_OPT_GV4_VARIANT:
        if (value < 0 || value > 5) break;
        o.gv4_variant = (int)value;
        return JL_OK;
#endif
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
    case JL_OPT_FIXED_KERNEL: return o.fixed_kernel;
    case JL_OPT_GV4_VARIANT: return o.gv4_variant;
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
    JL_HIP(hipStreamCreateWithFlags(&c.stream, hipStreamNonBlocking));
    std::vector<uint32_t> img = jlmath::build_lds_image();
    std::vector<uint32_t> aux = jlmath::build_aux();
    JL_HIP(hipMalloc(&c.d_img, jlmath::kImageBytes));
    JL_HIP(hipMalloc((void **)&c.d_aux, aux.size() * 4));
    JL_HIP(hipMalloc((void **)&c.d_zero, 4096));
    JL_HIP(hipMalloc((void **)&c.d_scratch, 4096));
    JL_HIP(hipMemcpy(c.d_img, img.data(), jlmath::kImageBytes, hipMemcpyHostToDevice));
    for (int i = 0; i < 4; i++) {
        std::vector<uint32_t> v4 = i < 3 ? jlmath::build_lds_image_v4(4 << i) : jlmath::build_lds_image_gv4();
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
    c.ready = true;
    return JL_OK;
}

int jl_shutdown(void) {
    Context &c = ctx();
    std::lock_guard<std::mutex> lk(c.mu);
    if (!c.ready) return JL_OK;
    (void)hipSetDevice(c.device);
    (void)hipStreamSynchronize(c.stream);
    for (DevBuf *b : {&c.ws_data, &c.ws_off, &c.ws_len, &c.ws_init, &c.ws_sfx, &c.ws_out, &c.ws_cnt, &c.ws_start,
                      &c.ws_ev, &c.ws_ok, &c.ws_tmp, &c.ws_slot, &c.ws_ls, &c.ws_lsev})
        b->release();
    for (auto &sl : c.slot) {
        sl.d_in.release();
        sl.d_out.release();
        if (sl.h_stage) (void)hipHostFree(sl.h_stage);
        if (sl.done) (void)hipEventDestroy(sl.done);
        if (sl.st) (void)hipStreamDestroy(sl.st);
        sl = Context::Slot();
    }
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
    (void)hipStreamDestroy(c.stream);
    c.d_img = nullptr;
    c.d_aux = nullptr;
    c.d_zero = nullptr;
    c.stream = nullptr;
    c.ready = false;
    c.device = -1;
    return JL_OK;
}

// ----------------------------------------------------------- batch checksums
int jl_crc32c_fixed_dev(const void *d_data, uint64_t block_bytes, uint64_t n_blocks, uint32_t flags,
                        uint32_t *d_out, void *stream) {
    if (int r = ensure_ready()) return r;
    if (n_blocks == 0) return JL_OK;
    if (!d_data || !d_out) return fail(JL_ERR_INVALID, "jl_crc32c_fixed_dev: null pointer");
    if (block_bytes > 0xffffffffull) return fail(JL_ERR_INVALID, "jl_crc32c_fixed_dev: block_bytes >= 4 GiB");
    hipStream_t st = pick(stream);
    if (block_bytes == 4096 && ((uintptr_t)d_data & 15) == 0) {
        const int chains = opt().fixed_kernel;
        if (chains == 7) {  // the v4 product kernel (fixed_v4.hip): 8 lanes/block, 8-slot ring, 1024 threads
            JL_HIP(jlk::launch_fixed4k_v4(ctx().d_img_v4[1], (const uint8_t *)d_data, n_blocks, flags, d_out,
                                          grid_for(n_blocks), 8, 1, 3, st));
            return JL_OK;
        }
#if JL_STUDY
        // study kernels: 8 = v4 16 lanes/block; 10 = v4 16-slot ring without nt; 11, 12 = v4 (8 slots, 512
        // threads), (16 slots, 512 threads); 13 = v4 16-slot ring; 2..6, 101..104 = the r1 kernels
        if (chains == 8 || (chains >= 10 && chains <= 13)) {
            const int lpb = chains == 8 ? 16 : 8;
            const int shape = (chains == 11 || chains == 12) ? chains - 10 : 0;
            JL_HIP(jlk::launch_fixed4k_v4(ctx().d_img_v4[lpb == 8 ? 1 : 2], (const uint8_t *)d_data, n_blocks, flags,
                                          d_out, grid_for(n_blocks), lpb, chains != 10, shape, st));
            return JL_OK;
        }
        JL_HIP(jlk::launch_fixed4k(ctx().d_img, (const uint8_t *)d_data, ctx().d_zero, n_blocks, flags, d_out,
                                   ctx().d_scratch, grid_for(n_blocks), 1, 1, chains, st));
        return JL_OK;
#endif
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
    Context &c = ctx();
    std::lock_guard<std::mutex> lk(c.mu);
    hipPointerAttribute_t attr;
    bool pinned = hipPointerGetAttributes(&attr, host) == hipSuccess && attr.type == hipMemoryTypeHost;
    (void)hipGetLastError();  // pageable memory reports an error here; clear it
    const uint64_t per = JL_STREAM_CHUNK_BYTES / block_bytes;  // blocks per chunk
    const uint64_t chunk_bytes = per * block_bytes;
    for (auto &sl : c.slot) {
        if (!sl.st) JL_HIP(hipStreamCreateWithFlags(&sl.st, hipStreamNonBlocking));
        if (!sl.done) JL_HIP(hipEventCreateWithFlags(&sl.done, hipEventDisableTiming));
        JL_HIP(sl.d_in.ensure(chunk_bytes));
        JL_HIP(sl.d_out.ensure(per * 4));
        if (!pinned && sl.h_cap < chunk_bytes) {
            if (sl.h_stage) (void)hipHostFree(sl.h_stage);
            sl.h_stage = nullptr;
            sl.h_cap = 0;
            if (hipHostMalloc(&sl.h_stage, chunk_bytes, hipHostMallocDefault) != hipSuccess)
                return fail(JL_ERR_NOMEM, "jl_crc32c_fixed: pinned staging allocation failed");
            sl.h_cap = chunk_bytes;
        }
    }
    for (uint64_t b0 = 0, i = 0; b0 < n_blocks; b0 += per, i++) {
        Context::Slot &sl = c.slot[i & 1];
        const uint64_t nb = std::min(per, n_blocks - b0);
        const uint8_t *src = host + b0 * block_bytes;
        if (!pinned) {  // the slot's previous copy out of its staging buffer must be done
            JL_HIP(hipEventSynchronize(sl.done));
            memcpy(sl.h_stage, src, nb * block_bytes);
            src = (const uint8_t *)sl.h_stage;
        }
        JL_HIP(hipMemcpyAsync(sl.d_in.p, src, nb * block_bytes, hipMemcpyHostToDevice, sl.st));
        if (int r = jl_crc32c_fixed_dev(sl.d_in.p, block_bytes, nb, flags, (uint32_t *)sl.d_out.p, sl.st)) return r;
        JL_HIP(hipMemcpyAsync(out + b0, sl.d_out.p, nb * 4, hipMemcpyDeviceToHost, sl.st));
        JL_HIP(hipEventRecord(sl.done, sl.st));
    }
    JL_HIP(hipStreamSynchronize(c.slot[0].st));
    JL_HIP(hipStreamSynchronize(c.slot[1].st));
    return JL_OK;
}

int jl_crc32c_batch_dev(const void *d_base, uint64_t base_bytes, const uint64_t *d_off, const uint32_t *d_len,
                        const uint32_t *d_init, const uint8_t *d_suffix, uint64_t n, uint32_t flags, uint32_t *d_out,
                        void *stream) {
    if (int r = ensure_ready()) return r;
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
    for (uint64_t i = 0; i < n; i++)
        if (off[i] + (uint64_t)len[i] > base_bytes) return fail(JL_ERR_INVALID, "jl_crc32c_batch: block out of range");
    Context &c = ctx();
    std::lock_guard<std::mutex> lk(c.mu);
    hipStream_t st = c.stream;
    JL_HIP(c.ws_data.ensure(base_bytes + 16));
    JL_HIP(c.ws_off.ensure(n * 8));
    JL_HIP(c.ws_len.ensure(n * 4));
    JL_HIP(c.ws_out.ensure(n * 4));
    JL_HIP(hipMemcpyAsync(c.ws_data.p, base, base_bytes, hipMemcpyHostToDevice, st));
    JL_HIP(hipMemcpyAsync(c.ws_off.p, off, n * 8, hipMemcpyHostToDevice, st));
    JL_HIP(hipMemcpyAsync(c.ws_len.p, len, n * 4, hipMemcpyHostToDevice, st));
    jlk::KParams P = base_params(c.ws_data.p, n, jlk::MODE_CRC);
    P.off = (const uint64_t *)c.ws_off.p;
    P.len = (const uint32_t *)c.ws_len.p;
    if (init) {
        JL_HIP(c.ws_init.ensure(n * 4));
        JL_HIP(hipMemcpyAsync(c.ws_init.p, init, n * 4, hipMemcpyHostToDevice, st));
        P.init = (const uint32_t *)c.ws_init.p;
    }
    if (suffix) {
        JL_HIP(c.ws_sfx.ensure(n));
        JL_HIP(hipMemcpyAsync(c.ws_sfx.p, suffix, n, hipMemcpyHostToDevice, st));
        P.suffix = (const uint8_t *)c.ws_sfx.p;
    }
    P.flags = flags;
    P.out32 = (uint32_t *)c.ws_out.p;
    if (int r = run_general(P, st)) return r;
    JL_HIP(hipMemcpyAsync(out, c.ws_out.p, n * 4, hipMemcpyDeviceToHost, st));
    JL_HIP(hipStreamSynchronize(st));
    return JL_OK;
}

// ------------------------------------------------------------- table shims
int jl_table_trailers_dev(const void *d_file, const uint64_t *d_off, const uint32_t *d_size, const uint8_t *d_type,
                          uint64_t n, uint8_t *d_trailer, void *stream) {
    if (int r = ensure_ready()) return r;
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
    for (uint64_t i = 0; i < n; i++)
        if (off[i] + (uint64_t)size[i] + 5 > file_bytes)
            return fail(JL_ERR_INVALID, "jl_table_verify: truncated block read");  // TableFormat.java:203-206
    Context &c = ctx();
    std::lock_guard<std::mutex> lk(c.mu);
    hipStream_t st = c.stream;
    JL_HIP(c.ws_data.ensure(file_bytes + 16));
    JL_HIP(c.ws_off.ensure(n * 8));
    JL_HIP(c.ws_len.ensure(n * 4));
    JL_HIP(c.ws_ok.ensure(n));
    JL_HIP(hipMemcpyAsync(c.ws_data.p, file, file_bytes, hipMemcpyHostToDevice, st));
    JL_HIP(hipMemcpyAsync(c.ws_off.p, off, n * 8, hipMemcpyHostToDevice, st));
    JL_HIP(hipMemcpyAsync(c.ws_len.p, size, n * 4, hipMemcpyHostToDevice, st));
    jlk::KParams P = base_params(c.ws_data.p, n, jlk::MODE_TABLE_VERIFY);
    P.off = (const uint64_t *)c.ws_off.p;
    P.len = (const uint32_t *)c.ws_len.p;
    P.len_add = 1;
    P.out8 = (uint8_t *)c.ws_ok.p;
    if (int r = run_general(P, st)) return r;
    JL_HIP(hipMemcpyAsync(status, c.ws_ok.p, n, hipMemcpyDeviceToHost, st));
    JL_HIP(hipStreamSynchronize(st));
    return JL_OK;
}

// --------------------------------------------------------------- log shims
int jl_log_headers_dev(const void *d_base, const uint64_t *d_off, const uint32_t *d_len, const uint8_t *d_type,
                       uint64_t n, uint8_t *d_header, void *stream) {
    if (int r = ensure_ready()) return r;
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
    if (n_frags == 0 && log_bytes == 0) return JL_OK;
    if (!d_log || (n_frags && (!d_src || !d_frag_hdr_off || !d_frag_src_off || !d_frag_len || !d_frag_type)))
        return fail(JL_ERR_INVALID, "jl_log_emit_dev: null pointer");
    Context &c = ctx();
    std::lock_guard<std::mutex> lk(c.mu);  // ws_off holds the payload offsets
    hipStream_t st = pick(stream);
    JL_HIP(hipMemsetAsync(d_log, 0, log_bytes, st));  // block trailers (J/db/LogWriter.java:101-107)
    if (n_frags == 0) return JL_OK;
    JL_HIP(c.ws_off.ensure(n_frags * 8));
    uint64_t *pay = (uint64_t *)c.ws_off.p;
    JL_HIP(jlk::launch_log_copy((const uint8_t *)d_src, d_frag_src_off, d_frag_hdr_off, d_frag_len, n_frags, d_log,
                                pay, st));
    jlk::KParams P = base_params(d_log, n_frags, jlk::MODE_LOG_HEADER);
    P.off = pay;
    P.len = d_frag_len;
    P.type = d_frag_type;
    P.out8 = d_log;
    P.hdr_off = d_frag_hdr_off;
    if (int r = run_general(P, st)) return r;
    // the workspace is reused by the next call: finish before releasing the lock
    JL_HIP(hipStreamSynchronize(st));
    return JL_OK;
}

// Fused path (log_stream.hip): one streaming kernel walks and verifies every
// block, a scan of the per-block event counts places them, one compaction
// kernel writes them in file order; one synchronisation at the end.  Blocks
// with more than kLogStreamCap events (average record < 121 B) do not fit the
// per-block slots: *fallback is set and nothing is written.
constexpr uint32_t kLogStreamCap = 256;

static int log_verify_stream(const void *d_log, uint64_t log_bytes, jl_log_event *d_events, uint64_t cap,
                             uint64_t *n_events, hipStream_t st, bool *fallback) {
    Context &c = ctx();
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
    JL_HIP(jlk::launch_logstream(c.d_img_log, A, c.cus, st));
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

static int log_verify_impl(const void *d_log, uint64_t log_bytes, int checksum, jl_log_event *d_events, uint64_t cap,
                           uint64_t *n_events, hipStream_t st) {
    Context &c = ctx();
    if (checksum == JL_LOG_CHECKSUM_FUSED) {  // the single-pass kernel, unless a block overflows its slots
        bool fallback = false;
        *n_events = 0;
        if (log_bytes == 0) return JL_OK;
        if (int r = log_verify_stream(d_log, log_bytes, d_events, cap, n_events, st, &fallback)) return r;
        if (!fallback) return JL_OK;
    }
    const uint64_t nb = (log_bytes + 32767) / 32768;
    *n_events = 0;
    if (nb == 0) return JL_OK;
    JL_HIP(c.ws_cnt.ensure((nb + 1) * 8));  // cnt[nb] = 0: the exclusive scan's start[nb] is the total
    JL_HIP(c.ws_start.ensure((nb + 1) * 8));
    JL_HIP(c.ws_slot.ensure(nb * jlk::kLogSlots * sizeof(jlk::LogSlot)));
    uint64_t *cnt = (uint64_t *)c.ws_cnt.p, *start = (uint64_t *)c.ws_start.p;
    jlk::LogSlot *slots = (jlk::LogSlot *)c.ws_slot.p;
    JL_HIP(jlk::launch_log_walk((const uint8_t *)d_log, log_bytes, nb, 0, cnt, nullptr, nullptr, nullptr, nullptr, slots,
                                st));
    JL_HIP(hipMemsetAsync(cnt + nb, 0, 8, st));
    size_t tmp = 0;
    JL_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, tmp, cnt, start, (int)(nb + 1), st));
    JL_HIP(c.ws_tmp.ensure(tmp));
    JL_HIP(hipcub::DeviceScan::ExclusiveSum(c.ws_tmp.p, tmp, cnt, start, (int)(nb + 1), st));
    uint64_t total = 0;  // one copy back: the event count sizes the next buffers
    JL_HIP(hipMemcpyAsync(&total, start + nb, 8, hipMemcpyDeviceToHost, st));
    JL_HIP(hipStreamSynchronize(st));
    *n_events = total;
    if (total > cap) return fail(JL_ERR_CAPACITY, "jl_log_verify: event array too small");
    if (total == 0) return JL_OK;
    JL_HIP(c.ws_off.ensure(total * 8));
    JL_HIP(c.ws_len.ensure(total * 4));
    JL_HIP(c.ws_ok.ensure(total));
    JL_HIP(jlk::launch_log_walk((const uint8_t *)d_log, log_bytes, nb, 1, cnt, start, (jlk::LogEvent *)d_events,
                                (uint64_t *)c.ws_off.p, (uint32_t *)c.ws_len.p, slots, st));
    if (checksum) {
        jlk::KParams P = base_params(d_log, total, jlk::MODE_LOG_VERIFY);
        P.off = (const uint64_t *)c.ws_off.p;
        P.len = (const uint32_t *)c.ws_len.p;
        P.out8 = (uint8_t *)c.ws_ok.p;
        if (int r = run_general(P, st)) return r;
        // firstbad scratch: the walk's slot workspace is free again (n_blocks words fit in it)
        JL_HIP(jlk::launch_log_finalize(nb, start, cnt, (const uint8_t *)c.ws_ok.p, (jlk::LogEvent *)d_events, 1, total,
                                        (unsigned long long *)c.ws_slot.p, st));
    }
    JL_HIP(hipStreamSynchronize(st));
    return JL_OK;
}

int jl_log_verify_dev(const void *d_log, uint64_t log_bytes, int checksum, jl_log_event *d_events, uint64_t cap,
                      uint64_t *n_events, void *stream) {
    if (int r = ensure_ready()) return r;
    if (!n_events || (log_bytes && !d_log)) return fail(JL_ERR_INVALID, "jl_log_verify_dev: null pointer");
    if (checksum < 0 || checksum > JL_LOG_CHECKSUM_FUSED) return fail(JL_ERR_INVALID, "jl_log_verify_dev: bad checksum mode");
    Context &c = ctx();
    std::lock_guard<std::mutex> lk(c.mu);  // shares the walk workspace
    return log_verify_impl(d_log, log_bytes, checksum, d_events, cap, n_events, pick(stream));
}

int jl_log_verify(const uint8_t *log, uint64_t log_bytes, int checksum, jl_log_event *events, uint64_t cap,
                  uint64_t *n_events) {
    if (int r = ensure_ready()) return r;
    if (!n_events || (log_bytes && !log)) return fail(JL_ERR_INVALID, "jl_log_verify: null pointer");
    if (checksum < 0 || checksum > JL_LOG_CHECKSUM_FUSED) return fail(JL_ERR_INVALID, "jl_log_verify: bad checksum mode");
    Context &c = ctx();
    std::lock_guard<std::mutex> lk(c.mu);
    hipStream_t st = c.stream;
    *n_events = 0;
    if (log_bytes == 0) return JL_OK;
    JL_HIP(c.ws_data.ensure(log_bytes + 16));
    JL_HIP(hipMemcpyAsync(c.ws_data.p, log, log_bytes, hipMemcpyHostToDevice, st));
    // events land in ws_ev, then copy out
    const uint64_t ev_cap = log_bytes / 7 + 2;  // upper bound on physical records
    JL_HIP(c.ws_ev.ensure(ev_cap * sizeof(jl_log_event)));
    uint64_t total = 0;
    int r = log_verify_impl(c.ws_data.p, log_bytes, checksum, (jl_log_event *)c.ws_ev.p, ev_cap, &total, st);
    *n_events = total;
    if (r) return r;
    if (total > cap) return fail(JL_ERR_CAPACITY, "jl_log_verify: event array too small");
    if (total) {
        JL_HIP(hipMemcpyAsync(events, c.ws_ev.p, total * sizeof(jl_log_event), hipMemcpyDeviceToHost, st));
        JL_HIP(hipStreamSynchronize(st));
    }
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
