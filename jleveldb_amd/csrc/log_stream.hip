// log_stream.hip — fused WAL / MANIFEST verification: LogReader.readPhysicalRecord
// (J/db/LogReader.java:297-383) over every 32 KiB block of a log in ONE pass
// over its bytes (no walk kernel, no descriptor list, no sort).
//
// Layout.  The v4 lane layout of the 4 KiB kernel applied to 32 KiB log blocks:
// a wave owns a ROUND of 8 consecutive log blocks; group q (lanes 8q..8q+7)
// streams block q window by window (window k = bytes [128k, 128k + 128), lane l
// holding [16l, 16l + 16)) with one buffer_load_dwordx4 per lane and window, so
// every wave instruction reads 8 whole 128-B lines (narrower per-block shapes —
// 1, 2, 4 lanes per block — read at 0.8-3.1 TB/s on this chip,
// profiles/r2b_lane_probe.log).  Chain (l, j) takes dword j of lane l's chunk:
// the gap tables z^(124+t)∘T0 of the general v4 kernel.  The register ring (8
// pinned slots above the compiler's register budget, touched only by inline asm)
// runs across rounds.
//
// Records.  Each group walks its block's headers from the streamed bytes: the
// window holding a header (plus the first 16 B of the next window) is staged
// in LDS and the 7 header bytes are read from there.  A record's crc covers
// [h + 6, h + 7 + len) (type byte || payload, J/db/LogWriter.java:147).  Its
// chains start from 0 in the window of its header with the seed word
// W0 = slice4^-1(0xffffffff) in place of header bytes [h + 2, h + 6) (the
// value() init, fed as the 4 bytes before the record as in general_v4.hip) and
// everything before them masked out; they stop at the next header, where the
// bytes from there on are masked out of the finished record — kept in a
// PENDING slot — and start the next one.  All byte masks of one data dword come
// from one 16-B LDS entry indexed by the header's position relative to that
// dword (crc_math.hpp, kLSMaskDword).  The pending records of all 8 groups are
// folded together — one wave-wide pass of the general v4 epilogue with the tail
// pad d = window end - record end — when a group is about to close its next
// record, and at the end of the round.
//
// Decisions, in the reference's order (J/db/LogReader.java:315-369): fewer than
// 7 bytes left (EOF_TRUNC in the file's last, short block; else the block's
// trailer, no event), a length past the block (BAD_LENGTH; EOF_BAD_LENGTH in the
// short block), type 0 with length 0 (ZERO_SKIP) — each ends the block's walk —
// else a record whose crc is checked.  Each walked event goes to the block's
// slots as it is parsed (tentatively OK); the first record of the block whose
// masked crc differs from its stored one is kept per block, and
// logstream_compact_kernel turns it into BAD_CRC and drops the block's later
// events (the reader clears its 32 KiB buffer, :359-367).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "engine_device.hpp"

namespace jlk {

typedef uint32_t v2u __attribute__((ext_vector_type(2)));
typedef uint32_t v4u __attribute__((ext_vector_type(4)));
typedef int32_t v4i __attribute__((ext_vector_type(4)));

#ifndef JL_LS_WAVES
#define JL_LS_WAVES 12
#endif
#ifndef JL_LS_NOSTORE
#define JL_LS_NOSTORE 0  // study only: 1 skips the event stores (results wrong)
#endif
#ifndef JL_LS_NOFOLD
#define JL_LS_NOFOLD 0  // study only: 1 skips the folds (results wrong)
#endif
static_assert(JL_LS_WAVES * 1152 <= (40960 - 36384) * 4, "header staging must fit the LDS image");
constexpr uint32_t kLSThreads = JL_LS_WAVES * 64;  // one workgroup per CU (the LDS image is the whole LDS)
constexpr uint32_t kLSStageWave = 1152;         // 8 groups x 144 B: the window + the next one's first chunk
constexpr uint32_t kLSInf = 0x40000000u;    // header position of a group whose walk has ended

// The 8 ring slots (slot, register quad, its registers), pinned in the top 32
// VGPRs a wave of this shape may use (v136..v167 at 12 waves per CU: 168 per
// wave), above the ~110 the compiler allocates (tests/test_asm.py rejects any
// compiler instruction touching them): the allocator can then never place a
// value of its own in a slot whose load is in flight.  Slots are copied out
// right after their wait.  JL_LS_S<u> = slot u and slot u + 1 (the next
// window), JL_LS_R<u> = slot u
#if JL_LS_WAVES == 12
#define JL_LS_SLOTS(X) \
    X(0, "v[136:139]", "v136", "v137", "v138", "v139") \
    X(1, "v[140:143]", "v140", "v141", "v142", "v143") \
    X(2, "v[144:147]", "v144", "v145", "v146", "v147") \
    X(3, "v[148:151]", "v148", "v149", "v150", "v151") \
    X(4, "v[152:155]", "v152", "v153", "v154", "v155") \
    X(5, "v[156:159]", "v156", "v157", "v158", "v159") \
    X(6, "v[160:163]", "v160", "v161", "v162", "v163") \
    X(7, "v[164:167]", "v164", "v165", "v166", "v167")
#define JL_LS_S0 "v[136:139]", "v136", "v137", "v138", "v139", "v140", "v141", "v142", "v143"
#define JL_LS_R0 "v[136:139]", "v136", "v137", "v138", "v139"
#define JL_LS_S1 "v[140:143]", "v140", "v141", "v142", "v143", "v144", "v145", "v146", "v147"
#define JL_LS_R1 "v[140:143]", "v140", "v141", "v142", "v143"
#define JL_LS_S2 "v[144:147]", "v144", "v145", "v146", "v147", "v148", "v149", "v150", "v151"
#define JL_LS_R2 "v[144:147]", "v144", "v145", "v146", "v147"
#define JL_LS_S3 "v[148:151]", "v148", "v149", "v150", "v151", "v152", "v153", "v154", "v155"
#define JL_LS_R3 "v[148:151]", "v148", "v149", "v150", "v151"
#define JL_LS_S4 "v[152:155]", "v152", "v153", "v154", "v155", "v156", "v157", "v158", "v159"
#define JL_LS_R4 "v[152:155]", "v152", "v153", "v154", "v155"
#define JL_LS_S5 "v[156:159]", "v156", "v157", "v158", "v159", "v160", "v161", "v162", "v163"
#define JL_LS_R5 "v[156:159]", "v156", "v157", "v158", "v159"
#define JL_LS_S6 "v[160:163]", "v160", "v161", "v162", "v163", "v164", "v165", "v166", "v167"
#define JL_LS_R6 "v[160:163]", "v160", "v161", "v162", "v163"
#define JL_LS_S7 "v[164:167]", "v164", "v165", "v166", "v167", "v136", "v137", "v138", "v139"
#define JL_LS_R7 "v[164:167]", "v164", "v165", "v166", "v167"
#elif JL_LS_WAVES == 8
#define JL_LS_SLOTS(X) \
    X(0, "v[224:227]", "v224", "v225", "v226", "v227") \
    X(1, "v[228:231]", "v228", "v229", "v230", "v231") \
    X(2, "v[232:235]", "v232", "v233", "v234", "v235") \
    X(3, "v[236:239]", "v236", "v237", "v238", "v239") \
    X(4, "v[240:243]", "v240", "v241", "v242", "v243") \
    X(5, "v[244:247]", "v244", "v245", "v246", "v247") \
    X(6, "v[248:251]", "v248", "v249", "v250", "v251") \
    X(7, "v[252:255]", "v252", "v253", "v254", "v255")
#define JL_LS_S0 "v[224:227]", "v224", "v225", "v226", "v227", "v228", "v229", "v230", "v231"
#define JL_LS_R0 "v[224:227]", "v224", "v225", "v226", "v227"
#define JL_LS_S1 "v[228:231]", "v228", "v229", "v230", "v231", "v232", "v233", "v234", "v235"
#define JL_LS_R1 "v[228:231]", "v228", "v229", "v230", "v231"
#define JL_LS_S2 "v[232:235]", "v232", "v233", "v234", "v235", "v236", "v237", "v238", "v239"
#define JL_LS_R2 "v[232:235]", "v232", "v233", "v234", "v235"
#define JL_LS_S3 "v[236:239]", "v236", "v237", "v238", "v239", "v240", "v241", "v242", "v243"
#define JL_LS_R3 "v[236:239]", "v236", "v237", "v238", "v239"
#define JL_LS_S4 "v[240:243]", "v240", "v241", "v242", "v243", "v244", "v245", "v246", "v247"
#define JL_LS_R4 "v[240:243]", "v240", "v241", "v242", "v243"
#define JL_LS_S5 "v[244:247]", "v244", "v245", "v246", "v247", "v248", "v249", "v250", "v251"
#define JL_LS_R5 "v[244:247]", "v244", "v245", "v246", "v247"
#define JL_LS_S6 "v[248:251]", "v248", "v249", "v250", "v251", "v252", "v253", "v254", "v255"
#define JL_LS_R6 "v[248:251]", "v248", "v249", "v250", "v251"
#define JL_LS_S7 "v[252:255]", "v252", "v253", "v254", "v255", "v224", "v225", "v226", "v227"
#define JL_LS_R7 "v[252:255]", "v252", "v253", "v254", "v255"
#else
#error "JL_LS_WAVES: 8 or 12"
#endif

// raw buffer resource over one round (8 blocks = 256 KiB); chunks past the log
// (and every byte of a round past the last one) read as zeros.  The range is
// rounded up to whole 16-B chunks: the range check drops a dwordx4 that
// crosses num_records, which would zero the log's last bytes.  The up to 15
// bytes read past the log stay in its last page; they are masked out of every
// record (bytes past a record's end) and never parsed (fewer than 7 bytes left).
__device__ __forceinline__ v4i ls_rsrc(const LogStreamArgs &A, uint32_t round, uint32_t rounds) {
    const uint64_t base = (uint64_t)round * 262144u;
    uint32_t n = 0;
    if (round < rounds) n = (uint32_t)(A.size - base < 262144u ? (A.size - base + 15u) & ~15ull : 262144u);
    const uint64_t a = (uint64_t)(uintptr_t)A.log + (round < rounds ? base : 0u);
    v4i r;
    r.x = (int32_t)(uint32_t)a;
    r.y = (int32_t)((uint32_t)(a >> 32) & 0xffffu);
    r.z = (int32_t)n;
    r.w = 0x00020000;
    return r;
}

// z^-(16 col) of lane column col (0..15) as 8 nibble lookups (kLSLaneByte:
// dword (p*16 + v)*16 + col)
__device__ __forceinline__ uint32_t ls_realign(const uint32_t *lds, uint32_t r, uint32_t col) {
    const uint32_t lc = kLSLaneByte | (col << 2);
    uint32_t c[8];
#pragma unroll
    for (int p = 0; p < 8; p++) c[p] = lds_at(lds, lc + 1024u * p + (((r >> (4 * p)) & 15u) << 6));
    return xor3(xor3(c[0], c[1], c[2]), xor3(c[3], c[4], c[5]), c[6] ^ c[7]);
}

// the mask entry of dword j for a header at byte rr of this lane's chunk:
// entry (clamp(rr, -10, 16) + 22 - 4j) of kLSMaskDword (crc_math.hpp)
__device__ __forceinline__ const v4u *ls_masks(const uint32_t *lds, int rr) {
    const int c = rr < -10 ? -10 : (rr > 16 ? 16 : rr);
    return (const v4u *)((const char *)lds + kLSMaskByte) + (c + 10);  // + (12 - 4j) per dword
}

__global__ __launch_bounds__(kLSThreads) void crc_logstream_kernel(
    const uint4 *__restrict__ img, LogStreamArgs A) {
    __shared__ uint32_t lds[kImageBytes / 4];
    load_image(lds, img);
    const uint32_t lane = threadIdx.x & 63u, q = lane >> 3, l = lane & 7u, wave = threadIdx.x >> 6;
    const uint32_t waves = gridDim.x * (kLSThreads / 64u);
    const uint32_t R = (A.n_blocks + 7u) / 8u;
    uint32_t r = uni(blockIdx.x * (kLSThreads / 64u) + wave);
    if (r >= R) return;
    const GLanes gl(lane);
    const uint32_t lane_off = q * 32768u + l * 16u;
    char *const lb = (char *)lds;
    const uint32_t stage = kLSStageByte + wave * kLSStageWave + q * 144u;

    // ---- group state (uniform in a group, one copy per lane)
    uint32_t b, blen, h, hs, cnt, fb, cst, cidx;
    bool eof, has_cur, spill;
    // pending (closed, not yet folded) record
    uint32_t p0 = 0, p1 = 0, p2 = 0, p3 = 0, pd = 0, pst = 0, pidx = 0;
    bool pend = false;
    uint32_t x0, x1, x2, x3;  // chains (x-form: state ^ this window's data word)
    auto setup = [&](uint32_t rr) {
        b = rr * 8u + q;
        const bool valid = b < A.n_blocks;
        const uint64_t bb = (uint64_t)b * 32768u;
        blen = valid ? (uint32_t)(A.size - bb < 32768u ? A.size - bb : 32768u) : 0u;
        eof = blen < 32768u;
        h = valid ? 0u : kLSInf;
        hs = 0;
        has_cur = spill = false;
        cnt = 0;
        fb = kLSNone;
        cst = cidx = 0;
        x0 = x1 = x2 = x3 = 0;
    };
    setup(r);

    // Fold every group's pending record (wave-wide; general_v4.hip's epilogue:
    // chain (l, j) ends 16 l + 4 j + d past the record's end, d = the tail pad)
    auto fold = [&]() {
        const uint32_t s0 = gstep_x3(lds, p0, gl, 0u), s1 = gstep_x3(lds, p1, gl, 0u);
        const uint32_t s2 = gstep_x3(lds, p2, gl, 0u), s3 = gstep_x3(lds, p3, gl, 0u);
        const uint32_t d = pd, sa = 512u * ((d >> 2) & 3u);
        const uint32_t c = xor3(ushift(lds, s0, kLSShiftByte + sa), ushift(lds, s1, kLSShiftByte + 512u + sa),
                                ushift(lds, s2, kLSShiftByte + 1024u + sa)) ^
                           ushift(lds, s3, kLSShiftByte + 1536u + sa);
        uint32_t st = group_xor<8>(ls_realign(lds, c, (l + (d >> 4)) & 15u));
        st = ushift(lds, st, kLSEByte + 512u * (d & 3u));
        if (pend && mask_crc(~st) != pst && fb == kLSNone) fb = pidx;
        pend = false;
    };

    // ---- the ring: windows k .. k+7 of this round (and the next) in flight
    v4i rs_cur = ls_rsrc(A, r, R), rs_nxt = ls_rsrc(A, r + waves, R);
#define JL_LS_LD(RQ, R0, R1, R2, R3, RS, K)                                                                   \
    {                                                                                                         \
        const uint32_t vo_ = lane_off + ((uint32_t)(K) << 7);                                                 \
        asm volatile("buffer_load_dwordx4 " RQ ", %0, %1, 0 offen nt" ::"v"(vo_), "s"(RS) : "memory", R0, R1, \
                     R2, R3);                                                                                 \
    }
#define JL_LS_CP(R0, R1, R2, R3, A0, A1, A2, A3)                                                              \
    asm volatile("v_mov_b32 %0, " R0 "\n\tv_mov_b32 %1, " R1 "\n\tv_mov_b32 %2, " R2 "\n\tv_mov_b32 %3, " R3 \
                 : "=v"(A0), "=v"(A1), "=v"(A2), "=v"(A3))
#define JL_LS_PRIME(u, RQ, R0, R1, R2, R3) JL_LS_LD(RQ, R0, R1, R2, R3, rs_cur, u)
    JL_LS_SLOTS(JL_LS_PRIME)
#undef JL_LS_PRIME

    uint32_t kt = 0;   // first window of the current turn (8 windows, one per slot)
    int bu = 0;        // slot of the step that took the boundary path
    uint32_t w0, w1, w2, w3, n0, n1, n2, n3;  // this window's words, the next window's (boundary steps)
    uint32_t t0, t1, t2, t3, u0, u1, u2, u3;  // the chains' lookups of this step
    int resume = -1;
    // One step per slot, unrolled over the 8 slots of a turn.  A step whose
    // window holds a header of some group jumps to the shared boundary code
    // (after copying the next window's words) and resumes at its slot's refill.
#define JL_LK(x, T, U)                                                                                     \
    T = xor3(lds_at(lds, JL_GADDR(gl.l3, x, 0u)), lds_at(lds, JL_GADDR(gl.l2, x, 1u)),                     \
             lds_at(lds, JL_GADDR(gl.l1, x, 2u)));                                                         \
    U = lds_at(lds, JL_GADDR(gl.l0, x, 3u));
#define JL_LS_STEP(u, RQ, R0, R1, R2, R3, N0, N1, N2, N3)                                                  \
    {                                                                                                      \
        /* windows k and k + 1 have landed (7 younger loads issued; loads return in order) */             \
        asm volatile("s_waitcnt vmcnt(6)" ::: "memory");                                                 \
        JL_LS_CP(R0, R1, R2, R3, w0, w1, w2, w3);                                                          \
        JL_LK(x0, t0, u0) JL_LK(x1, t1, u1) JL_LK(x2, t2, u2) JL_LK(x3, t3, u3)                             \
        if (__builtin_amdgcn_ballot_w64(h <= (kt + (u)) * 128u + 128u || spill) != 0) {                   \
            JL_LS_CP(N0, N1, N2, N3, n0, n1, n2, n3);                                                      \
            bu = (u);                                                                                      \
            goto boundary;                                                                                 \
        }                                                                                                  \
        x0 = xor3(t0, u0, w0);                                                                             \
        x1 = xor3(t1, u1, w1);                                                                             \
        x2 = xor3(t2, u2, w2);                                                                             \
        x3 = xor3(t3, u3, w3);                                                                             \
    }
#define JL_LS_CALL(M, ...) M(__VA_ARGS__)
#define JL_LS_REFILL(u, RQ, R0, R1, R2, R3)                                                                \
    if (kt + 8u + (u) < 256u) JL_LS_LD(RQ, R0, R1, R2, R3, rs_cur, kt + 8u + (u))                         \
    else JL_LS_LD(RQ, R0, R1, R2, R3, rs_nxt, kt + (u) - 248u)
    for (;;) {
        switch (resume) {
        case -1:
            JL_LS_CALL(JL_LS_STEP, 0, JL_LS_S0)
            [[fallthrough]];
        case 0:
            JL_LS_CALL(JL_LS_REFILL, 0, JL_LS_R0)
            JL_LS_CALL(JL_LS_STEP, 1, JL_LS_S1)
            [[fallthrough]];
        case 1:
            JL_LS_CALL(JL_LS_REFILL, 1, JL_LS_R1)
            JL_LS_CALL(JL_LS_STEP, 2, JL_LS_S2)
            [[fallthrough]];
        case 2:
            JL_LS_CALL(JL_LS_REFILL, 2, JL_LS_R2)
            JL_LS_CALL(JL_LS_STEP, 3, JL_LS_S3)
            [[fallthrough]];
        case 3:
            JL_LS_CALL(JL_LS_REFILL, 3, JL_LS_R3)
            JL_LS_CALL(JL_LS_STEP, 4, JL_LS_S4)
            [[fallthrough]];
        case 4:
            JL_LS_CALL(JL_LS_REFILL, 4, JL_LS_R4)
            JL_LS_CALL(JL_LS_STEP, 5, JL_LS_S5)
            [[fallthrough]];
        case 5:
            JL_LS_CALL(JL_LS_REFILL, 5, JL_LS_R5)
            JL_LS_CALL(JL_LS_STEP, 6, JL_LS_S6)
            [[fallthrough]];
        case 6:
            JL_LS_CALL(JL_LS_REFILL, 6, JL_LS_R6)
            JL_LS_CALL(JL_LS_STEP, 7, JL_LS_S7)
            [[fallthrough]];
        case 7:
            JL_LS_CALL(JL_LS_REFILL, 7, JL_LS_R7)
            break;
        default:
            break;
        }
        resume = -1;
        kt += 8u;
        if (kt == 256u) {  // ---- end of the round: every record of its blocks has closed
            if (__builtin_amdgcn_ballot_w64(pend) != 0) fold();
            if (l == 0u && b < A.n_blocks) {
                A.count[b] = cnt;
                A.first_bad[b] = fb;
                if (cnt > A.cap) atomicOr(A.overflow, 1u);
            }
            r = uni(r + waves);
            if (r >= R) break;
            rs_cur = rs_nxt;
            rs_nxt = ls_rsrc(A, r + waves, R);
            setup(r);
            kt = 0;
        }
        continue;

    boundary: {
        // ---- a header (or the tail of one) lies in window k = kt + bu for some
        // group.  Branch-light: every lane runs every iteration and keeps or
        // drops its results by selects; only the loop, the fold and the event
        // store branch.
        const uint32_t W = (kt + (uint32_t)bu) * 128u;
        // stage the group's window and the next window's first chunk
        *(v4u *)(lb + stage + 16u * l) = v4u{w0, w1, w2, w3};
        if (l == 0u) *(v4u *)(lb + stage + 128u) = v4u{n0, n1, n2, n3};
        uint32_t c0 = t0 ^ u0, c1 = t1 ^ u1, c2 = t2 ^ u2, c3 = t3 ^ u3;  // the chains' carry
        uint32_t v0 = w0, v1 = w1, v2 = w2, v3 = w3;                        // this window's words
        if (__builtin_amdgcn_ballot_w64(spill) != 0) {
            // the current record's header ended in the previous window: mask its tail here
            const v4u *m = ls_masks(lds, spill ? (int)hs - (int)W - (int)(16u * l) : -10);
            const v4u m0 = m[12], m1 = m[8], m2 = m[4], m3 = m[0];
            v0 = __builtin_amdgcn_bitop3_b32(w0, m0.y, m0.z, 0xEA);  // (w & nm) | sd (all-pass at -10)
            v1 = __builtin_amdgcn_bitop3_b32(w1, m1.y, m1.z, 0xEA);
            v2 = __builtin_amdgcn_bitop3_b32(w2, m2.y, m2.z, 0xEA);
            v3 = __builtin_amdgcn_bitop3_b32(w3, m3.y, m3.z, 0xEA);
            spill = false;
        }
        for (;;) {
            const bool ev = h <= W + 128u;
            if (__builtin_amdgcn_ballot_w64(ev) == 0) break;
            // a group about to close a record while it still holds one: fold them all first
            if (!JL_LS_NOFOLD && __builtin_amdgcn_ballot_w64(ev && has_cur && pend) != 0) fold();
            const uint32_t o = ev ? h - W : 0u;  // 0..128
            const v4u *m = ls_masks(lds, (int)o - (int)(16u * l));
            const v4u m0 = m[12], m1 = m[8], m2 = m[4], m3 = m[0];
            // header bytes [o, o + 8) from the staging: aligned reads, then a byte shift
            const uint32_t a = stage + (o & ~7u);
            const v2u lo = *(const v2u *)(lb + a), hi = *(const v2u *)(lb + a + 8u);
            // close the current record at h: keep its bytes < h
            const bool close = ev && has_cur;
            p0 = close ? __builtin_amdgcn_bitop3_b32(c0, v0, m0.x, 0x78) : p0;  // c ^ (v & om)
            p1 = close ? __builtin_amdgcn_bitop3_b32(c1, v1, m1.x, 0x78) : p1;
            p2 = close ? __builtin_amdgcn_bitop3_b32(c2, v2, m2.x, 0x78) : p2;
            p3 = close ? __builtin_amdgcn_bitop3_b32(c3, v3, m3.x, 0x78) : p3;
            pd = close ? W + 128u - h : pd;
            pst = close ? cst : pst;
            pidx = close ? cidx : pidx;
            pend = pend || close;
            // the header's decision (J/db/LogReader.java:315-353)
            const bool up = (o & 4u) != 0u;
            const uint32_t e0 = up ? lo.y : lo.x, e1 = up ? hi.x : lo.y, e2 = up ? hi.y : hi.x;
            const uint32_t H0 = __builtin_amdgcn_alignbyte(e1, e0, o & 3u);
            const uint32_t H1 = __builtin_amdgcn_alignbyte(e2, e1, o & 3u);
            const uint32_t rem = blen - h;
            const bool tiny = rem < 7u;
            const uint32_t len = tiny ? 0u : H1 & 0xffffu, type = tiny ? 0u : (H1 >> 16) & 0xffu;
            uint32_t kind = 1u;
            if (tiny) kind = (eof && rem > 0u) ? 6u : 0u;  // :315-322
            else if (7u + len > rem) kind = eof ? 5u : 3u;  // :334-345
            else if (type == 0u && len == 0u) kind = 4u;  // :347-353
            const bool emit = ev && kind != 0u;
            if (!JL_LS_NOSTORE && emit && l == 0u && cnt < A.cap) {
                const uint64_t off = (uint64_t)b * 32768u + h;
                *(v4u *)(A.slots + (uint64_t)b * A.cap + cnt) =
                    v4u{(uint32_t)off, (uint32_t)(off >> 32), len, type | (kind << 8)};
            }
            cidx = emit ? cnt : cidx;
            cst = emit ? H0 : cst;
            cnt += emit ? 1u : 0u;
            // a record: its chains start here, from 0, with the seed in its header
            const bool start = ev && kind == 1u;
            v0 = start ? __builtin_amdgcn_bitop3_b32(w0, m0.y, m0.z, 0xEA) : v0;  // (w & nm) | sd
            v1 = start ? __builtin_amdgcn_bitop3_b32(w1, m1.y, m1.z, 0xEA) : v1;
            v2 = start ? __builtin_amdgcn_bitop3_b32(w2, m2.y, m2.z, 0xEA) : v2;
            v3 = start ? __builtin_amdgcn_bitop3_b32(w3, m3.y, m3.z, 0xEA) : v3;
            c0 = start ? 0u : c0;
            c1 = start ? 0u : c1;
            c2 = start ? 0u : c2;
            c3 = start ? 0u : c3;
            hs = start ? h : hs;
            spill = start ? h + 6u > W + 128u : spill;
            has_cur = start || (has_cur && !ev);
            h = ev ? (start ? h + 7u + len : kLSInf) : h;  // anything else ends the block's walk
        }
        x0 = c0 ^ v0;
        x1 = c1 ^ v1;
        x2 = c2 ^ v2;
        x3 = c3 ^ v3;
        resume = bu;
    }
    }
#undef JL_LS_STEP
#undef JL_LS_REFILL
#undef JL_LS_CALL
#undef JL_LK
#undef JL_LS_LD
#undef JL_LS_CP
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the ring's trailing loads (past the last round)
}

// One wave per block: copies its walked events to their place in file order,
// applying the block's first crc failure (BAD_CRC, later events kind 0).
__global__ __launch_bounds__(256) void logstream_compact_kernel(LogStreamArgs A, const uint64_t *__restrict__ start,
                                                                LogEvent *__restrict__ ev, uint64_t cap_out) {
    const uint32_t b = blockIdx.x * 4u + (threadIdx.x >> 6), lane = threadIdx.x & 63u;
    if (b >= A.n_blocks) return;
    const uint32_t n = A.count[b] < A.cap ? A.count[b] : A.cap, fb = A.first_bad[b];
    const uint64_t s = start[b];
    for (uint32_t j = lane; j < n && s + j < cap_out; j += 64u) {
        LogEvent e = A.slots[(uint64_t)b * A.cap + j];
        if (fb != kLSNone && j >= fb) e.kind = j == fb ? 2u : 0u;
        ev[s + j] = e;
    }
}

hipError_t launch_logstream(const void *img, const LogStreamArgs &A, int grid, hipStream_t st) {
    hipLaunchKernelGGL(crc_logstream_kernel, dim3(grid), dim3(kLSThreads), 0, st, (const uint4 *)img, A);
    return hipGetLastError();
}

hipError_t launch_logstream_compact(const LogStreamArgs &A, const uint64_t *start, LogEvent *ev, uint64_t cap_out,
                                    hipStream_t st) {
    if (A.n_blocks == 0) return hipSuccess;
    hipLaunchKernelGGL(logstream_compact_kernel, dim3((A.n_blocks + 3u) / 4u), dim3(256), 0, st, A, start, ev, cap_out);
    return hipGetLastError();
}

}  // namespace jlk
