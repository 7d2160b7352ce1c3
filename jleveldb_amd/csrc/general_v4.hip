// general_v4.hip — general-path engine on the v4 lane layout (variable block
// lengths and alignment, per-block init/suffix, table/log verify epilogues).
// Compiled once per mode (-DJL_MODE=k, Makefile); the mode-independent helper
// kernels (rounds pipeline, split-block combine) live in the JL_MODE == 0 object.
//
// Work unit: a ROUND of up to 8 blocks with the same step count K, processed by
// one wave exactly as the 4 KiB kernel (fixed_v4.hip) processes 8 blocks: 8
// lanes per block, block-step 128 B, one 16-byte load per lane and step, 4
// chains per lane through the gap tables z^(124+t)∘T0, the same epilogue.
//
// A block [p, p+n) is viewed on the 128-B-ALIGNED grid of its memory: step k
// is the window [A + 128k, +128), A = p & ~127, K = ceil((f + n)/128) windows
// with a front pad of f = p - A bytes and a tail pad of d = 128K - f - n.
// Every ring load is then one aligned 16-B chunk and a group's step one whole
// 128-B line (unaligned dwordx4 loads that straddle lines made the texture
// addresser the bottleneck, r1 PMC: TA busy ~100 %).  A window that holds a
// byte of the block never leaves the block's pages, so no load can fault.
// Pad bytes are masked to zero in the first / last step; zeros in front are
// free, the d zeros behind advance the state by z^d, which the epilogue undoes
// inside shifts it does anyway (d = 16a + 4c + e: chain tables z^-4(j+c), lane
// column l+a, one z^-e).  Rounds only hold blocks of one K (a counting sort by
// K, the rounds pipeline at the end of this file, cuts every bin into rounds
// of 8; 128-B aligned fixed-stride batches need none).  Blocks above 512 KiB
// (crc mode) run as chunks folded per block afterwards (gv4_combine_kernel).
//
// Seeding needs no state shift (as in the stream kernel): W = slice4^-1(~init)
// is fed as the 4 data bytes just before the block, i.e. at virtual bytes
// [f-4, f); when f < 4 its low bytes fall in virtual dword -4, the chain
// (lane 7, dword 3) of step -1, which then starts from gstep(W << 8f).
//
// Entries of a round in the register ring (one wave-wide load each):
//   [side]  verify / init / suffix modes: lane 0 / 1 of each group load the
//           aligned 16-B chunks holding the first / last byte of the stored crc
//           (or holding init[i] / the suffix byte); other lanes load the zero page
//   K       steps 0..K-1 (0 and K-1 mask their pads)
// The ring (P = 8 entries, s_waitcnt vmcnt(P-2) before each use, refill right
// after) runs across rounds, so the HBM stream never drains.  Round
// descriptors are prefetched by vector loads into pinned registers (long
// rounds) or read with scalar loads (lgkmcnt, never the hand-counted vmcnt).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "engine_device.hpp"

#ifndef JL_MODE
#error "compile with -DJL_MODE=<jlk::MODE_*>"
#endif
#ifndef JL_GV4_THREADS
#define JL_GV4_THREADS 1024  // 16 waves per CU: 128 VGPRs per lane, 40 of them pinned
#endif

namespace jlk {

typedef uint32_t v4u __attribute__((ext_vector_type(4)));

// The gv4 image is the general v4 image ROTATED (crc_math.hpp
// build_lds_image_gv4): region B (epilogue tables) at byte 0, the G tables at
// kGOff.  Every region-B table base is then below 64 KiB and folds into the
// ds_read immediate offset (an epilogue nibble lookup costs 2 VALU instead of
// 3), and the G lookups reach their tables through the immediate kGOff.
constexpr uint32_t kGOff = 32768, kRB = 131072;  // G tables; region B of the unrotated image
constexpr uint32_t kLaneB = 0, kShiftB = kG4ShiftByte - kRB, kEB = kG4EByte - kRB, kUB = kG4UByte - kRB,
                   kT0B = kG4T0Byte - kRB, kSelB = kG4SelByte - kRB;
// MODE_LOG_CHUNK's image (crc_math.hpp build_lds_image_logchunk): chain tables
// z^-(4 (j + c) + e) and the byte selectors after the lane tables
constexpr uint32_t kLCMB = 16384, kLCSelB = 30720;

// The pinned registers: two round-descriptor sets (JL_GV4_DQ0/1) and the 8
// ring slots (slot, register quad, its 4 registers), the top 40 VGPRs a wave of
// this shape may use: v88..v127 at 16 waves per CU (1024 threads, 128 VGPRs),
// v216..v255 at 8 waves (512 threads).  The compiler allocates about 65 VGPRs
// below them; tests/test_asm.py rejects any compiler instruction touching them.
#if JL_GV4_THREADS == 1024
#define JL_GV4_PIN_FIRST 88
#define JL_GV4_SLOTS(X) \
    X(0, "v[96:99]", "v96", "v97", "v98", "v99") \
    X(1, "v[100:103]", "v100", "v101", "v102", "v103") \
    X(2, "v[104:107]", "v104", "v105", "v106", "v107") \
    X(3, "v[108:111]", "v108", "v109", "v110", "v111") \
    X(4, "v[112:115]", "v112", "v113", "v114", "v115") \
    X(5, "v[116:119]", "v116", "v117", "v118", "v119") \
    X(6, "v[120:123]", "v120", "v121", "v122", "v123") \
    X(7, "v[124:127]", "v124", "v125", "v126", "v127")
#define JL_GV4_SLOTS_LO(X) \
    X(0, "v[96:99]", "v96", "v97", "v98", "v99") \
    X(1, "v[100:103]", "v100", "v101", "v102", "v103") \
    X(2, "v[104:107]", "v104", "v105", "v106", "v107") \
    X(3, "v[108:111]", "v108", "v109", "v110", "v111")
#define JL_GV4_SLOTS_HI(X) \
    X(4, "v[112:115]", "v112", "v113", "v114", "v115") \
    X(5, "v[116:119]", "v116", "v117", "v118", "v119") \
    X(6, "v[120:123]", "v120", "v121", "v122", "v123") \
    X(7, "v[124:127]", "v124", "v125", "v126", "v127")
#define JL_GV4_DQ0 "v[88:91]"
#define JL_GV4_DR0 "v88", "v89", "v90", "v91"
#define JL_GV4_DMOV0 "v_mov_b32 %0, v88\n\tv_mov_b32 %1, v89\n\tv_mov_b32 %2, v90\n\tv_mov_b32 %3, v91"
#define JL_GV4_DQ1 "v[92:95]"
#define JL_GV4_DR1 "v92", "v93", "v94", "v95"
#define JL_GV4_DMOV1 "v_mov_b32 %0, v92\n\tv_mov_b32 %1, v93\n\tv_mov_b32 %2, v94\n\tv_mov_b32 %3, v95"
#elif JL_GV4_THREADS == 512
#define JL_GV4_PIN_FIRST 216
#define JL_GV4_SLOTS(X) \
    X(0, "v[224:227]", "v224", "v225", "v226", "v227") \
    X(1, "v[228:231]", "v228", "v229", "v230", "v231") \
    X(2, "v[232:235]", "v232", "v233", "v234", "v235") \
    X(3, "v[236:239]", "v236", "v237", "v238", "v239") \
    X(4, "v[240:243]", "v240", "v241", "v242", "v243") \
    X(5, "v[244:247]", "v244", "v245", "v246", "v247") \
    X(6, "v[248:251]", "v248", "v249", "v250", "v251") \
    X(7, "v[252:255]", "v252", "v253", "v254", "v255")
#define JL_GV4_SLOTS_LO(X) \
    X(0, "v[224:227]", "v224", "v225", "v226", "v227") \
    X(1, "v[228:231]", "v228", "v229", "v230", "v231") \
    X(2, "v[232:235]", "v232", "v233", "v234", "v235") \
    X(3, "v[236:239]", "v236", "v237", "v238", "v239")
#define JL_GV4_SLOTS_HI(X) \
    X(4, "v[240:243]", "v240", "v241", "v242", "v243") \
    X(5, "v[244:247]", "v244", "v245", "v246", "v247") \
    X(6, "v[248:251]", "v248", "v249", "v250", "v251") \
    X(7, "v[252:255]", "v252", "v253", "v254", "v255")
#define JL_GV4_DQ0 "v[216:219]"
#define JL_GV4_DR0 "v216", "v217", "v218", "v219"
#define JL_GV4_DMOV0 "v_mov_b32 %0, v216\n\tv_mov_b32 %1, v217\n\tv_mov_b32 %2, v218\n\tv_mov_b32 %3, v219"
#define JL_GV4_DQ1 "v[220:223]"
#define JL_GV4_DR1 "v220", "v221", "v222", "v223"
#define JL_GV4_DMOV1 "v_mov_b32 %0, v220\n\tv_mov_b32 %1, v221\n\tv_mov_b32 %2, v222\n\tv_mov_b32 %3, v223"
#else
#error "JL_GV4_THREADS: 512 or 1024"
#endif
#define JL_GV4_RING 8
// A ring use waits vmcnt(P - JL_RING_SLACK).  s_waitcnt vmcnt(N) leaves the N
// youngest vector-memory operations of any kind in flight, in issue order, so
// P - 1 would be exact for gv4; r3 same-box A/B with slack 1 (7 loads in flight
// instead of 6): C3 2.055 / 2.065 vs 2.059 / 2.06 ms, C5 1 056-B and mixed
// unchanged, so 2 stays (the 4 KiB kernel's ring also fails the dataflow check
// of tools/asm_ring_check.py at slack 1: a compiler copy of a slot sits before
// the wait that would then cover it).
#ifndef JL_RING_SLACK
#define JL_RING_SLACK 2
#endif

// (The per-wave start / end timing study of r4, JL_GV4_WAVETIME with
// tools/gv4_wavetime.py, and the bound-study variants of this kernel live on the
// branch study-r5-gv4-switches.)

template <int MODE>
struct GV4 {
    static constexpr bool VERIFY = MODE == MODE_TABLE_VERIFY || MODE == MODE_LOG_VERIFY;
    static constexpr bool LOGC = MODE == MODE_LOG_CHUNK;  // stored crc in the descriptor: no side entry
    // a side entry (stored crc / init / suffix chunk) heads every round; never in MODE_LOG_CHUNK
    __device__ static bool side(const GV4Args &A) { return !LOGC && (VERIFY || A.P.init || A.P.suffix); }
};

// Per-lane view of a round's descriptor (group q = lane >> 3).
struct RoundView {
    uint64_t p;    // per lane: the group's first byte
    uint32_t d;    // per lane: tail pad
    uint32_t idx;  // per lane (kGNull: no result)
    uint32_t K;    // wave-uniform
    uint32_t stored, seed;  // MODE_LOG_CHUNK: per lane, the group's stored crc and seed flag
    uint32_t f;             // MODE_LOG_CHUNK: p & 127 (p itself is dead in the round loop; a
                            // failure re-reads it from the descriptor)
};

__device__ __forceinline__ uint32_t sel8(uint32_t q, uint32_t a0, uint32_t a1, uint32_t a2, uint32_t a3, uint32_t a4,
                                         uint32_t a5, uint32_t a6, uint32_t a7) {
    const uint32_t lo = q & 4u ? (q & 2u ? (q & 1u ? a7 : a6) : (q & 1u ? a5 : a4))
                               : (q & 2u ? (q & 1u ? a3 : a2) : (q & 1u ? a1 : a0));
    return lo;
}

template <int MODE>
__device__ __forceinline__ RoundView round_view(const GV4Args &A, uint32_t r, uint32_t q) {
    RoundView v;
    v.stored = 0;
    v.f = 0;
    v.seed = 0;
    if (A.desc) {
        // the round's 8 descriptors (128 B) with two scalar loads: SMEM/lgkmcnt, so the
        // hand-counted vmcnt ring never sees them (a compiler-emitted vector load here
        // would be waited for with vmcnt and drain the ring).  Outputs are early-clobber:
        // the first load's destination must not overlap the address the second one
        // reads (r1: s[16:31] <- [s[16:17]] then [s[16:17] + 64] read a returned
        // descriptor word as the address when the wave was descheduled in between)
        typedef uint32_t v16u __attribute__((ext_vector_type(16)));
        const uint64_t ga = uni64((uint64_t)(uintptr_t)(A.desc + (uint64_t)r * 8u));
        v16u d0, d1;
        asm volatile("s_load_dwordx16 %0, %2, 0x0\n\ts_load_dwordx16 %1, %2, 0x40\n\ts_waitcnt lgkmcnt(0)"
                     : "=&s"(d0), "=&s"(d1) : "s"(ga) : "memory");
        const uint32_t w[32] = {d0[0],  d0[1],  d0[2],  d0[3],  d0[4],  d0[5],  d0[6],  d0[7],
                                d0[8],  d0[9],  d0[10], d0[11], d0[12], d0[13], d0[14], d0[15],
                                d1[0],  d1[1],  d1[2],  d1[3],  d1[4],  d1[5],  d1[6],  d1[7],
                                d1[8],  d1[9],  d1[10], d1[11], d1[12], d1[13], d1[14], d1[15]};
        uint32_t vl[8], vh[8], ix[8];
#pragma unroll
        for (int i = 0; i < 8; i++) {  // GDesc i = {pd lo, pd hi, idx, K} at dwords 4i..4i+3
            ix[i] = w[4 * i + 2];
            const bool nul = ix[i] == kGNull;
            vl[i] = nul ? w[0] : w[4 * i];
            vh[i] = nul ? w[1] : w[4 * i + 1];
        }
        v.K = w[3];  // one K per round
        const uint32_t lo = sel8(q, vl[0], vl[1], vl[2], vl[3], vl[4], vl[5], vl[6], vl[7]);
        const uint32_t hi = sel8(q, vh[0], vh[1], vh[2], vh[3], vh[4], vh[5], vh[6], vh[7]);
        v.p = ((uint64_t)(hi & 0xffffffu) << 32) | lo;
        v.d = hi >> 24;
        v.idx = sel8(q, ix[0], ix[1], ix[2], ix[3], ix[4], ix[5], ix[6], ix[7]);
        if constexpr (GV4<MODE>::LOGC) {  // pd = offset (40 bits) | K << 40 | seed << 48 | d << 56; K word = stored crc
            v.K = (w[1] >> 8) & 0xffu;
            v.p = (uint64_t)(uintptr_t)A.P.base + (((uint64_t)(hi & 0xffu) << 32) | lo);
            v.seed = (hi >> 16) & 1u;
            v.f = (uint32_t)(v.p & 127u);
            v.stored = sel8(q, w[3], w[7], w[11], w[15], w[19], w[23], w[27], w[31]);
        }
    } else {  // 128-B aligned base and stride (run_gv4): f = d = 0
        const uint64_t i = (uint64_t)uni(r) * 8u + q;
        const uint64_t ie = i < A.P.n ? i : (uint64_t)uni(r) * 8u;
        v.K = A.fixed_K;
        v.d = 0;
        v.p = (uint64_t)(uintptr_t)A.P.base + ie * A.P.fixed_bytes;
        v.idx = i < A.P.n ? (uint32_t)i : kGNull;
    }
    return v;
}

// Round descriptors prefetched with a VECTOR load into one of two pinned register
// sets (JL_GV4_DQ0 / JL_GV4_DQ1, each lane its group's 16-B GDesc), touched only
// by inline asm like the ring.  The prefetch cursor issues round k+1's load when
// it starts round k, if round k has >= P entries: the ring's own waits then
// cover it before either cursor reads it (at least P-1 younger ring loads), and
// the extra load only makes those waits stricter.  Otherwise (short rounds,
// first round) the scalar-load round_view is used.  r1: the scalar loads'
// latency was ~3.6 us per round and wave (1M x 4 KiB through descriptors 0.89
// vs 0.66 ms without any).
__device__ __forceinline__ void desc_issue(const GV4Args &A, uint32_t r, uint32_t q, uint32_t set) {
    const uint64_t a = (uint64_t)(uintptr_t)(A.desc + (uint64_t)r * 8u + q);
    if (set)
        asm volatile("global_load_dwordx4 " JL_GV4_DQ1 ", %0, off" ::"v"(a) : "memory", JL_GV4_DR1);
    else
        asm volatile("global_load_dwordx4 " JL_GV4_DQ0 ", %0, off" ::"v"(a) : "memory", JL_GV4_DR0);
}
template <int MODE>
__device__ __forceinline__ RoundView desc_read(const GV4Args &A, uint32_t set) {
    uint32_t lo, hi, ix, k;
    if (set)
        asm volatile(JL_GV4_DMOV1
                     : "=v"(lo), "=v"(hi), "=v"(ix), "=v"(k));
    else
        asm volatile(JL_GV4_DMOV0
                     : "=v"(lo), "=v"(hi), "=v"(ix), "=v"(k));
    // empty groups of a partial round mirror group 0 (lane 0)
    const bool nul = ix == kGNull;
    lo = nul ? (uint32_t)__builtin_amdgcn_readlane((int)lo, 0) : lo;
    hi = nul ? (uint32_t)__builtin_amdgcn_readlane((int)hi, 0) : hi;
    RoundView v;
    v.p = ((uint64_t)(hi & 0xffffffu) << 32) | lo;
    v.d = hi >> 24;
    v.idx = ix;
    v.K = (uint32_t)__builtin_amdgcn_readlane((int)k, 0);
    v.stored = 0;
    v.f = 0;
    v.seed = 0;
    if constexpr (GV4<MODE>::LOGC) {
        v.K = (uint32_t)__builtin_amdgcn_readlane((int)((hi >> 8) & 0xffu), 0);
        v.p = (uint64_t)(uintptr_t)A.P.base + (((uint64_t)(hi & 0xffu) << 32) | lo);
        v.seed = (hi >> 16) & 1u;
        v.f = (uint32_t)(v.p & 127u);
        v.stored = k;
    }
    return v;
}

template <int MODE>
__device__ __forceinline__ uint32_t n_entries(const GV4Args &A, uint32_t K) {
    return K + (GV4<MODE>::side(A) ? 1u : 0u);
}


// Round dealing (r4): workgroup b (XCD-major index bx of G) owns the rounds
// R - 1 - (j G + bx), j = 0, 1, ... — the table is sorted by K ascending, so
// heaviest first — and its 16 waves take them one at a time from a counter in
// LDS: a wave that runs faster takes more rounds, and the rounds left at the end
// are the lightest.  r3 dealt them statically in ascending K (round i W + w to
// wave w) and every wave had the same work, but the 4 waves of a SIMD do not run
// at the same rate — issue goes to the oldest first — so on C3 the waves of
// slots 0-3 finished at ~1.0 ms, slots 4-7 at ~1.3, 8-11 at ~1.7 and 12-15 at
// ~1.9 ms, and the kernel ran its last ~0.8 ms with ever fewer loads in flight
// (tools/gv4_wavetime.py on the branch study-r5-gv4-switches, profiles/r4i_gv4_wavetime.json); dealt dynamically but
// still ascending, C3's heaviest rounds (8 blocks of 64 KiB, ~0.3 ms for one
// wave) came last and left a 0.4 ms tail (r4j).  The taken rounds go through a
// 16-entry queue per wave in LDS: the prefetch cursor takes round i (and i + 1,
// whose descriptor it prefetches) from the counter, the compute cursor, up to P
// entries behind, reads the same sequence back.  The counter and queues sit in
// dwords [kGvDynDword, +257) of the LDS image, unused by both gv4 images (zero
// when the image is loaded).
// With a device counter (GV4Args::deal, zeroed before the kernel: by gv4_scan,
// or the log path's memset) only the heaviest 1/kGvStaticDiv of the rounds go by
// the stride; past them the workgroup's counter indexes BATCHES of kGvDealBatch
// consecutive rounds that the workgroups take from the device counter as they go
// (r4): the static stride balanced the waves of a CU but not the XCDs — on C3 the workgroups of four XCDs finished ~100 us after
// the other four's (XCD means 1 797-1 945 us, sigma ~14 us within an XCD; on the
// C5 mixed set the other four XCDs were the late ones; wave ends of r4l,
// tools/gv4_wavetime.py), and the kernel lasts until its slowest XCD.  The wave
// that opens batch b takes batch b + 1 from the device counter (the first one
// takes batches 0 and 1), so a batch's base is normally known before its first
// round is asked for; a wave that finds it missing waits on its tag in LDS.  The
// atomic's return makes the compiler wait vmcnt(0) (it cannot count the ring's
// asm loads), once per batch.  One device atomic per ROUND instead (batches of
// 2-8 rounds per wave) serialised on the counter's address: C5 1 056-B 0.97 ->
// 1.2-3.3 ms; batches from the first round on put C3's heaviest rounds on a few
// workgroups (64 per batch: 2.0 -> 2.43 ms), hence the static head.  Without a
// counter (implicit rounds), the stride above.
// batch size min(kGvDealBatch, R / (64 G)): every workgroup still takes >= ~48
// batches (the tail's granularity), and a call of fewer than 64 G rounds keeps
// the stride (its batches would leave most CUs idle).  The static head is the
// heaviest 1/kGvStaticDiv of the rounds (r4w: 1/2 and 1/8 within +-0.5 %).
constexpr uint32_t kGvDealBatch = 32;
constexpr uint32_t kGvStaticDiv = 4;
constexpr uint32_t kGvTagBits = 26, kGvTagMask = (1u << kGvTagBits) - 1u;  // reads <= kGvDealBatch < 64
static_assert(kGvDealBatch < 64u, "a slot's read count takes 6 bits");
constexpr uint32_t kGvNoRound = 0xffffffffu;  // >= any round count (< 2^31)

// Prefetch cursor: walks the wave's rounds (seq(i), from the workgroup's counter) entry by entry.
template <int MODE>
struct GPF {
    uint32_t r, R, G, bx;  // rounds (< 2^31); the workgroup's rounds are j G + bx
    uint32_t i;            // r = seq(i)
    uint32_t made;         // rounds taken into the queue so far (seq(i) for i < made is known)
    uint32_t *ctr, *Q;     // LDS: the workgroup's counter, this wave's queue
    uint32_t *deal;        // the device counter (null: the workgroup's)
    uint32_t J0;           // with deal: counter values below J0 take the stride, j G + bx
    uint32_t DB;           // with deal: rounds per batch
    uint32_t e, E, K;
    uint32_t k;      // sequence number of the current round (descriptor set k & 1)
    bool vec_next;   // the next round's descriptor was issued into set (k+1) & 1
    uint32_t Eprev;  // entries of round k-1
    uint64_t addr;        // per lane: next step's chunk address
    uint64_t side_addr;   // per lane: the side chunk
    uint64_t dummy;       // a mapped address (zero page) for lanes with nothing to load

    // the wave's i-th round: taken from the workgroup's counter the first time it
    // is asked for (i == made), read back from the queue after that
    __device__ __forceinline__ uint32_t seq(uint32_t i_) {
        if (i_ < made) return uni(Q[i_ & 15u]);
        const bool lane0 = __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)) == 0u;
        uint32_t j = 0;
        if (lane0) j = atomicAdd(ctr, 1u);
        j = uni(j);
        if (deal && j >= J0) {  // batches of rounds from the device counter
            const uint32_t k = j - J0, X0 = J0 * G;
            const uint32_t b = k / DB, o = k - b * DB;
            // slot s = {base, tag}: tag = (batch + 1) mod 2^kGvTagBits | rounds of that
            // batch whose base was read << kGvTagBits.  A slot is reused by batch
            // b + 16 only after all DB rounds of batch b read it: without that count
            // (r4) a wave delayed between taking a round of batch b and reading its
            // slot could find it overwritten by a batch 16 later (DB = 1 when the
            // call has just over 64 G rounds): a hang on the tag, or a wrong base
            volatile uint32_t *slot = ctr + (kGvBatchDword - kGvDynDword);
            if (o == 0u) {  // opens batch b: take batch b + 1 (b = 0: batches 0 and 1)
                const uint32_t n = b == 0u ? 2u * DB : DB;
                uint32_t g = 0;
                if (lane0) g = atomicAdd(deal, n);
                g = uni(g);
                if (lane0) {
                    if (b == 0u) {
                        slot[0] = g;
                        slot[1] = 1u;
                        g += DB;
                    }
                    const uint32_t s = 2u * ((b + 1u) & 15u);
                    // its previous batch (b - 15) had all its rounds taken before this one
                    // (the counter is monotonic), and each taker reads, then counts; its
                    // tag is checked too (its opener may not have written it yet)
                    if (b + 1u >= 16u)
                        while (slot[s + 1u] != (((b - 14u) & kGvTagMask) | (DB << kGvTagBits)))
                            __builtin_amdgcn_s_sleep(1);
                    slot[s] = g;  // base before tag: LDS writes of a wave land in order
                    slot[s + 1u] = (b + 2u) & kGvTagMask;
                }
            }
            const uint32_t s = 2u * (b & 15u);
            while ((uni(slot[s + 1u]) & kGvTagMask) != ((b + 1u) & kGvTagMask)) __builtin_amdgcn_s_sleep(1);
            const uint32_t base = uni(slot[s]);
            if (lane0) atomicAdd((uint32_t *)(slot + s + 1u), 1u << kGvTagBits);  // read: LDS ops of a wave stay in order
            const uint64_t x = (uint64_t)X0 + base + o;
            const uint32_t rr = x < R ? R - 1u - (uint32_t)x : kGvNoRound;
            Q[made & 15u] = rr;
            made++;
            return rr;
        }
        const uint64_t x = (uint64_t)j * G + bx;
        const uint32_t rr = x < R ? R - 1u - (uint32_t)x : kGvNoRound;  // heaviest first
        Q[made & 15u] = rr;  // every lane writes the same value
        made++;
        return rr;
    }
    __device__ __forceinline__ void setup(const GV4Args &A, uint32_t lane, bool vec) {
        const uint32_t q = lane >> 3, l = lane & 7u;  // group, lane in group
        RoundView v;
        if (vec) {
            v = desc_read<MODE>(A, k & 1u);
        } else {
            for (;;) {  // K == 0 rounds (empty blocks, results already written) are skipped
                v = round_view<MODE>(A, r, q);
                if (uni(v.K) != 0u) break;
                i++;
                r = seq(i);
                if (r >= R) return;
            }
        }
        K = uni(v.K);
        Eprev = E;
        E = uni(n_entries<MODE>(A, K));
        // issue round k+1's descriptor into set (k+1) & 1 = (k-1) & 1 when
        //  * E_k > P: >= P-2 ring loads are issued behind it before either cursor
        //    reads it (and none of round 0's P priming loads reaches round 1), and
        //  * E_{k-1} >= P: the compute cursor has already read round k-1's
        //    descriptor from that set (it is P entries behind)
        // gv4 finish() takes the same decision from the same E values
        const uint32_t rn = seq(i + 1u);
        vec_next = A.desc && E > (uint32_t)JL_GV4_RING && (k == 0u || Eprev >= (uint32_t)JL_GV4_RING) && rn < R;
        if (vec_next) desc_issue(A, rn, q, (k + 1u) & 1u);
        const uint64_t p = v.p;
        const uint64_t n = (uint64_t)K * 128u - (p & 127u) - v.d;
        const uint64_t pa = p & ~(uint64_t)15;
        addr = (p & ~(uint64_t)127) + 16u * l;
        // side chunks (16-B aligned, each holding a byte of what is needed): lane 0 / 1 of the group
        uint64_t c0 = pa, c1 = pa;
        if constexpr (GV4<MODE>::LOGC) {
            e = 0;
            return;
        } else if (GV4<MODE>::VERIFY) {
            const uint64_t sa = MODE == MODE_LOG_VERIFY ? p - 6u : p + n;  // stored crc
            c0 = sa & ~(uint64_t)15;
            c1 = (sa + 3u) & ~(uint64_t)15;
        } else {
            // real blocks only (idx < kGPart): chunk groups of a split block and empty groups load nothing
            if (A.P.init && v.idx < kGPart) c0 = (uint64_t)(uintptr_t)(A.P.init + v.idx) & ~(uint64_t)15;
            if (A.P.suffix && v.idx < kGPart) c1 = (uint64_t)(uintptr_t)(A.P.suffix + v.idx) & ~(uint64_t)15;
        }
        side_addr = l == 0u ? c0 : (l == 1u ? c1 : dummy);
        e = 0;
    }
    __device__ __forceinline__ void init(const GV4Args &A, uint32_t *lds, uint32_t g, uint32_t b, uint32_t nr,
                                         uint32_t lane, uint64_t dmy) {
        ctr = lds + kGvDynDword;
        Q = lds + kGvDynDword + 1u + 16u * (threadIdx.x >> 6);
        DB = nr / (64u * g) < kGvDealBatch ? nr / (64u * g) : kGvDealBatch;
        deal = DB ? A.deal : nullptr;
        J0 = nr / (kGvStaticDiv * g);
        made = 0;
        G = g;
        bx = b;
        R = nr;
        i = 0;
        r = seq(0);
        dummy = dmy;
        k = 0;
        E = 0;
        vec_next = false;
        if (r < R) setup(A, lane, false);
    }
    // Address of the next entry (advancing the cursor).  The ring load itself is
    // issued by the caller at ONE site per slot: a load asm in several branches
    // would give the slot's new value a phi at the join, and the register
    // allocator may resolve that phi with a copy of the still-in-flight register.
    __device__ __forceinline__ uint64_t next(const GV4Args &A, uint32_t lane) {
        if (r >= R) return dummy;  // past the wave's last round: keep the ring count exact
        const uint32_t e0 = GV4<MODE>::side(A) ? 1u : 0u;
        uint64_t a;
        if (e >= e0) {
            a = addr;
            addr += 128u;
        } else {
            a = side_addr;
        }
        if (++e == E) {
            i++;
            r = seq(i);
            k++;
            if (r < R) setup(A, lane, vec_next);
            r = uni(r);
        }
        e = uni(e);
        return a;
    }
};

// (r3-r5 measured bound-study variants of this kernel: strict waits, loads
// without nt, whole 8-entry fast turns, address checks, no fast path, no step
// math, L2-resident data, no epilogue math, no pad / seed handling — DESIGN.md
// §4.2; they live on the branch study-r5-gv4-switches.)
template <int MODE>
__global__ __launch_bounds__(JL_GV4_THREADS) void crc_gv4_kernel(const uint4 *__restrict__ img, GV4Args A,
                                                       const uint8_t *__restrict__ zero) {
    constexpr int P_ = JL_GV4_RING;
    __shared__ uint32_t lds[kImageBytes / 4];
    load_image(lds, img);
    const uint32_t *ldsG = lds + kGOff / 4u;  // the G tables (rotated image)
    const uint32_t lane = threadIdx.x & 63u, q = lane >> 3, l = lane & 7u;
    const GLanes gl(lane);
    const uint32_t waves = gridDim.x * (blockDim.x >> 6);
    // Workgroup ids XCD-major (workgroup b runs on XCD b % 8): consecutive rounds
    // go to neighbouring CUs of one XCD, so the run of heavy rounds at the end of
    // the K-sorted table spreads over every CU (r2: C3 2.19 -> 2.13 ms; with
    // blockIdx-major ids they all landed on the first ~60 CUs)
    const uint32_t G = gridDim.x, b = blockIdx.x;
    const uint32_t bx = (G & 7u) ? b : (b & 7u) * (G >> 3) + (b >> 3);
    const uint32_t R = A.desc ? *A.n_rounds : (uint32_t)((A.P.n + 7u) / 8u);  // rounds < 2^31
    (void)waves;
    // the prefetch cursor takes the wave's first round with K > 0 (round dealing
    // above); the compute cursor starts on the same one
    GPF<MODE> pf;
    pf.init(A, lds, G, bx, R, lane, (uint64_t)(uintptr_t)zero + 16u * lane);
    if (pf.r >= R) return;  // the workgroup's rounds are all taken: no ring started
    uint32_t ci = pf.i, cr = pf.r;
    RoundView cv = round_view<MODE>(A, cr, q);
    const uint32_t e0 = GV4<MODE>::side(A) ? 1u : 0u;
    uint32_t zero_v;
    asm volatile("v_mov_b32 %0, 0" : "=v"(zero_v));

    // The ring lives in PINNED registers (JL_GV4_SLOTS, the two prefetched
    // round-descriptor sets JL_GV4_DQ0/1 just below it), above what the
    // compiler allocates: the register allocator
    // can never copy, reuse or spill a slot while its load is in flight — with
    // compiler-allocated ring values this kernel's branchy rounds made it do that
    // (r1: intermittent faults).  Each slot is touched only by inline asm: the
    // load (which declares the slot clobbered), the wait, and the reads (the
    // chains' final XOR takes the data word straight from the slot register).
#define JL_GLD(RQ, ADDR, OFF, R0, R1, R2, R3)                                                                  \
    asm volatile("global_load_dwordx4 " RQ ", %0, off offset:%1 nt" ::"v"(ADDR), "n"(OFF)                      \
                 : "memory", R0, R1, R2, R3);
#define JL_LOAD(RQ, R0, R1, R2, R3)                                                                            \
    {                                                                                                          \
        const uint64_t a_ = pf.next(A, lane);                                                                  \
        JL_GLD(RQ, a_, 0, R0, R1, R2, R3)                                                                      \
    }
#define JL_PRIME(u, RQ, R0, R1, R2, R3) JL_LOAD(RQ, R0, R1, R2, R3)
    JL_GV4_SLOTS(JL_PRIME)
#undef JL_PRIME

    uint32_t cK = uni(cv.K), cE = uni(n_entries<MODE>(A, cK)), ce = 0, ck = 0, cEprev = 0;
    v4u side_c;  // lane 0 / 1 of each group: the side chunk
    uint32_t x0 = 0, x1 = 0, x2 = 0, x3 = 0;

    // rare entries of a round: the side chunk, step 0 (front pad, seed), step K-1 (tail pad)
    auto rare = [&](v4u wv) {
        if (ce < e0) {
            side_c = wv;
            return;
        }
        const uint32_t f = GV4<MODE>::LOGC ? cv.f : (uint32_t)(cv.p & 127u);
        uint32_t v[4] = {wv.x, wv.y, wv.z, wv.w};
        // byte selectors from the image (kG4SelByte): v_med3 + one LDS read + v_perm per
        // dword, no divergent shift code
        if (ce + 1u == cE) {  // last step: zero the tail pad (bytes >= 128 - d of the window)
            const int tl = (int)(128u - cv.d) - (int)(16u * l);
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const int tt = min(max(tl - 4 * j, 0), 4);
                v[j] = __builtin_amdgcn_perm(0u, v[j], lds_at(lds, (GV4<MODE>::LOGC ? kLCSelB : kSelB) + 52u + 4u * (uint32_t)tt));
            }
        }
        if (ce == e0) {
            // ---- step 0: zero the front pad, feed the seed word W as the 4 bytes before p
            // seed word of this block
            uint32_t W = A.seed0;
            if (!GV4<MODE>::VERIFY && !GV4<MODE>::LOGC && A.P.init) {
                // init[idx] from lane 0's side chunk, broadcast to the group's 8 lanes
                const uint64_t ia = (uint64_t)(uintptr_t)(A.P.init + (cv.idx == kGNull ? 0u : cv.idx));
                const uint32_t k = (uint32_t)(ia >> 2) & 3u;
                const uint32_t own = k & 2u ? (k & 1u ? side_c.w : side_c.z) : (k & 1u ? side_c.y : side_c.x);
                const uint32_t y = ~(uint32_t)__builtin_amdgcn_ds_bpermute((int)((lane & ~7u) << 2), (int)own);
                W = lds_at(lds, kUB + ((y & 0xffu) << 2)) ^ lds_at(lds, kUB + 1024u + (((y >> 8) & 0xffu) << 2)) ^
                    lds_at(lds, kUB + 2048u + (((y >> 16) & 0xffu) << 2)) ^ lds_at(lds, kUB + 3072u + ((y >> 24) << 2));
            }
            if (MODE == MODE_CRC && cv.idx >= kGPart) W = 0u;  // chunk of a split block: from state 0
            if constexpr (GV4<MODE>::LOGC) W = cv.seed ? A.seed0 : 0u;  // record chunks after the first: from 0
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const int t = min(max((int)(16u * l + 4u * j) - (int)f, -8), 4);  // dword start relative to p
                v[j] = __builtin_amdgcn_perm(W, v[j], lds_at(lds, (GV4<MODE>::LOGC ? kLCSelB : kSelB) + 4u * (uint32_t)(t + 8)));
            }
            // virtual dword -4 (chain lane 7 / dword 3 of step -1) when f < 4
            // (a divergent branch: most rounds have no such lane and skip it)
            uint32_t i73 = zero_v;
            if (l == 7u && f < 4u) i73 = gstep(ldsG, W << (8 * f), gl);
            x0 = zero_v ^ v[0];
            x1 = zero_v ^ v[1];
            x2 = zero_v ^ v[2];
            x3 = i73 ^ v[3];
        } else {
            x0 = gstep_x3(ldsG, x0, gl, v[0]);
            x1 = gstep_x3(ldsG, x1, gl, v[1]);
            x2 = gstep_x3(ldsG, x2, gl, v[2]);
            x3 = gstep_x3(ldsG, x3, gl, v[3]);
        }
    };
    // end of a round: epilogue, result, next round of the compute cursor; false when done
    auto finish = [&]() -> bool {
        // chain (l, j) ends at 16 l + 4 j past the last window, the window ends d
        // = 16 a + 4 c + e bytes past the block: shift by z^-(4 (j + c)), then by
        // z^-(16 (l + a)) (lane tables), group xor, then z^-e
        const uint32_t d = cv.d;
        const uint32_t col = ((l + (d >> 4)) & 15u) | ((q & 1u) << 4);
        uint32_t st;
        if constexpr (GV4<MODE>::LOGC) {
            // chain j: its pending gap step, then z^-(4 (j + c) + e), in one table
            // (uniform d mod 16; crc_math.hpp build_lds_image_logchunk)
            const uint32_t sm = kLCMB + 512u * (d & 15u);
            const uint32_t c = xor3(ushift(lds, x0, sm), ushift(lds, x1, sm + 2048u), ushift(lds, x2, sm + 4096u)) ^
                               ushift(lds, x3, sm + 6144u);
            st = group_xor<8>(realign(lds, c, kLaneB | (col << 2)));
        } else {
            // chain j: its pending gap step, then z^-(4 (j + c)), in one table
            const uint32_t sa = 512u * ((d >> 2) & 3u);
            const uint32_t c = xor3(ushift(lds, x0, kShiftB + sa), ushift(lds, x1, kShiftB + 512u + sa),
                                    ushift(lds, x2, kShiftB + 1024u + sa)) ^
                               ushift(lds, x3, kShiftB + 1536u + sa);
            st = group_xor<8>(realign(lds, c, kLaneB | (col << 2)));
            st = ushift(lds, st, kEB + 512u * (d & 3u));
        }
        // side chunks of lanes 0 and 1 of the group, seen from lane 0 (DPP row_shl:1)
        const uint32_t h0 = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)side_c.x, 0x101, 0xf, 0xf, false);
        const uint32_t h1 = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)side_c.y, 0x101, 0xf, 0xf, false);
        const uint32_t h2 = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)side_c.z, 0x101, 0xf, 0xf, false);
        const uint32_t h3 = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)side_c.w, 0x101, 0xf, 0xf, false);
        const uint64_t p = cv.p;
        const uint32_t raw = st;  // chunk groups of a split block report the raw state
        if (!GV4<MODE>::VERIFY && !GV4<MODE>::LOGC && A.P.suffix) {
            const uint64_t sa = (uint64_t)(uintptr_t)(A.P.suffix + (cv.idx == kGNull ? 0u : cv.idx));
            const uint32_t k = (uint32_t)(sa >> 2) & 3u;
            const uint32_t dw = k & 2u ? (k & 1u ? h3 : h2) : (k & 1u ? h1 : h0);
            const uint32_t sfx = (dw >> (8u * (uint32_t)(sa & 3u))) & 0xffu;
            st = (st >> 8) ^ lds_at(lds, kT0B + (((st ^ sfx) & 0xffu) << 2));
        }
        const uint32_t crc = ~st, m = mask_crc(crc);
        if (l == 0u && cv.idx != kGNull) {
            if constexpr (GV4<MODE>::LOGC) {
                if (cv.idx >= kGPart) {
                    A.parts[cv.idx - kGPart] = raw;
                } else if (m != cv.stored) {  // rare: first_bad[block] = min(header offset in the block)
                    // the chunk's offset from its descriptor (a rare vector load: the
                    // compiler's vmcnt(0) before its use only drains the ring here)
                    const uint64_t h = (A.desc[(uint64_t)cr * 8u + q].pd & 0xffffffffffull) - 6u;
                    atomicMin(A.P.out32 + (h >> 15), (uint32_t)(h & 32767u));
                }
            } else if (MODE == MODE_CRC) {
                if (cv.idx >= kGPart) A.parts[cv.idx - kGPart] = raw;
                else A.P.out32[cv.idx] = (A.P.flags & 1u) ? m : crc;
            } else {
                const uint32_t n = cK * 128u - (uint32_t)(p & 127u) - cv.d;
                const uint64_t sa = MODE == MODE_LOG_VERIFY ? p - 6u : p + n;
                // 32-B window: lane 0's chunk (sa & ~15) then lane 1's ((sa+3) & ~15, the same or the next)
                const uint32_t o = (uint32_t)(sa & 15u), a = o >> 2, b = o & 3u;
                const bool two = ((sa + 3u) & ~(uint64_t)15) != (sa & ~(uint64_t)15);
                const uint32_t D0 = side_c.x, D1 = side_c.y, D2 = side_c.z, D3 = side_c.w;
                const uint32_t D4 = two ? h0 : 0u;
                const uint32_t lo_w = a & 2u ? (a & 1u ? D3 : D2) : (a & 1u ? D1 : D0);
                const uint32_t hi_w = a & 2u ? (a & 1u ? D4 : D3) : (a & 1u ? D2 : D1);
                const uint32_t stored = __builtin_amdgcn_alignbyte(hi_w, lo_w, b);
                A.P.out8[cv.idx] = stored == m ? 1u : 0u;
            }
        }
        // next round of the compute cursor: from the descriptor set the prefetch
        // cursor loaded if the finished round had >= P entries, else scalar loads
        // (skipping K == 0 rounds)
        const bool vec = A.desc && cE > (uint32_t)P_ && (ck == 0u || cEprev >= (uint32_t)P_);  // as GPF::setup
        cEprev = cE;
        ck++;
        if (vec) {
            ci++;
            cr = pf.seq(ci);
            if (cr >= R) return false;
            cv = desc_read<MODE>(A, ck & 1u);
        } else {
            for (;;) {
                ci++;
                cr = pf.seq(ci);
                if (cr >= R) return false;
                cv = round_view<MODE>(A, cr, q);
                if (uni(cv.K) != 0u) break;
            }
        }
        cK = uni(cv.K);
        cE = uni(n_entries<MODE>(A, cK));
        ce = 0;
        return true;
    };

    // plain step: the 16 lookups of the 4 chains, then ONE asm with the 4 XORs
    // that take the data words straight from the slot registers (a volatile asm
    // orders memory operations around it, so one per chain would serialise the
    // chains' LDS latencies)
#define JL_LK(x, T, A3)                                                                                    \
    const uint32_t T = xor3(lds_at(ldsG, JL_GADDR(gl.l3, x, 0u)), lds_at(ldsG, JL_GADDR(gl.l2, x, 1u)),    \
                            lds_at(ldsG, JL_GADDR(gl.l1, x, 2u)));                                         \
    const uint32_t A3 = lds_at(ldsG, JL_GADDR(gl.l0, x, 3u));
#define JL_XS4(R0, R1, R2, R3)                                                                             \
    {                                                                                                      \
        JL_LK(x0, t0_, u0_) JL_LK(x1, t1_, u1_) JL_LK(x2, t2_, u2_) JL_LK(x3, t3_, u3_)                    \
        asm volatile("v_bitop3_b32 %0, %4, %5, " R0 " bitop3:0x96\n\t"                                   \
                     "v_bitop3_b32 %1, %6, %7, " R1 " bitop3:0x96\n\t"                                    \
                     "v_bitop3_b32 %2, %8, %9, " R2 " bitop3:0x96\n\t"                                    \
                     "v_bitop3_b32 %3, %10, %11, " R3 " bitop3:0x96"                                       \
                     : "=&v"(x0), "=&v"(x1), "=&v"(x2), "=&v"(x3)                                           \
                     : "v"(t0_), "v"(u0_), "v"(t1_), "v"(u1_), "v"(t2_), "v"(u2_), "v"(t3_), "v"(u3_));    \
    }
#define JL_G(u, RQ, R0, R1, R2, R3)                                                                        \
    {                                                                                                      \
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(P_ - JL_RING_SLACK) : "memory");                         \
        if (ce > e0 && ce + 1u < cE) {                                                                     \
            JL_XS4(R0, R1, R2, R3)                                                                         \
        } else {                                                                                           \
            v4u wv_;                                                                                       \
            uint32_t w0_, w1_, w2_, w3_;                                                                   \
            asm volatile("v_mov_b32 %0, " R0 "\n\tv_mov_b32 %1, " R1 "\n\tv_mov_b32 %2, " R2                   \
                         "\n\tv_mov_b32 %3, " R3                                                            \
                         : "=v"(w0_), "=v"(w1_), "=v"(w2_), "=v"(w3_));                                     \
            wv_.x = w0_;                                                                                   \
            wv_.y = w1_;                                                                                   \
            wv_.z = w2_;                                                                                   \
            wv_.w = w3_;                                                                                   \
            rare(wv_);                                                                                     \
        }                                                                                                  \
        if (++ce == cE && !finish()) break;                                                                \
        JL_LOAD(RQ, R0, R1, R2, R3)                                                                        \
    }
    // Fast half turn: the next 4 entries of BOTH cursors are plain steps of their
    // current rounds (no rare entry, no epilogue, no round switch), so they run
    // as straight-line code: wait, the 4 chains, and the refill at the cursor's
    // address + 128 (u mod 4) — no per-step bookkeeping.  Otherwise the half
    // takes the per-entry path (either way it ends on the next half's slot).
    // Half turns rather than whole 8-entry turns: a round boundary then blocks
    // fewer entries from the fast path (rounds of 32 entries: ~72 % fast vs ~47 %).
#define JL_F(u, RQ, R0, R1, R2, R3)                                                                        \
    {                                                                                                      \
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(P_ - JL_RING_SLACK) : "memory");                         \
        JL_XS4(R0, R1, R2, R3)                                                                             \
        JL_GLD(RQ, pf.addr, 128 * ((u) & 3), R0, R1, R2, R3)                                               \
    }
#define JL_HALF(SLOTS)                                                                                     \
    if (ce > e0 && ce + 4u < cE && pf.r < pf.R && pf.e >= e0 && pf.e + 4u < pf.E) {             \
        SLOTS(JL_F)                                                                                        \
        ce = uni(ce + 4u);                                                                                 \
        pf.e = uni(pf.e + 4u);                                                                             \
        pf.addr += 512u;                                                                                   \
    } else {                                                                                               \
        SLOTS(JL_G)                                                                                        \
    }
    for (;;) {
        JL_HALF(JL_GV4_SLOTS_LO)
        JL_HALF(JL_GV4_SLOTS_HI)
    }
#undef JL_HALF
#undef JL_F
#undef JL_G
#undef JL_XS4
#undef JL_LK
#undef JL_LOAD
#undef JL_GLD
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the ring drains before the wave ends
}

template <>
hipError_t launch_gv4_m<JL_MODE>(const void *img, const GV4Args &A, const uint8_t *zero, int grid, hipStream_t st) {
    hipLaunchKernelGGL((crc_gv4_kernel<JL_MODE>), dim3(grid), dim3(JL_GV4_THREADS), 0, st, (const uint4 *)img, A, zero);
    return hipGetLastError();
}

#if JL_MODE == 0
// ---------------------------------------------------------------------------
// Round pipeline (a counting sort by K; r1 replaced a 17-bit radix sort plus
// two scans, ~20 launches, with these three):
//   hist   per-workgroup LDS histogram of the bins b = gv4_key(K, d) of
//          its chunk of blocks, flushed with one global atomic per non-empty
//          bin (bins >= kLdsBins count globally); empty blocks get their
//          result here and take no bin
//   scan   one workgroup: rstart[b] = rounds of the bins before b, where a bin
//          of c blocks has ceil(c/8) rounds (kGSoloKey: c rounds, one block
//          each, since its blocks differ in K); total -> *n_rounds
//   place  each workgroup recounts its chunk in LDS (the LDS atomic returns
//          the block's rank in the chunk), reserves its ranks in every bin
//          with one global atomic, and writes each block's GDesc at round
//          rstart[b] + rank/8, group rank%8.
// The order of blocks inside a bin follows the atomics, so the composition of
// rounds varies from run to run; each block's result does not.
// ---------------------------------------------------------------------------
// block i: its first byte and length (fixed-stride batches that are not 128-B
// aligned come through here too, with P.off == null)
__device__ __forceinline__ void gv4_block(const KParams &P, uint64_t i, uint64_t &p, uint32_t &n) {
    if (P.off) {
        p = (uint64_t)(uintptr_t)P.base + P.off[i];
        n = P.len[i] + P.len_add;
    } else {
        p = (uint64_t)(uintptr_t)P.base + i * P.fixed_bytes;
        n = (uint32_t)P.fixed_bytes;
    }
}

// steps of block (p, n) on the 128-B aligned grid
__device__ __forceinline__ uint32_t gv4_K(uint64_t p, uint32_t n) {
    return n ? (uint32_t)(((p & 127u) + (uint64_t)n + 127u) >> 7) : 0u;
}

constexpr uint32_t kLdsBins = 4096;  // bins counted in LDS (K < 4096: blocks < 512 KiB)

// Sort key of a block of K steps with tail pad d: K.  (Keys by (K, d mod 16),
// which make one round's epilogue tables uniform, cost C3 14 % in r2: a K bin
// split 16 ways scatters neighbouring arena blocks over far-apart rounds.  The
// log path bins its chunks that way, log_chunks.hip.)
__device__ __forceinline__ uint32_t gv4_key(uint32_t K, uint32_t d) {
    (void)d;
    return K < kGSoloKey ? K : kGSoloKey;
}

// Wave-aggregated counting: for every distinct bin among the wave's lanes, one
// atomic adds the number of lanes in it (to the LDS counter for small bins, the
// global one otherwise); each lane gets its rank = the atomic's old value + the
// number of lower lanes in the same bin, so the wave's consecutive blocks of a
// bin take consecutive ranks (rounds of neighbouring blocks).
__device__ __forceinline__ uint32_t wave_rank(uint32_t b, uint32_t *lds_ctr, uint32_t *glob_ctr) {
    const uint32_t lane = __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
    uint64_t active = __builtin_amdgcn_ballot_w64(b != 0xffffffffu);
    uint32_t rank = 0;
    for (uint32_t it = 0; active; it++) {
        if (it == 2u) {
            // many distinct bins in the wave (C3's Zipf sizes: ~40 per wave): the
            // lanes left take their ranks with their own LDS atomics instead of one
            // ballot round per bin (C3: hist 43 -> 16 us, place 60 -> 22 us); only
            // global bins (blocks >= 512 KiB) keep the loop
            const bool mine = ((active >> lane) & 1ull) && b < kLdsBins;
            if (mine) rank = atomicAdd(&lds_ctr[b], 1u);
            active &= ~__builtin_amdgcn_ballot_w64(mine);
            if (!active) break;
        }
        const uint32_t leader = (uint32_t)__builtin_ctzll(active);
        const uint32_t b0 = (uint32_t)__builtin_amdgcn_readlane((int)b, (int)leader);
        const uint64_t mask = __builtin_amdgcn_ballot_w64(b == b0);
        uint32_t base = 0;
        if (lane == leader) {
            const uint32_t cnt = (uint32_t)__builtin_popcountll(mask);
            base = b0 < kLdsBins ? atomicAdd(&lds_ctr[b0], cnt) : atomicAdd(&glob_ctr[b0], cnt);
        }
        base = (uint32_t)__builtin_amdgcn_readlane((int)base, (int)leader);
        if (b == b0)
            rank = base + __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
        active &= ~mask;
    }
    return rank;
}

__device__ __forceinline__ void gv4_chunk(uint64_t n, uint64_t &i0, uint64_t &i1) {
    const uint64_t per = (n + gridDim.x - 1) / gridDim.x;
    i0 = (uint64_t)blockIdx.x * per;
    i1 = i0 + per < n ? i0 + per : n;
}

// bin of block i (0xffffffff: empty block, whose result is written here:
// extend(init, empty) = init, then the suffix byte)
__device__ __forceinline__ bool gv4_in_range(const KParams &P, uint64_t i) {
    return !P.off || block_in_range(P, P.off[i], P.len[i] + P.len_add);
}

__device__ __forceinline__ uint32_t gv4_bin(const KParams &P, uint64_t i, bool write_empty) {
    uint64_t p;
    uint32_t n;
    gv4_block(P, i, p, n);
    const bool bad = !gv4_in_range(P, i);
    const uint32_t K = bad ? 0u : gv4_K(p, n);
    if (K) return gv4_key(K, (uint32_t)((uint64_t)K * 128u - (p & 127u) - n));
    if (write_empty && bad) {  // a descriptor past the caller's bytes: nothing read, result 0
        if (P.mode == MODE_CRC) P.out32[i] = 0u;
        else P.out8[i] = 0u;
    } else if (write_empty) {
        uint32_t st = ~(P.init ? P.init[i] : 0u);
        if (P.suffix) st = (st >> 8) ^ P.aux[(st ^ P.suffix[i]) & 0xffu];
        const uint32_t crc = ~st;
        if (P.mode == MODE_CRC) P.out32[i] = (P.flags & 1u) ? mask_crc(crc) : crc;
        else P.out8[i] = 1u;
    }
    return 0xffffffffu;
}

// Split geometry of a block of n bytes (MODE_CRC, n > kGSplitMin): m <= 2048
// chunks of cs bytes (a multiple of 128, >= 64 KiB), the last one shorter.
// Every chunk starts at the block's offset in its 128-B window.
__device__ __forceinline__ bool gv4_split_geom(const KParams &P, const GSplit &S, uint32_t n, uint32_t &cs,
                                               uint32_t &m) {
    if (!S.part_cap || P.mode != MODE_CRC || (uint64_t)n <= kGSplitMin) return false;
    uint64_t c = ((uint64_t)n + 2047u) / 2048u;
    c = (c + 127u) & ~(uint64_t)127;
    if (c < (64u << 10)) c = 64u << 10;
    cs = (uint32_t)c;
    m = (uint32_t)(((uint64_t)n + c - 1u) / c);
    return true;
}

// bins and tail pads of a split block's full chunks (F) and last chunk (L)
struct GChunks {
    uint32_t kF, kL, dF, dL, L;
};
__device__ __forceinline__ GChunks gv4_chunks(uint64_t p, uint32_t n, uint32_t cs, uint32_t m) {
    GChunks g;
    const uint32_t f = (uint32_t)(p & 127u);
    g.L = n - (m - 1u) * cs;
    g.kF = (f + cs + 127u) >> 7;
    g.kL = (f + g.L + 127u) >> 7;
    g.dF = 128u * g.kF - f - cs;
    g.dL = 128u * g.kL - f - g.L;
    return g;
}

__global__ __launch_bounds__(1024) void gv4_hist_kernel(KParams P, GSplit S, uint32_t *hist) {
    __shared__ uint32_t h[kLdsBins];
    for (uint32_t b = threadIdx.x; b < kLdsBins; b += blockDim.x) h[b] = 0;
    __syncthreads();
    uint64_t i0, i1;
    gv4_chunk(P.n, i0, i1);
    for (uint64_t k0 = i0; k0 < i1; k0 += blockDim.x) {  // every lane runs every iteration (wave_rank)
        const uint64_t i = k0 + threadIdx.x;
        uint32_t b = 0xffffffffu;
        if (i < i1) {
            uint64_t p;
            uint32_t n, cs, m;
            gv4_block(P, i, p, n);
            bool split = false;
            if (gv4_in_range(P, i) && gv4_split_geom(P, S, n, cs, m)) {  // rare: blocks > 512 KiB
                const unsigned long long base = atomicAdd(&S.ctl[0], (unsigned long long)m);
                split = base + m <= S.part_cap;
                S.bigbase[i] = split ? (uint32_t)base : 0xffffffffu;
                if (split) {
                    const uint32_t bid = (uint32_t)atomicAdd(&S.ctl[1], 1ull);
                    GBig g;
                    g.i = i;
                    g.part0 = (uint32_t)base;
                    g.m = m;
                    S.big[bid] = g;
                    const GChunks c = gv4_chunks(p, n, cs, m);
                    const uint32_t bF = gv4_key(c.kF, c.dF), bL = gv4_key(c.kL, c.dL);
                    if (m > 1u) atomicAdd(&hist[bF], m - 1u);
                    atomicAdd(&hist[bL], 1u);
                    atomicMax(&hist[kGSoloKey + 1u], bF > bL ? bF : bL);
                }
            }
            if (!split) b = gv4_bin(P, i, true);
        }
        wave_rank(b, h, hist);
        if (b >= kLdsBins && b < kGSoloKey) atomicMax(&hist[kGSoloKey + 1u], b);  // rare: blocks >= 512 KiB
    }
    __shared__ uint32_t wg_max;
    if (threadIdx.x == 0) wg_max = 0;
    __syncthreads();
    uint32_t mx = 0;
    for (uint32_t b = threadIdx.x; b < kLdsBins; b += blockDim.x)
        if (h[b]) {
            atomicAdd(&hist[b], h[b]);
            mx = b;
        }
    if (mx) atomicMax(&wg_max, mx);  // LDS: one global atomic per workgroup below
    __syncthreads();
    if (threadIdx.x == 0 && wg_max) atomicMax(&hist[kGSoloKey + 1u], wg_max);
}

// hist[kGSoloKey + 1] holds the largest non-solo bin (atomicMax in the hist kernel):
// the scan only walks [0, that], in coalesced tiles of 4096 bins through LDS
// The scan also marks the empty groups of every bin's last, partial round
// (idx = kGNull; the main kernel mirrors group 0 there) and groups 1..7 of the
// solo rounds, so the descriptor table needs no clearing.
__device__ __forceinline__ void gv4_null_groups(GDesc *desc, uint64_t round, uint32_t from) {
    for (uint32_t g = from; g < 8u; g++) desc[round * 8u + g].idx = kGNull;
}

__global__ __launch_bounds__(1024) void gv4_scan_kernel(const uint32_t *hist, uint32_t *rstart, uint32_t *n_rounds,
                                                        GDesc *desc) {
    __shared__ uint32_t tile[4096];
    __shared__ uint32_t part[1024];
    const uint32_t t = threadIdx.x;
    const uint32_t nbins = hist[kGSoloKey + 1u] + 1u;  // non-solo bins [0, max]
    uint32_t carry = 0;
    for (uint32_t t0 = 0; t0 < nbins; t0 += 4096u) {
        for (uint32_t k = t; k < 4096u; k += 1024u) {
            const uint32_t c = t0 + k < nbins ? hist[t0 + k] : 0u;
            tile[k] = (c + 7u) / 8u;  // rounds of the bin
        }
        __syncthreads();
        const uint32_t r0 = tile[4 * t], r1 = tile[4 * t + 1], r2 = tile[4 * t + 2], r3 = tile[4 * t + 3];
        const uint32_t sum = r0 + r1 + r2 + r3;
        part[t] = sum;
        __syncthreads();
        for (uint32_t off = 1; off < 1024u; off <<= 1) {  // inclusive Hillis-Steele scan
            const uint32_t v = t >= off ? part[t - off] : 0u;
            __syncthreads();
            part[t] += v;
            __syncthreads();
        }
        const uint32_t ex = carry + part[t] - sum;
        const uint32_t b = t0 + 4 * t;
        const uint32_t st4[4] = {ex, ex + r0, ex + r0 + r1, ex + r0 + r1 + r2};
        for (uint32_t j = 0; j < 4u; j++) {
            if (b + j >= nbins) break;
            rstart[b + j] = st4[j];
            const uint32_t c = hist[b + j];
            if (c & 7u) gv4_null_groups(desc, (uint64_t)st4[j] + c / 8u, c & 7u);
        }
        carry += part[1023];
        __syncthreads();  // part / tile reused by the next tile
    }
    if (t == 0) {  // solo blocks (>= kGSoloKey steps, any K): one round each, after all others
        rstart[kGSoloKey] = carry;
        n_rounds[0] = carry + hist[kGSoloKey];
        n_rounds[1] = 0;  // crc_gv4_kernel's round counter (GV4Args::deal)
    }
    for (uint32_t j = t; j < hist[kGSoloKey]; j += 1024u) gv4_null_groups(desc, (uint64_t)carry + j, 1u);
}

__device__ __forceinline__ void gv4_put(GDesc *desc, const uint32_t *rstart, uint32_t b, uint32_t r, uint64_t p,
                                        uint64_t d, uint32_t idx, uint32_t K) {
    const uint64_t round = (uint64_t)rstart[b] + (b == kGSoloKey ? r : r / 8u);
    const uint32_t grp = b == kGSoloKey ? 0u : r % 8u;
    GDesc g;
    g.pd = p | (d << 56);
    g.idx = idx;
    g.K = K;
    desc[round * 8u + grp] = g;
}

constexpr uint32_t kSplitBin = 0xfffffffeu;  // place kernel: a split block (its chunks go to their bins)

__global__ __launch_bounds__(1024) void gv4_place_kernel(KParams P, GSplit S, const uint32_t *rstart, uint32_t *cursor,
                                                         GDesc *desc) {
    __shared__ uint32_t h[kLdsBins];
    __shared__ uint32_t base[kLdsBins];
    for (uint32_t b = threadIdx.x; b < kLdsBins; b += blockDim.x) h[b] = 0;
    __syncthreads();
    uint64_t i0, i1;
    gv4_chunk(P.n, i0, i1);
    // pass 1: ranks inside the chunk (LDS bins) or final ranks (global bins)
    constexpr int kMaxPer = 4;  // items per thread held in registers (chunk <= 4 * 1024)
    uint32_t rank[kMaxPer], bin[kMaxPer];
#pragma unroll
    for (int k = 0; k < kMaxPer; k++) {
        const uint64_t i = i0 + (uint64_t)k * blockDim.x + threadIdx.x;
        bin[k] = 0xffffffffu;
        if (i < i1) {
            uint64_t p;
            uint32_t n, cs, m;
            gv4_block(P, i, p, n);
            bin[k] = gv4_in_range(P, i) && gv4_split_geom(P, S, n, cs, m) && S.bigbase[i] != 0xffffffffu
                         ? kSplitBin
                         : gv4_bin(P, i, false);
        }
        rank[k] = wave_rank(bin[k] == kSplitBin ? 0xffffffffu : bin[k], h, cursor);
    }
    __syncthreads();
    // reserve the chunk's ranks in every LDS bin with one global atomic
    for (uint32_t b = threadIdx.x; b < kLdsBins; b += blockDim.x)
        base[b] = h[b] ? atomicAdd(&cursor[b], h[b]) : 0u;
    __syncthreads();
#pragma unroll
    for (int k = 0; k < kMaxPer; k++) {
        const uint32_t b = bin[k];
        if (b == 0xffffffffu) continue;
        const uint64_t i = i0 + (uint64_t)k * blockDim.x + threadIdx.x;
        uint64_t p;
        uint32_t n;
        gv4_block(P, i, p, n);
        if (b == kSplitBin) {  // chunks 0..m-2 of cs bytes and the last one, each its own group
            uint32_t cs, m;
            gv4_split_geom(P, S, n, cs, m);
            const GChunks c = gv4_chunks(p, n, cs, m);
            const uint32_t part0 = S.bigbase[i];
            const uint32_t bF = gv4_key(c.kF, c.dF), bL = gv4_key(c.kL, c.dL);
            const uint32_t rF = m > 1u ? atomicAdd(&cursor[bF], m - 1u) : 0u, rL = atomicAdd(&cursor[bL], 1u);
            for (uint32_t j = 0; j + 1u < m; j++)
                gv4_put(desc, rstart, bF, rF + j, p + (uint64_t)j * cs, c.dF, kGPart | (part0 + j), c.kF);
            gv4_put(desc, rstart, bL, rL, p + (uint64_t)(m - 1u) * cs, c.dL, kGPart | (part0 + m - 1u), c.kL);
            continue;
        }
        const uint32_t r = b < kLdsBins ? base[b] + rank[k] : rank[k];
        const uint32_t K = gv4_K(p, n);
        gv4_put(desc, rstart, b, r, p, (uint64_t)K * 128u - (p & 127u) - n, (uint32_t)i, K);
    }
}

hipError_t launch_gv4_rounds(const KParams &P, const GSplit &S, uint32_t *hist, uint32_t *cursor, uint32_t *rstart,
                             GDesc *desc, uint32_t *n_rounds, hipStream_t st) {
    // chunks of <= 4 * 1024 blocks (gv4_place_kernel keeps 4 per thread in registers)
    const uint64_t grid = (P.n + 4095) / 4096;
    if (grid > 0x7fffffffu) return hipErrorInvalidValue;
    hipLaunchKernelGGL(gv4_hist_kernel, dim3((unsigned)grid), dim3(1024), 0, st, P, S, hist);
    hipLaunchKernelGGL(gv4_scan_kernel, dim3(1), dim3(1024), 0, st, hist, rstart, n_rounds, desc);
    hipLaunchKernelGGL(gv4_place_kernel, dim3((unsigned)grid), dim3(1024), 0, st, P, S, rstart, cursor, desc);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Split blocks: state(A || B) = z^|B|(state(A)) ^ state_0(B) over GF(2), where
// state_0 starts from 0 and z^L, L zero bytes, is applied bit by bit of L with
// the z^(2^k) nibble tables in aux.  One wave per split block: lane t folds its
// consecutive chunks, a 6-level tree folds the lanes, lane 0 adds the init
// (update(~init, D) = z^|D|(~init) ^ state_0(D)), the suffix byte and the mask.
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t gv4_zpow(const uint32_t *aux, uint32_t s, uint32_t L) {
    while (L) {
        const uint32_t *t = aux + kAuxZpowDword + 128u * (uint32_t)__builtin_ctz(L);
        uint32_t r = 0;
#pragma unroll
        for (int q = 0; q < 8; q++) r ^= t[16 * q + ((s >> (4 * q)) & 15u)];
        s = r;
        L &= L - 1u;
    }
    return s;
}

__global__ __launch_bounds__(64) void gv4_combine_kernel(KParams P, GSplit S, const uint32_t *parts) {
    const uint32_t t = threadIdx.x;
    const uint64_t nbig = S.ctl[1];
    for (uint64_t bi = blockIdx.x; bi < nbig; bi += gridDim.x) {
        const GBig g = S.big[bi];
        uint64_t p;
        uint32_t n, cs, m;
        gv4_block(P, g.i, p, n);
        gv4_split_geom(P, S, n, cs, m);
        const uint32_t L = n - (m - 1u) * cs;
        const uint32_t per = (m + 63u) / 64u, c0 = t * per, c1 = c0 + per < m ? c0 + per : m;
        uint32_t s = 0, bytes = 0;
        for (uint32_t c = c0; c < c1; c++) {
            const uint32_t len = c + 1u == m ? L : cs;
            s = gv4_zpow(P.aux, s, len) ^ parts[g.part0 + c];
            bytes += len;
        }
        for (uint32_t off = 1; off < 64u; off <<= 1) {
            const uint32_t so = (uint32_t)__shfl_down((int)s, off), bo = (uint32_t)__shfl_down((int)bytes, off);
            if ((t & (2u * off - 1u)) == 0u && t + off < 64u) {
                s = gv4_zpow(P.aux, s, bo) ^ so;
                bytes += bo;
            }
        }
        if (t == 0u) {
            uint32_t st = gv4_zpow(P.aux, ~(P.init ? P.init[g.i] : 0u), n) ^ s;
            if (P.suffix) st = (st >> 8) ^ P.aux[(st ^ P.suffix[g.i]) & 0xffu];
            const uint32_t crc = ~st;
            P.out32[g.i] = (P.flags & 1u) ? mask_crc(crc) : crc;
        }
    }
}

hipError_t launch_gv4_combine(const KParams &P, const GSplit &S, const uint32_t *parts, hipStream_t st) {
    hipLaunchKernelGGL(gv4_combine_kernel, dim3(1024), dim3(64), 0, st, P, S, parts);
    return hipGetLastError();
}
#endif

}  // namespace jlk
