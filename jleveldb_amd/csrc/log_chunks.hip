// log_chunks.hip — WAL / MANIFEST verification without a global sort or a host
// round trip: LogReader.readPhysicalRecord (J/db/LogReader.java:297-383) over
// every 32 KiB block, the record crcs through crc_gv4_kernel<MODE_LOG_CHUNK>.
//
//   lc_walk     one thread per 32 KiB block follows the header chain (the
//               reference's decisions, in its order), keeps the first
//               kLCSlots events of the block (with the stored crc) and counts,
//               per workgroup of 256 blocks, the record CHUNKS by window count
//   (scans)     event starts per block; chunk ranks per (bin, workgroup)
//   lc_setup    first round of every bin, the empty groups of partial rounds
//   lc_build    events in file order; every chunk's descriptor at its round
//               (deterministic: a workgroup owns a contiguous rank range per bin)
//   gv4         rounds of 8 chunks of one window count K on the 128-B grid
//   lc_combine  records of several chunks: fold the chunk states, compare
//   lc_apply    the block's first failing record becomes BAD_CRC and its later
//               events kind 0 (the reader drops the rest of the block, :359-367)
//
// Chunks.  A record's crc range [h + 6, h + 7 + len) (type byte || payload,
// J/db/LogWriter.java:147) of n bytes starting at p covers K = ceil((f + n)/128)
// windows of the 128-B grid (f = p & 127, tail pad r = 128K - f - n).  It is cut
// into J = ceil(K/kLCWin) chunks of kLCWin windows, the last one K - kLCWin(J-1):
// chunk 0 is seeded with W0 = slice4^-1(0xffffffff) (value()'s init) before p,
// the others start from state 0; the last one's tail pad is r, the others end
// on a window edge.  With the chunk states s_j (positioned at their ends),
//   state(record) = s_{J-1} ^ XOR_{j < J-1} z^(f + n - 4096 (j+1)) (s_j),
// the shifts applied from the z^(128 a) and z^b nibble tables in aux.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "engine_device.hpp"

namespace jlk {

constexpr uint32_t kAuxZWDword = 5648;             // must equal jlmath::kAuxZW
constexpr uint32_t kAuxZBDword = 5648 + 256 * 128;  // jlmath::kAuxZB

// Window count, tail pad and chunk count of a crc range at absolute address pa.
struct LCGeom {
    uint32_t f, K, r, J;
};
__device__ __forceinline__ uint32_t lc_bin(uint32_t K, uint32_t d) { return (K - 1u) * 16u + (d & 15u); }
// Round of the j-th round of bin (K, d): the bins' rounds in bin order (rs:
// kLCBins + 1 round starts, saturating: the total is clamped past the descriptor
// capacity).  r3 interleaved the rounds of one K over its 16 d bins so that
// neighbouring records sit in adjacent rounds (their shared boundary lines from
// L2): slower; on the branch study-r4-switches.
__device__ __forceinline__ uint64_t lc_round(const uint32_t *rs, uint32_t K, uint32_t d, uint32_t j) {
    return (uint64_t)rs[lc_bin(K, d)] + j;
}
__device__ __forceinline__ LCGeom lc_geom(uint64_t pa, uint32_t n) {
    LCGeom g;
    g.f = (uint32_t)(pa & 127u);
    g.K = (g.f + n + 127u) >> 7;
    g.r = 128u * g.K - g.f - n;
    g.J = (g.K + kLCWin - 1u) / kLCWin;
    return g;
}

// One header decision of readPhysicalRecord at p (block [bs, be), eof: the
// file's last, short block).  w = header bytes 3..6 ([crc3][len lo][len hi][type]).
struct LCDecision {
    uint32_t kind, length, type;
    bool stop;
};
__device__ __forceinline__ LCDecision lc_decide(uint64_t rem, bool eof, uint32_t w) {
    // w: header bytes 3..6 ([crc3][len lo][len hi][type])
    LCDecision d{0u, 0u, 0u, false};
    if (rem < 7) {  // :315-322 (fewer than kHeaderSize bytes left)
        d.kind = (eof && rem > 0) ? 6u : 0u;
        d.stop = true;
        return d;
    }
    d.length = (w >> 8) & 0xffffu;
    d.type = w >> 24;
    if (7u + (uint64_t)d.length > rem) {  // :334-345
        d.kind = eof ? 5u : 3u;
        d.stop = true;
    } else if (d.type == 0 && d.length == 0) {  // :347-353
        d.kind = 4u;
        d.stop = true;
    } else {
        d.kind = 1u;
    }
    return d;
}

__device__ __forceinline__ uint32_t ld_u32u(const uint8_t *p) { return *(const u32u *)p; }
typedef uint64_t __attribute__((aligned(1))) u64u;

// Header bytes 0..6 at p ([crc 0..3][len lo][len hi][type]) as one 8-byte load
// when 8 bytes are left in the block (one memory request on the walk's serial
// chain), else two dword loads.
// Cache policy of lc_walk's header hops: nt.  r3 same-box A/B (tools/ab_lib.sh, 3
// rounds): C5 1 056-B 1.034 -> 1.011 ms with nt (and with sc0 sc1 nt), mixed and
// DBBench unchanged within noise; sc1 / sc0 sc1 alone no change.  The walk's
// random header lines are not re-read soon (the rounds read the records much
// later), so they should not displace L2-resident lines.
__device__ __forceinline__ uint64_t lc_header(const uint8_t *p, uint64_t rem) {
    if (rem >= 8) return *(const u64u *)p;
    return (uint64_t)ld_u32u(p) | ((uint64_t)(ld_u32u(p + 3) >> 8) << 32);
}
// Events, round descriptors and stash entries use the default cache policy: r3
// same-box A/B (tools/ab_lib.sh, C5 sets mixed / 1 056-B / DBBench, ms): default
// 0.82 / 1.014 / 1.59, non-temporal 0.825 / 1.035 / 1.587 (gv4 then reads its
// descriptors from HBM).
typedef uint32_t lc_v4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void lc_st16(void *p, lc_v4 v) { *(lc_v4 *)p = v; }
__device__ __forceinline__ uint64_t lc_ld8(const uint64_t *p) { return *p; }
// the walk's hop load (lc_walk): lc_header's bytes as a non-temporal asm load,
// waited for at once (the hop is a dependent chain anyway)
__device__ __forceinline__ uint64_t lc_hop(const uint8_t *p, uint64_t rem) {
    if (rem >= 8) {
        uint64_t v;
        asm volatile("global_load_dwordx2 %0, %1, off nt\n\ts_waitcnt vmcnt(0)" : "=v"(v) : "v"(p) : "memory");
        return v;
    }
    return lc_header(p, rem);
}

// Exclusive prefix sum over the wave's 64 lanes with DPP only (no LDS
// crossbar round trips): Hillis-Steele inside each row of 16 (row_shr 1/2/4/8),
// then the row totals through row_bcast:15 (rows 1, 3) and row_bcast:31 (rows
// 2, 3).  Lanes without a source add the `old` operand, 0.  All lanes active.
__device__ __forceinline__ uint32_t lc_wave_excl_sum(uint32_t v) {
    uint32_t x = v;
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, false);  // row_shr:1
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, false);  // row_shr:2
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, false);  // row_shr:4
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, false);  // row_shr:8
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xa, 0xf, false);  // row_bcast:15
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xc, 0xf, false);  // row_bcast:31
    return x - v;
}

// Adds one (s = 1) or removes one (s = ~0u) record of geometry g to the chunk
// histogram of its walk group: its chunks by bin, plus one multi-chunk record
// and its J parts when J > 1.
__device__ __forceinline__ void lc_hist(uint32_t *h, const LCGeom &g, uint32_t s) {
    if (g.J == 1u) {
        atomicAdd(&h[lc_bin(g.K, g.r)], s);
    } else {
        atomicAdd(&h[lc_bin(kLCWin, 0u)], (g.J - 1u) * s);
        atomicAdd(&h[lc_bin(g.K - kLCWin * (g.J - 1u), g.r)], s);
        atomicAdd(&h[kLCBig], s);
        atomicAdd(&h[kLCPart], g.J * s);
    }
}

// lc_hist into the global histogram of group grp (lc_dense: a dense block's long
// records, after lc_walk wrote the groups' counts and before lc_scan reads them)
__device__ __forceinline__ void lc_hist_global(const LCArgs &A, uint64_t grp, const LCGeom &g) {
    uint32_t *h = A.hist + grp;
    const uint64_t nw = A.n_grp;
    if (g.J == 1u) {
        atomicAdd(&h[lc_bin(g.K, g.r) * nw], 1u);
    } else {
        atomicAdd(&h[lc_bin(kLCWin, 0u) * nw], g.J - 1u);
        atomicAdd(&h[lc_bin(g.K - kLCWin * (g.J - 1u), g.r) * nw], 1u);
        atomicAdd(&h[kLCBig * nw], 1u);
        atomicAdd(&h[kLCPart * nw], g.J);
    }
}

// Walk groups of kLCGroup consecutive blocks, one per wave (4 per workgroup).
// The walk also initialises what later kernels accumulate into (first_bad,
// count[n_blocks], the scan's zero tail, cap_flag, the stash counter): no memsets.
//
// Latency: a block's headers form a chain of dependent loads, so the walk is
// one DRAM round trip per record.  The first kLCLdsSlots events of a block are
// buffered in LDS and written out after the walk: a global store in the loop
// makes every hop also wait for the store's acknowledgement (gfx9 counts stores
// in vmcnt, and the compiler waits vmcnt(0) with a store outstanding).
constexpr uint32_t kLCLdsSlots = 34;
__global__ __launch_bounds__(256) void lc_walk_kernel(LCArgs A) {
    __shared__ uint32_t h[4][kLCCounters];
    __shared__ uint64_t ls[256][kLCLdsSlots + 1];  // [thread][slot], padded: the write-back reads it in order
    const uint32_t wv = threadIdx.x >> 6;
    for (uint32_t i = threadIdx.x; i < 4 * kLCCounters; i += 256u) (&h[0][0])[i] = 0;
    __syncthreads();
    const uint32_t wg = blockIdx.x;
    const uint64_t b = (uint64_t)wg * 256u + threadIdx.x;
    if (b == 0) {
        A.count[A.n_blocks] = 0;
        // the work counters later kernels take ids from must be zero (lc_finish of the
        // verification before re-zeroes them; the host memsets them after a call that
        // stopped early): stale ones would start lc_dense / gv4 / lc_scan past their
        // work, so they are reported instead
        *A.cap_flag = (A.dense_ctr[1] | A.dense_ctr[2] | A.dense_ctr[3]) ? kLCFlagStale : 0u;
        *A.stash_ctr = 0;
    }
    uint32_t cnt = 0;
    bool listed = false;   // a dense block: appended to lc_dense's list below
    bool uniform = false;  // ... whose last walked records are equal (kDWUniform in its list entry)
    if (b < (A.n_blocks + kLSTile) / kLSTile) {  // the scans' look-back statuses, the placement's tile tags
        A.tstat[b] = A.tstat0[b] = 0;
        A.ready0[b] = 0;
    }
    if (b < A.n_blocks) {
        if (A.checksum) A.first_bad[b] = kLCNone;
        A.nlong[b] = 0;  // lc_dense's deferred long records
        const uint64_t bs = b * 32768u, be = bs + 32768u < A.size ? bs + 32768u : A.size;
        const bool eof = be - bs < 32768u;
        const uint64_t base = (uint64_t)(uintptr_t)A.log;
        uint64_t p = bs;
        uint64_t hv = be - p >= 7 ? lc_hop(A.log + p, be - p) : 0;
        bool dense = false;
        for (;;) {
            const LCDecision d = lc_decide(be - p, eof, (uint32_t)(hv >> 24));
            if (d.kind == 0) break;  // the block's trailer: no event
            // dense: a (kLCSlots + 1)-th event, or kLCProbe events within kLCProbe * 512 B
            if (cnt == kLCSlots || (cnt == kLCProbe && p - bs < kLCProbe * 512u)) {
                dense = true;
                break;
            }
            const uint64_t pn = p + 7u + d.length;
            const uint32_t stored = (uint32_t)hv;
            if (!d.stop && be - pn >= 7) hv = lc_hop(A.log + pn, be - pn);
            const uint64_t slot = d.length | (d.type << 16) | (d.kind << 24) | ((uint64_t)stored << 32);
            if (cnt < kLCLdsSlots) ls[threadIdx.x][cnt] = slot;
            else A.slots[b * kLCSlots + cnt] = slot;
            // chunk histogram: exactly the chunks lc_build places
            if (d.kind == 1u && A.checksum) lc_hist(h[wv], lc_geom(base + p + 6u, 1u + d.length), 1u);
            cnt++;
            if (d.stop) break;
            p = pn;
        }
        A.dense_off[b] = kLCNotDense;
        if (dense) {
            // lc_dense verifies the block and counts its events; the chunks of the
            // events walked so far leave the histogram again (only blocks of short
            // records take this second look at their slots)
            if (A.checksum) {
                uint64_t q = bs;
                for (uint32_t j = 0; j < cnt; j++) {
                    const uint64_t s = j < kLCLdsSlots ? ls[threadIdx.x][j] : A.slots[b * kLCSlots + j];
                    const uint32_t len = (uint32_t)s & 0xffffu;
                    if ((((uint32_t)s >> 24) & 0xffu) == 1u) lc_hist(h[wv], lc_geom(base + q + 6u, 1u + len), ~0u);
                    q += 7u + len;
                }
            }
            atomicAdd(&h[wv][kLCOver], 1u);
            // a block whose last kDWProbe walked records are equal (DBBench's) is left
            // to lc_dense's walk, whose trips measure such runs; the others are
            // walked by lc_dwalk first
            uniform = cnt >= kDWProbe + 1u;
            const uint64_t s0 = cnt - 1u < kLCLdsSlots ? ls[threadIdx.x][cnt - 1u] : A.slots[b * kLCSlots + cnt - 1u];
            for (uint32_t j = cnt - kDWProbe; uniform && j + 1u < cnt; j++) {
                const uint64_t sj = j < kLCLdsSlots ? ls[threadIdx.x][j] : A.slots[b * kLCSlots + j];
                uniform = (uint32_t)sj == (uint32_t)s0;
            }
            uniform = uniform && (((uint32_t)s0 >> 24) & 0xffu) == 1u;
            // the block's events, predicted (lc_dwalk predicts the others): the run to
            // the block's end, then the record that fills it (the writer's FIRST
            // fragment, J/db/LogWriter.java:100-118) or the trailer.  lc_dwalk checks two
            // headers of it when it matters (in-place events, lc_dense)
            if (uniform) {
                const uint32_t L = 7u + ((uint32_t)s0 & 0xffffu), left = (uint32_t)(be - p), rem = left % L;
                cnt += left / L + (rem >= 7u || (eof && rem > 0u) ? 1u : 0u);
                A.dw_info[b] = (uint32_t)(p - bs) | (L << 16);  // (lc_dense reads no dw_info of a run block)
            } else {
                cnt = kLCDense;
            }
            A.pred[b] = cnt;
            listed = true;
        }
        A.count[b] = cnt;
    }
    // the dense blocks into lc_dense's list: the waves' counts summed in LDS, one
    // global atomic per workgroup that has any (one per wave cost the DBBench set's
    // walk ~20 us: 2 048 atomics on one address at the same moment)
    __shared__ uint32_t s_dn, s_db, s_nu;
    if (threadIdx.x == 0) s_dn = s_nu = 0;
    __syncthreads();
    const uint64_t dm = __builtin_amdgcn_ballot_w64(listed);
    const uint64_t nm = __builtin_amdgcn_ballot_w64(listed && !uniform);  // lc_dwalk's blocks
    const uint32_t lane = threadIdx.x & 63u;
    uint32_t woff = 0;
    if (dm && lane == 0) woff = atomicAdd(&s_dn, (uint32_t)__builtin_popcountll(dm));
    if (nm && lane == 0) atomicAdd(&s_nu, (uint32_t)__builtin_popcountll(nm));
    woff = (uint32_t)__builtin_amdgcn_readfirstlane((int)woff);
    __syncthreads();
    if (threadIdx.x == 0 && s_dn) s_db = atomicAdd(&A.dense_ctr[0], s_dn);
    if (threadIdx.x == 0 && s_nu) atomicAdd(A.nu_ctr, s_nu);
    __syncthreads();
    if (listed)
        A.dense_list[s_db + woff + (uint32_t)__builtin_popcountll(dm & ((1ull << lane) - 1ull))] =
            (uint32_t)b | (uniform ? kDWUniform : 0u);
    // the LDS slots out, the workgroup's 256 blocks together: consecutive threads
    // store a block's consecutive slots (a run of kLCLdsSlots x 8 B per block; one
    // thread per block writing its own slots touched 64 lines per store, 33 us of
    // the C5 walk).  Slots past a block's count are never read.
    // Only the slots lc_build reads: a dense block's (lc_dense re-walks it) and the
    // slots past a block's count are skipped (r5: the DBBench set's walk wrote
    // 36 MB of abandoned slots).
    __shared__ uint32_t s_used[256];
    s_used[threadIdx.x] = listed ? 0u : cnt;
    __syncthreads();
    const uint64_t b0 = (uint64_t)wg * 256u;
    for (uint32_t e = threadIdx.x; e < 256u * kLCLdsSlots; e += 256u) {
        const uint32_t t = e / kLCLdsSlots, j = e - t * kLCLdsSlots;
        if (b0 + t < A.n_blocks && j < s_used[t]) A.slots[(b0 + t) * kLCSlots + j] = ls[t][j];
    }
    const uint64_t g0 = (uint64_t)wg * 4u;
    for (uint32_t i = threadIdx.x; i < 4 * kLCCounters; i += 256u) {
        const uint32_t g = i % 4u, c = i / 4u;  // 4 consecutive groups of one counter: one 16-B run
        if (g0 + g < A.n_grp) A.hist[(uint64_t)c * A.n_grp + g0 + g] = h[g][c];
    }
}

// The two scans of a verification in one launch (r4; before, two rocprim scans,
// ~24 us on every C5 set):
//   * workgroups [0, tiles): start = exclusive scan of count[0 .. n_blocks] (u32 ->
//     u64), tiles of kLSTile with a decoupled look-back (tstat, zeroed by lc_walk);
//   * the next kLCCounters: counter c's row of hist (its per-group counts) scanned
//     on its own, hscan[c n_grp + g] = the groups before g, rowtot[c] = the row's
//     total — all that lc_setup / lc_build / lc_combine / lc_finish use (a scan
//     across the rows gave the same numbers as differences).
// Tile / row chunks pass through LDS (coalesced loads and stores); every thread
// scans 16 consecutive values, the 256 thread totals by wave DPP sums.
__device__ __forceinline__ uint32_t ls_block_excl(uint32_t v, uint32_t *wsum, uint32_t *total) {
    const uint32_t t = threadIdx.x, lane = t & 63u, wv = t >> 6;
    const uint32_t ex = lc_wave_excl_sum(v);
    if (lane == 63u) wsum[wv] = ex + v;
    __syncthreads();
    uint32_t before = 0, tot = 0;
    for (uint32_t w = 0; w < 4u; w++) {
        before += w < wv ? wsum[w] : 0u;
        tot += wsum[w];
    }
    *total = tot;
    __syncthreads();  // wsum reused by the next call
    return before + ex;
}
constexpr uint32_t kLSPer = kLSTile / 256u;  // values per thread
static_assert(kLSTile % 256u == 0u, "kLSTile: a multiple of the workgroup");
// One tile of kLSTile event starts (lc_scan; and lc_dwalk's first placement over
// the predicted counts, r6): out[i] = the events of blocks [0, i), decoupled
// look-back over the tiles' statuses (tstat, zeroed by lc_walk).
// ready non-null (lc_dense's placement, read by other workgroups of the same
// kernel): out[] by agent-scope atomic stores, then ready[id] = A.gen.
__device__ __forceinline__ void ls_tile(const LCArgs &A, uint32_t id, uint64_t *tstat, uint64_t *out, uint32_t *buf,
                                        uint32_t *wsum, unsigned long long *s_pre, uint32_t *ready = nullptr) {
    const uint32_t t = threadIdx.x;
    const uint64_t k = id, base = k * kLSTile, n = (uint64_t)A.n_blocks + 1u;
    for (uint32_t j = t; j < kLSTile; j += 256u) buf[j] = base + j < n ? A.count[base + j] : 0u;
    __syncthreads();
    uint32_t v[kLSPer], s = 0;
#pragma unroll
    for (uint32_t j = 0; j < kLSPer; j++) {
        v[j] = buf[kLSPer * t + j];
        s += v[j];
    }
    uint32_t agg;
    const uint32_t ex = ls_block_excl(s, wsum, &agg);
    if (t == 0) {
        uint64_t P = 0;
        if (k == 0) {
            __hip_atomic_store(&tstat[0], kLDInc | agg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else {
            __hip_atomic_store(&tstat[k], kLDAgg | agg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            for (int64_t q = (int64_t)k - 1; q >= 0; q--) {
                uint64_t w;
                while ((w = __hip_atomic_load(&tstat[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) == 0)
                    __builtin_amdgcn_s_sleep(1);
                P += w & kLDVal;
                if (w & kLDInc) break;
            }
            __hip_atomic_store(&tstat[k], kLDInc | (P + agg), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        *s_pre = P;
    }
    __syncthreads();
    const uint64_t pre = *s_pre;
    uint32_t run = ex;
#pragma unroll
    for (uint32_t j = 0; j < kLSPer; j++) {  // exclusive values back into LDS, in place
        buf[kLSPer * t + j] = run;
        run += v[j];
    }
    __syncthreads();
    for (uint32_t j = t; j < kLSTile; j += 256u) {
        if (base + j >= n) continue;
        if (ready) __hip_atomic_store(&out[base + j], pre + buf[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        else out[base + j] = pre + buf[j];
    }
    if (ready) {
        __syncthreads();  // every thread's stores done
        if (t == 0) __hip_atomic_store(&ready[id], A.gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// Work ids come from a counter in dispatch order (dense_ctr[3], zero when
// lc_walk starts), not from blockIdx.x: tile k's look-back spins on tiles k - 1 ..., so
// it must not run before they have started, which a blockIdx order would only
// assume of the hardware's dispatch (rocPRIM takes its tile ids the same way).
__global__ __launch_bounds__(256) void lc_scan_kernel(LCArgs A) {
    __shared__ uint32_t buf[kLSTile];
    __shared__ uint32_t wsum[4];
    __shared__ unsigned long long s_pre;
    __shared__ uint32_t s_id;
    const uint32_t t = threadIdx.x;
    const uint32_t tiles = (A.n_blocks + kLSTile) / kLSTile;  // n_blocks + 1 values
    // the hist rows (independent) are workgroups [0, kLCCounters); only the tiles
    // take ordered ids (one atomic per tile, not per workgroup)
    if (blockIdx.x >= kLCCounters) {
        if (t == 0) s_id = atomicAdd(&A.dense_ctr[3], 1u);
        __syncthreads();
    }
    const uint32_t id = blockIdx.x >= kLCCounters ? s_id : tiles + blockIdx.x;
    if (id < tiles) {
        ls_tile(A, id, A.tstat, A.start, buf, wsum, &s_pre);
        return;
    }
    const uint32_t c = id - tiles;  // a hist row
    const uint64_t nw = A.n_grp, row = (uint64_t)c * nw;
    uint32_t carry = 0;
    for (uint64_t g0 = 0; g0 < nw; g0 += kLSTile) {
        for (uint32_t j = t; j < kLSTile; j += 256u) buf[j] = g0 + j < nw ? A.hist[row + g0 + j] : 0u;
        __syncthreads();
        uint32_t v[kLSPer], s = 0;
#pragma unroll
        for (uint32_t j = 0; j < kLSPer; j++) {
            v[j] = buf[kLSPer * t + j];
            s += v[j];
        }
        uint32_t tot;
        uint32_t run = carry + ls_block_excl(s, wsum, &tot);
#pragma unroll
        for (uint32_t j = 0; j < kLSPer; j++) {
            buf[kLSPer * t + j] = run;
            run += v[j];
        }
        __syncthreads();
        for (uint32_t j = t; j < kLSTile; j += 256u)
            if (g0 + j < nw) A.hscan[row + g0 + j] = buf[j];
        carry += tot;
        __syncthreads();  // buf reused
    }
    if (t == 0) A.rowtot[c] = carry;
}

// rstart[k] = rounds of the bins before k (ceil(count/8) rounds each; bin k =
// chunks of K = k/16 + 1 windows with tail pads d = k mod 16 (mod 16)),
// rstart[kLCBins] = all rounds (clamped to the descriptor capacity, cap_flag set
// past it); the missing groups of every bin's last round are marked empty.
__global__ __launch_bounds__(kLCBins) void lc_setup_kernel(LCArgs A) {
    __shared__ uint32_t wsum[kLCBins / 64];
    const uint32_t k = threadIdx.x, lane = k & 63u, wv = k >> 6;
    const uint32_t cnt = A.rowtot[k];
    const uint32_t rounds = (cnt + 7u) / 8u;
    uint32_t incl = rounds;  // inclusive scan: waves, then across the 8 wave sums
    for (uint32_t o = 1; o < 64u; o <<= 1) {
        const uint32_t v = (uint32_t)__shfl_up((int)incl, o);
        if (lane >= o) incl += v;
    }
    if (lane == 63u) wsum[wv] = incl;
    __syncthreads();
    uint32_t before = 0, total = 0;
    for (uint32_t w = 0; w < kLCBins / 64; w++) {
        before += w < wv ? wsum[w] : 0u;
        total += wsum[w];
    }
    const uint32_t ex = before + incl - rounds;
    A.rstart[k] = ex;
    if (k == 0) {
        const bool over = total > A.round_cap;
        A.rstart[kLCBins] = over ? (uint32_t)A.round_cap : total;
        if (over) atomicOr(A.cap_flag, kLCFlagCapacity);
    }
    const uint64_t r = (uint64_t)ex + cnt / 8u;
    if (cnt & 7u) {
        if (r < A.round_cap)
            for (uint32_t g = cnt & 7u; g < 8u; g++) A.desc[r * 8u + g].idx = kGNull;
    }
}

__device__ __forceinline__ void lc_desc(const LCArgs &A, const uint32_t *rs, uint32_t K, uint32_t rank, uint64_t prel,
                                        uint32_t seed, uint32_t d, uint32_t idx, uint32_t stored) {
    const uint64_t round = lc_round(rs, K, d, rank / 8u);
    if (round >= A.round_cap) return;  // cap_flag is set (lc_setup)
    const uint64_t pd = (prel & 0xffffffffffull) | ((uint64_t)K << 40) | ((uint64_t)seed << 48) | ((uint64_t)d << 56);
    lc_st16(&A.desc[round * 8u + rank % 8u], lc_v4{(uint32_t)pd, (uint32_t)(pd >> 32), idx, stored});
}

__device__ __forceinline__ uint32_t lc_wave_excl_sum(uint32_t v);
constexpr uint32_t kLDLinkKind = 0xffu;  // stash entry kind of a segment link (lc_dense)

// The chunk descriptors of one OK record per lane (ok false: none), all lanes
// calling.  Ranks come from LDS atomics per lane: with bins by (K, d mod 16) a
// wave's records spread over many bins, so ballot aggregation would loop once
// per distinct bin.  A one-chunk record places its descriptor from its own lane; the
// chunks of longer records are spread over the wave's lanes (lane c takes
// chunk c of the wave's chunk list, its record found by a binary search over
// the lanes' chunk offsets) instead of one lane placing its record's J chunks
// in turn.
__device__ __forceinline__ void lc_place_wave(const LCArgs &A, uint32_t *ctr, const uint32_t *rs, bool ok,
                                              uint64_t prel, uint32_t n, uint32_t stored) {
    const uint32_t lane = __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
    LCGeom g{0u, 0u, 0u, 0u};
    if (ok) g = lc_geom((uint64_t)(uintptr_t)A.log + prel, n);
    if (ok && g.J == 1u) lc_desc(A, rs, g.K, atomicAdd(&ctr[lc_bin(g.K, g.r)], 1u), prel, 1u, g.r, 0u, stored);
    const bool multi = ok && g.J > 1u;
    if (__builtin_amdgcn_ballot_w64(multi) == 0ull) return;
    uint32_t pi = 0, fits = 0;
    if (multi) {
        const uint32_t bi = atomicAdd(&ctr[kLCBig], 1u);
        pi = atomicAdd(&ctr[kLCPart], g.J);
        // past a capacity (cannot happen with the caller's bounds) the chunks still
        // take their ranks, as empty groups: no round of the table is left unwritten
        fits = bi < A.big_cap && (uint64_t)pi + g.J <= A.part_cap;
        if (fits) {
            LCBig big;
            big.p = prel;
            big.n = n;
            big.stored = stored;
            big.part0 = pi;
            big.J = g.J;
            A.big[bi] = big;
        } else {
            atomicOr(A.cap_flag, kLCFlagCapacity);
            if (bi < A.big_cap) A.big[bi].J = 0u;  // skipped by lc_combine
        }
    }
    const uint32_t m = multi ? g.J : 0u;
    const uint32_t off = lc_wave_excl_sum(m);
    const uint32_t total = (uint32_t)__builtin_amdgcn_readlane((int)(off + m), 63);
    for (uint32_t c0 = 0; c0 < total; c0 += 64u) {
        const uint32_t c = c0 + lane;
        uint32_t o = 0;  // the last lane whose chunk offset is <= c: chunk c's record
        for (uint32_t s = 32u; s; s >>= 1) {
            const uint32_t cand = o + s;
            if ((uint32_t)__shfl((int)off, (int)cand) <= c) o = cand;
        }
        const uint32_t j = c - (uint32_t)__shfl((int)off, (int)o);
        const uint32_t J = (uint32_t)__shfl((int)g.J, (int)o), Kr = (uint32_t)__shfl((int)g.K, (int)o);
        const uint32_t r = (uint32_t)__shfl((int)g.r, (int)o), f = (uint32_t)__shfl((int)g.f, (int)o);
        const uint32_t p0 = (uint32_t)__shfl((int)pi, (int)o), ft = (uint32_t)__shfl((int)fits, (int)o);
        const uint64_t pr = (uint64_t)(uint32_t)__shfl((int)(uint32_t)prel, (int)o) |
                            ((uint64_t)(uint32_t)__shfl((int)(uint32_t)(prel >> 32), (int)o) << 32);
        if (c < total) {
            const bool last = j + 1u == J;
            const uint32_t K = last ? Kr - kLCWin * j : kLCWin;
            const uint32_t d = last ? r : 0u;
            const uint32_t rank = atomicAdd(&ctr[lc_bin(K, d)], 1u);
            // chunks j >= 1 start on the grid, at the record's first window + 4096 j
            lc_desc(A, rs, K, rank, j ? pr - f + 4096ull * j : pr, j == 0u, d, ft ? kGPart | (p0 + j) : kGNull, 0u);
        }
    }
}

__device__ __forceinline__ void lc_event(const LCArgs &A, uint64_t at, uint64_t off, uint32_t length, uint32_t type,
                                         uint32_t kind) {
    if (at >= A.ev_cap) return;
    // LogEvent {u64 offset, u32 length, u8 type, u8 kind, u16 pad}
    lc_st16(&A.ev[at], lc_v4{(uint32_t)off, (uint32_t)(off >> 32), length, (type & 0xffu) | ((kind & 0xffu) << 8)});
}

// A workgroup builds the kLCGroup blocks one walk wave counted (their rank
// ranges per bin come from the scan): one wave per block at a time, lane j =
// event j (coalesced slot reads and event writes; the header offsets are the
// prefix sums of 7 + length over the lanes).
// 8 blocks per wave, all their loads issued first (r2: 8 waves x 8 blocks ran
// lc_build 77 -> 63 us against 4 x 16, C5 ~3 % faster; 16 x 4 about the same)
constexpr uint32_t kLCBuildWaves = 8;

// A dense block's events from its runs (lc_dense's stash segments): a wave takes
// 64 runs at a time (lane = run: its count, exclusive prefix over the lanes),
// then writes their events 64 at a time, lane = event, each finding its run by
// a binary search over the lanes' prefixes.  Event k of a run: header at offset
// + k (7 + length).
__device__ __forceinline__ void lc_expand_runs(const LCArgs &A, uint64_t b, uint64_t ev0, uint64_t doff, uint64_t e0) {
    const uint32_t lane = __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
    uint64_t so = doff & 0xffffffffffffull;
    uint32_t n = (uint32_t)(doff >> 48);
    uint64_t k0 = 0;  // events of the block written so far
    bool first = true;
    while (n) {
        uint32_t nn = 0;  // the next segment (a link in this one's last entry)
        uint64_t sn = 0;
        for (uint32_t r0 = 0; r0 < n; r0 += 64u) {
            // the first segment's first 64 entries came with the block's other loads (e0)
            const uint64_t e = r0 + lane < n ? (first ? e0 : lc_ld8(&A.stash[so + r0 + lane])) : 0ull;
            first = false;
            const bool link = r0 + lane < n && (e >> 56) == kLDLinkKind;
            const uint64_t lb = __builtin_amdgcn_ballot_w64(link);
            if (lb) {
                const uint32_t src = (uint32_t)__builtin_ctzll(lb);
                const uint64_t le = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(e >> 32), (int)src) << 32) |
                                    (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)e, (int)src);
                sn = le & 0xffffffffffull;
                nn = (uint32_t)(le >> 40) & 0xffffu;
            }
            const uint32_t cnt = r0 + lane < n && !link ? (uint32_t)(e >> 32) & 0xffffu : 0u;
            const uint32_t ex = lc_wave_excl_sum(cnt);
            const uint32_t tot = (uint32_t)__builtin_amdgcn_readlane((int)(ex + cnt), 63);
            if (__builtin_amdgcn_ballot_w64(cnt > 1u) == 0ull) {
                // runs of one record (lc_dwalk's blocks: records of random lengths):
                // event ex is this lane's own run, no search
                if (cnt) {
                    const uint32_t lo = (uint32_t)e, hi = (uint32_t)(e >> 32), len = lo >> 16;
                    lc_event(A, ev0 + k0 + ex, b * 32768u + (lo & 0xffffu), len, (hi >> 16) & 0xffu, hi >> 24);
                }
                k0 += tot;
                continue;
            }
            for (uint32_t c0 = 0; c0 < tot; c0 += 64u) {
                const uint32_t c = c0 + lane;
                uint32_t o = 0;  // the last lane whose prefix is <= c: event c's run
                for (uint32_t s = 32u; s; s >>= 1) {
                    const uint32_t cand = o + s;
                    if ((uint32_t)__shfl((int)ex, (int)cand) <= c) o = cand;
                }
                const uint32_t lo = (uint32_t)__shfl((int)(uint32_t)e, (int)o);
                const uint32_t hi = (uint32_t)__shfl((int)(uint32_t)(e >> 32), (int)o);
                const uint32_t eo = (uint32_t)__shfl((int)ex, (int)o);
                if (c < tot) {
                    const uint32_t len = lo >> 16;
                    lc_event(A, ev0 + k0 + c, b * 32768u + (lo & 0xffffu) + (uint64_t)(c - eo) * (7u + len), len,
                             (hi >> 16) & 0xffu, hi >> 24);
                }
            }
            k0 += tot;
        }
        so = sn;
        n = nn;
    }
}

// The last kernel of a verification (block 0, thread 0): the result words, and
// the work counters zeroed for the next verification of this workspace (no
// kernel of this one reads them after lc_build / gv4).
__device__ __forceinline__ void lc_finish(const LCArgs &A) {
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        A.result[0] = A.start[A.n_blocks];
        A.result[1] = A.rowtot[kLCOver];
        A.result[2] = *A.cap_flag;
        lc_st16(A.dense_ctr, lc_v4{0u, 0u, 0u, 0u});
        if (A.hint) *A.hint = *A.nu_ctr;  // the host's guess for the next verification's lc_dense
        lc_st16(A.dense_ctr + 4, lc_v4{0u, 0u, 0u, 0u});  // [6] nu_ctr, [7] lc_dwalk's blocks not predicted
    }
}

__global__ __launch_bounds__(64 * kLCBuildWaves) void lc_build_kernel(LCArgs A) {
    __shared__ uint32_t ctr[kLCCounters], rs[kLCBins + 1];
    const uint64_t nw = A.n_grp;
    for (uint32_t i = threadIdx.x; i < kLCCounters; i += blockDim.x)
        ctr[i] = A.checksum ? A.hscan[i * nw + blockIdx.x] : 0u;
    for (uint32_t i = threadIdx.x; i <= kLCBins && A.checksum; i += blockDim.x) rs[i] = A.rstart[i];
    __syncthreads();
    // the wave index as a uniform value: the blocks' counts, starts and dense
    // offsets then load with scalar loads into SGPRs (118 -> 57 VGPRs, 2 -> 3
    // workgroups per CU)
    const uint32_t lane = threadIdx.x & 63u, wv = (uint32_t)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    // the wave's blocks wv, wv + 16, ... of the group: all their loads first
    constexpr uint32_t kPer = kLCGroup / kLCBuildWaves;
    uint32_t cnt[kPer], nl[kPer];
    uint64_t st[kPer], sl[kPer], doff[kPer];
#pragma unroll
    for (uint32_t i = 0; i < kPer; i++) {
        const uint64_t b = (uint64_t)blockIdx.x * kLCGroup + wv + i * kLCBuildWaves;
        cnt[i] = b < A.n_blocks ? A.count[b] : 0u;  // dense blocks: counted by lc_dense
        nl[i] = b < A.n_blocks ? A.nlong[b] : 0u;   // dense blocks: long records left to the rounds
        st[i] = b < A.n_blocks ? A.start[b] : 0u;
        doff[i] = b < A.n_blocks ? A.dense_off[b] : kLCNotDense;
    }
    // a block whose events lc_dense wrote in place keeps them where its count was
    // as predicted and its start as placed then; else its stashed runs are expanded
    // here as any dense block's (a wrong prediction moves the blocks after it)
#pragma unroll
    for (uint32_t i = 0; i < kPer; i++) {
        const uint64_t b = (uint64_t)blockIdx.x * kLCGroup + wv + i * kLCBuildWaves;
        if (doff[i] != kLCNotDense && doff[i] != ~0ull && (doff[i] & kLDPlaced)) {
            const bool keep = cnt[i] == A.pred[b] && st[i] == A.start0[b];
            // a block without stashed runs (lc_dense: every count predicted) cannot move
            if (!keep && (doff[i] >> 48) == 0u && lane == 0) atomicOr(A.cap_flag, kLCFlagInconsistent);
            doff[i] = keep ? ~0ull : doff[i] & ~kLDPlaced;
        }
    }
    // a block's walk slots, or a dense block's first 64 stash entries (its runs)
#pragma unroll
    for (uint32_t i = 0; i < kPer; i++) {
        const uint64_t b = (uint64_t)blockIdx.x * kLCGroup + wv + i * kLCBuildWaves;
        if (doff[i] == kLCNotDense) {
            sl[i] = lane < cnt[i] && cnt[i] <= kLCSlots ? A.slots[b * kLCSlots + lane] : 0ull;
        } else {
            const uint32_t n0 = doff[i] == ~0ull ? 0u : (uint32_t)(doff[i] >> 48);
            sl[i] = lane < n0 ? lc_ld8(&A.stash[(doff[i] & 0xffffffffffffull) + lane]) : 0ull;
        }
    }
#pragma unroll
    for (uint32_t i = 0; i < kPer; i++) {
        const uint64_t b = (uint64_t)blockIdx.x * kLCGroup + wv + i * kLCBuildWaves;
        if (b >= A.n_blocks) break;
        if (doff[i] != kLCNotDense) {  // dense block: its events expanded from lc_dense's runs
            // (~0: they did not fit, the event array is too small anyway)
            if (doff[i] != ~0ull) lc_expand_runs(A, b, st[i], doff[i], sl[i]);
            if (A.checksum && nl[i]) {  // its long records' chunks (lc_dense counted them)
                const uint64_t s = lane < nl[i] ? A.slots[b * kLCSlots + lane] : 0ull;
                lc_place_wave(A, ctr, rs, lane < nl[i], b * 32768u + ((uint32_t)s & 0xffffu) + 6u,
                              1u + (((uint32_t)s >> 16) & 0xffffu), (uint32_t)(s >> 32));
            }
            continue;
        }
        const uint64_t bs = b * 32768u, s = sl[i];
        const bool have = lane < cnt[i];  // lane < kLCSlots always
        const uint32_t length = (uint32_t)s & 0xffffu, type = ((uint32_t)s >> 16) & 0xffu, kind = (uint32_t)s >> 24;
        const uint32_t stored = (uint32_t)(s >> 32);
        const uint64_t h = bs + lc_wave_excl_sum(have ? 7u + length : 0u);  // this event's header
        if (have) lc_event(A, st[i] + lane, h, length, type, kind);
        if (A.checksum) lc_place_wave(A, ctr, rs, have && kind == 1u, h + 6u, 1u + length, stored);
    }
    if (!A.checksum) lc_finish(A);  // the last kernel of a walk-only verification
}

// z^L(v) for L < 32768: z^(128 (L >> 7)) then z^(L & 127), 8 nibble lookups each
__device__ __forceinline__ uint32_t lc_nib(const uint32_t *t, uint32_t v) {
    uint32_t r = 0;
#pragma unroll
    for (int q = 0; q < 8; q++) r ^= t[16 * q + ((v >> (4 * q)) & 15u)];
    return r;
}
__device__ __forceinline__ uint32_t lc_zshift(const uint32_t *aux, uint32_t v, uint32_t L) {
    v = lc_nib(aux + kAuxZWDword + 128u * (L >> 7), v);
    return lc_nib(aux + kAuxZBDword + 128u * (L & 127u), v);
}

__global__ __launch_bounds__(256) void lc_combine_kernel(LCArgs A, uint32_t n_big_max) {
    const uint32_t nbig = A.rowtot[kLCBig];
    const uint32_t lim = nbig < n_big_max ? nbig : n_big_max;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < lim; i += gridDim.x * blockDim.x) {
        const LCBig g = A.big[i];
        if (g.J == 0u) continue;
        const uint32_t f = (uint32_t)(((uint64_t)(uintptr_t)A.log + g.p) & 127u);
        uint32_t s = A.parts[g.part0 + g.J - 1u];
        for (uint32_t j = 0; j + 1u < g.J; j++) s ^= lc_zshift(A.aux, A.parts[g.part0 + j], f + g.n - 4096u * (j + 1u));
        if (mask_crc(~s) != g.stored) {
            const uint64_t h = g.p - 6u;
            atomicMin(&A.first_bad[h >> 15], (uint32_t)(h & 32767u));
        }
    }
}

// One lane per block checks it; each block with a failure is then rewritten by
// its whole wave, lane = event (clean logs: one coalesced load per 64 blocks).
__global__ __launch_bounds__(256) void lc_apply_kernel(LCArgs A) {
    const uint64_t b = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t lane = threadIdx.x & 63u;
    lc_finish(A);  // the last kernel: the result words the host reads back
    const uint32_t fb = b < A.n_blocks ? A.first_bad[b] : kLCNone;
    uint64_t bad = __builtin_amdgcn_ballot_w64(fb != kLCNone);
    while (bad) {
        const uint32_t src = (uint32_t)__builtin_ctzll(bad);
        bad &= bad - 1u;
        const uint32_t f = (uint32_t)__builtin_amdgcn_readlane((int)fb, (int)src);
        const uint64_t bb = b - lane + src;
        const uint32_t cnt = A.count[bb];
        const uint64_t st = A.start[bb], bs = bb * 32768u;
        for (uint32_t k = lane; k < cnt; k += 64u) {
            const uint64_t i = st + k;
            if (i >= A.ev_cap) break;
            const uint32_t off = (uint32_t)(A.ev[i].offset - bs);
            if (off == f) A.ev[i].kind = 2u;      // BAD_CRC ("checksum mismatch")
            else if (off > f) A.ev[i].kind = 0u;  // dropped with the rest of the block
        }
    }
}

// ---------------------------------------------------------------------------
// Dense blocks (lc_walk's kLCDense: records of ~500 B and less, e.g. DBBench's
// default 100-B values make ~237 records of 138 B per 32 KiB block).  Cutting
// them into 8-chunk rounds would pay a round epilogue per ~2 windows, so a
// workgroup takes the whole block instead (persistent grid over the blocks
// lc_walk listed, 4 workgroups of 256 threads per CU, blocks taken in chunks of
// kLDChunk from a global counter; the next dense block's 32 KiB load into
// registers while the current one is worked on):
//   stage  the block into LDS
//   walk   RUNS of records: the header at p is read by every thread (a scalar
//          chain); when it repeats the record before it (length and type),
//          thread t checks the candidate header at p + (t + 1) L (L = 7 + its
//          length) — an OK record of the same length and type — and the first
//          failing candidate (ballot, LDS min) ends the run: a run of equal
//          records (DBBench's) is walked 257 headers per trip, one barrier each
//          (J/db/LogReader.java:297-383, the reference's decisions in its order)
//   crc    one thread per OK record, table lookups that never conflict (ld_map:
//          5-bit tables, one copy each): the record's dwords end-aligned in
//          pairs, two chains (position c of every pair) stepping z^8, folded
//          at the end with one z^4;
//          the record's first bytes are seeded with W0 (the 4 bytes before it
//          that take state 0 to value()'s 0xffffffff, so the first dword needs
//          no byte tables), its last dword is zero-padded and the stored crc
//          shifted over the same zeros instead; a failure atomicMin's its header
//          offset into first_bad[block] (lc_apply turns it into BAD_CRC and the
//          rest of the block into drops, :359-367, as for the other blocks)
//   stash  the block's runs (8 B each: offset, length, count, type, kind), not
//          its events: lc_build expands them into the event array
// A pass holds kLDRuns runs; a block of more (hundreds of short records of
// changing lengths) takes several passes, their stash segments chained by a
// link entry in the last slot of each.
// lc_dwalk (r5): the headers of the dense blocks, one lane per block, read from
// memory, before lc_dense.  lc_dense's own walk is one dependent chain per staged
// block (4 per CU): blocks of short records of random lengths (no runs to measure
// with its trips) cost ~1 K clocks per record on that chain, ~3 ms per GiB.  Here
// every dense block of the log walks at once (8-byte header loads that hit the
// block's lines in L2 after the first), and lc_dense only checks the crcs of the
// records whose offsets it finds in dw_off.  The walk stops at kDWMax offsets,
// at the first record that is not OK (lc_dense's walk decides it, as it decides
// the rest of the block), and at a run of kDWRun equal records (lc_dense's trips
// measure runs 257 records at a time: DBBench's blocks leave here after 8 hops).
// Offsets are u16 (p < 32 KiB), eight per 16-B store.  The walk reads nearly
// every line of its blocks at the HBM's random-line rate: a line prefetch 256 or
// 512 B ahead of each lane's walk made it slower (r5p, random 0-200 B set 2.62 ->
// 2.90 / 3.07 ms: the extra lines in flight evict the walk's own from L2), and so
// did a load of the next line beside each hop (r6zh, 2.53 -> 2.91 ms).
// One listed dense block (lc_dwalk's lane): a run block's prediction checked, the
// others' headers walked and their events predicted (count[b] = pred[b]).
__device__ __forceinline__ uint32_t dw_blen(const LCArgs &A, uint64_t b) {
    const uint64_t bs = b * 32768u;
    return (uint32_t)(A.size - bs < 32768u ? A.size - bs : 32768u);
}
// A run block's (kDWUniform) prediction holds, or nothing needs it.  lc_walk: a
// run, lc_dense walks it.  Its predicted event count (lc_walk's, from the walked
// records) places the blocks after it, which matters only when lc_dense writes
// events in place (some dense block is lc_dwalk's): checked at two headers, the
// next one repeats the run's length and the one after the run's predicted end
// fills the block.  A block of records of random lengths whose last walked ones
// were equal by chance fails and is walked by lc_dwalk instead (a wrong
// prediction costs lc_build the blocks after it)
__device__ __forceinline__ bool dw_run_holds(const LCArgs &A, uint64_t b) {
    if (*A.nu_ctr == 0u) return true;
    const uint64_t bs = b * 32768u;
    const uint32_t blen = dw_blen(A, b);
    const uint32_t info = A.dw_info[b], p = info & 0xffffu, L = info >> 16, left = blen - p;
    const uint32_t rem = left % L, k = left / L;
    const uint64_t h1 = k ? lc_header(A.log + bs + p, left) : 0ull;
    const uint64_t h2 = rem >= 7u ? lc_header(A.log + bs + p + k * L, rem) : 0ull;
    const bool ok1 = !k || 7u + ((uint32_t)(h1 >> 32) & 0xffffu) == L;
    const bool ok2 = rem < 7u || 7u + ((uint32_t)(h2 >> 32) & 0xffffu) == rem;
    return ok1 && ok2;
}
// the block's predicted events (count[b] = pred[b]) once its walk stopped at p
// after n offsets: the walk ended at the block's end (then the trailer, or the
// file's short last block's kind-6 event) or at a record that is not OK (`bad`:
// its event ends lc_dense's walk); after a run or kDWMax offsets: not predicted
// (kLCDense: the placement of the blocks after it is lc_build's)
__device__ __forceinline__ void dw_predict(const LCArgs &A, uint64_t b, uint32_t blen, uint32_t p, uint32_t n,
                                           bool bad) {
    A.dw_info[b] = n | (p << 16);
    const uint32_t rem = blen - p;
    uint32_t pred = kLCDense;
    if (rem < 7u)
        pred = n + (blen < 32768u && rem > 0u ? 1u : 0u);
    else if (bad)
        pred = n + 1u;
    A.count[b] = A.pred[b] = pred;
    if (pred == kLCDense) atomicAdd(&A.dense_ctr[7], 1u);  // lc_dense then stashes every block's runs
}
__device__ __forceinline__ void dw_block(const LCArgs &A, uint32_t i) {
    const uint32_t e = A.dense_list[i];
    const uint64_t b = e & ~kDWUniform, bs = b * 32768u;
    const uint32_t blen = dw_blen(A, b);
    if (e & kDWUniform) {
        if (dw_run_holds(A, b)) return;
        A.dense_list[i] = (uint32_t)b;  // not a run after all: walked here, its offsets to lc_dense
    }
    const uint8_t *blk = A.log + bs;
    lc_v4 *out = (lc_v4 *)(A.dw_off + b * kDWMax);
    uint32_t p = 0, n = 0, pk = ~0u, eq = 0;
    bool go = true;
    while (go) {
        uint32_t q[4] = {0u, 0u, 0u, 0u};
        const uint32_t n0 = n;
#pragma unroll
        for (uint32_t s = 0; s < 8u; s++) {
            // (straight-line flags, no continue: an early `continue` here was
            // miscompiled, the stored offset of a repeated record lost)
            const uint32_t rem = blen - p;
            bool st = !go || rem < 7u || n == kDWMax;
            uint32_t key = 0, len = 0;
            if (!st) {
                // header bytes 3..6: [crc3][len lo][len hi][type]; key = length | type << 16
                key = (uint32_t)(lc_header(blk + p, rem) >> 32) & 0xffffffu;
                len = key & 0xffffu;
                st = rem < 7u + len || key == 0u;  // not lc_decide's kind 1: lc_dense decides it
            }
            if (!st) {
                const bool same = key == pk;
                eq = same ? eq + 1u : 0u;
                pk = key;
                st = eq == kDWRun - 1u;  // a run: lc_dense measures it
            }
            const uint32_t put = st ? 0u : p << (16u * (s & 1u));
            q[s >> 1] |= put;
            n += st ? 0u : 1u;
            p += st ? 0u : 7u + len;
            go = go && !st;
        }
        if (n > n0) out[n0 / 8u] = lc_v4{q[0], q[1], q[2], q[3]};
    }
    const uint32_t rem = blen - p;
    bool bad = false;
    if (rem >= 7u && n < kDWMax) {
        const uint32_t key = (uint32_t)(lc_header(blk + p, rem) >> 32) & 0xffffffu;
        bad = rem < 7u + (key & 0xffffu) || key == 0u;
    }
    dw_predict(A, b, blen, p, n, bad);
}

// lc_dwalk: one lane per listed dense block (dw_block)
__global__ __launch_bounds__(256) void lc_dwalk_kernel(LCArgs A) {
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    if (i < A.dense_ctr[0]) dw_block(A, i);
}

// JL_OPT_FAILPOINT (tests only): lc_dwalk's results of the listed blocks it walked,
// perturbed one way per list index mod 6, so that each consistency check of
// lc_dense's first pass meets offsets that disagree with the block's bytes:
// 0 an inner offset one byte off, 1 more offsets than kDWMax, 2 the resume position
// one byte off, 3 the first offset not 0, 4 the last offset past the block, 5 none.
__global__ __launch_bounds__(256) void lc_failpoint_kernel(LCArgs A) {
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    if (i >= A.dense_ctr[0]) return;
    const uint32_t e = A.dense_list[i];
    if (e & kDWUniform) return;
    const uint64_t b = e;
    const uint32_t info = A.dw_info[b], n = info & 0xffffu;
    uint16_t *o = A.dw_off + b * kDWMax;
    switch (i % 6u) {
    case 0: if (n >= 2u) o[n / 2u] = (uint16_t)(o[n / 2u] + 1u); break;
    case 1: A.dw_info[b] = (info & 0xffff0000u) | (kDWMax + 1u); break;
    case 2: A.dw_info[b] = info + (1u << 16); break;
    case 3: if (n) o[0] = 7u; break;
    case 4: if (n) o[n - 1u] = 32765u; break;
    default: break;
    }
}
hipError_t launch_lc_failpoint(const LCArgs &A, hipStream_t st) {
    hipLaunchKernelGGL(lc_failpoint_kernel, dim3((A.n_blocks + 255u) / 256u), dim3(256), 0, st, A);
    return hipGetLastError();
}

constexpr uint32_t kLDThreads = 256;
__device__ __forceinline__ uint32_t lds32u(const uint32_t *d, uint32_t p) {  // bytes p..p+3, any alignment
    return __builtin_amdgcn_alignbyte(d[(p >> 2) + 1u], d[p >> 2], p & 3u);
}
// header bytes 3..6 at c when a whole header fits before blen, else 0
__device__ __forceinline__ uint32_t ld_hdr(const uint32_t *d, uint32_t blen, uint32_t c) {
    return c < blen && blen - c >= 7u ? lds32u(d, c + 3u) : 0u;
}
// z^(4k)(x) ^ w from 5-bit tables (k = 1, 2: 4 or 8 zero bytes; x: a
// chain's state XORed with its latest data dword):
//   z^(4k)(x) = XOR_i F_k,i[(x >> 5i) & 31],  F_k,i[v] = z^(4k)(v << 5i), i = 0..6
// (the last field 2 bits).  A 32-entry table fills the 32 banks a ds_read_b32
// lane group sees, so two lanes either read the same entry (broadcast) or
// different banks: these lookups never conflict, with ONE copy of each table
// (r3's byte tables, one copy beside the staged block, spent 58 % of the LDS
// cycles in bank conflicts, profiles/r3n_pmc_lc_dense.json).  7 lookups per
// dword, 2 VALU each for the address.  Nibble tables (8 lookups) with their
// addresses from one SDWA byte-select AND each (10 VALU per dword instead of 14)
// were no faster (r5e, DBBench 1.296 vs 1.290 ms, random lengths 3.38 vs 3.32):
// the crc phase is bound by the CU's LDS pipe, not by VALU issue, so lookups per
// dword are what count.
constexpr uint32_t kLDTabDwords = 7u * 32u;  // one map's tables
__device__ __forceinline__ uint32_t ld_map(const uint32_t *tab, uint32_t x, uint32_t w = 0u) {
    uint32_t r[7];
    r[0] = *(const uint32_t *)((const char *)tab + ((x << 2) & 0x7cu));
#pragma unroll
    for (uint32_t i = 1; i < 7; i++)
        r[i] = *(const uint32_t *)((const char *)tab + 128u * i + ((x >> (5u * i - 2u)) & 0x7cu));
    return xor3(xor3(r[0], r[1], r[2]), xor3(r[3], r[4], r[5]), r[6] ^ w);
}
// z(s) through T0 (one zero byte)
__device__ __forceinline__ uint32_t ld_z1(const uint32_t *T0, uint32_t s) { return (s >> 8) ^ T0[s & 0xffu]; }
// z^-1(s) through Ti[b] = (T0[i] << 8) | i, i the byte whose T0 entry has top byte b
// (z(r) = (r >> 8) ^ T0[r & 0xff] keeps T0's top byte, a permutation of i)
__device__ __forceinline__ uint32_t ld_zi1(const uint32_t *Ti, uint32_t s) { return (s << 8) ^ Ti[s >> 24]; }
// The crc tables of lc_dense / lc_small (LDS): N4 / N8 the 5-bit tables of z^4 / z^8
// (ld_map), Ti the inverse byte table (ld_zi1), W0 value()'s seed word and C_h =
// z^4(W0 << 8h) (a crc range starting h bytes into a dword)
struct LDTabs {
    const uint32_t *N4, *N8, *Ti;
    uint32_t W0, C1, C2, C3;
};
// One OK record's crc from the staged block dat (header at h, payload length len,
// crc range [h + 6, h + 7 + len) of at most kLDLongDw + 1 dwords): true when it
// equals the stored crc.  One thread per record.
__device__ __forceinline__ bool ld_crc_ok(const uint32_t *dat, const LDTabs &T, uint32_t h, uint32_t len) {
    const uint32_t q = h + 6u, e = h + 7u + len;  // crc range: type || payload
    const uint32_t a = q >> 2, hq = q & 3u, nd = ((e + 3u) >> 2) - a, tl = e & 3u;
    // the record's last dword is read whole: its 4 - tl bytes past the record
    // (the next header's) enter the chains' result s linearly, as themselves
    // (the last dword is chain 1's last word, XORed in unshifted), so s is
    // compared with want ^ those bytes instead of masking the dword in the loop
    const uint32_t gmask = tl ? ~((1u << (8u * tl)) - 1u) : 0u;
    // the chains end as u with z^4(u) = z^(4 - tl)(state) when the last dword
    // was padded with 4 - tl zeros (tl = 0: the state): so u = z^-tl(stored
    // state), tl = 0: z^-4 (inverse byte steps, ahead of the chains, so their
    // dependent lookups overlap the chains'; one z^4 fold of 7 lookups less)
    uint32_t want = ~unmask_crc(lds32u(dat, h));
    for (uint32_t z = tl ? tl : 4u; z; z--) want = ld_zi1(T.Ti, want);
    want ^= dat[a + nd - 1u] & gmask;
    // the first dword, seeded (C_h folds in the seed dword before it)
    const uint32_t d = dat[a];
    uint32_t x0 = ~d;
    if (hq) {
        const uint32_t c = hq == 1u ? T.C1 : (hq == 2u ? T.C2 : T.C3);
        x0 = c ^ ((T.W0 >> (32u - 8u * hq)) | (d & (~0u << (8u * hq))));
    }
    // two chains: the record's dwords end-aligned on pairs (o zero dwords in
    // front), chain c takes position c of every pair and steps z^8; at the
    // end chain 0 still owes z^4.  r4 ran four chains stepping z^16 and
    // folded them with z^12 / z^8 / z^4 (21 lookups per record against 7):
    // the crc phase is bound by the CU's LDS pipe and VALU issue together,
    // not by latency, so the fold's lookups cost more than the ILP gained
    // (r5l, same box: DBBench 1.274 -> 1.242 ms, random lengths 2.643 ->
    // 2.602).  Issuing both chains' 14 lookups together (the compiler
    // waits for chain 0's before reusing its registers for chain 1's
    // addresses) was no faster either (r5n: 1.264 vs 1.255 ms)
    const uint32_t o = nd & 1u, G = (nd + o) >> 1;
    const uint32_t *D = dat + a - o;  // D[j]: virtual dword j (j >= o)
    uint32_t y0 = o ? 0u : x0, y1 = o ? x0 : D[1];
    for (uint32_t g = 1; g < G; g++) {
        const uint32_t v0 = D[2u * g], v1 = D[2u * g + 1u];
        y0 = ld_map(T.N8, y0, v0);
        y1 = ld_map(T.N8, y1, v1);
    }
    const uint32_t sv = ld_map(T.N4, y0, y1);
    return sv == want;
}

// A workgroup's dense blocks come from lc_walk's list (dense_list[0 .. dense_ctr[0])),
// kLDChunk entries at a time from the counter dense_ctr[1], so a workgroup that
// runs faster takes more blocks (r4; r3 dealt the blocks statically,
// blockIdx.x + j gridDim.x, and the 4 workgroups of a CU do not run at the same
// rate: on the DBBench set they finished between 0.92 and 1.34 ms,
// profiles/r4i_ldprof.json).  The next chunk is always taken one chunk ahead and
// its list entries loaded then, so no wave waits for the counter or the list.
// Chunks of kLDChunk blocks, fewer when the list gives a workgroup fewer than 16
// chunks (ld_chunk): a log of blocks of short records of random lengths (~100 us
// of walk each) dealt 8 at a time left its workgroups ending 2.26 .. 3.24 ms
// (profiles/r4bc_walk_variants_ldprof.json)
constexpr uint32_t kLDChunk = 8;
__device__ __forceinline__ uint32_t ld_chunk(uint32_t nd) {
    const uint32_t c = nd / (16u * gridDim.x);
    return c < 1u ? 1u : (c > kLDChunk ? kLDChunk : c);
}
struct LDSched {
    uint32_t nd;        // dense blocks listed
    uint32_t ch;        // blocks per chunk (ld_chunk)
    uint32_t cur, nxt;  // list index of the current / next chunk (>= nd: none)
    uint32_t curb, nxtb;  // lane k < kLDChunk: their k-th block
    uint32_t idx;       // the current chunk's next entry
    __device__ __forceinline__ uint32_t load(const LCArgs &A, uint32_t c) const {
        const uint32_t k = c + (threadIdx.x & 63u);
        return (threadIdx.x & 63u) < ch && c < nd && k < nd ? A.dense_list[k] : 0u;
    }
    __device__ __forceinline__ void init(const LCArgs &A, uint32_t c0, uint32_t c1) {
        cur = c0;
        nxt = c1;
        curb = load(A, cur);
        nxtb = load(A, nxt);
        idx = 0;
    }
    // the next block (n_blocks when done); *moved: the current chunk was exhausted and
    // the next one taken over (the caller then starts the grab of the one after)
    __device__ __forceinline__ uint64_t next(const LCArgs &A, uint32_t s_new, bool *moved) {
        *moved = false;
        if (idx == ch || cur + idx >= nd) {
            cur = nxt;
            curb = nxtb;
            nxt = s_new;
            nxtb = load(A, nxt);
            idx = 0;
            *moved = true;
        }
        if (cur + idx >= nd) return A.n_blocks;
        return (uint32_t)__builtin_amdgcn_readlane((int)curb, (int)idx++);
    }
};
// a block can be loaded with whole 16-B vector loads (full, 16-B aligned)
__device__ __forceinline__ bool ld_vec(const LCArgs &A, uint64_t b) {
    return b < A.n_blocks && A.size - b * 32768u >= 32768u && ((uintptr_t)(A.log + b * 32768u) & 15u) == 0;
}
// A thread's 8 x 16 B of the next block, in named registers (an array here was
// placed in scratch memory by the compiler: every prefetched byte written out
// and read back, r3e PMC WRITE_SIZE 4.4 GB per 4 GiB log)
typedef uint32_t ld_v4 __attribute__((ext_vector_type(4)));  // (HIP's uint4 is a union-based class)
// the next dense block's bytes, non-temporal: each block is read once (r5zx:
// DBBench set 1.213 -> 1.179 ms against the default policy)
struct LDPre {
    ld_v4 a, b, c, d, e, f, g, h;
    __device__ __forceinline__ void load(const uint8_t *blk, uint32_t t) {
        const ld_v4 *s = (const ld_v4 *)blk + t;
        a = __builtin_nontemporal_load(s + 0 * kLDThreads);
        b = __builtin_nontemporal_load(s + 1 * kLDThreads);
        c = __builtin_nontemporal_load(s + 2 * kLDThreads);
        d = __builtin_nontemporal_load(s + 3 * kLDThreads);
        e = __builtin_nontemporal_load(s + 4 * kLDThreads);
        f = __builtin_nontemporal_load(s + 5 * kLDThreads);
        g = __builtin_nontemporal_load(s + 6 * kLDThreads);
        h = __builtin_nontemporal_load(s + 7 * kLDThreads);
    }
    __device__ __forceinline__ void store(uint32_t *dat, uint32_t t) const {
        ld_v4 *d4 = (ld_v4 *)dat + t;
        d4[0 * kLDThreads] = a;
        d4[1 * kLDThreads] = b;
        d4[2 * kLDThreads] = c;
        d4[3 * kLDThreads] = d;
        d4[4 * kLDThreads] = e;
        d4[5 * kLDThreads] = f;
        d4[6 * kLDThreads] = g;
        d4[7 * kLDThreads] = h;
    }
};

// A barrier over LDS only.  __syncthreads() also waits for every outstanding
// global access (vmcnt(0): gfx950 counts loads and stores together), which held
// each block's walk until the next block's prefetch had landed (r3 shader-clock
// phase counters: ~6 K of ~16 K clocks per block).
// lc_small's walk reads its headers from a 512-B window of the staged
// block held in registers, lane i its bytes 8 i .. 8 i + 7 of the window: a
// header inside the window costs three v_readlane (scalar results, no wait), a
// window one LDS trip per ~5 records of random lengths (r6: the small random-length
// log 117 -> 89 us).  r5 read every header from LDS: one dependent trip per record.
// lc_dense keeps the r5 form: the window cost its DBBench set ~1 % (r6j).
// q must be uniform; bytes past the staged block and its zero pad are never used
// (a header ends at most 3 bytes into the pad).
struct LDWin {
    uint32_t wb = 0x80000000u, wx = 0, wy = 0;  // the window's base (a multiple of 8), this lane's dwords
    __device__ __forceinline__ uint32_t at(const uint32_t *dat, uint32_t q, uint32_t lane) {  // == lds32u(dat, q)
        if (q - wb > 504u) {
            wb = q & ~7u;
            const uint64_t v = ((const uint64_t *)dat)[(wb >> 3) + lane];
            wx = (uint32_t)v;
            wy = (uint32_t)(v >> 32);
        }
        const uint32_t o = q - wb, k = o >> 2, l = k >> 1;
        const uint32_t a = __builtin_amdgcn_readlane(wx, l), b = __builtin_amdgcn_readlane(wy, l),
                       c = __builtin_amdgcn_readlane(wx, (l + 1u) & 63u);
        return __builtin_amdgcn_alignbyte(k & 1u ? c : b, k & 1u ? b : a, o & 3u);
    }
};

__device__ __forceinline__ void ld_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// stash entries: a run (offset in block | length << 16 | count << 32 | type << 48 |
// kind << 56) or, last in a segment, the link to the block's next segment
// (kLDLink << 56 | entries << 40 | stash offset)
constexpr uint64_t kLDLink = kLDLinkKind;
__device__ __forceinline__ uint64_t ld_run_entry(uint32_t ra, uint32_t rb, uint32_t cnt) {
    return (uint64_t)ra | ((uint64_t)cnt << 32) | ((uint64_t)(rb >> 16) << 48);
}

// The walk and a block's staging run at a higher wave priority than the crc
// phase (s_setprio 2, then 0): their dependent LDS trips then queue behind fewer
// of the other workgroups' lookups (r4: DBBench 1.371 -> 1.348 ms).  (The per-phase
// clock study, JL_LD_PROF / tools/ld_prof.py, lives on the branch study-r4-switches.)

// A record of more than kLDLongDw dwords in a dense block is not checked by one
// thread here: a 31 KiB record after a few short ones held its workgroup ~170 us
// (a 1 GiB log of such blocks took 40 ms against 0.33 for one record per block,
// tools/cliff_probe.py).  Its chunks join the rounds instead: counted into its
// group's histogram (lc_hist_global), its header offset, length and stored crc
// left in the block's walk slots (nlong[b] of them) for lc_build to place, the
// crc checked by crc_gv4_kernel<MODE_LOG_CHUNK> / lc_combine, a failure
// atomicMin'ed into first_bad[b] like the block's own.
// lc_dense's in-place events (lc_dwalk's blocks; only lc_dense_kernel<true>).
// The block's first event's place (lc_dense's first workgroups' placement, once
// its tile is out).
// its tile out; bounded (~0.2 s): past that the call is reported inconsistent
// and the block's events are not written, never a hang
__device__ __forceinline__ uint64_t ld_start0(const LCArgs &A, uint64_t b) {
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while (__hip_atomic_load(&A.ready0[b / kLSTile], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != A.gen) {
        if (__builtin_amdgcn_s_memrealtime() - t0 > 20000000ull) {  // (100 MHz clock)
            if ((threadIdx.x & 63u) == 0u) atomicOr(A.cap_flag, kLCFlagInconsistent);  // (any wave may wait)
            return ~0ull >> 1;
        }
        __builtin_amdgcn_s_sleep(2);
    }
    return uni64(__hip_atomic_load(&A.start0[b], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}
// events [ev0, ev0 + m) of block b: lc_dwalk's records, one each (header offsets doff)
__device__ __forceinline__ void ld_place_dw(const LCArgs &A, const uint32_t *dat, const uint32_t *doff, uint64_t b,
                                         uint32_t ev0, uint32_t m, uint32_t r0, uint32_t stride) {
    const uint64_t st0 = ld_start0(A, b) + ev0;
    for (uint32_t r = r0; r < m; r += stride) {
        const uint32_t h = (doff[r >> 1] >> (16u * (r & 1u))) & 0xffffu;
        const uint32_t w = __builtin_amdgcn_alignbyte(dat[((h + 3u) >> 2) + 1u], dat[(h + 3u) >> 2], (h + 3u) & 3u);
        lc_event(A, st0 + r, b * 32768u + h, (w >> 8) & 0xffffu, w >> 24, 1u);
    }
}
// events [ev0, ev0 + nev) of block b from a walk pass's runs
__device__ __forceinline__ void ld_place_runs(const LCArgs &A, const uint32_t *run_a, const uint32_t *run_b, uint64_t b,
                                           uint32_t ev0, uint32_t nr, uint32_t nev) {
    const uint64_t st0 = ld_start0(A, b) + ev0;
    for (uint32_t r = threadIdx.x; r < nev; r += 256u) {
        uint32_t j = 0;  // the run holding event r (as in the crc phase)
        for (uint32_t sh = nr > 1u ? 1u << (31 - __builtin_clz(nr - 1u)) : 0u; sh; sh >>= 1)
            if (j + sh < nr && (run_b[j + sh] & 0xffffu) <= r) j += sh;
        const uint32_t ra = run_a[j], rb = run_b[j], len = ra >> 16;
        lc_event(A, st0 + r, b * 32768u + (ra & 0xffffu) + (r - (rb & 0xffffu)) * (7u + len), len, (rb >> 16) & 0xffu,
                 rb >> 24);
    }
}
// the placement by the predicted counts: tiles k, k + grid, ... (kLSTile blocks
// each) by workgroup k (every workgroup does its first tile first, so a tile's
// look-back only waits for tiles already under way)
__device__ __forceinline__ void ld_place_tile(const LCArgs &A, uint32_t *buf, uint32_t *wsum, unsigned long long *s_pre) {
    const uint32_t tiles = (A.n_blocks + kLSTile) / kLSTile;
    for (uint32_t k = blockIdx.x; k < tiles; k += gridDim.x) {
        ls_tile(A, k, A.tstat0, A.start0, buf, wsum, s_pre, A.ready0);
        __syncthreads();  // buf / wsum / s_pre reused
    }
}

constexpr uint32_t kLDLongDw = 128;
static_assert(kLDLongDw * 4u * kLCSlots >= 32768u, "a block holds fewer long records than slots");
// Two kernels from one body (lc_dense_body.inc), either of them right for any log:
// lc_dense_kernel (no in-place events: lc_build places every dense block) and
// lc_dense_inplace_kernel (lc_dwalk's blocks' events in place when the log has
// such blocks).  The host launches the second when the previous verification of
// the workspace had lc_dwalk's blocks (LCArgs::hint, a guess that only decides
// speed).  One kernel with both paths cost the DBBench set's lc_dense ~2.5 % (108
// VGPRs and 75 SGPR spills against 101 and 45, r6w), out-of-line calls more
// (scratch), a template kernel's instances took 132 VGPRs (3 workgroups per CU)
// even with no change to the body, and both kernels launched (each returning at
// once on the other's logs) cost every set an empty launch, ~4.6 us
#define LD_KERNEL lc_dense_kernel
#define LD_INPLACE 0
#include "lc_dense_body.inc"
#undef LD_KERNEL
#undef LD_INPLACE
#define LD_KERNEL lc_dense_inplace_kernel
#define LD_INPLACE 1
#include "lc_dense_body.inc"
#undef LD_KERNEL
#undef LD_INPLACE


// ---------------------------------------------------------------------------
// lc_small: a small log (a WAL recovered at open, J/db/DBImpl.java:903; a
// MANIFEST, J/db/VersionSet.java:487) verified in ONE launch (VERDICT r5 item 5:
// the chunked path's ~11 dependent launches cost ~100 us even for a 0.25 MiB log).
// One workgroup per 32 KiB block, blocks taken in ticket order (so a workgroup's
// look-back only ever waits for workgroups that started before it):
//   stage   the block into LDS (as lc_dense)
//   walk    readPhysicalRecord's decisions in order (lc_dense's walk: runs of
//           equal records measured 257 headers per trip); the first pass counts
//           every event of the block and keeps up to kSRuns runs, a block of more
//           runs is processed in further passes from where the kept runs end
//   publish the block's event count (look-back status), before any crc work
//   crc     one thread per OK record (ld_crc_ok), one wave per record of more than
//           kLDLongDw dwords (ld_crc_wave_ok); the first failure's header offset
//           (atomicMin) makes that record BAD_CRC and the later events of the
//           block kind 0, as lc_apply does (J/db/LogReader.java:356-369)
//   place   the block's first event = the earlier blocks' events (decoupled
//           look-back by wave 0, 64 statuses per load), then the events in file
//           order straight into the caller's array
constexpr uint32_t kSRuns = 512;

// One OK record of more than kLDLongDw dwords, by a whole wave: the record's
// dwords end-aligned on 64 P virtual dwords (P = ceil(nd / 64); the zero dwords
// in front leave a zero chain zero), lane i runs the chain over its P of them
// (the first real dword seeded as in ld_crc_ok), then lane i's value is moved to
// the record's end, z^(4 P (63 - i)) (lc_zshift, aux tables), and XOR-reduced.
__device__ __forceinline__ bool ld_crc_wave_ok(const uint32_t *dat, const LDTabs &T, const uint32_t *aux, uint32_t h,
                                               uint32_t len, uint32_t lane) {
    const uint32_t q = h + 6u, e = h + 7u + len;
    const uint32_t a = q >> 2, hq = q & 3u, nd = ((e + 3u) >> 2) - a, tl = e & 3u;
    const uint32_t gmask = tl ? ~((1u << (8u * tl)) - 1u) : 0u;
    uint32_t want = ~unmask_crc(lds32u(dat, h));
    for (uint32_t z = tl ? tl : 4u; z; z--) want = ld_zi1(T.Ti, want);
    want ^= dat[a + nd - 1u] & gmask;
    const uint32_t d = dat[a];
    uint32_t x0 = ~d;
    if (hq) {
        const uint32_t c = hq == 1u ? T.C1 : (hq == 2u ? T.C2 : T.C3);
        x0 = c ^ ((T.W0 >> (32u - 8u * hq)) | (d & (~0u << (8u * hq))));
    }
    const uint32_t P = (nd + 63u) >> 6, front = 64u * P - nd;
    uint32_t y = 0;
    for (uint32_t j = 0; j < P; j++) {
        const uint32_t v = lane * P + j;
        const uint32_t k = v - front;
        const uint32_t w = v < front ? 0u : (k ? dat[a + k] : x0);
        y = ld_map(T.N4, y, w);
    }
    return wave_xor(lc_zshift(aux, y, 4u * P * (63u - lane))) == want;
}

__device__ __forceinline__ uint64_t ls_status(uint32_t gen, uint64_t flag, uint64_t v) {
    return ((uint64_t)gen << 32) | flag | (v & kLSVal);
}

__global__ __launch_bounds__(kLDThreads) void lc_small_kernel(LSmallArgs A) {
    __shared__ __attribute__((aligned(16))) uint32_t dat[8192 + 4];         // the block (+ zero pad: header reads near its end)
    __shared__ uint32_t nt[2 * kLDTabDwords];  // tables of z^4, z^8 (ld_map)
    __shared__ uint32_t t0[256];               // T0, then the inverse byte table
    __shared__ uint32_t run_a[kSRuns];         // offset in block | length << 16
    __shared__ uint32_t run_b[kSRuns];         // first event (of the block) | type << 16 | kind << 24
    __shared__ uint32_t lg[64];                // header offsets of the pass's long records
    __shared__ uint32_t s_w[6];                // the walk's results (wave 0) for the other waves
    __shared__ uint32_t s_bad, s_id;
    __shared__ unsigned long long s_pre;
    const uint32_t t = threadIdx.x, lane = t & 63u, wv = t >> 6;
    if (t == 0) {
        s_id = atomicAdd(A.ticket, 1u);
        if (s_id + 1u == A.n_blocks) *A.ticket = 0;  // every ticket taken: zero for the next call
        s_bad = kLCNone;
    }
    t0[t] = A.aux[t];
    ld_sync();
    const uint64_t b = uni(s_id);
    const uint64_t bs = b * 32768u;
    const uint32_t blen = (uint32_t)(A.size - bs < 32768u ? A.size - bs : 32768u);
    const bool eof = blen < 32768u;
    const bool vec = blen == 32768u && ((uintptr_t)(A.log + bs) & 15u) == 0;
    LDPre pre;
    if (vec) pre.load(A.log + bs, t);
    for (uint32_t w = t; w < 2u * kLDTabDwords; w += kLDThreads) {  // as lc_dense
        const uint32_t k = w / kLDTabDwords + 1u, e = w % kLDTabDwords;
        const uint32_t i = e >> 5, v = e & 31u;
        uint32_t x = i * 5u < 32u ? v << (5u * i) : 0u;
        for (uint32_t z = 0; z < 4u * k; z++) x = ld_z1(t0, x);
        nt[w] = x;
    }
    ld_sync();
    {  // t0 becomes the inverse table (ld_zi1)
        const uint32_t e = t0[t];
        ld_sync();
        t0[e >> 24] = (e << 8) | t;
    }
    if (vec) {
        pre.store(dat, t);
    } else {  // the log's short last block (or an unaligned log): bytes, nothing past its end
        const uint8_t *src = A.log + bs;
        for (uint32_t o = t; o < 8192u; o += kLDThreads) {
            uint32_t v = 0;
            for (uint32_t j = 0; j < 4; j++)
                if (4u * o + j < blen) v |= (uint32_t)src[4u * o + j] << (8 * j);
            dat[o] = v;
        }
    }
    if (t < 4) dat[8192 + t] = 0;
    ld_sync();
    const uint32_t *N4 = nt, *N8 = nt + kLDTabDwords;
    const uint32_t W0 = A.seed0;
    const LDTabs T{N4, N8, t0, W0, ld_map(N4, W0 << 8), ld_map(N4, W0 << 16), ld_map(N4, W0 << 24)};
    auto longrec = [&](uint32_t h, uint32_t len) { return ((h + 10u + len) >> 2) - ((h + 6u) >> 2) > kLDLongDw; };
    uint32_t p = 0, nev = 0;            // uniform: walk position, events walked so far
    uint32_t total = 0;                 // uniform: the block's events (known after the first walk)
    uint64_t start = 0;                 // uniform: the block's first event in the log
    bool first = true;
    for (;;) {
        // ---- walk from p: up to kSRuns runs kept; the first pass counts on to the block's
        // end.  Wave 0 alone walks (a chain of dependent LDS reads: the other waves'
        // copies of it only queued in front of its reads, and its trips of 64
        // candidates need no barrier); the others wait at the barrier below.
        const uint32_t ev0 = nev;
        if (wv == 0) {
            uint32_t nr = 0, nl = 0, pk = ~0u, ev_end = 0, p_end = 0;
            bool keep = true, more = false;
            // kept runs go into lane nr mod 64 of va / vb (no exec-mask switch and no
            // LDS store on the walk's chain), 64 at a time into LDS
            uint32_t va = 0, vb = 0;
            auto put = [&](uint32_t ra, uint32_t rb) {
                const bool mine = lane == (nr & 63u);  // (a compare and two selects: no exec-mask switch)
                va = mine ? ra : va;
                vb = mine ? rb : vb;
                if ((++nr & 63u) == 0u) {
                    run_a[nr - 64u + lane] = va;
                    run_b[nr - 64u + lane] = vb;
                }
            };
            LDWin win;  // the walk's header reads
            for (;;) {
                const uint32_t rem = blen - p, w = win.at(dat, p + 3u, lane), key = w >> 8, len = key & 0xffffu;
                const bool okrec = rem >= 7u + len && key != 0u;  // lc_decide's kind 1: an OK record
                if (okrec && key != pk && keep && nr < kSRuns && !longrec(p, len)) {
                    // the common step (records of changing lengths): a new run of one
                    put(p | (len << 16), nev | (w & 0xff000000u) >> 8 | (1u << 24));
                    pk = key;
                    nev++;
                    p += 7u + len;
                    continue;
                }
                if (okrec) {
                    if (key == pk) {  // it repeats the record before it: lane l checks p + (l + 1) L
                        const uint32_t L = 7u + len, c = p + (lane + 1u) * L;
                        const bool ok = c + L <= blen && (lds32u(dat, c + 3u) >> 8) == key;
                        const uint64_t nok = __builtin_amdgcn_ballot_w64(!ok);
                        const uint32_t m = 1u + (nok ? (uint32_t)__builtin_ctzll(nok) : 64u);
                        if (keep && longrec(p, len)) {  // < 64 records of > 512 B fit a block
                            if (lane < m && nl + lane < 64u) lg[nl + lane] = p + lane * L;
                            nl += m;
                        }
                        nev += m;
                        p += m * L;
                        continue;
                    }
                    if (keep && nr == kSRuns) {  // the first run not kept: a later pass starts here
                        keep = false;
                        more = true;
                        p_end = p;
                        ev_end = nev;
                        if (!first) break;
                    }
                    if (keep) {
                        if (longrec(p, len)) {
                            if (lane == 0 && nl < 64u) lg[nl] = p;
                            nl++;
                        }
                        put(p | (len << 16), nev | (w & 0xff000000u) >> 8 | (1u << 24));
                    }
                    pk = key;
                    nev++;
                    p += 7u + len;
                    continue;
                }
                // the block's end: the trailer (no event) or a record that stops the walk
                const LCDecision d0 = lc_decide(rem, eof, rem >= 7u ? w : 0u);
                if (d0.kind != 0u) {
                    if (keep && nr == kSRuns) {
                        keep = false;
                        more = true;
                        p_end = p;
                        ev_end = nev;
                    }
                    if (keep) put(p | (d0.length << 16), nev | (d0.type << 16) | (d0.kind << 24));
                    nev++;
                }
                break;
            }
            if ((nr & 63u) != 0u && lane < (nr & 63u)) {  // the last, partial group of kept runs
                run_a[(nr & ~63u) + lane] = va;
                run_b[(nr & ~63u) + lane] = vb;
            }
            if (keep) ev_end = nev;
            if (lane == 0) {
                s_w[0] = nr;
                s_w[1] = nl;
                s_w[2] = nev;
                s_w[3] = ev_end;
                s_w[4] = p_end;
                s_w[5] = more;
                if (first)  // the block's event count, published before any crc work
                    __hip_atomic_store(&A.tstat[b], ls_status(A.gen, b ? kLSAgg : kLSInc, nev), __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
            }
        }
        ld_sync();  // the pass's runs and long records are in LDS
        const uint32_t nr = uni(s_w[0]), nl = uni(s_w[1]), ev_end = uni(s_w[3]), p_end = uni(s_w[4]);
        const bool more = uni(s_w[5]) != 0u;
        nev = uni(s_w[2]);
        if (first) total = nev;
        const uint32_t npass = ev_end - ev0;
        if (A.checksum && uni(s_bad) == kLCNone) {  // (none once the block failed: the rest is dropped)
            for (uint32_t r = t; r < npass; r += kLDThreads) {
                uint32_t j = 0;  // the run holding event ev0 + r: the last with first <= it
                for (uint32_t sh = nr > 1u ? 1u << (31 - __builtin_clz(nr - 1u)) : 0u; sh; sh >>= 1)
                    if (j + sh < nr && (run_b[j + sh] & 0xffffu) <= ev0 + r) j += sh;
                const uint32_t ra = run_a[j], rb = run_b[j];
                if ((rb >> 24) != 1u) continue;
                const uint32_t len = ra >> 16, h = (ra & 0xffffu) + (ev0 + r - (rb & 0xffffu)) * (7u + len);
                if (longrec(h, len)) continue;  // the waves below
                if (!ld_crc_ok(dat, T, h, len)) atomicMin(&s_bad, h);
            }
            for (uint32_t k = wv; k < nl && k < 64u; k += kLDThreads / 64u) {
                const uint32_t h = lg[k], len = (lds32u(dat, h + 3u) >> 8) & 0xffffu;
                if (!ld_crc_wave_ok(dat, T, A.aux, h, len, lane) && lane == 0) atomicMin(&s_bad, h);
            }
        }
        if (first && wv == 0) {  // the block's first event: the events of the blocks before it
            uint64_t prev = 0;
            for (int64_t q = (int64_t)b - 1; q >= 0;) {
                const int64_t i = q - (int64_t)lane;
                const uint64_t st = i >= 0 ? __hip_atomic_load(&A.tstat[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                           : ls_status(A.gen, kLSInc, 0);
                const bool ready = (uint32_t)(st >> 32) == A.gen && (st & (kLSInc | kLSAgg)) != 0;
                const uint64_t im = __builtin_amdgcn_ballot_w64(ready && (st & kLSInc));
                const uint32_t lim = im ? (uint32_t)__builtin_ctzll(im) : 63u;
                const uint64_t need = lim == 63u ? ~0ull : (2ull << lim) - 1ull;
                if ((__builtin_amdgcn_ballot_w64(ready) & need) != need) {  // a status not yet published
                    __builtin_amdgcn_s_sleep(1);
                    continue;
                }
                const uint32_t v = lane <= lim ? (uint32_t)(st & kLSVal) : 0u;
                prev += (uint32_t)__builtin_amdgcn_readlane((int)(lc_wave_excl_sum(v) + v), 63);
                if (im) break;
                q -= 64;
            }
            if (lane == 0) {
                if (b) __hip_atomic_store(&A.tstat[b], ls_status(A.gen, kLSInc, prev + total), __ATOMIC_RELAXED,
                                          __HIP_MEMORY_SCOPE_AGENT);
                s_pre = prev;
                if (b + 1u == A.n_blocks) {  // the last block: the result words
                    A.result[0] = prev + total;
                    A.result[1] = 0;
                    A.result[2] = 0;
                }
            }
        }
        ld_sync();  // the crc phase's failures and the block's start
        if (first) start = uni64(s_pre);
        const uint32_t fb = uni(s_bad);
        for (uint32_t r = t; r < npass; r += kLDThreads) {  // the pass's events, in file order
            uint32_t j = 0;
            for (uint32_t sh = nr > 1u ? 1u << (31 - __builtin_clz(nr - 1u)) : 0u; sh; sh >>= 1)
                if (j + sh < nr && (run_b[j + sh] & 0xffffu) <= ev0 + r) j += sh;
            const uint32_t ra = run_a[j], rb = run_b[j];
            const uint32_t len = ra >> 16, h = (ra & 0xffffu) + (ev0 + r - (rb & 0xffffu)) * (7u + len);
            uint32_t kind = rb >> 24;
            if (A.checksum && fb != kLCNone) kind = h == fb ? 2u : (h > fb ? 0u : kind);
            const uint64_t at = start + ev0 + r, off = bs + h;
            if (at < A.ev_cap)
                lc_st16(&A.ev[at], lc_v4{(uint32_t)off, (uint32_t)(off >> 32), len, ((rb >> 16) & 0xffu) | (kind << 8)});
        }
        if (!more) break;
        ld_sync();  // the next pass rewrites the runs
        p = p_end;
        nev = ev_end;
        first = false;
    }
}
hipError_t launch_lc_small(const LSmallArgs &A, hipStream_t st) {
    hipLaunchKernelGGL(lc_small_kernel, dim3(A.n_blocks), dim3(kLDThreads), 0, st, A);
    return hipGetLastError();
}

// as many workgroups per CU as the LDS holds
uint32_t lc_dense_grid(int cus) {
    constexpr uint32_t lds = (8192 + 4) * 4 + 2 * kLDTabDwords * 4 + 256 * 4 + 2 * kLDRuns * 4 + kDWMax * 2 + 64;
    return (uint32_t)cus * (uint32_t)(kImageBytes / lds);
}
hipError_t launch_lc_dwalk(const LCArgs &A, hipStream_t st) {
    hipLaunchKernelGGL(lc_dwalk_kernel, dim3((A.n_blocks + 255u) / 256u), dim3(256), 0, st, A);
    return hipGetLastError();
}
hipError_t launch_lc_dense(const LCArgs &A, int cus, bool inplace, hipStream_t st) {
    if (inplace)
        hipLaunchKernelGGL(lc_dense_inplace_kernel, dim3(lc_dense_grid(cus)), dim3(kLDThreads), 0, st, A);
    else
        hipLaunchKernelGGL(lc_dense_kernel, dim3(lc_dense_grid(cus)), dim3(kLDThreads), 0, st, A);
    return hipGetLastError();
}

hipError_t launch_lc_walk(const LCArgs &A, hipStream_t st) {
    const uint32_t W = (A.n_grp + 3) / 4;
    hipLaunchKernelGGL(lc_walk_kernel, dim3(W), dim3(256), 0, st, A);
    return hipGetLastError();
}
hipError_t launch_lc_scan(const LCArgs &A, hipStream_t st) {
    const uint32_t tiles = (A.n_blocks + kLSTile) / kLSTile;
    hipLaunchKernelGGL(lc_scan_kernel, dim3(tiles + kLCCounters), dim3(256), 0, st, A);
    return hipGetLastError();
}
hipError_t launch_lc_setup(const LCArgs &A, hipStream_t st) {
    hipLaunchKernelGGL(lc_setup_kernel, dim3(1), dim3(kLCBins), 0, st, A);
    return hipGetLastError();
}
hipError_t launch_lc_build(const LCArgs &A, hipStream_t st) {
    hipLaunchKernelGGL(lc_build_kernel, dim3(A.n_grp), dim3(64 * kLCBuildWaves), 0, st, A);
    return hipGetLastError();
}
hipError_t launch_lc_combine(const LCArgs &A, hipStream_t st) {
    const uint32_t nmax = (uint32_t)(A.big_cap < 0xffffffffull ? A.big_cap : 0xffffffffull);
    hipLaunchKernelGGL(lc_combine_kernel, dim3(256), dim3(256), 0, st, A, nmax);
    return hipGetLastError();
}
hipError_t launch_lc_apply(const LCArgs &A, hipStream_t st) {
    const uint64_t n = (uint64_t)A.n_blocks;
    hipLaunchKernelGGL(lc_apply_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, A);
    return hipGetLastError();
}

}  // namespace jlk
