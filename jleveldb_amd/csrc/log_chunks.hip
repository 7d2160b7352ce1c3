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

__global__ __launch_bounds__(kLCWalkThreads) void lc_walk_kernel(LCArgs A) {
    __shared__ uint32_t h[kLCCounters];
    if (threadIdx.x < kLCCounters) h[threadIdx.x] = 0;
    __syncthreads();
    const uint64_t b = (uint64_t)blockIdx.x * kLCWalkThreads + threadIdx.x;
    if (b < A.n_blocks) {
        const uint64_t bs = b * 32768u, be = bs + 32768u < A.size ? bs + 32768u : A.size;
        const bool eof = be - bs < 32768u;
        const uint64_t base = (uint64_t)(uintptr_t)A.log;
        uint64_t p = bs;
        uint32_t cnt = 0;
        // header bytes 0..3 (stored crc) and 3..6 of the next header are loaded
        // before this record's slot store: vmcnt counts stores too on gfx9, and a
        // store issued first would put its latency on the walk's serial chain
        uint32_t w = 0, c = 0;
        if (be - p >= 7) {
            w = ld_u32u(A.log + p + 3);
            c = ld_u32u(A.log + p);
        }
        for (;;) {
            const LCDecision d = lc_decide(be - p, eof, w);
            if (d.kind == 0) break;  // the block's trailer: no event
            const uint64_t pn = p + 7u + d.length;
            const uint32_t wc = w, cc = c;
            if (!d.stop && be - pn >= 7) {
                w = ld_u32u(A.log + pn + 3);
                c = ld_u32u(A.log + pn);
            }
            const bool kept = cnt < kLCSlots;
            if (kept) {
                uint4 s;
                s.x = (uint32_t)(p - bs) | (d.length << 16);
                s.y = d.type | (d.kind << 8);
                s.z = cc;
                s.w = 0;
                reinterpret_cast<uint4 *>(A.slots)[b * kLCSlots + cnt] = s;
            }
            (void)wc;
            // chunk histogram: exactly the chunks lc_build places (in the fast
            // mode only the kept events: a block that overflows its slots makes
            // the caller re-run in the exact mode)
            if (d.kind == 1u && A.checksum && (kept || A.exact)) {
                const LCGeom g = lc_geom(base + p + 6u, 1u + d.length);
                if (g.J == 1u) {
                    atomicAdd(&h[g.K - 1u], 1u);
                } else {
                    atomicAdd(&h[kLCWin - 1u], g.J - 1u);
                    atomicAdd(&h[g.K - kLCWin * (g.J - 1u) - 1u], 1u);
                    atomicAdd(&h[kLCBig], 1u);
                    atomicAdd(&h[kLCPart], g.J);
                }
            }
            cnt++;
            if (d.stop) break;
            p = pn;
        }
        A.count[b] = cnt;
        if (cnt > kLCSlots) atomicOr(&A.overflow[0], 1u);
    }
    __syncthreads();
    if (threadIdx.x < kLCCounters) A.hist[(uint64_t)threadIdx.x * A.n_wg + blockIdx.x] = h[threadIdx.x];
}

// One wave: rstart[k] = rounds of the bins before k (bin k = chunks of k+1
// windows, ceil(count/8) rounds each), rstart[kLCWin] = all rounds (clamped to
// the descriptor capacity, overflow[1] set past it); the missing groups of every
// bin's last round are marked empty.
__global__ __launch_bounds__(64) void lc_setup_kernel(LCArgs A) {
    const uint32_t k = threadIdx.x;
    const uint64_t nw = A.n_wg;
    const uint32_t cnt = k < kLCWin ? A.hscan[(k + 1) * nw] - A.hscan[k * nw] : 0u;
    const uint32_t rounds = (cnt + 7u) / 8u;
    uint32_t incl = rounds;  // inclusive wave scan
    for (uint32_t o = 1; o < 64u; o <<= 1) {
        const uint32_t v = (uint32_t)__shfl_up((int)incl, o);
        if (k >= o) incl += v;
    }
    const uint32_t ex = incl - rounds;
    const uint32_t total = (uint32_t)__shfl((int)incl, 63);
    if (k < kLCWin) A.rstart[k] = ex;
    if (k == 0) {
        const bool over = total > A.round_cap;
        A.rstart[kLCWin] = over ? (uint32_t)A.round_cap : total;
        if (over) atomicOr(&A.overflow[1], 1u);
    }
    if (k < kLCWin && (cnt & 7u)) {
        const uint64_t r = (uint64_t)ex + cnt / 8u;
        if (r < A.round_cap)
            for (uint32_t g = cnt & 7u; g < 8u; g++) A.desc[r * 8u + g].idx = kGNull;
    }
}

__device__ __forceinline__ void lc_put(const LCArgs &A, uint32_t *ctr, uint32_t K, uint64_t prel, uint32_t seed,
                                       uint32_t d, uint32_t idx, uint32_t stored) {
    const uint32_t rank = atomicAdd(&ctr[K - 1u], 1u);
    const uint64_t round = (uint64_t)A.rstart[K - 1u] + rank / 8u;
    if (round >= A.round_cap) return;  // overflow[1] is set (lc_setup)
    GDesc g;
    g.pd = (prel & 0xffffffffffull) | ((uint64_t)K << 40) | ((uint64_t)seed << 48) | ((uint64_t)d << 56);
    g.idx = idx;
    g.K = stored;
    A.desc[round * 8u + rank % 8u] = g;
}

// The chunk descriptors of one OK record (crc range at prel, n bytes).
__device__ __forceinline__ void lc_place(const LCArgs &A, uint32_t *ctr, uint64_t prel, uint32_t n, uint32_t stored) {
    const LCGeom g = lc_geom((uint64_t)(uintptr_t)A.log + prel, n);
    if (g.J == 1u) {
        lc_put(A, ctr, g.K, prel, 1u, g.r, 0u, stored);
        return;
    }
    const uint32_t bi = atomicAdd(&ctr[kLCBig], 1u), pi = atomicAdd(&ctr[kLCPart], g.J);
    // past a capacity (cannot happen with the caller's bounds) the chunks still
    // take their ranks, as empty groups: no round of the table is left unwritten
    const bool fits = bi < A.big_cap && (uint64_t)pi + g.J <= A.part_cap;
    if (fits) {
        LCBig big;
        big.p = prel;
        big.n = n;
        big.stored = stored;
        big.part0 = pi;
        big.J = g.J;
        A.big[bi] = big;
    } else {
        atomicOr(&A.overflow[1], 1u);
        if (bi < A.big_cap) A.big[bi].J = 0u;  // skipped by lc_combine
    }
    const uint64_t arel = prel - g.f;  // the record's first window (chunks j >= 1 start on the grid)
    for (uint32_t j = 0; j < g.J; j++) {
        const bool last = j + 1u == g.J;
        const uint32_t K = last ? g.K - kLCWin * j : kLCWin;
        lc_put(A, ctr, K, j ? arel + 4096ull * j : prel, j == 0u, last ? g.r : 0u, fits ? kGPart | (pi + j) : kGNull,
               0u);
    }
}

__device__ __forceinline__ void lc_event(const LCArgs &A, uint64_t at, uint64_t off, uint32_t length, uint32_t type,
                                         uint32_t kind) {
    if (at >= A.ev_cap) return;
    LogEvent e;
    e.offset = off;
    e.length = length;
    e.type = (uint8_t)type;
    e.kind = (uint8_t)kind;
    e.pad = 0;
    A.ev[at] = e;
}

__global__ __launch_bounds__(kLCWalkThreads) void lc_build_kernel(LCArgs A) {
    __shared__ uint32_t ctr[kLCCounters];
    const uint64_t nw = A.n_wg;
    if (threadIdx.x < kLCCounters)
        ctr[threadIdx.x] = A.hscan[threadIdx.x * nw + blockIdx.x] - A.hscan[threadIdx.x * nw];
    __syncthreads();
    const uint64_t b = (uint64_t)blockIdx.x * kLCWalkThreads + threadIdx.x;
    if (b >= A.n_blocks) return;
    const uint32_t cnt = A.count[b];
    const uint64_t st = A.start[b], bs = b * 32768u;
    const uint32_t kept = cnt < kLCSlots ? cnt : kLCSlots;
    const uint4 *sl = reinterpret_cast<const uint4 *>(A.slots) + b * kLCSlots;
    for (uint32_t j = 0; j < kept; j++) {
        const uint4 s = sl[j];
        const uint32_t off = s.x & 0xffffu, length = s.x >> 16, type = s.y & 0xffu, kind = (s.y >> 8) & 0xffu;
        lc_event(A, st + j, bs + off, length, type, kind);
        if (kind == 1u && A.checksum) lc_place(A, ctr, bs + off + 6u, 1u + length, s.z);
    }
    if (cnt <= kLCSlots || !A.exact) return;
    // exact mode: the events past the slots (a block of many short records) are
    // walked again from the header after the last kept one (an OK record: only
    // OK records continue the walk)
    const uint4 s = sl[kLCSlots - 1u];
    uint64_t p = bs + (s.x & 0xffffu) + 7u + (s.x >> 16);
    const uint64_t be = bs + 32768u < A.size ? bs + 32768u : A.size;
    const bool eof = be - bs < 32768u;
    for (uint32_t j = kLCSlots; j < cnt; j++) {
        const uint32_t w = be - p >= 7 ? ld_u32u(A.log + p + 3) : 0u;
        const uint32_t c = be - p >= 7 ? ld_u32u(A.log + p) : 0u;
        const LCDecision d = lc_decide(be - p, eof, w);
        lc_event(A, st + j, p, d.length, d.type, d.kind);
        if (d.kind == 1u && A.checksum) lc_place(A, ctr, p + 6u, 1u + d.length, c);
        if (d.stop) break;
        p += 7u + d.length;
    }
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
    const uint64_t nw = A.n_wg;
    const uint32_t nbig = A.hscan[(kLCBig + 1u) * nw] - A.hscan[kLCBig * nw];
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

// One thread per (block, event mod kLCSlots): only blocks with a failure touch
// their events.
__global__ __launch_bounds__(256) void lc_apply_kernel(LCArgs A) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t b = t / kLCSlots;
    const uint32_t j = (uint32_t)(t % kLCSlots);
    if (b >= A.n_blocks) return;
    const uint32_t fb = A.first_bad[b];
    if (fb == kLCNone) return;
    const uint32_t cnt = A.count[b];
    const uint64_t st = A.start[b], bs = b * 32768u;
    for (uint32_t k = j; k < cnt; k += kLCSlots) {
        const uint64_t i = st + k;
        if (i >= A.ev_cap) break;
        const uint32_t off = (uint32_t)(A.ev[i].offset - bs);
        if (off == fb) A.ev[i].kind = 2u;       // BAD_CRC ("checksum mismatch")
        else if (off > fb) A.ev[i].kind = 0u;   // dropped with the rest of the block
    }
}

hipError_t launch_lc_walk(const LCArgs &A, hipStream_t st) {
    hipLaunchKernelGGL(lc_walk_kernel, dim3(A.n_wg), dim3(kLCWalkThreads), 0, st, A);
    return hipGetLastError();
}
hipError_t launch_lc_setup(const LCArgs &A, hipStream_t st) {
    hipLaunchKernelGGL(lc_setup_kernel, dim3(1), dim3(64), 0, st, A);
    return hipGetLastError();
}
hipError_t launch_lc_build(const LCArgs &A, hipStream_t st) {
    hipLaunchKernelGGL(lc_build_kernel, dim3(A.n_wg), dim3(kLCWalkThreads), 0, st, A);
    return hipGetLastError();
}
hipError_t launch_lc_combine(const LCArgs &A, hipStream_t st) {
    const uint32_t nmax = (uint32_t)(A.big_cap < 0xffffffffull ? A.big_cap : 0xffffffffull);
    hipLaunchKernelGGL(lc_combine_kernel, dim3(1024), dim3(256), 0, st, A, nmax);
    return hipGetLastError();
}
hipError_t launch_lc_apply(const LCArgs &A, hipStream_t st) {
    const uint64_t n = (uint64_t)A.n_blocks * kLCSlots;
    hipLaunchKernelGGL(lc_apply_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, A);
    return hipGetLastError();
}

}  // namespace jlk
