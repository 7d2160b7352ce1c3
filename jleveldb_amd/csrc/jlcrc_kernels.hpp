// jlcrc_kernels.hpp — launch interface between the C-ABI (jlcrc_api.hip) and the
// device kernels (jlcrc_kernels.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace jlk {

constexpr uint32_t kImageBytes = 163840;  // must equal jlmath::kImageBytes
// v4 image (fixed_v4.hip, crc_math.hpp build_lds_image_v4): region B offsets
constexpr uint32_t kV4U4Byte = 147456;   // uniform z^-4, z^-8, z^-12 nibble tables (512 B each)
constexpr uint32_t kV4SlotDword = 37248; // per-wave result slots (64 dwords per wave)
constexpr uint32_t kG4UByte = 153088;    // general v4: U_j[v] = slice4^-1(v << 8j), 4 x 256 dwords (seed of an init)
constexpr uint32_t kG4T0Byte = 157184;   // general v4: T0 (suffix byte step)
constexpr uint32_t kG4ShiftByte = 147456;  // general v4 image: U_k = z^-(4k), k = 0..6, nibble tables
constexpr uint32_t kG4EByte = 151040;      // general v4 image: E_e = z^-e, e = 0..3, nibble tables
constexpr uint32_t kG4SelByte = 158208;    // general v4 image: front / tail byte selectors (crc_math.hpp)
constexpr uint32_t kGNull = 0xffffffffu; // general v4: empty group of a round

enum : int {
    MODE_CRC = 0,           // out32[i] = crc / mask(crc)
    MODE_TABLE_VERIFY = 1,  // out8[i] = (LE32 @ ptr+n == mask(crc))   TableFormat.readBlock
    MODE_LOG_VERIFY = 2,    // out8[i] = (LE32 @ ptr-6 == mask(crc))   LogReader.readPhysicalRecord
    MODE_TRAILER = 3,       // out8[5i..] = [type][LE32 mask]          TableBuilder.writeRawBlock
    MODE_LOG_HEADER = 4,    // out8[7i..] = [LE32 mask][LE16 n][type]  LogWriter.emitPhysicalRecord
    MODE_LOG_CHUNK = 5,     // gv4 only: log record chunks (LDesc below); a failing record
                            // atomicMin's its header offset into out32[block] (first_bad)
};

struct KParams {
    const uint8_t *base;     // arena
    const uint64_t *off;     // per-block offsets (null = fixed stride)
    const uint32_t *len;     // per-block lengths
    uint32_t len_add;        // added to len[i] (table verify covers size+1 bytes)
    uint64_t fixed_bytes;    // stride/length when off == null
    const uint32_t *init;    // optional per-block extend() init
    const uint8_t *suffix;   // optional per-block suffix byte
    const uint8_t *type;     // record / compression type (trailer, log header)
    const uint32_t *aux;     // T0, inv_top, typeCrc (crc_math.hpp build_aux)
    const uint8_t *zero;     // 4 KiB of zeros: target of predicated-off loads
    uint64_t n;              // blocks
    uint32_t flags;          // JL_FLAG_MASK
    int mode;
    uint32_t *out32;
    uint8_t *out8;
    const uint64_t *hdr_off;  // MODE_LOG_HEADER: header i goes to out8 + hdr_off[i] (null: out8 + 7*i)
    // caller-supplied bytes at `base` (~0: unchecked, the engine's own descriptors):
    // a block (plus, for MODE_TABLE_VERIFY, its stored crc) reaching past it is
    // not read; its result is 0 (crc 0 / verify "mismatch")
    uint64_t base_bytes;
    // debug bounds checking (JL_STREAM_DEBUG): valid load range and a log of
    // offending accesses {block, entry, lane, address}; dbg == null: off
    uint64_t dbg_lo, dbg_hi;
    unsigned long long *dbg;
};

struct LogEvent {  // layout-identical to jl_log_event
    uint64_t offset;
    uint32_t length;
    uint8_t type;
    uint8_t kind;
    uint16_t pad;
};

// general v4 path (general_v4.hip): group descriptor of the sorted pipeline
// (16 B; 8 per round) and the kernel arguments
struct GDesc {
    uint64_t pd;    // first byte p (bits 0..55) | tail pad d << 56 of the 128-B-aligned grid
    uint32_t idx;   // block index (kGNull: empty group, mirrors group 0)
    uint32_t K;     // steps: the 128-B windows [p & ~127 + 128k, +128) that hold the block
};
struct GV4Args {
    KParams P;
    const GDesc *desc;          // null: implicit rounds of 8 consecutive fixed-stride blocks
    const uint32_t *n_rounds;   // device count of rounds (sorted pipeline)
    uint32_t seed0;             // W for init 0 = slice4^-1(0xffffffff)
    uint32_t fixed_K;           // implicit rounds (128-B aligned base and stride: no pads)
    uint32_t *parts;            // split blocks: raw chunk states (group idx = kGPart | part index)
    uint32_t *deal;             // rounds counter, zero at launch (null: each workgroup deals its own)
};
// A block above kGSplitMin (MODE_CRC) is cut into m <= 2048 chunks of S bytes
// (S a multiple of 128, >= 64 KiB; the last chunk shorter) computed as blocks of
// their own from state 0, then folded per block by gv4_combine_kernel.
constexpr uint32_t kGPart = 0x80000000u;
constexpr uint32_t kAuxZpowDword = 1552;  // must equal jlmath::kAuxZpow (z^(2^k) tables in aux)
constexpr uint64_t kGSplitMin = 512u << 10;
struct GBig {        // one split block (gv4_combine_kernel's work item)
    uint64_t i;      // block index
    uint32_t part0;  // its first chunk's slot in parts[]
    uint32_t m;      // chunks
};
struct GSplit {       // rounds-pipeline state of the block split
    uint32_t *bigbase;  // per block: part0, or 0xffffffff (not split)
    GBig *big;          // split blocks
    unsigned long long *ctl;  // [0] parts reserved (may exceed part_cap), [1] split blocks
    uint32_t part_cap;  // parts[] capacity (blocks beyond it stay whole)
};
constexpr uint32_t kGSoloKey = (1u << 17) - 1;  // sort key of blocks of >= 131071 steps: one per round

// ---------------------------------------------------------------------------
// Chunked log verification (log_chunks.hip + crc_gv4_kernel<MODE_LOG_CHUNK>).
// Every OK record's crc range [h + 6, h + 7 + len) is cut on the 128-B grid into
// chunks of at most kLCWin windows; chunks are sorted into rounds of 8 with the
// same window count K (exact bins 1..kLCWin) with no global atomics: per-
// workgroup histograms from the walk, one scan, deterministic placement.
// A record of one chunk is verified in the round's epilogue; the chunks of a
// longer record leave raw states in parts[] and log_combine_kernel folds them.
// GDesc fields in this mode (the same 16 B):
//   pd  = chunk start relative to the log (bits 0..39) | K << 40 | seed << 48 | d << 56
//         (seed: the chunk holds the record's first byte, W0 is fed before it)
//   idx = 0 (single-chunk record), kGPart | part index, or kGNull
//   K   = the record's stored masked crc (single-chunk records)
constexpr uint32_t kLCWin = 32;          // windows per chunk (4 KiB)
constexpr uint32_t kLCGroup = 64;        // 32 KiB blocks per walk group (one wave of the walk)
// chunk bins: (K - 1) * 16 + (d & 15): one round's groups share the epilogue's
// z^-(4c) and z^-e tables (d = 16a + 4c + e), so its lookups are bank-conflict free
constexpr uint32_t kLCBins = kLCWin * 16;
constexpr uint32_t kLCBig = kLCBins, kLCPart = kLCBins + 1, kLCOver = kLCBins + 2;
constexpr uint32_t kLCCounters = kLCBins + 3;  // per group: bins, multi-chunk records, parts, dense blocks
// walked events kept per 32 KiB block.  A block of more events, or whose first
// kLCProbe events end within kLCProbe * 512 bytes (records of ~500 B and less),
// is DENSE: lc_walk stops there (count = kLCDense), its chunks take no part in
// the rounds, and lc_dense verifies it whole from a copy staged in LDS, writes
// its exact event count and stashes its events (lc_build places them)
constexpr uint32_t kLCSlots = 64;
constexpr uint32_t kLCProbe = 4;
constexpr uint32_t kLCDense = 0xffffffffu;  // count[b] of a dense block whose events were not predicted, until lc_dense counts it
constexpr uint32_t kLDMaxEv = 4688;         // >= events (and runs) of one 32 KiB block (one per 7 bytes)
constexpr uint32_t kLCNone = 0xffffffffu;  // first_bad: no failure
struct LCBig {        // a record of more than one chunk
    uint64_t p;       // crc range start (h + 6) relative to the log
    uint32_t n;       // crc range bytes (1 + length)
    uint32_t stored;
    uint32_t part0;   // its chunk states parts[part0 .. part0 + J)
    uint32_t J;
};
struct LCArgs {
    const uint8_t *log;
    uint64_t size;
    uint32_t n_blocks, n_grp;  // 32 KiB blocks, walk groups of kLCGroup blocks
    int checksum;
    uint64_t *slots;       // n_blocks * kLCSlots walked events: length | type << 16 | kind << 24 | stored << 32
    uint32_t *count;       // n_blocks + 1 (count[n_blocks] = 0); dense blocks: see kLCDense
    // dense blocks' RUNS of events, 8 B each (offset in block | length << 16 | count
    // << 32 | type << 48 | kind << 56), block b's first stash segment at
    // dense_off[b] = stash offset | entries << 48; a segment's last entry may link
    // to the next one (kind 0xff: stash offset | entries << 40).  dense_off is
    // kLCNotDense for the other blocks (lc_walk), ~0 for a dense block whose runs
    // did not fit (the caller's event array is too small anyway)
    uint64_t *dense_off;
    uint64_t *stash;
    uint64_t stash_cap;
    // > 0: a workgroup takes stash entries stash_pool at a time (> kLDRuns; one
    // atomic per many blocks, whose wait would also wait for the prefetch loads);
    // 0: one atomic per pass (small logs)
    uint64_t stash_pool;
    unsigned long long *stash_ctr;  // zeroed by lc_walk
    uint64_t *start;       // n_blocks + 1: exclusive scan of count
    uint32_t *hist;        // kLCCounters * n_grp, counter-major (hist[c * n_grp + group])
    uint32_t *hscan;       // per counter (row): exclusive scan over the groups (lc_scan)
    uint32_t *rowtot;      // kLCCounters: the rows' totals
    uint64_t *tstat;       // lc_scan's tile look-back statuses (zeroed by lc_walk)
    uint32_t *nlong;       // n_blocks: a dense block's long records left to the rounds (zeroed by lc_walk)
    uint32_t *rstart;      // kLCBins + 1: first round of every bin; [kLCBins] = rounds
    uint32_t *first_bad;   // n_blocks: header offset of the block's first failing record
    uint32_t seed0;        // slice4^-1(0xffffffff): value()'s seed as 4 bytes before a crc range
    uint32_t *dense_list;  // n_blocks: the dense blocks (lc_walk appends, lc_dense takes them in chunks)
    uint32_t *dense_ctr;   // [0] dense blocks listed, [1] list entries taken, [2] gv4 deal, [3] lc_scan ids (zero at the start; lc_finish re-zeroes them)
    uint32_t *nu_ctr;      // dense_ctr + 6: lc_dwalk's blocks (lc_walk counts them; lc_finish zeroes it)
    // in-place events of lc_dwalk's blocks (r6): every dense block's predicted event
    // count (lc_walk / lc_dwalk; count[b] until lc_dense counts), the starts they give
    // (lc_dense's first workgroups, by agent-scope atomics), its look-back statuses,
    // and per tile of kLSTile blocks the call's tag once its starts are out
    uint32_t *pred;
    uint64_t *start0;
    uint64_t *tstat0;
    uint32_t *ready0;
    uint32_t gen;    // this verification's tag (never 0)
    uint32_t *hint;  // host-visible: lc_finish leaves *nu_ctr there (which lc_dense kernel comes next)
    uint32_t *cap_flag;    // set when a capacity was exceeded
    uint64_t *result;      // [0] events, [1] dense blocks, [2] cap_flag (written last)
    GDesc *desc;           // rounds * 8
    uint64_t round_cap;    // rounds the desc array holds
    LCBig *big;
    uint64_t big_cap;
    uint32_t *parts;
    uint64_t part_cap;
    LogEvent *ev;
    uint64_t ev_cap;
    const uint32_t *aux;
    // lc_dwalk -> lc_dense: a dense block's first header offsets (kDWMax per block)
    // and dw_info[b] = offsets | (where lc_dense's own walk resumes) << 16
    uint16_t *dw_off;
    uint32_t *dw_info;
};
// crc_gv4_kernel's round dealing state in its LDS image (general_v4.hip): dwords
// [kGvBatchDword, +32) = 16 batch slots {base, tag | reads << 26}, [kGvDynDword,
// kGvDynEnd) = the workgroup's counter and 16 queues of 16 rounds.  Both gv4
// images leave them zero (checked when the images are built, jlcrc_api.hip).
constexpr uint32_t kGvBatchDword = 7900, kGvDynDword = 7935, kGvDynEnd = kGvDynDword + 1 + 16 * 16;
hipError_t launch_lc_walk(const LCArgs &A, hipStream_t st);
hipError_t launch_lc_scan(const LCArgs &A, hipStream_t st);
hipError_t launch_lc_setup(const LCArgs &A, hipStream_t st);
hipError_t launch_lc_build(const LCArgs &A, hipStream_t st);
hipError_t launch_lc_combine(const LCArgs &A, hipStream_t st);
hipError_t launch_lc_apply(const LCArgs &A, hipStream_t st);
// inplace: lc_dense_inplace_kernel (lc_dwalk's blocks' events in place), else lc_dense_kernel
hipError_t launch_lc_dense(const LCArgs &A, int cus, bool inplace, hipStream_t st);
hipError_t launch_lc_dwalk(const LCArgs &A, hipStream_t st);
// Small logs in one launch (lc_small_kernel, log_chunks.hip): one workgroup per
// 32 KiB block (the blocks in ticket order) stages the block in LDS, walks it
// (readPhysicalRecord's decisions), checks every OK record's crc there (one
// thread per record, one wave per record of more than kLDLongDw dwords), takes
// its first event's place from a decoupled look-back over the earlier blocks'
// event counts and writes its events in file order: no scans, rounds or host
// round trip.  Scratch: the ticket counter (zero between calls: the last ticket's
// taker re-zeroes it) and one look-back status per block, tagged with the call's
// generation `gen` (statuses of earlier calls never match: no memset per call).
struct LSmallArgs {
    const uint8_t *log;
    uint64_t size;
    uint32_t n_blocks;
    int checksum;
    uint32_t seed0;          // slice4^-1(0xffffffff)
    uint32_t gen;            // this call's status tag (never 0)
    const uint32_t *aux;     // T0 and the z^L nibble tables (lc_zshift)
    LogEvent *ev;
    uint64_t ev_cap;
    uint32_t *ticket;
    uint64_t *tstat;         // n_blocks look-back statuses: gen << 32 | kLSInc / kLSAgg | events
    uint64_t *result;        // [0] events, [1] 0, [2] 0 (written by the last block's workgroup)
};
constexpr uint64_t kLSInc = 1ull << 31, kLSAgg = 1ull << 30, kLSVal = kLSAgg - 1;
hipError_t launch_lc_small(const LSmallArgs &A, hipStream_t st);
// cap_flag bits (result word 2): a capacity of the round table / multi-chunk records
// exceeded; records of one dense block that overlap (more long records than slots);
// the work counters were not zero when lc_walk started (an earlier verification of
// this workspace stopped before lc_finish)
constexpr uint32_t kLCFlagCapacity = 1u, kLCFlagInconsistent = 2u, kLCFlagStale = 4u;
// JL_OPT_FAILPOINT (tests): lc_dwalk's offsets of the listed dense blocks
// perturbed before lc_dense reads them (each of lc_dense's consistency checks hit)
hipError_t launch_lc_failpoint(const LCArgs &A, hipStream_t st);
// lc_dwalk: header offsets kept per dense block; a run of kDWRun equal records
// ends its walk (lc_dense's trips measure runs 257 records at a time)
constexpr uint32_t kDWMax = 512;
constexpr uint32_t kDWRun = 8;
// lc_walk: a dense block whose last kDWProbe walked records are equal skips lc_dwalk
// (its dense_list entry carries kDWUniform; block indices are < 2^31)
constexpr uint32_t kDWProbe = 3;
constexpr uint32_t kDWUniform = 0x80000000u;
uint32_t lc_dense_grid(int cus);                  // lc_dense's workgroups
constexpr uint64_t kLDPool = 16384;               // stash_pool of large logs
constexpr uint32_t kLDRuns = 256;                 // runs per lc_dense pass (a stash segment: + 1 link)
constexpr uint64_t kLCNotDense = 0xfffffffffffffffeull;
constexpr uint64_t kLDPlaced = 1ull << 47;  // dense_off: lc_dense wrote the block's events in place
#ifndef JL_LS_TILE
#define JL_LS_TILE 4096  // study builds: 256 runs the multi-tile / multi-step paths on small logs
#endif
constexpr uint32_t kLSTile = JL_LS_TILE;  // lc_scan: values per workgroup and step (256 threads x kLSTile / 256)
// decoupled look-back statuses (lc_scan): 0 = not yet, else a flag | value
constexpr uint64_t kLDAgg = 1ull << 62, kLDInc = 1ull << 63, kLDVal = kLDAgg - 1;

// block i of an offset/length batch lies (with its stored crc in MODE_TABLE_VERIFY)
// inside the caller's base_bytes
__host__ __device__ inline bool block_in_range(const KParams &P, uint64_t off, uint32_t n) {
    if (P.base_bytes == ~0ull) return true;
    const uint64_t need = (uint64_t)n + (P.mode == MODE_TABLE_VERIFY ? 4u : 0u);
    return off <= P.base_bytes && need <= P.base_bytes - off;
}

// v4 fast path (fixed_v4.hip): 8 lanes per block, 8 ring slots, 1024 threads; img = the 8-lane v4 image
hipError_t launch_fixed4k_v4(const void *img, const uint8_t *data, uint64_t n_blocks, uint32_t flags, uint32_t *out,
                             int grid, hipStream_t st);
// general v4 main kernel, one specialisation per mode (general_v4.hip -DJL_MODE=k; modes 0, 1, 5)
template <int MODE>
hipError_t launch_gv4_m(const void *img, const GV4Args &A, const uint8_t *zero, int grid, hipStream_t st);
// sorted-pipeline helpers (general_v4.hip, mode-0 object)
hipError_t launch_gv4_rounds(const KParams &P, const GSplit &S, uint32_t *hist, uint32_t *cursor, uint32_t *rstart,
                             GDesc *desc, uint32_t *n_rounds, hipStream_t st);
// folds the chunk states of every split block into its result (after the main kernel)
hipError_t launch_gv4_combine(const KParams &P, const GSplit &S, const uint32_t *parts, hipStream_t st);
hipError_t launch_stream(const void *img, const KParams &P, const uint64_t *part, int grid, int depth, hipStream_t st);
// one specialisation per mode, each in its own object (stream_kernel.hip -DJL_MODE=k)
template <int MODE>
hipError_t launch_stream_m(const void *img, const KParams &P, const uint64_t *part, int grid, int depth, hipStream_t st);
// Byte-balanced partition of n blocks over `parts` waves for the stream kernel:
// incl[i] = sum of weights of blocks 0..i (weight = len + per-block overhead);
// part[w] = first block of wave w (part[0] = 0, part[parts] = n).
hipError_t launch_partition(const uint64_t *incl, uint64_t n, uint64_t parts, uint64_t *part, hipStream_t st);
// Fused log verification (log_stream.hip): one pass over the log, 8 lanes per
// 32 KiB block and 8 blocks per wave; walks the headers from the streamed bytes
// and folds every record's crc.  Per block: the events it walked (up to `cap`
// in slots[b * cap ...], tentatively OK), their count and the index of the
// first record whose crc failed.
constexpr uint32_t kLSLaneByte = 32768u * 4u;   // must equal jlmath::kLS*Dword * 4
constexpr uint32_t kLSShiftByte = 34816u * 4u;
constexpr uint32_t kLSEByte = 35712u * 4u;
constexpr uint32_t kLSMaskByte = 36224u * 4u;
constexpr uint32_t kLSStageByte = 36384u * 4u;
constexpr uint32_t kLSNone = 0xffffffffu;       // first_bad: no failure
struct LogStreamArgs {
    const uint8_t *log;
    uint64_t size;
    uint32_t n_blocks;
    uint32_t cap;          // event slots per block
    LogEvent *slots;       // n_blocks * cap
    uint32_t *count;       // n_blocks: events walked
    uint32_t *first_bad;   // n_blocks: slot of the first BAD_CRC record (kLSNone: none)
    uint32_t *overflow;    // set when a block walked more than cap events
};
hipError_t launch_logstream(const void *img, const LogStreamArgs &A, int grid, hipStream_t st);
// copies the walked events of every block to ev[start[b] ...] (at most cap_out in
// all), applying first_bad: that record becomes BAD_CRC, later ones of its block
// kind 0 (dropped with the rest of the 32 KiB block, J/db/LogReader.java:359-367)
hipError_t launch_logstream_compact(const LogStreamArgs &A, const uint64_t *start, LogEvent *ev, uint64_t cap_out,
                                    hipStream_t st);
hipError_t launch_log_copy(const uint8_t *src, const uint64_t *frag_src_off, const uint64_t *frag_hdr_off,
                           const uint32_t *frag_len, uint64_t n_frags, uint8_t *log, uint64_t *pay_off, hipStream_t st);
hipError_t launch_event_rebase(LogEvent *ev, uint64_t n, uint64_t base, hipStream_t st);
hipError_t launch_read_stream(const void *src, uint64_t bytes, uint32_t *sink, int grid, hipStream_t st);
hipError_t launch_fill_random(void *dst, uint64_t bytes, uint64_t seed, uint64_t first_word, hipStream_t st);

}  // namespace jlk
