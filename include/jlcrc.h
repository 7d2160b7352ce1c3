/*
 * jlcrc.h — C-ABI of the MI355X-native masked-CRC32C engine for jleveldb.
 *
 * Drop-in boundary for the reference's checksum path.  J below abbreviates
 * src/main/java/com/tchaicatkovsky/jleveldb in ralgond/jleveldb.  The reference
 * has no FFI of its own: every entry point names the Java member it replaces;
 * INTEGRATION.md shows the JNI binding a maintainer adds on the Java side.
 *
 * Conventions
 *   - plain pointers and sizes only; every function is callable from C and JNI;
 *   - int-returning functions return JL_OK (0) or a negative JL_ERR_* code and
 *     never throw; jl_last_error() gives a thread-local message;
 *   - "_dev" functions take device pointers (HBM) and a hipStream_t (void*;
 *     NULL = the HIP null stream) and are asynchronous unless noted;
 *     the other batch functions take host memory and block until done;
 *   - the "_dev" compute functions (not jl_fill_random_dev / jl_read_stream_dev)
 *     refuse a stream that is being captured into a HIP graph with
 *     JL_ERR_INVALID, before enqueueing anything: scratch sizing and the
 *     ordering of a thread's calls are host-side, per call, and a replay would
 *     bypass them;
 *   - thread-safe: every calling thread gets its own streams, pinned staging
 *     and device scratch (created on its first call, freed when it exits), so
 *     concurrent callers do not serialise; jl_init / jl_shutdown must not race
 *     with other calls;
 *   - host-memory inputs stream through a double-buffered pipeline in chunks of
 *     JL_STREAM_CHUNK_BYTES (the copy of chunk i+1 overlaps the kernels of
 *     chunk i); pinned input is DMA'd directly, large pageable input is pinned
 *     for the call (JL_OPT_HOST_REGISTER) or copied through pinned staging;
 *   - there is no CPU fallback behind the batch / verify entry points: with no
 *     usable GPU they fail with JL_ERR_NO_DEVICE.  Only the scalar Crc32C
 *     statics (first block) run on the host, as the reference's do.
 */
#ifndef JLCRC_H
#define JLCRC_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ------------------------------------------------------------------ status */
#define JL_OK 0
#define JL_ERR_INVALID (-1)   /* bad argument (null pointer, size overflow)      */
#define JL_ERR_NO_DEVICE (-2) /* no HIP device / engine built without a GPU     */
#define JL_ERR_HIP (-3)       /* HIP runtime error (message in jl_last_error)   */
#define JL_ERR_NOMEM (-4)     /* device or pinned-host allocation failed         */
#define JL_ERR_CAPACITY (-5)  /* caller's output array too small                 */
#define JL_ERR_CORRUPT (-6)   /* input is not a well-formed sstable (message in jl_last_error) */

/* flags for the batch entry points */
#define JL_FLAG_MASK 1u /* store Crc32C.mask(crc) (the on-disk form), else the raw crc */

/* -------------------------------------------------- Crc32C statics (host) */
/* Replaces Crc32C.value(byte[],int,int) / value(Slice), J/util/Crc32C.java:85-93 */
uint32_t jl_crc32c_value(const uint8_t *data, size_t n);
/* Replaces Crc32C.extend(long,byte[],int,int), J/util/Crc32C.java:43-48 */
uint32_t jl_crc32c_extend(uint32_t init_crc, const uint8_t *data, size_t n);
/* Replaces Crc32C.mask(long), J/util/Crc32C.java:61-64 */
uint32_t jl_crc32c_mask(uint32_t crc);
/* Replaces Crc32C.unmask(long), J/util/Crc32C.java:72-75 */
uint32_t jl_crc32c_unmask(uint32_t masked_crc);
/* Replaces the java.util.zip.Checksum instance state of Crc32C
 * (J/util/Crc32C.java:96-167): `state` is the bit-flipped crc the Java object
 * holds in its `crc` field.  reset() == 0xffffffff; getValue() == ~state;
 * setValue(v) == ~v.  update(int b) is jl_crc32c_update(state, &b, 1). */
uint32_t jl_crc32c_update(uint32_t state, const uint8_t *data, size_t n);

/* --------------------------------------------------------------- lifecycle */
/* Binds the calling process to HIP device `device` (0-based ordinal within
 * HIP_VISIBLE_DEVICES), uploads the LDS table image and creates the engine
 * stream.  Idempotent for the same device.  (No reference counterpart: the Java
 * class is static; the JNI adapter calls this from its static initialiser.) */
int jl_init(int device);
int jl_shutdown(void);
const char *jl_last_error(void);
/* Number of visible HIP devices (0 when none). */
int jl_device_count(void);
/* Engine build/version string, e.g. "jlcrc 0.2 gfx950 (...)". */
const char *jl_version(void);

/* Engine options (process-wide; no reference counterpart).  The defaults are
 * the measured best; the options exist so tests and tuning can force each
 * kernel the engine may pick.  Returns JL_ERR_INVALID for an unknown option or
 * an out-of-range value; jl_get_option returns the current value.
 *   JL_OPT_GENERAL_PATH      offset/length batches: JL_PATH_AUTO (general v4
 *                            rounds pipeline, or the one-launch stream kernel for
 *                            verify batches under 4096 blocks), JL_PATH_STREAM,
 *                            JL_PATH_GV4
 *   JL_OPT_STREAM_DEPTH      stream kernel ring entries: 16 (default), 32, 48
 *   JL_OPT_STREAM_PARTITION  stream kernel: 1 = byte-balanced wave ranges (default),
 *                            0 = equal block counts
 *   JL_OPT_SPLIT_CAP         crc batches: chunks available to split blocks above
 *                            512 KiB (-1 = min(2^20, 2048 n), the default)
 *   JL_OPT_HOST_REGISTER     host-memory entry points: 1 = pin a pageable input of
 *                            >= 64 MiB with hipHostRegister for the call and DMA it
 *                            directly (the default), 0 = copy pageable input
 *                            through pinned staging buffers
 *   JL_OPT_STAGE_THREADS     host threads copying pageable input into staging (8)
 *   JL_OPT_STAGE_PIECE       staged copies: bytes per piece handed to the copy
 *                            engine while the host copies the next piece (a
 *                            chunk of <= 4 pieces' worth goes in 4 MiB pieces;
 *                            0 = one piece per chunk).  Default 16 MiB
 *   JL_OPT_HOST_THRESHOLD    host-memory entry points jl_crc32c_fixed / _batch,
 *                            jl_table_verify and jl_tables_verify: a call touching
 *                            fewer bytes than this runs on the calling thread's
 *                            SSE4.2 path (bit-identical; no device work; a device
 *                            must still be present); 0 = always the device.
 *                            Default JL_HOST_THRESHOLD_AUTO (-1): the engine
 *                            measures both paths per entry point and size class
 *                            (2^17 .. 2^25 B) on this box and sends each call to
 *                            the faster one (below 128 KiB always the host, from
 *                            64 MiB always the device)
 *   JL_OPT_LOG_HOST_THRESHOLD  the same for jl_log_verify (and jl_log_read_records);
 *                            default JL_HOST_THRESHOLD_AUTO
 *   JL_OPT_LOG_SMALL_MAX     log verification: a log (or a 64 MiB chunk of a
 *                            host-memory log) of at most this many bytes is
 *                            verified in one launch, one workgroup per 32 KiB
 *                            block; larger ones take the chunked path (walk,
 *                            rounds).  0 = always the chunked path.  Default 16 MiB
 *   JL_OPT_FAILPOINT         tests only: bit 0 perturbs the dense blocks' header
 *                            offsets between lc_dwalk and lc_dense (a different
 *                            inconsistency per block); results must not change
 *                            (lc_dense re-walks such a block itself).  Default 0
 */
#define JL_OPT_GENERAL_PATH 1
#define JL_OPT_STREAM_DEPTH 2
#define JL_OPT_STREAM_PARTITION 3
#define JL_OPT_SPLIT_CAP 4
#define JL_OPT_HOST_REGISTER 5
#define JL_OPT_STAGE_THREADS 6
#define JL_OPT_HOST_THRESHOLD 7
#define JL_OPT_LOG_HOST_THRESHOLD 8
#define JL_OPT_STAGE_PIECE 9
#define JL_OPT_FAILPOINT 10
#define JL_OPT_LOG_SMALL_MAX 11
#define JL_HOST_THRESHOLD_AUTO (-1)
/* Read-only (jl_get_option; jl_set_option refuses them): the staging copy pool
 * and the calling thread's last host-memory call, for diagnostics.
 *   JL_INFO_STAGE_WORKERS         copy-pool threads running
 *   JL_INFO_STAGE_SPAWN_FAILURES  copy-pool threads that could not be started
 *   JL_INFO_LAST_PATH             0 = the host path, 1 = the device, -1 = none yet
 *   JL_INFO_LAST_CALL_NS          its wall time
 *   JL_INFO_LAST_STAGE_NS         the part spent copying pageable input into
 *                                 pinned staging (0 when DMA'd directly) */
#define JL_INFO_STAGE_WORKERS 201
#define JL_INFO_STAGE_SPAWN_FAILURES 202
#define JL_INFO_LAST_PATH 203
#define JL_INFO_LAST_CALL_NS 204
#define JL_INFO_LAST_STAGE_NS 205
#define JL_PATH_AUTO 0
#define JL_PATH_STREAM 1
#define JL_PATH_GV4 2
int jl_set_option(int option, int64_t value);
int64_t jl_get_option(int option);

/* ------------------------------------------ device-resident batch checksums */
/* n_blocks contiguous blocks of block_bytes each starting at d_data
 * (block i = d_data[i*block_bytes, (i+1)*block_bytes)); d_out[i] = crc32c of
 * block i (masked with JL_FLAG_MASK).  The DBBench "crc32c" shape
 * (J/benchmark/DBBench.java:775-793) batched; block_bytes may be any size. */
int jl_crc32c_fixed_dev(const void *d_data, uint64_t block_bytes, uint64_t n_blocks, uint32_t flags,
                        uint32_t *d_out, void *stream);

/* Host-memory form of jl_crc32c_fixed_dev for blocks that start in host memory
 * (an mmap'd file, a pinned buffer): streams them through the engine in chunks
 * (JL_STREAM_CHUNK_BYTES), two HIP streams alternating so the H2D copy of
 * chunk i+1 overlaps the kernel of chunk i; out[] (host) is filled on return.
 * Pinned / hipHostRegister'ed memory is DMA'd directly; pageable memory is
 * first copied into pinned staging buffers.  Bound by PCIe, not HBM. */
int jl_crc32c_fixed(const uint8_t *host, uint64_t block_bytes, uint64_t n_blocks, uint32_t flags, uint32_t *out);
#define JL_STREAM_CHUNK_BYTES (64ull << 20)

/* Arbitrary blocks in one arena: block i = d_base[d_off[i], d_off[i]+d_len[i]).
 * base_bytes: the arena's size; a block reaching past it is not read and gets
 *   the result 0 (descriptors are checked on the device, so a corrupt handle is
 *   never an out-of-bounds HBM read).
 * d_init (nullable): per-block initial crc as in Crc32C.extend(init, ...),
 *   J/util/Crc32C.java:43-48 (LogWriter uses typeCrc[t], J/db/LogWriter.java:147).
 * d_suffix (nullable): one extra byte appended after each block, as
 *   TableBuilder.writeRawBlock appends the type byte, J/table/TableBuilder.java:313-315.
 * d_out[i] = crc (or mask(crc) with JL_FLAG_MASK). */
int jl_crc32c_batch_dev(const void *d_base, uint64_t base_bytes, const uint64_t *d_off, const uint32_t *d_len,
                        const uint32_t *d_init, const uint8_t *d_suffix, uint64_t n, uint32_t flags, uint32_t *d_out,
                        void *stream);

/* Host-memory form of jl_crc32c_batch_dev: streams the blocks to the device
 * and returns when out[] is filled.  With ascending offsets the blocks go in
 * chunks of <= JL_STREAM_CHUNK_BYTES of arena (double-buffered, only the bytes
 * the blocks cover are copied); otherwise one window spanning all of them.
 * Every block must lie in [0, base_bytes) (JL_ERR_INVALID otherwise). */
int jl_crc32c_batch(const uint8_t *base, uint64_t base_bytes, const uint64_t *off, const uint32_t *len,
                    const uint32_t *init, const uint8_t *suffix, uint64_t n, uint32_t flags, uint32_t *out);

/* ----------------------------------------------------- SSTable block shims */
/* Write side, batched TableBuilder.writeRawBlock (J/table/TableBuilder.java:305-323):
 * for block i = d_file[d_off[i], d_off[i]+d_size[i]) with compression type
 * d_type[i] (nullable = 0, kNoCompression, J/CompressionType.java) writes the
 * 5-byte trailer [type][LE32 mask(crc32c(block || type))] to d_trailer[5*i]. */
int jl_table_trailers_dev(const void *d_file, const uint64_t *d_off, const uint32_t *d_size, const uint8_t *d_type,
                          uint64_t n, uint8_t *d_trailer, void *stream);

/* Read side, batched TableFormat.readBlock checksum test
 * (J/table/TableFormat.java:207-218): for handle i (offset d_off[i], size
 * d_size[i]) sets d_status[i] = 1 when
 * unmask(LE32 @ off+size+1) == crc32c(file[off, off+size+1)), else 0 ("block
 * checksum mismatch").  A handle whose block and 5-byte trailer do not lie
 * inside [0, file_bytes) gets 0 and nothing past the file is read (checked on
 * the device: the handles may come from untrusted index blocks). */
int jl_table_verify_dev(const void *d_file, uint64_t file_bytes, const uint64_t *d_off, const uint32_t *d_size,
                        uint64_t n, uint8_t *d_status, void *stream);
/* Block handles of a whole SSTable image (host, no device work): parses the
 * footer (TableFormat.Footer.decodeFrom, J/table/TableFormat.java:126-146), the
 * index block's entries (Block.decodeEntry, J/table/Block.java:312-342; values
 * are BlockHandle varints, TableFormat.java:74-78) and the metaindex block's
 * (Table.readMeta, J/table/Table.java:287-310).  Writes *n handles (data blocks in
 * index order, then meta/filter blocks, the metaindex, the index) with
 * kind[i] = JL_BLOCK_*; every handle is checked to lie, with its 5-byte trailer,
 * inside the file.  The index and metaindex blocks are read as Table.open /
 * readMeta read them with paranoidChecks (TableFormat.readBlock,
 * TableFormat.java:195-258: trailer checksum, then type byte; the reference's
 * Snappy is a stub so only kNoCompression blocks are readable): a bad index
 * block fails the walk, a bad metaindex block only drops the meta handles.  The
 * arrays feed jl_table_verify[_dev] for whole-table verification.
 * JL_ERR_CORRUPT with the reference's message ("file is too short to be an
 * sstable", "not an sstable (bad magic number)", "block checksum mismatch",
 * "corrupted compressed block contents", "bad compress type N", "bad block
 * contents", "bad entry in block", "truncated block read") on a malformed file;
 * JL_ERR_CAPACITY (and *n set) when cap < *n.  kind may be NULL. */
#define JL_BLOCK_DATA 0
#define JL_BLOCK_INDEX 1
#define JL_BLOCK_METAINDEX 2
#define JL_BLOCK_META 3
int jl_table_block_handles(const uint8_t *file, uint64_t file_bytes, uint64_t *off, uint32_t *size, uint8_t *kind,
                           uint64_t cap, uint64_t *n);
/* Host-memory form (file = mmap'd .ldb bytes); blocking. */
int jl_table_verify(const uint8_t *file, uint64_t file_bytes, const uint64_t *off, const uint32_t *size, uint64_t n,
                    uint8_t *status);
/* Several tables at once: the input tables of a compaction, which
 * VersionSet.makeInputIterator opens with paranoidChecks
 * (J/db/VersionSet.java:820-823) and Table.open / TableFormat.readBlock verify
 * one block at a time.  Table t is files[t][0, file_bytes[t]); its handles are
 * off/size[first[t] .. first[t+1]) (offsets within table t; first[0] = 0,
 * first[n_tables] = total handles); status[i] as in jl_table_verify.  Tables
 * are packed into 64 MiB groups, one H2D copy and one launch per group. */
int jl_tables_verify(uint64_t n_tables, const uint8_t *const *files, const uint64_t *file_bytes, const uint64_t *first,
                     const uint64_t *off, const uint32_t *size, uint8_t *status);

/* ------------------------------------------------- WAL / MANIFEST log shims */
/* One physical-record decision of LogReader.readPhysicalRecord
 * (J/db/LogReader.java:297-383), in file order. */
typedef struct jl_log_event {
    uint64_t offset; /* file offset of the 7-byte header                     */
    uint32_t length; /* header length field                                   */
    uint8_t type;    /* header type byte (J/db/LogFormat.java:28-48)           */
    uint8_t kind;    /* JL_LOG_* below                                        */
    uint16_t pad;
} jl_log_event;

#define JL_LOG_OK 1             /* record accepted (CRC verified when checksum=1)             */
#define JL_LOG_BAD_CRC 2        /* "checksum mismatch": rest of the 32 KiB block dropped :356-369 */
#define JL_LOG_BAD_LENGTH 3     /* "bad record length": rest of block dropped :334-345        */
#define JL_LOG_ZERO_SKIP 4      /* type 0, length 0: rest of block skipped silently :347-353  */
#define JL_LOG_EOF_BAD_LENGTH 5 /* length past end of the final, short block: EOF :341-344    */
#define JL_LOG_EOF_TRUNC 6      /* 1..6 stray bytes at the end of the final block: EOF :315-322 */

/* Device-resident log verification: walks every 32 KiB block's headers,
 * verifies every record's masked CRC (crc over type || payload, LogWriter.java:147)
 * and truncates each block after its first failure, exactly as the reference
 * reader clears its buffer.  Writes up to `cap` events to d_events and the total
 * to *n_events (host pointer; this call synchronises on the stream).
 * `checksum` (LogReader's checksum flag, J/db/LogReader.java:356):
 *   JL_LOG_NO_CHECKSUM     header walk only, every record accepted;
 *   JL_LOG_CHECKSUM        header walk kernel, then every OK record's crc range
 *                          cut into chunks of <= 4 KiB sorted into rounds of one
 *                          window count through the general v4 kernel; blocks of
 *                          more than 64 records (DBBench's default 100-B values)
 *                          are verified whole from a copy in LDS instead (the
 *                          default; one pass for any log, no host round trip
 *                          before the final event count);
 *   JL_LOG_CHECKSUM_TWO_PASS  the same path (explicit name);
 *   JL_LOG_CHECKSUM_FUSED  one pass over the bytes that walks and verifies
 *                          together (log_stream.hip); same results, slower on
 *                          short records; blocks of more than 256
 *                          records fall back to the default path. */
#define JL_LOG_NO_CHECKSUM 0
#define JL_LOG_CHECKSUM 1
#define JL_LOG_CHECKSUM_TWO_PASS 2
#define JL_LOG_CHECKSUM_FUSED 3
int jl_log_verify_dev(const void *d_log, uint64_t log_bytes, int checksum, jl_log_event *d_events, uint64_t cap,
                      uint64_t *n_events, void *stream);
/* Asynchronous form of jl_log_verify_dev (same path and events): returns once
 * the kernels are enqueued on `stream`; the result words land in device memory
 * d_result[3] in stream order: [0] the event total (events past `cap` are not
 * written: the events are complete when [0] <= cap, for any log), [1] the
 * number of dense blocks the chunked path verified whole (more than 64 records;
 * informational; 0 on the one-launch path of logs up to JL_OPT_LOG_SMALL_MAX),
 * [2] non-zero if an internal capacity was exceeded or the scratch was not in the
 * state the call expects (cannot happen; reported rather than assumed).  checksum: JL_LOG_NO_CHECKSUM,
 * JL_LOG_CHECKSUM or JL_LOG_CHECKSUM_TWO_PASS.  A thread's log calls share its
 * scratch: a later call on another stream (the null stream included) first makes
 * its stream wait for this one (device-side).  Lets a caller
 * keep several verifications in flight back to back (no host round trip per
 * log); replaces the same readPhysicalRecord loop (J/db/LogReader.java:297-383). */
int jl_log_verify_dev_async(const void *d_log, uint64_t log_bytes, int checksum, jl_log_event *d_events, uint64_t cap,
                            uint64_t *d_result, void *stream);
/* Host-memory form (log = the on-disk .log / MANIFEST bytes); blocking. */
int jl_log_verify(const uint8_t *log, uint64_t log_bytes, int checksum, jl_log_event *events, uint64_t cap,
                  uint64_t *n_events);

/* LogReader.readRecord over a whole file (J/db/LogReader.java:146-252), driven
 * by jl_log_verify's events: reassembles fragmented records and produces the
 * same corruption reports the reference Reporter receives.
 *   records[i] = {offset (lastRecordOffset), arena offset, size}; payloads are
 *   appended to `arena`; reports[i] = {dropped bytes, reason, aux (type for
 *   JL_REASON_UNKNOWN_TYPE)}.  Returns JL_ERR_CAPACITY if an array is short. */
typedef struct jl_log_record {
    uint64_t offset;
    uint64_t arena_off;
    uint64_t size;
} jl_log_record;
typedef struct jl_log_report {
    uint64_t bytes;
    uint32_t reason;
    uint32_t aux;
} jl_log_report;

#define JL_REASON_BAD_LENGTH 1      /* "bad record length"                       */
#define JL_REASON_CHECKSUM 2        /* "checksum mismatch"                       */
#define JL_REASON_PARTIAL_1 3       /* "partial record without end(1)"           */
#define JL_REASON_PARTIAL_2 4       /* "partial record without end(2)"           */
#define JL_REASON_MISSING_START_1 5 /* "missing start of fragmented record(1)"   */
#define JL_REASON_MISSING_START_2 6 /* "missing start of fragmented record(2)"   */
#define JL_REASON_MIDDLE_ERROR 7    /* "error in middle of record"               */
#define JL_REASON_UNKNOWN_TYPE 8    /* "unknown record type N"                   */

int jl_log_read_records(const uint8_t *log, uint64_t log_bytes, int checksum, uint64_t initial_offset,
                        uint8_t *arena, uint64_t arena_cap, jl_log_record *records, uint64_t rec_cap,
                        uint64_t *n_records, jl_log_report *reports, uint64_t rep_cap, uint64_t *n_reports);

/* Batched LogWriter.emitPhysicalRecord headers (J/db/LogWriter.java:136-161):
 * for fragment i (payload d_base[d_off[i], +d_len[i]), d_len[i] <= 0xffff,
 * record type d_type[i]) writes [LE32 mask(extend(typeCrc[t], payload))][LE16 len][type]
 * to d_header[7*i].  Framing (fragment boundaries, trailers) stays with the
 * caller, as in LogWriter.addRecord. */
int jl_log_headers_dev(const void *d_base, const uint64_t *d_off, const uint32_t *d_len, const uint8_t *d_type,
                       uint64_t n, uint8_t *d_header, void *stream);

/* Framing plan of LogWriter.addRecord (J/db/LogWriter.java:88-134) for n
 * records appended to a log that is dest_length bytes long (LogWriter(dest,
 * destLength), :80-84): record r is src[rec_src_off[r], +rec_len[r]).  For every
 * physical fragment f: frag_hdr_off[f] = offset of its 7-byte header in the
 * appended bytes, frag_src_off[f] = its payload's offset in src, frag_len[f],
 * frag_type[f] (Full/First/Middle/Last).  Bytes not covered by a fragment are
 * the zero-filled block trailers (:101-107).  *n_frags / *log_bytes get the
 * totals; JL_ERR_CAPACITY when cap < *n_frags.  Host only, no checksum work. */
int jl_log_layout(const uint64_t *rec_src_off, const uint32_t *rec_len, uint64_t n, uint64_t dest_length,
                  uint64_t *frag_hdr_off, uint64_t *frag_src_off, uint32_t *frag_len, uint8_t *frag_type,
                  uint64_t cap, uint64_t *n_frags, uint64_t *log_bytes);

/* Batched LogWriter on the device: writes the log_bytes appended bytes of a
 * jl_log_layout plan to d_log — zero trailers, payload copied from d_src, and
 * every header [LE32 mask(extend(typeCrc[t], payload))][LE16 len][type]
 * (emitPhysicalRecord, J/db/LogWriter.java:136-161).  Asynchronous on stream;
 * the plan arrays are device pointers. */
int jl_log_emit_dev(const void *d_src, const uint64_t *d_frag_hdr_off, const uint64_t *d_frag_src_off,
                    const uint32_t *d_frag_len, const uint8_t *d_frag_type, uint64_t n_frags, uint64_t log_bytes,
                    uint8_t *d_log, void *stream);

/* ------------------------------------------------------------ bench helpers */
/* Fills d_dst[0, bytes) with the splitmix64 stream used by the benches
 * (word i = splitmix64(seed + (first_word + i + 1) * golden)), on device. */
int jl_fill_random_dev(void *d_dst, uint64_t bytes, uint64_t seed, uint64_t first_word, void *stream);

/* Read-only HBM stream over d_src[0, bytes) (bytes % 16 == 0), XOR-folded into
 * *d_sink: the measured read-bandwidth ceiling the roofline is quoted against. */
int jl_read_stream_dev(const void *d_src, uint64_t bytes, uint32_t *d_sink, void *stream);

#ifdef __cplusplus
}
#endif
#endif /* JLCRC_H */
