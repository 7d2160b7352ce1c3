/*
 * oracle/crc32c_oracle.c — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the reference (ralgond/jleveldb) masked-CRC32C path and of
 * the four call sites that frame it.  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load this library, and only as the checker or
 * as the timed CPU baseline.  The product (jleveldb_amd/libjlcrc.so) never links
 * or calls it.
 *
 * Parity pinning: the generated tables are checked (tests/test_oracle.py) against
 * the SHA-256 of the 2048 literal table values parsed from the reference source
 * (tests/golden/make_golden.py), and every function below is checked against the
 * reference's own known-answer tests (T/TestCrc32C.java:60-119) plus an
 * independent bit-serial CRC.
 *
 * Abbreviations: J = src/main/java/com/tchaicatkovsky/jleveldb
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define ORC_POLY 0x82F63B78u /* reflected Castagnoli, J/util/Crc32C.java:169-171 */

static uint32_t T[8][256]; /* T8_0 .. T8_7, J/util/Crc32C.java:173-334 */
static pthread_once_t tables_once = PTHREAD_ONCE_INIT;

static void build_tables(void) {
    for (uint32_t i = 0; i < 256; i++) {
        uint32_t c = i;
        for (int k = 0; k < 8; k++) c = (c >> 1) ^ ((c & 1u) ? ORC_POLY : 0u);
        T[0][i] = c;
    }
    /* T8_k[i] = CRC of byte i followed by k zero bytes */
    for (int k = 1; k < 8; k++)
        for (uint32_t i = 0; i < 256; i++)
            T[k][i] = (T[k - 1][i] >> 8) ^ T[0][T[k - 1][i] & 0xffu];
}

static void ensure_tables(void) { pthread_once(&tables_once, build_tables); }

/* Copy of the generated 8x256 table, in the reference's T8_0..T8_7 order. */
void orc_tables(uint32_t *out) {
    ensure_tables();
    memcpy(out, T, sizeof(T));
}

/* Crc32C.update(byte[] b, int off, int len), J/util/Crc32C.java:119-162.
 * `state` is the bit-flipped CRC held in the Java field `crc` (:96). */
uint32_t orc_update(uint32_t state, const uint8_t *b, size_t len) {
    ensure_tables();
    uint32_t c = state;
    while (len > 7) { /* :122-138, 8 bytes per step */
        uint32_t c0 = (b[0] ^ c) & 0xffu;
        uint32_t c1 = (b[1] ^ (c >> 8)) & 0xffu;
        uint32_t c2 = (b[2] ^ (c >> 16)) & 0xffu;
        uint32_t c3 = (b[3] ^ (c >> 24)) & 0xffu;
        c = (T[7][c0] ^ T[6][c1]) ^ (T[5][c2] ^ T[4][c3]);
        c ^= (T[3][b[4]] ^ T[2][b[5]]) ^ (T[1][b[6]] ^ T[0][b[7]]);
        b += 8;
        len -= 8;
    }
    while (len > 0) { /* :141-158, byte-at-a-time tail */
        c = (c >> 8) ^ T[0][(c ^ *b++) & 0xffu];
        len--;
    }
    return c;
}

/* Crc32C.update(int b), J/util/Crc32C.java:165-167 */
uint32_t orc_update_byte(uint32_t state, uint32_t b) {
    ensure_tables();
    return (state >> 8) ^ T[0][(state ^ b) & 0xffu];
}

/* Crc32C.value, J/util/Crc32C.java:85-89 (reset :113-115, getValue :107-110) */
uint32_t orc_value(const uint8_t *b, size_t n) { return ~orc_update(0xffffffffu, b, n); }

/* Crc32C.extend, J/util/Crc32C.java:43-48 (setValue :103-105) */
uint32_t orc_extend(uint32_t init_crc, const uint8_t *b, size_t n) { return ~orc_update(~init_crc, b, n); }

/* Crc32C.mask / unmask, J/util/Crc32C.java:31,61-75 */
uint32_t orc_mask(uint32_t crc) { return ((crc >> 15) | (crc << 17)) + 0xa282ead8u; }
uint32_t orc_unmask(uint32_t masked) {
    uint32_t rot = masked - 0xa282ead8u;
    return (rot >> 17) | (rot << 15);
}

/* Independent second oracle: bit-serial reflected CRC-32C. */
uint32_t orc_bitwise(const uint8_t *b, size_t n) {
    uint32_t c = 0xffffffffu;
    for (size_t i = 0; i < n; i++) {
        c ^= b[i];
        for (int k = 0; k < 8; k++) c = (c >> 1) ^ ((c & 1u) ? ORC_POLY : 0u);
    }
    return ~c;
}

/* Coding.encodeFixedNat32Long / decodeFixedNat32Long, J/util/Coding.java:168-184,225-240 (LE) */
static void put_le32(uint8_t *p, uint32_t v) {
    p[0] = (uint8_t)v; p[1] = (uint8_t)(v >> 8); p[2] = (uint8_t)(v >> 16); p[3] = (uint8_t)(v >> 24);
}
static uint32_t get_le32(const uint8_t *p) {
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}

/* ---------------------------------------------------------------- batches */
#define ORC_FLAG_MASK 1u

typedef struct {
    const uint8_t *base;
    const uint64_t *off;
    const uint32_t *len;
    const uint32_t *init;
    const uint8_t *suffix;
    uint64_t block_bytes; /* fixed mode when off == NULL */
    uint64_t lo, hi;
    uint32_t flags;
    uint32_t *out;
} batch_job;

static void *batch_worker(void *arg) {
    batch_job *j = (batch_job *)arg;
    for (uint64_t i = j->lo; i < j->hi; i++) {
        const uint8_t *p;
        size_t n;
        if (j->off) { p = j->base + j->off[i]; n = j->len[i]; }
        else { p = j->base + i * j->block_bytes; n = (size_t)j->block_bytes; }
        uint32_t st = j->init ? ~j->init[i] : 0xffffffffu;
        st = orc_update(st, p, n);
        if (j->suffix) st = orc_update(st, &j->suffix[i], 1); /* TableBuilder.java:314-315 */
        uint32_t crc = ~st;
        j->out[i] = (j->flags & ORC_FLAG_MASK) ? orc_mask(crc) : crc;
    }
    return NULL;
}

static void run_batch(batch_job proto, uint64_t n, int threads) {
    ensure_tables();
    if (threads < 1) threads = 1;
    if ((uint64_t)threads > n) threads = n ? (int)n : 1;
    pthread_t tid[256];
    batch_job jobs[256];
    if (threads > 256) threads = 256;
    for (int t = 0; t < threads; t++) {
        jobs[t] = proto;
        jobs[t].lo = n * (uint64_t)t / (uint64_t)threads;
        jobs[t].hi = n * (uint64_t)(t + 1) / (uint64_t)threads;
        if (t) pthread_create(&tid[t], NULL, batch_worker, &jobs[t]);
    }
    batch_worker(&jobs[0]);
    for (int t = 1; t < threads; t++) pthread_join(tid[t], NULL);
}

/* Per-block (masked) CRC of descriptors (off, len[, init][, suffix]). */
void orc_batch(const uint8_t *base, const uint64_t *off, const uint32_t *len, const uint32_t *init,
               const uint8_t *suffix, uint64_t n, uint32_t flags, uint32_t *out, int threads) {
    batch_job j = {base, off, len, init, suffix, 0, 0, 0, flags, out};
    run_batch(j, n, threads);
}

/* Per-block (masked) CRC of n contiguous blocks of block_bytes each. */
void orc_fixed(const uint8_t *base, uint64_t block_bytes, uint64_t n, uint32_t flags, uint32_t *out, int threads) {
    batch_job j = {base, NULL, NULL, NULL, NULL, block_bytes, 0, 0, flags, out};
    run_batch(j, n, threads);
}

/* ------------------------------------------------------------ table block */
/* TableBuilder.writeRawBlock trailer, J/table/TableBuilder.java:305-323:
 * trailer = [type][LE32 mask(crc32c(block || type))] */
void orc_table_trailer(const uint8_t *block, uint64_t n, uint8_t type, uint8_t *trailer5) {
    uint32_t st = orc_update(0xffffffffu, block, n);
    trailer5[0] = type;
    st = orc_update(st, trailer5, 1);
    put_le32(trailer5 + 1, orc_mask(~st));
}

/* TableFormat.readBlock checksum test, J/table/TableFormat.java:207-218.
 * Returns 1 when unmask(LE32 @ n+1) == value(data, n+1). */
int orc_table_verify(const uint8_t *file, uint64_t off, uint64_t n) {
    const uint8_t *d = file + off;
    return orc_unmask(get_le32(d + n + 1)) == orc_value(d, n + 1);
}

/* --------------------------------------------------------------- log write */
/* LogFormat, J/db/LogFormat.java:28-54 */
#define K_BLOCK 32768u
#define K_HEADER 7u

/* LogWriter.addRecord/emitPhysicalRecord, J/db/LogWriter.java:51-161, applied to
 * n records (payload ranges in `src`).  `dest_length` is the initial file length
 * (LogWriter(dest, destLength) :80-84).  Writes the appended bytes to `out`
 * (capacity `cap`) and returns the number written, or (uint64_t)-1 on overflow. */
uint64_t orc_log_write(const uint8_t *src, const uint64_t *off, const uint32_t *len, uint64_t n,
                       uint64_t dest_length, uint8_t *out, uint64_t cap) {
    ensure_tables();
    uint32_t type_crc[5];
    for (uint8_t t = 0; t < 5; t++) type_crc[t] = orc_value(&t, 1); /* initTypeCrc :51-57 */
    uint64_t w = 0;
    uint32_t block_offset = (uint32_t)(dest_length % K_BLOCK);
    for (uint64_t r = 0; r < n; r++) {
        const uint8_t *ptr = src + off[r];
        uint32_t left = len[r];
        int begin = 1;
        do { /* :98-132 */
            uint32_t leftover = K_BLOCK - block_offset;
            if (leftover < K_HEADER) {
                if (leftover > 0) {
                    if (w + leftover > cap) return (uint64_t)-1;
                    memset(out + w, 0, leftover);
                    w += leftover;
                }
                block_offset = 0;
            }
            uint32_t avail = K_BLOCK - block_offset - K_HEADER;
            uint32_t frag = left < avail ? left : avail;
            int end = (left == frag);
            uint8_t type = (begin && end) ? 1 : begin ? 2 : end ? 4 : 3;
            /* emitPhysicalRecord :136-161 */
            if (w + K_HEADER + frag > cap) return (uint64_t)-1;
            uint8_t *h = out + w;
            h[4] = (uint8_t)(frag & 0xff);
            h[5] = (uint8_t)((frag >> 8) & 0xff);
            h[6] = type;
            put_le32(h, orc_mask(orc_extend(type_crc[type], ptr, frag)));
            memcpy(h + K_HEADER, ptr, frag);
            w += K_HEADER + frag;
            block_offset += K_HEADER + frag;
            ptr += frag;
            left -= frag;
            begin = 0;
        } while (left > 0);
    }
    return w;
}

/* ---------------------------------------------------------------- log read */
/* Physical record types returned by readPhysicalRecord (J/db/LogReader.java:80-98) */
enum { T_ZERO = 0, T_FULL = 1, T_FIRST = 2, T_MIDDLE = 3, T_LAST = 4, T_EOF = 5, T_BAD = 6 };

/* Corruption reasons (J/db/LogReader.java:181-250, 297-383) */
enum {
    R_BAD_LENGTH = 1,      /* "bad record length" */
    R_CHECKSUM = 2,        /* "checksum mismatch" */
    R_PARTIAL_1 = 3,       /* "partial record without end(1)" */
    R_PARTIAL_2 = 4,       /* "partial record without end(2)" */
    R_MISSING_START_1 = 5, /* "missing start of fragmented record(1)" */
    R_MISSING_START_2 = 6, /* "missing start of fragmented record(2)" */
    R_MIDDLE_ERROR = 7,    /* "error in middle of record" */
    R_UNKNOWN_TYPE = 8     /* "unknown record type N" (N in `aux`) */
};

typedef struct {
    uint64_t offset; /* lastRecordOffset for the record (J/db/LogReader.java:193,237) */
    uint64_t data_off; /* offset into the caller's record arena */
    uint64_t size;
} orc_record;

typedef struct {
    uint64_t bytes;
    uint32_t reason;
    uint32_t aux;
} orc_report;

typedef struct {
    const uint8_t *file;
    uint64_t file_size, file_pos; /* SequentialFile position */
    int checksum;
    uint64_t initial_offset;
    const uint8_t *buf; /* Slice buffer: data pointer and size */
    uint64_t buf_size;
    int eof;
    uint64_t last_record_offset, end_of_buffer_offset;
    int resyncing;
    /* outputs */
    orc_report *rep;
    uint64_t rep_n, rep_cap;
} log_reader;

static void report_drop(log_reader *r, uint64_t bytes, uint32_t reason, uint32_t aux) {
    /* reportDrop, J/db/LogReader.java:396-401 (signed arithmetic as in Java longs) */
    int64_t lhs = (int64_t)r->end_of_buffer_offset - (int64_t)r->buf_size - (int64_t)bytes;
    if (lhs >= (int64_t)r->initial_offset && r->rep_n < r->rep_cap) {
        r->rep[r->rep_n].bytes = bytes;
        r->rep[r->rep_n].reason = reason;
        r->rep[r->rep_n].aux = aux;
        r->rep_n++;
    } else if (lhs >= (int64_t)r->initial_offset) {
        r->rep_n++; /* count overflow so the caller can detect it */
    }
}

/* readPhysicalRecord, J/db/LogReader.java:297-383 */
static int read_physical(log_reader *r, const uint8_t **frag, uint64_t *frag_size) {
    for (;;) {
        if (r->buf_size < K_HEADER) {
            if (!r->eof) {
                uint64_t n = r->file_size - r->file_pos;
                if (n > K_BLOCK) n = K_BLOCK;
                r->buf = r->file + r->file_pos;
                r->buf_size = n;
                r->file_pos += n;
                r->end_of_buffer_offset += n;
                if (n < K_BLOCK) r->eof = 1;
                continue;
            }
            r->buf_size = 0;
            return T_EOF;
        }
        const uint8_t *h = r->buf;
        uint32_t length = (uint32_t)h[4] | ((uint32_t)h[5] << 8);
        uint32_t type = h[6];
        if (K_HEADER + (uint64_t)length > r->buf_size) {
            uint64_t drop = r->buf_size;
            r->buf_size = 0;
            if (!r->eof) {
                report_drop(r, drop, R_BAD_LENGTH, 0);
                return T_BAD;
            }
            return T_EOF;
        }
        if (type == T_ZERO && length == 0) {
            r->buf_size = 0;
            return T_BAD;
        }
        if (r->checksum) {
            uint32_t expected = orc_unmask(get_le32(h));
            uint32_t actual = orc_value(h + 6, 1 + (size_t)length);
            if (actual != expected) {
                uint64_t drop = r->buf_size;
                r->buf_size = 0;
                report_drop(r, drop, R_CHECKSUM, 0);
                return T_BAD;
            }
        }
        r->buf += K_HEADER + length;
        r->buf_size -= K_HEADER + length;
        if ((int64_t)r->end_of_buffer_offset - (int64_t)r->buf_size - (int64_t)K_HEADER - (int64_t)length <
            (int64_t)r->initial_offset) {
            *frag_size = 0;
            return T_BAD;
        }
        *frag = h + K_HEADER;
        *frag_size = length;
        return (int)type;
    }
}

/* LogReader.readRecord loop (J/db/LogReader.java:146-252) over a whole file.
 * Logical records are appended to `arena` (capacity arena_cap) and described in
 * `recs` (capacity rec_cap).  Returns the number of records; reports go to `rep`.
 * *n_reports gets the number of reports.  Returns (uint64_t)-1 on overflow. */
uint64_t orc_log_read(const uint8_t *file, uint64_t file_size, int checksum, uint64_t initial_offset,
                      uint8_t *arena, uint64_t arena_cap, orc_record *recs, uint64_t rec_cap,
                      orc_report *rep, uint64_t rep_cap, uint64_t *n_reports) {
    log_reader r;
    memset(&r, 0, sizeof(r));
    r.file = file;
    r.file_size = file_size;
    r.checksum = checksum;
    r.initial_offset = initial_offset;
    r.resyncing = initial_offset > 0;
    r.rep = rep;
    r.rep_cap = rep_cap;
    uint64_t nrec = 0, arena_used = 0;
    int overflow = 0;

    /* skipToInitialBlock, :263-289 (called when lastRecordOffset < initialOffset) */
    if (r.last_record_offset < r.initial_offset) {
        uint64_t in_block = initial_offset % K_BLOCK;
        uint64_t start = initial_offset - in_block;
        if (in_block > K_BLOCK - 6) { in_block = 0; start += K_BLOCK; }
        r.end_of_buffer_offset = start;
        if (start > 0) {
            if (start > file_size) start = file_size; /* skip past EOF: reads then return 0 bytes */
            r.file_pos = start;
        }
    }

    for (;;) { /* one iteration per readRecord() call */
        uint64_t scratch_start = arena_used, scratch_size = 0;
        int in_frag = 0;
        uint64_t prospective = 0;
        const uint8_t *frag = NULL;
        uint64_t frag_size = 0;
        int got = 0, done = 0;
        while (!got && !done) {
            int type = read_physical(&r, &frag, &frag_size);
            uint64_t phys_off = r.end_of_buffer_offset - r.buf_size - K_HEADER - frag_size;
            if (r.resyncing) {
                if (type == T_MIDDLE) continue;
                if (type == T_LAST) { r.resyncing = 0; continue; }
                r.resyncing = 0;
            }
            switch (type) {
            case T_FULL:
                if (in_frag) {
                    if (scratch_size == 0) in_frag = 0;
                    else report_drop(&r, scratch_size, R_PARTIAL_1, 0);
                }
                prospective = phys_off;
                scratch_size = 0;
                if (arena_used + frag_size > arena_cap || nrec >= rec_cap) { overflow = 1; done = 1; break; }
                memcpy(arena + scratch_start, frag, frag_size);
                recs[nrec].offset = prospective;
                recs[nrec].data_off = scratch_start;
                recs[nrec].size = frag_size;
                nrec++;
                arena_used = scratch_start + frag_size;
                r.last_record_offset = prospective;
                got = 1;
                break;
            case T_FIRST:
                if (in_frag) {
                    if (scratch_size == 0) in_frag = 0;
                    else report_drop(&r, scratch_size, R_PARTIAL_2, 0);
                }
                prospective = phys_off;
                if (scratch_start + frag_size > arena_cap) { overflow = 1; done = 1; break; }
                memcpy(arena + scratch_start, frag, frag_size);
                scratch_size = frag_size;
                in_frag = 1;
                break;
            case T_MIDDLE:
                if (!in_frag) report_drop(&r, frag_size, R_MISSING_START_1, 0);
                else {
                    if (scratch_start + scratch_size + frag_size > arena_cap) { overflow = 1; done = 1; break; }
                    memcpy(arena + scratch_start + scratch_size, frag, frag_size);
                    scratch_size += frag_size;
                }
                break;
            case T_LAST:
                if (!in_frag) report_drop(&r, frag_size, R_MISSING_START_2, 0);
                else {
                    if (scratch_start + scratch_size + frag_size > arena_cap || nrec >= rec_cap) {
                        overflow = 1; done = 1; break;
                    }
                    memcpy(arena + scratch_start + scratch_size, frag, frag_size);
                    scratch_size += frag_size;
                    recs[nrec].offset = prospective;
                    recs[nrec].data_off = scratch_start;
                    recs[nrec].size = scratch_size;
                    nrec++;
                    arena_used = scratch_start + scratch_size;
                    r.last_record_offset = prospective;
                    got = 1;
                }
                break;
            case T_EOF:
                done = 1;
                break;
            case T_BAD:
                if (in_frag) {
                    report_drop(&r, scratch_size, R_MIDDLE_ERROR, 0);
                    in_frag = 0;
                    scratch_size = 0;
                }
                break;
            default:
                report_drop(&r, frag_size + (in_frag ? scratch_size : 0), R_UNKNOWN_TYPE, (uint32_t)type);
                in_frag = 0;
                scratch_size = 0;
                break;
            }
        }
        if (done) break;
    }
    *n_reports = r.rep_n;
    if (overflow || r.rep_n > rep_cap) return (uint64_t)-1;
    return nrec;
}

/* Physical-record events of readPhysicalRecord over the whole file, block by
 * block (what the device log walk + verify must reproduce).  Kinds:
 *   1 OK, 2 BAD_CRC (rest of block dropped), 3 BAD_LENGTH (rest dropped, reported),
 *   4 ZERO_SKIP (rest skipped silently), 5 EOF_BAD_LENGTH (eof, not reported),
 *   6 EOF_TRUNC_HEADER (eof with 1..6 stray bytes).
 * Each event: offset of the header, length field, type byte, kind. */
typedef struct {
    uint64_t offset;
    uint32_t length;
    uint8_t type;
    uint8_t kind;
    uint16_t pad;
} orc_event;

uint64_t orc_log_events(const uint8_t *file, uint64_t size, int checksum, orc_event *ev, uint64_t cap) {
    ensure_tables();
    uint64_t ne = 0;
    for (uint64_t bs = 0; bs < size; bs += K_BLOCK) {
        uint64_t be = bs + K_BLOCK < size ? bs + K_BLOCK : size;
        int eof = (be - bs) < K_BLOCK;
        uint64_t p = bs;
        for (;;) {
            uint64_t rem = be - p;
            if (rem < K_HEADER) {
                if (eof && rem > 0) {
                    if (ne < cap) { ev[ne].offset = p; ev[ne].length = 0; ev[ne].type = 0; ev[ne].kind = 6; }
                    ne++;
                }
                break;
            }
            const uint8_t *h = file + p;
            uint32_t length = (uint32_t)h[4] | ((uint32_t)h[5] << 8);
            uint8_t type = h[6];
            uint8_t kind = 1;
            int stop = 0;
            if (K_HEADER + (uint64_t)length > rem) { kind = eof ? 5 : 3; stop = 1; }
            else if (type == 0 && length == 0) { kind = 4; stop = 1; }
            else if (checksum && orc_unmask(get_le32(h)) != orc_value(h + 6, 1 + (size_t)length)) { kind = 2; stop = 1; }
            if (ne < cap) { ev[ne].offset = p; ev[ne].length = length; ev[ne].type = type; ev[ne].kind = kind; ev[ne].pad = 0; }
            ne++;
            if (stop) break;
            p += K_HEADER + length;
        }
    }
    return ne;
}

/* splitmix64 byte generator shared with the device generator (fixture shape). */
void orc_fill_splitmix(uint8_t *dst, uint64_t bytes, uint64_t seed, uint64_t first_word) {
    uint64_t i = 0;
    for (; i + 8 <= bytes; i += 8) {
        uint64_t z = seed + (first_word + i / 8 + 1) * 0x9E3779B97F4A7C15ull;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        z ^= z >> 31;
        memcpy(dst + i, &z, 8);
    }
    if (i < bytes) {
        uint64_t z = seed + (first_word + i / 8 + 1) * 0x9E3779B97F4A7C15ull;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        z ^= z >> 31;
        memcpy(dst + i, &z, bytes - i);
    }
}
