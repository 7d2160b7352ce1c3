// fuzz_host.cpp — AddressSanitizer / UndefinedBehaviorSanitizer harness for
// the engine's host-side code (test infrastructure only; built and run by
// tests/test_sanitize.py through tests/cpp/Makefile).
//
// Compiled with -fsanitize=address,undefined together with the product's host
// translation units — table_walker.cpp (jl_table_block_handles), log_writer.cpp
// (jl_log_layout), log_reader.cpp (jl_log_read_records), host_crc.cpp (the
// scalar Crc32C statics) — and the oracle (oracle/crc32c_oracle.c).  The one
// device call on these paths, jl_log_verify inside jl_log_read_records, is
// served here by the oracle's readPhysicalRecord walk (the GPU path's parity
// with that walk is what the -m gpu tests check), so the reader's bookkeeping
// runs under the sanitizers on the CPU.
//
// Inputs are every buffer sized exactly (heap vectors), so any read past an
// input is an ASan report:
//   * SSTable images (tests/golden/sstable.bin, table.bin) with random byte
//     flips, truncations and spliced garbage, walked at several capacities;
//   * log-writer plans for random record sets (0 B .. 100 KiB, lengths at the
//     32 KiB block edges, any dest_length), assembled into bytes and compared
//     with the oracle's LogWriter (orc_log_write);
//   * logs from orc_log_write, corrupted, read back with jl_log_read_records at
//     random initial offsets and capacities and compared record for record and
//     report for report with the oracle's LogReader (orc_log_read);
//   * the oracle's own walks (orc_log_events, orc_table_verify, orc_batch) on
//     random bytes;
//   * the small-call host paths (host_paths.cpp, JL_OPT_HOST_THRESHOLD): the
//     log walk on corrupted / random logs event for event, table verify and
//     batch (init, suffix, mask) block for block, against the oracle.
// Usage: fuzz_host <iterations> <sstable.bin> <table.bin>   (prints "OK n" on success)
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#include "../../include/jlcrc.h"
#include "host_paths.hpp"

extern "C" {
typedef struct {
    uint64_t offset;
    uint32_t length;
    uint8_t type, kind;
    uint16_t pad;
} orc_event;
uint32_t orc_value(const uint8_t *b, size_t n);
uint32_t orc_extend(uint32_t init_crc, const uint8_t *b, size_t n);
uint32_t orc_mask(uint32_t crc);
void orc_batch(const uint8_t *base, const uint64_t *off, const uint32_t *len, const uint32_t *init,
               const uint8_t *suffix, uint64_t n, uint32_t flags, uint32_t *out, int threads);
int orc_table_verify(const uint8_t *file, uint64_t off, uint64_t n);
uint64_t orc_log_write(const uint8_t *src, const uint64_t *off, const uint32_t *len, uint64_t n, uint64_t dest_length,
                       uint8_t *out, uint64_t cap);
uint64_t orc_log_read(const uint8_t *file, uint64_t file_size, int checksum, uint64_t initial_offset, uint8_t *arena,
                      uint64_t arena_cap, jl_log_record *recs, uint64_t rec_cap, jl_log_report *rep, uint64_t rep_cap,
                      uint64_t *n_reports);
uint64_t orc_log_events(const uint8_t *file, uint64_t size, int checksum, orc_event *ev, uint64_t cap);
}

// ---- stand-ins for the two engine symbols these translation units call
static std::string g_err;
void jl_set_error(const std::string &msg) { g_err = msg; }

extern "C" int jl_log_verify(const uint8_t *log, uint64_t log_bytes, int checksum, jl_log_event *events, uint64_t cap,
                             uint64_t *n_events) {
    static_assert(sizeof(orc_event) == sizeof(jl_log_event), "event layout");
    std::vector<orc_event> ev(log_bytes / 7 + 2);
    const uint64_t n = orc_log_events(log, log_bytes, checksum != 0, ev.data(), ev.size());
    *n_events = n;
    if (n > cap) return JL_ERR_CAPACITY;
    if (n) memcpy(events, ev.data(), n * sizeof(jl_log_event));
    return JL_OK;
}

// ---- helpers
static std::mt19937_64 rng(0x4A4C4442);
static uint64_t rnd(uint64_t n) { return n ? rng() % n : 0; }

#define CHECK(c)                                                                     \
    do {                                                                             \
        if (!(c)) {                                                                  \
            fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c);     \
            exit(1);                                                                 \
        }                                                                            \
    } while (0)

static std::vector<uint8_t> read_file(const char *path) {
    std::vector<uint8_t> v;
    FILE *f = fopen(path, "rb");
    CHECK(f != nullptr);
    uint8_t buf[65536];
    size_t k;
    while ((k = fread(buf, 1, sizeof(buf), f)) > 0) v.insert(v.end(), buf, buf + k);
    fclose(f);
    return v;
}

static void mutate(std::vector<uint8_t> &v) {
    const int m = 1 + (int)rnd(6);
    for (int i = 0; i < m && !v.empty(); i++) {
        switch (rnd(5)) {
        case 0: v[rnd(v.size())] ^= (uint8_t)(1u << rnd(8)); break;
        case 1: v[rnd(v.size())] = (uint8_t)rng(); break;
        case 2: v.resize(rnd(v.size() + 1)); break;  // truncate
        case 3: {                                    // garbage run
            const size_t at = rnd(v.size()), len = std::min<size_t>(v.size() - at, 1 + rnd(64));
            for (size_t j = 0; j < len; j++) v[at + j] = (uint8_t)rng();
            break;
        }
        default: {  // zero run (a torn write)
            const size_t at = rnd(v.size()), len = std::min<size_t>(v.size() - at, 1 + rnd(40000));
            memset(v.data() + at, 0, len);
        }
        }
    }
}

// ---- table walker
static void fuzz_table(const std::vector<uint8_t> &seed) {
    std::vector<uint8_t> f = seed;
    if (rnd(4)) mutate(f);
    // exactly-sized heap copy (an empty image is a distinct allocation too)
    uint8_t *img = (uint8_t *)malloc(f.size() ? f.size() : 1);
    if (!f.empty()) memcpy(img, f.data(), f.size());
    static const uint64_t caps[] = {0, 1, 3, 4096};
    const uint64_t cap = caps[rnd(4)];
    std::vector<uint64_t> off(cap ? cap : 1);
    std::vector<uint32_t> size(cap ? cap : 1);
    std::vector<uint8_t> kind(cap ? cap : 1);
    uint64_t n = 0;
    int rc = jl_table_block_handles(img, f.size(), cap ? off.data() : nullptr, cap ? size.data() : nullptr,
                                    kind.data(), cap, &n);
    CHECK(rc == JL_OK || rc == JL_ERR_CORRUPT || rc == JL_ERR_CAPACITY || rc == JL_ERR_INVALID);
    if (rc == JL_ERR_CAPACITY) {
        CHECK(n > cap);
        off.assign(n, 0);
        size.assign(n, 0);
        kind.assign(n, 0);
        uint64_t n2 = 0;
        rc = jl_table_block_handles(img, f.size(), off.data(), size.data(), kind.data(), n, &n2);
        CHECK(rc == JL_OK && n2 == n);
    }
    if (rc == JL_OK)
        for (uint64_t i = 0; i < n; i++) {
            CHECK(off[i] + size[i] + 5 <= f.size());  // every handle lies in the file with its trailer
            (void)orc_table_verify(img, off[i], size[i]);
        }
    free(img);
}

// ---- log writer: the plan assembled into bytes equals the oracle's LogWriter
static void fuzz_layout() {
    const uint64_t n = rnd(40);
    std::vector<uint32_t> len(n);
    std::vector<uint64_t> src(n);
    uint64_t total = 0;
    for (uint64_t r = 0; r < n; r++) {
        switch (rnd(4)) {
        case 0: len[r] = (uint32_t)rnd(64); break;
        case 1: len[r] = 32768 - 7 - 3 + (uint32_t)rnd(7); break;  // ends at / near a block edge
        case 2: len[r] = (uint32_t)rnd(100000); break;
        default: len[r] = (uint32_t)rnd(4096);
        }
        src[r] = total;
        total += len[r];
    }
    std::vector<uint8_t> payload(total ? total : 1);
    for (auto &b : payload) b = (uint8_t)rng();
    const uint64_t dest = rnd(3) ? rnd(5 * 32768) : 32768 - rnd(8);
    uint64_t nf = 0, lb = 0;
    int rc = jl_log_layout(src.data(), len.data(), n, dest, nullptr, nullptr, nullptr, nullptr, 0, &nf, &lb);
    CHECK(rc == (nf ? JL_ERR_CAPACITY : JL_OK));
    std::vector<uint64_t> ho(nf ? nf : 1), so(nf ? nf : 1);
    std::vector<uint32_t> fl(nf ? nf : 1);
    std::vector<uint8_t> ft(nf ? nf : 1);
    if (nf > 1) {  // a short plan array: capacity error, nothing written past it
        uint64_t nf2 = 0, lb2 = 0;
        CHECK(jl_log_layout(src.data(), len.data(), n, dest, ho.data(), so.data(), fl.data(), ft.data(), nf - 1, &nf2,
                            &lb2) == JL_ERR_CAPACITY &&
              nf2 == nf && lb2 == lb);
    }
    CHECK(jl_log_layout(src.data(), len.data(), n, dest, ho.data(), so.data(), fl.data(), ft.data(), nf, &nf, &lb) ==
          JL_OK);
    std::vector<uint8_t> log(lb ? lb : 1, 0);
    uint32_t type_crc[5];
    for (uint8_t t = 0; t < 5; t++) type_crc[t] = orc_value(&t, 1);
    for (uint64_t f = 0; f < nf; f++) {
        CHECK(ho[f] + 7 + fl[f] <= lb && fl[f] <= 0xffff && ft[f] >= 1 && ft[f] <= 4);
        uint8_t *h = log.data() + ho[f];
        const uint32_t crc = orc_mask(orc_extend(type_crc[ft[f]], payload.data() + so[f], fl[f]));
        for (int j = 0; j < 4; j++) h[j] = (uint8_t)(crc >> (8 * j));
        h[4] = (uint8_t)fl[f];
        h[5] = (uint8_t)(fl[f] >> 8);
        h[6] = ft[f];
        memcpy(h + 7, payload.data() + so[f], fl[f]);
    }
    std::vector<uint8_t> want(lb + 64);
    const uint64_t w = orc_log_write(payload.data(), src.data(), len.data(), n, dest, want.data(), want.size());
    CHECK(w == lb && (lb == 0 || memcmp(want.data(), log.data(), lb) == 0));
}

// ---- log reader vs the oracle's LogReader
static void fuzz_reader() {
    const uint64_t n = rnd(60);
    std::vector<uint32_t> len(n);
    std::vector<uint64_t> src(n);
    uint64_t total = 0;
    for (uint64_t r = 0; r < n; r++) {
        len[r] = rnd(3) ? (uint32_t)rnd(2000) : (uint32_t)rnd(70000);
        src[r] = total;
        total += len[r];
    }
    std::vector<uint8_t> payload(total ? total : 1);
    for (auto &b : payload) b = (uint8_t)rng();
    std::vector<uint8_t> buf(total + 7 * (2 * n + total / 32761 + 2) + 32768);
    const uint64_t lb = orc_log_write(payload.data(), src.data(), len.data(), n, 0, buf.data(), buf.size());
    CHECK(lb != ~0ull);
    std::vector<uint8_t> log(buf.begin(), buf.begin() + lb);
    if (rnd(3)) mutate(log);
    uint8_t *img = (uint8_t *)malloc(log.size() ? log.size() : 1);
    if (!log.empty()) memcpy(img, log.data(), log.size());
    const uint64_t init_off = rnd(2) ? 0 : rnd(log.size() + 40000);
    const int checksum = (int)rnd(2);
    const uint64_t arena_cap = rnd(4) ? log.size() + 1 : rnd(log.size() + 1);
    const uint64_t rec_cap = rnd(4) ? n + 1 : rnd(n + 1);
    const uint64_t rep_cap = rnd(4) ? 4 * (log.size() / 32768 + 2) + n : rnd(4);
    std::vector<uint8_t> arena(arena_cap ? arena_cap : 1), arena2(arena_cap ? arena_cap : 1);
    std::vector<jl_log_record> rec(rec_cap ? rec_cap : 1), rec2(rec_cap ? rec_cap : 1);
    std::vector<jl_log_report> rep(rep_cap ? rep_cap : 1), rep2(rep_cap ? rep_cap : 1);
    uint64_t nr = 0, np = 0, np2 = 0;
    const int rc = jl_log_read_records(log.empty() ? nullptr : img, log.size(), checksum, init_off, arena.data(),
                                       arena_cap, rec.data(), rec_cap, &nr, rep.data(), rep_cap, &np);
    CHECK(rc == JL_OK || rc == JL_ERR_CAPACITY);
    const uint64_t nr2 = orc_log_read(img, log.size(), checksum, init_off, arena2.data(), arena_cap, rec2.data(),
                                      rec_cap, rep2.data(), rep_cap, &np2);
    if (rc == JL_OK) {
        CHECK(nr2 == nr && np2 == np);
        for (uint64_t i = 0; i < nr; i++) {
            CHECK(rec[i].offset == rec2[i].offset && rec[i].size == rec2[i].size);
            CHECK(memcmp(arena.data() + rec[i].arena_off, arena2.data() + rec2[i].arena_off, rec[i].size) == 0);
        }
        for (uint64_t i = 0; i < np; i++) CHECK(rep[i].bytes == rep2[i].bytes && rep[i].reason == rep2[i].reason);
    }
    free(img);
}

// ---- the oracle's own walks on random bytes
static void fuzz_oracle() {
    std::vector<uint8_t> b(rnd(3 * 32768 + 10));
    for (auto &x : b) x = rnd(4) ? 0 : (uint8_t)rng();
    std::vector<orc_event> ev(b.size() / 7 + 2);
    (void)orc_log_events(b.data(), b.size(), (int)rnd(2), ev.data(), ev.size());
    const uint64_t n = 1 + rnd(50);
    std::vector<uint64_t> off(n);
    std::vector<uint32_t> len(n), init(n), out(n);
    std::vector<uint8_t> sfx(n);
    for (uint64_t i = 0; i < n; i++) {
        off[i] = rnd(b.size() + 1);
        len[i] = (uint32_t)rnd(b.size() - off[i] + 1);
        init[i] = (uint32_t)rng();
        sfx[i] = (uint8_t)rng();
    }
    orc_batch(b.data(), off.data(), len.data(), rnd(2) ? init.data() : nullptr, rnd(2) ? sfx.data() : nullptr, n, 1,
              out.data(), 1 + (int)rnd(3));
    for (uint64_t i = 0; i < n; i++) CHECK(out[i] == out[i]);
    if (b.size() > 5) (void)orc_table_verify(b.data(), 0, b.size() - 5);
}

// ---- host paths (the small-call dispatch) vs the oracle
static void fuzz_host_paths() {
    // a log: LogWriter records (dense or sparse), corrupted, or random bytes
    std::vector<uint8_t> log;
    if (rnd(4)) {
        const uint64_t n = rnd(400);
        std::vector<uint32_t> len(n);
        std::vector<uint64_t> src(n);
        uint64_t total = 0;
        const uint32_t mx = rnd(2) ? 40 : (rnd(2) ? 2000 : 70000);
        for (uint64_t r = 0; r < n; r++) {
            len[r] = (uint32_t)rnd(mx);
            src[r] = total;
            total += len[r];
        }
        std::vector<uint8_t> payload(total ? total : 1);
        for (auto &b : payload) b = (uint8_t)rng();
        std::vector<uint8_t> buf(total + 7 * (2 * n + total / 32761 + 2) + 32768);
        const uint64_t lb = orc_log_write(payload.data(), src.data(), len.data(), n, 0, buf.data(), buf.size());
        CHECK(lb != ~0ull);
        log.assign(buf.begin(), buf.begin() + lb);
        if (rnd(3)) mutate(log);
    } else {
        log.resize(rnd(3 * 32768 + 10));
        for (auto &x : log) x = rnd(4) ? 0 : (uint8_t)rng();
    }
    uint8_t *img = (uint8_t *)malloc(log.size() ? log.size() : 1);
    if (!log.empty()) memcpy(img, log.data(), log.size());
    const int checksum = (int)rnd(2);
    std::vector<orc_event> want(log.size() / 7 + 2);
    const uint64_t wn = orc_log_events(img, log.size(), checksum, want.data(), want.size());
    // the engine's event form counts the events a failing crc drops (kind 0, as
    // the device path does); the oracle stops the block there: compare the live ones
    uint64_t gn = 0;
    jlhost::log_verify(img, log.size(), checksum, nullptr, 0, &gn);
    CHECK(gn >= wn);
    const uint64_t cap = rnd(4) ? gn : rnd(gn + 1);
    std::vector<jl_log_event> got(cap ? cap : 1);
    uint64_t gn2 = 0;
    jlhost::log_verify(img, log.size(), checksum, got.data(), cap, &gn2);
    CHECK(gn2 == gn);
    if (cap == gn) {
        uint64_t j = 0;
        for (uint64_t i = 0; i < gn; i++) {
            if (got[i].kind == 0) continue;
            CHECK(j < wn);
            CHECK(got[i].offset == want[j].offset && got[i].length == want[j].length && got[i].type == want[j].type &&
                  got[i].kind == want[j].kind);
            j++;
        }
        CHECK(j == wn);
    }
    // blocks of the log bytes: table verify (with planted trailers) and batch
    const uint64_t n = 1 + rnd(40);
    std::vector<uint64_t> off(n);
    std::vector<uint32_t> len(n), init(n), out(n), ref(n);
    std::vector<uint8_t> sfx(n), st(n);
    std::vector<uint8_t> b(log.size() + 6);
    memcpy(b.data(), img, log.size());
    for (uint64_t i = 0; i < n; i++) {
        off[i] = rnd(b.size() - 5);
        len[i] = (uint32_t)rnd(b.size() - 5 - off[i] + 1);
        init[i] = (uint32_t)rng();
        sfx[i] = (uint8_t)rng();
    }
    const uint32_t flags = (uint32_t)rnd(2);
    const bool wi = rnd(2), ws = rnd(2);
    jlhost::batch(b.data(), off.data(), len.data(), wi ? init.data() : nullptr, ws ? sfx.data() : nullptr, n, flags,
                  out.data());
    orc_batch(b.data(), off.data(), len.data(), wi ? init.data() : nullptr, ws ? sfx.data() : nullptr, n, flags,
              ref.data(), 1);
    CHECK(out == ref);
    for (uint64_t i = 0; i < n; i++) {  // table blocks: handle (off, size) with size + 5 inside the buffer
        if (len[i] > 0 && rnd(2)) {
            const uint32_t sz = len[i] - 1;
            const uint32_t m = orc_mask(orc_value(b.data() + off[i], (size_t)sz + 1));
            if (off[i] + sz + 5 <= b.size()) memcpy(b.data() + off[i] + sz + 1, &m, 4);
        }
    }
    std::vector<uint32_t> tsz(n);
    for (uint64_t i = 0; i < n; i++) {
        tsz[i] = len[i] ? len[i] - 1 : 0;
        if (off[i] + tsz[i] + 5 > b.size()) off[i] = 0, tsz[i] = 0;
    }
    jlhost::table_verify(b.data(), off.data(), tsz.data(), n, st.data());
    for (uint64_t i = 0; i < n; i++) CHECK(st[i] == (orc_table_verify(b.data(), off[i], tsz[i]) ? 1 : 0));
    free(img);
}

int main(int argc, char **argv) {
    if (argc < 4) {
        fprintf(stderr, "usage: %s iterations sstable.bin table.bin\n", argv[0]);
        return 2;
    }
    const long iters = atol(argv[1]);
    const std::vector<uint8_t> t1 = read_file(argv[2]), t2 = read_file(argv[3]);
    for (long i = 0; i < iters; i++) {
        fuzz_table(i & 1 ? t1 : t2);
        if (i % 4 == 0) fuzz_layout();
        if (i % 4 == 1) fuzz_reader();
        if (i % 4 == 2) fuzz_oracle();
        if (i % 4 == 3) fuzz_host_paths();
        // the scalar statics on odd lengths / alignments
        std::vector<uint8_t> s(rnd(300));
        for (auto &x : s) x = (uint8_t)rng();
        const size_t a = rnd(s.size() + 1);
        CHECK(jl_crc32c_value(s.data() + a, s.size() - a) == orc_value(s.data() + a, s.size() - a));
        CHECK(jl_crc32c_extend(0x1234u, s.data(), s.size()) == orc_extend(0x1234u, s.data(), s.size()));
    }
    printf("OK %ld\n", iters);
    return 0;
}
