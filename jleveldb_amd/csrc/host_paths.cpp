// host_paths.cpp — the small-call dispatch of the host-memory entry points
// (JL_OPT_HOST_THRESHOLD, include/jlcrc.h): a call whose input is smaller than
// the threshold is verified on the calling thread with the product's SSE4.2
// scalar path (host_crc.cpp) instead of paying the device round trip (H2D copy,
// launches, D2H, synchronisation).  Results are bit-identical to the device
// path; the oracle is not involved (it is test infrastructure).
//
// The reference verifies at this granularity: one table of <= 2 MiB when it is
// opened (Options.java:208, TableCache.java:198-208), one WAL of <= 4 MiB at
// recovery (Options.java:203, DBImpl.java:903) — the batch shapes the
// threshold is measured on (bench.py "dispatch").
#include <cstdint>
#include <cstring>

#include "../../include/jlcrc.h"
#include "host_paths.hpp"

namespace jlhost {

static inline uint32_t le32(const uint8_t *p) {
    uint32_t v;
    memcpy(&v, p, 4);
    return v;
}

// jl_crc32c_batch: crc (or mask(crc)) of block i = extend(init[i], block) then
// the suffix byte (TableBuilder's type byte); ranges checked by the caller
void batch(const uint8_t *base, const uint64_t *off, const uint32_t *len, const uint32_t *init, const uint8_t *suffix,
           uint64_t n, uint32_t flags, uint32_t *out) {
    for (uint64_t i = 0; i < n; i++) {
        uint32_t s = ~(init ? init[i] : 0u);
        s = jl_crc32c_update(s, base + off[i], len[i]);
        if (suffix) s = jl_crc32c_update(s, suffix + i, 1);
        const uint32_t crc = ~s;
        out[i] = (flags & JL_FLAG_MASK) ? jl_crc32c_mask(crc) : crc;
    }
}

void fixed(const uint8_t *data, uint64_t block_bytes, uint64_t n, uint32_t flags, uint32_t *out) {
    for (uint64_t i = 0; i < n; i++) {
        const uint32_t crc = jl_crc32c_value(data + i * block_bytes, block_bytes);
        out[i] = (flags & JL_FLAG_MASK) ? jl_crc32c_mask(crc) : crc;
    }
}

// TableFormat.readBlock's test (J/table/TableFormat.java:207-218); ranges checked by the caller
void table_verify(const uint8_t *file, const uint64_t *off, const uint32_t *size, uint64_t n, uint8_t *status) {
    for (uint64_t i = 0; i < n; i++) {
        const uint8_t *b = file + off[i];
        status[i] = jl_crc32c_unmask(le32(b + size[i] + 1)) == jl_crc32c_value(b, (size_t)size[i] + 1) ? 1 : 0;
    }
}

// LogReader.readPhysicalRecord's decisions over every 32 KiB block
// (J/db/LogReader.java:297-383), in the engine's event form: every decision of
// the header walk is an event; with checksum the first OK record of a block
// whose crc fails becomes BAD_CRC and the block's later events kind 0 (the
// reader drops the rest of the block, :359-367).  Counts every event; writes the
// first `cap`.
void log_verify(const uint8_t *log, uint64_t bytes, int checksum, jl_log_event *ev, uint64_t cap, uint64_t *n_events) {
    uint64_t n = 0;
    for (uint64_t bs = 0; bs < bytes; bs += 32768) {
        const uint64_t be = bs + 32768 < bytes ? bs + 32768 : bytes;
        const bool eof = be - bs < 32768;
        bool dropped = false;  // a record of this block failed its crc
        for (uint64_t p = bs;;) {
            const uint64_t rem = be - p;
            jl_log_event e{p, 0, 0, 0, 0};
            bool stop = true;
            if (rem < 7) {  // :315-322 (fewer than kHeaderSize bytes left)
                if (!(eof && rem > 0)) break;  // the block's trailer: no event
                e.kind = JL_LOG_EOF_TRUNC;
            } else {
                e.length = (uint32_t)log[p + 4] | (uint32_t)log[p + 5] << 8;
                e.type = log[p + 6];
                if (7 + (uint64_t)e.length > rem) {  // :334-345
                    e.kind = eof ? JL_LOG_EOF_BAD_LENGTH : JL_LOG_BAD_LENGTH;
                } else if (e.type == 0 && e.length == 0) {  // :347-353
                    e.kind = JL_LOG_ZERO_SKIP;
                } else {
                    e.kind = JL_LOG_OK;
                    stop = false;
                }
            }
            if (dropped) {
                e.kind = 0;
            } else if (e.kind == JL_LOG_OK && checksum &&  // :356-369: crc over type || payload
                       jl_crc32c_unmask(le32(log + p)) != jl_crc32c_value(log + p + 6, 1 + (size_t)e.length)) {
                e.kind = JL_LOG_BAD_CRC;
                dropped = true;
            }
            if (n < cap) ev[n] = e;
            n++;
            if (stop) break;
            p += 7 + e.length;
        }
    }
    *n_events = n;
}

}  // namespace jlhost
