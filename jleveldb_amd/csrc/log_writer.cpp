// log_writer.cpp — framing plan of LogWriter.addRecord (J/db/LogWriter.java:88-134)
// for a batch of records: where every physical fragment's 7-byte header goes,
// which payload bytes it carries and its record type.  No checksum work here:
// the headers' masked CRCs are computed on the device by jl_log_emit_dev /
// jl_log_headers_dev (emitPhysicalRecord, :136-161).
#include <cstdint>

#include "../../include/jlcrc.h"

namespace {
constexpr uint32_t kBlockSize = 32768;  // LogFormat.kBlockSize, J/db/LogFormat.java:52
constexpr uint32_t kHeaderSize = 7;     // LogFormat.kHeaderSize, :54
enum : uint8_t { kFull = 1, kFirst = 2, kMiddle = 3, kLast = 4 };
}  // namespace

extern "C" int jl_log_layout(const uint64_t *rec_src_off, const uint32_t *rec_len, uint64_t n, uint64_t dest_length,
                             uint64_t *frag_hdr_off, uint64_t *frag_src_off, uint32_t *frag_len, uint8_t *frag_type,
                             uint64_t cap, uint64_t *n_frags, uint64_t *log_bytes) {
    if (!n_frags || !log_bytes || (n && (!rec_src_off || !rec_len))) return JL_ERR_INVALID;
    uint32_t block_offset = (uint32_t)(dest_length % kBlockSize);  // LogWriter(dest, destLength) :80-84
    uint64_t w = 0, f = 0;
    for (uint64_t r = 0; r < n; r++) {
        uint64_t src = rec_src_off[r];
        uint32_t left = rec_len[r];
        bool begin = true;
        do {  // :98-132
            const uint32_t leftover = kBlockSize - block_offset;
            if (leftover < kHeaderSize) {  // switch to a new block; trailer zero-filled :101-107
                w += leftover;
                block_offset = 0;
            }
            const uint32_t avail = kBlockSize - block_offset - kHeaderSize;
            const uint32_t frag = left < avail ? left : avail;
            const bool end = left == frag;
            const uint8_t type = (begin && end) ? kFull : begin ? kFirst : end ? kLast : kMiddle;
            if (f < cap) {
                frag_hdr_off[f] = w;
                frag_src_off[f] = src;
                frag_len[f] = frag;
                frag_type[f] = type;
            }
            f++;
            w += kHeaderSize + frag;
            block_offset += kHeaderSize + frag;
            src += frag;
            left -= frag;
            begin = false;
        } while (left > 0);
    }
    *n_frags = f;
    *log_bytes = w;
    return f > cap ? JL_ERR_CAPACITY : JL_OK;
}
