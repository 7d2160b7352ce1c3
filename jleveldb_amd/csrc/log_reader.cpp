// log_reader.cpp — host mirror of LogReader.readRecord (J/db/LogReader.java:146-252)
// driven by the device verification events of jl_log_verify.  The CRC work of
// readPhysicalRecord (:356-369) happened on the GPU; this replays the reader's
// buffer bookkeeping, fragment reassembly, initial-offset handling and
// Reporter calls exactly as the reference orders them.
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/jlcrc.h"

namespace {

constexpr uint64_t kBlockSize = 32768;  // LogFormat.kBlockSize, J/db/LogFormat.java:52
constexpr uint64_t kHeaderSize = 7;     // LogFormat.kHeaderSize, :54
enum { kZero = 0, kFull = 1, kFirst = 2, kMiddle = 3, kLast = 4, kEof = 5, kBadRecord = 6 };

struct Reader {
    const uint8_t *file = nullptr;
    uint64_t file_size = 0, file_pos = 0;
    const jl_log_event *ev = nullptr;
    uint64_t n_ev = 0, cursor = 0;
    uint64_t initial_offset = 0;
    uint64_t buf_size = 0;  // bytes left in `buffer` (the current block)
    bool eof = false;
    uint64_t last_record_offset = 0, end_of_buffer_offset = 0;
    bool resyncing = false;
    std::vector<jl_log_report> reports;
    bool sync_error = false;

    void report_drop(uint64_t bytes, uint32_t reason, uint32_t aux) {  // :396-401
        if ((int64_t)end_of_buffer_offset - (int64_t)buf_size - (int64_t)bytes >= (int64_t)initial_offset)
            reports.push_back(jl_log_report{bytes, reason, aux});
    }

    // readPhysicalRecord (:297-383) with the header decisions taken from the events
    int read_physical(const uint8_t **frag, uint64_t *frag_size) {
        for (;;) {
            if (buf_size < kHeaderSize) {
                if (!eof) {
                    uint64_t n = file_size - file_pos;
                    if (n > kBlockSize) n = kBlockSize;
                    buf_size = n;
                    file_pos += n;
                    end_of_buffer_offset += n;
                    if (n < kBlockSize) eof = true;
                    continue;
                }
                buf_size = 0;
                return kEof;
            }
            const uint64_t p = end_of_buffer_offset - buf_size;
            while (cursor < n_ev && (ev[cursor].offset < p || ev[cursor].kind == 0)) cursor++;
            if (cursor >= n_ev || ev[cursor].offset != p) {
                sync_error = true;
                return kEof;
            }
            const jl_log_event &e = ev[cursor++];
            switch (e.kind) {
            case JL_LOG_OK:
                break;
            case JL_LOG_BAD_CRC: {
                uint64_t drop = buf_size;
                buf_size = 0;
                report_drop(drop, JL_REASON_CHECKSUM, 0);
                return kBadRecord;
            }
            case JL_LOG_BAD_LENGTH: {
                uint64_t drop = buf_size;
                buf_size = 0;
                report_drop(drop, JL_REASON_BAD_LENGTH, 0);
                return kBadRecord;
            }
            case JL_LOG_ZERO_SKIP:
                buf_size = 0;
                return kBadRecord;
            case JL_LOG_EOF_BAD_LENGTH:
                buf_size = 0;
                return kEof;
            default:
                sync_error = true;
                return kEof;
            }
            const uint64_t length = e.length;
            buf_size -= kHeaderSize + length;
            if ((int64_t)end_of_buffer_offset - (int64_t)buf_size - (int64_t)kHeaderSize - (int64_t)length <
                (int64_t)initial_offset) {
                *frag_size = 0;
                return kBadRecord;
            }
            *frag = file + p + kHeaderSize;
            *frag_size = length;
            return e.type;
        }
    }
};

}  // namespace

extern "C" int jl_log_read_records(const uint8_t *log, uint64_t log_bytes, int checksum, uint64_t initial_offset,
                                   uint8_t *arena, uint64_t arena_cap, jl_log_record *records, uint64_t rec_cap,
                                   uint64_t *n_records, jl_log_report *reports, uint64_t rep_cap, uint64_t *n_reports) {
    if (!n_records || !n_reports || (log_bytes && !log)) return JL_ERR_INVALID;
    *n_records = 0;
    *n_reports = 0;
    std::vector<jl_log_event> ev;
    if (log_bytes) {
        // events for records of ~256 B and up (16 B of events per 256 B of log);
        // a denser log reports its event count and is verified once more into
        // an array of that size (r2 sized for 7-B records: 2.3x the log)
        ev.resize(std::min<uint64_t>(log_bytes / 7 + 2, log_bytes / 256 + 1024));
        uint64_t n_ev = 0;
        int r = jl_log_verify(log, log_bytes, checksum, ev.data(), ev.size(), &n_ev);
        if (r == JL_ERR_CAPACITY && n_ev > ev.size()) {
            ev.resize(n_ev);
            r = jl_log_verify(log, log_bytes, checksum, ev.data(), ev.size(), &n_ev);
        }
        if (r) return r;
        ev.resize(n_ev);
    }
    Reader R;
    R.file = log;
    R.file_size = log_bytes;
    R.ev = ev.data();
    R.n_ev = ev.size();
    R.initial_offset = initial_offset;
    R.resyncing = initial_offset > 0;

    if (R.last_record_offset < R.initial_offset) {  // skipToInitialBlock, :263-289
        uint64_t in_block = initial_offset % kBlockSize;
        uint64_t start = initial_offset - in_block;
        if (in_block > kBlockSize - 6) start += kBlockSize;
        R.end_of_buffer_offset = start;
        R.file_pos = start < log_bytes ? start : log_bytes;
    }

    uint64_t nrec = 0, arena_used = 0;
    bool overflow = false;
    for (;;) {  // one readRecord() call per iteration
        const uint64_t scratch_start = arena_used;
        uint64_t scratch_size = 0, prospective = 0, frag_size = 0;
        const uint8_t *frag = nullptr;
        bool in_frag = false, got = false, done = false;
        while (!got && !done) {
            int type = R.read_physical(&frag, &frag_size);
            uint64_t phys = R.end_of_buffer_offset - R.buf_size - kHeaderSize - frag_size;
            if (R.resyncing) {
                if (type == kMiddle) continue;
                if (type == kLast) { R.resyncing = false; continue; }
                R.resyncing = false;
            }
            switch (type) {
            case kFull:
                if (in_frag) {
                    if (scratch_size == 0) in_frag = false;
                    else R.report_drop(scratch_size, JL_REASON_PARTIAL_1, 0);
                }
                prospective = phys;
                if (scratch_start + frag_size > arena_cap || nrec >= rec_cap) { overflow = true; done = true; break; }
                memcpy(arena + scratch_start, frag, frag_size);
                records[nrec++] = jl_log_record{prospective, scratch_start, frag_size};
                arena_used = scratch_start + frag_size;
                R.last_record_offset = prospective;
                got = true;
                break;
            case kFirst:
                if (in_frag) {
                    if (scratch_size == 0) in_frag = false;
                    else R.report_drop(scratch_size, JL_REASON_PARTIAL_2, 0);
                }
                prospective = phys;
                if (scratch_start + frag_size > arena_cap) { overflow = true; done = true; break; }
                memcpy(arena + scratch_start, frag, frag_size);
                scratch_size = frag_size;
                in_frag = true;
                break;
            case kMiddle:
                if (!in_frag) R.report_drop(frag_size, JL_REASON_MISSING_START_1, 0);
                else {
                    if (scratch_start + scratch_size + frag_size > arena_cap) { overflow = true; done = true; break; }
                    memcpy(arena + scratch_start + scratch_size, frag, frag_size);
                    scratch_size += frag_size;
                }
                break;
            case kLast:
                if (!in_frag) R.report_drop(frag_size, JL_REASON_MISSING_START_2, 0);
                else {
                    if (scratch_start + scratch_size + frag_size > arena_cap || nrec >= rec_cap) {
                        overflow = true;
                        done = true;
                        break;
                    }
                    memcpy(arena + scratch_start + scratch_size, frag, frag_size);
                    scratch_size += frag_size;
                    records[nrec++] = jl_log_record{prospective, scratch_start, scratch_size};
                    arena_used = scratch_start + scratch_size;
                    R.last_record_offset = prospective;
                    got = true;
                }
                break;
            case kEof:
                done = true;  // a pending fragmented record is silently dropped (:227-233)
                break;
            case kBadRecord:
                if (in_frag) {
                    R.report_drop(scratch_size, JL_REASON_MIDDLE_ERROR, 0);
                    in_frag = false;
                    scratch_size = 0;
                }
                break;
            default:
                R.report_drop(frag_size + (in_frag ? scratch_size : 0), JL_REASON_UNKNOWN_TYPE, (uint32_t)type);
                in_frag = false;
                scratch_size = 0;
                break;
            }
        }
        if (done) break;
    }
    *n_records = nrec;
    *n_reports = R.reports.size();
    if (R.sync_error) return JL_ERR_HIP;
    if (overflow || R.reports.size() > rep_cap) return JL_ERR_CAPACITY;
    if (!R.reports.empty()) memcpy(reports, R.reports.data(), R.reports.size() * sizeof(jl_log_report));
    return JL_OK;
}
