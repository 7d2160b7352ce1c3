// table_walker.cpp — the block handles of an SSTable file image, so a whole
// table (data blocks, filter block, metaindex, index) can be checksum-verified
// from its bytes with no Java in the loop.  Host code:
// it touches the 48-byte footer and the index / metaindex blocks only.
//
//   footer            TableFormat.Footer.decodeFrom  J/table/TableFormat.java:126-146 (magic :161)
//   block handle      BlockHandle.decodeFrom         J/table/TableFormat.java:74-78
//   block entries     Block / Block.decodeEntry      J/table/Block.java:44-84, 312-342
//   metaindex walk    Table.readMeta                 J/table/Table.java:287-310
//   "too short"       Table.open                     J/table/Table.java:338-339
//   block read        TableFormat.readBlock          J/table/TableFormat.java:195-258
//
// Before trusting the index / metaindex contents the walker reads them the way
// Table.open / Table.readMeta do with paranoidChecks: trailer checksum, then the
// type byte (util/Snappy.java is a stub in the reference, so a kSnappyCompression
// block can never be read: "corrupted compressed block contents").  A bad index
// block fails the walk (the table cannot be opened); a bad metaindex block only
// drops the meta handles (readMeta returns without a filter) — its own handle is
// still emitted so the batched verification flags it.
#include <stdint.h>
#include <string.h>

#include <string>

#include "../../include/jlcrc.h"

namespace {

constexpr uint64_t kMagic = 0xdb4775248b80fb57ull;
constexpr uint64_t kFooterLen = 48;  // 2 * BlockHandle.MaxEncodedLength + 8
constexpr uint64_t kTrailer = 5;     // TableFormat.kBlockTrailerSize

bool varint64(const uint8_t *p, uint64_t limit, uint64_t &pos, uint64_t &v) {
    v = 0;
    for (int shift = 0; shift <= 63 && pos < limit; shift += 7) {
        const uint8_t b = p[pos++];
        v |= (uint64_t)(b & 0x7f) << shift;
        if (!(b & 0x80)) return true;
    }
    return false;
}

uint32_t le32(const uint8_t *p) {
    uint32_t v;
    memcpy(&v, p, 4);
    return v;
}

struct Out {
    uint64_t *off;
    uint32_t *len;
    uint8_t *kind;
    uint64_t cap, n;
    void add(uint64_t o, uint64_t s, uint8_t k) {
        if (n < cap) {
            off[n] = o;
            len[n] = (uint32_t)s;
            if (kind) kind[n] = k;
        }
        n++;
    }
};

// handle (offset, size) of a block that must lie, with its trailer, inside the file
bool handle_ok(uint64_t file, uint64_t off, uint64_t size, std::string &err) {
    if (size > 0xffffffffull || off > file || size + kTrailer > file - off) {
        err = "truncated block read";
        return false;
    }
    return true;
}

// TableFormat.readBlock(verifyChecksums=true) of a block whose handle is in bounds
bool read_block(const uint8_t *f, uint64_t off, uint64_t size, std::string &err) {
    const uint8_t *b = f + off;
    if (jl_crc32c_unmask(le32(b + size + 1)) != jl_crc32c_value(b, size + 1)) {
        err = "block checksum mismatch";
        return false;
    }
    if (b[size] == 1) {
        err = "corrupted compressed block contents";
        return false;
    }
    if (b[size] != 0) {
        err = "bad compress type " + std::to_string((int)(int8_t)b[size]);
        return false;
    }
    return true;
}

// every entry value of the block at [off, off+size) decoded as a BlockHandle
bool block_handles(const uint8_t *f, uint64_t file, uint64_t off, uint64_t size, uint8_t kind, Out &out,
                   std::string &err) {
    if (size < 4) {
        err = "bad block contents";
        return false;
    }
    const uint8_t *b = f + off;
    const uint64_t nres = le32(b + size - 4);
    if (nres > (size - 4) / 4) {
        err = "bad block contents";
        return false;
    }
    const uint64_t limit = size - (1 + nres) * 4;
    uint64_t pos = 0;
    while (pos < limit) {
        uint64_t shared, non_shared, vlen;
        if (!varint64(b, limit, pos, shared) || !varint64(b, limit, pos, non_shared) ||
            !varint64(b, limit, pos, vlen) || non_shared > limit - pos || vlen > limit - pos - non_shared) {
            err = "bad entry in block";
            return false;
        }
        pos += non_shared;
        uint64_t vp = 0, o, s;
        if (!varint64(b + pos, vlen, vp, o) || !varint64(b + pos, vlen, vp, s)) {
            err = "bad block handle";
            return false;
        }
        if (!handle_ok(file, o, s, err)) return false;
        out.add(o, s, kind);
        pos += vlen;
    }
    return true;
}

}  // namespace

void jl_set_error(const std::string &msg);  // jlcrc_api.hip (jl_last_error)

extern "C" int jl_table_block_handles(const uint8_t *file, uint64_t file_bytes, uint64_t *off, uint32_t *size,
                                      uint8_t *kind, uint64_t cap, uint64_t *n) {
    if (!n || (file_bytes && !file) || (cap && (!off || !size))) {
        jl_set_error("jl_table_block_handles: null pointer");
        return JL_ERR_INVALID;
    }
    *n = 0;
    std::string err;
    if (file_bytes < kFooterLen) {
        jl_set_error("file is too short to be an sstable");
        return JL_ERR_CORRUPT;
    }
    const uint8_t *ft = file + file_bytes - kFooterLen;
    if (((uint64_t)le32(ft + 44) << 32 | le32(ft + 40)) != kMagic) {
        jl_set_error("not an sstable (bad magic number)");
        return JL_ERR_CORRUPT;
    }
    uint64_t pos = 0, moff, msize, ioff, isize;
    if (!varint64(ft, 40, pos, moff) || !varint64(ft, 40, pos, msize) || !varint64(ft, 40, pos, ioff) ||
        !varint64(ft, 40, pos, isize)) {
        jl_set_error("bad block handle");
        return JL_ERR_CORRUPT;
    }
    Out out{off, size, kind, cap, 0};
    if (!handle_ok(file_bytes, ioff, isize, err) || !read_block(file, ioff, isize, err) ||
        !block_handles(file, file_bytes, ioff, isize, JL_BLOCK_DATA, out, err)) {
        jl_set_error(err);
        return JL_ERR_CORRUPT;
    }
    // readMeta failures are not fatal: keep the data handles, drop the meta ones
    const uint64_t n_data = out.n;
    std::string merr;
    if (!handle_ok(file_bytes, moff, msize, merr)) {
        jl_set_error(merr);
        return JL_ERR_CORRUPT;  // the metaindex handle itself must be in the file to be verified
    }
    if (!read_block(file, moff, msize, merr) || !block_handles(file, file_bytes, moff, msize, JL_BLOCK_META, out, merr))
        out.n = n_data;
    out.add(moff, msize, JL_BLOCK_METAINDEX);
    out.add(ioff, isize, JL_BLOCK_INDEX);
    *n = out.n;
    if (out.n > cap) {
        jl_set_error("jl_table_block_handles: handle arrays too small");
        return JL_ERR_CAPACITY;
    }
    return JL_OK;
}
