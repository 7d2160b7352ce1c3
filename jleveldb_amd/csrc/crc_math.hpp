// crc_math.hpp — GF(2) algebra of the reflected CRC-32C state, used on the
// host to build the device table images (jlcrc_api.hip) and by the host scalar
// path (host_crc.cpp).
//
// State convention: `s` is the bit-flipped crc, exactly the Java field
// `Crc32C.crc` (J/util/Crc32C.java:96): value() = ~update(~0, data).
//   one data byte   : s' = (s >> 8) ^ T0[(s ^ b) & 0xff]        (Crc32C.java:165-167)
//   one zero byte   : z(s) = (s >> 8) ^ T0[s & 0xff]            (linear over GF(2))
//   T_k[i]          = z^k(T0[i])  — the reference's T8_k tables (Crc32C.java:173-334)
//   slicing-by-4    : x = s ^ LE32(b0..b3);
//                     s' = T3[x&ff] ^ T2[x>>8&ff] ^ T1[x>>16&ff] ^ T0[x>>24]
// z is invertible (the top byte of T0[i] is a permutation of i), which gives the
// exact "un-shift" z^-1 used by the device engine to re-align lane chains.
#pragma once
#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <algorithm>
#include <utility>
#include <vector>

namespace jlmath {

constexpr uint32_t kPoly = 0x82F63B78u;  // reflected Castagnoli (Crc32C.java:169-171)
constexpr uint32_t kMaskDelta = 0xa282ead8u;  // Crc32C.java:31

struct Tables {
    uint32_t t[8][256];     // T_0..T_7 (slicing-by-8, host path)
    uint8_t inv_top[256];   // inv_top[T0[i] >> 24] = i
    Tables() {
        for (uint32_t i = 0; i < 256; i++) {
            uint32_t c = i;
            for (int k = 0; k < 8; k++) c = (c >> 1) ^ ((c & 1u) ? kPoly : 0u);
            t[0][i] = c;
        }
        for (int k = 1; k < 8; k++)
            for (uint32_t i = 0; i < 256; i++) t[k][i] = (t[k - 1][i] >> 8) ^ t[0][t[k - 1][i] & 0xffu];
        bool seen[256] = {false};
        for (uint32_t i = 0; i < 256; i++) {
            uint32_t top = t[0][i] >> 24;
            if (seen[top]) throw std::logic_error("CRC-32C table top byte is not a permutation");
            seen[top] = true;
            inv_top[top] = (uint8_t)i;
        }
    }
    uint32_t z(uint32_t s) const { return (s >> 8) ^ t[0][s & 0xffu]; }
    uint32_t zinv(uint32_t s) const {
        uint32_t i = inv_top[s >> 24];
        return ((s ^ t[0][i]) << 8) | i;
    }
    uint32_t zn(uint32_t s, uint64_t n) const {
        for (uint64_t i = 0; i < n; i++) s = z(s);
        return s;
    }
    uint32_t zinvn(uint32_t s, uint64_t n) const {
        for (uint64_t i = 0; i < n; i++) s = zinv(s);
        return s;
    }
};

inline const Tables &tables() {
    static const Tables T;
    return T;
}

inline uint32_t mask(uint32_t crc) { return ((crc >> 15) | (crc << 17)) + kMaskDelta; }
inline uint32_t unmask(uint32_t m) {
    uint32_t rot = m - kMaskDelta;
    return (rot >> 17) | (rot << 15);
}

// ----------------------------------------------------------------------------
// Device LDS image (160 KiB = the whole LDS of one CU), see DESIGN.md §3.
//
// The engine interleaves each 256-byte "step" of a block over the 64 lanes of a
// wave (lane l owns the dword at 4*l), so lane l's chain visits words
// 256*k + 4*l.  Each chain step therefore processes 4 data bytes followed by
// 252 bytes that belong to other lanes; their contribution is added by the
// other lanes, so the step table is the slicing-by-4 table shifted by 252 zero
// bytes:  G_j[i] = z^(252+j)(T0[i]), byte 0 of x uses G_3 ... byte 3 uses G_0.
//
// Region A (128 KiB): G_0..G_3 replicated 32x so that lane l always reads LDS
//   bank (l & 31) (ds_read_b32 serves lanes 0-31 and 32-63 in separate cycles,
//   so 32 copies make every lookup conflict-free).  Table t, index i, copy b
//   sits at byte address ((t>>1) << 16) | (i << 8) | ((t&1) << 7) | (b << 2):
//   the index occupies exactly address byte 1, so the device builds each
//   lookup address with one v_perm_b32 (byte k of x into byte 1, the lane's
//   constant bytes 0 and 2 around it) — see gstep() in jlcrc_kernels.hip.
// Region B (32 KiB, base 131072): per-lane re-alignment tables.  After its last
//   step lane l sits 4*l bytes past the end of the block, so its state is
//   corrected with z^-(4l), applied as 8 nibble lookups:
//   N_{l,j}[v] = z^-(4l)(v << 4j), dword index 32768 + (((l>>5)*8 + j)*16 + v)*32 + (l & 31).
// ----------------------------------------------------------------------------
inline size_t g_dword_index(int t, int i, int b) {
    return ((size_t)(t >> 1) << 14) | ((size_t)i << 6) | ((size_t)(t & 1) << 5) | (size_t)b;
}
constexpr int kGapBytes = 252;
constexpr size_t kImageDwords = 32768 + 8192;
constexpr size_t kImageBytes = kImageDwords * 4;  // 163840

inline std::vector<uint32_t> build_lds_image() {
    const Tables &T = tables();
    std::vector<uint32_t> img(kImageDwords);
    for (int t = 0; t < 4; t++)
        for (int i = 0; i < 256; i++) {
            uint32_t g = T.zn(T.t[0][i], (uint64_t)kGapBytes + t);
            for (int b = 0; b < 32; b++) img[g_dword_index(t, i, b)] = g;
        }
    for (int l = 0; l < 64; l++)
        for (int j = 0; j < 8; j++)
            for (int v = 0; v < 16; v++) {
                uint32_t c = T.zinvn((uint32_t)v << (4 * j), 4u * (uint32_t)l);
                img[32768 + ((size_t)((l >> 5) * 8 + j) * 16 + v) * 32 + (l & 31)] = c;
            }
    return img;
}

// slice4(x) = state after feeding the 4 LE bytes of x to a zero state
// (T3[x0] ^ T2[x1] ^ T1[x2] ^ T0[x3]); linear and invertible over GF(2).
inline uint32_t slice4(uint32_t x) {
    const Tables &T = tables();
    return T.t[3][x & 0xffu] ^ T.t[2][(x >> 8) & 0xffu] ^ T.t[1][(x >> 16) & 0xffu] ^ T.t[0][x >> 24];
}
// Seed word of the stream kernel: feeding W = slice4^-1(~init) as the 4 data
// bytes just before a block turns a zero state into ~init at the block start,
// so `extend(init, ...)` needs no state shift.
inline uint32_t slice4_inv(uint32_t y) {
    static const std::vector<uint32_t> cols = [] {  // columns of slice4^-1 by Gauss-Jordan
        uint32_t a[32], inv[32];
        for (int i = 0; i < 32; i++) {
            a[i] = slice4(1u << i);  // column i of the forward map
            inv[i] = 1u << i;
        }
        // row-reduce the set of (image, preimage) pairs so image i == bit i
        for (int bit = 0; bit < 32; bit++) {
            int piv = -1;
            for (int i = bit; i < 32; i++)
                if ((a[i] >> bit) & 1u) { piv = i; break; }
            if (piv < 0) throw std::logic_error("slice4 is not invertible");
            std::swap(a[piv], a[bit]);
            std::swap(inv[piv], inv[bit]);
            for (int i = 0; i < 32; i++)
                if (i != bit && ((a[i] >> bit) & 1u)) { a[i] ^= a[bit]; inv[i] ^= inv[bit]; }
        }
        return std::vector<uint32_t>(inv, inv + 32);  // slice4(inv[i]) == 1 << i
    }();
    uint32_t x = 0;
    for (int i = 0; i < 32; i++)
        if ((y >> i) & 1u) x ^= cols[i];
    return x;
}

// v4 image (fixed_v4.hip): lanes-per-block LPB, block-step STEP = 16*LPB bytes.
// Region A: the gap tables of chain dwords STEP bytes apart,
//   G_t[i] = z^(STEP-4+t)(T0[i]), same addressing as build_lds_image().
// Region B (dwords):
//   [32768, 36864)  per-lane shift z^-(16*(b % LPB)) as 8 nibble tables, copy b
//                   in bank b: dword 32768 + (p*16 + v)*32 + b   (realign() layout)
//   [36864, 37248)  uniform z^-4, z^-8, z^-12: dword 36864 + u*128 + p*16 + v
//   [37248, 38272)  per-wave result slots (64 dwords x 16 waves)
//   [38272, 39296)  U_j[v] = slice4^-1(v << 8j), j = 0..3 (general_v4.hip: seed of an init)
//   [39296, 39552)  T0 (general_v4.hip: suffix byte)
constexpr size_t kV4UDword = 36864;
constexpr size_t kV4SlotDword = 37248;
constexpr size_t kG4UDword = 38272;
constexpr size_t kG4T0Dword = 39296;
constexpr size_t kG4ShiftDword = 36864;  // gv4 image: 7 x 128 dwords (replaces the v4 U4 tables)
constexpr size_t kG4EDword = 37760;      // gv4 image: 4 x 128 dwords, ends at 38272 = kG4UDword
// gv4 image: v_perm_b32 byte selectors of a round's first / last step (after T0):
//   [0, 13)   front, dword starting t = -8..4 bytes from the block start p: byte i
//             at p + t + i is data (selector i) when >= 0, the seed W's byte
//             t + i + 4 (selector t + i + 8) when in [-4, 0), else zero (0x0c)
//   [13, 18)  tail, t' = 0..4 bytes of the dword before the tail pad: byte i kept
//             (selector i) when i < t', else zero
constexpr size_t kG4SelDword = 39552;
inline std::vector<uint32_t> build_lds_image_v4(int lpb) {
    const Tables &T = tables();
    const int gap = 16 * lpb - 4;
    std::vector<uint32_t> img(kImageDwords, 0);
    for (int t = 0; t < 4; t++)
        for (int i = 0; i < 256; i++) {
            uint32_t g = T.zn(T.t[0][i], (uint64_t)gap + t);
            for (int b = 0; b < 32; b++) img[g_dword_index(t, i, b)] = g;
        }
    for (int b = 0; b < 32; b++)
        for (int p = 0; p < 8; p++)
            for (int v = 0; v < 16; v++)
                img[32768 + (size_t)(p * 16 + v) * 32 + b] = T.zinvn((uint32_t)v << (4 * p), 16u * (uint32_t)(b % lpb));
    for (int u = 0; u < 3; u++)
        for (int p = 0; p < 8; p++)
            for (int v = 0; v < 16; v++)
                img[kV4UDword + (size_t)u * 128 + p * 16 + v] = T.zinvn((uint32_t)v << (4 * p), 4u * (uint32_t)(u + 1));
    for (int j = 0; j < 4; j++)
        for (uint32_t v = 0; v < 256; v++) img[kG4UDword + 256 * j + v] = slice4_inv(v << (8 * j));
    for (int i = 0; i < 256; i++) img[kG4T0Dword + i] = T.t[0][i];
    return img;
}

// The 8-lane gap step L(x) = G3[x.b0] ^ G2[x.b1] ^ G1[x.b2] ^ G0[x.b3], G_t =
// z^(124+t)∘T0 (linear): what a chain register still owes after a block's last
// window.  The gv4 epilogue tables absorb it.
inline uint32_t gap_step8(uint32_t x) {
    const Tables &T = tables();
    uint32_t r = 0;
    for (int t = 0; t < 4; t++) r ^= T.zn(T.t[0][(x >> (8 * t)) & 0xffu], 124u + 3u - (uint32_t)t);
    return r;
}

// General v4 image (general_v4.hip): the v4 image for 8 lanes per block with
// the epilogue tables re-cut so a block's tail pad d = 16a + 4c + e folds into
// shifts the epilogue does anyway:
//   lane tables   column b: z^-(16 (b % 16))   (realign by 16 (l + a))
//   kG4ShiftDword U_k = z^-(4k) ∘ L, k = 0..6   (chain j: its pending gap step
//                 L, gap_step8 below, then z^-(4 (j + c)))
//   kG4EDword     E_e = z^-e, e = 0..3          (after the group xor)
inline std::vector<uint32_t> build_lds_image_gv4() {
    const Tables &T = tables();
    std::vector<uint32_t> img = build_lds_image_v4(8);
    for (int b = 0; b < 32; b++)
        for (int p = 0; p < 8; p++)
            for (int v = 0; v < 16; v++)
                img[32768 + (size_t)(p * 16 + v) * 32 + b] = T.zinvn((uint32_t)v << (4 * p), 16u * (uint32_t)(b % 16));
    for (int k = 0; k < 7; k++)
        for (int p = 0; p < 8; p++)
            for (int v = 0; v < 16; v++)
                img[kG4ShiftDword + (size_t)k * 128 + p * 16 + v] = T.zinvn(gap_step8((uint32_t)v << (4 * p)), 4u * (uint32_t)k);
    for (int e = 0; e < 4; e++)
        for (int p = 0; p < 8; p++)
            for (int v = 0; v < 16; v++)
                img[kG4EDword + (size_t)e * 128 + p * 16 + v] = T.zinvn((uint32_t)v << (4 * p), (uint32_t)e);
    for (int t = -8; t <= 4; t++) {
        uint32_t sel = 0;
        for (int i = 0; i < 4; i++) {
            const int pos = t + i;
            const uint32_t b = pos >= 0 ? (uint32_t)i : (pos >= -4 ? (uint32_t)(pos + 8) : 0x0cu);
            sel |= b << (8 * i);
        }
        img[kG4SelDword + (size_t)(t + 8)] = sel;
    }
    for (int t = 0; t <= 4; t++) {
        uint32_t sel = 0;
        for (int i = 0; i < 4; i++) sel |= (i < t ? (uint32_t)i : 0x0cu) << (8 * i);
        img[kG4SelDword + 13 + (size_t)t] = sel;
    }
    return img;
}
// The gv4 kernel's image: build_lds_image_gv4() rotated so region B comes first
// (byte 0) and the G tables follow at byte 32768 (general_v4.hip kGOff): region-B
// table bases then fit the ds_read immediate offset.
inline std::vector<uint32_t> build_lds_image_gv4_rotated() {
    std::vector<uint32_t> img = build_lds_image_gv4();
    std::rotate(img.begin(), img.begin() + 32768, img.end());
    return img;
}
// The log-chunk kernel's image (crc_gv4_kernel<MODE_LOG_CHUNK>): the rotated gv4
// image with its region B re-cut after the lane tables.  A round's chunks share
// d mod 16 (bins by (K, d mod 16), log_chunks.hip), so the tail pad's z^-e joins
// the chain shifts: chain j uses M_m, m = 4 (j + c) + e (28 nibble tables) and
// the epilogue has no separate z^-e stage.  The tables also absorb the chains'
// last pending step (gap_step8), so M_m = z^-m ∘ L is applied to the chain
// registers directly (16 G lookups per round less).  No init / suffix
// tables (log records are crc'd from value()'s init with no suffix).
//   byte [16384, 30720)  M_m, m = 0..27, 128 dwords each
//   byte [30720, 30792)  the front / tail byte selectors (kG4SelDword layout)
constexpr size_t kLCMDword = 4096, kLCSelDword = 7680;
inline std::vector<uint32_t> build_lds_image_logchunk() {
    const Tables &T = tables();
    std::vector<uint32_t> img = build_lds_image_gv4_rotated();
    const std::vector<uint32_t> base = build_lds_image_gv4();
    for (size_t i = kLCMDword; i < 8192; i++) img[i] = 0;
    for (int m = 0; m < 28; m++)
        for (int p = 0; p < 8; p++)
            for (int v = 0; v < 16; v++)
                img[kLCMDword + (size_t)m * 128 + p * 16 + v] = T.zinvn(gap_step8((uint32_t)v << (4 * p)), (uint32_t)m);
    for (int i = 0; i < 18; i++) img[kLCSelDword + i] = base[kG4SelDword + i];
    return img;
}

// Log-stream image (log_stream.hip): region A = the general v4 gap tables
// (z^(124+t)∘T0, chains 128 B apart); region B re-cut for the fused log kernel
// (its fold is general_v4.hip's epilogue, with 16 lane-table columns):
//   [32768, 34816)  lane tables, column b: z^-(16 b) as 8 nibble tables,
//                   dword 32768 + (p*16 + v)*16 + b       (ls_realign())
//   [34816, 35712)  U_k = z^-(4k), k = 0..6, nibble tables (chain j: z^-(4 (j + c)))
//   [35712, 36224)  E_e = z^-e, e = 0..3, nibble tables
//   kLSMaskDword    39 entries x 4 dwords, entry t + 22 for t in [-22, 16]:
//                   the byte masks of one data dword when a record header
//                   starts at byte t of that dword (t may lie before or past it):
//                     [0] om = bytes < t          (the record that ends at t)
//                     [1] nm = bytes >= t + 6     (the next record's type byte, payload)
//                     [2] sd = W0 = slice4^-1(0xffffffff) at bytes [t + 2, t + 6)
//                          (the next record's crc init, fed as the 4 bytes before it)
//   kLSStageDword   per-wave header staging, 12 waves x 8 groups x 144 B: the
//                   group's window and the first 16 B of the next one
constexpr size_t kLSLaneDword = 32768;
constexpr size_t kLSShiftDword = 34816;
constexpr size_t kLSEDword = 35712;
constexpr size_t kLSMaskDword = 36224;
constexpr int kLSMaskLo = -22, kLSMaskHi = 16;
constexpr size_t kLSStageDword = 36384;  // 16-B aligned; 12 x 1152 B: ends at 39840 <= kImageDwords
inline std::vector<uint32_t> build_lds_image_logstream() {
    const Tables &T = tables();
    std::vector<uint32_t> img = build_lds_image_v4(8);  // region A: gap tables for 128-B steps
    for (size_t i = 32768; i < kImageDwords; i++) img[i] = 0;
    for (int b = 0; b < 16; b++)
        for (int p = 0; p < 8; p++)
            for (int v = 0; v < 16; v++)
                img[kLSLaneDword + (size_t)(p * 16 + v) * 16 + b] = T.zinvn((uint32_t)v << (4 * p), 16u * (uint32_t)b);
    for (int k = 0; k < 7; k++)
        for (int p = 0; p < 8; p++)
            for (int v = 0; v < 16; v++)
                img[kLSShiftDword + (size_t)k * 128 + p * 16 + v] = T.zinvn((uint32_t)v << (4 * p), 4u * (uint32_t)k);
    for (int e = 0; e < 4; e++)
        for (int p = 0; p < 8; p++)
            for (int v = 0; v < 16; v++)
                img[kLSEDword + (size_t)e * 128 + p * 16 + v] = T.zinvn((uint32_t)v << (4 * p), (uint32_t)e);
    const uint32_t w0 = slice4_inv(0xffffffffu);
    for (int t = kLSMaskLo; t <= kLSMaskHi; t++) {
        uint32_t om = 0, nm = 0, sd = 0;
        for (int i = 0; i < 4; i++) {
            if (i < t) om |= 0xffu << (8 * i);
            if (i >= t + 6) nm |= 0xffu << (8 * i);
            if (i >= t + 2 && i < t + 6) sd |= ((w0 >> (8 * (i - t - 2))) & 0xffu) << (8 * i);
        }
        const size_t e = kLSMaskDword + 4 * (size_t)(t - kLSMaskLo);
        img[e] = om;
        img[e + 1] = nm;
        img[e + 2] = sd;
    }
    return img;
}

// Small global-memory table used by the kernels' scalar epilogues:
//   [0,256)     T0
//   [256,512)   inv_top (as u32)
//   [512,517)   typeCrc[0..4] = value([t])  (LogWriter.initTypeCrc, J/db/LogWriter.java:51-57)
//   [520,525)   W(typeCrc[t]) = slice4^-1(~typeCrc[t])   (stream-kernel seeds)
//   [525]       W(0) = slice4^-1(0xffffffff)               (value(): init 0)
//   [528,1552)  U_j[v] = slice4^-1(v << 8j), j = 0..3     (seed of an arbitrary init)
//   [1552,5648) Z_k = z^(2^k), k = 0..31, nibble tables (8 x 16 each): the state
//               shift by 2^k zero bytes (folding the chunks of a split block)
//   [5648, +256*128)  ZW_a = z^(128 a), a = 0..255, nibble tables (log chunk fold)
//   [.., +128*128)    ZB_b = z^b, b = 0..127, nibble tables
constexpr size_t kAuxZpow = 1552;
constexpr size_t kAuxZW = kAuxZpow + 32 * 128;
constexpr size_t kAuxZB = kAuxZW + 256 * 128;
constexpr size_t kAuxDwords = kAuxZB + 128 * 128;
inline std::vector<uint32_t> build_aux() {
    const Tables &T = tables();
    std::vector<uint32_t> aux(kAuxDwords, 0);
    for (int i = 0; i < 256; i++) {
        aux[i] = T.t[0][i];
        aux[256 + i] = T.inv_top[i];
    }
    for (uint32_t t = 0; t < 5; t++) aux[512 + t] = ~((0xffffffffu >> 8) ^ T.t[0][(0xffffffffu ^ t) & 0xffu]);
    for (uint32_t t = 0; t < 5; t++) aux[520 + t] = slice4_inv(~aux[512 + t]);
    aux[525] = slice4_inv(0xffffffffu);
    for (int j = 0; j < 4; j++)
        for (uint32_t v = 0; v < 256; v++) aux[528 + 256 * j + v] = slice4_inv(v << (8 * j));
    // z^(2^k) by repeated squaring of the 32x32 GF(2) matrix of z (column b = z(e_b))
    uint32_t col[32], sq[32];
    for (int b = 0; b < 32; b++) col[b] = T.z(1u << b);
    auto apply = [](const uint32_t *m, uint32_t v) {  // column b of m = image of bit b
        uint32_t r = 0;
        for (int b = 0; b < 32; b++)
            if ((v >> b) & 1u) r ^= m[b];
        return r;
    };
    for (int k = 0; k < 32; k++) {
        for (int p = 0; p < 8; p++)
            for (uint32_t v = 0; v < 16; v++) aux[kAuxZpow + 128 * k + 16 * p + v] = apply(col, v << (4 * p));
        for (int b = 0; b < 32; b++) sq[b] = apply(col, col[b]);
        for (int b = 0; b < 32; b++) col[b] = sq[b];
    }
    // z^b (b < 128) and z^(128 a) (a < 256) by repeated multiplication
    uint32_t z1[32], zb[32], z128[32], zw[32];
    for (int b = 0; b < 32; b++) z1[b] = zb[b] = zw[b] = 1u << b;
    auto put = [&](size_t at, const uint32_t *m) {
        for (int p = 0; p < 8; p++)
            for (uint32_t v = 0; v < 16; v++) aux[at + 16 * p + v] = apply(m, v << (4 * p));
    };
    for (int b = 0; b < 32; b++) z1[b] = T.z(1u << b);
    for (int i = 0; i < 128; i++) {
        put(kAuxZB + 128 * (size_t)i, zb);
        for (int b = 0; b < 32; b++) sq[b] = apply(z1, zb[b]);
        for (int b = 0; b < 32; b++) zb[b] = sq[b];
    }
    for (int b = 0; b < 32; b++) z128[b] = zb[b];  // z^128
    for (int a = 0; a < 256; a++) {
        put(kAuxZW + 128 * (size_t)a, zw);
        for (int b = 0; b < 32; b++) sq[b] = apply(z128, zw[b]);
        for (int b = 0; b < 32; b++) zw[b] = sq[b];
    }
    return aux;
}

}  // namespace jlmath
