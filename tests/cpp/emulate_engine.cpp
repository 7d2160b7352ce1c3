// Host emulation of the device engine's per-lane algorithm (test only): checks
// the LDS image math (gap tables, per-lane z^-(4l) re-alignment, front
// injection z^-r(~init)) against a plain byte-serial CRC-32C.
#include "../../jleveldb_amd/csrc/crc_math.hpp"
#include <cstdio>
#include <random>
using namespace jlmath;

static uint32_t ref_update(uint32_t s, const uint8_t* p, size_t n) {
    const Tables& T = tables();
    for (size_t i = 0; i < n; i++) s = (s >> 8) ^ T.t[0][(s ^ p[i]) & 0xff];
    return s;
}

static uint32_t emulate(const std::vector<uint32_t>& img, const uint8_t* base, uint32_t n, uint32_t init) {
    const Tables& T = tables();
    uint32_t s0 = ~init;
    if (n == 0) return ~s0;
    uint32_t K = (n + 255) / 256, f = 256 * K - n, l0 = f >> 2, r = f & 3;
    uint32_t inj = T.zinvn(s0, r);
    uint32_t total = 0;
    for (int lane = 0; lane < 64; lane++) {
        uint32_t s = 0;
        for (uint32_t k = 0; k < K; k++) {
            int64_t p = 256 * (int64_t)k + 4 * lane - f;
            uint32_t w = 0;
            if (p >= 0) memcpy(&w, base + p, 4);
            else if (p > -4) { for (int j = 0; j < 4 + p; j++) w |= (uint32_t)base[j] << (8 * (j - p)); }
            if (k == 0 && (uint32_t)lane == l0) s = inj;
            uint32_t x = s ^ w;
            uint32_t b = lane & 31;
            s = img[g_dword_index(3, x & 0xff, b)] ^ img[g_dword_index(2, (x >> 8) & 0xff, b)] ^
                img[g_dword_index(1, (x >> 16) & 0xff, b)] ^ img[g_dword_index(0, x >> 24, b)];
        }
        uint32_t c = 0;
        for (int j = 0; j < 8; j++) {
            uint32_t v = (s >> (4 * j)) & 15;
            c ^= img[32768 + (((lane >> 5) * 8 + j) * 16 + v) * 32 + (lane & 31)];
        }
        total ^= c;
    }
    return ~total;
}

// The stream kernel's seeding (crc_stream_kernel): no state shift; the seed
// word W = slice4^-1(~init) is fed as data at virtual bytes [f-4, f): lane l0-1
// gets W << 8r, the straddling lane l0 gets (LE32 of the first real bytes << 8r)
// | W >> (32 - 8r); for l0 == 0 lane 63 starts from one gap step of W << 8r.
static uint32_t gstep_img(const std::vector<uint32_t>& img, uint32_t x, int lane) {
    uint32_t b = lane & 31;
    return img[g_dword_index(3, x & 0xff, b)] ^ img[g_dword_index(2, (x >> 8) & 0xff, b)] ^
           img[g_dword_index(1, (x >> 16) & 0xff, b)] ^ img[g_dword_index(0, x >> 24, b)];
}

static uint32_t emulate_stream(const std::vector<uint32_t>& img, const uint8_t* base, uint32_t n, uint32_t init) {
    if (n == 0) return init;
    const uint32_t W = slice4_inv(~init);
    uint32_t K = (n + 255) / 256, f = 256 * K - n, l0 = f >> 2, r = f & 3;
    uint32_t total = 0;
    for (int lane = 0; lane < 64; lane++) {
        uint32_t s = (l0 == 0 && lane == 63) ? gstep_img(img, W << (8 * r), lane) : 0u;
        for (uint32_t k = 0; k < K; k++) {
            int64_t p = 256 * (int64_t)k + 4 * lane - f;
            uint32_t w = 0;
            if (p >= 0) memcpy(&w, base + p, 4);
            if (k == 0 && (uint32_t)lane == l0 && r) {
                uint32_t dw = 0;
                memcpy(&dw, base, n < 4 ? n : 4);
                w = (dw << (8 * r)) | (W >> (32 - 8 * r));
            }
            if (k == 0 && l0 > 0 && (uint32_t)lane == l0 - 1) w = W << (8 * r);
            s = gstep_img(img, s ^ w, lane);
        }
        uint32_t c = 0;
        for (int j = 0; j < 8; j++) {
            uint32_t v = (s >> (4 * j)) & 15;
            c ^= img[32768 + (((lane >> 5) * 8 + j) * 16 + v) * 32 + (lane & 31)];
        }
        total ^= c;
    }
    return ~total;
}

// The v4 fixed kernel (fixed_v4.hip): LPB lanes per 4 KiB block, lane l' reads
// 16 B at 16*LPB*k + 16*l'; dword j feeds chain j through gap tables
// z^(16*LPB-4+t); chains folded with the uniform z^-4j tables, the lane with
// z^-(16 l') (bank copy b = lane & 31), lanes XORed.
static uint32_t emulate_v4(const std::vector<uint32_t>& img, const uint8_t* blk, int lpb, int lane_base) {
    const int step = 16 * lpb, S = 4096 / step;
    uint32_t total = 0;
    for (int lp = 0; lp < lpb; lp++) {
        const int lane = lane_base + lp, b = lane & 31;
        uint32_t s[4];
        for (int j = 0; j < 4; j++) {
            s[j] = (lp == 0 && j == 0) ? 0xffffffffu : 0u;
            for (int k = 0; k < S; k++) {
                uint32_t w;
                memcpy(&w, blk + step * k + 16 * lp + 4 * j, 4);
                uint32_t x = s[j] ^ w;
                s[j] = img[g_dword_index(3, x & 0xff, b)] ^ img[g_dword_index(2, (x >> 8) & 0xff, b)] ^
                       img[g_dword_index(1, (x >> 16) & 0xff, b)] ^ img[g_dword_index(0, x >> 24, b)];
            }
        }
        uint32_t c = s[0];
        for (int u = 0; u < 3; u++)
            for (int p = 0; p < 8; p++) c ^= img[kV4UDword + u * 128 + p * 16 + ((s[u + 1] >> (4 * p)) & 15)];
        uint32_t r = 0;
        for (int p = 0; p < 8; p++) r ^= img[32768 + (p * 16 + ((c >> (4 * p)) & 15)) * 32 + b];
        total ^= r;
    }
    return ~total;
}

// The general v4 kernel (general_v4.hip) on its 128-B aligned grid: block at
// offset f of its first window, K = ceil((f+n)/128) windows, tail pad d; the
// seed word W at virtual bytes [f-4, f) (chain lane 7 / dword 3 starts from
// gstep(W << 8f) when f < 4); epilogue with the gv4 image's U_{j+c}, lane
// column (l + a) & 15 | (q & 1) << 4 and E_e, d = 16a + 4c + e.
static uint32_t nib(const std::vector<uint32_t>& img, size_t base_dw, uint32_t s) {
    uint32_t r = 0;
    for (int p = 0; p < 8; p++) r ^= img[base_dw + p * 16 + ((s >> (4 * p)) & 15)];
    return r;
}

static uint32_t emulate_gv4(const std::vector<uint32_t>& img, const uint8_t* blk, uint32_t n, uint32_t f, uint32_t init,
                            int q) {
    if (n == 0) return init;
    const uint32_t K = (f + n + 127) / 128, d = 128 * K - f - n, W = slice4_inv(~init);
    std::vector<uint8_t> V(128 * K + 4, 0);  // V[t + 4] = virtual byte t, t >= -4
    for (int t = -4; t < (int)(128 * K); t++) {
        uint8_t b = 0;
        if (t >= (int)f && t < (int)(f + n)) b = blk[t - f];
        else if (t >= (int)f - 4 && t < (int)f) b = (uint8_t)(W >> (8 * (t - (int)f + 4)));
        V[t + 4] = b;
    }
    uint32_t total = 0;
    for (int l = 0; l < 8; l++) {
        const int lane = q * 8 + l;
        uint32_t c = 0;
        for (int j = 0; j < 4; j++) {
            uint32_t s = 0;
            for (int k = -1; k < (int)K; k++) {
                const int pos = 128 * k + 16 * l + 4 * j;
                uint32_t w = 0;
                if (pos >= -4) memcpy(&w, &V[pos + 4], 4);
                s = k + 1 < (int)K ? gstep_img(img, s ^ w, lane) : s ^ w;  // the last step stays pending
            }
            c ^= nib(img, kG4ShiftDword + 128 * (j + ((d >> 2) & 3)), s);  // its gap step is in the table
        }
        const uint32_t col = ((l + (d >> 4)) & 15) | ((q & 1) << 4);
        uint32_t r = 0;
        for (int p = 0; p < 8; p++) r ^= img[32768 + (p * 16 + ((c >> (4 * p)) & 15)) * 32 + col];
        total ^= r;
    }
    return ~nib(img, kG4EDword + 128 * (d & 3), total);
}

// The split-block fold (gv4_combine_kernel): chunk raw states from state 0,
// folded lane-sequentially then by a 6-level tree with z^L from the aux
// z^(2^k) tables, plus z^n(~init).
static uint32_t zpow_aux(const std::vector<uint32_t>& aux, uint32_t s, uint32_t L) {
    for (int k = 0; k < 32; k++)
        if ((L >> k) & 1u) {
            uint32_t r = 0;
            for (int q = 0; q < 8; q++) r ^= aux[kAuxZpow + 128 * k + 16 * q + ((s >> (4 * q)) & 15)];
            s = r;
        }
    return s;
}

static uint32_t emulate_split(const std::vector<uint32_t>& aux, const uint8_t* blk, uint32_t n, uint32_t cs,
                              uint32_t init) {
    const uint32_t m = (n + cs - 1) / cs, L = n - (m - 1) * cs, per = (m + 63) / 64;
    uint32_t s[64] = {0}, bytes[64] = {0};
    for (uint32_t t = 0; t < 64; t++)
        for (uint32_t c = t * per; c < m && c < (t + 1) * per; c++) {
            const uint32_t len = c + 1 == m ? L : cs;
            s[t] = zpow_aux(aux, s[t], len) ^ ref_update(0, blk + (size_t)c * cs, len);
            bytes[t] += len;
        }
    for (uint32_t off = 1; off < 64; off <<= 1)
        for (uint32_t t = 0; t + off < 64; t += 2 * off) {
            s[t] = zpow_aux(aux, s[t], bytes[t + off]) ^ s[t + off];
            bytes[t] += bytes[t + off];
        }
    return ~(zpow_aux(aux, ~init, n) ^ s[0]);
}

int main() {
    auto img = build_lds_image();
    std::mt19937_64 rng(42);
    std::vector<uint8_t> buf(70000 + 16);
    for (auto& b : buf) b = (uint8_t)rng();
    int bad = 0, cases = 0;
    for (uint32_t n = 0; n <= 1300; n++) {
        for (int a = 0; a < 4; a++) {
            uint32_t init = (n % 3 == 0) ? 0 : (uint32_t)rng();
            uint32_t want = ~ref_update(~init, buf.data() + a, n);
            uint32_t got = emulate(img, buf.data() + a, n, init);
            uint32_t got2 = emulate_stream(img, buf.data() + a, n, init);
            cases++;
            if (want != got && bad++ < 5) printf("mismatch n=%u a=%d %08x %08x\n", n, a, want, got);
            if (want != got2 && bad++ < 5) printf("stream mismatch n=%u a=%d %08x %08x\n", n, a, want, got2);
        }
    }
    for (uint32_t n : {4096u, 4097u, 8191u, 65536u, 65535u, 32768u, 65000u}) {
        uint32_t want = ~ref_update(~0u, buf.data() + 1, n);
        uint32_t got = emulate(img, buf.data() + 1, n, 0);
        cases++;
        if (want != got && bad++ < 10) printf("mismatch n=%u %08x %08x\n", n, want, got);
    }
    for (int lpb : {8, 16}) {
        auto img4 = build_lds_image_v4(lpb);
        for (int q = 0; q < 64 / lpb; q++) {
            const uint8_t* blk = buf.data() + 4096 * (q % 16);
            uint32_t want = ~ref_update(~0u, blk, 4096);
            uint32_t got = emulate_v4(img4, blk, lpb, q * lpb);
            cases++;
            if (want != got && bad++ < 10) printf("v4 mismatch lpb=%d q=%d %08x %08x\n", lpb, q, want, got);
        }
    }
    {
        auto imgg = build_lds_image_gv4();
        for (uint32_t n = 0; n <= 700; n++)
            for (uint32_t f : {0u, 1u, 3u, 4u, 5u, 17u, 63u, 100u, 124u, 127u}) {
                const uint32_t init = (n % 5 == 0) ? 0u : (uint32_t)rng();
                const int q = (int)((n + f) % 8);
                const uint8_t* blk = buf.data() + (n * 7 + f) % 5000;
                const uint32_t want = ~ref_update(~init, blk, n);
                const uint32_t got = emulate_gv4(imgg, blk, n, f, init, q);
                cases++;
                if (want != got && bad++ < 10) printf("gv4 mismatch n=%u f=%u q=%d %08x %08x\n", n, f, q, want, got);
            }
    }
    {
        auto aux = build_aux();
        std::vector<uint8_t> big(3 << 20);
        for (auto& b : big) b = (uint8_t)rng();
        for (uint32_t n : {1u, 1000u, 65536u, 65537u, 200000u, (uint32_t)big.size() - 7})
            for (uint32_t cs : {128u, 4096u, 65536u}) {
                if ((n + cs - 1) / cs > 2048) continue;
                const uint32_t init = (uint32_t)rng();
                const uint32_t want = ~ref_update(~init, big.data(), n);
                const uint32_t got = emulate_split(aux, big.data(), n, cs, init);
                cases++;
                if (want != got && bad++ < 10) printf("split mismatch n=%u cs=%u %08x %08x\n", n, cs, want, got);
            }
    }
    printf("%d cases, %d mismatches\n", cases, bad);
    return bad != 0;
}
