// host_crc.cpp — the scalar Crc32C statics of the C-ABI (include/jlcrc.h, first
// block).  These replace the reference's per-call static methods
// (J/util/Crc32C.java:43-167) for latency-bound single calls (one WAL record
// per write group, instance-API updates); they never sit behind a batch or
// verify entry point.  x86 SSE4.2 `crc32` computes exactly this polynomial
// (CRC-32C); the slicing-by-8 branch is for hosts without it.
#include <cstddef>
#include <cstdint>
#include <cstring>
#include <nmmintrin.h>

#include "../../include/jlcrc.h"
#include "crc_math.hpp"

namespace {

__attribute__((target("sse4.2"))) uint32_t update_sse42(uint32_t s, const uint8_t *p, size_t n) {
    uint64_t c = s;
    while (n >= 8) {
        uint64_t v;
        memcpy(&v, p, 8);
        c = _mm_crc32_u64(c, v);
        p += 8;
        n -= 8;
    }
    uint32_t c32 = (uint32_t)c;
    while (n--) c32 = _mm_crc32_u8(c32, *p++);
    return c32;
}

uint32_t update_sliced(uint32_t s, const uint8_t *p, size_t n) {
    const auto &T = jlmath::tables().t;
    while (n >= 8) {
        uint32_t lo, hi;
        memcpy(&lo, p, 4);
        memcpy(&hi, p + 4, 4);
        lo ^= s;
        s = T[7][lo & 0xff] ^ T[6][(lo >> 8) & 0xff] ^ T[5][(lo >> 16) & 0xff] ^ T[4][lo >> 24] ^ T[3][hi & 0xff] ^
            T[2][(hi >> 8) & 0xff] ^ T[1][(hi >> 16) & 0xff] ^ T[0][hi >> 24];
        p += 8;
        n -= 8;
    }
    while (n--) s = (s >> 8) ^ T[0][(s ^ *p++) & 0xff];
    return s;
}

const bool g_sse42 = __builtin_cpu_supports("sse4.2");

}  // namespace

extern "C" {

uint32_t jl_crc32c_update(uint32_t state, const uint8_t *data, size_t n) {
    if (n == 0) return state;
    return g_sse42 ? update_sse42(state, data, n) : update_sliced(state, data, n);
}

uint32_t jl_crc32c_value(const uint8_t *data, size_t n) { return ~jl_crc32c_update(0xffffffffu, data, n); }

uint32_t jl_crc32c_extend(uint32_t init_crc, const uint8_t *data, size_t n) {
    return ~jl_crc32c_update(~init_crc, data, n);
}

uint32_t jl_crc32c_mask(uint32_t crc) { return jlmath::mask(crc); }

uint32_t jl_crc32c_unmask(uint32_t masked_crc) { return jlmath::unmask(masked_crc); }

}  // extern "C"
