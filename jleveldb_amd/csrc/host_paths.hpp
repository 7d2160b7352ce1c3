// host_paths.hpp — host (SSE4.2) forms of the host-memory batch entry points,
// taken for calls below JL_OPT_HOST_THRESHOLD (host_paths.cpp).
#pragma once
#include <cstdint>

#include "../../include/jlcrc.h"

namespace jlhost {
void batch(const uint8_t *base, const uint64_t *off, const uint32_t *len, const uint32_t *init, const uint8_t *suffix,
           uint64_t n, uint32_t flags, uint32_t *out);
void fixed(const uint8_t *data, uint64_t block_bytes, uint64_t n, uint32_t flags, uint32_t *out);
void table_verify(const uint8_t *file, const uint64_t *off, const uint32_t *size, uint64_t n, uint8_t *status);
void log_verify(const uint8_t *log, uint64_t bytes, int checksum, jl_log_event *ev, uint64_t cap, uint64_t *n_events);
}  // namespace jlhost
