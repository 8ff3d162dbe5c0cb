// Fast zlib stream decoder (fast path of the PNG host inflate; see
// inflate_fast.cpp).  Returns true when the first `want` bytes of the stream
// decoded cleanly into out[0..want); false on anything irregular, in which
// case the caller re-runs system zlib.
#pragma once

#include <cstddef>
#include <cstdint>

namespace zpx {
bool inflate_fast(const uint8_t *in, size_t in_len, uint8_t *out, size_t want, size_t *produced);
// The same contract, decoded by `threads` threads (speculative chunks; false
// on anything irregular, the caller then runs the serial decoder).
bool inflate_parallel(const uint8_t *in, size_t in_len, uint8_t *out, size_t want, size_t *produced, int threads);
}
