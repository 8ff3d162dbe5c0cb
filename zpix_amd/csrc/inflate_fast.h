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
// Two streams decoded together on this thread (their decode chains overlap):
// ok[k] and produced[k] are inflate_fast's result for stream k.
void inflate_fast_pair(const uint8_t *const in[2], const size_t in_len[2], uint8_t *const out[2], const size_t want[2],
                       size_t produced[2], bool ok[2]);
// Releases inflate_parallel's recycled symbol buffers; the bytes released.
size_t inflate_pool_trim();
}
