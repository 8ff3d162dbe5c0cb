// CRC-32 (ISO-HDLC, PNG's chunk CRC) by carry-less multiplication folding
// (Intel, "Fast CRC Computation for Generic Polynomials Using PCLMULQDQ",
// bit-reflected constants; the arrangement zlib's SIMD ports use): 4 x 128-bit
// lanes folded per 64 bytes, Barrett reduction to 32 bits.  The tail (< 16 B)
// and CPUs without PCLMULQDQ go through zlib's crc32, so the value is zlib's.
// verifyChecksum (src/png/decoder.zig:1264-1277) runs over every IDAT byte;
// zlib's table CRC was ~20 % of the PNG host stage.
#include "crc32_fast.h"

#include <immintrin.h>
#include <zlib.h>

namespace zpx {
namespace {

__attribute__((target("pclmul,sse4.1")))
uint32_t crc32_fold(const unsigned char *buf, size_t len, uint32_t crc) {
    alignas(16) static const uint64_t k1k2[] = { 0x0154442bd4, 0x01c6e41596 };
    alignas(16) static const uint64_t k3k4[] = { 0x01751997d0, 0x00ccaa009e };
    alignas(16) static const uint64_t k5k0[] = { 0x0163cd6124, 0x0000000000 };
    alignas(16) static const uint64_t poly[] = { 0x01db710641, 0x01f7011641 };
    __m128i x0, x1, x2, x3, x4, x5, x6, x7, x8, y5, y6, y7, y8;
    x1 = _mm_loadu_si128((const __m128i *)(buf + 0x00));
    x2 = _mm_loadu_si128((const __m128i *)(buf + 0x10));
    x3 = _mm_loadu_si128((const __m128i *)(buf + 0x20));
    x4 = _mm_loadu_si128((const __m128i *)(buf + 0x30));
    x1 = _mm_xor_si128(x1, _mm_cvtsi32_si128(crc));
    x0 = _mm_load_si128((const __m128i *)k1k2);
    buf += 64; len -= 64;
    while (len >= 64) {
        x5 = _mm_clmulepi64_si128(x1, x0, 0x00); x6 = _mm_clmulepi64_si128(x2, x0, 0x00);
        x7 = _mm_clmulepi64_si128(x3, x0, 0x00); x8 = _mm_clmulepi64_si128(x4, x0, 0x00);
        x1 = _mm_clmulepi64_si128(x1, x0, 0x11); x2 = _mm_clmulepi64_si128(x2, x0, 0x11);
        x3 = _mm_clmulepi64_si128(x3, x0, 0x11); x4 = _mm_clmulepi64_si128(x4, x0, 0x11);
        y5 = _mm_loadu_si128((const __m128i *)(buf + 0x00)); y6 = _mm_loadu_si128((const __m128i *)(buf + 0x10));
        y7 = _mm_loadu_si128((const __m128i *)(buf + 0x20)); y8 = _mm_loadu_si128((const __m128i *)(buf + 0x30));
        x1 = _mm_xor_si128(_mm_xor_si128(x1, x5), y5); x2 = _mm_xor_si128(_mm_xor_si128(x2, x6), y6);
        x3 = _mm_xor_si128(_mm_xor_si128(x3, x7), y7); x4 = _mm_xor_si128(_mm_xor_si128(x4, x8), y8);
        buf += 64; len -= 64;
    }
    x0 = _mm_load_si128((const __m128i *)k3k4);
    x5 = _mm_clmulepi64_si128(x1, x0, 0x00); x1 = _mm_clmulepi64_si128(x1, x0, 0x11);
    x1 = _mm_xor_si128(_mm_xor_si128(x1, x2), x5);
    x5 = _mm_clmulepi64_si128(x1, x0, 0x00); x1 = _mm_clmulepi64_si128(x1, x0, 0x11);
    x1 = _mm_xor_si128(_mm_xor_si128(x1, x3), x5);
    x5 = _mm_clmulepi64_si128(x1, x0, 0x00); x1 = _mm_clmulepi64_si128(x1, x0, 0x11);
    x1 = _mm_xor_si128(_mm_xor_si128(x1, x4), x5);
    while (len >= 16) {
        x2 = _mm_loadu_si128((const __m128i *)buf);
        x5 = _mm_clmulepi64_si128(x1, x0, 0x00); x1 = _mm_clmulepi64_si128(x1, x0, 0x11);
        x1 = _mm_xor_si128(_mm_xor_si128(x1, x2), x5);
        buf += 16; len -= 16;
    }
    x2 = _mm_clmulepi64_si128(x1, x0, 0x10);
    x3 = _mm_setr_epi32(~0, 0, ~0, 0);
    x1 = _mm_srli_si128(x1, 8);
    x1 = _mm_xor_si128(x1, x2);
    x0 = _mm_loadl_epi64((const __m128i*)k5k0);
    x2 = _mm_srli_si128(x1, 4);
    x1 = _mm_and_si128(x1, x3);
    x1 = _mm_clmulepi64_si128(x1, x0, 0x00);
    x1 = _mm_xor_si128(x1, x2);
    x0 = _mm_load_si128((const __m128i*)poly);
    x2 = _mm_and_si128(x1, x3);
    x2 = _mm_clmulepi64_si128(x2, x0, 0x10);
    x2 = _mm_and_si128(x2, x3);
    x2 = _mm_clmulepi64_si128(x2, x0, 0x00);
    x1 = _mm_xor_si128(x1, x2);
    return (uint32_t)_mm_extract_epi32(x1, 1);
}
} // namespace

uint32_t crc32_fast(uint32_t crc, const uint8_t *buf, size_t len)
{
    static const bool simd = __builtin_cpu_supports("pclmul") && __builtin_cpu_supports("sse4.1");
    if (!simd) return static_cast<uint32_t>(::crc32(crc, buf, static_cast<uInt>(len)));
    if (len >= 64) {
        size_t chunk = len & ~size_t(15);
        crc = ~crc32_fold(buf, chunk, ~crc);
        buf += chunk; len -= chunk;
    }
    return len ? static_cast<uint32_t>(::crc32(crc, buf, static_cast<uInt>(len))) : crc;
}

} // namespace zpx
