// Integer IDCT of the JPEG pixel path shared by the gfx950 kernels
// (src/jpeg/idct.zig:77-201, bit-identical wrap-around i32 arithmetic; the
// translation units are built with -fwrapv).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#define ZPX_GLOBAL __attribute__((address_space(1)))

namespace zpx {
namespace {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef int32_t i32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

// natural -> zig-zag index (the inverse of decoder.zig:73-82's unzig table):
// ZPX_COEFFS_PIECES blocks hold their coefficients in zig-zag order
constexpr uint8_t kZigOf[64] = {0,  1,  5,  6,  14, 15, 27, 28, 2,  4,  7,  13, 16, 26, 29, 42,
                                3,  8,  12, 17, 25, 30, 41, 43, 9,  11, 18, 24, 31, 40, 44, 53,
                                10, 19, 23, 32, 39, 45, 52, 54, 20, 22, 33, 38, 46, 51, 55, 60,
                                21, 34, 37, 47, 50, 56, 59, 61, 35, 36, 48, 49, 57, 58, 62, 63};

// idct.zig:50-65
constexpr int32_t W1 = 2841, W2 = 2676, W3 = 2408, W5 = 1609, W6 = 1108, W7 = 565;
constexpr int32_t R2 = 181;

// Left shift with two's-complement wrap (no UB for negative operands).
__device__ __forceinline__ int32_t shl(int32_t x, int n) { return static_cast<int32_t>(static_cast<uint32_t>(x) << n); }

// Multiply by an IDCT constant.  NARROW: the host proved every operand of the
// stage-1/2 products fits in 24 signed bits (max |coef*q| <= 16384, see
// DESIGN.md), so v_mul_i32_i24 gives the same low 32 bits as a 32-bit product.
template <bool NARROW>
__device__ __forceinline__ int32_t mulc(int32_t c, int32_t x)
{
    if constexpr (NARROW) return __mul24(c, x);
    else return c * x;
}

// Horizontal 1-D IDCT of one row (idct.zig:79-145).  s[] holds dequantized
// coefficients of the row in natural order.
template <bool NARROW>
__device__ __forceinline__ void idct_row(int32_t s[8])
{
    const int32_t dc = s[0];
    const bool ac_zero = (s[1] | s[2] | s[3] | s[4] | s[5] | s[6] | s[7]) == 0;
    int32_t x0 = shl(s[0], 11) + 128, x1 = shl(s[4], 11), x2 = s[6], x3 = s[2];
    int32_t x4 = s[1], x5 = s[7], x6 = s[5], x7 = s[3], x8;
    x8 = mulc<NARROW>(W7, x4 + x5);
    x4 = x8 + mulc<NARROW>(W1 - W7, x4);
    x5 = x8 - mulc<NARROW>(W1 + W7, x5);
    x8 = mulc<NARROW>(W3, x6 + x7);
    x6 = x8 - mulc<NARROW>(W3 - W5, x6);
    x7 = x8 - mulc<NARROW>(W3 + W5, x7);
    x8 = x0 + x1;
    x0 -= x1;
    x1 = mulc<NARROW>(W6, x3 + x2);
    x2 = x1 - mulc<NARROW>(W2 + W6, x2);
    x3 = x1 + mulc<NARROW>(W2 - W6, x3);
    x1 = x4 + x6;
    x4 -= x6;
    x6 = x5 + x7;
    x5 -= x7;
    x7 = x8 + x3;
    x8 -= x3;
    x3 = x0 + x2;
    x0 -= x2;
    x2 = (R2 * (x4 + x5) + 128) >> 8;
    x4 = (R2 * (x4 - x5) + 128) >> 8;
    s[0] = (x7 + x1) >> 8;
    s[1] = (x3 + x2) >> 8;
    s[2] = (x0 + x4) >> 8;
    s[3] = (x8 + x6) >> 8;
    s[4] = (x8 - x6) >> 8;
    s[5] = (x0 - x4) >> 8;
    s[6] = (x3 - x2) >> 8;
    s[7] = (x7 - x1) >> 8;
    if constexpr (!NARROW) {
        // DC-only shortcut (idct.zig:84-97).  Identical to the full path
        // unless dc<<11 overflows, which only the wide variant can see.
        if (ac_zero) {
            const int32_t d = shl(dc, 3);
#pragma unroll
            for (int i = 0; i < 8; i++) s[i] = d;
        }
    } else {
        (void)dc;
        (void)ac_zero;
    }
}

// Vertical 1-D IDCT of one column (idct.zig:148-200) + level shift and clamp
// (decoder.zig:1622-1628): c<-128 -> 0, c>127 -> 255, else c+128.
// SIGNED_OUT leaves the level shift out: the sample minus 128, clamp(c, -128,
// 127), one instruction less per sample (callers fold the +128 into their
// colour constants, or into a per-dword xor 0x80 of packed bytes).
template <bool NARROW, bool SIGNED_OUT = false>
__device__ __forceinline__ void idct_col_clamp(int32_t s[8])
{
    int32_t y0 = shl(s[0], 8) + 8192, y1 = shl(s[4], 8), y2 = s[6], y3 = s[2];
    int32_t y4 = s[1], y5 = s[7], y6 = s[5], y7 = s[3], y8;
    y8 = mulc<NARROW>(W7, y4 + y5) + 4;
    y4 = (y8 + mulc<NARROW>(W1 - W7, y4)) >> 3;
    y5 = (y8 - mulc<NARROW>(W1 + W7, y5)) >> 3;
    y8 = mulc<NARROW>(W3, y6 + y7) + 4;
    y6 = (y8 - mulc<NARROW>(W3 - W5, y6)) >> 3;
    y7 = (y8 - mulc<NARROW>(W3 + W5, y7)) >> 3;
    y8 = y0 + y1;
    y0 -= y1;
    y1 = mulc<NARROW>(W6, y3 + y2) + 4;
    y2 = (y1 - mulc<NARROW>(W2 + W6, y2)) >> 3;
    y3 = (y1 + mulc<NARROW>(W2 - W6, y3)) >> 3;
    y1 = y4 + y6;
    y4 -= y6;
    y6 = y5 + y7;
    y5 -= y7;
    y7 = y8 + y3;
    y8 -= y3;
    y3 = y0 + y2;
    y0 -= y2;
    y2 = (R2 * (y4 + y5) + 128) >> 8;
    y4 = (R2 * (y4 - y5) + 128) >> 8;
    s[0] = (y7 + y1) >> 14;
    s[1] = (y3 + y2) >> 14;
    s[2] = (y0 + y4) >> 14;
    s[3] = (y8 + y6) >> 14;
    s[4] = (y8 - y6) >> 14;
    s[5] = (y0 - y4) >> 14;
    s[6] = (y3 - y2) >> 14;
    s[7] = (y7 - y1) >> 14;
#pragma unroll
    for (int i = 0; i < 8; i++) s[i] = min(max(s[i], -128), 127) + (SIGNED_OUT ? 0 : 128);
}


} // namespace
} // namespace zpx
