// gfx950 kernel for the pixel loop of bmp.decode (src/bmp/decoder.zig:160-307).
//
// The host parses the header and palette (readHeader, :42-158) and uploads the
// pixel-data region as it lies in the file: `height` rows of `row_bytes` each,
// bottom-up unless the height was negative.  One lane produces four output
// pixels of one row:
//   - 1/2/4/8 bpp: palette indices, MSB-first within a byte (:209-220);
//   - 24 bpp: B,G,R -> R,G,B,0xFF (.RGBA, :256-266);
//   - 32 bpp: B,G,R,A -> R,G,B,A, with A forced to 0xFF unless the header is
//     V4/V5 (.NRGBA, :291-303).
// A streaming, HBM-bound pass: every byte is read once and written once.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "kernels.h"

namespace zpx {
namespace {

template <int BPP, bool ALPHA>
__global__ __launch_bounds__(256) void bmp_rows_kernel(const uint8_t *__restrict__ src, uint64_t row_bytes,
                                                       uint8_t *__restrict__ dst, uint64_t dst_stride,
                                                       uint32_t width, uint32_t height, int top_down)
{
    const uint32_t groups = (width + 3) / 4;
    const uint64_t total = uint64_t(groups) * height;
    for (uint64_t t = uint64_t(blockIdx.x) * 256 + threadIdx.x; t < total; t += uint64_t(gridDim.x) * 256) {
        const uint32_t y = static_cast<uint32_t>(t / groups), g = static_cast<uint32_t>(t % groups);
        const uint32_t k = top_down ? y : height - 1 - y; // file row that holds image row y
        const uint8_t *s = src + uint64_t(k) * row_bytes;
        const uint32_t x0 = 4 * g, npx = min(4u, width - x0);
        uint8_t *d = dst + uint64_t(y) * dst_stride;
        if constexpr (BPP == 24 || BPP == 32) {
            uint32_t px[4];
            if constexpr (BPP == 24) {
                if (npx == 4) { // 12 bytes at a 4-aligned offset
                    const uint32_t *w = reinterpret_cast<const uint32_t *>(s + 12 * g);
                    const uint32_t a = w[0], b = w[1], c = w[2];
                    const uint64_t lo = uint64_t(b) << 32 | a, hi = uint64_t(c) << 16 | (b >> 16);
                    px[0] = uint32_t(lo);
                    px[1] = uint32_t(lo >> 24);
                    px[2] = uint32_t(hi);
                    px[3] = uint32_t(hi >> 24);
                } else {
                    for (uint32_t i = 0; i < npx; i++) {
                        const uint8_t *p = s + 3 * (x0 + i);
                        px[i] = p[0] | uint32_t(p[1]) << 8 | uint32_t(p[2]) << 16;
                    }
                }
#pragma unroll
                for (int i = 0; i < 4; i++) // BGR -> RGBA, A = 0xFF
                    px[i] = (px[i] >> 16 & 0xff) | (px[i] & 0xff00) | (px[i] & 0xff) << 16 | 0xff000000u;
            } else {
                const uint32_t *w = reinterpret_cast<const uint32_t *>(s) + x0;
#pragma unroll
                for (int i = 0; i < 4; i++) {
                    const uint32_t v = i < (int)npx ? w[i] : 0;
                    px[i] = (v >> 16 & 0xff) | (v & 0xff00) | (v & 0xff) << 16 | (ALPHA ? (v & 0xff000000u) : 0xff000000u);
                }
            }
            uint32_t *o = reinterpret_cast<uint32_t *>(d) + x0;
            if (npx == 4 && ((reinterpret_cast<uintptr_t>(o) & 15) == 0)) {
                *reinterpret_cast<uint4 *>(o) = make_uint4(px[0], px[1], px[2], px[3]);
            } else {
                for (uint32_t i = 0; i < npx; i++) o[i] = px[i];
            }
        } else {
            uint32_t idx[4];
            if constexpr (BPP == 8) {
                // rows are padded to 4 bytes, so the dword at x0 is inside the row
                const uint32_t v = *reinterpret_cast<const uint32_t *>(s + x0);
#pragma unroll
                for (int i = 0; i < 4; i++) idx[i] = v >> (8 * i) & 0xff;
            } else {
                // 4 pixels = 4*BPP bits starting at bit x0*BPP (MSB first)
                const uint32_t bit0 = x0 * BPP, byte0 = bit0 / 8;
                const uint32_t two = uint32_t(s[byte0]) << 8 | (BPP == 4 ? s[byte0 + 1] : 0u);
                const uint32_t sh0 = 16 - (bit0 % 8) - BPP;
#pragma unroll
                for (int i = 0; i < 4; i++) idx[i] = two >> (sh0 - BPP * i) & ((1u << BPP) - 1);
            }
            uint8_t *o = d + x0;
            if (npx == 4 && ((reinterpret_cast<uintptr_t>(o) & 3) == 0)) {
                *reinterpret_cast<uint32_t *>(o) = idx[0] | idx[1] << 8 | idx[2] << 16 | idx[3] << 24;
            } else {
                for (uint32_t i = 0; i < npx; i++) o[i] = static_cast<uint8_t>(idx[i]);
            }
        }
    }
}

template <int BPP, bool ALPHA>
int launch_t(const uint8_t *src, uint64_t row_bytes, uint8_t *dst, uint64_t dst_stride, uint32_t width,
             uint32_t height, int top_down, hipStream_t s)
{
    const uint64_t total = uint64_t((width + 3) / 4) * height;
    const uint64_t blocks = std::min<uint64_t>((total + 255) / 256, 256 * 64);
    hipLaunchKernelGGL((bmp_rows_kernel<BPP, ALPHA>), dim3(static_cast<uint32_t>(blocks)), dim3(256), 0, s, src,
                       row_bytes, dst, dst_stride, width, height, top_down);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

} // namespace

int launch_bmp_rows(int bpp, bool allow_alpha, const uint8_t *src, uint64_t row_bytes, uint8_t *dst,
                    uint64_t dst_stride, uint32_t width, uint32_t height, int top_down, hipStream_t s)
{
    if (width == 0 || height == 0) return 0;
    switch (bpp) {
    case 1: return launch_t<1, false>(src, row_bytes, dst, dst_stride, width, height, top_down, s);
    case 2: return launch_t<2, false>(src, row_bytes, dst, dst_stride, width, height, top_down, s);
    case 4: return launch_t<4, false>(src, row_bytes, dst, dst_stride, width, height, top_down, s);
    case 8: return launch_t<8, false>(src, row_bytes, dst, dst_stride, width, height, top_down, s);
    case 24: return launch_t<24, false>(src, row_bytes, dst, dst_stride, width, height, top_down, s);
    case 32:
        return allow_alpha ? launch_t<32, true>(src, row_bytes, dst, dst_stride, width, height, top_down, s)
                           : launch_t<32, false>(src, row_bytes, dst, dst_stride, width, height, top_down, s);
    default: return -2;
    }
}

} // namespace zpx
