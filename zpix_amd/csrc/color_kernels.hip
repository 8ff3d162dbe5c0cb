// gfx950 kernels for the colour side of the path:
//   - rgba_pixels_kernel: Image.rgbaPixels (src/image/image.zig:103-130) for
//     every image.Image kind, i.e. at() + Color.toRGBA() (src/color/color.zig:
//     31-131) + >>8, four pixels per lane, 16-byte stores;
//   - jpeg_rgb_kernel: convertToRGB (src/jpeg/decoder.zig:751-783);
//   - jpeg_cmyk_kernel: applyBlack's CMYK branch (decoder.zig:848-902).
// All are streaming, HBM-bound passes.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "device_types.h"
#include "kernels.h"

namespace zpx {
namespace {

__device__ __forceinline__ uint32_t pack4(uint32_t r, uint32_t g, uint32_t b, uint32_t a)
{
    return r | g << 8 | b << 16 | a << 24;
}

// Color.toRGBA .ycbcr then >>8 (color.zig:90-113): clamp(v>>16, 0, 255).
__device__ __forceinline__ uint32_t ycc_rgba8(int32_t Y, int32_t Cb, int32_t Cr)
{
    const int32_t yy1 = __mul24(Y, 0x10101), cb1 = Cb - 128, cr1 = Cr - 128;
    const int32_t r = yy1 + __mul24(91881, cr1);
    const int32_t g = yy1 - __mul24(22554, cb1) - __mul24(46802, cr1);
    const int32_t b = yy1 + __mul24(116130, cb1);
    // clamp before the shift: (v>>16 clamped to 0..255) == clamp(v, 0, 2^24-1) >> 16.  Written
    // this way hipcc (ROCm 7.2) does not select v_ashr_pk_u8_i32, which produced a wrong blue
    // byte on gfx950.
    return pack4(static_cast<uint32_t>(min(max(r, 0), 0xffffff)) >> 16, static_cast<uint32_t>(min(max(g, 0), 0xffffff)) >> 16,
                 static_cast<uint32_t>(min(max(b, 0), 0xffffff)) >> 16, 255);
}

// .nrgba premultiply (color.zig:52-72): ((c*0x101)*a/0xff) >> 8
__device__ __forceinline__ uint32_t nrgba_rgba8(uint32_t r, uint32_t g, uint32_t b, uint32_t a)
{
    return pack4(((r * 0x101u) * a / 0xffu) >> 8, ((g * 0x101u) * a / 0xffu) >> 8,
                 ((b * 0x101u) * a / 0xffu) >> 8, a);
}

__device__ __forceinline__ uint32_t be16(const uint8_t *p) { return uint32_t(p[0]) << 8 | p[1]; }

__device__ uint32_t pixel_rgba8(const DevImage &m, int x, int y)
{
    const size_t dy = static_cast<size_t>(y), dx = static_cast<size_t>(x);
    switch (m.kind) {
    case ZPX_GRAY: {
        const uint32_t v = m.pixels[dy * m.stride + dx];
        return pack4(v, v, v, 255);
    }
    case ZPX_GRAY16: {
        const uint32_t v = m.pixels[dy * m.stride + 2 * dx]; // (v16 >> 8)
        return pack4(v, v, v, 255);
    }
    case ZPX_YCBCR: {
        // YCbCrAt (image.zig:614-630) with cOffset (:594-605); rect.min is 0
        size_t ci;
        switch (m.subsample) {
        case ZPX_RATIO422: ci = dy * m.c_stride + dx / 2; break;
        case ZPX_RATIO420: ci = (dy / 2) * m.c_stride + dx / 2; break;
        case ZPX_RATIO440: ci = (dy / 2) * m.c_stride + dx; break;
        case ZPX_RATIO411: ci = dy * m.c_stride + dx / 4; break;
        case ZPX_RATIO410: ci = (dy / 2) * m.c_stride + dx / 4; break;
        default: ci = dy * m.c_stride + dx; break;
        }
        return ycc_rgba8(m.pixels[m.y_off + dy * m.y_stride + dx], m.pixels[m.cb_off + ci],
                         m.pixels[m.cr_off + ci]);
    }
    case ZPX_RGBA:
        return *reinterpret_cast<const uint32_t *>(m.pixels + dy * m.stride + 4 * dx);
    case ZPX_RGBA64: { // high byte of each BE channel
        const uint8_t *p = m.pixels + dy * m.stride + 8 * dx;
        return pack4(p[0], p[2], p[4], p[6]);
    }
    case ZPX_NRGBA: {
        const uint8_t *p = m.pixels + dy * m.stride + 4 * dx;
        return nrgba_rgba8(p[0], p[1], p[2], p[3]);
    }
    case ZPX_NRGBA64: { // color.zig:73-89: c*a/0xffff, then >>8
        const uint8_t *p = m.pixels + dy * m.stride + 8 * dx;
        const uint32_t a = be16(p + 6);
        return pack4((be16(p) * a / 0xffffu) >> 8, (be16(p + 2) * a / 0xffffu) >> 8,
                     (be16(p + 4) * a / 0xffffu) >> 8, a >> 8);
    }
    case ZPX_CMYK: { // color.zig:115-121
        const uint8_t *p = m.pixels + dy * m.stride + 4 * dx;
        const uint32_t w = 0xffffu - uint32_t(p[3]) * 0x101u;
        return pack4(((0xffffu - uint32_t(p[0]) * 0x101u) * w / 0xffffu) >> 8,
                     ((0xffffu - uint32_t(p[1]) * 0x101u) * w / 0xffffu) >> 8,
                     ((0xffffu - uint32_t(p[2]) * 0x101u) * w / 0xffffu) >> 8, 255);
    }
    case ZPX_PALETTED: { // PalettedImage.at (image.zig:856-866)
        if (m.palette_len == 0) return 0;
        const int idx = m.pixels[dy * m.stride + dx];
        if (idx >= m.palette_len) return 0;
        const zpx_color c = reinterpret_cast<const zpx_color *>(m.palette)[idx];
        return c.model == 0 ? pack4(c.r, c.g, c.b, c.a) : nrgba_rgba8(c.r, c.g, c.b, c.a);
    }
    }
    return 0;
}

__global__ __launch_bounds__(256) void rgba_pixels_kernel(DevImage m, uint8_t *__restrict__ out)
{
    const int y = blockIdx.y;
    const int x0 = (blockIdx.x * 256 + threadIdx.x) * 4;
    if (x0 >= m.width) return;
    uint8_t *o = out + (static_cast<size_t>(y) * m.width + x0) * 4;
    uint32_t p[4];
#pragma unroll
    for (int i = 0; i < 4; i++) p[i] = x0 + i < m.width ? pixel_rgba8(m, x0 + i, y) : 0;
    if (x0 + 4 <= m.width && (reinterpret_cast<uintptr_t>(o) & 15) == 0) {
        *reinterpret_cast<uint4 *>(o) = make_uint4(p[0], p[1], p[2], p[3]);
    } else {
        for (int i = 0; i < 4 && x0 + i < m.width; i++) reinterpret_cast<uint32_t *>(o)[i] = p[i];
    }
}

// convertToRGB: R = Y, G = Cb, B = Cr with c_scale horizontal and cOffset
// vertical indexing, A = 255.
__global__ __launch_bounds__(256) void jpeg_rgb_kernel(DevImage m, int c_scale, uint8_t *__restrict__ out)
{
    const int y = blockIdx.y;
    const int x = blockIdx.x * 256 + threadIdx.x;
    if (x >= m.width) return;
    const size_t dy = static_cast<size_t>(y);
    size_t co;
    switch (m.subsample) {
    case ZPX_RATIO420: case ZPX_RATIO440: case ZPX_RATIO410: co = (dy / 2) * m.c_stride; break;
    default: co = dy * m.c_stride; break;
    }
    const size_t xi = static_cast<size_t>(x);
    const uint32_t Y = m.pixels[m.y_off + dy * m.y_stride + xi];
    const uint32_t Cb = m.pixels[m.cb_off + co + xi / c_scale];
    const uint32_t Cr = m.pixels[m.cr_off + co + xi / c_scale];
    reinterpret_cast<uint32_t *>(out + dy * m.width * 4)[x] = pack4(Y, Cb, Cr, 255);
}

// applyBlack, CMYK branch: interleave 255 - v with 2x subsampling per channel.
__global__ __launch_bounds__(256) void jpeg_cmyk_kernel(DevImage m, const uint8_t *__restrict__ k_plane,
                                                        uint64_t k_stride, uint32_t sub_mask,
                                                        uint8_t *__restrict__ out)
{
    const int y = blockIdx.y;
    const int x = blockIdx.x * 256 + threadIdx.x;
    if (x >= m.width) return;
    const uint8_t *src[4] = {m.pixels + m.y_off, m.pixels + m.cb_off, m.pixels + m.cr_off, k_plane};
    const size_t str[4] = {m.y_stride, m.c_stride, m.c_stride, k_stride};
    uint32_t v[4];
#pragma unroll
    for (int t = 0; t < 4; t++) {
        size_t sy = static_cast<size_t>(y), sx = static_cast<size_t>(x);
        if (sub_mask & (1u << t)) {
            sy >>= 1;
            sx >>= 1;
        }
        v[t] = 255u - src[t][sy * str[t] + sx];
    }
    reinterpret_cast<uint32_t *>(out + static_cast<size_t>(y) * m.width * 4)[x] = pack4(v[0], v[1], v[2], v[3]);
}

} // namespace

int launch_rgba_pixels(const DevImage &m, uint8_t *out, hipStream_t s)
{
    if (m.width <= 0 || m.height <= 0) return 0;
    dim3 grid((m.width + 1023) / 1024, m.height);
    hipLaunchKernelGGL(rgba_pixels_kernel, grid, dim3(256), 0, s, m, out);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_jpeg_rgb(const DevImage &m, int c_scale, uint8_t *out, hipStream_t s)
{
    dim3 grid((m.width + 255) / 256, m.height);
    hipLaunchKernelGGL(jpeg_rgb_kernel, grid, dim3(256), 0, s, m, c_scale, out);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_jpeg_cmyk(const DevImage &m, const uint8_t *k_plane, uint64_t k_stride, uint32_t sub_mask,
                     uint8_t *out, hipStream_t s)
{
    dim3 grid((m.width + 255) / 256, m.height);
    hipLaunchKernelGGL(jpeg_cmyk_kernel, grid, dim3(256), 0, s, m, k_plane, k_stride, sub_mask, out);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

} // namespace zpx
