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

// The same for a batch of images of one kind (zpx_rgba_plan_create): a
// workgroup converts 1,024 pixels of one row of one image (grid z), and for
// the packed kinds each lane reads its 4 pixels as whole 4-32-byte pieces
// (consecutive lanes on consecutive pieces: whole lines per instruction)
// instead of byte by byte through the per-pixel switch; a row's last,
// partial piece and the YCbCr / Paletted kinds take pixel_rgba8.
template <int KIND>
__device__ __forceinline__ uint4 rgba4_packed(const uint8_t *row, int x0)
{
    if constexpr (KIND == ZPX_NRGBA64 || KIND == ZPX_RGBA64) {
        const uint4 a = *reinterpret_cast<const uint4 *>(row + 8 * x0);
        const uint4 b = *reinterpret_cast<const uint4 *>(row + 8 * x0 + 16);
        const uint32_t w[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
        uint32_t o[4];
#pragma unroll
        for (int i = 0; i < 4; i++) {
            const uint32_t lo = w[2 * i], hi = w[2 * i + 1]; // bytes r0 r1 g0 g1 | b0 b1 a0 a1 (big endian)
            if constexpr (KIND == ZPX_RGBA64) {
                o[i] = pack4(lo & 0xff, (lo >> 16) & 0xff, hi & 0xff, (hi >> 16) & 0xff);
            } else { // color.zig:73-89: c*a/0xffff, then >>8
                const uint32_t r = (lo & 0xff) << 8 | ((lo >> 8) & 0xff), g = ((lo >> 16) & 0xff) << 8 | (lo >> 24);
                const uint32_t bl = (hi & 0xff) << 8 | ((hi >> 8) & 0xff), al = ((hi >> 16) & 0xff) << 8 | (hi >> 24);
                o[i] = pack4((r * al / 0xffffu) >> 8, (g * al / 0xffffu) >> 8, (bl * al / 0xffffu) >> 8, al >> 8);
            }
        }
        return make_uint4(o[0], o[1], o[2], o[3]);
    } else if constexpr (KIND == ZPX_RGBA || KIND == ZPX_NRGBA || KIND == ZPX_CMYK) {
        const uint4 a = *reinterpret_cast<const uint4 *>(row + 4 * x0);
        if constexpr (KIND == ZPX_RGBA) return a;
        const uint32_t w[4] = {a.x, a.y, a.z, a.w};
        uint32_t o[4];
#pragma unroll
        for (int i = 0; i < 4; i++) {
            const uint32_t c0 = w[i] & 0xff, c1 = (w[i] >> 8) & 0xff, c2 = (w[i] >> 16) & 0xff, c3 = w[i] >> 24;
            if constexpr (KIND == ZPX_NRGBA) {
                o[i] = nrgba_rgba8(c0, c1, c2, c3);
            } else { // color.zig:115-121
                const uint32_t k = 0xffffu - c3 * 0x101u;
                o[i] = pack4(((0xffffu - c0 * 0x101u) * k / 0xffffu) >> 8, ((0xffffu - c1 * 0x101u) * k / 0xffffu) >> 8,
                             ((0xffffu - c2 * 0x101u) * k / 0xffffu) >> 8, 255);
            }
        }
        return make_uint4(o[0], o[1], o[2], o[3]);
    } else if constexpr (KIND == ZPX_GRAY16) {
        const uint2 a = *reinterpret_cast<const uint2 *>(row + 2 * x0);
        const uint32_t v[4] = {a.x & 0xff, (a.x >> 16) & 0xff, a.y & 0xff, (a.y >> 16) & 0xff}; // the BE high bytes
        return make_uint4(v[0] * 0x010101u | 0xff000000u, v[1] * 0x010101u | 0xff000000u,
                          v[2] * 0x010101u | 0xff000000u, v[3] * 0x010101u | 0xff000000u);
    } else { // ZPX_GRAY
        const uint32_t a = *reinterpret_cast<const uint32_t *>(row + x0);
        return make_uint4((a & 0xff) * 0x010101u | 0xff000000u, ((a >> 8) & 0xff) * 0x010101u | 0xff000000u,
                          ((a >> 16) & 0xff) * 0x010101u | 0xff000000u, (a >> 24) * 0x010101u | 0xff000000u);
    }
}

template <int KIND>
__device__ __forceinline__ void rgba_job_pixels(const DevRgbaJob &j)
{
    const DevImage &m = j.m;
    const int y = blockIdx.y;
    if (y >= m.height) return;
    const int x0 = (blockIdx.x * 256 + threadIdx.x) * 4;
    if (x0 >= m.width) return;
    uint8_t *o = j.out + (static_cast<size_t>(y) * m.width + x0) * 4;
    constexpr bool kPacked = KIND != ZPX_YCBCR && KIND != ZPX_PALETTED;
    if (kPacked && x0 + 4 <= m.width && j.vec) {
        *reinterpret_cast<uint4 *>(o) = rgba4_packed<KIND>(m.pixels + static_cast<size_t>(y) * m.stride, x0);
        return;
    }
    uint32_t p[4];
#pragma unroll
    for (int i = 0; i < 4; i++) p[i] = x0 + i < m.width ? pixel_rgba8(m, x0 + i, y) : 0;
    if (x0 + 4 <= m.width && (reinterpret_cast<uintptr_t>(o) & 15) == 0) {
        *reinterpret_cast<uint4 *>(o) = make_uint4(p[0], p[1], p[2], p[3]);
    } else {
        for (int i = 0; i < 4 && x0 + i < m.width; i++) reinterpret_cast<uint32_t *>(o)[i] = p[i];
    }
}
template <int KIND>
__global__ __launch_bounds__(256) void rgba_batch_kernel(const DevRgbaJob *__restrict__ jobs)
{
    rgba_job_pixels<KIND>(jobs[blockIdx.z]);
}
template <int KIND>
__global__ __launch_bounds__(256) void rgba_one_kernel(DevRgbaJob j)
{
    rgba_job_pixels<KIND>(j);
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

DevRgbaJob rgba_job(const DevImage &m, uint8_t *out)
{
    DevRgbaJob j{};
    j.m = m;
    j.out = out;
    j.vec = (reinterpret_cast<uintptr_t>(m.pixels) & 15) == 0 && (m.stride & 15) == 0 &&
            (reinterpret_cast<uintptr_t>(out) & 15) == 0 && (m.width & 3) == 0;
    return j;
}

int launch_rgba_pixels(const DevImage &m, uint8_t *out, hipStream_t s)
{
    if (m.width <= 0 || m.height <= 0) return 0;
    dim3 grid((m.width + 1023) / 1024, m.height);
    const DevRgbaJob j = rgba_job(m, out);
    switch (m.kind) {
#define ZPX_CASE(K) case K: hipLaunchKernelGGL(rgba_one_kernel<K>, grid, dim3(256), 0, s, j); break;
        ZPX_CASE(ZPX_GRAY) ZPX_CASE(ZPX_GRAY16) ZPX_CASE(ZPX_YCBCR) ZPX_CASE(ZPX_RGBA) ZPX_CASE(ZPX_RGBA64)
        ZPX_CASE(ZPX_NRGBA) ZPX_CASE(ZPX_NRGBA64) ZPX_CASE(ZPX_CMYK) ZPX_CASE(ZPX_PALETTED)
#undef ZPX_CASE
    default: hipLaunchKernelGGL(rgba_pixels_kernel, grid, dim3(256), 0, s, m, out); break;
    }
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_rgba_batch(int kind, const DevRgbaJob *jobs, int n, int max_w, int max_h, hipStream_t s)
{
    if (n <= 0 || max_w <= 0 || max_h <= 0) return 0;
    if (n > 65535 || max_h > 65535) return -2;
    const dim3 grid((max_w + 1023) / 1024, max_h, n);
    switch (kind) {
#define ZPX_CASE(K) case K: hipLaunchKernelGGL(rgba_batch_kernel<K>, grid, dim3(256), 0, s, jobs); break;
        ZPX_CASE(ZPX_GRAY) ZPX_CASE(ZPX_GRAY16) ZPX_CASE(ZPX_YCBCR) ZPX_CASE(ZPX_RGBA) ZPX_CASE(ZPX_RGBA64)
        ZPX_CASE(ZPX_NRGBA) ZPX_CASE(ZPX_NRGBA64) ZPX_CASE(ZPX_CMYK) ZPX_CASE(ZPX_PALETTED)
#undef ZPX_CASE
    default: return -2;
    }
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
