// gfx950 Adam7 merge (mergePassInto, src/png/decoder.zig:1289-1373, for the
// even output rows).  The paired-row unfilter kernel writes passes 1-6 of an
// interlaced image into a staging area as contiguous rows (whole-line stores)
// instead of scattering their pixels xf apart into the image: scattered, each
// 128-byte line of an even row is written in 2-4 partial pieces at different
// times, and a 64 x 4K RGBA16 launch took 8.1 ms against 5.0 ms for the same
// bytes without interlacing (5.0 ms with the scatter stores made contiguous,
// a timing-only build).  This kernel then builds every even row from the
// staged passes with whole 16-byte stores: per lane one 16-byte piece of the
// row (2 RGBA16 / 4 RGBA8 pixels), each pixel gathered from the pass that
// owns it (`interlacing`, decoder.zig:59-67).  Pass 7 (the odd rows) is
// written by the unfilter kernel directly.  Streaming, HBM-bound: the staged
// bytes are read once, the even rows written once.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdlib>

#include "device_types.h"
#include "kernels.h"

namespace zpx {
namespace {

#ifndef ZPX_A7_NT
#define ZPX_A7_NT 0 // 1: non-temporal stores of the merged rows
#endif
typedef uint32_t v4u __attribute__((ext_vector_type(4)));
typedef uint32_t v2u __attribute__((ext_vector_type(2)));

// Adam7 pass (0-based) owning pixel (x, y) of an even row y, with its column
// and row inside the pass.
__device__ __forceinline__ int adam7_owner(uint32_t x, uint32_t y, uint32_t &col, uint32_t &row)
{
    if (x & 1) { // pass 6: xo 1, xf 2, yo 0, yf 2
        col = x >> 1;
        row = y >> 1;
        return 5;
    }
    if (y & 2) { // pass 5: xo 0, xf 2, yo 2, yf 4
        col = x >> 1;
        row = y >> 2;
        return 4;
    }
    if (x & 2) { // pass 4: xo 2, xf 4, yo 0, yf 4
        col = x >> 2;
        row = y >> 2;
        return 3;
    }
    if (y & 4) { // pass 3: xo 0, xf 4, yo 4, yf 8
        col = x >> 2;
        row = y >> 3;
        return 2;
    }
    col = x >> 3;
    row = y >> 3;
    return (x & 4) ? 1 : 0; // pass 2: xo 4, xf 8; pass 1: xo 0, xf 8 (yo 0, yf 8)
}

template <int OBPX>
__device__ __forceinline__ void copy_px(const DevAdam7Merge &m, uint32_t x, uint32_t y, uint8_t *dst)
{
    uint32_t col, row;
    const int p = adam7_owner(x, y, col, row);
    const uint8_t *src = m.stage[p] + static_cast<size_t>(row) * m.sstride[p] + static_cast<size_t>(col) * OBPX;
    if constexpr (OBPX == 8)
        *reinterpret_cast<v2u *>(dst) = *reinterpret_cast<const v2u *>(src);
    else
        *reinterpret_cast<uint32_t *>(dst) = *reinterpret_cast<const uint32_t *>(src);
}

// grid: x = even rows (block-stride), y = image; a block's threads stride
// over the row's 16-byte pieces
template <int OBPX>
__global__ __launch_bounds__(256) void png_adam7_merge_kernel(const DevAdam7Merge *__restrict__ jobs)
{
    const DevAdam7Merge &m = jobs[blockIdx.y];
    constexpr uint32_t PPS = 16 / OBPX; // pixels per piece
    const uint32_t width = m.width, pieces = (width + PPS - 1) / PPS, erows = (m.height + 1) / 2;
    const bool vec = (reinterpret_cast<uintptr_t>(m.out) & 15) == 0 && (m.out_stride & 15) == 0;
    for (uint32_t r = blockIdx.x; r < erows; r += gridDim.x) {
        const uint32_t y = 2 * r;
        uint8_t *row = m.out + static_cast<size_t>(y) * m.out_stride;
        for (uint32_t s = threadIdx.x; s < pieces; s += blockDim.x) {
            const uint32_t x0 = s * PPS;
            uint8_t *d = row + static_cast<size_t>(x0) * OBPX;
            if (vec && x0 + PPS <= width) {
                uint32_t v[4];
#pragma unroll
                for (uint32_t k = 0; k < PPS; k++)
                    copy_px<OBPX>(m, x0 + k, y, reinterpret_cast<uint8_t *>(v) + k * OBPX);
    #if ZPX_A7_NT
            __builtin_nontemporal_store(v4u{v[0], v[1], v[2], v[3]}, reinterpret_cast<v4u *>(d));
#else
            *reinterpret_cast<v4u *>(d) = v4u{v[0], v[1], v[2], v[3]};
#endif
            } else { // ragged right edge or unaligned rows: pixel stores
                for (uint32_t k = 0; k < PPS && x0 + k < width; k++) copy_px<OBPX>(m, x0 + k, y, d + k * OBPX);
            }
        }
    }
}

} // namespace

int launch_png_adam7_merge(int obpx, const DevAdam7Merge *d_jobs, int njobs, uint32_t max_erows, hipStream_t s)
{
    if (njobs <= 0 || max_erows == 0) return 0;
    // about 32,768 blocks in all, a block per even row of an image at a time
    // (64 x 4K RGBA16: 1.59 ms; 8,192 blocks 1.60, 2,048 1.62; RGBA8 0.82 /
    // 0.91 / 0.85)
    constexpr uint32_t total = 32768u;
    uint32_t per = (total + static_cast<uint32_t>(njobs) - 1) / static_cast<uint32_t>(njobs);
    per = per < max_erows ? per : max_erows;
    const dim3 grid(per, static_cast<uint32_t>(njobs));
    if (obpx == 8)
        hipLaunchKernelGGL(png_adam7_merge_kernel<8>, grid, dim3(256), 0, s, d_jobs);
    else if (obpx == 4)
        hipLaunchKernelGGL(png_adam7_merge_kernel<4>, grid, dim3(256), 0, s, d_jobs);
    else
        return -2;
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

} // namespace zpx
