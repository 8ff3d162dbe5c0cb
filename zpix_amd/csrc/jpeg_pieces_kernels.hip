// gfx950 kernel that expands ZPX_COEFFS_PIECES blocks (JpegPieces,
// jpeg_host.h: the batch pipeline's compact transport of a baseline
// interleaved scan) into the dense natural-order coefficient
// grids that processSos accumulates into (src/jpeg/decoder.zig:1340-1345),
// for the kernels that read grids: the strip kernels, the RGB / CMYK paths
// and the geometries the block kernels' pieces instances do not cover.  The
// common frames never come here: the block kernels read the pieces straight
// into their coefficient image (jpeg_block_kernels.hip).
//
// One lane per block, consecutive lanes on consecutive blocks of one
// component: its index word, its pieces (16-byte loads, at most 4 int8 / 8
// int16 -- the rest zeros), the zig-zag -> natural reorder in registers (each
// output dword gathers its bytes / halves from the pieces by compile-time
// selects), and the block's 64 / 128 bytes as 16-byte stores.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "jpeg_idct.h"
#include "kernels.h"

namespace zpx {
namespace {

template <typename T>
__global__ __launch_bounds__(64) void jpeg_pieces_expand_kernel(const DevPiecesExpand *__restrict__ jobs)
{
    constexpr int P = 4 * static_cast<int>(sizeof(T)); // 16-byte pieces in a dense block
    const DevPiecesExpand j = jobs[blockIdx.y];
    const uint32_t b = blockIdx.x * 64u + threadIdx.x;
    if (b >= j.blocks) return;
    const uint32_t e = j.index[b];
    const uint32_t np = e & 15u;
    const u32x4 *src = reinterpret_cast<const u32x4 *>(j.pieces + static_cast<size_t>(e >> 4) * 16);
    u32x4 raw[P];
#pragma unroll
    for (int q = 0; q < P; q++) raw[q] = static_cast<uint32_t>(q) < np ? src[q] : u32x4{0, 0, 0, 0};
    u32x4 out[P];
#pragma unroll
    for (int d = 0; d < 16 * P / 4; d++) { // output dword d: natural coefficients from d * (4 / sizeof(T))
        uint32_t w = 0;
#pragma unroll
        for (int u = 0; u < 4 / static_cast<int>(sizeof(T)); u++) {
            const int n = d * (4 / static_cast<int>(sizeof(T))) + u;
            const int z = kZigOf[n];
            const int zd = z / (4 / static_cast<int>(sizeof(T))), zs = z % (4 / static_cast<int>(sizeof(T)));
            constexpr uint32_t mask = sizeof(T) == 1 ? 0xffu : 0xffffu;
            const uint32_t v = (raw[zd >> 2][zd & 3] >> (8 * sizeof(T) * zs)) & mask;
            w |= v << (8 * sizeof(T) * u);
        }
        out[d >> 2][d & 3] = w;
    }
    u32x4 *dst = reinterpret_cast<u32x4 *>(static_cast<uint8_t *>(j.grid) + static_cast<size_t>(b) * 64 * sizeof(T));
#pragma unroll
    for (int q = 0; q < P; q++) dst[q] = out[q];
}

} // namespace

int launch_jpeg_pieces_expand(const DevPiecesExpand *jobs, int njobs, uint32_t max_blocks, int coeff_bits,
                              hipStream_t s)
{
    if (njobs <= 0 || max_blocks == 0) return 0;
    const dim3 grid((max_blocks + 63) / 64, static_cast<uint32_t>(njobs));
    if (coeff_bits == 8)
        hipLaunchKernelGGL(jpeg_pieces_expand_kernel<int8_t>, grid, dim3(64), 0, s, jobs);
    else if (coeff_bits == 16)
        hipLaunchKernelGGL(jpeg_pieces_expand_kernel<int16_t>, grid, dim3(64), 0, s, jobs);
    else
        return -2;
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

} // namespace zpx
