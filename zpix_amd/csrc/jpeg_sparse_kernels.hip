// gfx950 kernel that expands the batch pipeline's sparse coefficient records
// (JpegSparse, jpeg_host.h) into the dense per-component grids the fused
// JPEG kernels read (a run-length upload instead of dense
// grids; a 4K q75 4:2:0 frame is ~13 MB of records against 25 MB of int8 or
// 50 MB of int16 grid).
//
// One lane per record, 64 records per wave: the lane's byte offset is the
// group offset of its 64 plus an exclusive wave scan of the record sizes
// (3 bytes per entry).  The record index gives (MCU, scan slot, block within
// the MCU) exactly as processSos visits them (src/jpeg/decoder.zig:1300-1345),
// hence the block's grid position.  The lane clears its block with 16-byte
// stores and then writes its entries (same-lane stores to one address stay in
// program order).  HBM-bound: the grid is written once, the records read once.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "kernels.h"

namespace zpx {
namespace {

template <typename T>
__global__ __launch_bounds__(256) void jpeg_sparse_expand_kernel(DevJpegSparse a)
{
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t r = (uint64_t(blockIdx.x) * 4 + (threadIdx.x >> 6)) * 64 + lane;
    const bool live = r < a.nrec;
    const uint32_t n = live ? a.counts[r] : 0;
    uint32_t inc = 3 * n; // inclusive wave scan of the record sizes
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t t = __shfl_up(inc, off);
        if (lane >= uint32_t(off)) inc += t;
    }
    if (!live) return;
    const uint8_t *d = a.data + a.groups[r / 64] + (inc - 3 * n);
    const uint64_t mcu = r / uint32_t(a.bpm);
    int t = static_cast<int>(r - mcu * uint32_t(a.bpm));
    int k = 0;
    while (k + 1 < a.ns && t >= a.h[k] * a.v[k]) {
        t -= a.h[k] * a.v[k];
        k++;
    }
    const uint32_t my = static_cast<uint32_t>(mcu / uint32_t(a.mxx)), mx = static_cast<uint32_t>(mcu % uint32_t(a.mxx));
    const uint32_t bx = a.h[k] * mx + t % a.h[k], by = a.v[k] * my + t / a.h[k];
    T *blk = static_cast<T *>(a.grid[k]) + (uint64_t(by) * uint32_t(a.gw[k]) + bx) * 64;
    uint4 *z = reinterpret_cast<uint4 *>(blk);
#pragma unroll
    for (int i = 0; i < int(64 * sizeof(T) / 16); i++) z[i] = make_uint4(0, 0, 0, 0);
    for (uint32_t i = 0; i < n; i++) {
        const int16_t v = static_cast<int16_t>(d[n + 2 * i] | uint32_t(d[n + 2 * i + 1]) << 8);
        blk[d[i]] = static_cast<T>(v);
    }
}

} // namespace

int launch_jpeg_sparse_expand(const DevJpegSparse &a, int coeff_bits, hipStream_t s)
{
    if (a.nrec == 0) return 0;
    const uint32_t blocks = static_cast<uint32_t>((a.nrec + 255) / 256);
    if (coeff_bits == 8)
        hipLaunchKernelGGL(jpeg_sparse_expand_kernel<int8_t>, dim3(blocks), dim3(256), 0, s, a);
    else if (coeff_bits == 16)
        hipLaunchKernelGGL(jpeg_sparse_expand_kernel<int16_t>, dim3(blocks), dim3(256), 0, s, a);
    else
        return -2;
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

} // namespace zpx
