// gfx950 kernel that expands the batch pipeline's sparse coefficient records
// (JpegSparse, jpeg_host.h) into the dense per-component grids the fused
// JPEG kernels read (a run-length upload instead of dense
// grids; a 4K q75 4:2:0 frame is ~13 MB of records against 25 MB of int8 or
// 50 MB of int16 grid).
//
// One lane per record, one 64-record group (a wave) per workgroup, in
// three steps:
//   1. the group's record bytes -- contiguous from its group offset -- come
//      into LDS with 16-byte loads, 1 KiB per instruction (the lane's byte
//      offset in them: an exclusive wave scan of the record sizes, 3 bytes
//      per entry);
//   2. the lane builds its block in LDS: zeros, then its entries;
//   3. it stores the block into the grid with 16-byte stores.
// The record index gives (MCU, scan slot, block within the MCU) exactly as
// processSos visits them (src/jpeg/decoder.zig:1300-1345), hence the block's
// grid position.  HBM-bound: the records are read and the grid written once,
// in whole 16-byte pieces (the previous version cleared each block with
// 16-byte stores, then wrote every entry with its own byte store: 44.6 us per
// 4K 4:2:0 int8 frame).
#include <hip/hip_runtime.h>

#include <cstdint>

#include "kernels.h"

namespace zpx {
namespace {

template <typename T>
__global__ __launch_bounds__(64) void jpeg_sparse_expand_kernel(DevJpegSparse a)
{
    constexpr int kRec = 64 * 64 * 3 + 16;            // a group's record bytes at most (+ alignment)
    constexpr int kBlk = 64 * int(sizeof(T)) + 16;    // a lane's block in LDS (+16: bank skew)
    __shared__ __attribute__((aligned(16))) uint8_t rec[kRec];
    __shared__ __attribute__((aligned(16))) uint8_t blks[64 * kBlk];
    const uint32_t lane = threadIdx.x;
    const uint64_t r = uint64_t(blockIdx.x) * 64 + lane;
    const bool live = r < a.nrec;
    const uint32_t n = live ? a.counts[r] : 0;
    uint32_t inc = 3 * n; // inclusive wave scan of the record sizes
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t t = __shfl_up(inc, off);
        if (lane >= uint32_t(off)) inc += t;
    }
    // 1. the group's records (the device copy has 16 readable bytes past the last)
    const uint8_t *g0 = a.data + a.groups[blockIdx.x];
    const uint8_t *b16 = reinterpret_cast<const uint8_t *>(reinterpret_cast<uintptr_t>(g0) & ~uintptr_t(15));
    const uint32_t lead = static_cast<uint32_t>(g0 - b16);
    const uint32_t span = lead + static_cast<uint32_t>(__shfl(inc, 63));
    for (uint32_t o = lane * 16; o < span; o += 1024)
        *reinterpret_cast<uint4 *>(rec + o) = *reinterpret_cast<const uint4 *>(b16 + o);
    // 2. the lane's block: zeros, then its entries
    uint8_t *blk = blks + lane * kBlk;
#pragma unroll
    for (int i = 0; i < int(64 * sizeof(T) / 16); i++) reinterpret_cast<uint4 *>(blk)[i] = make_uint4(0, 0, 0, 0);
    __syncthreads();
    const uint8_t *d = rec + lead + (inc - 3 * n);
    for (uint32_t i = 0; i < n; i++) {
        const int16_t v = static_cast<int16_t>(d[n + 2 * i] | uint32_t(d[n + 2 * i + 1]) << 8);
        reinterpret_cast<T *>(blk)[d[i]] = static_cast<T>(v);
    }
    if (!live) return;
    // 3. the block's grid position, and the block
    const uint64_t mcu = r / uint32_t(a.bpm);
    int t = static_cast<int>(r - mcu * uint32_t(a.bpm));
    int k = 0;
    while (k + 1 < a.ns && t >= a.h[k] * a.v[k]) {
        t -= a.h[k] * a.v[k];
        k++;
    }
    const uint32_t my = static_cast<uint32_t>(mcu / uint32_t(a.mxx)), mx = static_cast<uint32_t>(mcu % uint32_t(a.mxx));
    const uint32_t bx = a.h[k] * mx + t % a.h[k], by = a.v[k] * my + t / a.h[k];
    uint4 *dst = reinterpret_cast<uint4 *>(static_cast<T *>(a.grid[k]) + (uint64_t(by) * uint32_t(a.gw[k]) + bx) * 64);
#pragma unroll
    for (int i = 0; i < int(64 * sizeof(T) / 16); i++) dst[i] = reinterpret_cast<const uint4 *>(blk)[i];
}

} // namespace

int launch_jpeg_sparse_expand(const DevJpegSparse &a, int coeff_bits, hipStream_t s)
{
    if (a.nrec == 0) return 0;
    const uint32_t groups = static_cast<uint32_t>((a.nrec + 63) / 64);
    if (coeff_bits == 8)
        hipLaunchKernelGGL(jpeg_sparse_expand_kernel<int8_t>, dim3(groups), dim3(64), 0, s, a);
    else if (coeff_bits == 16)
        hipLaunchKernelGGL(jpeg_sparse_expand_kernel<int16_t>, dim3(groups), dim3(64), 0, s, a);
    else
        return -2;
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

} // namespace zpx
