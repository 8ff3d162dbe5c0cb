// gfx950 band-slab build: the paired-row PNG kernel's input layout
// (png_slab.cpp has the layout and the host builder) made on the device from
// the inflated stream that parseIdat hands readImagePass
// (src/png/decoder.zig:516-523).  So the host hands over the stream as
// inflate produced it and keeps no transposition work.
//
// A workgroup takes 16 rows of one band and walks their groups, 16 groups
// (128 chunks) a window, the next window's loads in flight during the
// current one's stores:
//   1. the band's 128 filter bytes -> the skew of every row (the kernel's
//      rule: row r minus the last row <= r that restarts the chain: a None /
//      Sub row, a row past the pass, or the band's first) and the band's
//      largest, hence its group count;
//   2. each row's window of the 16 groups, from its first chunk 8 g0 - skew
//      on, read as whole dwords with consecutive lanes on consecutive dwords
//      of one row (whole lines per instruction) into an LDS tile;
//   3. the 16-byte pieces in the slab's order (piece p = h NQ + q of rows
//      2 lane and 2 lane + 1's group windows interleaved two bytes at a
//      time -- 8 bytes of each row -- at 128 + ((2 g + h) NQ + q) KiB +
//      16 lane of the region), eight lanes on eight consecutive pieces, so
//      every store instruction writes whole 128-byte lines; bytes outside a
//      row are zeros.
// Streaming and HBM-bound: each stream byte is read once (plus the partial
// lines at a window's ends) and each slab byte written once.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "device_types.h"
#include "kernels.h"

namespace zpx {
namespace {

typedef uint32_t v4u __attribute__((ext_vector_type(4)));

constexpr int kRows = 16;   // rows per workgroup
constexpr int kGroups = 16; // groups (8 chunks each) per window
constexpr int kOOR = 0x7ffffff0;

template <int CB>
__global__ __launch_bounds__(256) void png_slab_kernel(const DevSlabBand *__restrict__ jobs)
{
    constexpr int NQ = CB / 2;                  // 16-byte pieces per row and group (8 CB / 16)
    constexpr int WIN = kGroups * 8 * CB;       // window bytes per row
    constexpr int NC = WIN / 16 + 1;            // 16-byte chunks loaded per row (+1: the window's misalignment)
    constexpr int RS = NC * 4 + 1;              // LDS dwords per row (odd: row starts spread over the banks)
    constexpr int NLD = (kRows * NC + 255) / 256; // chunk loads per thread per window
    constexpr int NPIECE = kGroups * 2 * NQ * 8;  // output pieces per window
    static_assert(NPIECE % 256 == 0, "whole output rounds");
    __shared__ uint32_t tile[kRows * RS];
    __shared__ uint8_t ft[128];
    __shared__ int32_t skew[128];
    __shared__ int32_t max_skew;
    const int tid = threadIdx.x;
    const int band = static_cast<int>(blockIdx.x) >> 3, R0 = (static_cast<int>(blockIdx.x) & 7) * kRows;
    typedef const __attribute__((address_space(4))) DevSlabBand *CJob;
    const auto &j = *(reinterpret_cast<CJob>(reinterpret_cast<uintptr_t>(jobs)) + band);
    const uint32_t rows = j.rows, rb = j.rb, rstride = rb + 1;
    const uintptr_t r0a = reinterpret_cast<uintptr_t>(j.rows0);
    const uint32_t delta = static_cast<uint32_t>(r0a & 15u);
    const auto src = __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void *>(r0a - delta), 0,
                                                       static_cast<int>(j.avail + delta), 0x00020000);
    // 1. filter bytes and skews (png_slab.cpp band_skews; png_pair_kernel)
    if (tid < 128) {
        const uint32_t o = static_cast<uint32_t>(tid) < rows ? static_cast<uint32_t>(tid) * rstride + delta : kOOR;
        ft[tid] = static_cast<uint8_t>(__builtin_amdgcn_raw_buffer_load_b8(src, o, 0, 0));
    }
    if (tid == 0) max_skew = 0;
    __syncthreads();
    if (tid < 128) {
        int l = tid;
        while (l > 0 && static_cast<uint32_t>(l) < rows && ft[l] >= 2) l--;
        skew[tid] = tid - l;
        if (static_cast<uint32_t>(tid) < rows) atomicMax(&max_skew, tid - l);
    }
    __syncthreads();
    const int ngroups = (static_cast<int>(j.nchunks) + max_skew + 7) / 8;
    if (R0 == 0 && tid < 32)
        reinterpret_cast<uint32_t *>(j.region)[tid] = reinterpret_cast<const uint32_t *>(ft)[tid];
    // a row's window of groups g0 .. g0 + 15 starts at its chunk 8 g0 - skew:
    // byte a of the band (from the descriptor base), loaded from a & ~15
    auto win_start = [&](int r, int g0) {
        return static_cast<uint32_t>(r) * rstride + 1u + static_cast<uint32_t>((8 * g0 - skew[r]) * CB) + delta;
    };
    // 2. the windows' 16-byte chunks, consecutive threads on consecutive
    // chunks of one row, into registers one window ahead
    v4u ld[NLD];
    auto load_window = [&](int g0) {
#pragma unroll
        for (int k = 0; k < NLD; k++) {
            const int idx = tid + 256 * k;
            const int rl = idx / NC, c = idx - rl * NC;
            const int r = R0 + rl;
            const bool in = idx < kRows * NC && static_cast<uint32_t>(r) < rows && 8 * g0 < ngroups * 8;
            const int o = in ? static_cast<int>((win_start(r, g0) & ~15u) + 16u * static_cast<uint32_t>(c)) : kOOR;
            ld[k] = __builtin_amdgcn_raw_buffer_load_b128(src, o, 0, 0);
        }
    };
    uint8_t *const groups = j.region + 128;
    load_window(0);
    for (int g0 = 0; g0 < ngroups; g0 += kGroups) {
        __syncthreads(); // the previous window's pieces are out of the tile
#pragma unroll
        for (int k = 0; k < NLD; k++) {
            const int idx = tid + 256 * k;
            if (idx < kRows * NC) {
                const int rl = idx / NC, c = idx - rl * NC;
                uint32_t *t = tile + rl * RS + 4 * c;
                t[0] = ld[k][0];
                t[1] = ld[k][1];
                t[2] = ld[k][2];
                t[3] = ld[k][3];
            }
        }
        __syncthreads();
        if (g0 + kGroups < ngroups) load_window(g0 + kGroups); // (in flight during the pieces below)
        // 3. the pieces, eight lanes per 128-byte line of the slab
#pragma unroll
        for (int k = 0; k < NPIECE / 256; k++) {
            const int idx = tid + 256 * k;
            const int l = idx & 7, rest = idx >> 3;
            const int q = rest % NQ, gh = rest / NQ, h = gh & 1, gl = gh >> 1;
            const int g = g0 + gl;
            const int pc = h * NQ + q; // the piece of the interleaved pair
            // 8 bytes of each of the two rows (2 dwords), zeros outside the row
            auto half = [&](int rl, uint32_t &d0, uint32_t &d1) __attribute__((always_inline)) {
                const int r = R0 + rl;
                d0 = d1 = 0;
                if (static_cast<uint32_t>(r) >= rows) return;
                const uint32_t local = (win_start(r, g0) & 15u) + static_cast<uint32_t>(8 * gl * CB + 8 * pc);
                const uint32_t *t = tile + rl * RS + (local >> 2);
                const uint32_t sh = local & 3u;
                const uint32_t w0 = t[0], w1 = t[1], w2 = t[2];
                d0 = __builtin_amdgcn_alignbyte(w1, w0, sh);
                d1 = __builtin_amdgcn_alignbyte(w2, w1, sh);
                const int p = (8 * g - skew[r]) * CB + 8 * pc; // the first byte in the row
                if (p < 0 || p + 8 > static_cast<int>(rb)) { // a row edge: zeros outside [0, rb)
                    uint32_t m0 = 0, m1 = 0;
#pragma unroll
                    for (int b = 0; b < 4; b++) {
                        m0 |= (p + b >= 0 && p + b < static_cast<int>(rb)) ? 0xffu << (8 * b) : 0u;
                        m1 |= (p + 4 + b >= 0 && p + 4 + b < static_cast<int>(rb)) ? 0xffu << (8 * b) : 0u;
                    }
                    d0 &= m0;
                    d1 &= m1;
                }
            };
            uint32_t a0, a1, b0, b1;
            half(2 * l, a0, a1);
            half(2 * l + 1, b0, b1);
            const v4u v = v4u{__builtin_amdgcn_perm(b0, a0, 0x05040100u), __builtin_amdgcn_perm(b0, a0, 0x07060302u),
                              __builtin_amdgcn_perm(b1, a1, 0x05040100u), __builtin_amdgcn_perm(b1, a1, 0x07060302u)};
            if (g < ngroups) {
                const int lane = (R0 >> 1) + l;
                *reinterpret_cast<v4u *>(groups + (static_cast<size_t>(2 * g + h) * NQ + q) * 1024 + lane * 16) = v;
            }
        }
    }
}

} // namespace

int launch_png_slab(int cb, const DevSlabBand *jobs, uint32_t njobs, uint32_t max_groups, hipStream_t s)
{
    if (njobs == 0) return 0;
    (void)max_groups; // (each workgroup walks its band's groups)
    const dim3 grid(njobs * 8);
    if (cb == 12) hipLaunchKernelGGL(png_slab_kernel<12>, grid, dim3(256), 0, s, jobs);
    else if (cb == 16) hipLaunchKernelGGL(png_slab_kernel<16>, grid, dim3(256), 0, s, jobs);
    else return -2;
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

} // namespace zpx
