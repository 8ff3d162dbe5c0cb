// gfx950 kernels of the JPEG pixel path:
//   - jpeg_planar_kernel: dequant + 8x8 integer IDCT + level shift/clamp into
//     the Y/Cb/Cr/K planes (reconstructBlock, src/jpeg/decoder.zig:1553-1634);
//   - jpeg_rgba_kernel: the same fused with nearest chroma upsample and
//     YCbCr->RGB (Image.rgbaPixels over a YCbCrImage: image.zig:103-130,
//     YCbCrAt :614-630, Color.toRGBA .ycbcr color.zig:90-113), one MCU strip
//     per workgroup, staged through LDS; the planes never reach HBM.
// Integer arithmetic is wrap-around i32 (built with -fwrapv), bit-identical to
// the reference's IDCT (src/jpeg/idct.zig:77-201).  MFMA is not used: no
// stage is a dense contraction.  The kernels are HBM-bound streaming passes.
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <type_traits>

#include <cstdint>

#include "device_types.h"
#include "jpeg_idct.h"
#include "kernels.h"
#include "options.h"

namespace zpx {
namespace {

constexpr int kThreads = 256;
constexpr int kStoreAux = 2; // the aligned-row RGBA stores: non-temporal (cached: 1.643 against 1.622 ms)
constexpr int kBlkStride = 72; // dwords per 8x8 block in LDS (64 + 8 pad: conflict-free column reads)

// Load one 8-coefficient row of a block (natural order) and dequantize it.
template <typename CoefT>
__device__ __forceinline__ void load_row(const CoefT *__restrict__ p, const int32_t *__restrict__ q,
                                         int32_t s[8])
{
    if constexpr (sizeof(CoefT) == 1) {
        const uint2 v = *reinterpret_cast<const uint2 *>(p);
        const uint32_t w[2] = {v.x, v.y};
#pragma unroll
        for (int i = 0; i < 8; i++) s[i] = static_cast<int32_t>(w[i >> 2] << (24 - 8 * (i & 3))) >> 24;
    } else if constexpr (sizeof(CoefT) == 2) {
        const uint4 v = *reinterpret_cast<const uint4 *>(p);
        const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int i = 0; i < 4; i++) {
            s[2 * i] = static_cast<int32_t>(static_cast<int16_t>(w[i] & 0xffff));
            s[2 * i + 1] = static_cast<int32_t>(w[i]) >> 16;
        }
    } else {
        const int4 a = *reinterpret_cast<const int4 *>(p);
        const int4 b = *reinterpret_cast<const int4 *>(p + 4);
        s[0] = a.x; s[1] = a.y; s[2] = a.z; s[3] = a.w;
        s[4] = b.x; s[5] = b.y; s[6] = b.z; s[7] = b.w;
    }
    // coefficients fit in 16 bits for the int8/int16 transports and q in 17
    // bits, so the 24-bit multiply is exact there
#pragma unroll
    for (int i = 0; i < 8; i++)
        s[i] = (sizeof(CoefT) <= 2) ? __mul24(s[i], q[i]) : s[i] * q[i];
}

__device__ __forceinline__ bool block_in_rule(int rule, int bx, int by, int hh, int vv, int W, int H)
{
    switch (rule) {
    case ZPX_BLOCKS_ALL: return true;
    case ZPX_BLOCKS_PROGRESSIVE: return bx * hh < W && by * vv < H; // decoder.zig:1649-1651
    case ZPX_BLOCKS_SCAN: return bx * 8 < W && by * 8 < H;          // decoder.zig:1334
    default: return false;
    }
}

// ---------------------------------------------------------------------------
// Planar reconstruct: each wave owns 8 horizontally adjacent blocks of one
// block row; lane = (block, row) for the row pass, (block, column) for the
// column pass, exchanging through LDS.  Grid: x = 32-block segments of a row,
// y = block row, z = frame*4 + component.
// ---------------------------------------------------------------------------
template <typename CoefT, bool NARROW>
__global__ __launch_bounds__(kThreads) void jpeg_planar_kernel(const DevJpegFrame *__restrict__ frames)
{
    __shared__ int32_t qs[64];
    __shared__ int32_t buf[4 * 8 * kBlkStride];
    const int f = blockIdx.z >> 2, comp = blockIdx.z & 3;
    const DevJpegFrame &fr = frames[f];
    if (comp >= fr.n_comp) return;
    const CoefT *grid = static_cast<const CoefT *>(fr.coeffs[comp]);
    const int rule = fr.rule[comp];
    if (grid == nullptr || rule == ZPX_BLOCKS_NONE) return;
    const int gw = fr.mxx * fr.h[comp], gh = fr.myy * fr.v[comp];
    const int by = blockIdx.y;
    if (by >= gh) return;
    const int bx0 = blockIdx.x * 32;
    if (bx0 >= gw) return;
    const int hh = 8 * (fr.h[0] / fr.h[comp]), vv = 8 * (fr.v[0] / fr.v[comp]);

    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    if (tid < 64) qs[tid] = fr.qt[comp][tid];
    __syncthreads();

    const int blk = lane >> 3, r = lane & 7; // row pass: block, row
    const int bx = bx0 + wave * 8 + blk;
    const bool live = bx < gw && block_in_rule(rule, bx, by, hh, vv, fr.width, fr.height);
    int32_t *wb = buf + wave * 8 * kBlkStride;
    int32_t s[8];
    if (live) {
        load_row<CoefT>(grid + (static_cast<size_t>(by) * gw + bx) * 64 + r * 8, qs + r * 8, s);
        idct_row<NARROW>(s);
#pragma unroll
        for (int i = 0; i < 8; i++) wb[blk * kBlkStride + r * 8 + i] = s[i];
    }
    __syncthreads();
    const int c = lane & 7; // column pass: block, column
    if (live) {
#pragma unroll
        for (int i = 0; i < 8; i++) s[i] = wb[blk * kBlkStride + i * 8 + c];
        idct_col_clamp<NARROW>(s);
        uint8_t *dst = fr.planes[comp] + 8 * (static_cast<size_t>(by) * fr.strides[comp] + bx) + c;
#pragma unroll
        for (int i = 0; i < 8; i++) dst[i * fr.strides[comp]] = static_cast<uint8_t>(s[i]);
    }
}

// ---------------------------------------------------------------------------
// Fused reconstruct + Image.rgbaPixels.  A workgroup owns a horizontal strip
// of T MCUs of one MCU row and walks strips persistently (grid-stride), with
// the next strip's coefficient rows prefetched into registers while the
// current one is in its LDS phases:
//   P1: lane = (block, row): dequant + row IDCT -> LDS row buffer;
//   P2: chroma columns -> clamped samples in an LDS chroma tile;
//   P3a: luma columns -> clamped Y kept in registers;
//   P3b: nearest chroma + YCbCr->RGB -> RGBA dwords in an LDS tile that
//        reuses the row buffer;
//   P3c: 16-byte stores, a wave writes 1 KiB of one output row per instruction.
// ---------------------------------------------------------------------------

// the workgroup's 256 threads share a strip of about 96 blocks (3
// coefficient rows per lane; 48 / 64 / 128-block strips ran 17-60 % slower)
constexpr int kGroup = kThreads;
constexpr int kStripBlocks = 96;
constexpr int strip_mcus(int blocks_per_mcu)
{
    return blocks_per_mcu >= kStripBlocks ? 1 : kStripBlocks / blocks_per_mcu;
}

// Barrier among the threads of one strip group.  A one-wave group needs no
// s_barrier: LDS operations of a wave complete in order, so a compiler fence
// plus lgkmcnt(0) orders the lanes' LDS writes before the reads.
template <int G>
__device__ __forceinline__ void group_sync()
{
    if constexpr (G == kThreads) {
        __syncthreads();
    } else {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_wave_barrier();
    }
}


// One coefficient row, raw (not yet dequantized): 8 B (int8), 16 B (int16)
// or 32 B (int32).
template <typename CoefT>
struct RowRegs {
    using A = typename std::conditional<sizeof(CoefT) == 1, u32x2, u32x4>::type;
    A a;
    u32x4 b; // int32 coefficients only
};

template <typename CoefT>
__device__ __forceinline__ void load_row_raw(const CoefT *p, RowRegs<CoefT> &r)
{
    using A = typename RowRegs<CoefT>::A;
    const ZPX_GLOBAL A *g = (const ZPX_GLOBAL A *)p;
    // non-temporal: every coefficient is read once (cached loads: 1.646 against 1.622 ms)
    r.a = __builtin_nontemporal_load(g);
    if constexpr (sizeof(CoefT) == 4) r.b = __builtin_nontemporal_load((const ZPX_GLOBAL u32x4 *)p + 1);
}

template <typename CoefT>
__device__ __forceinline__ void unpack_dequant(const RowRegs<CoefT> &r, const int32_t *__restrict__ q, int32_t s[8])
{
    if constexpr (sizeof(CoefT) == 1) {
#pragma unroll
        for (int i = 0; i < 8; i++) s[i] = static_cast<int32_t>(r.a[i >> 2] << (24 - 8 * (i & 3))) >> 24;
        // |coef| < 2^7 and q < 2^17: the 24-bit multiply is exact
#pragma unroll
        for (int i = 0; i < 8; i++) s[i] = __mul24(s[i], q[i]);
    } else if constexpr (sizeof(CoefT) == 2) {
#pragma unroll
        for (int i = 0; i < 4; i++) {
            const uint32_t w = r.a[i];
            s[2 * i] = static_cast<int32_t>(static_cast<int16_t>(w & 0xffff));
            s[2 * i + 1] = static_cast<int32_t>(w) >> 16;
        }
        // |coef| < 2^15 and q < 2^17: the 24-bit multiply is exact
#pragma unroll
        for (int i = 0; i < 8; i++) s[i] = __mul24(s[i], q[i]);
    } else {
#pragma unroll
        for (int i = 0; i < 4; i++) {
            s[i] = static_cast<int32_t>(r.a[i]);
            s[4 + i] = static_cast<int32_t>(r.b[i]);
        }
#pragma unroll
        for (int i = 0; i < 8; i++) s[i] = s[i] * q[i];
    }
}

// 5 waves per EU (87 VGPRs): 5 workgroups, 20 waves, per CU (4: +5 %)
template <typename CoefT, bool NARROW, int H0, int V0, int HC, int VC, int COLOR>
__global__ __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(5))) void jpeg_rgba_kernel(const DevJpegFrame *__restrict__ frames, int strips_x,
                                                             int strips_per_frame, int total_strips)
{
    constexpr bool kGray = COLOR == ZPX_JPEG_COLOR_GRAY;
    constexpr int kYB = H0 * V0;                      // luma blocks per MCU
    constexpr int kCB = kGray ? 0 : HC * VC;          // blocks per chroma component per MCU
    constexpr int G = kGroup;                         // threads that share a strip
    constexpr int NG = kThreads / G;                  // strip groups per workgroup
    constexpr int T = strip_mcus(kYB + 2 * kCB);      // MCUs per strip
    constexpr int NY = T * kYB, NC = T * kCB, NB = NY + 2 * NC;
    constexpr int YW = T * H0;                        // luma blocks across the strip
    constexpr int CW = T * HC;                        // chroma blocks across the strip
    constexpr int CPX = kGray ? 1 : CW * 8;           // chroma tile width (samples)
    constexpr int CROWS = kGray ? 1 : VC * 8;
    constexpr int RX = kGray ? 1 : H0 / HC, RY = kGray ? 1 : V0 / VC; // upsample ratios
    constexpr int PXW = YW * 8;                       // strip width in pixels
    constexpr int PXH = V0 * 8;                       // strip height in pixels
    constexpr int ROW_IT = (NB * 8 + G - 1) / G;
    constexpr int YCOL_IT = (NY * 8 + G - 1) / G;
    constexpr int CCOL_IT = (2 * NC * 8 + G - 1) / G;
    constexpr int CHUNKS = PXH * PXW / 4;             // 16-byte output chunks per strip
    constexpr int OUT_IT = (CHUNKS + G - 1) / G;
    static_assert(PXH * PXW <= NB * kBlkStride, "RGBA tile must fit in the row buffer");

    __shared__ int32_t qs_all[NG][3][64];
    __shared__ __attribute__((aligned(16))) int32_t buf_all[NG][NB * kBlkStride]; // row pass, then RGBA tile
    // chroma samples are clamped to 0..255: bytes keep the workgroup's LDS
    // at ~31 KiB, so 5 workgroups (20 waves) fit a CU instead of 4
    __shared__ uint8_t ctile_all[NG][kGray ? 1 : 2][CROWS * CPX];

    const int tid = threadIdx.x % G, group = threadIdx.x / G;
    auto (&qs) = qs_all[group];
    int32_t *const buf = buf_all[group];
    auto (&ctile) = ctile_all[group];
    constexpr int ncomp = kGray ? 1 : 3;

    // strip -> (frame, MCU row, first MCU column)
    auto strip_of = [&](int st, int &f, int &my, int &mx0) {
        f = st / strips_per_frame;
        const int r = st - f * strips_per_frame;
        my = r / strips_x;
        mx0 = (r - my * strips_x) * T;
    };
    // per-strip uniform view of the frame descriptor: the component grids are
    // read into scalars once, so that row addresses are a per-lane select of
    // uniform values (a lane-indexed fr.coeffs[comp] compiles to a vector load
    // plus a full vmcnt(0) wait in front of every prefetch)
    struct StripSrc {
        const CoefT *g[3];
        int gwy, gwc, myy;
    };
    auto src_of = [&](const DevJpegFrame &fr) {
        StripSrc s;
        s.g[0] = static_cast<const CoefT *>(fr.coeffs[0]);
        s.g[1] = static_cast<const CoefT *>(fr.coeffs[1]);
        s.g[2] = static_cast<const CoefT *>(fr.coeffs[2]);
        s.gwy = fr.mxx * H0;
        s.gwc = fr.mxx * HC;
        s.myy = fr.myy;
        return s;
    };
    // coefficient row address of row-task k of a strip (nullptr: nothing to load)
    auto row_ptr = [&](const StripSrc &ss, int my, int mx0, int k) -> const CoefT * {
        const int blk = k >> 3, r = k & 7;
        int bx, by, gw;
        const CoefT *grid;
        if (blk < NY) {
            grid = ss.g[0];
            bx = mx0 * H0 + blk % YW;
            by = my * V0 + blk / YW;
            gw = ss.gwy;
        } else {
            const int c = blk - NY;
            const int kk = NC > 0 ? c % NC : 0;
            grid = c < NC ? ss.g[1] : ss.g[2];
            bx = mx0 * HC + kk % CW;
            by = my * VC + kk / CW;
            gw = ss.gwc;
        }
        if (grid == nullptr || bx >= gw || blk >= NB || my >= ss.myy) return nullptr; // ragged batch: skip
        return grid + (static_cast<size_t>(by) * gw + bx) * 64 + r * 8;
    };

    // Rows without a block are loaded from a valid dummy address and zeroed in
    // P1: every prefetch and every store is issued unconditionally, so the
    // compiler's vmcnt before P1 counts only this strip's stores in flight
    // (a branchy load/store phase makes it wait for vmcnt(0), i.e. for the
    // previous strip's stores to complete).
    const CoefT *const dummy = reinterpret_cast<const CoefT *>(frames);
    RowRegs<CoefT> pre[ROW_IT];
    const int gstride = static_cast<int>(gridDim.x) * NG;
    int st = blockIdx.x * NG + group;
    int f = 0, my = 0, mx0 = 0;
    if (st < total_strips) {
        strip_of(st, f, my, mx0);
        const StripSrc ss0 = src_of(frames[f]);
#pragma unroll
        for (int it = 0; it < ROW_IT; it++) {
            const CoefT *p = row_ptr(ss0, my, mx0, it * G + tid);
            load_row_raw<CoefT>(p ? p : dummy, pre[it]);
        }
    }
    int qframe = -1;
    for (; st < total_strips; st += gstride) {
        const DevJpegFrame &fr = frames[f];
        const StripSrc ss = src_of(fr);
        if (f != qframe) { // quant tables of this frame (natural order)
            for (int i = tid; i < ncomp * 64; i += G) qs[i >> 6][i & 63] = fr.qt[i >> 6][i & 63];
            qframe = f;
            group_sync<G>();
        }
        // ---- P1: dequant + row IDCT of the prefetched rows
#pragma unroll
        for (int it = 0; it < ROW_IT; it++) {
            const int k = it * G + tid;
            if (k >= NB * 8) break;
            const int blk = k >> 3, r = k & 7;
            const int comp = blk < NY ? 0 : (blk < NY + NC ? 1 : 2);
            int32_t s[8] = {0, 0, 0, 0, 0, 0, 0, 0};
            if (row_ptr(ss, my, mx0, k) != nullptr) {
                unpack_dequant<CoefT>(pre[it], qs[comp] + r * 8, s);
                idct_row<NARROW>(s);
            }
            // two 16-byte LDS writes; rows 4..7 write their halves in swapped
            // order so the 8 lanes of a write group hit distinct banks
            int32_t *d = buf + blk * kBlkStride + r * 8;
            const bool sw = (r & 4) != 0;
            i32x4 lo = {s[0], s[1], s[2], s[3]}, hi = {s[4], s[5], s[6], s[7]};
            *reinterpret_cast<i32x4 *>(d + (sw ? 4 : 0)) = sw ? hi : lo;
            *reinterpret_cast<i32x4 *>(d + (sw ? 0 : 4)) = sw ? lo : hi;
        }
        // ---- prefetch the next strip's rows (consumed next iteration)
        // (past the end: the last strip again, loaded and never used)
        const int st_next = min(st + gstride, total_strips - 1);
        int fn, myn, mxn;
        {
            strip_of(st_next, fn, myn, mxn);
            const StripSrc ssn = src_of(frames[fn]);
#pragma unroll
            for (int it = 0; it < ROW_IT; it++) {
                const CoefT *p = row_ptr(ssn, myn, mxn, it * G + tid);
                load_row_raw<CoefT>(p ? p : dummy, pre[it]);
            }
        }
        group_sync<G>();

        // ---- P2: chroma columns -> LDS tile
        if constexpr (!kGray) {
            const bool cb_present = fr.coeffs[1] != nullptr, cr_present = fr.coeffs[2] != nullptr;
#pragma unroll
            for (int it = 0; it < CCOL_IT; it++) {
                const int task = it * G + tid;
                if (task >= 2 * NC * 8) break;
                const int k = task >> 3, c = task & 7;
                const int comp = k < NC ? 1 : 2;
                const int kk = k < NC ? k : k - NC;
                const int blk = NY + k;
                int32_t s[8];
#pragma unroll
                for (int i = 0; i < 8; i++) s[i] = buf[blk * kBlkStride + i * 8 + c];
                idct_col_clamp<NARROW>(s);
                const bool present = comp == 1 ? cb_present : cr_present; // never scanned: samples 0
                uint8_t *t = ctile[comp - 1] + ((kk / CW) * 8) * CPX + (kk % CW) * 8 + c;
#pragma unroll
                for (int i = 0; i < 8; i++) t[i * CPX] = static_cast<uint8_t>(present ? s[i] : 0);
            }
            group_sync<G>();
        }

        // ---- P3a: luma columns (a never-scanned luma plane stays 0)
        int32_t yv[YCOL_IT][8];
        const int32_t y_mask = fr.coeffs[0] != nullptr ? -1 : 0;
#pragma unroll
        for (int it = 0; it < YCOL_IT; it++) {
            const int task = it * G + tid;
            if (task < NY * 8) {
                const int blk = task >> 3, c = task & 7;
#pragma unroll
                for (int i = 0; i < 8; i++) yv[it][i] = buf[blk * kBlkStride + i * 8 + c];
                idct_col_clamp<NARROW>(yv[it]);
#pragma unroll
                for (int i = 0; i < 8; i++) yv[it][i] &= y_mask;
            }
        }
        group_sync<G>(); // row buffer is free: reuse it as the RGBA tile

        // ---- P3b: colour -> RGBA tile [PXH][PXW]
        uint32_t *otile = reinterpret_cast<uint32_t *>(buf);
#pragma unroll
        for (int it = 0; it < YCOL_IT; it++) {
            const int task = it * G + tid;
            if (task >= NY * 8) break;
            const int blk = task >> 3, c = task & 7;
            const int yrow = blk / YW, ycol = blk % YW;
            const int px = ycol * 8 + c;
            uint32_t *o = otile + (yrow * 8) * PXW + px;
#pragma unroll
            for (int i0 = 0; i0 < 8; i0 += RY) {
                int32_t cb = 0, cr = 0;
                if constexpr (!kGray) {
                    const int ci = ((yrow * 8 + i0) / RY) * CPX + px / RX;
                    cb = ctile[0][ci];
                    cr = ctile[1][ci];
                }
                // colour.zig:95-106 chroma terms, once per chroma sample (RY rows)
                const int32_t cb1 = cb - 128, cr1 = cr - 128;
                const int32_t t_r = __mul24(91881, cr1);
                const int32_t t_g = -(__mul24(22554, cb1) + __mul24(46802, cr1));
                const int32_t t_b = __mul24(116130, cb1);
#pragma unroll
                for (int j = 0; j < RY; j++) {
                    const int i = i0 + j;
                    const int32_t Yv = yv[it][i];
                    uint32_t pix;
                    if constexpr (kGray) {
                        pix = static_cast<uint32_t>(Yv) * 0x010101u | 0xff000000u;
                    } else if constexpr (COLOR == ZPX_JPEG_COLOR_RGB) {
                        pix = static_cast<uint32_t>(Yv) | static_cast<uint32_t>(cb) << 8 |
                              static_cast<uint32_t>(cr) << 16 | 0xff000000u;
                    } else {
                        // color.zig:95-106; 8-bit result of (v>>8 or clamp)>>8 == clamp(v, 0, 2^24-1)>>16
                        // (clamp before the shift: see ycc_rgba8 in color_kernels.hip).
                        // Per pixel: 3 v_mad_i32_i24, 3 v_med3_i32, and two v_perm_b32
                        // that take byte 2 of each clamped channel (= its >>16).
                        const int32_t r = __mul24(Yv, 0x10101) + t_r;
                        const int32_t g = __mul24(Yv, 0x10101) + t_g;
                        const int32_t b = __mul24(Yv, 0x10101) + t_b;
                        const uint32_t rc = static_cast<uint32_t>(min(max(r, 0), 0xffffff));
                        const uint32_t gc = static_cast<uint32_t>(min(max(g, 0), 0xffffff));
                        const uint32_t bc = static_cast<uint32_t>(min(max(b, 0), 0xffffff));
                        // {R, G, 0x00, 0xff}: bytes rc.2, gc.2, zero, 0xff
                        const uint32_t rg = __builtin_amdgcn_perm(gc, rc, 0x0d0c0602u);
                        // {R, G, B, 0xff}
                        pix = __builtin_amdgcn_perm(bc, rg, 0x03060100u);
                    }
                    o[i * PXW] = pix;
                }
            }
        }
        group_sync<G>();

        // ---- P3c: stores of the tile through a per-strip buffer descriptor.
        // Lanes outside the image get an offset past num_records and the
        // hardware drops their stores, so no store sits behind a branch.
        // The host guarantees PXH * rgba_stride < 2^31.
        const int W = fr.width, H = fr.height;
        const int X0 = mx0 * H0 * 8, Y0 = my * V0 * 8;
        const uint32_t ostride = static_cast<uint32_t>(fr.rgba_stride);
        uint8_t *const out = fr.rgba + static_cast<size_t>(Y0) * fr.rgba_stride;
        const int rows_here = max(0, min(PXH, H - Y0)); // ragged batch: a smaller frame ends above
        const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(out, 0, rows_here * static_cast<int>(ostride), 0x00020000);
        constexpr uint32_t kDrop = 0x80000000u;
        // 16-byte stores when every chunk of a row is whole and aligned
        const bool vec_ok = (ostride & 15) == 0 && (reinterpret_cast<uintptr_t>(out) & 15) == 0 && (W & 3) == 0;
        if (vec_ok) {
#pragma unroll
            for (int it = 0; it < OUT_IT; it++) {
                const int q = min(it * G + tid, CHUNKS - 1); // duplicates store the same bytes
                const int row = q / (PXW / 4), cx = (q % (PXW / 4)) * 4;
                const u32x4 v = *reinterpret_cast<const u32x4 *>(otile + row * PXW + cx);
                const uint32_t off = X0 + cx < W ? row * ostride + (X0 + cx) * 4 : kDrop;
                __builtin_amdgcn_raw_buffer_store_b128(v, rsrc, off, 0, kStoreAux);
            }
        } else {
            // rows only dword aligned (e.g. 4094-wide frames at stride 4W) or
            // a width % 4 != 0: whole chunks still leave as one 16-byte store
            // (dword-aligned; the memory system splits it), and only a row's
            // last, partial chunk as dwords.  Cached, not non-temporal: a
            // non-temporal store that covers part of a 16-byte piece goes to
            // HBM on its own (4-byte nt stores: 5.95 ms for 64 4094x4096
            // frames)
#pragma unroll
            for (int it = 0; it < OUT_IT; it++) {
                const int q = min(it * G + tid, CHUNKS - 1);
                const int row = q / (PXW / 4), cx = (q % (PXW / 4)) * 4;
                const u32x4 v = *reinterpret_cast<const u32x4 *>(otile + row * PXW + cx);
                const int x = X0 + cx;
                const uint32_t o = row * ostride + static_cast<uint32_t>(x) * 4;
                __builtin_amdgcn_raw_buffer_store_b128(v, rsrc, x + 3 < W ? o : kDrop, 0, 0);
                const bool part = x < W && x + 3 >= W; // 1..3 pixels of the chunk inside the row
#pragma unroll
                for (int e = 0; e < 3; e++)
                    __builtin_amdgcn_raw_buffer_store_b32(v[e], rsrc, part && x + e < W ? o + 4 * e : kDrop, 0, 0);
            }
        }
        group_sync<G>(); // tile / row buffer reused by the next strip
        f = fn;
        my = myn;
        mx0 = mxn;
    }
}

} // namespace

// ---------------------------------------------------------------------------
// launchers
// ---------------------------------------------------------------------------
int launch_jpeg_planar(const DevJpegFrame *d_frames, int n_frames, const JpegPlaneGeom &geom, int coeff_bits,
                       bool narrow, bool pieces, hipStream_t stream)
{
    // the block-per-lane kernel (jpeg_block_kernels.hip) takes the narrow
    // int8 / int16 frames; the test switch "jpeg_strip" forces this one
    if (pieces) return launch_jpeg_plane_block(d_frames, n_frames, geom, coeff_bits, narrow, true, stream);
    if (opt(Opt::JpegStrip) == 0) {
        const int rc = launch_jpeg_plane_block(d_frames, n_frames, geom, coeff_bits, narrow, false, stream);
        if (rc != -2) return rc;
    }
    int max_gw = 0, max_gh = 0;
    for (int c = 0; c < geom.ncomp; c++) {
        max_gw = max(max_gw, geom.max_mxx * geom.h[c]);
        max_gh = max(max_gh, geom.max_myy * geom.v[c]);
    }
    if (max_gw <= 0 || max_gh <= 0 || n_frames <= 0) return 0;
    dim3 grid((max_gw + 31) / 32, max_gh, n_frames * 4);
    if (coeff_bits == 8) {
        if (narrow) hipLaunchKernelGGL((jpeg_planar_kernel<int8_t, true>), grid, dim3(kThreads), 0, stream, d_frames);
        else hipLaunchKernelGGL((jpeg_planar_kernel<int8_t, false>), grid, dim3(kThreads), 0, stream, d_frames);
    } else if (coeff_bits == 32) {
        if (narrow) hipLaunchKernelGGL((jpeg_planar_kernel<int32_t, true>), grid, dim3(kThreads), 0, stream, d_frames);
        else hipLaunchKernelGGL((jpeg_planar_kernel<int32_t, false>), grid, dim3(kThreads), 0, stream, d_frames);
    } else {
        if (narrow) hipLaunchKernelGGL((jpeg_planar_kernel<int16_t, true>), grid, dim3(kThreads), 0, stream, d_frames);
        else hipLaunchKernelGGL((jpeg_planar_kernel<int16_t, false>), grid, dim3(kThreads), 0, stream, d_frames);
    }
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int device_cu_count()
{
    static const int n = [] {
        int dev = 0, cus = 256;
        if (hipGetDevice(&dev) == hipSuccess)
            (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
        return cus > 0 ? cus : 256;
    }();
    return n;
}

namespace {
// Resident workgroups on the device for one kernel instance: the occupancy
// API (registers + LDS).
template <typename K>
int persistent_workgroups(K kernel)
{
    int per_cu = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, kThreads, 0) != hipSuccess || per_cu < 1)
        per_cu = 4;
    return device_cu_count() * per_cu;
}

template <typename CoefT, bool NARROW, int H0, int V0, int HC, int VC, int COLOR>
void launch_rgba_t(const DevJpegFrame *d_frames, int n_frames, int max_mxx, int max_myy, hipStream_t stream)
{
    constexpr bool kGray = COLOR == ZPX_JPEG_COLOR_GRAY;
    constexpr int T = strip_mcus(H0 * V0 + 2 * (kGray ? 0 : HC * VC));
    constexpr int NG = kThreads / kGroup;
    const int strips_x = (max_mxx + T - 1) / T;
    const int per_frame = strips_x * max_myy;
    const int total = per_frame * n_frames;
    const int groups_needed = (total + NG - 1) / NG;
    auto kernel = jpeg_rgba_kernel<CoefT, NARROW, H0, V0, HC, VC, COLOR>;
    static const int resident = persistent_workgroups(kernel); // (one per instance: this function is)
    const int grid = groups_needed < resident ? groups_needed : resident;
    hipLaunchKernelGGL(kernel, dim3(grid), dim3(kThreads), 0, stream, d_frames, strips_x, per_frame, total);
}

template <typename CoefT, bool NARROW, int COLOR>
int dispatch_geom(int key, const DevJpegFrame *d, int n, int mxx, int myy, hipStream_t s)
{
    switch (key) {
    case 0x1111: launch_rgba_t<CoefT, NARROW, 1, 1, 1, 1, COLOR>(d, n, mxx, myy, s); break;
    case 0x1211: launch_rgba_t<CoefT, NARROW, 1, 2, 1, 1, COLOR>(d, n, mxx, myy, s); break;
    case 0x2111: launch_rgba_t<CoefT, NARROW, 2, 1, 1, 1, COLOR>(d, n, mxx, myy, s); break;
    case 0x2211: launch_rgba_t<CoefT, NARROW, 2, 2, 1, 1, COLOR>(d, n, mxx, myy, s); break;
    case 0x4111: launch_rgba_t<CoefT, NARROW, 4, 1, 1, 1, COLOR>(d, n, mxx, myy, s); break;
    case 0x4211: launch_rgba_t<CoefT, NARROW, 4, 2, 1, 1, COLOR>(d, n, mxx, myy, s); break;
    case 0x2212: launch_rgba_t<CoefT, NARROW, 2, 2, 1, 2, COLOR>(d, n, mxx, myy, s); break;
    case 0x2221: launch_rgba_t<CoefT, NARROW, 2, 2, 2, 1, COLOR>(d, n, mxx, myy, s); break;
    case 0x2121: launch_rgba_t<CoefT, NARROW, 2, 1, 2, 1, COLOR>(d, n, mxx, myy, s); break;
    case 0x1212: launch_rgba_t<CoefT, NARROW, 1, 2, 1, 2, COLOR>(d, n, mxx, myy, s); break;
    case 0x2222: launch_rgba_t<CoefT, NARROW, 2, 2, 2, 2, COLOR>(d, n, mxx, myy, s); break;
    default: return -2; // geometry without a fused kernel: caller uses planes + rgba pass
    }
    return 0;
}

template <typename CoefT, bool NARROW>
int dispatch_color(int color, int key, const DevJpegFrame *d, int n, int mxx, int myy, hipStream_t s)
{
    switch (color) {
    case ZPX_JPEG_COLOR_YCBCR: return dispatch_geom<CoefT, NARROW, ZPX_JPEG_COLOR_YCBCR>(key, d, n, mxx, myy, s);
    case ZPX_JPEG_COLOR_RGB: return dispatch_geom<CoefT, NARROW, ZPX_JPEG_COLOR_RGB>(key, d, n, mxx, myy, s);
    case ZPX_JPEG_COLOR_GRAY:
        launch_rgba_t<CoefT, NARROW, 1, 1, 1, 1, ZPX_JPEG_COLOR_GRAY>(d, n, mxx, myy, s);
        return 0;
    }
    return -2;
}
} // namespace

bool jpeg_rgba_supported(int color, int h0, int v0, int hc, int vc)
{
    if (color == ZPX_JPEG_COLOR_GRAY) return true;
    const int key = (h0 << 12) | (v0 << 8) | (hc << 4) | vc;
    switch (key) {
    case 0x1111: case 0x1211: case 0x2111: case 0x2211: case 0x4111: case 0x4211:
    case 0x2212: case 0x2221: case 0x2121: case 0x1212: case 0x2222:
        return true;
    }
    return false;
}

int launch_jpeg_rgba(const DevJpegFrame *d_frames, int n_frames, int color, int h0, int v0, int hc,
                     int vc, int max_mxx, int max_myy, int coeff_bits, bool narrow, bool vec_out, bool pieces,
                     hipStream_t stream)
{
    // the block-per-lane kernel (jpeg_block_kernels.hip) takes the common
    // frames; the test switch "jpeg_strip" forces the strip kernel
    if (pieces)
        return vec_out ? launch_jpeg_block(d_frames, n_frames, color, h0, v0, hc, vc, max_mxx, max_myy, coeff_bits,
                                           narrow, true, stream)
                       : -2;
    const bool strip_only = opt(Opt::JpegStrip) != 0;
    if (vec_out && !strip_only) {
        const int rc = launch_jpeg_block(d_frames, n_frames, color, h0, v0, hc, vc, max_mxx, max_myy, coeff_bits,
                                         narrow, false, stream);
        if (rc != -2) return rc;
    }
    const int key = (h0 << 12) | (v0 << 8) | (hc << 4) | vc;
    int rc;
    if (coeff_bits == 8)
        rc = narrow ? dispatch_color<int8_t, true>(color, key, d_frames, n_frames, max_mxx, max_myy, stream)
                    : dispatch_color<int8_t, false>(color, key, d_frames, n_frames, max_mxx, max_myy, stream);
    else if (coeff_bits == 32)
        rc = narrow ? dispatch_color<int32_t, true>(color, key, d_frames, n_frames, max_mxx, max_myy, stream)
                    : dispatch_color<int32_t, false>(color, key, d_frames, n_frames, max_mxx, max_myy, stream);
    else
        rc = narrow ? dispatch_color<int16_t, true>(color, key, d_frames, n_frames, max_mxx, max_myy, stream)
                    : dispatch_color<int16_t, false>(color, key, d_frames, n_frames, max_mxx, max_myy, stream);
    if (rc) return rc;
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

} // namespace zpx
