// gfx950 fused JPEG pixel kernel, one 8x8 block per lane: dequant + 8x8
// integer IDCT + level shift/clamp (reconstructBlock, src/jpeg/decoder.zig:
// 1553-1634; idct.zig:77-201) fused with nearest chroma upsample and
// YCbCr->RGB (Image.rgbaPixels over a YCbCrImage: image.zig:103-130, YCbCrAt
// :614-630, Color.toRGBA .ycbcr color.zig:90-113).  It takes the common
// frames -- int8/int16 coefficients within the 24-bit bound ("narrow"),
// 4:2:0 / 4:2:2 / 4:4:0 / 4:4:4 / gray, dword-aligned RGBA rows of any
// width -- and the strip kernel (jpeg_kernels.hip) the rest.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <type_traits>
#include <utility>

#include "device_types.h"
#include "jpeg_idct.h"
#include "kernels.h"

namespace zpx {
namespace {

// Ordering between LDS instructions of one wave (LDS -> LDS only; not for the
// LDS-DMA, which is a vector-memory operation): the LDS unit executes a wave's
// LDS instructions in issue order, all lanes of one before the next, so a
// compiler fence is enough -- no wait for the writes to complete (measured
// against lgkmcnt(0) at every such point: int8 1.201 -> 1.193 ms).
__device__ __forceinline__ void wave_lds_order()
{
    asm volatile("" ::: "memory");
    __builtin_amdgcn_wave_barrier();
}

// ---------------------------------------------------------------------------
// Fused RGBA kernel, one 8x8 block per lane (jpeg_block_kernel).
//
// A wave owns a task: MCU row `my`, the T = 64 / H0 MCUs from column mx0,
// i.e. 64 luma block columns.  A task is NP passes of (up to) 64 blocks, one
// block per lane.  A pass:
//   1. dequantizes its lane's block from the wave's LDS coefficient image
//      (written by the previous pass's LDS-DMA loads),
//   2. issues the next pass's loads into that image: global_load_lds of
//      1 KiB contiguous per instruction (16 int8 / 8 int16 blocks), the
//      per-lane source addresses permuted so that step 1's ds_read_b128 of
//      a block's 16-byte pieces is bank-conflict-free,
//   3. runs the 2-D IDCT + level shift + clamp in 64 registers (no LDS
//      transpose, no barrier),
//   4. then either writes the block's chroma samples as bytes to the task's
//      chroma tile in LDS (chroma pass), or -- luma pass -- for each of the
//      block's 8 pixel rows reads the row's chroma samples back (nearest
//      upsample: image.zig:614-630), converts YCbCr -> RGBA (color.zig:90-113)
//      and stores the row's 8 pixels as two 16-byte stores.
// Every load and store is unconditional (a block past the grid's edge reads
// a clamped address and never reaches the output; stores outside the image
// get an offset the buffer range check drops), so the vmcnt counts stay
// static and the next pass's loads overlap the whole IDCT + colour work of
// the current one.
// ---------------------------------------------------------------------------
// Fixed design choices, each measured against its alternative (DESIGN.md
// 4.1a "Measured and rejected"):
//   - waves per EU: 3 for the int8 instances (<= 168 VGPRs, no scratch), 2
//     for int16 (at 3 they spill);
//   - 4:4:4 chroma blocks stay in their lanes (32 VGPRs) instead of an LDS
//     tile: 16 waves per CU instead of 8;
//   - the coefficient DMA runs one pass ahead (two: slower at either
//     occupancy), non-temporal for the in-lane and int16 instances (4:4:4
//     1.90 -> 1.85 ms, int16 1.398 -> 1.378; int8 4:2:0 1 % slower with it);
//   - RGBA rows leave through a 2 KiB LDS row tile, as non-temporal
//     whole-line stores (two half-line stores per lane: 1.35 / 1.72 ms
//     against 1.26);
//   - workgroups renumbered so that one XCD holds consecutive tasks (1.7 %).
#ifndef ZPX_JPEG_W8
#define ZPX_JPEG_W8 3
#endif
constexpr int kWavesPerEu8 = ZPX_JPEG_W8, kWavesPerEu16 = 2;
#ifndef ZPX_JPEG_W444
#define ZPX_JPEG_W444 3
#endif
// waves per EU of an instance (the dense 4:4:4 int8 instance: ZPX_JPEG_W444,
// an A/B knob; its pieces twin spills at 4)
template <typename CoefT, int H0, int V0, int HC, int VC, bool ZZ>
constexpr int block_waves_per_eu()
{
    return sizeof(CoefT) == 2 ? kWavesPerEu16
                              : (!ZZ && H0 == 1 && V0 == 1 && HC == 1 && VC == 1 ? ZPX_JPEG_W444 : kWavesPerEu8);
}
constexpr int kStoreAux = 2; // nt
// low-frequency chroma blocks (lf_high): 0 off, 1 the 4x4 test, 2 the 3x3
// test and then the 4x4 one; ZPX_JPEGB_LF_INLANE: also 4:4:4's in-lane
// chroma passes
#ifndef ZPX_JPEGB_LF
#define ZPX_JPEGB_LF 1
#endif
#ifndef ZPX_JPEGB_LF_INLANE
#define ZPX_JPEGB_LF_INLANE 0
#endif
constexpr int kJpegLf = ZPX_JPEGB_LF;
#ifndef ZPX_JPEGB_LF_PARTIAL // (A/B knob: 0 lets 4:1:1's empty chroma lanes vote)
#define ZPX_JPEGB_LF_PARTIAL 1
#endif

// Samples stay in the signed domain (sample - 128, the IDCT's clamp range
// before its level shift): the +128 costs nothing folded into the colour
// constants (luma) or a per-dword xor (packed bytes), instead of an add per
// sample.
constexpr uint32_t kBias4 = 0x80808080u; // four samples of value 0

// The wave's LDS image of one pass's coefficients: 64 blocks as 16-byte
// pieces (P per block: 4 int8, 8 int16).  DMA instruction k (of P) covers
// blocks B*k .. B*k+B-1 (B = 64 / P; 1 KiB of the grid when the blocks are
// contiguous) and writes slots 64k .. 64k+63; block j's piece q sits in slot
//   64 * (j / B) + B * ((q + rot) % P) + j % B,   rot = (P == 8 ? j / B : 0),
// so that for every piece q the 16-lane groups of a ds_read_b128 (lanes j)
// hit 16 distinct 16-byte bank slots.
template <typename CoefT>
struct CoefImage {
    static constexpr int P = 4 * static_cast<int>(sizeof(CoefT)); // pieces per block
    static constexpr int B = 64 / P;                                // blocks per DMA instruction
    static __device__ __forceinline__ int slot(int j, int q)
    {
        const int k = j / B;
        return 64 * k + B * ((q + (P == 8 ? k : 0)) % P) + j % B;
    }
};

// One LDS-DMA load: 16 bytes from each lane's `src` to lds_base + 16 * lane.
// Inline asm, because for the builtin hipcc waits vmcnt(0) -- every store in
// flight -- before any later LDS read; the kernel counts these loads itself
// (the asm is absent from hipcc's s_waitcnt bookkeeping, which can only make
// hipcc's own waits longer, never shorter).  M0 is set and restored inside the
// statement (hipcc reserves it).
template <bool NT>
__device__ __forceinline__ void glds16(const void *src, const void *lds_base)
{
    const uint32_t dst = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(
        (const __attribute__((address_space(3))) void *)lds_base));
    uint32_t keep;
    if constexpr (NT)
        asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off nt\n\ts_mov_b32 m0, %0"
                     : "=&s"(keep) : "v"(src), "s"(dst) : "memory");
    else
        asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                     : "=&s"(keep) : "v"(src), "s"(dst) : "memory");
}

// ---- row IDCT over packed pairs -------------------------------------------
// Stages 1 and 2 of idct.zig's row pass (:99-120) are rotations of pairs of
// dequantized coefficients: x4' = x8 + (W1-W7)x4 with x8 = W7(x4+x5) is
// W1*x4 + W7*x5 exactly (no rounding between), and likewise for the other
// six outputs; x0 +/- x1 is 2048(s0 +/- s4) + 128.  With the block's
// coefficients dequantized as (i16, i16) pairs -- exact, |coef * q| <= 16384
// on the block kernel's frames -- each output is one v_dot2_i32_i16 (the
// exact sum, which equals the reference's wrap-around i32 value since it
// fits), 8 per row instead of 18 multiply/add instructions.
typedef short v2i16 __attribute__((ext_vector_type(2)));
typedef unsigned short v2u16 __attribute__((ext_vector_type(2)));

// (inline asm: for the builtin hipcc picks v_dot2c, whose accumulator is the
// destination, and spends a v_mov per product initialising it; the VOP3P
// form takes the packed constant from an SGPR and an inline 0 or a VGPR)
template <int32_t LO, int32_t HI>
__device__ __forceinline__ int32_t dot2(uint32_t p)
{
    constexpr uint32_t k = (static_cast<uint32_t>(LO) & 0xffffu) | static_cast<uint32_t>(HI) << 16;
    int32_t r;
    asm("v_dot2_i32_i16 %0, %1, %2, 0" : "=v"(r) : "v"(p), "s"(k));
    return r;
}
template <int32_t LO, int32_t HI>
__device__ __forceinline__ int32_t dot2(uint32_t p, int32_t acc)
{
    constexpr uint32_t k = (static_cast<uint32_t>(LO) & 0xffffu) | static_cast<uint32_t>(HI) << 16;
    int32_t r;
    asm("v_dot2_i32_i16 %0, %1, %2, %3" : "=v"(r) : "v"(p), "s"(k), "v"(acc));
    return r;
}
__device__ __forceinline__ uint32_t pk_mul16(uint32_t a, uint32_t b)
{
    return __builtin_bit_cast(uint32_t, __builtin_bit_cast(v2u16, a) * __builtin_bit_cast(v2u16, b));
}
// (asm: hipcc turns select(m, x * a, x * b) into x * select(m, a, b), which
// for scalar a, b costs two v_mov and a v_cndmask a dword)
__device__ __forceinline__ uint32_t pk_mul16_asm(uint32_t a, uint32_t b)
{
    uint32_t r;
    asm("v_pk_mul_lo_u16 %0, %1, %2" : "=v"(r) : "v"(a), "s"(b));
    return r;
}

// Quant-pair rows (DevJpegFrame::qp, built by the host): per row r, four
// dwords holding (q[r][1], q[r][7]), (q[r][5], q[r][3]), (q[r][2], q[r][6]),
// (q[r][0], q[r][4]) as u16 pairs (natural order; tables are at most 16-bit,
// decoder.zig:629-666).
// The coefficient pairs of row r, in the qpair order, sign-extended to i16.
// int8: a piece holds rows 2k and 2k+1 (natural order, 8 bytes a row); the
// v_perm sign selectors reach the odd bytes of a dword, so the even
// coefficients come from the row shifted up a byte.  int16: one row a piece.
template <typename CoefT>
__device__ __forceinline__ u32x4 row_coef_pairs(const u32x4 *raw, int r)
{
    if constexpr (sizeof(CoefT) == 1) {
        const uint32_t w0 = raw[r >> 1][2 * (r & 1)], w1 = raw[r >> 1][2 * (r & 1) + 1];
        const uint32_t w0s = w0 << 8, w1s = w1 << 8;
        return u32x4{__builtin_amdgcn_perm(w1, w0, 0x0b070801u), __builtin_amdgcn_perm(w1, w0, 0x09030a05u),
                     __builtin_amdgcn_perm(w1s, w0s, 0x0b070903u), __builtin_amdgcn_perm(w1s, w0s, 0x0a050801u)};
    } else {
        const u32x4 w = raw[r];
        return u32x4{__builtin_amdgcn_perm(w[3], w[0], 0x07060302u), __builtin_amdgcn_perm(w[1], w[2], 0x07060302u),
                     __builtin_amdgcn_perm(w[3], w[1], 0x05040100u), __builtin_amdgcn_perm(w[2], w[0], 0x05040100u)};
    }
}

// The same pairs from a ZPX_COEFFS_PIECES block: its coefficients in zig-zag
// order (the image's pieces hold 16 int8 / 8 int16 values).  Each pair is one
// v_perm of the two dwords holding its coefficients -- for int8, a value at
// an even byte comes from its dword shifted up a byte, so that the perm's
// sign selectors (which read bytes 1 and 3 of either source) reach it -- the
// same count as the natural order's perms and shifts.
template <typename CoefT>
__device__ __forceinline__ u32x4 row_coef_pairs_zz(const u32x4 *raw, int r)
{
    constexpr int kLo[4] = {1, 5, 2, 0}, kHi[4] = {7, 3, 6, 4}; // the qpair order
    u32x4 o;
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const int za = kZigOf[8 * r + kLo[k]], zb = kZigOf[8 * r + kHi[k]];
        if constexpr (sizeof(CoefT) == 1) {
            const int da = za >> 2, ba = za & 3, db = zb >> 2, bb = zb & 3;
            const uint32_t wa = raw[da >> 2][da & 3], wb = raw[db >> 2][db & 3];
            const uint32_t sa = (ba & 1) ? wa : wa << 8, sb = (bb & 1) ? wb : wb << 8;
            const uint32_t pa = static_cast<uint32_t>(ba | 1), pb = static_cast<uint32_t>(bb | 1);
            const uint32_t sel = pa | (pa == 1 ? 8u : 9u) << 8 | (4u + pb) << 16 | (pb == 1 ? 10u : 11u) << 24;
            o[k] = __builtin_amdgcn_perm(sb, sa, sel);
        } else {
            const int da = za >> 1, ha = za & 1, db = zb >> 1, hb = zb & 1;
            const uint32_t wa = raw[da >> 2][da & 3], wb = raw[db >> 2][db & 3];
            const uint32_t sel = static_cast<uint32_t>(2 * ha) | static_cast<uint32_t>(2 * ha + 1) << 8 |
                                 static_cast<uint32_t>(4 + 2 * hb) << 16 | static_cast<uint32_t>(5 + 2 * hb) << 24;
            o[k] = __builtin_amdgcn_perm(wb, wa, sel);
        }
    }
    return o;
}

// Lane j's block from the LDS image into registers (all LDS reads of the
// image issue here, so the caller's lgkmcnt(0) lets the next DMA refill it).
template <typename CoefT>
__device__ __forceinline__ void load_raw(const uint8_t *img, int j, u32x4 raw[CoefImage<CoefT>::P])
{
#pragma unroll
    for (int pc = 0; pc < CoefImage<CoefT>::P; pc++)
        raw[pc] = *reinterpret_cast<const u32x4 *>(img + 16 * CoefImage<CoefT>::slot(j, pc));
}

// Low-frequency blocks.  A block whose coefficients outside the top-left
// NxN (N = 4 or 3) are all zero (at q75 every chroma block of the 4:2:0
// bench frames, and about half the 64-block chroma passes of 4:4:4 ones)
// has all-zero rows N-7 after the row pass -- the reference's row pass maps
// a zero row to zeros (idct.zig:84-97 and the full path agree there) -- so
// those rows are not transformed, and the row pass of the others and the
// column pass run with their inputs N-7 known zero, which hipcc folds
// (x + 0, 0 * c: the same wrap-around values).  The test is per wave (a
// uniform branch): lf_high() ORs the lane's coefficient words under a mask
// of the positions outside NxN in the storage order (natural, or zig-zag
// for ZPX_COEFFS_PIECES blocks).
template <typename CoefT, bool ZZ, int N>
struct LfMask {
    static constexpr int NW = 16 * static_cast<int>(sizeof(CoefT)); // words per block
    uint32_t m[NW];
    constexpr LfMask() : m{}
    {
        constexpr int per = 4 / static_cast<int>(sizeof(CoefT)); // coefficients per word
        for (int i = 0; i < 64; i++) {
            int nat = i;
            if (ZZ)
                for (int k = 0; k < 64; k++)
                    if (kZigOf[k] == i) nat = k;
            if (nat / 8 >= N || nat % 8 >= N)
                m[i / per] |= (sizeof(CoefT) == 1 ? 0xffu : 0xffffu) << (8 * static_cast<int>(sizeof(CoefT)) * (i % per));
        }
    }
};
template <typename CoefT, bool ZZ, int N>
__device__ __forceinline__ uint32_t lf_high(const u32x4 raw[CoefImage<CoefT>::P])
{
    constexpr LfMask<CoefT, ZZ, N> M{};
    uint32_t acc = 0;
#pragma unroll
    for (int w = 0; w < LfMask<CoefT, ZZ, N>::NW; w++) {
        const uint32_t v = raw[w >> 2][w & 3];
        if (M.m[w] == 0xffffffffu) acc |= v;
        else if (M.m[w] != 0u) acc |= v & M.m[w];
    }
    return acc;
}

// Dequant + row pass (idct.zig:79-145) + column pass with clamp, as
// idct_block, from the raw block and the component's quant-pair table.
// N < 8: the block is low-frequency, its coefficients outside NxN zero (see
// lf_high).
template <typename CoefT, bool ZZ = false, int N = 8, typename QRow>
__device__ __forceinline__ void idct_block_pairs(const u32x4 raw[CoefImage<CoefT>::P], QRow &&qrow, int32_t s[64])
{
#pragma unroll
    for (int r = 0; r < N; r++) { // (rows N-7 are zeros, never read)
        const u32x4 p = qrow(r, ZZ ? row_coef_pairs_zz<CoefT>(raw, r) : row_coef_pairs<CoefT>(raw, r));
        const uint32_t p17 = p[0], p53 = p[1], p26 = p[2], p04 = p[3];
        int32_t x4 = dot2<W1, W7>(p17), x5 = dot2<W7, -W1>(p17);
        int32_t x6 = N <= 3 ? 0 : dot2<W5, W3>(p53), x7 = N <= 3 ? 0 : dot2<W3, -W5>(p53);
        // (N <= 4: coefficient 4 is zero, so x0 = x8; N <= 3: 3 and 5 too)
        int32_t x8 = dot2<2048, 2048>(p04, 128), x0 = N <= 4 ? x8 : dot2<2048, -2048>(p04, 128);
        int32_t x2 = dot2<W6, -W2>(p26), x3 = dot2<W2, W6>(p26);
        int32_t x1 = x4 + x6;
        x4 -= x6;
        x6 = x5 + x7;
        x5 -= x7;
        x7 = x8 + x3;
        x8 -= x3;
        x3 = x0 + x2;
        x0 -= x2;
        x2 = (R2 * (x4 + x5) + 128) >> 8;
        x4 = (R2 * (x4 - x5) + 128) >> 8;
        int32_t *o = s + 8 * r;
        o[0] = (x7 + x1) >> 8;
        o[1] = (x3 + x2) >> 8;
        o[2] = (x0 + x4) >> 8;
        o[3] = (x8 + x6) >> 8;
        o[4] = (x8 - x6) >> 8;
        o[5] = (x0 - x4) >> 8;
        o[6] = (x3 - x2) >> 8;
        o[7] = (x7 - x1) >> 8;
    }
    // (no scheduling barriers between the 1-D transforms: at 107 VGPRs
    // hipcc's interleaving is 0.6 % faster than keeping them apart)
#pragma unroll
    for (int c = 0; c < 8; c++) {
        int32_t t[8];
#pragma unroll
        for (int i = 0; i < 8; i++) t[i] = i >= N ? 0 : s[8 * i + c];
        idct_col_clamp<true, true>(t);
#pragma unroll
        for (int i = 0; i < 8; i++) s[8 * i + c] = t[i];
    }
}

// four signed samples (-128..127) -> one dword of their low bytes (the
// signed domain: xor kBias4 gives the samples' bytes)
__device__ __forceinline__ uint32_t pack4(const int32_t *v)
{
    const uint32_t lo = __builtin_amdgcn_perm(static_cast<uint32_t>(v[1]), static_cast<uint32_t>(v[0]), 0x0c0c0400u);
    const uint32_t hi = __builtin_amdgcn_perm(static_cast<uint32_t>(v[3]), static_cast<uint32_t>(v[2]), 0x0c0c0400u);
    return __builtin_amdgcn_perm(hi, lo, 0x05040100u);
}

// signed byte u (0..3) of a dword of packed signed samples
__device__ __forceinline__ int32_t sbyte(uint32_t w, int u) { return static_cast<int32_t>(w << (24 - 8 * u)) >> 24; }

// The chroma terms of color.zig:95-106 for one (Cb, Cr) sample, given as
// cb1 = Cb - 128, cr1 = Cr - 128 (the signed domain), each with the luma
// level shift 128 * 0x10101 folded in (so a pixel is mad24(Y - 128, 0x10101, t)).
struct ChromaTerms {
    int32_t r, g, b;
};
__device__ __forceinline__ ChromaTerms chroma_terms(int32_t cb1, int32_t cr1)
{
    constexpr int32_t kY = 128 * 0x10101;
    return ChromaTerms{__mul24(91881, cr1) + kY, kY - (__mul24(22554, cb1) + __mul24(46802, cr1)),
                       __mul24(116130, cb1) + kY};
}

// One RGBA pixel from a signed-domain luma sample (see P3b of
// jpeg_rgba_kernel for the clamp form); cb/cr are the signed-domain chroma
// samples (RGB frames only).
template <int COLOR>
__device__ __forceinline__ uint32_t rgba_pixel(int32_t Yv, int32_t cb, int32_t cr, ChromaTerms t)
{
    if constexpr (COLOR == ZPX_JPEG_COLOR_GRAY) {
        return static_cast<uint32_t>(__mul24(Yv, 0x010101) + 128 * 0x010101) | 0xff000000u;
    } else if constexpr (COLOR == ZPX_JPEG_COLOR_RGB) {
        const uint32_t rgb = __builtin_amdgcn_perm(static_cast<uint32_t>(cr), __builtin_amdgcn_perm(static_cast<uint32_t>(cb),
                                                   static_cast<uint32_t>(Yv), 0x0c0c0400u), 0x0c040100u);
        return (rgb ^ 0x808080u) | 0xff000000u;
    } else {
        const int32_t r = __mul24(Yv, 0x10101) + t.r;
        const int32_t g = __mul24(Yv, 0x10101) + t.g;
        const int32_t b = __mul24(Yv, 0x10101) + t.b;
        const uint32_t rc = static_cast<uint32_t>(min(max(r, 0), 0xffffff));
        const uint32_t gc = static_cast<uint32_t>(min(max(g, 0), 0xffffff));
        const uint32_t bc = static_cast<uint32_t>(min(max(b, 0), 0xffffff));
        const uint32_t rg = __builtin_amdgcn_perm(gc, rc, 0x0d0c0602u);
        return __builtin_amdgcn_perm(bc, rg, 0x03060100u);
    }
}

// Two horizontally adjacent YCbCr pixels (color.zig:90-113 as rgba_pixel):
// byte = clamp(v, 0, 0xffffff) >> 16 = clamp(v >> 16, 0, 255), so bytes 2-3
// of each channel's v (v >> 16 as i16: |v| < 2^25) pair up in one dword and
// v_sat_pk_u8_i16 clamps two at once -- 7 instructions a pixel instead of 8
// (3 x v_med3_i32 + 2 x v_perm_b32 after the three v_mad_i32_i24).
__device__ __forceinline__ uint32_t sat_pk_u8(uint32_t x)
{
    uint32_t r;
    asm("v_sat_pk_u8_i16 %0, %1" : "=v"(r) : "v"(x));
    return r;
}
__device__ __forceinline__ void ycbcr_pair(int32_t y0, int32_t y1, ChromaTerms t0, ChromaTerms t1, uint32_t &p0,
                                           uint32_t &p1)
{
    const uint32_t r0 = static_cast<uint32_t>(__mul24(y0, 0x10101) + t0.r), r1 = static_cast<uint32_t>(__mul24(y1, 0x10101) + t1.r);
    const uint32_t g0 = static_cast<uint32_t>(__mul24(y0, 0x10101) + t0.g), g1 = static_cast<uint32_t>(__mul24(y1, 0x10101) + t1.g);
    const uint32_t b0 = static_cast<uint32_t>(__mul24(y0, 0x10101) + t0.b), b1 = static_cast<uint32_t>(__mul24(y1, 0x10101) + t1.b);
    const uint32_t s0 = sat_pk_u8(__builtin_amdgcn_perm(g0, r0, 0x07060302u)); // R0 G0
    const uint32_t s1 = sat_pk_u8(__builtin_amdgcn_perm(g1, r1, 0x07060302u)); // R1 G1
    const uint32_t sb = sat_pk_u8(__builtin_amdgcn_perm(b1, b0, 0x07060302u)); // B0 B1
    p0 = __builtin_amdgcn_perm(sb, s0, 0x0d040100u);
    p1 = __builtin_amdgcn_perm(sb, s1, 0x0d050100u);
}

// The same from the pixels' own signed-domain chroma samples (4:4:4: no
// chroma terms to share), Y * 0x10101 + the level shift computed once a
// pixel: 5 v_mad_i32_i24 instead of 3 + chroma_terms' 4.
__device__ __forceinline__ void ycbcr_pair_direct(int32_t y0, int32_t y1, int32_t cb0, int32_t cr0, int32_t cb1,
                                                  int32_t cr1, uint32_t &p0, uint32_t &p1)
{
    constexpr int32_t kY = 128 * 0x10101;
    // (asm for G's chain: hipcc makes it two v_mul_i32_i24 + v_add3_u32)
    auto mad = [](int32_t a, int32_t k, int32_t c) {
        int32_t r;
        asm("v_mad_i32_i24 %0, %1, %2, %3" : "=v"(r) : "v"(a), "s"(k), "v"(c));
        return r;
    };
    const int32_t yk0 = __mul24(y0, 0x10101) + kY, yk1 = __mul24(y1, 0x10101) + kY;
    const uint32_t r0 = static_cast<uint32_t>(__mul24(91881, cr0) + yk0), r1 = static_cast<uint32_t>(__mul24(91881, cr1) + yk1);
    const uint32_t g0 = static_cast<uint32_t>(mad(cb0, -22554, mad(cr0, -46802, yk0)));
    const uint32_t g1 = static_cast<uint32_t>(mad(cb1, -22554, mad(cr1, -46802, yk1)));
    const uint32_t b0 = static_cast<uint32_t>(__mul24(116130, cb0) + yk0), b1 = static_cast<uint32_t>(__mul24(116130, cb1) + yk1);
    const uint32_t s0 = sat_pk_u8(__builtin_amdgcn_perm(g0, r0, 0x07060302u));
    const uint32_t s1 = sat_pk_u8(__builtin_amdgcn_perm(g1, r1, 0x07060302u));
    const uint32_t sb = sat_pk_u8(__builtin_amdgcn_perm(b1, b0, 0x07060302u));
    p0 = __builtin_amdgcn_perm(sb, s0, 0x0d040100u);
    p1 = __builtin_amdgcn_perm(sb, s1, 0x0d050100u);
}

template <typename F, int... I>
__device__ __forceinline__ void static_for_impl(F &f, std::integer_sequence<int, I...>)
{
    (f(std::integral_constant<int, I>{}), ...);
}
template <int N, typename F>
__device__ __forceinline__ void static_for(F &&f)
{
    static_for_impl(f, std::make_integer_sequence<int, N>{});
}

template <typename CoefT, bool NARROW, int H0, int V0, int HC, int VC, int COLOR, bool ZZ = false>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(block_waves_per_eu<CoefT, H0, V0, HC, VC, ZZ>())))
void jpeg_block_kernel(const DevJpegFrame *__restrict__ frames, int tasks_x, int tasks_per_frame, int total_tasks)
{
    constexpr bool kGray = COLOR == ZPX_JPEG_COLOR_GRAY;
    constexpr int T = 64 / H0;                                  // MCUs per task
    constexpr bool kInLane = !kGray && HC == H0 && VC == V0; // chroma block (x, y) <-> luma block (x, y)
    constexpr bool kDmaNt = kInLane || sizeof(CoefT) == 2;    // non-temporal coefficient DMA
    constexpr int CBW = kGray ? 1 : T * HC;                     // chroma blocks across a task, per component
    constexpr int CBH = kGray ? 1 : VC;
    constexpr int NCB = kGray ? 0 : 2 * CBW * CBH;              // chroma blocks of a task
    constexpr int CP = (kGray || kInLane) ? 0 : (NCB + 63) / 64; // chroma passes through the LDS tile
    constexpr int NP = kGray ? V0 : (kInLane ? 3 * V0 : CP + V0);
    constexpr int RX = kGray ? 1 : H0 / HC, RY = kGray ? 1 : V0 / VC; // upsample ratios
    constexpr int CPX = CBW * 8;                                // chroma tile row (bytes)
    constexpr int CTILE = (kGray || kInLane) ? 16 : CBH * 8 * CPX;
    constexpr int PXH = V0 * 8;                                 // task height in pixels
    constexpr int NS = 8 / RX;                                  // chroma samples per block row
    constexpr bool kDirect = !kGray && RX == 1 && RY == 1;      // 4:4:4: no chroma terms shared between pixels
    static_assert(T * H0 == 64, "a task spans 64 luma block columns");
    // pass p: kind 0 = luma row, 1 = chroma through LDS, 2 = Cb in lane, 3 = Cr in lane
    constexpr auto kind = [](int p) {
        return kGray ? 0 : kInLane ? (p % 3 == 2 ? 0 : 2 + p % 3) : (p < CP ? 1 : 0);
    };
    constexpr auto yrow = [](int p) { return kGray ? p : kInLane ? p / 3 : p - CP; };

    // (quant-pair rows come from the frame descriptor, DevJpegFrame::qp, by
    // scalar loads: no LDS table, 16 waves per CU for int8 4:2:0)
    constexpr int IMG = 64 * 64 * static_cast<int>(sizeof(CoefT)); // the pass's coefficient image
    __shared__ __attribute__((aligned(16))) uint8_t cimg[IMG];
    __shared__ __attribute__((aligned(16))) uint8_t ctile[2][CTILE];
    // one output row of the task (512 RGBA pixels), as 128 16-byte slots;
    // slot s lives at slot s ^ ((s >> 3) & 1), so that both the lanes'
    // 32-byte-strided writes (ds_write_b128: groups of 8 lanes, banks mod 32)
    // and the 16-byte reads of the whole-line stores (ds_read_b128: the 4
    // 16-lane groups, banks mod 64) are conflict-free
    __shared__ __attribute__((aligned(16))) uint8_t otile[2048];
    const int lane = threadIdx.x;
    // row tile: lane's two 16-byte pixel groups are slots 2 lane, 2 lane + 1;
    // it reads back slots lane and 64 + lane (see otile)
    const uint32_t wa0 = 16u * ((2u * lane) ^ ((lane >> 2) & 1u)), wa1 = 16u * ((2u * lane + 1u) ^ ((lane >> 2) & 1u));
    const uint32_t ra = 16u * (static_cast<uint32_t>(lane) ^ ((lane >> 3) & 1u));

    // per-frame uniform values, read once per frame change (frame fields
    // read inside the loop compile to vector loads whose vmcnt waits would
    // also wait for the stores in flight)
    struct TaskSrc {
        const CoefT *g[3]; // (ZZ: the components' piece index arrays)
        const uint8_t *pz; // ZZ: the frame's pieces
        uint64_t qp; // address of DevJpegFrame::qp[0] of the task's frame (uniform: scalar loads)
        uint8_t *rgba;
        int gwy, gwc, myy, width, height;
        uint32_t stride;
    };
    // (every field through readfirstlane: hipcc reads the descriptor with
    // vector loads, and a use of their results after the rare frame-change
    // branch would cost a vmcnt(0) -- a wait for every store in flight -- in
    // every task; this way the wait stays inside the branch)
    // The descriptor is read through the constant address space: scalar
    // loads (lgkmcnt).  Read as vector loads, its use after the loads cost a
    // vmcnt(0) -- every store and DMA in flight -- and a wave's consecutive
    // tasks lie in different frames (tstride waves > tasks per frame), so
    // that drain hit every task.
    typedef const __attribute__((address_space(4))) DevJpegFrame *CFrame;
    auto task_src = [&](int f) __attribute__((always_inline)) {
        const CFrame frp = reinterpret_cast<CFrame>(reinterpret_cast<uintptr_t>(frames)) + f;
        const auto &fr = *frp;
        auto u32 = [](uint32_t x) { return static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(x)); };
        auto ptr = [&](const void *p) {
            const uintptr_t a = reinterpret_cast<uintptr_t>(p);
            return reinterpret_cast<const void *>(static_cast<uintptr_t>(u32(static_cast<uint32_t>(a >> 32))) << 32 |
                                                  u32(static_cast<uint32_t>(a)));
        };
        TaskSrc s;
        s.g[0] = static_cast<const CoefT *>(ptr(fr.coeffs[0]));
        s.g[1] = kGray ? nullptr : static_cast<const CoefT *>(ptr(fr.coeffs[1]));
        s.g[2] = kGray ? nullptr : static_cast<const CoefT *>(ptr(fr.coeffs[2]));
        const int mxx = static_cast<int>(u32(static_cast<uint32_t>(fr.mxx)));
        s.gwy = mxx * H0;
        s.gwc = mxx * HC;
        s.myy = static_cast<int>(u32(static_cast<uint32_t>(fr.myy)));
        s.rgba = static_cast<uint8_t *>(const_cast<void *>(ptr(fr.rgba)));
        s.width = static_cast<int>(u32(static_cast<uint32_t>(fr.width)));
        s.height = static_cast<int>(u32(static_cast<uint32_t>(fr.height)));
        s.stride = u32(static_cast<uint32_t>(fr.rgba_stride));
        s.qp = reinterpret_cast<uint64_t>(ptr(reinterpret_cast<const void *>(reinterpret_cast<uintptr_t>(&fr.qp[0][0]))));
        s.pz = ZZ ? static_cast<const uint8_t *>(ptr(fr.pieces)) : nullptr;
        return s;
    };
    auto coords = [&](int t, int &f, int &my, int &mx0) __attribute__((always_inline)) {
        f = t / tasks_per_frame;
        const int r = t - f * tasks_per_frame;
        my = r / tasks_x;
        mx0 = (r - my * tasks_x) * T;
    };
    // lane's block of pass P: its component (-> quant table, 3 = zeros when
    // the block does not exist) and the chroma block's place in the tile
    struct PassBlock {
        int comp, cx, cy;
        bool ok;
    };
    auto pass_block = [&](auto P, int j) __attribute__((always_inline)) {
        constexpr int p = decltype(P)::value;
        PassBlock b{0, j, yrow(p), true};
        if constexpr (kind(p) == 1) {
            const int idx = p * 64 + j;
            constexpr int PER = CBW * CBH;
            b.ok = idx < NCB;
            b.comp = idx < PER ? 1 : 2;
            const int k = idx < PER ? idx : idx - PER;
            b.cx = k % CBW;
            b.cy = k / CBW;
        } else if constexpr (kind(p) >= 2) {
            b.comp = kind(p) - 1;
        }
        return b;
    };
    // workgroups are dealt to the 8 XCDs round-robin: renumber them so that
    // the waves of one XCD hold consecutive task indices (neighbouring tasks
    // share an XCD's L2)
    int task;
    {
        const int nw = static_cast<int>(gridDim.x), w = static_cast<int>(blockIdx.x);
        const int q = nw / 8, r = nw % 8, x = w % 8;
        task = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + w / 8;
    }
    if (task >= total_tasks) return;
    const int tstride = static_cast<int>(gridDim.x);
    int f, my, mx0;
    coords(task, f, my, mx0);
    TaskSrc ts = task_src(f);
    // one pass's 64 blocks -> cimg (LDS-DMA, see CoefImage).  DMA
    // instruction k carries blocks B*k .. B*k+B-1, which lie in one grid row
    // of one component (B divides a task's chroma blocks per component and
    // the 64 luma columns), so its row address is uniform; a block past the
    // grid's right edge is clamped onto the last one (its pixels never reach
    // the output), a missing grid or row reads the descriptor array.
    auto issue_pass = [&](const TaskSrc &t, int my_, int mx0_, auto P, uint8_t *img) __attribute__((always_inline)) {
        using I = CoefImage<CoefT>;
        constexpr int BYTES = 64 * static_cast<int>(sizeof(CoefT));
#pragma unroll
        for (int k = 0; k < I::P; k++) {
            const PassBlock b0 = pass_block(P, I::B * k);
            const int hh = b0.comp == 0 ? H0 : HC, vv = b0.comp == 0 ? V0 : VC;
            const int gw = b0.comp == 0 ? t.gwy : t.gwc;
            const CoefT *g = b0.comp == 0 ? t.g[0] : (b0.comp == 1 ? t.g[1] : t.g[2]);
            const bool row_ok = b0.ok && g != nullptr && my_ < t.myy;
            const uint8_t *row = row_ok ? reinterpret_cast<const uint8_t *>(g) +
                                              static_cast<size_t>(my_ * vv + b0.cy) * gw * BYTES
                                        : reinterpret_cast<const uint8_t *>(frames);
            const int last = row_ok ? gw - 1 : 0;
            const int bx = min(mx0_ * hh + b0.cx + lane % I::B, last);
            const int q = (lane / I::B + I::P - (I::P == 8 ? k : 0)) % I::P;
            glds16<kDmaNt>(row + static_cast<uint32_t>(bx * BYTES + 16 * q), img + 1024 * k);
        }
    };
    // ZPX_COEFFS_PIECES (ZZ): the index word of the lane's own block of pass
    // P (its pass_block; 0 -- all zeros -- for a block that does not
    // exist), one vector load, made one task ahead
    auto load_ix = [&](const TaskSrc &t, int my_, int mx0_, auto P) __attribute__((always_inline)) -> uint32_t {
        const PassBlock b = pass_block(P, lane);
        const int hh = b.comp == 0 ? H0 : HC, vv = b.comp == 0 ? V0 : VC;
        const int gw = b.comp == 0 ? t.gwy : t.gwc;
        const uint32_t *ix = reinterpret_cast<const uint32_t *>(b.comp == 0 ? t.g[0] : (b.comp == 1 ? t.g[1] : t.g[2]));
        if (!(b.ok && ix != nullptr && my_ < t.myy)) return 0u;
        const int bx = min(mx0_ * hh + b.cx, gw - 1);
        return ix[static_cast<size_t>(my_ * vv + b.cy) * static_cast<uint32_t>(gw) + static_cast<uint32_t>(bx)];
    };
    // ... and the pass's pieces -> cimg in the CoefImage layout: DMA
    // instruction k's lane fetches piece q of block j = B k + lane % B (whose
    // index word lane j holds: ds_bpermute); a piece past the block's count
    // is piece 0, zeros
    auto issue_pass_zz = [&](const TaskSrc &t, uint32_t ixv, uint8_t *img) __attribute__((always_inline)) {
        using I = CoefImage<CoefT>;
#pragma unroll
        for (int k = 0; k < I::P; k++) {
            const uint32_t e = static_cast<uint32_t>(__shfl(static_cast<int>(ixv), I::B * k + lane % I::B));
            const uint32_t q = static_cast<uint32_t>((lane / I::B + I::P - (I::P == 8 ? k : 0)) % I::P);
            const uint32_t piece = q < (e & 15u) ? (e >> 4) + q : 0u;
            glds16<kDmaNt>(t.pz + static_cast<size_t>(piece) * 16, img + 1024 * k);
        }
    };
    // vmcnt bookkeeping (the DMA is inline asm, so the kernel counts it):
    // S(p) stores per pass; the image of pass p was issued one pass earlier,
    // and at pass p's start the operations issued after it are that pass's
    // stores.
    constexpr auto S = [=](int p) { return kind(((p % NP) + NP) % NP) == 0 ? 16 : 0; }; // 8 rows x 2 stores
    constexpr auto vm_wait = [=](int p) { return S(p - 1); };
    // the loop head expects the steady state: the first image in flight,
    // followed by the previous task's stores it would have seen (dropped
    // stores: empty range, distinct offsets)
    const auto none = __builtin_amdgcn_make_buffer_rsrc(const_cast<DevJpegFrame *>(frames), 0, 0, 0x00020000);
    auto pad_stores = [&](int n) __attribute__((always_inline)) {
#pragma unroll
        for (int i = 0; i < 32; i++)
            if (i < n) __builtin_amdgcn_raw_buffer_store_b128(u32x4{0, 0, 0, 0}, none, 16 * i, 0, kStoreAux);
    };
    // ZZ: index words of the current task's passes (ixc) and, loaded at its
    // first pass before that pass's DMA, of the next task's (ixn)
    static_assert(!ZZ || NP >= 2, "the next task's index words load during its predecessor");
    uint32_t ixc[ZZ ? NP : 1], ixn[ZZ ? NP : 1];
    if constexpr (ZZ) {
        static_for<NP>([&](auto Q) __attribute__((always_inline)) { ixc[decltype(Q)::value] = load_ix(ts, my, mx0, Q); });
        issue_pass_zz(ts, ixc[0], cimg);
    } else {
        issue_pass(ts, my, mx0, std::integral_constant<int, 0>{}, cimg);
    }
    (void)ixn;
    pad_stores(S(NP - 1));
    uint32_t cbr[kInLane ? 16 : 1], crr[kInLane ? 16 : 1]; // in-lane chroma samples (bytes)
    (void)cbr;
    (void)crr;
    constexpr uint32_t kDrop = 0x80000000u;

    for (;;) {
        const int tn = task + tstride;
        const bool more = tn < total_tasks;
        int fn = f, myn = my, mxn = mx0;
        if (more) coords(tn, fn, myn, mxn);
        const TaskSrc tsn = fn == f ? ts : task_src(fn);
        // output rows of this task through a buffer descriptor (the host
        // guarantees 32 * rgba_stride < 2^31); a ragged batch's task past a
        // smaller frame's last MCU row gets an empty range
        const int W = ts.width, Y0 = my * PXH;
        const int rows_here = max(0, min(PXH, ts.height - Y0));
        const uint32_t ostride = ts.stride;
        uint8_t *const obase = ts.rgba + static_cast<size_t>(Y0) * ostride;
        // (readfirstlane: the values are uniform; without it hipcc keeps the
        // descriptor in VGPRs and wraps every store in a waterfall loop)
        const uintptr_t oa = reinterpret_cast<uintptr_t>(obase);
        const uint64_t oa_lo = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<uint32_t>(oa)));
        const uint64_t oa_hi = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<uint32_t>(oa >> 32)));
        const auto orsrc = __builtin_amdgcn_make_buffer_rsrc(
            reinterpret_cast<void *>(static_cast<uintptr_t>(oa_hi << 32 | oa_lo)), 0,
            __builtin_amdgcn_readfirstlane(rows_here * static_cast<int>(ostride)), 0x00020000);
        const bool y_present = ts.g[0] != nullptr;
        // the task holding the image's last 4-pixel piece when that piece is
        // partial (W % 4 != 0): its 1-3 pixels leave as dwords (uniform)
        const int X0 = mx0 * H0 * 8;
        const bool edge = (W & 3) != 0 && (W & ~3) >= X0 && (W & ~3) < X0 + 512;

        static_for<NP>([&](auto P) __attribute__((always_inline)) {
            constexpr int p = decltype(P)::value;
            int32_t s[64];
            // this pass's image has landed: the DMA was followed by the
            // previous pass's stores only (16 after a luma pass)
            asm volatile("s_waitcnt vmcnt(%0)" ::"i"(vm_wait(p)) : "memory");
            u32x4 raw[CoefImage<CoefT>::P];
            load_raw<CoefT>(cimg, lane, raw);
            // every lane's reads of the image are done before the DMA refills it
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            // pass p + 1's coefficients load while this pass computes
            constexpr int pn = p + 1;
            if constexpr (ZZ) {
                if constexpr (p == 0)
                    static_for<NP>([&](auto Q) __attribute__((always_inline)) {
                        ixn[decltype(Q)::value] = load_ix(tsn, myn, mxn, Q);
                    });
                if constexpr (pn < NP)
                    issue_pass_zz(ts, ixc[pn], cimg);
                else
                    issue_pass_zz(tsn, ixn[0], cimg);
            } else if constexpr (pn < NP) {
                issue_pass(ts, my, mx0, std::integral_constant<int, pn>{}, cimg);
            } else {
                issue_pass(tsn, myn, mxn, std::integral_constant<int, pn - NP>{}, cimg);
            }
            static_assert(NARROW, "the pair IDCT needs |coef * q| <= 16384");
            {
                // the pass's component(s): one for luma / in-lane passes, and
                // for a chroma pass Cb in lanes < kCb, Cr above (4:2:0, 4:2:2)
                constexpr int kCb = kind(p) == 1 ? (CBW * CBH - p * 64 < 0 ? 0 : CBW * CBH - p * 64) : 0;
                constexpr int c0 = kind(p) == 0 ? 0 : kind(p) >= 2 ? kind(p) - 1 : (kCb > 0 ? 1 : 2);
                // (constant address space: s_load, outside the vmcnt the kernel counts)
                typedef const __attribute__((address_space(4))) u32x4 *cq;
                const uint64_t q0 = ts.qp + 128 * c0, q2 = ts.qp + 256;
                // dequantized pairs of row r: coefficient pairs c x the row's quant pairs
                auto qrow = [&](int r, u32x4 c) __attribute__((always_inline)) {
                    const u32x4 a = *reinterpret_cast<cq>(q0 + 16 * r);
                    if constexpr (kind(p) == 1 && kCb > 0 && kCb < 64) {
                        const u32x4 b = *reinterpret_cast<cq>(q2 + 16 * r);
                        // (both products, then the select: 3 instructions a
                        // dword against 4 for selecting the scalar quant pair)
                        u32x4 o;
#pragma unroll
                        for (int i = 0; i < 4; i++) {
                            const uint32_t pa = pk_mul16_asm(c[i], a[i]), pb = pk_mul16_asm(c[i], b[i]);
                            o[i] = lane < kCb ? pa : pb;
                        }
                        return o;
                    } else {
                        (void)q2;
                        return u32x4{pk_mul16(c[0], a[0]), pk_mul16(c[1], a[1]), pk_mul16(c[2], a[2]), pk_mul16(c[3], a[3])};
                    }
                };
                // an in-lane chroma block's samples leave the transform's
                // registers inside each branch below (16 packed dwords live
                // across the merge instead of 64 values: 4:4:4 int8 spilled
                // otherwise)
                auto inlane_out = [&]() __attribute__((always_inline)) {
                    if constexpr (kind(p) >= 2) {
                        // chroma block kept in this lane: 8 rows x 8 bytes
                        const bool present = ts.g[kind(p) - 1] != nullptr;
                        uint32_t *dst = kind(p) == 2 ? cbr : crr;
#pragma unroll
                        for (int r = 0; r < 8; r++) {
                            dst[2 * r] = present ? pack4(s + 8 * r) : kBias4;
                            dst[2 * r + 1] = present ? pack4(s + 8 * r + 4) : kBias4;
                        }
                    }
                };
                // chroma passes: low-frequency blocks (every lane's) take the
                // short transform (lf_high)
                if constexpr (kJpegLf > 0 && (kind(p) == 1 || (ZPX_JPEGB_LF_INLANE && kind(p) >= 2))) {
                    // (a chroma pass's lanes past the task's chroma blocks --
                    // 4:1:1 / 4:1:0: lanes 32-63 -- read the descriptor array
                    // and never reach the output: left out of the test)
                    constexpr bool kPartial = ZPX_JPEGB_LF_PARTIAL && kind(p) == 1 && (p + 1) * 64 > NCB;
                    const bool real = !kPartial || p * 64 + lane < NCB;
                    if (kJpegLf >= 2 && __builtin_amdgcn_ballot_w64(real && lf_high<CoefT, ZZ, 3>(raw) != 0u) == 0) {
                        idct_block_pairs<CoefT, ZZ, 3>(raw, qrow, s);
                        inlane_out();
                    } else if (__builtin_amdgcn_ballot_w64(real && lf_high<CoefT, ZZ, 4>(raw) != 0u) == 0) {
                        idct_block_pairs<CoefT, ZZ, 4>(raw, qrow, s);
                        inlane_out();
                    } else {
                        idct_block_pairs<CoefT, ZZ, 8>(raw, qrow, s);
                        inlane_out();
                    }
                } else {
                    idct_block_pairs<CoefT, ZZ>(raw, qrow, s);
                    inlane_out();
                }
            }

            if constexpr (kind(p) == 1) {
                // chroma block -> tile (never-scanned component: samples 0)
                const PassBlock b = pass_block(P, lane);
                const bool present = (b.comp == 1 ? ts.g[1] : ts.g[2]) != nullptr;
                uint8_t *t = &ctile[b.comp - 1][(b.cy * 8) * CPX + b.cx * 8];
                if (b.ok) {
#pragma unroll
                    for (int r = 0; r < 8; r++)
                        *reinterpret_cast<u32x2 *>(t + r * CPX) =
                            present ? u32x2{pack4(s + 8 * r), pack4(s + 8 * r + 4)} : u32x2{kBias4, kBias4};
                }
                if constexpr (p == CP - 1) wave_lds_order(); // tile complete before the luma passes
            } else if constexpr (kind(p) >= 2) {
            } else {
                // luma block -> 8 rows of 8 RGBA pixels
                constexpr int yr = yrow(p);
                if (!y_present) { // never-scanned luma: samples 0
#pragma unroll
                    for (int i = 0; i < 64; i++) s[i] = -128;
                }
                uint32_t cs[kGray ? 1 : (NS + 3) / 4][2]; // this chroma row's samples, Cb / Cr
                ChromaTerms ct[kGray ? 1 : NS];
#pragma unroll
                for (int y = 0; y < 8; y++) {
                    if constexpr (!kGray) {
                        if (y % RY == 0) {
                            if constexpr (kInLane) {
                                cs[0][0] = cbr[2 * y];
                                cs[1][0] = cbr[2 * y + 1];
                                cs[0][1] = crr[2 * y];
                                cs[1][1] = crr[2 * y + 1];
                            } else {
                                const int crow = (yr * 8 + y) / RY;
                                const uint8_t *c0 = &ctile[0][crow * CPX + lane * NS];
                                const uint8_t *c1 = &ctile[1][crow * CPX + lane * NS];
                                if constexpr (NS == 8) {
                                    const u32x2 a = *reinterpret_cast<const u32x2 *>(c0);
                                    const u32x2 b = *reinterpret_cast<const u32x2 *>(c1);
                                    cs[0][0] = a[0];
                                    cs[1][0] = a[1];
                                    cs[0][1] = b[0];
                                    cs[1][1] = b[1];
                                } else if constexpr (NS == 4) {
                                    cs[0][0] = *reinterpret_cast<const uint32_t *>(c0);
                                    cs[0][1] = *reinterpret_cast<const uint32_t *>(c1);
                                } else {
                                    cs[0][0] = *reinterpret_cast<const uint16_t *>(c0);
                                    cs[0][1] = *reinterpret_cast<const uint16_t *>(c1);
                                }
                            }
                            if constexpr (COLOR == ZPX_JPEG_COLOR_YCBCR && !kDirect) {
#pragma unroll
                                for (int u = 0; u < NS; u++)
                                    ct[u] = chroma_terms(sbyte(cs[u >> 2][0], u & 3), sbyte(cs[u >> 2][1], u & 3));
                            }
                        }
                    }
                    uint32_t px[8];
                    if constexpr (COLOR == ZPX_JPEG_COLOR_YCBCR && kDirect) {
#pragma unroll
                        for (int x = 0; x < 8; x += 2)
                            ycbcr_pair_direct(s[8 * y + x], s[8 * y + x + 1], sbyte(cs[x >> 2][0], x & 3),
                                              sbyte(cs[x >> 2][1], x & 3), sbyte(cs[x >> 2][0], (x + 1) & 3),
                                              sbyte(cs[x >> 2][1], (x + 1) & 3), px[x], px[x + 1]);
                    } else if constexpr (COLOR == ZPX_JPEG_COLOR_YCBCR) {
#pragma unroll
                        for (int x = 0; x < 8; x += 2)
                            ycbcr_pair(s[8 * y + x], s[8 * y + x + 1], ct[x / RX], ct[(x + 1) / RX], px[x], px[x + 1]);
                    } else
#pragma unroll
                    for (int x = 0; x < 8; x++) {
                        const int u = x / RX;
                        int32_t cb = 0, cr = 0;
                        ChromaTerms t{0, 0, 0};
                        if constexpr (!kGray) {
                            cb = sbyte(cs[u >> 2][0], u & 3);
                            cr = sbyte(cs[u >> 2][1], u & 3);
                            if constexpr (COLOR == ZPX_JPEG_COLOR_YCBCR) t = ct[u];
                        }
                        px[x] = rgba_pixel<COLOR>(s[8 * y + x], cb, cr, t);
                    }
                    const uint32_t rowoff = static_cast<uint32_t>(yr * 8 + y) * ostride;
                    // (a 4-pixel piece wholly inside the row leaves as one
                    // 16-byte store, the partial last one as dwords)
                    // the row's 512 pixels through the LDS row tile (swizzled,
                    // see otile): each store instruction then writes 1 KiB
                    // contiguous (whole lines)
                    *reinterpret_cast<u32x4 *>(otile + wa0) = u32x4{px[0], px[1], px[2], px[3]};
                    *reinterpret_cast<u32x4 *>(otile + wa1) = u32x4{px[4], px[5], px[6], px[7]};
                    wave_lds_order(); // (cross-lane: keep hipcc from reordering around it)
                    const u32x4 va = *reinterpret_cast<const u32x4 *>(otile + ra);
                    const u32x4 vb = *reinterpret_cast<const u32x4 *>(otile + 1024 + ra);
                    wave_lds_order();
                    const int xa = X0 + 4 * lane, xb = xa + 256;
                    const uint32_t oa = xa + 4 <= W ? rowoff + static_cast<uint32_t>(xa) * 4 : kDrop;
                    const uint32_t ob = xb + 4 <= W ? rowoff + static_cast<uint32_t>(xb) * 4 : kDrop;
                    // (non-temporal on dword-aligned rows too: 64 x 4094x4096
                    // 1.61 -> 1.53 ms against cached stores there)
                    __builtin_amdgcn_raw_buffer_store_b128(va, orsrc, oa, 0, kStoreAux);
                    __builtin_amdgcn_raw_buffer_store_b128(vb, orsrc, ob, 0, kStoreAux);
                    if (edge) {
                        // (extra stores after the pass's DMA: the next pass's
                        // vmcnt wait then waits for more than it must, never less)
#pragma unroll
                        for (int u = 0; u < 3; u++) {
                            __builtin_amdgcn_raw_buffer_store_b32(
                                va[u], orsrc, xa + 4 > W && xa + u < W ? rowoff + static_cast<uint32_t>(xa + u) * 4 : kDrop,
                                0, 0);
                            __builtin_amdgcn_raw_buffer_store_b32(
                                vb[u], orsrc, xb + 4 > W && xb + u < W ? rowoff + static_cast<uint32_t>(xb + u) * 4 : kDrop,
                                0, 0);
                        }
                    }
                }
            }
        });
        if (!more) break;
        if constexpr (CP > 0) wave_lds_order(); // the tile's reads precede the next task's writes
        if constexpr (ZZ)
            static_for<NP>([&](auto Q) __attribute__((always_inline)) { ixc[decltype(Q)::value] = ixn[decltype(Q)::value]; });
        task = tn;
        f = fn;
        my = myn;
        mx0 = mxn;
        ts = tsn;
    }
}

// ---------------------------------------------------------------------------
// Planar reconstruct, one 8x8 block per lane (jpeg_plane_block_kernel):
// jpeg.load's output, reconstructBlock into makeImg's planes
// (src/jpeg/decoder.zig:1553-1634, :361-370; idct.zig:77-201).
//
// A task is 64 consecutive blocks of one block row of one component; a wave
// runs tasks persistently.  Per task: the lane's block comes from the wave's
// LDS coefficient image (the fused kernel's CoefImage layout, written by the
// LDS-DMA one task ahead), the next task's DMA is issued, then dequant + the
// dot2 row pass + the column pass with clamp run in registers, and the
// block's 8 rows leave as 8-byte stores: lane j writes bytes 8j..8j+7 of the
// pixel row, so each store instruction writes 512 contiguous bytes of one
// plane row (4 whole lines), non-temporal.  Lanes whose block is outside the
// grid or outside the component's block rule (decoder.zig:1334, :1649-1651)
// store nothing, exactly as the reference leaves those samples at makeImg's
// zero.  As in the fused kernel every load and store is unconditional
// (dropped through the buffer range check), so the vmcnt count is static:
// at a task's start the only operations issued after its DMA are the
// previous task's 8 stores.
// ---------------------------------------------------------------------------
#ifndef ZPX_PLANE_WPE
#define ZPX_PLANE_WPE 4
#endif
#ifndef ZPX_PLANE_DMA_NT
#define ZPX_PLANE_DMA_NT 1
#endif
#ifndef ZPX_PLANE_ST
#define ZPX_PLANE_ST 2
#endif
constexpr int kPlaneWavesPerEu = ZPX_PLANE_WPE; // <= 128 VGPRs: 16 waves per CU
constexpr int kPlaneStoreAux = ZPX_PLANE_ST;
#ifndef ZPX_PLANE_LF
#define ZPX_PLANE_LF 1
#endif
#ifndef ZPX_PLANE_ZZ_NT
#define ZPX_PLANE_ZZ_NT 0
#endif
constexpr bool kPlaneLf = ZPX_PLANE_LF != 0; // low-frequency tasks (lf_high)

template <typename CoefT, bool ZZ = false>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(kPlaneWavesPerEu)))
void jpeg_plane_block_kernel(const DevJpegFrame *__restrict__ frames, PlaneTaskGeom geo)
{
    using I = CoefImage<CoefT>;
    constexpr int BYTES = 64 * static_cast<int>(sizeof(CoefT)); // one block's coefficients
    __shared__ __attribute__((aligned(16))) uint8_t cimg[64 * BYTES];
    const int lane = threadIdx.x;
    typedef const __attribute__((address_space(4))) DevJpegFrame *CFrame;
    auto u32 = [](uint32_t x) { return static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(x)); };
    auto uptr = [&](const void *p) {
        const uintptr_t a = reinterpret_cast<uintptr_t>(p);
        return static_cast<uint64_t>(u32(static_cast<uint32_t>(a >> 32))) << 32 | u32(static_cast<uint32_t>(a));
    };
    // a task's uniform view (scalar loads of the descriptor through the
    // constant address space, as in jpeg_block_kernel)
    struct PTask {
        uint64_t grid, plane, qp; // (ZZ: grid = the component's piece index array)
        uint64_t pz;              // ZZ: the frame's pieces
        uint32_t stride;
        int gw, by, bx0, rule, hh, vv, width, height;
        bool ok;
    };
    auto task_of = [&](int t) __attribute__((always_inline)) {
        PTask k;
        const int f = t / geo.per_frame;
        const int r = t - f * geo.per_frame;
        const int my = r / geo.per_row; // the MCU row, then its component c's block rows
        const int q = r - my * geo.per_row;
        const int c = (q >= geo.start[1]) + (q >= geo.start[2]) + (q >= geo.start[3]);
        const int rr = q - geo.start[c];
        const int yr = rr / geo.segs[c];
        k.by = my * geo.vrows[c] + yr;
        k.bx0 = (rr - yr * geo.segs[c]) * 64;
        const auto &fr = *(reinterpret_cast<CFrame>(reinterpret_cast<uintptr_t>(frames)) + f);
        k.grid = uptr(fr.coeffs[c]);
        k.plane = uptr(fr.planes[c]);
        k.qp = uptr(reinterpret_cast<const void *>(reinterpret_cast<uintptr_t>(&fr.qp[c][0])));
        k.stride = u32(static_cast<uint32_t>(fr.strides[c]));
        k.gw = static_cast<int>(u32(static_cast<uint32_t>(fr.mxx * fr.h[c])));
        const int gh = static_cast<int>(u32(static_cast<uint32_t>(fr.myy * fr.v[c])));
        k.rule = static_cast<int>(u32(static_cast<uint32_t>(fr.rule[c])));
        k.width = static_cast<int>(u32(static_cast<uint32_t>(fr.width)));
        k.height = static_cast<int>(u32(static_cast<uint32_t>(fr.height)));
        k.hh = geo.hh[c];
        k.vv = geo.vv[c];
        k.pz = ZZ ? uptr(fr.pieces) : 0;
        // (a ragged batch's task past a smaller frame's grid, or a component
        // never scanned / without a plane, writes nothing)
        k.ok = k.by < gh && k.bx0 < k.gw && k.grid != 0 && k.plane != 0 && k.rule != ZPX_BLOCKS_NONE;
        return k;
    };
    // the task's 64 blocks -> cimg (see CoefImage): DMA instruction k carries
    // blocks B*k .. B*k+B-1 of the row; past the grid's right edge clamped
    // onto its last block, a task without blocks reads the descriptor array
    auto issue = [&](const PTask &k) __attribute__((always_inline)) {
        const uint8_t *row = k.ok ? reinterpret_cast<const uint8_t *>(k.grid) + static_cast<size_t>(k.by) * k.gw * BYTES
                                  : reinterpret_cast<const uint8_t *>(frames);
        const int last = k.ok ? k.gw - 1 : 0;
#pragma unroll
        for (int i = 0; i < I::P; i++) {
            const int bx = min(k.bx0 + I::B * i + lane % I::B, last);
            const int q = (lane / I::B + I::P - (I::P == 8 ? i : 0)) % I::P;
            glds16<ZPX_PLANE_DMA_NT != 0>(row + static_cast<uint32_t>(bx * BYTES + 16 * q), cimg + 1024 * i);
        }
    };
    // ZZ (ZPX_COEFFS_PIECES): the index word of the lane's block (0 past the
    // grid: zeros), and the task's pieces -> cimg as `issue` does: DMA
    // instruction i's lane fetches piece q of block j = B i + lane % B, whose
    // index word lane j holds (ds_bpermute); past the block's count, piece 0
    auto load_ix = [&](const PTask &k) __attribute__((always_inline)) -> uint32_t {
        if (!k.ok) return 0u;
        const uint32_t *ix = reinterpret_cast<const uint32_t *>(k.grid);
        return ix[static_cast<size_t>(k.by) * static_cast<uint32_t>(k.gw) + static_cast<uint32_t>(min(k.bx0 + lane, k.gw - 1))];
    };
    auto issue_zz = [&](const PTask &k, uint32_t ixv) __attribute__((always_inline)) {
        const uint8_t *pz = reinterpret_cast<const uint8_t *>(k.pz);
#pragma unroll
        for (int i = 0; i < I::P; i++) {
            const uint32_t e = static_cast<uint32_t>(__shfl(static_cast<int>(ixv), I::B * i + lane % I::B));
            const uint32_t q = static_cast<uint32_t>((lane / I::B + I::P - (I::P == 8 ? i : 0)) % I::P);
            const uint32_t piece = q < (e & 15u) ? (e >> 4) + q : 0u;
            // (cached, not non-temporal: the lines a task fetches also hold
            // the pieces of the MCU row's other blocks, which its
            // neighbouring tasks read soon after)
            glds16<ZPX_PLANE_ZZ_NT != 0>(pz + static_cast<size_t>(piece) * 16, cimg + 1024 * i);
        }
    };
    int task;
    {
        const int nw = static_cast<int>(gridDim.x), w = static_cast<int>(blockIdx.x);
        const int q = nw / 8, r = nw % 8, x = w % 8;
        task = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + w / 8; // XCD-consecutive tasks
    }
    if (task >= geo.total) return;
    const int tstride = static_cast<int>(gridDim.x);
    PTask k = task_of(task);
    // ZZ: the next task and its index word, loaded one task ahead of its DMA
    PTask kz = k;
    uint32_t ixz = 0;
    if constexpr (ZZ) {
        issue_zz(k, load_ix(k));
        if (task + tstride < geo.total) {
            kz = task_of(task + tstride);
            ixz = load_ix(kz);
        }
    } else {
        issue(k);
    }
    // the loop head expects the previous task's 8 stores behind the DMA
    // (dropped: empty range; offsets apart, so hipcc cannot merge them into
    // fewer, wider stores -- which would let vmcnt(8) pass before the DMA)
    const auto none = __builtin_amdgcn_make_buffer_rsrc(const_cast<DevJpegFrame *>(frames), 0, 0, 0x00020000);
#pragma unroll
    for (int i = 0; i < 8; i++) __builtin_amdgcn_raw_buffer_store_b64(u32x2{0, 0}, none, 4096 * i, 0, kPlaneStoreAux);
    constexpr uint32_t kDrop = 0x80000000u;
    for (;;) {
        const int tn = task + tstride;
        const bool more = tn < geo.total;
        asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
        u32x4 raw[I::P];
        load_raw<CoefT>(cimg, lane, raw);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        PTask kn = k;
        if constexpr (ZZ) {
            // (the index load after the DMA: the next vmcnt(8) waits for both)
            if (more) {
                kn = kz;
                issue_zz(kn, ixz);
                if (tn + tstride < geo.total) {
                    kz = task_of(tn + tstride);
                    ixz = load_ix(kz);
                }
            }
        } else if (more) {
            kn = task_of(tn);
            issue(kn);
        }
        int32_t s[64];
        typedef const __attribute__((address_space(4))) u32x4 *cq;
        auto qrow = [&](int r, u32x4 c) __attribute__((always_inline)) {
            const u32x4 a = *reinterpret_cast<cq>(k.qp + 16 * r);
            return u32x4{pk_mul16(c[0], a[0]), pk_mul16(c[1], a[1]), pk_mul16(c[2], a[2]), pk_mul16(c[3], a[3])};
        };
        // a task whose 64 blocks are all low-frequency (chroma, mostly)
        // takes the short transform (lf_high)
        if (kPlaneLf && __builtin_amdgcn_ballot_w64(lf_high<CoefT, ZZ, 4>(raw) != 0u) == 0)
            idct_block_pairs<CoefT, ZZ, 4>(raw, qrow, s);
        else
            idct_block_pairs<CoefT, ZZ>(raw, qrow, s);
        const int bx = k.bx0 + lane;
        bool live = k.ok && bx < k.gw;
        if (k.rule == ZPX_BLOCKS_PROGRESSIVE) live = live && bx * k.hh < k.width && k.by * k.vv < k.height;
        else if (k.rule == ZPX_BLOCKS_SCAN) live = live && bx * 8 < k.width && k.by * 8 < k.height;
        const auto prsrc = __builtin_amdgcn_make_buffer_rsrc(
            reinterpret_cast<void *>(k.plane + static_cast<uint64_t>(k.by) * 8 * k.stride), 0,
            static_cast<int>(u32(k.ok ? 8 * k.stride : 0)), 0x00020000);
        const uint32_t o0 = live ? static_cast<uint32_t>(bx) * 8 : kDrop;
#pragma unroll
        for (int r = 0; r < 8; r++) {
            const u32x2 v{pack4(s + 8 * r) ^ kBias4, pack4(s + 8 * r + 4) ^ kBias4};
            __builtin_amdgcn_raw_buffer_store_b64(v, prsrc, live ? o0 + r * k.stride : kDrop, 0, kPlaneStoreAux);
        }
        if (!more) break;
        task = tn;
        k = kn;
    }
}

} // namespace

namespace {
// resident one-wave workgroups on the device for one kernel instance
// (occupancy API: registers + LDS)
template <typename K>
int resident_waves(K kernel)
{
    int per_cu = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, 64, 0) != hipSuccess || per_cu < 1) per_cu = 8;
    // a multiple of the CU's 4 SIMDs: every wave gets the same number of
    // tasks, so a SIMD holding one wave more than the others would set the
    // launch's end (9 waves per CU ran 4:4:4 int16 22 % slower than 8)
    if (per_cu > 4) per_cu &= ~3;
    return device_cu_count() * per_cu;
}

template <typename CoefT, int H0, int V0, int HC, int VC, int COLOR, bool ZZ = false>
int launch_block_t(const DevJpegFrame *d_frames, int n_frames, int max_mxx, int max_myy, hipStream_t stream)
{
    constexpr int T = 64 / H0;
    const int tasks_x = (max_mxx + T - 1) / T;
    const int per_frame = tasks_x * max_myy;
    const int total = per_frame * n_frames;
    auto kernel = jpeg_block_kernel<CoefT, true, H0, V0, HC, VC, COLOR, ZZ>;
    static const int resident = resident_waves(kernel); // (one per instance: this function is)
    const int grid = total < resident ? total : resident;
    if (grid > 0) hipLaunchKernelGGL(kernel, dim3(grid), dim3(64), 0, stream, d_frames, tasks_x, per_frame, total);
    return 0;
}

template <typename CoefT, int COLOR>
int block_geom(int key, const DevJpegFrame *d, int n, int mxx, int myy, hipStream_t s)
{
    switch (key) {
    case 0x2211: return launch_block_t<CoefT, 2, 2, 1, 1, COLOR>(d, n, mxx, myy, s); // 4:2:0
    case 0x2111: return launch_block_t<CoefT, 2, 1, 1, 1, COLOR>(d, n, mxx, myy, s); // 4:2:2
    case 0x1211: return launch_block_t<CoefT, 1, 2, 1, 1, COLOR>(d, n, mxx, myy, s); // 4:4:0
    case 0x1111: return launch_block_t<CoefT, 1, 1, 1, 1, COLOR>(d, n, mxx, myy, s); // 4:4:4
#ifndef ZPX_JPEGB_COMMON_ONLY
    case 0x4111: return launch_block_t<CoefT, 4, 1, 1, 1, COLOR>(d, n, mxx, myy, s); // 4:1:1
    case 0x4211: return launch_block_t<CoefT, 4, 2, 1, 1, COLOR>(d, n, mxx, myy, s); // 4:1:0
    case 0x2212: return launch_block_t<CoefT, 2, 2, 1, 2, COLOR>(d, n, mxx, myy, s); // 2x2 luma, 1x2 chroma
    case 0x2221: return launch_block_t<CoefT, 2, 2, 2, 1, COLOR>(d, n, mxx, myy, s);
    case 0x2222: return launch_block_t<CoefT, 2, 2, 2, 2, COLOR>(d, n, mxx, myy, s); // 4:4:4 in 2x2 MCUs
    case 0x2121: return launch_block_t<CoefT, 2, 1, 2, 1, COLOR>(d, n, mxx, myy, s);
    case 0x1212: return launch_block_t<CoefT, 1, 2, 1, 2, COLOR>(d, n, mxx, myy, s);
#endif
    }
    return -2;
}

// the ZPX_COEFFS_PIECES instances (the batch pipeline's transport: baseline
// frames whose one scan interleaves Y, Cb, Cr)
template <typename CoefT>
int block_pieces(int color, int key, const DevJpegFrame *d, int n, int mxx, int myy, hipStream_t s)
{
    if (color != ZPX_JPEG_COLOR_YCBCR) return -2;
    switch (key) {
    case 0x2211: return launch_block_t<CoefT, 2, 2, 1, 1, ZPX_JPEG_COLOR_YCBCR, true>(d, n, mxx, myy, s);
    case 0x2111: return launch_block_t<CoefT, 2, 1, 1, 1, ZPX_JPEG_COLOR_YCBCR, true>(d, n, mxx, myy, s);
    case 0x1211: return launch_block_t<CoefT, 1, 2, 1, 1, ZPX_JPEG_COLOR_YCBCR, true>(d, n, mxx, myy, s);
    case 0x1111: return launch_block_t<CoefT, 1, 1, 1, 1, ZPX_JPEG_COLOR_YCBCR, true>(d, n, mxx, myy, s);
    }
    return -2;
}

template <typename CoefT>
int block_color(int color, int key, const DevJpegFrame *d, int n, int mxx, int myy, hipStream_t s)
{
    switch (color) {
    case ZPX_JPEG_COLOR_YCBCR: return block_geom<CoefT, ZPX_JPEG_COLOR_YCBCR>(key, d, n, mxx, myy, s);
    case ZPX_JPEG_COLOR_RGB: return block_geom<CoefT, ZPX_JPEG_COLOR_RGB>(key, d, n, mxx, myy, s);
    case ZPX_JPEG_COLOR_GRAY: return launch_block_t<CoefT, 1, 1, 1, 1, ZPX_JPEG_COLOR_GRAY>(d, n, mxx, myy, s);
    }
    return -2;
}
} // namespace

bool jpeg_block_pieces_supported(int color, int h0, int v0, int hc, int vc)
{
    const int key = (h0 << 12) | (v0 << 8) | (hc << 4) | vc;
    return color == ZPX_JPEG_COLOR_YCBCR && (key == 0x2211 || key == 0x2111 || key == 0x1211 || key == 0x1111);
}

int launch_jpeg_plane_block(const DevJpegFrame *d_frames, int n_frames, const JpegPlaneGeom &g, int coeff_bits,
                            bool narrow, bool pieces, hipStream_t stream)
{
    if (!narrow || (coeff_bits != 8 && coeff_bits != 16)) return -2;
    if (g.ncomp < 1 || g.ncomp > 4) return -2;
    PlaneTaskGeom geo{};
    int64_t row = 0; // tasks per MCU row
    for (int c = 0; c < 4; c++) {
        geo.start[c] = static_cast<int32_t>(row);
        geo.segs[c] = 1;
        if (c >= g.ncomp) continue;
        if (g.h[c] <= 0 || g.v[c] <= 0) return -2;
        const int gw = g.max_mxx * g.h[c];
        geo.segs[c] = (gw + 63) / 64;
        geo.rows[c] = g.max_myy * g.v[c];
        geo.vrows[c] = g.v[c];
        geo.hh[c] = 8 * (g.h[0] / g.h[c]);
        geo.vv[c] = 8 * (g.v[0] / g.v[c]);
        row += int64_t(geo.segs[c]) * g.v[c];
    }
    for (int c = g.ncomp; c < 4; c++) geo.start[c] = static_cast<int32_t>(row);
    const int64_t per = row * g.max_myy;
    const int64_t total = per * n_frames;
    if (total <= 0 || row <= 0) return 0;
    if (total >= (int64_t(1) << 31)) return -2;
    geo.per_row = static_cast<int32_t>(row);
    geo.per_frame = static_cast<int32_t>(per);
    geo.total = static_cast<int32_t>(total);
    auto kernel = pieces ? (coeff_bits == 8 ? jpeg_plane_block_kernel<int8_t, true> : jpeg_plane_block_kernel<int16_t, true>)
                         : (coeff_bits == 8 ? jpeg_plane_block_kernel<int8_t> : jpeg_plane_block_kernel<int16_t>);
    static const int resident8 = resident_waves(jpeg_plane_block_kernel<int8_t>);
    static const int resident16 = resident_waves(jpeg_plane_block_kernel<int16_t>);
    static const int resident8z = resident_waves(jpeg_plane_block_kernel<int8_t, true>);
    static const int resident16z = resident_waves(jpeg_plane_block_kernel<int16_t, true>);
    // waves per CU: as many as fit for int8 (20: 8 / 12 / 16 ran 0.855 /
    // 0.823 / 0.810 ms against 0.800 per 64 frames), 8 for int16 (0.952 /
    // 0.972 / 0.988 ms at 8 / 12 / 16 against 0.990 at all 16 that fit;
    // gpurun_out/plab2)
#ifndef ZPX_PLANE_WPCU16
#define ZPX_PLANE_WPCU16 8
#endif
#ifndef ZPX_PLANE_WPCU8Z
#define ZPX_PLANE_WPCU8Z 64
#endif
    const int resident = coeff_bits == 8 ? (pieces ? std::min(resident8z, device_cu_count() * ZPX_PLANE_WPCU8Z) : resident8)
                                         : std::min(pieces ? resident16z : resident16, device_cu_count() * ZPX_PLANE_WPCU16);
    const int grid = total < resident ? static_cast<int>(total) : resident;
    hipLaunchKernelGGL(kernel, dim3(grid), dim3(64), 0, stream, d_frames, geo);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_jpeg_block(const DevJpegFrame *d_frames, int n_frames, int color, int h0, int v0, int hc, int vc,
                      int max_mxx, int max_myy, int coeff_bits, bool narrow, bool pieces, hipStream_t stream)
{
    if (!narrow || (coeff_bits != 8 && coeff_bits != 16)) return -2;
    const int key = (h0 << 12) | (v0 << 8) | (hc << 4) | vc;
    int rc;
    if (pieces)
        rc = coeff_bits == 8 ? block_pieces<int8_t>(color, key, d_frames, n_frames, max_mxx, max_myy, stream)
                             : block_pieces<int16_t>(color, key, d_frames, n_frames, max_mxx, max_myy, stream);
    else
        rc = coeff_bits == 8 ? block_color<int8_t>(color, key, d_frames, n_frames, max_mxx, max_myy, stream)
                             : block_color<int16_t>(color, key, d_frames, n_frames, max_mxx, max_myy, stream);
    if (rc) return rc;
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

} // namespace zpx
