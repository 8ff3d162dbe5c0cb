// gfx950 kernel of the PNG pixel path: filter reconstruction (None/Sub/Up/
// Avg/Paeth, src/png/decoder.zig:806-842 and filterPaeth :1152-1182) fused
// with the per-colour-depth pixel store (:845-1140) and the Adam7 scatter
// (mergePassInto :1289-1373).
//
// The recurrence: byte i of row y depends on byte i-bpp of row y (Sub, Avg,
// Paeth) and on bytes i, i-bpp of row y-1 (Up, Avg, Paeth).  The only
// parallelism inside an image is the anti-diagonal wavefront, so:
//   - one wave owns a band of 64 rows, lane j = row j of the band;
//   - a row is cut into chunks of C pixels (CB = C*bpp = 12 or 16 bytes);
//     at step t lane j reconstructs chunk t-j (a one-chunk skew per row);
//   - the row above arrives from lane j-1 through a DPP wave_shr:1 of the
//     chunk it produced one step earlier (no LDS round trip);
//   - lane 0 takes the previous band's last row from a boundary buffer the
//     previous band's lane 63 fills with 8-byte {epoch, data} granules
//     (agent-scope sc1 stores, no drain), polled with sc1 loads until every
//     tag equals this launch's epoch (MI355X_MICROARCH.md visibility, R2:
//     the data is the flag).  A 16-chunk window is prefetched half a window
//     ahead, so the producer never stalls and the consumer rarely does.
//   - a persistent grid of waves dequeues bands with an atomic ticket in
//     band-major order; a wave only waits for a band with a smaller ticket,
//     which a running wave holds: no co-residency assumption, no deadlock;
//     every spin is bounded (timeout -> status word).
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

#include "device_types.h"
#include "kernels.h"

namespace zpx {
namespace {

// Fixed choices (each measured against its alternatives):
//   - boundary windows of 16 chunks (4 / 8 / 32: within 3 %);
//   - groups of 8 steps: one input burst and one output flush per group
//     (16-step groups do not unroll, and spill);
//   - output chunks through a per-lane LDS ring (16 slots + 1 of padding),
//     flushed as whole aligned lines by 8 lanes per row (one lane per row:
//     4.07 ms, register bursts: 4.37, against 3.6 per 64 x 4K tc8); the
//     cooperative line loads through LDS, paired bursts and a 12-byte raw
//     ring were slower or equal;
//   - 2 x 64 cycles of s_sleep between boundary polls (0 / 1: equal).
constexpr int kRegionChunks = 16;
constexpr int kGroup = 8;     // steps per input/output burst
constexpr int kOutSlots = 17; // 16 ring slots + 1 of padding per lane
#ifndef ZPX_PNG_SPIN_LIMIT
#define ZPX_PNG_SPIN_LIMIT (1u << 20) // default polls per wait
#endif
constexpr int kSleep = 2;

template <int DEPTH>
struct Traits;
#define ZPX_PNG_TRAITS(D, BITS)                                                \
    template <>                                                                \
    struct Traits<D> {                                                         \
        static constexpr int kBits = BITS;                                     \
        static constexpr int kBpp = (BITS + 7) / 8;                            \
        static constexpr int kCB = (kBpp == 3 || kBpp == 6) ? 12 : 16;         \
        static constexpr int kC = kCB / kBpp;                                  \
        static constexpr int kCW = kCB / 4;                                    \
    };
ZPX_PNG_TRAITS(ZPX_PNG_G1, 1)
ZPX_PNG_TRAITS(ZPX_PNG_G2, 2)
ZPX_PNG_TRAITS(ZPX_PNG_G4, 4)
ZPX_PNG_TRAITS(ZPX_PNG_G8, 8)
ZPX_PNG_TRAITS(ZPX_PNG_GA8, 16)
ZPX_PNG_TRAITS(ZPX_PNG_TC8, 24)
ZPX_PNG_TRAITS(ZPX_PNG_P1, 1)
ZPX_PNG_TRAITS(ZPX_PNG_P2, 2)
ZPX_PNG_TRAITS(ZPX_PNG_P4, 4)
ZPX_PNG_TRAITS(ZPX_PNG_P8, 8)
ZPX_PNG_TRAITS(ZPX_PNG_TCA8, 32)
ZPX_PNG_TRAITS(ZPX_PNG_G16, 16)
ZPX_PNG_TRAITS(ZPX_PNG_GA16, 32)
ZPX_PNG_TRAITS(ZPX_PNG_TC16, 48)
ZPX_PNG_TRAITS(ZPX_PNG_TCA16, 64)
#undef ZPX_PNG_TRAITS

// Steps a band takes: its chunks plus the largest lane skew.
__device__ __forceinline__ int nsteps_of(int nchunks, int max_skew) { return nchunks + max_skew; }

__device__ __forceinline__ uint32_t byte_of(const uint32_t *w, int i) { return (w[i >> 2] >> ((i & 3) * 8)) & 0xff; }

// Output pointers are global-address-space so stores are global_store_* (a
// flat store also counts against lgkmcnt and costs an aperture check).
#define ZPX_GLOBAL __attribute__((address_space(1)))
typedef ZPX_GLOBAL uint8_t gu8;
typedef uint32_t gv4 __attribute__((ext_vector_type(4)));
typedef uint32_t gv2 __attribute__((ext_vector_type(2)));
template <typename T> __device__ __forceinline__ ZPX_GLOBAL T *gcast(gu8 *p) { return reinterpret_cast<ZPX_GLOBAL T *>(p); }

// A 16-byte output store (cached: non-temporal ones skip the L2's write
// combining, and each piece became its own HBM write: 11.6 against 3.6 ms)
__device__ __forceinline__ void store16(ZPX_GLOBAL gv4 *p, gv4 v) { *p = v; }

template <int NB>
__device__ __forceinline__ void store_bytes(gu8 *dst, const uint32_t (&w)[(NB + 3) / 4])
{
    const uintptr_t a = reinterpret_cast<uintptr_t>(dst);
    if constexpr (NB % 16 == 0) {
        if ((a & 15) == 0) {
#pragma unroll
            for (int i = 0; i < NB / 16; i++)
                store16(gcast<gv4>(dst) + i, gv4{w[4 * i], w[4 * i + 1], w[4 * i + 2], w[4 * i + 3]});
            return;
        }
    }
    if constexpr (NB % 4 == 0) {
        if ((a & 3) == 0) {
#pragma unroll
            for (int i = 0; i < NB / 4; i++) gcast<uint32_t>(dst)[i] = w[i];
            return;
        }
    }
#pragma unroll
    for (int i = 0; i < NB; i++) dst[i] = static_cast<uint8_t>(w[i >> 2] >> ((i & 3) * 8));
}

// Output bytes per pixel of the image readImagePass allocates (:712-775).
template <int DEPTH>
__device__ __forceinline__ int out_bpp(bool trns)
{
    switch (DEPTH) {
    case ZPX_PNG_G1: case ZPX_PNG_G2: case ZPX_PNG_G4: case ZPX_PNG_G8: return trns ? 4 : 1;
    case ZPX_PNG_GA8: case ZPX_PNG_TC8: case ZPX_PNG_TCA8: return 4;
    case ZPX_PNG_G16: return trns ? 8 : 2;
    case ZPX_PNG_GA16: case ZPX_PNG_TC16: case ZPX_PNG_TCA16: return 8;
    default: return 1; // paletted indices
    }
}

// Write one reconstructed chunk (C units starting at unit u0) of pass row y.
template <int DEPTH>
__device__ __forceinline__ void store_chunk(const DevPngPass &ps, uint32_t y, uint32_t u0,
                                            const uint32_t (&ob)[Traits<DEPTH>::kCW], int &maxidx)
{
    using Tr = Traits<DEPTH>;
    constexpr int C = Tr::kC, BPP = Tr::kBpp;
    const bool trns = ps.use_trns != 0;
    const int obpp = out_bpp<DEPTH>(trns);
    gu8 *row = (gu8 *)(ps.out + static_cast<size_t>(y * ps.yf + ps.yo) * ps.out_stride);
    const uint32_t W = ps.width;

    if constexpr (Tr::kBits < 8 || DEPTH == ZPX_PNG_G8 || DEPTH == ZPX_PNG_P8) {
        // byte units carrying 8/bits pixels each
        constexpr int kBits = Tr::kBits;
        constexpr int kPpb = 8 / kBits;
        constexpr bool kPal = DEPTH >= ZPX_PNG_P1 && DEPTH <= ZPX_PNG_P8;
        constexpr uint32_t kMul = kBits == 1 ? 0xff : kBits == 2 ? 0x55 : kBits == 4 ? 0x11 : 1;
        const uint32_t ty = ps.trns[1];
        const uint32_t x0 = u0 * kPpb;
        if (!trns && ps.xf == 1 && x0 + C * kPpb <= W) {
            // contiguous gray / index bytes
            constexpr int NB = C * kPpb;
            uint32_t w[(NB + 3) / 4];
#pragma unroll
            for (int i = 0; i < (NB + 3) / 4; i++) w[i] = 0;
#pragma unroll
            for (int u = 0; u < C; u++) {
                const uint32_t byte = byte_of(ob, u);
#pragma unroll
                for (int j = 0; j < kPpb; j++) {
                    uint32_t v = (byte >> (8 - kBits * (j + 1))) & ((1u << kBits) - 1);
                    if (kPal) maxidx = max(maxidx, static_cast<int>(v));
                    else v *= kMul;
                    const int q = u * kPpb + j;
                    w[q >> 2] |= v << ((q & 3) * 8);
                }
            }
            store_bytes<NB>(row + static_cast<size_t>(x0 + ps.xo), w);
            return;
        }
#pragma unroll
        for (int u = 0; u < C; u++) {
            const uint32_t byte = byte_of(ob, u);
#pragma unroll
            for (int j = 0; j < kPpb; j++) {
                const uint32_t x = x0 + u * kPpb + j;
                if (x >= W) break;
                uint32_t v = (byte >> (8 - kBits * (j + 1))) & ((1u << kBits) - 1);
                if (kPal) maxidx = max(maxidx, static_cast<int>(v));
                else v *= kMul;
                gu8 *d = row + static_cast<size_t>(x * ps.xf + ps.xo) * obpp;
                if (trns && !kPal) {
                    d[0] = d[1] = d[2] = static_cast<uint8_t>(v);
                    d[3] = v == ty ? 0x00 : 0xff;
                } else {
                    d[0] = static_cast<uint8_t>(v);
                }
            }
        }
        return;
    } else {
        // multi-byte pixels: unit == pixel
        // output bytes per pixel without tRNS (Gray16 2, NRGBA/RGBA 4, *64 8)
        constexpr int OB = (DEPTH == ZPX_PNG_G16) ? 2
                           : (DEPTH == ZPX_PNG_GA16 || DEPTH == ZPX_PNG_TC16 || DEPTH == ZPX_PNG_TCA16) ? 8 : 4;
        uint32_t pix[C][2];
#pragma unroll
        for (int u = 0; u < C; u++) {
            const int b0 = u * BPP;
            uint32_t lo = 0, hi = 0;
            if constexpr (DEPTH == ZPX_PNG_GA8) { // NRGBA (y,y,y,a)
                const uint32_t g = byte_of(ob, b0), a = byte_of(ob, b0 + 1);
                lo = g | g << 8 | g << 16 | a << 24;
            } else if constexpr (DEPTH == ZPX_PNG_TC8) { // RGBA / NRGBA key
                const uint32_t r = byte_of(ob, b0), g = byte_of(ob, b0 + 1), b = byte_of(ob, b0 + 2);
                uint32_t a = 0xff;
                if (trns && r == ps.trns[1] && g == ps.trns[3] && b == ps.trns[5]) a = 0;
                lo = r | g << 8 | b << 16 | a << 24;
            } else if constexpr (DEPTH == ZPX_PNG_TCA8) {
                lo = ob[u];
            } else if constexpr (DEPTH == ZPX_PNG_G16) { // Gray16 BE / NRGBA64 key
                const uint32_t b1 = byte_of(ob, b0), b2 = byte_of(ob, b0 + 1);
                if (trns) {
                    const uint32_t a = (b1 == ps.trns[0] && b2 == ps.trns[1]) ? 0x0000 : 0xffff;
                    const uint32_t g = b1 | b2 << 8; // BE bytes
                    lo = g | g << 16;
                    hi = g | ((a >> 8) | (a & 0xff) << 8) << 16;
                } else {
                    lo = b1 | b2 << 8;
                }
            } else if constexpr (DEPTH == ZPX_PNG_GA16) { // NRGBA64 (y,y,y,a)
                const uint32_t g = byte_of(ob, b0) | byte_of(ob, b0 + 1) << 8;
                const uint32_t a = byte_of(ob, b0 + 2) | byte_of(ob, b0 + 3) << 8;
                lo = g | g << 16;
                hi = g | a << 16;
            } else if constexpr (DEPTH == ZPX_PNG_TC16) { // RGBA64 / NRGBA64 key
                const uint32_t r = byte_of(ob, b0) | byte_of(ob, b0 + 1) << 8;
                const uint32_t g = byte_of(ob, b0 + 2) | byte_of(ob, b0 + 3) << 8;
                const uint32_t b = byte_of(ob, b0 + 4) | byte_of(ob, b0 + 5) << 8;
                uint32_t a = 0xffff;
                if (trns && r == (uint32_t(ps.trns[0]) | uint32_t(ps.trns[1]) << 8) &&
                    g == (uint32_t(ps.trns[2]) | uint32_t(ps.trns[3]) << 8) &&
                    b == (uint32_t(ps.trns[4]) | uint32_t(ps.trns[5]) << 8))
                    a = 0;
                lo = r | g << 16;
                hi = b | a << 16;
            } else { // TCA16: NRGBA64 = raw bytes
                lo = ob[2 * u];
                hi = ob[2 * u + 1];
            }
            pix[u][0] = lo;
            pix[u][1] = hi;
        }
        const uint32_t x0 = u0;
        if (ps.xf == 1 && x0 + C <= W && OB == obpp) {
            constexpr int NB = C * OB;
            uint32_t w[(NB + 3) / 4];
#pragma unroll
            for (int u = 0; u < C; u++) {
                if constexpr (OB == 2) {
                    if (u & 1) w[u >> 1] |= pix[u][0] << 16;
                    else w[u >> 1] = pix[u][0];
                } else if constexpr (OB == 4) {
                    w[u] = pix[u][0];
                } else {
                    w[2 * u] = pix[u][0];
                    w[2 * u + 1] = pix[u][1];
                }
            }
            store_bytes<NB>(row + static_cast<size_t>(x0 + ps.xo) * OB, w);
            return;
        }
#pragma unroll
        for (int u = 0; u < C; u++) {
            const uint32_t x = x0 + u;
            if (x >= W) break;
            gu8 *d = row + static_cast<size_t>(x * ps.xf + ps.xo) * obpp;
            if (obpp == 2) {
                d[0] = static_cast<uint8_t>(pix[u][0]);
                d[1] = static_cast<uint8_t>(pix[u][0] >> 8);
            } else if (obpp == 4) {
                if ((reinterpret_cast<uintptr_t>(d) & 3) == 0) *gcast<uint32_t>(d) = pix[u][0];
                else for (int i = 0; i < 4; i++) d[i] = static_cast<uint8_t>(pix[u][0] >> (8 * i));
            } else {
                if ((reinterpret_cast<uintptr_t>(d) & 7) == 0) {
                    *gcast<gv2>(d) = gv2{pix[u][0], pix[u][1]};
                } else {
                    for (int i = 0; i < 4; i++) d[i] = static_cast<uint8_t>(pix[u][0] >> (8 * i));
                    for (int i = 0; i < 4; i++) d[4 + i] = static_cast<uint8_t>(pix[u][1] >> (8 * i));
                }
            }
        }
    }
}

__device__ __forceinline__ void st_sc1_64(uint64_t *p, uint64_t v)
{
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Reconstruct one byte: out = (f + pred) & 0xff with the predictor of the
// lane's filter.  b (up), c (up-left) and everything derived from them only
// are off the left-to-right dependency chain; a (left) is on it.
// Paeth (:1152-1182) as one v_min3 over keys (dist << 10 | tiebreak << 8 | value):
// the smallest distance wins, ties go a < b < c, exactly the reference's rule.
struct LaneFilter {
    bool sub, up, avg, paeth;
};
__device__ __forceinline__ uint32_t recon_byte(const LaneFilter &lf, uint32_t f, uint32_t a, uint32_t b, uint32_t c)
{
    const uint32_t pa = __builtin_amdgcn_sad_u16(b, c, 0);      // |p - a| = |b - c|
    const uint32_t pb = __builtin_amdgcn_sad_u16(a, c, 0);      // |p - b| = |a - c|
    const uint32_t s = a + b;
    const uint32_t pc = __builtin_amdgcn_sad_u16(s, 2 * c, 0);  // |p - c| = |a + b - 2c|
    const uint32_t m = min(min((pa << 10) | a, (pb << 10) | 0x100u | b), (pc << 10) | 0x200u | c);
    uint32_t t = lf.up ? b : 0u;
    t = lf.sub ? a : t;
    t = lf.avg ? (s >> 1) : t;
    t = lf.paeth ? m : t;
    return (f + t) & 0xffu;
}

// ---------------------------------------------------------------------------
// Input and output staging.  A wave owns 64 rows, one per lane, and each lane
// walks its own row: every vector memory instruction touches 64 different
// cache lines.  Reading 12-16 bytes of a row per step and writing 16 bytes per
// step kept ~2 lines per row live in L2 for 8-10 steps each; at 2048 waves
// (131k rows in flight) that working set is several times the 4 MB L2 of an
// XCD, and PMC showed ~4x the algorithmic bytes fetched and ~3x written.  So
// the step loop runs in groups of G steps: a lane loads the G chunks (+1
// carry dword) of its next group in one burst of 16-byte loads one group
// ahead, and (RGBA8 outputs) writes its G finished chunks as one contiguous
// burst at the end of the group, so a line is fetched once and written whole.
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// Raw buffer descriptor: base, stride 0, num_records bytes (the builtin's
// resource type keeps it in SGPRs).  Offsets outside [0, num_records) --
// negative ones included, as unsigned -- read as zero.
typedef __amdgpu_buffer_rsrc_t Rsrc;
__device__ __forceinline__ Rsrc make_rsrc(const void *base, uint32_t bytes)
{
    // readfirstlane: the inputs are wave-uniform, but hipcc cannot always
    // prove it, and a divergent descriptor would be placed in VGPRs.
    // (readfirstlane returns int: widen through uint32_t, never sign-extend)
    const uintptr_t a = reinterpret_cast<uintptr_t>(base);
    const uint64_t lo = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<uint32_t>(a)));
    const uint64_t hi = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<uint32_t>(a >> 32)));
    void *ua = reinterpret_cast<void *>(static_cast<uintptr_t>(hi << 32 | lo));
    return __builtin_amdgcn_make_buffer_rsrc(ua, 0, static_cast<int>(__builtin_amdgcn_readfirstlane(bytes)), 0x00020000);
}

// N dwords from byte offset off (dword aligned) into d[0..N): 16-byte loads
// then the remainder (no dead destination dwords: a register the code never
// reads would be reused at once and force a wait on the whole burst).
template <int N>
__device__ __forceinline__ void load_dwords(uint32_t (&d)[N], Rsrc rsrc, int off)
{
#pragma unroll
    for (int i = 0; i + 4 <= N; i += 4) {
        const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rsrc, off + 4 * i, 0, 0);
        d[i] = v[0];
        d[i + 1] = v[1];
        d[i + 2] = v[2];
        d[i + 3] = v[3];
    }
    constexpr int T = N & ~3;
    if constexpr (N - T == 1) {
        d[T] = __builtin_amdgcn_raw_buffer_load_b32(rsrc, off + 4 * T, 0, 0);
    } else if constexpr (N - T == 2) {
        const auto v = __builtin_amdgcn_raw_buffer_load_b64(rsrc, off + 4 * T, 0, 0);
        d[T] = v[0];
        d[T + 1] = v[1];
    } else if constexpr (N - T == 3) {
        const auto v = __builtin_amdgcn_raw_buffer_load_b96(rsrc, off + 4 * T, 0, 0);
        d[T] = v[0];
        d[T + 1] = v[1];
        d[T + 2] = v[2];
    }
}

// Boundary window: lane l fetches granules 2l and 2l+1 with two agent-scope
// (sc1) 8-byte loads.
__device__ __forceinline__ u32x4 load_window(const uint64_t *p)
{
    const uint64_t a = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint64_t b = __hip_atomic_load(p + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return u32x4{static_cast<uint32_t>(a), static_cast<uint32_t>(a >> 32), static_cast<uint32_t>(b),
                 static_cast<uint32_t>(b >> 32)};
}

// Depths whose contiguous store of one chunk is exactly 16 bytes of the
// output image (store_chunk's fast path): Gray/indices 8 (16 px), Gray16
// (8 px), RGB8 -> RGBA8/NRGBA8 (4 px), RGBA8 (4 px), RGB16 -> RGBA64 /
// NRGBA64 (2 px), RGBA16 (2 px).
template <int DEPTH>
constexpr bool group_store_depth()
{
    return DEPTH == ZPX_PNG_G8 || DEPTH == ZPX_PNG_P8 || DEPTH == ZPX_PNG_G16 || DEPTH == ZPX_PNG_TC8 ||
           DEPTH == ZPX_PNG_TCA8 || DEPTH == ZPX_PNG_TC16 || DEPTH == ZPX_PNG_TCA16;
}

// The 16 output bytes of one whole chunk, as store_chunk writes them
// (readImagePass :947-950, :963-968, :994-1015, :1033-1039, :1062-1078).
template <int DEPTH, int CW>
__device__ __forceinline__ void pack_chunk16(const DevPngPass &ps, const uint32_t (&ob)[CW], uint32_t (&w)[4])
{
    if constexpr (DEPTH == ZPX_PNG_TC8) { // RGBA (or NRGBA with the colour key)
        // 12 RGB bytes -> 4 RGBA words by byte selects (v_perm_b32), alpha 0xff
        w[0] = __builtin_amdgcn_perm(ob[0], ob[0], 0x0c020100u) | 0xff000000u;
        w[1] = __builtin_amdgcn_perm(ob[1], ob[0], 0x0c050403u) | 0xff000000u;
        w[2] = __builtin_amdgcn_perm(ob[2], ob[1], 0x0c040302u) | 0xff000000u;
        w[3] = __builtin_amdgcn_perm(ob[2], ob[2], 0x0c030201u) | 0xff000000u;
        if (ps.use_trns) { // wave-uniform: the colour key is per image
            const uint32_t key = uint32_t(ps.trns[1]) | uint32_t(ps.trns[3]) << 8 | uint32_t(ps.trns[5]) << 16;
#pragma unroll
            for (int u = 0; u < 4; u++)
                if ((w[u] & 0xffffffu) == key) w[u] &= 0xffffffu;
        }
    } else if constexpr (DEPTH == ZPX_PNG_TC16) { // RGBA64 / NRGBA64, big-endian channels
        const bool trns = ps.use_trns != 0;
#pragma unroll
        for (int u = 0; u < 2; u++) {
            const int b0 = 6 * u;
            const uint32_t r = byte_of(ob, b0) | byte_of(ob, b0 + 1) << 8;
            const uint32_t g = byte_of(ob, b0 + 2) | byte_of(ob, b0 + 3) << 8;
            const uint32_t b = byte_of(ob, b0 + 4) | byte_of(ob, b0 + 5) << 8;
            uint32_t a = 0xffff;
            if (trns && r == (uint32_t(ps.trns[0]) | uint32_t(ps.trns[1]) << 8) &&
                g == (uint32_t(ps.trns[2]) | uint32_t(ps.trns[3]) << 8) &&
                b == (uint32_t(ps.trns[4]) | uint32_t(ps.trns[5]) << 8))
                a = 0;
            w[2 * u] = r | g << 16;
            w[2 * u + 1] = b | a << 16;
        }
    } else { // the chunk's bytes are the output bytes (G8, P8, G16 BE, TCA8, TCA16)
#pragma unroll
        for (int i = 0; i < 4; i++) w[i] = ob[i];
    }
}

template <int DEPTH>
__global__ __launch_bounds__(64) void png_unfilter_kernel(const DevPngPass *__restrict__ passes,
                                                          const DevPngBand *__restrict__ sched, uint32_t nsched,
                                                          uint32_t *ctl, uint64_t *boundary, uint32_t band_granules,
                                                          uint32_t spin_limit)
{
    using Tr = Traits<DEPTH>;
    constexpr int BPP = Tr::kBpp, C = Tr::kC, CW = Tr::kCW;
    constexpr int CB = CW * 4;                  // bytes per chunk
    constexpr int WIN = kRegionChunks;          // chunks per boundary window
    constexpr int WG = WIN * CW;                // granules per window
    constexpr int G = kGroup;                   // steps per group
    constexpr int GD = G * CW + 1;              // input dwords per lane per group (+1: alignbyte carry)
    constexpr bool kGroupStore = group_store_depth<DEPTH>();
    static_assert(!kGroupStore || CW == 4 || DEPTH == ZPX_PNG_TC8 || DEPTH == ZPX_PNG_TC16, "16-byte output chunks");
    static_assert(WG <= 128, "a window is two 8-byte granules per lane");
    static_assert(G % 8 == 0, "the output ring flushes every 8 steps, 16 slots");
    __shared__ __attribute__((aligned(16))) uint64_t win_lds[WG];
    // output ring: 16 chunks of 16 bytes per lane, +1 slot of padding
    constexpr int kRingDw = 4 * kOutSlots; // dwords per lane
    __shared__ __attribute__((aligned(16))) uint32_t out_lds[kGroupStore ? 64 * kRingDw : 1];

    const int lane = threadIdx.x;
    const uint32_t epoch = __builtin_amdgcn_readfirstlane(ctl[0]);
    uint32_t *ticket = ctl + 1, *status = ctl + 2;
    bool timed_out = false;

    for (;;) {
        uint32_t t = 0;
        if (lane == 0) t = atomicAdd(ticket, 1u);
        t = __builtin_amdgcn_readfirstlane(__shfl(t, 0));
        if (t >= nsched) break;
        const DevPngBand bd = sched[t];
        const DevPngPass ps = passes[bd.pass]; // registers: no reloads after output stores
        const uint32_t rb = ps.row_bytes;
        const uint32_t nunits = (rb + BPP - 1) / BPP;
        const int nchunks = static_cast<int>((nunits + C - 1) / C);
        const uint32_t y = bd.band * 64 + lane;
        const bool row_ok = y < ps.rows;
        const uint32_t band_rows = min(64u, ps.rows - bd.band * 64);

        const int ft = row_ok ? ps.filtered[static_cast<size_t>(y) * (rb + 1)] : 0;
        const LaneFilter lf{ft == 1, ft == 2, ft == 3, ft == 4};
        // Dependency-aware skew: a row filtered with Up/Avg/Paeth needs the row
        // above one chunk ahead of it; a None/Sub row needs nothing above, so
        // it starts at step 0 and restarts the chain (lane 0 synchronises with
        // the previous band through the boundary granules instead).
        // skew(j) = j - (last lane <= j that restarts the chain).
        const bool dep = ft >= 2;
        const uint64_t restart = __ballot(!dep || lane == 0);
        const uint64_t upto = restart & (lane == 63 ? ~0ull : ((2ull << lane) - 1));
        const int skew = lane - (63 - __builtin_clzll(upto));
        int max_skew = row_ok ? skew : 0;
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) max_skew = max(max_skew, __shfl_xor(max_skew, off));
        max_skew = __builtin_amdgcn_readfirstlane(max_skew);
        const bool dep0 = (__ballot(dep) & 1ull) != 0;

        // band input: one descriptor based at the dword below the band's
        // first byte; its extent covers the band's rows plus ZPX_PNG_INPUT_PAD
        // bytes (the next band, the next pass or the pad is always behind
        // them), so a 16-byte load holding a row's last bytes is never cut by
        // the range check; loads wholly past it read zeros
        const uint8_t *band0 = ps.filtered + static_cast<size_t>(bd.band) * 64 * (rb + 1);
        const uint8_t *base4 = reinterpret_cast<const uint8_t *>(reinterpret_cast<uintptr_t>(band0) & ~uintptr_t(3));
        const uint32_t delta = static_cast<uint32_t>(band0 - base4);
        const uint64_t extent = delta + static_cast<uint64_t>(band_rows) * (rb + 1) + ZPX_PNG_INPUT_PAD;
        const uint32_t nrec = extent > 0x7ffffff0ull ? 0x7ffffff0u : static_cast<uint32_t>(extent);
        const Rsrc rsrc = make_rsrc(base4, nrec);
        const uint32_t row_off = delta + static_cast<uint32_t>(lane) * (rb + 1); // filter byte of my row
        const uint32_t mis = (row_off + 1) & 3;
        const int data_off = static_cast<int>(row_off + 1 - mis); // dword holding my row's first data byte

        const bool has_prev = bd.band > 0;
        const bool has_next = bd.band + 1 < ps.nbands;
        const bool poll = has_prev && dep0; // lane 0 reads the previous band's last row
        const uint64_t *prev_bnd =
            boundary + static_cast<size_t>(ps.band_base + bd.band - (has_prev ? 1 : 0)) * band_granules;
        uint64_t *my_bnd = boundary + static_cast<size_t>(ps.band_base + bd.band) * band_granules;
        // the current window is staged in LDS (one 16-byte write per lane) and
        // read back at a wave-uniform address: per-step polling waits on
        // lgkmcnt only, never on the input loads in flight
        auto fill_window = [&](int w0) {
            const u32x4 v = load_window(prev_bnd + (2 * lane < WG ? w0 * CW + 2 * lane : 0));
            if (2 * lane < WG) reinterpret_cast<u32x4 *>(win_lds)[lane] = v;
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        };

        // group stores: contiguous rows (xf == 1), 16-byte aligned, and an
        // output type a colour key does not change (Gray8/16 + tRNS -> NRGBA)
        constexpr bool kKeyWidens = DEPTH == ZPX_PNG_G8 || DEPTH == ZPX_PNG_G16;
        // Adam7 passes (xf > 1) of the 4- and 8-byte-pixel depths also go
        // through the ring: a chunk's pixels are scattered xf apart at flush
        constexpr bool kStrided = DEPTH == ZPX_PNG_TC8 || DEPTH == ZPX_PNG_TCA8 || DEPTH == ZPX_PNG_TC16 ||
                                  DEPTH == ZPX_PNG_TCA16;
        const bool gstore = kGroupStore && (ps.xf == 1 || kStrided) && !(kKeyWidens && ps.use_trns) &&
                            ((reinterpret_cast<uintptr_t>(ps.out) | ps.out_stride) & 15) == 0;
        // chunk k's 16 output bytes (pack_chunk16) into output row orow
        auto put_chunk = [&](gu8 *orow, int k, gv4 v) {
            if (ps.xf == 1) { // wave-uniform
                store16(gcast<gv4>(orow + static_cast<size_t>(k) * 16), v);
            } else if constexpr (kStrided) {
                constexpr int OBPX = 16 / C; // output bytes per pixel: 4 or 8
#pragma unroll
                for (int u = 0; u < C; u++) {
                    gu8 *d = orow + static_cast<size_t>((static_cast<uint32_t>(k * C + u)) * ps.xf + ps.xo) * OBPX;
                    if constexpr (OBPX == 8) *gcast<gv2>(d) = gv2{v[2 * u], v[2 * u + 1]};
                    else *gcast<uint32_t>(d) = v[u];
                }
            }
        };
        gu8 *out_row = (gu8 *)(ps.out + static_cast<size_t>(y * ps.yf + ps.yo) * ps.out_stride);
        // output ring slot (k & 15) of row r: write my chunk, read any row's
        auto ring_put = [&](int k, const uint32_t (&ob)[CW]) __attribute__((always_inline)) {
            uint32_t w[4];
            pack_chunk16<DEPTH, CW>(ps, ob, w);
            *reinterpret_cast<gv4 *>(&out_lds[lane * kRingDw + (k & 15) * 4]) = gv4{w[0], w[1], w[2], w[3]};
        };
        auto ring_get = [&](int r, int k) __attribute__((always_inline)) -> gv4 {
            return *reinterpret_cast<const gv4 *>(&out_lds[r * kRingDw + (k & 15) * 4]);
        };

        uint32_t left[BPP], ul[BPP];
#pragma unroll
        for (int i = 0; i < BPP; i++) left[i] = ul[i] = 0;
        uint32_t outp[CW];
#pragma unroll
        for (int i = 0; i < CW; i++) outp[i] = 0;
        int maxidx = 0;
        int flushed = 0;                                     // chunks [0, flushed) of my row are in HBM
        const int nfull = static_cast<int>(ps.width / C);    // chunks whose pixels are all inside the row

        // Output ring flush after `steps` steps: whole aligned 8-chunk blocks
        // (one 128-byte line of RGBA8) as soon as they are complete, and the
        // row's tail at its end. A line is written whole by one lane in one
        // burst, never in two halves a group apart. Called every 8 steps, so
        // at most 15 chunks are pending and 16 slots never collide.
        auto flush_out = [&](int steps) __attribute__((always_inline)) {
            if constexpr (kGroupStore) {
                if (!gstore) return; // wave-uniform
                const int done = min(steps - skew, nchunks); // chunks [0, done) reconstructed
                const int upto = done == nchunks ? done : (done & ~7);
                const int lo = row_ok ? flushed : 0;
                const int hi = row_ok ? max(lo, min(upto, nfull)) : 0;
                if (row_ok) flushed = max(flushed, upto);
                {
                    // Eight lanes write one row's aligned 8-chunk block: each
                    // store instruction covers 8 whole lines instead of 16 bytes
                    // of 64 lines. The block is read from the row's ring slots.
                    const int span = lo | (hi - lo) << 16;
#pragma unroll
                    for (int i = 0; i < 8; i++) {
                        const int r = 8 * i + (lane >> 3);
                        const int sp = __shfl(span, r);
                        const int k = (sp & 0xffff) + (lane & 7);
                        if ((lane & 7) < (sp >> 16)) {
                            const uint32_t yr = bd.band * 64 + static_cast<uint32_t>(r);
                            gu8 *orow = (gu8 *)(ps.out + static_cast<size_t>(yr * ps.yf + ps.yo) * ps.out_stride);
                            put_chunk(orow, k, ring_get(r, k));
                        }
                    }
                    for (int kf = lo + 8; kf < hi; kf++) // a row's tail past its last whole block (end of row only)
                        put_chunk(out_row, kf, ring_get(lane, kf));
                }
            }
        };

        // One group: G steps from step0 over this lane's chunks k0 .. k0+G-1
        // (k0 = step0 - skew), input dwords in `in`.
        auto run_group = [&](const uint32_t (&in)[GD], int step0) {
#pragma unroll
            for (int r = 0; r < G; r++) {
                const int step = step0 + r;
                if (step >= nsteps_of(nchunks, max_skew)) {
                    if ((r & 7) != 0) flush_out(step);
                    break;
                }
                const int k = step - skew;
                const bool act = row_ok && k >= 0 && k < nchunks;

                // ---- the row above: chunk k of row y-1 was produced by lane-1 one step ago
                uint32_t up[CW];
#pragma unroll
                for (int i = 0; i < CW; i++)
                    up[i] = __builtin_amdgcn_update_dpp(0, static_cast<int>(outp[i]), 0x138, 0xf, 0xf, false);
                if (poll && step < nchunks) { // lane 0: chunk `step` of the previous band's last row
                    // At a window's first chunk, wait until the previous band has
                    // published the WHOLE window (its last chunk's granules carry
                    // this launch's epoch), so the next WIN-1 steps read it with no
                    // reload: a band trails the one above by its skew + WIN chunks.
                    const int wi = step % WIN;
                    const int last = min(WIN, nchunks - (step - wi)) - 1; // last chunk of this window
                    if (wi == 0) fill_window(step);
                    auto chunk_ready = [&](int c) {
                        bool ok = true;
#pragma unroll
                        for (int i = 0; i < CW; i++) ok &= static_cast<uint32_t>(win_lds[c * CW + i] >> 32) == epoch;
                        return ok;
                    };
                    uint32_t spins = 0;
                    for (;;) {
                        // this chunk's granules (publication order is not visibility
                        // order), and at a window's start also its last chunk
                        if (chunk_ready(wi) && (wi != 0 || chunk_ready(last))) break;
                        // after a timeout (this wave's, or any wave's: the status
                        // word, checked every 256 polls) never spin again: the
                        // launch's result is already an error, and a stalled
                        // producer must cost one spin limit, not one per step
                        if (timed_out) break;
                        ++spins;
                        if (spins > spin_limit ||
                            ((spins & 255) == 0 &&
                             __hip_atomic_load(status, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0)) {
                            timed_out = true;
                            if (lane == 0) atomicOr(status, 1u);
                            break;
                        }
                        __builtin_amdgcn_s_sleep(kSleep);
                        fill_window(step - wi);
                    }
                    uint32_t gv[CW];
#pragma unroll
                    for (int i = 0; i < CW; i++) gv[i] = static_cast<uint32_t>(win_lds[wi * CW + i]);
                    if (lane == 0) {
#pragma unroll
                        for (int i = 0; i < CW; i++) up[i] = gv[i];
                    }
                } else if (lane == 0) {
#pragma unroll
                    for (int i = 0; i < CW; i++) up[i] = 0; // first row of a pass: zero previous row (:790-793)
                }

                // ---- filtered bytes of chunk k (every lane computes; only active lanes store)
                uint32_t f[CW];
#pragma unroll
                for (int i = 0; i < CW; i++) f[i] = __builtin_amdgcn_alignbyte(in[r * CW + i + 1], in[r * CW + i], mis);
                if (k == 0) {
#pragma unroll
                    for (int i = 0; i < BPP; i++) left[i] = ul[i] = 0;
                }
                // ---- reconstruct C units, left to right
                uint32_t ob[CW];
#pragma unroll
                for (int i = 0; i < CW; i++) ob[i] = 0;
#pragma unroll
                for (int u = 0; u < C; u++) {
#pragma unroll
                    for (int i = 0; i < BPP; i++) {
                        const int idx = u * BPP + i;
                        const uint32_t b = byte_of(up, idx);
                        const uint32_t v = recon_byte(lf, byte_of(f, idx), left[i], b, ul[i]);
                        ob[idx >> 2] |= v << ((idx & 3) * 8);
                        left[i] = v;
                        ul[i] = b;
                    }
                }
#pragma unroll
                for (int i = 0; i < CW; i++) outp[i] = ob[i];

                const bool full = k < nfull;
                if constexpr (kGroupStore) {
                    if (gstore && act && full) ring_put(k, ob);
                }
                if (act) {
                    if (!(gstore && full)) {
                        store_chunk<DEPTH>(ps, y, static_cast<uint32_t>(k * C), ob, maxidx);
                    } else if constexpr (DEPTH == ZPX_PNG_P8) { // palette growth (:1079-1134)
#pragma unroll
                        for (int i = 0; i < 16; i++) maxidx = max(maxidx, static_cast<int>(byte_of(ob, i)));
                    }
                    if (has_next && lane == 63) { // publish: the data is the flag
                        uint64_t *d = my_bnd + static_cast<size_t>(k) * CW;
#pragma unroll
                        for (int i = 0; i < CW; i++) st_sc1_64(d + i, static_cast<uint64_t>(epoch) << 32 | ob[i]);
                    }
                }
                if ((r & 7) == 7) flush_out(step + 1);
            }
        };

        // groups alternate between two input buffers: the loads of group g+1
        // are issued before group g runs (no register copies of loads in flight)
        const int nsteps = nsteps_of(nchunks, max_skew);
        // a group's burst starts before the row for a lane still in its skew
        // (k0 < 0): a 16-byte load at a negative offset reads as zeros whole,
        // so such groups (the first max_skew/G) load dword by dword
        auto load_group = [&](uint32_t (&b)[GD], int step0) {
            const int off = data_off + (step0 - skew) * CB;
            if (__ballot(off < 0) != 0) {
#pragma unroll
                for (int i = 0; i < GD; i++) {
                    // the range check does not wrap voffset + the instruction's
                    // immediate offset: a negative base with a folded +4i reads
                    // zero even where the sum is in range, so select per dword
                    const int o = off + 4 * i;
                    b[i] = __builtin_amdgcn_raw_buffer_load_b32(rsrc, o < 0 ? 0x7fffffff : o, 0, 0);
                }
            } else {
                load_dwords<GD>(b, rsrc, off);
            }
        };
        {
            uint32_t bufA[GD], bufB[GD];
            load_group(bufA, 0);
            for (int step0 = 0; step0 < nsteps; step0 += 2 * G) {
                load_group(bufB, step0 + G);
                run_group(bufA, step0);
                if (step0 + G >= nsteps) break;
                load_group(bufA, step0 + 2 * G);
                run_group(bufB, step0 + G);
            }
        }
        if constexpr (DEPTH >= ZPX_PNG_P1 && DEPTH <= ZPX_PNG_P8) {
            for (int off = 32; off > 0; off >>= 1) maxidx = max(maxidx, __shfl_xor(maxidx, off));
            if (lane == 0 && ps.max_index) atomicMax(ps.max_index, maxidx);
        }
    }
}

// Per-launch control block: the next epoch of the block's window (fresh
// granule tags, so the boundary buffer needs clearing only when the cycle
// wraps: PngControl::prepare), ticket = 0, the previous launch's status
// folded into the sticky word (read and cleared by zpx_plan_status), status = 0.
__global__ void png_ctl_kernel(uint32_t *ctl)
{
    ctl[0] = png_epoch_next(ctl[0], ctl[4], ctl[5]);
    ctl[1] = 0;
    ctl[3] |= ctl[2];
    ctl[2] = 0;
}

// persistent grid: 8 waves per CU (3, 4, 6, 12, 16, 24 measured slower or
// equal)
constexpr int kPngWavesPerCu = 8;

} // namespace

uint32_t png_default_spin_limit() { return static_cast<uint32_t>(ZPX_PNG_SPIN_LIMIT); }

namespace {

template <int DEPTH>
void launch_t(const DevPngPass *passes, const DevPngBand *sched, uint32_t nsched, uint32_t *ctl, uint64_t *boundary,
              uint32_t band_granules, uint32_t spin_limit, hipStream_t s)
{
    const uint32_t want = static_cast<uint32_t>(device_cu_count() * kPngWavesPerCu);
    const uint32_t grid = nsched < want ? nsched : want;
    hipLaunchKernelGGL(png_ctl_kernel, dim3(1), dim3(1), 0, s, ctl);
    hipLaunchKernelGGL((png_unfilter_kernel<DEPTH>), dim3(grid), dim3(64), 0, s, passes, sched, nsched, ctl, boundary,
                       band_granules, spin_limit ? spin_limit : png_default_spin_limit());
}

} // namespace

int png_chunk_bytes(int depth)
{
    switch (depth) {
    case ZPX_PNG_TC8: case ZPX_PNG_TC16: return 12;
    default: return 16;
    }
}

int png_band_granules(int depth, uint32_t max_row_bytes)
{
    const uint32_t cb = static_cast<uint32_t>(png_chunk_bytes(depth));
    const uint32_t nchunks = (max_row_bytes + cb - 1) / cb;
    const uint32_t gran = nchunks * (cb / 4) + 64; // + slack for the window's over-read
    return static_cast<int>((gran + 31) & ~31u);
}

int launch_png_unfilter(int depth, const DevPngPass *passes, const DevPngBand *sched, uint32_t nsched,
                        uint32_t *ctl, uint64_t *boundary, uint32_t band_granules, hipStream_t s,
                        uint32_t spin_limit)
{
    switch (depth) {
#define ZPX_CASE(D) case D: launch_t<D>(passes, sched, nsched, ctl, boundary, band_granules, spin_limit, s); break;
        ZPX_CASE(ZPX_PNG_G1) ZPX_CASE(ZPX_PNG_G2) ZPX_CASE(ZPX_PNG_G4) ZPX_CASE(ZPX_PNG_G8)
        ZPX_CASE(ZPX_PNG_GA8) ZPX_CASE(ZPX_PNG_TC8) ZPX_CASE(ZPX_PNG_P1) ZPX_CASE(ZPX_PNG_P2)
        ZPX_CASE(ZPX_PNG_P4) ZPX_CASE(ZPX_PNG_P8) ZPX_CASE(ZPX_PNG_TCA8) ZPX_CASE(ZPX_PNG_G16)
        ZPX_CASE(ZPX_PNG_GA16) ZPX_CASE(ZPX_PNG_TC16) ZPX_CASE(ZPX_PNG_TCA16)
#undef ZPX_CASE
    default: return -2;
    }
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

} // namespace zpx
