// gfx950 PNG filter reconstruction, two rows per lane in packed 16-bit halves
// (the unfilter loop of readImagePass, src/png/decoder.zig:806-842, filterPaeth
// :1152-1182, fused with the pixel store :845-1140 and the Adam7 scatter of
// mergePassInto :1289-1373) for the byte-aligned depths whose chunk is 16
// output bytes: RGB8 (RGBA / NRGBA with a colour key), RGBA8, Gray8, Gray16,
// RGB16 (RGBA64 / NRGBA64 with a colour key), RGBA16.
//
// Adam7 (api_internal.h, Adam7Stage): passes 1-5 are unfiltered into
// staging rows, pass 7 into the image's odd rows -- both contiguous -- and
// pass 6, in a second launch, writes every even row whole: its own pixels
// at the odd columns, the even columns read from the staged passes
// (flush_merge).  No pass scatters pixels xf apart into the image.
//
// Work layout.  A wave owns a band of 128 rows of one pass: lane j holds rows
// 2j (low 16-bit half of every register) and 2j+1 (high half), so one VALU
// instruction reconstructs a byte of each.  Rows are cut into chunks of CB
// bytes (12 for 3/6-byte pixels, else 16); at step t row r reconstructs chunk
// t - skew(r), where skew(r) = r - (last row <= r that restarts the chain:
// None/Sub filter, or the band's first row).  The row above arrives one step
// late from the previous step's outputs:
//   - row 2j+1 (high half) reads row 2j = the low half of its own lane,
//   - row 2j (low half) reads row 2j-1 = the high half of lane j-1, through a
//     DPP wave_shr:1 of the output registers; lane 0 takes the value the DPP
//     leaves in its `old` operand: the previous band's last row (boundary
//     granules, see png_kernels.hip) or zero (the first row of a pass).
// so up = alignbit(out, dpp_shr1(out), 16) = [lane j-1 hi, own lo].
//
// Per byte pair the whole filter set is one path: the Paeth keys
// dist * 8 + code (code = the byte position of a / b / c in a v_perm
// source pair; a and b tie harmlessly, c loses every tie -- the reference's
// a < b < c rule), the smallest key's code picks the predictor byte, and a
// per-half (KEEP, FORCE) pair overrides the code for None / Sub / Up / Avg
// (Avg's (a + b) >> 1 is a fourth byte of the same v_perm source).  The
// distances come from packed fp16 arithmetic on the bytes read as fp16
// denormals (the u16 value n is n * 2^-24; the kernel runs with f16
// denormals preserved, .amdhsa_float_denorm_mode_16_64 3): every
// difference and sum of them is exact, and the result's bits are sign |
// magnitude with the magnitude the integer distance, so one v_pk_mad_u16
// (x * 8 + code, mod 2^16: the sign bit shifts out) makes each key:
//   va = b - c, vb = a - c, vc = va + vb        (v_pk_add_f16, neg modifiers)
//   k* = v* * 8 + code*;  sel = (min3(ka, kb, kc) & KEEP) | FORCE
//   t = perm(c | lerp_u8(a, b) << 8, a | b << 8, sel);  out = (f + t) & 0x00ff00ff
// 14 instructions per byte PAIR (23 with packed-integer max - min distances
// and a separate add and shift for Avg), against ~21 per byte one row per lane.
//
// Memory: every lane burst-loads its two rows' next group of kG = 8 chunks one
// group ahead -- from the band slab (the rows interleaved two bytes at a time,
// png_slab.cpp: 1 KiB contiguous per instruction), or, in the STREAM
// instance, from the inflated stream as parseIdat hands it over (16-byte
// unaligned loads, a row's window on consecutive lanes, turned round into
// the row-per-lane registers through an LDS staging area) -- through buffer
// descriptors (every load and store of the group
// loop is unconditional -- out-of-range offsets read zero / drop the store --
// so s_waitcnt counts stay exact); each reconstructed chunk is expanded to
// its 16 output bytes (colour key, 16-bit order) into a per-row LDS ring of
// 2 FL slots (PairShape); every FL steps, a fixed 2 FL rounds of cooperative flush
// store each row's newly completed aligned 8-chunk block (one 128-byte line
// of RGBA8) with 8 lanes per row, from a transposed per-row flush state.
// The boundary window of the band above is prefetched one group ahead and
// polled out of line.  The hot loop is one group, so the loop body stays a
// few KB of code (the one-row-per-lane kernel's 94 KB loop missed the
// instruction cache).
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

#include "device_types.h"
#include "kernels.h"

namespace zpx {
namespace {

#define ZPX_GLOBAL __attribute__((address_space(1)))
typedef ZPX_GLOBAL uint8_t gu8;
typedef uint32_t v4u __attribute__((ext_vector_type(4)));
typedef uint32_t v2u __attribute__((ext_vector_type(2)));
template <typename T> __device__ __forceinline__ ZPX_GLOBAL T *gptr(gu8 *p) { return reinterpret_cast<ZPX_GLOBAL T *>(p); }

constexpr int kG = 8; // steps per group (input burst)
#ifndef ZPX_A7_NOLOAD
#define ZPX_A7_NOLOAD 0
#endif
#ifndef ZPX_A7_NT
#define ZPX_A7_NT 0
#endif
constexpr int kSleep = 2; // s_sleep between boundary polls (units of 64 cycles; 0 / 1 measured equal)

template <int DEPTH> struct PairTraits;
#define ZPX_PAIR_TRAITS(D, BPP_, OBPX_)                                        \
    template <> struct PairTraits<D> {                                         \
        static constexpr int BPP = BPP_;                 /* filter bytes/px */ \
        static constexpr int CB = (BPP_ == 3 || BPP_ == 6) ? 12 : 16;          \
        static constexpr int CW = CB / 4;                                      \
        static constexpr int C = CB / BPP_;              /* pixels/chunk */    \
        static constexpr int OBPX = OBPX_;               /* out bytes/px */    \
    };
ZPX_PAIR_TRAITS(ZPX_PNG_G8, 1, 1)
ZPX_PAIR_TRAITS(ZPX_PNG_G16, 2, 2)
ZPX_PAIR_TRAITS(ZPX_PNG_TC8, 3, 4)
ZPX_PAIR_TRAITS(ZPX_PNG_TCA8, 4, 4)
ZPX_PAIR_TRAITS(ZPX_PNG_TC16, 6, 8)
ZPX_PAIR_TRAITS(ZPX_PNG_TCA16, 8, 8)
#undef ZPX_PAIR_TRAITS

// Flush shape of an instance: FL = chunks per flushed block = steps between
// flushes; the ring holds 2 FL chunks a row (a pending block's FL - 1 plus
// FL new ones), and W waves per SIMD fit its LDS (128 rows x (2 FL + 1) x
// 16 B) and registers.  FL 8 (35 KiB of ring) leaves one wave per SIMD,
// which issues a VOP3 only every ~5 cycles.  FL 4 (18 KiB) fits two, whose
// instructions interleave (tools/ubench/valu_rate: 6.98 cycles each at 2
// waves per SIMD, 1.45x the SIMD's issue rate) -- but 64 x 4K tc8 ran 2.84
// ms that way against 2.32: with 2,048 resident waves every band of an
// image starts at once and waits for the band above it, and the input
// loads, 64 rows per instruction, are the limit rather than issue
// (tools/ubench/png_load_pattern: this load shape alone reads the stream at
// 2.2 TB/s).  Re-measured on the band slab (round 4, ZPX_PNG_FL=4
// ZPX_PNG_W=2: 256 VGPRs, 17.9 KiB of LDS, no scratch): 2.335 / 2.355 ms
// against 1.778 / 1.767 (gpurun_out/pnga).  So FL stays 8.
#ifndef ZPX_PNG_FL
#define ZPX_PNG_FL 8
#endif
#ifndef ZPX_PNG_W
#define ZPX_PNG_W 1
#endif
template <int DEPTH, bool MERGE>
struct PairShape {
    static constexpr int FL = MERGE ? 8 : ZPX_PNG_FL;
    static constexpr int W = MERGE ? 1 : ZPX_PNG_W;
};

// ---- packed 16-bit helpers (v_pk_*_u16, v_pk_add_f16)
typedef _Float16 h16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ h16x2 ash(uint32_t x) { return __builtin_bit_cast(h16x2, x); }
__device__ __forceinline__ uint32_t hbits(h16x2 x) { return __builtin_bit_cast(uint32_t, x); }
// key of a packed fp16 distance: |d| * 8 + code per half, one v_pk_mad_u16
// (hipcc splits the C form into a shift and an or)
__device__ __forceinline__ uint32_t pk_key(h16x2 d, uint32_t code)
{
    uint32_t k;
    asm("v_pk_mad_u16 %0, %1, 8, %2 op_sel_hi:[1,0,1]" : "=v"(k) : "v"(hbits(d)), "s"(code));
    return k;
}

// Paeth key codes: the byte position of each candidate in perm(cav, ab):
// ab = [a.lo, b.lo, a.hi, b.hi] (bytes 0-3), cav = [c.lo, avg.lo, c.hi, avg.hi]
// (bytes 4-7); low half codes a 0, b 1, c 4, avg 5; high half 2, 3, 6, 7.
constexpr uint32_t kKA = 0x00020000u, kKB = 0x00030001u, kKC = 0x00060004u;

struct PairFilter {
    uint32_t keep, force; // sel = (key & keep) | force, per 16-bit half
};
// filter type -> (keep, force) of one half (h = 0 low, 1 high)
__device__ __forceinline__ PairFilter half_filter(int ft, int h)
{
    const uint32_t sh = h ? 16u : 0u, base = h ? 2u : 0u;
    uint32_t keep = 0, force = 0x0c00u;
    switch (ft) {
    case 1: force |= base + 0; break;     // Sub: a
    case 2: force |= base + 1; break;     // Up: b
    case 3: force |= base + 5; break;     // Avg: (a + b) >> 1
    case 4: keep = 0x0007u; break;        // Paeth: the smallest key's code
    default: force = 0x0c0cu; break;      // None: zero
    }
    return PairFilter{keep << sh, force << sh};
}

// One byte pair: out = (f + predictor) mod 256 per half.  f's bytes 1 and 3
// may hold anything (the slab's interleaved bytes): the add is per 16-bit
// half (v_pk_add_u16), so nothing carries between the rows, and the mask
// keeps each half's low byte.
__device__ __forceinline__ uint32_t recon_pair(uint32_t f, uint32_t a, uint32_t b, uint32_t c, PairFilter pf)
{
    const h16x2 va = ash(b) - ash(c); // b - c: pa = |va|
    const h16x2 vb = ash(a) - ash(c); // a - c: pb = |vb|
    const h16x2 vc = va + vb;         // a + b - 2c: pc = |vc|
    // the keys (<= 510 * 8 + 7) are positive fp16 bit patterns, ordered as
    // the integers: one v_pk_minimum3_f16 takes the smallest
    const uint32_t m = hbits(__builtin_elementwise_minimum(
        __builtin_elementwise_minimum(ash(pk_key(va, kKA)), ash(pk_key(vb, kKB))), ash(pk_key(vc, kKC))));
    const uint32_t sel = (m & pf.keep) | pf.force;
    const uint32_t ab = a | (b << 8);
    const uint32_t cav = c | (__builtin_amdgcn_lerp(a, b, 0u) << 8); // avg = (a + b) >> 1 per byte (v_lerp_u8)
    const uint32_t t = __builtin_amdgcn_perm(cav, ab, sel);
    typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
    return __builtin_bit_cast(uint32_t, __builtin_bit_cast(u16x2, f) + __builtin_bit_cast(u16x2, t)) & 0x00ff00ffu;
}

// ---- output of one chunk: the 16 bytes store_chunk writes (readImagePass
// :947-950, :963-968, :994-1015, :1033-1039, :1062-1078), from CW raw dwords
template <int DEPTH, bool TRNS>
__device__ __forceinline__ v4u expand_chunk(const DevPngPass &ps, const uint32_t *ob)
{
    if constexpr (DEPTH == ZPX_PNG_TC8) { // RGBA, alpha 0xff (NRGBA with the colour key)
        v4u w;
        w[0] = __builtin_amdgcn_perm(ob[0], ob[0], 0x0d020100u); // selector 0x0d: byte 0xff
        w[1] = __builtin_amdgcn_perm(ob[1], ob[0], 0x0d050403u);
        w[2] = __builtin_amdgcn_perm(ob[2], ob[1], 0x0d040302u);
        w[3] = __builtin_amdgcn_perm(ob[2], ob[2], 0x0d030201u);
        if constexpr (TRNS) {
            const uint32_t key = uint32_t(ps.trns[1]) | uint32_t(ps.trns[3]) << 8 | uint32_t(ps.trns[5]) << 16;
#pragma unroll
            for (int u = 0; u < 4; u++)
                if ((w[u] & 0xffffffu) == key) w[u] &= 0xffffffu;
        }
        return w;
    } else if constexpr (DEPTH == ZPX_PNG_TC16) { // RGBA64 (NRGBA64 with the key), big-endian channels
        // bytes r0 r1 g0 g1 b0 b1 | r0 r1 g0 g1 b0 b1 in ob[0..2]
        v4u w;
        w[0] = ob[0];                                             // r, g of pixel 0
        w[1] = __builtin_amdgcn_perm(ob[1], ob[1], 0x0d0d0100u);  // b, alpha ffff
        w[2] = __builtin_amdgcn_perm(ob[2], ob[1], 0x05040302u);  // r, g of pixel 1
        w[3] = __builtin_amdgcn_perm(ob[2], ob[2], 0x0d0d0302u);  // b, alpha ffff
        if constexpr (TRNS) {
            const uint32_t k01 = uint32_t(ps.trns[0]) | uint32_t(ps.trns[1]) << 8 | uint32_t(ps.trns[2]) << 16 |
                                 uint32_t(ps.trns[3]) << 24;
            const uint32_t k2 = uint32_t(ps.trns[4]) | uint32_t(ps.trns[5]) << 8;
            if (w[0] == k01 && (w[1] & 0xffffu) == k2) w[1] &= 0xffffu;
            if (w[2] == k01 && (w[3] & 0xffffu) == k2) w[3] &= 0xffffu;
        }
        return w;
    } else { // the chunk's bytes are the output bytes (Gray8, Gray16 BE, RGBA8, RGBA16)
        return v4u{ob[0], ob[1], ob[2], ob[3]};
    }
}

// chunk k's 16 output bytes into a contiguous output row
template <int DEPTH>
__device__ __forceinline__ void put_chunk(gu8 *orow, int k, v4u v)
{
    *gptr<v4u>(orow + static_cast<size_t>(k) * 16) = v;
}

// the pixels [k C, k C + n) of chunk k (n <= C), xf apart, byte stores
template <int DEPTH>
__device__ __forceinline__ void put_partial(const DevPngPass &ps, gu8 *orow, int k, v4u v, int n)
{
    using T = PairTraits<DEPTH>;
    for (int u = 0; u < n; u++) {
        gu8 *d = orow + static_cast<size_t>(static_cast<uint32_t>(k * T::C + u) * ps.xf + ps.xo) * T::OBPX;
        for (int i = 0; i < T::OBPX; i++) {
            const int byte = u * T::OBPX + i;
            d[i] = static_cast<uint8_t>(v[byte >> 2] >> ((byte & 3) * 8));
        }
    }
}

// ---- Adam7 pass 6 (xo 1, xf 2, yo 0, yf 2) merged with the staged passes
// 1-5 (`interlacing`, png/decoder.zig:59-67; mergePassInto :1289-1373;
// DevAdam7Merge): the pixel at even column x = 2X of even image row y.
struct A7Src {
    const uint8_t *q2, *s4, *s5;
    uint64_t q2stride, s4stride, s5stride;
    uint32_t width; // image pixels
};
template <int OBPX>
__device__ __forceinline__ const ZPX_GLOBAL uint8_t *a7_even(const A7Src &a, uint32_t X, uint32_t y)
{
    const uint8_t *p;
    if (y & 2) p = a.s5 + static_cast<uint64_t>((y - 2) >> 2) * a.s5stride + static_cast<uint64_t>(X) * OBPX;
    else if (X & 1) p = a.s4 + static_cast<uint64_t>(y >> 2) * a.s4stride + static_cast<uint64_t>(X >> 1) * OBPX;
    else p = a.q2 + static_cast<uint64_t>(y >> 2) * a.q2stride + static_cast<uint64_t>(X >> 1) * OBPX;
    return (const ZPX_GLOBAL uint8_t *)p;
}
// the staged pixels X = C k .. C k + C - 1 (C = 16 / OBPX) of even row y as
// two 8-byte loads, in X order
template <int OBPX>
__device__ __forceinline__ v4u a7_chunk(const A7Src &a, uint32_t k, uint32_t y)
{
    const uint32_t X0 = k * (16 / OBPX);
    const bool s5 = (y & 2) != 0;
    const uint64_t row = s5 ? (y - 2) >> 2 : y >> 2;
    const uint8_t *pa = s5 ? a.s5 + row * a.s5stride + static_cast<uint64_t>(X0) * OBPX
                           : a.q2 + row * a.q2stride + static_cast<uint64_t>(X0 >> 1) * OBPX;
    const uint8_t *pb = s5 ? pa + 8 : a.s4 + row * a.s4stride + static_cast<uint64_t>(X0 >> 1) * OBPX;
#if ZPX_A7_NOLOAD // (timing-only A/B: the merge without its staged loads; wrong pixels)
    (void)pa;
    (void)pb;
    const v2u va{k, y}, vb{y, k};
#elif ZPX_A7_NT
    const v2u va = __builtin_nontemporal_load(reinterpret_cast<const ZPX_GLOBAL v2u *>((const ZPX_GLOBAL uint8_t *)pa));
    const v2u vb = __builtin_nontemporal_load(reinterpret_cast<const ZPX_GLOBAL v2u *>((const ZPX_GLOBAL uint8_t *)pb));
#else
    const v2u va = *reinterpret_cast<const ZPX_GLOBAL v2u *>((const ZPX_GLOBAL uint8_t *)pa);
    const v2u vb = *reinterpret_cast<const ZPX_GLOBAL v2u *>((const ZPX_GLOBAL uint8_t *)pb);
#endif
    if constexpr (OBPX == 8) return v4u{va[0], va[1], vb[0], vb[1]};
    else return s5 ? v4u{va[0], va[1], vb[0], vb[1]} : v4u{va[0], vb[0], va[1], vb[1]}; // Q2 / S4 alternate
}
// one pixel's OBPX bytes (4 or 8) as dwords
template <int OBPX>
__device__ __forceinline__ v2u a7_load(const ZPX_GLOBAL uint8_t *src)
{
    if constexpr (OBPX == 8) return *reinterpret_cast<const ZPX_GLOBAL v2u *>(src);
    else return v2u{*reinterpret_cast<const ZPX_GLOBAL uint32_t *>(src), 0u};
}
template <int OBPX>
__device__ __forceinline__ void a7_store(gu8 *dst, v2u v)
{
    if constexpr (OBPX == 8) *gptr<v2u>(dst) = v;
    else *gptr<uint32_t>(dst) = v[0];
}
typedef __amdgpu_buffer_rsrc_t Rsrc;
__device__ __forceinline__ Rsrc make_rsrc(const void *base, uint32_t bytes)
{
    const uintptr_t a = reinterpret_cast<uintptr_t>(base);
    const uint64_t lo = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<uint32_t>(a)));
    const uint64_t hi = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<uint32_t>(a >> 32)));
    void *ua = reinterpret_cast<void *>(static_cast<uintptr_t>(hi << 32 | lo));
    return __builtin_amdgcn_make_buffer_rsrc(ua, 0, static_cast<int>(__builtin_amdgcn_readfirstlane(bytes)), 0x00020000);
}

__device__ __forceinline__ void wave_lds_sync()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Polls one window of boundary granules (lane l holds granules 2l, 2l+1 at
// offset o) until every granule the band reads carries `epoch`; bounded:
// past spin_limit polls (or once any wave has timed out: the status word)
// it sets the status word and gives up.  Out of line: the group loop's own
// loads keep exact s_waitcnt counts.
struct Polled {
    v4u w;
    uint32_t timed_out;
};
__device__ __noinline__ Polled poll_window(Rsrc rsrc, int o, int need, uint32_t epoch, uint32_t spin_limit,
                                           uint32_t *status)
{
    const int lane = threadIdx.x;
    v4u w = v4u{0, 0, 0, 0};
    for (uint32_t spins = 1;; spins++) {
        if (spins > spin_limit ||
            ((spins & 255) == 0 && __hip_atomic_load(status, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0)) {
            if (lane == 0) atomicOr(status, 1u);
            return Polled{w, 1u};
        }
        __builtin_amdgcn_s_sleep(kSleep);
        w = __builtin_amdgcn_raw_buffer_load_b128(rsrc, o, 0, 16 /* sc1 */);
        const bool ok = (2 * lane >= need || w[1] == epoch) && (2 * lane + 1 >= need || w[3] == epoch);
        if (__ballot(!ok) == 0) return Polled{w, 0u};
    }
}


// Cache policy of the boundary hand-off (agent scope, the data is the flag):
// sc1 on the loads and stores (MI355X_MICROARCH.md, inter-workgroup visibility)
constexpr int kSc1 = 16;
// the flush's whole-line stores: non-temporal (64 x 4K RGBA16 3.90 -> 3.84
// ms, tc8 1.78 -> 1.77 in an alternating A/B; a line the image never reads
// back need not stay in L2)
constexpr int kNt = 2;
// an offset every buffer access drops (stores) or reads as zero (loads)
constexpr int kOOR = 0x7ffffff0;

template <int DEPTH, bool TRNS, bool MERGE, bool STREAM>
__global__ __launch_bounds__(64)
__attribute__((amdgpu_waves_per_eu(PairShape<DEPTH, MERGE>::W, PairShape<DEPTH, MERGE>::W)))
void png_pair_kernel(const DevPngPass *__restrict__ passes, const DevPngBand *__restrict__ sched, uint32_t nsched,
                     uint32_t *ctl, uint64_t *boundary, uint32_t band_granules, uint32_t spin_limit)
{
    using T = PairTraits<DEPTH>;
    constexpr int BPP = T::BPP, CB = T::CB, CW = T::CW, C = T::C;
    constexpr int GD = kG * CW;             // input dwords per row per group
    constexpr int FL = PairShape<DEPTH, MERGE>::FL; // chunks per flushed block, steps between flushes
    constexpr int kSlots = 2 * FL;          // ring slots per row
    constexpr int RPR = 64 / FL;            // rows per flush round (FL lanes each)
    constexpr int NR = 128 / RPR;           // flush rounds
#ifndef ZPX_PNG_RING_SWZ
#define ZPX_PNG_RING_SWZ 1
#endif
    // ring dwords per row: 2 FL output chunks of 16 bytes (+ 16 bytes of
    // bank skew without the swizzle).  With ZPX_PNG_RING_SWZ rows start on
    // bank 0 and the rows 2j, 2j+1 of odd lanes j keep chunk k in slot
    // (k mod 16) xor 8: a flush read (ds_read_b128, 16-lane groups over 4
    // rows x 4 chunks, banks mod 64) then meets 4 disjoint 16-dword bank
    // sets, and the step's ring writes (ds_write_b128, 8-lane groups, banks
    // mod 32) spread with the rows' skews instead of colliding along a chain
    constexpr int RS = ZPX_PNG_RING_SWZ ? kSlots * 4 : kSlots * 4 + 4;
    auto rslot = [](int k, int row) {
        return ((k & (kSlots - 1)) ^ (ZPX_PNG_RING_SWZ ? (kSlots / 2) * ((row >> 1) & 1) : 0)) * 4;
    };
    constexpr int WG = kG * CW;             // boundary granules of one window (kG chunks)
    static_assert(WG % 2 == 0 && WG / 2 <= 64, "window loads are granule pairs, one per lane");
    __shared__ __attribute__((aligned(16))) uint32_t ring[128 * RS + 4]; // + a trash slot
    // flush state, [row % RPR][row / RPR]: the posted block (fst), and for
    // contiguous rows its chunks' output byte offset (fso, kOOR when none)
    // and ring byte offset (fsr), so that a flush round is two adds
    __shared__ __attribute__((aligned(16))) uint32_t fst[128];
    __shared__ __attribute__((aligned(16))) uint32_t fso[128];
    __shared__ __attribute__((aligned(16))) uint32_t fsr[128];
    // STREAM: the group's stream windows arrive in units (row half h, window
    // part u), each loaded with kSP consecutive lanes on one row's kSP
    // pieces (a row's bytes contiguous per lane group, ~11-16 rows per
    // instruction instead of 64) and turned round through this staging area
    // into the row-per-lane registers.  The whole window a unit (kWH 1) for
    // 12-byte chunks (6 KiB of staging: the wave's LDS is then 40,464 bytes,
    // four waves a CU); halves for 16-byte chunks (4 KiB)
    constexpr int kWH = CB == 12 ? 1 : 2; // window parts per unit row
    constexpr int kSP = (8 * CB / 16) / kWH; // pieces per row per unit (3, 4 or 6)
    __shared__ __attribute__((aligned(16))) uint32_t stage[STREAM ? 64 * kSP * 4 : 4];
    // per-lane LDS byte offsets: unit write of instruction i (lane-piece n =
    // 64 i + lane: row n / kSP, piece n % kSP), and the row-per-lane read of
    // piece p; a row's pieces are permuted so that a 16-lane ds_read_b128
    // group meets 64 distinct banks: xor row & 3 (4 a row), rotated by
    // row / 8 (6 a row: rows 24 dwords apart pair up 8 lanes apart)
    auto slot = [](int r, int pc) {
        return kSP == 4 ? (pc ^ (r & 3)) : kSP == 6 ? (pc + (r >> 3)) % 6 : pc;
    };
    uint32_t stw[kSP], str[kSP];
#pragma unroll
    for (int i = 0; i < kSP; i++) {
        const int n = 64 * i + static_cast<int>(threadIdx.x), r = n / kSP, pc = n % kSP;
        stw[i] = static_cast<uint32_t>((r * kSP + slot(r, pc)) * 16);
        const int j = static_cast<int>(threadIdx.x);
        str[i] = static_cast<uint32_t>((j * kSP + slot(j, i)) * 16);
    }
    constexpr int kTrash = 128 * RS;

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
        const DevPngPass ps = passes[bd.pass];
        const uint32_t rb = ps.row_bytes;
        // Adam7 pass 6 (the only strided pass this kernel takes), in the
        // instance of the group's second launch (MERGE): its registers stay
        // out of the other instances (pass 7 runs in the first launch)
        const bool merge = MERGE && ps.merge != nullptr;
        A7Src a7{};
        if (merge) {
            const DevAdam7Merge &m = *ps.merge;
            a7.q2 = m.q2;
            a7.s4 = m.s4;
            a7.s5 = m.s5;
            a7.q2stride = m.q2stride;
            a7.s4stride = m.s4stride;
            a7.s5stride = m.s5stride;
            a7.width = m.width;
        }
        const int nchunks = static_cast<int>(((rb + BPP - 1) / BPP + C - 1) / C);
        const int nfull = static_cast<int>(ps.width / C); // chunks whose pixels are all inside the row
        const uint32_t base = bd.band * 128;
        const uint32_t band_rows = min(128u, ps.rows - base);
        const bool ok0 = 2u * lane < band_rows, ok1 = 2u * lane + 1 < band_rows;
        // STREAM: the band's rows in the inflated stream (filter byte, then
        // rb bytes each); else the band's slab region (png_slab.cpp): its 128
        // filter bytes, then its groups, from the frame's band offset table
        // (scalar loads)
        const uint8_t *region;
        int ft0, ft1;
        if constexpr (STREAM) {
            region = ps.filtered + static_cast<size_t>(base) * (rb + 1);
            ft0 = ok0 ? region[static_cast<size_t>(2 * lane) * (rb + 1)] : 0;
            ft1 = ok1 ? region[static_cast<size_t>(2 * lane + 1) * (rb + 1)] : 0;
        } else {
            typedef const __attribute__((address_space(4))) uint64_t *CU64;
            region = ps.filtered +
                     *(reinterpret_cast<CU64>(reinterpret_cast<uintptr_t>(ps.filtered)) + ps.slab_band0 + bd.band);
            ft0 = region[2 * lane];
            ft1 = region[2 * lane + 1]; // (0 past the pass)
        }

        // skew over the band's 128 rows (row 2j = low half of lane j, 2j+1 high)
        const uint64_t R0 = __ballot(!(ft0 >= 2) || lane == 0 || !ok0);
        const uint64_t R1 = __ballot(!(ft1 >= 2) || !ok1);
        const uint64_t upto = lane == 63 ? ~0ull : ((2ull << lane) - 1), below = (1ull << lane) - 1;
        const int i0 = 63 - __builtin_clzll(R0 & upto); // R0 bit 0 is always set
        const int last0 = max(2 * i0, (R1 & below) ? 2 * (63 - __builtin_clzll(R1 & below)) + 1 : -1);
        const int last1 = max(2 * i0, (R1 & upto) ? 2 * (63 - __builtin_clzll(R1 & upto)) + 1 : -1);
        const int skew0 = 2 * lane - last0, skew1 = 2 * lane + 1 - last1;
        int max_skew = max(ok0 ? skew0 : 0, ok1 ? skew1 : 0);
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) max_skew = max(max_skew, __shfl_xor(max_skew, off));
        max_skew = __builtin_amdgcn_readfirstlane(max_skew);
        const int nsteps = nchunks + max_skew;

        PairFilter pf;
        {
            const PairFilter a = half_filter(ft0, 0), b = half_filter(ft1, 1);
            pf = PairFilter{a.keep | b.keep, a.force | b.force};
        }

        // band input: one descriptor from the dword below the band's first
        // byte over its rows + ZPX_PNG_INPUT_PAD.  The host routes passes with
        // rows shorter than a chunk to the one-row kernel, so no lane's group
        // ever starts before the descriptor (skew <= row index).
        // band input: the region's groups -- group g's 16-byte pieces at
        // 128 + ((2 g + h) NQ + q) KiB + 16 lane (piece q of row 2 lane + h's
        // bytes from chunk 8 g - skew on, zeros outside the row), so each
        // load instruction reads 1 KiB contiguous, and a row's chunks before
        // its first (k < 0) are zeros: it outputs zeros there, the zero
        // left / up / up-left its first chunk starts from.  The prefetch past
        // the last group reads out of range (zeros).
        //   STREAM: the rows' group windows (chunk 8 g - skew on) come
        // straight from the stream, unaligned 16-byte loads through the
        // staging area (load_units / xfer); the chunks before a row's first
        // read the rows above and are zeroed in registers (the group loop's
        // ramp), and
        // the bytes past a row's end are the next row's, which only the
        // row's own unstored tail bytes read.  The descriptor spans the
        // band's rows + ZPX_PNG_INPUT_PAD, so the prefetch past the last
        // group reads zeros.
        constexpr int NQ = 8 * CB / 16;
        static_assert(NQ * 4 == GD, "a group is NQ 16-byte pieces per row");
        const uint64_t extent = STREAM ? static_cast<uint64_t>(band_rows) * (rb + 1) + ZPX_PNG_INPUT_PAD
                                       : 128ull + static_cast<uint64_t>((nsteps + kG - 1) / kG) * 2 * NQ * 1024;
        const Rsrc in_rsrc = make_rsrc(region, extent > 0x7ffffff0ull ? 0x7ffffff0u : static_cast<uint32_t>(extent));
        const int soff0 = static_cast<int>(2 * lane * (rb + 1) + 1) - skew0 * CB; // row 2j's chunk 0 - skew0
        const int soff1 = static_cast<int>((2 * lane + 1) * (rb + 1) + 1) - skew1 * CB;
        // (STREAM) each unit load's lane offset: the row's window start +
        // its piece, per row half h and instruction i
        int voff[2][kSP];
        if constexpr (STREAM) {
#pragma unroll
            for (int i = 0; i < kSP; i++) {
                const int n = 64 * i + lane;
                voff[0][i] = __shfl(soff0, n / kSP) + 16 * (n % kSP);
                voff[1][i] = __shfl(soff1, n / kSP) + 16 * (n % kSP);
            }
        }

        // boundary hand-off: the previous band's last row (read by lanes
        // 0..WG/2-1, one granule pair each; offsets out of range otherwise)
        // and this band's last row (written by lane 63 only), both through
        // descriptors whose extent is zero when there is no such band
        const bool has_prev = bd.band > 0, has_next = bd.band + 1 < ps.nbands;
        const bool wait_prev = has_prev && (__ballot(ft0 >= 2) & 1ull) != 0; // row 0 reads the row above
        const uint32_t gbytes = band_granules * 8u;
        const Rsrc prev_rsrc = make_rsrc(boundary + static_cast<size_t>(ps.band_base + bd.band - (has_prev ? 1 : 0)) *
                                                        band_granules, wait_prev ? gbytes : 0u);
        const Rsrc next_rsrc = make_rsrc(boundary + static_cast<size_t>(ps.band_base + bd.band) * band_granules,
                                         has_next ? gbytes : 0u);

        // band output: rows base .. base+127 of the pass in the image
        const uint64_t orow_bytes = static_cast<uint64_t>(ps.yf) * ps.out_stride; // one pass row to the next
        gu8 *obase = (gu8 *)(ps.out + static_cast<size_t>(base * ps.yf + ps.yo) * ps.out_stride);
        const uint64_t oext = static_cast<uint64_t>(band_rows) * orow_bytes;
        const Rsrc out_rsrc = make_rsrc(reinterpret_cast<const void *>(reinterpret_cast<uintptr_t>(obase)),
                                        oext > 0x7ffffff0ull ? 0x7ffffff0u : static_cast<uint32_t>(oext));

        // per-row state: the previous step's output bytes of both rows (the
        // row above of the next step), and the last pixel's pairs
        uint32_t plo[CW], phi[CW], left[BPP], ul[BPP];
#pragma unroll
        for (int w = 0; w < CW; w++) plo[w] = phi[w] = 0;
#pragma unroll
        for (int i = 0; i < BPP; i++) left[i] = ul[i] = 0;
        int k0 = -skew0, k1 = -skew1; // chunk of the current step
        int fl0 = 0, fl1 = 0;         // blocks of 8 chunks flushed
        const int ring0 = (2 * lane) * RS, ring1 = ring0 + RS;

        // every buffer access of the group loop is unconditional (masked
        // lanes use out-of-range offsets), so the number of vector memory
        // instructions per group is fixed and s_waitcnt counts stay exact:
        // a group waits only for the loads issued one group earlier
        uint32_t A0[GD], A1[GD], B0[GD], B1[GD];
        // STREAM: the next group's units are loaded at the group's start and
        // turned round at steps 4-7 (4 units) or 4 and 6 (2).  64 x 4K, ms
        // (gpurun_out/sab, sab2, sa72, lds1, full1): tc8 2.38 with each lane
        // loading its own rows' pieces (64 rows an instruction, the two rows
        // alternating), 2.24 a row's pieces back to back, 2.21 with the
        // second row mid-group, 2.01 through this staging in half windows,
        // 1.98 in whole windows; Adam7 RGBA16 6.21, 5.68-5.91, 5.73-5.76,
        // 5.24 (halves); non-temporal loads 3.53 / 8.85, sc0 no change.
        v4u T[2][kWH][kSP]; // the next group's units: row half, window part, instruction
        auto load_units = [&](int g0) {
#pragma unroll
            for (int h = 0; h < 2; h++)
#pragma unroll
                for (int u = 0; u < kWH; u++)
#pragma unroll
                    for (int i = 0; i < kSP; i++) // (the whole offset in voffset: the
                        // range check leaves a raw buffer's soffset out, and past the
                        // band's last group these offsets must read zeros, not the
                        // bytes after the stream)
                        T[h][u][i] = __builtin_amdgcn_raw_buffer_load_b128(
                            in_rsrc, voff[h][i] + g0 * CB + 16 * kSP * u, 0, 0);
        };
        // unit (h, u) through the staging area into B0 / B1 (in order behind
        // the previous unit's reads: one wave's LDS instructions do not pass
        // each other)
        auto xfer = [&](uint32_t (&d)[GD], int h, int u) {
#pragma unroll
            for (int i = 0; i < kSP; i++)
                *reinterpret_cast<v4u *>(reinterpret_cast<uint8_t *>(stage) + stw[i]) = T[h][u][i];
            wave_lds_sync();
#pragma unroll
            for (int p = 0; p < kSP; p++) {
                const v4u v = *reinterpret_cast<const v4u *>(reinterpret_cast<const uint8_t *>(stage) + str[p]);
#pragma unroll
                for (int e = 0; e < 4; e++) d[4 * (u * kSP + p) + e] = v[e];
            }
            wave_lds_sync();
        };
        // the slab: each lane's two rows' group pieces, 1 KiB contiguous per instruction
        auto load_group = [&](uint32_t (&d0)[GD], uint32_t (&d1)[GD], int g0) {
            const int gb = 128 + (g0 / kG) * 2 * NQ * 1024 + lane * 16;
#pragma unroll
            for (int q = 0; q < NQ; q++) {
                const v4u a = __builtin_amdgcn_raw_buffer_load_b128(in_rsrc, gb + q * 1024, 0, 0);
                const v4u b = __builtin_amdgcn_raw_buffer_load_b128(in_rsrc, gb + (NQ + q) * 1024, 0, 0);
#pragma unroll
                for (int e = 0; e < 4; e++) {
                    d0[4 * q + e] = a[e];
                    d1[4 * q + e] = b[e];
                }
            }
        };
        // window of kG chunks of the previous band's last row: WG granules
        // {data, epoch}; lane l < WG/2 holds granules 2l, 2l+1 (one 16-byte
        // load), and each step hands its chunk's data dwords to lane 0's DPP
        // `old` operand through v_readlane (SGPRs)
        v4u W, Wn;
        auto load_window = [&](v4u &w, int g0) {
            const int o = 2 * lane < WG ? (g0 * CW + 2 * lane) * 8 : kOOR;
            w = __builtin_amdgcn_raw_buffer_load_b128(prev_rsrc, o, 0, kSc1);
        };

        // every FL steps: each row that completed an aligned block of FL full
        // chunks (FL = 8: one 128-byte line of RGBA8) posts it; in round i,
        // lanes FL g .. FL g + FL - 1 store row RPR i + g's posted block from
        // the ring, one chunk each
        auto flush = [&](int t_end) {
            const int d0 = ok0 ? min(max(t_end - skew0, 0), nchunks) : 0;
            const int d1 = ok1 ? min(max(t_end - skew1, 0), nchunks) : 0;
            const bool p0 = min(d0, nfull) / FL > fl0, p1 = min(d1, nfull) / FL > fl1;
            const int r0 = 2 * lane, r1 = r0 + 1; // row r's state at fst[(r % RPR) * NR + r / RPR]
            const int x0 = (r0 % RPR) * NR + r0 / RPR, x1 = (r1 % RPR) * NR + r1 / RPR;
            const bool xf1 = ps.xf == 1;
            if (xf1) {
                fso[x0] = p0 ? static_cast<uint32_t>(r0) * static_cast<uint32_t>(orow_bytes) + fl0 * (FL * 16) : kOOR;
                fso[x1] = p1 ? static_cast<uint32_t>(r1) * static_cast<uint32_t>(orow_bytes) + fl1 * (FL * 16) : kOOR;
                fsr[x0] = 4 * (ring0 + rslot(fl0 * FL, r0));
                fsr[x1] = 4 * (ring1 + rslot(fl1 * FL, r1));
            } else {
                fst[x0] = p0 ? static_cast<uint32_t>(fl0) : 0xffffu;
                fst[x1] = p1 ? static_cast<uint32_t>(fl1) : 0xffffu;
            }
            fl0 += p0 ? 1 : 0;
            fl1 += p1 ? 1 : 0;
            wave_lds_sync();
            if (xf1) { // contiguous rows: every round's ring read first, then the 16-byte stores
                uint32_t so[NR], sr[NR];
#pragma unroll
                for (int q = 0; q < NR / 4; q++) {
                    const v4u a = *reinterpret_cast<const v4u *>(&fso[(lane / FL) * NR + 4 * q]);
                    const v4u b = *reinterpret_cast<const v4u *>(&fsr[(lane / FL) * NR + 4 * q]);
#pragma unroll
                    for (int e = 0; e < 4; e++) {
                        so[4 * q + e] = a[e];
                        sr[4 * q + e] = b[e];
                    }
                }
                const uint32_t lo = (lane % FL) * 16u;
                v4u e[NR];
#pragma unroll
                for (int i = 0; i < NR; i++)
                    e[i] = *reinterpret_cast<const v4u *>(reinterpret_cast<const uint8_t *>(ring) + sr[i] + lo);
#pragma unroll
                for (int i = 0; i < NR; i++)
                    __builtin_amdgcn_raw_buffer_store_b128(e[i], out_rsrc, so[i] + lo, 0, kNt);
                return;
            }
            uint32_t blk[NR]; // this lane group's rows RPR i + g, i = 0..NR-1
#pragma unroll
            for (int q = 0; q < NR / 4; q++) {
                const v4u v = *reinterpret_cast<const v4u *>(&fst[(lane / FL) * NR + 4 * q]);
                blk[4 * q] = v[0];
                blk[4 * q + 1] = v[1];
                blk[4 * q + 2] = v[2];
                blk[4 * q + 3] = v[3];
            }
            auto round = [&](int i, auto &&store) __attribute__((always_inline)) {
                const int r = RPR * i + lane / FL;
                const bool post = blk[i] != 0xffffu;
                const int k = static_cast<int>(post ? blk[i] : 0u) * FL + lane % FL;
                const v4u v = *reinterpret_cast<const v4u *>(&ring[r * RS + rslot(k, r)]);
                store(post, r * static_cast<int>(orow_bytes), k, v);
            };
            if (!merge) { // Adam7 passes 1-4 into Q: pixels xf (2 or 4) apart
#pragma unroll
                for (int i = 0; i < NR; i++)
                    round(i, [&](bool post, int ro, int k, v4u v) {
#pragma unroll
                        for (int u = 0; u < C; u++) {
                            const int xo =
                                static_cast<int>((static_cast<uint32_t>(k * C + u) * ps.xf + ps.xo) * T::OBPX);
                            if constexpr (T::OBPX == 8)
                                __builtin_amdgcn_raw_buffer_store_b64(v2u{v[2 * u], v[2 * u + 1]}, out_rsrc,
                                                                      post ? ro + xo : kOOR, 0, 0);
                            else
                                __builtin_amdgcn_raw_buffer_store_b32(v[u], out_rsrc, post ? ro + xo : kOOR, 0, 0);
                        }
                    });
            } else if constexpr (MERGE) { // Adam7 pass 6: 32 contiguous bytes per lane, whole lines per lane group
                // every round's staged pixels first (two 8-byte loads each, in flight together), then the
                // stores.  (Issuing the loads one step before the stores -- a posted block's ring slots
                // survive that step -- measured no faster, 3.65 against 3.60 ms per second launch: the
                // launch moves 17.2 GB at ~4.8 TB/s, and the staged pixels' 2.15 GB of reads are its cost.)
                v4u e[NR];
#pragma unroll
                for (int i = 0; i < NR; i++) {
                    const int r = RPR * i + lane / FL;
                    const bool post = blk[i] != 0xffffu;
                    const uint32_t k = post ? blk[i] * FL + lane % FL : 0u;
                    const uint32_t y = post ? 2 * (base + r) : 0u; // (row 0, pixel 0: a valid address)
                    e[i] = a7_chunk<T::OBPX>(a7, k, y);
                }
#pragma unroll
                for (int i = 0; i < NR; i++)
                    round(i, [&](bool post, int ro, int k, v4u v) {
                        v4u lo, hi;
                        if constexpr (T::OBPX == 8) {
                            lo = v4u{e[i][0], e[i][1], v[0], v[1]};
                            hi = v4u{e[i][2], e[i][3], v[2], v[3]};
                        } else {
                            lo = v4u{e[i][0], v[0], e[i][1], v[1]};
                            hi = v4u{e[i][2], v[2], e[i][3], v[3]};
                        }
                        const int o = ro + k * 32;
                        __builtin_amdgcn_raw_buffer_store_b128(lo, out_rsrc, post ? o : kOOR, 0, kNt);
                        __builtin_amdgcn_raw_buffer_store_b128(hi, out_rsrc, post ? o + 16 : kOOR, 0, kNt);
                    });
            }
        };

        if constexpr (STREAM) {
            load_units(0);
#pragma unroll
            for (int u = 0; u < kWH; u++) xfer(B0, 0, u);
#pragma unroll
            for (int u = 0; u < kWH; u++) xfer(B1, 1, u);
        } else {
            load_group(B0, B1, 0);
        }
        load_window(Wn, 0);
        // A group waits for its inputs with s_waitcnt vmcnt(N), N = the
        // vector memory operations issued since them: the previous group's
        // publish stores (2 per step) and flush stores (16).  The first
        // group's N must agree (the count is static, merged over the loop
        // entry and back edge), so the same number of dropped stores follows
        // the first loads here.
        {
            const Rsrc none = make_rsrc(region, 0u); // extent 0: every store is dropped
#pragma unroll
            for (int i = 0; i < 2 * kG + (kG / FL) * NR; i++) // distinct, unmergeable offsets
                __builtin_amdgcn_raw_buffer_store_b32(0u, none, 4096 * i + lane * 4, 0, 0);
        }
        for (int g0 = 0; g0 < nsteps; g0 += kG) {
#pragma unroll
            for (int i = 0; i < GD; i++) {
                A0[i] = B0[i];
                A1[i] = B1[i];
            }
            W = Wn;
            if constexpr (STREAM) load_units(g0 + kG);
            else load_group(B0, B1, g0 + kG);
            load_window(Wn, g0 + kG);
            if constexpr (STREAM) {
                if (g0 < max_skew) { // the ramp: a row's chunks before its first are zeros
#pragma unroll
                    for (int i = 0; i < kG; i++) {
                        const bool z0 = g0 + i < skew0, z1 = g0 + i < skew1;
#pragma unroll
                        for (int w = 0; w < CW; w++) {
                            A0[i * CW + w] = z0 ? 0u : A0[i * CW + w];
                            A1[i * CW + w] = z1 ? 0u : A1[i * CW + w];
                        }
                    }
                }
            }
            if (wait_prev) {
                // the window must carry this launch's epoch in every granule
                // the band reads (chunks < nchunks); else poll
                const int need = min(kG, nchunks - g0) * CW; // granules the band reads
                const bool ok = (2 * lane >= need || W[1] == epoch) && (2 * lane + 1 >= need || W[3] == epoch);
                if (__ballot(!ok) != 0 && !timed_out) { // the producer is behind: poll (rare, out of line)
                    const int o = 2 * lane < WG ? (g0 * CW + 2 * lane) * 8 : kOOR;
                    const Polled pw = poll_window(prev_rsrc, o, need, epoch, spin_limit, status);
                    W = pw.w;
                    timed_out = pw.timed_out != 0;
                }
            }
#pragma unroll
            for (int st = 0; st < kG; st++) {
                if constexpr (STREAM && kWH == 2) { // the units of the next group, steps 4-7
                    if (st == 4) xfer(B0, 0, 0);
                    if (st == 5) xfer(B0, 0, 1);
                    if (st == 6) xfer(B1, 1, 0);
                    if (st == 7) xfer(B1, 1, 1);
                } else if constexpr (STREAM) { // steps 4 and 6
                    if (st == 4) xfer(B0, 0, 0);
                    if (st == 6) xfer(B1, 1, 0);
                }
                // ---- the row above, one step late: row 2j reads lane j-1's
                // high row (DPP wave_shr:1; lane 0's `old` is the previous
                // band's last row, zero without one), row 2j+1 its own low row
                uint32_t up[CB];
#pragma unroll
                for (int w = 0; w < CW; w++) {
                    const int gi = st * CW + w; // granule: lane gi/2, dword 0 or 2
                    const uint32_t old = static_cast<uint32_t>(
                        __builtin_amdgcn_readlane(static_cast<int>((gi & 1) ? W[2] : W[0]), gi >> 1));
                    const uint32_t dh = static_cast<uint32_t>(__builtin_amdgcn_update_dpp(
                        static_cast<int>(old), static_cast<int>(phi[w]), 0x138, 0xf, 0xf, false));
#pragma unroll
                    for (int b = 0; b < 4; b++)
                        up[4 * w + b] = __builtin_amdgcn_perm(dh, plo[w], 0x0c000c04u | static_cast<uint32_t>(b) << 16 |
                                                                             static_cast<uint32_t>(b));
                }
                // ---- filtered bytes of both rows' chunks, packed: the
                // slab interleaves the rows two bytes at a time, so dword m
                // of the group (A0: the first 2 CB, A1: the rest) is byte
                // pair 2k of the packed form as is, and shifted down a byte
                // pair 2k + 1 (bytes 1 and 3 left over: recon_pair's add
                // is per half)
                // (STREAM: A0 / A1 are the two rows' windows, one v_perm a
                // pair)
                uint32_t f[CB];
                if constexpr (STREAM) {
#pragma unroll
                    for (int w = 0; w < CW; w++)
#pragma unroll
                        for (int b = 0; b < 4; b++)
                            f[4 * w + b] = __builtin_amdgcn_perm(A1[st * CW + w], A0[st * CW + w],
                                                                 0x0c000c00u | (4u + b) << 16 | static_cast<uint32_t>(b));
                } else {
#pragma unroll
                    for (int k = 0; k < CB / 2; k++) {
                        const int m = st * (CB / 2) + k;
                        const uint32_t d = m < GD ? A0[m] : A1[m - GD];
                        f[2 * k] = d;
                        f[2 * k + 1] = d >> 8;
                    }
                }
                // ---- reconstruct CB byte pairs, left to right
                uint32_t o[CB];
#pragma unroll
                for (int i = 0; i < CB; i++) {
                    const uint32_t a = i < BPP ? left[i] : o[i < BPP ? 0 : i - BPP];
                    const uint32_t c = i < BPP ? ul[i] : up[i < BPP ? 0 : i - BPP];
                    o[i] = recon_pair(f[i], a, up[i], c, pf);
                }
#pragma unroll
                for (int i = 0; i < BPP; i++) {
                    left[i] = o[CB - BPP + i];
                    ul[i] = up[CB - BPP + i];
                }
                // ---- bytes of each row: the next step's row above, the
                // output chunk (ring slot, or the trash slot), the boundary
#pragma unroll
                for (int w = 0; w < CW; w++) {
                    const uint32_t x01 = __builtin_amdgcn_perm(o[4 * w + 1], o[4 * w], 0x06020400u);
                    const uint32_t x23 = __builtin_amdgcn_perm(o[4 * w + 3], o[4 * w + 2], 0x06020400u);
                    plo[w] = __builtin_amdgcn_perm(x23, x01, 0x05040100u);
                    phi[w] = __builtin_amdgcn_perm(x23, x01, 0x07060302u);
                }
                // (a chunk k < 0 lands in the slot of chunk k + 16, which
                // overwrites it before any flush reads it; past the row's end
                // the trash slot keeps its unflushed last chunks)
                *reinterpret_cast<v4u *>(&ring[k0 < nchunks ? ring0 + rslot(k0, 2 * lane) : kTrash]) =
                    expand_chunk<DEPTH, TRNS>(ps, plo);
                *reinterpret_cast<v4u *>(&ring[k1 < nchunks ? ring1 + rslot(k1, 2 * lane + 1) : kTrash]) =
                    expand_chunk<DEPTH, TRNS>(ps, phi);
                const bool act1 = ok1 && k1 >= 0 && k1 < nchunks;
                // ---- publish the band's last row (row 127: lane 63's high
                // half) as {data, epoch} granules: the data is the flag
                {
                    const int po = (lane == 63 && act1) ? k1 * CW * 8 : kOOR;
                    __builtin_amdgcn_raw_buffer_store_b128(v4u{phi[0], epoch, phi[1], epoch}, next_rsrc, po, 0, kSc1);
                    if constexpr (CW == 4)
                        __builtin_amdgcn_raw_buffer_store_b128(v4u{phi[2], epoch, phi[3], epoch}, next_rsrc, po + 16,
                                                               0, kSc1);
                    else
                        __builtin_amdgcn_raw_buffer_store_b64(v2u{phi[2], epoch}, next_rsrc, po + 16, 0, kSc1);
                }
                k0++;
                k1++;
                if ((st + 1) % FL == 0) { // (every FL steps; st is a constant of the unrolled loop)
                    wave_lds_sync();
                    flush(g0 + st + 1);
                    wave_lds_sync(); // fst is rewritten at the next flush
                }
            }
                }
        // ---- row tails: the last (< 2 FL) unflushed chunks, the last partial
        gu8 *out0 = obase + static_cast<size_t>(2 * lane) * orow_bytes;
        gu8 *out1 = out0 + orow_bytes;
        for (int h = 0; h < 2; h++) {
            const bool ok = h ? ok1 : ok0;
            if (!ok) continue;
            const int fl = h ? fl1 : fl0;
            gu8 *orow = h ? out1 : out0;
            const int rbase = h ? ring1 : ring0;
            if (merge) {
                // the row's last (< 16) chunks with their staged pixels, 4
                // chunks at a time (their loads in flight together), then an
                // odd width's last column, which is a staged pixel
                const uint32_t y = 2 * (base + 2 * lane + h);
                for (int k0 = fl * FL; k0 < nchunks; k0 += 4) {
                    v2u te[4][C];
#pragma unroll
                    for (int j = 0; j < 4; j++) {
                        const int k = k0 + j;
                        const int n = k < nfull ? C : static_cast<int>(ps.width) - k * C; // (<= 0 past the row)
#pragma unroll
                        for (int u = 0; u < C; u++)
                            te[j][u] = a7_load<T::OBPX>(a7_even<T::OBPX>(a7, u < n ? static_cast<uint32_t>(k * C + u) : 0u,
                                                                         u < n ? y : 0u));
                    }
#pragma unroll
                    for (int j = 0; j < 4; j++) {
                        const int k = k0 + j;
                        if (k >= nchunks) break;
                        const int n = k < nfull ? C : static_cast<int>(ps.width) - k * C;
                        const v4u v = *reinterpret_cast<const v4u *>(&ring[rbase + rslot(k, 2 * lane + h)]);
                        for (int u = 0; u < n; u++) {
                            gu8 *d = orow + static_cast<size_t>(2 * (k * C + u)) * T::OBPX;
                            a7_store<T::OBPX>(d, te[j][u]);
                            if constexpr (T::OBPX == 8) a7_store<8>(d + 8, v2u{v[2 * u], v[2 * u + 1]});
                            else a7_store<4>(d + 4, v2u{v[u], 0u});
                        }
                    }
                }
                if (a7.width & 1) {
                    const uint32_t p = ps.width;
                    a7_store<T::OBPX>(orow + static_cast<size_t>(2 * p) * T::OBPX,
                                      a7_load<T::OBPX>(a7_even<T::OBPX>(a7, p, y)));
                }
            } else {
                for (int k = fl * FL; k < nchunks; k++) {
                    const v4u v = *reinterpret_cast<const v4u *>(&ring[rbase + rslot(k, 2 * lane + h)]);
                    if (k < nfull && ps.xf == 1) put_chunk<DEPTH>(orow, k, v);
                    else put_partial<DEPTH>(ps, orow, k, v, k < nfull ? C : static_cast<int>(ps.width) - k * C);
                }
            }
        }
        wave_lds_sync();
    }
}

// Per-launch control block (as png_kernels.hip): the next epoch of the
// block's window, ticket = 0, the previous launch's status folded into the
// sticky word, status = 0.
__global__ void png_pair_ctl_kernel(uint32_t *ctl)
{
    ctl[0] = png_epoch_next(ctl[0], ctl[4], ctl[5]);
    ctl[1] = 0;
    ctl[3] |= ctl[2];
    ctl[2] = 0;
}

template <int DEPTH, bool TRNS, bool MERGE, bool STREAM>
void launch_pair_t(const DevPngPass *passes, const DevPngBand *sched, uint32_t nsched, uint32_t *ctl,
                   uint64_t *boundary, uint32_t band_granules, uint32_t spin_limit, hipStream_t s)
{
    // resident waves per CU from the occupancy API (one per instance: a
    // function-local static, initialised once even from concurrent threads)
    static const int per_cu = [] {
        int occ = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, png_pair_kernel<DEPTH, TRNS, MERGE, STREAM>, 64, 0) != hipSuccess ||
            occ < 1)
            occ = 4;
        return occ;
    }();
    const uint32_t want = static_cast<uint32_t>(device_cu_count() * per_cu);
    const uint32_t grid = nsched < want ? nsched : want;
    hipLaunchKernelGGL(png_pair_ctl_kernel, dim3(1), dim3(1), 0, s, ctl);
    hipLaunchKernelGGL((png_pair_kernel<DEPTH, TRNS, MERGE, STREAM>), dim3(grid), dim3(64), 0, s, passes, sched, nsched, ctl,
                       boundary, band_granules, spin_limit);
}

} // namespace


bool png_pair_supported(int depth, int interlace, bool use_trns, uint32_t width, uint64_t out_stride)
{
    int bpp = 0, cb = 16;
    switch (depth) {
    case ZPX_PNG_TC8: bpp = 3; cb = 12; break;
    case ZPX_PNG_TCA8: bpp = 4; break;
    case ZPX_PNG_TC16: bpp = 6; cb = 12; break;
    case ZPX_PNG_TCA16: bpp = 8; break;
    case ZPX_PNG_G8: bpp = 1; break;
    case ZPX_PNG_G16: bpp = 2; break;
    default: return false;
    }
    if ((depth == ZPX_PNG_G8 || depth == ZPX_PNG_G16) && (interlace || use_trns)) return false;
    if (interlace && width < 2) return false; // Adam7 here needs a pass 6 to merge the staged passes
    // every (non-empty) pass row holds at least one chunk's bytes (no lane's
    // group starts before the band), and a band's 128 pass rows of output
    // span less than the 2 GiB buffer range
    static const uint32_t kA7[7][2] = {{0, 8}, {4, 8}, {0, 4}, {2, 4}, {0, 2}, {1, 2}, {0, 1}}; // xo, xf
    uint32_t min_w = width;
    if (interlace)
        for (const auto &p : kA7) {
            const uint32_t w = ((width > p[0] ? width - p[0] : 0) + p[1] - 1) / p[1];
            if (w) min_w = w < min_w ? w : min_w;
        }
    if (uint64_t(min_w) * bpp + 1 < uint64_t(cb)) return false;
    const uint64_t yf = interlace ? 8 : 1;
    const uint64_t in_band = 128ull * (uint64_t(width) * bpp + 1) + ZPX_PNG_INPUT_PAD + 4;
    return in_band < 0x7ffffff0ull && 128ull * yf * out_stride < 0x7ffffff0ull;
}

namespace {
template <bool MERGE, bool STREAM>
int dispatch_pair(int depth, bool trns, const DevPngPass *passes, const DevPngBand *sched, uint32_t nsched,
                  uint32_t *ctl, uint64_t *boundary, uint32_t band_granules, uint32_t sl, hipStream_t s)
{
#define ZPX_PAIR(D, K) launch_pair_t<D, K, MERGE, STREAM>(passes, sched, nsched, ctl, boundary, band_granules, sl, s)
    switch (depth) {
    case ZPX_PNG_G8: if constexpr (!MERGE) { ZPX_PAIR(ZPX_PNG_G8, false); break; } else return -2;
    case ZPX_PNG_G16: if constexpr (!MERGE) { ZPX_PAIR(ZPX_PNG_G16, false); break; } else return -2;
    case ZPX_PNG_TCA8: ZPX_PAIR(ZPX_PNG_TCA8, false); break;
    case ZPX_PNG_TCA16: ZPX_PAIR(ZPX_PNG_TCA16, false); break;
    case ZPX_PNG_TC8: if (trns) ZPX_PAIR(ZPX_PNG_TC8, true); else ZPX_PAIR(ZPX_PNG_TC8, false); break;
    case ZPX_PNG_TC16: if (trns) ZPX_PAIR(ZPX_PNG_TC16, true); else ZPX_PAIR(ZPX_PNG_TC16, false); break;
    default: return -2; // (Gray8 / Gray16 are never interlaced on this kernel: png_pair_supported)
    }
#undef ZPX_PAIR
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
} // namespace

int launch_png_pair(int depth, bool trns, bool stream, const DevPngPass *passes, const DevPngBand *sched,
                    uint32_t nsched, uint32_t *ctl, uint64_t *boundary, uint32_t band_granules, hipStream_t s,
                    uint32_t spin_limit)
{
    const uint32_t sl = spin_limit ? spin_limit : png_default_spin_limit();
    return stream ? dispatch_pair<false, true>(depth, trns, passes, sched, nsched, ctl, boundary, band_granules, sl, s)
                  : dispatch_pair<false, false>(depth, trns, passes, sched, nsched, ctl, boundary, band_granules, sl, s);
}

int launch_png_pair_merge(int depth, bool trns, bool stream, const DevPngPass *passes, const DevPngBand *sched,
                          uint32_t nsched, uint32_t *ctl, uint64_t *boundary, uint32_t band_granules, hipStream_t s)
{
    const uint32_t sl = png_default_spin_limit();
    return stream ? dispatch_pair<true, true>(depth, trns, passes, sched, nsched, ctl, boundary, band_granules, sl, s)
                  : dispatch_pair<true, false>(depth, trns, passes, sched, nsched, ctl, boundary, band_granules, sl, s);
}

} // namespace zpx
