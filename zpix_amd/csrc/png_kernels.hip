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

#include "device_types.h"
#include "kernels.h"

namespace zpx {
namespace {

constexpr int kRegionChunks = 16;
constexpr uint32_t kSpinLimit = 1u << 24;

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

__device__ __forceinline__ uint32_t byte_of(const uint32_t *w, int i) { return (w[i >> 2] >> ((i & 3) * 8)) & 0xff; }

// Store n bytes held in dwords w[] to dst, using 16-byte stores when aligned.
template <int NB>
__device__ __forceinline__ void store_bytes(uint8_t *dst, const uint32_t (&w)[(NB + 3) / 4])
{
    const uintptr_t a = reinterpret_cast<uintptr_t>(dst);
    if constexpr (NB % 16 == 0) {
        if ((a & 15) == 0) {
#pragma unroll
            for (int i = 0; i < NB / 16; i++)
                reinterpret_cast<uint4 *>(dst)[i] = make_uint4(w[4 * i], w[4 * i + 1], w[4 * i + 2], w[4 * i + 3]);
            return;
        }
    }
    if constexpr (NB % 4 == 0) {
        if ((a & 3) == 0) {
#pragma unroll
            for (int i = 0; i < NB / 4; i++) reinterpret_cast<uint32_t *>(dst)[i] = w[i];
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
    uint8_t *row = ps.out + static_cast<size_t>(y * ps.yf + ps.yo) * ps.out_stride;
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
                uint8_t *d = row + static_cast<size_t>(x * ps.xf + ps.xo) * obpp;
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
            uint8_t *d = row + static_cast<size_t>(x * ps.xf + ps.xo) * obpp;
            if (obpp == 2) {
                d[0] = static_cast<uint8_t>(pix[u][0]);
                d[1] = static_cast<uint8_t>(pix[u][0] >> 8);
            } else if (obpp == 4) {
                if ((reinterpret_cast<uintptr_t>(d) & 3) == 0) *reinterpret_cast<uint32_t *>(d) = pix[u][0];
                else for (int i = 0; i < 4; i++) d[i] = static_cast<uint8_t>(pix[u][0] >> (8 * i));
            } else {
                if ((reinterpret_cast<uintptr_t>(d) & 7) == 0) {
                    *reinterpret_cast<uint2 *>(d) = make_uint2(pix[u][0], pix[u][1]);
                } else {
                    for (int i = 0; i < 4; i++) d[i] = static_cast<uint8_t>(pix[u][0] >> (8 * i));
                    for (int i = 0; i < 4; i++) d[4 + i] = static_cast<uint8_t>(pix[u][1] >> (8 * i));
                }
            }
        }
    }
}

__device__ __forceinline__ uint64_t ld_sc1_64(const uint64_t *p)
{
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
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

template <int DEPTH>
__global__ __launch_bounds__(64) void png_unfilter_kernel(const DevPngPass *__restrict__ passes,
                                                          const DevPngBand *__restrict__ sched, uint32_t nsched,
                                                          uint32_t *ctl, uint64_t *boundary, uint32_t band_granules)
{
    using Tr = Traits<DEPTH>;
    constexpr int BPP = Tr::kBpp, C = Tr::kC, CW = Tr::kCW;
    constexpr int WIN = kRegionChunks;          // chunks per window
    constexpr int WG = WIN * CW;                // granules per window (<= 64)
    static_assert(WG <= 64, "window must fit one granule per lane");
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
        const uint8_t *frow = ps.filtered + static_cast<size_t>(y) * (rb + 1);
        const int ft = row_ok ? frow[0] : 0;
        const LaneFilter lf{ft == 1, ft == 2, ft == 3, ft == 4};
        const uint32_t mis = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(frow + 1) & 3);
        const uint32_t *src = reinterpret_cast<const uint32_t *>(frow + 1 - mis);

        const bool has_prev = bd.band > 0;
        const bool has_next = bd.band + 1 < ps.nbands;
        const uint64_t *prev_bnd =
            boundary + static_cast<size_t>(ps.band_base + bd.band - (has_prev ? 1 : 0)) * band_granules;
        uint64_t *my_bnd = boundary + static_cast<size_t>(ps.band_base + bd.band) * band_granules;

        uint32_t left[BPP], ul[BPP];
#pragma unroll
        for (int i = 0; i < BPP; i++) left[i] = ul[i] = 0;
        uint32_t outp[CW];
#pragma unroll
        for (int i = 0; i < CW; i++) outp[i] = 0;
        uint32_t carry = 0;
        uint64_t win = 0, win_next = 0;
        int maxidx = 0;

        auto load_window = [&](int w0) -> uint64_t {
            const int k = w0 + lane / CW;
            return (lane < WG && k < nchunks) ? ld_sc1_64(prev_bnd + static_cast<size_t>(w0) * CW + lane) : 0ull;
        };
        if (has_prev) win = load_window(0);

        const uint32_t band_rows = min(64u, ps.rows - bd.band * 64);
        const int nsteps = nchunks + static_cast<int>(band_rows) - 1;
        for (int step = 0; step < nsteps; ++step) {
            const int k = step - lane;
            const bool act = row_ok && k >= 0 && k < nchunks;

            // ---- the row above: chunk k of row y-1 was produced by lane-1 one step ago
            uint32_t up[CW];
#pragma unroll
            for (int i = 0; i < CW; i++)
                up[i] = __builtin_amdgcn_update_dpp(0, static_cast<int>(outp[i]), 0x138, 0xf, 0xf, false);
            if (has_prev && step < nchunks) { // lane 0: chunk `step` of the previous band's last row
                const int wi = step % WIN;
                if (wi == 0 && step > 0) win = win_next;
                if (wi == WIN / 2 && step + WIN / 2 < nchunks) win_next = load_window(step + WIN / 2);
                const int base = wi * CW;
                uint32_t spins = 0;
                for (;;) {
                    bool ready = true;
#pragma unroll
                    for (int i = 0; i < CW; i++) {
                        const uint32_t hi = __builtin_amdgcn_readlane(static_cast<int>(win >> 32), base + i);
                        ready &= hi == epoch;
                    }
                    if (ready) break;
                    if (++spins > kSpinLimit) {
                        timed_out = true;
                        break;
                    }
                    __builtin_amdgcn_s_sleep(1);
                    if (lane >= base && lane < base + CW)
                        win = ld_sc1_64(prev_bnd + static_cast<size_t>(step - wi) * CW + lane);
                }
#pragma unroll
                for (int i = 0; i < CW; i++) {
                    const uint32_t v = __builtin_amdgcn_readlane(static_cast<int>(win), base + i);
                    if (lane == 0) up[i] = v;
                }
            } else if (lane == 0) {
#pragma unroll
                for (int i = 0; i < CW; i++) up[i] = 0; // first row of a pass: zero previous row (:790-793)
            }

            if (act) {
                // ---- filtered bytes of chunk k (dword window + funnel shift)
                if (k == 0) carry = src[0];
                uint32_t in[CW + 1];
                in[0] = carry;
#pragma unroll
                for (int i = 1; i <= CW; i++) in[i] = src[k * CW + i];
                carry = in[CW];
                uint32_t f[CW];
#pragma unroll
                for (int i = 0; i < CW; i++) f[i] = __builtin_amdgcn_alignbyte(in[i + 1], in[i], mis);
                if (k == 0) {
#pragma unroll
                    for (int i = 0; i < BPP; i++) left[i] = ul[i] = 0;
                }
                // ---- reconstruct C units, left to right
                uint32_t ob[CW];
#pragma unroll
                for (int i = 0; i < CW; i++) ob[i] = 0;
                uint32_t prev_out[BPP], prev_up[BPP];
#pragma unroll
                for (int i = 0; i < BPP; i++) {
                    prev_out[i] = left[i];
                    prev_up[i] = ul[i];
                }
#pragma unroll
                for (int u = 0; u < C; u++) {
#pragma unroll
                    for (int i = 0; i < BPP; i++) {
                        const int idx = u * BPP + i;
                        const uint32_t b = byte_of(up, idx);
                        const uint32_t v = recon_byte(lf, byte_of(f, idx), prev_out[i], b, prev_up[i]);
                        ob[idx >> 2] |= v << ((idx & 3) * 8);
                        prev_out[i] = v;
                        prev_up[i] = b;
                    }
                }
#pragma unroll
                for (int i = 0; i < BPP; i++) {
                    left[i] = prev_out[i];
                    ul[i] = prev_up[i];
                }
#pragma unroll
                for (int i = 0; i < CW; i++) outp[i] = ob[i];

                store_chunk<DEPTH>(ps, y, static_cast<uint32_t>(k * C), ob, maxidx);

                if (has_next && lane == 63) { // publish: the data is the flag
                    uint64_t *d = my_bnd + static_cast<size_t>(k) * CW;
#pragma unroll
                    for (int i = 0; i < CW; i++) st_sc1_64(d + i, static_cast<uint64_t>(epoch) << 32 | ob[i]);
                }
            }
        }
        if constexpr (DEPTH >= ZPX_PNG_P1 && DEPTH <= ZPX_PNG_P8) {
            for (int off = 32; off > 0; off >>= 1) maxidx = max(maxidx, __shfl_xor(maxidx, off));
            if (lane == 0 && ps.max_index) atomicMax(ps.max_index, maxidx);
        }
    }
    if (timed_out && lane == 0) atomicOr(status, 1u);
}

// Per-launch control block: epoch++ (fresh granule tags, so the boundary
// buffer never needs clearing), ticket = 0, status = 0.
__global__ void png_ctl_kernel(uint32_t *ctl)
{
    ctl[0] += 1;
    ctl[1] = 0;
    ctl[2] = 0;
}

int png_waves_per_cu()
{
    static int n = 0;
    if (n == 0) {
        const char *e = getenv("ZPX_PNG_WAVES_PER_CU");
        n = e ? atoi(e) : 8;
        if (n < 1) n = 1;
        if (n > 32) n = 32;
    }
    return n;
}

int cus()
{
    static int n = 0;
    if (n == 0) {
        int dev = 0, c = 256;
        if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev);
        n = c;
    }
    return n;
}

template <int DEPTH>
void launch_t(const DevPngPass *passes, const DevPngBand *sched, uint32_t nsched, uint32_t *ctl, uint64_t *boundary,
              uint32_t band_granules, hipStream_t s)
{
    const uint32_t want = static_cast<uint32_t>(cus() * png_waves_per_cu());
    const uint32_t grid = nsched < want ? nsched : want;
    hipLaunchKernelGGL(png_ctl_kernel, dim3(1), dim3(1), 0, s, ctl);
    hipLaunchKernelGGL((png_unfilter_kernel<DEPTH>), dim3(grid), dim3(64), 0, s, passes, sched, nsched, ctl, boundary,
                       band_granules);
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
                        uint32_t *ctl, uint64_t *boundary, uint32_t band_granules, hipStream_t s)
{
    switch (depth) {
#define ZPX_CASE(D) case D: launch_t<D>(passes, sched, nsched, ctl, boundary, band_granules, s); break;
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
