// gfx950 QOI encoder: qoi.encode (src/qoi/encoder.zig:29-132) as a
// data-parallel pipeline whose output is byte-identical to the serial loop.
//
// The serial encoder carries two pieces of state from pixel to pixel: the
// current run length and the 64-entry index table.  Both are prefix functions
// of the pixel stream, so they scan:
//   - index[h] before pixel i is the last NON-RUN pixel j < i with hash h (a run
//     pixel equals its predecessor, so it never changes the table, and a table
//     hit leaves the table as it was), or zero when there is none;
//   - the run length before pixel i is the number of consecutive pixels equal
//     to their predecessor that end at i-1, modulo 62 (a run chunk is emitted
//     and the count reset every 62 pixels).
// The pixels are cut into segments of S pixels, one segment per lane and one
// block of 64 segments per wave:
//   1. qoi_summary_kernel: per segment, the last non-run pixel per hash (+ a
//      64-bit presence mask) and the run summary (all-run flag, trailing run);
//      per block, the same folded over its 64 segments;
//   2. qoi_block_scan_kernel: one workgroup scans the block summaries into
//      exclusive per-block prefixes (table + run length);
//   3. qoi_encode_kernel: each lane rebuilds its segment's incoming state from
//      the block prefix and the segments below it in the wave (ballot +
//      ds_bpermute), then runs the reference loop over its S pixels into a
//      private scratch slot (at most 5*S+1 bytes), dword stores;
//   4. qoi_offsets_kernel: one workgroup scans the per-block byte counts and
//      writes the header, the total length and the 8-byte end marker;
//   5. qoi_compact_kernel: each workgroup gathers its block's 64 slots into
//      the final byte stream (aligned dword stores).
// Tables are stored hash-major ([64][nseg]) so that every pass reads and
// writes them with whole-wave coalesced accesses.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "kernels.h"

namespace zpx {
namespace {

constexpr uint32_t kInit = 0xff000000u; // px_prev = {0,0,0,255} (encoder.zig:65)

__device__ __forceinline__ uint32_t qhash(uint32_t p)
{
    return ((p & 0xff) * 3 + (p >> 8 & 0xff) * 5 + (p >> 16 & 0xff) * 7 + (p >> 24) * 11) & 63;
}

// pixel i of an RGB(A) buffer as r | g<<8 | b<<16 | a<<24 (a = 255 for RGB)
template <int CH> __device__ __forceinline__ uint32_t load_px(const uint8_t *px, uint64_t i)
{
    if constexpr (CH == 4) {
        return *reinterpret_cast<const uint32_t *>(px + 4 * i);
    } else {
        const uint8_t *p = px + 3 * i;
        return p[0] | uint32_t(p[1]) << 8 | uint32_t(p[2]) << 16 | kInit;
    }
}

constexpr int kGroup = 16; // pixels per load group of one lane (64 B of RGBA)

// kGroup consecutive pixels starting at i (16-byte aligned, all < n)
template <int CH> __device__ __forceinline__ void load_group(const uint8_t *px, uint64_t i, uint32_t o[kGroup])
{
    const uint4 *v = reinterpret_cast<const uint4 *>(px + CH * i);
    uint32_t w[kGroup * CH / 4 + 1];
#pragma unroll
    for (int k = 0; k < kGroup * CH / 16; k++) {
        const uint4 t = v[k];
        w[4 * k] = t.x;
        w[4 * k + 1] = t.y;
        w[4 * k + 2] = t.z;
        w[4 * k + 3] = t.w;
    }
    if constexpr (CH == 4) {
#pragma unroll
        for (int j = 0; j < kGroup; j++) o[j] = w[j];
    } else {
        w[kGroup * 3 / 4] = 0;
#pragma unroll
        for (int j = 0; j < kGroup; j++)
            o[j] = (__builtin_amdgcn_alignbyte(w[3 * j / 4 + 1], w[3 * j / 4], (3 * j) % 4) & 0xffffffu) | kInit;
    }
}

// Calls f(p, i) for the pixels [start, end) of one lane: whole groups with the
// next two groups' loads in flight (a lane's work is a serial chain, so the
// wave cannot hide a load behind other work of its own; a group spans whole
// 64-byte pieces, so each line is fetched once per lane), then the tail.
// Prefetch addresses are clamped to the lane's last whole group.
template <int CH, typename F>
__device__ __forceinline__ void for_pixels(const uint8_t *px, uint64_t start, uint64_t end, F &&f)
{
    uint64_t i = start;
    const bool vec = (reinterpret_cast<uintptr_t>(px) & 15) == 0 && (start % kGroup) == 0;
    if (vec && start + kGroup <= end) {
        const uint64_t last = end - kGroup - (end - start) % kGroup;
        uint32_t q0[kGroup], q1[kGroup], q2[kGroup];
        load_group<CH>(px, i, q0);
        load_group<CH>(px, min(i + kGroup, last), q1);
        for (; i + kGroup <= end; i += kGroup) {
            load_group<CH>(px, min(i + 2 * kGroup, last), q2);
#pragma unroll
            for (int j = 0; j < kGroup; j++) f(q0[j], i + j);
#pragma unroll
            for (int j = 0; j < kGroup; j++) {
                q0[j] = q1[j];
                q1[j] = q2[j];
            }
        }
    }
    for (; i < end; i++) f(load_px<CH>(px, i), i);
}

__device__ __forceinline__ uint64_t lanes_below(uint32_t lane) { return (uint64_t(1) << lane) - 1; }
__device__ __forceinline__ int top_lane(uint64_t m) { return 63 - __builtin_clzll(m); }

template <typename T> __device__ __forceinline__ T bperm(T v, int src_lane)
{
    return static_cast<T>(__builtin_amdgcn_ds_bpermute(src_lane * 4, static_cast<int>(v)));
}

// A run summary (segment or block) is trail | all_run << 31: applied to the
// incoming run length c it gives all_run ? c + len : trail.

template <int CH>
__global__ __launch_bounds__(64) void qoi_summary_kernel(const uint8_t *__restrict__ px, uint64_t n, uint32_t S,
                                                         uint32_t nseg, uint32_t *__restrict__ seg_tbl,
                                                         uint64_t *__restrict__ seg_mask,
                                                         uint32_t *__restrict__ seg_run,
                                                         uint32_t *__restrict__ blk_tbl,
                                                         uint64_t *__restrict__ blk_mask,
                                                         uint32_t *__restrict__ blk_run)
{
    __shared__ uint32_t tbl[64][64]; // [hash][lane]: bank = lane, conflict-free
    const uint32_t lane = threadIdx.x, b = blockIdx.x, s = b * 64 + lane;
    const uint64_t start = min(n, uint64_t(s) * S), end = min(n, start + S);
    uint32_t prev = start > 0 ? load_px<CH>(px, start - 1) : kInit;
    uint64_t mask = 0;
    uint32_t trail = 0, all_run = 1;
    for_pixels<CH>(px, start, end, [&](uint32_t p, uint64_t) __attribute__((always_inline)) {
        // branch-free: a run pixel's write lands in an entry its mask bit does
        // not cover (or rewrites the value already there), so it is harmless
        const bool same = p == prev;
        const uint32_t h = qhash(p);
        tbl[h][lane] = p;
        mask |= same ? 0 : uint64_t(1) << h;
        trail = same ? trail + 1 : 0;
        all_run &= same;
        prev = p;
    });
    if (s < nseg) {
        seg_mask[s] = mask;
        seg_run[s] = trail | all_run << 31;
    }
    // every lane reads only its own table column; the block fold crosses lanes
    // through readlane on registers
    uint32_t agg = 0;
    uint64_t agg_mask = 0;
    for (uint32_t h = 0; h < 64; h++) {
        const uint32_t v = tbl[h][lane];
        if (s < nseg) seg_tbl[uint64_t(h) * nseg + s] = v;
        const uint64_t has = __ballot(mask >> h & 1);
        if (has) {
            const uint32_t last = __builtin_amdgcn_readlane(v, top_lane(has));
            if (lane == h) agg = last;
            agg_mask |= uint64_t(1) << h;
        }
    }
    blk_tbl[uint64_t(lane) * gridDim.x + b] = agg; // hash-major [64][nblk]
    const uint64_t broken = __ballot(!all_run);
    if (lane == 0) {
        blk_mask[b] = agg_mask;
        const uint64_t bstart = min(n, uint64_t(b) * 64 * S), bend = min(n, bstart + uint64_t(64) * S);
        uint32_t r;
        if (!broken) {
            r = uint32_t(bend - bstart) | 1u << 31;
        } else {
            const int k = top_lane(broken);
            const uint64_t kend = min(n, (uint64_t(b) * 64 + k + 1) * S);
            r = (__builtin_amdgcn_readlane(trail, k) + uint32_t(bend - kend));
        }
        blk_run[b] = r;
    }
}

// One workgroup of 16 waves: exclusive prefix over the block summaries.  A
// wave takes 64 blocks at a time, one per lane; per hash, ballot finds the
// blocks that wrote the entry and readlane / ds_bpermute move the values, so
// no loop carries a memory latency per block.
__global__ __launch_bounds__(1024) void qoi_block_scan_kernel(uint64_t n, uint32_t S, uint32_t nblk,
                                                              const uint32_t *__restrict__ blk_tbl,
                                                              const uint64_t *__restrict__ blk_mask,
                                                              const uint32_t *__restrict__ blk_run,
                                                              uint32_t *__restrict__ pre_tbl,
                                                              uint32_t *__restrict__ pre_run)
{
    __shared__ uint32_t w_val[16][64];
    __shared__ uint32_t w_has[16][64];
    __shared__ uint32_t w_run[16][3]; // all_run, trail, len
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint32_t nchunk = (nblk + 63) / 64, per = (nchunk + 15) / 16;
    const uint32_t c0 = min(nchunk, w * per), c1 = min(nchunk, c0 + per);
    const uint64_t bpx = uint64_t(64) * S;
    auto bend = [&](uint64_t b) __attribute__((always_inline)) { return min(n, (b + 1) * bpx); };
    auto bstart = [&](uint64_t b) __attribute__((always_inline)) { return min(n, b * bpx); };
    const uint64_t below = lanes_below(lane);

    // 1. fold this wave's chunks: lane h ends with the last value of hash h
    uint32_t val = 0, has = 0, all_run = 1, trail = 0;
    for (uint32_t c = c0; c < c1; c++) {
        const uint32_t b = c * 64 + lane;
        const bool live = b < nblk;
        const uint64_t m = live ? blk_mask[b] : 0;
        const uint32_t r = live ? blk_run[b] : 1u << 31;
        uint32_t v[64];
        const uint32_t bl = min(b, nblk - 1); // dead lanes load a live entry, masked out by m = 0
#pragma unroll
        for (int h = 0; h < 64; h++) v[h] = blk_tbl[uint64_t(h) * nblk + bl];
#pragma unroll
        for (int h = 0; h < 64; h++) {
            const uint64_t bits = __ballot(m >> h & 1);
            if (bits) {
                const uint32_t last = __builtin_amdgcn_readlane(v[h], top_lane(bits));
                if (lane == uint32_t(h)) {
                    val = last;
                    has = 1;
                }
            }
        }
        const uint64_t broken = __ballot(!(r >> 31));
        if (broken) {
            const int k = top_lane(broken);
            trail = __builtin_amdgcn_readlane(r, k) + uint32_t(bend(uint64_t(c) * 64 + 63) - bend(uint64_t(c) * 64 + k));
            all_run = 0;
        } else {
            trail += uint32_t(bend(uint64_t(c) * 64 + 63) - bstart(uint64_t(c) * 64));
        }
    }
    w_val[w][lane] = val;
    w_has[w][lane] = has;
    if (lane == 0) {
        w_run[w][0] = all_run;
        w_run[w][1] = trail;
        w_run[w][2] = uint32_t(bend(uint64_t(c1) * 64 - 1) - bstart(uint64_t(c0) * 64));
    }
    __syncthreads();
    // 2. exclusive prefix of the waves below (lane h: hash h)
    uint32_t carry_v = 0, carry_c = 0;
    for (uint32_t k = 0; k < w; k++) {
        if (w_has[k][lane]) carry_v = w_val[k][lane];
        carry_c = w_run[k][0] ? carry_c + w_run[k][2] : w_run[k][1];
    }
    // 3. rescan the chunks writing per-block exclusive prefixes
    for (uint32_t c = c0; c < c1; c++) {
        const uint32_t b = c * 64 + lane;
        const bool live = b < nblk;
        const uint64_t m = live ? blk_mask[b] : 0;
        const uint32_t r = live ? blk_run[b] : 1u << 31;
        uint32_t v[64];
        const uint32_t bl = min(b, nblk - 1); // dead lanes load a live entry, masked out by m = 0
#pragma unroll
        for (int h = 0; h < 64; h++) v[h] = blk_tbl[uint64_t(h) * nblk + bl];
        uint32_t next_v = carry_v;
#pragma unroll
        for (int h = 0; h < 64; h++) {
            const uint64_t bits = __ballot(m >> h & 1);
            const uint64_t lower = bits & below;
            const uint32_t from = bperm(v[h], lower ? top_lane(lower) : 0);
            const uint32_t in_h = __builtin_amdgcn_readlane(carry_v, h);
            if (live) pre_tbl[uint64_t(h) * nblk + b] = lower ? from : in_h;
            if (bits) {
                const uint32_t last = __builtin_amdgcn_readlane(v[h], top_lane(bits));
                if (lane == uint32_t(h)) next_v = last;
            }
        }
        carry_v = next_v;
        const uint64_t brk = __ballot(!(r >> 31));
        const uint64_t lower = brk & below;
        const int k = lower ? top_lane(lower) : 0;
        const uint32_t k_trail = bperm(r & 0x7fffffffu, k);
        const uint32_t cin = lower ? k_trail + uint32_t(bstart(b) - bend(uint64_t(c) * 64 + k))
                                   : carry_c + uint32_t(bstart(b) - bstart(uint64_t(c) * 64));
        if (live) pre_run[b] = cin;
        if (brk) {
            const int kk = top_lane(brk);
            carry_c = __builtin_amdgcn_readlane(r, kk) + uint32_t(bend(uint64_t(c) * 64 + 63) - bend(uint64_t(c) * 64 + kk));
        } else {
            carry_c += uint32_t(bend(uint64_t(c) * 64 + 63) - bstart(uint64_t(c) * 64));
        }
    }
}

// Byte queue of one lane: < 4 bytes pending in acc between calls, whole
// dwords staged in four registers and stored 16 bytes at a time (the slot is
// 16-byte aligned and has a spare 16 bytes).
struct ByteOut {
    uint4 *slot;
    uint32_t words = 0, pend = 0;
    uint64_t acc = 0;
    uint32_t w0 = 0, w1 = 0, w2 = 0, w3 = 0;
    __device__ __forceinline__ void push(uint32_t v)
    {
        const uint32_t k = words & 3;
        w0 = k == 0 ? v : w0;
        w1 = k == 1 ? v : w1;
        w2 = k == 2 ? v : w2;
        w3 = k == 3 ? v : w3;
        words++;
        if ((words & 3) == 0) slot[(words >> 2) - 1] = make_uint4(w0, w1, w2, w3);
    }
    __device__ __forceinline__ void put(uint64_t bytes, uint32_t nb)
    {
        acc |= (bytes & ((uint64_t(1) << (8 * nb)) - 1)) << (8 * pend);
        pend += nb;
        if (pend >= 4) {
            push(uint32_t(acc));
            acc >>= 32;
            pend -= 4;
            if (pend >= 4) {
                push(uint32_t(acc));
                acc >>= 32;
                pend -= 4;
            }
        }
    }
    __device__ __forceinline__ uint32_t finish()
    {
        const uint32_t n = 4 * words + pend;
        if (pend) push(uint32_t(acc));
        if (words & 3) slot[words >> 2] = make_uint4(w0, w1, w2, w3);
        return n;
    }
};

template <int CH>
__global__ __launch_bounds__(64) void qoi_encode_kernel(const uint8_t *__restrict__ px, uint64_t n, uint32_t S,
                                                        uint32_t nseg, uint32_t slot_words,
                                                        const uint32_t *__restrict__ seg_tbl,
                                                        const uint64_t *__restrict__ seg_mask,
                                                        const uint32_t *__restrict__ seg_run,
                                                        const uint32_t *__restrict__ pre_tbl,
                                                        const uint32_t *__restrict__ pre_run,
                                                        uint32_t *__restrict__ slots, uint32_t *__restrict__ seg_cnt,
                                                        uint64_t *__restrict__ blk_cnt)
{
    __shared__ uint32_t tbl[64][64]; // [hash][lane]
    const uint32_t lane = threadIdx.x, b = blockIdx.x, s = b * 64 + lane;
    const bool live = s < nseg;
    const uint64_t below = lanes_below(lane);
    const uint64_t mask = live ? seg_mask[s] : 0;
    // incoming index table: the nearest segment below in this block that wrote
    // the entry, else the block prefix
    {
        uint32_t v[64], pre[64];
        const uint32_t sl = min(s, nseg - 1), nblk = gridDim.x; // dead lanes load a live slot, masked out
#pragma unroll
        for (int h = 0; h < 64; h++) v[h] = seg_tbl[uint64_t(h) * nseg + sl];
#pragma unroll
        for (int h = 0; h < 64; h++) pre[h] = pre_tbl[uint64_t(h) * nblk + b];
#pragma unroll
        for (int h = 0; h < 64; h++) {
            const uint64_t lower = __ballot(mask >> h & 1) & below;
            const uint32_t from = bperm(v[h], lower ? top_lane(lower) : 0);
            tbl[h][lane] = lower ? from : pre[h];
        }
    }
    // incoming run length
    const uint64_t start = min(n, uint64_t(s) * S), end = min(n, start + S);
    const uint32_t r = live ? seg_run[s] : 1u << 31;
    const uint64_t lower = __ballot(!(r >> 31)) & below;
    const int k = lower ? top_lane(lower) : 0;
    const uint32_t k_trail = bperm(r & 0x7fffffffu, k);
    uint32_t c;
    if (lower) {
        const uint64_t kend = min(n, (uint64_t(b) * 64 + k + 1) * S);
        c = k_trail + uint32_t(start - kend);
    } else {
        c = pre_run[b] + uint32_t(start - min(n, uint64_t(b) * 64 * S));
    }
    uint32_t run = c % 62;

    ByteOut out{reinterpret_cast<uint4 *>(slots + uint64_t(s) * slot_words)};
    uint32_t prev = start > 0 ? load_px<CH>(px, start - 1) : kInit;
    for_pixels<CH>(px, start, end, [&](uint32_t p, uint64_t i) __attribute__((always_inline)) {
        // encoder.zig:70-124 with selects instead of branches (lanes would
        // otherwise serialise over the six chunk kinds)
        const bool same = p == prev;
        const uint32_t run1 = run + 1;
        const bool run_out = same ? (run1 == 62 || i + 1 == n) : run > 0; // QOI_OP_RUN now
        out.put(0xc0 | ((same ? run1 : run) - 1), run_out ? 1 : 0);
        run = same && !run_out ? run1 : 0;
        const uint32_t h = qhash(p), t = tbl[h][lane];
        const bool hit = t == p;
        tbl[h][lane] = same || hit ? t : p; // index[h] = px on a miss (:95)
        const int vr = int(p & 0xff) - int(prev & 0xff);
        const int vg = int(p >> 8 & 0xff) - int(prev >> 8 & 0xff);
        const int vb = int(p >> 16 & 0xff) - int(prev >> 16 & 0xff);
        const int vgr = vr - vg, vgb = vb - vg;
        const bool a_same = (p >> 24) == (prev >> 24);
        const bool diff = vr > -3 && vr < 2 && vg > -3 && vg < 2 && vb > -3 && vb < 2;
        const bool luma = vgr > -9 && vgr < 8 && vg > -33 && vg < 32 && vgb > -9 && vgb < 8;
        const uint32_t diff_b = 0x40 | (vr + 2) << 4 | (vg + 2) << 2 | (vb + 2);
        const uint32_t luma_b = (0x80 | (vg + 32)) | ((vgr + 8) << 4 | (vgb + 8)) << 8;
        const uint64_t rgb_b = 0xfe | uint64_t(p & 0xffffff) << 8, rgba_b = 0xff | uint64_t(p) << 8;
        uint64_t op = a_same ? (diff ? diff_b : luma ? luma_b : rgb_b) : rgba_b;
        uint32_t nb = a_same ? (diff ? 1 : luma ? 2 : 4) : 5;
        op = hit ? h : op;
        nb = same ? 0 : hit ? 1 : nb;
        out.put(op, nb);
        prev = p;
    });
    const uint32_t cnt = out.finish();
    if (live) seg_cnt[s] = cnt;
    uint64_t sum = live ? cnt : 0;
    for (int off = 32; off > 0; off >>= 1) sum += __shfl_xor(sum, off);
    if (lane == 0) blk_cnt[b] = sum;
}

// One workgroup: exclusive scan of the per-block byte counts; header, total
// length and end marker.
__global__ __launch_bounds__(1024) void qoi_offsets_kernel(uint32_t nblk, const uint64_t *__restrict__ blk_cnt,
                                                           uint64_t *__restrict__ blk_off, uint8_t *__restrict__ out,
                                                           uint64_t *__restrict__ out_len, uint32_t width,
                                                           uint32_t height, uint32_t channels, uint32_t colorspace)
{
    __shared__ uint64_t w_sum[16];
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint32_t per = ((nblk + 15) / 16 + 63) / 64 * 64, b0 = min(nblk, w * per), b1 = min(nblk, b0 + per);
    uint64_t tot = 0;
    for (uint32_t b = b0 + lane; b < b1; b += 64) tot += blk_cnt[b];
    for (int off = 32; off > 0; off >>= 1) tot += __shfl_xor(tot, off);
    if (lane == 0) w_sum[w] = tot;
    __syncthreads();
    uint64_t base = 0, all = 0;
    for (uint32_t k = 0; k < 16; k++) {
        if (k < w) base += w_sum[k];
        all += w_sum[k];
    }
    for (uint32_t b = b0; b < b1; b += 64) {
        const uint64_t v = b + lane < b1 ? blk_cnt[b + lane] : 0;
        uint64_t inc = v; // inclusive wave scan
        for (int off = 1; off < 64; off <<= 1) {
            const uint64_t t = __shfl_up(inc, off);
            if (lane >= uint32_t(off)) inc += t;
        }
        if (b + lane < b1) blk_off[b + lane] = base + inc - v;
        base += __shfl(inc, 63);
    }
    if (threadIdx.x == 0) {
        *out_len = 14 + all + 8;
        const uint32_t hdr[3] = {0x716F6966u, width, height};
        for (int i = 0; i < 3; i++)
            for (int j = 0; j < 4; j++) out[4 * i + j] = static_cast<uint8_t>(hdr[i] >> (24 - 8 * j));
        out[12] = static_cast<uint8_t>(channels);
        out[13] = static_cast<uint8_t>(colorspace);
    }
    if (threadIdx.x < 8) out[14 + all + threadIdx.x] = threadIdx.x == 7 ? 1 : 0; // QOI_PADDING
}

// One workgroup per block: the block's 64 slots are one contiguous run of
// output bytes at out + 14 + blk_off[b].  Each wave copies 16 of the slots:
// the aligned destination dwords of a slot take two aligned source loads and
// an alignbyte per lane (256 bytes per wave instruction); the at most 3 + 3
// bytes at its ends, which share dwords with the neighbouring slots, are
// stored bytewise.
__global__ __launch_bounds__(256) void qoi_compact_kernel(uint32_t nseg, uint32_t slot_words,
                                                          const uint32_t *__restrict__ slots,
                                                          const uint32_t *__restrict__ seg_cnt,
                                                          const uint64_t *__restrict__ blk_off,
                                                          uint8_t *__restrict__ out)
{
    __shared__ uint32_t offs[65];
    const uint32_t b = blockIdx.x, t = threadIdx.x, lane = t & 63, w = t >> 6;
    if (t < 64) {
        const uint32_t s = b * 64 + t;
        const uint32_t cnt = s < nseg ? seg_cnt[s] : 0;
        uint32_t inc = cnt;
        for (int off = 1; off < 64; off <<= 1) {
            const uint32_t x = __shfl_up(inc, off);
            if (t >= uint32_t(off)) inc += x;
        }
        offs[t + 1] = inc;
        if (t == 0) offs[0] = 0;
    }
    __syncthreads();
    const uintptr_t base = reinterpret_cast<uintptr_t>(out) + 14 + blk_off[b];
    for (uint32_t k = w; k < 64; k += 4) {
        const uint32_t o0 = offs[k], cnt = offs[k + 1] - o0;
        if (!cnt) continue;
        const uint8_t *src = reinterpret_cast<const uint8_t *>(slots + uint64_t(b * 64 + k) * slot_words);
        const uintptr_t d = base + o0, e = d + cnt;
        const uintptr_t qa = (d + 3) & ~uintptr_t(3), qb = e & ~uintptr_t(3);
        if (qb > qa) {
            for (uintptr_t q = qa + 4 * uintptr_t(lane); q < qb; q += 4 * 64) {
                const uintptr_t sa = reinterpret_cast<uintptr_t>(src) + (q - d);
                const uint32_t *sw = reinterpret_cast<const uint32_t *>(sa & ~uintptr_t(3));
                *reinterpret_cast<uint32_t *>(q) = __builtin_amdgcn_alignbyte(sw[1], sw[0], static_cast<uint32_t>(sa & 3));
            }
        }
        // head [d, min(qa, e)) and tail [max(qa, qb), e): at most 3 bytes each
        const uintptr_t head_end = qa < e ? qa : e, tail_start = qb > qa ? qb : qa;
        if (lane < 3) {
            const uintptr_t x = d + lane;
            if (x < head_end) *reinterpret_cast<uint8_t *>(x) = src[x - d];
        } else if (lane < 6) {
            const uintptr_t x = tail_start + (lane - 3);
            if (x < e && x >= head_end) *reinterpret_cast<uint8_t *>(x) = src[x - d];
        }
    }
}

template <int CH>
int launch_qoi_t(const QoiEncodeArgs &a, hipStream_t st)
{
    const uint32_t nblk = (a.nseg + 63) / 64;
    hipLaunchKernelGGL((qoi_summary_kernel<CH>), dim3(nblk), dim3(64), 0, st, a.pixels, a.n, a.S, a.nseg, a.seg_tbl,
                       a.seg_mask, a.seg_run, a.blk_tbl, a.blk_mask, a.blk_run);
    hipLaunchKernelGGL(qoi_block_scan_kernel, dim3(1), dim3(1024), 0, st, a.n, a.S, nblk, a.blk_tbl, a.blk_mask,
                       a.blk_run, a.pre_tbl, a.pre_run);
    hipLaunchKernelGGL((qoi_encode_kernel<CH>), dim3(nblk), dim3(64), 0, st, a.pixels, a.n, a.S, a.nseg,
                       a.slot_words, a.seg_tbl, a.seg_mask, a.seg_run, a.pre_tbl, a.pre_run, a.slots, a.seg_cnt,
                       a.blk_cnt);
    hipLaunchKernelGGL(qoi_offsets_kernel, dim3(1), dim3(1024), 0, st, nblk, a.blk_cnt, a.blk_off, a.out, a.out_len,
                       a.width, a.height, uint32_t(CH), a.colorspace);
    hipLaunchKernelGGL(qoi_compact_kernel, dim3(nblk), dim3(256), 0, st, a.nseg, a.slot_words, a.slots, a.seg_cnt,
                       a.blk_off, a.out);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

} // namespace

size_t qoi_scratch_layout(uint64_t n, uint32_t S, QoiEncodeArgs *a, uint8_t *base)
{
    const uint32_t nseg = static_cast<uint32_t>((n + S - 1) / S), nblk = (nseg + 63) / 64;
    const uint32_t slot_words = ((5 * S + 1 + 3) / 4 + 4 + 3) & ~3u; // 16-byte slots with a spare 16 bytes
    size_t off = 0;
    auto take = [&](size_t bytes) {
        const size_t o = off;
        off = (off + bytes + 255) & ~size_t(255);
        return base ? base + o : nullptr;
    };
    uint8_t *seg_tbl = take(size_t(64) * nseg * 4), *seg_mask = take(size_t(nseg) * 8),
            *seg_run = take(size_t(nseg) * 4), *seg_cnt = take(size_t(nseg) * 4),
            *blk_tbl = take(size_t(nblk) * 256), *blk_mask = take(size_t(nblk) * 8),
            *blk_run = take(size_t(nblk) * 4), *pre_tbl = take(size_t(nblk) * 256),
            *pre_run = take(size_t(nblk) * 4), *blk_cnt = take(size_t(nblk) * 8), *blk_off = take(size_t(nblk) * 8),
            *slots = take(size_t(nblk) * 64 * slot_words * 4);
    if (a) {
        a->n = n;
        a->S = S;
        a->nseg = nseg;
        a->slot_words = slot_words;
        a->seg_tbl = reinterpret_cast<uint32_t *>(seg_tbl);
        a->seg_mask = reinterpret_cast<uint64_t *>(seg_mask);
        a->seg_run = reinterpret_cast<uint32_t *>(seg_run);
        a->seg_cnt = reinterpret_cast<uint32_t *>(seg_cnt);
        a->blk_tbl = reinterpret_cast<uint32_t *>(blk_tbl);
        a->blk_mask = reinterpret_cast<uint64_t *>(blk_mask);
        a->blk_run = reinterpret_cast<uint32_t *>(blk_run);
        a->pre_tbl = reinterpret_cast<uint32_t *>(pre_tbl);
        a->pre_run = reinterpret_cast<uint32_t *>(pre_run);
        a->blk_cnt = reinterpret_cast<uint64_t *>(blk_cnt);
        a->blk_off = reinterpret_cast<uint64_t *>(blk_off);
        a->slots = reinterpret_cast<uint32_t *>(slots);
    }
    return off;
}

int launch_qoi_encode(int channels, const QoiEncodeArgs &a, hipStream_t st)
{
    if (a.n == 0 || a.nseg == 0) return -2;
    return channels == 4 ? launch_qoi_t<4>(a, st) : channels == 3 ? launch_qoi_t<3>(a, st) : -2;
}

} // namespace zpx
