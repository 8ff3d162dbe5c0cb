// Internals shared by the C-ABI translation units (zpx_api.cpp, batch.cpp):
// the context, HIP error reporting, device buffers and allocator helpers.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <mutex>
#include <string>
#include <vector>

#include "zpix_amd.h"
#include "device_types.h"
#include "kernels.h"
#include "options.h"

struct zpx_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    std::string last_error;
    // grow-only device scratch for stream-ordered work that needs no host
    // round trip (the QOI encoder's tables and slots), on `stream` or a
    // caller stream: every user takes scratch_mu while it enqueues, makes
    // its stream wait for scratch_ev (the previous user's work), and
    // records scratch_ev after its own, so uses on different streams run
    // one after the other on the device
    void *scratch = nullptr;
    size_t scratch_bytes = 0;
    hipEvent_t scratch_ev = nullptr;
    std::mutex scratch_mu;
};

namespace zpx {

inline int hip_fail(zpx_ctx *ctx, hipError_t e, const char *what)
{
    if (ctx) {
        char buf[256];
        snprintf(buf, sizeof(buf), "%s: %s", what, hipGetErrorString(e));
        ctx->last_error = buf;
    }
    return ZPX_E_HIP;
}

#define HIPCHK(ctx, call)                                                      \
    do {                                                                       \
        hipError_t e_ = (call);                                                \
        if (e_ != hipSuccess) return ::zpx::hip_fail((ctx), e_, #call);        \
    } while (0)

// Device buffer (RAII).
struct DevBuf {
    void *ptr = nullptr;
    size_t bytes = 0;
    DevBuf() = default;
    DevBuf(const DevBuf &) = delete;
    DevBuf &operator=(const DevBuf &) = delete;
    ~DevBuf() { release(); }
    void release()
    {
        if (ptr) (void)hipFree(ptr);
        ptr = nullptr;
        bytes = 0;
    }
    hipError_t alloc(size_t n)
    {
        release();
        bytes = n ? n : 1;
        return hipMalloc(&ptr, bytes);
    }
    // grow-only: keeps the buffer when it is already large enough
    hipError_t reserve(size_t n)
    {
        if (ptr && bytes >= n) return hipSuccess;
        return alloc(n);
    }
    template <typename T> T *as() const { return static_cast<T *>(ptr); }
};

inline void *al_alloc(const zpx_allocator *al, size_t n)
{
    if (al && al->alloc) return al->alloc(al->user, n ? n : 1);
    return malloc(n ? n : 1);
}
inline void al_free(const zpx_allocator *al, void *p, size_t n)
{
    if (!p) return;
    if (al && al->free) al->free(al->user, p, n);
    else free(p);
}

// Runs an entry point's body so that no C++ exception crosses the C-ABI
// (include/zpix_amd.h: "No exception or abort crosses the ABI").
template <typename F> int guarded(F &&f) noexcept
{
    try {
        return f();
    } catch (...) {
        return ZPX_E_OUT_OF_MEMORY;
    }
}

inline int read_file(const char *path, std::vector<uint8_t> &out)
{
    FILE *f = fopen(path, "rb");
    if (!f) return ZPX_E_FILE_NOT_FOUND;
    fseek(f, 0, SEEK_END);
    long n = ftell(f);
    fseek(f, 0, SEEK_SET);
    if (n < 0) {
        fclose(f);
        return ZPX_E_READ_FAILED;
    }
    out.resize(static_cast<size_t>(n));
    size_t got = n ? fread(out.data(), 1, static_cast<size_t>(n), f) : 0;
    fclose(f);
    return got == static_cast<size_t>(n) ? 0 : ZPX_E_READ_FAILED;
}

// ctx->scratch grown to at least n bytes (synchronises the device only when it grows)
inline hipError_t ctx_scratch(zpx_ctx *ctx, size_t n)
{
    if (ctx->scratch && ctx->scratch_bytes >= n) return hipSuccess;
    if (ctx->scratch) {
        hipError_t e = hipDeviceSynchronize();
        if (e != hipSuccess) return e;
        (void)hipFree(ctx->scratch);
        ctx->scratch = nullptr;
        ctx->scratch_bytes = 0;
    }
    hipError_t e = hipMalloc(&ctx->scratch, n ? n : 1);
    if (e == hipSuccess) ctx->scratch_bytes = n;
    else ctx->scratch = nullptr;
    return e;
}

struct CtxScope { // make ctx->device current for this call
    explicit CtxScope(zpx_ctx *c) { (void)hipSetDevice(c->device); }
};

struct JpegCoeffs;
struct HostBuf;
struct DevJpegFrame;
struct DevPngPass;
struct DevImage;

// zpx_batch_decode_rgba with a completion hook: on_done(user, i) runs on the
// pipeline's dispatcher thread as soon as item i's status is final and its
// result is complete in dst (the slot's last event has completed) -- what
// the sharded gather and zpx_batch_wait_prefix post their transfers on.
typedef void (*BatchDone)(void *user, int item);
int batch_decode_rgba_hook(zpx_ctx *ctx, zpx_batch_item *items, int n_items, const zpx_batch_opts *opts,
                           zpx_batch_stats *stats, BatchDone on_done, void *user);

// batch.cpp: frees the batch pipeline's cached slots (zpx_batch_cache_trim);
// returns their device bytes
size_t batch_slot_cache_trim();

// shard.cpp: destroy the cached gather communicators that include `device`
// (zpx_ctx_destroy); a call still gathering on one finishes first
void shard_release_comms(int device);

// zpx_api.cpp helpers shared with the batch pipeline
void jpeg_fill_frame(const JpegCoeffs &c, zpx_jpeg_frame *f, size_t *coeff_bytes);
DevJpegFrame dev_jpeg_frame(const zpx_jpeg_frame &f);
JpegPlaneGeom jpeg_plane_geom(const DevJpegFrame &d); // the planar kernel geometry of one frame
bool jpeg_fusable(const zpx_jpeg_frame &f); // the fused RGBA kernel takes this frame
int launch_jpeg_rgba_frame(const zpx_jpeg_frame &f, const DevJpegFrame *d_frame, hipStream_t st);
// dword-aligned RGBA rows, any width (the block-per-lane kernel takes it)
bool jpeg_rgba_vec_out(const zpx_jpeg_frame &f);
void png_frame_passes(const zpx_png_frame &f, std::vector<DevPngPass> &passes, std::vector<uint32_t> &rowbytes,
                      uint64_t &bytes);
// Band slab (png_slab.cpp) of a frame whose `filtered` is the HOST stream:
// the region offset of every band (returned size = slab bytes), then the fill.
size_t png_slab_layout(const zpx_png_frame &f, std::vector<uint64_t> &band_off);
void png_slab_fill(const zpx_png_frame &f, const std::vector<uint64_t> &band_off, uint8_t *out, int threads = 1);
// The same layout built on the device from the stream (png_slab_kernels.hip):
// region sizes for the largest possible skew (min(127, rows - 1)), so the
// layout follows from the frame's geometry alone and the host never reads the
// filtered bytes.  png_dev_slab_layout returns the slab bytes and every band's
// region offset (the slab's leading table, which the caller copies to the
// slab's start); png_dev_slab_jobs appends one DevSlabBand per band for the
// DEVICE stream `d_stream` (`stream_len` readable bytes, pad included) and
// slab `d_slab`; the largest group count of those bands goes to max_groups.
size_t png_dev_slab_layout(const zpx_png_frame &f, std::vector<uint64_t> &band_off);
void png_dev_slab_jobs(const zpx_png_frame &f, const std::vector<uint64_t> &band_off, const uint8_t *d_stream,
                       size_t stream_len, uint8_t *d_slab, std::vector<DevSlabBand> &jobs, uint32_t &max_groups);
int png_slab_chunk_bytes(int depth); // CB of the paired-row kernel (12 or 16; 0: not one it takes)
DevImage dev_image_of(const zpx_image *img, const void *d_pixels, const void *d_palette);
// planes + colour pass for frames the fused kernel does not take (async on st)
int jpeg_planes_to_rgba(zpx_ctx *ctx, const JpegCoeffs &c, zpx_jpeg_frame f, DevBuf &planes, DevBuf &desc,
                        HostBuf &hdesc, uint8_t *out, hipStream_t st);

// PNG control block of a plan group or batch slot (device_types.h layout:
// {epoch, ticket, status, sticky, base, cycle, 0, 0}) and the epoch window
// it owns.  Boundary granules carry the epoch of the launch that wrote them;
// a band accepts a granule only when it carries its own launch's epoch.  So
// a launch's epoch must differ from every tag its boundary buffer may hold:
//   - windows: every live block owns a window of its own (a process-wide
//     registry, handed out round robin from a per-process start and
//     returned when the block is destroyed), so two blocks never share an
//     epoch -- a destroyed block's buffer handed out again at the same
//     address holds tags of another window;
//   - cycle: a block's launches take base + 1 .. base + cycle - 1 in turn
//     (png_epoch_next: never 0, never base).  Before the launches that would
//     wrap the cycle, prepare() clears the boundary buffer and re-bases the
//     epoch on the launch stream, so a granule left from any earlier launch
//     -- a slot's previous image of another geometry, a timed-out launch --
//     holds a tag no later launch of this cycle uses.  (Launches the host
//     does not issue -- a captured graph replayed -- wrap on the device
//     without the clear; a plan's launches rewrite every granule they read,
//     so its granules hold the previous launch's epoch, never the next.)
// The cycle is kPngEpochWindow (2^20 launches) unless the test switch
// "png_epoch_cycle" sets a shorter one (>= 4).
uint32_t png_epoch_window_acquire(const void *owner); // 0: every window is taken
bool png_epoch_window_release(uint32_t window, const void *owner);
bool png_epoch_window_owned(uint32_t window, const void *owner);
// The launches that would wrap: the control kernel's next `launches` epochs
// from `shadow` leave the cycle (host mirror of png_epoch_next).
inline bool png_epoch_wraps(uint32_t shadow, uint32_t base, uint32_t cycle, int launches)
{
    for (int i = 0; i < launches; i++) {
        const uint32_t e = png_epoch_next(shadow, base, cycle);
        if (e <= shadow) return true;
        shadow = e;
    }
    return false;
}
class PngControl {
  public:
    PngControl() = default;
    PngControl(const PngControl &) = delete;
    PngControl &operator=(const PngControl &) = delete;
    ~PngControl();
    // Takes a window and allocates + initialises the block on the current
    // device (synchronously).  ZPX_E_OUT_OF_MEMORY when all 4095 windows
    // belong to live blocks.
    int init(zpx_ctx *ctx);
    // Before enqueueing `launches` control-kernel launches on `st`: checks
    // that the block still owns its window (ZPX_E_PANIC otherwise) and, when
    // one of them would wrap the cycle, clears `boundary` (bytes) and resets
    // the epoch to base on `st` first.
    int prepare(zpx_ctx *ctx, int launches, void *boundary, size_t bytes, hipStream_t st);
    uint32_t *words() const { return ctl_.as<uint32_t>(); }
    uint32_t window() const { return window_; }
    uint32_t wraps() const { return wraps_; } // re-bases so far (tests)

  private:
    DevBuf ctl_;
    uint32_t window_ = 0, base_ = 0, cycle_ = 0, shadow_ = 0, wraps_ = 0;
};

// The unfilter kernel addresses one band (64 filtered rows + the input pad)
// through a buffer descriptor with a 31-bit byte range, and row offsets in
// 32-bit registers: a pass whose band would exceed it is rejected
// (ZPX_E_UNSUPPORTED) instead of silently reading zeros past 2 GiB.
inline bool png_band_fits(uint32_t max_row_bytes, uint32_t band_rows = 128)
{
    return uint64_t(band_rows) * (uint64_t(max_row_bytes) + 1) + ZPX_PNG_INPUT_PAD + 4 < 0x7ffffff0ull;
}

// PNG band schedule (the ticket order of png_unfilter_kernel / png_pair_kernel).
// Longest bands first (LPT: a band's steps are its row's chunks), then by band
// index, then pass: band b of a pass still precedes band b+1 of it (the
// kernels' no-deadlock rule: a band's predecessor holds a lower ticket, so it
// is running or done).  With Adam7 the bands differ 8x in length (pass 1: 512
// pixels a row, pass 7: 4096); in output-row order the last tickets are the
// bottom bands of passes 6-7, and every wave but those idles for up to 2048
// steps (simulated over 64 x 4K RGBA16: makespan 5,160 steps against 4,096 of
// work a wave; longest-first: 4,372; measured 8.12 -> 7.79 ms).  Without
// interlacing both are band-major order.
inline std::vector<DevPngBand> png_schedule(const std::vector<DevPngPass> &passes, uint32_t band_rows)
{
    constexpr bool row_order = false; // (output-row order: measured slower, see above)
    std::vector<DevPngBand> sched;
    std::vector<uint64_t> key;
    for (size_t i = 0; i < passes.size(); i++)
        for (uint32_t b = 0; b < passes[i].nbands; b++) {
            sched.push_back(DevPngBand{static_cast<uint32_t>(i), b});
            key.push_back(row_order ? static_cast<uint64_t>(b) * band_rows * passes[i].yf + passes[i].yo
                                    : (static_cast<uint64_t>(0xffffffffu - passes[i].row_bytes) << 32) | b);
        }
    std::vector<size_t> idx(sched.size());
    for (size_t i = 0; i < idx.size(); i++) idx[i] = i;
    std::stable_sort(idx.begin(), idx.end(), [&](size_t a, size_t b) { return key[a] < key[b]; });
    std::vector<DevPngBand> out(sched.size());
    for (size_t i = 0; i < idx.size(); i++) out[i] = sched[idx[i]];
    return out;
}

// The device-side band layout of a group of PNG passes of one depth: the
// kernel that takes them (the paired-row kernel with 128-row bands, or the
// one-row-per-lane kernel with 64-row bands), each pass's band count and
// first band, the ticket schedule, and the boundary granules per band.
struct PngBandPlan {
    bool pair = false;
    uint32_t band_rows = 64, nbands = 0, granules = 0, max_rb = 0;
    std::vector<DevPngBand> sched;  // first launch: every band but the Adam7 merge passes'
    std::vector<DevPngBand> sched2; // second launch: pass 6 of Adam7 images (merging the staged 1-5)
};
int png_band_granules(int depth, uint32_t max_row_bytes);      // kernels.h
bool png_pair_supported(int depth, int interlace, bool use_trns, uint32_t width, uint64_t out_stride); // kernels.h
// Which kernel takes a PNG image: the paired-row kernel wherever it
// supports the depth (the test switch "png_pair" = 0 forces the
// one-row-per-lane kernel).
inline bool png_use_pair(int depth, int interlace, bool use_trns, uint32_t width, uint64_t out_stride)
{
    return opt(Opt::PngPair) && png_pair_supported(depth, interlace, use_trns, width, out_stride);
}
inline PngBandPlan png_plan_bands(int depth, bool pair, std::vector<DevPngPass> &passes,
                                  const std::vector<uint32_t> &rowbytes)
{
    PngBandPlan b;
    b.pair = pair;
    b.band_rows = pair ? 128 : 64;
    for (size_t i = 0; i < passes.size(); i++) {
        DevPngPass &p = passes[i];
        p.nbands = (p.rows + b.band_rows - 1) / b.band_rows;
        p.band_base = b.nbands;
        b.nbands += p.nbands;
        b.max_rb = std::max(b.max_rb, rowbytes[i]);
    }
    b.sched = png_schedule(passes, b.band_rows);
    b.granules = static_cast<uint32_t>(png_band_granules(depth, b.max_rb));
    // Adam7 pass 6 reads the staged passes 1-5: it runs in a second launch
    // (band order within a pass is kept by the stable partition).  Pass 7
    // (the odd rows, no dependency on the staging) runs in the first launch,
    // its long bands first beside passes 1-5's short ones: 64 x 4K RGBA16
    // 5.26 -> 5.10 ms, RGBA8 3.00 -> 2.92 against pass 7 beside pass 6 in
    // the second launch (gpurun_out/r05_a7, two rounds each).
    const auto merge_band = [&](const DevPngBand &d) { return passes[d.pass].launch2 != 0; };
    std::stable_partition(b.sched.begin(), b.sched.end(), [&](const DevPngBand &d) { return !merge_band(d); });
    const auto cut = std::find_if(b.sched.begin(), b.sched.end(), merge_band);
    b.sched2.assign(cut, b.sched.end());
    b.sched.erase(cut, b.sched.end());
    return b;
}


// Adam7 through staging areas (paired-row kernel).  The pixels of passes
// 1-5 are exactly those with an even row and an even column; they are
// unfiltered into staging (DevAdam7Merge): pass 5 as is (S5), pass 4 as is
// (S4), passes 1-3 into Q2[Y][X] = pixel (4X, 4Y) -- pass 3 its odd rows
// whole, passes 1 and 2 its even rows, 2 pixels apart -- and pass 6 then
// writes every even row y of the image whole: its own pixels at the odd
// columns, the staged ones at the even columns (two 8-byte loads per 16
// output bytes, whole-line stores).  Pass 7 writes the odd rows directly.
// Pass 6 runs in a second launch of the kernel over its own band
// schedule (PngBandPlan::sched2), so the staging is complete and visible
// when pass 6 reads it.  Every row of the image is then written once, whole:
// the scatter of all passes xf apart into the image took 8.1 ms per 64 x 4K
// RGBA16, staging passes 1-6 plus a merge kernel 6.5, passes 1-4 stored
// 2-4 pixels apart into one quarter image Q 5.43 (1.76 ms of it the first
// launch; 1.03 with their stores contiguous).
struct Adam7Stage {
    std::vector<DevAdam7Merge> jobs; // q relative to the staging base until png_adam7_rebase
    std::vector<size_t> merge_pass;  // jobs[j]'s pass 6 (index into passes)
    std::vector<size_t> staged;      // passes writing Q (their `out` relative likewise)
    size_t bytes = 0;                // staging bytes
};
// passes[first..] are frame f's, as png_frame_passes made them (Adam7 order,
// empty passes skipped)
inline void png_adam7_stage(const zpx_png_frame &f, int obpx, std::vector<DevPngPass> &passes, size_t first,
                            Adam7Stage &st)
{
    static const uint32_t kA7[6][4] = {{0, 0, 8, 8}, {4, 0, 8, 8}, {0, 4, 4, 8}, {2, 0, 4, 4}, {0, 2, 2, 4}, {1, 0, 2, 2}};
    size_t p6 = ~size_t(0);
    for (size_t i = first; i < passes.size(); i++)
        if (passes[i].xo == 1 && passes[i].xf == 2) p6 = i;
    if (p6 == ~size_t(0)) return; // (no pass 6: a 1-pixel-wide image, which png_pair_supported never takes)
    const uint64_t W = f.width, H = f.height;
    auto area = [&](uint64_t w, uint64_t h, uint64_t &stride) {
        stride = (w * obpx + 127) & ~uint64_t(127);
        st.bytes = (st.bytes + 255) & ~size_t(255);
        const size_t at = st.bytes;
        st.bytes += stride * h;
        return reinterpret_cast<const uint8_t *>(static_cast<uintptr_t>(at));
    };
    DevAdam7Merge m{};
    m.q2 = area((W + 3) / 4, (H + 3) / 4, m.q2stride);                     // pixel (4X, 4Y)
    m.s4 = area(W > 2 ? (W - 2 + 3) / 4 : 0, (H + 3) / 4, m.s4stride);     // pass 4
    m.s5 = area((W + 1) / 2, H > 2 ? (H - 2 + 3) / 4 : 0, m.s5stride);     // pass 5
    m.width = f.width;
    for (size_t i = first; i < passes.size(); i++) {
        DevPngPass &d = passes[i];
        int pno = -1;
        for (int p = 0; p < 6; p++)
            if (d.xo == kA7[p][0] && d.yo == kA7[p][1] && d.xf == kA7[p][2] && d.yf == kA7[p][3]) pno = p;
        if (pno < 0) continue; // pass 7 (the odd rows): the image, first launch
        if (pno == 5) {        // pass 6: the image, merging the staged passes, second launch
            d.launch2 = 1;
            continue;
        }
        if (pno <= 2) { // passes 1-3 in Q2's coordinates: (x, y) -> (x / 4, y / 4)
            d.out = const_cast<uint8_t *>(m.q2);
            d.out_stride = m.q2stride;
            d.xo /= 4;
            d.yo /= 4;
            d.xf /= 4;
            d.yf /= 4;
        } else { // passes 4, 5: their own pixels, as is
            d.out = const_cast<uint8_t *>(pno == 3 ? m.s4 : m.s5);
            d.out_stride = pno == 3 ? m.s4stride : m.s5stride;
            d.xo = d.yo = 0;
            d.xf = d.yf = 1;
        }
        st.staged.push_back(i);
    }
    // (a placeholder until png_adam7_rebase points it at the device job:
    // png_plan_bands only needs to know which passes merge)
    passes[p6].merge = reinterpret_cast<const DevAdam7Merge *>(static_cast<uintptr_t>(st.jobs.size() + 1));
    st.jobs.push_back(m);
    st.merge_pass.push_back(p6);
}
// staging at `base`, the jobs (one DevAdam7Merge each) at `jobs` on the device
inline void png_adam7_rebase(std::vector<DevPngPass> &passes, Adam7Stage &st, uint8_t *base,
                             const DevAdam7Merge *jobs)
{
    for (size_t i : st.staged) passes[i].out = base + reinterpret_cast<uintptr_t>(passes[i].out);
    for (size_t j = 0; j < st.jobs.size(); j++) {
        st.jobs[j].q2 = base + reinterpret_cast<uintptr_t>(st.jobs[j].q2);
        st.jobs[j].s4 = base + reinterpret_cast<uintptr_t>(st.jobs[j].s4);
        st.jobs[j].s5 = base + reinterpret_cast<uintptr_t>(st.jobs[j].s5);
        passes[st.merge_pass[j]].merge = jobs + j;
    }
}

} // namespace zpx
