// Batch / streaming decode (include/zpix_amd.h, zpx_batch_*): the host
// entropy stages run on a thread pool while the calling thread streams their
// results to the GPU and runs the kernels, so Huffman/inflate of image k+1..
// overlaps the PCIe copy of image k and the kernels of image k-1.
//
//   workers (host_threads)          dispatcher (calling thread)
//   ----------------------          -----------------------------------------
//   take item i, wait for a slot    pop a decoded item, bind it to a free slot
//   jpeg_entropy_decode / png_parse copy stream : H2D coefficients / filtered
//     into pinned (pooled) buffers                bytes -> ev_in
//   push to the ready queue         compute     : wait ev_in, descriptor H2D,
//                                                 fused JPEG / PNG kernels
//                                   d2h stream  : (dst_on_host) RGBA -> host
//                                   retire a slot once its ev_done completes
//
// Per image this is exactly zpix.fromBuffer + Image.rgbaPixels (src/root.zig:24-40,
// src/image/image.zig:103-130): the fused JPEG kernel for the interleaved
// geometries, the PNG unfilter kernel (+ rgbaPixels kernel when the decoded
// image type is not already RGBA8), and the per-image entry point for the
// rare JPEG kinds the fused kernel does not take (CMYK, YCCK, non-interleaved).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

#include "api_internal.h"
#include "device_types.h"
#include "host_cpus.h"
#include "jpeg_host.h"
#include "kernels.h"
#include "png_host.h"
#include "zpix_amd.h"

using namespace zpx;

namespace {

constexpr size_t kAlign = 256;
size_t align_up(size_t n) { return (n + kAlign - 1) & ~(kAlign - 1); }

// ZPX_BATCH_TRACE=1: one stderr line per pipeline event (debug aid)
bool trace_on()
{
    static const bool on = getenv("ZPX_BATCH_TRACE") != nullptr;
    return on;
}
double now_s()
{
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
// (trace lines carry a steady-clock time in ms, for timelines)
#define ZPX_TRACE(...)                                                                                     \
    do {                                                                                                   \
        if (trace_on()) {                                                                                  \
            fprintf(stderr, "[zpx batch %.3f] ", now_s() * 1e3);                                            \
            fprintf(stderr, __VA_ARGS__);                                                                   \
            fputc('\n', stderr);                                                                           \
        }                                                                                                  \
    } while (0)

struct Decoded {
    int item = -1;
    int fmt = 0; // 1 JPEG, 2 PNG
    int status = ZPX_OK;
    JpegCoeffs jc;
    PngStream ps;
};

struct Slot {
    DevBuf din, dout, dimg, ddesc, dbound, dgrid, dstage; // dstage: Adam7 passes 1-5 (Adam7Stage)
    PngControl ctl; // PNG control block and its epoch window
    DevBuf dslab; // the paired-row kernel's band slab, built on the device (png_slab_kernels.hip)
    HostBuf hdesc, hstatus; // pinned descriptor staging, PNG status word
    hipEvent_t ev_in = nullptr, ev_kernel = nullptr, ev_done = nullptr;
    std::unique_ptr<Decoded> dec;
    bool busy = false;
    int last_fmt = 0; // format of the slot's last item (its buffers' sizes follow it)
    bool check_png = false;
    bool failed = false; // the image failed after its slot was bound (status already set)
    DevPiecesExpand expand[4]; // a pieces frame the block kernels do not take: its expand jobs (issue_jpeg)
    int nexpand = 0;
    uint32_t expand_max = 0;
};

bool host_reserve(HostBuf &b, size_t n) { return b.bytes >= n || b.alloc(n, false); }

void destroy_slot(Slot &s)
{
    if (s.ev_in) (void)hipEventDestroy(s.ev_in);
    if (s.ev_kernel) (void)hipEventDestroy(s.ev_kernel);
    if (s.ev_done) (void)hipEventDestroy(s.ev_done);
    s.ev_in = s.ev_kernel = s.ev_done = nullptr;
}

size_t slot_bytes(const Slot &s)
{
    return s.din.bytes + s.dout.bytes + s.dimg.bytes + s.ddesc.bytes + s.dbound.bytes + s.dgrid.bytes + s.dstage.bytes +
           s.dslab.bytes;
}

// The slots of finished batches, per device, for the next batch on it: a
// batch's teardown freed ~3 x depth device buffers (hipFree unmaps them)
// and its setup created 3 x depth events, ~9-11 ms outside the decode loop
// of a 64 x 4K batch (~190 ms).  A slot is idle when it is cached (its
// pipeline synchronised every stream) and keeps its device buffers, events,
// pinned words and PNG epoch window; zpx_batch_cache_trim() frees them.
// (Never destroyed at exit: the HIP runtime may be gone by then.)
struct SlotCache {
    static constexpr size_t kMaxSlots = 256;
    static constexpr size_t kMaxBytes = size_t(32) << 30; // device bytes held at most
    std::mutex mu;
    size_t bytes = 0;
    std::vector<std::pair<int, std::unique_ptr<Slot>>> slots; // (device, slot)
};
SlotCache &slot_cache()
{
    static SlotCache *c = new SlotCache;
    return *c;
}

// test switch "jpeg_sparse" = 0: dense coefficient grids instead of pieces
bool jpeg_sparse_upload() { return opt(Opt::JpegSparse) != 0; }

class Pipeline {
  public:
    Pipeline(zpx_ctx *ctx, zpx_batch_item *items, int n, const zpx_batch_opts *o, BatchDone on_done, void *user)
        : ctx_(ctx), items_(items), n_(n), on_done_(on_done), user_(user)
    {
        threads_ = o && o->host_threads > 0 ? o->host_threads : std::min(16, host_cpu_budget());
        depth_ = o && o->depth > 0 ? o->depth : 2 * threads_;
        depth_ = std::max(depth_, 1);
        on_host_ = o && o->dst_on_host;
        tokens_ = depth_;
    }
    ~Pipeline();
    int run(zpx_batch_stats *stats);

  private:
    void worker(int w);
    int setup();
    int issue(Slot &s, bool &sync_done);
    int issue_jpeg(Slot &s, bool &sync_done);
    int upload_pieces(Slot &s, const JpegCoeffs &jc, zpx_jpeg_frame &f, bool direct);
    int issue_png(Slot &s);
    int finish_copy(Slot &s, const uint8_t *src, size_t src_stride, uint32_t W, uint32_t H, hipStream_t producer);
    void retire(Slot &s);
    void give_token();
    void finished(int item) // item's status and result are final
    {
        if (on_done_) on_done_(user_, item);
    }

    zpx_ctx *ctx_;
    zpx_batch_item *items_;
    int n_;
    BatchDone on_done_ = nullptr;
    void *user_ = nullptr;
    int threads_ = 1, depth_ = 1;
    bool on_host_ = false;

    hipStream_t h2d_ = nullptr, d2h_ = nullptr;
    std::vector<std::unique_ptr<Slot>> slots_;
    std::vector<std::thread> workers_;

    std::mutex mu_;
    std::condition_variable cv_ready_, cv_token_;
    std::deque<std::unique_ptr<Decoded>> ready_;
    std::vector<int> oom_items_; // items a worker could not even allocate for
    int tokens_ = 0;
    bool stop_ = false;
    // dispatch order of the host stage (take_item): the most expensive
    // untaken item of the look-ahead window [front_, front_ + 4 threads_)
    std::vector<double> cost_;
    std::vector<char> taken_;
    int front_ = 0, ntaken_ = 0;
    double untaken_cost_ = 0; // sum of cost_ over the untaken items
    // per worker, the virtual time (in host_cost_estimate's units) its
    // current item ends at: the schedule take_item plans the pairs on
    std::vector<double> vbusy_;
    std::vector<char> png_; // the item is a PNG (zpx_png_probe_buffer)
    int take_item(int w, int &remaining, int &partner);
    int png_partner(double max_cost); // (mu_ held)
    // the dispatch window (take_item): 4 x threads items; test switch
    // "batch_lookahead" 1: item order, k >= 2: k x threads
    int lookahead_window() const
    {
        const int o = opt(Opt::BatchLookahead);
        return o == 1 ? 1 : (o >= 2 ? o : 4) * std::max(1, threads_);
    }
    // A slot buffer at least n bytes large.  A buffer too small is replaced,
    // and the old one kept until the pipeline ends: hipFree waits for the
    // whole device, and freeing in the dispatch loop stalled it behind
    // every queued copy and kernel (a JPEG slot taking a PNG: 20-80 ms).
    hipError_t grow(DevBuf &b, size_t n)
    {
        if (b.ptr && b.bytes >= n) return hipSuccess;
        if (b.ptr) {
            retired_.push_back(b.ptr);
            b.ptr = nullptr;
            b.bytes = 0;
        }
        const double t = now_s();
        const hipError_t e = b.alloc(n);
        ZPX_TRACE("grow: %zu bytes in %.2f ms", n, (now_s() - t) * 1e3);
        return e;
    }
    std::vector<void *> retired_; // replaced slot buffers, freed by ~Pipeline
    bool reusable_ = false;        // run() completed: its slots may go to the SlotCache
    void push_decoded(std::unique_ptr<Decoded> d, double dt);
    double host_s_ = 0, host_jpeg_s_ = 0, host_png_s_ = 0;
    int jpeg_items_ = 0, png_items_ = 0;
    double h2d_bytes_ = 0, d2h_bytes_ = 0, pixels_ = 0;
    int failed_ = 0;
};

Pipeline::~Pipeline()
{
    {
        std::lock_guard<std::mutex> lk(mu_);
        stop_ = true;
    }
    cv_token_.notify_all();
    for (auto &t : workers_)
        if (t.joinable()) t.join();
    bool idle = hipStreamSynchronize(ctx_->stream) == hipSuccess;
    if (h2d_) idle = hipStreamSynchronize(h2d_) == hipSuccess && idle;
    if (d2h_) idle = hipStreamSynchronize(d2h_) == hipSuccess && idle;
    for (void *p : retired_) (void)hipFree(p);
    if (reusable_ && idle && opt(Opt::BatchSlotCache)) {
        SlotCache &c = slot_cache();
        std::lock_guard<std::mutex> lk(c.mu);
        for (auto &sp : slots_) {
            if (!sp || sp->busy || c.slots.size() >= SlotCache::kMaxSlots) continue;
            const size_t b = slot_bytes(*sp);
            if (c.bytes + b > SlotCache::kMaxBytes) continue;
            sp->dec.reset();
            c.bytes += b;
            c.slots.emplace_back(ctx_->device, std::move(sp));
        }
    }
    for (auto &s : slots_)
        if (s) destroy_slot(*s); // (not cached)
    if (h2d_) (void)hipStreamDestroy(h2d_);
    if (d2h_) (void)hipStreamDestroy(d2h_);
}

// The inflated stream's bytes of a PNG from its IHDR (every pass's rows x
// (1 + row bytes), readImagePass's layout, + ZPX_PNG_INPUT_PAD), 0 when the
// header does not parse -- the size of its upload buffer.
static size_t png_stream_bytes(const uint8_t *buf, size_t len)
{
    if (!zpx_png_probe_buffer(buf, len) || len < 29) return 0;
    auto be32 = [&](size_t o) { return uint32_t(buf[o]) << 24 | uint32_t(buf[o + 1]) << 16 | uint32_t(buf[o + 2]) << 8 | buf[o + 3]; };
    const uint64_t w = be32(16), h = be32(20);
    static const int kChannels[7] = {1, 0, 3, 1, 2, 0, 4}; // by colour type
    const int depth = buf[24], ct = buf[25] <= 6 ? buf[25] : 0;
    const uint64_t bits = uint64_t(depth) * uint64_t(std::max(1, kChannels[ct]));
    if (w == 0 || h == 0 || w > (1u << 20) || h > (1u << 20) || depth > 16) return 0;
    uint64_t total = 0;
    if (buf[28] == 1) { // Adam7: (x0, y0, dx, dy) per pass
        static const int kP[7][4] = {{0, 0, 8, 8}, {4, 0, 8, 8}, {0, 4, 4, 8}, {2, 0, 4, 4},
                                     {0, 2, 2, 4}, {1, 0, 2, 2}, {0, 1, 1, 2}};
        for (const auto &p : kP) {
            const uint64_t pw = w > uint64_t(p[0]) ? (w - p[0] + p[2] - 1) / p[2] : 0;
            const uint64_t ph = h > uint64_t(p[1]) ? (h - p[1] + p[3] - 1) / p[3] : 0;
            if (pw && ph) total += ph * (1 + (pw * bits + 7) / 8);
        }
    } else {
        total = h * (1 + (w * bits + 7) / 8);
    }
    return static_cast<size_t>(total) + ZPX_PNG_INPUT_PAD;
}

// Host cost estimate of an item (ns on the GPU boxes' Zen 5 cores, order
// of magnitude only: it orders the dispatch, nothing else).  PNG: inflate,
// ~2 ns per inflated byte (png_stream_bytes, from IHDR) + the CRC and
// copy of the compressed bytes; JPEG: Huffman decoding, ~14 ns per
// entropy-coded byte (the bench's 4K q75 frames: 2.8 MB in 39 ms, tc8 PNGs:
// 50 MB inflated in 106 ms).  Anything else costs nothing on the host.
static double host_cost_estimate(const uint8_t *buf, size_t len)
{
    if (zpx_png_probe_buffer(buf, len)) return 2.0 * double(png_stream_bytes(buf, len)) + 0.5 * double(len);
    if (zpx_jpeg_probe_buffer(buf, len)) return 14.0 * double(len);
    return 0;
}

// Next item for worker w: of the untaken items in the window [front_,
// front_ + 4 threads_), the one of the largest host cost (the first of
// equals), so the batch's long items -- a tc8 PNG's inflate is ~3x a JPEG's
// Huffman decode, a PNG pair ~5x -- do not start last and set the end of
// the host stage.  Measured on the bench's 64 alternating 4K JPEG / PNG
// items, 16 workers (tools/e2e_ab.py, batch_lookahead 0 vs 4): a window of
// 2 threads items let only half the PNGs start (and pair) in the first wave,
// and the pairs taken later ended the batch ~50 ms after the rest --
// 3,560-3,640 MPix/s against 4,340-4,460 with 4 threads.  An item waits at
// most one window behind its turn, so prefix completion
// (zpx_batch_wait_prefix) still follows item order.  -1 when none remain;
// `remaining` = the untaken items before this one was taken.
//
// `partner`: a second PNG whose inflate shares the worker's loop
// (png_parse_pair: two streams' decode chains overlap, ~1.3x the work per
// CPU second), or -1.  Only while every worker has items to spare, and only
// while the pair -- which ends later than either PNG alone would, after
// ~(c_i + c_j) / kPairGain -- fits the batch's projected remaining time per
// worker: the untaken items' costs plus what the other workers' current
// items have left, over the workers, on a virtual clock in cost units
// (vbusy_: each worker's current item ends at its start + its cost).  So
// once the first wave of pairs is under way, the PNGs left run one at a
// time beside the JPEGs instead of ending the batch as a late pair (14 or
// 15 workers on the bench's 32 PNG + 32 JPEG batch: the 2-4 PNGs left after
// the first wave ran as one or two pairs ~120 ms after every other item was
// done).  Test switch "batch_makespan" 0: pair whenever items are to spare.
int Pipeline::take_item(int w, int &remaining, int &partner)
{
    constexpr double kPairGain = 1.3;
    std::lock_guard<std::mutex> lk(mu_);
    partner = -1;
    while (front_ < n_ && taken_[front_]) front_++;
    if (front_ >= n_) return -1;
    // (test switch "batch_lookahead" = 1: item order)
    const int win = lookahead_window();
    const int end = std::min(n_, front_ + win);
    int best = -1;
    for (int i = front_; i < end; i++)
        if (!taken_[i] && (best < 0 || cost_[i] > cost_[best])) best = i;
    remaining = n_ - ntaken_;
    const double vt = vbusy_[size_t(w)];
    double busy = 0; // the other workers' current items, what is left of them at vt
    for (size_t o = 0; o < vbusy_.size(); o++)
        if (o != size_t(w)) busy += std::max(0.0, vbusy_[o] - vt);
    const double horizon = (busy + untaken_cost_) / std::max(1, threads_);
    taken_[best] = 1;
    ntaken_++;
    untaken_cost_ -= cost_[best];
    double d = cost_[best];
    const int sub = std::max(1, threads_ / std::max(1, remaining)); // (as worker())
    if (png_[best] && sub == 1 && remaining > 2 * threads_ && depth_ >= 2 && opt(Opt::InflatePair)) {
        const double max_partner = opt(Opt::BatchMakespan) ? kPairGain * horizon - cost_[best] : 1e300;
        if (max_partner > 0) partner = png_partner(max_partner);
        if (partner >= 0) d = (cost_[best] + cost_[partner]) / kPairGain;
    }
    vbusy_[size_t(w)] = vt + d;
    return best;
}

// A second PNG for a pair (take_item): of the untaken PNGs in the window,
// the one of the largest host cost, else the next untaken PNG past the
// window (taking an item early delays no prefix) -- in both cases one whose
// cost is at most max_cost; -1 when none.  (mu_ held)
int Pipeline::png_partner(double max_cost)
{
    const int win = lookahead_window();
    const int end = std::min(n_, front_ + win);
    int best = -1;
    for (int i = front_; i < end; i++)
        if (!taken_[i] && png_[i] && cost_[i] <= max_cost && (best < 0 || cost_[i] > cost_[best])) best = i;
    for (int i = end; best < 0 && i < n_; i++)
        if (!taken_[i] && png_[i] && cost_[i] <= max_cost) best = i;
    if (best >= 0) {
        taken_[best] = 1;
        ntaken_++;
        untaken_cost_ -= cost_[best];
    }
    return best;
}

void Pipeline::push_decoded(std::unique_ptr<Decoded> d, double dt)
{
    ZPX_TRACE("worker: item %d fmt %d status %d decoded in %.3fs", d->item, d->fmt, d->status, dt);
    {
        std::lock_guard<std::mutex> lk(mu_);
        host_s_ += dt;
        if (d->fmt == 1) {
            host_jpeg_s_ += dt;
            jpeg_items_++;
        } else if (d->fmt == 2) {
            host_png_s_ += dt;
            png_items_++;
        }
        ready_.push_back(std::move(d));
    }
    cv_ready_.notify_one();
}

void Pipeline::worker(int w)
{
    for (;;) {
        int remaining = 0, j = -1;
        const int i = take_item(w, remaining, j);
        if (i < 0) return;
        // threads this item may use: one while enough items remain to keep
        // every worker busy; the batch's last items split the workers that
        // are about to go idle (parallel inflate, restart-interval Huffman).
        // j: a second PNG inflated in the same loop (take_item)
        const int sub = std::max(1, threads_ / std::max(1, remaining));
        const int need = j >= 0 ? 2 : 1;
        ZPX_TRACE("worker: took item %d%s%d (remaining %d)", i, j >= 0 ? " + " : "", j, remaining);
        {
            std::unique_lock<std::mutex> lk(mu_);
            cv_token_.wait(lk, [&] { return tokens_ >= need || stop_; });
            if (stop_) return;
            tokens_ -= need;
        }
        ZPX_TRACE("worker: tokens for item %d", i);
        if (j >= 0) {
            std::unique_ptr<Decoded> d0(new (std::nothrow) Decoded), d1(new (std::nothrow) Decoded);
            if (!d0 || !d1) { // out of memory: report on the items, keep the pipeline going
                std::lock_guard<std::mutex> lk(mu_);
                oom_items_.push_back(i);
                oom_items_.push_back(j);
                cv_ready_.notify_one();
                continue;
            }
            d0->item = i;
            d1->item = j;
            d0->fmt = d1->fmt = 2;
            const double t0 = now_s();
            const uint8_t *buf[2] = {items_[i].buf, items_[j].buf};
            const size_t len[2] = {items_[i].len, items_[j].len};
            PngStream *out[2] = {&d0->ps, &d1->ps};
            int st[2];
            png_parse_pair(buf, len, out, st);
            d0->status = st[0];
            d1->status = st[1];
            const double dt = now_s() - t0;
            push_decoded(std::move(d0), dt / 2);
            push_decoded(std::move(d1), dt / 2);
            continue;
        }
        std::unique_ptr<Decoded> d(new (std::nothrow) Decoded);
        if (!d) { // out of memory: report on the item, keep the pipeline going
            std::lock_guard<std::mutex> lk(mu_);
            oom_items_.push_back(i);
            cv_ready_.notify_one();
            continue;
        }
        d->item = i;
        const zpx_batch_item &it = items_[i];
        const double t0 = now_s();
        if (png_[i]) {
            d->fmt = 2;
            d->status = png_parse(it.buf, it.len, d->ps, sub);
            // (the paired-row kernel's band slab is built on the device from
            // the uploaded stream: issue_png)
        } else if (zpx_jpeg_probe_buffer(it.buf, it.len)) {
            d->fmt = 1;
            d->status = jpeg_entropy_decode(it.buf, it.len, d->jc, sub, jpeg_sparse_upload());
        } else if (it.buf && it.len >= 4 && (memcmp(it.buf, "qoif", 4) == 0 || (it.buf[0] == 'B' && it.buf[1] == 'M'))) {
            d->status = ZPX_E_UNSUPPORTED; // QOI / BMP: out of scope (zpx_from_buffer)
        } else {
            d->status = ZPX_E_UNKNOWN_IMAGE_FORMAT;
        }
        push_decoded(std::move(d), now_s() - t0);
    }
}

void Pipeline::give_token()
{
    {
        std::lock_guard<std::mutex> lk(mu_);
        tokens_++;
    }
    // (notify_all: a worker holding a PNG pair waits for two tokens; woken
    // alone on one token it would sleep again while a one-token waiter
    // stayed asleep behind the free token)
    cv_token_.notify_all();
}

int Pipeline::setup()
{
    HIPCHK(ctx_, hipStreamCreateWithFlags(&h2d_, hipStreamNonBlocking));
    HIPCHK(ctx_, hipStreamCreateWithFlags(&d2h_, hipStreamNonBlocking));
    if (opt(Opt::BatchSlotCache)) { // the cached slots of this device first
        SlotCache &c = slot_cache();
        std::lock_guard<std::mutex> lk(c.mu);
        for (size_t k = c.slots.size(); k-- > 0 && int(slots_.size()) < depth_;)
            if (c.slots[k].first == ctx_->device) {
                c.bytes -= std::min(c.bytes, slot_bytes(*c.slots[k].second));
                slots_.push_back(std::move(c.slots[k].second));
                c.slots.erase(c.slots.begin() + static_cast<std::ptrdiff_t>(k));
            }
    }
    for (int i = int(slots_.size()); i < depth_; i++) {
        std::unique_ptr<Slot> s(new Slot);
        HIPCHK(ctx_, hipEventCreateWithFlags(&s->ev_in, hipEventDisableTiming));
        HIPCHK(ctx_, hipEventCreateWithFlags(&s->ev_kernel, hipEventDisableTiming));
        HIPCHK(ctx_, hipEventCreateWithFlags(&s->ev_done, hipEventDisableTiming));
        // PNG control block: set once (the slot's own epoch window,
        // PngControl); every launch moves the epoch on (png_ctl_kernel),
        // and issue_png re-bases it, clearing the boundary, before a wrap
        if (int e = s->ctl.init(ctx_)) return e;
        if (!s->hstatus.alloc(16, true)) return ZPX_E_OUT_OF_MEMORY;
        slots_.push_back(std::move(s));
    }
    // every slot's input buffer sized for the batch's largest PNG stream up
    // front (IHDR), when that takes at most a quarter of the free device
    // memory: a device allocation in the dispatch loop waits behind the
    // workers' pinned-memory allocations (hipMalloc of 50 MB: 20-65 ms in a
    // traced 4K batch, the dispatch of every later item held up with it)
    size_t max_in = 0;
    for (int i = 0; i < n_; i++)
        if (png_[i]) max_in = std::max(max_in, png_stream_bytes(items_[i].buf, items_[i].len));
    size_t free_b = 0, total_b = 0;
    if (max_in && hipMemGetInfo(&free_b, &total_b) == hipSuccess && max_in * slots_.size() <= free_b / 4)
        for (auto &s : slots_) HIPCHK(ctx_, grow(s->din, max_in));
    HIPCHK(ctx_, hipStreamSynchronize(ctx_->stream));
    return ZPX_OK;
}

// Copies a finished contiguous RGBA8 result (4W stride) into the item's dst.
int Pipeline::finish_copy(Slot &s, const uint8_t *src, size_t src_stride, uint32_t W, uint32_t H,
                          hipStream_t producer)
{
    const zpx_batch_item &it = items_[s.dec->item];
    const size_t stride = it.dst_stride ? it.dst_stride : size_t(W) * 4;
    if (on_host_) {
        HIPCHK(ctx_, hipEventRecord(s.ev_kernel, producer));
        HIPCHK(ctx_, hipStreamWaitEvent(d2h_, s.ev_kernel, 0));
        HIPCHK(ctx_, hipMemcpy2DAsync(it.dst, stride, src, src_stride, size_t(W) * 4, H, hipMemcpyDeviceToHost, d2h_));
        HIPCHK(ctx_, hipEventRecord(s.ev_done, d2h_));
        d2h_bytes_ += double(W) * H * 4;
    } else {
        if (src != it.dst)
            HIPCHK(ctx_, hipMemcpy2DAsync(it.dst, stride, src, src_stride, size_t(W) * 4, H, hipMemcpyDeviceToDevice,
                                          producer));
        HIPCHK(ctx_, hipEventRecord(s.ev_done, producer));
    }
    return ZPX_OK;
}

// A pieces frame (JpegPieces): H2D of its index arrays and pieces on the
// copy stream.  direct: the block kernels read them (f keeps the pieces
// layout with device pointers); otherwise the slot's expand jobs turn them
// into dense grids on the compute stream first (issue_jpeg) and f points at
// those.
int Pipeline::upload_pieces(Slot &s, const JpegCoeffs &jc, zpx_jpeg_frame &f, bool direct)
{
    const JpegPieces &p = jc.pieces;
    size_t ib = 0;
    for (int c = 0; c < jc.n_comp; c++) ib += align_up(p.blocks[c] * sizeof(uint32_t));
    HIPCHK(ctx_, grow(s.din, ib + p.data_bytes()));
    uint8_t *base = s.din.as<uint8_t>();
    const uint32_t *dix[4] = {};
    size_t off = 0;
    for (int c = 0; c < jc.n_comp; c++) {
        const size_t n = p.blocks[c] * sizeof(uint32_t);
        HIPCHK(ctx_, hipMemcpyAsync(base + off, p.index_of(c), n, hipMemcpyHostToDevice, h2d_));
        dix[c] = reinterpret_cast<const uint32_t *>(base + off);
        off += align_up(n);
    }
    uint8_t *dp = base + off;
    HIPCHK(ctx_, hipMemcpyAsync(dp, p.data.ptr, p.data_bytes(), hipMemcpyHostToDevice, h2d_));
    h2d_bytes_ += double(off + p.data_bytes());
    s.nexpand = 0;
    s.expand_max = 0;
    if (direct) {
        for (int c = 0; c < jc.n_comp; c++) f.coeffs[c] = dix[c];
        f.pieces = dp;
        return ZPX_OK;
    }
    size_t gbytes[4] = {}, total = 0;
    for (int c = 0; c < jc.n_comp; c++) {
        gbytes[c] = p.blocks[c] * 64 * (f.coeff_bits / 8);
        total += align_up(gbytes[c]);
    }
    HIPCHK(ctx_, grow(s.dgrid, total));
    off = 0;
    for (int c = 0; c < jc.n_comp; c++) {
        DevPiecesExpand &j = s.expand[s.nexpand++];
        j = DevPiecesExpand{};
        j.index = dix[c];
        j.pieces = dp;
        j.grid = s.dgrid.as<uint8_t>() + off;
        j.blocks = static_cast<uint32_t>(p.blocks[c]);
        s.expand_max = std::max(s.expand_max, j.blocks);
        f.coeffs[c] = j.grid;
        off += align_up(gbytes[c]);
    }
    f.layout = ZPX_COEFFS_GRID;
    f.pieces = nullptr;
    f.pieces_bytes = 0;
    return ZPX_OK;
}

int Pipeline::issue_jpeg(Slot &s, bool &sync_done)
{
    Decoded &d = *s.dec;
    zpx_batch_item &it = items_[d.item];
    zpx_jpeg_frame f;
    size_t cb[4];
    jpeg_fill_frame(d.jc, &f, cb);
    const uint32_t W = f.width, H = f.height;
    const size_t stride = it.dst_stride ? it.dst_stride : size_t(W) * 4;
    const JpegOut kind = jpeg_output_kind(d.jc);
    const bool fused = kind != JpegOut::CMYK && kind != JpegOut::YCCK && jpeg_fusable(f);
    if (kind == JpegOut::YCCK || (d.jc.n_comp == 4 && !d.jc.adobe_valid)) { // jpeg.decode's own errors
        it.status = kind == JpegOut::YCCK ? ZPX_E_UNSUPPORTED : ZPX_E_UNSUPPORTED_COLOR_MODEL;
        sync_done = true;
        return ZPX_OK;
    }
    // fused dequant + IDCT + upsample + colour straight into the destination
    if (d.jc.pieces.valid) {
        // the block kernels read the pieces (the RGBA rows they store are
        // dword aligned: a device destination's own stride, or the slot's
        // staging at 4W)
        const bool aligned = on_host_ || ((stride & 3) == 0 && (reinterpret_cast<uintptr_t>(it.dst) & 3) == 0);
        const bool direct = fused && f.narrow && (f.coeff_bits == 8 || f.coeff_bits == 16) &&
                            opt(Opt::JpegStrip) == 0 && aligned &&
                            jpeg_block_pieces_supported(f.color, f.h[0], f.v[0], f.h[1], f.v[1]);
        if (int e = upload_pieces(s, d.jc, f, direct)) return e;
    } else {
        size_t total = 0;
        for (int c = 0; c < 4; c++) total += f.coeffs[c] ? align_up(cb[c]) : 0;
        HIPCHK(ctx_, grow(s.din, total));
        size_t off = 0;
        for (int c = 0; c < 4; c++) {
            if (!f.coeffs[c]) continue;
            uint8_t *dst = s.din.as<uint8_t>() + off;
            HIPCHK(ctx_, hipMemcpyAsync(dst, f.coeffs[c], cb[c], hipMemcpyHostToDevice, h2d_));
            f.coeffs[c] = dst;
            off += align_up(cb[c]);
            h2d_bytes_ += double(cb[c]);
        }
    }
    HIPCHK(ctx_, hipEventRecord(s.ev_in, h2d_));
    HIPCHK(ctx_, hipStreamWaitEvent(ctx_->stream, s.ev_in, 0));
    if (d.jc.pieces.valid && s.nexpand) {
        // the jobs go up behind the frame descriptor's place in the staging
        // (the descriptor copy below must not overwrite them in flight)
        const size_t jo = align_up(sizeof(DevJpegFrame));
        HIPCHK(ctx_, grow(s.ddesc, jo + sizeof(s.expand)));
        if (!host_reserve(s.hdesc, jo + sizeof(s.expand))) return ZPX_E_OUT_OF_MEMORY;
        memcpy(static_cast<uint8_t *>(s.hdesc.ptr) + jo, s.expand, sizeof(s.expand));
        HIPCHK(ctx_, hipMemcpyAsync(s.ddesc.as<uint8_t>() + jo, static_cast<uint8_t *>(s.hdesc.ptr) + jo,
                                    sizeof(s.expand), hipMemcpyHostToDevice, ctx_->stream));
        if (launch_jpeg_pieces_expand(reinterpret_cast<const DevPiecesExpand *>(s.ddesc.as<uint8_t>() + jo), s.nexpand,
                                      s.expand_max, f.coeff_bits, ctx_->stream))
            return hip_fail(ctx_, hipGetLastError(), "batch: jpeg pieces expand");
    }
    if (!fused) {
        // planes + colour pass from the coefficients this worker already
        // decoded (no second entropy decode, no host sync): CMYK, Adobe RGB
        // with non-interleaved scans, ...; the colour kernels write 4W rows
        const bool direct = !on_host_ && stride == size_t(W) * 4;
        uint8_t *out = it.dst;
        if (!direct) {
            HIPCHK(ctx_, grow(s.dout, size_t(W) * H * 4));
            out = s.dout.as<uint8_t>();
        }
        if (int e = jpeg_planes_to_rgba(ctx_, d.jc, f, s.dimg, s.ddesc, s.hdesc, out, ctx_->stream)) {
            if (e == ZPX_E_HIP) return e;
            it.status = e; // the image's own error; the slot's queued copy is harmless
            HIPCHK(ctx_, hipEventRecord(s.ev_done, ctx_->stream));
            s.failed = true;
            return ZPX_OK;
        }
        if (direct) {
            HIPCHK(ctx_, hipEventRecord(s.ev_done, ctx_->stream));
            return ZPX_OK;
        }
        return finish_copy(s, out, size_t(W) * 4, W, H, ctx_->stream);
    }
    const bool direct = !on_host_;
    uint8_t *out;
    if (direct) {
        out = it.dst;
        f.rgba_stride = stride;
    } else {
        HIPCHK(ctx_, grow(s.dout, size_t(W) * H * 4));
        out = s.dout.as<uint8_t>();
        f.rgba_stride = size_t(W) * 4;
    }
    f.rgba = out;
    const DevJpegFrame df = dev_jpeg_frame(f);
    if (!host_reserve(s.hdesc, sizeof(df))) return ZPX_E_OUT_OF_MEMORY;
    memcpy(s.hdesc.ptr, &df, sizeof(df));
    HIPCHK(ctx_, grow(s.ddesc, sizeof(df)));
    HIPCHK(ctx_, hipMemcpyAsync(s.ddesc.ptr, s.hdesc.ptr, sizeof(df), hipMemcpyHostToDevice, ctx_->stream));
    if (int rc = launch_jpeg_rgba_frame(f, s.ddesc.as<DevJpegFrame>(), ctx_->stream))
        return rc == -2 ? ZPX_E_UNSUPPORTED : hip_fail(ctx_, hipGetLastError(), "batch: jpeg kernel");
    if (direct) {
        HIPCHK(ctx_, hipEventRecord(s.ev_done, ctx_->stream));
        return ZPX_OK;
    }
    return finish_copy(s, out, size_t(W) * 4, W, H, ctx_->stream);
}

int Pipeline::issue_png(Slot &s)
{
    Decoded &d = *s.dec;
    zpx_batch_item &it = items_[d.item];
    PngStream &ps = d.ps;
    const uint32_t W = ps.width, H = ps.height;
    const size_t stride = it.dst_stride ? it.dst_stride : size_t(W) * 4;
    // the inflated stream goes up as is, and the kernel reads it: the
    // paired-row kernel's stream instance, or the one-row-per-lane kernel
    // (under the test switch png_device_slab the paired-row kernel's band
    // slab is built from it on the device first, png_slab_kernels.hip)
    const bool pair = png_use_pair(ps.depth, ps.interlace, ps.use_transparent, W,
                                   ps.kind == ZPX_RGBA ? stride : size_t(W) * ps.out_bpp);
    const size_t in_len = ps.data_len + ZPX_PNG_INPUT_PAD;
    HIPCHK(ctx_, grow(s.din, in_len));
    const double th = now_s();
    HIPCHK(ctx_, hipMemcpyAsync(s.din.ptr, ps.data.ptr, in_len, hipMemcpyHostToDevice, h2d_));
    ZPX_TRACE("png: item %d H2D issue %.2f ms (pinned %d)", d.item, (now_s() - th) * 1e3, ps.data.pinned ? 1 : 0);
    h2d_bytes_ += double(ps.data_len);
    HIPCHK(ctx_, hipEventRecord(s.ev_in, h2d_));
    HIPCHK(ctx_, hipStreamWaitEvent(ctx_->stream, s.ev_in, 0));

    // readImagePass's image type: RGBA8 already is the rgbaPixels layout
    const bool rgba_native = ps.kind == ZPX_RGBA;
    const bool direct = !on_host_ && (rgba_native || stride == size_t(W) * 4);
    uint8_t *img_out;
    size_t img_stride;
    if (rgba_native) {
        if (direct) {
            img_out = it.dst;
            img_stride = stride;
        } else {
            HIPCHK(ctx_, grow(s.dout, size_t(W) * H * 4));
            img_out = s.dout.as<uint8_t>();
            img_stride = size_t(W) * 4;
        }
    } else {
        img_stride = size_t(W) * ps.out_bpp;
        HIPCHK(ctx_, grow(s.dimg, img_stride * H));
        img_out = s.dimg.as<uint8_t>();
    }
    zpx_png_frame f;
    memset(&f, 0, sizeof(f));
    f.width = W;
    f.height = H;
    f.depth = ps.depth;
    f.interlace = ps.interlace;
    f.use_transparent = ps.use_transparent;
    memcpy(f.transparent, ps.transparent, 6);
    f.filtered = s.din.as<uint8_t>();
    f.layout = ZPX_PNG_LAYOUT_STREAM;
    f.out = img_out;
    f.out_stride = img_stride;
    f.max_index = nullptr; // palette handled below with all 256 entries
    std::vector<uint64_t> slab_off;
    std::vector<DevSlabBand> sjobs;
    uint32_t slab_groups = 0;
    const bool dev_slab = pair && opt(Opt::PngDeviceSlab);
    if (dev_slab) {
        const size_t slab_b = png_dev_slab_layout(f, slab_off);
        HIPCHK(ctx_, grow(s.dslab, slab_b));
        png_dev_slab_jobs(f, slab_off, s.din.as<uint8_t>(), in_len, s.dslab.as<uint8_t>(), sjobs, slab_groups);
        f.filtered = s.dslab.as<uint8_t>();
        f.layout = ZPX_PNG_LAYOUT_SLAB;
    }
    std::vector<DevPngPass> passes;
    std::vector<uint32_t> rowbytes;
    uint64_t bytes = 0;
    png_frame_passes(f, passes, rowbytes, bytes);
    Adam7Stage a7;
    if (pair && ps.interlace) {
        png_adam7_stage(f, static_cast<int>(ps.out_bpp), passes, 0, a7);
        HIPCHK(ctx_, grow(s.dstage, a7.bytes));
    }
    const PngBandPlan bp = png_plan_bands(ps.depth, pair, passes, rowbytes);
    const uint32_t granules = bp.granules;
    const uint32_t base = bp.nbands;
    const uint32_t ns = static_cast<uint32_t>(bp.sched.size()), ns2 = static_cast<uint32_t>(bp.sched2.size());
    // descriptor staging: passes | sched, sched2 | palette (256 zpx_color) | Adam7 merge job |
    // slab band table | slab jobs
    const size_t pass_b = align_up(passes.size() * sizeof(DevPngPass));
    const size_t sched_b = align_up(std::max<size_t>(1, ns + ns2) * sizeof(DevPngBand));
    const size_t pal_b = align_up(256 * sizeof(zpx_color));
    const size_t merge_b = align_up(a7.jobs.size() * sizeof(DevAdam7Merge));
    const size_t table_b = align_up(slab_off.size() * sizeof(uint64_t));
    const size_t sjobs_b = sjobs.size() * sizeof(DevSlabBand);
    const size_t desc_b = pass_b + sched_b + pal_b + merge_b + table_b + sjobs_b;
    HIPCHK(ctx_, grow(s.ddesc, desc_b));
    uint8_t *dd = s.ddesc.as<uint8_t>();
    if (!a7.jobs.empty())
        png_adam7_rebase(passes, a7, s.dstage.as<uint8_t>(),
                         reinterpret_cast<const DevAdam7Merge *>(dd + pass_b + sched_b + pal_b));
    if (!host_reserve(s.hdesc, desc_b)) return ZPX_E_OUT_OF_MEMORY;
    uint8_t *h = static_cast<uint8_t *>(s.hdesc.ptr);
    memcpy(h, passes.data(), passes.size() * sizeof(DevPngPass));
    if (ns) memcpy(h + pass_b, bp.sched.data(), ns * sizeof(DevPngBand));
    if (ns2) memcpy(h + pass_b + ns * sizeof(DevPngBand), bp.sched2.data(), ns2 * sizeof(DevPngBand));
    memcpy(h + pass_b + sched_b, ps.palette, 256 * sizeof(zpx_color));
    if (!a7.jobs.empty()) memcpy(h + pass_b + sched_b + pal_b, a7.jobs.data(), a7.jobs.size() * sizeof(DevAdam7Merge));
    const size_t table_at = pass_b + sched_b + pal_b + merge_b, sjobs_at = table_at + table_b;
    if (!slab_off.empty()) memcpy(h + table_at, slab_off.data(), slab_off.size() * sizeof(uint64_t));
    if (sjobs_b) memcpy(h + sjobs_at, sjobs.data(), sjobs_b);
    HIPCHK(ctx_, hipMemcpyAsync(dd, h, desc_b, hipMemcpyHostToDevice, ctx_->stream));
    if (dev_slab) {
        // the slab: its band table, then the bands from the stream (once the
        // stream has landed: the compute stream waits for ev_in above)
        HIPCHK(ctx_, hipMemcpyAsync(s.dslab.ptr, dd + table_at, slab_off.size() * sizeof(uint64_t),
                                    hipMemcpyDeviceToDevice, ctx_->stream));
        if (launch_png_slab(png_slab_chunk_bytes(ps.depth), reinterpret_cast<const DevSlabBand *>(dd + sjobs_at),
                            static_cast<uint32_t>(sjobs.size()), slab_groups, ctx_->stream))
            return hip_fail(ctx_, hipGetLastError(), "batch: png slab kernel");
    }
    const size_t bound_b = std::max<size_t>(1, base) * granules * sizeof(uint64_t);
    if (s.dbound.bytes < bound_b) { // fresh granules carry tag 0, older than any epoch
        HIPCHK(ctx_, grow(s.dbound, bound_b));
        HIPCHK(ctx_, hipMemsetAsync(s.dbound.ptr, 0, bound_b, ctx_->stream));
    }
    ZPX_TRACE("png: item %d %ux%u depth %d interlace %d passes %zu bands %u+%u granules %u", d.item, W, H, ps.depth,
              ps.interlace, passes.size(), ns, ns2, granules);
    const DevPngPass *dp = reinterpret_cast<const DevPngPass *>(dd);
    const DevPngBand *dsch = reinterpret_cast<const DevPngBand *>(dd + pass_b);
    // control words {epoch, ticket, status, sticky}: each launch's ctl kernel
    // folds the previous launch's status into `sticky`, so an Adam7 item's
    // first launch reports through sticky -- clear it for this item (the
    // slot's words are reused) and read both words after the last launch
    HIPCHK(ctx_, hipMemsetAsync(s.ctl.words() + 3, 0, 4, ctx_->stream));
    // (a slot's images differ in geometry, so a granule may outlive many
    // launches unread: before the launches that would wrap the epoch cycle
    // the boundary buffer is cleared)
    if (int e = s.ctl.prepare(ctx_, ns2 ? 2 : 1, s.dbound.ptr, s.dbound.bytes, ctx_->stream)) return e;
    const int lrc = pair ? launch_png_pair(ps.depth, ps.use_transparent, !dev_slab, dp, dsch, ns, s.ctl.words(),
                                           s.dbound.as<uint64_t>(), granules, ctx_->stream)
                         : launch_png_unfilter(ps.depth, dp, dsch, ns, s.ctl.words(), s.dbound.as<uint64_t>(),
                                               granules, ctx_->stream);
    if (lrc)
        return hip_fail(ctx_, hipGetLastError(), "batch: png kernel");
    // Adam7: pass 6 merges the staged passes once the first launch is done
    if (ns2 && launch_png_pair_merge(ps.depth, ps.use_transparent, !dev_slab, dp, dsch + ns, ns2, s.ctl.words(),
                                     s.dbound.as<uint64_t>(), granules, ctx_->stream))
        return hip_fail(ctx_, hipGetLastError(), "batch: png adam7 merge pass");
    HIPCHK(ctx_, hipMemcpyAsync(s.hstatus.ptr, s.ctl.words() + 2, 8, hipMemcpyDeviceToHost, ctx_->stream));
    s.check_png = true;
    if (rgba_native) {
        if (direct) {
            HIPCHK(ctx_, hipEventRecord(s.ev_done, ctx_->stream));
            return ZPX_OK;
        }
        return finish_copy(s, img_out, size_t(W) * 4, W, H, ctx_->stream);
    }
    // Image.rgbaPixels of the decoded image type (premultiply, palette, 16-bit)
    zpx_image img{};
    img.kind = ps.kind;
    img.max_x = static_cast<int32_t>(W);
    img.max_y = static_cast<int32_t>(H);
    img.stride = img_stride;
    img.pixels_len = img_stride * H;
    // grown palette entries are opaque black (readImagePass :1079-1134), which
    // is what entries past PLTE/tRNS already hold, so all 256 are live
    img.palette_len = ps.kind == ZPX_PALETTED ? 256 : 0;
    const DevImage m = dev_image_of(&img, img_out, ps.kind == ZPX_PALETTED ? dd + pass_b + sched_b : nullptr);
    uint8_t *rgba;
    if (direct) {
        rgba = it.dst;
    } else {
        HIPCHK(ctx_, grow(s.dout, size_t(W) * H * 4));
        rgba = s.dout.as<uint8_t>();
    }
    if (launch_rgba_pixels(m, rgba, ctx_->stream)) return hip_fail(ctx_, hipGetLastError(), "batch: rgba kernel");
    ZPX_TRACE("png: item %d rgba kernel launched (kind %d)", d.item, ps.kind);
    if (direct) {
        HIPCHK(ctx_, hipEventRecord(s.ev_done, ctx_->stream));
        return ZPX_OK;
    }
    return finish_copy(s, rgba, size_t(W) * 4, W, H, ctx_->stream);
}

int Pipeline::issue(Slot &s, bool &sync_done)
{
    Decoded &d = *s.dec;
    zpx_batch_item &it = items_[d.item];
    const uint32_t W = d.fmt == 1 ? d.jc.width : d.ps.width, H = d.fmt == 1 ? d.jc.height : d.ps.height;
    it.width = W;
    it.height = H;
    const size_t stride = it.dst_stride ? it.dst_stride : size_t(W) * 4;
    const size_t need = H ? (size_t(H) - 1) * stride + size_t(W) * 4 : 0;
    if (!it.dst || stride < size_t(W) * 4 || it.dst_capacity < need || stride > (size_t(1) << 31) / 32) {
        it.status = ZPX_E_INVALID_ARGUMENT;
        sync_done = true;
        return ZPX_OK;
    }
    if (d.fmt == 2)
        for (int p = 0; p < d.ps.npasses; p++)
            if (!png_band_fits(d.ps.pass[p].row_bytes, 64)) { // (the paired-row kernel declines wider bands)
                it.status = ZPX_E_UNSUPPORTED;
                sync_done = true;
                return ZPX_OK;
            }
    sync_done = false;
    s.check_png = false;
    s.failed = false;
    return d.fmt == 1 ? issue_jpeg(s, sync_done) : issue_png(s);
}

void Pipeline::retire(Slot &s)
{
    zpx_batch_item &it = items_[s.dec->item];
    if (s.failed) {
        // it.status holds the image's error
    } else if (s.check_png && (static_cast<volatile uint32_t *>(s.hstatus.ptr)[0] |
                               static_cast<volatile uint32_t *>(s.hstatus.ptr)[1]) != 0) {
        ctx_->last_error = "png wavefront hand-off timed out";
        it.status = ZPX_E_HIP;
    } else {
        it.status = ZPX_OK;
        pixels_ += double(it.width) * it.height;
    }
    const int item = s.dec->item;
    s.dec.reset(); // pinned host buffers go back to the pool
    s.busy = false;
    give_token();
    finished(item);
}

int Pipeline::run(zpx_batch_stats *stats)
{
    const double t0 = now_s();
    for (int i = 0; i < n_; i++) {
        items_[i].status = ZPX_E_HIP; // until completed
        items_[i].width = items_[i].height = 0;
        items_[i].format = zpx_png_probe_buffer(items_[i].buf, items_[i].len) ? 2
                           : zpx_jpeg_probe_buffer(items_[i].buf, items_[i].len) ? 1 : 0;
    }
    cost_.resize(size_t(n_));
    taken_.assign(size_t(n_), 0);
    png_.assign(size_t(n_), 0);
    for (int i = 0; i < n_; i++) png_[i] = items_[i].format == 2;
    for (int i = 0; i < n_; i++) cost_[i] = host_cost_estimate(items_[i].buf, items_[i].len);
    untaken_cost_ = 0;
    for (int i = 0; i < n_; i++) untaken_cost_ += cost_[i];
    vbusy_.assign(size_t(std::max(1, std::min(threads_, std::max(n_, 1)))), 0.0);
    if (int e = setup()) return e;
    try {
        for (int t = 0; t < std::min(threads_, std::max(n_, 1)); t++) workers_.emplace_back([this, t] { worker(t); });
    } catch (...) {
        return ZPX_E_OUT_OF_MEMORY;
    }
    int done = 0, rc = ZPX_OK;
    while (done < n_ && rc == ZPX_OK) {
        std::unique_ptr<Decoded> d;
        bool any_busy = false;
        for (auto &s : slots_) any_busy |= s->busy;
        std::vector<int> oom;
        {
            std::unique_lock<std::mutex> lk(mu_);
            if (ready_.empty() && oom_items_.empty()) {
                if (any_busy) cv_ready_.wait_for(lk, std::chrono::microseconds(100));
                else cv_ready_.wait(lk, [&] { return !ready_.empty() || !oom_items_.empty(); });
            }
            if (!ready_.empty()) {
                d = std::move(ready_.front());
                ready_.pop_front();
            }
            oom.swap(oom_items_);
        }
        for (int i : oom) {
            items_[i].status = ZPX_E_OUT_OF_MEMORY;
            done++;
            give_token();
            finished(i);
        }
        if (d) {
            if (d->status != ZPX_OK) {
                items_[d->item].status = d->status;
                done++;
                give_token();
                finished(d->item);
            } else {
                // a free slot, one whose last item had this item's format if
                // any: its grow-only device buffers then fit without a new
                // allocation (hipFree / hipMalloc wait for the device: a PNG
                // bound to a slot that held JPEGs stalled this loop -- and so
                // every later item's dispatch -- for 20-80 ms)
                Slot *free_slot = nullptr;
                for (auto &s : slots_)
                    if (!s->busy && (!free_slot || (s->last_fmt == d->fmt && free_slot->last_fmt != d->fmt)))
                        free_slot = s.get();
                // a worker holds a token for every decoded item, and there are
                // as many tokens as slots, so a free slot always exists here
                Slot &s = *free_slot;
                s.last_fmt = d->fmt;
                s.dec = std::move(d);
                s.busy = true;
                bool sync_done = false;
                ZPX_TRACE("dispatch: item %d -> slot %p", s.dec->item, static_cast<void *>(&s));
                rc = issue(s, sync_done);
                ZPX_TRACE("dispatch: item %d issued rc %d sync %d", s.dec->item, rc, sync_done ? 1 : 0);
                if (rc == ZPX_OK && sync_done) {
                    const int item = s.dec->item;
                    if (items_[item].status == ZPX_OK)
                        pixels_ += double(items_[item].width) * items_[item].height;
                    s.dec.reset();
                    s.busy = false;
                    done++;
                    give_token();
                    finished(item);
                }
            }
        }
        for (auto &sp : slots_) {
            Slot &s = *sp;
            if (!s.busy) continue;
            const hipError_t q = hipEventQuery(s.ev_done);
            if (q == hipSuccess) {
                ZPX_TRACE("retire: item %d", s.dec->item);
                retire(s);
                done++;
            } else if (q != hipErrorNotReady) {
                rc = hip_fail(ctx_, q, "batch: event");
                break;
            }
        }
    }
    {
        std::lock_guard<std::mutex> lk(mu_);
        stop_ = true;
    }
    cv_token_.notify_all();
    for (auto &t : workers_) t.join();
    workers_.clear();
    bool device_ok = true; // (a slot of an item that failed on the device is not reused)
    for (int i = 0; i < n_; i++) {
        failed_ += items_[i].status != ZPX_OK;
        device_ok = device_ok && items_[i].status != ZPX_E_HIP;
    }
    reusable_ = rc == ZPX_OK && done == n_ && device_ok;
    if (stats) {
        memset(stats, 0, sizeof(*stats));
        stats->wall_s = now_s() - t0;
        stats->host_s = host_s_;
        stats->host_jpeg_s = host_jpeg_s_;
        stats->host_png_s = host_png_s_;
        stats->jpeg_items = jpeg_items_;
        stats->png_items = png_items_;
        stats->h2d_bytes = h2d_bytes_;
        stats->d2h_bytes = d2h_bytes_;
        stats->pixels = pixels_;
        stats->host_threads = threads_;
        stats->depth = depth_;
        stats->failed = failed_;
    }
    return rc;
}

} // namespace

size_t zpx::batch_slot_cache_trim()
{
    std::vector<std::pair<int, std::unique_ptr<Slot>>> out;
    {
        SlotCache &c = slot_cache();
        std::lock_guard<std::mutex> lk(c.mu);
        out.swap(c.slots);
        c.bytes = 0;
    }
    if (out.empty()) return 0;
    size_t bytes = 0;
    int cur = -1;
    (void)hipGetDevice(&cur);
    for (auto &e : out) {
        bytes += slot_bytes(*e.second);
        (void)hipSetDevice(e.first);
        destroy_slot(*e.second);
        e.second.reset(); // (its buffers, pinned words and epoch window)
    }
    if (cur >= 0) (void)hipSetDevice(cur);
    return bytes;
}

int zpx::batch_decode_rgba_hook(zpx_ctx *ctx, zpx_batch_item *items, int n_items, const zpx_batch_opts *opts,
                                zpx_batch_stats *stats, BatchDone on_done, void *user)
{
    if (!ctx || n_items < 0 || (n_items > 0 && !items)) return ZPX_E_INVALID_ARGUMENT;
    CtxScope scope(ctx);
    try {
        Pipeline p(ctx, items, n_items, opts, on_done, user);
        return p.run(stats);
    } catch (...) {
        return ZPX_E_OUT_OF_MEMORY;
    }
}

extern "C" int zpx_batch_decode_rgba(zpx_ctx *ctx, zpx_batch_item *items, int n_items, const zpx_batch_opts *opts,
                                     zpx_batch_stats *stats)
{
    return batch_decode_rgba_hook(ctx, items, n_items, opts, stats, nullptr, nullptr);
}

// zpx_batch_start's handle: the pipeline's thread, and which items are final
// (for zpx_batch_wait_prefix)
struct zpx_batch {
    std::thread th;
    int rc = ZPX_OK;
    zpx_batch_stats stats{};
    std::mutex mu;
    std::condition_variable cv;
    std::vector<uint8_t> done; // done[i]: item i is final
    int prefix = 0;            // items 0..prefix-1 are final
    bool ended = false;        // the pipeline returned
    static void on_done(void *user, int item)
    {
        zpx_batch *b = static_cast<zpx_batch *>(user);
        {
            std::lock_guard<std::mutex> lk(b->mu);
            b->done[static_cast<size_t>(item)] = 1;
            while (b->prefix < static_cast<int>(b->done.size()) && b->done[static_cast<size_t>(b->prefix)]) b->prefix++;
        }
        b->cv.notify_all();
    }
};

extern "C" int zpx_batch_start(zpx_ctx *ctx, zpx_batch_item *items, int n_items, const zpx_batch_opts *opts,
                               zpx_batch **out)
{
    if (!ctx || !out || n_items < 0 || (n_items > 0 && !items)) return ZPX_E_INVALID_ARGUMENT;
    *out = nullptr;
    zpx_batch_opts o{};
    if (opts) o = *opts;
    try {
        std::unique_ptr<zpx_batch> b(new zpx_batch);
        zpx_batch *bp = b.get();
        b->done.assign(static_cast<size_t>(n_items), 0);
        b->th = std::thread([=] {
            const int rc = batch_decode_rgba_hook(ctx, items, n_items, &o, &bp->stats, &zpx_batch::on_done, bp);
            {
                std::lock_guard<std::mutex> lk(bp->mu);
                bp->rc = rc;
                bp->ended = true;
            }
            bp->cv.notify_all();
        });
        *out = b.release();
    } catch (...) {
        return ZPX_E_OUT_OF_MEMORY;
    }
    return ZPX_OK;
}

extern "C" int zpx_batch_wait_prefix(zpx_batch *b, int n)
{
    if (!b) return ZPX_E_INVALID_ARGUMENT;
    std::unique_lock<std::mutex> lk(b->mu);
    b->cv.wait(lk, [&] { return b->prefix >= n || b->ended; });
    return b->prefix;
}

extern "C" int zpx_batch_wait(zpx_batch *b, zpx_batch_stats *stats)
{
    if (!b) return ZPX_E_INVALID_ARGUMENT;
    if (b->th.joinable()) b->th.join();
    const int rc = b->rc;
    if (stats) *stats = b->stats;
    delete b;
    return rc;
}
