// configs[3] in one process: a batch of independent
// images sharded one-per-device round-robin (image i -> device i mod ndev),
// every device running its own streaming pipeline (zpx_batch_decode_rgba:
// host entropy workers + H2D + kernels) on its own host thread, and every
// result gathered into its destination on device 0 over RCCL (xGMI) as soon
// as its device finishes it: grouped ncclSend from the owning device /
// ncclRecv on device 0, posted from one gather thread while later images
// still decode.
//
// The reference has no counterpart (zpix is single-threaded; its facade
// src/root.zig:24-40 decodes one image per call): this is the batch form of
// zpix.fromBuffer + Image.rgbaPixels (image.zig:103-130) per image, and one
// image is the unit the gather moves.
//
// RCCL is loaded at the first call (dlopen "librccl.so.1"): a process that
// already holds torch's RCCL reuses that copy, and the library has no link
// dependency on RCCL for callers that never shard.  The communicator calls
// go through a function table, so a test can put an in-process fake in
// RCCL's place (zpx_debug_shard_fake_comm) and run the send/recv branch on a
// one-GPU box.
#include <dlfcn.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <utility>
#include <vector>

#include "api_internal.h"
#include "host_cpus.h"
#include "zpix_amd.h"

using namespace zpx;

namespace {

// the handful of RCCL entry points used (rccl.h, ROCm 7.2)
typedef void *NcclComm;
typedef int NcclResult;
enum { kNcclSuccess = 0, kNcclSystemError = 2, kNcclInvalidUsage = 5, kNcclUint8 = 1 };

struct CommTable {
    NcclResult (*comm_init_all)(NcclComm *, int, const int *) = nullptr;
    NcclResult (*comm_destroy)(NcclComm) = nullptr;
    NcclResult (*send)(const void *, size_t, int, int, NcclComm, hipStream_t) = nullptr;
    NcclResult (*recv)(void *, size_t, int, int, NcclComm, hipStream_t) = nullptr;
    NcclResult (*group_start)() = nullptr;
    NcclResult (*group_end)() = nullptr;
    const char *(*error_string)(NcclResult) = nullptr;
    bool ok = false;
    bool per_context = false; // one communicator rank per context (the fake), else per distinct device
};

const CommTable &rccl()
{
    static const CommTable r = [] {
        CommTable x;
        void *h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
        if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
        if (!h) return x;
        x.comm_init_all = reinterpret_cast<decltype(x.comm_init_all)>(dlsym(h, "ncclCommInitAll"));
        x.comm_destroy = reinterpret_cast<decltype(x.comm_destroy)>(dlsym(h, "ncclCommDestroy"));
        x.send = reinterpret_cast<decltype(x.send)>(dlsym(h, "ncclSend"));
        x.recv = reinterpret_cast<decltype(x.recv)>(dlsym(h, "ncclRecv"));
        x.group_start = reinterpret_cast<decltype(x.group_start)>(dlsym(h, "ncclGroupStart"));
        x.group_end = reinterpret_cast<decltype(x.group_end)>(dlsym(h, "ncclGroupEnd"));
        x.error_string = reinterpret_cast<decltype(x.error_string)>(dlsym(h, "ncclGetErrorString"));
        x.ok = x.comm_init_all && x.comm_destroy && x.send && x.recv && x.group_start && x.group_end;
        return x;
    }();
    return r;
}

// ---------------------------------------------------------------- the fake
// An in-process communicator with RCCL's point-to-point semantics for the
// calls above: sends and receives posted inside a group are matched at the
// outermost ncclGroupEnd (send on rank s to peer p <-> the next unmatched
// receive on rank p from peer s, in posting order), and each pair becomes
// a device copy on the receive stream, ordered after the send stream's work
// so far, with the send stream ordered after the copy (the send buffer is
// free once the send stream passes it).  An unmatched operation or a size
// mismatch is ncclInvalidUsage (a real communicator would hang).
namespace fake {

struct Comm {
    int rank, nranks, device;
};
struct Op {
    bool is_send;
    const void *sbuf;
    void *rbuf;
    size_t n;
    int peer;
    Comm *comm;
    hipStream_t st;
    bool matched;
};
thread_local int g_depth = 0;
thread_local std::vector<Op> g_ops;

NcclResult comm_init_all(NcclComm *comms, int n, const int *devs)
{
    for (int r = 0; r < n; r++) comms[r] = new Comm{r, n, devs[r]};
    return kNcclSuccess;
}
NcclResult comm_destroy(NcclComm c)
{
    delete static_cast<Comm *>(c);
    return kNcclSuccess;
}

NcclResult pair(const Op &s, const Op &r)
{
    hipEvent_t sent = nullptr, copied = nullptr;
    bool ok = hipSetDevice(s.comm->device) == hipSuccess &&
              hipEventCreateWithFlags(&sent, hipEventDisableTiming) == hipSuccess &&
              hipEventRecord(sent, s.st) == hipSuccess && hipSetDevice(r.comm->device) == hipSuccess &&
              hipStreamWaitEvent(r.st, sent, 0) == hipSuccess &&
              hipMemcpyAsync(r.rbuf, s.sbuf, s.n, hipMemcpyDeviceToDevice, r.st) == hipSuccess &&
              hipEventCreateWithFlags(&copied, hipEventDisableTiming) == hipSuccess &&
              hipEventRecord(copied, r.st) == hipSuccess && hipSetDevice(s.comm->device) == hipSuccess &&
              hipStreamWaitEvent(s.st, copied, 0) == hipSuccess;
    if (sent) (void)hipEventDestroy(sent); // (released once the recorded work completes)
    if (copied) (void)hipEventDestroy(copied);
    return ok ? kNcclSuccess : kNcclSystemError;
}

NcclResult flush()
{
    std::vector<Op> ops;
    ops.swap(g_ops);
    int dev = 0;
    (void)hipGetDevice(&dev);
    NcclResult e = kNcclSuccess;
    for (Op &s : ops) {
        if (!s.is_send || e) continue;
        Op *r = nullptr;
        for (Op &c : ops)
            if (!c.is_send && !c.matched && c.comm->rank == s.peer && c.peer == s.comm->rank &&
                c.comm->nranks == s.comm->nranks) {
                r = &c;
                break;
            }
        if (!r || r->n != s.n) {
            e = kNcclInvalidUsage;
            break;
        }
        r->matched = s.matched = true;
        e = pair(s, *r);
    }
    for (const Op &o : ops)
        if (!e && !o.matched) e = kNcclInvalidUsage;
    (void)hipSetDevice(dev);
    return e;
}

NcclResult post(const Op &o)
{
    if (!o.comm || o.peer < 0 || o.peer >= o.comm->nranks || o.peer == o.comm->rank) return kNcclInvalidUsage;
    g_ops.push_back(o);
    return g_depth ? kNcclSuccess : flush();
}
NcclResult send(const void *b, size_t n, int type, int peer, NcclComm c, hipStream_t st)
{
    if (type != kNcclUint8) return kNcclInvalidUsage;
    return post(Op{true, b, nullptr, n, peer, static_cast<Comm *>(c), st, false});
}
NcclResult recv(void *b, size_t n, int type, int peer, NcclComm c, hipStream_t st)
{
    if (type != kNcclUint8) return kNcclInvalidUsage;
    return post(Op{false, nullptr, b, n, peer, static_cast<Comm *>(c), st, false});
}
NcclResult group_start()
{
    g_depth++;
    return kNcclSuccess;
}
NcclResult group_end()
{
    if (g_depth <= 0) return kNcclInvalidUsage;
    return --g_depth ? kNcclSuccess : flush();
}
const char *error_string(NcclResult e)
{
    return e == kNcclInvalidUsage ? "invalid usage (fake communicator)" : "system error (fake communicator)";
}

const CommTable &table()
{
    static const CommTable t = [] {
        CommTable x;
        x.comm_init_all = comm_init_all;
        x.comm_destroy = comm_destroy;
        x.send = send;
        x.recv = recv;
        x.group_start = group_start;
        x.group_end = group_end;
        x.error_string = error_string;
        x.ok = true;
        x.per_context = true;
        return x;
    }();
    return t;
}

} // namespace fake

std::atomic<int> g_use_fake{0};

// Communicators per (table, device list), created at the first call that
// needs them and kept (ncclCommInitAll costs far more than a gather; it used
// to run inside every call's gather window).  A call checks its set out for
// its whole gather (`use`): RCCL forbids driving one communicator from two
// threads at once, so two concurrent sharded calls on the same device set
// take turns.  zpx_ctx_destroy releases the sets holding its device
// (shard_release_comms).
struct CommSet {
    const CommTable *table = nullptr;
    std::vector<int> devs;
    std::vector<NcclComm> comms;
    std::mutex use;
};
std::mutex g_comm_mu;
std::map<std::pair<const CommTable *, std::vector<int>>, std::shared_ptr<CommSet>> g_comms;

NcclResult get_comms(const CommTable &T, const std::vector<int> &devs, std::shared_ptr<CommSet> &out)
{
    std::lock_guard<std::mutex> lk(g_comm_mu);
    auto key = std::make_pair(&T, devs);
    auto it = g_comms.find(key);
    if (it == g_comms.end()) {
        auto cs = std::make_shared<CommSet>();
        cs->table = &T;
        cs->devs = devs;
        cs->comms.assign(devs.size(), nullptr);
        int dev = 0;
        (void)hipGetDevice(&dev);
        const NcclResult e = T.comm_init_all(cs->comms.data(), static_cast<int>(devs.size()), devs.data());
        (void)hipSetDevice(dev);
        if (e) return e;
        it = g_comms.emplace(key, std::move(cs)).first;
    }
    out = it->second;
    return kNcclSuccess;
}

double now_s()
{
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// bytes of an RGBA8 result at `stride` (the last row is 4W, not stride)
size_t result_bytes(const zpx_batch_item &it)
{
    const size_t stride = it.dst_stride ? it.dst_stride : size_t(it.width) * 4;
    return it.height ? (size_t(it.height) - 1) * stride + size_t(it.width) * 4 : 0;
}

std::string comm_error(const CommTable &T, NcclResult r, const char *what)
{
    return std::string(what) + ": " + (T.error_string ? T.error_string(r) : "rccl error");
}

struct Stream { // a non-blocking stream on one device (RAII)
    hipStream_t s = nullptr;
    int device = 0;
    ~Stream()
    {
        if (!s) return;
        (void)hipSetDevice(device);
        (void)hipStreamSynchronize(s);
        (void)hipStreamDestroy(s);
    }
};

struct Shard {
    std::vector<int> ids;              // global item ids, in order
    std::vector<zpx_batch_item> local; // the pipeline's items (remote: dst = staging)
    std::unique_ptr<DevBuf[]> staging; // (DevBuf is not movable)
    std::vector<uint8_t> arrived;      // remote item k reached device 0
    zpx_batch_stats st{};
    int rc = ZPX_OK;
    std::string err;
};

struct Gather { // what the pipeline threads hand the gather thread
    std::mutex mu;
    std::condition_variable cv;
    std::deque<std::pair<int, int>> ready; // (shard, local index) of finished items
    int running = 0;
    double t_dec = 0; // when the last pipeline returned
};

struct HookArg {
    Gather *g;
    int r;
};

void on_item_done(void *user, int k)
{
    HookArg *a = static_cast<HookArg *>(user);
    {
        std::lock_guard<std::mutex> lk(a->g->mu);
        a->g->ready.emplace_back(a->r, k);
    }
    a->g->cv.notify_one();
}

int sharded(zpx_ctx *const *ctxs, int ndev, zpx_batch_item *items, int n, const zpx_batch_opts *opts,
            zpx_batch_stats *stats, zpx_gather_stats *gstats)
{
    zpx_ctx *root = ctxs[0];
    const CommTable &T = g_use_fake.load() ? fake::table() : rccl();
    // communicator ranks: rank 0 is device 0's GPU; RCCL has one rank per
    // distinct device (a context on device 0's GPU takes a device copy), the
    // fake one per context
    std::vector<int> devs{root->device};
    std::vector<int> rank_of(ndev, 0);
    for (int r = 1; r < ndev; r++) {
        int k = 0;
        if (T.per_context) {
            k = static_cast<int>(devs.size());
        } else {
            while (k < static_cast<int>(devs.size()) && devs[k] != ctxs[r]->device) k++;
        }
        if (k == static_cast<int>(devs.size())) devs.push_back(ctxs[r]->device);
        rank_of[r] = k;
    }
    // test switch "shard_rccl_self": a shard on device 0's GPU sends its
    // results over RCCL too -- grouped ncclSend / ncclRecv to itself on rank
    // 0's communicator (a one-rank communicator when every shard shares the
    // GPU) -- instead of a device copy, so the real library's loading, group
    // semantics and stream ordering run on a one-GPU box
    bool self_send = false;
    if (!T.per_context && opt(Opt::ShardRcclSelf) != 0)
        for (int r = 1; r < ndev; r++) self_send |= rank_of[r] == 0;
    const double tc = now_s();
    std::shared_ptr<CommSet> cset;
    std::unique_lock<std::mutex> in_use; // this call's turn on the communicator set
    if ((devs.size() > 1 || self_send) && n > 1) { // (some item lives on a rank other than 0, or sends to itself)
        if (!T.ok) {
            root->last_error = "RCCL (librccl.so.1) could not be loaded for the gather";
            return ZPX_E_UNSUPPORTED;
        }
        for (;;) {
            if (NcclResult e = get_comms(T, devs, cset)) {
                root->last_error = comm_error(T, e, "ncclCommInitAll");
                return ZPX_E_HIP;
            }
            in_use = std::unique_lock<std::mutex>(cset->use);
            if (!cset->comms.empty()) break;
            in_use.unlock(); // released (shard_release_comms) between the lookup and the lock: again
        }
    }
    const std::vector<NcclComm> comms = cset ? cset->comms : std::vector<NcclComm>();
    const double comm_setup_s = now_s() - tc;

    const double t0 = now_s();
    std::vector<Shard> sh(ndev);
    for (int i = 0; i < n; i++) sh[i % ndev].ids.push_back(i);
    for (int r = 0; r < ndev; r++) {
        Shard &s = sh[r];
        s.local.resize(s.ids.size());
        s.arrived.assign(s.ids.size(), 0);
        if (r != 0) s.staging.reset(new DevBuf[s.ids.size()]);
        CtxScope scope(ctxs[r]);
        for (size_t k = 0; k < s.ids.size(); k++) {
            s.local[k] = items[s.ids[k]];
            if (r == 0) continue;
            if (items[s.ids[k]].dst_capacity) HIPCHK(ctxs[r], s.staging[k].alloc(items[s.ids[k]].dst_capacity));
            s.local[k].dst = s.staging[k].as<uint8_t>();
        }
    }
    // gather streams: one on device 0 (receives, device copies), one per
    // remote shard (its sends); a pipeline's own streams stay its own
    std::vector<Stream> gs(ndev);
    for (int r = 0; r < ndev; r++) {
        if (r != 0 && rank_of[r] == 0) continue;
        gs[r].device = ctxs[r]->device;
        CtxScope scope(ctxs[r]);
        HIPCHK(root, hipStreamCreateWithFlags(&gs[r].s, hipStreamNonBlocking));
    }
    // per device: its share of the host's CPUs for the entropy / inflate
    // workers (ndev pipelines on one budget, as shard.rank_cpus splits it
    // between processes)
    zpx_batch_opts o{};
    if (opts) o = *opts;
    if (o.host_threads <= 0) o.host_threads = std::max(1, std::min(16, host_cpu_budget() / ndev));

    Gather g;
    g.running = ndev;
    std::vector<HookArg> hook(ndev);
    std::vector<std::thread> th;
    bool started = true;
    try {
        th.reserve(static_cast<size_t>(ndev));
        for (int r = 0; r < ndev; r++) {
            hook[r] = HookArg{&g, r};
            th.emplace_back([&, r] {
                Shard &s = sh[r];
                s.rc = batch_decode_rgba_hook(ctxs[r], s.local.data(), static_cast<int>(s.local.size()), &o, &s.st,
                                              r == 0 ? nullptr : on_item_done, &hook[r]);
                if (s.rc != ZPX_OK) s.err = ctxs[r]->last_error;
                {
                    std::lock_guard<std::mutex> lk(g.mu);
                    if (--g.running == 0) g.t_dec = now_s();
                }
                g.cv.notify_one();
            });
        }
    } catch (...) {
        started = false;
    }
    if (!started) { // the threads already running finish their shards, then the call fails
        for (auto &t : th) t.join();
        return ZPX_E_OUT_OF_MEMORY;
    }
    // the gather thread (this one): each finished remote item moves at once
    double gbytes = 0, t_first = 0;
    int gerr = ZPX_OK;
    std::string gmsg;
    for (;;) {
        std::deque<std::pair<int, int>> batch;
        {
            std::unique_lock<std::mutex> lk(g.mu);
            g.cv.wait(lk, [&] { return !g.ready.empty() || g.running == 0; });
            batch.swap(g.ready);
            if (batch.empty() && g.running == 0) break;
        }
        for (const auto &rk : batch) {
            const int r = rk.first;
            const size_t k = static_cast<size_t>(rk.second);
            Shard &s = sh[r];
            const zpx_batch_item &li = s.local[k];
            if (li.status != ZPX_OK || gerr != ZPX_OK) continue;
            zpx_batch_item &it = items[s.ids[k]];
            const size_t b = result_bytes(li);
            if (t_first == 0) t_first = now_s();
            if (rank_of[r] == 0 && !self_send) { // device 0's own GPU: a device copy
                CtxScope scope(root);
                const hipError_t e = hipMemcpyAsync(it.dst, li.dst, b, hipMemcpyDeviceToDevice, gs[0].s);
                if (e != hipSuccess) {
                    gerr = hip_fail(root, e, "gather copy");
                    gmsg = root->last_error;
                    continue;
                }
            } else {
                // (a self send/recv pair: both on rank 0's communicator and
                // gather stream, which RCCL turns into a local copy kernel)
                const hipStream_t ss = rank_of[r] == 0 ? gs[0].s : gs[r].s;
                NcclResult e = T.group_start();
                if (!e) e = T.send(li.dst, b, kNcclUint8, 0, comms[rank_of[r]], ss);
                if (!e) e = T.recv(it.dst, b, kNcclUint8, rank_of[r], comms[0], gs[0].s);
                const NcclResult e2 = T.group_end();
                if (!e) e = e2;
                if (e) {
                    gerr = ZPX_E_HIP;
                    gmsg = comm_error(T, e, "gather send/recv");
                    continue;
                }
            }
            s.arrived[k] = 1;
            gbytes += double(b);
        }
    }
    for (auto &t : th) t.join();
    // every transfer complete
    for (int r = 0; r < ndev; r++) {
        if (!gs[r].s) continue;
        CtxScope scope(ctxs[r]);
        const hipError_t e = hipStreamSynchronize(gs[r].s);
        if (e != hipSuccess && gerr == ZPX_OK) {
            gerr = hip_fail(root, e, "gather sync");
            gmsg = root->last_error;
            std::fill(sh[r].arrived.begin(), sh[r].arrived.end(), 0);
            if (r == 0)
                for (int q = 1; q < ndev; q++) std::fill(sh[q].arrived.begin(), sh[q].arrived.end(), 0);
        }
    }
    const double t1 = now_s();
    // statuses: device 0's items as decoded; a remote item is Ok only once it
    // arrived, else it carries its shard's error (or the gather's)
    int rc = ZPX_OK;
    for (int r = 0; r < ndev; r++) {
        Shard &s = sh[r];
        for (size_t k = 0; k < s.ids.size(); k++) {
            zpx_batch_item &it = items[s.ids[k]];
            it.status = s.local[k].status;
            it.width = s.local[k].width;
            it.height = s.local[k].height;
            it.format = s.local[k].format;
            if (r != 0 && it.status == ZPX_OK && !s.arrived[k])
                it.status = s.rc != ZPX_OK ? s.rc : gerr != ZPX_OK ? gerr : ZPX_E_HIP;
        }
        if (s.rc != ZPX_OK && rc == ZPX_OK) {
            rc = s.rc;
            root->last_error = s.err;
        }
    }
    if (rc == ZPX_OK && gerr != ZPX_OK) {
        rc = gerr;
        root->last_error = gmsg;
    }
    if (stats) {
        memset(stats, 0, sizeof(*stats));
        stats->wall_s = t1 - t0;
        for (auto &s : sh) {
            stats->host_s += s.st.host_s;
            stats->host_jpeg_s += s.st.host_jpeg_s;
            stats->host_png_s += s.st.host_png_s;
            stats->jpeg_items += s.st.jpeg_items;
            stats->png_items += s.st.png_items;
            stats->h2d_bytes += s.st.h2d_bytes;
            stats->d2h_bytes += s.st.d2h_bytes;
            stats->pixels += s.st.pixels;
            stats->host_threads += s.st.host_threads;
            stats->depth = std::max(stats->depth, s.st.depth);
        }
        for (int i = 0; i < n; i++) stats->failed += items[i].status != ZPX_OK;
    }
    if (gstats) {
        memset(gstats, 0, sizeof(*gstats));
        const double t_dec = g.t_dec > 0 ? g.t_dec : t1;
        gstats->decode_s = t_dec - t0;
        gstats->gather_s = t_first > 0 ? t1 - t_first : 0;
        gstats->tail_s = t1 - t_dec;
        gstats->gather_bytes = gbytes;
        gstats->ndev = ndev;
        gstats->comm_setup_s = comm_setup_s;
        gstats->comm_ranks = static_cast<int32_t>(devs.size());
    }
    return rc;
}

} // namespace

void zpx::shard_release_comms(int device)
{
    std::vector<std::shared_ptr<CommSet>> drop;
    {
        std::lock_guard<std::mutex> lk(g_comm_mu);
        for (auto it = g_comms.begin(); it != g_comms.end();) {
            const auto &d = it->second->devs;
            if (std::find(d.begin(), d.end(), device) != d.end()) {
                drop.push_back(it->second);
                it = g_comms.erase(it);
            } else {
                ++it;
            }
        }
    }
    int cur = 0;
    (void)hipGetDevice(&cur);
    for (auto &cs : drop) {
        std::lock_guard<std::mutex> lk(cs->use); // a call still gathering on it finishes first
        for (NcclComm c : cs->comms)
            if (c) (void)cs->table->comm_destroy(c);
        cs->comms.clear();
    }
    (void)hipSetDevice(cur);
}

extern "C" int zpx_batch_decode_sharded(zpx_ctx *const *ctxs, int ndev, zpx_batch_item *items, int n_items,
                                        const zpx_batch_opts *opts, zpx_batch_stats *stats,
                                        zpx_gather_stats *gather)
{
    if (!ctxs || ndev <= 0 || n_items < 0 || (n_items > 0 && !items)) return ZPX_E_INVALID_ARGUMENT;
    if (opts && opts->dst_on_host) return ZPX_E_INVALID_ARGUMENT; // results gather into device memory
    for (int r = 0; r < ndev; r++)
        if (!ctxs[r]) return ZPX_E_INVALID_ARGUMENT;
    try {
        return sharded(ctxs, ndev, items, n_items, opts, stats, gather);
    } catch (...) {
        return ZPX_E_OUT_OF_MEMORY;
    }
}

extern "C" int zpx_debug_shard_fake_comm(int on)
{
    return g_use_fake.exchange(on ? 1 : 0);
}
