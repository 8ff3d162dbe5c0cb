// configs[3] in one process: a batch of independent
// images sharded one-per-device round-robin (image i -> device i mod ndev),
// every device running its own streaming pipeline (zpx_batch_decode_rgba:
// host entropy workers + H2D + kernels) on its own host thread, and every
// result gathered into its destination on device 0 over RCCL (xGMI):
// grouped ncclSend from the owning device / ncclRecv on device 0, one
// communicator per device from ncclCommInitAll.
//
// The reference has no counterpart (zpix is single-threaded; its facade
// src/root.zig:24-40 decodes one image per call): this is the batch form of
// zpix.fromBuffer + Image.rgbaPixels (image.zig:103-130) per image.
//
// RCCL is loaded at the first call (dlopen "librccl.so.1"): a process that
// already holds torch's RCCL reuses that copy, and the library has no link
// dependency on RCCL for callers that never shard.
#include <dlfcn.h>
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstring>
#include <memory>
#include <algorithm>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "api_internal.h"
#include "zpix_amd.h"

using namespace zpx;

namespace {

// the handful of RCCL entry points used (rccl.h, ROCm 7.2)
typedef void *NcclComm;
typedef int NcclResult;
enum { kNcclUint8 = 1 };
struct Rccl {
    NcclResult (*comm_init_all)(NcclComm *, int, const int *) = nullptr;
    NcclResult (*comm_destroy)(NcclComm) = nullptr;
    NcclResult (*send)(const void *, size_t, int, int, NcclComm, hipStream_t) = nullptr;
    NcclResult (*recv)(void *, size_t, int, int, NcclComm, hipStream_t) = nullptr;
    NcclResult (*group_start)() = nullptr;
    NcclResult (*group_end)() = nullptr;
    const char *(*error_string)(NcclResult) = nullptr;
    bool ok = false;
};

const Rccl &rccl()
{
    static const Rccl r = [] {
        Rccl x;
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

int rccl_fail(zpx_ctx *ctx, NcclResult r, const char *what)
{
    std::string m = std::string(what) + ": " + (rccl().error_string ? rccl().error_string(r) : "rccl error");
    ctx->last_error = m;
    return ZPX_E_HIP;
}

int sharded(zpx_ctx *const *ctxs, int ndev, zpx_batch_item *items, int n, const zpx_batch_opts *opts,
            zpx_batch_stats *stats, zpx_gather_stats *gstats)
{
    const double t0 = now_s();
    zpx_ctx *root = ctxs[0];
    // per device: its shard's items; remote shards decode into device-local
    // staging of the caller's capacity and stride, then travel to device 0
    struct Shard {
        std::vector<int> ids;
        std::vector<zpx_batch_item> local;
        std::unique_ptr<DevBuf[]> staging; // (DevBuf is not movable)
        zpx_batch_stats st{};
        int rc = ZPX_OK;
    };
    std::vector<Shard> sh(ndev);
    for (int i = 0; i < n; i++) sh[i % ndev].ids.push_back(i);
    for (int r = 0; r < ndev; r++) {
        Shard &s = sh[r];
        s.local.resize(s.ids.size());
        if (r != 0) s.staging.reset(new DevBuf[s.ids.size()]);
        CtxScope scope(ctxs[r]);
        for (size_t k = 0; k < s.ids.size(); k++) {
            s.local[k] = items[s.ids[k]];
            if (r == 0) continue;
            if (items[s.ids[k]].dst_capacity) HIPCHK(ctxs[r], s.staging[k].alloc(items[s.ids[k]].dst_capacity));
            s.local[k].dst = s.staging[k].as<uint8_t>();
        }
    }
    // one pipeline per device, each on its own host thread
    std::vector<std::thread> th;
    for (int r = 0; r < ndev; r++)
        th.emplace_back([&, r] {
            Shard &s = sh[r];
            s.rc = zpx_batch_decode_rgba(ctxs[r], s.local.data(), static_cast<int>(s.local.size()), opts, &s.st);
        });
    for (auto &t : th) t.join();
    const double t_dec = now_s();
    int rc = ZPX_OK;
    for (int r = 0; r < ndev; r++) {
        Shard &s = sh[r];
        for (size_t k = 0; k < s.ids.size(); k++) {
            zpx_batch_item &it = items[s.ids[k]];
            it.status = s.local[k].status;
            it.width = s.local[k].width;
            it.height = s.local[k].height;
            it.format = s.local[k].format;
        }
        if (s.rc != ZPX_OK && rc == ZPX_OK) {
            rc = s.rc;
            root->last_error = ctxs[r]->last_error;
        }
    }
    // gather: every successful remote result into its destination on device
    // 0 -- RCCL between distinct devices (one communicator per device), a
    // device-to-device copy for a shard that lives on device 0's GPU itself
    double gbytes = 0;
    if (rc == ZPX_OK && ndev > 1) {
        std::vector<int> devs{root->device}; // communicator rank -> device
        std::vector<int> rank_of(ndev, 0);
        for (int r = 1; r < ndev; r++) {
            int k = 0;
            while (k < static_cast<int>(devs.size()) && devs[k] != ctxs[r]->device) k++;
            if (k == static_cast<int>(devs.size())) devs.push_back(ctxs[r]->device);
            rank_of[r] = k;
        }
        CtxScope scope(root);
        for (int r = 1; r < ndev; r++) {
            if (rank_of[r] != 0) continue;
            Shard &s = sh[r];
            for (size_t k = 0; k < s.ids.size(); k++) {
                zpx_batch_item &it = items[s.ids[k]];
                if (it.status != ZPX_OK) continue;
                const size_t b = result_bytes(it);
                HIPCHK(root, hipMemcpyAsync(it.dst, s.local[k].dst, b, hipMemcpyDeviceToDevice, root->stream));
                gbytes += double(b);
            }
        }
        if (devs.size() > 1) {
            const Rccl &R = rccl();
            if (!R.ok) {
                root->last_error = "RCCL (librccl.so.1) could not be loaded for the gather";
                return ZPX_E_UNSUPPORTED;
            }
            const int nd = static_cast<int>(devs.size());
            std::vector<NcclComm> comms(nd, nullptr);
            if (NcclResult e = R.comm_init_all(comms.data(), nd, devs.data()))
                return rccl_fail(root, e, "ncclCommInitAll");
            NcclResult e = R.group_start();
            for (int r = 1; r < ndev && !e; r++) {
                if (rank_of[r] == 0) continue;
                Shard &s = sh[r];
                for (size_t k = 0; k < s.ids.size() && !e; k++) {
                    zpx_batch_item &it = items[s.ids[k]];
                    if (it.status != ZPX_OK) continue;
                    const size_t b = result_bytes(it);
                    e = R.send(s.local[k].dst, b, kNcclUint8, 0, comms[rank_of[r]], ctxs[r]->stream);
                    if (!e) e = R.recv(it.dst, b, kNcclUint8, rank_of[r], comms[0], root->stream);
                    gbytes += double(b);
                }
            }
            const NcclResult e2 = R.group_end();
            if (!e) e = e2;
            for (int r = 0; r < ndev && !e; r++) {
                CtxScope sc(ctxs[r]);
                if (hipStreamSynchronize(ctxs[r]->stream) != hipSuccess) e = -1;
            }
            for (int k = 0; k < nd; k++) (void)R.comm_destroy(comms[k]);
            if (e) return e < 0 ? hip_fail(root, hipGetLastError(), "gather sync") : rccl_fail(root, e, "gather");
        }
        HIPCHK(root, hipStreamSynchronize(root->stream));
    }
    const double t1 = now_s();
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
            stats->failed += s.st.failed;
            stats->host_threads += s.st.host_threads;
            stats->depth = std::max(stats->depth, s.st.depth);
        }
    }
    if (gstats) {
        gstats->decode_s = t_dec - t0;
        gstats->gather_s = t1 - t_dec;
        gstats->gather_bytes = gbytes;
        gstats->ndev = ndev;
    }
    return rc;
}

} // namespace

extern "C" int zpx_batch_decode_sharded(zpx_ctx *const *ctxs, int ndev, zpx_batch_item *items, int n_items,
                                        const zpx_batch_opts *opts, zpx_batch_stats *stats,
                                        zpx_gather_stats *gather)
{
    if (!ctxs || ndev <= 0 || n_items < 0 || (n_items > 0 && !items)) return ZPX_E_INVALID_ARGUMENT;
    for (int r = 0; r < ndev; r++)
        if (!ctxs[r]) return ZPX_E_INVALID_ARGUMENT;
    try {
        return sharded(ctxs, ndev, items, n_items, opts, stats, gather);
    } catch (...) {
        return ZPX_E_OUT_OF_MEMORY;
    }
}
