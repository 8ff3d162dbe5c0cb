// C-ABI of the MI355X decode path (include/zpix_amd.h): contexts, device
// plans, and the drop-in jpeg/png/image entry points.  Host entropy stages
// live in jpeg_host.cpp / png_host.cpp; pixel loops in the .hip kernels.
// There is no CPU pixel path: every reconstruct / unfilter / colour step is a
// kernel launch, and a HIP failure is reported as ZPX_E_HIP.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <unistd.h>
#include <cstdio>
#include <cstdlib>
#include <atomic>
#include <cstring>
#include <map>
#include <memory>
#include <string>
#include <tuple>
#include <vector>

#include "api_internal.h"
#include "inflate_fast.h"
#include "device_types.h"
#include "jpeg_host.h"
#include "kernels.h"
#include "png_host.h"
#include "zpix_amd.h"

using namespace zpx;

// ------------------------------------------------------------------ errors
static const char *const kErrorNames[] = {
#define ZPX_NAME_(name, up) #name,
    ZPX_ERROR_LIST(ZPX_NAME_)
#undef ZPX_NAME_
};

extern "C" int zpx_abi_version(void) { return ZPX_ABI_VERSION; }
extern "C" size_t zpx_host_pools_trim(void) { return zpx::png_pool_trim(); }
extern "C" size_t zpx_batch_cache_trim(void) { return zpx::batch_slot_cache_trim(); }

extern "C" const char *zpx_error_name(int code)
{
    if (code < 0 || code >= ZPX_E__COUNT) return "Unknown";
    return kErrorNames[code];
}

extern "C" const char *zpx_last_error(const zpx_ctx *ctx) { return ctx ? ctx->last_error.c_str() : ""; }

// ------------------------------------------------------------------ context
static int zpx_ctx_create_impl(int device, zpx_ctx **out)
{
    if (!out) return ZPX_E_INVALID_ARGUMENT;
    *out = nullptr;
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess || n <= 0 || device < 0 || device >= n) return ZPX_E_HIP;
    std::unique_ptr<zpx_ctx> c(new zpx_ctx);
    c->device = device;
    if (hipSetDevice(device) != hipSuccess) return ZPX_E_HIP;
    if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) return ZPX_E_HIP;
    *out = c.release();
    return ZPX_OK;
}

extern "C" int zpx_ctx_create(int device, zpx_ctx **out)
{
    return guarded([&] { return zpx_ctx_create_impl(device, out); });
}

extern "C" void zpx_ctx_destroy(zpx_ctx *ctx)
{
    if (!ctx) return;
    shard_release_comms(ctx->device);
    (void)hipSetDevice(ctx->device);
    if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
    if (ctx->scratch_ev) {
        (void)hipEventSynchronize(ctx->scratch_ev);
        (void)hipEventDestroy(ctx->scratch_ev);
    }
    if (ctx->scratch) (void)hipFree(ctx->scratch);
    delete ctx;
}

extern "C" void *zpx_ctx_stream(zpx_ctx *ctx) { return ctx ? ctx->stream : nullptr; }
extern "C" int zpx_ctx_device(const zpx_ctx *ctx) { return ctx ? ctx->device : -1; }
extern "C" int zpx_ctx_synchronize(zpx_ctx *ctx)
{
    if (!ctx) return ZPX_E_INVALID_ARGUMENT;
    CtxScope s(ctx);
    HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
    return ZPX_OK;
}

// ------------------------------------------------------------------ image
extern "C" void zpx_image_free(const zpx_allocator *al, zpx_image *img)
{
    if (!img) return;
    al_free(al, img->pixels, img->pixels_len);
    if (img->palette) al_free(al, img->palette, 256 * sizeof(zpx_color));
    img->pixels = nullptr;
    img->palette = nullptr;
    img->pixels_len = 0;
}

DevImage zpx::dev_image_of(const zpx_image *img, const void *d_pixels, const void *d_palette)
{
    DevImage m{};
    m.pixels = static_cast<const uint8_t *>(d_pixels);
    m.palette = static_cast<const uint8_t *>(d_palette);
    m.stride = img->stride;
    m.y_off = img->y_off;
    m.cb_off = img->cb_off;
    m.cr_off = img->cr_off;
    m.y_stride = img->y_stride;
    m.c_stride = img->c_stride;
    m.kind = img->kind;
    m.subsample = img->subsample;
    m.width = img->max_x - img->min_x;
    m.height = img->max_y - img->min_y;
    m.palette_len = img->palette_len;
    return m;
}

// A Paletted image's palette as the colour kernels read it: at most 256
// entries (an index byte's range; the kernel reads entry i < palette_len),
// present whenever it has any
static bool palette_ok(const zpx_image &im)
{
    if (im.kind != ZPX_PALETTED) return true;
    return im.palette_len >= 0 && im.palette_len <= 256 && (im.palette_len == 0 || im.palette != nullptr);
}

extern "C" int zpx_dev_rgba_pixels(zpx_ctx *ctx, const zpx_image *img, uint8_t *out, void *stream)
{
    if (!ctx || !img || !out) return ZPX_E_INVALID_ARGUMENT;
    if (!palette_ok(*img)) return ZPX_E_INVALID_ARGUMENT;
    if (img->min_x != 0 || img->min_y != 0) return ZPX_E_UNSUPPORTED; // decoders always return min = (0,0)
    CtxScope s(ctx);
    const DevImage m = dev_image_of(img, img->pixels, img->palette);
    hipStream_t st = stream ? static_cast<hipStream_t>(stream) : ctx->stream;
    if (launch_rgba_pixels(m, out, st)) return hip_fail(ctx, hipGetLastError(), "rgba_pixels_kernel");
    return ZPX_OK;
}

static int zpx_image_rgba_pixels_impl(zpx_ctx *ctx, const zpx_allocator *al, const zpx_image *img, uint8_t **out,
                                     size_t *out_len)
{
    if (!ctx || !img || !out || !out_len) return ZPX_E_INVALID_ARGUMENT;
    *out = nullptr;
    *out_len = 0;
    if (!palette_ok(*img)) return ZPX_E_INVALID_ARGUMENT;
    if (img->min_x != 0 || img->min_y != 0) return ZPX_E_UNSUPPORTED;
    CtxScope s(ctx);
    const size_t w = size_t(img->max_x - img->min_x), h = size_t(img->max_y - img->min_y);
    const size_t n = w * h * 4;
    DevBuf dpix, dpal, dout;
    HIPCHK(ctx, dpix.alloc(img->pixels_len));
    HIPCHK(ctx, hipMemcpyAsync(dpix.ptr, img->pixels, img->pixels_len, hipMemcpyHostToDevice, ctx->stream));
    if (img->kind == ZPX_PALETTED && img->palette_len > 0) { // (its palette_len entries: the rest are never read)
        HIPCHK(ctx, dpal.alloc(256 * sizeof(zpx_color)));
        HIPCHK(ctx, hipMemcpyAsync(dpal.ptr, img->palette, size_t(img->palette_len) * sizeof(zpx_color),
                                   hipMemcpyHostToDevice, ctx->stream));
    }
    HIPCHK(ctx, dout.alloc(n));
    const DevImage m = dev_image_of(img, dpix.ptr, dpal.ptr);
    if (n && launch_rgba_pixels(m, dout.as<uint8_t>(), ctx->stream))
        return hip_fail(ctx, hipGetLastError(), "rgba_pixels_kernel");
    uint8_t *host = static_cast<uint8_t *>(al_alloc(al, n));
    if (!host) return ZPX_E_OUT_OF_MEMORY;
    hipError_t e = hipMemcpyAsync(host, dout.ptr, n, hipMemcpyDeviceToHost, ctx->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
    if (e != hipSuccess) {
        al_free(al, host, n);
        return hip_fail(ctx, e, "rgba_pixels copy-back");
    }
    *out = host;
    *out_len = n;
    return ZPX_OK;
}

extern "C" int zpx_image_rgba_pixels(zpx_ctx *ctx, const zpx_allocator *al, const zpx_image *img, uint8_t **out,
                                     size_t *out_len)
{
    return guarded([&] { return zpx_image_rgba_pixels_impl(ctx, al, img, out, out_len); });
}

// ------------------------------------------------------------------ plans
DevJpegFrame zpx::dev_jpeg_frame(const zpx_jpeg_frame &f)
{
    DevJpegFrame d{};
    for (int c = 0; c < 4; c++) {
        d.coeffs[c] = c < f.n_comp ? f.coeffs[c] : nullptr;
        d.planes[c] = f.planes[c];
        d.strides[c] = f.strides[c];
        d.h[c] = f.h[c];
        d.v[c] = f.v[c];
        d.rule[c] = c < f.n_comp ? f.rule[c] : ZPX_BLOCKS_NONE;
        memcpy(d.qt[c], f.qt[c], sizeof(d.qt[c]));
    }
    // quant-pair tables (jpeg_block_kernels.hip, idct_block_pairs); tables are at most 16-bit
    static const int kLo[4] = {1, 5, 2, 0}, kHi[4] = {7, 3, 6, 4};
    for (int c = 0; c < 4; c++)
        for (int i = 0; i < 32; i++) {
            const int r = i >> 2, k = i & 3;
            d.qp[c][i] = (static_cast<uint32_t>(f.qt[c][8 * r + kLo[k]]) & 0xffffu) |
                         static_cast<uint32_t>(f.qt[c][8 * r + kHi[k]]) << 16;
        }
    if (f.n_comp == 1) d.h[0] = d.v[0] = 1;
    d.rgba = f.rgba;
    d.rgba_stride = f.rgba_stride;
    d.width = static_cast<int32_t>(f.width);
    d.height = static_cast<int32_t>(f.height);
    d.mxx = f.mxx;
    d.myy = f.myy;
    d.n_comp = f.n_comp;
    d.color = f.color;
    d.pieces = f.layout == ZPX_COEFFS_PIECES ? static_cast<const uint8_t *>(f.pieces) : nullptr;
    return d;
}

JpegPlaneGeom zpx::jpeg_plane_geom(const DevJpegFrame &d)
{
    JpegPlaneGeom g;
    g.ncomp = d.n_comp;
    for (int c = 0; c < 4; c++) {
        g.h[c] = c < d.n_comp ? d.h[c] : 1;
        g.v[c] = c < d.n_comp ? d.v[c] : 1;
    }
    g.max_mxx = d.mxx;
    g.max_myy = d.myy;
    return g;
}

bool zpx::jpeg_fusable(const zpx_jpeg_frame &f)
{
    if (f.n_comp == 4) return false;
    const int color = f.n_comp == 1 ? ZPX_JPEG_COLOR_GRAY : f.color;
    const int h0 = f.n_comp == 1 ? 1 : f.h[0], v0 = f.n_comp == 1 ? 1 : f.v[0];
    const int hc = f.n_comp == 3 ? f.h[1] : 1, vc = f.n_comp == 3 ? f.v[1] : 1;
    return jpeg_rgba_supported(color, h0, v0, hc, vc);
}

int zpx::launch_jpeg_rgba_frame(const zpx_jpeg_frame &f, const DevJpegFrame *d_frame, hipStream_t st)
{
    const int color = f.n_comp == 1 ? ZPX_JPEG_COLOR_GRAY : f.color;
    const int h0 = f.n_comp == 1 ? 1 : f.h[0], v0 = f.n_comp == 1 ? 1 : f.v[0];
    const int hc = f.n_comp == 3 ? f.h[1] : 1, vc = f.n_comp == 3 ? f.v[1] : 1;
    return launch_jpeg_rgba(d_frame, 1, color, h0, v0, hc, vc, f.mxx, f.myy, f.coeff_bits, f.narrow != 0,
                            jpeg_rgba_vec_out(f), f.layout == ZPX_COEFFS_PIECES, st);
}

bool zpx::jpeg_rgba_vec_out(const zpx_jpeg_frame &f)
{
    // dword-aligned RGBA rows, any width (the block kernel stores a row's
    // partial last 4-pixel piece as dwords)
    return (f.rgba_stride & 3) == 0 && (reinterpret_cast<uintptr_t>(f.rgba) & 3) == 0;
}
// jpeg.decode's planes (reconstructBlock into makeImg's layout) followed by
// the colour pass of Image.rgbaPixels, for the frames the fused kernel does
// not take: Adobe RGB (convertToRGB, decoder.zig:751-783), CMYK (applyBlack,
// :792-902), Gray/YCbCr from non-interleaved scans.  `f` carries DEVICE
// coefficient pointers; everything is enqueued on `st` (no host sync): the
// planes go to `planes`, the descriptor through pinned `hdesc` to `desc`, and
// RGBA8 (stride 4W) to `out`.
int zpx::jpeg_planes_to_rgba(zpx_ctx *ctx, const JpegCoeffs &c, zpx_jpeg_frame f, DevBuf &planes, DevBuf &desc,
                             HostBuf &hdesc, uint8_t *out, hipStream_t st)
{
    const JpegOut kind = jpeg_output_kind(c);
    if (c.n_comp == 4 && !c.adobe_valid) return ZPX_E_UNSUPPORTED_COLOR_MODEL; // applyBlack :793-795
    if (kind == JpegOut::YCCK) {
        ctx->last_error = "YCbCrK (Adobe transform 2) goes through image/util.zig drawYCbCr: out of scope";
        return ZPX_E_UNSUPPORTED;
    }
    JpegLayout L;
    if (int e = jpeg_layout(c, L)) return e;
    const size_t kofs = (L.total + 255) & ~size_t(255);
    const size_t cmyk_ofs = (kofs + L.k_total + 255) & ~size_t(255); // CMYK image (kind CMYK, 4 B/px)
    const size_t cmyk_bytes = kind == JpegOut::CMYK ? size_t(c.width) * c.height * 4 : 0;
    HIPCHK(ctx, planes.reserve(cmyk_ofs + cmyk_bytes));
    HIPCHK(ctx, hipMemsetAsync(planes.ptr, 0, kofs + L.k_total, st)); // makeImg zeroes (image.zig:505-507)
    uint8_t *pb = planes.as<uint8_t>();
    f.planes[0] = pb;
    f.strides[0] = L.y_stride;
    if (c.n_comp >= 3) {
        f.planes[1] = pb + L.cb_off;
        f.planes[2] = pb + L.cr_off;
        f.strides[1] = f.strides[2] = L.c_stride;
    }
    if (c.n_comp == 4) {
        f.planes[3] = pb + kofs;
        f.strides[3] = L.k_stride;
    }
    const DevJpegFrame df = dev_jpeg_frame(f);
    if (hdesc.bytes < sizeof(df) && !hdesc.alloc(sizeof(df), false)) return ZPX_E_OUT_OF_MEMORY;
    memcpy(hdesc.ptr, &df, sizeof(df));
    HIPCHK(ctx, desc.reserve(sizeof(df)));
    HIPCHK(ctx, hipMemcpyAsync(desc.ptr, hdesc.ptr, sizeof(df), hipMemcpyHostToDevice, st));
    if (launch_jpeg_planar(desc.as<DevJpegFrame>(), 1, jpeg_plane_geom(df), f.coeff_bits, f.narrow != 0, false, st))
        return hip_fail(ctx, hipGetLastError(), "jpeg planar kernel");
    zpx_image planar{};
    planar.kind = c.n_comp == 1 ? ZPX_GRAY : ZPX_YCBCR;
    planar.max_x = static_cast<int32_t>(c.width);
    planar.max_y = static_cast<int32_t>(c.height);
    planar.stride = L.y_stride;
    planar.y_stride = L.y_stride;
    planar.c_stride = L.c_stride;
    planar.cb_off = L.cb_off;
    planar.cr_off = L.cr_off;
    planar.subsample = L.subsample;
    const DevImage m = dev_image_of(&planar, pb, nullptr);
    int rc;
    if (kind == JpegOut::RGB) {
        rc = launch_jpeg_rgb(m, c.comp[0].h / c.comp[1].h, out, st);
    } else if (kind == JpegOut::CMYK) {
        uint32_t sub = 0;
        for (int t = 0; t < 4; t++)
            if (c.comp[t].h != c.comp[0].h || c.comp[t].v != c.comp[0].v) sub |= 1u << t;
        // applyBlack builds the CMYK image; rgbaPixels converts it (color.zig:115-121)
        rc = launch_jpeg_cmyk(m, pb + kofs, L.k_stride, sub, pb + cmyk_ofs, st);
        if (!rc) {
            zpx_image cm{};
            cm.kind = ZPX_CMYK;
            cm.max_x = static_cast<int32_t>(c.width);
            cm.max_y = static_cast<int32_t>(c.height);
            cm.stride = size_t(c.width) * 4;
            rc = launch_rgba_pixels(dev_image_of(&cm, pb + cmyk_ofs, nullptr), out, st);
        }
    } else {
        rc = launch_rgba_pixels(m, out, st); // Gray / YCbCr: Color.toRGBA (color.zig:90-126)
    }
    if (rc) return hip_fail(ctx, hipGetLastError(), "jpeg colour kernel");
    return ZPX_OK;
}

struct JpegGroup {
    DevBuf frames;
    int n = 0;
    int bits = 16;
    bool narrow = true;
    int color = 0, h0 = 1, v0 = 1, hc = 1, vc = 1;
    int max_gw = 0, max_gh = 0, max_mxx = 0, max_myy = 0;
    bool vec_out = true; // every frame: dword-aligned RGBA rows (jpeg_rgba_vec_out)
    JpegPlaneGeom geom;  // planes output: the group's geometry (one per group)
    // ZPX_COEFFS_PIECES frames: read by the block kernels directly (pieces),
    // or expanded into the group's own dense grids at every launch first
    // (expand_jobs; `frames` then points at the grids)
    bool pieces = false;
    DevBuf grids, expand_jobs;
    int nexpand = 0;
    uint32_t expand_max_blocks = 0;
};
struct PngGroup {
    int depth = 0;
    bool pair = false; // png_pair_kernel (128-row bands) or png_unfilter_kernel (64)
    bool trns = false; // (pair kernel) the images carry a tRNS colour key
    bool stream = false; // (pair kernel) its stream instance: the frames' inflated streams as they are
    DevBuf passes, sched, boundary;
    PngControl ctl; // {epoch, ticket, status, sticky, ...} and the group's epoch window
    uint32_t nsched = 0, band_bytes = 0, nbands = 0;
    DevBuf staging, merge_jobs; // Adam7 passes 1-5 and pass 6's merge jobs (Adam7Stage)
    // stream-layout frames of the paired-row kernel under the test switch
    // png_device_slab: their band slabs, built on the device before the
    // kernel (png_slab_kernels.hip)
    DevBuf dslab, slab_jobs;
    uint32_t nslab_jobs = 0, slab_max_groups = 0;
    uint32_t nsched2 = 0;       // bands of the second launch (Adam7 pass 6), after the first nsched
};

struct RgbaGroup {
    int kind = 0, n = 0, max_w = 0, max_h = 0;
    DevBuf jobs; // DevRgbaJob per image
};

struct zpx_plan {
    zpx_ctx *ctx = nullptr;
    int kind = 0; // 0 jpeg planes, 1 jpeg rgba, 2 png, 3 rgbaPixels
    std::vector<std::unique_ptr<RgbaGroup>> rgba;
    std::vector<std::unique_ptr<JpegGroup>> jpeg;
    std::vector<std::unique_ptr<PngGroup>> png;
    HostBuf status_host; // pinned: per PNG group {status, sticky status}
    uint64_t bytes = 0;
};

// A group of ZPX_COEFFS_PIECES frames that the block kernels read directly
// (the others are expanded into dense grids first)
static bool jpeg_pieces_direct(int output, const JpegGroup &g)
{
    if (!g.narrow || (g.bits != 8 && g.bits != 16) || opt(Opt::JpegStrip) != 0) return false;
    if (output == ZPX_JPEG_PLANES) return true;
    return g.vec_out && jpeg_block_pieces_supported(g.color, g.h0, g.v0, g.hc, g.vc);
}

static int zpx_jpeg_plan_create_impl(zpx_ctx *ctx, const zpx_jpeg_frame *frames, int n_frames, int output,
                                    zpx_plan **out)
{
    if (!ctx || !frames || n_frames <= 0 || !out) return ZPX_E_INVALID_ARGUMENT;
    if (output != ZPX_JPEG_PLANES && output != ZPX_JPEG_RGBA) return ZPX_E_INVALID_ARGUMENT;
    *out = nullptr;
    CtxScope s(ctx);
    std::unique_ptr<zpx_plan> plan(new zpx_plan);
    plan->ctx = ctx;
    plan->kind = output == ZPX_JPEG_PLANES ? 0 : 1;
    // group frames by kernel variant
    std::map<std::tuple<int, int, int, int, int, int, int, int>, std::vector<int>> groups;
    for (int i = 0; i < n_frames; i++) {
        const zpx_jpeg_frame &f = frames[i];
        if (f.n_comp != 1 && f.n_comp != 3 && f.n_comp != 4) return ZPX_E_INVALID_ARGUMENT;
        if (f.coeff_bits != 8 && f.coeff_bits != 16 && f.coeff_bits != 32) return ZPX_E_INVALID_ARGUMENT;
        const int layout = f.layout;
        if (layout != ZPX_COEFFS_GRID && layout != ZPX_COEFFS_PIECES) return ZPX_E_INVALID_ARGUMENT;
        if (layout == ZPX_COEFFS_PIECES && (f.coeff_bits == 32 || !f.pieces || f.pieces_bytes < 16))
            return ZPX_E_INVALID_ARGUMENT;
        int color = 0, hc = 1, vc = 1;
        if (output == ZPX_JPEG_RGBA) {
            color = f.n_comp == 1 ? ZPX_JPEG_COLOR_GRAY : f.color;
            if (f.n_comp == 4) return ZPX_E_UNSUPPORTED;
            if (f.n_comp == 3) {
                hc = f.h[1];
                vc = f.v[1];
            }
            const int h0 = f.n_comp == 1 ? 1 : f.h[0], v0 = f.n_comp == 1 ? 1 : f.v[0];
            if (!jpeg_rgba_supported(color, h0, v0, hc, vc)) return ZPX_E_UNSUPPORTED;
            // the fused kernel addresses one strip (<= 32 rows) of output
            // through a buffer descriptor with a 31-bit range
            if (f.rgba_stride < size_t(f.width) * 4 || f.rgba_stride > (size_t(1) << 31) / 32)
                return ZPX_E_INVALID_ARGUMENT;
            groups[{f.coeff_bits, f.narrow, color, h0, v0, hc, vc, layout}].push_back(i);
        } else {
            // one group per geometry (the planar kernel's task space); the
            // stores address 8 plane rows through a 31-bit buffer range
            for (int c = 0; c < f.n_comp; c++)
                if (f.strides[c] > (size_t(1) << 31) / 8 - 1) return ZPX_E_INVALID_ARGUMENT;
            const DevJpegFrame d = dev_jpeg_frame(f);
            int hp = 0, vp = 0;
            for (int c = 0; c < f.n_comp; c++) {
                if (d.h[c] < 1 || d.h[c] > 15 || d.v[c] < 1 || d.v[c] > 15) return ZPX_E_INVALID_ARGUMENT;
                hp |= d.h[c] << (4 * c);
                vp |= d.v[c] << (4 * c);
            }
            groups[{f.coeff_bits, f.narrow, f.n_comp, hp, vp, 0, 0, layout}].push_back(i);
        }
    }
    uint64_t bytes = 0;
    for (auto &kv : groups) {
        std::unique_ptr<JpegGroup> g(new JpegGroup);
        g->bits = std::get<0>(kv.first);
        g->narrow = std::get<1>(kv.first) != 0;
        g->color = std::get<2>(kv.first);
        g->h0 = std::get<3>(kv.first);
        g->v0 = std::get<4>(kv.first);
        g->hc = std::get<5>(kv.first);
        g->vc = std::get<6>(kv.first);
        g->pieces = std::get<7>(kv.first) == ZPX_COEFFS_PIECES;
        std::vector<DevJpegFrame> df;
        for (int idx : kv.second) {
            const zpx_jpeg_frame &f = frames[idx];
            const DevJpegFrame d = dev_jpeg_frame(f);
            const size_t esz = f.coeff_bits / 8;
            df.push_back(d);
            for (int c = 0; c < f.n_comp; c++) {
                const int gw = f.mxx * d.h[c], gh = f.myy * d.v[c];
                g->max_gw = std::max(g->max_gw, gw);
                g->max_gh = std::max(g->max_gh, gh);
                // pieces: the index (4 B a block); the pieces themselves below
                if (f.coeffs[c]) bytes += uint64_t(gw) * gh * (g->pieces ? 4 : 64 * esz);
                if (output == ZPX_JPEG_PLANES) bytes += uint64_t(gw) * gh * 64;
            }
            if (g->pieces) bytes += f.pieces_bytes;
            bytes += uint64_t(f.n_comp) * 64 * 4; // quant tables
            if (output == ZPX_JPEG_RGBA) bytes += uint64_t(f.width) * f.height * 4;
            g->vec_out = g->vec_out && jpeg_rgba_vec_out(f);
            g->max_mxx = std::max(g->max_mxx, f.mxx);
            g->max_myy = std::max(g->max_myy, f.myy);
            g->geom = jpeg_plane_geom(d);
        }
        g->geom.max_mxx = g->max_mxx;
        g->geom.max_myy = g->max_myy;
        g->n = static_cast<int>(df.size());
        if (g->pieces && !jpeg_pieces_direct(output, *g)) {
            // the kernel that takes these frames reads dense grids: expand the
            // pieces into the group's own grids at every launch
            std::vector<DevPiecesExpand> jobs;
            size_t total = 0;
            const size_t esz = g->bits / 8;
            for (const DevJpegFrame &d : df)
                for (int c = 0; c < d.n_comp; c++)
                    if (d.coeffs[c]) total += (size_t(d.mxx) * d.h[c] * d.myy * d.v[c] * 64 * esz + 255) & ~size_t(255);
            HIPCHK(ctx, g->grids.alloc(std::max<size_t>(total, 256)));
            size_t off = 0;
            for (DevJpegFrame &d : df) {
                for (int c = 0; c < d.n_comp; c++) {
                    if (!d.coeffs[c]) continue;
                    const size_t blocks = size_t(d.mxx) * d.h[c] * d.myy * d.v[c];
                    DevPiecesExpand j;
                    j.index = static_cast<const uint32_t *>(d.coeffs[c]);
                    j.pieces = d.pieces;
                    j.grid = g->grids.as<uint8_t>() + off;
                    j.blocks = static_cast<uint32_t>(blocks);
                    jobs.push_back(j);
                    g->expand_max_blocks = std::max(g->expand_max_blocks, j.blocks);
                    d.coeffs[c] = j.grid;
                    off += (blocks * 64 * esz + 255) & ~size_t(255);
                }
                d.pieces = nullptr;
            }
            g->nexpand = static_cast<int>(jobs.size());
            HIPCHK(ctx, g->expand_jobs.alloc(std::max<size_t>(jobs.size(), 1) * sizeof(DevPiecesExpand)));
            HIPCHK(ctx, hipMemcpy(g->expand_jobs.ptr, jobs.data(), jobs.size() * sizeof(DevPiecesExpand),
                                  hipMemcpyHostToDevice));
            g->pieces = false;
        }
        HIPCHK(ctx, g->frames.alloc(df.size() * sizeof(DevJpegFrame)));
        HIPCHK(ctx, hipMemcpy(g->frames.ptr, df.data(), df.size() * sizeof(DevJpegFrame), hipMemcpyHostToDevice));
        plan->jpeg.push_back(std::move(g));
    }
    plan->bytes = bytes;
    *out = plan.release();
    return ZPX_OK;
}

extern "C" int zpx_jpeg_plan_create(zpx_ctx *ctx, const zpx_jpeg_frame *frames, int n_frames, int output,
                                    zpx_plan **out)
{
    return guarded([&] { return zpx_jpeg_plan_create_impl(ctx, frames, n_frames, output, out); });
}

// ---- PNG epoch windows (api_internal.h, PngControl)
namespace {
std::mutex g_win_mu;
const void *g_win_owner[kPngEpochWindows] = {};
uint32_t g_win_next = 0; // next window to try (0: not yet seeded)
} // namespace

uint32_t zpx::png_epoch_window_acquire(const void *owner)
{
    constexpr uint32_t n = kPngEpochWindows - 1; // windows 1 .. n
    std::lock_guard<std::mutex> lk(g_win_mu);
    if (g_win_next == 0) // (a per-process start: two processes' blocks rarely share windows either)
        g_win_next = 1 + static_cast<uint32_t>((uint64_t(getpid()) * 2654435761u) % n);
    for (uint32_t k = 0; k < n; k++) {
        const uint32_t w = 1 + (g_win_next - 1 + k) % n;
        if (g_win_owner[w]) continue;
        g_win_owner[w] = owner;
        g_win_next = w % n + 1; // round robin: a returned window is the last to be handed out again
        return w;
    }
    return 0;
}

bool zpx::png_epoch_window_release(uint32_t window, const void *owner)
{
    std::lock_guard<std::mutex> lk(g_win_mu);
    if (window == 0 || window >= kPngEpochWindows || g_win_owner[window] != owner) return false;
    g_win_owner[window] = nullptr;
    return true;
}

bool zpx::png_epoch_window_owned(uint32_t window, const void *owner)
{
    std::lock_guard<std::mutex> lk(g_win_mu);
    return window != 0 && window < kPngEpochWindows && g_win_owner[window] == owner;
}

zpx::PngControl::~PngControl()
{
    if (window_) (void)png_epoch_window_release(window_, this);
}

int zpx::PngControl::init(zpx_ctx *ctx)
{
    if (!window_) window_ = png_epoch_window_acquire(this);
    if (!window_) {
        ctx->last_error = "png: every epoch window belongs to a live plan or batch slot (4095)";
        return ZPX_E_OUT_OF_MEMORY;
    }
    const int c = opt(Opt::PngEpochCycle);
    base_ = window_ * kPngEpochWindow;
    cycle_ = c >= 4 && uint32_t(c) < kPngEpochWindow ? uint32_t(c) : kPngEpochWindow;
    shadow_ = base_;
    HIPCHK(ctx, ctl_.alloc(kPngCtlWords * sizeof(uint32_t)));
    const uint32_t w[kPngCtlWords] = {base_, 0, 0, 0, base_, cycle_, 0, 0};
    HIPCHK(ctx, hipMemcpy(ctl_.ptr, w, sizeof(w), hipMemcpyHostToDevice));
    return ZPX_OK;
}

int zpx::PngControl::prepare(zpx_ctx *ctx, int launches, void *boundary, size_t bytes, hipStream_t st)
{
    if (!png_epoch_window_owned(window_, this)) {
        ctx->last_error = "png: control block launched without its epoch window";
        return ZPX_E_PANIC;
    }
    if (png_epoch_wraps(shadow_, base_, cycle_, launches)) {
        HIPCHK(ctx, hipMemsetAsync(boundary, 0, bytes, st));
        HIPCHK(ctx, hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(ctl_.ptr), static_cast<int>(base_), 1, st));
        shadow_ = base_;
        wraps_++;
    }
    for (int i = 0; i < launches; i++) shadow_ = png_epoch_next(shadow_, base_, cycle_);
    return ZPX_OK;
}

static int png_build_group(zpx_ctx *ctx, PngGroup &g, const std::vector<DevPngPass> &passes_in,
                           const std::vector<uint32_t> &pass_rowbytes)
{
    std::vector<DevPngPass> passes = passes_in;
    const PngBandPlan bp = png_plan_bands(g.depth, g.pair, passes, pass_rowbytes);
    if (!png_band_fits(bp.max_rb, bp.band_rows)) {
        ctx->last_error = "png: a band of this image exceeds the kernel's 2 GiB band range";
        return ZPX_E_UNSUPPORTED;
    }
    std::vector<DevPngBand> sched = bp.sched; // longest first (api_internal.h), then the second launch's
    sched.insert(sched.end(), bp.sched2.begin(), bp.sched2.end());
    const uint32_t base = bp.nbands;
    g.nsched = static_cast<uint32_t>(bp.sched.size());
    g.nsched2 = static_cast<uint32_t>(bp.sched2.size());
    g.nbands = base;
    g.band_bytes = bp.granules; // granules per band
    HIPCHK(ctx, g.passes.alloc(passes.size() * sizeof(DevPngPass)));
    HIPCHK(ctx, hipMemcpy(g.passes.ptr, passes.data(), passes.size() * sizeof(DevPngPass), hipMemcpyHostToDevice));
    HIPCHK(ctx, g.sched.alloc(std::max<size_t>(1, sched.size()) * sizeof(DevPngBand)));
    if (!sched.empty())
        HIPCHK(ctx, hipMemcpy(g.sched.ptr, sched.data(), sched.size() * sizeof(DevPngBand), hipMemcpyHostToDevice));
    // the control block and its epoch window (PngControl); the boundary
    // granules start with tag 0, which no epoch is -- cleared and complete
    // before the first launch, whichever stream that is on
    if (int e = g.ctl.init(ctx)) return e;
    const size_t bbytes = std::max<size_t>(1, size_t(base)) * g.band_bytes * sizeof(uint64_t);
    HIPCHK(ctx, g.boundary.alloc(bbytes));
    HIPCHK(ctx, hipMemsetAsync(g.boundary.ptr, 0, bbytes, ctx->stream));
    HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
    return 0;
}

void zpx::png_frame_passes(const zpx_png_frame &f, std::vector<DevPngPass> &passes, std::vector<uint32_t> &rowbytes,
                           uint64_t &bytes)
{
    static const uint32_t kA7[7][4] = {{0, 0, 8, 8}, {4, 0, 8, 8}, {0, 4, 4, 8}, {2, 0, 4, 4},
                                       {0, 2, 2, 4}, {1, 0, 2, 2}, {0, 1, 1, 2}};
    int bits = 0;
    switch (f.depth) {
    case ZPX_PNG_G1: case ZPX_PNG_P1: bits = 1; break;
    case ZPX_PNG_G2: case ZPX_PNG_P2: bits = 2; break;
    case ZPX_PNG_G4: case ZPX_PNG_P4: bits = 4; break;
    case ZPX_PNG_G8: case ZPX_PNG_P8: bits = 8; break;
    case ZPX_PNG_GA8: case ZPX_PNG_G16: bits = 16; break;
    case ZPX_PNG_TC8: bits = 24; break;
    case ZPX_PNG_TCA8: case ZPX_PNG_GA16: bits = 32; break;
    case ZPX_PNG_TC16: bits = 48; break;
    default: bits = 64; break;
    }
    size_t off = 0;
    uint32_t slab_band = 0; // (slab layout: bands of 128 rows, png_slab.cpp)
    const int np = f.interlace ? 7 : 1;
    for (int p = 0; p < np; p++) {
        DevPngPass d{};
        uint32_t w = f.width, h = f.height, xo = 0, yo = 0, xf = 1, yf = 1;
        if (f.interlace) {
            xo = kA7[p][0];
            yo = kA7[p][1];
            xf = kA7[p][2];
            yf = kA7[p][3];
            w = ((f.width > xo ? f.width - xo : 0) + xf - 1) / xf;
            h = ((f.height > yo ? f.height - yo : 0) + yf - 1) / yf;
            if (w == 0 || h == 0) continue;
        }
        const uint32_t rb = static_cast<uint32_t>((uint64_t(bits) * w + 7) / 8);
        d.filtered = f.layout == ZPX_PNG_LAYOUT_SLAB ? f.filtered : f.filtered + off;
        d.slab = f.layout == ZPX_PNG_LAYOUT_SLAB ? 1 : 0;
        d.slab_band0 = slab_band;
        slab_band += (h + 127) / 128;
        d.out = f.out;
        d.max_index = f.max_index;
        d.out_stride = f.out_stride;
        d.width = w;
        d.rows = h;
        d.row_bytes = rb;
        d.xo = xo;
        d.yo = yo;
        d.xf = xf;
        d.yf = yf;
        memcpy(d.trns, f.transparent, 6);
        d.use_trns = f.use_transparent ? 1 : 0;
        passes.push_back(d);
        rowbytes.push_back(rb);
        off += size_t(h) * (size_t(rb) + 1);
    }
    bytes += off;
}

static int png_out_bpp(int depth, bool trns)
{
    switch (depth) {
    case ZPX_PNG_G1: case ZPX_PNG_G2: case ZPX_PNG_G4: case ZPX_PNG_G8: return trns ? 4 : 1;
    case ZPX_PNG_GA8: case ZPX_PNG_TC8: case ZPX_PNG_TCA8: return 4;
    case ZPX_PNG_G16: return trns ? 8 : 2;
    case ZPX_PNG_GA16: case ZPX_PNG_TC16: case ZPX_PNG_TCA16: return 8;
    default: return 1;
    }
}

static int zpx_png_plan_create_impl(zpx_ctx *ctx, const zpx_png_frame *frames, int n_frames, zpx_plan **out)
{
    if (!ctx || !frames || n_frames <= 0 || !out) return ZPX_E_INVALID_ARGUMENT;
    *out = nullptr;
    CtxScope s(ctx);
    std::unique_ptr<zpx_plan> plan(new zpx_plan);
    plan->ctx = ctx;
    plan->kind = 2;
    // one launch per (depth, kernel): the paired-row kernel takes what it supports
    std::map<std::tuple<int, bool, bool, bool>, std::vector<int>> by_depth; // (depth, pair kernel, colour key, stream)
    for (int i = 0; i < n_frames; i++) {
        if (frames[i].depth < ZPX_PNG_G1 || frames[i].depth > ZPX_PNG_TCA16) return ZPX_E_INVALID_ARGUMENT;
        const bool trns = frames[i].use_transparent != 0;
        // the paired-row kernel takes the stream layout (its stream
        // instance) and the slab layout; the rest take the one-row-per-lane
        // kernel
        const bool pair_ok = png_use_pair(frames[i].depth, frames[i].interlace, trns, frames[i].width,
                                          frames[i].out_stride);
        if (frames[i].layout > ZPX_PNG_LAYOUT_SLAB) return ZPX_E_INVALID_ARGUMENT;
        if (frames[i].layout == ZPX_PNG_LAYOUT_SLAB && !pair_ok) {
            ctx->last_error = "png: a slab-layout frame needs the paired-row kernel (zpx_png_stream_slab)";
            return ZPX_E_INVALID_ARGUMENT;
        }
        const bool pair = pair_ok;
        // (png_device_slab: stream frames get a device slab, read as slabs)
        const bool stream = pair && frames[i].layout == ZPX_PNG_LAYOUT_STREAM && !opt(Opt::PngDeviceSlab);
        by_depth[{frames[i].depth, pair, pair && trns, stream}].push_back(i);
    }
    uint64_t bytes = 0;
    for (auto &kv : by_depth) {
        std::unique_ptr<PngGroup> g(new PngGroup);
        g->depth = std::get<0>(kv.first);
        g->pair = std::get<1>(kv.first);
        g->trns = std::get<2>(kv.first);
        g->stream = std::get<3>(kv.first);
        std::vector<DevPngPass> passes;
        std::vector<uint32_t> rowbytes;
        Adam7Stage a7;
        // stream-layout frames on the paired-row kernel: one device slab each
        std::vector<std::vector<uint64_t>> slab_off(kv.second.size());
        std::vector<size_t> slab_at(kv.second.size(), 0);
        size_t slab_total = 0;
        for (size_t k = 0; k < kv.second.size() && g->pair && !g->stream; k++) {
            const zpx_png_frame &f = frames[kv.second[k]];
            if (f.layout != ZPX_PNG_LAYOUT_STREAM) continue;
            slab_at[k] = slab_total;
            slab_total = (slab_total + png_dev_slab_layout(f, slab_off[k]) + 255) & ~size_t(255);
        }
        std::vector<DevSlabBand> sjobs;
        if (slab_total) HIPCHK(ctx, g->dslab.alloc(slab_total));
        for (size_t k = 0; k < kv.second.size(); k++) {
            const int idx = kv.second[k];
            zpx_png_frame f = frames[idx];
            if (g->pair && !g->stream && f.layout == ZPX_PNG_LAYOUT_STREAM) {
                uint8_t *d_slab = g->dslab.as<uint8_t>() + slab_at[k];
                HIPCHK(ctx, hipMemcpy(d_slab, slab_off[k].data(), slab_off[k].size() * sizeof(uint64_t),
                                      hipMemcpyHostToDevice));
                std::vector<DevPngPass> sp;
                std::vector<uint32_t> srb;
                uint64_t sbytes = 0;
                png_frame_passes(f, sp, srb, sbytes); // (the stream's bytes)
                png_dev_slab_jobs(f, slab_off[k], f.filtered, sbytes + ZPX_PNG_INPUT_PAD, d_slab, sjobs,
                                  g->slab_max_groups);
                f.filtered = d_slab;
                f.layout = ZPX_PNG_LAYOUT_SLAB;
            }
            const size_t first = passes.size();
            png_frame_passes(f, passes, rowbytes, bytes);
            const int obpx = png_out_bpp(frames[idx].depth, frames[idx].use_transparent != 0);
            bytes += uint64_t(frames[idx].width) * frames[idx].height * obpx;
            if (g->pair && frames[idx].interlace) png_adam7_stage(frames[idx], obpx, passes, first, a7);
        }
        if (!sjobs.empty()) {
            g->nslab_jobs = static_cast<uint32_t>(sjobs.size());
            HIPCHK(ctx, g->slab_jobs.alloc(sjobs.size() * sizeof(DevSlabBand)));
            HIPCHK(ctx, hipMemcpy(g->slab_jobs.ptr, sjobs.data(), sjobs.size() * sizeof(DevSlabBand),
                                  hipMemcpyHostToDevice));
        }
        if (!a7.jobs.empty()) {
            HIPCHK(ctx, g->staging.alloc(a7.bytes));
            HIPCHK(ctx, g->merge_jobs.alloc(a7.jobs.size() * sizeof(DevAdam7Merge)));
            png_adam7_rebase(passes, a7, g->staging.as<uint8_t>(), g->merge_jobs.as<DevAdam7Merge>());
            HIPCHK(ctx, hipMemcpy(g->merge_jobs.ptr, a7.jobs.data(), a7.jobs.size() * sizeof(DevAdam7Merge),
                                  hipMemcpyHostToDevice));
        }
        if (int e = png_build_group(ctx, *g, passes, rowbytes)) return e;
        plan->png.push_back(std::move(g));
    }
    plan->bytes = bytes;
    *out = plan.release();
    return ZPX_OK;
}

extern "C" int zpx_png_plan_create(zpx_ctx *ctx, const zpx_png_frame *frames, int n_frames, zpx_plan **out)
{
    return guarded([&] { return zpx_png_plan_create_impl(ctx, frames, n_frames, out); });
}

// Image.rgbaPixels (image.zig:103-130) over a batch of device-resident
// images: one launch per image kind.
static int zpx_rgba_plan_create_impl(zpx_ctx *ctx, const zpx_image *imgs, uint8_t *const *outs, int n,
                                     zpx_plan **out)
{
    if (!ctx || !imgs || !outs || n <= 0 || !out) return ZPX_E_INVALID_ARGUMENT;
    *out = nullptr;
    CtxScope s(ctx);
    std::unique_ptr<zpx_plan> plan(new zpx_plan);
    plan->ctx = ctx;
    plan->kind = 3;
    std::map<int, std::vector<DevRgbaJob>> by_kind;
    uint64_t bytes = 0;
    for (int i = 0; i < n; i++) {
        const zpx_image &im = imgs[i];
        if (im.min_x != 0 || im.min_y != 0) return ZPX_E_UNSUPPORTED;
        if (im.kind < ZPX_GRAY || im.kind > ZPX_PALETTED || !outs[i] || !im.pixels || !palette_ok(im))
            return ZPX_E_INVALID_ARGUMENT;
        const uint64_t w = uint64_t(im.max_x), h = uint64_t(im.max_y);
        if (w > 65535u * 1024u || h > 65535) return ZPX_E_UNSUPPORTED;
        by_kind[im.kind].push_back(rgba_job(dev_image_of(&im, im.pixels, im.palette), outs[i]));
        // algorithmic bytes: the pixels the kind reads, then RGBA8
        static const int kBpp[9] = {1, 2, 0, 4, 8, 4, 8, 4, 1}; // zpx_kind order
        uint64_t in = w * h * uint64_t(kBpp[im.kind]);
        if (im.kind == ZPX_YCBCR) {
            const uint64_t cw = (im.subsample == ZPX_RATIO444 || im.subsample == ZPX_RATIO440) ? w
                                : (im.subsample == ZPX_RATIO411 || im.subsample == ZPX_RATIO410) ? (w + 3) / 4 : (w + 1) / 2;
            const uint64_t ch = (im.subsample == ZPX_RATIO420 || im.subsample == ZPX_RATIO440 ||
                                 im.subsample == ZPX_RATIO410) ? (h + 1) / 2 : h;
            in = w * h + 2 * cw * ch;
        }
        bytes += in + w * h * 4;
    }
    for (auto &kv : by_kind) {
        if (kv.second.size() > 65535) return ZPX_E_UNSUPPORTED;
        std::unique_ptr<RgbaGroup> g(new RgbaGroup);
        g->kind = kv.first;
        g->n = static_cast<int>(kv.second.size());
        for (const DevRgbaJob &j : kv.second) {
            g->max_w = std::max(g->max_w, j.m.width);
            g->max_h = std::max(g->max_h, j.m.height);
        }
        HIPCHK(ctx, g->jobs.alloc(kv.second.size() * sizeof(DevRgbaJob)));
        HIPCHK(ctx, hipMemcpy(g->jobs.ptr, kv.second.data(), kv.second.size() * sizeof(DevRgbaJob),
                              hipMemcpyHostToDevice));
        plan->rgba.push_back(std::move(g));
    }
    plan->bytes = bytes;
    *out = plan.release();
    return ZPX_OK;
}

extern "C" int zpx_rgba_plan_create(zpx_ctx *ctx, const zpx_image *imgs, uint8_t *const *outs, int n,
                                    zpx_plan **out)
{
    return guarded([&] { return zpx_rgba_plan_create_impl(ctx, imgs, outs, n, out); });
}

extern "C" int zpx_plan_launch(zpx_plan *plan, void *stream)
{
    if (!plan) return ZPX_E_INVALID_ARGUMENT;
    zpx_ctx *ctx = plan->ctx;
    CtxScope s(ctx);
    hipStream_t st = stream ? static_cast<hipStream_t>(stream) : ctx->stream;
    for (auto &g : plan->rgba)
        if (launch_rgba_batch(g->kind, g->jobs.as<DevRgbaJob>(), g->n, g->max_w, g->max_h, st))
            return hip_fail(ctx, hipGetLastError(), "rgba batch kernel launch");
    for (auto &g : plan->jpeg) {
        int rc;
        if (g->nexpand && launch_jpeg_pieces_expand(g->expand_jobs.as<DevPiecesExpand>(), g->nexpand,
                                                    g->expand_max_blocks, g->bits, st))
            return hip_fail(ctx, hipGetLastError(), "jpeg pieces expand launch");
        if (plan->kind == 0)
            rc = launch_jpeg_planar(g->frames.as<DevJpegFrame>(), g->n, g->geom, g->bits, g->narrow, g->pieces, st);
        else
            rc = launch_jpeg_rgba(g->frames.as<DevJpegFrame>(), g->n, g->color, g->h0, g->v0, g->hc, g->vc,
                                  g->max_mxx, g->max_myy, g->bits, g->narrow, g->vec_out, g->pieces, st);
        if (rc == -2) return ZPX_E_UNSUPPORTED;
        if (rc) return hip_fail(ctx, hipGetLastError(), "jpeg kernel launch");
    }
    for (auto &g : plan->png) {
        // the control kernels of this group's launches: re-base the epoch
        // (clearing the boundary) first if they would wrap its cycle
        if (int e = g->ctl.prepare(ctx, g->nsched2 ? 2 : 1, g->boundary.ptr, g->boundary.bytes, st)) return e;
        // stream-layout frames: their band slabs first
        if (g->nslab_jobs && launch_png_slab(png_slab_chunk_bytes(g->depth), g->slab_jobs.as<DevSlabBand>(),
                                             g->nslab_jobs, g->slab_max_groups, st))
            return hip_fail(ctx, hipGetLastError(), "png slab kernel launch");
        const int rc = g->pair ? launch_png_pair(g->depth, g->trns, g->stream, g->passes.as<DevPngPass>(),
                                                 g->sched.as<DevPngBand>(), g->nsched, g->ctl.words(),
                                                 g->boundary.as<uint64_t>(), g->band_bytes, st)
                               : launch_png_unfilter(g->depth, g->passes.as<DevPngPass>(), g->sched.as<DevPngBand>(),
                                                     g->nsched, g->ctl.words(), g->boundary.as<uint64_t>(),
                                                     g->band_bytes, st);
        if (rc) return hip_fail(ctx, hipGetLastError(), "png kernel launch");
        // Adam7: pass 6 merges the staged passes once the first launch is done
        if (g->nsched2 && launch_png_pair_merge(g->depth, g->trns, g->stream, g->passes.as<DevPngPass>(),
                                                g->sched.as<DevPngBand>() + g->nsched, g->nsched2,
                                                g->ctl.words(), g->boundary.as<uint64_t>(), g->band_bytes,
                                                st))
            return hip_fail(ctx, hipGetLastError(), "png adam7 merge pass launch");
    }
    return ZPX_OK;
}

// zpx_plan_status: control words {epoch, ticket, status, sticky}. The
// kernel sets `status` for its own launch; png_ctl_kernel folds it into
// `sticky` at the next launch's start, so a timeout in any launch since the
// last call is reported, not only the last launch's.
static int zpx_plan_status_impl(zpx_plan *plan, void *stream)
{
    if (!plan) return ZPX_E_INVALID_ARGUMENT;
    zpx_ctx *ctx = plan->ctx;
    CtxScope s(ctx);
    hipStream_t st = stream ? static_cast<hipStream_t>(stream) : ctx->stream;
    if (plan->png.empty()) {
        HIPCHK(ctx, hipStreamSynchronize(st));
        return ZPX_OK;
    }
    const size_t n = plan->png.size();
    if (plan->status_host.bytes < n * 8 && !plan->status_host.alloc(n * 8, true)) return ZPX_E_OUT_OF_MEMORY;
    uint32_t *h = static_cast<uint32_t *>(plan->status_host.ptr);
    for (size_t i = 0; i < n; i++) {
        uint32_t *ctl = plan->png[i]->ctl.words();
        HIPCHK(ctx, hipMemcpyAsync(h + 2 * i, ctl + 2, 8, hipMemcpyDeviceToHost, st));
        HIPCHK(ctx, hipMemsetAsync(ctl + 2, 0, 8, st));
    }
    HIPCHK(ctx, hipStreamSynchronize(st));
    for (size_t i = 0; i < n; i++)
        if (h[2 * i] | h[2 * i + 1]) {
            ctx->last_error = "png wavefront hand-off timed out";
            return ZPX_E_HIP;
        }
    return ZPX_OK;
}

extern "C" int zpx_plan_status(zpx_plan *plan, void *stream)
{
    return guarded([&] { return zpx_plan_status_impl(plan, stream); });
}

extern "C" uint64_t zpx_plan_bytes(const zpx_plan *plan) { return plan ? plan->bytes : 0; }
extern "C" int zpx_plan_kernel_count(const zpx_plan *plan)
{
    if (!plan) return 0;
    int n = static_cast<int>(plan->rgba.size());
    for (auto &g : plan->jpeg) n += 1 + (g->nexpand ? 1 : 0);
    for (auto &g : plan->png) n += 1 + (g->nslab_jobs ? 1 : 0) + (g->nsched2 ? 1 : 0);
    return n;
}
extern "C" void zpx_plan_destroy(zpx_plan *plan)
{
    if (!plan) return;
    (void)hipSetDevice(plan->ctx->device);
    delete plan;
}

// ------------------------------------------------------------------ host stages exposed
struct zpx_jpeg_coeffs {
    JpegCoeffs c;
};
struct zpx_png_stream {
    PngStream s;
    std::mutex slab_mu; // zpx_png_stream_slab builds s.slab once, whichever thread asks first
};

static int zpx_jpeg_entropy_decode_impl(const uint8_t *buf, size_t len, zpx_jpeg_coeffs **out, bool pieces)
{
    if (!out || (!buf && len)) return ZPX_E_INVALID_ARGUMENT;
    *out = nullptr;
    std::unique_ptr<zpx_jpeg_coeffs> c(new zpx_jpeg_coeffs);
    if (int e = jpeg_entropy_decode(buf, len, c->c, jpeg_huff_threads(), pieces)) return e;
    *out = c.release();
    return ZPX_OK;
}

extern "C" int zpx_jpeg_entropy_decode(const uint8_t *buf, size_t len, zpx_jpeg_coeffs **out)
{
    return guarded([&] { return zpx_jpeg_entropy_decode_impl(buf, len, out, false); });
}

extern "C" int zpx_jpeg_entropy_decode_pieces(const uint8_t *buf, size_t len, zpx_jpeg_coeffs **out)
{
    return guarded([&] { return zpx_jpeg_entropy_decode_impl(buf, len, out, true); });
}

void zpx::jpeg_fill_frame(const JpegCoeffs &c, zpx_jpeg_frame *f, size_t *coeff_bytes)
{
    memset(f, 0, sizeof(*f));
    f->width = c.width;
    f->height = c.height;
    f->n_comp = c.n_comp;
    f->mxx = c.mxx;
    f->myy = c.myy;
    int bits = 8;
    int64_t m = 0;
    for (int i = 0; i < c.n_comp; i++) {
        f->h[i] = c.comp[i].h;
        f->v[i] = c.comp[i].v;
        f->rule[i] = c.rule[i];
        memcpy(f->qt[i], c.qt_natural[i], sizeof(f->qt[i]));
        if (c.has_grid[i]) {
            bits = std::max(bits, c.grid[i].bits());
            m = std::max<int64_t>(m, int64_t(c.grid[i].max_abs()) * c.max_q[i]);
        }
    }
    if (c.pieces.valid) {
        bits = c.pieces.bits;
        for (int i = 0; i < c.n_comp; i++) m = std::max<int64_t>(m, int64_t(c.pieces.max_abs[i]) * c.max_q[i]);
    }
    f->coeff_bits = bits;
    f->narrow = m <= 16384 ? 1 : 0;
    switch (jpeg_output_kind(c)) {
    case JpegOut::Gray: f->color = ZPX_JPEG_COLOR_GRAY; break;
    case JpegOut::RGB: f->color = ZPX_JPEG_COLOR_RGB; break;
    default: f->color = ZPX_JPEG_COLOR_YCBCR; break;
    }
    if (c.pieces.valid) {
        f->layout = ZPX_COEFFS_PIECES;
        f->pieces = c.pieces.data.ptr;
        f->pieces_bytes = c.pieces.data_bytes();
        for (int i = 0; i < 4; i++) {
            const bool g = i < c.n_comp;
            f->coeffs[i] = g ? c.pieces.index_of(i) : nullptr;
            if (coeff_bytes) coeff_bytes[i] = g ? c.pieces.blocks[i] * sizeof(uint32_t) : 0;
        }
        return;
    }
    for (int i = 0; i < 4; i++) {
        const bool g = i < c.n_comp && c.has_grid[i];
        f->coeffs[i] = g ? c.grid[i].data() : nullptr;
        if (coeff_bytes) coeff_bytes[i] = g ? c.grid[i].blocks() * 64 * (bits / 8) : 0;
    }
}

extern "C" int zpx_jpeg_coeffs_frame(const zpx_jpeg_coeffs *cc, zpx_jpeg_frame *f, size_t *coeff_bytes)
{
    if (!cc || !f) return ZPX_E_INVALID_ARGUMENT;
    jpeg_fill_frame(cc->c, f, coeff_bytes);
    return ZPX_OK;
}

extern "C" void zpx_jpeg_coeffs_free(zpx_jpeg_coeffs *c) { delete c; }

extern "C" int zpx_jpeg_coeffs_widen(zpx_jpeg_coeffs *cc, int bits)
{
    if (!cc || (bits != 8 && bits != 16 && bits != 32)) return ZPX_E_INVALID_ARGUMENT;
    if (cc->c.pieces.valid) { // pieces are int8 or int16
        if (bits == 32) return ZPX_E_UNSUPPORTED;
        return bits == 16 && !cc->c.pieces.widen() ? ZPX_E_OUT_OF_MEMORY : ZPX_OK;
    }
    for (int i = 0; i < 4; i++)
        if (cc->c.has_grid[i] && !cc->c.grid[i].widen_to(bits)) return ZPX_E_OUT_OF_MEMORY;
    return ZPX_OK;
}

static int zpx_png_inflate_impl(const uint8_t *buf, size_t len, zpx_png_stream **out)
{
    if (!out || (!buf && len)) return ZPX_E_INVALID_ARGUMENT;
    *out = nullptr;
    std::unique_ptr<zpx_png_stream> s(new zpx_png_stream);
    if (int e = png_parse(buf, len, s->s, png_inflate_threads())) return e;
    *out = s.release();
    return ZPX_OK;
}

extern "C" int zpx_png_inflate(const uint8_t *buf, size_t len, zpx_png_stream **out)
{
    return guarded([&] { return zpx_png_inflate_impl(buf, len, out); });
}

extern "C" int zpx_debug_png_inflate_pair(const uint8_t *buf0, size_t len0, const uint8_t *buf1, size_t len1,
                                          zpx_png_stream **out0, zpx_png_stream **out1, int *status)
{
    return guarded([&]() -> int {
        if (!out0 || !out1 || !status || (!buf0 && len0) || (!buf1 && len1)) return ZPX_E_INVALID_ARGUMENT;
        *out0 = *out1 = nullptr;
        std::unique_ptr<zpx_png_stream> s0(new zpx_png_stream), s1(new zpx_png_stream);
        const uint8_t *buf[2] = {buf0, buf1};
        const size_t len[2] = {len0, len1};
        PngStream *ps[2] = {&s0->s, &s1->s};
        if (int e = png_parse_pair(buf, len, ps, status)) return e;
        if (status[0] == ZPX_OK) *out0 = s0.release();
        if (status[1] == ZPX_OK) *out1 = s1.release();
        return ZPX_OK;
    });
}

extern "C" int zpx_png_stream_frame(const zpx_png_stream *ss, zpx_png_frame *f, size_t *filtered_len)
{
    if (!ss || !f) return ZPX_E_INVALID_ARGUMENT;
    const PngStream &s = ss->s;
    memset(f, 0, sizeof(*f));
    f->width = s.width;
    f->height = s.height;
    f->depth = s.depth;
    f->interlace = s.interlace;
    f->use_transparent = s.use_transparent ? 1 : 0;
    memcpy(f->transparent, s.transparent, 6);
    f->filtered = static_cast<const uint8_t *>(s.data.ptr);
    f->out_stride = size_t(s.width) * s.out_bpp;
    if (filtered_len) *filtered_len = s.data_len;
    return ZPX_OK;
}

extern "C" const uint8_t *zpx_png_stream_data(const zpx_png_stream *s)
{
    return s ? static_cast<const uint8_t *>(s->s.data.ptr) : nullptr;
}
extern "C" int zpx_png_stream_slab(zpx_png_stream *s, const uint8_t **data, size_t *len)
{
    if (!s || !data || !len) return ZPX_E_INVALID_ARGUMENT;
    return guarded([&] {
        std::lock_guard<std::mutex> lk(s->slab_mu);
        if (!s->s.slab_len)
            if (int e = png_stream_build_slab(s->s, png_inflate_threads())) return e;
        *data = static_cast<const uint8_t *>(s->s.slab.ptr);
        *len = s->s.slab_len;
        return static_cast<int>(ZPX_OK);
    });
}
extern "C" void zpx_png_stream_free(zpx_png_stream *s) { delete s; }

// Test hook: the band slab of stream `s` as the plans build it on the device
// (png_slab_kernels.hip), copied back to `out` (cap bytes; *len = its size).
// Bytes the paired-row kernel never reads (groups past a band's last, region
// tails) are left as 0xa5.
static int zpx_debug_png_device_slab_impl(zpx_ctx *ctx, const zpx_png_stream *ss, uint8_t *out, size_t cap,
                                          size_t *len)
{
    if (!ctx || !ss || !len) return ZPX_E_INVALID_ARGUMENT;
    CtxScope scope(ctx);
    const PngStream &ps = ss->s;
    if (!png_use_pair(ps.depth, ps.interlace, ps.use_transparent, ps.width, size_t(ps.width) * ps.out_bpp))
        return ZPX_E_UNSUPPORTED;
    zpx_png_frame f;
    memset(&f, 0, sizeof(f));
    f.width = ps.width;
    f.height = ps.height;
    f.depth = ps.depth;
    f.interlace = ps.interlace;
    f.use_transparent = ps.use_transparent;
    f.out_stride = size_t(ps.width) * ps.out_bpp;
    std::vector<uint64_t> off;
    const size_t n = png_dev_slab_layout(f, off);
    *len = n;
    if (!out || cap < n) return out ? ZPX_E_INVALID_ARGUMENT : ZPX_OK;
    DevBuf din, dslab, djobs;
    const size_t in_len = ps.data_len + ZPX_PNG_INPUT_PAD;
    HIPCHK(ctx, din.alloc(in_len));
    HIPCHK(ctx, hipMemcpy(din.ptr, ps.data.ptr, in_len, hipMemcpyHostToDevice));
    HIPCHK(ctx, dslab.alloc(n));
    HIPCHK(ctx, hipMemset(dslab.ptr, 0xa5, n));
    HIPCHK(ctx, hipMemcpy(dslab.ptr, off.data(), off.size() * sizeof(uint64_t), hipMemcpyHostToDevice));
    std::vector<DevSlabBand> jobs;
    uint32_t groups = 0;
    png_dev_slab_jobs(f, off, din.as<uint8_t>(), in_len, dslab.as<uint8_t>(), jobs, groups);
    HIPCHK(ctx, djobs.alloc(jobs.size() * sizeof(DevSlabBand)));
    HIPCHK(ctx, hipMemcpy(djobs.ptr, jobs.data(), jobs.size() * sizeof(DevSlabBand), hipMemcpyHostToDevice));
    if (launch_png_slab(png_slab_chunk_bytes(ps.depth), djobs.as<DevSlabBand>(), static_cast<uint32_t>(jobs.size()),
                        groups, ctx->stream))
        return hip_fail(ctx, hipGetLastError(), "png slab kernel");
    HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
    HIPCHK(ctx, hipMemcpy(out, dslab.ptr, n, hipMemcpyDeviceToHost));
    return ZPX_OK;
}

extern "C" int zpx_debug_png_device_slab(zpx_ctx *ctx, const zpx_png_stream *s, uint8_t *out, size_t cap, size_t *len)
{
    return guarded([&] { return zpx_debug_png_device_slab_impl(ctx, s, out, cap, len); });
}

// ------------------------------------------------------------------ jpeg.decode
namespace {

struct JpegDeviceFrame {
    DevBuf coeffs[4];
    zpx_jpeg_frame f{};
};

int upload_jpeg(zpx_ctx *ctx, const JpegCoeffs &c, JpegDeviceFrame &d)
{
    size_t cbytes[4];
    jpeg_fill_frame(c, &d.f, cbytes);
    for (int i = 0; i < c.n_comp; i++) {
        if (!d.f.coeffs[i]) continue;
        HIPCHK(ctx, d.coeffs[i].alloc(cbytes[i]));
        HIPCHK(ctx, hipMemcpyAsync(d.coeffs[i].ptr, d.f.coeffs[i], cbytes[i], hipMemcpyHostToDevice, ctx->stream));
        d.f.coeffs[i] = d.coeffs[i].ptr;
    }
    return ZPX_OK;
}

int run_plan_once(zpx_ctx *ctx, const zpx_jpeg_frame &f, int output)
{
    zpx_plan *plan = nullptr;
    if (int e = zpx_jpeg_plan_create(ctx, &f, 1, output, &plan)) return e;
    int e = zpx_plan_launch(plan, ctx->stream);
    if (!e) {
        hipError_t he = hipStreamSynchronize(ctx->stream);
        if (he != hipSuccess) e = hip_fail(ctx, he, "jpeg kernel");
    }
    zpx_plan_destroy(plan);
    return e;
}

} // namespace

static int zpx_jpeg_decode_impl(zpx_ctx *ctx, const zpx_allocator *al, const uint8_t *buf, size_t len, zpx_image *out)
{
    if (!ctx || !out || (!buf && len)) return ZPX_E_INVALID_ARGUMENT;
    memset(out, 0, sizeof(*out));
    CtxScope s(ctx);
    JpegCoeffs c;
    if (int e = jpeg_entropy_decode(buf, len, c, jpeg_huff_threads())) return e;
    const JpegOut kind = jpeg_output_kind(c);
    if (c.n_comp == 4 && !c.adobe_valid) return ZPX_E_UNSUPPORTED_COLOR_MODEL; // applyBlack :793-795
    if (kind == JpegOut::YCCK) {
        ctx->last_error = "YCbCrK (Adobe transform 2) goes through image/util.zig drawYCbCr: out of scope";
        return ZPX_E_UNSUPPORTED;
    }
    JpegLayout L;
    if (int e = jpeg_layout(c, L)) return e;
    JpegDeviceFrame d;
    if (int e = upload_jpeg(ctx, c, d)) return e;
    DevBuf planes, kplane;
    HIPCHK(ctx, planes.alloc(L.total));
    HIPCHK(ctx, hipMemsetAsync(planes.ptr, 0, L.total, ctx->stream)); // makeImg zeroes (image.zig:505-507)
    uint8_t *pb = planes.as<uint8_t>();
    d.f.planes[0] = pb;
    d.f.strides[0] = L.y_stride;
    if (c.n_comp >= 3) {
        d.f.planes[1] = pb + L.cb_off;
        d.f.planes[2] = pb + L.cr_off;
        d.f.strides[1] = d.f.strides[2] = L.c_stride;
    }
    if (c.n_comp == 4) {
        HIPCHK(ctx, kplane.alloc(L.k_total));
        HIPCHK(ctx, hipMemsetAsync(kplane.ptr, 0, L.k_total, ctx->stream));
        d.f.planes[3] = kplane.as<uint8_t>();
        d.f.strides[3] = L.k_stride;
    }
    if (int e = run_plan_once(ctx, d.f, ZPX_JPEG_PLANES)) return e;

    const int W = static_cast<int>(c.width), H = static_cast<int>(c.height);
    zpx_image img{};
    img.max_x = W;
    img.max_y = H;
    if (kind == JpegOut::Gray || kind == JpegOut::YCbCr) {
        img.kind = kind == JpegOut::Gray ? ZPX_GRAY : ZPX_YCBCR;
        img.pixels_len = L.total;
        img.stride = L.y_stride;
        img.y_stride = L.y_stride;
        img.c_stride = L.c_stride;
        img.cb_off = L.cb_off;
        img.cr_off = L.cr_off;
        img.subsample = L.subsample;
        img.pixels = static_cast<uint8_t *>(al_alloc(al, L.total));
        if (!img.pixels) return ZPX_E_OUT_OF_MEMORY;
        hipError_t e = hipMemcpy(img.pixels, planes.ptr, L.total, hipMemcpyDeviceToHost);
        if (e != hipSuccess) {
            al_free(al, img.pixels, L.total);
            return hip_fail(ctx, e, "planes copy-back");
        }
        if (kind == JpegOut::Gray) img.y_stride = img.c_stride = img.cb_off = img.cr_off = 0;
        *out = img;
        return ZPX_OK;
    }
    // RGB (convertToRGB) or CMYK (applyBlack): one more device pass
    zpx_image planar{};
    planar.kind = ZPX_YCBCR;
    planar.max_x = W;
    planar.max_y = H;
    planar.y_stride = L.y_stride;
    planar.c_stride = L.c_stride;
    planar.cb_off = L.cb_off;
    planar.cr_off = L.cr_off;
    planar.subsample = L.subsample;
    const DevImage m = dev_image_of(&planar, planes.ptr, nullptr);
    const size_t n = size_t(W) * H * 4;
    DevBuf dout;
    HIPCHK(ctx, dout.alloc(n));
    int rc;
    if (kind == JpegOut::RGB) {
        rc = launch_jpeg_rgb(m, c.comp[0].h / c.comp[1].h, dout.as<uint8_t>(), ctx->stream);
        img.kind = ZPX_RGBA;
    } else {
        uint32_t sub = 0;
        for (int t = 0; t < 4; t++)
            if (c.comp[t].h != c.comp[0].h || c.comp[t].v != c.comp[0].v) sub |= 1u << t;
        rc = launch_jpeg_cmyk(m, kplane.as<uint8_t>(), L.k_stride, sub, dout.as<uint8_t>(), ctx->stream);
        img.kind = ZPX_CMYK;
    }
    if (rc) return hip_fail(ctx, hipGetLastError(), "jpeg colour kernel");
    img.pixels_len = n;
    img.stride = size_t(W) * 4;
    img.pixels = static_cast<uint8_t *>(al_alloc(al, n));
    if (!img.pixels) return ZPX_E_OUT_OF_MEMORY;
    hipError_t e = hipMemcpyAsync(img.pixels, dout.ptr, n, hipMemcpyDeviceToHost, ctx->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
    if (e != hipSuccess) {
        al_free(al, img.pixels, n);
        return hip_fail(ctx, e, "rgba copy-back");
    }
    *out = img;
    return ZPX_OK;
}

extern "C" int zpx_jpeg_decode(zpx_ctx *ctx, const zpx_allocator *al, const uint8_t *buf, size_t len, zpx_image *out)
{
    return guarded([&] { return zpx_jpeg_decode_impl(ctx, al, buf, len, out); });
}

static int zpx_jpeg_decode_rgba_impl(zpx_ctx *ctx, const zpx_allocator *al, const uint8_t *buf, size_t len,
                                    uint8_t **rgba, size_t *rgba_len, uint32_t *width, uint32_t *height)
{
    if (!ctx || !rgba || !rgba_len || (!buf && len)) return ZPX_E_INVALID_ARGUMENT;
    *rgba = nullptr;
    *rgba_len = 0;
    CtxScope s(ctx);
    JpegCoeffs c;
    if (int e = jpeg_entropy_decode(buf, len, c, jpeg_huff_threads())) return e;
    const JpegOut kind = jpeg_output_kind(c);
    const size_t n = size_t(c.width) * c.height * 4;
    bool fused = kind != JpegOut::CMYK && kind != JpegOut::YCCK;
    if (fused && c.n_comp == 3)
        fused = jpeg_rgba_supported(kind == JpegOut::RGB ? ZPX_JPEG_COLOR_RGB : ZPX_JPEG_COLOR_YCBCR, c.comp[0].h,
                                    c.comp[0].v, c.comp[1].h, c.comp[1].v);
    JpegDeviceFrame d;
    if (int e = upload_jpeg(ctx, c, d)) return e;
    DevBuf dout;
    HIPCHK(ctx, dout.alloc(n));
    if (!fused) { // planes + the colour pass of rgbaPixels, one entropy decode
        DevBuf planes, desc;
        HostBuf hdesc;
        if (int e = jpeg_planes_to_rgba(ctx, c, d.f, planes, desc, hdesc, dout.as<uint8_t>(), ctx->stream)) return e;
        HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
    } else {
        d.f.rgba = dout.as<uint8_t>();
        d.f.rgba_stride = size_t(c.width) * 4;
        if (int e = run_plan_once(ctx, d.f, ZPX_JPEG_RGBA)) return e;
    }
    uint8_t *host = static_cast<uint8_t *>(al_alloc(al, n));
    if (!host) return ZPX_E_OUT_OF_MEMORY;
    hipError_t e = hipMemcpy(host, dout.ptr, n, hipMemcpyDeviceToHost);
    if (e != hipSuccess) {
        al_free(al, host, n);
        return hip_fail(ctx, e, "rgba copy-back");
    }
    *rgba = host;
    *rgba_len = n;
    if (width) *width = c.width;
    if (height) *height = c.height;
    return ZPX_OK;
}

extern "C" int zpx_jpeg_decode_rgba(zpx_ctx *ctx, const zpx_allocator *al, const uint8_t *buf, size_t len,
                                    uint8_t **rgba, size_t *rgba_len, uint32_t *width, uint32_t *height)
{
    return guarded([&] { return zpx_jpeg_decode_rgba_impl(ctx, al, buf, len, rgba, rgba_len, width, height); });
}

// ------------------------------------------------------------------ png.decode
static int zpx_png_decode_impl(zpx_ctx *ctx, const zpx_allocator *al, const uint8_t *buf, size_t len, zpx_image *out)
{
    if (!ctx || !out || (!buf && len)) return ZPX_E_INVALID_ARGUMENT;
    memset(out, 0, sizeof(*out));
    CtxScope s(ctx);
    PngStream ps;
    if (int e = png_parse(buf, len, ps, png_inflate_threads())) return e;
    const size_t out_len = size_t(ps.width) * ps.height * ps.out_bpp;
    DevBuf din, dout, dmax;
    // the inflated stream goes up as is (both kernels read it)
    const void *hin = ps.data.ptr;
    const size_t in_len = ps.data_len + ZPX_PNG_INPUT_PAD;
    HIPCHK(ctx, din.alloc(in_len));
    HIPCHK(ctx, hipMemcpyAsync(din.ptr, hin, in_len, hipMemcpyHostToDevice, ctx->stream));
    HIPCHK(ctx, dout.alloc(out_len));
    HIPCHK(ctx, dmax.alloc(16));
    HIPCHK(ctx, hipMemsetAsync(dmax.ptr, 0, 16, ctx->stream));
    zpx_png_frame f;
    memset(&f, 0, sizeof(f));
    f.width = ps.width;
    f.height = ps.height;
    f.depth = ps.depth;
    f.interlace = ps.interlace;
    f.use_transparent = ps.use_transparent;
    memcpy(f.transparent, ps.transparent, 6);
    f.filtered = din.as<uint8_t>();
    f.layout = ZPX_PNG_LAYOUT_STREAM;
    f.out = dout.as<uint8_t>();
    f.out_stride = size_t(ps.width) * ps.out_bpp;
    f.max_index = ps.kind == ZPX_PALETTED ? dmax.as<int32_t>() : nullptr;
    zpx_plan *plan = nullptr;
    if (int e = zpx_png_plan_create(ctx, &f, 1, &plan)) return e;
    int e = zpx_plan_launch(plan, ctx->stream);
    if (!e) {
        hipError_t he = hipStreamSynchronize(ctx->stream);
        if (he != hipSuccess) e = hip_fail(ctx, he, "png kernel");
    }
    if (!e) e = zpx_plan_status(plan, ctx->stream);
    zpx_plan_destroy(plan);
    if (e) return e;
    zpx_image img{};
    img.kind = ps.kind;
    img.max_x = static_cast<int32_t>(ps.width);
    img.max_y = static_cast<int32_t>(ps.height);
    img.stride = f.out_stride;
    img.pixels_len = out_len;
    img.pixels = static_cast<uint8_t *>(al_alloc(al, out_len));
    if (!img.pixels) return ZPX_E_OUT_OF_MEMORY;
    hipError_t he = hipMemcpy(img.pixels, dout.ptr, out_len, hipMemcpyDeviceToHost);
    if (he != hipSuccess) {
        al_free(al, img.pixels, out_len);
        return hip_fail(ctx, he, "png copy-back");
    }
    if (ps.kind == ZPX_PALETTED) {
        int32_t maxidx = 0;
        he = hipMemcpy(&maxidx, dmax.ptr, 4, hipMemcpyDeviceToHost);
        if (he != hipSuccess) {
            zpx_image_free(al, &img);
            return hip_fail(ctx, he, "palette index copy-back");
        }
        img.palette = static_cast<zpx_color *>(al_alloc(al, 256 * sizeof(zpx_color)));
        if (!img.palette) {
            zpx_image_free(al, &img);
            return ZPX_E_OUT_OF_MEMORY;
        }
        memcpy(img.palette, ps.palette, sizeof(ps.palette));
        // implicit palette growth (readImagePass :1079-1134)
        img.palette_len = std::max(ps.palette_len, maxidx + 1);
    }
    *out = img;
    return ZPX_OK;
}

extern "C" int zpx_png_decode(zpx_ctx *ctx, const zpx_allocator *al, const uint8_t *buf, size_t len, zpx_image *out)
{
    return guarded([&] { return zpx_png_decode_impl(ctx, al, buf, len, out); });
}

// ------------------------------------------------------------------ probes / facade
extern "C" int zpx_jpeg_probe_buffer(const uint8_t *buf, size_t len)
{
    return buf && len >= 2 && buf[0] == 0xff && buf[1] == 0xd8;
}
extern "C" int zpx_png_probe_buffer(const uint8_t *buf, size_t len)
{
    static const uint8_t sig[8] = {0x89, 'P', 'N', 'G', '\r', '\n', 0x1a, '\n'};
    return buf && len >= 8 && memcmp(buf, sig, 8) == 0;
}

static int zpx_jpeg_decode_config_impl(const uint8_t *buf, size_t len, uint32_t *width, uint32_t *height,
                                      int32_t *color_model)
{
    if (!width || !height || !color_model || (!buf && len)) return ZPX_E_INVALID_ARGUMENT;
    uint32_t w = 0, h = 0;
    int m = 0;
    if (int e = jpeg_decode_config(buf, len, w, h, m)) return e;
    *width = w;
    *height = h;
    *color_model = m;
    return ZPX_OK;
}

extern "C" int zpx_jpeg_decode_config(const uint8_t *buf, size_t len, uint32_t *width, uint32_t *height,
                                      int32_t *color_model)
{
    return guarded([&] { return zpx_jpeg_decode_config_impl(buf, len, width, height, color_model); });
}

static int zpx_png_decode_config_impl(const uint8_t *buf, size_t len, uint32_t *width, uint32_t *height)
{
    if (!width || !height || (!buf && len)) return ZPX_E_INVALID_ARGUMENT;
    uint32_t w = 0, h = 0;
    if (int e = png_decode_config(buf, len, w, h)) return e;
    *width = w;
    *height = h;
    return ZPX_OK;
}

extern "C" int zpx_png_decode_config(const uint8_t *buf, size_t len, uint32_t *width, uint32_t *height)
{
    return guarded([&] { return zpx_png_decode_config_impl(buf, len, width, height); });
}

static int zpx_jpeg_load_impl(zpx_ctx *ctx, const zpx_allocator *al, const char *path, zpx_image *out)
{
    std::vector<uint8_t> data;
    if (!path) return ZPX_E_INVALID_ARGUMENT;
    if (int e = read_file(path, data)) return e;
    return zpx_jpeg_decode(ctx, al, data.data(), data.size(), out);
}

extern "C" int zpx_jpeg_load(zpx_ctx *ctx, const zpx_allocator *al, const char *path, zpx_image *out)
{
    return guarded([&] { return zpx_jpeg_load_impl(ctx, al, path, out); });
}

static int zpx_png_load_impl(zpx_ctx *ctx, const zpx_allocator *al, const char *path, zpx_image *out)
{
    std::vector<uint8_t> data;
    if (!path) return ZPX_E_INVALID_ARGUMENT;
    if (int e = read_file(path, data)) return e;
    return zpx_png_decode(ctx, al, data.data(), data.size(), out);
}

extern "C" int zpx_png_load(zpx_ctx *ctx, const zpx_allocator *al, const char *path, zpx_image *out)
{
    return guarded([&] { return zpx_png_load_impl(ctx, al, path, out); });
}

extern "C" int zpx_from_buffer(zpx_ctx *ctx, const zpx_allocator *al, const uint8_t *buf, size_t len, zpx_image *out)
{
    if (zpx_png_probe_buffer(buf, len)) return zpx_png_decode(ctx, al, buf, len, out);
    if (zpx_jpeg_probe_buffer(buf, len)) return zpx_jpeg_decode(ctx, al, buf, len, out);
    if (zpx_qoi_probe_buffer(buf, len)) return zpx_qoi_decode(ctx, al, buf, len, out);
    if (zpx_bmp_probe_buffer(buf, len)) return zpx_bmp_decode(ctx, al, buf, len, out);
    return ZPX_E_UNKNOWN_IMAGE_FORMAT;
}

static int zpx_from_file_path_impl(zpx_ctx *ctx, const zpx_allocator *al, const char *path, zpx_image *out)
{
    std::vector<uint8_t> data;
    if (!path) return ZPX_E_INVALID_ARGUMENT;
    if (int e = read_file(path, data)) return e;
    return zpx_from_buffer(ctx, al, data.data(), data.size(), out);
}

extern "C" int zpx_from_file_path(zpx_ctx *ctx, const zpx_allocator *al, const char *path, zpx_image *out)
{
    return guarded([&] { return zpx_from_file_path_impl(ctx, al, path, out); });
}

// ------------------------------------------------------------------ fault injection
// One stalled launch of either PNG kernel: a W x 2*band_rows RGB8 image,
// every row Up-filtered, of which only band 1 is scheduled, so its first row
// waits for band 0's last row forever.
static int png_stall_once(zpx_ctx *ctx, bool pair, uint32_t spin_limit, double &secs, bool &timed_out)
{
    const uint32_t band_rows = pair ? 128 : 64;
    const uint32_t W = 64, H = 2 * band_rows, rb = W * 3;
    std::vector<uint8_t> filt(size_t(H) * (rb + 1) + ZPX_PNG_INPUT_PAD, 0);
    for (uint32_t y = 0; y < H; y++) filt[size_t(y) * (rb + 1)] = 2;
    zpx_png_frame f;
    memset(&f, 0, sizeof(f));
    f.width = W;
    f.height = H;
    f.depth = ZPX_PNG_TC8;
    f.out_stride = size_t(W) * 4;
    if (pair) { // the paired-row kernel reads the band slab (png_slab.cpp)
        std::vector<uint64_t> off;
        f.filtered = filt.data();
        std::vector<uint8_t> slab(png_slab_layout(f, off));
        png_slab_fill(f, off, slab.data());
        filt.swap(slab);
        f.layout = ZPX_PNG_LAYOUT_SLAB;
    }
    DevBuf din, dout, bound, dpass, dsched;
    HIPCHK(ctx, din.alloc(filt.size()));
    HIPCHK(ctx, hipMemcpy(din.ptr, filt.data(), filt.size(), hipMemcpyHostToDevice));
    HIPCHK(ctx, dout.alloc(size_t(W) * H * 4));
    f.filtered = din.as<uint8_t>();
    f.out = dout.as<uint8_t>();
    std::vector<DevPngPass> passes;
    std::vector<uint32_t> rbs;
    uint64_t bytes = 0;
    png_frame_passes(f, passes, rbs, bytes);
    passes[0].nbands = 2;
    passes[0].band_base = 0;
    const DevPngBand only{0, 1}; // band 1 alone: band 0 never runs, so never publishes
    const uint32_t granules = static_cast<uint32_t>(png_band_granules(ZPX_PNG_TC8, rb));
    PngControl ctl;
    if (int e = ctl.init(ctx)) return e;
    HIPCHK(ctx, bound.alloc(size_t(2) * granules * sizeof(uint64_t)));
    HIPCHK(ctx, hipMemset(bound.ptr, 0, size_t(2) * granules * sizeof(uint64_t)));
    HIPCHK(ctx, dpass.alloc(sizeof(DevPngPass)));
    HIPCHK(ctx, hipMemcpy(dpass.ptr, passes.data(), sizeof(DevPngPass), hipMemcpyHostToDevice));
    HIPCHK(ctx, dsched.alloc(sizeof(DevPngBand)));
    HIPCHK(ctx, hipMemcpy(dsched.ptr, &only, sizeof(DevPngBand), hipMemcpyHostToDevice));
    HIPCHK(ctx, hipDeviceSynchronize());
    const auto t0 = std::chrono::steady_clock::now();
    const int rc = pair ? launch_png_pair(ZPX_PNG_TC8, false, false, dpass.as<DevPngPass>(), dsched.as<DevPngBand>(), 1,
                                          ctl.words(), bound.as<uint64_t>(), granules, ctx->stream, spin_limit)
                        : launch_png_unfilter(ZPX_PNG_TC8, dpass.as<DevPngPass>(), dsched.as<DevPngBand>(), 1,
                                              ctl.words(), bound.as<uint64_t>(), granules, ctx->stream,
                                              spin_limit);
    if (rc)
        return hip_fail(ctx, hipGetLastError(), "png stall kernel launch");
    HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
    secs = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    uint32_t st[2] = {0, 0};
    HIPCHK(ctx, hipMemcpy(st, ctl.words() + 2, 8, hipMemcpyDeviceToHost));
    timed_out = (st[0] | st[1]) != 0;
    return ZPX_OK;
}

static int zpx_debug_png_stall_impl(zpx_ctx *ctx, uint32_t spin_limit, double *seconds)
{
    if (!ctx || spin_limit == 0) return ZPX_E_INVALID_ARGUMENT;
    CtxScope s(ctx);
    double worst = 0;
    bool all_timed_out = true;
    for (bool pair : {false, true}) { // both kernels' bounded waits
        double secs = 0;
        bool to = false;
        if (int e = png_stall_once(ctx, pair, spin_limit, secs, to)) return e;
        worst = std::max(worst, secs);
        all_timed_out &= to;
    }
    if (seconds) *seconds = worst;
    if (all_timed_out) {
        ctx->last_error = "png wavefront hand-off timed out";
        return ZPX_E_HIP;
    }
    return ZPX_OK;
}

namespace zpx {
namespace {
// JpegStrip, JpegSparse, PngPair, QoiSegment, PngDeviceSlab, PngEpochCycle, ShardRcclSelf, BatchLookahead,
// InflatePair, BatchMakespan, BatchSlotCache
std::atomic<int> g_opt[static_cast<int>(Opt::Count)] = {{0}, {1}, {1}, {0}, {0}, {0}, {0}, {0}, {1}, {1}, {1}};
const char *const kOptNames[static_cast<int>(Opt::Count)] = {
    "jpeg_strip",      "jpeg_sparse",     "png_pair",        "qoi_segment",     "png_device_slab",
    "png_epoch_cycle", "shard_rccl_self", "batch_lookahead", "inflate_pair",    "batch_makespan",
    "batch_slot_cache"};
} // namespace
int opt(Opt o) { return g_opt[static_cast<int>(o)].load(std::memory_order_relaxed); }
} // namespace zpx

extern "C" int zpx_debug_option(const char *name, int value)
{
    for (int i = 0; name && i < static_cast<int>(Opt::Count); i++)
        if (strcmp(name, kOptNames[i]) == 0) return g_opt[i].exchange(value);
    return -1;
}

extern "C" int zpx_debug_png_stall(zpx_ctx *ctx, uint32_t spin_limit, double *seconds)
{
    return guarded([&] { return zpx_debug_png_stall_impl(ctx, spin_limit, seconds); });
}

extern "C" int64_t zpx_debug_jpeg_parallel_scans(void) { return jpeg_parallel_scans(); }
extern "C" int64_t zpx_debug_jpeg_parallel_progressive(void) { return jpeg_parallel_progressive(); }

// Test hook for the compact coefficient pieces (JpegPieces): decodes `buf`
// in pieces mode and expands them on the host, as jpeg_pieces_expand_kernel
// does, into int32 grids laid out component after component (blocks x 64,
// natural order), checking the layout's invariants on the way (piece 0 zero,
// every block's pieces inside the data and in order, nothing nonzero past a
// block's last piece's values).  Returns the number of blocks, 0 when the
// frame was decoded into grids instead, or -(error code).
extern "C" int64_t zpx_debug_jpeg_sparse_grids(const uint8_t *buf, size_t len, int32_t *grids, size_t grid_elems)
{
    return guarded([&]() -> int64_t {
        JpegCoeffs c;
        if (int e = jpeg_entropy_decode(buf, len, c, 1, true)) return -int64_t(e);
        const JpegPieces &p = c.pieces;
        if (!p.valid) return 0;
        size_t total = 0, blocks = 0;
        for (int i = 0; i < c.n_comp; i++) {
            total += p.blocks[i] * 64;
            blocks += p.blocks[i];
        }
        if (total > grid_elems) return -int64_t(ZPX_E_INVALID_ARGUMENT);
        const uint8_t *data = static_cast<const uint8_t *>(p.data.ptr);
        for (int k = 0; k < 16; k++)
            if (data[k]) return -int64_t(ZPX_E_PANIC);
        static const uint8_t kZz[64] = {0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,
                                        12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6,  7,  14, 21, 28,
                                        35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51,
                                        58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};
        const int per = p.bits == 8 ? 16 : 8;
        // every piece but piece 0 belongs to exactly one block (the streams
        // compacted back to back, JpegPieces::compact)
        std::vector<uint8_t> owner(p.npieces, 0);
        int32_t *o = grids;
        for (int ci = 0; ci < c.n_comp; ci++) {
            const uint32_t *ix = p.index_of(ci);
            for (size_t blk = 0; blk < p.blocks[ci]; blk++, o += 64) {
                const uint32_t np = ix[blk] & 15, first = ix[blk] >> 4;
                for (int i = 0; i < 64; i++) o[i] = 0;
                if (np == 0) {
                    if (first != 0) return -int64_t(ZPX_E_PANIC);
                    continue;
                }
                if (first == 0 || first + np > p.npieces || np * static_cast<uint32_t>(per) > uint32_t(64 + per - 1)) return -int64_t(ZPX_E_PANIC);
                for (uint32_t q = 0; q < np; q++)
                    if (owner[first + q]++) return -int64_t(ZPX_E_PANIC);
                for (uint32_t z = 0; z < np * per && z < 64; z++) {
                    int32_t v;
                    if (p.bits == 8) {
                        v = static_cast<int8_t>(data[size_t(first) * 16 + z]);
                    } else {
                        int16_t h;
                        memcpy(&h, data + size_t(first) * 16 + 2 * z, 2);
                        v = h;
                    }
                    o[kZz[z]] = v;
                }
            }
        }
        for (size_t q = 1; q < p.npieces; q++)
            if (!owner[q]) return -int64_t(ZPX_E_PANIC);
        return int64_t(blocks);
    });
}

// Test hook for the host inflate's fast decoders: 1 when the speculative
// parallel inflate (threads >= 2; inflate_parallel) or, for threads = 1, the
// serial fast decoder (inflate_fast) decoded the first `want` bytes of the
// zlib stream `z`; 0 when it declined (the PNG path then falls back: to the
// serial decoder, or from it to system zlib).
extern "C" int zpx_debug_inflate_parallel(const uint8_t *z, size_t len, uint8_t *out, size_t want, int threads)
{
    return guarded([&] {
        size_t produced = 0;
        if (threads == 1) return inflate_fast(z, len, out, want, &produced) && produced == want ? 1 : 0;
        return inflate_parallel(z, len, out, want, &produced, threads) && produced == want ? 1 : 0;
    });
}
