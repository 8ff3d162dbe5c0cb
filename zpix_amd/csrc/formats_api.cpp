// C-ABI of the format edges next to the JPEG/PNG path:
//   - bmp.decode: host header/palette parse (src/bmp/decoder.zig:42-158), the
//     row loop on the GPU (bmp_kernels.hip);
//   - qoi.decode: serial host loop (src/qoi/decoder.zig:28-130);
//   - qoi.encode: the GPU segmented-scan encoder (qoi_kernels.hip), host and
//     device forms.
#include <cstring>

#include "api_internal.h"
#include "kernels.h"

using namespace zpx;

namespace {

inline uint32_t le32(const uint8_t *b) { return b[0] | uint32_t(b[1]) << 8 | uint32_t(b[2]) << 16 | uint32_t(b[3]) << 24; }
inline uint32_t le16(const uint8_t *b) { return b[0] | uint32_t(b[1]) << 8; }
inline uint32_t be32(const uint8_t *b) { return uint32_t(b[0]) << 24 | uint32_t(b[1]) << 16 | uint32_t(b[2]) << 8 | b[3]; }

struct BmpHeader {
    uint32_t width = 0, height = 0, bpp = 0, ncol = 0;
    bool top_down = false, allow_alpha = false;
    size_t data = 0, row_bytes = 0; // pixel rows start at buf + data
    zpx_color palette[256]{};
};

// readHeader (decoder.zig:42-158), errors in the reference's order; the
// reader is a fixed buffer, so a short read is EndOfStream.
int bmp_parse(const uint8_t *b, size_t len, BmpHeader &h)
{
    if (len < 18) return ZPX_E_END_OF_STREAM;
    if (!(b[0] == 'B' && b[1] == 'M')) return ZPX_E_INVALID_SIGNATURE;
    const uint32_t pixel_off = le32(b + 10), info_len = le32(b + 14);
    if (info_len != 40 && info_len != 108 && info_len != 124) return ZPX_E_UNSUPPORTED_HEADER;
    if (len < 14 + size_t(info_len)) return ZPX_E_END_OF_STREAM;
    const int32_t w = static_cast<int32_t>(le32(b + 18));
    int32_t hh = static_cast<int32_t>(le32(b + 22));
    if (hh < 0) {
        if (hh == INT32_MIN) return ZPX_E_UNSUPPORTED_DIMENSIONS; // the reference's negation would trap
        hh = -hh;
        h.top_down = true;
    }
    if (w < 0) return ZPX_E_UNSUPPORTED_DIMENSIONS;
    const uint32_t planes = le16(b + 26), bpp = le16(b + 28);
    uint32_t compression = le32(b + 30);
    if (compression == 3 && info_len > 40 && le32(b + 54) == 0xff0000 && le32(b + 58) == 0x00ff00 &&
        le32(b + 62) == 0x0000ff && le32(b + 66) == 0xff000000u)
        compression = 0; // BI_BITFIELDS with the default masks (:77-86)
    if (planes != 1 || compression != 0) return ZPX_E_UNSUPPORTED_COMPRESSION;
    h.width = static_cast<uint32_t>(w);
    h.height = static_cast<uint32_t>(hh);
    h.bpp = bpp;
    h.allow_alpha = info_len > 40;
    size_t pos = 14 + size_t(info_len);
    if (bpp == 1 || bpp == 2 || bpp == 4 || bpp == 8) {
        uint32_t ncol = le32(b + 46);
        if (ncol == 0) ncol = 1u << bpp;
        else if (ncol > (1u << bpp)) return ZPX_E_UNSUPPORTED_PALETTE_SIZE;
        if (pixel_off != 14 + info_len + ncol * 4) return ZPX_E_UNSUPPORTED_COLOR_OFFSET;
        if (len - pos < size_t(ncol) * 4) return ZPX_E_END_OF_STREAM;
        for (uint32_t i = 0; i < ncol; i++) { // B,G,R,pad -> .rgba with A = 0xFF
            const uint8_t *e = b + pos + 4 * i;
            h.palette[i] = zpx_color{e[2], e[1], e[0], 0xff, 0, {0, 0, 0}};
        }
        h.ncol = ncol;
        pos += size_t(ncol) * 4;
        const uint32_t ppb = 8 / bpp;
        h.row_bytes = ((size_t(h.width) + ppb - 1) / ppb + 3) & ~size_t(3);
    } else if (bpp == 24 || bpp == 32) {
        if (pixel_off != 14 + info_len) return ZPX_E_UNSUPPORTED_COLOR_OFFSET;
        h.row_bytes = bpp == 24 ? (size_t(h.width) * 3 + 3) & ~size_t(3) : size_t(h.width) * 4;
    } else {
        return ZPX_E_UNSUPPORTED_BPP;
    }
    h.data = pos;
    return ZPX_OK;
}

int bmp_decode_impl(zpx_ctx *ctx, const zpx_allocator *al, const uint8_t *buf, size_t len, zpx_image *out)
{
    if (!out || (!buf && len)) return ZPX_E_INVALID_ARGUMENT;
    memset(out, 0, sizeof(*out));
    BmpHeader h;
    if (int e = bmp_parse(buf, len, h)) return e;
    const bool paletted = h.ncol != 0;
    const bool empty = h.width == 0 || h.height == 0;
    // the rows are read one after the other; a short file fails on the first missing row
    if (!empty && (len - h.data) / h.row_bytes < h.height) return ZPX_E_END_OF_STREAM;
    if (!ctx) return ZPX_E_INVALID_ARGUMENT;
    zpx_image img{};
    img.kind = paletted ? ZPX_PALETTED : h.bpp == 24 ? ZPX_RGBA : ZPX_NRGBA;
    // an empty Paletted image has rect (0,0,0,0) (:163-172); RGBA/NRGBA keep width x height
    img.max_x = static_cast<int32_t>(paletted && empty ? 0 : h.width);
    img.max_y = static_cast<int32_t>(paletted && empty ? 0 : h.height);
    img.stride = size_t(img.max_x) * (paletted ? 1 : 4);
    img.pixels_len = img.stride * size_t(img.max_y);
    if (paletted) {
        img.palette = static_cast<zpx_color *>(al_alloc(al, 256 * sizeof(zpx_color)));
        if (!img.palette) return ZPX_E_OUT_OF_MEMORY;
        memcpy(img.palette, h.palette, sizeof(h.palette));
        img.palette_len = static_cast<int32_t>(h.ncol);
    }
    img.pixels = static_cast<uint8_t *>(al_alloc(al, img.pixels_len));
    if (!img.pixels) {
        zpx_image_free(al, &img);
        return ZPX_E_OUT_OF_MEMORY;
    }
    if (img.pixels_len) {
        CtxScope s(ctx);
        const size_t in_bytes = h.row_bytes * h.height;
        DevBuf din, dout;
        int e = ZPX_OK;
        hipError_t he = din.alloc(in_bytes);
        if (he == hipSuccess) he = hipMemcpyAsync(din.ptr, buf + h.data, in_bytes, hipMemcpyHostToDevice, ctx->stream);
        if (he == hipSuccess) he = dout.alloc(img.pixels_len);
        if (he == hipSuccess &&
            launch_bmp_rows(static_cast<int>(h.bpp), h.allow_alpha, din.as<uint8_t>(), h.row_bytes, dout.as<uint8_t>(),
                            img.stride, h.width, h.height, h.top_down, ctx->stream)) {
            he = hipGetLastError();
            if (he == hipSuccess) he = hipErrorLaunchFailure;
        }
        if (he == hipSuccess)
            he = hipMemcpyAsync(img.pixels, dout.ptr, img.pixels_len, hipMemcpyDeviceToHost, ctx->stream);
        if (he == hipSuccess) he = hipStreamSynchronize(ctx->stream);
        if (he != hipSuccess) e = hip_fail(ctx, he, "bmp_rows_kernel");
        if (e) {
            zpx_image_free(al, &img);
            return e;
        }
    }
    *out = img;
    return ZPX_OK;
}

inline unsigned qoi_hash(const uint8_t *p) { return (p[0] * 3u + p[1] * 5u + p[2] * 7u + p[3] * 11u) & 63u; }
constexpr uint32_t kQoiPixelsMax = 400000000u;

// decodeFromBuffer (decoder.zig:28-130)
int qoi_decode_impl(const zpx_allocator *al, const uint8_t *data, size_t len, zpx_image *out)
{
    if (!out || (!data && len)) return ZPX_E_INVALID_ARGUMENT;
    memset(out, 0, sizeof(*out));
    if (len < 14 + 8) return ZPX_E_INVALID_QOI_DATA;
    if (be32(data) != 0x716F6966u) return ZPX_E_INVALID_QOI_HEADER;
    const uint32_t width = be32(data + 4), height = be32(data + 8);
    const uint8_t channels = data[12], colorspace = data[13];
    if (width == 0 || height == 0 || (channels != 3 && channels != 4) || colorspace > 1 ||
        height >= kQoiPixelsMax / width)
        return ZPX_E_INVALID_QOI_HEADER;
    const size_t n = size_t(width) * height, chunks_len = len - 8;
    zpx_image img{};
    img.kind = ZPX_RGBA;
    img.max_x = static_cast<int32_t>(width);
    img.max_y = static_cast<int32_t>(height);
    img.stride = size_t(width) * 4;
    img.pixels_len = n * 4;
    img.pixels = static_cast<uint8_t *>(al_alloc(al, img.pixels_len));
    if (!img.pixels) return ZPX_E_OUT_OF_MEMORY;
    uint8_t index[64][4] = {};
    uint8_t px[4] = {0, 0, 0, 255};
    size_t p = 14, run = 0;
    uint8_t *o = img.pixels;
    for (size_t i = 0; i < n; i++, o += 4) {
        if (run > 0) {
            run--;
        } else if (p < chunks_len) {
            const uint8_t b1 = data[p++];
            // payload bytes are read without the chunks_len check (:71-82); past
            // the end of the buffer the reference's bounds check panics, which
            // maps to ZPX_E_PANIC.  Its other safety trap -- @intCast of a
            // DIFF/LUMA step that leaves 0..255 (:97-114) -- is NOT mapped:
            // those steps wrap mod 256, as the QOI specification (and qoi.h's
            // encoder, which emits them for 255 -> 0) has them, and as a
            // ReleaseFast reference build truncates; the reference's own
            // encoder never emits one (encoder.zig:97-101).  The oracle does
            // the same (zo_qoi_decode), pinned by tests/test_oracle.py
            // test_qoi_decode_wrapping_diff.
            const size_t need = b1 == 0xfe ? 3 : b1 == 0xff ? 4 : (b1 & 0xc0) == 0x80 ? 1 : 0;
            if (p + need > len) {
                zpx_image_free(al, &img);
                return ZPX_E_PANIC;
            }
            switch (b1 >> 6) {
            case 3:
                if (b1 == 0xfe) {
                    memcpy(px, data + p, 3);
                    p += 3;
                } else if (b1 == 0xff) {
                    memcpy(px, data + p, 4);
                    p += 4;
                } else {
                    run = b1 & 0x3f; // QOI_OP_RUN
                }
                break;
            case 0: memcpy(px, index[b1 & 0x3f], 4); break;
            case 1: // QOI_OP_DIFF (mod 256, see above)
                px[0] = static_cast<uint8_t>(px[0] + ((b1 >> 4) & 3) - 2);
                px[1] = static_cast<uint8_t>(px[1] + ((b1 >> 2) & 3) - 2);
                px[2] = static_cast<uint8_t>(px[2] + (b1 & 3) - 2);
                break;
            default: { // QOI_OP_LUMA
                const uint8_t b2 = data[p++];
                const int dg = (b1 & 0x3f) - 32;
                px[0] = static_cast<uint8_t>(px[0] + dg + ((b2 >> 4) & 0xf) - 8);
                px[1] = static_cast<uint8_t>(px[1] + dg);
                px[2] = static_cast<uint8_t>(px[2] + dg + (b2 & 0xf) - 8);
            }
            }
            memcpy(index[qoi_hash(px)], px, 4);
        }
        memcpy(o, px, 4);
    }
    *out = img;
    return ZPX_OK;
}

bool qoi_desc_ok(const zpx_qoi_desc *d)
{
    return d->width != 0 && d->height != 0 && d->channels >= 3 && d->channels <= 4 && d->colorspace <= 1 &&
           d->height < kQoiPixelsMax / d->width;
}

uint32_t qoi_segment()
{
    // pixels per lane's segment: 128, or the test switch "qoi_segment"
    // (16..4096, whole load groups) -- the bytes are the same at every size
    const int v = opt(Opt::QoiSegment);
    return v >= 16 && v <= 4096 ? static_cast<uint32_t>(v) & ~15u : 128u;
}

int qoi_encode_device_impl(zpx_ctx *ctx, const uint8_t *d_pixels, const zpx_qoi_desc *desc, uint8_t *d_out,
                           size_t out_cap, uint64_t *d_out_len, void *stream)
{
    if (!ctx || !desc || !d_pixels || !d_out || !d_out_len) return ZPX_E_INVALID_ARGUMENT;
    if (!qoi_desc_ok(desc)) return ZPX_E_INVALID_QOI_HEADER;
    if (out_cap < zpx_qoi_encode_bound(desc)) return ZPX_E_INVALID_ARGUMENT;
    CtxScope s(ctx);
    const uint64_t n = uint64_t(desc->width) * desc->height;
    const uint32_t S = qoi_segment();
    QoiEncodeArgs a;
    const size_t scratch = qoi_scratch_layout(n, S, nullptr, nullptr);
    hipStream_t st = stream ? static_cast<hipStream_t>(stream) : ctx->stream;
    // the context's scratch is shared: order this encode after the previous
    // user's work, whatever stream that ran on (see zpx_ctx::scratch_ev)
    std::lock_guard<std::mutex> lk(ctx->scratch_mu);
    if (!ctx->scratch_ev) HIPCHK(ctx, hipEventCreateWithFlags(&ctx->scratch_ev, hipEventDisableTiming));
    else HIPCHK(ctx, hipStreamWaitEvent(st, ctx->scratch_ev, 0));
    HIPCHK(ctx, ctx_scratch(ctx, scratch));
    qoi_scratch_layout(n, S, &a, static_cast<uint8_t *>(ctx->scratch));
    a.pixels = d_pixels;
    a.width = desc->width;
    a.height = desc->height;
    a.colorspace = desc->colorspace;
    a.out = d_out;
    a.out_len = d_out_len;
    if (launch_qoi_encode(desc->channels, a, st)) return hip_fail(ctx, hipGetLastError(), "qoi encode kernels");
    HIPCHK(ctx, hipEventRecord(ctx->scratch_ev, st));
    return ZPX_OK;
}

int qoi_encode_impl(zpx_ctx *ctx, const zpx_allocator *al, const uint8_t *pixels, size_t pixels_len,
                    const zpx_qoi_desc *desc, uint8_t **out, size_t *out_len)
{
    if (!ctx || !desc || !out || !out_len) return ZPX_E_INVALID_ARGUMENT;
    *out = nullptr;
    *out_len = 0;
    if (!qoi_desc_ok(desc)) return ZPX_E_INVALID_QOI_HEADER;
    const size_t px_len = size_t(desc->width) * desc->height * desc->channels;
    if (!pixels || pixels_len < px_len) return ZPX_E_INVALID_ARGUMENT; // the reference indexes pixels[0..pxLen)
    CtxScope s(ctx);
    const size_t cap = zpx_qoi_encode_bound(desc);
    DevBuf din, dout, dlen;
    HIPCHK(ctx, din.alloc(px_len));
    HIPCHK(ctx, hipMemcpyAsync(din.ptr, pixels, px_len, hipMemcpyHostToDevice, ctx->stream));
    HIPCHK(ctx, dout.alloc(cap));
    HIPCHK(ctx, dlen.alloc(sizeof(uint64_t)));
    if (int e = qoi_encode_device_impl(ctx, din.as<uint8_t>(), desc, dout.as<uint8_t>(), cap, dlen.as<uint64_t>(),
                                       nullptr))
        return e;
    uint64_t n = 0;
    HIPCHK(ctx, hipMemcpyAsync(&n, dlen.ptr, sizeof(n), hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
    if (n < 22 || n > cap) {
        ctx->last_error = "qoi encode: impossible encoded length";
        return ZPX_E_PANIC;
    }
    uint8_t *host = static_cast<uint8_t *>(al_alloc(al, n));
    if (!host) return ZPX_E_OUT_OF_MEMORY;
    hipError_t he = hipMemcpy(host, dout.ptr, n, hipMemcpyDeviceToHost);
    if (he != hipSuccess) {
        al_free(al, host, n);
        return hip_fail(ctx, he, "qoi copy-back");
    }
    *out = host;
    *out_len = n;
    return ZPX_OK;
}

} // namespace

extern "C" int zpx_bmp_probe_buffer(const uint8_t *buf, size_t len) { return buf && len >= 2 && buf[0] == 'B' && buf[1] == 'M'; }

extern "C" int zpx_bmp_decode(zpx_ctx *ctx, const zpx_allocator *al, const uint8_t *buf, size_t len, zpx_image *out)
{
    return guarded([&] { return bmp_decode_impl(ctx, al, buf, len, out); });
}

extern "C" int zpx_bmp_load(zpx_ctx *ctx, const zpx_allocator *al, const char *path, zpx_image *out)
{
    return guarded([&] {
        std::vector<uint8_t> data;
        if (!path) return int(ZPX_E_INVALID_ARGUMENT);
        if (int e = read_file(path, data)) return e;
        return bmp_decode_impl(ctx, al, data.data(), data.size(), out);
    });
}

extern "C" int zpx_qoi_probe_buffer(const uint8_t *buf, size_t len) { return buf && len >= 4 && memcmp(buf, "qoif", 4) == 0; }

extern "C" int zpx_qoi_decode(zpx_ctx *, const zpx_allocator *al, const uint8_t *buf, size_t len, zpx_image *out)
{
    return guarded([&] { return qoi_decode_impl(al, buf, len, out); });
}

extern "C" int zpx_qoi_load(zpx_ctx *, const zpx_allocator *al, const char *path, zpx_image *out)
{
    return guarded([&] {
        std::vector<uint8_t> data;
        if (!path) return int(ZPX_E_INVALID_ARGUMENT);
        if (int e = read_file(path, data)) return e;
        return qoi_decode_impl(al, data.data(), data.size(), out);
    });
}

extern "C" size_t zpx_qoi_encode_bound(const zpx_qoi_desc *d)
{
    if (!d) return 0;
    return size_t(d->width) * d->height * (size_t(d->channels) + 1) + 14 + 8;
}

extern "C" int zpx_qoi_encode(zpx_ctx *ctx, const zpx_allocator *al, const uint8_t *pixels, size_t pixels_len,
                              const zpx_qoi_desc *desc, uint8_t **out, size_t *out_len)
{
    return guarded([&] { return qoi_encode_impl(ctx, al, pixels, pixels_len, desc, out, out_len); });
}

extern "C" int zpx_qoi_encode_device(zpx_ctx *ctx, const uint8_t *d_pixels, const zpx_qoi_desc *desc, uint8_t *d_out,
                                     size_t out_cap, uint64_t *d_out_len, void *stream)
{
    return guarded([&] { return qoi_encode_device_impl(ctx, d_pixels, desc, d_out, out_cap, d_out_len, stream); });
}
