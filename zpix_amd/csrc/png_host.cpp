// Host stage of the PNG path.  Follows the control flow of
// src/png/decoder.zig (decode :143-221, parseChunk :231-324, parseIhdr
// :326-401, parseIdat :404-545, parseTrns :547-602, parsePlte :604-646,
// verifyChecksum :1264-1277) so error names match; inflate uses system zlib
// (the reference uses Zig std.compress.flate; inflate is lossless, so the
// bytes are identical).
#include "png_host.h"
#include "host_cpus.h"

#include "crc32_fast.h"
#include "inflate_fast.h"

#include <zlib.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <thread>
#include <vector>

namespace zpx {
namespace {

constexpr uint32_t kAdam7[7][4] = {{0, 0, 8, 8}, {4, 0, 8, 8}, {0, 4, 4, 8}, {2, 0, 4, 4},
                                   {0, 2, 2, 4}, {1, 0, 2, 2}, {0, 1, 1, 2}};

inline uint32_t be32(const uint8_t *b)
{
    return uint32_t(b[0]) << 24 | uint32_t(b[1]) << 16 | uint32_t(b[2]) << 8 | b[3];
}

int bits_of(int depth)
{
    switch (depth) {
    case ZPX_PNG_G1: case ZPX_PNG_P1: return 1;
    case ZPX_PNG_G2: case ZPX_PNG_P2: return 2;
    case ZPX_PNG_G4: case ZPX_PNG_P4: return 4;
    case ZPX_PNG_G8: case ZPX_PNG_P8: return 8;
    case ZPX_PNG_GA8: case ZPX_PNG_G16: return 16;
    case ZPX_PNG_TC8: return 24;
    case ZPX_PNG_TCA8: case ZPX_PNG_GA16: return 32;
    case ZPX_PNG_TC16: return 48;
    case ZPX_PNG_TCA16: return 64;
    }
    return 0;
}
bool paletted(int d) { return d >= ZPX_PNG_P1 && d <= ZPX_PNG_P8; }

// System zlib over the whole stream: `produced` bytes written before it
// stopped; `data_error` when it stopped on corrupt data (vs. running out).
int inflate_zlib(const std::vector<uint8_t> &z, uint8_t *dst, size_t total, size_t &produced, bool &data_error)
{
    z_stream zs;
    memset(&zs, 0, sizeof(zs));
    if (inflateInit(&zs) != Z_OK) return ZPX_E_OUT_OF_MEMORY;
    zs.next_in = const_cast<Bytef *>(z.data());
    zs.avail_in = static_cast<uInt>(z.size());
    produced = 0;
    data_error = false;
    while (produced < total) {
        const size_t want = total - produced;
        zs.next_out = dst + produced;
        zs.avail_out = static_cast<uInt>(want > (1u << 30) ? (1u << 30) : want);
        const uInt before = zs.avail_out;
        const int r = inflate(&zs, Z_NO_FLUSH);
        produced += before - zs.avail_out;
        if (r == Z_STREAM_END) break;
        if (r == Z_OK) continue;
        if (r == Z_BUF_ERROR && zs.avail_in == 0) break; // truncated stream
        if (r == Z_BUF_ERROR) continue;
        data_error = true;
        break;
    }
    inflateEnd(&zs);
    return ZPX_OK;
}

// Reused buffers for the concatenated IDAT data: a fresh 40 MB vector per
// 4K image cost a page fault per 4 KiB page on its first touch (the IDAT
// copy ran at 1.5 GB/s into fresh pages, ~25 ms of a ~220 ms parse here);
// recycled ones keep their pages.  Bounded: at most kZPoolBytes held, and
// at most as many buffers as the batch pipeline's parsers can have in use
// at once (two per host worker, min(16, budget) workers: host_cpus.h) -- the
// working set of the busiest batch, which zpx_host_pools_trim() releases.
class ZPool {
  public:
    std::vector<uint8_t> take()
    {
        std::lock_guard<std::mutex> lk(mu_);
        if (free_.empty()) return {};
        std::vector<uint8_t> v = std::move(free_.back());
        free_.pop_back();
        held_ -= v.capacity();
        return v;
    }
    void give(std::vector<uint8_t> &&v)
    {
        static const size_t kMaxFree = 2 * size_t(std::min(16, host_cpu_budget())) + 2;
        std::vector<uint8_t> keep = std::move(v); // (freed on return unless pooled)
        keep.clear();
        std::lock_guard<std::mutex> lk(mu_);
        if (keep.capacity() == 0 || held_ + keep.capacity() > kZPoolBytes || free_.size() >= kMaxFree) return;
        held_ += keep.capacity();
        free_.push_back(std::move(keep));
    }
    size_t trim() // the bytes released
    {
        std::vector<std::vector<uint8_t>> gone;
        std::lock_guard<std::mutex> lk(mu_);
        const size_t n = held_;
        gone.swap(free_);
        held_ = 0;
        return n;
    }

  private:
    static constexpr size_t kZPoolBytes = size_t(2) << 30;
    std::mutex mu_;
    std::vector<std::vector<uint8_t>> free_;
    size_t held_ = 0;
};
ZPool &zpool()
{
    static ZPool *p = new ZPool; // (intentionally leaked, like the pinned pool)
    return *p;
}

class Parser {
  public:
    Parser(const uint8_t *p, size_t n, PngStream &o, int threads) : src_(p), len_(n), o_(o), threads_(threads) {}
    ~Parser() { zpool().give(std::move(z_)); }
    Parser(const Parser &) = delete;
    Parser &operator=(const Parser &) = delete;
    int run(bool header_only = false);
    // Deferred inflate (png_parse_pair): the IDAT stage only sets the job up
    // and the chunk walk goes on; complete() takes the inflated bytes'
    // checks after the caller inflated them (inflate_fast_pair).
    void defer() { defer_ = true; }
    bool pending() const { return pending_; }
    const std::vector<uint8_t> &job_z() const { return z_; }
    uint8_t *job_dst() const { return static_cast<uint8_t *>(o_.data.ptr); }
    size_t job_want() const { return o_.data_len; }
    // the job's inflate result (ok: inflate_fast's), else its zlib fallback,
    // then the row checks; `run_status` is run()'s, whose chunk errors
    // after the IDAT rank behind the image's own
    int complete(int run_status, bool ok, size_t produced);

  private:
    int read(uint8_t *p, size_t n)
    { // readSliceAll
        if (len_ - pos_ < n) {
            pos_ = len_;
            return ZPX_E_END_OF_STREAM;
        }
        memcpy(p, src_ + pos_, n);
        pos_ += n;
        return 0;
    }
    int read_crc(uint8_t *p, size_t n)
    {
        if (int e = read(p, n)) return e;
        crc_ = crc32_fast(crc_, p, n);
        return 0;
    }
    int verify()
    {
        uint8_t b[4];
        if (int e = read(b, 4)) return e;
        return be32(b) == crc_ ? 0 : ZPX_E_INVALID_CHECKSUM;
    }
    int skip(uint32_t n)
    {
        if (len_ - pos_ < n) {
            pos_ = len_;
            return ZPX_E_END_OF_STREAM;
        }
        crc_ = crc32_fast(crc_, src_ + pos_, n);
        pos_ += n;
        return 0;
    }
    int chunk();
    int ihdr(uint32_t len);
    int plte(uint32_t len);
    int trns(uint32_t len);
    int idat(uint32_t first_len);
    int prepare_image();
    int inflate_image(bool fast_done, bool fast_ok, size_t fast_produced);

    const uint8_t *src_;
    size_t len_, pos_ = 0;
    uint32_t crc_ = 0;
    int stage_ = 0; // start, ihdr, plte, trns, idat, iend
    bool have_image_ = false;
    PngStream &o_;
    int threads_ = 1; // inflate threads (inflate_parallel)
    std::vector<uint8_t> z_; // the concatenated IDAT data (the zlib stream)
    bool defer_ = false, pending_ = false;
};

int Parser::ihdr(uint32_t len)
{
    if (len != 13) return ZPX_E_INVALID_IHDR_LENGTH;
    uint8_t b[13];
    if (int e = read_crc(b, 13)) return e;
    if (b[10] != 0) return ZPX_E_UNSUPPORTED_COMPRESSION_METHOD;
    if (b[11] != 0) return ZPX_E_UNSUPPORTED_FILTER_METHOD;
    if (b[12] > 1) return ZPX_E_UNSUPPORTED_INTERLACE_METHOD;
    o_.interlace = b[12];
    const uint32_t w = be32(b), h = be32(b + 4);
    if (w == 0 || h == 0) return ZPX_E_INVALID_DIMENSION;
    const uint64_t np = uint64_t(w) * h;
    if (np >> 32) return ZPX_E_DIMENSION_OVERFLOW;
    if (uint32_t(np) != uint32_t(uint32_t(np) * 8u) / 8u) return ZPX_E_DIMENSION_OVERFLOW;
    const uint8_t depth = b[8], ct = b[9];
    if (ct != 0 && ct != 2 && ct != 3 && ct != 4 && ct != 6) return ZPX_E_INVALID_COLOR_TYPE;
    o_.width = w;
    o_.height = h;
    int d = 0;
    switch (depth) {
    case 1: d = ct == 0 ? ZPX_PNG_G1 : ct == 3 ? ZPX_PNG_P1 : 0; break;
    case 2: d = ct == 0 ? ZPX_PNG_G2 : ct == 3 ? ZPX_PNG_P2 : 0; break;
    case 4: d = ct == 0 ? ZPX_PNG_G4 : ct == 3 ? ZPX_PNG_P4 : 0; break;
    case 8:
        d = ct == 0 ? ZPX_PNG_G8 : ct == 2 ? ZPX_PNG_TC8 : ct == 3 ? ZPX_PNG_P8 : ct == 4 ? ZPX_PNG_GA8 : ZPX_PNG_TCA8;
        break;
    case 16:
        d = ct == 0 ? ZPX_PNG_G16 : ct == 2 ? ZPX_PNG_TC16 : ct == 4 ? ZPX_PNG_GA16 : ct == 6 ? ZPX_PNG_TCA16 : 0;
        break;
    default: return ZPX_E_UNSUPPORTED_BIT_DEPTH;
    }
    if (d == 0) return ZPX_E_INVALID_COLOR_TYPE_DEPTH_COMBO;
    o_.depth = d;
    return verify();
}

int Parser::plte(uint32_t len)
{
    const uint32_t n = len / 3;
    // the reference checks against 1 << IHDR bit depth
    uint32_t ihdr_depth = 8;
    switch (o_.depth) {
    case ZPX_PNG_G1: case ZPX_PNG_P1: ihdr_depth = 1; break;
    case ZPX_PNG_G2: case ZPX_PNG_P2: ihdr_depth = 2; break;
    case ZPX_PNG_G4: case ZPX_PNG_P4: ihdr_depth = 4; break;
    case ZPX_PNG_G16: case ZPX_PNG_GA16: case ZPX_PNG_TC16: case ZPX_PNG_TCA16: ihdr_depth = 16; break;
    default: break;
    }
    if (len % 3 != 0 || n == 0 || n > 256 || n > (1u << ihdr_depth)) return ZPX_E_BAD_PLTE_LENGTH;
    uint8_t b[768];
    if (int e = read_crc(b, n * 3)) return e;
    if (paletted(o_.depth)) {
        for (int i = 0; i < 256; i++) o_.palette[i] = zpx_color{0, 0, 0, 0xff, 0, {0, 0, 0}};
        for (uint32_t i = 0; i < n; i++) o_.palette[i] = zpx_color{b[3 * i], b[3 * i + 1], b[3 * i + 2], 0xff, 0, {0, 0, 0}};
        o_.palette_len = static_cast<int>(n);
        o_.has_palette = true;
    } else if (o_.depth != ZPX_PNG_TC8 && o_.depth != ZPX_PNG_TCA8 && o_.depth != ZPX_PNG_TC16 &&
               o_.depth != ZPX_PNG_TCA16) {
        return ZPX_E_PLTE_COLOR_TYPE_MISMATCH;
    }
    return verify();
}

int Parser::trns(uint32_t len)
{
    uint8_t b[256];
    switch (o_.depth) {
    case ZPX_PNG_G1: case ZPX_PNG_G2: case ZPX_PNG_G4: case ZPX_PNG_G8: case ZPX_PNG_G16: {
        if (len != 2) return ZPX_E_BAD_TRNS_LENGTH;
        if (int e = read_crc(b, 2)) return e;
        o_.transparent[0] = b[0];
        const uint32_t mul = o_.depth == ZPX_PNG_G1 ? 0xff : o_.depth == ZPX_PNG_G2 ? 0x55 : o_.depth == ZPX_PNG_G4 ? 0x11 : 1;
        o_.transparent[1] = static_cast<uint8_t>(b[1] * mul);
        o_.use_transparent = true;
        break;
    }
    case ZPX_PNG_TC8: case ZPX_PNG_TC16:
        if (len != 6) return ZPX_E_BAD_TRNS_LENGTH;
        if (int e = read_crc(b, 6)) return e;
        memcpy(o_.transparent, b, 6);
        o_.use_transparent = true;
        break;
    case ZPX_PNG_P1: case ZPX_PNG_P2: case ZPX_PNG_P4: case ZPX_PNG_P8:
        if (len > 256) return ZPX_E_BAD_TRNS_LENGTH;
        if (int e = read_crc(b, len)) return e;
        if (o_.palette_len < static_cast<int>(len)) o_.palette_len = static_cast<int>(len);
        for (uint32_t i = 0; i < len; i++) {
            o_.palette[i].a = b[i];
            o_.palette[i].model = 1; // .nrgba
        }
        break;
    default:
        return ZPX_E_TRNS_COLOR_TYPE_MISMATCH;
    }
    return verify();
}

// The passes' geometry and the inflated stream's buffer (readImagePass
// :655-673, :782-785).
int Parser::prepare_image()
{
    const uint32_t bits = static_cast<uint32_t>(bits_of(o_.depth));
    o_.npasses = 0;
    size_t total = 0;
    const int np = o_.interlace ? 7 : 1;
    for (int p = 0; p < np; p++) {
        PngPassInfo &pi = o_.pass[p];
        pi = PngPassInfo{};
        if (o_.interlace) {
            const uint32_t xo = kAdam7[p][0], yo = kAdam7[p][1], xf = kAdam7[p][2], yf = kAdam7[p][3];
            pi.width = ((o_.width > xo ? o_.width - xo : 0) + xf - 1) / xf;
            pi.rows = ((o_.height > yo ? o_.height - yo : 0) + yf - 1) / yf;
            pi.xo = xo;
            pi.yo = yo;
            pi.xf = xf;
            pi.yf = yf;
            if (pi.width == 0 || pi.rows == 0) {
                pi.width = pi.rows = 0; // EmptyPass
                continue;
            }
        } else {
            pi.width = o_.width;
            pi.rows = o_.height;
        }
        pi.row_bytes = static_cast<uint32_t>((uint64_t(bits) * pi.width + 7) / 8);
        pi.offset = total;
        total += size_t(pi.rows) * (size_t(pi.row_bytes) + 1);
        o_.npasses = p + 1;
    }
    o_.data_len = total;
    if (!o_.data.alloc(total + ZPX_PNG_INPUT_PAD, false)) return ZPX_E_OUT_OF_MEMORY;
    memset(static_cast<uint8_t *>(o_.data.ptr) + total, 0, ZPX_PNG_INPUT_PAD);
    return 0;
}

// Inflates exactly the bytes the passes read (std.compress.flate .zlib) --
// the fast decoder when the stream decodes cleanly (or its result, when the
// caller ran it: fast_done), else system zlib from the start, whose error
// behaviour the rest maps -- then the rows' checks and the output type.
int Parser::inflate_image(bool fast_done, bool fast_ok, size_t fast_produced)
{
    const size_t total = o_.data_len;
    uint8_t *dst = static_cast<uint8_t *>(o_.data.ptr);
    size_t produced = 0;
    bool data_error = false;
    bool ok;
    if (fast_done) {
        ok = fast_ok;
        produced = fast_produced;
    } else {
        // several threads for a large stream (speculative chunks, identical
        // bytes), else / on anything irregular the serial fast decoder
        ok = threads_ > 1 && total >= (size_t(4) << 20) &&
             inflate_parallel(z_.data(), z_.size(), dst, total, &produced, threads_);
        if (!ok) ok = inflate_fast(z_.data(), z_.size(), dst, total, &produced);
    }
    if (!ok) {
        produced = 0;
        if (int e = inflate_zlib(z_, dst, total, produced, data_error)) return e;
    }
    // rows in order: short data -> EndOfStream / ReadFailed, bad filter ->
    // InvalidFilterType (readImagePass :800, :839-841)
    for (int p = 0; p < o_.npasses; p++) {
        const PngPassInfo &pi = o_.pass[p];
        for (uint32_t y = 0; y < pi.rows; y++) {
            const size_t off = pi.offset + size_t(y) * (size_t(pi.row_bytes) + 1);
            if (off + pi.row_bytes + 1 > produced) return data_error ? ZPX_E_READ_FAILED : ZPX_E_END_OF_STREAM;
            if (dst[off] > 4) return ZPX_E_INVALID_FILTER_TYPE;
        }
    }
    // output image type (:712-775)
    const bool t = o_.use_transparent;
    switch (o_.depth) {
    case ZPX_PNG_G1: case ZPX_PNG_G2: case ZPX_PNG_G4: case ZPX_PNG_G8:
        o_.kind = t ? ZPX_NRGBA : ZPX_GRAY; o_.out_bpp = t ? 4 : 1; break;
    case ZPX_PNG_GA8: o_.kind = ZPX_NRGBA; o_.out_bpp = 4; break;
    case ZPX_PNG_GA16: o_.kind = ZPX_NRGBA64; o_.out_bpp = 8; break;
    case ZPX_PNG_G16: o_.kind = t ? ZPX_NRGBA64 : ZPX_GRAY16; o_.out_bpp = t ? 8 : 2; break;
    case ZPX_PNG_TC8: o_.kind = t ? ZPX_NRGBA : ZPX_RGBA; o_.out_bpp = 4; break;
    case ZPX_PNG_TC16: o_.kind = t ? ZPX_NRGBA64 : ZPX_RGBA64; o_.out_bpp = 8; break;
    case ZPX_PNG_TCA8: o_.kind = ZPX_NRGBA; o_.out_bpp = 4; break;
    case ZPX_PNG_TCA16: o_.kind = ZPX_NRGBA64; o_.out_bpp = 8; break;
    default:
        o_.kind = ZPX_PALETTED;
        o_.out_bpp = 1;
        if (!o_.has_palette) return ZPX_E_PANIC; // self.palette.? on null
        break;
    }
    have_image_ = true;
    return 0;
}

int Parser::idat(uint32_t first_len)
{ // parseIdat :404-545
    if (pending_) { // a second IDAT run (deferred): the first one's image is checked first, as undeferred
        pending_ = false;
        if (int e = inflate_image(false, false, 0)) return e;
    }
    std::vector<uint8_t> &all = z_;
    if (all.capacity() == 0) all = zpool().take();
    all.clear();
    { // reserve the whole stream once: sum the run of IDAT chunk lengths
      // ahead (a read-only scan; the loop below does the checks)
        size_t total = first_len, p = pos_ + size_t(first_len) + 4;
        while (p + 8 <= len_ && memcmp(src_ + p + 4, "IDAT", 4) == 0) {
            const uint32_t n = be32(src_ + p);
            total += n;
            p += size_t(n) + 12;
        }
        // the lengths are untrusted: never reserve more than the input holds
        all.reserve(std::min(total, len_ - pos_));
    }
    auto take = [&](uint32_t n) -> int {
        if (len_ - pos_ < n) {
            pos_ = len_;
            return ZPX_E_END_OF_STREAM;
        }
        crc_ = crc32_fast(crc_, src_ + pos_, n);
        all.insert(all.end(), src_ + pos_, src_ + pos_ + n);
        pos_ += n;
        return 0;
    };
    if (int e = take(first_len)) return e;
    if (int e = verify()) return e;
    for (;;) {
        uint8_t hb[8];
        if (read(hb, 8)) break; // :435-438
        if (memcmp(hb + 4, "IDAT", 4) != 0) {
            stage_ = 4;
            crc_ = static_cast<uint32_t>(crc32(0, hb + 4, 4));
            if (memcmp(hb + 4, "IEND", 4) == 0) {
                stage_ = 5;
                if (int e = verify()) return e;
            } else {
                if (int e = skip(be32(hb))) return e;
                if (int e = verify()) return e;
            }
            break;
        }
        crc_ = static_cast<uint32_t>(crc32(0, hb + 4, 4));
        if (int e = take(be32(hb))) return e;
        if (int e = verify()) return e;
    }
    if (all.empty()) return ZPX_E_EMPTY_IDAT_DATA;
    if (int e = prepare_image()) return e;
    if (defer_) {
        pending_ = true;
        return 0;
    }
    return inflate_image(false, false, 0);
}

int Parser::complete(int run_status, bool ok, size_t produced)
{
    if (!pending_) return run_status; // stopped before its image (or no job)
    pending_ = false;
    const int e = inflate_image(true, ok, produced);
    return e ? e : run_status;
}

int Parser::chunk()
{ // parseChunk :231-324
    uint8_t hb[8];
    if (int e = read(hb, 8)) return e;
    const uint32_t len = be32(hb);
    const uint8_t *t = hb + 4;
    crc_ = static_cast<uint32_t>(crc32(0, t, 4));
    if (!memcmp(t, "IHDR", 4)) {
        if (stage_ != 0) return ZPX_E_CHUNK_ORDER_IN_HEADER_ERROR;
        stage_ = 1;
        return ihdr(len);
    }
    if (!memcmp(t, "PLTE", 4)) {
        if (stage_ != 1) return ZPX_E_CHUNK_ORDER_PLTE_ERROR;
        stage_ = 2;
        return plte(len);
    }
    if (!memcmp(t, "IDAT", 4)) {
        if (stage_ < 1 || stage_ > 4 || (stage_ == 1 && paletted(o_.depth))) return ZPX_E_CHUNK_ORDER_IDAT_ERROR;
        stage_ = 4;
        return idat(len);
    }
    if (!memcmp(t, "tRNS", 4)) {
        if (paletted(o_.depth)) {
            if (stage_ != 2) return ZPX_E_CHUNK_ORDER_TRNS1_ERROR;
        } else if (o_.depth == ZPX_PNG_TC8 || o_.depth == ZPX_PNG_TC16) {
            if (stage_ != 1 && stage_ != 2) return ZPX_E_CHUNK_ORDER_TRNS2_ERROR;
        } else if (stage_ != 1) {
            return ZPX_E_CHUNK_ORDER_TRNS3_ERROR;
        }
        stage_ = 3;
        return trns(len);
    }
    if (!memcmp(t, "IEND", 4)) {
        if (stage_ != 4) return ZPX_E_CHUNK_ORDER_IEND_ERROR;
        stage_ = 5;
        return verify();
    }
    if (int e = skip(len)) return e;
    return verify();
}

int Parser::run(bool header_only)
{
    static const uint8_t kSig[8] = {0x89, 'P', 'N', 'G', '\r', '\n', 0x1a, '\n'};
    uint8_t sig[8];
    if (int e = read(sig, 8)) return e;
    if (memcmp(sig, kSig, 8) != 0) return ZPX_E_INVALID_PNG_HEADER;
    if (header_only) { // first chunk must be IHDR (parseChunk's stage check)
        if (int e = chunk()) return e;
        return stage_ == 1 ? 0 : ZPX_E_CHUNK_ORDER_IN_HEADER_ERROR;
    }
    while (stage_ != 5)
        if (int e = chunk()) return e;
    if (!have_image_ && !pending_) return ZPX_E_INVALID_IMAGE_DIMENSIONS;
    return 0;
}

} // namespace

size_t png_pool_trim() { return zpool().trim() + inflate_pool_trim(); }

int png_inflate_threads()
{
    static const int n = [] {
        if (const char *e = getenv("ZPX_INFLATE_THREADS")) return std::max(1, atoi(e));
        return std::min(8, host_cpu_budget());
    }();
    return n;
}

int png_parse(const uint8_t *buf, size_t len, PngStream &out, int threads)
{
    try { // no exception crosses the ABI (std::bad_alloc on a huge stream)
        Parser p(buf, len, out, threads);
        return p.run();
    } catch (...) {
        return ZPX_E_OUT_OF_MEMORY;
    }
}

int png_parse_pair(const uint8_t *const buf[2], const size_t len[2], PngStream *const out[2], int status[2])
{
    try {
        Parser a(buf[0], len[0], *out[0], 1), b(buf[1], len[1], *out[1], 1);
        Parser *p[2] = {&a, &b};
        int run[2];
        for (int k = 0; k < 2; k++) {
            p[k]->defer();
            run[k] = p[k]->run();
        }
        bool ok[2] = {false, false};
        size_t produced[2] = {0, 0};
        if (a.pending() && b.pending()) {
            const uint8_t *in[2] = {a.job_z().data(), b.job_z().data()};
            const size_t in_len[2] = {a.job_z().size(), b.job_z().size()};
            uint8_t *dst[2] = {a.job_dst(), b.job_dst()};
            const size_t want[2] = {a.job_want(), b.job_want()};
            inflate_fast_pair(in, in_len, dst, want, produced, ok);
        } else {
            for (int k = 0; k < 2; k++)
                if (p[k]->pending())
                    ok[k] = inflate_fast(p[k]->job_z().data(), p[k]->job_z().size(), p[k]->job_dst(), p[k]->job_want(),
                                         &produced[k]);
        }
        for (int k = 0; k < 2; k++) status[k] = p[k]->complete(run[k], ok[k], produced[k]);
        return 0;
    } catch (...) {
        status[0] = status[1] = ZPX_E_OUT_OF_MEMORY;
        return ZPX_E_OUT_OF_MEMORY;
    }
}

int png_decode_config(const uint8_t *buf, size_t len, uint32_t &w, uint32_t &h)
{
    PngStream s;
    Parser p(buf, len, s, 1);
    if (int e = p.run(true)) return e;
    w = s.width;
    h = s.height;
    return 0;
}

} // namespace zpx
