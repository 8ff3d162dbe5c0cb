/*
 * zpix_oracle.c — plain-C restatement of braheezy/zpix's JPEG/PNG decode
 * arithmetic (reference snapshot 2025-11-14, Zig 0.15.1).
 *
 * TEST INFRASTRUCTURE ONLY: the parity checker for zpix_amd.  Nothing in the
 * product library links or calls this file.  Every function cites the
 * reference file:line it restates.  Arithmetic is i32 with wrap-around
 * (compiled with -fwrapv), which is the Go semantics the Zig code was
 * translated from; for conforming streams no intermediate overflows, so this
 * equals the Zig result wherever the Zig result is defined.
 *
 * Deliberate deviations (documented in DESIGN.md §Oracle):
 *   - places where the reference hits a safety panic or reads undefined
 *     memory (decoder.zig:450, :1581, :1606, :1752; out-of-range palette
 *     indices png/decoder.zig:1086-1129) return an error code or follow the
 *     Go behaviour the translation came from, instead of crashing;
 *   - the 4-component YCbCrK branch (decoder.zig:811-846, which goes through
 *     the off-by-one image/util.zig drawYCbCr) is reported as Unsupported.
 */
#define _POSIX_C_SOURCE 200809L
#include "zpix_oracle.h"

#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <zlib.h>

/* CPU-baseline stage clock (bench.py cpu_baseline): seconds this thread
 * spent in PNG filter reconstruction + pixel store (readImagePass and
 * mergePassInto), so the caller can split png.decode into inflate+parse vs
 * unfilter+store.  Timing only; no decode result depends on it. */
static __thread double zo_png_unfilter_s;
static double zo_now(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}
double zo_png_unfilter_seconds(void)
{
    double t = zo_png_unfilter_s;
    zo_png_unfilter_s = 0;
    return t;
}

/* ------------------------------------------------------------------------ */
/* Error names: the Zig error-set names the path can raise.                 */
/* ------------------------------------------------------------------------ */
#define ZO_ERRORS(X)                                                           \
    X(Ok)                                                                      \
    X(UnexpectedEof)                                                           \
    X(InvalidSOIMarker)                                                        \
    X(ShortSegmentLength)                                                      \
    X(UnknownMarker)                                                           \
    X(UnsupportedMarker)                                                       \
    X(MultipleSofMarkers)                                                      \
    X(NumberComponents)                                                        \
    X(Precision)                                                               \
    X(SofWrongLength)                                                          \
    X(RepeatedComponentIdentifier)                                             \
    X(BadTqValue)                                                              \
    X(LumaChromaSubSamplingRatio)                                              \
    X(DriWrongLength)                                                          \
    X(BadPqValue)                                                              \
    X(DqtWrongLength)                                                          \
    X(MissingFF00)                                                             \
    X(UninitializedHuffmanTable)                                               \
    X(BadHuffmanCode)                                                          \
    X(DhtWrongLength)                                                          \
    X(BadTcValue)                                                              \
    X(BadThValue)                                                              \
    X(HuffZeroLength)                                                          \
    X(HuffTooLong)                                                             \
    X(MissingSosMarker)                                                        \
    X(SosWrongLength)                                                          \
    X(UnknownComponentSelector)                                                \
    X(BadTdValue)                                                              \
    X(BadTaValue)                                                              \
    X(SamplingFactorsTooLarge)                                                 \
    X(BadSpectralSelection)                                                    \
    X(ProgressiveACCoefficientsForMoreThanOneComponent)                        \
    X(BadSuccessiveApproximation)                                              \
    X(ExcessiveDCComponent)                                                    \
    X(UnexpectedHuffmanCode)                                                   \
    X(TooManyCoefficients)                                                     \
    X(BadRSTMarker)                                                            \
    X(UnsupportedComponent)                                                    \
    X(UnsupportedColorModel)                                                   \
    X(InvalidPngHeader)                                                        \
    X(ChunkOrderInHeaderError)                                                 \
    X(ChunkOrderPlteError)                                                     \
    X(ChunkOrderIdatError)                                                     \
    X(ChunkOrderTrns1Error)                                                    \
    X(ChunkOrderTrns2Error)                                                    \
    X(ChunkOrderTrns3Error)                                                    \
    X(ChunkOrderIendError)                                                     \
    X(InvalidIHDRLength)                                                       \
    X(UnsupportedCompressionMethod)                                            \
    X(UnsupportedFilterMethod)                                                 \
    X(UnsupportedInterlaceMethod)                                              \
    X(InvalidDimension)                                                        \
    X(DimensionOverflow)                                                       \
    X(InvalidColorType)                                                        \
    X(InvalidColorTypeDepthCombo)                                              \
    X(UnsupportedBitDepth)                                                     \
    X(EmptyIdatData)                                                           \
    X(BadTrnsLength)                                                           \
    X(TrnsColorTypeMismatch)                                                   \
    X(BadPlteLength)                                                           \
    X(PlteColorTypeMismatch)                                                   \
    X(InvalidFilterType)                                                       \
    X(InvalidChecksum)                                                         \
    X(EndOfStream)                                                             \
    X(ReadFailed)                                                              \
    X(InvalidImageDimensions)                                                  \
    X(OutOfMemory)                                                             \
    X(Unsupported)                                                             \
    X(Panic)                                                                   \
    X(InvalidSignature)                                                        \
    X(UnsupportedHeader)                                                       \
    X(UnsupportedDimensions)                                                   \
    X(UnsupportedCompression)                                                  \
    X(UnsupportedBPP)                                                          \
    X(UnsupportedPaletteSize)                                                  \
    X(UnsupportedColorOffset)                                                  \
    X(InvalidQoiData)                                                          \
    X(InvalidQoiHeader)

enum zo_err {
#define X(n) E_##n,
    ZO_ERRORS(X)
#undef X
    E__COUNT
};

static const char *const zo_err_names[] = {
#define X(n) #n,
    ZO_ERRORS(X)
#undef X
};

const char *zo_error_name(int code)
{
    if (code < 0 || code >= E__COUNT) return "Unknown";
    return zo_err_names[code];
}

#define TRY(expr)                                                              \
    do {                                                                       \
        int _e = (expr);                                                       \
        if (_e) return _e;                                                     \
    } while (0)

/* ======================================================================== */
/* JPEG                                                                      */
/* ======================================================================== */

/* unzig, src/jpeg/decoder.zig:73-82 */
static const uint8_t UNZIG[64] = {
    0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,
    12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6,  7,  14, 21, 28,
    35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51,
    58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63,
};

/* idct.zig:50-65 */
enum { W1 = 2841, W2 = 2676, W3 = 2408, W5 = 1609, W6 = 1108, W7 = 565 };
enum { W1PW7 = W1 + W7, W1MW7 = W1 - W7, W2PW6 = W2 + W6, W2MW6 = W2 - W6,
       W3PW5 = W3 + W5, W3MW5 = W3 - W5, R2 = 181 };

/* idct.transform, src/jpeg/idct.zig:77-201 */
void zo_idct(int32_t *src)
{
    /* horizontal pass, :79-145 */
    for (int y = 0; y < 8; y++) {
        int32_t *s = src + 8 * y;
        if (s[1] == 0 && s[2] == 0 && s[3] == 0 && s[4] == 0 && s[5] == 0 &&
            s[6] == 0 && s[7] == 0) {
            int32_t dc = s[0] << 3; /* :84-97 */
            for (int i = 0; i < 8; i++) s[i] = dc;
            continue;
        }
        int32_t x0 = (s[0] << 11) + 128, x1 = s[4] << 11, x2 = s[6], x3 = s[2];
        int32_t x4 = s[1], x5 = s[7], x6 = s[5], x7 = s[3], x8;
        x8 = W7 * (x4 + x5);
        x4 = x8 + W1MW7 * x4;
        x5 = x8 - W1PW7 * x5;
        x8 = W3 * (x6 + x7);
        x6 = x8 - W3MW5 * x6;
        x7 = x8 - W3PW5 * x7;
        x8 = x0 + x1;
        x0 -= x1;
        x1 = W6 * (x3 + x2);
        x2 = x1 - W2PW6 * x2;
        x3 = x1 + W2MW6 * x3;
        x1 = x4 + x6;
        x4 -= x6;
        x6 = x5 + x7;
        x5 -= x7;
        x7 = x8 + x3;
        x8 -= x3;
        x3 = x0 + x2;
        x0 -= x2;
        x2 = (R2 * (x4 + x5) + 128) >> 8;
        x4 = (R2 * (x4 - x5) + 128) >> 8;
        s[0] = (x7 + x1) >> 8;
        s[1] = (x3 + x2) >> 8;
        s[2] = (x0 + x4) >> 8;
        s[3] = (x8 + x6) >> 8;
        s[4] = (x8 - x6) >> 8;
        s[5] = (x0 - x4) >> 8;
        s[6] = (x3 - x2) >> 8;
        s[7] = (x7 - x1) >> 8;
    }
    /* vertical pass, :148-200 */
    for (int x = 0; x < 8; x++) {
        int32_t *s = src + x;
        int32_t y0 = (s[0] << 8) + 8192, y1 = s[32] << 8, y2 = s[48], y3 = s[16];
        int32_t y4 = s[8], y5 = s[56], y6 = s[40], y7 = s[24], y8;
        y8 = W7 * (y4 + y5) + 4;
        y4 = (y8 + W1MW7 * y4) >> 3;
        y5 = (y8 - W1PW7 * y5) >> 3;
        y8 = W3 * (y6 + y7) + 4;
        y6 = (y8 - W3MW5 * y6) >> 3;
        y7 = (y8 - W3PW5 * y7) >> 3;
        y8 = y0 + y1;
        y0 -= y1;
        y1 = W6 * (y3 + y2) + 4;
        y2 = (y1 - W2PW6 * y2) >> 3;
        y3 = (y1 + W2MW6 * y3) >> 3;
        y1 = y4 + y6;
        y4 -= y6;
        y6 = y5 + y7;
        y5 -= y7;
        y7 = y8 + y3;
        y8 -= y3;
        y3 = y0 + y2;
        y0 -= y2;
        y2 = (R2 * (y4 + y5) + 128) >> 8;
        y4 = (R2 * (y4 - y5) + 128) >> 8;
        s[0] = (y7 + y1) >> 14;
        s[8] = (y3 + y2) >> 14;
        s[16] = (y0 + y4) >> 14;
        s[24] = (y8 + y6) >> 14;
        s[32] = (y8 - y6) >> 14;
        s[40] = (y0 - y4) >> 14;
        s[48] = (y3 - y2) >> 14;
        s[56] = (y7 - y1) >> 14;
    }
}

/* HuffTable, src/jpeg/HuffTable.zig:1-32 */
typedef struct {
    int32_t num_codes;
    uint16_t lut[256];
    uint8_t vals[256];
    int32_t min_codes[16], max_codes[16], vals_indices[16];
} zo_huff;

typedef struct {
    int32_t h, v;
    uint8_t id, tq;
} zo_comp;

/* Decoder state, src/jpeg/decoder.zig:85-153 */
typedef struct {
    /* underlying std.Io.Reader.fixed(buffer) */
    const uint8_t *src;
    size_t src_len, src_pos;
    /* bytes, :107-116 */
    uint8_t buf[4096];
    size_t bi, bj, num_unreadable;
    /* bits, :90-97 */
    uint32_t ba, bm;
    int32_t bn;

    uint32_t width, height;
    /* destination */
    int have_gray, have_ycbcr;
    uint8_t *gray_pixels; /* 8*mxx x 8*myy, stride 8*mxx */
    size_t gray_stride;
    uint8_t *ycbcr_pixels; /* padded planes, see makeImg */
    size_t ycbcr_len, y_stride, c_stride, cb_off, cr_off;
    int32_t subsample;
    uint8_t *black_pixels;
    size_t black_stride;

    uint16_t restart_interval;
    uint8_t num_components;
    int baseline, progressive, jfif, adobe_transform_valid;
    int adobe_transform; /* 0 unknown, 1 ycbcr, 2 ycbcrk */
    uint16_t eob_run;
    zo_comp comp[4];
    int32_t *prog[4]; /* blocks of 64 */
    zo_huff huff[2][4];
    int32_t quant[4][64];
    uint8_t tmp[128];
    int coeffs_only; /* accumulate coefficients instead of reconstructing */
    int32_t mxx, myy;
} zo_jdec;

/* fill, decoder.zig:447-472 (reading through readSliceShort of a fixed reader) */
static int jd_fill(zo_jdec *d)
{
    if (d->bi != d->bj) return E_Panic; /* :449-451 */
    if (d->bj > 2) {
        d->buf[0] = d->buf[d->bj - 2];
        d->buf[1] = d->buf[d->bj - 1];
        d->bi = 2;
        d->bj = 2;
    } else {
        d->bi = 0;
        d->bj = 0;
    }
    size_t room = sizeof(d->buf) - d->bj;
    size_t avail = d->src_len - d->src_pos;
    size_t n = avail < room ? avail : room;
    memcpy(d->buf + d->bj, d->src + d->src_pos, n);
    d->src_pos += n;
    d->bj += n;
    if (n == 0) return E_UnexpectedEof;
    return 0;
}

/* unreadByteStuffedByte, :479-487 */
static void jd_unread_stuffed(zo_jdec *d)
{
    d->bi -= d->num_unreadable;
    d->num_unreadable = 0;
    if (d->bn >= 8) {
        d->ba >>= 8;
        d->bn -= 8;
        d->bm >>= 8;
    }
}

/* readByte, :402-410 */
static int jd_read_byte(zo_jdec *d, uint8_t *x)
{
    while (d->bi == d->bj) TRY(jd_fill(d));
    *x = d->buf[d->bi++];
    d->num_unreadable = 0;
    return 0;
}

/* readFull, :414-443 */
static int jd_read_full(zo_jdec *d, uint8_t *p, size_t len)
{
    size_t off = 0;
    if (d->num_unreadable > 0) {
        if (d->bn >= 8) jd_unread_stuffed(d);
        d->num_unreadable = 0;
    }
    while (off < len) {
        size_t avail = d->bj - d->bi;
        size_t c = avail < len - off ? avail : len - off;
        memcpy(p + off, d->buf + d->bi, c);
        d->bi += c;
        off += c;
        if (off == len) break;
        TRY(jd_fill(d));
    }
    return 0;
}

/* ignore, :376-398 */
static int jd_ignore(zo_jdec *d, int32_t n)
{
    if (d->num_unreadable > 0) {
        if (d->bn >= 8) jd_unread_stuffed(d);
        d->num_unreadable = 0;
    }
    for (;;) {
        size_t rem = d->bj - d->bi;
        if (rem > (size_t)n) rem = (size_t)n;
        d->bi += rem;
        n -= (int32_t)rem;
        if (n == 0) break;
        TRY(jd_fill(d));
    }
    return 0;
}

/* readByteStuffedByte, :712-749 */
static int jd_read_stuffed(zo_jdec *d, uint8_t *out)
{
    if (d->bi + 2 <= d->bj) {
        uint8_t x = d->buf[d->bi++];
        d->num_unreadable = 1;
        if (x != 0xff) {
            *out = x;
            return 0;
        }
        if (d->buf[d->bi] != 0x00) return E_MissingFF00;
        d->bi++;
        d->num_unreadable = 2;
        *out = 0xff;
        return 0;
    }
    d->num_unreadable = 0;
    uint8_t x;
    TRY(jd_read_byte(d, &x));
    d->num_unreadable = 1;
    if (x != 0xff) {
        *out = x;
        return 0;
    }
    TRY(jd_read_byte(d, &x));
    d->num_unreadable = 2;
    if (x != 0x00) return E_MissingFF00;
    *out = 0xff;
    return 0;
}

/* ensureNBits, :975-991 */
static int jd_ensure(zo_jdec *d, int32_t n)
{
    for (;;) {
        uint8_t c;
        TRY(jd_read_stuffed(d, &c));
        d->ba = (d->ba << 8) | c;
        d->bn += 8;
        if (d->bm == 0) d->bm = 1u << 7;
        else d->bm <<= 8;
        if (d->bn >= n) break;
    }
    return 0;
}

/* decodeHuffman, :909-970 */
static int jd_decode_huffman(zo_jdec *d, zo_huff *h, uint8_t *out)
{
    if (h->num_codes == 0) return E_UninitializedHuffmanTable;
    int slow = 0;
    if (d->bn < 8) {
        int e = jd_ensure(d, 8);
        if (e) {
            /* only MissingFF00 / ShortHuffmanData fall through (:917) */
            if (e != E_MissingFF00) return e;
            if (d->num_unreadable != 0) jd_unread_stuffed(d);
            slow = 1;
        }
    }
    if (!slow) {
        uint16_t lv = h->lut[(d->ba >> (d->bn - 8)) & 0xff];
        if (lv != 0) {
            int32_t nb = (int32_t)(lv & 0xff) - 1;
            d->bn -= nb;
            d->bm >>= nb;
            *out = (uint8_t)(lv >> 8);
            return 0;
        }
    }
    int32_t code = 0;
    for (int i = 0; i < 16; i++) {
        if (d->bn == 0) TRY(jd_ensure(d, 1));
        if (d->ba & d->bm) code |= 1;
        d->bn -= 1;
        d->bm >>= 1;
        if (code <= h->max_codes[i]) {
            int32_t idx = h->vals_indices[i] + code - h->min_codes[i];
            if (idx < 0 || idx > 255) return E_Panic;
            *out = h->vals[idx];
            return 0;
        }
        code <<= 1;
    }
    return E_BadHuffmanCode;
}

/* decodeBit, :994-1006 */
static int jd_decode_bit(zo_jdec *d, int *bit)
{
    if (d->bn == 0) TRY(jd_ensure(d, 1));
    *bit = (d->ba & d->bm) != 0;
    d->bn -= 1;
    d->bm >>= 1;
    return 0;
}

/* decodeBits, :1009-1022 */
static int jd_decode_bits(zo_jdec *d, int32_t n, uint32_t *out)
{
    if (d->bn < n) TRY(jd_ensure(d, n));
    uint32_t r = d->ba >> (d->bn - n);
    r &= (n >= 32) ? 0xffffffffu : ((1u << n) - 1);
    d->bn -= n;
    d->bm >>= n;
    *out = r;
    return 0;
}

/* receiveExtend, :1115-1134 */
static int jd_receive_extend(zo_jdec *d, uint8_t t, int32_t *out)
{
    if (d->bn < (int32_t)t) TRY(jd_ensure(d, t));
    d->bn -= t;
    d->bm >>= t;
    int32_t thr = (int32_t)1 << t;
    int32_t v = (int32_t)((d->ba >> d->bn) & (uint32_t)(thr - 1));
    if (v < (thr >> 1)) v += (int32_t)((uint32_t)-1 << t) + 1;
    *out = v;
    return 0;
}

/* processSof, :490-618 */
static int jd_process_sof(zo_jdec *d, int32_t n)
{
    if (d->num_components != 0) return E_MultipleSofMarkers;
    switch (n) {
    case 6 + 3 * 1: d->num_components = 1; break;
    case 6 + 3 * 3: d->num_components = 3; break;
    case 6 + 3 * 4: d->num_components = 4; break;
    default: return E_NumberComponents;
    }
    TRY(jd_read_full(d, d->tmp, (size_t)n));
    if (d->tmp[0] != 8) return E_Precision;
    d->height = ((uint32_t)d->tmp[1] << 8) + d->tmp[2];
    d->width = ((uint32_t)d->tmp[3] << 8) + d->tmp[4];
    if (d->tmp[5] != d->num_components) return E_SofWrongLength;
    for (int i = 0; i < d->num_components; i++) {
        d->comp[i].id = d->tmp[6 + 3 * i];
        for (int j = 0; j < i; j++)
            if (d->comp[i].id == d->comp[j].id) return E_RepeatedComponentIdentifier;
        d->comp[i].tq = d->tmp[8 + 3 * i];
        if (d->comp[i].tq > 3) return E_BadTqValue;
        uint8_t hv = d->tmp[7 + 3 * i];
        int32_t h = hv >> 4, v = hv & 0x0f;
        if (h < 1 || 4 < h || v < 1 || 4 < v) return E_LumaChromaSubSamplingRatio;
        if (h == 3 || v == 3) return E_LumaChromaSubSamplingRatio;
        switch (d->num_components) {
        case 1:
            h = 1;
            v = 1;
            break;
        case 3:
            if (i == 0) {
                if (v == 4) return E_LumaChromaSubSamplingRatio;
            } else if (i == 1) {
                if (d->comp[0].h % h != 0 || d->comp[0].v % v != 0)
                    return E_LumaChromaSubSamplingRatio;
            } else {
                if (d->comp[1].h != h || d->comp[1].v != v) return E_LumaChromaSubSamplingRatio;
            }
            break;
        case 4:
            if (i == 0) {
                if (hv != 0x11 && hv != 0x22) return E_LumaChromaSubSamplingRatio;
            } else if (i == 1 || i == 2) {
                if (hv != 0x11) return E_LumaChromaSubSamplingRatio;
            } else {
                if (d->comp[0].h != h || d->comp[0].v != v) return E_LumaChromaSubSamplingRatio;
            }
            break;
        }
        d->comp[i].h = h;
        d->comp[i].v = v;
    }
    return 0;
}

/* processDri, :621-627 */
static int jd_process_dri(zo_jdec *d, int32_t n)
{
    if (n != 2) return E_DriWrongLength;
    TRY(jd_read_full(d, d->tmp, 2));
    d->restart_interval = (uint16_t)(((uint16_t)d->tmp[0] << 8) + d->tmp[1]);
    return 0;
}

/* processDqt, :629-666 */
static int jd_process_dqt(zo_jdec *d, int32_t n)
{
    while (n > 0) {
        n -= 1;
        uint8_t qi;
        TRY(jd_read_byte(d, &qi));
        uint8_t tq = qi & 0x0f;
        if (tq > 3) return E_BadTqValue;
        switch (qi >> 4) {
        case 0:
            if (n < 64) goto done;
            n -= 64;
            TRY(jd_read_full(d, d->tmp, 64));
            for (int i = 0; i < 64; i++) d->quant[tq][i] = d->tmp[i];
            break;
        case 1:
            if (n < 128) goto done;
            n -= 128;
            TRY(jd_read_full(d, d->tmp, 128));
            for (int i = 0; i < 64; i++)
                d->quant[tq][i] = ((int32_t)d->tmp[2 * i] << 8) | d->tmp[2 * i + 1];
            break;
        default:
            return E_BadPqValue;
        }
    }
done:
    if (n != 0) return E_DqtWrongLength;
    return 0;
}

/* processApp0Marker, :668-680 */
static int jd_process_app0(zo_jdec *d, int32_t n)
{
    if (n < 5) return jd_ignore(d, n);
    TRY(jd_read_full(d, d->tmp, 5));
    d->jfif = d->tmp[0] == 'J' && d->tmp[1] == 'F' && d->tmp[2] == 'I' && d->tmp[3] == 'F' &&
              d->tmp[4] == 0;
    return jd_ignore(d, n - 5);
}

/* processApp14Marker, :682-697 */
static int jd_process_app14(zo_jdec *d, int32_t n)
{
    if (n < 12) return jd_ignore(d, n);
    TRY(jd_read_full(d, d->tmp, 12));
    if (d->tmp[0] == 'A' && d->tmp[1] == 'd' && d->tmp[2] == 'o' && d->tmp[3] == 'b' &&
        d->tmp[4] == 'e') {
        d->adobe_transform_valid = 1;
        d->adobe_transform = d->tmp[11];
    }
    return jd_ignore(d, n - 12);
}

/* isRgb, :699-709 */
static int jd_is_rgb(const zo_jdec *d)
{
    if (d->jfif) return 0;
    if (d->adobe_transform_valid && d->adobe_transform == 0) return 1;
    return d->comp[0].id == 'R' && d->comp[1].id == 'G' && d->comp[2].id == 'B';
}

/* processDht, :1026-1111 */
static int jd_process_dht(zo_jdec *d, int32_t n)
{
    while (n > 0) {
        if (n < 17) return E_DhtWrongLength;
        TRY(jd_read_full(d, d->tmp, 17));
        uint8_t tc = d->tmp[0] >> 4;
        if (tc > 1) return E_BadTcValue;
        uint8_t th = d->tmp[0] & 0x0f;
        if (th > 3 || (d->baseline && th > 1)) return E_BadThValue;
        zo_huff *h = &d->huff[tc][th];
        int32_t ncodes[16];
        h->num_codes = 0;
        for (int i = 0; i < 16; i++) {
            ncodes[i] = d->tmp[i + 1];
            h->num_codes += ncodes[i];
        }
        if (h->num_codes == 0) return E_HuffZeroLength;
        if (h->num_codes > 256) return E_HuffTooLong;
        n -= h->num_codes + 17;
        if (n < 0) return E_DhtWrongLength;
        TRY(jd_read_full(d, h->vals, (size_t)h->num_codes));
        memset(h->lut, 0, sizeof(h->lut));
        uint32_t code = 0;
        int vi = 0;
        for (int i = 0; i < 8; i++) {
            code <<= 1;
            for (int j = 0; j < ncodes[i]; j++) {
                uint32_t base = code << (7 - i);
                uint16_t lv = (uint16_t)(((uint16_t)h->vals[vi] << 8) | (uint16_t)(2 + i));
                for (uint32_t k = 0; k < (1u << (7 - i)); k++) {
                    if ((base | k) > 255) return E_Panic; /* over-full table */
                    h->lut[base | k] = lv;
                }
                code++;
                vi++;
            }
        }
        int32_t cb = 0, idx = 0;
        for (int i = 0; i < 16; i++) {
            if (ncodes[i] == 0) {
                h->min_codes[i] = -1;
                h->max_codes[i] = -1;
                h->vals_indices[i] = -1;
            } else {
                h->min_codes[i] = cb;
                h->max_codes[i] = cb + ncodes[i] - 1;
                h->vals_indices[i] = idx;
                cb += ncodes[i];
                idx += ncodes[i];
            }
            cb <<= 1;
        }
    }
    return 0;
}

/* YCbCrImage.yCbCrSize, src/image/image.zig:521-555, for rect (0,0,w,h) */
static void ycbcr_size(int32_t w, int32_t h, int sub, int32_t *cw, int32_t *ch)
{
    switch (sub) {
    case ZO_422: *cw = (w + 1) / 2; *ch = h; break;
    case ZO_420: *cw = (w + 1) / 2; *ch = (h + 1) / 2; break;
    case ZO_440: *cw = w; *ch = (h + 1) / 2; break;
    case ZO_411: *cw = (w + 3) / 4; *ch = h; break;
    case ZO_410: *cw = (w + 3) / 4; *ch = (h + 1) / 2; break;
    default: *cw = w; *ch = h; break;
    }
}

/* makeImg, decoder.zig:1708-1783 (+ YCbCrImage.init/subImage image.zig:484-583) */
static int jd_make_img(zo_jdec *d, int32_t mxx, int32_t myy)
{
    if (d->num_components == 1) {
        /* a fresh gray image on every SOS (:1710-1735); its pixels are
         * uninitialised in the reference; every in-bounds block is written. */
        free(d->gray_pixels);
        size_t w = (size_t)(8 * mxx), h = (size_t)(8 * myy);
        d->gray_pixels = (uint8_t *)calloc((w * h) != 0 ? (w * h) : 1, 1);
        if (!d->gray_pixels) return E_OutOfMemory;
        d->gray_stride = w;
        d->have_gray = 1;
        return 0;
    }
    int32_t h0 = d->comp[0].h, v0 = d->comp[0].v;
    int32_t hr = h0 / d->comp[1].h, vr = v0 / d->comp[1].v;
    int sub;
    switch ((hr << 4) | vr) {
    case 0x11: sub = ZO_444; break;
    case 0x12: sub = ZO_440; break;
    case 0x21: sub = ZO_422; break;
    case 0x22: sub = ZO_420; break;
    case 0x41: sub = ZO_411; break;
    case 0x42: sub = ZO_410; break;
    default: return E_Panic; /* unreachable at :1752 */
    }
    int32_t w = 8 * h0 * mxx, h = 8 * v0 * myy, cw, ch;
    ycbcr_size(w, h, sub, &cw, &ch);
    size_t total = (size_t)w * h + 2 * (size_t)cw * ch;
    d->ycbcr_pixels = (uint8_t *)calloc(total ? total : 1, 1);
    if (!d->ycbcr_pixels) return E_OutOfMemory;
    d->ycbcr_len = total;
    d->y_stride = (size_t)w;
    d->c_stride = (size_t)cw;
    d->cb_off = (size_t)w * h;
    d->cr_off = (size_t)w * h + (size_t)cw * ch;
    d->subsample = sub;
    d->have_ycbcr = 1;
    if (d->num_components == 4) {
        int32_t h3 = d->comp[3].h, v3 = d->comp[3].v;
        size_t bl = (size_t)(8 * h3 * mxx) * (size_t)(8 * v3 * myy);
        d->black_pixels = (uint8_t *)calloc(bl ? bl : 1, 1);
        if (!d->black_pixels) return E_OutOfMemory;
        d->black_stride = (size_t)(8 * h3 * mxx);
    }
    return 0;
}

/* reconstructBlock, decoder.zig:1553-1634 (level shift + clamp :1611-1633) */
static void reconstruct_into(int32_t *b, const int32_t *qt, uint8_t *dst, size_t stride)
{
    for (int z = 0; z < 64; z++) b[UNZIG[z]] *= qt[z];
    zo_idct(b);
    for (int y = 0; y < 8; y++) {
        for (int x = 0; x < 8; x++) {
            int32_t c = b[8 * y + x];
            if (c < -128) c = 0;
            else if (c > 127) c = 255;
            else c += 128;
            dst[y * stride + x] = (uint8_t)c;
        }
    }
}

static int jd_reconstruct_block(zo_jdec *d, int32_t *b, int32_t bx, int32_t by, int ci)
{
    const int32_t *qt = d->quant[d->comp[ci].tq];
    uint8_t *dst;
    size_t stride;
    if (d->num_components == 1) {
        if (!d->have_gray) return E_Panic; /* :1581 */
        stride = d->gray_stride;
        dst = d->gray_pixels + 8 * ((size_t)by * stride + (size_t)bx);
    } else {
        if (!d->have_ycbcr) return E_Panic; /* :1606 */
        switch (ci) {
        case 0: stride = d->y_stride; dst = d->ycbcr_pixels; break;
        case 1: stride = d->c_stride; dst = d->ycbcr_pixels + d->cb_off; break;
        case 2: stride = d->c_stride; dst = d->ycbcr_pixels + d->cr_off; break;
        case 3: stride = d->black_stride; dst = d->black_pixels; break;
        default: return E_UnsupportedComponent;
        }
        dst += 8 * ((size_t)by * stride + (size_t)bx);
    }
    reconstruct_into(b, qt, dst, stride);
    return 0;
}

/* refineNonZeroes, :1522-1549 */
static int jd_refine_nonzeroes(zo_jdec *d, int32_t *b, int32_t zig, int32_t zig_end, int32_t nz,
                               int32_t delta, int32_t *out_zig)
{
    for (; zig <= zig_end; zig++) {
        int idx = UNZIG[zig];
        if (b[idx] == 0) {
            if (nz == 0) break;
            nz--;
            continue;
        }
        int bit;
        TRY(jd_decode_bit(d, &bit));
        if (!bit) continue;
        if (b[idx] >= 0) b[idx] += delta;
        else b[idx] -= delta;
    }
    *out_zig = zig;
    return 0;
}

/* refine, :1459-1518 */
static int jd_refine(zo_jdec *d, int32_t *b, zo_huff *h, int32_t zig_start, int32_t zig_end,
                     int32_t delta)
{
    if (zig_start == 0) {
        if (zig_end != 0) return E_Panic;
        int bit;
        TRY(jd_decode_bit(d, &bit));
        if (bit) b[0] |= delta;
        return 0;
    }
    int32_t zig = zig_start;
    if (d->eob_run == 0) {
        for (; zig <= zig_end; zig++) {
            int32_t z = 0;
            uint8_t value;
            TRY(jd_decode_huffman(d, h, &value));
            uint8_t val0 = value >> 4, val1 = value & 0x0f;
            if (val1 == 0) {
                if (val0 != 0x0f) {
                    d->eob_run = (uint16_t)(1u << val0);
                    if (val0 != 0) {
                        uint32_t bits;
                        TRY(jd_decode_bits(d, val0, &bits));
                        d->eob_run |= (uint16_t)bits;
                    }
                    break;
                }
            } else if (val1 == 1) {
                z = delta;
                int bit;
                TRY(jd_decode_bit(d, &bit));
                if (!bit) z = -z;
            } else {
                return E_UnexpectedHuffmanCode;
            }
            TRY(jd_refine_nonzeroes(d, b, zig, zig_end, val0, delta, &zig));
            if (zig > zig_end) return E_TooManyCoefficients;
            if (z != 0) b[UNZIG[zig]] = z;
        }
    }
    if (d->eob_run > 0) {
        d->eob_run--;
        int32_t dummy;
        TRY(jd_refine_nonzeroes(d, b, zig, zig_end, -1, delta, &dummy));
    }
    return 0;
}

/* findRst, :1671-1705 */
static int jd_find_rst(zo_jdec *d, uint8_t expected)
{
    for (;;) {
        size_t i = 0;
        if (d->tmp[0] == 0xff) {
            if (d->tmp[1] == expected) return 0;
            else if (d->tmp[1] == 0xff) i = 1;
            else if (d->tmp[1] != 0x00) return E_BadRSTMarker;
        } else if (d->tmp[1] == 0xff) {
            d->tmp[0] = 0xff;
            i = 1;
        }
        TRY(jd_read_full(d, d->tmp + i, 2 - i));
    }
}

/* processSos, :1148-1455 */
static int jd_process_sos(zo_jdec *d, int32_t n)
{
    if (d->num_components == 0) return E_MissingSosMarker;
    if (n < 6 || 4 + 2 * d->num_components < n || n % 2 != 0) return E_SosWrongLength;
    TRY(jd_read_full(d, d->tmp, (size_t)n));
    uint8_t n_comp = d->tmp[0];
    if (n != 4 + 2 * n_comp) return E_SosWrongLength;
    struct { uint8_t id, td, ta; } scan[4];
    memset(scan, 0, sizeof(scan));
    int32_t total_hv = 0;
    for (int i = 0; i < n_comp; i++) {
        uint8_t sel = d->tmp[1 + 2 * i];
        int found = -1;
        for (int j = 0; j < d->num_components; j++)
            if (sel == d->comp[j].id) {
                found = j;
                break;
            }
        if (found < 0) return E_UnknownComponentSelector;
        scan[i].id = (uint8_t)found;
        for (int j = 0; j < i; j++)
            if (scan[i].id == scan[j].id) return E_RepeatedComponentIdentifier;
        total_hv += d->comp[found].h * d->comp[found].v;
        scan[i].td = d->tmp[2 + 2 * i] >> 4;
        if (scan[i].td > 3 || (d->baseline && scan[i].td > 1)) return E_BadTdValue;
        scan[i].ta = d->tmp[2 + 2 * i] & 0x0f;
        if (scan[i].ta > 3 || (d->baseline && scan[i].ta > 1)) return E_BadTaValue;
    }
    if (d->num_components > 1 && total_hv > 10) return E_SamplingFactorsTooLarge;

    int32_t zig_start = 0, zig_end = 63;
    uint32_t ah = 0, al = 0;
    if (d->progressive) {
        zig_start = d->tmp[1 + 2 * n_comp];
        zig_end = d->tmp[2 + 2 * n_comp];
        ah = d->tmp[3 + 2 * n_comp] >> 4;
        al = d->tmp[3 + 2 * n_comp] & 0x0f;
        if ((zig_start == 0 && zig_end != 0) || zig_start > zig_end || 64 <= zig_end)
            return E_BadSpectralSelection;
        if (zig_start != 0 && n_comp != 1) return E_ProgressiveACCoefficientsForMoreThanOneComponent;
        if (ah != 0 && ah != al + 1) return E_BadSuccessiveApproximation;
    }

    int32_t h0 = d->comp[0].h, v0 = d->comp[0].v;
    int32_t w = (int32_t)d->width, hgt = (int32_t)d->height;
    int32_t mxx = (w + 8 * h0 - 1) / (8 * h0);
    int32_t myy = (hgt + 8 * v0 - 1) / (8 * v0);
    d->mxx = mxx;
    d->myy = myy;
    if (!d->have_ycbcr) TRY(jd_make_img(d, mxx, myy));

    int accumulate = d->progressive || d->coeffs_only;
    if (accumulate) {
        /* loops over num_components using scan[i].id (:1269-1282) */
        for (int i = 0; i < d->num_components; i++) {
            int ci = scan[i].id;
            if (!d->prog[ci]) {
                size_t nb = (size_t)mxx * myy * d->comp[ci].h * d->comp[ci].v;
                d->prog[ci] = (int32_t *)calloc((nb * 64) != 0 ? (nb * 64) : 64, sizeof(int32_t));
                if (!d->prog[ci]) return E_OutOfMemory;
            }
        }
    }

    d->ba = 0;
    d->bm = 0;
    d->bn = 0;
    int32_t mcu = 0;
    uint8_t expected_rst = 0xd0;
    int32_t bx = 0, by = 0, block_count = 0;
    int32_t dc[4] = {0, 0, 0, 0};
    int32_t b[64];

    for (int32_t my = 0; my < myy; my++) {
        for (int32_t mx = 0; mx < mxx; mx++) {
            for (int k = 0; k < n_comp; k++) {
                int ci = scan[k].id;
                int32_t hi = d->comp[ci].h, vi = d->comp[ci].v;
                for (int32_t j = 0; j < hi * vi; j++) {
                    if (n_comp != 1) {
                        bx = hi * mx + j % hi;
                        by = vi * my + j / hi;
                    } else {
                        bx = block_count % (mxx * hi);
                        by = block_count / (mxx * hi);
                        block_count++;
                        if (bx * 8 >= (int32_t)d->width || by * 8 >= (int32_t)d->height) continue;
                    }
                    size_t bidx = (size_t)by * mxx * hi + bx;
                    /* progressive loads the partial block (:1340-1343); baseline starts
                     * from an empty block (:1344) even when only accumulating */
                    if (d->progressive) memcpy(b, d->prog[ci] + 64 * bidx, sizeof(b));
                    else memset(b, 0, sizeof(b));

                    if (ah != 0) {
                        TRY(jd_refine(d, b, &d->huff[1][scan[k].ta], zig_start, zig_end,
                                      (int32_t)1 << al));
                    } else {
                        int32_t zig = zig_start;
                        if (zig == 0) {
                            zig++;
                            uint8_t value;
                            TRY(jd_decode_huffman(d, &d->huff[0][scan[k].td], &value));
                            if (value > 16) return E_ExcessiveDCComponent;
                            int32_t delta;
                            TRY(jd_receive_extend(d, value, &delta));
                            dc[ci] += delta;
                            b[0] = dc[ci] << al;
                        }
                        if (zig <= zig_end && d->eob_run > 0) {
                            d->eob_run--;
                        } else {
                            zo_huff *hf = &d->huff[1][scan[k].ta];
                            for (; zig <= zig_end; zig++) {
                                uint8_t value;
                                TRY(jd_decode_huffman(d, hf, &value));
                                uint8_t val0 = value >> 4, val1 = value & 0x0f;
                                if (val1 != 0) {
                                    zig += val0;
                                    if (zig > zig_end) break;
                                    int32_t ac;
                                    TRY(jd_receive_extend(d, val1, &ac));
                                    b[UNZIG[zig]] = ac << al;
                                } else {
                                    if (val0 != 0x0f) {
                                        d->eob_run = (uint16_t)(1u << val0);
                                        if (val0 != 0) {
                                            uint32_t bits;
                                            TRY(jd_decode_bits(d, val0, &bits));
                                            d->eob_run |= (uint16_t)bits;
                                        }
                                        d->eob_run--;
                                        break;
                                    }
                                    zig += 0x0f;
                                }
                            }
                        }
                    }
                    if (accumulate) {
                        memcpy(d->prog[ci] + 64 * bidx, b, sizeof(b));
                        continue;
                    }
                    TRY(jd_reconstruct_block(d, b, bx, by, ci));
                }
            }
            mcu++;
            if (d->restart_interval > 0 && mcu % d->restart_interval == 0 && mcu < mxx * myy) {
                TRY(jd_read_full(d, d->tmp, 2));
                if (d->tmp[0] != 0xff || d->tmp[1] != expected_rst)
                    TRY(jd_find_rst(d, expected_rst));
                expected_rst++;
                if (expected_rst == 0xd8) expected_rst = 0xd0;
                d->ba = 0;
                d->bm = 0;
                d->bn = 0;
                memset(dc, 0, sizeof(dc));
                d->eob_run = 0;
            }
        }
    }
    return 0;
}

/* reconstructProgressiveImage, :1636-1661 */
static int jd_reconstruct_progressive(zo_jdec *d)
{
    int32_t h0 = d->comp[0].h;
    int32_t mxx = ((int32_t)d->width + 8 * h0 - 1) / (8 * h0);
    for (int i = 0; i < d->num_components; i++) {
        if (!d->prog[i]) continue;
        size_t v = (size_t)(8 * (d->comp[0].v / d->comp[i].v));
        size_t h = (size_t)(8 * (d->comp[0].h / d->comp[i].h));
        size_t stride = (size_t)(mxx * d->comp[i].h);
        for (size_t by = 0; by * v < d->height; by++)
            for (size_t bx = 0; bx * h < d->width; bx++)
                TRY(jd_reconstruct_block(d, d->prog[i] + 64 * (by * stride + bx), (int32_t)bx,
                                         (int32_t)by, i));
    }
    return 0;
}

static void jd_free(zo_jdec *d)
{
    free(d->gray_pixels);
    free(d->ycbcr_pixels);
    free(d->black_pixels);
    for (int i = 0; i < 4; i++) free(d->prog[i]);
}

/* decodeInner marker loop, decoder.zig:220-355 */
static int jd_markers(zo_jdec *d)
{
    TRY(jd_read_full(d, d->tmp, 2));
    if (d->tmp[0] != 0xff || d->tmp[1] != 0xd8) return E_InvalidSOIMarker;
    for (;;) {
        TRY(jd_read_full(d, d->tmp, 2));
        while (d->tmp[0] != 0xff) {
            d->tmp[0] = d->tmp[1];
            TRY(jd_read_byte(d, &d->tmp[1]));
        }
        uint8_t marker = d->tmp[1];
        if (marker == 0) continue;
        while (marker == 0xff) TRY(jd_read_byte(d, &marker));
        if (marker == 0xd9) break;
        if (0xd0 <= marker && marker <= 0xd7) continue;
        TRY(jd_read_full(d, d->tmp, 2));
        int32_t n = ((int32_t)d->tmp[0] << 8) + d->tmp[1] - 2;
        if (n < 0) return E_ShortSegmentLength;
        switch (marker) {
        case 0xc0:
        case 0xc1:
        case 0xc2:
            d->baseline = marker == 0xc0;
            d->progressive = marker == 0xc2;
            TRY(jd_process_sof(d, n));
            break;
        case 0xdb: TRY(jd_process_dqt(d, n)); break;
        case 0xdd: TRY(jd_process_dri(d, n)); break;
        case 0xc4: TRY(jd_process_dht(d, n)); break;
        case 0xda: TRY(jd_process_sos(d, n)); break;
        case 0xe0: TRY(jd_process_app0(d, n)); break;
        case 0xee: TRY(jd_process_app14(d, n)); break;
        default:
            if ((0xe0 <= marker && marker <= 0xef) || marker == 0xfe) TRY(jd_ignore(d, n));
            else if (marker < 0xc0) return E_UnknownMarker;
            else return E_UnsupportedMarker;
        }
    }
    return 0;
}

static void jd_init(zo_jdec *d, const uint8_t *buf, size_t len)
{
    memset(d, 0, sizeof(*d));
    d->src = buf;
    d->src_len = len;
}

int zo_jpeg_decode(const uint8_t *buf, size_t len, zo_image *out)
{
    memset(out, 0, sizeof(*out));
    zo_jdec *d = (zo_jdec *)calloc(1, sizeof(zo_jdec));
    if (!d) return E_OutOfMemory;
    jd_init(d, buf, len);
    int e = jd_markers(d);
    if (!e && d->progressive) e = jd_reconstruct_progressive(d);
    if (e) {
        jd_free(d);
        free(d);
        return e;
    }
    /* output select, :361-372 */
    if (d->have_gray) {
        out->kind = ZO_GRAY;
        out->max_x = (int32_t)d->width;
        out->max_y = (int32_t)d->height;
        out->pixels = d->gray_pixels;
        out->pixels_len = d->gray_stride * (size_t)(8 * d->myy);
        out->stride = d->gray_stride;
        d->gray_pixels = NULL;
    } else if (d->have_ycbcr) {
        int32_t w = (int32_t)d->width, h = (int32_t)d->height;
        if (d->black_pixels) {
            /* applyBlack, :792-902 */
            if (!d->adobe_transform_valid) e = E_UnsupportedColorModel;
            else if (d->adobe_transform != 0) e = E_Unsupported; /* YCbCrK via drawYCbCr: out */
            else {
                uint8_t *px = (uint8_t *)malloc((size_t)w * h * 4 + 1);
                if (!px) e = E_OutOfMemory;
                else {
                    const uint8_t *srcs[4] = {d->ycbcr_pixels, d->ycbcr_pixels + d->cb_off,
                                              d->ycbcr_pixels + d->cr_off, d->black_pixels};
                    size_t strides[4] = {d->y_stride, d->c_stride, d->c_stride, d->black_stride};
                    for (int t = 0; t < 4; t++) {
                        int sub = d->comp[t].h != d->comp[0].h || d->comp[t].v != d->comp[0].v;
                        for (int32_t y = 0; y < h; y++) {
                            size_t sy = (size_t)y;
                            if (sub) sy >>= 1;
                            for (int32_t x = 0; x < w; x++) {
                                size_t sx = (size_t)x;
                                if (sub) sx >>= 1;
                                px[((size_t)y * w + x) * 4 + t] =
                                    (uint8_t)(255 - srcs[t][sy * strides[t] + sx]);
                            }
                        }
                    }
                    out->kind = ZO_CMYK;
                    out->max_x = w;
                    out->max_y = h;
                    out->pixels = px;
                    out->pixels_len = (size_t)w * h * 4;
                    out->stride = (size_t)w * 4;
                }
            }
        } else if (jd_is_rgb(d)) {
            /* convertToRGB, :751-783 */
            size_t c_scale = (size_t)(d->comp[0].h / d->comp[1].h);
            uint8_t *px = (uint8_t *)malloc((size_t)w * h * 4 + 1);
            if (!px) e = E_OutOfMemory;
            else {
                zo_image tmpi;
                memset(&tmpi, 0, sizeof(tmpi));
                for (int32_t y = 0; y < h; y++) {
                    size_t po = (size_t)y * w * 4;
                    size_t yo = (size_t)y * d->y_stride;
                    size_t co;
                    switch (d->subsample) {
                    case ZO_420: case ZO_440: case ZO_410: co = (size_t)(y / 2) * d->c_stride; break;
                    default: co = (size_t)y * d->c_stride; break;
                    }
                    for (int32_t i = 0; i < w; i++) {
                        px[po + 4 * i + 0] = d->ycbcr_pixels[yo + i];
                        px[po + 4 * i + 1] = d->ycbcr_pixels[d->cb_off + co + i / c_scale];
                        px[po + 4 * i + 2] = d->ycbcr_pixels[d->cr_off + co + i / c_scale];
                        px[po + 4 * i + 3] = 255;
                    }
                }
                out->kind = ZO_RGBA;
                out->max_x = w;
                out->max_y = h;
                out->pixels = px;
                out->pixels_len = (size_t)w * h * 4;
                out->stride = (size_t)w * 4;
            }
        } else {
            out->kind = ZO_YCBCR;
            out->max_x = w;
            out->max_y = h;
            out->pixels = d->ycbcr_pixels;
            out->pixels_len = d->ycbcr_len;
            out->y_off = 0;
            out->cb_off = d->cb_off;
            out->cr_off = d->cr_off;
            out->y_stride = d->y_stride;
            out->c_stride = d->c_stride;
            out->subsample = d->subsample;
            d->ycbcr_pixels = NULL;
        }
    } else {
        e = E_MissingSosMarker;
    }
    jd_free(d);
    free(d);
    return e;
}

int zo_jpeg_decode_coeffs(const uint8_t *buf, size_t len, zo_jpeg_coeffs *out)
{
    memset(out, 0, sizeof(*out));
    zo_jdec *d = (zo_jdec *)calloc(1, sizeof(zo_jdec));
    if (!d) return E_OutOfMemory;
    jd_init(d, buf, len);
    d->coeffs_only = 1;
    int e = jd_markers(d);
    if (!e && !d->have_gray && !d->have_ycbcr) e = E_MissingSosMarker;
    if (!e) {
        out->width = d->width;
        out->height = d->height;
        out->n_comp = d->num_components;
        for (int i = 0; i < 4; i++) {
            out->h[i] = d->comp[i].h;
            out->v[i] = d->comp[i].v;
            out->tq[i] = d->comp[i].tq;
            out->comp_id[i] = d->comp[i].id;
            out->grid[i] = d->prog[i];
            d->prog[i] = NULL;
        }
        out->mxx = d->mxx;
        out->myy = d->myy;
        out->progressive = d->progressive;
        out->jfif = d->jfif;
        out->adobe_valid = d->adobe_transform_valid;
        out->adobe_transform = d->adobe_transform;
        memcpy(out->quant, d->quant, sizeof(out->quant));
    }
    jd_free(d);
    free(d);
    return e;
}

void zo_jpeg_coeffs_free(zo_jpeg_coeffs *c)
{
    for (int i = 0; i < 4; i++) {
        free(c->grid[i]);
        c->grid[i] = NULL;
    }
}

void zo_jpeg_reconstruct_grids(int32_t n_comp, uint32_t width, uint32_t height, const int32_t *h,
                               const int32_t *v, int32_t mxx, int32_t myy, int32_t *const *coeffs,
                               const int32_t *const *qt_zigzag, int32_t progressive,
                               uint8_t *const *planes, const size_t *strides)
{
    int32_t b[64];
    for (int c = 0; c < n_comp; c++) {
        if (!coeffs[c]) continue;
        size_t gw = (size_t)(mxx * h[c]);
        size_t gh = (size_t)(myy * v[c]);
        size_t bv = (size_t)(8 * (v[0] / v[c])), bh = (size_t)(8 * (h[0] / h[c]));
        for (size_t by = 0; by < gh; by++) {
            if (progressive && by * bv >= height) break;
            for (size_t bx = 0; bx < gw; bx++) {
                if (progressive && bx * bh >= width) break;
                memcpy(b, coeffs[c] + 64 * (by * gw + bx), sizeof(b));
                reconstruct_into(b, qt_zigzag[c], planes[c] + 8 * (by * strides[c] + bx),
                                 strides[c]);
            }
        }
    }
}

/* ======================================================================== */
/* Color / Image                                                            */
/* ======================================================================== */

/* Color.toRGBA .ycbcr, src/color/color.zig:90-113 */
static void ycbcr_to_rgba16(uint8_t Y, uint8_t Cb, uint8_t Cr, uint32_t o[4])
{
    int32_t yy1 = (int32_t)Y * 0x10101;
    int32_t cb1 = (int32_t)Cb - 128;
    int32_t cr1 = (int32_t)Cr - 128;
    int32_t r = yy1 + 91881 * cr1;
    r = (((uint32_t)r & 0xff000000u) == 0) ? (r >> 8) : (~(r >> 31) & 0xffff);
    int32_t g = yy1 - 22554 * cb1 - 46802 * cr1;
    g = (((uint32_t)g & 0xff000000u) == 0) ? (g >> 8) : (~(g >> 31) & 0xffff);
    int32_t bb = yy1 + 116130 * cb1;
    bb = (((uint32_t)bb & 0xff000000u) == 0) ? (bb >> 8) : (~(bb >> 31) & 0xffff);
    o[0] = (uint32_t)r;
    o[1] = (uint32_t)g;
    o[2] = (uint32_t)bb;
    o[3] = 0xffff;
}

/* Color.toRGBA, color.zig:31-131, for a {r,g,b,a,tag} color */
static void color_rgba16(int tag, const uint8_t *c, uint32_t o[4])
{
    uint32_t r = c[0], g = c[1], b = c[2], a = c[3];
    if (tag == 0) { /* .rgba :34-44 */
        o[0] = r | r << 8;
        o[1] = g | g << 8;
        o[2] = b | b << 8;
        o[3] = a | a << 8;
    } else { /* .nrgba :52-72 */
        o[0] = ((r | r << 8) * a) / 0xff;
        o[1] = ((g | g << 8) * a) / 0xff;
        o[2] = ((b | b << 8) * a) / 0xff;
        o[3] = a | a << 8;
    }
}

static int pt_in(const zo_image *m, int32_t x, int32_t y)
{
    return x >= m->min_x && x < m->max_x && y >= m->min_y && y < m->max_y;
}

/* Image.at(x,y).toRGBA(), image.zig:54-66 with each concrete at() */
void zo_at_rgba16(const zo_image *m, int32_t x, int32_t y, uint32_t o[4])
{
    o[0] = o[1] = o[2] = o[3] = 0;
    int in = pt_in(m, x, y);
    size_t dx = (size_t)(x - m->min_x), dy = (size_t)(y - m->min_y);
    switch (m->kind) {
    case ZO_GRAY: { /* .gray :122-126 */
        uint32_t v = in ? m->pixels[dy * m->stride + dx] : 0;
        v |= v << 8;
        o[0] = o[1] = o[2] = v;
        o[3] = 0xffff;
        break;
    }
    case ZO_GRAY16: { /* .gray16 :127-130 */
        uint32_t v = 0;
        if (in) {
            const uint8_t *s = m->pixels + dy * m->stride + 2 * dx;
            v = (uint32_t)s[0] << 8 | s[1];
        }
        o[0] = o[1] = o[2] = v;
        o[3] = 0xffff;
        break;
    }
    case ZO_YCBCR: { /* YCbCrAt image.zig:614-630 */
        if (!in) {
            ycbcr_to_rgba16(0, 0, 0, o);
            break;
        }
        size_t yi = dy * m->y_stride + dx;
        size_t ci;
        size_t cdy = (size_t)(y / 2 - m->min_y / 2), cdx2 = (size_t)(x / 2 - m->min_x / 2),
               cdx4 = (size_t)(x / 4 - m->min_x / 4);
        switch (m->subsample) { /* cOffset :594-605 */
        case ZO_422: ci = dy * m->c_stride + cdx2; break;
        case ZO_420: ci = cdy * m->c_stride + cdx2; break;
        case ZO_440: ci = cdy * m->c_stride + dx; break;
        case ZO_411: ci = dy * m->c_stride + cdx4; break;
        case ZO_410: ci = cdy * m->c_stride + cdx4; break;
        default: ci = dy * m->c_stride + dx; break;
        }
        ycbcr_to_rgba16(m->pixels[m->y_off + yi], m->pixels[m->cb_off + ci],
                        m->pixels[m->cr_off + ci], o);
        break;
    }
    case ZO_RGBA:
    case ZO_NRGBA: {
        uint8_t c[4] = {0, 0, 0, 0};
        if (in) memcpy(c, m->pixels + dy * m->stride + 4 * dx, 4);
        color_rgba16(m->kind == ZO_NRGBA, c, o);
        break;
    }
    case ZO_RGBA64: { /* .rgba64 :45-51 */
        if (!in) break; /* Color{.rgba = .{}} -> zeros */
        const uint8_t *s = m->pixels + dy * m->stride + 8 * dx;
        for (int k = 0; k < 4; k++) o[k] = (uint32_t)s[2 * k] << 8 | s[2 * k + 1];
        break;
    }
    case ZO_NRGBA64: { /* .nrgba64 :73-89 */
        if (!in) break;
        const uint8_t *s = m->pixels + dy * m->stride + 8 * dx;
        uint32_t r = (uint32_t)s[0] << 8 | s[1], g = (uint32_t)s[2] << 8 | s[3],
                 b = (uint32_t)s[4] << 8 | s[5], a = (uint32_t)s[6] << 8 | s[7];
        o[0] = r * a / 0xffff;
        o[1] = g * a / 0xffff;
        o[2] = b * a / 0xffff;
        o[3] = a;
        break;
    }
    case ZO_CMYK: { /* .cmyk :115-121 */
        uint8_t c[4] = {0, 0, 0, 0};
        if (in) memcpy(c, m->pixels + dy * m->stride + 4 * dx, 4);
        uint32_t w = 0xffff - (uint32_t)c[3] * 0x101;
        o[0] = (0xffff - (uint32_t)c[0] * 0x101) * w / 0xffff;
        o[1] = (0xffff - (uint32_t)c[1] * 0x101) * w / 0xffff;
        o[2] = (0xffff - (uint32_t)c[2] * 0x101) * w / 0xffff;
        o[3] = 0xffff;
        break;
    }
    case ZO_PALETTED: { /* PalettedImage.at image.zig:856-866 */
        if (m->palette_len == 0) break;
        int idx = in ? m->pixels[dy * m->stride + dx] : 0;
        if (idx >= m->palette_len) break; /* cannot happen after growth */
        const uint8_t *p = m->palette + 5 * idx;
        color_rgba16(p[4], p, o);
        break;
    }
    }
}

/* Image.rgbaPixels, image.zig:103-130 */
int zo_rgba_pixels(const zo_image *m, uint8_t *out)
{
    int32_t w = m->max_x - m->min_x, h = m->max_y - m->min_y;
    for (int32_t y = m->min_y; y < m->max_y; y++) {
        for (int32_t x = m->min_x; x < m->max_x; x++) {
            uint32_t c[4];
            zo_at_rgba16(m, x, y, c);
            size_t i = ((size_t)(y - m->min_y) * w + (size_t)(x - m->min_x)) * 4;
            out[i + 0] = (uint8_t)(c[0] >> 8);
            out[i + 1] = (uint8_t)(c[1] >> 8);
            out[i + 2] = (uint8_t)(c[2] >> 8);
            out[i + 3] = (uint8_t)(c[3] >> 8);
        }
    }
    (void)h;
    return 0;
}

void zo_image_free(zo_image *m)
{
    free(m->pixels);
    free(m->palette);
    m->pixels = NULL;
    m->palette = NULL;
}

/* ======================================================================== */
/* PNG                                                                       */
/* ======================================================================== */

enum { CD_INVALID, CD_G1, CD_G2, CD_G4, CD_G8, CD_GA8, CD_TC8, CD_P1, CD_P2, CD_P4, CD_P8,
       CD_TCA8, CD_G16, CD_GA16, CD_TC16, CD_TCA16 };

/* interlacing, src/png/decoder.zig:59-67 */
static const uint32_t ADAM7[7][4] = {
    {0, 0, 8, 8}, {4, 0, 8, 8}, {0, 4, 4, 8}, {2, 0, 4, 4},
    {0, 2, 2, 4}, {1, 0, 2, 2}, {0, 1, 1, 2},
};

/* filter reconstruction for one row, decoder.zig:806-842 + filterPaeth :1152-1182 */
static int unfilter_row(uint8_t ft, uint8_t *c, const uint8_t *p, size_t n, size_t bpp)
{
    switch (ft) {
    case 0: break;
    case 1:
        for (size_t i = bpp; i < n; i++) c[i] = (uint8_t)(c[i] + c[i - bpp]);
        break;
    case 2:
        for (size_t i = 0; i < n; i++) c[i] = (uint8_t)(c[i] + p[i]);
        break;
    case 3:
        for (size_t i = 0; i < bpp && i < n; i++) c[i] = (uint8_t)(c[i] + p[i] / 2);
        for (size_t i = bpp; i < n; i++)
            c[i] = (uint8_t)(c[i] + (uint8_t)(((uint16_t)c[i - bpp] + (uint16_t)p[i]) / 2));
        break;
    case 4:
        for (size_t i = 0; i < bpp && i < n; i++) c[i] = (uint8_t)(c[i] + p[i]);
        for (size_t i = bpp; i < n; i++) {
            int a = c[i - bpp], b = p[i], cc = p[i - bpp];
            int pp = a + b - cc;
            int pa = pp > a ? pp - a : a - pp;
            int pb = pp > b ? pp - b : b - pp;
            int pc = pp > cc ? pp - cc : cc - pp;
            int pred;
            if (pa <= pb && pa <= pc) pred = a;
            else if (pb <= pc) pred = b;
            else pred = cc;
            c[i] = (uint8_t)(c[i] + pred);
        }
        break;
    default:
        return E_InvalidFilterType;
    }
    return 0;
}

int zo_png_unfilter(const uint8_t *filtered, uint32_t rows, uint32_t row_bytes,
                    uint32_t bytes_per_pixel, uint8_t *out)
{
    const uint8_t *prev = NULL;
    uint8_t *zero = (uint8_t *)calloc(row_bytes + 1, 1);
    if (!zero) return E_OutOfMemory;
    prev = zero;
    for (uint32_t y = 0; y < rows; y++) {
        const uint8_t *f = filtered + (size_t)y * (row_bytes + 1);
        uint8_t *c = out + (size_t)y * row_bytes;
        memcpy(c, f + 1, row_bytes);
        int e = unfilter_row(f[0], c, prev, row_bytes, bytes_per_pixel);
        if (e) {
            free(zero);
            return e;
        }
        prev = c;
    }
    free(zero);
    return 0;
}

typedef struct {
    const uint8_t *src;
    size_t len, pos;
    uint32_t crc;
    uint32_t width, height;
    uint8_t depth, color_type;
    int cd;
    int interlace;
    int stage; /* 0 start 1 ihdr 2 plte 3 trns 4 idat 5 iend */
    uint8_t *palette; /* 5 bytes/entry */
    int32_t palette_len, palette_cap;
    int use_transparent;
    uint8_t transparent[6];
    zo_image img;
    int have_img;
} zo_pdec;

/* r.readSliceAll over a fixed reader */
static int pd_read(zo_pdec *d, uint8_t *p, size_t n)
{
    if (d->len - d->pos < n) {
        d->pos = d->len;
        return E_EndOfStream;
    }
    memcpy(p, d->src + d->pos, n);
    d->pos += n;
    return 0;
}

static uint32_t be32(const uint8_t *b) { return (uint32_t)b[0] << 24 | (uint32_t)b[1] << 16 | (uint32_t)b[2] << 8 | b[3]; }

/* verifyChecksum, :1264-1277 */
static int pd_verify(zo_pdec *d)
{
    uint8_t b[4];
    TRY(pd_read(d, b, 4));
    if (be32(b) != d->crc) return E_InvalidChecksum;
    return 0;
}

static int pd_read_crc(zo_pdec *d, uint8_t *p, size_t n)
{
    TRY(pd_read(d, p, n));
    d->crc = (uint32_t)crc32(d->crc, p, (uInt)n);
    return 0;
}

/* skipChunk, :1184-1197 */
static int pd_skip(zo_pdec *d, uint32_t len)
{
    uint8_t scratch[768];
    while (len > 0) {
        uint32_t k = len < sizeof(scratch) ? len : (uint32_t)sizeof(scratch);
        TRY(pd_read_crc(d, scratch, k));
        len -= k;
    }
    return 0;
}

/* parseIhdr, :326-401 */
static int pd_ihdr(zo_pdec *d, uint32_t length)
{
    if (length != 13) return E_InvalidIHDRLength;
    uint8_t b[13];
    TRY(pd_read_crc(d, b, 13));
    if (b[10] != 0) return E_UnsupportedCompressionMethod;
    if (b[11] != 0) return E_UnsupportedFilterMethod;
    d->interlace = b[12];
    if (d->interlace != 0 && d->interlace != 1) return E_UnsupportedInterlaceMethod;
    uint32_t w = be32(b), h = be32(b + 4);
    if (w == 0 || h == 0) return E_InvalidDimension;
    uint64_t np = (uint64_t)w * h;
    if (np >> 32) return E_DimensionOverflow;
    if ((uint32_t)np != (uint32_t)((uint32_t)np * 8u) / 8u) return E_DimensionOverflow;
    d->depth = b[8];
    uint8_t ct = b[9];
    if (ct != 0 && ct != 2 && ct != 3 && ct != 4 && ct != 6) return E_InvalidColorType;
    d->color_type = ct;
    d->width = w;
    d->height = h;
    switch (d->depth) {
    case 1: d->cd = ct == 0 ? CD_G1 : ct == 3 ? CD_P1 : CD_INVALID; break;
    case 2: d->cd = ct == 0 ? CD_G2 : ct == 3 ? CD_P2 : CD_INVALID; break;
    case 4: d->cd = ct == 0 ? CD_G4 : ct == 3 ? CD_P4 : CD_INVALID; break;
    case 8:
        d->cd = ct == 0 ? CD_G8 : ct == 2 ? CD_TC8 : ct == 3 ? CD_P8 : ct == 4 ? CD_GA8 : CD_TCA8;
        break;
    case 16:
        d->cd = ct == 0 ? CD_G16 : ct == 2 ? CD_TC16 : ct == 4 ? CD_GA16 : ct == 6 ? CD_TCA16 : CD_INVALID;
        break;
    default: return E_UnsupportedBitDepth;
    }
    if (d->cd == CD_INVALID) return E_InvalidColorTypeDepthCombo;
    return pd_verify(d);
}

static int cd_paletted(int cd) { return cd >= CD_P1 && cd <= CD_P8; }

/* parsePlte, :604-646 */
static int pd_plte(zo_pdec *d, uint32_t length)
{
    uint32_t np = length / 3;
    if (length % 3 != 0 || np == 0 || np > 256 || np > (1u << d->depth)) return E_BadPlteLength;
    uint8_t b[768];
    TRY(pd_read_crc(d, b, np * 3));
    if (cd_paletted(d->cd)) {
        free(d->palette);
        d->palette = (uint8_t *)calloc(256, 5);
        if (!d->palette) return E_OutOfMemory;
        for (uint32_t i = 0; i < np; i++) {
            d->palette[5 * i + 0] = b[3 * i];
            d->palette[5 * i + 1] = b[3 * i + 1];
            d->palette[5 * i + 2] = b[3 * i + 2];
            d->palette[5 * i + 3] = 0xff;
            d->palette[5 * i + 4] = 0;
        }
        /* entries past the PLTE: opaque black (Go's behaviour; see header) */
        for (uint32_t i = np; i < 256; i++) d->palette[5 * i + 3] = 0xff;
        d->palette_len = (int32_t)np;
    } else if (d->cd == CD_TC8 || d->cd == CD_TCA8 || d->cd == CD_TC16 || d->cd == CD_TCA16) {
        /* ignored */
    } else {
        return E_PlteColorTypeMismatch;
    }
    return pd_verify(d);
}

/* parseTrns, :547-602 */
static int pd_trns(zo_pdec *d, uint32_t length)
{
    uint8_t b[256];
    switch (d->cd) {
    case CD_G1: case CD_G2: case CD_G4: case CD_G8: case CD_G16:
        if (length != 2) return E_BadTrnsLength;
        TRY(pd_read_crc(d, b, length));
        memcpy(d->transparent, b, 2);
        d->transparent[1] = (uint8_t)(d->transparent[1] *
                                      (d->cd == CD_G1 ? 0xff : d->cd == CD_G2 ? 0x55 : d->cd == CD_G4 ? 0x11 : 1));
        d->use_transparent = 1;
        break;
    case CD_TC8: case CD_TC16:
        if (length != 6) return E_BadTrnsLength;
        TRY(pd_read_crc(d, b, length));
        memcpy(d->transparent, b, 6);
        d->use_transparent = 1;
        break;
    case CD_P1: case CD_P2: case CD_P4: case CD_P8:
        if (length > 256) return E_BadTrnsLength;
        TRY(pd_read_crc(d, b, length));
        if (d->palette_len < (int32_t)length) d->palette_len = (int32_t)length;
        for (uint32_t i = 0; i < length; i++) {
            d->palette[5 * i + 3] = b[i];
            d->palette[5 * i + 4] = 1; /* .nrgba */
        }
        break;
    default:
        return E_TrnsColorTypeMismatch;
    }
    return pd_verify(d);
}

static int bits_per_pixel(int cd)
{
    switch (cd) {
    case CD_G1: case CD_P1: return 1;
    case CD_G2: case CD_P2: return 2;
    case CD_G4: case CD_P4: return 4;
    case CD_G8: case CD_P8: return 8;
    case CD_GA8: return 16;
    case CD_TC8: return 24;
    case CD_TCA8: return 32;
    case CD_G16: return 16;
    case CD_GA16: return 32;
    case CD_TC16: return 48;
    case CD_TCA16: return 64;
    }
    return 0;
}

/* the image type readImagePass allocates, :712-775 */
static int img_kind_for(const zo_pdec *d, size_t *bpp_out)
{
    switch (d->cd) {
    case CD_G1: case CD_G2: case CD_G4: case CD_G8:
        *bpp_out = d->use_transparent ? 4 : 1;
        return d->use_transparent ? ZO_NRGBA : ZO_GRAY;
    case CD_GA8: *bpp_out = 4; return ZO_NRGBA;
    case CD_GA16: *bpp_out = 8; return ZO_NRGBA64;
    case CD_G16:
        *bpp_out = d->use_transparent ? 8 : 2;
        return d->use_transparent ? ZO_NRGBA64 : ZO_GRAY16;
    case CD_TC8:
        *bpp_out = 4;
        return d->use_transparent ? ZO_NRGBA : ZO_RGBA;
    case CD_TC16:
        *bpp_out = 8;
        return d->use_transparent ? ZO_NRGBA64 : ZO_RGBA64;
    case CD_TCA8: *bpp_out = 4; return ZO_NRGBA;
    case CD_TCA16: *bpp_out = 8; return ZO_NRGBA64;
    default: *bpp_out = 1; return ZO_PALETTED;
    }
}

static void put16(uint8_t *p, uint32_t v)
{
    p[0] = (uint8_t)(v >> 8);
    p[1] = (uint8_t)(v & 0xff);
}

/* pixel store for one row, readImagePass :845-1140. pal_len is the pass
 * image's palette length (grown on out-of-range indices). */
static void store_row(zo_pdec *d, const uint8_t *c, uint32_t width, uint8_t *dst,
                      int32_t *pal_len)
{
    uint8_t ty8 = d->transparent[1];
    switch (d->cd) {
    case CD_G1: case CD_G2: case CD_G4: {
        int bits = d->cd == CD_G1 ? 1 : d->cd == CD_G2 ? 2 : 4;
        int mul = d->cd == CD_G1 ? 0xff : d->cd == CD_G2 ? 0x55 : 0x11;
        int per = 8 / bits;
        for (uint32_t x = 0; x < width; x++) {
            uint8_t byte = c[x / per];
            int shift = 8 - bits * (int)(x % per + 1);
            uint8_t v = (uint8_t)(((byte >> shift) & ((1 << bits) - 1)) * mul);
            if (d->use_transparent) {
                uint8_t *o = dst + 4 * x;
                o[0] = o[1] = o[2] = v;
                o[3] = v == ty8 ? 0x00 : 0xff;
            } else {
                dst[x] = v;
            }
        }
        break;
    }
    case CD_G8:
        for (uint32_t x = 0; x < width; x++) {
            if (d->use_transparent) {
                uint8_t *o = dst + 4 * x;
                o[0] = o[1] = o[2] = c[x];
                o[3] = c[x] == ty8 ? 0x00 : 0xff;
            } else {
                dst[x] = c[x];
            }
        }
        break;
    case CD_G16: {
        uint32_t ty = (uint32_t)d->transparent[0] << 8 | d->transparent[1];
        for (uint32_t x = 0; x < width; x++) {
            uint32_t v = (uint32_t)c[2 * x] << 8 | c[2 * x + 1];
            if (d->use_transparent) {
                uint8_t *o = dst + 8 * x;
                put16(o, v);
                put16(o + 2, v);
                put16(o + 4, v);
                put16(o + 6, v == ty ? 0 : 0xffff);
            } else {
                put16(dst + 2 * x, v);
            }
        }
        break;
    }
    case CD_TC8:
        for (uint32_t x = 0; x < width; x++) {
            uint8_t *o = dst + 4 * x;
            uint8_t r = c[3 * x], g = c[3 * x + 1], b = c[3 * x + 2];
            o[0] = r;
            o[1] = g;
            o[2] = b;
            if (d->use_transparent)
                o[3] = (r == d->transparent[1] && g == d->transparent[3] && b == d->transparent[5]) ? 0x00 : 0xff;
            else
                o[3] = 0xff;
        }
        break;
    case CD_TC16: {
        uint32_t tr = (uint32_t)d->transparent[0] << 8 | d->transparent[1];
        uint32_t tg = (uint32_t)d->transparent[2] << 8 | d->transparent[3];
        uint32_t tb = (uint32_t)d->transparent[4] << 8 | d->transparent[5];
        for (uint32_t x = 0; x < width; x++) {
            const uint8_t *s = c + 6 * x;
            uint32_t r = (uint32_t)s[0] << 8 | s[1], g = (uint32_t)s[2] << 8 | s[3],
                     b = (uint32_t)s[4] << 8 | s[5];
            uint8_t *o = dst + 8 * x;
            put16(o, r);
            put16(o + 2, g);
            put16(o + 4, b);
            uint32_t a = 0xffff;
            if (d->use_transparent && r == tr && g == tg && b == tb) a = 0;
            put16(o + 6, a);
        }
        break;
    }
    case CD_GA8:
        for (uint32_t x = 0; x < width; x++) {
            uint8_t *o = dst + 4 * x;
            o[0] = o[1] = o[2] = c[2 * x];
            o[3] = c[2 * x + 1];
        }
        break;
    case CD_GA16:
        for (uint32_t x = 0; x < width; x++) {
            uint8_t *o = dst + 8 * x;
            for (int k = 0; k < 3; k++) {
                o[2 * k] = c[4 * x];
                o[2 * k + 1] = c[4 * x + 1];
            }
            o[6] = c[4 * x + 2];
            o[7] = c[4 * x + 3];
        }
        break;
    case CD_TCA8: memcpy(dst, c, (size_t)width * 4); break;
    case CD_TCA16: memcpy(dst, c, (size_t)width * 8); break;
    case CD_P1: case CD_P2: case CD_P4: case CD_P8: {
        int bits = d->cd == CD_P1 ? 1 : d->cd == CD_P2 ? 2 : d->cd == CD_P4 ? 4 : 8;
        int per = 8 / bits;
        for (uint32_t x = 0; x < width; x++) {
            uint8_t idx;
            if (bits == 8) idx = c[x];
            else {
                int shift = 8 - bits * (int)(x % per + 1);
                idx = (uint8_t)((c[x / per] >> shift) & ((1 << bits) - 1));
            }
            if (*pal_len <= idx) *pal_len = idx + 1; /* implicit palette growth */
            dst[x] = idx;
        }
        break;
    }
    }
}

/* readImagePass, :649-1149.  Writes a pass image of (pw x ph) pixels. */
static int pd_read_pass(zo_pdec *d, const uint8_t *data, size_t data_len, int data_err,
                        size_t *pos, uint32_t pw, uint32_t ph, uint8_t *dst, size_t dst_stride,
                        int32_t *pal_len)
{
    uint32_t bits = (uint32_t)bits_per_pixel(d->cd);
    size_t bpp = (bits + 7) / 8;
    size_t row_size = 1 + ((size_t)bits * pw + 7) / 8;
    uint8_t *cr = (uint8_t *)calloc(row_size, 1), *pr = (uint8_t *)calloc(row_size, 1);
    if (!cr || !pr) {
        free(cr);
        free(pr);
        return E_OutOfMemory;
    }
    int e = 0;
    for (uint32_t y = 0; y < ph; y++) {
        if (data_len - *pos < row_size) {
            e = data_err ? E_ReadFailed : E_EndOfStream;
            break;
        }
        memcpy(cr, data + *pos, row_size);
        *pos += row_size;
        e = unfilter_row(cr[0], cr + 1, pr + 1, row_size - 1, bpp);
        if (e) break;
        store_row(d, cr + 1, pw, dst + (size_t)y * dst_stride, pal_len);
        uint8_t *t = pr;
        pr = cr;
        cr = t;
    }
    free(cr);
    free(pr);
    return e;
}

/* inflate the concatenated IDAT payload (std.compress.flate .zlib, :516-518) */
static int inflate_all(const uint8_t *in, size_t in_len, uint8_t **out, size_t *out_len,
                       int *data_err)
{
    z_stream zs;
    memset(&zs, 0, sizeof(zs));
    if (inflateInit(&zs) != Z_OK) return E_OutOfMemory;
    size_t cap = in_len * 4 + 1024, len = 0;
    uint8_t *buf = (uint8_t *)malloc(cap);
    if (!buf) {
        inflateEnd(&zs);
        return E_OutOfMemory;
    }
    zs.next_in = (Bytef *)in;
    zs.avail_in = (uInt)in_len;
    *data_err = 0;
    for (;;) {
        if (len == cap) {
            cap *= 2;
            uint8_t *nb = (uint8_t *)realloc(buf, cap);
            if (!nb) {
                free(buf);
                inflateEnd(&zs);
                return E_OutOfMemory;
            }
            buf = nb;
        }
        zs.next_out = buf + len;
        zs.avail_out = (uInt)(cap - len);
        int r = inflate(&zs, Z_NO_FLUSH);
        len = cap - zs.avail_out;
        if (r == Z_STREAM_END) break;
        if (r == Z_OK) continue;
        if (r == Z_BUF_ERROR && zs.avail_out == 0) continue;
        if (r == Z_BUF_ERROR) break; /* input exhausted: short stream */
        *data_err = 1;
        break;
    }
    inflateEnd(&zs);
    *out = buf;
    *out_len = len;
    return 0;
}

static int pd_alloc_image(zo_pdec *d, zo_image *m, uint32_t w, uint32_t h)
{
    size_t bpp;
    memset(m, 0, sizeof(*m));
    m->kind = img_kind_for(d, &bpp);
    m->max_x = (int32_t)w;
    m->max_y = (int32_t)h;
    m->stride = (size_t)w * bpp;
    m->pixels_len = m->stride * h;
    m->pixels = (uint8_t *)calloc(m->pixels_len ? m->pixels_len : 1, 1);
    if (!m->pixels) return E_OutOfMemory;
    if (m->kind == ZO_PALETTED) {
        m->palette = (uint8_t *)calloc(256, 5);
        if (!m->palette) return E_OutOfMemory;
        if (d->palette) memcpy(m->palette, d->palette, 256 * 5);
        else for (int i = 0; i < 256; i++) m->palette[5 * i + 3] = 0xff;
        m->palette_len = d->palette_len;
    }
    return 0;
}

/* parseIdat, :404-545 */
static int pd_idat(zo_pdec *d, uint32_t first_len)
{
    size_t cap = (size_t)first_len + 4096, len = 0;
    uint8_t *all = (uint8_t *)malloc(cap);
    if (!all) return E_OutOfMemory;
    int e = 0;
#define APPEND(p, n)                                                           \
    do {                                                                       \
        if (len + (n) > cap) {                                                 \
            while (len + (n) > cap) cap *= 2;                                  \
            uint8_t *nb = (uint8_t *)realloc(all, cap);                        \
            if (!nb) { e = E_OutOfMemory; goto out; }                          \
            all = nb;                                                          \
        }                                                                      \
        memcpy(all + len, (p), (n));                                           \
        len += (n);                                                            \
    } while (0)
    {
        uint8_t scratch[768];
        uint32_t rem = first_len;
        while (rem > 0) {
            uint32_t k = rem < sizeof(scratch) ? rem : (uint32_t)sizeof(scratch);
            if ((e = pd_read_crc(d, scratch, k))) goto out;
            APPEND(scratch, k);
            rem -= k;
        }
        if ((e = pd_verify(d))) goto out;
        for (;;) {
            uint8_t hb[8];
            if (pd_read(d, hb, 8)) break; /* :435-438 */
            if (memcmp(hb + 4, "IDAT", 4) != 0) {
                d->stage = 4;
                d->crc = (uint32_t)crc32(0, hb + 4, 4);
                if (memcmp(hb + 4, "IEND", 4) == 0) {
                    d->stage = 5;
                    if ((e = pd_verify(d))) goto out;
                } else {
                    if ((e = pd_skip(d, be32(hb)))) goto out;
                    if ((e = pd_verify(d))) goto out;
                }
                break;
            }
            uint32_t cl = be32(hb);
            d->crc = (uint32_t)crc32(0, hb + 4, 4);
            rem = cl;
            while (rem > 0) {
                uint32_t k = rem < sizeof(scratch) ? rem : (uint32_t)sizeof(scratch);
                if ((e = pd_read_crc(d, scratch, k))) goto out;
                APPEND(scratch, k);
                rem -= k;
            }
            if ((e = pd_verify(d))) goto out;
        }
    }
    if (len == 0) {
        e = E_EmptyIdatData;
        goto out;
    }
    {
        uint8_t *data = NULL;
        size_t dlen = 0;
        int derr = 0;
        if ((e = inflate_all(all, len, &data, &dlen, &derr))) goto out;
        const double t_pass = zo_now();
        size_t pos = 0;
        if (d->have_img) zo_image_free(&d->img);
        if ((e = pd_alloc_image(d, &d->img, d->width, d->height))) {
            free(data);
            goto out;
        }
        d->have_img = 1;
        if (d->interlace == 0) {
            e = pd_read_pass(d, data, dlen, derr, &pos, d->width, d->height, d->img.pixels,
                             d->img.stride, &d->img.palette_len);
        } else {
            size_t bpp = d->img.stride / d->width;
            for (int p = 0; p < 7 && !e; p++) {
                uint32_t xo = ADAM7[p][0], yo = ADAM7[p][1], xf = ADAM7[p][2], yf = ADAM7[p][3];
                /* saturating pass dims, :665-666 */
                uint32_t pw = d->width > xo ? d->width - xo : 0;
                pw = (pw + xf - 1) / xf;
                uint32_t ph = d->height > yo ? d->height - yo : 0;
                ph = (ph + yf - 1) / yf;
                if (pw == 0 || ph == 0) continue; /* EmptyPass */
                zo_image pass;
                if ((e = pd_alloc_image(d, &pass, pw, ph))) break;
                e = pd_read_pass(d, data, dlen, derr, &pos, pw, ph, pass.pixels, pass.stride,
                                 &pass.palette_len);
                if (!e) {
                    /* mergePassInto, :1289-1373 */
                    if (d->img.kind == ZO_PALETTED && d->img.palette_len < pass.palette_len)
                        d->img.palette_len = pass.palette_len;
                    size_t s = 0;
                    for (uint32_t y = 0; y < ph; y++) {
                        size_t dbase = (size_t)(y * yf + yo) * d->img.stride + (size_t)xo * bpp;
                        for (uint32_t x = 0; x < pw; x++) {
                            memcpy(d->img.pixels + dbase + (size_t)x * xf * bpp, pass.pixels + s, bpp);
                            s += bpp;
                        }
                    }
                }
                zo_image_free(&pass);
            }
        }
        free(data);
        zo_png_unfilter_s += zo_now() - t_pass;
    }
out:
    free(all);
    return e;
#undef APPEND
}

/* parseChunk, :231-324 */
static int pd_chunk(zo_pdec *d)
{
    uint8_t hb[8];
    TRY(pd_read(d, hb, 8));
    uint32_t length = be32(hb);
    const uint8_t *t = hb + 4;
    d->crc = (uint32_t)crc32(0, t, 4);
    if (!memcmp(t, "IHDR", 4)) {
        if (d->stage != 0) return E_ChunkOrderInHeaderError;
        d->stage = 1;
        return pd_ihdr(d, length);
    }
    if (!memcmp(t, "PLTE", 4)) {
        if (d->stage != 1) return E_ChunkOrderPlteError;
        d->stage = 2;
        return pd_plte(d, length);
    }
    if (!memcmp(t, "IDAT", 4)) {
        if (d->stage < 1 || d->stage > 4 || (d->stage == 1 && cd_paletted(d->cd)))
            return E_ChunkOrderIdatError;
        if (d->stage != 4) d->stage = 4;
        return pd_idat(d, length);
    }
    if (!memcmp(t, "tRNS", 4)) {
        if (cd_paletted(d->cd)) {
            if (d->stage != 2) return E_ChunkOrderTrns1Error;
        } else if (d->cd == CD_TC8 || d->cd == CD_TC16) {
            if (d->stage != 1 && d->stage != 2) return E_ChunkOrderTrns2Error;
        } else {
            if (d->stage != 1) return E_ChunkOrderTrns3Error;
        }
        d->stage = 3;
        return pd_trns(d, length);
    }
    if (!memcmp(t, "IEND", 4)) {
        if (d->stage != 4) return E_ChunkOrderIendError;
        d->stage = 5;
        return pd_verify(d);
    }
    TRY(pd_skip(d, length));
    return pd_verify(d);
}

/* png Decoder.decode, :143-221 */
int zo_png_decode(const uint8_t *buf, size_t len, zo_image *out)
{
    memset(out, 0, sizeof(*out));
    zo_pdec d;
    memset(&d, 0, sizeof(d));
    d.src = buf;
    d.len = len;
    int e = 0;
    uint8_t sig[8];
    static const uint8_t PNG_SIG[8] = {0x89, 'P', 'N', 'G', '\r', '\n', 0x1a, '\n'};
    if ((e = pd_read(&d, sig, 8))) goto fail;
    if (memcmp(sig, PNG_SIG, 8) != 0) {
        e = E_InvalidPngHeader;
        goto fail;
    }
    while (d.stage != 5)
        if ((e = pd_chunk(&d))) goto fail;
    if (!d.have_img || d.img.max_x == 0 || d.img.max_y == 0) {
        e = E_InvalidImageDimensions;
        goto fail;
    }
    *out = d.img;
    free(d.palette);
    return 0;
fail:
    if (d.have_img) zo_image_free(&d.img);
    free(d.palette);
    return e;
}

/* ======================================================================== */
/* BMP                                                                       */
/* ======================================================================== */

static uint32_t le32(const uint8_t *b) { return (uint32_t)b[0] | (uint32_t)b[1] << 8 | (uint32_t)b[2] << 16 | (uint32_t)b[3] << 24; }
static uint32_t le16(const uint8_t *b) { return (uint32_t)b[0] | (uint32_t)b[1] << 8; }

/* bmp Decoder.decode (src/bmp/decoder.zig:25-40), readHeader (:42-158),
 * decodePaletted (:160-229), decodeRGB (:231-270), decodeNRGBA (:272-307).
 * The reader is a fixed buffer: every short read is EndOfStream. */
int zo_bmp_decode(const uint8_t *buf, size_t len, zo_image *out)
{
    memset(out, 0, sizeof(*out));
    size_t pos = 0;
#define BMP_READ(n)                                                            \
    do {                                                                       \
        if (len - pos < (size_t)(n)) return E_EndOfStream;                     \
    } while (0)
    BMP_READ(18);
    const uint8_t *b = buf;
    if (!(b[0] == 'B' && b[1] == 'M')) return E_InvalidSignature;
    const uint32_t pixel_off = le32(b + 10), info_len = le32(b + 14);
    if (info_len != 40 && info_len != 108 && info_len != 124) return E_UnsupportedHeader;
    pos = 18;
    BMP_READ(14 + info_len - 18);
    pos = 14 + info_len;
    const int32_t w = (int32_t)le32(b + 18);
    int32_t hh = (int32_t)le32(b + 22);
    int top_down = 0;
    if (hh < 0) {
        if (hh == INT32_MIN) return E_UnsupportedDimensions; /* Zig would trap on the negation */
        hh = -hh;
        top_down = 1;
    }
    if (w < 0) return E_UnsupportedDimensions;
    const uint32_t planes = le16(b + 26), bpp = le16(b + 28);
    uint32_t compression = le32(b + 30);
    if (compression == 3 && info_len > 40) { /* :77-86 */
        if (le32(b + 54) == 0xff0000 && le32(b + 58) == 0x00ff00 && le32(b + 62) == 0x0000ff &&
            le32(b + 66) == 0xff000000u)
            compression = 0;
    }
    if (planes != 1 || compression != 0) return E_UnsupportedCompression;
    const uint32_t width = (uint32_t)w, height = (uint32_t)hh;
    const int allow_alpha = info_len > 40;
    uint32_t ncol = 0;
    uint8_t pal[256 * 5];
    if (bpp == 1 || bpp == 2 || bpp == 4 || bpp == 8) {
        ncol = le32(b + 46);
        if (ncol == 0) ncol = 1u << bpp;
        else if (ncol > (1u << bpp)) return E_UnsupportedPaletteSize;
        if (pixel_off != 14 + info_len + ncol * 4) return E_UnsupportedColorOffset;
        BMP_READ((size_t)ncol * 4);
        for (uint32_t i = 0; i < ncol; i++) { /* B,G,R,pad -> .rgba, A=0xff */
            pal[5 * i + 0] = b[pos + 4 * i + 2];
            pal[5 * i + 1] = b[pos + 4 * i + 1];
            pal[5 * i + 2] = b[pos + 4 * i + 0];
            pal[5 * i + 3] = 0xff;
            pal[5 * i + 4] = 0;
        }
        pos += (size_t)ncol * 4;
    } else if (bpp == 24 || bpp == 32) {
        if (pixel_off != 14 + info_len) return E_UnsupportedColorOffset;
    } else {
        return E_UnsupportedBPP;
    }

    if (ncol) {
        /* Paletted; an empty image has rect (0,0,0,0) (:163-172) */
        const int empty = width == 0 || height == 0;
        out->kind = ZO_PALETTED;
        out->max_x = empty ? 0 : (int32_t)width;
        out->max_y = empty ? 0 : (int32_t)height;
        out->stride = empty ? 0 : width;
        out->pixels_len = out->stride * (empty ? 0 : height);
        out->palette = (uint8_t *)calloc(256, 5); /* oracle images carry 256 entries */
        out->pixels = (uint8_t *)calloc(out->pixels_len ? out->pixels_len : 1, 1);
        if (!out->palette || !out->pixels) {
            zo_image_free(out);
            return E_OutOfMemory;
        }
        memcpy(out->palette, pal, ncol * 5);
        out->palette_len = (int32_t)ncol;
        if (empty) return 0;
        const uint32_t ppb = 8 / bpp, mask = (1u << bpp) - 1;
        const size_t row = ((((size_t)width + ppb - 1) / ppb) + 3) & ~(size_t)3;
        for (uint32_t r = 0; r < height; r++) {
            if (len - pos < row) {
                zo_image_free(out);
                return E_EndOfStream;
            }
            const uint32_t y = top_down ? r : height - 1 - r;
            uint8_t *p = out->pixels + (size_t)y * out->stride;
            size_t bi = 0;
            int bit = 8;
            for (uint32_t x = 0; x < width; x++) {
                bit -= (int)bpp;
                p[x] = (uint8_t)((buf[pos + bi] >> bit) & mask);
                if (bit == 0) {
                    bi++;
                    bit = 8;
                }
            }
            pos += row;
        }
        return 0;
    }
    out->kind = bpp == 24 ? ZO_RGBA : ZO_NRGBA;
    out->max_x = (int32_t)width;
    out->max_y = (int32_t)height;
    out->stride = (size_t)width * 4;
    out->pixels_len = out->stride * height;
    out->pixels = (uint8_t *)calloc(out->pixels_len ? out->pixels_len : 1, 1);
    if (!out->pixels) return E_OutOfMemory;
    if (width == 0 || height == 0) return 0;
    const size_t row = bpp == 24 ? ((size_t)width * 3 + 3) & ~(size_t)3 : (size_t)width * 4;
    for (uint32_t r = 0; r < height; r++) {
        if (len - pos < row) {
            zo_image_free(out);
            return E_EndOfStream;
        }
        const uint32_t y = top_down ? r : height - 1 - r;
        uint8_t *p = out->pixels + (size_t)y * out->stride;
        const uint8_t *s = buf + pos;
        for (uint32_t x = 0; x < width; x++) {
            if (bpp == 24) {
                p[4 * x + 0] = s[3 * x + 2];
                p[4 * x + 1] = s[3 * x + 1];
                p[4 * x + 2] = s[3 * x + 0];
                p[4 * x + 3] = 0xff;
            } else {
                p[4 * x + 0] = s[4 * x + 2];
                p[4 * x + 1] = s[4 * x + 1];
                p[4 * x + 2] = s[4 * x + 0];
                p[4 * x + 3] = allow_alpha ? s[4 * x + 3] : 0xff;
            }
        }
        pos += row;
    }
    return 0;
#undef BMP_READ
}

/* ======================================================================== */
/* QOI                                                                       */
/* ======================================================================== */

#define QOI_PIXELS_MAX 400000000u
static unsigned qoi_hash(const uint8_t *px) { return (px[0] * 3u + px[1] * 5u + px[2] * 7u + px[3] * 11u) & 63u; }

/* qoi decodeFromBuffer, src/qoi/decoder.zig:28-130 -> .RGBA image.
 * DIFF/LUMA steps that leave 0..255 trap in the reference's @intCast
 * (:97-114, safety-checked builds); here they wrap mod 256 as the QOI
 * specification (and a ReleaseFast build's truncation) has them.  The
 * reference's own encoder never emits such steps (encoder.zig:97-101). */
int zo_qoi_decode(const uint8_t *data, size_t len, zo_image *out)
{
    memset(out, 0, sizeof(*out));
    if (len < 14 + 8) return E_InvalidQoiData;
    if (be32(data) != 0x716F6966u) return E_InvalidQoiHeader;
    const uint32_t width = be32(data + 4), height = be32(data + 8);
    const uint8_t channels = data[12], colorspace = data[13];
    if (width == 0 || height == 0 || (channels != 3 && channels != 4) || colorspace > 1 ||
        height >= QOI_PIXELS_MAX / width)
        return E_InvalidQoiHeader;
    const size_t n = (size_t)width * height, chunks_len = len - 8;
    out->kind = ZO_RGBA;
    out->max_x = (int32_t)width;
    out->max_y = (int32_t)height;
    out->stride = (size_t)width * 4;
    out->pixels_len = n * 4;
    out->pixels = (uint8_t *)malloc(n * 4);
    if (!out->pixels) return E_OutOfMemory;
    uint8_t index[64][4];
    memset(index, 0, sizeof(index));
    uint8_t px[4] = {0, 0, 0, 255};
    size_t p = 14, run = 0;
    for (size_t i = 0; i < n; i++) {
        if (run > 0) {
            run--;
        } else if (p < chunks_len) {
            /* payload bytes are read without the chunks_len check (:71-82):
             * within the 8 padding bytes they are read as they are, past the
             * end of the buffer the reference's bounds check panics */
            const uint8_t b1 = data[p++];
            const size_t need = b1 == 0xfe ? 3 : b1 == 0xff ? 4 : (b1 & 0xc0) == 0x80 ? 1 : 0;
            if (p + need > len) {
                zo_image_free(out);
                return E_Panic;
            }
            if (b1 == 0xfe) {
                px[0] = data[p]; px[1] = data[p + 1]; px[2] = data[p + 2];
                p += 3;
            } else if (b1 == 0xff) {
                px[0] = data[p]; px[1] = data[p + 1]; px[2] = data[p + 2]; px[3] = data[p + 3];
                p += 4;
            } else if ((b1 & 0xc0) == 0x00) {
                memcpy(px, index[b1 & 0x3f], 4);
            } else if ((b1 & 0xc0) == 0x40) {
                px[0] = (uint8_t)(px[0] + ((b1 >> 4) & 3) - 2);
                px[1] = (uint8_t)(px[1] + ((b1 >> 2) & 3) - 2);
                px[2] = (uint8_t)(px[2] + (b1 & 3) - 2);
            } else if ((b1 & 0xc0) == 0x80) {
                const uint8_t b2 = data[p];
                p += 1;
                const int dg = (b1 & 0x3f) - 32;
                px[0] = (uint8_t)(px[0] + dg + ((b2 >> 4) & 0xf) - 8);
                px[1] = (uint8_t)(px[1] + dg);
                px[2] = (uint8_t)(px[2] + dg + (b2 & 0xf) - 8);
            } else {
                run = b1 & 0x3f;
            }
            memcpy(index[qoi_hash(px)], px, 4);
        }
        memcpy(out->pixels + 4 * i, px, 4);
    }
    return 0;
}

/* qoi encode, src/qoi/encoder.zig:29-132.  *out is malloc'd; returns 0 or
 * InvalidQoiHeader. */
int zo_qoi_encode(const uint8_t *pixels, uint32_t width, uint32_t height, uint8_t channels, uint8_t colorspace,
                  uint8_t **out, size_t *out_len)
{
    *out = NULL;
    *out_len = 0;
    if (width == 0 || height == 0 || channels < 3 || channels > 4 || colorspace > 1 ||
        height >= QOI_PIXELS_MAX / width)
        return E_InvalidQoiHeader;
    const size_t px_len = (size_t)width * height * channels;
    uint8_t *o = (uint8_t *)malloc((size_t)width * height * (channels + 1) + 14 + 8);
    if (!o) return E_OutOfMemory;
    size_t n = 0;
    const uint32_t hdr[3] = {0x716F6966u, width, height};
    for (int k = 0; k < 3; k++)
        for (int s = 24; s >= 0; s -= 8) o[n++] = (uint8_t)(hdr[k] >> s);
    o[n++] = channels;
    o[n++] = colorspace;
    uint8_t index[64][4];
    memset(index, 0, sizeof(index));
    uint8_t prev[4] = {0, 0, 0, 255}, px[4] = {0, 0, 0, 255};
    uint32_t run = 0;
    for (size_t i = 0; i < px_len; i += channels) {
        px[0] = pixels[i];
        px[1] = pixels[i + 1];
        px[2] = pixels[i + 2];
        if (channels == 4) px[3] = pixels[i + 3];
        if (!memcmp(px, prev, 4)) {
            run++;
            if (run == 62 || i + channels == px_len) {
                o[n++] = (uint8_t)(0xc0 | (run - 1));
                run = 0;
            }
        } else {
            if (run > 0) {
                o[n++] = (uint8_t)(0xc0 | (run - 1));
                run = 0;
            }
            const unsigned h = qoi_hash(px);
            if (!memcmp(index[h], px, 4)) {
                o[n++] = (uint8_t)h;
            } else {
                memcpy(index[h], px, 4);
                if (px[3] == prev[3]) {
                    const int vr = px[0] - prev[0], vg = px[1] - prev[1], vb = px[2] - prev[2];
                    const int vgr = vr - vg, vgb = vb - vg;
                    if (vr > -3 && vr < 2 && vg > -3 && vg < 2 && vb > -3 && vb < 2) {
                        o[n++] = (uint8_t)(0x40 | (vr + 2) << 4 | (vg + 2) << 2 | (vb + 2));
                    } else if (vgr > -9 && vgr < 8 && vg > -33 && vg < 32 && vgb > -9 && vgb < 8) {
                        o[n++] = (uint8_t)(0x80 | (vg + 32));
                        o[n++] = (uint8_t)((vgr + 8) << 4 | (vgb + 8));
                    } else {
                        o[n++] = 0xfe;
                        o[n++] = px[0];
                        o[n++] = px[1];
                        o[n++] = px[2];
                    }
                } else {
                    o[n++] = 0xff;
                    memcpy(o + n, px, 4);
                    n += 4;
                }
            }
        }
        memcpy(prev, px, 4);
    }
    static const uint8_t pad[8] = {0, 0, 0, 0, 0, 0, 0, 1};
    memcpy(o + n, pad, 8);
    n += 8;
    *out = o;
    *out_len = n;
    return 0;
}
