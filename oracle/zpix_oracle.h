/*
 * zpix_oracle.h — CPU restatement of braheezy/zpix's decode arithmetic.
 *
 * TEST INFRASTRUCTURE ONLY.  This oracle is the parity checker for the
 * MI355X decode path in zpix_amd/.  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load it.  The product library never links
 * or calls it.
 *
 * Parity pins:
 *   - PNG: the 35 PngSuite .sng goldens (reference src/png/decoder_test.zig:8-129)
 *     and the BMP parity pairs (src/bmp/decoder_test.zig:24-61), bit-exact.
 *   - JPEG: baseline == progressive for the 10 pairs
 *     (src/jpeg/decoder.zig:1843-1920) and the error cases :1942-2279.
 *     Absolute JPEG pixels are not pinned by any reference golden; they follow
 *     the restated integer arithmetic (idct.zig:77-201, decoder.zig:1553-1634,
 *     color.zig:90-113).
 */
#ifndef ZPIX_ORACLE_H
#define ZPIX_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* image.Image tags, src/image/image.zig:24-34 */
enum zo_kind {
    ZO_GRAY = 0,
    ZO_GRAY16 = 1,
    ZO_YCBCR = 2,
    ZO_RGBA = 3,
    ZO_RGBA64 = 4,
    ZO_NRGBA = 5,
    ZO_NRGBA64 = 6,
    ZO_CMYK = 7,
    ZO_PALETTED = 8,
};

/* image.YCbCrSubsample, src/image/image.zig:465-472 */
enum zo_subsample {
    ZO_444 = 0,
    ZO_422 = 1,
    ZO_420 = 2,
    ZO_440 = 3,
    ZO_411 = 4,
    ZO_410 = 5,
};

typedef struct zo_image {
    int32_t kind;
    int32_t min_x, min_y, max_x, max_y; /* rect */
    uint8_t *pixels;                    /* owning buffer */
    size_t pixels_len;
    size_t stride;                      /* all kinds except YCbCr */
    /* YCbCr only: planes are views into pixels */
    size_t y_off, cb_off, cr_off;
    size_t y_stride, c_stride;
    int32_t subsample;
    /* Paletted only: palette_len entries of {r,g,b,a,tag} (tag 0=.rgba, 1=.nrgba) */
    uint8_t *palette;
    int32_t palette_len;
} zo_image;

/* Error codes: 0 = ok, otherwise an index into zo_error_name(). */
const char *zo_error_name(int code);

/* jpeg.decode (src/jpeg/decoder.zig:155-176) over an in-memory buffer. */
int zo_jpeg_decode(const uint8_t *buf, size_t len, zo_image *out);
/* png.decode (src/png/decoder.zig:143-221) over an in-memory buffer. */
int zo_png_decode(const uint8_t *buf, size_t len, zo_image *out);
/* bmp.decode (src/bmp/decoder.zig:25-307): .Paletted, .RGBA (24 bpp) or
 * .NRGBA (32 bpp). */
int zo_bmp_decode(const uint8_t *buf, size_t len, zo_image *out);
/* qoi.decode (src/qoi/decoder.zig:28-130): .RGBA. */
int zo_qoi_decode(const uint8_t *buf, size_t len, zo_image *out);
/* qoi.encode (src/qoi/encoder.zig:29-132): *out malloc'd, free() it. */
int zo_qoi_encode(const uint8_t *pixels, uint32_t width, uint32_t height, uint8_t channels,
                  uint8_t colorspace, uint8_t **out, size_t *out_len);
/* Image.rgbaPixels (src/image/image.zig:103-130): out has 4*dX*dY bytes. */
int zo_rgba_pixels(const zo_image *img, uint8_t *out);
/* Image.at(x,y).toRGBA() (16-bit premultiplied), src/image/image.zig:54-66 */
void zo_at_rgba16(const zo_image *img, int32_t x, int32_t y, uint32_t out[4]);
void zo_image_free(zo_image *img);

/* ---- stage-level hooks used by kernel parity tests ---- */

/* idct.transform (src/jpeg/idct.zig:77-201), in place on 64 i32. */
void zo_idct(int32_t *block);

/*
 * reconstructBlock over whole component grids (decoder.zig:1553-1634) for a
 * frame described by the arguments, writing planes with the reference layout
 * of makeImg (decoder.zig:1708-1783).
 *   coeffs[c]: grid of (mxx*h[c]) x (myy*v[c]) blocks, 64 i32 natural order,
 *              index by*mxx*h[c]+bx (decoder.zig:1341).
 *   qt_zigzag[c]: the quant table the component uses, zig-zag order.
 *   progressive: use the in-bounds rule of reconstructProgressiveImage
 *                (decoder.zig:1636-1661) instead of all blocks.
 *   planes[c], strides[c]: destination planes.
 */
void zo_jpeg_reconstruct_grids(int32_t n_comp, uint32_t width, uint32_t height,
                               const int32_t *h, const int32_t *v,
                               int32_t mxx, int32_t myy,
                               int32_t *const *coeffs,
                               const int32_t *const *qt_zigzag,
                               int32_t progressive,
                               uint8_t *const *planes, const size_t *strides);

/*
 * Entropy-decode a JPEG and return its coefficient grids instead of pixels
 * (the "accumulate coefficients" form of processSos, decoder.zig:1340-1345).
 * Caller frees with zo_jpeg_coeffs_free.
 */
typedef struct zo_jpeg_coeffs {
    uint32_t width, height;
    int32_t n_comp;
    int32_t h[4], v[4], tq[4];
    int32_t mxx, myy;
    int32_t progressive;
    int32_t jfif, adobe_valid, adobe_transform;
    int32_t comp_id[4];
    int32_t *grid[4];        /* NULL when the component got no coefficients */
    int32_t quant[4][64];    /* zig-zag order, as decoder.quant */
} zo_jpeg_coeffs;

int zo_jpeg_decode_coeffs(const uint8_t *buf, size_t len, zo_jpeg_coeffs *out);
void zo_jpeg_coeffs_free(zo_jpeg_coeffs *c);

/*
 * PNG filter reconstruction over a whole filtered stream (decoder.zig:798-842,
 * 1152-1182): rows of (1 + row_bytes) bytes, bytes_per_pixel as :782.
 * Writes the unfiltered row bytes (row_bytes per row) to out.
 * Returns 0 or the InvalidFilterType error code.
 */
int zo_png_unfilter(const uint8_t *filtered, uint32_t rows, uint32_t row_bytes,
                    uint32_t bytes_per_pixel, uint8_t *out);

/* CPU-baseline stage clock: seconds the calling thread spent in PNG filter
 * reconstruction + pixel store (+ Adam7 merge) since the last call; resets. */
double zo_png_unfilter_seconds(void);

#ifdef __cplusplus
}
#endif
#endif
