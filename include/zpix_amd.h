/*
 * zpix_amd.h — C-ABI of the MI355X-native decode path for braheezy/zpix.
 *
 * The reference is a pure-Zig library; its API is Zig-ABI (allocator + error
 * union).  This header is the C-ABI shim a Zig host binds with `extern "c"`
 * (see INTEGRATION.md).  Every entry point cites the reference interface it
 * replaces.  Conventions that mirror the reference:
 *   - Ownership: the caller passes an allocator (zpx_allocator, the C shape of
 *     std.mem.Allocator; NULL = malloc/free).  A returned zpx_image owns
 *     `pixels` (and `palette` for Paletted) allocated from it; release with
 *     zpx_image_free (Image.free, src/image/image.zig:68-99).
 *   - Errors: int return, 0 = ok, otherwise a ZPX_E_* code whose
 *     zpx_error_name() is the reference's Zig error name (e.g.
 *     "UnexpectedEof", "BadRSTMarker", "InvalidFilterType").  No exception or
 *     abort crosses the ABI.
 *   - Threading: a zpx_ctx (one per GPU) is not shared by host threads
 *     concurrently; calls on different contexts are independent.
 *
 * Layer split: serial entropy decoding (Huffman, zlib
 * inflate) runs on the host inside this library; dequant + IDCT + level
 * shift, chroma upsample + YCbCr->RGB, PNG unfilter + pixel store + Adam7
 * merge, and Image.rgbaPixels run as HIP kernels on gfx950.  There is no CPU
 * fallback: if the device path cannot run, calls fail with ZPX_E_HIP or
 * ZPX_E_UNSUPPORTED.
 */
#ifndef ZPIX_AMD_H
#define ZPIX_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Version of this header's structs and entry points.  2: zpx_jpeg_frame
 * gained `layout`, `pieces` and `pieces_bytes` (ZPX_COEFFS_PIECES), which
 * changed its size, so an array of version-1 frames is read at the wrong
 * offsets; zpx_abi_version() returns the library's value, and a binding
 * checks it against the header it was generated from. */
#define ZPX_ABI_VERSION 2

typedef struct zpx_ctx zpx_ctx;

/* ---------------------------------------------------------------------- */
/* errors                                                                  */
/* ---------------------------------------------------------------------- */
/* Status codes.  Every name is the reference's Zig error name (the JPEG set
 * from src/jpeg/decoder.zig, the PNG set from src/png/decoder.zig, the BMP set
 * from src/bmp/decoder.zig:317-325, the QOI set from src/qoi/{decoder,encoder}.zig), plus
 * Unsupported / Panic / Hip / InvalidArgument for conditions of the device
 * path itself.  zpx_error_name(code) returns the name. */
#define ZPX_ERROR_LIST(X) \
    X(Ok, OK) \
    X(UnexpectedEof, UNEXPECTED_EOF) \
    X(InvalidSOIMarker, INVALID_SOI_MARKER) \
    X(ShortSegmentLength, SHORT_SEGMENT_LENGTH) \
    X(UnknownMarker, UNKNOWN_MARKER) \
    X(UnsupportedMarker, UNSUPPORTED_MARKER) \
    X(MultipleSofMarkers, MULTIPLE_SOF_MARKERS) \
    X(NumberComponents, NUMBER_COMPONENTS) \
    X(Precision, PRECISION) \
    X(SofWrongLength, SOF_WRONG_LENGTH) \
    X(RepeatedComponentIdentifier, REPEATED_COMPONENT_IDENTIFIER) \
    X(BadTqValue, BAD_TQ_VALUE) \
    X(LumaChromaSubSamplingRatio, LUMA_CHROMA_SUB_SAMPLING_RATIO) \
    X(DriWrongLength, DRI_WRONG_LENGTH) \
    X(BadPqValue, BAD_PQ_VALUE) \
    X(DqtWrongLength, DQT_WRONG_LENGTH) \
    X(MissingFF00, MISSING_FF00) \
    X(UninitializedHuffmanTable, UNINITIALIZED_HUFFMAN_TABLE) \
    X(BadHuffmanCode, BAD_HUFFMAN_CODE) \
    X(DhtWrongLength, DHT_WRONG_LENGTH) \
    X(BadTcValue, BAD_TC_VALUE) \
    X(BadThValue, BAD_TH_VALUE) \
    X(HuffZeroLength, HUFF_ZERO_LENGTH) \
    X(HuffTooLong, HUFF_TOO_LONG) \
    X(MissingSosMarker, MISSING_SOS_MARKER) \
    X(SosWrongLength, SOS_WRONG_LENGTH) \
    X(UnknownComponentSelector, UNKNOWN_COMPONENT_SELECTOR) \
    X(BadTdValue, BAD_TD_VALUE) \
    X(BadTaValue, BAD_TA_VALUE) \
    X(SamplingFactorsTooLarge, SAMPLING_FACTORS_TOO_LARGE) \
    X(BadSpectralSelection, BAD_SPECTRAL_SELECTION) \
    X(ProgressiveACCoefficientsForMoreThanOneComponent, PROGRESSIVE_AC_COEFFICIENTS_FOR_MORE_THAN_ONE_COMPONENT) \
    X(BadSuccessiveApproximation, BAD_SUCCESSIVE_APPROXIMATION) \
    X(ExcessiveDCComponent, EXCESSIVE_DC_COMPONENT) \
    X(UnexpectedHuffmanCode, UNEXPECTED_HUFFMAN_CODE) \
    X(TooManyCoefficients, TOO_MANY_COEFFICIENTS) \
    X(BadRSTMarker, BAD_RST_MARKER) \
    X(UnsupportedComponent, UNSUPPORTED_COMPONENT) \
    X(UnsupportedColorModel, UNSUPPORTED_COLOR_MODEL) \
    X(InvalidPngHeader, INVALID_PNG_HEADER) \
    X(ChunkOrderInHeaderError, CHUNK_ORDER_IN_HEADER_ERROR) \
    X(ChunkOrderPlteError, CHUNK_ORDER_PLTE_ERROR) \
    X(ChunkOrderIdatError, CHUNK_ORDER_IDAT_ERROR) \
    X(ChunkOrderTrns1Error, CHUNK_ORDER_TRNS1_ERROR) \
    X(ChunkOrderTrns2Error, CHUNK_ORDER_TRNS2_ERROR) \
    X(ChunkOrderTrns3Error, CHUNK_ORDER_TRNS3_ERROR) \
    X(ChunkOrderIendError, CHUNK_ORDER_IEND_ERROR) \
    X(InvalidIHDRLength, INVALID_IHDR_LENGTH) \
    X(UnsupportedCompressionMethod, UNSUPPORTED_COMPRESSION_METHOD) \
    X(UnsupportedFilterMethod, UNSUPPORTED_FILTER_METHOD) \
    X(UnsupportedInterlaceMethod, UNSUPPORTED_INTERLACE_METHOD) \
    X(InvalidDimension, INVALID_DIMENSION) \
    X(DimensionOverflow, DIMENSION_OVERFLOW) \
    X(InvalidColorType, INVALID_COLOR_TYPE) \
    X(InvalidColorTypeDepthCombo, INVALID_COLOR_TYPE_DEPTH_COMBO) \
    X(UnsupportedBitDepth, UNSUPPORTED_BIT_DEPTH) \
    X(EmptyIdatData, EMPTY_IDAT_DATA) \
    X(BadTrnsLength, BAD_TRNS_LENGTH) \
    X(TrnsColorTypeMismatch, TRNS_COLOR_TYPE_MISMATCH) \
    X(BadPlteLength, BAD_PLTE_LENGTH) \
    X(PlteColorTypeMismatch, PLTE_COLOR_TYPE_MISMATCH) \
    X(InvalidFilterType, INVALID_FILTER_TYPE) \
    X(InvalidChecksum, INVALID_CHECKSUM) \
    X(EndOfStream, END_OF_STREAM) \
    X(ReadFailed, READ_FAILED) \
    X(InvalidImageDimensions, INVALID_IMAGE_DIMENSIONS) \
    X(OutOfMemory, OUT_OF_MEMORY) \
    X(Unsupported, UNSUPPORTED) \
    X(Panic, PANIC) \
    X(Hip, HIP) \
    X(InvalidArgument, INVALID_ARGUMENT) \
    X(FileNotFound, FILE_NOT_FOUND) \
    X(UnknownImageFormat, UNKNOWN_IMAGE_FORMAT) \
    X(InvalidSignature, INVALID_SIGNATURE) \
    X(UnsupportedHeader, UNSUPPORTED_HEADER) \
    X(UnsupportedDimensions, UNSUPPORTED_DIMENSIONS) \
    X(UnsupportedCompression, UNSUPPORTED_COMPRESSION) \
    X(UnsupportedBPP, UNSUPPORTED_BPP) \
    X(UnsupportedPaletteSize, UNSUPPORTED_PALETTE_SIZE) \
    X(UnsupportedColorOffset, UNSUPPORTED_COLOR_OFFSET) \
    X(InvalidQoiData, INVALID_QOI_DATA) \
    X(InvalidQoiHeader, INVALID_QOI_HEADER)

enum zpx_status {
#define ZPX_ENUM_(name, up) ZPX_E_##up,
    ZPX_ERROR_LIST(ZPX_ENUM_)
#undef ZPX_ENUM_
    ZPX_E__COUNT
};
#define ZPX_OK ZPX_E_OK
/* Name of any status code ("Ok", "UnexpectedEof", ... as in the reference). */
const char *zpx_error_name(int code);
/* ZPX_ABI_VERSION of the library's build. */
int zpx_abi_version(void);
/* Releases the host stages' recycled buffers -- the PNG IDAT buffers and the
 * parallel inflate's symbol buffers, which a batch of large PNGs leaves
 * pooled (up to ~2 x host threads and 64 buffers, 2 GiB and 1 GiB at most)
 * for the next batch to reuse with their pages -- and returns the bytes
 * released.  Safe at any time; buffers in use are not touched. */
size_t zpx_host_pools_trim(void);
/* Frees the batch pipeline's cached slots: zpx_batch_decode_rgba keeps a
 * finished batch's slots (per device: their device buffers -- the largest
 * image's input and coefficients, ~80 MB a slot for 4K -- events and pinned
 * status words; at most 256 slots) for the next batch on the device, whose
 * setup and teardown then allocate and free nothing.  Returns the device
 * bytes released.  Safe at any time; slots of running batches are not
 * touched. */
size_t zpx_batch_cache_trim(void);
/* Detail message of the last failure on this context (never NULL). */
const char *zpx_last_error(const zpx_ctx *ctx);

/* ---------------------------------------------------------------------- */
/* context                                                                 */
/* ---------------------------------------------------------------------- */
/* One context per GPU: owns a compute stream, a copy stream, pinned staging
 * and device scratch.  Replaces nothing in the reference (it has no device). */
int zpx_ctx_create(int device, zpx_ctx **out);
void zpx_ctx_destroy(zpx_ctx *ctx);
/* The context's compute stream (a hipStream_t). */
void *zpx_ctx_stream(zpx_ctx *ctx);
int zpx_ctx_device(const zpx_ctx *ctx);
/* Blocks until all work queued by this context is complete. */
int zpx_ctx_synchronize(zpx_ctx *ctx);

/* std.mem.Allocator in C form. alloc returns NULL on failure. */
typedef struct zpx_allocator {
    void *(*alloc)(void *user, size_t len);
    void (*free)(void *user, void *ptr, size_t len);
    void *user;
} zpx_allocator;

/* ---------------------------------------------------------------------- */
/* image.Image                                                             */
/* ---------------------------------------------------------------------- */
/* Image tags, src/image/image.zig:24-34 */
enum zpx_kind {
    ZPX_GRAY = 0,
    ZPX_GRAY16 = 1,
    ZPX_YCBCR = 2,
    ZPX_RGBA = 3,
    ZPX_RGBA64 = 4,
    ZPX_NRGBA = 5,
    ZPX_NRGBA64 = 6,
    ZPX_CMYK = 7,
    ZPX_PALETTED = 8,
};
/* YCbCrSubsample, src/image/image.zig:465-472 */
enum zpx_subsample {
    ZPX_RATIO444 = 0,
    ZPX_RATIO422 = 1,
    ZPX_RATIO420 = 2,
    ZPX_RATIO440 = 3,
    ZPX_RATIO411 = 4,
    ZPX_RATIO410 = 5,
};
/* A palette Color: the .rgba (model 0) or .nrgba (model 1) arm of
 * color.Color (src/color/color.zig:13-23). */
typedef struct zpx_color {
    uint8_t r, g, b, a;
    uint8_t model;
    uint8_t pad[3];
} zpx_color;

/* image.Image (src/image/image.zig:24-34 + the concrete pixel buffers
 * :133-890).  Pixel layouts are the reference's: RGBA/NRGBA/CMYK 4 B/px,
 * RGBA64/NRGBA64 8 B/px big-endian per channel, Gray 1, Gray16 2 (BE),
 * Paletted 1 (+palette).  YCbCr planes are views into `pixels`. */
typedef struct zpx_image {
    int32_t kind;
    int32_t min_x, min_y, max_x, max_y;
    uint8_t *pixels;
    size_t pixels_len;
    size_t stride;
    size_t y_off, cb_off, cr_off;  /* YCbCr */
    size_t y_stride, c_stride;     /* YCbCr */
    int32_t subsample;             /* YCbCr */
    zpx_color *palette;            /* Paletted */
    int32_t palette_len;
} zpx_image;

/* Image.free, src/image/image.zig:68-99 */
void zpx_image_free(const zpx_allocator *al, zpx_image *img);

/* Image.rgbaPixels, src/image/image.zig:103-130: 8-bit RGBA, 4*dX*dY bytes,
 * caller-owned (allocated from al).  Runs the conversion on the GPU. */
int zpx_image_rgba_pixels(zpx_ctx *ctx, const zpx_allocator *al, const zpx_image *img,
                          uint8_t **out, size_t *out_len);

/* ---------------------------------------------------------------------- */
/* codecs (host entropy decode + device pixel loops)                       */
/* ---------------------------------------------------------------------- */
/* jpeg.decode / jpeg.loadFromBuffer: src/jpeg/decoder.zig:155-176,
 * src/jpeg/root.zig:10-15.  Returns .Gray, .YCbCr, .RGBA (Adobe RGB) or .CMYK
 * exactly as decodeInner's output select (decoder.zig:357-372). */
int zpx_jpeg_decode(zpx_ctx *ctx, const zpx_allocator *al, const uint8_t *buf, size_t len,
                    zpx_image *out);
/* jpeg.load, src/jpeg/root.zig:36-53 */
int zpx_jpeg_load(zpx_ctx *ctx, const zpx_allocator *al, const char *path, zpx_image *out);
/* jpeg.probeBuffer, src/jpeg/root.zig:17-21 */
int zpx_jpeg_probe_buffer(const uint8_t *buf, size_t len);

/* color.Model, src/color/color.zig:161-165 */
enum zpx_model { ZPX_MODEL_RGB = 0, ZPX_MODEL_YCBCR = 1, ZPX_MODEL_RGBA = 2, ZPX_MODEL_GRAY = 3 };
/* jpeg.decodeConfig, src/jpeg/decoder.zig:178-218 (image.Config: width,
 * height, color_model; 4-component frames report YCbCr as the reference does).
 * Host-only header parse: no context needed. */
int zpx_jpeg_decode_config(const uint8_t *buf, size_t len, uint32_t *width, uint32_t *height,
                           int32_t *color_model);
/* Width/height of a PNG from its IHDR (signature + IHDR checks of
 * png/decoder.zig:224-402); host-only.  Used to size batch destinations. */
int zpx_png_decode_config(const uint8_t *buf, size_t len, uint32_t *width, uint32_t *height);

/* jpeg.decode followed by Image.rgbaPixels, fused on the device (one kernel:
 * dequant + IDCT + level shift + upsample + YCbCr->RGB). */
int zpx_jpeg_decode_rgba(zpx_ctx *ctx, const zpx_allocator *al, const uint8_t *buf, size_t len,
                         uint8_t **rgba, size_t *rgba_len, uint32_t *width, uint32_t *height);

/* png.decode / png.loadFromBuffer: src/png/decoder.zig:143-221,
 * src/png/root.zig:29-34 */
int zpx_png_decode(zpx_ctx *ctx, const zpx_allocator *al, const uint8_t *buf, size_t len,
                   zpx_image *out);
/* png.load, src/png/root.zig:13-27 */
int zpx_png_load(zpx_ctx *ctx, const zpx_allocator *al, const char *path, zpx_image *out);
/* png.probeBuffer, src/png/root.zig:37-40 */
int zpx_png_probe_buffer(const uint8_t *buf, size_t len);

/* bmp.decode / bmp.loadFromBuffer: src/bmp/decoder.zig:25-40,
 * src/bmp/root.zig:21-25.  The header and palette (readHeader :42-158) are
 * parsed on the host; the row loop (bottom-up flip, BGR(A) -> RGBA, palette
 * index unpack; :160-307) is a HIP kernel.  Returns .Paletted (1/2/4/8 bpp),
 * .RGBA (24 bpp) or .NRGBA (32 bpp); a short file is EndOfStream. */
int zpx_bmp_decode(zpx_ctx *ctx, const zpx_allocator *al, const uint8_t *buf, size_t len,
                   zpx_image *out);
/* bmp.load, src/bmp/root.zig:8-19 */
int zpx_bmp_load(zpx_ctx *ctx, const zpx_allocator *al, const char *path, zpx_image *out);
/* bmp.probeBuffer, src/bmp/root.zig:28-31 */
int zpx_bmp_probe_buffer(const uint8_t *buf, size_t len);

/* qoi.decode / qoi.loadFromBuffer: src/qoi/decoder.zig:20-130,
 * src/qoi/root.zig:34-38.  Returns .RGBA.  Every QOI chunk depends on the
 * previous pixel and on a hash table whose slot is picked by decoded values,
 * so this is a serial host loop like Huffman and inflate; ctx may be NULL. */
int zpx_qoi_decode(zpx_ctx *ctx, const zpx_allocator *al, const uint8_t *buf, size_t len,
                   zpx_image *out);
/* qoi.load, src/qoi/root.zig:20-31 */
int zpx_qoi_load(zpx_ctx *ctx, const zpx_allocator *al, const char *path, zpx_image *out);
/* qoi.probeBuffer, src/qoi/root.zig:41-49 */
int zpx_qoi_probe_buffer(const uint8_t *buf, size_t len);

/* qoi.Desc, src/qoi/encoder.zig:20-25 */
typedef struct zpx_qoi_desc {
    uint32_t width, height;
    uint8_t channels;   /* 3 = RGB, 4 = RGBA */
    uint8_t colorspace; /* 0 = sRGB with linear alpha, 1 = all linear */
    uint8_t pad[2];
} zpx_qoi_desc;
/* qoi.encode, src/qoi/encoder.zig:29-132: pixels (host, width*height*channels
 * bytes) -> QOI file bytes, caller-owned from al.  Encoded on the GPU as a
 * segmented scan; byte-identical to the serial loop.  InvalidQoiHeader for a
 * desc the reference rejects (:34-36). */
int zpx_qoi_encode(zpx_ctx *ctx, const zpx_allocator *al, const uint8_t *pixels, size_t pixels_len,
                   const zpx_qoi_desc *desc, uint8_t **out, size_t *out_len);
/* Upper bound of the encoded size (the reference's maxSize, encoder.zig:41-42). */
size_t zpx_qoi_encode_bound(const zpx_qoi_desc *desc);
/* Device form: d_pixels and d_out (>= zpx_qoi_encode_bound bytes) are device
 * pointers; the encoded length lands in *d_out_len (device uint64).  Enqueued
 * on `stream` (NULL = the context's stream) with no host synchronisation once
 * the context's scratch is large enough. */
int zpx_qoi_encode_device(zpx_ctx *ctx, const uint8_t *d_pixels, const zpx_qoi_desc *desc, uint8_t *d_out,
                          size_t out_cap, uint64_t *d_out_len, void *stream);

/* zpix.fromBuffer / zpix.fromFilePath, src/root.zig:24-40: probes PNG, JPEG,
 * QOI, BMP in that order; UnknownImageFormat otherwise. */
int zpx_from_buffer(zpx_ctx *ctx, const zpx_allocator *al, const uint8_t *buf, size_t len,
                    zpx_image *out);
int zpx_from_file_path(zpx_ctx *ctx, const zpx_allocator *al, const char *path, zpx_image *out);

/* ---------------------------------------------------------------------- */
/* device-level plans (device pointers, asynchronous, graph-capturable)    */
/* ---------------------------------------------------------------------- */
typedef struct zpx_plan zpx_plan;

/* What a JPEG frame's reconstruct writes. */
enum zpx_jpeg_output {
    ZPX_JPEG_PLANES = 0, /* reconstructBlock into Y/Cb/Cr/K planes (decoder.zig:1553-1634) */
    ZPX_JPEG_RGBA = 1,   /* planes + Image.rgbaPixels fused (RGBA8, stride rgba_stride) */
};
/* Which blocks of a component are reconstructed. */
enum zpx_block_rule {
    ZPX_BLOCKS_ALL = 0,         /* baseline interleaved scan: every MCU block */
    ZPX_BLOCKS_PROGRESSIVE = 1, /* by*v<H && bx*h<W, decoder.zig:1649-1651 */
    ZPX_BLOCKS_SCAN = 2,        /* non-interleaved baseline scan: bx*8<W && by*8<H (:1334) */
    ZPX_BLOCKS_NONE = 3,        /* component never scanned: plane stays zero */
};
/* Colour handling of the fused RGBA output. */
enum zpx_jpeg_color {
    ZPX_JPEG_COLOR_YCBCR = 0, /* Color.toRGBA .ycbcr (color.zig:90-113) */
    ZPX_JPEG_COLOR_RGB = 1,   /* Adobe/RGB ids: convertToRGB (decoder.zig:751-783) */
    ZPX_JPEG_COLOR_GRAY = 2,  /* 1 component: .gray (color.zig:122-126) */
};

/* How a frame's coefficients are laid out in memory. */
enum zpx_coeff_layout {
    ZPX_COEFFS_GRID = 0,   /* coeffs[c]: (mxx*h) x (myy*v) blocks x 64 natural-order coefficients */
    ZPX_COEFFS_PIECES = 1, /* coeffs[c]: a uint32 per block in grid order, first_piece << 4 | pieces;
                              the block's coefficients are `pieces` 16-byte pieces from `first_piece` of
                              zpx_jpeg_frame.pieces, in zig-zag order up to its last nonzero one (the rest
                              of the last piece zero), int8 (16 a piece) or int16 (8 a piece) per
                              coeff_bits; pieces 0: an all-zero block.  Piece 0 must be zeros. */
};

/* One JPEG frame after host entropy decoding: coefficient grids
 * (processSos accumulate form, decoder.zig:1340-1345) + frame geometry. */
typedef struct zpx_jpeg_frame {
    uint32_t width, height;
    int32_t n_comp;          /* 1, 3 or 4 */
    int32_t h[4], v[4];      /* sampling factors after processSof (decoder.zig:490-618) */
    int32_t mxx, myy;        /* MCU grid (decoder.zig:1262-1263) */
    int32_t rule[4];         /* zpx_block_rule per component */
    int32_t coeff_bits;      /* 8, 16 or 32: int8 / int16 / int32 grids (the narrowest that holds the frame) */
    int32_t narrow;          /* 1 if max|coef*q| <= 16384 for every component */
    int32_t color;           /* zpx_jpeg_color (fused output only) */
    const void *coeffs[4];   /* DEVICE: (mxx*h) x (myy*v) blocks, 64 natural-order coefs each */
    int32_t qt[4][64];       /* per component, NATURAL order (unzig applied) */
    uint8_t *planes[4];      /* DEVICE, ZPX_JPEG_PLANES: plane base per component */
    size_t strides[4];
    uint8_t *rgba;           /* DEVICE, ZPX_JPEG_RGBA */
    size_t rgba_stride;
    int32_t layout;          /* zpx_coeff_layout of coeffs[] */
    const void *pieces;      /* DEVICE, ZPX_COEFFS_PIECES: the frame's 16-byte pieces */
    size_t pieces_bytes;     /* ZPX_COEFFS_PIECES: bytes at `pieces` */
} zpx_jpeg_frame;

/* Uploads the frame descriptors once; zpx_plan_launch then only enqueues
 * kernels (no host allocation or sync, so it can be captured in a hipGraph). */
int zpx_jpeg_plan_create(zpx_ctx *ctx, const zpx_jpeg_frame *frames, int n_frames, int output,
                         zpx_plan **out);

/* PNG ColorBitDepth, src/png/decoder.zig:88-118 */
enum zpx_png_depth {
    ZPX_PNG_G1 = 1, ZPX_PNG_G2, ZPX_PNG_G4, ZPX_PNG_G8, ZPX_PNG_GA8, ZPX_PNG_TC8,
    ZPX_PNG_P1, ZPX_PNG_P2, ZPX_PNG_P4, ZPX_PNG_P8, ZPX_PNG_TCA8, ZPX_PNG_G16,
    ZPX_PNG_GA16, ZPX_PNG_TC16, ZPX_PNG_TCA16,
};
/* Readable bytes the device input must have past its last filtered row. */
#define ZPX_PNG_INPUT_PAD 256
/* Layout of zpx_png_frame.filtered.  STREAM: the inflated stream as is
 * (what parseIdat hands readImagePass, png/decoder.zig:516-523), followed by
 * ZPX_PNG_INPUT_PAD readable bytes.  SLAB: the same bytes rearranged per
 * 128-row band in the order the paired-row kernel reads them
 * (zpx_png_stream_slab builds it on the host; only for frames that kernel
 * takes, i.e. zpx_png_stream_slab succeeds).  The paired-row kernel reads
 * either: a STREAM frame straight from the stream (its stream instance), a
 * SLAB frame with whole-line loads. */
enum zpx_png_layout { ZPX_PNG_LAYOUT_STREAM = 0, ZPX_PNG_LAYOUT_SLAB = 1 };

/* One PNG image after host inflate (parseIdat, png/decoder.zig:404-545). */
typedef struct zpx_png_frame {
    uint32_t width, height;
    int32_t depth;           /* zpx_png_depth */
    int32_t interlace;       /* 0 none, 1 Adam7 */
    int32_t use_transparent; /* tRNS colour key (png/decoder.zig:547-602) */
    uint8_t transparent[6];
    uint8_t layout;          /* zpx_png_layout of `filtered` */
    uint8_t pad;
    const uint8_t *filtered; /* DEVICE: inflated stream, filter byte per row, all passes
                                (ZPX_PNG_LAYOUT_STREAM), or its band slab (ZPX_PNG_LAYOUT_SLAB) */
    uint8_t *out;            /* DEVICE: pixels of the image type readImagePass allocates */
    size_t out_stride;
    int32_t *max_index;      /* DEVICE, paletted only: receives max palette index (or NULL) */
} zpx_png_frame;

/* Unfilter (Sub/Up/Avg/Paeth) + per-depth pixel store (+ Adam7 merge) of
 * readImagePass (png/decoder.zig:649-1149, 1289-1373).  Filter bytes must be
 * valid (<= 4): the host checks them (InvalidFilterType) before planning.
 * Kernels: the paired-row kernel for RGB8/RGBA8/Gray8/Gray16/RGB16/RGBA16
 * (interlaced or not, tRNS colour keys on RGB; either layout: its stream
 * instance reads a STREAM frame's inflated rows directly, its slab instance
 * a SLAB frame's band slab -- a slab built on the device from a STREAM frame
 * is a test-only path, the switch "png_device_slab"), the one-row-per-lane kernel
 * for every other depth (sub-byte gray, paletted, gray+alpha) and for STREAM
 * frames the paired-row kernel declines (png_pair_supported: e.g. rows shorter
 * than one 12/16-byte chunk, bands past the 2 GiB buffer range). */
int zpx_png_plan_create(zpx_ctx *ctx, const zpx_png_frame *frames, int n_frames, zpx_plan **out);

/* Enqueue the plan's kernels on `stream` (NULL = the context's stream). */
int zpx_plan_launch(zpx_plan *plan, void *stream);
/* Error status of the plan's launches since the last call: ZPX_OK, or
 * ZPX_E_HIP ("Hip", with zpx_last_error "png wavefront hand-off timed out")
 * when any PNG wavefront hand-off gave up waiting, i.e. that launch's output
 * is invalid.  The reference's contract is that every decode step returns an
 * error union (src/png/decoder.zig:143-221); zpx_plan_launch only enqueues,
 * so this is where an asynchronous launch reports.  Waits for `stream` (NULL
 * = the context's stream), then clears the status.  JPEG plans always report
 * ZPX_OK (their kernels have no wait that can time out). */
int zpx_plan_status(zpx_plan *plan, void *stream);
/* Algorithmic bytes (read + written) one launch of the plan moves. */
uint64_t zpx_plan_bytes(const zpx_plan *plan);
/* Number of kernel launches one zpx_plan_launch enqueues. */
int zpx_plan_kernel_count(const zpx_plan *plan);
void zpx_plan_destroy(zpx_plan *plan);

/* Image.rgbaPixels on device memory: img->pixels / img->palette are DEVICE
 * pointers; out is a DEVICE buffer of 4*dX*dY bytes. */
int zpx_dev_rgba_pixels(zpx_ctx *ctx, const zpx_image *img, uint8_t *out, void *stream);
/* Image.rgbaPixels (image.zig:103-130) of n device-resident images as one
 * plan: imgs[i].pixels / palette are DEVICE pointers, outs[i] a DEVICE
 * buffer of 4*dX*dY bytes (RGBA8, stride 4*dX).  zpx_plan_launch enqueues
 * one kernel per image kind (no host work); zpx_plan_bytes counts the pixels
 * each kind reads plus the RGBA8 written. */
int zpx_rgba_plan_create(zpx_ctx *ctx, const zpx_image *imgs, uint8_t *const *outs, int n, zpx_plan **out);

/* ---------------------------------------------------------------------- */
/* host entropy stage exposed for batching / parity                        */
/* ---------------------------------------------------------------------- */
typedef struct zpx_jpeg_coeffs zpx_jpeg_coeffs;
/* Runs the host half of jpeg.decode (markers, DHT/DQT/SOF/SOS, Huffman,
 * progressive refinement) and keeps the coefficient grids in pinned memory. */
int zpx_jpeg_entropy_decode(const uint8_t *buf, size_t len, zpx_jpeg_coeffs **out);
/* The same, but a baseline frame whose single scan interleaves all three
 * components is kept as ZPX_COEFFS_PIECES (the batch pipeline's transport:
 * about 40 % of the dense int8 grid for a q75 photo, and the block kernels
 * read it directly); other frames still decode into grids. */
int zpx_jpeg_entropy_decode_pieces(const uint8_t *buf, size_t len, zpx_jpeg_coeffs **out);
/* Fills a frame descriptor (host pointers for coeffs, and for pieces with
 * layout ZPX_COEFFS_PIECES; coeff_bytes_per_comp then counts the index
 * arrays) from decoded coefficients. */
int zpx_jpeg_coeffs_frame(const zpx_jpeg_coeffs *c, zpx_jpeg_frame *frame,
                          size_t *coeff_bytes_per_comp /* [4] */);
void zpx_jpeg_coeffs_free(zpx_jpeg_coeffs *c);
/* Widens every grid to at least `bits` (16 or 32) coefficient bits.  The
 * entropy stage keeps the narrowest width that holds the frame (8, 16 or 32:
 * zpx_jpeg_frame.coeff_bits); a caller that wants one fixed transport format
 * (or an A/B of the transports) widens here. */
int zpx_jpeg_coeffs_widen(zpx_jpeg_coeffs *c, int bits);

typedef struct zpx_png_stream zpx_png_stream;
/* Host half of png.decode: chunk parse + CRC + inflate into pinned memory. */
int zpx_png_inflate(const uint8_t *buf, size_t len, zpx_png_stream **out);
int zpx_png_stream_frame(const zpx_png_stream *s, zpx_png_frame *frame, size_t *filtered_len);
const uint8_t *zpx_png_stream_data(const zpx_png_stream *s);
/* The stream's band slab (ZPX_PNG_LAYOUT_SLAB; built on first use, pinned
 * host memory owned by the stream): upload *len bytes of *data and set the
 * frame's layout to ZPX_PNG_LAYOUT_SLAB.  ZPX_E_UNSUPPORTED when the
 * paired-row kernel does not take the image (the stream layout still works). */
int zpx_png_stream_slab(zpx_png_stream *s, const uint8_t **data, size_t *len);
void zpx_png_stream_free(zpx_png_stream *s);

/* ---------------------------------------------------------------------- */
/* batch / streaming decode                    */
/* ---------------------------------------------------------------------- */
/* Many encoded JPEG/PNG buffers -> RGBA8 in the layout of Image.rgbaPixels
 * (image.zig:103-130), i.e. what `zpix.fromBuffer` + `img.rgbaPixels` give per
 * image, without any per-image host sync:
 *   - a pool of host threads runs the serial entropy stages (Huffman /
 *     inflate, decoder.zig:1148-1455, png/decoder.zig:404-545) into pinned
 *     buffers;
 *   - the calling thread streams each result to the device with
 *     hipMemcpyAsync on a copy stream, the context's compute stream waits on
 *     that copy's event and runs the kernels, and (dst_on_host) a third
 *     stream copies the RGBA back;
 *   - at most `depth` images are staged at once; a slot is recycled when its
 *     last event completes.
 * Items complete independently: a malformed image sets its own `status`
 * (the reference's error for it) and the rest of the batch proceeds. */
typedef struct zpx_batch_item {
    const uint8_t *buf;      /* encoded bytes (caller-owned, valid until the batch completes) */
    size_t len;
    uint8_t *dst;            /* RGBA8 output: DEVICE pointer, or HOST pointer when dst_on_host */
    size_t dst_stride;       /* bytes between output rows; 0 = 4 * width */
    size_t dst_capacity;     /* bytes available at dst (checked: ZPX_E_INVALID_ARGUMENT if short) */
    int32_t status;          /* out: ZPX_OK or the image's error code */
    uint32_t width, height;  /* out */
    int32_t format;          /* out: 1 JPEG, 2 PNG, 0 unknown */
} zpx_batch_item;

typedef struct zpx_batch_opts {
    int32_t host_threads;    /* entropy/inflate workers; 0 = min(16, the process's CPU budget: affinity
                                capped by the cgroup quota); sharded: that budget / ndev per device */
    int32_t depth;           /* images staged on the device at once; 0 = 2 * host_threads */
    int32_t dst_on_host;     /* 1: dst are host pointers (results copied back over PCIe) */
} zpx_batch_opts;

typedef struct zpx_batch_stats {
    double wall_s;           /* batch wall time */
    double host_s;           /* summed host entropy/inflate time over all workers */
    double h2d_bytes, d2h_bytes;
    double pixels;           /* decoded pixels of the successful items */
    int32_t host_threads, depth;
    int32_t failed;          /* items with status != ZPX_OK */
    int32_t pad;
    double host_jpeg_s;      /* host_s split by stage: JPEG entropy decode (processSos) */
    double host_png_s;       /*   and PNG chunk walk + inflate (parseIdat) */
    int32_t jpeg_items, png_items;
} zpx_batch_stats;

/* Decodes the whole batch and returns when every item is complete.
 * Returns ZPX_OK when the batch ran (see each item's status), ZPX_E_HIP on a
 * device failure, ZPX_E_INVALID_ARGUMENT on bad arguments. */
int zpx_batch_decode_rgba(zpx_ctx *ctx, zpx_batch_item *items, int n_items, const zpx_batch_opts *opts,
                          zpx_batch_stats *stats /* may be NULL */);

/* Asynchronous form: starts the same pipeline on a background thread and
 * returns at once; zpx_batch_wait joins it (and frees the handle). The items
 * array and buffers must stay valid until then; the context must not be used
 * by other calls meanwhile. */
typedef struct zpx_batch zpx_batch;
int zpx_batch_start(zpx_ctx *ctx, zpx_batch_item *items, int n_items, const zpx_batch_opts *opts,
                    zpx_batch **out);
int zpx_batch_wait(zpx_batch *b, zpx_batch_stats *stats /* may be NULL */);
/* Blocks until items 0..n-1 of a started batch are final (status set, RGBA
 * complete in dst) or the batch has ended, and returns how many leading
 * items are final.  Lets a caller move finished results on (the chunked
 * gather of configs[3]) while later items still decode. */
int zpx_batch_wait_prefix(zpx_batch *b, int n);

/* configs[3] in one process: image i of `items` is
 * decoded on ctxs[i % ndev] -- one streaming pipeline (zpx_batch_decode_rgba,
 * `opts` per device) per device, each on its own host thread -- and every
 * result is gathered into items[i].dst on ctxs[0]'s device: grouped
 * ncclSend/ncclRecv over RCCL (xGMI) between distinct devices, a device copy
 * when a context shares device 0's GPU.  items[i].dst are DEVICE pointers on
 * ctxs[0]'s device (dst_capacity bytes each); every other device decodes into
 * staging of that capacity first.  Statuses, widths and heights come back in
 * items as from zpx_batch_decode_rgba.  Each result moves as soon as its
 * device finishes it (the gather overlaps the decode of later images); the
 * communicators are created once per device set and cached.  A remote item
 * is ZPX_OK only once it has arrived; one its shard's pipeline or the
 * gather failed before moving carries that error.  opts->dst_on_host must be
 * 0 (ZPX_E_INVALID_ARGUMENT).  `stats` sums over the devices (wall_s = the
 * whole job, gather included); `gather` (may be NULL) splits the wall time
 * into decode and the gather's tail.  The reference has no counterpart (it is
 * single-threaded, src/root.zig:24-40); per image the result is
 * zpix.fromBuffer + Image.rgbaPixels (image.zig:103-130). */
typedef struct zpx_gather_stats {
    double decode_s;      /* until every device's pipeline finished */
    double gather_s;      /* from the first transfer posted to the last one complete (overlaps decode_s) */
    double gather_bytes;  /* bytes moved to device 0 */
    int32_t ndev, pad;
    double tail_s;        /* the gather's part after decode_s (wall_s = decode_s + tail_s) */
    double comm_setup_s;  /* communicator creation in this call, outside wall_s (0 once cached) */
    int32_t comm_ranks;   /* communicator ranks used (1: no send/recv, device copies only) */
    int32_t pad2;
} zpx_gather_stats;
int zpx_batch_decode_sharded(zpx_ctx *const *ctxs, int ndev, zpx_batch_item *items, int n_items,
                             const zpx_batch_opts *opts, zpx_batch_stats *stats /* may be NULL */,
                             zpx_gather_stats *gather /* may be NULL */);

/* ---------------------------------------------------------------------- */
/* fault injection (tests)                                                 */
/* ---------------------------------------------------------------------- */
/* Launches each PNG unfilter kernel (one row per lane, and paired rows) on a
 * 2-band image whose second band waits for a first band that is never
 * scheduled (a producer that never publishes), with `spin_limit` polls per
 * wait, and returns what zpx_plan_status reports: ZPX_E_HIP when both
 * bounded waits gave up (the expected outcome).  `seconds` (may be NULL)
 * receives the slower launch's wall time, which must stay about one spin
 * limit, not one per step. */
int zpx_debug_png_stall(zpx_ctx *ctx, uint32_t spin_limit, double *seconds);

/* Test hook: the band slab of an inflated stream as the plans build it on the
 * device (ZPX_PNG_LAYOUT_STREAM frames on the paired-row kernel), copied back
 * to host `out` of `cap` bytes; *len receives its size (with out == NULL only
 * the size).  Region sizes follow the geometry's largest skew, so the table
 * of region offsets at its start differs from zpx_png_stream_slab's; every
 * byte the kernel reads is equal.  ZPX_E_UNSUPPORTED when the paired-row
 * kernel does not take the image. */
int zpx_debug_png_device_slab(zpx_ctx *ctx, const zpx_png_stream *s, uint8_t *out, size_t cap, size_t *len);

/* Number of scans the host entropy stage has decoded restart-interval-
 * parallel in this process (tests: the parallel path ran, not its serial
 * fallback).  Host-only. */
int64_t zpx_debug_jpeg_parallel_scans(void);
/* Number of progressive frames whose scans the host entropy stage has
 * decoded concurrently (dependency-ordered, checked against the serial
 * loop's continuation; a frame that fails the check is decoded serially and
 * not counted).  Host-only. */
int64_t zpx_debug_jpeg_parallel_progressive(void);
/* Test hook for zpx_batch_decode_sharded: 1 installs an in-process fake
 * communicator table in place of RCCL -- ncclSend/ncclRecv pairs matched at
 * ncclGroupEnd and carried out as stream-ordered device copies (the receive
 * stream waits for the send stream and the send stream for the copy) -- with
 * one communicator rank per CONTEXT, so the send/recv branch runs even when
 * every context shares one GPU; 0 restores RCCL.  Returns the previous
 * setting. */
int zpx_debug_shard_fake_comm(int on);
/* Test switches (process-wide): sets option `name` to `value` and returns its
 * previous value (-1: unknown name).  Each selects between two paths with
 * the same results, so a test can cover both:
 *   "jpeg_strip"  1: the fused JPEG plans use the strip kernel for every
 *                 frame (default 0: the block-per-lane kernel where it applies);
 *   "jpeg_sparse" 0: the batch pipeline uploads dense coefficient grids
 *                 (default 1: ZPX_COEFFS_PIECES);
 *   "png_pair"    0: PNG frames use the one-row-per-lane kernel (default 1);
 *   "png_device_slab" 1: stream-layout PNG frames on the paired-row kernel
 *                 get their band slab built on the device at each launch
 *                 and read it (default 0: the kernel reads the stream);
 *   "qoi_segment" pixels per lane segment of the QOI encoder (16..4096;
 *                 default 0 = 128);
 *   "png_epoch_cycle" epochs a PNG control block cycles through before its
 *                 boundary buffer is cleared and the epoch re-based (>= 4;
 *                 default 0 = 2^20, the whole window; blocks created after
 *                 the call take it): a short cycle runs the wrap path;
 *   "shard_rccl_self" 1: zpx_batch_decode_sharded moves the results of a
 *                 shard on device 0's GPU by grouped ncclSend / ncclRecv to
 *                 rank 0 itself (RCCL; a one-rank communicator when every
 *                 context shares the GPU) instead of a device copy
 *                 (default 0);
 *   "batch_lookahead" 1: the batch pipeline's host workers take items in
 *                 item order; k >= 2: the costliest of the next k x host_threads
 *                 items first (default 0: k = 4);
 *   "inflate_pair" 0: a batch worker inflates one PNG at a time (default 1:
 *                 two PNGs' inflates in one loop while the batch has more
 *                 than 2 x host_threads items left to take);
 *   "batch_makespan" 0: a batch worker pairs two PNGs whenever the batch
 *                 has items to spare (default 1: only while the pair's
 *                 estimated host time fits the batch's projected remaining
 *                 time per worker, so late PNGs run alone);
 *   "batch_slot_cache" 0: every batch creates its slots and frees them at
 *                 the end (default 1: reused from zpx_batch_cache_trim's
 *                 cache). */
int zpx_debug_option(const char *name, int value);
/* Test hook: decodes a baseline 3-component interleaved JPEG into the
 * ZPX_COEFFS_PIECES form the batch pipeline uploads and
 * expands it on the host into int32 grids (component after component,
 * blocks x 64, natural order), checking the layout's invariants.  Returns
 * the block count, 0 if the frame took grids, or -(status). */
int64_t zpx_debug_jpeg_sparse_grids(const uint8_t *buf, size_t len, int32_t *grids, size_t grid_elems);
/* Test hook: the speculative multi-threaded inflate of one zlib stream (the
 * PNG host stage for large single images).  1 when it decoded
 * the first `want` bytes into out on `threads` threads, 0 when it declined;
 * threads = 1 runs the serial fast decoder instead. */
int zpx_debug_inflate_parallel(const uint8_t *z, size_t len, uint8_t *out, size_t want, int threads);
/* Test hook: the host stages of two PNGs as a batch worker runs them
 * together (their inflates in one loop): status[k] is what zpx_png_inflate
 * returns for buffer k, and *out_k its stream when that is ZPX_OK (free with
 * zpx_png_stream_free), else NULL.  Returns ZPX_OK or an argument error. */
int zpx_debug_png_inflate_pair(const uint8_t *buf0, size_t len0, const uint8_t *buf1, size_t len1,
                               zpx_png_stream **out0, zpx_png_stream **out1, int *status);

#ifdef __cplusplus
}
#endif
#endif /* ZPIX_AMD_H */
