// Descriptors shared by the host planner and the gfx950 kernels.
#pragma once

#include <cstdint>

namespace zpx {

// One JPEG frame as the kernels see it (uploaded once per plan).
struct DevJpegFrame {
    const void *coeffs[4];   // (mxx*h) x (myy*v) blocks x 64 coefficients (int16 or int32)
    uint8_t *planes[4];      // planar output
    uint64_t strides[4];
    uint8_t *rgba;           // fused output
    uint64_t rgba_stride;
    int32_t width, height, mxx, myy;
    int32_t h[4], v[4];
    int32_t rule[4];
    int32_t n_comp, color;
    int32_t qt[4][64];       // natural order
    uint32_t qp[4][32];      // quant-pair tables of the block kernels' row pass, per component
                             // (per row r: (q1,q7), (q5,q3), (q2,q6), (q0,q4) as u16 pairs)
    const uint8_t *pieces;   // ZPX_COEFFS_PIECES: the 16-byte pieces; coeffs[c] are then the
                             // per-block index arrays (first piece << 4 | pieces), else null
};

// One component of a ZPX_COEFFS_PIECES frame expanded into its dense grid
// (jpeg_pieces_expand_kernel).
struct DevPiecesExpand {
    const uint32_t *index;
    const uint8_t *pieces;
    void *grid;
    uint32_t blocks;
    uint32_t pad;
};

// The planar block kernel's task space for one plan group (frames of one
// geometry), MCU row by MCU row: in each, per component c, vrows[c] block
// rows of segs[c] 64-block segments, tasks start[c] .. start[c+1) of the
// MCU row (start[c] = per_row for absent components) -- so the tasks that
// read one MCU row's coefficients run together (a ZPX_COEFFS_PIECES frame
// keeps an MCU's blocks side by side).
struct PlaneTaskGeom {
    int32_t segs[4], rows[4], start[4];
    int32_t hh[4], vv[4];    // 8 * h0 / h_c, 8 * v0 / v_c: the progressive block rule (decoder.zig:1649-1651)
    int32_t vrows[4];        // block rows of component c per MCU row (v_c)
    int32_t per_row, per_frame, total;
};

// One PNG unfilter job: a (pass of a) PNG image.  Rows are processed by the
// skewed wavefront kernel in bands of 64 rows (one row per lane).
struct DevAdam7Merge;
struct DevPngPass {
    const uint8_t *filtered; // first filter byte of this pass
    uint8_t *out;            // output image base
    const DevAdam7Merge *merge; // Adam7 pass 6 on the paired-row kernel: the staged passes 1-5 it merges
                                // into whole even rows (png_pair_kernels.hip), else null
    int32_t *max_index;      // paletted: max index seen (atomicMax), else null
    uint64_t out_stride;     // bytes between output rows of the full image
    uint32_t width;          // pixels in a pass row
    uint32_t rows;           // rows in the pass
    uint32_t row_bytes;      // filtered bytes per row without the filter byte
    uint32_t xo, yo, xf, yf; // Adam7 placement (0,0,1,1 when not interlaced)
    uint32_t nbands;         // ceil(rows / 64)
    uint32_t band_base;      // index of this pass's first band in the progress table
    uint8_t trns[6];         // tRNS colour key (raw bytes)
    uint8_t use_trns;
    uint8_t launch2; // paired-row kernel: the band runs in the group's second launch (Adam7 pass 6)
    uint8_t slab;    // paired-row kernel: `filtered` is the frame's band slab (png_slab.cpp), not the stream
    uint32_t slab_band0; // slab: this pass's first band in the slab's band offset table
};

// Adam7 on the paired-row kernel, per interlaced image: passes 1-5 are
// unfiltered into staging -- exactly the even-row, even-column pixels -- and
// pass 6 (the odd columns of the even rows) writes every even row y whole,
// taking its even columns x = 2X from the staging (png_pair_kernels.hip):
//   y = 2 mod 4:            pass 5 as is, S5[(y - 2) / 4][X]
//   y = 0 mod 4, X odd:     pass 4 as is, S4[y / 4][(X - 1) / 2]
//   y = 0 mod 4, X even:    Q2[y / 4][X / 2], Q2[Y][X'] = pixel (4X', 4Y):
//                           pass 3 its odd rows whole, passes 1 and 2 its
//                           even rows' even and odd columns
// so only passes 1 and 2 (1/32 of the pixels) store pixels apart.
struct DevAdam7Merge {
    const uint8_t *q2, *s4, *s5;
    uint64_t q2stride, s4stride, s5stride; // bytes between rows
    uint32_t width;           // image width in pixels
    uint32_t pad;
};

// One band of the device-built band slab (png_slab_kernels.hip): the
// paired-row kernel's input layout (png_slab.cpp) made on the device from
// the inflated stream.
struct DevSlabBand {
    const uint8_t *rows0; // the band's first row (its filter byte) in the stream
    uint8_t *region;      // the band's slab region: 128 filter bytes, then the groups
    uint32_t avail;       // stream bytes readable from rows0 (to the stream's end + pad)
    uint32_t rows;        // rows of the band in its pass (<= 128)
    uint32_t rb;          // filtered bytes per row, without the filter byte
    uint32_t nchunks;     // chunks per row
};

// A scheduled band: which pass and which band in it.  Bands are ordered so
// that band b of a pass always precedes band b+1 of the same pass.
struct DevPngBand {
    uint32_t pass;
    uint32_t band;
};

// PNG control block, kPngCtlWords device words:
//   {epoch, ticket, status, sticky, base, cycle, 0, 0}
// Each launch's control kernel moves `epoch` on with png_epoch_next; the
// block owns the epoch window [base, base + kPngEpochWindow) (PngControl,
// api_internal.h), base = window index * kPngEpochWindow with index >= 1,
// and its launches cycle through base + 1 .. base + cycle - 1 of it.  So an
// epoch is never 0 (the tag of never-written granules) nor another live
// block's, whatever the number of launches.
constexpr int kPngCtlWords = 8;
constexpr uint32_t kPngEpochWindow = 1u << 20;
constexpr uint32_t kPngEpochWindows = 4096; // (window 0 holds tag 0: never handed out)
// (constexpr: a host and device function both)
constexpr uint32_t png_epoch_next(uint32_t epoch, uint32_t base, uint32_t cycle)
{
    return epoch + 1u - base < cycle ? epoch + 1u : base + 1u;
}

} // namespace zpx

namespace zpx {

// An image.Image on the device (pixels / palette are device pointers).
struct DevImage {
    const uint8_t *pixels;
    const uint8_t *palette; // zpx_color entries
    uint64_t stride, y_off, cb_off, cr_off, y_stride, c_stride;
    int32_t kind, subsample, width, height, palette_len, pad;
};

// One image of a batched Image.rgbaPixels (zpx_rgba_plan_create).
struct DevRgbaJob {
    DevImage m;
    uint8_t *out;  // RGBA8, stride 4 * width
    int32_t vec;   // rows and out 16-byte aligned: whole 4-pixel pieces load and store as vectors
    int32_t pad;
};

} // namespace zpx
