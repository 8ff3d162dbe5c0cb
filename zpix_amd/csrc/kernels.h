// Launchers of the gfx950 kernels (implemented in the .hip translation units).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "device_types.h"
#include "zpix_amd.h"

namespace zpx {

// jpeg_kernels.hip
// coeff_bits: 8, 16 or 32 (int8 / int16 / int32 coefficient grids)
// The planar output (jpeg.load) of frames of one geometry: ncomp components
// sampled h[c] x v[c] (gray: 1 x 1), MCU grids up to max_mxx x max_myy.
struct JpegPlaneGeom {
    int ncomp = 0;
    int h[4] = {1, 1, 1, 1}, v[4] = {1, 1, 1, 1};
    int max_mxx = 0, max_myy = 0;
};
// pieces: the frames are ZPX_COEFFS_PIECES (only the block kernels read
// them: -2 when they do not take the frames -- expand them first)
int launch_jpeg_planar(const DevJpegFrame *d_frames, int n_frames, const JpegPlaneGeom &geom, int coeff_bits,
                       bool narrow, bool pieces, hipStream_t stream);
bool jpeg_rgba_supported(int color, int h0, int v0, int hc, int vc);
// vec_out: every frame's RGBA rows are dword aligned (jpeg_rgba_vec_out:
// the block-per-lane kernel's store layout)
int launch_jpeg_rgba(const DevJpegFrame *d_frames, int n_frames, int color, int h0, int v0, int hc, int vc,
                     int max_mxx, int max_myy, int coeff_bits, bool narrow, bool vec_out, bool pieces,
                     hipStream_t stream);

// jpeg_block_kernels.hip: -2 when the frame kind is not one it takes
int launch_jpeg_block(const DevJpegFrame *d_frames, int n_frames, int color, int h0, int v0, int hc, int vc,
                      int max_mxx, int max_myy, int coeff_bits, bool narrow, bool pieces, hipStream_t stream);
// the fused kernel's ZPX_COEFFS_PIECES instances: YCbCr 4:2:0 / 4:2:2 / 4:4:0 / 4:4:4
bool jpeg_block_pieces_supported(int color, int h0, int v0, int hc, int vc);
// the planar block kernel (narrow int8 / int16 frames); -2 for the rest
int launch_jpeg_plane_block(const DevJpegFrame *d_frames, int n_frames, const JpegPlaneGeom &geom, int coeff_bits,
                            bool narrow, bool pieces, hipStream_t stream);
// ZPX_COEFFS_PIECES -> dense natural-order grids (njobs components, up to
// max_blocks blocks each)
int launch_jpeg_pieces_expand(const DevPiecesExpand *jobs, int njobs, uint32_t max_blocks, int coeff_bits,
                              hipStream_t stream);

// png_kernels.hip
// CUs of the current device (read once: the node's GPUs are alike; a
// function-local static, so concurrent first calls from the per-device
// pipeline threads are safe)
int device_cu_count();
int png_chunk_bytes(int depth);
// uint64 granules of boundary buffer per band for rows of up to max_row_bytes
int png_band_granules(int depth, uint32_t max_row_bytes);
// ctl: 4 device words {epoch, ticket, status, pad}; boundary: nbands * band_granules.
// spin_limit: polls per boundary wait before the launch gives up and sets
// the status word (0 = the default, env ZPX_PNG_SPIN_LIMIT or 2^20).
int launch_png_unfilter(int depth, const DevPngPass *passes, const DevPngBand *sched, uint32_t nsched,
                        uint32_t *ctl, uint64_t *boundary, uint32_t band_granules, hipStream_t s,
                        uint32_t spin_limit = 0);

uint32_t png_default_spin_limit();

// png_pair_kernels.hip: two rows per lane, 128-row bands (the byte-aligned
// depths whose chunk is 16 output bytes); the rest take launch_png_unfilter
bool png_pair_supported(int depth, int interlace, bool use_trns, uint32_t width, uint64_t out_stride);
// trns: the images carry a tRNS colour key (RGB8 / RGB16; one value per
// launch); stream: the passes' `filtered` is the inflated stream itself
// (ZPX_PNG_LAYOUT_STREAM), else their band slabs
int launch_png_pair(int depth, bool trns, bool stream, const DevPngPass *passes, const DevPngBand *sched,
                    uint32_t nsched, uint32_t *ctl, uint64_t *boundary, uint32_t band_granules, hipStream_t s,
                    uint32_t spin_limit = 0);
// the second launch of an Adam7 group: its pass-6 bands (sched), merged with
// the staged passes 1-5 into whole even rows (the 4- and 8-byte-pixel depths)
int launch_png_pair_merge(int depth, bool trns, bool stream, const DevPngPass *passes, const DevPngBand *sched,
                          uint32_t nsched, uint32_t *ctl, uint64_t *boundary, uint32_t band_granules, hipStream_t s);

// png_slab_kernels.hip: the band slab of `njobs` bands built on the device
// (cb: the depth's chunk bytes, 12 or 16; max_groups: the most groups any of
// the bands can have)
int launch_png_slab(int cb, const DevSlabBand *jobs, uint32_t njobs, uint32_t max_groups, hipStream_t s);

int launch_rgba_pixels(const DevImage &m, uint8_t *out, hipStream_t s);
// the batched form's job for one image (vec: the aligned vector path applies)
DevRgbaJob rgba_job(const DevImage &m, uint8_t *out);
// Image.rgbaPixels of n images of one kind (grid z = image; rows up to max_h)
int launch_rgba_batch(int kind, const DevRgbaJob *jobs, int n, int max_w, int max_h, hipStream_t s);
int launch_jpeg_rgb(const DevImage &m, int c_scale, uint8_t *out, hipStream_t s);
int launch_jpeg_cmyk(const DevImage &m, const uint8_t *k_plane, uint64_t k_stride, uint32_t sub_mask,
                     uint8_t *out, hipStream_t s);

// bmp_kernels.hip: the pixel loop of bmp.decode over the file's row data
// (bpp 1/2/4/8 -> palette indices, 24 -> RGBA, 32 -> NRGBA)
int launch_bmp_rows(int bpp, bool allow_alpha, const uint8_t *src, uint64_t row_bytes, uint8_t *dst,
                    uint64_t dst_stride, uint32_t width, uint32_t height, int top_down, hipStream_t s);

// qoi_kernels.hip: qoi.encode as a segmented scan (see the file header)
struct QoiEncodeArgs {
    const uint8_t *pixels = nullptr; // device, width*height*channels bytes
    uint64_t n = 0;                  // pixels
    uint32_t S = 0, nseg = 0, slot_words = 0;
    uint32_t width = 0, height = 0, colorspace = 0;
    uint8_t *out = nullptr;          // device, >= qoi bound bytes
    uint64_t *out_len = nullptr;     // device
    uint32_t *seg_tbl = nullptr, *seg_run = nullptr, *seg_cnt = nullptr;
    uint64_t *seg_mask = nullptr;
    uint32_t *blk_tbl = nullptr, *blk_run = nullptr, *pre_tbl = nullptr, *pre_run = nullptr;
    uint64_t *blk_mask = nullptr, *blk_cnt = nullptr, *blk_off = nullptr;
    uint32_t *slots = nullptr;
};
// scratch bytes for n pixels in segments of S; with base != nullptr also
// points a's scratch fields into base
size_t qoi_scratch_layout(uint64_t n, uint32_t S, QoiEncodeArgs *a, uint8_t *base);
int launch_qoi_encode(int channels, const QoiEncodeArgs &a, hipStream_t st);

} // namespace zpx
