// Host (serial) half of jpeg.decode: marker parsing, DHT/DQT/SOF/SOS and the
// Huffman / progressive-refinement entropy decoder.  It never reconstructs
// pixels: every scan writes into coefficient grids (the accumulate form of
// processSos, src/jpeg/decoder.zig:1340-1345) that the GPU consumes.
#pragma once

#include <cstddef>
#include <cstdint>
#include <utility>
#include <vector>

#include "zpix_amd.h"

namespace zpx {

// Host buffer that prefers pinned (page-locked) memory so H2D copies are
// DMA-direct; falls back to ordinary memory when no HIP device is usable.
// Pinned buffers are recycled through a process-wide pool (hipHostMalloc of a
// 50 MB grid costs milliseconds; a batch decodes thousands of them).
struct HostBuf {
    void *ptr = nullptr;
    size_t bytes = 0;
    size_t cap = 0; // allocation size (pool size class) of a pinned buffer
    bool pinned = false;
    HostBuf() = default;
    HostBuf(const HostBuf &) = delete;
    HostBuf &operator=(const HostBuf &) = delete;
    HostBuf(HostBuf &&o) noexcept { *this = static_cast<HostBuf &&>(o); }
    HostBuf &operator=(HostBuf &&o) noexcept;
    ~HostBuf() { release(); }
    bool alloc(size_t n, bool zero);
    void release();
};

// Block rule per component (see zpx_block_rule).
struct JpegComponent {
    int32_t h = 0, v = 0;
    uint8_t id = 0, tq = 0;
};

class CoeffGrid {
  public:
    // Blocks of 64 natural-order coefficients, stored in the narrowest of
    // int8 / int16 / int32 that holds every value so far: a grid starts as
    // int8 and is widened (copied) the first time a value does not fit.
    // Conforming 8-bit streams never need int32; the bench's q75 frames fit
    // int8, natural photos usually need int16 (iceberg.jpg: max |AC| 157).
    bool init(size_t blocks, bool zero = true, int bits = 8); // zero = false: every block will be stored
    int bits() const { return bits_; }
    bool wide() const { return bits_ == 32; }
    size_t blocks() const { return blocks_; }
    const void *data() const { return buf_.ptr; }
    size_t bytes() const { return blocks_ * 64 * (bits_ / 8); }
    void load(size_t blk, int32_t *b) const;
    bool store(size_t blk, const int32_t *b); // false only on allocation failure
    // Baseline fast path: the block is zero except at the n natural-order
    // positions pos[] (all distinct).
    bool store_sparse(size_t blk, const int32_t *b, const uint8_t *pos, int n);
    bool widen_to(int bits);                  // no-op when already that wide
    // One coefficient (natural index i of block blk), for the progressive
    // scans, which touch only their band's coefficients: set widens as store.
    int32_t get(size_t blk, int i) const
    {
        const size_t k = blk * 64 + static_cast<size_t>(i);
        return bits_ == 8 ? static_cast<const int8_t *>(buf_.ptr)[k]
                          : bits_ == 16 ? static_cast<const int16_t *>(buf_.ptr)[k] : static_cast<const int32_t *>(buf_.ptr)[k];
    }
    bool set(size_t blk, int i, int32_t v);
    // The parallel progressive scans write an int16 grid directly (no
    // widening); afterwards the grid takes the running max and, when every
    // value fits, narrows to int8 (`threads` share the copy).
    int16_t *data16() { return bits_ == 16 ? static_cast<int16_t *>(buf_.ptr) : nullptr; }
    void note_max_abs(int32_t m) { max_abs_ = m > max_abs_ ? m : max_abs_; }
    bool narrow_to8(int threads);
    // Concurrent stores into the grid at its current width: disjoint blocks
    // from several threads, no widening; a value too wide for the grid goes
    // to `overflow` (element index, value) and the running max |value| to
    // max_abs.  After the threads: apply_overflow widens to the width the
    // max needs and writes the overflowed values.
    bool store_sparse_fixed(size_t blk, const int32_t *b, const uint8_t *pos, int n, int32_t &max_abs,
                            std::vector<std::pair<size_t, int32_t>> &overflow) const;
    bool apply_overflow(int32_t max_abs, const std::vector<std::pair<size_t, int32_t>> &overflow);
    int32_t max_abs() const { return max_abs_; }

  private:
    HostBuf buf_;
    size_t blocks_ = 0;
    int bits_ = 8;
    int32_t max_abs_ = 0;
};

// Compact coefficient blocks ("pieces"): the batch pipeline's H2D form of a
// baseline frame whose one scan interleaves every component.
// A block keeps its coefficients in zig-zag order up to its last nonzero one
// (the end of block of processSos, src/jpeg/decoder.zig:1300-1345) as whole
// 16-byte pieces of int8 (16 coefficients a piece) or int16 (8) values, the
// rest of the last piece zero; piece 0 is all zeros.  Per component a u32 per
// block, in grid order, indexes them:
//   index = first piece << 4 | pieces   (pieces 0: the block is all zeros)
// The block kernels read the pieces straight into their LDS coefficient
// image -- a piece past a block's count reads piece 0 -- so no dense grid is
// ever written or read back (jpeg_block_kernels.hip); the other kernels take
// grids expanded from them on the device (launch_jpeg_pieces_expand).
// The width starts at int8 and is widened (every piece so far copied) the
// first time a value does not fit.
//
// Pieces are stored per block row class: stream (c, yy) holds the pieces of
// component c's blocks in block rows by with by mod v_c == yy, in grid order
// (for 4:2:0: Y's even block rows, Y's odd block rows, Cb, Cr).  So the 64
// blocks a kernel task reads from one block row of one component have their
// pieces in one contiguous span, as a dense grid's 64 blocks are -- not
// spread over the MCU row between the other rows' and components' pieces,
// as decode order leaves them.  While decoding, stream s fills its own
// region [base[s], base[s] + 8 x its blocks) of the allocation; compact()
// closes the gaps once the scan is done (a memmove of the streams after the
// first and one pass over the index words).
struct JpegPieces {
    static constexpr int kMaxStreams = 16;
    bool valid = false;
    int bits = 8;                 // 8 or 16: the values of every piece
    HostBuf data;                 // npieces x 16 bytes
    HostBuf index;                // u32 per block: component c's blocks from first[c]
    size_t first[4] = {0, 0, 0, 0}, blocks[4] = {0, 0, 0, 0};
    size_t npieces = 0, cap = 0;  // pieces (after compact()) / allocated
    int32_t max_abs[4] = {0, 0, 0, 0};
    // streams: component c's are s0[c] .. s0[c] + v[c] - 1 (block row mod v[c])
    int nstreams = 0, s0[4] = {0, 0, 0, 0}, v[4] = {1, 1, 1, 1};
    size_t gw[4] = {1, 1, 1, 1};  // component c's grid width in blocks
    size_t base[kMaxStreams] = {}, next[kMaxStreams] = {};
    int stream_of(int c, size_t blk) const { return s0[c] + static_cast<int>((blk / gw[c]) % size_t(v[c])); }
    size_t data_bytes() const { return npieces * 16; }
    uint32_t *index_of(int c) const { return static_cast<uint32_t *>(index.ptr) + first[c]; }
    bool widen(); // int8 -> int16 pieces
    void compact(); // the streams back to back from piece 1; sets npieces
};

struct JpegCoeffs {
    uint32_t width = 0, height = 0;
    int n_comp = 0;
    JpegComponent comp[4];
    int32_t mxx = 0, myy = 0;
    bool progressive = false, baseline = false;
    bool jfif = false, adobe_valid = false;
    int adobe_transform = 0;
    int rule[4] = {ZPX_BLOCKS_NONE, ZPX_BLOCKS_NONE, ZPX_BLOCKS_NONE, ZPX_BLOCKS_NONE};
    CoeffGrid grid[4];
    bool has_grid[4] = {false, false, false, false};
    // quant table each component is reconstructed with, natural order
    int32_t qt_natural[4][64] = {};
    int32_t max_q[4] = {0, 0, 0, 0};
    JpegPieces pieces; // valid: the scan's coefficients are compact pieces, not grids
};

// Decode `buf` into coefficient grids.  Returns ZPX_E_* (ZPX_E_OK on success),
// with the reference's error for malformed input.
// Host entropy stage; on success every grid of the frame has the same
// coefficient width (the widest any grid needed).
// threads > 1: baseline scans with a restart interval decode their restart
// segments in parallel (identical result; anything irregular falls back to
// the serial loop).
// pieces: a baseline frame whose one scan interleaves every component (and is
// not split by restart intervals over threads) is decoded into out.pieces
// instead of grids; anything else decodes into grids as usual.
int jpeg_entropy_decode(const uint8_t *buf, size_t len, JpegCoeffs &out, int threads = 1, bool pieces = false);
// default thread count of the single-image entry points: ZPX_HUFF_THREADS,
// else min(8, hardware threads)
int jpeg_huff_threads();
int64_t jpeg_parallel_scans(); // scans decoded restart-interval-parallel so far
int64_t jpeg_parallel_progressive(); // progressive frames decoded scan-parallel so far

// jpeg.decodeConfig (decoder.zig:178-218): markers up to SOF (JFIF) or SOS,
// skipping DQT/DRI/DHT.  model: ZPX_MODEL_GRAY or ZPX_MODEL_YCBCR.
int jpeg_decode_config(const uint8_t *buf, size_t len, uint32_t &w, uint32_t &h, int &model);

// Output kind decodeInner would return (decoder.zig:361-372).
enum class JpegOut { Gray, YCbCr, RGB, CMYK, YCCK };
JpegOut jpeg_output_kind(const JpegCoeffs &c);

// makeImg layout (decoder.zig:1708-1783, image.zig:484-555).
struct JpegLayout {
    int subsample = ZPX_RATIO444;
    size_t y_stride = 0, c_stride = 0, k_stride = 0;
    size_t y_rows = 0, c_rows = 0, k_rows = 0;
    size_t cb_off = 0, cr_off = 0, total = 0, k_total = 0;
};
int jpeg_layout(const JpegCoeffs &c, JpegLayout &l);

} // namespace zpx
