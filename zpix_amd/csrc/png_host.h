// Host (serial) half of png.decode: signature, chunk walk with CRC checks,
// IHDR/PLTE/tRNS/IDAT handling and zlib inflate into pinned memory.  Filter
// reconstruction and pixel store run on the GPU (png_kernels.hip).
#pragma once

#include <cstddef>
#include <cstdint>

#include "jpeg_host.h" // HostBuf
#include "zpix_amd.h"

namespace zpx {

struct PngPassInfo {
    uint32_t width = 0, rows = 0;   // pass pixel dims (0 = empty pass)
    uint32_t row_bytes = 0;         // without the filter byte
    uint32_t xo = 0, yo = 0, xf = 1, yf = 1;
    size_t offset = 0;              // of the pass's first filter byte in the stream
};

struct PngStream {
    uint32_t width = 0, height = 0;
    int depth = 0;                  // zpx_png_depth
    int interlace = 0;
    bool use_transparent = false;
    uint8_t transparent[6] = {};
    zpx_color palette[256] = {};
    int palette_len = 0;
    bool has_palette = false;
    int kind = ZPX_GRAY;            // image type readImagePass allocates
    int out_bpp = 1;                // bytes per output pixel
    int npasses = 0;
    PngPassInfo pass[7];
    HostBuf data;                   // inflated stream (+ZPX_PNG_INPUT_PAD)
    size_t data_len = 0;            // bytes the passes consume
    HostBuf slab;                   // band slab of `data` (png_slab.cpp), when built
    size_t slab_len = 0;
};

// The band slab of ps.data for the paired-row kernel (png_slab.cpp), into
// ps.slab, bands split over `threads` threads: ZPX_OK, ZPX_E_UNSUPPORTED
// when that kernel does not take the image, ZPX_E_OUT_OF_MEMORY.
int png_stream_build_slab(PngStream &ps, int threads = 1);

// Parse + inflate.  On success every row's data is present and every filter
// byte is valid; otherwise returns the reference's error for the first row
// that would fail (EndOfStream / ReadFailed / InvalidFilterType) or the
// chunk-level error.
// threads > 1: a large stream inflates on that many threads (inflate_parallel)
int png_parse(const uint8_t *buf, size_t len, PngStream &out, int threads = 1);
// Two PNGs' host stages on this thread, their inflates in one loop
// (inflate_fast_pair: two decode chains overlap on a core): status[k] is
// png_parse(buf[k], len[k], *out[k]).
int png_parse_pair(const uint8_t *const buf[2], const size_t len[2], PngStream *const out[2], int status[2]);
// default inflate threads of the single-image entry points: ZPX_INFLATE_THREADS,
// else min(8, hardware threads)
int png_inflate_threads();
// Releases the host stages' recycled buffers (the IDAT pool here, the
// parallel inflate's symbol pool): the bytes released (zpx_host_pools_trim)
size_t png_pool_trim();

// Signature + IHDR only (dimensions of the image png.decode would return).
int png_decode_config(const uint8_t *buf, size_t len, uint32_t &w, uint32_t &h);

} // namespace zpx
