// Band slab: the paired-row PNG kernel's input layout (png_pair_kernels.hip).
//
// The kernel reconstructs a band of 128 rows of a pass with lane j holding
// rows 2j and 2j+1; at group g (steps 8g .. 8g+7) row r reads the CB-byte
// chunks 8g - skew(r) .. 8g - skew(r) + 7 of its filtered bytes (the
// unfilter loop of readImagePass, src/png/decoder.zig:806-842, walks each
// row left to right; skew(r) = r - the last row <= r that restarts the
// dependency chain: a None / Sub row or the band's first).  Read from the
// inflated stream, each of the kernel's 16-byte loads touches 64 different
// rows -- 64 cache lines per instruction, which caps the read at ~2.5 TB/s
// (tools/ubench/png_load_pattern mode 0) against ~6 TB/s for 1 KiB
// contiguous per instruction (mode 2).  The slab stores each band's bytes in
// the order the kernel reads them:
//
//   slab   = u64 region offset per band (every band of every non-empty pass,
//            Adam7 order), then the regions, 256-byte aligned
//   region = the band's 128 filter-type bytes (0 for rows past the pass),
//            then per group g, tile h < 2, piece q < NQ: 1 KiB = 64 lanes x
//            16 bytes, piece h NQ + q of the lane's two group windows (rows
//            2 lane and 2 lane + 1, each from its chunk 8 g - skew(r) on,
//            zeros outside the row) interleaved two bytes at a time:
//            a0 a1 b0 b1 a2 a3 b2 b3 ... -- so a loaded dword holds two
//            byte pairs of the kernel's packed form (row 2j in the low
//            16-bit half, 2j+1 in the high) and the kernel unpacks with a
//            shift instead of a v_perm per pair
//
// NQ = 8 CB / 16 (6 for 3- and 6-byte pixels, else 8), and a band has
// ceil((chunks + max skew) / 8) groups, exactly the groups the kernel walks.
// The host builds it after inflate (one pass over the bytes); the skew rule
// here and in the kernel must agree (tests/test_abi.py checks the layout
// against a Python model, every -m gpu PNG test the kernel on it).
#include <emmintrin.h>

#include <algorithm>
#include <atomic>
#include <cstring>
#include <thread>

#include "api_internal.h"
#include "device_types.h"
#include "png_host.h"

namespace zpx {

namespace {

struct SlabGeom {
    int bpp = 0, cb = 16;
};

SlabGeom slab_geom(int depth)
{
    SlabGeom g;
    switch (depth) {
    case ZPX_PNG_G8: g.bpp = 1; break;
    case ZPX_PNG_G16: g.bpp = 2; break;
    case ZPX_PNG_TC8: g.bpp = 3; g.cb = 12; break;
    case ZPX_PNG_TCA8: g.bpp = 4; break;
    case ZPX_PNG_TC16: g.bpp = 6; g.cb = 12; break;
    case ZPX_PNG_TCA16: g.bpp = 8; break;
    default: break;
    }
    return g;
}

constexpr size_t kRegionAlign = 256;
size_t align_up(size_t x) { return (x + kRegionAlign - 1) & ~(kRegionAlign - 1); }

// skew(r) of the band's 128 rows, as the kernel computes them (ballots over
// rows that restart: row 0, a None / Sub row, a row past the pass); returns
// the largest skew of a row inside the pass
int band_skews(const uint8_t *ft, uint32_t rows, int skew[128])
{
    int last = 0, mx = 0;
    for (int r = 0; r < 128; r++) {
        const bool in = static_cast<uint32_t>(r) < rows;
        if (r == 0 || !in || ft[r] < 2) last = r;
        skew[r] = r - last;
        if (in) mx = std::max(mx, skew[r]);
    }
    return mx;
}

} // namespace

size_t png_slab_layout(const zpx_png_frame &f, std::vector<uint64_t> &band_off)
{
    band_off.clear();
    const SlabGeom sg = slab_geom(f.depth);
    if (!sg.bpp) return 0;
    std::vector<DevPngPass> passes;
    std::vector<uint32_t> rowbytes;
    uint64_t bytes = 0;
    zpx_png_frame hf = f;
    hf.layout = ZPX_PNG_LAYOUT_STREAM;
    png_frame_passes(hf, passes, rowbytes, bytes);
    const int c = sg.cb / sg.bpp, nq = 8 * sg.cb / 16;
    size_t nb = 0;
    for (const DevPngPass &p : passes) nb += (p.rows + 127) / 128;
    size_t off = align_up(nb * sizeof(uint64_t));
    for (const DevPngPass &p : passes) {
        const uint32_t rb = p.row_bytes;
        const int nchunks = static_cast<int>((p.width + c - 1) / c);
        for (uint32_t base = 0; base < p.rows; base += 128) {
            const uint32_t rows = std::min(128u, p.rows - base);
            uint8_t ft[128] = {};
            for (uint32_t r = 0; r < rows; r++) ft[r] = p.filtered[size_t(base + r) * (rb + 1)];
            int skew[128];
            const int ngroups = (nchunks + band_skews(ft, rows, skew) + 7) / 8;
            band_off.push_back(off);
            off = align_up(off + 128 + size_t(ngroups) * 2 * nq * 1024);
        }
    }
    return off;
}

namespace {

// one band's region: filter bytes, the groups in the kernel's read order,
// the alignment tail
void fill_band(const DevPngPass &p, const SlabGeom &sg, uint32_t base, uint8_t *slab, size_t off)
{
    uint8_t *region = slab + off;
    const int c = sg.cb / sg.bpp, nq = 8 * sg.cb / 16;
    const uint32_t rb = p.row_bytes;
    const int nchunks = static_cast<int>((p.width + c - 1) / c);
    const uint32_t rows = std::min(128u, p.rows - base);
    uint8_t *ft = region;
    memset(ft, 0, 128);
    for (uint32_t r = 0; r < rows; r++) ft[r] = p.filtered[size_t(base + r) * (rb + 1)];
    int skew[128];
    const int ngroups = (nchunks + band_skews(ft, rows, skew) + 7) / 8;
    const size_t gbytes = size_t(2) * nq * 1024;
    uint8_t *groups = region + 128;
    const uint8_t *rowp[128];
    for (int r = 0; r < 128; r++)
        rowp[r] = static_cast<uint32_t>(r) < rows ? p.filtered + size_t(base + r) * (rb + 1) + 1 : nullptr;
    // destination order: each group's two NQ KiB tiles are written lane by
    // lane from the lane's two rows' windows (16 NQ bytes each), their
    // 16-byte pieces interleaved by 16-bit units (unpacklo / unpackhi)
    auto window = [&](int r, int g, int q, __m128i &v) {
        const uint8_t *row = rowp[r];
        const int64_t start = (int64_t(8) * g - skew[r]) * sg.cb + 16 * q; // this piece's first byte
        if (row && start >= 0 && start + 16 <= int64_t(rb)) {
            v = _mm_loadu_si128(reinterpret_cast<const __m128i *>(row + start));
            return;
        }
        alignas(16) uint8_t piece[16];
        for (int i = 0; i < 16; i++) {
            const int64_t x = start + i;
            piece[i] = (row && x >= 0 && x < int64_t(rb)) ? row[x] : 0;
        }
        v = _mm_load_si128(reinterpret_cast<const __m128i *>(piece));
    };
    for (int g = 0; g < ngroups; g++) {
        uint8_t *gdst = groups + size_t(g) * gbytes;
        for (int lane = 0; lane < 64; lane++)
            for (int q = 0; q < nq; q++) {
                __m128i a, b;
                window(2 * lane, g, q, a);
                window(2 * lane + 1, g, q, b);
                // pieces 2q and 2q + 1 of the interleaved pair: tile p / NQ, piece p % NQ
                const int p0 = 2 * q, p1 = 2 * q + 1;
                _mm_storeu_si128(reinterpret_cast<__m128i *>(gdst + size_t(p0 / nq) * nq * 1024 + size_t(p0 % nq) * 1024 +
                                                             size_t(lane) * 16),
                                 _mm_unpacklo_epi16(a, b));
                _mm_storeu_si128(reinterpret_cast<__m128i *>(gdst + size_t(p1 / nq) * nq * 1024 + size_t(p1 % nq) * 1024 +
                                                             size_t(lane) * 16),
                                 _mm_unpackhi_epi16(a, b));
            }
    }
    const size_t end = off + 128 + size_t(ngroups) * gbytes; // (the next region starts at its alignment)
    memset(slab + end, 0, align_up(end) - end);
}

} // namespace

void png_slab_fill(const zpx_png_frame &f, const std::vector<uint64_t> &band_off, uint8_t *out, int threads)
{
    const SlabGeom sg = slab_geom(f.depth);
    std::vector<DevPngPass> passes;
    std::vector<uint32_t> rowbytes;
    uint64_t bytes = 0;
    zpx_png_frame hf = f;
    hf.layout = ZPX_PNG_LAYOUT_STREAM;
    png_frame_passes(hf, passes, rowbytes, bytes);
    const size_t nb = band_off.size();
    memcpy(out, band_off.data(), nb * sizeof(uint64_t));
    memset(out + nb * sizeof(uint64_t), 0, align_up(nb * sizeof(uint64_t)) - nb * sizeof(uint64_t));
    struct Job {
        const DevPngPass *p;
        uint32_t base;
    };
    std::vector<Job> jobs;
    for (const DevPngPass &p : passes)
        for (uint32_t base = 0; base < p.rows; base += 128) jobs.push_back(Job{&p, base});
    auto run = [&](size_t b) { fill_band(*jobs[b].p, sg, jobs[b].base, out, band_off[b]); };
    const int nthr = std::max(1, std::min<int>(threads, static_cast<int>(nb)));
    std::atomic<size_t> next_job{0};
    auto worker = [&] {
        for (size_t b; (b = next_job.fetch_add(1)) < nb;) run(b);
    };
    std::vector<std::thread> pool;
    try {
        for (int i = 1; i < nthr; i++) pool.emplace_back(worker);
    } catch (...) {
        // (thread creation failed: this thread does the remaining bands)
    }
    worker();
    for (auto &t : pool) t.join();
}

int png_slab_chunk_bytes(int depth)
{
    const SlabGeom sg = slab_geom(depth);
    return sg.bpp ? sg.cb : 0;
}

namespace {
// the passes of f in stream layout (their `filtered` = offsets from f.filtered)
void stream_passes(const zpx_png_frame &f, std::vector<DevPngPass> &passes)
{
    std::vector<uint32_t> rowbytes;
    uint64_t bytes = 0;
    zpx_png_frame hf = f;
    hf.layout = ZPX_PNG_LAYOUT_STREAM;
    png_frame_passes(hf, passes, rowbytes, bytes);
}
// groups of a band of `rows` rows with chunks per row `nchunks`, for its
// largest possible skew
uint32_t worst_groups(uint32_t nchunks, uint32_t rows)
{
    return (nchunks + std::min(127u, rows ? rows - 1 : 0u) + 7) / 8;
}
} // namespace

size_t png_dev_slab_layout(const zpx_png_frame &f, std::vector<uint64_t> &band_off)
{
    band_off.clear();
    const SlabGeom sg = slab_geom(f.depth);
    if (!sg.bpp) return 0;
    std::vector<DevPngPass> passes;
    stream_passes(f, passes);
    const int c = sg.cb / sg.bpp, nq = 8 * sg.cb / 16;
    size_t nb = 0;
    for (const DevPngPass &p : passes) nb += (p.rows + 127) / 128;
    size_t off = align_up(nb * sizeof(uint64_t));
    for (const DevPngPass &p : passes) {
        const uint32_t nchunks = (p.width + c - 1) / c;
        for (uint32_t base = 0; base < p.rows; base += 128) {
            band_off.push_back(off);
            off = align_up(off + 128 + size_t(worst_groups(nchunks, std::min(128u, p.rows - base))) * 2 * nq * 1024);
        }
    }
    return off;
}

void png_dev_slab_jobs(const zpx_png_frame &f, const std::vector<uint64_t> &band_off, const uint8_t *d_stream,
                       size_t stream_len, uint8_t *d_slab, std::vector<DevSlabBand> &jobs, uint32_t &max_groups)
{
    const SlabGeom sg = slab_geom(f.depth);
    std::vector<DevPngPass> passes;
    stream_passes(f, passes);
    const int c = sg.cb / sg.bpp;
    size_t b = 0, at = 0; // band index, stream offset of the pass
    for (const DevPngPass &p : passes) {
        const uint32_t nchunks = (p.width + c - 1) / c;
        for (uint32_t base = 0; base < p.rows; base += 128, b++) {
            DevSlabBand j{};
            const size_t first = at + size_t(base) * (size_t(p.row_bytes) + 1);
            j.rows0 = d_stream + first;
            j.region = d_slab + band_off[b];
            const size_t avail = stream_len > first ? stream_len - first : 0;
            j.avail = static_cast<uint32_t>(std::min<size_t>(avail, 0x7fffff00u));
            j.rows = std::min(128u, p.rows - base);
            j.rb = p.row_bytes;
            j.nchunks = nchunks;
            max_groups = std::max(max_groups, worst_groups(nchunks, j.rows));
            jobs.push_back(j);
        }
        at += size_t(p.rows) * (size_t(p.row_bytes) + 1);
    }
}

int png_stream_build_slab(PngStream &ps, int threads)
{
    if (ps.slab_len) return ZPX_OK;
    if (!png_use_pair(ps.depth, ps.interlace, ps.use_transparent, ps.width, size_t(ps.width) * ps.out_bpp))
        return ZPX_E_UNSUPPORTED;
    zpx_png_frame f;
    memset(&f, 0, sizeof(f));
    f.width = ps.width;
    f.height = ps.height;
    f.depth = ps.depth;
    f.interlace = ps.interlace;
    f.use_transparent = ps.use_transparent ? 1 : 0;
    memcpy(f.transparent, ps.transparent, 6);
    f.filtered = static_cast<const uint8_t *>(ps.data.ptr);
    f.out_stride = size_t(ps.width) * ps.out_bpp;
    std::vector<uint64_t> off;
    const size_t n = png_slab_layout(f, off);
    if (!n) return ZPX_E_UNSUPPORTED;
    if (!ps.slab.alloc(n, false)) return ZPX_E_OUT_OF_MEMORY;
    png_slab_fill(f, off, static_cast<uint8_t *>(ps.slab.ptr), threads);
    ps.slab_len = n;
    return ZPX_OK;
}

} // namespace zpx
