// Host-side planning logic of the PNG path, checked without a GPU (built and
// run by tests/test_host_logic.py against libzpix_amd.so):
//   - png_schedule (api_internal.h): every band's predecessor in its pass holds
//     a lower ticket (the kernels' no-deadlock rule), and tickets go longest
//     row first;
//   - png_adam7_stage / png_adam7_rebase: passes 1-6 redirected into
//     disjoint, aligned staging rows with xf = yf = 1, pass 7 untouched, and
//     merge jobs whose stage pointers and strides match the redirected passes;
//   - dev_jpeg_frame: the quant-pair tables of the block kernel's row pass.
// Prints "ok" and exits 0, or names the first failed check and exits 1.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <vector>

#include "api_internal.h"

using namespace zpx;

static int fails = 0;
#define CHECK(c)                                                                                                       \
    do {                                                                                                               \
        if (!(c)) {                                                                                                    \
            fprintf(stderr, "check failed: %s (line %d)\n", #c, __LINE__);                                           \
            fails++;                                                                                                   \
        }                                                                                                              \
    } while (0)

static void check_schedule(const std::vector<DevPngPass> &passes, uint32_t band_rows)
{
    std::vector<DevPngPass> p = passes;
    uint32_t nb = 0;
    for (auto &d : p) {
        d.nbands = (d.rows + band_rows - 1) / band_rows;
        d.band_base = nb;
        nb += d.nbands;
    }
    const std::vector<DevPngBand> s = png_schedule(p, band_rows);
    CHECK(s.size() == nb);
    std::map<std::pair<uint32_t, uint32_t>, size_t> ticket;
    for (size_t t = 0; t < s.size(); t++) ticket[{s[t].pass, s[t].band}] = t;
    CHECK(ticket.size() == nb); // every band exactly once
    for (size_t t = 0; t < s.size(); t++) {
        if (s[t].band > 0) CHECK(ticket.at({s[t].pass, s[t].band - 1}) < t);
        if (t > 0) CHECK(p[s[t - 1].pass].row_bytes >= p[s[t].pass].row_bytes); // longest first
    }
}

int main()
{
    // ---- a batch: two Adam7 RGBA16 images (one ragged), one flat tc8 image
    struct Img { uint32_t w, h; int depth, interlace, obpx; };
    const Img imgs[] = {{4096, 4096, ZPX_PNG_TCA16, 1, 8}, {77, 45, ZPX_PNG_TCA16, 1, 8}, {301, 97, ZPX_PNG_TC8, 0, 4}};
    std::vector<DevPngPass> passes;
    std::vector<uint32_t> rowbytes;
    uint64_t bytes = 0;
    Adam7Stage st;
    std::vector<uint8_t> fake_out(16);
    std::vector<size_t> first_of;
    for (const Img &im : imgs) {
        zpx_png_frame f;
        memset(&f, 0, sizeof(f));
        f.width = im.w;
        f.height = im.h;
        f.depth = im.depth;
        f.interlace = im.interlace;
        f.out = fake_out.data();
        f.out_stride = uint64_t(im.w) * im.obpx;
        const size_t first = passes.size();
        first_of.push_back(first);
        png_frame_passes(f, passes, rowbytes, bytes);
        CHECK(passes.size() - first == (im.interlace ? 7u : 1u));
        if (im.interlace) png_adam7_stage(f, im.obpx, passes, first, st);
    }
    check_schedule(passes, 128);
    check_schedule(passes, 64);

    CHECK(st.jobs.size() == 2);
    CHECK(st.staged.size() == 12);
    CHECK(st.max_erows == 2048);
    std::vector<uint8_t> staging(st.bytes + 256);
    uint8_t *base = reinterpret_cast<uint8_t *>((reinterpret_cast<uintptr_t>(staging.data()) + 255) & ~uintptr_t(255));
    png_adam7_rebase(passes, st, base);
    // staged passes: contiguous, aligned, disjoint rows inside the staging area
    std::vector<std::pair<uint8_t *, uint8_t *>> spans;
    for (size_t i : st.staged) {
        const DevPngPass &d = passes[i];
        CHECK(d.xf == 1 && d.yf == 1 && d.xo == 0 && d.yo == 0);
        CHECK(d.out_stride % 128 == 0 && d.out_stride >= uint64_t(d.width) * 8);
        CHECK((reinterpret_cast<uintptr_t>(d.out) & 255) == 0);
        CHECK(d.out >= base && d.out + d.out_stride * d.rows <= base + st.bytes);
        spans.push_back({d.out, d.out + d.out_stride * d.rows});
    }
    for (size_t a = 0; a < spans.size(); a++)
        for (size_t b = a + 1; b < spans.size(); b++)
            CHECK(spans[a].second <= spans[b].first || spans[b].second <= spans[a].first);
    // pass 7 of each Adam7 image still writes the odd rows of the image
    for (int k = 0; k < 2; k++) {
        const DevPngPass &p7 = passes[first_of[k] + 6];
        CHECK(p7.xo == 0 && p7.yo == 1 && p7.xf == 1 && p7.yf == 2 && p7.out == fake_out.data());
    }
    // merge jobs name the same staging rows as the redirected passes, by Adam7 pass
    for (int k = 0; k < 2; k++) {
        const DevAdam7Merge &m = st.jobs[k];
        CHECK(m.width == imgs[k].w && m.height == imgs[k].h && m.out == fake_out.data());
        for (int p = 0; p < 6; p++) {
            const DevPngPass &d = passes[first_of[k] + p];
            CHECK(m.stage[p] == d.out && m.sstride[p] == d.out_stride);
        }
    }

    // ---- quant-pair tables of dev_jpeg_frame
    zpx_jpeg_frame jf;
    memset(&jf, 0, sizeof(jf));
    jf.n_comp = 3;
    for (int c = 0; c < 4; c++)
        for (int i = 0; i < 64; i++) jf.qt[c][i] = (c + 1) * 1000 + i * 257;
    const DevJpegFrame df = dev_jpeg_frame(jf);
    const int lo[4] = {1, 5, 2, 0}, hi[4] = {7, 3, 6, 4};
    for (int c = 0; c < 3; c++)
        for (int r = 0; r < 8; r++)
            for (int k = 0; k < 4; k++) {
                const uint32_t v = df.qp[c][4 * r + k];
                CHECK((v & 0xffff) == uint32_t(jf.qt[c][8 * r + lo[k]]) && (v >> 16) == uint32_t(jf.qt[c][8 * r + hi[k]]));
            }

    if (fails) return 1;
    printf("ok\n");
    return 0;
}
