// Host-side planning logic of the PNG path, checked without a GPU (built and
// run by tests/test_host_logic.py against libzpix_amd.so):
//   - png_schedule (api_internal.h): every band's predecessor in its pass holds
//     a lower ticket (the kernels' no-deadlock rule), and tickets go longest
//     row first;
//   - png_adam7_stage / png_adam7_rebase: passes 1-5 redirected into the
//     staging areas Q2 / S4 / S5 (every even-row, even-column pixel written
//     exactly once, where pass 6's merge looks it up), passes 6-7 writing
//     the image, pass 6 pointing at its merge job, and
//     png_plan_bands putting pass 6 (and only that) in the second
//     launch's schedule;
//   - dev_jpeg_frame: the quant-pair tables of the block kernel's row pass;
//   - the PNG epoch windows and cycle (check_epoch_windows).
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

// PNG epoch windows (api_internal.h, PngControl): every live owner holds a
// window of its own, never window 0; a released window is handed out again
// only after every other free one; the registry is exhausted at 4095 live
// owners; the control kernel's epoch sequence (png_epoch_next) never leaves
// [base + 1, base + cycle), never reaches 0, and png_epoch_wraps predicts
// exactly the launches at which it wraps.
static void check_epoch_windows()
{
    const uint32_t n = kPngEpochWindows - 1;
    std::vector<int> owners(n + 8);
    std::vector<uint32_t> got;
    std::map<uint32_t, int> seen;
    for (uint32_t i = 0; i < n; i++) { // (other blocks of this process may hold none: no GPU here)
        const uint32_t w = png_epoch_window_acquire(&owners[i]);
        CHECK(w >= 1 && w < kPngEpochWindows);
        CHECK(seen.count(w) == 0);
        seen[w] = int(i);
        got.push_back(w);
    }
    CHECK(png_epoch_window_acquire(&owners[n]) == 0); // exhausted
    CHECK(!png_epoch_window_release(got[5], &owners[6])); // not its owner
    CHECK(png_epoch_window_owned(got[5], &owners[5]) && !png_epoch_window_owned(got[5], &owners[6]));
    CHECK(png_epoch_window_release(got[5], &owners[5]));
    CHECK(!png_epoch_window_owned(got[5], &owners[5]));
    CHECK(png_epoch_window_acquire(&owners[n + 1]) == got[5]); // the only free one
    CHECK(png_epoch_window_release(got[5], &owners[n + 1]));
    CHECK(png_epoch_window_release(got[7], &owners[7]));
    // round robin: got[5] was returned first, but the cursor stands past
    // got[5]'s window, so got[7]'s window comes first unless it lies before
    const uint32_t a = png_epoch_window_acquire(&owners[n + 2]), b = png_epoch_window_acquire(&owners[n + 3]);
    CHECK(a != b && (a == got[5] || a == got[7]) && (b == got[5] || b == got[7]));
    CHECK(png_epoch_window_release(a, &owners[n + 2]) && png_epoch_window_release(b, &owners[n + 3]));
    for (uint32_t i = 0; i < n; i++)
        if (i != 5 && i != 7) CHECK(png_epoch_window_release(got[i], &owners[i]));
    CHECK(!png_epoch_window_release(0, nullptr));
    // a freed registry hands out a window other than the one just returned
    const uint32_t c = png_epoch_window_acquire(&owners[0]);
    CHECK(c != 0 && c != got[n - 1]);
    CHECK(png_epoch_window_release(c, &owners[0]));

    // the epoch sequence of one block, simulated over several cycles
    for (uint32_t cycle : {4u, 5u, 17u}) {
        const uint32_t base = 3 * kPngEpochWindow;
        uint32_t e = base, shadow = base;
        for (int launch = 0; launch < 100; launch++) {
            const int k = launch % 3 == 0 ? 2 : 1; // (an Adam7 item: two launches)
            if (png_epoch_wraps(shadow, base, cycle, k)) shadow = e = base; // the host's re-base
            for (int i = 0; i < k; i++) {
                const uint32_t nx = png_epoch_next(e, base, cycle);
                CHECK(nx > e); // no wrap inside launches the host announced
                e = nx;
                CHECK(e > base && e < base + cycle && e != 0);
            }
            shadow = e;
        }
    }
    // the device's own wrap (launches the host does not see) and the extremes
    CHECK(png_epoch_next(5 * kPngEpochWindow + 9, 5 * kPngEpochWindow, 10) == 5 * kPngEpochWindow + 1);
    const uint32_t top = (kPngEpochWindows - 1) * kPngEpochWindow;
    CHECK(png_epoch_next(top + kPngEpochWindow - 1, top, kPngEpochWindow) == top + 1); // 0xffffffff -> never 0
    CHECK(png_epoch_next(0, top, kPngEpochWindow) == top + 1); // a corrupted word re-enters the window
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
    {
        std::vector<DevPngPass> p = passes;
        const PngBandPlan bp = png_plan_bands(ZPX_PNG_TCA16, true, p, rowbytes);
        CHECK(bp.sched.size() + bp.sched2.size() == bp.nbands);
        // pass 6: 2048 rows of the 4K image, 23 of the 77x45 one
        CHECK(bp.sched2.size() == 16 + 1);
        for (const DevPngBand &b : bp.sched) CHECK(p[b.pass].merge == nullptr && !p[b.pass].launch2);
        std::map<uint32_t, uint32_t> next_band;
        for (size_t t = 0; t < bp.sched2.size(); t++) {
            const DevPngPass &d = p[bp.sched2[t].pass];
            CHECK(d.launch2 && d.yf == 2 && d.xf == 2 && d.merge != nullptr);
            CHECK(bp.sched2[t].band == next_band[bp.sched2[t].pass]++); // band order within a pass
        }
        // pass 7 (the longest rows) leads the first launch's tickets
        CHECK(!bp.sched.empty() && p[bp.sched[0].pass].xf == 1 && p[bp.sched[0].pass].yf == 2);
    }

    CHECK(st.jobs.size() == 2 && st.merge_pass.size() == 2);
    CHECK(st.staged.size() == 10);
    std::vector<uint8_t> staging(st.bytes + 256);
    uint8_t *base = reinterpret_cast<uint8_t *>((reinterpret_cast<uintptr_t>(staging.data()) + 255) & ~uintptr_t(255));
    std::vector<DevAdam7Merge> jobs_dev(2);
    png_adam7_rebase(passes, st, base, jobs_dev.data());
    // passes 1-5 write the staging areas of DevAdam7Merge (S5: pass 5 as
    // is, S4: pass 4 as is, Q2[Y][X] = pixel (4X, 4Y): passes 1-3), inside
    // the staging, every even-row / even-column pixel exactly once, at the
    // place pass 6's merge (png_pair_kernels.hip a7_even) looks it up
    static const uint32_t kA7[5][4] = {{0, 0, 8, 8}, {4, 0, 8, 8}, {0, 4, 4, 8}, {2, 0, 4, 4}, {0, 2, 2, 4}};
    for (int k = 0; k < 2; k++) {
        const DevAdam7Merge &m = st.jobs[k];
        const uint32_t W = imgs[k].w, H = imgs[k].h, ob = imgs[k].obpx;
        CHECK(m.width == W);
        const uint8_t *areas[3] = {m.q2, m.s4, m.s5};
        const uint64_t strides[3] = {m.q2stride, m.s4stride, m.s5stride};
        const uint64_t aw[3] = {(W + 3) / 4, (W - 2 + 3) / 4, (W + 1) / 2}, ah[3] = {(H + 3) / 4, (H + 3) / 4, (H - 2 + 3) / 4};
        for (int a = 0; a < 3; a++) {
            CHECK((reinterpret_cast<uintptr_t>(areas[a]) & 255) == 0 && strides[a] % 128 == 0 && strides[a] >= aw[a] * ob);
            CHECK(areas[a] >= base && areas[a] + strides[a] * ah[a] <= base + st.bytes);
        }
        // the merge's lookup of image pixel (x = 2X, y even)
        auto lookup = [&](uint32_t x, uint32_t y) -> const uint8_t * {
            const uint32_t X = x / 2;
            if (y & 2) return m.s5 + uint64_t((y - 2) >> 2) * m.s5stride + uint64_t(X) * ob;
            if (X & 1) return m.s4 + uint64_t(y >> 2) * m.s4stride + uint64_t(X >> 1) * ob;
            return m.q2 + uint64_t(y >> 2) * m.q2stride + uint64_t(X >> 1) * ob;
        };
        std::map<const uint8_t *, int> written;
        for (int p = 0; p < 5; p++) {
            const DevPngPass &d = passes[first_of[k] + p];
            CHECK(!d.launch2 && d.merge == nullptr);
            CHECK(d.out == (p <= 2 ? m.q2 : p == 3 ? m.s4 : m.s5));
            for (uint32_t r = 0; r < d.rows; r++)
                for (uint32_t c = 0; c < d.width; c++) {
                    const uint8_t *at = d.out + uint64_t(r * d.yf + d.yo) * d.out_stride + uint64_t(c * d.xf + d.xo) * ob;
                    const uint32_t x = c * kA7[p][2] + kA7[p][0], y = r * kA7[p][3] + kA7[p][1];
                    CHECK(x < W && y < H && x % 2 == 0 && y % 2 == 0 && at == lookup(x, y));
                    written[at]++;
                }
        }
        CHECK(written.size() == size_t((W + 1) / 2) * ((H + 1) / 2));
        bool once = true;
        for (auto &kv : written) once &= kv.second == 1;
        CHECK(once);
    }
    // passes 6 and 7 of each Adam7 image still write the image: pass 7 the
    // odd rows, pass 6 (merging Q) the even ones
    for (int k = 0; k < 2; k++) {
        const DevPngPass &p7 = passes[first_of[k] + 6];
        CHECK(p7.xo == 0 && p7.yo == 1 && p7.xf == 1 && p7.yf == 2 && p7.out == fake_out.data() && !p7.merge);
        const DevPngPass &p6 = passes[first_of[k] + 5];
        CHECK(p6.xo == 1 && p6.yo == 0 && p6.xf == 2 && p6.yf == 2 && p6.out == fake_out.data());
        CHECK(p6.merge == jobs_dev.data() + k && p6.launch2 && !p7.launch2);
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

    check_epoch_windows();
    if (fails) return 1;
    printf("ok\n");
    return 0;
}
