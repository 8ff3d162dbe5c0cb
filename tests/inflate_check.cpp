// Host check of the fast inflate (zpix_amd/csrc/inflate_fast.cpp), built by
// tests/test_inflate_host.py with g++ and the host sanitizers: the serial and
// the speculative parallel decoders against zlib's bytes on a stream given as
// files.  Usage: inflate_check <zlib stream> <expected bytes>; prints "ok".
//   inflate_check pairs <want> <stream>...: streams that may be malformed
// (truncated, bit-flipped, a distance past the output's start, a last block
// ending short of want): inflate_fast_pair's ok / produced / bytes for every
// ordered pair of them must be inflate_fast's for each stream alone -- its
// careful path, stored-block checks and one stream failing while the other
// goes on alone all run under the sanitizers -- and inflate_parallel must
// decline or agree.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "inflate_fast.h"

static bool read_file(const char *p, std::vector<uint8_t> &v)
{
    FILE *f = fopen(p, "rb");
    if (!f) return false;
    fseek(f, 0, SEEK_END);
    v.resize(static_cast<size_t>(ftell(f)));
    fseek(f, 0, SEEK_SET);
    const bool ok = fread(v.data(), 1, v.size(), f) == v.size();
    fclose(f);
    return ok;
}

static int check_pairs(size_t want, int n, char **files)
{
    const size_t nn = static_cast<size_t>(n);
    std::vector<std::vector<uint8_t>> z(nn), single(nn);
    std::vector<size_t> produced(nn);
    std::vector<char> ok(nn);
    for (int i = 0; i < n; i++) {
        if (!read_file(files[i], z[size_t(i)])) return 2;
        single[size_t(i)].assign(want + 64, 0);
        size_t got = 0;
        ok[size_t(i)] = zpx::inflate_fast(z[size_t(i)].data(), z[size_t(i)].size(), single[size_t(i)].data(), want, &got);
        produced[size_t(i)] = got;
        std::vector<uint8_t> par(want + 64, 0);
        for (int threads : {2, 3, 5}) {
            size_t pg = 0;
            if (zpx::inflate_parallel(z[size_t(i)].data(), z[size_t(i)].size(), par.data(), want, &pg, threads) &&
                (!ok[size_t(i)] || pg != got || memcmp(par.data(), single[size_t(i)].data(), want))) {
                fprintf(stderr, "parallel decode of stream %d on %d threads disagrees\n", i, threads);
                return 1;
            }
        }
    }
    std::vector<uint8_t> o0(want + 64), o1(want + 64);
    for (int a = 0; a < n; a++)
        for (int b = 0; b < n; b++) {
            memset(o0.data(), 0, o0.size());
            memset(o1.data(), 0, o1.size());
            const uint8_t *in[2] = {z[size_t(a)].data(), z[size_t(b)].data()};
            const size_t in_len[2] = {z[size_t(a)].size(), z[size_t(b)].size()};
            uint8_t *dst[2] = {o0.data(), o1.data()};
            const size_t w[2] = {want, want};
            size_t pr[2] = {0, 0};
            bool pk[2] = {false, false};
            zpx::inflate_fast_pair(in, in_len, dst, w, pr, pk);
            const int ks[2] = {a, b};
            const std::vector<uint8_t> *os[2] = {&o0, &o1};
            for (int k = 0; k < 2; k++) {
                const size_t s = size_t(ks[k]);
                if (pk[k] != bool(ok[s]) || (pk[k] && (pr[k] != produced[s] || memcmp(os[k]->data(), single[s].data(), want)))) {
                    fprintf(stderr, "pair (%d, %d): stream %d ok %d/%d produced %zu/%zu\n", a, b, ks[k], int(pk[k]),
                            int(ok[s]), pr[k], produced[s]);
                    return 1;
                }
            }
        }
    int nok = 0;
    for (char c : ok) nok += c != 0;
    printf("ok %d of %d accepted\n", nok, n);
    return 0;
}

int main(int argc, char **argv)
{
    if (argc >= 4 && strcmp(argv[1], "pairs") == 0) return check_pairs(strtoull(argv[2], nullptr, 10), argc - 3, argv + 3);
    std::vector<uint8_t> z, raw;
    if (argc != 3 || !read_file(argv[1], z) || !read_file(argv[2], raw)) {
        fprintf(stderr, "usage: inflate_check <zlib stream> <expected bytes>\n");
        return 2;
    }
    std::vector<uint8_t> out(raw.size() + 64);
    for (size_t want : {raw.size(), raw.size() / 3}) {
        size_t got = 0;
        if (!zpx::inflate_fast(z.data(), z.size(), out.data(), want, &got) || got != want ||
            memcmp(out.data(), raw.data(), want)) {
            fprintf(stderr, "serial decode differs (want %zu, got %zu)\n", want, got);
            return 1;
        }
        for (int threads : {2, 3, 4, 7}) {
            memset(out.data(), 0, out.size());
            got = 0;
            // (declining is allowed: the caller then decodes serially)
            if (zpx::inflate_parallel(z.data(), z.size(), out.data(), want, &got, threads) &&
                (got != want || memcmp(out.data(), raw.data(), want))) {
                fprintf(stderr, "parallel decode on %d threads differs (want %zu)\n", threads, want);
                return 1;
            }
        }
    }
    // two streams in one loop (inflate_fast_pair): the stream with itself,
    // whole and a third (their fast zones end at different points)
    std::vector<uint8_t> out2(raw.size() + 64);
    const size_t wants[3][2] = {{raw.size(), raw.size()}, {raw.size(), raw.size() / 3}, {raw.size() / 3, raw.size()}};
    for (const auto &w : wants) {
        memset(out.data(), 0, out.size());
        memset(out2.data(), 0, out2.size());
        const uint8_t *in[2] = {z.data(), z.data()};
        const size_t in_len[2] = {z.size(), z.size()};
        uint8_t *dst[2] = {out.data(), out2.data()};
        size_t produced[2] = {0, 0};
        bool ok[2] = {false, false};
        zpx::inflate_fast_pair(in, in_len, dst, w, produced, ok);
        if (!ok[0] || !ok[1] || produced[0] != w[0] || produced[1] != w[1] || memcmp(out.data(), raw.data(), w[0]) ||
            memcmp(out2.data(), raw.data(), w[1])) {
            fprintf(stderr, "pair decode differs (want %zu / %zu)\n", w[0], w[1]);
            return 1;
        }
    }
    printf("ok\n");
    return 0;
}
