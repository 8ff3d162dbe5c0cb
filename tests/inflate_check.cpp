// Host check of the fast inflate (zpix_amd/csrc/inflate_fast.cpp), built by
// tests/test_inflate_host.py with g++ and the host sanitizers: the serial and
// the speculative parallel decoders against zlib's bytes on a stream given as
// files.  Usage: inflate_check <zlib stream> <expected bytes>; prints "ok".
#include <cstdio>
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

int main(int argc, char **argv)
{
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
