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
    printf("ok\n");
    return 0;
}
