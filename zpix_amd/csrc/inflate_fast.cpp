// Fast zlib/DEFLATE decoder for the PNG host stage (RFC 1950/1951).
//
// The PNG path inflates every IDAT stream on the host (src/png/decoder.zig
// :404-545, Zig std.compress.flate); for noisy 4K truecolor images system
// zlib runs at ~100-200 MB/s and is the end-to-end bottleneck.  This decoder
// is the fast path only: it accepts a stream when it decodes cleanly and
// rejects anything irregular (bad header, invalid or incomplete code sets, a
// distance past the start of the output, running out of input, ...), in
// which case the caller re-runs system zlib from the start, so error
// behaviour is zlib's by construction.  A stream it accepts is one zlib
// accepts too, and DEFLATE output is unique, so the bytes are identical.
//
// Design: 64-bit bit buffer refilled 8 bytes at a time; literal/length codes
// through an 11-bit table (symbol + length, or a flag for longer codes that
// a canonical first-code walk resolves), distances through an 8-bit table.
#include "inflate_fast.h"

#include <cstring>

namespace zpx {
namespace {

constexpr int kLitBits = 11, kDistBits = 8;

struct Table {
    // fast[code >> (15 - bits)] = symbol << 4 | length (0 = code longer than `bits`)
    uint16_t fast[1 << kLitBits];
    int bits;
    // canonical tables for the slow walk
    uint16_t count[16];
    uint16_t first[16]; // first code of each length (left-aligned in `len` bits)
    uint16_t index[16]; // index in `sorted` of the first symbol of each length
    uint16_t sorted[320];
    int max_len;
};

// Builds a canonical Huffman table; false on an over-subscribed or
// incomplete set (zlib allows a lone length-1 distance code: we reject it and
// let zlib handle that stream).
bool build(Table &t, const uint8_t *lens, int n, int fast_bits)
{
    memset(t.count, 0, sizeof(t.count));
    for (int i = 0; i < n; i++) t.count[lens[i]]++;
    t.count[0] = 0;
    int left = 1;
    for (int l = 1; l < 16; l++) {
        left <<= 1;
        left -= t.count[l];
        if (left < 0) return false; // over-subscribed
    }
    if (left != 0) return false; // incomplete (or empty)
    // canonical first codes (RFC 1951 3.2.2) and sorted symbol order
    uint16_t code = 0, idx = 0;
    t.max_len = 0;
    for (int l = 1; l < 16; l++) {
        code = static_cast<uint16_t>((code + t.count[l - 1]) << 1);
        t.first[l] = code;
        t.index[l] = idx;
        idx = static_cast<uint16_t>(idx + t.count[l]);
        if (t.count[l]) t.max_len = l;
    }
    uint16_t offs[16], next[16];
    for (int l = 1; l < 16; l++) {
        offs[l] = t.index[l];
        next[l] = t.first[l];
    }
    for (int s = 0; s < n; s++)
        if (lens[s]) t.sorted[offs[lens[s]]++] = static_cast<uint16_t>(s);
    // fast table, indexed by the next `fast_bits` stream bits: codes are
    // stored MSB-first in an LSB-first bit stream, so by the reversed code
    t.bits = fast_bits;
    memset(t.fast, 0, sizeof(uint16_t) << fast_bits);
    for (int s = 0; s < n; s++) {
        const int l = lens[s];
        if (!l) continue;
        const uint16_t c = next[l]++;
        if (l > fast_bits) continue;
        uint32_t r = 0;
        for (int k = 0; k < l; k++) r |= ((c >> k) & 1u) << (l - 1 - k);
        for (uint32_t k = r; k < (1u << fast_bits); k += (1u << l)) t.fast[k] = static_cast<uint16_t>(s << 4 | l);
    }
    return true;
}

struct Bits {
    const uint8_t *in;
    size_t len, pos = 0; // bytes of `in` whose bits are counted in cnt (or consumed)
    uint64_t buf = 0;    // bits above cnt are the next input bits or zero
    int cnt = 0;
    int pad = 0;         // zero bits counted past the end of the input

    inline void refill()
    {
        if (cnt >= 48) return; // callers decode up to 45 bits (three codes) per refill
        if (pos + 8 <= len) {
            uint64_t w;
            memcpy(&w, in + pos, 8);
            buf |= w << cnt;
            const int take = (63 - cnt) >> 3;
            pos += take;
            cnt += take * 8;
        } else {
            while (cnt <= 56) {
                if (pos < len) buf |= uint64_t(in[pos++]) << cnt;
                else pad += 8;
                cnt += 8;
            }
        }
    }
    // true once a consumed bit lay past the end of the input
    inline bool overrun() const { return cnt < pad; }
    inline uint32_t peek(int n) const { return static_cast<uint32_t>(buf & ((uint64_t(1) << n) - 1)); }
    inline void drop(int n)
    {
        buf >>= n;
        cnt -= n;
    }
    inline uint32_t take(int n)
    {
        const uint32_t v = peek(n);
        drop(n);
        return v;
    }
};

// Decodes one symbol (bit buffer holds >= 15 bits); -1 on an invalid code.
inline int decode(Bits &b, const Table &t)
{
    const uint16_t e = t.fast[b.peek(t.bits)];
    if (e) {
        b.drop(e & 15);
        return e >> 4;
    }
    // canonical walk for codes longer than the fast table
    uint32_t code = 0;
    for (int l = 1; l <= 15; l++) {
        code |= (b.peek(l) >> (l - 1)) & 1u;
        const int cnt = t.count[l];
        if (static_cast<int>(code) - static_cast<int>(t.first[l]) < cnt && code >= t.first[l]) {
            b.drop(l);
            return t.sorted[t.index[l] + (code - t.first[l])];
        }
        code <<= 1;
    }
    return -1;
}

const uint16_t kLenBase[29] = {3,  4,  5,  6,  7,  8,  9,  10, 11,  13,  15,  17,  19,  23, 27,
                               31, 35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195, 227, 258};
const uint8_t kLenExtra[29] = {0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0};
const uint16_t kDistBase[30] = {1,   2,   3,   4,   5,   7,    9,    13,   17,   25,   33,   49,   65,    97,    129,
                                193, 257, 385, 513, 769, 1025, 1537, 2049, 3073, 4097, 6145, 8193, 12289, 16385, 24577};
const uint8_t kDistExtra[30] = {0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13};

} // namespace

bool inflate_fast(const uint8_t *in, size_t in_len, uint8_t *out, size_t want, size_t *produced)
{
    *produced = 0;
    if (in_len < 2) return false;
    const uint32_t cmf = in[0], flg = in[1];
    if ((cmf & 15) != 8 || (cmf >> 4) > 7 || ((cmf << 8) | flg) % 31 != 0 || (flg & 0x20)) return false;
    Bits b;
    b.in = in + 2;
    b.len = in_len - 2;
    size_t o = 0;
    static thread_local Table lit, dist;
    bool last = false;
    while (!last && o < want) {
        b.refill();
        last = b.take(1) != 0;
        const uint32_t type = b.take(2);
        if (type == 0) { // stored
            if (b.overrun()) return false;
            b.drop((b.cnt - b.pad) & 7);
            // re-sync the byte position to the bit buffer (whole real bytes
            // still buffered go back to the input)
            const size_t bytes_in_buf = static_cast<size_t>((b.cnt - b.pad) >> 3);
            size_t p = b.pos - bytes_in_buf;
            b.buf = 0;
            b.cnt = 0;
            b.pad = 0;
            b.pos = p;
            if (p + 4 > b.len) return false;
            const uint32_t len = b.in[p] | uint32_t(b.in[p + 1]) << 8;
            const uint32_t nlen = b.in[p + 2] | uint32_t(b.in[p + 3]) << 8;
            if ((len ^ 0xffffu) != nlen) return false;
            p += 4;
            if (p + len > b.len) return false;
            const size_t n = len < want - o ? len : want - o;
            memcpy(out + o, b.in + p, n);
            o += n;
            b.pos = p + len;
            continue;
        }
        if (type == 1) { // fixed codes
            uint8_t l[320];
            for (int i = 0; i < 144; i++) l[i] = 8;
            for (int i = 144; i < 256; i++) l[i] = 9;
            for (int i = 256; i < 280; i++) l[i] = 7;
            for (int i = 280; i < 288; i++) l[i] = 8;
            // zlib's fixed table has 288 literal/length symbols (286, 287 invalid when used)
            if (!build(lit, l, 288, kLitBits)) return false;
            uint8_t d[32];
            for (int i = 0; i < 32; i++) d[i] = 5;
            if (!build(dist, d, 32, kDistBits)) return false;
        } else if (type == 2) { // dynamic
            b.refill();
            const int hlit = static_cast<int>(b.take(5)) + 257;
            const int hdist = static_cast<int>(b.take(5)) + 1;
            const int hclen = static_cast<int>(b.take(4)) + 4;
            if (hlit > 286 || hdist > 30) return false;
            static const uint8_t kOrd[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};
            uint8_t cl[19] = {};
            for (int i = 0; i < hclen; i++) {
                b.refill();
                cl[kOrd[i]] = static_cast<uint8_t>(b.take(3));
            }
            static thread_local Table clt;
            if (!build(clt, cl, 19, 7)) return false;
            uint8_t lens[320];
            int n = 0;
            while (n < hlit + hdist) {
                b.refill();
                const int sym = decode(b, clt);
                if (sym < 0 || b.overrun()) return false;
                if (sym < 16) {
                    lens[n++] = static_cast<uint8_t>(sym);
                } else {
                    int rep;
                    uint8_t v = 0;
                    if (sym == 16) {
                        if (n == 0) return false;
                        v = lens[n - 1];
                        rep = 3 + static_cast<int>(b.take(2));
                    } else if (sym == 17) {
                        rep = 3 + static_cast<int>(b.take(3));
                    } else {
                        rep = 11 + static_cast<int>(b.take(7));
                    }
                    if (n + rep > hlit + hdist) return false;
                    while (rep--) lens[n++] = v;
                }
            }
            if (lens[256] == 0) return false; // no end-of-block code
            if (!build(lit, lens, hlit, kLitBits)) return false;
            if (!build(dist, lens + hlit, hdist, kDistBits)) return false;
        } else {
            return false;
        }
        if (b.overrun()) return false;
        // ---- the block's symbols
        for (;;) {
            // one refill leaves >= 56 bits: up to three literal codes (<= 15
            // bits each) decode before the next refill
            b.refill();
            int sym = decode(b, lit);
            if (sym < 256 && sym >= 0) {
                if (b.overrun() || o >= want) {
                    if (b.overrun()) return false;
                    break;
                }
                out[o++] = static_cast<uint8_t>(sym);
                sym = decode(b, lit);
                if (sym < 256 && sym >= 0) {
                    if (b.overrun() || o >= want) {
                        if (b.overrun()) return false;
                        break;
                    }
                    out[o++] = static_cast<uint8_t>(sym);
                    sym = decode(b, lit);
                    if (sym < 256 && sym >= 0) {
                        if (b.overrun() || o >= want) {
                            if (b.overrun()) return false;
                            break;
                        }
                        out[o++] = static_cast<uint8_t>(sym);
                        continue;
                    }
                }
            }
            if (sym < 0 || b.overrun()) return false;
            if (sym == 256) break;
            b.refill();
            const int li = sym - 257;
            if (li >= 29) return false; // 286, 287
            const uint32_t len = kLenBase[li] + b.take(kLenExtra[li]);
            b.refill();
            const int ds = decode(b, dist);
            if (ds < 0 || ds >= 30) return false;
            const uint32_t d = kDistBase[ds] + b.take(kDistExtra[ds]);
            if (b.overrun()) return false;
            if (d > o) return false; // distance past the start of the output
            size_t n = len < want - o ? len : want - o;
            uint8_t *dst = out + o;
            const uint8_t *src = dst - d;
            if (d >= 8 && n >= 8) {
                // 8-byte chunks: with d >= 8 a chunk never reads bytes it writes
                size_t k = 0;
                for (; k + 8 <= n; k += 8) {
                    uint64_t w;
                    memcpy(&w, src + k, 8);
                    memcpy(dst + k, &w, 8);
                }
                for (; k < n; k++) dst[k] = src[k];
            } else {
                for (size_t k = 0; k < n; k++) dst[k] = src[k];
            }
            o += n;
            if (o >= want) break;
        }
    }
    *produced = o;
    return o >= want; // anything short of the requested bytes: let zlib decide
}

} // namespace zpx
