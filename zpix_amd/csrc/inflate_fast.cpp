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
// Design: 64-bit bit buffer refilled 8 bytes at a time; two-level decode
// tables of 32-bit entries (an 11-bit literal/length root and an 8-bit
// distance root, subtables for longer codes) whose entries carry the decoded
// result -- literal byte, or length / distance base and extra-bit count -- so
// a symbol costs one or two lookups and no bit loop.  A "fast zone" loop runs
// while at least 32 input bytes and 258 + 8 output bytes remain: there no
// literal needs an end-of-input or end-of-output check.
#include "inflate_fast.h"

#include <cstring>

namespace zpx {
namespace {

constexpr int kLitBits = 11, kDistBits = 8;

// entry: bits 0-4 = bits to drop; bits 5-8 = extra-bit count (length /
// distance) or index bits (subtable); flags in bits 9-12; payload in bits
// 16-31 = the literal byte, the length / distance base (<= 24577), the
// subtable's offset from the table start, or the code-length symbol
constexpr uint32_t kLiteral = 1u << 9;
constexpr uint32_t kSub = 1u << 10;
constexpr uint32_t kEob = 1u << 11;     // end of block
constexpr uint32_t kInvalid = 1u << 12; // symbol 286/287 or distance 30/31
inline uint32_t drop_of(uint32_t e) { return e & 31; }
inline uint32_t extra_of(uint32_t e) { return (e >> 5) & 15; }
inline uint32_t payload(uint32_t e) { return e >> 16; }

constexpr int kLitEntries = 8192, kDistEntries = 4096; // root + worst-case subtables

const uint16_t kLenBase[29] = {3,  4,  5,  6,  7,  8,  9,  10, 11,  13,  15,  17,  19,  23, 27,
                               31, 35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195, 227, 258};
const uint8_t kLenExtra[29] = {0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0};
const uint16_t kDistBase[30] = {1,   2,   3,   4,   5,   7,    9,    13,   17,   25,   33,   49,   65,    97,    129,
                                193, 257, 385, 513, 769, 1025, 1537, 2049, 3073, 4097, 6145, 8193, 12289, 16385, 24577};
const uint8_t kDistExtra[30] = {0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13};

enum class Kind { LitLen, Dist, CodeLen };

// the decoded result of symbol s, without the drop count
uint32_t result(Kind k, int s)
{
    switch (k) {
    case Kind::LitLen:
        if (s < 256) return kLiteral | uint32_t(s) << 16;
        if (s == 256) return kEob;
        if (s - 257 >= 29) return kInvalid;
        return uint32_t(kLenBase[s - 257]) << 16 | uint32_t(kLenExtra[s - 257]) << 5;
    case Kind::Dist:
        if (s >= 30) return kInvalid;
        return uint32_t(kDistBase[s]) << 16 | uint32_t(kDistExtra[s]) << 5;
    default:
        return uint32_t(s) << 16; // code-length alphabet: the symbol
    }
}

// bit-reversed bytes, for the MSB-first codes of an LSB-first stream
struct Rev8 {
    uint8_t v[256];
    constexpr Rev8() : v()
    {
        for (int i = 0; i < 256; i++) {
            int r = 0;
            for (int k = 0; k < 8; k++) r |= ((i >> k) & 1) << (7 - k);
            v[i] = static_cast<uint8_t>(r);
        }
    }
};
constexpr Rev8 kRev8;
inline uint32_t reverse(uint32_t code, int len)
{
    return (uint32_t(kRev8.v[code & 0xff]) << 8 | kRev8.v[(code >> 8) & 0xff]) >> (16 - len);
}

// Builds a two-level canonical Huffman table (root `root` bits); false on an
// over-subscribed or incomplete set (zlib allows a lone length-1 distance
// code: we reject it and let zlib handle that stream).  Runs once per
// dynamic block (~3,000 per 4K image), so it avoids per-call clears: the
// subtable-size scratch is kept zero between calls.
bool build(uint32_t *t, int cap, const uint8_t *lens, int n, int root, Kind kind)
{
    uint16_t count[16] = {};
    for (int i = 0; i < n; i++) count[lens[i]]++;
    count[0] = 0;
    int left = 1;
    for (int l = 1; l < 16; l++) {
        left <<= 1;
        left -= count[l];
        if (left < 0) return false; // over-subscribed
    }
    if (left != 0) return false; // incomplete (or empty)
    uint16_t next[16];
    uint16_t code = 0;
    for (int l = 1; l < 16; l++) {
        code = static_cast<uint16_t>((code + count[l - 1]) << 1);
        next[l] = code;
    }
    uint16_t rev[320];
    static thread_local uint8_t sub_bits[1 << 12]; // zero between calls
    uint16_t longp[320];
    int nlong = 0;
    for (int s = 0; s < n; s++) {
        const int l = lens[s];
        if (!l) continue;
        const uint32_t r = reverse(next[l]++, l);
        rev[s] = static_cast<uint16_t>(r);
        if (l > root) {
            const uint32_t p = r & ((1u << root) - 1);
            if (!sub_bits[p]) longp[nlong++] = static_cast<uint16_t>(p);
            if (l - root > sub_bits[p]) sub_bits[p] = static_cast<uint8_t>(l - root);
        }
    }
    const int nroot = 1 << root;
    int used = nroot;
    bool fits = true;
    for (int i = 0; i < nlong; i++) {
        const int p = longp[i];
        const int size = 1 << sub_bits[p];
        if (used + size > cap) fits = false;
        else t[p] = kSub | uint32_t(used) << 16 | uint32_t(sub_bits[p]) << 5 | uint32_t(root);
        used += size;
    }
    for (int i = 0; i < nlong; i++) sub_bits[longp[i]] = 0;
    if (!fits) return false;
    for (int s = 0; s < n; s++) {
        const int l = lens[s];
        if (!l) continue;
        const uint32_t r = rev[s];
        if (l <= root) {
            const uint32_t e = result(kind, s) | uint32_t(l);
            for (uint32_t k = r; k < uint32_t(nroot); k += (1u << l)) t[k] = e;
        } else {
            const uint32_t p = r & (uint32_t(nroot) - 1), rest = r >> root;
            const uint32_t off = payload(t[p]), sb = extra_of(t[p]);
            const uint32_t e = result(kind, s) | uint32_t(l - root);
            for (uint32_t k = rest; k < (1u << sb); k += (1u << (l - root))) t[off + k] = e;
        }
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
        if (cnt >= 48) return;
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
    // refill with at least 8 readable input bytes (the fast zone)
    inline void refill_fast()
    {
        uint64_t w;
        memcpy(&w, in + pos, 8);
        buf |= w << cnt;
        const int take = (63 - cnt) >> 3;
        pos += take;
        cnt += take * 8;
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

// One symbol's entry (the buffer holds >= 15 bits); its bits are consumed.
inline uint32_t decode(Bits &b, const uint32_t *t, int root)
{
    uint32_t e = t[b.peek(root)];
    if (e & kSub) {
        b.drop(root);
        e = t[payload(e) + b.peek(static_cast<int>(extra_of(e)))];
    }
    b.drop(static_cast<int>(drop_of(e)));
    return e;
}

// match copy of n bytes from distance d (d <= bytes already written)
inline void copy_match(uint8_t *dst, size_t d, size_t n)
{
    const uint8_t *src = dst - d;
    if (d >= 8) {
        size_t k = 0;
        for (; k + 8 <= n; k += 8) { // with d >= 8 a chunk never reads bytes it writes
            uint64_t w;
            memcpy(&w, src + k, 8);
            memcpy(dst + k, &w, 8);
        }
        for (; k < n; k++) dst[k] = src[k];
    } else {
        for (size_t k = 0; k < n; k++) dst[k] = src[k];
    }
}

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
    static thread_local uint32_t lit[kLitEntries], dist[kDistEntries];
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
            if (!build(lit, kLitEntries, l, 288, kLitBits, Kind::LitLen)) return false;
            uint8_t d[32];
            for (int i = 0; i < 32; i++) d[i] = 5;
            if (!build(dist, kDistEntries, d, 32, kDistBits, Kind::Dist)) return false;
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
            static thread_local uint32_t clt[1 << 7];
            if (!build(clt, 1 << 7, cl, 19, 7, Kind::CodeLen)) return false;
            uint8_t lens[320];
            int n = 0;
            while (n < hlit + hdist) {
                b.refill();
                const int sym = static_cast<int>(payload(decode(b, clt, 7)));
                if (b.overrun()) return false;
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
            if (!build(lit, kLitEntries, lens, hlit, kLitBits, Kind::LitLen)) return false;
            if (!build(dist, kDistEntries, lens + hlit, hdist, kDistBits, Kind::Dist)) return false;
        } else {
            return false;
        }
        if (b.overrun()) return false;
        // ---- the block's symbols
        for (;;) {
            uint32_t e;
            if (b.pos + 32 <= b.len && o + 258 + 8 <= want) {
                // fast zone: real input bytes behind every bit and room for a
                // whole match -- no end checks per symbol
                b.refill_fast();
                e = decode(b, lit, kLitBits);
                if (e & kLiteral) {
                    out[o++] = static_cast<uint8_t>(payload(e));
                    e = decode(b, lit, kLitBits);
                    if (e & kLiteral) {
                        out[o++] = static_cast<uint8_t>(payload(e));
                        e = decode(b, lit, kLitBits);
                        if (e & kLiteral) {
                            out[o++] = static_cast<uint8_t>(payload(e));
                            continue;
                        }
                    }
                }
                if (e & (kEob | kInvalid)) {
                    if (e & kInvalid) return false;
                    break;
                }
                // a length: its extra bits, then the distance (one refill covers
                // extra <= 5 + distance code <= 15 + extra <= 13 bits)
                b.refill_fast();
                const uint32_t len = payload(e) + b.take(static_cast<int>(extra_of(e)));
                const uint32_t de = decode(b, dist, kDistBits);
                if (de & kInvalid) return false;
                const uint32_t d = payload(de) + b.take(static_cast<int>(extra_of(de)));
                if (d > o) return false; // distance past the start of the output
                copy_match(out + o, d, len);
                o += len;
                continue;
            }
            // careful path near the end of the input or the output
            b.refill();
            e = decode(b, lit, kLitBits);
            if (b.overrun() || (e & kInvalid)) return false;
            if (e & kLiteral) {
                if (o >= want) break;
                out[o++] = static_cast<uint8_t>(payload(e));
                continue;
            }
            if (e & kEob) break;
            b.refill();
            const uint32_t len = payload(e) + b.take(static_cast<int>(extra_of(e)));
            b.refill();
            const uint32_t de = decode(b, dist, kDistBits);
            if (de & kInvalid) return false;
            const uint32_t d = payload(de) + b.take(static_cast<int>(extra_of(de)));
            if (b.overrun()) return false;
            if (d > o) return false;
            const size_t n = len < want - o ? len : want - o;
            copy_match(out + o, d, n);
            o += n;
            if (o >= want) break;
        }
    }
    *produced = o;
    return o >= want; // anything short of the requested bytes: let zlib decide
}

} // namespace zpx
