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
// tables of 32-bit entries (a 12-bit literal/length root and an 8-bit
// distance root, subtables for longer codes) whose entries carry the decoded
// result -- literal byte (or two, see pair_literals), or length / distance
// base and extra-bit count -- so a symbol costs one or two lookups and no bit
// loop.  A "fast zone" loop runs
// while at least 32 input bytes and 258 + 8 output bytes remain: there no
// literal needs an end-of-input or end-of-output check.
#include "inflate_fast.h"

#include <algorithm>
#include <atomic>
#include <cstring>
#include <memory>
#include <mutex>
#include <utility>
#include <thread>
#include <vector>

namespace zpx {
namespace {

constexpr int kLitBits = 12, kDistBits = 8;

// entry: bits 0-5 = bits to drop (the low 6 bits, so that the bit buffer's
// 64-bit shift takes the entry itself as its count: one instruction less on
// the lookup -> shift dependency chain that bounds a literal, 3-10 % on a
// noisy 4K truecolor stream); bits 6-9 = extra-bit count (length / distance)
// or index bits (subtable); flags in bits 10-14; payload in bits 16-31 = the
// literal byte, the length / distance base (<= 24577), the subtable's offset
// from the table start, or the code-length symbol
constexpr uint32_t kLiteral = 1u << 10;
constexpr uint32_t kSub = 1u << 11;
constexpr uint32_t kEob = 1u << 12;     // end of block
constexpr uint32_t kInvalid = 1u << 13; // symbol 286/287 or distance 30/31
constexpr uint32_t kLiteral2 = 1u << 14; // (with kLiteral) two literals: payload = first | second << 8
inline uint32_t drop_of(uint32_t e) { return e & 63; }
inline uint32_t extra_of(uint32_t e) { return (e >> 6) & 15; }
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
        return uint32_t(kLenBase[s - 257]) << 16 | uint32_t(kLenExtra[s - 257]) << 6;
    case Kind::Dist:
        if (s >= 30) return kInvalid;
        return uint32_t(kDistBase[s]) << 16 | uint32_t(kDistExtra[s]) << 6;
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
// (rev_out: the symbols' bit-reversed codes, for pair_literals; 320 entries)
bool build(uint32_t *t, int cap, const uint8_t *lens, int n, int root, Kind kind, uint16_t *rev_out = nullptr)
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
    uint16_t rev_local[320];
    uint16_t *const rev = rev_out ? rev_out : rev_local;
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
    // the root, shortest codes first: with the codes of < l bits complete in
    // the first 2^(l-1) entries, one copy doubles them to 2^l, and each code
    // of l bits is then one store (4,096 strided stores a 12-bit root before)
    {
        uint16_t ord[320];
        int end[17] = {};
        for (int l = 1; l <= root; l++) end[l] = end[l - 1] + count[l];
        int at[17];
        for (int l = 1; l <= root; l++) at[l] = end[l - 1];
        for (int s = 0; s < n; s++)
            if (lens[s] && lens[s] <= root) ord[at[lens[s]]++] = static_cast<uint16_t>(s);
        t[0] = 0;
        int size = 1;
        for (int l = 1; l <= root; l++) {
            memcpy(t + size, t, sizeof(uint32_t) * static_cast<size_t>(size));
            size <<= 1;
            for (int i = end[l - 1]; i < end[l]; i++) t[rev[ord[i]]] = result(kind, ord[i]) | uint32_t(l);
        }
    }
    int used = nroot;
    bool fits = true;
    for (int i = 0; i < nlong; i++) {
        const int p = longp[i];
        const int size = 1 << sub_bits[p];
        if (used + size > cap) fits = false;
        else t[p] = kSub | uint32_t(used) << 16 | uint32_t(sub_bits[p]) << 6 | uint32_t(root);
        used += size;
    }
    for (int i = 0; i < nlong; i++) sub_bits[longp[i]] = 0;
    if (!fits) return false;
    for (int s = 0; s < n; s++) {
        const int l = lens[s];
        if (l <= root) continue;
        const uint32_t r = rev[s];
        {
            const uint32_t p = r & (uint32_t(nroot) - 1), rest = r >> root;
            const uint32_t off = payload(t[p]), sb = extra_of(t[p]);
            const uint32_t e = result(kind, s) | uint32_t(l - root);
            for (uint32_t k = rest; k < (1u << sb); k += (1u << (l - root))) t[off + k] = e;
        }
    }
    return true;
}

// Literal pairs in the root table: an entry whose bits hold a literal of l1
// bits followed by one of l2 bits, l1 + l2 <= root, decodes both (drop
// l1 + l2) -- one lookup for two bytes.  The second code is the entry at the
// index shifted by l1, which depends only on its low l2 bits when l2 <= root
// - l1.  The pass writes exactly the pair entries: the candidate second
// codes j (entries below 2^(root - minlen), minlen the shortest literal code,
// read from a copy taken before any of them turns into a pair) are sorted by
// the budget they need, max(their code length, bit length of j), so that a
// first literal of l1 bits walks just the prefix of budget <= root - l1.
// (Walking every entry of every short literal, with its data-dependent
// branch, cost ~16k cycles a block -- a tenth of a noisy 4K image's decode.)
void pair_literals(uint32_t *t, int root, const uint8_t *lens, int n, const uint16_t *rev)
{
    int minlen = 16;
    for (int s = 0; s < 256 && s < n; s++)
        if (lens[s] && lens[s] < minlen) minlen = lens[s];
    const int maxb = root - minlen; // the largest second-code budget
    if (maxb < minlen) return;      // no two literals fit the root
    // candidate second codes by budget (counting sort)
    uint16_t cnt[17] = {}, cand[1 << 12];
    uint32_t sec[1 << 12];
    const int ncand = 1 << maxb;
    uint8_t key[1 << 12];
    for (int j = 0; j < ncand; j++) {
        const uint32_t e = t[j];
        int k = 0;
        if (e & kLiteral) {
            const int d = static_cast<int>(drop_of(e));
            const int bl = j ? 32 - __builtin_clz(static_cast<uint32_t>(j)) : 0;
            k = d > bl ? d : bl;
        }
        key[j] = static_cast<uint8_t>(k);
        if (k) cnt[k]++;
    }
    uint16_t start[18];
    start[0] = 0;
    for (int k = 0; k <= 16; k++) start[k + 1] = static_cast<uint16_t>(start[k] + (k ? cnt[k] : 0));
    for (int j = 0; j < ncand; j++)
        if (key[j]) { // (sec: the pair entry less the first literal's byte and length)
            const uint16_t at = start[key[j]]++;
            cand[at] = static_cast<uint16_t>(j);
            sec[at] = kLiteral | kLiteral2 | payload(t[j]) << 24 | drop_of(t[j]);
        }
    // (start[k] now ends budget k's run: the candidates of budget <= b are
    // cand[0 .. start[b]))
    for (int s = 0; s < 256 && s < n; s++) {
        const int l1 = lens[s];
        if (!l1 || l1 > maxb) continue;
        const uint32_t r1 = rev[s]; // (the root's canonical code, from build())
        const int end = start[root - l1];
        const uint32_t add = uint32_t(s) << 16 | uint32_t(l1);
        for (int i = 0; i < end; i++) t[r1 | static_cast<uint32_t>(cand[i]) << l1] = sec[i] + add;
    }
}

// One or two literals (a kLiteral entry) at o, in the fast zone: the second
// slot is written either way (a single literal's is overwritten next)
template <typename T> inline T *put_literals(T *o, uint32_t e)
{
    o[0] = static_cast<T>(payload(e) & 0xff);
    o[1] = static_cast<T>(payload(e) >> 8);
    return o + 1 + ((e >> 14) & 1);
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
    // input bit position of the next unconsumed bit
    inline uint64_t bitpos() const { return uint64_t(pos) * 8 + uint64_t(pad) - uint64_t(cnt); }
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

// match copy of n elements from distance d (d <= elements already written)
template <typename T> inline void copy_match(T *dst, size_t d, size_t n)
{
    const T *src = dst - d;
    if (d * sizeof(T) >= 8) {
        size_t k = 0;
        constexpr size_t kStep = 8 / sizeof(T);
        for (; k + kStep <= n; k += kStep) { // with d >= 8 bytes a chunk never reads what it writes
            uint64_t w;
            memcpy(&w, src + k, 8);
            memcpy(dst + k, &w, 8);
        }
        for (; k < n; k++) dst[k] = src[k];
    } else {
        for (size_t k = 0; k < n; k++) dst[k] = src[k];
    }
}

// Output of one decode run: a fixed buffer (capacity = the bytes wanted) or
// a growable one (the parallel path's speculative chunks).
// A vector whose resize() leaves new elements uninitialised (the decoder
// writes every element it keeps)
template <class T> struct NoInitAlloc : std::allocator<T> {
    template <class U> struct rebind {
        using other = NoInitAlloc<U>;
    };
    NoInitAlloc() = default;
    template <class U> NoInitAlloc(const NoInitAlloc<U> &) noexcept {}
    template <class U> void construct(U *p) noexcept { ::new (static_cast<void *>(p)) U; }
    template <class U, class... A> void construct(U *p, A &&...a)
    {
        ::new (static_cast<void *>(p)) U(std::forward<A>(a)...);
    }
};
template <typename T> using RawVec = std::vector<T, NoInitAlloc<T>>;

// The speculative chunks' symbol buffers, recycled: 8 MB a chunk, zeroed and
// page-faulted in on every call when they were fresh vectors (at most
// 1 GiB and 64 buffers held -- the chunks of 8 concurrent 8-thread
// inflates; inflate_pool_trim releases them)
class SymPool {
  public:
    RawVec<uint16_t> take()
    {
        std::lock_guard<std::mutex> lk(mu_);
        if (free_.empty()) return {};
        RawVec<uint16_t> v = std::move(free_.back());
        free_.pop_back();
        held_ -= v.capacity() * 2;
        return v;
    }
    void give(RawVec<uint16_t> &&v)
    {
        RawVec<uint16_t> keep = std::move(v); // (freed on return unless pooled)
        std::lock_guard<std::mutex> lk(mu_);
        if (keep.capacity() == 0 || held_ + keep.capacity() * 2 > (size_t(1) << 30) || free_.size() >= 64) return;
        held_ += keep.capacity() * 2;
        free_.push_back(std::move(keep));
    }
    size_t trim()
    {
        std::vector<RawVec<uint16_t>> gone;
        std::lock_guard<std::mutex> lk(mu_);
        const size_t n = held_;
        gone.swap(free_);
        held_ = 0;
        return n;
    }

  private:
    std::mutex mu_;
    std::vector<RawVec<uint16_t>> free_;
    size_t held_ = 0;
};
SymPool &sym_pool()
{
    static SymPool *p = new SymPool; // (intentionally leaked)
    return *p;
}

// `o` is the committed end (a block's start while its symbols decode).
template <typename T> struct Out {
    T *p = nullptr;
    size_t o = 0, cap = 0;
    RawVec<T> *grow = nullptr;
    // room for n elements from element `at` (a growable buffer grows; p may move)
    bool room(size_t at, size_t n)
    {
        if (at + n <= cap) return true;
        if (!grow) return false;
        const size_t nc = std::max(2 * cap, at + n + (size_t(1) << 20));
        grow->resize(nc);
        p = grow->data();
        cap = nc;
        return true;
    }
};

// The dynamic block header (RFC 1951 3.2.7) after BTYPE: both tables.
// (lit_lens: the literal/length code lengths, for pair_literals; may be null)
bool read_dynamic(Bits &b, uint32_t *lit, uint32_t *dist, uint8_t *lit_lens = nullptr, int *nlit = nullptr,
                  uint16_t *lit_rev = nullptr)
{
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
    uint32_t clt[1 << 7];
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
    if (!build(lit, kLitEntries, lens, hlit, kLitBits, Kind::LitLen, lit_rev)) return false;
    if (lit_lens) {
        memcpy(lit_lens, lens, static_cast<size_t>(hlit));
        *nlit = hlit;
    }
    if (!build(dist, kDistEntries, lens + hlit, hdist, kDistBits, Kind::Dist)) return false;
    return !b.overrun();
}

// A stored block (its 3 header bits consumed): the byte offset `at` of its
// `len` data bytes in b.in; b moves past them.  False when it is irregular.
bool stored_block(Bits &b, size_t &at, uint32_t &len)
{
    if (b.overrun()) return false;
    b.drop((b.cnt - b.pad) & 7);
    // re-sync the byte position to the bit buffer (whole real bytes still
    // buffered go back to the input)
    const size_t bytes_in_buf = static_cast<size_t>((b.cnt - b.pad) >> 3);
    size_t p = b.pos - bytes_in_buf;
    b.buf = 0;
    b.cnt = 0;
    b.pad = 0;
    b.pos = p;
    if (p + 4 > b.len) return false;
    len = b.in[p] | uint32_t(b.in[p + 1]) << 8;
    const uint32_t nlen = b.in[p + 2] | uint32_t(b.in[p + 3]) << 8;
    if ((len ^ 0xffffu) != nlen) return false;
    p += 4;
    if (p + len > b.len) return false;
    at = p;
    b.pos = p + len;
    return true;
}

// The decode tables of a fixed (type 1) or dynamic (type 2) block whose 3
// header bits are consumed, literal pairs included.  False when irregular.
bool block_tables(Bits &b, uint32_t type, uint32_t *lit, uint32_t *dist)
{
    uint16_t rev[320];
    uint8_t l[320];
    int nl = 0;
    if (type == 1) { // fixed codes
        for (int i = 0; i < 144; i++) l[i] = 8;
        for (int i = 144; i < 256; i++) l[i] = 9;
        for (int i = 256; i < 280; i++) l[i] = 7;
        for (int i = 280; i < 288; i++) l[i] = 8;
        // zlib's fixed table has 288 literal/length symbols (286, 287 invalid when used)
        if (!build(lit, kLitEntries, l, 288, kLitBits, Kind::LitLen, rev)) return false;
        nl = 288;
        uint8_t d[32];
        for (int i = 0; i < 32; i++) d[i] = 5;
        if (!build(dist, kDistEntries, d, 32, kDistBits, Kind::Dist)) return false;
    } else if (type == 2) { // dynamic
        if (!read_dynamic(b, lit, dist, l, &nl, rev)) return false;
    } else {
        return false;
    }
    pair_literals(lit, kLitBits, l, nl, rev);
    return !b.overrun();
}

// One step of a block's symbols in the fast zone (real input bytes behind
// every bit, room for a whole match + a pair's second slot): up to three
// literal lookups, or one match.  0: go on, 1: the block ended, 2: an invalid
// symbol or a distance before the output's start (`floor` elements before
// base are readable).
// The rest of a fast-zone step from its (k+1)-th lookup, whose entry is e
// (k < 3 lookups done since the step's refill).
template <typename T>
inline int fast_step_from(Bits &b, T *&o, uint32_t e, int k, const uint32_t *lt, const uint32_t *dt, const T *base,
                          size_t floor)
{
    while (e & kLiteral) {
        o = put_literals(o, e);
        if (++k == 3) return 0;
        e = decode(b, lt, kLitBits);
    }
    if (e & (kEob | kInvalid)) return (e & kInvalid) ? 2 : 1;
    // a length: its extra bits, then the distance (one refill covers extra
    // <= 5 + distance code <= 15 + extra <= 13 bits)
    b.refill_fast();
    const uint32_t len = payload(e) + b.take(static_cast<int>(extra_of(e)));
    const uint32_t de = decode(b, dt, kDistBits);
    if (de & kInvalid) return 2;
    const uint32_t d = payload(de) + b.take(static_cast<int>(extra_of(de)));
    if (d > size_t(o - base) + floor) return 2;
    copy_match(o, d, len);
    o += len;
    return 0;
}

template <typename T>
inline int fast_step(Bits &b, T *&o, const uint32_t *lt, const uint32_t *dt, const T *base, size_t floor)
{
    b.refill_fast();
    return fast_step_from(b, o, decode(b, lt, kLitBits), 0, lt, dt, base, floor);
}

// Steps of two streams a and b with their lookups interleaved (a's and b's
// chains side by side while both decode literals): ra / rb as fast_step's.
inline void fast_step2(Bits &a, uint8_t *&oa, const uint32_t *la, const uint32_t *da, const uint8_t *ba, int &ra,
                       Bits &b, uint8_t *&ob, const uint32_t *lb, const uint32_t *db, const uint8_t *bb, int &rb)
{
    a.refill_fast();
    b.refill_fast();
    uint32_t ea = decode(a, la, kLitBits), eb = decode(b, lb, kLitBits);
    int k = 0;
    while (ea & eb & kLiteral) {
        oa = put_literals(oa, ea);
        ob = put_literals(ob, eb);
        if (++k == 3) {
            ra = rb = 0;
            return;
        }
        ea = decode(a, la, kLitBits);
        eb = decode(b, lb, kLitBits);
    }
    ra = fast_step_from(a, oa, ea, k, la, da, ba, 0);
    rb = fast_step_from(b, ob, eb, k, lb, db, bb, 0);
}

enum class Run { Want, Final, AtStop, Error };

// Decodes blocks from b's position into out until out.o reaches `want`
// (Want), the final block ends (Final), or a block header is about to start
// at bit `stop` (AtStop; nothing of it consumed).  A block header past `stop`
// sets `overshot` (the caller then moves the stop on).  `floor` is how far
// back a distance may reach before out.p[0] (the speculative window).
template <typename T>
Run decode_blocks(Bits &b, Out<T> &out, size_t want, uint64_t stop, bool &overshot, size_t floor)
{
    // the tables on the stack (48 KiB): a thread_local's address in this
    // -fPIC library is a __tls_get_addr call, which gcc re-issued before
    // every lookup of the symbol loop instead of keeping it in a register
    uint32_t lit[kLitEntries], dist[kDistEntries];
    for (;;) {
        if (out.o >= want) return Run::Want;
        const uint64_t at = b.bitpos();
        if (at == stop) return Run::AtStop;
        if (at > stop) overshot = true;
        b.refill();
        const bool last = b.take(1) != 0;
        const uint32_t type = b.take(2);
        if (type == 0) { // stored
            size_t at;
            uint32_t len;
            if (!stored_block(b, at, len)) return Run::Error;
            size_t n = len;
            if (!out.room(out.o, n)) n = std::min<size_t>(n, out.cap - out.o);
            n = std::min(n, want - out.o);
            for (size_t k = 0; k < n; k++) out.p[out.o + k] = b.in[at + k];
            out.o += n;
            if (last) return out.o >= want ? Run::Want : Run::Final;
            continue;
        }
        if (!block_tables(b, type, lit, dist)) return Run::Error;
        // ---- the block's symbols.  The loop keeps the bit reader, the
        // tables and the output pointers in locals: `o`'s stores (bytes) may
        // alias any memory, so members of b / out would be re-read around
        // every symbol.
        Bits bl = b;
        const uint32_t *const lt = lit, *const dt = dist;
        T *base = out.p, *o = base + out.o;
        // the fast zone: real input bytes behind every bit and room for a
        // whole match + a pair's second slot (258 + 8) -- no end checks
        // per symbol; it holds while o <= fend
        size_t lim = std::min(want, out.cap);
        T *fend = base + (lim >= 266 ? lim - 266 : 0);
        bool fast_ok = lim >= 266;
        for (;;) {
            uint32_t e;
            if (fast_ok && o <= fend && bl.pos + 32 <= bl.len) {
                const int r = fast_step(bl, o, lt, dt, base, floor);
                if (r == 0) continue;
                if (r == 2) {
                    b = bl;
                    return Run::Error;
                }
                break; // the block's end
            }
            const size_t done = static_cast<size_t>(o - base);
            if (out.grow && bl.pos + 32 <= bl.len && done + 266 <= want && done + 266 > out.cap) {
                // a growable buffer out of fast-zone room: grow it and go on fast
                out.room(done, size_t(1) << 16);
                base = out.p;
                o = base + done;
                lim = std::min(want, out.cap);
                fend = base + (lim >= 266 ? lim - 266 : 0);
                fast_ok = lim >= 266;
                continue;
            }
            // careful path near the end of the input or the output
            bl.refill();
            e = decode(bl, lt, kLitBits);
            if (bl.overrun() || (e & kInvalid)) {
                b = bl;
                return Run::Error;
            }
            if (e & kLiteral) {
                if (done >= want) break;
                const size_t n = std::min<size_t>((e & kLiteral2) ? 2 : 1, want - done);
                if (!out.room(done, n)) {
                    b = bl;
                    return Run::Error;
                }
                base = out.p;
                base[done] = static_cast<T>(payload(e) & 0xff);
                if (n == 2) base[done + 1] = static_cast<T>(payload(e) >> 8);
                o = base + done + n;
                continue;
            }
            if (e & kEob) break;
            bl.refill();
            const uint32_t len = payload(e) + bl.take(static_cast<int>(extra_of(e)));
            bl.refill();
            const uint32_t de = decode(bl, dt, kDistBits);
            if (de & kInvalid) {
                b = bl;
                return Run::Error;
            }
            const uint32_t d = payload(de) + bl.take(static_cast<int>(extra_of(de)));
            if (bl.overrun() || d > done + floor) {
                b = bl;
                return Run::Error;
            }
            size_t n = len < want - done ? len : want - done;
            if (!out.room(done, n)) {
                b = bl;
                return Run::Error;
            }
            base = out.p;
            copy_match(base + done, d, n);
            o = base + done + n;
            if (done + n >= want) break;
        }
        b = bl;
        // (base == out.p: every growth above re-read it)
        out.o = static_cast<size_t>(o - base);
        if (out.o >= want) return Run::Want;
        if (last) return Run::Final;
    }
}

bool zlib_header_ok(const uint8_t *in, size_t in_len)
{
    if (in_len < 2) return false;
    const uint32_t cmf = in[0], flg = in[1];
    return (cmf & 15) == 8 && (cmf >> 4) <= 7 && ((cmf << 8) | flg) % 31 == 0 && !(flg & 0x20);
}

inline Bits bits_at(const uint8_t *in, size_t len, uint64_t bit)
{
    Bits b;
    b.in = in;
    b.len = len;
    b.pos = static_cast<size_t>(bit >> 3);
    b.refill();
    b.drop(static_cast<int>(bit & 7));
    return b;
}

// A dynamic-Huffman block header could start at `bit`: BTYPE 2 and both
// code sets complete (the speculative chunks' start search).
bool plausible_block(const uint8_t *in, size_t len, uint64_t bit)
{
    const size_t byte = static_cast<size_t>(bit >> 3);
    if (byte + 2 >= len) return false;
    const uint32_t w = (in[byte] | uint32_t(in[byte + 1]) << 8 | uint32_t(in[byte + 2]) << 16) >> (bit & 7);
    if ((w >> 1 & 3) != 2) return false;                  // BTYPE = dynamic
    if ((w >> 3 & 31) > 29 || (w >> 8 & 31) > 29) return false; // HLIT, HDIST
    Bits b = bits_at(in, len, bit + 3);
    static thread_local uint32_t lit[kLitEntries], dist[kDistEntries];
    return read_dynamic(b, lit, dist);
}


// ---- Two streams in one loop (inflate_fast_pair).  A noisy stream's symbol
// loop is one dependency chain -- table lookup, shift, the next lookup --
// that leaves most of a core's issue slots idle; two independent streams
// stepped in turn in one loop overlap their chains.
struct PairDec {
    Bits b;
    uint8_t *p = nullptr;
    size_t o = 0, want = 0;
    bool last = false;
    enum State { Header, Symbols, Done, Fail } st = Header;
    uint32_t lit[kLitEntries], dist[kDistEntries];
    bool fast() const { return want >= 266 && o <= want - 266 && b.pos + 32 <= b.len; }
};

// st Header: the next block's header -- a stored block is copied whole, a
// Huffman block's tables are built (st Symbols) -- Done once `want` bytes
// are out, Fail on anything irregular or a stream that ends short
// (decode_blocks' rules with a fixed output)
void pair_header(PairDec &d)
{
    Bits &b = d.b;
    while (d.st == PairDec::Header) {
        if (d.o >= d.want) {
            d.st = PairDec::Done;
            return;
        }
        if (d.last) {
            d.st = PairDec::Fail;
            return;
        }
        b.refill();
        d.last = b.take(1) != 0;
        const uint32_t type = b.take(2);
        if (type == 0) {
            size_t at;
            uint32_t len;
            if (!stored_block(b, at, len)) {
                d.st = PairDec::Fail;
                return;
            }
            const size_t n = std::min<size_t>(len, d.want - d.o);
            memcpy(d.p + d.o, b.in + at, n);
            d.o += n;
            continue;
        }
        d.st = block_tables(b, type, d.lit, d.dist) ? PairDec::Symbols : PairDec::Fail;
    }
}

// st Symbols outside the fast zone: the block's rest symbol by symbol with
// every end check (decode_blocks' careful path); st Header at its end or
// when the output is full, Fail on anything irregular
void pair_careful(PairDec &d)
{
    Bits &b = d.b;
    for (;;) {
        const size_t done = d.o;
        b.refill();
        const uint32_t e = decode(b, d.lit, kLitBits);
        if (b.overrun() || (e & kInvalid)) break;
        if (e & kLiteral) {
            if (done >= d.want) {
                d.st = PairDec::Header;
                return;
            }
            const size_t n = std::min<size_t>((e & kLiteral2) ? 2 : 1, d.want - done);
            d.p[done] = static_cast<uint8_t>(payload(e) & 0xff);
            if (n == 2) d.p[done + 1] = static_cast<uint8_t>(payload(e) >> 8);
            d.o = done + n;
            continue;
        }
        if (e & kEob) {
            d.st = PairDec::Header;
            return;
        }
        b.refill();
        const uint32_t len = payload(e) + b.take(static_cast<int>(extra_of(e)));
        b.refill();
        const uint32_t de = decode(b, d.dist, kDistBits);
        if (de & kInvalid) break;
        const uint32_t dd = payload(de) + b.take(static_cast<int>(extra_of(de)));
        if (b.overrun() || dd > done) break;
        const size_t n = std::min<size_t>(len, d.want - done);
        copy_match(d.p + done, dd, n);
        d.o = done + n;
        if (d.o >= d.want) {
            d.st = PairDec::Header;
            return;
        }
    }
    d.st = PairDec::Fail;
}

// Headers and careful stretches until the stream is in a block's fast zone
// (st Symbols with fast()), Done or Fail.
void pair_settle(PairDec &d)
{
    for (;;) {
        if (d.st == PairDec::Header) pair_header(d);
        else if (d.st == PairDec::Symbols && !d.fast()) pair_careful(d);
        else return;
    }
}

// The fast zones of N streams (st Symbols, fast()), stepped in turn until
// one leaves its zone or its block ends; their state is written back.
template <int N>
void pair_fast(PairDec *const *d)
{
    Bits b[N];
    uint8_t *base[N], *o[N], *end[N];
    const uint32_t *lt[N], *dt[N];
    int r[N];
#pragma GCC unroll 2
    for (int k = 0; k < N; k++) {
        b[k] = d[k]->b;
        base[k] = d[k]->p;
        o[k] = base[k] + d[k]->o;
        end[k] = base[k] + (d[k]->want - 266);
        lt[k] = d[k]->lit;
        dt[k] = d[k]->dist;
        r[k] = 0;
    }
    for (;;) {
        bool go = true;
#pragma GCC unroll 2
        for (int k = 0; k < N; k++) go = go && o[k] <= end[k] && b[k].pos + 32 <= b[k].len;
        if (!go) break;
        if constexpr (N == 2) {
            fast_step2(b[0], o[0], lt[0], dt[0], base[0], r[0], b[1], o[1], lt[1], dt[1], base[1], r[1]);
            if (r[0] | r[1]) break;
        } else {
            r[0] = fast_step(b[0], o[0], lt[0], dt[0], base[0], 0);
            if (r[0]) break;
        }
    }
#pragma GCC unroll 2
    for (int k = 0; k < N; k++) {
        d[k]->b = b[k];
        d[k]->o = static_cast<size_t>(o[k] - base[k]);
        if (r[k] == 1) d[k]->st = PairDec::Header;
        else if (r[k] == 2) d[k]->st = PairDec::Fail;
    }
}

} // namespace

bool inflate_fast(const uint8_t *in, size_t in_len, uint8_t *out, size_t want, size_t *produced)
{
    *produced = 0;
    if (!zlib_header_ok(in, in_len)) return false;
    Bits b = bits_at(in, in_len, 16);
    Out<uint8_t> o{out, 0, want, nullptr};
    bool overshot = false;
    const Run r = decode_blocks(b, o, want, ~uint64_t(0), overshot, 0);
    *produced = o.o;
    return r == Run::Want; // anything short of the requested bytes: let zlib decide
}

void inflate_fast_pair(const uint8_t *const in[2], const size_t in_len[2], uint8_t *const out[2], const size_t want[2],
                       size_t produced[2], bool ok[2])
{
    std::unique_ptr<PairDec> d0(new PairDec), d1(new PairDec);
    PairDec *d[2] = {d0.get(), d1.get()};
    for (int k = 0; k < 2; k++) {
        produced[k] = 0;
        if (!zlib_header_ok(in[k], in_len[k])) {
            d[k]->st = PairDec::Fail;
            continue;
        }
        d[k]->b = bits_at(in[k], in_len[k], 16);
        d[k]->p = out[k];
        d[k]->want = want[k];
    }
    for (;;) {
        pair_settle(*d[0]);
        pair_settle(*d[1]);
        const bool s0 = d[0]->st == PairDec::Symbols, s1 = d[1]->st == PairDec::Symbols;
        if (s0 && s1) pair_fast<2>(d);
        else if (s0) pair_fast<1>(d);
        else if (s1) pair_fast<1>(d + 1);
        else break;
    }
    for (int k = 0; k < 2; k++) {
        produced[k] = d[k]->o;
        ok[k] = d[k]->st == PairDec::Done;
    }
}

// Parallel inflate of one stream (the reference's single call
// at src/png/decoder.zig:516-518).  DEFLATE blocks are not independent (a
// match may reach 32 KiB back), so this is speculative, after the two-stage
// scheme of parallel gzip decoders:
//   1. the compressed bytes are cut into `threads` ranges; each range after
//      the first searches forward for a bit position where a dynamic block
//      header parses with complete code sets;
//   2. chunk 0 decodes from the stream start into the output, every other
//      chunk from its candidate into 16-bit symbols behind a 32 KiB window of
//      markers (value 256 + i = "byte i of the 32 KiB before this chunk"), so
//      matches that reach before the chunk copy markers.  A chunk stops at a
//      block header exactly at the next chunk's candidate: landing on it
//      proves the candidate a real block boundary; passing it moves the stop
//      to the candidate after (the passed chunk is discarded);
//   3. the chunks' last 32 KiB resolve in order (each only needs the previous
//      output's last 32 KiB), then the rest of every chunk in parallel.
// Anything irregular returns false and the caller runs the serial decoder,
// so results are the serial path's by construction.
// Runs job(i) for i in [first, n) on new threads, then job(i) for i < first
// on this one, and joins them all.  False when a thread could not be started
// (thread or pid limit): the threads already running are joined, nothing
// unwinds past a joinable std::thread, and the caller falls back to the
// serial decoder.
template <typename F>
bool run_pool(int first, int n, F &&job)
{
    std::vector<std::thread> pool;
    bool started = true;
    try {
        pool.reserve(static_cast<size_t>(n > first ? n - first : 0));
        for (int i = first; i < n; i++) pool.emplace_back(job, i);
    } catch (...) {
        started = false;
    }
    if (started)
        for (int i = 0; i < first; i++) job(i);
    for (auto &t : pool) t.join();
    return started;
}

bool inflate_parallel(const uint8_t *in, size_t in_len, uint8_t *out, size_t want, size_t *produced, int threads)
{
    *produced = 0;
    constexpr size_t kWin = 32768;
    if (threads < 2 || !zlib_header_ok(in, in_len)) return false;
    const int T = threads;
    std::vector<uint64_t> cand(T + 1, ~uint64_t(0));
    cand[0] = 16;
    const uint64_t total_bits = uint64_t(in_len) * 8;
    // 1. candidate starts
    auto search = [&](int i) {
        const uint64_t lo = total_bits * uint64_t(i) / uint64_t(T);
        const uint64_t hi = total_bits * uint64_t(i + 1) / uint64_t(T);
        for (uint64_t p = lo; p < hi; p++)
            if (plausible_block(in, in_len, p)) {
                cand[i] = p;
                return;
            }
    };
    if (!run_pool(1, T, [&](int i) { if (i) search(i); })) return false; // (cand[0] is the stream start)
    // 2. speculative decode, chunk i from cand[i] to the next candidate it lands on
    struct Chunk {
        RawVec<uint16_t> sym = sym_pool().take();
        ~Chunk() { sym_pool().give(std::move(sym)); }
        Chunk() = default;
        Chunk(Chunk &&) = default;
        size_t n = 0;       // output elements (without the window)
        int next = -1;      // index of the candidate it landed on (T = the stream end)
        bool ok = false;
    };
    std::vector<Chunk> ch(T);
    auto run = [&](int i) {
        Chunk &c = ch[i];
        if (cand[i] == ~uint64_t(0)) return;
        Bits b = bits_at(in, in_len, cand[i]);
        int nx = i + 1;
        while (nx < T && cand[nx] == ~uint64_t(0)) nx++;
        if (i == 0) {
            Out<uint8_t> o{out, 0, want, nullptr};
            for (;;) {
                bool over = false;
                const Run r = decode_blocks(b, o, want, nx < T ? cand[nx] : ~uint64_t(0), over, 0);
                if (r == Run::AtStop) {
                    c.ok = true;
                    c.next = nx;
                    break;
                }
                if (r == Run::Want) {
                    c.ok = true;
                    c.next = T;
                    break;
                }
                if (r != Run::Error && over && nx < T) { // passed a false candidate: aim at the next
                    do nx++;
                    while (nx < T && cand[nx] == ~uint64_t(0));
                    continue;
                }
                break;
            }
            c.n = o.o;
            return;
        }
        // the 32 KiB window of markers, then the chunk's symbols (growable)
        c.sym.resize(kWin + (size_t(1) << 22));
        for (size_t k = 0; k < kWin; k++) c.sym[k] = static_cast<uint16_t>(256 + k);
        Out<uint16_t> o{c.sym.data(), kWin, c.sym.size(), &c.sym};
        for (;;) {
            bool over = false;
            const Run r = decode_blocks(b, o, ~size_t(0) >> 1, nx < T ? cand[nx] : ~uint64_t(0), over, 0);
            if (r == Run::AtStop) {
                c.ok = true;
                c.next = nx;
                break;
            }
            if (r == Run::Final) {
                c.ok = true;
                c.next = T;
                break;
            }
            if (r != Run::Error && over && nx < T) {
                do nx++;
                while (nx < T && cand[nx] == ~uint64_t(0));
                continue;
            }
            break;
        }
        o.o -= kWin;
        c.n = o.o;
    };
    if (!run_pool(1, T, run)) return false; // (chunk 0 on this thread)
    // the chain of chunks that landed on each other, from chunk 0 to the end
    std::vector<int> chain;
    size_t total = 0;
    for (int i = 0; i < T;) {
        if (!ch[i].ok) return false;
        chain.push_back(i);
        total += ch[i].n;
        if (ch[i].next >= T) break;
        i = ch[i].next;
    }
    if (ch[chain.back()].next < T) return false;
    if (total < want) return false;
    // 3. resolve: offsets, tails in order, then the bulk in parallel
    std::vector<size_t> off(chain.size());
    size_t acc = 0;
    for (size_t k = 0; k < chain.size(); k++) {
        off[k] = acc;
        acc += ch[chain[k]].n;
    }
    auto resolve = [&](size_t k, size_t from, size_t to) -> bool {
        const Chunk &c = ch[chain[k]];
        const size_t base = off[k];
        if (base < kWin) { // a marker would reach before the stream start
            for (size_t j = from; j < to; j++)
                if (c.sym[kWin + j] >= 256 && base + (c.sym[kWin + j] - 256) < kWin) return false;
        }
        const uint8_t *win = out + base - kWin; // only dereferenced for markers, which are in range
        const size_t end = std::min(to, want - std::min(want, base));
        for (size_t j = from; j < end; j++) {
            const uint16_t s = c.sym[kWin + j];
            out[base + j] = s < 256 ? static_cast<uint8_t>(s) : win[s - 256];
        }
        return true;
    };
    for (size_t k = 1; k < chain.size(); k++) {
        const size_t n = ch[chain[k]].n;
        if (off[k] >= want) break;
        if (!resolve(k, n > kWin ? n - kWin : 0, n)) return false;
    }
    std::atomic<bool> bad{false};
    std::vector<size_t> bulk; // chunks with a bulk before their last 32 KiB
    for (size_t k = 1; k < chain.size(); k++)
        if (ch[chain[k]].n > kWin && off[k] < want) bulk.push_back(k);
    const bool started = run_pool(0, static_cast<int>(bulk.size()), [&](int j) {
        const size_t k = bulk[static_cast<size_t>(j)];
        if (!resolve(k, 0, ch[chain[k]].n - kWin)) bad = true;
    });
    if (!started || bad) return false;
    *produced = want;
    return true;
}

size_t inflate_pool_trim() { return sym_pool().trim(); }

} // namespace zpx
