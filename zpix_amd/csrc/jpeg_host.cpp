// Host entropy stage of the JPEG path.  Same observable behaviour as the
// reference decoder (coefficients and error names), organised for the device
// split: scans always accumulate into coefficient grids and no pixel is
// produced here.  References are to src/jpeg/decoder.zig unless noted.
#include "jpeg_host.h"
#include "host_cpus.h"

#include <hip/hip_runtime.h>

#include <cstdlib>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <condition_variable>
#include <memory>
#include <type_traits>
#include <cstring>
#include <thread>
#include <map>
#include <mutex>

namespace zpx {

// ---------------------------------------------------------------- HostBuf
HostBuf &HostBuf::operator=(HostBuf &&o) noexcept
{
    if (this != &o) {
        release();
        ptr = o.ptr;
        bytes = o.bytes;
        cap = o.cap;
        pinned = o.pinned;
        o.ptr = nullptr;
        o.bytes = 0;
        o.cap = 0;
        o.pinned = false;
    }
    return *this;
}

static bool pinned_allowed()
{
    // function-local static: initialised once, thread-safe (batch workers
    // allocate concurrently)
    static const bool ok = [] {
        const char *env = getenv("ZPX_NO_PINNED");
        int n = 0;
        return !(env && env[0] == '1') && hipGetDeviceCount(&n) == hipSuccess && n > 0;
    }();
    return ok;
}

namespace {
// Free pinned buffers by capacity.  Never freed at exit (the HIP runtime may
// already be gone); bounded by ZPX_PINNED_POOL_MB (default 2048).
struct PinnedPool {
    std::mutex mu;
    std::multimap<size_t, void *> free_;
    size_t held = 0, limit = 0;
    PinnedPool()
    {
        const char *env = getenv("ZPX_PINNED_POOL_MB");
        limit = size_t(env ? atol(env) : 2048) << 20;
    }
    static size_t size_class(size_t n)
    {
        const size_t g = n >= (size_t(1) << 20) ? (size_t(1) << 20) : 4096;
        return (n + g - 1) / g * g;
    }
    void *take(size_t c, size_t &got) // a buffer of capacity got in [c, 1.25c]
    {
        std::lock_guard<std::mutex> lk(mu);
        auto it = free_.lower_bound(c);
        if (it == free_.end() || it->first > c + c / 4) return nullptr;
        void *p = it->second;
        got = it->first;
        held -= it->first;
        free_.erase(it);
        return p;
    }
    bool give(void *p, size_t c)
    {
        std::lock_guard<std::mutex> lk(mu);
        if (held + c > limit) return false;
        free_.emplace(c, p);
        held += c;
        return true;
    }
};
PinnedPool &pinned_pool()
{
    static PinnedPool *pool = new PinnedPool; // intentionally leaked
    return *pool;
}
} // namespace

bool HostBuf::alloc(size_t n, bool zero)
{
    release();
    if (n == 0) n = 1;
    if (pinned_allowed()) {
        const size_t c = PinnedPool::size_class(n);
        size_t got = c;
        ptr = pinned_pool().take(c, got);
        if (!ptr && hipHostMalloc(&ptr, c, hipHostMallocDefault) != hipSuccess) ptr = nullptr;
        if (ptr) {
            pinned = true;
            cap = got;
        }
    }
    if (!ptr) {
        ptr = aligned_alloc(64, (n + 63) & ~size_t(63));
        pinned = false;
        cap = 0;
        if (!ptr) return false;
    }
    bytes = n;
    if (zero) memset(ptr, 0, n);
    return true;
}

void HostBuf::release()
{
    if (ptr) {
        if (pinned) {
            if (!pinned_pool().give(ptr, cap)) (void)hipHostFree(ptr);
        } else {
            free(ptr);
        }
    }
    ptr = nullptr;
    bytes = 0;
    cap = 0;
    pinned = false;
}

// ---------------------------------------------------------------- CoeffGrid
bool CoeffGrid::init(size_t blocks, bool zero, int bits)
{
    blocks_ = blocks;
    bits_ = bits;
    max_abs_ = 0;
    return buf_.alloc(blocks * 64 * static_cast<size_t>(bits / 8), zero);
}

bool CoeffGrid::set(size_t blk, int i, int32_t v)
{
    const int32_t a = v < 0 ? (v == INT32_MIN ? INT32_MAX : -v) : v;
    if (a > max_abs_) {
        max_abs_ = a;
        const int need = a > 32767 ? 32 : a > 127 ? 16 : 8;
        if (need > bits_ && !widen_to(need)) return false;
    }
    const size_t k = blk * 64 + static_cast<size_t>(i);
    if (bits_ == 8) static_cast<int8_t *>(buf_.ptr)[k] = static_cast<int8_t>(v);
    else if (bits_ == 16) static_cast<int16_t *>(buf_.ptr)[k] = static_cast<int16_t>(v);
    else static_cast<int32_t *>(buf_.ptr)[k] = v;
    return true;
}

bool CoeffGrid::narrow_to8(int threads)
{
    if (bits_ != 16 || max_abs_ > 127) return true;
    HostBuf nb;
    const size_t n = blocks_ * 64;
    if (!nb.alloc(n, false)) return false;
    const int16_t *src = static_cast<const int16_t *>(buf_.ptr);
    int8_t *dst = static_cast<int8_t *>(nb.ptr);
    const int nthr = static_cast<int>(std::max<size_t>(1, std::min<size_t>(static_cast<size_t>(std::max(1, threads)),
                                                                             n / (1u << 20))));
    auto part = [&](int t) {
        const size_t a = n * t / nthr, z = n * (t + 1) / nthr;
        for (size_t i = a; i < z; i++) dst[i] = static_cast<int8_t>(src[i]);
    };
    std::vector<std::thread> th;
    for (int t = 1; t < nthr; t++) {
        try {
            th.emplace_back(part, t);
        } catch (...) {
            part(t);
        }
    }
    part(0);
    for (auto &t : th) t.join();
    buf_ = static_cast<HostBuf &&>(nb);
    bits_ = 8;
    return true;
}

void CoeffGrid::load(size_t blk, int32_t *b) const
{
    if (bits_ == 32) {
        memcpy(b, static_cast<const int32_t *>(buf_.ptr) + blk * 64, 64 * sizeof(int32_t));
    } else if (bits_ == 16) {
        const int16_t *s = static_cast<const int16_t *>(buf_.ptr) + blk * 64;
        for (int i = 0; i < 64; i++) b[i] = s[i];
    } else {
        const int8_t *s = static_cast<const int8_t *>(buf_.ptr) + blk * 64;
        for (int i = 0; i < 64; i++) b[i] = s[i];
    }
}

bool CoeffGrid::widen_to(int bits)
{
    if (bits <= bits_) return true;
    HostBuf nb;
    const size_t n = blocks_ * 64;
    if (!nb.alloc(n * (bits / 8), false)) return false;
    for (size_t i = 0; i < n; i++) {
        const int32_t v = bits_ == 8 ? static_cast<const int8_t *>(buf_.ptr)[i] : static_cast<const int16_t *>(buf_.ptr)[i];
        if (bits == 16) static_cast<int16_t *>(nb.ptr)[i] = static_cast<int16_t>(v);
        else static_cast<int32_t *>(nb.ptr)[i] = v;
    }
    buf_ = static_cast<HostBuf &&>(nb);
    bits_ = bits;
    return true;
}

bool CoeffGrid::store(size_t blk, const int32_t *b)
{
    int32_t m = max_abs_;
    for (int i = 0; i < 64; i++) {
        int32_t a = b[i] < 0 ? -b[i] : b[i];
        if (a > m || a < 0) m = (a < 0) ? INT32_MAX : a;
    }
    max_abs_ = m;
    const int need = m > 32767 ? 32 : m > 127 ? 16 : 8;
    if (need > bits_ && !widen_to(need)) return false;
    if (bits_ == 32) {
        memcpy(static_cast<int32_t *>(buf_.ptr) + blk * 64, b, 64 * sizeof(int32_t));
    } else if (bits_ == 16) {
        int16_t *d = static_cast<int16_t *>(buf_.ptr) + blk * 64;
        for (int i = 0; i < 64; i++) d[i] = static_cast<int16_t>(b[i]);
    } else {
        int8_t *d = static_cast<int8_t *>(buf_.ptr) + blk * 64;
        for (int i = 0; i < 64; i++) d[i] = static_cast<int8_t>(b[i]);
    }
    return true;
}

bool CoeffGrid::store_sparse(size_t blk, const int32_t *b, const uint8_t *pos, int n)
{
    int32_t m = max_abs_;
    for (int i = 0; i < n; i++) {
        const int32_t v = b[pos[i]];
        int32_t a = v < 0 ? -v : v;
        if (a > m || a < 0) m = (a < 0) ? INT32_MAX : a;
    }
    max_abs_ = m;
    const int need = m > 32767 ? 32 : m > 127 ? 16 : 8;
    if (need > bits_ && !widen_to(need)) return false;
    if (bits_ == 8) {
        int8_t *d = static_cast<int8_t *>(buf_.ptr) + blk * 64;
        memset(d, 0, 64);
        for (int i = 0; i < n; i++) d[pos[i]] = static_cast<int8_t>(b[pos[i]]);
    } else if (bits_ == 16) {
        int16_t *d = static_cast<int16_t *>(buf_.ptr) + blk * 64;
        memset(d, 0, 128);
        for (int i = 0; i < n; i++) d[pos[i]] = static_cast<int16_t>(b[pos[i]]);
    } else {
        int32_t *d = static_cast<int32_t *>(buf_.ptr) + blk * 64;
        memset(d, 0, 256);
        for (int i = 0; i < n; i++) d[pos[i]] = b[pos[i]];
    }
    return true;
}

bool CoeffGrid::store_sparse_fixed(size_t blk, const int32_t *b, const uint8_t *pos, int n, int32_t &max_abs,
                                   std::vector<std::pair<size_t, int32_t>> &overflow) const
{
    const int lim = bits_ == 8 ? 127 : bits_ == 16 ? 32767 : INT32_MAX;
    const size_t base = blk * 64;
    if (bits_ == 8) memset(static_cast<int8_t *>(buf_.ptr) + base, 0, 64);
    else if (bits_ == 16) memset(static_cast<int16_t *>(buf_.ptr) + base, 0, 128);
    else memset(static_cast<int32_t *>(buf_.ptr) + base, 0, 256);
    for (int i = 0; i < n; i++) {
        const int32_t v = b[pos[i]];
        const int32_t a = v < 0 ? (v == INT32_MIN ? INT32_MAX : -v) : v;
        max_abs = a > max_abs ? a : max_abs;
        if (a > lim) {
            overflow.emplace_back(base + pos[i], v);
            continue;
        }
        if (bits_ == 8) static_cast<int8_t *>(buf_.ptr)[base + pos[i]] = static_cast<int8_t>(v);
        else if (bits_ == 16) static_cast<int16_t *>(buf_.ptr)[base + pos[i]] = static_cast<int16_t>(v);
        else static_cast<int32_t *>(buf_.ptr)[base + pos[i]] = v;
    }
    return true;
}

bool CoeffGrid::apply_overflow(int32_t max_abs, const std::vector<std::pair<size_t, int32_t>> &overflow)
{
    max_abs_ = max_abs > max_abs_ ? max_abs : max_abs_;
    const int need = max_abs_ > 32767 ? 32 : max_abs_ > 127 ? 16 : 8;
    if (!widen_to(need)) return false;
    for (const auto &o : overflow) {
        if (bits_ == 16) static_cast<int16_t *>(buf_.ptr)[o.first] = static_cast<int16_t>(o.second);
        else static_cast<int32_t *>(buf_.ptr)[o.first] = o.second;
    }
    return true;
}

bool JpegPieces::widen()
{
    if (bits == 16) return true;
    HostBuf nd;
    if (!nd.alloc((cap + 8) * 16, false)) return false;
    uint8_t *o = static_cast<uint8_t *>(nd.ptr);
    const int8_t *src = static_cast<const int8_t *>(data.ptr);
    memset(o, 0, 16);
    size_t nx[kMaxStreams];
    for (int s = 0; s < nstreams; s++) nx[s] = base[s];
    for (int c = 0; c < 4; c++) {
        if (blocks[c] == 0) continue;
        uint32_t *ix = index_of(c);
        for (size_t k = 0; k < blocks[c]; k++) {
            if (ix[k] == 0) continue;
            const int8_t *v8 = src + size_t(ix[k] >> 4) * 16;
            int eob = static_cast<int>(ix[k] & 15) * 16;
            while (eob > 0 && v8[eob - 1] == 0) eob--;
            const size_t np = static_cast<size_t>((eob + 7) / 8);
            size_t &n = nx[stream_of(c, k)];
            if (n + np > cap) return false;
            int16_t *d = reinterpret_cast<int16_t *>(o + n * 16);
            for (size_t z = 0; z < np * 8; z++) d[z] = static_cast<int16_t>(z < size_t(eob) ? v8[z] : 0);
            ix[k] = np ? static_cast<uint32_t>(n << 4 | np) : 0u;
            n += np;
        }
    }
    data = static_cast<HostBuf &&>(nd);
    for (int s = 0; s < nstreams; s++) next[s] = nx[s];
    bits = 16;
    return true;
}

void JpegPieces::compact()
{
    uint8_t *d = static_cast<uint8_t *>(data.ptr);
    size_t at = 1, shift[kMaxStreams];
    for (int s = 0; s < nstreams; s++) {
        const size_t n = next[s] - base[s];
        shift[s] = base[s] - at;
        if (shift[s] && n) memmove(d + at * 16, d + base[s] * 16, n * 16);
        base[s] = at;
        next[s] = at + n;
        at += n;
    }
    for (int c = 0; c < 4; c++) {
        if (blocks[c] == 0) continue;
        uint32_t *ix = index_of(c);
        const size_t rows = blocks[c] / gw[c];
        for (size_t by = 0; by < rows; by++) {
            const uint32_t d = static_cast<uint32_t>(shift[s0[c] + static_cast<int>(by % size_t(v[c]))] << 4);
            uint32_t *row = ix + by * gw[c];
            if (d)
                for (size_t k = 0; k < gw[c]; k++) row[k] -= row[k] ? d : 0u;
        }
    }
    npieces = at;
}

// ---------------------------------------------------------------- decoder
namespace {

// zig-zag -> natural index (decoder.zig:73-82)
constexpr uint8_t kUnzig[64] = {
    0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,
    12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6,  7,  14, 21, 28,
    35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51,
    58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63,
};
// natural -> zig-zag index
struct ZigOf {
    uint8_t z[64];
    constexpr ZigOf() : z()
    {
        for (int i = 0; i < 64; i++) z[kUnzig[i]] = static_cast<uint8_t>(i);
    }
};
constexpr ZigOf kZigOf{};

// AC symbols whose code (<= 8 bits) and magnitude bits fit the next
// kAcFastBits bits of the stream, decoded by one lookup (Huff::ac): entry =
// bits used (0: not here) | kAcEob | run << 8 | value << 16 (the extended
// coefficient, receiveExtend's).  A baseline q75 frame's AC codes are
// mostly 2-8 bits with 1-3 magnitude bits.
#ifndef ZPX_HUFF_FAST_BITS
#define ZPX_HUFF_FAST_BITS 11
#endif
constexpr int kAcFastBits = ZPX_HUFF_FAST_BITS;
constexpr uint32_t kAcEob = 16;
struct Huff { // HuffTable.zig
    int32_t num_codes = 0;
    uint16_t lut[256] = {};
    uint8_t vals[256] = {};
    int32_t min_codes[16] = {}, max_codes[16] = {}, vals_indices[16] = {};
    uint32_t ac[1u << kAcFastBits] = {}; // (dht; DC tables: the difference, run 0)
};

// internal status: the frame does not fit the pieces (jpeg_entropy_decode
// then decodes it again into grids); never returned to a caller
constexpr int kSparseAbort = 1 << 20;

#define ZTRY(e)                                                                \
    do {                                                                       \
        int e_ = (e);                                                          \
        if (e_) return e_;                                                     \
    } while (0)

class Decoder {
  public:
    Decoder(const uint8_t *p, size_t n, JpegCoeffs &out, bool config_only = false, int threads = 1,
            bool sparse = false)
        : src_(p), len_(n), o_(out), config_only_(config_only), threads_(threads), sparse_ok_(sparse)
    {
    }
    int run();
    static constexpr int kConfigOnly = -1; // decodeInner's error.ConfigOnly

  private:
    // --- byte source (the whole input stays addressable, so the
    //     unread-by-up-to-two-bytes of unreadByteStuffedByte (:479-487)
    //     is a plain rewind)
    int byte(uint8_t &x)
    { // readByte :402-410
        if (pos_ >= len_) return ZPX_E_UNEXPECTED_EOF;
        x = src_[pos_++];
        unread_ = 0;
        return 0;
    }
    void unread_stuffed()
    {
        pos_ -= unread_;
        unread_ = 0;
        if (bn_ >= 8) {
            ba_ >>= 8;
            bn_ -= 8;
            bm_ >>= 8;
        }
    }
    void settle()
    { // common prologue of readFull / ignore
        if (unread_ > 0) {
            if (bn_ >= 8) unread_stuffed();
            unread_ = 0;
        }
    }
    int full(uint8_t *p, size_t n)
    { // readFull :414-443
        settle();
        if (len_ - pos_ < n) {
            pos_ = len_;
            return ZPX_E_UNEXPECTED_EOF;
        }
        memcpy(p, src_ + pos_, n);
        pos_ += n;
        return 0;
    }
    int skip(int32_t n)
    { // ignore :376-398
        settle();
        if (len_ - pos_ < static_cast<size_t>(n)) {
            pos_ = len_;
            return ZPX_E_UNEXPECTED_EOF;
        }
        pos_ += static_cast<size_t>(n);
        return 0;
    }
    inline int stuffed(uint8_t &out)
    { // readByteStuffedByte :712-749
        if (pos_ + 2 <= len_) {
            uint8_t x = src_[pos_++];
            unread_ = 1;
            if (x != 0xff) {
                out = x;
                return 0;
            }
            if (src_[pos_] != 0x00) return ZPX_E_MISSING_FF00;
            pos_++;
            unread_ = 2;
            out = 0xff;
            return 0;
        }
        unread_ = 0;
        uint8_t x;
        ZTRY(byte(x));
        unread_ = 1;
        if (x != 0xff) {
            out = x;
            return 0;
        }
        ZTRY(byte(x));
        unread_ = 2;
        if (x != 0x00) return ZPX_E_MISSING_FF00;
        out = 0xff;
        return 0;
    }
    inline int ensure(int32_t n)
    { // ensureNBits :975-991
        do {
            uint8_t c;
            ZTRY(stuffed(c));
            ba_ = (ba_ << 8) | c;
            bn_ += 8;
            bm_ = bm_ == 0 ? 0x80u : bm_ << 8;
        } while (bn_ < n);
        return 0;
    }
    inline int huffman(const Huff &h, uint8_t &out)
    { // decodeHuffman :909-970
        if (h.num_codes == 0) return ZPX_E_UNINITIALIZED_HUFFMAN_TABLE;
        bool slow = false;
        if (bn_ < 8) {
            int e = ensure(8);
            if (e) {
                if (e != ZPX_E_MISSING_FF00) return e;
                if (unread_ != 0) unread_stuffed();
                slow = true;
            }
        }
        if (!slow) {
            uint16_t lv = h.lut[(ba_ >> (bn_ - 8)) & 0xff];
            if (lv != 0) {
                int32_t nb = static_cast<int32_t>(lv & 0xff) - 1;
                bn_ -= nb;
                bm_ >>= nb;
                out = static_cast<uint8_t>(lv >> 8);
                return 0;
            }
            // a code longer than 8 bits: resolve it from the bits already
            // buffered when they suffice -- exactly the bit loop below
            // (code after i+1 bits = the top i+1 buffered bits), without
            // reading a byte the loop would not have read
            for (int i = 8; i < 16 && i < bn_; i++) {
                const int32_t code = static_cast<int32_t>((ba_ >> (bn_ - (i + 1))) & ((1u << (i + 1)) - 1));
                if (code <= h.max_codes[i]) {
                    const int32_t idx = h.vals_indices[i] + code - h.min_codes[i];
                    if (idx < 0 || idx > 255) return ZPX_E_PANIC;
                    bn_ -= i + 1;
                    bm_ >>= i + 1;
                    out = h.vals[idx];
                    return 0;
                }
            }
        }
        int32_t code = 0;
        for (int i = 0; i < 16; i++) {
            if (bn_ == 0) ZTRY(ensure(1));
            if (ba_ & bm_) code |= 1;
            bn_--;
            bm_ >>= 1;
            if (code <= h.max_codes[i]) {
                int32_t idx = h.vals_indices[i] + code - h.min_codes[i];
                if (idx < 0 || idx > 255) return ZPX_E_PANIC;
                out = h.vals[idx];
                return 0;
            }
            code <<= 1;
        }
        return ZPX_E_BAD_HUFFMAN_CODE;
    }
    int bit(bool &b)
    { // decodeBit :994-1006
        if (bn_ == 0) ZTRY(ensure(1));
        b = (ba_ & bm_) != 0;
        bn_--;
        bm_ >>= 1;
        return 0;
    }
    int bits(int32_t n, uint32_t &out)
    { // decodeBits :1009-1022
        if (bn_ < n) ZTRY(ensure(n));
        uint32_t r = ba_ >> (bn_ - n);
        r &= n >= 32 ? 0xffffffffu : ((1u << n) - 1);
        bn_ -= n;
        bm_ >>= n;
        out = r;
        return 0;
    }
    inline int receive_extend(uint8_t t, int32_t &out)
    { // receiveExtend :1115-1134
        if (bn_ < static_cast<int32_t>(t)) ZTRY(ensure(t));
        bn_ -= t;
        bm_ >>= t;
        int32_t thr = int32_t(1) << t;
        int32_t v = static_cast<int32_t>((ba_ >> bn_) & static_cast<uint32_t>(thr - 1));
        v += ((v - (thr >> 1)) >> 31) & (static_cast<int32_t>(0xffffffffu << t) + 1); // (branch-free)
        out = v;
        return 0;
    }

    // one scan's parameters (processSos :1148-1296)
    struct Scan {
        int ns = 0;
        struct {
            uint8_t id = 0, td = 0, ta = 0;
        } c[4];
        int32_t zs = 0, ze = 63, mxx = 0, myy = 0;
        uint32_t ah = 0, al = 0;
        bool prog = false;
    };
    // how one decoded block is stored: the serial path widens the grid as
    // values need it; the parallel path writes a grid of fixed width
    struct SerialSink {
        JpegCoeffs &o;
        int put(int ci, size_t blk, int32_t *b, const uint8_t *pos, int n)
        {
            return o.grid[ci].store_sparse(blk, b, pos, n) ? 0 : ZPX_E_OUT_OF_MEMORY;
        }
    };
    // appends a block's pieces to o.pieces (see JpegPieces)
    struct PieceSink {
        JpegPieces &p;
        int put(int ci, size_t blk, int32_t *b, const uint8_t *pos, int n)
        {
            int32_t m = p.max_abs[ci];
            for (int i = 0; i < n; i++) {
                const int32_t v = b[pos[i]];
                const int32_t a = v < 0 ? -v : v;
                if (a > m || a < 0) m = a < 0 ? INT32_MAX : a;
            }
            if (m > 32767) return kSparseAbort;
            p.max_abs[ci] = m;
            if (p.bits == 8 && m > 127 && !p.widen()) return kSparseAbort;
            // pos[] is in decode (zig-zag) order and every AC entry is
            // nonzero: the end of block follows the last entry, unless the
            // block's only entry is a zero DC
            uint32_t &ix = p.index_of(ci)[blk];
            if (n == 0 || (n == 1 && b[pos[0]] == 0)) {
                ix = 0;
                return 0;
            }
            const int eob = kZigOf.z[pos[n - 1]] + 1;
            size_t &cur = p.next[p.stream_of(ci, blk)];
            uint8_t *d = static_cast<uint8_t *>(p.data.ptr) + cur * 16;
            size_t np;
            if (p.bits == 8) { // (the whole 64-byte block cleared: the data has that slack)
                np = static_cast<size_t>((eob + 15) >> 4);
                memset(d, 0, 64);
                for (int i = 0; i < n; i++) reinterpret_cast<int8_t *>(d)[kZigOf.z[pos[i]]] = static_cast<int8_t>(b[pos[i]]);
            } else {
                np = static_cast<size_t>((eob + 7) >> 3);
                memset(d, 0, 128);
                for (int i = 0; i < n; i++) {
                    const int16_t v = static_cast<int16_t>(b[pos[i]]);
                    memcpy(d + 2 * kZigOf.z[pos[i]], &v, 2);
                }
            }
            ix = static_cast<uint32_t>(cur << 4 | np);
            cur += np;
            return 0;
        }
    };
    struct FixedSink {
        JpegCoeffs &o;
        int32_t max_abs[4] = {0, 0, 0, 0};
        std::vector<std::pair<size_t, int32_t>> overflow[4]; // values too wide for the grid
        int put(int ci, size_t blk, int32_t *b, const uint8_t *pos, int n)
        {
            return o.grid[ci].store_sparse_fixed(blk, b, pos, n, max_abs[ci], overflow[ci]) ? 0 : ZPX_E_PANIC;
        }
    };
    // Bit readers of a first scan's block (first_block).  MemberBits is the
    // Decoder's own: huffman / receive_extend / bits above, the reference's
    // lazy byte-at-a-time reads (ensureNBits / readByteStuffedByte).
    // FastBits decodes from a 64-bit look-ahead of the stream instead -- the
    // member's buffered bits, then plain bytes up to the next 0xFF -- and
    // tracks what the member would have read: C bits consumed and H, the
    // furthest bit any operation needed (ensure(n) = C + n); the member's
    // reads being lazy and whole bytes, it would hold (H - bn0) / 8 bytes
    // more, rounded up, so sync() rebuilds (ba_, bn_, bm_, pos_, unread_)
    // exactly.  An operation whose bits reach a 0xFF byte (a stuffed byte or
    // a marker), or a code the member would finish bit by bit, syncs, runs
    // the member function and reloads, so its outcome -- value or error -- is
    // the member's.  Used while kFastSlack input bytes remain (no read
    // reaches the end); the pieces path keeps one for a whole MCU
    // (mcu_pieces).  (The members, updated through `this` beside the int32
    // block stores, were reloaded and stored around every symbol; the
    // byte-at-a-time copy of them branched on every byte.)
    static constexpr size_t kFastSlack = 2048; // > any block's entropy-coded bytes (64 x 27 bits, stuffed x2)
    struct MemberBits {
        Decoder &d;
        static constexpr bool kAcFast = false;
        uint32_t peek_ac(const Huff &) { return 0; }
        void take_ac(uint32_t) {}
        int huffman(const Huff &h, uint8_t &out) { return d.huffman(h, out); }
        int receive_extend(uint8_t t, int32_t &out) { return d.receive_extend(t, out); }
        int bits(int32_t n, uint32_t &out) { return d.bits(n, out); }
        int bit(bool &out) { return d.bit(out); }
    };
    struct FastBits {
        Decoder &d;
        const uint8_t *src;
        uint64_t acc = 0;
        int avail = 0;
        size_t q = 0;
        uint32_t ba0 = 0;
        int32_t bn0 = 0, C = 0, H = 0;
        size_t pos0 = 0;
        size_t unread0 = 0;
        explicit FastBits(Decoder &dd) : d(dd), src(dd.src_) { load(); }
        static constexpr bool kAcFast = true;
        // the combined AC entry (Huff::ac) of the next bits, 0 when they are
        // not all buffered (a marker or the input's end ahead: the symbol
        // path then reads them the reference's way)
        __attribute__((always_inline)) uint32_t peek_ac(const Huff &h)
        {
            if (avail < kAcFastBits) refill();
            return avail >= kAcFastBits ? h.ac[acc >> (64 - kAcFastBits)] : 0u;
        }
        // consume it: the reference's huffman ensures 8 bits, then
        // receiveExtend its magnitude bits (need(8), need(size))
        __attribute__((always_inline)) void take_ac(uint32_t e)
        {
            const int tot = static_cast<int>(e & 15);
            H = std::max(H, C + std::max(8, tot));
            consume(tot);
        }
        __attribute__((always_inline)) void sync()
        {
            const int32_t k = H > bn0 ? (H - bn0 + 7) >> 3 : 0;
            uint32_t ba = ba0;
            if (k >= 4) {
                ba = uint32_t(src[pos0 + k - 4]) << 24 | uint32_t(src[pos0 + k - 3]) << 16 |
                     uint32_t(src[pos0 + k - 2]) << 8 | src[pos0 + k - 1];
            } else {
                for (int32_t i = 0; i < k; i++) ba = (ba << 8) | src[pos0 + static_cast<size_t>(i)];
            }
            d.ba_ = ba;
            d.bn_ = bn0 + 8 * k - C;
            d.bm_ = d.bn_ > 0 ? 1u << (d.bn_ - 1) : 0u;
            d.pos_ = pos0 + static_cast<size_t>(k);
            d.unread_ = k > 0 ? 1 : unread0;
        }
        __attribute__((always_inline)) void load()
        {
            ba0 = d.ba_;
            bn0 = d.bn_;
            pos0 = d.pos_;
            unread0 = d.unread_;
            C = H = 0;
            acc = bn0 > 0 ? uint64_t(ba0 & (bn0 >= 32 ? ~0u : (1u << bn0) - 1)) << (64 - bn0) : 0;
            avail = bn0;
            q = pos0;
            refill();
        }
        __attribute__((always_inline)) void refill()
        {
            uint64_t le;
            memcpy(&le, src + q, 8);
            const uint64_t x = ~le;
            const uint64_t z = (x - 0x0101010101010101ull) & ~x & 0x8080808080808080ull;
            const int plain = z ? __builtin_ctzll(z) >> 3 : 8;
            const int nb = std::min((64 - avail) >> 3, plain);
            if (nb > 0) {
                acc |= (__builtin_bswap64(le) >> (64 - 8 * nb)) << (64 - avail - 8 * nb);
                avail += 8 * nb;
                q += static_cast<size_t>(nb);
            }
        }
        __attribute__((always_inline)) bool need(int n)
        {
            if (avail < n) refill();
            if (avail < n) return false;
            H = std::max(H, C + n);
            return true;
        }
        __attribute__((always_inline)) void consume(int n)
        {
            C += n;
            acc = n < 64 ? acc << n : 0;
            avail -= n;
        }
        __attribute__((always_inline)) int slow_huffman(const Huff &h, uint8_t &out)
        {
            sync();
            const int e = d.huffman(h, out);
            load();
            return e;
        }
        __attribute__((always_inline)) int huffman(const Huff &h, uint8_t &out)
        {
            if (h.num_codes == 0 || !need(8)) return slow_huffman(h, out);
            const uint16_t lv = h.lut[acc >> 56];
            if (lv != 0) {
                consume(static_cast<int>(lv & 0xff) - 1);
                out = static_cast<uint8_t>(lv >> 8);
                return 0;
            }
            const int32_t k = (H - bn0 + 7) >> 3;
            const int held = bn0 + 8 * k - C;
            if (avail < 16) refill();
            for (int i = 8; i < 16 && i < held && i < avail; i++) {
                const int32_t code = static_cast<int32_t>(acc >> (63 - i));
                if (code <= h.max_codes[i]) {
                    const int32_t idx = h.vals_indices[i] + code - h.min_codes[i];
                    if (idx < 0 || idx > 255) break;
                    consume(i + 1);
                    out = h.vals[idx];
                    return 0;
                }
            }
            return slow_huffman(h, out);
        }
        __attribute__((always_inline)) int receive_extend(uint8_t t, int32_t &out)
        {
            if (!need(t)) {
                sync();
                const int e = d.receive_extend(t, out);
                load();
                return e;
            }
            const int32_t thr = int32_t(1) << t;
            int32_t v = t ? static_cast<int32_t>(acc >> (64 - t)) : 0;
            consume(t);
            v += ((v - (thr >> 1)) >> 31) & (static_cast<int32_t>(0xffffffffu << t) + 1);
            out = v;
            return 0;
        }
        __attribute__((always_inline)) int bit(bool &out)
        {
            if (!need(1)) {
                sync();
                const int e = d.bit(out);
                load();
                return e;
            }
            out = (acc >> 63) != 0;
            consume(1);
            return 0;
        }
        __attribute__((always_inline)) int bits(int32_t n, uint32_t &out)
        {
            if (n > 32 || !need(n)) {
                sync();
                const int e = d.bits(n, out);
                load();
                return e;
            }
            out = n ? static_cast<uint32_t>(acc >> (64 - n)) : 0u;
            consume(n);
            return 0;
        }
    };
    template <class R>
    __attribute__((always_inline)) int first_block(R &r, const Scan &sc, const Huff &hdc, const Huff &hac,
                                                   int32_t &dcv, int32_t *b, uint8_t *nzpos, int &nnz);
    // first_block + PieceSink::put in one pass (the batch path's baseline
    // scans): the block decodes straight into zig-zag order -- the pieces'
    // own -- in zz (zero on entry and on return), and its pieces are written
    // from there, with no natural-order block or position list in between
    template <class R>
    __attribute__((always_inline)) int first_block_pieces(R &r, const Scan &sc, const Huff &hdc, const Huff &hac,
                                                          int32_t &dcv, JpegPieces &p, int ci, size_t blk, int yy,
                                                          int32_t *zz);
    template <class Sink>
    int mcu(const Scan &sc, int32_t my, int32_t mx, int32_t &block_count, int32_t *dc, int32_t *b, uint8_t *nzpos,
            Sink &sink);
    // an interleaved baseline MCU into pieces (first_block_pieces per block)
    // on one register reader for the whole MCU
    int mcu_pieces(const Scan &sc, int32_t my, int32_t mx, int32_t *dc, int32_t *zz, JpegPieces &p);
    template <class R>
    __attribute__((always_inline)) int mcu_pieces_with(R &r, const Scan &sc, int32_t my, int32_t mx, int32_t *dc,
                                                       int32_t *zz, JpegPieces &p);
    // one block of a progressive scan, touching only the scan's band
    template <class R>
    int prog_block(R &r, const Scan &sc, int ci, size_t blk, const Huff &hdc, const Huff &hac, int32_t *dc);
    // (out of line: inlined into mcu() beside the baseline path's register
    // reader, the progressive decode ran 10-20 % slower; tools/prog_ab.py)
    __attribute__((noinline)) int prog_block_member(const Scan &sc, int ci, size_t blk, const Huff &hdc, const Huff &hac,
                                                    int32_t *dc)
    {
        MemberBits mb{*this};
        return prog_block(mb, sc, ci, blk, hdc, hac, dc);
    }
    // coefficient z (zig-zag order) of block blk of component ci: set also
    // marks it nonzero in the block's mask (a refinement then visits only
    // the nonzero coefficients of its band; a coefficient never returns to
    // zero: refinements only add to its magnitude or set new ones)
    int prog_set(int ci, size_t blk, int z, int32_t v)
    {
        const int i = kUnzig[z];
        if (int16_t *g = fixed16_[ci]) { // parallel scan: int16 grid, no widening
            const int32_t a = v < 0 ? (v == INT32_MIN ? INT32_MAX : -v) : v;
            if (a > 32767) return kParallelAbort;
            job_max_[ci] = a > job_max_[ci] ? a : job_max_[ci];
            if (z == 0) { // DC apart from the block (the DC scans run beside the AC scans)
                dc16_[ci][blk] = static_cast<int16_t>(v);
                return 0;
            }
            g[blk * 64 + static_cast<size_t>(i)] = static_cast<int16_t>(v);
            // (no two AC scans of one component run at once: run_deferred_scans)
            if (v != 0) (*nz_[ci])[blk] |= uint64_t(1) << z;
            return 0;
        }
        if (v != 0 && z != 0) (*nz_[ci])[blk] |= uint64_t(1) << z;
        return o_.grid[ci].set(blk, i, v) ? 0 : ZPX_E_OUT_OF_MEMORY;
    }
    int32_t prog_get(int ci, size_t blk, int z) const
    {
        if (const int16_t *g = fixed16_[ci])
            return z == 0 ? dc16_[ci][blk] : g[blk * 64 + static_cast<size_t>(kUnzig[z])];
        return o_.grid[ci].get(blk, kUnzig[z]);
    }
    uint64_t prog_mask(int ci, size_t blk) const { return (*nz_[ci])[blk]; }
    // refine :1459-1518 / refineNonZeroes :1522-1549 of an AC band on the
    // grid itself, through the nonzero masks
    template <class R>
    int prog_refine_ac(R &r, int ci, size_t blk, const Huff &h, int32_t zs, int32_t ze, int32_t delta);
    template <class R>
    int prog_refine_nonzero(R &r, int ci, size_t blk, uint64_t mask, int32_t zig, int32_t ze, int32_t nz, int32_t delta,
                            int32_t &zout);
    // the MCU loop of one scan, restart markers included (processSos
    // :1298-1455), from the scan's first entropy-coded byte
    int scan_loop(const Scan &sc, bool pieces);
    int restart_parallel(const Scan &sc, bool &done);
    friend int run_deferred_scans(std::vector<std::unique_ptr<Decoder>> &jobs, JpegCoeffs &o, int threads);
    // the run() loop head from byte p: the position after the next marker
    // byte and that marker (false: the input ends first)
    bool next_marker(size_t p, size_t &after, uint8_t &marker) const;
    int sof(int32_t n);
    int dqt(int32_t n);
    int dht(int32_t n);
    int sos(int32_t n);
    int refine(int32_t *b, const Huff &h, int32_t zs, int32_t ze, int32_t delta);
    int refine_nonzero(int32_t *b, int32_t zig, int32_t ze, int32_t nz, int32_t delta,
                       int32_t &zout);
    int find_rst(uint8_t expected);
    void snapshot_quant(int c);

    const uint8_t *src_;
    size_t len_, pos_ = 0, unread_ = 0;
    uint32_t ba_ = 0, bm_ = 0;
    int32_t bn_ = 0;
    JpegCoeffs &o_;
    uint16_t restart_interval_ = 0;
    uint16_t eob_run_ = 0;
    Huff huff_[2][4];
    int32_t quant_[4][64] = {}; // zig-zag order, as the reference keeps it
    uint8_t tmp_[128] = {};
    bool seen_sos_ = false;
    bool config_only_ = false;
    bool interleaved_[4] = {}, noninterleaved_[4] = {};
    int threads_ = 1; // restart-interval-parallel Huffman (baseline scans with DRI)
    bool sparse_ok_ = false; // emit JpegPieces for a single interleaved baseline scan
  public:
    // Progressive scans decoded in parallel (run_deferred_scans): the first
    // pass walks the markers and, at each SOS, keeps a copy of the decoder --
    // Huffman tables, restart interval and the scan as they are there --
    // then skips the scan's entropy-coded bytes to the next marker.
    std::vector<std::unique_ptr<Decoder>> *deferred_ = nullptr;
  private:
    Scan job_scan_;
    size_t job_start_ = 0, job_skip_ = 0; // the scan's first byte; where the first pass resumed
    int16_t *fixed16_[4] = {nullptr, nullptr, nullptr, nullptr};
    int16_t *dc16_[4] = {nullptr, nullptr, nullptr, nullptr}; // parallel scans: the DC coefficients, per block
    std::shared_ptr<std::vector<uint64_t>> nz_[4]; // progressive: per block, its nonzero coefficients (zig-zag bits)
    int32_t job_max_[4] = {0, 0, 0, 0};
    static constexpr int kParallelAbort = (1 << 20) + 1; // internal: a value past int16 in a parallel scan
};

int Decoder::sof(int32_t n)
{ // processSof :490-618
    if (o_.n_comp != 0) return ZPX_E_MULTIPLE_SOF_MARKERS;
    if (n == 9) o_.n_comp = 1;
    else if (n == 15) o_.n_comp = 3;
    else if (n == 18) o_.n_comp = 4;
    else return ZPX_E_NUMBER_COMPONENTS;
    ZTRY(full(tmp_, static_cast<size_t>(n)));
    if (tmp_[0] != 8) return ZPX_E_PRECISION;
    o_.height = (uint32_t(tmp_[1]) << 8) + tmp_[2];
    o_.width = (uint32_t(tmp_[3]) << 8) + tmp_[4];
    if (tmp_[5] != o_.n_comp) return ZPX_E_SOF_WRONG_LENGTH;
    JpegComponent *c = o_.comp;
    for (int i = 0; i < o_.n_comp; i++) {
        c[i].id = tmp_[6 + 3 * i];
        for (int j = 0; j < i; j++)
            if (c[i].id == c[j].id) return ZPX_E_REPEATED_COMPONENT_IDENTIFIER;
        c[i].tq = tmp_[8 + 3 * i];
        if (c[i].tq > 3) return ZPX_E_BAD_TQ_VALUE;
        const uint8_t hv = tmp_[7 + 3 * i];
        int32_t h = hv >> 4, v = hv & 0x0f;
        if (h < 1 || h > 4 || v < 1 || v > 4 || h == 3 || v == 3)
            return ZPX_E_LUMA_CHROMA_SUB_SAMPLING_RATIO;
        if (o_.n_comp == 1) {
            h = v = 1; // non-interleaved by definition (A.2)
        } else if (o_.n_comp == 3) {
            bool bad = (i == 0 && v == 4) || (i == 1 && (c[0].h % h != 0 || c[0].v % v != 0)) ||
                       (i == 2 && (c[1].h != h || c[1].v != v));
            if (bad) return ZPX_E_LUMA_CHROMA_SUB_SAMPLING_RATIO;
        } else {
            bool bad = (i == 0 && hv != 0x11 && hv != 0x22) || ((i == 1 || i == 2) && hv != 0x11) ||
                       (i == 3 && (c[0].h != h || c[0].v != v));
            if (bad) return ZPX_E_LUMA_CHROMA_SUB_SAMPLING_RATIO;
        }
        c[i].h = h;
        c[i].v = v;
    }
    return 0;
}

int Decoder::dqt(int32_t n)
{ // processDqt :629-666
    while (n > 0) {
        n--;
        uint8_t qi;
        ZTRY(byte(qi));
        const uint8_t tq = qi & 0x0f;
        if (tq > 3) return ZPX_E_BAD_TQ_VALUE;
        const int pq = qi >> 4;
        if (pq > 1) return ZPX_E_BAD_PQ_VALUE;
        const int32_t need = pq == 0 ? 64 : 128;
        if (n < need) break;
        n -= need;
        ZTRY(full(tmp_, static_cast<size_t>(need)));
        for (int i = 0; i < 64; i++)
            quant_[tq][i] = pq == 0 ? tmp_[i] : ((int32_t(tmp_[2 * i]) << 8) | tmp_[2 * i + 1]);
    }
    return n != 0 ? ZPX_E_DQT_WRONG_LENGTH : 0;
}

int Decoder::dht(int32_t n)
{ // processDht :1026-1111
    while (n > 0) {
        if (n < 17) return ZPX_E_DHT_WRONG_LENGTH;
        ZTRY(full(tmp_, 17));
        const uint8_t tc = tmp_[0] >> 4, th = tmp_[0] & 0x0f;
        if (tc > 1) return ZPX_E_BAD_TC_VALUE;
        if (th > 3 || (o_.baseline && th > 1)) return ZPX_E_BAD_TH_VALUE;
        Huff &h = huff_[tc][th];
        int32_t count[16];
        h.num_codes = 0;
        for (int i = 0; i < 16; i++) h.num_codes += (count[i] = tmp_[1 + i]);
        if (h.num_codes == 0) return ZPX_E_HUFF_ZERO_LENGTH;
        if (h.num_codes > 256) return ZPX_E_HUFF_TOO_LONG;
        n -= h.num_codes + 17;
        if (n < 0) return ZPX_E_DHT_WRONG_LENGTH;
        ZTRY(full(h.vals, static_cast<size_t>(h.num_codes)));
        memset(h.lut, 0, sizeof(h.lut));
        uint32_t code = 0;
        int vi = 0;
        for (int len = 1; len <= 8; len++) {
            code <<= 1;
            for (int j = 0; j < count[len - 1]; j++, code++, vi++) {
                const uint32_t base = code << (8 - len);
                const uint16_t lv = static_cast<uint16_t>((h.vals[vi] << 8) | (len + 1));
                for (uint32_t k = 0; k < (1u << (8 - len)); k++) {
                    if ((base | k) > 255) return ZPX_E_PANIC; // over-full code set
                    h.lut[base | k] = lv;
                }
            }
        }
        // the combined AC table (Huff::ac): codes of <= 8 bits, their
        // symbol's magnitude bits with them when both fit kAcFastBits
        memset(h.ac, 0, sizeof(h.ac));
        if (tc == 0) { // DC: the difference's size t and its t bits (run 0, never kAcEob)
            uint32_t c2 = 0;
            int v2 = 0;
            for (int len = 1; len <= 8; len++) {
                c2 <<= 1;
                for (int j = 0; j < count[len - 1]; j++, c2++, v2++) {
                    const int size = h.vals[v2];
                    const int tot = len + size;
                    if (size > 16 || tot > kAcFastBits) continue; // (t > 16: ExcessiveDCComponent, the symbol path)
                    for (uint32_t x = 0; x < (1u << size); x++) {
                        int32_t v = static_cast<int32_t>(x);
                        if (size > 0 && v < (int32_t(1) << (size - 1))) v += static_cast<int32_t>(0xffffffffu << size) + 1;
                        const uint32_t e = static_cast<uint32_t>(tot) | static_cast<uint32_t>(v) << 16;
                        const uint32_t base = ((c2 << size) | x) << (kAcFastBits - tot);
                        for (uint32_t k = 0; k < (1u << (kAcFastBits - tot)); k++)
                            if ((base | k) < (1u << kAcFastBits)) h.ac[base | k] = e;
                    }
                }
            }
        } else {
            uint32_t c2 = 0;
            int v2 = 0;
            for (int len = 1; len <= 8; len++) {
                c2 <<= 1;
                for (int j = 0; j < count[len - 1]; j++, c2++, v2++) {
                    const uint8_t sym = h.vals[v2];
                    const int size = sym & 15, run = sym >> 4;
                    if (size == 0 && run != 0) continue; // ZRL, EOBn: the symbol path
                    const int tot = len + size;
                    if (tot > kAcFastBits) continue;
                    for (uint32_t x = 0; x < (1u << size); x++) {
                        uint32_t e = static_cast<uint32_t>(tot) | static_cast<uint32_t>(run) << 8;
                        if (size == 0) {
                            e |= kAcEob;
                        } else { // receiveExtend (decoder.zig:975-991) of the magnitude bits x
                            int32_t v = static_cast<int32_t>(x);
                            if (v < (int32_t(1) << (size - 1))) v += static_cast<int32_t>(0xffffffffu << size) + 1;
                            e |= static_cast<uint32_t>(v) << 16;
                        }
                        const uint32_t base = ((c2 << size) | x) << (kAcFastBits - tot);
                        for (uint32_t k = 0; k < (1u << (kAcFastBits - tot)); k++)
                            if ((base | k) < (1u << kAcFastBits)) h.ac[base | k] = e;
                    }
                }
            }
        }
        int32_t cb = 0, idx = 0;
        for (int i = 0; i < 16; i++) {
            if (count[i] == 0) {
                h.min_codes[i] = h.max_codes[i] = h.vals_indices[i] = -1;
            } else {
                h.min_codes[i] = cb;
                h.max_codes[i] = cb + count[i] - 1;
                h.vals_indices[i] = idx;
                cb += count[i];
                idx += count[i];
            }
            cb <<= 1;
        }
    }
    return 0;
}

int Decoder::refine_nonzero(int32_t *b, int32_t zig, int32_t ze, int32_t nz, int32_t delta,
                            int32_t &zout)
{ // refineNonZeroes :1522-1549
    for (; zig <= ze; zig++) {
        const int idx = kUnzig[zig];
        if (b[idx] == 0) {
            if (nz == 0) break;
            nz--;
            continue;
        }
        bool set;
        ZTRY(bit(set));
        if (!set) continue;
        b[idx] += b[idx] >= 0 ? delta : -delta;
    }
    zout = zig;
    return 0;
}

int Decoder::refine(int32_t *b, const Huff &h, int32_t zs, int32_t ze, int32_t delta)
{ // refine :1459-1518
    if (zs == 0) {
        if (ze != 0) return ZPX_E_PANIC;
        bool set;
        ZTRY(bit(set));
        if (set) b[0] |= delta;
        return 0;
    }
    int32_t zig = zs;
    if (eob_run_ == 0) {
        for (; zig <= ze; zig++) {
            int32_t z = 0;
            uint8_t value;
            ZTRY(huffman(h, value));
            const uint8_t v0 = value >> 4, v1 = value & 0x0f;
            if (v1 == 0) {
                if (v0 != 0x0f) {
                    eob_run_ = static_cast<uint16_t>(1u << v0);
                    if (v0 != 0) {
                        uint32_t x;
                        ZTRY(bits(v0, x));
                        eob_run_ |= static_cast<uint16_t>(x);
                    }
                    break;
                }
            } else if (v1 == 1) {
                bool positive;
                ZTRY(bit(positive));
                z = positive ? delta : -delta;
            } else {
                return ZPX_E_UNEXPECTED_HUFFMAN_CODE;
            }
            ZTRY(refine_nonzero(b, zig, ze, v0, delta, zig));
            if (zig > ze) return ZPX_E_TOO_MANY_COEFFICIENTS;
            if (z != 0) b[kUnzig[zig]] = z;
        }
    }
    if (eob_run_ > 0) {
        eob_run_--;
        int32_t ignored;
        ZTRY(refine_nonzero(b, zig, ze, -1, delta, ignored));
    }
    return 0;
}

int Decoder::find_rst(uint8_t expected)
{ // findRst :1671-1705
    for (;;) {
        size_t i = 0;
        if (tmp_[0] == 0xff) {
            if (tmp_[1] == expected) return 0;
            if (tmp_[1] == 0xff) i = 1;
            else if (tmp_[1] != 0x00) return ZPX_E_BAD_RST_MARKER;
        } else if (tmp_[1] == 0xff) {
            tmp_[0] = 0xff;
            i = 1;
        }
        ZTRY(full(tmp_ + i, 2 - i));
    }
}

void Decoder::snapshot_quant(int c)
{
    const int32_t *q = quant_[o_.comp[c].tq];
    int32_t m = 0;
    for (int z = 0; z < 64; z++) {
        o_.qt_natural[c][kUnzig[z]] = q[z];
        int32_t a = q[z] < 0 ? -q[z] : q[z];
        m = a > m ? a : m;
    }
    o_.max_q[c] = m;
}

int Decoder::sos(int32_t n)
{ // processSos :1148-1455
    if (o_.n_comp == 0) return ZPX_E_MISSING_SOS_MARKER;
    if (n < 6 || 4 + 2 * o_.n_comp < n || n % 2 != 0) return ZPX_E_SOS_WRONG_LENGTH;
    ZTRY(full(tmp_, static_cast<size_t>(n)));
    const int ns = tmp_[0];
    if (n != 4 + 2 * ns) return ZPX_E_SOS_WRONG_LENGTH;
    struct {
        uint8_t id = 0, td = 0, ta = 0;
    } scan[4];
    int32_t total_hv = 0;
    for (int i = 0; i < ns; i++) {
        const uint8_t sel = tmp_[1 + 2 * i];
        int ci = -1;
        for (int j = 0; j < o_.n_comp; j++)
            if (o_.comp[j].id == sel) {
                ci = j;
                break;
            }
        if (ci < 0) return ZPX_E_UNKNOWN_COMPONENT_SELECTOR;
        scan[i].id = static_cast<uint8_t>(ci);
        for (int j = 0; j < i; j++)
            if (scan[j].id == scan[i].id) return ZPX_E_REPEATED_COMPONENT_IDENTIFIER;
        total_hv += o_.comp[ci].h * o_.comp[ci].v;
        scan[i].td = tmp_[2 + 2 * i] >> 4;
        if (scan[i].td > 3 || (o_.baseline && scan[i].td > 1)) return ZPX_E_BAD_TD_VALUE;
        scan[i].ta = tmp_[2 + 2 * i] & 0x0f;
        if (scan[i].ta > 3 || (o_.baseline && scan[i].ta > 1)) return ZPX_E_BAD_TA_VALUE;
    }
    if (o_.n_comp > 1 && total_hv > 10) return ZPX_E_SAMPLING_FACTORS_TOO_LARGE;

    int32_t zs = 0, ze = 63;
    uint32_t ah = 0, al = 0;
    if (o_.progressive) {
        zs = tmp_[1 + 2 * ns];
        ze = tmp_[2 + 2 * ns];
        ah = tmp_[3 + 2 * ns] >> 4;
        al = tmp_[3 + 2 * ns] & 0x0f;
        if ((zs == 0 && ze != 0) || zs > ze || ze >= 64) return ZPX_E_BAD_SPECTRAL_SELECTION;
        if (zs != 0 && ns != 1) return ZPX_E_PROGRESSIVE_AC_COEFFICIENTS_FOR_MORE_THAN_ONE_COMPONENT;
        if (ah != 0 && ah != al + 1) return ZPX_E_BAD_SUCCESSIVE_APPROXIMATION;
    }

    const int32_t h0 = o_.comp[0].h, v0 = o_.comp[0].v;
    const int32_t mxx = (static_cast<int32_t>(o_.width) + 8 * h0 - 1) / (8 * h0);
    const int32_t myy = (static_cast<int32_t>(o_.height) + 8 * v0 - 1) / (8 * v0);
    o_.mxx = mxx;
    o_.myy = myy;
    if (o_.pieces.valid) return kSparseAbort; // a second scan after a pieces scan: redo with grids
    bool pieces = sparse_ok_ && !seen_sos_ && !o_.progressive && ns == 3 && o_.n_comp == 3 &&
                   !(threads_ > 1 && restart_interval_ > 0);
    seen_sos_ = true;
    size_t nblocks = 0;
    for (int c = 0; c < o_.n_comp; c++) nblocks += size_t(mxx) * size_t(myy) * size_t(o_.comp[c].h * o_.comp[c].v);
    // int16 worst case: 8 pieces a block, plus the zero piece; the index
    // holds a piece number in 28 bits
    const size_t cap = 1 + 8 * nblocks;
    if (cap >= (size_t(1) << 28)) pieces = false;
    if (pieces) {
        JpegPieces &pc = o_.pieces;
        // (+8 pieces: a block's writes clear its whole dense extent)
        if (!pc.index.alloc(nblocks * sizeof(uint32_t), true) || !pc.data.alloc((cap + 8) * 16, false))
            return ZPX_E_OUT_OF_MEMORY;
        size_t first = 0, sb = 1;
        pc.nstreams = 0;
        for (int c = 0; c < o_.n_comp; c++) {
            pc.first[c] = first;
            pc.blocks[c] = size_t(mxx) * size_t(myy) * size_t(o_.comp[c].h * o_.comp[c].v);
            first += pc.blocks[c];
            // streams of the component: its block rows mod v (JpegPieces),
            // each with room for 8 pieces (int16) per block
            pc.s0[c] = pc.nstreams;
            pc.v[c] = o_.comp[c].v;
            pc.gw[c] = size_t(mxx) * size_t(o_.comp[c].h);
            for (int yy = 0; yy < pc.v[c]; yy++) {
                pc.base[pc.nstreams] = pc.next[pc.nstreams] = sb;
                sb += 8 * (pc.blocks[c] / size_t(pc.v[c]));
                pc.nstreams++;
            }
        }
        memset(pc.data.ptr, 0, 16); // piece 0
        pc.cap = cap;
        pc.npieces = 1;
        pc.bits = 8;
        pc.valid = true;
    }
    // Grids: like progressive_coefficients, allocated for scan[i].id over
    // i < n_comp (:1269-1282; slots past ns read component 0).  A baseline
    // scan interleaving several components writes every block of every MCU,
    // so its grids need no clearing.
    const bool full_cover = !o_.progressive && ns > 1;
    for (int i = 0; i < o_.n_comp && !pieces; i++) {
        const int ci = scan[i].id;
        if (!o_.has_grid[ci]) {
            const size_t nb = size_t(mxx) * size_t(myy) * size_t(o_.comp[ci].h * o_.comp[ci].v);
            bool in_scan = false;
            for (int k = 0; k < ns; k++) in_scan |= scan[k].id == ci;
            const bool defer = deferred_ != nullptr && o_.progressive;
            if (!o_.grid[ci].init(nb, defer || !(full_cover && in_scan), defer ? 16 : 8)) return ZPX_E_OUT_OF_MEMORY;
            if (o_.progressive) nz_[ci] = std::make_shared<std::vector<uint64_t>>(nb, 0);
            o_.has_grid[ci] = true;
        }
    }
    for (int k = 0; k < ns; k++) (ns != 1 ? interleaved_ : noninterleaved_)[scan[k].id] = true;

    Scan sc;
    sc.ns = ns;
    for (int k = 0; k < ns; k++) {
        sc.c[k].id = scan[k].id;
        sc.c[k].td = scan[k].td;
        sc.c[k].ta = scan[k].ta;
    }
    sc.zs = zs;
    sc.ze = ze;
    sc.ah = ah;
    sc.al = al;
    sc.prog = o_.progressive;
    sc.mxx = mxx;
    sc.myy = myy;
    ba_ = bm_ = 0;
    bn_ = 0;
    if (deferred_ != nullptr && o_.progressive) {
        // first pass of the parallel progressive decode: keep this scan's
        // decoder, skip its entropy-coded bytes (to the first 0xFF that is
        // not a stuffed byte or a restart marker)
        std::unique_ptr<Decoder> job(new Decoder(*this));
        job->deferred_ = nullptr;
        job->job_scan_ = sc;
        job->job_start_ = pos_;
        size_t q = pos_;
        while (q + 1 < len_ && !(src_[q] == 0xff && src_[q + 1] != 0x00 && (src_[q + 1] < 0xd0 || src_[q + 1] > 0xd7)))
            q++;
        if (q + 1 >= len_) q = len_;
        job->job_skip_ = q;
        deferred_->push_back(std::move(job));
        pos_ = q;
        unread_ = 0;
        return 0;
    }
    ZTRY(scan_loop(sc, pieces));
    // baseline reconstructs during the scan with the table current now
    if (!o_.progressive)
        for (int k = 0; k < ns; k++) snapshot_quant(scan[k].id);
    return 0;
}

int Decoder::scan_loop(const Scan &sc, bool pieces)
{
    const int32_t mxx = sc.mxx, myy = sc.myy;
    bool done = false;
    if (!pieces) ZTRY(restart_parallel(sc, done));
    if (!done) {
        int32_t mcu_i = 0, block_count = 0;
        uint8_t expected_rst = 0xd0;
        int32_t dc[4] = {0, 0, 0, 0};
        int32_t b[64];
        uint8_t nzpos[64];
        memset(b, 0, sizeof(b));
        SerialSink serial{o_};
        PieceSink rec{o_.pieces};
        for (int32_t my = 0; my < myy; my++) {
            for (int32_t mx = 0; mx < mxx; mx++) {
                ZTRY(pieces ? mcu(sc, my, mx, block_count, dc, b, nzpos, rec)
                             : mcu(sc, my, mx, block_count, dc, b, nzpos, serial));
                mcu_i++;
                if (restart_interval_ > 0 && mcu_i % restart_interval_ == 0 && mcu_i < mxx * myy) {
                    ZTRY(full(tmp_, 2));
                    if (tmp_[0] != 0xff || tmp_[1] != expected_rst) ZTRY(find_rst(expected_rst));
                    expected_rst = expected_rst == 0xd7 ? 0xd0 : static_cast<uint8_t>(expected_rst + 1);
                    ba_ = bm_ = 0;
                    bn_ = 0;
                    dc[0] = dc[1] = dc[2] = dc[3] = 0;
                    eob_run_ = 0;
                }
            }
        }
    }
    return 0;
}

// One MCU of a scan: its blocks' Huffman / refinement decode and store (the
// body of processSos's MCU loop, :1300-1431).  b is all-zero on entry for
// baseline scans; the positions a block writes are recorded and cleared
// after its store.
// One block of a first scan (processSos :1300-1345: the DC difference, then
// the AC run/size loop with its end-of-band run), over a bit reader R: the
// Decoder's own (MemberBits) or register copies of it (FastBits).
template <class R>
int Decoder::first_block(R &r, const Scan &sc, const Huff &hdc, const Huff &hac, int32_t &dcv, int32_t *b,
                         uint8_t *nzpos, int &nnz)
{
    const int32_t ze = sc.ze, al = sc.al; // (locals: the byte stores below may alias sc)
    int32_t zig = sc.zs;
    if (zig == 0) {
        zig++;
        int32_t delta;
        uint32_t e = 0;
        if constexpr (R::kAcFast) e = r.peek_ac(hdc); // (the DC difference in one lookup)
        if (e & 15) {
            r.take_ac(e);
            delta = static_cast<int32_t>(e) >> 16;
        } else {
            uint8_t t;
            ZTRY(r.huffman(hdc, t));
            if (t > 16) return ZPX_E_EXCESSIVE_DC_COMPONENT;
            ZTRY(r.receive_extend(t, delta));
        }
        dcv += delta;
        b[0] = dcv << al;
        nzpos[nnz++] = 0;
    }
    if (zig <= ze && eob_run_ > 0) {
        eob_run_--;
        return 0;
    }
    for (; zig <= ze; zig++) {
        if constexpr (R::kAcFast) { // one lookup: code and magnitude bits (Huff::ac)
            const uint32_t e = r.peek_ac(hac);
            if (e & kAcEob) {
                r.take_ac(e);
                eob_run_ = 0; // (1 << 0) - 1
                break;
            }
            const int32_t run = static_cast<int32_t>((e >> 8) & 15);
            if ((e & 15) != 0 && zig + run <= ze) {
                r.take_ac(e);
                zig += run;
                b[kUnzig[zig]] = (static_cast<int32_t>(e) >> 16) << al;
                nzpos[nnz++] = kUnzig[zig];
                continue;
            }
        }
        uint8_t value;
        ZTRY(r.huffman(hac, value));
        const uint8_t v0r = value >> 4, v1 = value & 0x0f;
        if (v1 != 0) {
            zig += v0r;
            if (zig > ze) break;
            int32_t ac;
            ZTRY(r.receive_extend(v1, ac));
            b[kUnzig[zig]] = ac << al;
            nzpos[nnz++] = kUnzig[zig];
        } else {
            if (v0r != 0x0f) {
                eob_run_ = static_cast<uint16_t>(1u << v0r);
                if (v0r != 0) {
                    uint32_t x;
                    ZTRY(r.bits(v0r, x));
                    eob_run_ |= static_cast<uint16_t>(x);
                }
                eob_run_--;
                break;
            }
            zig += 0x0f;
        }
    }
    return 0;
}

template <class R>
int Decoder::first_block_pieces(R &r, const Scan &sc, const Huff &hdc, const Huff &hac, int32_t &dcv, JpegPieces &p,
                                int ci, size_t blk, int yy, int32_t *zz)
{
    const int32_t ze = sc.ze, al = sc.al;
    int32_t zig = sc.zs;
    int last = -1; // the last coefficient written, zig-zag order
    uint32_t m = 0; // the largest magnitude (INT32_MIN's: 2^31)
    auto mag = [](int32_t v) { return v < 0 ? 0u - static_cast<uint32_t>(v) : static_cast<uint32_t>(v); };
    if (zig == 0) {
        zig++;
        int32_t delta;
        uint32_t e = 0;
        if constexpr (R::kAcFast) e = r.peek_ac(hdc); // (the DC difference in one lookup)
        if (e & 15) {
            r.take_ac(e);
            delta = static_cast<int32_t>(e) >> 16;
        } else {
            uint8_t t;
            ZTRY(r.huffman(hdc, t));
            if (t > 16) return ZPX_E_EXCESSIVE_DC_COMPONENT;
            ZTRY(r.receive_extend(t, delta));
        }
        dcv += delta;
        const int32_t v = dcv << al;
        zz[0] = v;
        last = 0;
        m = mag(v);
    }
    if (zig <= ze && eob_run_ > 0) {
        eob_run_--;
    } else {
        for (; zig <= ze; zig++) {
            if constexpr (R::kAcFast) { // one lookup: code and magnitude bits (Huff::ac)
                const uint32_t e = r.peek_ac(hac);
                if (e & kAcEob) {
                    r.take_ac(e);
                    eob_run_ = 0; // (1 << 0) - 1
                    break;
                }
                const int32_t run = static_cast<int32_t>((e >> 8) & 15);
                if ((e & 15) != 0 && zig + run <= ze) {
                    r.take_ac(e);
                    zig += run;
                    const int32_t v = (static_cast<int32_t>(e) >> 16) << al;
                    zz[zig] = v;
                    last = zig;
                    m = std::max(m, mag(v));
                    continue;
                }
            }
            uint8_t value;
            ZTRY(r.huffman(hac, value));
            const uint8_t v0r = value >> 4, v1 = value & 0x0f;
            if (v1 != 0) {
                zig += v0r;
                if (zig > ze) break;
                int32_t ac;
                ZTRY(r.receive_extend(v1, ac));
                const int32_t v = ac << al;
                zz[zig] = v;
                last = zig;
                m = std::max(m, mag(v));
            } else {
                if (v0r != 0x0f) {
                    eob_run_ = static_cast<uint16_t>(1u << v0r);
                    if (v0r != 0) {
                        uint32_t x;
                        ZTRY(r.bits(v0r, x));
                        eob_run_ |= static_cast<uint16_t>(x);
                    }
                    eob_run_--;
                    break;
                }
                zig += 0x0f;
            }
        }
    }
    // PieceSink::put's rules on the zig-zag block (every AC entry is nonzero)
    int rc = 0;
    const uint32_t mm = std::max(m, static_cast<uint32_t>(p.max_abs[ci]));
    if (mm > 32767) {
        rc = kSparseAbort;
    } else {
        p.max_abs[ci] = static_cast<int32_t>(mm);
        if (p.bits == 8 && mm > 127 && !p.widen()) rc = kSparseAbort;
    }
    if (rc == 0) {
        uint32_t &ix = p.index_of(ci)[blk];
        if (last < 0 || (last == 0 && zz[0] == 0)) {
            ix = 0;
        } else {
            const int eob = last + 1;
            size_t &cur = p.next[p.s0[ci] + yy];
            uint8_t *d = static_cast<uint8_t *>(p.data.ptr) + cur * 16;
            size_t np;
            if (p.bits == 8) {
                np = static_cast<size_t>((eob + 15) >> 4);
                for (size_t k = 0; k < np; k++)
                    for (int j = 0; j < 16; j++) reinterpret_cast<int8_t *>(d)[16 * k + j] = static_cast<int8_t>(zz[16 * k + j]);
            } else {
                np = static_cast<size_t>((eob + 7) >> 3);
                for (size_t k = 0; k < np; k++)
                    for (int j = 0; j < 8; j++) {
                        const int16_t v = static_cast<int16_t>(zz[8 * k + j]);
                        memcpy(d + 16 * k + 2 * j, &v, 2);
                    }
            }
            ix = static_cast<uint32_t>(cur << 4 | np);
            cur += np;
        }
    }
    for (int i = 0; i <= last; i++) zz[i] = 0;
    return rc;
}

template <class R>
int Decoder::mcu_pieces_with(R &r, const Scan &sc, int32_t my, int32_t mx, int32_t *dc, int32_t *zz, JpegPieces &p)
{
    const int32_t mxx = sc.mxx;
    for (int k = 0; k < sc.ns; k++) {
        const int ci = sc.c[k].id;
        const int32_t hi = o_.comp[ci].h, vi = o_.comp[ci].v;
        const Huff &hdc = huff_[0][sc.c[k].td];
        const Huff &hac = huff_[1][sc.c[k].ta];
        for (int32_t j = 0; j < hi * vi; j++) {
            const int32_t bx = hi * mx + j % hi, by = vi * my + j / hi;
            // (the block's stream: its block row mod v = j / hi, JpegPieces)
            ZTRY(first_block_pieces(r, sc, hdc, hac, dc[ci], p, ci, size_t(by) * size_t(mxx * hi) + size_t(bx), j / hi, zz));
        }
    }
    return 0;
}

int Decoder::mcu_pieces(const Scan &sc, int32_t my, int32_t mx, int32_t *dc, int32_t *zz, JpegPieces &p)
{
    constexpr size_t kMcuSlack = 8192; // > an MCU's entropy-coded bytes (<= 10 blocks x 216, stuffed x2)
    if (len_ - pos_ >= kMcuSlack) {
        FastBits fb(*this);
        const int e = mcu_pieces_with(fb, sc, my, mx, dc, zz, p);
        fb.sync();
        return e;
    }
    MemberBits mb{*this};
    return mcu_pieces_with(mb, sc, my, mx, dc, zz, p);
}

template <class Sink>
int Decoder::mcu(const Scan &sc, int32_t my, int32_t mx, int32_t &block_count, int32_t *dc, int32_t *b,
                 uint8_t *nzpos, Sink &sink)
{
    if constexpr (std::is_same<Sink, PieceSink>::value) {
        // (b: the zig-zag block, zero between blocks)
        if (!sc.prog && sc.ah == 0 && sc.ns != 1) return mcu_pieces(sc, my, mx, dc, b, sink.p);
    }
    const int32_t mxx = sc.mxx;
    for (int k = 0; k < sc.ns; k++) {
        const int ci = sc.c[k].id;
        const int32_t hi = o_.comp[ci].h, vi = o_.comp[ci].v;
        const Huff &hdc = huff_[0][sc.c[k].td];
        const Huff &hac = huff_[1][sc.c[k].ta];
        for (int32_t j = 0; j < hi * vi; j++) {
            int32_t bx, by;
            if (sc.ns != 1) {
                bx = hi * mx + j % hi;
                by = vi * my + j / hi;
            } else {
                bx = block_count % (mxx * hi);
                by = block_count / (mxx * hi);
                block_count++;
                if (bx * 8 >= static_cast<int32_t>(o_.width) || by * 8 >= static_cast<int32_t>(o_.height))
                    continue;
            }
            const size_t blk = size_t(by) * size_t(mxx * hi) + size_t(bx);
            if (sc.prog) {
                // (the Decoder's own reader: a progressive scan reads a few
                // bits a block -- a DC bit, an end-of-band run -- and copying
                // the reader in and out per block cost more than it saved)
                ZTRY(prog_block_member(sc, ci, blk, hdc, hac, dc));
                continue;
            }
            if constexpr (std::is_same<Sink, PieceSink>::value) {
                if (sc.ah == 0) { // (b: the zig-zag block, zero between blocks)
                    int e;
                    if (len_ - pos_ >= kFastSlack) {
                        FastBits fb(*this);
                        e = first_block_pieces(fb, sc, hdc, hac, dc[ci], sink.p, ci, blk, by % vi, b);
                        fb.sync();
                    } else {
                        MemberBits mb{*this};
                        e = first_block_pieces(mb, sc, hdc, hac, dc[ci], sink.p, ci, blk, by % vi, b);
                    }
                    if (e) return e;
                    continue;
                }
            }
            int nnz = 0;
            if (sc.ah != 0) {
                ZTRY(refine(b, hac, sc.zs, sc.ze, int32_t(1) << sc.al));
            } else if (len_ - pos_ >= kFastSlack) {
                FastBits fb(*this); // (the block's bit reads in registers)
                const int e = first_block(fb, sc, hdc, hac, dc[ci], b, nzpos, nnz);
                fb.sync();
                if (e) return e;
            } else {
                MemberBits mb{*this};
                ZTRY(first_block(mb, sc, hdc, hac, dc[ci], b, nzpos, nnz));
            }
            ZTRY(sink.put(ci, blk, b, nzpos, nnz));
            for (int i = 0; i < nnz; i++) b[nzpos[i]] = 0;
        }
    }
    return 0;
}

// A progressive scan's block (processSos :1340-1431 with refine :1459-1549):
// the reference loads the whole block, updates the scan's band and stores
// the whole block back; only the band can change, so only the band is read
// and only the coefficients that changed are written -- the same grid, and
// no cost for the blocks an EOB run skips.
template <class R>
int Decoder::prog_block(R &r, const Scan &sc, int ci, size_t blk, const Huff &hdc, const Huff &hac, int32_t *dc)
{
    if (sc.ah != 0) {
        const int32_t delta = int32_t(1) << sc.al;
        if (sc.zs == 0) { // refine :1461-1470
            if (sc.ze != 0) return ZPX_E_PANIC;
            bool set;
            ZTRY(r.bit(set));
            if (set) ZTRY(prog_set(ci, blk, 0, prog_get(ci, blk, 0) | delta));
            return 0;
        }
        return prog_refine_ac(r, ci, blk, hac, sc.zs, sc.ze, delta);
    }
    int32_t zig = sc.zs;
    if (zig == 0) {
        zig++;
        uint8_t t;
        ZTRY(r.huffman(hdc, t));
        if (t > 16) return ZPX_E_EXCESSIVE_DC_COMPONENT;
        int32_t delta;
        ZTRY(r.receive_extend(t, delta));
        dc[ci] += delta;
        ZTRY(prog_set(ci, blk, 0, dc[ci] << sc.al));
    }
    if (zig <= sc.ze && eob_run_ > 0) {
        eob_run_--;
        return 0;
    }
    for (; zig <= sc.ze; zig++) {
        uint8_t value;
        ZTRY(r.huffman(hac, value));
        const uint8_t v0r = value >> 4, v1 = value & 0x0f;
        if (v1 != 0) {
            zig += v0r;
            if (zig > sc.ze) break;
            int32_t ac;
            ZTRY(r.receive_extend(v1, ac));
            ZTRY(prog_set(ci, blk, zig, ac << sc.al));
        } else {
            if (v0r != 0x0f) {
                eob_run_ = static_cast<uint16_t>(1u << v0r);
                if (v0r != 0) {
                    uint32_t x;
                    ZTRY(r.bits(v0r, x));
                    eob_run_ |= static_cast<uint16_t>(x);
                }
                eob_run_--;
                break;
            }
            zig += 0x0f;
        }
    }
    return 0;
}

// refineNonZeroes :1522-1549: from zig, each nonzero coefficient takes a
// correction bit; the loop stops at the (nz+1)-th zero coefficient (nz = -1:
// the band's end) and returns its position.  With the block's nonzero mask
// the stop is found by bit arithmetic and the correction bits, one per
// nonzero coefficient before it in zig-zag order, are read together (up to
// 16 at a time: exactly the bits, and so the bytes, the reference's loop
// reads one at a time).
template <class R>
int Decoder::prog_refine_nonzero(R &r, int ci, size_t blk, uint64_t mask, int32_t zig, int32_t ze, int32_t nz,
                                 int32_t delta, int32_t &zout)
{
    if (zig > ze) {
        zout = zig;
        return 0;
    }
    const uint64_t band = ((~uint64_t(0)) << zig) & (ze >= 63 ? ~uint64_t(0) : (uint64_t(2) << ze) - 1);
    int32_t end = ze + 1;
    if (nz >= 0) {
        uint64_t zeros = ~mask & band;
        for (int32_t k = 0; k < nz && zeros; k++) zeros &= zeros - 1;
        if (zeros) end = __builtin_ctzll(zeros);
    }
    uint64_t m = mask & band & (end >= 64 ? ~uint64_t(0) : (uint64_t(1) << end) - 1);
    while (m) {
        const int n = std::min(16, __builtin_popcountll(m));
        uint32_t corr;
        ZTRY(r.bits(n, corr));
        for (int k = n - 1; k >= 0; k--) {
            const int z = __builtin_ctzll(m);
            m &= m - 1;
            if (!((corr >> k) & 1)) continue;
            const int32_t v = prog_get(ci, blk, z);
            ZTRY(prog_set(ci, blk, z, v + (v >= 0 ? delta : -delta)));
        }
    }
    zout = end;
    return 0;
}

template <class R>
int Decoder::prog_refine_ac(R &r, int ci, size_t blk, const Huff &h, int32_t zs, int32_t ze, int32_t delta)
{ // refine :1471-1518
    int32_t zig = zs;
    // (a coefficient this scan sets is outside the mask of the zeros the
    // runs count, and is behind zig before the mask is read again)
    if (eob_run_ == 0) {
        for (; zig <= ze; zig++) {
            int32_t z = 0;
            uint8_t value;
            ZTRY(r.huffman(h, value));
            const uint8_t v0 = value >> 4, v1 = value & 0x0f;
            if (v1 == 0) {
                if (v0 != 0x0f) {
                    eob_run_ = static_cast<uint16_t>(1u << v0);
                    if (v0 != 0) {
                        uint32_t x;
                        ZTRY(r.bits(v0, x));
                        eob_run_ |= static_cast<uint16_t>(x);
                    }
                    break;
                }
            } else if (v1 == 1) {
                bool positive;
                ZTRY(r.bit(positive));
                z = positive ? delta : -delta;
            } else {
                return ZPX_E_UNEXPECTED_HUFFMAN_CODE;
            }
            ZTRY(prog_refine_nonzero(r, ci, blk, prog_mask(ci, blk), zig, ze, v0, delta, zig));
            if (zig > ze) return ZPX_E_TOO_MANY_COEFFICIENTS;
            if (z != 0) ZTRY(prog_set(ci, blk, zig, z));
        }
    }
    if (eob_run_ > 0) {
        eob_run_--;
        int32_t ignored;
        ZTRY(prog_refine_nonzero(r, ci, blk, prog_mask(ci, blk), zig, ze, -1, delta, ignored));
    }
    return 0;
}

bool Decoder::next_marker(size_t p, size_t &after, uint8_t &marker) const
{ // run()'s loop head (decodeInner :240-283)
    for (;;) {
        if (p + 2 > len_) return false;
        uint8_t t0 = src_[p], t1 = src_[p + 1];
        p += 2;
        while (t0 != 0xff) {
            if (p >= len_) return false;
            t0 = t1;
            t1 = src_[p++];
        }
        uint8_t m = t1;
        if (m == 0) continue;
        while (m == 0xff) {
            if (p >= len_) return false;
            m = src_[p++];
        }
        if (m >= 0xd0 && m <= 0xd7) continue; // a stray RST
        after = p;
        marker = m;
        return true;
    }
}

std::atomic<int64_t> g_parallel_scans{0}; // zpx_debug_jpeg_parallel_scans

// Restart-interval-parallel Huffman decoding of a baseline scan with DRI.
// The RSTn markers (byte aligned; 0xFF inside entropy-coded data is always
// stuffed as FF 00) split the scan into independent segments: each restarts
// with an empty bit buffer, zero DC predictors and no EOB run (:1432-1452).
// Segments decode on `threads_` threads, each with its own copy of the bit
// reader over the whole input (so reads that run into a marker behave as in
// the serial loop), and each must end exactly where the serial loop would
// read its RST marker.  Anything else -- markers out of order or missing,
// fill bytes, an error inside a segment, a segment ending elsewhere, a value
// too wide for the grid -- leaves done = false, and the caller runs the
// serial loop from the scan's start: its result and error are the
// reference's by construction.  The last segment runs on this decoder, so
// the state after the scan is the serial loop's.
int Decoder::restart_parallel(const Scan &sc, bool &done)
{
    done = false;
    const int32_t total = sc.mxx * sc.myy, ri = restart_interval_;
    if (sc.prog || threads_ <= 1 || ri <= 0) return 0;
    const char *mn = getenv("ZPX_HUFF_PAR_MIN_MCUS");
    if (total < (mn ? atoi(mn) : 4096)) return 0;
    const int32_t nseg = (total + ri - 1) / ri;
    if (nseg < 2 || unread_ != 0) return 0;
    std::vector<size_t> start(static_cast<size_t>(nseg)), end(static_cast<size_t>(nseg), len_);
    start[0] = pos_;
    int32_t k = 0;
    for (size_t i = pos_; i + 1 < len_; i++) {
        if (src_[i] != 0xff) continue;
        const uint8_t m = src_[i + 1];
        if (m == 0x00) {
            i++;
            continue;
        }
        if (m >= 0xd0 && m <= 0xd7 && k < nseg - 1) {
            if (m != 0xd0 + (k & 7)) return 0;
            end[static_cast<size_t>(k)] = i;
            start[static_cast<size_t>(k) + 1] = i + 2;
            k++;
            i++;
            continue;
        }
        break; // any other marker ends the scan's data
    }
    if (k != nseg - 1) return 0;
    const int nthr = std::min<int>(threads_, nseg);
    std::atomic<bool> ok{true};
    std::vector<FixedSink> sinks(static_cast<size_t>(nthr), FixedSink{o_, {0, 0, 0, 0}, {}});
    // segment s: MCUs [s * ri, min(total, (s + 1) * ri)) from byte start[s]
    auto run_segment = [&](Decoder &d, FixedSink &sink, int32_t s) -> bool {
        d.pos_ = start[static_cast<size_t>(s)];
        d.unread_ = 0;
        d.ba_ = d.bm_ = 0;
        d.bn_ = 0;
        d.eob_run_ = 0;
        int32_t dc[4] = {0, 0, 0, 0}, b[64];
        uint8_t nzpos[64];
        memset(b, 0, sizeof(b));
        const int32_t m0 = s * ri, m1 = std::min(total, m0 + ri);
        int32_t block_count = 0;
        if (sc.ns == 1) block_count = m0 * o_.comp[sc.c[0].id].h * o_.comp[sc.c[0].id].v;
        for (int32_t m = m0; m < m1; m++)
            if (d.mcu(sc, m / sc.mxx, m % sc.mxx, block_count, dc, b, nzpos, sink)) return false;
        if (s == nseg - 1) return true;
        d.settle(); // what the serial loop's readFull of the marker does first
        return d.pos_ == end[static_cast<size_t>(s)];
    };
    // thread t takes the contiguous segments [nseg * t / nthr, nseg * (t+1) / nthr);
    // workers run on copies of this decoder (made before any thread runs),
    // this thread takes the last run, so it ends in the serial loop's state
    std::vector<Decoder> copies;
    copies.reserve(static_cast<size_t>(nthr - 1));
    for (int t = 0; t < nthr - 1; t++) copies.emplace_back(*this);
    auto run_range = [&](Decoder &d, int t) {
        const int32_t a = nseg * t / nthr, z = nseg * (t + 1) / nthr;
        for (int32_t s = a; s < z && ok.load(std::memory_order_relaxed); s++)
            if (!run_segment(d, sinks[static_cast<size_t>(t)], s)) ok = false;
    };
    std::vector<std::thread> th;
    for (int t = 0; t < nthr - 1 && ok; t++) {
        try {
            th.emplace_back([&, t] { run_range(copies[static_cast<size_t>(t)], t); });
        } catch (...) { // no thread: the serial loop
            ok = false;
        }
    }
    const size_t scan_start = start[0];
    if (ok) run_range(*this, nthr - 1);
    const bool last_ok = ok;
    for (auto &t : th) t.join();
    if (!ok || !last_ok) { // serial from the scan's start
        pos_ = scan_start;
        unread_ = 0;
        ba_ = bm_ = 0;
        bn_ = 0;
        eob_run_ = 0;
        return 0;
    }
    for (int j = 0; j < sc.ns; j++) { // the width the values need, then the values too wide before
        const int ci = sc.c[j].id;
        int32_t m = 0;
        std::vector<std::pair<size_t, int32_t>> ov;
        for (auto &sk : sinks) {
            m = std::max(m, sk.max_abs[ci]);
            ov.insert(ov.end(), sk.overflow[ci].begin(), sk.overflow[ci].end());
        }
        if (!o_.grid[ci].apply_overflow(m, ov)) return ZPX_E_OUT_OF_MEMORY;
    }
    done = true;
    g_parallel_scans.fetch_add(1, std::memory_order_relaxed);
    return 0;
}

int Decoder::run()
{ // decodeInner :220-373
    ZTRY(full(tmp_, 2));
    if (tmp_[0] != 0xff || tmp_[1] != 0xd8) return ZPX_E_INVALID_SOI_MARKER;
    for (;;) {
        ZTRY(full(tmp_, 2));
        while (tmp_[0] != 0xff) { // extraneous data (:246-269)
            tmp_[0] = tmp_[1];
            ZTRY(byte(tmp_[1]));
        }
        uint8_t marker = tmp_[1];
        if (marker == 0) continue;
        while (marker == 0xff) ZTRY(byte(marker));
        if (marker == 0xd9) break;                    // EOI
        if (marker >= 0xd0 && marker <= 0xd7) continue; // stray RST
        ZTRY(full(tmp_, 2));
        const int32_t n = (int32_t(tmp_[0]) << 8) + tmp_[1] - 2;
        if (n < 0) return ZPX_E_SHORT_SEGMENT_LENGTH;
        switch (marker) {
        case 0xc0:
        case 0xc1:
        case 0xc2:
            o_.baseline = marker == 0xc0;
            o_.progressive = marker == 0xc2;
            ZTRY(sof(n));
            if (config_only_ && o_.jfif) return kConfigOnly; // :311-313
            break;
        case 0xdb:
            if (config_only_) ZTRY(skip(n)); // :315-321
            else ZTRY(dqt(n));
            break;
        case 0xdd: // processDri :621-627
            if (config_only_) {
                ZTRY(skip(n));
                break;
            }
            if (n != 2) return ZPX_E_DRI_WRONG_LENGTH;
            ZTRY(full(tmp_, 2));
            restart_interval_ = static_cast<uint16_t>((tmp_[0] << 8) + tmp_[1]);
            break;
        case 0xc4:
            if (config_only_) ZTRY(skip(n));
            else ZTRY(dht(n));
            break;
        case 0xda:
            if (config_only_) return kConfigOnly; // :336-340
            ZTRY(sos(n));
            break;
        case 0xe0: // processApp0Marker :668-680
            if (n < 5) {
                ZTRY(skip(n));
                break;
            }
            ZTRY(full(tmp_, 5));
            o_.jfif = memcmp(tmp_, "JFIF\0", 5) == 0;
            ZTRY(skip(n - 5));
            break;
        case 0xee: // processApp14Marker :682-697
            if (n < 12) {
                ZTRY(skip(n));
                break;
            }
            ZTRY(full(tmp_, 12));
            if (memcmp(tmp_, "Adobe", 5) == 0) {
                o_.adobe_valid = true;
                o_.adobe_transform = tmp_[11];
            }
            ZTRY(skip(n - 12));
            break;
        default:
            if ((marker >= 0xe0 && marker <= 0xef) || marker == 0xfe) ZTRY(skip(n));
            else if (marker < 0xc0) return ZPX_E_UNKNOWN_MARKER;
            else return ZPX_E_UNSUPPORTED_MARKER;
        }
    }
    if (!seen_sos_) return ZPX_E_MISSING_SOS_MARKER; // :372
    for (int c = 0; c < o_.n_comp; c++) {
        if (o_.progressive) {
            if (o_.has_grid[c]) snapshot_quant(c); // reconstructProgressiveImage uses final tables
            o_.rule[c] = o_.has_grid[c] ? ZPX_BLOCKS_PROGRESSIVE : ZPX_BLOCKS_NONE;
        } else if (interleaved_[c]) {
            o_.rule[c] = ZPX_BLOCKS_ALL;
        } else if (noninterleaved_[c]) {
            o_.rule[c] = ZPX_BLOCKS_SCAN;
        } else {
            o_.rule[c] = ZPX_BLOCKS_NONE;
        }
    }
    return 0;
}

std::atomic<int64_t> g_parallel_prog{0}; // progressive frames decoded scan-parallel (zpx_debug_jpeg_parallel_scans)

// The scans of a progressive frame, decoded concurrently (the reference's
// processSos runs them one after another, decoder.zig:1148-1455, refine
// :1459-1549).  Scan j waits for every earlier scan that touches a
// coefficient it touches (a common component with overlapping spectral
// bands: refinements follow their band's first scan, DC refinement the DC
// scan); the rest run at once on `threads` threads -- with the standard
// scripts the luma bands, the chroma scans and the DC scans overlap.  Each
// scan runs on the copy of the decoder made at its SOS (its Huffman tables
// and restart interval), from its first entropy-coded byte, with an empty
// bit buffer, zero DC predictors and no EOB run, into int16 grids (a value
// past int16 aborts).  The result is the serial loop's when (checked after):
// every scan but the last ends with no EOB run pending (the next one started
// with none), and the marker loop resumed from where each scan's decoding
// stopped reaches the same next marker as the first pass did.  Anything
// else -- an error in any scan included -- returns false, and the caller
// decodes the frame serially from the start, so results and errors are the
// reference's by construction.
int run_deferred_scans(std::vector<std::unique_ptr<Decoder>> &jobs, JpegCoeffs &o, int threads)
{
    const size_t n = jobs.size();
    // the components and zig-zag band each scan touches
    std::vector<std::vector<size_t>> deps(n);
    for (size_t j = 0; j < n; j++) {
        const auto &a = jobs[j]->job_scan_;
        for (size_t i = 0; i < j; i++) {
            const auto &b = jobs[i]->job_scan_;
            bool common = false;
            for (int x = 0; x < a.ns; x++)
                for (int y = 0; y < b.ns; y++) common |= a.c[x].id == b.c[y].id;
            // overlapping bands; and any two AC scans of one component, which
            // share its blocks' nonzero masks
            if (common && ((a.zs <= b.ze && b.zs <= a.ze) || (a.zs > 0 && b.zs > 0))) deps[j].push_back(i);
        }
    }
    std::vector<int16_t> dc[4]; // the DC coefficients, apart from the blocks until the scans are done
    for (int c = 0; c < o.n_comp; c++)
        if (o.has_grid[c]) dc[c].assign(o.grid[c].blocks(), 0);
    for (size_t j = 0; j < n; j++) {
        Decoder &d = *jobs[j];
        for (int c = 0; c < o.n_comp; c++) {
            d.fixed16_[c] = o.has_grid[c] ? o.grid[c].data16() : nullptr;
            d.dc16_[c] = o.has_grid[c] ? dc[c].data() : nullptr;
        }
        for (int k = 0; k < d.job_scan_.ns; k++)
            if (!d.fixed16_[d.job_scan_.c[k].id]) return false;
    }
    std::vector<int> rc(n, 0);
    std::vector<char> state(n, 0); // 0 waiting, 1 running, 2 done
    std::mutex mu;
    std::condition_variable cv;
    bool failed = false;
    size_t finished = 0;
    auto worker = [&] {
        std::unique_lock<std::mutex> lk(mu);
        for (;;) {
            size_t pick = n;
            for (size_t j = 0; j < n && pick == n && !failed; j++) {
                if (state[j] != 0) continue;
                bool ready = true;
                for (size_t i : deps[j]) ready &= state[i] == 2;
                if (ready) pick = j;
            }
            if (pick == n) {
                if (failed || finished == n) return;
                cv.wait(lk);
                continue;
            }
            state[pick] = 1;
            lk.unlock();
            Decoder &d = *jobs[pick];
            d.pos_ = d.job_start_;
            d.unread_ = 0;
            d.ba_ = d.bm_ = 0;
            d.bn_ = 0;
            d.eob_run_ = 0;
            int r = 0;
            const auto t0 = std::chrono::steady_clock::now();
            try {
                r = d.scan_loop(d.job_scan_, false);
            } catch (...) {
                r = ZPX_E_OUT_OF_MEMORY;
            }
            if (getenv("ZPX_JPEG_PROG_TRACE"))
                fprintf(stderr, "scan %zu ns %d c0 %d zs %d ze %d ah %u al %u: %.1f ms\n", pick, d.job_scan_.ns,
                        d.job_scan_.c[0].id, d.job_scan_.zs, d.job_scan_.ze, d.job_scan_.ah, d.job_scan_.al,
                        std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() * 1e3);
            lk.lock();
            rc[pick] = r;
            state[pick] = 2;
            finished++;
            if (r) failed = true;
            cv.notify_all();
        }
    };
    const int nthr = std::max(1, std::min<int>(threads, static_cast<int>(n)));
    std::vector<std::thread> th;
    for (int t = 1; t < nthr; t++) {
        try {
            th.emplace_back(worker);
        } catch (...) {
            break;
        }
    }
    worker();
    for (auto &t : th) t.join();
    if (failed || finished != n) return false;
    for (size_t j = 0; j < n; j++) {
        const Decoder &d = *jobs[j];
        if (j + 1 < n && d.eob_run_ != 0) return false;
        // where the serial loop resumes: readFull's settle() first
        const size_t resume = (d.unread_ > 0 && d.bn_ >= 8) ? d.pos_ - d.unread_ : d.pos_;
        size_t a0 = 0, a1 = 0;
        uint8_t m0 = 0, m1 = 0;
        const bool ok0 = d.next_marker(resume, a0, m0), ok1 = d.next_marker(d.job_skip_, a1, m1);
        if (!ok0 || !ok1 || a0 != a1 || m0 != m1) return false;
    }
    for (int c = 0; c < o.n_comp; c++) {
        if (!o.has_grid[c]) continue;
        int32_t m = 0;
        for (auto &d : jobs) m = std::max(m, d->job_max_[c]);
        int16_t *g = o.grid[c].data16();
        const size_t nb = o.grid[c].blocks();
        for (size_t b = 0; b < nb; b++) g[b * 64] = dc[c][b];
        o.grid[c].note_max_abs(m);
        if (!o.grid[c].narrow_to8(threads)) return false;
    }
    g_parallel_prog.fetch_add(1, std::memory_order_relaxed);
    return true;
}

} // namespace

int jpeg_entropy_decode(const uint8_t *buf, size_t len, JpegCoeffs &out, int threads, bool pieces)
{
    try { // no exception crosses the ABI
        int e = 0;
        bool decoded = false;
        static const bool prog_par = [] {
            const char *v = getenv("ZPX_JPEG_PROG_PARALLEL");
            return !(v && v[0] == '0');
        }();
        if (threads > 1 && prog_par) {
            // progressive scans in parallel (run_deferred_scans); a frame
            // without deferred scans was decoded by this run as usual
            std::vector<std::unique_ptr<Decoder>> jobs;
            {
                Decoder d(buf, len, out, false, threads, pieces);
                d.deferred_ = &jobs;
                e = d.run();
            }
            decoded = jobs.empty() || (!e && run_deferred_scans(jobs, out, threads));
            if (!decoded) out = JpegCoeffs{}; // the serial loop from the start
        }
        if (!decoded) {
            Decoder d(buf, len, out, false, threads, pieces);
            e = d.run();
        }
        if (e == kSparseAbort) { // pieces could not hold this frame: grids from the start
            out = JpegCoeffs{};
            Decoder d(buf, len, out, false, threads, false);
            e = d.run();
        }
        if (e) return e;
        if (out.pieces.valid) {
            out.pieces.compact();
            return ZPX_OK;
        }
        // one width per frame (the kernels take one coefficient type per frame)
        int bits = 8;
        for (int i = 0; i < 4; i++)
            if (out.has_grid[i]) bits = std::max(bits, out.grid[i].bits());
        for (int i = 0; i < 4; i++)
            if (out.has_grid[i] && !out.grid[i].widen_to(bits)) return ZPX_E_OUT_OF_MEMORY;
        return ZPX_OK;
    } catch (...) {
        return ZPX_E_OUT_OF_MEMORY;
    }
}

int64_t jpeg_parallel_scans() { return g_parallel_scans.load(); }
int64_t jpeg_parallel_progressive() { return g_parallel_prog.load(); }

int jpeg_huff_threads()
{
    static const int n = [] {
        if (const char *e = getenv("ZPX_HUFF_THREADS")) return std::max(1, atoi(e));
        return std::min(8, host_cpu_budget());
    }();
    return n;
}

int jpeg_decode_config(const uint8_t *buf, size_t len, uint32_t &w, uint32_t &h, int &model)
{ // decodeConfig :178-218
    JpegCoeffs c;
    Decoder d(buf, len, c, true);
    const int e = d.run();
    if (e != Decoder::kConfigOnly) return e ? e : ZPX_E_MISSING_SOS_MARKER;
    w = c.width;
    h = c.height;
    switch (c.n_comp) {
    case 1: model = ZPX_MODEL_GRAY; return ZPX_OK;
    case 3: case 4: model = ZPX_MODEL_YCBCR; return ZPX_OK; // "TODO: Support CMYK" (:212-216)
    default: return ZPX_E_INVALID_SOI_MARKER;
    }
}

JpegOut jpeg_output_kind(const JpegCoeffs &c)
{
    if (c.n_comp == 1) return JpegOut::Gray;
    if (c.n_comp == 4) return (c.adobe_valid && c.adobe_transform == 0) ? JpegOut::CMYK : JpegOut::YCCK;
    // isRgb :699-709
    if (!c.jfif && ((c.adobe_valid && c.adobe_transform == 0) ||
                    (c.comp[0].id == 'R' && c.comp[1].id == 'G' && c.comp[2].id == 'B')))
        return JpegOut::RGB;
    return JpegOut::YCbCr;
}

int jpeg_layout(const JpegCoeffs &c, JpegLayout &l)
{
    l = JpegLayout{};
    if (c.n_comp == 1) { // GrayImage.init on the MCU rect (:1717-1722)
        l.y_stride = size_t(8 * c.mxx);
        l.y_rows = size_t(8 * c.myy);
        l.total = l.y_stride * l.y_rows;
        return 0;
    }
    const int32_t h0 = c.comp[0].h, v0 = c.comp[0].v;
    const int32_t hr = h0 / c.comp[1].h, vr = v0 / c.comp[1].v;
    switch ((hr << 4) | vr) { // :1745-1753
    case 0x11: l.subsample = ZPX_RATIO444; break;
    case 0x12: l.subsample = ZPX_RATIO440; break;
    case 0x21: l.subsample = ZPX_RATIO422; break;
    case 0x22: l.subsample = ZPX_RATIO420; break;
    case 0x41: l.subsample = ZPX_RATIO411; break;
    case 0x42: l.subsample = ZPX_RATIO410; break;
    default: return ZPX_E_PANIC;
    }
    const int32_t w = 8 * h0 * c.mxx, h = 8 * v0 * c.myy; // padded rect
    int32_t cw = w, ch = h;                               // yCbCrSize (image.zig:521-555)
    switch (l.subsample) {
    case ZPX_RATIO422: cw = (w + 1) / 2; break;
    case ZPX_RATIO420: cw = (w + 1) / 2; ch = (h + 1) / 2; break;
    case ZPX_RATIO440: ch = (h + 1) / 2; break;
    case ZPX_RATIO411: cw = (w + 3) / 4; break;
    case ZPX_RATIO410: cw = (w + 3) / 4; ch = (h + 1) / 2; break;
    default: break;
    }
    l.y_stride = size_t(w);
    l.y_rows = size_t(h);
    l.c_stride = size_t(cw);
    l.c_rows = size_t(ch);
    l.cb_off = size_t(w) * size_t(h);
    l.cr_off = l.cb_off + size_t(cw) * size_t(ch);
    l.total = l.cr_off + size_t(cw) * size_t(ch);
    if (c.n_comp == 4) {
        l.k_stride = size_t(8 * c.comp[3].h * c.mxx);
        l.k_rows = size_t(8 * c.comp[3].v * c.myy);
        l.k_total = l.k_stride * l.k_rows;
    }
    return 0;
}

} // namespace zpx
