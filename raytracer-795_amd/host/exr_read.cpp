// exr_read.cpp — OpenEXR decoder for image textures and environment maps (hw5/hw6 .exr
// textures, src/Texture.cpp:13-17, 69-73, 185-189).
//
// The reference decodes with its vendored tinyexr (LoadEXR, src/Helper.cpp:346-359) and keeps
// RGBA floats; the texture code reads R, G, B.  This is a restatement of the published
// OpenEXR 2 file layout (magic/version, attribute header, offset table, chunks) and of its
// codecs, written from the format description (the PIZ wavelet's inverse is derived from the
// forward lifting equations, see wavelet_inverse_2d):
//   RLE   signed run counts, then the byte predictor and the two-half interleave
//   ZIPS/ZIP  zlib (1 / 16 lines per chunk), same predictor and interleave
//   PIZ   per-block value bitmap + forward LUT, canonical Huffman with run-length pseudo
//         symbol, 2-D Haar-like wavelet (14- or 16-bit lifting), 32 lines per chunk
// Only what texture loading needs is supported (single part, scanline or one-level tiled,
// x/y sampling 1); anything else fails loudly with a message.  Decoding is host I/O, once
// per texture, outside the hot path.
#include "exr_read.hpp"

#include <string.h>
#include <zlib.h>

#include <algorithm>
#include <cstdint>
#include <fstream>
#include <sstream>
#include <stdexcept>

namespace rtgh {
namespace {

enum { kUint = 0, kHalf = 1, kFloat = 2 };
enum { kNone = 0, kRle = 1, kZips = 2, kZip = 3, kPiz = 4 };

struct Chan {
    std::string name;
    int type;
};

struct Reader {
    const unsigned char* p;
    const unsigned char* end;
    bool ok = true;
    uint32_t u32() {
        if (end - p < 4) { ok = false; p = end; return 0; }
        uint32_t v = (uint32_t)p[0] | (uint32_t)p[1] << 8 | (uint32_t)p[2] << 16 | (uint32_t)p[3] << 24;
        p += 4;
        return v;
    }
    int32_t i32() { return (int32_t)u32(); }
    uint64_t u64() { uint64_t lo = u32(); return lo | (uint64_t)u32() << 32; }
    std::string cstr() {
        const unsigned char* z = (const unsigned char*)memchr(p, 0, end - p);
        if (!z) { ok = false; p = end; return std::string(); }
        std::string s((const char*)p, z - p);
        p = z + 1;
        return s;
    }
};

float half_to_float(uint16_t h) {
    const uint32_t s = (uint32_t)(h >> 15) << 31;
    uint32_t e = (h >> 10) & 0x1f, m = h & 0x3ff, bits;
    if (e == 0) {
        if (m == 0) {
            bits = s;
        } else {                        // subnormal half -> normal float
            e = 113;
            while (!(m & 0x400)) { m <<= 1; e--; }
            bits = s | (e << 23) | ((m & 0x3ff) << 13);
        }
    } else if (e == 31) {
        bits = s | 0x7f800000u | (m << 13);
    } else {
        bits = s | ((e + 112) << 23) | (m << 13);
    }
    float f;
    memcpy(&f, &bits, 4);
    return f;
}

// ---- RLE / ZIP: byte predictor + interleave of the two halves
void unpredict_interleave(std::vector<unsigned char>& t, unsigned char* out) {
    const size_t n = t.size();
    for (size_t i = 1; i < n; i++) t[i] = (unsigned char)((int)t[i - 1] + (int)t[i] - 128);
    const unsigned char* t1 = t.data();
    const unsigned char* t2 = t.data() + (n + 1) / 2;
    for (size_t i = 0; i < n; i++) out[i] = (i & 1) ? *t2++ : *t1++;
}

bool rle_decode(const unsigned char* in, size_t n, std::vector<unsigned char>& out, size_t expect) {
    out.clear();
    out.reserve(expect);
    size_t i = 0;
    while (i < n) {
        const int c = (signed char)in[i++];
        if (c < 0) {
            const size_t k = (size_t)(-c);
            if (i + k > n || out.size() + k > expect) return false;
            out.insert(out.end(), in + i, in + i + k);
            i += k;
        } else {
            if (i >= n || out.size() + c + 1 > expect) return false;
            out.insert(out.end(), (size_t)c + 1, in[i++]);
        }
    }
    return out.size() == expect;
}

// ---- PIZ
constexpr int kUshortRange = 1 << 16;
constexpr int kBitmapSize = kUshortRange >> 3;
constexpr int kSymbols = (1 << 16) + 1;     // 16-bit values plus one run-length pseudo symbol
constexpr int kMaxLen = 58;                 // longest code length a 6-bit length field can name

// The PIZ entropy stream, as the OpenEXR 2 format describes it:
//   header   int32 lo, int32 hi (symbol range, hi = the run-length pseudo symbol),
//            int32 table bytes, int32 payload bit count, int32 reserved      (20 bytes)
//   lengths  one 6-bit field per symbol lo..hi, most significant bit first; a field of
//            1..58 is that symbol's code length, 0 means "no code", 59..62 stand for a
//            stretch of 2..5 symbols without a code, and 63 is followed by an 8-bit field k
//            for a stretch of k + 6 such symbols
//   payload  the codes, most significant bit first; the pseudo symbol is followed by an
//            8-bit repeat count of the value decoded before it
// The codes are canonical with the *longest* codes numerically smallest: going from length
// 58 down to 1, the first code of a length is the value just past the last code of the next
// longer length, halved (rounded down), and within one length the codes ascend with the
// symbol.  So every code of length L at least first[L] is a complete code word, and every
// value below first[L] is the prefix of a longer one; decoding reads bit by bit and stops
// at the first length whose code range holds the bits read so far (the code-range decoder
// of canonical prefix codes).

// Reads bits MSB first from a byte string of `nbits` valid bits (codes are at most 58 bits long:
// the decoder takes the shortest length first, then one bit at a time).
struct MsbBits {
    const unsigned char* data;
    uint64_t nbits;
    uint64_t at = 0;
    // the next n (1..57) bits without consuming them; bits past the end read as 0
    uint64_t peek(int n) const {
        const uint64_t byte = at >> 3, nbytes = (nbits + 7) >> 3;
        uint64_t w = 0;
        for (int k = 0; k < 8; k++) w = (w << 8) | (byte + k < nbytes ? data[byte + k] : 0u);
        uint64_t v = (w << (at & 7)) >> (64 - n);
        const uint64_t left = nbits > at ? nbits - at : 0;
        if (left < (uint64_t)n) v &= ~((1ull << (n - left)) - 1);
        return v;
    }
    bool take(int n, uint64_t& v) {      // n <= 64
        if (at + (uint64_t)n > nbits) return false;
        v = 0;
        for (int k = n; k > 0;) {           // peek covers 57 bits: at most 32 per step
            const int m = k < 32 ? k : 32;
            v = (v << m) | peek(m);
            at += (uint64_t)m;
            k -= m;
        }
        return true;
    }
    bool take(int n, uint32_t& v) {      // n <= 32
        uint64_t w;
        if (!take(n, w)) return false;
        v = (uint32_t)w;
        return true;
    }
};

struct CanonicalCode {
    uint64_t first[kMaxLen + 2] = {};   // first code value of each length
    uint32_t count[kMaxLen + 2] = {};   // codes of each length
    uint32_t start[kMaxLen + 2] = {};   // position of the length's first symbol in `by_code`
    std::vector<int> by_code;           // symbols sorted by (length, code)
    int shortest = 0, longest = 0;
    // direct lookup of the codes of at most kLut bits: entry = symbol << 8 | length (0: none)
    std::vector<uint32_t> lut;
};
constexpr int kLut = 12;

// Length table -> canonical code; false with `err` set if the lengths do not form a prefix
// code (a code that does not fit its length, or a shorter code equal to a longer one's prefix).
bool build_canonical(const std::vector<uint8_t>& len, int lo, CanonicalCode& cc, std::string& err) {
    for (uint8_t l : len) cc.count[l]++;
    cc.count[0] = 0;
    uint64_t past = 0;                      // value just past the last code of length L + 1
    for (int L = kMaxLen; L >= 1; L--) {
        cc.first[L] = past >> 1;
        past = cc.first[L] + cc.count[L];
        if (cc.count[L] && past > (1ull << L)) { err = "PIZ: Huffman code does not fit its length"; return false; }
    }
    for (int L = 1; L <= kMaxLen; L++)
        if (cc.count[L]) {
            if (!cc.shortest) cc.shortest = L;
            cc.longest = L;
        }
    // prefix-free: the largest length-S prefix of the length-L codes (L > S) lies below first[S]
    for (int S = 1; S <= kMaxLen; S++) {
        if (!cc.count[S]) continue;
        for (int L = S + 1; L <= kMaxLen; L++)
            if (cc.count[L] && ((cc.first[L] + cc.count[L] - 1) >> (L - S)) >= cc.first[S]) {
                err = "PIZ: Huffman lengths do not form a prefix code";
                return false;
            }
    }
    uint32_t acc = 0;
    for (int L = 1; L <= kMaxLen; L++) {
        cc.start[L] = acc;
        acc += cc.count[L];
    }
    cc.by_code.assign(acc, 0);
    std::vector<uint32_t> fill(cc.start, cc.start + kMaxLen + 1);
    for (size_t i = 0; i < len.size(); i++)          // ascending symbols -> ascending codes
        if (len[i]) cc.by_code[fill[len[i]]++] = lo + (int)i;
    // every kLut-bit window that starts with a code of length L <= kLut (prefix-free: at most one)
    cc.lut.assign((size_t)1 << kLut, 0u);
    for (int L = 1; L <= kLut; L++)
        for (uint32_t k = 0; k < cc.count[L]; k++) {
            const uint64_t code = cc.first[L] + k;
            const uint32_t e = (uint32_t)cc.by_code[cc.start[L] + k] << 8 | (uint32_t)L;
            for (uint64_t j = 0; j < (1ull << (kLut - L)); j++) cc.lut[(size_t)(code << (kLut - L) | j)] = e;
        }
    return true;
}

bool read_code_lengths(MsbBits& b, int lo, int hi, std::vector<uint8_t>& len, std::string& err) {
    len.assign((size_t)(hi - lo + 1), 0);
    size_t sym = 0;
    while (sym < len.size()) {
        uint32_t field;
        if (!b.take(6, field)) { err = "PIZ: truncated Huffman table"; return false; }
        if (field <= (uint32_t)kMaxLen) {
            len[sym++] = (uint8_t)field;
            continue;
        }
        uint32_t stretch = field - 57;               // 59..62 -> 2..5
        if (field == 63) {
            uint32_t k;
            if (!b.take(8, k)) { err = "PIZ: truncated Huffman table"; return false; }
            stretch = k + 6;
        }
        if (stretch > len.size() - sym) { err = "PIZ: Huffman table runs past its symbol range"; return false; }
        sym += stretch;                              // lengths already 0
    }
    return true;
}

bool huf_decode(const unsigned char* in, size_t n_in, uint16_t* out, size_t n_out, std::string& err) {
    if (n_in == 0) {
        if (n_out) { err = "PIZ: empty Huffman stream"; return false; }
        return true;
    }
    if (n_in < 20) { err = "PIZ: truncated Huffman header"; return false; }
    auto i32 = [&](int o) { return (int32_t)((uint32_t)in[o] | (uint32_t)in[o + 1] << 8 | (uint32_t)in[o + 2] << 16 | (uint32_t)in[o + 3] << 24); };
    const int lo = i32(0), hi = i32(4), table_bytes = i32(8), payload_bits = i32(12);
    if (lo < 0 || hi < lo || hi >= kSymbols || payload_bits < 0) { err = "PIZ: bad Huffman table size"; return false; }
    (void)table_bytes;                  // the table is self-delimiting; its bits are read below
    const unsigned char* body = in + 20;
    const size_t body_bytes = n_in - 20;

    MsbBits tb{body, 8ull * body_bytes};
    std::vector<uint8_t> len;
    if (!read_code_lengths(tb, lo, hi, len, err)) return false;
    CanonicalCode cc;
    if (!build_canonical(len, lo, cc, err)) return false;
    const size_t payload_at = (size_t)((tb.at + 7) / 8);        // the payload starts on a byte
    if ((uint64_t)payload_bits > 8ull * (body_bytes - payload_at)) { err = "PIZ: Huffman bit count exceeds the chunk"; return false; }
    if (payload_bits && !cc.longest) { err = "PIZ: Huffman payload without codes"; return false; }

    MsbBits pb{body + payload_at, (uint64_t)payload_bits};
    const int repeat_symbol = hi;
    size_t written = 0;
    while (pb.at < pb.nbits) {
        int sym = -1;
        // short codes: one table lookup (a window past the end reads zeros, so the length is checked)
        const uint32_t e = cc.lut[(size_t)pb.peek(kLut)];
        if (e && pb.at + (e & 0xFFu) <= pb.nbits) {
            sym = (int)(e >> 8);
            pb.at += e & 0xFFu;
        }
        uint64_t v = 0;
        int L = cc.shortest;
        if (sym < 0 && !pb.take(cc.shortest, v)) { err = "PIZ: truncated code"; return false; }
        for (; sym < 0;) {
            if (cc.count[L] && v >= cc.first[L] && v - cc.first[L] < cc.count[L]) {
                sym = cc.by_code[cc.start[L] + (uint32_t)(v - cc.first[L])];
                break;
            }
            if (L == cc.longest) break;
            uint32_t bit;
            if (!pb.take(1, bit)) break;
            v = (v << 1) | bit;
            L++;
        }
        if (sym < 0) { err = "PIZ: invalid code"; return false; }
        if (sym == repeat_symbol) {
            uint32_t times;
            if (!pb.take(8, times)) { err = "PIZ: truncated run"; return false; }
            if (written == 0) { err = "PIZ: run without a value"; return false; }
            if (written + times > n_out) { err = "PIZ: too much data"; return false; }
            std::fill(out + written, out + written + times, out[written - 1]);
            written += times;
        } else {
            if (written >= n_out) { err = "PIZ: too much data"; return false; }
            out[written++] = (uint16_t)sym;
        }
    }
    if (written != n_out) { err = "PIZ: not enough data"; return false; }
    return true;
}

// PIZ's wavelet (OpenEXR 2 format description, "PIZ compression"): a multi-level 2-D Haar-like
// transform with integer lifting.  One forward step maps a pair (a, b) to
//   narrow form (every value < 2^14):   lo = (a + b) >> 1,      hi = a - b        (signed 16-bit)
//   wide form (modular, values >= 2^14): hi = (a + 2^15 - b) mod 2^16,
//                                        lo = (a + 2^15 + b) / 2 mod 2^16 (2^15 added when a + 2^15 < b)
// The inverse steps below follow from those definitions: in the narrow form a + b and a - b
// have the same parity, so a = lo + (hi + (hi & 1)) / 2 exactly and b = a - hi; in the wide form
// b = lo - hi / 2 and a = hi + b - 2^15, both mod 2^16.
struct InverseLift {
    bool wide;
    void operator()(uint16_t lo, uint16_t hi, uint16_t& a, uint16_t& b) const {
        if (!wide) {
            const int h = (int16_t)hi;
            const int av = (int16_t)lo + ((h + (h & 1)) >> 1);
            a = (uint16_t)(int16_t)av;
            b = (uint16_t)(int16_t)(av - h);
        } else {
            const unsigned bv = ((unsigned)lo - ((unsigned)hi >> 1)) & 0xFFFFu;
            a = (uint16_t)(((unsigned)hi + bv + 0x8000u) & 0xFFFFu);   // - 2^15 == + 2^15 mod 2^16
            b = (uint16_t)bv;
        }
    }
};

// Inverse transform of one nx x ny plane of 16-bit words at `base`, sample (i, j) at
// base[i * sx + j * sy].  The encoder halves the lattice level by level: at the level with pair
// distance p (lattice step q = 2p) every q-aligned 2x2 cell {(i, j), (i+p, j), (i, j+p), (i+p, j+p)}
// was transformed along x, then along y; a last odd column (nx & p) or row (ny & p) of cells was
// transformed along one axis only.  Decoding runs the levels coarse to fine: p from half the
// largest power of two <= min(nx, ny) down to 1, each cell along y first, then along x.
void wavelet_inverse_2d(uint16_t* base, int nx, int ny, int sx, int sy, uint16_t maxval) {
    const InverseLift lift{maxval >= (1 << 14)};
    auto at = [&](int i, int j) -> uint16_t& { return base[(ptrdiff_t)i * sx + (ptrdiff_t)j * sy]; };
    const int n = std::min(nx, ny);
    int top = 1;
    while (top * 2 <= n) top *= 2;               // largest power of two <= n
    for (int p = top / 2; p >= 1; p /= 2) {
        const int q = 2 * p;
        const int ci = (nx - q) / q + 1, cj = (ny - q) / q + 1;   // full cells per row / column
        for (int cy = 0; cy < cj; cy++) {
            const int j = cy * q;
            for (int cx = 0; cx < ci; cx++) {
                const int i = cx * q;
                uint16_t t00, t01, t10, t11;
                lift(at(i, j), at(i, j + p), t00, t10);          // along y, left column
                lift(at(i + p, j), at(i + p, j + p), t01, t11);  // along y, right column
                lift(t00, t01, at(i, j), at(i + p, j));          // along x, top row
                lift(t10, t11, at(i, j + p), at(i + p, j + p));  // along x, bottom row
            }
            if (nx & p) {                                        // odd column of cells: y only
                const int i = ci * q;
                uint16_t a, b;
                lift(at(i, j), at(i, j + p), a, b);
                at(i, j) = a;
                at(i, j + p) = b;
            }
        }
        if (ny & p) {                                            // odd row of cells: x only
            const int j = cj * q;
            for (int cx = 0; cx < ci; cx++) {
                const int i = cx * q;
                uint16_t a, b;
                lift(at(i, j), at(i + p, j), a, b);
                at(i, j) = a;
                at(i + p, j) = b;
            }
        }
    }
}

int type_bytes(int t) { return t == kHalf ? 2 : 4; }

bool piz_decode(const unsigned char* in, size_t n, unsigned char* out, int nx, int ny, const std::vector<Chan>& chans,
                std::string& err) {
    if (n < 4) { err = "PIZ: truncated chunk"; return false; }
    std::vector<unsigned char> bitmap(kBitmapSize, 0);
    const int minnz = in[0] | in[1] << 8, maxnz = in[2] | in[3] << 8;
    size_t o = 4;
    if (maxnz >= kBitmapSize) { err = "PIZ: bad bitmap range"; return false; }
    if (minnz <= maxnz) {
        const size_t k = (size_t)(maxnz - minnz + 1);
        if (o + k > n) { err = "PIZ: truncated bitmap"; return false; }
        memcpy(bitmap.data() + minnz, in + o, k);
        o += k;
    }
    std::vector<uint16_t> lut(kUshortRange, 0);
    int k = 0;
    for (int i = 0; i < kUshortRange; i++)
        if (i == 0 || (bitmap[i >> 3] & (1 << (i & 7)))) lut[k++] = (uint16_t)i;
    const uint16_t maxv = (uint16_t)(k - 1);
    if (o + 4 > n) { err = "PIZ: truncated length"; return false; }
    const uint32_t len = (uint32_t)in[o] | (uint32_t)in[o + 1] << 8 | (uint32_t)in[o + 2] << 16 | (uint32_t)in[o + 3] << 24;
    o += 4;
    if ((size_t)len > n - o) { err = "PIZ: Huffman data exceeds the chunk"; return false; }
    size_t total = 0;
    for (const Chan& c : chans) total += (size_t)nx * ny * (type_bytes(c.type) / 2);
    std::vector<uint16_t> tmp(total ? total : 1);
    if (!huf_decode(in + o, len, tmp.data(), total, err)) return false;
    size_t start = 0;
    for (const Chan& c : chans) {
        const int size = type_bytes(c.type) / 2;
        for (int j = 0; j < size; j++) wavelet_inverse_2d(tmp.data() + start + j, nx, ny, size, nx * size, maxv);
        start += (size_t)nx * ny * size;
    }
    for (size_t i = 0; i < total; i++) tmp[i] = lut[tmp[i]];
    // planar per channel -> per line, per channel (little-endian 16-bit words)
    std::vector<size_t> cur(chans.size());
    start = 0;
    for (size_t c = 0; c < chans.size(); c++) {
        cur[c] = start;
        start += (size_t)nx * ny * (type_bytes(chans[c].type) / 2);
    }
    unsigned char* w = out;
    for (int y = 0; y < ny; y++)
        for (size_t c = 0; c < chans.size(); c++) {
            const size_t m = (size_t)nx * (type_bytes(chans[c].type) / 2);
            for (size_t i = 0; i < m; i++) {
                const uint16_t v = tmp[cur[c] + i];
                *w++ = (unsigned char)(v & 0xff);
                *w++ = (unsigned char)(v >> 8);
            }
            cur[c] += m;
        }
    return true;
}

// Decode one chunk (nx x ny pixels) into the uncompressed per-line, per-channel layout.
bool decode_chunk(int comp, const unsigned char* data, size_t n, int nx, int ny, const std::vector<Chan>& chans,
                  std::vector<unsigned char>& raw, std::string& err) {
    size_t line = 0;
    for (const Chan& c : chans) line += (size_t)nx * type_bytes(c.type);
    const size_t expect = line * ny;
    raw.resize(expect);
    if (n == expect || comp == kNone) {     // stored uncompressed
        if (n != expect) { err = "uncompressed chunk has the wrong size"; return false; }
        memcpy(raw.data(), data, expect);
        return true;
    }
    std::vector<unsigned char> t;
    switch (comp) {
    case kRle:
        if (!rle_decode(data, n, t, expect)) { err = "RLE: corrupt chunk"; return false; }
        unpredict_interleave(t, raw.data());
        return true;
    case kZips:
    case kZip: {
        t.resize(expect);
        uLongf dl = (uLongf)expect;
        if (uncompress(t.data(), &dl, data, (uLong)n) != Z_OK || dl != expect) { err = "ZIP: corrupt chunk"; return false; }
        unpredict_interleave(t, raw.data());
        return true;
    }
    case kPiz:
        return piz_decode(data, n, raw.data(), nx, ny, chans, err);
    default:
        err = "compression " + std::to_string(comp) + " not supported (NONE, RLE, ZIPS, ZIP, PIZ are)";
        return false;
    }
}

}  // namespace

namespace {
bool read_exr_impl(const std::string& path, std::vector<float>& rgba, int& w, int& h, std::string& err) {
    std::string file;
    {
        std::ifstream f(path, std::ios::binary);
        if (!f) { err = "cannot read EXR " + path; return false; }
        std::ostringstream ss;
        ss << f.rdbuf();
        file = ss.str();
    }
    const unsigned char* base = (const unsigned char*)file.data();
    Reader r{base, base + file.size()};
    if (file.size() < 8 || r.u32() != 20000630u) { err = "not an OpenEXR file: " + path; return false; }
    const uint32_t ver = r.u32();
    if ((ver & 0xff) != 2) { err = "unsupported OpenEXR version in " + path; return false; }
    const bool tiled = ver & 0x200;
    if (ver & 0x800) { err = "deep OpenEXR images are not supported: " + path; return false; }
    if (ver & 0x1000) { err = "multi-part OpenEXR files are not supported: " + path; return false; }

    std::vector<Chan> chans;
    int comp = -1, xmin = 0, ymin = 0, xmax = -1, ymax = -1;
    uint32_t tx = 0, ty = 0;
    int level_mode = 0;
    bool have_dw = false;
    for (;;) {
        const std::string name = r.cstr();
        if (!r.ok) { err = "truncated EXR header: " + path; return false; }
        if (name.empty()) break;
        const std::string type = r.cstr();
        const int32_t size = r.i32();
        if (!r.ok || size < 0 || r.end - r.p < size) { err = "truncated EXR header: " + path; return false; }
        Reader a{r.p, r.p + size};
        if (name == "channels" && type == "chlist") {
            for (;;) {
                const std::string cn = a.cstr();
                if (!a.ok || cn.empty()) break;
                Chan c{cn, a.i32()};
                a.u32();                    // pLinear + reserved
                const int xs = a.i32(), ys = a.i32();
                if (!a.ok) break;
                if (c.type < kUint || c.type > kFloat) { err = "bad EXR channel type in " + path; return false; }
                if (xs != 1 || ys != 1) { err = "subsampled EXR channels are not supported: " + path; return false; }
                chans.push_back(c);
            }
        } else if (name == "compression" && size >= 1) {
            comp = r.p[0];
        } else if (name == "dataWindow" && size >= 16) {
            xmin = a.i32(); ymin = a.i32(); xmax = a.i32(); ymax = a.i32();
            have_dw = true;
        } else if (name == "tiles" && size >= 9) {
            tx = a.u32(); ty = a.u32();
            level_mode = a.p[0] & 0x0f;
        }
        r.p += size;
    }
    if (chans.empty() || comp < 0 || !have_dw) { err = "EXR header lacks channels/compression/dataWindow: " + path; return false; }
    if ((int64_t)xmax - xmin + 1 <= 0 || (int64_t)ymax - ymin + 1 <= 0 ||
        ((int64_t)xmax - xmin + 1) * ((int64_t)ymax - ymin + 1) > (1ll << 28)) {
        err = "bad EXR data window in " + path; return false;
    }
    w = xmax - xmin + 1;
    h = ymax - ymin + 1;
    if (tiled && (tx == 0 || ty == 0 || tx > (1u << 20) || ty > (1u << 20) || level_mode != 0)) { err = "only one-level tiled EXR images are supported: " + path; return false; }
    const int lpb = comp == kZip ? 16 : comp == kPiz ? 32 : 1;
    const int64_t nchunks = tiled ? (int64_t)((w + tx - 1) / tx) * ((h + ty - 1) / ty) : (h + lpb - 1) / lpb;
    if (nchunks <= 0 || (uint64_t)nchunks * 8 > file.size()) { err = "EXR offset table exceeds the file: " + path; return false; }
    std::vector<uint64_t> offsets(nchunks);
    for (auto& o : offsets) o = r.u64();
    if (!r.ok) { err = "truncated EXR offset table: " + path; return false; }

    const size_t np = (size_t)w * h;
    std::vector<std::vector<float>> planes(chans.size(), std::vector<float>(np, 0.0f));
    std::vector<unsigned char> raw;
    for (int64_t ci = 0; ci < nchunks; ci++) {
        if (offsets[ci] >= file.size()) { err = "bad EXR chunk offset in " + path; return false; }
        Reader c{base + offsets[ci], base + file.size()};
        int x0, y0, nx, ny;
        if (tiled) {
            const int tix = c.i32(), tiy = c.i32();
            c.i32(); c.i32();               // level (0, 0)
            if (tix < 0 || tiy < 0 || (int64_t)tix * tx >= w || (int64_t)tiy * ty >= h) {
                err = "bad EXR tile coordinates in " + path;
                return false;
            }
            x0 = tix * (int)tx;
            y0 = tiy * (int)ty;
            nx = std::min<int>((int)tx, w - x0);
            ny = std::min<int>((int)ty, h - y0);
        } else {
            y0 = c.i32() - ymin;
            if (y0 < 0 || y0 >= h) { err = "bad EXR scanline in " + path; return false; }
            x0 = 0;
            nx = w;
            ny = std::min(lpb, h - y0);
        }
        const int32_t n = c.i32();
        if (!c.ok || n < 0 || c.end - c.p < n) { err = "truncated EXR chunk in " + path; return false; }
        if (!decode_chunk(comp, c.p, (size_t)n, nx, ny, chans, raw, err)) { err += " (" + path + ")"; return false; }
        const unsigned char* q = raw.data();
        for (int y = 0; y < ny; y++)
            for (size_t k = 0; k < chans.size(); k++) {
                float* dst = planes[k].data() + (size_t)(y0 + y) * w + x0;
                for (int x = 0; x < nx; x++) {
                    if (chans[k].type == kHalf) {
                        dst[x] = half_to_float((uint16_t)(q[0] | q[1] << 8));
                        q += 2;
                    } else {                // FLOAT, or UINT bits read as float like LoadEXR
                        const uint32_t b = (uint32_t)q[0] | (uint32_t)q[1] << 8 | (uint32_t)q[2] << 16 | (uint32_t)q[3] << 24;
                        memcpy(&dst[x], &b, 4);
                        q += 4;
                    }
                }
            }
    }

    // LoadEXR's channel selection (names after the last '.', first four channels searched)
    int iR = -1, iG = -1, iB = -1, iA = -1;
    for (size_t k = 0; k < chans.size() && k < 4; k++) {
        std::string s = chans[k].name;
        const size_t dot = s.find_last_of('.');
        if (dot != std::string::npos) s = s.substr(dot + 1);
        if (s == "R") iR = (int)k; else if (s == "G") iG = (int)k; else if (s == "B") iB = (int)k; else if (s == "A") iA = (int)k;
    }
    rgba.resize(np * 4);
    if (chans.size() == 1) {
        for (size_t i = 0; i < np; i++) rgba[4 * i] = rgba[4 * i + 1] = rgba[4 * i + 2] = rgba[4 * i + 3] = planes[0][i];
        return true;
    }
    if (iR < 0 || iG < 0 || iB < 0) { err = std::string(iR < 0 ? "R" : iG < 0 ? "G" : "B") + " channel not found in " + path; return false; }
    for (size_t i = 0; i < np; i++) {
        rgba[4 * i] = planes[iR][i];
        rgba[4 * i + 1] = planes[iG][i];
        rgba[4 * i + 2] = planes[iB][i];
        rgba[4 * i + 3] = iA >= 0 ? planes[iA][i] : 1.0f;
    }
    return true;
}

}  // namespace

bool read_exr_rgba(const std::string& path, std::vector<float>& rgba, int& w, int& h, std::string& err) {
    try {                               // the C ABI above never throws
        return read_exr_impl(path, rgba, w, h, err);
    } catch (const std::exception& e) {
        err = std::string("EXR decode of ") + path + ": " + e.what();
        return false;
    }
}

}  // namespace rtgh
