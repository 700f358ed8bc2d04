// The watermark's payload codec, host side: QR Model 2 encode / decode
// and AES-CBC, behind the C ABI (include/tmfwm.h, tmfwm_qr_* / tmfwm_aes_*).
//
// The reference produces the watermark with modules/qrcode_generator.py:10-44 (python-qrcode:
// byte mode, error correction H, smallest version >= 1 that fits, box 10, border 4) around
// modules/encryption.py:8-40 (AES-CBC, random IV prepended, PKCS#7), and consumes the
// extracted tile with qrcode_to_text (:47-76, pyzbar / zbar) and decrypt_watermark
// (encryption.py:43-68, pycryptodome).  None of those libraries is in this image, so this
// file restates the published algorithms: ISO/IEC 18004 (QR: Reed-Solomon over GF(256)
// with x^8+x^4+x^3+x^2+1, BCH format / version information, the eight data masks and the
// four penalty rules) and FIPS-197 / SP 800-38A (AES, CBC).  Versions 1-10 (up to 271 data
// bytes at level L, 119 at level H: a 64-byte AES payload after base64 needs version 6 at H).
//
// The encoder follows python-qrcode's choices so that a watermark made here is the one the
// reference makes: its segmentation (util.optimal_data_chunks: runs of >= 20 digits in
// numeric mode, runs of >= 20 alphanumeric characters in alphanumeric mode, the rest in byte
// mode; whole-string modes for <= 20 characters), the smallest version that fits, and its
// mask choice -- the lowest ISO penalty with the format / version modules and the dark
// module left light, as its best_mask_pattern() scores them.  (python-qrcode is not in this
// image: the bytes are pinned only by the standard and round trips -- "parity unpinned".)
//
// The decoder is for what the app feeds it: an axis-aligned QR image (the extracted tile,
// extract_watermark :288-292) -- global Otsu threshold, finder patterns by 1:1:3:1:1 run
// ratios along rows and columns, an affine module grid from the three finder centres,
// format information from either copy (nearest valid BCH word, <= 3 bit errors),
// Reed-Solomon error correction per block (Berlekamp-Massey, Chien, Forney), then the
// numeric / alphanumeric / byte segments.  Extraction never rotates the tile, so only the
// upright orientation is searched.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

#include "../../include/tmfwm.h"
#include "tmfwm_internal.h"

namespace {

using tmf::report;

// ---------------------------------------------------------------------------
// GF(256), primitive polynomial 0x11D, generator alpha = 2
// ---------------------------------------------------------------------------
struct GF {
    uint8_t exp[512], log[256];
    GF()
    {
        int x = 1;
        for (int i = 0; i < 255; ++i) {
            exp[i] = (uint8_t)x;
            log[x] = (uint8_t)i;
            x <<= 1;
            if (x & 0x100) x ^= 0x11D;
        }
        for (int i = 255; i < 512; ++i) exp[i] = exp[i - 255];
        log[0] = 0;
    }
    uint8_t mul(uint8_t a, uint8_t b) const { return (a && b) ? exp[log[a] + log[b]] : 0; }
    uint8_t div(uint8_t a, uint8_t b) const { return a ? exp[(log[a] + 255 - log[b]) % 255] : 0; }
    uint8_t pow_a(int e) const { return exp[((e % 255) + 255) % 255]; }
};
const GF &gf()
{
    static const GF g;
    return g;
}

// generator polynomial prod_{i<n} (x - alpha^i), highest degree first (monic, n+1 terms)
std::vector<uint8_t> rs_generator(int n)
{
    const GF &G = gf();
    std::vector<uint8_t> g{1};
    for (int i = 0; i < n; ++i) {
        std::vector<uint8_t> h(g.size() + 1, 0);
        for (size_t k = 0; k < g.size(); ++k) {
            h[k] ^= g[k];
            h[k + 1] ^= G.mul(g[k], G.exp[i]);
        }
        g.swap(h);
    }
    return g;
}

// EC codewords of one block: remainder of data * x^n modulo the generator
void rs_encode(const uint8_t *data, int k, int n, uint8_t *ec)
{
    const GF &G = gf();
    const std::vector<uint8_t> g = rs_generator(n);
    std::vector<uint8_t> r(n, 0);
    for (int i = 0; i < k; ++i) {
        const uint8_t f = data[i] ^ r[0];
        for (int j = 0; j < n - 1; ++j) r[j] = r[j + 1] ^ G.mul(f, g[j + 1]);
        r[n - 1] = G.mul(f, g[n]);
    }
    std::memcpy(ec, r.data(), n);
}

// Correct one block in place (codeword c[0] is the highest power); returns corrected count or -1
int rs_decode(uint8_t *c, int len, int nsym)
{
    const GF &G = gf();
    std::vector<uint8_t> S(nsym);
    bool clean = true;
    for (int j = 0; j < nsym; ++j) {  // S_j = c(alpha^j)
        uint8_t s = 0;
        for (int i = 0; i < len; ++i) s = G.mul(s, G.exp[j]) ^ c[i];
        S[j] = s;
        clean = clean && s == 0;
    }
    if (clean) return 0;
    // Berlekamp-Massey: Lambda(x) lowest degree first
    std::vector<uint8_t> L{1}, B{1};
    int Ldeg = 0, m = 1;
    uint8_t b = 1;
    for (int r = 0; r < nsym; ++r) {
        uint8_t d = S[r];
        for (int i = 1; i <= Ldeg && i < (int)L.size(); ++i) d ^= G.mul(L[i], S[r - i]);
        if (d == 0) {
            ++m;
            continue;
        }
        std::vector<uint8_t> T = L;
        const uint8_t coef = G.div(d, b);
        if (L.size() < B.size() + m) L.resize(B.size() + m, 0);
        for (size_t i = 0; i < B.size(); ++i) L[i + m] ^= G.mul(coef, B[i]);
        if (2 * Ldeg <= r) {
            Ldeg = r + 1 - Ldeg;
            B = T;
            b = d;
            m = 1;
        } else {
            ++m;
        }
    }
    L.resize(Ldeg + 1, 0);
    if (Ldeg == 0 || 2 * Ldeg > nsym) return -1;
    // Chien search: error at position p (power len-1-i) iff Lambda(alpha^-(len-1-i)) == 0
    std::vector<int> pos;
    for (int i = 0; i < len; ++i) {
        const int e = len - 1 - i;
        uint8_t v = 0;
        for (int k = Ldeg; k >= 0; --k) v = G.mul(v, G.pow_a(-e)) ^ L[k];
        if (v == 0) pos.push_back(i);
    }
    if ((int)pos.size() != Ldeg) return -1;
    // Omega = S(x) Lambda(x) mod x^nsym (S(x) = sum S_j x^j)
    std::vector<uint8_t> Om(nsym, 0);
    for (int i = 0; i < nsym; ++i)
        for (int k = 0; k <= Ldeg && k <= i; ++k) Om[i] ^= G.mul(S[i - k], L[k]);
    // Forney (first consecutive root alpha^0): e = X * Omega(X^-1) / Lambda'(X^-1)
    for (int i : pos) {
        const int e = len - 1 - i;
        const uint8_t Xi = G.pow_a(-e), X = G.pow_a(e);
        uint8_t om = 0;
        for (int k = nsym - 1; k >= 0; --k) om = G.mul(om, Xi) ^ Om[k];
        uint8_t dl = 0;  // formal derivative: odd terms
        for (int k = 1; k <= Ldeg; k += 2) dl ^= G.mul(L[k], G.pow_a(-e * (k - 1)));
        if (dl == 0) return -1;
        c[i] ^= G.mul(X, G.div(om, dl));
    }
    for (int j = 0; j < nsym; ++j) {  // verify
        uint8_t s = 0;
        for (int i = 0; i < len; ++i) s = G.mul(s, G.exp[j]) ^ c[i];
        if (s) return -1;
    }
    return Ldeg;
}

// ---------------------------------------------------------------------------
// QR tables, versions 1-10.  Levels indexed by format bits: 0 = M, 1 = L, 2 = H, 3 = Q.
// Blocks: {count1, total1, data1, count2, total2, data2}
// ---------------------------------------------------------------------------
constexpr int kMaxVersion = 10;
const int kBlocks[kMaxVersion + 1][4][6] = {
    {},
    {{1, 26, 16, 0, 0, 0}, {1, 26, 19, 0, 0, 0}, {1, 26, 9, 0, 0, 0}, {1, 26, 13, 0, 0, 0}},
    {{1, 44, 28, 0, 0, 0}, {1, 44, 34, 0, 0, 0}, {1, 44, 16, 0, 0, 0}, {1, 44, 22, 0, 0, 0}},
    {{1, 70, 44, 0, 0, 0}, {1, 70, 55, 0, 0, 0}, {2, 35, 13, 0, 0, 0}, {2, 35, 17, 0, 0, 0}},
    {{2, 50, 32, 0, 0, 0}, {1, 100, 80, 0, 0, 0}, {4, 25, 9, 0, 0, 0}, {2, 50, 24, 0, 0, 0}},
    {{2, 67, 43, 0, 0, 0}, {1, 134, 108, 0, 0, 0}, {2, 33, 11, 2, 34, 12}, {2, 33, 15, 2, 34, 16}},
    {{4, 43, 27, 0, 0, 0}, {2, 86, 68, 0, 0, 0}, {4, 43, 15, 0, 0, 0}, {4, 43, 19, 0, 0, 0}},
    {{4, 49, 31, 0, 0, 0}, {2, 98, 78, 0, 0, 0}, {4, 39, 13, 1, 40, 14}, {2, 32, 14, 4, 33, 15}},
    {{2, 60, 38, 2, 61, 39}, {2, 121, 97, 0, 0, 0}, {4, 40, 14, 2, 41, 15}, {4, 40, 18, 2, 41, 19}},
    {{3, 58, 36, 2, 59, 37}, {2, 146, 116, 0, 0, 0}, {4, 36, 12, 4, 37, 13}, {4, 36, 16, 4, 37, 17}},
    {{4, 69, 43, 1, 70, 44}, {2, 86, 68, 2, 87, 69}, {6, 43, 15, 2, 44, 16}, {6, 43, 19, 2, 44, 20}},
};
const int kAlign[kMaxVersion + 1][3] = {{}, {}, {6, 18}, {6, 22}, {6, 26}, {6, 30}, {6, 34}, {6, 22, 38}, {6, 24, 42},
                                        {6, 26, 46}, {6, 28, 50}};
// API level (0 L, 1 M, 2 Q, 3 H) -> format bits
const int kLevelBits[4] = {1, 0, 3, 2};

int qr_size(int v) { return 17 + 4 * v; }
int data_codewords(int v, int lv)
{
    const int *b = kBlocks[v][lv];
    return b[0] * b[2] + b[3] * b[5];
}
int total_codewords(int v, int lv)
{
    const int *b = kBlocks[v][lv];
    return b[0] * b[1] + b[3] * b[4];
}

uint32_t bch(uint32_t data, uint32_t gen, int gen_bits)
{
    uint32_t d = data << (gen_bits - 1);
    for (int i = 31; i >= gen_bits - 1; --i)
        if (d & (1u << i)) d ^= gen << (i - (gen_bits - 1));
    return (data << (gen_bits - 1)) | d;
}
uint32_t format_word(int lvbits, int mask) { return bch((uint32_t)(lvbits << 3 | mask), 0x537, 11) ^ 0x5412; }
uint32_t version_word(int v) { return bch((uint32_t)v, 0x1F25, 13); }

bool mask_bit(int m, int r, int c)
{
    switch (m) {
    case 0: return (r + c) % 2 == 0;
    case 1: return r % 2 == 0;
    case 2: return c % 3 == 0;
    case 3: return (r + c) % 3 == 0;
    case 4: return (r / 2 + c / 3) % 2 == 0;
    case 5: return (r * c) % 2 + (r * c) % 3 == 0;
    case 6: return ((r * c) % 2 + (r * c) % 3) % 2 == 0;
    default: return ((r + c) % 2 + (r * c) % 3) % 2 == 0;
    }
}

// Module matrix with a function-pattern map.  m: 1 dark; fn: 1 reserved (not data).
struct Grid {
    int n = 0;
    std::vector<uint8_t> m, fn;
    explicit Grid(int v) : n(qr_size(v)), m(n * n, 0), fn(n * n, 0) { place_function(v); }
    uint8_t &at(int r, int c) { return m[r * n + c]; }
    void set_fn(int r, int c, int dark)
    {
        m[r * n + c] = (uint8_t)dark;
        fn[r * n + c] = 1;
    }
    void finder(int r0, int c0)
    {
        for (int dr = -1; dr <= 7; ++dr)
            for (int dc = -1; dc <= 7; ++dc) {
                const int r = r0 + dr, c = c0 + dc;
                if (r < 0 || c < 0 || r >= n || c >= n) continue;
                const bool in = dr >= 0 && dr <= 6 && dc >= 0 && dc <= 6;
                const bool dark = in && (dr == 0 || dr == 6 || dc == 0 || dc == 6 || (dr >= 2 && dr <= 4 && dc >= 2 && dc <= 4));
                set_fn(r, c, dark);
            }
    }
    void place_function(int v)
    {
        finder(0, 0);
        finder(0, n - 7);
        finder(n - 7, 0);
        for (int i = 8; i < n - 8; ++i) {
            set_fn(6, i, i % 2 == 0);
            set_fn(i, 6, i % 2 == 0);
        }
        const int *a = kAlign[v];
        const int na = v < 2 ? 0 : (v < 7 ? 2 : 3);
        for (int i = 0; i < na; ++i)
            for (int j = 0; j < na; ++j) {
                const int r = a[i], c = a[j];
                if ((r < 9 && c < 9) || (r < 9 && c >= n - 9) || (r >= n - 9 && c < 9)) continue;  // finder corners
                for (int dr = -2; dr <= 2; ++dr)
                    for (int dc = -2; dc <= 2; ++dc)
                        set_fn(r + dr, c + dc, std::max(std::abs(dr), std::abs(dc)) != 1);
            }
        // format areas (values written later) and the dark module
        for (int i = 0; i < 9; ++i) {
            if (!fn[8 * n + i]) set_fn(8, i, 0);
            if (!fn[i * n + 8]) set_fn(i, 8, 0);
        }
        for (int i = 0; i < 8; ++i) {
            set_fn(8, n - 1 - i, 0);
            set_fn(n - 1 - i, 8, 0);
        }
        set_fn(n - 8, 8, 1);
        if (v >= 7) {
            const uint32_t w = version_word(v);
            for (int i = 0; i < 18; ++i) {
                const int bit = (w >> i) & 1, r = i / 3, c = n - 11 + i % 3;
                set_fn(r, c, bit);
                set_fn(c, r, bit);
            }
        }
    }
    // format bits, both copies (bit i of the 15-bit word, i = 0 least significant)
    void put_format(uint32_t w)
    {
        for (int i = 0; i < 15; ++i) {
            const uint8_t bit = (w >> i) & 1;
            const int vr = i < 6 ? i : (i < 8 ? i + 1 : n - 15 + i);
            m[vr * n + 8] = bit;
            const int hc = i < 8 ? n - i - 1 : (i < 9 ? 15 - i : 14 - i);
            m[8 * n + hc] = bit;
        }
        m[(n - 8) * n + 8] = 1;
    }
};

// data-module visiting order (two-column zig-zag from the bottom right, skipping column 6)
std::vector<int> data_order(const Grid &g)
{
    std::vector<int> ord;
    const int n = g.n;
    int row = n - 1, inc = -1;
    for (int col = n - 1; col > 0; col -= 2) {
        if (col == 6) --col;
        for (;;) {
            for (int c = col; c > col - 2; --c)
                if (!g.fn[row * n + c]) ord.push_back(row * n + c);
            row += inc;
            if (row < 0 || row >= n) {
                row -= inc;
                inc = -inc;
                break;
            }
        }
    }
    return ord;
}


struct BitBuf {
    std::vector<uint8_t> bytes;
    int nbits = 0;
    void put(uint32_t v, int len)
    {
        for (int i = len - 1; i >= 0; --i) {
            if (nbits % 8 == 0) bytes.push_back(0);
            if ((v >> i) & 1) bytes.back() |= (uint8_t)(0x80 >> (nbits % 8));
            ++nbits;
        }
    }
};

// ---- python-qrcode segmentation (util.optimal_data_chunks, minimum = 20)
constexpr int kModeNum = 1, kModeAlnum = 2, kModeByte = 4;
const char kAlnumChars[] = "0123456789ABCDEFGHIJKLMNOPQRSTUVWXYZ $%*+-./:";
struct Segment {
    int mode;
    std::vector<uint8_t> d;
};
bool is_digit(uint8_t c) { return c >= '0' && c <= '9'; }
bool is_alnum(uint8_t c) { return c && std::strchr(kAlnumChars, c) != nullptr; }
int alnum_value(uint8_t c) { return (int)(std::strchr(kAlnumChars, c) - kAlnumChars); }

// re.search(pattern{20,}) split: maximal runs of >= 20 matching bytes are "in", the rest "out";
// for data of <= 20 bytes the whole string is "in" iff every byte matches (^pattern+$)
template <typename Pred>
std::vector<std::pair<bool, std::vector<uint8_t>>> optimal_split(const std::vector<uint8_t> &d, Pred match, size_t whole_len)
{
    std::vector<std::pair<bool, std::vector<uint8_t>>> out;
    if (d.empty()) return out;
    if (whole_len <= 20) {
        bool all = true;
        for (uint8_t c : d) all = all && match(c);
        out.push_back({all, d});
        return out;
    }
    size_t i = 0, start = 0;
    while (i < d.size()) {
        if (!match(d[i])) {
            ++i;
            continue;
        }
        size_t j = i;
        while (j < d.size() && match(d[j])) ++j;
        if (j - i >= 20) {
            if (i > start) out.push_back({false, std::vector<uint8_t>(d.begin() + start, d.begin() + i)});
            out.push_back({true, std::vector<uint8_t>(d.begin() + i, d.begin() + j)});
            start = j;
        }
        i = j;
    }
    if (start < d.size()) out.push_back({false, std::vector<uint8_t>(d.begin() + start, d.end())});
    return out;
}

std::vector<Segment> chunk_segments(const uint8_t *data, int len)
{
    std::vector<Segment> segs;
    const std::vector<uint8_t> all(data, data + len);
    for (auto &num : optimal_split(all, is_digit, all.size())) {
        if (num.first) {
            segs.push_back({kModeNum, num.second});
            continue;
        }
        // the alphanumeric pass sees the chunk, but its length test is on the whole data
        for (auto &al : optimal_split(num.second, is_alnum, all.size()))
            segs.push_back({al.first ? kModeAlnum : kModeByte, al.second});
    }
    return segs;  // empty data: no segment at all, as python-qrcode
}

int count_bits(int mode, int v)
{
    if (mode == kModeNum) return v < 10 ? 10 : 12;
    if (mode == kModeAlnum) return v < 10 ? 9 : 11;
    return v < 10 ? 8 : 16;
}

int segment_bits(const std::vector<Segment> &segs, int v)
{
    int bits = 0;
    for (const Segment &s : segs) {
        const int n = (int)s.d.size();
        bits += 4 + count_bits(s.mode, v);
        if (s.mode == kModeNum) bits += 10 * (n / 3) + (n % 3 == 2 ? 7 : n % 3 == 1 ? 4 : 0);
        else if (s.mode == kModeAlnum) bits += 11 * (n / 2) + 6 * (n % 2);
        else bits += 8 * n;
    }
    return bits;
}

void put_segment(BitBuf &bb, const Segment &s, int v)
{
    const int n = (int)s.d.size();
    bb.put((uint32_t)s.mode, 4);
    bb.put((uint32_t)n, count_bits(s.mode, v));
    if (s.mode == kModeNum) {
        int i = 0;
        for (; i + 3 <= n; i += 3) bb.put((uint32_t)((s.d[i] - '0') * 100 + (s.d[i + 1] - '0') * 10 + (s.d[i + 2] - '0')), 10);
        if (n - i == 2) bb.put((uint32_t)((s.d[i] - '0') * 10 + (s.d[i + 1] - '0')), 7);
        else if (n - i == 1) bb.put((uint32_t)(s.d[i] - '0'), 4);
    } else if (s.mode == kModeAlnum) {
        int i = 0;
        for (; i + 2 <= n; i += 2) bb.put((uint32_t)(alnum_value(s.d[i]) * 45 + alnum_value(s.d[i + 1])), 11);
        if (i < n) bb.put((uint32_t)alnum_value(s.d[i]), 6);
    } else {
        for (uint8_t c : s.d) bb.put(c, 8);
    }
}

// data bits into the non-function modules, masked (python-qrcode map_data)
void fill_data(Grid &g, const std::vector<int> &ord, const std::vector<uint8_t> &cw, int mk)
{
    for (size_t i = 0; i < ord.size(); ++i) {
        const int idx = ord[i], r = idx / g.n, c = idx % g.n;
        int bit = i < cw.size() * 8 ? (cw[i >> 3] >> (7 - (i & 7))) & 1 : 0;
        if (mask_bit(mk, r, c)) bit ^= 1;
        g.m[idx] = (uint8_t)bit;
    }
}

// ISO 18004 penalty (rules N1-N4) of a finished symbol
int penalty(const Grid &g)
{
    const int n = g.n;
    auto M = [&](int r, int c) { return (int)g.m[r * n + c]; };
    int p = 0;
    for (int pass = 0; pass < 2; ++pass)  // N1 runs, N3 finder-like patterns, rows then columns
        for (int i = 0; i < n; ++i) {
            int run = 1;
            for (int j = 1; j <= n; ++j) {
                const bool same = j < n && (pass ? M(j, i) == M(j - 1, i) : M(i, j) == M(i, j - 1));
                if (same) {
                    ++run;
                } else {
                    if (run >= 5) p += 3 + (run - 5);
                    run = 1;
                }
            }
            for (int j = 0; j + 10 < n + 1; ++j) {
                static const int pat[11] = {1, 0, 1, 1, 1, 0, 1, 0, 0, 0, 0};
                bool f1 = j + 11 <= n, f2 = j + 11 <= n;
                for (int k = 0; k < 11 && (f1 || f2); ++k) {
                    const int v = j + k < n ? (pass ? M(j + k, i) : M(i, j + k)) : 0;
                    f1 = f1 && v == pat[k];
                    f2 = f2 && v == pat[10 - k];
                }
                if (f1) p += 40;
                if (f2) p += 40;
            }
        }
    for (int r = 0; r + 1 < n; ++r)  // N2 2x2 blocks
        for (int c = 0; c + 1 < n; ++c) {
            const int v = M(r, c);
            if (v == M(r + 1, c) && v == M(r, c + 1) && v == M(r + 1, c + 1)) p += 3;
        }
    int dark = 0;  // N4 balance
    for (uint8_t v : g.m) dark += v;
    const int k = std::abs(dark * 20 - n * n * 10) / (n * n);
    return p + k * 10;
}

// ---------------------------------------------------------------------------
// Decoder
// ---------------------------------------------------------------------------
struct Pt {
    double x, y;
};

int otsu(const uint8_t *g, int h, int w, int64_t stride)
{
    int64_t hist[256] = {};
    for (int y = 0; y < h; ++y)
        for (int x = 0; x < w; ++x) ++hist[g[y * stride + x]];
    const double total = (double)h * w;
    double sum = 0;
    for (int i = 0; i < 256; ++i) sum += (double)i * hist[i];
    double wb = 0, sb = 0, best = -1;
    int thr = 128;
    for (int t = 0; t < 256; ++t) {
        wb += hist[t];
        if (wb == 0) continue;
        const double wf = total - wb;
        if (wf == 0) break;
        sb += (double)t * hist[t];
        const double mb = sb / wb, mf = (sum - sb) / wf, v = wb * wf * (mb - mf) * (mb - mf);
        if (v > best) {
            best = v;
            thr = t;
        }
    }
    return thr;  // dark iff value <= thr
}

struct Bin {
    int h, w;
    std::vector<uint8_t> d;  // 1 = dark
    int at(int y, int x) const { return (y < 0 || x < 0 || y >= h || x >= w) ? 0 : d[y * w + x]; }
};

// centre of a 1:1:3:1:1 run pattern ending before position `end` along a line; state = run lengths
bool ratio_ok(const int *s)
{
    const int tot = s[0] + s[1] + s[2] + s[3] + s[4];
    if (tot < 7) return false;
    const double u = tot / 7.0, tol = u * 0.5;  // ZXing's variance: a 1:1:1:1:1 checkerboard fails
    return std::fabs(s[0] - u) < tol && std::fabs(s[1] - u) < tol && std::fabs(s[2] - 3 * u) < 3 * tol &&
           std::fabs(s[3] - u) < tol && std::fabs(s[4] - u) < tol;
}

// run-length check along a vertical line through (x, yc); returns centre y or NAN
double cross_check(const Bin &b, int x, int yc, bool vertical, int expect)
{
    auto at = [&](int t) { return vertical ? b.at(t, x) : b.at(x, t); };
    const int lim = vertical ? b.h : b.w;
    int s[5] = {};
    int t = yc;
    if (!at(t)) return NAN;
    while (t >= 0 && at(t)) { ++s[2]; --t; }
    while (t >= 0 && !at(t) && s[1] <= expect) { ++s[1]; --t; }
    while (t >= 0 && at(t) && s[0] <= expect) { ++s[0]; --t; }
    t = yc + 1;
    while (t < lim && at(t)) { ++s[2]; ++t; }
    while (t < lim && !at(t) && s[3] <= expect) { ++s[3]; ++t; }
    while (t < lim && at(t) && s[4] <= expect) { ++s[4]; ++t; }
    if (!s[0] || !s[1] || !s[3] || !s[4] || !ratio_ok(s)) return NAN;
    return (double)(t - s[4] - s[3]) - s[2] / 2.0;
}

struct Cand {
    double x, y, mod;
    int hits;
};

std::vector<Cand> find_finders(const Bin &b)
{
    std::vector<Cand> cands;
    for (int y = 0; y < b.h; ++y) {
        int s[5] = {}, k = 0;
        for (int x = 0; x <= b.w; ++x) {
            const int v = x < b.w ? b.at(y, x) : 0;
            // state machine over alternating runs dark/light/dark/light/dark
            if ((k % 2 == 0) == (v == 1)) {
                ++s[k];
                continue;
            }
            if (k < 4) {
                if (k == 0 && s[0] == 0) continue;  // waiting for the first dark run
                ++k;
                s[k] = 1;
                continue;
            }
            // completed five runs at a light pixel after the last dark run
            if (ratio_ok(s)) {
                const int tot = s[0] + s[1] + s[2] + s[3] + s[4];
                const double cx = x - s[4] - s[3] - s[2] / 2.0;
                const double cy = cross_check(b, (int)cx, y, true, tot);
                if (!std::isnan(cy)) {
                    const double cx2 = cross_check(b, (int)cy, (int)cx, false, tot);
                    if (!std::isnan(cx2)) {
                        const double mod = tot / 7.0;
                        bool merged = false;
                        for (auto &c : cands)
                            if (std::fabs(c.x - cx2) < mod * 2 && std::fabs(c.y - cy) < mod * 2) {
                                c.x = (c.x * c.hits + cx2) / (c.hits + 1);
                                c.y = (c.y * c.hits + cy) / (c.hits + 1);
                                c.mod = (c.mod * c.hits + mod) / (c.hits + 1);
                                ++c.hits;
                                merged = true;
                                break;
                            }
                        if (!merged) cands.push_back({cx2, cy, mod, 1});
                    }
                }
            }
            // shift: keep the last light/dark runs as the start of a new pattern
            s[0] = s[2];
            s[1] = s[3];
            s[2] = s[4];
            s[3] = 1;
            s[4] = 0;
            k = 3;
        }
    }
    return cands;
}

// sample module (r, c) of an n-module symbol through the affine map
struct Affine {
    Pt o, dx, dy;  // pixel of module (0,0) centre, per-column and per-row steps
    Pt at(double r, double c) const { return {o.x + c * dx.x + r * dy.x, o.y + c * dx.y + r * dy.y}; }
};

int sample(const Bin &b, const Affine &A, int r, int c)
{
    const Pt p = A.at(r, c);  // continuous coordinates: pixel (i, j) covers [j, j+1) x [i, i+1)
    return b.at((int)std::floor(p.y), (int)std::floor(p.x));
}

int hamming(uint32_t a, uint32_t b) { return __builtin_popcount(a ^ b); }

// decode the data bytes from codewords in byte / numeric / alphanumeric mode segments
bool parse_segments(const std::vector<uint8_t> &dw, int v, std::vector<uint8_t> &out)
{
    int pos = 0;
    const int nbits = (int)dw.size() * 8;
    auto get = [&](int len, bool &ok) -> uint32_t {
        if (pos + len > nbits) {
            ok = false;
            return 0;
        }
        uint32_t r = 0;
        for (int i = 0; i < len; ++i, ++pos) r = (r << 1) | ((dw[pos >> 3] >> (7 - (pos & 7))) & 1);
        return r;
    };
    static const char kAlnum[] = "0123456789ABCDEFGHIJKLMNOPQRSTUVWXYZ $%*+-./:";
    for (;;) {
        if (nbits - pos < 4) return true;
        bool ok = true;
        const uint32_t mode = get(4, ok);
        if (!ok || mode == 0) return true;
        if (mode == 4) {  // byte
            const uint32_t len = get(v < 10 ? 8 : 16, ok);
            for (uint32_t i = 0; i < len && ok; ++i) out.push_back((uint8_t)get(8, ok));
            if (!ok) return false;
        } else if (mode == 1) {  // numeric
            uint32_t len = get(v < 10 ? 10 : 12, ok);
            while (ok && len >= 3) {
                const uint32_t x = get(10, ok);
                out.push_back('0' + x / 100);
                out.push_back('0' + x / 10 % 10);
                out.push_back('0' + x % 10);
                len -= 3;
            }
            if (ok && len == 2) {
                const uint32_t x = get(7, ok);
                out.push_back('0' + x / 10);
                out.push_back('0' + x % 10);
            } else if (ok && len == 1) {
                out.push_back('0' + get(4, ok));
            }
            if (!ok) return false;
        } else if (mode == 2) {  // alphanumeric
            uint32_t len = get(v < 10 ? 9 : 11, ok);
            while (ok && len >= 2) {
                const uint32_t x = get(11, ok);
                if (x / 45 >= 45) return false;
                out.push_back(kAlnum[x / 45]);
                out.push_back(kAlnum[x % 45]);
                len -= 2;
            }
            if (ok && len == 1) {
                const uint32_t x = get(6, ok);
                if (x >= 45) return false;
                out.push_back(kAlnum[x]);
            }
            if (!ok) return false;
        } else if (mode == 7) {  // ECI designator: skip its value
            const uint32_t first = get(8, ok);
            if ((first & 0x80) == 0x80) get((first & 0x40) ? 16 : 8, ok);
            if (!ok) return false;
        } else {
            return false;  // kanji / structured append / FNC1: not produced by the app
        }
    }
}

// read the symbol through A (version v); true with the payload on success
bool read_symbol(const Bin &b, const Affine &A, int v, std::vector<uint8_t> &payload)
{
    const int n = qr_size(v);
    Grid g(v);
    for (int r = 0; r < n; ++r)
        for (int c = 0; c < n; ++c) g.m[r * n + c] = (uint8_t)sample(b, A, r, c);
    // format information: both copies, nearest valid word
    uint32_t f1 = 0, f2 = 0;
    for (int i = 0; i < 15; ++i) {
        const int vr = i < 6 ? i : (i < 8 ? i + 1 : n - 15 + i);
        const int hc = i < 8 ? n - i - 1 : (i < 9 ? 15 - i : 14 - i);
        f1 |= (uint32_t)g.m[vr * n + 8] << i;
        f2 |= (uint32_t)g.m[8 * n + hc] << i;
    }
    int best = 99, lvbits = 0, mask = 0;
    for (int lb = 0; lb < 4; ++lb)
        for (int mk = 0; mk < 8; ++mk) {
            const uint32_t w = format_word(lb, mk);
            const int d = std::min(hamming(w, f1), hamming(w, f2));
            if (d < best) {
                best = d;
                lvbits = lb;
                mask = mk;
            }
        }
    if (best > 3) return false;
    const int *bl = kBlocks[v][lvbits];
    const int nblocks = bl[0] + bl[3], total = total_codewords(v, lvbits);
    const std::vector<int> ord = data_order(g);
    std::vector<uint8_t> cw(total, 0);
    for (int i = 0; i < total * 8 && i < (int)ord.size(); ++i) {
        const int idx = ord[i], r = idx / n, c = idx % n;
        const int bit = g.m[idx] ^ (mask_bit(mask, r, c) ? 1 : 0);
        if (bit) cw[i >> 3] |= (uint8_t)(0x80 >> (i & 7));
    }
    // de-interleave
    std::vector<std::vector<uint8_t>> blocks(nblocks);
    std::vector<int> dlen(nblocks), tlen(nblocks);
    for (int k = 0; k < nblocks; ++k) {
        const bool second = k >= bl[0];
        dlen[k] = second ? bl[5] : bl[2];
        tlen[k] = second ? bl[4] : bl[1];
        blocks[k].assign(tlen[k], 0);
    }
    int p = 0;
    const int maxd = *std::max_element(dlen.begin(), dlen.end());
    for (int i = 0; i < maxd; ++i)
        for (int k = 0; k < nblocks; ++k)
            if (i < dlen[k]) blocks[k][i] = cw[p++];
    const int necc = tlen[0] - dlen[0];
    for (int i = 0; i < necc; ++i)
        for (int k = 0; k < nblocks; ++k) blocks[k][dlen[k] + i] = cw[p++];
    std::vector<uint8_t> dw;
    for (int k = 0; k < nblocks; ++k) {
        if (rs_decode(blocks[k].data(), tlen[k], necc) < 0) return false;
        dw.insert(dw.end(), blocks[k].begin(), blocks[k].begin() + dlen[k]);
    }
    payload.clear();
    return parse_segments(dw, v, payload);
}

bool decode_bin(const Bin &b, std::vector<uint8_t> &payload)
{
    std::vector<Cand> c = find_finders(b);
    if (c.size() < 3) return false;
    std::sort(c.begin(), c.end(), [](const Cand &a, const Cand &d) { return a.hits > d.hits; });
    const int nc = std::min<int>((int)c.size(), 8);
    // every triple of the strongest candidates, as (top-left, top-right, bottom-left)
    for (int i = 0; i < nc; ++i)
        for (int j = 0; j < nc; ++j)
            for (int k = 0; k < nc; ++k) {
                if (i == j || j == k || i == k) continue;
                const Pt tl{c[i].x, c[i].y}, tr{c[j].x, c[j].y}, bl{c[k].x, c[k].y};
                const double ux = tr.x - tl.x, uy = tr.y - tl.y, vx = bl.x - tl.x, vy = bl.y - tl.y;
                if (ux * vy - uy * vx <= 0) continue;  // TR clockwise from BL in image coordinates
                const double du = std::hypot(ux, uy), dv = std::hypot(vx, vy);
                if (du < 1e-6 || dv < 1e-6 || std::fabs(du - dv) > 0.2 * std::max(du, dv)) continue;
                const double mod = (c[i].mod + c[j].mod + c[k].mod) / 3.0;
                const int v0 = (int)std::lround(((du + dv) / 2.0 / mod + 7 - 17) / 4.0);
                for (int dvv = 0; dvv <= 2; ++dvv)
                    for (int sgn = -1; sgn <= 1; sgn += 2) {
                        const int v = v0 + sgn * dvv;
                        if (v < 1 || v > kMaxVersion || (dvv == 0 && sgn == 1)) continue;
                        const int n = qr_size(v);
                        Affine A;
                        A.dx = {ux / (n - 7), uy / (n - 7)};
                        A.dy = {vx / (n - 7), vy / (n - 7)};
                        A.o = {tl.x - 3 * A.dx.x - 3 * A.dy.x, tl.y - 3 * A.dx.y - 3 * A.dy.y};
                        if (read_symbol(b, A, v, payload)) return true;
                    }
            }
    return false;
}

// ---------------------------------------------------------------------------
// AES (FIPS-197), CBC (SP 800-38A)
// ---------------------------------------------------------------------------
struct Aes {
    uint8_t sbox[256], inv[256];
    Aes()
    {
        uint8_t p = 1, q = 1;
        do {  // p * 3, q / 3 walk the multiplicative group
            p = p ^ (uint8_t)(p << 1) ^ (p & 0x80 ? 0x1B : 0);
            q ^= q << 1;
            q ^= q << 2;
            q ^= q << 4;
            if (q & 0x80) q ^= 0x09;
            const uint8_t x = q ^ rotl(q, 1) ^ rotl(q, 2) ^ rotl(q, 3) ^ rotl(q, 4);
            sbox[p] = x ^ 0x63;
        } while (p != 1);
        sbox[0] = 0x63;
        for (int i = 0; i < 256; ++i) inv[sbox[i]] = (uint8_t)i;
    }
    static uint8_t rotl(uint8_t x, int s) { return (uint8_t)((x << s) | (x >> (8 - s))); }
};
const Aes &aes_tables()
{
    static const Aes a;
    return a;
}

uint8_t xt(uint8_t x) { return (uint8_t)((x << 1) ^ (x & 0x80 ? 0x1B : 0)); }
uint8_t gmul(uint8_t a, uint8_t b)
{
    uint8_t r = 0;
    while (b) {
        if (b & 1) r ^= a;
        a = xt(a);
        b >>= 1;
    }
    return r;
}

// round keys: 4*(Nr+1) words as bytes
int expand_key(const uint8_t *key, int klen, uint8_t *rk)
{
    const int nk = klen / 4, nr = nk + 6;
    const Aes &T = aes_tables();
    std::memcpy(rk, key, klen);
    uint8_t rcon = 1;
    for (int i = nk; i < 4 * (nr + 1); ++i) {
        uint8_t t[4];
        std::memcpy(t, rk + 4 * (i - 1), 4);
        if (i % nk == 0) {
            const uint8_t t0 = t[0];
            t[0] = T.sbox[t[1]] ^ rcon;
            t[1] = T.sbox[t[2]];
            t[2] = T.sbox[t[3]];
            t[3] = T.sbox[t0];
            rcon = xt(rcon);
        } else if (nk > 6 && i % nk == 4) {
            for (int k = 0; k < 4; ++k) t[k] = T.sbox[t[k]];
        }
        for (int k = 0; k < 4; ++k) rk[4 * i + k] = rk[4 * (i - nk) + k] ^ t[k];
    }
    return nr;
}

void encrypt_block(const uint8_t *rk, int nr, const uint8_t *in, uint8_t *out)
{
    const Aes &T = aes_tables();
    uint8_t s[16];
    for (int i = 0; i < 16; ++i) s[i] = in[i] ^ rk[i];
    for (int r = 1; r <= nr; ++r) {
        uint8_t t[16];
        for (int i = 0; i < 16; ++i) t[i] = T.sbox[s[i]];
        for (int c = 0; c < 4; ++c)  // ShiftRows: row k of column c comes from column c + k
            for (int k = 0; k < 4; ++k) s[4 * c + k] = t[4 * ((c + k) % 4) + k];
        if (r != nr)
            for (int c = 0; c < 4; ++c) {
                uint8_t *a = s + 4 * c;
                const uint8_t a0 = a[0], a1 = a[1], a2 = a[2], a3 = a[3];
                a[0] = xt(a0) ^ (xt(a1) ^ a1) ^ a2 ^ a3;
                a[1] = a0 ^ xt(a1) ^ (xt(a2) ^ a2) ^ a3;
                a[2] = a0 ^ a1 ^ xt(a2) ^ (xt(a3) ^ a3);
                a[3] = (xt(a0) ^ a0) ^ a1 ^ a2 ^ xt(a3);
            }
        for (int i = 0; i < 16; ++i) s[i] ^= rk[16 * r + i];
    }
    std::memcpy(out, s, 16);
}

void decrypt_block(const uint8_t *rk, int nr, const uint8_t *in, uint8_t *out)
{
    const Aes &T = aes_tables();
    uint8_t s[16];
    for (int i = 0; i < 16; ++i) s[i] = in[i] ^ rk[16 * nr + i];
    for (int r = nr - 1; r >= 0; --r) {
        uint8_t t[16];
        for (int c = 0; c < 4; ++c)  // InvShiftRows
            for (int k = 0; k < 4; ++k) t[4 * ((c + k) % 4) + k] = s[4 * c + k];
        for (int i = 0; i < 16; ++i) s[i] = T.inv[t[i]] ^ rk[16 * r + i];
        if (r != 0)
            for (int c = 0; c < 4; ++c) {
                uint8_t *a = s + 4 * c;
                const uint8_t a0 = a[0], a1 = a[1], a2 = a[2], a3 = a[3];
                a[0] = gmul(a0, 14) ^ gmul(a1, 11) ^ gmul(a2, 13) ^ gmul(a3, 9);
                a[1] = gmul(a0, 9) ^ gmul(a1, 14) ^ gmul(a2, 11) ^ gmul(a3, 13);
                a[2] = gmul(a0, 13) ^ gmul(a1, 9) ^ gmul(a2, 14) ^ gmul(a3, 11);
                a[3] = gmul(a0, 11) ^ gmul(a1, 13) ^ gmul(a2, 9) ^ gmul(a3, 14);
            }
    }
    std::memcpy(out, s, 16);
}

int check_aes_args(const uint8_t *key, int32_t key_len, const uint8_t *iv, const uint8_t *in, int64_t len, const uint8_t *out)
{
    if (key_len != 16 && key_len != 24 && key_len != 32)
        return report(TMFWM_ERR_INVALID, "Incorrect AES key length (%d bytes)", key_len);
    if (!key || !iv || (len > 0 && (!in || !out))) return report(TMFWM_ERR_INVALID, "NULL pointer");
    if (len < 0 || len % 16) return report(TMFWM_ERR_INVALID, "Data must be padded to 16 byte boundary in CBC mode");
    return 0;
}

}  // namespace

extern "C" {

int tmfwm_qr_encode(const uint8_t *data, int32_t len, int32_t ec_level, int32_t min_version, int32_t mask, uint8_t *modules,
                    int32_t capacity, int32_t *size_out)
{
    tmf::clear_error();
    if (size_out) *size_out = 0;
    if (len < 0 || (len > 0 && !data) || !size_out) return report(TMFWM_ERR_INVALID, "bad arguments");
    if (ec_level < 0 || ec_level > 3) return report(TMFWM_ERR_INVALID, "error correction level %d (0 L, 1 M, 2 Q, 3 H)", ec_level);
    if (mask < -1 || mask > 7) return report(TMFWM_ERR_INVALID, "mask %d", mask);
    const int lv = kLevelBits[ec_level];
    const std::vector<Segment> segs = chunk_segments(data, len);
    int v = std::max(1, min_version);
    for (; v <= kMaxVersion; ++v)
        if (segment_bits(segs, v) <= 8 * data_codewords(v, lv)) break;
    if (v > kMaxVersion) return report(TMFWM_ERR_UNSUPPORTED, "%d bytes do not fit a version <= %d symbol", len, kMaxVersion);
    const int n = qr_size(v);
    *size_out = n;
    if (!modules || capacity < n * n) return report(TMFWM_ERR_INVALID, "modules buffer needs %d bytes", n * n);
    // data codewords: segments, terminator, byte alignment, pad bytes (python-qrcode create_data)
    const int ndata = data_codewords(v, lv);
    BitBuf bb;
    for (const Segment &sg : segs) put_segment(bb, sg, v);
    bb.put(0, std::min(4, ndata * 8 - bb.nbits));
    if (bb.nbits % 8) bb.put(0, 8 - bb.nbits % 8);
    for (int i = 0; (int)bb.bytes.size() < ndata; ++i) bb.put(i % 2 ? 0x11 : 0xEC, 8);
    // blocks, EC, interleaving
    const int *bl = kBlocks[v][lv];
    const int nblocks = bl[0] + bl[3], necc = bl[1] - bl[2];
    std::vector<std::vector<uint8_t>> dblk(nblocks), eblk(nblocks);
    int off = 0;
    for (int k = 0; k < nblocks; ++k) {
        const int dl = k < bl[0] ? bl[2] : bl[5];
        dblk[k].assign(bb.bytes.begin() + off, bb.bytes.begin() + off + dl);
        off += dl;
        eblk[k].resize(necc);
        rs_encode(dblk[k].data(), dl, necc, eblk[k].data());
    }
    std::vector<uint8_t> cw;
    const int maxd = std::max(bl[2], bl[5]);
    for (int i = 0; i < maxd; ++i)
        for (int k = 0; k < nblocks; ++k)
            if (i < (int)dblk[k].size()) cw.push_back(dblk[k][i]);
    for (int i = 0; i < necc; ++i)
        for (int k = 0; k < nblocks; ++k) cw.push_back(eblk[k][i]);
    // masks: scored as python-qrcode's best_mask_pattern does (makeImpl(test=True): format,
    // version and dark modules light), first minimum wins
    Grid base(v);
    const std::vector<int> ord = data_order(base);
    std::vector<uint8_t> reserved(n * n, 0);  // format / version / dark module cells
    {
        Grid probe(v);
        probe.put_format(0x7FFF);
        for (int i = 0; i < n * n; ++i) reserved[i] = probe.fn[i] && probe.m[i] != base.m[i];
        reserved[(n - 8) * n + 8] = 1;
        if (v >= 7)
            for (int i = 0; i < 18; ++i) {
                const int r = i / 3, c = n - 11 + i % 3;
                reserved[r * n + c] = reserved[c * n + r] = 1;
            }
    }
    int best_pen = 0, best_mask = 0;
    for (int mk = 0; mk < 8; ++mk) {
        if (mask >= 0 && mk != mask) continue;
        Grid g = base;
        fill_data(g, ord, cw, mk);
        for (int i = 0; i < n * n; ++i)
            if (reserved[i]) g.m[i] = 0;
        const int pen = penalty(g);
        if (mask >= 0 || mk == 0 || pen < best_pen) {
            best_pen = pen;
            best_mask = mk;
        }
    }
    Grid g = base;
    fill_data(g, ord, cw, best_mask);
    g.put_format(format_word(lv, best_mask));
    std::memcpy(modules, g.m.data(), (size_t)n * n);
    return 0;
}

int tmfwm_qr_decode(const uint8_t *gray, int32_t height, int32_t width, int64_t row_stride, uint8_t *out, int32_t capacity,
                    int32_t *len_out)
{
    tmf::clear_error();
    if (len_out) *len_out = 0;
    if (!gray || height <= 0 || width <= 0 || row_stride < width || !len_out)
        return report(TMFWM_ERR_INVALID, "bad image arguments");
    const int thr = otsu(gray, height, width, row_stride);
    Bin b{height, width, std::vector<uint8_t>((size_t)height * width)};
    for (int y = 0; y < height; ++y)
        for (int x = 0; x < width; ++x) b.d[(size_t)y * width + x] = gray[y * row_stride + x] <= thr;
    std::vector<uint8_t> payload;
    if (!decode_bin(b, payload)) return report(TMFWM_ERR_NODATA, "no decodable QR code in the %dx%d image", width, height);
    *len_out = (int32_t)payload.size();
    if (!out || capacity < (int32_t)payload.size()) return report(TMFWM_ERR_INVALID, "payload of %zu bytes exceeds the buffer", payload.size());
    std::memcpy(out, payload.data(), payload.size());
    return 0;
}

int tmfwm_qr_decode_batch(const uint8_t *tiles, int64_t n_tiles, int32_t height, int32_t width, uint8_t *out, int32_t capacity,
                          int32_t *lens)
{
    tmf::clear_error();
    if (n_tiles < 0 || !lens || (n_tiles > 0 && (!tiles || !out))) return report(TMFWM_ERR_INVALID, "bad arguments");
#pragma omp parallel for schedule(dynamic)
    for (int64_t i = 0; i < n_tiles; ++i) {
        int32_t len = 0;
        const int rc = tmfwm_qr_decode(tiles + i * (int64_t)height * width, height, width, width, out + i * capacity, capacity, &len);
        lens[i] = rc == 0 ? len : -1;
    }
    tmf::clear_error();
    return 0;
}

int tmfwm_aes_cbc_encrypt(const uint8_t *key, int32_t key_len, const uint8_t *iv, const uint8_t *in, int64_t len, uint8_t *out)
{
    tmf::clear_error();
    if (int rc = check_aes_args(key, key_len, iv, in, len, out)) return rc;
    uint8_t rk[240], prev[16];
    const int nr = expand_key(key, key_len, rk);
    std::memcpy(prev, iv, 16);
    for (int64_t o = 0; o < len; o += 16) {
        uint8_t x[16];
        for (int i = 0; i < 16; ++i) x[i] = in[o + i] ^ prev[i];
        encrypt_block(rk, nr, x, out + o);
        std::memcpy(prev, out + o, 16);
    }
    return 0;
}

int tmfwm_aes_cbc_decrypt(const uint8_t *key, int32_t key_len, const uint8_t *iv, const uint8_t *in, int64_t len, uint8_t *out)
{
    tmf::clear_error();
    if (int rc = check_aes_args(key, key_len, iv, in, len, out)) return rc;
    uint8_t rk[240], prev[16], cur[16];
    const int nr = expand_key(key, key_len, rk);
    std::memcpy(prev, iv, 16);
    for (int64_t o = 0; o < len; o += 16) {
        std::memcpy(cur, in + o, 16);  // in and out may be the same buffer
        decrypt_block(rk, nr, cur, out + o);
        for (int i = 0; i < 16; ++i) out[o + i] ^= prev[i];
        std::memcpy(prev, cur, 16);
    }
    return 0;
}

}  // extern "C"
