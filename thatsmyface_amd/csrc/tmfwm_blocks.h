// Shared device code of the watermark kernels (gfx950): byte-row I/O, the LDS-mediated
// 2-D transforms and the fused embed kernel template.  Included by tmfwm_kernels.hip
// (every other instantiation, the extract kernels and the launchers) and by
// tmfwm_embed8.hip, which instantiates embed_kernel<8> -- the benchmark's kernel -- in a
// TU of its own so that it can be scheduled for ILP (Makefile) without the register
// growth that scheduler costs the other block sizes.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "tmfwm_device.h"
#include "tmfwm_internal.h"

namespace tmf {

// Opt-in phase profile (make stamps): per-wave s_memtime deltas summed per phase.
#ifdef TMF_STAMPS
__device__ unsigned long long g_stamps[16];
struct Stamp {
    unsigned long long *t;
    TMF_DEVI void operator()(int k) const
    {
        const unsigned long long now = __builtin_amdgcn_s_memtime();
        if ((threadIdx.x & 63) == 0 && (blockIdx.x & 63) == 0) atomicAdd(&g_stamps[k], now - *t);  // 1/64 of the waves
        *t = now;
    }
};
#define TMF_STAMP_INIT unsigned long long tmf_t0 = __builtin_amdgcn_s_memtime(); const Stamp stamp{&tmf_t0}
#else
using Stamp = NoStamp;
#define TMF_STAMP_INIT const Stamp stamp{}
#endif

// Lanes per block L (== oracle jac_chunks): a power of two for the DPP butterflies,
// with R = ceil(B/L) rows per lane (rows past B are zero padding).
template <int B>
struct Geo {
    static constexpr int L = B == 4 ? 1 : B <= 8 ? 2 : B <= 12 ? 4 : 8;
    static constexpr int R = kRows<B, L>;          // rows per lane
    static constexpr int BPW = 64 / L;             // blocks per wave
    static constexpr int NBYTES = B * 3;           // bytes per pixel row of a block
    static constexpr int NW = (NBYTES + 3) / 4;    // u32 words holding them
    static constexpr bool WORDS = NBYTES % 4 == 0; // dword I/O possible (b = 4, 8, 12, 16)
};
static_assert(Geo<6>::L == 2 && Geo<10>::L == 4 && Geo<14>::L == 8 && Geo<14>::R == 2, "lane layout");

// ---- byte rows: dword I/O when the row segment is whole dwords and aligned,
// otherwise bytes (b = 6, 10, 14: 18, 30, 42 bytes per row)
template <int B>
TMF_DEVI void load_words(const uint8_t *p, bool aligned, uint32_t (&w)[Geo<B>::NW])
{
    constexpr int NW = Geo<B>::NW, NB = Geo<B>::NBYTES;
    if (Geo<B>::WORDS && aligned) {
        const uint32_t *q = reinterpret_cast<const uint32_t *>(p);
#pragma unroll
        for (int i = 0; i < NW; ++i) w[i] = q[i];
    } else {
#pragma unroll
        for (int i = 0; i < NW; ++i) {
            uint32_t v = 0;
#pragma unroll
            for (int k = 0; k < 4; ++k)
                if (4 * i + k < NB) v |= (uint32_t)p[4 * i + k] << (8 * k);
            w[i] = v;
        }
    }
}

template <int B>
TMF_DEVI void store_words(uint8_t *p, bool aligned, const uint32_t (&w)[Geo<B>::NW])
{
    constexpr int NW = Geo<B>::NW, NB = Geo<B>::NBYTES;
    if (Geo<B>::WORDS && aligned) {
        uint32_t *q = reinterpret_cast<uint32_t *>(p);
#pragma unroll
        for (int i = 0; i < NW; ++i) q[i] = w[i];
    } else {
#pragma unroll
        for (int i = 0; i < NW; ++i)
#pragma unroll
            for (int k = 0; k < 4; ++k)
                if (4 * i + k < NB) p[4 * i + k] = (uint8_t)(w[i] >> (8 * k));
    }
}

TMF_DEVI uint32_t byte_at(const uint32_t *w, int k) { return (w[k >> 2] >> (8 * (k & 3))) & 0xFFu; }

// ---- LDS-mediated 2-D transforms on a block held in rows layout ---------------
// tile: this block's [B][B+1] LDS region.  x: this lane's R rows.  Column pass
// first (axis 0), then rows (watermarking.py:76-83).
template <int B>
TMF_DEVI bool real_row(int q, int r) { return Geo<B>::R * Geo<B>::L == B || q * Geo<B>::R + r < B; }

template <int B, bool INVERSE>
TMF_DEVI void dct2d_rows_layout(float (&x)[Geo<B>::R][B], float *tile, int q)
{
    constexpr int R = Geo<B>::R, LD = B + 1;
#pragma unroll
    for (int r = 0; r < R; ++r)
        if (real_row<B>(q, r))
#pragma unroll
            for (int c = 0; c < B; ++c) tile[(q * R + r) * LD + c] = x[r][c];
    __syncthreads();
    // column pass: this lane takes columns [q*R, q*R+R) that exist
#pragma unroll
    for (int cc = 0; cc < R; ++cc) {
        if (!real_row<B>(q, cc)) continue;
        float col[B];
#pragma unroll
        for (int r = 0; r < B; ++r) col[r] = tile[r * LD + q * R + cc];
        if constexpr (INVERSE) dct::dct3<B>(col); else dct::dct2<B>(col);
#pragma unroll
        for (int r = 0; r < B; ++r) tile[r * LD + q * R + cc] = col[r];
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < R; ++r) {
        float row[B];
#pragma unroll
        for (int c = 0; c < B; ++c) row[c] = real_row<B>(q, r) ? tile[(q * R + r) * LD + c] : 0.0f;
        if constexpr (INVERSE) dct::dct3<B>(row); else dct::dct2<B>(row);
#pragma unroll
        for (int c = 0; c < B; ++c) x[r][c] = real_row<B>(q, r) ? row[c] : 0.0f;
    }
    __syncthreads();
}

// The same 2-D IDCT on intervals: lower ends through `tl`, upper ends through
// `th` (both [B][B+1] tiles of this block), every pass on Ivf end points.
template <int B>
TMF_DEVI void idct2d_rows_layout_iv(float (&xl)[Geo<B>::R][B], float (&xh)[Geo<B>::R][B], float *tl, float *th, int q)
{
    constexpr int R = Geo<B>::R, LD = B + 1;
#pragma unroll
    for (int r = 0; r < R; ++r)
        if (real_row<B>(q, r))
#pragma unroll
            for (int c = 0; c < B; ++c) {
                tl[(q * R + r) * LD + c] = xl[r][c];
                th[(q * R + r) * LD + c] = xh[r][c];
            }
    __syncthreads();
#pragma unroll
    for (int cc = 0; cc < R; ++cc) {
        if (!real_row<B>(q, cc)) continue;
        Ivf col[B];
#pragma unroll
        for (int r = 0; r < B; ++r) col[r] = {tl[r * LD + q * R + cc], th[r * LD + q * R + cc]};
        dct::dct3<B>(col);
#pragma unroll
        for (int r = 0; r < B; ++r) {
            tl[r * LD + q * R + cc] = col[r].lo;
            th[r * LD + q * R + cc] = col[r].hi;
        }
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < R; ++r) {
        Ivf row[B];
#pragma unroll
        for (int c = 0; c < B; ++c)
            row[c] = real_row<B>(q, r) ? Ivf{tl[(q * R + r) * LD + c], th[(q * R + r) * LD + c]} : Ivf{0.0f, 0.0f};
        dct::dct3<B>(row);
#pragma unroll
        for (int c = 0; c < B; ++c) {
            xl[r][c] = real_row<B>(q, r) ? row[c].lo : 0.0f;
            xh[r][c] = real_row<B>(q, r) ? row[c].hi : 0.0f;
        }
    }
    __syncthreads();
}

struct StripPos {
    int64_t frame;
    int bi, bj;
    bool valid;
};

template <int B>
TMF_DEVI StripPos strip_pos(int strips_per_row, int nbw)
{
    StripPos p;
    const int strip = blockIdx.x % strips_per_row;
    p.bi = blockIdx.x / strips_per_row;
    p.frame = blockIdx.y;
    const int g = (threadIdx.x & 63) / Geo<B>::L;
    p.bj = strip * Geo<B>::BPW + g;
    p.valid = p.bj < nbw;
    return p;
}

// Load this lane's R pixel rows of its block (garbage-free zeros for blocks past
// the right edge of the block grid) and return luma rows.
template <int B>
TMF_DEVI void load_block_rows(const uint8_t *frame_base, int W, const StripPos &pos, int q, bool aligned,
                              uint32_t (&words)[Geo<B>::R][Geo<B>::NW])
{
    constexpr int R = Geo<B>::R;
#pragma unroll
    for (int r = 0; r < R; ++r) {
        if (pos.valid && real_row<B>(q, r)) {
            const uint8_t *p = frame_base + ((int64_t)(pos.bi * B + q * R + r) * W + (int64_t)pos.bj * B) * 3;
            load_words<B>(p, aligned, words[r]);
        } else {
#pragma unroll
            for (int i = 0; i < Geo<B>::NW; ++i) words[r][i] = 0u;
        }
    }
}

template <int B>
TMF_DEVI void luma_rows(const uint32_t (&words)[Geo<B>::R][Geo<B>::NW], float (&y)[Geo<B>::R][B])
{
#pragma unroll
    for (int r = 0; r < Geo<B>::R; ++r)
#pragma unroll
        for (int c = 0; c < B; ++c) {
            const uint32_t R8 = byte_at(words[r], 3 * c), G8 = byte_at(words[r], 3 * c + 1), B8 = byte_at(words[r], 3 * c + 2);
            y[r][c] = luma(R8, G8, B8);
        }
}

// ---------------------------------------------------------------------------
// Embed: watermarking.py:163-216 fused, one launch per batch.
// ---------------------------------------------------------------------------
// Waves per SIMD the register allocation must allow (1 = unconstrained: with the byte
// certificate's second end points the compiler overflows into AGPRs at b >= 8 and runs one
// wave per SIMD).  Forcing 2 is faster even where it costs scratch (round 4, before the
// certificate: embed<12> 283 -> 201 us, embed<16> 531 -> 345 us per 4K frame).
template <int B>
constexpr int kEmbedWaves = (B == 8 || B == 10 || B == 12 || B == 14 || B == 16) ? 2 : 1;

// Strip pass: once at most kDeferMax blocks of a wave still need f64 sweeps after a sweep
// and its Newton try, the wave leaves them to the list pass instead of running another
// sweep for them (they write nothing here; the list pass redoes them from their pixels with
// the whole loop).  On noise covers at b = 8, 1 % of blocks need a second sweep and 26 % of
// waves would run one for them; on photo-like covers nearly every block needs two, and the
// waves keep going as before.
template <int B>
constexpr int kDeferMax = B == 8 ? 4 : 0;

// b = 16 parks D in LDS during phase 1 (svd3, PARK): frees 32 VGPRs (scratch 264 -> 216 B
// per lane); at b = 10 / 14 the allocation without it fits 2 waves per SIMD spill-free and
// with it does not, at b = 12 it gains nothing
template <int B>
constexpr bool kParkD = B == 16;
// per-block LDS tile stride (floats): the [B][B+1] transpose tile, or svd3's scratch if larger
// (8-lane blocks: the Newton table past the norms / partials; b = 16: the parked D past
// phase 1's parameter slots), even for 8-byte alignment
template <int B>
constexpr int kEmbedTS0 = B * (B + 1) > kScratchFloats<B, Geo<B>::L> ? B * (B + 1) : kScratchFloats<B, Geo<B>::L>;
template <int B>
constexpr int kEmbedTS1 = ((kParkD<B> && kParkOff<Geo<B>::L> + B * B > kEmbedTS0<B> ? kParkOff<Geo<B>::L> + B * B : kEmbedTS0<B>) + 1) & ~1;
// Bank spreading for the reconstruction's LDS reads (ds_read_b32: bank = dword address mod 32
// over each 32-lane half): at b = 8 a half holds 16 blocks, at b = 16 four, and each lane reads
// its block's lower-end or upper-end tile.  Tile strides 73 (b = 8: 9 g mod 32, distinct over
// 16 blocks) and 344 (b = 16: 24 g mod 32; the scratch it must hold rounded up to that) in both regions, with the upper-end region kHiPad dwords
// further on (16 / 4), put every (block, end) of a half on a bank of its own; with strides 72
// and 72 (b = 16: 312 and 272) four (two) of them shared one, and bank conflicts were 75 % of
// embed<8>'s LDS cycles (profiles/r05/r05h).
template <int B>
constexpr int kEmbedTS = B == 8 ? 73 : B == 16 ? kEmbedTS1<B> + ((24 - kEmbedTS1<B> % 32) + 32) % 32 : kEmbedTS1<B>;
static_assert(kEmbedTS<8> >= kEmbedTS1<8> && kEmbedTS<16> % 32 == 24, "tile strides");

// Byte certificate of the hybrid route (oracle tmfwm_cert.cpp): LAPACK's f64
// factors lie within E_k = kCertScale s1 / g_k of the Jacobi route's, every singular value
// within kCertScale s1 (K = 256 units of 2^-53 s1 / g_k; LAPACK's own V is off by up to 94,
// the Jacobi route's by up to 30, tools/exp/cert_study.py).
constexpr double kCertScale = 0x1p-45;

// LDS of one wave: `lds` holds each block's [B][B+1] transpose tile (or svd3's scratch if
// larger); `lds2` first parks this lane's source bytes during the SVD, then holds the
// certificate's upper-end tiles ([B][B+1] floats per block)
template <int B>
constexpr int kPixWords = Geo<B>::R * Geo<B>::NW * 64;
template <int B>
constexpr int kHiTile = B == 8 || B == 16 ? kEmbedTS<B> : B * (B + 1);
template <int B>
constexpr int kHiPad = B == 8 ? 16 : B == 16 ? 4 : 0;
template <int B>
constexpr int kLds2Floats = kPixWords<B> > Geo<B>::BPW * kHiTile<B> ? kPixWords<B> : Geo<B>::BPW * kHiTile<B>;

// The reconstruction picks each row's b end by an LDS offset (b = 8, 16) or by value selects
// (the other sizes, where the offset form costs registers)
template <int B>
constexpr bool kOffsetPick = B == 8 || B == 16;

// b = 16 reads its source bytes again from global memory (L2) for the colour phase instead of
// parking them in LDS and carrying them through the certificate in registers: spilled VGPRs
// 27 -> 8, embed<16> -1 % per 4K frame; at b = 8 it is slower (+1.5 % on noise covers,
// profiles/r05/r05q_ab.log)
template <int B>
constexpr bool kReloadBytes = B == 16;

// b = 10 / 14 keep the reconstruction's fma chains in their (k-outer) source order: left free,
// the compiler regroups them per output element and spills every element of Bm it reads
// ahead of its use (272 / 282 VGPRs spilled -> 0 / 5; embed<14> 613 -> 360 us per 4K frame,
// embed<10> 271 -> 247).  At b = 8 / 16 the free schedule is faster (128 vs 139 us, 334 vs 364).
template <int B>
constexpr bool kPinChain = B == 10 || B == 14;

// One wave's blocks: strip mode (LIST = false: the strip of blockIdx) or list mode (pos and
// id from the slow list).  id = (frame * nbh + bi) * nbw + bj, relative to a.src.
template <int B, bool LIST>
TMF_DEVI void embed_blocks(const EmbedArgs &a, const StripPos &pos, uint32_t id, float *lds, float *lds2)
{
    constexpr int L = Geo<B>::L, R = Geo<B>::R, LD = B + 1, NW = Geo<B>::NW, TS = kEmbedTS<B>;
    constexpr bool kPark = kParkD<B>;
    const int lane = threadIdx.x & 63, g = lane / L, q = lane % L;
    float *tile = lds + g * TS;
    float *tile2 = lds2 + g * kHiTile<B>;
    uint32_t (*pix)[64] = reinterpret_cast<uint32_t (*)[64]>(lds2);
    const uint8_t *src = a.src + pos.frame * a.frame_stride;
    uint8_t *dst = a.dst + pos.frame * a.frame_stride;

    TMF_STAMP_INIT;
    float x[R][B];
    {
        uint32_t words[R][NW];
        load_block_rows<B>(src, a.W, pos, q, a.aligned, words);
        luma_rows<B>(words, x);
        if constexpr (!kReloadBytes<B>) {
#pragma unroll
            for (int r = 0; r < R; ++r)
#pragma unroll
                for (int i = 0; i < NW; ++i) pix[r * NW + i][lane] = words[r][i];
        }
    }
    dct2d_rows_layout<B, false>(x, tile, q);  // :192
    stamp(0);
    // a flat block (D zero but for D[0][0]) has the same factors on both routes (oracle tmfwm_cert.cpp)
    int ac = 0;
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
        for (int c = 0; c < B; ++c)
            if (r > 0 || c > 0 || q > 0) ac |= x[r][c] != 0.0f ? 1 : 0;
    const bool flat = group_or<L>(ac) == 0;

    double A[R][B], V[R][B];
    // :195 (SVD); svd3's scratch and (b = 16) the parked D in the block's tile
    static_assert(!kPark || kParkOff<L> + B * B <= TS, "parked D fits the tile");
    bool slow = false;  // strip pass: this block was left to the list pass
    svd3<B, L, kPark>(x, A, V, q, stamp, tile, tile + kParkOff<L>, !LIST && a.slow_list ? kDeferMax<B> : 0, &slow);
    if (slow && pos.valid && q == 0) {
        const uint32_t row = blockIdx.y * (uint32_t)a.nbh + (uint32_t)pos.bi, s = row % kListShards;
        a.slow_list[shard_base(s, (uint32_t)a.nframes * (uint32_t)a.nbh, (uint32_t)a.nbw) +
                    atomicAdd(a.slow_shards + s * kShardStride, 1u)] = id;
    }
    // this lane's source bytes back to registers (b = 16: from global memory at the colour
    // phase instead): their LDS becomes the upper-end tiles
    uint32_t words[R][NW];
    if constexpr (!kReloadBytes<B>) {
#pragma unroll
        for (int r = 0; r < R; ++r)
#pragma unroll
            for (int i = 0; i < NW; ++i) words[r][i] = pix[r * NW + i][lane];
    }
    __syncthreads();

    // singular values (oracle orc_svd_block: sigma_k = |a_k|, u_k = a_k / sigma_k)
    double sig[B];
#pragma unroll
    for (int k = 0; k < B; ++k) sig[k] = cdot_part<R, B>(A, k, k);
#pragma unroll
    for (int k = 0; k < B; ++k) sig[k] = __builtin_sqrt(group_sum<L>(sig[k]));
    // Conditioning test (oracle orc_svd_flag): m = min over triplets reaching the
    // output (f32(sigma_k) != 0) of g_k = min(sigma_k, distance to the nearest other sigma); the
    // block takes the dgesdd route iff m * 2^20 < sigma_1.  (Per-k minima first: folding every
    // pair into one running minimum is the same value but a 36-deep dependent chain, +1.5 % on
    // embed<8>, profiles/r03/r03r.)
    double gk[B], s1 = 0.0;
#pragma unroll
    for (int k = 0; k < B; ++k) {
        gk[k] = sig[k];
        s1 = sig[k] > s1 ? sig[k] : s1;
    }
#pragma unroll
    for (int k = 0; k < B; ++k)
#pragma unroll
        for (int j = k + 1; j < B; ++j) {
            const double d = __builtin_fabs(sig[k] - sig[j]);
            gk[k] = d < gk[k] ? d : gk[k];
            gk[j] = d < gk[j] ? d : gk[j];
        }
    double m = s1;
#pragma unroll
    for (int k = 0; k < B; ++k) m = ((float)sig[k] != 0.0f && gk[k] < m) ? gk[k] : m;
    const bool zero = s1 == 0.0;  // N6: D == 0 -> U = I, Vt = I on both routes
    const bool flag20 = m * 1048576.0 < s1;
    // Byte certificate: the interval bounds of the blocks whose bytes it decides (zero,
    // flagged and deferred blocks keep point intervals: the point path's values)
    const bool cert = !zero && !flat && !flag20 && !slow;
    const double tE = cert ? kCertScale * s1 : 0.0;
    // E_k = f32(tE / g_k): in [2^-45, 2^-25] for a certified block (g_k >= 2^-20 s1), held as a float
    float E[B];
#pragma unroll
    for (int k = 0; k < B; ++k) E[k] = cert && (float)sig[k] != 0.0f ? (float)(tE / gk[k]) : 0.0f;
    // Sort descending (oracle: odd-even transposition sort, stable) as ranks: k goes to
    // position rk[k] = #{j < k: sig[j] >= sig[k]} + #{j > k: sig[j] > sig[k]}.  The
    // permutation is applied through LDS: U's columns here, Vt's rows with the B store.
    int rk[B];
#pragma unroll
    for (int k = 0; k < B; ++k) rk[k] = 0;
#pragma unroll
    for (int k = 1; k < B; ++k)
#pragma unroll
        for (int j = 0; j < k; ++j) {
            const int ge = sig[j] >= sig[k] ? 1 : 0;
            rk[k] += ge;
            rk[j] += 1 - ge;
        }
    // U = A / sigma as f32 intervals [f32(u - E), f32(u + E)]; triplets that do not reach the
    // output (f32(sigma) == 0) take U = [2, 2] against B = [-2 S', 2 S'] (|f32 entries| <= 1)
    // over this lane's rows of the triplets that reach the output: an interval that contains 0,
    // an interval that is not a point
    int str = 0, wid = 0;
#pragma unroll
    for (int k = 0; k < B; ++k) {
        const double inv = 1.0 / sig[k];
#pragma unroll
        for (int r = 0; r < R; ++r) {
            // branch-free (selects): the three cases are lane-divergent
            const double u = A[r][k] * inv;
            float ul = (float)(u - (double)E[k]), uh = (float)(u + (double)E[k]);
            const float id = (q * R + r == k) ? 1.0f : 0.0f;
            const bool out = (float)sig[k] != 0.0f;  // the triplet reaches the output
            ul = zero ? id : out ? ul : 2.0f;
            uh = zero ? id : out ? uh : 2.0f;

            if (real_row<B>(q, r)) {
                tile[(q * R + r) * LD + rk[k]] = ul;
                tile2[(q * R + r) * LD + rk[k]] = uh;
            }
        }
    }
    __syncthreads();
    float Ul[R][B], Uh[R][B];
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
        for (int t = 0; t < B; ++t) {
            Ul[r][t] = real_row<B>(q, r) ? tile[(q * R + r) * LD + t] : 0.0f;
            Uh[r][t] = real_row<B>(q, r) ? tile2[(q * R + r) * LD + t] : 0.0f;
            str |= (int)(Ul[r][t] < 0.0f) & (int)(Uh[r][t] > 0.0f);
            wid |= (int)(Ul[r][t] != Uh[r][t]);
        }
    __syncthreads();

    // N7 blend (:198): S[0] = f32(f64(S[0]) + alpha * (w / 255.0)), S[0] the largest; as
    // intervals [f32(max(sigma - Es, 0)), f32(sigma + Es)] blended at both ends
    const uint32_t wv = pos.valid ? a.wm[(int64_t)pos.bi * a.nbw + pos.bj] : 0u;
    const double cw = a.alpha * ((double)wv / 255.0);
    float Sl[B], Sh[B];
    bool neg = false;  // alpha < 0 pushing S'[0] below zero: outside the certificate's S' >= 0
#pragma unroll
    for (int k = 0; k < B; ++k) {
        const double lo = sig[k] - tE;
        Sl[k] = (float)(lo > 0.0 ? lo : 0.0);
        Sh[k] = (float)(sig[k] + tE);
        const bool top = rk[k] == 0;
        const float bl0 = (float)((double)Sl[k] + cw), bh0 = (float)((double)Sh[k] + cw);
        Sl[k] = top ? bl0 : Sl[k];
        Sh[k] = top ? bh0 : Sh[k];
        neg = neg || (top && !(bl0 >= 0.0f));
    }
    // N8 (:201): Bm[t][j] = S'[t] * Vt[t][j] (this lane's rows j of V, row t = rank), then M = U @ Bm,
    // both ends (S' >= 0: the lower end is S'lo v if v >= 0, else S'hi v; the upper alike)
#pragma unroll
    for (int k = 0; k < B; ++k) {
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const float vl = (float)(V[r][k] - (double)E[k]), vh = (float)(V[r][k] + (double)E[k]);
            float bl = vl >= 0.0f ? Sl[k] * vl : Sh[k] * vl;
            float bh = vh <= 0.0f ? Sl[k] * vh : Sh[k] * vh;
            const float bid = Sl[k] * ((q * R + r == k) ? 1.0f : 0.0f);
            const bool out = (float)sig[k] != 0.0f;
            bl = zero ? bid : out ? bl : -2.0f * Sh[k];
            bh = zero ? bid : out ? bh : 2.0f * Sh[k];
            if (real_row<B>(q, r)) {
                str |= (int)(zero || (float)sig[k] != 0.0f) & (int)(bl < 0.0f) & (int)(bh > 0.0f);
                wid |= (int)(bl != bh);
                tile[rk[k] * LD + q * R + r] = bl;
                tile2[rk[k] * LD + q * R + r] = bh;
            }
        }
    }
    __syncthreads();
    // k outermost: each element of Bm is read from LDS once and used by this lane's R rows at
    // once (row by row, the compiler hoisted all b^2 reads across the rows and spilled them,
    // profiles/r04/r04b).  Every M[r][j] is the fma chain over k = 0..b-1; on intervals, the
    // lower end takes the corner of the smallest product: u's lower end if b >= 0, else its
    // upper one, and b's lower end if u >= 0, else its upper one (exact when neither interval
    // contains 0, or one of them is a point; blocks where neither holds take the dgesdd route).
    float Ml[R][B], Mh[R][B];
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
        for (int j = 0; j < B; ++j) Ml[r][j] = Mh[r][j] = 0.0f;
    // The end-point selection is exact unless some rank has an interval containing 0 on one side of
    // the product and a non-point interval on the other (exact zeros of structured blocks); a block
    // with an interval containing 0 and a non-point interval anywhere goes to the dgesdd route
    // (oracle tmfwm_cert.cpp: the same block-level test)
    const bool mixed = (group_or<L>(str) & group_or<L>(wid)) != 0;
    // b's end for each row comes from the LDS tile the row's u sign picks (an offset select per
    // row and rank instead of a value select per element; both tiles live in one LDS array)
    const int dt = (int)(tile2 - tile);
    if constexpr (kOffsetPick<B>) {
#pragma unroll
    for (int k = 0; k < B; ++k) {
        int ol[R], oh[R];
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const bool up = Ul[r][k] >= 0.0f;
            ol[r] = up ? 0 : dt;
            oh[r] = up ? dt : 0;
        }
#pragma unroll
        for (int j = 0; j < B; ++j) {
            const bool bp = tile[k * LD + j] >= 0.0f;
#pragma unroll
            for (int r = 0; r < R; ++r) {
                Ml[r][j] = __builtin_fmaf(bp ? Ul[r][k] : Uh[r][k], tile[ol[r] + k * LD + j], Ml[r][j]);
                Mh[r][j] = __builtin_fmaf(bp ? Uh[r][k] : Ul[r][k], tile[oh[r] + k * LD + j], Mh[r][j]);
                if constexpr (kPinChain<B>) pin_order(Ml[r][j], Mh[r][j]);
            }
        }
    }
    } else {
#pragma unroll
        for (int k = 0; k < B; ++k)
#pragma unroll
            for (int j = 0; j < B; ++j) {
                lds_order();  // one element of Bm at a time (hoisting them spills at b = 10..14)
                const float bl = tile[k * LD + j], bh = tile2[k * LD + j];
                const bool bp = bl >= 0.0f;
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    const bool up = Ul[r][k] >= 0.0f;
                    Ml[r][j] = __builtin_fmaf(bp ? Ul[r][k] : Uh[r][k], up ? bl : bh, Ml[r][j]);
                    Mh[r][j] = __builtin_fmaf(bp ? Uh[r][k] : Ul[r][k], up ? bh : bl, Mh[r][j]);
                    if constexpr (kPinChain<B>) pin_order(Ml[r][j], Mh[r][j]);
                }
            }
    }
    __syncthreads();
    stamp(4);
    idct2d_rows_layout_iv<B>(Ml, Mh, tile, tile2, q);  // :204
    stamp(5);

    // :207-216 write back and ycbcr_to_rgb with this lane's original chroma: the lower ends'
    // bytes; a pixel whose ends give other bytes leaves the block undecided
    bool unc = neg;
    if (pos.valid && !slow) {
        if constexpr (kReloadBytes<B>) load_block_rows<B>(src, a.W, pos, q, a.aligned, words);
#pragma unroll
        for (int r = 0; r < R; ++r) {
            uint32_t out[Geo<B>::NW];
#pragma unroll
            for (int i = 0; i < Geo<B>::NW; ++i) out[i] = 0u;
#pragma unroll
            for (int c = 0; c < B; ++c) {
                float cbs, crs;
                const uint32_t R0 = byte_at(words[r], 3 * c), G0 = byte_at(words[r], 3 * c + 1), B0 = byte_at(words[r], 3 * c + 2);
                chroma(R0, G0, B0, cbs, crs);
                uint32_t R8, G8, B8;
                float fr;
                colour_inv_frac(Ml[r][c], cbs, crs, R8, G8, B8, fr);
                // Every channel is monotone in Y, and from Y's lower end to its upper end each
                // scaled value p = f32(clip(v) * 255) grows by at most 255 dY + 255 * 2^-24 +
                // 2^-16 (v's f32 rounding on [0, 1], then p's) < 255.1 dY + 2^-14, dY = f32(Yh -
                // Yl); so the bytes cannot differ unless frac(p) + that reaches 1, and only then
                // are the upper end's bytes computed
                const float dy = Mh[r][c] - Ml[r][c];
                const bool wide = dy != 0.0f && fr + __builtin_fmaf(dy, 255.1f, 0x1p-14f) >= 1.0f;
                if (__builtin_amdgcn_ballot_w64(wide) != 0 && wide) {
                    uint32_t R9, G9, B9;
                    colour_inv(Mh[r][c], cbs, crs, R9, G9, B9);
                    unc = unc || R9 != R8 || G9 != G8 || B9 != B8;
                }
                const int k0 = 3 * c;
                out[k0 >> 2] |= R8 << (8 * (k0 & 3));
                out[(k0 + 1) >> 2] |= G8 << (8 * ((k0 + 1) & 3));
                out[(k0 + 2) >> 2] |= B8 << (8 * ((k0 + 2) & 3));
            }
            uint8_t *p = dst + ((int64_t)(pos.bi * B + q * R + r) * a.W + (int64_t)pos.bj * B) * 3;
            if (real_row<B>(q, r)) store_words<B>(p, a.aligned, out);
        }
    }
    // the dgesdd route (embed_fixup_kernel) redoes flagged blocks and blocks with an undecided byte
    const bool fix = flag20 || (cert && mixed) || group_or<L>(unc && cert ? 1 : 0) != 0;
    if (fix && pos.valid && !slow && q == 0) a.fb_list[atomicAdd(a.fb_count, 1u)] = id;
    stamp(6);
}

template <int B, bool LIST = false>
__global__ __launch_bounds__(64, kEmbedWaves<B>) void embed_kernel(EmbedArgs a)
{
    constexpr int L = Geo<B>::L, BPW = Geo<B>::BPW, TS = kEmbedTS<B>;
    // the transpose tiles (also svd3's scratch during the SVD), then the source bytes / the
    // upper-end tiles, in one array (the reconstruction picks a tile by an offset)
    __shared__ __attribute__((aligned(16))) float lds_all[BPW * TS + kHiPad<B> + kLds2Floats<B>];
    float *lds = lds_all, *lds2 = lds_all + BPW * TS + kHiPad<B>;
    if constexpr (LIST) {
        // grid-stride over the slow list's segments (their lengths are known on the device only)
        const uint32_t per_frame = (uint32_t)a.nbh * (uint32_t)a.nbw, rows = (uint32_t)a.nframes * (uint32_t)a.nbh;
        const int g = (threadIdx.x & 63) / L;
        for (uint32_t s = blockIdx.x; s < kListShards; s += gridDim.x) {
            const uint32_t n = a.slow_shards[s * kShardStride], base = shard_base(s, rows, (uint32_t)a.nbw);
            if (n != 0 && (threadIdx.x & 63) == 0) atomicAdd(a.slow_count, n);
            for (uint32_t t0 = 0; t0 < n; t0 += BPW) {
                StripPos pos;
                pos.valid = t0 + g < n;
                const uint32_t id = pos.valid ? a.slow_list[base + t0 + g] : 0u;
                pos.frame = id / per_frame;
                const uint32_t rem = id % per_frame;
                pos.bi = (int)(rem / (uint32_t)a.nbw);
                pos.bj = (int)(rem % (uint32_t)a.nbw);
                embed_blocks<B, true>(a, pos, id, lds, lds2);
                __syncthreads();  // the LDS tiles are reused by the next listed blocks
            }
        }
    } else {
        const StripPos pos = strip_pos<B>(a.strips_per_row, a.nbw);
        const uint32_t id = (uint32_t)(((int64_t)blockIdx.y * a.nbh + pos.bi) * a.nbw + pos.bj);
        embed_blocks<B, false>(a, pos, id, lds, lds2);
    }
}

}  // namespace tmf
