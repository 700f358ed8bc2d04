// The rank-1 pre-pass of the hybrid route (TMFWM_ROUTE_RANK1, round 6): photo mode.
//
// The reference reconstructs every block from all of LAPACK's factors rounded to f32
// (watermarking.py:195-201), but only S[0] changes, so its M_ref = fl(U32 fl(S'32 Vt32)) is
// D + c u1 v1^T up to rounding (c = alpha w / 255).  This pass computes, per block, the top
// singular pair (u, v) by an f64 power iteration with an a-posteriori bound, M_fast =
// f32(D + c u v^T), Y_fast = IDCT_fl(M_fast), and a per-pixel bound eps_Y >= |Y_ref - Y_fast|:
//   dM_ij <= alpha' G_ij + beta' P_ij + gamma'      (tools/exp/fastpath_study.py, round 4)
//     G_ij = |D_i,:|^(1/2) |D_:,j|^(1/2) bounds sum_t |U_it| s_t |V_jt| (Cauchy-Schwarz: the rows of
//       U and V are unit vectors), P_ij = (|u_i| + e)(|v_j| + e) bounds |u1_i| |v1_j| of LAPACK's top
//       pair (e = eps_uv, below), alpha' = 1.01 (b + 6) 2^-24 (the b fmaf roundings of the chain,
//       the 4 factor roundings, f32(M_fast)), beta' = 1.01 ((b + 6) 2^-24 |c| + 2^-23 (s1 + |c|))
//       (S[0]'s and S'[0]'s f32 roundings), gamma' = 2^-40 s1 (LAPACK's residual |U S V^T - D|,
//       8192 units of 2^-53 s1, 84 times the worst measured) + |c| e (2 + e);
//   eps_Y = |C'| dM |C'|^T + 2 (u (E Mb |C'|^T + |C'| Mb E^T) + u^2 E Mb E^T),  Mb = G + |c| P + dM
//     bounding both |M_ref| and |M_fast|; C' the f32 IDCT's exact linear map, E the first-order
//     bound of its roundings per input (|IDCT_fl(x) - C' x| <= u E |x|), both from a transcription
//     of the op sequence (tools/exp/idct_bound.py -> tmfwm_idct_bounds.h, every slider length) --
//     rank-three, so per pixel six products of |C'|- and E-transformed vectors;
// and keeps a block's bytes when every channel gives the same byte at Y_fast - eps_Y and
// Y_fast + eps_Y (each channel is monotone in Y).  Top pair: with v the iterate, rho = |Dv|^2 /
// |v|^2, r = D^T D v - rho v and F = |D|_F^2, the extract's Kato-Temple margins (sigma1_certified)
// give lambda_1 in [rho, rho + |r|^2 / gap], gap = 2 rho - F, and Davis-Kahan sin(v, v1) <=
// |r| / (|v| gap); u = D v / |D v| is no further from u1; LAPACK's own top pair is within
// 1024 2^-53 s1 / (s1 - s2) (6.4 times the worst measured, tools/exp/lapack_bounds.py; the
// pass requires e <= 2^-30, so e's share of the bound is below 2^-29 |c| whatever that constant).
// A block that fails any test (no spectral gap, an undecided byte) writes nothing and goes to the
// slow list, whose list pass (embed_kernel<b, true>) redoes it on the full hybrid route -- Jacobi
// SVD, byte certificate, dgesdd route (TMFWM_ROUTE_RANK1) -- or straight to the dgesdd route
// (TMFWM_ROUTE_RANK1_REFERENCE, no Jacobi factors and so no K), so every byte is the reference's
// either way.
#include "tmfwm_blocks.h"
#include "tmfwm_idct_bounds.h"

namespace tmf {

extern template __global__ void embed_kernel<8, true>(EmbedArgs);  // tmfwm_embed8.hip
// the list passes of the other sizes exist for this route only (the hybrid route's strip pass
// there runs every block to the end, kDeferMax<b> = 0): instantiated in tmfwm_rank1_lists.hip
extern template __global__ void embed_kernel<4, true>(EmbedArgs);
extern template __global__ void embed_kernel<6, true>(EmbedArgs);
extern template __global__ void embed_kernel<10, true>(EmbedArgs);
extern template __global__ void embed_kernel<12, true>(EmbedArgs);
extern template __global__ void embed_kernel<14, true>(EmbedArgs);
extern template __global__ void embed_kernel<16, true>(EmbedArgs);

constexpr int kRank1Iters = 4;  // f64 power steps before the a-posteriori test

// value of element k (0 <= k < B) of a per-row quantity held as R rows per lane (lane k / R)
template <int B, int L, int K>
TMF_DEVI float row_value(const float (&own)[kRows<B, L>])
{
    constexpr int R = kRows<B, L>;
    return group_bcast<L, K / R>(own[K % R]);
}

template <int B>
__global__ __launch_bounds__(64, B <= 8 ? 3 : 2) void embed_rank1_kernel(EmbedArgs a)
{
    constexpr int L = Geo<B>::L, R = Geo<B>::R, BPW = Geo<B>::BPW, LD = B + 1, NW = Geo<B>::NW;
    constexpr double u53 = 1.1102230246251565e-16;  // 2^-53
    constexpr float u24 = 5.9604644775390625e-08f;  // 2^-24
    __shared__ float lds[BPW * B * LD];
    __shared__ uint32_t pix[R * NW][64];
    const int lane = threadIdx.x & 63, g = lane / L, q = lane % L;
    float *tile = lds + g * B * LD;
    const StripPos pos = strip_pos<B>(a.strips_per_row, a.nbw);
    const uint32_t id = (uint32_t)(((int64_t)blockIdx.y * a.nbh + pos.bi) * a.nbw + pos.bj);
    const uint8_t *src = a.src + pos.frame * a.frame_stride;
    uint8_t *dst = a.dst + pos.frame * a.frame_stride;

    float x[R][B];
    {
        uint32_t words[R][NW];
        load_block_rows<B>(src, a.W, pos, q, a.aligned, words);
        luma_rows<B>(words, x);
        // the source bytes wait in LDS until the colour phase
#pragma unroll
        for (int r = 0; r < R; ++r)
#pragma unroll
            for (int i = 0; i < NW; ++i) pix[r * NW + i][lane] = words[r][i];
    }
    dct2d_rows_layout<B, false>(x, tile, q);  // :192, D in rows layout
    double xd[R][B];  // D in f64 (exact), the f32 copy is dead until M_fast
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
        for (int j = 0; j < B; ++j) xd[r][j] = (double)x[r][j];

    // squared row norms (this lane's rows), squared column norms and |D|_F^2, in f64
    double rn[R], cn[B], F = 0.0;
#pragma unroll
    for (int r = 0; r < R; ++r) {
        double acc = 0.0;
#pragma unroll
        for (int j = 0; j < B; ++j) acc = __builtin_fma(xd[r][j], xd[r][j], acc);
        rn[r] = acc;
    }
#pragma unroll
    for (int j = 0; j < B; ++j) {
        double acc = 0.0;
#pragma unroll
        for (int r = 0; r < R; ++r) acc = __builtin_fma(xd[r][j], xd[r][j], acc);
        cn[j] = group_sum<L>(acc);
        F += cn[j];
    }
    const bool zero = F == 0.0;

    // power iteration on D^T D from the column norms
    double v[B];
#pragma unroll
    for (int j = 0; j < B; ++j) v[j] = zero ? (j == 0 ? 1.0 : 0.0) : cn[j];
    double t[R];
#pragma unroll
    for (int it = 0; it < kRank1Iters; ++it) {
#pragma unroll
        for (int r = 0; r < R; ++r) {
            double acc = 0.0;
#pragma unroll
            for (int j = 0; j < B; ++j) acc = __builtin_fma(xd[r][j], v[j], acc);
            t[r] = acc;
        }
        double w[B], nn = 0.0;
#pragma unroll
        for (int j = 0; j < B; ++j) {
            double acc = 0.0;
#pragma unroll
            for (int r = 0; r < R; ++r) acc = __builtin_fma(xd[r][j], t[r], acc);
            w[j] = group_sum<L>(acc);
            nn = __builtin_fma(w[j], w[j], nn);
        }
        const bool live = nn > 0.0 && nn < 1e300;
        const double inv = live ? 1.0 / __builtin_sqrt(nn) : 1.0;
#pragma unroll
        for (int j = 0; j < B; ++j) v[j] = live ? w[j] * inv : v[j];
    }
    // a-posteriori (sigma1_certified's margins): rho = |Dv|^2 / |v|^2, r = D^T D v - rho v
    double nv = 0.0, rho_p = 0.0;
#pragma unroll
    for (int j = 0; j < B; ++j) nv = __builtin_fma(v[j], v[j], nv);
#pragma unroll
    for (int r = 0; r < R; ++r) {
        double acc = 0.0;
#pragma unroll
        for (int j = 0; j < B; ++j) acc = __builtin_fma(xd[r][j], v[j], acc);
        t[r] = acc;
        rho_p = __builtin_fma(acc, acc, rho_p);
    }
    const double tt = group_sum<L>(rho_p), rho = tt / nv;
    double rn2 = 0.0;
#pragma unroll
    for (int j = 0; j < B; ++j) {
        double acc = 0.0;
#pragma unroll
        for (int r = 0; r < R; ++r) acc = __builtin_fma(xd[r][j], t[r], acc);
        const double rj = group_sum<L>(acc) - rho * v[j];
        rn2 = __builtin_fma(rj, rj, rn2);
    }
    const double rr0 = __builtin_sqrt(rn2 / nv) * (1.0 + 16.0 * u53) + 256.0 * u53 * F;
    const double rlo = rho * (1.0 - 256.0 * u53), fhi = F * (1.0 + 256.0 * u53);
    const double gap = (rlo + rlo) - fhi;
    const double lhi = (rho + rr0 * rr0 / (gap > 0.0 ? gap : 1.0)) * (1.0 + 256.0 * u53);
    const double s1hi = __builtin_sqrt(lhi) * (1.0 + 512.0 * u53);
    const double s1lo = __builtin_sqrt(rlo) * (1.0 - 512.0 * u53);
    const double s2hi = __builtin_sqrt(fhi - rlo > 0.0 ? fhi - rlo : 0.0) * (1.0 + 512.0 * u53);
    const double g1 = s1lo - s2hi;
    const double theta = rr0 / (gap > 0.0 ? gap : 1.0);
    const double eps_uv = zero ? 0.0 : 1.01 * theta + 1024.0 * u53 * s1hi / (g1 > 0.0 ? g1 : 1.0) + 0x1p-45;
    bool ok = zero || (gap > 0.0 && g1 > 0.0 && eps_uv <= 0x1p-30 && rho == rho);

    // the unit top pair: v / |v|, u = D v / |D v| (this lane's rows)
    const double vinv = zero ? 1.0 : 1.0 / __builtin_sqrt(nv), tinv = zero ? 1.0 : 1.0 / __builtin_sqrt(tt);
    double uu[R];
#pragma unroll
    for (int r = 0; r < R; ++r) uu[r] = zero ? ((q * R + r) == 0 ? 1.0 : 0.0) : t[r] * tinv;
#pragma unroll
    for (int j = 0; j < B; ++j) v[j] = v[j] * vinv;

    // M_fast = f32(D + c u v^T) (:198 + :201 with the top pair alone)
    const uint32_t wv = pos.valid ? a.wm[(int64_t)pos.bi * a.nbw + pos.bj] : 0u;
    const double cw = a.alpha * ((double)wv / 255.0);
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
        for (int j = 0; j < B; ++j) x[r][j] = (float)__builtin_fma(cw * uu[r], v[j], xd[r][j]);

    // eps_Y (tools/exp/idct_bound.py): |M_ref - M_fast| <= dM = al a b^T + be u' v'^T + ga 1 1^T and
    // |M_ref|, |M_fast| <= Mb = (1 + al) a b^T + (|c| + be) u' v'^T + ga 1 1^T; the f32 IDCT is
    // IDCT_fl(M) = C' M C'^T + R, |R| <= u (E |M| |C'|^T + |C'| |M| E^T) + u^2 E |M| E^T (C' its exact
    // map, E its first-order rounding bound: IdctBound<B>), so with d_t, m_t the weights above,
    //   eps_Y = sum_t d_t (|C'| x_t)(|C'| y_t)^T + 2 u m_t ((E x_t)(|C'| y_t)^T + (|C'| x_t)(E y_t)^T
    //           + u (E x_t)(E y_t)^T),
    // per pixel (p, q): sum_t A_t(p) P_t(q) + EA_t(p) Q_t(q), P_t = d_t B_t + 2 u m_t EB_t,
    // Q_t = 2 u m_t (B_t + u EB_t), A_t = |C'| x_t, EA_t = E x_t, B_t = |C'| y_t, EB_t = E y_t
    using Tb = IdctBound<B>;
    const float e = (float)eps_uv * (1.0f + 0x1p-20f);
    const float cabs = (float)__builtin_fabs(cw) * (1.0f + 0x1p-20f), s1f = (float)s1hi * (1.0f + 0x1p-20f);
    const float al = 1.01f * (B + 6) * u24, be = 1.01f * ((B + 6) * u24 * cabs + 2.0f * u24 * (s1f + cabs));
    const float ga = 0x1p-40f * s1f + cabs * e * (2.0f + e);
    const float w1 = 2.0f * u24 * (1.0f + al), w2 = 2.0f * u24 * (cabs + be);  // 2 u m_1, 2 u m_2
    float ra[R], ru[R];  // a_i = |D_i,:|^(1/2), u'_i = |u_i| + e on this lane's rows
#pragma unroll
    for (int r = 0; r < R; ++r) {
        ra[r] = __builtin_sqrtf(__builtin_sqrtf((float)rn[r] * (1.0f + 0x1p-20f))) * (1.0f + 0x1p-20f);
        ru[r] = (float)__builtin_fabs(uu[r]) + e;
    }
    float av[B], uv[B];  // all rows' a_i and u'_i
    static_for<B>([&](auto K) {
        av[K] = row_value<B, L, K>(ra);
        uv[K] = row_value<B, L, K>(ru);
    });
    float P1[B], Q1[B], P2[B], Q2[B];  // terms a b^T and u' v'^T, every column q
#pragma unroll
    for (int qq = 0; qq < B; ++qq) {
        float sb = 0.0f, eb = 0.0f, sv = 0.0f, ev = 0.0f;
#pragma unroll
        for (int j = 0; j < B; ++j) {
            const float bj = __builtin_sqrtf(__builtin_sqrtf((float)cn[j] * (1.0f + 0x1p-20f))) * (1.0f + 0x1p-20f);
            const float vj = (float)__builtin_fabs(v[j]) + e;
            sb = __builtin_fmaf(Tb::absc[qq][j], bj, sb);
            eb = __builtin_fmaf(Tb::err[qq][j], bj, eb);
            sv = __builtin_fmaf(Tb::absc[qq][j], vj, sv);
            ev = __builtin_fmaf(Tb::err[qq][j], vj, ev);
        }
        P1[qq] = __builtin_fmaf(al, sb, w1 * eb);
        Q1[qq] = w1 * __builtin_fmaf(u24, eb, sb);
        P2[qq] = __builtin_fmaf(be, sv, w2 * ev);
        Q2[qq] = w2 * __builtin_fmaf(u24, ev, sv);
    }

    dct2d_rows_layout<B, true>(x, tile, q);  // :204, Y_fast

    // :207-216 at both ends of [Y_fast - eps_Y, Y_fast + eps_Y]
    bool unc = false;
    uint32_t outw[R][NW];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        float Ap = 0.0f, EAp = 0.0f, Up = 0.0f, EUp = 0.0f, Sp = 0.0f, ESp = 0.0f;
        // A_t(p), EA_t(p): the tables' row of this pixel row (p = q R + r is lane-dependent: the
        // entries come from the tables by a select over the L lanes' rows)
        static_for<B>([&](auto I) {
            float cpi = Tb::absc[r][I], epi = Tb::err[r][I];
            static_for<L - 1>([&](auto Q1_) {
                constexpr int QQ = Q1_ + 1;
                if (QQ * R + r < B) {
                    cpi = q == QQ ? Tb::absc[(QQ * R + r) % B][I] : cpi;
                    epi = q == QQ ? Tb::err[(QQ * R + r) % B][I] : epi;
                }
            });
            Ap = __builtin_fmaf(cpi, av[I], Ap);
            EAp = __builtin_fmaf(epi, av[I], EAp);
            Up = __builtin_fmaf(cpi, uv[I], Up);
            EUp = __builtin_fmaf(epi, uv[I], EUp);
            Sp += cpi;
            ESp += epi;
        });
        uint32_t words[NW];
#pragma unroll
        for (int i = 0; i < NW; ++i) {
            outw[r][i] = 0u;
            words[i] = pix[r * NW + i][lane];
        }
#pragma unroll
        for (int c = 0; c < B; ++c) {
            const float y = x[r][c];
            // the ones term's column factors are compile-time sums of the tables
            float B3 = 0.0f, EB3 = 0.0f;
#pragma unroll
            for (int j = 0; j < B; ++j) {
                B3 += Tb::absc[c][j];
                EB3 += Tb::err[c][j];
            }
            const float t3 = Sp * __builtin_fmaf(2.0f * u24, EB3, B3) + ESp * (2.0f * u24) * __builtin_fmaf(u24, EB3, B3);
            const float ey = (Ap * P1[c] + EAp * Q1[c] + Up * P2[c] + EUp * Q2[c] + ga * t3) * (1.0f + 0x1p-16f) +
                             __builtin_fabsf(y) * 0x1p-22f + 0x1p-40f;
            float cbs, crs;
            const uint32_t R0 = byte_at(words, 3 * c), G0 = byte_at(words, 3 * c + 1), B0 = byte_at(words, 3 * c + 2);
            chroma(R0, G0, B0, cbs, crs);
            uint32_t R8, G8, B8;
            float fr;
            colour_inv_frac(y - ey, cbs, crs, R8, G8, B8, fr);
            const float dy = 2.0f * ey;
            const bool wide = fr + __builtin_fmaf(dy, 255.1f, 0x1p-14f) >= 1.0f;
            if (__builtin_amdgcn_ballot_w64(wide) != 0 && wide) {
                uint32_t R9, G9, B9;
                colour_inv(y + ey, cbs, crs, R9, G9, B9);
                unc = unc || R9 != R8 || G9 != G8 || B9 != B8;
            }
            const int k0 = 3 * c;
            outw[r][k0 >> 2] |= R8 << (8 * (k0 & 3));
            outw[r][(k0 + 1) >> 2] |= G8 << (8 * ((k0 + 1) & 3));
            outw[r][(k0 + 2) >> 2] |= B8 << (8 * ((k0 + 2) & 3));
        }
    }
    ok = ok && group_or<L>(unc ? 1 : 0) == 0;
    if (!pos.valid) return;
    if (ok) {
#pragma unroll
        for (int r = 0; r < R; ++r) {
            uint8_t *pp = dst + ((int64_t)(pos.bi * B + q * R + r) * a.W + (int64_t)pos.bj * B) * 3;
            if (real_row<B>(q, r)) store_words<B>(pp, a.aligned, outw[r]);
        }
    } else if (q == 0) {
        if (a.slow_list) {  // TMFWM_ROUTE_RANK1: the full hybrid route in the list pass
            const uint32_t row = blockIdx.y * (uint32_t)a.nbh + (uint32_t)pos.bi, s = row % kListShards;
            a.slow_list[shard_base(s, (uint32_t)a.nframes * (uint32_t)a.nbh, (uint32_t)a.nbw) +
                        atomicAdd(a.slow_shards + s * kShardStride, 1u)] = id;
        } else {  // TMFWM_ROUTE_RANK1_REFERENCE: the dgesdd route (embed_fixup_kernel)
            a.fb_list[atomicAdd(a.fb_count, 1u)] = id;
        }
    }
}

template <int B>
static hipError_t launch_rank1_b(EmbedArgs a, hipStream_t st)
{
    a.strips_per_row = (a.nbw + Geo<B>::BPW - 1) / Geo<B>::BPW;
    const int64_t gx = (int64_t)a.strips_per_row * a.nbh;
    for (int64_t f0 = 0; f0 < a.nframes; f0 += 65535) {
        EmbedArgs c = a;
        const int64_t nf = a.nframes - f0 < 65535 ? a.nframes - f0 : 65535;
        c.src = a.src + f0 * a.frame_stride;
        c.dst = a.dst + f0 * a.frame_stride;
        hipLaunchKernelGGL((embed_rank1_kernel<B>), dim3((unsigned)gx, (unsigned)nf), dim3(64), 0, st, c);
    }
    if (a.slow_list) {  // TMFWM_ROUTE_RANK1: the list pass over the blocks the pre-pass left
        const int64_t rows = a.nframes * a.nbh;
        const unsigned grid = (unsigned)(rows < (int64_t)kListShards ? rows : (int64_t)kListShards);
        hipLaunchKernelGGL((embed_kernel<B, true>), dim3(grid), dim3(64), 0, st, a);
    }
    return hipGetLastError();
}

bool rank1_block(int block) { return block >= 4 && block <= 16 && block % 2 == 0; }

// The rank-1 pre-pass over every block (every slider size, b = 4..16 even), then the edge pixels.  TMFWM_ROUTE_RANK1
// (a.slow_list set): the list pass (embed_kernel<b, true>: the full hybrid route) over the blocks
// it left; TMFWM_ROUTE_RANK1_REFERENCE (no slow list): those blocks went to the dgesdd-route list.
// Either way the caller runs the dgesdd-route fixup next.  The caller handles other block sizes.
hipError_t launch_embed_rank1(EmbedArgs a, hipStream_t st)
{
    if (!rank1_block(a.block)) return hipErrorInvalidValue;
    if (a.nbh > 0 && a.nbw > 0) {
        hipError_t e = hipErrorInvalidValue;
        switch (a.block) {
        case 4: e = launch_rank1_b<4>(a, st); break;
        case 6: e = launch_rank1_b<6>(a, st); break;
        case 8: e = launch_rank1_b<8>(a, st); break;
        case 10: e = launch_rank1_b<10>(a, st); break;
        case 12: e = launch_rank1_b<12>(a, st); break;
        case 14: e = launch_rank1_b<14>(a, st); break;
        case 16: e = launch_rank1_b<16>(a, st); break;
        }
        if (e != hipSuccess) return e;
    }
    return launch_edges(a.src, a.dst, a.nframes, a.H, a.W, a.frame_stride, a.block, st);
}

}  // namespace tmf
