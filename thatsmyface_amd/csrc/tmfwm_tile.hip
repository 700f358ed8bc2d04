// Watermark-tile preparation on the GPU: resize_watermark (watermarking.py:102-132)
// after the host's PNG decode + convert("L").  Pillow 12.2.0's Image.resize(LANCZOS)
// on an 8-bit image (Resample.c) is two integer passes over 22-bit fixed-point
// coefficients: a horizontal pass over the source rows the vertical filter uses,
// then a vertical pass; preserve_ratio pastes the result centred on a white canvas.
//
// The coefficient tables are built on the host here (double precision, the same
// libm sin() Pillow calls, so the rounding to fixed point is Pillow's), uploaded
// once per call, and the passes run as kernels -- one thread per output byte.  The
// tile is tiny (<= 480 x 270 for a 4K frame at b = 8); doing it on the device lets
// a multi-GPU job build the broadcast tile where it is consumed, without PIL.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cmath>
#include <vector>

#include "tmfwm_internal.h"

namespace tmf {

namespace {

constexpr int kPrecisionBits = 32 - 8 - 2;

double sinc(double x)
{
    if (x == 0.0) return 1.0;
    x = x * 3.14159265358979323846;  // M_PI
    return std::sin(x) / x;
}

double lanczos(double x) { return (-3.0 <= x && x < 3.0) ? sinc(x) * sinc(x / 3) : 0.0; }

}  // namespace

// Resample.c precompute_coeffs + normalize_coeffs_8bpc for box (0, in_size) -> out_size.
void ResampleAxis::build(int in_size, int out_size)
{
    const float in0 = 0.0f, in1 = (float)in_size;
    double filterscale, scale;
    filterscale = scale = (double)(in1 - in0) / out_size;
    if (filterscale < 1.0) filterscale = 1.0;
    const double support = 3.0 * filterscale;
    ksize = (int)std::ceil(support) * 2 + 1;
    bounds.assign((size_t)out_size * 2, 0);
    kk.assign((size_t)out_size * ksize, 0);
    std::vector<double> k((size_t)ksize);
    for (int xx = 0; xx < out_size; xx++) {
        const double center = in0 + (xx + 0.5) * scale, ss = 1.0 / filterscale;
        double ww = 0.0;
        int xmin = (int)(center - support + 0.5);
        if (xmin < 0) xmin = 0;
        int xmax = (int)(center + support + 0.5);
        if (xmax > in_size) xmax = in_size;
        xmax -= xmin;
        int x;
        for (x = 0; x < xmax; x++) {
            const double w = lanczos((x + xmin - center + 0.5) * ss);
            k[x] = w;
            ww += w;
        }
        for (x = 0; x < xmax; x++)
            if (ww != 0.0) k[x] /= ww;
        for (; x < ksize; x++) k[x] = 0;
        for (x = 0; x < ksize; x++)
            kk[(size_t)xx * ksize + x] =
                k[x] < 0 ? (int)(-0.5 + k[x] * (1 << kPrecisionBits)) : (int)(0.5 + k[x] * (1 << kPrecisionBits));
        bounds[xx * 2] = xmin;
        bounds[xx * 2 + 1] = xmax;
    }
}

__device__ __forceinline__ uint8_t clip8(int v)
{
    v >>= kPrecisionBits;
    return (uint8_t)(v < 0 ? 0 : v > 255 ? 255 : v);
}

// out[yy][xx] = clip8(2^21 + sum_x in[yy + y0][xmin + x] * k[xx][x])
__global__ __launch_bounds__(256) void resample_h_kernel(const uint8_t *__restrict__ in, int iw, int y0, int rows, int ow,
                                                         const int *__restrict__ bounds, const int *__restrict__ kk, int ks,
                                                         uint8_t *__restrict__ out, int ldo)
{
    const int xx = blockIdx.x * blockDim.x + threadIdx.x, yy = blockIdx.y;
    if (xx >= ow || yy >= rows) return;
    const int xmin = bounds[2 * xx], xmax = bounds[2 * xx + 1];
    const uint8_t *src = in + (int64_t)(yy + y0) * iw + xmin;
    const int *k = kk + (int64_t)xx * ks;
    int ss = 1 << (kPrecisionBits - 1);
    for (int x = 0; x < xmax; x++) ss += (int)src[x] * k[x];
    out[(int64_t)yy * ldo + xx] = clip8(ss);
}

// out[yy][xx] = clip8(2^21 + sum_y in[ymin + y][xx] * k[yy][y])
__global__ __launch_bounds__(256) void resample_v_kernel(const uint8_t *__restrict__ in, int iw, int oh,
                                                         const int *__restrict__ bounds, const int *__restrict__ kk, int ks,
                                                         uint8_t *__restrict__ out, int ldo)
{
    const int xx = blockIdx.x * blockDim.x + threadIdx.x, yy = blockIdx.y;
    if (xx >= iw || yy >= oh) return;
    const int ymin = bounds[2 * yy], ymax = bounds[2 * yy + 1];
    const int *k = kk + (int64_t)yy * ks;
    int ss = 1 << (kPrecisionBits - 1);
    for (int y = 0; y < ymax; y++) ss += (int)in[(int64_t)(y + ymin) * iw + xx] * k[y];
    out[(int64_t)yy * ldo + xx] = clip8(ss);
}

__global__ __launch_bounds__(256) void copy_rows_kernel(const uint8_t *__restrict__ in, int iw, int rows,
                                                        uint8_t *__restrict__ out, int ldo)
{
    const int x = blockIdx.x * blockDim.x + threadIdx.x, y = blockIdx.y;
    if (x < iw && y < rows) out[(int64_t)y * ldo + x] = in[(int64_t)y * iw + x];
}

static dim3 grid2(int w, int h) { return dim3((unsigned)((w + 255) / 256), (unsigned)h); }

// Image.resize((ow, oh), LANCZOS) of in (ih x iw) into out (row stride ldo).
// tables: device copy of [bounds_h | kk_h | bounds_v | kk_v] (ResamplePlan::pack),
// tmp: device scratch of plan.tmp_bytes().
hipError_t launch_resize_lanczos(const uint8_t *in, const ResamplePlan &plan, const int *tables, uint8_t *tmp, uint8_t *out,
                                 int ldo, hipStream_t st)
{
    const int ih = plan.ih, iw = plan.iw, oh = plan.oh, ow = plan.ow;
    if (oh == ih && ow == iw) {  // Image.resize returns a copy
        hipLaunchKernelGGL(copy_rows_kernel, grid2(iw, ih), dim3(256), 0, st, in, iw, ih, out, ldo);
        return hipGetLastError();
    }
    const int *bh = tables, *kh = bh + plan.h.bounds.size(), *bv = kh + plan.h.kk.size(), *kv = bv + plan.v.bounds.size();
    const uint8_t *src = in;
    int sw = iw;
    if (plan.need_h) {
        hipLaunchKernelGGL(resample_h_kernel, grid2(ow, plan.rows()), dim3(256), 0, st, in, iw, plan.y_first, plan.rows(), ow,
                           bh, kh, plan.h.ksize, tmp, ow);
        src = tmp;
        sw = ow;
    }
    if (plan.need_v)
        hipLaunchKernelGGL(resample_v_kernel, grid2(sw, oh), dim3(256), 0, st, src, sw, oh, bv, kv, plan.v.ksize, out, ldo);
    else
        hipLaunchKernelGGL(copy_rows_kernel, grid2(sw, oh), dim3(256), 0, st, src, sw, oh, out, ldo);
    return hipGetLastError();
}

void ResamplePlan::build(int in_h, int in_w, int out_h, int out_w)
{
    ih = in_h;
    iw = in_w;
    oh = out_h;
    ow = out_w;
    need_h = ow != iw;
    need_v = oh != ih;
    h.build(iw, ow);
    v.build(ih, oh);
    y_first = v.bounds[0];
    y_last = v.bounds[(size_t)oh * 2 - 2] + v.bounds[(size_t)oh * 2 - 1];
    if (need_h)  // the vertical pass reads the horizontally resampled rows [y_first, y_last)
        for (int i = 0; i < oh; i++) v.bounds[(size_t)i * 2] -= y_first;
}

std::vector<int> ResamplePlan::pack() const
{
    std::vector<int> t;
    t.reserve(h.bounds.size() + h.kk.size() + v.bounds.size() + v.kk.size());
    t.insert(t.end(), h.bounds.begin(), h.bounds.end());
    t.insert(t.end(), h.kk.begin(), h.kk.end());
    t.insert(t.end(), v.bounds.begin(), v.bounds.end());
    t.insert(t.end(), v.kk.begin(), v.kk.end());
    return t;
}

}  // namespace tmf
