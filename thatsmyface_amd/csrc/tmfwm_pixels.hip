// Pixel-format conversion for the drop-in's zero-copy PIL path (tmfwm_embed_px /
// tmfwm_extract_px, ABI 8): PIL keeps a mode-"RGB" image in memory as 4 bytes per pixel
// (R, G, B, pad), which Image.__arrow_c_array__ / Image.fromarrow hand over without a
// copy; the watermark kernels read and write 3-byte pixels.  These two HBM-bound kernels
// convert on the device, so the host never packs or unpacks the image (the np.asarray /
// Image.fromarray copies of the drop-in).  Four pixels per thread: one 16-byte
// RGBX access against three 4-byte RGB accesses (byte accesses when a frame base or stride
// is not aligned, and for the last pixels of a frame).  Frame = blockIdx.y.
#include "tmfwm_internal.h"

namespace tmf {
namespace {

constexpr int kPixThreads = 256;

__global__ __launch_bounds__(kPixThreads) void pack_rgbx_kernel(const uint8_t *__restrict__ src, int64_t sstride,
                                                               uint8_t *__restrict__ dst, int64_t dstride, int64_t npix,
                                                               int vec)
{
    const int64_t p0 = ((int64_t)blockIdx.x * kPixThreads + threadIdx.x) * 4;
    if (p0 >= npix) return;
    const uint8_t *s = src + blockIdx.y * sstride + p0 * 4;
    uint8_t *d = dst + blockIdx.y * dstride + p0 * 3;
    if (vec && p0 + 4 <= npix) {
        const uint4 v = *reinterpret_cast<const uint4 *>(s);
        uint32_t *o = reinterpret_cast<uint32_t *>(d);
        o[0] = (v.x & 0xFFFFFFu) | (v.y << 24);
        o[1] = ((v.y >> 8) & 0xFFFFu) | (v.z << 16);
        o[2] = ((v.z >> 16) & 0xFFu) | (v.w << 8);
        return;
    }
    const int m = npix - p0 < 4 ? (int)(npix - p0) : 4;
    for (int k = 0; k < m; ++k) {
        d[3 * k] = s[4 * k];
        d[3 * k + 1] = s[4 * k + 1];
        d[3 * k + 2] = s[4 * k + 2];
    }
}

__global__ __launch_bounds__(kPixThreads) void unpack_rgbx_kernel(const uint8_t *__restrict__ src, int64_t sstride,
                                                                 uint8_t *__restrict__ dst, int64_t dstride, int64_t npix,
                                                                 int vec)
{
    const int64_t p0 = ((int64_t)blockIdx.x * kPixThreads + threadIdx.x) * 4;
    if (p0 >= npix) return;
    const uint8_t *s = src + blockIdx.y * sstride + p0 * 3;
    uint8_t *d = dst + blockIdx.y * dstride + p0 * 4;
    if (vec && p0 + 4 <= npix) {
        const uint32_t *w = reinterpret_cast<const uint32_t *>(s);
        const uint32_t w0 = w[0], w1 = w[1], w2 = w[2];
        uint4 v;
        v.x = (w0 & 0xFFFFFFu) | 0xFF000000u;
        v.y = (w0 >> 24) | ((w1 & 0xFFFFu) << 8) | 0xFF000000u;
        v.z = (w1 >> 16) | ((w2 & 0xFFu) << 16) | 0xFF000000u;
        v.w = (w2 >> 8) | 0xFF000000u;
        *reinterpret_cast<uint4 *>(d) = v;
        return;
    }
    const int m = npix - p0 < 4 ? (int)(npix - p0) : 4;
    for (int k = 0; k < m; ++k) {
        d[4 * k] = s[3 * k];
        d[4 * k + 1] = s[3 * k + 1];
        d[4 * k + 2] = s[3 * k + 2];
        d[4 * k + 3] = 0xFF;
    }
}

bool aligned(const void *p, int64_t stride, int a) { return reinterpret_cast<uintptr_t>(p) % a == 0 && stride % a == 0; }

}  // namespace

hipError_t launch_pack_rgbx(const uint8_t *src4, int64_t sstride, uint8_t *dst3, int64_t dstride, int64_t n, int H, int W,
                     hipStream_t st)
{
    const int64_t npix = (int64_t)H * W, quads = (npix + 3) / 4;
    if (n <= 0 || npix == 0) return hipSuccess;
    const int vec = aligned(src4, sstride, 16) && aligned(dst3, dstride, 4);
    for (int64_t f0 = 0; f0 < n; f0 += 65535) {  // grid.y limit
        const int64_t nf = n - f0 < 65535 ? n - f0 : 65535;
        const dim3 grid((unsigned)((quads + kPixThreads - 1) / kPixThreads), (unsigned)nf);
        hipLaunchKernelGGL(pack_rgbx_kernel, grid, dim3(kPixThreads), 0, st, src4 + f0 * sstride, sstride, dst3 + f0 * dstride,
                           dstride, npix, vec);
    }
    return hipGetLastError();
}

hipError_t launch_unpack_rgbx(const uint8_t *src3, int64_t sstride, uint8_t *dst4, int64_t dstride, int64_t n, int H, int W,
                       hipStream_t st)
{
    const int64_t npix = (int64_t)H * W, quads = (npix + 3) / 4;
    if (n <= 0 || npix == 0) return hipSuccess;
    const int vec = aligned(src3, sstride, 4) && aligned(dst4, dstride, 16);
    for (int64_t f0 = 0; f0 < n; f0 += 65535) {  // grid.y limit
        const int64_t nf = n - f0 < 65535 ? n - f0 : 65535;
        const dim3 grid((unsigned)((quads + kPixThreads - 1) / kPixThreads), (unsigned)nf);
        hipLaunchKernelGGL(unpack_rgbx_kernel, grid, dim3(kPixThreads), 0, st, src3 + f0 * sstride, sstride, dst4 + f0 * dstride,
                           dstride, npix, vec);
    }
    return hipGetLastError();
}

}  // namespace tmf
