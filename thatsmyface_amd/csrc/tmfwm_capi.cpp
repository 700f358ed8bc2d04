// C ABI of libtmfwm.so (declared in include/tmfwm.h): argument checking, host
// staging for TMFWM_MEM_HOST, stream selection and error reporting around the
// kernel launchers of tmfwm_kernels.hip.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <string>
#include <vector>

#include "../../include/tmfwm.h"
#include "tmfwm_internal.h"

namespace {

thread_local std::string t_err;

int fail(int code, const char *fmt, ...)
{
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    t_err = buf;
    return code;
}

#define TMF_HIP(call)                                                                                   \
    do {                                                                                                \
        hipError_t e_ = (call);                                                                         \
        if (e_ != hipSuccess) return fail(TMFWM_ERR_HIP, "%s failed: %s", #call, hipGetErrorString(e_)); \
    } while (0)

hipStream_t pick_stream(void *s) { return s ? reinterpret_cast<hipStream_t>(s) : hipStreamPerThread; }

bool supported_block(int b) { return b >= 4 && b <= 16 && b % 2 == 0; }  // the UI slider values

// A device pointer handed in as TMFWM_MEM_DEVICE must really be device memory:
// a host pointer dereferenced by a kernel would fault the GPU.
int check_device_ptr(const void *p, const char *name)
{
    if (p == nullptr) return fail(TMFWM_ERR_INVALID, "%s is NULL", name);
    hipPointerAttribute_t at;
    hipError_t e = hipPointerGetAttributes(&at, p);
    if (e != hipSuccess) {
        (void)hipGetLastError();
        return fail(TMFWM_ERR_INVALID, "%s is not a HIP device pointer (%s)", name, hipGetErrorString(e));
    }
    if (at.type != hipMemoryTypeDevice && at.type != hipMemoryTypeManaged)
        return fail(TMFWM_ERR_INVALID, "%s is not device memory (memory type %d)", name, (int)at.type);
    return 0;
}

// Device scratch for the host-memory path, released in the destructor.
struct DevBuf {
    void *p = nullptr;
    hipStream_t st = nullptr;
    ~DevBuf()
    {
        if (p) (void)hipFreeAsync(p, st);
    }
    int alloc(size_t n, hipStream_t s, const char *what)
    {
        st = s;
        if (n == 0) return 0;
        hipError_t e = hipMallocAsync(&p, n, s);
        if (e != hipSuccess) {
            p = nullptr;
            (void)hipGetLastError();
            return fail(TMFWM_ERR_NOMEM, "device allocation of %zu bytes for %s failed: %s", n, what, hipGetErrorString(e));
        }
        return 0;
    }
};

int check_frames(int64_t n, int32_t H, int32_t W, int64_t stride, int32_t block)
{
    if (n < 0 || H < 0 || W < 0) return fail(TMFWM_ERR_INVALID, "negative size (n=%lld, H=%d, W=%d)", (long long)n, H, W);
    if (!supported_block(block)) return fail(TMFWM_ERR_UNSUPPORTED, "block size %d not supported (even, 4..16)", block);
    if (stride < (int64_t)H * W * 3) return fail(TMFWM_ERR_INVALID, "frame_stride %lld < H*W*3", (long long)stride);
    return 0;
}

// After argument validation: there is no CPU fallback, so no device is an error.
int need_device()
{
    int dev = 0;
    if (hipGetDeviceCount(&dev) != hipSuccess || dev == 0) {
        (void)hipGetLastError();
        return fail(TMFWM_ERR_NODEVICE, "no HIP device available");
    }
    return 0;
}

// [a, a+na) and [b, b+nb) share a byte (the kernels read one while writing the other)
bool ranges_overlap(const void *a, size_t na, const void *b, size_t nb)
{
    const uintptr_t x = reinterpret_cast<uintptr_t>(a), y = reinterpret_cast<uintptr_t>(b);
    return na && nb && x < y + nb && y < x + na;
}

size_t span_bytes(int64_t n, int64_t stride, int64_t frame_bytes) { return n == 0 ? 0 : (size_t)((n - 1) * stride + frame_bytes); }

}  // namespace

extern "C" {

int tmfwm_abi_version(void) { return TMFWM_ABI_VERSION; }

const char *tmfwm_last_error(void) { return t_err.c_str(); }

int tmfwm_device_count(void)
{
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) {
        (void)hipGetLastError();
        return 0;
    }
    return n;
}

int tmfwm_embed(const uint8_t *rgb, int64_t n_frames, int32_t height, int32_t width, int64_t frame_stride,
                const uint8_t *wm_tile, int32_t block, double alpha, uint8_t *out, int32_t mem_kind, void *hip_stream)
{
    t_err.clear();
    if (int rc = check_frames(n_frames, height, width, frame_stride, block)) return rc;
    if (!std::isfinite(alpha)) return fail(TMFWM_ERR_INVALID, "alpha is not finite");
    if (int rc = need_device()) return rc;
    if (n_frames == 0 || height == 0 || width == 0) return 0;
    const int nbh = height / block, nbw = width / block;
    const int64_t fbytes = (int64_t)height * width * 3;
    const size_t span = span_bytes(n_frames, frame_stride, fbytes), tbytes = (size_t)nbh * nbw;
    hipStream_t st = pick_stream(hip_stream);
    tmf::EmbedArgs a{};
    a.nframes = n_frames;
    a.frame_stride = frame_stride;
    a.H = height;
    a.W = width;
    a.block = block;
    a.nbh = nbh;
    a.nbw = nbw;
    a.alpha = alpha;
    if (mem_kind == TMFWM_MEM_DEVICE) {
        if (int rc = check_device_ptr(rgb, "rgb")) return rc;
        if (int rc = check_device_ptr(out, "out")) return rc;
        if (tbytes) {
            if (int rc = check_device_ptr(wm_tile, "wm_tile")) return rc;
        }
        if (ranges_overlap(rgb, span, out, span)) return fail(TMFWM_ERR_INVALID, "out overlaps rgb (in-place embed is not supported)");
        if (tbytes && ranges_overlap(wm_tile, tbytes, out, span)) return fail(TMFWM_ERR_INVALID, "out overlaps wm_tile");
        a.src = rgb;
        a.dst = out;
        a.wm = wm_tile;
        a.aligned = ((reinterpret_cast<uintptr_t>(rgb) | reinterpret_cast<uintptr_t>(out)) % 4 == 0) && frame_stride % 4 == 0 && width % 4 == 0;
        TMF_HIP(tmf::launch_embed(a, st));
        return 0;
    }
    if (mem_kind != TMFWM_MEM_HOST) return fail(TMFWM_ERR_INVALID, "mem_kind %d", mem_kind);
    if (!rgb || !out || (tbytes && !wm_tile)) return fail(TMFWM_ERR_INVALID, "NULL host pointer");
    DevBuf din, dout, dwm;
    if (int rc = din.alloc(span, st, "input frames")) return rc;
    if (int rc = dout.alloc(span, st, "output frames")) return rc;
    if (int rc = dwm.alloc(tbytes, st, "watermark tile")) return rc;
    TMF_HIP(hipMemcpyAsync(din.p, rgb, span, hipMemcpyHostToDevice, st));
    if (tbytes) TMF_HIP(hipMemcpyAsync(dwm.p, wm_tile, tbytes, hipMemcpyHostToDevice, st));
    a.src = static_cast<const uint8_t *>(din.p);
    a.dst = static_cast<uint8_t *>(dout.p);
    a.wm = static_cast<const uint8_t *>(dwm.p);
    a.aligned = frame_stride % 4 == 0 && width % 4 == 0;
    TMF_HIP(tmf::launch_embed(a, st));
    if (frame_stride == fbytes) {
        TMF_HIP(hipMemcpyAsync(out, dout.p, span, hipMemcpyDeviceToHost, st));
    } else {
        for (int64_t f = 0; f < n_frames; ++f)
            TMF_HIP(hipMemcpyAsync(out + f * frame_stride, static_cast<uint8_t *>(dout.p) + f * frame_stride, (size_t)fbytes,
                                   hipMemcpyDeviceToHost, st));
    }
    TMF_HIP(hipStreamSynchronize(st));
    return 0;
}

int tmfwm_extract(const uint8_t *wm_rgb, const uint8_t *orig_rgb, int64_t n_frames, int32_t height, int32_t width,
                  int64_t frame_stride, int32_t block, double alpha, uint8_t *out_tiles, int32_t mem_kind, void *hip_stream)
{
    t_err.clear();
    if (int rc = check_frames(n_frames, height, width, frame_stride, block)) return rc;
    if (!std::isfinite(alpha) || alpha == 0.0) return fail(TMFWM_ERR_INVALID, "alpha must be finite and non-zero");
    if (int rc = need_device()) return rc;
    const int nbh = height / block, nbw = width / block;
    const int64_t tbytes = (int64_t)nbh * nbw;
    if (n_frames == 0 || tbytes == 0) return 0;
    const int64_t fbytes = (int64_t)height * width * 3;
    const size_t span = span_bytes(n_frames, frame_stride, fbytes);
    hipStream_t st = pick_stream(hip_stream);
    tmf::ExtractArgs a{};
    a.nframes = n_frames;
    a.frame_stride = frame_stride;
    a.tile_stride = tbytes;
    a.H = height;
    a.W = width;
    a.block = block;
    a.nbh = nbh;
    a.nbw = nbw;
    a.alpha32 = (float)alpha;
    if (mem_kind == TMFWM_MEM_DEVICE) {
        if (int rc = check_device_ptr(wm_rgb, "wm_rgb")) return rc;
        if (int rc = check_device_ptr(orig_rgb, "orig_rgb")) return rc;
        if (int rc = check_device_ptr(out_tiles, "out_tiles")) return rc;
        const size_t obytes = (size_t)(tbytes * n_frames);
        if (ranges_overlap(out_tiles, obytes, wm_rgb, span) || ranges_overlap(out_tiles, obytes, orig_rgb, span))
            return fail(TMFWM_ERR_INVALID, "out_tiles overlaps an input batch");
        a.wsrc = wm_rgb;
        a.osrc = orig_rgb;
        a.out = out_tiles;
        a.aligned = ((reinterpret_cast<uintptr_t>(wm_rgb) | reinterpret_cast<uintptr_t>(orig_rgb)) % 4 == 0) && frame_stride % 4 == 0 && width % 4 == 0;
        TMF_HIP(tmf::launch_extract(a, st));
        return 0;
    }
    if (mem_kind != TMFWM_MEM_HOST) return fail(TMFWM_ERR_INVALID, "mem_kind %d", mem_kind);
    if (!wm_rgb || !orig_rgb || !out_tiles) return fail(TMFWM_ERR_INVALID, "NULL host pointer");
    DevBuf dw, dor, dout;
    if (int rc = dw.alloc(span, st, "watermarked frames")) return rc;
    if (int rc = dor.alloc(span, st, "original frames")) return rc;
    if (int rc = dout.alloc((size_t)(tbytes * n_frames), st, "extracted tiles")) return rc;
    TMF_HIP(hipMemcpyAsync(dw.p, wm_rgb, span, hipMemcpyHostToDevice, st));
    TMF_HIP(hipMemcpyAsync(dor.p, orig_rgb, span, hipMemcpyHostToDevice, st));
    a.wsrc = static_cast<const uint8_t *>(dw.p);
    a.osrc = static_cast<const uint8_t *>(dor.p);
    a.out = static_cast<uint8_t *>(dout.p);
    a.aligned = frame_stride % 4 == 0 && width % 4 == 0;
    TMF_HIP(tmf::launch_extract(a, st));
    TMF_HIP(hipMemcpyAsync(out_tiles, dout.p, (size_t)(tbytes * n_frames), hipMemcpyDeviceToHost, st));
    TMF_HIP(hipStreamSynchronize(st));
    return 0;
}

int tmfwm_rgb_to_ycbcr(const uint8_t *rgb, int64_t npix, float *ycc, int32_t mem_kind, void *hip_stream)
{
    t_err.clear();
    if (npix < 0) return fail(TMFWM_ERR_INVALID, "npix < 0");
    if (npix == 0) return 0;
    if (int rc = need_device()) return rc;
    hipStream_t st = pick_stream(hip_stream);
    if (mem_kind == TMFWM_MEM_DEVICE) {
        if (int rc = check_device_ptr(rgb, "rgb")) return rc;
        if (int rc = check_device_ptr(ycc, "ycc")) return rc;
        TMF_HIP(tmf::launch_rgb_to_ycbcr(rgb, npix, ycc, st));
        return 0;
    }
    if (mem_kind != TMFWM_MEM_HOST || !rgb || !ycc) return fail(TMFWM_ERR_INVALID, "bad host arguments");
    DevBuf di, dy;
    if (int rc = di.alloc((size_t)npix * 3, st, "rgb")) return rc;
    if (int rc = dy.alloc((size_t)npix * 12, st, "ycc")) return rc;
    TMF_HIP(hipMemcpyAsync(di.p, rgb, (size_t)npix * 3, hipMemcpyHostToDevice, st));
    TMF_HIP(tmf::launch_rgb_to_ycbcr(static_cast<const uint8_t *>(di.p), npix, static_cast<float *>(dy.p), st));
    TMF_HIP(hipMemcpyAsync(ycc, dy.p, (size_t)npix * 12, hipMemcpyDeviceToHost, st));
    TMF_HIP(hipStreamSynchronize(st));
    return 0;
}

int tmfwm_ycbcr_to_rgb(const float *ycc, int64_t npix, uint8_t *rgb, int32_t mem_kind, void *hip_stream)
{
    t_err.clear();
    if (npix < 0) return fail(TMFWM_ERR_INVALID, "npix < 0");
    if (npix == 0) return 0;
    if (int rc = need_device()) return rc;
    hipStream_t st = pick_stream(hip_stream);
    if (mem_kind == TMFWM_MEM_DEVICE) {
        if (int rc = check_device_ptr(ycc, "ycc")) return rc;
        if (int rc = check_device_ptr(rgb, "rgb")) return rc;
        TMF_HIP(tmf::launch_ycbcr_to_rgb(ycc, npix, rgb, st));
        return 0;
    }
    if (mem_kind != TMFWM_MEM_HOST || !rgb || !ycc) return fail(TMFWM_ERR_INVALID, "bad host arguments");
    DevBuf dy, dr;
    if (int rc = dy.alloc((size_t)npix * 12, st, "ycc")) return rc;
    if (int rc = dr.alloc((size_t)npix * 3, st, "rgb")) return rc;
    TMF_HIP(hipMemcpyAsync(dy.p, ycc, (size_t)npix * 12, hipMemcpyHostToDevice, st));
    TMF_HIP(tmf::launch_ycbcr_to_rgb(static_cast<const float *>(dy.p), npix, static_cast<uint8_t *>(dr.p), st));
    TMF_HIP(hipMemcpyAsync(rgb, dr.p, (size_t)npix * 3, hipMemcpyDeviceToHost, st));
    TMF_HIP(hipStreamSynchronize(st));
    return 0;
}

int tmfwm_dct2d_blocks(float *blocks, int64_t n_blocks, int32_t block, int32_t inverse, int32_t mem_kind, void *hip_stream)
{
    t_err.clear();
    if (n_blocks < 0) return fail(TMFWM_ERR_INVALID, "n_blocks < 0");
    if (int rc = check_frames(0, 0, 0, 0, block)) return rc;
    if (int rc = need_device()) return rc;
    if (n_blocks == 0) return 0;
    hipStream_t st = pick_stream(hip_stream);
    const size_t bytes = (size_t)n_blocks * block * block * sizeof(float);
    if (mem_kind == TMFWM_MEM_DEVICE) {
        if (int rc = check_device_ptr(blocks, "blocks")) return rc;
        TMF_HIP(tmf::launch_dct2d_blocks(blocks, n_blocks, block, inverse != 0, st));
        return 0;
    }
    if (mem_kind != TMFWM_MEM_HOST || !blocks) return fail(TMFWM_ERR_INVALID, "bad host arguments");
    DevBuf d;
    if (int rc = d.alloc(bytes, st, "blocks")) return rc;
    TMF_HIP(hipMemcpyAsync(d.p, blocks, bytes, hipMemcpyHostToDevice, st));
    TMF_HIP(tmf::launch_dct2d_blocks(static_cast<float *>(d.p), n_blocks, block, inverse != 0, st));
    TMF_HIP(hipMemcpyAsync(blocks, d.p, bytes, hipMemcpyDeviceToHost, st));
    TMF_HIP(hipStreamSynchronize(st));
    return 0;
}

int tmfwm_svd_blocks(const float *D, int64_t n_blocks, int32_t block, float *U, float *S, float *Vt, int32_t *sweeps,
                     int32_t mem_kind, void *hip_stream)
{
    t_err.clear();
    if (n_blocks < 0) return fail(TMFWM_ERR_INVALID, "n_blocks < 0");
    if (int rc = check_frames(0, 0, 0, 0, block)) return rc;
    if (int rc = need_device()) return rc;
    if (n_blocks == 0) return 0;
    hipStream_t st = pick_stream(hip_stream);
    const size_t mb = (size_t)n_blocks * block * block * sizeof(float), sb = (size_t)n_blocks * block * sizeof(float);
    if (mem_kind == TMFWM_MEM_DEVICE) {
        for (auto [p, nm] : {std::pair<const void *, const char *>{D, "D"}, {U, "U"}, {S, "S"}, {Vt, "Vt"}})
            if (int rc = check_device_ptr(p, nm)) return rc;
        if (sweeps)
            if (int rc = check_device_ptr(sweeps, "sweeps")) return rc;
        TMF_HIP(tmf::launch_svd_blocks(D, n_blocks, block, U, S, Vt, sweeps, st));
        return 0;
    }
    if (mem_kind != TMFWM_MEM_HOST || !D || !U || !S || !Vt) return fail(TMFWM_ERR_INVALID, "bad host arguments");
    DevBuf dD, dU, dS, dV, dW;
    if (int rc = dD.alloc(mb, st, "D")) return rc;
    if (int rc = dU.alloc(mb, st, "U")) return rc;
    if (int rc = dS.alloc(sb, st, "S")) return rc;
    if (int rc = dV.alloc(mb, st, "Vt")) return rc;
    if (sweeps)
        if (int rc = dW.alloc((size_t)n_blocks * 4, st, "sweeps")) return rc;
    TMF_HIP(hipMemcpyAsync(dD.p, D, mb, hipMemcpyHostToDevice, st));
    TMF_HIP(tmf::launch_svd_blocks(static_cast<const float *>(dD.p), n_blocks, block, static_cast<float *>(dU.p),
                                   static_cast<float *>(dS.p), static_cast<float *>(dV.p), static_cast<int32_t *>(dW.p), st));
    TMF_HIP(hipMemcpyAsync(U, dU.p, mb, hipMemcpyDeviceToHost, st));
    TMF_HIP(hipMemcpyAsync(S, dS.p, sb, hipMemcpyDeviceToHost, st));
    TMF_HIP(hipMemcpyAsync(Vt, dV.p, mb, hipMemcpyDeviceToHost, st));
    if (sweeps) TMF_HIP(hipMemcpyAsync(sweeps, dW.p, (size_t)n_blocks * 4, hipMemcpyDeviceToHost, st));
    TMF_HIP(hipStreamSynchronize(st));
    return 0;
}

int tmfwm_synth_frames(uint64_t seed, int64_t frame0, int64_t n_frames, int64_t frame_bytes, uint8_t *out, void *hip_stream)
{
    t_err.clear();
    if (n_frames < 0 || frame_bytes < 0 || frame0 < 0) return fail(TMFWM_ERR_INVALID, "negative size");
    if (n_frames == 0 || frame_bytes == 0) return 0;
    if (int rc = need_device()) return rc;
    if (int rc = check_device_ptr(out, "out")) return rc;
    TMF_HIP(tmf::launch_synth(seed, frame0, n_frames, frame_bytes, out, pick_stream(hip_stream)));
    return 0;
}

int tmfwm_prepare_tile(const uint8_t *wm, int32_t wm_height, int32_t wm_width, int32_t tile_height, int32_t tile_width,
                       int32_t preserve_ratio, uint8_t *tile, int32_t mem_kind, void *hip_stream)
{
    t_err.clear();
    if (wm_height <= 0 || wm_width <= 0 || tile_height <= 0 || tile_width <= 0)
        return fail(TMFWM_ERR_INVALID, "height and width must be > 0 (watermark %dx%d, tile %dx%d)", wm_width, wm_height,
                    tile_width, tile_height);
    if (mem_kind != TMFWM_MEM_HOST && mem_kind != TMFWM_MEM_DEVICE) return fail(TMFWM_ERR_INVALID, "mem_kind %d", mem_kind);
    // watermarking.py:105-110: ratio = min(tw/ow, th/oh); new size int(size * ratio)
    int rh = tile_height, rw = tile_width, px = 0, py = 0;
    if (preserve_ratio) {
        const double fw = (double)tile_width / (double)wm_width, fh = (double)tile_height / (double)wm_height;
        const double ratio = fh < fw ? fh : fw;  // Python min() keeps the first of equals
        rw = (int)((double)wm_width * ratio);
        rh = (int)((double)wm_height * ratio);
        if (rw <= 0 || rh <= 0) return fail(TMFWM_ERR_INVALID, "height and width must be > 0 (resized %dx%d)", rw, rh);
        px = (tile_width - rw) / 2;  // :120-121
        py = (tile_height - rh) / 2;
    }
    if (mem_kind == TMFWM_MEM_DEVICE) {
        if (int rc = check_device_ptr(wm, "wm")) return rc;
        if (int rc = check_device_ptr(tile, "tile")) return rc;
    } else if (!wm || !tile) {
        return fail(TMFWM_ERR_INVALID, "NULL host pointer");
    }
    if (int rc = need_device()) return rc;
    hipStream_t st = pick_stream(hip_stream);
    tmf::ResamplePlan plan;
    plan.build(wm_height, wm_width, rh, rw);
    const std::vector<int> tables = plan.pack();
    const size_t wbytes = (size_t)wm_height * wm_width, tbytes = (size_t)tile_height * tile_width;
    DevBuf dtab, dtmp, dwm, dtile;
    if (int rc = dtab.alloc(tables.size() * sizeof(int), st, "resample tables")) return rc;
    if (int rc = dtmp.alloc(plan.tmp_bytes(), st, "resample scratch")) return rc;
    const uint8_t *src = wm;
    uint8_t *dst = tile;
    if (mem_kind == TMFWM_MEM_HOST) {
        if (int rc = dwm.alloc(wbytes, st, "watermark")) return rc;
        if (int rc = dtile.alloc(tbytes, st, "tile")) return rc;
        TMF_HIP(hipMemcpyAsync(dwm.p, wm, wbytes, hipMemcpyHostToDevice, st));
        src = static_cast<const uint8_t *>(dwm.p);
        dst = static_cast<uint8_t *>(dtile.p);
    }
    TMF_HIP(hipMemcpyAsync(dtab.p, tables.data(), tables.size() * sizeof(int), hipMemcpyHostToDevice, st));
    if (preserve_ratio) TMF_HIP(hipMemsetAsync(dst, 255, tbytes, st));  // Image.new("L", ..., 255) (:116)
    TMF_HIP(tmf::launch_resize_lanczos(src, plan, static_cast<const int *>(dtab.p), static_cast<uint8_t *>(dtmp.p),
                                       dst + (size_t)py * tile_width + px, tile_width, st));
    if (mem_kind == TMFWM_MEM_HOST) TMF_HIP(hipMemcpyAsync(tile, dst, tbytes, hipMemcpyDeviceToHost, st));
    // the host-side tables (and, for the host path, the result) must outlive the copies
    TMF_HIP(hipStreamSynchronize(st));
    return 0;
}

}  // extern "C"
