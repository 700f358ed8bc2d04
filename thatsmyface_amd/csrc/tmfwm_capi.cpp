// C ABI of libtmfwm.so (declared in include/tmfwm.h): argument checking, host
// staging for TMFWM_MEM_HOST, stream selection and error reporting around the
// kernel launchers of tmfwm_kernels.hip.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/tmfwm.h"
#include "tmfwm_internal.h"

namespace {

thread_local std::string t_err;
thread_local int64_t t_list_pass = -1;  // tmfwm_last_list_pass_blocks

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

// The library's own stream-ordered pool per device (never the device's default pool, which
// torch's allocator and other libraries share): freed blocks stay cached up to kPoolKeep
// bytes -- enough for the per-call dgesdd lists and the host path's staging of an app-sized
// call -- and anything above is returned to the device at the next synchronisation.
constexpr uint64_t kPoolKeep = uint64_t(1) << 30;

hipMemPool_t lib_pool(int dev)
{
    static std::mutex mu;
    static std::vector<std::pair<int, hipMemPool_t>> pools;
    std::lock_guard<std::mutex> lk(mu);
    for (auto &p : pools)
        if (p.first == dev) return p.second;
    hipMemPoolProps props{};
    props.allocType = hipMemAllocationTypePinned;
    props.handleTypes = hipMemHandleTypeNone;
    props.location.type = hipMemLocationTypeDevice;
    props.location.id = dev;
    hipMemPool_t pool = nullptr;
    if (hipMemPoolCreate(&pool, &props) != hipSuccess) {
        (void)hipGetLastError();
        return nullptr;
    }
    uint64_t keep = kPoolKeep;
    (void)hipMemPoolSetAttribute(pool, hipMemPoolAttrReleaseThreshold, &keep);
    pools.emplace_back(dev, pool);
    return pool;
}

// the device a stream belongs to (the null / per-thread stream: the current device)
int stream_device(hipStream_t st)
{
    int dev = 0;
    if (st != nullptr && st != hipStreamPerThread) {
        hipDevice_t d = 0;
        if (hipStreamGetDevice(st, &d) == hipSuccess) return (int)d;
        (void)hipGetLastError();
    }
    if (hipGetDevice(&dev) != hipSuccess) (void)hipGetLastError();
    return dev;
}

// Device scratch for one call, stream-ordered from the library's pool on the stream's
// device, released (stream-ordered) in the destructor.
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
        hipMemPool_t pool = lib_pool(stream_device(s));
        hipError_t e = pool ? hipMallocFromPoolAsync(&p, n, pool, s) : hipMallocAsync(&p, n, s);
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

// Second-pass bookkeeping: frames go in chunks of at most kListCap
// blocks (and 65535 frames, the grid's y limit); each chunk's first pass appends the
// blocks that need the dgesdd route to one shared id list (u32, chunk-relative) and
// counts them in its own slot of `counts`; its fixup pass runs right after it on the
// same stream.  The fixup pass is latency-bound (one serial dgesdd per thread, a few ms
// whatever the list length), so chunks are made as large as the list allows:
// kListCap = 2^29 ids = 2 GiB (4 bytes per block, 2 % of the frames' own bytes at b = 8),
// i.e. 4142 4K frames at b = 8 -- configs[2] / [3] take one chunk per GPU.
// TMFWM_DEBUG_LIST_CAP (ids) lowers it so that the tests can exercise several chunks.
constexpr int64_t kListCap = int64_t(1) << 29;

// TMFWM_DEBUG_FORCE_NONCONV=1 marks one dgesdd-route block of every chunk as not converged
// (tests: the non-convergence report of the synchronising calls, include/tmfwm.h)
bool force_nonconv()
{
    const char *e = std::getenv("TMFWM_DEBUG_FORCE_NONCONV");
    return e && *e && *e != '0';
}

int64_t list_cap()
{
    const char *e = std::getenv("TMFWM_DEBUG_LIST_CAP");
    if (!e || !*e) return kListCap;
    const long long v = std::atoll(e);
    return v > 0 && v < kListCap ? (int64_t)v : kListCap;
}

struct Chunks {
    int64_t per_frame = 0, frames = 0, n = 0, cap = 0;
    void plan(int64_t nframes, int64_t blocks_per_frame)
    {
        per_frame = blocks_per_frame;
        frames = blocks_per_frame > 0 ? list_cap() / blocks_per_frame : nframes;
        if (frames < 1) frames = 1;
        if (frames > 65535) frames = 65535;
        if (frames > nframes) frames = nframes;
        n = frames > 0 ? (nframes + frames - 1) / frames : 0;
        cap = frames * blocks_per_frame;
    }
};

// sum the per-chunk counts h[0 .. 3*nchunks) (dgesdd-route, non-convergence, list-pass)
int sum_host_counts(const uint32_t *h, int64_t nchunks, int64_t *out)
{
    int64_t t = 0, bad = 0, slow = 0;
    for (int64_t c = 0; c < nchunks; ++c) {
        t += h[c];
        bad += h[nchunks + c];
        slow += h[2 * nchunks + c];
    }
    if (out) *out = t;
    t_list_pass = slow;
    if (bad)
        return fail(TMFWM_ERR_HIP, "dgesdd route: dbdsqr did not converge on %lld block(s) (np.linalg.svd raises LinAlgError there)",
                    (long long)bad);
    return 0;
}

// copy the per-chunk counts back (synchronises the stream) and sum them
int sum_counts(const uint32_t *dcounts, int64_t nchunks, hipStream_t st, int64_t *out)
{
    std::vector<uint32_t> h((size_t)(3 * nchunks));
    if (nchunks) {
        hipError_t e = hipMemcpyAsync(h.data(), dcounts, (size_t)nchunks * 12, hipMemcpyDeviceToHost, st);
        if (e == hipSuccess) e = hipStreamSynchronize(st);
        if (e != hipSuccess) {
            t_list_pass = -1;
            return fail(TMFWM_ERR_HIP, "reading the dgesdd-route counts failed: %s", hipGetErrorString(e));
        }
    }
    return sum_host_counts(h.data(), nchunks, out);
}

// Pinned landing zones for the per-chunk counts of host-memory calls: the counts travel with the
// call's last copy and are read after its one synchronisation (no extra round trip between the
// kernels and the copy back).  A small process-wide free list, so no thread keeps pinned memory.
constexpr int64_t kSinkChunks = 16;
std::mutex g_sink_mu;
std::vector<uint32_t *> g_sinks;

struct HostSink {
    uint32_t *p = nullptr;
    hipStream_t st = nullptr;
    HostSink(int64_t nchunks, hipStream_t s) : st(s)
    {
        if (nchunks > kSinkChunks) return;  // the synchronous read-back instead
        {
            std::lock_guard<std::mutex> g(g_sink_mu);
            if (!g_sinks.empty()) {
                p = g_sinks.back();
                g_sinks.pop_back();
                return;
            }
        }
        if (hipHostMalloc(reinterpret_cast<void **>(&p), kSinkChunks * 12, hipHostMallocDefault) != hipSuccess) {
            (void)hipGetLastError();
            p = nullptr;
        }
    }
    ~HostSink()
    {
        if (!p) return;
        (void)hipStreamSynchronize(st);  // an error return may leave the copy into it in flight
        (void)hipGetLastError();
        std::lock_guard<std::mutex> g(g_sink_mu);
        g_sinks.push_back(p);
    }
    HostSink(const HostSink &) = delete;
    HostSink &operator=(const HostSink &) = delete;
};

}  // namespace

namespace tmf {
int report(int code, const char *fmt, ...)
{
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    t_err = buf;
    return code;
}

void clear_error() { t_err.clear(); }

int check_frames(int64_t n, int32_t H, int32_t W, int64_t stride, int32_t block) { return ::check_frames(n, H, W, stride, block); }

// Both passes of embed over device-resident frames (a.src / a.dst / a.wm set).  The
// per-chunk counts (dgesdd-route blocks, dbdsqr non-convergence, list-pass blocks) are read
// back -- which synchronises the stream -- when the caller asks for the count (n_lapack) or
// when `check` is set (the host-memory calls, which synchronise anyway): a dbdsqr that did not
// converge then fails the call (np.linalg.svd raises LinAlgError there).  An asynchronous
// device-memory call without a count pointer is not checked (include/tmfwm.h).
int run_embed(EmbedArgs a, hipStream_t st, int64_t *n_lapack, bool check, uint32_t *sink = nullptr, int route = TMFWM_ROUTE_HYBRID)
{
    Chunks ch;
    ch.plan(a.nframes, (int64_t)a.nbh * a.nbw);
    DevBuf list, slow, shards, counts;
    if (ch.cap > 0) {
        if (int rc = list.alloc((size_t)ch.cap * 4, st, "dgesdd-route block list")) return rc;
        if ((embed_defers(a.block) && route != TMFWM_ROUTE_REFERENCE && route != TMFWM_ROUTE_RANK1_REFERENCE) ||
            (route == TMFWM_ROUTE_RANK1 && rank1_block(a.block))) {
            if (int rc = slow.alloc((size_t)ch.cap * 4, st, "list-pass block list")) return rc;
            if (int rc = shards.alloc((size_t)kListShards * kShardStride * 4, st, "list-pass segment counters")) return rc;
        }
        // per chunk: dgesdd-route count, non-convergence count, list-pass count
        if (int rc = counts.alloc((size_t)ch.n * 12, st, "block-list counts")) return rc;
        TMF_HIP(hipMemsetAsync(counts.p, 0, (size_t)ch.n * 12, st));
    }
    if (ch.cap == 0) {  // no full block: colour round trip only
        TMF_HIP(launch_embed(a, st));
        if (sink) std::fill(sink, sink + 3 * ch.n, 0u);
        if (n_lapack) {
            *n_lapack = 0;
            t_list_pass = 0;
        }
        return 0;
    }
    for (int64_t c = 0; c < ch.n; ++c) {
        EmbedArgs k = a;
        const int64_t f0 = c * ch.frames;
        k.nframes = a.nframes - f0 < ch.frames ? a.nframes - f0 : ch.frames;
        k.src = a.src + f0 * a.frame_stride;
        k.dst = a.dst + f0 * a.frame_stride;
        k.fb_list = static_cast<uint32_t *>(list.p);
        k.fb_count = static_cast<uint32_t *>(counts.p) + c;
        k.fb_bad = static_cast<uint32_t *>(counts.p) + ch.n + c;
        k.slow_list = static_cast<uint32_t *>(slow.p);  // null unless embed_defers(block)
        k.slow_count = static_cast<uint32_t *>(counts.p) + 2 * ch.n + c;
        k.slow_shards = static_cast<uint32_t *>(shards.p);
        if (shards.p) TMF_HIP(hipMemsetAsync(shards.p, 0, (size_t)kListShards * kShardStride * 4, st));
        const bool pre = (route == TMFWM_ROUTE_RANK1 || route == TMFWM_ROUTE_RANK1_REFERENCE) && rank1_block(k.block);
        if (route == TMFWM_ROUTE_REFERENCE || (route == TMFWM_ROUTE_RANK1_REFERENCE && !pre)) {
            // every block on the dgesdd route; the edges as always
            TMF_HIP(launch_edges(k.src, k.dst, k.nframes, k.H, k.W, k.frame_stride, k.block, st));
            TMF_HIP(launch_list_all(k.fb_list, k.fb_count, k.nframes * ch.per_frame, st));
        } else if (pre) {  // the rank-1 pre-pass (+ its list pass for TMFWM_ROUTE_RANK1), the edges
            if (route == TMFWM_ROUTE_RANK1_REFERENCE) k.slow_list = nullptr;
            TMF_HIP(launch_embed_rank1(k, st));
        } else {
            TMF_HIP(launch_embed(k, st));
        }
        TMF_HIP(launch_embed_fixup(k, k.fb_list, k.fb_count, k.nframes * ch.per_frame, st));
        if (force_nonconv()) TMF_HIP(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(k.fb_bad), 1, 1, st));
    }
    if (sink) {  // tmf::embed_device_async / extract_device_async: the caller sums after its sync
        TMF_HIP(hipMemcpyAsync(sink, counts.p, (size_t)ch.n * 12, hipMemcpyDeviceToHost, st));
        return 0;
    }
    if (n_lapack || check) return sum_counts(static_cast<const uint32_t *>(counts.p), ch.n, st, n_lapack);
    return 0;
}

int run_extract(ExtractArgs a, hipStream_t st, int64_t *n_lapack, bool check, uint32_t *sink = nullptr,
                int route = TMFWM_ROUTE_HYBRID)
{
    Chunks ch;
    ch.plan(a.nframes, (int64_t)a.nbh * a.nbw);
    if (ch.cap == 0) {
        if (sink) std::fill(sink, sink + 3 * ch.n, 0u);
        if (n_lapack) {
            *n_lapack = 0;
            t_list_pass = 0;
        }
        return 0;
    }
    DevBuf list, slow, shards, counts;
    if (int rc = list.alloc((size_t)ch.cap * 4, st, "dgesdd-route block list")) return rc;
    if (route != TMFWM_ROUTE_REFERENCE) {  // hybrid (TMFWM_ROUTE_RANK1: extract is the hybrid route)
        if (int rc = slow.alloc((size_t)ch.cap * 4, st, "list-pass block list")) return rc;
        if (int rc = shards.alloc((size_t)kListShards * kShardStride * 4, st, "list-pass segment counters")) return rc;
    }
    if (int rc = counts.alloc((size_t)ch.n * 12, st, "block-list counts")) return rc;  // as run_embed's
    TMF_HIP(hipMemsetAsync(counts.p, 0, (size_t)ch.n * 12, st));
    for (int64_t c = 0; c < ch.n; ++c) {
        ExtractArgs k = a;
        const int64_t f0 = c * ch.frames;
        k.nframes = a.nframes - f0 < ch.frames ? a.nframes - f0 : ch.frames;
        k.wsrc = a.wsrc + f0 * a.frame_stride;
        k.osrc = a.osrc + f0 * a.frame_stride;
        k.out = a.out + f0 * a.tile_stride;
        k.fb_list = static_cast<uint32_t *>(list.p);
        k.fb_count = static_cast<uint32_t *>(counts.p) + c;
        k.fb_bad = static_cast<uint32_t *>(counts.p) + ch.n + c;
        k.slow_list = static_cast<uint32_t *>(slow.p);
        k.slow_count = static_cast<uint32_t *>(counts.p) + 2 * ch.n + c;
        k.slow_shards = static_cast<uint32_t *>(shards.p);
        if (shards.p) TMF_HIP(hipMemsetAsync(shards.p, 0, (size_t)kListShards * kShardStride * 4, st));
        if (route == TMFWM_ROUTE_REFERENCE) TMF_HIP(launch_list_all(k.fb_list, k.fb_count, k.nframes * ch.per_frame, st));
        else TMF_HIP(launch_extract(k, st));
        TMF_HIP(launch_extract_fixup(k, k.fb_list, k.fb_count, k.nframes * ch.per_frame, st));
        if (force_nonconv()) TMF_HIP(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(k.fb_bad), 1, 1, st));
    }
    if (sink) {  // tmf::embed_device_async / extract_device_async: the caller sums after its sync
        TMF_HIP(hipMemcpyAsync(sink, counts.p, (size_t)ch.n * 12, hipMemcpyDeviceToHost, st));
        return 0;
    }
    if (n_lapack || check) return sum_counts(static_cast<const uint32_t *>(counts.p), ch.n, st, n_lapack);
    return 0;
}
EmbedArgs embed_args(int64_t n, int32_t H, int32_t W, int64_t stride, int32_t block, double alpha)
{
    EmbedArgs a{};
    a.nframes = n;
    a.frame_stride = stride;
    a.H = H;
    a.W = W;
    a.block = block;
    a.nbh = H / block;
    a.nbw = W / block;
    a.alpha = alpha;
    return a;
}

ExtractArgs extract_args(int64_t n, int32_t H, int32_t W, int64_t stride, int32_t block, double alpha)
{
    ExtractArgs a{};
    a.nframes = n;
    a.frame_stride = stride;
    a.tile_stride = (int64_t)(H / block) * (W / block);
    a.H = H;
    a.W = W;
    a.block = block;
    a.nbh = H / block;
    a.nbw = W / block;
    a.alpha32 = (float)alpha;
    return a;
}

bool dev_aligned(const void *p, const void *q, int64_t stride, int W)
{
    return ((reinterpret_cast<uintptr_t>(p) | reinterpret_cast<uintptr_t>(q)) % 4 == 0) && stride % 4 == 0 && W % 4 == 0;
}

int64_t count_chunks(int64_t nframes, int H, int W, int block)
{
    Chunks ch;
    ch.plan(nframes, (int64_t)(H / block) * (W / block));
    return ch.n;
}

int embed_device_async(const uint8_t *src, int64_t n, int H, int W, int64_t stride, const uint8_t *tile, int block,
                       double alpha, uint8_t *dst, hipStream_t st, uint32_t *sink, int route)
{
    if (int rc = ::check_frames(n, H, W, stride, block)) return rc;
    if (n == 0 || H == 0 || W == 0) {
        std::fill(sink, sink + 3 * count_chunks(n, H, W, block), 0u);
        return 0;
    }
    EmbedArgs a = embed_args(n, H, W, stride, block, alpha);
    a.src = src;
    a.dst = dst;
    a.wm = tile;
    a.aligned = dev_aligned(src, dst, stride, W);
    return run_embed(a, st, nullptr, false, sink, route);
}

int extract_device_async(const uint8_t *wsrc, const uint8_t *osrc, int64_t n, int H, int W, int64_t stride, int block,
                         double alpha, uint8_t *out, hipStream_t st, uint32_t *sink, int route)
{
    if (int rc = ::check_frames(n, H, W, stride, block)) return rc;
    if (n == 0 || (H / block) * (W / block) == 0) {
        std::fill(sink, sink + 3 * count_chunks(n, H, W, block), 0u);
        return 0;
    }
    ExtractArgs a = extract_args(n, H, W, stride, block, alpha);
    a.wsrc = wsrc;
    a.osrc = osrc;
    a.out = out;
    a.aligned = dev_aligned(wsrc, osrc, stride, W);
    return run_extract(a, st, nullptr, false, sink, route);
}

int sum_sink(const uint32_t *sink, int64_t nchunks, int64_t *lapack) { return sum_host_counts(sink, nchunks, lapack); }
}  // namespace tmf

extern "C" {

int tmfwm_abi_version(void) { return TMFWM_ABI_VERSION; }

const char *tmfwm_last_error(void) { return t_err.c_str(); }

int64_t tmfwm_last_list_pass_blocks(void) { return t_list_pass; }

int tmfwm_embed_list_pass(int32_t block) { return supported_block(block) && tmf::embed_defers(block) ? 1 : 0; }

int tmfwm_device_count(void)
{
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) {
        (void)hipGetLastError();
        return 0;
    }
    return n;
}

int tmfwm_embed_route(const uint8_t *rgb, int64_t n_frames, int32_t height, int32_t width, int64_t frame_stride,
                      const uint8_t *wm_tile, int32_t block, double alpha, uint8_t *out, int32_t mem_kind, void *hip_stream,
                      int32_t route, int64_t *n_lapack_blocks)
{
    t_err.clear();
    if (route < TMFWM_ROUTE_HYBRID || route > TMFWM_ROUTE_RANK1_REFERENCE) return fail(TMFWM_ERR_INVALID, "route %d", route);
    if (n_lapack_blocks) {
        *n_lapack_blocks = 0;
        t_list_pass = 0;  // this call's count from here on (an early return leaves 0)
    }
    if (int rc = check_frames(n_frames, height, width, frame_stride, block)) return rc;
    if (!std::isfinite(alpha)) return fail(TMFWM_ERR_INVALID, "alpha is not finite");
    if (int rc = need_device()) return rc;
    if (n_frames == 0 || height == 0 || width == 0) return 0;
    const int nbh = height / block, nbw = width / block;
    const int64_t fbytes = (int64_t)height * width * 3;
    const size_t span = span_bytes(n_frames, frame_stride, fbytes), tbytes = (size_t)nbh * nbw;
    hipStream_t st = pick_stream(hip_stream);
    tmf::EmbedArgs a = tmf::embed_args(n_frames, height, width, frame_stride, block, alpha);
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
        a.aligned = tmf::dev_aligned(rgb, out, frame_stride, width);
        return tmf::run_embed(a, st, n_lapack_blocks, false, nullptr, route);
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
    const int64_t nch = tmf::count_chunks(n_frames, height, width, block);
    HostSink sink(nch, st);
    if (int rc = tmf::run_embed(a, st, n_lapack_blocks, true, sink.p, route)) return rc;
    if (frame_stride == fbytes) {
        TMF_HIP(hipMemcpyAsync(out, dout.p, span, hipMemcpyDeviceToHost, st));
    } else {
        for (int64_t f = 0; f < n_frames; ++f)
            TMF_HIP(hipMemcpyAsync(out + f * frame_stride, static_cast<uint8_t *>(dout.p) + f * frame_stride, (size_t)fbytes,
                                   hipMemcpyDeviceToHost, st));
    }
    TMF_HIP(hipStreamSynchronize(st));
    return sink.p ? tmf::sum_sink(sink.p, nch, n_lapack_blocks) : 0;
}

int tmfwm_embed_ex(const uint8_t *rgb, int64_t n_frames, int32_t height, int32_t width, int64_t frame_stride,
                   const uint8_t *wm_tile, int32_t block, double alpha, uint8_t *out, int32_t mem_kind, void *hip_stream,
                   int64_t *n_lapack_blocks)
{
    return tmfwm_embed_route(rgb, n_frames, height, width, frame_stride, wm_tile, block, alpha, out, mem_kind, hip_stream,
                             TMFWM_ROUTE_HYBRID, n_lapack_blocks);
}

int tmfwm_embed(const uint8_t *rgb, int64_t n_frames, int32_t height, int32_t width, int64_t frame_stride,
                const uint8_t *wm_tile, int32_t block, double alpha, uint8_t *out, int32_t mem_kind, void *hip_stream)
{
    return tmfwm_embed_ex(rgb, n_frames, height, width, frame_stride, wm_tile, block, alpha, out, mem_kind, hip_stream, nullptr);
}

int tmfwm_extract_route(const uint8_t *wm_rgb, const uint8_t *orig_rgb, int64_t n_frames, int32_t height, int32_t width,
                        int64_t frame_stride, int32_t block, double alpha, uint8_t *out_tiles, int32_t mem_kind,
                        void *hip_stream, int32_t route, int64_t *n_lapack_blocks)
{
    t_err.clear();
    if (route < TMFWM_ROUTE_HYBRID || route > TMFWM_ROUTE_RANK1_REFERENCE) return fail(TMFWM_ERR_INVALID, "route %d", route);
    if (n_lapack_blocks) {
        *n_lapack_blocks = 0;
        t_list_pass = 0;  // this call's count from here on (an early return leaves 0)
    }
    if (int rc = check_frames(n_frames, height, width, frame_stride, block)) return rc;
    if (!std::isfinite(alpha) || alpha == 0.0) return fail(TMFWM_ERR_INVALID, "alpha must be finite and non-zero");
    if (int rc = need_device()) return rc;
    const int nbh = height / block, nbw = width / block;
    const int64_t tbytes = (int64_t)nbh * nbw;
    if (n_frames == 0 || tbytes == 0) return 0;
    const int64_t fbytes = (int64_t)height * width * 3;
    const size_t span = span_bytes(n_frames, frame_stride, fbytes);
    hipStream_t st = pick_stream(hip_stream);
    tmf::ExtractArgs a = tmf::extract_args(n_frames, height, width, frame_stride, block, alpha);
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
        a.aligned = tmf::dev_aligned(wm_rgb, orig_rgb, frame_stride, width);
        return tmf::run_extract(a, st, n_lapack_blocks, false, nullptr, route);
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
    const int64_t nch = tmf::count_chunks(n_frames, height, width, block);
    HostSink sink(nch, st);
    if (int rc = tmf::run_extract(a, st, n_lapack_blocks, true, sink.p, route)) return rc;
    TMF_HIP(hipMemcpyAsync(out_tiles, dout.p, (size_t)(tbytes * n_frames), hipMemcpyDeviceToHost, st));
    TMF_HIP(hipStreamSynchronize(st));
    return sink.p ? tmf::sum_sink(sink.p, nch, n_lapack_blocks) : 0;
}

int tmfwm_extract_ex(const uint8_t *wm_rgb, const uint8_t *orig_rgb, int64_t n_frames, int32_t height, int32_t width,
                     int64_t frame_stride, int32_t block, double alpha, uint8_t *out_tiles, int32_t mem_kind, void *hip_stream,
                     int64_t *n_lapack_blocks)
{
    return tmfwm_extract_route(wm_rgb, orig_rgb, n_frames, height, width, frame_stride, block, alpha, out_tiles, mem_kind,
                               hip_stream, TMFWM_ROUTE_HYBRID, n_lapack_blocks);
}

int tmfwm_extract(const uint8_t *wm_rgb, const uint8_t *orig_rgb, int64_t n_frames, int32_t height, int32_t width,
                  int64_t frame_stride, int32_t block, double alpha, uint8_t *out_tiles, int32_t mem_kind, void *hip_stream)
{
    return tmfwm_extract_ex(wm_rgb, orig_rgb, n_frames, height, width, frame_stride, block, alpha, out_tiles, mem_kind,
                            hip_stream, nullptr);
}

// ---- 4-byte pixels (ABI 8): the core runs on compact RGB device buffers; RGBX inputs are
// packed and RGBX outputs unpacked on the device (tmfwm_pixels.hip)
extern "C++" {
namespace {
int check_px(int32_t px, int64_t stride, int32_t H, int32_t W, const char *what)
{
    if (px != TMFWM_PIX_RGB && px != TMFWM_PIX_RGBX) return fail(TMFWM_ERR_INVALID, "%s pixel bytes %d (3 or 4)", what, px);
    if (stride < (int64_t)H * W * px) return fail(TMFWM_ERR_INVALID, "%s frame_stride %lld < H*W*%d", what, (long long)stride, px);
    return 0;
}

// frames (host or device, 3 or 4 bytes per pixel) -> device RGB with stride *s3; buf / tmp own
// whatever had to be allocated
int device_rgb(const uint8_t *src, int32_t px, int64_t stride, int64_t n, int32_t H, int32_t W, int32_t mem_kind,
               hipStream_t st, const char *what, DevBuf &buf, DevBuf &tmp, const uint8_t **out, int64_t *s3)
{
    const int64_t f3 = (int64_t)H * W * 3;
    const size_t span = span_bytes(n, stride, (int64_t)H * W * px);
    const uint8_t *p = src;
    if (mem_kind == TMFWM_MEM_DEVICE) {
        if (int rc = check_device_ptr(src, what)) return rc;
    } else {
        if (!src) return fail(TMFWM_ERR_INVALID, "NULL host pointer (%s)", what);
        if (int rc = (px == 3 ? buf : tmp).alloc(span, st, what)) return rc;
        p = static_cast<const uint8_t *>((px == 3 ? buf : tmp).p);
        TMF_HIP(hipMemcpyAsync(const_cast<uint8_t *>(p), src, span, hipMemcpyHostToDevice, st));
    }
    if (px == 3) {
        *out = p;
        *s3 = stride;
        return 0;
    }
    if (int rc = buf.alloc((size_t)(n * f3), st, what)) return rc;
    TMF_HIP(tmf::launch_pack_rgbx(p, stride, static_cast<uint8_t *>(buf.p), f3, n, H, W, st));
    *out = static_cast<const uint8_t *>(buf.p);
    *s3 = f3;
    return 0;
}
}  // namespace
}  // extern "C++"

int tmfwm_embed_px(const uint8_t *rgb, int32_t in_pixel_bytes, int64_t in_frame_stride, int64_t n_frames, int32_t height,
                   int32_t width, const uint8_t *wm_tile, int32_t block, double alpha, uint8_t *out, int32_t out_pixel_bytes,
                   int64_t out_frame_stride, int32_t mem_kind, void *hip_stream, int32_t route, int64_t *n_lapack_blocks)
{
    t_err.clear();
    if (in_pixel_bytes == TMFWM_PIX_RGB && out_pixel_bytes == TMFWM_PIX_RGB) {
        if (in_frame_stride != out_frame_stride) return fail(TMFWM_ERR_INVALID, "3-byte input and output need one frame_stride");
        return tmfwm_embed_route(rgb, n_frames, height, width, in_frame_stride, wm_tile, block, alpha, out, mem_kind, hip_stream,
                                 route, n_lapack_blocks);
    }
    if (route < TMFWM_ROUTE_HYBRID || route > TMFWM_ROUTE_RANK1_REFERENCE) return fail(TMFWM_ERR_INVALID, "route %d", route);
    if (n_lapack_blocks) {
        *n_lapack_blocks = 0;
        t_list_pass = 0;
    }
    if (int rc = check_frames(n_frames, height, width, (int64_t)height * width * 3, block)) return rc;
    if (int rc = check_px(in_pixel_bytes, in_frame_stride, height, width, "input")) return rc;
    if (int rc = check_px(out_pixel_bytes, out_frame_stride, height, width, "output")) return rc;
    if (!std::isfinite(alpha)) return fail(TMFWM_ERR_INVALID, "alpha is not finite");
    if (mem_kind != TMFWM_MEM_HOST && mem_kind != TMFWM_MEM_DEVICE) return fail(TMFWM_ERR_INVALID, "mem_kind %d", mem_kind);
    if (int rc = need_device()) return rc;
    if (n_frames == 0 || height == 0 || width == 0) return 0;
    const int nbh = height / block, nbw = width / block;
    const size_t tbytes = (size_t)nbh * nbw;
    const int64_t f3 = (int64_t)height * width * 3, fo = (int64_t)height * width * out_pixel_bytes;
    const size_t ospan = span_bytes(n_frames, out_frame_stride, fo);
    hipStream_t st = pick_stream(hip_stream);
    if (mem_kind == TMFWM_MEM_DEVICE) {
        if (int rc = check_device_ptr(out, "out")) return rc;
        if (ranges_overlap(rgb, span_bytes(n_frames, in_frame_stride, (int64_t)height * width * in_pixel_bytes), out, ospan))
            return fail(TMFWM_ERR_INVALID, "out overlaps rgb (in-place embed is not supported)");
        if (tbytes) {
            if (int rc = check_device_ptr(wm_tile, "wm_tile")) return rc;
        }
    } else if (!out || (tbytes && !wm_tile)) {
        return fail(TMFWM_ERR_INVALID, "NULL host pointer");
    }
    DevBuf src3, tmp, dst3, dst4, dwm;
    const uint8_t *s3p = nullptr;
    int64_t s3 = 0;
    if (int rc = device_rgb(rgb, in_pixel_bytes, in_frame_stride, n_frames, height, width, mem_kind, st, "input frames", src3, tmp,
                            &s3p, &s3))
        return rc;
    const uint8_t *wm = wm_tile;
    if (mem_kind == TMFWM_MEM_HOST && tbytes) {
        if (int rc = dwm.alloc(tbytes, st, "watermark tile")) return rc;
        TMF_HIP(hipMemcpyAsync(dwm.p, wm_tile, tbytes, hipMemcpyHostToDevice, st));
        wm = static_cast<const uint8_t *>(dwm.p);
    }
    if (int rc = dst3.alloc(span_bytes(n_frames, s3, f3), st, "output frames")) return rc;
    tmf::EmbedArgs a = tmf::embed_args(n_frames, height, width, s3, block, alpha);
    a.src = s3p;
    a.dst = static_cast<uint8_t *>(dst3.p);
    a.wm = wm;
    a.aligned = tmf::dev_aligned(a.src, a.dst, s3, width);
    const int64_t nch = tmf::count_chunks(n_frames, height, width, block);
    HostSink sink(mem_kind == TMFWM_MEM_HOST ? nch : kSinkChunks + 1, st);
    if (int rc = tmf::run_embed(a, st, n_lapack_blocks, mem_kind == TMFWM_MEM_HOST, sink.p, route)) return rc;
    uint8_t *o = out;  // device destination of the output's final layout
    if (mem_kind == TMFWM_MEM_HOST) {
        if (int rc = dst4.alloc(ospan, st, "output staging")) return rc;
        o = static_cast<uint8_t *>(dst4.p);
    }
    if (out_pixel_bytes == TMFWM_PIX_RGBX)
        TMF_HIP(tmf::launch_unpack_rgbx(a.dst, s3, o, out_frame_stride, n_frames, height, width, st));
    else
        TMF_HIP(hipMemcpy2DAsync(o, (size_t)out_frame_stride, a.dst, (size_t)s3, (size_t)f3, (size_t)n_frames,
                                 hipMemcpyDeviceToDevice, st));
    if (mem_kind == TMFWM_MEM_HOST) {  // the caller's bytes between frames stay as they are
        if (n_frames == 1 || out_frame_stride == fo)
            TMF_HIP(hipMemcpyAsync(out, o, ospan, hipMemcpyDeviceToHost, st));
        else
            TMF_HIP(hipMemcpy2DAsync(out, (size_t)out_frame_stride, o, (size_t)out_frame_stride, (size_t)fo, (size_t)n_frames,
                                     hipMemcpyDeviceToHost, st));
        TMF_HIP(hipStreamSynchronize(st));
        if (sink.p) return tmf::sum_sink(sink.p, nch, n_lapack_blocks);
    }
    return 0;
}

int tmfwm_extract_px(const uint8_t *wm_rgb, int32_t wm_pixel_bytes, int64_t wm_frame_stride, const uint8_t *orig_rgb,
                     int32_t orig_pixel_bytes, int64_t orig_frame_stride, int64_t n_frames, int32_t height, int32_t width,
                     int32_t block, double alpha, uint8_t *out_tiles, int32_t mem_kind, void *hip_stream, int32_t route,
                     int64_t *n_lapack_blocks)
{
    t_err.clear();
    if (wm_pixel_bytes == TMFWM_PIX_RGB && orig_pixel_bytes == TMFWM_PIX_RGB && wm_frame_stride == orig_frame_stride)
        return tmfwm_extract_route(wm_rgb, orig_rgb, n_frames, height, width, wm_frame_stride, block, alpha, out_tiles, mem_kind,
                                   hip_stream, route, n_lapack_blocks);
    if (route < TMFWM_ROUTE_HYBRID || route > TMFWM_ROUTE_RANK1_REFERENCE) return fail(TMFWM_ERR_INVALID, "route %d", route);
    if (n_lapack_blocks) {
        *n_lapack_blocks = 0;
        t_list_pass = 0;
    }
    if (int rc = check_frames(n_frames, height, width, (int64_t)height * width * 3, block)) return rc;
    if (int rc = check_px(wm_pixel_bytes, wm_frame_stride, height, width, "watermarked")) return rc;
    if (int rc = check_px(orig_pixel_bytes, orig_frame_stride, height, width, "original")) return rc;
    if (!std::isfinite(alpha) || alpha == 0.0) return fail(TMFWM_ERR_INVALID, "alpha must be finite and non-zero");
    if (mem_kind != TMFWM_MEM_HOST && mem_kind != TMFWM_MEM_DEVICE) return fail(TMFWM_ERR_INVALID, "mem_kind %d", mem_kind);
    if (int rc = need_device()) return rc;
    const int nbh = height / block, nbw = width / block;
    const int64_t tbytes = (int64_t)nbh * nbw, f3 = (int64_t)height * width * 3;
    if (n_frames == 0 || tbytes == 0) return 0;
    const size_t obytes = (size_t)(tbytes * n_frames);
    hipStream_t st = pick_stream(hip_stream);
    if (mem_kind == TMFWM_MEM_DEVICE) {
        if (int rc = check_device_ptr(out_tiles, "out_tiles")) return rc;
        if (ranges_overlap(out_tiles, obytes, wm_rgb, span_bytes(n_frames, wm_frame_stride, (int64_t)height * width * wm_pixel_bytes)) ||
            ranges_overlap(out_tiles, obytes, orig_rgb, span_bytes(n_frames, orig_frame_stride, (int64_t)height * width * orig_pixel_bytes)))
            return fail(TMFWM_ERR_INVALID, "out_tiles overlaps an input batch");
    } else if (!out_tiles) {
        return fail(TMFWM_ERR_INVALID, "NULL host pointer");
    }
    // both images as compact RGB (one frame stride for the kernels)
    DevBuf w3, wtmp, o3, otmp, wc, oc, dout;
    const uint8_t *wp = nullptr, *op = nullptr;
    int64_t ws = 0, os = 0;
    if (int rc = device_rgb(wm_rgb, wm_pixel_bytes, wm_frame_stride, n_frames, height, width, mem_kind, st, "watermarked frames", w3,
                            wtmp, &wp, &ws))
        return rc;
    if (int rc = device_rgb(orig_rgb, orig_pixel_bytes, orig_frame_stride, n_frames, height, width, mem_kind, st, "original frames",
                            o3, otmp, &op, &os))
        return rc;
    if (ws != f3) {
        if (int rc = wc.alloc((size_t)(n_frames * f3), st, "watermarked frames")) return rc;
        TMF_HIP(hipMemcpy2DAsync(wc.p, (size_t)f3, wp, (size_t)ws, (size_t)f3, (size_t)n_frames, hipMemcpyDeviceToDevice, st));
        wp = static_cast<const uint8_t *>(wc.p);
    }
    if (os != f3) {
        if (int rc = oc.alloc((size_t)(n_frames * f3), st, "original frames")) return rc;
        TMF_HIP(hipMemcpy2DAsync(oc.p, (size_t)f3, op, (size_t)os, (size_t)f3, (size_t)n_frames, hipMemcpyDeviceToDevice, st));
        op = static_cast<const uint8_t *>(oc.p);
    }
    tmf::ExtractArgs a = tmf::extract_args(n_frames, height, width, f3, block, alpha);
    a.wsrc = wp;
    a.osrc = op;
    if (mem_kind == TMFWM_MEM_HOST) {
        if (int rc = dout.alloc(obytes, st, "extracted tiles")) return rc;
        a.out = static_cast<uint8_t *>(dout.p);
    } else {
        a.out = out_tiles;
    }
    a.aligned = tmf::dev_aligned(wp, op, f3, width);
    const int64_t nch = tmf::count_chunks(n_frames, height, width, block);
    HostSink sink(mem_kind == TMFWM_MEM_HOST ? nch : kSinkChunks + 1, st);
    if (int rc = tmf::run_extract(a, st, n_lapack_blocks, mem_kind == TMFWM_MEM_HOST, sink.p, route)) return rc;
    if (mem_kind == TMFWM_MEM_HOST) {
        TMF_HIP(hipMemcpyAsync(out_tiles, dout.p, obytes, hipMemcpyDeviceToHost, st));
        TMF_HIP(hipStreamSynchronize(st));
        if (sink.p) return tmf::sum_sink(sink.p, nch, n_lapack_blocks);
    }
    return 0;
}

extern "C++" {
namespace {

// One elementwise colour helper: in_bytes / out_bytes per pixel; launch(in, out, st)
// on device pointers.  Host calls stage through library-pool memory.
template <typename Launch>
int colour_helper(const void *in, int64_t npix, size_t in_px, void *out, size_t out_px, int32_t mem_kind, void *hip_stream,
                  Launch launch)
{
    t_err.clear();
    if (npix < 0) return fail(TMFWM_ERR_INVALID, "npix < 0");
    if (npix == 0) return 0;
    if (int rc = need_device()) return rc;
    hipStream_t st = pick_stream(hip_stream);
    if (mem_kind == TMFWM_MEM_DEVICE) {
        if (int rc = check_device_ptr(in, "input")) return rc;
        if (int rc = check_device_ptr(out, "output")) return rc;
        TMF_HIP(launch(in, out, st));
        return 0;
    }
    if (mem_kind != TMFWM_MEM_HOST || !in || !out) return fail(TMFWM_ERR_INVALID, "bad host arguments");
    DevBuf di, dout;
    if (int rc = di.alloc((size_t)npix * in_px, st, "input pixels")) return rc;
    if (int rc = dout.alloc((size_t)npix * out_px, st, "output pixels")) return rc;
    TMF_HIP(hipMemcpyAsync(di.p, in, (size_t)npix * in_px, hipMemcpyHostToDevice, st));
    TMF_HIP(launch(di.p, dout.p, st));
    TMF_HIP(hipMemcpyAsync(out, dout.p, (size_t)npix * out_px, hipMemcpyDeviceToHost, st));
    TMF_HIP(hipStreamSynchronize(st));
    return 0;
}

size_t dtype_bytes(int32_t dtype)
{
    switch (dtype) {
    case TMFWM_DT_F16: return 2;
    case TMFWM_DT_F32: return 4;
    case TMFWM_DT_F64: return 8;
    default: return 0;
    }
}

}  // namespace
}  // extern "C++"

int tmfwm_rgb_to_ycbcr(const uint8_t *rgb, int64_t npix, float *ycc, int32_t mem_kind, void *hip_stream)
{
    return colour_helper(rgb, npix, 3, ycc, 12, mem_kind, hip_stream, [npix](const void *i, void *o, hipStream_t st) {
        return tmf::launch_rgb_to_ycbcr(static_cast<const uint8_t *>(i), npix, static_cast<float *>(o), st);
    });
}

int tmfwm_rgb_to_ycbcr_f32(const float *rgb, int64_t npix, float *ycc, int32_t mem_kind, void *hip_stream)
{
    return colour_helper(rgb, npix, 12, ycc, 12, mem_kind, hip_stream, [npix](const void *i, void *o, hipStream_t st) {
        return tmf::launch_rgb_to_ycbcr_f32(static_cast<const float *>(i), npix, static_cast<float *>(o), st);
    });
}

int tmfwm_ycbcr_to_rgb_typed(const void *ycc, int32_t dtype, int64_t npix, uint8_t *rgb, int32_t mem_kind, void *hip_stream)
{
    const size_t eb = dtype_bytes(dtype);
    if (!eb) {
        t_err.clear();
        return fail(TMFWM_ERR_INVALID, "dtype %d (TMFWM_DT_F16 / _F32 / _F64)", dtype);
    }
    return colour_helper(ycc, npix, 3 * eb, rgb, 3, mem_kind, hip_stream, [npix, dtype](const void *i, void *o, hipStream_t st) {
        return tmf::launch_ycbcr_to_rgb(i, dtype, npix, static_cast<uint8_t *>(o), st);
    });
}

int tmfwm_ycbcr_to_rgb(const float *ycc, int64_t npix, uint8_t *rgb, int32_t mem_kind, void *hip_stream)
{
    return tmfwm_ycbcr_to_rgb_typed(ycc, TMFWM_DT_F32, npix, rgb, mem_kind, hip_stream);
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

int tmfwm_lapack_svd_blocks(const float *D, int64_t n_blocks, int32_t block, float *U, float *S, float *Vt, int32_t want_vectors,
                            int32_t mem_kind, void *hip_stream)
{
    t_err.clear();
    if (n_blocks < 0) return fail(TMFWM_ERR_INVALID, "n_blocks < 0");
    if (int rc = check_frames(0, 0, 0, 0, block)) return rc;
    if (int rc = need_device()) return rc;
    if (n_blocks == 0) return 0;
    hipStream_t st = pick_stream(hip_stream);
    const size_t mb = (size_t)n_blocks * block * block * sizeof(float), sb = (size_t)n_blocks * block * sizeof(float);
    DevBuf dinfo;
    if (int rc = dinfo.alloc((size_t)n_blocks * 4, st, "info")) return rc;
    int32_t *info = static_cast<int32_t *>(dinfo.p);
    const float *dD = D;
    float *dU = U, *dS = S, *dVt = Vt;
    DevBuf bD, bU, bS, bV;
    if (mem_kind == TMFWM_MEM_DEVICE) {
        if (int rc = check_device_ptr(D, "D")) return rc;
        if (int rc = check_device_ptr(S, "S")) return rc;
        if (want_vectors) {
            if (int rc = check_device_ptr(U, "U")) return rc;
            if (int rc = check_device_ptr(Vt, "Vt")) return rc;
        }
    } else {
        if (mem_kind != TMFWM_MEM_HOST || !D || !S || (want_vectors && (!U || !Vt))) return fail(TMFWM_ERR_INVALID, "bad host arguments");
        if (int rc = bD.alloc(mb, st, "D")) return rc;
        if (int rc = bS.alloc(sb, st, "S")) return rc;
        if (want_vectors) {
            if (int rc = bU.alloc(mb, st, "U")) return rc;
            if (int rc = bV.alloc(mb, st, "Vt")) return rc;
        }
        TMF_HIP(hipMemcpyAsync(bD.p, D, mb, hipMemcpyHostToDevice, st));
        dD = static_cast<const float *>(bD.p);
        dS = static_cast<float *>(bS.p);
        dU = static_cast<float *>(bU.p);
        dVt = static_cast<float *>(bV.p);
    }
    TMF_HIP(tmf::launch_lapack_svd_blocks(dD, n_blocks, block, dU, dS, dVt, want_vectors != 0, info, st));
    if (mem_kind == TMFWM_MEM_HOST) {
        TMF_HIP(hipMemcpyAsync(S, dS, sb, hipMemcpyDeviceToHost, st));
        if (want_vectors) {
            TMF_HIP(hipMemcpyAsync(U, dU, mb, hipMemcpyDeviceToHost, st));
            TMF_HIP(hipMemcpyAsync(Vt, dVt, mb, hipMemcpyDeviceToHost, st));
        }
    }
    // dbdsqr's convergence flag of every block (LAPACK's info > 0): reported, never silent
    std::vector<int32_t> h((size_t)n_blocks);
    TMF_HIP(hipMemcpyAsync(h.data(), info, (size_t)n_blocks * 4, hipMemcpyDeviceToHost, st));
    TMF_HIP(hipStreamSynchronize(st));
    for (int64_t k = 0; k < n_blocks; ++k)
        if (h[(size_t)k]) return fail(TMFWM_ERR_INVALID, "dbdsqr did not converge on block %lld", (long long)k);
    return 0;
}

int tmfwm_lapack_nrm2(const double *x, int64_t n_vectors, int32_t n, int32_t inc, double *out, int32_t mem_kind, void *hip_stream)
{
    t_err.clear();
    if (n_vectors < 0 || n < 0 || inc < 1) return fail(TMFWM_ERR_INVALID, "bad sizes");
    if (int rc = need_device()) return rc;
    if (n_vectors == 0) return 0;
    hipStream_t st = pick_stream(hip_stream);
    const size_t xb = (size_t)n_vectors * n * inc * sizeof(double), ob = (size_t)n_vectors * sizeof(double);
    if (mem_kind == TMFWM_MEM_DEVICE) {
        if (xb)
            if (int rc = check_device_ptr(x, "x")) return rc;
        if (int rc = check_device_ptr(out, "out")) return rc;
        TMF_HIP(tmf::launch_lapack_nrm2(x, n_vectors, n, inc, out, st));
        return 0;
    }
    if (mem_kind != TMFWM_MEM_HOST || !out || (xb && !x)) return fail(TMFWM_ERR_INVALID, "bad host arguments");
    DevBuf dx, dout;
    if (int rc = dx.alloc(xb, st, "x")) return rc;
    if (int rc = dout.alloc(ob, st, "out")) return rc;
    if (xb) TMF_HIP(hipMemcpyAsync(dx.p, x, xb, hipMemcpyHostToDevice, st));
    TMF_HIP(tmf::launch_lapack_nrm2(static_cast<const double *>(dx.p), n_vectors, n, inc, static_cast<double *>(dout.p), st));
    TMF_HIP(hipMemcpyAsync(out, dout.p, ob, hipMemcpyDeviceToHost, st));
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
