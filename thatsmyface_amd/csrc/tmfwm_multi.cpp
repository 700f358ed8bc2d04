// Multi-GPU entry points of the C ABI (include/tmfwm.h: tmfwm_embed_multi,
// tmfwm_extract_multi) for callers without torch.distributed: one process drives
// several MI355X devices.
//
// The batch is split into contiguous frame shards (thatsmyface_amd.dist.shard_range's
// split: sizes differ by at most one), one host thread and one HIP stream per shard.  The
// frames are independent (watermarking.py:183-210: no halo, no inter-block dependency),
// so there is no data-path collective.  The one exchange is the watermark tile: it is
// copied to the first shard's device and broadcast to every other device with RCCL
// (ncclBroadcast over xGMI, communicators from ncclCommInitAll, cached per device set).
// Shards that share a device (logical shards, e.g. several shards on a one-GPU box) share
// that device's copy of the tile.
//
// librccl is opened on first use (dlopen), so libtmfwm.so itself keeps no link-time
// dependency on it; under torch the already-loaded librccl.so.1 is reused.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <dlfcn.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <map>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/tmfwm.h"
#include "tmfwm_internal.h"

namespace {

using tmf::report;

// ---- RCCL, resolved at run time -------------------------------------------------
struct Rccl {
    decltype(&ncclCommInitAll) comm_init_all = nullptr;
    decltype(&ncclBroadcast) broadcast = nullptr;
    decltype(&ncclGroupStart) group_start = nullptr;
    decltype(&ncclGroupEnd) group_end = nullptr;
    decltype(&ncclGetErrorString) error_string = nullptr;
    std::string why;  // empty when loaded

    static Rccl &get()
    {
        static Rccl r = load();
        return r;
    }
    bool ok() const { return why.empty(); }

private:
    static Rccl load()
    {
        Rccl r;
        void *h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
        if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
        if (!h) {
            const char *e = dlerror();
            r.why = std::string("librccl.so.1 not loadable: ") + (e ? e : "?");
            return r;
        }
        r.comm_init_all = reinterpret_cast<decltype(r.comm_init_all)>(dlsym(h, "ncclCommInitAll"));
        r.broadcast = reinterpret_cast<decltype(r.broadcast)>(dlsym(h, "ncclBroadcast"));
        r.group_start = reinterpret_cast<decltype(r.group_start)>(dlsym(h, "ncclGroupStart"));
        r.group_end = reinterpret_cast<decltype(r.group_end)>(dlsym(h, "ncclGroupEnd"));
        r.error_string = reinterpret_cast<decltype(r.error_string)>(dlsym(h, "ncclGetErrorString"));
        if (!r.comm_init_all || !r.broadcast || !r.group_start || !r.group_end || !r.error_string)
            r.why = "librccl.so.1 lacks ncclCommInitAll / ncclBroadcast / ncclGroupStart / ncclGroupEnd";
        return r;
    }
};

// Communicators per ordered device set (root = first device), created once and kept for
// the life of the process.  The mutex also serialises the broadcasts of concurrent calls
// on the same communicators (RCCL communicators are not thread-safe).
struct CommCache {
    std::mutex mu;
    std::map<std::vector<int>, std::vector<ncclComm_t>> comms;
};
CommCache &comm_cache()
{
    static CommCache c;
    return c;
}

bool force_rccl()
{
    const char *e = std::getenv("TMFWM_DEBUG_FORCE_RCCL");  // exercise RCCL even with one device (tests)
    return e && *e && *e != '0';
}

// Contiguous [start, stop) of n frames for shard s of k (dist.shard_range).
void shard_range(int64_t n, int s, int k, int64_t &start, int64_t &stop)
{
    const int64_t base = n / k, rem = n % k;
    start = s * base + std::min<int64_t>(s, rem);
    stop = start + base + (s < rem ? 1 : 0);
}

struct Shard {
    int device = 0;
    int unique = 0;  // index into the unique device list
    int64_t start = 0, stop = 0;
    hipStream_t st = nullptr;
    int rc = 0;
    std::string err;
    int64_t lapack = 0;
};

struct DeviceTile {
    int device = 0;
    hipStream_t st = nullptr;
    uint8_t *tile = nullptr;
    hipEvent_t ready = nullptr;
};

// Frames per pass of a shard: two pass slots of at most ~2 GiB each (inputs + outputs), so
// that a pass's transfers overlap the neighbouring pass's kernels.
int64_t pass_frames(int64_t frame_bytes)
{
    int64_t budget = int64_t(1) << 30;
    // TMFWM_DEBUG_PASS_BYTES lowers the slot size so that the tests run several passes
    if (const char *e = std::getenv("TMFWM_DEBUG_PASS_BYTES"); e && *e) {
        const long long v = std::atoll(e);
        if (v > 0 && v < budget) budget = (int64_t)v;
    }
    const int64_t f = frame_bytes > 0 ? budget / frame_bytes : 1;
    return f < 1 ? 1 : f;
}

// Device staging buffers, kept per device across calls (an app batch loop calls the multi
// entry points over and over; hipMalloc / hipFree of GiBs per call would cost more than a
// pass).  A shard leases the buffers it needs and gives them back when it is done.  The cache
// keeps at most kKeep free buffers per device (two pass slots of two shards); a lease takes the
// smallest free buffer that fits and is at most twice the request (a small call does not hold a
// GiB slot), and when hipMalloc fails it frees the device's cached buffers and tries once more.
// tmfwm_release_cached_buffers() frees every cached buffer.
struct BufCache {
    static constexpr int kKeep = 4;
    std::mutex mu;
    std::multimap<int, std::pair<size_t, void *>> free;  // device -> (bytes, pointer)
    std::map<void *, size_t> sizes;
    static BufCache &get()
    {
        static BufCache c;
        return c;
    }
    void *lease(int dev, size_t bytes)
    {
        {
            std::lock_guard<std::mutex> lk(mu);
            auto r = free.equal_range(dev);
            auto best = free.end();
            for (auto it = r.first; it != r.second; ++it)
                if (it->second.first >= bytes && it->second.first <= 2 * bytes &&
                    (best == free.end() || it->second.first < best->second.first))
                    best = it;
            if (best != free.end()) {
                void *p = best->second.second;
                free.erase(best);
                return p;
            }
        }
        void *p = nullptr;
        if (hipMalloc(&p, bytes) != hipSuccess) {
            (void)hipGetLastError();
            release(dev);
            if (hipMalloc(&p, bytes) != hipSuccess) {
                (void)hipGetLastError();
                return nullptr;
            }
        }
        std::lock_guard<std::mutex> lk(mu);
        sizes[p] = bytes;
        return p;
    }
    // hipFree synchronises the device: it runs after the mutex is released, so returning a
    // buffer never stalls the other shards' lease / give_back behind an idle-wait
    void give_back(int dev, void *p)
    {
        if (!p) return;
        void *evict = nullptr;
        {
            std::lock_guard<std::mutex> lk(mu);
            if ((int)free.count(dev) >= kKeep) {  // the oldest cached buffer of the device goes
                auto it = free.find(dev);
                evict = it->second.second;
                sizes.erase(evict);
                free.erase(it);
            }
            free.emplace(dev, std::make_pair(sizes[p], p));
        }
        if (evict) (void)hipFree(evict);
    }
    // frees the cached (not leased) buffers of one device, or of every device (dev < 0)
    int release(int dev)
    {
        std::vector<void *> gone;
        {
            std::lock_guard<std::mutex> lk(mu);
            for (auto it = free.begin(); it != free.end();) {
                if (dev >= 0 && it->first != dev) {
                    ++it;
                    continue;
                }
                gone.push_back(it->second.second);
                sizes.erase(it->second.second);
                it = free.erase(it);
            }
        }
        for (void *p : gone) (void)hipFree(p);
        return (int)gone.size();
    }
};

int plan_shards(const int32_t *devices, int32_t n_shards, int64_t n_frames, std::vector<Shard> &sh, std::vector<DeviceTile> &uniq)
{
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
        (void)hipGetLastError();
        return report(TMFWM_ERR_NODEVICE, "no HIP device available");
    }
    const int k = n_shards > 0 ? n_shards : (devices ? 0 : ndev);
    if (k <= 0) return report(TMFWM_ERR_INVALID, "n_shards must be > 0 when devices is given");
    sh.resize(k);
    for (int s = 0; s < k; ++s) {
        const int d = devices ? devices[s] : s;
        if (d < 0 || d >= ndev) return report(TMFWM_ERR_INVALID, "shard %d: device %d out of range (%d visible)", s, d, ndev);
        sh[s].device = d;
        shard_range(n_frames, s, k, sh[s].start, sh[s].stop);
        int u = 0;
        while (u < (int)uniq.size() && uniq[u].device != d) ++u;
        if (u == (int)uniq.size()) {
            DeviceTile t;
            t.device = d;
            uniq.push_back(t);
        }
        sh[s].unique = u;
    }
    return 0;
}

// Releases the per-call streams, events and tiles, and gives the calling thread back its
// current device.
struct Cleanup {
    std::vector<Shard> *sh;
    std::vector<DeviceTile> *uniq;
    int caller_device = -1;
    Cleanup(std::vector<Shard> *s, std::vector<DeviceTile> *u) : sh(s), uniq(u)
    {
        if (hipGetDevice(&caller_device) != hipSuccess) {
            caller_device = -1;
            (void)hipGetLastError();
        }
    }
    ~Cleanup()
    {
        for (auto &s : *sh)
            if (s.st) {
                (void)hipSetDevice(s.device);
                (void)hipStreamSynchronize(s.st);
                (void)hipStreamDestroy(s.st);
            }
        for (auto &u : *uniq) {
            (void)hipSetDevice(u.device);
            if (u.st) (void)hipStreamSynchronize(u.st);
            if (u.tile) (void)hipFree(u.tile);
            if (u.ready) (void)hipEventDestroy(u.ready);
            if (u.st) (void)hipStreamDestroy(u.st);
        }
        if (caller_device >= 0) (void)hipSetDevice(caller_device);
        (void)hipGetLastError();
    }
};

#define TMF_HIPM(call)                                                                                        \
    do {                                                                                                      \
        hipError_t e_ = (call);                                                                               \
        if (e_ != hipSuccess) return report(TMFWM_ERR_HIP, "%s failed: %s", #call, hipGetErrorString(e_));     \
    } while (0)

// Tile onto every device of the shard set: H2D to the root, RCCL broadcast to the rest.
int distribute_tile(const uint8_t *wm_tile, size_t tbytes, std::vector<DeviceTile> &uniq)
{
    for (auto &u : uniq) {
        TMF_HIPM(hipSetDevice(u.device));
        TMF_HIPM(hipStreamCreateWithFlags(&u.st, hipStreamNonBlocking));
        TMF_HIPM(hipEventCreateWithFlags(&u.ready, hipEventDisableTiming));
        if (tbytes) TMF_HIPM(hipMalloc(&u.tile, tbytes));
    }
    if (tbytes) TMF_HIPM(hipSetDevice(uniq[0].device));
    if (tbytes) TMF_HIPM(hipMemcpyAsync(uniq[0].tile, wm_tile, tbytes, hipMemcpyHostToDevice, uniq[0].st));
    if (tbytes && (uniq.size() > 1 || force_rccl())) {
        Rccl &r = Rccl::get();
        if (!r.ok()) return report(TMFWM_ERR_HIP, "tile broadcast needs RCCL: %s", r.why.c_str());
        std::vector<int> devs;
        for (auto &u : uniq) devs.push_back(u.device);
        CommCache &cc = comm_cache();
        std::lock_guard<std::mutex> lk(cc.mu);
        auto it = cc.comms.find(devs);
        if (it == cc.comms.end()) {
            std::vector<ncclComm_t> c(devs.size());
            const ncclResult_t e = r.comm_init_all(c.data(), (int)devs.size(), devs.data());
            if (e != ncclSuccess) return report(TMFWM_ERR_HIP, "ncclCommInitAll over %zu devices failed: %s", devs.size(), r.error_string(e));
            it = cc.comms.emplace(devs, std::move(c)).first;
        }
        ncclResult_t e = r.group_start();
        for (size_t i = 0; i < uniq.size() && e == ncclSuccess; ++i) {
            (void)hipSetDevice(uniq[i].device);
            e = r.broadcast(uniq[0].tile, uniq[i].tile, tbytes, ncclUint8, 0, it->second[i], uniq[i].st);
        }
        const ncclResult_t e2 = r.group_end();
        if (e != ncclSuccess || e2 != ncclSuccess)
            return report(TMFWM_ERR_HIP, "ncclBroadcast of the watermark tile failed: %s", r.error_string(e != ncclSuccess ? e : e2));
    }
    for (auto &u : uniq) {
        TMF_HIPM(hipSetDevice(u.device));
        TMF_HIPM(hipEventRecord(u.ready, u.st));
    }
    return 0;
}

// One shard, on its own thread: passes of at most pass_frames() frames in two alternating
// slots.  Three streams: uploads, kernels (s.st), downloads.  Pass p's kernels wait for its
// upload and for the download of pass p - 2 (which used the same output slot); its upload
// waits for the kernels of pass p - 2 (same input slot).  The host thread enqueues pass p's
// kernels before it copies pass p - 1 down and pass p + 1 up, so with pageable host memory
// (each copy call returns once its data has been staged) the kernels of one pass run while
// the neighbouring passes move over PCIe.  The per-pass counts (dgesdd-route blocks,
// non-convergence) land in pinned host memory and are summed once the shard is done.
template <typename Up, typename Kern, typename Down>
void run_shard(Shard &s, const DeviceTile &u, int64_t in_bytes, int64_t out_bytes, int n_inputs, int H, int W, int block,
               Up up, Kern kern, Down down)
{
    auto fail_here = [&](int rc, const std::string &m) {
        if (s.rc == 0) {
            s.rc = rc;
            s.err = m;
        }
    };
    if (hipSetDevice(s.device) != hipSuccess) return fail_here(TMFWM_ERR_HIP, "hipSetDevice failed");
    const int64_t n = s.stop - s.start;
    if (n == 0) return;
    const int64_t per = std::min<int64_t>(n, pass_frames(in_bytes * n_inputs + out_bytes));
    const int64_t npass = (n + per - 1) / per;
    const size_t in_slot = (size_t)(per * in_bytes * n_inputs), out_slot = (size_t)(per * out_bytes);
    const int64_t chunks_per_pass = tmf::count_chunks(per, H, W, block);  // a shorter last pass has no more
    BufCache &bc = BufCache::get();
    uint8_t *din[2] = {nullptr, nullptr}, *dout[2] = {nullptr, nullptr};
    hipStream_t sup = nullptr, sdown = nullptr;
    hipEvent_t up_done[2] = {}, kern_done[2] = {}, down_done[2] = {};
    uint32_t *sink = nullptr;  // 3 * chunks_per_pass per pass, pinned
    const size_t sink_n = (size_t)(3 * chunks_per_pass * npass);
    auto cleanup = [&] {
        for (hipStream_t x : {sup, s.st, sdown})
            if (x) (void)hipStreamSynchronize(x);
        for (int k = 0; k < 2; ++k) {
            bc.give_back(s.device, din[k]);
            bc.give_back(s.device, dout[k]);
            for (hipEvent_t e : {up_done[k], kern_done[k], down_done[k]})
                if (e) (void)hipEventDestroy(e);
        }
        if (sup) (void)hipStreamDestroy(sup);
        if (sdown) (void)hipStreamDestroy(sdown);
        if (sink) (void)hipHostFree(sink);
        (void)hipGetLastError();
    };
    hipError_t e = hipSuccess;
    for (int k = 0; k < (npass > 1 ? 2 : 1) && e == hipSuccess; ++k) {
        din[k] = static_cast<uint8_t *>(bc.lease(s.device, in_slot));
        dout[k] = static_cast<uint8_t *>(bc.lease(s.device, out_slot));
        if (!din[k] || !dout[k]) e = hipErrorOutOfMemory;
    }
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&sup, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&sdown, hipStreamNonBlocking);
    for (int k = 0; k < 2 && e == hipSuccess; ++k)
        for (hipEvent_t *ev : {&up_done[k], &kern_done[k], &down_done[k]})
            if (e == hipSuccess) e = hipEventCreateWithFlags(ev, hipEventDisableTiming);
    if (e == hipSuccess) e = hipHostMalloc(reinterpret_cast<void **>(&sink), sink_n * 4, hipHostMallocDefault);
    if (e == hipSuccess) std::fill(sink, sink + sink_n, 0u);
    if (e == hipSuccess) e = hipStreamWaitEvent(s.st, u.ready, 0);
    if (e != hipSuccess) {
        cleanup();
        return fail_here(e == hipErrorOutOfMemory ? TMFWM_ERR_NOMEM : TMFWM_ERR_HIP, std::string("shard setup: ") + hipGetErrorString(e));
    }
    auto frames_of = [&](int64_t p) { return std::min<int64_t>(per, n - p * per); };
    auto upload = [&](int64_t p) -> int {
        const int k = (int)(p & 1);
        if (p >= 2 && hipStreamWaitEvent(sup, kern_done[k], 0) != hipSuccess) return report(TMFWM_ERR_HIP, "stream wait failed");
        if (int rc = up(s.start + p * per, frames_of(p), din[k], per * in_bytes, sup)) return rc;
        return hipEventRecord(up_done[k], sup) == hipSuccess ? 0 : report(TMFWM_ERR_HIP, "event record failed");
    };
    auto download = [&](int64_t p) -> int {
        const int k = (int)(p & 1);
        if (hipStreamWaitEvent(sdown, kern_done[k], 0) != hipSuccess) return report(TMFWM_ERR_HIP, "stream wait failed");
        if (int rc = down(s.start + p * per, frames_of(p), dout[k], sdown)) return rc;
        return hipEventRecord(down_done[k], sdown) == hipSuccess ? 0 : report(TMFWM_ERR_HIP, "event record failed");
    };
    int rc = upload(0);
    for (int64_t p = 0; p < npass && rc == 0; ++p) {
        const int k = (int)(p & 1);
        if (hipStreamWaitEvent(s.st, up_done[k], 0) != hipSuccess ||
            (p >= 2 && hipStreamWaitEvent(s.st, down_done[k], 0) != hipSuccess)) {
            rc = report(TMFWM_ERR_HIP, "stream wait failed");
            break;
        }
        rc = kern(frames_of(p), din[k], per * in_bytes, dout[k], s.st, sink + 3 * chunks_per_pass * p);
        if (rc == 0 && hipEventRecord(kern_done[k], s.st) != hipSuccess) rc = report(TMFWM_ERR_HIP, "event record failed");
        if (rc == 0 && p >= 1) rc = download(p - 1);
        if (rc == 0 && p + 1 < npass) rc = upload(p + 1);
    }
    if (rc == 0) rc = download(npass - 1);
    hipError_t se = hipSuccess;
    for (hipStream_t x : {sup, s.st, sdown})
        if (se == hipSuccess) se = hipStreamSynchronize(x);
    if (rc == 0 && se != hipSuccess) rc = report(TMFWM_ERR_HIP, "shard stream failed: %s", hipGetErrorString(se));
    for (int64_t p = 0; p < npass && rc == 0; ++p) {
        int64_t cnt = 0;
        rc = tmf::sum_sink(sink + 3 * chunks_per_pass * p, tmf::count_chunks(frames_of(p), H, W, block), &cnt);
        s.lapack += cnt;
    }
    if (rc) fail_here(rc, tmfwm_last_error());
    cleanup();
}

int join(std::vector<Shard> &sh, std::vector<std::thread> &th, int64_t *n_lapack)
{
    for (auto &t : th) t.join();
    int64_t total = 0;
    for (auto &s : sh) {
        if (s.rc) return report(s.rc, "shard on device %d (frames %lld..%lld): %s", s.device, (long long)s.start, (long long)s.stop,
                                s.err.c_str());
        total += s.lapack;
    }
    if (n_lapack) *n_lapack = total;
    return 0;
}

int make_streams(std::vector<Shard> &sh)
{
    for (auto &s : sh) {
        TMF_HIPM(hipSetDevice(s.device));
        TMF_HIPM(hipStreamCreateWithFlags(&s.st, hipStreamNonBlocking));
    }
    return 0;
}

}  // namespace

extern "C" {

int tmfwm_embed_multi_route(const uint8_t *rgb, int64_t n_frames, int32_t height, int32_t width, int64_t frame_stride,
                            const uint8_t *wm_tile, int32_t block, double alpha, uint8_t *out, const int32_t *devices,
                            int32_t n_shards, int32_t route, int64_t *n_lapack_blocks)
{
    tmf::clear_error();
    if (n_lapack_blocks) *n_lapack_blocks = 0;
    if (route < TMFWM_ROUTE_HYBRID || route > TMFWM_ROUTE_RANK1_REFERENCE) return report(TMFWM_ERR_INVALID, "route %d", route);
    if (int rc = tmf::check_frames(n_frames, height, width, frame_stride, block)) return rc;
    if (!std::isfinite(alpha)) return report(TMFWM_ERR_INVALID, "alpha is not finite");
    const int nbh = height / block, nbw = width / block;
    const size_t tbytes = (size_t)nbh * nbw;
    if (n_frames > 0 && (!rgb || !out || (tbytes && !wm_tile))) return report(TMFWM_ERR_INVALID, "NULL host pointer");
    std::vector<Shard> sh;
    std::vector<DeviceTile> uniq;
    Cleanup cleanup(&sh, &uniq);
    if (int rc = plan_shards(devices, n_shards, n_frames, sh, uniq)) return rc;
    if (n_frames == 0 || height == 0 || width == 0) return 0;
    if (int rc = make_streams(sh)) return rc;
    if (int rc = distribute_tile(wm_tile, tbytes, uniq)) return rc;
    const int64_t fbytes = (int64_t)height * width * 3;
    std::vector<std::thread> th;
    for (Shard &shard : sh) {
        Shard *sp = &shard;
        const DeviceTile *up = &uniq[shard.unique];
        th.emplace_back([=] {
            const DeviceTile &u = *up;
            run_shard(
                *sp, u, fbytes, fbytes, 1, height, width, block,
                [&](int64_t f, int64_t k, uint8_t *din, int64_t, hipStream_t st) -> int {
                    if (frame_stride == fbytes)
                        return hipMemcpyAsync(din, rgb + f * frame_stride, (size_t)(k * fbytes), hipMemcpyHostToDevice, st) == hipSuccess
                                   ? 0 : report(TMFWM_ERR_HIP, "frame upload failed");
                    for (int64_t i = 0; i < k; ++i)
                        if (hipMemcpyAsync(din + i * fbytes, rgb + (f + i) * frame_stride, (size_t)fbytes, hipMemcpyHostToDevice, st) !=
                            hipSuccess)
                            return report(TMFWM_ERR_HIP, "frame upload failed");
                    return 0;
                },
                [&](int64_t k, const uint8_t *din, int64_t, uint8_t *dout, hipStream_t st, uint32_t *sink) -> int {
                    return tmf::embed_device_async(din, k, height, width, fbytes, u.tile, block, alpha, dout, st, sink, route);
                },
                [&](int64_t f, int64_t k, const uint8_t *dout, hipStream_t st) -> int {
                    if (frame_stride == fbytes)
                        return hipMemcpyAsync(out + f * frame_stride, dout, (size_t)(k * fbytes), hipMemcpyDeviceToHost, st) == hipSuccess
                                   ? 0 : report(TMFWM_ERR_HIP, "frame download failed");
                    for (int64_t i = 0; i < k; ++i)
                        if (hipMemcpyAsync(out + (f + i) * frame_stride, dout + i * fbytes, (size_t)fbytes, hipMemcpyDeviceToHost, st) !=
                            hipSuccess)
                            return report(TMFWM_ERR_HIP, "frame download failed");
                    return 0;
                });
        });
    }
    return join(sh, th, n_lapack_blocks);
}

int tmfwm_extract_multi_route(const uint8_t *wm_rgb, const uint8_t *orig_rgb, int64_t n_frames, int32_t height, int32_t width,
                              int64_t frame_stride, int32_t block, double alpha, uint8_t *out_tiles, const int32_t *devices,
                              int32_t n_shards, int32_t route, int64_t *n_lapack_blocks)
{
    tmf::clear_error();
    if (n_lapack_blocks) *n_lapack_blocks = 0;
    if (route < TMFWM_ROUTE_HYBRID || route > TMFWM_ROUTE_RANK1_REFERENCE) return report(TMFWM_ERR_INVALID, "route %d", route);
    if (int rc = tmf::check_frames(n_frames, height, width, frame_stride, block)) return rc;
    if (!std::isfinite(alpha) || alpha == 0.0) return report(TMFWM_ERR_INVALID, "alpha must be finite and non-zero");
    const int64_t tbytes = (int64_t)(height / block) * (width / block);
    if (n_frames > 0 && (!wm_rgb || !orig_rgb || !out_tiles)) return report(TMFWM_ERR_INVALID, "NULL host pointer");
    std::vector<Shard> sh;
    std::vector<DeviceTile> uniq;
    Cleanup cleanup(&sh, &uniq);
    if (int rc = plan_shards(devices, n_shards, n_frames, sh, uniq)) return rc;
    if (n_frames == 0 || tbytes == 0) return 0;
    if (int rc = make_streams(sh)) return rc;
    if (int rc = distribute_tile(nullptr, 0, uniq)) return rc;  // no tile: events only
    const int64_t fbytes = (int64_t)height * width * 3;
    std::vector<std::thread> th;
    for (Shard &shard : sh) {
        Shard *sp = &shard;
        const DeviceTile *up = &uniq[shard.unique];
        th.emplace_back([=] {
            run_shard(
                *sp, *up, fbytes, tbytes, 2, height, width, block,
                [&](int64_t f, int64_t k, uint8_t *din, int64_t half, hipStream_t st) -> int {
                    for (int64_t i = 0; i < k; ++i)
                        if (hipMemcpyAsync(din + i * fbytes, wm_rgb + (f + i) * frame_stride, (size_t)fbytes, hipMemcpyHostToDevice, st) !=
                                hipSuccess ||
                            hipMemcpyAsync(din + half + i * fbytes, orig_rgb + (f + i) * frame_stride, (size_t)fbytes,
                                           hipMemcpyHostToDevice, st) != hipSuccess)
                            return report(TMFWM_ERR_HIP, "frame upload failed");
                    return 0;
                },
                [&](int64_t k, const uint8_t *din, int64_t half, uint8_t *dout, hipStream_t st, uint32_t *sink) -> int {
                    return tmf::extract_device_async(din, din + half, k, height, width, fbytes, block, alpha, dout, st, sink,
                                                     route);
                },
                [&](int64_t f, int64_t k, const uint8_t *dout, hipStream_t st) -> int {
                    return hipMemcpyAsync(out_tiles + f * tbytes, dout, (size_t)(k * tbytes), hipMemcpyDeviceToHost, st) == hipSuccess
                               ? 0 : report(TMFWM_ERR_HIP, "tile download failed");
                });
        });
    }
    return join(sh, th, n_lapack_blocks);
}

int tmfwm_release_cached_buffers(void) { return BufCache::get().release(-1); }

int tmfwm_embed_multi(const uint8_t *rgb, int64_t n_frames, int32_t height, int32_t width, int64_t frame_stride,
                      const uint8_t *wm_tile, int32_t block, double alpha, uint8_t *out, const int32_t *devices,
                      int32_t n_shards, int64_t *n_lapack_blocks)
{
    return tmfwm_embed_multi_route(rgb, n_frames, height, width, frame_stride, wm_tile, block, alpha, out, devices, n_shards,
                                   TMFWM_ROUTE_HYBRID, n_lapack_blocks);
}

int tmfwm_extract_multi(const uint8_t *wm_rgb, const uint8_t *orig_rgb, int64_t n_frames, int32_t height, int32_t width,
                        int64_t frame_stride, int32_t block, double alpha, uint8_t *out_tiles, const int32_t *devices,
                        int32_t n_shards, int64_t *n_lapack_blocks)
{
    return tmfwm_extract_multi_route(wm_rgb, orig_rgb, n_frames, height, width, frame_stride, block, alpha, out_tiles, devices,
                                     n_shards, TMFWM_ROUTE_HYBRID, n_lapack_blocks);
}

}  // extern "C"
