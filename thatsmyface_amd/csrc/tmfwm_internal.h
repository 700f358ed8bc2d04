// Internal launch interface between the C-ABI (tmfwm_capi.cpp) and the kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <vector>

#include "../../include/tmfwm.h"

namespace tmf {

// One append counter per segment instead of one per launch: at b = 4 most strip-pass waves
// append, and device-scope atomics on one address serialise.
constexpr uint32_t kListShards = 2048, kShardStride = 16;  // counters 64 bytes apart

// first slot of segment s when rows block rows of nbw blocks are dealt round-robin over
// kListShards segments (segment s holds rows s, s + kListShards, ...; exact capacity)
__host__ __device__ inline uint32_t shard_base(uint32_t s, uint32_t rows, uint32_t nbw)
{
    const uint32_t q = rows / kListShards, r = rows % kListShards;
    return (uint32_t)(((uint64_t)s * q + (s < r ? s : r)) * nbw);
}

struct EmbedArgs {
    const uint8_t *src;
    uint8_t *dst;
    const uint8_t *wm;       // nbh x nbw tile, shared by all frames
    int64_t nframes;
    int64_t frame_stride;    // bytes between frames (>= H*W*3)
    int H, W, block, nbh, nbw, strips_per_row;
    int aligned;             // 4-byte aligned pixel rows: dword loads/stores
    double alpha;
    // blocks the conditioning test sends to the dgesdd route: ids (frame * nbh + bi) * nbw + bj
    // relative to this launch, appended at fb_list[atomicAdd(fb_count, 1)]
    uint32_t *fb_list;
    uint32_t *fb_count;
    uint32_t *fb_bad;        // dgesdd-route blocks whose dbdsqr did not converge (may be null)
    // list pass: blocks the first pass leaves unfinished after its f64 sweep
    // budget, same ids; null: the first pass runs every block to the end.  Segmented as
    // ExtractArgs' list (kListShards, shard_base, slow_shards)
    uint32_t *slow_list;
    uint32_t *slow_count;
    uint32_t *slow_shards;
};

struct ExtractArgs {
    const uint8_t *wsrc;
    const uint8_t *osrc;
    uint8_t *out;            // nframes x (nbh x nbw), tile_stride bytes apart
    int64_t nframes;
    int64_t frame_stride;
    int64_t tile_stride;
    int H, W, block, nbh, nbw, strips_per_row;
    int aligned;
    float alpha32;           // f32(alpha): numpy-2 weak-scalar promotion (watermarking.py:285)
    uint32_t *fb_list;       // blocks whose sigma_1 enclosure is undecided (dgesdd route)
    uint32_t *fb_count;
    uint32_t *fb_bad;        // dgesdd-route blocks whose dbdsqr did not converge (may be null)
    // list pass: blocks the strip pass's power iterations left undecided, redone
    // with more iterations before the dgesdd route; null: straight to the dgesdd route.  The
    // list is kListShards segments (shard_base); block row r = frame * nbh + bi appends to
    // segment r % kListShards through its own counter slow_shards[s * kShardStride] (zeroed by
    // the caller); the list pass adds the segments' lengths into *slow_count.
    uint32_t *slow_list;
    uint32_t *slow_count;
    uint32_t *slow_shards;
};

struct EdgeArgs {
    const uint8_t *src;
    uint8_t *dst;
    int64_t frame_stride;
    int H, W, core_h, core_w, edge_w;
};

// error reporting and argument checks of the C ABI (tmfwm_capi.cpp), shared with tmfwm_multi.cpp
int report(int code, const char *fmt, ...);  // sets this thread's tmfwm_last_error(); returns code
void clear_error();
int check_frames(int64_t n, int32_t H, int32_t W, int64_t stride, int32_t block);

// Device-memory embed / extract that never synchronise (tmfwm_multi.cpp's pipelined passes).
// Instead of reading the per-chunk counts back, they go to `sink` -- pinned host memory of
// 3 * count_chunks(...) uint32 entries: the chunks' dgesdd-route counts, then their dbdsqr
// non-convergence counts, then their list-pass counts -- by a copy enqueued on the stream; the
// caller sums them with sum_sink() once the stream is done.  Arguments as tmfwm_embed_ex /
// tmfwm_extract_ex with TMFWM_MEM_DEVICE (checked the same way).
int64_t count_chunks(int64_t nframes, int H, int W, int block);
int embed_device_async(const uint8_t *src, int64_t n, int H, int W, int64_t stride, const uint8_t *tile, int block,
                       double alpha, uint8_t *dst, hipStream_t st, uint32_t *sink, int route = TMFWM_ROUTE_HYBRID);
int extract_device_async(const uint8_t *wsrc, const uint8_t *osrc, int64_t n, int H, int W, int64_t stride, int block,
                         double alpha, uint8_t *out, hipStream_t st, uint32_t *sink, int route = TMFWM_ROUTE_HYBRID);
int sum_sink(const uint32_t *sink, int64_t nchunks, int64_t *lapack);  // TMFWM_ERR_HIP on non-convergence

hipError_t launch_embed(const EmbedArgs &a, hipStream_t st);
hipError_t launch_embed_rank1(EmbedArgs a, hipStream_t st);  // TMFWM_ROUTE_RANK1 (tmfwm_rank1.hip)
bool rank1_block(int block);  // the block sizes TMFWM_ROUTE_RANK1 has a pre-pass for
bool embed_defers(int block);  // the strip pass of embed_kernel<block> can leave blocks to a list pass
hipError_t launch_edges(const uint8_t *src, uint8_t *dst, int64_t nframes, int H, int W, int64_t frame_stride, int block, hipStream_t st);
hipError_t launch_extract(const ExtractArgs &a, hipStream_t st);
hipError_t launch_rgb_to_ycbcr(const uint8_t *rgb, int64_t npix, float *ycc, hipStream_t st);
hipError_t launch_rgb_to_ycbcr_f32(const float *rgb, int64_t npix, float *ycc, hipStream_t st);
hipError_t launch_ycbcr_to_rgb(const void *ycc, int dtype, int64_t npix, uint8_t *rgb, hipStream_t st); // dtype TMFWM_DT_F16/F32/F64
hipError_t launch_dct2d_blocks(float *blocks, int64_t nb, int block, int inverse, hipStream_t st);
// second pass on the dgesdd route (tmfwm_fallback.hip); max_entries bounds the list
hipError_t launch_embed_fixup(const EmbedArgs &a, const uint32_t *list, const uint32_t *count, int64_t max_entries, hipStream_t st);
hipError_t launch_extract_fixup(const ExtractArgs &a, const uint32_t *list, const uint32_t *count, int64_t max_entries, hipStream_t st);
// the reference route: list = 0 .. n-1, *count = n (every block of a launch on the dgesdd route)
hipError_t launch_list_all(uint32_t *list, uint32_t *count, int64_t n, hipStream_t st);
// RGBX (4 bytes per pixel, PIL's in-memory "RGB") <-> RGB (3 bytes) per frame (tmfwm_pixels.hip);
// strides in bytes between frames; unpack writes 255 into the pad byte
hipError_t launch_pack_rgbx(const uint8_t *src4, int64_t sstride, uint8_t *dst3, int64_t dstride, int64_t n, int H, int W,
                            hipStream_t st);
hipError_t launch_unpack_rgbx(const uint8_t *src3, int64_t sstride, uint8_t *dst4, int64_t dstride, int64_t n, int H, int W,
                              hipStream_t st);
hipError_t launch_lapack_svd_blocks(const float *D, int64_t nb, int block, float *U, float *S, float *Vt, int want_v, int32_t *info,
                                    hipStream_t st);
hipError_t launch_lapack_nrm2(const double *x, int64_t nvec, int n, int inc, double *out, hipStream_t st);
hipError_t launch_svd_blocks(const float *D, int64_t nb, int block, float *U, float *S, float *Vt, int32_t *sweeps, hipStream_t st);
// Watermark-tile preparation (tmfwm_tile.hip): Pillow's LANCZOS resample tables.
struct ResampleAxis {
    int ksize = 0;
    std::vector<int> bounds;  // 2 per output sample: first input index, count
    std::vector<int> kk;      // ksize 22-bit fixed-point taps per output sample
    void build(int in_size, int out_size);
};

struct ResamplePlan {
    int ih = 0, iw = 0, oh = 0, ow = 0, y_first = 0, y_last = 0;
    bool need_h = false, need_v = false;
    ResampleAxis h, v;
    void build(int in_h, int in_w, int out_h, int out_w);
    int rows() const { return y_last - y_first; }
    size_t tmp_bytes() const { return need_h ? (size_t)rows() * ow : 0; }
    std::vector<int> pack() const;  // [bounds_h | kk_h | bounds_v | kk_v]
};

hipError_t launch_resize_lanczos(const uint8_t *in, const ResamplePlan &plan, const int *tables, uint8_t *tmp, uint8_t *out,
                                 int ldo, hipStream_t st);
hipError_t launch_synth(uint64_t seed, int64_t frame0, int64_t nframes, int64_t frame_bytes, uint8_t *out, hipStream_t st);

}  // namespace tmf
