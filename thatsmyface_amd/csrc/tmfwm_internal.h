// Internal launch interface between the C-ABI (tmfwm_capi.cpp) and the kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace tmf {

struct EmbedArgs {
    const uint8_t *src;
    uint8_t *dst;
    const uint8_t *wm;       // nbh x nbw tile, shared by all frames
    int64_t nframes;
    int64_t frame_stride;    // bytes between frames (>= H*W*3)
    int H, W, block, nbh, nbw, strips_per_row;
    int aligned;             // 4-byte aligned pixel rows: dword loads/stores
    double alpha;
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
};

struct EdgeArgs {
    const uint8_t *src;
    uint8_t *dst;
    int64_t frame_stride;
    int H, W, core_h, core_w, edge_w;
};

hipError_t launch_embed(const EmbedArgs &a, hipStream_t st);
hipError_t launch_edges(const uint8_t *src, uint8_t *dst, int64_t nframes, int H, int W, int64_t frame_stride, int block, hipStream_t st);
hipError_t launch_extract(const ExtractArgs &a, hipStream_t st);
hipError_t launch_rgb_to_ycbcr(const uint8_t *rgb, int64_t npix, float *ycc, hipStream_t st);
hipError_t launch_ycbcr_to_rgb(const float *ycc, int64_t npix, uint8_t *rgb, hipStream_t st);
hipError_t launch_dct2d_blocks(float *blocks, int64_t nb, int block, int inverse, hipStream_t st);
hipError_t launch_svd_blocks(const float *D, int64_t nb, int block, float *U, float *S, float *Vt, int32_t *sweeps, hipStream_t st);
hipError_t launch_synth(uint64_t seed, int64_t frame0, int64_t nframes, int64_t frame_bytes, uint8_t *out, hipStream_t st);

}  // namespace tmf
