/*
 * tmfwm.h -- C ABI of libtmfwm.so, the MI355X (gfx950) implementation of the
 * block-wise DCT+SVD watermark path of ThatsMyFace (modules/watermarking.py).
 *
 * Drop-in boundary: the reference's Python functions keep their signatures
 * (thatsmyface_amd/watermarking.py mirrors them); underneath, each per-pixel /
 * per-block loop of the reference becomes one call below.  Plain pointers and
 * sizes only.  The caller owns every buffer.  No exceptions cross the ABI.
 *
 * Status codes: 0 ok, negative errno-style values on error; the thread-local
 * message is available from tmfwm_last_error().  All entry points are
 * re-entrant (Streamlit runs sessions on threads): no mutable global state,
 * per-call or per-thread HIP streams.
 *
 * Memory: mem_kind = TMFWM_MEM_DEVICE -> every pointer is device memory of the
 * current HIP device (e.g. a torch tensor's data_ptr()); work is enqueued on
 * `hip_stream` (NULL = the per-thread default stream) and the call returns
 * without synchronising.  mem_kind = TMFWM_MEM_HOST -> pointers are host
 * memory; the library stages through device memory and returns after the
 * results are back in host memory.
 *
 * Image layout: n_frames frames of height x width x 3 uint8, HWC interleaved
 * (numpy / PIL "RGB" order), frame i at base + i * frame_stride bytes
 * (frame_stride >= height*width*3).  Block grid: nbh = height / block,
 * nbw = width / block.  Supported block sizes: 4, 6, 8, 10, 12, 14, 16 -- the app's
 * slider values (others return TMFWM_ERR_UNSUPPORTED).
 *
 * SVD routes: every block goes through a fused Jacobi SVD; the
 * blocks whose factors could round differently from LAPACK's (conditioning test) and,
 * since ABI 9, every block whose output bytes the byte certificate cannot prove equal to
 * LAPACK's (interval arithmetic through the reconstruct, IDCT and inverse colour) are
 * redone by a second pass on the dgesdd route -- numpy's np.linalg.svd restated
 * operation by operation (LAPACK 3.12 + OpenBLAS 0.3.29 SkylakeX kernels) -- so the
 * bytes are the reference's.  The _ex entry points report how many blocks took it.
 */
#ifndef TMFWM_H
#define TMFWM_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define TMFWM_ABI_VERSION 10

#define TMFWM_MEM_HOST 0
#define TMFWM_MEM_DEVICE 1

/* SVD routes of embed / extract (tmfwm_embed_route, tmfwm_extract_route) */
#define TMFWM_ROUTE_HYBRID 0    /* Jacobi on every block, the dgesdd route for the blocks the
                                   conditioning test flags or whose bytes the certificate cannot
                                   prove (the throughput route: tmfwm_embed) */
#define TMFWM_ROUTE_REFERENCE 1 /* the dgesdd route -- np.linalg.svd's own arithmetic -- for every
                                   block: the reference's bytes by construction */
#define TMFWM_ROUTE_RANK1 2     /* (ABI 10) embed: a rank-1 pre-pass keeps the bytes of every
                                   block whose f32(D + c u1 v1^T) it proves equal to the reference's
                                   (photo mode) and sends the rest through the hybrid
                                   route (every slider size, b = 4..16 even); extract:
                                   TMFWM_ROUTE_HYBRID */
#define TMFWM_ROUTE_RANK1_REFERENCE 3 /* (ABI 10) the same pre-pass in front of the dgesdd route: no
                                   Jacobi SVD and so no K -- embed rests on the pre-pass's rank-one
                                   bound (its constants on LAPACK's residual and top pair enter
                                   scaled by ~2^-24), extract on the certified sigma_1 enclosure
                                   (TMFWM_ROUTE_HYBRID's extract); every slider size */

#define TMFWM_OK 0
#define TMFWM_ERR_INVALID (-22)     /* bad argument (EINVAL) */
#define TMFWM_ERR_NOMEM (-12)       /* device allocation failed (ENOMEM) */
#define TMFWM_ERR_HIP (-5)          /* HIP runtime / launch error (EIO) */
#define TMFWM_ERR_UNSUPPORTED (-95) /* block size not an even 4..16 (EOPNOTSUPP) */
#define TMFWM_ERR_NODEVICE (-19)    /* no usable gfx950 device (ENODEV) */
#define TMFWM_ERR_NODATA (-61)      /* no decodable QR code in the image (ENODATA) */

/* ABI version (TMFWM_ABI_VERSION) compiled into the library. */
int tmfwm_abi_version(void);

/* Message of the last failed call on this thread ("" if none). */
const char *tmfwm_last_error(void);

/* Work report of the last tmfwm_embed_ex / tmfwm_extract_ex call on this thread that asked
 * for one (non-NULL n_lapack_blocks): the number of blocks the strip pass left to the list
 * pass -- embed: blocks needing more f64 Jacobi sweeps than the rest of their wave (DESIGN.md
 * 4); extract: blocks whose sigma_1 the strip pass's power iterations did not decide (DESIGN.md
 * 5); -1 before any such call.  Diagnostics only: the output does not depend on it. */
int64_t tmfwm_last_list_pass_blocks(void);

/* 1 when tmfwm_embed at this block size runs a list pass after its strip pass (the strip pass
 * may leave blocks that need more f64 Jacobi sweeps than the rest of their wave to it,
 * DESIGN.md 4), else 0 (also for unsupported sizes).  Describes the launches of a call; the
 * output does not depend on it.  (ABI 7) */
int tmfwm_embed_list_pass(int32_t block);

/* Number of visible HIP devices (0 when none); never fails. */
int tmfwm_device_count(void);

/*
 * Embed: replaces the body of embed_watermark() (watermarking.py:163-219):
 * RGB->YCbCr (:166), per-block 2-D DCT (:192), SVD (:195), S[0] += alpha*w/255
 * (:198), U diag(S) Vt (:201), IDCT (:204), write-back (:207-213), YCbCr->RGB
 * (:216).  wm_tile is the already-resized watermark (resize_watermark :86,
 * host side), nbh x nbw uint8, shared by all frames.  out may not alias rgb.
 */
int tmfwm_embed(const uint8_t *rgb, int64_t n_frames, int32_t height, int32_t width, int64_t frame_stride,
                const uint8_t *wm_tile, int32_t block, double alpha, uint8_t *out, int32_t mem_kind, void *hip_stream);

/*
 * tmfwm_embed with a report: *n_lapack_blocks (optional, host pointer) receives the
 * number of blocks that took the dgesdd route.  Passing it makes the call wait for
 * `hip_stream` (the count lives on the device); NULL keeps TMFWM_MEM_DEVICE calls
 * asynchronous.
 *
 * A dgesdd-route block on which dbdsqr does not converge (np.linalg.svd raises LinAlgError
 * there) fails the call with TMFWM_ERR_HIP whenever the call synchronises: every
 * TMFWM_MEM_HOST call, and every call with a non-NULL n_lapack_blocks.  An asynchronous
 * TMFWM_MEM_DEVICE call without a count pointer cannot report it (the same holds for extract).
 */
int tmfwm_embed_ex(const uint8_t *rgb, int64_t n_frames, int32_t height, int32_t width, int64_t frame_stride,
                   const uint8_t *wm_tile, int32_t block, double alpha, uint8_t *out, int32_t mem_kind, void *hip_stream,
                   int64_t *n_lapack_blocks);

/*
 * tmfwm_embed_ex with an explicit SVD route (ABI 7): TMFWM_ROUTE_HYBRID is tmfwm_embed_ex;
 * TMFWM_ROUTE_REFERENCE sends every block through the dgesdd route (LAPACK dgesdd + the
 * OpenBLAS kernels numpy calls, restated operation by operation), so each output byte is
 * computed by the reference's own arithmetic, with no certificate and no error bound to rely
 * on (the hybrid route's bytes equal it through its byte certificate, which rests on one
 * measured bound).  About two orders of magnitude less
 * throughput than the hybrid route; *n_lapack_blocks then counts every block.
 * TMFWM_ROUTE_RANK1 (ABI 10): the hybrid route behind a rank-1 pre-pass (b = 4..16; photographs,
 * whose blocks it mostly decides alone); tmfwm_last_list_pass_blocks() then counts the blocks
 * it left to the hybrid route.
 */
int tmfwm_embed_route(const uint8_t *rgb, int64_t n_frames, int32_t height, int32_t width, int64_t frame_stride,
                      const uint8_t *wm_tile, int32_t block, double alpha, uint8_t *out, int32_t mem_kind, void *hip_stream,
                      int32_t route, int64_t *n_lapack_blocks);

/*
 * Extract: replaces the body of extract_watermark() (watermarking.py:246-292):
 * luma of both images, per-block sigma_1 of the DCT of each, (s_w - s_o)/alpha
 * in float32, clip to [0,1], *255, truncation.  Both images have the same
 * height x width (the caller crops a larger original, as the reference's
 * slicing does).  out_tiles: n_frames tiles of nbh x nbw uint8, back to back.
 */
int tmfwm_extract(const uint8_t *wm_rgb, const uint8_t *orig_rgb, int64_t n_frames, int32_t height, int32_t width,
                  int64_t frame_stride, int32_t block, double alpha, uint8_t *out_tiles, int32_t mem_kind,
                  void *hip_stream);

/* tmfwm_extract with a report: *n_lapack_blocks (optional) receives the number of
 * blocks whose sigma_1 pair was computed on the dgesdd route (the rest are certified). */
int tmfwm_extract_ex(const uint8_t *wm_rgb, const uint8_t *orig_rgb, int64_t n_frames, int32_t height, int32_t width,
                     int64_t frame_stride, int32_t block, double alpha, uint8_t *out_tiles, int32_t mem_kind,
                     void *hip_stream, int64_t *n_lapack_blocks);

/* tmfwm_extract_ex with an explicit SVD route (ABI 7): TMFWM_ROUTE_REFERENCE computes both
 * sigma_1 of every block on the dgesdd route instead of certifying the Jacobi enclosure. */
int tmfwm_extract_route(const uint8_t *wm_rgb, const uint8_t *orig_rgb, int64_t n_frames, int32_t height, int32_t width,
                        int64_t frame_stride, int32_t block, double alpha, uint8_t *out_tiles, int32_t mem_kind,
                        void *hip_stream, int32_t route, int64_t *n_lapack_blocks);

/* Pixel layouts of tmfwm_embed_px / tmfwm_extract_px (ABI 8) */
#define TMFWM_PIX_RGB 3  /* 3 bytes per pixel, R G B (numpy / Image.tobytes order) */
#define TMFWM_PIX_RGBX 4 /* 4 bytes per pixel, R G B pad: how PIL holds a mode-"RGB" image in memory
                            (Image.__arrow_c_array__ / Image.fromarrow share it without a copy);
                            the pad byte is ignored on input and written as 255 */

/*
 * tmfwm_embed_route with a pixel layout per side (ABI 8): the input frames have
 * in_pixel_bytes per pixel (TMFWM_PIX_*) and in_frame_stride bytes between frames, the
 * output out_pixel_bytes and out_frame_stride.  The bytes of every pixel's R, G, B are
 * tmfwm_embed's.  4-byte frames are converted on the device, so the drop-in hands PIL's
 * own image memory to the library and wraps the output as an image without a host-side
 * pack or unpack.  3 -> 3 is tmfwm_embed_route (one frame stride for both).
 */
int tmfwm_embed_px(const uint8_t *rgb, int32_t in_pixel_bytes, int64_t in_frame_stride, int64_t n_frames, int32_t height,
                   int32_t width, const uint8_t *wm_tile, int32_t block, double alpha, uint8_t *out, int32_t out_pixel_bytes,
                   int64_t out_frame_stride, int32_t mem_kind, void *hip_stream, int32_t route, int64_t *n_lapack_blocks);

/* tmfwm_extract_route with a pixel layout and frame stride per input image (ABI 8). */
int tmfwm_extract_px(const uint8_t *wm_rgb, int32_t wm_pixel_bytes, int64_t wm_frame_stride, const uint8_t *orig_rgb,
                     int32_t orig_pixel_bytes, int64_t orig_frame_stride, int64_t n_frames, int32_t height, int32_t width,
                     int32_t block, double alpha, uint8_t *out_tiles, int32_t mem_kind, void *hip_stream, int32_t route,
                     int64_t *n_lapack_blocks);

/*
 * Multi-GPU embed / extract for callers without torch.distributed (one process drives
 * several devices).  Host memory only: rgb / out (wm_rgb / orig_rgb / out_tiles) are host
 * buffers laid out as for tmfwm_embed / tmfwm_extract, and the call returns when every
 * result is back.  The n_frames frames are split into n_shards contiguous shards (sizes
 * differ by at most one, shard s gets frames [s*n/k + min(s, n%k), ...)), shard s runs on
 * HIP device devices[s] (devices = NULL: device s; n_shards <= 0 with devices = NULL: every
 * visible device) on its own host thread and streams, in passes through two device slots of ~1 GiB of
 * frames.  The watermark tile is uploaded to devices[0] and broadcast to every other
 * device of the set with RCCL (ncclBroadcast over xGMI; librccl.so.1 is loaded on first
 * use).  Shards naming the same device share its tile (logical shards).  Replaces the
 * app's per-image loop (internal_pages/embed_watermark_page.py:492-558) for a batch; the
 * per-frame arithmetic is tmfwm_embed's.  *n_lapack_blocks (optional) sums the shards'
 * dgesdd-route blocks.  The calling thread's current HIP device is preserved.
 */
int tmfwm_embed_multi(const uint8_t *rgb, int64_t n_frames, int32_t height, int32_t width, int64_t frame_stride,
                      const uint8_t *wm_tile, int32_t block, double alpha, uint8_t *out, const int32_t *devices,
                      int32_t n_shards, int64_t *n_lapack_blocks);

int tmfwm_extract_multi(const uint8_t *wm_rgb, const uint8_t *orig_rgb, int64_t n_frames, int32_t height, int32_t width,
                        int64_t frame_stride, int32_t block, double alpha, uint8_t *out_tiles, const int32_t *devices,
                        int32_t n_shards, int64_t *n_lapack_blocks);

/* The multi-GPU calls with an explicit SVD route (ABI 8; TMFWM_ROUTE_*, as tmfwm_embed_route):
 * tmfwm_embed_multi / tmfwm_extract_multi are these with TMFWM_ROUTE_HYBRID. */
int tmfwm_embed_multi_route(const uint8_t *rgb, int64_t n_frames, int32_t height, int32_t width, int64_t frame_stride,
                            const uint8_t *wm_tile, int32_t block, double alpha, uint8_t *out, const int32_t *devices,
                            int32_t n_shards, int32_t route, int64_t *n_lapack_blocks);
int tmfwm_extract_multi_route(const uint8_t *wm_rgb, const uint8_t *orig_rgb, int64_t n_frames, int32_t height, int32_t width,
                              int64_t frame_stride, int32_t block, double alpha, uint8_t *out_tiles, const int32_t *devices,
                              int32_t n_shards, int32_t route, int64_t *n_lapack_blocks);

/* Frees the device staging buffers the multi-GPU calls keep between calls (at most four free
 * buffers per device are kept; ABI 9).  Returns the number of buffers freed. */
int tmfwm_release_cached_buffers(void);

/* rgb_to_ycbcr (watermarking.py:23): npix RGB uint8 pixels -> npix x 3 float32 (Y, Cb+0.5, Cr+0.5). */
int tmfwm_rgb_to_ycbcr(const uint8_t *rgb, int64_t npix, float *ycc, int32_t mem_kind, void *hip_stream);

/* ycbcr_to_rgb (watermarking.py:53): npix x 3 float32 -> RGB uint8 (clip, *255, truncate). */
int tmfwm_ycbcr_to_rgb(const float *ycc, int64_t npix, uint8_t *rgb, int32_t mem_kind, void *hip_stream);

/* Element types of the typed helper entry points below. */
#define TMFWM_DT_F16 1
#define TMFWM_DT_F32 2
#define TMFWM_DT_F64 3

/* rgb_to_ycbcr (watermarking.py:23-50) of a non-uint8 input: rgb holds npix x 3 float32
 * values on the 0..255 scale, i.e. the input after the reference's own cast
 * np.array(img, dtype=np.float32) (:29), which stays with the caller; the "/ 255.0" and
 * the rest run here.  For integral values it equals tmfwm_rgb_to_ycbcr. */
int tmfwm_rgb_to_ycbcr_f32(const float *rgb, int64_t npix, float *ycc, int32_t mem_kind, void *hip_stream);

/* ycbcr_to_rgb (watermarking.py:53-73) of an npix x 3 array of element type dtype
 * (TMFWM_DT_F16 = IEEE binary16 / numpy float16, _F32, _F64).  The reference computes in the
 * input's own type (:55 img.copy()): "-= 0.5", the stored dot product, clip and "* 255" are
 * rounded to that type, so a float64 input is not the float32 result of its cast.
 * TMFWM_DT_F32 is tmfwm_ycbcr_to_rgb.  Non-finite inputs have no defined uint8 (neither in
 * the reference: NaN -> uint8 is undefined in C and numpy). */
int tmfwm_ycbcr_to_rgb_typed(const void *ycc, int32_t dtype, int64_t npix, uint8_t *rgb, int32_t mem_kind,
                             void *hip_stream);

/* apply_dct_to_block / apply_idct_to_block (watermarking.py:76, :81) on n_blocks
 * contiguous row-major block x block float32 blocks, in place. */
int tmfwm_dct2d_blocks(float *blocks, int64_t n_blocks, int32_t block, int32_t inverse, int32_t mem_kind,
                       void *hip_stream);

/* np.linalg.svd(D) as the reference consumes it (watermarking.py:195): U, S
 * (descending), Vt in float32 for n_blocks blocks.  sweeps (optional, may be
 * NULL) receives the Jacobi sweeps per block: f64 sweeps | (f32 sweeps << 8)
 * (0 for an all-zero block). */
int tmfwm_svd_blocks(const float *D, int64_t n_blocks, int32_t block, float *U, float *S, float *Vt, int32_t *sweeps,
                     int32_t mem_kind, void *hip_stream);

/* np.linalg.svd(D) on the dgesdd route (the reference's own arithmetic, restated for the
 * GPU): U, S (descending), Vt in float32 for n_blocks row-major blocks.  want_vectors = 0
 * computes S only (U and Vt may be NULL).  Synchronises `hip_stream`; a block on which
 * dbdsqr does not converge returns TMFWM_ERR_INVALID. */
int tmfwm_lapack_svd_blocks(const float *D, int64_t n_blocks, int32_t block, float *U, float *S, float *Vt,
                            int32_t want_vectors, int32_t mem_kind, void *hip_stream);

/* OpenBLAS dnrm2 as LAPACK's dlarfg sees it (x87 extended arithmetic, emulated): out[v]
 * = nrm2 of n elements, stride inc, of vector v (vectors n*inc doubles apart). */
int tmfwm_lapack_nrm2(const double *x, int64_t n_vectors, int32_t n, int32_t inc, double *out, int32_t mem_kind,
                      void *hip_stream);

/* Synthetic frames generated in device memory (bench inputs):
 * out[f*frame_bytes + i] = splitmix64(seed ^ ((frame0+f) << 40) ^ i) & 0xFF. */
int tmfwm_synth_frames(uint64_t seed, int64_t frame0, int64_t n_frames, int64_t frame_bytes, uint8_t *out,
                       void *hip_stream);

/*
 * Watermark preparation: replaces resize_watermark() (watermarking.py:86-132)
 * after its PNG decode and convert("L") (:98-103), which stay with the caller.
 * wm: wm_height x wm_width 8-bit grey pixels.  tile: tile_height x tile_width.
 * preserve_ratio = 0: Pillow 12.2.0 Image.resize((tile_width, tile_height),
 * LANCZOS) (:127-130).  preserve_ratio != 0: LANCZOS to (int(w*r), int(h*r)),
 * r = min(tile_width/w, tile_height/h), pasted centred on a white (255) canvas
 * (:105-123).  Bytes equal Pillow's (fixed-point Resample.c).  Synchronises
 * `hip_stream` before returning (the resample tables are built on the host).
 * Empty sizes return TMFWM_ERR_INVALID (PIL raises ValueError there).
 */
int tmfwm_prepare_tile(const uint8_t *wm, int32_t wm_height, int32_t wm_width, int32_t tile_height, int32_t tile_width,
                       int32_t preserve_ratio, uint8_t *tile, int32_t mem_kind, void *hip_stream);

/*
 * The watermark's payload, host-side C++ (no GPU, no torch): the QR codec
 * and AES-CBC the app wraps around embed / extract.  The reference builds the watermark with
 * modules/encryption.py:8-40 (encrypt_watermark: random 16-byte IV + AES-CBC of the
 * PKCS#7-padded text) and modules/qrcode_generator.py:10-44 (text_to_qrcode: base64 text,
 * python-qrcode ERROR_CORRECT_H, version >= 1 fitted, box 10, border 4, 300 x 300), and reads
 * it back with qrcode_to_text (:47-76, pyzbar) and decrypt_watermark (encryption.py:43-68,
 * pycryptodome) at internal_pages/extract_watermark_page.py:356-364.
 *
 * tmfwm_qr_encode: data -> size x size modules (1 = dark, row-major) of the smallest version
 * >= min_version (1..10) that fits at ec_level (0 L, 1 M, 2 Q, 3 H), segmented and masked as
 * python-qrcode does (mask = -1: lowest penalty; 0..7 forces one).  *size_out = 17 + 4 v
 * (also on a too-small buffer, TMFWM_ERR_INVALID).  Data beyond version 10: TMFWM_ERR_UNSUPPORTED.
 */
int tmfwm_qr_encode(const uint8_t *data, int32_t len, int32_t ec_level, int32_t min_version, int32_t mask, uint8_t *modules,
                    int32_t capacity, int32_t *size_out);

/* tmfwm_qr_decode: an upright QR symbol (versions 1..10) in an 8-bit grey image (dark =
 * low), e.g. an extracted watermark tile, -> its payload bytes (numeric, alphanumeric and
 * byte segments, Reed-Solomon corrected).  TMFWM_ERR_NODATA when no symbol decodes;
 * *len_out = payload length (also when capacity is too small: TMFWM_ERR_INVALID). */
int tmfwm_qr_decode(const uint8_t *gray, int32_t height, int32_t width, int64_t row_stride, uint8_t *out, int32_t capacity,
                    int32_t *len_out);

/* tmfwm_qr_decode over n_tiles back-to-back height x width tiles (tmfwm_extract's output
 * layout), on host threads: payload of tile i at out + i*capacity, lens[i] = its length or
 * -1 when the tile holds no decodable symbol (or it exceeds capacity). */
int tmfwm_qr_decode_batch(const uint8_t *tiles, int64_t n_tiles, int32_t height, int32_t width, uint8_t *out, int32_t capacity,
                          int32_t *lens);

/* AES-CBC (FIPS-197, SP 800-38A) with a 16 / 24 / 32-byte key and a 16-byte IV over len bytes
 * (a multiple of 16; padding is the caller's: PKCS#7 in the app).  out may equal in. */
int tmfwm_aes_cbc_encrypt(const uint8_t *key, int32_t key_len, const uint8_t *iv, const uint8_t *in, int64_t len,
                          uint8_t *out);
int tmfwm_aes_cbc_decrypt(const uint8_t *key, int32_t key_len, const uint8_t *iv, const uint8_t *in, int64_t len,
                          uint8_t *out);

#ifdef __cplusplus
}
#endif

#endif /* TMFWM_H */
