/* ORACLE -- test infrastructure only.  Shared between tmfwm_oracle.c and tmfwm_cert.cpp:
 * the pocketfft fp32 plan of one DCT length (tmfwm_oracle.c plan_init). */
#ifndef ORC_PLAN_H
#define ORC_PLAN_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
    int n;
    int nf;
    int fct[4];            /* rfftp factor list (pocketfft factorize: 4s, then a 2 moved to the front, then odd) */
    float tw[4][3 * 16];   /* rfftp twiddles per factor: tw[k][(j-1)*(ido-1) + 2i-2 / 2i-1] */
    float tws[4][2 * 16];  /* generic-radix (ip > 5) table: tws[2m], tws[2m+1] = cos, sin(2 pi m / ip) */
    float dtw[16];         /* DCT twiddle[i] = cos(2 pi (i+1) / (4n)) */
    float norm;            /* f32(1/sqrt(2n)) (scipy norm_fct, ortho) */
} dct_plan;

const dct_plan *orc_plan(int n);                                     /* n = 4, 6, ..., 16 */
void orc_colour_inv_px(float y, float cbs, float crs, uint8_t out[3]); /* N9 for one pixel */

/* tmfwm_cert.cpp: the hybrid route's byte certificate */
int orc_cert_block(const float *D, const double *U, const double *sig, const double *V, int b, uint8_t w, double alpha,
                   const float *cbs, const float *crs, int64_t *stats);

#ifdef __cplusplus
}
#endif
#endif
