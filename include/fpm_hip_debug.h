/* fpm_hip_debug.h -- test-only entry points of libfpm_hip.so (not part of the
 * drop-in boundary include/fpm_hip.h): device helpers exposed so the tests can
 * pin them on extreme inputs no valid stack reaches, and a fault injector for
 * the multi-workgroup handoffs. */
#ifndef FPM_HIP_DEBUG_H
#define FPM_HIP_DEBUG_H

#ifdef __cplusplus
extern "C" {
#endif

typedef struct fpm_ctx fpm_ctx;

/* The object update and pupil numerator of n support pixels exactly as every
 * fused kernel evaluates them (update.hpp slot_update, fpmMain.cpp:405-471):
 * with D = f - o p,
 *   nv  = o + D conj(p) |p| / ((|p|^2 + delta2 + i d2_im) pm)
 *   num = D conj(o) |o| / ((|o|^2 + delta1 + i d1_im))
 *   oa  = |o|
 * f, o, p, nv, num are interleaved complex [n][2]; pm, oa are [n].  Runs on the
 * current HIP device; returns 0 or an FPM_ERR_* code. */
int fpm_debug_slot_update(const float *f, const float *o, const float *p, const float *pm, int n, float delta1,
                          float delta2, float d1_im, float d2_im, float *nv, float *num, float *oa);

/* The general path's update coefficient f / ((a + i c) m) (fpm_state.hpp
 * upd_coef_div, general.hip / np1024.hip) for n host inputs; out[2k], out[2k+1]
 * = real, imaginary part. */
int fpm_debug_update_coef(const float *a, const float *c, const float *m, const float *f, float *out, int n);

/* Split / distributed mode fault injection: from LED position `led` of every
 * later fpm_run on, the last workgroup of each patch stops publishing its
 * handoffs, so its partners time out (~1 s) and fpm_run must report
 * FPM_ERR_DEVICE; -1 switches it off. */
int fpm_debug_set_stall(fpm_ctx *ctx, int led);

#ifdef __cplusplus
}
#endif
#endif
