/* fpm_hip_debug.h -- test-only entry points of libfpm_hip.so (not part of the
 * drop-in boundary include/fpm_hip.h): device helpers exposed so the tests can
 * pin them on extreme inputs no valid stack reaches. */
#ifndef FPM_HIP_DEBUG_H
#define FPM_HIP_DEBUG_H

#ifdef __cplusplus
extern "C" {
#endif

/* The ePIE update coefficient f / ((a + i c) m) of fpmMain.cpp:417-419 /
 * :469-471 as the kernels evaluate it, for n host inputs a, c, m, f;
 * out[2k], out[2k+1] = real, imaginary part.  form 0: update.hpp
 * upd_coef_safe (fused kernels), 1: fpm_state.hpp upd_coef (times f),
 * 2: fpm_state.hpp upd_coef_div (general path, times f).  Runs on the current
 * HIP device; returns 0 or an FPM_ERR_* code. */
int fpm_debug_update_coef(const float *a, const float *c, const float *m, const float *f, float *out, int n,
                          int form);

#ifdef __cplusplus
}
#endif
#endif
