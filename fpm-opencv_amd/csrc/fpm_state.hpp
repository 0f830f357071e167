// fpm_state.hpp -- device-resident solver state shared by the kernels.
//
// HBM layout (per context, n_patch = B patches):
//   spec   float2 [B][L][L]     CENTRED high-resolution spectrum (objF after
//                               fftShift).  Storing it centred removes the three
//                               full-spectrum fftShift copies per LED the
//                               reference makes (fpmMain.cpp:358,427,447): the
//                               sub-aperture is a plain window at
//                               (crop_y0 + Np/2 + ky, crop_x0 + Np/2 + kx).
//   pupil  float2 [B][nb][nb]   pupil on its support box, ky,kx in [-r, r]
//                               (un-centred frequencies, DC at [r][r]).  P is
//                               zero outside the support forever
//                               (fpmMain.cpp:312,472), so the Np x Np pupil is
//                               never stored densely.
//   meas   u16    [nS][B][Np][Np]  LED-major measurement stack.
//   tmax   float  [B][nty][ntx] max |spec| per 16x16 tile: the exact global
//                               max|objF| of fpmMain.cpp:460,467 without an
//                               L x L pass per LED.
//   rmax   float  [B][nty]      general path: max of tmax over each tile row,
//                               so max|objF| is a max over nty values.
//   pmax   float  [B][npart]    max |P| (fpmMain.cpp:415) for the next LED, as
//                               npart partial maxima (one per pupil-commit
//                               block of the general path; npart = 1 fused).
//
// fp16 storage (FPM_FLAG_SPEC_FP16, BASELINE config 5): the spectrum is held
// as __half2 [B][L][L] scaled by a power of two, hscale = 2^-ceil(log2 Np^2)
// (|objF| <= Np^2 max sqrt(I) <= 256 Np^2, so the stored magnitude stays
// <= 256 < 65504); every kernel loads it into fp32, computes in fp32 and
// rounds once on the store.  spec is then null and spec16 non-null.
#pragma once
#include <hip/hip_fp16.h>
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace fpm {

constexpr int kTile = 16;
constexpr int kStamps = 13;  // FPM_STAMPS phase counters of the fused kernel (per recorded wave)

// one LED step of the general path (general.hip, np1024.hip)
struct StepArgs {
    int xc, yc;      // centre of the sub-aperture in the centred spectrum
    int led;         // stack index
};

struct DevState {
    float2 *spec;
    __half2 *spec16;  // fp16 storage of the spectrum (spec == nullptr then)
    float2 *pupil;
    const uint16_t *meas;
    float2 *T;        // [B][nb][Np] row-transform scratch (general path)
    // Np 1024 with fp16 spectrum storage (config 5): T held as __half2
    // [B][nb][Np] (T == nullptr then), block-scaled by powers of two: the
    // row IDFT stores each box row with its own scale (tsr, the inverse,
    // [B][nb]), the column pass each column with its own (tsc, [B][Np])
    __half2 *T16;
    float *tsr, *tsc;
    float2 *dP;       // [B][nb][nb] pupil-update numerator (general path)
    float *tmax;      // [B][nty][ntx]
    unsigned *tdirty; // [B][ceil(ntx*nty/32)] fused path: tiles whose max is an upper bound
    float *rmax;      // [B][nty] general path: row maxima of tmax
    float *pmax;      // [B][npart]
    const uint8_t *disk;  // [nb][nb] support mask
    int np, L, r, nb, B, ntx, nty;
    int mB;           // patches per LED image in meas (= B; a patch-group view keeps the
                      // context's count, since meas is LED-major over all patches)
    int npart;        // partial max|P| values per patch
    float delta1, delta2, eps;
    // imaginary parts of the scalars the reference adds with cv::add(UMat c2,
    // double) (fpmMain.cpp:390,417,469): OpenCV unrolls a double into every
    // channel, so these equal eps / delta1 / delta2 by default and are 0 under
    // FPM_FLAG_SCALAR_RE_ONLY.  Update denominators are (a + i c) * max.
    float eps_im, d1_im, d2_im;
    float hscale, hinv;  // fp16 storage scale and its inverse (powers of two)
    // live band of the centred spectrum, inclusive: spec is zeroed by fpm_init
    // and only ever changes on the support boxes of the init placement
    // (L/2 +- r) and of the used LEDs ((crop0 + Np/2) +- r), so rows outside
    // [sy0, sy1] and columns outside [sx0, sx1] stay exactly 0 (objCrop skips them)
    int sy0, sy1, sx0, sx1;
    // layout of meas: 0 = C-ABI [led][patch][y][x]; g > 0 = the fused kernels'
    // column layout [led][patch][x][t][m] = I[t + g m][x] (meas_layout)
    int meas_g;
    // launch clock probe of the fused kernels (fused_sync.hpp ClockProbe):
    // [3] = block 0's shader cycles, 100 MHz ticks, launches; null = off
    unsigned long long *clk;
};

// patches [b0, b0 + n) of a context as a DevState of n patches (the general
// path's patch groups, launched on concurrent streams): every per-patch array
// is offset, meas keeps its LED-major stride mB
inline DevState patch_view(const DevState &st, int b0, int n) {
    DevState v = st;
    const size_t L2 = (size_t)st.L * st.L, nb2 = (size_t)st.nb * st.nb;
    if (v.spec) v.spec += b0 * L2;
    if (v.spec16) v.spec16 += b0 * L2;
    if (v.pupil) v.pupil += b0 * nb2;
    if (v.meas) v.meas += (size_t)b0 * st.np * st.np;
    if (v.T) v.T += (size_t)b0 * st.nb * st.np;
    if (v.T16) v.T16 += (size_t)b0 * st.nb * st.np;
    if (v.tsr) v.tsr += (size_t)b0 * st.nb;
    if (v.tsc) v.tsc += (size_t)b0 * st.np;
    if (v.dP) v.dP += b0 * nb2;
    if (v.tmax) v.tmax += (size_t)b0 * st.nty * st.ntx;
    if (v.tdirty) v.tdirty += (size_t)b0 * ((st.ntx * st.nty + 31) / 32);
    if (v.rmax) v.rmax += (size_t)b0 * st.nty;
    if (v.pmax) v.pmax += (size_t)b0 * st.npart;
    v.B = n;
    return v;
}

// spectrum element i of patch b (i = y*L + x in the centred spectrum)
__device__ __forceinline__ float2 spec_ld(const DevState &st, int b, size_t i) {
    const size_t o = (size_t)b * st.L * st.L + i;
    if (st.spec16) {
        const float2 f = __half22float2(st.spec16[o]);
        return make_float2(f.x * st.hinv, f.y * st.hinv);
    }
    return st.spec[o];
}
__device__ __forceinline__ void spec_st(const DevState &st, int b, size_t i, float2 v) {
    const size_t o = (size_t)b * st.L * st.L + i;
    if (st.spec16)
        st.spec16[o] = __float22half2_rn(make_float2(v.x * st.hscale, v.y * st.hscale));
    else
        st.spec[o] = v;
}

// block scale of fp16 scratch: a power of two s with m s < 2^14 for the
// block's largest component magnitude m (m = 0: s = 1); returns s, *inv = 1/s
__device__ __forceinline__ float h16_scale(float m, float *inv) {
    int e = 0;
    (void)frexpf(m, &e);  // m < 2^e
    if (!(m > 0.f)) e = 0;
    // a block maximum below 2^-100 keeps the scale 2^114 (finite): an
    // unclamped 2^(14 - e) overflows to +inf for e < -113 and turns the
    // block's exact zeros into NaN (0 * inf)
    if (e < -100) e = -100;
    *inv = ldexpf(1.0f, e - 14);
    return ldexpf(1.0f, 14 - e);
}

// ePIE update coefficient 1 / ((a + i c) m) of the general path for the
// complex denominators of fpmMain.cpp:417-419 / :469-471 (c = 0 under
// FPM_FLAG_SCALAR_RE_ONLY), a = |X|^2 + delta >= delta > 0, taken
// scale-safely with IEEE divisions: with q = c / a,
// 1 / ((a + ic) m) = (1 - iq) / (a (1 + q^2) m) -- no |X|^4 term.
__device__ __forceinline__ float2 upd_coef_div(float a, float c, float m) {
    const float q = c / a;
    const float d = a * __builtin_fmaf(q, q, 1.0f) * m;
    return make_float2(1.0f / d, -q / d);
}

}  // namespace fpm
