// debug.hip -- test-only entry points (include/fpm_hip_debug.h): the device
// helpers the kernels share, exposed over plain host arrays so tests can pin
// them on inputs no valid stack reaches (|O| up to 1e15, |O|^2 + delta ~ 1e30).
#include <hip/hip_runtime.h>

#include "fpm_hip.h"
#include "fpm_hip_debug.h"
#include "fpm_state.hpp"
#include "update.hpp"

namespace fpm {
namespace {
// slot_update itself, the function every fused kernel calls
__global__ void k_slot_update(const float2 *f, const float2 *o, const float2 *p, const float *pm, int n, DevState st,
                              float2 *nv, float2 *num, float *oa) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    float2 nm;
    float a;
    nv[i] = slot_update(f[i], o[i], p[i], pm[i], st, nm, a);
    num[i] = nm;
    oa[i] = a;
}
__global__ void k_update_coef(const float *a, const float *c, const float *m, const float *f, float2 *out, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float2 r = upd_coef_div(a[i], c[i], m[i]);
    out[i] = make_float2(r.x * f[i], r.y * f[i]);
}

// device scratch of one call, freed on every return path
struct Buf {
    void *p = nullptr;
    ~Buf() { (void)hipFree(p); }
};
}  // namespace
}  // namespace fpm

extern "C" int fpm_debug_slot_update(const float *f, const float *o, const float *p, const float *pm, int n,
                                     float delta1, float delta2, float d1_im, float d2_im, float *nv, float *num,
                                     float *oa) {
    if (!f || !o || !p || !pm || !nv || !num || !oa || n < 0) return FPM_ERR_INVAL;
    if (n == 0) return FPM_OK;
    const size_t c2 = (size_t)n * sizeof(float2), r1 = (size_t)n * sizeof(float);
    fpm::Buf b;
    if (hipMalloc(&b.p, 5 * c2 + 2 * r1) != hipSuccess) return FPM_ERR_NOMEM;
    char *d = (char *)b.p;
    float2 *df = (float2 *)d, *dO = (float2 *)(d + c2), *dp = (float2 *)(d + 2 * c2), *dnv = (float2 *)(d + 3 * c2),
           *dnum = (float2 *)(d + 4 * c2);
    float *dpm = (float *)(d + 5 * c2), *doa = (float *)(d + 5 * c2 + r1);
    if (hipMemcpy(df, f, c2, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(dO, o, c2, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(dp, p, c2, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(dpm, pm, r1, hipMemcpyHostToDevice) != hipSuccess)
        return FPM_ERR_DEVICE;
    fpm::DevState st{};
    st.delta1 = delta1;
    st.delta2 = delta2;
    st.d1_im = d1_im;
    st.d2_im = d2_im;
    hipLaunchKernelGGL(fpm::k_slot_update, dim3((n + 255) / 256), dim3(256), 0, nullptr, df, dO, dp, dpm, n, st, dnv,
                       dnum, doa);
    if (hipGetLastError() != hipSuccess || hipDeviceSynchronize() != hipSuccess ||
        hipMemcpy(nv, dnv, c2, hipMemcpyDeviceToHost) != hipSuccess ||
        hipMemcpy(num, dnum, c2, hipMemcpyDeviceToHost) != hipSuccess ||
        hipMemcpy(oa, doa, r1, hipMemcpyDeviceToHost) != hipSuccess)
        return FPM_ERR_DEVICE;
    return FPM_OK;
}

extern "C" int fpm_debug_update_coef(const float *a, const float *c, const float *m, const float *f, float *out,
                                     int n) {
    if (!a || !c || !m || !f || !out || n < 0) return FPM_ERR_INVAL;
    if (n == 0) return FPM_OK;
    const size_t nb = (size_t)n * sizeof(float);
    fpm::Buf b;
    if (hipMalloc(&b.p, 6 * nb) != hipSuccess) return FPM_ERR_NOMEM;
    float *d = (float *)b.p;
    if (hipMemcpy(d, a, nb, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(d + n, c, nb, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(d + 2 * (size_t)n, m, nb, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(d + 3 * (size_t)n, f, nb, hipMemcpyHostToDevice) != hipSuccess)
        return FPM_ERR_DEVICE;
    hipLaunchKernelGGL(fpm::k_update_coef, dim3((n + 255) / 256), dim3(256), 0, nullptr, d, d + n, d + 2 * (size_t)n,
                       d + 3 * (size_t)n, (float2 *)(d + 4 * (size_t)n), n);
    if (hipGetLastError() != hipSuccess || hipDeviceSynchronize() != hipSuccess ||
        hipMemcpy(out, d + 4 * (size_t)n, 2 * nb, hipMemcpyDeviceToHost) != hipSuccess)
        return FPM_ERR_DEVICE;
    return FPM_OK;
}
