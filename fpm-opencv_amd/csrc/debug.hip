// debug.hip -- test-only entry points (include/fpm_hip_debug.h): the device
// helpers the kernels share, exposed over plain host arrays so tests can pin
// them on inputs no valid stack reaches (|O| ~ 1e9 .. 1e30).
#include <hip/hip_runtime.h>

#include "fpm_hip.h"
#include "fpm_hip_debug.h"
#include "fpm_state.hpp"
#include "update.hpp"

namespace fpm {
namespace {
__global__ void k_update_coef(const float *a, const float *c, const float *m, const float *f, float2 *out, int n,
                              int form) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    float2 r;
    if (form == 0) {
        r = upd_coef_safe(a[i], c[i], m[i], f[i]);
    } else {
        r = form == 1 ? upd_coef(a[i], c[i], m[i]) : upd_coef_div(a[i], c[i], m[i]);
        r = make_float2(r.x * f[i], r.y * f[i]);
    }
    out[i] = r;
}
}  // namespace
}  // namespace fpm

extern "C" int fpm_debug_update_coef(const float *a, const float *c, const float *m, const float *f, float *out,
                                     int n, int form) {
    if (!a || !c || !m || !f || !out || n < 0 || form < 0 || form > 2) return FPM_ERR_INVAL;
    if (n == 0) return FPM_OK;
    float *d = nullptr;
    const size_t nb = (size_t)n * sizeof(float);
    if (hipMalloc(&d, 6 * nb) != hipSuccess) return FPM_ERR_NOMEM;
    int rc = FPM_OK;
    if (hipMemcpy(d, a, nb, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(d + n, c, nb, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(d + 2 * (size_t)n, m, nb, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(d + 3 * (size_t)n, f, nb, hipMemcpyHostToDevice) != hipSuccess) {
        rc = FPM_ERR_DEVICE;
    } else {
        hipLaunchKernelGGL(fpm::k_update_coef, dim3((n + 255) / 256), dim3(256), 0, nullptr, d, d + n, d + 2 * (size_t)n,
                           d + 3 * (size_t)n, (float2 *)(d + 4 * (size_t)n), n, form);
        if (hipGetLastError() != hipSuccess || hipDeviceSynchronize() != hipSuccess ||
            hipMemcpy(out, d + 4 * (size_t)n, 2 * nb, hipMemcpyDeviceToHost) != hipSuccess)
            rc = FPM_ERR_DEVICE;
    }
    (void)hipFree(d);
    return rc;
}
