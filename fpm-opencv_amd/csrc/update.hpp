// update.hpp -- the per-pixel object update and pupil numerator shared by
// the fused LED-update kernels (fpm_fused.hip, fused_mr.hip).
#pragma once
#include <hip/hip_runtime.h>

#include "cpk.hpp"
#include "fft_lds.hpp"
#include "fpm_state.hpp"

namespace fpm {

// Object update and pupil numerator of one support pixel (fpmMain.cpp:405-471),
// packed FP32: with D = Objfup - ObjfcropP (:409),
//   O' = O + D conj(P) |P| / ((|P|^2 + d2 + i d2im) max|P|)      (:406-419,433)
//   num = D conj(O) |O| / (|O|^2 + d1 + i d1im)  (/ max|objF| at the commit)
// The complex reciprocal is taken scale-safely: with a = |X|^2 + delta and
// q = c / a, 1 / ((a + ic) m) = (1 - iq) / (a (1 + q^2) m), so no intermediate
// exceeds a (the form (a - ic) / ((a^2 + c^2) m) squares a = |O|^2 + d1, i.e.
// |O|^4, which overflows fp32 once |O| reaches ~3e9).  The real factor |P|
// (|O|) is folded into the coefficient.  The object and the pupil coefficient
// are computed side by side: every transcendental is followed by the other
// chain's independent one instead of its own use (a trans-use hazard wait
// state each time in the chained order), and never more than two in a row
// (four in a row measured slower).  Every fused kernel
// calls this one function; tests/test_gpu_update_coef.py pins it through
// fpm_debug_slot_update up to |O|^2 + delta1 = 1e30.
__device__ __forceinline__ float2 slot_update(float2 f, float2 o, float2 p, float pm, const DevState &st,
                                              float2 &num, float &oa) {
    const pf2 po = pin(o), pp = pin(p);
    const float pa2 = cabs2(p), oa2 = cabs2(o);
    const float pa = __builtin_amdgcn_sqrtf(pa2);
    oa = __builtin_amdgcn_sqrtf(oa2);
    const pf2 D = pin(f) - pmul(po, pp);
    const float ap = __builtin_fmaf(pa, pa, st.delta2), ao = __builtin_fmaf(oa, oa, st.delta1);
    const float rp = __builtin_amdgcn_rcpf(ap), ro = __builtin_amdgcn_rcpf(ao);
    const pf2 dp = pmulc(D, pp), dq = pmulc(D, po);
    const float qp = st.d2_im * rp, qo = st.d1_im * ro;
    const float xp = __builtin_fmaf(qp, qp, 1.0f) * pm, xo = __builtin_fmaf(qo, qo, 1.0f) * 1.0f;
    const float sp0 = __builtin_amdgcn_rcpf(xp), so0 = __builtin_amdgcn_rcpf(xo);
    const float fp = rp * pa, fo = ro * oa;
    const float sp = sp0 * fp, so = so0 * fo;
    num = pout(pmul(dq, (pf2){so, -qo * so}));
    return pout(po + pmul(dp, (pf2){sp, -qp * sp}));
}

}  // namespace fpm
