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
// 1/((a + ic) m) = (a - ic) / ((a^2 + c^2) m) and the real factor |P| (|O|)
// is folded into that coefficient.  |X| is cmag (the tile maxima's function).
__device__ __forceinline__ float2 slot_update(float2 f, float2 o, float2 p, float pm, const DevState &st,
                                              float2 &num, float &oa) {
    const pf2 po = pin(o), pp = pin(p);
    const pf2 D = pin(f) - pmul(po, pp);
    const float pa = cmag(p);
    const float ap = __builtin_fmaf(pa, pa, st.delta2);
    const float rp = __builtin_amdgcn_rcpf(__builtin_fmaf(ap, ap, st.d2_im * st.d2_im) * pm) * pa;
    const pf2 nv = po + pmul(pmulc(D, pp), (pf2){ap * rp, -st.d2_im * rp});
    oa = cmag(o);
    const float ao = __builtin_fmaf(oa, oa, st.delta1);
    const float ro = __builtin_amdgcn_rcpf(__builtin_fmaf(ao, ao, st.d1_im * st.d1_im)) * oa;
    num = pout(pmul(pmulc(D, po), (pf2){ao * ro, -st.d1_im * ro}));
    return pout(nv);
}

}  // namespace fpm
