// dftL.hpp -- L = 256*M point transforms (M = 2, 3, 4) held entirely in the
// registers of one 16-lane group: M four-step 256-point DFTs (dft16.hpp) of
// the stride-M sub-sequences, then a lane-local radix-M combine.  Shared by
// the objCrop transform (objcrop.hip) and the Np 1024 row/column kernels of
// the general path (np1024.hip).
#pragma once
#include <hip/hip_runtime.h>

#include <type_traits>

#include "cpk.hpp"
#include "dft16.hpp"
#include "fft_lds.hpp"

namespace fpm {

// Four-step twiddles W256^{k1 t} of lane t: either held in registers
// (float2 wt[16], load_twiddles) or read from the LDS W_L table on use
// (LdsTw: 32 fewer VGPRs, one ds_read per twiddle multiply).
struct LdsTw {
    const float2 *twL;
    int t, step;  // step = M: W256^{k t} = W_L^{M k t}
    __device__ __forceinline__ float2 operator[](int k) const { return twL[((k * t) & 255) * step]; }
};
// Fresh LDS table pointers per transform: laundered through an empty asm, so
// the compiler cannot keep twiddles loaded for one transform live (CSE) until
// the next one -- two 1024-point transforms in one kernel otherwise held
// ~100 VGPRs of reloadable twiddles and spilled 200 VGPRs.
__device__ __forceinline__ const float2 *fresh_lds(const float2 *p) { return p + opaque_int(0); }
__device__ __forceinline__ const float2 (&fresh_tw(const float2 (&w)[16]))[16] { return w; }
__device__ __forceinline__ LdsTw fresh_tw(const LdsTw &w) { return LdsTw{fresh_lds(w.twL), w.t, w.step}; }

// 256-point DFT of x[m] (m = t + 16 j held as v[j]) -> out[r] = X[t + 16 r]
// HX: half-tile exchange (scr holds XTILE_H complex, xrd = exch_rbase_half(t))
template <bool INV, bool HX = false, typename TW>
__device__ __forceinline__ void dft256_full(float2 (&v)[16], float2 (&out)[16], float2 *scr,
                                            const TW &wt, int t, int xrd) {
    constexpr bool packed = !std::is_same_v<TW, LdsTw>;
    if constexpr (!packed) {
    // scalar float2 butterflies, one cmul per twiddle: the Np 1024 kernels
    // (LDS twiddles; memory-bound) measured 4 % slower with the packed form
    // (config 5: 58.5-58.9 vs 56.1-56.6 ms of LED steps per iteration)
    float2 y[16];
    dft16<INV>(v, y);
    const auto &w = fresh_tw(wt);
#pragma unroll
    for (int k1 = 1; k1 < 16; ++k1) y[k1] = cmul(y[k1], INV ? cconj(w[k1]) : w[k1]);
    float2 z[16];
    if constexpr (HX)
        exchange16_half(scr, t, xrd, y, z);
    else
        exchange16(scr, t, xrd, y, z);
    dft16<INV>(z, out);
    } else {
    // packed FP32 (cpk.hpp), the twiddles in asm blocks of five (products,
    // then fmas): objCrop (register twiddles) 0.658 -> 0.636 ms per step
    pf2 pv[16], py[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) pv[k] = pin(v[k]);
    pdft16<INV>(pv, py);
    const auto &w = fresh_tw(wt);
#pragma unroll
    for (int m0 = 1; m0 < 16; m0 += 5) {
        pf2 w5[5];
#pragma unroll
        for (int i = 0; i < 5; ++i) w5[i] = pin(w[m0 + i]);
        ptw_block<INV, 5>(&py[m0], w5);
    }
    float2 y[16], z[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) y[k] = pout(py[k]);
    if constexpr (HX)
        exchange16_half(scr, t, xrd, y, z);
    else
        exchange16(scr, t, xrd, y, z);
#pragma unroll
    for (int k = 0; k < 16; ++k) pv[k] = pin(z[k]);
    pdft16<INV>(pv, py);
#pragma unroll
    for (int k = 0; k < 16; ++k) out[k] = pout(py[k]);
    }
}

template <int M, bool INV>
__device__ __forceinline__ void dftM(float2 *v) {
    if (M == 2) dft2<INV>(v);
    if (M == 3) dft3<INV>(v);
    if (M == 4) dft4<INV>(v);
}

// x[c][j] = element M*(t + 16 j) + c;  on return x[p][r] = X[t + 16 r + 256 p]
template <int M, bool INV, typename TW>
__device__ __forceinline__ void dftL_regs(float2 (&x)[M][16], float2 *scr, const TW &wt,
                                          const float2 *twL, int t, int xrd) {
    twL = fresh_lds(twL);
#pragma unroll
    for (int c = 0; c < M; ++c) {
        float2 o[16];
        dft256_full<INV>(x[c], o, scr, wt, t, xrd);
#pragma unroll
        for (int r = 0; r < 16; ++r) x[c][r] = o[r];
    }
    constexpr int L = 256 * M;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const int kp = t + 16 * r;
        float2 z[M];
        z[0] = x[0][r];
#pragma unroll
        for (int c = 1; c < M; ++c) {
            const float2 w = twL[(c * kp) % L];
            z[c] = cmul(x[c][r], INV ? cconj(w) : w);
        }
        dftM<M, INV>(z);
#pragma unroll
        for (int p = 0; p < M; ++p) x[p][r] = z[p];
    }
}

// per-lane four-step twiddles W256^{m t} and the W_L table, staged in LDS
__device__ __forceinline__ void load_twiddles(float2 *twL, const float2 *__restrict__ tw_L, int L, int step,
                                              float2 (&wt)[16], int t) {
    for (int i = threadIdx.x; i < L; i += blockDim.x) twL[i] = tw_L[i];
    __syncthreads();
#pragma unroll
    for (int m = 0; m < 16; ++m) wt[m] = twL[((m * t) & 255) * step];  // W256^{mt} = W_L^{M m t}
}

}  // namespace fpm
