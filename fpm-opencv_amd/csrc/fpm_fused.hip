// fpm_fused.hip -- the fused per-patch FPM iteration for Np = 256 (the metric
// configuration): ONE launch per runFPM iteration, one 1024-thread workgroup
// per patch, walking every LED of the order (fpmMain.cpp:348-476) without
// leaving the kernel.  Patches never interact, so there is no inter-workgroup
// communication at all.
//
// Per LED step, per workgroup (R = naRadius, box = 2R+1 rows, 16-lane groups):
//   A  gather O = spec[yc+ky][xc+kx] on the support, X = O*P      (:358-364)
//      row IDFTs of the box rows  -> T (global, L2-resident)     (:365 rows)
//   B  per column x: column IDFT (only box rows non-zero), 1/Np^2,
//      psi' = sqrt(I) psi/|psi + eps| (eps on Re), column DFT, keep the box
//      rows  -> T (in place)                                     (:365-394)
//   C  row DFTs of the box rows, pruned to the support columns; object
//      update written to the centred spectrum; pupil numerator  (:394-447,457-464)
//   D  tile maxima of |spec| under the ROI -> exact max|objF|  (:460,467)
//      P += num/max * S, max|P| for the next LED                 (:468-475,415)
//
// 256-point transforms are 16x16 four-step DFTs: a 16-lane group holds 16
// complex values per lane (element index = lane + 16*register), does the two
// 16-point DFTs in registers and exchanges once through an XOR-swizzled,
// conflict-free 2 KiB LDS tile.  Every distribution lines up: the row IDFT
// input, the row DFT output and the pupil/object registers share the
// "kx = lane + 16*k" layout, so P and the pre-update O never move.  Only
// k in {0,1,2,13,14,15} (|kx| <= 47) can be inside the support, so inputs of
// the inverse transforms and outputs of the forward ones are pruned to those
// six registers.  Box rows beyond the 64 groups ("tail rows", the outermost
// rows of the disk with a handful of pixels) are transformed by direct DFT
// sums spread over all threads.
#include <hip/hip_runtime.h>

#include <vector>

#include "fft_lds.hpp"
#include "fpm_state.hpp"

namespace fpm {

namespace fz {
constexpr int NP = 256;
constexpr int NT = 512;            // 8 waves: 2 per SIMD, 256-VGPR budget
constexpr int NG = NT / 16;         // 32 groups of 16 lanes
constexpr int NROWS = 64;           // FFT rows per patch (2 per group)
constexpr int RPG = NROWS / NG;     // rows per group
constexpr int MAXTAIL = 64;         // tail pixels (one owner thread each)
constexpr int MAXTAILROWS = 8;
constexpr int SK[6] = {0, 1, 2, 13, 14, 15};  // registers that can hold |kx| <= 47
constexpr int KYOFF = 48;                     // sigma table covers ky in [-48, 47]
}  // namespace fz

struct FusedArgs {
    DevState st;
    const uint16_t *meas_perm;  // [nS][B][x][t][m2]: I[t + 16 m2][x]
    const int *order, *x0, *y0;
    const float2 *tw;           // exp(-2 pi i k / 256), k < 256
    int n_order;
    int ky_lo, n_fft_rows;      // FFT rows ky_lo .. ky_lo + n_fft_rows - 1 (sigma 0..)
    int n_tail_rows;
    int tail_ky[fz::MAXTAILROWS];  // sigma = 64 + i
    int n_tail_px;
    int2 tail_px[fz::MAXTAIL];  // (ky, kx)
    int nbp;                    // rows of T, multiple of 4
    int ntiles;
};

// ---------------------------------------------------------------- 16-pt DFTs
// W16^j for the forward transform; the inverse uses the conjugate.
template <bool INV>
__device__ __forceinline__ float2 w16(float2 a, int j) {
    constexpr float C1 = 0.92387953251128675613f, S1 = 0.38268343236508977173f, R2 = 0.70710678118654752440f;
    float c, s;  // W16^j = c - i s (forward)
    switch (j & 15) {
        case 1: c = C1; s = S1; break;
        case 2: c = R2; s = R2; break;
        case 3: c = S1; s = C1; break;
        case 6: c = -R2; s = R2; break;
        case 9: c = -C1; s = -S1; break;
        default: c = 1.f; s = 0.f; break;
    }
    if (j == 4) return INV ? make_float2(-a.y, a.x) : make_float2(a.y, -a.x);
    const float si = INV ? -s : s;
    // (a.x + i a.y)(c - i si)
    return make_float2(a.x * c + a.y * si, a.y * c - a.x * si);
}

template <bool INV>
__device__ __forceinline__ void bf4(float2 &a0, float2 &a1, float2 &a2, float2 &a3) {
    float2 q[4] = {a0, a1, a2, a3};
    dft4<INV>(q);
    a0 = q[0];
    a1 = q[1];
    a2 = q[2];
    a3 = q[3];
}

// twiddles between the two radix-4 stages: position k1 + 4 m1 *= W16^{k1 m1}
template <bool INV>
__device__ __forceinline__ void mid_tw(float2 (&v)[16]) {
    v[5] = w16<INV>(v[5], 1);
    v[6] = w16<INV>(v[6], 2);
    v[7] = w16<INV>(v[7], 3);
    v[9] = w16<INV>(v[9], 2);
    v[10] = w16<INV>(v[10], 4);
    v[11] = w16<INV>(v[11], 6);
    v[13] = w16<INV>(v[13], 3);
    v[14] = w16<INV>(v[14], 6);
    v[15] = w16<INV>(v[15], 9);
}

// dense 16-point DFT: in v[k], out r[m] = sum_k v[k] W16^{+-km}
template <bool INV>
__device__ __forceinline__ void dft16(float2 (&v)[16], float2 (&r)[16]) {
#pragma unroll
    for (int k1 = 0; k1 < 4; ++k1) bf4<INV>(v[k1], v[k1 + 4], v[k1 + 8], v[k1 + 12]);
    mid_tw<INV>(v);
#pragma unroll
    for (int m1 = 0; m1 < 4; ++m1) bf4<INV>(v[4 * m1], v[4 * m1 + 1], v[4 * m1 + 2], v[4 * m1 + 3]);
#pragma unroll
    for (int m = 0; m < 16; ++m) r[m] = v[4 * (m & 3) + (m >> 2)];
}

// 16-point DFT whose input is zero except v[0,1,2,13,14,15]
template <bool INV>
__device__ __forceinline__ void dft16_in6(float2 (&v)[16], float2 (&r)[16]) {
    // stage 1, butterfly k1 over (v[k1], v[k1+4], v[k1+8], v[k1+12])
    const float2 a0 = v[0], b1 = v[1], b13 = v[13], c2 = v[2], c14 = v[14], d15 = v[15];
    // k1 = 0: (a0,0,0,0)
    v[0] = a0; v[4] = a0; v[8] = a0; v[12] = a0;
    // k1 = 1: (b1,0,0,b13): U[m] = b1 + b13 W4^{3m};  W4^3 = +i forward, -i inverse
    {
        const float2 ib = INV ? make_float2(b13.y, -b13.x) : make_float2(-b13.y, b13.x);  // W4^3 * b13
        v[1] = cadd(b1, b13);
        v[5] = cadd(b1, ib);
        v[9] = csub(b1, b13);
        v[13] = csub(b1, ib);
    }
    {
        const float2 ic = INV ? make_float2(c14.y, -c14.x) : make_float2(-c14.y, c14.x);
        v[2] = cadd(c2, c14);
        v[6] = cadd(c2, ic);
        v[10] = csub(c2, c14);
        v[14] = csub(c2, ic);
    }
    // k1 = 3: (0,0,0,d15): U[m] = d15 W4^{3m}
    {
        const float2 id = INV ? make_float2(d15.y, -d15.x) : make_float2(-d15.y, d15.x);
        v[3] = d15;
        v[7] = id;
        v[11] = make_float2(-d15.x, -d15.y);
        v[15] = make_float2(-id.x, -id.y);
    }
    mid_tw<INV>(v);
#pragma unroll
    for (int m1 = 0; m1 < 4; ++m1) bf4<INV>(v[4 * m1], v[4 * m1 + 1], v[4 * m1 + 2], v[4 * m1 + 3]);
#pragma unroll
    for (int m = 0; m < 16; ++m) r[m] = v[4 * (m & 3) + (m >> 2)];
}

// 16-point DFT returning only outputs m in {0,1,2,13,14,15} as o[0..5]
template <bool INV>
__device__ __forceinline__ void dft16_out6(float2 (&v)[16], float2 (&o)[6]) {
#pragma unroll
    for (int k1 = 0; k1 < 4; ++k1) bf4<INV>(v[k1], v[k1 + 4], v[k1 + 8], v[k1 + 12]);
    mid_tw<INV>(v);
    // stage 2 over k1 for fixed m1 (positions 4 m1 + k1): y0 = sum, y3 = (a0-a2) - W4(a1-a3)
    auto y0 = [](float2 a0, float2 a1, float2 a2, float2 a3) { return cadd(cadd(a0, a2), cadd(a1, a3)); };
    auto y3 = [](float2 a0, float2 a1, float2 a2, float2 a3) {
        return csub(csub(a0, a2), mul_mi<INV>(csub(a1, a3)));
    };
    o[0] = y0(v[0], v[1], v[2], v[3]);                 // m = 0  (m1 0, m2 0)
    o[1] = y0(v[4], v[5], v[6], v[7]);                 // m = 1  (m1 1, m2 0)
    o[2] = y0(v[8], v[9], v[10], v[11]);               // m = 2
    o[3] = y3(v[4], v[5], v[6], v[7]);                 // m = 13 (m1 1, m2 3)
    o[4] = y3(v[8], v[9], v[10], v[11]);               // m = 14
    o[5] = y3(v[12], v[13], v[14], v[15]);             // m = 15
}

// ------------------------------------------------------- four-step exchange
// Lane t of a 16-lane group holds y[m1] (m1 = 0..15); afterwards lane t holds
// z[j] = y_of_lane_j[t].  XOR-swizzled so both the write (16 lanes, one row)
// and the read (32 lanes, two groups) are bank-conflict free.
__device__ __forceinline__ void exchange16(float2 *scr, int t, int gb, const float2 (&y)[16], float2 (&z)[16]) {
#pragma unroll
    for (int m1 = 0; m1 < 16; ++m1) scr[m1 * 16 + (t ^ m1 ^ gb)] = y[m1];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
    for (int j = 0; j < 16; ++j) z[j] = scr[t * 16 + (j ^ t ^ gb)];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// inverse 256-point DFT (unscaled), input v[k] = X[t + 16 k] (only the six
// SK registers may be non-zero), output r[m2] = x[t + 16 m2]
__device__ __forceinline__ void idft256_in6(float2 (&v)[16], float2 (&r)[16], float2 *scr, const float2 *tw2,
                                            int t, int gb) {
    float2 y[16];
    dft16_in6<true>(v, y);
#pragma unroll
    for (int m1 = 1; m1 < 16; ++m1) y[m1] = cmul(y[m1], cconj(tw2[m1 * 16 + t]));
    exchange16(scr, t, gb, y, v);
    dft16<true>(v, r);
}

// forward 256-point DFT, input v[n2] = x[t + 16 n2], output o[s] = X[t + 16 SK[s]]
__device__ __forceinline__ void dft256_out6(float2 (&v)[16], float2 (&o)[6], float2 *scr, const float2 *tw2,
                                            int t, int gb) {
    float2 y[16];
    dft16<false>(v, y);
#pragma unroll
    for (int k1 = 1; k1 < 16; ++k1) y[k1] = cmul(y[k1], tw2[k1 * 16 + t]);
    exchange16(scr, t, gb, y, v);
    dft16_out6<false>(v, o);
}

__device__ __forceinline__ int slot_kx(int t, int s) { return t + 16 * fz::SK[s] - (s >= 3 ? fz::NP : 0); }

__device__ __forceinline__ size_t tidx(int sigma, int x) {
    return ((size_t)(sigma >> 2) * fz::NP + x) * 4 + (sigma & 3);
}

__device__ __forceinline__ float wmax16(float v) {
#pragma unroll
    for (int o = 8; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
    return v;
}

__global__ void __launch_bounds__(fz::NT, 1) k_fused_iteration(FusedArgs a) {
    using namespace fz;
    extern __shared__ __attribute__((aligned(16))) float2 sm[];
    float2 *scr_all = sm;                           // NG * 256
    float2 *tw2 = scr_all + NG * NP;                // [m1][t] = W256^{m1 t}
    float2 *tw = tw2 + 256;                         // W256^k
    float2 *tailX = tw + 256;                       // MAXTAIL
    float2 *tailF = tailX + MAXTAIL;                // MAXTAIL
    float *red = (float *)(tailF + MAXTAIL);        // 32
    int *sig = (int *)(red + 32);                   // 96: sigma of ky in [-48, 47], -1 outside the box
    int2 *tpx = (int2 *)(sig + 96);                 // MAXTAIL tail pixels (ky, kx)
    int *tky = (int *)(tpx + MAXTAIL);              // MAXTAILROWS tail rows
    float2 *numer = (float2 *)(tky + MAXTAILROWS);  // NG * RPG*6*16 pupil numerators
    float *tmx = (float *)(numer + NG * RPG * 6 * 16);  // ntiles

    const DevState &st = a.st;
    const int tid = threadIdx.x, g = tid >> 4, t = tid & 15, gb = g & 1;
    const int lane = tid & 63, w = tid >> 6;
    const int b = blockIdx.x;
    const int R = st.r, NB = st.nb, L = st.L;
    float2 *scr = scr_all + g * NP;
    float2 *gnum = numer + g * (RPG * 6 * 16);

    // ---- one-time setup (kernel-argument tables indexed with uniform indices only)
    if (tid == 0) {
#pragma unroll
        for (int i = 0; i < MAXTAIL; ++i) tpx[i] = a.tail_px[i];
#pragma unroll
        for (int i = 0; i < MAXTAILROWS; ++i) tky[i] = a.tail_ky[i];
    }
    for (int i = tid; i < 256; i += NT) {
        tw[i] = a.tw[i];
        tw2[i] = a.tw[((i >> 4) * (i & 15)) & 255];
    }
    for (int i = tid; i < 96; i += NT) {
        const int ky = i - KYOFF;
        int s = -1;
        if (ky >= -R && ky <= R) {
            if (ky >= a.ky_lo && ky < a.ky_lo + a.n_fft_rows) s = ky - a.ky_lo;
#pragma unroll
            for (int q = 0; q < MAXTAILROWS; ++q)
                if (q < a.n_tail_rows && a.tail_ky[q] == ky) s = NROWS + q;
        }
        sig[i] = s;
    }
    float *tmax_g = st.tmax + (size_t)b * a.ntiles;
    for (int i = tid; i < a.ntiles; i += NT) tmx[i] = tmax_g[i];

    float2 *spec = st.spec + (size_t)b * L * L;
    float2 *pup = st.pupil + (size_t)b * NB * NB;
    float2 *T = st.T + (size_t)b * a.nbp * NP;
    int kyr[RPG];
    bool ron[RPG];
    float2 P[RPG][6];
    unsigned inmask[RPG];
#pragma unroll
    for (int j = 0; j < RPG; ++j) {
        kyr[j] = a.ky_lo + g + NG * j;
        ron[j] = g + NG * j < a.n_fft_rows;
        inmask[j] = 0;
#pragma unroll
        for (int s = 0; s < 6; ++s) {
            const int kx = slot_kx(t, s);
            const bool in = ron[j] && (kyr[j] * kyr[j] + kx * kx <= R * R);
            inmask[j] |= (in ? 1u : 0u) << s;
            P[j][s] = in ? pup[(kyr[j] + R) * NB + kx + R] : make_float2(0.f, 0.f);
        }
    }
    __syncthreads();  // tpx / tky
    const bool towner = tid < a.n_tail_px;
    const int2 tp = towner ? tpx[tid] : make_int2(0, 0);
    float2 Pt = towner ? pup[(tp.x + R) * NB + tp.y + R] : make_float2(0.f, 0.f);
    float2 Ot = make_float2(0.f, 0.f), NPt = make_float2(0.f, 0.f);
    float pm = st.pmax[b];
    const float inv_n2 = 1.0f / (float)(NP * NP);
    __syncthreads();

    for (int it = 0; it < a.n_order; ++it) {
        const int led = a.order[it];
        const int xc = a.x0[led] + NP / 2, yc = a.y0[led] + NP / 2;
        float2 *srow = spec + (unsigned)(yc * L + xc);   // spec[yc + ky][xc + kx] = srow[ky*L + kx]

        // ---- A: gather, X = O P, row IDFTs
        float2 v[16], r[16];
        if (towner) {
            Ot = srow[tp.x * L + tp.y];
            tailX[tid] = cmul(Ot, Pt);
        }
#pragma unroll
        for (int j = 0; j < RPG; ++j) {
            if (!ron[j]) continue;
#pragma unroll
            for (int k = 0; k < 16; ++k) v[k] = make_float2(0.f, 0.f);
#pragma unroll
            for (int s = 0; s < 6; ++s)
                if ((inmask[j] >> s) & 1) v[SK[s]] = cmul(srow[kyr[j] * L + slot_kx(t, s)], P[j][s]);
            idft256_in6(v, r, scr, tw2, t, gb);
#pragma unroll
            for (int m2 = 0; m2 < 16; ++m2) T[tidx(g + NG * j, t + 16 * m2)] = r[m2];
        }
        __syncthreads();  // tailX
        for (int idx = tid; idx < a.n_tail_rows * NP; idx += NT) {
            const int q = idx / NP, x = idx - q * NP;
            const int rky = tky[q];
            float2 acc = make_float2(0.f, 0.f);
            for (int p = 0; p < a.n_tail_px; ++p) {
                if (tpx[p].x != rky) continue;
                const float2 wv = cconj(tw[(x * (tpx[p].y + NP)) & (NP - 1)]);  // e^{+2 pi i x kx / 256}
                acc = cadd(acc, cmul(tailX[p], wv));
            }
            T[tidx(NROWS + q, x)] = acc;
        }
        __syncthreads();  // T complete

        // ---- B: column passes (4 columns per wave per round)
        const uint16_t *Ib = a.meas_perm + ((size_t)led * st.B + b) * NP * NP;
#pragma unroll 1
        for (int q = 0; q < NP / (4 * (NT / 64)); ++q) {
            const int x = 4 * (w + (NT / 64) * q) + ((tid >> 4) & 3);
            // measurement: 16 consecutive uint16 = I[t + 16 m2][x]
            const uint4 *ip = (const uint4 *)(Ib + (x * 16 + t) * 16);
            const uint4 i0 = ip[0], i1 = ip[1];
#pragma unroll
            for (int k = 0; k < 16; ++k) v[k] = make_float2(0.f, 0.f);
#pragma unroll
            for (int s = 0; s < 6; ++s) {
                const int sg = sig[slot_kx(t, s) + KYOFF];
                if (sg >= 0) v[SK[s]] = T[tidx(sg, x)];
            }
            idft256_in6(v, r, scr, tw2, t, gb);
            const unsigned iw[8] = {i0.x, i0.y, i0.z, i0.w, i1.x, i1.y, i1.z, i1.w};
#pragma unroll
            for (int m2 = 0; m2 < 16; ++m2) {
                const float I = (float)((iw[m2 >> 1] >> (16 * (m2 & 1))) & 0xFFFFu);
                const float2 psi = cscale(r[m2], inv_n2);
                const float tre = psi.x + st.eps;
                const float mag2 = tre * tre + psi.y * psi.y;
                const float s = __builtin_amdgcn_sqrtf(I) * __builtin_amdgcn_rsqf(mag2);
                v[m2] = make_float2(psi.x * s, psi.y * s);
            }
            float2 o[6];
            dft256_out6(v, o, scr, tw2, t, gb);
#pragma unroll
            for (int s = 0; s < 6; ++s) {
                const int sg = sig[slot_kx(t, s) + KYOFF];
                if (sg >= 0) T[tidx(sg, x)] = o[s];
            }
        }
        __syncthreads();

        // ---- C: row DFTs (pruned), object update, pupil numerator
#pragma unroll
        for (int j = 0; j < RPG; ++j) {
            if (!ron[j]) continue;
#pragma unroll
            for (int n2 = 0; n2 < 16; ++n2) v[n2] = T[tidx(g + NG * j, t + 16 * n2)];
            float2 F[6];
            dft256_out6(v, F, scr, tw2, t, gb);
#pragma unroll
            for (int s = 0; s < 6; ++s) {
                if (!((inmask[j] >> s) & 1)) continue;
                float2 *sp = srow + kyr[j] * L + slot_kx(t, s);
                // pre-update Objfcrop (:361): spec is not written between phases A and C
                const float2 p = P[j][s], o = *sp;
                const float2 D = csub(F[s], cmul(o, p));
                const float pa = sqrtf(cabs2(p));
                const float rin = __builtin_amdgcn_rcpf((pa * pa + st.delta2) * pm);
                *sp = cadd(o, cscale(cmul(D, cscale(cconj(p), pa)), rin));
                const float oa = sqrtf(cabs2(o));
                const float rip = __builtin_amdgcn_rcpf(oa * oa + st.delta1);
                gnum[(j * 6 + s) * 16 + t] = cscale(cmul(D, cscale(cconj(o), oa)), rip);
            }
        }
        // tail pixels: 16 lanes per pixel sum the 256-term forward DFT
        for (int pp = g; pp < a.n_tail_px; pp += NG) {
            const int2 px = tpx[pp];
            const int sg = sig[px.x + KYOFF];
            float2 acc = make_float2(0.f, 0.f);
#pragma unroll 4
            for (int j = 0; j < 16; ++j) {
                const int x = t + 16 * j;
                acc = cadd(acc, cmul(T[tidx(sg, x)], tw[(x * (px.y + NP)) & (NP - 1)]));
            }
#pragma unroll
            for (int o = 8; o > 0; o >>= 1) {
                acc.x += __shfl_xor(acc.x, o, 64);
                acc.y += __shfl_xor(acc.y, o, 64);
            }
            if (t == 0) tailF[pp] = acc;
        }
        __syncthreads();  // tailF
        if (towner) {
            const float2 p = Pt, o = Ot;
            const float2 D = csub(tailF[tid], cmul(o, p));
            const float pa = sqrtf(cabs2(p));
            const float rin = __builtin_amdgcn_rcpf((pa * pa + st.delta2) * pm);
            srow[tp.x * L + tp.y] = cadd(o, cscale(cmul(D, cscale(cconj(p), pa)), rin));
            const float oa = sqrtf(cabs2(o));
            const float rip = __builtin_amdgcn_rcpf(oa * oa + st.delta1);
            NPt = cscale(cmul(D, cscale(cconj(o), oa)), rip);
        }
        __syncthreads();  // all spectrum writes

        // ---- D: tile maxima under the ROI box, global max|objF|
        {
            const int ty0 = (yc - R) >> 4, ty1 = (yc + R) >> 4, tx0 = (xc - R) >> 4, tx1 = (xc + R) >> 4;
            const int ntw = tx1 - tx0 + 1, nt = (ty1 - ty0 + 1) * ntw;
            for (int tt = w; tt < nt; tt += NT / 64) {
                const int ty = ty0 + tt / ntw, tx = tx0 + tt % ntw;
                float m = 0.f;
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const int p = lane + 64 * j;
                    m = fmaxf(m, cabs2(spec[(unsigned)((ty * 16 + (p >> 4)) * L + tx * 16 + (p & 15))]));
                }
                m = wave_max(m);
                if (lane == 0) tmx[ty * st.ntx + tx] = sqrtf(m);
            }
        }
        __syncthreads();
        float m = 0.f;
        for (int i = tid; i < a.ntiles; i += NT) m = fmaxf(m, tmx[i]);
        m = wave_max(m);
        if (lane == 0) red[w] = m;
        __syncthreads();
        float omax = red[0];
#pragma unroll
        for (int i = 1; i < NT / 64; ++i) omax = fmaxf(omax, red[i]);
        const float rom = 1.0f / omax;
        // P += num / max|objF| on the support; max|P| for the next LED
        float pmx = 0.f;
#pragma unroll
        for (int j = 0; j < RPG; ++j)
#pragma unroll
            for (int s = 0; s < 6; ++s) {
                if (!((inmask[j] >> s) & 1)) continue;
                const float2 n = gnum[(j * 6 + s) * 16 + t];
                P[j][s] = make_float2(P[j][s].x + n.x * rom, P[j][s].y + n.y * rom);
                pmx = fmaxf(pmx, cabs2(P[j][s]));
            }
        if (towner) {
            Pt = make_float2(Pt.x + NPt.x * rom, Pt.y + NPt.y * rom);
            pmx = fmaxf(pmx, cabs2(Pt));
        }
        pmx = wave_max(pmx);
        __syncthreads();  // everyone has read red[] (omax)
        if (lane == 0) red[w] = pmx;
        __syncthreads();
        float pm2 = red[0];
#pragma unroll
        for (int i = 1; i < NT / 64; ++i) pm2 = fmaxf(pm2, red[i]);
        pm = sqrtf(pm2);
        __syncthreads();  // red[] and the group tiles are reused next LED
    }

    // ---- write back the per-patch state
#pragma unroll
    for (int j = 0; j < RPG; ++j)
#pragma unroll
        for (int s = 0; s < 6; ++s)
            if ((inmask[j] >> s) & 1) pup[(kyr[j] + R) * NB + slot_kx(t, s) + R] = P[j][s];
    if (towner) pup[(tp.x + R) * NB + tp.y + R] = Pt;
    for (int i = tid; i < a.ntiles; i += NT) tmax_g[i] = tmx[i];
    if (tid == 0) st.pmax[b] = pm;
}

// measurement permutation for coalesced column reads:
// out[s][b][x][t][m2] = in[s][b][t + 16 m2][x]
__global__ void k_permute_meas(const uint16_t *__restrict__ in, uint16_t *__restrict__ out, size_t nimg) {
    const size_t img = blockIdx.y;
    if (img >= nimg) return;
    const uint16_t *src = in + img * fz::NP * fz::NP;
    uint16_t *dst = out + img * fz::NP * fz::NP;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < fz::NP * fz::NP; i += gridDim.x * blockDim.x) {
        const int y = i / fz::NP, x = i % fz::NP;  // coalesced read
        const int t = y & 15, m2 = y >> 4;
        dst[((size_t)x * 16 + t) * 16 + m2] = src[i];
    }
}

// ------------------------------------------------------------------ host side
namespace {
struct FusedGeom {
    bool ok = false;
    int ky_lo = 0, n_fft_rows = 0, n_tail_rows = 0, tail_ky[fz::MAXTAILROWS] = {0};
    int n_tail_px = 0;
    int2 tail_px[fz::MAXTAIL];
    int nbp = 0;
};

FusedGeom fused_geometry(int np, int r) {
    FusedGeom g;
    if (np != fz::NP || r < 1 || r > 47) return g;
    const int nb = 2 * r + 1;
    const int nfft = nb < fz::NROWS ? nb : fz::NROWS;
    const int extra = nb - nfft;
    g.ky_lo = -r + extra / 2;  // the 64 central rows go to the FFT groups
    g.n_fft_rows = nfft;
    for (int ky = -r; ky <= r; ++ky) {
        if (ky >= g.ky_lo && ky < g.ky_lo + nfft) continue;
        if (g.n_tail_rows >= fz::MAXTAILROWS) return g;
        g.tail_ky[g.n_tail_rows++] = ky;
        for (int kx = -r; kx <= r; ++kx)
            if (ky * ky + kx * kx <= r * r) {
                if (g.n_tail_px >= fz::MAXTAIL) return g;
                g.tail_px[g.n_tail_px++] = make_int2(ky, kx);
            }
    }
    g.nbp = ((fz::NROWS + g.n_tail_rows) + 3) / 4 * 4;
    g.ok = true;
    return g;
}

size_t fused_lds_bytes(int ntiles) {
    return (size_t)(fz::NG * fz::NP + 256 + 256 + 2 * fz::MAXTAIL) * sizeof(float2) + 32 * sizeof(float) +
           96 * sizeof(int) + fz::MAXTAIL * sizeof(int2) + fz::MAXTAILROWS * sizeof(int) +
           (size_t)fz::NG * fz::RPG * 6 * 16 * sizeof(float2) + (size_t)ntiles * sizeof(float);
}
}  // namespace

bool fused_supported(int np, int r, int L) {
    const FusedGeom g = fused_geometry(np, r);
    const int ntiles = ((L + kTile - 1) / kTile) * ((L + kTile - 1) / kTile);
    return g.ok && (L % kTile == 0) && fused_lds_bytes(ntiles) <= 160 * 1024;
}

size_t fused_T_elems(int np, int r, int B) {
    const FusedGeom g = fused_geometry(np, r);
    return (size_t)B * g.nbp * fz::NP;
}

size_t fused_meas_bytes(int np, int B, int n_stack) { return (size_t)n_stack * B * np * np * sizeof(uint16_t); }

hipError_t fused_permute(const uint16_t *meas, uint16_t *meas_perm, int n_stack, int B, hipStream_t s) {
    const size_t nimg = (size_t)n_stack * B;
    for (size_t i0 = 0; i0 < nimg; i0 += 65535) {
        const size_t n = (nimg - i0 < 65535) ? nimg - i0 : 65535;
        hipLaunchKernelGGL(k_permute_meas, dim3(64, (unsigned)n), dim3(256), 0, s,
                           meas + i0 * fz::NP * fz::NP, meas_perm + i0 * fz::NP * fz::NP, n);
    }
    return hipGetLastError();
}

hipError_t launch_fused_iteration(const DevState &st, const uint16_t *meas_perm, const int *order_dev,
                                  const int *x0_dev, const int *y0_dev, int n_order, const float2 *tw_np,
                                  hipStream_t s) {
    const FusedGeom g = fused_geometry(st.np, st.r);
    if (!g.ok) return hipErrorInvalidValue;
    FusedArgs a;
    a.st = st;
    a.meas_perm = meas_perm;
    a.order = order_dev;
    a.x0 = x0_dev;
    a.y0 = y0_dev;
    a.tw = tw_np;
    a.n_order = n_order;
    a.ky_lo = g.ky_lo;
    a.n_fft_rows = g.n_fft_rows;
    a.n_tail_rows = g.n_tail_rows;
    for (int i = 0; i < fz::MAXTAILROWS; ++i) a.tail_ky[i] = g.tail_ky[i];
    a.n_tail_px = g.n_tail_px;
    for (int i = 0; i < fz::MAXTAIL; ++i) a.tail_px[i] = i < g.n_tail_px ? g.tail_px[i] : make_int2(0, 0);
    a.nbp = g.nbp;
    a.ntiles = st.ntx * st.nty;
    const size_t lds = fused_lds_bytes(a.ntiles);
    hipError_t e = hipFuncSetAttribute((const void *)k_fused_iteration, hipFuncAttributeMaxDynamicSharedMemorySize,
                                       (int)lds);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_fused_iteration, dim3(st.B), dim3(fz::NT), lds, s, a);
    return hipGetLastError();
}

}  // namespace fpm
