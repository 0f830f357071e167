// np1024.hip -- the general path's row and column passes for Np = 1024
// (BASELINE config 5: Np 1024, L 4096, naRadius 333, fp16 spectrum storage),
// one 1024-point transform per wavefront held in registers (16 values per
// lane) instead of mixed-radix Stockham passes over LDS tiles.
//
// Same three steps and the same scratch as general.hip's K1-K3
// (fpmMain.cpp:358-447,457-464); K4/K5 (tile maxima, pupil commit) follow
// unchanged:
//   R1 k_rows1024_inv   a wave per support-box row: gather O*P on the disk,
//                       row IDFT, T row stored as 128-byte segments
//   C  k_cols1024       a block per 8 adjacent columns (a wave each): box rows
//                       of T staged through an LDS strip, column IDFT,
//                       amplitude replacement against the stack read
//                       column-major (meas_layout g = Np), column DFT, box rows
//                       back to T; blocks mapped so that one XCD owns a
//                       contiguous run of columns (shared L2 lines of T)
//   R2 k_rows1024_fwd   a wave per box row: T row in, row DFT, object update
//                       and pupil numerator on the disk pixels of the row
//
// Config 5 holds only 8 patches, so one LED step is ~19 k transforms: too few
// for a 16-lane group per transform to hide its serial latency (measured: a
// 16-lane-group version at 1-2 waves per SIMD ran 45-88 us per launch).  A
// wave per transform quarters the per-lane chain and needs far fewer VGPRs.
//
// Wave transform (lane = 16 c + t, group c < 4, t < 16), 1024 = 4 x 256:
//   layout D (decimated): x[j]       = element 4 (t + 16 j) + c
//   layout N (natural):   x[4 p + b] = element t + 16 (4 c + b) + 256 p
//   D -> N (w1k_DN): group c runs the four-step 256-point DFT of sub-sequence
//     c (dft256_full), a cross-group LDS exchange gives lane (c, t) the four
//     sub-results at k' = t + 16 (4 c + b), then the radix-4 combine
//     X[k' + 256 p] = sum_c' W1024^{c' k'} W4^{c' p} Y_c'[k'].
//   N -> D (w1k_ND): the same steps transposed (radix-4 over p and the
//     W1024^{c' k'} twiddles first, exchange, then the 256-point DFTs), since
//     X[4 m + c] = sum_k' W256^{k' m} W1024^{k' c} sum_p x[k' + 256 p] W4^{p c}.
#include <hip/hip_runtime.h>

#include "cpk.hpp"
#include "dftL.hpp"
#include "fpm_state.hpp"
#include "fused_sync.hpp"

#include <algorithm>
#include <cstdlib>
#include <type_traits>

namespace fpm {

namespace n1k {
constexpr int N = 1024, H = N / 2;
constexpr int WPB = 4;             // waves (rows / columns) per block
constexpr int NT = 64 * WPB;
constexpr int CXP = 17;            // cross-group exchange row pitch (complex)
// per-wave LDS: four half exchange16 tiles (dft16.hpp exchange16_half); the
// cross-group exchange runs in two rounds (b = 0,1 then 2,3) through a
// 4 x 8 x CXP tile in the same space.  Half tiles: 4.6 KB per wave instead of
// 18 KB, so R1/R2 fit six blocks per CU instead of three.
constexpr int WTILE = 4 * XTILE_H;
static_assert(4 * 8 * CXP <= WTILE, "cross-group tile");
}  // namespace n1k

// R1 holds its row's loads in registers (hoisted ahead of the pupil stores):
// 128 VGPRs = 4 waves per SIMD with a few spills (measured 38.5 -> 36.3 us per
// launch at config 5; 3 waves without the spills measured slower).  The same
// hoisting in R2 measured slower (36.4 -> 40.0 us) and is not used.

namespace {

__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ float2 w1024(const float2 *twL, int e, bool inv) {
    const float2 w = twL[e & (n1k::N - 1)];
    return inv ? cconj(w) : w;
}

// cross-group tile row of (group c'', b) in round b / 2: c'' * 2 + b % 2
__device__ __forceinline__ int xrow(int cg, int b) { return cg * 2 + (b & 1); }

// layout D -> layout N.  wt: this wave's LDS tile (n1k::WTILE complex)
template <bool INV>
__device__ __forceinline__ void w1k_DN(float2 (&x)[16], float2 *wt, const float2 *twL, int c, int t, int xrd) {
    using namespace n1k;
    float2 y[16];
    dft256_full<INV, true>(x, y, wt + c * XTILE_H, LdsTw{twL, t, 4}, t, xrd);   // y[r] = Y_c[t + 16 r]
    const float2 *tl = fresh_lds(twL);
#pragma unroll
    for (int hb = 0; hb < 2; ++hb) {   // b = 2 hb, 2 hb + 1
        wave_sync();
#pragma unroll
        for (int r = 0; r < 16; ++r)
            if (((r & 3) >> 1) == hb) wt[(c * 8 + xrow(r >> 2, r)) * CXP + t] = y[r];   // r = 4 c'' + b
        wave_sync();
#pragma unroll
        for (int b = 2 * hb; b < 2 * hb + 2; ++b) {
            const int kp = t + 16 * (4 * c + b);
            float2 z[4];
            z[0] = wt[(0 * 8 + xrow(c, b)) * CXP + t];
#pragma unroll
            for (int cc = 1; cc < 4; ++cc) z[cc] = cmul(wt[(cc * 8 + xrow(c, b)) * CXP + t], w1024(tl, cc * kp, INV));
            dft4<INV>(z);
#pragma unroll
            for (int p = 0; p < 4; ++p) x[4 * p + b] = z[p];
        }
    }
    wave_sync();  // the tile is free for the next exchange
}

// layout N -> layout D
template <bool INV>
__device__ __forceinline__ void w1k_ND(float2 (&x)[16], float2 *wt, const float2 *twL, int c, int t, int xrd) {
    using namespace n1k;
    const float2 *tl = fresh_lds(twL);
    float2 v[16];
#pragma unroll
    for (int hb = 0; hb < 2; ++hb) {
        wave_sync();
#pragma unroll
        for (int b = 2 * hb; b < 2 * hb + 2; ++b) {
            const int kp = t + 16 * (4 * c + b);
            float2 z[4];
#pragma unroll
            for (int p = 0; p < 4; ++p) z[p] = x[4 * p + b];
            dft4<INV>(z);
            wt[(0 * 8 + xrow(c, b)) * CXP + t] = z[0];
#pragma unroll
            for (int cc = 1; cc < 4; ++cc) wt[(cc * 8 + xrow(c, b)) * CXP + t] = cmul(z[cc], w1024(tl, cc * kp, INV));
        }
        wave_sync();
#pragma unroll
        for (int r = 0; r < 16; ++r)
            if (((r & 3) >> 1) == hb) v[r] = wt[(c * 8 + xrow(r >> 2, r)) * CXP + t];   // Z_c[t + 16 r]
    }
    wave_sync();
    dft256_full<INV, true>(v, x, wt + c * XTILE_H, LdsTw{twL, t, 4}, t, xrd);   // x[j] = X[4 (t + 16 j) + c]
}

__device__ __forceinline__ int fold(int k) { return k < n1k::H ? k : k - n1k::N; }  // signed frequency

// stage the N-point twiddle table; returns the table
__device__ __forceinline__ float2 *stage_twiddles(float2 *sm, const float2 *__restrict__ tw) {
    for (int i = threadIdx.x; i < n1k::N; i += blockDim.x) sm[i] = tw[i];
    __syncthreads();
    return sm;
}

// Memory access of the row / column bodies below.  PlainMem: the per-LED
// kernels (every cross-workgroup hand-off is a kernel boundary).  CohMem: the
// persistent chain kernel (k_chain1024), whose workgroups of one patch hand T,
// the spectrum, the tile maxima and the max|P| partials to each other inside
// one launch: every such load bypasses the CU's L1 (relaxed agent-scope
// atomic load = global_load sc1, served by the L2), and the stores are plain
// when every workgroup of the patch sits on one XCD (the XCD's L2 is the
// coherence point, fused_sync.hpp) or write-through (sc1) otherwise.  The
// pupil and its numerator are only ever touched by their row's owner wave and
// stay plain.
struct PlainMem {
    template <class V> __device__ __forceinline__ V ld(const V *p) const { return *p; }
    template <class V> __device__ __forceinline__ void st(V *p, V v) const { *p = v; }
};
template <bool LOCAL>
struct CohMem {
    static constexpr bool local = LOCAL;
    template <class V> __device__ __forceinline__ V ld(const V *p) const {
        using U = typename std::conditional<sizeof(V) == 8, unsigned long long, unsigned>::type;
        return __builtin_bit_cast(V, __hip_atomic_load((U *)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    }
    template <class V> __device__ __forceinline__ void st(V *p, V v) const {
        using U = typename std::conditional<sizeof(V) == 8, unsigned long long, unsigned>::type;
        if (LOCAL) *p = v;
        else __hip_atomic_store((U *)p, __builtin_bit_cast(U, v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
};

// spec_ld / spec_st (fpm_state.hpp) through a memory policy: the same arithmetic
template <class M>
__device__ __forceinline__ float2 spec_get(const M &m, const DevState &st, int b, size_t i) {
    const size_t o = (size_t)b * st.L * st.L + i;
    if (st.spec16) {
        const float2 f = __half22float2(m.ld(st.spec16 + o));
        return make_float2(f.x * st.hinv, f.y * st.hinv);
    }
    return m.ld(st.spec + o);
}
template <class M>
__device__ __forceinline__ void spec_put(const M &m, const DevState &st, int b, size_t i, float2 v) {
    const size_t o = (size_t)b * st.L * st.L + i;
    if (st.spec16) m.st(st.spec16 + o, __float22half2_rn(make_float2(v.x * st.hscale, v.y * st.hscale)));
    else m.st(st.spec + o, v);
}

// R1 body, one wave, box row `row` of patch b.  Also the previous LED's pupil
// commit (general.hip K5, folded in when `commit`): P += dP / max|objF| on
// this row's disk pixels (:468-475), with omax = max|objF| from the tile-row
// maxima K4 left (:460,467), and the row's max|P| for this LED's update (:415)
// as partial pmax[row] -- the same arithmetic as K5, so the results are
// bit-identical; K5 itself then runs once, after the last LED.
template <class M>
__device__ __forceinline__ void row_inv(const M &m, const DevState &st, const StepArgs &sa, int b, int row,
                                        float omax, bool commit, const float2 *twL, float2 *wt, int c, int t,
                                        int xrd, int lane) {
    using namespace n1k;
    const int r = st.r, nb = st.nb;
    const int ky = row - r, w2 = r * r - ky * ky;
    float2 *pup = st.pupil + ((size_t)b * nb + row) * nb + r;         // indexed by kx
    const float2 *dP = st.dP + ((size_t)b * nb + row) * nb + r;
    const size_t srow = (size_t)(sa.yc + ky) * st.L + sa.xc;         // + kx (:358-362)
    float2 x[16];
    float pmx = 0.f;
    // every load of the row first, then the arithmetic and the pupil stores:
    // a store to pup between the loads made the compiler keep them in program
    // order (pup may alias the spectrum and dP), one memory latency per j
    float2 pv[16], dv[16], ov[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) {
        const int kx = fold(4 * (t + 16 * j) + c);
        const bool in = kx * kx <= w2;
        pv[j] = in ? pup[kx] : make_float2(0.f, 0.f);
        dv[j] = (in && commit) ? dP[kx] : make_float2(0.f, 0.f);
        ov[j] = in ? spec_get(m, st, b, srow + kx) : make_float2(0.f, 0.f);
    }
#pragma unroll
    for (int j = 0; j < 16; ++j) {
        const int kx = fold(4 * (t + 16 * j) + c);
        x[j] = make_float2(0.f, 0.f);
        if (kx * kx <= w2) {
            float2 p = pv[j];
            if (commit) {
                p.x += dv[j].x / omax;
                p.y += dv[j].y / omax;
                pup[kx] = p;
            }
            pmx = fmaxf(pmx, cmag(p));
            x[j] = cmul(ov[j], p);  // :364
        }
    }
    pmx = wave_max(pmx);
    if (lane == 0) m.st(st.pmax + (size_t)b * st.npart + row, pmx);
    w1k_DN<true>(x, wt, twL, c, t, xrd);                                 // :365 (rows)
    if (st.T16) {  // fp16 scratch: one power-of-two scale per box row
        float mx = 0.f;
#pragma unroll
        for (int j = 0; j < 16; ++j) mx = fmaxf(mx, fmaxf(fabsf(x[j].x), fabsf(x[j].y)));
        float inv;
        const float sc = h16_scale(wave_max(mx), &inv);
        __half2 *T = st.T16 + ((size_t)b * nb + row) * N + t + 64 * c;
#pragma unroll
        for (int p = 0; p < 4; ++p)
#pragma unroll
            for (int bb = 0; bb < 4; ++bb)
                m.st(T + 16 * bb + 256 * p, __float22half2_rn(make_float2(x[4 * p + bb].x * sc, x[4 * p + bb].y * sc)));
        if (lane == 0) m.st(st.tsr + (size_t)b * nb + row, inv);
        return;
    }
    float2 *T = st.T + ((size_t)b * nb + row) * N + t + 64 * c;
#pragma unroll
    for (int p = 0; p < 4; ++p)
#pragma unroll
        for (int bb = 0; bb < 4; ++bb) m.st(T + 16 * bb + 256 * p, x[4 * p + bb]);
}

// C body, one block of CW waves: columns x0 .. x0 + CW - 1 of patch b, a wave
// each.  strip: nb x (CW + 1) complex of LDS, aliased by the wave tiles
template <class M, int CW>
__device__ __forceinline__ void cols_block(const M &m, const DevState &st, const StepArgs &sa, int b, int x0,
                                           const float2 *twL, float2 *strip, int tid, int w, int c, int t, int xrd) {
    using namespace n1k;
    constexpr int NTC = 64 * CW, SPCC = CW + 1;
    float2 *wt = strip + w * WTILE;    // aliases the strip while every column is in registers
    const int r = st.r, nb = st.nb;
    float2 *T = st.T ? st.T + (size_t)b * nb * N + x0 : nullptr;
    __half2 *T16 = st.T16 ? st.T16 + (size_t)b * nb * N + x0 : nullptr;
    // FFT row i of a column is box row j = i + r (i <= r) or i - N + r
    // (i >= N - r) (:364: every other row is zero)
    for (int idx = tid; idx < nb * CW; idx += NTC) {
        const int j = idx / CW, cc = idx - j * CW;
        if (T16) {
            const float2 h = __half22float2(m.ld(T16 + (size_t)j * N + cc));
            const float is = m.ld(st.tsr + (size_t)b * nb + j);
            strip[j * SPCC + cc] = make_float2(h.x * is, h.y * is);
        } else {
            strip[j * SPCC + cc] = m.ld(T + (size_t)j * N + cc);
        }
    }
    __syncthreads();
    auto boxrow = [&](int i) { return i <= r ? i + r : (i >= N - r ? i - N + r : -1); };
    float2 x[16];
#pragma unroll
    for (int p = 0; p < 4; ++p)
#pragma unroll
        for (int bb = 0; bb < 4; ++bb) {
            const int j = boxrow(t + 16 * (4 * c + bb) + 256 * p);
            x[4 * p + bb] = j >= 0 ? strip[j * SPCC + w] : make_float2(0.f, 0.f);
        }
    __syncthreads();
    w1k_ND<true>(x, wt, twL, c, t, xrd);                                 // :365 (columns)
    // amplitude replacement (:378-394) on row y = 4 (t + 16 j) + c of column
    // x0 + w: with v the unscaled IDFT value, psi = v / N^2 and
    // sqrt(I) psi / |psi + eps (1 + i)| = v / sqrt(|v + eps N^2 (1 + i)|^2 / I)
    const float nn = (float)N * (float)N, epsn = st.eps * nn, epsn_im = st.eps_im * nn;
    const uint16_t *Ic = st.meas + (((size_t)sa.led * st.mB + b) * N + x0 + w) * N + c;  // meas_layout g = Np
#pragma unroll
    for (int j = 0; j < 16; ++j) {
        const float iv = (float)Ic[4 * (t + 16 * j)];
        const float2 v = x[j];
        const float tr = v.x + epsn, ti = v.y + epsn_im;
        const float s = amp_scale(__builtin_fmaf(tr, tr, ti * ti), iv);
        x[j] = make_float2(v.x * s, v.y * s);
    }
    w1k_DN<false>(x, wt, twL, c, t, xrd);                                // :394 (columns)
    float sc = 1.f;
    if (T16) {  // fp16 scratch: one power-of-two scale per column (over all its rows)
        float mx = 0.f;
#pragma unroll
        for (int j = 0; j < 16; ++j) mx = fmaxf(mx, fmaxf(fabsf(x[j].x), fabsf(x[j].y)));
        float inv;
        sc = h16_scale(wave_max(mx), &inv);
        if ((tid & 63) == 0) m.st(st.tsc + (size_t)b * N + x0 + w, inv);
    }
    __syncthreads();  // every wave is done with its tile before the strip is rewritten
#pragma unroll
    for (int p = 0; p < 4; ++p)
#pragma unroll
        for (int bb = 0; bb < 4; ++bb) {
            const int j = boxrow(t + 16 * (4 * c + bb) + 256 * p);
            if (j >= 0) strip[j * SPCC + w] = make_float2(x[4 * p + bb].x * sc, x[4 * p + bb].y * sc);
        }
    __syncthreads();
    for (int idx = tid; idx < nb * CW; idx += NTC) {
        const int j = idx / CW, cc = idx - j * CW;
        if (T16) m.st(T16 + (size_t)j * N + cc, __float22half2_rn(strip[j * SPCC + cc]));
        else m.st(T + (size_t)j * N + cc, strip[j * SPCC + cc]);
    }
}

// R2 body, one wave, box row `row` of patch b; pm = max|P| of the last commit
template <class M>
__device__ __forceinline__ void row_fwd(const M &m, const DevState &st, const StepArgs &sa, int b, int row, float pm,
                                        const float2 *twL, float2 *wt, int c, int t, int xrd) {
    using namespace n1k;
    const int r = st.r, nb = st.nb;
    const int ky = row - r, w2 = r * r - ky * ky;
    float2 x[16];
    if (st.T16) {  // column j's element times its column scale
        const __half2 *Tr = st.T16 + ((size_t)b * nb + row) * N + c;
        const float *is = st.tsc + (size_t)b * N + c;
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            const float2 h = __half22float2(m.ld(Tr + 4 * (t + 16 * j)));
            const float s = m.ld(is + 4 * (t + 16 * j));
            x[j] = make_float2(h.x * s, h.y * s);
        }
    } else {
        const float2 *Tr = st.T + ((size_t)b * nb + row) * N + c;
#pragma unroll
        for (int j = 0; j < 16; ++j) x[j] = m.ld(Tr + 4 * (t + 16 * j));
    }
    w1k_DN<false>(x, wt, twL, c, t, xrd);                                // :394 (rows)
    float2 *pup = st.pupil + ((size_t)b * nb + row) * nb + r;
    float2 *dP = st.dP + ((size_t)b * nb + row) * nb + r;
    const size_t srow = (size_t)(sa.yc + ky) * st.L + sa.xc;
#pragma unroll
    for (int p = 0; p < 4; ++p)
#pragma unroll
        for (int bb = 0; bb < 4; ++bb) {
            const int kx = fold(t + 16 * (4 * c + bb) + 256 * p);
            if (kx * kx > w2) continue;
            const size_t si = srow + kx;
            const float2 o = spec_get(m, st, b, si);             // pre-update Objfcrop (:361)
            const float2 pp = pup[kx];
            const float2 D = csub(x[4 * p + bb], cmul(o, pp));   // Objfup - ObjfcropP (:409,463)
            const float pa = cmag(pp);                           // object update (:406-419,433)
            const float2 dpc = cmul(cmul(D, cscale(cconj(pp), pa)), upd_coef_div(pa * pa + st.delta2, st.d2_im, pm));
            spec_put(m, st, b, si, cadd(o, dpc));
            const float oa = cmag(o);                            // pupil numerator (:459-464,469)
            dP[kx] = cmul(cmul(D, cscale(cconj(o), oa)), upd_coef_div(oa * oa + st.delta1, st.d1_im, 1.0f));
        }
}

// R1: grid (ceil(nb / WPB), B), block NT
__global__ void __launch_bounds__(n1k::NT) __attribute__((amdgpu_waves_per_eu(4))) k_rows1024_inv(DevState st, StepArgs sa, const float2 *__restrict__ tw,
                                                          int commit) {
    using namespace n1k;
    extern __shared__ __attribute__((aligned(16))) float2 sm[];
    __shared__ float red[WPB];
    const int w = threadIdx.x >> 6, c = (threadIdx.x >> 4) & 3, t = threadIdx.x & 15, xrd = exch_rbase_half(t);
    const float2 *twL = stage_twiddles(sm, tw);
    const int b = blockIdx.y, row = blockIdx.x * WPB + w;
    float omax = 1.f;
    if (commit) {  // block-uniform
        float mx = 0.f;
        for (int i = threadIdx.x; i < st.nty; i += NT) mx = fmaxf(mx, st.rmax[(size_t)b * st.nty + i]);
        omax = block_max(mx, red);
    }
    if (row >= st.nb) return;  // wave-uniform; no block barrier follows
    row_inv(PlainMem{}, st, sa, b, row, omax, commit != 0, twL, sm + N + w * WTILE, c, t, xrd, threadIdx.x & 63);
}

// C: grid (N / CW, B), block 64 CW: CW adjacent columns, a wave each (CW 8:
// 64-byte row segments of T per block; 4 and 16 measured slower)
template <int CW>
__global__ void __launch_bounds__(64 * CW) __attribute__((amdgpu_waves_per_eu(4))) k_cols1024(DevState st, StepArgs sa, const float2 *__restrict__ tw) {
    using namespace n1k;
    extern __shared__ __attribute__((aligned(16))) float2 sm[];
    const int w = threadIdx.x >> 6, c = (threadIdx.x >> 4) & 3, t = threadIdx.x & 15, xrd = exch_rbase_half(t);
    const float2 *twL = stage_twiddles(sm, tw);
    // XCD-aware column groups: the dispatcher deals blocks round-robin over the
    // 8 XCDs, so XCD k gets column groups k*G/8 .. (k+1)*G/8 - 1 (contiguous)
    constexpr int G = N / CW;
    const int cg = (blockIdx.x & 7) * (G / 8) + (blockIdx.x >> 3);
    cols_block<PlainMem, CW>(PlainMem{}, st, sa, blockIdx.y, cg * CW, twL, sm + N, threadIdx.x, w, c, t, xrd);
}

// R2: grid (ceil(nb / WPB), B), block NT
__global__ void __launch_bounds__(n1k::NT) k_rows1024_fwd(DevState st, StepArgs sa, const float2 *__restrict__ tw) {
    using namespace n1k;
    extern __shared__ __attribute__((aligned(16))) float2 sm[];
    __shared__ float red[WPB];
    const int w = threadIdx.x >> 6, c = (threadIdx.x >> 4) & 3, t = threadIdx.x & 15, xrd = exch_rbase_half(t);
    const float2 *twL = stage_twiddles(sm, tw);
    const int b = blockIdx.y, row = blockIdx.x * WPB + w;
    // max|P| of the previous commit from its npart partial maxima (:415)
    float pm = 0.f;
    for (int i = threadIdx.x; i < st.npart; i += NT) pm = fmaxf(pm, st.pmax[b * st.npart + i]);
    pm = block_max(pm, red);
    if (row >= st.nb) return;
    row_fwd(PlainMem{}, st, sa, b, row, pm, twL, sm + N + w * WTILE, c, t, xrd);
}

// ---- persistent chain: a whole iteration of Np 1024 LED steps in one launch
//
// The per-LED kernels above spend most of each launch in its ramp and its
// last partial round: one LED step of config 5's 8 patches is only ~19 k
// 1024-point transforms (valu_issue 0.10-0.18, wait_any 0.5-0.75 by counters).
// k_chain1024 instead gives every patch its own set of G co-resident
// workgroups -- patch b on XCD slot b % 8, so under round-robin dispatch one
// XCD per patch and T (2.7 MB fp16) stays in that XCD's 4 MB L2 between the
// phases -- and runs the patch's whole LED chain with patch-local barriers:
//   R1 (box rows)  | C (column groups of 8)  | R2 (box rows)  | K4 (ROI tile rows)
// Each phase is the per-LED kernel's body on the same arithmetic (bit-identical
// results, tests/test_gpu_np1024.py).  A box row keeps its owner wave for the
// whole launch, so the pupil and its numerator never leave that wave's CU.
// The barrier: every wave's stores acknowledged, one flag per workgroup,
// one vector load polls all G flags (fused_sync.hpp protocol; bounded spins
// raise the sticky abort word, so a grid that could not be co-resident fails
// instead of hanging).
constexpr int kChainG = 128;   // most workgroups per patch
constexpr int kChainNT = 512;  // 8 waves: R phases 8 rows, C phase 8 columns at a time
constexpr int kChainFresh = 80;  // ROI tile columns of one tile row (2 r / 16 + 2 <= 65 for r < 512)

struct ChainArgs {
    DevState st;
    const float2 *tw;
    const int *order, *x0, *y0;
    int n_order;
    int G;      // workgroups per patch
    int b0;     // first patch of this launch (8 per launch)
    int *flags; // [8][kChainG] barrier words, [8][kChainG] XCC ids, then the sticky abort word
};

// wave 0 waits until words w[0..G) all reach `value` (lane l polls w[l] and
// w[l + 64]); false after an abort or ~1 s.  Result in every thread.
__device__ __forceinline__ bool chain_wait(int *w, int G, int value, int *abort_w, int *okw) {
    const int l = opaque_int(threadIdx.x);  // the poll addresses are not hoisted out of the caller's loop
    if (l < 64) {
        bool d0 = l >= G, d1 = l + 64 >= G;
        int ok = 1;
        for (int spins = 0;; ++spins) {
            if (!d0) d0 = __hip_atomic_load(w + l, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= value;
            if (!d1) d1 = __hip_atomic_load(w + l + 64, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= value;
            if (__all(d0 && d1)) break;
            if ((spins & 31) == 31) {
                const int ab = __hip_atomic_load(abort_w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (ab != 0 || spins > (1 << 22)) {
                    if (l == 0) __hip_atomic_store(abort_w, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    ok = 0;
                    break;
                }
            }
            __builtin_amdgcn_s_sleep(2);
        }
        if (l == 0) *okw = ok;
    }
    __syncthreads();
    return *okw != 0;
}

// the LED chain of patch b (after the XCC handshake); LOCAL: every workgroup
// of the patch on one XCD
template <bool LOCAL>
__device__ __forceinline__ void chain_run(const ChainArgs &a, int b, int slot, int part, float2 *sm, float *red,
                                          float *fresh, int *okw) {
    using namespace n1k;
    constexpr int NWB = kChainNT / 64, CW = NWB;
    const int G = a.G;
    const DevState &st = a.st;
    int *bar = a.flags + slot * kChainG;
    int *abort_w = a.flags + 16 * kChainG;
    const float2 *twL = sm;
    float2 *U = sm + N;            // wave tiles (row phases) or the column strip
    // lane indices laundered at every row / column: without it the compiler
    // hoists every lane-derived index (the 16 slot frequencies of each row
    // body, the exchange addresses) out of the loops and spills them
    struct Ids {
        int tid, w, lane, c, t, xrd;
    };
    auto ids = [&]() {
        const int tid = opaque_int(threadIdx.x);
        const int ln = tid & 63, tt = ln & 15;
        return Ids{tid, tid >> 6, ln, (ln >> 4) & 3, tt, exch_rbase_half(tt)};
    };
    const CohMem<LOCAL> m{};
    int phase = 0;
    auto barrier = [&]() {
        ++phase;
        handoff_publish(bar + part, phase, LOCAL);
        return chain_wait(bar, G, phase, abort_w, okw);
    };

    // box row k of the patch -> wave (k mod 8G), enumerated wave-major across
    // the workgroups so the rows beyond the first 8G spread over all of them
    const int NWv = NWB * G;
    const int nty = st.nty, npart = st.npart, nb = st.nb;
    for (int i = 0; i < a.n_order; ++i) {
        const int led = a.order[i];
        StepArgs sa;
        sa.led = led;
        sa.xc = a.x0[led] + N / 2;
        sa.yc = a.y0[led] + N / 2;
        const int tid = opaque_int(threadIdx.x);  // nothing lane-derived is hoisted out of the LED loop
        // R1 (with the previous LED's pupil commit)
        const bool commit = i > 0;
        float omax = 1.f;
        if (commit) {
            float mx = 0.f;
            for (int k = tid; k < nty; k += kChainNT) mx = fmaxf(mx, m.ld(st.rmax + (size_t)b * nty + k));
            omax = block_max(mx, red);
        }
        for (int row = (tid >> 6) * G + part; row < nb; row += NWv) {
            const Ids q = ids();
            row_inv(m, st, sa, b, row, omax, commit, twL, U + q.w * WTILE, q.c, q.t, q.xrd, q.lane);
        }
        if (!barrier()) return;
        // C
#ifndef XNO_C
        for (int cg = part; cg < N / CW; cg += G) {
            const Ids q = ids();
            __syncthreads();  // the previous group's strip has been written back
            cols_block<CohMem<LOCAL>, CW>(m, st, sa, b, cg * CW, twL, U, q.tid, q.w, q.c, q.t, q.xrd);
        }
#endif
        if (!barrier()) return;
        // R2
#ifndef XNO_R2
        float pm = 0.f;
        for (int k = tid; k < npart; k += kChainNT) pm = fmaxf(pm, m.ld(st.pmax + (size_t)b * npart + k));
        pm = block_max(pm, red);
        for (int row = (tid >> 6) * G + part; row < nb; row += NWv) {
            const Ids q = ids();
            row_fwd(m, st, sa, b, row, pm, twL, U + q.w * WTILE, q.c, q.t, q.xrd);
        }
#endif
        if (!barrier()) return;
        // K4 (general.hip k_tile_rows): one ROI tile row per workgroup
#ifndef XNO_K4
        const int ty0 = (sa.yc - st.r) / kTile, tx0 = (sa.xc - st.r) / kTile, tx1 = (sa.xc + st.r) / kTile;
        const int nrow = (sa.yc + st.r) / kTile - ty0 + 1;
        for (int k = part; k < nrow; k += G) {
            const Ids q = ids();
            const int w = q.w, lane = q.lane;
            const int ty = ty0 + k;
            float *tmax = st.tmax + ((size_t)b * nty + ty) * st.ntx;
            for (int tx = tx0 + w; tx <= tx1; tx += NWB) {
                float mx = 0.f;
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const int p = lane + 64 * j;
                    const int y = ty * kTile + (p >> 4), x = tx * kTile + (p & 15);
                    if (y < st.L && x < st.L) mx = fmaxf(mx, cmag(spec_get(m, st, b, (size_t)y * st.L + x)));
                }
                mx = wave_max(mx);
                if (lane == 0) {
                    m.st(tmax + tx, mx);
                    fresh[tx - tx0] = mx;
                }
            }
            __syncthreads();
            float mx = 0.f;
            for (int tx = q.tid; tx < st.ntx; tx += kChainNT)
                mx = fmaxf(mx, (tx >= tx0 && tx <= tx1) ? fresh[tx - tx0] : m.ld(tmax + tx));
            mx = block_max(mx, red);
            if (q.tid == 0) m.st(st.rmax + (size_t)b * nty + ty, mx);
        }
#endif
        if (!barrier()) return;
    }
    // the last LED's pupil commit (general.hip K5: P += dP / max|objF| on the
    // disk, the row's max|P| as partial pmax[row] = K5's part row, npart = nb)
    if (a.n_order > 0) {
        const Ids q = ids();
        const int lane = q.lane, gw = q.w * G + part;
        float mx = 0.f;
        for (int k = q.tid; k < nty; k += kChainNT) mx = fmaxf(mx, m.ld(st.rmax + (size_t)b * nty + k));
        const float omax = block_max(mx, red);
        for (int row = gw; row < nb; row += NWv) {
            float2 *pup = st.pupil + ((size_t)b * nb + row) * nb;
            const float2 *dP = st.dP + ((size_t)b * nb + row) * nb;
            const uint8_t *dk = st.disk + (size_t)row * nb;
            float pmx = 0.f;
            for (int j = lane; j < nb; j += 64) {
                if (!dk[j]) continue;
                float2 p = pup[j];
                const float2 d = dP[j];
                p.x += d.x / omax;
                p.y += d.y / omax;
                pup[j] = p;
                pmx = fmaxf(pmx, cmag(p));
            }
            pmx = wave_max(pmx);
            if (lane == 0) st.pmax[(size_t)b * npart + row] = pmx;
        }
    }
}


__global__ void __launch_bounds__(kChainNT) __attribute__((amdgpu_waves_per_eu(4))) k_chain1024(ChainArgs a) {
    using namespace n1k;
    constexpr int NWB = kChainNT / 64;
    extern __shared__ __attribute__((aligned(16))) float2 sm[];
    __shared__ float red[NWB];
    __shared__ float fresh[kChainFresh];
    __shared__ int okw, same_w;
    const int slot = blockIdx.x & 7, part = blockIdx.x >> 3, G = a.G;
    const int b = a.b0 + slot;
    if (b >= a.st.B) return;  // block-uniform: this launch has fewer than 8 patches
    int *xcc = a.flags + (8 + slot) * kChainG;
    int *abort_w = a.flags + 16 * kChainG;
    (void)stage_twiddles(sm, a.tw);
    // are all G workgroups of the patch on one XCD?  (stores plain then)
    if (threadIdx.x == 0) __hip_atomic_store(xcc + part, xcc_id() + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (!chain_wait(xcc, G, 1, abort_w, &okw)) return;
    if (threadIdx.x < 64) {
        const int mine = xcc_id() + 1, l = threadIdx.x;
        const bool s0 = l >= G || __hip_atomic_load(xcc + l, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == mine;
        const bool s1 = l + 64 >= G || __hip_atomic_load(xcc + l + 64, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == mine;
        const bool all = __all(s0 && s1);
        if (l == 0) same_w = all ? 1 : 0;
    }
    __syncthreads();
    if (same_w) chain_run<true>(a, b, slot, part, sm, red, fresh, &okw);
    else chain_run<false>(a, b, slot, part, sm, red, fresh, &okw);
}

}  // namespace

// Register path for this context?  Np 1024 with the stack in the transposed
// layout (the caller permutes it when this returns true).
bool np1024_supported(int np, int r) { return np == n1k::N && r >= 1 && r < n1k::H; }

hipError_t launch_np1024_rows_cols(const DevState &st, const StepArgs &sa, const float2 *tw, bool commit,
                                   hipStream_t s) {
    using namespace n1k;
    if (!np1024_supported(st.np, st.r) || st.meas_g != N || st.npart < st.nb) return hipErrorInvalidValue;
    const size_t lds_r = (size_t)(N + WPB * WTILE) * sizeof(float2);
    // column-pass width: 8 columns per block (64-byte row segments of T;
    // config 5: 56.5-57.4 vs 58.3-59.1 ms of LED steps with 4, 16 slower again)
    constexpr int cw = 8;
    const size_t strip = std::max((size_t)st.nb * (cw + 1), (size_t)cw * WTILE);
    const size_t lds_c = (N + strip) * sizeof(float2);
    const void *fc = (const void *)k_cols1024<cw>;
    hipError_t e = hipFuncSetAttribute(fc, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_c);
    if (e != hipSuccess) return e;
    const dim3 rgrid((st.nb + WPB - 1) / WPB, st.B);
    hipLaunchKernelGGL(k_rows1024_inv, rgrid, dim3(NT), lds_r, s, st, sa, tw, commit ? 1 : 0);
    hipLaunchKernelGGL(k_cols1024<cw>, dim3(N / cw, st.B), dim3(64 * cw), lds_c, s, st, sa, tw);
    hipLaunchKernelGGL(k_rows1024_fwd, rgrid, dim3(NT), lds_r, s, st, sa, tw);
    return hipGetLastError();
}

// ---- persistent chain (k_chain1024) -----------------------------------------
int np1024_chain_flag_words() { return 16 * kChainG + 1; }

static size_t chain_lds_bytes(int nb) {
    using namespace n1k;
    constexpr int CW = kChainNT / 64;
    return (size_t)(N + std::max(CW * WTILE, nb * (CW + 1))) * sizeof(float2);
}

// workgroups per patch: every patch of a launch (8) with its G workgroups
// resident at once; 0 when the chain does not apply
int np1024_chain_parts(const DevState &st) {
    using namespace n1k;
    if (!np1024_supported(st.np, st.r) || st.npart != st.nb) return 0;
    if (2 * st.r / kTile + 2 > kChainFresh) return 0;
    const size_t lds = chain_lds_bytes(st.nb);
    if (lds > 160 * 1024) return 0;
    const void *fn = (const void *)k_chain1024;
    int dev = 0, n_cu = 0, per_cu = 0;
    if (hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess) return 0;
    if (hipGetDevice(&dev) != hipSuccess) return 0;
    if (hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, kChainNT, lds) != hipSuccess) return 0;
    return std::min(kChainG, per_cu * n_cu / 8);
}

// one launch per 8 patches (patch b0 + k on XCD slot k); flags: np1024_chain_flag_words() ints
hipError_t launch_np1024_chain(const DevState &st, const int *order_dev, const int *x0_dev, const int *y0_dev,
                               int n_order, const float2 *tw, int *flags, int G, hipStream_t s) {
    if (G < 1 || G > kChainG || !flags || st.meas_g != n1k::N || G != np1024_chain_parts(st)) return hipErrorInvalidValue;
    const size_t lds = chain_lds_bytes(st.nb);
    for (int b0 = 0; b0 < st.B; b0 += 8) {
        ChainArgs a{};
        a.st = st;
        a.tw = tw;
        a.order = order_dev;
        a.x0 = x0_dev;
        a.y0 = y0_dev;
        a.n_order = n_order;
        a.G = G;
        a.b0 = b0;
        a.flags = flags;
        // barrier words and XCC ids restart at zero; the abort word is sticky
        hipError_t e = hipMemsetAsync(flags, 0, (size_t)16 * kChainG * sizeof(int), s);
        if (e == hipSuccess) e = launch_coresident((const void *)k_chain1024, 8 * G, kChainNT, lds, &a, s);
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

}  // namespace fpm
