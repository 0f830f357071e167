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

#include <algorithm>
#include <cstdlib>

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
// launch at config 5; 3 waves without the spills measured slower).  R2 hoists
// half a row at a time (all of it measured slower, 36.4 -> 40.0 us).

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

// R1: grid (ceil(nb / WPB), B), block NT.  Also the previous LED's pupil
// commit (general.hip K5, folded in when `commit`): P += dP / max|objF| on
// this row's disk pixels (:468-475), with max|objF| from the tile-row maxima
// K4 left (:460,467), and the row's max|P| for this LED's update (:415) as
// partial pmax[row] -- the same arithmetic as K5, so the results are
// bit-identical; K5 itself then runs once, after the last LED.
__global__ void __launch_bounds__(n1k::NT) __attribute__((amdgpu_waves_per_eu(4))) k_rows1024_inv(DevState st, StepArgs sa, const float2 *__restrict__ tw,
                                                          int commit) {
    using namespace n1k;
    extern __shared__ __attribute__((aligned(16))) float2 sm[];
    __shared__ float red[WPB];
    const int w = threadIdx.x >> 6, c = (threadIdx.x >> 4) & 3, t = threadIdx.x & 15, xrd = exch_rbase_half(t);
    const int lane = threadIdx.x & 63;
    const int r = st.r, nb = st.nb, b = blockIdx.y, row = blockIdx.x * WPB + w;
    // the twiddle table's loads, max|objF| of the previous LED from K4's
    // tile-row maxima, then the first half row's loads, all issued before the
    // twiddle stores and the reduction's barriers: their memory latencies
    // overlap instead of following each other (loads unconditional: a branch
    // on `commit` waited for its load)
    static_assert(N % NT == 0, "whole rounds");
    float2 twv[N / NT];
#pragma unroll
    for (int i = 0; i < N / NT; ++i) twv[i] = tw[threadIdx.x + NT * i];
    const float2 *twL = sm;
    float2 *wt = sm + N + w * WTILE;
    float rm[2];
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        const int i = threadIdx.x + NT * k;
        rm[k] = st.rmax[(size_t)b * st.nty + (i < st.nty ? i : 0)];
    }
    const int rowc = row < nb ? row : nb - 1;  // rows past the box: in-bounds loads, discarded
    const int ky = rowc - r, w2 = r * r - ky * ky;
    float2 *pup = st.pupil + ((size_t)b * nb + rowc) * nb + r;        // indexed by kx
    const float2 *dP = st.dP + ((size_t)b * nb + rowc) * nb + r;
    const size_t srow = (size_t)(sa.yc + ky) * st.L + sa.xc;         // + kx (:358-362)
    float2 x[16];
    float pmx = 0.f;
    // The row's loads half a row at a time, each half's loads all issued
    // before its arithmetic and pupil stores (a store to pup between the loads
    // made the compiler keep them in program order: pup may alias the
    // spectrum and dP).  The loads are unconditional (a lane off the disk
    // reads the row's centre pixel, in bounds, and its value is masked) and
    // the fp16 spectrum is widened after them: a masked spec_ld, converting
    // where it loaded, waited for each of its loads in turn (16 memory round
    // trips per row); all sixteen at once spilled 22 VGPRs.
    struct Half {
        float2 pv[8], dv[8], ov[8];
        __half2 hv[8];
        int kc[8];
    };
    auto load_half = [&](int hh, Half &q) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int kx = fold(4 * (t + 16 * (8 * hh + i)) + c);
            q.kc[i] = kx * kx <= w2 ? kx : 0;
            q.pv[i] = pup[q.kc[i]];
            q.dv[i] = dP[q.kc[i]];  // unconditional (used only when commit): a branch here waited for the load
        }
        if (st.spec16) {  // uniform
            const __half2 *sp = st.spec16 + (size_t)b * st.L * st.L + srow;
#pragma unroll
            for (int i = 0; i < 8; ++i) q.hv[i] = sp[q.kc[i]];
        } else {
            const float2 *sp = st.spec + (size_t)b * st.L * st.L + srow;
#pragma unroll
            for (int i = 0; i < 8; ++i) q.ov[i] = sp[q.kc[i]];
        }
    };
    Half q;
    load_half(0, q);
#pragma unroll
    for (int i = 0; i < N / NT; ++i) sm[threadIdx.x + NT * i] = twv[i];
    if (!commit) __syncthreads();  // block-uniform; else block_max's barriers order the stores
    float omax = 1.f;
    if (commit) {  // block-uniform
        float m = 0.f;
#pragma unroll
        for (int k = 0; k < 2; ++k)
            if ((int)threadIdx.x + NT * k < st.nty) m = fmaxf(m, rm[k]);
        for (int i = threadIdx.x + 2 * NT; i < st.nty; i += NT) m = fmaxf(m, st.rmax[(size_t)b * st.nty + i]);  // L > 8192 only
        omax = block_max_nonneg(m, red);
    }
    if (row >= nb) return;  // wave-uniform; no block barrier follows
    auto body = [&](int j, float2 p, float2 d, float2 o) {
        const int kx = fold(4 * (t + 16 * j) + c);
        x[j] = make_float2(0.f, 0.f);
        if (kx * kx <= w2) {
            if (commit) {
                p.x += d.x / omax;
                p.y += d.y / omax;
                pup[kx] = p;
            }
            pmx = fmaxf(pmx, cmag(p));
            x[j] = cmul(o, p);  // :364
        }
    };
#pragma unroll
    for (int hh = 0; hh < 2; ++hh) {
        if (hh == 1) load_half(1, q);  // behind the first half's pupil stores
        if (st.spec16) {  // uniform
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const float2 f = __half22float2(q.hv[i]);
                body(8 * hh + i, q.pv[i], q.dv[i], make_float2(f.x * st.hinv, f.y * st.hinv));
            }
        } else {
#pragma unroll
            for (int i = 0; i < 8; ++i) body(8 * hh + i, q.pv[i], q.dv[i], q.ov[i]);
        }
    }
    pmx = wave_max_nonneg(pmx);
    if (lane == 0) st.pmax[(size_t)b * st.npart + row] = pmx;
    w1k_DN<true>(x, wt, twL, c, t, xrd);                                 // :365 (rows)
    if (st.T16) {  // fp16 scratch: one power-of-two scale per box row
        float m = 0.f;
#pragma unroll
        for (int j = 0; j < 16; ++j) m = fmaxf(m, fmaxf(fabsf(x[j].x), fabsf(x[j].y)));
        float inv;
        const float sc = h16_scale(wave_max_nonneg(m), &inv);
        __half2 *T = st.T16 + ((size_t)b * nb + row) * N + t + 64 * c;
#pragma unroll
        for (int p = 0; p < 4; ++p)
#pragma unroll
            for (int bb = 0; bb < 4; ++bb)
                T[16 * bb + 256 * p] = __float22half2_rn(make_float2(x[4 * p + bb].x * sc, x[4 * p + bb].y * sc));
        if (lane == 0) st.tsr[(size_t)b * nb + row] = inv;
        return;
    }
    float2 *T = st.T + ((size_t)b * nb + row) * N + t + 64 * c;
#pragma unroll
    for (int p = 0; p < 4; ++p)
#pragma unroll
        for (int bb = 0; bb < 4; ++bb) T[16 * bb + 256 * p] = x[4 * p + bb];
}

// C: grid (N / CW, B), block 64 CW: CW adjacent columns, a wave each (CW 8:
// 64-byte row segments of T per block; 4 and 16 measured slower)
template <int CW>
__global__ void __launch_bounds__(64 * CW) __attribute__((amdgpu_waves_per_eu(4))) k_cols1024(DevState st, StepArgs sa, const float2 *__restrict__ tw) {
    using namespace n1k;
    constexpr int NTC = 64 * CW, SPCC = CW + 1;
    extern __shared__ __attribute__((aligned(16))) float2 sm[];
    const int w = threadIdx.x >> 6, c = (threadIdx.x >> 4) & 3, t = threadIdx.x & 15, xrd = exch_rbase_half(t);
    // the twiddle table and the strip staged together, under one barrier: a
    // thread's twiddle loads, then its strip loads, all issued before any LDS
    // store (the twiddles' own barrier kept the strip's loads behind it)
    static_assert(N % NTC == 0, "whole rounds");
    float2 twv[N / NTC];
#pragma unroll
    for (int i = 0; i < N / NTC; ++i) twv[i] = tw[threadIdx.x + NTC * i];
    const float2 *twL = sm;
    float2 *strip = sm + N;            // nb x SPCC (box rows only); the wave tiles
    float2 *wt = strip + w * WTILE;    // alias it while every column is in registers
    // XCD-aware column groups: the dispatcher deals blocks round-robin over the
    // 8 XCDs, so XCD k gets column groups k*G/8 .. (k+1)*G/8 - 1 (contiguous)
    constexpr int G = N / CW;
    const int cg = (blockIdx.x & 7) * (G / 8) + (blockIdx.x >> 3);
    const int r = st.r, nb = st.nb, b = blockIdx.y, x0 = cg * CW;
    float2 *T = st.T ? st.T + (size_t)b * nb * N + x0 : nullptr;
    __half2 *T16 = st.T16 ? st.T16 + (size_t)b * nb * N + x0 : nullptr;
    // FFT row i of a column is box row j = i + r (i <= r) or i - N + r
    // (i >= N - r) (:364: every other row is zero)
    // the box rows of the strip: a thread's loads all issued before its LDS
    // stores (clamped indices, masked stores; the rolled loop waited for each
    // load in turn, ~10 memory round trips per thread at config 5)
    {
        constexpr int KMAX = (N * CW + NTC - 1) / NTC;  // nb <= N rows
        const int tot = nb * CW;
        auto store_tw = [&]() {
#pragma unroll
            for (int i = 0; i < N / NTC; ++i) sm[threadIdx.x + NTC * i] = twv[i];
        };
        if (T16) {  // uniform
            __half2 hv[KMAX];
            float sv[KMAX];
#pragma unroll
            for (int k = 0; k < KMAX; ++k) {
                const int idx = min((int)threadIdx.x + NTC * k, tot - 1), j = idx / CW, cc = idx - j * CW;
                if (NTC * k < tot) {  // uniform
                    hv[k] = T16[(size_t)j * N + cc];
                    sv[k] = st.tsr[(size_t)b * nb + j];
                }
            }
            store_tw();
#pragma unroll
            for (int k = 0; k < KMAX; ++k) {
                const int idx = (int)threadIdx.x + NTC * k, j = idx / CW, cc = idx - j * CW;
                if (NTC * k < tot && idx < tot) {
                    const float2 h = __half22float2(hv[k]);
                    strip[j * SPCC + cc] = make_float2(h.x * sv[k], h.y * sv[k]);
                }
            }
        } else {
            float2 tv[KMAX];
#pragma unroll
            for (int k = 0; k < KMAX; ++k) {
                const int idx = min((int)threadIdx.x + NTC * k, tot - 1), j = idx / CW, cc = idx - j * CW;
                if (NTC * k < tot) tv[k] = T[(size_t)j * N + cc];
            }
            store_tw();
#pragma unroll
            for (int k = 0; k < KMAX; ++k) {
                const int idx = (int)threadIdx.x + NTC * k, j = idx / CW, cc = idx - j * CW;
                if (NTC * k < tot && idx < tot) strip[j * SPCC + cc] = tv[k];
            }
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
        float m = 0.f;
#pragma unroll
        for (int j = 0; j < 16; ++j) m = fmaxf(m, fmaxf(fabsf(x[j].x), fabsf(x[j].y)));
        float inv;
        sc = h16_scale(wave_max_nonneg(m), &inv);
        if ((threadIdx.x & 63) == 0) st.tsc[(size_t)b * N + x0 + w] = inv;
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
    for (int idx = threadIdx.x; idx < nb * CW; idx += NTC) {
        const int j = idx / CW, cc = idx - j * CW;
        if (T16) T16[(size_t)j * N + cc] = __float22half2_rn(strip[j * SPCC + cc]);
        else T[(size_t)j * N + cc] = strip[j * SPCC + cc];
    }
}

// R2: grid (ceil(nb / WPB), B), block NT
__global__ void __launch_bounds__(n1k::NT) k_rows1024_fwd(DevState st, StepArgs sa, const float2 *__restrict__ tw) {
    using namespace n1k;
    extern __shared__ __attribute__((aligned(16))) float2 sm[];
    __shared__ float red[WPB];
    const int w = threadIdx.x >> 6, c = (threadIdx.x >> 4) & 3, t = threadIdx.x & 15, xrd = exch_rbase_half(t);
    static_assert(N % NT == 0, "whole rounds");
    float2 twv[N / NT];  // the twiddle table: loads first, stored before block_max's barriers
#pragma unroll
    for (int i = 0; i < N / NT; ++i) twv[i] = tw[threadIdx.x + NT * i];
    const float2 *twL = sm;
    float2 *wt = sm + N + w * WTILE;
    const int r = st.r, nb = st.nb, b = blockIdx.y, row = blockIdx.x * WPB + w;
    // the row's T first (its memory latency runs under the max|P| reduction
    // below), then max|P| of the previous commit from its npart partial
    // maxima (:415) -- every load of both issued before the first use (the
    // rolled partial loop waited for each load in turn)
    const int rowc = row < nb ? row : nb - 1;  // rows past the box: in-bounds loads, discarded
    float2 x[16];
    __half2 hT[16];
    float sT[16];
    if (st.T16) {  // uniform
        const __half2 *Tr = st.T16 + ((size_t)b * nb + rowc) * N + c;
        const float *is = st.tsc + (size_t)b * N + c;
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            hT[j] = Tr[4 * (t + 16 * j)];
            sT[j] = is[4 * (t + 16 * j)];
        }
    } else {
        const float2 *Tr = st.T + ((size_t)b * nb + rowc) * N + c;
#pragma unroll
        for (int j = 0; j < 16; ++j) x[j] = Tr[4 * (t + 16 * j)];
    }
    constexpr int KP = (N + NT - 1) / NT;  // npart = nb <= N partials
    float pv4[KP];
#pragma unroll
    for (int k = 0; k < KP; ++k) {
        const int i = threadIdx.x + NT * k;
        pv4[k] = st.pmax[b * st.npart + (i < st.npart ? i : 0)];
    }
    float pm = 0.f;
#pragma unroll
    for (int k = 0; k < KP; ++k)
        if ((int)threadIdx.x + NT * k < st.npart) pm = fmaxf(pm, pv4[k]);
#pragma unroll
    for (int i = 0; i < N / NT; ++i) sm[threadIdx.x + NT * i] = twv[i];
    pm = block_max_nonneg(pm, red);
    if (row >= nb) return;
    const int ky = row - r, w2 = r * r - ky * ky;
    if (st.T16) {  // column j's element times its column scale
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            const float2 h = __half22float2(hT[j]);
            x[j] = make_float2(h.x * sT[j], h.y * sT[j]);
        }
    }
    w1k_DN<false>(x, wt, twL, c, t, xrd);                                // :394 (rows)
    float2 *pup = st.pupil + ((size_t)b * nb + row) * nb + r;
    float2 *dP = st.dP + ((size_t)b * nb + row) * nb + r;
    const size_t srow = (size_t)(sa.yc + ky) * st.L + sa.xc;
    // the loads of half the row's pixels ahead of their stores (the stores may
    // alias the loads, so the compiler keeps program order: one memory latency
    // per pixel otherwise; config 5 +1.3 %, profiles/r04_ab/wave_dpp_r2_ab.txt;
    // all sixteen ahead measured slower, 36.4 -> 40.0 us)
#pragma unroll
    for (int hp = 0; hp < 2; ++hp) {
        float2 ov[8], pv[8];
        // unconditional loads (off-disk lanes read the row's centre pixel,
        // masked below), the fp16 spectrum widened after all of them (see R1)
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int kx = fold(t + 16 * (4 * c + (i & 3)) + 256 * (2 * hp + (i >> 2)));
            pv[i] = pup[kx * kx <= w2 ? kx : 0];
        }
        if (st.spec16) {  // uniform
            const __half2 *sp = st.spec16 + (size_t)b * st.L * st.L + srow;
            __half2 hv[8];
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const int kx = fold(t + 16 * (4 * c + (i & 3)) + 256 * (2 * hp + (i >> 2)));
                hv[i] = sp[kx * kx <= w2 ? kx : 0];
            }
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const float2 f = __half22float2(hv[i]);
                ov[i] = make_float2(f.x * st.hinv, f.y * st.hinv);
            }
        } else {
            const float2 *sp = st.spec + (size_t)b * st.L * st.L + srow;
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const int kx = fold(t + 16 * (4 * c + (i & 3)) + 256 * (2 * hp + (i >> 2)));
                ov[i] = sp[kx * kx <= w2 ? kx : 0];
            }
        }
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int p = 2 * hp + (i >> 2), bb = i & 3;
            const int kx = fold(t + 16 * (4 * c + bb) + 256 * p);
            if (kx * kx > w2) continue;
            const size_t si = srow + kx;
            const float2 o = ov[i];                              // pre-update Objfcrop (:361)
            const float2 pp = pv[i];
            const float2 D = csub(x[4 * p + bb], cmul(o, pp));   // Objfup - ObjfcropP (:409,463)
            const float pa = cmag(pp);                           // object update (:406-419,433)
            const float2 dpc = cmul(cmul(D, cscale(cconj(pp), pa)), upd_coef_div(pa * pa + st.delta2, st.d2_im, pm));
            spec_st(st, b, si, cadd(o, dpc));
            const float oa = cmag(o);                            // pupil numerator (:459-464,469)
            dP[kx] = cmul(cmul(D, cscale(cconj(o), oa)), upd_coef_div(oa * oa + st.delta1, st.d1_im, 1.0f));
        }
    }
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

}  // namespace fpm
