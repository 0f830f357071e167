// objcrop.hip -- objCrop = IDFT2(objF) / L^2 every iteration (fpmMain.cpp:481)
// for L = 256*M, M in {2, 3, 4} (the fused path's L = Np * resImprovementFactor
// with Np = 256).  objF = fftShift(spec), spec being the centred spectrum the
// solver stores (fpm_state.hpp).
//
// One L-point transform per 16-lane group, entirely in registers:
//   x[i], i = M*m + c  (c < M, m < 256):  Y_c = DFT256(x[M*m + c])      (M four-step 256s)
//   X[k' + 256 p] = sum_c W_L^{c k'} W_M^{c p} Y_c[k']                  (radix-M combine)
// Lane t holds, for every c, the sub-sequence elements m = t + 16 j (j < 16);
// after each 256-point four-step it holds Y_c[t + 16 r] (r < 16), so the
// radix-M combine is lane-local.  The fftShift of objF is free: rolling the
// row index is a different source row, rolling the element index by L/2 =
// 8*16*M is the register relabel j -> j + 8.
//
// Pass 1 (rows): spec rows -> objcrop rows, direct global loads/stores
//   (lane t reads x[M t + c + 16 M j]: each (c, j) covers 16*M contiguous
//   complex per group; it writes X[t + 16 r + 256 p]: 128 contiguous bytes).
// Pass 2 (columns, in place): a block stages a strip of G columns x L rows
//   through LDS (rows of G*8 contiguous bytes), each group transforms one
//   column in registers, scales by 1/L^2 and the strip is written back.
// HBM: at most 2 x 2 x 8 L^2 bytes per patch per iteration; only the live band
// of the spectrum (fpm_state.hpp) is read in pass 1 and re-read in pass 2.
#include <hip/hip_runtime.h>

#include "dft16.hpp"
#include "dftL.hpp"
#include "dft200.hpp"
#include "dft90.hpp"
#include "fpm_state.hpp"


namespace fpm {

typedef float f32x4_nt __attribute__((ext_vector_type(4)));

namespace {

// live-band test: a <= i <= b
__device__ __forceinline__ bool in_band(int i, int a, int b) { return (unsigned)(i - a) <= (unsigned)(b - a); }

// pass 1: row IDFTs of fftShift(spec) over the live rows [sy0, sy1] only
// (fpm_state.hpp: every other spec row is exactly zero, so its objF row's
// IDFT is zero; pass 2 treats those rows as zero instead of reading them),
// loading only the live columns [sx0, sx1].  grid (ceil((sy1-sy0+1) / G), B),
// block 16 G
template <int M, int G>
__global__ void __launch_bounds__(16 * G) k_crop_rows(const float2 *__restrict__ spec, float2 *__restrict__ out,
                                                      const float2 *__restrict__ tw_L, int sy0, int sy1, int sx0,
                                                      int sx1) {
    constexpr int L = 256 * M;
    extern __shared__ __attribute__((aligned(16))) float2 sm[];
    float2 *twL = sm;                  // L
    float2 *scr_all = sm + L;          // G exchange tiles
    const int g = threadIdx.x >> 4, t = threadIdx.x & 15;
    const int xrd = exch_rbase(t);
    float2 *scr = scr_all + g * XTILE;
    float2 wt[16];
    load_twiddles(twL, tw_L, L, M, wt, t);
    const int b = blockIdx.y, srow = sy0 + blockIdx.x * G + g;
    const bool live = srow <= sy1;     // group-uniform; no block barrier follows
    const int row = srow + L / 2 < L ? srow + L / 2 : srow - L / 2;     // objF row = spec row + L/2
    const float2 *src = spec + (size_t)b * L * L + (size_t)(live ? srow : sy1) * L;
    float2 x[M][16];
#pragma unroll
    for (int j = 0; j < 16; ++j)
#pragma unroll
        for (int c = 0; c < M; ++c) {  // element roll by L/2
            const int sc = M * (t + 16 * j) + c;
            x[c][(j + 8) & 15] = in_band(sc, sx0, sx1) ? src[sc] : make_float2(0.f, 0.f);
        }
    dftL_regs<M, true>(x, scr, wt, twL, t, xrd);
    if (!live) return;
    float2 *dst = out + (size_t)b * L * L + (size_t)row * L;
#pragma unroll
    for (int p = 0; p < M; ++p)
#pragma unroll
        for (int r = 0; r < 16; ++r) dst[t + 16 * r + 256 * p] = x[p][r];
}

// pass 2: column IDFTs in place, scaled 1/L^2.  grid (L / G, B), block 16 G.
// The strip goes through LDS in two halves of L/2 rows: element i of a column
// is in half i / (L/2), i.e. register j / 8 on input (i = M (t + 16 j) + c) and
// the compile-time set r + 16 p < 8 M on output (k = t + 16 r + 256 p), so a
// half-size strip (58 KB at L = 768) lets two blocks share a CU and overlap
// one block's HBM phase with the other's transform.
// Rows of the intermediate outside the live band (objF row i <-> spec row
// i + L/2 mod L) were not written by pass 1 and are read as zero.
template <int M, int G>
__global__ void __launch_bounds__(16 * G) k_crop_cols(float2 *__restrict__ io, const float2 *__restrict__ tw_L,
                                                      float scale, int sy0, int sy1) {
    constexpr int L = 256 * M, H = L / 2;
    constexpr int SP = G + 1;          // strip row pitch (complex)
    extern __shared__ __attribute__((aligned(16))) float2 sm[];
    float2 *twL = sm;                  // L
    float2 *strip = sm + L;            // H x SP
    float2 *scr_all = strip;           // G exchange tiles, inside the strip: used
                                       // only while every column is in registers
    const int g = threadIdx.x >> 4, t = threadIdx.x & 15;
    const int xrd = exch_rbase(t);
    float2 *scr = scr_all + g * XTILE;
    float2 wt[16];
    load_twiddles(twL, tw_L, L, M, wt, t);
    const int b = blockIdx.y, c0 = blockIdx.x * G;
    float2 *base = io + (size_t)b * L * L + c0;
    constexpr int NTH = 16 * G;
    float2 x[M][16];
    constexpr int G2 = G / 2;
    // Both halves' strip loads are issued before the first barrier (twice
    // the bytes in flight per block), parked in registers until their half's
    // LDS round: objCrop 0.636 -> 0.584 ms per step at the metric config
    // (same box, profiles/r03_ab/crop_preload_ab.txt).  L = 1024 would need
    // 257 VGPRs for it and keeps the per-half loads.
    constexpr bool PRELOAD = M <= 3;
    constexpr int NLD = PRELOAD ? (H * G2 + NTH - 1) / NTH : 1;
    float4 qh[2][NLD];
    if constexpr (PRELOAD) {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int ya = max(sy0 - (1 - h) * H, 0), yb = min(sy1 - (1 - h) * H, H - 1);
#pragma unroll
            for (int k = 0; k < NLD; ++k) {
                const int idx = ya * G2 + threadIdx.x + k * NTH;
                if (idx < (yb + 1) * G2) {
                    const int y = idx / G2, cc = 2 * (idx - y * G2);
                    qh[h][k] = *(const float4 *)(base + (size_t)(y + h * H) * L + cc);
                }
            }
        }
    }
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        // objF row y + h H is spec row y + (1 - h) H: the live rows of this
        // half are the contiguous range [ya, yb]
        const int ya = max(sy0 - (1 - h) * H, 0), yb = min(sy1 - (1 - h) * H, H - 1);
        if constexpr (PRELOAD) {
#pragma unroll
            for (int k = 0; k < NLD; ++k) {
                const int idx = ya * G2 + threadIdx.x + k * NTH;
                if (idx < (yb + 1) * G2) {
                    const int y = idx / G2, cc = 2 * (idx - y * G2);
                    strip[y * SP + cc] = make_float2(qh[h][k].x, qh[h][k].y);
                    strip[y * SP + cc + 1] = make_float2(qh[h][k].z, qh[h][k].w);
                }
            }
        } else {
            // strip load: consecutive threads take consecutive column pairs of a row
            // (16-byte loads: twice the bytes in flight per load instruction)
#pragma unroll 4  // strip load/store loop: loads in flight per thread
            for (int idx = ya * G2 + threadIdx.x; idx < (yb + 1) * G2; idx += NTH) {
                const int y = idx / G2, cc = 2 * (idx - y * G2);
                const float4 q = *(const float4 *)(base + (size_t)(y + h * H) * L + cc);
                strip[y * SP + cc] = make_float2(q.x, q.y);
                strip[y * SP + cc + 1] = make_float2(q.z, q.w);
            }
        }
        __syncthreads();
#pragma unroll
        for (int j = 8 * h; j < 8 * h + 8; ++j)
#pragma unroll
            for (int c = 0; c < M; ++c) {
                const int y = M * (t + 16 * j) + c - h * H;
                x[c][j] = (y >= ya && y <= yb) ? strip[y * SP + g] : make_float2(0.f, 0.f);  // ya > yb: none
            }
        __syncthreads();
    }
    dftL_regs<M, true>(x, scr, wt, twL, t, xrd);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        __syncthreads();  // exchange tiles / previous half's reads are done
#pragma unroll
        for (int p = 0; p < M; ++p)
#pragma unroll
            for (int r = 0; r < 16; ++r)
                if ((r + 16 * p < 8 * M) == (h == 0))
                    strip[(t + 16 * r + 256 * p - h * H) * SP + g] = cscale(x[p][r], scale);
        __syncthreads();
#pragma unroll 4  // strip load/store loop: loads in flight per thread
        for (int idx = threadIdx.x; idx < H * G / 2; idx += NTH) {
            const int y = idx / (G / 2), cc = 2 * (idx - y * (G / 2));
            const float2 p0 = strip[y * SP + cc], p1 = strip[y * SP + cc + 1];
            // the output is not re-read: non-temporal stores (0.584 -> 0.569 ms
            // per step at L 768; the 600-point pass measured 1 % slower with them)
            __builtin_nontemporal_store((f32x4_nt){p0.x, p0.y, p1.x, p1.y}, (f32x4_nt *)(base + (size_t)(y + h * H) * L + cc));
        }
    }
}

template <int M, int GR, int G>
hipError_t launch_crop(const DevState &st, float2 *out, const float2 *tw_L, hipStream_t s) {
    constexpr int L = 256 * M;
    const size_t lds_rows = (size_t)(L + GR * XTILE) * sizeof(float2);
    // the exchange tiles alias the half strip: allocate the larger of the two
    constexpr size_t strip = (size_t)L / 2 * (G + 1) > (size_t)G * XTILE ? (size_t)L / 2 * (G + 1) : (size_t)G * XTILE;
    const size_t lds_cols = (L + strip) * sizeof(float2);
    hipError_t e = hipFuncSetAttribute((const void *)k_crop_rows<M, GR>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                       (int)lds_rows);
    if (e != hipSuccess) return e;
    e = hipFuncSetAttribute((const void *)k_crop_cols<M, G>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)lds_cols);
    if (e != hipSuccess) return e;
    if (st.sy0 < 0 || st.sy1 >= L || st.sy0 > st.sy1 || st.sx0 < 0 || st.sx1 >= L || st.sx0 > st.sx1)
        return hipErrorInvalidValue;
    const int nrows = st.sy1 - st.sy0 + 1;
    hipLaunchKernelGGL((k_crop_rows<M, GR>), dim3((nrows + GR - 1) / GR, st.B), dim3(16 * GR), lds_rows, s,
                       (const float2 *)st.spec, out, tw_L, st.sy0, st.sy1, st.sx0, st.sx1);
    hipLaunchKernelGGL((k_crop_cols<M, G>), dim3(L / G, st.B), dim3(16 * G), lds_cols, s, out, tw_L,
                       1.0f / ((float)L * (float)L), st.sy0, st.sy1);
    return hipGetLastError();
}

// ------------------------------------------------------------ L = 600 (= 200 x 3)
// BASELINE config 3 (Np 200, resImprovementFactor 3).  One 600-point transform
// per 10-lane group (dft200.hpp, six groups per wave, lanes 60..63 idle):
//   x[i], i = 3 m + c (c < 3, m < 200): Y_c = DFT200(x[3 m + c]), lane l
//   holding m = l + 10 k (k < 20); then the lane-local radix-3 combine
//   X[k' + 200 p] = sum_c W600^{c k'} W3^{c p} Y_c[k'],  k' = l + 10 k.
// fftShift: the element roll by L/2 = 300 = 3 * 100 is the register relabel
// k -> k + 10 (mod 20); the row roll is the source row, as for L = 256 M.
namespace c600 {
constexpr int L = 600, H = 300, GPW = 6;

// x[c][k] = element 3 (l + 10 k) + c; on return x[p][k] = X[l + 10 k + 200 p]
template <bool INV>
__device__ __forceinline__ void dft600_regs(float2 (&x)[3][20], float2 *tile, const float2 *tw2, const float2 *twL,
                                            int l, int xrd) {
#pragma unroll
    for (int c = 0; c < 3; ++c) dft200<INV, false>(x[c], tile, tw2, l, xrd);
#pragma unroll
    for (int k = 0; k < 20; ++k) {
        const int kp = l + 10 * k;
        float2 z[3];
        z[0] = x[0][k];
        const float2 w1 = twL[kp], w2 = twL[2 * kp];
        z[1] = pout(INV ? pmulc(pin(x[1][k]), pin(w1)) : pmul(pin(x[1][k]), pin(w1)));
        z[2] = pout(INV ? pmulc(pin(x[2][k]), pin(w2)) : pmul(pin(x[2][k]), pin(w2)));
        dft3<INV>(z);
#pragma unroll
        for (int p = 0; p < 3; ++p) x[p][k] = z[p];
    }
}

// W600 table and the four-step table tw2[m1][l] = W200^{l m1} = W600^{3 l m1}
__device__ __forceinline__ void load_tw600(float2 *twL, float2 *tw2, const float2 *__restrict__ tw_L) {
    for (int i = threadIdx.x; i < L; i += blockDim.x) twL[i] = tw_L[i];
    for (int i = threadIdx.x; i < 200; i += blockDim.x) tw2[i] = tw_L[(3 * (i / 10) * (i % 10)) % L];
    __syncthreads();
}

// pass 1: row IDFTs of the live spectrum rows (see k_crop_rows).  grid
// (ceil(nlive / (6 W)), B), block 64 W
template <int W>
__global__ void __launch_bounds__(64 * W) k_crop_rows600(const float2 *__restrict__ spec, float2 *__restrict__ out,
                                                         const float2 *__restrict__ tw_L, int sy0, int sy1, int sx0,
                                                         int sx1) {
    extern __shared__ __attribute__((aligned(16))) float2 sm[];
    float2 *twL = sm, *tw2 = sm + L, *tiles = tw2 + 200;  // 6 W exchange tiles of 100 + a dummy
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, gw = lane / 10;
    const bool act = gw < GPW;
    const int l = act ? lane - 10 * gw : 0, g = w * GPW + (act ? gw : 0);
    // lanes 60..63 run the transform too (no divergence); their exchange goes
    // to a dummy tile so it cannot race with group 0's
    float2 *tile = tiles + (act ? g : GPW * W) * 100;
    const int xrd = opaque_i(l * kXP10);
    load_tw600(twL, tw2, tw_L);
    const int b = blockIdx.y, srow = sy0 + blockIdx.x * GPW * W + g;
    const bool live = act && srow <= sy1;
    const int row = srow + H < L ? srow + H : srow - H;  // objF row = spec row + L/2
    const float2 *src = spec + (size_t)b * L * L + (size_t)(srow <= sy1 ? srow : sy1) * L;
    float2 x[3][20];
#pragma unroll
    for (int k = 0; k < 20; ++k)
#pragma unroll
        for (int c = 0; c < 3; ++c) {  // element roll by L/2: register k -> k + 10
            const int sc = 3 * (l + 10 * k) + c;
            x[c][(k + 10) % 20] = in_band(sc, sx0, sx1) ? src[sc] : make_float2(0.f, 0.f);
        }
    dft600_regs<true>(x, tile, tw2, twL, l, xrd);
    if (!live) return;
    float2 *dst = out + (size_t)b * L * L + (size_t)row * L;
#pragma unroll
    for (int p = 0; p < 3; ++p)
#pragma unroll
        for (int k = 0; k < 20; ++k) dst[l + 10 * k + 200 * p] = x[p][k];
}

// pass 2: column IDFTs in place, scaled 1/L^2, one strip of G = 6 W columns
// per block staged through LDS in NH pieces of L / NH rows (see k_crop_cols).
// Piece h holds input registers k in [h K, (h + 1) K), K = 20 / NH (element
// 3 (l + 10 k) + c, 3 l + c < 30, never straddles a piece boundary of a
// multiple of 30 rows) and the output registers whose rows 10 k + 200 p + l
// (l < 10) fall in it.  The strip moves as 16-byte loads and stores (two
// columns per thread); the loads of piece h + 2 are issued as soon as piece h
// has left its registers, so two pieces are in flight while the block works
// (round 3's version loaded piece by piece with 8-byte loads: 2.4 TB/s, SQ
// wait_any 0.65 of wave cycles).  W 4 / NH 2: 24-column strips (192-byte row
// segments, 64-byte aligned), 59 KB pieces, both pieces' loads in flight from
// the start (round 5: NH 4 -> 2 took config 3's objCrop from 0.448 to 0.345
// ms per step; NH 1, a 600-row strip and one block per CU, 0.45 ms;
// profiles/r05_ab/crop600_pieces_ab.txt).
// grid (ceil(L / G), B), block 64 W
template <int W, int NH>
__global__ void __launch_bounds__(64 * W) k_crop_cols600(float2 *__restrict__ io, const float2 *__restrict__ tw_L,
                                                         float scale, int sy0, int sy1) {
    constexpr int G = GPW * W, SP = G + 1, HH = L / NH, K = 20 / NH, G2 = G / 2;
    static_assert(L % NH == 0 && HH % 30 == 0 && 20 % NH == 0, "pieces of whole 30-row runs");
    static_assert(L % G == 0 && G % 2 == 0, "whole strips of column pairs");
    extern __shared__ __attribute__((aligned(16))) float2 sm[];
    float2 *twL = sm, *tw2 = sm + L, *strip = tw2 + 200;  // HH x SP
    float2 *tiles = strip;  // exchange tiles inside the strip: used only while every column is in registers
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, gw = lane / 10;
    const bool act = gw < GPW;
    const int l = act ? lane - 10 * gw : 0, g = w * GPW + (act ? gw : 0);
    float2 *tile = tiles + (act ? g : G) * 100;  // lanes 60..63: dummy tile (see k_crop_rows600)
    const int xrd = opaque_i(l * kXP10);
    load_tw600(twL, tw2, tw_L);
    const int b = blockIdx.y, c0 = blockIdx.x * G;
    float2 *base = io + (size_t)b * L * L + c0;
    constexpr int NTH = 64 * W, NLD = (HH * G2 + NTH - 1) / NTH;
    // objF row y (0 <= y < L) is spec row (y + H) mod L: the live rows of
    // piece h, [h HH, (h+1) HH), form the contiguous range [ya, yb] relative
    // to the piece (HH divides H, so a piece never wraps)
    auto live = [&](int h, int &ya, int &yb) {
        const int s0 = h * HH >= H ? h * HH - H : h * HH + H;  // spec row of the piece's first row
        ya = max(sy0 - s0, 0);
        yb = min(sy1 - s0, HH - 1);
    };
    float4 q[2][NLD];
    auto issue = [&](int h) {
        int ya, yb;
        live(h, ya, yb);
#pragma unroll
        for (int k = 0; k < NLD; ++k) {
            const int idx = ya * G2 + threadIdx.x + k * NTH;
            if (idx < (yb + 1) * G2) {
                const int y = idx / G2, cc = 2 * (idx - y * G2);
                q[h & 1][k] = *(const float4 *)(base + (size_t)(y + h * HH) * L + cc);
            }
        }
    };
    issue(0);
    issue(1);
    float2 x[3][20];
#pragma unroll
    for (int h = 0; h < NH; ++h) {
        int ya, yb;
        live(h, ya, yb);
#pragma unroll
        for (int k = 0; k < NLD; ++k) {
            const int idx = ya * G2 + threadIdx.x + k * NTH;
            if (idx < (yb + 1) * G2) {
                const int y = idx / G2, cc = 2 * (idx - y * G2);
                strip[y * SP + cc] = make_float2(q[h & 1][k].x, q[h & 1][k].y);
                strip[y * SP + cc + 1] = make_float2(q[h & 1][k].z, q[h & 1][k].w);
            }
        }
        if (h + 2 < NH) issue(h + 2);
        __syncthreads();
#pragma unroll
        for (int k = K * h; k < K * h + K; ++k)
#pragma unroll
            for (int c = 0; c < 3; ++c) {
                const int y = 3 * (l + 10 * k) + c - h * HH;
                x[c][k] = (act && y >= ya && y <= yb) ? strip[y * SP + g] : make_float2(0.f, 0.f);
            }
        __syncthreads();
    }
    dft600_regs<true>(x, tile, tw2, twL, l, xrd);
#pragma unroll
    for (int h = 0; h < NH; ++h) {
        __syncthreads();  // exchange tiles / previous piece's reads are done
        if (act) {
#pragma unroll
            for (int p = 0; p < 3; ++p)
#pragma unroll
                for (int k = 0; k < 20; ++k)
                    if ((10 * k + 200 * p) / HH == h)
                        strip[(l + 10 * k + 200 * p - h * HH) * SP + g] = cscale(x[p][k], scale);
        }
        __syncthreads();
#pragma unroll 4
        for (int idx = threadIdx.x; idx < HH * G2; idx += NTH) {
            const int y = idx / G2, cc = 2 * (idx - y * G2);
            const float2 p0 = strip[y * SP + cc], p1 = strip[y * SP + cc + 1];
            *(float4 *)(base + (size_t)(y + h * HH) * L + cc) = make_float4(p0.x, p0.y, p1.x, p1.y);
        }
    }
}

template <int WR, int WC, int NHC>
hipError_t launch_crop600(const DevState &st, float2 *out, const float2 *tw_L, hipStream_t s) {
    constexpr int GC = GPW * WC;
    const size_t lds_rows = (size_t)(L + 200 + (GPW * WR + 1) * 100) * sizeof(float2);
    constexpr size_t strip = (size_t)(L / NHC) * (GC + 1) > (size_t)(GC + 1) * 100 ? (size_t)(L / NHC) * (GC + 1)
                                                                                  : (size_t)(GC + 1) * 100;
    const size_t lds_cols = (L + 200 + strip) * sizeof(float2);
    hipError_t e = hipFuncSetAttribute((const void *)k_crop_rows600<WR>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                       (int)lds_rows);
    if (e != hipSuccess) return e;
    e = hipFuncSetAttribute((const void *)k_crop_cols600<WC, NHC>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)lds_cols);
    if (e != hipSuccess) return e;
    if (st.sy0 < 0 || st.sy1 >= L || st.sy0 > st.sy1 || st.sx0 < 0 || st.sx1 >= L || st.sx0 > st.sx1)
        return hipErrorInvalidValue;
    const int nrows = st.sy1 - st.sy0 + 1, gr = GPW * WR;
    hipLaunchKernelGGL(k_crop_rows600<WR>, dim3((nrows + gr - 1) / gr, st.B), dim3(64 * WR), lds_rows, s,
                       (const float2 *)st.spec, out, tw_L, st.sy0, st.sy1, st.sx0, st.sx1);
    hipLaunchKernelGGL((k_crop_cols600<WC, NHC>), dim3((L + GC - 1) / GC, st.B), dim3(64 * WC), lds_cols, s, out, tw_L,
                       1.0f / ((float)L * (float)L), st.sy0, st.sy1);
    return hipGetLastError();
}
}  // namespace c600

// ------------------------------------------------------------ L = 360 (= 90 x 4)
// BASELINE configs 1 and 2 (dataset_mono: Np 90, resImprovementFactor 4).
// One 360-point transform per 10-lane group (dft90.hpp, six groups per wave,
// lanes 60..63 idle): x[i], i = 4 m + c (c < 4, m < 90): Y_c = DFT90 of
// x[4 m + c], lane l holding m = l + 10 k (layout A, k < 9), which dft90_ab
// leaves in layout B (lane j < 9 holds Y_c[j + 9 k'], k' < 10); the radix-4
// combine X[k + 90 p] = sum_c W360^{c k} W4^{c p} Y_c[k], k = j + 9 k', is
// lane-local.  The element roll of fftShift (L/2 = 180 = 4 x 45) is not a
// register relabel here, so pass 1 gathers each element from its rolled
// source column.  (Round 3 ran L 360 on the mixed-radix k_fft_batch: full
// rows and columns, 0.15 ms per step at config 2.)
namespace c360 {
constexpr int L = 360, H = 180, GPW = 6;

// x[c][k] = element 4 (l + 10 k) + c (k < 9; x[c][9] scratch); on return
// x[p][k'] = X[j + 9 k' + 90 p] on lanes j < 9
template <bool INV>
__device__ __forceinline__ void dft360_regs(float2 (&x)[4][10], float2 *tile, const float2 *tw90, const float2 *twL,
                                            int l, int xrd) {
#pragma unroll
    for (int c = 0; c < 4; ++c) dft90_ab<INV>(x[c], tile, tw90, l, xrd);
#pragma unroll
    for (int k = 0; k < 10; ++k) {
        const int kk = (l < 9 ? l : 0) + 9 * k;
        float2 z[4];
        z[0] = x[0][k];
#pragma unroll
        for (int c = 1; c < 4; ++c) {
            const pf2 w = pin(twL[c * kk]);  // c kk < 270 < L
            z[c] = pout(INV ? pmulc(pin(x[c][k]), w) : pmul(pin(x[c][k]), w));
        }
        dft4<INV>(z);
#pragma unroll
        for (int p = 0; p < 4; ++p) x[p][k] = z[p];
    }
}

// W360 table and tw90[a * 10 + b] = W90^{a b} = W360^{4 a b}
__device__ __forceinline__ void load_tw360(float2 *twL, float2 *tw90, const float2 *__restrict__ tw_L) {
    for (int i = threadIdx.x; i < L; i += blockDim.x) twL[i] = tw_L[i];
    for (int i = threadIdx.x; i < 100; i += blockDim.x) tw90[i] = tw_L[(4 * (i / 10) * (i % 10)) % L];
    __syncthreads();
}

// objF row / column i holds spec row / column (i + H) mod L
__device__ __forceinline__ int roll360(int i) { return i + H < L ? i + H : i - H; }

// pass 1: row IDFTs of the live spectrum rows.  grid (ceil(nlive / (6 W)), B), block 64 W
template <int W>
__global__ void __launch_bounds__(64 * W) k_crop_rows360(const float2 *__restrict__ spec, float2 *__restrict__ out,
                                                         const float2 *__restrict__ tw_L, int sy0, int sy1, int sx0,
                                                         int sx1) {
    extern __shared__ __attribute__((aligned(16))) float2 sm[];
    float2 *twL = sm, *tw90 = sm + L, *tiles = tw90 + 100;  // 6 W exchange tiles of 100 + a dummy
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, gw = lane / 10;
    const bool act = gw < GPW;
    const int l = act ? lane - 10 * gw : 0, g = w * GPW + (act ? gw : 0);
    float2 *tile = tiles + (act ? g : GPW * W) * 100;
    const int xrd = opaque_i(l * kXP90);
    load_tw360(twL, tw90, tw_L);
    const int b = blockIdx.y, srow = sy0 + blockIdx.x * GPW * W + g;
    const bool live = act && srow <= sy1;
    const float2 *src = spec + (size_t)b * L * L + (size_t)(srow <= sy1 ? srow : sy1) * L;
    float2 x[4][10];
#pragma unroll
    for (int k = 0; k < 9; ++k)
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            const int sc = roll360(4 * (l + 10 * k) + c);  // objF element i <- spec column (i + H) mod L
            x[c][k] = in_band(sc, sx0, sx1) ? src[sc] : make_float2(0.f, 0.f);
        }
    dft360_regs<true>(x, tile, tw90, twL, l, xrd);
    if (!live || l >= 9) return;
    float2 *dst = out + (size_t)b * L * L + (size_t)roll360(srow) * L;  // objF row = spec row + L/2
#pragma unroll
    for (int p = 0; p < 4; ++p)
#pragma unroll
        for (int k = 0; k < 10; ++k) dst[l + 9 * k + 90 * p] = x[p][k];
}

// pass 2: column IDFTs in place, scaled 1/L^2, one strip of G = 6 W columns
// per block through LDS in one piece (L x (G + 1) complex: 72 KB at W 4, two
// blocks per CU), 16-byte loads and stores.  Rows of the intermediate outside
// the live band were not written by pass 1 and are read as zero.
// grid (L / G, B), block 64 W
template <int W>
__global__ void __launch_bounds__(64 * W) k_crop_cols360(float2 *__restrict__ io, const float2 *__restrict__ tw_L,
                                                         float scale, int sy0, int sy1) {
    constexpr int G = GPW * W, SP = G + 1, G2 = G / 2, NTH = 64 * W;
    static_assert(L % G == 0 && G % 2 == 0, "whole strips of column pairs");
    extern __shared__ __attribute__((aligned(16))) float2 sm[];
    float2 *twL = sm, *tw90 = sm + L, *strip = tw90 + 100;  // L x SP
    float2 *tiles = strip;  // exchange tiles inside the strip: used only while every column is in registers
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, gw = lane / 10;
    const bool act = gw < GPW;
    const int l = act ? lane - 10 * gw : 0, g = w * GPW + (act ? gw : 0);
    float2 *tile = tiles + (act ? g : G) * 100;
    const int xrd = opaque_i(l * kXP90);
    load_tw360(twL, tw90, tw_L);
    const int b = blockIdx.y, c0 = blockIdx.x * G;
    float2 *base = io + (size_t)b * L * L + c0;
    auto live = [&](int y) { return in_band(roll360(y), sy0, sy1); };
    // live objF rows: [0, sy1 - H] and [sy0 + H, L) when the band straddles
    // the spectrum's middle row, [sy0 - H, sy1 - H] or [sy0 + H, sy1 + H] otherwise
    for (int idx = threadIdx.x; idx < L * G2; idx += NTH) {
        const int y = idx / G2, cc = 2 * (idx - y * G2);
        if (live(y)) {
            const float4 q = *(const float4 *)(base + (size_t)y * L + cc);
            strip[y * SP + cc] = make_float2(q.x, q.y);
            strip[y * SP + cc + 1] = make_float2(q.z, q.w);
        }
    }
    __syncthreads();
    float2 x[4][10];
#pragma unroll
    for (int k = 0; k < 9; ++k)
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            const int y = 4 * (l + 10 * k) + c;
            x[c][k] = (act && live(y)) ? strip[y * SP + g] : make_float2(0.f, 0.f);
        }
    __syncthreads();
    dft360_regs<true>(x, tile, tw90, twL, l, xrd);
    __syncthreads();  // exchange tiles are done before the strip is rewritten
    if (act && l < 9) {
#pragma unroll
        for (int p = 0; p < 4; ++p)
#pragma unroll
            for (int k = 0; k < 10; ++k) strip[(l + 9 * k + 90 * p) * SP + g] = cscale(x[p][k], scale);
    }
    __syncthreads();
#pragma unroll 4
    for (int idx = threadIdx.x; idx < L * G2; idx += NTH) {
        const int y = idx / G2, cc = 2 * (idx - y * G2);
        const float2 p0 = strip[y * SP + cc], p1 = strip[y * SP + cc + 1];
        *(float4 *)(base + (size_t)y * L + cc) = make_float4(p0.x, p0.y, p1.x, p1.y);
    }
}

template <int WR, int WC>
hipError_t launch_crop360(const DevState &st, float2 *out, const float2 *tw_L, hipStream_t s) {
    constexpr int GC = GPW * WC;
    const size_t lds_rows = (size_t)(L + 100 + (GPW * WR + 1) * 100) * sizeof(float2);
    constexpr size_t strip = (size_t)L * (GC + 1) > (size_t)(GC + 1) * 100 ? (size_t)L * (GC + 1) : (size_t)(GC + 1) * 100;
    const size_t lds_cols = (L + 100 + strip) * sizeof(float2);
    hipError_t e = hipFuncSetAttribute((const void *)k_crop_rows360<WR>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                       (int)lds_rows);
    if (e != hipSuccess) return e;
    e = hipFuncSetAttribute((const void *)k_crop_cols360<WC>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)lds_cols);
    if (e != hipSuccess) return e;
    if (st.sy0 < 0 || st.sy1 >= L || st.sy0 > st.sy1 || st.sx0 < 0 || st.sx1 >= L || st.sx0 > st.sx1)
        return hipErrorInvalidValue;
    const int nrows = st.sy1 - st.sy0 + 1, gr = GPW * WR;
    hipLaunchKernelGGL(k_crop_rows360<WR>, dim3((nrows + gr - 1) / gr, st.B), dim3(64 * WR), lds_rows, s,
                       (const float2 *)st.spec, out, tw_L, st.sy0, st.sy1, st.sx0, st.sx1);
    hipLaunchKernelGGL(k_crop_cols360<WC>, dim3(L / GC, st.B), dim3(64 * WC), lds_cols, s, out, tw_L,
                       1.0f / ((float)L * (float)L), st.sy0, st.sy1);
    return hipGetLastError();
}
}  // namespace c360

}  // namespace

constexpr int kCropG = 16;   // columns per strip: 128-byte row segments
constexpr int kCropGR = 4;   // rows per block in the row pass

// hipErrorNotSupported when L is not 512 / 768 / 1024 / 600 / 360 (caller falls back to
// the mixed-radix batched transform)
hipError_t launch_objcrop_regs(const DevState &st, float2 *out, const float2 *tw_L, hipStream_t s) {
    switch (st.L) {
        case 512: return launch_crop<2, kCropGR, kCropG>(st, out, tw_L, s);
        case 768: return launch_crop<3, kCropGR, kCropG>(st, out, tw_L, s);
        case 1024: return launch_crop<4, kCropGR, kCropG>(st, out, tw_L, s);
        // L 600: row pass 12 rows per block (2 waves; 6 rows: 0.345 -> 0.336 ms
        // per step), column pass 24-column strips in two pieces
        case 600: return c600::launch_crop600<2, 4, 2>(st, out, tw_L, s);
        case 360: return c360::launch_crop360<1, 4>(st, out, tw_L, s);
        default: return hipErrorNotSupported;
    }
}

}  // namespace fpm
