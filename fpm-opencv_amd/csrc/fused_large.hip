// fused_large.hip -- the fused per-patch FPM iteration for Np 256 at pupil
// radii beyond the one-workgroup Np 256 kernel (34 < r < 128; dataset_mono
// at cropSizeX 256: r 84, L 1024).  ONE launch per runFPM iteration, one
// 1024-thread workgroup per patch walking every LED of the order
// (fpmMain.cpp:348-476), with no inter-workgroup communication.
//
// At r 84 the support box has 169 rows and the row-transform intermediate T
// (169 x 256 complex, 346 KB) does not fit in LDS (fpm_fused.hip keeps its
// 67 x 128 halves there), so T lives in a per-patch global scratch that the
// workgroup writes and reads back within one LED step: on one CU, from the
// XCD's L2 (8 patches of one XCD hold 2.8 MB of T).  Per LED step, 64 16-lane
// groups (g, lane t) run the np256.hip transforms (dft256_full, natural order:
// lane t holds elements t + 16 j):
//
//   A  row IDFTs of the box rows (group g: rows g, g + 64, ...): O * P on the
//      disk, IDFT, the T row stored as 128-byte segments           (:358-365)
//   B  four rounds of 64 columns (one per group): the box rows of T staged
//      through an LDS strip with 512-byte row segments, column IDFT,
//      amplitude replacement against the stack in the fused column layout
//      (g = 16), column DFT, box rows back to T                 (:365-394)
//   C  row DFTs of the box rows, object update and pupil numerator on the
//      disk pixels                                       (:394-447,457-464)
//   max  tile maxima of the window's 16 x 16 tiles (general.hip K4's values),
//      the tile-row maxima in LDS, exact max|objF|                (:460,467)
//   P  P += num / max|objF| on the disk, max|P| for the next LED  (:468-475,415)
//
// Every pixel a lane touches in A, C and P is the same (row, kx) in all three,
// so the pupil, numerator and spectrum values it stores and later loads need
// no barrier between those phases; the barriers order T (A -> B -> C) and the
// window's spectrum (C -> tile maxima -> next A).
#include <hip/hip_runtime.h>

#include "cpk.hpp"
#include "dftL.hpp"
#include "fpm_state.hpp"
#include "fused_sync.hpp"
#include "ledtab.hpp"

#include <algorithm>

namespace fpm {

#ifndef FPM_LARGE_NT
#define FPM_LARGE_NT 512
#endif
namespace flg {
constexpr int N = 256, H = N / 2;
constexpr int NT = FPM_LARGE_NT, NG = NT / 16, NW = NT / 64;  // 32 groups, 8 waves
constexpr int CR = NG;                                 // columns per pass-B round (one per group)
constexpr int SPB = CR + 1;                            // strip row pitch (complex)
constexpr int KST = N * CR / NT;                       // strip elements per thread (nb <= N)
static_assert(N / CR * CR == N, "whole rounds");
}  // namespace flg

#ifndef FPM_LARGE_STAMPS
#define FPM_LARGE_STAMPS 0  // 1: phase stamps (FPM_STAMPS=1); compiled out by default
#endif

struct LargeArgs {
    DevState st;
    const uint16_t *meas;  // [nS][B][x][16 t + m] = I[t + 16 m][x] (meas_layout g = 16)
    LedTab tab;
    const float2 *tw;      // exp(-2 pi i k / 256), k < 256
    int n_order;
    int tab_off;           // byte offset of the LDS LED table, or -1
    unsigned long long *dbg;  // FPM_STAMPS=1 phase cycles (FPM_LARGE_STAMPS builds), else null
};

namespace {

__device__ __forceinline__ int fold_l(int k) { return k < flg::H ? k : k - flg::N; }  // signed frequency

__global__ void __launch_bounds__(flg::NT, 1) k_fused_large(LargeArgs a) {
    using namespace flg;
    extern __shared__ __attribute__((aligned(16))) float2 sm[];
    __shared__ float red[NW];
    ClockProbe probe;
    probe.start();
    const DevState &st = a.st;
    const int tid = threadIdx.x, g = tid >> 4, t = tid & 15, lane = tid & 63, w = tid >> 6;
    const int xrd = exch_rbase_half(t);
    const int b = blockIdx.x, r = st.r, nb = st.nb, L = st.L, nty = st.nty, ntx = st.ntx;
    const int nrr = (nb + NG - 1) / NG;  // box rows per group (rounds of A, C and P)
    float2 *twL = sm;
    float2 *strip0 = sm + N;                       // nb x SPB in pass B; the group tiles otherwise
    float2 *wt0 = strip0 + g * XTILE_H;
    const size_t xregion = std::max((size_t)nb * SPB, (size_t)NG * XTILE_H);
    float *rmx = (float *)(strip0 + xregion);       // [nty] tile-row maxima of |objF|
    LedTab tab = a.tab;
    if (a.tab_off >= 0) {
        int2 *tl = (int2 *)((char *)sm + a.tab_off);
        tab.fill(tl, a.n_order, tid, NT);
        tab.lds = tl;
    }
    for (int i = tid; i < N; i += NT) twL[i] = a.tw[i];
    float2 *spec0 = st.spec + (size_t)b * L * L;
    float2 *pup0 = st.pupil + (size_t)b * nb * nb + r;  // + row * nb + kx
    float2 *dP0 = st.dP + (size_t)b * nb * nb + r;
    float2 *Tg0 = st.T + (size_t)b * nb * N;
    float *tmax = st.tmax + (size_t)b * nty * ntx;
    // the tile-row maxima of the whole spectrum, from the tile maxima
    // (fpm_init's, then this kernel's own: exact, no dirty tiles)
    for (int ty = w; ty < nty; ty += NW) {
        float m = 0.f;
        for (int tx = lane; tx < ntx; tx += 64) m = fmaxf(m, tmax[(size_t)ty * ntx + tx]);
        m = wave_max_nonneg(m);
        if (lane == 0) rmx[ty] = m;
    }
    float pm = st.pmax[b];  // max|P| (:415); npart = 1 on the fused path
    __syncthreads();
    const LdsTw tw1{twL, t, 1};
    const float nn = (float)N * (float)N, epsn = st.eps * nn, epsn_im = st.eps_im * nn;
    auto boxrow = [&](int i) { return i <= r ? i + r : (i >= N - r ? i - N + r : -1); };

    unsigned long long acc[kStamps] = {};
    unsigned long long prev = (FPM_LARGE_STAMPS && a.dbg) ? __builtin_amdgcn_s_memtime() : 0ull;
#define FPM_STAMP(i)                                                  \
    if (FPM_LARGE_STAMPS && a.dbg) {                                  \
        const unsigned long long now_ = __builtin_amdgcn_s_memtime(); \
        acc[i] += now_ - prev;                                        \
        prev = now_;                                                  \
    }
    for (int it = 0; it < a.n_order; ++it) {
        const LedPos lp = tab.at(it);
        // per-LED base pointers and lane indices laundered through an empty
        // asm: otherwise the compiler hoists every phase's lane addresses and
        // LDS offsets out of the LED loop and keeps them live across it (126
        // values spilled in the loop preheader, 240 VGPRs of spills in all)
        const int z = opaque_int(0);
        float2 *const spec = spec0 + z, *const pup = pup0 + z, *const dP = dP0 + z, *const Tg = Tg0 + z;
        float2 *const strip = strip0 + z, *const wt = wt0 + z;
        // ---- A: row IDFTs of the box rows (:358-365)
#pragma unroll 1
        for (int k = 0; k < nrr; ++k) {
            const int tq = opaque_int(t), gq = opaque_int(g);
            const int row = gq + NG * k;
            if (row >= nb) break;  // group-uniform
            const int ky = row - r, w2 = r * r - ky * ky;
            const float2 *pr = pup + (size_t)row * nb;
            const float2 *sr = spec + (size_t)(lp.yc + ky) * L + lp.xc;
            float2 x[16];
#pragma unroll
            for (int hh = 0; hh < 2; ++hh) {  // half a row's loads before their use
                float2 pv[8], ov[8];
#pragma unroll
                for (int i = 0; i < 8; ++i) {
                    const int kx = fold_l(tq + 16 * (8 * hh + i)), kc = kx * kx <= w2 ? kx : 0;
                    pv[i] = pr[kc];
                    ov[i] = sr[kc];
                }
#pragma unroll
                for (int i = 0; i < 8; ++i) {
                    const int kx = fold_l(tq + 16 * (8 * hh + i));
                    x[8 * hh + i] = kx * kx <= w2 ? cmul(ov[i], pv[i]) : make_float2(0.f, 0.f);  // :364
                }
            }
            float2 y[16];
            dft256_full<true, true>(x, y, wt, tw1, tq, xrd);  // y[j] = X[tq + 16 j]
            float2 *Tr = Tg + (size_t)row * N + tq;
#pragma unroll
            for (int j = 0; j < 16; ++j) Tr[16 * j] = y[j];
        }
        FPM_STAMP(0)
        __syncthreads();  // T rows of every group
        FPM_STAMP(1)
        // ---- B: columns, four rounds of 64 (:365-394)
        const uint16_t *Im = a.meas + ((size_t)lp.led * st.mB + b) * N * N;
        const int tot = nb * CR;
#pragma unroll 1
        for (int q = 0; q < N / CR; ++q) {
            const int tq = opaque_int(t), gq = opaque_int(g), tidq = opaque_int(tid);
            const int x0 = q * CR;
            // this group's measurement column and the strip's row segments,
            // every load issued before the first LDS store
            const uint4 *Ic = (const uint4 *)(Im + (size_t)(x0 + gq) * N + 16 * tq);
            const uint4 ia = Ic[0], ib = Ic[1];
            float2 tv[KST];
#pragma unroll
            for (int k = 0; k < KST; ++k) {
                const int idx = min(tidq + NT * k, tot - 1);
                if (NT * k < tot) tv[k] = Tg[(size_t)(idx / CR) * N + x0 + (idx % CR)];  // uniform guard
            }
            if (q > 0) __syncthreads();  // the previous round's T stores have read the strip
#pragma unroll
            for (int k = 0; k < KST; ++k) {
                const int idx = tidq + NT * k;
                if (NT * k < tot && idx < tot) strip[(idx / CR) * SPB + (idx % CR)] = tv[k];
            }
            __syncthreads();
            float2 v[16];
#pragma unroll
            for (int m = 0; m < 16; ++m) {
                const int j = boxrow(tq + 16 * m);
                v[m] = j >= 0 ? strip[j * SPB + gq] : make_float2(0.f, 0.f);
            }
            __syncthreads();  // the strip is the group tiles from here
            float2 y[16];
            dft256_full<true, true>(v, y, wt, tw1, tq, xrd);  // y[m] = row tq + 16 m
            const unsigned iw[8] = {ia.x, ia.y, ia.z, ia.w, ib.x, ib.y, ib.z, ib.w};
#pragma unroll
            for (int m = 0; m < 16; ++m) {  // np1024.hip's form of :378-394
                const float iv = (float)((iw[m >> 1] >> (16 * (m & 1))) & 0xffffu);
                const float2 u = y[m];
                const float tr = u.x + epsn, ti = u.y + epsn_im;
                const float s = amp_scale(__builtin_fmaf(tr, tr, ti * ti), iv);
                y[m] = make_float2(u.x * s, u.y * s);
            }
            dft256_full<false, true>(y, v, wt, tw1, tq, xrd);  // :394 (columns)
            __syncthreads();  // every group is done with its tile
#pragma unroll
            for (int m = 0; m < 16; ++m) {
                const int j = boxrow(tq + 16 * m);
                if (j >= 0) strip[j * SPB + gq] = v[m];
            }
            __syncthreads();
            for (int idx = tidq; idx < tot; idx += NT) Tg[(size_t)(idx / CR) * N + x0 + (idx % CR)] = strip[(idx / CR) * SPB + (idx % CR)];
        }
        FPM_STAMP(2)
        __syncthreads();  // T columns of every round; the strip is the group tiles again
        FPM_STAMP(3)
        // ---- C: row DFTs, object update, pupil numerator (:394-447,457-464)
#pragma unroll 1
        for (int k = 0; k < nrr; ++k) {
            const int tq = opaque_int(t), gq = opaque_int(g);
            const int row = gq + NG * k;
            if (row >= nb) break;  // group-uniform
            const int ky = row - r, w2 = r * r - ky * ky;
            const float2 *Tr = Tg + (size_t)row * N + tq;
            float2 x[16];
#pragma unroll
            for (int j = 0; j < 16; ++j) x[j] = Tr[16 * j];
            float2 F[16];
            dft256_full<false, true>(x, F, wt, tw1, tq, xrd);  // F[j] = X[tq + 16 j]
            float2 *pr = pup + (size_t)row * nb;
            float2 *nr = dP + (size_t)row * nb;
            float2 *sr = spec + (size_t)(lp.yc + ky) * L + lp.xc;
#pragma unroll
            for (int hp = 0; hp < 2; ++hp) {
                float2 ov[8], pp[8];
#pragma unroll
                for (int i = 0; i < 8; ++i) {
                    const int kx = fold_l(tq + 16 * (8 * hp + i)), kc = kx * kx <= w2 ? kx : 0;
                    pp[i] = pr[kc];
                    ov[i] = sr[kc];
                }
#pragma unroll
                for (int i = 0; i < 8; ++i) {
                    const int kx = fold_l(tq + 16 * (8 * hp + i));
                    if (kx * kx > w2) continue;
                    const float2 o = ov[i], p = pp[i];                     // pre-update Objfcrop (:361)
                    const float2 D = csub(F[8 * hp + i], cmul(o, p));      // Objfup - ObjfcropP (:409,463)
                    const float pa = cmag(p);                              // object update (:406-419,433)
                    const float2 dpc =
                        cmul(cmul(D, cscale(cconj(p), pa)), upd_coef_div(pa * pa + st.delta2, st.d2_im, pm));
                    sr[kx] = cadd(o, dpc);
                    const float oa = cmag(o);                              // pupil numerator (:459-464,469)
                    nr[kx] = cmul(cmul(D, cscale(cconj(o), oa)), upd_coef_div(oa * oa + st.delta1, st.d1_im, 1.0f));
                }
            }
        }
        FPM_STAMP(4)
        __syncthreads();  // the window's spectrum
        FPM_STAMP(5)
        // ---- tile maxima of the window's tiles (general.hip K4's values)
        const int ty0 = (lp.yc - r) / kTile, ty1 = (lp.yc + r) / kTile;
        {
        const int tx0 = (lp.xc - r) / kTile, tx1 = (lp.xc + r) / kTile;
        const int ntc = tx1 - tx0 + 1, ntiles = (ty1 - ty0 + 1) * ntc;
        for (int k0 = w; k0 < ntiles; k0 += 4 * NW) {  // four tiles of a wave at once
            float m[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int k = min(k0 + NW * u, ntiles - 1), tyk = ty0 + k / ntc, txk = tx0 + k % ntc;
                float2 pv[4];
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const int p = lane + 64 * i, yy = tyk * kTile + (p >> 4), xx = txk * kTile + (p & 15);
                    pv[i] = spec[(yy < L && xx < L) ? (size_t)yy * L + xx : 0];
                }
                float mm = 0.f;
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const int p = lane + 64 * i, yy = tyk * kTile + (p >> 4), xx = txk * kTile + (p & 15);
                    mm = fmaxf(mm, (yy < L && xx < L) ? cmag(pv[i]) : 0.f);
                }
                m[u] = mm;
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int k = k0 + NW * u;
                if (k < ntiles) {  // wave-uniform
                    const float v = wave_max_nonneg(m[u]);
                    if (lane == 0) tmax[(size_t)(ty0 + k / ntc) * ntx + tx0 + k % ntc] = v;
                }
            }
        }
        }
        __syncthreads();
        FPM_STAMP(6)
        // the window's tile rows' maxima (the row's other tiles are unchanged)
        for (int ty = ty0 + w; ty <= ty1; ty += NW) {
            float m = 0.f;
            for (int tx = lane; tx < ntx; tx += 64) m = fmaxf(m, tmax[(size_t)ty * ntx + tx]);
            m = wave_max_nonneg(m);
            if (lane == 0) rmx[ty] = m;
        }
        __syncthreads();
        // exact max|objF| over the whole spectrum (:460,467), in every wave
        float om = 0.f;
        for (int ty = lane; ty < nty; ty += 64) om = fmaxf(om, rmx[ty]);
        const float omax = wave_max_nonneg(om);
        FPM_STAMP(7)
        // ---- P += num / max|objF| on the disk (:468-475), max|P| (:415)
        float pmx = 0.f;
#pragma unroll 1
        for (int k = 0; k < nrr; ++k) {
            const int tq = opaque_int(t), gq = opaque_int(g);
            const int row = gq + NG * k;
            if (row >= nb) break;  // group-uniform
            const int ky = row - r, w2 = r * r - ky * ky;
            float2 *pr = pup + (size_t)row * nb;
            const float2 *nr = dP + (size_t)row * nb;
#pragma unroll
            for (int hp = 0; hp < 2; ++hp) {
                float2 pv[8], dv[8];
#pragma unroll
                for (int i = 0; i < 8; ++i) {
                    const int kx = fold_l(tq + 16 * (8 * hp + i)), kc = kx * kx <= w2 ? kx : 0;
                    pv[i] = pr[kc];
                    dv[i] = nr[kc];
                }
#pragma unroll
                for (int i = 0; i < 8; ++i) {
                    const int kx = fold_l(tq + 16 * (8 * hp + i));
                    if (kx * kx > w2) continue;
                    float2 p = pv[i];
                    p.x += dv[i].x / omax;
                    p.y += dv[i].y / omax;
                    pr[kx] = p;
                    pmx = fmaxf(pmx, cmag(p));
                }
            }
        }
        FPM_STAMP(8)
        pmx = wave_max_nonneg(pmx);
        if (lane == 0) red[w] = pmx;
        __syncthreads();
        FPM_STAMP(9)
        pm = red[0];
#pragma unroll
        for (int i = 1; i < NW; ++i) pm = fmaxf(pm, red[i]);
    }
#undef FPM_STAMP
    if (FPM_LARGE_STAMPS && a.dbg && (tid == 0 || tid == NT - 64))
        for (int i = 0; i < kStamps; ++i) atomicAdd(&a.dbg[(tid ? kStamps : 0) + i], acc[i]);
    probe.stop(st.clk);
    if (tid == 0) st.pmax[b] = pm;
}

size_t large_lds_bytes(int nb, int nty) {
    using namespace flg;
    return (size_t)(N + std::max((size_t)nb * SPB, (size_t)NG * XTILE_H)) * sizeof(float2) + (size_t)nty * sizeof(float);
}

}  // namespace

// Np 256 beyond the one-workgroup kernel's radius (34 < r < 128), fp32
// spectrum, the scratch and its LDS within one CU's 160 KB.
bool fused_large_supported(int np, int r, const DevState &st) {
    if (np != flg::N || r <= 34 || r >= flg::H || st.spec16) return false;
    return large_lds_bytes(2 * r + 1, st.nty) <= 160 * 1024;
}

hipError_t launch_fused_large_iteration(const DevState &st, const uint16_t *meas, const int *order_dev,
                                        const int *x0_dev, const int *y0_dev, int n_order, const float2 *tw_np,
                                        unsigned long long *dbg, hipStream_t s) {
    if (!fused_large_supported(st.np, st.r, st) || !st.T || !st.dP || st.meas_g != 16 || st.npart != 1)
        return hipErrorInvalidValue;
    LargeArgs a;
    a.st = st;
    a.meas = meas;
    a.tab = LedTab{nullptr, order_dev, x0_dev, y0_dev, st.np / 2};
    a.tw = tw_np;
    a.n_order = n_order;
    a.dbg = dbg;
    size_t lds = 0;
    a.tab_off = ledtab_offset(large_lds_bytes(st.nb, st.nty), n_order, st.L, 160 * 1024, lds);
    hipError_t e = hipFuncSetAttribute((const void *)k_fused_large, hipFuncAttributeMaxDynamicSharedMemorySize,
                                       (int)lds);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_fused_large, dim3(st.B), dim3(flg::NT), lds, s, a);
    return hipGetLastError();
}

}  // namespace fpm
