// np256.hip -- the general path's row and column passes for Np = 256 at pupil
// radii beyond the fused Np 256 kernels (r > 34: the dataset_mono geometry at
// cropSizeX 256 has naRadius 84, L 1024), one 256-point transform per 16-lane
// group held in registers (dft256_full, dftL.hpp: two register 16-point DFTs
// and one LDS exchange) instead of the mixed-radix Stockham passes over LDS
// tiles of general.hip's K1-K3.
//
// Same steps and scratch as general.hip (fpmMain.cpp:358-447,457-475):
//   R1 k_rows256_inv   a group per support-box row: the previous LED's pupil
//                      commit on the row (P += dP / max|objF|, folded in as in
//                      np1024.hip, with the row's max|P| partial), O*P on the
//                      disk, row IDFT, the T row stored as 128-byte segments
//   C  k_cols256       a block per 16 adjacent columns (a group each): box
//                      rows of T staged through an LDS strip, column IDFT,
//                      amplitude replacement against the stack in the fused
//                      column layout (meas_layout g = 16: lane t holds rows
//                      t + 16 m of its column, 32 contiguous bytes), column
//                      DFT, box rows back to T
//   R2 k_rows256_fwd   a block per 16-row tile row of the spectrum, a group
//                      per box row: T row in, row DFT, object update and pupil
//                      numerator on the row's disk pixels, then the tile
//                      maxima of the window's tiles in that tile row and the
//                      tile row's maximum (general.hip K4's values, bit for
//                      bit: 1.01 -> 1.18 M LED-updates/s at dataset_mono Np 256)
// Three launches per LED: K4 is inside R2, and K5 (the commit) runs only after
// an iteration's last LED (launch_pupil_commit).
//
// Natural layout everywhere: lane t of a group holds elements t + 16 j (j =
// 0..15) of its row / column, which is both dft256_full's input and output
// order, so no relabelling between the passes.
//
// Blocks are mapped so that every kernel's blocks of patch b land on XCD
// b mod 8 (round-robin dispatch; only a placement, correctness does not
// depend on it): a patch's T (nb x 256 x 8 B = 346 KB at r 84), window and
// pupil are written and read back on one XCD.
#include <hip/hip_runtime.h>

#include "cpk.hpp"
#include "dftL.hpp"
#include "fpm_state.hpp"

#include <algorithm>

namespace fpm {

namespace n256 {
constexpr int N = 256, H = N / 2;
constexpr int WPB = 4;            // waves per block
constexpr int NT = 64 * WPB;
constexpr int GPB = 4 * WPB;      // 16-lane groups per block: rows (R1, R2) or columns (C) per block
constexpr int SP = GPB + 1;       // strip row pitch (complex)
static_assert(NT == N, "one twiddle per thread");
}  // namespace n256

namespace {

__device__ __forceinline__ int fold256(int k) { return k < n256::H ? k : k - n256::N; }  // signed frequency

// max over each row of 16 lanes (one group) of values >= +0, in every lane of
// the row (the DPP steps of wave_max_nonneg without the cross-row fold)
__device__ __forceinline__ float row16_max_nonneg(float x) {
    unsigned v = __float_as_uint(x) & 0x7fffffffu;
    v = max(v, (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xF, 0xF, false));   // lane ^ 1
    v = max(v, (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xF, 0xF, false));   // lane ^ 2
    v = max(v, (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x141, 0xF, 0xF, false));  // row_half_mirror
    v = max(v, (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x140, 0xF, 0xF, false));  // row_mirror
    return __uint_as_float(v);
}

// block -> (patch b, sub-block) of a 1-D grid of nsub * xcd_patches(B)
// blocks, patch b on XCD b mod 8; false for the padding blocks of patches
// b >= B (B not a multiple of 8), which exit at once.  Against the plain
// b = block / nsub: 1.20-1.22 -> 1.22-1.24 M at dataset_mono Np 256, 64
// patches (profiles/r06_ab/np256_register_path_ab.txt)
__host__ __device__ __forceinline__ int xcd_patches(int B) { return (B + 7) & ~7; }
__device__ __forceinline__ bool xcd_block(int nsub, int B, int &b, int &sub) {
    const int id = blockIdx.x;
    const int k = id >> 3, q = k / nsub;
    b = (id & 7) + 8 * q;
    sub = k - q * nsub;
    return b < B;
}

// R1: grid (ceil(nb / GPB) * xcd_patches(B)), block NT, LDS (N + GPB XTILE_H) complex
__global__ void __launch_bounds__(n256::NT) k_rows256_inv(DevState st, StepArgs sa, const float2 *__restrict__ tw,
                                                          int commit) {
    using namespace n256;
    extern __shared__ __attribute__((aligned(16))) float2 sm[];
    __shared__ float red[WPB];
    const int g = threadIdx.x >> 4, t = threadIdx.x & 15, xrd = exch_rbase_half(t);
    const int r = st.r, nb = st.nb;
    int b, sub;
    if (!xcd_block((nb + GPB - 1) / GPB, st.B, b, sub)) return;  // block-uniform
    const int row = sub * GPB + g;
    // the twiddle, the previous LED's tile-row maxima and the first half
    // row's loads all issued before the first store or barrier (np1024.hip R1)
    const float2 twv = tw[threadIdx.x];
    float2 *twL = sm;
    float2 *wt = sm + N + g * XTILE_H;
    float rm[2];  // nty <= 2 NT (L <= 8192, checked by the launcher)
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        const int i = threadIdx.x + NT * k;
        rm[k] = st.rmax[(size_t)b * st.nty + (i < st.nty ? i : 0)];
    }
    const int rowc = row < nb ? row : nb - 1;  // groups past the box: in-bounds loads, discarded
    const int ky = rowc - r, w2 = r * r - ky * ky;
    float2 *pup = st.pupil + ((size_t)b * nb + rowc) * nb + r;  // indexed by kx
    const float2 *dP = st.dP + ((size_t)b * nb + rowc) * nb + r;
    const float2 *sp = st.spec + (size_t)b * st.L * st.L + (size_t)(sa.yc + ky) * st.L + sa.xc;  // + kx (:358-362)
    // half a row at a time, every load of a half before its arithmetic and
    // pupil stores (unconditional: a lane off the disk reads the row's centre
    // pixel and masks it)
    struct Half {
        float2 pv[8], dv[8], ov[8];
    };
    auto load_half = [&](int hh, Half &q) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int kx = fold256(t + 16 * (8 * hh + i));
            const int kc = kx * kx <= w2 ? kx : 0;
            q.pv[i] = pup[kc];
            q.dv[i] = dP[kc];  // unconditional (used only when commit)
            q.ov[i] = sp[kc];
        }
    };
    Half q;
    load_half(0, q);
    sm[threadIdx.x] = twv;
    if (!commit) __syncthreads();  // block-uniform; else block_max's barriers order the stores
    float omax = 1.f;
    if (commit) {  // block-uniform: max|objF| of the previous LED (:460,467)
        float m = 0.f;
#pragma unroll
        for (int k = 0; k < 2; ++k)
            if ((int)threadIdx.x + NT * k < st.nty) m = fmaxf(m, rm[k]);
        omax = block_max_nonneg(m, red);
    }
    if (row >= nb) return;  // group-uniform; no block barrier follows
    float2 x[16];
    float pmx = 0.f;
    auto body = [&](int j, float2 p, float2 d, float2 o) {
        const int kx = fold256(t + 16 * j);
        x[j] = make_float2(0.f, 0.f);
        if (kx * kx <= w2) {
            if (commit) {  // :470-475 (general.hip K5's arithmetic)
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
#pragma unroll
        for (int i = 0; i < 8; ++i) body(8 * hh + i, q.pv[i], q.dv[i], q.ov[i]);
    }
    pmx = row16_max_nonneg(pmx);
    if (t == 0) st.pmax[(size_t)b * st.npart + row] = pmx;  // this row's max|P| (:415)
    float2 y[16];
    dft256_full<true, true>(x, y, wt, LdsTw{twL, t, 1}, t, xrd);  // :365 (rows); y[k] = X[t + 16 k]
    float2 *T = st.T + ((size_t)b * nb + row) * N + t;
#pragma unroll
    for (int k = 0; k < 16; ++k) T[16 * k] = y[k];
}

// C: grid ((N / GPB) * xcd_patches(B)), block NT, LDS (N + max(nb SP, GPB XTILE_H)) complex
__global__ void __launch_bounds__(n256::NT) k_cols256(DevState st, StepArgs sa, const float2 *__restrict__ tw) {
    using namespace n256;
    extern __shared__ __attribute__((aligned(16))) float2 sm[];
    const int g = threadIdx.x >> 4, t = threadIdx.x & 15, xrd = exch_rbase_half(t);
    const int r = st.r, nb = st.nb;
    int b, sub;
    if (!xcd_block(N / GPB, st.B, b, sub)) return;  // block-uniform
    const int x0 = sub * GPB;
    const float2 twv = tw[threadIdx.x];
    float2 *twL = sm;
    float2 *strip = sm + N;              // nb x SP (box rows only); the group tiles
    float2 *wt = strip + g * XTILE_H;    // alias it while every column is in registers
    float2 *T = st.T + (size_t)b * nb * N + x0;
    // this group's measurement column, rows t + 16 m (meas_layout g = 16:
    // stored[x Np + 16 t + m] = I[t + 16 m][x]), two 16-byte loads per lane
    const uint4 *Ic = (const uint4 *)(st.meas + (((size_t)sa.led * st.mB + b) * N + x0 + g) * N + 16 * t);
    const uint4 ia = Ic[0], ib = Ic[1];
    // the box rows of the strip: 128-byte row segments, every load of a
    // thread issued before its LDS stores (clamped, masked)
    constexpr int KMAX = N * GPB / NT;  // nb <= N rows
    const int tot = nb * GPB;
    float2 tv[KMAX];
#pragma unroll
    for (int k = 0; k < KMAX; ++k) {
        const int idx = min((int)threadIdx.x + NT * k, tot - 1);
        if (NT * k < tot) tv[k] = T[(size_t)(idx / GPB) * N + (idx % GPB)];  // uniform guard
    }
    sm[threadIdx.x] = twv;
#pragma unroll
    for (int k = 0; k < KMAX; ++k) {
        const int idx = (int)threadIdx.x + NT * k;
        if (NT * k < tot && idx < tot) strip[(idx / GPB) * SP + (idx % GPB)] = tv[k];
    }
    __syncthreads();
    // FFT row i of a column is box row i + r (i <= r) or i - N + r (i >= N - r);
    // every other row is zero (:364)
    auto boxrow = [&](int i) { return i <= r ? i + r : (i >= N - r ? i - N + r : -1); };
    float2 v[16];
#pragma unroll
    for (int m = 0; m < 16; ++m) {
        const int j = boxrow(t + 16 * m);
        v[m] = j >= 0 ? strip[j * SP + g] : make_float2(0.f, 0.f);
    }
    __syncthreads();  // the strip is the groups' exchange space from here
    float2 y[16];
    dft256_full<true, true>(v, y, wt, LdsTw{twL, t, 1}, t, xrd);  // :365 (columns); y[m] = row t + 16 m
    // amplitude replacement (:378-394), np1024.hip's form: with y the unscaled
    // IDFT value, psi = y / N^2 and sqrt(I) psi / |psi + eps (1 + i)| =
    // y sqrt(I) / |y + eps N^2 (1 + i)|
    const float nn = (float)N * (float)N, epsn = st.eps * nn, epsn_im = st.eps_im * nn;
    const unsigned iw[8] = {ia.x, ia.y, ia.z, ia.w, ib.x, ib.y, ib.z, ib.w};
#pragma unroll
    for (int m = 0; m < 16; ++m) {
        const float iv = (float)((iw[m >> 1] >> (16 * (m & 1))) & 0xffffu);
        const float2 u = y[m];
        const float tr = u.x + epsn, ti = u.y + epsn_im;
        const float s = amp_scale(__builtin_fmaf(tr, tr, ti * ti), iv);
        y[m] = make_float2(u.x * s, u.y * s);
    }
    dft256_full<false, true>(y, v, wt, LdsTw{twL, t, 1}, t, xrd);  // :394 (columns)
    __syncthreads();  // every group is done with its tile before the strip is rewritten
#pragma unroll
    for (int m = 0; m < 16; ++m) {
        const int j = boxrow(t + 16 * m);
        if (j >= 0) strip[j * SP + g] = v[m];
    }
    __syncthreads();
    for (int idx = threadIdx.x; idx < tot; idx += NT) T[(size_t)(idx / GPB) * N + (idx % GPB)] = strip[(idx / GPB) * SP + (idx % GPB)];
}

// R2: grid (ntr * xcd_patches(B)), block NT, LDS as R1: one block per 16-row tile row of
// the spectrum (ntr = the most tile rows a window of nb rows spans), group g
// on spectrum row 16 ty + g.  After the update the block re-reads its tile
// row's window tiles and writes their maxima and the tile row's maximum --
// general.hip K4's values, bit for bit, without its launch.
constexpr int kMaxWinTiles = (2 * (n256::H - 1) + 15) / kTile + 1;  // tile columns a window spans, r < 128
__global__ void __launch_bounds__(n256::NT) __attribute__((amdgpu_waves_per_eu(4))) k_rows256_fwd(DevState st, StepArgs sa, const float2 *__restrict__ tw) {
    using namespace n256;
    extern __shared__ __attribute__((aligned(16))) float2 sm[];
    __shared__ float red[WPB];
    __shared__ float tred[WPB][kMaxWinTiles];
    const int g = threadIdx.x >> 4, t = threadIdx.x & 15, xrd = exch_rbase_half(t);
    const int r = st.r, nb = st.nb, L = st.L;
    const int ty0 = (sa.yc - r) / kTile, ty1 = (sa.yc + r) / kTile;
    int b, sub;
    if (!xcd_block((2 * r + 15) / kTile + 1, st.B, b, sub)) return;  // block-uniform
    const int ty = ty0 + sub;
    if (ty > ty1) return;  // block-uniform, before any barrier
    const int row = ty * kTile + g - (sa.yc - r);  // box row of this group's spectrum row
    const bool act = row >= 0 && row < nb;
    // the tile row's maxima outside the window: unchanged by this launch,
    // their loads issued first
    const int tx0 = (sa.xc - r) / kTile, tx1 = (sa.xc + r) / kTile, ntx = st.ntx;
    float *tmax = st.tmax + ((size_t)b * st.nty + ty) * ntx;
    float tm[2];
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        const int i = threadIdx.x + NT * k;
        tm[k] = tmax[i < ntx ? i : 0];
    }
    const float2 twv = tw[threadIdx.x];
    float2 *twL = sm;
    float2 *wt = sm + N + g * XTILE_H;
    // the row's T first (its latency runs under the max|P| reduction), then
    // max|P| of the previous commit from the npart <= NT partial maxima (:415)
    const int rowc = act ? row : (row < 0 ? 0 : nb - 1);
    const float2 *Tr = st.T + ((size_t)b * nb + rowc) * N + t;
    float2 x[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) x[j] = Tr[16 * j];
    const int i = threadIdx.x;
    const float pv = st.pmax[(size_t)b * st.npart + (i < st.npart ? i : 0)];
    sm[threadIdx.x] = twv;
    const float pm = block_max_nonneg(i < st.npart ? pv : 0.f, red);  // its barriers publish the twiddles
    float2 *sp0 = st.spec + (size_t)b * L * L;
    if (act) {  // group-uniform
        const int ky = row - r, w2 = r * r - ky * ky;
        float2 *pup = st.pupil + ((size_t)b * nb + row) * nb + r;
        float2 *dP = st.dP + ((size_t)b * nb + row) * nb + r;
        float2 *sp = sp0 + (size_t)(sa.yc + ky) * L + sa.xc;
        // half the row's loads ahead of their stores (the stores may alias the
        // loads, so the compiler keeps program order otherwise)
        float2 ov[8], pp[8];
        auto load_half = [&](int hp) {
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const int kx = fold256(t + 16 * (8 * hp + k));
                const int kc = kx * kx <= w2 ? kx : 0;
                pp[k] = pup[kc];
                ov[k] = sp[kc];
            }
        };
        float2 F[16];
        dft256_full<false, true>(x, F, wt, LdsTw{twL, t, 1}, t, xrd);  // :394 (rows); F[k] = X[t + 16 k]
#pragma unroll
        for (int hp = 0; hp < 2; ++hp) {
            load_half(hp);  // (the first half issued before the transform: no change, r06_ab)
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const int kx = fold256(t + 16 * (8 * hp + k));
                if (kx * kx > w2) continue;
                const float2 o = ov[k];                                 // pre-update Objfcrop (:361)
                const float2 p = pp[k];
                const float2 D = csub(F[8 * hp + k], cmul(o, p));       // Objfup - ObjfcropP (:409,463)
                const float pa = cmag(p);                               // object update (:406-419,433)
                const float2 dpc = cmul(cmul(D, cscale(cconj(p), pa)), upd_coef_div(pa * pa + st.delta2, st.d2_im, pm));
                sp[kx] = cadd(o, dpc);
                const float oa = cmag(o);                               // pupil numerator (:459-464,469)
                dP[kx] = cmul(cmul(D, cscale(cconj(o), oa)), upd_coef_div(oa * oa + st.delta1, st.d1_im, 1.0f));
            }
        }
    }
    // max|objF| bookkeeping (:460,467): the window's tiles of this tile row
    // re-read after the block's stores (workgroup scope: one L1 per block),
    // group g reading row g of every tile, every load issued before the first
    // reduction (clamped in-bounds, masked)
    __syncthreads();
    const int yy = ty * kTile + g;
    float m[kMaxWinTiles];
#pragma unroll
    for (int k = 0; k < kMaxWinTiles; ++k) {
        const int xx = (tx0 + k) * kTile + t;
        const bool ok = tx0 + k <= tx1 && yy < L && xx < L;
        const float2 v = sp0[ok ? (size_t)yy * L + xx : 0];
        m[k] = ok ? cmag(v) : 0.f;
    }
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
    for (int k = 0; k < kMaxWinTiles; ++k) {
        if (tx0 + k <= tx1) {  // block-uniform
            const float v = wave_max_nonneg(m[k]);
            if (lane == 0) tred[w][k] = v;
        }
    }
    __syncthreads();
    float mx = 0.f;
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        const int ix = threadIdx.x + NT * k;
        if (ix >= ntx) continue;
        float v = tm[k];
        if (ix >= tx0 && ix <= tx1) {
            v = tred[0][ix - tx0];
#pragma unroll
            for (int ww = 1; ww < WPB; ++ww) v = fmaxf(v, tred[ww][ix - tx0]);
            tmax[ix] = v;
        }
        mx = fmaxf(mx, v);
    }
    mx = block_max_nonneg(mx, red);
    if (threadIdx.x == 0) st.rmax[(size_t)b * st.nty + ty] = mx;
}

}  // namespace

// Register path for this context?  Np 256, fp32 spectrum, r < 128 (every box
// row's frequencies inside one 256-point period), the stack in the fused
// column layout g = 16 (the caller permutes it when this returns true).
bool np256_supported(int np, int r, int L, bool fp16) {
    return np == n256::N && r >= 1 && r < n256::H && !fp16 && L <= 2 * n256::NT * kTile;
}

hipError_t launch_np256_rows_cols(const DevState &st, const StepArgs &sa, const float2 *tw, bool commit,
                                  hipStream_t s) {
    using namespace n256;
    if (!np256_supported(st.np, st.r, st.L, st.spec16 != nullptr) || st.meas_g != 16 || st.npart < st.nb ||
        st.npart > NT || !st.T || !st.spec)
        return hipErrorInvalidValue;
    const size_t lds_r = (size_t)(N + GPB * XTILE_H) * sizeof(float2);
    const size_t lds_c = (size_t)(N + std::max(st.nb * SP, GPB * XTILE_H)) * sizeof(float2);
    const int nsr = (st.nb + GPB - 1) / GPB, Bp = xcd_patches(st.B);
    hipLaunchKernelGGL(k_rows256_inv, dim3(nsr * Bp), dim3(NT), lds_r, s, st, sa, tw, commit ? 1 : 0);
    hipLaunchKernelGGL(k_cols256, dim3((N / GPB) * Bp), dim3(NT), lds_c, s, st, sa, tw);
    const int ntr = (2 * st.r + 15) / kTile + 1;  // tile rows a window can span
    hipLaunchKernelGGL(k_rows256_fwd, dim3(ntr * Bp), dim3(NT), lds_r, s, st, sa, tw);
    return hipGetLastError();
}

}  // namespace fpm
