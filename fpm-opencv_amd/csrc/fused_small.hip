// fused_small.hip -- the fused per-patch FPM iteration for small patches
// (Np <= 96, any Np = 2^a 3^b 5^c; BASELINE configs 1 and 2: dataset_mono,
// Np 90, L 360, naRadius 30).  ONE launch per runFPM iteration, one 1024-thread
// workgroup per patch walking every LED of the order (fpmMain.cpp:348-476).
//
// On the general path such a patch costs five launches per LED whose work is
// a few microseconds of latency each (47 us per LED at config 2); here the
// whole sub-aperture field lives in LDS and each LED step is a chain of
// mixed-radix Stockham passes (fft_lds.hpp) over two Np x Np buffers:
//
//   gather   O*P on the support into the box rows (FFT column index kx mod Np)
//   rows     IDFT of the nb box rows                             (:364-365)
//   T        -> column-major Np x Np, rows outside the box zero
//   columns  IDFT, amplitude replacement, DFT                    (:365-394)
//   T        -> box rows
//   rows     DFT of the box rows                                 (:394)
//   update   object update on the support + pupil numerator (slot_update),
//            incremental tile maxima, exact max|objF|, P += num/max, max|P|
//            (:405-475; the same scheme as fpm_fused.hip)
//
// Each thread owns up to 4 pixels of the support box (pixel p = tid + 256 i)
// and keeps their P, pre-update O and numerator in registers.  The
// measurement is read in the transposed layout [x][y] (meas_layout, g = Np),
// so the amplitude step reads it in the column-major order of the buffer.
#include <hip/hip_runtime.h>

#include "cpk.hpp"
#include "fft_lds.hpp"
#include "fpm_state.hpp"
#include "update.hpp"

namespace fpm {

#ifndef FPM_SMALL_STAMPS
#define FPM_SMALL_STAMPS 0  // 1: phase stamps (FPM_STAMPS=1); compiled out by default (register pressure)
#endif

namespace fs {
constexpr int NT = 1024;
constexpr int SP = 4;        // support-box pixels per thread: nb^2 <= NT * SP (r <= 31)
constexpr int NPMAX = 96;    // two Np x Np complex buffers in 160 KB of LDS
constexpr int KM = (90 * 90 / 2 + NT - 1) / NT;  // Np 90: measurement dwords per thread
}  // namespace fs

struct SmallArgs {
    DevState st;
    const uint16_t *meas;   // [nS][B][x][y] = I[y][x] (meas_layout with g = Np)
    const int *order, *x0, *y0;
    const float2 *tw;       // exp(-2 pi i k / Np), k < Np
    FftPlan pl;             // mixed-radix plan of Np (the generic instance)
    int n_order;
    int btx0, bty0, nbx, nbt;  // live-band tiles (fpm_fused.hip FusedArgs)
    float rnbx;
    unsigned long long *dbg;   // FPM_STAMPS=1 phase cycles, else null
};

// NPC = 90: Np and the plan fixed at compile time, two composite-radix passes
// 10 x 9 per transform (BASELINE configs 1/2; the runtime plan 2*3*3*5 takes
// four passes and, with a radix switch at each of the four call sites, more
// registers: 1.89 M -> 3.19 M LED-updates/s at config 2); NPC = 0: any
// Np <= 96 with the runtime plan
template <int NPC>
__global__ void __launch_bounds__(fs::NT, 1) k_fused_small(SmallArgs a) {
    using namespace fs;
    extern __shared__ __attribute__((aligned(16))) float2 sm[];
    const DevState &st = a.st;
    const int Np = NPC ? NPC : st.np, L = st.L, R = st.r, NB = st.nb, NN = Np * Np;

    float2 *A = sm, *Bf = sm + NN, *twl = Bf + NN;
    float *tmx = (float *)(twl + Np);                  // band-tile maxima
#define FPM_SMALL_FFT(INV, x, y, C)                                                        \
    (NPC == 90 ? stockham_t<INV, 90, 1, 10, 9>((x), (y), (C), twl, tid, NT) \
               : stockham<INV>((x), (y), (C), a.pl, twl, tid, NT))
    unsigned *dirty = (unsigned *)(tmx + a.nbt);       // band-tile dirty bits
    float *red = (float *)(dirty + ((a.nbt + 31) >> 5));  // 3 x 16: per-wave maxima
    uint16_t *ims = (uint16_t *)(red + 48);               // Np 90: staged measurement image
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, b = blockIdx.x;
    constexpr int NW = NT / 64;
    const int nwords = (a.nbt + 31) >> 5;

    for (int i = tid; i < Np; i += NT) twl[i] = a.tw[i];
    auto band_dy = [&](int k) { return (int)(((float)k + 0.5f) * a.rnbx); };
    auto band_gtile = [&](int k) {
        const int dy = band_dy(k);
        return (a.bty0 + dy) * st.ntx + a.btx0 + (k - dy * a.nbx);
    };
    float *tmax_g = st.tmax + (size_t)b * st.ntx * st.nty;
    unsigned *dirty_g = st.tdirty + (size_t)b * ((st.ntx * st.nty + 31) / 32);
    for (int k = tid; k < a.nbt; k += NT) tmx[k] = tmax_g[band_gtile(k)];
    for (int i = tid; i < nwords; i += NT) dirty[i] = dirty_g[i];

    float2 *spec = st.spec + (size_t)b * L * L;
    float2 *pup = st.pupil + (size_t)b * NB * NB;
    // this thread's support-box pixels: (ky, kx) of box pixel p = tid + NT i
    float2 P[SP], Op[SP], NUM[SP];
    unsigned inm = 0;  // bit i: pixel i lies on the support disk
#pragma unroll
    for (int i = 0; i < SP; ++i) {
        const int p = tid + NT * i;
        const int ky = p / NB - R, kx = p % NB - R;
        const bool in = p < NB * NB && ky * ky + kx * kx <= R * R;
        inm |= (in ? 1u : 0u) << i;
        P[i] = in ? pup[p] : make_float2(0.f, 0.f);
        NUM[i] = make_float2(0.f, 0.f);
    }
    auto pix = [&](int i, int &ky, int &kx) {
        const int p = tid + NT * i;
        ky = p / NB - R;
        kx = p % NB - R;
    };
    float pm = st.pmax[b];
    const float epsn = st.eps * (float)NN, epsn_im = st.eps_im * (float)NN;  // eps on the unscaled IDFT
    auto window = [&](int itn) {
        const int ln = a.order[itn];
        return spec + (unsigned)((a.y0[ln] + Np / 2) * L + a.x0[ln] + Np / 2);
    };
    auto loadO = [&](const float2 *sr) {
#pragma unroll
        for (int i = 0; i < SP; ++i) {
            int ky, kx;
            pix(i, ky, kx);
            Op[i] = ((inm >> i) & 1) ? sr[ky * L + kx] : make_float2(0.f, 0.f);
        }
    };
    if (a.n_order > 0) loadO(window(0));
    __syncthreads();

    unsigned *tmu = (unsigned *)tmx;
    auto note = [&](int py, int px, float ao, float an) {  // fpm_fused.hip: exact incremental tile maxima
        const int ti = ((py >> 4) - a.bty0) * a.nbx + ((px >> 4) - a.btx0);
        const unsigned cur = tmu[ti];
        if (an < ao && cur <= __float_as_uint(ao)) atomicOr(&dirty[ti >> 5], 1u << (ti & 31));
        if (__float_as_uint(an) > cur) atomicMax(&tmu[ti], __float_as_uint(an));
    };
    auto fidx = [&](int k) { return k < 0 ? k + Np : k; };  // FFT index of frequency k, |k| < Np

    unsigned long long acc[kStamps] = {};
    unsigned long long prev = (FPM_SMALL_STAMPS && a.dbg) ? __builtin_amdgcn_s_memtime() : 0ull;
#define FPM_STAMP(i)                                                  \
    if (FPM_SMALL_STAMPS && a.dbg) {                                  \
        const unsigned long long now_ = __builtin_amdgcn_s_memtime(); \
        acc[i] += now_ - prev;                                        \
        prev = now_;                                                  \
    }
    // Np 90: each LED's image is staged in LDS (ims) -- loaded into mreg one
    // LED ahead (with the next window's O), stored with the gather -- so the
    // amplitude step does not wait on HBM latency (7.1k -> 2.2k cycles per LED)
    uint32_t mreg[KM];
    auto load_meas = [&](int itn) {
        const uint32_t *I32 = (const uint32_t *)(a.meas + ((size_t)a.order[itn] * st.B + b) * NN);  // NN even
#pragma unroll
        for (int k = 0; k < KM; ++k) {
            const int i = tid + NT * k;
            mreg[k] = i < NN / 2 ? I32[i] : 0u;
        }
    };
    if (NPC == 90 && a.n_order > 0) load_meas(0);
    for (int it = 0; it < a.n_order; ++it) {
        const int led = a.order[it];
        const int xc = a.x0[led] + Np / 2, yc = a.y0[led] + Np / 2;
        float2 *srow = spec + (unsigned)(yc * L + xc);  // spec[yc + ky][xc + kx] = srow[ky*L + kx]
        const uint16_t *Ib = a.meas + ((size_t)led * st.B + b) * NN;

        const float2 *F;
        if constexpr (NPC == 90) {
            // Gather and both transposes folded into the transforms' first
            // passes (stockham_t_ld): the owners write the support box densely
            // (O*P on the disk, 0 elsewhere) into Bf, the row IDFT's first pass
            // reads it as box rows, the column passes read the other
            // orientation in place -- no zero fill and no transpose passes.
#pragma unroll
            for (int i = 0; i < SP; ++i) {
                const int p = tid + NT * i;
                if (p < NB * NB)
                    Bf[p] = ((inm >> i) & 1) ? pout(pmul(pin(Op[i]), pin(P[i]))) : make_float2(0.f, 0.f);  // :358-364
            }
            {  // read after the row/column IDFT barriers
                uint32_t *ims32 = (uint32_t *)ims;
#pragma unroll
                for (int k = 0; k < KM; ++k) {
                    const int i = tid + NT * k;
                    if (i < NN / 2) ims32[i] = mreg[k];
                }
            }
            __syncthreads();
            FPM_STAMP(0)
            // row IDFTs (:365): element i of box row s is frequency kx = i (i <= R) or i - Np
            const float2 *box = Bf;
            float2 *res = stockham_t_ld<true, 90, 10, 9>(
                [&](int s, int i) {
                    const int kx = i <= R ? i : i - Np;
                    return (kx >= -R && kx <= R) ? box[s * NB + kx + R] : make_float2(0.f, 0.f);
                },
                A, Bf, NB, twl, tid, NT);  // -> Bf
            FPM_STAMP(7)
            // column IDFTs: element y of column x is box row ky = y (y <= R) or y - Np of res
            float2 *col = stockham_t_ld<true, 90, 10, 9>(
                [&](int x, int y) {
                    const int ky = y <= R ? y : y - Np;
                    return (ky >= -R && ky <= R) ? res[(ky + R) * Np + x] : make_float2(0.f, 0.f);
                },
                A, Bf, Np, twl, tid, NT);  // -> Bf
            FPM_STAMP(10)
            // ---- amplitude replacement (:365-394), see the generic branch
            for (int e = tid; e < NN; e += NT) {
                const float Iv = (float)ims[e];
                const pf2 r = pin(col[e]);
                const pf2 tt = r + (pf2){epsn, epsn_im};
                const float mag2 = __builtin_fmaf(tt.x, tt.x, tt.y * tt.y);
                col[e] = pout(r * amp_scale(mag2, Iv));
            }
            __syncthreads();
            FPM_STAMP(2)
            float2 *colF = stockham_t<false, 90, 1, 10, 9>(col, A, Np, twl, tid, NT);  // -> Bf
            FPM_STAMP(8)
            // row DFTs (:394): element x of box row s is column x's FFT row fidx(s - R)
            F = stockham_t_ld<false, 90, 10, 9>(
                [&](int s, int x) { return colF[x * Np + fidx(s - R)]; }, A, Bf, NB, twl, tid, NT);  // -> Bf
            FPM_STAMP(9)
        } else {
        // ---- gather O*P into the box rows (:358-364)
        for (int e = tid; e < NB * Np; e += NT) A[e] = make_float2(0.f, 0.f);
        __syncthreads();
#pragma unroll
        for (int i = 0; i < SP; ++i)
            if ((inm >> i) & 1) {
                int ky, kx;
                pix(i, ky, kx);
                A[(ky + R) * Np + fidx(kx)] = pout(pmul(pin(Op[i]), pin(P[i])));
            }
        __syncthreads();
        FPM_STAMP(0)
        // ---- row IDFTs of the box rows, then column-major with zero rows (:365)
        float2 *res = FPM_SMALL_FFT(true, A, Bf, NB);
        FPM_STAMP(7)
        float2 *col = res == A ? Bf : A;
        for (int e = tid; e < NN; e += NT) {
            const int x = e / Np, y = e - x * Np;
            const int ky = y <= R ? y : y - Np;
            col[e] = (ky >= -R && ky <= R) ? res[(ky + R) * Np + x] : make_float2(0.f, 0.f);
        }
        __syncthreads();
        FPM_STAMP(1)
        col = FPM_SMALL_FFT(true, col, res, Np);
        FPM_STAMP(10)
        // ---- amplitude replacement (:365-394): psi = r/Np^2,
        // sqrt(I) psi/|psi + eps| = r / sqrt(|r + eps Np^2|^2 / I), eps on both channels (:390)
        for (int e = tid; e < NN; e += NT) {
            const float Iv = (float)Ib[e];
            const pf2 r = pin(col[e]);
            const pf2 tt = r + (pf2){epsn, epsn_im};
            const float mag2 = __builtin_fmaf(tt.x, tt.x, tt.y * tt.y);
            col[e] = pout(r * amp_scale(mag2, Iv));
        }
        __syncthreads();
        FPM_STAMP(2)
        float2 *colF = FPM_SMALL_FFT(false, col, col == A ? Bf : A, Np);
        FPM_STAMP(8)
        // ---- back to the box rows, row DFTs (:394)
        float2 *rw = colF == A ? Bf : A;
        for (int e = tid; e < NB * Np; e += NT) {
            const int row = e / Np, x = e - row * Np;
            rw[e] = colF[x * Np + fidx(row - R)];
        }
        __syncthreads();
        FPM_STAMP(3)
        F = FPM_SMALL_FFT(false, rw, colF, NB);
        FPM_STAMP(9)
        }

        // ---- object update on the support (:405-447), pupil numerator (:457-464)
#pragma unroll
        for (int i = 0; i < SP; ++i)
            if ((inm >> i) & 1) {
                int ky, kx;
                pix(i, ky, kx);
                float oa;
                const float2 nv =
                    slot_update(F[(ky + R) * Np + fidx(kx)], Op[i], P[i], pm, st, NUM[i], oa);
                srow[ky * L + kx] = nv;
                note(yc + ky, xc + kx, oa, cmag(nv));
            }
        __syncthreads();  // spectrum writes, tile maxima, dirty bits
        if (it + 1 < a.n_order) {
            loadO(window(it + 1));
            if (NPC == 90) load_meas(it + 1);
        }
        FPM_STAMP(4)

        // ---- exact max|objF| (:460,467) from the band-tile maxima
        float cm = 0.f, dm = 0.f;
        for (int k = tid; k < a.nbt; k += NT) {
            const bool d = (dirty[k >> 5] >> (k & 31)) & 1u;
            if (d) dm = fmaxf(dm, tmx[k]);
            else cm = fmaxf(cm, tmx[k]);
        }
        cm = wave_max_nonneg(cm);
        dm = wave_max_nonneg(dm);
        if (lane == 0) {
            red[w] = cm;
            red[16 + w] = dm;
        }
        __syncthreads();
        cm = red[0];
        dm = red[16];
#pragma unroll
        for (int i = 1; i < NW; ++i) {
            cm = fmaxf(cm, red[i]);
            dm = fmaxf(dm, red[16 + i]);
        }
        float omax = cm;
        if (dm > cm) {  // block-uniform
            for (int k = w; k < a.nbt; k += NW) {
                if (!((dirty[k >> 5] >> (k & 31)) & 1u) || !(tmx[k] > cm)) continue;  // wave-uniform
                const int ty = a.bty0 + band_dy(k), tx = a.btx0 + k - band_dy(k) * a.nbx;
                float mm = 0.f;
                // the tile's four loads issued together (clamped in bounds, masked
                // after): a conditional load waited for each in turn
                float2 e[4];
                bool ok[4];
#pragma unroll
                for (int jj = 0; jj < 4; ++jj) {
                    const int pp = lane + 64 * jj;
                    const int yy = ty * 16 + (pp >> 4), xx = tx * 16 + (pp & 15);
                    ok[jj] = yy < L && xx < L;
                    e[jj] = spec[ok[jj] ? (unsigned)(yy * L + xx) : 0u];
                }
#pragma unroll
                for (int jj = 0; jj < 4; ++jj)
                    if (ok[jj]) mm = fmaxf(mm, cmag(e[jj]));
                mm = wave_max_nonneg(mm);
                if (lane == 0) {
                    tmx[k] = mm;
                    atomicAnd(&dirty[k >> 5], ~(1u << (k & 31)));
                }
            }
            __syncthreads();
            float m2 = 0.f;
            for (int k = tid; k < a.nbt; k += NT)
                if (!((dirty[k >> 5] >> (k & 31)) & 1u)) m2 = fmaxf(m2, tmx[k]);
            m2 = wave_max_nonneg(m2);
            __syncthreads();
            if (lane == 0) red[w] = m2;
            __syncthreads();
            omax = red[0];
#pragma unroll
            for (int i = 1; i < NW; ++i) omax = fmaxf(omax, red[i]);
        }
        FPM_STAMP(5)
        const float rom = 1.0f / omax;
        // ---- P += num / max|objF| on the support (:468-475); max|P| (:415)
        float pmx = 0.f;
#pragma unroll
        for (int i = 0; i < SP; ++i) {
            P[i] = make_float2(P[i].x + NUM[i].x * rom, P[i].y + NUM[i].y * rom);
            pmx = fmaxf(pmx, cabs2(P[i]));
        }
        pmx = wave_max_nonneg(pmx);
        if (lane == 0) red[32 + w] = pmx;
        __syncthreads();
        float pm2 = red[32];
#pragma unroll
        for (int i = 1; i < NW; ++i) pm2 = fmaxf(pm2, red[32 + i]);
        pm = sqrtf(pm2);
        FPM_STAMP(6)
    }
#undef FPM_STAMP
#undef FPM_SMALL_FFT
    if (FPM_SMALL_STAMPS && a.dbg && (tid == 0 || tid == NT - 64))
        for (int i = 0; i < kStamps; ++i) atomicAdd(&a.dbg[(tid ? kStamps : 0) + i], acc[i]);

#pragma unroll
    for (int i = 0; i < SP; ++i)
        if ((inm >> i) & 1) pup[tid + NT * i] = P[i];
    for (int k = tid; k < a.nbt; k += NT) tmax_g[band_gtile(k)] = tmx[k];
    for (int i = tid; i < nwords; i += NT) dirty_g[i] = dirty[i];
    if (tid == 0) st.pmax[b] = pm;
}

// ------------------------------------------------------------------ host side
namespace {
struct SmallBand {
    int bty0, btx0, nbx, nbt;
};
SmallBand small_band(const DevState &st) {
    SmallBand b;
    b.bty0 = st.sy0 / kTile;
    b.btx0 = st.sx0 / kTile;
    b.nbx = st.sx1 / kTile - b.btx0 + 1;
    b.nbt = b.nbx * (st.sy1 / kTile - b.bty0 + 1);
    return b;
}
size_t small_lds_bytes(int np, int nbt) {
    return (size_t)(2 * np * np + np) * sizeof(float2) + (size_t)nbt * sizeof(float) +
           (size_t)(nbt + 31) / 32 * sizeof(unsigned) + 48 * sizeof(float) +
           (np == 90 ? (size_t)np * np * sizeof(uint16_t) : 0);  // the Np 90 instance's staged image
}
}  // namespace

// Small-patch fused kernel available for this geometry?
bool fused_small_supported(int np, int r, const DevState &st) {
    if (np < 8 || np > fs::NPMAX || r < 1 || 2 * r + 1 > np) return false;
    if ((2 * r + 1) * (2 * r + 1) > fs::NT * fs::SP) return false;
    if (st.sy0 < 0 || st.sy1 >= st.L || st.sy0 > st.sy1 || st.sx0 < 0 || st.sx1 >= st.L || st.sx0 > st.sx1)
        return false;
    return small_lds_bytes(np, small_band(st).nbt) <= 160 * 1024;
}

hipError_t launch_fused_small_iteration(const DevState &st, const uint16_t *meas, const int *order_dev,
                                        const int *x0_dev, const int *y0_dev, int n_order, const float2 *tw_np,
                                        const FftPlan &pl, unsigned long long *dbg, hipStream_t s) {
    if (!fused_small_supported(st.np, st.r, st)) return hipErrorInvalidValue;
    SmallArgs a;
    a.st = st;
    a.meas = meas;
    a.order = order_dev;
    a.x0 = x0_dev;
    a.y0 = y0_dev;
    a.tw = tw_np;
    a.pl = pl;
    a.dbg = dbg;
    a.n_order = n_order;
    const SmallBand bd = small_band(st);
    a.bty0 = bd.bty0;
    a.btx0 = bd.btx0;
    a.nbx = bd.nbx;
    a.nbt = bd.nbt;
    a.rnbx = 1.0f / (float)a.nbx;
    const size_t lds = small_lds_bytes(st.np, a.nbt);
    // Np 90 (configs 1/2): the instance with the transform fixed at compile time
    const bool c90 = st.np == 90;
    const void *fn = c90 ? (const void *)k_fused_small<90> : (const void *)k_fused_small<0>;
    hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
    if (c90)
        hipLaunchKernelGGL(k_fused_small<90>, dim3(st.B), dim3(fs::NT), lds, s, a);
    else
        hipLaunchKernelGGL(k_fused_small<0>, dim3(st.B), dim3(fs::NT), lds, s, a);
    return hipGetLastError();
}

}  // namespace fpm
