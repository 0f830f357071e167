// fused_s90.hip -- the fused per-patch FPM iteration for Np = 90 (BASELINE
// configs 1 and 2, dataset_mono.json: Np 90, L 360, naRadius 30): ONE launch
// per runFPM iteration, one 1024-thread workgroup per patch walking every LED
// of the order (fpmMain.cpp:348-476), the whole per-LED intermediate in LDS.
//
// The generic small-patch kernel (fused_small.hip) runs each transform as
// block-wide Stockham passes, each pass a barrier and an LDS round trip with
// one butterfly per thread (~2.6k cycles per pass at config 2).  Here every
// 90-point transform runs in the registers of one 10-lane group (dft90.hpp:
// 9 x 10 four-step, one group-local exchange), as the Np 200 kernel does
// (fused_mr.hip):
//
//   96 groups (6 per wave, lanes 60..63 idle) >= 90 columns >= box rows, so
//   every phase is one round: group g owns box row g (rows) and column g
//   (columns).
//   A  row IDFT of box row g of O*P (:358-365), layout A -> B, into T (LDS)
//   B  column g: box rows of T in layout A, IDFT -> layout B, amplitude
//      replacement against the stack column (meas_layout g = 9: lane j reads
//      I[j + 9 k][x], k < 10, one 20-byte run), DFT back to layout A, box
//      rows into T (:365-394)
//   C  row DFT of box row g (layout B -> A): F on the lane's own pixels (:394)
//   update / exact max|objF| / pupil update as fused_mr.hip (:405-475)
//
// Each lane keeps P and the pre-update O of its nine layout-A pixels of its
// box row in registers (kx = fold(l + 10 k)).
#include <hip/hip_runtime.h>

#include <cstdlib>

#include "cpk.hpp"
#include "dft90.hpp"
#include "fft_lds.hpp"
#include "fpm_state.hpp"
#include "fused_sync.hpp"
#include "ledtab.hpp"
#include "tilemax.hpp"
#include "update.hpp"

namespace fpm {

namespace f90 {
constexpr int NP = 90;
constexpr int N2 = 10;                 // lanes per group
constexpr int GPW = 6;                 // groups per wave (lanes 60..63 idle)
constexpr int NT = 1024;               // 16 waves: 4 per SIMD (128-VGPR budget)
constexpr int NW = NT / 64;
constexpr int NG = NW * GPW;           // 96 groups >= 90 columns
static_assert(NG >= NP, "one group per column");
constexpr int XT = 10 * kXP90;         // exchange tile per group (complex)
constexpr int TLD = NP + 1;            // T row pitch (complex), dense layout
// LDS bank layout (tools/lds_s90.py models every LDS instruction of an LED
// step with the gfx950 lane-group table).  Dense layout: tiles at a uniform
// stride of 100 and T rows of pitch 91 put 45 % of the modelled LDS-array
// cycles into bank conflicts (SQ counted 28 % at config 2): the 8-byte tile
// row writes of the two groups sharing a 16-lane batch overlap, and so do
// the column reads of T.  Conflict-light layout (when LDS allows, r <= 30):
// the six tiles of a wave at offsets with residues 0, 26, 6, 4, 30, 26
// (mod 32 complex), found by a search over the tile writes and the 16-byte
// row reads, in a 704-complex wave slot (704 = 0 mod 32, so every wave sees
// the same banks), and T rows of pitch 106 (= 10 mod 32).
constexpr int XW_DENSE = GPW * XT;     // wave slot of the dense layout
constexpr int XW_FAST = 704;
constexpr int XG_FAST[GPW] = {0, 122, 230, 356, 478, 602};
constexpr int TLD_FAST = 106;
constexpr int RMAX = 44;               // 2 r + 1 <= Np
static_assert((2 * RMAX + 1 + GPW - 1) / GPW < NW, "a wave with no box row (tilemax.hpp)");
}  // namespace f90

struct FusedS90Args {
    DevState st;
    const uint16_t *meas;    // [nS][B][x][j][k] = I[j + 9 k][x] (meas_layout g = 9)
    const int *order, *x0, *y0;
    const float2 *tw;        // exp(-2 pi i k / 90), k < 90
    int n_order;
    int btx0, bty0, nbx, nbt;  // live-band tiles (fpm_fused.hip FusedArgs)
    float rnbx;
    int xw;                    // exchange tiles: wave slot (complex)
    int xg[f90::GPW];          // tile offset of group gw in the wave slot
    int tld;                   // T row pitch (complex)
    int ledtab_off;            // LED table in dynamic LDS (ledtab.hpp), or -1
    unsigned long long *dbg;   // FPM_STAMPS=1 phase cycles (fused_mr.hip's slots), else null
};

// signed frequency of FFT index n (|k| <= r <= 44 lies on the right side of the fold)
__device__ __forceinline__ int f90_fold(int n) { return n < f90::NP / 2 ? n : n - f90::NP; }

__global__ void __launch_bounds__(f90::NT, 1) k_fused_s90(FusedS90Args a) {
    using namespace f90;
    ClockProbe probe;
    probe.start();
    extern __shared__ __attribute__((aligned(16))) float2 sm[];
    const DevState &st = a.st;
    const int R = st.r, NB = st.nb, L = st.L;
    float2 *tiles = sm;                        // NG * xt exchange tiles
    const int TLD = a.tld;
    float2 *th = tiles + NW * a.xw;            // (NB + 2) * TLD: T rows, zero row, dummy row
    float2 *tw = th + (NB + 2) * TLD;          // [a][b] = W90^{a b}, a, b < 10
    float *red = (float *)(tw + 100);          // 52: maxima per wave; [48..49] outside-window tile maxima
    unsigned *omx = (unsigned *)(red + 48);
    int *rowoff = (int *)(red + 52);           // 90: T offset of FFT row y (the zero row outside the box)
    float *tmx = (float *)(rowoff + NP);       // nbt band-tile maxima
    unsigned *dirty = (unsigned *)(tmx + a.nbt);

    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int gw = lane / N2;                  // group within the wave (6 = idle lanes)
    const bool act = gw < GPW;
    const int l = act ? lane - N2 * gw : 0;    // lane within the group
    const int g = w * GPW + (act ? gw : 0);    // group in the workgroup
    const int b = blockIdx.x;
    int xgo = a.xg[0];  // group offset (uniform kernel-argument values, selected per lane)
#pragma unroll
    for (int i = 1; i < GPW; ++i) xgo = gw == i ? a.xg[i] : xgo;
    float2 *tile = tiles + w * a.xw + xgo;
    const int xrd = opaque_i(l * kXP90);
    const int nwords = (a.nbt + 31) >> 5;

    for (int i = tid; i < 100; i += NT) tw[i] = a.tw[((i / 10) * (i % 10)) % NP];
    for (int i = tid; i < NP; i += NT) {
        const int ky = f90_fold(i);
        rowoff[i] = (ky >= -R && ky <= R) ? (ky + R) * TLD : NB * TLD;
    }
    auto band_dy = [&](int k) { return (int)(((float)k + 0.5f) * a.rnbx); };
    auto band_gtile = [&](int k) {
        const int dy = band_dy(k);
        return (a.bty0 + dy) * st.ntx + a.btx0 + (k - dy * a.nbx);
    };
    float *tmax_g = st.tmax + (size_t)b * st.ntx * st.nty;
    unsigned *dirty_g = st.tdirty + (size_t)b * ((st.ntx * st.nty + 31) / 32);
    for (int k = tid; k < a.nbt; k += NT) tmx[k] = tmax_g[band_gtile(k)];
    for (int i = tid; i < nwords; i += NT) dirty[i] = dirty_g[i];
    const int zoff = NB * TLD;
    for (int i = tid; i < 2 * TLD; i += NT) th[zoff + i] = make_float2(0.f, 0.f);

    float2 *spec = st.spec + (size_t)b * L * L;
    float2 *pup = st.pupil + (size_t)b * NB * NB;
    // box row of this group, its nine layout-A pixels kx = fold(l + 10 k)
    const bool ron = act && g < NB;
    const int wi0 = (NB + GPW - 1) / GPW;  // first wave with no box row (< NW: r <= RMAX)
    const int kyr = g - R;
    unsigned inmask = 0;
    float2 P[9];
#pragma unroll
    for (int k = 0; k < 9; ++k) {
        const int kx = f90_fold(l + 10 * k);
        const bool in = ron && (kyr * kyr + kx * kx <= R * R);
        inmask |= (in ? 1u : 0u) << k;
        P[k] = in ? pup[(kyr + R) * NB + kx + R] : make_float2(0.f, 0.f);
    }
    // the launch's LED order as an LDS table (ledtab.hpp)
    int2 *ltl = a.ledtab_off >= 0 ? (int2 *)((char *)sm + a.ledtab_off) : nullptr;
    const LedTab lt{ltl, a.order, a.x0, a.y0, NP / 2};
    if (ltl) lt.fill(ltl, a.n_order, tid, NT);
    if (tid == 0) omx[0] = omx[1] = 0u;
    __syncthreads();  // rowoff, tw
    // column pass: T row offset of this lane's layout-A FFT row y = l + 10 k
    // (zero row outside the box), looked up per use (registers are short)
    auto roff = [&](int k) { return rowoff[l + 10 * k]; };
    const bool con = act && g < NP;            // this group's column
    float pm = st.pmax[b];
    const float epsn = st.eps * (float)(NP * NP);
    const float epsn_im = st.eps_im * (float)(NP * NP);

    auto window = [&](int itn) {
        const LedPos p = lt.at(itn);
        return spec + (unsigned)(p.yc * L + p.xc);
    };
    auto ldO = [&](const float2 *sr, int k) {
        return ((inmask >> k) & 1) ? sr[kyr * L + f90_fold(l + 10 * k)] : make_float2(0.f, 0.f);
    };
    float2 Opre[9];
    if (a.n_order > 0) {
        const float2 *sr = window(0);
#pragma unroll
        for (int k = 0; k < 9; ++k) Opre[k] = ldO(sr, k);
    }
    unsigned *tmu = (unsigned *)tmx;
    auto note = [&](int py, int px, float ao, float an) {  // fpm_fused.hip: exact incremental tile maxima
        const int ti = ((py >> 4) - a.bty0) * a.nbx + ((px >> 4) - a.btx0);
        const unsigned cur = tmu[ti];
        if (an < ao && cur <= __float_as_uint(ao)) atomicOr(&dirty[ti >> 5], 1u << (ti & 31));
        if (__float_as_uint(an) > cur) atomicMax(&tmu[ti], __float_as_uint(an));
    };

    unsigned long long acc[kStamps] = {};
    unsigned long long prev = a.dbg ? __builtin_amdgcn_s_memtime() : 0ull;
#define FPM_STAMP(i)                                                  \
    if (a.dbg) {                                                      \
        const unsigned long long now_ = __builtin_amdgcn_s_memtime(); \
        acc[i] += now_ - prev;                                        \
        prev = now_;                                                  \
    }
    for (int it = 0; it < a.n_order; ++it) {
        const LedPos lp = lt.at(it);
        const int led = lp.led, xc = lp.xc, yc = lp.yc;
        float2 *srow = spec + (unsigned)(yc * L + xc);
        const uint16_t *Ib = a.meas + ((size_t)led * st.B + b) * NP * NP;
        float2 v[10];

        // ---- A: row IDFT of box row g of O*P (:358-365) -> T
        if (ron) {
#pragma unroll
            for (int k = 0; k < 9; ++k) v[k] = pout(pmul(pin(Opre[k]), pin(P[k])));  // :364
            v[9] = make_float2(0.f, 0.f);
            dft90_ab<true>(v, tile, tw, l, xrd);
            if (l < 9) {
                float2 *row = th + g * TLD + l;
#pragma unroll
                for (int m = 0; m < 10; ++m) row[9 * m] = v[m];
            }
        }
        // this column's measurement run, issued before the barrier (its
        // latency overlaps the wait): lane j < 9 holds I[j + 9 k][x], k < 10
        uint32_t mi[5] = {0u, 0u, 0u, 0u, 0u};
        if (con && l < 9) {
            const uint32_t *ip = (const uint32_t *)(Ib + (g * 9 + l) * 10);  // 20 B, 4-B aligned
#pragma unroll
            for (int i = 0; i < 5; ++i) mi[i] = ip[i];
        }
        __syncthreads();  // T complete; the previous LED's max|P| partials
        FPM_STAMP(7)
        if (it > 0) {  // max|P| of the previous pupil update (:415)
            float pm2 = red[32];
#pragma unroll
            for (int i = 1; i < NW; ++i) pm2 = fmaxf(pm2, red[32 + i]);
            pm = sqrtf(pm2);
        }

        // ---- B: column g: IDFT, amplitude replacement, DFT (:365-394)
        if (con) {
            const int x = g;
#pragma unroll
            for (int k = 0; k < 9; ++k) v[k] = th[roff(k) + x];
            v[9] = make_float2(0.f, 0.f);
            dft90_ab<true>(v, tile, tw, l, xrd);
            // layout B: v[m] = r at y = l + 9 m (lane 9 idle).  psi = r / Np^2
            // (:365); sqrt(I) psi / |psi + eps| = r / sqrt(|r + eps Np^2|^2 / I)
#pragma unroll
            for (int m = 0; m < 10; ++m) {
                const uint32_t wd = l < 9 ? mi[m >> 1] : 0u;
                const float Iv = (float)((m & 1) ? (wd >> 16) : (wd & 0xffffu));
                const pf2 tt = pin(v[m]) + (pf2){epsn, epsn_im};
                const float mag2 = __builtin_fmaf(tt.x, tt.x, tt.y * tt.y);
                v[m] = pout(pin(v[m]) * amp_scale(mag2, Iv));
            }
            dft90_ba<false>(v, tile, tw, l, xrd);
#pragma unroll
            for (int k = 0; k < 9; ++k) {
                const int ro = roff(k);
                th[ro + (ro == zoff ? TLD : 0) + x] = v[k];
            }
        }
        FPM_STAMP(10)
        __syncthreads();
        FPM_STAMP(2)

        // ---- C: row DFT of box row g, layout B -> A: F on this lane's pixels (:394)
        float2 F[9];
        if (ron) {
            const float2 *row = th + g * TLD + (l < 9 ? l : 0);
#pragma unroll
            for (int m = 0; m < 10; ++m) v[m] = row[9 * m];
            dft90_ba<false>(v, tile, tw, l, xrd);
#pragma unroll
            for (int k = 0; k < 9; ++k) F[k] = v[k];
        } else {
#pragma unroll
            for (int k = 0; k < 9; ++k) F[k] = make_float2(0.f, 0.f);
        }
        // no barrier: a group reads and rewrites only its own T row g in C and
        // in the update below
        FPM_STAMP(8)

        // ---- object update on the support (:405-447) and pupil numerator
        // (:457-464); tile maxima kept exact incrementally (fpm_fused.hip)
        // only the disk pixels (P = 0 elsewhere: no update, zero numerator);
        // slots off the disk in every lane of a wave are skipped whole
#pragma unroll
        for (int k = 0; k < 9; ++k) {
            if ((inmask >> k) & 1) {
                float2 num;
                float oa;
                const float2 nv = slot_update(F[k], Opre[k], P[k], pm, st, num, oa);
                th[g * TLD + k * 10 + l] = num;
                const int kx = f90_fold(l + 10 * k);
                srow[kyr * L + kx] = nv;
                note(yc + kyr, xc + kx, oa, cmag(nv));
            }
        }
        // the waves with no box row (idle in C and the update): max over the
        // band tiles outside this LED's window, which no update touches
        if (w >= wi0) {
            float c, d;
            const TileWin wn = tile_window(yc, xc, R, a.bty0, a.btx0);  // the band tiles this LED's update touches
            outside_max(tmx, dirty, a.nbt, a.nbx, a.rnbx, wn, tid - 64 * wi0, NT - 64 * wi0, c, d);
            if (lane == 0) {  // >= 0: the float bits order as unsigned
                atomicMax(&omx[0], __float_as_uint(c));
                atomicMax(&omx[1], __float_as_uint(d));
            }
        }
        FPM_STAMP(9)
        __syncthreads();  // spectrum writes, tile maxima, dirty bits; outside maxima
        if (it + 1 < a.n_order) {
            const float2 *sr = window(it + 1);
#pragma unroll
            for (int k = 0; k < 9; ++k) Opre[k] = ldO(sr, k);
        }
        FPM_STAMP(4)

        // ---- exact max|objF| (:460,467) from the band-tile maxima
        // the last wave folds the window tiles into the outside maxima
        // (tilemax.hpp) and hands them over through one barrier
        if (w == NW - 1) {
            float c, d;
            const TileWin wn = tile_window(yc, xc, R, a.bty0, a.btx0);  // (recomputed: registers are short)
            window_max(tmx, dirty, a.nbx, wn, lane, __uint_as_float(omx[0]), __uint_as_float(omx[1]), c, d);
            if (lane == 0) {
                red[0] = c;
                red[16] = d;
                // the next LED's scans start after the barrier below; the zero is
                // materialised here (the compiler spilled a hoisted constant
                // zero pair and reloaded it from scratch on this path)
                unsigned z;
                asm volatile("v_mov_b32 %0, 0" : "=v"(z));
                omx[0] = z;
                omx[1] = z;
            }
        }
        __syncthreads();
        const float cm = red[0], dm = red[16];
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
        // P += num / max|objF| on the support (:468-475); max|P| for the next LED (:415)
        float pmx = 0.f;
#pragma unroll
        for (int k = 0; k < 9; ++k) {
            if ((inmask >> k) & 1) {
                const float2 n = th[g * TLD + k * 10 + l];
                P[k] = make_float2(P[k].x + n.x * rom, P[k].y + n.y * rom);
                pmx = fmaxf(pmx, cabs2(P[k]));
            }
        }
        // max|P| partials per wave; folded after the next LED's A barrier (the
        // next update is its first use), so this phase needs no barrier
        pmx = wave_max_nonneg(pmx);
        if (lane == 0) red[32 + w] = pmx;
        FPM_STAMP(6)
    }
    auto fold_pm = [&]() {
        float pm2 = red[32];
#pragma unroll
        for (int i = 1; i < NW; ++i) pm2 = fmaxf(pm2, red[32 + i]);
        return sqrtf(pm2);
    };
    if (a.n_order > 0) {
        __syncthreads();  // the last LED's red[32..]
        pm = fold_pm();
    }
#undef FPM_STAMP
    probe.stop(st.clk);
    if (a.dbg && (tid == 0 || tid == NT - 64))
        for (int i = 0; i < kStamps; ++i) atomicAdd(&a.dbg[(tid ? kStamps : 0) + i], acc[i]);

#pragma unroll
    for (int k = 0; k < 9; ++k)
        if ((inmask >> k) & 1) pup[(kyr + R) * NB + f90_fold(l + 10 * k) + R] = P[k];
    for (int k = tid; k < a.nbt; k += NT) tmax_g[band_gtile(k)] = tmx[k];
    for (int i = tid; i < nwords; i += NT) dirty_g[i] = dirty[i];
    if (tid == 0) st.pmax[b] = pm;
}

// ------------------------------------------------------------------ host side
namespace {
size_t s90_lds_bytes(int nb, int nbt, int xw, int tld) {
    return (size_t)(f90::NW * xw + (nb + 2) * tld + 100) * sizeof(float2) + 52 * sizeof(float) +
           f90::NP * sizeof(int) + (size_t)nbt * sizeof(float) + (size_t)(nbt + 31) / 32 * sizeof(unsigned);
}
}  // namespace

// Np 90 fused kernel available for this geometry (band inside the spectrum, LDS fits)?
bool fused_s90_supported(int np, int r, const DevState &st) {
    if (np != f90::NP || r < 1 || r > f90::RMAX) return false;
    if (st.sy0 < 0 || st.sy1 >= st.L || st.sy0 > st.sy1 || st.sx0 < 0 || st.sx1 >= st.L || st.sx0 > st.sx1)
        return false;
    const int bty0 = st.sy0 / kTile, btx0 = st.sx0 / kTile;
    const int nbx = st.sx1 / kTile - btx0 + 1, nbt = nbx * (st.sy1 / kTile - bty0 + 1);
    return s90_lds_bytes(2 * r + 1, nbt, f90::XW_DENSE, f90::TLD) <= 160 * 1024;
}

hipError_t launch_fused_s90_iteration(const DevState &st, const uint16_t *meas, const int *order_dev,
                                      const int *x0_dev, const int *y0_dev, int n_order, const float2 *tw_np,
                                      unsigned long long *dbg, hipStream_t s) {
    if (!fused_s90_supported(st.np, st.r, st)) return hipErrorInvalidValue;
    FusedS90Args a;
    a.st = st;
    a.meas = meas;
    a.order = order_dev;
    a.x0 = x0_dev;
    a.y0 = y0_dev;
    a.tw = tw_np;
    a.n_order = n_order;
    a.bty0 = st.sy0 / kTile;
    a.btx0 = st.sx0 / kTile;
    a.nbx = st.sx1 / kTile - a.btx0 + 1;
    a.nbt = a.nbx * (st.sy1 / kTile - a.bty0 + 1);
    a.rnbx = 1.0f / (float)a.nbx;
    // the conflict-light layout when it fits (FPM_S90_DENSE=1 forces the dense one)
    const bool fast = !getenv("FPM_S90_DENSE") && s90_lds_bytes(st.nb, a.nbt, f90::XW_FAST, f90::TLD_FAST) <= 160 * 1024;
    a.xw = fast ? f90::XW_FAST : f90::XW_DENSE;
    for (int i = 0; i < f90::GPW; ++i) a.xg[i] = fast ? f90::XG_FAST[i] : i * f90::XT;
    a.tld = fast ? f90::TLD_FAST : f90::TLD;
    a.dbg = dbg;
    size_t lds;  // the kernel's own LDS + the LED table when it fits
    a.ledtab_off = ledtab_offset(s90_lds_bytes(st.nb, a.nbt, a.xw, a.tld), n_order, st.L, 160 * 1024, lds);
    hipError_t e = hipFuncSetAttribute((const void *)k_fused_s90, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_fused_s90, dim3(st.B), dim3(f90::NT), lds, s, a);
    return hipGetLastError();
}

}  // namespace fpm
