// fused_mr.hip -- the fused per-patch FPM iteration for Np = 200 (BASELINE
// config 3, dataset_dogStomach.json literal: Np 200, L 600, naRadius 26):
// ONE launch per runFPM iteration, one 768-thread workgroup per patch walking
// every LED of the order (fpmMain.cpp:348-476), the whole per-LED
// intermediate in LDS.  Same step as fpm_fused.hip (Np 256), with a
// mixed-radix register transform:
//
//   200-point DFT as a 20 x 10 four-step on a 10-lane group: lane l holds
//   x[l + 10 k], k = 0..19 (the "slot layout").  Stage 1 is a 20-point DFT
//   over the registers (5 x 4), then the twiddles W200^{l m1}, one LDS
//   exchange in two rounds (m1 < 10, then m1 >= 10: lane l' reads row l' of a
//   10 x 10 tile each time), and stage 2 is two 10-point DFTs (5 x 2) per lane
//   (m1 = l' and m1 = l' + 10).  Their outputs X[m1 + 20 m2] land in register
//   k = 2 m2 (+1 for m1 = l' + 10): exactly the slot layout again, so the
//   spatial samples after the inverse and the inputs of the forward transform
//   share registers, and amplitude replacement needs no data movement.
//   Six lanes groups per wave (lanes 60..63 idle), 72 groups per workgroup.
//
// Support pruning: the pupil box |k| <= r (r <= 29) occupies registers
// k in {0,1,2,17,18,19} of every lane, so the inverse transforms' inputs and
// the forward transforms' outputs are pruned to those six "slots".  The
// whole 200-column T (box rows x 200, 88 KB for r = 26) stays in LDS, so
// every box row gets its own group (no tail rows) and the row transforms run
// once per LED.
//
// Per LED step, per workgroup:
//   A  row IDFTs of the box rows of O*P (fpmMain.cpp:358-365) -> T
//   B  per column x: column IDFT, 1/Np^2, psi' = sqrt(I) psi/|psi + eps|
//      (eps on Re and Im), column DFT, box rows -> T
//      (:365-394)
//   C  row DFTs of the box rows, output-pruned to the support (:394)
//   update, exact max|objF| from incremental tile maxima, pupil update
//      (:405-475), as in fpm_fused.hip.
#include <hip/hip_runtime.h>

#include <cstdlib>

#include "cpk.hpp"
#include "dft200.hpp"
#include "fft_lds.hpp"
#include "fpm_state.hpp"
#include "fused_sync.hpp"
#include "ledtab.hpp"
#include "tilemax.hpp"
#include "update.hpp"

namespace fpm {

namespace fm {
constexpr int NP = 200;
constexpr int N1 = 20;   // registers per lane (stage-1 length)
constexpr int N2 = 10;   // lanes per group (stage-2 length)
constexpr int GPW = 6;   // groups per wave (lanes 60..63 idle)
constexpr int NT = 768;  // 12 waves: 3 per SIMD (168-VGPR budget)
constexpr int NW = NT / 64;
constexpr int NG = NW * GPW;              // 72 groups >= box rows (r <= 35)
constexpr int SK[6] = {0, 1, 2, 17, 18, 19};  // registers that can hold |k| <= 29
constexpr int RMAX = 29;
static_assert((2 * RMAX + 1 + GPW - 1) / GPW < NW, "a wave with no box row (tilemax.hpp)");
static_assert(NG >= 2 * RMAX + 1, "one group per box row");
constexpr int KYOFF = 32;                 // sig table covers ky in [-32, 31]
constexpr int XP = 10;                    // exchange-tile row pitch (complex)
constexpr int XT = 10 * XP;               // exchange tile per group (complex)
// Exchange-tile layouts, per wave slot (six group tiles of 100 complex):
//   dense   stride 100 (slot 600)
//   stride  106 = 10 (mod 32): the 8-byte row writes of the groups sharing a
//           16-lane batch land on disjoint banks (slot 636)
//   shifted the s90 kernel's offsets 0, 122, 230, 356, 478, 602 (slot 704;
//           fused_s90.hip): writes and 16-byte row reads both spread
//           (tools/lds_s90.py: 80 LDS cycles per exchange round vs 90 with
//           stride 106 and 60 conflict-free)
// The largest that fits with the T pitch below is used.
constexpr int XW_DENSE = 600, XW_STRIDE = 636, XW_SHIFT = 704;
constexpr int XG_SHIFT[GPW] = {0, 122, 230, 356, 478, 602};
constexpr int TLD = NP + 1;               // T row pitch (complex), dense
// T row pitch when LDS allows: 202 = 10 (mod 32), so the column reads of
// pass B (consecutive rows for the ten lanes of a group, adjacent columns for
// the groups) and the row accesses of passes A / C spread over the banks
// (tools/lds_s90.py --mr: modelled LDS-array cycles of the T accesses 6056 ->
// 4150 per LED, conflict-free 3096)
constexpr int TLD_FAST = 202;
}  // namespace fm

struct FusedMRArgs {
    DevState st;
    const uint16_t *meas;    // [nS][B][x][l][k] = I[l + 10 k][x] (meas_layout, preprocess.hip)
    const int *order, *x0, *y0;
    const float2 *tw;        // exp(-2 pi i k / 200), k < 200
    int n_order;
    int btx0, bty0, nbx, nbt;  // live-band tiles (fpm_fused.hip FusedArgs)
    float rnbx;
    unsigned long long *dbg;   // FPM_STAMPS=1 phase cycles, else null
    int xw;                    // exchange tiles: wave slot (complex)
    int xg[fm::GPW];           // tile offset of group gw in the wave slot
    int tld;                   // T row pitch (complex): TLD_FAST or fm::TLD
    int ledtab_off;            // LED table in dynamic LDS (ledtab.hpp), or -1
};

__device__ __forceinline__ int mr_slot_k(int s) { return fm::SK[s]; }
// signed frequency of slot s on lane l: l + 10 SK[s] (- Np for the upper slots)
__device__ __forceinline__ int mr_kx(int l, int s) { return l + 10 * fm::SK[s] - (fm::SK[s] >= 10 ? fm::NP : 0); }

__global__ void __launch_bounds__(fm::NT, 1) k_fused_mr(FusedMRArgs a) {
    using namespace fm;
    ClockProbe probe;
    probe.start();
    extern __shared__ __attribute__((aligned(16))) float2 sm[];
    const DevState &st = a.st;
    const int R = st.r, NB = st.nb, L = st.L;
    float2 *tiles = sm;                        // NG * XT exchange tiles
    const int TLD = a.tld;
    float2 *th = tiles + NW * a.xw;            // (NB + 2) * TLD: T rows, zero row, dummy row
    float2 *tw2 = th + (NB + 2) * TLD;         // [m1][l] = W200^{l m1}
    float *red = (float *)(tw2 + 200);         // 48: maxima per wave; [44..45] outside-window tile maxima
    unsigned *omx = (unsigned *)(red + 44);
    int *sig = (int *)(red + 48);              // 64: T row of ky in [-32, 31], -1 outside the box
    float *tmx = (float *)(sig + 64);          // nbt band-tile maxima
    unsigned *dirty = (unsigned *)(tmx + a.nbt);
    int *ccnt = (int *)(dirty + ((a.nbt + 31) >> 5));  // pass-B column-block counter

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
    const int xrd = opaque_i(l * XP);
    const int nwords = (a.nbt + 31) >> 5;

    for (int i = tid; i < 200; i += NT) tw2[i] = a.tw[((i / 10) * (i % 10)) % NP];
    for (int i = tid; i < 64; i += NT) {
        const int ky = i - KYOFF;
        sig[i] = (ky >= -R && ky <= R) ? ky + R : -1;
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
    // box row of this group (all box rows are transformed: NG >= NB)
    const bool ron = act && g < NB;
    const int wi0 = (NB + GPW - 1) / GPW;  // first wave with no box row (< NW: r <= RMAX)
    const int kyr = g - R;
    unsigned inmask = 0;
    float2 P[6];
#pragma unroll
    for (int s = 0; s < 6; ++s) {
        const int kx = mr_kx(l, s);
        const bool in = ron && (kyr * kyr + kx * kx <= R * R);
        inmask |= (in ? 1u : 0u) << s;
        P[s] = in ? pup[(kyr + R) * NB + kx + R] : make_float2(0.f, 0.f);
    }
    // the launch's LED order as an LDS table (ledtab.hpp)
    int2 *ltl = a.ledtab_off >= 0 ? (int2 *)((char *)sm + a.ledtab_off) : nullptr;
    const LedTab lt{ltl, a.order, a.x0, a.y0, NP / 2};
    if (ltl) lt.fill(ltl, a.n_order, tid, NT);
    if (tid == 0) omx[0] = omx[1] = 0u;
    __syncthreads();  // sig, tw2
    // T row offsets of this lane's six column slots (zero row outside the box)
    int roff[6];
#pragma unroll
    for (int s = 0; s < 6; ++s) {
        const int kx = mr_kx(l, s);
        const int sg = (kx >= -KYOFF && kx < KYOFF) ? sig[kx + KYOFF] : -1;
        roff[s] = sg >= 0 ? sg * TLD : zoff;
    }
    float pm = st.pmax[b];
    const float epsn = st.eps * (float)(NP * NP);
    const float epsn_im = st.eps_im * (float)(NP * NP);

    unsigned long long acc[kStamps] = {};
    unsigned long long prev = a.dbg ? __builtin_amdgcn_s_memtime() : 0ull;
#define FPM_STAMP(i)                                                  \
    if (a.dbg) {                                                      \
        const unsigned long long now_ = __builtin_amdgcn_s_memtime(); \
        acc[i] += now_ - prev;                                        \
        prev = now_;                                                  \
    }
    auto window = [&](int itn) {
        const LedPos p = lt.at(itn);
        return spec + (unsigned)(p.yc * L + p.xc);
    };
    // slot s of this lane's box row at a compile-time offset from one base
    auto soff = [](int s) { return 10 * fm::SK[s] - (fm::SK[s] >= 10 ? fm::NP : 0); };
    auto ldO = [&](const float2 *sr, int s) {
        const float2 *lr = sr + (kyr * L + l);
        return ((inmask >> s) & 1) ? lr[soff(s)] : make_float2(0.f, 0.f);
    };
    float2 Opre[6];
    if (a.n_order > 0) {
        const float2 *sr = window(0);
#pragma unroll
        for (int s = 0; s < 6; ++s) Opre[s] = ldO(sr, s);
    }
    for (int it = 0; it < a.n_order; ++it) {
        const LedPos lp = lt.at(it);
        const int led = lp.led, xc = lp.xc, yc = lp.yc;
        float2 *srow = spec + (unsigned)(yc * L + xc);
        const uint16_t *Ib = a.meas + ((size_t)led * st.B + b) * NP * NP;
        float2 v[20];

        // ---- A: row IDFTs of the box rows of O*P (:358-365) -> T
        if (ron) {
#pragma unroll
            for (int k = 0; k < 20; ++k) v[k] = make_float2(0.f, 0.f);
#pragma unroll
            for (int s = 0; s < 6; ++s) v[SK[s]] = pout(pmul(pin(Opre[s]), pin(P[s])));
            dft200<true, true>(v, tile, tw2, l, xrd);
            float2 *row = th + g * TLD + l;
#pragma unroll
            for (int k = 0; k < 20; ++k) row[10 * k] = v[k];
        }
        if (tid == 0) *ccnt = NW;  // pass-B block counter (blocks 0..NW-1 are preassigned)
        __syncthreads();  // T complete; the previous LED's max|P| partials
        FPM_STAMP(7)
        if (it > 0) {  // max|P| of the previous pupil update (:415)
            float pm2 = red[32];
#pragma unroll
            for (int i = 1; i < NW; ++i) pm2 = fmaxf(pm2, red[32 + i]);
            pm = sqrtf(pm2);
        }

        // ---- B: IDFT, amplitude replacement, DFT per column (:365-394).  Column
        // blocks of GPW: block c gives group gw of a wave column GPW c + gw; wave w
        // starts with block w and claims the next from an LDS counter (the VALU
        // arbiter's age order makes a static split finish unevenly, fpm_fused.hip)
        constexpr int NBLK = (NP + GPW - 1) / GPW;
        int cb = w;
#pragma unroll 1
        while (true) {
            int nx = 0;
            if (lane == 0) nx = atomicAdd(ccnt, 1);
            nx = __builtin_amdgcn_readfirstlane(nx);
            const int x = GPW * cb + gw;
            if (act && x < NP) {
            const uint2 *ip = (const uint2 *)(Ib + (x * N2 + l) * N1);  // 20 uint16, 8-B aligned
            uint2 mi[5];
#pragma unroll
            for (int i = 0; i < 5; ++i) mi[i] = ip[i];
#pragma unroll
            for (int k = 0; k < 20; ++k) v[k] = make_float2(0.f, 0.f);
#pragma unroll
            for (int s = 0; s < 6; ++s) v[SK[s]] = th[roff[s] + x];
            dft200<true, true>(v, tile, tw2, l, xrd);
            const unsigned iw[10] = {mi[0].x, mi[0].y, mi[1].x, mi[1].y, mi[2].x,
                                     mi[2].y, mi[3].x, mi[3].y, mi[4].x, mi[4].y};
#pragma unroll
            for (int k = 0; k < 20; ++k) {
                // psi = r/Np^2 (:365); sqrt(I) psi/|psi + eps| = r / sqrt(|r + eps Np^2|^2 / I)
                const float Iv = (float)((k & 1) ? (iw[k >> 1] >> 16) : (iw[k >> 1] & 0xffffu));
                const pf2 tt = pin(v[k]) + (pf2){epsn, epsn_im};
                const float mag2 = __builtin_fmaf(tt.x, tt.x, tt.y * tt.y);
                const float sc = amp_scale(mag2, Iv);
                v[k] = pout(pin(v[k]) * sc);
            }
            dft200<false, false>(v, tile, tw2, l, xrd);
#pragma unroll
            for (int s = 0; s < 6; ++s) th[roff[s] + (roff[s] == zoff ? TLD : 0) + x] = v[SK[s]];
            }
            if (nx >= NBLK) break;
            cb = nx;
        }
        FPM_STAMP(10)  // this wave's own columns done
        __syncthreads();
        FPM_STAMP(2)

        // ---- C: row DFTs of the box rows, output-pruned to the support (:394)
        float2 F[6];
#pragma unroll
        for (int s = 0; s < 6; ++s) Opre[s] = ldO(srow, s);
        if (ron) {
            const float2 *row = th + g * TLD + l;
#pragma unroll
            for (int k = 0; k < 20; ++k) v[k] = row[10 * k];
            dft200<false, false>(v, tile, tw2, l, xrd);
#pragma unroll
            for (int s = 0; s < 6; ++s) F[s] = v[SK[s]];
        } else {
#pragma unroll
            for (int s = 0; s < 6; ++s) F[s] = make_float2(0.f, 0.f);
        }
        // no barrier: a group reads and rewrites only its own T row g in C and
        // in the update below
        FPM_STAMP(8)

        // ---- object update on the support (:405-447) and pupil numerator
        // (:457-464); tile maxima kept exact incrementally (fpm_fused.hip)
        unsigned *tmu = (unsigned *)tmx;
        auto note = [&](int py, int px, float ao, float an) {
            const int ti = ((py >> 4) - a.bty0) * a.nbx + ((px >> 4) - a.btx0);
            const unsigned cur = tmu[ti];
            if (an < ao && cur <= __float_as_uint(ao)) atomicOr(&dirty[ti >> 5], 1u << (ti & 31));
            if (__float_as_uint(an) > cur) atomicMax(&tmu[ti], __float_as_uint(an));
        };
        if (ron) {  // support pixels only (a slot off the disk in the whole wave is skipped)
#pragma unroll
            for (int s = 0; s < 6; ++s) {
                float2 num = make_float2(0.f, 0.f);
                if ((inmask >> s) & 1) {
                    float oa;
                    const float2 nv = slot_update(F[s], Opre[s], P[s], pm, st, num, oa);
                    (srow + (kyr * L + l))[soff(s)] = nv;
                    note(yc + kyr, xc + mr_kx(l, s), oa, cmag(nv));
                }
                th[g * TLD + s * 10 + l] = num;
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
            for (int s = 0; s < 6; ++s) Opre[s] = ldO(sr, s);
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
        if (ron) {
#pragma unroll
            for (int s = 0; s < 6; ++s) {
                const float2 n = th[g * TLD + s * 10 + l];
                P[s] = make_float2(P[s].x + n.x * rom, P[s].y + n.y * rom);
                pmx = fmaxf(pmx, cabs2(P[s]));
            }
        }
        // max|P| partials per wave, folded after the next LED's A barrier (the
        // next update is the first use): this phase needs no barrier
        pmx = wave_max_nonneg(pmx);
        if (lane == 0) red[32 + w] = pmx;
        FPM_STAMP(6)
    }
#undef FPM_STAMP
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
    probe.stop(st.clk);
    // stamps of the first and the last wave (the barrier waits show who is slow)
    if (a.dbg && (tid == 0 || tid == NT - 64))
        for (int i = 0; i < kStamps; ++i) atomicAdd(&a.dbg[(tid ? kStamps : 0) + i], acc[i]);

#pragma unroll
    for (int s = 0; s < 6; ++s)
        if ((inmask >> s) & 1) pup[(kyr + R) * NB + mr_kx(l, s) + R] = P[s];
    for (int k = tid; k < a.nbt; k += NT) tmax_g[band_gtile(k)] = tmx[k];
    for (int i = tid; i < nwords; i += NT) dirty_g[i] = dirty[i];
    if (tid == 0) st.pmax[b] = pm;
}

// ------------------------------------------------------------------ host side
namespace {
size_t mr_lds_bytes(int nb, int nbt, int xw = fm::XW_DENSE, int tld = fm::TLD) {
    return (size_t)(fm::NW * xw + (nb + 2) * tld + 200) * sizeof(float2) + 48 * sizeof(float) +
           64 * sizeof(int) + (size_t)nbt * sizeof(float) + (size_t)(nbt + 31) / 32 * sizeof(unsigned) +
           sizeof(int);
}
}  // namespace

// Np 200 fused kernel available for this geometry (r <= 29, T + tiles fit)?
bool fused_mr_supported(int np, int r, const DevState &st) {
    if (np != fm::NP || r < 1 || r > fm::RMAX) return false;
    if (st.sy0 < 0 || st.sy1 >= st.L || st.sy0 > st.sy1 || st.sx0 < 0 || st.sx1 >= st.L || st.sx0 > st.sx1)
        return false;
    const int bty0 = st.sy0 / kTile, btx0 = st.sx0 / kTile;
    const int nbx = st.sx1 / kTile - btx0 + 1, nbt = nbx * (st.sy1 / kTile - bty0 + 1);
    return mr_lds_bytes(2 * r + 1, nbt) <= 160 * 1024;
}

hipError_t launch_fused_mr_iteration(const DevState &st, const uint16_t *meas, const int *order_dev,
                                     const int *x0_dev, const int *y0_dev, int n_order, const float2 *tw_np,
                                     unsigned long long *dbg, hipStream_t s) {
    if (!fused_mr_supported(st.np, st.r, st)) return hipErrorInvalidValue;
    FusedMRArgs a;
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
    a.dbg = dbg;
    // bank-friendly strides while LDS allows: tiles first, then the T pitch
    // (FPM_MR_DENSE=1 forces the dense layout, test_gpu_fused_mr.py)
    const bool dense = getenv("FPM_MR_DENSE") != nullptr;
    auto fits = [&](int xw, int tld) { return !dense && mr_lds_bytes(st.nb, a.nbt, xw, tld) <= 160 * 1024; };
    a.tld = fits(fm::XW_STRIDE, fm::TLD_FAST) ? fm::TLD_FAST : fm::TLD;
    a.xw = fits(fm::XW_SHIFT, a.tld) ? fm::XW_SHIFT : fits(fm::XW_STRIDE, a.tld) ? fm::XW_STRIDE : fm::XW_DENSE;
    for (int i = 0; i < fm::GPW; ++i)
        a.xg[i] = a.xw == fm::XW_SHIFT ? fm::XG_SHIFT[i] : i * (a.xw == fm::XW_STRIDE ? 106 : fm::XT);
    size_t lds;  // the kernel's own LDS + the LED table when it fits
    a.ledtab_off = ledtab_offset(mr_lds_bytes(st.nb, a.nbt, a.xw, a.tld), n_order, st.L, 160 * 1024, lds);
    hipError_t e = hipFuncSetAttribute((const void *)k_fused_mr, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_fused_mr, dim3(st.B), dim3(fm::NT), lds, s, a);
    return hipGetLastError();
}

}  // namespace fpm
