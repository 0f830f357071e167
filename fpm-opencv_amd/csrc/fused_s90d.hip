// fused_s90d.hip -- the Np 90 LED-update iteration (fused_s90.hip) DISTRIBUTED
// over KS = 2 or 4 workgroups per patch, for BASELINE config 2
// (dataset_mono.json: Np 90, L 360, 64 patches).  One workgroup per patch
// leaves 192 of the 256 CUs idle at 64 patches, and the LEDs of a patch are
// strictly sequential (fpmMain.cpp:345-476), so only intra-patch parallelism
// can use them.  Same partition as the Np 256 distributed kernel
// (fused_dist.hip), on fused_s90.hip's register transforms (dft90.hpp):
//
//   part p owns the box rows g = p, p + KS, p + 2 KS, ... (group g / KS) and
//   the columns [p TH, p TH + TH) (TH = ceil(90 / KS), one per group).
//   A        row IDFT of each own box row of O*P (layout A -> B), all 90
//            outputs -> Tg (a per-patch T image in L2-resident global memory)
//                                                                        (:358-365)
//   sync 1   (carries each part's max|P| partial of the previous LED; the
//            other waves form the band-tile maxima outside the LED's window
//            while the first polls)
//   B        Tg[box rows][own columns] -> LDS, column IDFT, amplitude
//            replacement, column DFT (fused_s90.hip pass B), back to Tg  (:365-394)
//   sync 2
//   C        row DFT of each own box row from Tg (layout B -> A): F on the
//            lane's pixels, complete (no partial sums)                   (:394)
//   update   own rows' disk pixels: spectrum, pupil numerator, LDS tile maxima
//                                                                 (:405-447,457-464)
//   sync 3   (carries the window's tile maxima / dirty bits)
//   merge    every part folds the partners' window tiles into its copy and
//            the outside maxima of sync 1: identical tile maxima and exact
//            max|objF| in every part                                    (:460,467)
//   P        P += num / max|objF| on the own rows (:468-475), max|P| partial
//
// Every element is computed by the same operations as in fused_s90.hip (the
// Tg round trip is exact), so the results are bit-identical to it.  Handoffs,
// coherence and timeouts: fused_sync.hpp, as in fused_dist.hip.
#include <hip/hip_runtime.h>

#include <cstdlib>

#include "cpk.hpp"
#include "dft90.hpp"
#include "fft_lds.hpp"
#include "fpm_state.hpp"
#include "fused_sync.hpp"
#include "ledtab.hpp"
#include "update.hpp"

namespace fpm {

namespace f90d {
constexpr int NP = 90;
constexpr int N2 = 10;                 // lanes per group
constexpr int GPW = 6;                 // groups per wave (lanes 60..63 idle)
constexpr int XT = 10 * kXP90;         // exchange tile per group (complex)
constexpr int RMAX = 44;               // 2 r + 1 <= Np
constexpr int kTgRows = 2 * RMAX + 1;  // Tg rows (box rows)
constexpr int kWinTiles = 64;          // window tiles published per part (<= 5 x 5 used at r <= 44)
template <int KS>
struct Cfg {
    static constexpr int TH = (NP + KS - 1) / KS;          // own columns (the last part may have fewer)
    static constexpr int NROWS = (kTgRows + KS - 1) / KS;  // own box rows, at most
    static constexpr int NW = KS == 2 ? 8 : 4;
    static constexpr int NT = 64 * NW;
    static constexpr int NG = NW * GPW;
    static constexpr int TLD = TH + 1;                     // own-column T row pitch (complex)
    static_assert(NG >= TH && NG >= NROWS, "one group per own column and per own row");
};
// per-patch area (float2): Tg, then KS x kWinTiles tile publications (max,
// dirty flag), then KS max|P| partials
constexpr size_t patch_elems(int ks) { return (size_t)kTgRows * NP + (size_t)ks * kWinTiles + ks; }
}  // namespace f90d

struct FusedS90DArgs {
    DevState st;
    const uint16_t *meas;    // [nS][B][x][j][k] = I[j + 9 k][x] (meas_layout g = 9)
    const int *order, *x0, *y0;
    const float2 *tw;        // exp(-2 pi i k / 90), k < 90
    int n_order;
    int btx0, bty0, nbx, nbt;  // live-band tiles (fpm_fused.hip FusedArgs)
    float rnbx;
    int ledtab_off;            // LED table in dynamic LDS (ledtab.hpp), or -1
    unsigned long long *dbg;   // FPM_STAMPS=1 phase cycles (fused_dist.hip's slots), else null
    float2 *xch;               // B x patch_elems(KS)
    int *flags;                // [KS B] handoff flags, abort word, [KS B] XCC ids
    int *abort_flag;
    int stall_led;             // fault injection (fpm_debug_set_stall), else -1
};

__device__ __forceinline__ int f90d_fold(int n) { return n < f90d::NP / 2 ? n : n - f90d::NP; }

template <int KS>
__global__ void __launch_bounds__(f90d::Cfg<KS>::NT, 1) k_fused_s90d(FusedS90DArgs a) {
    using namespace f90d;
    using C = Cfg<KS>;
    constexpr int NT = C::NT, NW = C::NW, TH = C::TH, TLD = C::TLD;
    extern __shared__ __attribute__((aligned(16))) float2 sm[];
    const DevState &st = a.st;
    const int R = st.r, NB = st.nb, L = st.L;
    float2 *tiles = sm;                        // NW * GPW * XT exchange tiles
    float2 *th = tiles + NW * GPW * XT;        // (NB + 2) * TLD: own columns of T, zero row, dummy row
    float2 *tw = th + (NB + 2) * TLD;          // [a][b] = W90^{a b}, a, b < 10
    float *red = (float *)(tw + 100);          // 52: maxima per wave; [40..41] outside-window tile maxima
    unsigned *omx = (unsigned *)(red + 40);
    int *rowoff = (int *)(red + 52);           // 90: T offset of FFT row y (the zero row outside the box)
    float *tmx = (float *)(rowoff + NP);       // nbt band-tile maxima
    unsigned *dirty = (unsigned *)(tmx + a.nbt);
    int *ccnt = (int *)(dirty + ((a.nbt + 31) >> 5));  // [1] handoff result

    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int gw = lane / N2;                  // group within the wave (6 = idle lanes)
    const bool act = gw < GPW;
    const int l = act ? lane - N2 * gw : 0;    // lane within the group
    const int g = w * GPW + (act ? gw : 0);    // group in the workgroup
    // block k -> patch 8 (k / (8 KS)) + k % 8, part (k / 8) % KS: the parts of
    // a patch land on one XCD under round-robin dispatch (fused_dist.hip)
    const int hown = (int)((blockIdx.x >> 3) % KS);
    const int b = (int)((blockIdx.x / (8 * KS)) * 8 + (blockIdx.x & 7));
    if (b >= st.B) return;  // grid rounded up to 8 KS blocks (block-uniform)
    float2 *area = a.xch + (size_t)b * patch_elems(KS);
    int *flg = a.flags + KS * b;
    int *xccs = a.flags + KS * st.B + 1 + KS * b;
    float2 *tile = tiles + g * XT;
    const int xrd = opaque_i(l * kXP90);
    const int nwords = (a.nbt + 31) >> 5;
    constexpr int TILES_OFF = kTgRows * NP, PMX_OFF = TILES_OFF + KS * kWinTiles;
    const int x0p = hown * TH, ncol = min(TH, NP - x0p);  // own columns
    const int nown = (NB - hown + KS - 1) / KS;           // own box rows

    for (int i = tid; i < 100; i += NT) tw[i] = a.tw[((i / 10) * (i % 10)) % NP];
    for (int i = tid; i < NP; i += NT) {
        const int ky = f90d_fold(i);
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
    // own box row of this group, its nine layout-A pixels kx = fold(l + 10 k)
    const bool ron = act && g < nown;
    const int grow = hown + KS * g;            // box row
    const int kyr = grow - R;
    unsigned inmask = 0;
    float2 P[9];
#pragma unroll
    for (int k = 0; k < 9; ++k) {
        const int kx = f90d_fold(l + 10 * k);
        const bool in = ron && (kyr * kyr + kx * kx <= R * R);
        inmask |= (in ? 1u : 0u) << k;
        P[k] = in ? pup[(kyr + R) * NB + kx + R] : make_float2(0.f, 0.f);
    }
    const bool con = act && g < ncol;          // own column x0p + g
    // the launch's LED order as an LDS table (ledtab.hpp)
    int2 *ltl = a.ledtab_off >= 0 ? (int2 *)((char *)sm + a.ledtab_off) : nullptr;
    const LedTab lt{ltl, a.order, a.x0, a.y0, NP / 2};
    if (ltl) lt.fill(ltl, a.n_order, tid, NT);
    float pm = st.pmax[b];
    const float epsn = st.eps * (float)(NP * NP);
    const float epsn_im = st.eps_im * (float)(NP * NP);

    // ---- coherence of the patch's shared data (fused_sync.hpp, fused_dist.hip)
    bool local = false;
    if (tid == 0) {
        const int mine = xcc_id() + 1;
        __hip_atomic_store(xccs + hown, mine, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        bool same = true;
#pragma unroll
        for (int p = 0; p < KS; ++p) {
            if (p == hown) continue;
            int other = 0;
            for (int spins = 0;
                 (other = __hip_atomic_load(xccs + p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) == 0; ++spins) {
                if (spins > (1 << 23) || __hip_atomic_load(a.abort_flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
                    __hip_atomic_store(a.abort_flag, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    break;
                }
                __builtin_amdgcn_s_sleep(2);
            }
            same = same && other == mine;
        }
        ccnt[1] = same;
    }
    __syncthreads();  // rowoff, tw, tile maxima, LED table; ccnt
    local = ccnt[1] != 0;
    __syncthreads();
    typedef unsigned u32x2_t __attribute__((ext_vector_type(2)));
    const __amdgpu_buffer_rsrc_t ra =
        __builtin_amdgcn_make_buffer_rsrc(area, 0, (int)(patch_elems(KS) * sizeof(float2)), 0x00020000);
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(spec, 0, L * L * (int)sizeof(float2), 0x00020000);
    const __amdgpu_buffer_rsrc_t rf = __builtin_amdgcn_make_buffer_rsrc(flg, 0, KS * (int)sizeof(int), 0x00020000);
    // partner-visible loads / stores (fused_dist.hip): loads L1-bypassing
    // (sc1); stores plain inside one XCD, write-through (sc1) across XCDs
    auto cld = [&](__amdgpu_buffer_rsrc_t r, int elem) {
        return __builtin_bit_cast(float2, __builtin_amdgcn_raw_buffer_load_b64(r, elem * (int)sizeof(float2), 0, 16));
    };
    auto cst = [&](__amdgpu_buffer_rsrc_t r, int elem, float2 v) {
        const int off = elem * (int)sizeof(float2);
        const u32x2_t d = __builtin_bit_cast(u32x2_t, v);
        if (local) __builtin_amdgcn_raw_buffer_store_b64(d, r, off, 0, 0);
        else __builtin_amdgcn_raw_buffer_store_b64(d, r, off, 0, 16);
    };
    int sync_no = 0;  // handoffs of this launch (flag values are 1, 2, 3, ...)
    bool aborted = false;
    int cur = 0;      // LED position of the handoffs below
    auto handoff = [&](auto &&idle) {
        ++sync_no;
        // fault injection (fpm_debug_set_stall): the last part stops
        // publishing from LED position stall_led on, its partners time out
        if (a.stall_led < 0 || cur < a.stall_led || hown != KS - 1) handoff_publish(flg + hown, sync_no, local);
        if (w > 0) idle();
        return handoff_wait<KS>(flg, hown, sync_no, a.abort_flag, ccnt + 1, local, rf);
    };
    auto nothing = []() {};

    auto wbase = [&](int itn) {
        const LedPos p = lt.at(itn);
        return p.yc * L + p.xc;
    };
    float2 Opre[9];
    auto load_window = [&](int itn) {  // own row's pixels (partners' spectrum writes visible)
        const int wb = wbase(itn) + kyr * L;
        float2 e[9];
#pragma unroll
        for (int k = 0; k < 9; ++k) e[k] = cld(rs, ron ? wb + f90d_fold(l + 10 * k) : 0);
#pragma unroll
        for (int k = 0; k < 9; ++k) Opre[k] = ((inmask >> k) & 1) ? e[k] : make_float2(0.f, 0.f);
    };
    if (a.n_order > 0) load_window(0);
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
        cur = it;
        const LedPos lp = lt.at(it);
        const int led = lp.led, xc = lp.xc, yc = lp.yc;
        const int wb0 = yc * L + xc;
        const uint16_t *Ib = a.meas + ((size_t)led * st.B + b) * NP * NP;
        float2 v[10];

        if (tid == 0) omx[0] = omx[1] = 0u;  // read by the previous LED's merge, before its last barrier
        __syncthreads();  // red[32..] of the previous pupil phase
        FPM_STAMP(0)
        // ---- A: row IDFT of each own box row of O*P (:358-365) -> Tg
        if (ron) {
#pragma unroll
            for (int k = 0; k < 9; ++k) v[k] = pout(pmul(pin(Opre[k]), pin(P[k])));  // :364
            v[9] = make_float2(0.f, 0.f);
            dft90_ab<true>(v, tile, tw, l, xrd);
            if (l < 9) {
#pragma unroll
                for (int m = 0; m < 10; ++m) cst(ra, grow * NP + l + 9 * m, v[m]);
            }
        }
        // this column's measurement run, issued before the handoff (its
        // latency overlaps the wait): lane j < 9 holds I[j + 9 k][x], k < 10
        uint32_t mi[5] = {0u, 0u, 0u, 0u, 0u};
        if (con && l < 9) {
            const uint32_t *ip = (const uint32_t *)(Ib + ((x0p + g) * 9 + l) * 10);  // 20 B, 4-B aligned
#pragma unroll
            for (int i = 0; i < 5; ++i) mi[i] = ip[i];
        }
        FPM_STAMP(1)
        // ---- sync 1, with this part's max|P| partial of the previous LED
        if (it > 0 && tid == 0) {
            float m2 = red[32];
#pragma unroll
            for (int i = 1; i < NW; ++i) m2 = fmaxf(m2, red[32 + i]);
            cst(ra, PMX_OFF + hown, make_float2(m2, 0.f));
        }
        // while the first wave polls: the max over the band tiles OUTSIDE this
        // LED's window (no part's update touches them), folded into omx
        const int wty0 = (yc - R) >> 4, wtx0 = (xc - R) >> 4;
        const int wty1 = (yc + R) >> 4, wtx1 = (xc + R) >> 4;
        if (!handoff([&]() {
                float c = 0.f, d = 0.f;
                for (int k = tid - 64; k < a.nbt; k += NT - 64) {
                    const int dy = band_dy(k), ty = a.bty0 + dy, tx = a.btx0 + k - dy * a.nbx;
                    if (ty >= wty0 && ty <= wty1 && tx >= wtx0 && tx <= wtx1) continue;
                    const float vv = tmx[k];
                    if ((dirty[k >> 5] >> (k & 31)) & 1u) d = fmaxf(d, vv);
                    else c = fmaxf(c, vv);
                }
                c = wave_max(c);
                d = wave_max(d);
                if (lane == 0) {
                    atomicMax(&omx[0], __float_as_uint(c));
                    atomicMax(&omx[1], __float_as_uint(d));
                }
            })) {
            aborted = true;
            break;
        }
        if (it > 0) {  // max|P| of the previous LED's pupil over all parts (:415)
            float2 e[KS];
#pragma unroll
            for (int p = 0; p < KS; ++p) e[p] = cld(ra, PMX_OFF + p);
            float m2 = 0.f;
#pragma unroll
            for (int p = 0; p < KS; ++p) m2 = fmaxf(m2, e[p].x);
            pm = sqrtf(m2);
        }
        FPM_STAMP(2)

        // ---- B: own columns of T from Tg, column IDFT, amplitude, DFT (:365-394)
        {   // every load issued before the first LDS store (clamped, masked after)
            constexpr int NLD = (kTgRows * TH + NT - 1) / NT;
            const int tot = NB * ncol;
            float2 q[NLD];
#pragma unroll
            for (int k = 0; k < NLD; ++k) {
                const int i = min(tid + NT * k, tot - 1), row = i / ncol, c = i - row * ncol;
                q[k] = cld(ra, row * NP + x0p + c);
            }
#pragma unroll
            for (int k = 0; k < NLD; ++k) {
                const int i = tid + NT * k, row = i / ncol, c = i - row * ncol;
                if (i < tot) th[row * TLD + c] = q[k];
            }
        }
        __syncthreads();
        if (con) {
            const int x = g;
#pragma unroll
            for (int k = 0; k < 9; ++k) v[k] = th[rowoff[l + 10 * k] + x];
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
                const int ro = rowoff[l + 10 * k];
                th[ro + (ro == zoff ? TLD : 0) + x] = v[k];
            }
        }
        __syncthreads();
        for (int i = tid; i < NB * ncol; i += NT) {
            const int row = i / ncol, c = i - row * ncol;
            cst(ra, row * NP + x0p + c, th[row * TLD + c]);
        }
        FPM_STAMP(3)
        if (!handoff(nothing)) {  // ---- sync 2
            aborted = true;
            break;
        }
        FPM_STAMP(4)

        // ---- C: row DFT of each own box row, layout B -> A: F on the lane's pixels (:394)
        float2 F[9];
        if (ron) {
#pragma unroll
            for (int m = 0; m < 10; ++m) v[m] = cld(ra, grow * NP + (l < 9 ? l : 0) + 9 * m);
            dft90_ba<false>(v, tile, tw, l, xrd);
#pragma unroll
            for (int k = 0; k < 9; ++k) F[k] = v[k];
        } else {
#pragma unroll
            for (int k = 0; k < 9; ++k) F[k] = make_float2(0.f, 0.f);
        }
        FPM_STAMP(5)

        // ---- object update of the own rows' disk pixels (:405-447), pupil
        // numerator (:457-464) into the group's exchange tile; tile maxima
        // kept exact incrementally (fpm_fused.hip)
        if (ron) {
#pragma unroll
            for (int k = 0; k < 9; ++k) {
                float2 num = make_float2(0.f, 0.f);
                if ((inmask >> k) & 1) {
                    float oa;
                    const float2 nv = slot_update(F[k], Opre[k], P[k], pm, st, num, oa);
                    const int kx = f90d_fold(l + 10 * k);
                    cst(rs, wb0 + kyr * L + kx, nv);
                    note(yc + kyr, xc + kx, oa, cmag(nv));
                }
                tile[k * 10 + l] = num;
            }
        }
        __syncthreads();  // tile maxima of this part's pixels
        // publish the window's tiles (the only ones any part changed)
        const int wnx = wtx1 - wtx0 + 1, wnt = wnx * (wty1 - wty0 + 1);
        auto wtile = [&](int k) {  // band index of window tile k
            const int dy = k / wnx;
            return (wty0 + dy - a.bty0) * a.nbx + (wtx0 + k - dy * wnx - a.btx0);
        };
        if (tid < wnt) {
            const int bk = wtile(tid);
            cst(ra, TILES_OFF + hown * kWinTiles + tid,
                make_float2(tmx[bk], __uint_as_float((dirty[bk >> 5] >> (bk & 31)) & 1u)));
        }
        FPM_STAMP(6)
        if (!handoff(nothing)) {  // ---- sync 3
            aborted = true;
            break;
        }
        FPM_STAMP(7)
        // the next window first (its loads overlap the merge), then the
        // merge: every part ends with the same maxima and dirty bits
        if (it + 1 < a.n_order) load_window(it + 1);
        float wcm = 0.f;  // merged window tile of this thread (tid < wnt)
        bool wdirty = false;
        if (tid < wnt) {
            const int bk = wtile(tid);
            float2 e[KS - 1];
#pragma unroll
            for (int q = 0; q < KS - 1; ++q) e[q] = cld(ra, TILES_OFF + (q < hown ? q : q + 1) * kWinTiles + tid);
            float m = tmx[bk];
            unsigned d = 0;
#pragma unroll
            for (int q = 0; q < KS - 1; ++q) {
                m = fmaxf(m, e[q].x);
                d |= __float_as_uint(e[q].y);
            }
            tmx[bk] = m;
            if (d) atomicOr(&dirty[bk >> 5], 1u << (bk & 31));
            wcm = m;
            wdirty = d || ((dirty[bk >> 5] >> (bk & 31)) & 1u);
        }
        if (w == 0) {  // the merge wave folds the window tiles into the outside maxima
            float c = wdirty ? 0.f : wcm, d = wdirty ? wcm : 0.f;
            c = wave_max(c);
            d = wave_max(d);
            if (lane == 0) {
                red[0] = fmaxf(c, __uint_as_float(omx[0]));
                red[16] = fmaxf(d, __uint_as_float(omx[1]));
            }
        }
        __syncthreads();
        FPM_STAMP(8)

        // ---- exact max|objF| (:460,467), identical in every part
        const float cm = red[0], dm = red[16];
        float omax = cm;
        if (dm > cm) {  // block-uniform
            for (int k = w; k < a.nbt; k += NW) {
                if (!((dirty[k >> 5] >> (k & 31)) & 1u) || !(tmx[k] > cm)) continue;  // wave-uniform
                const int ty = a.bty0 + band_dy(k), tx = a.btx0 + k - band_dy(k) * a.nbx;
                // the tile's four loads issued together (clamped in bounds, masked after)
                float2 e[4];
                bool ok[4];
#pragma unroll
                for (int jj = 0; jj < 4; ++jj) {
                    const int pp = lane + 64 * jj;
                    const int yy = ty * 16 + (pp >> 4), xx = tx * 16 + (pp & 15);
                    ok[jj] = yy < L && xx < L;
                    e[jj] = cld(rs, ok[jj] ? yy * L + xx : 0);
                }
                float mm = 0.f;
#pragma unroll
                for (int jj = 0; jj < 4; ++jj)
                    if (ok[jj]) mm = fmaxf(mm, cmag(e[jj]));
                mm = wave_max(mm);
                if (lane == 0) {
                    tmx[k] = mm;
                    atomicAnd(&dirty[k >> 5], ~(1u << (k & 31)));
                }
            }
            __syncthreads();
            float m2 = 0.f;
            for (int k = tid; k < a.nbt; k += NT)
                if (!((dirty[k >> 5] >> (k & 31)) & 1u)) m2 = fmaxf(m2, tmx[k]);
            m2 = wave_max(m2);
            __syncthreads();
            if (lane == 0) red[w] = m2;
            __syncthreads();
            omax = red[0];
#pragma unroll
            for (int i = 1; i < NW; ++i) omax = fmaxf(omax, red[i]);
        }
        FPM_STAMP(9)
        const float rom = 1.0f / omax;
        // ---- P += num / max|objF| on the own rows (:468-475), max|P| partial (:415)
        float pmx = 0.f;
        if (ron) {
#pragma unroll
            for (int k = 0; k < 9; ++k) {
                if ((inmask >> k) & 1) {
                    const float2 n = tile[k * 10 + l];
                    P[k] = make_float2(P[k].x + n.x * rom, P[k].y + n.y * rom);
                    pmx = fmaxf(pmx, cabs2(P[k]));
                }
            }
        }
        pmx = wave_max(pmx);
        if (lane == 0) red[32 + w] = pmx;
        FPM_STAMP(10)
    }
#undef FPM_STAMP
    __syncthreads();  // red[32..]
    if (a.dbg && tid == 0 && (hown == 0 || hown == KS - 1))
        for (int i = 0; i < kStamps; ++i) atomicAdd(&a.dbg[(hown ? kStamps : 0) + i], acc[i]);
    // ---- write back: each part its own pupil rows; part 0 the tile maxima
    // (identical in every part) and max|P| over all parts
#pragma unroll
    for (int k = 0; k < 9; ++k)
        if ((inmask >> k) & 1) pup[(kyr + R) * NB + f90d_fold(l + 10 * k) + R] = P[k];
    if (a.n_order > 0 && !aborted) {
        if (tid == 0) {
            float m2 = red[32];
#pragma unroll
            for (int i = 1; i < NW; ++i) m2 = fmaxf(m2, red[32 + i]);
            cst(ra, PMX_OFF + hown, make_float2(m2, 0.f));
        }
        if (handoff(nothing) && hown == 0 && tid == 0) {
            float m2 = 0.f;
#pragma unroll
            for (int p = 0; p < KS; ++p) m2 = fmaxf(m2, cld(ra, PMX_OFF + p).x);
            st.pmax[b] = sqrtf(m2);
        }
    }
    if (hown == 0) {
        for (int k = tid; k < a.nbt; k += NT) tmax_g[band_gtile(k)] = tmx[k];
        for (int i = tid; i < nwords; i += NT) dirty_g[i] = dirty[i];
    }
}

// ------------------------------------------------------------------ host side
namespace {
size_t s90d_lds_bytes(int ks, int nb, int nbt) {
    const int nw = ks == 2 ? f90d::Cfg<2>::NW : f90d::Cfg<4>::NW;
    const int tld = ks == 2 ? f90d::Cfg<2>::TLD : f90d::Cfg<4>::TLD;
    return (size_t)(nw * f90d::GPW * f90d::XT + (nb + 2) * tld + 100) * sizeof(float2) + 52 * sizeof(float) +
           f90d::NP * sizeof(int) + (size_t)nbt * sizeof(float) + (size_t)(nbt + 31) / 32 * sizeof(unsigned) +
           2 * sizeof(int);
}
}  // namespace

size_t fused_s90d_elems(int B, int ks) { return (size_t)B * f90d::patch_elems(ks); }

// Workgroups per patch for the Np 90 kernel: FPM_S90D=2/4 selects the
// distributed kernel when every part fits co-resident (8 KS ceil(B / 8) <= CUs),
// else 0 (one workgroup per patch, fused_s90.hip).
int fused_s90d_parts(int B, int n_cu) {
    const char *e = getenv("FPM_S90D");
    if (!e || B < 1) return 0;
    const int ks = atoi(e);
    return (ks == 2 || ks == 4) && 8 * ks * ((B + 7) / 8) <= n_cu ? ks : 0;
}

hipError_t launch_fused_s90d(const DevState &st, const uint16_t *meas, const int *order_dev, const int *x0_dev,
                             const int *y0_dev, int n_order, const float2 *tw_np, int ks, unsigned long long *dbg,
                             float2 *area, int *flags, int stall_led, hipStream_t s) {
    if (st.np != f90d::NP || st.r < 1 || st.r > f90d::RMAX || (ks != 2 && ks != 4) || !area || !flags)
        return hipErrorInvalidValue;
    if (st.sy0 < 0 || st.sy1 >= st.L || st.sy0 > st.sy1 || st.sx0 < 0 || st.sx1 >= st.L || st.sx0 > st.sx1)
        return hipErrorInvalidValue;
    FusedS90DArgs a;
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
    a.xch = area;
    a.flags = flags;
    a.abort_flag = flags + ks * st.B;
    a.stall_led = stall_led;
    const size_t lds0 = s90d_lds_bytes(ks, st.nb, a.nbt);
    if (lds0 > 160 * 1024) return hipErrorInvalidValue;
    size_t lds;  // + the LED table when it fits
    a.ledtab_off = ledtab_offset(lds0, n_order, 160 * 1024, lds);
    const void *fn = ks == 4 ? (const void *)k_fused_s90d<4> : (const void *)k_fused_s90d<2>;
    const int nt = ks == 4 ? f90d::Cfg<4>::NT : f90d::Cfg<2>::NT;
    hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
    // handoff counters and XCC ids restart at zero; the abort word is sticky
    e = hipMemsetAsync(flags, 0, (size_t)ks * st.B * sizeof(int), s);
    if (e == hipSuccess) e = hipMemsetAsync(flags + ks * st.B + 1, 0, (size_t)ks * st.B * sizeof(int), s);
    if (e != hipSuccess) return e;
    return launch_coresident(fn, 8 * ks * ((st.B + 7) / 8), nt, lds, &a, s);
}

}  // namespace fpm
