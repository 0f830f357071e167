// fused_dist.hip -- the Np 256 LED-update iteration DISTRIBUTED over KS = 2,
// 4 or 8 workgroups per patch (small batches: a 256-patch field strong-scaled
// over 2 / 4 / 8 GPUs leaves 128 / 64 / 32 patches per GPU, and one workgroup
// per patch would leave most of the 256 CUs idle; the LEDs of a patch are
// strictly sequential, fpmMain.cpp:345-476, so only intra-patch parallelism
// can fill the chip).
//
// Split mode (fpm_fused.hip) gives each workgroup a column part but keeps the
// row passes and the object/pupil update redundant in every workgroup; here
// every phase is partitioned, at the price of three handoffs per LED:
//
//   part p owns FFT rows i = p, p + KS, p + 2 KS, ... of the 64 (one per
//   16-lane group), tail rows q = p (mod KS), and the column part
//   [p 256/KS, (p+1) 256/KS).
//   gather   O = spec (own rows, on the support), X = O P              (:358-364)
//   A        row IDFTs of the own rows, all 256 outputs -> Tg (a per-patch
//            T image in L2-resident global memory)                      (:365)
//   sync 1   (also carries each part's max|P| partial of the previous LED)
//   B        Tg[box rows][own columns] -> LDS, column IDFT, 1/Np^2,
//            amplitude replacement, column DFT (pass B of fpm_fused.hip
//            verbatim), box rows back to Tg                              (:365-394)
//   sync 2
//   C        row DFTs of the own rows from Tg (full input), pruned to the
//            support columns -> F complete, no partial sums               (:394)
//   update   object update of the own rows on the support (:405-447), pupil
//            numerator (:457-464), tile maxima of |spec| in LDS
//   sync 3   the window's tile maxima / dirty bits as tagged words: the
//            words themselves are the handoff (no flag)
//   merge    every part folds the partners' window tiles into its LDS copy,
//            so all parts hold identical tile maxima
//   max      exact max|objF| (:460,467), redundant in every part (identical)
//   P        P += num / max|objF| on the own rows (:468-475), max|P| partial
//
// Handoffs: one monotone flag per part for syncs 1 and 2, tagged tile words
// for sync 3 (the tag counts LEDs across launches, FusedArgs::tag_base); Tg, the tile
// publications and the spectrum move with device-coherent policies (plain
// stores + L1-bypassing loads when every part of the patch sits on one XCD --
// the L2 is the coherence point -- sc1 otherwise), see fused_sync.hpp.
// Tg needs no double buffering: in A and C a part touches only its own rows,
// in B only its own columns, and every phase change is behind a handoff.
#include <hip/hip_runtime.h>

#include "dft16.hpp"
#include "fpm_state.hpp"
#include "fused256.hpp"
#include "fused_common.hpp"
#include "fused_sync.hpp"
#include "ledtab.hpp"
#include "update.hpp"

namespace fpm {

namespace {
constexpr int kTgRows = fz::NROWS + fz::MAXTAILROWS;  // Tg rows: 64 FFT rows + tail rows
constexpr int kWinTiles = 64;                         // window tiles published per part (<= 6 x 6 used)
// per-patch distributed-mode area (float2): Tg, then KS x kWinTiles tile
// publications (max, dirty flag), then KS max|P| partials
constexpr size_t dist_patch_elems(int ks) { return (size_t)kTgRows * fz::NP + (size_t)ks * kWinTiles + ks; }
}  // namespace

template <int KS>
__global__ void __launch_bounds__(512, 1) k_fused_dist(FusedArgs a) {
    using namespace fz;
    constexpr int NT = 512, NG = 32, NW = 8;
    constexpr int TH = NP / KS, TLD = TH + 1;          // own column part
    constexpr int NOWN = NROWS / KS;                   // own FFT row slots (groups 0 .. NOWN-1)
    constexpr int CB = TH / 4 < 16 ? TH / 4 : 16;      // pass-B block: columns (r8 % CB) + CB gg + 4 CB (r8 / CB)
    constexpr int NBLK = TH / 4;
    static_assert(KS == 2 || KS == 4 || KS == 8, "two, four or eight parts");
    ClockProbe probe;
    probe.start();
    extern __shared__ __attribute__((aligned(16))) float2 sm[];
    const int nrows = NROWS + a.n_tail_rows;
    float2 *scr_all = sm;                           // NG * XTILE exchange tiles
    float2 *th = scr_all + NG * XTILE;              // (nrows + 2) * TLD: own columns of T
    float2 *tw2 = th + (nrows + 2) * TLD;           // [m][t] = W256^{m t}
    float2 *tw = tw2 + 256;                         // W256^k
    float2 *tailX = tw + 256;                       // MAXTAIL
    float2 *tailF = tailX + MAXTAIL;                // MAXTAIL
    float *red = (float *)(tailF + MAXTAIL);        // 48: clean / dirty / pupil maxima per wave
    int *sig = (int *)(red + 48);                   // 96: T row of ky in [-48, 47], -1 outside the box
    int2 *tpx = (int2 *)(sig + 96);                 // MAXTAIL tail pixels (ky, kx)
    int *tpq = (int *)(tpx + MAXTAIL);              // MAXTAIL: tail row of each tail pixel
    float *tmx = (float *)(tpq + MAXTAIL);          // nbt: max|spec| per band tile (upper bound if dirty)
    unsigned *dirty = (unsigned *)(tmx + a.nbt);    // nbt bits
    int *ccnt = (int *)(dirty + ((a.nbt + 31) >> 5));  // [0] pass-B block counter, [1] handoff result

    const DevState &st = a.st;
    const int tid = threadIdx.x, g = tid >> 4, t = tid & 15, gg = (tid >> 4) & 3;
    const int xrd = exch_rbase(t);
    const int lane = tid & 63, w = tid >> 6;
    // block k -> patch 8 (k / (8 KS)) + k % 8, part (k / 8) % KS: the parts of a
    // patch land on one XCD under round-robin dispatch (a speed matter only)
    const int hown = (int)((blockIdx.x >> 3) % KS);
    const int b = (int)((blockIdx.x / (8 * KS)) * 8 + (blockIdx.x & 7));
    if (b >= st.B) return;  // grid rounded up to 8 KS blocks (block-uniform)
    float2 *area = a.xch + (size_t)b * dist_patch_elems(KS);
    int *flg = a.flags + KS * b;
    int *xccs = a.flags + KS * st.B + 1 + KS * b;
    const int R = st.r, NB = st.nb, L = st.L;
    float2 *scr = scr_all + g * XTILE;
    const int nwords = (a.nbt + 31) >> 5;
    // spread object update (KS 8): F, O, P of the own rows' slots staged in
    // the exchange tiles of the groups that own no FFT row (free in C and the
    // update).  32-patch shard 2.74 -> 2.83 M (update 3.6k -> 2.2k cycles per
    // LED); at KS 4 (four owner waves) the staging stores in C cost what the
    // spread saved (64-patch shard 4.16 vs 4.10 M), profiles/r05_ab/dist_max_upd_ab.txt
    // (round 6, with the arithmetic slot_kx: at KS 4 still 0.5 % slower,
    // profiles/r06_ab/dist_tail_pairs_spread4_ab.txt)
    constexpr bool kSpreadUpd = KS == 8;
    static_assert(!kSpreadUpd || 3 * NOWN * 96 <= (NG - NOWN) * XTILE, "staging fits the idle groups' tiles");
    float2 *upd_f = scr_all + NOWN * XTILE, *upd_o = upd_f + NOWN * 96, *upd_p = upd_o + NOWN * 96;
    constexpr int TILES_OFF = kTgRows * NP, PMX_OFF = TILES_OFF + KS * kWinTiles;

    // ---- one-time setup
    if (tid == 0) {
#pragma unroll
        for (int i = 0; i < MAXTAIL; ++i) {
            tpx[i] = a.tail_px[i];
            int q = 0;
#pragma unroll
            for (int k = 0; k < MAXTAILROWS; ++k)
                if (k < a.n_tail_rows && a.tail_ky[k] == a.tail_px[i].x) q = k;
            tpq[i] = q;
        }
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
    // own FFT row of this group: i = hown + KS g
    const int irow = hown + KS * g;
    const int kyr = a.ky_lo + irow;
    const bool ron = g < NOWN && irow < a.n_fft_rows;
    float2 P[6];
    unsigned inmask = 0;
#pragma unroll
    for (int s = 0; s < 6; ++s) {
        const int kx = slot_kx(t, s);
        const bool in = ron && (kyr * kyr + kx * kx <= R * R);
        inmask |= (in ? 1u : 0u) << s;
        P[s] = in ? pup[(kyr + R) * NB + kx + R] : make_float2(0.f, 0.f);
    }
    // the launch's LED order as an LDS table (ledtab.hpp)
    int2 *ltl = a.ledtab_off >= 0 ? (int2 *)((char *)sm + a.ledtab_off) : nullptr;
    const LedTab lt{ltl, a.order, a.x0, a.y0, NP / 2};
    if (ltl) lt.fill(ltl, a.n_order, tid, NT);
    __syncthreads();  // tpx / tpq / sig; LED table
    const int zoff = nrows * TLD;
    int roff[6];
#pragma unroll
    for (int s = 0; s < 6; ++s) {
        const int sg = sig[slot_kx(t, s) + KYOFF];
        roff[s] = sg >= 0 ? sg * TLD : zoff;
    }
    for (int i = tid; i < TLD; i += NT) th[zoff + i] = make_float2(0.f, 0.f);
    // tail pixel ti: this part owns it when its row q = tpq[ti] is q = hown
    // (mod KS).  At KS 8 thread NT - 1 - ti (the last wave, which owns no FFT
    // row: the tail updates and window-tile merges run beside the row
    // updates) -- 32-patch shard +1.2 %; at KS 4 the first wave measured
    // 0.6 % faster (profiles/r04_ab/dist_lastwave_ab.txt)
    const int ti = KS == 8 ? NT - 1 - tid : tid;
    const bool towner = ti < a.n_tail_px && (tpq[ti] % KS) == hown;
    const int2 tp = ti < a.n_tail_px ? tpx[ti] : make_int2(0, 0);
    float2 Pt = towner ? pup[(tp.x + R) * NB + tp.y + R] : make_float2(0.f, 0.f);
    float2 NPt = make_float2(0.f, 0.f), Ot = make_float2(0.f, 0.f);
    float pm = st.pmax[b];
    float pmx_part = 0.f;  // this part's max|P|^2 of the last pupil phase

    // ---- coherence of the patch's shared data (see fused_sync.hpp)
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
    __syncthreads();
    local = ccnt[1] != 0;
    __syncthreads();
    typedef unsigned u32x2_t __attribute__((ext_vector_type(2)));
    const __amdgpu_buffer_rsrc_t ra =
        __builtin_amdgcn_make_buffer_rsrc(area, 0, (int)(dist_patch_elems(KS) * sizeof(float2)), 0x00020000);
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(spec, 0, L * L * (int)sizeof(float2), 0x00020000);
    const __amdgpu_buffer_rsrc_t rf = __builtin_amdgcn_make_buffer_rsrc(flg, 0, KS * (int)sizeof(int), 0x00020000);
    // partner-visible loads / stores: every load L1-bypassing (sc1, served by
    // the L2 or memory); stores plain inside one XCD (the line stays in the
    // shared L2), device-scope write-through (sc1) across XCDs
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
    // idle(): work for waves 1 .. NW-1 while the first wave polls the
    // partners' flags (this part's flag is already out)
    auto handoff = [&](auto &&idle) {
        ++sync_no;
        // fault injection (fpm_debug_set_stall): the last part stops
        // publishing from LED position stall_led on, its partners time out
        if (a.stall_led < 0 || cur < a.stall_led || hown != KS - 1) handoff_publish(flg + hown, sync_no, local);
        if (w > 0) idle();
        return handoff_wait<KS>(flg, hown, sync_no, a.abort_flag, ccnt + 1, local, rf);
    };
    auto nothing = []() {};
    // exact max|objF| (:460,467): the window's tiles are merged on one wave
    // (the last at KS 8, where thread NT-1-k merges tile k; else the first)
    constexpr int WMERGE = KS == 8 ? NW - 1 : 0;
    unsigned *omx = (unsigned *)(red + 40);  // [0] clean / [1] dirty max over the tiles outside the window

    unsigned long long acc[kStamps] = {};
    unsigned long long prev = a.dbg ? __builtin_amdgcn_s_memtime() : 0ull;
#define FPM_STAMP(i)                                                  \
    if (a.dbg) {                                                      \
        const unsigned long long now_ = __builtin_amdgcn_s_memtime(); \
        acc[i] += now_ - prev;                                        \
        prev = now_;                                                  \
    }
    auto soff = [](int s) { return 16 * fz::SK[s] - (s >= 3 ? fz::NP : 0); };
    // window of LED `itn` in the centred spectrum: element offset of (ky, kx) = (0, 0)
    auto wbase = [&](int itn) {
        const LedPos p = lt.at(itn);
        return p.yc * L + p.xc;
    };
    float2 Opre[6];
    auto load_window = [&](int itn) {
        const int wb = wbase(itn) + kyr * L + t;
#pragma unroll
        for (int s = 0; s < 6; ++s) Opre[s] = ((inmask >> s) & 1) ? cld(rs, wb + soff(s)) : make_float2(0.f, 0.f);
        if (towner) Ot = cld(rs, wbase(itn) + tp.x * L + tp.y);
    };
    if (a.n_order > 0) load_window(0);
    const float epsn = st.eps * (float)(NP * NP);
    const float epsn_im = st.eps_im * (float)(NP * NP);
    unsigned *tmu = (unsigned *)tmx;

    for (int it = 0; it < a.n_order; ++it) {
        cur = it;
        const LedPos lp = lt.at(it);
        const int led = lp.led, xc = lp.xc, yc = lp.yc;
        const int wb0 = yc * L + xc;
        const uint16_t *Ib = a.meas + ((size_t)led * st.B + b) * NP * NP;
        Tw wt;
        wt.load(tw2, t);
        float2 v[16], r[16];

        // ---- gather + A: row IDFTs of the own rows, all 256 outputs to Tg (:358-365)
        if (towner) tailX[ti] = pout(pmul(pin(Ot), pin(Pt)));
        if (tid == 0) omx[0] = omx[1] = 0u;  // read by the previous LED's merge, two barriers ago
        __syncthreads();  // tailX
        FPM_STAMP(0)
        if (g < NOWN) {  // group-uniform
#pragma unroll
            for (int k = 0; k < 16; ++k) v[k] = make_float2(0.f, 0.f);
#pragma unroll
            for (int s = 0; s < 6; ++s) v[SK[s]] = pout(pmul(pin(Opre[s]), pin(P[s])));   // :364
            idft256_in6(v, r, scr, wt, t, xrd);
            if (ron) {
#pragma unroll
                for (int m = 0; m < 16; ++m) cst(ra, irow * NP + t + 16 * m, r[m]);
            }
        }
        // own tail rows: direct sums over the row's pixels for every column x,
        // on the LAST waves (the FFT-row groups g < NOWN sit in the first
        // waves, so at KS 4 / 8 the sums run beside the row IDFTs)
        for (int q = hown; q < a.n_tail_rows; q += KS) {
            const int p0 = a.tail_row_p0[q], np_ = a.tail_row_np[q];
            for (int x = NT - 1 - tid; x < NP; x += NT) {
                const int ti = (x * (a.tail_row_kx0[q] + NP)) & (NP - 1);
                pf2 wa = pin(tw[ti]), wb = pin(tw[(ti + x) & (NP - 1)]);
                const pf2 wstep = pin(tw[(2 * x) & (NP - 1)]);
                pf2 s2 = {0.f, 0.f}, s3 = {0.f, 0.f};
                int p = 0;
                for (; p + 1 < np_; p += 2) {
                    s2 += pmulc(pin(tailX[p0 + p]), wa);
                    s3 += pmulc(pin(tailX[p0 + p + 1]), wb);
                    wa = pmul(wa, wstep);
                    wb = pmul(wb, wstep);
                }
                if (p < np_) s2 += pmulc(pin(tailX[p0 + p]), wa);
                cst(ra, (NROWS + q) * NP + x, pout(s2 + s3));
            }
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
        // LED's window (no part's update touches them) on waves 1 .. NW-1,
        // folded into omx by LDS atomics (float bits of values >= 0 order as
        // unsigned)
        const int wty0 = (yc - R) >> 4, wtx0 = (xc - R) >> 4;
        const int wty1 = (yc + R) >> 4, wtx1 = (xc + R) >> 4;
        if (!handoff([&]() {
                float c = 0.f, d = 0.f;
                for (int k = tid - 64; k < a.nbt; k += NT - 64) {
                    const int dy = band_dy(k), ty = a.bty0 + dy, tx = a.btx0 + k - dy * a.nbx;
                    if (ty >= wty0 && ty <= wty1 && tx >= wtx0 && tx <= wtx1) continue;
                    const float v = tmx[k];
                    if ((dirty[k >> 5] >> (k & 31)) & 1u) d = fmaxf(d, v);
                    else c = fmaxf(c, v);
                }
                c = wave_max_nonneg(c);
                d = wave_max_nonneg(d);
                if (lane == 0) {
                    atomicMax(&omx[0], __float_as_uint(c));
                    atomicMax(&omx[1], __float_as_uint(d));
                }
            })) {
            aborted = true;
            break;
        }
        if (it > 0) {  // max|P| of the previous LED's pupil over all parts (:415)
            float m2 = 0.f;
#pragma unroll
            for (int p = 0; p < KS; ++p) m2 = fmaxf(m2, cld(ra, PMX_OFF + p).x);
            pm = sqrtf(m2);
        }
        FPM_STAMP(2)

        // ---- B: own columns of T from Tg, column IDFT, amplitude, DFT (:365-394)
        {   // 16-byte loads, all issued before the first LDS write (one L2
            // round trip, not one per row: the per-row loop measured 13k cycles)
            constexpr int NQ2 = TH / 2, NLD = (kTgRows * NQ2 + NT - 1) / NT;
            typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));
            u32x4_t q[NLD];
#pragma unroll
            for (int k = 0; k < NLD; ++k) {
                const int i = tid + NT * k, row = i / NQ2, c2 = i - row * NQ2;
                q[k] = i < nrows * NQ2 ? __builtin_amdgcn_raw_buffer_load_b128(
                                             ra, (row * NP + TH * hown + 2 * c2) * (int)sizeof(float2), 0, 16)
                                       : (u32x4_t){0u, 0u, 0u, 0u};
            }
#pragma unroll
            for (int k = 0; k < NLD; ++k) {
                const int i = tid + NT * k, row = i / NQ2, c2 = i - row * NQ2;
                if (i < nrows * NQ2) {
                    th[row * TLD + 2 * c2] = make_float2(__uint_as_float(q[k].x), __uint_as_float(q[k].y));
                    th[row * TLD + 2 * c2 + 1] = make_float2(__uint_as_float(q[k].z), __uint_as_float(q[k].w));
                }
            }
        }
        if (tid == 0) *ccnt = NW;
        __syncthreads();
        {
            auto colx = [&](int r8) { return (r8 % CB) + CB * gg + 4 * CB * (r8 / CB); };
            auto ldI = [&](int xl, uint4 (&n)[2]) {
                const uint4 *ip = (const uint4 *)(Ib + ((xl + TH * hown) * 16 + t) * 16);
#pragma unroll
                for (int i = 0; i < 2; ++i) n[i] = ld_stream(ip + i);
            };
            float2 tin[6];
#pragma unroll
            for (int s = 0; s < 6; ++s) tin[s] = th[roff[s] + colx(w)];
            int r8 = w;
            if (r8 < NBLK) {
#pragma unroll 1
                for (;;) {
                    const int xl = colx(r8);
                    uint4 cI[2];
                    int nx = 0;
                    if (lane == 0) nx = atomicAdd(ccnt, 1);
                    nx = __builtin_amdgcn_readfirstlane(nx);
                    ldI(xl, cI);
#pragma unroll
                    for (int k = 0; k < 16; ++k) v[k] = make_float2(0.f, 0.f);
#pragma unroll
                    for (int s = 0; s < 6; ++s) v[SK[s]] = tin[s];
                    idft256_in6(v, r, scr, wt, t, xrd);
                    {
                        const int xn = colx(nx < NBLK ? nx : r8);
#pragma unroll
                        for (int s = 0; s < 6; ++s) tin[s] = th[roff[s] + xn];
                    }
                    const unsigned iw[8] = {cI[0].x, cI[0].y, cI[0].z, cI[0].w, cI[1].x, cI[1].y, cI[1].z, cI[1].w};
#pragma unroll
                    for (int m2 = 0; m2 < 16; ++m2) {
                        const float Iv = (float)((m2 & 1) ? (iw[m2 >> 1] >> 16) : (iw[m2 >> 1] & 0xffffu));
                        const pf2 tt = pin(r[m2]) + (pf2){epsn, epsn_im};
                        const float mag2 = __builtin_fmaf(tt.x, tt.x, tt.y * tt.y);
                        v[m2] = pout(pin(r[m2]) * amp_scale(mag2, Iv));
                    }
                    float2 o[6];
                    dft256_out6(v, o, scr, wt, t, xrd);
#pragma unroll
                    for (int s = 0; s < 6; ++s) th[roff[s] + (roff[s] == zoff ? TLD : 0) + xl] = o[s];
                    if (nx >= NBLK) break;
                    r8 = nx;
                }
            }
        }
        __syncthreads();
        for (int i = tid; i < nrows * (TH / 2); i += NT) {  // 16-byte stores
            const int row = i / (TH / 2), c2 = i - row * (TH / 2);
            const float2 e0 = th[row * TLD + 2 * c2], e1 = th[row * TLD + 2 * c2 + 1];
            typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));
            const u32x4_t d = {__float_as_uint(e0.x), __float_as_uint(e0.y), __float_as_uint(e1.x), __float_as_uint(e1.y)};
            const int off = (row * NP + TH * hown + 2 * c2) * (int)sizeof(float2);
            if (local) __builtin_amdgcn_raw_buffer_store_b128(d, ra, off, 0, 0);
            else __builtin_amdgcn_raw_buffer_store_b128(d, ra, off, 0, 16);
        }
        FPM_STAMP(3)
        if (!handoff(nothing)) {  // ---- sync 2
            aborted = true;
            break;
        }
        FPM_STAMP(4)

        // ---- C: row DFTs of the own rows (full input) -> F (:394)
        float2 F[6];
        if (g < NOWN) {
#pragma unroll
            for (int m = 0; m < 16; ++m) v[m] = ron ? cld(ra, irow * NP + t + 16 * m) : make_float2(0.f, 0.f);
            dft256_out6(v, F, scr, wt, t, xrd);
#ifdef FPM_DIST_SUBSTAMP
            FPM_STAMP(11)  // C: own FFT rows (waves with rows)
#endif
            if constexpr (kSpreadUpd) {
                // stage F, O, P of the row's slots for the spread update below
                // in the idle groups' exchange tiles (no transform uses them in C)
#pragma unroll
                for (int s = 0; s < 6; ++s) {
                    const int i = (g * 6 + s) * 16 + t;
                    upd_f[i] = F[s];
                    upd_o[i] = Opre[s];
                    upd_p[i] = P[s];
                }
            }
        } else {
#pragma unroll
            for (int s = 0; s < 6; ++s) F[s] = make_float2(0.f, 0.f);
        }
        // own tail pixels: a 16-lane group sums the 256 columns of the pixel's
        // row; pixels go to the last groups first, which own no FFT row at
        // KS 4 / 8, so the sums overlap the row DFTs instead of following them
        // on the same groups (round 3: C 7.5k cycles per LED on the parts
        // that own a tail row vs 3.2k on the part that owns none, at KS 4)
        for (int pp = NG - 1 - g; pp < a.n_tail_px; pp += NG) {
            if ((tpq[pp] % KS) != hown) continue;  // group-uniform
            const int2 px = tpx[pp];
            const int row = NROWS + tpq[pp];
            // the row's 16 values first: one L2 round trip (loads interleaved
            // with the twiddle recurrence waited for each in turn, 16 round
            // trips on every part that owns a tail row)
            float2 e[16];
#pragma unroll
            for (int m = 0; m < 16; ++m) e[m] = cld(ra, row * NP + t + 16 * m);
            pf2 s2p = {0.f, 0.f};
            pf2 wk = pin(tw[(t * (px.y + NP)) & (NP - 1)]);
            const pf2 wstep = pin(tw[(16 * (px.y + NP)) & (NP - 1)]);
#pragma unroll
            for (int m = 0; m < 16; ++m) {
                s2p += pmul(pin(e[m]), wk);
                if (m < 15) wk = pmul(wk, wstep);
            }
            float2 s2 = pout(s2p);
            s2.x = row16_sum(s2.x);  // the group's 16 lanes (DPP, bit-identical to the xor butterfly)
            s2.y = row16_sum(s2.y);
            if (t == 0) tailF[pp] = s2;
        }
        __syncthreads();  // tailF
        FPM_STAMP(5)

        // ---- object update of the own rows (:405-447), pupil numerator (:457-464)
        auto note = [&](int py, int px, float ao, float an) {
            const int ti = ((py >> 4) - a.bty0) * a.nbx + ((px >> 4) - a.btx0);
            const unsigned cur = tmu[ti];
            if (an < ao && cur <= __float_as_uint(ao)) atomicOr(&dirty[ti >> 5], 1u << (ti & 31));
            if (__float_as_uint(an) > cur) atomicMax(&tmu[ti], __float_as_uint(an));
        };
        if constexpr (kSpreadUpd) {
            // the own rows' NOWN x 96 slots spread over all NT threads (the
            // row owners are NOWN / 4 waves, one per SIMD at KS 8: six
            // updates per lane at the one-wave issue rate); numerators into
            // the owner group's exchange tile as before
#pragma unroll
            for (int j = 0; j < (NOWN * 96 + NT - 1) / NT; ++j) {
                const int i = tid + NT * j;
                if (NOWN * 96 % NT != 0 && i >= NOWN * 96) break;
                const int gi = i / 96, si = (i - gi * 96) >> 4, tt = i & 15;
                const int rowi = hown + KS * gi, ky = a.ky_lo + rowi, kx = slot_kx(tt, si);
                float2 num = make_float2(0.f, 0.f);
                if (rowi < a.n_fft_rows && ky * ky + kx * kx <= R * R) {
                    float oa;
                    const float2 nv = slot_update(upd_f[i], upd_o[i], upd_p[i], pm, st, num, oa);
                    cst(rs, wb0 + ky * L + kx, nv);
                    note(yc + ky, xc + kx, oa, cmag(nv));
                }
                scr_all[gi * XTILE + si * 16 + tt] = num;
            }
        } else if (ron) {  // support pixels only (a slot off the disk in the whole wave is skipped)
#pragma unroll
            for (int s = 0; s < 6; ++s) {
                float2 num = make_float2(0.f, 0.f);
                if ((inmask >> s) & 1) {
                    float oa;
                    const float2 nv = slot_update(F[s], Opre[s], P[s], pm, st, num, oa);
                    cst(rs, wb0 + kyr * L + t + soff(s), nv);
                    note(yc + kyr, xc + slot_kx(t, s), oa, cmag(nv));
                }
                scr[s * 16 + t] = num;
            }
        }
        if (towner) {
            float oa;
            const float2 nv = slot_update(tailF[ti], Ot, Pt, pm, st, NPt, oa);
            cst(rs, wb0 + tp.x * L + tp.y, nv);
            note(yc + tp.x, xc + tp.y, oa, cmag(nv));
        }
        // ---- sync 3 as tagged tile words (round 6).  Every wave's spectrum
        // stores are acknowledged before the barrier, so once a part's window
        // tile words carry this LED's tag its spectrum writes are visible: the
        // words are the handoff.  The merge wave publishes this part's words
        // and polls the partners' until every tag matches, holding the values
        // it needs for the merge -- no flag store behind a second
        // acknowledgement, no data load behind the flag.
        __builtin_amdgcn_s_waitcnt(0);  // this wave's spectrum stores acknowledged
        __syncthreads();  // tile maxima of this part's pixels; every wave's stores acknowledged
        FPM_STAMP(6)
        const int wnx = wtx1 - wtx0 + 1, wnt = wnx * (wty1 - wty0 + 1);
        auto wtile = [&](int k) {  // band index of window tile k
            const int dy = k / wnx;
            return (wty0 + dy - a.bty0) * a.nbx + (wtx0 + k - dy * wnx - a.btx0);
        };
        if (w == WMERGE) {
            // thread ti < wnt owns window tile ti (see towner: ti spans 0..63
            // over this wave); the lane with ti == kWinTiles - 1 (never a
            // tile: wnt <= 36) watches the abort word
            const bool mine = ti < wnt, watch = ti == kWinTiles - 1;
            const int bk = mine ? wtile(ti) : 0;
            const float own = mine ? tmx[bk] : 0.f;
            const unsigned odirty = mine ? (dirty[bk >> 5] >> (bk & 31)) & 1u : 0u;
            const unsigned tag = (a.tag_base + (unsigned)it + 1u) & 0x7fffffffu;
            // fault injection (fpm_debug_set_stall) as for the flags
            const bool publish = a.stall_led < 0 || it < a.stall_led || hown != KS - 1;
            if (mine && publish) cst(ra, TILES_OFF + hown * kWinTiles + ti, make_float2(own, __uint_as_float(tag << 1 | odirty)));
            float2 e[KS - 1];
            bool ok = true;
            for (int spins = 0;; ++spins) {
                // every partner word of this lane's tile in one round trip
                // (lane part of the offset in one VGPR, the partner's block
                // offset in the scalar soffset: no per-partner address held
                // across the LED loop)
#pragma unroll
                for (int q = 0; q < KS - 1; ++q)
                    e[q] = mine ? __builtin_bit_cast(
                                      float2, __builtin_amdgcn_raw_buffer_load_b64(
                                                  ra, ti * (int)sizeof(float2),
                                                  (TILES_OFF + (q < hown ? q : q + 1) * kWinTiles) * (int)sizeof(float2),
                                                  kAuxL2Volatile))
                                : make_float2(0.f, 0.f);
                const int ab = watch ? __hip_atomic_load(a.abort_flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0;
                bool done = true;
#pragma unroll
                for (int q = 0; q < KS - 1; ++q) done = done && (!mine || (__float_as_uint(e[q].y) >> 1) == tag);
                if (__all(done)) break;
                if (__any(ab != 0) || spins > (1 << 23)) {
                    if (watch) __hip_atomic_store(a.abort_flag, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    ok = false;
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
            }
            FPM_STAMP(7)
            // merge: every part ends with the same maxima and dirty bits
            float m = own;
            unsigned d = 0;
#pragma unroll
            for (int q = 0; q < KS - 1; ++q) {
                m = fmaxf(m, e[q].x);
                d |= __float_as_uint(e[q].y) & 1u;
            }
            if (mine) {
                tmx[bk] = m;
                if (d) atomicOr(&dirty[bk >> 5], 1u << (bk & 31));
            }
            const bool wdirty = (d | odirty) != 0;
            // fold the window tiles into the outside maxima of sync 1
            float c = mine && !wdirty ? m : 0.f, dd = mine && wdirty ? m : 0.f;
            c = wave_max_nonneg(c);
            dd = wave_max_nonneg(dd);
            if (lane == 0) {
                red[0] = fmaxf(c, __uint_as_float(omx[0]));
                red[16] = fmaxf(dd, __uint_as_float(omx[1]));
                ccnt[1] = ok;
            }
        }
        __syncthreads();
        if (!ccnt[1]) {
            aborted = true;
            break;
        }
        // the next window: partners' spectrum writes are visible; its loads
        // are consumed at the next LED's gather, behind the max and P phases
        if (it + 1 < a.n_order) load_window(it + 1);
        FPM_STAMP(8)

        // ---- exact max|objF| (:460,467), identical in every part: the
        // outside maxima of sync 1 and the merged window tiles
        const float cm = red[0], dm = red[16];
        float omax = cm;
        if (dm > cm) {
            for (int k = w; k < a.nbt; k += NW) {
                if (!((dirty[k >> 5] >> (k & 31)) & 1u) || !(tmx[k] > cm)) continue;
                const int ty = a.bty0 + band_dy(k), tx = a.btx0 + k - band_dy(k) * a.nbx;
                float2 e[4];  // all four loads before the first use
#pragma unroll
                for (int jj = 0; jj < 4; ++jj) {
                    const int pp = lane + 64 * jj;
                    e[jj] = cld(rs, (ty * 16 + (pp >> 4)) * L + tx * 16 + (pp & 15));
                }
                float mm = 0.f;
#pragma unroll
                for (int jj = 0; jj < 4; ++jj) mm = fmaxf(mm, cmag(e[jj]));
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
        FPM_STAMP(9)
        const float rom = 1.0f / omax;
        // ---- P += num / max|objF| on the own rows (:468-475), max|P| partial (:415)
        float pmx = 0.f;
        if (ron) {
#pragma unroll
            for (int s = 0; s < 6; ++s) {
                const float2 n = scr[s * 16 + t];
                P[s] = make_float2(P[s].x + n.x * rom, P[s].y + n.y * rom);
                pmx = fmaxf(pmx, cabs2(P[s]));
            }
        }
        if (towner) {
            Pt = make_float2(Pt.x + NPt.x * rom, Pt.y + NPt.y * rom);
            pmx = fmaxf(pmx, cabs2(Pt));
        }
        pmx = wave_max_nonneg(pmx);
        if (lane == 0) red[32 + w] = pmx;
        FPM_STAMP(10)
    }
#undef FPM_STAMP
    __syncthreads();  // red[32..]
    probe.stop(a.st.clk);
#ifndef FPM_STAMP_PART2
#define FPM_STAMP_PART2 (KS - 1)  // diagnostic builds: the part recorded in the second stamp slot
#endif
    if (a.dbg && tid == 0 && (hown == 0 || hown == FPM_STAMP_PART2))
        for (int i = 0; i < kStamps; ++i) atomicAdd(&a.dbg[(hown ? kStamps : 0) + i], acc[i]);
    // ---- write back: each part its own pupil rows and tail pixels; part 0
    // the tile maxima (identical in every part) and max|P| over all parts
    if (ron) {
#pragma unroll
        for (int s = 0; s < 6; ++s)
            if ((inmask >> s) & 1) pup[(kyr + R) * NB + slot_kx(t, s) + R] = P[s];
    }
    if (towner) pup[(tp.x + R) * NB + tp.y + R] = Pt;
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
    (void)pmx_part;
    (void)pm;
}

// ------------------------------------------------------------------ host side
size_t fused_dist_lds_bytes(int ks, int nbt, int n_tail_rows) {
    const int tld = fz::NP / ks + 1;
    return (size_t)(32 * XTILE + (fz::NROWS + n_tail_rows + 2) * tld + 512 + 2 * fz::MAXTAIL) * sizeof(float2) +
           48 * sizeof(float) + 96 * sizeof(int) + fz::MAXTAIL * (sizeof(int2) + sizeof(int)) +
           (size_t)nbt * sizeof(float) + (size_t)(nbt + 31) / 32 * sizeof(unsigned) + 2 * sizeof(int);
}

// distributed-mode area (float2 elements) for B patches
size_t fused_dist_elems(int B, int ks) { return (size_t)B * dist_patch_elems(ks); }

// Workgroups per patch of the distributed mode: KS = 8 when 8 B <= CUs, 4 when
// 4 B <= CUs (every part must be co-resident: launch_coresident), else 0 (not
// used).  Measured on MI355X at the metric geometry: 32
// patches 5.32 ms per iteration (split mode KS 4: 5.66), 64 patches 5.54
// (split 5.66); at 128 patches the two-part version is SLOWER than split
// mode (7.17 vs 6.71 ms: T crosses the L2 four times per LED), so KS = 2 is
// only used when forced.  FPM_NO_DIST=1 disables it; FPM_DIST=2/4/8 forces
// a count that fits.
int fused_dist_parts(int B, int n_cu, int r, int L) {
    if (B < 1 || getenv("FPM_NO_DIST")) return 0;
    const FusedGeom g = fused_geometry(fz::NP, r);
    if (!g.ok || L % kTile) return 0;
    auto fits = [&](int ks) { return 8 * ks * ((B + 7) / 8) <= n_cu; };
    if (const char *e = getenv("FPM_DIST")) {
        const int ks = atoi(e);
        return (ks == 2 || ks == 4 || ks == 8) && fits(ks) ? ks : 0;
    }
    return fits(8) ? 8 : fits(4) ? 4 : 0;
}

hipError_t launch_fused_dist(const DevState &st, const uint16_t *meas, const int *order_dev, const int *x0_dev,
                             const int *y0_dev, int n_order, const float2 *tw_np, int ks, unsigned long long *dbg,
                             float2 *area, int *flags, int stall_led, unsigned tag_base, hipStream_t s) {
    const FusedGeom g = fused_geometry(st.np, st.r);
    if (!g.ok || (ks != 2 && ks != 4 && ks != 8) || !area || !flags) return hipErrorInvalidValue;
    if (st.sy0 < 0 || st.sy1 >= st.L || st.sy0 > st.sy1 || st.sx0 < 0 || st.sx1 >= st.L || st.sx0 > st.sx1)
        return hipErrorInvalidValue;
    FusedArgs a{};
    a.st = st;
    a.meas = meas;
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
    for (int q = 0; q < fz::MAXTAILROWS; ++q) {
        a.tail_row_p0[q] = a.tail_row_np[q] = a.tail_row_kx0[q] = 0;
        for (int p = 0; p < g.n_tail_px && q < g.n_tail_rows; ++p)
            if (g.tail_px[p].x == g.tail_ky[q]) {
                if (a.tail_row_np[q] == 0) {
                    a.tail_row_p0[q] = p;
                    a.tail_row_kx0[q] = g.tail_px[p].y;
                }
                ++a.tail_row_np[q];
            }
    }
    for (int i = 0; i < fz::MAXTAIL; ++i) a.tail_px[i] = i < g.n_tail_px ? g.tail_px[i] : make_int2(0, 0);
    const Band bd = band_of(st);
    a.bty0 = bd.bty0;
    a.btx0 = bd.btx0;
    a.nbx = bd.nbx;
    a.nbt = bd.nbt;
    a.rnbx = 1.0f / (float)a.nbx;
    a.dbg = dbg;
    a.xch = area;
    a.flags = flags;
    a.abort_flag = flags + ks * st.B;
    a.stall_led = stall_led;
    a.tag_base = tag_base;
    const size_t lds0 = fused_dist_lds_bytes(ks, a.nbt, g.n_tail_rows);
    if (lds0 > 160 * 1024) return hipErrorInvalidValue;
    size_t lds;  // + the LED table when it fits
    a.ledtab_off = ledtab_offset(lds0, n_order, st.L, 160 * 1024, lds);
    const void *fn = ks == 8   ? (const void *)k_fused_dist<8>
                     : ks == 4 ? (const void *)k_fused_dist<4>
                               : (const void *)k_fused_dist<2>;
    hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
    // handoff counters and XCC ids restart at zero; the abort word is sticky
    e = hipMemsetAsync(flags, 0, (size_t)ks * st.B * sizeof(int), s);
    if (e == hipSuccess) e = hipMemsetAsync(flags + ks * st.B + 1, 0, (size_t)ks * st.B * sizeof(int), s);
    if (e != hipSuccess) return e;
    return launch_coresident(fn, 8 * ks * ((st.B + 7) / 8), 512, lds, &a, s);
}

}  // namespace fpm
