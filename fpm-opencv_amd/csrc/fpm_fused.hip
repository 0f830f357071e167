// fpm_fused.hip -- the fused per-patch FPM iteration for Np = 256 (the metric
// configuration): ONE launch per runFPM iteration, one 512-thread workgroup
// per patch, walking every LED of the order (fpmMain.cpp:348-476) without
// leaving the kernel.  Patches never interact, so there is no inter-workgroup
// communication at all; the whole per-LED intermediate lives in LDS.
//
// Per LED step, per workgroup (R = naRadius, box = 2R+1 rows, 16-lane groups):
//   gather  O = spec[yc+ky][xc+kx] on the support into registers   (:358-362)
//   for each half h of the columns (x in [128h, 128h+128)):
//     A  row IDFTs of the box rows of O*P (:364-365), the half's 128
//        outputs -> LDS half-T (64 FFT rows + <= 8 "tail" rows by direct sums)
//     B  per column x: column IDFT (only box rows are non-zero), 1/Np^2,
//        psi' = sqrt(I) psi/|psi + eps| (eps on Re and Im),
//        column DFT, keep the box
//        rows -> half-T in place                                   (:365-394)
//     C  row DFTs of the half rows, output-pruned to the support columns,
//        accumulated over the two halves in registers              (:394)
//   update  object update into the centred spectrum (:405-447) and pupil
//           numerator (:457-464); tile maxima of |spec| kept exact
//           incrementally (atomicMax + dirty bits)
//   max     exact max|objF| from the tile maxima (:460,467), dirty tiles re-read
//           only when their bound exceeds the clean maximum
//   P       P += num/max * S, max|P| for the next LED            (:468-475,415)
//
// 256-point transforms are 16x16 four-step DFTs: a 16-lane group holds 16
// complex values per lane (element index = lane + 16*register), does the two
// 16-point DFTs in registers and exchanges once through a padded (pitch 18),
// conflict-free LDS tile (dft16.hpp).  The row IDFT input, the row DFT output and the
// pupil/object registers share the "kx = lane + 16*k" layout, so P and the
// pre-update O never move.  Only k in {0,1,2,13,14,15} (|kx| <= 47) can be
// inside the support, so inputs of the inverse transforms and outputs of the
// forward ones are pruned to those six registers.  Box rows beyond the 64
// FFT rows ("tail rows", the outermost rows of the disk with a handful of
// pixels) are transformed by direct DFT sums spread over all threads.
#include <hip/hip_runtime.h>

#include <vector>

#include "dft16.hpp"
#include "fft_lds.hpp"
#include "fpm_state.hpp"
#include "fused256.hpp"
#include "fused_common.hpp"
#include "fused_sync.hpp"
#include "ledtab.hpp"
#include "update.hpp"

namespace fpm {

// Column parts: T (the row IDFTs of the box rows) is held in LDS one column
// part at a time -- two halves of 128 columns walked in turn by the
// one-workgroup kernel (KS = 1), or the one part a split-mode workgroup owns
// (KS = 2: a half, KS = 4: a quarter of 64 columns).  Row pitch part + 1
// complex, so the 16 lanes of a column read hit 16 different bank pairs.
constexpr int n_parts(int ks) { return ks == 1 ? 2 : ks; }
constexpr int part_cols(int ks) { return fz::NP / n_parts(ks); }

// Kernel configuration (NT = 512): 32 groups, 2 FFT rows each, 2 waves per
// SIMD (256 VGPRs), full exchange tiles, T slots prefetched one pass-B column
// ahead, P and F in registers throughout.  (A 1024-thread variant at 4 waves
// per SIMD -- half exchange tiles, P / F parked in global scratch -- measured
// 28 % slower and was removed in round 4)
template <int NT>
struct FzCfg {
    static_assert(NT == 512, "512 threads per workgroup");
    static constexpr int NG = NT / 16;            // 16-lane groups
    static constexpr int RPG = fz::NROWS / NG;    // FFT rows per group
    static constexpr int NW = NT / 64;            // waves
    static constexpr int XT = XTILE;              // exchange tile per group (complex)
};

// KS workgroups per patch: 1 (both column halves in turn), or split mode with
// 2 / 4 workgroups each owning one column part
template <int NT, int KS>
__global__ void __launch_bounds__(NT, 1) k_fused_iteration(FusedArgs a) {
    using namespace fz;
    using C = FzCfg<NT>;
    constexpr int NG = C::NG, RPG = C::RPG, NW = C::NW;
    ClockProbe probe;
    probe.start();
    static_assert(KS == 1 || KS == 2 || KS == 4, "one workgroup per patch, or split mode with 2 / 4");
    static_assert(6 * RPG * 16 <= C::XT, "pupil numerators are parked in the group's exchange tile");
    constexpr int NPARTS = n_parts(KS), TH = part_cols(KS), TLD = TH + 1;
    extern __shared__ __attribute__((aligned(16))) float2 sm[];
    const int nrows = NROWS + a.n_tail_rows;
    float2 *scr_all = sm;                           // NG * XT: per-group exchange tiles
    float2 *th = scr_all + NG * C::XT;              // (nrows + 2) * TLD: one column part of T = row IDFTs of the box rows
    float2 *tw2 = th + (nrows + 2) * TLD;           // [m][t] = W256^{m t}  (after the zero + dummy rows)
    float2 *tw = tw2 + 256;                         // W256^k
    float2 *tailX = tw + 256;                       // MAXTAIL
    float2 *tailF = tailX + MAXTAIL;                // MAXTAIL
    float *red = (float *)(tailF + MAXTAIL);        // 48: clean / dirty / pupil maxima per wave
    int *sig = (int *)(red + 48);                   // 96: T row of ky in [-48, 47], -1 outside the box
    int2 *tpx = (int2 *)(sig + 96);                 // MAXTAIL tail pixels (ky, kx)
    int *tky = (int *)(tpx + MAXTAIL);              // MAXTAILROWS tail rows
    float *tmx = (float *)(tky + MAXTAILROWS);      // nbt: max|spec| per band tile (upper bound if dirty)
    unsigned *dirty = (unsigned *)(tmx + a.nbt);    // nbt bits: tile max may be stale-high
    int *ccnt = (int *)(dirty + ((a.nbt + 31) >> 5));  // [0] pass-B column-block counter, [1] handoff result

    const DevState &st = a.st;
    const int tid = threadIdx.x, g = tid >> 4, t = tid & 15, gg = (tid >> 4) & 3;
    // exchange read base (see exchange16 / xchg)
    const int xrd = exch_rbase(t);
    const int lane = tid & 63, w = tid >> 6;
    // split mode: block k -> patch 8 (k / (8 KS)) + k % 8, part (k / 8) % KS, so
    // the parts of a patch are 8 blocks apart (the same XCD under round-robin
    // dispatch; only a speed matter, the handoff does not assume it)
    constexpr bool split = KS > 1;  // separate instances: the one-workgroup kernel carries no split state
    const int hown = split ? (int)((blockIdx.x >> 3) % KS) : -1;
    const int b = split ? (int)((blockIdx.x / (8 * KS)) * 8 + (blockIdx.x & 7)) : (int)blockIdx.x;
    if (b >= st.B) return;  // split grid rounded up to 8 KS blocks (block-uniform)
    const int hb = hown < 0 ? 0 : hown, he = hown < 0 ? NPARTS : hown + 1;  // parts this workgroup runs
    float2 *xch = split ? a.xch + (size_t)b * xch_patch_elems(KS) : nullptr;
    int *flg = split ? a.flags + KS * b : nullptr;
    int *xccs = split ? a.flags + KS * st.B + 1 + KS * b : nullptr;  // [KS]: XCC_ID + 1 of each part
    const int R = st.r, NB = st.nb, L = st.L;
    float2 *scr = scr_all + g * C::XT;
    const int nwords = (a.nbt + 31) >> 5;

    // ---- one-time setup (kernel-argument tables indexed with uniform indices only)
    if (tid == 0) {
#pragma unroll
        for (int i = 0; i < MAXTAIL; ++i) tpx[i] = a.tail_px[i];
#pragma unroll
        for (int i = 0; i < MAXTAILROWS; ++i) tky[i] = a.tail_ky[i];
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
    // band tiles k <-> global tile (bty0 + k / nbx, btx0 + k % nbx); (k + 0.5) / nbx
    // is never within float rounding of an integer for k < 2^16
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
    int kyr[RPG];
    bool ron[RPG];
    float2 P[RPG][6];
    unsigned inmask[RPG];
#pragma unroll
    for (int j = 0; j < RPG; ++j) {
        kyr[j] = a.ky_lo + g + NG * j;
        ron[j] = g + NG * j < a.n_fft_rows;
        inmask[j] = 0;
#pragma unroll
        for (int s = 0; s < 6; ++s) {
            const int kx = slot_kx(t, s);
            const bool in = ron[j] && (kyr[j] * kyr[j] + kx * kx <= R * R);
            inmask[j] |= (in ? 1u : 0u) << s;
            P[j][s] = in ? pup[(kyr[j] + R) * NB + kx + R] : make_float2(0.f, 0.f);
        }
    }
    // the launch's LED order as an LDS table (ledtab.hpp)
    int2 *ltl = a.ledtab_off >= 0 ? (int2 *)((char *)sm + a.ledtab_off) : nullptr;
    const LedTab lt{ltl, a.order, a.x0, a.y0, NP / 2};
    if (ltl) lt.fill(ltl, a.n_order, tid, NT);
    __syncthreads();  // tpx / tky / sig; LED table
    // per-lane half-T row offsets of this lane's six column slots; rows
    // outside the box read the zero row `nrows` and write the dummy row after it
    const int zoff = nrows * TLD;
    int roff[6];
#pragma unroll
    for (int s = 0; s < 6; ++s) {
        const int sg = sig[slot_kx(t, s) + KYOFF];
        roff[s] = sg >= 0 ? sg * TLD : zoff;
    }
    for (int i = tid; i < TLD; i += NT) th[zoff + i] = make_float2(0.f, 0.f);
    const bool towner = tid < a.n_tail_px;
    const int2 tp = towner ? tpx[tid] : make_int2(0, 0);
    float2 Pt = towner ? pup[(tp.x + R) * NB + tp.y + R] : make_float2(0.f, 0.f);
    float2 NPt = make_float2(0.f, 0.f), Ot = make_float2(0.f, 0.f);
    float pm = st.pmax[b];
    // max|P| = sqrt of the per-wave maxima of |P|^2 the pupil phase leaves in red[32..]
    auto pm_of_red = [&]() {
        float pm2 = red[32];
#pragma unroll
        for (int i = 1; i < NW; ++i) pm2 = fmaxf(pm2, red[32 + i]);
        return sqrtf(pm2);
    };
    bool pupil_done = false;  // red[32..] holds a pupil phase's maxima
    // split mode: learn whether the partner shares this XCD (then L2-level
    // handoffs, see ld_l2) -- one coherent exchange per launch
    bool local = false;
    // (descriptors are built unconditionally: the type has no empty state)
    const __amdgpu_buffer_rsrc_t rx =
        __builtin_amdgcn_make_buffer_rsrc(xch, 0, split ? xch_patch_elems(KS) * (int)sizeof(float2) : 0, 0x00020000);
    const __amdgpu_buffer_rsrc_t rf = __builtin_amdgcn_make_buffer_rsrc(flg, 0, split ? KS * (int)sizeof(int) : 0, 0x00020000);
    // the spectrum window of split mode (see sst): patch-sized descriptor
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc(split ? st.spec + (size_t)b * L * L : nullptr, 0,
                                          split ? L * L * (int)sizeof(float2) : 0, 0x00020000);
    if (split) {
        if (tid == 0) {
            const int mine = xcc_id() + 1;
            __hip_atomic_store(xccs + hown, mine, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            bool same = true;
#pragma unroll
            for (int p = 0; p < KS; ++p) {
                if (p == hown) continue;
                int other = 0;
                for (int spins = 0; (other = __hip_atomic_load(xccs + p, __ATOMIC_RELAXED,
                                                               __HIP_MEMORY_SCOPE_AGENT)) == 0; ++spins) {
                    if (spins > (1 << 23) ||
                        __hip_atomic_load(a.abort_flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
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
        __syncthreads();  // ccnt[1] is reused by handoff_wait
    }
    // exchange-area and partner-visible spectrum accesses of split mode
    // Exchange-area accesses go through buffer instructions: one per-lane VGPR
    // offset (the lane's 8-byte slot) plus the slot's compile-time byte offset
    // in the SGPR soffset, so no 64-bit address per slot is kept live (with
    // plain pointers the 13 P stores had their addresses spilled to scratch,
    // each store paying a reload and a vmcnt(0): 9k cycles per LED).
    // cache policy: sc1 (16) when the partner is on another XCD; loads are
    // volatile (bit 31) and bypass the L1 (sc1) when it shares this one.
    typedef unsigned u32x2_t __attribute__((ext_vector_type(2)));
    const int lane_off = tid * (int)sizeof(float2);
    auto xst = [&](int slot, float2 v) {  // slot: the lane-independent part of the index
        const u32x2_t d = __builtin_bit_cast(u32x2_t, v);
        if (local) __builtin_amdgcn_raw_buffer_store_b64(d, rx, lane_off, slot * (int)sizeof(float2), 0);
        else __builtin_amdgcn_raw_buffer_store_b64(d, rx, lane_off, slot * (int)sizeof(float2), 16);
    };
    auto xld = [&](int slot) {
        return __builtin_bit_cast(
            float2, local ? __builtin_amdgcn_raw_buffer_load_b64(rx, lane_off, slot * (int)sizeof(float2), kAuxL2Volatile)
                          : __builtin_amdgcn_raw_buffer_load_b64(rx, lane_off, slot * (int)sizeof(float2),
                                                                 (int)(16u | (1u << 31))));
    };
    // spectrum stores: in split mode every part runs the identical update and
    // writes identical values, and each reads back only its own writes (the
    // next window, the dirty-tile re-scan).  Parts that share an XCD share its
    // L2, so plain stores serve them.  Parts on different XCDs store with the
    // device-scope (sc1) policy: a dirty line a lagging partner left in ITS
    // L2 could otherwise be written back over this part's newer value after
    // this part's own line was evicted, and a later miss would read it stale;
    // sc1 stores reach memory before the flag that orders the next LED.
    auto sst = [&](float2 *p, float2 v) {
        if (split && !local) {
            const int off = (int)((p - (st.spec + (size_t)b * L * L)) * (int)sizeof(float2));
            __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2_t, v), rs, off, 0, 16);
        } else {
            *p = v;
        }
    };
    const float epsn = st.eps * (float)(NP * NP);  // eps on the unscaled IDFT
    const float epsn_im = st.eps_im * (float)(NP * NP);
    __syncthreads();

    // diagnostic: shader-clock cycles per phase, summed over LEDs (wave-uniform)
    unsigned long long acc[kStamps] = {};  // phases: see api.cpp stamp names
    unsigned long long prev = a.dbg ? __builtin_amdgcn_s_memtime() : 0ull;
#define FPM_STAMP(i)                                                  \
    if (a.dbg) {                                                      \
        const unsigned long long now_ = __builtin_amdgcn_s_memtime(); \
        acc[i] += now_ - prev;                                        \
        prev = now_;                                                  \
    }
    // O (pre-update Objfcrop on the support, fpmMain.cpp:358-362) is never
    // held in registers through pass B: Opre is loaded at the start of pass C
    // for the second half's pass A and the object update, and right after the
    // object update for the next LED's first pass A.
    auto window = [&](int itn) {
        const LedPos p = lt.at(itn);
        return spec + (unsigned)(p.yc * L + p.xc);
    };
    // slot s of row j sits at a compile-time offset from the lane's row base
    // (kx = t + 16 SK[s] - Np [s >= 3]), so one base register serves all six
    auto soff = [](int s) { return 16 * fz::SK[s] - (s >= 3 ? fz::NP : 0); };
    auto ldO = [&](const float2 *sr, int j, int s) {
        const float2 *lr = sr + (kyr[j] * L + t);
        return ((inmask[j] >> s) & 1) ? lr[soff(s)] : make_float2(0.f, 0.f);
    };
    float2 Opre[RPG][6];
    if (a.n_order > 0) {
        const float2 *sr = window(0);
#pragma unroll
        for (int j = 0; j < RPG; ++j)
#pragma unroll
            for (int s = 0; s < 6; ++s) Opre[j][s] = ldO(sr, j, s);
        if (towner) Ot = sr[tp.x * L + tp.y];
    }
    for (int it = 0; it < a.n_order; ++it) {
        const LedPos lp = lt.at(it);
        const int led = lp.led, xc = lp.xc, yc = lp.yc;
        float2 *srow = spec + (unsigned)(yc * L + xc);   // spec[yc + ky][xc + kx] = srow[ky*L + kx]
        const uint16_t *Ib = a.meas + ((size_t)led * st.B + b) * NP * NP;

        // ---- gather the sub-aperture on the support (pre-update Objfcrop,
        // fpmMain.cpp:358-362); the tail pixels' O was loaded with Opre
        if (towner) tailX[tid] = pout(pmul(pin(Ot), pin(Pt)));
        __syncthreads();  // tailX
        FPM_STAMP(0)

        float2 v[16], r[16];
        float2 F[RPG][6];  // row-DFT outputs; complete after the second half
        bool aborted = false;
#pragma unroll 1
        for (int h = hb; h < he; ++h) {
            // this lane's four-step twiddles W256^{m t}, m = 0..15 (Tw)
            Tw wt;
            wt.load(tw2, t);
            // measurement I[t + 16 m2][x] for this lane's pass-B columns,
            // loaded at the top of each pass-B round (one round ahead measured
            // 5 % slower: 16 VGPRs the scheduler needs)
            // pass B works on 32 column blocks per half: block r8 gives group gg
            // of a wave column (r8 & 15) + 16 gg + 64 (r8 >> 4)
            constexpr int NBLK = TH / 4;
            auto colx = [&](int r8) { return (r8 & 15) + 16 * gg + 64 * (r8 >> 4); };
            // the lane's 16 uint16 pixels of column x: 32 contiguous bytes
            auto ldI = [&](int xl, uint4 (&n)[2]) {
                const uint4 *ip = (const uint4 *)(Ib + ((xl + TH * h) * 16 + t) * 16);
#pragma unroll
                for (int i = 0; i < 2; ++i) n[i] = ld_stream(ip + i);
            };
            // ---- A: row IDFTs of the box rows, columns [128h, 128h+128) kept
            float2 X[RPG][6];
#pragma unroll
            for (int j = 0; j < RPG; ++j)
#pragma unroll
                for (int s = 0; s < 6; ++s) X[j][s] = pout(pmul(pin(Opre[j][s]), pin(P[j][s])));   // :364
#pragma unroll
            for (int j = 0; j < RPG; ++j) {
                if (!ron[j]) continue;
#pragma unroll
                for (int k = 0; k < 16; ++k) v[k] = make_float2(0.f, 0.f);
#pragma unroll
                for (int s = 0; s < 6; ++s) v[SK[s]] = X[j][s];
                idft256_in6(v, r, scr, wt, t, xrd);
                // keep the column part h: row[16 m'] = r[h MPP + m'] (one branch
                // per part keeps every register index static; a shared helper
                // made the compiler select between addresses of r and put r
                // in scratch)
                float2 *row = th + (g + NG * j) * TLD + t;
                if constexpr (NPARTS == 2) {
                    if (h == 0) {
#pragma unroll
                        for (int m = 0; m < 8; ++m) row[16 * m] = r[m];
                    } else {
#pragma unroll
                        for (int m = 0; m < 8; ++m) row[16 * m] = r[8 + m];
                    }
                } else {
                    if (h == 0) {
#pragma unroll
                        for (int m = 0; m < 4; ++m) row[16 * m] = r[m];
                    } else if (h == 1) {
#pragma unroll
                        for (int m = 0; m < 4; ++m) row[16 * m] = r[4 + m];
                    } else if (h == 2) {
#pragma unroll
                        for (int m = 0; m < 4; ++m) row[16 * m] = r[8 + m];
                    } else {
#pragma unroll
                        for (int m = 0; m < 4; ++m) row[16 * m] = r[12 + m];
                    }
                }
            }
            FPM_STAMP(7)
            // tail rows: direct sums, on the first half of the waves only (the
            // VALU arbiter favours them, so they finish their rows first)
            for (int idx = tid; tid < NT / 2 && idx < a.n_tail_rows * TH; idx += NT / 2) {
                // q is wave-uniform (TH = 1 or 2 waves): the row's pixel range comes
                // from scalar loads; kx runs over a contiguous range, so the
                // twiddle index advances by x per term
                const int q = idx / TH, xl = idx - q * TH, x = xl + TH * h;
                const int p0 = a.tail_row_p0[q], np_ = a.tail_row_np[q];
                // twiddle W^{-x kx} by recurrence from two table values: a
                // per-term table read with lane-dependent x conflicts on LDS banks
                // (even and odd terms on two chains)
                // (wa, wb hold W^{+x kx}; pmulc applies the conjugate)
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
                th[(NROWS + q) * TLD + xl] = pout(s2 + s3);
            }
            if (tid == 0) *ccnt = NW;  // pass-B block counter (blocks 0..NW-1 are preassigned)
            __syncthreads();  // half-T complete
            FPM_STAMP(1)

            // ---- B: columns x in [128h, 128h+128): IDFT, amplitude replacement, DFT (:365-394)
            // Column blocks are claimed dynamically (NT 512): wave w starts with
            // block w and takes the next unclaimed block from an LDS counter.  At
            // two waves per SIMD the VALU arbiter favours the older wave of each
            // pair by thousands of cycles over a pass; with a static split the
            // younger wave then finished its share alone at half the SIMD's issue
            // rate while the older one waited at the barrier (stamps: 29.8k vs
            // 44.3k cycles per LED).  The claim for the next block is issued at
            // the top of a round and consumed after the inverse transform.
            float2 tin[6];  // the column's six half-T slots, read one round ahead
#pragma unroll
            for (int s = 0; s < 6; ++s) tin[s] = th[roff[s] + colx(w)];
            int r8 = w;
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
                    // next block's T slots; unconditional (the last round
                    // re-reads its own column) so the loads are not sunk into
                    // a branch
                    const int xn = colx(nx < NBLK ? nx : r8);
#pragma unroll
                    for (int s = 0; s < 6; ++s) tin[s] = th[roff[s] + xn];
                }
                const unsigned iw[8] = {cI[0].x, cI[0].y, cI[0].z, cI[0].w, cI[1].x, cI[1].y, cI[1].z, cI[1].w};
#pragma unroll
                for (int m2 = 0; m2 < 16; ++m2) {
                    const float Iv = (float)((m2 & 1) ? (iw[m2 >> 1] >> 16) : (iw[m2 >> 1] & 0xffffu));
                    // psi = r/Np^2 (:365); sqrt(I) psi/|psi + eps| = r / sqrt(|r + eps Np^2|^2 / I)
                    // (cv::add(UMat c2, double) puts eps on both channels, :390); I = 0 gives
                    // 1/I = +inf and a zero scale, the reference's sqrt(0) factor
                    const pf2 tt = pin(r[m2]) + (pf2){epsn, epsn_im};
                    const float mag2 = __builtin_fmaf(tt.x, tt.x, tt.y * tt.y);
                    const float sc = amp_scale(mag2, Iv);
                    v[m2] = pout(pin(r[m2]) * sc);
                }
                float2 o[6];
                dft256_out6(v, o, scr, wt, t, xrd);
#pragma unroll
                for (int s = 0; s < 6; ++s) th[roff[s] + (roff[s] == zoff ? TLD : 0) + xl] = o[s];
                if (nx >= NBLK) break;
                r8 = nx;
            }
            FPM_STAMP(10)  // this wave's own columns done
            __syncthreads();
            FPM_STAMP(2)

            // ---- C: this half's share of the pruned row DFTs (:394)
#pragma unroll
            for (int j = 0; j < RPG; ++j)
#pragma unroll
                for (int s = 0; s < 6; ++s) Opre[j][s] = ldO(srow, j, s);
#pragma unroll
            for (int j = 0; j < RPG; ++j) {
                if (!ron[j]) {
#pragma unroll
                    for (int s = 0; s < 6; ++s) F[j][s] = make_float2(0.f, 0.f);
                    continue;
                }
                float2 o[6];
                row_dft_part<NPARTS>(th + (g + NG * j) * TLD + t, v, o, scr, wt, t, xrd, h);
#pragma unroll
                for (int s = 0; s < 6; ++s) F[j][s] = h == hb ? o[s] : cadd(F[j][s], o[s]);
            }
            FPM_STAMP(8)
            // tail pixels: 16 lanes sum the part's TH terms; first half of the waves only
            for (int pp = g; g < NG / 2 && pp < a.n_tail_px; pp += NG / 2) {
                const int2 px = tpx[pp];
                const float2 *row = th + sig[px.x + KYOFF] * TLD;
                // W^{x kx} for x = t + 16 m + TH h by recurrence over m (two
                // table reads instead of eight bank-conflicting ones)
                pf2 s2p = {0.f, 0.f};
                pf2 wk = pin(tw[((t + TH * h) * (px.y + NP)) & (NP - 1)]);
                const pf2 wstep = pin(tw[(16 * (px.y + NP)) & (NP - 1)]);
#pragma unroll
                for (int m = 0; m < TH / 16; ++m) {
                    s2p += pmul(pin(row[t + 16 * m]), wk);
                    if (m < TH / 16 - 1) wk = pmul(wk, wstep);
                }
                float2 s2 = pout(s2p);
                s2.x = row16_sum(s2.x);  // the group's 16 lanes (DPP, bit-identical to the xor butterfly)
                s2.y = row16_sum(s2.y);
                if (t == 0) tailF[pp] = h != hb ? cadd(tailF[pp], s2) : s2;
            }
            __syncthreads();  // half-T reusable; tailF
            FPM_STAMP(3)
        }
        if (split) {
            // symmetric handoff: publish this part's F partials, take the
            // partners', and every part runs the same update (bit-identical
            // across the parts: each sums ((F_0 + F_1) + F_2) + F_3 in part
            // order, its own partial from registers); one handoff per LED, and
            // no part waits for another's update.  KS = 2 matches the
            // one-workgroup kernel bit for bit (it forms F_0 + F_1 the same way).
            const int par = it & 1;
            const int mine = (hown * 2 + par) * kXchHalf;
            if (it < a.stall_led || a.stall_led < 0 || hown != KS - 1) {
                // F only matters on the support: the partner loads the
                // support slots only, so only those are published (the box
                // slots off the disk are 47 % of them at r 33)
#pragma unroll
                for (int j = 0; j < RPG; ++j)
#pragma unroll
                    for (int s = 0; s < 6; ++s)
                        if ((inmask[j] >> s) & 1) xst(mine + (j * 6 + s) * NT, F[j][s]);
                if (tid < a.n_tail_px) xst(mine + kXchTF, tailF[tid]);
                FPM_STAMP(11)
                handoff_publish(flg + hown, it + 1, local);
            }
            if (!handoff_wait<KS>(flg, hown, it + 1, a.abort_flag, ccnt + 1, local, rf)) {
                aborted = true;
                break;
            }
            FPM_STAMP(12)
            // every partner partial is loaded before the first is used (one
            // L2 round trip for all of them); F only matters on the support
            float2 ox[KS > 1 ? KS - 1 : 1][RPG][6];
#pragma unroll
            for (int q = 0; q < KS - 1; ++q) {
                const int pp = q < hown ? q : q + 1;  // partner part (block-uniform)
                const int base = (pp * 2 + par) * kXchHalf;
#pragma unroll
                for (int j = 0; j < RPG; ++j)
#pragma unroll
                    for (int s = 0; s < 6; ++s) {
                        const bool in = (inmask[j] >> s) & 1;
                        ox[q][j][s] = in ? xld(base + (j * 6 + s) * NT) : make_float2(0.f, 0.f);
                    }
            }
#pragma unroll
            for (int j = 0; j < RPG; ++j)
#pragma unroll
                for (int s = 0; s < 6; ++s) {
                    float2 acc = make_float2(0.f, 0.f);
#pragma unroll
                    for (int p = 0; p < KS; ++p) {
                        // part p's partial: own registers, or partner slot p (p < hown) / p - 1
                        const float2 lo = ox[p < KS - 1 ? p : KS - 2][j][s], hi = ox[p > 0 ? p - 1 : 0][j][s];
                        const float2 o = p == hown ? F[j][s] : p < hown ? lo : hi;
                        acc = p == 0 ? o : cadd(acc, o);
                    }
                    F[j][s] = acc;
                }
            if (tid < a.n_tail_px) {
                float2 acc = make_float2(0.f, 0.f);
#pragma unroll
                for (int p = 0; p < KS; ++p) {
                    const float2 o = p == hown ? tailF[tid] : xld(((p * 2 + par) * kXchHalf) + kXchTF);
                    acc = p == 0 ? o : cadd(acc, o);
                }
                tailF[tid] = acc;
            }
        }

        // ---- object update on the support (:405-447) and pupil numerator (:457-464).
        // Tile maxima stay exact incrementally: a changed pixel raises its
        // tile max (LDS atomic max on the float bits); a tile whose maximum
        // pixel decreased is marked dirty (its value becomes an upper bound).
        unsigned *tmu = (unsigned *)tmx;
        // The atomic max is issued only when the new value exceeds the tile
        // maximum this lane read: tmu only grows, so a skipped max was never
        // needed (64 lanes of a wave hit 2-4 tile words, and an unfiltered
        // LDS atomic serialises them: 3.7k cycles per LED).
        auto note = [&](int py, int px, float ao, float an) {
            const int ti = ((py >> 4) - a.bty0) * a.nbx + ((px >> 4) - a.btx0);  // band tile
            const unsigned cur = tmu[ti];
            if (an < ao && cur <= __float_as_uint(ao)) atomicOr(&dirty[ti >> 5], 1u << (ti & 31));
            if (__float_as_uint(an) > cur) atomicMax(&tmu[ti], __float_as_uint(an));
        };
        if (it > 0) pm = pm_of_red();  // the previous LED's pupil (:415)
        // Only support pixels are updated: outside the support O = P = 0 and the
        // numerator is exactly 0.  The mask is per lane, so a slot whose row
        // misses the disk in every lane of the wave is skipped whole (exec
        // zero): at r 33 the outer slots |kx| >= 32 of all rows |ky| > 8 and
        // |kx| >= 16 of the rows |ky| > 28, 27 of the 96 (wave, row, slot)
        // updates per LED.
#pragma unroll
        for (int j = 0; j < RPG; ++j)
#pragma unroll
            for (int s = 0; s < 6; ++s) {
                float2 num = make_float2(0.f, 0.f);
                if ((inmask[j] >> s) & 1) {
                    float oa;
                    const float2 nv = slot_update(F[j][s], Opre[j][s], P[j][s], pm, st, num, oa);
                    sst(srow + (kyr[j] * L + t) + soff(s), nv);  // read by a split partner
                    note(yc + kyr[j], xc + slot_kx(t, s), oa, cmag(nv));
                }
                // park the numerator in this group's own exchange tile (idle
                // until the next LED's pass A; 6 RPG 16 <= its 8 XP complex);
                // a T row is too narrow for it when the part is 64 columns
                scr[(j * 6 + s) * 16 + t] = num;
            }
        if (towner) {
            // D = Objfup - ObjfcropP with ObjfcropP = tailX (gathered O*P): pass F = tailF
            // and the slot helper recomputes O*P the same way the gather did
            float oa;
            const float2 nv = slot_update(tailF[tid], Ot, Pt, pm, st, NPt, oa);
            sst(srow + tp.x * L + tp.y, nv);
            note(yc + tp.x, xc + tp.y, oa, cmag(nv));
        }
        FPM_STAMP(9)
        __syncthreads();  // spectrum writes, tile maxima, dirty bits
        if (it + 1 < a.n_order) {
            const float2 *sr = window(it + 1);
#pragma unroll
            for (int j = 0; j < RPG; ++j)
#pragma unroll
                for (int s = 0; s < 6; ++s) Opre[j][s] = ldO(sr, j, s);
            if (towner) Ot = sr[tp.x * L + tp.y];
        }
        FPM_STAMP(4)

        // ---- exact max|objF| (:460,467): max over clean tiles; dirty tiles
        // only matter (and are re-read) when their bound exceeds that max
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
        if (dm > cm) {  // block-uniform: rare (bright-field LEDs, first LED of an iteration)
            for (int k = w; k < a.nbt; k += NW) {
                if (!((dirty[k >> 5] >> (k & 31)) & 1u) || !(tmx[k] > cm)) continue;  // wave-uniform
                const int ty = a.bty0 + band_dy(k), tx = a.btx0 + k - band_dy(k) * a.nbx;
                float2 e[4];  // all four loads before the first use (else one round trip each)
#pragma unroll
                for (int jj = 0; jj < 4; ++jj) {
                    const int pp = lane + 64 * jj;
                    e[jj] = spec[(unsigned)((ty * 16 + (pp >> 4)) * L + tx * 16 + (pp & 15))];
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
            __syncthreads();  // red[] reads above are done
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
        for (int j = 0; j < RPG; ++j)
#pragma unroll
            for (int s = 0; s < 6; ++s) {
                const float2 n = scr[(j * 6 + s) * 16 + t];
                P[j][s] = make_float2(P[j][s].x + n.x * rom, P[j][s].y + n.y * rom);
                pmx = fmaxf(pmx, cabs2(P[j][s]));
            }
        if (towner) {
            Pt = make_float2(Pt.x + NPt.x * rom, Pt.y + NPt.y * rom);
            pmx = fmaxf(pmx, cabs2(Pt));
        }
        // red[32..47] is not used by the max phase, so no barrier is needed
        // before writing it; nothing read below is rewritten by another
        // thread before the next LED's first barrier (numerators sit in this
        // thread's own exchange-tile slots, tailX was last read in pass A).
        // max|P| is first needed by the next LED's object update, several
        // barriers later: it is reduced there (pm_of_red), not behind a
        // barrier of its own here.
        pmx = wave_max_nonneg(pmx);
        if (lane == 0) red[32 + w] = pmx;
        pupil_done = true;
        FPM_STAMP(6)
        (void)aborted;
    }
#undef FPM_STAMP
    __syncthreads();  // the last LED's red[32..]
    probe.stop(a.st.clk);
    if (pupil_done) pm = pm_of_red();
    // stamps of the first and the last wave (the barrier waits show who is slow)
    // (split mode: the first wave of the first and of the last part's workgroup)
    if (a.dbg && (split ? (tid == 0 && (hown == 0 || hown == KS - 1)) : (tid == 0 || tid == NT - 64)))
        for (int i = 0; i < kStamps; ++i) atomicAdd(&a.dbg[((split ? hown : tid) ? kStamps : 0) + i], acc[i]);
    if (hown > 0) return;  // the first part's workgroup owns the per-patch state

    // ---- write back the per-patch state
#pragma unroll
    for (int j = 0; j < RPG; ++j)
#pragma unroll
        for (int s = 0; s < 6; ++s)
            if ((inmask[j] >> s) & 1) pup[(kyr[j] + R) * NB + slot_kx(t, s) + R] = P[j][s];
    if (towner) pup[(tp.x + R) * NB + tp.y + R] = Pt;
    for (int k = tid; k < a.nbt; k += NT) tmax_g[band_gtile(k)] = tmx[k];
    for (int i = tid; i < nwords; i += NT) dirty_g[i] = dirty[i];
    if (tid == 0) st.pmax[b] = pm;
}

// ------------------------------------------------------------------ host side
namespace {
size_t fused_lds_bytes(int ks, int nbt, int n_tail_rows) {
    const int tld = part_cols(ks) + 1;
    return (size_t)(32 * XTILE + (fz::NROWS + n_tail_rows + 2) * tld + 512 + 2 * fz::MAXTAIL) * sizeof(float2) +
           48 * sizeof(float) + 96 * sizeof(int) + fz::MAXTAIL * sizeof(int2) + fz::MAXTAILROWS * sizeof(int) +
           (size_t)nbt * sizeof(float) + (size_t)(nbt + 31) / 32 * sizeof(unsigned) + 2 * sizeof(int);
}

}  // namespace

// Threads per workgroup of the fused kernel for this geometry: 512 (2 waves
// per SIMD), or 0 when its LDS does not fit (fused path unsupported).
int fused_threads(int np, int r, int L, const DevState &st) {
    const FusedGeom g = fused_geometry(np, r);
    if (!g.ok || L % kTile != 0) return 0;
    if (st.sy0 < 0 || st.sy1 >= L || st.sy0 > st.sy1 || st.sx0 < 0 || st.sx1 >= L || st.sx0 > st.sx1) return 0;
    const Band bd = band_of(st);
    return fused_lds_bytes(1, bd.nbt, g.n_tail_rows) <= 160 * 1024 ? 512 : 0;
}

size_t fused_T_elems(int, int, int) { return 1; }  // the intermediate lives in LDS

// split mode: exchange-area elements and flag words for B patches on KS parts
size_t fused_xch_elems(int B, int ks) { return (size_t)B * xch_patch_elems(ks); }
size_t fused_flag_words(int B, int ks) { return 2 * (size_t)ks * B + 1; }

// Workgroups per patch of the Np 256 fused kernel (split mode, section 4.1b of
// DESIGN.md).  Splitting pays off when one workgroup per patch would leave
// CUs idle (BASELINE config 4: 1024 patches over 8 GPUs = 128 per GPU; a
// 256-patch field strong-scaled over 4 / 8 GPUs: 64 / 32 per GPU) and needs
// every block co-resident (the parts wait on each other; launch_coresident
// checks the grid against the occupancy query): KS = 4 when 4 B <= CUs, KS = 2
// when 2 B <= CUs, else 1.  FPM_NO_SPLIT=1 disables it; FPM_SPLIT=1/2/4 forces
// a part count where the grid still fits.
int fused_split_parts(int nt, int B, int n_cu) {
    if (nt != 512 || B < 1 || getenv("FPM_NO_SPLIT")) return 1;
    auto fits = [&](int ks) { return 8 * ks * ((B + 7) / 8) <= n_cu; };
    if (const char *e = getenv("FPM_SPLIT")) {
        const int ks = atoi(e);
        return (ks == 2 || ks == 4) && fits(ks) ? ks : 1;
    }
    return fits(4) ? 4 : fits(2) ? 2 : 1;
}

hipError_t launch_fused_iteration(const DevState &st, const uint16_t *meas, const int *order_dev,
                                  const int *x0_dev, const int *y0_dev, int n_order, const float2 *tw_np,
                                  int ks, unsigned long long *dbg, float2 *xch, int *flags, int stall_led,
                                  hipStream_t s) {
    const FusedGeom g = fused_geometry(st.np, st.r);
    if (!g.ok) return hipErrorInvalidValue;
    if (ks != 1 && ((ks != 2 && ks != 4) || !xch || !flags)) return hipErrorInvalidValue;
    if (st.sy0 < 0 || st.sy1 >= st.L || st.sy0 > st.sy1 || st.sx0 < 0 || st.sx1 >= st.L || st.sx0 > st.sx1)
        return hipErrorInvalidValue;
    FusedArgs a;
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
    a.xch = ks > 1 ? xch : nullptr;
    a.flags = ks > 1 ? flags : nullptr;
    a.abort_flag = ks > 1 ? flags + ks * st.B : nullptr;
    a.stall_led = ks > 1 ? stall_led : -1;
    const size_t lds0 = fused_lds_bytes(ks, a.nbt, g.n_tail_rows);
    if (lds0 > 160 * 1024) return hipErrorInvalidValue;
    size_t lds;  // + the LED table when it fits
    a.ledtab_off = ledtab_offset(lds0, n_order, st.L, 160 * 1024, lds);
    const void *fn = ks == 4   ? (const void *)k_fused_iteration<512, 4>
                     : ks == 2 ? (const void *)k_fused_iteration<512, 2>
                               : (const void *)k_fused_iteration<512, 1>;
    hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
    if (ks > 1) {
        // flags count LEDs of this launch and XCC ids are re-learnt: both start
        // from zero; the abort word between them is sticky (fpm_run reads and
        // clears it, so a timeout in any iteration of a multi-iteration run
        // is reported, and every later launch leaves at once)
        e = hipMemsetAsync(flags, 0, (size_t)ks * st.B * sizeof(int), s);
        if (e == hipSuccess) e = hipMemsetAsync(flags + ks * st.B + 1, 0, (size_t)ks * st.B * sizeof(int), s);
        if (e != hipSuccess) return e;
        return launch_coresident(fn, 8 * ks * ((st.B + 7) / 8), 512, lds, &a, s);
    }
    hipLaunchKernelGGL((k_fused_iteration<512, 1>), dim3(st.B), dim3(512), lds, s, a);
    return hipGetLastError();
}

}  // namespace fpm
