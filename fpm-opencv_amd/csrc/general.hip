// general.hip -- the general (any Np = 2^a 3^b 5^c, any pupil radius) path of
// the per-LED update, fpmMain.cpp:348-476, as four batched kernels per LED
// step.  Every launch covers all B patches of the context.
//
//   K1 k_gather_rowifft   sub-aperture gather x pupil, row IDFTs over the
//                         support box rows          (fpmMain.cpp:358-365)
//   K2 k_colpass          column IDFT, amplitude replacement, column DFT,
//                         only the box rows kept   (fpmMain.cpp:365-394)
//   K3 k_rowfft_update    row DFT of the box rows, object update written to
//                         the centred spectrum, pupil-update numerator
//                                                   (fpmMain.cpp:394-447,457-464)
//   K4 k_tile_rows        tile maxima of |spec| under the ROI and the maxima
//                         of those tile rows                (fpmMain.cpp:460,467)
//   K5 k_pupil_commit     exact max|objF| from the row maxima, P += num/max * S
//                         on a slice of the support box, partial max|P| for
//                         the next LED                       (fpmMain.cpp:459-475,415)
// K4 and K5 spread one patch over many workgroups, so a context with a few
// large patches (config 5: Np 1024, L 4096) still fills the chip.
//
// Pruning: P vanishes outside the support disk, so the inverse transform has
// nonzero input only on the (2r+1)^2 box and only the box outputs of the
// forward transform are ever used.  Row passes therefore run on nb = 2r+1 rows,
// not Np.
#include <algorithm>
#include <cstdlib>

#include "fft_lds.hpp"
#include "fpm_state.hpp"

namespace fpm {

// ---- K1 ---------------------------------------------------------------------
// grid (nb, B), block 256, LDS 2*Np float2
__global__ void __launch_bounds__(256) k_gather_rowifft(DevState st, StepArgs sa, FftPlan pl,
                                                        const float2 *__restrict__ tw) {
    extern __shared__ __attribute__((aligned(16))) float2 smem[];
    const int np = st.np, r = st.r, nb = st.nb;
    const int row = blockIdx.x, b = blockIdx.y;
    const int ky = row - r;
    float2 *bufa = smem, *bufb = smem + np;
    const float2 *pup = st.pupil + (size_t)b * nb * nb;
    for (int i = threadIdx.x; i < np; i += blockDim.x) bufa[i] = make_float2(0.f, 0.f);
    __syncthreads();
    const int yrow = sa.yc + ky;
    for (int j = threadIdx.x; j < nb; j += blockDim.x) {
        if (st.disk[row * nb + j]) {
            const int kx = j - r;
            float2 o = spec_ld(st, b, (size_t)yrow * st.L + sa.xc + kx);
            float2 p = pup[row * nb + j];
            bufa[(kx + np) % np] = cmul(o, p);
        }
    }
    __syncthreads();
    float2 *res = stockham<true>(bufa, bufb, 1, pl, tw, threadIdx.x, blockDim.x);
    float2 *T = st.T + ((size_t)b * nb + row) * np;
    for (int i = threadIdx.x; i < np; i += blockDim.x) T[i] = res[i];
}

// ---- K2 ---------------------------------------------------------------------
// grid (Np, B), block 256, LDS 2*Np float2. One column per block.
__global__ void __launch_bounds__(256) k_colpass(DevState st, StepArgs sa, FftPlan pl,
                                                 const float2 *__restrict__ tw) {
    extern __shared__ __attribute__((aligned(16))) float2 smem[];
    const int np = st.np, r = st.r, nb = st.nb;
    const int x = blockIdx.x, b = blockIdx.y;
    float2 *bufa = smem, *bufb = smem + np;
    float2 *T = st.T + (size_t)b * nb * np;
    for (int i = threadIdx.x; i < np; i += blockDim.x) bufa[i] = make_float2(0.f, 0.f);
    __syncthreads();
    for (int j = threadIdx.x; j < nb; j += blockDim.x) bufa[(j - r + np) % np] = T[(size_t)j * np + x];
    __syncthreads();
    float2 *res = stockham<true>(bufa, bufb, 1, pl, tw, threadIdx.x, blockDim.x);
    float2 *oth = (res == bufa) ? bufb : bufa;
    // amplitude replacement, fpmMain.cpp:378-393:
    //   psi = ifft2(.) (1/Np^2 scale), psi' = sqrt(I) * psi / |psi + eps| (eps on Re and Im)
    const float inv_n2 = 1.0f / ((float)np * (float)np);
    const uint16_t *I = st.meas + ((size_t)sa.led * st.mB + b) * np * np;
    for (int y = threadIdx.x; y < np; y += blockDim.x) {
        float2 psi = cscale(res[y], inv_n2);
        float a = sqrtf((float)I[(size_t)y * np + x]);
        float tre = psi.x + st.eps, tim = psi.y + st.eps_im;
        float mag = sqrtf(tre * tre + tim * tim);
        float s = a / mag;
        res[y] = make_float2(psi.x * s, psi.y * s);
    }
    __syncthreads();
    res = stockham<false>(res, oth, 1, pl, tw, threadIdx.x, blockDim.x);
    for (int j = threadIdx.x; j < nb; j += blockDim.x) T[(size_t)j * np + x] = res[(j - r + np) % np];
}

// ---- K3 ---------------------------------------------------------------------
// grid (nb, B), block 256, LDS 2*Np float2
__global__ void __launch_bounds__(256) k_rowfft_update(DevState st, StepArgs sa, FftPlan pl,
                                                       const float2 *__restrict__ tw) {
    extern __shared__ __attribute__((aligned(16))) float2 smem[];
    const int np = st.np, r = st.r, nb = st.nb;
    const int row = blockIdx.x, b = blockIdx.y;
    const int ky = row - r;
    float2 *bufa = smem, *bufb = smem + np;
    const float2 *T = st.T + ((size_t)b * nb + row) * np;
    for (int i = threadIdx.x; i < np; i += blockDim.x) bufa[i] = T[i];
    __syncthreads();
    float2 *res = stockham<false>(bufa, bufb, 1, pl, tw, threadIdx.x, blockDim.x);
    float2 *pup = st.pupil + (size_t)b * nb * nb;
    float2 *dP = st.dP + (size_t)b * nb * nb;
    // max|P| of the previous commit: the block reads the npart partial maxima
    // in parallel (a serial scalar-load chain cost ~30 us at npart ~ 100)
    __shared__ float red[4];
    float pm = 0.f;
    for (int i = threadIdx.x; i < st.npart; i += blockDim.x) pm = fmaxf(pm, st.pmax[b * st.npart + i]);
    pm = block_max_nonneg(pm, red);
    const int yrow = sa.yc + ky;
    for (int j = threadIdx.x; j < nb; j += blockDim.x) {
        if (!st.disk[row * nb + j]) continue;
        const int kx = j - r;
        const size_t si = (size_t)yrow * st.L + sa.xc + kx;
        const float2 o = spec_ld(st, b, si);     // pre-update Objfcrop (:361)
        const float2 p = pup[row * nb + j];
        const float2 F = res[(kx + np) % np];    // Objfup (:394)
        const float2 D = csub(F, cmul(o, p));    // Objfup - ObjfcropP (:409,463)
        // object update (:406-419,433): D |P| P* / ((|P|^2 + d2) max|P|)
        const float pa = cmag(p);
        const float2 dpc = cmul(cmul(D, cscale(cconj(p), pa)), upd_coef_div(pa * pa + st.delta2, st.d2_im, pm));
        spec_st(st, b, si, cadd(o, dpc));
        // pupil numerator (:459-464,469): D |O| O* / (|O|^2 + d1); max|objF| in K4
        const float oa = cmag(o);
        dP[row * nb + j] = cmul(cmul(D, cscale(cconj(o), oa)), upd_coef_div(oa * oa + st.delta1, st.d1_im, 1.0f));
    }
}

// ---- K4 ---------------------------------------------------------------------
// grid (ROI tile rows, B), block 256 or 1024: one tile row of the ROI box per block.
// Each wave refreshes whole 16x16 tiles (4 pixels per lane, no barrier),
// issuing every load of its tiles before the first reduction; the row's other
// (unchanged) tile maxima are loaded first and folded in with one block max.
// Block size: one wave per ROI tile column up to 16 waves (1024 threads for
// config 5's 42-tile rows; 256 for config 3's 4-5 tiles, where 16 mostly
// idle waves per block only added latency).
template <int kRowThreads>
__global__ void __launch_bounds__(kRowThreads) k_tile_rows(DevState st, StepArgs sa) {
    constexpr int NW = kRowThreads / 64, MT = 5;  // tiles a wave refreshes at once
    __shared__ float red[NW];
    const int r = st.r, L = st.L, ntx = st.ntx;
    const int b = blockIdx.y;
    const int ty = (sa.yc - r) / kTile + blockIdx.x;
    const int tx0 = (sa.xc - r) / kTile, tx1 = (sa.xc + r) / kTile;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    float *tmax = st.tmax + (size_t)b * st.nty * ntx + (size_t)ty * ntx;
    // the row's unchanged tile maxima first: their loads overlap the refresh
    float mx = 0.f;
    for (int tx = threadIdx.x; tx < ntx; tx += kRowThreads)
        if (tx < tx0 || tx > tx1) mx = fmaxf(mx, tmax[tx]);
    // the ROI tiles: every load of a wave's (up to MT) tiles before the first
    // reduction -- one memory latency instead of one per tile
    // (unconditional loads of clamped in-bounds pixels, masked after all of
    // them: a masked spec_ld, widening fp16 where it loaded, waited for each
    // of its loads in turn -- 20 memory round trips per wave)
    auto pix = [&](int base, int i, int j, bool &ok) {  // pixel j of tile i: its index, ok = inside the ROI row
        const int tx = base + i * NW, p = lane + 64 * j;
        const int y = ty * kTile + (p >> 4), x = min(tx, tx1) * kTile + (p & 15);
        ok = tx <= tx1 && y < L && x < L;
        return ok ? (size_t)y * L + x : (size_t)0;
    };
    for (int base = tx0 + w; base <= tx1; base += MT * NW) {
        float m[MT];
        if (st.spec16) {  // uniform
            const __half2 *sp = st.spec16 + (size_t)b * L * L;
            __half2 hv[MT][4];
            bool ok[MT][4];
#pragma unroll
            for (int i = 0; i < MT; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j) hv[i][j] = sp[pix(base, i, j, ok[i][j])];
#pragma unroll
            for (int i = 0; i < MT; ++i) {
                m[i] = 0.f;
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const float2 f = __half22float2(hv[i][j]);
                    const float a = cmag(make_float2(f.x * st.hinv, f.y * st.hinv));  // spec_ld's widening
                    m[i] = fmaxf(m[i], ok[i][j] ? a : 0.f);
                }
            }
        } else {
            const float2 *sp = st.spec + (size_t)b * L * L;
            float2 ov[MT][4];
            bool ok[MT][4];
#pragma unroll
            for (int i = 0; i < MT; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j) ov[i][j] = sp[pix(base, i, j, ok[i][j])];
#pragma unroll
            for (int i = 0; i < MT; ++i) {
                m[i] = 0.f;
#pragma unroll
                for (int j = 0; j < 4; ++j) m[i] = fmaxf(m[i], ok[i][j] ? cmag(ov[i][j]) : 0.f);
            }
        }
#pragma unroll
        for (int i = 0; i < MT; ++i) {
            const int tx = base + i * NW;
            if (tx > tx1) break;  // wave-uniform
            const float t = wave_max_nonneg(m[i]);
            if (lane == 0) tmax[tx] = t;
            mx = fmaxf(mx, t);
        }
    }
    mx = block_max_nonneg(mx, red);
    if (threadIdx.x == 0) st.rmax[(size_t)b * st.nty + ty] = mx;
}

// ---- K5 ---------------------------------------------------------------------
// grid (npart, B), block 256: global max|objF| (fpmMain.cpp:467) from the nty
// row maxima, then P += num / max * S (fpmMain.cpp:470-475) on this block's
// slice of the support box and its partial max|P| for the next LED (:415).
constexpr int kCommitThreads = 256;
constexpr int kCommitPx = 1024;  // support-box pixels per K5 block (a multiple of kCommitThreads)
__global__ void __launch_bounds__(kCommitThreads) k_pupil_commit(DevState st) {
    __shared__ float red[kCommitThreads / 64];
    const int nb = st.nb, b = blockIdx.y, part = blockIdx.x;
    const float *rmax = st.rmax + (size_t)b * st.nty;
    const int n = nb * nb, chunk = (n + st.npart - 1) / st.npart;
    const int i0 = part * chunk, i1 = min(n, i0 + chunk);
    float2 *pup = st.pupil + (size_t)b * nb * nb;
    const float2 *dP = st.dP + (size_t)b * nb * nb;
    // this thread's pixels (chunk <= kCommitPx) are loaded before the max
    // reduction, so their latency overlaps the rmax round trip
    constexpr int KP = kCommitPx / kCommitThreads;
    float2 pv[KP], dv[KP];
    bool on[KP];
#pragma unroll
    for (int k = 0; k < KP; ++k) {
        const int i = i0 + threadIdx.x + k * kCommitThreads;
        on[k] = i < i1 && st.disk[i];
        pv[k] = on[k] ? pup[i] : make_float2(0.f, 0.f);
        dv[k] = on[k] ? dP[i] : make_float2(0.f, 0.f);
    }
    float m = 0.f;
    for (int i = threadIdx.x; i < st.nty; i += kCommitThreads) m = fmaxf(m, rmax[i]);
    const float omax = block_max_nonneg(m, red);
    float pm = 0.f;
#pragma unroll
    for (int k = 0; k < KP; ++k) {
        if (!on[k]) continue;
        float2 p = pv[k];
        p.x += dv[k].x / omax;
        p.y += dv[k].y / omax;
        pup[i0 + threadIdx.x + k * kCommitThreads] = p;
        pm = fmaxf(pm, cmag(p));
    }
    pm = block_max_nonneg(pm, red);
    if (threadIdx.x == 0) st.pmax[b * st.npart + part] = pm;
}

int pupil_parts(int nb) { return std::max(1, (nb * nb + kCommitPx - 1) / kCommitPx); }

// ---- init / output kernels -------------------------------------------------

// Batched 1-D transforms of `nseq` sequences of length pl.n per patch.
// element i of sequence s of patch b:
//   in [b*in_bs + ((s+sroll)%nseq)*in_ss + ((i+iroll)%n)*in_es]
//   out[b*out_bs + s*out_ss + i*out_es] = scale * DFT(in)[i]
// A block owns C = 2^lc consecutive sequences.  When the sequences are
// columns (in_es != 1) consecutive threads read consecutive sequences, so a
// wave touches 16 rows x C*8 contiguous bytes; the LDS tile is then
// sequence-interleaved (lss 1, les C).  For rows it is row-major with one pad
// element per row (lss n+1, les 1) so the butterflies of C sequences hit
// distinct banks.  The transform runs IN PLACE over one LDS buffer: every pass
// lifts all of a thread's butterflies into registers, barriers, and stores
// (<= kFftRegElems complex values per thread), so C*n can reach
// kFftRegElems*blockDim without a ping-pong buffer.
constexpr int kFftThreads = 512;
constexpr int kFftRegElems = 24;
// complex values a radix-R in-place pass can lift into registers across the block
static int fft_pass_capacity(int R, int nt = kFftThreads, int e = kFftRegElems) { return e / R * R * nt; }

template <int R, bool INV, int NT = kFftThreads, int E = kFftRegElems>
__device__ __forceinline__ void fft_inplace_pass(float2 *buf, int n, int lc, int lss, int les, int Ns,
                                                 const float2 *__restrict__ tw) {
    constexpr int Q = E / R;
    const int nR = n / R, total = nR << lc, tmul = n / (Ns * R);
    const bool pow2 = (Ns & (Ns - 1)) == 0;
    const int lNs = 31 - __builtin_clz(Ns);
    const float rNs = 1.0f / (float)Ns;
    float2 v[Q][R];
    int dst[Q];
#pragma unroll
    for (int q = 0; q < Q; ++q) {
        const int jj = threadIdx.x + q * NT;
        if (jj < total) {
            const int sq = jj & ((1 << lc) - 1), j = jj >> lc;
            const float2 *src = buf + sq * lss;
#pragma unroll
            for (int r = 0; r < R; ++r) v[q][r] = src[(j + r * nR) * les];
            const int jq = pow2 ? (j >> lNs) : udiv(j, Ns, rNs);
            const int k = j - jq * Ns;
            if (Ns > 1) {
                const int ts = tmul * k;
#pragma unroll
                for (int r = 1; r < R; ++r) {
                    float2 w = tw[r * ts];
                    if (INV) w.y = -w.y;
                    v[q][r] = cmul(v[q][r], w);
                }
            }
            if (R == 2) dft2<INV>(v[q]);
            if (R == 3) dft3<INV>(v[q]);
            if (R == 4) dft4<INV>(v[q]);
            if (R == 5) dft5<INV>(v[q]);
            if (R == 8) dft8<INV>(v[q]);
            dst[q] = sq * lss + (jq * Ns * R + k) * les;
        }
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < Q; ++q) {
        const int jj = threadIdx.x + q * NT;
        if (jj < total) {
#pragma unroll
            for (int r = 0; r < R; ++r) buf[dst[q] + r * Ns * les] = v[q][r];
        }
    }
    __syncthreads();
}

// Input band of a batched transform: sequences gs outside [qlo, qhi] and
// elements gi with (gi + eroll) mod n outside [elo, ehi] are known to be
// exactly zero and are not read (objCrop over the spectrum's live band,
// fpm_state.hpp); the default covers everything.
struct FftBand {
    int qlo = 0, qhi = 0x7fffffff, elo = 0, ehi = 0x7fffffff, eroll = 0;
};

template <bool INV>
__global__ void __launch_bounds__(kFftThreads) k_fft_batch(const float2 *in, float2 *out, FftPlan pl,
                                                           const float2 *__restrict__ tw, int lc, int nseq,
                                                           size_t in_bs, int in_ss, int in_es, size_t out_bs,
                                                           int out_ss, int out_es, int sroll, int iroll,
                                                           float scale, const __half2 *in16, float in16_scale,
                                                           FftBand band) {
    extern __shared__ __attribute__((aligned(16))) float2 smem[];
    const int n = pl.n, C = 1 << lc, cm = C - 1;
    const int s0 = blockIdx.x << lc, b = blockIdx.y;
    const int cs = min(C, nseq - s0);
    const bool colmajor = in_es != 1;
    const int lss = colmajor ? 1 : n + 1, les = colmajor ? C : 1;
    const float rn = 1.0f / (float)n;
    in += (size_t)b * in_bs;
    if (in16) in16 += (size_t)b * in_bs;
    out += (size_t)b * out_bs;
    const int tot = n << lc;
    // twiddle table in LDS after the tile (a global read per butterfly put an
    // L1 round trip on every pass's critical path)
    float2 *stw = smem + (size_t)C * (n + 1);
    for (int i = threadIdx.x; i < n; i += kFftThreads) stw[i] = tw[i];
    // all of a thread's loads are issued before any LDS store so their
    // latencies overlap (a rolled loop waits for each one in turn)
    float2 v[kFftRegElems];
    int at[kFftRegElems];
#pragma unroll
    for (int q = 0; q < kFftRegElems; ++q) {
        const int idx = threadIdx.x + q * kFftThreads;
        v[q] = make_float2(0.f, 0.f);
        at[q] = -1;
        if (idx < tot) {
            int sq, i;
            if (colmajor) { sq = idx & cm; i = idx >> lc; }
            else { sq = udiv(idx, n, rn); i = idx - sq * n; }
            at[q] = sq * lss + i * les;
            int gs = s0 + sq + sroll, gi = i + iroll;
            if (gs >= nseq) gs -= nseq;
            if (gi >= n) gi -= n;
            int eb = gi + band.eroll;
            if (eb >= n) eb -= n;
            // outside the band the input is exactly zero: skip the load
            if (sq < cs && gs >= band.qlo && gs <= band.qhi && eb >= band.elo && eb <= band.ehi) {
                const size_t ii = (size_t)gs * in_ss + (size_t)gi * in_es;
                if (in16) {  // fp16-stored spectrum (config 5): widen, undo the storage scale
                    const float2 f = __half22float2(in16[ii]);
                    v[q] = make_float2(f.x * in16_scale, f.y * in16_scale);
                } else {
                    v[q] = in[ii];
                }
            }
        }
    }
#pragma unroll
    for (int q = 0; q < kFftRegElems; ++q)
        if (at[q] >= 0) smem[at[q]] = v[q];
    __syncthreads();
    int Ns = 1;
    for (int st = 0; st < pl.nstages; ++st) {
        const int R = pl.radix[st];
        switch (R) {
            case 8: fft_inplace_pass<8, INV>(smem, n, lc, lss, les, Ns, stw); break;
            case 4: fft_inplace_pass<4, INV>(smem, n, lc, lss, les, Ns, stw); break;
            case 2: fft_inplace_pass<2, INV>(smem, n, lc, lss, les, Ns, stw); break;
            case 3: fft_inplace_pass<3, INV>(smem, n, lc, lss, les, Ns, stw); break;
            default: fft_inplace_pass<5, INV>(smem, n, lc, lss, les, Ns, stw); break;
        }
        Ns *= R;
    }
    const bool ocol = out_es != 1;
    for (int idx = threadIdx.x; idx < tot; idx += kFftThreads) {
        int sq, i;
        if (ocol) { sq = idx & cm; i = idx >> lc; }
        else { sq = udiv(idx, n, rn); i = idx - sq * n; }
        if (sq < cs) out[(size_t)(s0 + sq) * out_ss + (size_t)i * out_es] = cscale(smem[sq * lss + i * les], scale);
    }
}

// runs the plan's passes in place over a C = 2^lc column tile (element i of
// column c at buf[i*C + c]); every thread of the block must call it
template <bool INV, int NT, int E>
__device__ __forceinline__ void tile_transform(float2 *buf, const FftPlan &pl, int lc, const float2 *stw) {
    int Ns = 1;
    for (int st = 0; st < pl.nstages; ++st) {
        const int R = pl.radix[st];
        switch (R) {
            case 8: fft_inplace_pass<8, INV, NT, E>(buf, pl.n, lc, 1, 1 << lc, Ns, stw); break;
            case 4: fft_inplace_pass<4, INV, NT, E>(buf, pl.n, lc, 1, 1 << lc, Ns, stw); break;
            case 2: fft_inplace_pass<2, INV, NT, E>(buf, pl.n, lc, 1, 1 << lc, Ns, stw); break;
            case 3: fft_inplace_pass<3, INV, NT, E>(buf, pl.n, lc, 1, 1 << lc, Ns, stw); break;
            default: fft_inplace_pass<5, INV, NT, E>(buf, pl.n, lc, 1, 1 << lc, Ns, stw); break;
        }
        Ns *= R;
    }
}

// the plan's passes in place over C = 2^lc sequences with arbitrary strides
// (row tiles: lss = n + 1, les = 1)
template <bool INV, int NT, int E>
__device__ __forceinline__ void tile_transform_ex(float2 *buf, const FftPlan &pl, int lc, int lss, int les,
                                                  const float2 *stw) {
    // radices smallest first, as in wave_transform: the stride-R writes of
    // the Ns = 1 pass then spread over the banks
    int Ns = 1;
    for (int st = pl.nstages - 1; st >= 0; --st) {
        const int R = pl.radix[st];
        switch (R) {
            case 8: fft_inplace_pass<8, INV, NT, E>(buf, pl.n, lc, lss, les, Ns, stw); break;
            case 4: fft_inplace_pass<4, INV, NT, E>(buf, pl.n, lc, lss, les, Ns, stw); break;
            case 2: fft_inplace_pass<2, INV, NT, E>(buf, pl.n, lc, lss, les, Ns, stw); break;
            case 3: fft_inplace_pass<3, INV, NT, E>(buf, pl.n, lc, lss, les, Ns, stw); break;
            default: fft_inplace_pass<5, INV, NT, E>(buf, pl.n, lc, lss, les, Ns, stw); break;
        }
        Ns *= R;
    }
}

// ---- K1 / K3 (tiled) ------------------------------------------------------------
// Row pitch of a C = 2^lc row tile: >= Np + 1 and = 32/C (mod 32), so the C
// rows a 32-lane read group touches (32/C consecutive elements each) are
// 64/C banks apart and cover the 64 banks once (Np + 1 put the C rows 2 banks
// apart: 2-4 way conflicts on every pass read).
__host__ __device__ inline int row_pitch(int np, int lc) {
    const int m = lc >= 5 ? 1 : 32 >> lc;
    int p = np + 1;
    while ((p & 31) != (m & 31)) ++p;
    return p;
}
// C = 2^lc box rows per block in one row-major LDS tile (pitch Np + 1) with
// the twiddles beside it: the row transforms of a block run together, in
// place, instead of one 256-thread block per row with global twiddle reads.
// grid (ceil(nb / C), B), block NT.
template <int NT, int E>
__global__ void __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(E <= 16 ? 4 : 1))) k_gather_rowifft_tiled(DevState st, StepArgs sa, FftPlan pl,
                                                             const float2 *__restrict__ tw, int lc) {
    extern __shared__ __attribute__((aligned(16))) float2 smem[];
    const int np = st.np, r = st.r, nb = st.nb, C = 1 << lc, lss = row_pitch(np, lc);
    const int j0 = blockIdx.x << lc, b = blockIdx.y;
    const int cs = min(C, nb - j0);
    float2 *tile = smem, *stw = smem + (size_t)C * lss;
    const float2 *pup = st.pupil + (size_t)b * nb * nb;
    for (int i = threadIdx.x; i < np; i += NT) stw[i] = tw[i];
    for (int i = threadIdx.x; i < C * lss; i += NT) tile[i] = make_float2(0.f, 0.f);
    __syncthreads();
    const float rnb = 1.0f / (float)nb;
    for (int idx = threadIdx.x; idx < cs * nb; idx += NT) {
        const int c = udiv(idx, nb, rnb), j = idx - c * nb, row = j0 + c;
        if (!st.disk[row * nb + j]) continue;
        const int kx = j - r;
        const float2 o = spec_ld(st, b, (size_t)(sa.yc + row - r) * st.L + sa.xc + kx);  // :358-362
        tile[c * lss + (kx < 0 ? kx + np : kx)] = cmul(o, pup[row * nb + j]);            // :364
    }
    __syncthreads();
    tile_transform_ex<true, NT, E>(tile, pl, lc, lss, 1, stw);                              // :365
    float2 *T = st.T + ((size_t)b * nb + j0) * np;
    const float rnp = 1.0f / (float)np;
    for (int idx = threadIdx.x; idx < cs * np; idx += NT) {
        const int c = udiv(idx, np, rnp), i = idx - c * np;
        T[(size_t)c * np + i] = tile[c * lss + i];
    }
}

template <int NT, int E>
__global__ void __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(E <= 16 ? 4 : 1))) k_rowfft_update_tiled(DevState st, StepArgs sa, FftPlan pl,
                                                            const float2 *__restrict__ tw, int lc) {
    extern __shared__ __attribute__((aligned(16))) float2 smem[];
    __shared__ float red[NT / 64];
    const int np = st.np, r = st.r, nb = st.nb, C = 1 << lc, lss = row_pitch(np, lc);
    const int j0 = blockIdx.x << lc, b = blockIdx.y;
    const int cs = min(C, nb - j0);
    float2 *tile = smem, *stw = smem + (size_t)C * lss;
    for (int i = threadIdx.x; i < np; i += NT) stw[i] = tw[i];
    const float2 *T = st.T + ((size_t)b * nb + j0) * np;
    const float rnp = 1.0f / (float)np;
    for (int idx = threadIdx.x; idx < C * np; idx += NT) {
        const int c = udiv(idx, np, rnp), i = idx - c * np;
        tile[c * lss + i] = c < cs ? T[(size_t)c * np + i] : make_float2(0.f, 0.f);
    }
    // max|P| of the previous commit from its npart partial maxima
    float pm = 0.f;
    for (int i = threadIdx.x; i < st.npart; i += NT) pm = fmaxf(pm, st.pmax[b * st.npart + i]);
    pm = block_max_nonneg(pm, red);  // its barriers also publish the tile
    tile_transform_ex<false, NT, E>(tile, pl, lc, lss, 1, stw);                             // :394
    float2 *pup = st.pupil + (size_t)b * nb * nb;
    float2 *dP = st.dP + (size_t)b * nb * nb;
    const float rnb = 1.0f / (float)nb;
    for (int idx = threadIdx.x; idx < cs * nb; idx += NT) {
        const int c = udiv(idx, nb, rnb), j = idx - c * nb, row = j0 + c;
        if (!st.disk[row * nb + j]) continue;
        const int kx = j - r;
        const size_t si = (size_t)(sa.yc + row - r) * st.L + sa.xc + kx;
        const float2 o = spec_ld(st, b, si);                    // pre-update Objfcrop (:361)
        const float2 p = pup[row * nb + j];
        const float2 F = tile[c * lss + (kx < 0 ? kx + np : kx)];  // Objfup (:394)
        const float2 D = csub(F, cmul(o, p));                   // Objfup - ObjfcropP (:409,463)
        const float pa = cmag(p);                               // object update (:406-419,433)
        const float2 dpc = cmul(cmul(D, cscale(cconj(p), pa)), upd_coef_div(pa * pa + st.delta2, st.d2_im, pm));
        spec_st(st, b, si, cadd(o, dpc));
        const float oa = cmag(o);                               // pupil numerator (:459-464,469)
        dP[row * nb + j] = cmul(cmul(D, cscale(cconj(o), oa)), upd_coef_div(oa * oa + st.delta1, st.d1_im, 1.0f));
    }
}

// ---- K2 (tiled) ---------------------------------------------------------------
// The column pass for C = 2^lc adjacent columns per block: the box rows of T
// are read as C*8-byte row segments (coalesced), the column IDFT, amplitude
// replacement and column DFT run in place in one LDS tile, and only the box
// rows are written back.  The last tile may be partial (Np not a multiple of
// C: its missing columns are zero and never stored).  grid (ceil(Np / C), B),
// block NT (256 when the tile fits its register-lifted passes, so a 16 x 200
// tile keeps every wave busy instead of idling half of a 512-thread block).
template <int NT, int E>
__global__ void __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(E <= 16 ? 4 : 1))) k_colpass_tiled(DevState st, StepArgs sa, FftPlan pl,
                                                      const float2 *__restrict__ tw, int lc) {
    extern __shared__ __attribute__((aligned(16))) float2 smem[];
    const int np = st.np, r = st.r, nb = st.nb, C = 1 << lc, cm = C - 1;
    const int x0 = blockIdx.x << lc, b = blockIdx.y;
    const int cs = min(C, np - x0);            // columns present in this tile
    float2 *tile = smem;                       // np * C
    float2 *stw = smem + (size_t)np * C;       // np twiddles
    float2 *T = st.T + (size_t)b * nb * np;
    for (int i = threadIdx.x; i < np; i += NT) stw[i] = tw[i];
    for (int i = threadIdx.x; i < np * C; i += NT) tile[i] = make_float2(0.f, 0.f);
    __syncthreads();
    for (int idx = threadIdx.x; idx < nb * C; idx += NT) {
        const int j = idx >> lc, c = idx & cm;
        const int i = j - r < 0 ? j - r + np : j - r;
        if (c < cs) tile[i * C + c] = T[(size_t)j * np + x0 + c];
    }
    __syncthreads();
    tile_transform<true, NT, E>(tile, pl, lc, stw);
    // amplitude replacement, fpmMain.cpp:378-393 (same arithmetic as k_colpass)
    const float inv_n2 = 1.0f / ((float)np * (float)np);
    const uint16_t *I = st.meas + ((size_t)sa.led * st.mB + b) * np * np;
    for (int idx = threadIdx.x; idx < np * C; idx += NT) {
        const int y = idx >> lc, c = idx & cm;
        if (c >= cs) continue;
        const float2 psi = cscale(tile[idx], inv_n2);
        const float a = sqrtf((float)I[(size_t)y * np + x0 + c]);
        const float tre = psi.x + st.eps, tim = psi.y + st.eps_im;
        const float mag = sqrtf(tre * tre + tim * tim);
        const float sc = a / mag;
        tile[idx] = make_float2(psi.x * sc, psi.y * sc);
    }
    __syncthreads();
    tile_transform<false, NT, E>(tile, pl, lc, stw);
    for (int idx = threadIdx.x; idx < nb * C; idx += NT) {
        const int j = idx >> lc, c = idx & cm;
        const int i = j - r < 0 ? j - r + np : j - r;
        if (c < cs) T[(size_t)j * np + x0 + c] = tile[i * C + c];
    }
}

// ---- K2 (wave-private columns) ----------------------------------------------------
// Same column pass, but every wave owns CW whole columns of the block's
// C = NW*CW-column tile, so the radix passes synchronise the wave only (LDS
// operations of one wave execute in issue order; the fence pair keeps the
// compiler from moving them) instead of the whole block: two block barriers
// per launch (after the coalesced tile load, before the coalesced store)
// instead of two per radix pass.  Within a wave, 64/CW consecutive lanes
// serve one column (column-major, pitch P), so a lane's column and its base
// address are fixed for the whole transform and every butterfly element is
// an immediate offset from it.  The measurement values a lane needs for
// amplitude replacement (rows lane + 64q of its wave's columns) are loaded
// into registers before the inverse transform, so their latency hides behind
// it.
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
constexpr int kWaveElems = 16;  // register elements per lane in a wave pass

// one radix-R Stockham pass over the lane's column `cb` (lanes l, l + LPC,
// ... of the column's butterflies: l = lane % LPC)
template <int R, bool INV, int LPC>
__device__ __forceinline__ void wave_pass(float2 *cb, int n, int Ns, const float2 *__restrict__ tw, int l) {
    constexpr int Q = kWaveElems / R;
    const int nR = n / R, tmul = n / (Ns * R);
    const bool pow2 = (Ns & (Ns - 1)) == 0;
    const int lNs = 31 - __builtin_clz(Ns);
    const float rNs = 1.0f / (float)Ns;
    float2 v[Q][R];
    int base[Q];
#pragma unroll
    for (int q = 0; q < Q; ++q) {
        const int j = l + LPC * q;
        base[q] = -1;
        if (j < nR) {
#pragma unroll
            for (int r = 0; r < R; ++r) v[q][r] = cb[j + r * nR];
            const int jq = pow2 ? (j >> lNs) : udiv(j, Ns, rNs);
            const int k = j - jq * Ns;
            if (Ns > 1) {
                const int ts = tmul * k;
#pragma unroll
                for (int r = 1; r < R; ++r) {
                    float2 w = tw[r * ts];
                    if (INV) w.y = -w.y;
                    v[q][r] = cmul(v[q][r], w);
                }
            }
            if (R == 2) dft2<INV>(v[q]);
            if (R == 3) dft3<INV>(v[q]);
            if (R == 4) dft4<INV>(v[q]);
            if (R == 5) dft5<INV>(v[q]);
            if (R == 8) dft8<INV>(v[q]);
            base[q] = jq * Ns * R + k;
        }
    }
    wave_sync();
#pragma unroll
    for (int q = 0; q < Q; ++q) {
        if (base[q] >= 0) {
#pragma unroll
            for (int r = 0; r < R; ++r) cb[base[q] + r * Ns] = v[q][r];
        }
    }
    wave_sync();
}

// The plan's radices run in reverse (smallest first: 200 = 5*5*8), so the
// stride-R writes of the Ns = 1 pass come from a radix whose stride spreads
// over the banks (a radix-8 first pass is a 4-way conflict on every write).
template <bool INV, int LPC>
__device__ __forceinline__ void wave_transform(float2 *cb, const FftPlan &pl, const float2 *stw, int l) {
    int Ns = 1;
    for (int s = pl.nstages - 1; s >= 0; --s) {
        const int R = pl.radix[s];
        switch (R) {
            case 8: wave_pass<8, INV, LPC>(cb, pl.n, Ns, stw, l); break;
            case 4: wave_pass<4, INV, LPC>(cb, pl.n, Ns, stw, l); break;
            case 2: wave_pass<2, INV, LPC>(cb, pl.n, Ns, stw, l); break;
            case 3: wave_pass<3, INV, LPC>(cb, pl.n, Ns, stw, l); break;
            default: wave_pass<5, INV, LPC>(cb, pl.n, Ns, stw, l); break;
        }
        Ns *= R;
    }
}

// column pitch of the tile: Np rounded to 2 mod 4, so the C columns of the
// coalesced load/store land in distinct banks and every column is 16-byte
// aligned
int colw_pitch(int np) {
    int p = np;
    while ((p & 3) != 2) ++p;
    return p;
}

// grid (ceil(Np / (NW*CW)), B), block 64*NW, LDS (NW*CW*pitch + Np) float2
template <int NW, int CW>
__global__ void __launch_bounds__(64 * NW)
k_colpass_wave(DevState st, StepArgs sa, FftPlan pl, const float2 *__restrict__ tw, int P) {
    constexpr int NT = 64 * NW, C = NW * CW, NQY = 16 / CW;
    extern __shared__ __attribute__((aligned(16))) float2 smem[];
    const int np = st.np, r = st.r, nb = st.nb;
    const int x0 = blockIdx.x * C, b = blockIdx.y;
    const int cs = min(C, np - x0);
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    constexpr int LPC = 64 / CW;
    float2 *stw = smem + (size_t)C * P;
    float2 *wb = smem + (size_t)w * CW * P;
    float2 *cb = wb + (lane / LPC) * P;  // this lane's column in the radix passes
    const int l = lane % LPC;
    float2 *T = st.T + (size_t)b * nb * np;
    // this lane's measurement values: rows lane + 64q of the wave's columns
    const uint16_t *I = st.meas + ((size_t)sa.led * st.mB + b) * np * np;
    uint16_t iv[NQY * CW];
#pragma unroll
    for (int q = 0; q < NQY; ++q) {
        const int y = lane + 64 * q;
#pragma unroll
        for (int c = 0; c < CW; ++c) {
            const int x = w * CW + c;
            iv[q * CW + c] = (y < np && x < cs) ? I[(size_t)y * np + x0 + x] : (uint16_t)0;
        }
    }
    for (int i = threadIdx.x; i < np; i += NT) stw[i] = tw[i];
    // every tile element written once: box rows from T, zeros elsewhere
    const float rC = 1.0f / (float)C;
    for (int idx = threadIdx.x; idx < np * C; idx += NT) {
        const int i = udiv(idx, C, rC), c = idx - i * C;
        const int ky = i < np / 2 ? i : i - np, j = ky + r;
        float2 v = make_float2(0.f, 0.f);
        if (c < cs && j >= 0 && j < nb) v = T[(size_t)j * np + x0 + c];
        smem[c * P + i] = v;
    }
    __syncthreads();
    wave_transform<true, LPC>(cb, pl, stw, l);
    // amplitude replacement, fpmMain.cpp:378-393 (same arithmetic as k_colpass)
    const float inv_n2 = 1.0f / ((float)np * (float)np);
#pragma unroll
    for (int q = 0; q < NQY; ++q) {
        const int y = lane + 64 * q;
        if (y >= np) continue;
#pragma unroll
        for (int c = 0; c < CW; ++c) {
            float2 *e = wb + c * P + y;
            const float2 psi = cscale(*e, inv_n2);
            const float a = sqrtf((float)iv[q * CW + c]);
            const float tre = psi.x + st.eps, tim = psi.y + st.eps_im;
            const float mag = sqrtf(tre * tre + tim * tim);
            const float sc = a / mag;
            *e = make_float2(psi.x * sc, psi.y * sc);
        }
    }
    wave_sync();
    wave_transform<false, LPC>(cb, pl, stw, l);
    __syncthreads();
    for (int idx = threadIdx.x; idx < nb * C; idx += NT) {
        const int j = udiv(idx, C, rC), c = idx - j * C;
        const int i = j - r < 0 ? j - r + np : j - r;
        if (c < cs) T[(size_t)j * np + x0 + c] = smem[c * P + i];
    }
}

// columns per wave of k_colpass_wave for this plan: the largest CW in {4,2,1}
// for which 64/CW lanes hold a column's butterflies in every radix pass
// (kWaveElems values per lane);
// 0 when even one column does not fit
int colw_cw(const FftPlan &pl) {
    for (int cw = 4; cw >= 1; cw >>= 1) {
        bool ok = true;
        for (int i = 0; i < pl.nstages; ++i) {
            const int R = pl.radix[i];
            const int lpc = 64 / cw;
            if ((pl.n / R + lpc - 1) / lpc > kWaveElems / R) ok = false;
        }
        if (ok) return cw;
    }
    return 0;
}

// sqrt of the init image as complex, fpmMain.cpp:319-322. grid (Np, B)
// meas in either layout (DevState::meas_g)
__global__ void k_init_amp(const uint16_t *__restrict__ meas, float2 *__restrict__ out, int np, int B,
                           int led, size_t out_bs, int g) {
    const int y = blockIdx.x, b = blockIdx.y;
    const uint16_t *I = meas + ((size_t)led * B + b) * np * np;
    float2 *o = out + (size_t)b * out_bs + (size_t)y * np;
    const int col = g ? (y % g) * (np / g) + y / g : 0;  // position of row y inside a stored column
    for (int x = threadIdx.x; x < np; x += blockDim.x) {
        const uint16_t v = g ? I[(size_t)x * np + col] : I[(size_t)y * np + x];
        o[x] = make_float2(sqrtf((float)v), 0.f);
    }
}

// zero the spectrum, place fftShift(fft2(A) * S) at the centre
// (fpmMain.cpp:326-343), P = S, max|P| = 1.  grid (nb, B)
__global__ void k_init_place(DevState st, const float2 *__restrict__ F, size_t f_bs) {
    const int row = blockIdx.x, b = blockIdx.y;
    const int np = st.np, r = st.r, nb = st.nb, L = st.L;
    const int ky = row - r;
    float2 *pup = st.pupil + (size_t)b * nb * nb;
    const float2 *f = F + (size_t)b * f_bs;
    for (int j = threadIdx.x; j < nb; j += blockDim.x) {
        const int kx = j - r;
        const bool in = st.disk[row * nb + j];
        if (in)
            spec_st(st, b, (size_t)(L / 2 + ky) * L + L / 2 + kx, f[(size_t)((ky + np) % np) * np + (kx + np) % np]);
        pup[row * nb + j] = make_float2(in ? 1.f : 0.f, 0.f);
    }
    // max|P0| = 1 (partial maxima other than part 0 were zeroed by launch_init)
    if (row == 0 && threadIdx.x == 0) st.pmax[b * st.npart] = (st.disk[r * nb + r] ? 1.f : 0.f);
}

// tile maxima of |spec| after k_init_place. grid (ntx*nty, B), block 256.
// The spectrum was just zeroed except the init box [L/2 - r, L/2 + r]^2, so a
// tile outside it is 0 without reading it (init read the whole spectrum
// again: 1.2 GB at the metric config)
__global__ void __launch_bounds__(256) k_tile_max_all(DevState st) {
    __shared__ float red[8];
    const int t = blockIdx.x, b = blockIdx.y, L = st.L;
    const int ty = t / st.ntx, tx = t % st.ntx;
    const int lo = L / 2 - st.r, hi = L / 2 + st.r;
    if (ty * kTile > hi || ty * kTile + kTile - 1 < lo || tx * kTile > hi || tx * kTile + kTile - 1 < lo) {
        if (threadIdx.x == 0) st.tmax[(size_t)b * st.nty * st.ntx + t] = 0.f;  // block-uniform
        return;
    }
    const int y = ty * kTile + (threadIdx.x >> 4), x = tx * kTile + (threadIdx.x & 15);
    float m = 0.f;
    if (y < L && x < L) m = cmag(spec_ld(st, b, (size_t)y * L + x));
    m = block_max_nonneg(m, red);
    if (threadIdx.x == 0) st.tmax[(size_t)b * st.nty * st.ntx + t] = m;
}

// row maxima of the tile maxima after init (general path). grid (nty, B)
__global__ void __launch_bounds__(256) k_row_max_all(DevState st) {
    __shared__ float red[4];
    const int ty = blockIdx.x, b = blockIdx.y;
    const float *tm = st.tmax + ((size_t)b * st.nty + ty) * st.ntx;
    float m = 0.f;
    for (int i = threadIdx.x; i < st.ntx; i += 256) m = fmaxf(m, tm[i]);
    m = block_max_nonneg(m, red);
    if (threadIdx.x == 0) st.rmax[(size_t)b * st.nty + ty] = m;
}

// ---- host-side launchers ----------------------------------------------------
// C = 2^lc sequences of pl.n fit the in-place transform's register budget
static bool fft_fits(const FftPlan &pl, int lc, int nt = kFftThreads, int e = kFftRegElems) {
    for (int i = 0; i < pl.nstages; ++i)
        if ((pl.n << lc) > fft_pass_capacity(pl.radix[i], nt, e)) return false;
    return true;
}

hipError_t launch_np1024_rows_cols(const DevState &st, const StepArgs &sa, const float2 *tw, bool commit,
                                   hipStream_t s);
hipError_t launch_np256_rows_cols(const DevState &st, const StepArgs &sa, const float2 *tw, bool commit,
                                  hipStream_t s);

// the register row / column kernels (np1024.hip, np256.hip) fold the pupil
// commit into the next LED's row IDFT
bool commit_folded(const DevState &st) {
    return (st.np == 1024 && st.meas_g == 1024) || (st.np == 256 && st.meas_g == 16);
}

// first: the iteration's first LED (Np 1024: no pupil commit pending)
hipError_t launch_general_step(const DevState &st, int led, int x0, int y0, const FftPlan &pl,
                               const float2 *tw, bool first, hipStream_t s) {
    StepArgs sa;
    sa.led = led;
    sa.xc = x0 + st.np / 2;
    sa.yc = y0 + st.np / 2;
    if (st.np == 1024 && st.meas_g == 1024) {
        // Np 1024: register-resident row/column transforms (np1024.hip)
        const hipError_t e = launch_np1024_rows_cols(st, sa, tw, !first, s);
        if (e != hipSuccess) return e;
    } else if (st.np == 256 && st.meas_g == 16) {
        // Np 256 beyond the fused kernels' radius: register row/column
        // transforms (np256.hip); K4 runs inside its R2, K5 folded into the next R1
        return launch_np256_rows_cols(st, sa, tw, !first, s);
    } else {
        const size_t lds = 2 * (size_t)st.np * sizeof(float2);
        // row kernels: up to 16 box rows per block, fewer while a few large
        // patches would leave the chip short of blocks (one row per block when
        // not even 2 rows fit a 256-thread tile)
        int lr = 4;
        while (lr > 0 && !fft_fits(pl, lr, 256)) --lr;
        auto rblk = [&](int l) { return ((st.nb + (1 << l) - 1) >> l) * st.B; };
        while (lr > 1 && rblk(lr) < 512) --lr;
        const size_t ldr = ((size_t)row_pitch(st.np, lr) * (1 << lr) + st.np) * sizeof(float2);
        const dim3 rgrid((st.nb + (1 << lr) - 1) >> lr, st.B);
        // 16 register elements per thread when the tile allows (fewer VGPRs, more
        // waves per SIMD to hide the LDS round trips of each pass), else 24
        const bool r16 = lr > 0 && fft_fits(pl, lr, 256, 16);
        if (lr > 0 && r16)
            hipLaunchKernelGGL(HIP_KERNEL_NAME(k_gather_rowifft_tiled<256, 16>), rgrid, dim3(256), ldr, s, st, sa, pl, tw, lr);
        else if (lr > 0)
            hipLaunchKernelGGL(HIP_KERNEL_NAME(k_gather_rowifft_tiled<256, 24>), rgrid, dim3(256), ldr, s, st, sa, pl, tw, lr);
        else
            hipLaunchKernelGGL(k_gather_rowifft, dim3(st.nb, st.B), dim3(256), lds, s, st, sa, pl, tw);
        // tiled column pass: up to 16 columns per block while the tile fits the
        // in-place register-lifted transform, fewer (down to 4) when a few large
        // patches would leave the chip short of blocks; one column per block when
        // not even 2 columns fit
        int lc = 4;
        while (lc > 0 && !fft_fits(pl, lc)) --lc;
        auto nblk = [&](int l) { return ((st.np + (1 << l) - 1) >> l) * st.B; };
        while (lc > 2 && nblk(lc) < 512) --lc;
        const int cw = colw_cw(pl);
        if (cw > 1 && !std::getenv("FPM_NO_WAVE_COLS")) {
            // wave-private columns: 4 waves x CW columns, 8 waves when a wave
            // holds a single (long) column
            const int P = colw_pitch(st.np);
            const int nw = cw == 1 ? 8 : 4, C = nw * cw;
            const size_t ldw = ((size_t)C * P + st.np) * sizeof(float2);
            const dim3 grid((st.np + C - 1) / C, st.B);
            if (cw == 4)
                hipLaunchKernelGGL(HIP_KERNEL_NAME(k_colpass_wave<4, 4>), grid, dim3(256), ldw, s, st, sa, pl, tw, P);
            else if (cw == 2)
                hipLaunchKernelGGL(HIP_KERNEL_NAME(k_colpass_wave<4, 2>), grid, dim3(256), ldw, s, st, sa, pl, tw, P);
            else
                hipLaunchKernelGGL(HIP_KERNEL_NAME(k_colpass_wave<8, 1>), grid, dim3(512), ldw, s, st, sa, pl, tw, P);
        } else if (lc > 0) {
            const size_t ldt = ((size_t)st.np * (1 << lc) + st.np) * sizeof(float2);
            const dim3 grid((st.np + (1 << lc) - 1) >> lc, st.B);
            if (fft_fits(pl, lc, 256, 16))
                hipLaunchKernelGGL(HIP_KERNEL_NAME(k_colpass_tiled<256, 16>), grid, dim3(256), ldt, s, st, sa, pl, tw, lc);
            else if (fft_fits(pl, lc, 256))
                hipLaunchKernelGGL(HIP_KERNEL_NAME(k_colpass_tiled<256, 24>), grid, dim3(256), ldt, s, st, sa, pl, tw, lc);
            else if (fft_fits(pl, lc, kFftThreads, 16))
                hipLaunchKernelGGL(HIP_KERNEL_NAME(k_colpass_tiled<kFftThreads, 16>), grid, dim3(kFftThreads), ldt, s, st, sa, pl, tw, lc);
            else
                hipLaunchKernelGGL(HIP_KERNEL_NAME(k_colpass_tiled<kFftThreads, 24>), grid, dim3(kFftThreads), ldt, s, st, sa, pl, tw, lc);
        } else {
            hipLaunchKernelGGL(k_colpass, dim3(st.np, st.B), dim3(256), lds, s, st, sa, pl, tw);
        }
        if (lr > 0 && r16)
            hipLaunchKernelGGL(HIP_KERNEL_NAME(k_rowfft_update_tiled<256, 16>), rgrid, dim3(256), ldr, s, st, sa, pl, tw, lr);
        else if (lr > 0)
            hipLaunchKernelGGL(HIP_KERNEL_NAME(k_rowfft_update_tiled<256, 24>), rgrid, dim3(256), ldr, s, st, sa, pl, tw, lr);
        else
            hipLaunchKernelGGL(k_rowfft_update, dim3(st.nb, st.B), dim3(256), lds, s, st, sa, pl, tw);
    }
    const int nrow = (sa.yc + st.r) / kTile - (sa.yc - st.r) / kTile + 1;
    const int ncol = (sa.xc + st.r) / kTile - (sa.xc - st.r) / kTile + 1;
    if (ncol > 8)
        hipLaunchKernelGGL(HIP_KERNEL_NAME(k_tile_rows<1024>), dim3(nrow, st.B), dim3(1024), 0, s, st, sa);
    else
        hipLaunchKernelGGL(HIP_KERNEL_NAME(k_tile_rows<256>), dim3(nrow, st.B), dim3(256), 0, s, st, sa);
    // Np 1024 / 256 register kernels: the commit is folded into the next LED's
    // row IDFT and runs here only after the iteration's last LED
    // (launch_pupil_commit)
    if (!commit_folded(st))
        hipLaunchKernelGGL(k_pupil_commit, dim3(st.npart, st.B), dim3(kCommitThreads), 0, s, st);
    return hipGetLastError();
}

hipError_t launch_pupil_commit(const DevState &st, hipStream_t s) {
    hipLaunchKernelGGL(k_pupil_commit, dim3(st.npart, st.B), dim3(kCommitThreads), 0, s, st);
    return hipGetLastError();
}

// largest C = 2^lc with C*n complex values in registers across the block
// (kFftRegElems per thread; radix-5 passes hold 20) and at most 16 sequences
int fft_log2_seq_per_block(const FftPlan &pl) {
    int cap = kFftRegElems * kFftThreads;
    for (int i = 0; i < pl.nstages; ++i) cap = std::min(cap, fft_pass_capacity(pl.radix[i]));
    int lc = 0;
    while (lc < 4 && (pl.n << (lc + 1)) <= cap) ++lc;
    return (pl.n << lc) <= cap ? lc : -1;
}

int fft_max_len() { return fft_pass_capacity(5); }  // the smallest of the radix-2/3/4/5 capacities

hipError_t launch_fft_batch(bool inverse, const float2 *in, float2 *out, const FftPlan &pl, const float2 *tw,
                            int nseq, int B, size_t in_bs, int in_ss, int in_es, size_t out_bs, int out_ss,
                            int out_es, int sroll, int iroll, float scale, hipStream_t s,
                            const __half2 *in16 = nullptr, float in16_scale = 1.f, FftBand band = FftBand()) {
    const int lc = fft_log2_seq_per_block(pl);
    if (lc < 0) return hipErrorInvalidValue;
    const int C = 1 << lc;
    // row-major tiles carry one pad element per sequence
    const size_t lds = ((size_t)C * (pl.n + 1) + pl.n) * sizeof(float2);  // tile + twiddles
    dim3 grid((nseq + C - 1) / C, B);
    hipError_t e = hipFuncSetAttribute(inverse ? (const void *)k_fft_batch<true> : (const void *)k_fft_batch<false>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
    if (inverse)
        hipLaunchKernelGGL(k_fft_batch<true>, grid, dim3(kFftThreads), lds, s, in, out, pl, tw, lc, nseq, in_bs,
                           in_ss, in_es, out_bs, out_ss, out_es, sroll, iroll, scale, in16, in16_scale, band);
    else
        hipLaunchKernelGGL(k_fft_batch<false>, grid, dim3(kFftThreads), lds, s, in, out, pl, tw, lc, nseq, in_bs,
                           in_ss, in_es, out_bs, out_ss, out_es, sroll, iroll, scale, in16, in16_scale, band);
    return hipGetLastError();
}

hipError_t launch_init(const DevState &st, int init_led, float2 *scratch, const FftPlan &pl_np,
                       const float2 *tw_np, hipStream_t s) {
    const int np = st.np;
    const size_t bs = (size_t)np * np;
    hipLaunchKernelGGL(k_init_amp, dim3(np, st.B), dim3(256), 0, s, st.meas, scratch, np, st.B, init_led, bs,
                       st.meas_g);
    // fft2: rows then columns, in place (fpmMain.cpp:325)
    hipError_t e = launch_fft_batch(false, scratch, scratch, pl_np, tw_np, np, st.B, bs, np, 1, bs, np, 1, 0, 0,
                                    1.f, s);
    if (e != hipSuccess) return e;
    e = launch_fft_batch(false, scratch, scratch, pl_np, tw_np, np, st.B, bs, 1, np, bs, 1, np, 0, 0, 1.f, s);
    if (e != hipSuccess) return e;
    e = st.spec16 ? hipMemsetAsync(st.spec16, 0, (size_t)st.B * st.L * st.L * sizeof(__half2), s)
                  : hipMemsetAsync(st.spec, 0, (size_t)st.B * st.L * st.L * sizeof(float2), s);
    if (e != hipSuccess) return e;
    e = hipMemsetAsync(st.pmax, 0, (size_t)st.B * st.npart * sizeof(float), s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_init_place, dim3(st.nb, st.B), dim3(256), 0, s, st, (const float2 *)scratch, bs);
    hipLaunchKernelGGL(k_tile_max_all, dim3(st.ntx * st.nty, st.B), dim3(256), 0, s, st);
    if (st.rmax) hipLaunchKernelGGL(k_row_max_all, dim3(st.nty, st.B), dim3(256), 0, s, st);
    e = hipMemsetAsync(st.tdirty, 0, (size_t)st.B * ((st.ntx * st.nty + 31) / 32) * sizeof(unsigned), s);
    if (e != hipSuccess) return e;
    return hipGetLastError();
}

// objCrop = IDFT(objF)/L^2 with objF = fftShift(spec) (fpmMain.cpp:481):
// rows of the rolled spectrum, then columns, scaled by 1/L^2.
hipError_t launch_objcrop_regs(const DevState &st, float2 *out, const float2 *tw_L, hipStream_t s);

// ---- objCrop for L = 4096 (config 5) ----------------------------------------
// The batched transform above fits only C = 2 sequences of 4096 points in a
// block, so its column pass reads 16-byte column segments (the counters:
// 3x the pass's bytes, 3.6 ms per iteration at config 5).  Here the column
// IDFT runs first, straight from the (read-only) spectrum, as a six-step
// 4096 = 64 x 64 transform whose passes read and write 128-byte row segments
// of 16 adjacent columns; the row IDFT then runs in place, the same 64 x 64
// split inside a block per row (k_crop4k_rows).  With
// n = n1 + 64 n2 and k = k2 + 64 k1 (inverse, W = e^{+2 pi i / 4096}):
//   X[k2 + 64 k1] = sum_n1 W64^{n1 k1} [ W^{n1 k2} sum_n2 x[n1 + 64 n2] W64^{n2 k2} ]
//   pass 1 (block n1): the bracket for all k2, stored at row k2 + 64 n1
//   pass 2 (block k2): reads rows k2 + 64 n1, writes X at rows k2 + 64 k1 --
//                      the same rows, so it runs in place
namespace c4k {
constexpr int L = 4096, CW = 16, NT = 8 * CW;  // 16 columns x 8 lanes per block

// 64-point inverse DFT of the block's 16 columns, 8 lanes per column (8 x 8:
// DFT8 over the lane's values, W64 twiddles, LDS exchange, DFT8): lane (c, j)
// holds x[j + 8 b] in v[b] and returns X[j + 8 q] in v[q].  One barrier; lds
// is used once per launch.
__device__ __forceinline__ void idft64(float2 (&v)[8], float2 *lds, int c, int j, const float2 *__restrict__ tw) {
    dft8<true>(v);  // Z_j[p] = sum_b x[j + 8 b] W8^{b p}
#pragma unroll
    for (int p = 1; p < 8; ++p) v[p] = cmul(v[p], cconj(tw[(64 * j * p) & (L - 1)]));  // W64^{j p}
#pragma unroll
    for (int p = 0; p < 8; ++p) lds[(c * 8 + j) * 9 + p] = v[p];
    __syncthreads();
#pragma unroll
    for (int a = 0; a < 8; ++a) v[a] = lds[(c * 8 + a) * 9 + j];  // Z_a[j]
    dft8<true>(v);  // X[j + 8 q] = sum_a Z_a[j] W8^{a q}
}

// pass 1: grid (L / CW, 64 (n1), B); objF row y, column x = spec row / column
// (y + L/2, x + L/2) mod L; zero outside the live band (fpm_state.hpp)
__global__ void __launch_bounds__(NT) k_crop4k_cols1(DevState st, float2 *out, const float2 *__restrict__ tw) {
    __shared__ float2 lds[CW * 8 * 9];
    const int c = threadIdx.x & (CW - 1), j = threadIdx.x / CW;
    const int x = blockIdx.x * CW + c, n1 = blockIdx.y, b = blockIdx.z;
    const int sx = (x + L / 2) & (L - 1);
    const bool live = sx >= st.sx0 && sx <= st.sx1;
    float2 v[8];
    // unconditional loads of clamped indices, masked after all eight (a
    // masked spec_ld widens fp16 where it loads: one round trip per q)
    bool ok[8];
    size_t idx[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
        const int sy = (n1 + 64 * (j + 8 * q) + L / 2) & (L - 1);
        ok[q] = live && sy >= st.sy0 && sy <= st.sy1;
        idx[q] = (size_t)b * L * L + (ok[q] ? (size_t)sy * L + sx : 0);
    }
    if (st.spec16) {  // uniform
        __half2 hv[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) hv[q] = st.spec16[idx[q]];
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            const float2 f = __half22float2(hv[q]);
            v[q] = ok[q] ? make_float2(f.x * st.hinv, f.y * st.hinv) : make_float2(0.f, 0.f);
        }
    } else {
#pragma unroll
        for (int q = 0; q < 8; ++q) v[q] = st.spec[idx[q]];
#pragma unroll
        for (int q = 0; q < 8; ++q) v[q] = ok[q] ? v[q] : make_float2(0.f, 0.f);
    }
    idft64(v, lds, c, j, tw);
    float2 *o = out + (size_t)b * L * L + x;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
        const int k2 = j + 8 * q;
        o[(size_t)(k2 + 64 * n1) * L] = cmul(v[q], cconj(tw[(n1 * k2) & (L - 1)]));  // W^{n1 k2}
    }
}

// pass 2: grid (L / CW, 64 (k2), B), in place on out
__global__ void __launch_bounds__(NT) k_crop4k_cols2(float2 *out, const float2 *__restrict__ tw) {
    __shared__ float2 lds[CW * 8 * 9];
    const int c = threadIdx.x & (CW - 1), j = threadIdx.x / CW;
    const int x = blockIdx.x * CW + c, k2 = blockIdx.y, b = blockIdx.z;
    float2 *o = out + (size_t)b * L * L + x;
    float2 v[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) v[q] = o[(size_t)(k2 + 64 * (j + 8 * q)) * L];
    idft64(v, lds, c, j, tw);
#pragma unroll
    for (int q = 0; q < 8; ++q) o[(size_t)(k2 + 64 * (j + 8 * q)) * L] = v[q];
}

// rows: grid (L, B), block 512, in place on out: the same 64 x 64 split within
// the row held by the block -- lane (n1, j) runs the DFT64 over n2 for column
// n1 of the row's 64 x 64 matrix x[n1 + 64 n2], the twiddled results are
// transposed through LDS, lane (k2, j) runs the DFT64 over n1; every load and
// store is 512 contiguous bytes per wave.  Elements x with spec column
// (x + L/2) mod L outside the live band are zero and not read.
constexpr int NTR = 512;
__global__ void __launch_bounds__(NTR) k_crop4k_rows(DevState st, float2 *out, const float2 *__restrict__ tw,
                                                      float scale) {
    __shared__ float2 lds[64 * 8 * 9];
    const int i64 = threadIdx.x & 63, j = threadIdx.x >> 6;
    float2 *row = out + ((size_t)blockIdx.y * L + blockIdx.x) * L;
    float2 v[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
        const int x = i64 + 64 * (j + 8 * q), sx = (x + L / 2) & (L - 1);
        v[q] = sx >= st.sx0 && sx <= st.sx1 ? row[x] : make_float2(0.f, 0.f);
    }
    idft64(v, lds, i64, j, tw);  // lane (n1 = i64, j): bracket values for k2 = j + 8 q
    __syncthreads();             // the exchange reads are done: lds is the transpose tile now
#pragma unroll
    for (int q = 0; q < 8; ++q) {
        const int k2 = j + 8 * q;
        lds[i64 * 65 + k2] = cmul(v[q], cconj(tw[(i64 * k2) & (L - 1)]));  // A[n1][k2] W^{n1 k2}
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < 8; ++q) v[q] = lds[(j + 8 * q) * 65 + i64];  // lane (k2 = i64, j): A[j + 8 q][k2]
    __syncthreads();             // before idft64's exchange overwrites lds
    idft64(v, lds, i64, j, tw);  // X[k2 + 64 (j + 8 q)]
#pragma unroll
    for (int q = 0; q < 8; ++q) row[i64 + 64 * (j + 8 * q)] = cscale(v[q], scale);
}
}  // namespace c4k

static hipError_t launch_crop4096(const DevState &st, float2 *out, const float2 *tw_L, hipStream_t s) {
    using namespace c4k;
    const dim3 grid(L / CW, 64, st.B);
    hipLaunchKernelGGL(k_crop4k_cols1, grid, dim3(NT), 0, s, st, out, tw_L);
    hipLaunchKernelGGL(k_crop4k_cols2, grid, dim3(NT), 0, s, out, tw_L);
    hipLaunchKernelGGL(k_crop4k_rows, dim3(L, st.B), dim3(NTR), 0, s, st, out, tw_L, 1.0f / ((float)L * (float)L));
    return hipGetLastError();
}

hipError_t launch_objcrop(const DevState &st, float2 *out, const FftPlan &pl_L, const float2 *tw_L,
                          hipStream_t s) {
    // L = 512 / 768 / 1024: register-resident transforms (objcrop.hip)
    if (!st.spec16) {
        const hipError_t r = launch_objcrop_regs(st, out, tw_L, s);
        if (r != hipErrorNotSupported) return r;
    }
    if (st.L == c4k::L && !std::getenv("FPM_NO_CROP4K")) return launch_crop4096(st, out, tw_L, s);
    const int L = st.L;
    const size_t bs = (size_t)L * L;
    // rows: spec rows (sequences) and columns (elements) outside the live band
    // are zero; columns: objF row i of the intermediate is spec row i + L/2
    FftBand rows, cols;
    rows.qlo = st.sy0;
    rows.qhi = st.sy1;
    rows.elo = st.sx0;
    rows.ehi = st.sx1;
    cols.elo = st.sy0;
    cols.ehi = st.sy1;
    cols.eroll = L / 2;
    hipError_t e = launch_fft_batch(true, st.spec, out, pl_L, tw_L, L, st.B, bs, L, 1, bs, L, 1, L / 2, L / 2, 1.f,
                                    s, st.spec16, st.hinv, rows);
    if (e != hipSuccess) return e;
    return launch_fft_batch(true, out, out, pl_L, tw_L, L, st.B, bs, 1, L, bs, 1, L, 0, 0,
                            1.0f / ((float)L * (float)L), s, nullptr, 1.f, cols);
}

}  // namespace fpm
