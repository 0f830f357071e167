// fpm_oracle.cpp -- TEST INFRASTRUCTURE ONLY: the CPU checker and the timed
// CPU baseline ("port").  Only tests/, __graft_entry__.smoke() and bench.py's
// cpu_baseline leg load liboracle.so; the product (fpm-opencv_amd/) never does.
//
// A reference-faithful complex128 restatement of runFPM
// (/root/reference/fpmMain.cpp:274-498) for one patch, op for op, with the
// same temporaries the reference materialises:
//   - three full L x L fftShift copies per LED (fpmMain.cpp:358,427,447),
//   - complexAbs of the whole L x L spectrum + minMaxLoc per LED (:460,467),
//   - element-wise complex ops as separate passes (:364-475),
//   - the per-iteration objCrop IDFT (:481).
// The DFTs are this file's own mixed-radix (2/3/4/5) Stockham FFT in double.
// cvComplex semantics assumed as in SURVEY.md 8(c)(i)-(iii),(v)-(vii) (parity
// unpinned at that boundary: the library is not in the reference tree).
// (iv) is replaced by OpenCV's published scalar rule: cv::add / cv::multiply
// (UMat CV_64FC2, double) unroll the double into every channel (arithm_op ->
// checkScalar -> convertAndUnrollScalar), so eps lands on Re and Im (:390)
// and the update denominators are complex (:417-418, :469-470).  all_ch = 0
// restates the real-channel-only assumption (FPM_FLAG_SCALAR_RE_ONLY).
//
// C ABI (ctypes from tests / bench):
//   int oracle_run_fpm(...)        one patch
//   int oracle_run_fpm_batch(...)  n_patch patches on n_threads std::threads
//   int oracle_fft2(...)           KAT hook for the FFT
#include <cmath>
#include <complex>
#include <cstdint>
#include <cstring>
#include <thread>
#include <vector>

namespace {

using cplx = std::complex<double>;

struct Fft {
    int n = 0;
    std::vector<int> radix;
    std::vector<cplx> tw;  // exp(-2 pi i k / n)
    explicit Fft(int n_) : n(n_) {
        int m = n;
        for (int r : {4, 2, 3, 5})
            while (m % r == 0) {
                radix.push_back(r);
                m /= r;
            }
        if (m != 1) radix.clear();
        tw.resize(n);
        for (int k = 0; k < n; ++k) tw[k] = std::polar(1.0, -2.0 * M_PI * k / n);
    }
    bool ok() const { return !radix.empty() || n == 1; }

    // unscaled DFT of a[0..n) (stride 1), result in a; s is scratch of n
    void run(cplx *a, cplx *s, bool inverse) const {
        cplx *src = a, *dst = s;
        int Ns = 1;
        for (int R : radix) {
            const int nR = n / R, tm = n / (Ns * R);
            for (int j = 0; j < nR; ++j) {
                const int k = j % Ns;
                cplx v[5];
                for (int r = 0; r < R; ++r) {
                    v[r] = src[j + r * nR];
                    if (r && Ns > 1) {
                        cplx w = tw[r * tm * k];
                        if (inverse) w = std::conj(w);
                        v[r] *= w;
                    }
                }
                cplx y[5];
                if (R == 4) {  // radix-4 butterfly (-i forward, +i inverse)
                    const cplx s02 = v[0] + v[2], d02 = v[0] - v[2], s13 = v[1] + v[3];
                    const cplx d13 = (v[1] - v[3]) * (inverse ? cplx(0, 1) : cplx(0, -1));
                    y[0] = s02 + s13;
                    y[1] = d02 + d13;
                    y[2] = s02 - s13;
                    y[3] = d02 - d13;
                } else if (R == 2) {
                    y[0] = v[0] + v[1];
                    y[1] = v[0] - v[1];
                } else
                for (int q = 0; q < R; ++q) {  // small direct DFT, exact twiddles
                    cplx acc = 0;
                    for (int r = 0; r < R; ++r) {
                        cplx w = tw[(size_t)((r * q) % R) * (n / R)];
                        if (inverse) w = std::conj(w);
                        acc += v[r] * w;
                    }
                    y[q] = acc;
                }
                const int base = (j / Ns) * Ns * R + k;
                for (int r = 0; r < R; ++r) dst[base + r * Ns] = y[r];
            }
            std::swap(src, dst);
            Ns *= R;
        }
        if (src != a) std::memcpy(a, src, sizeof(cplx) * n);
    }
};

// 2-D DFT of rows x cols row-major; scale applied at the end
void fft2(std::vector<cplx> &a, int rows, int cols, bool inverse, double scale, const Fft &fr, const Fft &fc) {
    std::vector<cplx> s(std::max(rows, cols)), col(rows);
    for (int y = 0; y < rows; ++y) fr.run(&a[(size_t)y * cols], s.data(), inverse);
    for (int x = 0; x < cols; ++x) {
        for (int y = 0; y < rows; ++y) col[y] = a[(size_t)y * cols + x];
        fc.run(col.data(), s.data(), inverse);
        for (int y = 0; y < rows; ++y) a[(size_t)y * cols + x] = col[y] * scale;
    }
}

// cvComplex fftShift on an even-sized array: quadrant swap into `out`
void fftshift(const std::vector<cplx> &in, std::vector<cplx> &out, int rows, int cols) {
    out.resize((size_t)rows * cols);
    for (int y = 0; y < rows; ++y) {
        const int ys = (y + rows / 2) % rows;
        for (int x = 0; x < cols; ++x) out[(size_t)ys * cols + (x + cols / 2) % cols] = in[(size_t)y * cols + x];
    }
}

struct Params {
    int np, L, n_stack, n_order, r, iters;
    const uint16_t *stack;
    const int *order, *x0, *y0;
    double d1, d2, eps;
    int all_ch;  // 1: cv::add(c2, double) acts on both channels (OpenCV default)
};

int run_one(const Params &P, double *objF_out, double *objCrop_out, double *pupil_out) {
    const int np = P.np, L = P.L;
    const size_t NN = (size_t)np * np, LL = (size_t)L * L;
    Fft fnp(np), fl(L);
    if (!fnp.ok() || !fl.ok() || (np & 1) || (L & 1) || P.n_order < 2) return -22;
    // :302-313 support = filled disk at (Np/2, Np/2), fftShift
    std::vector<cplx> planes0(NN, 0.0), support, pupil;
    const int c = np / 2;
    for (int y = 0; y < np; ++y)
        for (int x = 0; x < np; ++x)
            if ((x - c) * (x - c) + (y - c) * (y - c) <= P.r * P.r) planes0[(size_t)y * np + x] = 1.0;
    fftshift(planes0, support, np, np);
    pupil = support;
    // :319-327
    const uint16_t *I0 = P.stack + (size_t)P.order[1] * NN;
    std::vector<cplx> ci(NN), tmp, tmp2;
    for (size_t i = 0; i < NN; ++i) ci[i] = std::sqrt((double)I0[i]);
    fft2(ci, np, np, false, 1.0, fnp, fnp);
    for (size_t i = 0; i < NN; ++i) ci[i] *= support[i];
    fftshift(ci, tmp, np, np);
    // :330-343
    std::vector<cplx> objF(LL, 0.0), objFc;
    const int c0 = L / 2 - np / 2;
    for (int y = 0; y < np; ++y)
        for (int x = 0; x < np; ++x) objF[(size_t)(c0 + y) * L + c0 + x] = tmp[(size_t)y * np + x];
    fftshift(objF, objFc, L, L);
    objF.swap(objFc);

    std::vector<cplx> roi(NN), objfcrop, objfcropP(NN), objcropP, objfup, pabs(NN), pconj(NN), num(NN), dO(NN),
        oabs(NN), oconj(NN), dP(NN), amp(NN), objCrop;
    std::vector<double> objf_abs(LL);
    for (int itr = 1; itr <= P.iters; ++itr) {
        for (int ii = 0; ii < P.n_order; ++ii) {
            const int led = P.order[ii];
            const int xs = P.x0[led], ys = P.y0[led];
            // :358-362
            fftshift(objF, objFc, L, L);
            for (int y = 0; y < np; ++y)
                for (int x = 0; x < np; ++x) roi[(size_t)y * np + x] = objFc[(size_t)(ys + y) * L + xs + x];
            fftshift(roi, objfcrop, np, np);
            // :364-365
            for (size_t i = 0; i < NN; ++i) objfcropP[i] = objfcrop[i] * pupil[i];
            objcropP = objfcropP;
            fft2(objcropP, np, np, true, 1.0 / (double)NN, fnp, fnp);
            // :378-387
            const uint16_t *I = P.stack + (size_t)led * NN;
            for (size_t i = 0; i < NN; ++i) amp[i] = cplx(std::sqrt((double)I[i]), 0.0);
            // :390-394
            tmp.resize(NN);
            const double sim = P.all_ch ? 1.0 : 0.0;  // imaginary share of a cv::add scalar
            for (size_t i = 0; i < NN; ++i) tmp[i] = objcropP[i] + cplx(P.eps, sim * P.eps);
            for (size_t i = 0; i < NN; ++i) tmp[i] = cplx(std::abs(tmp[i]), 0.0);
            for (size_t i = 0; i < NN; ++i) tmp[i] = objcropP[i] / tmp[i];
            for (size_t i = 0; i < NN; ++i) tmp[i] = tmp[i] * amp[i];
            objfup = tmp;
            fft2(objfup, np, np, false, 1.0, fnp, fnp);
            // :405-419 object update
            double pmax = 0.0;
            for (size_t i = 0; i < NN; ++i) {
                pabs[i] = cplx(std::abs(pupil[i]), 0.0);
                pconj[i] = std::conj(pupil[i]);
            }
            for (size_t i = 0; i < NN; ++i) num[i] = pabs[i] * pconj[i];
            for (size_t i = 0; i < NN; ++i) dO[i] = objfup[i] - objfcropP[i];
            for (size_t i = 0; i < NN; ++i) num[i] = dO[i] * num[i];
            for (size_t i = 0; i < NN; ++i) pmax = std::max(pmax, pabs[i].real());
            for (size_t i = 0; i < NN; ++i) dO[i] = ((pabs[i] * pabs[i]) + cplx(P.d2, sim * P.d2)) * pmax;
            for (size_t i = 0; i < NN; ++i) dO[i] = num[i] / dO[i];
            // :427-447
            fftshift(objF, objFc, L, L);
            fftshift(dO, tmp2, np, np);
            for (int y = 0; y < np; ++y)
                for (int x = 0; x < np; ++x) {
                    cplx &o = objFc[(size_t)(ys + y) * L + xs + x];
                    o = tmp2[(size_t)y * np + x] + o;
                }
            fftshift(objFc, objF, L, L);
            // :457-475 pupil update (pre-update objfcrop)
            double omax = 0.0;
            for (size_t i = 0; i < NN; ++i) {
                oabs[i] = cplx(std::abs(objfcrop[i]), 0.0);
                oconj[i] = std::conj(objfcrop[i]);
            }
            for (size_t i = 0; i < LL; ++i) objf_abs[i] = std::abs(objF[i]);
            for (size_t i = 0; i < NN; ++i) num[i] = oabs[i] * oconj[i];
            for (size_t i = 0; i < NN; ++i) dP[i] = objfup[i] - objfcropP[i];
            for (size_t i = 0; i < NN; ++i) num[i] = dP[i] * num[i];
            for (size_t i = 0; i < LL; ++i) omax = std::max(omax, objf_abs[i]);
            for (size_t i = 0; i < NN; ++i) dP[i] = ((oabs[i] * oabs[i]) + cplx(P.d1, sim * P.d1)) * omax;
            for (size_t i = 0; i < NN; ++i) dP[i] = num[i] / dP[i];
            for (size_t i = 0; i < NN; ++i) dP[i] = dP[i] * support[i];
            for (size_t i = 0; i < NN; ++i) pupil[i] = pupil[i] + dP[i];
        }
        // :481
        objCrop = objF;
        fft2(objCrop, L, L, true, 1.0 / (double)LL, fl, fl);
    }
    if (P.iters <= 0) {
        objCrop = objF;
        fft2(objCrop, L, L, true, 1.0 / (double)LL, fl, fl);
    }
    // :496 centred pupil
    std::vector<cplx> pc;
    fftshift(pupil, pc, np, np);
    if (objF_out) std::memcpy(objF_out, objF.data(), LL * sizeof(cplx));
    if (objCrop_out) std::memcpy(objCrop_out, objCrop.data(), LL * sizeof(cplx));
    if (pupil_out) std::memcpy(pupil_out, pc.data(), NN * sizeof(cplx));
    return 0;
}

}  // namespace

extern "C" {

// stack: uint16 [n_stack][Np][Np]; outputs complex128 interleaved (may be NULL)
int oracle_run_fpm(int np, int L, int n_stack, const uint16_t *stack, int n_order, const int *order,
                   const int *x0, const int *y0, int radius, double delta1, double delta2, double eps, int iters,
                   int all_channels, double *objF, double *objCrop, double *pupil) {
    Params P{np, L, n_stack, n_order, radius, iters, stack, order, x0, y0, delta1, delta2, eps, all_channels};
    return run_one(P, objF, objCrop, pupil);
}

// n_patch patches, stack LED-major [n_stack][n_patch][Np][Np] (the HIP layout);
// patches are spread over n_threads std::threads.  Outputs per patch.
int oracle_run_fpm_batch(int np, int L, int n_stack, int n_patch, const uint16_t *stack, int n_order,
                         const int *order, const int *x0, const int *y0, int radius, double delta1, double delta2,
                         double eps, int iters, int all_channels, int n_threads, double *objF, double *objCrop,
                         double *pupil) {
    const size_t NN = (size_t)np * np, LL = (size_t)L * L;
    std::vector<int> rc(n_patch, 0);
    auto work = [&](int t) {
        std::vector<uint16_t> own((size_t)n_stack * NN);
        for (int b = t; b < n_patch; b += n_threads) {
            for (int s = 0; s < n_stack; ++s)
                std::memcpy(&own[(size_t)s * NN], stack + ((size_t)s * n_patch + b) * NN, NN * sizeof(uint16_t));
            Params P{np, L, n_stack, n_order, radius, iters, own.data(), order, x0, y0, delta1, delta2, eps,
                     all_channels};
            rc[b] = run_one(P, objF ? objF + 2 * LL * b : nullptr, objCrop ? objCrop + 2 * LL * b : nullptr,
                            pupil ? pupil + 2 * NN * b : nullptr);
        }
    };
    if (n_threads < 1) n_threads = 1;
    std::vector<std::thread> th;
    for (int t = 0; t < n_threads; ++t) th.emplace_back(work, t);
    for (auto &x : th) x.join();
    for (int v : rc)
        if (v) return v;
    return 0;
}

// KAT hook: in-place 2-D DFT (complex128 interleaved), inverse scaled by 1/(rows*cols)
int oracle_fft2(double *data, int rows, int cols, int inverse) {
    Fft fr(cols), fc(rows);
    if (!fr.ok() || !fc.ok()) return -22;
    std::vector<cplx> a((size_t)rows * cols);
    std::memcpy(a.data(), data, a.size() * sizeof(cplx));
    fft2(a, rows, cols, inverse != 0, inverse ? 1.0 / ((double)rows * cols) : 1.0, fr, fc);
    std::memcpy(data, a.data(), a.size() * sizeof(cplx));
    return 0;
}

}  // extern "C"
