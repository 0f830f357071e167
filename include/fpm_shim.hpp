/*
 * fpm_shim.hpp -- reference-side binding of runFPM onto the C ABI.
 *
 * Replaces the body of the reference's
 *     void runFPM(FPM_Dataset *dataset);     fpmMain.h:119, fpmMain.cpp:274-498
 * with create / upload / init / run / download on libfpm_hip.so
 * (include/fpm_hip.h).  Header-only and free of OpenCV: the caller passes two
 * small adapters for its image type (INTEGRATION.md has the cv::UMat ones),
 * so the same code is compiled by the reference build and by the mock-dataset
 * test (tests/shim/mock_runfpm.cpp).
 *
 * What it reads from FPM_Dataset (fpmMain.h:43-101), exactly as runFPM does:
 *   Np, Nlarge, objectiveNA, ps_eff, lambda, delta1, delta2, eps, itrCount,
 *   ledUsedCount, sortedIndicies, imageStack[led].{Image, cropXStart,
 *   cropYStart}.
 * imageStack is indexed by LED NUMBER with ledCount+1 slots (slot 0 is a
 * dummy, fpmMain.cpp:49-57); slots of unused LEDs keep the CV_8UC1 zero image
 * of fpmMain.cpp:42 with indeterminate crop offsets.  Only the
 * sortedIndicies[0..ledUsedCount) slots are touched: their images are copied
 * into a compact stack in processing order (stack index i = sortedIndicies[i],
 * so fpm_problem.order = 0..n-1) and only their crops are passed on.
 *
 * Adapters:
 *   bool copy_image(const Img &slot, uint16_t *dst, int np)
 *        copy slot.Image (must be 16-bit, Np x Np) row-major into dst;
 *        false if it is not (the reference's uint16 reads, fpmMain.cpp:380,
 *        would misread it too)
 *   void store(const float *objF, const float *objCrop, const float *pupil,
 *              const float *support, int L, int np)
 *        interleaved complex64 objF / objCrop [L][L], centred pupil [Np][Np]
 *        (fpmMain.cpp:496), real support [Np][Np] (un-centred pupilSupport,
 *        fpmMain.cpp:310-313); convert into the dataset's CV_64FC2 members.
 * Log lines are the reference's (fpmMain.cpp:477-479, 489-490), wall time.
 * Returns FPM_OK or the fpm_hip error code (runFPM itself would throw).
 */
#ifndef FPM_SHIM_HPP
#define FPM_SHIM_HPP

#include <chrono>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <ostream>
#include <vector>

#include "fpm_hip.h"

namespace fpm_shim {

// naRadius exactly as fpmMain.cpp:304-305 computes it (the dataset's own
// float fields, int16 truncation of ceil)
template <class Dataset>
int na_radius(const Dataset *d) {
    return (int16_t)std::ceil(d->objectiveNA * d->ps_eff * d->Np / d->lambda);
}

template <class Dataset, class CopyImage, class Store>
int runFPM(Dataset *d, CopyImage &&copy_image, Store &&store, std::ostream &log, int device = 0,
           int path = FPM_PATH_AUTO) {
    using clk = std::chrono::steady_clock;
    const auto t_all = clk::now();
    const int np = d->Np, L = d->Nlarge, n = d->ledUsedCount;
    if (n < 2 || (int)d->sortedIndicies.size() < n) {  // sortedIndicies.at(1) (:319)
        log << "runFPM: ledUsedCount " << n << " with " << d->sortedIndicies.size() << " sorted indices" << std::endl;
        return FPM_ERR_INVAL;
    }
    std::vector<int32_t> order(n), x0(n), y0(n);
    std::vector<uint16_t> stack((size_t)n * np * np);
    for (int i = 0; i < n; ++i) {
        const int led = d->sortedIndicies[i];  // :350
        if (led < 0 || led >= (int)d->imageStack.size()) {
            log << "runFPM: sortedIndicies[" << i << "] = " << led << " outside imageStack" << std::endl;
            return FPM_ERR_INVAL;
        }
        const auto &slot = d->imageStack[led];
        if (!copy_image(slot, &stack[(size_t)i * np * np], np)) {
            log << "runFPM: image of LED " << led << " is not a 16-bit " << np << "x" << np << " image" << std::endl;
            return FPM_ERR_INVAL;
        }
        order[i] = i;
        x0[i] = slot.cropXStart;  // :157-159
        y0[i] = slot.cropYStart;  // :163-165
    }
    fpm_problem p;
    std::memset(&p, 0, sizeof p);
    p.np = np;
    p.nlarge = L;
    p.n_stack = n;
    p.n_order = n;
    p.order = order.data();
    p.crop_x0 = x0.data();
    p.crop_y0 = y0.data();
    p.na_radius = na_radius(d);
    p.init_pos = 1;  // sortedIndicies.at(1) (:319)
    p.delta1 = d->delta1;
    p.delta2 = d->delta2;
    p.eps = d->eps;  // float eps = 1e-10 (fpmMain.h:99)
    p.n_patch = 1;
    p.path = path;
    fpm_ctx *ctx = nullptr;
    int rc = fpm_create(&p, device, &ctx);
    if (!rc) rc = fpm_upload_stack(ctx, stack.data());
    if (!rc) rc = fpm_init(ctx);  // :300-343
    for (int itr = 1; !rc && itr <= d->itrCount; ++itr) {  // :345-482
        const auto t1 = clk::now();
        rc = fpm_run(ctx, 1);
        if (!rc)
            log << "Iteration " << itr << " Completed (Time: "
                << std::chrono::duration<float>(clk::now() - t1).count() << " sec)" << std::endl;
    }
    std::vector<float> objF(2 * (size_t)L * L), objCrop(2 * (size_t)L * L), pupil(2 * (size_t)np * np),
        support((size_t)np * np);
    if (!rc) rc = fpm_download(ctx, objF.data(), objCrop.data(), pupil.data(), support.data());
    if (rc) log << "runFPM: " << fpm_last_error() << std::endl;
    fpm_destroy(ctx);
    if (rc) return rc;
    log << "FP Processing Completed (Time: " << std::chrono::duration<float>(clk::now() - t_all).count()
        << " sec)" << std::endl;
    store(objF.data(), objCrop.data(), pupil.data(), support.data(), L, np);
    return FPM_OK;
}

}  // namespace fpm_shim

#endif  // FPM_SHIM_HPP
