// api.cpp -- the extern "C" boundary of libfpm_hip.so (include/fpm_hip.h).
//
// Mirrors runFPM(FPM_Dataset*) (fpmMain.cpp:274-498): fpm_init performs the
// pupil/spectrum initialisation (fpmMain.cpp:302-343), fpm_run the
// itrCount x ledUsedCount update loop and the per-iteration objCrop IDFT
// (fpmMain.cpp:345-482), fpm_download hands back objF / objCrop / pupil /
// pupilSupport in the reference's conventions.  Errors are negative codes plus
// fpm_last_error(); nothing here ever falls back to a CPU path.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdlib>
#include <cstdarg>
#include <cstddef>
#include <cstdio>
#include <algorithm>
#include <mutex>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/fpm_hip.h"
#include "../../include/fpm_hip_debug.h"
#include "fft_lds.hpp"
#include "fpm_state.hpp"

namespace fpm {
hipError_t launch_general_step(const DevState &st, int led, int x0, int y0, const FftPlan &pl,
                               const float2 *tw, bool first, hipStream_t s);
hipError_t launch_pupil_commit(const DevState &st, hipStream_t s);
int fft_max_len();
int pupil_parts(int nb);
hipError_t launch_init(const DevState &st, int init_led, float2 *scratch, const FftPlan &pl_np,
                       const float2 *tw_np, hipStream_t s);
hipError_t launch_objcrop(const DevState &st, float2 *out, const FftPlan &pl_L, const float2 *tw_L,
                          hipStream_t s);
// fused path (fpm_fused.hip)
int fused_threads(int np, int r, int L, const DevState &st);
// Np 200 fused kernel (fused_mr.hip)
bool fused_mr_supported(int np, int r, const DevState &st);
hipError_t launch_fused_mr_iteration(const DevState &st, const uint16_t *meas, const int *order_dev,
                                     const int *x0_dev, const int *y0_dev, int n_order, const float2 *tw_np,
                                     unsigned long long *dbg, hipStream_t s);
// Np 90 fused kernel (fused_s90.hip)
bool fused_s90_supported(int np, int r, const DevState &st);
hipError_t launch_fused_s90_iteration(const DevState &st, const uint16_t *meas, const int *order_dev,
                                      const int *x0_dev, const int *y0_dev, int n_order, const float2 *tw_np,
                                      unsigned long long *dbg, hipStream_t s);
// small-patch fused kernel (fused_small.hip, Np <= 96)
bool fused_small_supported(int np, int r, const DevState &st);
hipError_t launch_fused_small_iteration(const DevState &st, const uint16_t *meas, const int *order_dev,
                                        const int *x0_dev, const int *y0_dev, int n_order, const float2 *tw_np,
                                        const FftPlan &pl, unsigned long long *dbg, hipStream_t s);
// Np 1024 / Np 256 register row/column kernels of the general path
// (np1024.hip, np256.hip; both fold the pupil commit into the next LED)
bool np1024_supported(int np, int r);
bool np256_supported(int np, int r, int L, bool fp16);
bool commit_folded(const DevState &st);
hipError_t launch_fused_iteration(const DevState &st, const uint16_t *meas, const int *order_dev,
                                  const int *x0_dev, const int *y0_dev, int n_order, const float2 *tw_np,
                                  int ks, unsigned long long *dbg, float2 *xch, int *flags, int stall_led,
                                  hipStream_t s);
size_t fused_xch_elems(int B, int ks);
size_t fused_flag_words(int B, int ks);
int fused_split_parts(int nt, int B, int n_cu);
// distributed mode of the Np 256 kernel (fused_dist.hip)
size_t fused_dist_elems(int B, int ks);
int fused_dist_parts(int B, int n_cu, int r, int L);
hipError_t launch_fused_dist(const DevState &st, const uint16_t *meas, const int *order_dev, const int *x0_dev,
                             const int *y0_dev, int n_order, const float2 *tw_np, int ks, unsigned long long *dbg,
                             float2 *area, int *flags, int stall_led, unsigned tag_base, hipStream_t s);
// in-place measurement layout of the fused kernels (preprocess.hip)
hipError_t meas_layout(uint16_t *meas, int np, int g, size_t nimg, bool fwd, hipStream_t s);
bool meas_layout_copy(const uint16_t *src, uint16_t *dst, int np, int g, size_t nimg, hipStream_t s,
                      hipError_t *err);
hipError_t launch_preprocess_frame(const uint16_t *frame, int width, int np, int B, const int *px0_dev,
                                   const int *py0_dev, int bk1x, int bk1y, int bk2x, int bk2y, double bg_threshold,
                                   double dark_mult, bool darkfield, unsigned long long *sums, uint16_t *out,
                                   int16_t *bg_out_dev, hipStream_t s);
size_t fused_T_elems(int np, int r, int B);

// Co-resident grids (split / distributed modes, fused_sync.hpp): the
// occupancy check, then a plain launch ordered after the previous co-resident
// grid of this process on the same device (another context, another stream),
// so two grids that each need every block resident never share the device.
// A capturing stream is refused (hipErrorStreamCaptureUnsupported): an event
// recorded outside the capture cannot be waited on inside it, so a replayed
// graph would carry no such order (fpm_run refuses capture before this).
// Only co-resident grids are ordered against each other; other kernels on
// other streams may still hold CUs, and then the waits' ~1 s timeout reports
// the launch.
hipError_t launch_coresident_raw(const void *fn, int grid, int block, size_t lds, void **args, hipStream_t s) {
    int dev = 0, n_cu = 0, per_cu = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e == hipSuccess) e = hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev);
    if (e == hipSuccess) e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, block, lds);
    if (e != hipSuccess) return e;
    if ((long long)per_cu * n_cu < grid) return hipErrorCooperativeLaunchTooLarge;
    hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
    if ((e = hipStreamIsCapturing(s, &cap)) != hipSuccess) return e;
    if (cap != hipStreamCaptureStatusNone) return hipErrorStreamCaptureUnsupported;
    constexpr int kMaxDev = 64;
    struct Serial {
        std::mutex mu;
        hipEvent_t last = nullptr;  // completion of the device's latest co-resident grid
    };
    static Serial serial[kMaxDev];
    if (dev < 0 || dev >= kMaxDev) return hipErrorInvalidDevice;
    Serial &sd = serial[dev];
    std::lock_guard<std::mutex> lk(sd.mu);
    if (!sd.last && (e = hipEventCreateWithFlags(&sd.last, hipEventDisableTiming)) != hipSuccess) {
        sd.last = nullptr;
        return e;
    }
    // an event never recorded counts as complete, so the first wait is free
    if ((e = hipStreamWaitEvent(s, sd.last, 0)) != hipSuccess) return e;
    if ((e = hipLaunchKernel(fn, dim3(grid), dim3(block), args, lds, s)) != hipSuccess) return e;
    if (hipEventRecord(sd.last, s) != hipSuccess) {
        // the grid is running but the next co-resident grid could not be
        // ordered after it: drain the stream here instead (the event, never
        // re-recorded, still reads complete), so the launch itself succeeds
        (void)hipStreamSynchronize(s);
    }
    return hipSuccess;
}
}  // namespace fpm

using namespace fpm;

namespace {

thread_local std::string g_err;

int set_err(int code, const char *fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

#define HIP_TRY(expr)                                                                          \
    do {                                                                                       \
        hipError_t e_ = (expr);                                                                \
        if (e_ != hipSuccess)                                                                  \
            return set_err(FPM_ERR_DEVICE, "%s failed: %s (%s:%d)", #expr, hipGetErrorString(e_), \
                           __FILE__, __LINE__);                                                \
    } while (0)

bool make_plan(int n, FftPlan *pl) {
    std::memset(pl, 0, sizeof *pl);
    pl->n = n;
    int m = n, k = 0;
    while (m % 8 == 0) { pl->radix[k++] = 8; m /= 8; }
    while (m % 4 == 0) { pl->radix[k++] = 4; m /= 4; }
    while (m % 2 == 0) { pl->radix[k++] = 2; m /= 2; }
    while (m % 3 == 0) { pl->radix[k++] = 3; m /= 3; }
    while (m % 5 == 0) { pl->radix[k++] = 5; m /= 5; }
    pl->nstages = k;
    return m == 1 && k < 24;
}

std::vector<float2> twiddles(int n) {
    std::vector<float2> t(n);
    for (int k = 0; k < n; ++k) {
        const double a = -2.0 * M_PI * (double)k / (double)n;
        t[k] = make_float2((float)std::cos(a), (float)std::sin(a));
    }
    return t;
}

}  // namespace

struct fpm_ctx {
    fpm_problem prob{};
    std::vector<int32_t> order, x0, y0;
    int device = 0;
    hipStream_t stream = nullptr;
    hipStream_t own_stream = nullptr;
    DevState st{};
    int path = FPM_PATH_GENERAL;
    int support_px = 0;
    FftPlan pl_np{}, pl_L{};
    float2 *tw_np = nullptr, *tw_L = nullptr;
    float2 *objcrop = nullptr;
    uint16_t *meas = nullptr;
    int meas_g = 0;                 // meas holds the column layout of meas_layout with g-lane groups
                                    // once uploaded (16: Np 256, 10: Np 200, Np: the small-patch
                                    // kernel and the Np 1024 general path, transposed); 0: C-ABI
    int fused_nt = 0;               // Np 256 fused kernel: threads per workgroup (512), 0 = not used
    int split_ks = 1;               // split / distributed mode: workgroups per patch (2, 4, 8), else 1
    bool dist = false;              // distributed mode (fused_dist.hip) instead of split mode
    float2 *xch = nullptr;          //   exchange area
    int *split_flags = nullptr;     //   handoff flags [KS B] + sticky abort flag + XCC ids [KS B]
    int stall_led = -1;             //   fpm_debug_set_stall (tests): the last part stops publishing
    unsigned dist_tags = 0;         //   distributed mode: LEDs launched so far (tile-word tags)
    bool fused_mr = false;          // fused path runs the Np 200 kernel (fused_mr.hip)
    bool fused_small = false;       // fused path runs the small-patch kernel (fused_small.hip)
    bool fused_s90 = false;         // fused path runs the Np 90 kernel (fused_s90.hip)
    int *order_dev = nullptr, *x0_dev = nullptr, *y0_dev = nullptr;
    uint8_t *disk_dev = nullptr;
    std::vector<void *> allocs;
    size_t bytes = 0;
    bool uploaded = false, initialized = false, objcrop_valid = false;
    std::vector<hipEvent_t> evpool;
    unsigned long long *dbg = nullptr;  // FPM_STAMPS=1: fused-kernel phase cycles
    unsigned long long *clk = nullptr;  // fused kernels' launch clock probe [3] (ClockProbe)
    fpm_clock clock{};                  // of the most recent fpm_run
    fpm_timing timing{};
    // general path: one iteration's 4*n_order launches captured once and
    // replayed as a single graph launch (FPM_NO_GRAPH=1 launches them directly)
    // general path: the patches split into ngroups groups whose LED chains run
    // on concurrent streams (forked from and joined back to the run stream), so
    // one group's launches fill the other's partial last round of workgroups;
    // one captured graph per group
    int ngroups = 1;
    static constexpr int kMaxGroups = 8;
    hipGraph_t led_graph[kMaxGroups] = {};
    hipGraphExec_t led_graph_exec[kMaxGroups] = {};
    hipStream_t gstream[kMaxGroups] = {};
    hipEvent_t gfork = nullptr, gjoin[kMaxGroups] = {};
};

namespace {

template <typename T>
int dalloc(fpm_ctx *c, T **p, size_t count) {
    void *q = nullptr;
    const size_t nb = count * sizeof(T);
    hipError_t e = hipMalloc(&q, nb > 0 ? nb : 16);
    if (e != hipSuccess) return set_err(FPM_ERR_NOMEM, "hipMalloc(%zu) failed: %s", nb, hipGetErrorString(e));
    c->allocs.push_back(q);
    c->bytes += nb;
    *p = (T *)q;
    return FPM_OK;
}

void free_all(fpm_ctx *c) {
    for (int g = 0; g < fpm_ctx::kMaxGroups; ++g) {
        if (c->led_graph_exec[g]) (void)hipGraphExecDestroy(c->led_graph_exec[g]);
        if (c->led_graph[g]) (void)hipGraphDestroy(c->led_graph[g]);
        c->led_graph_exec[g] = nullptr;
        c->led_graph[g] = nullptr;
    }
    for (void *p : c->allocs) (void)hipFree(p);
    c->allocs.clear();
    for (auto e : c->evpool) (void)hipEventDestroy(e);
    c->evpool.clear();
    for (int g = 0; g < fpm_ctx::kMaxGroups; ++g) {
        if (c->gstream[g]) (void)hipStreamDestroy(c->gstream[g]);
        if (c->gjoin[g]) (void)hipEventDestroy(c->gjoin[g]);
        c->gstream[g] = nullptr;
        c->gjoin[g] = nullptr;
    }
    if (c->gfork) (void)hipEventDestroy(c->gfork);
    c->gfork = nullptr;
    if (c->own_stream) (void)hipStreamDestroy(c->own_stream);
}

int validate(const fpm_problem *p) {
    if (!p) return set_err(FPM_ERR_INVAL, "null problem");
    if (p->np < 4 || (p->np & 1)) return set_err(FPM_ERR_INVAL, "Np=%d must be even and >= 4", p->np);
    if (p->nlarge < p->np || (p->nlarge & 1))
        return set_err(FPM_ERR_INVAL, "Nlarge=%d must be even and >= Np", p->nlarge);
    FftPlan t;
    if (!make_plan(p->np, &t)) return set_err(FPM_ERR_INVAL, "Np=%d is not 2^a 3^b 5^c", p->np);
    if (!make_plan(p->nlarge, &t)) return set_err(FPM_ERR_INVAL, "Nlarge=%d is not 2^a 3^b 5^c", p->nlarge);
    if (p->nlarge > fft_max_len())
        return set_err(FPM_ERR_INVAL, "Nlarge=%d exceeds the batched transform limit %d", p->nlarge, fft_max_len());
    if (p->na_radius < 0 || 2 * p->na_radius + 1 > p->np)
        return set_err(FPM_ERR_INVAL, "naRadius=%d needs 2r+1 <= Np=%d", p->na_radius, p->np);
    if (p->n_stack < 1 || p->n_order < 2)
        return set_err(FPM_ERR_INVAL, "need n_stack>=1 and ledUsedCount>=2 (init uses sortedIndicies.at(1))");
    if (!p->order || !p->crop_x0 || !p->crop_y0) return set_err(FPM_ERR_INVAL, "null order/crop arrays");
    if (p->init_pos < 0 || p->init_pos >= p->n_order) return set_err(FPM_ERR_INVAL, "init_pos out of range");
    if (!(p->delta2 > 0.0))
        return set_err(FPM_ERR_INVAL, "delta2=%g: the reference divides 0/0 outside the support when delta2==0",
                       p->delta2);
    if (!(p->delta1 > 0.0)) return set_err(FPM_ERR_INVAL, "delta1=%g must be > 0", p->delta1);
    if (p->n_patch < 1) return set_err(FPM_ERR_INVAL, "n_patch=%d", p->n_patch);
    for (int i = 0; i < p->n_order; ++i)
        if (p->order[i] < 0 || p->order[i] >= p->n_stack)
            return set_err(FPM_ERR_INVAL, "order[%d]=%d outside the stack", i, p->order[i]);
    for (int i = 0; i < p->n_stack; ++i) {
        // cv::Rect(cropXStart, cropYStart, Np, Np) must lie inside objF (fpmMain.cpp:361)
        if (p->crop_x0[i] < 0 || p->crop_x0[i] > p->nlarge - p->np || p->crop_y0[i] < 0 ||
            p->crop_y0[i] > p->nlarge - p->np)
            return set_err(FPM_ERR_INVAL, "LED %d crop (%d,%d) leaves the %dx%d spectrum", i, p->crop_x0[i],
                           p->crop_y0[i], p->nlarge, p->nlarge);
    }
    return FPM_OK;
}

}  // namespace

namespace {
// device scratch owned by one fpm_upload_frames call
struct Scratch {
    std::vector<void *> p;
    ~Scratch() {
        for (void *q : p) (void)hipFree(q);
    }
    template <typename T>
    hipError_t get(T **out, size_t n) {
        void *q = nullptr;
        hipError_t e = hipMalloc(&q, n * sizeof(T) > 0 ? n * sizeof(T) : 16);
        if (e == hipSuccess) p.push_back(q);
        *out = (T *)q;
        return e;
    }
};
}  // namespace


extern "C" {

const char *fpm_last_error(void) { return g_err.c_str(); }

const char *fpm_version(void) { return "libfpm_hip 0.2 (gfx950, fp32 complex state, optional fp16 spectrum storage)"; }

int fpm_create(const fpm_problem *prob, int device, fpm_ctx **out) {
    if (!out) return set_err(FPM_ERR_INVAL, "null out");
    *out = nullptr;
    int rc = validate(prob);
    if (rc) return rc;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0)
        return set_err(FPM_ERR_NODEV, "no HIP device visible");
    if (device < 0 || device >= ndev) return set_err(FPM_ERR_NODEV, "device %d of %d", device, ndev);
    hipDeviceProp_t pr;
    HIP_TRY(hipGetDeviceProperties(&pr, device));
    if (std::strncmp(pr.gcnArchName, "gfx950", 6) != 0)
        return set_err(FPM_ERR_NODEV, "device %d is %s, this library is built for gfx950", device, pr.gcnArchName);
    HIP_TRY(hipSetDevice(device));

    fpm_ctx *c = new fpm_ctx();
    c->prob = *prob;
    c->device = device;
    c->order.assign(prob->order, prob->order + prob->n_order);
    c->x0.assign(prob->crop_x0, prob->crop_x0 + prob->n_stack);
    c->y0.assign(prob->crop_y0, prob->crop_y0 + prob->n_stack);
    c->prob.order = c->order.data();
    c->prob.crop_x0 = c->x0.data();
    c->prob.crop_y0 = c->y0.data();

    auto fail = [&](int code) {
        free_all(c);
        delete c;
        return code;
    };
    if (hipStreamCreateWithFlags(&c->own_stream, hipStreamNonBlocking) != hipSuccess)
        return fail(set_err(FPM_ERR_DEVICE, "hipStreamCreate failed"));
    c->stream = c->own_stream;

    const int np = prob->np, L = prob->nlarge, r = prob->na_radius, nb = 2 * r + 1, B = prob->n_patch;
    DevState &st = c->st;
    st.np = np;
    st.L = L;
    st.r = r;
    st.nb = nb;
    st.B = B;
    st.mB = B;
    st.ntx = (L + kTile - 1) / kTile;
    st.nty = st.ntx;
    st.delta1 = (float)prob->delta1;
    st.delta2 = (float)prob->delta2;
    st.eps = (float)prob->eps;
    {   // cv::add(UMat CV_64FC2, double) semantics (fpm_hip.h FPM_FLAG_SCALAR_RE_ONLY)
        const bool re_only = (prob->flags & FPM_FLAG_SCALAR_RE_ONLY) != 0;
        st.eps_im = re_only ? 0.f : st.eps;
        st.d1_im = re_only ? 0.f : st.delta1;
        st.d2_im = re_only ? 0.f : st.delta2;
    }
    make_plan(np, &c->pl_np);
    make_plan(L, &c->pl_L);
    // live band of the centred spectrum (fpm_state.hpp): the init placement at
    // L/2 (fpmMain.cpp:332-343) and every used LED's support box (:405-447)
    st.sy0 = st.sx0 = L / 2 - r;
    st.sy1 = st.sx1 = L / 2 + r;
    for (int i = 0; i < prob->n_order; ++i) {
        const int led = c->order[i];
        st.sy0 = std::min(st.sy0, c->y0[led] + np / 2 - r);
        st.sy1 = std::max(st.sy1, c->y0[led] + np / 2 + r);
        st.sx0 = std::min(st.sx0, c->x0[led] + np / 2 - r);
        st.sx1 = std::max(st.sx1, c->x0[led] + np / 2 + r);
    }
    st.sy0 = std::max(st.sy0, 0);
    st.sx0 = std::max(st.sx0, 0);
    st.sy1 = std::min(st.sy1, L - 1);
    st.sx1 = std::min(st.sx1, L - 1);

    // support disk on the box: Euclidean disk == filled cv::circle (fpmMain.cpp:307)
    std::vector<uint8_t> disk((size_t)nb * nb);
    for (int i = 0; i < nb; ++i)
        for (int j = 0; j < nb; ++j) {
            const int ky = i - r, kx = j - r;
            disk[(size_t)i * nb + j] = (ky * ky + kx * kx <= r * r) ? 1 : 0;
            c->support_px += disk[(size_t)i * nb + j];
        }

    const bool fp16 = (prob->flags & FPM_FLAG_SPEC_FP16) != 0;
    c->fused_nt = fused_threads(np, r, L, st);
    c->fused_mr = !c->fused_nt && fused_mr_supported(np, r, st);
    // Np 90 (configs 1 / 2): the register-transform kernel unless FPM_NO_S90=1
    // selects the generic small-patch kernel
    c->fused_s90 = !c->fused_nt && !c->fused_mr && !getenv("FPM_NO_S90") && fused_s90_supported(np, r, st);
    c->fused_small = !c->fused_nt && !c->fused_mr && !c->fused_s90 && fused_small_supported(np, r, st);
    const bool fused_ok = c->fused_nt || c->fused_mr || c->fused_s90 || c->fused_small;
    if (prob->path == FPM_PATH_FUSED && (fp16 || !fused_ok))
        return fail(set_err(FPM_ERR_INVAL, "fused path unsupported for Np=%d r=%d L=%d%s", np, r, L,
                            fp16 ? " with fp16 spectrum storage" : ""));
    c->path = (prob->path == FPM_PATH_GENERAL || fp16) ? FPM_PATH_GENERAL
              : fused_ok                               ? FPM_PATH_FUSED
                                                       : FPM_PATH_GENERAL;
    // fp16 storage scale: 2^-ceil(log2 Np^2) (fpm_state.hpp)
    int e2 = 0;
    while ((1ll << e2) < (long long)np * np) ++e2;
    st.hscale = std::ldexp(1.0f, -e2);
    st.hinv = std::ldexp(1.0f, e2);

    const size_t specn = (size_t)B * L * L;
    if (fp16) {
        if ((rc = dalloc(c, &st.spec16, specn))) return fail(rc);
    } else {
        if ((rc = dalloc(c, &st.spec, specn))) return fail(rc);
    }
    if ((rc = dalloc(c, &c->objcrop, specn))) return fail(rc);
    if ((rc = dalloc(c, &st.pupil, (size_t)B * nb * nb))) return fail(rc);
    if ((rc = dalloc(c, &st.tmax, (size_t)B * st.ntx * st.nty))) return fail(rc);
    if ((rc = dalloc(c, &st.tdirty, (size_t)B * ((st.ntx * st.nty + 31) / 32)))) return fail(rc);
    // Np 1024 general path: register row/column kernels reading the stack
    // transposed; Np 256 beyond the fused kernels' radius: register kernels
    // reading the fused column layout (g = 16).  Their row IDFT writes one
    // max|P| partial per box row
    const bool reg1024 = c->path == FPM_PATH_GENERAL && np1024_supported(np, r) && !getenv("FPM_NO_REG1024");
    const bool reg256 =
        c->path == FPM_PATH_GENERAL && np256_supported(np, r, L, fp16) && !getenv("FPM_NO_REG256");
    st.npart = (c->path == FPM_PATH_GENERAL) ? (reg1024 || reg256 ? std::max(pupil_parts(nb), nb) : pupil_parts(nb))
                                             : 1;
    if ((rc = dalloc(c, &st.pmax, (size_t)B * st.npart))) return fail(rc);
    if ((rc = dalloc(c, &c->disk_dev, disk.size()))) return fail(rc);
    if ((rc = dalloc(c, &c->meas, (size_t)prob->n_stack * B * np * np))) return fail(rc);
    if ((rc = dalloc(c, &c->order_dev, (size_t)prob->n_order))) return fail(rc);
    if ((rc = dalloc(c, &c->x0_dev, (size_t)prob->n_stack))) return fail(rc);
    if ((rc = dalloc(c, &c->y0_dev, (size_t)prob->n_stack))) return fail(rc);
    if (c->path == FPM_PATH_GENERAL) {
        if (reg1024) c->meas_g = np;
        if (reg256) c->meas_g = 16;
        // fp16 spectrum storage on the Np 1024 register kernels: the row /
        // column scratch T block-scaled in fp16 too (half its HBM traffic;
        // FPM_T32=1 keeps it fp32)
        if (reg1024 && fp16 && !getenv("FPM_T32")) {
            if ((rc = dalloc(c, &st.T16, (size_t)B * nb * np))) return fail(rc);
            if ((rc = dalloc(c, &st.tsr, (size_t)B * nb))) return fail(rc);
            if ((rc = dalloc(c, &st.tsc, (size_t)B * np))) return fail(rc);
        } else {
            if ((rc = dalloc(c, &st.T, (size_t)B * nb * np))) return fail(rc);
        }
        if ((rc = dalloc(c, &st.dP, (size_t)B * nb * nb))) return fail(rc);
        if ((rc = dalloc(c, &st.rmax, (size_t)B * st.nty))) return fail(rc);
        // patch groups on concurrent streams (FPM_PATCH_GROUPS=n overrides):
        // two for the Np 1024 kernels, whose row launches cover a few patches
        // in 1.3 rounds of workgroups (config 5, 8 patches: 65.5 -> 57.5 ms of
        // LED steps per iteration; 3 or 4 groups measured slower, 79 / 77 ms),
        // and for the Np 256 register kernels, whose three short launches per
        // LED then overlap one group's tail with the other's start (dataset_mono
        // at Np 256, 64 patches: 1.18 -> 1.25 M LED-updates/s)
        const char *pg = getenv("FPM_PATCH_GROUPS");
        c->ngroups = pg ? atoi(pg) : (reg1024 || reg256 ? 2 : 1);
        c->ngroups = std::max(1, std::min({c->ngroups, B, (int)fpm_ctx::kMaxGroups}));
        for (int g = 1; g < c->ngroups; ++g) {
            if (hipStreamCreateWithFlags(&c->gstream[g], hipStreamNonBlocking) != hipSuccess ||
                hipEventCreateWithFlags(&c->gjoin[g], hipEventDisableTiming) != hipSuccess)
                return fail(set_err(FPM_ERR_DEVICE, "patch-group stream / event creation failed"));
        }
        if (c->ngroups > 1 && hipEventCreateWithFlags(&c->gfork, hipEventDisableTiming) != hipSuccess)
            return fail(set_err(FPM_ERR_DEVICE, "patch-group event creation failed"));
    } else {
        c->meas_g = c->fused_small ? np : c->fused_s90 ? 9 : c->fused_mr ? 10 : 16;
        if ((rc = dalloc(c, &st.T, fused_T_elems(np, r, B)))) return fail(rc);
        int n_cu = 0;
        (void)hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, device);
        // small batches: every phase distributed over KS workgroups per patch
        // (fused_dist.hip), else split mode (column parts only), else one
        // workgroup per patch
        const int dks = c->fused_nt ? fused_dist_parts(B, n_cu, r, L) : 0;
        c->dist = dks > 1;
        c->split_ks = c->dist ? dks : c->fused_nt ? fused_split_parts(c->fused_nt, B, n_cu) : 1;
        if (c->split_ks > 1) {
            const size_t nx = c->dist ? fused_dist_elems(B, c->split_ks) : fused_xch_elems(B, c->split_ks);
            if ((rc = dalloc(c, &c->xch, nx))) return fail(rc);
            // distributed mode's tile words start at tag 0, which no LED uses
            if (hipMemset(c->xch, 0, nx * sizeof(float2)) != hipSuccess)
                return fail(set_err(FPM_ERR_DEVICE, "memset failed"));
            const size_t nf = fused_flag_words(B, c->split_ks);
            if ((rc = dalloc(c, &c->split_flags, nf))) return fail(rc);
            if (hipMemset(c->split_flags, 0, nf * sizeof(int)) != hipSuccess)
                return fail(set_err(FPM_ERR_DEVICE, "memset failed"));
        }
    }
    st.meas = c->meas;
    st.disk = c->disk_dev;
    if (c->path == FPM_PATH_FUSED) {
        if ((rc = dalloc(c, &c->clk, 3))) return fail(rc);
        if (hipMemset(c->clk, 0, 3 * sizeof(unsigned long long)) != hipSuccess)
            return fail(set_err(FPM_ERR_DEVICE, "memset failed"));
        st.clk = c->clk;
    }
    if (getenv("FPM_STAMPS") && c->path == FPM_PATH_FUSED) {
        if ((rc = dalloc(c, &c->dbg, 2 * kStamps))) return fail(rc);
        if (hipMemset(c->dbg, 0, 2 * kStamps * sizeof(unsigned long long)) != hipSuccess)
            return fail(set_err(FPM_ERR_DEVICE, "memset failed"));
    }
    auto twn = twiddles(np), twl = twiddles(L);
    if ((rc = dalloc(c, &c->tw_np, twn.size()))) return fail(rc);
    if ((rc = dalloc(c, &c->tw_L, twl.size()))) return fail(rc);
    if (hipMemcpy(c->tw_np, twn.data(), twn.size() * sizeof(float2), hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(c->tw_L, twl.data(), twl.size() * sizeof(float2), hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(c->disk_dev, disk.data(), disk.size(), hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(c->order_dev, c->order.data(), c->order.size() * sizeof(int), hipMemcpyHostToDevice) !=
            hipSuccess ||
        hipMemcpy(c->x0_dev, c->x0.data(), c->x0.size() * sizeof(int), hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(c->y0_dev, c->y0.data(), c->y0.size() * sizeof(int), hipMemcpyHostToDevice) != hipSuccess)
        return fail(set_err(FPM_ERR_DEVICE, "table upload failed"));
    *out = c;
    return FPM_OK;
}

void fpm_destroy(fpm_ctx *c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    free_all(c);
    delete c;
}

int fpm_set_stream(fpm_ctx *c, void *s) {
    if (!c) return set_err(FPM_ERR_INVAL, "null ctx");
    c->stream = s ? (hipStream_t)s : c->own_stream;
    return FPM_OK;
}

static int after_upload(fpm_ctx *c) {
    // the fused kernels read the stack column-major, permuted in place (2 B per pixel)
    if (c->meas_g)
        HIP_TRY(meas_layout(c->meas, c->st.np, c->meas_g, (size_t)c->prob.n_stack * c->st.B, true, c->stream));
    c->st.meas_g = c->meas_g;
    c->uploaded = true;
    c->initialized = false;
    return FPM_OK;
}

int fpm_upload_stack(fpm_ctx *c, const uint16_t *meas) {
    if (!c || !meas) return set_err(FPM_ERR_INVAL, "null argument");
    HIP_TRY(hipSetDevice(c->device));
    const size_t n = (size_t)c->prob.n_stack * c->st.B * c->st.np * c->st.np;
    HIP_TRY(hipMemcpyAsync(c->meas, meas, n * sizeof(uint16_t), hipMemcpyHostToDevice, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    return after_upload(c);
}

int fpm_upload_stack_device(fpm_ctx *c, const uint16_t *meas) {
    if (!c || !meas) return set_err(FPM_ERR_INVAL, "null argument");
    HIP_TRY(hipSetDevice(c->device));
    const size_t n = (size_t)c->prob.n_stack * c->st.B * c->st.np * c->st.np;
    if (c->meas_g && meas != c->meas) {
        // the fused layouts of Np 256 / 200: copy and permute in one pass
        hipError_t e = hipSuccess;
        if (meas_layout_copy(meas, c->meas, c->st.np, c->meas_g, (size_t)c->prob.n_stack * c->st.B, c->stream, &e)) {
            HIP_TRY(e);
            c->st.meas_g = c->meas_g;
            c->uploaded = true;
            c->initialized = false;
            return FPM_OK;
        }
    }
    HIP_TRY(hipMemcpyAsync(c->meas, meas, n * sizeof(uint16_t), hipMemcpyDeviceToDevice, c->stream));
    return after_upload(c);
}

int fpm_upload_frames(fpm_ctx *c, const fpm_frames *f, const uint16_t *data, int on_device, int16_t *bg_val) {
    if (!c || !f || !data || !f->patch_x0 || !f->patch_y0) return set_err(FPM_ERR_INVAL, "null argument");
    const int np = c->st.np, B = c->st.B, H = f->height, W = f->width, n = c->prob.n_stack;
    if (H < np || W < np) return set_err(FPM_ERR_INVAL, "frame %dx%d smaller than Np=%d", H, W, np);
    auto inside = [&](int x, int y) { return x >= 0 && y >= 0 && x + np <= W && y + np <= H; };
    for (int b = 0; b < B; ++b)
        if (!inside(f->patch_x0[b], f->patch_y0[b]))
            return set_err(FPM_ERR_INVAL, "patch %d window (%d,%d) outside the %dx%d frame", b, f->patch_x0[b],
                           f->patch_y0[b], W, H);
    if (!inside(f->bk1_x, f->bk1_y) || !inside(f->bk2_x, f->bk2_y))
        return set_err(FPM_ERR_INVAL, "background window outside the frame (cv::Rect assertion in the reference)");
    if (!(f->darkfield_exp_multiplier > 0.0)) return set_err(FPM_ERR_INVAL, "darkfieldExpMultiplier must be > 0");
    HIP_TRY(hipSetDevice(c->device));
    Scratch sc;
    int *px0 = nullptr, *py0 = nullptr;
    unsigned long long *sums = nullptr;
    int16_t *bg_dev = nullptr;
    uint16_t *stage = nullptr;
    HIP_TRY(sc.get(&px0, B));
    HIP_TRY(sc.get(&py0, B));
    HIP_TRY(sc.get(&sums, 2 * (size_t)n));
    HIP_TRY(sc.get(&bg_dev, n));
    HIP_TRY(hipMemcpyAsync(px0, f->patch_x0, B * sizeof(int), hipMemcpyHostToDevice, c->stream));
    HIP_TRY(hipMemcpyAsync(py0, f->patch_y0, B * sizeof(int), hipMemcpyHostToDevice, c->stream));
    const size_t fpx = (size_t)H * W;
    if (!on_device) HIP_TRY(sc.get(&stage, fpx));
    for (int i = 0; i < n; ++i) {
        const uint16_t *frame = data + (size_t)i * fpx;
        if (!on_device) {  // host frames go through one staging buffer (PCIe)
            HIP_TRY(hipMemcpyAsync(stage, frame, fpx * sizeof(uint16_t), hipMemcpyHostToDevice, c->stream));
            frame = stage;
        }
        HIP_TRY(launch_preprocess_frame(frame, W, np, B, px0, py0, f->bk1_x, f->bk1_y, f->bk2_x, f->bk2_y,
                                        f->bg_threshold, f->darkfield_exp_multiplier,
                                        f->darkfield ? f->darkfield[i] != 0 : false, sums + 2 * i,
                                        c->meas + (size_t)i * B * np * np, bg_dev + i, c->stream));
    }
    if (bg_val) HIP_TRY(hipMemcpyAsync(bg_val, bg_dev, n * sizeof(int16_t), hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));  // scratch is freed on return
    return after_upload(c);
}

int fpm_download_stack(fpm_ctx *c, uint16_t *meas) {
    if (!c || !meas) return set_err(FPM_ERR_INVAL, "null argument");
    if (!c->uploaded) return set_err(FPM_ERR_STATE, "no stack uploaded");
    HIP_TRY(hipSetDevice(c->device));
    const size_t n = (size_t)c->prob.n_stack * c->st.B * c->st.np * c->st.np;
    const size_t nimg = (size_t)c->prob.n_stack * c->st.B;
    // back to the C-ABI layout for the copy, then forward again
    if (c->meas_g) HIP_TRY(meas_layout(c->meas, c->st.np, c->meas_g, nimg, false, c->stream));
    HIP_TRY(hipMemcpyAsync(meas, c->meas, n * sizeof(uint16_t), hipMemcpyDeviceToHost, c->stream));
    if (c->meas_g) HIP_TRY(meas_layout(c->meas, c->st.np, c->meas_g, nimg, true, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    return FPM_OK;
}

int fpm_init(fpm_ctx *c) {
    if (!c) return set_err(FPM_ERR_INVAL, "null ctx");
    if (!c->uploaded) return set_err(FPM_ERR_STATE, "fpm_init before fpm_upload_stack");
    HIP_TRY(hipSetDevice(c->device));
    const int init_led = c->order[c->prob.init_pos];
    HIP_TRY(launch_init(c->st, init_led, c->objcrop, c->pl_np, c->tw_np, c->stream));
    c->initialized = true;
    c->objcrop_valid = false;
    return FPM_OK;
}

namespace {

#define HIP_RET(x)                                   \
    do {                                             \
        const hipError_t e_ = (x);                   \
        if (e_ != hipSuccess) return e_;             \
    } while (0)

// patch group g = patches [g B / G, (g + 1) B / G)
DevState group_view(const fpm_ctx *c, int g) {
    const int G = c->ngroups, B = c->st.B;
    return G == 1 ? c->st : patch_view(c->st, g * B / G, (g + 1) * B / G - g * B / G);
}

// one group's LED chain of an iteration on stream s
hipError_t launch_group_chain(const fpm_ctx *c, const DevState &v, hipStream_t s) {
    for (int i = 0; i < c->prob.n_order; ++i) {
        const int led = c->order[i];
        HIP_RET(launch_general_step(v, led, c->x0[led], c->y0[led], c->pl_np, c->tw_np, i == 0, s));
    }
    // Np 1024 / 256 register kernels: the last LED's pupil commit (the others
    // are folded into the next LED's row IDFT)
    if (commit_folded(v)) HIP_RET(launch_pupil_commit(v, s));
    return hipSuccess;
}

// stream of group g when the run stream is s (group 0 runs on s itself)
hipStream_t group_stream(const fpm_ctx *c, int g, hipStream_t s) { return g == 0 ? s : c->gstream[g]; }

// fork the group streams from s / join them back to s
hipError_t fork_groups(fpm_ctx *c, hipStream_t s) {
    if (c->ngroups < 2) return hipSuccess;
    HIP_RET(hipEventRecord(c->gfork, s));
    for (int g = 1; g < c->ngroups; ++g) HIP_RET(hipStreamWaitEvent(c->gstream[g], c->gfork, 0));
    return hipSuccess;
}
hipError_t join_groups(fpm_ctx *c, hipStream_t s) {
    for (int g = 1; g < c->ngroups; ++g) {
        HIP_RET(hipEventRecord(c->gjoin[g], c->gstream[g]));
        HIP_RET(hipStreamWaitEvent(s, c->gjoin[g], 0));
    }
    return hipSuccess;
}

// direct launches (FPM_NO_GRAPH=1): issued LED by LED across the groups so
// that no group's queue runs ahead
hipError_t launch_general_iteration(fpm_ctx *c, hipStream_t s) {
    const int G = c->ngroups;
    DevState view[fpm_ctx::kMaxGroups];
    for (int g = 0; g < G; ++g) view[g] = group_view(c, g);
    HIP_RET(fork_groups(c, s));
    for (int i = 0; i < c->prob.n_order; ++i) {
        const int led = c->order[i];
        for (int g = 0; g < G; ++g)
            HIP_RET(launch_general_step(view[g], led, c->x0[led], c->y0[led], c->pl_np, c->tw_np, i == 0,
                                        group_stream(c, g, s)));
    }
    if (commit_folded(c->st))
        for (int g = 0; g < G; ++g) HIP_RET(launch_pupil_commit(view[g], group_stream(c, g, s)));
    return join_groups(c, s);
}

// The general path issues four launches per LED (~1200 per iteration at 293
// LEDs); every argument is fixed once the context exists, so each group's
// chain of one iteration is captured once (on its own stream) and replayed:
// one graph launch per group per iteration, the groups' graphs on forked streams.
int general_graph(fpm_ctx *c) {
    if (c->led_graph_exec[0]) return FPM_OK;
    for (int g = 0; g < c->ngroups; ++g) {
        hipStream_t cs = group_stream(c, g, c->own_stream);
        HIP_TRY(hipStreamBeginCapture(cs, hipStreamCaptureModeThreadLocal));
        hipError_t e = launch_group_chain(c, group_view(c, g), cs);
        hipGraph_t gr = nullptr;
        hipError_t e2 = hipStreamEndCapture(cs, &gr);
        if (e == hipSuccess) e = e2;
        if (e == hipSuccess) e = hipGraphInstantiate(&c->led_graph_exec[g], gr, nullptr, nullptr, 0);
        if (e != hipSuccess) {
            if (gr) (void)hipGraphDestroy(gr);
            c->led_graph_exec[g] = nullptr;
            for (int h = 0; h < g; ++h) {
                (void)hipGraphExecDestroy(c->led_graph_exec[h]);
                (void)hipGraphDestroy(c->led_graph[h]);
                c->led_graph_exec[h] = nullptr;
                c->led_graph[h] = nullptr;
            }
            return set_err(FPM_ERR_DEVICE, "general-path graph capture: %s", hipGetErrorString(e));
        }
        c->led_graph[g] = gr;
    }
    return FPM_OK;
}

hipError_t launch_general_graphs(fpm_ctx *c, hipStream_t s) {
    HIP_RET(fork_groups(c, s));
    for (int g = 0; g < c->ngroups; ++g) HIP_RET(hipGraphLaunch(c->led_graph_exec[g], group_stream(c, g, s)));
    return join_groups(c, s);
}

}  // namespace

int fpm_run(fpm_ctx *c, int iters) {
    if (!c) return set_err(FPM_ERR_INVAL, "null ctx");
    if (!c->initialized) return set_err(FPM_ERR_STATE, "fpm_run before fpm_init");
    if (iters < 0) return set_err(FPM_ERR_INVAL, "iters=%d", iters);
    HIP_TRY(hipSetDevice(c->device));
    {   // blocking (event waits, the abort-word read-back): never inside a capture
        hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
        HIP_TRY(hipStreamIsCapturing(c->stream, &cap));
        if (cap != hipStreamCaptureStatusNone)
            return set_err(FPM_ERR_INVAL, "fpm_run on a capturing stream: fpm_run is blocking and its %s cannot be "
                           "replayed from a graph (fpm_hip.h)",
                           c->split_ks > 1 ? "co-resident grids" : "launches");
    }
    if (c->clk) HIP_TRY(hipMemsetAsync(c->clk, 0, 3 * sizeof(unsigned long long), c->stream));
    const bool last_only = (c->prob.flags & FPM_FLAG_OBJCROP_LAST_ONLY) != 0;
    // one event pair per iteration around the LED-update launches, one pair
    // around the objCrop IDFT; read back once at the end (fpm_run is blocking)
    const size_t need = 3 * (size_t)iters + 2;
    while (c->evpool.size() < need) {
        hipEvent_t e;
        HIP_TRY(hipEventCreate(&e));
        c->evpool.push_back(e);
    }
    const bool use_graph = c->path != FPM_PATH_FUSED && iters > 0 && !getenv("FPM_NO_GRAPH");
    if (use_graph) {
        const int r = general_graph(c);
        if (r != FPM_OK) return r;
    }
    hipEvent_t *ev = c->evpool.data();
    HIP_TRY(hipEventRecord(ev[0], c->stream));
    for (int it = 0; it < iters; ++it) {
        HIP_TRY(hipEventRecord(ev[1 + 3 * it], c->stream));
        if (c->path == FPM_PATH_FUSED && c->fused_s90) {
            HIP_TRY(launch_fused_s90_iteration(c->st, c->meas, c->order_dev, c->x0_dev, c->y0_dev,
                                               c->prob.n_order, c->tw_np, c->dbg, c->stream));
        } else if (c->path == FPM_PATH_FUSED && c->fused_small) {
            HIP_TRY(launch_fused_small_iteration(c->st, c->meas, c->order_dev, c->x0_dev, c->y0_dev,
                                                 c->prob.n_order, c->tw_np, c->pl_np, c->dbg, c->stream));
        } else if (c->path == FPM_PATH_FUSED && c->fused_mr) {
            HIP_TRY(launch_fused_mr_iteration(c->st, c->meas, c->order_dev, c->x0_dev, c->y0_dev,
                                              c->prob.n_order, c->tw_np, c->dbg, c->stream));
        } else if (c->path == FPM_PATH_FUSED && c->dist) {
            HIP_TRY(launch_fused_dist(c->st, c->meas, c->order_dev, c->x0_dev, c->y0_dev, c->prob.n_order, c->tw_np,
                                      c->split_ks, c->dbg, c->xch, c->split_flags, c->stall_led, c->dist_tags,
                                      c->stream));
            c->dist_tags = (c->dist_tags + (unsigned)c->prob.n_order) & 0x7fffffffu;
        } else if (c->path == FPM_PATH_FUSED) {
            HIP_TRY(launch_fused_iteration(c->st, c->meas, c->order_dev, c->x0_dev, c->y0_dev,
                                           c->prob.n_order, c->tw_np, c->split_ks, c->dbg, c->xch,
                                           c->split_flags, c->stall_led, c->stream));
        } else if (use_graph) {
            HIP_TRY(launch_general_graphs(c, c->stream));
        } else {
            HIP_TRY(launch_general_iteration(c, c->stream));
        }
        HIP_TRY(hipEventRecord(ev[2 + 3 * it], c->stream));
        if (!last_only || it == iters - 1) {
            HIP_TRY(launch_objcrop(c->st, c->objcrop, c->pl_L, c->tw_L, c->stream));
            c->objcrop_valid = true;
        }
        HIP_TRY(hipEventRecord(ev[3 + 3 * it], c->stream));
    }
    HIP_TRY(hipEventRecord(ev[need - 1], c->stream));
    HIP_TRY(hipEventSynchronize(ev[need - 1]));
    if (c->split_flags) {
        // a split-mode handoff that timed out in ANY iteration leaves the
        // results undefined: the abort word is sticky across launches; report
        // it, clear it, and require a fresh fpm_init before the next run
        int ab = 0;
        int *abw = c->split_flags + (size_t)c->split_ks * c->st.B;
        HIP_TRY(hipMemcpy(&ab, abw, sizeof(int), hipMemcpyDeviceToHost));
        if (ab) {
            HIP_TRY(hipMemset(abw, 0, sizeof(int)));
            c->initialized = false;
            c->objcrop_valid = false;
            return set_err(FPM_ERR_DEVICE,
                           "split-mode handoff between the %d workgroups of a patch timed out; results are "
                           "undefined, call fpm_init again", c->split_ks);
        }
    }
    double led_ms = 0, crop_ms = 0;
    for (int it = 0; it < iters; ++it) {
        float a = 0, b = 0;
        HIP_TRY(hipEventElapsedTime(&a, ev[1 + 3 * it], ev[2 + 3 * it]));
        HIP_TRY(hipEventElapsedTime(&b, ev[2 + 3 * it], ev[3 + 3 * it]));
        led_ms += a;
        crop_ms += b;
    }
    float tot = 0;
    HIP_TRY(hipEventElapsedTime(&tot, ev[0], ev[need - 1]));
    c->timing.run_ms = tot;
    c->timing.led_ms = led_ms;
    c->timing.objcrop_ms = crop_ms;
    c->timing.led_launches = (c->path == FPM_PATH_FUSED) ? iters : iters * c->prob.n_order;
    if (c->dbg) {
        unsigned long long h[2 * kStamps];
        HIP_TRY(hipMemcpy(h, c->dbg, sizeof h, hipMemcpyDeviceToHost));
        HIP_TRY(hipMemset(c->dbg, 0, sizeof h));
        const double steps = (double)iters * c->prob.n_order * c->st.B;
        const char *names_f[kStamps] = {"gather", "A:tail+sync", "B:columns", "C:tail+sync", "upd:sync+Opre", "max",
                                        "P",      "A:rowIDFT",   "C:rowDFT",  "upd:body",    "B:loop",
                                        "split:Fstores", "split:Fwait"};
        const char *names_d[kStamps] = {"gather", "A", "sync1", "B", "sync2", "C", "update", "sync3",
                                        "merge+Opre", "max", "P", "C:rows(sub)", "sync3:acks(sub)"};
        const char *const *names = c->dist ? names_d : names_f;
        for (int v = 0; v < 2; ++v) {
            fprintf(stderr, "[fpm stamps] cycles per LED step (%s wave view, mean over blocks):", v ? "last" : "first");
            for (int i = 0; i < kStamps; ++i) fprintf(stderr, " %s=%.0f", names[i], h[v * kStamps + i] / steps);
            fprintf(stderr, "\n");
        }
    }
    c->timing.led_launch_ms = c->timing.led_launches ? led_ms / c->timing.led_launches : 0.0;
    c->clock = fpm_clock{};
    if (c->clk) {
        unsigned long long h[3] = {0, 0, 0};
        HIP_TRY(hipMemcpy(h, c->clk, sizeof h, hipMemcpyDeviceToHost));
        int khz = 0;  // s_memrealtime rate
        if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, c->device) != hipSuccess || khz <= 0)
            khz = 100000;
        if (h[2] > 0 && h[1] > 0) {
            const double sec = (double)h[1] / (khz * 1e3);
            c->clock.clock_mhz = (double)h[0] / sec / 1e6;
            c->clock.cycles_per_launch = (double)h[0] / (double)h[2];
            c->clock.ms_per_launch = sec * 1e3 / (double)h[2];
            c->clock.launches = (int32_t)h[2];
        }
    }
    return FPM_OK;
}

int fpm_get_clock(const fpm_ctx *c, fpm_clock *clock) {
    if (!c || !clock) return set_err(FPM_ERR_INVAL, "null argument");
    *clock = c->clock;
    return FPM_OK;
}

int fpm_synchronize(fpm_ctx *c) {
    if (!c) return set_err(FPM_ERR_INVAL, "null ctx");
    HIP_TRY(hipSetDevice(c->device));
    HIP_TRY(hipStreamSynchronize(c->stream));
    return FPM_OK;
}

int fpm_download(fpm_ctx *c, float *objF, float *objCrop, float *pupil, float *support) {
    if (!c) return set_err(FPM_ERR_INVAL, "null ctx");
    if (!c->initialized) return set_err(FPM_ERR_STATE, "fpm_download before fpm_init");
    HIP_TRY(hipSetDevice(c->device));
    HIP_TRY(hipStreamSynchronize(c->stream));
    const DevState &st = c->st;
    const int L = st.L, np = st.np, r = st.r, nb = st.nb, B = st.B;
    const size_t ll = (size_t)L * L;
    if (objF) {
        // spec is centred; objF = fftShift(spec) (fpmMain.cpp:447)
        std::vector<float2> h(ll);
        std::vector<__half2> h16(st.spec16 ? ll : 0);
        for (int b = 0; b < B; ++b) {
            if (st.spec16) {
                HIP_TRY(hipMemcpy(h16.data(), st.spec16 + b * ll, ll * sizeof(__half2), hipMemcpyDeviceToHost));
                for (size_t i = 0; i < ll; ++i) {
                    const float2 f = __half22float2(h16[i]);
                    h[i] = make_float2(f.x * st.hinv, f.y * st.hinv);
                }
            } else {
                HIP_TRY(hipMemcpy(h.data(), st.spec + b * ll, ll * sizeof(float2), hipMemcpyDeviceToHost));
            }
            float2 *o = (float2 *)objF + b * ll;
            for (int y = 0; y < L; ++y)
                for (int x = 0; x < L; ++x) o[(size_t)y * L + x] = h[(size_t)((y + L / 2) % L) * L + (x + L / 2) % L];
        }
    }
    if (objCrop) {
        if (!c->objcrop_valid) HIP_TRY(launch_objcrop(c->st, c->objcrop, c->pl_L, c->tw_L, c->stream));
        c->objcrop_valid = true;
        HIP_TRY(hipStreamSynchronize(c->stream));
        HIP_TRY(hipMemcpy(objCrop, c->objcrop, B * ll * sizeof(float2), hipMemcpyDeviceToHost));
    }
    if (pupil || support) {
        std::vector<float2> h((size_t)B * nb * nb);
        HIP_TRY(hipMemcpy(h.data(), st.pupil, h.size() * sizeof(float2), hipMemcpyDeviceToHost));
        for (int b = 0; b < B; ++b) {
            if (pupil) {
                // centred pupil (fftShift at fpmMain.cpp:496): P[Np/2+ky][Np/2+kx]
                float2 *o = (float2 *)pupil + (size_t)b * np * np;
                std::memset(o, 0, sizeof(float2) * np * np);
                for (int i = 0; i < nb; ++i)
                    for (int j = 0; j < nb; ++j) o[(size_t)(np / 2 + i - r) * np + np / 2 + j - r] = h[((size_t)b * nb + i) * nb + j];
            }
            if (support) {
                float *o = support + (size_t)b * np * np;
                std::memset(o, 0, sizeof(float) * np * np);
                for (int i = 0; i < nb; ++i)
                    for (int j = 0; j < nb; ++j) {
                        const int ky = i - r, kx = j - r;
                        if (ky * ky + kx * kx <= r * r) o[(size_t)((ky + np) % np) * np + (kx + np) % np] = 1.f;
                    }
            }
        }
    }
    return FPM_OK;
}

int fpm_download_objcrop_device(fpm_ctx *c, float *dst) {
    if (!c || !dst) return set_err(FPM_ERR_INVAL, "null argument");
    if (!c->initialized) return set_err(FPM_ERR_STATE, "download before fpm_init");
    HIP_TRY(hipSetDevice(c->device));
    if (!c->objcrop_valid) HIP_TRY(launch_objcrop(c->st, c->objcrop, c->pl_L, c->tw_L, c->stream));
    c->objcrop_valid = true;
    const size_t n = (size_t)c->st.B * c->st.L * c->st.L * sizeof(float2);
    HIP_TRY(hipMemcpyAsync(dst, c->objcrop, n, hipMemcpyDeviceToDevice, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    return FPM_OK;
}

int fpm_abi_version(void) { return FPM_ABI_VERSION; }

// The whole fpm_info of this header (every field of every ABI revision).
static void fill_info(const fpm_ctx *c, fpm_info *info) {
    std::memset(info, 0, sizeof *info);
    info->path = c->path;
    info->box = c->st.nb;
    info->support_px = c->support_px;
    info->device = c->device;
    info->device_bytes = c->bytes;
    info->wg_per_patch = c->split_ks;
    info->fused_kernel = c->path != FPM_PATH_FUSED ? FPM_KERNEL_GENERAL
                         : c->fused_s90        ? FPM_KERNEL_FUSED_NP90
                         : c->fused_small      ? FPM_KERNEL_FUSED_SMALL
                         : c->fused_mr         ? FPM_KERNEL_FUSED_NP200
                         : c->dist             ? FPM_KERNEL_FUSED_NP256_DIST
                                               : FPM_KERNEL_FUSED_NP256;
    info->threads_per_wg = c->path != FPM_PATH_FUSED ? 0
                           : c->fused_s90 || c->fused_small ? 1024
                           : c->fused_mr ? 768
                                         : c->fused_nt;
}

int fpm_get_info_sized(const fpm_ctx *c, fpm_info *info, size_t info_size) {
    if (!c || !info) return set_err(FPM_ERR_INVAL, "null argument");
    if (info_size < FPM_INFO_V3_SIZE)
        return set_err(FPM_ERR_INVAL, "fpm_info of %zu bytes predates every released layout", info_size);
    fpm_info full;
    fill_info(c, &full);
    std::memcpy(info, &full, std::min(info_size, sizeof full));
    return FPM_OK;
}

// Frozen at the ABI-3 layout (FPM_INFO_V3_SIZE bytes, the fields up to
// fused_kernel): a binary built against that header passes a struct of that
// size, so this entry point never writes past it.  Later fields are reported
// through fpm_get_info_sized only.
int fpm_get_info(const fpm_ctx *c, fpm_info *info) {
    if (!c || !info) return set_err(FPM_ERR_INVAL, "null argument");
    fpm_info full;
    fill_info(c, &full);
    std::memcpy(info, &full, FPM_INFO_V3_SIZE);
    return FPM_OK;
}

int fpm_get_timing(const fpm_ctx *c, fpm_timing *t) {
    if (!c || !t) return set_err(FPM_ERR_INVAL, "null argument");
    *t = c->timing;
    return FPM_OK;
}

int fpm_debug_set_stall(fpm_ctx *c, int led) {
    if (!c) return set_err(FPM_ERR_INVAL, "null ctx");
    c->stall_led = led;
    return FPM_OK;
}

int fpm_runFPM(const fpm_problem *prob, int device, const uint16_t *meas, int iters, float *objF, float *objCrop,
               float *pupil, float *support) {
    fpm_ctx *c = nullptr;
    int rc = fpm_create(prob, device, &c);
    if (rc) return rc;
    if (!(rc = fpm_upload_stack(c, meas)) && !(rc = fpm_init(c)) && !(rc = fpm_run(c, iters)))
        rc = fpm_download(c, objF, objCrop, pupil, support);
    std::string keep = g_err;
    fpm_destroy(c);
    g_err = keep;
    return rc;
}

}  // extern "C"
