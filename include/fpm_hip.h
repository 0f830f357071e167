/*
 * fpm_hip.h -- C ABI of the MI355X-native FPM solver (libfpm_hip.so).
 *
 * Drop-in boundary for the reference's hot path
 *     void runFPM(FPM_Dataset *dataset);      fpmMain.h:119, fpmMain.cpp:274-498
 * which is called once from main after loadFPMDataset (fpmMain.cpp:590-591).
 * FPM_Dataset is a C++ class full of cv::UMat, so the ABI flattens exactly the
 * fields runFPM reads into plain integers, doubles and
 * pointers; the outputs runFPM writes (objF, objCrop, pupil, pupilSupport) are
 * copied out by fpm_download.  No torch or OpenCV types cross this boundary.
 *
 * Conventions
 *   - complex arrays are interleaved float32 pairs (re, im), row-major;
 *   - "stack index" = position of an LED image in the uploaded stack
 *     (the reference indexes imageStack by LED number; the host front-end maps
 *     LED numbers to stack indices, fpm_host.h);
 *   - every call returns FPM_OK (0) or a negative errno-style code, and
 *     fpm_last_error() describes the most recent failure on this thread;
 *   - the caller owns host buffers, the library owns device buffers;
 *   - one context per GPU; a context is not shared between threads.
 */
#ifndef FPM_HIP_H
#define FPM_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ABI revision of this header.  Round 4 (4): fpm_info gained threads_per_wg,
 * readable only through fpm_get_info_sized.  Round 6 (5): fpm_get_info writes
 * only the ABI-3 struct size (path .. fused_kernel) -- under ABI 4 it wrote
 * the whole struct, so a caller reading threads_per_wg from it must move to
 * fpm_get_info_sized; fpm_get_clock added; fpm_run refuses a capturing
 * stream.  fpm_abi_version() reports the library's revision. */
#define FPM_ABI_VERSION   5

#define FPM_OK            0
#define FPM_ERR_INVAL   (-22)   /* bad argument / unsupported geometry      */
#define FPM_ERR_NOMEM   (-12)   /* device or host allocation failed          */
#define FPM_ERR_DEVICE   (-5)   /* HIP runtime / kernel launch failure       */
#define FPM_ERR_STATE   (-71)   /* call out of order (e.g. run before init)  */
#define FPM_ERR_NODEV   (-19)   /* no usable gfx950 device                   */

/* Solver path selection (fpm_problem.path). */
#define FPM_PATH_AUTO     0     /* fused per-patch kernel when it applies    */
#define FPM_PATH_GENERAL  1     /* 4 kernels per LED step, any Np / radius   */
#define FPM_PATH_FUSED    2     /* one persistent launch per iteration       */

/*
 * Raw sensor frames for fpm_upload_frames: the loader preprocessing of
 * loadFPMDataset (fpmMain.cpp:124-144) on the device, for n_patch patches
 * cut from each full frame:
 *   Image  = frame[patch_y0 + y][patch_x0 + x]                 (:124-125)
 *   Image  = saturate(rint(Image / darkfield_exp_multiplier))  when darkfield[i]
 *            and the multiplier != 1                            (:128-129)
 *   bg     = (mean(bk1 window) + mean(bk2 window)) / 2 of the UNDIVIDED
 *            frame, clamped to bg_threshold, rounded to int16   (:131-140)
 *   Image  = saturate(Image - bg)                               (:143-144)
 * Background windows are Np x Np and shared by all patches of a frame.
 */
typedef struct fpm_frames {
    int32_t height, width;        /* full frame size                              */
    const int32_t *patch_x0;      /* [n_patch] cropX of each patch (column)       */
    const int32_t *patch_y0;      /* [n_patch] cropY of each patch (row)          */
    int32_t bk1_x, bk1_y;         /* bk1cropX / bk1cropY                          */
    int32_t bk2_x, bk2_y;         /* bk2cropX / bk2cropY                          */
    double  bg_threshold;         /* bgThresh (JSON asInt)                        */
    double  darkfield_exp_multiplier;  /* darkfieldExpMultiplier                  */
    const uint8_t *darkfield;     /* [n_stack] 1 where illumination NA > objective NA */
} fpm_frames;

/* fpm_problem.flags */
#define FPM_FLAG_OBJCROP_LAST_ONLY 1u  /* compute objCrop only after the last
                                          iteration of fpm_run (the reference
                                          recomputes it every iteration,
                                          fpmMain.cpp:481; default keeps that) */
#define FPM_FLAG_SPEC_FP16         2u  /* store the high-resolution spectrum as
                                          fp16 (scaled by a power of two), compute
                                          in fp32: BASELINE config 5 ("fp16
                                          storage / fp32 accumulate"); general
                                          path only.  The reference keeps
                                          CV_64FC2 objF (fpmMain.h:92) */
#define FPM_FLAG_SCALAR_RE_ONLY    4u  /* legacy semantics for the reference's
                                          cv::add / cv::multiply(UMat CV_64FC2,
                                          double) at fpmMain.cpp:390,417-418,
                                          469-470: the scalar touches the real
                                          channel only.  Default (flag clear) is
                                          OpenCV's published behaviour: a double
                                          becomes a 1x1 array that arithm_op's
                                          convertAndUnrollScalar replicates into
                                          EVERY channel, so eps is added to Re and
                                          Im and the update denominators are
                                          complex, ((|P|^2+d2) + i d2) max|P| and
                                          ((|O|^2+d1) + i d1) max|objF| (DESIGN.md
                                          section 2) */

/*
 * Problem description: the FPM_Dataset fields runFPM reads
 * (fpmMain.h:43-101, read at fpmMain.cpp:290-481).
 */
typedef struct fpm_problem {
    int32_t np;            /* Np: ROI size (cropSizeX, fpmMain.cpp:519); even    */
    int32_t nlarge;        /* Nlarge == Mlarge == Np*resImprovementFactor (:564) */
    int32_t n_stack;       /* images in the uploaded stack                       */
    int32_t n_order;       /* ledUsedCount: LEDs processed per iteration (:348)  */
    const int32_t *order;  /* [n_order] stack indices in processing order:
                              sortedIndicies[0..ledUsedCount) (fpmMain.cpp:350)  */
    const int32_t *crop_x0;/* [n_stack] cropXStart in the centred spectrum (:157) */
    const int32_t *crop_y0;/* [n_stack] cropYStart (:163)                        */
    int32_t na_radius;     /* naRadius = ceil(objNA*ps_eff*Np/lambda) (:305)     */
    int32_t init_pos;      /* position in order[] of the init image; the
                              reference uses sortedIndicies.at(1) (:319) -> 1    */
    double  delta1;        /* pupil-update regulariser, JSON asInt (:567)         */
    double  delta2;        /* object-update regulariser, JSON asInt (:568); > 0  */
    double  eps;           /* amplitude-replacement eps, float 1e-10 (fpmMain.h:99) */
    int32_t n_patch;       /* independent patches batched on this device (>= 1) */
    int32_t path;          /* FPM_PATH_*                                          */
    uint32_t flags;        /* FPM_FLAG_*                                          */
} fpm_problem;

typedef struct fpm_ctx fpm_ctx;

/* fpm_info.fused_kernel: the LED-update kernel fpm_run launches */
#define FPM_KERNEL_GENERAL      0  /* general path: 4-5 launches per LED          */
#define FPM_KERNEL_FUSED_NP256  1  /* k_fused_iteration (Np 256, r <= 34)          */
#define FPM_KERNEL_FUSED_NP200  2  /* k_fused_mr (Np 200)                          */
#define FPM_KERNEL_FUSED_SMALL  3  /* k_fused_small (Np <= 96)                     */
#define FPM_KERNEL_FUSED_NP256_DIST 4  /* k_fused_dist (Np 256, every phase distributed
                                          over wg_per_patch workgroups; small batches) */
#define FPM_KERNEL_FUSED_NP90   5  /* k_fused_s90 (Np 90: register 9 x 10 transforms) */

/* Which path the context runs and its per-launch geometry. */
typedef struct fpm_info {
    int32_t path;          /* FPM_PATH_GENERAL or FPM_PATH_FUSED */
    int32_t box;           /* 2*na_radius+1: side of the pupil box             */
    int32_t support_px;    /* pixels in the pupil support disk                  */
    int32_t device;
    size_t  device_bytes;  /* device memory owned by the context               */
    int32_t wg_per_patch;  /* fused Np 256 path: workgroups per patch (1, or 2 /
                              4 / 8 in split or distributed mode when
                              wg_per_patch * n_patch <= CUs)                   */
    int32_t fused_kernel;  /* FPM_KERNEL_*                                      */
    int32_t threads_per_wg;/* threads per workgroup of the LED-update kernel (ABI 4) */
} fpm_info;

/* bytes of the ABI-3 struct, fields path .. fused_kernel: what fpm_get_info writes */
#define FPM_INFO_V3_SIZE  (offsetof(fpm_info, fused_kernel) + sizeof(int32_t))

/* Per-kernel timing of the most recent fpm_run, from HIP events recorded on
 * the stream the kernels were launched on. */
typedef struct fpm_timing {
    double run_ms;         /* whole fpm_run, event to event                    */
    double led_ms;         /* LED-update kernels only (all iterations)         */
    double led_launch_ms;  /* average duration of one LED-update launch        */
    int32_t led_launches;  /* number of LED-update launches measured           */
    double objcrop_ms;     /* per-iteration objCrop IDFT kernels               */
} fpm_timing;

/* Create a context on `device`; validates geometry, allocates device state. */
int  fpm_create(const fpm_problem *prob, int device, fpm_ctx **out);
void fpm_destroy(fpm_ctx *ctx);

/* Upload the measurement stack, uint16 [n_stack][n_patch][Np][Np]
 * (LED-major: every LED step reads one contiguous slab). Host pointer. */
int  fpm_upload_stack(fpm_ctx *ctx, const uint16_t *meas);
/* Same, from device memory on the context's device (no PCIe round trip). */
int  fpm_upload_stack_device(fpm_ctx *ctx, const uint16_t *meas_dev);

/* Upload raw frames [n_stack][height][width] (host memory, or device memory on
 * the context's device when frames_on_device != 0) and build the measurement
 * stack on the GPU (fpm_frames above).  bg_val, when not NULL, receives the
 * per-image background [n_stack] (FPMImage::bg_val, fpmMain.h:33). */
int  fpm_upload_frames(fpm_ctx *ctx, const fpm_frames *frames, const uint16_t *data,
                       int frames_on_device, int16_t *bg_val);

/* Copy the measurement stack [n_stack][n_patch][Np][Np] back to the host. */
int  fpm_download_stack(fpm_ctx *ctx, uint16_t *meas);

/* fpmMain.cpp:302-343: pupil = support disk, spectrum from order[init_pos]. */
int  fpm_init(fpm_ctx *ctx);

/* fpmMain.cpp:345-482: `iters` sequential passes over order[], each followed
 * by the objCrop IDFT (fpmMain.cpp:481) unless FPM_FLAG_OBJCROP_LAST_ONLY.
 * Enqueued on the context stream; returns when the work has completed
 * (per-kernel HIP-event timings are then available from fpm_get_timing).
 * Blocking, so it cannot be recorded into a graph: on a stream that is being
 * captured it returns FPM_ERR_INVAL before enqueuing anything (the capture
 * stays valid).  The split / distributed modes also need every workgroup of
 * a grid resident at once, which a replayed graph could not guarantee
 * beside other co-resident grids. */
int  fpm_run(fpm_ctx *ctx, int iters);

/* Wait for all work on the context stream. */
int  fpm_synchronize(fpm_ctx *ctx);

/* Copy results to host (any pointer may be NULL):
 *   objF    [n_patch][L][L][2]   un-centred spectrum, like dataset->objF
 *   objCrop [n_patch][L][L][2]   IDFT(objF)/L^2 (fpmMain.cpp:481)
 *   pupil   [n_patch][Np][Np][2] centred pupil (fpmMain.cpp:496)
 *   support [n_patch][Np][Np]    un-centred pupilSupport (real part, 0/1)  */
int  fpm_download(fpm_ctx *ctx, float *objF, float *objCrop, float *pupil,
                  float *support);

/* Device-to-device copy of objCrop [n_patch][L][L][2] into caller memory on
 * the context's device (for the multi-GPU gather). */
int  fpm_download_objcrop_device(fpm_ctx *ctx, float *dst_dev);

/* Use a caller-provided hipStream_t (NULL = the context's own stream). */
int  fpm_set_stream(fpm_ctx *ctx, void *hip_stream);

/* fpm_get_info is frozen at the ABI-3 layout: it writes FPM_INFO_V3_SIZE
 * bytes (path .. fused_kernel) and never a later field, so a binary built
 * against the ABI-3 header, whose struct is that size, stays safe.  Fields
 * appended since (threads_per_wg, ABI 4) are read with fpm_get_info_sized,
 * which writes only the first info_size bytes: pass sizeof(fpm_info) of the
 * header the caller was built with (fields are only ever appended). */
int  fpm_get_info(const fpm_ctx *ctx, fpm_info *info);
int  fpm_get_info_sized(const fpm_ctx *ctx, fpm_info *info, size_t info_size);
int  fpm_get_timing(const fpm_ctx *ctx, fpm_timing *timing);

/* Clock of the LED-update launches of the most recent fpm_run (fused path;
 * ABI 5): block 0 of every launch reads the shader-cycle counter (s_memtime)
 * and the constant-rate real-time counter (s_memrealtime) at entry and after
 * its last LED, so clock_mhz = cycles / real time is the shader clock the
 * kernel actually ran at and cycles_per_launch its length in cycles, which a
 * slower clock does not change (MI355X_MICROARCH.md, DVFS).  launches = 0 on
 * the general path, which has no probe. */
typedef struct fpm_clock {
    double clock_mhz;          /* mean shader clock over the probed launches   */
    double cycles_per_launch;  /* block 0's shader cycles per launch           */
    double ms_per_launch;      /* block 0's real time per launch               */
    int32_t launches;          /* launches probed                              */
} fpm_clock;
int  fpm_get_clock(const fpm_ctx *ctx, fpm_clock *clock);

/* One-shot equivalent of runFPM for n_patch patches: create, upload, init,
 * run, download, destroy.  Blocking. */
int  fpm_runFPM(const fpm_problem *prob, int device, const uint16_t *meas,
                int iters, float *objF, float *objCrop, float *pupil,
                float *support);

/* Description of the most recent error on the calling thread. */
const char *fpm_last_error(void);

/* Library build identification (also proves the .so loaded). */
const char *fpm_version(void);
/* FPM_ABI_VERSION the library was built with; a caller compiled against a
 * newer header than the library refuses to run. */
int fpm_abi_version(void);

#ifdef __cplusplus
}
#endif
#endif /* FPM_HIP_H */
