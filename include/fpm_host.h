/*
 * fpm_host.h -- C ABI of the host front-end library (libfpm_host.so).
 *
 * The reference's main()/loadFPMDataset (fpmMain.cpp:36-271, 500-592) turn a
 * dataset JSON plus a directory of TIFF frames into the FPM_Dataset fields
 * runFPM consumes.  This library does the same on the host and hands the
 * result to libfpm_hip.so (fpm_hip.h) as an fpm_problem plus a uint16 stack.
 *
 *   fpm_host_open            Json::Reader::parse + the 30 get() calls (:512-575)
 *   fpm_host_set_led_table   explicit LED coordinates (dome fallback when the
 *                            JSON has no holeCoordinates)
 *   fpm_host_set_present     LED numbers whose images exist (synthetic runs)
 *   fpm_host_scan            readdir of datasetRoot (:63-75)
 *   fpm_host_geometry        sin(theta), NA filter, k-space offsets (:77-168)
 *                            and the std::sort LED order (:246-258)
 *   fpm_host_load_images     imread + crop + darkfield + background (:109-144)
 *   fpm_host_load_frames     imread only: full frames for fpm_upload_frames
 *
 * Stack convention handed to fpm_hip: stack index i holds the LED
 * sortedIndicies[i], so the processing order is 0,1,...,ledUsedCount-1.
 */
#ifndef FPM_HOST_H
#define FPM_HOST_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct fpm_host fpm_host;

/* Scalar FPM_Dataset fields after main() (fpmMain.h:43-101). */
typedef struct fpm_host_config {
    int32_t np;                   /* cropSizeX                        */
    int32_t nlarge;               /* Nlarge = Np * resImprovementFactor */
    int32_t res_improvement_factor;
    int32_t na_radius;            /* fpmMain.cpp:305-306              */
    int32_t led_count;
    int32_t crop_x, crop_y;
    int32_t bk1_crop_x, bk1_crop_y, bk2_crop_x, bk2_crop_y;
    int32_t center_led;
    int32_t darkfield_exp_multiplier;
    int32_t color, flip_x, flip_y, debug;
    int32_t hole_coordinates_present;  /* JSON holeCoordinates is an array */
    int32_t hole_coordinates_count;
    int32_t json_ok;              /* Json::Reader::parse result (reference ignores it) */
    float pixel_size, objective_mag, objective_na, max_illumination_na, lambda;
    float ps_eff, du, ps, bg_threshold, delta1, delta2;
    double array_rotation;
    char dataset_root[1024];
    char file_prefix[128];
    char file_extension[32];
} fpm_host_config;

/* One LED (FPMimg fields, fpmMain.h:19-41). */
typedef struct fpm_host_led {
    int32_t led;                  /* LED number                       */
    int32_t used;                 /* NA < maxIlluminationNA           */
    float pos[3];
    double sin_theta_x, sin_theta_y;
    float illumination_na;
    float uled, vled;
    int32_t idx_u, idx_v;
    int32_t crop_x0, crop_y0, crop_x1, crop_y1;
    int32_t bg_val;               /* after fpm_host_load_images       */
} fpm_host_led;

int  fpm_host_open(const char *json_path, fpm_host **out);
int  fpm_host_open_text(const char *json_text, fpm_host **out);
void fpm_host_close(fpm_host *h);
int  fpm_host_get_config(const fpm_host *h, fpm_host_config *cfg);
/* Override scalar keys after parsing (e.g. cropSizeX / maxIlluminationNA for
 * the metric configuration); re-derives ps_eff, du, L, naRadius like main(). */
int  fpm_host_override(fpm_host *h, const char *key, double value);

int  fpm_host_set_led_table(fpm_host *h, const float *xyz, int n_leds);
int  fpm_host_set_present(fpm_host *h, const int32_t *led_numbers, int n);
int  fpm_host_scan(fpm_host *h);
int  fpm_host_geometry(fpm_host *h);

int  fpm_host_n_present(const fpm_host *h);
int  fpm_host_n_used(const fpm_host *h);
int  fpm_host_get_leds(const fpm_host *h, fpm_host_led *out, int n);
/* sortedIndicies: LED numbers in processing order, ledUsedCount entries. */
int  fpm_host_get_order(const fpm_host *h, int32_t *led_numbers, int n);
/* crop starts in stack order (stack index i == order position i). */
int  fpm_host_get_crops(const fpm_host *h, int32_t *x0, int32_t *y0, int n);

int  fpm_host_load_images(fpm_host *h);
/* uint16 [ledUsedCount][Np][Np] in stack order. */
int  fpm_host_get_stack(const fpm_host *h, uint16_t *out, size_t n_elems);

/* Raw full frames of the used LEDs, uint16 [ledUsedCount][height][width] in
 * stack order, input of fpm_upload_frames: many patches per frame, preprocessing on
 * the GPU.  out == NULL only reports the frame size.  Returns the frame
 * count (0 for a size query). */
int  fpm_host_load_frames(const fpm_host *h, uint16_t *out, size_t n_elems, int32_t *width, int32_t *height);

/* 16-bit grayscale TIFF I/O (the frame format the loader reads). */
int  fpm_host_read_tiff(const char *path, uint16_t *out, size_t cap, int32_t *width, int32_t *height);
int  fpm_host_write_tiff16(const char *path, const uint16_t *px, int32_t width, int32_t height);

const char *fpm_host_last_error(void);

#ifdef __cplusplus
}
#endif
#endif /* FPM_HOST_H */
