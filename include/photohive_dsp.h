/* photohive_dsp.h -- C-ABI of PhotoHive_DSP_lib/libreport_data.so (MI355X build).
 *
 * Drop-in for the reference's libreport_data.so: the three legacy entry points
 * keep their exact signatures and struct layouts, so the reference's own
 * ctypes binding (/root/reference/lib.py:20-37, structures.py:6-106) loads
 * this library unchanged.  Behind them the hot path (rgb2hsv, RGB statistics,
 * HSV-grid colour palette, 2-D FFT magnitude + polar blur binning) runs as
 * hand-written HIP kernels on a gfx950 GPU; there is no CPU fallback -- without
 * a usable GPU every entry point returns NULL / a negative status and
 * phd_last_error() says why.
 *
 * Everything here is plain C: pointers, ints and doubles, no HIP/torch types.
 */
#ifndef PHOTOHIVE_DSP_H
#define PHOTOHIVE_DSP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- struct layouts: byte-identical to the reference ------------------- */
typedef double Pixel;                                  /* src/types.h:5 */

typedef struct Pixel_HSV {                             /* src/image_processing.h:12-17 */
    int parent_id;
    double h, s, v;
} Pixel_HSV;

typedef struct Image_RGB {                             /* src/image_processing.h:31-36 */
    int height, width;
    Pixel *r, *g, *b;
} Image_RGB;

typedef struct Image_PGM {                             /* src/image_processing.h:63-66 */
    int height, width;
    Pixel* data;
} Image_PGM;

typedef struct RGB_Statistics {                        /* src/image_processing.h:73-80 */
    Pixel Br, Bg, Bb, Cr, Cg, Cb;
} RGB_Statistics;

typedef struct Crop_Boundaries {                       /* src/image_processing.h:92-98 */
    int N;
    int *top, *bottom, *left, *right;
} Crop_Boundaries;

typedef struct Color_Palette {                         /* src/color_quantization.h:11-15 */
    int N;
    Pixel_HSV* averages;
    double* percentages;
} Color_Palette;

typedef double Bin;                                    /* src/blur_profile.h:8 */

typedef struct Blur_Profile {                          /* src/blur_profile.h:20-24 */
    int num_angle_bins, num_radius_bins;
    int angle_bin_size, radius_bin_size;
    Bin** bins;                                        /* [angle][radius] */
} Blur_Profile;

typedef struct Blur_Vector {                           /* src/blur_profile.h:52-55 */
    int angle;
    float magnitude;
} Blur_Vector;

typedef struct Blur_Vector_Group {                     /* src/blur_profile.h:58-61 */
    int len_vectors;
    Blur_Vector* blur_vectors;
} Blur_Vector_Group;

typedef struct Sharpnesses {                           /* src/utilities.h:25-28 */
    int N;
    Pixel* sharpness;
} Sharpnesses;

typedef struct Full_Report_Data {                      /* src/utilities.h:30-37 */
    RGB_Statistics* rgb_stats;
    Color_Palette* color_palette;
    Blur_Profile* blur_profile;
    Blur_Vector_Group* blur_vectors;
    Pixel average_saturation;
    Sharpnesses* sharpness;
} Full_Report_Data;

/* ---- legacy entry points (reference signatures) ------------------------- */

/* Replaces get_full_report_data, src/interface.h:16-23 / src/interface.c:20-94.
 * Input: planar doubles (as utils.py:30-46 produces).  Inputs that are all
 * exactly k/255.0 take the RGB8 pipeline; any other finite doubles run the fp64
 * planar kernels (planar.hip: the reference's own double arithmetic); non-finite
 * values are rejected with a message.  Returns NULL on the reference's error
 * cases (src/utilities.c:64-87) and on GPU errors. */
Full_Report_Data* get_full_report_data(Image_RGB* image, Crop_Boundaries* salient_characters,
                                       int h_partitions, int s_partitions, int v_partitions,
                                       double black_thresh, double gray_thresh,
                                       double coverage_thresh, int linked_list_size,
                                       int downsample_rate, int radius_partitions,
                                       int angle_partitions, float quantity_weight,
                                       float saturation_value_weight, double fft_streak_thresh,
                                       double magnitude_thresh, int blur_cutoff_ratio_denom);

/* Replaces free_full_report, src/interface.c:97-111: releases the whole tree
 * and sets *report = NULL.
 *  - A report of get_full_report_data has the reference's allocation shape:
 *    every structure and array is its own malloc (the blur profile's row
 *    pointers and each row included), so a C caller may free() a member itself
 *    (then set it to NULL); this call frees the rest member by member.
 *  - A report of the batch / u8 entry points (phd_report_*) is one heap block
 *    holding the whole tree, recycled for later reports of the same size:
 *    release it only through this call (or phd_free_reports), never by free()
 *    on a member.
 * A pointer that is neither (foreign, or already freed) is ignored; freeing a
 * stale pointer after its memory was reused by a later report is undefined,
 * as with free(). */
void free_full_report(Full_Report_Data** report);
/* free_full_report over an array of n reports (a batch call's `out`); NULL entries are skipped. */
void phd_free_reports(Full_Report_Data** reports, int n);

/* Replaces get_blur_profile_visual, src/blur_profile.c:140-180 (bound by
 * /root/reference/lib.py:36-37).  Caller owns the result (free with
 * phd_free_pgm; the reference's Python caller leaks it). */
Image_PGM* get_blur_profile_visual(Blur_Profile* blur_profile, int height, int width);

/* ---- new entry points ---------------------------------------------------- */

/* The 16 scalar hyper-parameters of get_report (core.py:442-448), reentrant. */
typedef struct phd_config {
    int h_partitions, s_partitions, v_partitions;
    double black_thresh, gray_thresh, coverage_thresh;
    int linked_list_size, downsample_rate;
    int radius_partitions, angle_partitions;
    float quantity_weight, saturation_value_weight;
    double fft_streak_thresh, magnitude_thresh;
    int blur_cutoff_ratio_denom;
} phd_config;

/* Fill *cfg with the get_report defaults (18,2,3,0.1,0.1,0.95,1000,1,40,72,
 * 0.1f,0.9f,1.20,0.3,2). */
void phd_config_default(phd_config* cfg);

/* One image from an interleaved RGB8 HOST buffer (row_stride bytes per row;
 * 0 = 3*width).  No planar-double conversion.  NULL on error. */
Full_Report_Data* phd_report_u8(const uint8_t* rgb, int height, int width, size_t row_stride,
                                const phd_config* cfg, const Crop_Boundaries* crops);

/* A batch of same-size images already resident in GPU memory (d_rgb points at
 * n_images * image_stride bytes on the current HIP device; rows are 3*width
 * bytes).  stream: a hipStream_t or NULL for the library's own stream.
 * out[i] receives each report (NULL on per-image error, status[i] < 0).
 * Returns 0 when every image succeeded, else the number of failures, or -1
 * on a setup error. */
int phd_report_batch_device(const uint8_t* d_rgb, int n_images, int height, int width,
                            size_t image_stride, const phd_config* cfg, Full_Report_Data** out,
                            int* status, void* stream);

/* rgb2hsv + get_hsv_average + get_rgb_statistics over n device-resident RGB8
 * images (BASELINE.json config 3).  Replaces the reference's
 * rgb2hsv (src/image_processing.c:372-417), get_hsv_average (:533-540) and
 * get_rgb_statistics (:543-553) as called from get_full_report_data
 * (src/interface.c:46-55) with downsample_rate 1; the HSV image itself is never
 * materialised.  stats[i] / avg_saturation[i] per image.  0 or -1. */
int phd_hsv_stats_batch_device(const uint8_t* d_rgb, int n_images, int height, int width,
                               size_t image_stride, RGB_Statistics* stats, double* avg_saturation,
                               void* stream);

/* The FFT + blur-profile path alone over n device-resident RGB8 images of one
 * size (BASELINE.json config 4): rgb2pgm, remove_dc_bias, pgm_fft,
 * pgm_normalize_fft, cartesian_to_polar_conversion, calculate_blur_profile
 * and vectorize_blur_profile (src/image_processing.c:505-512,
 * src/blur_profile.c:34-126,233-238,324-458, src/fft_processing.c:18-63,
 * 173-213) as get_full_report_data runs them (src/interface.c:50,62-86).
 * bins_out: n x angle_partitions x radius_partitions doubles (the
 * Blur_Profile bins, angle-major); vectors_out: n x 10 Blur_Vector.  The
 * values equal the full report's.  0 or -1. */
int phd_blur_batch_device(const uint8_t* d_rgb, int n_images, int height, int width, size_t image_stride,
                          const phd_config* cfg, double* bins_out, Blur_Vector* vectors_out, void* stream);

/* Device-resident images of any sizes (config 5 of BASELINE.json): one
 * batched run per group of same-size images (64 images, or as many as hold
 * 64 x 12 MP when that is more: up to 1024 small images in one run).  Returns
 * 0 when every image succeeded, else the number of failures, or -1 on a setup
 * error. */
int phd_report_batch_device_mixed(const uint8_t* const* d_images, const int* heights, const int* widths,
                                  int n_images, const phd_config* cfg, Full_Report_Data** out, int* status,
                                  void* stream);

/* A batch of host images of any sizes (config 5 of BASELINE.json). */
int phd_report_batch_u8(const uint8_t* const* images, const int* heights, const int* widths,
                        int n_images, const phd_config* cfg, Full_Report_Data** out, int* status);

/* Palette intermediates of one device-resident image, for bit-exact checks:
 * hist[TL] (arm_octree quantities), parents[*n_parents] (valid_parents in
 * palette order), kept[*n_parents] (pixels surviving group_irregular_pixels).
 * Arrays must hold total_length (hist) / total_length (parents, kept) ints.
 * Returns total_length, or < 0 on error. */
int phd_palette_trace_device(const uint8_t* d_rgb, int height, int width, const phd_config* cfg,
                             int* hist, int* parents, int* kept, int* n_parents);

/* Per-bin element counts of the polar blur table for a height x width image
 * (image-independent, src/blur_profile.c:87-98), [angle][radius] row-major.
 * Returns 0 or < 0. */
int phd_blur_counts(int height, int width, int radius_partitions, int angle_partitions,
                    long long* counts);

/* Fill n bytes of device memory with the splitmix64 stream of
 * photohive_dsp_amd/synth.py:uniform (byte j = byte j%8 of word j/8). */
int phd_fill_uniform_device(uint8_t* d_dst, size_t n, uint64_t seed, void* stream);

/* Fill height x width x 3 bytes of device memory with
 * photohive_dsp_amd/synth.py:structured(height, width, seed, blur, blur_axis)
 * (gradient + disks + noise, then a `blur`-tap box blur along blur_axis when
 * blur > 1): the bench's SURVEY 8(d) row 2(b) images.  0 or -1. */
int phd_fill_structured_device(uint8_t* d_dst, int height, int width, uint64_t seed, int blur, int blur_axis,
                               void* stream);

/* Validation hook: per-pixel rgb2hsv and octree group id of n_pixels device
 * RGB8 pixels into d_gid[n] (and d_hsv[3n] if non-NULL). */
int phd_debug_hsv_groups_device(const uint8_t* d_rgb, long n_pixels, const phd_config* cfg, int* d_gid,
                                double* d_hsv);

/* Validation hook, host only (no GPU): the production K1's per-pixel
 * classification (k1_pixel.h) of n interleaved host RGB8 pixels -- the hue
 * cell of the fused palette, h, s, and (if deferred != NULL) whether the pixel
 * took the exact double path.  Returns 0 or -1. */
int phd_debug_k1_pixels(const uint8_t* rgb, long n, const phd_config* cfg, int* cell, double* h, double* s,
                        int* deferred);

/* Micro-benchmark hook: average ms per launch of one pipeline kernel (0 hsv_stats,
 * 1 fft_rows, 2 fft_cols) over `iters` launches on a device image; `ablate` is a
 * debug mask (0 = production kernel). */
int phd_debug_time_kernel(int kernel, const uint8_t* d_rgb, int height, int width, const phd_config* cfg,
                          int ablate, int iters, double* avg_ms);

/* Validation hook: the power spectrum |X[u][k]|^2 (src/fft_processing.c:48-50)
 * of one device RGB8 image through the production FFT kernels, column-major
 * into d_out[(width/2+1) * height] (device memory).  0, -2 when the size has
 * no compile-time FFT plan, or -1. */
int phd_debug_power_spectrum(const uint8_t* d_rgb, int height, int width, double* d_out);
/* log_mant, the polar bins' table-driven fp64 log, over n positive device doubles. */
int phd_debug_log_mant(const double* d_x, double* d_y, long n);
/* Host only (no device needed): entries (runs of one polar bin + a sentinel)
 * of the longest spectrum column of this size and bin grid.  Above 256 the
 * compile-time column pass cannot hold the column's list and the size takes
 * the runtime-plan FFT.  Returns the count or -1. */
int phd_debug_col_runs_max(int height, int width, int radius_partitions, int angle_partitions);
/* Test hook: the compile-time column pass's form for later calls of this
 * process: -1 the library's choice (default), 0 the half-prefetch form, 1 the
 * full-prefetch form where the plan has one.
 * Returns the previous setting. */
int phd_debug_column_form(int mode);

/* Validation hook for the global-memory FFTs behind sides above 8192 px and
 * lengths with a large prime factor (the reference's FFTW r2c takes any
 * length, src/fft_processing.c:18-63): `count` contiguous complex sequences
 * of length n (device, interleaved re/im) -> their unnormalised forward DFTs
 * (e^{-i}) in d_out (d_out == d_in allowed).  Returns the plan kind (0 one
 * LDS pass, 1 four-step, 2 Bluestein) or -1. */
int phd_debug_gfft(const double* d_in, double* d_out, int n, long count);

/* Test hook (no GPU): a report tree in get_full_report_data's allocation shape
 * (n_palette colours, na x nr bins, n_crops sharpnesses or none when < 0),
 * filled with a fixed pattern and live for free_full_report. */
Full_Report_Data* phd_debug_legacy_report(int n_palette, int na, int nr, int n_crops);

/* Free an Image_PGM returned by get_blur_profile_visual. */
void phd_free_pgm(Image_PGM* img);

/* Human-readable reason for the last failure on this thread ("" if none). */
const char* phd_last_error(void);

/* Device name / arch / CU count into buf; returns the HIP device ordinal or < 0. */
int phd_device_info(char* buf, int buflen);

/* Stage timing of the most recent report call (ms).  Device, from HIP events:
 * [0] K1 (hsv + stats + palette sums), [1] FFT rows + columns, [2] palette
 * pass 2 left after the FFTs, [3] whole device span.  Host wall clock: [4]
 * whole call, [5] enqueue, [6] palette decisions + pass-2 enqueue, [7]
 * report assembly.  Returns the number of stages written (<= n). */
int phd_last_timings(double* ms, int n);

/* Per-kernel GPU time from HIP events recorded on the launch stream around
 * every launch of the kernels in `mask` (bit k = kernel k: 0 hsv_stats,
 * 1 fft_rows, 2 fft_cols, 3 palette_cutoffs, 4 palette_sums, 5 sharpness).
 * phd_profile_kernels resets the counters; phd_profile_read returns the
 * accumulated milliseconds and launch count of one kernel. */
int phd_profile_kernels(unsigned mask);
int phd_profile_read(int kernel, double* total_ms, long* launches);

/* Lanes a device batch of >= 16 images on the library's stream is split over
 * (1 or 2; default 2, or PHD_LANES).  Each lane is an independent context with
 * its own streams and workspaces; the second runs on a library thread, so the
 * two halves' kernels, host phases and launch gaps overlap (+10-13 % images/s
 * at 4000x3000 over one lane, bench.py's one_lane object).  It applies to
 * phd_report_batch_device, phd_blur_batch_device (the second half of the
 * batch on lane 1) and phd_report_batch_device_mixed (size groups to the
 * lanes in turn).  Results do not
 * depend on it.  With
 * two lanes, phd_last_timings and PHD_VERBOSE's stage lines cover lane 0's half
 * of a batch only (the stage timings are per calling thread).  lanes < 1 only
 * queries.  Returns the previous setting. */
int phd_set_lanes(int lanes);

/* Explicit teardown (no counterpart in the reference, which frees per call,
 * src/interface.c:88-92): joins the library's threads (the second lane's
 * worker, the host pools) and releases every context's device buffers, pinned
 * buffers, events and streams after their queued work.  The library registers
 * it with atexit at its first HIP use, so it also runs before HIP's own
 * finalizers at exit; a caller may run it earlier (the next call then starts
 * afresh).  Do not call it while another thread is inside a library call. */
void phd_shutdown(void);

/* Crash triage: on SIGSEGV / SIGBUS / SIGILL / SIGFPE / SIGABRT write
 * /proc/self/maps to "<prefix>.<pid>.maps" (async-signal-safe), then hand the
 * signal to the handler installed before (or the default action).  0 on
 * success. */
int phd_install_crash_maps(const char* prefix);

/* Test hook: the library threads alive in this process (lane worker + host
 * pool threads); start != 0 creates them first. */
int phd_debug_library_threads(int start);

#ifdef __cplusplus
}
#endif
#endif /* PHOTOHIVE_DSP_H */
