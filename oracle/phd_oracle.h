/* phd_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * Plain-C CPU restatement of the PhotoHive_DSP hot path (reference
 * @2024-11-25, /root/reference/src).  Used by tests/, by
 * __graft_entry__.smoke() and by bench.py's cpu_baseline leg as the CHECKER;
 * never linked into or called by the product library.
 *
 * Parity pinning: every function here is checked against the reference's own
 * C (oracle/_ref/libphd_ref.so, built from /root/reference/src at -O0 by
 * oracle/Makefile) through oracle/ref_pipeline.py and the committed golden
 * fixtures in tests/golden/.  The 2-D DFT is not restated (it is FFTW in the
 * reference); callers pass the power spectrum |X|^2 computed by numpy/scipy.
 */
#ifndef PHD_ORACLE_H
#define PHD_ORACLE_H

#include <stdint.h>

typedef struct orc_config {
    int h_parts, s_parts, v_parts;
    double black_thresh, gray_thresh, coverage;
    int linked_list_size, downsample_rate;
    int radius_parts, angle_parts;
    float quantity_weight, sv_weight;
    double streak_thresh, mag_thresh;
    int cutoff_denom;
} orc_config;

/* utilities.c:64-87; returns 1 when the reference would return NULL. */
int orc_precheck(int height, int width);

/* image_processing.c:543-553 + filtering.c:125-148 on interleaved u8 RGB:
   out = {Br, Bg, Bb, Cr, Cg, Cb}. */
void orc_rgb_stats(const uint8_t* rgb, int height, int width, double out[6]);

/* Per-pixel HSV (image_processing.c:372-417) for k/255 inputs. */
void orc_rgb2hsv_px(double r, double g, double b, double* h, double* s, double* v);

typedef struct orc_palette {
    int total_length;         /* TL = h*s*v + v + 1                              */
    int n_hsv;                /* pixels in the (downsampled) HSV image           */
    double average_saturation;/* image_processing.c:533-540                      */
    int n_parents;
    int* hist;                /* [TL] arm_octree quantities                      */
    int* parents;             /* [n_parents] valid_parents, palette order        */
    int* kept;                /* [n_parents] pixels left in each parent's list   */
    double* hsv;              /* [n_parents*3] calculate_avg_hsv h,s,v           */
    double* pct;              /* [n_parents] percentages                         */
} orc_palette;

/* get_color_palette (color_quantization.c:652-684) plus S-bar, on the image
   (downsampled per image_processing.c:344-366 when rate > 1).
   Returns 0 on success, <0 when the reference's behaviour is undefined. */
int orc_palette_run(const uint8_t* rgb, int height, int width, const orc_config* cfg,
                    orc_palette* out);
void orc_palette_free(orc_palette* p);

/* Per-pixel HSV (image_processing.c:384-415) and arm_octree group id
   (color_quantization.c:131-145) of n interleaved u8 pixels. */
void orc_group_ids(const uint8_t* rgb, long n, const orc_config* cfg, int* gid, double* hsv);

/* rgb2pgm (image_processing.c:505-512) followed by remove_dc_bias
   (blur_profile.c:233-238): out[i] = (0.299r+0.587g+0.114b) - avg. */
void orc_pgm_dc(const uint8_t* rgb, int height, int width, double avg, double* out);

/* pgm_normalize_fft (fft_processing.c:173-213) + cartesian_to_polar_conversion
   (blur_profile.c:427-458) + calculate_blur_profile (blur_profile.c:34-126)
   on a power spectrum of height x wf.  bins/counts are [na*nr] row-major
   [angle][radius].  Returns 0, or -1 if a radius bin falls outside the table. */
int orc_blur_profile(const double* power, int height, int wf, int nr, int na,
                     double* bins, long long* counts, double* fft_max,
                     int* angle_bin_size, int* radius_bin_size);

/* The (phi_bin, r_bin) of one spectrum element (blur_profile.c:87-97). */
void orc_blur_bin_of(int u, int x, int height, int wf, int nr, int na, int* phi_bin, int* r_bin);

/* vectorize_blur_profile (blur_profile.c:324-416). Always 10 vectors. */
void orc_vectorize(const double* bins, int na, int nr, double streak_thresh,
                   double mag_thresh, int cutoff_denom, int angles[10], float mags[10]);

/* newton_int_sqrt (utilities.c:43-52). */
int orc_newton_int_sqrt(double val);

/* get_variance_sharpness (filtering.c:151-183) on the pgm BEFORE dc removal. */
int orc_sharpness(const uint8_t* rgb, int height, int width, int n, const int* top,
                  const int* bottom, const int* left, const int* right, double* out);

#endif
