/* sanitize_main.c -- TEST INFRASTRUCTURE ONLY.
 *
 * Drives the C restatement (phd_oracle.c) under AddressSanitizer and
 * UndefinedBehaviorSanitizer (oracle/Makefile target `sanitize`): every entry
 * point on synthetic images of odd and even sizes, fine and coarse grids,
 * small linked-list sizes (the tie/overflow keep rules), downsampling, crops
 * and a naive DFT power spectrum.  Any sanitizer report aborts with a
 * non-zero status (tests/test_oracle_sanitize.py). */
#define _GNU_SOURCE
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "phd_oracle.h"

static uint64_t mix(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

/* kind 0 uniform, 1 smooth gradient with few colours, 2 one dominant colour */
static void make(uint8_t* rgb, int h, int w, int kind, uint64_t seed) {
    for (long i = 0; i < (long)h * w; i++) {
        const uint64_t r = mix(seed + (uint64_t)(i + 1) * 0x9E3779B97F4A7C15ull);
        const int y = (int)(i / w), x = (int)(i % w);
        for (int c = 0; c < 3; c++) {
            int v;
            if (kind == 0) v = (int)((r >> (8 * c)) & 255);
            else if (kind == 1) v = ((x * (c + 1) + y * (3 - c)) / 7 + (int)((r >> (8 * c)) & 7)) & 255;
            else v = ((r & 15) < 11) ? 40 + 80 * c : (int)((r >> (8 * c)) & 255);
            rgb[3 * i + c] = (uint8_t)v;
        }
    }
}

/* |X|^2 of the rfft2 of (pgm - avg), height x (w/2+1), naive O(N^2) DFT */
static void power(const double* pgm, int h, int w, double* out) {
    const int wf = w / 2 + 1;
    double* re = calloc((size_t)h * wf, sizeof(double));
    double* im = calloc((size_t)h * wf, sizeof(double));
    for (int y = 0; y < h; y++)
        for (int k = 0; k < wf; k++)
            for (int x = 0; x < w; x++) {
                const double a = -2 * M_PI * (double)k * x / w;
                re[(size_t)y * wf + k] += pgm[(size_t)y * w + x] * cos(a);
                im[(size_t)y * wf + k] += pgm[(size_t)y * w + x] * sin(a);
            }
    for (int u = 0; u < h; u++)
        for (int k = 0; k < wf; k++) {
            double sr = 0, si = 0;
            for (int y = 0; y < h; y++) {
                const double a = -2 * M_PI * (double)u * y / h;
                const double xr = re[(size_t)y * wf + k], xi = im[(size_t)y * wf + k];
                sr += xr * cos(a) - xi * sin(a);
                si += xr * sin(a) + xi * cos(a);
            }
            out[(size_t)u * wf + k] = sr * sr + si * si;
        }
    free(re);
    free(im);
}

static int run(int h, int w, int kind, orc_config cfg, int with_blur) {
    uint8_t* rgb = malloc((size_t)h * w * 3);
    make(rgb, h, w, kind, (uint64_t)(h * 131 + w * 7 + kind));
    double st[6];
    orc_rgb_stats(rgb, h, w, st);
    orc_palette pal;
    memset(&pal, 0, sizeof(pal));
    const int rc = orc_palette_run(rgb, h, w, &cfg, &pal);
    if (rc == 0) orc_palette_free(&pal);
    int top[2] = {0, h / 3}, bottom[2] = {h / 2, h}, left[2] = {0, w / 4}, right[2] = {w / 2, w};
    double sh[2];
    orc_sharpness(rgb, h, w, 2, top, bottom, left, right, sh);
    if (with_blur) {
        const int wf = w / 2 + 1;
        double* pgm = malloc(sizeof(double) * (size_t)h * w);
        double* pw = malloc(sizeof(double) * (size_t)h * wf);
        orc_pgm_dc(rgb, h, w, (st[0] + st[1] + st[2]) / 3.0, pgm);
        power(pgm, h, w, pw);
        const int na = cfg.angle_parts, nr = cfg.radius_parts;
        double* bins = malloc(sizeof(double) * na * nr);
        long long* cnt = malloc(sizeof(long long) * na * nr);
        double fmax;
        int abs_, rbs;
        if (orc_blur_profile(pw, h, wf, nr, na, bins, cnt, &fmax, &abs_, &rbs) == 0) {
            int ang[10];
            float mg[10];
            orc_vectorize(bins, na, nr, cfg.streak_thresh, cfg.mag_thresh, cfg.cutoff_denom, ang, mg);
        }
        free(pgm), free(pw), free(bins), free(cnt);
    }
    free(rgb);
    return rc;
}

int main(void) {
    const orc_config base = {18, 2, 3, 0.1, 0.1, 0.95, 1000, 1, 40, 72, 0.1f, 0.9f, 1.20, 0.3, 2};
    orc_config c;
    int n = 0;
    for (int kind = 0; kind < 3; kind++) {
        c = base;
        run(360, 370, kind, c, kind == 1), n++;
        c.linked_list_size = 7;                       /* every tie overflows */
        run(401, 577, kind, c, 0), n++;
        c = base;
        c.h_parts = 36, c.s_parts = 4, c.v_parts = 5, c.coverage = 1.0;
        run(577, 401, kind, c, 0), n++;
        c = base;
        c.downsample_rate = 3;
        run(700, 900, kind, c, 0), n++;
        c = base;
        c.h_parts = 1, c.s_parts = 1, c.v_parts = 1, c.radius_parts = 5, c.angle_parts = 8;
        run(351, 353, kind, c, kind == 0), n++;
    }
    if (!orc_precheck(349, 400) || !orc_precheck(2001, 400)) return 2;
    for (int v = 0; v < 100000; v += 7) (void)orc_newton_int_sqrt((double)v);
    printf("sanitize OK: %d runs\n", n);
    return 0;
}
