/* phd_oracle.c -- TEST INFRASTRUCTURE ONLY (see phd_oracle.h).
 *
 * A clean-room CPU restatement of the reference hot path.  The reference keeps
 * every pixel of every octree group in chains of fixed-size nodes and rewires
 * them (color_quantization.c:108-161, 342-479); this file instead derives, per
 * group, WHICH pixels survive the rewiring (the "keep rules" of SURVEY.md 8a
 * row 8d) and sums them in the order the reference's list walk visits them.
 * Every numeric expression keeps the reference's evaluation order and types so
 * that float results agree bit-for-bit with the -O0 reference build.
 */
#include "phd_oracle.h"

#include <limits.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define REF_PI 3.14159265          /* blur_profile.c:10 (truncated pi) */
#define MAX_SAT 0.999999           /* image_processing.c:8 */
#define MAX_VAL 0.999999           /* image_processing.c:9 */

/* ---------------------------------------------------------------- checks */
int orc_precheck(int height, int width) {
    /* utilities.c:69-81 (the NULL-pointer checks do not apply to a u8 buffer) */
    if (height < 350 || width < 350) return 1;
    if ((long long)height * width > 120000000LL) return 1;
    float ar = (float)height / (float)width;
    if (ar < 1.0 / 5.0 || ar > 5.0 / 1.0) return 1;
    return 0;
}

/* ------------------------------------------------------------ statistics */
void orc_rgb_stats(const uint8_t* rgb, int height, int width, double out[6]) {
    /* get_average / get_variance (filtering.c:125-148), one channel at a time,
       sequential double accumulation of k/255.0 exactly as the reference. */
    long n = (long)height * width;
    for (int c = 0; c < 3; c++) {
        double acc = 0.0;
        for (long i = 0; i < n; i++) acc += (double)rgb[3 * i + c] / 255.0;
        out[c] = acc / (double)n;
    }
    for (int c = 0; c < 3; c++) {
        double acc = 0.0, mu = out[c];
        for (long i = 0; i < n; i++) {
            double d = (double)rgb[3 * i + c] / 255.0 - mu;
            acc += d * d;
        }
        out[3 + c] = sqrt(acc / (double)n);
    }
}

/* ------------------------------------------------------------------ HSV */
void orc_rgb2hsv_px(double r, double g, double b, double* ph, double* ps, double* pv) {
    /* image_processing.c:387-414 */
    double mx = fmax(fmax(r, g), b);
    double mn = fmin(fmin(r, g), b);
    double d = mx - mn;
    double h;
    if (d == 0) h = 0;
    else if (mx == r) h = 60 * ((g - b) / d);
    else if (mx == g) h = 60 * (2 + (b - r) / d);
    else h = 60 * (4 + (r - g) / d);
    if (h < 0) { while (h < 0) h += 360; }
    else if (h > 360) { while (h > 360) h -= 360; }
    *ph = h;
    *pv = (mx == 1) ? MAX_VAL : mx;
    if (mx == 0) *ps = 0;
    else if (d == mx) *ps = MAX_SAT;
    else *ps = d / mx;
}

/* -------------------------------------------------------------- palette */
typedef struct grid {
    int hp, sp, vp, ng, tl;
    double Lh, Ls, Lv, bt, gt;
    double *ch, *cs, *cv;      /* group centres, initialize_octree :57-99 */
} grid;

static int grid_init(grid* G, const orc_config* c) {
    G->hp = c->h_parts; G->sp = c->s_parts; G->vp = c->v_parts; G->ng = c->v_parts;
    if (G->hp <= 0 || G->sp <= 0 || G->vp <= 0) return -1;
    G->tl = G->hp * G->sp * G->vp + G->ng + 1;
    G->Lh = 360 / G->hp;                         /* integer division, :41 */
    G->Ls = (1 - c->gray_thresh) / G->sp;        /* :43 */
    G->Lv = (1 - c->black_thresh) / G->vp;       /* :45 */
    G->bt = c->black_thresh; G->gt = c->gray_thresh;
    G->ch = calloc(G->tl, sizeof(double));
    G->cs = calloc(G->tl, sizeof(double));
    G->cv = calloc(G->tl, sizeof(double));
    double half_h = G->Lh / 2, s_offs = G->Ls / 2 + G->gt, v_offs = G->Lv / 2 + G->bt;
    int i = 0;
    for (int h = 0; h < G->hp; h++)
        for (int s = 0; s < G->sp; s++)
            for (int v = 0; v < G->vp; v++) {
                i = h * G->sp * G->vp + s * G->vp + v;
                G->ch[i] = h * G->Lh + half_h;
                G->cs[i] = s * G->Ls + s_offs;
                G->cv[i] = v * G->Lv + v_offs;
            }
    double l_gray = (1.0f - G->bt) / (double)G->ng;   /* :78 */
    for (int j = 0; j < G->ng; j++) {
        i++;
        G->ch[i] = 0; G->cs[i] = 0; G->cv[i] = l_gray * j + v_offs;
    }
    return 0;   /* black group (TL-1) stays at (0,0,0) */
}

static void grid_free(grid* G) { free(G->ch); free(G->cs); free(G->cv); }

/* arm_octree's group choice (color_quantization.c:131-145). -1 if out of range. */
static int group_of(const grid* G, double h, double s, double v) {
    int g;
    if (v < G->bt) {
        g = G->tl - 1;
    } else if (s < G->gt) {
        /* (int)(v-bt) binds first: for v in [bt,1) this is always gray group 0 */
        int vi = (int)((double)((int)(v - G->bt) * G->ng) / (1 - G->bt));
        g = G->tl - (G->ng + 1) + vi;
    } else {
        int vi = (int)((v - G->bt) / G->Lv);
        int si = (int)((s - G->gt) / G->Ls);
        int hi = (int)(h / G->Lh);
        g = (hi * G->sp + si) * G->vp + vi;
    }
    return (g < 0 || g >= G->tl) ? -1 : g;
}

/* saliency (color_quantization.c:588-595), all float arithmetic. */
static float saliency_of(int q, double s, double v, float qw, float svw) {
    float s_v = s * v;
    float sal = (float)q * (qw + svw * s_v);
    return sal * 1000;
}

/* compare_quantities (:601-611): (int)(sal_b - sal_a) compiled to cvttss2si,
   which yields INT_MIN for NaN and |x| >= 2^31 (the "integer indefinite"). */
static int cmp_sal(float sal_a, float sal_b) {
    float d = sal_b - sal_a;
    if (!(d > -2147483648.0f && d < 2147483648.0f)) return INT_MIN;
    return (int)d;
}

/* get_node_distance_heuristic (:253-288) */
static double node_dist(const grid* G, int gi, int pi) {
    int gray_start = G->tl - (G->ng + 1), black = G->tl - 1;
    if (gi < gray_start && pi < gray_start) {
        double hd = fabs(G->ch[gi] - G->ch[pi]);
        if (hd > 180) hd = 360 - hd;
        hd *= (1.0) / (360.0);
        double sd = G->cs[gi] - G->cs[pi], vd = G->cv[gi] - G->cv[pi];
        return hd * hd + sd * sd + vd * vd;
    }
    if ((gray_start <= gi && gi < black && pi < gray_start) ||
        (gray_start <= pi && pi < black && gi < gray_start)) {
        double sd = G->cs[gi] - G->cs[pi], vd = G->cv[gi] - G->cv[pi];
        return sd * sd + vd * vd;
    }
    double vd = G->cv[gi] - G->cv[pi];
    return vd * vd;
}

/* one segment of a parent's list: `count` pixels of group `grp` starting at
   rank `first` of that group's raster-ordered pixel list */
typedef struct seg { int grp, first, count; } seg;

int orc_palette_run(const uint8_t* rgb, int height, int width, const orc_config* cfg,
                    orc_palette* out) {
    memset(out, 0, sizeof(*out));
    grid G;
    if (grid_init(&G, cfg)) return -1;
    const int L = cfg->linked_list_size;
    if (L <= 0) { grid_free(&G); return -1; }

    /* downsample_rgb (image_processing.c:344-366): new (y,x) <- old row y*(N-1),
       col x*N (the row increment at :351 is one row short). */
    int N = cfg->downsample_rate > 1 ? cfg->downsample_rate : 1;
    int hh = N > 1 ? height / N : height, ww = N > 1 ? width / N : width;
    /* rgb2hsv iterates over (short)height*(short)width pixels (:378-383) */
    long n = (long)(short)hh * (short)ww;
    out->n_hsv = (int)n;
    out->total_length = G.tl;

    double* H = malloc(sizeof(double) * n);
    double* S = malloc(sizeof(double) * n);
    double* V = malloc(sizeof(double) * n);
    int* gid = malloc(sizeof(int) * n);
    double s_acc = 0.0;
    int* hist = calloc(G.tl, sizeof(int));
    for (long j = 0; j < n; j++) {
        long y = j / ww, x = j % ww;
        long src = N > 1 ? (y * (N - 1) * (long)width + x * N) : j;
        double r = (double)rgb[3 * src + 0] / 255.0;
        double g = (double)rgb[3 * src + 1] / 255.0;
        double b = (double)rgb[3 * src + 2] / 255.0;
        orc_rgb2hsv_px(r, g, b, &H[j], &S[j], &V[j]);
        s_acc += S[j];                                   /* :536-538 */
        int grp = group_of(&G, H[j], S[j], V[j]);
        if (grp < 0) { free(H); free(S); free(V); free(gid); free(hist); grid_free(&G); return -2; }
        gid[j] = grp;
        hist[grp]++;
    }
    out->average_saturation = s_acc / (double)n;
    out->hist = hist;

    /* raster-ordered pixel list per group (counting sort) */
    long* start = calloc(G.tl + 1, sizeof(long));
    for (int g = 0; g < G.tl; g++) start[g + 1] = start[g] + hist[g];
    long* fillp = malloc(sizeof(long) * G.tl);
    memcpy(fillp, start, sizeof(long) * G.tl);
    long* order = malloc(sizeof(long) * (n ? n : 1));
    for (long j = 0; j < n; j++) order[fillp[gid[j]]++] = j;
    free(fillp);

    /* find_valid_octree_parents (:174-203): stable insertion sort by saliency
       (custom_sort, utilities.c:132-153), then cover `coverage` of the pixels. */
    float* sal = malloc(sizeof(float) * G.tl);
    for (int g = 0; g < G.tl; g++)
        sal[g] = saliency_of(hist[g], G.cs[g], G.cv[g], cfg->quantity_weight, cfg->sv_weight);
    int* ids = malloc(sizeof(int) * G.tl);
    for (int g = 0; g < G.tl; g++) ids[g] = g;
    for (int i = 1; i < G.tl; i++)
        for (int j = i; j > 0; j--) {
            if (cmp_sal(sal[ids[j]], sal[ids[j - 1]]) < 0) {
                int t = ids[j]; ids[j] = ids[j - 1]; ids[j - 1] = t;
            } else break;
        }
    int goal = (int)((double)n * cfg->coverage);
    int np = -1;
    for (int i = 0; i < G.tl; i++) {
        goal -= hist[ids[i]];
        if (goal <= 0) { np = i + 1; break; }
    }
    free(sal);
    if (np < 0) {   /* reference leaves valid_parents uninitialised (UB) */
        free(ids); free(order); free(start); free(H); free(S); free(V); free(gid);
        grid_free(&G); return -3;
    }
    out->n_parents = np;
    out->parents = malloc(sizeof(int) * np);
    memcpy(out->parents, ids, sizeof(int) * np);
    free(ids);
    char* is_parent = calloc(G.tl, 1);
    int* slot = malloc(sizeof(int) * G.tl);
    for (int i = 0; i < np; i++) { is_parent[out->parents[i]] = 1; slot[out->parents[i]] = i; }

    /* group_irregular_pixels (:342-479) as keep rules.
       tail_fill[p]: pixels in the node cur_groups[p] points at;
       a tie that overflows that node leaves one "dangling" node (its last
       pixel) hanging off the stale tail pointer; any later event on p
       replaces it (:435-440, :459-462). */
    int* tail_fill = malloc(sizeof(int) * np);
    seg** segs = malloc(sizeof(seg*) * np);
    int* nseg = calloc(np, sizeof(int));
    int* capseg = malloc(sizeof(int) * np);
    int* dangle_grp = malloc(sizeof(int) * np);
    for (int i = 0; i < np; i++) {
        int q = hist[out->parents[i]];
        tail_fill[i] = q == 0 ? 0 : ((q - 1) % L) + 1;
        capseg[i] = 8;
        segs[i] = malloc(sizeof(seg) * capseg[i]);
        segs[i][0] = (seg){out->parents[i], 0, q};
        nseg[i] = 1;
        dangle_grp[i] = -1;
    }
    double* dist = malloc(sizeof(double) * np);
    for (int g = 0; g < G.tl; g++) {
        if (hist[g] == 0 || is_parent[g]) continue;
        double best = (double)G.tl * G.tl;   /* :368 */
        int nmin = 0;
        for (int j = 0; j < np; j++) {
            double d = node_dist(&G, g, out->parents[j]);
            if (d < best) { best = d; nmin = 1; }
            else if (d == best) nmin++;
            dist[j] = d;
        }
        int pj = -1;   /* first parent at the minimum, in valid_parents order */
        for (int j = 0; j < np; j++) if (dist[j] == best) { pj = j; break; }
        int ng = hist[g], keep;
        if (nmin > 1) {
            /* tie: get_distance_pixel_to_parent has no return statement; at -O0
               it returns the pixel pointer's bits (a positive subnormal, equal
               for every candidate), so every pixel goes to the FIRST tied parent
               and is appended through the stale tail pointer. */
            int room = L - tail_fill[pj];
            keep = ng < room ? ng : room;
            tail_fill[pj] += keep;
            if (ng > keep) dangle_grp[pj] = g;       /* replaces any older one */
            else if (keep > 0) dangle_grp[pj] = -1;  /* (room>0 => none existed) */
        } else {
            /* single nearest parent: splice the whole chain (:455-474) */
            keep = ng;
            dangle_grp[pj] = -1;
            tail_fill[pj] = ((ng - 1) % L) + 1;
        }
        if (keep > 0) {
            if (nseg[pj] == capseg[pj]) {
                capseg[pj] *= 2;
                segs[pj] = realloc(segs[pj], sizeof(seg) * capseg[pj]);
            }
            segs[pj][nseg[pj]++] = (seg){g, 0, keep};
        }
    }
    free(dist);

    /* calculate_avg_hsv (:510-576), walking each parent's list in order */
    out->kept = malloc(sizeof(int) * np);
    out->hsv = malloc(sizeof(double) * 3 * np);
    out->pct = malloc(sizeof(double) * np);
    double inv_n = 1.0 / (int)n;                     /* :518 */
    for (int i = 0; i < np; i++) {
        int p = out->parents[i];
        double off = 180 - G.ch[p];
        double ht = 0, st = 0, vt = 0;
        int tot = 0;
        for (int k = 0; k <= nseg[i]; k++) {
            const seg* sg;
            seg dseg;
            if (k < nseg[i]) sg = &segs[i][k];
            else {
                if (dangle_grp[i] < 0) break;
                int dg = dangle_grp[i];
                dseg = (seg){dg, hist[dg] - 1, 1};   /* the group's last pixel */
                sg = &dseg;
            }
            for (int t = 0; t < sg->count; t++) {
                long j = order[start[sg->grp] + sg->first + t];
                double tp = H[j] + off;
                if (tp > 360) tp -= 360;
                else if (tp < 0) tp += 360;
                ht += tp; st += S[j]; vt += V[j];
            }
            tot += sg->count;
        }
        double inv = 1.0 / (double)tot;
        double h = ht * inv;
        h -= off;
        if (h < 0) h += 360;
        else if (h > 360) h -= 360;
        out->hsv[3 * i + 0] = h;
        out->hsv[3 * i + 1] = st * inv;
        out->hsv[3 * i + 2] = vt * inv;
        out->pct[i] = (double)tot * inv_n;
        out->kept[i] = tot;
    }
    for (int i = 0; i < np; i++) free(segs[i]);
    free(segs); free(nseg); free(capseg); free(dangle_grp); free(tail_fill);
    free(is_parent); free(slot); free(order); free(start);
    free(H); free(S); free(V); free(gid);
    grid_free(&G);
    return 0;
}

void orc_palette_free(orc_palette* p) {
    free(p->hist); free(p->parents); free(p->kept); free(p->hsv); free(p->pct);
    memset(p, 0, sizeof(*p));
}

void orc_group_ids(const uint8_t* rgb, long n, const orc_config* cfg, int* gid, double* hsv) {
    grid G;
    grid_init(&G, cfg);
    for (long i = 0; i < n; i++) {
        double h, s, v;
        orc_rgb2hsv_px((double)rgb[3 * i] / 255.0, (double)rgb[3 * i + 1] / 255.0,
                       (double)rgb[3 * i + 2] / 255.0, &h, &s, &v);
        gid[i] = group_of(&G, h, s, v);
        if (hsv) { hsv[3 * i] = h; hsv[3 * i + 1] = s; hsv[3 * i + 2] = v; }
    }
    grid_free(&G);
}

/* ------------------------------------------------------------ luminance */
void orc_pgm_dc(const uint8_t* rgb, int height, int width, double avg, double* out) {
    long n = (long)height * width;
    for (long i = 0; i < n; i++) {
        double r = (double)rgb[3 * i] / 255.0, g = (double)rgb[3 * i + 1] / 255.0,
               b = (double)rgb[3 * i + 2] / 255.0;
        double p = 0.299 * r + 0.587 * g + 0.114 * b;   /* image_processing.c:509 */
        out[i] = p - avg;                                /* blur_profile.c:236 */
    }
}

/* ---------------------------------------------------------- blur profile */
int orc_newton_int_sqrt(double val) {
    if (val == 0) return 0;
    double x = val, s;
    for (;;) {
        s = 0.5 * (x + (val / x));
        if (fabs(s - x) < 1) return (int)s;
        x = s;
    }
}

void orc_blur_bin_of(int u, int x, int height, int wf, int nr, int na, int* phi_bin, int* r_bin) {
    /* cartesian_to_polar_conversion (blur_profile.c:439-456): rows below H/2
       use y=u, phi=-atan2; the rest y=H-1-u, phi=+atan2 (for odd H the middle
       row is written twice and the second, "bottom", write wins). */
    int y;
    double phi;
    if (u < height / 2) { y = u; phi = -atan2(y, x); }
    else { y = height - 1 - u; phi = atan2(y, x); }
    int r_sq = x * x + y * y;
    double rbss = (double)((wf * wf + height * height / 4) / (nr * nr));   /* :61 */
    *phi_bin = (int)((phi + REF_PI * 0.5f) / REF_PI * (double)(na - 1)); /* :94 */
    int rb = orc_newton_int_sqrt(((double)r_sq) / rbss);                 /* :96 */
    if (rb == nr) rb--;                                                  /* :97 */
    *r_bin = rb;
}

int orc_blur_profile(const double* power, int height, int wf, int nr, int na,
                     double* bins, long long* counts, double* fft_max,
                     int* angle_bin_size, int* radius_bin_size) {
    long n = (long)height * wf;
    /* pgm_normalize_fft: max seeded from the middle element, strict '<' */
    double mx = power[n / 2];
    for (long i = 0; i < n; i++) if (mx < power[i]) mx = power[i];
    double gs = 1 / (2 * log(sqrt(mx) + 1));
    *fft_max = mx;
    *angle_bin_size = (int)(double)(180 / na);                               /* :56 */
    double max_radius = sqrt(wf * wf + height * height / 4);                 /* :57 */
    *radius_bin_size = (int)(double)(max_radius / nr);                       /* :58 */
    memset(bins, 0, sizeof(double) * na * nr);
    memset(counts, 0, sizeof(long long) * na * nr);
    for (int u = 0; u < height; u++)
        for (int x = 0; x < wf; x++) {
            double p = power[(long)u * wf + x];
            double val = p < 1 ? 0 : log(p) * gs;                            /* :197-198 */
            int pb, rb;
            orc_blur_bin_of(u, x, height, wf, nr, na, &pb, &rb);
            if (pb < 0 || pb >= na || rb < 0 || rb >= nr) return -1;
            counts[pb * nr + rb]++;
            bins[pb * nr + rb] += val;
        }
    for (int k = 0; k < na * nr; k++) {                                      /* :106-116 */
        double q = (double)counts[k];
        if (q != 0) bins[k] /= q;
        else bins[k] = 0;
    }
    return 0;
}

void orc_vectorize(const double* bins, int na, int nr, double streak_thresh,
                   double mag_thresh, int cutoff_denom, int angles[10], float mags[10]) {
    /* vectorize_blur_profile (blur_profile.c:324-416) */
    for (int i = 0; i < 10; i++) { angles[i] = 0; mags[i] = 0.0f; }
    double* tot = calloc(na, sizeof(double));
    double avg = 0;
    int rc = nr / cutoff_denom;
    for (int i = 0; i < na; i++) {
        for (int j = 0; j < rc; j++) tot[i] += bins[i * nr + j];
        avg += tot[i];
    }
    avg /= na;
    /* convolve_1d with a 5-tap box of ones, then /5 (filtering.c:12-34) */
    double* sm = calloc(na, sizeof(double));
    for (int i = 0; i < na; i++) {
        for (int j = 0; j < 5; j++) sm[i] += tot[((i - j) % na + na) % na] * 1.0;
    }
    for (int i = 0; i < na; i++) sm[i] /= 5;
    int idx[10], m = 0;
    if (sm[0] > sm[na - 1] && sm[0] > sm[1] && sm[0] > avg * streak_thresh && m < 10) idx[m++] = 0;
    for (int i = 1; i < na - 1; i++)
        if (sm[i] > sm[i - 1] && sm[i] > sm[i + 1] && sm[i] > avg * streak_thresh && m < 10)
            idx[m++] = i;
    if (sm[na - 1] > sm[na - 2] && sm[na - 1] > sm[0] && sm[na - 1] > avg * streak_thresh && m < 10)
        idx[m++] = na - 1;
    for (int i = 0; i < m; i++) {
        int a = (idx[i] + na / 2) % na;
        const double* sig = bins + (long)a * nr;
        double bavg = 0;
        for (int j = 0; j < rc; j++) bavg += sig[j];
        if (bavg > avg) { angles[i] = 0; mags[i] = 0.0f; continue; }
        int rmax = nr;
        for (int j = 0; j < nr; j++) if (sig[j] < mag_thresh) { rmax = j; break; }
        mags[i] = ((float)rmax / (float)nr);
        angles[i] = (int)(180 * ((float)a / (float)na) - 90);
    }
    free(sm); free(tot);
}

/* --------------------------------------------------------------- sharpness */
int orc_sharpness(const uint8_t* rgb, int height, int width, int n, const int* top,
                  const int* bottom, const int* left, const int* right, double* out) {
    static const double lap[9] = {-1, -1, -1, -1, 8, -1, -1, -1, -1};  /* filtering.c:40-50 */
    for (int k = 0; k < n; k++) {
        if (right[k] > width || left[k] > width || bottom[k] > height || top[k] > height ||
            left[k] < 0 || right[k] < 0 || top[k] < 0 || bottom[k] < 0)
            return -1;                                           /* crop_pgm :215-218 */
        int cw = right[k] - left[k], ch = bottom[k] - top[k];
        if (cw <= 0 || ch <= 0) return -1;
        long cn = (long)cw * ch;
        double* crop = malloc(sizeof(double) * cn);
        for (int y = 0; y < ch; y++)
            for (int x = 0; x < cw; x++) {
                long i = (long)(y + top[k]) * width + x + left[k];
                double r = (double)rgb[3 * i] / 255.0, g = (double)rgb[3 * i + 1] / 255.0,
                       b = (double)rgb[3 * i + 2] / 255.0;
                crop[(long)y * cw + x] = 0.299 * r + 0.587 * g + 0.114 * b;
            }
        double* f = malloc(sizeof(double) * cn);
        for (int y = 0; y < ch; y++)                              /* filter_image :81-107 */
            for (int x = 0; x < cw; x++) {
                double dp = 0.0;
                for (int fy = 0; fy < 3; fy++)
                    for (int fx = 0; fx < 3; fx++) {
                        int iy = y + fy - 1, ix = x + fx - 1;
                        if (iy >= 0 && iy < ch && ix >= 0 && ix < cw)
                            dp += crop[(long)iy * cw + ix] * lap[fy * 3 + fx];
                    }
                f[(long)y * cw + x] = dp;
            }
        double acc = 0;
        for (long i = 0; i < cn; i++) acc += f[i];
        double avg = acc / (double)cn;
        double va = 0;
        for (long i = 0; i < cn; i++) { double d = f[i] - avg; va += d * d; }
        va = va / (double)cn;
        out[k] = va / avg;                                        /* :175 */
        free(f); free(crop);
    }
    return 0;
}
