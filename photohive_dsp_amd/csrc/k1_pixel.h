// k1_pixel.h -- K1's per-pixel classification (k1.hip), host + device.
//
// One pixel (kr, kg, kb) of the full report's first pass becomes one hue cell
// of the fused palette (HueCells layout, phd_internal.h) plus the h and s that
// rgb2hsv gives it (src/image_processing.c:384-415); arm_octree's group
// (src/color_quantization.c:131-145) is a function of the cell.  The same
// source runs in the kernel and, through phd_debug_k1_pixels, on the host,
// where tests/test_k1_pixel.py checks it against the oracle over every RGB8
// triple.
//
// The hue is the exact rational h = 60 X / kd with X = sector * kd + num in
// [0, 6 kd) (kd = max - min); its half-bin cell c = floor(2 h / Lh) =
// floor(120 X / (Lh kd)) is integer arithmetic (an fp32 reciprocal whose
// error stays far inside the 0.5 / (Lh kd) margin, since 120 X < 2^18).  A
// pixel whose rational hue lies exactly on a half-bin boundary (onb) is either
//   * special (two channels equal: X / kd is an integer, i.e. the boundary is
//     a multiple of 60 degrees, where rgb2hsv's double hue is exact): it stays
//     on the fast path, counted on the side calculate_avg_hsv's wrap test
//     puts an exact boundary hue (`below`, src/color_quantization.c:527-547);
//   * otherwise deferred: rgb2hsv's double rounding decides its hue bin and
//     side, so k1_exact evaluates the reference's own double expression.
// Everything arm_octree decides without the hue (black, the gray group, or
// the colour group's (Si, Vi)) is one byte `code` of a table built on the host
// from the reference's doubles (make_class_tables).
#pragma once

#include <cmath>

#include "phd_internal.h"

#if defined(__HIPCC__)
#define K1_HD __host__ __device__ __forceinline__
#else
#define K1_HD inline
#endif

namespace phd {

// Grid constants of one launch (uniform).
struct K1Grid {
    int lh;          // Lh = 360 / h_partitions (integer, color_quantization.c:41)
    float rlh;       // 1 / Lh in fp32 (k1_halfbin)
    int hp, hp2;     // h_partitions, 2 h_partitions
    int spvp;        // colour codes: 0 .. spvp - 1
    int ac;          // 4 spvp - 2: cell step per hue bin of a colour code
    int gray_cb;     // cgs - 2 hp spvp: gray / black cell base (code >= spvp)
    int gs;          // gray_start: first gray / black group
    int ncell;       // HueCells::count; cell ncell is the dummy of deferred pixels
    int small_c;     // every c < 64: the boundary properties are bit masks
    unsigned long long below_m;   // bit c: an exact boundary hue at B_c counts below it
    unsigned long long defer_m;   // bit c: B_c is not a multiple of 60 (onb pixels defer)
};

// a * b for 0 <= a, b < 2^24 (and a * b < 2^32): one full-rate v_mul_u32_u24
// on the device, where a 32-bit v_mul_lo_u32 is quarter rate
K1_HD int k1_mul(int a, int b) {
#if defined(__HIP_DEVICE_COMPILE__)
    return (int)__umul24((unsigned)a, (unsigned)b);
#else
    return a * b;
#endif
}

// The reciprocals a pixel needs, per k in [1, 255]: 1 / k to double (h = 60 X
// / kd and s = kd / kmax as one multiply each, within an ulp of the exact
// rational) and to float (the half-bin cell's fp32 quotient).
struct K1Inv {
    double inv;
    float rcp;
    unsigned pad;
};
// From the VALU: the fp32 reciprocal and one fp64 Newton step (1 - k r is
// exact in an fma; ~2^-45 relative), no table read.
K1_HD K1Inv k1_inv_valu(int k) {
#if defined(__HIP_DEVICE_COMPILE__)
    const float r = __builtin_amdgcn_rcpf((float)k);
#else
    const float r = 1.0f / (float)k;
#endif
    const double d = (double)r;
    const double e = std::fma(-(double)k, d, 1.0);
    return K1Inv{std::fma(d, e, d), r, 0u};
}

K1_HD void k1_grid_init(K1Grid& G, const GridParams& g) {
    G.lh = 360 / g.hp;
    G.rlh = 1.0f / (float)G.lh;
    G.hp = g.hp;
    G.hp2 = 2 * g.hp;
    G.spvp = g.sp * g.vp;
    G.ac = 4 * G.spvp - 2;
    G.gs = g.tl - g.ng - 1;
    G.gray_cb = 4 * G.gs - G.hp2 * G.spvp;
    G.ncell = 4 * G.gs + (g.ng + 1) * 2 * g.hp;
    // c < 720 / Lh (X < 6 kd)
    G.small_c = (720 + G.lh - 1) / G.lh <= 64;
    G.below_m = G.defer_m = 0ull;
    for (int c = 0; c < 64 && G.small_c; c++) {
        const bool mult60 = (c * G.lh) % 120 == 0;            // B_c = c Lh / 2 is a multiple of 60
        const int ch = c - g.hp;
        const bool below = mult60 && ch >= 0 && ((ch & 1) || ch == 0);
        if (below) G.below_m |= 1ull << c;
        if (!mult60) G.defer_m |= 1ull << c;
    }
}

// c = floor(n2 / (Lh kd1)) for n2 = 120 X < 2^18: q = (n2 + 1/2) / (Lh kd1)
// lies at least 1/2 / (Lh kd1) from an integer, i.e. a relative margin of
// 0.5 / (n2 + 0.5) >= 2.7e-6 (n2 < 120 * 6 * 255).  The fp32 form below
// (n2 + 1/2 exact; 1 / Lh correctly rounded, 0.5 ulp; 1 / kd1 from
// v_rcp_f32 on the device, <= 1 ulp, correctly rounded on the host; two
// products, 0.5 ulp each) errs by at most 2.5 ulp = 3.0e-7 relative, nine
// times inside the margin, so device and host agree on c for every Lh <= 360
// and kd <= 255.  (tests/test_k1_pixel.py runs the host twin over the RGB
// cube; test_table_k1_exhaustive_rgb_cube_palette runs the device kernel.)
K1_HD int k1_halfbin(int n2, float rkd, const K1Grid& G) {
    return (int)(((float)n2 + 0.5f) * G.rlh * rkd);
}

struct K1Px {
    int cell;        // ncell when deferred
    unsigned lo, hi; // the cell word: lo = 1 | (kmax == 255) << 16, hi = kmax
    double h, s;
};

// The fast path.  kd = kmx - kmn; code = the table's byte for (kmx, kd); ekd
// = the K1Inv entry of max(kd, 1), ikm = 1 / max(kmx, 1) (the caller reads
// them with the code, ahead of the previous pixels' LDS atomics).  Deferred
// pixels get cell = ncell (their count and sums land in the dummy cell, never
// read) and are redone by k1_exact.
template <bool SMALL>   // SMALL == G.small_c
K1_HD K1Px k1_pixel(int kr, int kg, int kb, int kmx, int kmn, int kd, int code, const K1Inv& ekd, double ikm,
                    const K1Grid& G) {
    const int kd1 = kd > 1 ? kd : 1;
    const bool isr = kr == kmx, isg = kg == kmx;
    // X = sector kd + num: rgb2hsv's three branches (max == r first, then g)
    const int t1 = isg ? kb - kr : kr - kg;
    const int xs = (kd << (isg ? 1 : 2)) + t1;
    const int xr = kg - kb + (kg < kb ? k1_mul(6, kd) : 0);
    const int X = isr ? xr : xs;
    const int n2 = k1_mul(120, X);
    const int D = k1_mul(G.lh, kd1);
    const int c = k1_halfbin(n2, ekd.rcp, G);
    const bool onb = k1_mul(c, D) == n2;
    bool below, def;
    if (SMALL) {
        // one 64-bit shift of a uniform mask per property (v_lshrrev_b64; the
        // two 32-bit words selected by c >= 32 cost a compare, two moves of
        // the words and a select each)
        below = onb && (unsigned)(G.below_m >> c) & 1u;
        def = onb && (unsigned)(G.defer_m >> c) & 1u;
    } else {
        const bool special = (kr == kg) | (kg == kb) | (kr == kb);
        const int ch = c - G.hp;
        below = onb && special && ch >= 0 && ((ch & 1) || ch == 0);
        def = onb && !special;
    }
    const bool color = code < G.spvp;
    // colour: 4 (hi spvp + code) + 1 + (c - 2 hi); gray / black: 4 gs + j 2 hp + c
    const int mul = color ? 4 : G.hp2;
    const int add = color ? k1_mul(c >> 1, G.ac) + 1 : G.gray_cb;
    const int cell = k1_mul(code, mul) + add + c - (below ? 1 : 0);
    K1Px p;
    p.cell = def ? G.ncell : cell;
    p.lo = 1u + ((unsigned)((kmx + 1) >> 8) << 16);
    p.hi = (unsigned)kmx;
    // rgb2hsv: h = 60 X / kd (0 for kd = 0); s = kd / kmx, 0.999999 when
    // min == 0 < max (src/image_processing.c:408-414), 0 for black
    p.h = (double)k1_mul(60, X) * ekd.inv;
    p.s = (kmn == 0 && kmx != 0) ? 0.999999 : (double)kd * ikm;     // black: kd = 0
    return p;
}

// A deferred pixel: rgb2hsv's double hue (the reference's expression on the
// doubles k / 255.0, k255[k]) decides the hue bin ((int)(h / Lh),
// color_quantization.c:143) and the side of B_c the wrap test puts h on.
// (k255 == nullptr: k / 255.0 divided here, the same correctly rounded double)
K1_HD double k1_hue_exact(int kr, int kg, int kb, const double* k255) {
    const double r = k255 ? k255[kr] : (double)kr / 255.0, g = k255 ? k255[kg] : (double)kg / 255.0,
                 b = k255 ? k255[kb] : (double)kb / 255.0;
    const int kmx = kr > kg ? (kr > kb ? kr : kb) : (kg > kb ? kg : kb);
    const int kmn = kr < kg ? (kr < kb ? kr : kb) : (kg < kb ? kg : kb);
    const double d = (k255 ? k255[kmx] : (double)kmx / 255.0) - (k255 ? k255[kmn] : (double)kmn / 255.0);
    const bool isr = kr == kmx, isg = kg == kmx;
    const double num = isr ? g - b : (isg ? b - r : r - g);
    const double sector = isr ? 0.0 : (isg ? 2.0 : 4.0);
    double h = 60 * (sector + num / d);
    h = kmx == kmn ? 0.0 : h;
    return h < 0 ? h + 360 : h;
}

K1_HD K1Px k1_exact(int kr, int kg, int kb, int code, double Lh, const double* k255, const K1Grid& G) {
    const double h = k1_hue_exact(kr, kg, kb, k255);
    const int kmx = kr > kg ? (kr > kb ? kr : kb) : (kg > kb ? kg : kb);
    const int kmn = kr < kg ? (kr < kb ? kr : kb) : (kg < kb ? kg : kb);
    const int kd = kmx - kmn, kd1 = kd > 1 ? kd : 1;
    const bool isr = kr == kmx, isg = kg == kmx;
    const int t1 = isg ? kb - kr : kr - kg;
    const int X = isr ? kg - kb + (kg < kb ? 6 * kd : 0) : (kd << (isg ? 1 : 2)) + t1;
    const int n2 = 120 * X;
    const int c = k1_halfbin(n2, 1.0f / (float)kd1, G);             // as k1_pixel: exact
    const double B = (double)c * (double)G.lh * 0.5;
    const int ch = c - G.hp;
    int below;
    if (ch < 0) below = ((c + G.hp) & 1) ? (int)((h + (-B)) < 0) : 0;   // off = 180 - hp_j = -B
    else if (ch == 0) below = (int)!((h + 180.0) > 360);                // gray / black parent, off = 180
    else if (ch & 1) below = (int)!((h + (360.0 - B)) > 360);           // off = 360 - B
    else below = 0;
    const int cg = c - below;
    K1Px p;
    if (code < G.spvp) {
        const int hi = (int)(h / Lh);
        const int l = cg - 2 * hi + 1;
        p.cell = 4 * (hi * G.spvp + code) + (l < 0 ? 0 : (l > 3 ? 3 : l));
    } else {
        p.cell = G.gray_cb + code * G.hp2 + cg;
    }
    p.lo = 1u + ((unsigned)((kmx + 1) >> 8) << 16);
    p.hi = (unsigned)kmx;
    p.h = h;
    p.s = kmx == 0 ? 0.0 : (kmn == 0 ? 0.999999 : (double)kd * (1.0 / (double)kmx));
    return p;
}

}  // namespace phd
