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
    float rlh2;      // rlh / 2 (exact): the fast path's half-bin quotient (k1_pixel)
    int hp, hp2;     // h_partitions, 2 h_partitions
    int spvp;        // colour codes: 0 .. spvp - 1
    int ac;          // 4 spvp - 2: cell step per hue bin of a colour code
    int gray_cb;     // cgs - 2 hp spvp: gray / black cell base (code >= spvp)
    int gs;          // gray_start: first gray / black group
    int ncell;       // HueCells::count; cell ncell is the dummy of deferred pixels
    int tl;          // groups; group tl is the dummy of deferred pixels (K1's per-group h / s sums)
    int gmg;         // gs - spvp: a gray / black code's group is code + gmg
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

// The one reciprocal a pixel needs (round 6; two before): r = 1 / (kd1 km1)
// with kd1 = max(kd, 1), km1 = max(kmax, 1) (kd1 km1 <= 65025, exact in fp32),
// from the fp32 reciprocal and one fp64 Newton step (1 - p r is exact in an
// fma; ~2^-45 relative).  h = 60 X / kd = (60 X km1) r and s = kd / kmax =
// kd^2 r then take one fp64 multiply of an exact integer each, and the fp32
// 1 / kd of the half-bin quotient is km1 * (fp32 r).  (Two reciprocals cost
// eight fp64 instructions per pixel, this one four; fp64 issues at half rate.)
struct K1Inv {
    double inv;      // 1 / (kd1 km1)
    float rkd;       // 1 / kd1 in fp32: <= 1.5 ulp on the device, 1 ulp on the host
    unsigned pad;
};
K1_HD K1Inv k1_inv_p(int p, int km1) {      // p = kd1 km1 (the kernel forms it for a u16 pair at once)
    const float pf = (float)p;
#if defined(__HIP_DEVICE_COMPILE__)
    const float r = __builtin_amdgcn_rcpf(pf);
#else
    const float r = 1.0f / pf;
#endif
    // the Newton residual 1 - p r in ONE fp32 fma (p r exact inside it; |1 - p
    // r| <= 2^-23, so its fp32 rounding errs by <= 2^-47), then r (1 + e) in
    // fp64: three fp64 instructions instead of four, ~2^-46 relative
    const float e = std::fma(-pf, r, 1.0f);
    const double d = (double)r;
    return K1Inv{std::fma(d, (double)e, d), (float)km1 * r, 0u};
}
K1_HD K1Inv k1_inv_pair(int kd1, int km1) { return k1_inv_p(k1_mul(kd1, km1), km1); }

// 1 / x in fp32: v_rcp_f32 on the device (<= 1 ulp), correctly rounded on the host
K1_HD float k1_rcpf(float x) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_rcpf(x);
#else
    return 1.0f / x;
#endif
}

// q - floor(q) for 0 <= q < 2^23 (exact in fp32)
K1_HD float k1_fract(float q, int c) {
#if defined(__HIP_DEVICE_COMPILE__)
    (void)c;
    return __builtin_amdgcn_fractf(q);
#else
    return q - (float)c;
#endif
}

K1_HD void k1_grid_init(K1Grid& G, const GridParams& g) {
    G.lh = 360 / g.hp;
    G.rlh = 1.0f / (float)G.lh;
    G.rlh2 = 0.5f * G.rlh;
    G.hp = g.hp;
    G.hp2 = 2 * g.hp;
    G.spvp = g.sp * g.vp;
    G.ac = 4 * G.spvp - 2;
    G.gs = g.tl - g.ng - 1;
    G.gray_cb = 4 * G.gs - G.hp2 * G.spvp;
    G.ncell = 4 * G.gs + (g.ng + 1) * 2 * g.hp;
    G.tl = g.tl;
    G.gmg = G.gs - G.spvp;
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
    int grp;         // the cell's group (arm_octree's), tl when deferred
    unsigned dfr;    // 1 when deferred
    unsigned lo, hi; // the cell word: lo = 1 | (kmax == 255) << 16, hi = kmax
    double h, s;
};

// What a code contributes to its pixel's hue cell and group (round 6: read per
// pixel from a small LDS table, code-indexed, instead of selecting between the
// colour and the gray / black formulas): cell = a + m (c / 2) + c - below,
// group = g0 + mg (c / 2).  Colour code: a = 4 code + 1, m = 4 spvp - 2, g0 =
// code, mg = spvp (cell = 4 (hi spvp + code) + 1 + c - 2 hi - below); gray /
// black code: a = gray_cb + code 2 hp, g0 = code + gs - spvp, m = mg = 0.
struct K1Code {
    unsigned short a, m, g0, mg;   // all non-negative (ncell < 2^16: codes_ok grids)
};
K1_HD K1Code k1_code_entry(const K1Grid& G, int code) {
    K1Code e;
    if (code < G.spvp) {
        e.a = (unsigned short)(4 * code + 1);
        e.m = (unsigned short)G.ac;
        e.g0 = (unsigned short)code;
        e.mg = (unsigned short)G.spvp;
    } else {
        e.a = (unsigned short)(G.gray_cb + code * G.hp2);
        e.m = 0;
        e.g0 = (unsigned short)(code + G.gmg);
        e.mg = 0;
    }
    return e;
}
// codes of a grid: spvp colour codes, then the gray groups and black
K1_HD int k1_ncodes(const K1Grid& G) { return G.spvp + G.tl - G.gs; }

typedef unsigned short k1_u16x2 __attribute__((ext_vector_type(2)));
typedef short k1_i16x2 __attribute__((ext_vector_type(2)));

// X = sector kd + num (k1_pixel) for the two pixels of a u16 pair at once, in
// 16-bit lanes (round 6; v_pk_* ops on the device, ~8 VALU per pixel instead
// of ~15): the three branch values, and the first-max selection by masks --
// (max - 1) - channel is -1 exactly where that channel is the max (it is
// never below -1), so its arithmetic shift by 15 is the all-ones select mask.
// All values fit i16 (|X| < 6 * 256).
// The all-ones mask of each 16-bit lane of x that is negative.  On the device
// an opaque v_pk_ashrrev_i16: the compiler would otherwise see the sign splat,
// turn the mask-and-merge below into per-lane compares and selects and repack
// the halves (13 VALU per pair instead of 4).
K1_HD k1_i16x2 k1_neg_mask(k1_i16x2 x) {
#if defined(__HIP_DEVICE_COMPILE__)
    unsigned r;
    asm("v_pk_ashrrev_i16 %0, 15, %1 op_sel_hi:[0,1]" : "=v"(r) : "v"(__builtin_bit_cast(unsigned, x)));
    return __builtin_bit_cast(k1_i16x2, r);
#else
    return x >> (k1_i16x2){15, 15};
#endif
}

K1_HD k1_u16x2 k1_x_pair(k1_u16x2 r, k1_u16x2 g, k1_u16x2 b, k1_u16x2 mx, k1_u16x2 kd) {
    const k1_i16x2 R = __builtin_bit_cast(k1_i16x2, r), Gc = __builtin_bit_cast(k1_i16x2, g),
                   B = __builtin_bit_cast(k1_i16x2, b), K = __builtin_bit_cast(k1_i16x2, kd);
    const k1_i16x2 m1 = __builtin_bit_cast(k1_i16x2, mx) - (k1_i16x2){1, 1};
    const k1_i16x2 sh15 = {15, 15};
    const k1_i16x2 mr = k1_neg_mask(m1 - R);                   // -1: r is the max (first)
    const k1_i16x2 mg = k1_neg_mask(m1 - Gc);                  // -1: g is the max
    const k1_i16x2 d = Gc - B;
    const k1_i16x2 xr = d + ((d >> sh15) & (K * (k1_i16x2){6, 6}));   // g - b, + 6 kd when negative
    const k1_i16x2 xg = (K << (k1_i16x2){1, 1}) + B - R;
    const k1_i16x2 xb = (K << (k1_i16x2){2, 2}) + R - Gc;
    const k1_i16x2 X = (mr & xr) | (~mr & ((mg & xg) | (~mg & xb)));
    return __builtin_bit_cast(k1_u16x2, X);
}

// The fast path.  kd = kmx - kmn; code = the table's byte for (kmx, kd); e =
// k1_inv_pair(max(kd, 1), max(kmx, 1)) (the caller computes it with the code
// read, ahead of the previous pixels' LDS atomics).  Deferred pixels get cell
// = ncell (their count and sums land in the dummy cell, never read) and are
// redone by k1_exact.
//
// The half-bin cell and the boundary test (round 6): with u = 1 / (Lh kd1),
// the exact quotient q* = (n2 + 1/2) u = m + (j + 1/2) u, m = floor(n2 u), j =
// n2 mod (Lh kd1); the pixel is on a boundary (onb) iff j = 0.  The fp32 q =
// (2 n2 + 1) * (rlh/2 * rkd) errs by at most ~3 ulp = 3.6e-7 q* relative (2 n2
// + 1 exact, rlh/2 0.5 ulp, rkd 1.5, two products 0.5 each); as q* < 720 / Lh
// + 1 and u >= 1 / (255 Lh), that is at most 3.6e-7 (720 + Lh) 255 u <= 0.1 u
// for every Lh <= 360 and kd <= 255.  So c = (int)q = m, and fract(q) lies within 0.1 u of (j + 1/2) u: in
// [0.4 u, 0.6 u] on a boundary, >= 1.4 u off it; the threshold thr = 2 (rlh/2
// rkd) = u (1 +- 3e-7) splits them with 0.4 u to spare on both sides, on the
// device (v_rcp_f32, 1 ulp) and on the host (correctly rounded) alike.  (Before
// round 6: onb = (c Lh kd1 == n2), one quarter-rate v_mul_lo_u32 per pixel.)
//
// k1_pixel_x takes X from k1_x_pair (the kernel) and `special` (two channels
// equal; read only by the !SMALL form); k1_pixel computes both itself.
template <bool SMALL>   // SMALL == G.small_c
K1_HD K1Px k1_pixel_x(int X, bool special, int kmx, int kmn, int kd, const K1Code& ce, const K1Inv& e,
                      const K1Grid& G) {
    const int km1 = kmx > 1 ? kmx : 1;
    const float thr2 = G.rlh2 * e.rkd;                          // u / 2
    // (2 n2 + 1) u / 2 with one rounding: the fma of the exact 240 X
    const float q = std::fma((float)k1_mul(240, X), thr2, thr2);   // (n2 + 1/2) u, n2 = 120 X
    const int c = (int)q;
    const unsigned onb = k1_fract(q, c) < thr2 + thr2 ? 1u : 0u;
    unsigned below, def;        // 0 / 1
    if (SMALL) {
        // one 64-bit shift of a uniform mask per property (v_lshrrev_b64; the
        // two 32-bit words selected by c >= 32 cost a compare, two moves of
        // the words and a select each), its low bit masked by onb
        below = onb & (unsigned)(G.below_m >> c);
        def = onb & (unsigned)(G.defer_m >> c);
    } else {
        const int ch = c - G.hp;
        below = onb && special && ch >= 0 && ((ch & 1) || ch == 0);
        def = onb && !special;
    }
    // colour: 4 (hi spvp + code) + 1 + (c - 2 hi); gray / black: 4 gs + j 2 hp + c
    // (K1Code); its group: colour (c / 2) spvp + code (= cell / 4), gray /
    // black code + gs - spvp
    const int hi = c >> 1;
    const int cell = (int)ce.a + k1_mul(ce.m, hi) + c - (int)below;
    const int grp = (int)ce.g0 + k1_mul(ce.mg, hi);
    K1Px p;
    p.cell = def ? G.ncell : cell;
    p.grp = def ? G.tl : grp;
    p.dfr = def;
    p.lo = 1u + ((unsigned)((kmx + 1) >> 8) << 16);
    p.hi = (unsigned)kmx;
    // rgb2hsv: h = 60 X / kd (0 for kd = 0); s = kd / kmx, 0.999999 when
    // min == 0 < max (src/image_processing.c:408-414), 0 for black
    p.h = (double)k1_mul(k1_mul(X, km1), 60) * e.inv;       // 60 X km1 < 2^25
    p.s = (kmn == 0 && kmx != 0) ? 0.999999 : (double)k1_mul(kd, kd) * e.inv;     // black: kd = 0
    return p;
}

template <bool SMALL>
K1_HD K1Px k1_pixel(int kr, int kg, int kb, int kmx, int kmn, int kd, int code, const K1Inv& e,
                    const K1Grid& G) {
    const bool isr = kr == kmx, isg = kg == kmx;
    // X = sector kd + num: rgb2hsv's three branches (max == r first, then g)
    const int t1 = isg ? kb - kr : kr - kg;
    const int xs = (kd << (isg ? 1 : 2)) + t1;
    const int xr = kg - kb + (kg < kb ? k1_mul(6, kd) : 0);
    const int X = isr ? xr : xs;
    const bool special = (kr == kg) | (kg == kb) | (kr == kb);
    return k1_pixel_x<SMALL>(X, special, kmx, kmn, kd, k1_code_entry(G, code), e, G);
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
    // (round 6: v_rcp_f32 on the device, the <= 1 ulp k1_halfbin allows, where
    // 1.0f / kd1 was a correctly rounded division of ~12 instructions)
    const int c = k1_halfbin(n2, k1_rcpf((float)kd1), G);           // as k1_pixel: exact
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
        p.grp = hi * G.spvp + code;
        p.cell = 4 * p.grp + (l < 0 ? 0 : (l > 3 ? 3 : l));
    } else {
        p.grp = code + G.gmg;
        p.cell = G.gray_cb + code * G.hp2 + cg;
    }
    p.dfr = 0u;
    p.lo = 1u + ((unsigned)((kmx + 1) >> 8) << 16);
    p.hi = (unsigned)kmx;
    p.h = h;
    // s as the fast path's (kd^2 / (kd1 km1) through k1_inv_pair, ~2^-45
    // relative; round 6, where kd * (1.0 / kmx) took an fp64 division)
    const int km1 = kmx > 1 ? kmx : 1;
    p.s = kmn == 0 && kmx != 0 ? 0.999999 : (double)k1_mul(kd, kd) * k1_inv_pair(kd1, km1).inv;
    return p;
}

}  // namespace phd
