// phd_device.h -- device helpers shared by the HIP kernels.
//
// Every fp64 expression keeps the reference's operation order; the library is
// compiled with -ffp-contract=off so no multiply-add is fused, and HIP's fp64
// '/' is the IEEE correctly-rounded division, so results are bit-identical to
// the reference's x86-64 SSE2 code.
#pragma once

#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

// Ablation switches for timing experiments exist only in builds made with
// -DPHD_ABLATE_BUILD (a separate library, tools/); in the product they are 0.
#ifdef PHD_ABLATE_BUILD
#define PHD_ABL(x) (x)
#else
#define PHD_ABL(x) 0
#endif

#include <algorithm>

#include "phd_internal.h"

namespace phd {

// Every kernel launch of the library: a profiled launch (launch_events set)
// records the profiler's events with the dispatch itself.
template <typename F, typename... Args>
inline void phd_launch(F kernel, dim3 grid, dim3 block, size_t lds, hipStream_t st, Args... args) {
    LaunchEvents& e = launch_events();
    const bool timed = (e.start != nullptr || e.stop != nullptr) && !e.used;
    hipExtLaunchKernelGGL(kernel, grid, block, (std::uint32_t)lds, st, timed ? e.start : nullptr,
                          timed ? e.stop : nullptr, 0u, args...);
    if (timed) e.used = true;
}


// rgb2hsv for one pixel (src/image_processing.c:387-414).  The inputs are the
// doubles k/255.0 of the reference's planar image (utils.py:30-46).
__device__ __forceinline__ void rgb2hsv(double r, double g, double b, double& h, double& s,
                                        double& v) {
    const double mx = fmax(fmax(r, g), b);
    const double mn = fmin(fmin(r, g), b);
    const double d = mx - mn;
    if (d == 0) h = 0;
    else if (mx == r) h = 60 * ((g - b) / d);
    else if (mx == g) h = 60 * (2 + (b - r) / d);
    else h = 60 * (4 + (r - g) / d);
    // only the first branch can go negative (>= -60): one wrap == the while loop
    if (h < 0) h += 360;
    v = (mx == 1) ? 0.999999 : mx;
    s = (mx == 0) ? 0.0 : ((d == mx) ? 0.999999 : d / mx);
}

// arm_octree's group choice (src/color_quantization.c:131-145).
__device__ __forceinline__ int group_of(const GridParams& gp, double h, double s, double v) {
    if (v < gp.bt) return gp.tl - 1;
    if (s < gp.gt) {
        // `(int)(v - bt)` binds before the multiply: gray pixels all map to
        // gray group 0 for v in [bt, 1).
        const int vi = (int)((double)((int)(v - gp.bt) * gp.ng) / (1 - gp.bt));
        return gp.tl - (gp.ng + 1) + vi;
    }
    const int vi = (int)((v - gp.bt) / gp.Lv);
    const int si = (int)((s - gp.gt) / gp.Ls);
    const int hi = (int)(h / gp.Lh);
    return (hi * gp.sp + si) * gp.vp + vi;
}

// Group id of a pixel (or -2: take the exact path) and its HSV saturation.
// Vi, the gray group and Si come from tables of the reference's own double
// results; the hue bin is exact integer arithmetic: with N = 60*num + base*d
// and D = Lh*d (num = the channel difference of rgb2hsv's branch, d = max -
// min, base = 0/120/240, or 360 for a negative red-sector hue), Hi = floor(N/D).
// N, D < 2^17, so (N + 0.5) * rcp(D) in fp32 is within 0.02 of the half-way
// gap to any integer and truncates to floor(N/D) exactly.  When D divides N
// and num is not 0 or +-d, the reference's double hue may round either side
// of the edge: those pixels (-2) take the fp64 path.  Select-only code.
// 1 / k for k in [1, 255] to within an ulp (v_rcp_f64 + one Newton step).
__device__ __forceinline__ double inv_k(int k) {
    const double d = (double)k;
    const double r = __builtin_amdgcn_rcp(d);
    return fma(fma(-d, r, 1.0), r, r);
}

// rgb2hsv's s (src/image_processing.c:408-414) to within an ulp: 0 for d == 0,
// 0.999999 for d == max, else d / max.  Feeds only sums (S-bar, palette).
__device__ __forceinline__ double sat_of(int kmx, int kmn) {
    const int kd = kmx - kmn;
    const double s = (double)kd * inv_k(max(kmx, 1));
    return kd == 0 ? 0.0 : (kmn == 0 ? 0.999999 : s);
}

// Si of arm_octree (src/color_quantization.c:140) for (kmax, kd): the threshold
// count of the pixel's ClsEnt (kThr: FastCls::use_thr), or the full table in
// global memory.  Kernels are instantiated for both, so the per-pixel code has
// no branch and no global load on the threshold path.
template <bool kThr>
__device__ __forceinline__ int si_of(const ClsEnt& e, int kmx, int kd, const signed char* si8g) {
    if constexpr (kThr) {
        const unsigned u = (unsigned)kd;
        return -1 + (int)(u >= (e.thr[0] & 0xFFFFu)) + (int)(u >= (e.thr[0] >> 16)) +
               (int)(u >= (e.thr[1] & 0xFFFFu)) + (int)(u >= (e.thr[1] >> 16)) +
               (int)(u >= (e.thr[2] & 0xFFFFu)) + (int)(u >= (e.thr[2] >> 16));
    }
    return si8g[(kmx << 8) | kd];
}

// classify() from the pixel's table entry (ent[max channel], read by the
// caller so that several pixels' LDS reads are in flight together).
// Branch-free: bitwise ands and selects only.
// Also returns hN and hD: rgb2hsv's hue is hN / hD exactly (hD = max - min,
// or hN = 0, hD = 1 for a gray pixel), so a caller that needs h for sums gets it
// from one reciprocal, and gcol, the colour group of hue bin floor(N / D): for
// a -2 pixel (on a bin edge) the exact group is gcol or the group one hue bin
// below (the reference's double hue rounds to either side of the edge).
template <bool kThr>
__device__ __forceinline__ int classify_e(int kr, int kg, int kb, const ClsEnt& e, const signed char* si8g,
                                          const GridParams& gp, const FastCls& F, int& hN, int& hD, int& gcol) {
    const int kmx = max(kr, max(kg, kb)), kmn = min(kr, min(kg, kb)), kd = kmx - kmn;
    const int si = si_of<kThr>(e, kmx, kd, si8g);
    // hue bin
    const bool isr = kr == kmx, isg = kg == kmx;
    const int a = isr ? kg : (isg ? kb : kr), b = isr ? kb : (isg ? kr : kg);
    const int num = a - b;
    const int base = isr ? (num < 0 ? 360 : 0) : (isg ? 120 : 240);
    const int kd1 = max(kd, 1);
    const int N = __mul24(base, kd1) + 60 * num, D = __mul24(F.lh, kd1);
    hN = kd == 0 ? 0 : N;
    hD = kd1;
    const int hi = (int)(((float)N + 0.5f) * __builtin_amdgcn_rcpf((float)D));
    const int special = (int)(num == 0) | (int)(num == kd) | (int)(num == -kd);
    const int edge = (special ^ 1) & (int)(__mul24(hi, D) == N);
    const int vi = (e.vpack << 16) >> 16, gray = e.vpack >> 16;
    const int g = __mul24(__mul24(hi, gp.sp) + si, gp.vp) + vi;
    gcol = g;
    // black (v < bt) > gray (s < gt) > edge > colour, as masks: a select chain
    // here is turned into a branch around the whole hue arithmetic
    const int mblack = -(int)(vi < 0);
    const int mgray = -(int)(si < 0) & ~mblack;
    const int medge = -edge & ~(mblack | mgray);
    return (g & ~(mblack | mgray | medge)) | ((gp.tl - 1) & mblack) | (gray & mgray) | (-2 & medge);
}

template <bool kThr>
__device__ __forceinline__ int classify_e(int kr, int kg, int kb, const ClsEnt& e, const signed char* si8g,
                                          const GridParams& gp, const FastCls& F, int& hN, int& hD) {
    int gcol;
    return classify_e<kThr>(kr, kg, kb, e, si8g, gp, F, hN, hD, gcol);
}

// The fused K1's classification: classify_e() on the half-bin grid (cells of
// Lh/2 = the wrap thresholds of calculate_avg_hsv, see HueCells) plus the
// pixel's hue cell.  c = floor(2h / Lh) from the same exact integer form
// (2N < 2^18 keeps the fp32 margin); the hue bin is c >> 1.  A non-special
// pixel exactly on a half-bin boundary -- of any kind, grey and black
// included, since its wrap side needs the reference's double -- returns -2
// and is resolved after the stream (fused_exact).  A special pixel on a
// boundary has the exact double hue B_c, which wraps for no parent whose
// threshold is B_c: it goes to the side that never wraps (below for the
// up-wrap thresholds B_c >= 180, above otherwise).  `cell` is the index into
// the image's cell array (HueCells::cell_of).
template <bool kThr>
__device__ __forceinline__ int classify_f(int kr, int kg, int kb, const ClsEnt& e, const signed char* si8g,
                                          const GridParams& gp, const FastCls& F, int& hN, int& hD,
                                          int& cell) {
    const int kmx = max(kr, max(kg, kb)), kmn = min(kr, min(kg, kb)), kd = kmx - kmn;
    const int si = si_of<kThr>(e, kmx, kd, si8g);
    const bool isr = kr == kmx, isg = kg == kmx;
    const int a = isr ? kg : (isg ? kb : kr), b = isr ? kb : (isg ? kr : kg);
    const int num = a - b;
    const int base = isr ? (num < 0 ? 360 : 0) : (isg ? 120 : 240);
    const int kd1 = max(kd, 1);
    const int N = __mul24(base, kd1) + 60 * num, D = __mul24(F.lh, kd1);
    hN = kd == 0 ? 0 : N;
    hD = kd1;
    const int c = (int)(((float)(2 * N) + 0.5f) * __builtin_amdgcn_rcpf((float)D));
    const int hi = c >> 1;
    const int special = (int)(num == 0) | (int)(num == kd) | (int)(num == -kd);
    const int onb = (int)(__mul24(c, D) == 2 * N);
    const int def = onb & (special ^ 1);
    const int ch = c - gp.hp;
    const int below = onb & special & (int)(ch >= 0) & ((ch & 1) | (int)(ch == 0));
    const int vi = (e.vpack << 16) >> 16, gray = e.vpack >> 16;
    const int g = __mul24(__mul24(hi, gp.sp) + si, gp.vp) + vi;
    const int mblack = -(int)(vi < 0);
    const int mgray = -(int)(si < 0) & ~mblack;
    const int mdef = -def;
    const int gg = (g & ~(mblack | mgray)) | ((gp.tl - 1) & mblack) | (gray & mgray);
    const int gs = gp.tl - gp.ng - 1;
    // colour group: 4 cells from the bin's lower edge; grey / black: 2*hp cells
    const int cc = 4 * gg + 1 + (c & 1) - below;
    const int cgray = 4 * gs + __mul24(gg - gs, 2 * gp.hp) + c - below;
    const int cl = (mblack | mgray) ? cgray : cc;
    cell = (cl & ~mdef) | ((4 * gs + (gp.ng + 1) * 2 * gp.hp) & mdef);
    return (gg & ~mdef) | (-2 & mdef);
}

// The exact group and hue cell of a pixel classify_f() deferred (-2): its
// rgb2hsv doubles, and on the boundary B_c the side calculate_avg_hsv's wrap
// test puts it (src/color_quantization.c:538-546) for the one parent whose
// threshold is B_c: up-wrap thresholds (B_c = hp_j + 180 or, for grey / black
// parents, 180) go above when h + off > 360; down-wrap thresholds
// (B_c = hp_j - 180) go below when h + off < 0.
__device__ __forceinline__ int fused_exact(int kr, int kg, int kb, const double* k255, const GridParams& gp,
                                           int lh, double& h, int& cell) {
    double s, v;
    rgb2hsv(k255[kr], k255[kg], k255[kb], h, s, v);
    const int g = group_of(gp, h, s, v);
    const int kmx = max(kr, max(kg, kb)), kd = kmx - min(kr, min(kg, kb));
    const bool isr = kr == kmx, isg = kg == kmx;
    const int num = isr ? kg - kb : (isg ? kb - kr : kr - kg);
    const int base = isr ? (num < 0 ? 360 : 0) : (isg ? 120 : 240);
    const int kd1 = max(kd, 1);
    const int c = (2 * (base * kd1 + 60 * num)) / (lh * kd1);          // on the boundary: exact
    const double B = (double)c * (double)lh * 0.5;                     // c * Lh / 2, exact
    const int ch = c - gp.hp;
    int below;
    if (ch < 0) {
        below = ((c + gp.hp) & 1) ? (int)((h + (-B)) < 0) : 0;         // off = 180 - hp_j = -B
    } else if (ch == 0) {
        below = (int)!((h + 180.0) > 360);                             // grey / black parent, off = 180
    } else if (ch & 1) {
        below = (int)!((h + (360.0 - B)) > 360);                       // off = 180 - hp_j = 360 - B
    } else {
        below = 0;
    }
    const int gs = gp.tl - gp.ng - 1;
    const int cg = c - below;
    if (g < gs) {
        const int hi = g / (gp.sp * gp.vp);
        cell = 4 * g + min(3, max(0, cg - 2 * hi + 1));
    } else {
        cell = 4 * gs + (g - gs) * 2 * gp.hp + cg;
    }
    return g;
}

template <bool kThr>
__device__ __forceinline__ int classify_e(int kr, int kg, int kb, const ClsEnt& e, const signed char* si8g,
                                          const GridParams& gp, const FastCls& F) {
    int hN, hD;
    return classify_e<kThr>(kr, kg, kb, e, si8g, gp, F, hN, hD);
}

template <bool kThr>
__device__ __forceinline__ int classify(int kr, int kg, int kb, const ClsEnt* ent, const signed char* si8g,
                                        const GridParams& gp, const FastCls& F, double& s_out) {
    const int kmx = max(kr, max(kg, kb)), kmn = min(kr, min(kg, kb));
    s_out = sat_of(kmx, kmn);
    return classify_e<kThr>(kr, kg, kb, ent[kmx], si8g, gp, F);
}

// rgb2hsv's hue, bit-exact (same doubles, same operation order), select-only:
// the branch's channel difference over d, plus 0/2/4 sectors, times 60.
__device__ __forceinline__ double hue_exact(int kr, int kg, int kb, const double* k255) {
    const double r = k255[kr], g = k255[kg], b = k255[kb];
    const int kmx = max(kr, max(kg, kb)), kmn = min(kr, min(kg, kb));
    const double d = k255[kmx] - k255[kmn];
    const bool isr = kr == kmx, isg = kg == kmx;
    const double num = isr ? g - b : (isg ? b - r : r - g);
    const double sector = isr ? 0.0 : (isg ? 2.0 : 4.0);
    // 60 * (0 + q) == 60 * q exactly; d == 0 gives NaN here and is selected away
    double h = 60 * (sector + num / d);
    h = kmx == kmn ? 0.0 : h;
    return h < 0 ? h + 360 : h;
}

// rgb2hsv's hue to within a few ulps (the quotient through inv_k): for sums.
__device__ __forceinline__ double hue_fast(int kr, int kg, int kb) {
    const int kmx = max(kr, max(kg, kb)), kmn = min(kr, min(kg, kb)), kd = kmx - kmn;
    const bool isr = kr == kmx, isg = kg == kmx;
    const int num = isr ? kg - kb : (isg ? kb - kr : kr - kg);
    const double sector = isr ? 0.0 : (isg ? 2.0 : 4.0);
    const double h = 60 * (sector + (double)num * inv_k(max(kd, 1)));
    return kd == 0 ? 0.0 : (h < 0 ? h + 360 : h);
}

// rgb2hsv's v (k/255, 0.999999 for 255) to within an ulp: for sums.
__device__ __forceinline__ double v_fast(int kmx) {
    return kmx == 255 ? 0.999999 : (double)kmx * (1.0 / 255.0);
}

// The group of a pixel that classify() left on a hue bin edge (-2: a colour
// pixel), from its exact hue: arm_octree's (int)(h / Lh).
template <bool kThr>
__device__ __forceinline__ int edge_group(int kr, int kg, int kb, double h, const ClsEnt* ent,
                                          const signed char* si8g, const GridParams& gp) {
    const int kmx = max(kr, max(kg, kb)), kd = kmx - min(kr, min(kg, kb));
    const ClsEnt e = ent[kmx];
    const int si = si_of<kThr>(e, kmx, kd, si8g);
    const int vi = (e.vpack << 16) >> 16;
    const int hi = (int)(h / gp.Lh);
    return (hi * gp.sp + si) * gp.vp + vi;
}

// v of rgb2hsv for max channel value k: k/255, 0.999999 for 255.
__device__ __forceinline__ double v_of(int kmx, const double* k255) { return kmx == 255 ? 0.999999 : k255[kmx]; }

// HSV saturation alone (rgb2hsv's s), for the statistics-only pass.
__device__ __forceinline__ double sat_only(int kr, int kg, int kb) {
    return sat_of(max(kr, max(kg, kb)), min(kr, min(kg, kb)));
}

// The reference's exact group of a pixel (rgb2hsv in fp64 + arm_octree).
__device__ __forceinline__ int exact_group(int kr, int kg, int kb, const double* k255, const GridParams& gp) {
    double h, s, v;
    rgb2hsv(k255[kr], k255[kg], k255[kb], h, s, v);
    return group_of(gp, h, s, v);
}

// Source pixel of hsv-index j (downsample_rgb's row quirk for ds > 1:
// new (y, x) <- old (y*(ds-1), x*ds), src/image_processing.c:344-366).
__device__ __forceinline__ long src_pixel(long j, int width, int ds, int nw) {
    if (ds <= 1) return j;
    const long y = j / nw, x = j - y * nw;
    return y * (long)(ds - 1) * width + x * ds;
}

__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }

template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// log of a positive finite x for the polar bins (a run's mantissa product in
// the column passes, an element's p in the runtime-plan pass), fp64 to a few ulp, table-driven (~16 instructions against ~100 for the library log):
// x = f 2^e with f in [1, 2); i = the top 5 fraction bits of f; with c_i =
// 1 + (i + 1/2) / 32, log f = log c_i + log1p(r), r = f / c_i - 1 = fma(f,
// 1 / c_i, -1) (|r| <= 2^-6), log1p by 9 terms (error < |r|^10 / 10 < 2^-63).
// The table (LDS, 32 x {1 / c_i, -log(1 / c_i)}, 512 bytes: it fits beside
// two blocks' columns of 4000) is filled per block by log_table_init; the
// stored reciprocal is what r uses and its exact log is what is added back,
// so the reciprocal's rounding cancels.
constexpr int kLogTab = 32;
__device__ __forceinline__ void log_table_init(double2* lt, int tid, int nt) {
    for (int i = tid; i < kLogTab; i += nt) {
        const double inv = 1.0 / (1.0 + (i + 0.5) / kLogTab);
        lt[i] = make_double2(inv, -log(inv));
    }
}
__device__ __forceinline__ double log_mant(double m, const double2* __restrict__ lt) {
    int e;
    const double f = 2.0 * frexp(m, &e);                 // f in [1, 2), x = f 2^(e - 1)
    const int i = (int)((__double_as_longlong(f) >> 47) & (kLogTab - 1));
    const double2 t = lt[i];
    const double r = fma(f, t.x, -1.0);
    // log1p(r) = sum_{k=1..9} (-1)^(k+1) r^k / k (Horner in r)
    double q = 1.0 / 9.0;
    q = fma(q, r, -1.0 / 8.0);
    q = fma(q, r, 1.0 / 7.0);
    q = fma(q, r, -1.0 / 6.0);
    q = fma(q, r, 1.0 / 5.0);
    q = fma(q, r, -1.0 / 4.0);
    q = fma(q, r, 1.0 / 3.0);
    q = fma(q, r, -0.5);
    q = fma(q, r, 1.0);
    return fma(q, r, t.y) + (double)(e - 1) * 0.69314718055994530942;
}

// a non-negative sum of log(p) as bin_scale fixed point (round to nearest)
__device__ __forceinline__ unsigned long long bin_fixed(double x, double scale) { return __double2ull_rn(x * scale); }

__device__ __forceinline__ double wave_max(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o, 64));
    return v;
}

}  // namespace phd
