// phd_device.h -- device helpers shared by the HIP kernels.
//
// Every fp64 expression keeps the reference's operation order; the library is
// compiled with -ffp-contract=off so no multiply-add is fused, and HIP's fp64
// '/' is the IEEE correctly-rounded division, so results are bit-identical to
// the reference's x86-64 SSE2 code.
#pragma once

#include <hip/hip_runtime.h>

#include <algorithm>

#include "phd_internal.h"

namespace phd {

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

// Group id from integer facts and an fp32 estimate, or -2 when the pixel's
// hue or saturation quotient lies within the guard band of a bin edge and must
// take the exact path (rgb2hsv + group_of).  Away from the band the fp32 and
// the reference's fp64 quotients truncate to the same integer: the fp32 error
// is < 1e-4 of a bin while a non-integral hue quotient (base + 60 n/kd)/Lh with
// Lh | 360 sits >= 1/(6 kd) >= 6.5e-4 from an integer.  Exact special cases:
// v-classes come from a table over kmax; s == 0 (kd == 0) and s == 0.999999
// (kmin == 0); hue quotients 0 and +-1 (num == 0, +-kd) are exact in fp64.
__device__ __forceinline__ int fast_group(int kr, int kg, int kb, const short* vcol,
                                          const short* vgray, const GridParams& gp, const FastCls& F) {
    const int kmx = max(kr, max(kg, kb)), kmn = min(kr, min(kg, kb)), kd = kmx - kmn;
    const int vi = vcol[kmx];
    if (vi < 0) return gp.tl - 1;                       // v < black_thresh
    int si;
    if (kd == 0) si = F.si_zero;                        // s == 0 (also kmax == 0)
    else if (kmn == 0) si = F.si_full;                  // d == max: s = 0.999999
    else {
        const float sf = (float)kd * __builtin_amdgcn_rcpf((float)kmx);
        const float q = (sf - F.gt) * F.inv_ls;
        if (fabsf(q - rintf(q)) < F.guard_s) return -2;
        si = q < 0.f ? -1 : (int)q;
    }
    if (si < 0) return F.gray_base + vgray[kmx];        // s < gray_thresh
    int hi;
    if (kd == 0) {
        hi = 0;                                         // h = 0
    } else {
        int num, c;
        if (kr == kmx) { num = kg - kb; c = 0; }
        else if (kg == kmx) { num = kb - kr; c = 1; }
        else { num = kr - kg; c = 2; }
        if (num == 0) hi = F.hx[3 * c];
        else if (num == kd) hi = F.hx[3 * c + 1];
        else if (num == -kd) hi = F.hx[3 * c + 2];
        else {
            float h = (float)(120 * c) + (60.f * (float)num) * __builtin_amdgcn_rcpf((float)kd);
            if (h < 0.f) h += 360.f;
            const float q = h * F.inv_lh;
            if (fabsf(q - rintf(q)) < F.guard_h) return -2;
            hi = (int)q;
        }
    }
    return (hi * gp.sp + si) * gp.vp + vi;
}

// The reference's exact group of a pixel (rgb2hsv in fp64 + arm_octree).
__device__ __forceinline__ int exact_group(int kr, int kg, int kb, const double* k255, const GridParams& gp) {
    double h, s, v;
    rgb2hsv(k255[kr], k255[kg], k255[kb], h, s, v);
    return group_of(gp, h, s, v);
}

// Saturation for the S-bar sum: kd * (1/kmax) from a table, within a few ulp
// of the reference's (max - min) / max (get_hsv_average's contract is 1e-4
// relative; the sum over an image agrees to ~1e-15).
__device__ __forceinline__ double sat_of(int kr, int kg, int kb, const double* rinv) {
    const int kmx = max(kr, max(kg, kb)), kmn = min(kr, min(kg, kb));
    if (kmx == kmn) return 0.0;
    if (kmn == 0) return 0.999999;
    return (double)(kmx - kmn) * rinv[kmx];
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

__device__ __forceinline__ double wave_max(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o, 64));
    return v;
}

}  // namespace phd
