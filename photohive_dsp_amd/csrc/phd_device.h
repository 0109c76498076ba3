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
