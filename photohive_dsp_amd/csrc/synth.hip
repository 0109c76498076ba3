// synth.hip -- the bench's structured synthetic images generated on the
// device, byte for byte the images of photohive_dsp_amd/synth.py:structured
// (gradient background + 8 coloured disks + noise, optionally a centred box
// blur), so a bench batch of SURVEY.md 8(d) row 2(b) images needs no host
// generation or upload.  Every double expression is evaluated in numpy's
// order without contraction, so the result is exact, not approximate
// (tests/test_gpu_round4.py compares it with synth.py).
#include <hip/hip_runtime.h>

#include <algorithm>

#include "phd_device.h"

#pragma clang fp contract(off)

namespace phd {

namespace {

__host__ __device__ inline unsigned long long sm64_word(unsigned long long seed, unsigned long long i) {
    // synth.py:splitmix64: word i = mix(seed + (i + 1) * golden)
    unsigned long long z = seed + (i + 1) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__host__ __device__ inline double sm64_unit(unsigned long long seed, unsigned long long i) {
    return (double)(sm64_word(seed, i) >> 11) * (1.0 / 9007199254740992.0);   // synth.py:_unit
}

struct Disks {
    double blue;          // 255 (0.5 + 0.4 u0)
    double cy[8], cx[8], r2[8];
    double col[8][3];
};

// synth.py:structured before the blur: the clipped, rounded value of channel
// c at (y, x)
__device__ inline void base_px(int y, int x, int h, int w, unsigned long long seed, const Disks& D, double v[3]) {
    const double yy = (double)y, xx = (double)x;
    v[0] = 255.0 * (0.2 + 0.6 * xx / (double)(w - 1 > 1 ? w - 1 : 1));
    v[1] = 255.0 * (0.3 + 0.5 * yy / (double)(h - 1 > 1 ? h - 1 : 1));
    v[2] = D.blue;
#pragma unroll
    for (int d = 0; d < 8; d++) {
        const double dy = yy - D.cy[d], dx = xx - D.cx[d];
        if (dy * dy + dx * dx < D.r2[d]) {
            v[0] = D.col[d][0];
            v[1] = D.col[d][1];
            v[2] = D.col[d][2];
        }
    }
    const unsigned long long i0 = 3ull * ((unsigned long long)y * w + x);
#pragma unroll
    for (int c = 0; c < 3; c++) {
        const double noise = (sm64_unit(seed + 1, i0 + c) - 0.5) * 24.0;
        v[c] = fmin(fmax(rint(v[c] + noise), 0.0), 255.0);
    }
}

// blur <= 1: the base image; else the centred `blur`-tap box blur (edge
// clamped) along axis 1 (rows) or 0 (columns), rint(sum / blur) (synth.py:box_blur)
__global__ __launch_bounds__(256) void k_fill_structured(uint8_t* __restrict__ dst, int h, int w,
                                                         unsigned long long seed, Disks D, int blur, int axis) {
    const long n = (long)h * w;
    for (long p = (long)blockIdx.x * 256 + threadIdx.x; p < n; p += (long)gridDim.x * 256) {
        const int y = (int)(p / w), x = (int)(p - (long)y * w);
        double out[3];
        if (blur <= 1) {
            base_px(y, x, h, w, seed, D, out);
        } else {
            double s[3] = {0.0, 0.0, 0.0};
            const int lo = blur / 2;
            for (int t = -lo; t < blur - lo; t++) {
                double v[3];
                if (axis == 0) base_px(min(max(y + t, 0), h - 1), x, h, w, seed, D, v);
                else base_px(y, min(max(x + t, 0), w - 1), h, w, seed, D, v);
                s[0] += v[0];
                s[1] += v[1];
                s[2] += v[2];
            }
            for (int c = 0; c < 3; c++) out[c] = fmin(fmax(rint(s[c] / (double)blur), 0.0), 255.0);
        }
        dst[3 * p] = (uint8_t)out[0];
        dst[3 * p + 1] = (uint8_t)out[1];
        dst[3 * p + 2] = (uint8_t)out[2];
    }
}

}  // namespace

hipError_t launch_fill_structured(uint8_t* dst, int h, int w, uint64_t seed, int blur, int axis, hipStream_t st) {
    if (h < 1 || w < 1) return hipErrorInvalidValue;
    Disks D;
    double u[64];
    for (int i = 0; i < 64; i++) u[i] = sm64_unit(seed, (unsigned long long)i);
    D.blue = 255.0 * (0.5 + 0.4 * u[0]);
    for (int d = 0; d < 8; d++) {
        D.cy[d] = u[1 + d] * h;
        D.cx[d] = u[9 + d] * w;
        const double rad = (0.05 + 0.2 * u[17 + d]) * (double)std::min(h, w);
        D.r2[d] = rad * rad;
        for (int c = 0; c < 3; c++) D.col[d][c] = 255.0 * u[25 + 8 * c + d];
    }
    const long n = (long)h * w;
    const int blocks = (int)std::min<long>((n + 255) / 256, 8L * num_cus());
    phd_launch(k_fill_structured, dim3(blocks), dim3(256), 0, st, dst, h, w, (unsigned long long)seed, D, blur, axis);
    return hipGetLastError();
}

}  // namespace phd
