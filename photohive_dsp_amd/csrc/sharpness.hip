// sharpness.hip -- Laplacian-variance sharpness of crop boxes.
//
// Replaces get_variance_sharpness (src/filtering.c:151-183): crop_pgm
// (src/image_processing.c:213-232) of the full-resolution luma, 3x3 Laplacian
// with zero padding at the CROP border (filter_image, filtering.c:81-107),
// then var(filtered) / mean(filtered) with the reference's two passes.
// The luma is recomputed from the RGB8 bytes; the filtered crop is never
// stored: pass 1 sums f, pass 2 sums (f - mean)^2.
#include "phd_device.h"

namespace phd {

namespace {

// the luma of pixel i: rgb2pgm of the RGB8 bytes, or the fp64 plane (planar input)
__device__ __forceinline__ double luma(const uint8_t* __restrict__ img, const double* __restrict__ pgm, long i,
                                       const double* k255) {
    if (pgm) return pgm[i];
    return 0.299 * k255[img[3 * i]] + 0.587 * k255[img[3 * i + 1]] + 0.114 * k255[img[3 * i + 2]];
}

// f(y,x) of filter_image: sum over the 3x3 window in (fy, fx) order of
// input * coef, skipping taps outside the crop.
__device__ __forceinline__ double lap_at(const uint8_t* __restrict__ img, const double* __restrict__ pgm, int width,
                                         int top, int left, int ch, int cw, int y, int x, const double* k255) {
    double dp = 0.0;
#pragma unroll
    for (int fy = 0; fy < 3; fy++)
#pragma unroll
        for (int fx = 0; fx < 3; fx++) {
            const int iy = y + fy - 1, ix = x + fx - 1;
            if (iy >= 0 && iy < ch && ix >= 0 && ix < cw) {
                const double coef = (fy == 1 && fx == 1) ? 8.0 : -1.0;
                dp += luma(img, pgm, (long)(iy + top) * width + ix + left, k255) * coef;
            }
        }
    return dp;
}

__global__ __launch_bounds__(kThreads) void k_sharp_pass(const uint8_t* __restrict__ img,
                                                         const double* __restrict__ pgm, int width, int top,
                                                         int left, int ch, int cw,
                                                         const double* __restrict__ k255g,
                                                         const double* __restrict__ mean_src, long n_mean,
                                                         double* __restrict__ out) {
    __shared__ double k255[256];
    __shared__ double red[kThreads / 64];
    k255[threadIdx.x] = k255g[threadIdx.x];
    __syncthreads();
    const long n = (long)ch * cw;
    const double mean = mean_src ? *mean_src / (double)n_mean : 0.0;
    double acc = 0.0;
    for (long i = (long)blockIdx.x * kThreads + threadIdx.x; i < n; i += (long)gridDim.x * kThreads) {
        const int y = (int)(i / cw), x = (int)(i - (long)y * cw);
        const double f = lap_at(img, pgm, width, top, left, ch, cw, y, x, k255);
        if (mean_src) {
            const double d = f - mean;
            acc += d * d;
        } else {
            acc += f;
        }
    }
    acc = wave_sum(acc);
    if (lane_id() == 0) red[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0) {
        double t = 0.0;
        for (int q = 0; q < kThreads / 64; q++) t += red[q];
        atomicAdd(out, t);
    }
}

}  // namespace

// sums[2*k] = sum f, sums[2*k+1] = sum (f - mean)^2 for crop k.  `sums` zeroed by the caller.
hipError_t launch_sharpness(const uint8_t* img, int height, int width, int n, const int* top,
                            const int* bottom, const int* left, const int* right, const double* k255,
                            double* sums, hipStream_t st) {
    return launch_sharpness_src(img, nullptr, height, width, n, top, bottom, left, right, k255, sums, st);
}

hipError_t launch_sharpness_src(const uint8_t* img, const double* pgm, int height, int width, int n, const int* top,
                                const int* bottom, const int* left, const int* right, const double* k255,
                                double* sums, hipStream_t st) {
    (void)height;
    for (int k = 0; k < n; k++) {
        const int cw = right[k] - left[k], ch = bottom[k] - top[k];
        const long cn = (long)cw * ch;
        const int blocks = (int)std::min<long>(1024, (cn + kThreads - 1) / kThreads);
        phd_launch(k_sharp_pass, dim3(blocks), dim3(kThreads), 0, st, img, pgm, width, top[k], left[k],
                           ch, cw, k255, (const double*)nullptr, 0L, sums + 2 * k);
        phd_launch(k_sharp_pass, dim3(blocks), dim3(kThreads), 0, st, img, pgm, width, top[k], left[k],
                           ch, cw, k255, (const double*)(sums + 2 * k), cn, sums + 2 * k + 1);
    }
    return hipGetLastError();
}

}  // namespace phd
