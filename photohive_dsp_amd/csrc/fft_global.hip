// fft_global.hip -- batched 1-D complex fp64 FFTs over sequences in HBM, and
// the generic 2-D power-spectrum path built from them.
//
// The fused passes of fft.hip / fft_ct.hip keep a whole row or column in LDS
// (at most 8192 complex fp64 = 128 KiB).  pgm_fft (src/fft_processing.c:18-63)
// accepts any image pre_compute_error_checks lets through
// (src/utilities.c:64-87: up to 120 MP, aspect 1:5..5:1, so a side can reach
// 24494 px), and FFTW handles any length.  This file covers the rest:
//
//  * direct:     n <= 8192 with small prime factors: G sequences per block,
//                one LDS transform (fft_runtime.h), in place.
//  * four-step:  n = n1 * n2 (both direct lengths): n1-point transforms over
//                stride-n2 gathers, times W_n^(j2 k1), into a scratch
//                [n1][n2]; then n2-point transforms of its contiguous rows,
//                written to X[k1 + n1 k2].  Two HBM round trips.
//  * Bluestein:  n with a large prime factor (a prime side such as 7919 or
//                10007): X_k = c_k sum_j (x_j c_j) conj(c_(k-j)), c_j =
//                exp(-pi i j^2 / n), as a cyclic convolution of a smooth
//                length M >= 2n - 1 through two length-M transforms.
//
// The generic 2-D path (one image): the row pairs of the luma minus the DC
// bias as complex rows [H/2][W] (k_pairs), their length-W transforms, the two
// real rows' half spectra separated and transposed to the column-major
// [W/2+1][H] layout of fft.hip (k_split_t), the length-H column transforms,
// then the power, its maximum and the polar log-binning (k_power_bins) --
// pgm_normalize_fft (src/fft_processing.c:173-213) and the binning loop of
// calculate_blur_profile (src/blur_profile.c:87-100).
#include "fft_runtime.h"

namespace phd {

using namespace rt;

namespace {

__device__ __forceinline__ double2 cconj(double2 a) { return make_double2(a.x, -a.y); }

// G sequences of length n per block, in place (in == out allowed).
// LDS: [ G*n complex | twiddles (64 + n_hi) ]
template <int T, bool GEN>
__global__ __launch_bounds__(T) void k_gfft_direct(const double2* in, double2* out, long count, int G,
                                                   FftPlan plan) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    double2* buf = reinterpret_cast<double2*>(smem);
    const int n = plan.n;
    double2* tw = buf + (size_t)G * n;
    const int tid = threadIdx.x;
    const long s0 = (long)blockIdx.x * G;
    const int ns = (int)min((long)G, count - s0);
    load_twiddles(tw, plan);
    const double2* src = in + s0 * n;
    for (int i = tid; i < ns * n; i += T) buf[i] = src[i];
    __syncthreads();
    fft_lds<T, GEN ? 2 : 0>(buf, ns, plan, tw, tw + 64);
    double2* dst = out + s0 * n;
    for (int i = tid; i < ns * n; i += T) dst[i] = buf[i];
}

// Four-step, step A: sequence blockIdx.y, columns j2 in [j20, j20 + G):
// y[k1][j2] = W_n^(j2 k1) * sum_j1 x[j1 n2 + j2] W_n1^(j1 k1).
// LDS: [ G*n1 complex | twiddles of the n1 plan ]
template <int T, bool GEN>
__global__ __launch_bounds__(T) void k_gfft_4a(const double2* __restrict__ in, double2* __restrict__ scr, int n,
                                               int n2, int G, FftPlan p1, const double2* __restrict__ twn) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    double2* buf = reinterpret_cast<double2*>(smem);
    const int n1 = p1.n;
    double2* tw = buf + (size_t)G * n1;
    const int tid = threadIdx.x;
    const long s = blockIdx.y;
    const int j20 = blockIdx.x * G;
    const int g = min(G, n2 - j20);
    load_twiddles(tw, p1);
    const double2* x = in + s * n;
    // consecutive threads read consecutive j2 of one j1 (a contiguous run of g)
    for (int i = tid; i < G * n1; i += T) {
        const int j1 = i / G, jj = i - j1 * G;
        buf[jj * n1 + j1] = jj < g ? x[(long)j1 * n2 + j20 + jj] : make_double2(0.0, 0.0);
    }
    __syncthreads();
    fft_lds<T, GEN ? 2 : 0>(buf, G, p1, tw, tw + 64);
    double2* y = scr + s * n;
    for (int i = tid; i < G * n1; i += T) {
        const int k1 = i / G, jj = i - k1 * G;
        if (jj < g) y[(long)k1 * n2 + j20 + jj] = cmul(buf[jj * n1 + k1], twn[(j20 + jj) * k1]);
    }
}

// Four-step, step B: sequence blockIdx.y, rows k1 in [k10, k10 + G) of the
// scratch: X[k1 + n1 k2] = sum_j2 y[k1][j2] W_n2^(j2 k2).
template <int T, bool GEN>
__global__ __launch_bounds__(T) void k_gfft_4b(const double2* __restrict__ scr, double2* __restrict__ out, int n,
                                               int n1, int G, FftPlan p2) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    double2* buf = reinterpret_cast<double2*>(smem);
    const int n2 = p2.n;
    double2* tw = buf + (size_t)G * n2;
    const int tid = threadIdx.x;
    const long s = blockIdx.y;
    const int k10 = blockIdx.x * G;
    const int g = min(G, n1 - k10);
    load_twiddles(tw, p2);
    const double2* src = scr + s * n + (long)k10 * n2;
    for (int i = tid; i < G * n2; i += T) buf[i] = i < g * n2 ? src[i] : make_double2(0.0, 0.0);
    __syncthreads();
    fft_lds<T, GEN ? 2 : 0>(buf, G, p2, tw, tw + 64);
    double2* X = out + s * n;
    for (int i = tid; i < G * n2; i += T) {
        const int k2 = i / G, kk = i - k2 * G;
        if (kk < g) X[k10 + kk + (long)n1 * k2] = buf[kk * n2 + k2];
    }
}

// Bluestein: a[s][j] = x[s][j] c_j (j < n), 0 up to M.
__global__ __launch_bounds__(256) void k_blu_pre(const double2* __restrict__ x, double2* __restrict__ a, int n, int M,
                                                 long count, const double2* __restrict__ chirp) {
    const long total = count * M;
    for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
        const long s = i / M;
        const int j = (int)(i - s * M);
        a[i] = j < n ? cmul(x[s * n + j], chirp[j]) : make_double2(0.0, 0.0);
    }
}

// Bluestein: a = conj(FFT(a) * FFT(b)) (the inverse transform as a forward one)
__global__ __launch_bounds__(256) void k_blu_mid(double2* __restrict__ a, long total, int M,
                                                 const double2* __restrict__ bhat) {
    for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < total; i += (long)gridDim.x * 256)
        a[i] = cconj(cmul(a[i], bhat[i % M]));
}

// Bluestein: X[s][k] = c_k conj(z[s][k]) / M
__global__ __launch_bounds__(256) void k_blu_post(const double2* __restrict__ z, double2* __restrict__ out, int n,
                                                  int M, long count, const double2* __restrict__ chirp, double invM) {
    const long total = count * n;
    for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
        const long s = i / n;
        const int k = (int)(i - s * n);
        const double2 v = cmul(chirp[k], cconj(z[s * M + k]));
        out[i] = make_double2(v.x * invM, v.y * invM);
    }
}

// rgb2pgm (src/image_processing.c:505-512) of pixel i from RGB8 or an fp64
// luma plane (already rgb2pgm of the caller's doubles).
__device__ __forceinline__ double luma_at(const uint8_t* __restrict__ img, const double* __restrict__ pgm, long i,
                                          const double* k255) {
    if (pgm) return pgm[i];
    return 0.299 * k255[img[3 * i]] + 0.587 * k255[img[3 * i + 1]] + 0.114 * k255[img[3 * i + 2]];
}

// Row pairs of pgm - avg (remove_dc_bias, src/blur_profile.c:233-238) as
// complex rows: Z[p][x] = (pgm(2p, x) - avg) + i (pgm(2p+1, x) - avg).
// avg = (Br + Bg + Bb) / 3 (src/interface.c:78): from the exact RGB8 channel
// sums (sums), or given (avgd, the fp64 planar path).
__global__ __launch_bounds__(256) void k_pairs(const uint8_t* __restrict__ img, const double* __restrict__ pgm,
                                               int H, int W, const double* __restrict__ k255g,
                                               const unsigned long long* __restrict__ sums,
                                               const double* __restrict__ avgd, double2* __restrict__ Z) {
    __shared__ double k255[256];
    k255[threadIdx.x] = k255g[threadIdx.x];
    __syncthreads();
    double avg;
    if (avgd) {
        avg = *avgd;
    } else {
        const double n = (double)H * (double)W;
        avg = ((double)sums[0] / 255.0 / n + (double)sums[1] / 255.0 / n + (double)sums[2] / 255.0 / n) / 3.0;
    }
    const long p = blockIdx.y;
    const int x = blockIdx.x * 256 + threadIdx.x;
    if (x >= W) return;
    const long y0 = 2 * p, y1 = y0 + 1;
    const double v0 = luma_at(img, pgm, y0 * W + x, k255) - avg;
    const double v1 = y1 < H ? luma_at(img, pgm, y1 * W + x, k255) - avg : 0.0;
    Z[p * W + x] = make_double2(v0, v1);
}

// Separate the two real rows' spectra of each row pair and transpose them to
// the column-major half spectrum inter[k][y] (k < W/2+1): A[k] = (Z[k] +
// conj Z[W-k]) / 2 (row 2p), B[k] = (Z[k] - conj Z[W-k]) / (2i) (row 2p+1).
// Tiles of kTp row pairs x kTk columns through LDS: reads and writes are
// contiguous runs.
constexpr int kTp = 16, kTk = 32;
__global__ __launch_bounds__(256) void k_split_t(const double2* __restrict__ Z, int H, int W,
                                                 double2* __restrict__ inter) {
    __shared__ double2 za[kTp][kTk + 1], zb[kTp][kTk + 1];
    const int wf = W / 2 + 1, hp = (H + 1) / 2;
    const int k0 = blockIdx.x * kTk, p0 = blockIdx.y * kTp;
    for (int i = threadIdx.x; i < kTp * kTk; i += 256) {
        const int pp = i / kTk, kk = i - pp * kTk;
        const int p = p0 + pp, k = k0 + kk;
        if (p < hp && k < wf) {
            za[pp][kk] = Z[(long)p * W + k];
            zb[pp][kk] = Z[(long)p * W + (k == 0 ? 0 : W - k)];
        }
    }
    __syncthreads();
    for (int i = threadIdx.x; i < kTk * 2 * kTp; i += 256) {
        const int kk = i / (2 * kTp), q = i - kk * (2 * kTp);
        const int pp = q >> 1, second = q & 1;
        const int k = k0 + kk, y = 2 * (p0 + pp) + second;
        if (k < wf && p0 + pp < hp && y < H) {
            const double2 zk = za[pp][kk], zm = zb[pp][kk];
            inter[(long)k * H + y] = second ? make_double2(0.5 * (zk.y + zm.y), -0.5 * (zk.x - zm.x))
                                            : make_double2(0.5 * (zk.x + zm.x), 0.5 * (zk.y - zm.y));
        }
    }
}

// p = re^2 + im^2 (src/fft_processing.c:48-50) of every element of the
// column-major half spectrum, its maximum (one partial per block) and, for
// p >= 1 (src/fft_processing.c:197-198), log(p) into the element's polar bin
// as bin_scale fixed point (order-independent integer sums).
template <bool kLdsBins>
__global__ __launch_bounds__(256) void k_power_bins(const double2* __restrict__ X, long total,
                                                    const uint16_t* __restrict__ binmap, int nbins,
                                                    unsigned long long* __restrict__ bin_sums,
                                                    double* __restrict__ fmax_part, double bscale) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    unsigned long long* lb = reinterpret_cast<unsigned long long*>(smem);
    __shared__ double red[4];
    const int tid = threadIdx.x;
    if (kLdsBins)
        for (int i = tid; i < nbins; i += 256) lb[i] = 0ull;
    __syncthreads();
    unsigned long long* acc = kLdsBins ? lb : bin_sums;
    double mx = 0.0;
    const long stride = (long)gridDim.x * 256;
    for (long i0 = (long)blockIdx.x * 256; i0 < total; i0 += stride) {
        const long i = i0 + tid;
        int b = -1;
        unsigned long long lg = 0ull;
        if (i < total) {
            const double2 v = X[i];
            const double p = v.x * v.x + v.y * v.y;
            mx = fmax(mx, p);
            if (p >= 1) {
                b = binmap[i];
                lg = bin_fixed(log(p), bscale);
            }
        }
        const int b0 = __builtin_amdgcn_readfirstlane(b);
        if (__all(b == b0)) {
            const unsigned long long t = wave_sum(lg);
            if (b0 >= 0 && lane_id() == 0) atomicAdd(&acc[b0], t);
        } else if (b >= 0) {
            atomicAdd(&acc[b], lg);
        }
    }
    mx = wave_max(mx);
    if (lane_id() == 0) red[tid >> 6] = mx;
    __syncthreads();
    if (tid == 0) fmax_part[blockIdx.x] = fmax(fmax(red[0], red[1]), fmax(red[2], red[3]));
    if (kLdsBins) {
        for (int i = tid; i < nbins; i += 256) {
            const unsigned long long a = lb[i];
            if (a != 0ull) atomicAdd(&bin_sums[i], a);
        }
    }
}

template <typename K>
void allow_big_lds(K kernel) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kernel), hipFuncAttributeMaxDynamicSharedMemorySize,
                              160 * 1024);
}

size_t plan_lds(const FftPlan& p, int G) { return sizeof(double2) * ((size_t)G * p.n + 64 + p.n_hi); }

// launch kernel K<T, GEN> with T chosen by the elements per block
#define PHD_GFFT_DISPATCH(KERN, elems, gen, grid, lds, st, ...)                                   \
    do {                                                                                          \
        if ((elems) <= 2048) {                                                                    \
            if (gen) { static bool o = (allow_big_lds(KERN<256, true>), true); (void)o;           \
                       phd_launch((KERN<256, true>), grid, dim3(256), lds, st, __VA_ARGS__); }    \
            else { static bool o = (allow_big_lds(KERN<256, false>), true); (void)o;              \
                   phd_launch((KERN<256, false>), grid, dim3(256), lds, st, __VA_ARGS__); }       \
        } else if ((elems) <= 4096) {                                                             \
            if (gen) { static bool o = (allow_big_lds(KERN<512, true>), true); (void)o;           \
                       phd_launch((KERN<512, true>), grid, dim3(512), lds, st, __VA_ARGS__); }    \
            else { static bool o = (allow_big_lds(KERN<512, false>), true); (void)o;              \
                   phd_launch((KERN<512, false>), grid, dim3(512), lds, st, __VA_ARGS__); }       \
        } else {                                                                                  \
            if (gen) { static bool o = (allow_big_lds(KERN<1024, true>), true); (void)o;          \
                       phd_launch((KERN<1024, true>), grid, dim3(1024), lds, st, __VA_ARGS__); }  \
            else { static bool o = (allow_big_lds(KERN<1024, false>), true); (void)o;             \
                   phd_launch((KERN<1024, false>), grid, dim3(1024), lds, st, __VA_ARGS__); }     \
        }                                                                                         \
    } while (0)

// sequences per block for length n (G * n <= 8192 elements: 8 per thread at 1024 threads)
int seqs_per_block(int n, int cap) { return std::max(1, std::min(cap, kFftMaxLds / n)); }

}  // namespace

hipError_t launch_gfft_direct(const double2* in, double2* out, long count, const FftPlan& plan, hipStream_t st) {
    const int G = seqs_per_block(plan.n, 64);
    const long blocks = (count + G - 1) / G;
    const size_t lds = plan_lds(plan, G);
    const int elems = G * plan.n;
    PHD_GFFT_DISPATCH(k_gfft_direct, elems, plan.generic, dim3((unsigned)blocks), lds, st, in, out, count, G, plan);
    return hipGetLastError();
}

hipError_t launch_gfft_4step(const double2* in, double2* out, double2* scr, long count, int n, const FftPlan& p1,
                             const FftPlan& p2, const double2* twn, hipStream_t st) {
    const int n1 = p1.n, n2 = p2.n;
    const int Ga = seqs_per_block(n1, 64), Gb = seqs_per_block(n2, 64);
    // grid.y is the sequence: at most 65535 per launch
    for (long s0 = 0; s0 < count; s0 += 65535) {
        const unsigned cs = (unsigned)std::min<long>(65535, count - s0);
        PHD_GFFT_DISPATCH(k_gfft_4a, Ga * n1, p1.generic, dim3((unsigned)((n2 + Ga - 1) / Ga), cs), plan_lds(p1, Ga),
                          st, in + s0 * n, scr + s0 * n, n, n2, Ga, p1, twn);
        PHD_GFFT_DISPATCH(k_gfft_4b, Gb * n2, p2.generic, dim3((unsigned)((n1 + Gb - 1) / Gb), cs), plan_lds(p2, Gb),
                          st, scr + s0 * n, out + s0 * n, n, n1, Gb, p2);
    }
    return hipGetLastError();
}

static unsigned ew_blocks(long total) { return (unsigned)std::max<long>(1, std::min<long>(8192, (total + 255) / 256)); }

hipError_t launch_blu_pre(const double2* x, double2* a, int n, int M, long count, const double2* chirp,
                          hipStream_t st) {
    phd_launch(k_blu_pre, dim3(ew_blocks(count * M)), dim3(256), 0, st, x, a, n, M, count, chirp);
    return hipGetLastError();
}

hipError_t launch_blu_mid(double2* a, long count, int M, const double2* bhat, hipStream_t st) {
    phd_launch(k_blu_mid, dim3(ew_blocks(count * M)), dim3(256), 0, st, a, count * M, M, bhat);
    return hipGetLastError();
}

hipError_t launch_blu_post(const double2* z, double2* out, int n, int M, long count, const double2* chirp,
                           hipStream_t st) {
    phd_launch(k_blu_post, dim3(ew_blocks(count * n)), dim3(256), 0, st, z, out, n, M, count, chirp, 1.0 / (double)M);
    return hipGetLastError();
}

hipError_t launch_pairs(const uint8_t* img, const double* pgm, int height, int width, const double* k255,
                        const unsigned long long* sums, const double* avgd, double2* Z, hipStream_t st) {
    const int hp = (height + 1) / 2;
    phd_launch(k_pairs, dim3((unsigned)((width + 255) / 256), (unsigned)hp), dim3(256), 0, st, img, pgm, height, width,
               k255, sums, avgd, Z);
    return hipGetLastError();
}

hipError_t launch_split_t(const double2* Z, int height, int width, double2* inter, hipStream_t st) {
    const int wf = width / 2 + 1, hp = (height + 1) / 2;
    phd_launch(k_split_t, dim3((unsigned)((wf + kTk - 1) / kTk), (unsigned)((hp + kTp - 1) / kTp)), dim3(256), 0, st,
               Z, height, width, inter);
    return hipGetLastError();
}

hipError_t launch_power_bins(const double2* X, int height, int wf, const uint16_t* binmap, int nbins,
                             unsigned long long* bin_sums, double* fmax_part, hipStream_t st, double bscale) {
    const long total = (long)height * wf;
    if (bscale <= 0.0) bscale = bin_scale(height, wf);
    const size_t lds = sizeof(unsigned long long) * nbins;
    if (lds <= 48 * 1024) {
        phd_launch(k_power_bins<true>, dim3(kPowerBinBlocks), dim3(256), lds, st, X, total, binmap, nbins, bin_sums,
                   fmax_part, bscale);
    } else {
        phd_launch(k_power_bins<false>, dim3(kPowerBinBlocks), dim3(256), 0, st, X, total, binmap, nbins, bin_sums,
                   fmax_part, bscale);
    }
    return hipGetLastError();
}

}  // namespace phd
