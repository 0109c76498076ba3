// fft.hip -- 2-D real FFT power spectrum fused with the polar blur binning.
//
// Replaces pgm_fft + pgm_normalize_fft (src/fft_processing.c:18-63, 173-213; the
// DFT itself is FFTW3 r2c, unnormalised, e^{-i}), rgb2pgm + remove_dc_bias
// (src/image_processing.c:505-512, src/blur_profile.c:233-238) and the binning
// loop of calculate_blur_profile (src/blur_profile.c:87-100).
//
//  * Row pass: one block per PAIR of image rows.  Luma - avg of row y0 (real)
//    and row y0+1 (imaginary) is built straight from the RGB8 bytes, one
//    complex FFT of length W runs in LDS, and the two half spectra
//    (W/2+1 bins each) are separated and written COLUMN-major to `inter`
//    ([W/2+1][H]): a column pass that gathers 16-32 B per row from a row-major
//    spectrum ran at ~0.5 TB/s (ablation), a contiguous one streams.
//  * Column pass: one block per C adjacent spectrum columns; C length-H FFTs
//    in LDS, then the epilogue forms p = re*re + im*im, keeps a running max and
//    accumulates log(p) for p >= 1 into the element's polar bin (LDS), so the
//    normalised spectrum is never written: G_s = 1/(2 log(sqrt(max)+1)) is a
//    common factor applied on the host ( sum(log p * G_s) = G_s * sum(log p) ).
//
// FFT engine: in-place Stockham autosort in LDS, every pass = all threads read
// their butterflies' inputs into registers, barrier, write.  Twiddles come
// from a host-built table tw[t] = exp(-2 pi i t/n) (long-double accurate).
#include <cstdlib>

#include "fft_runtime.h"

namespace phd {

using namespace rt;

namespace {

// LDS: [ W complex | twiddles (64 + n_hi) | k255 (256 doubles) ]
template <int T, int MODE>
__global__ __launch_bounds__(T) void k_fft_rows(const uint8_t* __restrict__ img0,
                                                const uint8_t* const* __restrict__ imgs, int H, int W, FftPlan plan,
                                                const unsigned long long* __restrict__ sums0, long sums_stride,
                                                const double* __restrict__ k255g, double2* __restrict__ inter0,
                                                size_t inter_stride) {
    // blockIdx.y: the image of a batch (imgs[y], sums0 + y * sums_stride u64,
    // inter0 + y * inter_stride elements); imgs == nullptr: img0 alone
    const uint8_t* img = imgs ? imgs[blockIdx.y] : img0;
    const unsigned long long* sums = sums0 + (size_t)blockIdx.y * sums_stride;
    double2* inter = inter0 + (size_t)blockIdx.y * inter_stride;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    double2* buf = reinterpret_cast<double2*>(smem);
    double2* tw = buf + W;
    double* k255 = reinterpret_cast<double*>(tw + 64 + plan.n_hi);
    const int tid = threadIdx.x;
    for (int i = tid; i < 256; i += T) k255[i] = k255g[i];
    load_twiddles(tw, plan);
    // avg = (Br + Bg + Bb) / 3 (src/interface.c:78) from the exact integer sums
    const double n = (double)H * (double)W;
    const double avg = ((double)sums[0] / 255.0 / n + (double)sums[1] / 255.0 / n +
                        (double)sums[2] / 255.0 / n) / 3.0;
    __syncthreads();
    // XCD-aware order: 4 consecutive row pairs (8 rows = one 128-byte line of
    // each column of the column-major output) run back to back on one XCD so
    // their 32-byte partial-line writes merge in that XCD's L2.
    int pb = blockIdx.x;
    {
        const int group = 32;                       // 8 XCD slots x 4 pairs
        const int full = (int)(gridDim.x / group) * group;
        if (pb < full) {
            const int x = pb % 8, t = pb / 8;
            pb = (t / 4) * group + x * 4 + (t % 4);
        }
    }
    const int y0 = 2 * pb, y1 = y0 + 1;
    const bool two = y1 < H;
    const uint8_t* r0 = img + (size_t)y0 * W * 3;
    const uint8_t* r1 = img + (size_t)(two ? y1 : y0) * W * 3;
    for (int x = tid; x < W; x += T) {
        // rgb2pgm (image_processing.c:509), then remove_dc_bias (blur_profile.c:236)
        const double p0 = 0.299 * k255[r0[3 * x]] + 0.587 * k255[r0[3 * x + 1]] + 0.114 * k255[r0[3 * x + 2]];
        const double p1 = 0.299 * k255[r1[3 * x]] + 0.587 * k255[r1[3 * x + 1]] + 0.114 * k255[r1[3 * x + 2]];
        buf[x] = make_double2(p0 - avg, two ? p1 - avg : 0.0);
    }
    __syncthreads();
    fft_lds<T, MODE>(buf, 1, plan, tw, tw + 64);
    // Z = A + iB with A, B the spectra of the two real rows:
    // A[k] = (Z[k] + conj Z[W-k]) / 2, B[k] = (Z[k] - conj Z[W-k]) / (2i)
    // written column-major, inter[k][y] (ld = H): lane pairs cover (k, y0), (k, y1)
    const int wf = W / 2 + 1;
    for (int i = tid; i < 2 * wf; i += T) {
        const int k = i >> 1, second = i & 1;
        if (second && !two) continue;
        const double2 zk = buf[k], zm = buf[k == 0 ? 0 : W - k];
        inter[(size_t)k * H + y0 + second] =
            second ? make_double2(0.5 * (zk.y + zm.y), -0.5 * (zk.x - zm.x))
                   : make_double2(0.5 * (zk.x + zm.x), 0.5 * (zk.y - zm.y));
    }
}

// LDS: [ C*H complex | twiddles (64 + n_hi) | log_mant table | polar bins (nbins u64, if lds_bins) ]
template <int T, int MODE>
__global__ __launch_bounds__(T) void k_fft_cols(const double2* __restrict__ inter0, size_t inter_stride, int H,
                                                int wf, int C, FftPlan plan, const uint16_t* __restrict__ binmap,
                                                int nbins, int lds_bins, unsigned long long* __restrict__ bin_sums0,
                                                double* __restrict__ fmax_part0, long out_stride, double bscale,
                                                int ablate) {
    // blockIdx.y: the image of a batch (inter0 + y * inter_stride elements,
    // bin sums and max partials at + y * out_stride doubles)
    const double2* inter = inter0 + (size_t)blockIdx.y * inter_stride;
    unsigned long long* bin_sums = bin_sums0 + (size_t)blockIdx.y * out_stride;
    double* fmax_part = fmax_part0 + (size_t)blockIdx.y * out_stride;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    double2* buf = reinterpret_cast<double2*>(smem);
    double2* tw = buf + (size_t)C * H;
    double2* lt = tw + 64 + plan.n_hi;
    unsigned long long* lb = reinterpret_cast<unsigned long long*>(lt + kLogTab);
    const int tid = threadIdx.x;
    const int cb = blockIdx.x;
    const int k0 = cb * C;
    const int nc = min(C, wf - k0);
    load_twiddles(tw, plan);
    log_table_init(lt, tid, T);
    if (lds_bins)
        for (int i = tid; i < nbins; i += T) lb[i] = 0ull;
    {
        // the nc columns are one contiguous run of the column-major spectrum
        const double2* src = inter + (size_t)k0 * H;
        for (int i = tid; i < nc * H; i += T) buf[i] = src[i];
    }
    __syncthreads();
    // this thread's contiguous run of elements and their bin ids, loaded
    // before the FFT so the loads are in flight during it (element i of the
    // block is row i % H of column k0 + i / H; the nc columns' bin ids are
    // one contiguous run of the map)
    constexpr int kPer = 8;                               // elements per thread (nc * H <= 8 T)
    const int total = (ablate & 2) ? 0 : nc * H;
    const int per = (total + T - 1) / T, i0 = tid * per, i1 = min(total, i0 + per);
    int bv[kPer];
    {
        const uint16_t* bmap = binmap + (size_t)k0 * H;
#pragma unroll
        for (int j = 0; j < kPer; j++) bv[j] = i0 + j < i1 ? (int)bmap[i0 + j] : -1;
    }
    if (!(ablate & 1)) fft_lds<T, MODE>(buf, nc, plan, tw, tw + 64);
    // p = |X|^2 per element (1 for p < 1, whose log the reference clamps
    // away), written over the spectrum as doubles: read to registers first
    double mx = 0.0;
    double pv[kPer];
#pragma unroll
    for (int j = 0; j < kPer; j++) {
        const int i = tid + j * T;
        pv[j] = 1.0;
        if (i < total) {
            const double2 X = buf[i];
            const double p = X.x * X.x + X.y * X.y;          // fft_processing.c:49
            mx = fmax(mx, p);
            pv[j] = p >= 1 ? p : 1.0;                        // fft_processing.c:197-198
        }
    }
    __syncthreads();
    double* lgb = reinterpret_cast<double*>(buf);
#pragma unroll
    for (int j = 0; j < kPer; j++)
        if (tid + j * T < total) lgb[tid + j * T] = pv[j];
    __syncthreads();
    // runs of one polar bin summed as the log of their product (frexp
    // mantissas multiply, exponents add, one fp64 log per run), one atomic per
    // run; the thread's first two runs are logged after the unrolled walk (as
    // fft_ct.hip's walk_runs)
    {
        auto flush = [&](int b, double m, int e) {
            const double a = fmax((double)e * 0.69314718055994530942 + log_mant(m, lt), 0.0);
            if (a > 0.0) {
                if (lds_bins) atomicAdd(&lb[b], bin_fixed(a, bscale));
                else atomicAdd(&bin_sums[b], bin_fixed(a, bscale));
            }
        };
        int cur = -1, esum = 0, n = 0, b0 = 0, b1 = 0, e0 = 0, e1 = 0;
        double mprod = 1.0, m0 = 1.0, m1 = 1.0;
        auto close = [&]() {
            if (n == 0) { b0 = cur; m0 = mprod; e0 = esum; n = 1; }
            else if (n == 1) { b1 = cur; m1 = mprod; e1 = esum; n = 2; }
            else flush(cur, mprod, esum);
        };
#pragma unroll
        for (int j = 0; j < kPer; j++) {
            if (bv[j] >= 0) {
                if (bv[j] != cur) {
                    if (cur >= 0) close();
                    cur = bv[j];
                    mprod = 1.0;
                    esum = 0;
                }
                int e;
                mprod *= frexp(lgb[i0 + j], &e);
                esum += e;
            }
        }
        if (cur >= 0) close();
        if (n > 0) flush(b0, m0, e0);
        if (n > 1) flush(b1, m1, e1);
    }
    // block max -> one partial per block (a per-wave atomicMax on one word
    // serialised ~16K atomics per image: ~160 us, DESIGN.md ablation)
    mx = wave_max(mx);
    __syncthreads();                      // buf is free now: reuse it as scratch
    double* red = reinterpret_cast<double*>(buf);
    if (lane_id() == 0) red[tid >> 6] = mx;
    __syncthreads();
    if (tid == 0) {
        double m = 0.0;
        for (int w = 0; w < T / 64; w++) m = fmax(m, red[w]);
        fmax_part[blockIdx.x] = m;
    }
    if (lds_bins && !(ablate & 4)) {
        for (int i = tid; i < nbins; i += T) {
            const unsigned long long a = lb[i];
            if (a != 0ull) atomicAdd(&bin_sums[i], a);
        }
    }
}

}  // namespace

template <typename K>
static void allow_big_lds(K kernel) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kernel), hipFuncAttributeMaxDynamicSharedMemorySize,
                              160 * 1024);
}

template <int T, int MODE>
static hipError_t rows_impl(const uint8_t* img, const uint8_t* const* imgs, int n, int height, int width,
                            const FftPlan& plan, const unsigned long long* sums, long sums_stride, const double* k255,
                            double2* inter, size_t inter_stride, hipStream_t st) {
    static bool once = (allow_big_lds(k_fft_rows<T, MODE>), true);
    (void)once;
    const size_t lds = sizeof(double2) * (width + 64 + plan.n_hi) + 256 * sizeof(double);
    phd_launch((k_fft_rows<T, MODE>), dim3((height + 1) / 2, n), dim3(T), lds, st, img, imgs, height, width,
                       plan, sums, sums_stride, k255, inter, inter_stride);
    return hipGetLastError();
}

// kernel mode of a plan (fft_runtime.h fft_lds)
static int plan_mode(const FftPlan& p) { return (p.composite ? 1 : 0) | (p.generic ? 2 : 0); }

static hipError_t rows_t(const uint8_t* img, const uint8_t* const* imgs, int n, int height, int width,
                         const FftPlan& plan, const unsigned long long* sums, long sums_stride, const double* k255,
                         double2* inter, size_t inter_stride, hipStream_t st) {
#define PHD_ROWS(T, M) rows_impl<T, M>(img, imgs, n, height, width, plan, sums, sums_stride, k255, inter, inter_stride, st)
    // composite plans (n <= 4096): 256 threads up to 2048 (8 elements each),
    // measured on 64-image groups, rows of 1920: 117 us per launch against
    // 205 at 512 threads; 512: 83 against 200
    switch (plan_mode(plan)) {
        case 1: return width <= 2048 ? PHD_ROWS(256, 1) : PHD_ROWS(512, 1);
        case 3: return width <= 2048 ? PHD_ROWS(256, 3) : PHD_ROWS(512, 3);
        case 2: return width <= 4096 ? PHD_ROWS(512, 2) : PHD_ROWS(1024, 2);
        default: return width <= 4096 ? PHD_ROWS(512, 0) : PHD_ROWS(1024, 0);
    }
#undef PHD_ROWS
}

hipError_t launch_fft_rows_batch(const uint8_t* const* d_imgs, int n, int height, int width, const FftPlan& plan,
                                 const unsigned long long* sums0, long sums_stride, const double* k255,
                                 double2* inter0, size_t inter_stride, hipStream_t st) {
    return rows_t(nullptr, d_imgs, n, height, width, plan, sums0, sums_stride, k255, inter0, inter_stride, st);
}

hipError_t launch_fft_rows(const uint8_t* img, int height, int width, const FftPlan& plan,
                           const unsigned long long* sums, const double* k255, double2* inter,
                           hipStream_t st) {
    return rows_t(img, nullptr, 1, height, width, plan, sums, 0, k255, inter, 0, st);
}

template <int T, int MODE>
static hipError_t cols_impl(const double2* inter, size_t inter_stride, int n, int height, int wf, int C,
                            const FftPlan& plan, const uint16_t* binmap, int nbins, int lds_bins, size_t lds,
                            unsigned long long* bin_sums, double* fmax_part, long out_stride, double bscale,
                            hipStream_t st) {
    static bool once = (allow_big_lds(k_fft_cols<T, MODE>), true);
    (void)once;
    static const int ablate = phd_knob("PHD_ABLATE") ? atoi(phd_knob("PHD_ABLATE")) : 0;   // debug only
    phd_launch((k_fft_cols<T, MODE>), dim3((wf + C - 1) / C, n), dim3(T), lds, st, inter, inter_stride, height,
                       wf, C, plan, binmap, nbins, lds_bins, bin_sums, fmax_part, out_stride,
                       bscale > 0.0 ? bscale : bin_scale(height, wf),
                       ablate);
    return hipGetLastError();
}

int fft_cols_blocks(int height, int wf, int nbins, const FftPlan& plan, size_t* lds_out, int* lds_bins_out) {
    constexpr size_t kLdsBudget = 158 * 1024;
    const size_t bins_bytes = sizeof(unsigned long long) * nbins;
    const int lds_bins = bins_bytes <= 48 * 1024;
    const size_t fixed = sizeof(double2) * (64 + plan.n_hi + kLogTab) + (lds_bins ? bins_bytes : 0);
    const size_t col_bytes = sizeof(double2) * height;
    // columns per block: up to ~3k elements (several blocks per CU; measured
    // on 64-image groups, per launch: 1080 rows C = 2 142 us against C = 8 196,
    // 720 rows C = 4 130 against 171, 512 rows C = 4 54 against 69)
    static const int cmax = phd_knob("PHD_FFT_COLS_C") ? atoi(phd_knob("PHD_FFT_COLS_C")) : 8;   // tuning
    int C = 1;
    while (C < cmax && (size_t)(2 * C) * height <= 3072 && (2 * C) * col_bytes + fixed <= kLdsBudget) C *= 2;
    if (lds_out) *lds_out = C * col_bytes + fixed;
    if (lds_bins_out) *lds_bins_out = lds_bins;
    return C;
}

static hipError_t cols_t(const double2* inter0, size_t inter_stride, int n, int height, int wf, const FftPlan& plan,
                         const uint16_t* binmap, int nbins, unsigned long long* bin_sums0, double* fmax_part0, long out_stride,
                         hipStream_t st, double bscale = 0.0) {
    size_t lds;
    int lds_bins;
    const int C = fft_cols_blocks(height, wf, nbins, plan, &lds, &lds_bins);
    const size_t e = (size_t)C * height;
#define PHD_COLS(T, M) cols_impl<T, M>(inter0, inter_stride, n, height, wf, C, plan, binmap, nbins, lds_bins, lds, \
                                       bin_sums0, fmax_part0, out_stride, bscale, st)
    switch (plan_mode(plan)) {
        case 1: return e <= 2048 ? PHD_COLS(256, 1) : PHD_COLS(512, 1);
        case 3: return e <= 2048 ? PHD_COLS(256, 3) : PHD_COLS(512, 3);
        case 2: return e <= 4096 ? PHD_COLS(512, 2) : PHD_COLS(1024, 2);
        default: return e <= 4096 ? PHD_COLS(512, 0) : PHD_COLS(1024, 0);
    }
#undef PHD_COLS
}

hipError_t launch_fft_cols_batch(const double2* inter0, size_t inter_stride, int n, int height, int wf,
                                 const FftPlan& plan, const uint16_t* binmap, int nbins, unsigned long long* bin_sums0,
                                 double* fmax_part0, long out_stride, hipStream_t st) {
    return cols_t(inter0, inter_stride, n, height, wf, plan, binmap, nbins, bin_sums0, fmax_part0, out_stride, st);
}

hipError_t launch_fft_cols(const double2* inter, int height, int wf, const FftPlan& plan,
                           const uint16_t* binmap, int nbins, unsigned long long* bin_sums,
                           double* fmax_part, hipStream_t st, double bscale) {
    return cols_t(inter, 0, 1, height, wf, plan, binmap, nbins, bin_sums, fmax_part, 0, st, bscale);
}

}  // namespace phd
