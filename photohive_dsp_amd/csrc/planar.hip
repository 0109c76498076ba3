// planar.hip -- the legacy entry point's fp64 planar input.
//
// get_full_report_data (src/interface.c:20-94) takes three planes of doubles.
// The Python binding fills them with k/255.0 (utils.py:30-46); then the
// library converts them back to RGB8 on the device (k_planar_to_u8) and runs
// the RGB8 pipeline, whose arithmetic reproduces the reference's on those
// doubles exactly.  A C caller may pass any doubles (a 16-bit image / 65535,
// a tone-mapped float image): this file runs the reference's own fp64
// arithmetic on them --
//   * get_rgb_statistics (src/image_processing.c:543-553, get_average /
//     get_variance src/filtering.c:125-148): fp64 sums per block, reduced in a
//     fixed order (run-to-run identical), the variance's second pass on the
//     means;
//   * rgb2pgm (src/image_processing.c:505-512) into an fp64 luma plane for the
//     generic FFT path (fft_global.hip) and the sharpness crops;
//   * rgb2hsv + arm_octree (src/image_processing.c:372-417,
//     src/color_quantization.c:108-161) per pixel in fp64 (phd_device.h),
//     the group histogram and its per-chunk counts, sum(s) for S-bar;
//   * the tie-overflow cut-off search and calculate_avg_hsv's per-slot sums
//     (src/color_quantization.c:414-450, 510-576) after the host decisions.
#include "phd_device.h"

namespace phd {

namespace {

constexpr int kPT = 256;

// flags (device int): bit 0 some value is not k/255 (not an 8-bit image);
// bit 1 a value is not finite; bit 2 a pixel's group index falls outside the
// octree (values above 1: the reference indexes out of bounds).  Any other
// finite values are the reference's to report on: negative channels, luma
// outside [0, 1] (the polar bins' fixed-point scale follows the observed luma
// range, bin_scale)
constexpr int kFlagNotU8 = 1, kFlagNonFinite = 2, kFlagGroupRange = 4;

__device__ __forceinline__ void flag_wave(int* flags, bool bad, int bit) {
    if (__any(bad) && lane_id() == 0) atomicOr(flags, bit);
}

// fixed-order block sum of one double per thread (wave shuffles, then waves in order)
__device__ __forceinline__ double block_sum(double x, double* red) {
    x = wave_sum(x);
    __syncthreads();
    if (lane_id() == 0) red[threadIdx.x >> 6] = x;
    __syncthreads();
    double t = 0.0;
    for (int q = 0; q < kPT / 64; q++) t += red[q];
    return t;
}

// The 8-bit test: every value is exactly (double)k / 255.0 for an integer k
// in [0, 255] (utils.py:30-46); the RGB8 image is written as it goes.
__global__ __launch_bounds__(kPT) void k_planar_to_u8(PlanarSrc P, long n, uint8_t* __restrict__ rgb,
                                                      int* __restrict__ flags) {
    for (long i = (long)blockIdx.x * kPT + threadIdx.x; i - threadIdx.x < n; i += (long)gridDim.x * kPT) {
        bool bad = false;
        if (i < n) {
            const double x[3] = {P.r[i], P.g[i], P.b[i]};
#pragma unroll
            for (int c = 0; c < 3; c++) {
                const bool in = x[c] >= 0.0 && x[c] <= 1.0;      // false for NaN
                const int k = in ? (int)rint(x[c] * 255.0) : 0;
                bad |= !in || (double)k / 255.0 != x[c];
                rgb[3 * i + c] = (uint8_t)k;
            }
        }
        flag_wave(flags, bad, kFlagNotU8);
    }
}

// Channel sums (one partial per block and channel: part[3 * block + c]), the
// luma plane pgm = 0.299 r + 0.587 g + 0.114 b and its range per block
// (lrng[2 * block] = -min, lrng[2 * block + 1] = max; -inf for no pixel).
__global__ __launch_bounds__(kPT) void k_planar_moments(PlanarSrc P, long n, double* __restrict__ pgm,
                                                        double* __restrict__ part, double* __restrict__ lrng,
                                                        int* __restrict__ flags) {
    __shared__ double red[kPT / 64];
    double s[3] = {0.0, 0.0, 0.0};
    double nlo = -__builtin_inf(), hi = -__builtin_inf();
    for (long i0 = (long)blockIdx.x * kPT; i0 < n; i0 += (long)gridDim.x * kPT) {
        const long i = i0 + threadIdx.x;
        bool bad = false;
        if (i < n) {
            const double r = P.r[i], g = P.g[i], b = P.b[i];
            bad = !isfinite(r) || !isfinite(g) || !isfinite(b);
            s[0] += r;
            s[1] += g;
            s[2] += b;
            const double y = 0.299 * r + 0.587 * g + 0.114 * b;
            pgm[i] = y;
            nlo = fmax(nlo, -y);
            hi = fmax(hi, y);
        }
        flag_wave(flags, bad, kFlagNonFinite);
    }
    for (int c = 0; c < 3; c++) {
        const double t = block_sum(s[c], red);
        if (threadIdx.x == 0) part[3 * blockIdx.x + c] = t;
    }
    double m[2] = {nlo, hi};
    for (int k = 0; k < 2; k++) {
        double x = wave_max(m[k]);
        __syncthreads();
        if (lane_id() == 0) red[threadIdx.x >> 6] = x;
        __syncthreads();
        for (int q = 0; q < kPT / 64; q++) x = fmax(x, red[q]);
        if (threadIdx.x == 0) lrng[2 * blockIdx.x + k] = x;
    }
}

// get_average's mean per channel from the block partials, summed in a fixed
// order (the same in every block): B = sum / N.
__device__ __forceinline__ void planar_means(const double* __restrict__ part, int nb, long n, double* mean) {
    if (threadIdx.x < 3) {
        double a = 0.0;
        for (int k = 0; k < nb; k++) a += part[3 * k + threadIdx.x];
        mean[threadIdx.x] = a / (double)n;
    }
    __syncthreads();
}

// get_variance's second pass: sum (x - B)^2 per channel (part2), and the DC
// bias avg = (Br + Bg + Bb) / 3.0 (src/interface.c:78) for the FFT.
__global__ __launch_bounds__(kPT) void k_planar_var(PlanarSrc P, long n, const double* __restrict__ part1, int nb,
                                                    double* __restrict__ part2, double* __restrict__ avg_out) {
    __shared__ double red[kPT / 64];
    __shared__ double mean[3];
    planar_means(part1, nb, n, mean);
    const double br = mean[0], bg = mean[1], bb = mean[2];
    if (blockIdx.x == 0 && threadIdx.x == 0) *avg_out = (br + bg + bb) / 3.0;
    double s[3] = {0.0, 0.0, 0.0};
    for (long i = (long)blockIdx.x * kPT + threadIdx.x; i < n; i += (long)gridDim.x * kPT) {
        const double dr = P.r[i] - br, dg = P.g[i] - bg, db = P.b[i] - bb;
        s[0] += dr * dr;
        s[1] += dg * dg;
        s[2] += db * db;
    }
    for (int c = 0; c < 3; c++) {
        const double t = block_sum(s[c], red);
        if (threadIdx.x == 0) part2[3 * blockIdx.x + c] = t;
    }
}

__device__ __forceinline__ int planar_group(const PlanarSrc& P, long p, const GridParams& gp, double& h, double& s,
                                            double& v) {
    rgb2hsv(P.r[p], P.g[p], P.b[p], h, s, v);
    return group_of(gp, h, s, v);
}

// K1 on doubles: one block per chunk of kChunk hsv pixels (downsample_rgb's
// mapping for ds > 1): group histogram (hist, and the chunk's counts for the
// cut-off search) and the chunk's sum of s (get_hsv_average).
__global__ __launch_bounds__(kPT) void k_planar_k1(PlanarSrc P, long npix, int width, int ds, int nw, GridParams gp,
                                                   unsigned* __restrict__ hist, unsigned short* __restrict__ chunk_hist,
                                                   double* __restrict__ s_part, int* __restrict__ flags) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    unsigned* lh = reinterpret_cast<unsigned*>(smem);
    __shared__ double red[kPT / 64];
    for (int i = threadIdx.x; i < gp.tl; i += kPT) lh[i] = 0;
    __syncthreads();
    const long base = (long)blockIdx.x * kChunk;
    const long end = min(base + (long)kChunk, npix);
    double ssum = 0.0;
    for (long j0 = base; j0 < end; j0 += kPT) {
        const long j = j0 + threadIdx.x;
        bool bad = false;
        if (j < end) {
            double h, s, v;
            const int g = planar_group(P, src_pixel(j, width, ds, nw), gp, h, s, v);
            ssum += s;
            bad = g < 0 || g >= gp.tl;
            if (!bad) atomicAdd(&lh[g], 1u);
        }
        flag_wave(flags, bad, kFlagGroupRange);
    }
    const double t = block_sum(ssum, red);
    if (threadIdx.x == 0) s_part[blockIdx.x] = t;
    __syncthreads();
    for (int i = threadIdx.x; i < gp.tl; i += kPT) {
        const unsigned c = lh[i];
        chunk_hist[(long)blockIdx.x * gp.tl + i] = (unsigned short)c;
        if (c) atomicAdd(&hist[i], c);
    }
}

__device__ int scan_excl(int x, int& excl, int* scratch) {
    const int lane = lane_id(), w = threadIdx.x >> 6;
    int incl = x;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(incl, o, 64);
        if (lane >= o) incl += y;
    }
    if (lane == 63) scratch[w] = incl;
    __syncthreads();
    int wpre = 0, tot = 0;
    for (int q = 0; q < kPT / 64; q++) {
        if (q < w) wpre += scratch[q];
        tot += scratch[q];
    }
    __syncthreads();
    excl = wpre + incl - x;
    return tot;
}

// The cut-off search of group_irregular_pixels' tie path on doubles: one
// block per searched group, the raster index of its keep-th pixel (the chunk
// from the per-chunk counts, then a block scan inside it) and of its last.
__global__ __launch_bounds__(kPT) void k_planar_cutoffs(PlanarSrc P, long npix, int width, int ds, int nw,
                                                        GridParams gp, const unsigned short* __restrict__ chunk_hist,
                                                        int nchunks, GroupRule* rules,
                                                        const int* __restrict__ search) {
    __shared__ int scratch[kPT / 64];
    __shared__ int s_chunk, s_rank, s_last_chunk, s_found;
    __shared__ unsigned s_idx;
    const int tid = threadIdx.x;
    const int g = search[blockIdx.x];
    const int keep = rules[g].keep;
    const int want_cut = rules[g].partial && keep > 0;
    const int want_last = rules[g].partial && rules[g].dangle;
    if (tid == 0) {
        s_chunk = -1;
        s_last_chunk = -1;
    }
    __syncthreads();
    int carry = 0;
    for (int c0 = 0; c0 < nchunks; c0 += kPT) {
        const int c = c0 + tid;
        const int cnt = c < nchunks ? (int)chunk_hist[(long)c * gp.tl + g] : 0;
        int excl;
        const int tot = scan_excl(cnt, excl, scratch);
        if (want_cut && cnt > 0 && carry + excl < keep && keep <= carry + excl + cnt) {
            s_chunk = c;
            s_rank = keep - (carry + excl);
        }
        if (cnt > 0) atomicMax(&s_last_chunk, c);
        carry += tot;
        __syncthreads();
    }
    for (int pass = 0; pass < 2; pass++) {
        const int c = pass == 0 ? (want_cut ? s_chunk : -1) : (want_last ? s_last_chunk : -1);
        if (c < 0) continue;
        const long base = (long)c * kChunk, end = min(base + (long)kChunk, npix);
        int rank = s_rank;
        if (tid == 0) {
            s_found = 0;
            s_idx = 0;
        }
        __syncthreads();
        for (long j0 = base; j0 < end; j0 += kPT) {
            const long j = j0 + tid;
            int hit = 0;
            if (j < end) {
                double h, s, v;
                hit = planar_group(P, src_pixel(j, width, ds, nw), gp, h, s, v) == g;
            }
            if (pass == 0) {
                int excl;
                const int tot = scan_excl(hit, excl, scratch);
                if (hit && excl + 1 == rank) {
                    s_idx = (unsigned)j;
                    s_found = 1;
                }
                rank -= tot;
                __syncthreads();
                if (s_found) break;
            } else if (hit) {
                atomicMax(&s_idx, (unsigned)j);
            }
        }
        __syncthreads();
        if (tid == 0) {
            if (pass == 0) rules[g].cutoff = s_idx + 1;
            else rules[g].last = s_idx;
        }
        __syncthreads();
    }
}

// calculate_avg_hsv's per-slot sums over the kept pixels (K3 on doubles):
// out[4 slot + {0,1,2,3}] = sum wrap(h + off), sum s, sum v, n.
__global__ __launch_bounds__(kPT) void k_planar_sums(PlanarSrc P, long npix, int width, int ds, int nw, GridParams gp,
                                                     const GroupRule* __restrict__ rules_g,
                                                     const double* __restrict__ off_g, int nslots,
                                                     double* __restrict__ out) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    double* acc = reinterpret_cast<double*>(smem);                       // nslots * 4
    double* off = acc + 4 * nslots;                                      // nslots
    GroupRule* rules = reinterpret_cast<GroupRule*>(off + nslots);       // tl
    const int tid = threadIdx.x;
    for (int i = tid; i < 4 * nslots; i += kPT) acc[i] = 0.0;
    for (int i = tid; i < nslots; i += kPT) off[i] = off_g[i];
    for (int i = tid; i < gp.tl; i += kPT) rules[i] = rules_g[i];
    __syncthreads();
    const long base = (long)blockIdx.x * kChunk;
    const long end = min(base + (long)kChunk, npix);
    for (long j0 = base; j0 < end; j0 += kPT) {
        const long j = j0 + tid;
        int slot = -1;
        double h = 0.0, s = 0.0, v = 0.0, tp = 0.0;
        if (j < end) {
            const int g = planar_group(P, src_pixel(j, width, ds, nw), gp, h, s, v);
            if (g >= 0 && g < gp.tl) {
                const GroupRule& R = rules[g];
                const unsigned idx = (unsigned)j;
                if (R.slot >= 0 && (!R.partial || idx < R.cutoff || (R.dangle && idx == R.last))) {
                    slot = R.slot;
                    tp = h + off[slot];                    // src/color_quantization.c:538-546
                    if (tp > 360) tp -= 360;
                    else if (tp < 0) tp += 360;
                }
            }
        }
        const int s0 = __builtin_amdgcn_readfirstlane(slot);
        if (__all(slot == s0)) {
            if (s0 >= 0) {
                const double th = wave_sum(tp), ts = wave_sum(s), tv = wave_sum(v);
                const double cnt = wave_sum(1.0);
                if (lane_id() == 0) {
                    atomicAdd(&acc[4 * s0 + 0], th);
                    atomicAdd(&acc[4 * s0 + 1], ts);
                    atomicAdd(&acc[4 * s0 + 2], tv);
                    atomicAdd(&acc[4 * s0 + 3], cnt);
                }
            }
        } else if (slot >= 0) {
            atomicAdd(&acc[4 * slot + 0], tp);
            atomicAdd(&acc[4 * slot + 1], s);
            atomicAdd(&acc[4 * slot + 2], v);
            atomicAdd(&acc[4 * slot + 3], 1.0);
        }
    }
    __syncthreads();
    for (int i = tid; i < 4 * nslots; i += kPT) {
        const double a = acc[i];
        if (a != 0.0) atomicAdd(&out[i], a);
    }
}

unsigned grid_for(long n) { return (unsigned)std::max<long>(1, std::min<long>(kPlanarBlocks, (n + kPT - 1) / kPT)); }

}  // namespace

hipError_t launch_planar_to_u8(const PlanarSrc& P, long n, uint8_t* rgb, int* flags, hipStream_t st) {
    phd_launch(k_planar_to_u8, dim3(grid_for(n)), dim3(kPT), 0, st, P, n, rgb, flags);
    return hipGetLastError();
}

int planar_blocks(long n) { return (int)grid_for(n); }

hipError_t launch_planar_stats(const PlanarSrc& P, long n, double* pgm, double* part1, double* part2, double* avg,
                               double* lrng, int* flags, hipStream_t st) {
    const unsigned nb = grid_for(n);
    phd_launch(k_planar_moments, dim3(nb), dim3(kPT), 0, st, P, n, pgm, part1, lrng, flags);
    phd_launch(k_planar_var, dim3(nb), dim3(kPT), 0, st, P, n, (const double*)part1, (int)nb, part2, avg);
    return hipGetLastError();
}

hipError_t launch_planar_k1(const PlanarSrc& P, int height, int width, int ds, const GridParams& gp, unsigned* hist,
                            unsigned short* chunk_hist, double* s_part, int* flags, hipStream_t st) {
    int nw = width;
    long npix = (long)height * width;
    if (ds > 1) {
        nw = width / ds;
        npix = (long)(short)(height / ds) * (short)nw;
    }
    const unsigned nchunks = (unsigned)((npix + kChunk - 1) / kChunk);
    phd_launch(k_planar_k1, dim3(nchunks), dim3(kPT), sizeof(unsigned) * gp.tl, st, P, npix, width, ds, nw, gp, hist,
               chunk_hist, s_part, flags);
    return hipGetLastError();
}

hipError_t launch_planar_tail(const PlanarSrc& P, int height, int width, int ds, const GridParams& gp,
                              const unsigned short* chunk_hist, int nchunks, GroupRule* rules, const int* search,
                              int n_search, const double* off, int nslots, double* out, hipStream_t st) {
    int nw = width;
    long npix = (long)height * width;
    if (ds > 1) {
        nw = width / ds;
        npix = (long)(short)(height / ds) * (short)nw;
    }
    if (n_search > 0)
        phd_launch(k_planar_cutoffs, dim3((unsigned)n_search), dim3(kPT), 0, st, P, npix, width, ds, nw, gp,
                   chunk_hist, nchunks, rules, search);
    if (nslots > 0) {
        const size_t lds = sizeof(double) * 5 * nslots + sizeof(GroupRule) * gp.tl;
        static bool once = ((void)hipFuncSetAttribute(reinterpret_cast<const void*>(k_planar_sums),
                                                      hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024),
                            true);
        (void)once;
        phd_launch(k_planar_sums, dim3((unsigned)((npix + kChunk - 1) / kChunk)), dim3(kPT), lds, st, P, npix, width,
                   ds, nw, gp, (const GroupRule*)rules, off, nslots, out);
    }
    return hipGetLastError();
}

}  // namespace phd
