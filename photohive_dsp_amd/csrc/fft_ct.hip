// fft_ct.hip -- the 2-D power spectrum and polar binning for image sizes with a
// compile-time FFT plan (fft_engine.h; the plan lists are PHD_CT_ROWS /
// PHD_CT_COLS in phd_internal.h).  Other sizes take fft.hip's runtime-plan
// kernels.
//
// Replaces rgb2pgm + remove_dc_bias (src/image_processing.c:505-512,
// src/blur_profile.c:233-238), pgm_fft (src/fft_processing.c:18-63: FFTW r2c,
// unnormalised, e^{-i}), pgm_normalize_fft (:173-213) and the binning loop of
// calculate_blur_profile (src/blur_profile.c:87-100).
//
// Intermediate layout (half spectrum after the row pass), tiled so that both
// passes move whole 64-byte pieces: element (y, k) of row pair p = y/2 and
// column pair kp = k/2 sits at p * RS + (kp * 2 + k%2) * 2 + y%2, with
// KP = ceil((W/2+1) / 2) and RS = ct_row_stride(W), 4 KP rounded up to 8
// elements so each row pair starts on a 128-byte line.  A row pair's spectrum
// is one contiguous 64 KB run (W = 4000); a column pair is 1500 pieces of 64 B
// (H = 3000).
//
// Row kernel (persistent, 2 blocks per CU).  Each step handles one pair of
// image rows.  Both rows' RGB8 bytes were prefetched into registers (dwordx3 =
// 4 pixels) during the previous step.  They become luma - avg and are packed
// as one complex row (row y0 real, row y0+1 imaginary) in LDS (no DC removal:
// the column pass does it on column 0, so the rows need nothing from K1).  The next pair's
// loads are issued, then the FFT runs in LDS.  The two half spectra are
// separated, A[k] = (Z[k] + conj Z[W-k]) / 2 and B[k] = (Z[k] - conj Z[W-k]) / 2i,
// and stored as the pair's contiguous tile row.
//
// Column kernel (persistent, two blocks of T threads per CU, one column at a
// time per block; blocks b, b^8, b^16, b^24 of one XCD take the four columns
// of the same 128-byte lines, each block a contiguous range of line pairs).
// The next column streams into LDS by LDS-DMA while the current one finishes
// (the full- or half-prefetch form, ColK).
// The last pass's outputs never go back to LDS as spectra: the epilogue forms
// p = re^2 + im^2, keeps the block's max and writes p (1 for p < 1, whose log
// the reference clamps away) per spectrum row to LDS; each thread then walks a
// contiguous run of rows and adds one LDS atomic per run of one polar bin.  The
// block adds its non-zero bins to the image's bin sums at the end.
//
// log(p) for the bins: a run's sum of log p is the log of its product.  The
// frexp mantissas (in [1/2, 1)) multiply in fp64 and the exponents add, and
// one fp64 log of the mantissa product closes the run: e ln2 + log(m), as
// pgm_normalize_fft's per-element fp64 log (src/fft_processing.c:196-199) to
// ~1e-15 per run.  The max and the p >= 1 test stay in fp64.
#include <algorithm>
#include <cstdlib>

// Nothing in this file needs the reference's rounding (the FFT only has to be
// within the north_star tolerance), so fused multiply-adds are allowed here.
#pragma clang fp contract(fast)

#include "fft_engine.h"
#include "phd_device.h"

namespace phd {

namespace {

using namespace fe;

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));   // a native 128-bit register tuple

constexpr double kWr = 0.299 / 255.0, kWg = 0.587 / 255.0, kWb = 0.114 / 255.0;

// 12 bytes (4 RGB8 pixels) as one dwordx3 register tuple; 4-byte alignment
typedef unsigned u32x3a __attribute__((ext_vector_type(3), aligned(4)));
// ... read through a global-address-space pointer: the image pointer comes from
// a device array, and a generic (flat) load would also count against the LDS
// counter, so every LDS wait of the FFT would wait for the prefetched pixels
typedef const __attribute__((address_space(1))) u32x3a gu32x3a;
// The row pass's pixel loads are plain loads (round 6; PHD_ROW_NT=1, an A/B
// build, makes them non-temporal as before): a 12000-byte image row starts
// 0-96 B into a 128-B line, so two wave-instructions share the line at each
// 768-byte boundary, and the non-temporal first request let the stores'
// traffic evict it before the second.  Rows 41.2-41.3 -> 39.2-39.6 us, their
// HBM traffic 142.2 -> 137.2 MB per image (1.039x the algorithmic bytes;
// profiles/r06/row_loads_temporal_ab.log).
#ifndef PHD_ROW_NT
#define PHD_ROW_NT 0
#endif

__device__ __forceinline__ int byte_of(const u32x3a& w, int b) {
    const unsigned x = (b >> 2) == 0 ? w.x : ((b >> 2) == 1 ? w.y : w.z);   // b is a constant
    return (x >> (8 * (b & 3))) & 255;
}

// x of the lane next to this one in its pair (lanes 2m, 2m + 1), by DPP
// (quad_perm [1, 0, 3, 2])
__device__ __forceinline__ double dpp_pair_swap(double x) {
    const unsigned long long u = __builtin_bit_cast(unsigned long long, x);
    const unsigned lo = (unsigned)__builtin_amdgcn_mov_dpp((int)(unsigned)u, 0xB1, 0xF, 0xF, false);
    const unsigned hi = (unsigned)__builtin_amdgcn_mov_dpp((int)(unsigned)(u >> 32), 0xB1, 0xF, 0xF, false);
    return __builtin_bit_cast(double, ((unsigned long long)hi << 32) | lo);
}

// The 4 pixels of a 12-byte group rotated by r (0-3) pixels, i.e. its bytes
// by 3 r = 4 q + sh: pixel e of the result is pixel (e + r) & 3 of w (word i
// of the result: bytes sh.. of word q + i and the low bytes of word q + i + 1)
__device__ __forceinline__ u32x3a rot_px(const u32x3a& w, int r) {
    const int b = 3 * r, q = b >> 2, sh = b & 3;
    const unsigned l0 = q == 0 ? w.x : (q == 1 ? w.y : w.z);
    const unsigned l1 = q == 0 ? w.y : (q == 1 ? w.z : w.x);
    const unsigned l2 = q == 0 ? w.z : (q == 1 ? w.x : w.y);
    u32x3a o;
    o.x = __builtin_amdgcn_alignbyte(l1, l0, (unsigned)sh);
    o.y = __builtin_amdgcn_alignbyte(l2, l1, (unsigned)sh);
    o.z = __builtin_amdgcn_alignbyte(l0, l2, (unsigned)sh);
    return o;
}

// One thread's walk over E consecutive rows of a column: p per row in LDS
// (lgb[r0 + j]), the column's bin runs in LDS (rl: start row << 16 | bin id,
// ColRuns), sg = the thread's segment word (ColBins::seg: the run holding row
// r0, bits 0-7, and the rows j > 0 where a run starts, bit 8 + j).  Contiguous
// rows of one bin form a run whose sum of log p is the log of its product: the
// frexp mantissas multiply (>= 2^-E, no underflow), the exponents add, and one
// fp64 log closes the run (pgm_normalize_fft's fp64 log, src/fft_processing.c:
// 196-199).  Each run adds bin_scale fixed point to its run's LDS slot (sl,
// indexed like rl) with one LDS atomic (order-independent sums); the block
// adds the column's slots to the image's bins afterwards.
//
// Fast form (round 6), a wave whose lanes each meet at most two run starts
// (~97 % of the waves of 4000x3000 / 72x40): branch-free, the starts f1 < f2
// from the segment word, the product restarting at each and the first two
// runs' products kept in registers; the wave then evaluates the fp64 log two
// or three times.  Otherwise the general walk: the run list's entries in
// registers, one branch per row (some lane of 64 changes bin on most rows).
// Both multiply the same rows in the same order: identical bins.
// HFULL: H % E == 0, so a thread with r0 < H has all E rows.
template <int E, bool HFULL>
__device__ __forceinline__ void walk_runs(const double* __restrict__ lgb, int r0, int rend, const unsigned* rl,
                                          unsigned sg, unsigned long long* sl, double bscale,
                                          const double2* __restrict__ lt) {
    auto flush = [&](int k, double m, int e) {
        const double acc = fmax((double)e * 0.69314718055994530942 + log_mant(m, lt), 0.0);
        atomicAdd(&sl[k], bin_fixed(acc, bscale));
    };
    if (r0 >= rend) return;
    const int idx = (int)(sg & 255u);
    const unsigned chm = sg >> 8;
    if (__all(__popc(chm) <= 2)) {
        const int f1 = __builtin_ctz(chm | 0x80000000u), f2 = __builtin_ctz((chm & (chm - 1)) | 0x80000000u);
        double mp = 1.0, m0 = 1.0, m1 = 1.0;
        int es = 0, e0 = 0, e1 = 0;
#pragma unroll
        for (int j = 0; j < E; j++) {
            const int r = r0 + j;
            if (HFULL || r < rend) {
                const double pv = lgb[r];
                if (j > 0) {
                    const bool c1 = f1 == j, c2 = f2 == j;
                    m0 = c1 ? mp : m0;
                    e0 = c1 ? es : e0;
                    m1 = c2 ? mp : m1;
                    e1 = c2 ? es : e1;
                    mp = (c1 || c2) ? 1.0 : mp;
                    es = (c1 || c2) ? 0 : es;
                }
                int e;
                mp *= frexp(pv, &e);
                es += e;
            }
        }
        const int n = __popc(chm);
        flush(idx, n == 0 ? mp : m0, n == 0 ? es : e0);
        if (n >= 1) flush(idx + 1, n == 1 ? mp : m1, n == 1 ? es : e1);
        if (n == 2) flush(idx + 2, mp, es);
        return;
    }
    // general walk: the thread's first four entries in registers (one LDS
    // latency), refilled one entry per run change; entries past the column's
    // sentinel are never used (the sentinel's start is the height).  A thread's
    // first two runs are kept in registers and logged after the walk.
    unsigned q1 = rl[idx + 1], q2 = rl[min(idx + 2, kColRunsMax - 1)], q3 = rl[min(idx + 3, kColRunsMax - 1)];
    int qi = idx + 4;
    int cur = idx, nxt = (int)(q1 >> 16);                   // cur: the run's slot
    int esum = 0, n = 0, b0 = 0, b1 = 0, e0 = 0, e1 = 0;
    // (round 6: the product in two interleaved chains, even / odd rows,
    // measured the same, 48.1-48.9 against 48.3-49.0 us: not the bound)
    double mp = 1.0;
    double m0 = 1.0, m1 = 1.0;
    auto close = [&]() {
        if (n == 0) {
            b0 = cur; m0 = mp; e0 = esum; n = 1;
        } else if (n == 1) {
            b1 = cur; m1 = mp; e1 = esum; n = 2;
        } else {
            flush(cur, mp, esum);
        }
    };
#pragma unroll
    for (int j = 0; j < E; j++) {
        const int r = r0 + j;
        if (HFULL || r < rend) {
            const double pv = lgb[r];
            if (r >= nxt) {                       // the next run starts here (runs are never empty)
                close();
                cur++;
                q1 = q2;
                q2 = q3;
                q3 = rl[min(qi++, kColRunsMax - 1)];
                nxt = (int)(q1 >> 16);
                mp = 1.0;
                esum = 0;
            }
            int e;
            mp *= frexp(pv, &e);
            esum += e;
        }
    }
    close();
    if (n > 0) flush(b0, m0, e0);
    if (n > 1) flush(b1, m1, e1);
}

template <int W, int T, int... Rs>
struct RowK {
    static constexpr int NTW = tw_entries<1, Rs...>();
    static constexpr int G4 = W / 4;                       // 4-pixel groups per row
    static constexpr int LR = (G4 + T - 1) / T;            // groups per thread
    static constexpr size_t lds = sizeof(double2) * (W + NTW);
    static_assert(W % 4 == 0, "row plans need W % 4 == 0");
    static_assert(Radices<Rs...>::product == W, "plan");
    // waves per SIMD the launch bounds ask for: 2 blocks per CU, fewer when
    // the LDS holds fewer (W = 6000: one block, so twice the VGPRs)
    static constexpr int BPC = (int)((160 * 1024) / lds) < 2 ? (int)((160 * 1024) / lds) : 2;
    static constexpr int MINW = (T >= 512 ? 4 : 2) * BPC / 2 > 0 ? (T >= 512 ? 4 : 2) * BPC / 2 : 1;
};

template <int W, int T, int... Rs>
__global__ __launch_bounds__(T, (RowK<W, T, Rs...>::MINW)) void k_rows_ct(const uint8_t* __restrict__ img, int H,
                                               const unsigned long long* __restrict__ sums,
                                               const double* __restrict__ k255g, const double2* __restrict__ twg,
                                               double2* __restrict__ inter, int ablate_arg,
                                               unsigned long long* __restrict__ rsum,
                                               const uint8_t* const* __restrict__ imgs, int nimg, long istride) {
    using K = RowK<W, T, Rs...>;
    const int ablate = PHD_ABL(ablate_arg);
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    double2* buf = reinterpret_cast<double2*>(smem);
    double2* tw = buf + W;
    const int tid = threadIdx.x;
    for (int i = tid; i < K::NTW; i += T) tw[i] = twg[i];
    // schedule: line group m (pairs 4m..4m+3) on XCD m % 8, its 4 pairs on 4
    // blocks of that XCD (gridDim.x is a multiple of 32).  A batch (imgs, nimg
    // images whose P is a multiple of 4, intermediates istride apart) numbers
    // its images' line groups one after the other.
    const int P = (H + 1) / 2, G = (P + 3) / 4;
    const int x = blockIdx.x & 7, q = blockIdx.x >> 3, QA = gridDim.x >> 5;
    const int a = q >> 2, i4 = q & 3;
    // step s's image and row pair (false past the last)
    auto item = [&](int s, int& im, int& pr) {
        const int m = x + 8 * (a + s * QA);
        im = m / G;
        pr = 4 * (m - im * G) + i4;
        return im < nimg && pr < P;
    };

    // the next pair's pixels, loaded straight into the registers the luma code
    // reads (no moves, so nothing waits for the loads before they are used);
    // groups past the row end re-load group 0 (unused, no branch)
    u32x3a rg[K::LR][2];
    auto fetch = [&](int im, int pr) {
        // (byte addressing: a 3-vector's sizeof is 16, a group is 12 bytes)
        const int y0 = 2 * pr;
        const uint8_t* r0 = (imgs ? imgs[im] : img) + (size_t)y0 * 3 * W;
        const uint8_t* r1 = (y0 + 1 < H) ? r0 + 3 * W : r0;
#pragma unroll
        for (int j = 0; j < K::LR; j++) {
            const int g = (K::G4 % T == 0 || tid + j * T < K::G4) ? tid + j * T : 0;
#if PHD_ROW_NT
            rg[j][0] = __builtin_nontemporal_load((gu32x3a*)(r0 + 12 * g));
            rg[j][1] = __builtin_nontemporal_load((gu32x3a*)(r1 + 12 * g));
#else
            rg[j][0] = *(gu32x3a*)(r0 + 12 * g);
            rg[j][1] = *(gu32x3a*)(r1 + 12 * g);
#endif
        }
    };
    int s = 0, im = 0, pr = 0;
    bool live = item(0, im, pr);
    if (live) fetch(im, pr);
    __syncthreads();
    unsigned cs[3] = {0u, 0u, 0u};    // this thread's channel sums (u32: a few row pairs of bytes)
    // b128 write swizzle: 8 lanes of a group hit 8 distinct 16-B slots (the
    // group's pixels rotated by rot in its bytes, rot_px)
    const int rot = (tid >> 1) & 3;
    // one row pair.  The loop head is reached with the same memory operations in
    // flight on every path (the prefetch, then the stores: a step's or, before
    // the first step, as many dummy stores to a per-block slot), so the wait for
    // the prefetched pixels counts the stores instead of draining them.
    constexpr int WF_ = W / 2 + 1, KP_ = (WF_ + 1) / 2, NSO_ = (4 * KP_ + T - 1) / T;
    {
        // a scratch run just past the tiles (inter_elems: 1024 elements of slack)
        double2* slot = inter + (size_t)P * ct_row_stride(W) + (blockIdx.x & 63) * NSO_;
#pragma unroll
        for (int j = 0; j < NSO_; j++)
            if ((4 * KP_) % T == 0 || tid + j * T < 4 * KP_) slot[j] = make_double2(0.0, 0.0);
    }
    auto step = [&]() __attribute__((always_inline)) {
        const int y0 = 2 * pr;
        const bool two = y0 + 1 < H;
#pragma unroll
        for (int j = 0; j < K::LR; j++) {
            const int g = tid + j * T;
            if (K::G4 % T == 0 || g < K::G4) {
                double2 z[4];
                // the swizzle on the bytes: pixel e of w0 / w1 is pixel (e + rot) & 3,
                // stored to its own slot.  (Round 6: 41.1-41.2 us against 42.2-42.7
                // for selecting the rotated values as doubles, 48 v_cndmask per
                // group, and 42.0-42.7 without a swizzle; profiles/r06/
                // row_swizzle_ab.log)
                const u32x3a w0 = rot_px(rg[j][0], rot), w1 = rot_px(rg[j][1], rot);
#pragma unroll
                for (int e = 0; e < 4; e++) {
                    // rgb2pgm (src/image_processing.c:509) with k/255 folded into the
                    // weights (within 2 ulp); remove_dc_bias is the column pass's
                    const double p0 = kWr * byte_of(w0, 3 * e) + kWg * byte_of(w0, 3 * e + 1) +
                                      kWb * byte_of(w0, 3 * e + 2);
                    const double p1 = kWr * byte_of(w1, 3 * e) + kWg * byte_of(w1, 3 * e + 1) +
                                      kWb * byte_of(w1, 3 * e + 2);
                    z[e] = make_double2(p0, two ? p1 : 0.0);
                    // rsum (the blur-only path, which runs no K1): the channel sums
                    // of the column pass's DC bias, exact integers
                    if (rsum) {                                   // uniform
                        cs[0] += byte_of(w0, 3 * e) + (two ? byte_of(w1, 3 * e) : 0);
                        cs[1] += byte_of(w0, 3 * e + 1) + (two ? byte_of(w1, 3 * e + 1) : 0);
                        cs[2] += byte_of(w0, 3 * e + 2) + (two ? byte_of(w1, 3 * e + 2) : 0);
                    }
                }
#pragma unroll
                for (int e = 0; e < 4; e++) buf[4 * g + ((e + rot) & 3)] = z[e];
            }
        }
        // unconditional (past the last pair it re-reads this one): every path into
        // the loop head then has the same memory operations in flight
        int imn, prn;
        const bool next = item(s + 1, imn, prn);
        if (!(ablate & 4)) fetch(next ? imn : im, next ? prn : pr);
        __syncthreads();
        if (!(ablate & 1)) fft_lds<W, T, 1, Rs...>(buf, tw, tid);
        constexpr int WF = W / 2 + 1, KP = (WF + 1) / 2;
        // the pair's tile row, contiguous and 128-byte aligned (ct_row_stride):
        // thread i -> (column pair i/4, column k = 2(i/4) + (i/2)%2, row y0 +
        // i%2); the phantom column WF (odd WF) is 0 (a fixed, unrolled count per
        // thread, branch-free: the next step's wait for its prefetched pixels can
        // then count these stores exactly)
        // (round 6: one thread per column writing both rows' 32 contiguous bytes
        // -- half the LDS reads, no per-lane operand selects -- measured slower,
        // 44.6-45.8 against 42.3-42.7 us: its stores cover each 1 KB span in two
        // half-density instructions)
        // (ablation bit 8, timing builds: every block stores to one of 8 fixed
        // tile rows, so the stores stay L2-resident -- the row-pass FETCH study)
        double2* orow = inter + ((ablate & 8) ? (size_t)(blockIdx.x & 7) * ct_row_stride(W)
                                              : im * istride + (size_t)pr * ct_row_stride(W));
        constexpr int NSO = (4 * KP + T - 1) / T;
#pragma unroll
        for (int j = 0; j < NSO; j++) {
            const int i = tid + j * T;
            if ((4 * KP) % T == 0 || i < 4 * KP) {
                if (ablate & 2) continue;
                const int k = 2 * (i >> 2) + ((i >> 1) & 1);
                const bool second = i & 1;
                const int kk = k < WF ? k : 0;
                // first row: (Z[k] + conj Z[W-k]) / 2; second: (Z[k] - conj Z[W-k]) / 2i.
                // The lanes i, i + 1 (one column k) split the reads (round 6): the
                // even lane reads Z[k] as (A, B) = (x, y), the odd lane Z[W-k] with
                // its halves swapped, (A, B) = (y, x), and each takes its
                // partner's (A', B') by DPP.  Both rows are then re = (A + B') / 2,
                // im = (B - A') / 2 (first: Z[k].x + Z[W-k].x, Z[k].y - Z[W-k].y;
                // second: Z[W-k].y + Z[k].y, Z[W-k].x - Z[k].x): one b64 read pair
                // per element and no operand selects, where each lane read both Z
                // and selected its operands by row.
                const int e = second ? (kk == 0 ? 0 : W - kk) : kk;
                const double* zp = reinterpret_cast<const double*>(buf + e);
                const double A = zp[second ? 1 : 0], B = zp[second ? 0 : 1];
                const double Ap = dpp_pair_swap(A), Bp = dpp_pair_swap(B);
                const double f = (k < WF && (two || !second)) ? 0.5 : 0.0;   // 0: the phantom column / row
                orow[i] = make_double2(f * (A + Bp), f * (B - Ap));
            }
        }
        __syncthreads();
        s++;
        im = imn;
        pr = prn;
        live = next;
    };
    while (live) step();
    if (rsum) {
        // block sums through LDS (free after the last step's barrier), one atomic per channel
        unsigned long long* red = reinterpret_cast<unsigned long long*>(smem);
        unsigned long long w3[3];
#pragma unroll
        for (int c = 0; c < 3; c++) w3[c] = wave_sum((unsigned long long)cs[c]);
        if (lane_id() == 0)
#pragma unroll
            for (int c = 0; c < 3; c++) red[(tid >> 6) * 3 + c] = w3[c];
        __syncthreads();
        if (tid < 3) {
            unsigned long long t = 0;
            for (int w = 0; w < T / 64; w++) t += red[w * 3 + tid];
            if (t) atomicAdd(&rsum[tid], t);
        }
    }
}

// FULL: the full-prefetch form (p in an LDS array of its own), else the
// half-prefetch form (p in the lower half of the column buffer)
template <int H, int T, bool FULL, int... Rs>
struct ColK {
    using PL = Plan<H, T, 1, Rs...>;
    using L = typename PL::Last;
    static constexpr int R = Radices<Rs...>::count > 0 ? H / L::NB : 1;   // last radix
    static constexpr int NTW = tw_entries<1, Rs...>();
    static constexpr int P = (H + 1) / 2;                                 // row pairs
    static constexpr int CR = (2 * P + T - 1) / T;                        // load rounds
    static constexpr int E = (H + T - 1) / T;                             // epilogue run per thread
    // the run list of the block's column (ColRuns): kColRunsMax entries, RPT
    // per thread
    static constexpr int RPT = (kColRunsMax + T - 1) / T;
    // the column, the twiddles, log_mant's table, the column's run list and
    // one u64 slot per run (the bins are summed per run, then added to the
    // image's bins column by column: no LDS array of all na x nr bins)
    static constexpr size_t lds_base =
        sizeof(double2) * (H + NTW + kLogTab) + (sizeof(unsigned) + sizeof(unsigned long long)) * kColRunsMax;
    static_assert(Radices<Rs...>::product == H, "plan");
    static_assert(T % 2 == 0, "threads cover whole row pairs");
    static_assert(H % 2 == 0, "column plans: whole row pairs (the half-prefetch split)");
    // waves per SIMD of the launch bounds: sized for two resident blocks per
    // CU, one when the column and twiddles fill the LDS
    static constexpr int BPC1 = (int)((160 * 1024) / (sizeof(double2) * (H + NTW) + 1024)) < 2 ? 1 : 2;
    // (round 6: 3000 rows at 320 threads, three passes, needs three waves per
    // SIMD for two blocks, i.e. 168 VGPRs: 50-60 spilled; not pursued)
#ifdef PHD_COL_MINW3
    // (A/B build: the 3000-row half-prefetch form at three waves per SIMD,
    // three blocks per CU in its 54.2 KB of LDS; 168 VGPRs, ~66 spilled)
    static constexpr int MINW = (H == 3000 && !FULL) ? 3 : (T >= 512 ? 4 : (T >= 384 ? 3 : 2)) * BPC1 / 2;
#else
    static constexpr int MINW = (T >= 512 ? 4 : (T >= 384 ? 3 : 2)) * BPC1 / 2;
#endif
    // The next column streams into the column buffer by LDS-DMA (no
    // registers) while the current one finishes (round 5).
    //  * Full-prefetch form (PF): p per row gets an LDS array of its own, so
    //    the whole buffer is free once the last pass has read it and the
    //    whole next column is issued then -- where that fits beside as many
    //    blocks per CU as without it (3000 and 2000 rows: two; 6000: one;
    //    4000 rows would drop to one block and take the half form).
    //  * Half-prefetch form: p stays in the lower half of the buffer; the
    //    upper half streams in during the run walk, the lower half after
    //    it, beside the atomics.  No LDS beyond the register-staged form's it
    //    replaced (round 4), which measured slower in every configuration.
    static constexpr size_t lds_pf = lds_base + sizeof(double) * H;
    static constexpr bool PF = FULL && lds_pf * BPC1 <= 160 * 1024;
    static constexpr size_t lds = PF ? lds_pf : lds_base;
};

// One column per block: blocks b, b^8, b^16, b^24 (one XCD) take the four
// columns of the same 128-byte lines (two tiles), so each line is fetched once
// into that XCD's L2 (the grid is a multiple of 32).  The tiles of a step were
// issued as LDS-DMA during the previous step (ColK's forms; prefetching into
// registers measured slower in round 3: it cost VGPRs).
// One 16-byte LDS-DMA per lane: global g -> LDS at the wave's base + lane x 16
// (global_load_lds_dwordx4; M0 holds the wave-uniform LDS base).  Inline asm
// rather than the builtin: the compiler would make every later LDS read wait
// for the DMA (it cannot tell the regions apart), draining the prefetch at
// the epilogue's first read; the kernel waits for it itself (vmcnt, then a
// barrier) before the buffer is read.
__device__ __forceinline__ void lds_dma16(const void* g, void* lds_wave_base) {
#if defined(__HIP_DEVICE_COMPILE__)
    const unsigned m = __builtin_amdgcn_readfirstlane(
        (unsigned)(uintptr_t)(__attribute__((address_space(3))) void*)lds_wave_base);
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(g), "s"(m)
                 : "memory");
#else
    (void)g;
    (void)lds_wave_base;
#endif
}

// every vector memory operation of the wave done (vmcnt(0); expcnt, lgkmcnt
// left alone): a DMA-filled buffer may be read after this and a barrier
__device__ __forceinline__ void wait_vmem() { __builtin_amdgcn_s_waitcnt(0x0F70); }

template <int H, int T, bool FULL, int... Rs>
__global__ __launch_bounds__(T, (ColK<H, T, FULL, Rs...>::MINW)) void k_cols_ct(const double2* __restrict__ inter0, int wf,
                                                     const unsigned* __restrict__ runs,
                                                     const unsigned* __restrict__ segidx, int rstride,
                                                     unsigned long long* __restrict__ bin_sums0, double* __restrict__ fmax_part0,
                                                     const double2* __restrict__ twg,
                                                     const unsigned long long* __restrict__ sums0, int width,
                                                     double* __restrict__ dbg, double bscale, int ablate_arg,
                                                     int nimg, long istride, long bstride, long fstride, long sstride) {
    using K = ColK<H, T, FULL, Rs...>;
    const int ablate = PHD_ABL(ablate_arg);
    using L = typename K::L;
    constexpr int R = K::R;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    double2* buf = reinterpret_cast<double2*>(smem);          // [H]
    double2* tw = buf + H;
    double2* lt = tw + K::NTW;                                 // log_mant's table
    unsigned long long* sl = reinterpret_cast<unsigned long long*>(lt + kLogTab);   // [kColRunsMax]
    unsigned* rl = reinterpret_cast<unsigned*>(sl + kColRunsMax);                   // [kColRunsMax]
    // p per spectrum row: its own array in the full-prefetch form, else the
    // lower half of the column buffer (free once the last pass has read it)
    double* lgb = K::PF ? reinterpret_cast<double*>(rl + kColRunsMax) : reinterpret_cast<double*>(buf);
    const int tid = threadIdx.x;
    // a batch: nimg images of one size, their intermediates, bin sums, max
    // partials and channel sums istride / bstride / fstride / sstride apart;
    // each block runs its columns of every image in turn
    const double2* inter = inter0;
    unsigned long long* bin_sums = bin_sums0;
    double* fmax_part = fmax_part0;
    const unsigned long long* sums = sums0;
    // blocks b, b^8, b^16, b^24 (one XCD) take the four columns of a 128-byte
    // line (two tiles), so each line is fetched once into that L2
    const int quad = (int)((blockIdx.x >> 3) & 3);
    const int half = quad & 1;                                 // column of the pair
    for (int i = tid; i < K::NTW; i += T) tw[i] = twg[i];
    for (int i = tid; i < kColRunsMax; i += T) sl[i] = 0ull;
    log_table_init(lt, tid, T);
    const int kpn = (wf + 1) / 2;
    const size_t rs = (size_t)((4 * kpn + 7) & ~7);           // row-pair stride (ct_row_stride)
    const int nunit = (kpn + 1) / 2;                          // tile pairs (128-byte lines)
    const int nlog = (int)gridDim.x / 4;
    const int lblk = (int)((blockIdx.x >> 5) * 8 + (blockIdx.x & 7));
    // a batch numbers its images' units one after the other: a block's range
    // may span the end of one image and the start of the next (small images)
    const long nall = (long)nimg * nunit;
    const int c0 = (int)(lblk * nall / nlog), c1 = (int)((lblk + 1) * nall / nlog);
    // the column pair of step u (tile 2u or 2u+1; past the last tile the block
    // re-reads the last one and idles)
    auto pair_at = [&](int u) { return min(2 * u + (quad >> 1), kpn - 1); };
    // the tiles: element 4p + 2c + r is (row 2p + r, column 2kp + c); a thread
    // loads its column's 32-B half of tiles (row pair tid/2, row tid%2), as raw
    // 16-byte words that land in the registers the LDS stores read
    const int prow0 = tid / 2, psub = 2 * half + (tid & 1);
    // the column of step u into the buffer by LDS-DMA (PF): element 2 prow0 +
    // (tid & 1) + c T is lane-linear, the wave's base + lane x 16 B
    // part 0: the whole column; 1: its upper half (buffer elements >= H / 2,
    // free while p sits in the lower half), 2: the lower half
    auto dma = [&](int u, int part) {
        const u32x4* src = reinterpret_cast<const u32x4*>(inter) + (size_t)prow0 * rs + (size_t)pair_at(u) * 4 + psub;
#pragma unroll 1
        for (int c = 0; c < K::CR; c++) {
            const int pr = min(c * (T / 2), K::P - 1 - prow0);
            const int y = 2 * (prow0 + c * (T / 2)) + (psub & 1);
            if (((2 * K::P) % T == 0 || tid + c * T < 2 * K::P) && (H % 2 == 0 || y < H) &&
                (part == 0 || (part == 1) == (tid + c * T >= H / 2)))
                lds_dma16(src + (size_t)pr * rs, buf + (tid & ~63) + c * T);
        }
    };
    // (ablation bit 32, timing builds: the prefetch form loads each column at
    // its own step instead, i.e. synchronously)
    const bool pf_late = (ablate & 32) != 0;
    // (a block without units still runs one empty segment: its max partial and
    // bins are written as the one-image form always did)
    for (int seg = c0, im = c0 / nunit, first = 1; first || seg < c1; im++, first = 0) {
    // this image's units in the block's range: [u0, un) of image im
    const int u0 = seg - im * nunit, un = min(c1 - im * nunit, nunit);
    seg = im * nunit + un;
    inter = inter0 + im * istride;
    bin_sums = bin_sums0 + im * bstride;
    fmax_part = fmax_part0 + im * fstride;
    sums = sums0 + im * sstride;
    double mx = 0.0;
    __syncthreads();
    if (u0 < un && !pf_late) dma(u0, 0);
    for (int u = u0; u < un; u++) {
        const int kp = pair_at(u);
        if (pf_late) dma(u, 0);
        wait_vmem();                              // this wave's DMA of the column is in LDS
        const int col = 2 * (2 * u + (quad >> 1)) + half;
        const bool live = col < wf;                       // the phantom column of an odd wf idles
        // the column's bin runs (image-independent, ~0.3 KB per column; ColRuns)
        // and this thread's segment word (walk_runs): loaded now, the list stored
        // to LDS after the FFT (a phantom column reads column 0's: its p are 1)
        unsigned rreg[K::RPT];
        unsigned sidx;
        {
            const int rc = live ? col : 0;
            const unsigned* rsrc = runs + (size_t)rc * rstride;
#pragma unroll
            for (int k = 0; k < K::RPT; k++) {
                const int e = tid + k * T;
                rreg[k] = e < rstride ? rsrc[e] : 0u;
            }
            sidx = segidx[(size_t)rc * T + tid];
        }
        __syncthreads();
        if (kp == 0) {                                    // block-uniform
            // remove_dc_bias (src/blur_profile.c:233-238): a constant per image only
            // moves the row spectra's k = 0 column, by W * avg per row, with avg =
            // (Br + Bg + Bb) / 3 (src/interface.c:78) from K1's exact channel sums
            if (col == 0) {
                const double n = (double)H * (double)width;
                const double avg = ((double)sums[0] / 255.0 / n + (double)sums[1] / 255.0 / n +
                                    (double)sums[2] / 255.0 / n) / 3.0;
                const double dc = (double)width * avg;
                for (int y = tid; y < H; y += T) buf[y].x -= dc;
            }
            __syncthreads();
        }
        if (!(ablate & 1)) K::PL::all_but_last(buf, tw, tid);
        double2 v[L::ROUNDS][R];
        if (!(ablate & 16)) {
            L::load(buf, v, tid);
            L::compute(v, tw + K::PL::last_tw_offset, tid);
        }
        // Full form: nothing waits for the buffer after the last pass's reads, so
        // p, the run list and the barrier come first and the whole next column
        // is issued behind them (the walk and the atomics run while it lands).
        // Half form: a barrier first (p then overwrites the lower half), the
        // upper half issued behind the next barrier, the lower after the walk.
        if (!K::PF) __syncthreads();               // every thread has read its last-pass inputs
        // lgb: p per spectrum row, 1 for p < 1 (log 0)
#pragma unroll
        for (int q = 0; q < L::ROUNDS; q++) {
            const int b = tid + q * T;
            if (L::active(b) && !(ablate & 16)) {
#pragma unroll
                for (int k = 0; k < R; k++) {
                    const double2 X = v[q][k];
                    const double p = X.x * X.x + X.y * X.y;          // src/fft_processing.c:49
                    if (live) mx = fmax(mx, p);
                    if (dbg && live) dbg[(size_t)col * H + b + k * L::NB] = p;
                    lgb[b + k * L::NB] = (live && p >= 1) ? p : 1.0;   // src/fft_processing.c:197-198
                }
            }
        }
#pragma unroll
        for (int k = 0; k < K::RPT; k++)
            if (tid + k * T < kColRunsMax) rl[tid + k * T] = rreg[k];
        // PF: the run loads (and any debug stores) retire before a DMA is in
        // flight, so no later wait of the compiler's counts the DMA
        wait_vmem();
        __syncthreads();
        if (u + 1 < un && !pf_late) dma(u + 1, K::PF ? 0 : 1);
        // contiguous runs of one bin: one LDS atomic per run (bins change every
        // few tens of rows along a column; walk_runs)
        if (!(ablate & 2)) walk_runs<K::E, H % K::E == 0>(lgb, tid * K::E, H, rl, sidx, sl, bscale, lt);
        __syncthreads();
        if (!K::PF && u + 1 < un && !pf_late) dma(u + 1, 2);   // p is read: the lower half too
        // the column's run sums into the image's bins (a bin met by two runs of
        // a column gets two atomics); entries past the sentinel start at H
        if (!(ablate & 8)) {
#pragma unroll
            for (int k = 0; k < K::RPT; k++) {
                const int t = tid + k * T;
                if (t < kColRunsMax && t < rstride) {
                    const unsigned e = rl[t];
                    const unsigned long long v = sl[t];
                    if ((int)(e >> 16) < H && v) {
                        sl[t] = 0ull;
                        atomicAdd(&bin_sums[e & 0xFFFFu], v);
                    }
                }
            }
        }
    }
    // block max -> one partial per block
    mx = wave_max(mx);
    double* red = reinterpret_cast<double*>(buf);
    if (lane_id() == 0) red[tid >> 6] = mx;
    __syncthreads();
    if (tid == 0) {
        double m = 0.0;
        for (int w = 0; w < (T + 63) / 64; w++) m = fmax(m, red[w]);
        fmax_part[blockIdx.x] = m;
    }
    if (seg < c1) __syncthreads();                             // red (in the buffer) is reused
    }
}

template <typename K>
void allow_big_lds(K kernel) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kernel), hipFuncAttributeMaxDynamicSharedMemorySize,
                              160 * 1024);
}

// resident blocks per CU x CUs (the persistent grids)
template <typename K>
int resident_grid(K kernel, int threads, size_t lds) {
    allow_big_lds(kernel);
    int nb = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, kernel, threads, lds) != hipSuccess || nb < 1) nb = 1;
    return nb * num_cus();
}

// (timing builds: PHD_COL_BPC / PHD_ROW_BPC cap the persistent grids' blocks
// per CU, so that two lanes' FFT passes can share the CUs -- the co-residency
// study of round 6)
static int bpc_cap(const char* knob, int g) {
    const char* v = phd_knob(knob);
    if (!v || atoi(v) < 1) return g;
    return std::min(g, atoi(v) * num_cus());
}

template <int W, int T, int... Rs>
hipError_t rows_ct(const uint8_t* img, int H, const unsigned long long* sums, const double* k255,
                   const double2* tw, double2* inter, unsigned long long* rsum, hipStream_t st,
                   const uint8_t* const* imgs = nullptr, int nimg = 1, long istride = 0) {
    const size_t lds = RowK<W, T, Rs...>::lds;
    static const int grid = [&] {
        const int g = bpc_cap("PHD_ROW_BPC", resident_grid(k_rows_ct<W, T, Rs...>, T, lds)) / 32 * 32;   // % 32
        return g > 32 ? g : 32;
    }();
    phd_launch((k_rows_ct<W, T, Rs...>), dim3(grid), dim3(T), lds, st, img, H, sums, k255, tw, inter,
               g_ablate, rsum, imgs, nimg, istride);
    return hipGetLastError();
}

template <int H, int T, bool PF, int... Rs>
int cols_grid_form() {
    const int g = bpc_cap("PHD_COL_BPC", resident_grid(k_cols_ct<H, T, PF, Rs...>, T, ColK<H, T, PF, Rs...>::lds)) /
                  32 * 32;   // XCD quads
    return g < 32 ? 32 : g;
}

// the max partials per image: the larger of the two forms' grids (a form with
// fewer blocks leaves its slots at the workspace's zero)
template <int H, int T, int... Rs>
int cols_grid() {
    static const int g = [] {
        int a = cols_grid_form<H, T, false, Rs...>();
        if constexpr (ColK<H, T, true, Rs...>::PF) a = std::max(a, cols_grid_form<H, T, true, Rs...>());
        return a;
    }();
    return g;
}

template <int H, int T, bool PF, int... Rs>
hipError_t cols_ct_form(const double2* inter, int width, int wf, const ColBins& cb, unsigned long long* bin_sums,
                        double* fmax_part, const double2* tw, const unsigned long long* sums, double* dbg,
                        hipStream_t st, int nimg, long istride, long bstride, long fstride, long sstride) {
    static const int grid = cols_grid_form<H, T, PF, Rs...>();
    phd_launch((k_cols_ct<H, T, PF, Rs...>), dim3(grid), dim3(T), ColK<H, T, PF, Rs...>::lds, st, inter, wf,
               cb.runs, cb.seg, cb.rstride, bin_sums, fmax_part, tw, sums, width, dbg, bin_scale(H, wf), g_ablate,
               nimg, istride, bstride, fstride, sstride);
    return hipGetLastError();
}

// pf: the full-prefetch form where the plan has one (FftSel::col_pf), else
// the half-prefetch form
template <int H, int T, int... Rs>
hipError_t cols_ct(const double2* inter, int width, int wf, const ColBins& cb, unsigned long long* bin_sums,
                   double* fmax_part, const double2* tw, const unsigned long long* sums, double* dbg,
                   hipStream_t st, bool pf, int nimg = 1, long istride = 0, long bstride = 0, long fstride = 0,
                   long sstride = 0) {
    if constexpr (ColK<H, T, true, Rs...>::PF) {
        if (pf)
            return cols_ct_form<H, T, true, Rs...>(inter, width, wf, cb, bin_sums, fmax_part, tw, sums, dbg, st,
                                                   nimg, istride, bstride, fstride, sstride);
    }
    return cols_ct_form<H, T, false, Rs...>(inter, width, wf, cb, bin_sums, fmax_part, tw, sums, dbg, st, nimg,
                                            istride, bstride, fstride, sstride);
}

// log_mant over an array (tests: its accuracy against the host's log)
__global__ __launch_bounds__(256) void k_log_mant(const double* __restrict__ x, double* __restrict__ y, long n) {
    __shared__ double2 lt[kLogTab];
    log_table_init(lt, threadIdx.x, 256);
    __syncthreads();
    const long i = (long)blockIdx.x * 256 + threadIdx.x;
    if (i < n) y[i] = log_mant(x[i], lt);
}

}  // namespace

hipError_t launch_log_mant(const double* x, double* y, long n, hipStream_t st) {
    if (n <= 0) return hipSuccess;
    phd_launch(k_log_mant, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, x, y, n);
    return hipGetLastError();
}

bool ct_rows_plan(int w, std::vector<int>* radices) {
#define PHD_X(N, T, ...)                                       \
    if (w == N) {                                              \
        if (radices) *radices = std::vector<int>{__VA_ARGS__}; \
        return true;                                           \
    }
    PHD_CT_ROWS(PHD_X)
#undef PHD_X
    return false;
}

bool ct_cols_plan(int h, std::vector<int>* radices) {
#define PHD_X(N, T, ...)                                       \
    if (h == N) {                                              \
        if (radices) *radices = std::vector<int>{__VA_ARGS__}; \
        return true;                                           \
    }
    PHD_CT_COLS(PHD_X)
#undef PHD_X
    return false;
}

int fft_cols_ct_threads(int h) {
#define PHD_X(N, T, ...) \
    if (h == N) return T;
    PHD_CT_COLS(PHD_X)
#undef PHD_X
    return 0;
}

size_t fft_cols_ct_lds(int h) {
#define PHD_X(N, T, ...) \
    if (h == N) return ColK<N, T, false, __VA_ARGS__>::lds;
    PHD_CT_COLS(PHD_X)
#undef PHD_X
    return 0;
}

int fft_cols_ct_blocks(int h) {
#define PHD_X(N, T, ...) \
    if (h == N) return cols_grid<N, T, __VA_ARGS__>();
    PHD_CT_COLS(PHD_X)
#undef PHD_X
    return 0;
}

hipError_t launch_fft_rows_ct(const uint8_t* img, int height, int width, const unsigned long long* sums,
                              const double* k255, const double2* tw, double2* inter, hipStream_t st,
                              unsigned long long* rsum) {
#define PHD_X(N, T, ...) \
    if (width == N) return rows_ct<N, T, __VA_ARGS__>(img, height, sums, k255, tw, inter, rsum, st);
    PHD_CT_ROWS(PHD_X)
#undef PHD_X
    return hipErrorInvalidValue;
}

hipError_t launch_fft_rows_ct_batch(const uint8_t* const* d_imgs, int n, int height, int width, const double* k255,
                                    const double2* tw, double2* inter, long inter_stride, hipStream_t st) {
    if (n < 1 || ((height + 1) / 2) % 4 != 0) return hipErrorInvalidValue;   // whole line groups per image
#define PHD_X(N, T, ...)                                                                              \
    if (width == N)                                                                                   \
        return rows_ct<N, T, __VA_ARGS__>(nullptr, height, nullptr, k255, tw, inter, nullptr, st, d_imgs, n, \
                                          inter_stride);
    PHD_CT_ROWS(PHD_X)
#undef PHD_X
    return hipErrorInvalidValue;
}

hipError_t launch_fft_cols_ct_batch(const double2* inter, long inter_stride, int n, int height, int width, int wf,
                                    const ColBins& cb, unsigned long long* bin_sums, long bin_stride,
                                    double* fmax_part, long fmax_stride, const double2* tw,
                                    const unsigned long long* sums, long sums_stride, hipStream_t st, bool pf) {
    if (n < 1) return hipErrorInvalidValue;
#define PHD_X(N, T, ...)                                                                                       \
    if (height == N)                                                                                           \
        return cols_ct<N, T, __VA_ARGS__>(inter, width, wf, cb, bin_sums, fmax_part, tw, sums, nullptr, st, pf, n, \
                                          inter_stride, bin_stride, fmax_stride, sums_stride);
    PHD_CT_COLS(PHD_X)
#undef PHD_X
    return hipErrorInvalidValue;
}

hipError_t launch_fft_cols_ct(const double2* inter, int height, int width, int wf, const ColBins& cb,
                              unsigned long long* bin_sums, double* fmax_part, const double2* tw,
                              const unsigned long long* sums, double* dbg, hipStream_t st, bool pf) {
#define PHD_X(N, T, ...) \
    if (height == N)     \
        return cols_ct<N, T, __VA_ARGS__>(inter, width, wf, cb, bin_sums, fmax_part, tw, sums, dbg, st, pf);
    PHD_CT_COLS(PHD_X)
#undef PHD_X
    return hipErrorInvalidValue;
}

}  // namespace phd
