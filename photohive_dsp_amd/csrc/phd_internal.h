// phd_internal.h -- shared between the host C++ (phd_*.cpp) and the HIP kernels
// (*.hip).  Plain POD types and launcher declarations only.
#pragma once

#include <hip/hip_runtime_api.h>
#include <stddef.h>
#include <stdint.h>
#include <stdlib.h>

#include <vector>

namespace phd {

// Experiment switches (PHD_* variables of the timing experiments recorded in
// alternate schedules, measured-and-rejected kernel forms, ablation
// masks).  Only the timing build (`make -C photohive_dsp_amd/csrc ablate`,
// PHD_ABLATE_BUILD) reads them; the production library never looks at the
// environment for them and always takes the default.
inline const char* phd_knob(const char* name) {
#ifdef PHD_ABLATE_BUILD
    return getenv(name);
#else
    (void)name;
    return nullptr;
#endif
}

// Events that the next profiled launch records as part of its own dispatch
// (hipExtLaunchKernel: the kernel's start and end, no event packets between
// back-to-back kernels).  KernelProfiler::begin sets them; phd_launch uses
// them once.
struct LaunchEvents {
    hipEvent_t start = nullptr, stop = nullptr;
    bool used = false;
};
LaunchEvents& launch_events();   // thread-local


// Pixels per palette chunk: the unit of work of the hsv/stats kernel and the
// palette-sums kernel, and the granularity of the per-chunk group histograms
// the tie-overflow cutoff search walks (counts fit uint16).
constexpr int kChunk = 16384;
constexpr int kThreads = 256;
// Largest FFT length kept resident in LDS (complex fp64, 16 B/element).
constexpr int kFftMaxLds = 8192;
constexpr int kMaxFftPasses = 24;
// Largest prime radix the LDS transforms take as an O(R) direct-DFT pass;
// lengths with a larger prime factor go through Bluestein (fft_global.hip).
constexpr int kMaxDirectPrime = 61;
// Polar-bin sums of log(p) are accumulated as unsigned 64-bit fixed point
// (value * bin_scale): integer additions commute, so the bins -- and the
// strict threshold comparisons vectorize_blur_profile makes on them -- are the
// same on every run whatever order the atomics land in.  The scale is the
// largest power of two that keeps any bin of an H x Wf half spectrum below
// 2^62: |X| <= N * M with M >= |pgm - avg| (M = 1 for RGB8 images, whose luma
// lies in [0, 1]; the planar path passes its luma range), so log p <= 2 ln(N M)
// and a bin holds at most H * Wf elements (2^-35 per element at 4000x3000,
// 2^-41 at 640x480; 2^-30 at the reference's 120 MP limit).
inline double bin_scale(int height, int wf, double lrange = 1.0) {
    const double n = (double)height * (2.0 * wf);
    const double m = lrange > 1.0 ? lrange : 1.0;
    const double bound = (double)height * wf * 2.0 * (__builtin_log(n > 2.0 ? n : 2.0) + __builtin_log(m)) + 1.0;
    return __builtin_ldexp(1.0, 62 - (int)__builtin_ceil(__builtin_log2(bound)));
}

// The HSV grid of initialize_octree (src/color_quantization.c:22-101).
struct GridParams {
    int hp, sp, vp, ng, tl;
    double Lh, Ls, Lv, bt, gt;
};

// Exact pixel classification (phd_device.h: classify) from tables built on the
// host with the reference's own double expressions (make_class_tables) plus an
// exact integer form of the hue bin.  Only pixels whose hue lies exactly on a
// bin edge (where the reference's double rounding decides) take the fp64 path.
struct FastCls {
    int lh;                    // Lh = 360 / h_partitions (integer division, :41)
    int use_thr;               // Si from ClsEnt::thr (s_partitions <= 6), else si8 in global memory
    int k1t_cshift = -1;       // >= 0: the table K1 (k1.hip) runs this grid (its accumulator layout, k1_cfg)
    int k1t_cshift2 = -1;      // ... as two 512-thread blocks per CU (triangular code table): its layout, else -1
};
// Si is non-decreasing in kd = kmax - kmin for a fixed kmax (s = d / max is), so
// it is -1 plus the number of thresholds kd reaches.
constexpr int kSiThresholds = 6;
struct ClsEnt {                // per max channel value k (16 B: one LDS read per pixel)
    int vpack;                 // low 16 bits (signed): Vi of v(k), -1 when v < black_thresh;
                               // high 16 bits: gray group id of v(k)
    unsigned thr[3];           // u16 j (low half of thr[j/2] for even j): the smallest kd with
                               // Si >= j, 0xFFFF = never (j < kSiThresholds)
};
struct ClassTables {           // device copy; ent is staged into LDS by the kernels
    ClsEnt ent[256];
    signed char si8[256 * 256];   // [kmax][kmax - kmin]: Si of s, -1 when s < gray_thresh
    // the table K1 (k1.hip) classifies with: per (kmax, kd <= kmax) a code
    // (u8) for everything arm_octree decides without the hue -- the colour
    // group's (Si, Vi) as Si * vp + Vi, else sp * vp + (gray / black group -
    // gray_start)
    unsigned char code8[256 * 256];
    unsigned char code_tri[256 * 257 / 2];   // the same codes, kd <= kmax only: [kmax (kmax + 1) / 2 + kd]
    double inv[256];              // 1.0 / k (inv[0] = 0)
    int codes_ok;                 // every (kmax, kd) got a code (sp * vp + ng + 1 <= 256)
};

// Per-image device workspace views used by the palette kernels.
struct PaletteDev {
    unsigned long long* sums;     // [6] sum k_r, k_g, k_b, k_r^2, k_g^2, k_b^2 (full image)
    double* s_part;               // [nchunks] per-chunk sum of HSV saturation
    unsigned* hist;               // [TL] group quantities
    unsigned short* chunk_hist;   // [nchunks][TL]
    double* gsum = nullptr;       // fused K1: [3][TL] sum h, sum s, sum v per group
    unsigned* gcell = nullptr;    // fused K1: [HueCells::count] pixels per (group, hue cell)
    unsigned long long* kd_sum = nullptr;   // statistics pass (stats.hip mode 3): [256] sum of
                                            // max - min over the pixels of each max value
};

// Hue cells of the fused palette pass.  calculate_avg_hsv
// (src/color_quantization.c:527-547) adds off = 180 - h_parent to each hue and
// wraps by 360 when the result leaves [0, 360]: with Lh = 360 / h_parts, the
// thresholds h_parent +- 180 (and 180 for grey / black parents, h = 0) all
// lie on the half-bin grid B_c = c * Lh / 2.  So the number of a group's
// pixels that wrap for ANY parent is a sum of its counts per half-bin cell
// [B_c, B_c+1).  A colour group (hue bin j) only holds hues in
// [B_2j, B_2j+2]: 4 cells, global c = 2j - 1 + l; a grey or black group holds
// any hue: 2 * h_parts cells.  Pixels exactly on a threshold are put on the
// side the reference's double comparison puts them (classify_f / fused_exact).
struct HueCells {
    __host__ __device__ static int gray_start(const GridParams& g) { return g.tl - g.ng - 1; }
    __host__ __device__ static int count(const GridParams& g) {
        return 4 * gray_start(g) + (g.ng + 1) * 2 * g.hp;
    }
};

// Keep rule of one octree group after group_irregular_pixels.
struct GroupRule {
    int slot;            // palette slot (index into valid_parents) or -1 = dropped
    int partial;         // 0: every pixel kept; 1: first `keep` pixels (+ last if dangle)
    int keep;            // pixels kept in raster order (partial only)
    int dangle;          // the group's last pixel survives as a dangling node
    unsigned cutoff;     // raster index bound: kept iff idx < cutoff (filled on device)
    unsigned last;       // raster index of the group's last pixel (filled on device)
};

// A mixed-radix FFT plan for one length.  Twiddles W_n^e = exp(-2 pi i e/n)
// come from two small tables (e = 64*hi + lo) that each block stages in LDS;
// the full table is only used by the generic-radix pass.
struct FftPlan {
    int n;
    int npass;
    int generic;               // some radix is outside {2,3,4,5,6,8,9,10,12,16}
    int composite;             // some radix is 6, 9, 10, 12 or 16 (image-pass plans only)
    int n_hi;                  // entries of tw_hi = ceil(n / 64)
    int radix[kMaxFftPasses];
    const double2* tw;         // device: tw[t] = W_n^t, t in [0, n)
    const double2* tw_lo;      // device: W_n^t, t in [0, 64)
    const double2* tw_hi;      // device: W_n^(64 t), t in [0, n_hi)
};

// ---- launchers (kernels in *.hip) ------------------------------------------
extern int g_ablate;   // ablation mask read by kernels under phd_debug_time_kernel
int env_ablate();      // PHD_ABLATE (timing builds only)
int num_cus();         // compute units of the current device
// K1's two-block form: blocks per CU (2; 1 when this call runs split over two
// lanes, so a K1 launch leaves half of every CU to the other lane's FFT
// blocks: 7.89k against 7.66k images/s with two lanes, and 6.78k against
// 7.07k with one, where K1 runs alone; PHD_K1_BPC overrides)
int k1_blocks_per_cu();
// Scope guard: the calling thread's current call runs on n lanes (on_lanes)
struct CallLanes {
    explicit CallLanes(int n);
    ~CallLanes();
    CallLanes(const CallLanes&) = delete;
    CallLanes& operator=(const CallLanes&) = delete;
    int prev_;
};
// hsv/stats/histogram pass over one image (K1).  ds = downsample rate.
// K1 over a batch of same-size images (ds == 1); d_imgs is a device array of
// n image pointers; image i's records sit at out0 + i * a_stride (sums, hist,
// s_part) and out0.chunk_hist + i * h_stride bytes.  hist == false computes
// only the moments and sum(s) (the rgb2hsv + statistics pass).  sums (needs
// hist and fused_palette_ok): also the per-group hsv sums and hue-cell counts
// (out0.gsum / out0.gcell, every a_stride bytes).  aligned: every image
// pointer is 4-byte aligned (word loads; else byte loads).
hipError_t launch_hsv_stats_batch(const uint8_t* const* d_imgs, int n, int height, int width,
                                  const GridParams& gp, const FastCls& fc, const ClassTables* tabs,
                                  const PaletteDev& out0, long a_stride, long h_stride, int nchunks,
                                  const double* k255, bool hist, bool sums, bool aligned, hipStream_t st);
// The rgb2hsv + statistics pass alone (moments and sum(s), no histogram) over
// a batch of 4-byte-aligned images: stats.hip (out0.sums, out0.s_part).
hipError_t launch_rgb_stats_batch(const uint8_t* const* d_imgs, int n, int height, int width, const PaletteDev& out0,
                                  long a_stride, int nchunks, hipStream_t st);
// The statistics batch's per-image finish (stats.hip): from n A records
// (a_stride apart: six u64 moments, chunk s partials at s_off, 256 sums of d
// per max value at kd_off) to out[8 i ..]: the moments, then sum(s) / npix.
hipError_t launch_stats_finish(const uint8_t* rec, int n, long a_stride, long s_off, long kd_off, int nchunks,
                               long npix, unsigned long long* out, hipStream_t st);
// The fused K1 of k1.hip (table classification, packed counts): cshift of its
// lane-private copies, or -1 when this grid does not fit it (palette.hip's
// fused K1 then runs).
int k1t_cshift(const GridParams& gp, const ClassTables& host_tabs);
int k1t_cshift2(const GridParams& gp, const ClassTables& host_tabs);
hipError_t launch_k1t_batch(const uint8_t* const* d_imgs, int n, int height, int width, const GridParams& gp,
                            const ClassTables* tabs, const PaletteDev& out0, long a_stride, long h_stride,
                            int nchunks, const double* k255, int cshift, int cshift2, hipStream_t st);
// K1's per-pixel classification (k1_pixel.h) run on the host: hue cell, h, s
// and whether the pixel took the deferred (exact double) path; -1 when the
// grid has no code table.
int k1_host_pixels(const GridParams& gp, const ClassTables& t, const uint8_t* rgb, long n, int* cell, double* h,
                   double* s, int* deferred);
// The fused K1's LDS fits this grid (else the palette uses K1 + K3).
bool fused_palette_ok(const GridParams& gp);
// Fused palette: the slot sums of the partial (tie-overflow) groups, added
// into out0 (every c_stride bytes) after Kcut filled their cutoff / last.
// entries: (image, group), image-major; max_per_image: the most entries of
// one image (one prefix walk per image when small, else one per entry).
hipError_t launch_partial_sums_batch(const uint8_t* const* d_imgs, const uint8_t* const* h_imgs, int n,
                                     int height, int width, const GridParams& gp, const FastCls& fc,
                                     const ClassTables* tabs, const double* k255, const int2* entries,
                                     int n_entries, const unsigned short* chunk_hist0, long h_stride,
                                     const GroupRule* rules0, const double* off0, long b_stride, double* out0,
                                     long c_stride, int max_per_image, hipStream_t st);
// Kcut and K3 over a batch (ds == 1): entries = (image, group) pairs needing a
// cutoff search; B records (rules at rules0, slot offsets at off0) every
// b_stride bytes; palette sums at out0 every c_stride bytes.  h_imgs: the same
// image pointers on the host (alignment check).
hipError_t launch_cutoffs_batch(const uint8_t* const* d_imgs, const uint8_t* const* h_imgs, int n, int height,
                                int width, const GridParams& gp, const FastCls& fc, const ClassTables* tabs,
                                const double* k255, const int2* entries, int n_entries,
                                const unsigned short* chunk_hist0, long h_stride, GroupRule* rules0,
                                long b_stride, hipStream_t st);
size_t palette_sums_b_lds(int tl, int max_slots);
hipError_t launch_palette_sums_batch(const uint8_t* const* d_imgs, const uint8_t* const* h_imgs, int n,
                                     int height, int width, const GridParams& gp, const FastCls& fc,
                                     const ClassTables* tabs, const double* k255, const GroupRule* rules0,
                                     const double* off0, long b_stride, const int* nslots_img, int max_slots,
                                     double* out0, long c_stride, hipStream_t st);
// K1 for downsample_rate > 1 (one image).
hipError_t launch_hsv_ds(const uint8_t* img, int height, int width, int ds, const GridParams& gp,
                         const FastCls& fc, const ClassTables* tabs, const PaletteDev& out, int nchunks,
                         const double* k255, hipStream_t st);
// Locate the keep cutoff / last pixel for groups with rule.partial (Kcut).
hipError_t launch_palette_cutoffs(const uint8_t* img, int height, int width, int ds,
                                  const GridParams& gp, const unsigned short* chunk_hist,
                                  int nchunks, GroupRule* rules, const int* search_groups,
                                  int n_search, const double* k255, hipStream_t st);
// Per-slot sums over kept pixels (K3): out[slot*4 + {0,1,2,3}] = sum wrap(h+off), s, v, n.
hipError_t launch_palette_sums(const uint8_t* img, int height, int width, int ds,
                               const GridParams& gp, const GroupRule* rules,
                               const double* slot_off, int nslots, double* out,
                               const double* k255, hipStream_t st);
// Row pass: luma - avg of two rows as one complex sequence, FFT, split, write
// the half spectra column-major into inter[wf][height].
// Runtime-plan FFT passes over a batch of same-size images in one launch each
// (grid.y = image): image y's pixels d_imgs[y] (device array), channel sums
// at sums0 + y * sums_stride, intermediate at inter0 + y * inter_stride
// elements; the column pass's bin sums and max partials at + y * out_stride
// doubles.
hipError_t launch_fft_rows_batch(const uint8_t* const* d_imgs, int n, int height, int width, const FftPlan& plan,
                                 const unsigned long long* sums0, long sums_stride, const double* k255,
                                 double2* inter0, size_t inter_stride, hipStream_t st);
hipError_t launch_fft_cols_batch(const double2* inter0, size_t inter_stride, int n, int height, int wf,
                                 const FftPlan& plan, const uint16_t* binmap, int nbins, unsigned long long* bin_sums0,
                                 double* fmax_part0, long out_stride, hipStream_t st);
hipError_t launch_fft_rows(const uint8_t* img, int height, int width, const FftPlan& plan,
                           const unsigned long long* sums, const double* k255,
                           double2* inter, hipStream_t st);
// Column pass + epilogue: power, running max, sum log(p) over p >= 1 per
// polar bin (binmap[wf][height], uint16 bin ids).  Accumulates into
// bin_sums[na*nr] (bin_scale fixed point) and writes one max power per block to fmax_part.
// (bscale: the fixed-point scale, 0 = bin_scale(height, wf))
hipError_t launch_fft_cols(const double2* inter, int height, int wf, const FftPlan& plan,
                           const uint16_t* binmap, int nbins, unsigned long long* bin_sums,
                           double* fmax_part, hipStream_t st, double bscale = 0.0);
// Column blocks of launch_fft_cols (= entries of fmax_part); optional LDS size.
int fft_cols_blocks(int height, int wf, int nbins, const FftPlan& plan, size_t* lds, int* lds_bins);

// ---- compile-time FFT plans (fft_ct.hip / fft_engine.h) ------------------------
// X(length, threads per block, radices...).  The first radix is odd (LDS
// bank-conflict-free first pass, fft_engine.h).  Rows need length % 4 == 0.
// Plan choices measured in rounds 2-4 (DESIGN.md sections 9-11; the rejected
// variants live in git history): rows of 4000 at 512 threads 43.2 us against
// 43.7 for (25 16 10) at 256, 47.3 at 400, 56.0 at 384; a last row pass that
// separates the two rows' spectra in registers 48.9-64.6.  Columns of 3000:
// (15 10 20) at 256 threads 54.8 us (ct_sweep), (15 20 10) 55.5, (25 12 10)
// 56.0, four-pass plans at 300 / 512 threads 61.2 / 61.4, two columns per
// block 63.2, register prefetch of the next column 64.5-72.3, pass 0 from
// registers 83.0, three blocks per CU at 168 VGPRs 94-107, global-atomic bins
// 92-148.  Columns of 6000: (15 20 20) 128 us, (10 20 30) 133; of 4000 at 256
// threads 130 us, 320 threads 126 (two blocks per CU since round 4's run
// lists); rows of 6000 at 512 threads 93 us.
#define PHD_CT_ROWS(X)           \
    X(4000, 512, 5, 8, 10, 10)   \
    X(6000, 512, 6, 10, 10, 10)  \
    X(3000, 384, 5, 6, 10, 10)   \
    X(2000, 256, 5, 4, 10, 10)   \
    /* config 5's sizes below 3 MP (round 3; batched launches, launch_fft_rows_ct_batch) */ \
    X(2048, 256, 8, 16, 16)      \
    X(1920, 256, 15, 8, 16)      \
    X(1280, 256, 5, 16, 16)      \
    X(720, 192, 5, 9, 16)        \
    X(640, 128, 5, 8, 16)        \
    X(480, 128, 5, 6, 16)        \
    X(512, 64, 8, 8, 8)
// (the 3000-row plan's threads and radices are overridable for A/B builds:
// make variant VFLAGS="-DPHD_C3000_T=320 -DPHD_C3000_R=20,15,10")
#ifndef PHD_C3000_T
#define PHD_C3000_T 256
#endif
#ifndef PHD_C3000_R
#define PHD_C3000_R 15, 10, 20
#endif
#define PHD_CT_COLS(X)           \
    X(3000, PHD_C3000_T, PHD_C3000_R) \
    X(6000, 512, 15, 20, 20)     \
    X(4000, 256, 10, 20, 20)     \
    X(2000, 256, 10, 10, 20)     \
    /* config 5's sizes below 3 MP (round 3; batched launches, launch_fft_cols_ct_batch) */ \
    X(1536, 256, 3, 8, 8, 8)     \
    X(1080, 192, 15, 8, 9)       \
    X(1280, 256, 5, 16, 16)      \
    X(720, 192, 5, 9, 16)        \
    X(640, 128, 5, 8, 16)        \
    X(480, 128, 5, 6, 16)        \
    X(512, 64, 8, 8, 8)
// radices of the compile-time plan for a row / column length (false: none)
bool ct_rows_plan(int w, std::vector<int>* radices);
bool ct_cols_plan(int h, std::vector<int>* radices);
// The polar bins the compile-time column pass sums into, as per-column run
// lists (round 4; the round-3 per-block LDS windows of bins are gone: the pass
// sums each run in an LDS slot and adds the slots to the image's bins).
// The compile-time FFT passes' half-spectrum intermediate (fft_ct.hip): row
// pair p's tile row of 4 KP elements (KP = ceil((W/2+1) / 2) column pairs,
// 16 B each) starts at p * ct_row_stride(W), a multiple of 8 elements, so every
// tile row -- and every pair of 64-byte tiles the column pass's XCD quads
// share -- begins on a 128-byte line (an unaligned start made the row pass's
// partial-line stores fetch their lines: +10 MB per 4000x3000 image).
constexpr int ct_row_stride(int width) { return (4 * (((width / 2 + 1) + 1) / 2) + 7) & ~7; }
// elements of one image's intermediate, for either FFT layout (+ scratch past
// the tiles for the row pass's dummy stores)
inline size_t inter_elems(int height, int width) {
    const size_t generic = (size_t)(height + 1) * (width / 2 + 2);
    const size_t ct = (size_t)((height + 1) / 2) * ct_row_stride(width);
    return (generic > ct ? generic : ct) + 1024;
}
constexpr int kColRunsMax = 256;   // entries (runs + sentinel) of one column's list (LDS)
struct ColBins {
    const uint32_t* runs = nullptr;  // [wf][rstride] runs of one polar bin (ColRuns, phd_host.h)
    // [wf][T] per thread: the run holding its first row (bits 0-7) and the rows
    // j = 1 .. E-1 of its E where a run starts (bit 8 + j; E <= 24)
    const uint32_t* seg = nullptr;
    int rstride = 0;                 // entries per column
};
size_t fft_cols_ct_lds(int height);
// threads per column of the compile-time column plan for a height (0: none)
int fft_cols_ct_threads(int height);
// log_mant (phd_device.h) over n positive doubles (tests)
hipError_t launch_log_mant(const double* x, double* y, long n, hipStream_t st);
// persistent grid of the column kernel (= entries of fmax_part)
int fft_cols_ct_blocks(int height);
// tw: the plan's per-pass tables W_{NS*R}^jm (jm < NS) for passes 1.. (host built).
// The row pass transforms the luma as is (sums unused): it does not wait for K1.
// rsum (optional, the blur-only path): the image's exact channel sums, accumulated
hipError_t launch_fft_rows_ct(const uint8_t* img, int height, int width, const unsigned long long* sums,
                              const double* k255, const double2* tw, double2* inter, hipStream_t st,
                              unsigned long long* rsum = nullptr);
// The column pass removes the DC bias (K1's channel sums) from column 0 first.
// dbg (optional): the power spectrum, column-major [wf][height]
hipError_t launch_fft_cols_ct(const double2* inter, int height, int width, int wf, const ColBins& cb,
                              unsigned long long* bin_sums, double* fmax_part, const double2* tw,
                              const unsigned long long* sums, double* dbg, hipStream_t st, bool pf = true);
// Batches of n images of one size in one launch each (sizes whose row pairs
// form whole line groups, (height + 1) / 2 % 4 == 0): d_imgs is a device array
// of image pointers; image i's intermediate, bin sums, max partials and channel
// sums sit i * inter_stride / bin_stride / fmax_stride / sums_stride elements
// from the first.  Small images are otherwise bound by per-launch costs.
hipError_t launch_fft_rows_ct_batch(const uint8_t* const* d_imgs, int n, int height, int width, const double* k255,
                                    const double2* tw, double2* inter, long inter_stride, hipStream_t st);
hipError_t launch_fft_cols_ct_batch(const double2* inter, long inter_stride, int n, int height, int width, int wf,
                                    const ColBins& cb, unsigned long long* bin_sums, long bin_stride,
                                    double* fmax_part, long fmax_stride, const double2* tw,
                                    const unsigned long long* sums, long sums_stride, hipStream_t st,
                                    bool pf = true);
// Same, the luma from an fp64 plane when pgm != nullptr (planar input).
hipError_t launch_sharpness_src(const uint8_t* img, const double* pgm, int height, int width, int n, const int* top,
                                const int* bottom, const int* left, const int* right, const double* k255,
                                double* sums, hipStream_t st);

// ---- fp64 planar input of the legacy entry point (planar.hip) ---------------
struct PlanarSrc {
    const double* r;
    const double* g;
    const double* b;
};
constexpr int kPlanarBlocks = 1024;
// flags: bit 0 not an 8-bit image, bit 1 non-finite value, bit 2 group index out of range
hipError_t launch_planar_to_u8(const PlanarSrc& P, long n, uint8_t* rgb, int* flags, hipStream_t st);
int planar_blocks(long n);   // partials of launch_planar_stats (per channel)
// part1 / part2 [planar_blocks][3]: sums of x and of (x - mean)^2; *avg = (Br + Bg + Bb) / 3; pgm = luma plane;
// lrng [planar_blocks][2]: -min and max of the luma per block
hipError_t launch_planar_stats(const PlanarSrc& P, long n, double* pgm, double* part1, double* part2, double* avg,
                               double* lrng, int* flags, hipStream_t st);
hipError_t launch_planar_k1(const PlanarSrc& P, int height, int width, int ds, const GridParams& gp, unsigned* hist,
                            unsigned short* chunk_hist, double* s_part, int* flags, hipStream_t st);
hipError_t launch_planar_tail(const PlanarSrc& P, int height, int width, int ds, const GridParams& gp,
                              const unsigned short* chunk_hist, int nchunks, GroupRule* rules, const int* search,
                              int n_search, const double* off, int nslots, double* out, hipStream_t st);

// ---- global-memory batched FFTs and the generic 2-D path (fft_global.hip) ----
// Blocks of the generic path's power / binning pass (= its max partials).
constexpr int kPowerBinBlocks = 1024;
// `count` contiguous sequences of length plan.n <= 8192, in place allowed.
hipError_t launch_gfft_direct(const double2* in, double2* out, long count, const FftPlan& plan, hipStream_t st);
// n = p1.n * p2.n: in -> scr (n1-point transforms, twiddles twn[e] = W_n^e) -> out.
hipError_t launch_gfft_4step(const double2* in, double2* out, double2* scr, long count, int n, const FftPlan& p1,
                             const FftPlan& p2, const double2* twn, hipStream_t st);
// Bluestein's pointwise steps (chirp c_j = exp(-pi i j^2 / n), bhat = FFT_M(conj c)).
hipError_t launch_blu_pre(const double2* x, double2* a, int n, int M, long count, const double2* chirp,
                          hipStream_t st);
hipError_t launch_blu_mid(double2* a, long count, int M, const double2* bhat, hipStream_t st);
hipError_t launch_blu_post(const double2* z, double2* out, int n, int M, long count, const double2* chirp,
                           hipStream_t st);
// Row pairs of the luma minus the DC bias: Z [ceil(H/2)][W] complex.  Luma from
// RGB8 (img, k255) or an fp64 plane (pgm); avg from RGB8 sums or *avgd.
hipError_t launch_pairs(const uint8_t* img, const double* pgm, int height, int width, const double* k255,
                        const unsigned long long* sums, const double* avgd, double2* Z, hipStream_t st);
// Row-pair spectra Z -> the column-major half spectrum inter [W/2+1][H].
hipError_t launch_split_t(const double2* Z, int height, int width, double2* inter, hipStream_t st);
// Power, max partials (kPowerBinBlocks) and polar log-binning of inter [wf][H].
hipError_t launch_power_bins(const double2* X, int height, int wf, const uint16_t* binmap, int nbins,
                             unsigned long long* bin_sums, double* fmax_part, hipStream_t st, double bscale = 0.0);

hipError_t launch_debug_hsv(const uint8_t* img, long n, const GridParams& gp, const FastCls& fc,
                            const ClassTables* tabs, const double* k255, int* gid, double* hsv, hipStream_t st);
hipError_t launch_fill_uniform(uint8_t* dst, size_t n, uint64_t seed, hipStream_t st);
// synth.py:structured on the device (synth.hip): h x w x 3 bytes
hipError_t launch_fill_structured(uint8_t* dst, int h, int w, uint64_t seed, int blur, int axis, hipStream_t st);
// Laplacian-variance sharpness of n crop boxes: sums[2k] = sum f, sums[2k+1] =
// sum (f - mean)^2 (sums zeroed by the caller).
hipError_t launch_sharpness(const uint8_t* img, int height, int width, int n, const int* top,
                            const int* bottom, const int* left, const int* right, const double* k255,
                            double* sums, hipStream_t st);

}  // namespace phd
