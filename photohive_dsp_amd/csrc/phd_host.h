// phd_host.h -- host-side internals of libreport_data.so (C++17).
#pragma once

#include <atomic>
#include <condition_variable>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <thread>
#include <string>
#include <tuple>
#include <vector>

#include <sys/types.h>

#include "../../include/photohive_dsp.h"
#include "phd_internal.h"

namespace phd {

// ---- errors ---------------------------------------------------------------
void set_error(const std::string& msg);   // thread-local, also printed to stderr
void clear_error();

#define PHD_HIP(expr)                                                                   \
    do {                                                                                \
        hipError_t e_ = (expr);                                                         \
        if (e_ != hipSuccess) {                                                         \
            ::phd::set_error(std::string("HIP error ") + hipGetErrorString(e_) + " at " \
                             + __FILE__ + ":" + std::to_string(__LINE__) + " (" #expr ")"); \
            return false;                                                               \
        }                                                                               \
    } while (0)

// ---- validated configuration ----------------------------------------------
// Returns false (with phd_last_error) for configurations where the reference's
// behaviour is undefined (see DESIGN.md "Deliberate rejections").
bool validate_config(const phd_config& cfg, std::string* why);
GridParams make_grid(const phd_config& cfg);
// Group centres of initialize_octree (src/color_quantization.c:57-99).
struct GroupCenters {
    std::vector<double> h, s, v;
};
GroupCenters make_centers(const GridParams& gp);
// Exact classification tables for fast_group (phd_device.h).
void make_class_tables(const GridParams& gp, FastCls* fc, ClassTables* t);

// ---- palette decisions (host) ---------------------------------------------
struct PaletteDecision {
    std::vector<int> parents;            // valid_parents, palette order
    std::vector<GroupRule> rules;        // [TL]
    std::vector<long long> kept;         // pixels each parent keeps
    std::vector<double> off;             // 180 - h_centre(parent)
    std::vector<int> search;             // groups needing the device cutoff search
};
// For each group i, every group ordered by (node_distance(i, p), p): the
// nearest-parent search of group_irregular_pixels walks it to the first
// parent instead of measuring every parent.  tl * tl u16; empty above
// kNearMaxGroups groups (then the search measures every parent).
constexpr int kNearMaxGroups = 2048;
std::vector<uint16_t> make_near_order(const GridParams& gp, const GroupCenters& gc);
// find_valid_octree_parents + group_irregular_pixels as keep rules.  near:
// make_near_order's table or nullptr.
bool decide_palette(const GridParams& gp, const GroupCenters& gc, const unsigned* hist, long n_hsv,
                    const phd_config& cfg, PaletteDecision* out, const uint16_t* near = nullptr);

// ---- blur profile helpers (host) ------------------------------------------
struct BlurTable {
    int height = 0, wf = 0, nr = 0, na = 0;
    std::vector<long long> counts;       // [na*nr]
    std::vector<uint16_t> map;           // host [wf][height] (the column run lists are made from it)
    uint16_t* d_map = nullptr;           // device [wf][height]
    int angle_bin_size = 0, radius_bin_size = 0;
};
// The compile-time column pass's polar bins as runs (ColBins): along each
// column the bin id changes a few tens of times (~76 runs per column at
// 4000x3000, 72 x 40 bins), so a column is its list of runs -- u32 start row
// << 16 | bin id, then a sentinel whose start is the height -- and each of the
// kernel's T threads per column gets the index of the run holding its first
// row (rows [t E, t E + E), E = ceil(height / T)).  ~1.5 MB per size instead
// of the 12 MB u16 bin of every element.
struct ColRuns {
    int T = 0, stride = 0;               // threads per column; entries per column (runs + sentinel)
    uint32_t* d_runs = nullptr;          // device [wf][stride]
    uint32_t* d_seg = nullptr;           // device [wf][T]: run index | run-start rows << 8 (ColBins::seg)
    int max_entries = 0;                 // the longest column's runs + sentinel
    bool too_many = false;               // max_entries > kColRunsMax: runtime-plan FFT for this size
};
// false when a column needs more than kColRunsMax entries (too_many: that size
// then takes the runtime-plan FFT) or on an upload error (nothing allocated).
bool build_col_runs(const uint16_t* map, int height, int wf, int T, ColRuns* r);
// Exact (phi_bin, r_bin) of every spectrum element, glibc atan2 + newton_int_sqrt
// exactly as src/blur_profile.c:87-97 / 427-458.
// upload == false: host map and counts only (no device copy)
bool build_blur_table(int height, int width, int nr, int na, BlurTable* t, bool upload = true);
void vectorize_blur(const double* bins, int na, int nr, double streak, double mag, int denom,
                    Blur_Vector* out10);

// ---- FFT plans --------------------------------------------------------------
struct FftPlanHost {
    FftPlan plan{};
    double2* d_tw = nullptr;
};
// composite: radices up to 16 (the image passes' kernels, fft.hip); else 2, 3,
// 4, 5, 8 and generic (fft_global.hip, which runs them at up to 1024 threads)
bool make_fft_plan(int n, FftPlanHost* p, bool composite = false);

// A batched 1-D transform of length n over sequences in HBM (fft_global.hip):
// one LDS pass (direct), two (four-step n = n1 * n2) or Bluestein's
// convolution through a smooth length M >= 2n - 1.
struct GfftPlan {
    enum { kDirect = 0, kFourStep = 1, kBluestein = 2 };
    int n = 0, kind = kDirect;
    const FftPlanHost* p = nullptr;                    // direct
    const FftPlanHost *p1 = nullptr, *p2 = nullptr;    // four-step
    double2* d_twn = nullptr;                          // four-step: W_n^e, e < n
    int M = 0;                                         // Bluestein
    const struct GfftPlan* sub = nullptr;
    double2* d_chirp = nullptr;                        // c_j = exp(-pi i j^2 / n)
    double2* d_bhat = nullptr;                         // FFT_M(conj c, wrapped)
};
// A length the LDS transforms take in one pass (n <= 8192, prime factors <= kMaxDirectPrime).
bool gfft_direct_ok(int n);
size_t gfft_scratch_elems(const GfftPlan& p, long count);
// in -> out (in == out allowed), scratch of gfft_scratch_elems(p, count) elements
bool gfft_run(const GfftPlan& p, const double2* in, double2* out, long count, double2* scr, hipStream_t st);

// ---- per-kernel event timing (opt-in, phd_profile_kernels) -----------------
enum KernelId { kK1 = 0, kFftRows = 1, kFftCols = 2, kCutoffs = 3, kPalSums = 4, kSharp = 5, kNumKernels = 6 };
struct KernelProfiler {
    unsigned mask = 0;                              // kernels to bracket with events
    // mask bits 24-30: stride s > 1, only every s-th batch call is bracketed
    // (all its launches; the events between back-to-back launches cost ~6% of
    // a bracketed call's time)
    unsigned calls = 0;                             // batch calls since the mask was set
    std::vector<std::pair<hipEvent_t, hipEvent_t>> pool;
    std::vector<int> pending;                       // kernel id per used pair (-1: launch not timed)
    double total_ms[kNumKernels] = {};
    long launches[kNumKernels] = {};
    // record the opening event of a launch of kernel k (no-op unless enabled)
    int begin(int k, hipStream_t st);
    void end(int slot, hipStream_t st);
    void collect();                                 // after the stream is drained
};

// ---- device context ---------------------------------------------------------
// A few persistent host threads for the per-image host work of a batch (the
// palette decisions): parallel_for(n, f) runs f(0 .. n-1) on them and on the
// caller.  The threads are detached and the pool is never destroyed.
class HostPool {
public:
    explicit HostPool(int threads);
    // f(0 .. n-1) on the pool's threads and the caller; a pool busy with
    // another caller's job (the other lane) runs f inline on the caller instead
    // of queueing behind it (one lane's assembly no longer waits for
    // the other lane's palette decisions)
    void parallel_for(int n, const std::function<void(int)>& f);
    int size() const { return nthreads_; }
    // waits for a running job, then ends and joins the threads (phd_shutdown)
    void stop();

private:
    void worker();
    int nthreads_ = 0;
    std::mutex m_, job_m_;
    std::condition_variable cv_, done_;
    const std::function<void(int)>* fn_ = nullptr;
    std::atomic<int> next_{0};
    int n_ = 0, busy_ = 0;
    unsigned gen_ = 0;
    bool stop_ = false;
    std::vector<std::thread> th_;
};
HostPool* host_pool();
HostPool* copy_pool();   // threads for host-buffer staging copies (phd_upload.cpp)
// phd_shutdown's parts: join the pools' threads (and forget the pools); the
// number of live pool threads
void stop_copy_pool();
int copy_pool_threads();
int library_threads();    // lane worker + pool threads alive in this process

struct Context {
    int device = -1;
    pid_t pid = 0;                                  // the process that created it (phd_shutdown)
    hipStream_t stream = nullptr;
    double* d_k255 = nullptr;                       // k/255.0 for k in [0,256)
    std::map<std::pair<int, bool>, FftPlanHost> plans;   // (length, composite)
    std::map<std::pair<int, int>, double2*> ct_tw;  // (length, rows?) -> compile-time plan twiddles
    std::map<std::tuple<int, int, int, int>, BlurTable> tables;
    std::map<std::tuple<int, int, int, int, int>, ColRuns> colruns;  // (H, W, nr, na, T): full-table runs
    std::map<int, GfftPlan> gplans;                 // global-memory FFT plans by length
    double2* d_gbuf = nullptr;                      // generic 2-D path: row pairs + scratch
    size_t gbuf_bytes = 0;
    double* d_planes = nullptr;                     // planar input: r | g | b | luma (fp64)
    size_t planes_bytes = 0;
    void* d_prec = nullptr;                         // planar input: per-call records
    size_t prec_bytes = 0;
    struct Cls {
        FastCls fc;
        ClassTables* d = nullptr;
        GroupCenters gc;                            // initialize_octree's centres
        std::vector<uint16_t> near;                 // make_near_order
    };
    std::map<std::tuple<int, int, int, double, double>, Cls> cls;
    // grow-only workspaces
    std::vector<PaletteDecision> dec_scratch;       // run_reports' per-image decisions
    std::vector<std::vector<double>> hsum_scratch;  // and host slot sums
    void* d_ws = nullptr;
    size_t ws_bytes = 0;
    void* h_pin = nullptr;
    size_t pin_bytes = 0;
    double2* d_inter = nullptr;
    size_t inter_bytes = 0;
    uint8_t* d_stage = nullptr;                    // upload staging for host images
    void* d_ptrs = nullptr;                        // small device pointer arrays (debug hooks)
    size_t ptrs_bytes = 0;
    size_t stage_bytes = 0;
    hipEvent_t ev[8] = {};
    // two streams per context: `stream` (K1, then the FFT chain) and `tail`
    // (the A-record download, the palette's second pass -- rules upload, Kcut,
    // partial sums -- concurrent with the FFTs, then each image's C-record
    // download as soon as its column pass is done), joined by events
    hipStream_t tail = nullptr;
    hipEvent_t ev_k1 = nullptr, ev_tail = nullptr;
    hipEvent_t ev_dl_sd = nullptr;                  // the tail stream's last copy of a call
    hipEvent_t ev_fft = nullptr;                    // the FFT chain's end
    std::vector<hipEvent_t> ev_img_fft, ev_img_dl;
    KernelProfiler prof;
    hipEvent_t ev_null = nullptr;                   // orders the library stream after the null stream
    // host-buffer uploads (phd_upload.cpp): pinned slot ring on the h2d stream,
    // two device staging buffers for overlapping groups
    hipStream_t h2d = nullptr;
    hipStream_t h2d2 = nullptr;     // second upload stream (every other image of a group)
    hipEvent_t ev_h2d2 = nullptr;
    uint8_t* h2d_slots = nullptr;
    std::vector<hipEvent_t> ev_slot;
    std::vector<char> slot_used;
    int next_slot = 0;
    hipEvent_t ev_up[2] = {};
    uint8_t* d_stage2[2] = {};
    size_t stage2_bytes[2] = {};
    std::mutex mu;
};
// The context of the current HIP device (created on first use).  nullptr if no GPU.
// Lanes: independent contexts of one device (own streams, workspaces and
// tables).  A large device batch is split over them and the halves run
// concurrently, so one half's host phases and launch gaps overlap the other's
// kernels.  Lane 0 is the context every single call uses.
constexpr int kLanes = 2;
Context* get_context();
Context* get_context_lane(int lane);
// flags of the events that only order device streams (no system-scope fence
// unless PHD_EV_FENCE is set; timing enabled, so a launch can record them)
unsigned device_event_flags();
std::vector<Context*> device_contexts();
// A persistent thread that runs one job at a time (the second lane).
class LaneWorker {
public:
    LaneWorker();
    void run(std::function<void()> f);
    void wait();
    // ends the thread after its current job (waiting up to timeout_ms for
    // it) and joins it; false (thread detached, left to the process) when
    // the job did not finish in time
    bool stop(int timeout_ms);
    // one caller at a time owns the worker (run .. wait); a busy worker is
    // not waited for: the caller runs its whole batch on lane 0 instead
    bool try_acquire() { return user_mu_.try_lock(); }
    void release() { user_mu_.unlock(); }

private:
    std::mutex user_mu_;
    void loop();
    std::mutex m_;
    std::condition_variable cv_, done_cv_;
    std::function<void()> job_;
    bool has_job_ = false;
    bool stop_ = false;
    std::thread th_;
};
LaneWorker* lane_worker();
// lanes a large device batch is split over (PHD_LANES, default 2; phd_set_lanes)
int lanes_setting();
// The stream a call works on: the caller's, or (NULL) the library's own stream
// ordered after every prior operation of the legacy null stream, so device
// buffers a caller (or PyTorch's default stream) is still producing are
// complete before the library reads them.
hipStream_t work_stream(Context* c, void* stream);
bool ensure_device(void** p, size_t* cap, size_t need);
bool ensure_pinned(Context* c, size_t need);
const FftPlanHost* get_plan(Context* c, int n, bool composite = false);
// Per-pass twiddle tables of the compile-time plan of length n (rows or columns).
const double2* get_ct_twiddles(Context* c, int n, bool rows);

// The FFT kernels one image size takes: the compile-time plans when both
// lengths have one (fft_ct.hip), else the runtime-plan kernels (fft.hip).
struct FftSel {
    bool ct = false;
    const FftPlanHost* prow = nullptr;
    const FftPlanHost* pcol = nullptr;
    const double2* tw_r = nullptr;
    const double2* tw_c = nullptr;
    int col_blocks = 0;   // entries of the per-block max partials
    ColBins cbins;        // compile-time column pass: its per-column polar-bin runs
    // compile-time column pass: its full-prefetch form (the whole next column
    // streams into LDS during the epilogue) where the plan has one, else the
    // half-prefetch form; run_reports takes the half form when another lane's
    // two-block K1 shares the CUs (measured)
    bool col_pf = true;
    // phd_debug_column_form: -1 the library's choice, 0 half-prefetch, 1 full
    static int forced_form();
    // the generic path (a side above the LDS limit or with a large prime
    // factor): row pairs -> global row transforms -> split / transpose, then
    // the fused runtime column pass (cols_fused) or global column transforms
    // + the power / binning pass
    bool generic = false, cols_fused = false;
    const GfftPlan* grow = nullptr;
    const GfftPlan* gcol = nullptr;
    double2* gbuf = nullptr;
};
// tbl: the polar-bin table of the size (the compile-time column pass's run
// lists are made from it; nullptr: no compile-time column pass can launch)
bool select_fft(Context* c, int height, int width, int nbins, const uint8_t* const* imgs, int n, FftSel* s,
                const BlurTable* tbl, bool batch = false);
hipError_t launch_rows_sel(const FftSel& s, const uint8_t* img, int height, int width,
                           const unsigned long long* sums, const double* k255, double2* inter, hipStream_t st,
                           unsigned long long* rsum = nullptr);
// sums: K1's channel sums of the image (the compile-time column pass removes the DC bias)
hipError_t launch_cols_sel(const FftSel& s, const double2* inter, int height, int width, int wf,
                           const uint16_t* binmap, int nbins, unsigned long long* bin_sums, double* fmax_part,
                           const unsigned long long* sums, double* dbg, hipStream_t st);
const GfftPlan* get_gfft(Context* c, int n);
bool select_generic(Context* c, int height, int width, int nbins, FftSel* s);
// The generic path's row stage: luma from RGB8 (img, sums) or an fp64 plane
// (pgm, avgd) into the column-major half spectrum `inter`.
hipError_t generic_rows(const FftSel& s, const uint8_t* img, const double* pgm, int height, int width,
                        const unsigned long long* sums, const double* avgd, const double* k255, double2* inter,
                        hipStream_t st);
// (bscale: the bins' fixed-point scale, 0 = bin_scale(height, wf))
hipError_t generic_cols(const FftSel& s, double2* inter, int height, int wf, const uint16_t* binmap, int nbins,
                        unsigned long long* bin_sums, double* fmax_part, hipStream_t st, double bscale = 0.0);
const BlurTable* get_table(Context* c, int height, int width, int nr, int na);
// Classification tables of a grid (uploaded once per configuration).
const Context::Cls* get_cls(Context* c, const GridParams& gp);

// ---- the pipeline -----------------------------------------------------------
// pre_compute_error_checks (src/utilities.c:64-87) on the dimensions / crop boxes.
bool precheck(int height, int width);
bool check_crops(const Crop_Boundaries* cb, int height, int width);
// pixels of the HSV image (downsample_rgb's size through `short`, src/image_processing.c:378-379)
long hsv_count(int height, int width, int ds);
// The Full_Report_Data tree (compile_full_report, src/utilities.c:210-226) from
// the statistics, the palette decision and its slot sums pal[4k + {h, s, v, n}],
// the polar bin sums (fixed point at bscale, 0 = bin_scale(H, Wf)) and
// spectrum max, the crop sums.
Full_Report_Data* assemble(const RGB_Statistics& st, double s_bar, const PaletteDecision& dec,
                           const double* pal, long n_hsv, const BlurTable& tbl, const unsigned long long* bin_sums,
                           double fmax, const phd_config& cfg, const Crop_Boundaries* crops,
                           const double* sharp_sums, std::string* why, double bscale = 0.0);
// get_full_report_data's reports in the reference's allocation shape
// (phd_legacy.cpp): a separately malloc'd copy, its registration as a live
// tree, and its release (false when r is not a live tree)
Full_Report_Data* legacy_tree_copy(const Full_Report_Data* src);
void legacy_tree_free(Full_Report_Data* r);
void legacy_register(const Full_Report_Data* r);
bool legacy_release(Full_Report_Data* r);
// get_full_report_data on the caller's planar doubles (phd_planar.cpp): the
// RGB8 pipeline when every value is k/255.0, else the fp64 planar kernels.
Full_Report_Data* report_planar(Context* c, const double* r, const double* g, const double* b, int height,
                                int width, const phd_config& cfg, const Crop_Boundaries* crops);
struct ImageIn {
    const uint8_t* d_img;   // device RGB8, rows of 3*width bytes
};
// Run the full report on n same-size device images.  out[i]/status[i] per image.
bool run_reports(Context* c, const uint8_t* const* d_imgs, int n, int height, int width,
                 const phd_config& cfg, const Crop_Boundaries* crops, Full_Report_Data** out,
                 int* status, hipStream_t stream);
// Palette intermediates only (for parity tests).
bool run_palette_trace(Context* c, const uint8_t* d_img, int height, int width, const phd_config& cfg,
                       std::vector<unsigned>* hist, PaletteDecision* dec,
                       std::vector<double>* device_counts);

void record_timings(const double* ms, int n);

// ---- host-buffer uploads (phd_upload.cpp) -------------------------------------
bool upload_init(Context* c);
// Copy `bytes` host bytes to d_dst through the pinned slot ring on c->h2d.  On
// return the caller's buffer has been read; the DMA may still run.
bool upload_async(Context* c, uint8_t* d_dst, const uint8_t* src, size_t bytes, std::string* why,
                  hipStream_t s = nullptr);
// 2 (PHD_UPLOAD_STREAMS=2; default 1): a group's images alternate between the
// h2d and h2d2 streams, each fed by its own host thread (runtime pageable path only)
int upload_streams();

}  // namespace phd
