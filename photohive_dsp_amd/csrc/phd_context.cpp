// phd_context.cpp -- per-device state: stream, constant tables, FFT plans,
// polar bin tables and grow-only workspaces.  One context per HIP device; a
// mutex serialises calls that share it (the API itself keeps no globals per
// call, unlike the reference's QUANTITY_WEIGHT / num_cores / FFTW state).
#include <atomic>
#include <cmath>
#include <cstdio>
#include <cstring>

#include <chrono>
#include <cstdlib>
#include <thread>

#include <unistd.h>

#include "phd_host.h"

namespace phd {

namespace {
void register_shutdown();
thread_local std::string g_error;
thread_local double g_timings[8];
thread_local int g_ntimings = 0;
std::mutex g_ctx_mu;
Context* g_ctx[64][kLanes] = {};
}  // namespace

void set_error(const std::string& msg) {
    g_error = msg;
    // the reference's own messages (pre_compute_error_checks, src/utilities.c:64-87)
    // are printed verbatim; the library's own ones carry the same "Error: " prefix
    if (!getenv("PHD_QUIET"))
        fprintf(stderr, "%s%s\n", msg.compare(0, 7, "Error: ") == 0 ? "" : "Error: ", msg.c_str());
}
void clear_error() { g_error.clear(); }

void record_timings(const double* ms, int n) {
    g_ntimings = n < 8 ? n : 8;
    for (int i = 0; i < g_ntimings; i++) g_timings[i] = ms[i];
}

Context* get_context() { return get_context_lane(0); }

Context* get_context_lane(int lane) {
    int dev = -1;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) {
        int n = 0;
        if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) {
            set_error("no HIP device available: the MI355X path has no CPU fallback");
            return nullptr;
        }
        dev = 0;
        if (hipSetDevice(0) != hipSuccess) {
            set_error("hipSetDevice(0) failed");
            return nullptr;
        }
    }
    std::lock_guard<std::mutex> lk(g_ctx_mu);
    if (g_ctx[dev][lane]) return g_ctx[dev][lane];
    // HIP is initialised now (hipGetDevice above): a handler registered here
    // runs before the finalizers HIP registered at its own start (atexit order
    // is last-in, first-out), so the library's threads, streams, events and
    // buffers are released while the runtime is still whole
    register_shutdown();
    auto* c = new Context();
    c->device = dev;
    c->pid = getpid();
    if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
        set_error("hipStreamCreate failed");
        delete c;
        return nullptr;
    }
    double k255[256];
    for (int k = 0; k < 256; k++) k255[k] = (double)k / 255.0;   // utils.py:30-46 (== C's k/255.0)
    if (hipMalloc(&c->d_k255, sizeof(k255)) != hipSuccess ||
        hipMemcpy(c->d_k255, k255, sizeof(k255), hipMemcpyHostToDevice) != hipSuccess) {
        set_error("device table upload failed");
        delete c;
        return nullptr;
    }
    // ev[4] / ev[5] are waited on by the host for data in host memory (system
    // fence); the rest only time stages and need no cache writeback (~30 us of
    // idle GPU when recorded before a download)
    for (int i = 0; i < 8; i++)
        (void)hipEventCreateWithFlags(&c->ev[i], (i == 4 || i == 5) ? hipEventDefault : hipEventDisableSystemFence);
    // the events that only order one device stream after another: no
    // system-scope fence either (each fenced record left the GPU idle ~5.7 us
    // between two kernels; PHD_EV_FENCE=1 restores it)
    const unsigned of = device_event_flags();
    if (hipStreamCreateWithFlags(&c->tail, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreateWithFlags(&c->ev_k1, of) != hipSuccess ||
        hipEventCreateWithFlags(&c->ev_tail, of) != hipSuccess ||
        hipEventCreateWithFlags(&c->ev_dl_sd, of) != hipSuccess ||
        hipEventCreateWithFlags(&c->ev_fft, of) != hipSuccess ||
        hipEventCreateWithFlags(&c->ev_null, of) != hipSuccess) {
        set_error("hipStreamCreate failed");
        delete c;
        return nullptr;
    }
    if (lane > 0 && g_ctx[dev][0]) c->prof.mask = g_ctx[dev][0]->prof.mask;   // profiled like lane 0
    g_ctx[dev][lane] = c;
    return c;
}

unsigned device_event_flags() {
    static const bool fence = phd_knob("PHD_EV_FENCE") != nullptr;
    return fence ? hipEventDisableTiming : hipEventDisableSystemFence;
}

// the contexts of this thread's device that exist (lane 0 first)
std::vector<Context*> device_contexts() {
    std::vector<Context*> out;
    int dev = -1;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return out;
    std::lock_guard<std::mutex> lk(g_ctx_mu);
    for (int l = 0; l < kLanes; l++)
        if (g_ctx[dev][l]) out.push_back(g_ctx[dev][l]);
    return out;
}

LaneWorker::LaneWorker() : th_([this] { loop(); }) {}

bool LaneWorker::stop(int timeout_ms) {
    std::unique_lock<std::mutex> lk(m_);
    if (!done_cv_.wait_for(lk, std::chrono::milliseconds(timeout_ms), [this] { return !has_job_; })) {
        th_.detach();
        return false;
    }
    stop_ = true;
    cv_.notify_all();
    lk.unlock();
    th_.join();
    return true;
}

void LaneWorker::run(std::function<void()> f) {
    std::lock_guard<std::mutex> lk(m_);
    job_ = std::move(f);
    has_job_ = true;
    cv_.notify_all();
}

void LaneWorker::wait() {
    std::unique_lock<std::mutex> lk(m_);
    done_cv_.wait(lk, [this] { return !has_job_; });
}

void LaneWorker::loop() {
    std::unique_lock<std::mutex> lk(m_);
    for (;;) {
        cv_.wait(lk, [this] { return has_job_ || stop_; });
        if (!has_job_) return;                              // stop()
        std::function<void()> f = std::move(job_);
        lk.unlock();
        f();
        lk.lock();
        has_job_ = false;
        done_cv_.notify_all();
    }
}

namespace {
std::atomic<int> g_lanes{-1};
}

int lanes_setting() {
    int l = g_lanes.load();
    if (l < 0) {
        const char* e = getenv("PHD_LANES");
        // two lanes unless asked for: each large call split into two concurrent
        // halves (+10-13 % images/s at 4000x3000, DESIGN.md "Lanes")
        l = e ? std::min(std::max(atoi(e), 1), kLanes) : 2;
        g_lanes.store(l);
    }
    return l;
}

namespace {
// lanes the calling thread's current call really runs on (on_lanes sets it
// around each lane's body; 1 outside a split call)
thread_local int t_call_lanes = 1;
}

CallLanes::CallLanes(int n) : prev_(t_call_lanes) { t_call_lanes = n; }
CallLanes::~CallLanes() { t_call_lanes = prev_; }

int k1_blocks_per_cu() {
    static const int env = phd_knob("PHD_K1_BPC") ? std::max(1, std::min(2, atoi(phd_knob("PHD_K1_BPC")))) : 0;
    // one block per CU only when this call is split over two lanes: the other
    // half of each CU then runs the other lane's FFT blocks; an unsplit call
    // (small batch, caller stream, host APIs) keeps both blocks
    return env ? env : (t_call_lanes >= 2 ? 1 : 2);
}

namespace {
// one lane worker and one decision pool per process (a forked child has none
// of its parent's threads: it makes its own and never touches the parent's)
std::mutex g_lw_mu, g_pool_mu;
LaneWorker* g_lw = nullptr;
pid_t g_lw_owner = 0;
HostPool* g_pool = nullptr;
pid_t g_pool_owner = 0;
}  // namespace

LaneWorker* lane_worker() {
    std::lock_guard<std::mutex> lk(g_lw_mu);
    if (!g_lw || g_lw_owner != getpid()) {
        g_lw = new LaneWorker();   // joined by phd_shutdown (at exit at the latest)
        g_lw_owner = getpid();
    }
    return g_lw;
}

hipStream_t work_stream(Context* c, void* stream) {
    if (stream) return (hipStream_t)stream;
    // the library stream is non-blocking: without this it would not wait for
    // work the caller queued on the null stream (e.g. a torch op producing the input)
    if (hipEventRecord(c->ev_null, nullptr) == hipSuccess) (void)hipStreamWaitEvent(c->stream, c->ev_null, 0);
    return c->stream;
}

// A growth frees the old buffer only once the device is idle (round 6, ADVICE
// r5: a pinned or device block freed under an in-flight copy would be a
// use-after-unmap; every entry point drains its streams before it returns,
// so this is belt and braces, and growth is rare).
bool ensure_device(void** p, size_t* cap, size_t need) {
    if (*cap >= need && *p) return true;
    if (*p) {
        (void)hipDeviceSynchronize();
        (void)hipFree(*p);
    }
    *p = nullptr;
    *cap = 0;
    size_t sz = need + need / 4 + 4096;
    if (hipMalloc(p, sz) != hipSuccess) {
        set_error("hipMalloc of " + std::to_string(sz) + " bytes failed");
        *p = nullptr;
        return false;
    }
    *cap = sz;
    return true;
}

bool ensure_pinned(Context* c, size_t need) {
    if (c->pin_bytes >= need && c->h_pin) return true;
    if (c->h_pin) {
        (void)hipDeviceSynchronize();
        (void)hipHostFree(c->h_pin);
    }
    c->h_pin = nullptr;
    size_t sz = need + need / 4 + 4096;
    if (hipHostMalloc(&c->h_pin, sz, hipHostMallocDefault) != hipSuccess) {
        set_error("hipHostMalloc failed");
        c->pin_bytes = 0;
        return false;
    }
    c->pin_bytes = sz;
    return true;
}

// ---- FFT plans ---------------------------------------------------------------
bool make_fft_plan(int n, FftPlanHost* p, bool composite) {
    if (n < 1 || n > kFftMaxLds) {
        set_error("FFT length " + std::to_string(n) + " exceeds the LDS-resident limit " +
                  std::to_string(kFftMaxLds) + " of this build");
        return false;
    }
    FftPlan& P = p->plan;
    P.n = n;
    P.npass = 0;
    int m = n;
    static const bool small_radices = phd_knob("PHD_FFT_SMALL_RADICES") != nullptr;   // A/B only
    if (composite && n <= 4096 && !small_radices) {
        // largest radix first: fewer LDS passes (1920 = 16 12 10 in three
        // instead of 8 8 5 3 2 in five)
        for (int r : {16, 12, 10, 9, 8, 6, 5, 4, 3, 2})
            while (m % r == 0 && P.npass < kMaxFftPasses) { P.radix[P.npass++] = r; m /= r; }
    }
    // radix order: 8s, then 4, then 2, 5, 3, then any remaining prime factor
    while (m % 8 == 0 && P.npass < kMaxFftPasses) { P.radix[P.npass++] = 8; m /= 8; }
    if (m % 4 == 0) { P.radix[P.npass++] = 4; m /= 4; }
    if (m % 2 == 0) { P.radix[P.npass++] = 2; m /= 2; }
    while (m % 5 == 0 && P.npass < kMaxFftPasses) { P.radix[P.npass++] = 5; m /= 5; }
    while (m % 3 == 0 && P.npass < kMaxFftPasses) { P.radix[P.npass++] = 3; m /= 3; }
    for (int f = 7; m > 1 && P.npass < kMaxFftPasses;) {
        if ((long)f * f > m) { P.radix[P.npass++] = m; m = 1; break; }
        if (m % f == 0) { P.radix[P.npass++] = f; m /= f; }
        else f += 2;
    }
    if (m != 1) {
        set_error("FFT length " + std::to_string(n) + " has too many factors");
        return false;
    }
    P.generic = 0;
    P.composite = 0;
    for (int i = 0; i < P.npass; i++) {
        const int r = P.radix[i];
        const bool comp = r == 6 || r == 9 || r == 10 || r == 12 || r == 16;
        if (r != 2 && r != 3 && r != 4 && r != 5 && r != 8 && !comp) P.generic = 1;
        P.composite |= comp ? 1 : 0;
    }
    P.n_hi = (n + 63) / 64;
    const long double two_pi = 6.283185307179586476925286766559005768L;
    auto w = [&](long t) {
        const long double a = two_pi * (long double)(t % n) / (long double)n;
        return make_double2((double)cosl(a), (double)-sinl(a));
    };
    std::vector<double2> tw(n + 64 + P.n_hi);
    for (int t = 0; t < n; t++) tw[t] = w(t);
    for (int t = 0; t < 64; t++) tw[n + t] = w(t);
    for (int t = 0; t < P.n_hi; t++) tw[n + 64 + t] = w(64L * t);
    if (hipMalloc(&p->d_tw, sizeof(double2) * tw.size()) != hipSuccess ||
        hipMemcpy(p->d_tw, tw.data(), sizeof(double2) * tw.size(), hipMemcpyHostToDevice) != hipSuccess) {
        set_error("twiddle upload failed");
        return false;
    }
    P.tw = p->d_tw;
    P.tw_lo = p->d_tw + n;
    P.tw_hi = p->d_tw + n + 64;
    return true;
}

const FftPlanHost* get_plan(Context* c, int n, bool composite) {
    const auto key = std::make_pair(n, composite);
    auto it = c->plans.find(key);
    if (it != c->plans.end()) return &it->second;
    FftPlanHost p;
    if (!make_fft_plan(n, &p, composite)) return nullptr;
    return &(c->plans[key] = p);
}

const double2* get_ct_twiddles(Context* c, int n, bool rows) {
    const auto key = std::make_pair(n, rows ? 1 : 0);
    auto it = c->ct_tw.find(key);
    if (it != c->ct_tw.end()) return it->second;
    std::vector<int> rad;
    if (!(rows ? ct_rows_plan(n, &rad) : ct_cols_plan(n, &rad))) {
        set_error("no compile-time FFT plan for length " + std::to_string(n));
        return nullptr;
    }
    // pass p (NS = R0 * ... * R(p-1) > 1): W_{NS*Rp}^jm for jm < NS
    const long double two_pi = 6.283185307179586476925286766559005768L;
    std::vector<double2> tw;
    long ns = 1;
    for (int r : rad) {
        if (ns > 1)
            for (long jm = 0; jm < ns; jm++) {
                const long double a = two_pi * (long double)jm / (long double)(ns * r);
                tw.push_back(make_double2((double)cosl(a), (double)-sinl(a)));
            }
        ns *= r;
    }
    if (tw.empty()) tw.push_back(make_double2(1.0, 0.0));
    double2* d = nullptr;
    if (hipMalloc(&d, sizeof(double2) * tw.size()) != hipSuccess ||
        hipMemcpy(d, tw.data(), sizeof(double2) * tw.size(), hipMemcpyHostToDevice) != hipSuccess) {
        set_error("compile-time FFT twiddle upload failed");
        return nullptr;
    }
    c->ct_tw[key] = d;
    return d;
}

// batch: the caller will run the compile-time passes as batched launches
// (one row and one column launch per group of same-size images)
namespace {
#ifndef PHD_COLUMN_FORM
#define PHD_COLUMN_FORM -1   // (A/B variant builds: the initial phd_debug_column_form)
#endif
std::atomic<int> g_column_form{PHD_COLUMN_FORM};
}

int FftSel::forced_form() { return g_column_form.load(std::memory_order_relaxed); }

bool select_fft(Context* c, int height, int width, int nbins, const uint8_t* const* imgs, int n, FftSel* s,
                const BlurTable* tbl, bool batch) {
    *s = FftSel{};
    if (FftSel::forced_form() >= 0) s->col_pf = FftSel::forced_form() == 1;
    static const bool force_generic = phd_knob("PHD_FFT_GENERIC") != nullptr;   // A/B experiments only
    bool ct = !force_generic && ct_rows_plan(width, nullptr) && ct_cols_plan(height, nullptr) &&
              fft_cols_ct_lds(height) <= 160 * 1024;
    for (int i = 0; ct && i < n; i++)
        if (reinterpret_cast<uintptr_t>(imgs[i]) & 3) ct = false;   // dword row loads
    // the column pass sums bins from per-column run lists (ColRuns); a table
    // with more than kColRunsMax runs in a column takes the runtime plans
    const ColRuns* runs = nullptr;
    if (ct && tbl) {
        // (round 4: the column pass sums its bins per run, so the per-block
        // bin windows that once shrank its LDS bin array are not used)
        const int T = fft_cols_ct_threads(height);
        (void)batch;
        {
            const auto key = std::make_tuple(height, width, tbl->nr, tbl->na, T);
            auto f = c->colruns.find(key);
            if (f == c->colruns.end()) {
                ColRuns r;
                // a size whose columns hold too many runs is remembered as such
                // (no rescan of the map per call); an upload error is not
                if (build_col_runs(tbl->map.data(), tbl->height, tbl->wf, T, &r) || r.too_many)
                    f = c->colruns.emplace(key, r).first;
            }
            if (f != c->colruns.end() && f->second.d_runs) runs = &f->second;
            else ct = false;
        }
    }
    if (ct) {
        s->ct = true;
        s->tw_r = get_ct_twiddles(c, width, true);
        s->tw_c = get_ct_twiddles(c, height, false);
        if (!s->tw_r || !s->tw_c) return false;
        s->cbins = ColBins{runs ? runs->d_runs : nullptr, runs ? runs->d_seg : nullptr, runs ? runs->stride : 0};
        s->col_blocks = fft_cols_ct_blocks(height);
        return true;
    }
    if (!gfft_direct_ok(width) || !gfft_direct_ok(height)) return select_generic(c, height, width, nbins, s);
    // composite radices for the row pass only: measured on 64-image groups
    // (per launch) rows of 1280 130 against 213 us, of 640 97 against 136;
    // the column pass ran slower with them (1080-row columns 176 against 146)
    s->prow = get_plan(c, width, true);
    s->pcol = get_plan(c, height);
    if (!s->prow || !s->pcol) return false;
    const int wf = width / 2 + 1;
    const int C = fft_cols_blocks(height, wf, nbins, s->pcol->plan, nullptr, nullptr);
    s->col_blocks = (wf + C - 1) / C;
    return true;
}

hipError_t launch_rows_sel(const FftSel& s, const uint8_t* img, int height, int width,
                           const unsigned long long* sums, const double* k255, double2* inter, hipStream_t st,
                           unsigned long long* rsum) {
    if (s.generic) return generic_rows(s, img, nullptr, height, width, sums, nullptr, k255, inter, st);
    return s.ct ? launch_fft_rows_ct(img, height, width, sums, k255, s.tw_r, inter, st, rsum)
                : launch_fft_rows(img, height, width, s.prow->plan, sums, k255, inter, st);
}

hipError_t launch_cols_sel(const FftSel& s, const double2* inter, int height, int width, int wf,
                           const uint16_t* binmap, int nbins, unsigned long long* bin_sums, double* fmax_part,
                           const unsigned long long* sums, double* dbg, hipStream_t st) {
    if (s.ct) {
        if (!s.cbins.runs) return hipErrorInvalidValue;   // select_fft without a table
        return launch_fft_cols_ct(inter, height, width, wf, s.cbins, bin_sums, fmax_part, s.tw_c, sums, dbg, st,
                                  s.col_pf);
    }
    if (dbg) return hipErrorNotSupported;
    if (s.generic) return generic_cols(s, const_cast<double2*>(inter), height, wf, binmap, nbins, bin_sums, fmax_part, st);
    return launch_fft_cols(inter, height, wf, s.pcol->plan, binmap, nbins, bin_sums, fmax_part, st);
}

const BlurTable* get_table(Context* c, int height, int width, int nr, int na) {
    auto key = std::make_tuple(height, width, nr, na);
    auto it = c->tables.find(key);
    if (it != c->tables.end()) return &it->second;
    BlurTable t;
    if (!build_blur_table(height, width, nr, na, &t)) return nullptr;
    return &(c->tables[key] = std::move(t));
}

HostPool::HostPool(int threads) : nthreads_(threads) {
    for (int t = 0; t < threads; t++) th_.emplace_back([this] { worker(); });
}

void HostPool::stop() {
    std::lock_guard<std::mutex> job(job_m_);              // a running job finishes first
    {
        std::lock_guard<std::mutex> lk(m_);
        stop_ = true;
    }
    cv_.notify_all();
    for (auto& t : th_)
        if (t.joinable()) t.join();
    th_.clear();
    nthreads_ = 0;
}

void HostPool::worker() {
    unsigned seen = 0;
    for (;;) {
        const std::function<void(int)>* fn;
        int n;
        {
            std::unique_lock<std::mutex> lk(m_);
            cv_.wait(lk, [&] { return stop_ || gen_ != seen; });
            if (stop_) return;
            seen = gen_;
            fn = fn_;
            n = n_;
        }
        for (int i; (i = next_.fetch_add(1)) < n;) (*fn)(i);
        std::lock_guard<std::mutex> lk(m_);
        if (--busy_ == 0) done_.notify_one();
    }
}

void HostPool::parallel_for(int n, const std::function<void(int)>& f) {
    // one job at a time; a caller that finds the pool busy (the other lane,
    // another device's context) runs its items itself rather than wait
    std::unique_lock<std::mutex> job(job_m_, std::try_to_lock);
    if (!job.owns_lock() || nthreads_ == 0) {
        for (int i = 0; i < n; i++) f(i);
        return;
    }
    {
        std::lock_guard<std::mutex> lk(m_);
        fn_ = &f;
        n_ = n;
        next_.store(0);
        busy_ = nthreads_;
        gen_++;
    }
    cv_.notify_all();
    for (int i; (i = next_.fetch_add(1)) < n;) f(i);
    std::unique_lock<std::mutex> lk(m_);
    done_.wait(lk, [&] { return busy_ == 0; });
    fn_ = nullptr;
}

HostPool* host_pool() {
    std::lock_guard<std::mutex> lk(g_pool_mu);
    if (!g_pool || g_pool_owner != getpid()) {
        const unsigned hc = std::thread::hardware_concurrency();
        g_pool = new HostPool(hc > 1 ? (int)std::min(hc - 1, 7u) : 0);
        g_pool_owner = getpid();
    }
    return g_pool;
}

// ---- teardown (phd_shutdown) --------------------------------------------------
namespace {

template <class T>
void dfree(T*& p) {
    if (p) (void)hipFree((void*)p);
    p = nullptr;
}
void ev_destroy(hipEvent_t& e) {
    if (e) (void)hipEventDestroy(e);
    e = nullptr;
}
void st_destroy(hipStream_t& s) {
    if (s) (void)hipStreamDestroy(s);
    s = nullptr;
}

// Releases everything a context owns: its queued work is waited for, then its
// device buffers, pinned buffers, events and streams are released.
void destroy_context(Context* c) {
    (void)hipSetDevice(c->device);
    for (hipStream_t s : {c->stream, c->tail, c->h2d, c->h2d2})
        if (s) (void)hipStreamSynchronize(s);
    dfree(c->d_k255);
    for (auto& kv : c->plans) dfree(kv.second.d_tw);
    for (auto& kv : c->ct_tw) dfree(kv.second);
    for (auto& kv : c->tables) dfree(kv.second.d_map);
    for (auto& kv : c->colruns) {
        dfree(kv.second.d_runs);
        dfree(kv.second.d_seg);
    }
    for (auto& kv : c->gplans) {
        dfree(kv.second.d_twn);
        dfree(kv.second.d_chirp);
        dfree(kv.second.d_bhat);
    }
    for (auto& kv : c->cls) dfree(kv.second.d);
    dfree(c->d_gbuf);
    dfree(c->d_planes);
    dfree(c->d_prec);
    dfree(c->d_ws);
    dfree(c->d_inter);
    dfree(c->d_stage);
    dfree(c->d_ptrs);
    for (auto& p : c->d_stage2) dfree(p);
    if (c->h_pin) (void)hipHostFree(c->h_pin);
    c->h_pin = nullptr;
    if (c->h2d_slots) (void)hipHostFree(c->h2d_slots);
    c->h2d_slots = nullptr;
    for (auto& e : c->ev) ev_destroy(e);
    for (hipEvent_t* e : {&c->ev_k1, &c->ev_tail, &c->ev_dl_sd, &c->ev_fft, &c->ev_null, &c->ev_h2d2}) ev_destroy(*e);
    for (auto& e : c->ev_img_fft) ev_destroy(e);
    for (auto& e : c->ev_img_dl) ev_destroy(e);
    for (auto& e : c->ev_slot) ev_destroy(e);
    for (auto& e : c->ev_up) ev_destroy(e);
    for (auto& pr : c->prof.pool) {
        ev_destroy(pr.first);
        ev_destroy(pr.second);
    }
    st_destroy(c->stream);
    st_destroy(c->tail);
    st_destroy(c->h2d);
    st_destroy(c->h2d2);
}

std::atomic<bool> g_in_exit{false};

void shutdown_at_exit() {
    g_in_exit.store(true);
    phd_shutdown();
}

void register_shutdown() {
    static std::once_flag once;
    std::call_once(once, [] { std::atexit(shutdown_at_exit); });
}

}  // namespace

int library_threads() {
    int n = 0;
    {
        std::lock_guard<std::mutex> lk(g_lw_mu);
        n += g_lw && g_lw_owner == getpid();
    }
    {
        std::lock_guard<std::mutex> lk(g_pool_mu);
        if (g_pool && g_pool_owner == getpid()) n += g_pool->size();
    }
    return n + copy_pool_threads();
}

int KernelProfiler::begin(int k, hipStream_t st) {
    if (!(mask & (1u << k))) return -1;
    const unsigned stride = (mask >> 24) & 127u;
    if (stride > 1 && calls % stride != 0) return -1;
    const size_t slot = pending.size();
    if (slot >= pool.size()) {
        hipEvent_t a, b;
        // timing only: no system-scope fence around the profiled kernels
        if (hipEventCreateWithFlags(&a, hipEventDisableSystemFence) != hipSuccess ||
            hipEventCreateWithFlags(&b, hipEventDisableSystemFence) != hipSuccess)
            return -1;
        pool.emplace_back(a, b);
    }
    pending.push_back(k);
    launch_events() = LaunchEvents{pool[slot].first, pool[slot].second, false};
    return (int)slot;
}

void KernelProfiler::end(int slot, hipStream_t st) {
    if (slot < 0) return;
    if (!launch_events().used) pending[slot] = -1;   // no phd_launch took the events
    launch_events() = LaunchEvents{};
}

LaunchEvents& launch_events() {
    static thread_local LaunchEvents e;
    return e;
}

void KernelProfiler::collect() {
    calls++;
    for (size_t i = 0; i < pending.size(); i++) {
        if (pending[i] < 0) continue;
        float ms = 0.f;
        if (hipEventElapsedTime(&ms, pool[i].first, pool[i].second) == hipSuccess) {
            total_ms[pending[i]] += ms;
            launches[pending[i]]++;
        }
    }
    pending.clear();
}

const Context::Cls* get_cls(Context* c, const GridParams& gp) {
    auto key = std::make_tuple(gp.hp, gp.sp, gp.vp, gp.bt, gp.gt);
    auto it = c->cls.find(key);
    if (it != c->cls.end()) return &it->second;
    Context::Cls e;
    ClassTables t;
    make_class_tables(gp, &e.fc, &t);
    e.gc = make_centers(gp);
    e.near = make_near_order(gp, e.gc);
    if (hipMalloc(&e.d, sizeof(ClassTables)) != hipSuccess ||
        hipMemcpy(e.d, &t, sizeof(ClassTables), hipMemcpyHostToDevice) != hipSuccess) {
        set_error("classification table upload failed");
        return nullptr;
    }
    return &(c->cls[key] = e);
}

}  // namespace phd

// The library's explicit teardown (round 6): the lane worker and the host
// pools' threads are stopped and joined, then every context of this process
// waits for its streams and releases its device buffers, pinned buffers,
// events and streams.  Registered with atexit at the first HIP use, so it runs
// before HIP's own finalizers; callable earlier (then the next call starts
// afresh).  Not to be called while another thread is inside a library call.
extern "C" void phd_shutdown(void) {
    using namespace phd;
    const pid_t me = getpid();
    {
        std::lock_guard<std::mutex> lk(g_lw_mu);
        if (g_lw && g_lw_owner == me) {
            if (g_lw->stop(5000)) delete g_lw;   // else left running (a stuck job): not ours to free
        }
        g_lw = nullptr;
    }
    {
        std::lock_guard<std::mutex> lk(g_pool_mu);
        if (g_pool && g_pool_owner == me) {
            g_pool->stop();
            delete g_pool;
        }
        g_pool = nullptr;
    }
    stop_copy_pool();
    std::vector<Context*> mine;
    {
        std::lock_guard<std::mutex> lk(g_ctx_mu);
        for (auto& per_dev : g_ctx)
            for (auto& c : per_dev) {
                if (c && c->pid == me) mine.push_back(c);
                c = nullptr;                         // another process's (fork): forgotten, never touched
            }
    }
    int dev0 = -1;
    const bool have_dev = hipGetDevice(&dev0) == hipSuccess;
    for (Context* c : mine) {
        // a context still held by a call on another thread is left alone
        std::unique_lock<std::mutex> lk(c->mu, std::try_to_lock);
        for (int t = 0; t < 200 && !lk.owns_lock(); t++) {
            std::this_thread::sleep_for(std::chrono::milliseconds(10));
            lk.try_lock();
        }
        if (!lk.owns_lock()) continue;
        destroy_context(c);
        lk.unlock();
        if (!g_in_exit.load()) delete c;            // at exit its host maps are left to the process
    }
    if (have_dev && dev0 >= 0) (void)hipSetDevice(dev0);
}

extern "C" int phd_debug_library_threads(int start) {
    if (start) {
        (void)phd::lane_worker();
        (void)phd::host_pool();
        (void)phd::copy_pool();
    }
    return phd::library_threads();
}

extern "C" int phd_set_lanes(int lanes) {
    const int prev = phd::lanes_setting();
    if (lanes >= 1) phd::g_lanes.store(std::min(lanes, phd::kLanes));
    return prev;
}

extern "C" int phd_profile_kernels(unsigned mask) {
    if (!phd::get_context()) return -1;
    for (phd::Context* c : phd::device_contexts()) {     // every lane of this device
        std::lock_guard<std::mutex> lk(c->mu);
        c->prof.mask = mask;
        c->prof.calls = 0;
        c->prof.pending.clear();
        for (int k = 0; k < phd::kNumKernels; k++) {
            c->prof.total_ms[k] = 0.0;
            c->prof.launches[k] = 0;
        }
    }
    return 0;
}

extern "C" int phd_profile_read(int kernel, double* total_ms, long* launches) {
    if (!phd::get_context() || kernel < 0 || kernel >= phd::kNumKernels) return -1;
    *total_ms = 0.0;
    *launches = 0;
    for (phd::Context* c : phd::device_contexts()) {     // summed over the lanes
        std::lock_guard<std::mutex> lk(c->mu);
        *total_ms += c->prof.total_ms[kernel];
        *launches += c->prof.launches[kernel];
    }
    return 0;
}

extern "C" const char* phd_last_error(void) { return phd::g_error.c_str(); }

extern "C" int phd_last_timings(double* ms, int n) {
    int k = n < phd::g_ntimings ? n : phd::g_ntimings;
    for (int i = 0; i < k; i++) ms[i] = phd::g_timings[i];
    return k;
}

extern "C" int phd_device_info(char* buf, int buflen) {
    int dev = -1, n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) {
        if (buf && buflen > 0) snprintf(buf, buflen, "no HIP device");
        return -1;
    }
    if (hipGetDevice(&dev) != hipSuccess) dev = 0;
    hipDeviceProp_t pr;
    if (hipGetDeviceProperties(&pr, dev) != hipSuccess) return -1;
    if (buf && buflen > 0)
        snprintf(buf, buflen, "%s %s CUs=%d HBM=%.1fGB", pr.name, pr.gcnArchName, pr.multiProcessorCount,
                 pr.totalGlobalMem / 1e9);
    return dev;
}

extern "C" int phd_debug_column_form(int mode) {
    return phd::g_column_form.exchange(mode < 0 ? -1 : (mode ? 1 : 0));
}
