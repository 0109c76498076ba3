// phd_gfft.cpp -- plans and drivers of the global-memory FFTs (fft_global.hip)
// and of the generic 2-D power-spectrum path: image sides above the LDS limit
// (the reference accepts up to 120 MP within 1:5..5:1, src/utilities.c:12,
// 73-80, and FFTW any length, src/fft_processing.c:18-63), lengths with a
// large prime factor (Bluestein instead of an O(n p) direct DFT pass) and the
// fp64 planar input of the legacy entry point.
#include <cmath>

#include "phd_host.h"

namespace phd {

namespace {

int largest_prime_factor(int n) {
    int p = 1;
    for (int f = 2; (long)f * f <= n; f++)
        while (n % f == 0) {
            p = f;
            n /= f;
        }
    return n > 1 ? std::max(p, n) : p;
}

bool smooth5(int m) {
    for (int f : {2, 3, 5})
        while (m % f == 0) m /= f;
    return m == 1;
}

const long double kTwoPi = 6.283185307179586476925286766559005768L;

bool upload(double2** d, const std::vector<double2>& h) {
    if (hipMalloc(d, sizeof(double2) * h.size()) != hipSuccess ||
        hipMemcpy(*d, h.data(), sizeof(double2) * h.size(), hipMemcpyHostToDevice) != hipSuccess) {
        set_error("FFT table upload failed");
        return false;
    }
    return true;
}

// Sequences of a Bluestein chunk: its two length-M buffers stay within 2 GiB.
long blu_chunk(int M) { return std::max<long>(1, ((long)1 << 27) / M); }

}  // namespace

bool gfft_direct_ok(int n) { return n >= 1 && n <= kFftMaxLds && largest_prime_factor(n) <= kMaxDirectPrime; }

const GfftPlan* get_gfft(Context* c, int n) {
    auto it = c->gplans.find(n);
    if (it != c->gplans.end()) return &it->second;
    GfftPlan P;
    P.n = n;
    if (gfft_direct_ok(n)) {
        P.kind = GfftPlan::kDirect;
        if (!(P.p = get_plan(c, n))) return nullptr;
        return &(c->gplans[n] = P);
    }
    // four-step: the most balanced split into two direct lengths
    int best = 0;
    for (int n1 = 1; (long)n1 * n1 <= n; n1++)
        if (n % n1 == 0 && gfft_direct_ok(n1) && gfft_direct_ok(n / n1)) best = n1;
    if (best > 0) {
        P.kind = GfftPlan::kFourStep;
        if (!(P.p1 = get_plan(c, best)) || !(P.p2 = get_plan(c, n / best))) return nullptr;
        std::vector<double2> tw(n);
        for (int e = 0; e < n; e++) {
            const long double a = kTwoPi * (long double)e / (long double)n;
            tw[e] = make_double2((double)cosl(a), (double)-sinl(a));
        }
        if (!upload(&P.d_twn, tw)) return nullptr;
        return &(c->gplans[n] = P);
    }
    // Bluestein over the smallest 5-smooth M >= 2n - 1
    int M = 2 * n - 1;
    while (!smooth5(M)) M++;
    const GfftPlan* sub = get_gfft(c, M);
    if (!sub || sub->kind == GfftPlan::kBluestein) {
        if (sub) set_error("no FFT plan for length " + std::to_string(n));
        return nullptr;
    }
    P.kind = GfftPlan::kBluestein;
    P.M = M;
    P.sub = sub;
    // c_j = exp(-pi i j^2 / n): j^2 mod 2n exactly, the angle in long double
    std::vector<double2> ch(n), b(M, make_double2(0.0, 0.0));
    for (long j = 0; j < n; j++) {
        const long e = (j * j) % (2L * n);
        const long double a = kTwoPi * 0.5L * (long double)e / (long double)n;
        ch[j] = make_double2((double)cosl(a), (double)-sinl(a));
        b[j] = make_double2(ch[j].x, -ch[j].y);          // conj(c_j)
        if (j > 0) b[M - j] = b[j];
    }
    if (!upload(&P.d_chirp, ch) || !upload(&P.d_bhat, b)) return nullptr;
    // bhat = FFT_M(b), once, on the library stream
    double2* scr = nullptr;
    const size_t se = gfft_scratch_elems(*sub, 1);
    if (se && hipMalloc(&scr, sizeof(double2) * se) != hipSuccess) {
        set_error("Bluestein plan scratch allocation failed");
        return nullptr;
    }
    const bool ok = gfft_run(*sub, P.d_bhat, P.d_bhat, 1, scr, c->stream) && hipStreamSynchronize(c->stream) == hipSuccess;
    if (scr) (void)hipFree(scr);
    if (!ok) {
        set_error("Bluestein plan setup failed");
        return nullptr;
    }
    return &(c->gplans[n] = P);
}

size_t gfft_scratch_elems(const GfftPlan& p, long count) {
    switch (p.kind) {
        case GfftPlan::kDirect: return 0;
        case GfftPlan::kFourStep: return (size_t)count * p.n;
        default: {
            const long cs = std::min(count, blu_chunk(p.M));
            return (size_t)cs * p.M * (p.sub->kind == GfftPlan::kFourStep ? 2 : 1);
        }
    }
}

bool gfft_run(const GfftPlan& p, const double2* in, double2* out, long count, double2* scr, hipStream_t st) {
    switch (p.kind) {
        case GfftPlan::kDirect:
            PHD_HIP(launch_gfft_direct(in, out, count, p.p->plan, st));
            return true;
        case GfftPlan::kFourStep:
            PHD_HIP(launch_gfft_4step(in, out, scr, count, p.n, p.p1->plan, p.p2->plan, p.d_twn, st));
            return true;
        default: {
            const long cs = std::min(count, blu_chunk(p.M));
            double2* a = scr;
            double2* s2 = scr + (size_t)cs * p.M;
            for (long s0 = 0; s0 < count; s0 += cs) {
                const long m = std::min(cs, count - s0);
                PHD_HIP(launch_blu_pre(in + s0 * p.n, a, p.n, p.M, m, p.d_chirp, st));
                if (!gfft_run(*p.sub, a, a, m, s2, st)) return false;
                PHD_HIP(launch_blu_mid(a, m, p.M, p.d_bhat, st));
                if (!gfft_run(*p.sub, a, a, m, s2, st)) return false;
                PHD_HIP(launch_blu_post(a, out + s0 * p.n, p.n, p.M, m, p.d_chirp, st));
            }
            return true;
        }
    }
}

// ---- the generic 2-D path ------------------------------------------------------
bool select_generic(Context* c, int height, int width, int nbins, FftSel* s) {
    const int wf = width / 2 + 1, hp = (height + 1) / 2;
    s->generic = true;
    s->grow = get_gfft(c, width);
    if (!s->grow) return false;
    s->cols_fused = gfft_direct_ok(height);
    if (s->cols_fused) {
        s->pcol = get_plan(c, height);
        if (!s->pcol) return false;
        const int C = fft_cols_blocks(height, wf, nbins, s->pcol->plan, nullptr, nullptr);
        s->col_blocks = (wf + C - 1) / C;
    } else {
        s->gcol = get_gfft(c, height);
        if (!s->gcol) return false;
        s->col_blocks = kPowerBinBlocks;
    }
    // [ row pairs Z | scratch of the row transforms ]; the column transforms'
    // scratch reuses it (Z is consumed by the split before they run)
    const size_t rows = (size_t)hp * width + gfft_scratch_elems(*s->grow, hp);
    const size_t cols = s->gcol ? gfft_scratch_elems(*s->gcol, wf) : 0;
    if (!ensure_device((void**)&c->d_gbuf, &c->gbuf_bytes, sizeof(double2) * std::max(rows, cols))) return false;
    s->gbuf = c->d_gbuf;
    return true;
}

hipError_t generic_rows(const FftSel& s, const uint8_t* img, const double* pgm, int height, int width,
                        const unsigned long long* sums, const double* avgd, const double* k255, double2* inter,
                        hipStream_t st) {
    const int hp = (height + 1) / 2;
    double2* Z = s.gbuf;
    double2* scr = s.gbuf + (size_t)hp * width;
    hipError_t e = launch_pairs(img, pgm, height, width, k255, sums, avgd, Z, st);
    if (e != hipSuccess) return e;
    if (!gfft_run(*s.grow, Z, Z, hp, scr, st)) return hipErrorLaunchFailure;
    return launch_split_t(Z, height, width, inter, st);
}

hipError_t generic_cols(const FftSel& s, double2* inter, int height, int wf, const uint16_t* binmap, int nbins,
                        unsigned long long* bin_sums, double* fmax_part, hipStream_t st, double bscale) {
    if (s.cols_fused)
        return launch_fft_cols(inter, height, wf, s.pcol->plan, binmap, nbins, bin_sums, fmax_part, st, bscale);
    if (!gfft_run(*s.gcol, inter, inter, wf, s.gbuf, st)) return hipErrorLaunchFailure;
    return launch_power_bins(inter, height, wf, binmap, nbins, bin_sums, fmax_part, st, bscale);
}

}  // namespace phd

using namespace phd;

// Validation hook: `count` contiguous complex sequences of length n (device,
// interleaved re/im doubles) -> their unnormalised forward DFTs (e^{-i}) in
// d_out (d_out == d_in allowed).  Returns the plan kind (0 direct, 1
// four-step, 2 Bluestein) or -1.
extern "C" int phd_debug_gfft(const double* d_in, double* d_out, int n, long count) {
    clear_error();
    Context* c = get_context();
    if (!c || !d_in || !d_out || n < 1 || count < 1) return -1;
    std::lock_guard<std::mutex> lk(c->mu);
    const GfftPlan* p = get_gfft(c, n);
    if (!p) return -1;
    double2* scr = nullptr;
    const size_t se = gfft_scratch_elems(*p, count);
    if (se && hipMalloc(&scr, sizeof(double2) * se) != hipSuccess) {
        set_error("scratch allocation failed");
        return -1;
    }
    const bool ok = gfft_run(*p, (const double2*)d_in, (double2*)d_out, count, scr, c->stream) &&
                    hipStreamSynchronize(c->stream) == hipSuccess;
    if (scr) (void)hipFree(scr);
    if (!ok) {
        set_error("global FFT failed");
        return -1;
    }
    return p->kind;
}
