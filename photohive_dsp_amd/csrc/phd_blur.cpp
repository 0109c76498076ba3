// phd_blur.cpp -- host pieces of the blur profile:
//  * the image-independent polar bin table of a spectrum size (which
//    (angle, radius) bin every element of the H x (W/2+1) half spectrum lands
//    in, and how many elements each bin holds).  It is evaluated once per
//    (H, W, nr, na) with glibc atan2 and the reference's newton_int_sqrt, so
//    the device binning is bit-exact by construction; the device reads the
//    uint16 bin id of each element from it;
//  * vectorize_blur_profile (src/blur_profile.c:324-416), 72x40 doubles in,
//    10 vectors out -- tiny, sequential, host C++;
//  * get_blur_profile_visual (src/blur_profile.c:140-180), the third
//    exported symbol of the reference library.
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <thread>

#include "phd_host.h"

namespace phd {

namespace {

constexpr double kRefPi = 3.14159265;   // src/blur_profile.c:10 (truncated)

int newton_int_sqrt(double val) {       // src/utilities.c:43-52
    if (val == 0) return 0;
    double x = val;
    for (;;) {
        const double s = 0.5 * (x + (val / x));
        if (std::fabs(s - x) < 1) return (int)s;
        x = s;
    }
}

}  // namespace

// T <= 1024 threads: at most 2046 bytes of run plus a 16-byte load
constexpr size_t kBinMapPad = 4096;

bool build_blur_table(int height, int width, int nr, int na, BlurTable* t, bool upload) {
    const int wf = width / 2 + 1;
    t->height = height;
    t->wf = wf;
    t->nr = nr;
    t->na = na;
    // calculate_blur_profile's integer arithmetic (src/blur_profile.c:56-61)
    const long ext = (long)wf * wf + ((long)height * height) / 4;
    t->angle_bin_size = (int)(double)(180 / na);
    t->radius_bin_size = (int)(double)(std::sqrt((double)ext) / nr);
    const double rbss = (double)(ext / ((long)nr * nr));
    if (rbss == 0) {
        set_error("radius_partitions too large for this image (radius bin size 0)");
        return false;
    }
    std::vector<uint16_t> map((size_t)wf * height);
    const unsigned nth = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    std::vector<std::vector<long long>> part(nth, std::vector<long long>((size_t)na * nr, 0));
    std::vector<int> bad(nth, 0);
    auto work = [&](unsigned tid) {
        for (int x = tid; x < wf; x += nth) {
            for (int u = 0; u < height; u++) {
                // cartesian_to_polar_conversion (src/blur_profile.c:439-456): rows
                // u < H/2 hold y = u, phi = -atan2; the others y = H-1-u, phi = +atan2
                // (odd H: the middle row's second, "bottom", write wins).
                int y;
                double phi;
                if (u < height / 2) {
                    y = u;
                    phi = -std::atan2((double)y, (double)x);
                } else {
                    y = height - 1 - u;
                    phi = std::atan2((double)y, (double)x);
                }
                const int r_sq = x * x + y * y;
                const int pb = (int)((phi + kRefPi * 0.5f) / kRefPi * (double)(na - 1));   // :94
                int rb = newton_int_sqrt(((double)r_sq) / rbss);                            // :96
                if (rb == nr) rb--;                                                         // :97
                if (pb < 0 || pb >= na || rb < 0 || rb >= nr) {
                    bad[tid] = 1;
                    continue;
                }
                const int b = pb * nr + rb;
                map[(size_t)x * height + u] = (uint16_t)b;
                part[tid][b]++;
            }
        }
    };
    std::vector<std::thread> th;
    for (unsigned i = 1; i < nth; i++) th.emplace_back(work, i);
    work(0);
    for (auto& x : th) x.join();
    for (unsigned i = 0; i < nth; i++)
        if (bad[i]) {
            set_error("a spectrum element falls outside the polar bin table (the reference writes out "
                      "of bounds here, src/blur_profile.c:97-99)");
            return false;
        }
    t->counts.assign((size_t)na * nr, 0);
    for (unsigned i = 0; i < nth; i++)
        for (size_t b = 0; b < t->counts.size(); b++) t->counts[b] += part[i][b];
    if (!upload) {
        t->map = std::move(map);
        return true;
    }
    // + kBinMapPad bytes: the runtime-plan column kernels may load a run of bin
    // ids past the last column's end
    if (hipMalloc(&t->d_map, map.size() * sizeof(uint16_t) + kBinMapPad) != hipSuccess) {
        set_error("hipMalloc of the blur bin table failed");
        return false;
    }
    if (hipMemcpy(t->d_map, map.data(), map.size() * sizeof(uint16_t), hipMemcpyHostToDevice) != hipSuccess) {
        set_error("upload of the blur bin table failed");
        return false;
    }
    t->map = std::move(map);
    return true;
}

bool build_col_runs(const uint16_t* map, int height, int wf, int T, ColRuns* r) {
    const int H = height, E = (H + T - 1) / T;
    std::vector<int> nrun(wf, 0);
    int stride = 0;
    for (int x = 0; x < wf; x++) {
        const uint16_t* col = map + (size_t)x * H;
        int n = 1;
        for (int u = 1; u < H; u++) n += col[u] != col[u - 1];
        nrun[x] = n;
        stride = std::max(stride, n + 1);                  // + the sentinel
    }
    r->max_entries = stride;
    // (E <= 24: a thread's run-start rows are bits 8 .. 31 of its segment word)
    if (stride > kColRunsMax || H > 65535 || E > 24) {
        r->too_many = true;                                // a fixed property of the size: cached
        return false;
    }
    std::vector<uint32_t> runs((size_t)wf * stride, (uint32_t)H << 16);
    std::vector<uint32_t> seg((size_t)wf * T, 0u);
    for (int x = 0; x < wf; x++) {
        const uint16_t* col = map + (size_t)x * H;
        uint32_t* rl = runs.data() + (size_t)x * stride;
        int k = 0;
        for (int u = 0; u < H; u++) {
            const bool start = u == 0 || col[u] != col[u - 1];
            if (start) rl[k++] = ((uint32_t)u << 16) | col[u];
            // thread t's first row t E lies in run k - 1; a run starting at its
            // row j > 0 sets bit 8 + j
            if (u % E == 0) seg[(size_t)x * T + u / E] = (uint32_t)(k - 1);
            else if (start) seg[(size_t)x * T + u / E] |= 1u << (8 + u % E);
        }
        rl[k] = (uint32_t)H << 16;                         // sentinel (its bin is never read)
    }
    if (hipMalloc(&r->d_runs, runs.size() * sizeof(uint32_t)) != hipSuccess ||
        hipMalloc(&r->d_seg, seg.size() * sizeof(uint32_t)) != hipSuccess ||
        hipMemcpy(r->d_runs, runs.data(), runs.size() * sizeof(uint32_t), hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(r->d_seg, seg.data(), seg.size() * sizeof(uint32_t), hipMemcpyHostToDevice) != hipSuccess) {
        set_error("upload of the column bin runs failed");
        if (r->d_runs) (void)hipFree(r->d_runs);
        if (r->d_seg) (void)hipFree(r->d_seg);
        r->d_runs = nullptr;
        r->d_seg = nullptr;
        return false;
    }
    r->T = T;
    r->stride = stride;
    return true;
}

void vectorize_blur(const double* bins, int na, int nr, double streak, double mag, int denom,
                    Blur_Vector* out) {
    for (int i = 0; i < 10; i++) out[i] = Blur_Vector{0, 0.0f};   // calloc, :297-302
    std::vector<double> tot(na, 0.0), sm(na, 0.0);
    const int rc = nr / denom;                                     // :342
    double avg = 0;
    for (int i = 0; i < na; i++) {
        for (int j = 0; j < rc; j++) tot[i] += bins[(size_t)i * nr + j];
        avg += tot[i];
    }
    avg /= na;
    // convolve_1d with the 5-tap box of ones, then /5 (src/filtering.c:12-24)
    for (int i = 0; i < na; i++) {
        for (int j = 0; j < 5; j++) sm[i] += tot[((i - j) % na + na) % na] * 1.0;
        sm[i] /= 5;
    }
    int idx[10], m = 0;
    const double thr = avg * streak;
    if (sm[0] > sm[na - 1] && sm[0] > sm[1] && sm[0] > thr && m < 10) idx[m++] = 0;
    for (int i = 1; i < na - 1; i++)
        if (sm[i] > sm[i - 1] && sm[i] > sm[i + 1] && sm[i] > thr && m < 10) idx[m++] = i;
    if (sm[na - 1] > sm[na - 2] && sm[na - 1] > sm[0] && sm[na - 1] > thr && m < 10) idx[m++] = na - 1;
    for (int i = 0; i < m; i++) {
        const int a = (idx[i] + na / 2) % na;                      // :387
        const double* sig = bins + (size_t)a * nr;
        double bavg = 0;
        for (int j = 0; j < rc; j++) bavg += sig[j];
        if (bavg > avg) {                                          // :396-400
            out[i] = Blur_Vector{0, 0.0f};
            continue;
        }
        int rmax = nr;
        for (int j = 0; j < nr; j++)
            if (sig[j] < mag) {
                rmax = j;
                break;
            }
        out[i].magnitude = ((float)rmax / (float)nr);
        out[i].angle = (int)(180 * ((float)a / (float)na) - 90);
    }
}

}  // namespace phd

extern "C" Image_PGM* get_blur_profile_visual(Blur_Profile* bp, int height, int width) {
    // src/blur_profile.c:140-180, element for element
    if (!bp || height <= 0 || width <= 0) {
        phd::set_error("get_blur_profile_visual: bad arguments");
        return nullptr;
    }
    Image_PGM* img = (Image_PGM*)malloc(sizeof(Image_PGM));
    if (!img) return nullptr;
    img->height = height;
    img->width = width;
    img->data = (Pixel*)malloc((size_t)height * width * sizeof(Pixel));
    if (!img->data) {
        free(img);
        phd::set_error("get_blur_profile_visual: out of memory");
        return nullptr;
    }
    // independent per element: blocks of rows on the host pool (every element
    // is the same sequence of double operations as the reference's loop)
    constexpr int kRows = 64;
    auto rows = [&](int blk) {
        const int y1 = std::min(height, (blk + 1) * kRows);
        for (int y = blk * kRows; y < y1; y++)
            for (int x = 0; x < width; x++) {
                const double dx = x;
                const double dy = (y < height / 2) ? -y : (double)(height - y);
                const double r = std::sqrt(dx * dx + dy * dy);
                const double phi = std::atan2(dy, dx);
                int rb = (int)(r / bp->radius_bin_size);
                if (rb >= bp->num_radius_bins) rb = bp->num_radius_bins - 1;
                int pb = (int)((phi + phd::kRefPi * 0.5f) / phd::kRefPi * (double)(bp->num_angle_bins - 1));
                if (pb >= bp->num_angle_bins) pb = bp->num_angle_bins - 1;
                if (pb < 0) pb = 0;
                img->data[(size_t)y * width + x] = bp->bins[pb][rb];
            }
    };
    const int nblk = (height + kRows - 1) / kRows;
    phd::HostPool* pool = phd::host_pool();
    if (pool->size() > 0 && (long)height * width >= (1L << 16)) pool->parallel_for(nblk, rows);
    else
        for (int b = 0; b < nblk; b++) rows(b);
    return img;
}

extern "C" void phd_free_pgm(Image_PGM* img) {
    if (!img) return;
    free(img->data);
    free(img);
}

extern "C" int phd_debug_col_runs_max(int height, int width, int radius_partitions, int angle_partitions) {
    phd::BlurTable t;
    if (height < 2 || width < 2 || radius_partitions < 1 || angle_partitions < 1 ||
        !phd::build_blur_table(height, width, radius_partitions, angle_partitions, &t, false))
        return -1;
    int mx = 0;
    for (int x = 0; x < t.wf; x++) {
        const uint16_t* col = t.map.data() + (size_t)x * t.height;
        int n = 1;
        for (int u = 1; u < t.height; u++) n += col[u] != col[u - 1];
        mx = std::max(mx, n + 1);
    }
    return mx;
}
