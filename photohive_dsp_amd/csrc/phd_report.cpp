// phd_report.cpp -- the report pipeline and the exported C-ABI.
//
// Stage order of get_full_report_data (src/interface.c:20-94), per batch of
// same-size device images on one stream:
//
//   K1  hsv/stats/histogram           every image        (palette.hip)
//   D2H group histograms + moments    -> host decisions  (phd_palette.cpp)
//   K4  FFT rows, K5 FFT columns      every image        (fft.hip)   || host decides
//   H2D keep rules;  Kcut; K3 sums    every image        (palette.hip)
//   sharpness (crops only)                                (sharpness.hip)
//   D2H bins / max / palette sums -> host finalisation (G_s, averages, vectors)
//
// The FFT of an image depends only on K1's channel sums (for the DC bias), so
// the host's palette decisions overlap the GPU's FFT work.
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <thread>
#include <unistd.h>
#include <unordered_map>
#include <unordered_set>

#include "phd_host.h"

namespace phd {

namespace {

constexpr size_t kAlign = 256;
size_t al(size_t x) { return (x + kAlign - 1) / kAlign * kAlign; }

struct Layout {
    // per-image records
    size_t a_sums, a_hist, a_spart, a_gsum, a_gcell, a_bytes;  // read back after K1 (zeroed)
    size_t c_bins, c_fmax, c_pal, c_sharp, c_bytes;         // read back at the end (zeroed)
    size_t b_rules, b_search, b_off, b_bytes;               // uploaded before K3
    size_t chunk_bytes;                                      // device only
    size_t ptr_bytes;                                        // image pointer array (pinned -> device)
    size_t e_entries, e_ns, e_bytes;                         // Kcut (image, group) list + slots per image
    size_t dev_total, pin_total;
    size_t A(int i) const { return (size_t)i * a_bytes; }
    size_t C(int n, int i) const { return (size_t)n * a_bytes + (size_t)i * c_bytes; }
    size_t B(int n, int i) const { return (size_t)n * (a_bytes + c_bytes) + (size_t)i * b_bytes; }
    // E follows the B records on both sides, so one H2D copy carries both
    size_t E_dev(int n) const { return (size_t)n * (a_bytes + c_bytes + b_bytes); }
    size_t E_pin(int n) const { return E_dev(n); }
    size_t H(int n, int i) const { return E_dev(n) + e_bytes + (size_t)i * chunk_bytes; }
    size_t P_dev(int n) const { return H(n, n); }
    size_t P_pin(int n) const { return E_pin(n) + e_bytes; }
};

// ncell > 0: the fused palette's per-group sums and hue-cell counts ride in
// the K1 record.
Layout make_layout(int n, int tl, int nchunks, int nbins, int ncrops, int ncolblocks, int ncell = 0) {
    Layout L{};
    L.a_sums = 0;
    L.a_hist = al(6 * sizeof(unsigned long long));
    L.a_spart = L.a_hist + al(sizeof(unsigned) * tl);
    L.a_gsum = L.a_spart + al(sizeof(double) * nchunks);
    L.a_gcell = L.a_gsum + (ncell > 0 ? al(sizeof(double) * 3 * tl) : 0);
    L.a_bytes = L.a_gcell + (ncell > 0 ? al(sizeof(unsigned) * ncell) : 0);
    L.c_bins = 0;
    L.c_fmax = al(sizeof(double) * nbins);
    L.c_pal = L.c_fmax + al(sizeof(double) * (ncolblocks > 0 ? ncolblocks : 1));
    L.c_sharp = L.c_pal + al(sizeof(double) * 4 * tl);
    L.c_bytes = L.c_sharp + al(sizeof(double) * 2 * (ncrops > 0 ? ncrops : 1));
    L.b_rules = 0;
    L.b_search = al(sizeof(GroupRule) * tl);
    L.b_off = L.b_search + al(sizeof(int) * tl);
    L.b_bytes = L.b_off + al(sizeof(double) * tl);
    L.chunk_bytes = al(sizeof(unsigned short) * (size_t)nchunks * tl);
    L.ptr_bytes = al(sizeof(void*) * (size_t)n);
    L.e_entries = 0;
    L.e_ns = al(2 * sizeof(int) * (size_t)n * tl);
    L.e_bytes = L.e_ns + al(sizeof(int) * (size_t)n);
    L.dev_total = (size_t)n * (L.a_bytes + L.c_bytes + L.b_bytes + L.chunk_bytes) + L.ptr_bytes + L.e_bytes;
    L.pin_total = (size_t)n * (L.a_bytes + L.c_bytes + L.b_bytes) + L.ptr_bytes + L.e_bytes;
    return L;
}

}  // namespace

// shared with the planar path (phd_planar.cpp)
bool check_crops(const Crop_Boundaries* cb, int height, int width) {
    if (!cb) return true;
    if (cb->N < 0 || (cb->N > 0 && (!cb->top || !cb->bottom || !cb->left || !cb->right))) {
        set_error("Crop_Boundaries has NULL arrays");
        return false;
    }
    for (int k = 0; k < cb->N; k++) {
        const int t = cb->top[k], b = cb->bottom[k], l = cb->left[k], r = cb->right[k];
        // crop_pgm's bounds test (src/image_processing.c:215-218); an empty or
        // inverted box makes the reference divide by zero / misallocate.
        if (r > width || l > width || b > height || t > height || l < 0 || r < 0 || t < 0 || b < 0 ||
            r <= l || b <= t) {
            set_error("crop boundaries outside of image boundaries (crop " + std::to_string(k) + ")");
            return false;
        }
    }
    return true;
}

// pre_compute_error_checks (src/utilities.c:64-87) on the dimensions.
bool precheck(int height, int width) {
    if (height < 350 || width < 350) {
        set_error("Error: Image height and width must be greater than 350. Height: " + std::to_string(height) +
                  "\tWidth" + std::to_string(width));
        return false;
    }
    if ((long long)height * width > 120000000LL) {
        set_error("Error: Image must have less than 120000000 pixels.");
        return false;
    }
    const float ar = (float)height / (float)width;
    if (ar < 1.0 / 5.0 || ar > 5.0 / 1.0) {
        set_error("Error: Invalid aspect ratio: " + std::to_string(ar));
        return false;
    }
    return true;
}

long hsv_count(int height, int width, int ds) {
    const int hh = ds > 1 ? height / ds : height, ww = ds > 1 ? width / ds : width;
    return (long)(short)hh * (short)ww;
}

float ms_between(hipEvent_t a, hipEvent_t b) {
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, a, b) != hipSuccess) return -1.f;
    return ms;
}

// pgm_normalize_fft's G_s (src/fft_processing.c:192) applied to the binned
// sums of log(p); calculate_blur_profile's averaging (src/blur_profile.c:106-116);
// vectorize_blur_profile (src/blur_profile.c:324-416).  flat: na x nr.
void finish_blur(const BlurTable& tbl, const unsigned long long* bin_sums, double fmax, const phd_config& cfg,
                 double* flat, Blur_Vector* vectors, double bscale = 0.0) {
    const int na = cfg.angle_partitions, nr = cfg.radius_partitions;
    const double gs = 1 / (2 * std::log(std::sqrt(fmax) + 1));
    const double scale = bscale > 0.0 ? bscale : bin_scale(tbl.height, tbl.wf);
    for (size_t b = 0; b < (size_t)na * nr; b++) {
        const double q = (double)tbl.counts[b];
        // the device sums are bin_scale fixed point (order-independent)
        const double sum = bin_sums[b] == 0ull ? 0.0 : (double)bin_sums[b] / scale * gs;
        flat[b] = q != 0 ? sum / q : 0;
    }
    vectorize_blur(flat, na, nr, cfg.fft_streak_thresh, cfg.magnitude_thresh, cfg.blur_cutoff_ratio_denom, vectors);
}

namespace {

// A report is one heap block (a 16-byte header with its size, then every
// structure and array of Full_Report_Data), and free_full_report hands the
// block to a pool that the next report of the same size takes it from: a
// 256-image batch's 3,000 separate mallocs and frees (and the heap trims and
// page faults between batches) cost ~0.9 ms per batch with the GPU idle.
constexpr size_t kReportHdr = 16;
constexpr unsigned long long kReportMagic = 0x5048445245504f52ull;   // "PHDREPOR"
// The pool also keeps the set of blocks that are live reports: free_full_report
// pools a block only if it is in that set, so a pointer this library did not
// return (or a report already freed and not yet handed out again) is ignored
// without reading memory around it.  A stale pointer to a block that a later
// report has taken again cannot be told from that report (as with free()):
// freeing it twice after such a reuse is undefined.
struct ReportPool {
    pid_t pid = 0;                                           // the process that made this pool
    std::mutex m;
    std::unordered_map<size_t, std::vector<void*>> blocks;   // by block size
    std::unordered_set<const void*> live;                    // blocks handed out as reports
    size_t bytes = 0;
    static constexpr size_t kCap = (size_t)512 << 20;        // pooled bytes at most
    void* take(size_t sz) {
        void* b = nullptr;
        {
            std::lock_guard<std::mutex> lk(m);
            auto it = blocks.find(sz);
            if (it != blocks.end() && !it->second.empty()) {
                b = it->second.back();
                it->second.pop_back();
                bytes -= sz;
            }
        }
        if (!b) b = malloc(sz);
        if (b) {
            std::lock_guard<std::mutex> lk(m);
            live.insert(b);
        }
        return b;
    }
    // returns false (and leaves the block alone) when b is not a live report
    bool give(void* b) {
        std::lock_guard<std::mutex> lk(m);
        if (!live.erase(b)) return false;
        const size_t sz = (size_t)reinterpret_cast<unsigned long long*>(b)[0];
        reinterpret_cast<unsigned long long*>(b)[1] = 0;
        if (bytes + sz > kCap) {
            free(b);
            return true;
        }
        blocks[sz].push_back(b);
        bytes += sz;
        return true;
    }
};
ReportPool& report_pool() {
    // process lifetime (reports may be freed at exit); a forked child starts a
    // pool of its own (the parent's mutex may have been held at the fork).  One
    // pointer holds both the pool and the pid that made it, so a thread cannot
    // pair one process's pool with another's pid.
    static std::atomic<ReportPool*> p{nullptr};
    ReportPool* q = p.load(std::memory_order_acquire);
    const pid_t me = getpid();
    if (!q || q->pid != me) {
        static std::mutex init;
        std::lock_guard<std::mutex> lk(init);
        q = p.load(std::memory_order_acquire);
        if (!q || q->pid != me) {
            q = new ReportPool;
            q->pid = me;
            p.store(q, std::memory_order_release);
        }
    }
    return *q;
}
size_t al16(size_t x) { return (x + 15) & ~(size_t)15; }

}  // namespace

Full_Report_Data* assemble(const RGB_Statistics& st, double s_bar, const PaletteDecision& dec,
                           const double* pal, long n_hsv, const BlurTable& tbl, const unsigned long long* bin_sums,
                           double fmax, const phd_config& cfg, const Crop_Boundaries* crops,
                           const double* sharp_sums, std::string* why, double bscale) {
    const int np = (int)dec.parents.size();
    const int na = cfg.angle_partitions, nr = cfg.radius_partitions;
    const int nsh = crops ? (crops->N > 0 ? crops->N : 1) : 0;
    // the block: header | report | stats | palette + arrays | profile + row
    // pointers + rows | vector group + 10 vectors | sharpnesses + values
    size_t o = kReportHdr;
    const size_t o_r = o; o = al16(o + sizeof(Full_Report_Data));
    const size_t o_rs = o; o = al16(o + sizeof(RGB_Statistics));
    const size_t o_cp = o; o = al16(o + sizeof(Color_Palette));
    const size_t o_avg = o; o = al16(o + sizeof(Pixel_HSV) * (np > 0 ? np : 1));
    const size_t o_pct = o; o = al16(o + sizeof(double) * (np > 0 ? np : 1));
    const size_t o_bp = o; o = al16(o + sizeof(Blur_Profile));
    const size_t o_bptr = o; o = al16(o + sizeof(Bin*) * (na > 0 ? na : 1));
    const size_t o_rows = o; o = al16(o + sizeof(Bin) * ((size_t)na * nr > 0 ? (size_t)na * nr : 1));
    const size_t o_bv = o; o = al16(o + sizeof(Blur_Vector_Group));
    const size_t o_vec = o; o = al16(o + sizeof(Blur_Vector) * 10);
    const size_t o_sh = o; o = al16(o + (crops ? sizeof(Sharpnesses) : 0));
    const size_t o_shv = o; o = al16(o + sizeof(Pixel) * (size_t)nsh);
    const size_t size = (o + 4095) & ~(size_t)4095;           // a few size classes for the pool
    char* blk = (char*)report_pool().take(size);
    if (!blk) {
        *why = "report allocation failed";
        return nullptr;
    }
    reinterpret_cast<unsigned long long*>(blk)[0] = size;
    reinterpret_cast<unsigned long long*>(blk)[1] = kReportMagic;
    // calculate_avg_hsv (src/color_quantization.c:510-576)
    Color_Palette* cp = (Color_Palette*)(blk + o_cp);
    cp->N = np;
    cp->averages = (Pixel_HSV*)(blk + o_avg);
    cp->percentages = (double*)(blk + o_pct);
    const double inv_n = 1.0 / (int)n_hsv;
    for (int k = 0; k < np; k++) {
        const double cnt = pal[4 * k + 3];
        static const bool ablating = phd_knob("PHD_ABLATE") != nullptr;   // timing experiments only
        if (cnt != (double)dec.kept[k] && !ablating) {
            *why = "palette self-check failed: device kept " + std::to_string((long long)cnt) +
                   " pixels for slot " + std::to_string(k) + ", host rules predict " +
                   std::to_string(dec.kept[k]);
            report_pool().give(blk);
            return nullptr;
        }
        const int tot = (int)dec.kept[k];
        const double inv = 1.0 / (double)tot;
        double h = pal[4 * k + 0] * inv;
        h -= dec.off[k];
        if (h < 0) h += 360;
        else if (h > 360) h -= 360;
        cp->averages[k].parent_id = dec.parents[k];   // uninitialised in the reference
        cp->averages[k].h = h;
        cp->averages[k].s = pal[4 * k + 1] * inv;
        cp->averages[k].v = pal[4 * k + 2] * inv;
        cp->percentages[k] = (double)tot * inv_n;
    }
    // pgm_normalize_fft's G_s (src/fft_processing.c:192) applied to the binned
    // sums of log(p); calculate_blur_profile's averaging (src/blur_profile.c:106-116)
    Blur_Profile* bp = (Blur_Profile*)(blk + o_bp);
    bp->num_angle_bins = na;
    bp->num_radius_bins = nr;
    bp->angle_bin_size = tbl.angle_bin_size;
    bp->radius_bin_size = tbl.radius_bin_size;
    // bins[angle][radius] as the reference's row pointers into one run of rows
    bp->bins = (Bin**)(blk + o_bptr);
    Bin* rows = (Bin*)(blk + o_rows);                          // finish_blur writes every bin
    for (int a = 0; a < na; a++) bp->bins[a] = rows + (size_t)a * nr;
    Blur_Vector_Group* bv = (Blur_Vector_Group*)(blk + o_bv);
    bv->len_vectors = 10;
    bv->blur_vectors = (Blur_Vector*)(blk + o_vec);
    memset(bv->blur_vectors, 0, sizeof(Blur_Vector) * 10);    // calloc in the reference
    finish_blur(tbl, bin_sums, fmax, cfg, rows, bv->blur_vectors, bscale);
    Sharpnesses* sh = nullptr;
    if (crops) {   // get_variance_sharpness (src/filtering.c:151-183)
        sh = (Sharpnesses*)(blk + o_sh);
        sh->N = crops->N;
        sh->sharpness = (Pixel*)(blk + o_shv);
        memset(sh->sharpness, 0, sizeof(Pixel) * (size_t)nsh);
        for (int k = 0; k < crops->N; k++) {
            const double cn = (double)((long)(crops->right[k] - crops->left[k]) *
                                       (crops->bottom[k] - crops->top[k]));
            const double avg = sharp_sums[2 * k] / cn;
            const double var = sharp_sums[2 * k + 1] / cn;
            sh->sharpness[k] = var / avg;
        }
    }
    RGB_Statistics* rs = (RGB_Statistics*)(blk + o_rs);
    *rs = st;
    Full_Report_Data* r = (Full_Report_Data*)(blk + o_r);
    r->rgb_stats = rs;
    r->color_palette = cp;
    r->blur_profile = bp;
    r->blur_vectors = bv;
    r->average_saturation = s_bar;
    r->sharpness = sh;
    return r;
}

namespace {

RGB_Statistics stats_from_sums(const unsigned long long* m, long n) {
    // mean = sum(k)/255/N; population variance from exact integer moments:
    // var = (N*sum(k^2) - sum(k)^2) / (255^2 N^2)   (filtering.c:125-148 in exact arithmetic)
    RGB_Statistics s;
    double* out = &s.Br;
    for (int c = 0; c < 3; c++) {
        out[c] = (double)m[c] / 255.0 / (double)n;
        const unsigned __int128 num = (unsigned __int128)n * m[3 + c] - (unsigned __int128)m[c] * m[c];
        const double var = (double)num / 65025.0 / ((double)n * (double)n);
        out[3 + c] = std::sqrt(var);
    }
    return s;
}

}  // namespace

bool all_aligned(const uint8_t* const* p, int n) {
    for (int i = 0; i < n; i++)
        if (reinterpret_cast<uintptr_t>(p[i]) & 3) return false;
    return true;
}

// K1 for n same-size images: one batched launch (ds == 1) over the device
// pointer array staged in the workspace, or per-image launches (ds > 1).
bool launch_k1(Context* c, const Layout& L, int n, const uint8_t* const* d_imgs, int height, int width, int ds,
               const GridParams& gp, const Context::Cls* cls, int nchunks, bool fused, hipStream_t st) {
    uint8_t* dw = (uint8_t*)c->d_ws;
    uint8_t* hp = (uint8_t*)c->h_pin;
    PaletteDev pd;
    pd.sums = (unsigned long long*)(dw + L.A(0) + L.a_sums);
    pd.hist = (unsigned*)(dw + L.A(0) + L.a_hist);
    pd.s_part = (double*)(dw + L.A(0) + L.a_spart);
    pd.chunk_hist = (unsigned short*)(dw + L.H(n, 0));
    pd.gsum = (double*)(dw + L.A(0) + L.a_gsum);
    pd.gcell = (unsigned*)(dw + L.A(0) + L.a_gcell);
    // the device image-pointer array: K1 (ds == 1), the batched runtime-plan FFT
    // passes and the batched palette tail read it, whatever the downsample rate
    memcpy(hp + L.P_pin(n), d_imgs, sizeof(void*) * n);
    PHD_HIP(hipMemcpyAsync(dw + L.P_dev(n), hp + L.P_pin(n), sizeof(void*) * n, hipMemcpyHostToDevice, st));
    const int ps = c->prof.begin(kK1, st);
    if (ds <= 1) {
        PHD_HIP(launch_hsv_stats_batch((const uint8_t* const*)(dw + L.P_dev(n)), n, height, width, gp, cls->fc,
                                       cls->d, pd, (long)L.a_bytes, (long)L.chunk_bytes, nchunks, c->d_k255,
                                       true, fused, all_aligned(d_imgs, n), st));
    } else {
        for (int i = 0; i < n; i++) {
            PaletteDev pi;
            pi.sums = (unsigned long long*)(dw + L.A(i) + L.a_sums);
            pi.hist = (unsigned*)(dw + L.A(i) + L.a_hist);
            pi.s_part = (double*)(dw + L.A(i) + L.a_spart);
            pi.chunk_hist = (unsigned short*)(dw + L.H(n, i));
            PHD_HIP(launch_hsv_ds(d_imgs[i], height, width, ds, gp, cls->fc, cls->d, pi, nchunks, c->d_k255, st));
        }
    }
    c->prof.end(ps, st);
    return true;
}

// calculate_avg_hsv's slot sums (src/color_quantization.c:520-550) of every
// group a slot keeps whole, from the fused K1's per-group records: sum over
// the group of wrap(h + off) = sum(h) + n * off - 360 * #(h + off > 360)
// + 360 * #(h + off < 0), the wrap counts being sums of hue-cell counts on
// one side of the parent's threshold (HueCells).  Partial groups are left to
// the device (k_partial_sums_b).  Adds into hs[4 * slot + {h, s, v, n}].
bool fused_slot_sums(const GridParams& gp, const PaletteDecision& dec, const unsigned* hist, const double* gsum,
                     const unsigned* gcell, double* hs, std::string* why) {
    const int tl = gp.tl, gs = HueCells::gray_start(gp), hp = gp.hp, sv = gp.sp * gp.vp;
    for (int g = 0; g < tl; g++) {
        const GroupRule& r = dec.rules[g];
        if (r.slot < 0 || r.partial || hist[g] == 0) continue;
        const int k = r.slot, p = dec.parents[k];
        // the parent's threshold cell cT and direction: +1 wraps down (-360)
        // above cT, -1 wraps up (+360) below cT, 0 never
        int cT = 0, dir = 0;
        if (p >= gs) {
            cT = hp;                                   // h = 0, off = 180: h > 180 wraps
            dir = 1;
        } else {
            const int t = 2 * (p / sv) + 1;            // 2 * h_parent / Lh
            if (t < hp) { cT = t + hp; dir = 1; }
            else if (t > hp) { cT = t - hp; dir = -1; }
        }
        long long tot = 0, above = 0;
        auto cell = [&](int cg, unsigned cnt) {
            tot += cnt;
            if (cg >= cT) above += cnt;
        };
        if (g < gs) {
            const int hi = g / sv;
            for (int l = 0; l < 4; l++) cell(std::max(0, 2 * hi - 1 + l), gcell[4 * g + l]);
        } else {
            for (int cg = 0; cg < 2 * hp; cg++) cell(cg, gcell[4 * gs + (g - gs) * 2 * hp + cg]);
        }
        if (tot != (long long)hist[g]) {
            *why = "fused palette self-check failed: hue cells of group " + std::to_string(g) + " hold " +
                   std::to_string(tot) + " pixels, the histogram " + std::to_string(hist[g]);
            return false;
        }
        const double n = (double)hist[g];
        double wrap = 0.0;
        if (dir > 0) wrap = -360.0 * (double)above;
        else if (dir < 0) wrap = 360.0 * (double)(tot - above);
        hs[4 * k + 0] += gsum[g] + n * dec.off[k] + wrap;
        hs[4 * k + 1] += gsum[tl + g];
        hs[4 * k + 2] += gsum[2 * tl + g];
        hs[4 * k + 3] += n;
    }
    return true;
}

bool run_reports(Context* c, const uint8_t* const* d_imgs, int n, int height, int width,
                 const phd_config& cfg, const Crop_Boundaries* crops, Full_Report_Data** out, int* status,
                 hipStream_t stream) {
    const auto t_host0 = std::chrono::steady_clock::now();
    for (int i = 0; i < n; i++) {
        out[i] = nullptr;
        status[i] = -1;
    }
    std::string why;
    if (!validate_config(cfg, &why)) {
        set_error(why);
        return false;
    }
    if (!precheck(height, width) || !check_crops(crops, height, width)) return false;
    const hipStream_t st = work_stream(c, stream);
    // ev_img_fft only orders the download stream after a column pass on this
    // device (device_event_flags: no system-scope fence)
    while ((int)c->ev_img_fft.size() < n) {
        hipEvent_t a, b;
        PHD_HIP(hipEventCreateWithFlags(&a, device_event_flags()));
        PHD_HIP(hipEventCreateWithFlags(&b, hipEventDisableTiming));
        c->ev_img_fft.push_back(a);
        c->ev_img_dl.push_back(b);
    }
    // a failed earlier call may have left work on the side stream
    PHD_HIP(hipStreamSynchronize(c->tail));
    const GridParams gp = make_grid(cfg);
    const int ds = cfg.downsample_rate > 1 ? cfg.downsample_rate : 1;
    const long n_hsv = hsv_count(height, width, ds);
    const int nchunks = (int)((n_hsv + kChunk - 1) / kChunk);
    const int nbins = cfg.radius_partitions * cfg.angle_partitions;
    const int ncrops = crops ? crops->N : 0;
    const int wf = width / 2 + 1;
    const BlurTable* tbl = get_table(c, height, width, cfg.radius_partitions, cfg.angle_partitions);
    if (!tbl) return false;
    FftSel fs;
    // compile-time plans: images small enough that two or more half-spectrum
    // intermediates fit 128 MB (half the MALL) run as one row and one column
    // launch per group of images (sizes whose row pairs form whole line groups
    // of the row schedule); small images are otherwise bound by per-launch costs
    const size_t inter_one = sizeof(double2) * inter_elems(height, width);
    static const bool ctbatch_off = phd_knob("PHD_CT_NO_BATCH") != nullptr;
    const int q_ct = (int)std::min<size_t>((size_t)n, ((size_t)128 << 20) / inter_one);
    const bool ct_batchable = !ctbatch_off && n > 1 && q_ct >= 2 && ((height + 1) / 2) % 4 == 0;
    if (!select_fft(c, height, width, nbins, d_imgs, n, &fs, tbl, ct_batchable)) return false;
    const Context::Cls* cls = get_cls(c, gp);
    if (!cls) return false;
    // the column pass's full-prefetch form (24 KB more LDS per block): on a
    // call split over two lanes whose K1 runs the two-block form (one
    // 512-thread block per CU beside the other lane's FFTs) the half-prefetch
    // form measured 9.05k images/s against its 8.67k at 4000x3000, 18/2/3,
    // where FFT-only calls and the fine grids' one-block K1 gain with the full
    // form
    if (FftSel::forced_form() < 0 && ds <= 1 && k1_blocks_per_cu() == 1 && cls->fc.k1t_cshift2 >= 0)
        fs.col_pf = false;

    const int ncolblocks = fs.col_blocks;
    // images whose result records go to the host together (one event and one
    // copy per group; the last image always ends a group).  Each event between
    // back-to-back FFT kernels costs ~5 us; larger groups delay the host's
    // assembly of the early images.  Measured at 4000x3000, 8 images: groups
    // of 1 / 2 / 4 / 8 give FFT stages of 0.857 / 0.838 / 0.828 / 0.823 ms and
    // 6.16k / 6.21k / 6.17k / 6.08k images/s.
    static const int dl_group = phd_knob("PHD_DL_GROUP") ? std::max(1, atoi(phd_knob("PHD_DL_GROUP"))) : 2;
    // fused palette (one pixel pass): ds == 1 and the fused K1's LDS fits; else K1 + K3
    const bool fused = ds <= 1 && fused_palette_ok(gp);
    const Layout L = make_layout(n, gp.tl, nchunks, nbins, ncrops, ncolblocks, fused ? HueCells::count(gp) : 0);
    // half-spectrum intermediates: one per image of a group of Q (the group's row
    // passes run before its column passes); large images one at a time, so the
    // intermediate stays in the 256 MB MALL between its two passes (round 2:
    // a two-stream pipeline of rows i+1 beside columns i measured 10 % slower)
    // (+ 1024 elements of scratch past the tiles for the row pass's dummy stores)
    int Q = 1;
    // runtime-plan sizes: the passes of a group of images are one launch each
    // (grid.y = image), the group's intermediates within 128 MB (half the
    // MALL); small images are otherwise bound by per-launch latency
    static const bool gbatch_off = phd_knob("PHD_FFT_NO_BATCH") != nullptr;
    const bool gbatch = !fs.ct && !fs.generic && !gbatch_off && n > 1 && L.a_bytes % 8 == 0 && L.c_bytes % 8 == 0;
    if (gbatch) Q = std::max(1, std::min(n, (int)(((size_t)128 << 20) / inter_one)));
    const bool ctbatch = fs.ct && ct_batchable && L.a_bytes % 8 == 0 && L.c_bytes % 8 == 0;
    if (ctbatch) Q = q_ct;
    // batched FFT launches finish a whole group of Q images at once: one
    // event, one download and one host wait per group (small images were
    // bound by ~3 HIP calls and a wait per pair of images: DESIGN.md section 12)
    const int dlg = gbatch || ctbatch ? Q : dl_group;
    auto dl_end = [&](int i) { return (i + 1) % dlg == 0 || i == n - 1; };
    auto dl_last = [&](int i) { return std::min(n - 1, (i / dlg + 1) * dlg - 1); };
    if (!ensure_device(&c->d_ws, &c->ws_bytes, L.dev_total) || !ensure_pinned(c, L.pin_total) ||
        !ensure_device((void**)&c->d_inter, &c->inter_bytes, (size_t)Q * inter_one))
        return false;
    uint8_t* dw = (uint8_t*)c->d_ws;
    uint8_t* hp = (uint8_t*)c->h_pin;
    std::vector<int> crop_arr;
    if (ncrops) {
        crop_arr.resize(4 * ncrops);
        for (int k = 0; k < ncrops; k++) {
            crop_arr[k] = crops->top[k];
            crop_arr[ncrops + k] = crops->bottom[k];
            crop_arr[2 * ncrops + k] = crops->left[k];
            crop_arr[3 * ncrops + k] = crops->right[k];
        }
    }

    PHD_HIP(hipMemsetAsync(dw, 0, (size_t)n * (L.a_bytes + L.c_bytes), st));
    // An unprofiled one-launch K1 records its stage events with its own
    // dispatch and completion (no marker packets between it and the first row
    // pass), and ev[1] then stands for ev_k1; the A records go down on the
    // download stream, beside the FFTs instead of ahead of them.
    static const bool k1_events_off = phd_knob("PHD_K1_MARKERS") != nullptr;
    const bool k1_own = ds <= 1 && !(c->prof.mask & (1u << kK1)) && !k1_events_off &&
                        device_event_flags() == hipEventDisableSystemFence;
    if (k1_own) launch_events() = LaunchEvents{c->ev[0], c->ev[1], false};
    else PHD_HIP(hipEventRecord(c->ev[0], st));
    const bool k1_ok = launch_k1(c, L, n, d_imgs, height, width, ds, gp, cls, nchunks, fused, st);
    const bool k1_rec = k1_own && launch_events().used;
    if (k1_own) launch_events() = LaunchEvents{};
    if (!k1_ok) return false;
    if (k1_own && !k1_rec) PHD_HIP(hipEventRecord(c->ev[0], st));   // (a K1 path without phd_launch: timing only)
    if (!k1_rec) PHD_HIP(hipEventRecord(c->ev[1], st));
    if (!k1_rec) PHD_HIP(hipEventRecord(c->ev_k1, st));
    const hipEvent_t ev_k1 = k1_rec ? c->ev[1] : c->ev_k1;
    // the A records go down on the side stream (tail), beside the FFTs
    const hipStream_t sa = k1_rec ? c->tail : st;
    if (sa != st) PHD_HIP(hipStreamWaitEvent(sa, ev_k1, 0));
    PHD_HIP(hipMemcpyAsync(hp, dw, (size_t)n * L.a_bytes, hipMemcpyDeviceToHost, sa));
    PHD_HIP(hipEventRecord(c->ev[5], sa));
    // The FFT chain follows K1 on its stream and takes its channel sums (the
    // column pass's DC bias): a cross-stream event wait left the GPU idle
    // ~20 us between K1 and the first row pass.
    const hipStream_t sf = st;
    const size_t inter_elems = inter_one / sizeof(double2);
    for (int g0 = 0; gbatch && g0 < n; g0 += Q) {
        const int g1 = std::min(n, g0 + Q);
        const uint8_t* const* d_ptrs = (const uint8_t* const*)(dw + L.P_dev(n));
        int ps = c->prof.begin(kFftRows, sf);
        PHD_HIP(launch_fft_rows_batch(d_ptrs + g0, g1 - g0, height, width, fs.prow->plan,
                                      (const unsigned long long*)(dw + L.A(g0) + L.a_sums), (long)(L.a_bytes / 8),
                                      c->d_k255, c->d_inter, inter_elems, sf));
        c->prof.end(ps, sf);
        ps = c->prof.begin(kFftCols, sf);
        PHD_HIP(launch_fft_cols_batch(c->d_inter, inter_elems, g1 - g0, height, wf, fs.pcol->plan, tbl->d_map, nbins,
                                      (unsigned long long*)(dw + L.C(n, g0) + L.c_bins),
                                      (double*)(dw + L.C(n, g0) + L.c_fmax),
                                      (long)(L.c_bytes / 8), sf));
        c->prof.end(ps, sf);
        for (int i = g0; i < g1; i++) {
            if (ncrops)
                PHD_HIP(launch_sharpness(d_imgs[i], height, width, ncrops, crop_arr.data(),
                                         crop_arr.data() + ncrops, crop_arr.data() + 2 * ncrops,
                                         crop_arr.data() + 3 * ncrops, c->d_k255,
                                         (double*)(dw + L.C(n, i) + L.c_sharp), sf));
            if (dl_end(i)) PHD_HIP(hipEventRecord(c->ev_img_fft[i], sf));
        }
    }
    for (int g0 = 0; ctbatch && g0 < n; g0 += Q) {
        const int g1 = std::min(n, g0 + Q);
        const uint8_t* const* d_ptrs = (const uint8_t* const*)(dw + L.P_dev(n));
        int ps = c->prof.begin(kFftRows, sf);
        PHD_HIP(launch_fft_rows_ct_batch(d_ptrs + g0, g1 - g0, height, width, c->d_k255, fs.tw_r, c->d_inter,
                                         (long)inter_elems, sf));
        c->prof.end(ps, sf);
        ps = c->prof.begin(kFftCols, sf);
        PHD_HIP(launch_fft_cols_ct_batch(c->d_inter, (long)inter_elems, g1 - g0, height, width, wf, fs.cbins,
                                         (unsigned long long*)(dw + L.C(n, g0) + L.c_bins), (long)(L.c_bytes / 8),
                                         (double*)(dw + L.C(n, g0) + L.c_fmax), (long)(L.c_bytes / 8), fs.tw_c,
                                         (const unsigned long long*)(dw + L.A(g0) + L.a_sums), (long)(L.a_bytes / 8),
                                         sf, fs.col_pf));
        c->prof.end(ps, sf);
        for (int i = g0; i < g1; i++) {
            if (ncrops)
                PHD_HIP(launch_sharpness(d_imgs[i], height, width, ncrops, crop_arr.data(),
                                         crop_arr.data() + ncrops, crop_arr.data() + 2 * ncrops,
                                         crop_arr.data() + 3 * ncrops, c->d_k255,
                                         (double*)(dw + L.C(n, i) + L.c_sharp), sf));
            if (dl_end(i)) PHD_HIP(hipEventRecord(c->ev_img_fft[i], sf));
        }
    }
    for (int g0 = 0; g0 < (gbatch || ctbatch ? 0 : n); g0 += Q) {
        const int g1 = std::min(n, g0 + Q);
        for (int i = g0; i < g1; i++) {
            const unsigned long long* sums = (const unsigned long long*)(dw + L.A(i) + L.a_sums);
            const int ps = c->prof.begin(kFftRows, sf);
            PHD_HIP(launch_rows_sel(fs, d_imgs[i], height, width, sums, c->d_k255,
                                    c->d_inter + (size_t)(i - g0) * inter_elems, sf, nullptr));
            c->prof.end(ps, sf);
        }
        for (int i = g0; i < g1; i++) {
            const unsigned long long* sums = (const unsigned long long*)(dw + L.A(i) + L.a_sums);
            auto* bins = (unsigned long long*)(dw + L.C(n, i) + L.c_bins);
            double* fmx = (double*)(dw + L.C(n, i) + L.c_fmax);
            const int ps = c->prof.begin(kFftCols, sf);
            // an unprofiled column pass that ends a download group records the
            // group's event itself (its completion signal): a separate event
            // record between two kernels leaves the GPU idle ~4 us
            // (compile-time plans only: one launch is the whole column pass)
            const bool own = fs.ct && ps < 0 && dl_end(i) && !ncrops &&
                             device_event_flags() == hipEventDisableSystemFence;
            if (own) launch_events() = LaunchEvents{nullptr, c->ev_img_fft[i], false};
            PHD_HIP(launch_cols_sel(fs, c->d_inter + (size_t)(i - g0) * inter_elems, height, width, wf, tbl->d_map,
                                    nbins, bins, fmx, sums, nullptr, sf));
            const bool recorded = own && launch_events().used;
            if (own) launch_events() = LaunchEvents{};
            c->prof.end(ps, sf);
            if (ncrops) {
                // crop boxes: sharpness on the full-resolution luma before DC removal
                PHD_HIP(launch_sharpness(d_imgs[i], height, width, ncrops, crop_arr.data(),
                                         crop_arr.data() + ncrops, crop_arr.data() + 2 * ncrops,
                                         crop_arr.data() + 3 * ncrops, c->d_k255,
                                         (double*)(dw + L.C(n, i) + L.c_sharp), sf));
            }
            if (dl_end(i) && !recorded) PHD_HIP(hipEventRecord(c->ev_img_fft[i], sf));
        }
    }
    // the last column pass ends the FFT work (it waited for the last row pass)
    PHD_HIP(hipEventRecord(c->ev[2], sf));
    PHD_HIP(hipEventRecord(c->ev_fft, sf));

    // host decisions while the FFTs run
    const auto t_enq = std::chrono::steady_clock::now();
    PHD_HIP(hipEventSynchronize(c->ev[5]));
    const auto t_k1 = std::chrono::steady_clock::now();
    // per-image decision records reused across calls (their vectors keep their
    // capacity: no per-call allocation and release of ~1,500 small vectors)
    if (c->dec_scratch.size() < (size_t)n) c->dec_scratch.resize(n);
    if (c->hsum_scratch.size() < (size_t)n) c->hsum_scratch.resize(n);
    std::vector<PaletteDecision>& dec = c->dec_scratch;
    std::vector<int> ok(n, 1);
    std::vector<std::vector<double>>& hsum = c->hsum_scratch;   // fused: host part of the slot sums
    int* h_ent = (int*)(hp + L.E_pin(n) + L.e_entries);
    int* h_ns = (int*)(hp + L.E_pin(n) + L.e_ns);
    int n_ent = 0, max_slots = 1, max_per_img = 0;
    // per image, independent: the decision, its device records and (fused) the
    // host part of the slot sums; on the host pool when the decisions are
    // costly (fine grids), then the batch-wide lists in image order
    std::vector<std::string> fail_why(n);
    auto decide_one = [&](int i) {
        const unsigned* hist = (const unsigned*)(hp + L.A(i) + L.a_hist);
        uint8_t* b = hp + (size_t)n * (L.a_bytes + L.c_bytes) + (size_t)i * L.b_bytes;
        if (!decide_palette(gp, cls->gc, hist, n_hsv, cfg, &dec[i],
                            cls->near.empty() ? nullptr : cls->near.data())) {
            ok[i] = 0;
            GroupRule* r = (GroupRule*)(b + L.b_rules);     // no slot: pass 2 keeps nothing
            for (int g = 0; g < gp.tl; g++) r[g] = GroupRule{-1, 0, 0, 0, 0xFFFFFFFFu, 0u};
            return;
        }
        memcpy(b + L.b_rules, dec[i].rules.data(), sizeof(GroupRule) * gp.tl);
        memcpy(b + L.b_search, dec[i].search.data(), sizeof(int) * dec[i].search.size());
        memcpy(b + L.b_off, dec[i].off.data(), sizeof(double) * dec[i].off.size());
        if (fused) {
            hsum[i].assign(4 * dec[i].parents.size(), 0.0);
            if (!fused_slot_sums(gp, dec[i], hist, (const double*)(hp + L.A(i) + L.a_gsum),
                                 (const unsigned*)(hp + L.A(i) + L.a_gcell), hsum[i].data(), &fail_why[i]))
                ok[i] = 0;
        }
    };
    HostPool* pool = host_pool();
    if (n >= 4 && gp.tl >= 200 && pool->size() > 0) pool->parallel_for(n, decide_one);
    else
        for (int i = 0; i < n; i++) decide_one(i);
    const auto t_dec_only = std::chrono::steady_clock::now();
    for (int i = 0; i < n; i++) {
        h_ns[i] = 0;
        if (!ok[i]) {
            // the message, on this thread (decide_palette is deterministic)
            if (!fail_why[i].empty()) set_error(fail_why[i]);
            else {
                PaletteDecision d;
                (void)decide_palette(gp, cls->gc, (const unsigned*)(hp + L.A(i) + L.a_hist), n_hsv, cfg, &d);
            }
            continue;
        }
        for (int g : dec[i].search) {
            h_ent[2 * n_ent] = i;
            h_ent[2 * n_ent + 1] = g;
            n_ent++;
        }
        max_per_img = std::max(max_per_img, (int)dec[i].search.size());
        h_ns[i] = (int)dec[i].parents.size();
        max_slots = std::max(max_slots, h_ns[i]);
    }
    // the second pass on the tail stream, after K1, concurrent with the FFTs
    const hipStream_t s2 = c->tail;
    if (sa != s2) PHD_HIP(hipStreamWaitEvent(s2, ev_k1, 0));
    uint8_t* hb = hp + (size_t)n * (L.a_bytes + L.c_bytes);
    const bool batched = ds <= 1 && (fused || palette_sums_b_lds(gp.tl, max_slots) <= 160 * 1024);
    // the B records (and, batched, the Kcut list right after them): one copy
    PHD_HIP(hipMemcpyAsync(dw + L.B(n, 0), hb, (size_t)n * L.b_bytes + (batched ? L.e_bytes : 0),
                           hipMemcpyHostToDevice, s2));
    if (batched) {
        // one Kcut and one K3 launch over the whole batch
        const uint8_t* const* d_ptrs = (const uint8_t* const*)(dw + L.P_dev(n));
        // timing experiments only: PHD_ABLATE bit 1024 skips the tail kernels (wrong palette sums)
        const bool skip_tail = (env_ablate() & 1024) != 0;
        int ps = n_ent ? c->prof.begin(kCutoffs, s2) : -1;
        if (!skip_tail) PHD_HIP(launch_cutoffs_batch(d_ptrs, d_imgs, n, height, width, gp, cls->fc, cls->d, c->d_k255,
                                     (const int2*)(dw + L.E_dev(n) + L.e_entries), n_ent,
                                     (const unsigned short*)(dw + L.H(n, 0)), (long)L.chunk_bytes,
                                     (GroupRule*)(dw + L.B(n, 0) + L.b_rules), (long)L.b_bytes, s2));
        c->prof.end(ps, s2);
        if (fused) {
            // only the partial groups' kept prefixes are left to sum on the device
            ps = n_ent ? c->prof.begin(kPalSums, s2) : -1;
            if (!skip_tail) PHD_HIP(launch_partial_sums_batch(d_ptrs, d_imgs, n, height, width, gp, cls->fc, cls->d, c->d_k255,
                                              (const int2*)(dw + L.E_dev(n) + L.e_entries), n_ent,
                                              (const unsigned short*)(dw + L.H(n, 0)), (long)L.chunk_bytes,
                                              (const GroupRule*)(dw + L.B(n, 0) + L.b_rules),
                                              (const double*)(dw + L.B(n, 0) + L.b_off), (long)L.b_bytes,
                                              (double*)(dw + L.C(n, 0) + L.c_pal), (long)L.c_bytes, max_per_img, s2));
            c->prof.end(ps, s2);
        } else {
            ps = c->prof.begin(kPalSums, s2);
            PHD_HIP(launch_palette_sums_batch(d_ptrs, d_imgs, n, height, width, gp, cls->fc, cls->d, c->d_k255,
                                              (const GroupRule*)(dw + L.B(n, 0) + L.b_rules),
                                              (const double*)(dw + L.B(n, 0) + L.b_off), (long)L.b_bytes,
                                              (const int*)(dw + L.E_dev(n) + L.e_ns), max_slots,
                                              (double*)(dw + L.C(n, 0) + L.c_pal), (long)L.c_bytes, s2));
            c->prof.end(ps, s2);
        }
    } else {
        for (int i = 0; i < n; i++) {
            if (!ok[i]) continue;
            GroupRule* rules = (GroupRule*)(dw + L.B(n, i) + L.b_rules);
            const int* search = (const int*)(dw + L.B(n, i) + L.b_search);
            const double* off = (const double*)(dw + L.B(n, i) + L.b_off);
            int ps = dec[i].search.empty() ? -1 : c->prof.begin(kCutoffs, s2);
            PHD_HIP(launch_palette_cutoffs(d_imgs[i], height, width, ds, gp,
                                           (const unsigned short*)(dw + L.H(n, i)), nchunks, rules, search,
                                           (int)dec[i].search.size(), c->d_k255, s2));
            c->prof.end(ps, s2);
            ps = c->prof.begin(kPalSums, s2);
            PHD_HIP(launch_palette_sums(d_imgs[i], height, width, ds, gp, rules, off,
                                        (int)dec[i].parents.size(), (double*)(dw + L.C(n, i) + L.c_pal),
                                        c->d_k255, s2));
            c->prof.end(ps, s2);
        }
    }
    PHD_HIP(hipEventRecord(c->ev_tail, s2));
    // the stream that finishes last downloads the last results after an event
    // of the other that is already complete (waiting on a pending event from
    // another stream costs ~30 us of idle GPU): a single image's palette tail
    // (decisions, Kcut, partial sums) ends after its FFTs, a batch's FFTs end
    // after the tail
    const bool last_on_st = true;                             // the FFTs run on st
    const bool tail_last = n == 1;
    if (!tail_last) {
        PHD_HIP(hipStreamWaitEvent(st, c->ev_tail, 0));
        PHD_HIP(hipEventRecord(c->ev[3], st));
    } else {
        PHD_HIP(hipStreamWaitEvent(s2, c->ev_fft, 0));
        PHD_HIP(hipEventRecord(c->ev[3], s2));
    }
    // image i's C record (bins, max partials, palette sums, sharpness) goes to
    // the host once its column pass and the palette tail are done (on the tail
    // stream, after the tail's kernels); the host assembles it while the later
    // images' FFTs run.  Two streams per lane: two lanes fit HIP's default
    // four hardware queues (round 5: five streams per lane needed
    // GPU_MAX_HW_QUEUES=8 to keep unrelated work from sharing a queue)
    uint8_t* hc = hp + (size_t)n * L.a_bytes;
    const hipStream_t sd = s2;
    const hipStream_t s_end = tail_last ? s2 : st;           // the last group's stream
    bool sd_used = false;
    for (int i0 = 0; i0 < n; i0 = dl_last(i0) + 1) {
        const int i1 = dl_last(i0);
        const bool on_st = last_on_st && i1 == n - 1;
        const hipStream_t s_dl = on_st ? s_end : sd;
        if (!on_st) {
            PHD_HIP(hipStreamWaitEvent(sd, c->ev_img_fft[i1], 0));
            sd_used = true;
        }
        PHD_HIP(hipMemcpyAsync(hc + (size_t)i0 * L.c_bytes, dw + L.C(n, i0), (size_t)(i1 - i0 + 1) * L.c_bytes,
                               hipMemcpyDeviceToHost, s_dl));
        PHD_HIP(hipEventRecord(c->ev_img_dl[i1], s_dl));
    }
    if (last_on_st) {
        if (sd_used) {
            PHD_HIP(hipEventRecord(c->ev_dl_sd, sd));
            PHD_HIP(hipStreamWaitEvent(s_end, c->ev_dl_sd, 0));
        }
        PHD_HIP(hipEventRecord(c->ev[4], s_end));   // the host waits on it before returning
    } else {
        PHD_HIP(hipEventRecord(c->ev[4], sd));
        PHD_HIP(hipStreamWaitEvent(st, c->ev[4], 0));
    }
    const auto t_dec = std::chrono::steady_clock::now();
    auto t_sync = t_dec;

    // each download group's reports are assembled once its copy is done; a
    // group of 8 or more (batched FFT groups of small images, ~10 us per
    // report at 36/4/5) on the host pool
    std::vector<std::string>& asm_why = fail_why;             // the decisions' messages are set already
    auto assemble_one = [&](int i) {
        if (!ok[i]) return;
        asm_why[i].clear();
        const uint8_t* a = hp + L.A(i);
        const uint8_t* cc = hc + (size_t)i * L.c_bytes;
        const unsigned long long* sums = (const unsigned long long*)(a + L.a_sums);
        const double* spart = (const double*)(a + L.a_spart);
        double s_acc = 0.0;
        for (int k = 0; k < nchunks; k++) s_acc += spart[k];
        const RGB_Statistics st_i = stats_from_sums(sums, (long)height * width);
        // pgm_normalize_fft's max (src/fft_processing.c:181-184) over the block partials
        const double* fpart = (const double*)(cc + L.c_fmax);
        double fmax = 0.0;
        for (int b = 0; b < ncolblocks; b++) fmax = fpart[b] > fmax ? fpart[b] : fmax;
        const double* pal = (const double*)(cc + L.c_pal);
        if (fused) {                                         // whole groups (host) + partial groups (device)
            for (size_t k = 0; k < hsum[i].size(); k++) hsum[i][k] += pal[k];
            pal = hsum[i].data();
        }
        out[i] = assemble(st_i, s_acc / (double)n_hsv, dec[i], pal, n_hsv, *tbl,
                          (const unsigned long long*)(cc + L.c_bins), fmax, cfg, crops,
                          (const double*)(cc + L.c_sharp), &asm_why[i]);
        if (out[i]) status[i] = 0;
    };
    for (int i0 = 0; i0 < n; i0 = dl_last(i0) + 1) {
        const int i1 = dl_last(i0), m = i1 - i0 + 1;
        PHD_HIP(hipEventSynchronize(c->ev_img_dl[i1]));
        if (i1 == n - 1) t_sync = std::chrono::steady_clock::now();
        if (m >= 8 && pool->size() > 0) pool->parallel_for(m, [&](int k) { assemble_one(i0 + k); });
        else
            for (int i = i0; i <= i1; i++) assemble_one(i);
    }
    int failures = 0;
    for (int i = 0; i < n; i++) {
        if (ok[i] && !out[i]) set_error(asm_why[i]);          // on this thread (thread-local message)
        failures += !out[i];
    }
    const auto t_end = std::chrono::steady_clock::now();
    PHD_HIP(hipEventSynchronize(c->ev[4]));
    c->prof.collect();
    auto ms = [](std::chrono::steady_clock::time_point a, std::chrono::steady_clock::time_point b) {
        return std::chrono::duration<double, std::milli>(b - a).count();
    };
    // device stages, then host: total, enqueue, decisions + pass-2 enqueue, assembly
    // (a per-image D2H + assembly pipeline was measured slower: extra stream
    // joins; the host pool assembles only groups of 8 or more, where its
    // wake-up latency is paid once per group)
    double tm[8] = {ms_between(c->ev[0], c->ev[1]), ms_between(c->ev[1], c->ev[2]),
                    ms_between(c->ev[2], c->ev[3]), ms_between(c->ev[0], c->ev[4]), ms(t_host0, t_end),
                    ms(t_host0, t_enq), ms(t_k1, t_dec), ms(t_sync, t_end)};
    record_timings(tm, 8);
    static const bool verbose = getenv("PHD_VERBOSE") != nullptr;
    if (verbose) {
        // END_TIMING's format (src/utilities.h:12-18), one line per stage of this
        // pipeline (the device stages are HIP-event spans of the whole batch)
        const char* names[8] = {"rgb2hsv + rgb statistics + hsv average + palette histogram (K1)",
                                "rgb2pgm + fft + blur profile (FFT rows + columns)",
                                "color palette (second pass after the FFTs)", "device total",
                                "full report (host wall clock)", "enqueue", "color palette decisions",
                                "compile full report"};
        for (int k = 0; k < 8; k++) printf("%s took %f seconds to execute \n", names[k], tm[k] / 1e3);
        printf("color palette decisions alone (%d images) took %f seconds to execute \n", n,
               ms(t_k1, t_dec_only) / 1e3);
        printf("palette tail and download enqueue took %f seconds to execute \n", ms(t_dec_only, t_dec) / 1e3);
        printf("palette tail: %d partial-group entries, at most %d per image\n", n_ent, max_per_img);
    }
    return failures == 0;
}

bool run_palette_trace(Context* c, const uint8_t* d_img, int height, int width, const phd_config& cfg,
                       std::vector<unsigned>* hist, PaletteDecision* dec, std::vector<double>* dcounts) {
    std::string why;
    if (!validate_config(cfg, &why)) {
        set_error(why);
        return false;
    }
    const hipStream_t st = c->stream;
    const GridParams gp = make_grid(cfg);
    const GroupCenters gc = make_centers(gp);
    const int ds = cfg.downsample_rate > 1 ? cfg.downsample_rate : 1;
    const long n_hsv = hsv_count(height, width, ds);
    const int nchunks = (int)((n_hsv + kChunk - 1) / kChunk);
    const Layout L = make_layout(1, gp.tl, nchunks, 1, 0, 1);
    if (!ensure_device(&c->d_ws, &c->ws_bytes, L.dev_total) || !ensure_pinned(c, L.pin_total)) return false;
    uint8_t* dw = (uint8_t*)c->d_ws;
    uint8_t* hp = (uint8_t*)c->h_pin;
    PHD_HIP(hipMemsetAsync(dw, 0, L.a_bytes + L.c_bytes, st));
    PaletteDev pd;
    pd.sums = (unsigned long long*)(dw + L.a_sums);
    pd.hist = (unsigned*)(dw + L.a_hist);
    pd.s_part = (double*)(dw + L.a_spart);
    pd.chunk_hist = (unsigned short*)(dw + L.H(1, 0));
    const Context::Cls* cls = get_cls(c, gp);
    if (!cls) return false;
    if (!launch_k1(c, L, 1, &d_img, height, width, ds, gp, cls, nchunks, false, st)) return false;
    PHD_HIP(hipMemcpyAsync(hp, dw, L.a_bytes, hipMemcpyDeviceToHost, st));
    PHD_HIP(hipStreamSynchronize(st));
    hist->assign((const unsigned*)(hp + L.a_hist), (const unsigned*)(hp + L.a_hist) + gp.tl);
    if (!decide_palette(gp, gc, hist->data(), n_hsv, cfg, dec)) return false;
    uint8_t* b = hp + L.a_bytes + L.c_bytes;
    memcpy(b + L.b_rules, dec->rules.data(), sizeof(GroupRule) * gp.tl);
    memcpy(b + L.b_search, dec->search.data(), sizeof(int) * dec->search.size());
    memcpy(b + L.b_off, dec->off.data(), sizeof(double) * dec->off.size());
    PHD_HIP(hipMemcpyAsync(dw + L.B(1, 0), b, L.b_bytes, hipMemcpyHostToDevice, st));
    GroupRule* rules = (GroupRule*)(dw + L.B(1, 0) + L.b_rules);
    const int np_ = (int)dec->parents.size();
    if (ds <= 1 && palette_sums_b_lds(gp.tl, np_) <= 160 * 1024) {
        // the production (batched) kernels, with a batch of one
        int* h_ent = (int*)(hp + L.E_pin(1) + L.e_entries);
        int* h_ns = (int*)(hp + L.E_pin(1) + L.e_ns);
        const int n_ent = (int)dec->search.size();
        for (int k = 0; k < n_ent; k++) {
            h_ent[2 * k] = 0;
            h_ent[2 * k + 1] = dec->search[k];
        }
        h_ns[0] = np_;
        PHD_HIP(hipMemcpyAsync(dw + L.E_dev(1), hp + L.E_pin(1), L.e_bytes, hipMemcpyHostToDevice, st));
        const uint8_t* const* d_ptrs = (const uint8_t* const*)(dw + L.P_dev(1));
        PHD_HIP(launch_cutoffs_batch(d_ptrs, &d_img, 1, height, width, gp, cls->fc, cls->d, c->d_k255,
                                     (const int2*)(dw + L.E_dev(1) + L.e_entries), n_ent, pd.chunk_hist,
                                     (long)L.chunk_bytes, rules, (long)L.b_bytes, st));
        PHD_HIP(launch_palette_sums_batch(d_ptrs, &d_img, 1, height, width, gp, cls->fc, cls->d, c->d_k255,
                                          rules, (const double*)(dw + L.B(1, 0) + L.b_off), (long)L.b_bytes,
                                          (const int*)(dw + L.E_dev(1) + L.e_ns), np_,
                                          (double*)(dw + L.C(1, 0) + L.c_pal), (long)L.c_bytes, st));
    } else {
        PHD_HIP(launch_palette_cutoffs(d_img, height, width, ds, gp, pd.chunk_hist, nchunks, rules,
                                       (const int*)(dw + L.B(1, 0) + L.b_search), (int)dec->search.size(),
                                       c->d_k255, st));
        PHD_HIP(launch_palette_sums(d_img, height, width, ds, gp, rules, (const double*)(dw + L.B(1, 0) + L.b_off),
                                    np_, (double*)(dw + L.C(1, 0) + L.c_pal), c->d_k255, st));
    }
    const int np = (int)dec->parents.size();
    std::vector<double> pal(4 * np);
    PHD_HIP(hipMemcpyAsync(pal.data(), dw + L.C(1, 0) + L.c_pal, sizeof(double) * 4 * np,
                           hipMemcpyDeviceToHost, st));
    PHD_HIP(hipStreamSynchronize(st));
    dcounts->resize(np);
    for (int k = 0; k < np; k++) (*dcounts)[k] = pal[4 * k + 3];
    return true;
}

}  // namespace phd

// ============================================================================
// exported C-ABI
// ============================================================================
using namespace phd;

extern "C" void phd_config_default(phd_config* c) {
    // get_report defaults, /root/reference/core.py:442-448
    c->h_partitions = 18;
    c->s_partitions = 2;
    c->v_partitions = 3;
    c->black_thresh = 0.1;
    c->gray_thresh = 0.1;
    c->coverage_thresh = 0.95;
    c->linked_list_size = 1000;
    c->downsample_rate = 1;
    c->radius_partitions = 40;
    c->angle_partitions = 72;
    c->quantity_weight = 0.1f;
    c->saturation_value_weight = 0.9f;
    c->fft_streak_thresh = 1.20;
    c->magnitude_thresh = 0.3;
    c->blur_cutoff_ratio_denom = 2;
}

static Full_Report_Data* report_from_host(const uint8_t* rgb, int height, int width, size_t row_stride,
                                          const phd_config* cfg, const Crop_Boundaries* crops) {
    clear_error();
    if (!rgb || !cfg) {
        set_error("Error: Image pointer is NULL.");
        return nullptr;
    }
    if (!precheck(height, width)) return nullptr;
    Context* c = get_context();
    if (!c) return nullptr;
    std::lock_guard<std::mutex> lk(c->mu);
    const size_t row = 3 * (size_t)width;
    const size_t bytes = row * height;
    if (!ensure_device((void**)&c->d_stage, &c->stage_bytes, bytes) || !upload_init(c)) return nullptr;
    if (row_stride == 0 || row_stride == row) {
        std::string why;
        if (!upload_async(c, c->d_stage, rgb, bytes, &why)) {
            set_error(why);
            return nullptr;
        }
    } else {
        const hipError_t e = hipMemcpy2DAsync(c->d_stage, row, rgb, row_stride, row, height, hipMemcpyHostToDevice,
                                              c->h2d);
        if (e != hipSuccess) {
            set_error(std::string("upload failed: ") + hipGetErrorString(e));
            return nullptr;
        }
    }
    if (hipEventRecord(c->ev_up[0], c->h2d) != hipSuccess || hipStreamWaitEvent(c->stream, c->ev_up[0], 0) != hipSuccess) {
        set_error("upload ordering failed");
        return nullptr;
    }
    const uint8_t* imgs[1] = {c->d_stage};
    Full_Report_Data* out = nullptr;
    int status = -1;
    run_reports(c, imgs, 1, height, width, *cfg, crops, &out, &status, nullptr);
    // the caller's buffer may be freed on return: drain the upload on every path
    (void)hipStreamSynchronize(c->h2d);
    (void)hipStreamSynchronize(c->stream);
    return out;
}

extern "C" Full_Report_Data* phd_report_u8(const uint8_t* rgb, int height, int width, size_t row_stride,
                                           const phd_config* cfg, const Crop_Boundaries* crops) {
    return report_from_host(rgb, height, width, row_stride, cfg, crops);
}

extern "C" Full_Report_Data* get_full_report_data(Image_RGB* image, Crop_Boundaries* crops, int h_partitions,
                                                  int s_partitions, int v_partitions, double black_thresh,
                                                  double gray_thresh, double coverage_thresh,
                                                  int linked_list_size, int downsample_rate,
                                                  int radius_partitions, int angle_partitions,
                                                  float quantity_weight, float saturation_value_weight,
                                                  double fft_streak_thresh, double magnitude_thresh,
                                                  int blur_cutoff_ratio_denom) {
    clear_error();
    // pre_compute_error_checks (src/utilities.c:64-87), same order and messages
    if (!image) {
        set_error("Error: Image pointer is NULL.");
        return nullptr;
    }
    if (!precheck(image->height, image->width)) return nullptr;
    if (!image->r || !image->g || !image->b) {
        set_error("Error: At least one color channel was a NULL pointer.");
        return nullptr;
    }
    phd_config cfg{h_partitions, s_partitions, v_partitions, black_thresh, gray_thresh, coverage_thresh,
                   linked_list_size, downsample_rate, radius_partitions, angle_partitions,
                   quantity_weight, saturation_value_weight, fft_streak_thresh, magnitude_thresh,
                   blur_cutoff_ratio_denom};
    if (getenv("PHD_VERBOSE"))   // interface.c:34-35 prints this unconditionally
        printf("\n There are %d cores available to the C program.\n\n", (int)sysconf(_SC_NPROCESSORS_ONLN));
    // planar doubles: the RGB8 pipeline when they are k/255.0 (utils.py:30-46),
    // else the reference's fp64 arithmetic on them (phd_planar.cpp)
    Context* c = get_context();
    if (!c) return nullptr;
    Full_Report_Data* pooled;
    {
        std::lock_guard<std::mutex> lk(c->mu);
        pooled = report_planar(c, image->r, image->g, image->b, image->height, image->width, cfg, crops);
    }
    if (!pooled) return nullptr;
    // the reference's C callers get the reference's allocation shape: every
    // member its own malloc, so free() of a member is valid (phd_legacy.cpp)
    Full_Report_Data* tree = legacy_tree_copy(pooled);
    free_full_report(&pooled);
    if (!tree) {
        set_error("report allocation failed");
        return nullptr;
    }
    legacy_register(tree);
    return tree;
}

extern "C" void phd_free_reports(Full_Report_Data** reports, int n) {
    for (int i = 0; reports && i < n; i++) free_full_report(&reports[i]);
}

extern "C" void free_full_report(Full_Report_Data** report) {
    // src/interface.c:97-111 frees each structure.  A report of the batch
    // entry points is one block (assemble), which goes back to the report
    // pool; a report of get_full_report_data is a tree of separate mallocs
    // (phd_legacy.cpp), freed member by member.  Neither (foreign, or already
    // freed): ignored, without reading memory around the pointer.
    if (!report || !*report) return;
    if (legacy_release(*report)) {
        *report = nullptr;
        return;
    }
    char* blk = reinterpret_cast<char*>(*report) - kReportHdr;
    if (!report_pool().give(blk) && getenv("PHD_VERBOSE"))
        fprintf(stderr, "free_full_report: %p is not a live report of this library; ignored\n", (void*)*report);
    *report = nullptr;
}

// Runs body(context, lane, lanes) under the context's lock: on lane 0 (this
// thread) only, or -- when `want`, lanes_setting() >= 2 and the lane worker is
// free -- on lanes 0 and 1 concurrently, lane 1 (its own context, streams and
// workspaces) on the lane worker thread.  An error of lane 1 is reported on
// this thread unless lane 0 failed too.
template <class F>
static void on_lanes(Context* c0, bool want, F&& body) {
    Context* c1 = nullptr;
    if (want && lanes_setting() >= 2) {
        c1 = get_context_lane(1);
        if (!c1) clear_error();     // no second context: one lane
    }
    LaneWorker* lw = c1 ? lane_worker() : nullptr;
    if (!lw || !lw->try_acquire()) {
        std::lock_guard<std::mutex> lk(c0->mu);
        CallLanes cl(1);
        body(c0, 0, 1);
        return;
    }
    int dev = 0;
    (void)hipGetDevice(&dev);
    std::string err1;
    lw->run([&] {
        clear_error();
        (void)hipSetDevice(dev);
        {
            std::lock_guard<std::mutex> lk1(c1->mu);
            CallLanes cl(2);
            body(c1, 1, 2);
        }
        err1 = phd_last_error();
    });
    {
        std::lock_guard<std::mutex> lk(c0->mu);
        CallLanes cl(2);
        body(c0, 0, 2);
    }
    lw->wait();
    lw->release();
    if (!err1.empty() && std::string(phd_last_error()).empty()) set_error(err1);
}

extern "C" int phd_report_batch_device(const uint8_t* d_rgb, int n_images, int height, int width,
                                       size_t image_stride, const phd_config* cfg, Full_Report_Data** out,
                                       int* status, void* stream) {
    clear_error();
    if (!d_rgb || !cfg || !out || !status || n_images <= 0) {
        set_error("phd_report_batch_device: bad arguments");
        return -1;
    }
    Context* c = get_context();
    if (!c) return -1;
    const size_t stride = image_stride ? image_stride : 3 * (size_t)width * height;
    std::vector<const uint8_t*> imgs(n_images);
    for (int i = 0; i < n_images; i++) imgs[i] = d_rgb + (size_t)i * stride;
    // two lanes for large batches on the library's streams: the second half on
    // lane 1, so each half's host phases and launch gaps overlap the other's
    // kernels.  Lane 0 takes 51.2 % (262 of 512): with equal halves lane 1
    // finished ~1.6 ms after lane 0 per 512-image call at 4000x3000, and the
    // call took 56.2 ms against 55.8-55.9 with 262 / 250 (56.0-56.3 with 268 /
    // 244; profiles/r05/lane_split_ab.log)
    on_lanes(c, n_images >= 16 && !stream, [&](Context* cl, int lane, int nl) {
        const int h = nl == 2 ? (int)(((long)n_images * 131 + 128) / 256) : n_images;
        const int i0 = lane ? h : 0, m = lane ? n_images - h : h;
        run_reports(cl, imgs.data() + i0, m, height, width, *cfg, nullptr, out + i0, status + i0,
                    (hipStream_t)stream);
    });
    int fails = 0;
    for (int i = 0; i < n_images; i++) fails += status[i] != 0;
    return fails;
}

// rgb2hsv + get_hsv_average + get_rgb_statistics (src/image_processing.c:372-417,
// 533-553) over a batch of device images: one K1 launch without the group
// histogram.  HSV is never materialised; S-bar is the mean of the HSV s channel.
extern "C" int phd_hsv_stats_batch_device(const uint8_t* d_rgb, int n_images, int height, int width,
                                          size_t image_stride, RGB_Statistics* stats, double* avg_saturation,
                                          void* stream) {
    clear_error();
    if (!d_rgb || !stats || !avg_saturation || n_images <= 0 || height <= 0 || width <= 0 ||
        height > 32767 || width > 32767) {
        set_error("phd_hsv_stats_batch_device: bad arguments");
        return -1;
    }
    Context* c = get_context();
    if (!c) return -1;
    std::lock_guard<std::mutex> lk(c->mu);
    const hipStream_t st = work_stream(c, stream);
    const size_t stride = image_stride ? image_stride : 3 * (size_t)width * height;
    const long npix = (long)height * width;
    const int nchunks = (int)((npix + kChunk - 1) / kChunk);
    // A record: 6 moments | per-chunk s partials | 256 sums of d per max value
    const size_t a_kd = al(6 * sizeof(unsigned long long)) + al(sizeof(double) * nchunks);
    const size_t a_stride = a_kd + al(256 * sizeof(unsigned long long));
    const size_t rec = (size_t)n_images * a_stride, ptrs = al(sizeof(void*) * (size_t)n_images);
    const size_t fin = (size_t)n_images * 8 * sizeof(unsigned long long);   // k_stats_finish's records
    if (!ensure_device(&c->d_ws, &c->ws_bytes, rec + ptrs + fin) || !ensure_pinned(c, rec + ptrs + fin))
        return -1;
    uint8_t* dw = (uint8_t*)c->d_ws;
    uint8_t* hp = (uint8_t*)c->h_pin;
    const uint8_t** hptr = (const uint8_t**)(hp + rec);
    for (int i = 0; i < n_images; i++) hptr[i] = d_rgb + (size_t)i * stride;
    const GridParams gp = make_grid([] { phd_config d; phd_config_default(&d); return d; }());
    const Context::Cls* cls = get_cls(c, gp);
    if (!cls) return -1;
    PaletteDev pd{};
    pd.sums = (unsigned long long*)dw;
    pd.s_part = (double*)(dw + al(6 * sizeof(unsigned long long)));
    pd.kd_sum = (unsigned long long*)(dw + a_kd);
    auto fail = [&](hipError_t e, const char* what) {
        set_error(std::string("phd_hsv_stats_batch_device: ") + what + ": " + hipGetErrorString(e));
        return -1;
    };
    hipError_t e;
    if ((e = hipMemsetAsync(dw, 0, rec, st)) != hipSuccess) return fail(e, "memset");
    if ((e = hipMemcpyAsync(dw + rec, hptr, sizeof(void*) * n_images, hipMemcpyHostToDevice, st)) != hipSuccess)
        return fail(e, "pointer upload");
    const int ps = c->prof.begin(kK1, st);
    if ((e = launch_hsv_stats_batch((const uint8_t* const*)(dw + rec), n_images, height, width, gp, cls->fc,
                                    cls->d, pd, (long)a_stride, 0, nchunks, c->d_k255, false, false,
                                    all_aligned(hptr, n_images), st)) != hipSuccess)
        return fail(e, "launch");
    c->prof.end(ps, st);
    // sum(s) = the chunk s partials (the partial final group and -(1 - 0.999999)
    // per min == 0 < max pixel) + sum_m (sum of d at max m) / m, finished on the
    // device per image (k_stats_finish): 64 bytes per image come back
    unsigned long long* dfin = (unsigned long long*)(dw + rec + ptrs);
    if ((e = launch_stats_finish(dw, n_images, (long)a_stride, (long)al(6 * sizeof(unsigned long long)),
                                 (long)a_kd, nchunks, npix, dfin, st)) != hipSuccess)
        return fail(e, "finish launch");
    if ((e = hipMemcpyAsync(hp, dfin, fin, hipMemcpyDeviceToHost, st)) != hipSuccess) return fail(e, "readback");
    if ((e = hipStreamSynchronize(st)) != hipSuccess) return fail(e, "sync");
    c->prof.collect();
    const unsigned long long* hf = (const unsigned long long*)hp;
    for (int i = 0; i < n_images; i++) {
        stats[i] = stats_from_sums(hf + 8 * (size_t)i, npix);
        avg_saturation[i] = __builtin_bit_cast(double, hf[8 * (size_t)i + 6]);
    }
    return 0;
}

// The FFT + blur-profile path alone (BASELINE config 4) over n same-size
// device images on one context (its lock held by the caller): the row and
// column passes per image on the context's stream, the channel sums of
// remove_dc_bias from the row pass (compile-time plans) or the statistics pass
// (others), one read-back.  `lanes`: the lanes the whole call is split over.
static int blur_run(Context* c, int lanes, const uint8_t* const* imgs, int n_images, int height, int width,
                    const phd_config* cfg, double* bins_out, Blur_Vector* vectors_out, void* stream) {
    const hipStream_t st = work_stream(c, stream);
    const int nbins = cfg->radius_partitions * cfg->angle_partitions, wf = width / 2 + 1;
    const BlurTable* tbl = get_table(c, height, width, cfg->radius_partitions, cfg->angle_partitions);
    if (!tbl) return -1;
    FftSel fs;
    if (!select_fft(c, height, width, nbins, imgs, n_images, &fs, tbl)) return -1;
    // the half-prefetch column form when the other lane's column passes share
    // the CUs (13.12k vs 13.0k images/s at config 4)
    if (FftSel::forced_form() < 0 && lanes >= 2) fs.col_pf = false;
    // per image: bins, max partials, channel sums (+ the statistics pass's chunk slots)
    const long npix = (long)height * width;
    const int nchunks = (int)((npix + kChunk - 1) / kChunk);
    const size_t r_bins = 0, r_fmax = al(sizeof(double) * nbins);
    const size_t r_sums = r_fmax + al(sizeof(double) * (fs.col_blocks > 0 ? fs.col_blocks : 1));
    const size_t r_spart = r_sums + al(6 * sizeof(unsigned long long));
    const size_t r_kd = r_spart + al(sizeof(double) * nchunks);   // the statistics pass's sums of d (unused)
    const size_t rb = r_kd + al(256 * sizeof(unsigned long long));
    const size_t ptrs = al(sizeof(void*) * (size_t)n_images);
    const size_t inter_one = sizeof(double2) * inter_elems(height, width);
    if (!ensure_device(&c->d_ws, &c->ws_bytes, (size_t)n_images * rb + ptrs) ||
        !ensure_pinned(c, (size_t)n_images * rb + ptrs) ||
        !ensure_device((void**)&c->d_inter, &c->inter_bytes, inter_one))
        return -1;
    uint8_t* dw = (uint8_t*)c->d_ws;
    uint8_t* hp = (uint8_t*)c->h_pin;
    auto fail = [&](hipError_t e, const char* what) {
        set_error(std::string("phd_blur_batch_device: ") + what + ": " + hipGetErrorString(e));
        return -1;
    };
    hipError_t e;
    if ((e = hipMemsetAsync(dw, 0, (size_t)n_images * rb, st)) != hipSuccess) return fail(e, "memset");
    if (!fs.ct) {
        // the runtime-plan row pass removes the DC bias itself: channel sums first
        const uint8_t** hptr = (const uint8_t**)(hp + (size_t)n_images * rb);
        for (int i = 0; i < n_images; i++) hptr[i] = imgs[i];
        if ((e = hipMemcpyAsync(dw + (size_t)n_images * rb, hptr, sizeof(void*) * n_images, hipMemcpyHostToDevice,
                                st)) != hipSuccess)
            return fail(e, "pointer upload");
        const GridParams gp = make_grid(*cfg);
        const Context::Cls* cls = get_cls(c, gp);
        if (!cls) return -1;
        PaletteDev pd{};
        pd.sums = (unsigned long long*)(dw + r_sums);
        pd.s_part = (double*)(dw + r_spart);
        pd.kd_sum = (unsigned long long*)(dw + r_kd);
        if ((e = launch_hsv_stats_batch((const uint8_t* const*)(dw + (size_t)n_images * rb), n_images, height,
                                        width, gp, cls->fc, cls->d, pd, (long)rb, 0, nchunks, c->d_k255, false,
                                        false, all_aligned(hptr, n_images), st)) != hipSuccess)
            return fail(e, "statistics pass");
    }
    for (int i = 0; i < n_images; i++) {
        unsigned long long* sums = (unsigned long long*)(dw + (size_t)i * rb + r_sums);
        int ps = c->prof.begin(kFftRows, st);
        if ((e = launch_rows_sel(fs, imgs[i], height, width, sums, c->d_k255, c->d_inter, st,
                                 fs.ct ? sums : nullptr)) != hipSuccess)
            return fail(e, "row pass");
        c->prof.end(ps, st);
        ps = c->prof.begin(kFftCols, st);
        if ((e = launch_cols_sel(fs, c->d_inter, height, width, wf, tbl->d_map, nbins,
                                 (unsigned long long*)(dw + (size_t)i * rb + r_bins),
                                 (double*)(dw + (size_t)i * rb + r_fmax),
                                 sums, nullptr, st)) != hipSuccess)
            return fail(e, "column pass");
        c->prof.end(ps, st);
    }
    if ((e = hipMemcpyAsync(hp, dw, (size_t)n_images * rb, hipMemcpyDeviceToHost, st)) != hipSuccess)
        return fail(e, "readback");
    if ((e = hipStreamSynchronize(st)) != hipSuccess) return fail(e, "sync");
    c->prof.collect();
    for (int i = 0; i < n_images; i++) {
        const uint8_t* r = hp + (size_t)i * rb;
        const double* fpart = (const double*)(r + r_fmax);
        double fmax = 0.0;
        for (int b = 0; b < fs.col_blocks; b++) fmax = fpart[b] > fmax ? fpart[b] : fmax;
        finish_blur(*tbl, (const unsigned long long*)(r + r_bins), fmax, *cfg, bins_out + (size_t)i * nbins,
                    vectors_out + (size_t)i * 10);
    }
    return 0;
}

extern "C" int phd_blur_batch_device(const uint8_t* d_rgb, int n_images, int height, int width,
                                     size_t image_stride, const phd_config* cfg, double* bins_out,
                                     Blur_Vector* vectors_out, void* stream) {
    clear_error();
    if (!d_rgb || !cfg || !bins_out || !vectors_out || n_images <= 0) {
        set_error("phd_blur_batch_device: bad arguments");
        return -1;
    }
    std::string why;
    if (!validate_config(*cfg, &why)) {
        set_error(why);
        return -1;
    }
    if (!precheck(height, width)) return -1;
    Context* c = get_context();
    if (!c) return -1;
    const size_t stride = image_stride ? image_stride : 3 * (size_t)width * height;
    std::vector<const uint8_t*> imgs(n_images);
    for (int i = 0; i < n_images; i++) imgs[i] = d_rgb + (size_t)i * stride;
    const int nbins = cfg->radius_partitions * cfg->angle_partitions;
    // two lanes for large batches on the library's streams, as the full
    // report's batches: the second half on lane 1 (its own context, stream
    // and intermediate), each lane's launch gaps and kernel tails under the
    // other's kernels
    int rc[2] = {0, 0};
    on_lanes(c, n_images >= 16 && !stream, [&](Context* cl, int lane, int nl) {
        const int h = nl == 2 ? n_images / 2 : n_images;
        const int i0 = lane ? h : 0, m = lane ? n_images - h : h;
        rc[lane] = blur_run(cl, nl, imgs.data() + i0, m, height, width, cfg, bins_out + (size_t)i0 * nbins,
                            vectors_out + (size_t)i0 * 10, stream);
    });
    return rc[0] < 0 || rc[1] < 0 ? -1 : 0;
}

constexpr long kMixedGroupMax = 1024;                         // images per run, any size

// Image indices grouped by size (groups in order of first appearance, each in
// index order), at most `cap` per group, or (pix_cap > 0) as many as fit
// pix_cap pixels when that is more: one batched run per group.
static std::vector<std::vector<int>> size_groups(const int* heights, const int* widths, int n, int cap,
                                                 long pix_cap = 0) {
    std::vector<std::vector<int>> g;
    std::map<std::pair<int, int>, int> open;                  // size -> its group still filling
    for (int i = 0; i < n; i++) {
        const auto key = std::make_pair(heights[i], widths[i]);
        auto it = open.find(key);
        const long npix = (long)heights[i] * widths[i];
        const int c = std::max<long>(cap, std::min<long>(kMixedGroupMax, pix_cap / std::max(npix, 1L)));
        if (it == open.end() || (int)g[it->second].size() >= c) {
            open[key] = (int)g.size();
            g.emplace_back();
        }
        g[open[key]].push_back(i);
    }
    return g;
}

// Device-resident images of any sizes (BASELINE config 5): one batched run
// (K1, FFTs, palette tail, per-image read-back) per group of same-size images.
extern "C" int phd_report_batch_device_mixed(const uint8_t* const* d_images, const int* heights, const int* widths,
                                             int n_images, const phd_config* cfg, Full_Report_Data** out,
                                             int* status, void* stream) {
    clear_error();
    if (!d_images || !heights || !widths || !cfg || !out || !status || n_images <= 0) {
        set_error("phd_report_batch_device_mixed: bad arguments");
        return -1;
    }
    Context* c = get_context();
    if (!c) return -1;
    // 64 images a run, or as many as 64 of the 12 MP headline size hold (small
    // images: one run for a whole size instead of one per 64, so the per-run
    // launches, host round trip and partly filled grids are paid a few times)
    const auto groups = size_groups(heights, widths, n_images, 64, 64L * 12000000L);
    // the groups go to the lanes in order, each lane taking the next one when
    // it is done with its last
    std::atomic<size_t> next{0};
    on_lanes(c, groups.size() >= 2 && !stream, [&](Context* cl, int, int) {
        for (size_t gi; (gi = next.fetch_add(1)) < groups.size();) {
            const auto& grp = groups[gi];
            const int m = (int)grp.size();
            std::vector<const uint8_t*> ptrs(m);
            std::vector<Full_Report_Data*> o(m, nullptr);
            std::vector<int> st(m, -1);
            for (int k = 0; k < m; k++) ptrs[k] = d_images[grp[k]];
            run_reports(cl, ptrs.data(), m, heights[grp[0]], widths[grp[0]], *cfg, nullptr, o.data(), st.data(),
                        (hipStream_t)stream);
            for (int k = 0; k < m; k++) {
                out[grp[k]] = o[k];
                status[grp[k]] = st[k];
            }
        }
    });
    int fails = 0;
    for (int i = 0; i < n_images; i++) fails += status[i] != 0;
    return fails;
}

// Host images of any sizes: each same-size group (<= 16) is uploaded into one
// of two device staging buffers and reported as one batch; the next group's
// upload (pinned slot ring, copy threads + DMA) runs on an uploader thread
// while the current group computes.
extern "C" int phd_report_batch_u8(const uint8_t* const* images, const int* heights, const int* widths,
                                   int n_images, const phd_config* cfg, Full_Report_Data** out, int* status) {
    clear_error();
    if (!images || !heights || !widths || !cfg || !out || !status || n_images <= 0) {
        set_error("phd_report_batch_u8: bad arguments");
        return -1;
    }
    for (int i = 0; i < n_images; i++) {
        out[i] = nullptr;
        status[i] = -1;
        if (!images[i]) {
            set_error("Error: Image pointer is NULL.");
            return -1;
        }
    }
    Context* c = get_context();
    if (!c) return -1;
    std::lock_guard<std::mutex> lk(c->mu);
    if (!upload_init(c)) return -1;
    std::vector<std::vector<int>> groups;
    static const int gcap = phd_knob("PHD_HOST_GROUP") ? std::max(1, atoi(phd_knob("PHD_HOST_GROUP"))) : 16;
    for (auto& g : size_groups(heights, widths, n_images, gcap)) {
        if (precheck(heights[g[0]], widths[g[0]])) groups.push_back(std::move(g));
    }
    int fails = 0;
    // device buffers first (the uploader thread must not allocate)
    size_t need = 0;
    for (const auto& g : groups) need = std::max(need, g.size() * 3 * (size_t)widths[g[0]] * heights[g[0]]);
    for (int b = 0; b < 2 && !groups.empty(); b++)
        if (!ensure_device((void**)&c->d_stage2[b], &c->stage2_bytes[b], need)) return -1;
    struct Up {
        bool ok = true;
        std::string why;
    };
    auto upload = [c, images, heights, widths](const std::vector<int>& g, int b, Up* u) {
        const size_t bytes = 3 * (size_t)widths[g[0]] * heights[g[0]];
        if (upload_streams() == 2 && g.size() > 1) {
            // odd images on h2d2 from a second thread: two pageable copies in flight
            Up u2;
            std::thread t2([&] {
                for (size_t k = 1; k < g.size() && u2.ok; k += 2)
                    u2.ok = upload_async(c, c->d_stage2[b] + k * bytes, images[g[k]], bytes, &u2.why, c->h2d2);
            });
            for (size_t k = 0; k < g.size() && u->ok; k += 2)
                u->ok = upload_async(c, c->d_stage2[b] + k * bytes, images[g[k]], bytes, &u->why, c->h2d);
            t2.join();
            if (u->ok && !u2.ok) *u = u2;
            if (u->ok && (hipEventRecord(c->ev_h2d2, c->h2d2) != hipSuccess ||
                          hipStreamWaitEvent(c->h2d, c->ev_h2d2, 0) != hipSuccess)) {
                u->ok = false;
                u->why = "upload event failed";
            }
        } else {
            for (size_t k = 0; k < g.size() && u->ok; k++)
                u->ok = upload_async(c, c->d_stage2[b] + k * bytes, images[g[k]], bytes, &u->why);
        }
        if (u->ok && hipEventRecord(c->ev_up[b], c->h2d) != hipSuccess) {
            u->ok = false;
            u->why = "upload event failed";
        }
    };
    std::vector<Up> ups(groups.size());
    std::thread th;
    if (!groups.empty()) th = std::thread(upload, std::cref(groups[0]), 0, &ups[0]);
    for (size_t gi = 0; gi < groups.size(); gi++) {
        th.join();                                   // group gi is enqueued (its host buffers are read)
        const auto& g = groups[gi];
        const int b = (int)(gi & 1);
        // the next group's upload runs under this group's reports (its buffer's
        // previous group finished: run_reports returns after the GPU is done)
        if (gi + 1 < groups.size()) th = std::thread(upload, std::cref(groups[gi + 1]), 1 - b, &ups[gi + 1]);
        const int m = (int)g.size(), h = heights[g[0]], w = widths[g[0]];
        const size_t bytes = 3 * (size_t)w * h;
        std::vector<const uint8_t*> ptrs(m);
        for (int k = 0; k < m; k++) ptrs[k] = c->d_stage2[b] + (size_t)k * bytes;
        std::vector<Full_Report_Data*> o(m, nullptr);
        std::vector<int> st(m, -1);
        if (!ups[gi].ok) set_error(ups[gi].why);
        else if (hipStreamWaitEvent(c->stream, c->ev_up[b], 0) != hipSuccess) set_error("upload ordering failed");
        else run_reports(c, ptrs.data(), m, h, w, *cfg, nullptr, o.data(), st.data(), nullptr);
        for (int k = 0; k < m; k++) {
            out[g[k]] = o[k];
            status[g[k]] = st[k];
        }
    }
    if (th.joinable()) th.join();
    // the caller's buffers may be freed on return: every transfer has completed
    (void)hipStreamSynchronize(c->h2d);
    (void)hipStreamSynchronize(c->h2d2);
    (void)hipStreamSynchronize(c->stream);
    for (int i = 0; i < n_images; i++) fails += status[i] != 0;
    return fails;
}

extern "C" int phd_palette_trace_device(const uint8_t* d_rgb, int height, int width, const phd_config* cfg,
                                        int* hist, int* parents, int* kept, int* n_parents) {
    clear_error();
    Context* c = get_context();
    if (!c || !cfg) return -1;
    std::lock_guard<std::mutex> lk(c->mu);
    std::vector<unsigned> h;
    PaletteDecision dec;
    std::vector<double> dcount;
    if (!run_palette_trace(c, d_rgb, height, width, *cfg, &h, &dec, &dcount)) return -1;
    const int np = (int)dec.parents.size();
    for (size_t g = 0; g < h.size(); g++) hist[g] = (int)h[g];
    for (int k = 0; k < np; k++) {
        parents[k] = dec.parents[k];
        kept[k] = (int)dcount[k];     // what the device actually summed
    }
    *n_parents = np;
    for (int k = 0; k < np; k++)
        if (dcount[k] != (double)dec.kept[k]) {
            set_error("device kept count differs from the host keep rules");
            return -2;
        }
    return (int)h.size();
}

extern "C" int phd_blur_counts(int height, int width, int radius_partitions, int angle_partitions,
                               long long* counts) {
    clear_error();
    Context* c = get_context();
    if (!c) return -1;
    std::lock_guard<std::mutex> lk(c->mu);
    const BlurTable* tb = get_table(c, height, width, radius_partitions, angle_partitions);
    if (!tb) return -1;
    memcpy(counts, tb->counts.data(), sizeof(long long) * tb->counts.size());
    return 0;
}

extern "C" int phd_fill_uniform_device(uint8_t* d_dst, size_t n, uint64_t seed, void* stream) {
    clear_error();
    Context* c = get_context();
    if (!c) return -1;
    hipStream_t st = work_stream(c, stream);
    if (launch_fill_uniform(d_dst, n, seed, st) != hipSuccess) {
        set_error("fill kernel launch failed");
        return -1;
    }
    if (hipStreamSynchronize(st) != hipSuccess) {
        set_error("fill kernel failed");
        return -1;
    }
    return 0;
}

extern "C" int phd_fill_structured_device(uint8_t* d_dst, int height, int width, uint64_t seed, int blur,
                                          int blur_axis, void* stream) {
    clear_error();
    Context* c = get_context();
    if (!c || !d_dst || height < 1 || width < 1 || blur < 0 || (blur_axis != 0 && blur_axis != 1)) return -1;
    hipStream_t st = work_stream(c, stream);
    if (launch_fill_structured(d_dst, height, width, seed, blur, blur_axis, st) != hipSuccess) {
        set_error("structured fill kernel launch failed");
        return -1;
    }
    if (hipStreamSynchronize(st) != hipSuccess) {
        set_error("structured fill kernel failed");
        return -1;
    }
    return 0;
}

extern "C" int phd_debug_hsv_groups_device(const uint8_t* d_rgb, long n_pixels, const phd_config* cfg, int* d_gid,
                                           double* d_hsv) {
    clear_error();
    Context* c = get_context();
    if (!c || !cfg) return -1;
    std::string why;
    if (!validate_config(*cfg, &why)) {
        set_error(why);
        return -1;
    }
    std::lock_guard<std::mutex> lk(c->mu);
    const GridParams gp = make_grid(*cfg);
    const Context::Cls* cls = get_cls(c, gp);
    if (!cls) return -1;
    if (launch_debug_hsv(d_rgb, n_pixels, gp, cls->fc, cls->d, c->d_k255, d_gid, d_hsv, c->stream) != hipSuccess ||
        hipStreamSynchronize(c->stream) != hipSuccess) {
        set_error("debug hsv kernel failed");
        return -1;
    }
    return 0;
}

// K1's per-pixel logic on the host, no GPU (tests/test_k1_pixel.py): for n
// interleaved RGB8 pixels the hue cell (HueCells layout), h, s and the
// deferred flag exactly as k1.hip classifies them.
extern "C" int phd_debug_k1_pixels(const uint8_t* rgb, long n, const phd_config* cfg, int* cell, double* h,
                                   double* s, int* deferred) {
    clear_error();
    if (!rgb || !cfg || !cell || !h || !s || n < 0) return -1;
    std::string why;
    if (!validate_config(*cfg, &why)) {
        set_error(why);
        return -1;
    }
    const GridParams gp = make_grid(*cfg);
    FastCls fc;
    std::unique_ptr<ClassTables> t(new ClassTables());
    make_class_tables(gp, &fc, t.get());
    if (k1_host_pixels(gp, *t, rgb, n, cell, h, s, deferred) != 0) {
        set_error("phd_debug_k1_pixels: this grid has no K1 code table");
        return -1;
    }
    return 0;
}

// Micro-benchmark hook: launch one pipeline kernel `iters` times on a device
// image (after one untimed full report to set up its inputs) and return the
// average launch time in ms from HIP events.  `ablate` is a debug mask read by
// the kernel to skip parts of its work (0 = the production kernel).
extern "C" int phd_debug_time_kernel(int kernel, const uint8_t* d_rgb, int height, int width, const phd_config* cfg,
                                     int ablate, int iters, double* avg_ms) {
    clear_error();
    Context* c = get_context();
    if (!c || !cfg || iters <= 0) return -1;
    {
        Full_Report_Data* r = nullptr;
        int st = -1;
        std::lock_guard<std::mutex> lk(c->mu);
        const uint8_t* imgs[1] = {d_rgb};
        if (!run_reports(c, imgs, 1, height, width, *cfg, nullptr, &r, &st, nullptr)) return -1;
        free_full_report(&r);
    }
    std::lock_guard<std::mutex> lk(c->mu);
    const GridParams gp = make_grid(*cfg);
    const int ds = cfg->downsample_rate > 1 ? cfg->downsample_rate : 1;
    const long n_hsv = hsv_count(height, width, ds);
    const int nchunks = (int)((n_hsv + kChunk - 1) / kChunk);
    const Context::Cls* cls = get_cls(c, gp);
    const int wf = width / 2 + 1;
    const BlurTable* tbl = get_table(c, height, width, cfg->radius_partitions, cfg->angle_partitions);
    FftSel fs;
    if (!cls || !tbl || !select_fft(c, height, width, cfg->radius_partitions * cfg->angle_partitions, &d_rgb, 1, &fs, tbl))
        return -1;
    // scratch outputs in the (large enough) workspace of the report just run
    uint8_t* dw = (uint8_t*)c->d_ws;
    PaletteDev pd;
    pd.sums = (unsigned long long*)dw;
    pd.hist = (unsigned*)(dw + 256);
    pd.s_part = (double*)(dw + 256 + 4 * 4096);
    pd.chunk_hist = (unsigned short*)(dw + 256 + 4 * 4096 + 8 * (size_t)nchunks);
    // K1 is timed as the report runs it: fused when the report fuses
    const bool fused = ds <= 1 && fused_palette_ok(gp);
    void* fscratch = nullptr;
    if (fused || kernel == kNumKernels) {
        // the fused K1's group sums and cell counts; the statistics pass's sums of d
        if (hipMalloc(&fscratch, sizeof(double) * 3 * gp.tl + sizeof(unsigned) * HueCells::count(gp) +
                                     256 * sizeof(unsigned long long)) != hipSuccess)
            return -1;
        pd.kd_sum = (unsigned long long*)fscratch;
        pd.gsum = (double*)fscratch + 256;
        pd.gcell = (unsigned*)((double*)fscratch + 256 + 3 * gp.tl);
    }
    struct FreeOnExit {
        void* p;
        ~FreeOnExit() { if (p) (void)hipFree(p); }
    } free_scratch{fscratch};
    // the column pass's bins and per-block max partials: a buffer of their own
    // (a small image's workspace is smaller than a persistent grid's partials)
    const int nbins = cfg->radius_partitions * cfg->angle_partitions;
    void* cscratch = nullptr;
    if (kernel == kFftCols &&
        hipMalloc(&cscratch, sizeof(double) * ((size_t)nbins + std::max(4096, fs.col_blocks))) != hipSuccess)
        return -1;
    FreeOnExit free_cscratch{cscratch};
    const uint8_t** d_ptr = nullptr;
    if (!ensure_device((void**)&c->d_ptrs, &c->ptrs_bytes, sizeof(void*))) return -1;
    d_ptr = (const uint8_t**)c->d_ptrs;
    if (hipMemcpy(d_ptr, &d_rgb, sizeof(void*), hipMemcpyHostToDevice) != hipSuccess) return -1;
    g_ablate = ablate;
    const hipStream_t st = c->stream;
    hipEvent_t a = c->ev[6], b = c->ev[7];
    for (int it = -1; it < iters; it++) {
        if (it == 0) (void)hipEventRecord(a, st);
        hipError_t e = hipSuccess;
        switch (kernel) {
            case kK1:
            case kNumKernels:   // K1 without the group histogram (the rgb2hsv + statistics pass)
                e = ds > 1 ? launch_hsv_ds(d_rgb, height, width, ds, gp, cls->fc, cls->d, pd, nchunks, c->d_k255, st)
                           : launch_hsv_stats_batch(d_ptr, 1, height, width, gp, cls->fc, cls->d, pd, 0, 0, nchunks,
                                                    c->d_k255, kernel == kK1, kernel == kK1 && fused,
                                                    all_aligned(&d_rgb, 1), st);
                break;
            case kFftRows: e = launch_rows_sel(fs, d_rgb, height, width, pd.sums, c->d_k255, c->d_inter, st); break;
            case kFftCols: e = launch_cols_sel(fs, c->d_inter, height, width, wf, tbl->d_map, nbins,
                                               (unsigned long long*)cscratch, (double*)cscratch + nbins, pd.sums,
                                               nullptr, st); break;
            default: set_error("kernel not supported by the timing hook"); g_ablate = 0; return -1;
        }
        if (e != hipSuccess) {
            set_error(std::string("launch failed: ") + hipGetErrorString(e));
            g_ablate = 0;
            return -1;
        }
    }
    (void)hipEventRecord(b, st);
    g_ablate = 0;
    if (hipEventSynchronize(b) != hipSuccess) return -1;
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    *avg_ms = ms / iters;
    return 0;
}

// Validation hook: the power spectrum |X[u][k]|^2 of one device image through
// the production FFT kernels (compile-time plans only), column-major into
// d_out[(W/2+1) * H] (device).  Returns 0, -2 when the size has no
// compile-time plan, or -1.
extern "C" int phd_debug_log_mant(const double* d_x, double* d_y, long n) {
    clear_error();
    Context* c = get_context();
    if (!c) return -1;
    std::lock_guard<std::mutex> lk(c->mu);
    hipError_t e = launch_log_mant(d_x, d_y, n, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    if (e != hipSuccess) {
        set_error(std::string("phd_debug_log_mant: ") + hipGetErrorString(e));
        return -1;
    }
    return 0;
}


extern "C" int phd_debug_power_spectrum(const uint8_t* d_rgb, int height, int width, double* d_out) {
    clear_error();
    Context* c = get_context();
    if (!c || !d_out) return -1;
    phd_config cfg;
    phd_config_default(&cfg);
    {
        Full_Report_Data* r = nullptr;
        int st = -1;
        std::lock_guard<std::mutex> lk(c->mu);
        const uint8_t* imgs[1] = {d_rgb};
        if (!run_reports(c, imgs, 1, height, width, cfg, nullptr, &r, &st, nullptr)) return -1;
        free_full_report(&r);
    }
    std::lock_guard<std::mutex> lk(c->mu);
    const int nbins = cfg.radius_partitions * cfg.angle_partitions;
    const BlurTable* tbl = get_table(c, height, width, cfg.radius_partitions, cfg.angle_partitions);
    FftSel fs;
    if (!tbl || !select_fft(c, height, width, nbins, &d_rgb, 1, &fs, tbl)) return -1;
    if (!fs.ct) {
        set_error("no compile-time FFT plan for this size");
        return -2;
    }
    // the report just run left the image's channel sums at the start of the workspace
    uint8_t* dw = (uint8_t*)c->d_ws;
    const int wf = width / 2 + 1;
    double* scratch = nullptr;
    if (hipMalloc(&scratch, sizeof(double) * (nbins + std::max(4096, fs.col_blocks))) != hipSuccess) return -1;
    auto* scratch_bins = reinterpret_cast<unsigned long long*>(scratch);
    const hipStream_t st = c->stream;
    hipError_t e = launch_rows_sel(fs, d_rgb, height, width, (const unsigned long long*)dw, c->d_k255, c->d_inter, st);
    if (e == hipSuccess)
        e = launch_cols_sel(fs, c->d_inter, height, width, wf, tbl->d_map, nbins, scratch_bins, scratch + nbins,
                            (const unsigned long long*)dw, d_out, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    (void)hipFree(scratch);
    if (e != hipSuccess) {
        set_error(std::string("power spectrum hook: ") + hipGetErrorString(e));
        return -1;
    }
    return 0;
}
