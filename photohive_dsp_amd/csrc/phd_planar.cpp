// phd_planar.cpp -- get_full_report_data (src/interface.c:20-94) on the
// caller's three planes of doubles.
//
// The planes go to the device once.  k_planar_to_u8 tests whether every value
// is exactly k/255.0 (what the reference's Python binding produces,
// utils.py:30-46) and writes the RGB8 image as it goes: then the RGB8
// pipeline (run_reports) computes the report, its arithmetic on those doubles
// being the reference's.  Otherwise the fp64 planar kernels (planar.hip) run
// the reference's arithmetic on the doubles themselves, with the generic FFT
// path (fft_global.hip) on the fp64 luma plane.  Values the reference cannot
// handle (non-finite, or a group index past the octree: values above 1 can
// index out of bounds in arm_octree, src/color_quantization.c:131-145) are
// rejected with NULL, like its other undefined cases.  Any other finite values
// (negative channels, luma outside [0, 1]) get a report: the polar bins'
// fixed-point scale follows the image's largest |pgm - avg| (bin_scale).
#include <cmath>
#include <cstring>

#include "phd_host.h"

namespace phd {

namespace {

constexpr size_t kAl = 256;
size_t al(size_t x) { return (x + kAl - 1) / kAl * kAl; }

// device / pinned-free host records of one planar call
struct PRec {
    size_t flags, avg, lrng, part1, part2, hist, spart, chunk, rules, search, off, pal, bins, fmax, sharp, total;
};

PRec prec_layout(int nb, int tl, int nchunks, int nbins, int ncolblocks, int ncrops) {
    PRec R{};
    size_t o = 0;
    auto take = [&](size_t bytes) {
        const size_t at = o;
        o += al(bytes);
        return at;
    };
    R.flags = take(sizeof(int));
    R.avg = take(sizeof(double));
    R.lrng = take(sizeof(double) * 2 * nb);
    R.part1 = take(sizeof(double) * 3 * nb);
    R.part2 = take(sizeof(double) * 3 * nb);
    R.hist = take(sizeof(unsigned) * tl);
    R.spart = take(sizeof(double) * nchunks);
    R.chunk = take(sizeof(unsigned short) * (size_t)nchunks * tl);
    R.rules = take(sizeof(GroupRule) * tl);
    R.search = take(sizeof(int) * tl);
    R.off = take(sizeof(double) * tl);
    R.pal = take(sizeof(double) * 4 * tl);
    R.bins = take(sizeof(unsigned long long) * nbins);
    R.fmax = take(sizeof(double) * std::max(1, ncolblocks));
    R.sharp = take(sizeof(double) * 2 * std::max(1, ncrops));
    R.total = o;
    return R;
}

#define PHD_HIPN(expr)                                                                  \
    do {                                                                                \
        hipError_t e_ = (expr);                                                         \
        if (e_ != hipSuccess) {                                                         \
            set_error(std::string("HIP error ") + hipGetErrorString(e_) + " at " + __FILE__ + ":" + \
                      std::to_string(__LINE__) + " (" #expr ")");                       \
            return nullptr;                                                             \
        }                                                                               \
    } while (0)

}  // namespace

Full_Report_Data* report_planar(Context* c, const double* r, const double* g, const double* b, int height,
                                int width, const phd_config& cfg, const Crop_Boundaries* crops) {
    std::string why;
    if (!validate_config(cfg, &why)) {
        set_error(why);
        return nullptr;
    }
    if (!precheck(height, width) || !check_crops(crops, height, width)) return nullptr;
    const long n = (long)height * width;
    const hipStream_t st = c->stream;
    if (!ensure_device((void**)&c->d_planes, &c->planes_bytes, sizeof(double) * 4 * (size_t)n) ||
        !ensure_device((void**)&c->d_stage, &c->stage_bytes, 3 * (size_t)n))
        return nullptr;
    double* dp = c->d_planes;
    const PlanarSrc P{dp, dp + n, dp + 2 * n};
    double* pgm = dp + 3 * n;
    const int nb = planar_blocks(n);
    const GridParams gp = make_grid(cfg);
    const int ds = cfg.downsample_rate > 1 ? cfg.downsample_rate : 1;
    const long n_hsv = hsv_count(height, width, ds);
    const int nchunks = (int)((n_hsv + kChunk - 1) / kChunk);
    const int nbins = cfg.radius_partitions * cfg.angle_partitions, wf = width / 2 + 1;
    const int ncrops = crops ? crops->N : 0;
    if (!ensure_device(&c->d_prec, &c->prec_bytes, kAl)) return nullptr;
    int* flags = (int*)c->d_prec;
    PHD_HIPN(hipMemsetAsync(flags, 0, sizeof(int), st));
    PHD_HIPN(hipMemcpyAsync((void*)P.r, r, sizeof(double) * n, hipMemcpyHostToDevice, st));
    PHD_HIPN(hipMemcpyAsync((void*)P.g, g, sizeof(double) * n, hipMemcpyHostToDevice, st));
    PHD_HIPN(hipMemcpyAsync((void*)P.b, b, sizeof(double) * n, hipMemcpyHostToDevice, st));
    PHD_HIPN(launch_planar_to_u8(P, n, c->d_stage, flags, st));
    int hflags = 0;
    PHD_HIPN(hipMemcpyAsync(&hflags, flags, sizeof(int), hipMemcpyDeviceToHost, st));
    PHD_HIPN(hipStreamSynchronize(st));
    if (!(hflags & 1)) {
        // an 8-bit image: the RGB8 pipeline, exactly the reference's arithmetic on these doubles
        const uint8_t* imgs[1] = {c->d_stage};
        Full_Report_Data* out = nullptr;
        int status = -1;
        run_reports(c, imgs, 1, height, width, cfg, crops, &out, &status, nullptr);
        (void)hipStreamSynchronize(c->stream);
        return out;
    }
    // every allocation of the planar pipeline before its first launch (the stream is idle)
    FftSel fs;
    if (!select_generic(c, height, width, nbins, &fs)) return nullptr;
    const BlurTable* tbl = get_table(c, height, width, cfg.radius_partitions, cfg.angle_partitions);
    const Context::Cls* cls = get_cls(c, gp);
    if (!tbl || !cls) return nullptr;
    const PRec R = prec_layout(nb, gp.tl, nchunks, nbins, fs.col_blocks, ncrops);
    if (!ensure_device(&c->d_prec, &c->prec_bytes, R.total) ||
        !ensure_device((void**)&c->d_inter, &c->inter_bytes, sizeof(double2) * ((size_t)height * wf + 1024)))
        return nullptr;
    uint8_t* dr = (uint8_t*)c->d_prec;
    flags = (int*)(dr + R.flags);
    PHD_HIPN(hipMemsetAsync(dr, 0, R.total, st));
    // ---- the fp64 planar pipeline -------------------------------------------------
    double* avg = (double*)(dr + R.avg);
    PHD_HIPN(launch_planar_stats(P, n, pgm, (double*)(dr + R.part1), (double*)(dr + R.part2), avg,
                                 (double*)(dr + R.lrng), flags, st));
    // |pgm - avg| <= max(max - avg, avg - min) bounds every spectrum element
    // (|X| <= N max|pgm - avg|): the polar bins' fixed-point scale
    std::vector<double> lr(2 * nb + 1);
    PHD_HIPN(hipMemcpyAsync(lr.data(), dr + R.avg, sizeof(double), hipMemcpyDeviceToHost, st));
    PHD_HIPN(hipMemcpyAsync(lr.data() + 1, dr + R.lrng, sizeof(double) * 2 * nb, hipMemcpyDeviceToHost, st));
    PHD_HIPN(hipStreamSynchronize(st));
    const double av = lr[0];
    double lrange = 0.0;                                   // (NaN propagates: a non-finite channel)
    for (int k = 0; k < nb; k++) {
        const double nlo = lr[1 + 2 * k], hi = lr[2 + 2 * k];   // -min, max of block k
        const double m = std::max(hi - av, av + nlo);
        lrange = (m != m || lrange != lrange) ? NAN : std::max(lrange, m);
    }
    if (!(lrange < 1e100) || av != av) {
        set_error(std::isfinite(lrange) && av == av ? "Error: channel values too large for a finite power spectrum."
                                                    : "Error: channel values must be finite (NaN or infinity in the "
                                                      "image).");
        return nullptr;
    }
    const double bscale = bin_scale(height, wf, lrange);
    PHD_HIPN(launch_planar_k1(P, height, width, ds, gp, (unsigned*)(dr + R.hist), (unsigned short*)(dr + R.chunk),
                              (double*)(dr + R.spart), flags, st));
    std::vector<uint8_t> h(R.total);
    // the records the host decides on: flags .. s_part
    PHD_HIPN(hipMemcpyAsync(h.data(), dr, R.chunk, hipMemcpyDeviceToHost, st));
    PHD_HIPN(hipEventRecord(c->ev[5], st));
    // the blur profile on the luma plane while the host decides
    unsigned long long* bins = (unsigned long long*)(dr + R.bins);
    double* fmx = (double*)(dr + R.fmax);
    PHD_HIPN(generic_rows(fs, nullptr, pgm, height, width, nullptr, avg, c->d_k255, c->d_inter, st));
    PHD_HIPN(generic_cols(fs, c->d_inter, height, wf, tbl->d_map, nbins, bins, fmx, st, bscale));
    if (ncrops) {
        // get_variance_sharpness runs on the luma before the DC removal (src/interface.c:70-73)
        std::vector<int> ca(4 * ncrops);
        for (int k = 0; k < ncrops; k++) {
            ca[k] = crops->top[k];
            ca[ncrops + k] = crops->bottom[k];
            ca[2 * ncrops + k] = crops->left[k];
            ca[3 * ncrops + k] = crops->right[k];
        }
        PHD_HIPN(launch_sharpness_src(nullptr, pgm, height, width, ncrops, ca.data(), ca.data() + ncrops,
                                      ca.data() + 2 * ncrops, ca.data() + 3 * ncrops, c->d_k255,
                                      (double*)(dr + R.sharp), st));
    }
    PHD_HIPN(hipEventSynchronize(c->ev[5]));
    const int hf = *(const int*)(h.data() + R.flags);
    if (hf & (2 | 4)) {
        (void)hipStreamSynchronize(st);
        set_error(hf & 2 ? "Error: channel values must be finite (NaN or infinity in the image)."
                         : "Error: channel values put pixels outside the octree (out-of-bounds group in "
                           "arm_octree).");
        return nullptr;
    }
    // get_rgb_statistics: the partials in the order the device summed them
    RGB_Statistics stt;
    double* so = &stt.Br;
    for (int ch = 0; ch < 3; ch++) {
        double a = 0.0;
        for (int k = 0; k < nb; k++) a += ((const double*)(h.data() + R.part1))[3 * k + ch];
        so[ch] = a / (double)n;
    }
    const unsigned* hist = (const unsigned*)(h.data() + R.hist);
    const double* spart = (const double*)(h.data() + R.spart);
    double s_acc = 0.0;
    for (int k = 0; k < nchunks; k++) s_acc += spart[k];
    PaletteDecision dec;
    if (!decide_palette(gp, cls->gc, hist, n_hsv, cfg, &dec, cls->near.empty() ? nullptr : cls->near.data())) {
        (void)hipStreamSynchronize(st);
        return nullptr;
    }
    PHD_HIPN(hipMemcpyAsync(dr + R.rules, dec.rules.data(), sizeof(GroupRule) * gp.tl, hipMemcpyHostToDevice, st));
    if (!dec.search.empty())
        PHD_HIPN(hipMemcpyAsync(dr + R.search, dec.search.data(), sizeof(int) * dec.search.size(),
                                hipMemcpyHostToDevice, st));
    if (!dec.off.empty())
        PHD_HIPN(hipMemcpyAsync(dr + R.off, dec.off.data(), sizeof(double) * dec.off.size(), hipMemcpyHostToDevice,
                                st));
    PHD_HIPN(launch_planar_tail(P, height, width, ds, gp, (const unsigned short*)(dr + R.chunk), nchunks,
                                (GroupRule*)(dr + R.rules), (const int*)(dr + R.search), (int)dec.search.size(),
                                (const double*)(dr + R.off), (int)dec.parents.size(), (double*)(dr + R.pal), st));
    PHD_HIPN(hipMemcpyAsync(h.data() + R.part2, dr + R.part2, R.total - R.part2, hipMemcpyDeviceToHost, st));
    PHD_HIPN(hipStreamSynchronize(st));
    for (int ch = 0; ch < 3; ch++) {
        double a = 0.0;
        for (int k = 0; k < nb; k++) a += ((const double*)(h.data() + R.part2))[3 * k + ch];
        so[3 + ch] = std::sqrt(a / (double)n);
    }
    const double* fpart = (const double*)(h.data() + R.fmax);
    double fmax = 0.0;
    for (int k = 0; k < fs.col_blocks; k++) fmax = fpart[k] > fmax ? fpart[k] : fmax;
    Full_Report_Data* out = assemble(stt, s_acc / (double)n_hsv, dec, (const double*)(h.data() + R.pal), n_hsv, *tbl,
                                     (const unsigned long long*)(h.data() + R.bins), fmax, cfg, crops,
                                     (const double*)(h.data() + R.sharp), &why, bscale);
    if (!out) set_error(why);
    return out;
}

}  // namespace phd
