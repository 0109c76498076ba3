// k1.hip -- K1 of the full report with the one-pass palette, by table: per
// pixel the channel moments, the exact octree group (arm_octree), its hue
// cell and the group's h, s, v sums -- everything calculate_avg_hsv needs for
// the groups a palette slot keeps whole.
//
// Replaces the per-pixel loops of rgb2hsv (src/image_processing.c:384-415),
// get_rgb_statistics / get_average / get_variance (image_processing.c:543-553,
// filtering.c:125-148), get_hsv_average (image_processing.c:533-540),
// arm_octree (src/color_quantization.c:127-159) and, for whole groups,
// calculate_avg_hsv (color_quantization.c:529-558).
//
// Same outputs as palette.hip's fused K1 (the host code is shared); what
// differs is how a pixel is classified and counted, with the VALU count per
// pixel as the design target (K1 is instruction-bound):
//   * 4 pixels (one dwordx3) become six u16 pairs by v_perm; the moments are
//     v_dot2_u32_u16, max / min / d are v_pk_max / v_pk_min / v_pk_sub;
//   * everything arm_octree decides without the hue -- black, the gray group,
//     or the colour group's (Si, Vi) -- is ONE byte of a 64 KiB LDS table
//     indexed by (kmax, kd), built on the host from the reference's own double
//     expressions (make_class_tables: si8 + ClsEnt), and one u32 per code for
//     the group and hue-cell bases;
//   * the hue half-bin cell c = floor(2N / (Lh kd)) is the exact integer form
//     of palette.hip's classify_f (same fp32 reciprocal, same margin);
//   * counts: ONE u64 LDS atomic per pixel into its (hue cell, lane copy):
//     count (bits 0-15) | sum(kmax) (16-39) | #(kmax == 255) (40-63), so the
//     chunk's group counts, the run's cell counts and sum(v) = (sum kmax - 255
//     n255) / 255 + 0.999999 n255 all follow from it; h and s are two fp64 LDS
//     atomics (h = N * (1/kd), s = kd * (1/kmax) or rgb2hsv's 0.999999, the
//     reciprocals from an LDS table).
// A non-special hue exactly on a half-bin boundary (rare) is counted after the
// chunk's classification by its own thread in fp64 (t_exact, palette.hip's
// fused_exact decisions).
//
// Persistent blocks: one of 1024 threads per CU (the full code table takes
// 64 KiB of LDS), or two of 512 threads (the triangular table, below); each
// block walks a contiguous run of (image, 16384-pixel chunk) items, 16 or 32
// pixels per thread per chunk, the next chunk's loads issued before the
// current chunk's fold.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>

#include "phd_device.h"

namespace phd {

namespace {

// Two forms (k1t_cshift / k1t_cshift2): one 1024-thread block per CU with the
// full 256 x 256 code table, or -- when the grid's records fit 79 KiB -- two
// 512-thread blocks per CU with the kd <= kmax triangle of the table (32896
// bytes): the same 16 waves per CU, but the two blocks' barriers and chunk
// folds no longer stall each other (K1 716 against 758 us per 16 images).

typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
typedef const __attribute__((address_space(1))) unsigned gu32t;

__device__ __forceinline__ u16x2 as2(unsigned x) { return __builtin_bit_cast(u16x2, x); }
__device__ __forceinline__ unsigned as1(u16x2 x) { return __builtin_bit_cast(unsigned, x); }

template <bool TRI>
constexpr int code_bytes() { return TRI ? 256 * 257 / 2 : 65536; }
template <bool TRI>
__device__ __forceinline__ int code_idx(int kmx, int kd) {
    if constexpr (TRI) return (int)(__umul24(kmx, kmx + 1) >> 1) + kd;
    else return (kmx << 8) | kd;
}

// LDS carve (bytes).  Every base a pixel touches (cells, h/s sums, the
// reciprocals, the code tables) lies below 64 KiB, so it is a DS
// instruction's immediate offset (no address add per access); the per-run
// records and the queue follow the 64 KiB code table.
struct TVar {
    int cells, gs2, ce, inv, sinv, k255, red, code, rcell, cg, seg, r255, rmx, end;
};
__host__ __device__ inline TVar t_var(int tl, int ncell, int cshift, int code_bytes) {
    const int C = 1 << cshift;
    TVar v;
    v.cells = 0;                                                    // (ncell+1) * C u64
    v.gs2 = v.cells + 8 * (ncell + 1) * C;                          // (tl+1) * C * {h, s} f64
    v.ce = v.gs2 + 16 * (tl + 1) * C;                               // 256 u32
    v.inv = v.ce + 1024;                                            // 256 f64: 0.5 / k (h = 2N * (0.5 / kd))
    v.sinv = v.inv + 2048;                                          // 512 f64: s = kd * sinv[2 kmax + (kd == kmax)]
    v.k255 = v.sinv + 4096;                                         // 256 f64: k / 255.0 (the exact path)
    v.red = v.k255 + 2048;                                          // 16 waves x 8 x u64
    v.code = v.red + 1024;                                          // code_bytes u8
    v.rcell = v.code + code_bytes;                                  // ncell u32
    v.cg = v.rcell + 4 * ncell;                                     // tl u32
    v.seg = v.cg + 4 * tl;                                          // tl u32
    v.r255 = v.seg + 4 * tl;                                        // tl u32
    v.rmx = (v.r255 + 4 * tl + 7) & ~7;                             // tl u64
    v.end = v.rmx + 8 * tl;
    return v;
}

struct TConst {
    int lh, hp, spvp, ac, tl, gs, cgs, hp2, ncell, cshift, mycopy;
};

__host__ __device__ inline TConst make_tconst(const GridParams& gp, int cshift, int mycopy) {
    TConst X;
    X.lh = (360 / gp.hp) & 0xFFFF;                            // 16 bits: v_mul_u32_u24
    X.hp = gp.hp;
    X.spvp = gp.sp * gp.vp;
    X.ac = 4 * X.spvp - 2;
    X.tl = gp.tl;
    X.gs = gp.tl - gp.ng - 1;
    X.cgs = 4 * X.gs;
    X.hp2 = 2 * gp.hp;
    X.ncell = HueCells::count(gp);
    X.cshift = cshift;
    X.mycopy = mycopy;
    return X;
}

// The group of hue cell q (HueCells layout).
__device__ __forceinline__ int group_of_cell(int q, const TConst& X) {
    // (q - 4 gs) / (2 hp) for q - 4 gs < 2^16: fp32 with a half-unit margin
    return q < 4 * X.gs ? (q >> 2)
                        : X.gs + (int)(((float)(q - 4 * X.gs) + 0.5f) * __builtin_amdgcn_rcpf((float)(2 * X.hp)));
}

// Classify and count one pixel.  Returns true when the pixel is deferred
// (a non-special hue on a half-bin boundary: fp64 after the chunk); its
// count went to the dummy cell / group, which are never read.
struct TRead {
    int code;
    double ikd, imx;
};
// The pixel's three table reads (issued for PHD_K1_RDB pixels of a group before their
// atomics: LDS operations complete in order, so a read placed after an atomic
// would wait for it).
template <bool TRI>
__device__ __forceinline__ TRead t_read(int kmx, int kd, const unsigned char* __restrict__ code8,
                                        const double* __restrict__ inv) {
    const double* sinv = inv + 256;
    // inv[k] = 0.5 / k; sinv[2k] = 1 / k, sinv[2k + 1] = 0.999999 / k (rgb2hsv's
    // s when min == 0, src/image_processing.c:408-414; within an ulp, for sums)
    // (the two reciprocals by v_rcp_f64 + Newton instead of LDS reads measured
    // 2.56 against 2.51 ms per 64-image K1 stage, round 3)
    return TRead{code8[code_idx<TRI>(kmx, kd)], inv[max(kd, 1)], sinv[2 * kmx + (kd == kmx ? 1 : 0)]};
}
__device__ __forceinline__ bool t_pixel(int kr, int kg, int kb, int kmx, int kmn, int kd, const TRead& rd,
                                        unsigned long long* __restrict__ cells, double* __restrict__ gs2,
                                        const TConst& X, int abl) {
    const int kd1 = max(kd, 1);
    const int code = rd.code;
    const double ikd = rd.ikd, imx = rd.imx;
    const bool isr = kr == kmx, isg = kg == kmx;
    const int num = isr ? kg - kb : (isg ? kb - kr : kr - kg);
    const int b2 = isr ? ((num >> 31) & 720) : (isg ? 240 : 480);   // 2 base = 240 t
    // two channels equal <=> num is 0 or +-kd (rgb2hsv's hue is then exact)
    const bool special = (kr == kg) | (kg == kb) | (kr == kb);
    const int n2 = __mul24(b2, kd1) + 120 * num;                 // 2N, N = base kd + 60 num
    const int D = __mul24(X.lh, kd1);
    const int c = (int)(((float)n2 + 0.5f) * __builtin_amdgcn_rcpf((float)D));
    const bool onb = __mul24(c, D) == n2;
    const bool color = code < X.spvp;
    const int hie = color ? (c >> 1) : 0;                       // hue bin, colour groups only
    const int j = code - X.spvp;                                // gray / black: group - gray_start
    const int gg = color ? __mul24(hie, X.spvp) + code : X.gs + j;
    const int ch = c - X.hp;
    const bool below = onb & special & (ch >= 0) & (((ch & 1) != 0) | (ch == 0));
    // colour: 4 gg + 1 + (c - 2 hi); gray / black: 4 gs + j 2 hp + c (HueCells)
    const int cbase = color ? 4 * code + 1 + __mul24(hie, X.ac) : X.cgs + __mul24(j, X.hp2);
    const int cell = cbase + c - (int)below;
    const bool def = onb & !special;
    const int gsel = def ? X.tl : gg, csel = def ? X.ncell : cell;
    const unsigned lo = 1u + ((unsigned)kmx << 16);
    const unsigned hi32 = (unsigned)(kmx + 1) & 256u;            // #(kmax == 255) at bit 40
    if (!(abl & 1)) atomicAdd(&cells[(csel << X.cshift) | X.mycopy], ((unsigned long long)hi32 << 32) | lo);
    const double h = (double)n2 * ikd;                          // (2N) (0.5 / kd) == N (1 / kd)
    const double s = (double)kd * imx;
    double* a = gs2 + 2 * ((gsel << X.cshift) | X.mycopy);
    if (!(abl & 2)) {
        atomicAdd(a, h);
        atomicAdd(a + 1, s);
    } else if (h == 12345.0 && s == 0.5) {
        a[0] = 1.0;                                           // keep h, s live (ablation timing only)
    }
    return def;
}

// A deferred pixel (its rational hue lies exactly on the half-bin boundary
// B_c = c Lh / 2, and num is not 0 or +-kd): rgb2hsv's double hue decides.
// Black / gray / (Si, Vi) are the table's (they do not depend on the hue);
// the hue bin is arm_octree's (int)(h / Lh) (src/color_quantization.c:143)
// and the cell the side of B_c calculate_avg_hsv's wrap test puts h on, as
// palette.hip's fused_exact.
template <bool TRI>
__device__ __forceinline__ void t_exact(int kr, int kg, int kb, const double* k255g, const GridParams& gp,
                                        const unsigned char* code8, const double* inv,
                                        unsigned long long* cells, double* gs2, const TConst& X) {
    const double h = hue_exact(kr, kg, kb, k255g);
    const int kmx = max(kr, max(kg, kb)), kmn = min(kr, min(kg, kb)), kd = kmx - kmn;
    const bool isr = kr == kmx, isg = kg == kmx;
    const int num = isr ? kg - kb : (isg ? kb - kr : kr - kg);
    const int t = isr ? (num < 0 ? 3 : 0) : (isg ? 1 : 2);
    const int kd1 = max(kd, 1);
    const int n2 = 240 * t * kd1 + 120 * num, D = X.lh * kd1;
    const int c = (int)(((float)n2 + 0.5f) * __builtin_amdgcn_rcpf((float)D));   // as t_pixel: exact
    const double B = (double)c * (double)X.lh * 0.5;
    const int ch = c - X.hp;
    int below;
    if (ch < 0) below = ((c + X.hp) & 1) ? (int)((h + (-B)) < 0) : 0;      // off = 180 - hp_j = -B
    else if (ch == 0) below = (int)!((h + 180.0) > 360);                  // gray / black parent, off = 180
    else if (ch & 1) below = (int)!((h + (360.0 - B)) > 360);             // off = 360 - B
    else below = 0;
    const int cg = c - below;
    const int code = code8[code_idx<TRI>(kmx, kd)];
    int g, cell;
    if (code < X.spvp) {
        const int hi = (int)(h / gp.Lh);
        g = hi * X.spvp + code;
        cell = 4 * g + min(3, max(0, cg - 2 * hi + 1));
    } else {
        g = X.gs + code - X.spvp;
        cell = X.cgs + (code - X.spvp) * X.hp2 + cg;
    }
    const double s = (kmn == 0 && kmx != 0) ? 0.999999 : (double)kd * inv[256 + 2 * kmx];   // 1 / kmx
    const unsigned lo = 1u + ((unsigned)kmx << 16), hi32 = (unsigned)(kmx + 1) & 256u;
    atomicAdd(&cells[(cell << X.cshift) | X.mycopy], ((unsigned long long)hi32 << 32) | lo);
    double* a = gs2 + 2 * ((g << X.cshift) | X.mycopy);
    atomicAdd(a, h);
    atomicAdd(a + 1, s);
}

struct Mom {
    unsigned sr, sg, sb, qr, qg, qb;
};

// 4 pixels: moments (packed), then each pixel classified; bit i of the
// result = pixel i deferred.
template <bool TRI>
__device__ __forceinline__ unsigned t_group(unsigned w0, unsigned w1, unsigned w2, Mom& m,
                                            const unsigned char* __restrict__ code8, const double* __restrict__ inv,
                                            unsigned long long* __restrict__ cells, double* __restrict__ gs2,
                                            const TConst& X, int abl) {
    const u16x2 one = {1, 1};
    const u16x2 r02 = as2(__builtin_amdgcn_perm(w1, w0, 0x0c060c00u));
    const u16x2 r13 = as2(__builtin_amdgcn_perm(w2, w0, 0x0c050c03u));
    const u16x2 g02 = as2(__builtin_amdgcn_perm(w1, w0, 0x0c070c01u));
    const u16x2 g13 = as2(__builtin_amdgcn_perm(w2, w1, 0x0c060c00u));
    const u16x2 b02 = as2(__builtin_amdgcn_perm(w2, w0, 0x0c040c02u));
    const u16x2 b13 = as2(__builtin_amdgcn_perm(w2, w1, 0x0c070c01u));
    m.sr = __builtin_amdgcn_udot2(r02, one, m.sr, false);
    m.sr = __builtin_amdgcn_udot2(r13, one, m.sr, false);
    m.sg = __builtin_amdgcn_udot2(g02, one, m.sg, false);
    m.sg = __builtin_amdgcn_udot2(g13, one, m.sg, false);
    m.sb = __builtin_amdgcn_udot2(b02, one, m.sb, false);
    m.sb = __builtin_amdgcn_udot2(b13, one, m.sb, false);
    m.qr = __builtin_amdgcn_udot2(r02, r02, m.qr, false);
    m.qr = __builtin_amdgcn_udot2(r13, r13, m.qr, false);
    m.qg = __builtin_amdgcn_udot2(g02, g02, m.qg, false);
    m.qg = __builtin_amdgcn_udot2(g13, g13, m.qg, false);
    m.qb = __builtin_amdgcn_udot2(b02, b02, m.qb, false);
    m.qb = __builtin_amdgcn_udot2(b13, b13, m.qb, false);
    const unsigned M02 = as1(__builtin_elementwise_max(__builtin_elementwise_max(r02, g02), b02));
    const unsigned M13 = as1(__builtin_elementwise_max(__builtin_elementwise_max(r13, g13), b13));
    const unsigned N02 = as1(__builtin_elementwise_min(__builtin_elementwise_min(r02, g02), b02));
    const unsigned N13 = as1(__builtin_elementwise_min(__builtin_elementwise_min(r13, g13), b13));
    const unsigned R[2] = {as1(r02), as1(r13)}, G[2] = {as1(g02), as1(g13)}, B[2] = {as1(b02), as1(b13)};
    const unsigned Mx[2] = {M02, M13}, Mn[2] = {N02, N13};
    unsigned def = 0;
    if (abl & 32) return 0;
    // the table reads of two pixels are issued before their atomics (LDS
    // operations complete in order, so a read placed after an atomic waits for
    // it); four at a time held 20 more VGPRs and the 512-thread form spilled
    // 15 of them: 9.87 -> 9.78 ms per 256-image launch with two (round 3)
#ifndef PHD_K1_RDB
#define PHD_K1_RDB 2
#endif
    constexpr int RB = PHD_K1_RDB;                              // pixels whose table reads are batched
#pragma unroll
    for (int i0 = 0; i0 < 4; i0 += RB) {
        TRead rd[RB];
#pragma unroll
        for (int i = i0; i < i0 + RB; i++) {
            const int q = i & 1, sh = 16 * (i >> 1);           // pixel i: pair q, half i >> 1
            const int kmx = (Mx[q] >> sh) & 0xFFFF, kmn = (Mn[q] >> sh) & 0xFFFF;
            rd[i - i0] = t_read<TRI>(kmx, kmx - kmn, code8, inv);
        }
#pragma unroll
        for (int i = i0; i < i0 + RB; i++) {
            const int q = i & 1, sh = 16 * (i >> 1);
            const int kr = (R[q] >> sh) & 0xFFFF, kg = (G[q] >> sh) & 0xFFFF, kb = (B[q] >> sh) & 0xFFFF;
            const int kmx = (Mx[q] >> sh) & 0xFFFF, kmn = (Mn[q] >> sh) & 0xFFFF;
            def |= (unsigned)t_pixel(kr, kg, kb, kmx, kmn, kmx - kmn, rd[i - i0], cells, gs2, X, abl) << i;
        }
    }
    return def;
}

template <int KT, bool TRI>
__global__ __launch_bounds__(KT, 4) void k_k1t(const uint8_t* const* __restrict__ imgs, long npix, int nchunks,
                                               long nitems, GridParams gp, const ClassTables* __restrict__ tabs,
                                               const double* __restrict__ k255g, PaletteDev out, long a_stride,
                                               long h_stride, int cshift, int ablate_arg) {
    const int abl = PHD_ABL(ablate_arg);   // timing builds only: 1 cell atomics, 2 h/s atomics, 4 deferred,
                                           // 8 chunk fold, 32 classification
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int tid = threadIdx.x;
    const long it0 = (long)blockIdx.x * nitems / gridDim.x, it1 = (long)(blockIdx.x + 1) * nitems / gridDim.x;
    if (it0 >= it1) return;                                     // block-uniform
    const int C = 1 << cshift, cm = C - 1;
    const TConst X = make_tconst(gp, cshift, tid & cm);
    constexpr int kT = KT, kG = kChunk / (4 * KT);              // threads; 4-pixel groups per thread per chunk
    static_assert(kG == 4 || kG == 8, "K1 tile");
    const TVar V = t_var(X.tl, X.ncell, cshift, code_bytes<TRI>());
    unsigned char* code8 = smem + V.code;
    double* inv = reinterpret_cast<double*>(smem + V.inv);
    unsigned long long* red = reinterpret_cast<unsigned long long*>(smem + V.red);
    unsigned long long* cells = reinterpret_cast<unsigned long long*>(smem + V.cells);
    double* gs2 = reinterpret_cast<double*>(smem + V.gs2);
    unsigned* rcell = reinterpret_cast<unsigned*>(smem + V.rcell);
    unsigned* cg = reinterpret_cast<unsigned*>(smem + V.cg);
    unsigned* seg = reinterpret_cast<unsigned*>(smem + V.seg);
    unsigned* r255 = reinterpret_cast<unsigned*>(smem + V.r255);
    unsigned long long* rmx = reinterpret_cast<unsigned long long*>(smem + V.rmx);
    double* k255 = reinterpret_cast<double*>(smem + V.k255);
    {
        static_assert(code_bytes<TRI>() % 16 == 0, "uint4 copy");
        const uint4* src = reinterpret_cast<const uint4*>(TRI ? tabs->code_tri : tabs->code8);
        uint4* dst = reinterpret_cast<uint4*>(code8);
        for (int i = tid; i < code_bytes<TRI>() / 16; i += kT) dst[i] = src[i];
        for (int i = tid; i < 256; i += kT) {
            inv[i] = 0.5 * tabs->inv[i];                                    // 0.5 / k
            inv[256 + 2 * i] = tabs->inv[i];                                // 1 / k
            inv[257 + 2 * i] = i ? 0.999999 / (double)i : 0.0;              // rgb2hsv's 0.999999 (min == 0) / k
            k255[i] = k255g[i];
        }
        unsigned* z = reinterpret_cast<unsigned*>(smem);
        for (int i = tid; i < V.ce / 4; i += kT) z[i] = 0u;                        // cells, h/s sums
        for (int i = V.rcell / 4 + tid; i < V.end / 4; i += kT) z[i] = 0u;         // run records, queue
    }
    const int ng1 = (X.tl + 1) * C;
    // the (0, 0, 0) pixel's cell: masked groups past the image end are zero
    // pixels (c = 0, hue bin 0, not below)
    const int code0 = tabs->code8[0];
    const int zcell = code0 < X.spvp ? 4 * code0 + 1 : X.cgs + (code0 - X.spvp) * X.hp2;
    __syncthreads();

    const long full_end = npix & ~3L;
    int img = (int)(it0 / nchunks), c = (int)(it0 - (long)img * nchunks);
    const uint8_t* ip = imgs[img];
    unsigned w[kG][3];
    auto issue = [&](const uint8_t* p, int cc) {
        const long base = (long)cc * kChunk;
        const unsigned off0 = (unsigned)(3 * (base + 4L * tid));
#pragma unroll
        for (int st = 0; st < kG; st++) {
            const long p0 = base + 4L * tid + 4L * kT * st;
            // a group not wholly inside the image re-reads pixel 0 (masked below)
            const unsigned off = p0 < full_end ? off0 + 12u * kT * st : 0u;
            gu32t* q = (gu32t*)(p + off);
            w[st][0] = q[0];
            w[st][1] = q[1];
            w[st][2] = q[2];
        }
    };
    issue(ip, c);
    Mom m{0, 0, 0, 0, 0, 0};
    int seg_c0 = c;
    long seg_it0 = it0;
    for (long it = it0; it < it1; it++) {
        const long base = (long)c * kChunk;
        unsigned cw[kG][3];
        const bool whole = base + kChunk <= full_end;             // block-uniform
#pragma unroll
        for (int st = 0; st < kG; st++) {
            const bool ok = whole || base + 4L * tid + 4L * kT * st < full_end;
            cw[st][0] = ok ? w[st][0] : 0u;
            cw[st][1] = ok ? w[st][1] : 0u;
            cw[st][2] = ok ? w[st][2] : 0u;
        }
        const int cimg = img, cc = c;
        if (++c == nchunks) {
            c = 0;
            img++;
        }
        const bool more = it + 1 < it1;
        if (more) {
            if (img != cimg) ip = imgs[img];
            issue(ip, c);
        }
        const uint8_t* cip = imgs[cimg];
        unsigned emask = 0;                                       // deferred pixels (bit 4 st + i)
#pragma unroll
        for (int st = 0; st < kG; st++)
            emask |= t_group<TRI>(cw[st][0], cw[st][1], cw[st][2], m, code8, inv, cells, gs2, X, abl) << (4 * st);
        if (abl & 4) emask = 0;
        const bool last_chunk = base + kChunk >= npix;            // block-uniform
        if (last_chunk && tid == 0) {
            // the < 4 pixels of a partial final group
            for (long p = full_end; p < npix; p++) {
                const int kr = cip[3 * p], kg = cip[3 * p + 1], kb = cip[3 * p + 2];
                m.sr += kr; m.sg += kg; m.sb += kb;
                m.qr += kr * kr; m.qg += kg * kg; m.qb += kb * kb;
                const int kmx = max(kr, max(kg, kb)), kmn = min(kr, min(kg, kb));
                if (t_pixel(kr, kg, kb, kmx, kmn, kmx - kmn, t_read<TRI>(kmx, kmx - kmn, code8, inv), cells, gs2, X, 0))
                    t_exact<TRI>(kr, kg, kb, k255, gp, code8, inv, cells, gs2, X);
            }
        }
        // deferred pixels (a hue exactly on a half-bin boundary, ~1.7 % of uniform
        // pixels): the thread counts its own in fp64, re-reading the pixel from
        // global memory (no LDS queue, no extra barrier; measured the same time as
        // the queue resolved by the whole block, and as a 4 MiB decision table; a
        // per-wave queue filled by a lane scan, round 3, 2.55 against 2.51 ms per
        // 64-image launch: its extra registers doubled the VGPR spills).  The
        // re-read instead of selecting the pixel from the chunk's words, which then
        // had to stay live through the whole chunk: 9.98 -> 9.86 ms per 256-image
        // launch (20 -> 15 VGPRs spilled in the 512-thread form); a rolling
        // prefetch (group st of the next chunk loaded as group st of this one is
        // consumed) on top of it measured 10.27 ms (31 spilled)
        while (emask) {
            const int bt = __ffs(emask) - 1;
            emask &= emask - 1;
            const int gst = bt >> 2, pi = bt & 3;
            // re-read the pixel (L2-resident: its chunk was just loaded) instead of
            // keeping the chunk's words live through the classification
            const uint8_t* q = cip + 3 * (base + 4L * tid + 4L * kT * gst + pi);
            t_exact<TRI>(q[0], q[1], q[2], k255, gp, code8, inv, cells, gs2, X);
        }
        const long pad = base + kChunk - full_end;                // zero pixels of masked groups
        if (pad > 0 && tid == 0) atomicAdd(&cells[zcell << cshift], (unsigned long long)(-pad));
        __syncthreads();
        // fold the chunk's cells: one thread per cell sums its C copies (consecutive
        // u64); the run's cell counts, per-group sum(kmax) / n255 and the chunk's group counts
        for (int q = tid; q < ((abl & 8) ? 0 : X.ncell + 1); q += kT) {
            unsigned long long v = 0;
            unsigned long long* cp = cells + (q << cshift);
            if (C >= 2) {
                for (int k = 0; k < C; k += 2) {
                    const ulonglong2 t2 = *reinterpret_cast<const ulonglong2*>(cp + k);
                    v += t2.x + t2.y;
                    *reinterpret_cast<ulonglong2*>(cp + k) = ulonglong2{0ull, 0ull};
                }
            } else {
                v = cp[0];
                cp[0] = 0;
            }
            if (q < X.ncell && v) {
                const unsigned cnt = (unsigned)(v & 0xFFFFu);
                const int g = group_of_cell(q, X);
                rcell[q] += cnt;
                atomicAdd(&cg[g], cnt);
                atomicAdd(&rmx[g], (v >> 16) & 0xFFFFFFull);
                atomicAdd(&r255[g], (unsigned)(v >> 40));
            }
        }
        __syncthreads();
        unsigned short* chunk_out =
            reinterpret_cast<unsigned short*>(reinterpret_cast<char*>(out.chunk_hist) + cimg * h_stride) +
            (long)cc * X.tl;
        for (int g = tid; g < X.tl; g += kT) {
            const unsigned n = cg[g];
            chunk_out[g] = (unsigned short)n;
            seg[g] += n;
            cg[g] = 0;
        }
        if (!more || img != cimg || it + 1 - seg_it0 == 4096) {
            // the run leaves image cimg (or its u32 moments could overflow): flush
            const int wv = tid >> 6;
            const unsigned mom[6] = {m.sr, m.sg, m.sb, m.qr, m.qg, m.qb};
            unsigned long long m64[6];
#pragma unroll
            for (int k = 0; k < 6; k++) m64[k] = wave_sum((unsigned long long)mom[k]);
            if (lane_id() == 0)
#pragma unroll
                for (int k = 0; k < 6; k++) red[wv * 8 + k] = m64[k];
            // per-group h and s sums: fold the copies; S-bar's run sum on the side
            char* arec = reinterpret_cast<char*>(out.sums) + cimg * a_stride;   // image's A record base
            double* gsum = reinterpret_cast<double*>(reinterpret_cast<char*>(out.gsum) + cimg * a_stride);
            double sacc = 0.0;
            for (int i0 = tid; i0 < ((2 * ng1 + kT - 1) & ~(kT - 1)); i0 += kT) {
                // entry i0: field i0 & 1 of slot i0 >> 1 (slot = group << cshift | copy)
                double a = 0.0;
                if (i0 < 2 * ng1) {
                    a = gs2[i0];
                    gs2[i0] = 0.0;
                }
                for (int o = 2; o < 2 * C; o <<= 1) a += __shfl_xor(a, o, 64);
                const int g = (i0 >> 1) >> cshift, f = i0 & 1;
                if (i0 < 2 * ng1 && ((i0 >> 1) & cm) == 0 && g < X.tl && a != 0.0) {
                    atomicAdd(&gsum[f * X.tl + g], a);
                    if (f) sacc += a;
                }
            }
            const double sw = wave_sum(sacc);
            if (lane_id() == 0) reinterpret_cast<double*>(red)[wv * 8 + 6] = sw;
            __syncthreads();
            if (tid < 6) {
                unsigned long long t = 0;
                for (int qq = 0; qq < kT / 64; qq++) t += red[qq * 8 + tid];
                atomicAdd(reinterpret_cast<unsigned long long*>(arec) + tid, t);
            } else if (tid == 6) {
                double t = 0.0;
                for (int qq = 0; qq < kT / 64; qq++) t += reinterpret_cast<const double*>(red)[qq * 8 + 6];
                reinterpret_cast<double*>(reinterpret_cast<char*>(out.s_part) + cimg * a_stride)[seg_c0] = t;
            }
            unsigned* hist = reinterpret_cast<unsigned*>(reinterpret_cast<char*>(out.hist) + cimg * a_stride);
            unsigned* gcell = reinterpret_cast<unsigned*>(reinterpret_cast<char*>(out.gcell) + cimg * a_stride);
            for (int g = tid; g < X.tl; g += kT) {
                const unsigned n = seg[g];
                if (n) {
                    atomicAdd(&hist[g], n);
                    const unsigned n255 = r255[g];
                    const double sv = (double)(rmx[g] - 255ull * n255) * (1.0 / 255.0) + 0.999999 * (double)n255;
                    atomicAdd(&gsum[2 * X.tl + g], sv);
                }
                seg[g] = 0;
                r255[g] = 0;
                rmx[g] = 0;
            }
            for (int q = tid; q < X.ncell; q += kT) {
                const unsigned n = rcell[q];
                if (n) atomicAdd(&gcell[q], n);
                rcell[q] = 0;
            }
            m = Mom{0, 0, 0, 0, 0, 0};
            seg_c0 = c;
            seg_it0 = it + 1;
            __syncthreads();                                      // red is reused by the next flush
        }
    }
}

}  // namespace

int k1t_cshift(const GridParams& gp, const ClassTables& t) {
    if (!t.codes_ok) return -1;
    const int ncell = HueCells::count(gp);
    static const int budget = getenv("PHD_K1_LDS_KB") ? atoi(getenv("PHD_K1_LDS_KB")) : 158;
    for (int cs = 4; cs >= 0; cs--)
        if (t_var(gp.tl, ncell, cs, code_bytes<false>()).end <= budget * 1024) return cs;
    return -1;
}

int k1t_cshift2(const GridParams& gp, const ClassTables& t) {
    if (!t.codes_ok || getenv("PHD_K1_ONE_BLOCK")) return -1;
    const int ncell = HueCells::count(gp);
    for (int cs = 4; cs >= 2; cs--)                       // >= 4 lane copies (fewer: bank conflicts)
        if (t_var(gp.tl, ncell, cs, code_bytes<true>()).end <= 79 * 1024) return cs;
    return -1;
}

hipError_t launch_k1t_batch(const uint8_t* const* d_imgs, int n, int height, int width, const GridParams& gp,
                            const ClassTables* tabs, const PaletteDev& out0, long a_stride, long h_stride,
                            int nchunks, const double* k255, int cshift, int cshift2, hipStream_t st) {
    const long npix = (long)height * width;
    const long nitems = (long)n * nchunks;
    const int ncell = HueCells::count(gp);
    // once per process, thread-safe (two lanes may launch concurrently)
    static const bool attr = [] {
        (void)hipFuncSetAttribute((const void*)k_k1t<1024, false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  160 * 1024);
        (void)hipFuncSetAttribute((const void*)k_k1t<512, true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  160 * 1024);
        (void)hipFuncSetAttribute((const void*)k_k1t<1024, true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  160 * 1024);
        return true;
    }();
    (void)attr;
    // the two-block form runs a chunk in ~1.9x the time of the one-block form
    // (half a CU each): it wins when it has at least ~2 chunks per block
    // (measured at 16 x 732 chunks), not for a single image's 732 chunks
    // where its last chunks form the tail (3 x 1 against 2 x 1.9)
    const long cus = num_cus();
    const bool two = cshift2 >= 0 &&
                     (cshift < 0 || 19 * ((nitems + 2 * cus - 1) / (2 * cus)) < 10 * ((nitems + cus - 1) / cus));
    if (two) {                                            // two 512-thread blocks per CU
        const size_t lds = (size_t)t_var(gp.tl, ncell, cshift2, code_bytes<true>()).end;
        // with two lanes, one block per CU: the other half of each CU stays free
        // for the other lane's FFT blocks (k1_blocks_per_cu)
        const int grid = (int)std::min<long>(nitems, (long)k1_blocks_per_cu() * num_cus());
        phd_launch((k_k1t<512, true>), dim3(grid), dim3(512), lds, st, d_imgs, npix, nchunks, nitems, gp, tabs, k255,
                   out0, a_stride, h_stride, cshift2, g_ablate | env_ablate());
    } else {                                              // one 1024-thread block per CU
        const int grid = (int)std::min<long>(nitems, (long)num_cus());
        // the triangular code table leaves 31 KiB more for lane copies of the
        // cells (fine grids: 36/4/5's 3312 hue cells fit one copy beside the
        // full table, two beside the triangle)
        static const bool tri_off = getenv("PHD_K1_TRI1024") && atoi(getenv("PHD_K1_TRI1024")) == 0;
        int cs_tri = -1;
        for (int cs = 4; cs > cshift && !tri_off && cs_tri < 0; cs--)
            if (t_var(gp.tl, ncell, cs, code_bytes<true>()).end <= 158 * 1024) cs_tri = cs;
        if (cs_tri > cshift) {
            const size_t lds = (size_t)t_var(gp.tl, ncell, cs_tri, code_bytes<true>()).end;
            phd_launch((k_k1t<1024, true>), dim3(grid), dim3(1024), lds, st, d_imgs, npix, nchunks, nitems, gp,
                       tabs, k255, out0, a_stride, h_stride, cs_tri, g_ablate | env_ablate());
        } else {
            const size_t lds = (size_t)t_var(gp.tl, ncell, cshift, code_bytes<false>()).end;
            phd_launch((k_k1t<1024, false>), dim3(grid), dim3(1024), lds, st, d_imgs, npix, nchunks, nitems, gp,
                       tabs, k255, out0, a_stride, h_stride, cshift, g_ablate | env_ablate());
        }
    }
    return hipGetLastError();
}

}  // namespace phd
