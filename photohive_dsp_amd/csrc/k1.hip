// k1.hip -- K1 of the full report with the one-pass palette: per pixel the
// channel moments, the exact octree group (arm_octree), its hue cell and the
// h, s, v sums calculate_avg_hsv needs for the groups a palette slot keeps
// whole.
//
// Replaces the per-pixel loops of rgb2hsv (src/image_processing.c:384-415),
// get_rgb_statistics / get_average / get_variance (image_processing.c:543-553,
// filtering.c:125-148), get_hsv_average (image_processing.c:533-540),
// arm_octree (src/color_quantization.c:127-159) and, for whole groups,
// calculate_avg_hsv (color_quantization.c:529-558).
//
// The kernel is bound by LDS throughput, not by its VALU (round-3 counters:
// ~103 LDS cycles per 64-pixel wave-group against ~60 CU-cycles of VALU), and
// what cost the LDS most were random-address fp64 atomics into few slots
// (tools/lds_probe.hip: a ds_add_f64 into 113 groups x 4 copies takes ~20
// cycles per wave-instruction, into ~2k slots ~9).  So the design is
//   * ONE LDS table read per pixel (the class code, k1_pixel.h), the
//     reciprocals of h = 60 X / kd and s = kd / kmax by an fp32 reciprocal and
//     one fp64 Newton step in registers (no reciprocal tables);
//   * three LDS atomics per pixel at ONE address: the pixel's hue cell (lane
//     copy) holds {u64 count | #(kmax == 255) << 16 | sum kmax << 32, f64
//     sum h, f64 sum s} (24 B), so h and s are summed per hue cell (~5x the
//     slots of per-group sums) and folded into groups once per run;
//   * moments of 4 pixels (one dwordx3) as six u16 pairs by v_perm and
//     v_dot2_u32_u16, max / min by v_pk_max_u16 / v_pk_min_u16.
// The count words are folded per 16384-pixel chunk (the chunk's group counts,
// for the palette's tie-overflow cut-offs), the h / s sums per run.
//
// Persistent blocks: two of 512 threads per CU with the kd <= kmax triangle
// of the code table where the records fit 79 KiB, else one of 1024 threads;
// each block walks a contiguous run of (image, chunk) items, 16 or 32 pixels
// per thread per chunk, the next chunk's loads issued before the current
// chunk's classification.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <type_traits>
#include <cstdlib>

#include "k1_pixel.h"
#include "phd_device.h"

namespace phd {

namespace {

typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
typedef const __attribute__((address_space(1))) unsigned gu32t;
// global (not flat) byte loads: a flat load also counts against the LDS counter
typedef const __attribute__((address_space(1))) uint8_t gu8t;

__device__ __forceinline__ u16x2 as2(unsigned x) { return __builtin_bit_cast(u16x2, x); }
__device__ __forceinline__ unsigned as1(u16x2 x) { return __builtin_bit_cast(unsigned, x); }

template <bool TRI>
constexpr int code_bytes() { return TRI ? 256 * 257 / 2 : 65536; }
template <bool TRI>
__device__ __forceinline__ int code_idx(int kmx, int kd) {
    if constexpr (TRI) return (int)(__umul24(kmx, kmx + 1) >> 1) + kd;
    else return (kmx << 8) | kd;
}

// code_idx for the two pixels of a u16 pair at once (u16 lanes: no overflow,
// kmx (kmx + 1) <= 65280)
template <bool TRI>
__device__ __forceinline__ u16x2 code_idx2(u16x2 mx, u16x2 kd) {
    const u16x2 one = {1, 1};
    if constexpr (TRI) return ((mx * (mx + one)) >> one) + kd;
    else {
        const u16x2 eight = {8, 8};
        return (mx << eight) | kd;
    }
}

// LDS carve (bytes).
constexpr int kDq = 48;          // deferred-pixel queue entries per wave (u16 chunk offsets; ~35 per chunk)

// The accumulators (round 6; before, one 24-byte {count, sum h, sum s} record
// per hue cell and lane copy, whose random addresses cost LDS bank conflicts):
//  * per hue cell and lane copy (cs: log2 copies) the u64 count word,
//    cnt[(cell << cs) | copy];
//  * per GROUP and lane copy (hs: log2 copies, up to 16) fp64 sum h and sum s,
//    hsum[(g << hs) | copyh], the s array soff bytes after it.  Only counts
//    are needed per cell (calculate_avg_hsv's wrap sides, fused_slot_sums);
//    h and s per group.  With 16 copies indexed by lane & 15 every lane of an
//    instruction's 16-lane group hits its own bank pair: conflict-free.
// The launch picks (cs, hs) by an expected-conflict cost (k1_config).
__host__ __device__ inline int k1_cfg(int cs, int hs) { return cs | (hs << 4); }
__host__ __device__ inline int k1_cs(int cfg) { return cfg & 15; }
__host__ __device__ inline int k1_hs(int cfg) { return cfg >> 4; }

struct LVar {
    int cells, hsum, soff, code, k255, red, dq, rcell, cg, seg, r255, rmx, ctab, end;
};
__host__ __device__ inline LVar l_var(int tl, int ncell, int cfg, int code_bytes, int ncodes) {
    LVar v;
    v.cells = 0;                                                    // (ncell + 1) << cs u64 count words
    v.hsum = (8 * ((ncell + 1) << k1_cs(cfg)) + 15) & ~15;          // (tl + 1) << hs f64 sum h, then sum s
    v.soff = 8 * ((tl + 1) << k1_hs(cfg));
    v.code = v.hsum + 2 * v.soff;                                   // code_bytes u8
    v.k255 = (v.code + code_bytes + 15) & ~15;                      // 256 f64: k / 255.0 (deferred pixels)
    v.red = v.k255 + 2048;                                          // 16 waves x 8 u64
    v.dq = v.red + 1024;                                            // 16 waves x kDq u16: deferred pixels
    v.rcell = v.dq + 16 * kDq * 2;                                  // ncell u32: the run's cell counts
    v.cg = v.rcell + 4 * ncell;                                     // tl u32: the chunk's group counts
    v.seg = v.cg + 4 * tl;                                          // tl u32: the run's group counts
    v.r255 = v.seg + 4 * tl;                                        // tl u32: the run's #(kmax == 255)
    v.rmx = (v.r255 + 4 * tl + 7) & ~7;                             // tl u64: the run's sum kmax
    v.ctab = v.rmx + 8 * tl;                                        // ncodes K1Code: cell / group terms
    v.end = v.ctab + 8 * ncodes;
    return v;
}

// The group of hue cell q (HueCells layout).
__device__ __forceinline__ int group_of_cell(int q, const K1Grid& G) {
    // (q - 4 gs) / (2 hp) for q - 4 gs < 2^16: fp32 with a half-unit margin
    return q < 4 * G.gs ? (q >> 2)
                        : G.gs + (int)(((float)(q - 4 * G.gs) + 0.5f) * __builtin_amdgcn_rcpf((float)G.hp2));
}

// A thread's accumulator addresses: the LDS base, the copy shifts and its
// copies (byte offsets are 32-bit: a 64-bit pointer product costs a
// quarter-rate v_mad_u64_u32)
struct Acc {
    unsigned char* base;     // the count words at base, sum h at base + hsum, sum s soff further
    int hsum, soff;
    int cs, hs;
    unsigned copy8, copyh8;  // this thread's copies x 8 bytes
};

__device__ __forceinline__ void acc_add(const Acc& A, int cell, int g, unsigned lo, unsigned hi, double h, double s) {
    atomicAdd(reinterpret_cast<unsigned long long*>(A.base + (((unsigned)cell << (A.cs + 3)) | A.copy8)),
              ((unsigned long long)hi << 32) | lo);
    unsigned char* ha = A.base + A.hsum + (((unsigned)g << (A.hs + 3)) | A.copyh8);
    atomicAdd(reinterpret_cast<double*>(ha), h);
    atomicAdd(reinterpret_cast<double*>(ha + A.soff), s);
}
__device__ __forceinline__ void acc_add(const Acc& A, const K1Px& p) { acc_add(A, p.cell, p.grp, p.lo, p.hi, p.h, p.s); }

struct Mom {
    unsigned sr, sg, sb, qr, qg, qb;
};

// Sums over the wave of a small per-lane count v < 2^B by bit slices: one
// ballot per bit, counted with s_bcnt1 (and mbcnt for the lanes below this
// one), instead of six cross-lane shuffles, each an LDS round trip of ~100+
// cycles on the chunk's critical path (round 6).
template <int B>
__device__ __forceinline__ unsigned wave_sum_bits(unsigned v) {
    unsigned t = 0;
#pragma unroll
    for (int b = 0; b < B; b++) t += (unsigned)__popcll(__ballot((v >> b) & 1u)) << b;
    return t;
}
// the exclusive prefix over the lanes below this one; the wave's total in tot
template <int B>
__device__ __forceinline__ unsigned wave_prefix_bits(unsigned v, unsigned& tot) {
    unsigned pre = 0, t = 0;
#pragma unroll
    for (int b = 0; b < B; b++) {
        const unsigned long long m = __ballot((v >> b) & 1u);
        pre += __builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u)) << b;
        t += (unsigned)__popcll(m) << b;
    }
    tot = t;
    return pre;
}

// A thread's run of pixels in one hue cell (MERGE): consecutive pixels of a
// thread that land in the same cell are summed in registers and added to the
// LDS with one set of atomics when the cell changes (flat image regions put
// most of a wave's lanes on one address, where LDS atomics serialise).
struct CellRun {
    int cell;            // -1: empty
    int grp;
    unsigned lo, hi;
    double h, s;
};

// 4 pixels (one dwordx3): moments, then each pixel classified and counted;
// bit i of the result = pixel i deferred.
template <bool TRI, bool SMALL, bool MERGE>
__device__ __forceinline__ unsigned k1_group(unsigned w0, unsigned w1, unsigned w2, Mom& m,
                                             const unsigned char* __restrict__ code8,
                                             const K1Code* __restrict__ ctab, const Acc& A,
                                             const K1Grid& G, CellRun* run, unsigned& nsame) {
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
    const u16x2 mx02 = __builtin_elementwise_max(__builtin_elementwise_max(r02, g02), b02);
    const u16x2 mx13 = __builtin_elementwise_max(__builtin_elementwise_max(r13, g13), b13);
    const u16x2 mn02 = __builtin_elementwise_min(__builtin_elementwise_min(r02, g02), b02);
    const u16x2 mn13 = __builtin_elementwise_min(__builtin_elementwise_min(r13, g13), b13);
    const unsigned Mx[2] = {as1(mx02), as1(mx13)}, Mn[2] = {as1(mn02), as1(mn13)};
    const unsigned Kd[2] = {as1(mx02 - mn02), as1(mx13 - mn13)};
    const unsigned R[2] = {as1(r02), as1(r13)}, Gc[2] = {as1(g02), as1(g13)}, B[2] = {as1(b02), as1(b13)};
    // the four code reads first: LDS operations complete in order, so a read
    // placed after an atomic would wait for it.  The table index of both
    // pixels of a pair in packed u16 arithmetic (round 6: kmx (kmx + 1) / 2 +
    // kd <= 32895, three v_pk ops per pair instead of five VALU per pixel)
    const u16x2 kd02 = mx02 - mn02, kd13 = mx13 - mn13;
    const unsigned Ix[2] = {as1(code_idx2<TRI>(mx02, kd02)), as1(code_idx2<TRI>(mx13, kd13))};
    int code[4];
#pragma unroll
    for (int i = 0; i < 4; i++) {
        const int q = i & 1, sh = 16 * (i >> 1);           // pixel i: pair q, half i >> 1
        code[i] = code8[(Ix[q] >> sh) & 0xFFFF];
    }
    // the reciprocal's operands of both pixels of a pair in u16 lanes:
    // max(kd, 1) max(kmx, 1) <= 65025
    const u16x2 km02 = __builtin_elementwise_max(mx02, one), km13 = __builtin_elementwise_max(mx13, one);
    const unsigned Pp[2] = {as1(__builtin_elementwise_max(kd02, one) * km02),
                            as1(__builtin_elementwise_max(kd13, one) * km13)};
    const unsigned Km[2] = {as1(km02), as1(km13)};
    K1Inv ekd[4];
#pragma unroll
    for (int i = 0; i < 4; i++) {
        const int q = i & 1, sh = 16 * (i >> 1);
        // from the VALU (round 4: an LDS table of reciprocals measured slower,
        // 46 against 40 us per image -- the LDS is the busier pipe); one
        // reciprocal of kd kmax per pixel since round 6
        ekd[i] = k1_inv_p((Pp[q] >> sh) & 0xFFFF, (Km[q] >> sh) & 0xFFFF);
    }
    // the codes' cell / group terms, all four read before this group's
    // atomics (LDS operations complete in order: a read issued after an atomic
    // would wait for it)
    K1Code ce[4];
#pragma unroll
    for (int i = 0; i < 4; i++) ce[i] = ctab[code[i]];
    // X of both pixels of each pair in 16-bit lanes (k1_x_pair)
    const unsigned Xp[2] = {as1(k1_x_pair(r02, g02, b02, mx02, kd02)), as1(k1_x_pair(r13, g13, b13, mx13, kd13))};
    unsigned def = 0;
    int cell0 = 0;
    bool same = true;
#pragma unroll
    for (int i = 0; i < 4; i++) {
        const int q = i & 1, sh = 16 * (i >> 1);
        const int kmx = (Mx[q] >> sh) & 0xFFFF, kmn = (Mn[q] >> sh) & 0xFFFF, kd = (Kd[q] >> sh) & 0xFFFF;
        bool special = false;
        if constexpr (!SMALL) {
            const int kr = (R[q] >> sh) & 0xFFFF, kg = (Gc[q] >> sh) & 0xFFFF, kb = (B[q] >> sh) & 0xFFFF;
            special = (kr == kg) | (kg == kb) | (kr == kb);
        }
        const K1Px p = k1_pixel_x<SMALL>((int)((Xp[q] >> sh) & 0xFFFF), special, kmx, kmn, kd, ce[i], ekd[i], G);
        if constexpr (MERGE) {
#if defined(PHD_K1_MERGE_SEL)
            // (A/B build) the run update by selects, only the flush's atomics
            // under a branch; the same sums (0 + x = x exactly)
            const bool same = p.cell == run->cell;
            if (!same && run->cell >= 0) acc_add(A, run->cell, run->grp, run->lo, run->hi, run->h, run->s);
            run->lo = (same ? run->lo : 0u) + p.lo;
            run->hi = (same ? run->hi : 0u) + p.hi;
            run->h = (same ? run->h : 0.0) + p.h;
            run->s = (same ? run->s : 0.0) + p.s;
            run->cell = p.cell;
            run->grp = p.grp;
#else
            if (p.cell == run->cell) {
                run->lo += p.lo;
                run->hi += p.hi;
                run->h += p.h;
                run->s += p.s;
            } else {
                if (run->cell >= 0) acc_add(A, run->cell, run->grp, run->lo, run->hi, run->h, run->s);
                *run = CellRun{p.cell, p.grp, p.lo, p.hi, p.h, p.s};
            }
#endif
        } else {
            acc_add(A, p);
        }
        def |= p.dfr << i;
        // the vote sample: are all four pixels in one cell?  (every group
        // since round 6: a sample of step 0 only cost two selects per pixel in
        // every step of the un-unrolled loop)
        if (i == 0) cell0 = p.cell;
        else same = same && p.cell == cell0;
    }
    nsame += same ? 1u : 0u;
    return def;
}

// Per-thread cell runs (CellRun) for the next chunk when more than a fifth of
// this chunk's 4-pixel groups lie in one cell (round 6: every group counted;
// before, each thread's first only),
// else every pixel's atomics -- flat images (SURVEY 8(d) row 2(b)'s blurred
// structured ones: 81 % of groups) pay for the runs' selects, noise does not
// (round 4: runs always 43.8 against 40.6 us on noise, never 80 against 48
// on hblur).
template <int KT, bool TRI, bool SMALL>
__global__ __launch_bounds__(KT, 4) void k_k1t(const uint8_t* const* __restrict__ imgs, long npix, int nchunks,
                                               long nitems, GridParams gp, K1Grid G,
                                               const ClassTables* __restrict__ tabs,
                                               const double* __restrict__ k255g, PaletteDev out, long a_stride,
                                               long h_stride, int cfg) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int tid = threadIdx.x;
    const long it0 = (long)blockIdx.x * nitems / gridDim.x, it1 = (long)(blockIdx.x + 1) * nitems / gridDim.x;
    if (it0 >= it1) return;                                     // block-uniform
    const int cshift = k1_cs(cfg), hshift = k1_hs(cfg);
    const int C = 1 << cshift, CH = 1 << hshift;
    constexpr int kT = KT, kG = kChunk / (4 * KT);              // threads; 4-pixel groups per thread per chunk
    static_assert(kG == 4 || kG == 8, "K1 tile");
    const int tl = gp.tl, ncell = G.ncell;
    const int ncodes = k1_ncodes(G);
    const LVar V = l_var(tl, ncell, cfg, code_bytes<TRI>(), ncodes);
    K1Code* ctab = reinterpret_cast<K1Code*>(smem + V.ctab);
    unsigned char* cells = smem + V.cells;
    unsigned long long* cnt = reinterpret_cast<unsigned long long*>(cells);
    double* hsum = reinterpret_cast<double*>(smem + V.hsum);
    double* ssum = hsum + V.soff / 8;
    const Acc A{cells, V.hsum, V.soff, cshift, hshift, (unsigned)(tid & (C - 1)) << 3, (unsigned)(tid & (CH - 1)) << 3};
    unsigned char* code8 = smem + V.code;
    double* k255 = reinterpret_cast<double*>(smem + V.k255);
    unsigned long long* red = reinterpret_cast<unsigned long long*>(smem + V.red);
    // the two chunk-parity vote counters, in the unused slot 7 of waves 0 and
    // 1's flush records (vote[0], vote[16])
    unsigned* vote = reinterpret_cast<unsigned*>(red + 7);
    int merge = 0, vpar = 0;                                    // block-uniform
    unsigned* rcell = reinterpret_cast<unsigned*>(smem + V.rcell);
    unsigned* cg = reinterpret_cast<unsigned*>(smem + V.cg);
    unsigned* seg = reinterpret_cast<unsigned*>(smem + V.seg);
    unsigned* r255 = reinterpret_cast<unsigned*>(smem + V.r255);
    unsigned long long* rmx = reinterpret_cast<unsigned long long*>(smem + V.rmx);
    {
        static_assert(code_bytes<TRI>() % 16 == 0, "uint4 copy");
        const uint4* src = reinterpret_cast<const uint4*>(TRI ? tabs->code_tri : tabs->code8);
        uint4* dst = reinterpret_cast<uint4*>(code8);
        for (int i = tid; i < code_bytes<TRI>() / 16; i += kT) dst[i] = src[i];
        for (int i = tid; i < 256; i += kT) k255[i] = k255g[i];
        for (int i = tid; i < ncodes; i += kT) ctab[i] = k1_code_entry(G, i);
        unsigned* z = reinterpret_cast<unsigned*>(smem);
        for (int i = tid; i < V.code / 4; i += kT) z[i] = 0u;                        // counts, h / s sums
        for (int i = V.rcell / 4 + tid; i < V.ctab / 4; i += kT) z[i] = 0u;          // run records
        if (tid < 2) vote[16 * tid] = 0u;
    }
    // the (0, 0, 0) pixel's cell: masked groups past the image end are zero
    // pixels (c = 0, not below)
    const int code0 = tabs->code8[0];
    const int zcell = code0 < G.spvp ? 4 * code0 + 1 : G.gray_cb + code0 * G.hp2;
    __syncthreads();

    const long full_end = npix & ~3L;
    int img = (int)(it0 / nchunks), c = (int)(it0 - (long)img * nchunks);
    Mom m{0, 0, 0, 0, 0, 0};
    int seg_c0 = c;
    long seg_it0 = it0;
    // the next chunk's first 4-pixel group, loaded before the fold of the
    // current one (its HBM latency then passes under the fold's barriers)
    unsigned p0 = 0, p1 = 0, p2 = 0;
    bool have_pf = false, p_ok = false;                         // (have_pf block-uniform)
    for (long it = it0; it < it1; it++) {
        const long base = (long)c * kChunk;
        const int cimg = img, cc = c;
        if (++c == nchunks) {
            c = 0;
            img++;
        }
        const bool more = it + 1 < it1;
        const uint8_t* cip = imgs[cimg];
        unsigned emask = 0;                                       // deferred pixels (bit 4 st + i)
        {
            // one group (4 pixels) ahead only and the group loop not unrolled:
            // ~100 VGPRs without spills where the whole next chunk in registers
            // took 128 and spilled; the other waves of the CU hide the loads
            // (groups past the image end read pixel 0, masked below)
            const bool full = base + kChunk <= full_end;          // block-uniform: no group past the end
            // always a valid address, so the loads are unconditional (a
            // guarded load became an exec-masked branch per word); the words
            // of a group past the image end are masked where they are used
            // (a load whose value is selected at once, or that sits under a
            // branch, is waited for right there)
            auto ld_raw = [&](int st, unsigned& x0, unsigned& x1, unsigned& x2) {
                const bool ok = full || base + 4L * tid + 4L * kT * st < full_end;
                gu32t* q = (gu32t*)(cip + (ok ? (unsigned)(3 * (base + 4L * tid)) + 12u * kT * st : 0u));
                x0 = q[0];
                x1 = q[1];
                x2 = q[2];
                return ok;
            };
            auto ld = [&](int st, unsigned& x0, unsigned& x1, unsigned& x2) {
                const bool ok = ld_raw(st, x0, x1, x2);
                x0 = ok ? x0 : 0u;
                x1 = ok ? x1 : 0u;
                x2 = ok ? x2 : 0u;
            };
            // (the prefetch's mask applied here, so nothing waits for it before the fold)
            unsigned a0 = p_ok ? p0 : 0u, a1 = p_ok ? p1 : 0u, a2 = p_ok ? p2 : 0u;
            if (!have_pf) ld(0, a0, a1, a2);
            CellRun run{-1, 0, 0u, 0u, 0.0, 0.0};
            unsigned nsame = 0;                                   // this thread's groups in one cell
            auto loop = [&](auto mg) __attribute__((always_inline)) {
                constexpr bool M = decltype(mg)::value;
#pragma unroll 1
                for (int st = 0; st < kG; st++) {
                    // the next group (the last step reloads its own: unused)
                    unsigned n0, n1, n2;
                    const bool nok = ld_raw(st + 1 < kG ? st + 1 : st, n0, n1, n2);
                    emask |= k1_group<TRI, SMALL, M>(a0, a1, a2, m, code8, ctab, A, G, &run, nsame)
                             << (4 * st);
                    a0 = nok ? n0 : 0u;
                    a1 = nok ? n1 : 0u;
                    a2 = nok ? n2 : 0u;
                }
                if (M && run.cell >= 0) acc_add(A, run.cell, run.grp, run.lo, run.hi, run.h, run.s);
            };
            if (merge) loop(std::true_type{});
            else loop(std::false_type{});
            static_assert(kG < 16, "nsame <= kG: four bit slices");
            const unsigned nw = wave_sum_bits<4>(nsame);
            if (lane_id() == 0) atomicAdd(&vote[16 * vpar], nw);
        }
        const bool last_chunk = base + kChunk >= npix;            // block-uniform
        if (last_chunk && tid == 0) {
            // the < 4 pixels of a partial final group
            for (long p = full_end; p < npix; p++) {
                gu8t* pp = (gu8t*)(cip + 3 * p);
                const int kr = pp[0], kg = pp[1], kb = pp[2];
                m.sr += kr; m.sg += kg; m.sb += kb;
                m.qr += kr * kr; m.qg += kg * kg; m.qb += kb * kb;
                const int kmx = max(kr, max(kg, kb)), kmn = min(kr, min(kg, kb));
                const int code = code8[code_idx<TRI>(kmx, kmx - kmn)];
                K1Px px = k1_pixel<SMALL>(kr, kg, kb, kmx, kmn, kmx - kmn, code,
                                          k1_inv_pair(kmx - kmn > 1 ? kmx - kmn : 1, kmx > 1 ? kmx : 1), G);
                if (px.cell == ncell) px = k1_exact(kr, kg, kb, code, gp.Lh, k255, G);
                acc_add(A, px);
            }
        }
        // deferred pixels (a non-special hue exactly on a half-bin boundary,
        // ~1.7 % of uniform pixels, ~35 per wave and chunk) are redone in fp64 by
        // the whole wave: each lane queues its own (chunk offsets, this wave's LDS
        // queue), then every lane takes one, re-reading the pixel from global
        // memory (L2-resident: its chunk was just loaded).  One pass of the fp64
        // path per <= kDq deferred pixels of the wave, where each lane redoing its
        // own ran it as often as the wave's busiest lane had pixels (~3 times).
#if defined(PHD_K1_ABL_NODEFER)
        emask = 0u;                  // timing experiment only (wrong sums): no deferred pass
#endif
        {
            unsigned short* dq = reinterpret_cast<unsigned short*>(smem + V.dq) + (tid >> 6) * kDq;
            const int lane = lane_id();
            while (true) {                                        // wave-uniform
                unsigned utot;                                    // cnt <= 32: six bit slices
                int off = (int)wave_prefix_bits<6>((unsigned)__popc(emask), utot);
                const int total = (int)utot;
                if (total == 0) break;
                while (emask && off < kDq) {                      // what fits this round
                    const int bt = __ffs(emask) - 1;
                    emask &= emask - 1;
                    dq[off++] = (unsigned short)(4 * tid + 4 * kT * (bt >> 2) + (bt & 3));
                }
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                for (int k = lane; k < min(total, kDq); k += 64) {
                    gu8t* q = (gu8t*)(cip + 3 * (base + (long)dq[k]));
                    const int kr = q[0], kg = q[1], kb = q[2];
                    const int kmx = max(kr, max(kg, kb)), kmn = min(kr, min(kg, kb));
                    const K1Px px = k1_exact(kr, kg, kb, code8[code_idx<TRI>(kmx, kmx - kmn)], gp.Lh, k255, G);
                    acc_add(A, px);
                }
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();                  // the queue is read before it is refilled
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            }
        }
        const long pad = base + kChunk - full_end;                // zero pixels of masked groups
        if (pad > 0 && tid == 0)
            atomicAdd(cnt + (zcell << cshift), (unsigned long long)(-pad));
        {
            // (c, img) are the next chunk's already; as ld(0) of that chunk
            // (unconditional: a load under a branch is waited for at the join)
            have_pf = more;
            const long nbase = (long)c * kChunk;
            p_ok = more && (nbase + kChunk <= full_end || nbase + 4L * tid < full_end);
            gu32t* q = (gu32t*)((more ? imgs[img] : cip) + (p_ok ? (unsigned)(3 * (nbase + 4L * tid)) : 0u));
            p0 = q[0];
            p1 = q[1];
            p2 = q[2];
        }
        __syncthreads();
#if defined(PHD_K1_MERGE_DEN)
        merge = PHD_K1_MERGE_DEN * vote[16 * vpar] > (unsigned)(kT * kG);   // A/B builds: other thresholds
#else
        merge = 5 * vote[16 * vpar] > (unsigned)(kT * kG);       // the next chunk's mode: > 1/5 of groups
#endif
        // fold the chunk's count words: one thread per cell sums its C copies;
        // the run's cell counts, the chunk's group counts, per-group sum kmax / n255
#if defined(PHD_K1_ABL_NOFOLD)
        for (int q = tid; q <= 0; q += kT) {   // timing experiment only (wrong counts): no chunk fold
#else
        for (int q = tid; q <= ncell; q += kT) {
#endif
            unsigned long long v = 0;
            for (int k = 0; k < C; k++) {
                unsigned long long* wp = cnt + ((q << cshift) + k);
                v += *wp;
                *wp = 0ull;
            }
            if (q < ncell && v) {
                const unsigned cnt = (unsigned)(v & 0xFFFFu);
                const int g = group_of_cell(q, G);
                rcell[q] += cnt;
                atomicAdd(&cg[g], cnt);
                atomicAdd(&rmx[g], v >> 32);
                atomicAdd(&r255[g], (unsigned)(v >> 16) & 0xFFFFu);
            }
        }
        __syncthreads();
        if (tid == 0) vote[16 * vpar] = 0u;                      // read by every thread before this barrier
        vpar ^= 1;
        unsigned short* chunk_out =
            reinterpret_cast<unsigned short*>(reinterpret_cast<char*>(out.chunk_hist) + cimg * h_stride) +
            (long)cc * tl;
        for (int g = tid; g < tl; g += kT) {
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
            __syncthreads();
            char* arec = reinterpret_cast<char*>(out.sums) + cimg * a_stride;   // image's A record base
            double* gsum = reinterpret_cast<double*>(reinterpret_cast<char*>(out.gsum) + cimg * a_stride);
            unsigned* hist = reinterpret_cast<unsigned*>(reinterpret_cast<char*>(out.hist) + cimg * a_stride);
            unsigned* gcell = reinterpret_cast<unsigned*>(reinterpret_cast<char*>(out.gcell) + cimg * a_stride);
            double sacc = 0.0;
            for (int g = tid; g < tl; g += kT) {
                const unsigned n = seg[g];
                if (n) {
                    atomicAdd(&hist[g], n);
                    const unsigned n255 = r255[g];
                    const double sv = (double)(rmx[g] - 255ull * n255) * (1.0 / 255.0) + 0.999999 * (double)n255;
                    atomicAdd(&gsum[2 * tl + g], sv);
                }
                // the run's h / s sums of group g: its CH copies (one thread per group)
                double h = 0.0, s = 0.0;
                for (int k = 0; k < CH; k++) {
                    h += hsum[(g << hshift) + k];
                    s += ssum[(g << hshift) + k];
                    hsum[(g << hshift) + k] = 0.0;
                    ssum[(g << hshift) + k] = 0.0;
                }
                if (h != 0.0) atomicAdd(&gsum[g], h);
                if (s != 0.0) atomicAdd(&gsum[tl + g], s);
                sacc += s;
                seg[g] = 0;
                r255[g] = 0;
                rmx[g] = 0;
            }
            if (tid < CH) {                                       // the deferred pixels' dummy group
                hsum[(tl << hshift) + tid] = 0.0;
                ssum[(tl << hshift) + tid] = 0.0;
            }
            for (int q = tid; q < ncell; q += kT) {
                const unsigned n = rcell[q];
                if (n) atomicAdd(&gcell[q], n);
                rcell[q] = 0;
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
            m = Mom{0, 0, 0, 0, 0, 0};
            seg_c0 = c;
            seg_it0 = it + 1;
            __syncthreads();                                      // red is reused by the next flush
        }
    }
}

template <int KT, bool TRI>
void launch_form(int grid, size_t lds, hipStream_t st, const uint8_t* const* d_imgs, long npix, int nchunks,
                 long nitems, const GridParams& gp, const K1Grid& G, const ClassTables* tabs, const double* k255,
                 const PaletteDev& out0, long a_stride, long h_stride, int cfg) {
    if (G.small_c)
        phd_launch((k_k1t<KT, TRI, true>), dim3(grid), dim3(KT), lds, st, d_imgs, npix, nchunks, nitems, gp, G, tabs,
                   k255, out0, a_stride, h_stride, cfg);
    else
        phd_launch((k_k1t<KT, TRI, false>), dim3(grid), dim3(KT), lds, st, d_imgs, npix, nchunks, nitems, gp, G,
                   tabs, k255, out0, a_stride, h_stride, cfg);
}

constexpr int kLds1 = 158 * 1024;   // one block per CU
constexpr int kLds2 = 79 * 1024;    // two blocks per CU

}  // namespace

// Expected LDS cycles of one 16-lane group's 64-bit atomic into an array of
// (slots x 2^k lane copies), copy = lane & (2^k - 1), slots random: the lanes
// of one copy spread over 16 / 2^k bank pairs, the group takes the largest
// pile (16 copies: one cycle, conflict-free).
static double k1_conflicts(int k) {
    static const double e[5] = {3.3, 3.1, 2.5, 2.0, 1.0};
    return e[k < 0 ? 0 : (k > 4 ? 4 : k)];
}

// The accumulator layout (k1_cfg: count-word and h / s copy shifts) of least
// expected conflict cost -- one count atomic and two h / s atomics per pixel --
// that fits `lds` bytes with code table `code_bytes`, or -1.  At least
// 2^cs_min count copies (flat images put many lanes on one cell).
static int k1_config(const GridParams& gp, int code_bytes, int lds, int cs_min) {
    const int ncell = HueCells::count(gp);
    int best = -1;
    double bc = 1e30;
    for (int cs = 3; cs >= cs_min; cs--)
        for (int hs = 4; hs >= 0; hs--) {
            const int cfg = k1_cfg(cs, hs);
            if (l_var(gp.tl, ncell, cfg, code_bytes, gp.sp * gp.vp + gp.ng + 1).end > lds) continue;
            const double c = k1_conflicts(cs) + 2.0 * k1_conflicts(hs);
            if (c < bc - 1e-9) {
                bc = c;
                best = cfg;
            }
        }
    return best;
}

// the one-block form's layouts: the full code table, and the triangular one
// (fine grids: 36/4/5's 3312 hue cells only fit with it)
static int cfg_full(const GridParams& gp) { return k1_config(gp, code_bytes<false>(), kLds1, 0); }
static int cfg_tri1(const GridParams& gp) { return k1_config(gp, code_bytes<true>(), kLds1, 0); }
static double cfg_cost(int cfg) { return cfg < 0 ? 1e30 : k1_conflicts(k1_cs(cfg)) + 2.0 * k1_conflicts(k1_hs(cfg)); }

// >= 0 when the table K1 runs this grid (a k1_cfg of the one-block form)
int k1t_cshift(const GridParams& gp, const ClassTables& t) {
    if (!t.codes_ok) return -1;
    return std::max(cfg_full(gp), cfg_tri1(gp));
}

// the two-block form's layout (triangular code table, >= 2 count copies), -1
// when it does not fit
int k1t_cshift2(const GridParams& gp, const ClassTables& t) {
    if (!t.codes_ok) return -1;
    return k1_config(gp, code_bytes<true>(), kLds2, 1);
}

hipError_t launch_k1t_batch(const uint8_t* const* d_imgs, int n, int height, int width, const GridParams& gp,
                            const ClassTables* tabs, const PaletteDev& out0, long a_stride, long h_stride,
                            int nchunks, const double* k255, int cshift, int cshift2, hipStream_t st) {
    const long npix = (long)height * width;
    const long nitems = (long)n * nchunks;
    const int ncell = HueCells::count(gp);
    K1Grid G;
    k1_grid_init(G, gp);
    // once per process, thread-safe (two lanes may launch concurrently)
    static const bool attr = [] {
        const void* fs[] = {(const void*)k_k1t<1024, false, true>, (const void*)k_k1t<1024, false, false>,
                            (const void*)k_k1t<1024, true, true>,  (const void*)k_k1t<1024, true, false>,
                            (const void*)k_k1t<512, true, true>,   (const void*)k_k1t<512, true, false>};
        for (const void* f : fs) (void)hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        return true;
    }();
    (void)attr;
    // the two-block form runs a chunk in ~1.9x the time of the one-block form
    // (half a CU each): it wins when it has at least ~2 chunks per block, not
    // for a single image's 732 chunks where its last chunks form the tail.
    // Measured and removed (round 4): three 512-thread
    // blocks per CU (44.9 against 40.9 us per image), reciprocals from an LDS
    // table (45.7), the whole next chunk prefetched into registers (spills).
    const long cus = num_cus();
    const bool two = cshift2 >= 0 && 19 * ((nitems + 2 * cus - 1) / (2 * cus)) < 10 * ((nitems + cus - 1) / cus);
    if (two) {                                            // two 512-thread blocks per CU
        const size_t lds = (size_t)l_var(gp.tl, ncell, cshift2, code_bytes<true>(), k1_ncodes(G)).end;   // (a k1_cfg)
        // on a call split over two lanes, one block per CU: the other half of
        // each CU stays free for the other lane's FFT blocks (k1_blocks_per_cu)
        const int grid = (int)std::min<long>(nitems, (long)k1_blocks_per_cu() * cus);
        launch_form<512, true>(grid, lds, st, d_imgs, npix, nchunks, nitems, gp, G, tabs, k255, out0, a_stride,
                               h_stride, cshift2);
    } else {                                              // one 1024-thread block per CU
        const int grid = (int)std::min<long>(nitems, cus);
        // the triangular code table leaves 31 KiB more for the accumulators'
        // lane copies (fine grids: 36/4/5's 3312 hue cells only fit with it);
        // the full table where its layout is as good
        const int c_full = cfg_full(gp), c_tri = cfg_tri1(gp);
        if (c_tri < 0 && c_full < 0) return hipErrorInvalidValue;   // k1t_cshift said no
        if (cfg_cost(c_tri) < cfg_cost(c_full) - 1e-9) {
            const size_t lds = (size_t)l_var(gp.tl, ncell, c_tri, code_bytes<true>(), k1_ncodes(G)).end;
            launch_form<1024, true>(grid, lds, st, d_imgs, npix, nchunks, nitems, gp, G, tabs, k255, out0, a_stride,
                                    h_stride, c_tri);
        } else {
            const size_t lds = (size_t)l_var(gp.tl, ncell, c_full, code_bytes<false>(), k1_ncodes(G)).end;
            launch_form<1024, false>(grid, lds, st, d_imgs, npix, nchunks, nitems, gp, G, tabs, k255, out0,
                                     a_stride, h_stride, c_full);
        }
    }
    return hipGetLastError();
}

// The per-pixel logic of K1 run on the host (tests/test_k1_pixel.py): for n
// interleaved RGB8 pixels, the hue cell (HueCells layout), h and s, exactly
// as the kernel classifies them (deferred pixels through k1_exact).
int k1_host_pixels(const GridParams& gp, const ClassTables& t, const uint8_t* rgb, long n, int* cell, double* h,
                   double* s, int* deferred) {
    if (!t.codes_ok) return -1;
    K1Grid G;
    k1_grid_init(G, gp);
    double k255[256];
    for (int k = 0; k < 256; k++) k255[k] = (double)k / 255.0;
    for (long i = 0; i < n; i++) {
        const int kr = rgb[3 * i], kg = rgb[3 * i + 1], kb = rgb[3 * i + 2];
        const int kmx = std::max(kr, std::max(kg, kb)), kmn = std::min(kr, std::min(kg, kb)), kd = kmx - kmn;
        const int code = t.code8[kmx * 256 + kd];
        const K1Inv e = k1_inv_pair(kd > 1 ? kd : 1, kmx > 1 ? kmx : 1);   // as the production kernel
        // X through the kernel's packed pair form (this pixel in the high
        // half, its channel-rotated twin in the low half: both lanes checked)
        const k1_u16x2 r2 = {(unsigned short)kg, (unsigned short)kr}, g2 = {(unsigned short)kb, (unsigned short)kg},
                       b2 = {(unsigned short)kr, (unsigned short)kb};
        const k1_u16x2 m2 = {(unsigned short)kmx, (unsigned short)kmx}, d2 = {(unsigned short)kd, (unsigned short)kd};
        const k1_u16x2 x2 = k1_x_pair(r2, g2, b2, m2, d2);
        const int X = x2[1];
        const bool special = (kr == kg) | (kg == kb) | (kr == kb);
        if (x2[0] != k1_x_pair((k1_u16x2){(unsigned short)kg, 0}, (k1_u16x2){(unsigned short)kb, 0},
                               (k1_u16x2){(unsigned short)kr, 0}, m2, d2)[0])
            return -2;                                   // the two lanes of a pair disagree
        const K1Code ce = k1_code_entry(G, code);
        K1Px p = G.small_c ? k1_pixel_x<true>(X, special, kmx, kmn, kd, ce, e, G)
                           : k1_pixel_x<false>(X, special, kmx, kmn, kd, ce, e, G);
        const bool def = p.cell == G.ncell;
        if (def) p = k1_exact(kr, kg, kb, code, gp.Lh, k255, G);
        // the group the kernel's h / s atomics use must be the cell's (HueCells)
        const int want_g = p.cell < 4 * G.gs ? p.cell >> 2 : G.gs + (p.cell - 4 * G.gs) / G.hp2;
        if (p.grp != want_g) return -3;
        cell[i] = p.cell;
        h[i] = p.h;
        s[i] = p.s;
        if (deferred) deferred[i] = def;
    }
    return 0;
}

}  // namespace phd
