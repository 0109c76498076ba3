// palette.hip -- K1 (hsv + RGB statistics + group histogram), Kcut (keep-cutoff
// search for tie-overflow groups) and K3 (per-palette-slot sums).
//
// Replaces the per-pixel loops of rgb2hsv (src/image_processing.c:384-415),
// get_rgb_statistics / get_average / get_variance (image_processing.c:543-553,
// filtering.c:125-148), get_hsv_average (image_processing.c:533-540),
// arm_octree (src/color_quantization.c:127-159) and calculate_avg_hsv
// (color_quantization.c:529-558).  The HSV image is never materialised: both
// passes recompute HSV from the RGB8 bytes in registers.
//
// Layout: one image = interleaved RGB8, row-major, 3*W bytes per row.  A block
// owns kChunk consecutive hsv pixels; each thread consumes 4 consecutive pixels
// (12 bytes, one dwordx3 load) per step so a wave reads 768 contiguous bytes.
#include <cstdlib>

#include "phd_device.h"

namespace phd {

namespace {

// LDS carve of K1 (one dynamic array, 16-B aligned base: no static __shared__).
constexpr int kK1Threads = 1024;             // Kcut block: 16 waves over one kChunk
constexpr int kPalThreads = 512;             // K1 block: 8 waves, two resident per CU
constexpr int kK3Threads = 1024;             // K3 block: one per CU (its LDS sums want the room)
struct K1Lds {
    static constexpr int k255 = 0;           // 256 doubles
    static constexpr int ent = 2048;         // 256 ClsEnt (16 B)
    static constexpr int red = 6144;         // 16 waves x 8 x u64
    static constexpr int qn = 7168;          // Kcut scratch (16 B)
    static constexpr int area = 7184;        // K1: 2 x (tl+1) x C chunk-count copies + tl; K3: rules, sums
};
static_assert(sizeof(ClsEnt) == 16, "ClsEnt is one 16-B LDS read");

__device__ __forceinline__ void stage_tables(unsigned char* smem, const double* __restrict__ k255g,
                                             const ClassTables* __restrict__ tabs) {
    const int tid = threadIdx.x;
    for (int i = tid; i < 256; i += blockDim.x) {
        reinterpret_cast<double*>(smem + K1Lds::k255)[i] = k255g[i];
        reinterpret_cast<ClsEnt*>(smem + K1Lds::ent)[i] = tabs->ent[i];
    }
}

__device__ __forceinline__ void load4(const uint8_t* __restrict__ img, long p0, long end,
                                      bool aligned, unsigned (&k)[12], int& nvalid) {
    if (aligned && p0 + 3 < end) {
        const unsigned* w = reinterpret_cast<const unsigned*>(img + 3 * p0);
        const unsigned w0 = w[0], w1 = w[1], w2 = w[2];
#pragma unroll
        for (int i = 0; i < 4; i++) {
            k[i] = (w0 >> (8 * i)) & 255u;
            k[4 + i] = (w1 >> (8 * i)) & 255u;
            k[8 + i] = (w2 >> (8 * i)) & 255u;
        }
        nvalid = 4;
    } else {
        nvalid = 0;
#pragma unroll
        for (int i = 0; i < 4; i++) {
            if (p0 + i < end) {
                k[3 * i + 0] = img[3 * (p0 + i) + 0];
                k[3 * i + 1] = img[3 * (p0 + i) + 1];
                k[3 * i + 2] = img[3 * (p0 + i) + 2];
                nvalid++;
            } else {
                k[3 * i + 0] = k[3 * i + 1] = k[3 * i + 2] = 0;
            }
        }
    }
}

typedef const __attribute__((address_space(1))) unsigned gu32;   // global (not flat) loads

__device__ __forceinline__ int px_byte(const unsigned (&w)[3], int b) { return (w[b >> 2] >> (8 * (b & 3))) & 255; }
// One of four words by a runtime index, from values the compiler cannot trace
// back to a register array (it would turn the selects into a dynamically
// indexed array, i.e. scratch memory)
__device__ __forceinline__ unsigned sel4_opaque(int k, unsigned a, unsigned b, unsigned c, unsigned d) {
    asm volatile("" : "+v"(a), "+v"(b), "+v"(c), "+v"(d));
    return k == 0 ? a : (k == 1 ? b : (k == 2 ? c : d));
}
// pixel i (runtime, 0-3) of a 4-pixel group's words w0 w1 w2 in bits 0-23
__device__ __forceinline__ unsigned px_word(unsigned w0, unsigned w1, unsigned w2, int i) {
    const unsigned p1 = __builtin_amdgcn_alignbyte(w1, w0, 3u), p2 = __builtin_amdgcn_alignbyte(w2, w1, 2u);
    return i == 0 ? w0 : (i == 1 ? p1 : (i == 2 ? p2 : w2 >> 8));
}

// Add one to lds[g] for every lane with g >= 0; a wave whose lanes all hit the
// same group issues one atomic (flat regions of real images).
__device__ __forceinline__ void hist_add(unsigned* lds, int g) {
    const int g0 = __builtin_amdgcn_readfirstlane(g);
    const unsigned long long active = __ballot(1);   // before any lane-dependent branch
    if (__all(g == g0)) {
        if (g0 >= 0 && lane_id() == 0) atomicAdd(&lds[g0], (unsigned)__popcll(active));
    } else if (g >= 0) {
        atomicAdd(&lds[g], 1u);
    }
}

// ablate (PHD_ABLATE, timing runs only): K1 8 classify, 16 hist atomic, 32 sat,
// 64 chunk fold, 128 global atomics; K3 8 classify, 16 LDS sums, 32 hue
#ifndef PHD_K1_MINWAVES
#define PHD_K1_MINWAVES 8        // waves/SIMD the statistics-only K1 is sized for (2 blocks/CU)
#endif
#ifndef PHD_K1_MINWAVES_HIST
#define PHD_K1_MINWAVES_HIST 4   // histogram K1 (1024 threads, <= 128 VGPRs: one block per CU)
#endif

// Per-image outputs of a batch: image i's records sit at i * stride bytes.
__device__ __forceinline__ unsigned long long* img_sums(const PaletteDev& o, long a_stride, int i) {
    return reinterpret_cast<unsigned long long*>(reinterpret_cast<char*>(o.sums) + i * a_stride);
}
__device__ __forceinline__ unsigned* img_hist(const PaletteDev& o, long a_stride, int i) {
    return reinterpret_cast<unsigned*>(reinterpret_cast<char*>(o.hist) + i * a_stride);
}
__device__ __forceinline__ double* img_spart(const PaletteDev& o, long a_stride, int i) {
    return reinterpret_cast<double*>(reinterpret_cast<char*>(o.s_part) + i * a_stride);
}
__device__ __forceinline__ unsigned short* img_chunks(const PaletteDev& o, long h_stride, int i) {
    return reinterpret_cast<unsigned short*>(reinterpret_cast<char*>(o.chunk_hist) + i * h_stride);
}

__device__ __forceinline__ double* img_gsum(const PaletteDev& o, long a_stride, int i) {
    return reinterpret_cast<double*>(reinterpret_cast<char*>(o.gsum) + i * a_stride);
}
__device__ __forceinline__ unsigned* img_gcell(const PaletteDev& o, long a_stride, int i) {
    return reinterpret_cast<unsigned*>(reinterpret_cast<char*>(o.gcell) + i * a_stride);
}

// Bytes of K1's chunk-count copies and run counts (the fused sums follow, 8-B aligned).
__host__ __device__ __forceinline__ int k1_count_bytes(int tl, int cshift) {
    return (4 * (2 * (tl + 1) * (1 << cshift) + tl) + 15) & ~15;
}

typedef const __attribute__((address_space(1))) uint8_t gu8;

// Byte b of pixel group st of w (registers; st is not a compile-time index).
template <int kSteps>
__device__ __forceinline__ int step_byte(const unsigned (&w)[kSteps][3], int st, int b) {
    unsigned x = 0;
#pragma unroll
    for (int k = 0; k < kSteps; k++) x = k == st ? w[k][b >> 2] : x;
    return (x >> (8 * (b & 3))) & 255;
}

// The 12 bytes of pixels p0..p0+3 of an image as three little-endian words.
// Groups not wholly inside the image load from pixel 0 and are masked by the
// caller (the `ok` bits); so every load is unconditional and stays in flight.
template <bool kAligned>
__device__ __forceinline__ void load_group(const uint8_t* ip, long p0, bool ok, unsigned (&w)[3]) {
    const long a = ok ? 3 * p0 : 0;
    if (kAligned) {
        gu32* q = (gu32*)(ip + a);
        w[0] = q[0];
        w[1] = q[1];
        w[2] = q[2];
    } else {
        gu8* b = (gu8*)(ip + a);
#pragma unroll
        for (int k = 0; k < 3; k++)
            w[k] = (unsigned)b[4 * k] | (unsigned)b[4 * k + 1] << 8 | (unsigned)b[4 * k + 2] << 16 |
                   (unsigned)b[4 * k + 3] << 24;
    }
}

// K1 for downsample_rate == 1, over a whole batch of same-size images in one
// launch: channel moments, sum(s) and (kHist) the group histogram.
//
// The batch is a sequence of (image, chunk) work items of kChunk pixels; each
// persistent block (2 per CU) takes one contiguous run of items, so it crosses
// at most a few image boundaries.  Moments and sum(s) stay in registers and
// are flushed (block reduction + one atomic per counter) when the run leaves
// an image.  The per-chunk group counts are built in LDS (double-buffered, so
// a chunk costs two barriers), written out for the cutoff search, and summed
// into a per-run LDS histogram that is flushed with the moments.  Pixels
// classify through classify_e() (branch-free, four pixels' table reads in
// flight); the few whose hue lies exactly on a bin edge are marked in a
// per-thread mask and classified exactly after the chunk's stream.  The
// next item's loads are issued before the current chunk's barriers.
// The chunk counts have C = 1 << cshift lane-private copies (lane l adds to
// copy l mod C), so the per-pixel LDS atomics never collide within a wave.
// kHist == false is the rgb2hsv + statistics pass alone (S-bar and moments).
//
// Each thread owns kSteps groups of 4 pixels (12 bytes, one dwordx3) per
// chunk, a wave reading 768 contiguous bytes per group step.  Groups past the
// image end are masked to (0, 0, 0) pixels, which add nothing to the moments
// or sum(s) and are taken back out of the histogram; the < 4 pixels of a
// partial final group are done by one thread of the last chunk.
//
// kSums (the fused palette pass, needs kHist): per group, also sum(h), sum(s),
// sum(v) and the counts per hue cell (HueCells), so calculate_avg_hsv's slot
// sums of every group kept whole follow on the host without a second pass.
// They have the same C lane-private copies and are flushed with the run.
template <bool kHist, bool kSums, bool kAligned, bool kThr>
__global__ __launch_bounds__(kPalThreads, kHist ? PHD_K1_MINWAVES_HIST : PHD_K1_MINWAVES) void k_hsv_stats(
        const uint8_t* const* __restrict__ imgs, long npix, int nchunks, long nitems, GridParams gp, FastCls fc,
        const ClassTables* __restrict__ tabs, const double* __restrict__ k255g, PaletteDev out, long a_stride,
        long h_stride, int cshift, int ablate_arg) {
    const int ablate = PHD_ABL(ablate_arg);
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const double* k255 = reinterpret_cast<const double*>(smem + K1Lds::k255);
    const ClsEnt* ent = reinterpret_cast<const ClsEnt*>(smem + K1Lds::ent);
    const signed char* si8 = tabs->si8;                                 // global (s_partitions > 8 only)
    unsigned long long* red = reinterpret_cast<unsigned long long*>(smem + K1Lds::red);
    const int tl = gp.tl;
    const int tl1 = tl + 1;                                             // + dummy slot (deferred pixels)
    const int C = 1 << cshift, cm = C - 1;
    unsigned* lh = reinterpret_cast<unsigned*>(smem + K1Lds::area);   // [2][tl1][C] chunk counts
    unsigned* seg = lh + 2 * tl1 * C;                                  // [tl] counts of the run
    const int ncell = HueCells::count(gp);
    double* acc = reinterpret_cast<double*>(smem + K1Lds::area + k1_count_bytes(tl, cshift));  // [3][tl1][C]
    unsigned* cel = reinterpret_cast<unsigned*>(acc + 3 * tl1 * C);   // [ncell + 1][C]
    const int tid = threadIdx.x;
    const int mycopy = tid & cm;
    const long it0 = (long)blockIdx.x * nitems / gridDim.x, it1 = (long)(blockIdx.x + 1) * nitems / gridDim.x;
    if (it0 >= it1) return;                                 // block-uniform
    stage_tables(smem, k255g, tabs);
    if (kHist) {
        for (int i = tid; i < 2 * tl1 * C + tl; i += kPalThreads) lh[i] = 0;
    }
    if (kSums) {
        for (int i = tid; i < 3 * tl1 * C; i += kPalThreads) acc[i] = 0.0;
        for (int i = tid; i < (ncell + 1) * C; i += kPalThreads) cel[i] = 0;
    }
    __syncthreads();

    constexpr int kSteps = kChunk / (4 * kPalThreads);
    static_assert(kSteps >= 2 && kSteps <= 8, "K1 step count");
    const long full_end = npix & ~3L;                       // groups wholly inside the image
    unsigned w[kSteps][3];
    unsigned okb = 0;                                       // bit st: group st is inside
    auto issue = [&](const uint8_t* ip, int c) {
        okb = 0;
#pragma unroll
        for (int st = 0; st < kSteps; st++) {
            const long p0 = (long)c * kChunk + 4L * tid + 4L * kPalThreads * st;
            const bool ok = p0 < full_end;
            okb |= (unsigned)ok << st;
            load_group<kAligned>(ip, p0, ok, w[st]);
        }
    };
    int img = (int)(it0 / nchunks), c = (int)(it0 - (long)img * nchunks);
    const uint8_t* ip = imgs[img];
    issue(ip, c);
    // per-thread moments of the current run: u32 holds 4096 chunks of squares
    // (16 px * 255^2 each), so a run is flushed at the latest after 4096 chunks
    unsigned sr = 0, sg = 0, sb = 0, qr = 0, qg = 0, qb = 0;
    double ssum = 0.0;
    int seg_c0 = c, par = 0;
    long seg_it0 = it0;
    for (long it = it0; it < it1; it++, par ^= 1) {
        unsigned* ch = lh + par * tl1 * C;
        const long base = (long)c * kChunk;
        // one group (4 pixels) per iteration; the words rotate through
        // registers so the loop is not unrolled (bounded live state)
        unsigned bits = okb;
        unsigned emask = 0;                                  // this thread's edge pixels (bit 4*st + i)
        unsigned c0 = (bits & 1) ? w[0][0] : 0u, c1 = (bits & 1) ? w[0][1] : 0u, c2 = (bits & 1) ? w[0][2] : 0u;
#pragma unroll 1
        for (int st = 0; st < kSteps; st++) {
            const unsigned cw[3] = {c0, c1, c2};
            // phase 1: bytes, moments, the 4 table reads; phase 2: groups
            int kr[4], kg[4], kb[4];
            ClsEnt e[4];
#pragma unroll
            for (int i = 0; i < 4; i++) {
                kr[i] = px_byte(cw, 3 * i);
                kg[i] = px_byte(cw, 3 * i + 1);
                kb[i] = px_byte(cw, 3 * i + 2);
                sr += kr[i]; sg += kg[i]; sb += kb[i];
                qr += kr[i] * kr[i]; qg += kg[i] * kg[i]; qb += kb[i] * kb[i];
                if (kHist) e[i] = ent[max(kr[i], max(kg[i], kb[i]))];
            }
#pragma unroll
            for (int i = 0; i < 4; i++) {
                const int kmx = max(kr[i], max(kg[i], kb[i])), kmn = min(kr[i], min(kg[i], kb[i]));
                const double sv = sat_of(kmx, kmn);
                if (!(ablate & 32)) ssum += sv;
                if (kSums) {
                    int hN, hD, cell;
                    const int g = classify_f<kThr>(kr[i], kg[i], kb[i], e[i], si8, gp, fc, hN, hD, cell);
                    // a non-special hue on a half-bin boundary (g == -2): after the stream
                    const int edge = g == -2;
                    emask |= (unsigned)edge << (4 * st + i);
                    const int a = ((edge ? tl : g) << cshift) | mycopy;
                    atomicAdd(&ch[a], 1u);
                    atomicAdd(&acc[a], (double)hN * inv_k(hD));
                    atomicAdd(&acc[tl1 * C + a], sv);
                    atomicAdd(&acc[2 * tl1 * C + a], v_fast(kmx));
                    atomicAdd(&cel[(cell << cshift) | mycopy], 1u);
                } else if (kHist) {
                    const int g = (ablate & 8) ? (kr[i] % tl) : classify_e<kThr>(kr[i], kg[i], kb[i], e[i], si8, gp, fc);
                    // a hue exactly on a bin edge (g == -2): counted after the stream
                    const int edge = g == -2;
                    emask |= (unsigned)edge << (4 * st + i);
                    if (!(ablate & 16)) atomicAdd(&ch[((edge ? tl : g) << cshift) | mycopy], 1u);
                }
            }
            bits >>= 1;
            const bool okn = bits & 1;
            c0 = okn ? w[1][0] : 0u;
            c1 = okn ? w[1][1] : 0u;
            c2 = okn ? w[1][2] : 0u;
#pragma unroll
            for (int k = 1; k + 1 < kSteps; k++) {
                w[k][0] = w[k + 1][0]; w[k][1] = w[k + 1][1]; w[k][2] = w[k + 1][2];
            }
        }
        const bool last_chunk = base + kChunk >= npix;         // block-uniform
        const int tail = (int)(npix & 3);
        if (last_chunk && tail && tid == 0) {
            // the partial final group of the image: one lane, plain atomics
            for (long p = full_end; p < npix; p++) {
                const int kr = ip[3 * p], kg = ip[3 * p + 1], kb = ip[3 * p + 2];
                sr += kr; sg += kg; sb += kb;
                qr += kr * kr; qg += kg * kg; qb += kb * kb;
                double sv;
                if (kSums) {
                    const int kmx = max(kr, max(kg, kb));
                    sv = sat_of(kmx, min(kr, min(kg, kb)));
                    int hN, hD, cell;
                    double h;
                    int g = classify_f<kThr>(kr, kg, kb, ent[kmx], si8, gp, fc, hN, hD, cell);
                    if (g == -2) g = fused_exact(kr, kg, kb, k255, gp, fc.lh, h, cell);
                    else h = (double)hN * inv_k(hD);
                    atomicAdd(&ch[g << cshift], 1u);
                    atomicAdd(&acc[g << cshift], h);
                    atomicAdd(&acc[(tl1 * C) + (g << cshift)], sv);
                    atomicAdd(&acc[(2 * tl1 * C) + (g << cshift)], v_fast(kmx));
                    atomicAdd(&cel[cell << cshift], 1u);
                } else if (kHist) {
                    int g = classify<kThr>(kr, kg, kb, ent, si8, gp, fc, sv);
                    if (g == -2) g = exact_group(kr, kg, kb, k255, gp);
                    atomicAdd(&ch[g << cshift], 1u);
                } else {
                    sv = sat_only(kr, kg, kb);
                }
                ssum += sv;
            }
        }
        // this thread's edge pixels: the exact group (fp64 hue, rgb2hsv's order)
        while (kHist && emask) {
            const int bt = __ffs(emask) - 1;
            emask &= emask - 1;
            const long p = base + 4L * tid + 4L * kPalThreads * (bt >> 2) + (bt & 3);
            const int kr = ip[3 * p], kg = ip[3 * p + 1], kb = ip[3 * p + 2];
            if (kSums) {
                double h;
                int cell;
                const int g = fused_exact(kr, kg, kb, k255, gp, fc.lh, h, cell);
                const int kmx = max(kr, max(kg, kb));
                const int a = (g << cshift) | mycopy;
                atomicAdd(&ch[a], 1u);
                atomicAdd(&acc[a], h);
                atomicAdd(&acc[tl1 * C + a], sat_of(kmx, min(kr, min(kg, kb))));
                atomicAdd(&acc[2 * tl1 * C + a], v_fast(kmx));
                atomicAdd(&cel[(cell << cshift) | mycopy], 1u);
            } else {
                const int g = exact_group(kr, kg, kb, k255, gp);
                atomicAdd(&ch[(g << cshift) | mycopy], 1u);
            }
        }
        // next work item: prefetch its pixels now
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
        if (kHist) {
            // zero pixels of masked groups (a whole-group count per chunk)
            const long pad = base + kChunk - full_end;
            if (pad > 0 && tid == 0) {
                double sv;
                atomicSub(&ch[classify<kThr>(0, 0, 0, ent, si8, gp, fc, sv) << cshift], (unsigned)pad);
                if (kSums) {
                    int hN, hD, cell;
                    (void)classify_f<kThr>(0, 0, 0, ent[0], si8, gp, fc, hN, hD, cell);
                    atomicSub(&cel[cell << cshift], (unsigned)pad);
                }
            }
            __syncthreads();
            // fold the C copies of each group (C consecutive lanes) with shuffles
            unsigned short* chunk_out = img_chunks(out, h_stride, cimg) + (long)cc * tl;
            const int ncopy = (ablate & 64) ? 0 : tl << cshift;
            for (int i0 = tid; i0 < ((ncopy + kPalThreads - 1) & ~(kPalThreads - 1)); i0 += kPalThreads) {
                unsigned n = 0;
                if (i0 < ncopy) {
                    n = ch[i0];
                    ch[i0] = 0;
                }
                for (int o = 1; o < C; o <<= 1) n += __shfl_xor(n, o, 64);
                if (i0 < ncopy && (i0 & cm) == 0) {
                    const int g = i0 >> cshift;
                    chunk_out[g] = (unsigned short)n;
                    seg[g] += n;
                }
            }
            if (tid < C) ch[(tl << cshift) + tid] = 0;        // the edge-pixel slot
        }
        if (!more || img != cimg || it + 1 - seg_it0 == 4096) {
            // the run leaves image cimg (or its u32 moments could overflow):
            // flush its moments, sum(s) and counts
            const int wv = tid >> 6;
            const unsigned mom[6] = {sr, sg, sb, qr, qg, qb};
            unsigned long long m64[6];
#pragma unroll
            for (int k = 0; k < 6; k++) m64[k] = wave_sum((unsigned long long)mom[k]);
            const double sw = wave_sum(ssum);
            if (lane_id() == 0) {
#pragma unroll
                for (int k = 0; k < 6; k++) red[wv * 8 + k] = m64[k];
                reinterpret_cast<double*>(red)[wv * 8 + 6] = sw;
            }
            __syncthreads();
            if (tid < 6) {
                unsigned long long t = 0;
                for (int q = 0; q < kPalThreads / 64; q++) t += red[q * 8 + tid];
                if (!(ablate & 128)) atomicAdd(&img_sums(out, a_stride, cimg)[tid], t);
            } else if (tid == 6) {
                double t = 0.0;
                for (int q = 0; q < kPalThreads / 64; q++) t += reinterpret_cast<double*>(red)[q * 8 + 6];
                img_spart(out, a_stride, cimg)[seg_c0] = t;   // one slot per run (host sums them)
            }
            if (kHist) {
                unsigned* hist = img_hist(out, a_stride, cimg);
                for (int i = tid; i < tl; i += kPalThreads) {
                    const unsigned n = seg[i];
                    if (n && !(ablate & 128)) atomicAdd(&hist[i], n);
                    seg[i] = 0;
                }
            }
            if (kSums) {
                // fold the C copies (consecutive lanes) of the sums and cell counts;
                // the deferred-pixel dummies (group tl, cell ncell) are just zeroed
                double* gsum = img_gsum(out, a_stride, cimg);
                unsigned* gcell = img_gcell(out, a_stride, cimg);
                const int nacc = 3 * tl1 * C;
                for (int i0 = tid; i0 < ((nacc + kPalThreads - 1) & ~(kPalThreads - 1)); i0 += kPalThreads) {
                    double a = 0.0;
                    if (i0 < nacc) {
                        a = acc[i0];
                        acc[i0] = 0.0;
                    }
                    for (int o = 1; o < C; o <<= 1) a += __shfl_xor(a, o, 64);
                    if (i0 < nacc && (i0 & cm) == 0) {
                        const int f = i0 / (tl1 * C), g = (i0 - f * tl1 * C) >> cshift;
                        if (g < tl && a != 0.0) atomicAdd(&gsum[f * tl + g], a);
                    }
                }
                const int ncel = (ncell + 1) * C;
                for (int i0 = tid; i0 < ((ncel + kPalThreads - 1) & ~(kPalThreads - 1)); i0 += kPalThreads) {
                    unsigned n = 0;
                    if (i0 < ncel) {
                        n = cel[i0];
                        cel[i0] = 0;
                    }
                    for (int o = 1; o < C; o <<= 1) n += __shfl_xor(n, o, 64);
                    const int q = i0 >> cshift;
                    if (i0 < ncel && (i0 & cm) == 0 && q < ncell && n) atomicAdd(&gcell[q], n);
                }
            }
            sr = sg = sb = qr = qg = qb = 0;
            ssum = 0.0;
            seg_c0 = c;
            seg_it0 = it + 1;
            __syncthreads();                                  // red is reused by the next flush
        }
    }
}

// Exclusive scan of one int per thread over a block of kK1Threads threads.
__device__ int block_excl_scan_k1(int x, int& excl, int* scratch) {
    const int lane = lane_id(), w = threadIdx.x >> 6;
    int incl = x;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(incl, o, 64);
        if (lane >= o) incl += y;
    }
    if (lane == 63) scratch[w] = incl;
    __syncthreads();
    int wpre = 0, tot = 0;
    for (int q = 0; q < kK1Threads / 64; q++) {
        if (q < w) wpre += scratch[q];
        tot += scratch[q];
    }
    __syncthreads();
    excl = wpre + incl - x;
    return tot;
}

// The same for a u64 (packed per-step counts).
__device__ unsigned long long block_excl_scan_k1_u64(unsigned long long x, unsigned long long& excl,
                                                     unsigned long long* scratch) {
    const int lane = lane_id(), w = threadIdx.x >> 6;
    unsigned long long incl = x;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const unsigned long long y = __shfl_up(incl, o, 64);
        if (lane >= o) incl += y;
    }
    if (lane == 63) scratch[w] = incl;
    __syncthreads();
    unsigned long long wpre = 0, tot = 0;
    for (int q = 0; q < kK1Threads / 64; q++) {
        if (q < w) wpre += scratch[q];
        tot += scratch[q];
    }
    __syncthreads();
    excl = wpre + incl - x;
    return tot;
}

// Exact group of a pixel: classify(), and the exact hue on a bin edge.
template <bool kThr>
__device__ __forceinline__ int exact_group_t(int kr, int kg, int kb, const ClsEnt* ent, const signed char* si8, const double* k255, const GridParams& gp,
                                             const FastCls& fc, double& s) {
    int g = classify<kThr>(kr, kg, kb, ent, si8, gp, fc, s);
    if (g == -2) g = edge_group<kThr>(kr, kg, kb, hue_exact(kr, kg, kb, k255), ent, si8, gp);
    return g;
}

// Is the pixel's exact group g?  Integer work for all but a pixel on a hue-bin
// edge whose candidate groups (classify_e's gcol, one hue bin below) include g.
template <bool kThr>
__device__ __forceinline__ bool in_group(int kr, int kg, int kb, int g, const ClsEnt* ent, const signed char* si8,
                                         const double* k255, const GridParams& gp, const FastCls& fc) {
    int hN, hD, gc;
    const int q = classify_e<kThr>(kr, kg, kb, ent[max(kr, max(kg, kb))], si8, gp, fc, hN, hD, gc);
    if (q != -2) return q == g;
    if (gc != g && gc - gp.sp * gp.vp != g) return false;
    return edge_group<kThr>(kr, kg, kb, hue_exact(kr, kg, kb, k255), ent, si8, gp) == g;
}

// Kcut for downsample_rate == 1, all images of a batch in one launch: one block
// per (image, group) whose keep rule needs raster positions (the tie path of
// group_irregular_pixels appends pixels in raster order until the parent's tail
// node is full, src/color_quantization.c:435-440): the index of the group's
// keep-th pixel (cutoff = index + 1) and of its last pixel (the dangling
// node).  The per-chunk counts of K1 locate the chunk; one pass over that
// chunk's 16384 pixels (16 per thread) and a block scan find the pixel.
template <bool kAligned, bool kThr>
__global__ __launch_bounds__(kK1Threads, 4) void k_cutoffs_b(
        const uint8_t* const* __restrict__ imgs, long npix, int nchunks, GridParams gp, FastCls fc,
        const ClassTables* __restrict__ tabs, const double* __restrict__ k255g, const int2* __restrict__ entries,
        const unsigned short* __restrict__ chunk_hist0, long h_stride, GroupRule* rules0, long b_stride) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const double* k255 = reinterpret_cast<const double*>(smem + K1Lds::k255);
    const ClsEnt* ent = reinterpret_cast<const ClsEnt*>(smem + K1Lds::ent);
    const signed char* si8 = tabs->si8;
    int* scratch = reinterpret_cast<int*>(smem + K1Lds::red);          // 16 x u64
    int* misc = reinterpret_cast<int*>(smem + K1Lds::red + 256);       // chunk, rank, last chunk
    unsigned* found = reinterpret_cast<unsigned*>(smem + K1Lds::qn);
    const int tid = threadIdx.x;
    stage_tables(smem, k255g, tabs);
    const int img = entries[blockIdx.x].x, g = entries[blockIdx.x].y;
    const uint8_t* ip = imgs[img];
    GroupRule* rules = reinterpret_cast<GroupRule*>(reinterpret_cast<char*>(rules0) + img * b_stride);
    const unsigned short* chunk_hist =
            reinterpret_cast<const unsigned short*>(reinterpret_cast<const char*>(chunk_hist0) + img * h_stride);
    const int tl = gp.tl;
    const int keep = rules[g].keep;
    const bool want_cut = rules[g].partial && keep > 0;
    const bool want_last = rules[g].partial && rules[g].dangle;
    if (tid == 0) { misc[0] = -1; misc[2] = -1; }
    __syncthreads();
    // chunk holding the keep-th pixel, and the last non-empty chunk
    int carry = 0;
    for (int c0 = 0; c0 < nchunks; c0 += kK1Threads) {
        const int c = c0 + tid;
        const int cnt = c < nchunks ? (int)chunk_hist[(long)c * tl + g] : 0;
        int excl;
        const int tot = block_excl_scan_k1(cnt, excl, scratch);
        if (want_cut && cnt > 0 && carry + excl < keep && keep <= carry + excl + cnt) {
            misc[0] = c;
            misc[1] = keep - (carry + excl);   // 1-based rank inside the chunk
        }
        if (cnt > 0) atomicMax(&misc[2], c);
        carry += tot;
    }
    __syncthreads();
    constexpr int kSteps = kChunk / (4 * kK1Threads);
    const long full_end = npix & ~3L;
    for (int pass = 0; pass < 2; pass++) {
        const int c = pass == 0 ? (want_cut ? misc[0] : -1) : (want_last ? misc[2] : -1);
        if (c < 0) continue;                                  // uniform across the block
        // this thread's 16 pixels: hit bits in raster order
        unsigned hits = 0;
#pragma unroll
        for (int st = 0; st < kSteps; st++) {
            const long p0 = (long)c * kChunk + 4L * tid + 4L * kK1Threads * st;
            unsigned w[3];
            load_group<kAligned>(ip, p0, p0 < full_end, w);
#pragma unroll
            for (int i = 0; i < 4; i++) {
                const long p = p0 + i;
                int kr, kg, kb;
                if (p0 < full_end) {
                    kr = px_byte(w, 3 * i); kg = px_byte(w, 3 * i + 1); kb = px_byte(w, 3 * i + 2);
                } else if (p < npix) {                        // partial final group
                    kr = ip[3 * p]; kg = ip[3 * p + 1]; kb = ip[3 * p + 2];
                } else {
                    continue;
                }
                if (in_group<kThr>(kr, kg, kb, g, ent, si8, k255, gp, fc)) hits |= 1u << (4 * st + i);
            }
        }
        if (tid == 0) *found = 0;
        // raster order inside the chunk is (step, thread, pixel): scan the
        // per-step hit counts (4 x 16-bit fields) over the threads
        unsigned long long packed = 0;
#pragma unroll
        for (int st = 0; st < kSteps; st++)
            packed |= (unsigned long long)__popc((hits >> (4 * st)) & 15u) << (16 * st);
        unsigned long long excl;
        const unsigned long long tot =
                block_excl_scan_k1_u64(packed, excl, reinterpret_cast<unsigned long long*>(scratch));
        if (pass == 0) {
            const int rank = misc[1];
            int before = 0;                                   // hits of the earlier steps
#pragma unroll
            for (int st = 0; st < kSteps; st++) {
                const int e = before + (int)((excl >> (16 * st)) & 0xFFFF);
                const int n = (int)((packed >> (16 * st)) & 0xFFFF);
                if (e < rank && rank <= e + n) {
                    unsigned m = (hits >> (4 * st)) & 15u;
                    for (int k = rank - e; k > 1; k--) m &= m - 1;   // drop the lower hits
                    const int i = __ffs(m) - 1;
                    *found = (unsigned)((long)c * kChunk + 4L * tid + 4L * kK1Threads * st + i) + 1;
                }
                before += (int)((tot >> (16 * st)) & 0xFFFF);
            }
        } else if (hits) {
            const int b = 31 - __clz(hits);
            atomicMax(found, (unsigned)((long)c * kChunk + 4L * tid + 4L * kK1Threads * (b >> 2) + (b & 3)) + 1);
        }
        __syncthreads();
        if (tid == 0) {
            if (pass == 0) rules[g].cutoff = *found;          // index + 1 of the keep-th pixel
            else rules[g].last = *found - 1;
        }
        __syncthreads();
    }
}

// K3 for downsample_rate == 1, all images of a batch in one launch: per palette
// slot, over the pixels its parent keeps (calculate_avg_hsv,
// src/color_quantization.c:529-558): sum wrap(h + off), sum s, sum v, count.
// Persistent blocks walk contiguous runs of (image, chunk) items like K1;
// per image the keep rules are packed into LDS as {slot, cut, last}: a pixel
// of a slotted group is kept when its index < cut or == last.  The sums have
// C = 1 << cshift lane-private copies per slot (lane l adds to copy l mod C):
// the fp64 LDS atomics of one wave hit distinct addresses (and, for C = 32,
// distinct banks), whatever the image.  Per image, the copies are folded and
// go to HBM with one atomic per slot and field.
template <bool kAligned, bool kThr>
__global__ __launch_bounds__(kK3Threads, 4) void k_palette_sums_b(
        const uint8_t* const* __restrict__ imgs, long npix, int nchunks, long nitems, GridParams gp, FastCls fc,
        const ClassTables* __restrict__ tabs, const double* __restrict__ k255g,
        const GroupRule* __restrict__ rules0, const double* __restrict__ off0, long b_stride,
        const int* __restrict__ nslots_img, int max_slots, double* out0, long c_stride, int cshift,
        int ablate_arg) {
    const int ablate = PHD_ABL(ablate_arg);
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const double* k255 = reinterpret_cast<const double*>(smem + K1Lds::k255);
    const ClsEnt* ent = reinterpret_cast<const ClsEnt*>(smem + K1Lds::ent);
    const signed char* si8 = tabs->si8;
    const int tl = gp.tl;
    const int C = 1 << cshift, cm = C - 1;
    // slot ms = max_slots and rule tl are dummies: pixels that are not kept
    // add into them, so the per-pixel code has no branch
    const int ms = max_slots + 1;
    uint4* rec = reinterpret_cast<uint4*>(smem + K1Lds::area);        // [tl + 1] {slot, cut, last, -}
    double* off = reinterpret_cast<double*>(rec + tl + 1);             // [ms]
    double* acc = off + ms;                                            // [3][ms][C] h, s, v
    unsigned* cnt = reinterpret_cast<unsigned*>(acc + 3 * ms * C);     // [ms][C]
    const int tid = threadIdx.x;
    const int mycopy = tid & cm;
    const long it0 = (long)blockIdx.x * nitems / gridDim.x, it1 = (long)(blockIdx.x + 1) * nitems / gridDim.x;
    if (it0 >= it1) return;                                 // block-uniform
    stage_tables(smem, k255g, tabs);
    for (int i = tid; i < ms * C; i += kK3Threads) {
        acc[i] = acc[ms * C + i] = acc[2 * ms * C + i] = 0.0;
        cnt[i] = 0;
    }
    if (tid == 0) {
        rec[tl] = make_uint4(0xFFFFFFFFu, 0u, 0xFFFFFFFFu, 0u);
        off[max_slots] = 0.0;
    }

    constexpr int kSteps = kChunk / (4 * kK3Threads);
    const long full_end = npix & ~3L;
    int img = (int)(it0 / nchunks), c = (int)(it0 - (long)img * nchunks);
    int cur = -1, ns = 0;
    for (long it = it0; it < it1; it++) {
        if (img != cur) {                                    // block-uniform: load image img's rules
            const GroupRule* rules =
                    reinterpret_cast<const GroupRule*>(reinterpret_cast<const char*>(rules0) + img * b_stride);
            const double* offi = reinterpret_cast<const double*>(reinterpret_cast<const char*>(off0) + img * b_stride);
            ns = nslots_img[img];
            for (int i = tid; i < tl; i += kK3Threads) {
                const GroupRule r = rules[i];
                uint4 q;
                q.x = (unsigned)r.slot;
                q.y = r.partial ? r.cutoff : 0xFFFFFFFFu;
                q.z = (r.partial && r.dangle) ? r.last : 0xFFFFFFFFu;
                q.w = 0;
                rec[i] = q;
            }
            for (int i = tid; i < ns; i += kK3Threads) off[i] = offi[i];
            for (int i = ns + tid; i < max_slots; i += kK3Threads) off[i] = 0.0;
            cur = img;
            __syncthreads();
        }
        const uint8_t* ip = imgs[img];
        const long base = (long)c * kChunk;
        unsigned w[kSteps][3];
#pragma unroll
        for (int st = 0; st < kSteps; st++) {
            const long p0 = base + 4L * tid + 4L * kK3Threads * st;
            load_group<kAligned>(ip, p0, p0 < full_end, w[st]);
        }
        unsigned emask = 0;                                  // this thread's edge pixels (bit 4*st + i)
#pragma unroll 1
        for (int st = 0; st < kSteps; st++) {
            const long p0 = base + 4L * tid + 4L * kK3Threads * st;
            const bool okg = p0 < full_end;
            unsigned cw[3];
#pragma unroll
            for (int k = 0; k < kSteps; k++)
                if (k == st) { cw[0] = w[k][0]; cw[1] = w[k][1]; cw[2] = w[k][2]; }
            // phases over the 4 pixels, so each step has 4 independent LDS reads
            // in flight: class entry -> group -> keep rule -> slot offset
            int kr[4], kg[4], kb[4], sl[4], hN[4], hD[4];
            ClsEnt e[4];
            uint4 q[4];
            double o[4];
#pragma unroll
            for (int i = 0; i < 4; i++) {
                kr[i] = px_byte(cw, 3 * i);
                kg[i] = px_byte(cw, 3 * i + 1);
                kb[i] = px_byte(cw, 3 * i + 2);
                e[i] = ent[max(kr[i], max(kg[i], kb[i]))];
            }
#pragma unroll
            for (int i = 0; i < 4; i++) {
                const int g = classify_e<kThr>(kr[i], kg[i], kb[i], e[i], si8, gp, fc, hN[i], hD[i]);
                const int edge = g == -2;                    // exact group after the stream
                emask |= (unsigned)(edge & (int)okg) << (4 * st + i);
                q[i] = rec[edge ? tl : g];
            }
#pragma unroll
            for (int i = 0; i < 4; i++) {
                const unsigned idx = (unsigned)(p0 + i);
                const bool kept = okg && (int)q[i].x >= 0 && (idx < q[i].y || idx == q[i].z);
                sl[i] = kept ? (int)q[i].x : max_slots;
                o[i] = off[sl[i]];
            }
#pragma unroll
            for (int i = 0; i < 4; i++) {
                // wrap(h + off) (calculate_avg_hsv, src/color_quantization.c:536-540): h = hN / hD
                // through a reciprocal (within an ulp); the exact quotient decides the wrap
                // whenever h + off is within 1e-9 of 0 or 360
                const int kmx = max(kr[i], max(kg[i], kb[i])), kmn = min(kr[i], min(kg[i], kb[i]));
                double tp = ((ablate & 32) ? 0.0 : (double)hN[i] * inv_k(hD[i])) + o[i];
                if (fabs(tp - 360.0) < 1e-9 || fabs(tp) < 1e-9) tp = hue_exact(kr[i], kg[i], kb[i], k255) + o[i];
                tp = tp > 360 ? tp - 360 : (tp < 0 ? tp + 360 : tp);
                const int a = (sl[i] << cshift) | mycopy;
                if (!(ablate & 16)) {
                    atomicAdd(&acc[a], tp);
                    atomicAdd(&acc[ms * C + a], sat_of(kmx, kmn));
                    atomicAdd(&acc[2 * ms * C + a], v_fast(kmx));
                    atomicAdd(&cnt[a], 1u);
                }
            }
        }
        // this thread's edge pixels: exact hue and group (rgb2hsv's order)
        while (emask) {
            const int bt = __ffs(emask) - 1;
            emask &= emask - 1;
            const int st = bt >> 2, i = bt & 3;
            const long p = base + 4L * tid + 4L * kK3Threads * st + i;
            const int kr = step_byte(w, st, 3 * i), kg = step_byte(w, st, 3 * i + 1), kb = step_byte(w, st, 3 * i + 2);
            const double hx = hue_exact(kr, kg, kb, k255);
            const int g = edge_group<kThr>(kr, kg, kb, hx, ent, si8, gp);
            const uint4 r = rec[g];
            const unsigned idx = (unsigned)p;
            if ((int)r.x >= 0 && (idx < r.y || idx == r.z)) {
                const int sl = (int)r.x;
                double tp = hx + off[sl];
                tp = tp > 360 ? tp - 360 : (tp < 0 ? tp + 360 : tp);
                const int kmx = max(kr, max(kg, kb)), kmn = min(kr, min(kg, kb));
                const int a = (sl << cshift) | mycopy;
                atomicAdd(&acc[a], tp);
                atomicAdd(&acc[ms * C + a], sat_of(kmx, kmn));
                atomicAdd(&acc[2 * ms * C + a], v_fast(kmx));
                atomicAdd(&cnt[a], 1u);
            }
        }
        if (base + kChunk >= npix && tid == 0) {
            // the partial final group of the image: one lane
            for (long p = full_end; p < npix; p++) {
                const int kr = ip[3 * p], kg = ip[3 * p + 1], kb = ip[3 * p + 2];
                double sv;
                const double hx = hue_exact(kr, kg, kb, k255);
                int g = classify<kThr>(kr, kg, kb, ent, si8, gp, fc, sv);
                if (g == -2) g = edge_group<kThr>(kr, kg, kb, hx, ent, si8, gp);
                const uint4 q = rec[g];
                const unsigned idx = (unsigned)p;
                if ((int)q.x >= 0 && (idx < q.y || idx == q.z)) {
                    const int sl = (int)q.x;
                    double tp = hx + off[sl];
                    tp = tp > 360 ? tp - 360 : (tp < 0 ? tp + 360 : tp);
                    const int a = sl << cshift;
                    atomicAdd(&acc[a], tp);
                    atomicAdd(&acc[ms * C + a], sv);
                    atomicAdd(&acc[2 * ms * C + a], v_of(max(kr, max(kg, kb)), k255));
                    atomicAdd(&cnt[a], 1u);
                }
            }
        }
        const int cimg = img;
        if (++c == nchunks) {
            c = 0;
            img++;
        }
        if (it + 1 == it1 || img != cimg) {                  // flush image cimg's sums
            __syncthreads();
            double* out = reinterpret_cast<double*>(reinterpret_cast<char*>(out0) + cimg * c_stride);
            // one (field, slot, copy) per lane; the C copies of a slot are
            // consecutive lanes and fold with shuffles
            const int ncopy = ns << cshift;
            const int total = 4 * ncopy;
            for (int i0 = tid; i0 < ((total + kK3Threads - 1) & ~(kK3Threads - 1)); i0 += kK3Threads) {
                const int f = i0 / max(ncopy, 1), j = i0 - f * ncopy;
                double a = 0.0;
                if (i0 < total) {
                    if (f < 3) {
                        double* src = &acc[f * ms * C + j];
                        a = *src;
                        *src = 0.0;
                    } else {
                        a = (double)cnt[j];
                        cnt[j] = 0;
                    }
                }
                for (int o = 1; o < C; o <<= 1) a += __shfl_xor(a, o, 64);
                if (i0 < total && (j & cm) == 0 && a != 0.0) atomicAdd(&out[4 * (j >> cshift) + f], a);
            }
            __syncthreads();
        }
    }
}

// Partial-group sums of the fused palette (downsample_rate == 1): the groups a
// tie sent to a parent's tail node keep only their first `keep` pixels in
// raster order plus, maybe, their last one (group_irregular_pixels,
// src/color_quantization.c:435-447; the cutoff and last index come from Kcut).
// Blocks (entry, split) walk the 4096-pixel units before the cutoff whose chunk
// holds pixels of the group (K1's chunk counts), split-strided, and add calculate_avg_hsv's
// terms of the kept pixels (:536-550: wrap(h + off), s, v, count) in
// registers; one atomic per field and block.  Typical partial groups keep a
// few hundred pixels of their first chunks.
constexpr int kPartThreads = 256;
template <bool kAligned, bool kThr>
__global__ __launch_bounds__(kPartThreads) void k_partial_sums_b(
        const uint8_t* const* __restrict__ imgs, long npix, GridParams gp, FastCls fc,
        const ClassTables* __restrict__ tabs, const double* __restrict__ k255g, const int2* __restrict__ entries,
        const unsigned short* __restrict__ chunk_hist0, long h_stride, const GroupRule* __restrict__ rules0,
        const double* __restrict__ off0, long b_stride, double* out0, long c_stride) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const double* k255 = reinterpret_cast<const double*>(smem + K1Lds::k255);
    const ClsEnt* ent = reinterpret_cast<const ClsEnt*>(smem + K1Lds::ent);
    double* red = reinterpret_cast<double*>(smem + K1Lds::red);       // [4 waves][4]
    const signed char* si8 = tabs->si8;
    const int tid = threadIdx.x;
    stage_tables(smem, k255g, tabs);
    __syncthreads();
    const int img = entries[blockIdx.x].x, g = entries[blockIdx.x].y;
    const uint8_t* ip = imgs[img];
    const GroupRule r = reinterpret_cast<const GroupRule*>(reinterpret_cast<const char*>(rules0) + img * b_stride)[g];
    const double off = reinterpret_cast<const double*>(reinterpret_cast<const char*>(off0) + img * b_stride)[r.slot];
    const unsigned short* chunk_hist =
            reinterpret_cast<const unsigned short*>(reinterpret_cast<const char*>(chunk_hist0) + img * h_stride);
    const int tl = gp.tl;
    const unsigned cut = (r.partial && r.keep > 0) ? r.cutoff : 0u;
    const long full_end = npix & ~3L;
    double th = 0.0, ts = 0.0, tv = 0.0, tn = 0.0;
    auto add = [&](int kr, int kg, int kb) {
        if (!in_group<kThr>(kr, kg, kb, g, ent, si8, k255, gp, fc)) return;
        const double sv = sat_of(max(kr, max(kg, kb)), min(kr, min(kg, kb)));
        double tp = hue_exact(kr, kg, kb, k255) + off;
        tp = tp > 360 ? tp - 360 : (tp < 0 ? tp + 360 : tp);
        th += tp;
        ts += sv;
        tv += v_of(max(kr, max(kg, kb)), k255);
        tn += 1.0;
    };
    // units of kPartUnit pixels (4 groups of 4 per thread, loads issued together)
    constexpr int kUnit = 16 * kPartThreads;
    static_assert(kChunk % kUnit == 0, "units tile a chunk");
    const long umax = cut > 0 ? (long)(cut - 1) / kUnit : -1;
    for (long u = blockIdx.y; u <= umax; u += gridDim.y) {
        if (chunk_hist[(u * kUnit / kChunk) * tl + g] == 0) continue;   // block-uniform
        const long end = std::min<long>((u + 1) * kUnit, (long)cut);
        unsigned w[4][3];
        bool okg[4];
#pragma unroll
        for (int st = 0; st < 4; st++) {
            const long p0 = u * kUnit + 4L * tid + 4L * kPartThreads * st;
            okg[st] = p0 + 3 < full_end;
            load_group<kAligned>(ip, p0, okg[st], w[st]);
        }
#pragma unroll
        for (int st = 0; st < 4; st++) {
            const long p0 = u * kUnit + 4L * tid + 4L * kPartThreads * st;
            if (p0 >= end) continue;
            if (okg[st]) {
#pragma unroll
                for (int i = 0; i < 4; i++)
                    if (p0 + i < end) add(px_byte(w[st], 3 * i), px_byte(w[st], 3 * i + 1), px_byte(w[st], 3 * i + 2));
            } else {
                for (long p = p0; p < p0 + 4 && p < end && p < npix; p++) add(ip[3 * p], ip[3 * p + 1], ip[3 * p + 2]);
            }
        }
    }
    if (blockIdx.y == 0 && tid == 0 && r.partial && r.dangle && r.last != 0xFFFFFFFFu && r.last >= cut) {
        const long p = r.last;                               // the dangling node's pixel
        add(ip[3 * p], ip[3 * p + 1], ip[3 * p + 2]);
    }
    const double v4[4] = {wave_sum(th), wave_sum(ts), wave_sum(tv), wave_sum(tn)};
    if (lane_id() == 0)
        for (int f = 0; f < 4; f++) red[(tid >> 6) * 4 + f] = v4[f];
    __syncthreads();
    if (tid < 4) {
        double a = 0.0;
        for (int q = 0; q < kPartThreads / 64; q++) a += red[q * 4 + tid];
        double* out = reinterpret_cast<double*>(reinterpret_cast<char*>(out0) + img * c_stride);
        if (a != 0.0) atomicAdd(&out[4 * r.slot + tid], a);
    }
}

// The same sums with one walk per image instead of one per (image, group):
// block (image, split) classifies every pixel of the image's prefix up to the
// largest cutoff once, and a pixel of one of the image's partial groups
// (LDS group -> entry map) before that group's cutoff adds its terms to the
// entry's LDS accumulators (rare: a few hundred pixels per group).  With many
// partial groups whose cutoffs lie deep in the image (fine grids: 36/4/5 on
// uniform images keeps ~1000 of ~16k pixels per group, cutoffs ~700k pixels
// in) this reads and classifies the prefix once instead of once per group.
constexpr int kPartImgMax = 64;                   // partial groups per image (else k_partial_sums_b)
struct PartImgLds {
    static constexpr int se = K1Lds::qn;          // first entry, entry count
    static constexpr int acc = K1Lds::area;       // kPartImgMax x 4 doubles
    static constexpr int off = acc + 32 * kPartImgMax;
    static constexpr int cut = off + 8 * kPartImgMax;
    static constexpr int grp = cut + 4 * kPartImgMax;
    static constexpr int slot = grp + 4 * kPartImgMax;
    static constexpr int gent = slot + 4 * kPartImgMax;   // tl shorts
    static size_t bytes(int tl) { return (size_t)gent + 2 * (size_t)tl; }
};

template <bool kAligned, bool kThr>
__global__ __launch_bounds__(kPartThreads) void k_partial_sums_img(
        const uint8_t* const* __restrict__ imgs, long npix, GridParams gp, FastCls fc,
        const ClassTables* __restrict__ tabs, const double* __restrict__ k255g, const int2* __restrict__ entries,
        int n_entries, const unsigned short* __restrict__ chunk_hist0, long h_stride,
        const GroupRule* __restrict__ rules0, const double* __restrict__ off0, long b_stride, double* out0,
        long c_stride) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const double* k255 = reinterpret_cast<const double*>(smem + K1Lds::k255);
    const ClsEnt* ent = reinterpret_cast<const ClsEnt*>(smem + K1Lds::ent);
    int* se = reinterpret_cast<int*>(smem + PartImgLds::se);
    double* acc = reinterpret_cast<double*>(smem + PartImgLds::acc);
    double* eoff = reinterpret_cast<double*>(smem + PartImgLds::off);
    unsigned* ecut = reinterpret_cast<unsigned*>(smem + PartImgLds::cut);
    int* egrp = reinterpret_cast<int*>(smem + PartImgLds::grp);
    int* eslot = reinterpret_cast<int*>(smem + PartImgLds::slot);
    short* gent = reinterpret_cast<short*>(smem + PartImgLds::gent);
    const signed char* si8 = tabs->si8;
    const int tid = threadIdx.x, img = blockIdx.x, tl = gp.tl;
    stage_tables(smem, k255g, tabs);
    if (tid < 2) se[tid] = 0;
    for (int g = tid; g < tl; g += kPartThreads) gent[g] = -1;
    __syncthreads();
    // this image's entries: a contiguous run of the image-major list
    for (int k = tid; k < n_entries; k += kPartThreads) {
        if (entries[k].x != img) continue;
        if (k == 0 || entries[k - 1].x != img) se[0] = k;
        atomicAdd(&se[1], 1);
    }
    __syncthreads();
    const int e0 = se[0], ne = se[1];
    if (ne == 0) return;                                     // block-uniform
    const uint8_t* ip = imgs[img];
    const GroupRule* rules =
            reinterpret_cast<const GroupRule*>(reinterpret_cast<const char*>(rules0) + img * b_stride);
    const double* offs = reinterpret_cast<const double*>(reinterpret_cast<const char*>(off0) + img * b_stride);
    const unsigned short* chunk_hist =
            reinterpret_cast<const unsigned short*>(reinterpret_cast<const char*>(chunk_hist0) + img * h_stride);
    for (int e = tid; e < ne; e += kPartThreads) {
        const int g = entries[e0 + e].y;
        const GroupRule r = rules[g];
        gent[g] = (short)e;
        egrp[e] = g;
        eslot[e] = r.slot;
        eoff[e] = offs[r.slot];
        ecut[e] = (r.partial && r.keep > 0) ? r.cutoff : 0u;
    }
    for (int i = tid; i < 4 * ne; i += kPartThreads) acc[i] = 0.0;
    __syncthreads();
    unsigned cmax = 0;
    for (int e = 0; e < ne; e++) cmax = max(cmax, ecut[e]);
    // calculate_avg_hsv's terms of one kept pixel into entry e
    auto put = [&](int e, int kr, int kg, int kb, double sv) {
        double tp = hue_exact(kr, kg, kb, k255) + eoff[e];
        tp = tp > 360 ? tp - 360 : (tp < 0 ? tp + 360 : tp);
        atomicAdd(&acc[4 * e + 0], tp);
        atomicAdd(&acc[4 * e + 1], sv);
        atomicAdd(&acc[4 * e + 2], v_of(max(kr, max(kg, kb)), k255));
        atomicAdd(&acc[4 * e + 3], 1.0);
    };
    // a pixel by its exact group (the deferred and the unaligned tail pixels)
    auto add = [&](long p, int kr, int kg, int kb) {
        double sv;
        const int g = exact_group_t<kThr>(kr, kg, kb, ent, si8, k255, gp, fc, sv);
        const int e = g >= 0 ? gent[g] : -1;
        if (e >= 0 && p < (long)ecut[e]) put(e, kr, kg, kb, sv);
    };
    // The walk classifies every pixel of the prefix to find the few of the
    // partial groups, so the common case is all integer work: the group from
    // classify_e (no saturation, no fp64); a pixel on a hue-bin edge (-2) is
    // resolved exactly only when one of its two candidate groups (hue bins hi
    // and hi - 1, gcol) is an entry, after the unit (a wave would otherwise run
    // the fp64 hue for a pixel of one of its lanes on most steps).
    const int svp = gp.sp * gp.vp;
    constexpr int kUnit = 16 * kPartThreads;
    const long full_end = npix & ~3L;
    const long umax = cmax > 0 ? (long)(cmax - 1) / kUnit : -1;
    const int lane = lane_id();
    // one unit: 16 pixels per thread (4 groups of 4, loaded together) and, in
    // lane l < ne, entry l's pixel count in the unit's chunk (the skip test)
    struct Unit {
        unsigned w[4][3];
        bool ok[4];
        unsigned hv;
    };
    // (unconditional loads, lanes >= ne reading entry ne - 1's count: a load
    // whose value is selected at once, or that sits under a branch, is
    // waited for right there; process() tests lane < ne)
    auto fetch = [&](long u, Unit& x) {
        const long ub = u * kUnit;
        x.hv = chunk_hist[(ub / kChunk) * tl + egrp[lane < ne ? lane : ne - 1]];
#pragma unroll
        for (int st = 0; st < 4; st++) {
            const long p0 = ub + 4L * tid + 4L * kPartThreads * st;
            x.ok[st] = p0 + 3 < full_end;
            load_group<kAligned>(ip, p0, x.ok[st], x.w[st]);
        }
    };
    auto process = [&](long u, const Unit& x) {
        // wave-uniform: skip a unit no entry needs (past its cutoff or none of
        // its group's pixels in the chunk)
        const long ub = u * kUnit;
        if (__ballot(lane < ne && ub < (long)ecut[lane] && x.hv != 0u) == 0ull) return;
        const long end = std::min<long>(ub + kUnit, (long)cmax);
        unsigned cand = 0;                                   // bit 4 st + i: resolve exactly
#pragma unroll
        for (int st = 0; st < 4; st++) {
            const long p0 = ub + 4L * tid + 4L * kPartThreads * st;
            if (p0 >= end) continue;
            if (x.ok[st]) {
                int g[4], gc[4];
#pragma unroll
                for (int i = 0; i < 4; i++) {
                    const int kr = px_byte(x.w[st], 3 * i), kg = px_byte(x.w[st], 3 * i + 1),
                              kb = px_byte(x.w[st], 3 * i + 2);
                    int hN, hD;
                    g[i] = classify_e<kThr>(kr, kg, kb, ent[max(kr, max(kg, kb))], si8, gp, fc, hN, hD, gc[i]);
                }
                // both candidates' entries read unconditionally (a select, not a
                // branch per pixel that waits on its own LDS read): the group
                // itself, or an edge pixel's colour groups gcol and one bin below
                int ea[4], eb[4];
#pragma unroll
                for (int i = 0; i < 4; i++) {
                    const int ga = g[i] >= 0 ? g[i] : gc[i];
                    const int gb = (g[i] < 0 && gc[i] >= svp) ? gc[i] - svp : ga;
                    ea[i] = gent[ga];
                    eb[i] = gent[gb];
                }
#pragma unroll
                for (int i = 0; i < 4; i++)
                    cand |= (unsigned)((ea[i] >= 0 || eb[i] >= 0) && p0 + i < end) << (4 * st + i);
            } else {
                for (long p = p0; p < p0 + 4 && p < end && p < npix; p++) add(p, ip[3 * p], ip[3 * p + 1], ip[3 * p + 2]);
            }
        }
        while (cand) {
            const int bt = __ffs(cand) - 1;
            cand &= cand - 1;
            const int st = bt >> 2, i = bt & 3;
            // the group's words and the pixel's bytes by selects: a register
            // array indexed by a runtime st or byte put the unit in scratch
            // memory (round 6), and a kernel with scratch stalls the other
            // lane's concurrent kernels
            unsigned ws[3];
#pragma unroll
            for (int k = 0; k < 3; k++)
                ws[k] = sel4_opaque(st, x.w[0][k], x.w[1][k], x.w[2][k], x.w[3][k]);
            const unsigned pw = px_word(ws[0], ws[1], ws[2], i);
            add(ub + 4L * tid + 4L * kPartThreads * st + i, (int)(pw & 255u), (int)((pw >> 8) & 255u),
                (int)((pw >> 16) & 255u));
        }
    };
    // two units in flight: the next one's loads are issued before this one's
    // classification (the walk is otherwise bound by the load latency)
    // (a unit past the walk's end is fetched as its last unit, and not used)
    const long gy = gridDim.y;
    Unit cur;
    if ((long)blockIdx.y <= umax) fetch(blockIdx.y, cur);
#pragma unroll 1
    for (long u = blockIdx.y; u <= umax; u += gy) {
        Unit nxt;
        fetch(u + gy <= umax ? u + gy : umax, nxt);
        process(u, cur);
        cur = nxt;
    }
    if (blockIdx.y == 0)
        for (int e = tid; e < ne; e += kPartThreads) {
            const GroupRule r = rules[egrp[e]];
            if (r.partial && r.dangle && r.last != 0xFFFFFFFFu && r.last >= ecut[e]) {
                const long p = r.last;                       // the dangling node's pixel
                const int kr = ip[3 * p], kg = ip[3 * p + 1], kb = ip[3 * p + 2];
                double sv;
                if (exact_group_t<kThr>(kr, kg, kb, ent, si8, k255, gp, fc, sv) == egrp[e]) put(e, kr, kg, kb, sv);
            }
        }
    __syncthreads();
    double* out = reinterpret_cast<double*>(reinterpret_cast<char*>(out0) + img * c_stride);
    for (int i = tid; i < 4 * ne; i += kPartThreads) {
        const double a = acc[i];
        if (a != 0.0) atomicAdd(&out[4 * eslot[i >> 2] + (i & 3)], a);
    }
}

// K1 for downsample_rate > 1: HSV over the decimated pixels only (gathered).
template <bool kThr>
__global__ __launch_bounds__(kThreads) void k_hsv_ds(const uint8_t* __restrict__ img, long npix,
                                                     int width, int ds, int nw, GridParams gp, FastCls fc,
                                                     const ClassTables* __restrict__ tabs,
                                                     const double* __restrict__ k255g, PaletteDev out) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const double* k255 = reinterpret_cast<const double*>(smem + K1Lds::k255);
    const ClsEnt* ent = reinterpret_cast<const ClsEnt*>(smem + K1Lds::ent);
    const signed char* si8 = tabs->si8;
    double* red = reinterpret_cast<double*>(smem + K1Lds::red);
    unsigned* lh = reinterpret_cast<unsigned*>(smem + K1Lds::area);
    const int tid = threadIdx.x;
    stage_tables(smem, k255g, tabs);
    for (int i = tid; i < gp.tl; i += kThreads) lh[i] = 0;
    __syncthreads();
    const long base = (long)blockIdx.x * kChunk;
    const long end = min(base + (long)kChunk, npix);
    double ssum = 0.0;
    for (long j = base + tid; j < end; j += kThreads) {
        const long p = src_pixel(j, width, ds, nw);
        const int kr = img[3 * p], kg = img[3 * p + 1], kb = img[3 * p + 2];
        double sv;
        int g = classify<kThr>(kr, kg, kb, ent, si8, gp, fc, sv);
        ssum += sv;
        if (g == -2) g = exact_group(kr, kg, kb, k255, gp);
        hist_add(lh, g);
    }
    const double sw = wave_sum(ssum);
    if (lane_id() == 0) red[tid >> 6] = sw;
    __syncthreads();
    if (tid == 0) {
        double t = 0.0;
        for (int q = 0; q < kThreads / 64; q++) t += red[q];
        out.s_part[blockIdx.x] = t;
    }
    for (int i = tid; i < gp.tl; i += kThreads) {
        const unsigned c = lh[i];
        out.chunk_hist[(long)blockIdx.x * gp.tl + i] = (unsigned short)c;
        if (c) atomicAdd(&out.hist[i], c);
    }
}

// RGB integer moments over the full image (used when ds > 1).
__global__ __launch_bounds__(kThreads) void k_stats(const uint8_t* __restrict__ img, long nbytes,
                                                    unsigned long long* __restrict__ sums) {
    __shared__ unsigned long long red[4][8];
    unsigned long long m[6] = {0, 0, 0, 0, 0, 0};
    const long stride = (long)gridDim.x * kThreads;
    for (long p = (long)blockIdx.x * kThreads + threadIdx.x; 3 * p < nbytes; p += stride) {
        const unsigned kr = img[3 * p], kg = img[3 * p + 1], kb = img[3 * p + 2];
        m[0] += kr; m[1] += kg; m[2] += kb;
        m[3] += kr * kr; m[4] += kg * kg; m[5] += kb * kb;
    }
#pragma unroll
    for (int c = 0; c < 6; c++) m[c] = wave_sum(m[c]);
    if (lane_id() == 0)
        for (int c = 0; c < 6; c++) red[threadIdx.x >> 6][c] = m[c];
    __syncthreads();
    if (threadIdx.x < 6) {
        unsigned long long t = 0;
        for (int q = 0; q < kThreads / 64; q++) t += red[q][threadIdx.x];
        atomicAdd(&sums[threadIdx.x], t);
    }
}

// Block-wide exclusive scan of one int per thread; returns the block total.
__device__ int block_excl_scan(int x, int& excl, int* scratch) {
    const int lane = lane_id(), w = threadIdx.x >> 6;
    int incl = x;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(incl, o, 64);
        if (lane >= o) incl += y;
    }
    if (lane == 63) scratch[w] = incl;
    __syncthreads();
    int wpre = 0, tot = 0;
    for (int q = 0; q < kThreads / 64; q++) {
        if (q < w) wpre += scratch[q];
        tot += scratch[q];
    }
    __syncthreads();
    excl = wpre + incl - x;
    return tot;
}

// Kcut: one block per group whose keep rule needs raster positions: the index
// of its keep-th pixel (the tie path of group_irregular_pixels appends pixels
// in raster order until the parent's tail node is full,
// src/color_quantization.c:414-450) and of its last pixel (the dangling node).
__global__ __launch_bounds__(kThreads) void k_cutoffs(const uint8_t* __restrict__ img, long npix,
                                                      int width, int ds, int nw, GridParams gp,
                                                      const unsigned short* __restrict__ chunk_hist,
                                                      int nchunks, GroupRule* rules,
                                                      const int* __restrict__ search,
                                                      const double* __restrict__ k255g) {
    __shared__ double k255[256];
    __shared__ int scratch[kThreads / 64];
    __shared__ int s_chunk, s_rank, s_last_chunk, s_found;
    __shared__ unsigned s_idx;
    const int tid = threadIdx.x;
    k255[tid] = k255g[tid];
    const int g = search[blockIdx.x];
    const int keep = rules[g].keep;
    const int want_cut = rules[g].partial && keep > 0;
    const int want_last = rules[g].partial && rules[g].dangle;
    if (tid == 0) { s_chunk = -1; s_last_chunk = -1; }
    __syncthreads();
    // pass over chunk counts: chunk holding the keep-th pixel, and last non-empty chunk
    int carry = 0;
    for (int c0 = 0; c0 < nchunks; c0 += kThreads) {
        const int c = c0 + tid;
        const int cnt = c < nchunks ? (int)chunk_hist[(long)c * gp.tl + g] : 0;
        int excl;
        const int tot = block_excl_scan(cnt, excl, scratch);
        if (want_cut && cnt > 0 && carry + excl < keep && keep <= carry + excl + cnt) {
            s_chunk = c;
            s_rank = keep - (carry + excl);   // 1-based rank inside the chunk
        }
        if (cnt > 0) atomicMax(&s_last_chunk, c);
        carry += tot;
        __syncthreads();
    }
    for (int pass = 0; pass < 2; pass++) {
        const int c = pass == 0 ? (want_cut ? s_chunk : -1) : (want_last ? s_last_chunk : -1);
        if (c < 0) continue;   // uniform across the block
        const long base = (long)c * kChunk, end = min(base + (long)kChunk, npix);
        int rank = s_rank;
        if (tid == 0) { s_found = 0; s_idx = 0; }
        __syncthreads();
        for (long p0 = base + 4L * tid, r0 = base; r0 < end; p0 += 4L * kThreads, r0 += 4L * kThreads) {
            int hits = 0;
            unsigned hit_mask = 0;
#pragma unroll
            for (int i = 0; i < 4; i++) {
                const long j = p0 + i;
                if (j < end) {
                    const long p = src_pixel(j, width, ds, nw);
                    double h, s, v;
                    rgb2hsv(k255[img[3 * p]], k255[img[3 * p + 1]], k255[img[3 * p + 2]], h, s, v);
                    if (group_of(gp, h, s, v) == g) { hits++; hit_mask |= 1u << i; }
                }
            }
            if (pass == 0) {
                int excl;
                const int tot = block_excl_scan(hits, excl, scratch);
                if (excl < rank && rank <= excl + hits) {
                    int want = rank - excl;   // 1-based within this thread's 4 pixels
                    for (int i = 0; i < 4; i++)
                        if (hit_mask & (1u << i)) {
                            if (--want == 0) { s_idx = (unsigned)(p0 + i); s_found = 1; }
                        }
                }
                rank -= tot;
                __syncthreads();
                if (s_found) break;
            } else if (hit_mask) {
                atomicMax(&s_idx, (unsigned)(p0 + 31 - __builtin_clz(hit_mask)));
            }
        }
        __syncthreads();
        if (tid == 0) {
            if (pass == 0) rules[g].cutoff = s_idx + 1;
            else rules[g].last = s_idx;
        }
        __syncthreads();
    }
}

// K3: per-slot sums over the pixels each palette parent keeps
// (calculate_avg_hsv, src/color_quantization.c:529-558): wrap(h + off), s, v, n.
__global__ __launch_bounds__(kThreads) void k_palette_sums(const uint8_t* __restrict__ img, long npix,
                                                           int width, int ds, int nw, GridParams gp,
                                                           const GroupRule* __restrict__ rules_g,
                                                           const double* __restrict__ off_g, int nslots,
                                                           double* __restrict__ out,
                                                           const double* __restrict__ k255g,
                                                           int aligned) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    double* k255 = reinterpret_cast<double*>(smem);                       // 256
    double* acc = k255 + 256;                                              // nslots*4
    double* off = acc + 4 * nslots;                                        // nslots
    GroupRule* rules = reinterpret_cast<GroupRule*>(off + nslots);         // tl
    const int tid = threadIdx.x;
    k255[tid] = k255g[tid];
    for (int i = tid; i < 4 * nslots; i += kThreads) acc[i] = 0.0;
    for (int i = tid; i < nslots; i += kThreads) off[i] = off_g[i];
    for (int i = tid; i < gp.tl; i += kThreads) rules[i] = rules_g[i];
    __syncthreads();
    const long base = (long)blockIdx.x * kChunk;
    const long end = min(base + (long)kChunk, npix);
    for (long p0 = base + 4L * tid; p0 < end; p0 += 4L * kThreads) {
        unsigned k[12];
        int nv;
        if (ds <= 1) {
            load4(img, p0, end, aligned != 0, k, nv);
        } else {
            nv = 0;
            for (int i = 0; i < 4; i++) {
                if (p0 + i < end) {
                    const long p = src_pixel(p0 + i, width, ds, nw);
                    k[3 * i] = img[3 * p]; k[3 * i + 1] = img[3 * p + 1]; k[3 * i + 2] = img[3 * p + 2];
                    nv++;
                } else {
                    k[3 * i] = k[3 * i + 1] = k[3 * i + 2] = 0;
                }
            }
        }
#pragma unroll
        for (int i = 0; i < 4; i++) {
            double h, s, v;
            rgb2hsv(k255[k[3 * i]], k255[k[3 * i + 1]], k255[k[3 * i + 2]], h, s, v);
            const int g = group_of(gp, h, s, v);
            const GroupRule& R = rules[g];
            const unsigned idx = (unsigned)(p0 + i);
            const bool kept = i < nv && R.slot >= 0 &&
                              (!R.partial || idx < R.cutoff || (R.dangle && idx == R.last));
            const int slot = kept ? R.slot : -1;
            double tp = 0.0;
            if (kept) {
                tp = h + off[slot];
                if (tp > 360) tp -= 360;
                else if (tp < 0) tp += 360;
            }
            const int s0 = __builtin_amdgcn_readfirstlane(slot);
            const unsigned long long active = __ballot(1);
            if (__all(slot == s0)) {
                if (s0 >= 0) {
                    const double th = wave_sum(tp), ts = wave_sum(s), tv = wave_sum(v);
                    if (lane_id() == 0) {
                        atomicAdd(&acc[4 * s0 + 0], th);
                        atomicAdd(&acc[4 * s0 + 1], ts);
                        atomicAdd(&acc[4 * s0 + 2], tv);
                        atomicAdd(&acc[4 * s0 + 3], (double)__popcll(active));
                    }
                }
            } else if (slot >= 0) {
                atomicAdd(&acc[4 * slot + 0], tp);
                atomicAdd(&acc[4 * slot + 1], s);
                atomicAdd(&acc[4 * slot + 2], v);
                atomicAdd(&acc[4 * slot + 3], 1.0);
            }
        }
    }
    __syncthreads();
    for (int i = tid; i < 4 * nslots; i += kThreads) {
        const double a = acc[i];
        if (a != 0.0) atomicAdd(&out[i], a);
    }
}

// Per-pixel group id through the production classifier (classify, exact
// fallback) and exact HSV: validation of the device arithmetic.
template <bool kThr>
__global__ void k_debug_hsv(const uint8_t* __restrict__ img, long n, GridParams gp, FastCls fc,
                            const ClassTables* __restrict__ tabs, const double* __restrict__ k255,
                            int* __restrict__ gid, double* __restrict__ hsv) {
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
        const int kr = img[3 * i], kg = img[3 * i + 1], kb = img[3 * i + 2];
        double sv;
        int g = classify<kThr>(kr, kg, kb, tabs->ent, tabs->si8, gp, fc, sv);
        if (g == -2) g = exact_group(kr, kg, kb, k255, gp);
        gid[i] = g;
        if (hsv) {
            double h, s, v;
            rgb2hsv(k255[kr], k255[kg], k255[kb], h, s, v);
            hsv[3 * i] = h;
            hsv[3 * i + 1] = s;
            hsv[3 * i + 2] = v;
        }
    }
}

__global__ void k_fill_uniform(uint8_t* __restrict__ dst, size_t n, unsigned long long seed) {
    const size_t nw = (n + 7) / 8;
    for (size_t w = (size_t)blockIdx.x * blockDim.x + threadIdx.x; w < nw;
         w += (size_t)gridDim.x * blockDim.x) {
        unsigned long long z = seed + (w + 1) * 0x9E3779B97F4A7C15ull;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        z = z ^ (z >> 31);
        if (8 * w + 8 <= n) {
            reinterpret_cast<unsigned long long*>(dst)[w] = z;   // dst is 8-B aligned
        } else {
            for (size_t b = 8 * w; b < n; b++) dst[b] = (uint8_t)(z >> (8 * (b - 8 * w)));
        }
    }
}

}  // namespace

int g_ablate = 0;   // timing experiments only (phd_debug_time_kernel)

int num_cus() {
    static int n = 0;
    if (!n) {
        int dev = 0;
        hipDeviceProp_t p;
        n = (hipGetDevice(&dev) == hipSuccess && hipGetDeviceProperties(&p, dev) == hipSuccess)
                ? p.multiProcessorCount : 256;
    }
    return n;
}

static inline long hsv_pixels(int height, int width, int ds, int* nw) {
    const int hh = ds > 1 ? height / ds : height, ww = ds > 1 ? width / ds : width;
    *nw = ww;
    return (long)(short)hh * (short)ww;   // rgb2hsv's short dimensions, image_processing.c:378-383
}

int env_ablate() {
    static const int a = phd_knob("PHD_ABLATE") ? atoi(phd_knob("PHD_ABLATE")) : 0;   // timing runs only
    return a;
}

// lane-private copies of K1's chunk counts: as many as fit 40 KiB (<= 32)
int k1_cshift(int tl) {
    int c = 5;
    while (c > 0 && 2 * (size_t)(tl + 1) * (4u << c) > 40 * 1024) c--;
    return c;
}

// ... and of K3's slot sums (28 B per copy): <= 96 KiB
int k3_cshift(int max_slots) {
    int c = 5;
    while (c > 0 && ((size_t)max_slots + 1) * (28u << c) > 96 * 1024) c--;
    return c;
}

// LDS of K1: tables, chunk-count copies, run counts and (fused) the sums and
// cell-count copies.
size_t k1_lds_bytes(const GridParams& gp, int cshift, bool sums) {
    const size_t C = (size_t)1 << cshift;
    return (size_t)K1Lds::area + k1_count_bytes(gp.tl, cshift) +
           (sums ? 8 * 3 * ((size_t)gp.tl + 1) * C + 4 * ((size_t)HueCells::count(gp) + 1) * C : 0);
}

// Fused K1's copies: the most (<= 16) with two blocks per CU, else one copy in
// one block per CU, else -1 (the palette takes the two-pass path).
int k1_fused_cshift(const GridParams& gp) {
    for (int c = 4; c >= 0; c--)
        if (k1_lds_bytes(gp, c, true) <= 78 * 1024) return c;
    return k1_lds_bytes(gp, 0, true) <= 150 * 1024 ? 0 : -1;
}

bool fused_palette_ok(const GridParams& gp) { return k1_fused_cshift(gp) >= 0; }

size_t hsv_stats_lds(const GridParams& gp, bool hist, bool sums) {
    if (sums) return k1_lds_bytes(gp, k1_fused_cshift(gp), true);
    return hist ? k1_lds_bytes(gp, k1_cshift(gp.tl), false) : (size_t)K1Lds::red + 1024;
}

hipError_t launch_hsv_stats_batch(const uint8_t* const* d_imgs, int n, int height, int width,
                                  const GridParams& gp, const FastCls& fc, const ClassTables* tabs,
                                  const PaletteDev& out0, long a_stride, long h_stride, int nchunks,
                                  const double* k255, bool hist, bool sums, bool aligned, hipStream_t st) {
    const long npix = (long)height * width;
    const long nitems = (long)n * nchunks;
    if (sums && (!hist || !fused_palette_ok(gp))) return hipErrorInvalidValue;
    // the fused palette pass over word-aligned images: the table K1 (k1.hip)
    if (sums && aligned && fc.k1t_cshift >= 0)
        return launch_k1t_batch(d_imgs, n, height, width, gp, tabs, out0, a_stride, h_stride, nchunks, k255,
                                fc.k1t_cshift, fc.k1t_cshift2, st);
    // the statistics-only pass over word-aligned images: the lean kernel (stats.hip)
    if (!hist && aligned)
        return launch_rgb_stats_batch(d_imgs, n, height, width, out0, a_stride, nchunks, st);
    const size_t lds = hsv_stats_lds(gp, hist, sums);
    const int cshift = sums ? k1_fused_cshift(gp) : k1_cshift(gp.tl);
    const void* kfn = nullptr;
#define PHD_K1_FN(H, S, A, T) (const void*)k_hsv_stats<H, S, A, T>
    if (sums)
        kfn = fc.use_thr ? (aligned ? PHD_K1_FN(true, true, true, true) : PHD_K1_FN(true, true, false, true))
                         : (aligned ? PHD_K1_FN(true, true, true, false) : PHD_K1_FN(true, true, false, false));
    else if (hist)
        kfn = fc.use_thr ? (aligned ? PHD_K1_FN(true, false, true, true) : PHD_K1_FN(true, false, false, true))
                         : (aligned ? PHD_K1_FN(true, false, true, false) : PHD_K1_FN(true, false, false, false));
    else
        kfn = PHD_K1_FN(false, false, false, true);       // (unaligned: aligned images took k_rgb_stats)
#undef PHD_K1_FN
    // persistent blocks: as many as are resident at once
    (void)hipFuncSetAttribute(kfn, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    int per_cu = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kfn, kPalThreads, lds) != hipSuccess || per_cu < 1)
        per_cu = 1;
    const int grid = (int)std::min<long>(nitems, (long)per_cu * num_cus());
    void* args[] = {(void*)&d_imgs, (void*)&npix, (void*)&nchunks, (void*)&nitems, (void*)&gp, (void*)&fc,
                    (void*)&tabs, (void*)&k255, (void*)&out0, (void*)&a_stride, (void*)&h_stride,
                    (void*)&cshift, nullptr};
    const int abl = env_ablate();
    args[12] = (void*)&abl;
    return hipLaunchKernel(kfn, dim3(grid), dim3(kPalThreads), args, lds, st);
}

hipError_t launch_hsv_ds(const uint8_t* img, int height, int width, int ds, const GridParams& gp,
                         const FastCls& fc, const ClassTables* tabs, const PaletteDev& out, int nchunks,
                         const double* k255, hipStream_t st) {
    int nw;
    const long n = hsv_pixels(height, width, ds, &nw);
    const size_t lds = K1Lds::area + sizeof(unsigned) * ((gp.tl + 3) & ~3);
    if (fc.use_thr)
        phd_launch(k_hsv_ds<true>, dim3(nchunks), dim3(kThreads), lds, st, img, n, width, ds, nw, gp, fc,
                           tabs, k255, out);
    else
        phd_launch(k_hsv_ds<false>, dim3(nchunks), dim3(kThreads), lds, st, img, n, width, ds, nw, gp, fc,
                           tabs, k255, out);
    const long nbytes = 3L * height * width;
    const int blocks = (int)std::min<long>(2048, (nbytes / 3 + kThreads - 1) / kThreads);
    phd_launch(k_stats, dim3(blocks), dim3(kThreads), 0, st, img, nbytes, out.sums);
    return hipGetLastError();
}

hipError_t launch_palette_cutoffs(const uint8_t* img, int height, int width, int ds,
                                  const GridParams& gp, const unsigned short* chunk_hist, int nchunks,
                                  GroupRule* rules, const int* search_groups, int n_search,
                                  const double* k255, hipStream_t st) {
    if (n_search <= 0) return hipSuccess;
    int nw;
    const long n = hsv_pixels(height, width, ds, &nw);
    phd_launch(k_cutoffs, dim3(n_search), dim3(kThreads), 0, st, img, n, width, ds, nw, gp,
                       chunk_hist, nchunks, rules, search_groups, k255);
    return hipGetLastError();
}

hipError_t launch_palette_sums(const uint8_t* img, int height, int width, int ds, const GridParams& gp,
                               const GroupRule* rules, const double* slot_off, int nslots, double* out,
                               const double* k255, hipStream_t st) {
    int nw;
    const long n = hsv_pixels(height, width, ds, &nw);
    const int nchunks = (int)((n + kChunk - 1) / kChunk);
    const size_t lds = sizeof(double) * (256 + 5 * (size_t)nslots) + sizeof(GroupRule) * gp.tl;
    const int aligned = (reinterpret_cast<uintptr_t>(img) & 3) == 0;
    phd_launch(k_palette_sums, dim3(nchunks), dim3(kThreads), lds, st, img, n, width, ds, nw,
                       gp, rules, slot_off, nslots, out, k255, aligned);
    return hipGetLastError();
}

size_t palette_sums_b_lds(int tl, int max_slots) {
    return (size_t)K1Lds::area + 16 * ((size_t)tl + 1) + 8 * ((size_t)max_slots + 1) +
           ((size_t)max_slots + 1) * (28u << k3_cshift(max_slots));
}

hipError_t launch_cutoffs_batch(const uint8_t* const* d_imgs, const uint8_t* const* h_imgs, int n, int height,
                                int width, const GridParams& gp, const FastCls& fc, const ClassTables* tabs,
                                const double* k255, const int2* entries, int n_entries,
                                const unsigned short* chunk_hist0, long h_stride, GroupRule* rules0,
                                long b_stride, hipStream_t st) {
    if (n_entries <= 0) return hipSuccess;
    const long npix = (long)height * width;
    const int nchunks = (int)((npix + kChunk - 1) / kChunk);
    bool aligned = true;
    for (int i = 0; i < n; i++) aligned = aligned && (reinterpret_cast<uintptr_t>(h_imgs[i]) & 3) == 0;
    const size_t lds = K1Lds::area;
#define PHD_KCUT_LAUNCH(A, T)                                                                               \
    do {                                                                                                    \
        /* a function-local static initialiser runs once, thread-safe */                                  \
        static const bool attr_ = ((void)hipFuncSetAttribute((const void*)k_cutoffs_b<A, T>,                       \
                                                       hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024), \
                                   true);                                                                   \
        (void)attr_;                                                                                        \
        phd_launch((k_cutoffs_b<A, T>), dim3(n_entries), dim3(kK1Threads), lds, st, d_imgs, npix,        \
                           nchunks, gp, fc, tabs, k255, entries, chunk_hist0, h_stride, rules0, b_stride);  \
    } while (0)
    if (fc.use_thr) {
        if (aligned) PHD_KCUT_LAUNCH(true, true);
        else PHD_KCUT_LAUNCH(false, true);
    } else {
        if (aligned) PHD_KCUT_LAUNCH(true, false);
        else PHD_KCUT_LAUNCH(false, false);
    }
#undef PHD_KCUT_LAUNCH
    return hipGetLastError();
}

hipError_t launch_palette_sums_batch(const uint8_t* const* d_imgs, const uint8_t* const* h_imgs, int n,
                                     int height, int width, const GridParams& gp, const FastCls& fc,
                                     const ClassTables* tabs, const double* k255, const GroupRule* rules0,
                                     const double* off0, long b_stride, const int* nslots_img, int max_slots,
                                     double* out0, long c_stride, hipStream_t st) {
    const long npix = (long)height * width;
    const int nchunks = (int)((npix + kChunk - 1) / kChunk);
    const long nitems = (long)n * nchunks;
    bool aligned = true;
    for (int i = 0; i < n; i++) aligned = aligned && (reinterpret_cast<uintptr_t>(h_imgs[i]) & 3) == 0;
    const size_t lds = palette_sums_b_lds(gp.tl, max_slots);
    int per_cu = 0;
    const void* kfn = fc.use_thr ? (aligned ? (const void*)k_palette_sums_b<true, true>
                                            : (const void*)k_palette_sums_b<false, true>)
                                 : (aligned ? (const void*)k_palette_sums_b<true, false>
                                            : (const void*)k_palette_sums_b<false, false>);
    (void)hipFuncSetAttribute(kfn, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kfn, kK3Threads, lds) != hipSuccess || per_cu < 1)
        per_cu = 1;
    const int grid = (int)std::min<long>(nitems, (long)per_cu * num_cus());
#define PHD_K3_LAUNCH(A, T)                                                                                 \
    do {                                                                                                    \
        static const bool attr_ = ((void)hipFuncSetAttribute((const void*)k_palette_sums_b<A, T>,                  \
                                                       hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024), \
                                   true);                                                                   \
        (void)attr_;                                                                                        \
        phd_launch((k_palette_sums_b<A, T>), dim3(grid), dim3(kK3Threads), lds, st, d_imgs, npix,        \
                           nchunks, nitems, gp, fc, tabs, k255, rules0, off0, b_stride, nslots_img,         \
                           max_slots, out0, c_stride, k3_cshift(max_slots), env_ablate());                  \
    } while (0)
    if (fc.use_thr) {
        if (aligned) PHD_K3_LAUNCH(true, true);
        else PHD_K3_LAUNCH(false, true);
    } else {
        if (aligned) PHD_K3_LAUNCH(true, false);
        else PHD_K3_LAUNCH(false, false);
    }
#undef PHD_K3_LAUNCH
    return hipGetLastError();
}

hipError_t launch_partial_sums_batch(const uint8_t* const* d_imgs, const uint8_t* const* h_imgs, int n,
                                     int height, int width, const GridParams& gp, const FastCls& fc,
                                     const ClassTables* tabs, const double* k255, const int2* entries,
                                     int n_entries, const unsigned short* chunk_hist0, long h_stride,
                                     const GroupRule* rules0, const double* off0, long b_stride, double* out0,
                                     long c_stride, int max_per_image, hipStream_t st) {
    if (n_entries <= 0) return hipSuccess;
    const long npix = (long)height * width;
    bool aligned = true;
    for (int i = 0; i < n; i++) aligned = aligned && (reinterpret_cast<uintptr_t>(h_imgs[i]) & 3) == 0;
    if (max_per_image <= kPartImgMax && max_per_image > 1) {
        const size_t lds = PartImgLds::bytes(gp.tl);
        // (grid.y 16: same step time; 4: 4 % slower, the walks then outlast the FFTs they share the CUs with)
        // split each image's walk over ~4096 blocks in all, at least 64 per
        // image (grid.y 256 measured the same as 64 in config 5's 64-image
        // groups; a single image's walk over 64 blocks outlasts its FFTs)
        const dim3 grid(n, std::max(64, std::min(1024, 4096 / std::max(n, 1))));
#define PHD_PI_LAUNCH(A, T)                                                                                     \
    phd_launch((k_partial_sums_img<A, T>), grid, dim3(kPartThreads), lds, st, d_imgs, npix, gp, fc, tabs, \
                       k255, entries, n_entries, chunk_hist0, h_stride, rules0, off0, b_stride, out0, c_stride)
        if (fc.use_thr) {
            if (aligned) PHD_PI_LAUNCH(true, true);
            else PHD_PI_LAUNCH(false, true);
        } else {
            if (aligned) PHD_PI_LAUNCH(true, false);
            else PHD_PI_LAUNCH(false, false);
        }
#undef PHD_PI_LAUNCH
        return hipGetLastError();
    }
    const size_t lds = K1Lds::qn;
    // ~4096 blocks in all, at least 32 per entry (a single entry's walk over 32
    // blocks took 61 us at 4000x3000, past the image's FFTs)
    const dim3 grid(n_entries, std::max(32, std::min(1024, 4096 / std::max(n_entries, 1))));
    if (fc.use_thr) {
        if (aligned)
            phd_launch((k_partial_sums_b<true, true>), grid, dim3(kPartThreads), lds, st, d_imgs, npix, gp, fc,
                               tabs, k255, entries, chunk_hist0, h_stride, rules0, off0, b_stride, out0, c_stride);
        else
            phd_launch((k_partial_sums_b<false, true>), grid, dim3(kPartThreads), lds, st, d_imgs, npix, gp,
                               fc, tabs, k255, entries, chunk_hist0, h_stride, rules0, off0, b_stride, out0, c_stride);
    } else {
        if (aligned)
            phd_launch((k_partial_sums_b<true, false>), grid, dim3(kPartThreads), lds, st, d_imgs, npix, gp,
                               fc, tabs, k255, entries, chunk_hist0, h_stride, rules0, off0, b_stride, out0, c_stride);
        else
            phd_launch((k_partial_sums_b<false, false>), grid, dim3(kPartThreads), lds, st, d_imgs, npix, gp,
                               fc, tabs, k255, entries, chunk_hist0, h_stride, rules0, off0, b_stride, out0, c_stride);
    }
    return hipGetLastError();
}

hipError_t launch_debug_hsv(const uint8_t* img, long n, const GridParams& gp, const FastCls& fc,
                            const ClassTables* tabs, const double* k255, int* gid, double* hsv, hipStream_t st) {
    if (fc.use_thr)
        phd_launch(k_debug_hsv<true>, dim3(2048), dim3(256), 0, st, img, n, gp, fc, tabs, k255, gid, hsv);
    else
        phd_launch(k_debug_hsv<false>, dim3(2048), dim3(256), 0, st, img, n, gp, fc, tabs, k255, gid, hsv);
    return hipGetLastError();
}

hipError_t launch_fill_uniform(uint8_t* dst, size_t n, uint64_t seed, hipStream_t st) {
    const size_t nw = (n + 7) / 8;
    const int blocks = (int)std::min<size_t>(4096, (nw + 255) / 256);
    phd_launch(k_fill_uniform, dim3(blocks > 0 ? blocks : 1), dim3(256), 0, st, dst, n,
                       (unsigned long long)seed);
    return hipGetLastError();
}

}  // namespace phd
