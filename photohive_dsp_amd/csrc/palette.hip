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
constexpr int kQueue = kChunk;               // deferred exact-path pixels (u16 offsets): never overflows
constexpr int kK1Threads = 1024;             // K1 block: 16 waves over one kChunk
struct K1Lds {
    static constexpr int k255 = 0;           // 256 doubles
    static constexpr int rinv = 2048;        // 256 doubles
    static constexpr int vcol = 4096;        // 256 int16
    static constexpr int vgray = 4608;       // 256 int16
    static constexpr int red = 5120;         // 16 waves x 8 x u64
    static constexpr int qn = 6144;          // int (+pad)
    static constexpr int queue = 6160;       // kQueue x u16 (pixel offset in the chunk)
    static constexpr int hist = 6160 + 2 * kQueue;   // tl x u32
};

__device__ __forceinline__ void stage_tables(unsigned char* smem, const double* __restrict__ k255g,
                                             const ClassTables* __restrict__ tabs) {
    const int tid = threadIdx.x;
    if (tid >= 256) return;
    reinterpret_cast<double*>(smem + K1Lds::k255)[tid] = k255g[tid];
    reinterpret_cast<double*>(smem + K1Lds::rinv)[tid] = tabs->rinv[tid];
    reinterpret_cast<short*>(smem + K1Lds::vcol)[tid] = tabs->vcol[tid];
    reinterpret_cast<short*>(smem + K1Lds::vgray)[tid] = tabs->vgray[tid];
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

// Raw form of load4: the three little-endian words holding pixels p0..p0+3
// (bytes past `end` are zero); unpack with px_byte.
__device__ __forceinline__ int load4_raw(const uint8_t* __restrict__ img, long p0, long end, bool aligned,
                                         unsigned (&w)[3]) {
    if (aligned && p0 + 3 < end) {
        const unsigned* q = reinterpret_cast<const unsigned*>(img + 3 * p0);
        w[0] = q[0];
        w[1] = q[1];
        w[2] = q[2];
        return 4;
    }
    w[0] = w[1] = w[2] = 0;
    int nv = 0;
    for (int b = 0; b < 12; b++)
        if (p0 + b / 3 < end) {
            w[b >> 2] |= (unsigned)img[3 * p0 + b] << (8 * (b & 3));
            nv = b / 3 + 1;
        }
    return nv;
}

__device__ __forceinline__ int px_byte(const unsigned (&w)[3], int b) { return (w[b >> 2] >> (8 * (b & 3))) & 255; }

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

// K1 for downsample_rate == 1: stats and HSV over the same pixels.
// Persistent blocks (2 per CU) walk the image's kChunk-pixel chunks; per chunk
// the group histogram is built in LDS and written out (the cutoff search walks
// these per-chunk counts); channel moments and sum(s) stay in registers and are
// reduced once per block.  Pixels classify through fast_group; the few near a
// bin edge are queued in LDS and classified exactly after the chunk's stream,
// so waves stay convergent.  Next-chunk loads are issued before the current
// chunk's flush.
__global__ __launch_bounds__(kK1Threads, 8) void k_hsv_stats(const uint8_t* __restrict__ img, long npix,
                                                        int nchunks, GridParams gp, FastCls fc,
                                                        const ClassTables* __restrict__ tabs,
                                                        const double* __restrict__ k255g,
                                                        int aligned, PaletteDev out, int ablate) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const double* k255 = reinterpret_cast<const double*>(smem + K1Lds::k255);
    const double* rinv = reinterpret_cast<const double*>(smem + K1Lds::rinv);
    const short* vcol = reinterpret_cast<const short*>(smem + K1Lds::vcol);
    const short* vgray = reinterpret_cast<const short*>(smem + K1Lds::vgray);
    unsigned long long* red = reinterpret_cast<unsigned long long*>(smem + K1Lds::red);
    int* qn = reinterpret_cast<int*>(smem + K1Lds::qn);
    unsigned short* queue = reinterpret_cast<unsigned short*>(smem + K1Lds::queue);
    unsigned* lh = reinterpret_cast<unsigned*>(smem + K1Lds::hist);
    const int tid = threadIdx.x;
    stage_tables(smem, k255g, tabs);
    unsigned long long mom[6] = {0, 0, 0, 0, 0, 0};
    double ssum = 0.0;
    constexpr int kSteps = kChunk / (4 * kK1Threads);
    unsigned w[kSteps][3];
    int nv[kSteps];
    auto issue = [&](int c) {
        const long base = (long)c * kChunk, end = min(base + (long)kChunk, npix);
#pragma unroll
        for (int it = 0; it < kSteps; it++)
            nv[it] = load4_raw(img, base + 4L * tid + 4L * kK1Threads * it, end, aligned != 0, w[it]);
    };
    int c = blockIdx.x;
    if (c < nchunks) issue(c);
    for (; c < nchunks; c += gridDim.x) {
        for (int i = tid; i < gp.tl; i += kK1Threads) lh[i] = 0;
        if (tid == 0) *qn = 0;
        __syncthreads();
        const long base = (long)c * kChunk;
        unsigned sr = 0, sg = 0, sb = 0, qr = 0, qg = 0, qb = 0;
#pragma unroll
        for (int it = 0; it < kSteps; it++) {
            const long p0 = base + 4L * tid + 4L * kK1Threads * it;
#pragma unroll
            for (int i = 0; i < 4; i++) {
                const int kr = px_byte(w[it], 3 * i), kg = px_byte(w[it], 3 * i + 1), kb = px_byte(w[it], 3 * i + 2);
                const bool valid = i < nv[it];
                if (valid) {
                    sr += kr; sg += kg; sb += kb;
                    qr += kr * kr; qg += kg * kg; qb += kb * kb;
                }
                if (!(ablate & 32)) ssum += valid ? sat_of(kr, kg, kb, rinv) : 0.0;
                int g = !valid ? -1 : (ablate & 8) ? (kr & 7) : fast_group(kr, kg, kb, vcol, vgray, gp, fc);
                if (g == -2) {                // near a bin edge: classify exactly after the stream
                    queue[atomicAdd(qn, 1)] = (unsigned short)(p0 + i - base);
                    g = -1;
                }
                if (!(ablate & 16)) hist_add(lh, g);
                else if (g >= 0) ssum += g;
            }
        }
        mom[0] += sr; mom[1] += sg; mom[2] += sb; mom[3] += qr; mom[4] += qg; mom[5] += qb;
        if (c + (int)gridDim.x < nchunks) issue(c + gridDim.x);   // prefetch the next chunk
        __syncthreads();
        const int nq = *qn;
        for (int q = tid; q < nq; q += kK1Threads) {
            const long p = base + queue[q];
            atomicAdd(&lh[exact_group(img[3 * p], img[3 * p + 1], img[3 * p + 2], k255, gp)], 1u);
        }
        __syncthreads();
        for (int i = tid; i < gp.tl; i += kK1Threads) {
            const unsigned n = lh[i];
            out.chunk_hist[(long)c * gp.tl + i] = (unsigned short)n;
            if (n && !(ablate & 128)) atomicAdd(&out.hist[i], n);
        }
        __syncthreads();
    }
    // block reduction of the integer moments (exact) and of sum(s), once
    const int wv = tid >> 6;
#pragma unroll
    for (int k = 0; k < 6; k++) mom[k] = wave_sum(mom[k]);
    const double sw = wave_sum(ssum);
    if (lane_id() == 0) {
#pragma unroll
        for (int k = 0; k < 6; k++) red[wv * 8 + k] = mom[k];
        reinterpret_cast<double*>(red)[wv * 8 + 6] = sw;
    }
    __syncthreads();
    if (tid < 6) {
        unsigned long long t = 0;
        for (int q = 0; q < kK1Threads / 64; q++) t += red[q * 8 + tid];
        if (!(ablate & 128)) atomicAdd(&out.sums[tid], t);
    } else if (tid == 6) {
        double t = 0.0;
        for (int q = 0; q < kK1Threads / 64; q++) t += reinterpret_cast<double*>(red)[q * 8 + 6];
        out.s_part[blockIdx.x] = t;        // one partial per block (host sums them)
    }
}

// K1 for downsample_rate > 1: HSV over the decimated pixels only (gathered).
__global__ __launch_bounds__(kThreads) void k_hsv_ds(const uint8_t* __restrict__ img, long npix,
                                                     int width, int ds, int nw, GridParams gp, FastCls fc,
                                                     const ClassTables* __restrict__ tabs,
                                                     const double* __restrict__ k255g, PaletteDev out) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const double* k255 = reinterpret_cast<const double*>(smem + K1Lds::k255);
    const double* rinv = reinterpret_cast<const double*>(smem + K1Lds::rinv);
    const short* vcol = reinterpret_cast<const short*>(smem + K1Lds::vcol);
    const short* vgray = reinterpret_cast<const short*>(smem + K1Lds::vgray);
    double* red = reinterpret_cast<double*>(smem + K1Lds::red);
    unsigned* lh = reinterpret_cast<unsigned*>(smem + K1Lds::hist);
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
        ssum += sat_of(kr, kg, kb, rinv);
        int g = fast_group(kr, kg, kb, vcol, vgray, gp, fc);
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

// Per-pixel group id through the production classifier (fast_group, exact
// fallback) and exact HSV: validation of the device arithmetic.
__global__ void k_debug_hsv(const uint8_t* __restrict__ img, long n, GridParams gp, FastCls fc,
                            const ClassTables* __restrict__ tabs, const double* __restrict__ k255,
                            int* __restrict__ gid, double* __restrict__ hsv) {
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
        const int kr = img[3 * i], kg = img[3 * i + 1], kb = img[3 * i + 2];
        int g = fast_group(kr, kg, kb, tabs->vcol, tabs->vgray, gp, fc);
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

hipError_t launch_hsv_stats(const uint8_t* img, int height, int width, int ds, const GridParams& gp,
                            const FastCls& fc, const ClassTables* tabs, const PaletteDev& out, int nchunks,
                            const double* k255, hipStream_t st) {
    int nw;
    const long n = hsv_pixels(height, width, ds, &nw);
    const size_t lds = K1Lds::hist + sizeof(unsigned) * ((gp.tl + 3) & ~3);
    if (ds <= 1) {
        const int aligned = (reinterpret_cast<uintptr_t>(img) & 3) == 0;
        const int grid = std::min(nchunks, 2 * num_cus());
        hipLaunchKernelGGL(k_hsv_stats, dim3(grid), dim3(kK1Threads), lds, st, img, n, nchunks, gp, fc, tabs,
                           k255, aligned, out, g_ablate);
    } else {
        hipLaunchKernelGGL(k_hsv_ds, dim3(nchunks), dim3(kThreads), lds, st, img, n, width, ds, nw, gp, fc,
                           tabs, k255, out);
        const long nbytes = 3L * height * width;
        const int blocks = (int)std::min<long>(2048, (nbytes / 3 + kThreads - 1) / kThreads);
        hipLaunchKernelGGL(k_stats, dim3(blocks), dim3(kThreads), 0, st, img, nbytes, out.sums);
    }
    return hipGetLastError();
}

hipError_t launch_palette_cutoffs(const uint8_t* img, int height, int width, int ds,
                                  const GridParams& gp, const unsigned short* chunk_hist, int nchunks,
                                  GroupRule* rules, const int* search_groups, int n_search,
                                  const double* k255, hipStream_t st) {
    if (n_search <= 0) return hipSuccess;
    int nw;
    const long n = hsv_pixels(height, width, ds, &nw);
    hipLaunchKernelGGL(k_cutoffs, dim3(n_search), dim3(kThreads), 0, st, img, n, width, ds, nw, gp,
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
    hipLaunchKernelGGL(k_palette_sums, dim3(nchunks), dim3(kThreads), lds, st, img, n, width, ds, nw,
                       gp, rules, slot_off, nslots, out, k255, aligned);
    return hipGetLastError();
}

hipError_t launch_debug_hsv(const uint8_t* img, long n, const GridParams& gp, const FastCls& fc,
                            const ClassTables* tabs, const double* k255, int* gid, double* hsv, hipStream_t st) {
    hipLaunchKernelGGL(k_debug_hsv, dim3(2048), dim3(256), 0, st, img, n, gp, fc, tabs, k255, gid, hsv);
    return hipGetLastError();
}

hipError_t launch_fill_uniform(uint8_t* dst, size_t n, uint64_t seed, hipStream_t st) {
    const size_t nw = (n + 7) / 8;
    const int blocks = (int)std::min<size_t>(4096, (nw + 255) / 256);
    hipLaunchKernelGGL(k_fill_uniform, dim3(blocks > 0 ? blocks : 1), dim3(256), 0, st, dst, n,
                       (unsigned long long)seed);
    return hipGetLastError();
}

}  // namespace phd
