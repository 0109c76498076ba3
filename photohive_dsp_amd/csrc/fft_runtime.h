// fft_runtime.h -- runtime-plan mixed-radix Stockham FFT in LDS (fp64 complex).
//
// Shared by the fused image passes (fft.hip) and the global-memory batched
// transforms (fft_global.hip).  A block transforms `nseq` sequences of length
// plan.n stored back to back in LDS; at most 8 elements per thread.
// Twiddles come from a host-built table tw[t] = exp(-2 pi i t/n) (long-double
// accurate) and two small staged tables (e = 64*hi + lo).
#pragma once

#include "fft_engine.h"
#include "phd_device.h"

namespace phd {
namespace rt {


__device__ __forceinline__ double2 cadd(double2 a, double2 b) { return make_double2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ double2 csub(double2 a, double2 b) { return make_double2(a.x - b.x, a.y - b.y); }
__device__ __forceinline__ double2 cmul(double2 a, double2 b) {
    return make_double2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x);
}
__device__ __forceinline__ double2 mul_negi(double2 a) { return make_double2(a.y, -a.x); }   // a * (-i)
__device__ __forceinline__ double2 cscale(double2 a, double s) { return make_double2(a.x * s, a.y * s); }

template <int R>
__device__ __forceinline__ void butterfly(double2 (&v)[R]);

template <>
__device__ __forceinline__ void butterfly<2>(double2 (&v)[2]) {
    const double2 a = v[0], b = v[1];
    v[0] = cadd(a, b);
    v[1] = csub(a, b);
}

template <>
__device__ __forceinline__ void butterfly<3>(double2 (&v)[3]) {
    constexpr double s1 = 0.86602540378443864676;   // sin(2 pi / 3)
    const double2 t = cadd(v[1], v[2]);
    const double2 d = mul_negi(cscale(csub(v[1], v[2]), s1));   // -i s1 (v1 - v2)
    const double2 m = make_double2(v[0].x - 0.5 * t.x, v[0].y - 0.5 * t.y);
    v[0] = cadd(v[0], t);
    v[1] = cadd(m, d);
    v[2] = csub(m, d);
}

template <>
__device__ __forceinline__ void butterfly<4>(double2 (&v)[4]) {
    const double2 t0 = cadd(v[0], v[2]), t1 = csub(v[0], v[2]);
    const double2 t2 = cadd(v[1], v[3]), t3 = mul_negi(csub(v[1], v[3]));
    v[0] = cadd(t0, t2);
    v[2] = csub(t0, t2);
    v[1] = cadd(t1, t3);
    v[3] = csub(t1, t3);
}

template <>
__device__ __forceinline__ void butterfly<5>(double2 (&v)[5]) {
    constexpr double c1 = 0.30901699437494742410;    // cos(2 pi / 5)
    constexpr double c2 = -0.80901699437494742410;   // cos(4 pi / 5)
    constexpr double s1 = 0.95105651629515357212;    // sin(2 pi / 5)
    constexpr double s2 = 0.58778525229247312917;    // sin(4 pi / 5)
    const double2 t1 = cadd(v[1], v[4]), t2 = cadd(v[2], v[3]);
    const double2 t3 = csub(v[1], v[4]), t4 = csub(v[2], v[3]);
    const double2 a1 = make_double2(v[0].x + c1 * t1.x + c2 * t2.x, v[0].y + c1 * t1.y + c2 * t2.y);
    const double2 a2 = make_double2(v[0].x + c2 * t1.x + c1 * t2.x, v[0].y + c2 * t1.y + c1 * t2.y);
    const double2 b1 = mul_negi(make_double2(s1 * t3.x + s2 * t4.x, s1 * t3.y + s2 * t4.y));
    const double2 b2 = mul_negi(make_double2(s2 * t3.x - s1 * t4.x, s2 * t3.y - s1 * t4.y));
    v[0] = cadd(v[0], cadd(t1, t2));
    v[1] = cadd(a1, b1);
    v[4] = csub(a1, b1);
    v[2] = cadd(a2, b2);
    v[3] = csub(a2, b2);
}

template <>
__device__ __forceinline__ void butterfly<8>(double2 (&v)[8]) {
    constexpr double h = 0.70710678118654752440;   // sqrt(1/2)
    double2 e[4] = {v[0], v[2], v[4], v[6]}, o[4] = {v[1], v[3], v[5], v[7]};
    butterfly<4>(e);
    butterfly<4>(o);
    // o[k] *= W8^k
    o[1] = make_double2(h * (o[1].x + o[1].y), h * (o[1].y - o[1].x));
    o[2] = mul_negi(o[2]);
    o[3] = make_double2(h * (o[3].y - o[3].x), -h * (o[3].x + o[3].y));
#pragma unroll
    for (int k = 0; k < 4; k++) {
        v[k] = cadd(e[k], o[k]);
        v[k + 4] = csub(e[k], o[k]);
    }
}

// Composite radices (fewer LDS passes for the image lengths of config 5:
// 1920 = 16 12 10, 1080 = 12 10 9): the compile-time engine's register
// four-step DFTs (fft_engine.h, constant twiddles from fft_consts.h).
template <int R>
constexpr bool kComposite = R == 6 || R == 9 || R == 10 || R == 12 || R == 16;
template <> __device__ __forceinline__ void butterfly<6>(double2 (&v)[6]) { fe::dft<6>(v); }
template <> __device__ __forceinline__ void butterfly<9>(double2 (&v)[9]) { fe::dft<9>(v); }
template <> __device__ __forceinline__ void butterfly<10>(double2 (&v)[10]) { fe::dft<10>(v); }
template <> __device__ __forceinline__ void butterfly<12>(double2 (&v)[12]) { fe::dft<12>(v); }
template <> __device__ __forceinline__ void butterfly<16>(double2 (&v)[16]) { fe::dft<16>(v); }

// a / d for 0 <= a < 2^23 through one float multiply and an exact correction
// (the float quotient is off by at most one at these magnitudes).
__device__ __forceinline__ int fdiv(int a, int d, float inv) {
    int q = (int)((float)a * inv);
    const int r = a - q * d;
    q += (r >= d) ? 1 : 0;
    q -= (r < 0) ? 1 : 0;
    return q;
}

// LDS pointers for the out-of-line passes: a generic pointer there compiles
// every LDS access to a flat instruction (slower issue, and it also counts
// against the vector-memory counter)
#if defined(__HIP_DEVICE_COMPILE__)
typedef __attribute__((address_space(3))) double2 lds_d2;
typedef const __attribute__((address_space(3))) double2 lds_cd2;
typedef const __attribute__((address_space(1))) double2 glb_cd2;
#else
typedef double2 lds_d2;            // (the host pass only parses these functions)
typedef const double2 lds_cd2;
typedef const double2 glb_cd2;
#endif

// W_n^e from the two LDS tables (e = 64*hi + lo).
__device__ __forceinline__ double2 twiddle(lds_cd2* lo, lds_cd2* hi, int e) {
    return cmul(hi[e >> 6], lo[e & 63]);
}

// One Stockham pass of radix R over `nseq` sequences of length n stored at
// buf + seq*n (Govindaraju et al.: read stride n/R, write expanded index
// (j/Ns)*Ns*R + j%Ns + r*Ns).  Every thread reads its butterflies' inputs to
// registers, applies w^r (w = W_n^{(j%Ns)*n/(Ns*R)}, powers by multiplication),
// runs the radix-R DFT, then -- after one barrier -- writes them back.
// CAP = elements per block the kernel instance supports (8 per thread).
template <int R, int T>
__device__ __noinline__ void stockham_pass(lds_d2* buf, int n, int nseq, int Ns, lds_cd2* lo, lds_cd2* hi) {
    constexpr int NB = (8 * T + R * T - 1) / (R * T);
    const int nb = n / R, total = nb * nseq, tstep = n / (Ns * R);
    const float inb = 1.0f / (float)nb, ins = 1.0f / (float)Ns;
    double2 v[NB][R];
    int dst[NB];
#pragma unroll
    for (int b = 0; b < NB; b++) {
        const int t = threadIdx.x + b * T;
        dst[b] = -1;
        if (t < total) {
            const int seq = nseq == 1 ? 0 : fdiv(t, nb, inb);
            const int j = t - seq * nb;
            lds_cd2* s = buf + seq * n;
#pragma unroll
            for (int r = 0; r < R; r++) v[b][r] = s[j + r * nb];
            const int jh = fdiv(j, Ns, ins), jm = j - jh * Ns;
            if (jm != 0) {
                const double2 w = twiddle(lo, hi, jm * tstep);
                if constexpr (kComposite<R>) {
                    fe::twiddle_powers<R>(v[b], w);          // four interleaved power chains
                } else {
                    double2 wr = w;
                    v[b][1] = cmul(v[b][1], w);
#pragma unroll
                    for (int r = 2; r < R; r++) {
                        wr = cmul(wr, w);
                        v[b][r] = cmul(v[b][r], wr);
                    }
                }
            }
            butterfly<R>(v[b]);
            dst[b] = seq * n + jh * Ns * R + jm;
        }
    }
    __syncthreads();
#pragma unroll
    for (int b = 0; b < NB; b++) {
        if (dst[b] >= 0) {
#pragma unroll
            for (int r = 0; r < R; r++) buf[dst[b] + r * Ns] = v[b][r];
        }
    }
    __syncthreads();
}

// Generic radix (any R, incl. a prime length itself): output-parallel direct DFT.
template <int T>
__device__ __noinline__ void generic_pass(lds_d2* buf, int n, int nseq, int Ns, int R,
                                          glb_cd2* __restrict__ tw) {
    constexpr int EG = 8;   // outputs per thread (nseq*n <= 8*T)
    const int nb = n / R, total = n * nseq, tstep = n / (Ns * R), nr = n / R;
    double2 out[EG];
    int dst[EG];
#pragma unroll
    for (int e = 0; e < EG; e++) {
        const int t = threadIdx.x + e * T;
        dst[e] = -1;
        if (t < total) {
            const int seq = t / n, rem = t - seq * n;
            const int j = rem / R, k = rem - j * R;       // butterfly j, output k
            lds_cd2* s = buf + seq * n;
            const int jm = j % Ns;
            const int step = (jm * tstep + k * nr) % n;   // twiddle exponent per input r (mod n)
            double2 acc = make_double2(0.0, 0.0);
            int ex = 0;
            for (int r = 0; r < R; r++) {
                acc = cadd(acc, cmul(s[j + r * nb], tw[ex]));
                ex += step;
                if (ex >= n) ex -= n;
            }
            out[e] = acc;
            dst[e] = seq * n + (j / Ns) * Ns * R + jm + k * Ns;
        }
    }
    __syncthreads();
#pragma unroll
    for (int e = 0; e < EG; e++)
        if (dst[e] >= 0) buf[dst[e]] = out[e];
    __syncthreads();
}

// MODE bits over the radices 2, 3, 4, 5, 8: 1 the composites, 2 any other
// radix (generic_pass).  A kernel instance holds only the passes its MODE
// needs (a 16-point pass takes ~150 VGPRs, the small radices ~90).
template <int T, int MODE>
__device__ void fft_lds(double2* buf_, int nseq, const FftPlan& plan, const double2* lo_, const double2* hi_) {
    lds_d2* buf = (lds_d2*)buf_;                 // (the kernels' extern __shared__ arrays)
    lds_cd2* lo = (lds_cd2*)lo_;
    lds_cd2* hi = (lds_cd2*)hi_;
    int Ns = 1;
    for (int p = 0; p < plan.npass; p++) {
        const int R = plan.radix[p];
        switch (R) {
            case 2: stockham_pass<2, T>(buf, plan.n, nseq, Ns, lo, hi); break;
            case 3: stockham_pass<3, T>(buf, plan.n, nseq, Ns, lo, hi); break;
            case 4: stockham_pass<4, T>(buf, plan.n, nseq, Ns, lo, hi); break;
            case 5: stockham_pass<5, T>(buf, plan.n, nseq, Ns, lo, hi); break;
            case 8: stockham_pass<8, T>(buf, plan.n, nseq, Ns, lo, hi); break;
            default:
                if constexpr ((MODE & 1) != 0) {
                    if (R == 6) { stockham_pass<6, T>(buf, plan.n, nseq, Ns, lo, hi); break; }
                    if (R == 9) { stockham_pass<9, T>(buf, plan.n, nseq, Ns, lo, hi); break; }
                    if (R == 10) { stockham_pass<10, T>(buf, plan.n, nseq, Ns, lo, hi); break; }
                    if (R == 12) { stockham_pass<12, T>(buf, plan.n, nseq, Ns, lo, hi); break; }
                    if (R == 16) { stockham_pass<16, T>(buf, plan.n, nseq, Ns, lo, hi); break; }
                }
                if constexpr ((MODE & 2) != 0)
                    generic_pass<T>(buf, plan.n, nseq, Ns, R, (glb_cd2*)plan.tw);
                break;
        }
        Ns *= R;
    }
}

// Stage the two twiddle tables in LDS at `tw` (64 + n_hi entries).
__device__ __forceinline__ void load_twiddles(double2* tw, const FftPlan& plan) {
    for (int i = threadIdx.x; i < 64 + plan.n_hi; i += blockDim.x)
        tw[i] = i < 64 ? plan.tw_lo[i] : plan.tw_hi[i - 64];
}

}  // namespace rt
}  // namespace phd
