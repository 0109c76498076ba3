// fft_engine.h -- compile-time mixed-radix Stockham FFT building blocks (fp64
// complex, gfx950).
//
// A transform of length N is a list of radices R0 R1 ... (N = product).  Pass p
// (NS = R0*...*R(p-1)) is the Stockham autosort step: butterfly b in [0, N/R)
// reads x[b + r*N/R], r < R, multiplies input r by W_{NS*R}^{(b mod NS)*r},
// runs an R-point DFT and writes output k to (b/NS)*NS*R + b mod NS + k*NS.
// Every size, radix, round count and division is a compile-time constant, so
// the index arithmetic folds to shifts and multiply-highs.
//
// R-point DFTs: 2, 3, 4, 5 and 8 are written out.  Any other R = A*B is a
// small four-step in registers (A-point DFTs over n2, constant twiddles
// W_R^{n2*k1} from fft_consts.h with +-1 and +-i folded, then B-point DFTs).
//
// LDS bank conflicts.  A b128 write group is 8 lanes.  Pass 0 writes with a
// lane stride of R0 complex, so an odd R0 makes those writes conflict-free.
// Later passes write runs of NS consecutive elements.  Reads are consecutive.
// The plans therefore start with an odd radix (tools/ fft plan notes,
// DESIGN.md).
#pragma once

#include <hip/hip_runtime.h>

#include <utility>

#include "fft_consts.h"

namespace phd {
namespace fe {

__device__ __forceinline__ double2 cadd(double2 a, double2 b) { return make_double2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ double2 csub(double2 a, double2 b) { return make_double2(a.x - b.x, a.y - b.y); }
__device__ __forceinline__ double2 cmul(double2 a, double2 b) {
    return make_double2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x);
}
__device__ __forceinline__ double2 mul_negi(double2 a) { return make_double2(a.y, -a.x); }   // a * (-i)
__device__ __forceinline__ double2 mul_posi(double2 a) { return make_double2(-a.y, a.x); }   // a * (+i)

// compile-time for: f(std::integral_constant<int, I>) for I in [0, N)
template <typename F, int... Is>
__device__ __forceinline__ void sfor_impl(F&& f, std::integer_sequence<int, Is...>) {
    (f(std::integral_constant<int, Is>{}), ...);
}
template <int N, typename F>
__device__ __forceinline__ void sfor(F&& f) {
    sfor_impl(f, std::make_integer_sequence<int, N>{});
}

// a * W_R^M, W_R = exp(-2 pi i / R), with the trivial cases folded
template <int R, int M>
__device__ __forceinline__ double2 twm(double2 a) {
    constexpr int m = M % R;
    constexpr double h = 0.70710678118654752440;
    if constexpr (m == 0) return a;
    else if constexpr (2 * m == R) return make_double2(-a.x, -a.y);
    else if constexpr (4 * m == R) return mul_negi(a);
    else if constexpr (4 * m == 3 * R) return mul_posi(a);
    else if constexpr (8 * m == R) return make_double2(h * (a.x + a.y), h * (a.y - a.x));
    else if constexpr (8 * m == 3 * R) return make_double2(h * (a.y - a.x), -h * (a.x + a.y));
    else if constexpr (8 * m == 5 * R) return make_double2(-h * (a.x + a.y), h * (a.x - a.y));
    else if constexpr (8 * m == 7 * R) return make_double2(h * (a.x - a.y), h * (a.x + a.y));
    else {
        constexpr double c = TwTab<R>::c[m], s = TwTab<R>::s[m];   // W = c - i s
        return make_double2(a.x * c + a.y * s, a.y * c - a.x * s);
    }
}

template <int R>
__device__ __forceinline__ void dft(double2 (&v)[R]);

template <>
__device__ __forceinline__ void dft<1>(double2 (&)[1]) {}

template <>
__device__ __forceinline__ void dft<2>(double2 (&v)[2]) {
    const double2 a = v[0], b = v[1];
    v[0] = cadd(a, b);
    v[1] = csub(a, b);
}

template <>
__device__ __forceinline__ void dft<3>(double2 (&v)[3]) {
    constexpr double s1 = 0.86602540378443864676;   // sin(2 pi / 3)
    const double2 t = cadd(v[1], v[2]);
    const double2 d = mul_negi(make_double2(s1 * (v[1].x - v[2].x), s1 * (v[1].y - v[2].y)));
    const double2 m = make_double2(v[0].x - 0.5 * t.x, v[0].y - 0.5 * t.y);
    v[0] = cadd(v[0], t);
    v[1] = cadd(m, d);
    v[2] = csub(m, d);
}

template <>
__device__ __forceinline__ void dft<4>(double2 (&v)[4]) {
    const double2 t0 = cadd(v[0], v[2]), t1 = csub(v[0], v[2]);
    const double2 t2 = cadd(v[1], v[3]), t3 = mul_negi(csub(v[1], v[3]));
    v[0] = cadd(t0, t2);
    v[2] = csub(t0, t2);
    v[1] = cadd(t1, t3);
    v[3] = csub(t1, t3);
}

template <>
__device__ __forceinline__ void dft<5>(double2 (&v)[5]) {
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
__device__ __forceinline__ void dft<8>(double2 (&v)[8]) {
    double2 e[4] = {v[0], v[2], v[4], v[6]}, o[4] = {v[1], v[3], v[5], v[7]};
    dft<4>(e);
    dft<4>(o);
    o[1] = twm<8, 1>(o[1]);
    o[2] = mul_negi(o[2]);
    o[3] = twm<8, 3>(o[3]);
#pragma unroll
    for (int k = 0; k < 4; k++) {
        v[k] = cadd(e[k], o[k]);
        v[k + 4] = csub(e[k], o[k]);
    }
}

// first factor of a composite radix
constexpr int split_of(int r) { return (r % 4 == 0 && r > 8) ? 4 : (r % 5 == 0 ? 5 : (r % 3 == 0 ? 3 : 2)); }

// R = A*B: x[B n1 + n2] -> A-point DFTs over n1 (per n2) -> * W_R^{n2 k1}
// -> B-point DFTs over n2 (per k1) -> X[k1 + A k2]
template <int A, int B>
__device__ __forceinline__ void dft_ab(double2 (&v)[A * B]) {
    constexpr int R = A * B;
    double2 y[B][A];
    sfor<B>([&](auto n2_) {
        constexpr int n2 = decltype(n2_)::value;
        sfor<A>([&](auto n1_) {
            constexpr int n1 = decltype(n1_)::value;
            y[n2][n1] = v[B * n1 + n2];
        });
        dft<A>(y[n2]);
        sfor<A>([&](auto k1_) {
            constexpr int k1 = decltype(k1_)::value;
            y[n2][k1] = twm<R, n2 * k1>(y[n2][k1]);
        });
    });
    sfor<A>([&](auto k1_) {
        constexpr int k1 = decltype(k1_)::value;
        double2 z[B];
        sfor<B>([&](auto n2_) { z[decltype(n2_)::value] = y[decltype(n2_)::value][k1]; });
        dft<B>(z);
        sfor<B>([&](auto k2_) { v[k1 + A * decltype(k2_)::value] = z[decltype(k2_)::value]; });
    });
}

template <int R>
__device__ __forceinline__ void dft(double2 (&v)[R]) {
    dft_ab<split_of(R), R / split_of(R)>(v);
}

// v[r] *= w^r for r = 1..R-1.  The powers come from four interleaved chains
// (w^r = w^(r-4) w^4), so the longest dependent run of complex products is
// about R/4 + 2 instead of R - 1 (latency: the passes run at 2-4 waves per SIMD).
template <int R>
__device__ __forceinline__ void twiddle_powers(double2 (&v)[R], const double2 w) {
    if constexpr (R <= 4) {
        double2 wr = w;
        v[1] = cmul(v[1], w);
#pragma unroll
        for (int r = 2; r < R; r++) {
            wr = cmul(wr, w);
            v[r] = cmul(v[r], wr);
        }
    } else {
        double2 p[4];
        p[1] = w;
        p[2] = cmul(w, w);
        p[3] = cmul(p[2], w);
        p[0] = cmul(p[2], p[2]);                                  // w^4
        const double2 w4 = p[0];
#pragma unroll
        for (int r = 1; r < R; r++) {
            if (r > 4) p[r & 3] = cmul(p[r & 3], w4);
            v[r] = cmul(v[r], p[r & 3]);
        }
    }
}

// ---- one Stockham pass --------------------------------------------------------
// CLAMP: the lanes past the last butterfly of a partial round load and compute
// the last butterfly's values (unused, never stored), so v is defined on every
// path and carries no phi copies (the column plans: 252 -> 243 VGPRs at 3000
// rows, no spills at 4000 / 6000); without it they skip the round (the row
// plans keep fewer live registers that way: 114 against 128 + spills at 4000).
// jm = 0 multiplies by tw[0] = 1 exactly instead of branching around it.
template <int N, int T, int R, int NS, bool CLAMP = false>
struct Pass {
    static constexpr int NB = N / R;                 // butterflies
    static constexpr int ROUNDS = (NB + T - 1) / T;  // per thread
    static constexpr bool FULL = NB % T == 0;
    static_assert(N % R == 0, "radix must divide N");

    __device__ static __forceinline__ bool active(int b) { return FULL || b < NB; }
    __device__ static __forceinline__ int bfly(int tid, int q) {
        return (FULL || !CLAMP) ? tid + q * T : min(tid + q * T, NB - 1);
    }

    __device__ static __forceinline__ void load(const double2* buf, double2 (&v)[ROUNDS][R], int tid) {
#pragma unroll
        for (int q = 0; q < ROUNDS; q++) {
            const int b = bfly(tid, q);
            if (CLAMP || active(b)) {
#pragma unroll
                for (int r = 0; r < R; r++) v[q][r] = buf[b + r * NB];
            }
        }
    }
    // twiddles (tw[jm] = W_{NS*R}^jm for jm < NS) and the R-point DFTs
    __device__ static __forceinline__ void compute(double2 (&v)[ROUNDS][R], const double2* tw, int tid) {
#pragma unroll
        for (int q = 0; q < ROUNDS; q++) {
            const int b = bfly(tid, q);
            if (CLAMP || active(b)) {
                if constexpr (NS > 1) twiddle_powers<R>(v[q], tw[b % NS]);
                dft<R>(v[q]);
            }
        }
    }
    __device__ static __forceinline__ void store(double2* buf, const double2 (&v)[ROUNDS][R], int tid) {
#pragma unroll
        for (int q = 0; q < ROUNDS; q++) {
            const int b = tid + q * T;
            if (active(b)) {
                const int jh = b / NS, jm = b - jh * NS;
                const int base = jh * NS * R + jm;
#pragma unroll
                for (int k = 0; k < R; k++) buf[base + k * NS] = v[q][k];
            }
        }
    }
};

// ---- plans --------------------------------------------------------------------
template <int... Rs>
struct Radices {
    static constexpr int count = sizeof...(Rs);
    static constexpr int product = (1 * ... * Rs);
};

// Twiddle entries a plan needs: sum over passes p >= 1 of NS_p.
template <int NS, int R, int... Rest>
constexpr int tw_entries() {
    if constexpr (sizeof...(Rest) == 0) return NS > 1 ? NS : 0;
    else return (NS > 1 ? NS : 0) + tw_entries<NS * R, Rest...>();
}


// All passes in LDS (natural order in and out).  buf: N elements; tw: the
// plan's concatenated per-pass tables.  Ends with a barrier.
template <int N, int T, int NS, int R, int... Rest>
__device__ __forceinline__ void fft_lds(double2* buf, const double2* tw, int tid) {
    using P = Pass<N, T, R, NS>;
    double2 v[P::ROUNDS][R];
    P::load(buf, v, tid);
    P::compute(v, tw, tid);
    __syncthreads();
    P::store(buf, v, tid);
    __syncthreads();
    if constexpr (sizeof...(Rest) > 0) fft_lds<N, T, NS * R, Rest...>(buf, tw + (NS > 1 ? NS : 0), tid);
}

// (PHD_COL_CLAMP=0: an A/B build with the column plans' passes unclamped)
#ifndef PHD_COL_CLAMP
#define PHD_COL_CLAMP 1
#endif
// Every pass but the last in LDS; Last::load/compute are left to the caller
// (whose outputs, element b + k*N/R_last of round q, stay in registers).
// Clamped passes (the column plans).
template <int N, int T, int NS, int R, int... Rest>
struct Plan {
    using Last = typename Plan<N, T, NS * R, Rest...>::Last;
    static constexpr int last_tw_offset = (NS > 1 ? NS : 0) + Plan<N, T, NS * R, Rest...>::last_tw_offset;
    __device__ static __forceinline__ void all_but_last(double2* buf, const double2* tw, int tid) {
        using P = Pass<N, T, R, NS, PHD_COL_CLAMP != 0>;
        double2 v[P::ROUNDS][R];
        P::load(buf, v, tid);
        P::compute(v, tw, tid);
        __syncthreads();
        P::store(buf, v, tid);
        __syncthreads();
        Plan<N, T, NS * R, Rest...>::all_but_last(buf, tw + (NS > 1 ? NS : 0), tid);
    }
};
template <int N, int T, int NS, int R>
struct Plan<N, T, NS, R> {
    using Last = Pass<N, T, R, NS, PHD_COL_CLAMP != 0>;
    static constexpr int last_tw_offset = 0;
    __device__ static __forceinline__ void all_but_last(double2*, const double2*, int) {}
};

}  // namespace fe
}  // namespace phd
