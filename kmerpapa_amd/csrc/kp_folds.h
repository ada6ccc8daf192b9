// kp_folds.h -- cross-validation fold split on the host, bit-identical to the reference.
//
// The reference splits every k-mer's counts into folds with numpy's legacy
// RandomState.hypergeometric, colour by colour (src/kmerpapa/CV_tools.py sample :5-27,
// make_all_folds_contextD_patterns :30-62).  In Python that is one interpreter round trip
// per colour per fold (~1 s at 9-mers, the serial term of multi-GPU CV).  This is the same
// random stream in C++: numpy's MT19937 (legacy 53-bit doubles) and the legacy
// hypergeometric samplers (HYP for samples <= 10, HRUA otherwise, with numpy's loggam),
// restated from numpy's published algorithms (numpy/random/src/legacy/
// legacy-distributions.c, distributions.c; the legacy stream is frozen by numpy's policy).
// tests/test_folds_native.py pins it draw for draw against numpy itself.
//
// Compiled without FMA contraction (-ffp-contract=off) and with the system libm, like
// numpy's x86-64 build of these routines.
#pragma once
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#if !defined(__HIP_DEVICE_COMPILE__)
#include <immintrin.h>
#endif

#include "kp_logdata.h"

namespace kpf {

struct mt19937 {
    uint32_t key[624];
    int pos;

    void gen() {
        static const uint32_t UPPER = 0x80000000u, LOWER = 0x7fffffffu, MATRIX_A = 0x9908b0dfu;
        int i;
        uint32_t y;
        for (i = 0; i < 624 - 397; i++) {
            y = (key[i] & UPPER) | (key[i + 1] & LOWER);
            key[i] = key[i + 397] ^ (y >> 1) ^ (-(y & 1) & MATRIX_A);
        }
        for (; i < 624 - 1; i++) {
            y = (key[i] & UPPER) | (key[i + 1] & LOWER);
            key[i] = key[i + (397 - 624)] ^ (y >> 1) ^ (-(y & 1) & MATRIX_A);
        }
        y = (key[623] & UPPER) | (key[0] & LOWER);
        key[623] = key[396] ^ (y >> 1) ^ (-(y & 1) & MATRIX_A);
        pos = 0;
    }
    uint32_t next32() {
        if (pos >= 624) gen();
        uint32_t y = key[pos++];
        y ^= (y >> 11);
        y ^= (y << 7) & 0x9d2c5680u;
        y ^= (y << 15) & 0xefc60000u;
        y ^= (y >> 18);
        return y;
    }
    // legacy 53-bit double in [0, 1)
    double next_double() {
        const int32_t a = (int32_t)(next32() >> 5), b = (int32_t)(next32() >> 6);
        return (a * 67108864.0 + b) / 9007199254740992.0;
    }
};

inline double loggam(double x) {
    static const double a[10] = {8.333333333333333e-02, -2.777777777777778e-03, 7.936507936507937e-04,
                                 -5.952380952380952e-04, 8.417508417508418e-04, -1.917526917526918e-03,
                                 6.410256410256410e-03, -2.955065359477124e-02, 1.796443723688307e-01,
                                 -1.39243221690590e+00};
    int64_t k, n;
    if (x == 1.0 || x == 2.0) return 0.0;
    n = (x < 7.0) ? (int64_t)(7 - x) : 0;
    double x0 = x + n;
    const double x2 = (1.0 / x0) * (1.0 / x0);
    const double lg2pi = 1.8378770664093453e+00;
    double gl0 = a[9];
    for (k = 8; k >= 0; k--) {
        gl0 *= x2;
        gl0 += a[k];
    }
    double gl = gl0 / x0 + 0.5 * lg2pi + (x0 - 0.5) * log(x0) - x0;
    if (x < 7.0) {
        for (k = 1; k <= n; k++) {
            gl -= log(x0 - 1.0);
            x0 -= 1.0;
        }
    }
    return gl;
}

// loggam of whole numbers (every argument the sampler passes is one, >= 1), four at a time:
// the small ones -- a k-mer's count and the draws from it -- from a table of loggam's own
// values (bit-identical by construction, and it skips the up-to-seven logs loggam spends
// below 7); the large ones run loggam's own operations side by side (the same IEEE
// operations in the same order per argument, so the same bits, without one argument's
// 10-step polynomial waiting on the previous one's).
struct loggam_table {
    enum { N = 8192 };
    double v[N];
    loggam_table() {
        v[0] = 0.0;
        for (int i = 1; i < N; ++i) v[i] = loggam((double)i);
    }
};

inline const loggam_table &loggam_tab() {
    static const loggam_table t;
    return t;
}

#if !defined(__HIP_DEVICE_COMPILE__)
// loggam_sum4 with the four arguments' large-argument work in one 4-wide AVX2 + FMA
// register each: the same IEEE operations in the same order per lane (the polynomial's
// multiplies and adds unfused, as loggam is compiled; the divisions), and the C library's
// log restated (kp_libm.h kp_libm_log: glibc's __log_fma, its table path -- every argument
// here is >= 8) with its FMAs, so every lane's bits equal the scalar path's.  The split's
// critical path is this function: ~3 calls per colour, ~75 % of a fold's draw.
// 4 lanes of loggam's large-argument path (x0 = k, every k >= 8): the same IEEE operations
// in the same order per lane as the scalar loggam (the polynomial's multiplies and adds
// unfused, the divisions) and the C library's log restated (kp_libm.h kp_libm_log: glibc's
// __log_fma table path) with its FMAs, so each lane's bits equal the scalar path's
__attribute__((target("avx2,fma"))) inline __m256d loggam_big4(const __m256d X0) {
    static const double a[10] = {8.333333333333333e-02, -2.777777777777778e-03, 7.936507936507937e-04,
                                 -5.952380952380952e-04, 8.417508417508418e-04, -1.917526917526918e-03,
                                 6.410256410256410e-03, -2.955065359477124e-02, 1.796443723688307e-01,
                                 -1.39243221690590e+00};
    static const double tab[256] = KP_LOG_TAB;
    static const double A[5] = KP_LOG_POLY;
    const __m256d inv = _mm256_div_pd(_mm256_set1_pd(1.0), X0);
    const __m256d X2 = _mm256_mul_pd(inv, inv);
    __m256d G = _mm256_set1_pd(a[9]);
    for (int i = 8; i >= 0; --i) G = _mm256_add_pd(_mm256_mul_pd(G, X2), _mm256_set1_pd(a[i]));
    const __m256i ix = _mm256_castpd_si256(X0);
    const __m256i tmp = _mm256_sub_epi64(ix, _mm256_set1_epi64x(0x3fe6000000000000ll));
    const __m256i idx = _mm256_slli_epi64(_mm256_and_si256(_mm256_srli_epi64(tmp, 45), _mm256_set1_epi64x(127)), 1);
    const __m256i kk = _mm256_srli_epi64(tmp, 52);  // >= 2 for x0 >= 8: a logical shift is the arithmetic one
    const __m256i iz = _mm256_sub_epi64(ix, _mm256_and_si256(tmp, _mm256_set1_epi64x((long long)0xfff0000000000000ull)));
    const __m256d invc = _mm256_i64gather_pd(tab, idx, 8);
    const __m256d logc = _mm256_i64gather_pd(tab + 1, idx, 8);
    const __m256d two52 = _mm256_set1_pd(4503599627370496.0);  // (double)k = bits(2^52 + k) - 2^52, exact
    const __m256d kd = _mm256_sub_pd(_mm256_castsi256_pd(_mm256_or_si256(kk, _mm256_castpd_si256(two52))), two52);
    const __m256d z = _mm256_castsi256_pd(iz);
    const __m256d r = _mm256_fmadd_pd(z, invc, _mm256_set1_pd(-1.0));
    const __m256d w = _mm256_fmadd_pd(kd, _mm256_set1_pd(KP_LOG_LN2HI), logc);
    const __m256d hi = _mm256_add_pd(r, w);
    const __m256d lo = _mm256_fmadd_pd(kd, _mm256_set1_pd(KP_LOG_LN2LO), _mm256_add_pd(_mm256_sub_pd(w, hi), r));
    const __m256d r2 = _mm256_mul_pd(r, r);
    const __m256d t1 = _mm256_fmadd_pd(r, _mm256_set1_pd(A[2]), _mm256_set1_pd(A[1]));
    const __m256d r3 = _mm256_mul_pd(r, r2);
    const __m256d t2 = _mm256_fmadd_pd(r, _mm256_set1_pd(A[4]), _mm256_set1_pd(A[3]));
    const __m256d lo2 = _mm256_fmadd_pd(r2, _mm256_set1_pd(A[0]), lo);
    const __m256d poly = _mm256_fmadd_pd(t2, r2, t1);
    const __m256d L = _mm256_add_pd(_mm256_fmadd_pd(r3, poly, lo2), hi);
    // gl0 / x0 + 0.5 * lg2pi + (x0 - 0.5) * log(x0) - x0, left to right
    __m256d R = _mm256_add_pd(_mm256_div_pd(G, X0), _mm256_set1_pd(0.5 * 1.8378770664093453e+00));
    R = _mm256_add_pd(R, _mm256_mul_pd(_mm256_sub_pd(X0, _mm256_set1_pd(0.5)), L));
    return _mm256_sub_pd(R, X0);
}

// two independent loggam_sum4 sums at once (HRUA's d10 and its first candidate's term: the
// candidate needs only the random draws, not d10): two dependent chains side by side
__attribute__((target("avx2,fma"))) inline void loggam_sum4x2_avx2(const int64_t (&k)[8], const bool (&big)[8],
                                                                   double *s0, double *s1) {
    alignas(32) double x0[8];
    for (int j = 0; j < 8; ++j) x0[j] = big[j] ? (double)k[j] : 8.0;
    const __m256d R0 = loggam_big4(_mm256_load_pd(x0));
    const __m256d R1 = loggam_big4(_mm256_load_pd(x0 + 4));
    alignas(32) double r[8];
    _mm256_store_pd(r, R0);
    _mm256_store_pd(r + 4, R1);
    const loggam_table &t = loggam_tab();
    for (int j = 0; j < 8; ++j)
        if (!big[j]) r[j] = t.v[k[j]];
    *s0 = ((r[0] + r[1]) + r[2]) + r[3];
    *s1 = ((r[4] + r[5]) + r[6]) + r[7];
}

inline bool cpu_avx2_fma() {
    static const bool ok = __builtin_cpu_supports("avx2") && __builtin_cpu_supports("fma") && !getenv("KP_FOLDS_SCALAR");
    return ok;
}
#endif

inline double loggam_sum4(int64_t k0, int64_t k1, int64_t k2, int64_t k3) {
    const loggam_table &t = loggam_tab();

    static const double a[10] = {8.333333333333333e-02, -2.777777777777778e-03, 7.936507936507937e-04,
                                 -5.952380952380952e-04, 8.417508417508418e-04, -1.917526917526918e-03,
                                 6.410256410256410e-03, -2.955065359477124e-02, 1.796443723688307e-01,
                                 -1.39243221690590e+00};
    const int64_t k[4] = {k0, k1, k2, k3};
    double r[4], x0[4], gl0[4], x2[4];
    bool big[4];
    for (int j = 0; j < 4; ++j) {
        big[j] = !((uint64_t)(k[j] - 1) < (uint64_t)(loggam_table::N - 1));
        x0[j] = big[j] ? (double)k[j] : 8.0;  // >= 7 for every argument that takes this path
        x2[j] = (1.0 / x0[j]) * (1.0 / x0[j]);
        gl0[j] = a[9];
    }
    for (int i = 8; i >= 0; --i)
        for (int j = 0; j < 4; ++j) {
            gl0[j] *= x2[j];
            gl0[j] += a[i];
        }
    for (int j = 0; j < 4; ++j) {
        if (!big[j]) {
            r[j] = t.v[k[j]];
        } else if (k[j] < 7) {  // k <= 0: loggam's own path (never taken by the sampler)
            r[j] = loggam((double)k[j]);
        } else {
            r[j] = gl0[j] / x0[j] + 0.5 * 1.8378770664093453e+00 + (x0[j] - 0.5) * log(x0[j]) - x0[j];
        }
    }
    return ((r[0] + r[1]) + r[2]) + r[3];
}

// loggam_sum4 of two argument sets: *s0 = set 0 (a0..a3), *s1 = set 1 (b0..b3), each bit for
// bit loggam_sum4's value; with AVX2 + FMA the two sets' large arguments run as two 4-lane
// chains side by side
inline void loggam_sum4_pair(int64_t a0, int64_t a1, int64_t a2, int64_t a3, int64_t b0, int64_t b1, int64_t b2,
                             int64_t b3, double *s0, double *s1) {
#if !defined(__HIP_DEVICE_COMPILE__)
    if (cpu_avx2_fma()) {
        const int64_t k[8] = {a0, a1, a2, a3, b0, b1, b2, b3};
        bool big[8], ok = true;
        for (int j = 0; j < 8; ++j) {
            big[j] = !((uint64_t)(k[j] - 1) < (uint64_t)(loggam_table::N - 1));
            ok &= !big[j] || k[j] >= 8;  // (k <= 0 takes loggam's own path)
        }
        if (ok) {
            loggam_sum4x2_avx2(k, big, s0, s1);
            return;
        }
    }
#endif
    *s0 = loggam_sum4(a0, a1, a2, a3);
    *s1 = loggam_sum4(b0, b1, b2, b3);
}

inline int64_t hypergeometric_hyp(mt19937 &rng, int64_t good, int64_t bad, int64_t sample) {
    const int64_t d1 = bad + good - sample;
    const double d2 = (double)(bad < good ? bad : good);
    double y = d2;
    int64_t k = sample;
    while (y > 0.0) {
        const double u = rng.next_double();
        y -= (int64_t)floor(u + y / (double)(d1 + k));
        k--;
        if (k == 0) break;
    }
    int64_t z = (int64_t)(d2 - y);
    if (good > bad) z = sample - z;
    return z;
}

inline int64_t hypergeometric_hrua(mt19937 &rng, int64_t good, int64_t bad, int64_t sample) {
    const double D1 = 1.7155277699214135, D2 = 0.8989161620588988;
    const int64_t mingoodbad = good < bad ? good : bad;
    const int64_t popsize = good + bad;
    const int64_t maxgoodbad = good > bad ? good : bad;
    const int64_t m = sample < popsize - sample ? sample : popsize - sample;
    const double d4 = ((double)mingoodbad) / popsize;
    const double d5 = 1.0 - d4;
    const double d6 = m * d4 + 0.5;
    const double d7 = sqrt((double)(popsize - m) * sample * d4 * d5 / (popsize - 1) + 0.5);
    const double d8 = D1 * d7 + D2;
    const int64_t d9 = (int64_t)floor((double)(m + 1) * (mingoodbad + 1) / (popsize + 2));
    // d10 = loggam_sum4(d9 + 1, mingoodbad - d9 + 1, m - d9 + 1, maxgoodbad - m + d9 + 1): the
    // same value whenever it is computed, so it is computed together with the first candidate
    // that needs it (two independent chains side by side: the loop's latency is loggam's)
    double d10 = 0.0;
    bool have_d10 = false;
    const double mm = (double)(m < mingoodbad ? m : mingoodbad) + 1.0, fl = floor(d6 + 16 * d7);
    const double d11 = mm < fl ? mm : fl;
    int64_t Z;
    while (true) {
        const double X = rng.next_double();
        const double Y = rng.next_double();
        const double W = d6 + d8 * (Y - 0.5) / X;
        if (W < 0.0 || W >= d11) continue;  // fast rejection
        Z = (int64_t)floor(W);
        double T;
        if (!have_d10) {
            have_d10 = true;
            double s1;
            loggam_sum4_pair(d9 + 1, mingoodbad - d9 + 1, m - d9 + 1, maxgoodbad - m + d9 + 1, Z + 1,
                             mingoodbad - Z + 1, m - Z + 1, maxgoodbad - m + Z + 1, &d10, &s1);
            T = Z == d9 ? 0.0 : d10 - s1;
        } else {
            // (Z == d9: the same four arguments as d10, so the difference is exactly +0.0)
            T = Z == d9 ? 0.0 : d10 - loggam_sum4(Z + 1, mingoodbad - Z + 1, m - Z + 1, maxgoodbad - m + Z + 1);
        }
        if ((X * (4.0 - X) - 3.0) <= T) break;  // fast acceptance
        if (X * (X - T) >= 1) continue;         // fast rejection
        if (2.0 * log(X) <= T) break;           // accept
    }
    if (good > bad) Z = m - Z;
    if (m < sample) Z = good - Z;
    return Z;
}

// numpy legacy RandomState.hypergeometric(ngood, nbad, nsample) for one draw
inline int64_t hypergeometric(mt19937 &rng, int64_t good, int64_t bad, int64_t sample) {
    if (sample > 10) return hypergeometric_hrua(rng, good, bad, sample);
    if (sample > 0) return hypergeometric_hyp(rng, good, bad, sample);
    return 0;
}

// sample() of CV_tools.py:5-27: draw m balls colour by colour, stop when nothing is left;
// the last colour takes the remainder.  tail[i] = balls in colours i..n-1.
inline void sample(mt19937 &rng, uint64_t m, const uint64_t *colors, const uint64_t *tail, uint64_t n,
                   uint64_t *out) {
    for (uint64_t i = 0; i < n; ++i) out[i] = 0;
    int64_t left = (int64_t)m;
    for (uint64_t i = 0; i + 1 < n; ++i) {
        if (left < 1) break;
        const int64_t got = hypergeometric(rng, (int64_t)colors[i], (int64_t)tail[i + 1], left);
        out[i] = (uint64_t)got;
        left -= got;
    }
    if (n) out[n - 1] = (uint64_t)left;
}

}  // namespace kpf
