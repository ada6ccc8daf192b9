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

inline double loggam_sum4(int64_t k0, int64_t k1, int64_t k2, int64_t k3) {
    static const loggam_table t;
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
    const double d10 = loggam_sum4(d9 + 1, mingoodbad - d9 + 1, m - d9 + 1, maxgoodbad - m + d9 + 1);
    const double mm = (double)(m < mingoodbad ? m : mingoodbad) + 1.0, fl = floor(d6 + 16 * d7);
    const double d11 = mm < fl ? mm : fl;
    int64_t Z;
    while (true) {
        const double X = rng.next_double();
        const double Y = rng.next_double();
        const double W = d6 + d8 * (Y - 0.5) / X;
        if (W < 0.0 || W >= d11) continue;  // fast rejection
        Z = (int64_t)floor(W);
        const double T = d10 - loggam_sum4(Z + 1, mingoodbad - Z + 1, m - Z + 1, maxgoodbad - m + Z + 1);
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
