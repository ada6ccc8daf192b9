// kp_libm.h -- the host C library's float64 log and log1p, restated operation for operation
// (host and device), so that the GPU reproduces bit for bit the values the reference gets:
// numba lowers np.log / np.log1p to libm calls, and the oracle calls libm directly.
//
//  * kp_libm_log   = glibc 2.35 x86-64 __log_fma (the variant its ifunc selects on CPUs with
//                    FMA3): every fused multiply-add and every rounding in the order of that
//                    binary's instructions; its data block (ln2 in two parts, 5 + 11
//                    polynomial coefficients, 128 (1/c, log c) entries) is read from the
//                    system libm by gen_logdata.py into kp_logdata.h.
//  * kp_libm_log1p = glibc 2.35 __log1p (fdlibm's algorithm, compiled without FMA): plain
//                    float64 operations in the binary's order.
//
// The sweep keeps ROCm's ocml log on its fast path (within 1 ulp of these) and falls back to
// these only when a float32 store could depend on that last bit (kp_core.h).  Tests:
// test_libm_restatement (host, against the process's own libm) and the GPU test
// test_device_libm_log_exact (device, against the GPU box's libm).
#pragma once
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "kp_logdata.h"

__host__ __device__ inline uint64_t kp_asu64(double x) { return __builtin_bit_cast(uint64_t, x); }
__host__ __device__ inline double kp_asf64(uint64_t u) { return __builtin_bit_cast(double, u); }

#ifdef __HIP_DEVICE_COMPILE__
__device__ static const double kp_log_tab_d[256] = KP_LOG_TAB;
#define KP_LOG_TABLE kp_log_tab_d
#else
static const double kp_log_tab_h[256] = KP_LOG_TAB;
#define KP_LOG_TABLE kp_log_tab_h
#endif

// (out of line: in the sweep these are cold paths, and inlined their constants and table
// reads would load the kernel's registers)
__host__ __device__ __attribute__((noinline)) inline double kp_libm_log(double x) {
    const double A[5] = KP_LOG_POLY;
    const double B[11] = KP_LOG_POLY1;
    uint64_t ix = kp_asu64(x);
    const uint32_t top = (uint32_t)(ix >> 48);
    if (ix - 0x3fee000000000000ull < 0x0003090000000000ull) {  // |x - 1| small: no table
        if (ix == 0x3ff0000000000000ull) return 0.0;
        const double r = x - 1.0;
        const double r2 = r * r;
        const double r3 = r * r2;
        const double v1 = fma(r2, B[3], fma(r, B[2], B[1]));
        const double v2 = fma(r2, B[6], fma(r, B[5], B[4]));
        const double v3 = fma(r3, B[10], fma(r2, B[9], fma(r, B[8], B[7])));
        // y = r3 * (v1 + r3 * (v2 + r3 * v3)) + lo, with the split of r into rhi + rlo
        const double outer = fma(fma(v3, r3, v2), r3, v1);
        const double t = fma(r, 0x1p27, r);  // r + r * 2^27
        const double rhi = fma(-0x1p27, r, t);
        const double rlo = r - rhi;
        const double rhi2 = rhi * rhi;
        const double hi = fma(rhi2, B[0], r);
        double lo = fma(rhi2, B[0], r - hi);
        lo = fma(B[0] * rlo, r + rhi, lo);
        const double y = fma(outer, r3, lo);
        return hi + y;
    }
    if (top - 0x0010u >= 0x7ff0u - 0x0010u) {  // subnormal, zero, negative, inf or NaN
        if (ix * 2 == 0) return -__builtin_huge_val();
        if (ix == 0x7ff0000000000000ull) return x;
        if ((top & 0x8000u) || (top & 0x7ff0u) == 0x7ff0u) return (x - x) / (x - x);  // NaN (an input NaN propagates)
        ix = kp_asu64(x * 0x1p52) - (52ull << 52);  // normalise the subnormal
    }
    const uint64_t tmp = ix - 0x3fe6000000000000ull;
    const int i = (int)((tmp >> 45) & 127u);
    const int k = (int)((int64_t)tmp >> 52);
    const uint64_t iz = ix - (tmp & 0xfff0000000000000ull);
    const double invc = KP_LOG_TABLE[2 * i], logc = KP_LOG_TABLE[2 * i + 1];
    const double z = kp_asf64(iz);
    const double r = fma(z, invc, -1.0);
    const double kd = (double)k;
    const double w = fma(kd, KP_LOG_LN2HI, logc);
    const double hi = r + w;
    const double lo = fma(kd, KP_LOG_LN2LO, (w - hi) + r);
    const double r2 = r * r;
    const double t1 = fma(r, A[2], A[1]);
    const double r3 = r * r2;
    const double t2 = fma(r, A[4], A[3]);
    const double lo2 = fma(r2, A[0], lo);
    const double poly = fma(t2, r2, t1);
    const double y = fma(r3, poly, lo2);
    return y + hi;
}

__host__ __device__ __attribute__((noinline)) inline double kp_libm_log1p(double x) {
    const double ln2_hi = 0x1.62e42fee00000p-1, ln2_lo = 0x1.a39ef35793c76p-33;
    const double Lp1 = 0x1.5555555555593p-1, Lp2 = 0x1.999999997fa04p-2, Lp3 = 0x1.2492494229359p-2,
                 Lp4 = 0x1.c71c51d8e78afp-3, Lp5 = 0x1.7466496cb03dep-3, Lp6 = 0x1.39a09d078c69fp-3,
                 Lp7 = 0x1.2f112df3e5244p-3;
    const int32_t hx = (int32_t)(kp_asu64(x) >> 32);
    const int32_t ax = hx & 0x7fffffff;
    int32_t k = 1, hu = 0;
    double f = 0.0, c = 0.0;
    if (hx < 0x3FDA827A) {  // x < 0.41422
        if (ax >= 0x3ff00000) {  // x <= -1 (or a negative NaN)
            if (x == -1.0) return -__builtin_huge_val();
            return (x - x) / (x - x);  // NaN (an input NaN propagates)
        }
        if (ax < 0x3e200000) {  // |x| < 2^-29
            if (ax < 0x3c900000) return x;
            return x - x * x * 0.5;
        }
        if (hx > 0 || hx <= (int32_t)0xbfd2bec4) {  // -0.2929 < x < 0.41422
            k = 0;
            f = x;
            hu = 1;
        }
    } else if (hx >= 0x7ff00000) {
        return x + x;
    }
    if (k != 0) {
        double u;
        if (hx < 0x43400000) {
            u = 1.0 + x;
            hu = (int32_t)(kp_asu64(u) >> 32);
            k = (hu >> 20) - 1023;
            c = (k > 0) ? 1.0 - (u - x) : x - (u - 1.0);  // correction term
            c /= u;
        } else {
            u = x;
            hu = (int32_t)(kp_asu64(u) >> 32);
            k = (hu >> 20) - 1023;
            c = 0;
        }
        hu &= 0x000fffff;
        const uint64_t ulo = kp_asu64(u) & 0xffffffffull;
        if (hu < 0x6a09e) {
            u = kp_asf64(((uint64_t)(uint32_t)(hu | 0x3ff00000) << 32) | ulo);  // normalise u
        } else {
            k += 1;
            u = kp_asf64(((uint64_t)(uint32_t)(hu | 0x3fe00000) << 32) | ulo);  // normalise u / 2
            hu = (0x00100000 - hu) >> 2;
        }
        f = u - 1.0;
    }
    const double hfsq = 0.5 * f * f;
    if (hu == 0) {  // |f| < 2^-20
        if (f == 0.0) {
            if (k == 0) return 0.0;
            c += k * ln2_lo;
            return k * ln2_hi + c;
        }
        const double R = hfsq * (1.0 - 0.66666666666666666 * f);
        if (k == 0) return f - R;
        return k * ln2_hi - ((R - (k * ln2_lo + c)) - f);
    }
    const double s = f / (2.0 + f);
    const double z = s * s;
    const double R1 = z * Lp1, z2 = z * z;
    const double R2 = Lp2 + z * Lp3, z4 = z2 * z2;
    const double R3 = Lp4 + z * Lp5, z6 = z4 * z2;
    const double R4 = Lp6 + z * Lp7;
    const double R = R1 + z2 * R2 + z4 * R3 + z6 * R4;
    if (k == 0) return f - (hfsq - s * (hfsq + R));
    return k * ln2_hi - ((hfsq - (s * (hfsq + R) + (k * ln2_lo + c))) - f);
}

// kp_fast_log -- the sweep's fast float64 log (device and host, no table, no FMA): fdlibm's
// __ieee754_log algorithm (the table-free ancestor of glibc's log; error < 1 ulp), written
// branch-light for the GPU: both of fdlibm's final formulas are evaluated and one selected
// exactly as fdlibm's branch would.  It stands in for ROCm's ocml log (85 instructions) on
// the sweep's fast path, where any log within 2 ulp of the C library's is admissible: the
// store guard (kp_core.h kp_store_unsafe) sends every float32 result that could depend on
// the last bits to the C library's restated log.  |kp_fast_log - libm log| <= 1 ulp is
// checked at build time (kp_libm_check) and on the GPU (test_device_fast_log_within_1ulp).
// Arguments outside the normal positive range (0, subnormals, negatives, inf, NaN) take
// the device's own log.
__host__ __device__ inline double kp_fast_log(double x) {
    const double ln2_hi = 0x1.62e42fee00000p-1, ln2_lo = 0x1.a39ef35793c76p-33;
    const double Lg1 = 0x1.5555555555593p-1, Lg2 = 0x1.999999997fa04p-2, Lg3 = 0x1.2492494229359p-2,
                 Lg4 = 0x1.c71c51d8e78afp-3, Lg5 = 0x1.7466496cb03dep-3, Lg6 = 0x1.39a09d078c69fp-3,
                 Lg7 = 0x1.2f112df3e5244p-3;
    const uint64_t ix = kp_asu64(x);
    int32_t hx = (int32_t)(ix >> 32);
    if (__builtin_expect(hx < 0x00100000 || hx >= 0x7ff00000, 0)) return log(x);
    int32_t k = (hx >> 20) - 1023;
    hx &= 0x000fffff;
    const int32_t i0 = (hx + 0x95f64) & 0x100000;
    const double xn = kp_asf64(((uint64_t)(uint32_t)(hx | (i0 ^ 0x3ff00000)) << 32) | (ix & 0xffffffffull));
    k += (i0 >> 20);
    const double f = xn - 1.0;
    const double dk = (double)k;
    if (__builtin_expect((0x000fffff & (2 + hx)) < 3, 0)) {  // -2^-20 <= f < 2^-20
        if (f == 0.0) return k == 0 ? 0.0 : dk * ln2_hi + dk * ln2_lo;
        const double R = f * f * (0.5 - 0.33333333333333333 * f);
        return k == 0 ? f - R : dk * ln2_hi - ((R - dk * ln2_lo) - f);
    }
    const double s = f / (2.0 + f);
    const double z = s * s;
    const double w = z * z;
    const double t1 = w * (Lg2 + w * (Lg4 + w * Lg6));
    const double t2 = z * (Lg1 + w * (Lg3 + w * (Lg5 + w * Lg7)));
    const double R = t2 + t1;
    const bool big = ((hx - 0x6147a) | (0x6b851 - hx)) > 0;
    const double hfsq = 0.5 * f * f;
    // fdlibm: if big  f - (hfsq - s*(hfsq+R))  /  dk*ln2_hi - ((hfsq - (s*(hfsq+R) + dk*ln2_lo)) - f)
    //         else    f - s*(f-R)              /  dk*ln2_hi - ((s*(f-R) - dk*ln2_lo) - f)
    const double a = big ? hfsq - s * (hfsq + R) : s * (f - R);
    if (k == 0) return f - a;
    const double b = big ? hfsq - (s * (hfsq + R) + dk * ln2_lo) : s * (f - R) - dk * ln2_lo;
    return dk * ln2_hi - (b - f);
}

// kp_fma_log -- fdlibm's log algorithm (as kp_fast_log) rewritten for throughput on the
// GPU: the quotient s = f / (2 + f) from the hardware reciprocal refined by Newton steps
// (no IEEE division sequence), the polynomials and the quotient's correction as fused
// multiply-adds, fdlibm's k == 0 and small-f branches folded into the general formula
// (the same values up to rounding), and both of its final formulas evaluated and one
// selected.  Not bit-identical to fdlibm or the C library: within 2 ulp of the C library's
// log, which is what the store guard admits (kp_core.h kp_store_unsafe; checked at build
// time by kp_libm_check on the host's form -- exact reciprocal -- and on the GPU by
// test_device_fma_log_within_2ulp).  Arguments outside the normal positive range take the
// C library's restated log (out of line).
__host__ __device__ inline double kp_fma_log(double x) {
    const double ln2_hi = 0x1.62e42fee00000p-1, ln2_lo = 0x1.a39ef35793c76p-33;
    const double Lg1 = 0x1.5555555555593p-1, Lg2 = 0x1.999999997fa04p-2, Lg3 = 0x1.2492494229359p-2,
                 Lg4 = 0x1.c71c51d8e78afp-3, Lg5 = 0x1.7466496cb03dep-3, Lg6 = 0x1.39a09d078c69fp-3,
                 Lg7 = 0x1.2f112df3e5244p-3;
    const uint64_t ix = kp_asu64(x);
    int32_t hx = (int32_t)(ix >> 32);
    if (__builtin_expect(hx < 0x00100000 || hx >= 0x7ff00000, 0)) return kp_libm_log(x);
    int32_t k = (hx >> 20) - 1023;
    hx &= 0x000fffff;
    const int32_t i0 = (hx + 0x95f64) & 0x100000;  // mantissa >= sqrt(2): halve it (fdlibm)
    const double xn = kp_asf64(((uint64_t)(uint32_t)(hx | (i0 ^ 0x3ff00000)) << 32) | (ix & 0xffffffffull));
    k += (i0 >> 20);
    const double f = xn - 1.0;  // exact
    const double d = 2.0 + f;
#if defined(__HIP_DEVICE_COMPILE__)
    double r = __builtin_amdgcn_rcp(d);  // d in [1.7, 2.5]: no scaling needed
    r = __builtin_fma(__builtin_fma(-d, r, 1.0), r, r);
    r = __builtin_fma(__builtin_fma(-d, r, 1.0), r, r);
#else
    const double r = 1.0 / d;
#endif
    double s = f * r;
    s = __builtin_fma(__builtin_fma(-s, d, f), r, s);
    const double z = s * s;
    const double w = z * z;
    const double t1 = w * __builtin_fma(w, __builtin_fma(w, Lg6, Lg4), Lg2);
    const double t2 = z * __builtin_fma(w, __builtin_fma(w, __builtin_fma(w, Lg7, Lg5), Lg3), Lg1);
    const double R = t2 + t1;
    const bool big = ((hx - 0x6147a) | (0x6b851 - hx)) > 0;
    const double dk = (double)k;
    const double hfsq = 0.5 * f * f;
    // fdlibm: big  dk*ln2_hi - ((hfsq - (s*(hfsq+R) + dk*ln2_lo)) - f)
    //         else dk*ln2_hi - ((s*(f-R) - dk*ln2_lo) - f)          (k == 0: the same with dk = 0)
    // as one expression b = a0 - (s*b0 + dk*ln2_lo): for "else" a0 = 0, b0 = R - f, and
    // 0 - fma(s, R - f, c) is fma(s, f - R, -c) exactly (negation is exact, rounding symmetric)
    const double a0 = big ? hfsq : 0.0, b0 = big ? hfsq + R : R - f;
    const double b = a0 - __builtin_fma(s, b0, dk * ln2_lo);
    return __builtin_fma(dk, ln2_hi, -(b - f));
}
