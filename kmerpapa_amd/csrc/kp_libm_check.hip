// kp_libm_check.hip -- build-time guard (host code only): the restatement of the C
// library's log / log1p in kp_libm.h must reproduce THIS host's libm bit for bit, else the
// GPU's exact-log path (the k-mer cells, the backtrack, the guarded single terms) would no
// longer round like the reference (numba -> libm) and the oracle (libm).  kp_logdata.h is
// read from the host libm by gen_logdata.py, but glibc selects its log variant at run time
// (ifunc: __log_fma on FMA3 CPUs, others elsewhere) and another glibc may change the
// algorithm: either would make the restatement wrong without failing the build.  The
// Makefile runs this before it builds the library and stops on any mismatch.
//
// Inputs: 2^20 pseudo-random doubles in (0, 1) (every rate p and 1 - p of the DP lies
// there), 2^19 log-uniform over the whole positive range (subnormals included), 2^18 near
// 1 (log's table-free path), the log1p argument -p for p in (0, 1), and special values.
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include "kp_libm.h"

static uint64_t g_state = 0x243f6a8885a308d3ull;

static uint64_t next_u64() {  // splitmix64
    uint64_t z = (g_state += 0x9e3779b97f4a7c15ull);
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}

static double unit() { return (double)(next_u64() >> 11) * 0x1p-53; }

// bit-identical, NaNs included (glibc passes an input NaN through with its sign and payload)
static bool same(double a, double b) { return memcmp(&a, &b, sizeof(double)) == 0; }

static long g_bad = 0, g_n = 0, g_fast_far = 0, g_fast_diff = 0;

// distance in units in the last place between two finite doubles of the same sign
static uint64_t ulps(double a, double b) {
    int64_t ia, ib;
    memcpy(&ia, &a, 8);
    memcpy(&ib, &b, 8);
    if (ia < 0) ia = INT64_MIN - ia;
    if (ib < 0) ib = INT64_MIN - ib;
    return ia > ib ? (uint64_t)(ia - ib) : (uint64_t)(ib - ia);
}

static void one(double x) {
    // volatile: the host compiler must call libm, not fold the call with its own arithmetic
    volatile double vx = x;
    const double ref_log = log(vx), ref_log1p = log1p(-vx);
    const double got_log = kp_libm_log(x), got_log1p = kp_libm_log1p(-x);
    ++g_n;
    if (!same(ref_log, got_log)) {
        if (g_bad < 5) fprintf(stderr, "kp_libm_check: log(%a) libm %a restated %a\n", x, ref_log, got_log);
        ++g_bad;
    }
    // the sweep's fast log: within 1 ulp of the C library's (the store guard's premise
    // allows 2); only finite results of the normal positive range are its own
    if (x > 0x1p-1022 && x < HUGE_VAL) {
        const double fl = kp_fast_log(x), fl1 = kp_fast_log(1.0 - x);
        const double ref1 = (1.0 - x > 0x1p-1022) ? log((volatile double)(1.0 - x)) : 0.0;
        const uint64_t d = ulps(fl, ref_log), d1 = (1.0 - x > 0x1p-1022) ? ulps(fl1, ref1) : 0;
        g_fast_diff += (d != 0) + (d1 != 0);
        if (d > 1 || d1 > 1) {
            if (g_fast_far < 5) fprintf(stderr, "kp_libm_check: fast log(%a) off by %llu / %llu ulp\n", x,
                                        (unsigned long long)d, (unsigned long long)d1);
            ++g_fast_far;
        }
        // kp_fma_log (the host form: exact reciprocal) within 2 ulp, the guard's premise
        const uint64_t e = ulps(kp_fma_log(x), ref_log), e1 = (1.0 - x > 0x1p-1022) ? ulps(kp_fma_log(1.0 - x), ref1) : 0;
        if (e > 2 || e1 > 2) {
            if (g_fast_far < 5) fprintf(stderr, "kp_libm_check: fma log(%a) off by %llu / %llu ulp\n", x,
                                        (unsigned long long)e, (unsigned long long)e1);
            ++g_fast_far;
        }
    }
    if (!same(ref_log1p, got_log1p)) {
        if (g_bad < 5) fprintf(stderr, "kp_libm_check: log1p(%a) libm %a restated %a\n", -x, ref_log1p, got_log1p);
        ++g_bad;
    }
}

int main() {
    for (int i = 0; i < (1 << 20); ++i) one(unit());
    for (int i = 0; i < (1 << 19); ++i) {
        uint64_t u = next_u64() & 0x7fefffffffffffffull;  // finite, positive
        double x;
        memcpy(&x, &u, 8);
        one(x);
    }
    for (int i = 0; i < (1 << 18); ++i) one(1.0 + (unit() - 0.5) * 0x1p-4);
    const double special[] = {0.0, -0.0, 1.0, 0.5, 2.0, 0x1p-1074, 0x1p-1022, 0x1.fffffffffffffp-1,
                              0x1.0000000000001p0, 1e-300, 1e300, HUGE_VAL, -1.0, -2.0, NAN, -NAN};
    for (double x : special) one(x);
    if (g_fast_far) {
        fprintf(stderr, "kp_libm_check: FAILED: kp_fast_log more than 1 ulp (kp_fma_log: 2) from the C library's log on %ld inputs\n",
                g_fast_far);
        return 1;
    }
    if (g_bad) {
        fprintf(stderr,
                "kp_libm_check: FAILED: %ld of %ld log/log1p results of kp_libm.h differ from this host's C "
                "library; the build stops (see kp_libm.h, gen_logdata.py)\n",
                g_bad, 2 * g_n);
        return 1;
    }
    printf("kp_libm_check: kp_libm.h log/log1p bit-identical to the host C library on %ld inputs; kp_fast_log "
           "within 1 ulp of its log (%ld of the results differ), kp_fma_log within 2\n", 2 * g_n, g_fast_diff);
    return 0;
}
