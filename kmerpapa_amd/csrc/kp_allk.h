// kp_allk.h -- `--score all_kmers`: one rate per k-mer, cross-validated over the pseudo
// count (reference src/kmerpapa/algorithms/all_kmers_CV.py, v0.2.4).  Included by kp_hip.hip.
//
// There is no lattice here: every k-mer is its own pattern, so the loss of a fold is a sum
// over k-mers of a closed form (test_folds :8-13):
//     p    = (trM + a) / (trM + trU + a + b_f)          trM = sum_g M[i][g] - M[i][f]  (:41-42)
//     term = -2 * (xlogy(teM, p) + xlog1py(teU, -p))
// with (teM, teU) = (trM, trU) for the train sum and the fold's own counts for the test sum
// (:43-44).  The reference accumulates those terms k-mer by k-mer in float64
// (`sum_test += ...` in matches(gen_pat) order, :36-44), so the sum is done sequentially
// in that order here too -- one thread per (fold, kind) column -- after a fully parallel
// pass that evaluates every term with the C library's log / log1p (kp_libm.h), the
// functions scipy's xlogy / xlog1py call.  Results are bit-identical to the reference.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "kp_core.h"

// terms[kind][f][i] (kind 0 = train, 1 = test) of one alpha; M, U: [n][nf] uint64
__global__ void __launch_bounds__(256) kp_allk_terms(const uint64_t *__restrict__ M, const uint64_t *__restrict__ U,
                                                     uint64_t n, int nf, double alpha, const double *__restrict__ betas,
                                                     double *__restrict__ terms) {
    const uint64_t total = n * (uint64_t)nf;
    for (uint64_t e = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; e < total;
         e += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t i = e / (uint64_t)nf;
        const int f = (int)(e % (uint64_t)nf);
        const uint64_t *mr = M + i * nf, *ur = U + i * nf;
        uint64_t sm = 0, su = 0;
        for (int g = 0; g < nf; ++g) {  // the row total (uint64, exact)
            sm += mr[g];
            su += ur[g];
        }
        kp_cnt c;
        c.mte = mr[f];
        c.ute = ur[f];
        c.mtr = sm - c.mte;
        c.utr = su - c.ute;
        const double p = kp_rate(c, alpha, betas[f]);
        const double tr = -2.0 * (kp_xlogy((double)c.mtr, p) + kp_xlog1py((double)c.utr, -p));
        const double te = -2.0 * (kp_xlogy((double)c.mte, p) + kp_xlog1py((double)c.ute, -p));
        terms[(uint64_t)f * n + i] = tr;
        terms[((uint64_t)nf + f) * n + i] = te;
    }
}

// sums[col] = 0.0 + terms[col][0] + terms[col][1] + ... in k-mer order, one thread per
// column (2 * nf columns); the loads run ahead of the dependent float64 adds
__global__ void __launch_bounds__(64) kp_allk_sums(const double *__restrict__ terms, uint64_t n, int ncol,
                                                   double *__restrict__ sums) {
    const int col = (int)(blockIdx.x * blockDim.x + threadIdx.x);
    if (col >= ncol) return;
    const double *t = terms + (uint64_t)col * n;
    double s = 0.0;
    uint64_t i = 0;
    for (; i + 8 <= n; i += 8) {
        double v[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) v[q] = t[i + q];
#pragma unroll
        for (int q = 0; q < 8; ++q) s += v[q];
    }
    for (; i < n; ++i) s += t[i];
    sums[col] = s;
}
