/*
 * kp_oracle.c -- CPU restatement of kmerPaPa's penalized-likelihood lattice DP.
 *
 * TEST INFRASTRUCTURE ONLY.  This file is the checker: tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load it; the product path (kmerpapa_amd/) never
 * does.  It restates, cell by cell and in the reference's order of operations, the two
 * numba kernels of BesenbacherLab/kmerPaPa v0.2.4:
 *
 *   kpo_cv  : src/kmerpapa/algorithms/bottum_up_array_penalty_plus_pseudo_CV.py
 *             score_test_folds :15-20, get_train :22-24, handle_pattern :26-78,
 *             driver loop :143-157
 *   kpo_fit : src/kmerpapa/algorithms/bottum_up_array_w_numba.py
 *             score :26-29, handle_pattern :31-64, driver :67-124
 *
 * Lattice tables follow src/kmerpapa/pattern_utils.py:5-100 (IUPAC code, perm_code,
 * complements).  Parity is pinned by tests/test_oracle_golden.py against vectors the
 * reference itself produced (tests/golden/make_golden.py).
 *
 * Arithmetic notes (why each line is written the way it is):
 *  - scores are stored as float32 (ftype = np.float32, CV :89, Fit :79); split sums are
 *    float32 + float32; the single-pattern term is float64 and compared as float64
 *    against the float32 store (numba / numpy<2 promotion) before rounding to float32.
 *  - counts are itype = uint32 or uint64 (CV :94-97); aggregation wraps at itype width;
 *    fold totals are summed in uint64 (numpy sum of uint32 -> uint64).
 *  - level 0 uses xlogy / xlog1py (scipy: 0 if x == 0 and y is not NaN) in the order
 *    -2*(a+b)+c; levels >= 1 use log(p), log(1-p) in the order c + a + b.
 *  Build with -ffp-contract=off (no fused multiply-add), -O2, no fast-math.
 *  - nthreads > 1 splits each level's cells over OpenMP threads: a cell reads only cells of
 *    strictly lower levels, so every value is the same as with one thread (the reference
 *    walks a level in any order it likes, CV :156, Fit :119).
 */
#include <math.h>
#include <omp.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define KPO_MAXK 32

typedef struct {
    int k;
    int radix[KPO_MAXK];
    uint64_t cg[KPO_MAXK];
    int lev[KPO_MAXK][16];
    int np[KPO_MAXK][16];
    int pa[KPO_MAXK][16][7];
    int pb[KPO_MAXK][16][7];
    uint64_t npat;
    int maxlev;
} kpo_lat;

/* IUPAC data, pattern_utils.py:5-19 (code), :86-100 (perm_code), :48-57 (complements) */
static const char *IU_CODES = "ACGTRYSWKMBDHVN";
static const char *IU_NUC[15] = {"A", "C", "G", "T", "AG", "CT", "GC", "AT", "GT", "AC",
                                 "CGT", "AGT", "ACT", "ACG", "ACGT"};
static const char *IU_PERM[15] = {"A", "C", "G", "T", "AGR", "CTY", "GCS", "ATW", "GTK", "ACM",
                                  "CGTSYKB", "AGTRWKD", "ACTMWYH", "ACGMRSV", "ACGTRYSWKMBDHVN"};
static const char *IU_SPLIT[15] = {"", "", "", "", "AG", "CT", "GC", "AT", "GT", "AC",
                                   "CKGYTS", "AKGWTR", "AYCWTM", "ASCRGM", "SWKMRYABCDGHTV"};

static int iu_index(char c) {
    const char *p = strchr(IU_CODES, c);
    return (p && c) ? (int)(p - IU_CODES) : -1;
}

static int lat_build(const char *gp, kpo_lat *L) {
    memset(L, 0, sizeof(*L));
    L->k = (int)strlen(gp);
    if (L->k <= 0 || L->k > KPO_MAXK) return -1;
    uint64_t acc = 1;
    for (int i = 0; i < L->k; ++i) {
        int g = iu_index(gp[i]);
        if (g < 0) return -1;
        const char *perm = IU_PERM[g];
        int r = (int)strlen(perm);
        L->radix[i] = r;
        L->cg[i] = acc;
        acc *= (uint64_t)r;
        L->maxlev += (int)strlen(IU_NUC[g]) - 1;
        for (int d = 0; d < r; ++d) {
            int x = iu_index(perm[d]);
            L->lev[i][d] = (int)strlen(IU_NUC[x]) - 1;
            const char *sp = IU_SPLIT[x];
            int n = (int)strlen(sp) / 2;
            L->np[i][d] = n;
            for (int j = 0; j < n; ++j) {
                L->pa[i][d][j] = (int)(strchr(perm, sp[2 * j]) - perm);
                L->pb[i][d][j] = (int)(strchr(perm, sp[2 * j + 1]) - perm);
            }
        }
    }
    L->npat = acc;
    return 0;
}

/* cells bucketed by level, ascending index inside a level (the reference walks a level in
 * subpatterns_level_ord_np order; the order inside a level does not change any value
 * because a cell only reads strictly lower levels). */
static uint64_t *level_order(const kpo_lat *L, uint64_t *off /* [maxlev+2] */) {
    uint64_t *out = (uint64_t *)malloc(sizeof(uint64_t) * L->npat);
    uint8_t *lv = (uint8_t *)malloc(L->npat);
    if (!out || !lv) { free(out); free(lv); return NULL; }
    memset(off, 0, sizeof(uint64_t) * (L->maxlev + 2));
    for (uint64_t n = 0; n < L->npat; ++n) {
        uint64_t q = n;
        int s = 0;
        for (int i = 0; i < L->k; ++i) { s += L->lev[i][q % L->radix[i]]; q /= L->radix[i]; }
        lv[n] = (uint8_t)s;
        off[s + 1]++;
    }
    for (int s = 0; s <= L->maxlev; ++s) off[s + 1] += off[s];
    uint64_t *fill = (uint64_t *)calloc(L->maxlev + 1, sizeof(uint64_t));
    for (uint64_t n = 0; n < L->npat; ++n) out[off[lv[n]] + fill[lv[n]]++] = n;
    free(fill);
    free(lv);
    return out;
}

static inline double xlogy_(double x, double y) { return (x == 0.0 && !isnan(y)) ? 0.0 : x * log(y); }
static inline double xlog1py_(double x, double y) { return (x == 0.0 && !isnan(y)) ? 0.0 : x * log1p(y); }

uint64_t kpo_npat(const char *gp) {
    kpo_lat L;
    return lat_build(gp, &L) ? 0 : L.npat;
}

/*
 * CV pass for one (alpha, penalty) over all folds.
 *   M, U  : [npat][nf] counts; the k-mer (level-0) rows are inputs, all other rows are
 *           outputs (aggregated like the reference, wrapping at itype_bits).
 *   betas : [nf]
 *   score, test : [npat][nf] float32 outputs (train score and test -2LL of every cell).
 */
int kpo_cv(const char *gp, int nf, uint64_t *M, uint64_t *U, int itype_bits,
           double alpha, const double *betas, double penalty, float *score, float *test, int nthreads) {
    kpo_lat L;
    if (lat_build(gp, &L) || nf <= 0 || nf > 64) return -1;
    const uint64_t mask = itype_bits >= 64 ? ~0ULL : ((1ULL << itype_bits) - 1);
    uint64_t off[KPO_MAXK * 3 + 2];
    uint64_t *ord = level_order(&L, off);
    if (!ord) return -2;
    const float inf32 = (float)1e100; /* np.full(..., 1e100, float32) -> +inf (CV :143) */
    const int nt = nthreads > 0 ? nthreads : 1;
#pragma omp parallel for num_threads(nt) schedule(static)
    for (uint64_t n = 0; n < L.npat * (uint64_t)nf; ++n) { score[n] = inf32; test[n] = 0.0f; }

    /* level 0: score_test_folds (CV :15-20) on every k-mer row, get_train (:22-24) */
#pragma omp parallel for num_threads(nt) schedule(static)
    for (uint64_t q = off[0]; q < off[1]; ++q) {
        uint64_t n = ord[q];
        const uint64_t *m = M + n * nf, *u = U + n * nf;
        uint64_t sm = 0, su = 0;
        for (int f = 0; f < nf; ++f) { sm += m[f]; su += u[f]; }
        for (int f = 0; f < nf; ++f) {
            uint64_t trm = sm - m[f], tru = su - u[f];
            double p = ((double)trm + alpha) / (((double)(trm + tru) + alpha) + betas[f]);
            double tr = -2.0 * (xlogy_((double)trm, p) + xlog1py_((double)tru, -p)) + penalty;
            double te = -2.0 * (xlogy_((double)m[f], p) + xlog1py_((double)u[f], -p));
            score[n * nf + f] = (float)tr;
            test[n * nf + f] = (float)te;
        }
    }
    /* levels >= 1: handle_pattern (CV :26-78), one level after the other */
    for (int lev = 1; lev <= L.maxlev; ++lev)
#pragma omp parallel for num_threads(nt) schedule(static)
    for (uint64_t q = off[lev]; q < off[lev + 1]; ++q) {
        uint64_t n = ord[q];
        float *rs = score + n * nf, *rt = test + n * nf;
        int first = 1;
        uint64_t rest = n;
        for (int i = 0; i < L.k; ++i) {
            int d = (int)(rest % L.radix[i]);
            rest /= L.radix[i];
            for (int j = 0; j < L.np[i][d]; ++j) {
                uint64_t base = n - (uint64_t)d * L.cg[i];
                uint64_t c1 = base + (uint64_t)L.pa[i][d][j] * L.cg[i];
                uint64_t c2 = base + (uint64_t)L.pb[i][d][j] * L.cg[i];
                for (int f = 0; f < nf; ++f) {
                    float nt = score[c1 * nf + f] + score[c2 * nf + f];
                    float ne = test[c1 * nf + f] + test[c2 * nf + f];
                    if (nt < rs[f]) { rs[f] = nt; rt[f] = ne; }
                }
                if (first) {
                    for (int f = 0; f < nf; ++f) {
                        M[n * nf + f] = (M[c1 * nf + f] + M[c2 * nf + f]) & mask;
                        U[n * nf + f] = (U[c1 * nf + f] + U[c2 * nf + f]) & mask;
                    }
                    first = 0;
                }
            }
        }
        const uint64_t *m = M + n * nf, *u = U + n * nf;
        uint64_t sm = 0, su = 0;
        for (int f = 0; f < nf; ++f) { sm += m[f]; su += u[f]; }
        for (int f = 0; f < nf; ++f) {
            uint64_t trm = sm - m[f], tru = su - u[f];
            double p = ((double)trm + alpha) / (((double)(trm + tru) + alpha) + betas[f]);
            double logp = log(p), log1mp = log(1.0 - p);
            double s = penalty;
            if (trm > 0) s += (-2.0 * (double)trm) * logp;
            if (tru > 0) s += (-2.0 * (double)tru) * log1mp;
            if (s < (double)rs[f]) {
                rs[f] = (float)s;
                double t = 0.0;
                if (m[f] > 0) t += (-2.0 * (double)m[f]) * logp;
                if (u[f] > 0) t += (-2.0 * (double)u[f]) * log1mp;
                rt[f] = (float)t;
            }
        }
    }
    free(ord);
    return 0;
}

/*
 * One CV lane over a whole lattice, memory-lean: the train score of every cell for ONE fold
 * (train counts = all data - that fold, CV :22-24, :56-59) and one (alpha, beta_f, penalty),
 * the same per-cell recurrence as kpo_cv (CV :15-20 at k-mers, :26-71 above) -- the train
 * scores of a lane depend on nothing else (the test array only feeds test_score_mem).
 * Memory: the score array (caller's, float32 [npat]) + train counts of every cell
 * (uint32 when ``itype_bits`` is 32, else uint64), 12 B/cell at 32 bits: a 7.7e9-cell
 * 9-mer lane in 92 GB, where kpo_cv's [npat][nf] layout would need 38 B/cell/fold.
 * Counts are aggregated over the first split pair like the reference (CV :52-55); with the
 * reference's itype rule (CV :94-97: uint32 only if all counts sum below 2^32) no cell's
 * train count can wrap, so summing train counts equals summing folds and subtracting.
 *   kcell[n_kmers]: cell index of each k-mer; m, u: its train counts.
 * Cells are walked level by level, each level's cells split over OpenMP threads through a
 * low/high decomposition of the index (no [npat] level-order array): low = the first
 * positions whose radix product is <= 4096, a cell's level = low level + high level.
 */
#define KPO_LANE_BODY(CT)                                                                              \
    do {                                                                                               \
        CT *M = (CT *)calloc(L.npat, sizeof(CT)), *U = (CT *)calloc(L.npat, sizeof(CT));              \
        if (!M || !U) { free(M); free(U); rc = -2; break; }                                           \
        for (uint64_t j = 0; j < n_kmers; ++j) { M[kcell[j]] = (CT)m[j]; U[kcell[j]] = (CT)u[j]; }      \
        for (int lev = 0; lev <= L.maxlev; ++lev) {                                                    \
            _Pragma("omp parallel for num_threads(nt) schedule(dynamic, 64)")                          \
            for (uint64_t h = 0; h < nhi; ++h) {                                                       \
                const int ll = lev - (int)hlev[h];                                                     \
                if (ll < 0 || ll > lomax) continue;                                                    \
                int dg[KPO_MAXK];                                                                      \
                uint64_t hq = h;                                                                       \
                for (int i = t; i < L.k; ++i) { dg[i] = (int)(hq % L.radix[i]); hq /= L.radix[i]; }    \
                for (uint64_t q = looff[ll]; q < looff[ll + 1]; ++q) {                                 \
                    const uint64_t n = h * B + lolist[q];                                              \
                    if (lev == 0) { /* a k-mer: score_test_folds (CV :15-20) */                        \
                        const uint64_t trm = M[n], tru = U[n];                                         \
                        double p = ((double)trm + alpha) / (((double)(trm + tru) + alpha) + beta);     \
                        score[n] = (float)(-2.0 * (xlogy_((double)trm, p) + xlog1py_((double)tru, -p)) \
                                           + penalty);                                                 \
                        continue;                                                                      \
                    }                                                                                  \
                    float rs = inf32;                                                                  \
                    int first = 1;                                                                     \
                    for (int i = 0; i < t; ++i) dg[i] = lodig[lolist[q] * (uint64_t)t + i];           \
                    for (int i = 0; i < L.k; ++i) {                                                    \
                        const int d = dg[i];                                                           \
                        for (int j = 0; j < L.np[i][d]; ++j) {                                         \
                            uint64_t base = n - (uint64_t)d * L.cg[i];                                 \
                            uint64_t c1 = base + (uint64_t)L.pa[i][d][j] * L.cg[i];                    \
                            uint64_t c2 = base + (uint64_t)L.pb[i][d][j] * L.cg[i];                    \
                            float ns = score[c1] + score[c2];                                          \
                            if (ns < rs) rs = ns;                                                      \
                            if (first) { M[n] = M[c1] + M[c2]; U[n] = U[c1] + U[c2]; first = 0; }      \
                        }                                                                              \
                    }                                                                                  \
                    const uint64_t trm = M[n], tru = U[n];                                             \
                    double p = ((double)trm + alpha) / (((double)(trm + tru) + alpha) + beta);         \
                    double s = penalty;                                                                \
                    if (trm > 0) s += (-2.0 * (double)trm) * log(p);                                   \
                    if (tru > 0) s += (-2.0 * (double)tru) * log(1.0 - p);                             \
                    score[n] = (s < (double)rs) ? (float)s : rs;                                       \
                }                                                                                      \
            }                                                                                          \
        }                                                                                              \
        free(M);                                                                                       \
        free(U);                                                                                       \
    } while (0)

int kpo_cv_lane(const char *gp, uint64_t n_kmers, const uint64_t *kcell, const uint64_t *m, const uint64_t *u,
                int itype_bits, double alpha, double beta, double penalty, float *score, int nthreads) {
    kpo_lat L;
    if (lat_build(gp, &L)) return -1;
    for (uint64_t j = 0; j < n_kmers; ++j)
        if (kcell[j] >= L.npat) return -1;
    const float inf32 = (float)1e100;
    const int nt = nthreads > 0 ? nthreads : 1;
    /* low positions 0..t-1 (radix product B <= 4096), high = the rest */
    int t = 0;
    uint64_t B = 1;
    while (t < L.k && B * (uint64_t)L.radix[t] <= 4096) B *= (uint64_t)L.radix[t++];
    const uint64_t nhi = L.npat / B;
    int lomax = 0;
    for (int i = 0; i < t; ++i) lomax += L.lev[i][L.radix[i] - 1];
    uint64_t looff[KPO_MAXK * 3 + 2] = {0};
    uint32_t *lolist = (uint32_t *)malloc(sizeof(uint32_t) * B);
    uint8_t *hlev = (uint8_t *)malloc(nhi ? nhi : 1);
    uint8_t *lodig = (uint8_t *)malloc(B * (uint64_t)(t ? t : 1));
    if (!lolist || !hlev || !lodig) { free(lolist); free(hlev); free(lodig); return -2; }
    for (uint64_t x = 0; x < B; ++x) {
        uint64_t q = x;
        for (int i = 0; i < t; ++i) { lodig[x * t + i] = (uint8_t)(q % L.radix[i]); q /= L.radix[i]; }
    }
    for (uint64_t x = 0; x < B; ++x) {  /* low cells bucketed by low level, ascending */
        uint64_t q = x;
        int s = 0;
        for (int i = 0; i < t; ++i) { s += L.lev[i][q % L.radix[i]]; q /= L.radix[i]; }
        looff[s + 1]++;
    }
    for (int s = 0; s <= lomax; ++s) looff[s + 1] += looff[s];
    {
        uint64_t fill[KPO_MAXK * 3 + 2] = {0};
        for (uint64_t x = 0; x < B; ++x) {
            uint64_t q = x;
            int s = 0;
            for (int i = 0; i < t; ++i) { s += L.lev[i][q % L.radix[i]]; q /= L.radix[i]; }
            lolist[looff[s] + fill[s]++] = (uint32_t)x;
        }
    }
#pragma omp parallel for num_threads(nt) schedule(static)
    for (uint64_t h = 0; h < nhi; ++h) {
        uint64_t q = h;
        int s = 0;
        for (int i = t; i < L.k; ++i) { s += L.lev[i][q % L.radix[i]]; q /= L.radix[i]; }
        hlev[h] = (uint8_t)s;
    }
#pragma omp parallel for num_threads(nt) schedule(static)
    for (uint64_t n = 0; n < L.npat; ++n) score[n] = inf32;
    int rc = 0;
    if (itype_bits <= 32) KPO_LANE_BODY(uint32_t);
    else KPO_LANE_BODY(uint64_t);
    free(lolist);
    free(hlev);
    free(lodig);
    return rc;
}

/* the host C library's log / log1p over an array (fn 0 / 1): what numba's np.log / np.log1p
 * lower to and what scipy's xlogy / xlog1py multiply (oracle/treecheck.py's vectorised
 * single terms) */
void kpo_libm_array(const double *x, double *y, uint64_t n, int fn) {
    for (uint64_t i = 0; i < n; ++i) y[i] = fn ? log1p(x[i]) : log(x[i]);
}

/*
 * Fit DP (one fold, full data) with back-pointers.
 *   M, U      : [npat]; k-mer rows are inputs, the rest outputs.
 *   score     : [npat] float32 output, backtrack : [npat] output (c1 of the winning split,
 *               or the cell itself when it is kept whole), as Fit :46-49, :62-64.
 */
int kpo_fit(const char *gp, uint64_t *M, uint64_t *U, int itype_bits, double alpha, double beta,
            double penalty, float *score, uint64_t *backtrack, int nthreads) {
    kpo_lat L;
    if (lat_build(gp, &L)) return -1;
    const uint64_t mask = itype_bits >= 64 ? ~0ULL : ((1ULL << itype_bits) - 1);
    uint64_t off[KPO_MAXK * 3 + 2];
    uint64_t *ord = level_order(&L, off);
    if (!ord) return -2;
    const float inf32 = (float)1e100;
    const int nt = nthreads > 0 ? nthreads : 1;
#pragma omp parallel for num_threads(nt) schedule(static)
    for (uint64_t n = 0; n < L.npat; ++n) score[n] = inf32;
    /* level 0: score(M, U) (Fit :26-29, :106-114) */
#pragma omp parallel for num_threads(nt) schedule(static)
    for (uint64_t q = off[0]; q < off[1]; ++q) {
        uint64_t n = ord[q];
        double m = (double)M[n], u = (double)U[n];
        double p = (m + alpha) / (((double)(M[n] + U[n]) + alpha) + beta);
        score[n] = (float)(-2.0 * (xlogy_(m, p) + xlog1py_(u, -p)) + penalty);
        backtrack[n] = n;
    }
    /* levels >= 1: handle_pattern (Fit :31-64), one level after the other */
    for (int lev = 1; lev <= L.maxlev; ++lev)
#pragma omp parallel for num_threads(nt) schedule(static)
    for (uint64_t q = off[lev]; q < off[lev + 1]; ++q) {
        uint64_t n = ord[q];
        int first = 1;
        uint64_t rest = n;
        for (int i = 0; i < L.k; ++i) {
            int d = (int)(rest % L.radix[i]);
            rest /= L.radix[i];
            for (int j = 0; j < L.np[i][d]; ++j) {
                uint64_t base = n - (uint64_t)d * L.cg[i];
                uint64_t c1 = base + (uint64_t)L.pa[i][d][j] * L.cg[i];
                uint64_t c2 = base + (uint64_t)L.pb[i][d][j] * L.cg[i];
                float ns = score[c1] + score[c2];
                if (ns < score[n]) { score[n] = ns; backtrack[n] = c1; }
                if (first) {
                    M[n] = (M[c1] + M[c2]) & mask;
                    U[n] = (U[c1] + U[c2]) & mask;
                    first = 0;
                }
            }
        }
        uint64_t m = M[n], u = U[n];
        double p = ((double)m + alpha) / (((double)((m + u) & mask) + alpha) + beta);
        double s = penalty;
        if (m > 0) s += (-2.0 * (double)m) * log(p);
        if (u > 0) s += (-2.0 * (double)u) * log(1.0 - p);
        if (s < (double)score[n]) { score[n] = (float)s; backtrack[n] = n; }
    }
    free(ord);
    return 0;
}
