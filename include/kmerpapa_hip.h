/*
 * kmerpapa_hip.h -- C-ABI of the MI355X lattice-DP engine (libkmerpapa_hip.so).
 *
 * Plain C types only (no torch, no HIP types).  Every call returns KP_OK (0) or a
 * negative KP_E_* code; kp_last_error() gives the thread's last message.  Host buffers
 * are owned by the caller and only read (or written, for outputs) during the call.
 * Device memory is owned by the plan and cached across passes.
 *
 * What each entry point replaces in the reference (BesenbacherLab/kmerPaPa v0.2.4;
 * "CV" = src/kmerpapa/algorithms/bottum_up_array_penalty_plus_pseudo_CV.py,
 *  "Fit" = src/kmerpapa/algorithms/bottum_up_array_w_numba.py):
 *
 *   kp_plan_create   per-pattern globals and tables: CV :82-122, Fit :68-92;
 *                    pattern_utils.py pattern_max :587, get_cum_genpat_pos_level :237,
 *                    subpatterns_level_ord_np :513 (level order)
 *   kp_set_counts    level-0 rows of M_mem/U_mem written by
 *                    CV_tools.make_all_folds_contextD_patterns (CV :130) or by the Fit
 *                    level-0 loop (Fit :106-114), plus every aggregated row
 *                    (first-pair sums, CV :52-55 / Fit :50-53)
 *   kp_pass          the level sweep CV :143-157 (score_test_folds :15-20 and
 *                    handle_pattern :26-78 for every cell) and its root read-out
 *                    :158-163; with fold = -1 the Fit sweep Fit :106-120
 *   kp_fit_leaves    backtrack(gen_pat, ...) Fit :17-24, 121
 *   kp_counts_begin / kp_counts_fold   the same, one fold at a time
 *   kp_fold_split    CV_tools.py sample :5-27 and the fold loop of
 *                    make_all_folds_contextD_patterns :44-57 (host code, numpy legacy RNG);
 *                    kp_fold_sample: one fold of it (sample :5-27)
 *   kp_kmer_parse    io_utils.py read_dict :82-136 (with downsize_contextD's centring,
 *                    :50-79) and read_joint_kmer_counts :3-46 (host code)
 *   kp_format_long_rows  the -l rows of cli.py:301-316 (host code)
 */
#ifndef KMERPAPA_HIP_H
#define KMERPAPA_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define KP_OK 0
#define KP_E_ARG (-1)     /* bad argument (pattern, sizes, lane count)            */
#define KP_E_NOMEM (-2)   /* lattice x lanes does not fit device memory             */
#define KP_E_HIP (-3)     /* HIP runtime / launch failure                           */
#define KP_E_STATE (-4)   /* call order violated (e.g. kp_pass before kp_set_counts) */
#define KP_E_PARITY (-5)  /* internal consistency check failed (argmin tree broken) */

#define KP_GROUP_MAX_LANES 8

typedef struct kp_ctx kp_ctx;
typedef struct kp_plan kp_plan;

/* One (pseudo-count alpha, fold) group: n_lanes penalties share the fold's counts.
 * fold in [0, nf) = cross-validation on that fold (train = all other folds);
 * fold = -1      = fit on all data (the Fit module's DP). */
typedef struct {
    int32_t fold;
    int32_t n_lanes;
    double alpha;
    double beta;
    double penalty[KP_GROUP_MAX_LANES];
} kp_group;

typedef struct {
    uint64_t npat;        /* lattice cells = pattern_max(gen_pat)                  */
    uint64_t nblocks;     /* LDS blocks                                            */
    uint64_t n_kmers;     /* k-mers matching gen_pat                               */
    uint32_t block;       /* cells per block (low positions)                       */
    uint32_t block_pad;   /* row stride of a block lane                            */
    int32_t k, low_positions, max_level, high_levels;
    double pairs_total;   /* split pairs summed over all cells (SURVEY 8d "P")    */
    double pairs_high;    /* ... of which at high (gathered) positions             */
    uint64_t bytes_per_lane; /* device bytes per lane: f32 train score per cell
                                (value-only sweep) + backtrack node pool + leaves */
    uint32_t lanes_per_workgroup; /* lanes one sweep workgroup holds at the plan's count
                                     width (32-bit until counts are set): passes cut
                                     into pieces of this width run best */
    uint32_t pad_;
} kp_plan_info;

typedef struct {
    double dp_ms;         /* device time of the DP sweep kernels (HIP events)      */
    double backtrack_ms;  /* device time of the backtrack kernel                   */
    double total_ms;      /* host wall time of the whole kp_pass call              */
    uint64_t units;       /* cells x lanes scored in the pass                      */
    uint64_t dp_launches; /* kernel launches of the sweep                          */
    double alg_bytes;     /* algorithmic bytes of the pass (SURVEY 8d definition)  */
    double gather_bytes;  /* bytes the sweep gathers from HBM/L2 (high splits)     */
} kp_pass_stats;

const char *kp_last_error(void);
int kp_device_count(int *n);

int kp_create(int device, kp_ctx **out);
void kp_destroy(kp_ctx *ctx);
/* free / total device memory of the context's GPU (bytes) */
int kp_device_mem(kp_ctx *ctx, uint64_t *free_bytes, uint64_t *total_bytes);

/* max_block = 0 -> default LDS block budget (4096 cells). */
int kp_plan_create(kp_ctx *ctx, const char *gen_pat, uint32_t max_block, kp_plan **out);
void kp_plan_destroy(kp_plan *plan);
int kp_plan_get_info(const kp_plan *plan, kp_plan_info *out);
/* Host-only (no GPU): build the plan's tables on the host and report their info -- the
 * lattice size and device bytes per lane a job would need, before any device is touched. */
int kp_plan_host(const char *gen_pat, uint32_t max_block, kp_plan_info *out);
/* The same at count width itype_bytes (4 or 8, CV :94-97's itype): lanes_per_workgroup is
 * then the width kp_pass cuts device groups by on an MI355X (160 KiB of LDS per CU), the
 * group size a multi-GPU job deals whole to its ranks. */
int kp_plan_host_counts(const char *gen_pat, uint32_t max_block, int itype_bytes, kp_plan_info *out);
/* Checks of the block list (test hooks; no reference counterpart).  The device builds the
 * plan's block list (blocks by high level) from a closed-form rank rule.
 * kp_block_order_check, host-only: *mismatches = blocks whose closed-form slot differs from
 * the host's block walk.  kp_plan_block_check: *mismatches = entries of the plan's device
 * list that differ from the host walk. */
int kp_block_order_check(const char *gen_pat, uint32_t max_block, uint64_t *mismatches);
int kp_plan_block_check(kp_plan *plan, uint64_t *mismatches);

/* Upload fold counts of every k-mer: M, U are [n_kmers][nf] arrays of itype_bytes (4 or
 * 8) unsigned integers, k-mers in KmerEnumeration order (position 0 fastest, nucleotide
 * index = position in code[g]).  Builds the per-block k-mer-low count tables. */
int kp_set_counts(kp_plan *plan, const void *M, const void *U, uint64_t n_kmers, int nf, int itype_bytes);

/* The same tables fold by fold, so that passes can start while the host still draws the
 * later folds (the CV driver's pipelined fold split).  kp_counts_begin: M_all, U_all
 * [n_kmers] = counts of all data (the sum of the folds to come; the train counts of fold f
 * are all data minus fold f, CV :22-24); it discards any fold set before.
 * kp_counts_fold: M_fold, U_fold [n_kmers] = fold `fold`'s counts; asynchronous (the
 * counts are copied before it returns, the table fills on the plan's count stream, and
 * every later device read of it waits for that on the device), so it may be called from
 * another host thread while a kp_pass of another fold runs.  kp_pass refuses a group
 * whose fold has not been set (KP_E_STATE). */
int kp_counts_begin(kp_plan *plan, const void *M_all, const void *U_all, uint64_t n_kmers, int nf, int itype_bytes);
int kp_counts_fold(kp_plan *plan, int fold, const void *M_fold, const void *U_fold, uint64_t n_kmers);

/* One DP sweep of every lane of every group over the whole lattice.
 * Lanes are numbered group-major; per lane the outputs are the root's train score
 * (f32, as stored by the reference), the root's test -2LL (CV) and the number of
 * patterns of the optimal partition. */
int kp_pass(kp_plan *plan, const kp_group *groups, int n_groups, float *root_train, float *root_test,
            uint64_t *n_leaves);
int kp_last_pass_stats(const kp_plan *plan, kp_pass_stats *out);
/* Host-only (no GPU): the workgroups ("device groups") kp_pass would run `groups` as, with
 * `lanes_per_workgroup` lanes per workgroup (kp_plan_info): lane0[i] / nl[i] = first lane
 * and lanes of device group i (lanes numbered group-major), nl2[i] = its trailing lanes
 * that take a second (alpha, beta) (a mixed group of two same-fold groups; 0 = one alpha).
 * *n_out = number of device groups; at most cap entries are written. */
int kp_device_groups(const kp_group *groups, int n_groups, int lanes_per_workgroup, int32_t *lane0, int32_t *nl,
                     int32_t *nl2, int cap, int *n_out);
/* Tuning: with KP_LAUNCH_TIMES=1 in the environment, the device time (ms) of every sweep
 * launch of the last pass (lane classes in order, high levels ascending); *n = launches
 * (0 without the variable), at most cap written to ms. */
int kp_last_launch_ms(const kp_plan *plan, float *ms, int cap, int *n);

/* Allocate the per-lane device buffers (score rows, backtrack nodes) for `lanes` lanes now,
 * so that later passes of up to that many lanes allocate nothing.  Buffers only grow.
 * Re-allocating after a free is slow on MI355X (freed HBM is wiped first), so a job that
 * knows its largest pass should reserve it once.  KP_E_NOMEM if it does not fit.
 * (No reference counterpart: the reference allocates its [npat, nf] arrays per call, CV
 * :93-102.) */
int kp_reserve_lanes(kp_plan *plan, uint32_t lanes);

/* Leaves (cell indices) of lane `lane` of the last pass, in the reference's backtrack
 * order.  cap = capacity of `leaves`; *n_out = number of leaves. */
int kp_fit_leaves(kp_plan *plan, uint32_t lane, uint64_t *leaves, uint64_t cap, uint64_t *n_out);

/* Debug / parity: copy one lane's train scores and argmin codes, in cell-index order
 * ([npat] each; either pointer may be NULL). */
int kp_dump_lane(kp_plan *plan, uint32_t lane, float *score, uint8_t *code);

/* Debug / parity: the train scores of the cells cells[0..n) (cell indices < npat) of lane
 * `lane` of the last pass, into out[n] -- e.g. every cell of a sub-pattern embedded in a
 * full-size lattice, whose values depend only on its own sub-lattice. */
int kp_gather_cells(kp_plan *plan, uint32_t lane, const uint64_t *cells, uint64_t n, float *out);

/* Parity check of the device's float64 log (the log of the single-pattern term, CV :61-62 /
 * Fit :56-57; ROCm's ocml): y[i] = log(x[i]) computed on the context's GPU. */
int kp_math_log(kp_ctx *ctx, const double *x, double *y, uint64_t n);

/* Parity check of the C library's log / log1p as restated for the GPU (kp_libm.h: the
 * sweep's exact fallback, the backtrack and the k-mer terms): fn 1 = log, 2 = log1p
 * (fn 0 = the device's own log, as kp_math_log; fn 3 = kp_fast_log, the table-free fdlibm
 * log; fn 4 = kp_fma_log, its FMA / hardware-reciprocal form), computed on the context's GPU. */
int kp_math_libm(kp_ctx *ctx, const double *x, double *y, uint64_t n, int fn);

/* --score all_kmers on the context's GPU: one rate per k-mer, no lattice DP
 * (src/kmerpapa/algorithms/all_kmers_CV.py: test_folds :8-13 and the k-mer loop :36-46).
 * M, U: [n][nf] uint64 fold counts, rows in the reference's matches(gen_pat) order; per
 * alpha a (alphas[na]) and fold f, with betas[a][f] (get_betas of the fold-train totals):
 *   sum_train[a][f] = sum over rows i of test_folds(trM, trU, trM, trU, alpha_a, beta_af)
 *   sum_test[a][f]  = sum over rows i of test_folds(trM, trU, M[i][f], U[i][f], alpha_a, beta_af)
 * trM = sum_g M[i][g] - M[i][f] (likewise trU); each sum in float64, row by row from 0.0,
 * as the reference's `sum_train += ...` loop; xlogy / xlog1py with the C library's logs. */
int kp_allkmers_cv(kp_ctx *ctx, const uint64_t *M, const uint64_t *U, uint64_t n, int nf, const double *alphas,
                   const double *betas, int na, double *sum_train, double *sum_test);

/* Host-only (no GPU needed): the cross-validation fold split of CV_tools.py
 * make_all_folds_contextD_patterns :44-57 / sample :5-27 with numpy's legacy
 * RandomState stream.  mt_key[624] / *mt_pos = the MT19937 state of the caller's
 * RandomState (RandomState.get_state()[1:3]), advanced in place exactly as numpy would.
 * colors[n] = ball counts per colour; folds[n][nf] receives each colour's fold counts
 * (folds 0..nf-2 sampled, the last takes the remainder). */
int kp_fold_split(uint32_t *mt_key, int32_t *mt_pos, const uint64_t *colors, uint64_t n, int nf, uint64_t *folds);
/* One fold of that split: CV_tools.py sample :5-27 (m balls drawn colour by colour from
 * colors[n]; out[n] = the balls drawn of each colour), same RNG state convention. */
int kp_fold_sample(uint32_t *mt_key, int32_t *mt_pos, const uint64_t *colors, uint64_t n, uint64_t m,
                   uint64_t *out);

/* k-mer count text (host code, no GPU).  Parses `nbytes` of file text into a table of
 * unique k-mers as 2-bit codes (A=0 C=1 G=2 T=3, first letter most significant: code
 * order = sorted k-mer order) with counts:
 *   columns = 2: "kmer count" lines (io_utils.read_dict :82-136).  Counts of equal k-mers
 *     are summed into c0 (c1 = 0); total0 = sum of kept counts.  length > 0 keeps the
 *     central `length` letters (width//2 - length//2 ...); with a super pattern and
 *     length <= 0 the pattern's length is used.  Negative counts are an error.
 *   columns = 3: "kmer positive background" lines (read_joint_kmer_counts :3-46).  The
 *     last line of a k-mer wins: c0 = positive, c1 = background - positive (an error if
 *     negative); total0 = n_negative_total, total1 = n_positive_total over every kept line.
 * super_pattern (IUPAC, may be NULL or "") keeps only matching k-mers.  Lines whose k-mer
 * has a letter other than A/C/G/T are skipped; a line with the wrong number of tokens,
 * a bad count or k-mers of different lengths is KP_E_ARG with kp_last_error() text. */
typedef struct kp_kmer_table kp_kmer_table;
int kp_kmer_parse(const char *text, uint64_t nbytes, int columns, const char *super_pattern, int length,
                  kp_kmer_table **out);
int kp_kmer_table_info(const kp_kmer_table *t, uint64_t *n, int32_t *k, int64_t *total0, int64_t *total1);
/* codes[n], c0[n], c1[n]: caller-allocated (n from kp_kmer_table_info) */
int kp_kmer_table_copy(const kp_kmer_table *t, uint64_t *codes, int64_t *c0, int64_t *c1);
void kp_kmer_table_free(kp_kmer_table *t);

/* The long output table (host code, no GPU): cli.py:301-316 with -l prints, for every k-mer
 * of every pattern, f"{context} {c_neg} {c_pos} {c_rate}" + the pattern's tail
 * " {pattern} {p_neg} {p_pos} {p_rate}\n", c_rate = c_pos / (c_pos + c_neg) as Python's
 * repr() writes a float.  kmers: n * k letters; pid[i] = row i's tail; tail t is
 * tails[tail_off[t] .. tail_off[t + 1]).  Writes at most cap bytes to out, *out_len = bytes
 * written.  KP_E_ARG if cap is too small or a row has c_pos + c_neg == 0 (where Python
 * raises ZeroDivisionError). */
int kp_format_long_rows(const char *kmers, int k, const int64_t *c_neg, const int64_t *c_pos, const uint32_t *pid,
                        uint64_t n, const char *tails, const uint64_t *tail_off, uint64_t n_tails, char *out,
                        uint64_t cap, uint64_t *out_len);
/* Python repr() of x[0..n), one per line (the float format of kp_format_long_rows). */
int kp_py_repr(const double *x, uint64_t n, char *out, uint64_t cap, uint64_t *out_len);

#ifdef __cplusplus
}
#endif
#endif
