// kp_core.h -- data layout and per-item arithmetic of the blocked lattice DP.
//
// Shared by the gfx950 kernels (kp_hip.hip) and by the host-side test emulator
// (tests/emu/kp_emu.hip), both compiled by hipcc.  Everything here is plain
// __host__ __device__ code: no launches, no LDS declarations.
//
// The recurrence is the reference's (src/kmerpapa/algorithms/
// bottum_up_array_penalty_plus_pseudo_CV.py handle_pattern :26-78 and
// bottum_up_array_w_numba.py handle_pattern :31-64); the layout is ours:
//
//   cell index  n = l + B * h        l = low part (positions 0..t-1), h = high part
//   S[h][lane][Bpad]  f32  train score of cell (h,l) for one lane (lane = one penalty of
//                          one (alpha, fold) group)
//   C[h][lane][Bpad]  u8   argmin code: (position << 3) | pair, or KP_SINGLE
//   K[nf+1][q][kl][2] CT   counts (M, U) of the block's k-mer-low cells kl; slot 0 = all
//                          data (the sum over folds), slot 1 + f = fold f (slot-major, so a
//                          fold's table is filled and read with contiguous rows); rows in
//                          the plan's block-list order q (the sweep's workgroup knows q
//                          before it has loaded its block h; kpos[h] = q)
//
// Tie rule: the reference scans positions 0..k-1, pairs in table order, with a strict
// "<" starting from +inf, then the single-pattern term with a strict "<" in float64.
// The scan is split here into (low positions, in LDS) and (high positions, gathered);
// low positions come first in scan order, so the low winner beats the high winner on
// equal value.  NaN candidates never win, exactly as with the sequential scan.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "kp_libm.h"

#define KP_MAXK 16          // pattern length limit (15^16 cells is far beyond any HBM)
#define KP_MAXT 8           // low positions per block
#define KP_GROUP_LANES 8    // penalties per (alpha, fold) group
#define KP_SINGLE 0xFFu     // argmin code: keep the cell as one pattern
#define KP_NONE 0xFEu       // argmin code: no candidate (only +inf/NaN seen)
#define KP_MAX_HPAIRS 128   // high split pairs of one block (<= (k-t) * 7)
#define KP_MAXDEPTH (3 * KP_MAXK + 2)

// per position: for every digit its level, number of split pairs and the digit pairs
struct kp_postab {
    uint8_t lev[16];
    uint8_t np[16];
    uint8_t pa[16][8];
    uint8_t pb[16][8];
};

// one (alpha, fold) group of lanes; fold < 0 = fit mode (train counts = all data).  A
// mixed group (nl2 > 0) holds the lanes of two user groups of the same fold: its last nl2
// lanes take (alpha2, beta2) -- the count tables are shared, only the logs differ
struct kp_group_dev {
    int32_t fold;
    int32_t lane0;
    int32_t nl;
    int32_t nl2;
    double alpha;
    double beta;
    double pen[KP_GROUP_LANES];
    double alpha2;
    double beta2;
};

// (alpha, beta) of lane j (0-based inside the group)
__host__ __device__ inline bool kp_lane_set2(const kp_group_dev &G, int j) { return j >= G.nl - G.nl2; }
__host__ __device__ inline double kp_lane_alpha(const kp_group_dev &G, int j) {
    return kp_lane_set2(G, j) ? G.alpha2 : G.alpha;
}
__host__ __device__ inline double kp_lane_beta(const kp_group_dev &G, int j) {
    return kp_lane_set2(G, j) ? G.beta2 : G.beta;
}

// lattice geometry, passed by value to every kernel
struct kp_geom {
    int k, t, kh;          // positions, low positions, high positions
    int nf;                // folds held in K (nf + 1 slots per k-mer-low cell, slot 0 = all data)
    uint32_t B, Bpad;      // cells per block, padded row length (multiple of 32: 128-byte rows)
    uint32_t n_kl;         // k-mer-low cells per block
    uint32_t Ltot;         // lanes held in S / C
    uint64_t nblocks;      // number of blocks = npat / B
    uint32_t r[KP_MAXK];   // radix of every position
    uint32_t n[KP_MAXK];   // nucleotides of every position's general code
    uint64_t cgl[KP_MAXK]; // global place value of every position (cell index units)
    uint64_t hcg[KP_MAXK]; // place value of high position i (block index units)
    uint64_t khw[KP_MAXK]; // k-mer index weight of high position i
};

struct kp_cnt {
    uint64_t mtr, utr, mte, ute;  // train / test counts of one cell for one fold
};

struct kp_hpair {
    uint64_t h1, h2;  // child blocks
    uint32_t code;    // argmin code of this split
    uint32_t pad_;
};

// one low cell in level order: what the level phase needs, in one 16-byte load
struct kp_lowdesc {
    uint32_t l;      // low cell index inside the block (a whole word: the kernel uses it as loaded)
    uint16_t kl;     // k-mer-low index (k-mer-low cells only)
    uint16_t pad_;
    uint32_t info;   // packed low digits (4 bits per position)
    uint32_t pl;     // low split pairs: (first 4-pair chunk in kp_plan's lpairs) << 8 | count
};

// a block's high split pair (child blocks h - d1 and h - d2, at high position pos) as one
// word of the plan's hpd table (d1, d2 < 2^29 blocks)
__host__ __device__ inline uint64_t kp_hpd_word(uint64_t d1, uint64_t d2, uint32_t pos) {
    return d1 | (d2 << 29) | ((uint64_t)pos << 58);
}

// ---------------------------------------------------------------------------
// scoring arithmetic (float64, order of operations as in the reference)
// ---------------------------------------------------------------------------

// scipy.special.xlogy / xlog1py: 0 when x == 0 and y is not NaN; the logs are the C
// library's (kp_libm.h), as scipy's are
__host__ __device__ inline double kp_xlogy(double x, double y) {
    return (x == 0.0 && y == y) ? 0.0 : x * kp_libm_log(y);  // y == y: not NaN
}
__host__ __device__ inline double kp_xlog1py(double x, double y) {
    return (x == 0.0 && y == y) ? 0.0 : x * kp_libm_log1p(y);
}

// p = (M_tr + a) / (M_tr + U_tr + a + beta), summed left to right (CV :60, Fit :56)
__host__ __device__ inline double kp_rate(const kp_cnt &c, double a, double b) {
    return ((double)c.mtr + a) / (((double)(c.mtr + c.utr) + a) + b);
}

// k-mer cell: -2*(xlogy(M,p) + xlog1py(U,-p)) + c  (CV score_test_folds :15-20, Fit score :26-29)
__host__ __device__ inline float kp_kmer_train(const kp_cnt &c, double a, double b, double pen) {
    double p = kp_rate(c, a, b);
    return (float)(-2.0 * (kp_xlogy((double)c.mtr, p) + kp_xlog1py((double)c.utr, -p)) + pen);
}
__host__ __device__ inline float kp_kmer_test(const kp_cnt &c, double a, double b) {
    double p = kp_rate(c, a, b);
    return (float)(-2.0 * (kp_xlogy((double)c.mte, p) + kp_xlog1py((double)c.ute, -p)));
}

// level >= 1 single-pattern term: c + (-2 M) log p + (-2 U) log(1-p)  (CV :63-70, Fit :56-61)
__host__ __device__ inline double kp_single_train(const kp_cnt &c, double logp, double log1mp, double pen) {
    double s = pen;
    if (c.mtr > 0) s += (-2.0 * (double)c.mtr) * logp;
    if (c.utr > 0) s += (-2.0 * (double)c.utr) * log1mp;
    return s;
}
// matching test -2LL (CV :73-78)
__host__ __device__ inline float kp_single_test(const kp_cnt &c, double logp, double log1mp) {
    double s = 0.0;
    if (c.mte > 0) s += (-2.0 * (double)c.mte) * logp;
    if (c.ute > 0) s += (-2.0 * (double)c.ute) * log1mp;
    return (float)s;
}

// ---------------------------------------------------------------------------
// counts
// ---------------------------------------------------------------------------

// count slots in K (all data + one per fold) and the elements of one slot
__host__ __device__ inline uint32_t kp_kslots(const kp_geom &g) { return (uint32_t)g.nf + 1u; }
__host__ __device__ inline uint64_t kp_kslot_elems(const kp_geom &g) { return g.nblocks * (uint64_t)g.n_kl * 2; }

// counts of one k-mer-low cell of the block whose count rows are row krow of K (on the
// device the block's position in the plan's block list, kp_dev_tables.kpos) for group
// fold f (f < 0: fit mode)
template <typename CT>
__host__ __device__ inline kp_cnt kp_kl_counts(const kp_geom &g, const CT *K, uint64_t krow, uint32_t kl, int fold) {
    const CT *row = K + (krow * g.n_kl + kl) * 2;
    const uint64_t sm = (uint64_t)row[0], su = (uint64_t)row[1];
    kp_cnt c;
    if (fold < 0) {
        c.mtr = sm; c.utr = su; c.mte = 0; c.ute = 0;
    } else {
        const CT *fr = row + kp_kslot_elems(g) * (uint64_t)(1 + fold);
        c.mte = (uint64_t)fr[0];
        c.ute = (uint64_t)fr[1];
        c.mtr = sm - c.mte;  // get_train (CV :22-24, :56-59): all data minus the fold
        c.utr = su - c.ute;
    }
    return c;
}

// ---------------------------------------------------------------------------
// digits
// ---------------------------------------------------------------------------

__host__ __device__ inline uint32_t kp_low_digit(uint32_t lowinfo, int i) { return (lowinfo >> (4 * i)) & 15u; }

// digit of high position i (0-based among high positions) of block h
__host__ __device__ inline uint32_t kp_high_digit(const kp_geom &g, uint64_t h, int i) {
    return (uint32_t)((h / g.hcg[i]) % g.r[g.t + i]);
}

// ordered list of the split pairs at high positions of block h (scan order)
__host__ __device__ inline int kp_high_pairs(const kp_geom &g, const kp_postab *tabs, uint64_t h, kp_hpair *out) {
    int np = 0;
    for (int i = 0; i < g.kh; ++i) {
        const kp_postab &T = tabs[g.t + i];
        uint32_t d = kp_high_digit(g, h, i);
        for (int j = 0; j < T.np[d]; ++j) {
            out[np].h1 = h + ((uint64_t)T.pa[d][j] - d) * g.hcg[i];  // a < d, unsigned wrap is exact
            out[np].h2 = h + ((uint64_t)T.pb[d][j] - d) * g.hcg[i];
            out[np].code = (uint32_t)(((g.t + i) << 3) | j);
            ++np;
        }
    }
    return np;
}

__host__ __device__ inline int kp_high_pair_count(const kp_geom &g, const kp_postab *tabs, uint64_t h) {
    int np = 0;
    for (int i = 0; i < g.kh; ++i) np += tabs[g.t + i].np[kp_high_digit(g, h, i)];
    return np;
}

__host__ __device__ inline int kp_high_level(const kp_geom &g, const kp_postab *tabs, uint64_t h) {
    int s = 0;
    for (int i = 0; i < g.kh; ++i) s += tabs[g.t + i].lev[kp_high_digit(g, h, i)];
    return s;
}

// the block order of kp::build_plan (high positions perm[0] fastest) in closed form
struct kp_blockgen {
    int hs;                 // high level sums 0 .. hs - 1
    int8_t perm[KP_MAXK];   // high positions, fastest first
};

// Slot of block h in the plan's block list (blocks by high level, each level in the
// mixed-radix order of perm) from build_plan's rank table brank[kh][16][hs] and level
// offsets hoff; *hd / *hn = the block's packed high digits (4 bits) and split-pair counts
// (3 bits per high position).  nblocks < 2^32 (build_plan), so 32-bit divisions suffice.
__host__ __device__ inline uint64_t kp_block_slot(const kp_geom &g, const kp_postab *tabs, const kp_blockgen &bg,
                                                  const uint32_t *brank, const uint64_t *hoff, uint64_t h,
                                                  uint64_t *hd, uint64_t *hn) {
    uint32_t dig[KP_MAXK];
    uint32_t s = 0;
    uint64_t w = 0, n = 0;
    for (int i = 0; i < g.kh; ++i) {
        const uint32_t d = ((uint32_t)h / (uint32_t)g.hcg[i]) % g.r[g.t + i];
        const kp_postab &T = tabs[g.t + i];
        dig[i] = d;
        s += T.lev[d];
        w |= (uint64_t)d << (4 * i);
        n |= (uint64_t)T.np[d] << (3 * i);
    }
    uint64_t rank = 0;
    uint32_t above = 0;
    for (int j = g.kh - 1; j >= 0; --j) {
        const int i = bg.perm[j];
        rank += brank[((uint32_t)j * 16u + dig[i]) * (uint32_t)bg.hs + (s - above)];
        above += tabs[g.t + i].lev[dig[i]];
    }
    *hd = w;
    *hn = n;
    return hoff[s] + rank;
}

// is cell (h, l) a k-mer (every digit a nucleotide)?
__host__ __device__ inline bool kp_is_kmer(const kp_geom &g, uint64_t h, uint32_t lowinfo) {
    for (int i = 0; i < g.t; ++i)
        if (kp_low_digit(lowinfo, i) >= g.n[i]) return false;
    for (int i = 0; i < g.kh; ++i)
        if (kp_high_digit(g, h, i) >= g.n[g.t + i]) return false;
    return true;
}

__host__ __device__ inline uint64_t kp_lane_row(const kp_geom &g, uint64_t h, uint32_t lane) {
    return (h * g.Ltot + lane) * (uint64_t)g.Bpad;
}

// float64 single-pattern context of one cell, shared by every lane of a group
struct kp_single_ctx {
    bool kmer;      // level-0 cell: reference uses the xlogy formula and no splits
    double logp, log1mp;
    kp_cnt c;
    bool exact;     // every cell takes the C library's logs (KP_EXACT_LOGS=1, or !kp_fast_logs_ok)
    // mixed groups only (the MIX instantiations): lanes j >= js take the second set
    int js;
    double a2, b2, logp2, log1mp2;
};

// ---------------------------------------------------------------------------
// pair words: everything the level phase needs about the splits of one digit at one low
// position, in one 64-bit load.  bits 8p..8p+3 = d - pa[d][p], bits 8p+4..8p+7 =
// d - pb[d][p] (p < np <= 7, scan order), bits 56..63 = np.  Child of pair p at low
// position i of cell l: l - delta * cgl[i].
// ---------------------------------------------------------------------------
__host__ __device__ inline uint64_t kp_pair_word(const kp_postab &T, uint32_t d) {
    uint64_t w = (uint64_t)T.np[d] << 56;
    for (uint32_t p = 0; p < T.np[d]; ++p)
        w |= (uint64_t)(((d - T.pa[d][p]) & 15u) | (((d - T.pb[d][p]) & 15u) << 4)) << (8 * p);
    return w;
}

// 24-bit multiply (operands known < 2^24: one full-rate v_mul_u32_u24 on gfx950)
__host__ __device__ inline uint32_t kp_mul24(uint32_t a, uint32_t b) { return (a & 0xFFFFFFu) * (b & 0xFFFFFFu); }

// ---------------------------------------------------------------------------
// VALUE-ONLY DP.  A cell's stored float32 score is min(best split, single term) and does
// not depend on which candidate achieved it, so the sweep keeps values only and the
// argmin (with the reference's first-wins tie rule) is recomputed for the few cells of
// the optimal tree at backtrack time (kp_cell_decide).  Split candidates combine with
// fminf: it ignores NaN exactly as "v < best" does, and every score is >= +0 (no -0).
// ---------------------------------------------------------------------------

// min over NP split pairs of one low position for W lanes starting at lane j0 (lane
// stride NL); all 2*NP*W LDS reads issue before the first min (fully unrolled)
template <int NL, int W, int NP, typename SP>
__host__ __device__ inline void kp_pairs_minv(SP st, uint32_t l, uint32_t cg, uint64_t w, uint32_t j0, float *lmin) {
    float va[NP][W], vb[NP][W];
    const uint32_t w0 = (uint32_t)w, w1 = (uint32_t)(w >> 32);
#pragma unroll
    for (int p = 0; p < NP; ++p) {
        const uint32_t wp = (p < 4) ? (w0 >> (8 * p)) : (w1 >> (8 * (p - 4)));
        const uint32_t l1 = l - kp_mul24(wp & 15u, cg);
        const uint32_t l2 = l - kp_mul24((wp >> 4) & 15u, cg);
#pragma unroll
        for (int j = 0; j < W; ++j) {
            va[p][j] = st[l1 * NL + j0 + j];
            vb[p][j] = st[l2 * NL + j0 + j];
        }
    }
#pragma unroll
    for (int p = 0; p < NP; ++p)
#pragma unroll
        for (int j = 0; j < W; ++j) lmin[j] = fminf(lmin[j], va[p][j] + vb[p][j]);
}

// Float32 stores that cannot depend on the last bit of a float64 log.  The sweep takes its
// logs from the device's own log (ROCm ocml: within 1 ulp of the C library's,
// test_device_log_vs_libm), cheaper in this kernel than the C library's algorithm.  A
// single-pattern term s = c + (-2 M) log p + (-2 U) log(1-p) reaches the store only as
// float32(s) when s < best (otherwise the stored value is best, and then a nearby s rounds
// to best as well); so the result equals the C library's unless s lies close to a float32
// rounding midpoint.  Premise (kp_fast_logs_ok): c, alpha, beta >= 0, so every term is >= 0
// and s is exactly 0 or a float32 normal (the smallest nonzero s is ~ min(beta, 1/total) >>
// 2^-126).  Then a 2-ulp difference of the two logs moves s by less than 2.5 x 2^-51 |s|
// through the reference's three float64 operations, i.e. by fewer than 11 units in the last
// place of s, and the float32 rounding midpoints are the float64 values whose low 29
// mantissa bits are 2^28.  kp_store_unsafe flags an s whose low 29 bits are within 64
// units of 2^28 (s = 0 never is); a cell with a flagged lane recomputes its logs with the C
// library's algorithm (kp_libm_log, out of line) -- about 2.4e-7 of the lanes.  Groups
// outside the premise take that path for every cell (kp_single_ctx.exact).
__host__ __device__ inline bool kp_store_unsafe(double s) {
    const uint32_t lo = (uint32_t)__builtin_bit_cast(uint64_t, s);
    return ((lo + 64u) & 0x1FFFFF80u) == 0x10000000u;
}

// The reference's store of a single-pattern term (CV :71-72): `if s < best: best = f32(s)`,
// s float64, best float32.  Rounding to nearest is monotone, so f32(s) <= best exactly when
// s < best or f32(s) == best, and min(f32(s), best) is that same store in one float32 min
// (no float64 compare); a NaN s drops out of fminf as it fails the compare (best is never
// NaN: split candidates enter through fminf too, and every score is >= +0).
__host__ __device__ inline float kp_store_min(double s, float best) { return fminf((float)s, best); }

// the fast path's premise (kp_store_unsafe): penalties, alpha and beta not negative, and
// beta either 0 or not so small that a single term could fall below float32's normal range
__host__ __device__ inline bool kp_fast_logs_ok(const double *pen, int n, double alpha, double beta) {
    bool ok = alpha >= 0.0 && alpha < 1e30 && (beta == 0.0 || (beta >= 1e-30 * (1.0 + alpha) && beta < 1e30));
    for (int j = 0; j < n; ++j) ok = ok && pen[j] >= 0.0 && pen[j] < 1e30;
    return ok;
}

// a cell's final score per lane: min(best split, single term).  MIX: lanes j0 + j >= sc.js
// take the second (alpha, beta) set (sc.logp2 / sc.log1mp2; sc.a2 / sc.b2)
template <int W, bool MIX = false, typename SP>
__host__ __device__ inline void kp_cell_store(SP row, const float *lmin, const kp_single_ctx &sc, const double *pen,
                                              double alpha, double beta, uint32_t j0 = 0) {
    float out[W];
    bool unsafe = sc.exact;
    if (MIX) {  // one loop, each lane's term computed once (A/B: 1-2 ms faster per mixed pass)
#pragma unroll
        for (int j = 0; j < W; ++j) {
            const bool s2 = (int)(j0 + j) >= sc.js;
            const double s = kp_single_train(sc.c, s2 ? sc.logp2 : sc.logp, s2 ? sc.log1mp2 : sc.log1mp, pen[j]);
            out[j] = kp_store_min(s, lmin[j]);
            unsafe = unsafe || kp_store_unsafe(s);
        }
    } else {
#pragma unroll
        for (int j = 0; j < W; ++j) {
            const bool s2 = MIX && (int)(j0 + j) >= sc.js;
            const double s = kp_single_train(sc.c, s2 ? sc.logp2 : sc.logp, s2 ? sc.log1mp2 : sc.log1mp, pen[j]);
            out[j] = kp_store_min(s, lmin[j]);  // the float64 compare against the float32 store (CV :71)
        }
#pragma unroll
        for (int j = 0; j < W; ++j) {  // (every lane, stored or not: cheaper than telling them apart)
            const bool s2 = MIX && (int)(j0 + j) >= sc.js;
            unsafe = unsafe || kp_store_unsafe(kp_single_train(sc.c, s2 ? sc.logp2 : sc.logp,
                                                               s2 ? sc.log1mp2 : sc.log1mp, pen[j]));
        }
    }
    if (__builtin_expect(unsafe, 0)) {  // the C library's logs (rare; laid out away from the hot path)
        const double p = kp_rate(sc.c, alpha, beta);
        const double lp = kp_libm_log(p), l1p = kp_libm_log(1.0 - p);
        double lp2 = lp, l1p2 = l1p;
        if (MIX && (int)(j0 + W) > sc.js) {
            const double p2 = kp_rate(sc.c, sc.a2, sc.b2);
            lp2 = kp_libm_log(p2);
            l1p2 = kp_libm_log(1.0 - p2);
        }
#pragma unroll
        for (int j = 0; j < W; ++j) {
            const bool s2 = MIX && (int)(j0 + j) >= sc.js;
            float best = lmin[j];
            const double v = kp_single_train(sc.c, s2 ? lp2 : lp, s2 ? l1p2 : l1p, pen[j]);
            best = kp_store_min(v, best);
            out[j] = best;
        }
    }
#pragma unroll
    for (int j = 0; j < W; ++j) row[j] = out[j];
}

// one DP cell for lanes j0 .. j0+W-1 of the NL lanes interleaved in LDS
// (st[cell * NL + lane]); st[l] holds the best high-position split gathered from HBM.
// pw = pair words [t][16]; pen = the W penalties of those lanes.  W = NL is the normal
// mode (one thread per cell); W = 1 splits a cell's lanes over threads when a level has
// few cells (shorter dependent chains on the narrow top levels of a block).
template <int NL, int W, typename SP, typename WP>
__host__ __device__ inline void kp_dp_cell_values(const kp_geom &g, WP pw, uint32_t l, uint32_t lowinfo, SP st,
                                                  const kp_single_ctx &sc, double alpha, double beta,
                                                  const double *pen, uint32_t j0 = 0) {
    SP row = st + l * NL + j0;
    if (__builtin_expect(sc.kmer, 0)) {  // level 0 (CV :145-151 / Fit :106-114)
#pragma unroll
        for (int j = 0; j < W; ++j) row[j] = kp_kmer_train(sc.c, alpha, beta, pen[j]);
        return;
    }
    float lmin[W];
#pragma unroll
    for (int j = 0; j < W; ++j) lmin[j] = row[j];
    uint64_t w[KP_MAXT];
#pragma unroll
    for (int i = 0; i < KP_MAXT; ++i) w[i] = (i < g.t) ? pw[i * 16 + kp_low_digit(lowinfo, i)] : 0;
    // np is 0, 1, 3 or 7 for every IUPAC code and, because cells of a wave share their
    // split signature (kp_plan.h), nearly always wave-uniform
#pragma unroll
    for (int i = 0; i < KP_MAXT; ++i) {
        if (i >= g.t) continue;
        const uint32_t np = (uint32_t)(w[i] >> 56);
        const uint32_t cg = (uint32_t)g.cgl[i] & 0xFFFFu;  // low place values are < 2^16 (block <= 65535)
        if (np == 1) {
            kp_pairs_minv<NL, W, 1>(st, l, cg, w[i], j0, lmin);
        } else if (np == 3) {
            kp_pairs_minv<NL, W, 3>(st, l, cg, w[i], j0, lmin);
        } else if (np == 7) {
            kp_pairs_minv<NL, W, 7>(st, l, cg, w[i], j0, lmin);
        } else {
            for (uint32_t p = 0; p < np; ++p) {  // not produced by the IUPAC tables; kept general
                const uint32_t l1 = l - (uint32_t)((w[i] >> (8 * p)) & 15u) * cg;
                const uint32_t l2 = l - (uint32_t)((w[i] >> (8 * p + 4)) & 15u) * cg;
#pragma unroll
                for (int j = 0; j < W; ++j)
                    lmin[j] = fminf(lmin[j], st[l1 * NL + j0 + j] + st[l2 * NL + j0 + j]);
            }
        }
    }
    kp_cell_store<W>(row, lmin, sc, pen, alpha, beta);
}

// Pair-list decode of the SDWA builds (kp_sdwa_on): the byte offset K * (half HI of a
// pair-list word) = c * NL * 4 for a child cell c is one v_mul_u32_u24 whose source
// operand selects the 16-bit half, and the LDS read takes it as its address (the dynamic
// LDS array starts at address 0: the kernels declare no static LDS, checked at launch,
// kp_hip.hip launch_dp_hz).  The plain form (mask or shift, multiply-add, add of the array
// base) costs 3 VALU per child instead of 1.  Per build, as measured
// (profiles/r04/experiments/sdwa_ab.txt): 1 lane 111.5 -> 109.1 ms, 3 lanes 251 -> 243,
// mixed 5 lanes 402 -> 399; 5 lanes unchanged, 4 lanes 311 -> 326 (register allocation).
// Bit NL of the mask = the NL-lane build, bit 0 = the mixed builds.
#ifndef KP_SDWA_MASK
#define KP_SDWA_MASK 0x0Fu  // mixed, 1, 2, 3 lanes
#endif
template <int NL, bool MIX>
__host__ __device__ constexpr bool kp_sdwa_on() {
    return ((KP_SDWA_MASK >> (MIX ? 0 : NL)) & 1u) != 0;
}

template <uint32_t K, int HI>
__host__ __device__ inline uint32_t kp_half_mul(uint32_t e) {
#if defined(__HIP_DEVICE_COMPILE__)
    static_assert(K <= 64, "inline constant");
    uint32_t r;
    if constexpr (HI)
        asm("v_mul_u32_u24_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:DWORD"
            : "=v"(r) : "v"(e), "i"(K));
    else
        asm("v_mul_u32_u24_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_0 src1_sel:DWORD"
            : "=v"(r) : "v"(e), "i"(K));
    return r;
#else
    return (HI ? e >> 16 : e & 0xFFFFu) * K;
#endif
}

// the float at byte offset off of the LDS row array (device: LDS address off) / of a
// host array st
#if defined(__HIP_DEVICE_COMPILE__)
__device__ inline float kp_at_bytes(__attribute__((address_space(3))) float *, uint32_t off) {
    return *(__attribute__((address_space(3))) float *)(uintptr_t)off;
}
#endif
template <typename SP>
__host__ __device__ inline float kp_at_bytes(SP st, uint32_t off) { return st[off / 4u]; }

// min over one 4-pair chunk of a cell's split-pair list (c1 | c2 << 16 per pair, kp_plan.h
// lpairs) for W lanes from j0; all 8*W LDS reads issue before the first min
// KP_CHUNK_SPLIT: builds whose threads scan W >= KP_CHUNK_SPLIT lanes run a 4-pair chunk as
// two 2-pair halves (4*W LDS values in flight instead of 8*W; the same minima in the same
// order): 5 lanes 374.6 -> 373.9 ms, mixed 2 + 3 lanes 396.9 -> 395.7, 4 lanes (not split)
// 308.6 -> 309.5 with it (profiles/r04/experiments/chunk_split_ab.txt)
#ifndef KP_CHUNK_SPLIT
#define KP_CHUNK_SPLIT 5
#endif
template <int NL, int W, int NPC = 4, bool SDWA = false, typename SP>
__host__ __device__ inline void kp_chunk_minv(SP st, const uint4 c, uint32_t j0, float *lmin) {
    if constexpr (NPC == 4 && W >= KP_CHUNK_SPLIT) {
        kp_chunk_minv<NL, W, 2, SDWA>(st, c, j0, lmin);
        kp_chunk_minv<NL, W, 2, SDWA>(st, make_uint4(c.z, c.w, c.z, c.w), j0, lmin);
        return;
    }
    const uint32_t e[4] = {c.x, c.y, c.z, c.w};
    float va[4][W], vb[4][W];
#pragma unroll
    for (int p = 0; p < NPC; ++p) {
        if constexpr (SDWA) {
            const uint32_t o1 = kp_half_mul<4u * NL, 0>(e[p]), o2 = kp_half_mul<4u * NL, 1>(e[p]);
#pragma unroll
            for (int j = 0; j < W; ++j) {
                va[p][j] = kp_at_bytes(st, o1 + 4u * (j0 + j));
                vb[p][j] = kp_at_bytes(st, o2 + 4u * (j0 + j));
            }
        } else {
            const uint32_t c1 = e[p] & 0xFFFFu, c2 = e[p] >> 16;
#pragma unroll
            for (int j = 0; j < W; ++j) {
                va[p][j] = st[c1 * NL + j0 + j];
                vb[p][j] = st[c2 * NL + j0 + j];
            }
        }
    }
#pragma unroll
    for (int p = 0; p < NPC; ++p)
#pragma unroll
        for (int j = 0; j < W; ++j) lmin[j] = fminf(lmin[j], va[p][j] + vb[p][j]);
}

#define KP_PRE_CHUNKS 4  // pair-list chunks a thread loads ahead (16 pairs; longer lists load the rest on use)

// The same cell from its flat split-pair list (the sweep kernel's form): npairs pairs in
// 4-pair chunks, the first KP_PRE_CHUNKS already loaded into pre[] by the caller (so the
// loads overlap the logs), the rest read from lp.  The wave runs as many chunks as its
// longest list; shorter lists end in (B, B) pairs that read the +inf slot B.
template <int NL, int W, bool MIX = false, int PRE = KP_PRE_CHUNKS, typename SP>
__host__ __device__ inline void kp_dp_cell_list(uint32_t l, uint32_t npairs, const uint4 *pre, const uint4 *lp, SP st,
                                                const kp_single_ctx &sc, double alpha, double beta,
                                                const double *pen, uint32_t j0 = 0) {
    SP row = st + l * NL + j0;
    if (__builtin_expect(sc.kmer, 0)) {  // level 0 (CV :145-151 / Fit :106-114)
#pragma unroll
        for (int j = 0; j < W; ++j) {
            const bool s2 = MIX && (int)(j0 + j) >= sc.js;
            row[j] = kp_kmer_train(sc.c, s2 ? sc.a2 : alpha, s2 ? sc.b2 : beta, pen[j]);
        }
        return;
    }
    float lmin[W];
#pragma unroll
    for (int j = 0; j < W; ++j) lmin[j] = row[j];
#ifdef KP_HALF_CHUNKS
    // a chunk whose last two pairs are padding runs as a 2-pair chunk
#pragma unroll
    for (int k = 0; k < PRE; ++k)
        if (4u * k < npairs) {
            if (npairs - 4u * k > 2u)
                kp_chunk_minv<NL, W, 4, kp_sdwa_on<NL, MIX>()>(st, pre[k], j0, lmin);
            else
                kp_chunk_minv<NL, W, 2, kp_sdwa_on<NL, MIX>()>(st, pre[k], j0, lmin);
        }
    for (uint32_t k = PRE; 4u * k < npairs; ++k) kp_chunk_minv<NL, W, 4, kp_sdwa_on<NL, MIX>()>(st, lp[k], j0, lmin);
#else
#pragma unroll
    for (int k = 0; k < PRE; ++k)
        if (4u * k < npairs) kp_chunk_minv<NL, W, 4, kp_sdwa_on<NL, MIX>()>(st, pre[k], j0, lmin);
    for (uint32_t k = PRE; 4u * k < npairs; ++k) kp_chunk_minv<NL, W, 4, kp_sdwa_on<NL, MIX>()>(st, lp[k], j0, lmin);
#endif
    kp_cell_store<W, MIX>(row, lmin, sc, pen, alpha, beta, j0);
}

// ---------------------------------------------------------------------------
// separable count tables of one block (train counts of one group fold).
// T_0[kl] = the block's k-mer-low rows; T_{s+1} expands low position s from nucleotides
// to digits (sum over the digit's nucleotides); T_{t-1} = ptab.  Cell l's counts are then
// a sum of <= 4 ptab entries (kp_ptab_counts).  lm = nucleotide masks [t][16].
// Entries are (M, U) pairs of CT.  tid/nth = this thread and the thread count; sync()
// separates the steps (a workgroup barrier on the GPU, nothing on the host).
// ---------------------------------------------------------------------------
// pre (optional): this thread's first row (k-mer-low cell tid), loaded by the caller ahead
// of time so the load's latency overlaps other work.
template <typename CT, typename LM, typename SyncFn>
__host__ __device__ inline void kp_build_count_table(const kp_geom &g, const CT *K, uint64_t krow, int fold, LM lm,
                                                     CT *bufA, CT *bufB, CT *ptab, uint32_t tid, uint32_t nth,
                                                     SyncFn sync, const kp_cnt *pre = nullptr) {
    CT *out0 = (g.t == 1) ? ptab : bufA;
    for (uint32_t kl = tid; kl < g.n_kl; kl += nth) {
        const kp_cnt c = (pre && kl == tid) ? *pre : kp_kl_counts<CT>(g, K, krow, kl, fold);
        out0[2 * kl] = (CT)c.mtr;
        out0[2 * kl + 1] = (CT)c.utr;
    }
    CT *in = out0;
    uint32_t Rs = 1;
    for (int s = 0; s + 1 < g.t; ++s) {
        sync();
        uint32_t rest = 1;
        for (int i = s + 1; i < g.t; ++i) rest *= g.n[i];
        const uint32_t rs = g.r[s], ns = g.n[s];
        const uint32_t entries = Rs * rs * rest;
        CT *out = (s + 2 == g.t) ? ptab : (in == bufA ? bufB : bufA);
        for (uint32_t e = tid; e < entries; e += nth) {
            const uint32_t D = e % Rs, q = e / Rs, ds = q % rs, Nr = q / rs;
            const uint32_t m = lm[s * 16 + ds];
            CT sm = 0, su = 0;
            for (uint32_t a = 0; a < ns; ++a)
                if (m & (1u << a)) {
                    const uint32_t src = D + Rs * (a + ns * Nr);
                    sm += in[2 * src];
                    su += in[2 * src + 1];
                }
            out[2 * e] = sm;
            out[2 * e + 1] = su;
        }
        in = out;
        Rs *= rs;
    }
}

// train counts of low cell l (packed low digits info) from the block's count table
template <typename CT, bool ALL = false, typename LM, typename PT>
__host__ __device__ inline void kp_ptab_counts(const kp_geom &g, LM lm, PT ptab, uint32_t l, uint32_t info,
                                               uint64_t *mtr, uint64_t *utr) {
    const int tl = g.t - 1;
    const uint32_t Rl = (uint32_t)g.cgl[tl];
    const uint32_t dl = kp_low_digit(info, tl);
    const uint32_t m = lm[tl * 16 + dl];
    const uint32_t base = l - dl * Rl;
    CT mt = 0, ut = 0;
    if (ALL) {
        // all four entries read unconditionally (in flight together, not one LDS round trip
        // per set bit inside a branch), then masked: m has no bits at or past n[tl] <= 4
#pragma unroll
        for (uint32_t c = 0; c < 4; ++c) {
            const uint32_t e = 2 * (base + Rl * (c < g.n[tl] ? c : 0u));
            const CT a = ptab[e], b = ptab[e + 1];
            const CT on = ((m >> c) & 1u) ? (CT)~(CT)0 : (CT)0;
            mt += a & on;
            ut += b & on;
        }
    } else {
        for (uint32_t c = 0; c < g.n[tl]; ++c)
            if (m & (1u << c)) {
                mt += ptab[2 * (base + Rl * c)];
                ut += ptab[2 * (base + Rl * c) + 1];
            }
    }
    *mtr = (uint64_t)mt;
    *utr = (uint64_t)ut;
}

// ---------------------------------------------------------------------------
// whole-lattice helpers for the backtrack (cells addressed by their global index)
// ---------------------------------------------------------------------------

// packed digits of cell x, 4 bits per position
__host__ __device__ inline uint64_t kp_cell_digits(const kp_geom &g, uint64_t x) {
    uint64_t w = 0;
    for (int i = 0; i < g.k; ++i) {
        w |= (x % g.r[i]) << (4 * i);
        x /= g.r[i];
    }
    return w;
}

__host__ __device__ inline uint32_t kp_dig(uint64_t dig, int i) { return (uint32_t)(dig >> (4 * i)) & 15u; }

__host__ __device__ inline bool kp_dig_is_kmer(const kp_geom &g, uint64_t dig) {
    for (int i = 0; i < g.k; ++i)
        if (kp_dig(dig, i) >= g.n[i]) return false;
    return true;
}

// train/test counts of cell x for a group fold: K rows of its block over the matching
// k-mer-low cells (sums are exact in itype, so any order equals the reference's)
// (kpos: block -> count row of K; nullptr = rows in block order, the host emulator's K)
template <typename CT>
__host__ __device__ inline kp_cnt kp_cell_counts(const kp_geom &g, const uint32_t *klofs, const uint16_t *kllist,
                                                 const CT *K, uint64_t x, int fold, const uint32_t *kpos = nullptr) {
    const uint64_t h = x / g.B;
    const uint64_t krow = kpos ? (uint64_t)kpos[h] : h;
    const uint32_t l = (uint32_t)(x % g.B);
    kp_cnt c = {0, 0, 0, 0};
    for (uint32_t q = klofs[l]; q < klofs[l + 1]; ++q) {
        const kp_cnt e = kp_kl_counts<CT>(g, K, krow, kllist[q], fold);
        c.mtr += e.mtr;
        c.utr += e.utr;
        c.mte += e.mte;
        c.ute += e.ute;
    }
    return c;
}

// test -2LL term of a leaf (CV :73-78; level 0: score_test_folds :15-20)
__host__ __device__ inline float kp_leaf_test_term(const kp_cnt &c, bool kmer, int fold, double alpha, double beta) {
    if (fold < 0) return 0.0f;
    if (kmer) return kp_kmer_test(c, alpha, beta);
    const double p = kp_rate(c, alpha, beta);
    return kp_single_test(c, kp_libm_log(p), kp_libm_log(1.0 - p));
}

// The reference's decision for one cell, recomputed from final child scores: splits in
// scan order (positions ascending, pairs in table order, strict "<" from +inf), then the
// single term in float64 (CV :36-78, Fit :37-64).  SF(cell) -> float32 score.  Returns the
// code ((pos << 3) | pair, or KP_SINGLE) and the cell's value in *value.
template <typename SF>
__host__ __device__ inline uint32_t kp_cell_decide(const kp_geom &g, const kp_postab *tabs, uint64_t x, uint64_t dig,
                                                   SF score, const kp_cnt &c, double alpha, double beta, double pen,
                                                   float *value) {
    if (kp_dig_is_kmer(g, dig)) {
        *value = kp_kmer_train(c, alpha, beta, pen);
        return KP_SINGLE;
    }
    float best = __builtin_huge_valf();
    uint32_t code = KP_NONE;
    for (int i = 0; i < g.k; ++i) {
        const uint32_t d = kp_dig(dig, i);
        const kp_postab &T = tabs[i];
        for (int j = 0; j < T.np[d]; ++j) {
            const uint64_t c1 = x - (uint64_t)(d - T.pa[d][j]) * g.cgl[i];
            const uint64_t c2 = x - (uint64_t)(d - T.pb[d][j]) * g.cgl[i];
            const float v = score(c1) + score(c2);
            if (v < best) {
                best = v;
                code = (uint32_t)((i << 3) | j);
            }
        }
    }
    const double p = kp_rate(c, alpha, beta);
    const double s = kp_single_train(c, kp_libm_log(p), kp_libm_log(1.0 - p), pen);
    if (s < (double)best) {
        best = (float)s;
        code = KP_SINGLE;
    }
    *value = best;
    return code;
}

// ---------------------------------------------------------------------------
// sequential backtrack of one lane (host emulator; the GPU runs a breadth-first version):
// DFS over the recomputed argmin tree from the root.  Returns the root's test -2LL summed
// along the tree in float32 (test[c1] + test[c2], CV :47) and lists the leaves in the
// reference's order (left subtree first, Fit :17-24).
//   decide(x, dig, &cnt) -> code   leaf(x, dig, cnt) -> test term
// ---------------------------------------------------------------------------
struct kp_frame {
    uint64_t x, dig, x2, dig2;
    float v1;
    uint32_t st;
};

template <typename DecideFn, typename LeafFn>
__host__ __device__ inline float kp_backtrack_dfs(const kp_geom &g, const kp_postab *tabs, DecideFn decide,
                                                  LeafFn leaf, uint64_t *leaves, uint64_t cap, uint64_t *nleaves,
                                                  uint32_t *bad) {
    kp_frame stk[KP_MAXDEPTH];
    int sp = 1;
    stk[0].x = g.nblocks * g.B - 1;  // the general pattern is the last cell
    stk[0].dig = kp_cell_digits(g, stk[0].x);
    stk[0].st = 0;
    float ret = 0.0f;
    uint64_t nl = 0;
    uint32_t err = 0;
    while (sp > 0) {
        kp_frame &f = stk[sp - 1];
        if (f.st == 0) {
            kp_cnt c;
            const uint32_t code = decide(f.x, f.dig, &c);
            if (code == KP_SINGLE || code == KP_NONE) {
                if (code == KP_NONE) err = 1;
                ret = leaf(f.x, f.dig, c);
                if (leaves && nl < cap) leaves[nl] = f.x;
                ++nl;
                --sp;
            } else {
                const int i = (int)(code >> 3), j = (int)(code & 7u);
                const uint32_t d = kp_dig(f.dig, i);
                const kp_postab &T = tabs[i];
                const uint64_t clear = ~(15ull << (4 * i));
                const uint64_t x1 = f.x - (uint64_t)(d - T.pa[d][j]) * g.cgl[i];
                const uint64_t dig1 = (f.dig & clear) | ((uint64_t)T.pa[d][j] << (4 * i));
                f.x2 = f.x - (uint64_t)(d - T.pb[d][j]) * g.cgl[i];
                f.dig2 = (f.dig & clear) | ((uint64_t)T.pb[d][j] << (4 * i));
                f.st = 1;
                if (sp >= KP_MAXDEPTH) { err = 2; break; }
                stk[sp].x = x1;
                stk[sp].dig = dig1;
                stk[sp].st = 0;
                ++sp;
                continue;
            }
        } else if (f.st == 1) {
            f.v1 = ret;
            f.st = 2;
            if (sp >= KP_MAXDEPTH) { err = 2; break; }
            stk[sp].x = f.x2;
            stk[sp].dig = f.dig2;
            stk[sp].st = 0;
            ++sp;
            continue;
        } else {
            ret = f.v1 + ret;  // f32 + f32, test[c1] + test[c2] (CV :47)
            --sp;
        }
    }
    *nleaves = nl;
    *bad = err;
    return ret;
}
