// kp_hip.hip -- gfx950 kernels and C-ABI of the blocked lattice DP (libkmerpapa_hip.so).
//
// The sweep is VALUE-ONLY (kp_core.h): a cell's float32 score does not depend on which
// candidate won, so only scores are stored; the argmin of the few cells on the optimal
// tree is recomputed with the reference's tie rule at backtrack time.
//
// Kernels:
//   kp_counts_kernel : per-block fold counts K[h] of the block's k-mer-low cells (replaces
//                      the first-pair M/U aggregation, CV :52-55, Fit :50-53); one launch
//                      per high level, once per fold table
//   kp_dp_kernel     : the DP of every cell of one block for NL lanes (CV handle_pattern
//                      :26-78 / score_test_folds :15-20, Fit handle_pattern :31-64 / score
//                      :26-29); one launch per (high level, lane class)
//       counts : separable count tables of the block in LDS (no recurrence)
//       gather : every high-position split pair = two coalesced float4 reads of whole
//                child-block rows (HBM/L2), min-reduced
//       levels : low-position splits inside LDS, level by level, then the float64
//                single-pattern term
//       store  : the block's score rows, float4
//   kp_bt_*          : breadth-first backtrack of every lane at once: one wave per tree
//                      node recomputes the node's decision (kp_cell_decide semantics),
//                      checks it reproduces the stored score, and appends the children;
//                      kp_bt_finish sums the test -2LL along the tree in float32 (CV
//                      :158-163) and lists the leaves in the reference's order (Fit :17-24)
//   kp_codes_kernel  : argmin code of every cell (parity dumps only)
//   kp_allk_terms / kp_allk_sums : --score all_kmers (kp_allk.h; all_kmers_CV.py :8-46):
//                      every (k-mer, fold) term in parallel, then the reference's
//                      sequential float64 sum over k-mers, one thread per column
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdlib>
#include <string>
#include <vector>

#include "../../include/kmerpapa_hip.h"
#include "kp_allk.h"
#include "kp_core.h"
#include "kp_dp_kernel.h"
#include "kp_dp_ws.h"
#include "kp_folds.h"
#include "kp_io.h"
#include "kp_out.h"
#include "kp_plan.h"


// ---------------------------------------------------------------------------
// kernels
// ---------------------------------------------------------------------------


// Fills count slots s0 .. s0+ncol-1 of every block of high level H.  Kin_M/Kin_U are
// [n_kmers][ncol] (k-mer order): column c goes to slot s0 + c.  K is slot-major
// (kp_core.h), so a block's rows of one slot are n_kl contiguous (M, U) pairs.  A
// workgroup fills KP_CROWS blocks' rows, KP_CTPR threads per row: a row is only 2 n_kl
// counts (512 B at 9-mers) behind a chain of dependent index loads (block list, digits,
// child rows), so one row per workgroup left the launch latency-bound (2.55 ms per fold
// table at 9-mers).
#define KP_CTPR 32
#define KP_CROWS (256 / KP_CTPR)
template <typename CT>
__global__ void __launch_bounds__(256) kp_counts_kernel(kp_geom g, kp_dev_tables T, uint64_t hbase, uint64_t nb,
                                                        int H, const CT *__restrict__ Kin_M,
                                                        const CT *__restrict__ Kin_U, uint32_t ncol, uint32_t s0,
                                                        CT *__restrict__ K) {
    const uint64_t q = (uint64_t)blockIdx.x * KP_CROWS + threadIdx.x / KP_CTPR;
    if (q >= nb) return;
    const uint32_t lt = threadIdx.x % KP_CTPR;
    const uint64_t h = T.hlist[hbase + q];
    const uint64_t se = kp_kslot_elems(g), row = (hbase + q) * (uint64_t)g.n_kl * 2;  // list order
    if (H == 0) {
        // all high digits are nucleotides: the block's k-mer-low cells are k-mers
        uint64_t kbase = 0;
        for (int i = 0; i < g.kh; ++i) kbase += (uint64_t)kp_high_digit(g, h, i) * g.khw[i];
        for (uint32_t e = lt; e < g.n_kl * ncol; e += KP_CTPR) {
            const uint32_t c = e / g.n_kl, kl = e % g.n_kl;
            const uint64_t src = (kbase + kl) * (uint64_t)ncol + c;
            CT *dst = K + se * (s0 + c) + row + 2 * kl;
            dst[0] = Kin_M[src];
            dst[1] = Kin_U[src];
        }
        return;
    }
    // any split partitions the same k-mers; take the first ambiguous high position's
    // first pair like the reference does (sums are exact: itype never overflows)
    uint64_t h1 = h, h2 = h;
    for (int i = 0; i < g.kh; ++i) {
        uint32_t d = kp_high_digit(g, h, i);
        const kp_postab &P = T.tabs[g.t + i];
        if (P.np[d] > 0) {
            h1 = h - (uint64_t)(d - P.pa[d][0]) * g.hcg[i];
            h2 = h - (uint64_t)(d - P.pb[d][0]) * g.hcg[i];
            break;
        }
    }
    const uint64_t r1 = (uint64_t)T.kpos[h1] * g.n_kl * 2, r2 = (uint64_t)T.kpos[h2] * g.n_kl * 2;
    for (uint32_t e = lt; e < g.n_kl * ncol * 2; e += KP_CTPR) {
        const uint32_t c = e / (2 * g.n_kl), r = e % (2 * g.n_kl);
        const uint64_t base = se * (s0 + c);
        K[base + row + r] = K[base + r1 + r] + K[base + r2 + r];
    }
}

// ---------------------------------------------------------------------------
// breadth-first backtrack
// ---------------------------------------------------------------------------

struct kp_node {
    uint64_t x;      // cell
    uint64_t dig;    // its packed digits
    uint32_t child;  // first child (the second is child + 1); 0 = leaf
    uint32_t nleaf;  // leaves of the subtree
    uint32_t off;    // position of the subtree's first leaf in backtrack order
    float test;      // test -2LL of the subtree, float32 sums along the tree
};

struct kp_bt_params {
    kp_geom g;
    kp_dev_tables T;
    const void *K;
    const float *S;
    const kp_group_dev *groups;
    const uint32_t *lanegrp;
    kp_node *nodes;    // [Ltot][cap]
    uint32_t cap;
    uint32_t *cnt;     // [Ltot] nodes allocated
    uint32_t *dend;    // [Ltot][KP_MAXDEPTH + 1] end of each depth's node range
    uint32_t *bad;     // [Ltot] 1 = no candidate, 2 = node pool full, 4 = score not reproduced
    float *root_train, *root_test;
    uint64_t *nleaves;
    uint64_t *leaves;  // [Ltot][leafcap]
    uint64_t leafcap;
    int depth;
    int maxdepth;
};

__device__ inline uint64_t kp_wave_sum(uint64_t v) {
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    return v;
}

__host__ __device__ inline uint64_t kp_s_off(const kp_geom &g, uint64_t h, uint32_t lane, uint32_t l) {
    return (h * g.Ltot + lane) * (uint64_t)g.Bpad + l;
}

__global__ void kp_bt_init(kp_bt_params P, uint64_t root_x, uint64_t root_dig) {
    const uint32_t lane = blockIdx.x * blockDim.x + threadIdx.x;
    if (lane >= P.g.Ltot) return;
    kp_node *N = P.nodes + (uint64_t)lane * P.cap;
    N[0].x = root_x;
    N[0].dig = root_dig;
    N[0].child = 0;
    N[0].nleaf = 0;
    N[0].off = 0;
    N[0].test = 0.0f;
    P.cnt[lane] = 1;
    P.dend[(uint64_t)lane * (KP_MAXDEPTH + 1)] = 1;
    P.bad[lane] = 0;
}

__global__ void kp_bt_advance(kp_bt_params P) {
    const uint32_t lane = blockIdx.x * blockDim.x + threadIdx.x;
    if (lane >= P.g.Ltot) return;
    P.dend[(uint64_t)lane * (KP_MAXDEPTH + 1) + P.depth + 1] = P.cnt[lane];
}

// one wave per node of depth P.depth; grid (waves, lanes)
template <typename CT>
__global__ void __launch_bounds__(256) kp_bt_level(kp_bt_params P) {
    const kp_geom &g = P.g;
    const uint32_t lane = blockIdx.y;
    const uint32_t lid = threadIdx.x & 63u;
    const uint32_t *de = P.dend + (uint64_t)lane * (KP_MAXDEPTH + 1);
    const uint32_t lo = P.depth ? de[P.depth - 1] : 0u, hi = de[P.depth];
    const kp_group_dev *G = P.groups + P.lanegrp[lane];
    const int fold = G->fold;
    const int jl = (int)(lane - (uint32_t)G->lane0);
    const double alpha = kp_lane_alpha(*G, jl), beta = kp_lane_beta(*G, jl);
    const double pen = G->pen[jl];
    const CT *K = reinterpret_cast<const CT *>(P.K);
    kp_node *N = P.nodes + (uint64_t)lane * P.cap;
    const uint32_t nw = (gridDim.x * blockDim.x) >> 6;
    for (uint32_t n = lo + ((blockIdx.x * blockDim.x + threadIdx.x) >> 6); n < hi; n += nw) {
        const uint64_t x = N[n].x, dig = N[n].dig;
        const uint64_t h = x / g.B;
        const uint32_t l = (uint32_t)(x % g.B);
        const bool kmer = kp_dig_is_kmer(g, dig);
        // counts: the wave splits the k-mer-low rows of the cell, then reduces
        uint64_t mtr = 0, utr = 0, mte = 0, ute = 0;
        const uint32_t q0 = P.T.klofs[l], q1 = P.T.klofs[l + 1];
        for (uint32_t q = q0 + lid; q < q1; q += 64) {
            const kp_cnt c = kp_kl_counts<CT>(g, K, P.T.kpos[h], P.T.kllist[q], fold);
            mtr += c.mtr; utr += c.utr; mte += c.mte; ute += c.ute;
        }
        kp_cnt c;
        c.mtr = kp_wave_sum(mtr);
        c.utr = kp_wave_sum(utr);
        c.mte = kp_wave_sum(mte);
        c.ute = kp_wave_sum(ute);
        // split candidates: one (position, pair) per lane, scan order = code order
        float best = __builtin_huge_valf();
        uint32_t code = KP_NONE;
        if (!kmer) {
            uint32_t npt = 0;
            for (int i = 0; i < g.k; ++i) npt += P.T.tabs[i].np[kp_dig(dig, i)];
            for (uint32_t p = lid; p < npt; p += 64) {
                uint32_t rem = p, d = 0;
                int i = 0;
                for (; i < g.k; ++i) {
                    d = kp_dig(dig, i);
                    const uint32_t npi = P.T.tabs[i].np[d];
                    if (rem < npi) break;
                    rem -= npi;
                }
                const kp_postab &T = P.T.tabs[i];
                const uint32_t da = d - T.pa[d][rem], db = d - T.pb[d][rem];
                uint64_t o1, o2;
                if (i < g.t) {
                    const uint32_t cg = (uint32_t)g.cgl[i];
                    o1 = kp_s_off(g, h, lane, l - da * cg);
                    o2 = kp_s_off(g, h, lane, l - db * cg);
                } else {
                    o1 = kp_s_off(g, h - (uint64_t)da * g.hcg[i - g.t], lane, l);
                    o2 = kp_s_off(g, h - (uint64_t)db * g.hcg[i - g.t], lane, l);
                }
                const float v = P.S[o1] + P.S[o2];
                if (v < best) {  // a lane sees its pairs in increasing code order
                    best = v;
                    code = (uint32_t)((i << 3) | rem);
                }
            }
            // first minimum over the wave: smaller value, then smaller code (= earlier in scan)
            for (int off = 32; off > 0; off >>= 1) {
                const float ob = __shfl_xor(best, off, 64);
                const uint32_t oc = __shfl_xor(code, off, 64);
                if (ob < best || (ob == best && oc < code)) {
                    best = ob;
                    code = oc;
                }
            }
        }
        // single pattern term; the stored score must be reproduced exactly
        float value;
        float test = 0.0f;
        if (kmer) {
            value = kp_kmer_train(c, alpha, beta, pen);
            code = KP_SINGLE;
            if (fold >= 0) test = kp_kmer_test(c, alpha, beta);
        } else {
            const double pr = kp_rate(c, alpha, beta);
            const double lp = kp_libm_log(pr), l1p = kp_libm_log(1.0 - pr);  // the C library's (kp_libm.h)
            const double s = kp_single_train(c, lp, l1p, pen);
            value = best;
            if (s < (double)best) {
                value = (float)s;
                code = KP_SINGLE;
            }
            if (code == KP_SINGLE && fold >= 0) test = kp_single_test(c, lp, l1p);
        }
        if (lid == 0) {
            const float stored = P.S[kp_s_off(g, h, lane, l)];
            const bool same = (__float_as_uint(stored) == __float_as_uint(value)) || (stored != stored && value != value);
            uint32_t err = same ? 0u : 4u;
            if (code == KP_SINGLE) {
                N[n].child = 0;
                N[n].test = test;
            } else if (code == KP_NONE) {
                err |= 1u;
                N[n].child = 0;
                N[n].test = 0.0f;
            } else {
                const uint32_t base = atomicAdd(P.cnt + lane, 2u);
                if (base + 2 > P.cap) {
                    err |= 2u;
                    N[n].child = 0;
                } else {
                    const int i = (int)(code >> 3), j = (int)(code & 7u);
                    const uint32_t d = kp_dig(dig, i);
                    const kp_postab &T = P.T.tabs[i];
                    const uint64_t clear = ~(15ull << (4 * i));
                    kp_node a, b;
                    a.x = x - (uint64_t)(d - T.pa[d][j]) * g.cgl[i];
                    a.dig = (dig & clear) | ((uint64_t)T.pa[d][j] << (4 * i));
                    b.x = x - (uint64_t)(d - T.pb[d][j]) * g.cgl[i];
                    b.dig = (dig & clear) | ((uint64_t)T.pb[d][j] << (4 * i));
                    a.child = b.child = 0;
                    a.nleaf = b.nleaf = 0;
                    a.off = b.off = 0;
                    a.test = b.test = 0.0f;
                    N[base] = a;
                    N[base + 1] = b;
                    N[n].child = base;
                }
            }
            if (err) atomicOr(P.bad + lane, err);
        }
    }
}

// one workgroup per lane: float32 test sums bottom-up, then leaf order top-down
__global__ void __launch_bounds__(256) kp_bt_finish(kp_bt_params P) {
    const kp_geom &g = P.g;
    const uint32_t lane = blockIdx.x;
    const uint32_t *de = P.dend + (uint64_t)lane * (KP_MAXDEPTH + 1);
    kp_node *N = P.nodes + (uint64_t)lane * P.cap;
    for (int d = P.maxdepth; d >= 0; --d) {
        const uint32_t lo = d ? de[d - 1] : 0u, hi = de[d];
        for (uint32_t n = lo + threadIdx.x; n < hi; n += blockDim.x) {
            const uint32_t c = N[n].child;
            if (c) {
                N[n].test = N[c].test + N[c + 1].test;  // test[c1] + test[c2] (CV :47)
                N[n].nleaf = N[c].nleaf + N[c + 1].nleaf;
            } else {
                N[n].nleaf = 1;
            }
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) N[0].off = 0;
    __syncthreads();
    uint64_t *leaves = P.leaves + (uint64_t)lane * P.leafcap;
    for (int d = 0; d <= P.maxdepth; ++d) {
        const uint32_t lo = d ? de[d - 1] : 0u, hi = de[d];
        for (uint32_t n = lo + threadIdx.x; n < hi; n += blockDim.x) {
            const uint32_t c = N[n].child, off = N[n].off;
            if (c) {
                N[c].off = off;
                N[c + 1].off = off + N[c].nleaf;
            } else if (off < P.leafcap) {
                leaves[off] = N[n].x;
            }
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        P.root_train[lane] = P.S[kp_s_off(g, g.nblocks - 1, lane, g.B - 1)];
        P.root_test[lane] = N[0].test;
        P.nleaves[lane] = N[0].nleaf;
    }
}

// The high split pairs of every block of the block list, in scan order (positions
// ascending, pairs in table order: the order kp_dp_kernel's pair setup walks them), as
// child-block deltas: hpd[q][0 .. np) = kp_hpd_word, the rest of the hps-word row 0.  One
// thread per block, once per plan.
__global__ void kp_hpd_kernel(kp_geom g, const kp_postab *__restrict__ tabs, const uint64_t *__restrict__ hdig,
                              uint64_t nblocks, uint32_t hps, uint64_t *__restrict__ hpd) {
    for (uint64_t q = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; q < nblocks;
         q += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t hd = hdig[q];
        uint64_t *row = hpd + q * hps;
        uint32_t n = 0;
        for (int i = 0; i < g.kh; ++i) {
            const kp_postab &T = tabs[g.t + i];
            const uint32_t d = (uint32_t)(hd >> (4 * i)) & 15u;
            for (uint32_t r = 0; r < T.np[d]; ++r)
                row[n++] = kp_hpd_word((uint64_t)(d - T.pa[d][r]) * g.hcg[i], (uint64_t)(d - T.pb[d][r]) * g.hcg[i],
                                       (uint32_t)i);
        }
        for (; n < hps; ++n) row[n] = 0;
    }
}

// The block list (hlist / kpos / hdig / hnp) of kp::build_plan's block order, built on the
// device from the plan's rank table instead of walked and uploaded by the host (2.3 M
// blocks at 9-mers: the walk was most of the plan's start-up, before the first pass).  One
// thread per block h; every slot is written once (kp_block_slot is a bijection).
__global__ void kp_blocks_kernel(kp_geom g, const kp_postab *__restrict__ tabs, kp_blockgen bg,
                                 const uint32_t *__restrict__ brank, const uint64_t *__restrict__ hoff,
                                 uint32_t *__restrict__ hlist, uint32_t *__restrict__ kpos, uint64_t *__restrict__ hdig,
                                 uint64_t *__restrict__ hnp) {
    for (uint64_t h = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; h < g.nblocks;
         h += (uint64_t)gridDim.x * blockDim.x) {
        uint64_t hd, hn;
        const uint64_t q = kp_block_slot(g, tabs, bg, brank, hoff, h, &hd, &hn);
        hlist[q] = (uint32_t)h;
        kpos[h] = (uint32_t)q;
        hdig[q] = hd;
        hnp[q] = hn;
    }
}

static kp_blockgen blockgen_of(const kp::host_plan &hp) {
    kp_blockgen bg;
    memset(&bg, 0, sizeof(bg));
    bg.hs = hp.hs;
    for (int j = 0; j < hp.g.kh; ++j) bg.perm[j] = (int8_t)hp.perm[j];
    return bg;
}

// the C library's log (fn 1) or log1p (fn 2) as restated for the device (kp_libm.h), the
// device's own log (fn 0), the table-free fast log (fn 3, kp_fast_log) or its FMA form (fn 4, kp_fma_log)
__global__ void kp_libm_kernel(const double *__restrict__ x, double *__restrict__ y, uint64_t n, int fn) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        y[i] = fn == 1 ? kp_libm_log(x[i]) : fn == 2 ? kp_libm_log1p(x[i]) : fn == 3 ? kp_fast_log(x[i])
             : fn == 4 ? kp_fma_log(x[i]) : log(x[i]);
}

// float32 scores of the given cells of one lane (parity checks of a full-size pass: the
// cells of an embedded sub-lattice, against the oracle run on that sub-lattice alone)
__global__ void kp_gather_cells_kernel(kp_geom g, const float *__restrict__ S, uint32_t lane,
                                       const uint64_t *__restrict__ cells, uint64_t n, float *__restrict__ out) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t x = cells[i];
        out[i] = S[kp_s_off(g, x / g.B, lane, (uint32_t)(x % g.B))];
    }
}

// argmin code of every cell of one lane (parity dumps): the sequential decision of kp_core.h
template <typename CT>
__global__ void kp_codes_kernel(kp_geom g, kp_dev_tables T, const CT *K, const float *S, kp_group_dev G,
                                uint32_t lane, double pen, uint8_t *code) {
    const uint64_t npat = g.nblocks * g.B;
    for (uint64_t x = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; x < npat;
         x += (uint64_t)gridDim.x * blockDim.x) {
        const kp_cnt c = kp_cell_counts<CT>(g, T.klofs, T.kllist, K, x, G.fold, T.kpos);
        const uint64_t dig = kp_cell_digits(g, x);
        auto score = [&](uint64_t y) { return S[kp_s_off(g, y / g.B, lane, (uint32_t)(y % g.B))]; };
        float v;
        const int jl = (int)(lane - (uint32_t)G.lane0);
        code[x] = (uint8_t)kp_cell_decide(g, T.tabs, x, dig, score, c, kp_lane_alpha(G, jl), kp_lane_beta(G, jl), pen,
                                          &v);
    }
}

// ---------------------------------------------------------------------------
// C-ABI
// ---------------------------------------------------------------------------

static thread_local std::string g_err;

static int fail(int code, const std::string &msg) {
    g_err = msg;
    return code;
}

#define KP_HIP(expr)                                                                                  \
    do {                                                                                              \
        hipError_t e_ = (expr);                                                                       \
        if (e_ != hipSuccess)                                                                         \
            return fail(KP_E_HIP, std::string(#expr) + ": " + hipGetErrorString(e_));                 \
    } while (0)

#define KP_SIDE_STREAMS 3

struct kp_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    hipEvent_t ev[4] = {nullptr, nullptr, nullptr, nullptr};
    // side streams: the lane classes of one pass (device groups of different widths, e.g. a
    // 5-lane and a 1-lane group, or the 4 + 3 split of a 7-penalty group) are independent,
    // so each class runs its launch sequence on a stream of its own and the classes overlap
    hipStream_t side[KP_SIDE_STREAMS] = {nullptr, nullptr, nullptr};
    hipEvent_t side_ev[KP_SIDE_STREAMS] = {nullptr, nullptr, nullptr};
    size_t lds_max = 65536;
    int cus = 256;  // compute units (the persistent sweep's grid)
};

struct kp_plan {
    kp_ctx *ctx = nullptr;
    kp::host_plan hp;
    uint32_t max_block = 4096;  // the block budget build_plan ran with (kp_plan_block_check rebuilds with it)
    // device tables
    kp_postab *d_tabs = nullptr;
    uint32_t *d_lowinfo = nullptr;
    int32_t *d_loff = nullptr;
    uint32_t *d_klofs = nullptr;
    uint16_t *d_kllist = nullptr;
    uint32_t *d_hlist = nullptr;
    uint32_t *d_kpos = nullptr;
    kp_lowdesc *d_ldesc = nullptr;
    uint64_t *d_hdig = nullptr;
    uint64_t *d_hnp = nullptr;
    uint64_t *d_hpd = nullptr;  // [nblocks][hps] high split pairs per block (kp_hpd_kernel)
    uint32_t hps = 0;
    uint8_t *d_lowmask = nullptr;
    uint32_t *d_lpairs = nullptr;
    // counts
    void *d_K = nullptr;     // [nf + 1][q][kl][2] CT, rows in block-list order (kp_core.h)
    int nf = 0;
    int ct_bytes = 0;
    std::vector<uint8_t> fold_set;  // fold f's slot holds counts (kp_counts_fold / kp_set_counts)
    // kp_counts_fold runs asynchronously on a stream of its own (a fold's table fills while
    // the previous fold's pass runs): pinned + device staging of one fold's counts, the
    // event that frees the pinned copy, and per fold the event its passes wait for
    hipStream_t cstream = nullptr;
    void *h_stage = nullptr, *d_stage = nullptr;
    size_t stage_bytes = 0;
    hipEvent_t stage_ev = nullptr;
    std::vector<hipEvent_t> fold_ev;
    std::vector<uint8_t> fold_async;  // fold f's table was filled on cstream (passes wait on fold_ev[f])
    // lanes
    float *d_S = nullptr;
    bool S_pool = false;  // d_S came from the device's stream-ordered pool (see alloc_scores)
    uint64_t lanes_cap = 0;
    kp_node *d_nodes = nullptr;
    uint32_t node_cap = 0;  // nodes per lane
    kp_group_dev *d_groups = nullptr;
    uint32_t *d_lanegrp = nullptr;
    float *d_rtrain = nullptr, *d_rtest = nullptr;
    kp_dp_params *d_wsp = nullptr;  // launch parameters of the pass's kp_dp_ws_kernel launches (device copy)
    size_t wsp_cap = 0;
    uint32_t *d_werr = nullptr;  // kp_dp_ws_kernel's error word (a hand-over wait timed out)
    uint64_t *d_nleaves = nullptr;
    uint32_t *d_bad = nullptr;
    uint32_t *d_cnt = nullptr;
    uint32_t *d_dend = nullptr;
    uint64_t *d_leaves = nullptr;
    uint64_t small_cap = 0;  // lanes the small buffers above can hold
    uint32_t last_ltot = 0;
    std::vector<kp_group_dev> last_groups;  // device groups of the last pass (dump)
    std::vector<uint32_t> last_lanegrp;
    kp_pass_stats stats{};
    std::vector<hipEvent_t> lev;     // per-launch events (KP_LAUNCH_TIMES=1)
    std::vector<float> launch_ms;    // per-launch times of the last pass (class-major, H ascending)
};

static void free_scores(kp_plan *p);  // the score rows (pool or hipMalloc), defined below

static kp_dev_tables tables_of(const kp_plan *p) {
    kp_dev_tables T;
    T.tabs = p->d_tabs;
    T.lowinfo = p->d_lowinfo;
    T.loff = p->d_loff;
    T.klofs = p->d_klofs;
    T.kllist = p->d_kllist;
    T.hlist = p->d_hlist;
    T.kpos = p->d_kpos;
    T.ldesc = p->d_ldesc;
    T.hdig = p->d_hdig;
    T.hnp = p->d_hnp;
    T.hpd = p->d_hpd;
    T.hps = p->hps;
    T.lowmask = p->d_lowmask;
    T.lpairs = reinterpret_cast<const uint4 *>(p->d_lpairs);
    return T;
}

// Device memory: plain hipMalloc.  On this platform an allocation of HBM that was used
// before (by this or an earlier process) waits for the driver to wipe it, ~30 ms per GB
// (4-6 s for the 150 GB of a 9-mer pass; fresh HBM 0.05 s per 100 GB), so the library
// allocates the large per-lane buffers once (kp_reserve_lanes) and only grows them.  The
// stream-ordered allocator (hipMallocAsync) skips that wait but is not usable: a 140 GB
// request served from a freed 100 GB pool block returned memory that did not hold what
// was written to it (tools/async_check.hip).
template <typename T>
static hipError_t dmalloc(T **p, size_t bytes) {
    return hipMalloc(reinterpret_cast<void **>(p), std::max<size_t>(bytes, 1));
}

template <typename T>
static int upload(T **dptr, const std::vector<T> &v) {
    size_t bytes = std::max<size_t>(1, v.size()) * sizeof(T);
    KP_HIP(dmalloc(dptr, bytes));
    if (!v.empty()) KP_HIP(hipMemcpy(*dptr, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice));
    return KP_OK;
}

static void dfree(void *p) {
    if (p) (void)hipFree(p);
}

// nodes of one lane's backtrack tree: at most 2 * leaves - 1 <= 2 * n_kmers - 1
static uint32_t node_cap_of(const kp::host_plan &hp) { return (uint32_t)(2 * hp.n_kmers + 2); }

extern "C" {

const char *kp_last_error(void) { return g_err.c_str(); }

int kp_device_count(int *n) {
    if (!n) return fail(KP_E_ARG, "null");
    KP_HIP(hipGetDeviceCount(n));
    return KP_OK;
}

int kp_create(int device, kp_ctx **out) {
    if (!out) return fail(KP_E_ARG, "null out");
    int n = 0;
    KP_HIP(hipGetDeviceCount(&n));
    if (device < 0 || device >= n) return fail(KP_E_ARG, "device " + std::to_string(device) + " not present");
    KP_HIP(hipSetDevice(device));
    kp_ctx *c = new kp_ctx();
    c->device = device;
    KP_HIP(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
    for (auto &e : c->ev) KP_HIP(hipEventCreate(&e));
    for (int i = 0; i < KP_SIDE_STREAMS; ++i) {
        KP_HIP(hipStreamCreateWithFlags(&c->side[i], hipStreamNonBlocking));
        KP_HIP(hipEventCreateWithFlags(&c->side_ev[i], hipEventDisableTiming));
    }
    int lds = 0;
    if (hipDeviceGetAttribute(&lds, hipDeviceAttributeMaxSharedMemoryPerBlock, device) == hipSuccess && lds > 0)
        c->lds_max = (size_t)lds;
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) == hipSuccess && cus > 0) c->cus = cus;
    *out = c;
    return KP_OK;
}

int kp_device_mem(kp_ctx *c, uint64_t *free_bytes, uint64_t *total_bytes) {
    if (!c) return fail(KP_E_ARG, "null ctx");
    KP_HIP(hipSetDevice(c->device));
    size_t fr = 0, tot = 0;
    KP_HIP(hipMemGetInfo(&fr, &tot));
    if (free_bytes) *free_bytes = fr;
    if (total_bytes) *total_bytes = tot;
    return KP_OK;
}

void kp_destroy(kp_ctx *c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    for (auto e : c->ev)
        if (e) (void)hipEventDestroy(e);
    for (int i = 0; i < KP_SIDE_STREAMS; ++i) {
        if (c->side_ev[i]) (void)hipEventDestroy(c->side_ev[i]);
        if (c->side[i]) (void)hipStreamDestroy(c->side[i]);
    }
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
}

}  // extern "C"

// The plan's block list built on the device (kp_blocks_kernel): rank table and level
// offsets up, one launch, the small tables freed once it has run.
static int device_blocks(kp_plan *p) {
    const kp_geom &g = p->hp.g;
    uint32_t *d_brank = nullptr;
    uint64_t *d_hoff = nullptr;
    int rc;
    if ((rc = upload(&d_brank, p->hp.brank)) || (rc = upload(&d_hoff, p->hp.hoff))) {
        dfree(d_brank);
        dfree(d_hoff);
        return rc;
    }
    hipError_t he = dmalloc(&p->d_hlist, g.nblocks * sizeof(uint32_t));
    if (he == hipSuccess) he = dmalloc(&p->d_kpos, g.nblocks * sizeof(uint32_t));
    if (he == hipSuccess) he = dmalloc(&p->d_hdig, g.nblocks * sizeof(uint64_t));
    if (he == hipSuccess) he = dmalloc(&p->d_hnp, g.nblocks * sizeof(uint64_t));
    if (he == hipSuccess) {
        const unsigned nb = (unsigned)std::min<uint64_t>((g.nblocks + 255) / 256, 16384);
        hipLaunchKernelGGL(kp_blocks_kernel, dim3(nb), dim3(256), 0, p->ctx->stream, g, p->d_tabs, blockgen_of(p->hp),
                           d_brank, d_hoff, p->d_hlist, p->d_kpos, p->d_hdig, p->d_hnp);
        he = hipGetLastError();
        if (he == hipSuccess) he = hipStreamSynchronize(p->ctx->stream);
    }
    dfree(d_brank);
    dfree(d_hoff);
    if (he == hipErrorOutOfMemory)  // the block-list tables do not fit: the lattice is too big here
        return fail(KP_E_NOMEM, "block list of " + p->hp.gp + " (" + std::to_string(g.nblocks) +
                                    " blocks): out of device memory");
    if (he != hipSuccess) return fail(KP_E_HIP, std::string("block list: ") + hipGetErrorString(he));
    return KP_OK;
}

extern "C" {

int kp_plan_create(kp_ctx *ctx, const char *gen_pat, uint32_t max_block, kp_plan **out) {
    if (!ctx || !gen_pat || !out) return fail(KP_E_ARG, "null argument");
    KP_HIP(hipSetDevice(ctx->device));
    kp_plan *p = new kp_plan();
    p->ctx = ctx;
    p->max_block = max_block ? max_block : 4096u;
    std::string err = kp::build_plan(gen_pat, p->max_block, p->hp, false);
    if (!err.empty()) {
        delete p;
        return fail(KP_E_ARG, err);
    }
    int rc;
    if ((rc = upload(&p->d_tabs, p->hp.tabs)) || (rc = upload(&p->d_lowinfo, p->hp.lowinfo)) ||
        (rc = upload(&p->d_loff, p->hp.loff)) || (rc = upload(&p->d_klofs, p->hp.klofs)) ||
        (rc = upload(&p->d_kllist, p->hp.kllist)) || (rc = upload(&p->d_ldesc, p->hp.ldesc)) ||
        (rc = upload(&p->d_lowmask, p->hp.lowmask)) || (rc = upload(&p->d_lpairs, p->hp.lpairs))) {
        kp_plan_destroy(p);
        return rc;
    }
    if (p->hp.blocks_on_host) {  // an experiment block order (KP_BLOCK_TILE / KP_BLOCK_ORDER)
        if ((rc = upload(&p->d_hlist, p->hp.hlist)) || (rc = upload(&p->d_kpos, p->hp.kpos)) ||
            (rc = upload(&p->d_hdig, p->hp.hdig)) || (rc = upload(&p->d_hnp, p->hp.hnp))) {
            kp_plan_destroy(p);
            return rc;
        }
    } else if ((rc = device_blocks(p))) {
        kp_plan_destroy(p);
        return rc;
    }
    // the blocks' high split pairs as child-block deltas (one load per pair in the sweep's
    // block setup); only when every block has at most 64 pairs (one wave) and the deltas
    // fit their 29-bit fields -- otherwise the sweep derives them from hdig and tabs
    {
        const kp_geom &g = p->hp.g;
        uint32_t most = 0;
        for (int i = 0; i < g.kh; ++i) {
            uint32_t m = 0;
            for (uint32_t d = 0; d < g.r[g.t + i]; ++d) m = std::max<uint32_t>(m, p->hp.tabs[g.t + i].np[d]);
            most += m;
        }
        const char *e = getenv("KP_HPD");
        if ((!e || atoi(e) != 0) && most >= 1 && most <= 64 && g.nblocks < (1ull << 29)) {
            // optional: if it cannot be set up (e.g. out of memory) the plan keeps the
            // hdig/tabs setup instead of failing
            hipError_t he = dmalloc(&p->d_hpd, g.nblocks * most * sizeof(uint64_t));
            if (he == hipSuccess) {
                const unsigned nb = (unsigned)std::min<uint64_t>((g.nblocks + 255) / 256, 16384);
                hipLaunchKernelGGL(kp_hpd_kernel, dim3(nb), dim3(256), 0, ctx->stream, g, p->d_tabs, p->d_hdig,
                                   (uint64_t)g.nblocks, most, p->d_hpd);
                he = hipGetLastError();
                if (he == hipSuccess) he = hipStreamSynchronize(ctx->stream);
            }
            if (he == hipSuccess) {
                p->hps = most;
            } else {
                (void)hipGetLastError();  // clear a sticky launch / allocation error
                dfree(p->d_hpd);
                p->d_hpd = nullptr;
                p->hps = 0;
            }
        }
    }
    *out = p;
    return KP_OK;
}

void kp_plan_destroy(kp_plan *p) {
    if (!p) return;
    if (p->ctx) (void)hipSetDevice(p->ctx->device);
    free_scores(p);
    void *bufs[] = {p->d_tabs,    p->d_lowinfo, p->d_loff,   p->d_klofs,   p->d_kllist, p->d_hlist, p->d_kpos, p->d_ldesc,
                    p->d_hdig,    p->d_hnp,     p->d_hpd,     p->d_lowmask, p->d_lpairs, p->d_K,      p->d_nodes, p->d_groups,
                    p->d_lanegrp, p->d_rtrain,  p->d_rtest,  p->d_nleaves, p->d_bad,    p->d_cnt,   p->d_dend,
                    p->d_leaves};
    if (p->cstream) (void)hipStreamSynchronize(p->cstream);
    for (void *b : bufs) dfree(b);
    dfree(p->d_wsp);
    dfree(p->d_werr);
    dfree(p->d_stage);
    if (p->h_stage) (void)hipHostFree(p->h_stage);
    if (p->stage_ev) (void)hipEventDestroy(p->stage_ev);
    for (hipEvent_t e : p->fold_ev) (void)hipEventDestroy(e);
    if (p->cstream) (void)hipStreamDestroy(p->cstream);
    for (hipEvent_t e : p->lev) (void)hipEventDestroy(e);
    delete p;
}

static int wg_lanes(const kp::host_plan &hp, size_t ct_bytes, size_t lds_max);  // defined with the launch code

// ct_bytes / lds_max: the count width and LDS of the plan's device once counts are set
// (lanes_per_workgroup is then what kp_pass uses); 4 bytes and 160 KiB before that
static void info_of(const kp::host_plan &h, kp_plan_info *o, size_t ct_bytes = 4, size_t lds_max = 160u * 1024u) {
    o->npat = h.npat;
    o->nblocks = h.g.nblocks;
    o->n_kmers = h.n_kmers;
    o->block = h.g.B;
    o->block_pad = h.g.Bpad;
    o->k = h.g.k;
    o->low_positions = h.g.t;
    o->max_level = h.maxlev;
    o->high_levels = h.hmax + 1;
    o->pairs_total = h.pairs_total;
    o->pairs_high = h.pairs_high;
    // train scores + backtrack node pool + leaf list
    o->bytes_per_lane = h.g.nblocks * (uint64_t)h.g.Bpad * 4 + (uint64_t)node_cap_of(h) * sizeof(kp_node) +
                        h.n_kmers * 8 + 4096;
    o->lanes_per_workgroup = (uint32_t)wg_lanes(h, ct_bytes, lds_max);
    o->pad_ = 0;
}

int kp_plan_get_info(const kp_plan *p, kp_plan_info *o) {
    if (!p || !o) return fail(KP_E_ARG, "null argument");
    info_of(p->hp, o, p->ct_bytes ? (size_t)p->ct_bytes : 4u, p->ctx ? p->ctx->lds_max : 160u * 1024u);
    return KP_OK;
}

int kp_plan_host(const char *gen_pat, uint32_t max_block, kp_plan_info *o) {
    if (!gen_pat || !o) return fail(KP_E_ARG, "null argument");
    kp::host_plan hp;
    std::string err = kp::build_plan(gen_pat, max_block ? max_block : 4096u, hp, false);
    if (!err.empty()) return fail(KP_E_ARG, err);
    info_of(hp, o);
    return KP_OK;
}

int kp_plan_host_counts(const char *gen_pat, uint32_t max_block, int itype_bytes, kp_plan_info *o) {
    if (!gen_pat || !o || (itype_bytes != 4 && itype_bytes != 8)) return fail(KP_E_ARG, "bad arguments");
    kp::host_plan hp;
    std::string err = kp::build_plan(gen_pat, max_block ? max_block : 4096u, hp, false);
    if (!err.empty()) return fail(KP_E_ARG, err);
    info_of(hp, o, (size_t)itype_bytes);
    return KP_OK;
}

// Host-only (no GPU): the closed-form block order (kp_block_slot) against build_plan's
// block walk, every block of the lattice; *mismatches = blocks whose slot, digits or
// split-pair counts differ.
int kp_block_order_check(const char *gen_pat, uint32_t max_block, uint64_t *mismatches) {
    if (!gen_pat || !mismatches) return fail(KP_E_ARG, "null argument");
    kp::host_plan hp;
    std::string err = kp::build_plan(gen_pat, max_block ? max_block : 4096u, hp, true);
    if (!err.empty()) return fail(KP_E_ARG, err);
    const kp_blockgen bg = blockgen_of(hp);
    uint64_t bad = 0;
    std::vector<uint8_t> seen(hp.g.nblocks, 0);
    for (uint64_t h = 0; h < hp.g.nblocks; ++h) {
        uint64_t hd, hn;
        const uint64_t q = kp_block_slot(hp.g, hp.tabs.data(), bg, hp.brank.data(), hp.hoff.data(), h, &hd, &hn);
        if (q >= hp.g.nblocks || seen[q] || hp.hlist[q] != h || hp.kpos[h] != q || hp.hdig[q] != hd || hp.hnp[q] != hn)
            ++bad;
        else
            seen[q] = 1;
    }
    *mismatches = bad;
    return KP_OK;
}

// The plan's device block list (kp_blocks_kernel, or the upload of an experiment order)
// against build_plan's host walk; *mismatches = differing entries of hlist, kpos, hdig
// and hnp together.
int kp_plan_block_check(kp_plan *p, uint64_t *mismatches) {
    if (!p || !mismatches) return fail(KP_E_ARG, "null argument");
    KP_HIP(hipSetDevice(p->ctx->device));
    kp::host_plan hp;  // the host walk with the plan's own block budget
    std::string err = kp::build_plan(p->hp.gp.c_str(), p->max_block, hp, true);
    if (!err.empty()) return fail(KP_E_ARG, err);
    if (hp.g.nblocks != p->hp.g.nblocks || hp.g.B != p->hp.g.B)
        return fail(KP_E_ARG, "the host walk does not rebuild the plan's block size");
    const uint64_t n = hp.g.nblocks;
    std::vector<uint32_t> hl(n), kp(n);
    std::vector<uint64_t> hd(n), hn(n);
    KP_HIP(hipStreamSynchronize(p->ctx->stream));
    KP_HIP(hipMemcpy(hl.data(), p->d_hlist, n * sizeof(uint32_t), hipMemcpyDeviceToHost));
    KP_HIP(hipMemcpy(kp.data(), p->d_kpos, n * sizeof(uint32_t), hipMemcpyDeviceToHost));
    KP_HIP(hipMemcpy(hd.data(), p->d_hdig, n * sizeof(uint64_t), hipMemcpyDeviceToHost));
    KP_HIP(hipMemcpy(hn.data(), p->d_hnp, n * sizeof(uint64_t), hipMemcpyDeviceToHost));
    uint64_t bad = 0;
    for (uint64_t q = 0; q < n; ++q)
        bad += (hl[q] != hp.hlist[q]) + (kp[q] != hp.kpos[q]) + (hd[q] != hp.hdig[q]) + (hn[q] != hp.hnp[q]);
    *mismatches = bad;
    return KP_OK;
}

}  // extern "C"

// (Re)allocate the count tables for nf folds (nf + 1 slots) and forget which folds are set.
template <typename CT>
static int counts_alloc(kp_plan *p, int nf) {
    const kp_geom &g = p->hp.g;
    if (p->cstream) KP_HIP(hipStreamSynchronize(p->cstream));  // no fold fill still writing the old tables
    size_t kbytes = g.nblocks * (size_t)g.n_kl * (nf + 1) * 2 * sizeof(CT);
    if (p->d_K && (p->nf != nf || p->ct_bytes != (int)sizeof(CT))) {
        dfree(p->d_K);
        p->d_K = nullptr;
    }
    if (!p->d_K) {
        size_t fr = 0, tot = 0;
        KP_HIP(hipMemGetInfo(&fr, &tot));
        if (kbytes + (64u << 20) > fr) return fail(KP_E_NOMEM, "count tables need " + std::to_string(kbytes) + " bytes");
        KP_HIP(dmalloc(&p->d_K, kbytes));
    }
    p->nf = nf;
    p->ct_bytes = (int)sizeof(CT);
    p->fold_set.assign(nf, 0);
    p->fold_async.assign(nf, 0);
    while ((int)p->fold_ev.size() < nf) {
        hipEvent_t e = nullptr;
        KP_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        p->fold_ev.push_back(e);
    }
    return KP_OK;
}

// Fill slots s0 .. s0+ncol-1 from [n_kmers][ncol] host arrays (one launch per high level:
// a level's aggregated rows sum two rows of lower levels).
template <typename CT>
static void counts_launch(kp_plan *p, hipStream_t st, const CT *dM, const CT *dU, uint32_t ncol, uint32_t s0,
                          hipError_t &e) {
    kp_geom g = p->hp.g;
    g.nf = p->nf;
    kp_dev_tables T = tables_of(p);
    for (int H = 0; H <= p->hp.hmax && e == hipSuccess; ++H) {
        uint64_t nb = p->hp.hoff[H + 1] - p->hp.hoff[H];
        if (!nb) continue;
        hipLaunchKernelGGL(kp_counts_kernel<CT>, dim3((unsigned)((nb + KP_CROWS - 1) / KP_CROWS)), dim3(256), 0, st, g,
                           T, p->hp.hoff[H], nb, H, dM, dU, ncol, s0, reinterpret_cast<CT *>(p->d_K));
        e = hipGetLastError();
    }
}

template <typename CT>
static int counts_fill(kp_plan *p, const void *M, const void *U, uint32_t ncol, uint32_t s0) {
    kp_ctx *c = p->ctx;
    const size_t in_bytes = p->hp.n_kmers * (size_t)ncol * sizeof(CT);
    CT *dM = nullptr, *dU = nullptr;
    KP_HIP(dmalloc(&dM, in_bytes));
    KP_HIP(dmalloc(&dU, in_bytes));
    hipError_t e = hipMemcpyAsync(dM, M, in_bytes, hipMemcpyHostToDevice, c->stream);
    if (e == hipSuccess) e = hipMemcpyAsync(dU, U, in_bytes, hipMemcpyHostToDevice, c->stream);
    counts_launch<CT>(p, c->stream, dM, dU, ncol, s0, e);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    dfree(dM);
    dfree(dU);
    if (e != hipSuccess) return fail(KP_E_HIP, std::string("count tables: ") + hipGetErrorString(e));
    return KP_OK;
}

// One fold's table, asynchronously on the plan's count stream: the counts are copied into
// pinned staging (once the previous fold's upload has left it), uploaded and aggregated on
// cstream, and fold_ev[fold] marks the end; run_pass makes the pass's stream wait for it.
template <typename CT>
static int counts_fill_async(kp_plan *p, int fold, const void *M, const void *U) {
    const size_t in_bytes = p->hp.n_kmers * sizeof(CT);
    if (!p->cstream) KP_HIP(hipStreamCreateWithFlags(&p->cstream, hipStreamNonBlocking));
    if (!p->stage_ev) KP_HIP(hipEventCreateWithFlags(&p->stage_ev, hipEventDisableTiming));
    if (p->stage_bytes < 2 * in_bytes) {
        KP_HIP(hipStreamSynchronize(p->cstream));
        dfree(p->d_stage);
        p->d_stage = nullptr;
        if (p->h_stage) KP_HIP(hipHostFree(p->h_stage));
        p->h_stage = nullptr;
        p->stage_bytes = 0;
        KP_HIP(hipHostMalloc(&p->h_stage, 2 * in_bytes, hipHostMallocDefault));
        KP_HIP(dmalloc(&p->d_stage, 2 * in_bytes));
        p->stage_bytes = 2 * in_bytes;
    }
    KP_HIP(hipEventSynchronize(p->stage_ev));  // the previous upload has left the pinned copy
    char *h = static_cast<char *>(p->h_stage);
    memcpy(h, M, in_bytes);
    memcpy(h + in_bytes, U, in_bytes);
    CT *dM = static_cast<CT *>(p->d_stage), *dU = dM + p->hp.n_kmers;
    hipError_t e = hipMemcpyAsync(dM, h, 2 * in_bytes, hipMemcpyHostToDevice, p->cstream);
    if (e == hipSuccess) e = hipEventRecord(p->stage_ev, p->cstream);
    counts_launch<CT>(p, p->cstream, dM, dU, 1, 1u + (uint32_t)fold, e);
    if (e == hipSuccess) e = hipEventRecord(p->fold_ev[fold], p->cstream);
    if (e != hipSuccess) return fail(KP_E_HIP, std::string("fold count table: ") + hipGetErrorString(e));
    p->fold_async[fold] = 1;
    return KP_OK;
}

// every fold at once: slot 0 = the sum over folds (exact in itype), slots 1.. = the folds
template <typename CT>
static int run_counts(kp_plan *p, const void *M, const void *U, uint64_t n_kmers, int nf) {
    const CT *m = static_cast<const CT *>(M), *u = static_cast<const CT *>(U);
    std::vector<CT> tm(n_kmers), tu(n_kmers);
    for (uint64_t i = 0; i < n_kmers; ++i) {
        CT a = 0, b = 0;
        for (int f = 0; f < nf; ++f) {
            a += m[i * nf + f];
            b += u[i * nf + f];
        }
        tm[i] = a;
        tu[i] = b;
    }
    if (int rc = counts_alloc<CT>(p, nf)) return rc;
    if (int rc = counts_fill<CT>(p, tm.data(), tu.data(), 1, 0)) return rc;
    if (int rc = counts_fill<CT>(p, M, U, (uint32_t)nf, 1)) return rc;
    std::fill(p->fold_set.begin(), p->fold_set.end(), (uint8_t)1);
    return KP_OK;
}

extern "C" {

int kp_set_counts(kp_plan *p, const void *M, const void *U, uint64_t n_kmers, int nf, int itype_bytes) {
    if (!p || !M || !U) return fail(KP_E_ARG, "null argument");
    if (n_kmers != p->hp.n_kmers)
        return fail(KP_E_ARG, "n_kmers " + std::to_string(n_kmers) + " != " + std::to_string(p->hp.n_kmers));
    if (nf < 1 || nf > 64) return fail(KP_E_ARG, "nf must be 1..64");
    KP_HIP(hipSetDevice(p->ctx->device));
    if (itype_bytes == 4) return run_counts<uint32_t>(p, M, U, n_kmers, nf);
    if (itype_bytes == 8) return run_counts<uint64_t>(p, M, U, n_kmers, nf);
    return fail(KP_E_ARG, "itype_bytes must be 4 or 8");
}

int kp_counts_begin(kp_plan *p, const void *M_all, const void *U_all, uint64_t n_kmers, int nf, int itype_bytes) {
    if (!p || !M_all || !U_all) return fail(KP_E_ARG, "null argument");
    if (n_kmers != p->hp.n_kmers)
        return fail(KP_E_ARG, "n_kmers " + std::to_string(n_kmers) + " != " + std::to_string(p->hp.n_kmers));
    if (nf < 1 || nf > 64) return fail(KP_E_ARG, "nf must be 1..64");
    if (itype_bytes != 4 && itype_bytes != 8) return fail(KP_E_ARG, "itype_bytes must be 4 or 8");
    KP_HIP(hipSetDevice(p->ctx->device));
    if (itype_bytes == 4) {
        if (int rc = counts_alloc<uint32_t>(p, nf)) return rc;
        return counts_fill<uint32_t>(p, M_all, U_all, 1, 0);
    }
    if (int rc = counts_alloc<uint64_t>(p, nf)) return rc;
    return counts_fill<uint64_t>(p, M_all, U_all, 1, 0);
}

int kp_counts_fold(kp_plan *p, int fold, const void *M_fold, const void *U_fold, uint64_t n_kmers) {
    if (!p || !M_fold || !U_fold) return fail(KP_E_ARG, "null argument");
    if (!p->d_K) return fail(KP_E_STATE, "kp_counts_begin must come first");
    if (n_kmers != p->hp.n_kmers)
        return fail(KP_E_ARG, "n_kmers " + std::to_string(n_kmers) + " != " + std::to_string(p->hp.n_kmers));
    if (fold < 0 || fold >= p->nf) return fail(KP_E_ARG, "fold out of range");
    KP_HIP(hipSetDevice(p->ctx->device));
    int rc = p->ct_bytes == 4 ? counts_fill_async<uint32_t>(p, fold, M_fold, U_fold)
                              : counts_fill_async<uint64_t>(p, fold, M_fold, U_fold);
    if (rc == KP_OK) p->fold_set[fold] = 1;
    return rc;
}

}  // extern "C"

// dynamic LDS of kp_dp_kernel (carve order and rounding exactly as in the kernel)
static size_t dp_lds_bytes(const kp::host_plan &hp, int nl, size_t ct_bytes) {
    const kp_geom &g = hp.g;
    const size_t st = (size_t)nl * g.Bpad * 4;
    const size_t scratch = (((size_t)hp.pscratch_entries * 4 * ct_bytes) + 15) & ~(size_t)15;  // 2 build buffers
    const size_t ptab = ((((size_t)hp.ptab_entries * 2 + 3) & ~(size_t)3)) * ct_bytes;
    return std::max(st, scratch) + ptab + (size_t)(g.kh * 7 + 1) * sizeof(kp_hpair) +
           (((size_t)g.t * 16 + 15) & ~(size_t)15) + 16
#ifdef KP_STAMPS
           + 32 * sizeof(unsigned long long)
#endif
        ;
}

template <typename CT, int NL, bool HZ, bool MIX>
static int launch_dp_hz(hipStream_t st, const kp_dp_params &P, unsigned nb, unsigned ngroups, int threads, size_t lds) {
    if constexpr (kp_sdwa_on<NL, MIX>()) {  // its scan reads the row array at LDS address 0 (kp_at_bytes)
        static std::atomic<bool> checked{false};
        if (!checked.load(std::memory_order_relaxed)) {
            hipFuncAttributes fa;
            KP_HIP(hipFuncGetAttributes(&fa, reinterpret_cast<const void *>(&kp_dp_kernel<CT, NL, HZ, MIX>)));
            if (fa.sharedSizeBytes != 0)
                return fail(KP_E_HIP, "kp_dp_kernel has static LDS: its dynamic LDS does not start at address 0");
            checked.store(true, std::memory_order_relaxed);
        }
    }
    if (lds > 65536)
        KP_HIP(hipFuncSetAttribute(reinterpret_cast<const void *>(&kp_dp_kernel<CT, NL, HZ, MIX>),
                                   hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    hipLaunchKernelGGL((kp_dp_kernel<CT, NL, HZ, MIX>), dim3(nb, ngroups), dim3(threads), lds, st, P);
    KP_HIP(hipGetLastError());
    return KP_OK;
}

// Groups of 1-3 lanes (80 VGPRs at 6 waves per SIMD) run high levels >= 1 without the
// k-mer code (fewer spills: 1-lane pass 149 -> 144 ms); wider groups keep one kernel for
// every level (the split build measured slower there: 5 lanes 395 -> 402 ms)
// (the mixed builds always split: their k-mer code adds register spills at every width)
template <typename CT, int NL, bool MIX>
static int launch_dp(hipStream_t st, const kp_dp_params &P, unsigned nb, unsigned ngroups, int threads, size_t lds) {
    constexpr bool one_build = NL > 3 && !MIX;  // (mixed, one build for all levels: +1-2 ms)
    return (P.H == 0 || one_build) ? launch_dp_hz<CT, NL, true, MIX>(st, P, nb, ngroups, threads, lds)
                                : launch_dp_hz<CT, NL, false, MIX>(st, P, nb, ngroups, threads, lds);
}

// mixed groups (two (alpha, beta) sets) need at least 2 lanes
template <typename CT, int NL>
static int launch_dp_mix(bool mix, hipStream_t st, const kp_dp_params &P, unsigned nb, unsigned ngroups, int threads,
                         size_t lds) {
    if constexpr (NL >= 2) {
        if (mix) return launch_dp<CT, NL, true>(st, P, nb, ngroups, threads, lds);
    }
    return launch_dp<CT, NL, false>(st, P, nb, ngroups, threads, lds);
}

template <typename CT>
static int launch_dp_nl(int nl, bool mix, hipStream_t c, const kp_dp_params &P, unsigned nb, unsigned ngroups,
                        int threads, size_t lds) {
    switch (nl) {
        case 1: return launch_dp_mix<CT, 1>(mix, c, P, nb, ngroups, threads, lds);
        case 2: return launch_dp_mix<CT, 2>(mix, c, P, nb, ngroups, threads, lds);
        case 3: return launch_dp_mix<CT, 3>(mix, c, P, nb, ngroups, threads, lds);
        case 4: return launch_dp_mix<CT, 4>(mix, c, P, nb, ngroups, threads, lds);
        case 5: return launch_dp_mix<CT, 5>(mix, c, P, nb, ngroups, threads, lds);
        case 6: return launch_dp_mix<CT, 6>(mix, c, P, nb, ngroups, threads, lds);
        case 7: return launch_dp_mix<CT, 7>(mix, c, P, nb, ngroups, threads, lds);
        case 8: return launch_dp_mix<CT, 8>(mix, c, P, nb, ngroups, threads, lds);
    }
    return fail(KP_E_ARG, "lanes per workgroup must be 1..8");
}

// The wave-specialised persistent sweep (kp_dp_ws.h) for 1-lane device groups above high
// level 0, with KP_WS=1 (A/B; off by default until it measures faster).
static bool ws_enabled() {
    const char *e = getenv("KP_WS");
    return e && atoi(e) != 0;
}

// its build buffers: the largest count table before the last step (T_0 .. T_{t-2})
static uint32_t ws_scratch_entries(const kp::host_plan &hp) {
    const kp_geom &g = hp.g;
    uint64_t R = 1, mx = 1;
    for (int s = 0; s + 1 < g.t; ++s) {
        uint64_t nn = 1;
        for (int i = s; i < g.t; ++i) nn *= g.n[i];
        mx = std::max<uint64_t>(mx, R * nn);
        R *= g.r[s];
    }
    return (uint32_t)mx;
}

// dynamic LDS of kp_dp_ws_kernel (carve order as in the kernel)
static size_t ws_lds_bytes(const kp::host_plan &hp, size_t ct_bytes) {
    const kp_geom &g = hp.g;
    const size_t ptab = (((size_t)hp.ptab_entries * 2 + 3) & ~(size_t)3) * ct_bytes;
    const size_t scr = (((size_t)ws_scratch_entries(hp) * 2 + 3) & ~(size_t)3) * ct_bytes;
    return 2 * (size_t)KP_WS_BASE1 + 2 * ptab + 2 * scr + (size_t)(g.kh * 7 + 1) * sizeof(kp_hpair) +
           (((size_t)g.t * 16 + 15) & ~(size_t)15) + sizeof(kp_ws_sync);
}

// can this launch (one high level of a class of nl-lane device groups) run on the
// wave-specialised sweep?  Its slots need a level per count-table step and a gather slot,
// its row buffers a block of <= 4128 floats, its consumers every level's cells
static bool ws_fits(const kp::host_plan &hp, const kp_dp_params &P, int nl, bool mix, size_t ct_bytes,
                    size_t lds_max) {
    if (!ws_enabled() || nl != 1 || mix || P.H == 0 || !P.T.hpd || !P.lanesplit) return false;
    const kp_geom &g = hp.g;
    const int L = hp.lmax + 1;
    if (L < 2 || g.t > L || (size_t)g.Bpad * 4 > KP_WS_BASE1) return false;
    for (int l = 0; l <= hp.lmax; ++l)
        if (hp.loff[l + 1] - hp.loff[l] > KP_WS_CW * 64 * KP_IPT) return false;
    return ws_lds_bytes(hp, ct_bytes) <= std::min<size_t>(lds_max, 80u * 1024u);  // two workgroups per CU
}

template <typename CT>
static int launch_ws(hipStream_t st, const kp_dp_params *dP, unsigned nb, unsigned ngroups, int cus, size_t lds) {
    static std::atomic<bool> checked{false};
    if (!checked.load(std::memory_order_relaxed)) {  // its scan reads the row buffers at fixed LDS addresses
        hipFuncAttributes fa;
        KP_HIP(hipFuncGetAttributes(&fa, reinterpret_cast<const void *>(&kp_dp_ws_kernel<CT, 1>)));
        if (fa.sharedSizeBytes != 0) return fail(KP_E_HIP, "kp_dp_ws_kernel has static LDS");
        checked.store(true, std::memory_order_relaxed);
    }
    if (lds > 65536)
        KP_HIP(hipFuncSetAttribute(reinterpret_cast<const void *>(&kp_dp_ws_kernel<CT, 1>),
                                   hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    // persistent: as many workgroups as are resident at once (waves per SIMD x 4 SIMDs per CU
    // over the workgroup's waves; LDS), shared by the class's device groups, a multiple of 8
    // per group (one XCD per workgroup's blocks)
    const int per_cu = std::max(1, std::min<int>((4 * KP_WS_WAVES) / (KP_WS_THREADS / 64),
                                                 (int)((160u * 1024u) / std::max<size_t>(lds, 1))));
    unsigned wmax = (unsigned)std::max(8, (per_cu * cus / (int)std::max(1u, ngroups)) & ~7);
    const unsigned W = std::min(nb, wmax);
    hipLaunchKernelGGL((kp_dp_ws_kernel<CT, 1>), dim3(W, ngroups), dim3(KP_WS_THREADS), lds, st, dP, nb);
    KP_HIP(hipGetLastError());
    return KP_OK;
}

static int dp_threads() {
    const char *e = getenv("KP_DP_THREADS");
    int v = e ? atoi(e) : 512;
    return (v == 64 || v == 128 || v == 256 || v == 512 || v == 1024) ? v : 512;
}

// a wide group's lanes as full workgroups first (7 lanes as 5 + 2: 9-mer pass 603 -> 593
// ms, profiles/r03/experiments/wide_split.txt); KP_WIDE_SPLIT=0: near-equal (4 + 3)
static bool wide_split_greedy() {
    const char *e = getenv("KP_WIDE_SPLIT");
    return !e || atoi(e) != 0;
}

static int lanes_per_wg_default() {
    const char *e = getenv("KP_LANES_PER_WG");
    int v = e ? atoi(e) : 5;
    return std::min(std::max(v, 1), KP_GROUP_LANES);
}

// lanes per workgroup of the sweep: KP_LANES_PER_WG (default 5), fewer if two workgroups
// per CU would not fit LDS (KP_LDS_BUDGET: another per-workgroup budget; A/B only)
static int wg_lanes(const kp::host_plan &hp, size_t ct_bytes, size_t lds_max) {
    int per_wg = lanes_per_wg_default();
    const size_t lds_two = std::min<size_t>(lds_max, getenv("KP_LDS_BUDGET") ? (size_t)atol(getenv("KP_LDS_BUDGET"))
                                                                            : 160u * 1024u / 2u);
    while (per_wg > 1 && dp_lds_bytes(hp, per_wg, ct_bytes) > lds_two) --per_wg;
    return per_wg;
}

// Score rows + backtrack node pool for `lanes` lanes.  Grown only (a pass with fewer lanes
// uses the front of the buffers), never cleared: every pass writes every row of its lanes
// before any read.  Freeing and re-allocating a large buffer is slow on this platform
// (the driver wipes freed memory before handing it out again: ~4 s for 100-150 GB,
// tools/alloc_probe.hip), so callers reserve the largest pass up front (kp_reserve_lanes).
// ---- the score rows: the one very large allocation ----
// Plain hipMalloc.  A hipMalloc of HBM that was used before waits for the driver's wipe
// (~30 ms per GB); the device's stream-ordered pool does not, but re-serving a freed pool
// block for a larger request returned memory that does not hold what is written to it
// (tools/async_check.hip), so the pool is NOT used by default.  Opt-in only
// (KP_POOL_SCORES=1, for allocation-time experiments): then the FIRST score buffer of a
// process on a device comes from the pool (nothing was ever freed there) and is written
// with a pattern and read back before use; every later one comes from hipMalloc.
static std::atomic<bool> g_pool_touched[64];

__global__ void kp_fill_pattern(uint32_t *p, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        p[i] = (uint32_t)(i * 2654435761u) ^ 0x5bd1e995u;
}

__global__ void kp_check_pattern(const uint32_t *p, size_t n, unsigned long long *bad) {
    unsigned long long b = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        b += (p[i] != ((uint32_t)(i * 2654435761u) ^ 0x5bd1e995u));
    for (int off = 32; off > 0; off >>= 1) b += __shfl_xor(b, off, 64);
    if ((threadIdx.x & 63u) == 0 && b) atomicAdd(bad, b);
}

static void free_scores(kp_plan *p) {
    if (!p->d_S) return;
    if (p->S_pool) {
        (void)hipFreeAsync(p->d_S, p->ctx->stream);
        (void)hipStreamSynchronize(p->ctx->stream);
    } else {
        (void)hipFree(p->d_S);
    }
    p->d_S = nullptr;
    p->S_pool = false;
}

static int alloc_scores(kp_plan *p, size_t bytes) {
    kp_ctx *c = p->ctx;
    const char *e = getenv("KP_POOL_SCORES");
    const bool allow = e && atoi(e) == 1 && c->device >= 0 && c->device < 64;
    if (allow && !g_pool_touched[c->device].exchange(true)) {
        void *q = nullptr;
        if (hipMallocAsync(&q, bytes, c->stream) == hipSuccess && hipStreamSynchronize(c->stream) == hipSuccess) {
            unsigned long long *d_bad = nullptr, bad = 1;
            const size_t n = bytes / 4;
            if (hipMalloc(&d_bad, sizeof(bad)) == hipSuccess &&
                hipMemsetAsync(d_bad, 0, sizeof(bad), c->stream) == hipSuccess) {
                hipLaunchKernelGGL(kp_fill_pattern, dim3(16384), dim3(256), 0, c->stream, (uint32_t *)q, n);
                hipLaunchKernelGGL(kp_check_pattern, dim3(16384), dim3(256), 0, c->stream, (const uint32_t *)q, n,
                                   d_bad);
                if (hipMemcpyAsync(&bad, d_bad, sizeof(bad), hipMemcpyDeviceToHost, c->stream) != hipSuccess ||
                    hipStreamSynchronize(c->stream) != hipSuccess)
                    bad = 1;
            }
            if (d_bad) (void)hipFree(d_bad);
            if (bad == 0) {
                p->d_S = static_cast<float *>(q);
                p->S_pool = true;
                return KP_OK;
            }
            (void)hipFreeAsync(q, c->stream);
            (void)hipStreamSynchronize(c->stream);
        }
        (void)hipGetLastError();  // fall back to hipMalloc below
    }
    KP_HIP(dmalloc(&p->d_S, bytes));
    p->S_pool = false;
    return KP_OK;
}

static int ensure_lanes(kp_plan *p, uint64_t lanes) {
    if (lanes <= p->lanes_cap) return KP_OK;
    const kp::host_plan &hp = p->hp;
    const uint32_t ncap = node_cap_of(hp);
    free_scores(p);
    dfree(p->d_nodes);
    p->d_S = nullptr;
    p->d_nodes = nullptr;
    p->lanes_cap = 0;
    size_t sb = hp.g.nblocks * (size_t)lanes * hp.g.Bpad * 4, nb = (size_t)lanes * ncap * sizeof(kp_node);
    size_t fr = 0, tot = 0;
    KP_HIP(hipMemGetInfo(&fr, &tot));
    if (sb + nb + (256u << 20) > fr)
        return fail(KP_E_NOMEM, "lanes need " + std::to_string(sb + nb) + " bytes, free " + std::to_string(fr));
    if (int rc = alloc_scores(p, sb)) return rc;
    KP_HIP(dmalloc(&p->d_nodes, nb));
    p->lanes_cap = lanes;
    p->node_cap = ncap;
    return KP_OK;
}

// The device groups of a pass (host code; kp_pass, and kp_device_groups for tests): user
// groups in order, lanes group-major, lane0 = first lane of each device group
static void plan_device_groups(const kp_group *groups, int n_groups, int per_wg, std::vector<kp_group_dev> &dg) {
    dg.clear();
    uint32_t lane = 0;
    // lanes [s, s + n) of the run of user groups g0.. (group-major) as one device group;
    // lanes of a second user group with another (alpha, beta) become the mixed set 2
    auto chunk = [&](int g0, int s, int n) -> bool {
        kp_group_dev d;
        memset(&d, 0, sizeof(d));
        d.fold = groups[g0].fold;
        d.lane0 = (int32_t)lane;
        d.nl = n;
        d.alpha = d.alpha2 = groups[g0].alpha;
        d.beta = d.beta2 = groups[g0].beta;
        int gi = g0, off = s;
        while (off >= groups[gi].n_lanes) off -= groups[gi++].n_lanes;
        const int first = gi;
        for (int j = 0; j < n; ++j, ++off) {
            if (off == groups[gi].n_lanes) {
                off = 0;
                ++gi;
            }
            const kp_group &u = groups[gi];
            if (j == 0) {
                d.alpha = d.alpha2 = u.alpha;
                d.beta = d.beta2 = u.beta;
            } else if (gi != first) {
                if (gi > first + 1) return false;  // at most two user groups per device group
                const bool same = u.alpha == groups[first].alpha && u.beta == groups[first].beta;
                if (!same && d.nl2 == 0) {
                    d.alpha2 = u.alpha;
                    d.beta2 = u.beta;
                }
                if (!same) ++d.nl2;
            }
            d.pen[j] = u.penalty[off];
        }
        dg.push_back(d);
        lane += (uint32_t)n;
        return true;
    };
    // Each user group becomes as few device groups as the workgroup width allows, full
    // workgroups first (wide_split_greedy).  Consecutive user groups of the same fold share their count tables: when
    // cutting the run's lanes together gives fewer device groups, they are cut together
    // (mixed groups, e.g. the 2 + 3 lanes of two alphas as one 5-lane group; at most two
    // (alpha, beta) sets each; KP_MIX_GROUPS=0 disables)
    const bool mixing = !getenv("KP_MIX_GROUPS") || atoi(getenv("KP_MIX_GROUPS")) != 0;
    for (int i = 0; i < n_groups;) {
        int e = i + 1, tot = groups[i].n_lanes, sep = (groups[i].n_lanes + per_wg - 1) / per_wg;
        while (mixing && e < n_groups && groups[e].fold == groups[i].fold) {
            tot += groups[e].n_lanes;
            sep += (groups[e].n_lanes + per_wg - 1) / per_wg;
            ++e;
        }
        const int nd = (tot + per_wg - 1) / per_wg;
        bool merged = false;
        if (e > i + 1 && nd < sep) {
            const size_t dg0 = dg.size();
            const uint32_t lane0 = lane;
            merged = true;
            for (int q = 0, s = 0; q < nd && merged; ++q) {
                const int n = wide_split_greedy() ? std::min(per_wg, tot - s) : tot / nd + (q < tot % nd ? 1 : 0);
                merged = chunk(i, s, n);
                s += n;
            }
            if (!merged) {  // a chunk would span three user groups: cut them one by one
                dg.resize(dg0);
                lane = lane0;
            }
        }
        if (!merged)
            for (int q = i; q < e; ++q) {
                const kp_group &u = groups[q];
                const int nq = (u.n_lanes + per_wg - 1) / per_wg;
                for (int r = 0, s = 0; r < nq; ++r) {
                    const int n = wide_split_greedy() ? std::min(per_wg, u.n_lanes - s)
                                                      : u.n_lanes / nq + (r < u.n_lanes % nq ? 1 : 0);
                    chunk(q, s, n);
                    s += n;
                }
            }
        i = e;
    }
}

template <typename CT>
static int run_pass(kp_plan *p, const kp_group *groups, int n_groups, float *root_train, float *root_test,
                    uint64_t *n_leaves) {
    auto t0 = std::chrono::steady_clock::now();
    kp_ctx *c = p->ctx;
    const kp::host_plan &hp = p->hp;
    kp_geom g = hp.g;
    g.nf = p->nf;
    // split user groups into device groups that fit two workgroups per CU in LDS when
    // possible (LDS is the occupancy limit of the sweep)
    const int per_wg = wg_lanes(hp, sizeof(CT), c->lds_max);
    if (dp_lds_bytes(hp, 1, sizeof(CT)) > c->lds_max) return fail(KP_E_ARG, "block does not fit LDS");
    for (int i = 0; i < n_groups; ++i) {
        const kp_group &u = groups[i];
        if (u.n_lanes < 1 || u.n_lanes > KP_GROUP_MAX_LANES) return fail(KP_E_ARG, "group lanes must be 1..8");
        if (u.fold >= p->nf || u.fold < -1) return fail(KP_E_ARG, "fold out of range");
        if (u.fold >= 0 && !p->fold_set[u.fold])
            return fail(KP_E_STATE, "counts of fold " + std::to_string(u.fold) + " are not set (kp_counts_fold)");
    }
    for (int i = 0; i < n_groups; ++i)  // folds whose tables are still filling on the count stream
        if (groups[i].fold >= 0 && p->fold_async[groups[i].fold])
            KP_HIP(hipStreamWaitEvent(c->stream, p->fold_ev[groups[i].fold], 0));
    std::vector<kp_group_dev> dg;
    plan_device_groups(groups, n_groups, per_wg, dg);
    uint32_t lane = 0;
    for (const kp_group_dev &d : dg) lane += (uint32_t)d.nl;
    const uint32_t Ltot = lane;
    g.Ltot = Ltot;
    // launch classes: device groups with equal lane counts share one launch per level
    std::stable_sort(dg.begin(), dg.end(), [](const kp_group_dev &a, const kp_group_dev &b) { return a.nl > b.nl; });
    std::vector<uint32_t> lanegrp(Ltot, 0);
    for (size_t i = 0; i < dg.size(); ++i)
        for (int j = 0; j < dg[i].nl; ++j) lanegrp[dg[i].lane0 + j] = (uint32_t)i;
    // threads per workgroup: every level of the block must fit KP_IPT cells per thread
    int max_level_cells = 0;
    for (int l = 0; l <= hp.lmax; ++l) max_level_cells = std::max(max_level_cells, hp.loff[l + 1] - hp.loff[l]);
    int threads = dp_threads();
    while (threads < KP_DP_MAX_THREADS && threads * KP_IPT < max_level_cells) threads *= 2;
    if (threads * KP_IPT < max_level_cells) return fail(KP_E_ARG, "block level too wide for one workgroup");
    // lane storage: scores, and the backtrack node pool
    if (int rc = ensure_lanes(p, Ltot)) return rc;
    if (Ltot > p->small_cap || dg.size() > p->small_cap) {
        void *bufs[] = {p->d_groups, p->d_lanegrp, p->d_rtrain, p->d_rtest, p->d_nleaves,
                        p->d_bad,    p->d_cnt,     p->d_dend,   p->d_leaves};
        for (void *b : bufs) dfree(b);
        uint64_t cap = std::max<uint64_t>(Ltot, 64);
        KP_HIP(dmalloc(&p->d_groups, cap * sizeof(kp_group_dev)));
        KP_HIP(dmalloc(&p->d_lanegrp, cap * sizeof(uint32_t)));
        KP_HIP(dmalloc(&p->d_rtrain, cap * sizeof(float)));
        KP_HIP(dmalloc(&p->d_rtest, cap * sizeof(float)));
        KP_HIP(dmalloc(&p->d_nleaves, cap * sizeof(uint64_t)));
        KP_HIP(dmalloc(&p->d_bad, cap * sizeof(uint32_t)));
        KP_HIP(dmalloc(&p->d_cnt, cap * sizeof(uint32_t)));
        KP_HIP(dmalloc(&p->d_dend, cap * (KP_MAXDEPTH + 1) * sizeof(uint32_t)));
        KP_HIP(dmalloc(&p->d_leaves, cap * hp.n_kmers * sizeof(uint64_t)));
        p->small_cap = cap;
    }
    KP_HIP(hipMemcpyAsync(p->d_groups, dg.data(), dg.size() * sizeof(kp_group_dev), hipMemcpyHostToDevice, c->stream));
    KP_HIP(hipMemcpyAsync(p->d_lanegrp, lanegrp.data(), lanegrp.size() * sizeof(uint32_t), hipMemcpyHostToDevice,
                          c->stream));

    kp_dp_params P;
    memset(&P, 0, sizeof(P));
    P.g = g;
    P.T = tables_of(p);
    P.K = p->d_K;
    P.S = p->d_S;
    P.groups = p->d_groups;
    P.lmax = hp.lmax;
    if (hp.lmax > KP_DP_MAX_LEVELS) return fail(KP_E_ARG, "too many low levels");
    for (int l = 0; l <= hp.lmax + 1; ++l) P.loffv[l] = hp.loff[l];
    for (int l = 0; l <= hp.lmax; ++l)  // (the sweep's descriptor loads assume every level holds a cell)
        if (hp.loff[l + 1] <= hp.loff[l]) return fail(KP_E_ARG, "empty low level");
    P.ptab_entries = hp.ptab_entries;
    P.pscratch_entries = hp.pscratch_entries;
    P.wscratch_entries = ws_scratch_entries(hp);
#ifdef KP_ABLATION
    // timing-ablation build only (make ablation -> libkmerpapa_hip_ablation.so): phases
    // skipped by KP_DEBUG_SKIP give wrong scores, so the pass reports KP_E_STATE below
    P.dbg = getenv("KP_DEBUG_SKIP") ? atoi(getenv("KP_DEBUG_SKIP")) : 0;
#else
    P.dbg = 0;  // the product build has no phase-skipping path
#endif
    // runs of 40 consecutive blocks per XCD (workgroups are dealt round-robin over the 8
    // XCDs): neighbours in the reuse order share their L2; measured -1 % against none
    // (DESIGN.md §5), 16 against 8 -1.5 ms per 5-lane pass (12: -1.2, 32: -0.4), 24 against
    // 16 -1 ms (20: -0.5) and 40 against 24 -1 ms (32: +2, 64: +5; non-monotonic;
    // profiles/r04/experiments/remap_ab.txt)
    P.remap = getenv("KP_XCD_REMAP") ? atoi(getenv("KP_XCD_REMAP")) : 40;
    P.lanesplit = getenv("KP_LANE_SPLIT") ? atoi(getenv("KP_LANE_SPLIT")) : 1;
    // KP_EXACT_LOGS=1: no fast device log at all (same results; exercises the exact path)
    P.exact = getenv("KP_EXACT_LOGS") ? atoi(getenv("KP_EXACT_LOGS")) : 0;
    P.ntstore = getenv("KP_NT_STORE") ? atoi(getenv("KP_NT_STORE")) : 1;
    // child rows along the KP_NT_SLOW slowest-varying high positions of the block order
    // (default 3) are read non-temporally: under that order they are not re-read while
    // still in the Infinity Cache, so they no longer evict the rows of the fast positions
    // that are (9-mer pass 403-408 -> 397-398 ms; 2: 399-400, 4: 417)
    // KP_NT_SLOW_H = comma list: a count per high level (launch), for per-launch tuning;
    // levels past the list (or without it) take KP_NT_SLOW
    std::vector<uint32_t> ntmask_h(hp.hmax + 1, 0);
    {
        const int nslow = getenv("KP_NT_SLOW") ? atoi(getenv("KP_NT_SLOW")) : 3;
        std::vector<int> per(hp.hmax + 1, nslow);
        if (const char *e = getenv("KP_NT_SLOW_H")) {
            int H = 0;
            for (const char *q = e; *q && H <= hp.hmax; ++H) {
                per[H] = atoi(q);
                while (*q && *q != ',') ++q;
                if (*q == ',') ++q;
            }
        }
        // (counted among the positions that have split pairs: a fixed base of the general
        // pattern, radix 1, sits last in the block order but has no child rows -- the 11-mer
        // super pattern ANNNNMNNNNA has one, which left it with two non-temporal positions)
        std::vector<int> slow_order;
        for (int q = (int)hp.perm.size() - 1; q >= 0; --q)
            if (g.r[g.t + hp.perm[q]] > 1) slow_order.push_back(hp.perm[q]);
        for (int H = 0; H <= hp.hmax; ++H)
            for (int q = 0; q < per[H] && q < (int)slow_order.size(); ++q) ntmask_h[H] |= 1u << slow_order[q];
        P.ntmask = ntmask_h[0];
    }
    P.stamps = nullptr;
#ifdef KP_STAMPS
    static unsigned long long *d_stamps = nullptr;
    if (!d_stamps) KP_HIP(dmalloc(&d_stamps, 32 * sizeof(unsigned long long)));
    KP_HIP(hipMemsetAsync(d_stamps, 0, 32 * sizeof(unsigned long long), c->stream));
    P.stamps = d_stamps;
#endif
    KP_HIP(hipEventRecord(c->ev[0], c->stream));
    // lane classes: runs of device groups with equal lane counts (dg is sorted by width);
    // one launch per (class, high level).  With several classes and KP_CLASS_STREAMS=1,
    // class q > 0 runs its whole launch sequence on side stream q - 1
    std::vector<std::pair<size_t, size_t>> classes;
    for (size_t i = 0; i < dg.size();) {
        size_t j = i;
        while (j < dg.size() && dg[j].nl == dg[i].nl) ++j;
        classes.emplace_back(i, j);
        i = j;
    }
    // the launches that run on the wave-specialised sweep (kp_dp_ws.h) read their parameters
    // from device memory: all of the pass's, uploaded once before the first launch
    auto launch_params = [&](size_t i, int H) {
        kp_dp_params Q = P;
        Q.hbase = hp.hoff[H];
        Q.H = H;
        Q.groups = p->d_groups + i;
        Q.ntmask = ntmask_h[H];
        return Q;
    };
    if (!p->d_werr) KP_HIP(dmalloc(&p->d_werr, sizeof(uint32_t)));
    KP_HIP(hipMemsetAsync(p->d_werr, 0, sizeof(uint32_t), c->stream));
    P.werr = p->d_werr;
    std::vector<kp_dp_params> wsq;
    std::vector<int> wsat(classes.size() * (size_t)(hp.hmax + 1), -1);
    for (size_t q = 0; q < classes.size(); ++q) {
        const size_t i = classes[q].first, j = classes[q].second;
        bool mix = false;
        for (size_t q2 = i; q2 < j; ++q2) mix = mix || dg[q2].nl2 > 0;
        for (int H = 0; H <= hp.hmax; ++H) {
            if (hp.hoff[H + 1] == hp.hoff[H]) continue;
            const kp_dp_params Q = launch_params(i, H);
            if (ws_fits(hp, Q, dg[i].nl, mix, sizeof(CT), c->lds_max)) {
                wsat[q * (hp.hmax + 1) + H] = (int)wsq.size();
                wsq.push_back(Q);
            }
        }
    }
    if (!wsq.empty()) {
        if (wsq.size() > p->wsp_cap) {
            dfree(p->d_wsp);
            p->d_wsp = nullptr;
            p->wsp_cap = 0;
            KP_HIP(dmalloc(&p->d_wsp, wsq.size() * sizeof(kp_dp_params)));
            p->wsp_cap = wsq.size();
        }
        KP_HIP(hipMemcpyAsync(p->d_wsp, wsq.data(), wsq.size() * sizeof(kp_dp_params), hipMemcpyHostToDevice,
                              c->stream));
    }
    // KP_CLASS_STREAMS=1 runs the classes concurrently.  Off by default: measured on one
    // MI355X, 9-mer passes of 4+3 lanes (one 7-penalty group) 620 -> 603 ms and 5+1 / 4+2
    // (two groups) -0.5 %, but the 11-mer step (4+3 lanes, ANNNNMNNNNA) 606 -> 627 ms
    const bool multi = classes.size() > 1 && getenv("KP_CLASS_STREAMS") && atoi(getenv("KP_CLASS_STREAMS")) == 1;
    if (multi) {
        KP_HIP(hipEventRecord(c->ev[3], c->stream));
        for (size_t q = 1; q < classes.size() && q <= KP_SIDE_STREAMS; ++q)
            KP_HIP(hipStreamWaitEvent(c->side[q - 1], c->ev[3], 0));
    }
    uint64_t launches = 0;
    // KP_LAUNCH_TIMES=1: HIP events around every launch (kp_last_launch_ms; tuning only)
    const bool timed = getenv("KP_LAUNCH_TIMES") && atoi(getenv("KP_LAUNCH_TIMES")) == 1;
    for (size_t q = 0; q < classes.size(); ++q) {
        const hipStream_t st = (multi && q > 0) ? c->side[(q - 1) % KP_SIDE_STREAMS] : c->stream;
        const size_t i = classes[q].first, j = classes[q].second;
        for (int H = 0; H <= hp.hmax; ++H) {
            uint64_t nb = hp.hoff[H + 1] - hp.hoff[H];
            if (!nb) continue;
            kp_dp_params Q = P;
            Q.hbase = hp.hoff[H];
            Q.H = H;
            Q.groups = p->d_groups + i;
            Q.ntmask = ntmask_h[H];
            size_t lds = dp_lds_bytes(hp, dg[i].nl, sizeof(CT));
#ifdef KP_ABLATION
            // ablation build only: extra LDS per workgroup to force lower occupancy
            if (getenv("KP_LDS_PAD")) lds += (size_t)atol(getenv("KP_LDS_PAD"));
#endif
            if (timed) {
                while (p->lev.size() < 2 * (launches + 1)) {
                    hipEvent_t e;
                    KP_HIP(hipEventCreate(&e));
                    p->lev.push_back(e);
                }
                KP_HIP(hipEventRecord(p->lev[2 * launches], st));
            }
            bool mix = false;
            for (size_t q2 = i; q2 < j; ++q2) mix = mix || dg[q2].nl2 > 0;
            int rc;
            const int wi = wsat[q * (hp.hmax + 1) + H];
            if (wi >= 0)
                rc = launch_ws<CT>(st, p->d_wsp + wi, (unsigned)nb, (unsigned)(j - i), c->cus,
                                   ws_lds_bytes(hp, sizeof(CT)));
            else
                rc = launch_dp_nl<CT>(dg[i].nl, mix, st, Q, (unsigned)nb, (unsigned)(j - i), threads, lds);
            if (rc) return rc;
            if (timed) KP_HIP(hipEventRecord(p->lev[2 * launches + 1], st));
            ++launches;
        }
    }
    if (multi)
        for (size_t q = 1; q < classes.size() && q <= KP_SIDE_STREAMS; ++q) {
            KP_HIP(hipEventRecord(c->side_ev[q - 1], c->side[q - 1]));
            KP_HIP(hipStreamWaitEvent(c->stream, c->side_ev[q - 1], 0));
        }
    KP_HIP(hipEventRecord(c->ev[1], c->stream));
    // breadth-first backtrack of every lane: depth d holds cells of level <= maxlev - d
    kp_bt_params B;
    memset(&B, 0, sizeof(B));
    B.g = g;
    B.T = P.T;
    B.K = p->d_K;
    B.S = p->d_S;
    B.groups = p->d_groups;
    B.lanegrp = p->d_lanegrp;
    B.nodes = p->d_nodes;
    B.cap = p->node_cap;
    B.cnt = p->d_cnt;
    B.dend = p->d_dend;
    B.bad = p->d_bad;
    B.root_train = p->d_rtrain;
    B.root_test = p->d_rtest;
    B.nleaves = p->d_nleaves;
    B.leaves = p->d_leaves;
    B.leafcap = hp.n_kmers;
    B.maxdepth = hp.maxlev;
    const bool bt = !P.dbg;
    if (bt) {
        const unsigned lb = (Ltot + 63) / 64;
        const uint64_t root = hp.npat - 1;
        hipLaunchKernelGGL(kp_bt_init, dim3(lb), dim3(64), 0, c->stream, B, root, kp_cell_digits(g, root));
        KP_HIP(hipGetLastError());
        for (int d = 0; d <= hp.maxlev; ++d) {
            B.depth = d;
            hipLaunchKernelGGL(kp_bt_level<CT>, dim3(64, Ltot), dim3(256), 0, c->stream, B);
            KP_HIP(hipGetLastError());
            hipLaunchKernelGGL(kp_bt_advance, dim3(lb), dim3(64), 0, c->stream, B);
            KP_HIP(hipGetLastError());
        }
        hipLaunchKernelGGL(kp_bt_finish, dim3(Ltot), dim3(256), 0, c->stream, B);
        KP_HIP(hipGetLastError());
    }
    KP_HIP(hipEventRecord(c->ev[2], c->stream));
    std::vector<uint32_t> bad(Ltot, 0);
    std::vector<float> rtr(Ltot), rte(Ltot);
    std::vector<uint64_t> nlv(Ltot);
    if (bt) {
        KP_HIP(hipMemcpyAsync(rtr.data(), p->d_rtrain, Ltot * sizeof(float), hipMemcpyDeviceToHost, c->stream));
        KP_HIP(hipMemcpyAsync(rte.data(), p->d_rtest, Ltot * sizeof(float), hipMemcpyDeviceToHost, c->stream));
        KP_HIP(hipMemcpyAsync(nlv.data(), p->d_nleaves, Ltot * sizeof(uint64_t), hipMemcpyDeviceToHost, c->stream));
        KP_HIP(hipMemcpyAsync(bad.data(), p->d_bad, Ltot * sizeof(uint32_t), hipMemcpyDeviceToHost, c->stream));
    }
    uint32_t werr = 0;
    KP_HIP(hipMemcpyAsync(&werr, p->d_werr, sizeof(uint32_t), hipMemcpyDeviceToHost, c->stream));
    KP_HIP(hipStreamSynchronize(c->stream));
    if (werr) return fail(KP_E_HIP, "kp_dp_ws_kernel: a hand-over wait timed out (results invalid)");
    float dp_ms = 0, bt_ms = 0;
    KP_HIP(hipEventElapsedTime(&dp_ms, c->ev[0], c->ev[1]));
#ifdef KP_STAMPS
    {
        unsigned long long hs[32];
        KP_HIP(hipMemcpy(hs, P.stamps, sizeof(hs), hipMemcpyDeviceToHost));
        fprintf(stderr, "KP_STAMPS init %.4g gather %.4g store %.4g wg_ticks %.4g wg_real100MHz %.4g levels",
                (double)hs[0], (double)hs[1], (double)hs[2], (double)hs[30], (double)hs[31]);
        for (int l = 0; l <= hp.lmax; ++l) fprintf(stderr, " %.4g", (double)hs[3 + l]);
        fprintf(stderr, "\n");
    }
#endif
    KP_HIP(hipEventElapsedTime(&bt_ms, c->ev[1], c->ev[2]));
    p->launch_ms.clear();
    if (timed)
        for (uint64_t q = 0; q < launches; ++q) {
            float ms = 0;
            KP_HIP(hipEventElapsedTime(&ms, p->lev[2 * q], p->lev[2 * q + 1]));
            p->launch_ms.push_back(ms);
        }
    if (P.dbg) {  // ablation build: timings only, never numbers
        p->stats.dp_ms = dp_ms;
        p->stats.backtrack_ms = 0;
        p->stats.units = hp.npat * (uint64_t)Ltot;
        p->stats.dp_launches = launches;
        return fail(KP_E_STATE, "KP_DEBUG_SKIP ablation pass: timings only, results are invalid");
    }
    for (uint32_t i = 0; i < Ltot; ++i) {
        if (bad[i])
            return fail(KP_E_PARITY, "backtrack of lane " + std::to_string(i) + " failed (flags " +
                                         std::to_string(bad[i]) +
                                         ": 1 no candidate, 2 node pool, 4 score not reproduced)");
        if (root_train) root_train[i] = rtr[i];
        if (root_test) root_test[i] = rte[i];
        if (n_leaves) n_leaves[i] = nlv[i];
    }
    p->last_ltot = Ltot;
    p->last_groups = dg;
    p->last_lanegrp = lanegrp;
    kp_pass_stats &s = p->stats;
    s.dp_ms = dp_ms;
    s.backtrack_ms = bt_ms;
    s.units = hp.npat * (uint64_t)Ltot;
    s.dp_launches = launches;
    const double sz = (double)sizeof(CT), npat = (double)hp.npat, nk = (double)hp.n_kmers;
    // 16 B per split pair, 8 B per cell write, 6s per aggregated cell, 2s per k-mer
    s.alg_bytes = (double)Ltot * (16.0 * hp.pairs_total + 8.0 * npat + 6.0 * sz * (npat - nk) + 2.0 * sz * nk);
    // compulsory HBM bytes of the blocked sweep: high-split gathers (2 x f32) + score writes
    const double padf = (double)g.Bpad / (double)g.B;
    s.gather_bytes = (double)Ltot * padf * (8.0 * hp.pairs_high + 4.0 * npat);
    s.total_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    return KP_OK;
}

template <typename CT>
static int run_codes(kp_plan *p, uint32_t lane, uint8_t *code) {
    kp_ctx *c = p->ctx;
    const kp::host_plan &hp = p->hp;
    kp_geom g = hp.g;
    g.nf = p->nf;
    g.Ltot = p->last_ltot;
    const kp_group_dev &G = p->last_groups[p->last_lanegrp[lane]];
    const double pen = G.pen[lane - (uint32_t)G.lane0];
    uint8_t *d_code = nullptr;
    KP_HIP(dmalloc(&d_code, hp.npat));
    for (int f = 0; f < p->nf; ++f)  // a fold table refilled since the pass may still be filling
        if (p->fold_async[f]) KP_HIP(hipStreamWaitEvent(c->stream, p->fold_ev[f], 0));
    const unsigned nb = (unsigned)std::min<uint64_t>((hp.npat + 255) / 256, 65535);
    hipLaunchKernelGGL(kp_codes_kernel<CT>, dim3(nb), dim3(256), 0, c->stream, g, tables_of(p),
                       reinterpret_cast<const CT *>(p->d_K), p->d_S, G, lane, pen, d_code);
    hipError_t e = hipGetLastError();
    if (e == hipSuccess) e = hipMemcpyAsync(code, d_code, hp.npat, hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    dfree(d_code);
    if (e != hipSuccess) return fail(KP_E_HIP, std::string("codes kernel: ") + hipGetErrorString(e));
    return KP_OK;
}

extern "C" {

int kp_device_groups(const kp_group *groups, int n_groups, int lanes_per_workgroup, int32_t *lane0, int32_t *nl,
                     int32_t *nl2, int cap, int *n_out) {
    if (!groups || n_groups <= 0 || !n_out || lanes_per_workgroup < 1 || lanes_per_workgroup > KP_GROUP_LANES)
        return fail(KP_E_ARG, "bad arguments");
    for (int i = 0; i < n_groups; ++i)
        if (groups[i].n_lanes < 1 || groups[i].n_lanes > KP_GROUP_MAX_LANES)
            return fail(KP_E_ARG, "group lanes must be 1..8");
    std::vector<kp_group_dev> dg;
    plan_device_groups(groups, n_groups, lanes_per_workgroup, dg);
    *n_out = (int)dg.size();
    for (int i = 0; i < (int)dg.size() && i < cap; ++i) {
        if (lane0) lane0[i] = dg[i].lane0;
        if (nl) nl[i] = dg[i].nl;
        if (nl2) nl2[i] = dg[i].nl2;
    }
    return KP_OK;
}

int kp_pass(kp_plan *p, const kp_group *groups, int n_groups, float *root_train, float *root_test,
            uint64_t *n_leaves) {
    if (!p || !groups || n_groups <= 0) return fail(KP_E_ARG, "bad arguments");
    if (!p->d_K) return fail(KP_E_STATE, "kp_set_counts must come first");
    KP_HIP(hipSetDevice(p->ctx->device));
    if (p->ct_bytes == 4) return run_pass<uint32_t>(p, groups, n_groups, root_train, root_test, n_leaves);
    return run_pass<uint64_t>(p, groups, n_groups, root_train, root_test, n_leaves);
}

int kp_reserve_lanes(kp_plan *p, uint32_t lanes) {
    if (!p) return fail(KP_E_ARG, "null plan");
    KP_HIP(hipSetDevice(p->ctx->device));
    const uint64_t had = p->lanes_cap;
    if (int rc = ensure_lanes(p, lanes)) return rc;
    if (p->lanes_cap != had && !p->S_pool) {  // fault the new pages in now rather than in the first pass
        KP_HIP(hipMemsetAsync(p->d_S, 0, p->hp.g.nblocks * (size_t)p->lanes_cap * p->hp.g.Bpad * 4, p->ctx->stream));
        KP_HIP(hipStreamSynchronize(p->ctx->stream));
    }
    return KP_OK;
}

int kp_last_launch_ms(const kp_plan *p, float *ms, int cap, int *n) {
    if (!p || !n || (cap > 0 && !ms)) return fail(KP_E_ARG, "null argument");
    *n = (int)p->launch_ms.size();
    for (int i = 0; i < cap && i < *n; ++i) ms[i] = p->launch_ms[i];
    return KP_OK;
}

int kp_last_pass_stats(const kp_plan *p, kp_pass_stats *out) {
    if (!p || !out) return fail(KP_E_ARG, "null argument");
    *out = p->stats;
    return KP_OK;
}

int kp_fit_leaves(kp_plan *p, uint32_t lane, uint64_t *leaves, uint64_t cap, uint64_t *n_out) {
    if (!p || !n_out) return fail(KP_E_ARG, "null argument");
    if (lane >= p->last_ltot) return fail(KP_E_STATE, "lane not in last pass");
    KP_HIP(hipSetDevice(p->ctx->device));
    uint64_t n = 0;
    KP_HIP(hipMemcpy(&n, p->d_nleaves + lane, sizeof(uint64_t), hipMemcpyDeviceToHost));
    *n_out = n;
    uint64_t m = std::min(n, std::min(cap, p->hp.n_kmers));
    if (leaves && m)
        KP_HIP(hipMemcpy(leaves, p->d_leaves + (uint64_t)lane * p->hp.n_kmers, m * sizeof(uint64_t),
                         hipMemcpyDeviceToHost));
    return KP_OK;
}

int kp_dump_lane(kp_plan *p, uint32_t lane, float *score, uint8_t *code) {
    if (!p) return fail(KP_E_ARG, "null argument");
    if (lane >= p->last_ltot) return fail(KP_E_STATE, "lane not in last pass");
    KP_HIP(hipSetDevice(p->ctx->device));
    const kp_geom &g = p->hp.g;
    const uint64_t ltot = p->last_ltot;
    if (score) {
        std::vector<float> rowf(g.Bpad);
        for (uint64_t h = 0; h < g.nblocks; ++h) {
            uint64_t off = (h * ltot + lane) * (uint64_t)g.Bpad;
            KP_HIP(hipMemcpy(rowf.data(), p->d_S + off, g.Bpad * sizeof(float), hipMemcpyDeviceToHost));
            memcpy(score + h * g.B, rowf.data(), g.B * sizeof(float));
        }
    }
    if (code) return p->ct_bytes == 4 ? run_codes<uint32_t>(p, lane, code) : run_codes<uint64_t>(p, lane, code);
    return KP_OK;
}

int kp_gather_cells(kp_plan *p, uint32_t lane, const uint64_t *cells, uint64_t n, float *out) {
    if (!p || (n && (!cells || !out))) return fail(KP_E_ARG, "null argument");
    if (lane >= p->last_ltot) return fail(KP_E_STATE, "lane not in last pass");
    for (uint64_t i = 0; i < n; ++i)
        if (cells[i] >= p->hp.npat) return fail(KP_E_ARG, "cell " + std::to_string(cells[i]) + " out of range");
    if (!n) return KP_OK;
    KP_HIP(hipSetDevice(p->ctx->device));
    kp_ctx *c = p->ctx;
    kp_geom g = p->hp.g;
    g.Ltot = p->last_ltot;
    const uint64_t chunk = std::min<uint64_t>(n, 1ull << 26);
    uint64_t *d_cells = nullptr;
    float *d_out = nullptr;
    KP_HIP(dmalloc(&d_cells, chunk * sizeof(uint64_t)));
    hipError_t e = dmalloc(&d_out, chunk * sizeof(float));
    for (uint64_t i0 = 0; i0 < n && e == hipSuccess; i0 += chunk) {
        const uint64_t m = std::min(chunk, n - i0);
        e = hipMemcpyAsync(d_cells, cells + i0, m * sizeof(uint64_t), hipMemcpyHostToDevice, c->stream);
        if (e != hipSuccess) break;
        const unsigned nb = (unsigned)std::min<uint64_t>((m + 255) / 256, 65536);
        hipLaunchKernelGGL(kp_gather_cells_kernel, dim3(nb), dim3(256), 0, c->stream, g, p->d_S, lane, d_cells, m,
                           d_out);
        e = hipGetLastError();
        if (e == hipSuccess) e = hipMemcpyAsync(out + i0, d_out, m * sizeof(float), hipMemcpyDeviceToHost, c->stream);
        if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    }
    dfree(d_cells);
    dfree(d_out);
    if (e != hipSuccess) return fail(KP_E_HIP, std::string("kp_gather_cells: ") + hipGetErrorString(e));
    return KP_OK;
}

}  // extern "C"

extern "C" {

int kp_math_log(kp_ctx *c, const double *x, double *y, uint64_t n) { return kp_math_libm(c, x, y, n, 0); }

int kp_math_libm(kp_ctx *c, const double *x, double *y, uint64_t n, int fn) {
    if (!c || (n && (!x || !y)) || fn < 0 || fn > 4) return fail(KP_E_ARG, "bad arguments");
    if (!n) return KP_OK;
    KP_HIP(hipSetDevice(c->device));
    double *dx = nullptr, *dy = nullptr;
    KP_HIP(dmalloc(&dx, n * sizeof(double)));
    hipError_t e = dmalloc(&dy, n * sizeof(double));
    if (e == hipSuccess) e = hipMemcpyAsync(dx, x, n * sizeof(double), hipMemcpyHostToDevice, c->stream);
    if (e == hipSuccess) {
        const unsigned nb = (unsigned)std::min<uint64_t>((n + 255) / 256, 16384);
        hipLaunchKernelGGL(kp_libm_kernel, dim3(nb), dim3(256), 0, c->stream, dx, dy, n, fn);
        e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipMemcpyAsync(y, dy, n * sizeof(double), hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    dfree(dx);
    dfree(dy);
    if (e != hipSuccess) return fail(KP_E_HIP, std::string("kp_math_libm: ") + hipGetErrorString(e));
    return KP_OK;
}

int kp_allkmers_cv(kp_ctx *c, const uint64_t *M, const uint64_t *U, uint64_t n, int nf, const double *alphas,
                   const double *betas, int na, double *sum_train, double *sum_test) {
    if (!c || nf < 1 || na < 0 || (n && (!M || !U)) || (na && (!alphas || !betas || !sum_train || !sum_test)))
        return fail(KP_E_ARG, "kp_allkmers_cv: bad arguments");
    if (!na) return KP_OK;
    if (!n) {  // no k-mers: every sum is the reference's numpy.zeros(nf)
        for (int a = 0; a < na; ++a)
            for (int f = 0; f < nf; ++f) sum_train[a * nf + f] = sum_test[a * nf + f] = 0.0;
        return KP_OK;
    }
    KP_HIP(hipSetDevice(c->device));
    const size_t cnt_bytes = n * (size_t)nf * sizeof(uint64_t);
    uint64_t *dM = nullptr, *dU = nullptr;
    double *dB = nullptr, *dT = nullptr, *dS = nullptr;
    hipError_t e = dmalloc(&dM, cnt_bytes);
    if (e == hipSuccess) e = dmalloc(&dU, cnt_bytes);
    if (e == hipSuccess) e = dmalloc(&dB, (size_t)na * nf * sizeof(double));
    if (e == hipSuccess) e = dmalloc(&dT, 2 * (size_t)nf * n * sizeof(double));  // one alpha's terms at a time
    if (e == hipSuccess) e = dmalloc(&dS, (size_t)na * 2 * nf * sizeof(double));
    if (e == hipSuccess) e = hipMemcpyAsync(dM, M, cnt_bytes, hipMemcpyHostToDevice, c->stream);
    if (e == hipSuccess) e = hipMemcpyAsync(dU, U, cnt_bytes, hipMemcpyHostToDevice, c->stream);
    if (e == hipSuccess)
        e = hipMemcpyAsync(dB, betas, (size_t)na * nf * sizeof(double), hipMemcpyHostToDevice, c->stream);
    const uint64_t items = n * (uint64_t)nf;
    const unsigned nb = (unsigned)std::min<uint64_t>((items + 255) / 256, 8192);
    for (int a = 0; a < na && e == hipSuccess; ++a) {
        hipLaunchKernelGGL(kp_allk_terms, dim3(nb), dim3(256), 0, c->stream, dM, dU, n, nf, alphas[a],
                           dB + (size_t)a * nf, dT);
        e = hipGetLastError();
        if (e == hipSuccess) {
            hipLaunchKernelGGL(kp_allk_sums, dim3((2 * nf + 63) / 64), dim3(64), 0, c->stream, dT, n, 2 * nf,
                               dS + (size_t)a * 2 * nf);
            e = hipGetLastError();
        }
    }
    std::vector<double> hs((size_t)na * 2 * nf);
    if (e == hipSuccess) e = hipMemcpyAsync(hs.data(), dS, hs.size() * sizeof(double), hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    dfree(dM);
    dfree(dU);
    dfree(dB);
    dfree(dT);
    dfree(dS);
    if (e != hipSuccess) return fail(KP_E_HIP, std::string("kp_allkmers_cv: ") + hipGetErrorString(e));
    for (int a = 0; a < na; ++a)
        for (int f = 0; f < nf; ++f) {
            sum_train[a * nf + f] = hs[((size_t)a * 2 + 0) * nf + f];
            sum_test[a * nf + f] = hs[((size_t)a * 2 + 1) * nf + f];
        }
    return KP_OK;
}

int kp_fold_sample(uint32_t *mt_key, int32_t *mt_pos, const uint64_t *colors, uint64_t n, uint64_t m,
                   uint64_t *out) {
    if (!mt_key || !mt_pos || (n && (!colors || !out))) return fail(KP_E_ARG, "bad arguments");
    if (*mt_pos < 0 || *mt_pos > 624) return fail(KP_E_ARG, "MT19937 position out of range");
    if (!n) return KP_OK;
    kpf::mt19937 rng;
    memcpy(rng.key, mt_key, sizeof(rng.key));
    rng.pos = *mt_pos;
    std::vector<uint64_t> tail(n);
    uint64_t acc = 0;
    for (uint64_t i = n; i-- > 0;) {
        acc += colors[i];
        tail[i] = acc;
    }
    kpf::sample(rng, m, colors, tail.data(), n, out);
    memcpy(mt_key, rng.key, sizeof(rng.key));
    *mt_pos = rng.pos;
    return KP_OK;
}

int kp_fold_split(uint32_t *mt_key, int32_t *mt_pos, const uint64_t *colors, uint64_t n, int nf, uint64_t *folds) {
    if (!mt_key || !mt_pos || (n && (!colors || !folds)) || nf < 1) return fail(KP_E_ARG, "bad arguments");
    if (*mt_pos < 0 || *mt_pos > 624) return fail(KP_E_ARG, "MT19937 position out of range");
    kpf::mt19937 rng;
    memcpy(rng.key, mt_key, sizeof(rng.key));
    rng.pos = *mt_pos;
    std::vector<uint64_t> col(colors, colors + n), tail(n), s(n);
    uint64_t total = 0;
    for (uint64_t i = 0; i < n; ++i) total += col[i];
    const uint64_t per_fold = total / (uint64_t)nf;  // n_samples = n // n_folds (CV_tools.py:51)
    for (int f = 0; f + 1 < nf; ++f) {
        uint64_t acc = 0;
        for (uint64_t i = n; i-- > 0;) {
            acc += col[i];
            tail[i] = acc;
        }
        kpf::sample(rng, per_fold, col.data(), tail.data(), n, s.data());
        for (uint64_t i = 0; i < n; ++i) {
            folds[i * (uint64_t)nf + f] = s[i];
            col[i] -= s[i];
        }
    }
    for (uint64_t i = 0; i < n; ++i) folds[i * (uint64_t)nf + (nf - 1)] = col[i];
    memcpy(mt_key, rng.key, sizeof(rng.key));
    *mt_pos = rng.pos;
    return KP_OK;
}

// ---- k-mer count files (host code) ----
struct kp_kmer_table {
    kpio::table t;
};

int kp_kmer_parse(const char *text, uint64_t nbytes, int columns, const char *super_pattern, int length,
                  kp_kmer_table **out) {
    if (!out || (nbytes && !text)) return fail(KP_E_ARG, "bad arguments");
    *out = nullptr;
    kp_kmer_table *t = new kp_kmer_table();
    const std::string err = kpio::parse(text, nbytes, columns, super_pattern, length, t->t);
    if (!err.empty()) {
        delete t;
        return fail(KP_E_ARG, err);
    }
    *out = t;
    return KP_OK;
}

int kp_kmer_table_info(const kp_kmer_table *t, uint64_t *n, int32_t *k, int64_t *total0, int64_t *total1) {
    if (!t || !n || !k || !total0 || !total1) return fail(KP_E_ARG, "null argument");
    *n = t->t.code.size();
    *k = t->t.k;
    *total0 = t->t.total0;
    *total1 = t->t.total1;
    return KP_OK;
}

int kp_kmer_table_copy(const kp_kmer_table *t, uint64_t *codes, int64_t *c0, int64_t *c1) {
    if (!t) return fail(KP_E_ARG, "null table");
    const size_t n = t->t.code.size();
    if (n && (!codes || !c0 || !c1)) return fail(KP_E_ARG, "null output");
    if (n) {
        memcpy(codes, t->t.code.data(), n * sizeof(uint64_t));
        memcpy(c0, t->t.c0.data(), n * sizeof(int64_t));
        memcpy(c1, t->t.c1.data(), n * sizeof(int64_t));
    }
    return KP_OK;
}

void kp_kmer_table_free(kp_kmer_table *t) { delete t; }

// ---- the long output table (host code) ----
int kp_format_long_rows(const char *kmers, int k, const int64_t *c_neg, const int64_t *c_pos, const uint32_t *pid,
                        uint64_t n, const char *tails, const uint64_t *tail_off, uint64_t n_tails, char *out,
                        uint64_t cap, uint64_t *out_len) {
    if (!out_len || k < 1 || (n && (!kmers || !c_neg || !c_pos || !pid || !tails || !tail_off || !out)))
        return fail(KP_E_ARG, "bad arguments");
    const int64_t w = kpout::long_rows(kmers, k, c_neg, c_pos, pid, n, tails, tail_off, n_tails, out, cap);
    if (w == -1) return fail(KP_E_ARG, "output buffer too small");
    if (w == -2) return fail(KP_E_ARG, "division by zero: a k-mer with no counts in the long output");
    if (w == -3) return fail(KP_E_ARG, "pattern index out of range");
    *out_len = (uint64_t)w;
    return KP_OK;
}

int kp_py_repr(const double *x, uint64_t n, char *out, uint64_t cap, uint64_t *out_len) {
    if (!out_len || (n && (!x || !out))) return fail(KP_E_ARG, "bad arguments");
    uint64_t w = 0;
    for (uint64_t i = 0; i < n; ++i) {
        if (w + 40 > cap) return fail(KP_E_ARG, "output buffer too small");
        w += (uint64_t)kpout::py_repr(x[i], out + w);
        out[w++] = '\n';
    }
    *out_len = w;
    return KP_OK;
}

}  // extern "C"
