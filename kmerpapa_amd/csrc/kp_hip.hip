// kp_hip.hip -- gfx950 kernels and C-ABI of the blocked lattice DP (libkmerpapa_hip.so).
//
// Kernels (one launch per high level for the first two, kp_core.h for the layout):
//   kp_counts_kernel    : per-block k-mer-low fold counts K[h] (replaces the first-pair
//                         M/U aggregation, CV :52-55, Fit :50-53)
//   kp_dp_kernel        : the DP of every cell of one block for one lane group
//                         (CV handle_pattern :26-78 / score_test_folds :15-20,
//                          Fit handle_pattern :31-64 / score :26-29)
//       phase 1  gather: every high-position split pair = two coalesced float4 reads of
//                        whole child-block rows (HBM/L2), first-min in scan order
//       phase 2  levels: low-position splits inside LDS, level by level, then the
//                        single-pattern term in float64
//       phase 3  store : train row (f32) + argmin codes (u8), coalesced
//   kp_backtrack_kernel : root read-out; test -2LL of the root by a DFS over the argmin
//                         tree (CV :158-163), leaves for the Fit (Fit :17-24)
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <string>
#include <vector>

#include "../../include/kmerpapa_hip.h"
#include "kp_core.h"
#include "kp_plan.h"

#define KP_DP_MAX_THREADS 1024

// LDS-qualified element types: pointers to them are 32-bit and address LDS directly
typedef __attribute__((address_space(3))) float kp_lds_f32;
typedef __attribute__((address_space(3))) uint64_t kp_lds_u64;

// ---------------------------------------------------------------------------
// kernels
// ---------------------------------------------------------------------------

struct kp_dev_tables {
    const kp_postab *tabs;
    const uint32_t *lowinfo;
    const uint16_t *lorder;
    const int32_t *loff;
    const uint32_t *klofs;
    const uint16_t *kllist;
    const uint32_t *hlist;
    const kp_lowdesc *ldesc;
    const uint16_t *kl2l;
    const uint64_t *pw;
};

template <typename CT>
__global__ void __launch_bounds__(256) kp_counts_kernel(kp_geom g, kp_dev_tables T, uint64_t hbase, int H,
                                                        const CT *__restrict__ Kin_M, const CT *__restrict__ Kin_U,
                                                        CT *__restrict__ K) {
    const uint64_t h = T.hlist[hbase + blockIdx.x];
    const uint32_t per = g.n_kl * (uint32_t)g.nf;
    CT *dst = K + h * (uint64_t)per * 2;
    if (H == 0) {
        // all high digits are nucleotides: the block's k-mer-low cells are k-mers
        uint64_t kbase = 0;
        for (int i = 0; i < g.kh; ++i) kbase += (uint64_t)kp_high_digit(g, h, i) * g.khw[i];
        for (uint32_t e = threadIdx.x; e < per; e += blockDim.x) {
            uint32_t kl = e / (uint32_t)g.nf, f = e % (uint32_t)g.nf;
            uint64_t src = (kbase + kl) * (uint64_t)g.nf + f;
            dst[2 * e] = Kin_M[src];
            dst[2 * e + 1] = Kin_U[src];
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
    const CT *a = K + h1 * (uint64_t)per * 2;
    const CT *b = K + h2 * (uint64_t)per * 2;
    for (uint32_t e = threadIdx.x; e < 2 * per; e += blockDim.x) dst[e] = a[e] + b[e];
}

struct kp_dp_params {
    kp_geom g;
    kp_dev_tables T;
    const void *K;
    float *S;
    uint8_t *C;
    const kp_group_dev *groups;
    uint64_t hbase;
    int H;
    int lmax;
    int remap;  // 1 = XCD-contiguous block order (KP_XCD_REMAP=1; measured 4% slower, off by default)
    int dbg;  // timing ablation only (KP_DEBUG_SKIP, wrong results): 1 = skip gather, 2 = skip level phase,
              // 4 = skip logs, 8 = skip low split scan, 16 = no level barrier, 32 = no count recurrence
};

// first-min update of one float4 of candidates (strict "<": the earlier pair keeps ties)
__device__ inline void kp_min4(float4 &best, uint32_t &c0, uint32_t &c1, uint32_t &c2, uint32_t &c3, const float4 a,
                               const float4 b, uint32_t code) {
    float v;
    v = a.x + b.x; if (v < best.x) { best.x = v; c0 = code; }
    v = a.y + b.y; if (v < best.y) { best.y = v; c1 = code; }
    v = a.z + b.z; if (v < best.z) { best.z = v; c2 = code; }
    v = a.w + b.w; if (v < best.w) { best.w = v; c3 = code; }
}

#define KP_IPT 2  // low cells per thread per level (host checks level sizes)

template <typename CT, int NL>
__global__ void __launch_bounds__(KP_DP_MAX_THREADS) kp_dp_kernel(kp_dp_params P) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const kp_geom &g = P.g;
    // XCD-aware order: workgroups are dealt round-robin over the 8 XCDs, so give each XCD a
    // contiguous run of the level's block list (neighbouring blocks share child rows in L2)
    uint32_t widx = blockIdx.x;
    if (P.remap) {
        const uint32_t nb = gridDim.x, q = nb >> 3, r = nb & 7u, x = blockIdx.x & 7u;
        widx = x * q + (x < r ? x : r) + (blockIdx.x >> 3);
    }
    const uint64_t h = P.T.hlist[P.hbase + widx];
    const kp_group_dev *G = P.groups + blockIdx.y;
    const uint32_t lane0 = (uint32_t)G->lane0;
    const int fold = G->fold;
    const double alpha = G->alpha, beta = G->beta;
    const uint32_t Bpad = g.Bpad;
    double pen[NL];
#pragma unroll
    for (int j = 0; j < NL; ++j) pen[j] = G->pen[j];

    // LDS: st[Bpad][NL] f32 (lanes interleaved) | cd[NL][Bpad] u8 argmin codes | cm[Bpad] CT | cu[Bpad] CT |
    //      hp[] | pw[t][16]   (Bpad is a multiple of 16, so every carve stays 16-byte aligned)
    float *st = reinterpret_cast<float *>(smem);
    uint8_t *cd = smem + (size_t)NL * Bpad * 4;
    CT *cm = reinterpret_cast<CT *>(cd + (size_t)NL * Bpad);
    CT *cu = cm + Bpad;
    kp_hpair *hp = reinterpret_cast<kp_hpair *>(cu + Bpad);
    uint64_t *pw = reinterpret_cast<uint64_t *>(hp + (g.kh * 7 + 1));

    const CT *K = reinterpret_cast<const CT *>(P.K);
    const int np = (P.dbg & 1) ? 0 : kp_high_pair_count(g, P.T.tabs, h);  // wave-uniform
    const uint64_t rowstride = (uint64_t)g.Ltot * Bpad;
    if (threadIdx.x == 0) {
        kp_high_pairs(g, P.T.tabs, h, hp);
        for (int p = 0; p < np; ++p) {  // child rows as element offsets of lane 0
            hp[p].h1 *= rowstride;
            hp[p].h2 *= rowstride;
        }
    }
    {
        const uint32_t *src = reinterpret_cast<const uint32_t *>(P.T.pw);
        uint32_t *dst = reinterpret_cast<uint32_t *>(pw);
        const uint32_t words = (uint32_t)g.t * 32u;
        for (uint32_t e = threadIdx.x; e < words; e += blockDim.x) dst[e] = src[e];
    }
    // train counts of the block's k-mer-low cells; the level loop aggregates the rest
    for (uint32_t kl = threadIdx.x; kl < g.n_kl; kl += blockDim.x) {
        const kp_cnt c = kp_kl_counts<CT>(g, K, h, kl, fold);
        const uint32_t l = P.T.kl2l[kl];
        cm[l] = (CT)c.mtr;
        cu[l] = (CT)c.utr;
    }
    __syncthreads();

    // ---- phase 1: high-position splits, gathered as whole child-block rows ----
    // winner value -> LDS (interleaved), winner code -> global C directly
    const uint32_t nch = Bpad / 4;
    for (uint32_t item = threadIdx.x; item < (uint32_t)NL * nch; item += blockDim.x) {
        const uint32_t ll = item / nch, c = item % nch;
        const uint64_t lrow = (uint64_t)(lane0 + ll) * Bpad + 4 * c;
        const float *base = P.S + lrow;
        float4 best = make_float4(__builtin_huge_valf(), __builtin_huge_valf(), __builtin_huge_valf(),
                                  __builtin_huge_valf());
        uint32_t c0 = KP_NONE, c1 = KP_NONE, c2 = KP_NONE, c3 = KP_NONE;
        int p = 0;
        for (; p + 4 <= np; p += 4) {
            const float4 a0 = *reinterpret_cast<const float4 *>(base + hp[p].h1);
            const float4 b0 = *reinterpret_cast<const float4 *>(base + hp[p].h2);
            const float4 a1 = *reinterpret_cast<const float4 *>(base + hp[p + 1].h1);
            const float4 b1 = *reinterpret_cast<const float4 *>(base + hp[p + 1].h2);
            const float4 a2 = *reinterpret_cast<const float4 *>(base + hp[p + 2].h1);
            const float4 b2 = *reinterpret_cast<const float4 *>(base + hp[p + 2].h2);
            const float4 a3 = *reinterpret_cast<const float4 *>(base + hp[p + 3].h1);
            const float4 b3 = *reinterpret_cast<const float4 *>(base + hp[p + 3].h2);
            kp_min4(best, c0, c1, c2, c3, a0, b0, hp[p].code);
            kp_min4(best, c0, c1, c2, c3, a1, b1, hp[p + 1].code);
            kp_min4(best, c0, c1, c2, c3, a2, b2, hp[p + 2].code);
            kp_min4(best, c0, c1, c2, c3, a3, b3, hp[p + 3].code);
        }
        for (; p < np; ++p) {
            const float4 a0 = *reinterpret_cast<const float4 *>(base + hp[p].h1);
            const float4 b0 = *reinterpret_cast<const float4 *>(base + hp[p].h2);
            kp_min4(best, c0, c1, c2, c3, a0, b0, hp[p].code);
        }
        float *sl = st + (size_t)(4 * c) * NL + ll;
        sl[0] = best.x;
        sl[NL] = best.y;
        sl[2 * NL] = best.z;
        sl[3 * NL] = best.w;
        *reinterpret_cast<uint32_t *>(cd + (size_t)ll * Bpad + 4 * c) = c0 | (c1 << 8) | (c2 << 16) | (c3 << 24);
    }
    __syncthreads();

    // ---- phase 2: low levels inside the block ----
    // one thread per cell: counts and the float64 logs once per cell for all NL lanes;
    // the next level's descriptors are loaded while the current level computes
    const bool high_zero = (P.H == 0);
    const int lmax = (P.dbg & 2) ? -1 : P.lmax;
    const uint4 *desc = reinterpret_cast<const uint4 *>(P.T.ldesc);
    uint4 cur[KP_IPT], nxt[KP_IPT];
    {
        const int beg = P.T.loff[0], cnt = P.T.loff[1] - beg;
#pragma unroll
        for (int k = 0; k < KP_IPT; ++k) {
            const int q = (int)threadIdx.x + k * (int)blockDim.x;
            if (q < cnt) cur[k] = desc[beg + q];
        }
    }
    for (int lam = 0; lam <= lmax; ++lam) {
        const int beg = P.T.loff[lam], cnt = P.T.loff[lam + 1] - beg;
        if (lam < lmax) {
            const int nbeg = P.T.loff[lam + 1], ncnt = P.T.loff[lam + 2] - nbeg;
#pragma unroll
            for (int k = 0; k < KP_IPT; ++k) {
                const int q = (int)threadIdx.x + k * (int)blockDim.x;
                if (q < ncnt) nxt[k] = desc[nbeg + q];
            }
        }
#pragma unroll
        for (int k = 0; k < KP_IPT; ++k) {
            const int q = (int)threadIdx.x + k * (int)blockDim.x;
            if (q < cnt) {
                const uint32_t l = cur[k].x & 0xFFFFu;
                const uint32_t l1 = cur[k].x >> 16, l2 = cur[k].y & 0xFFFFu;
                const uint32_t info = cur[k].z;
                CT mt, ut;
                if (lam == 0) {
                    mt = cm[l];
                    ut = cu[l];
                } else if (P.dbg & 32) {  // timing ablation: no count recurrence
                    mt = (CT)l1;
                    ut = (CT)l2;
                } else {
                    // count recurrence on the first split (the reference's M_mem/U_mem rows)
                    mt = cm[l1] + cm[l2];
                    ut = cu[l1] + cu[l2];
                    cm[l] = mt;
                    cu[l] = ut;
                }
                kp_single_ctx sc;
                sc.kmer = high_zero && lam == 0;
                sc.c.mtr = (uint64_t)mt;
                sc.c.utr = (uint64_t)ut;
                sc.c.mte = sc.c.ute = 0;
                sc.logp = sc.log1mp = 0.0;
                if (!sc.kmer && !(P.dbg & 4)) {
                    const double pr = kp_rate(sc.c, alpha, beta);
                    sc.logp = log(pr);
                    sc.log1mp = log(1.0 - pr);
                }
                uint32_t code[NL];
                if (!(P.dbg & 8)) {
                    kp_dp_cell_lanes<NL>(g, (const kp_lds_u64 *)pw, l, info, (kp_lds_f32 *)st, sc, alpha, beta, pen,
                                         code);
                } else {  // timing ablation: no split scan, keep the single term
#pragma unroll
                    for (int j = 0; j < NL; ++j) {
                        st[l * NL + j] = (float)kp_single_train(sc.c, sc.logp, sc.log1mp, pen[j]);
                        code[j] = KP_SINGLE;
                    }
                }
#pragma unroll
                for (int j = 0; j < NL; ++j)
                    if (code[j] != KP_NONE) cd[(size_t)j * Bpad + l] = (uint8_t)code[j];
            }
        }
        if (!(P.dbg & 16)) __syncthreads();  // (ablation 16: timing without the level barrier)
#pragma unroll
        for (int k = 0; k < KP_IPT; ++k) cur[k] = nxt[k];
    }

    // ---- phase 3: store the block's train rows ----
    for (uint32_t item = threadIdx.x; item < (uint32_t)NL * nch; item += blockDim.x) {
        const uint32_t ll = item / nch, c = item % nch;
        const float *sl = st + (size_t)(4 * c) * NL + ll;
        *reinterpret_cast<float4 *>(P.S + h * rowstride + (uint64_t)(lane0 + ll) * Bpad + 4 * c) =
            make_float4(sl[0], sl[NL], sl[2 * NL], sl[3 * NL]);
    }
    // ... and its argmin codes, 16 per store
    const uint32_t nc16 = Bpad / 16;
    for (uint32_t item = threadIdx.x; item < (uint32_t)NL * nc16; item += blockDim.x) {
        const uint32_t ll = item / nc16, c = item % nc16;
        *reinterpret_cast<uint4 *>(P.C + h * rowstride + (uint64_t)(lane0 + ll) * Bpad + 16 * c) =
            *reinterpret_cast<const uint4 *>(cd + (size_t)ll * Bpad + 16 * c);
    }
}

__device__ inline uint64_t kp_wave_sum(uint64_t v) {
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    return v;
}

// test -2LL of a leaf cell: the wave splits the leaf's k-mer-low rows, then reduces
template <typename CT>
__device__ inline float kp_leaf_test_wave(const kp_geom &g, const kp_dev_tables &T, const CT *K, uint64_t x, int fold,
                                          double alpha, double beta) {
    const uint64_t h = x / g.B;
    const uint32_t l = (uint32_t)(x % g.B);
    const uint32_t b = T.klofs[l], e = T.klofs[l + 1];
    uint64_t mtr = 0, utr = 0, mte = 0, ute = 0;
    for (uint32_t q = b + (threadIdx.x & 63u); q < e; q += 64) {
        const kp_cnt c = kp_kl_counts<CT>(g, K, h, T.kllist[q], fold);
        mtr += c.mtr; utr += c.utr; mte += c.mte; ute += c.ute;
    }
    kp_cnt c;
    c.mtr = kp_wave_sum(mtr);
    c.utr = kp_wave_sum(utr);
    c.mte = kp_wave_sum(mte);
    c.ute = kp_wave_sum(ute);
    if (fold < 0) return 0.0f;
    if (kp_is_kmer(g, h, T.lowinfo[l])) return kp_kmer_test(c, alpha, beta);
    const double p = kp_rate(c, alpha, beta);
    return kp_single_test(c, log(p), log(1.0 - p));
}

// one wave per lane: the DFS runs in lockstep in all 64 threads (uniform control flow)
template <typename CT>
__global__ void __launch_bounds__(64) kp_backtrack_kernel(kp_geom g, kp_dev_tables T, const CT *K, const float *S,
                                                          const uint8_t *C, const kp_group_dev *groups,
                                                          const uint32_t *lanegrp, float *root_train,
                                                          float *root_test, uint64_t *nleaves, uint32_t *bad,
                                                          uint64_t *leaves, uint64_t cap) {
    const uint32_t lane = blockIdx.x;
    const kp_group_dev *G = groups + lanegrp[lane];
    const int fold = G->fold;
    const double alpha = G->alpha, beta = G->beta;
    uint64_t n = 0;
    uint32_t err = 0;
    auto leaf = [&](uint64_t x) { return kp_leaf_test_wave<CT>(g, T, K, x, fold, alpha, beta); };
    const bool writer = threadIdx.x == 0;
    float t = kp_backtrack_lane(g, T.tabs, C, lane, leaf, writer && leaves ? leaves + (uint64_t)lane * cap : nullptr,
                                cap, &n, &err);
    if (writer) {
        root_train[lane] = S[kp_lane_row(g, g.nblocks - 1, lane) + (g.B - 1)];
        root_test[lane] = t;
        nleaves[lane] = n;
        bad[lane] = err;
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

struct kp_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    hipEvent_t ev[4] = {nullptr, nullptr, nullptr, nullptr};
    size_t lds_max = 65536;
};

struct kp_plan {
    kp_ctx *ctx = nullptr;
    kp::host_plan hp;
    // device tables
    kp_postab *d_tabs = nullptr;
    uint32_t *d_lowinfo = nullptr;
    uint16_t *d_lorder = nullptr;
    int32_t *d_loff = nullptr;
    uint32_t *d_klofs = nullptr;
    uint16_t *d_kllist = nullptr;
    uint32_t *d_hlist = nullptr;
    kp_lowdesc *d_ldesc = nullptr;
    uint16_t *d_kl2l = nullptr;
    uint64_t *d_pw = nullptr;
    // counts
    void *d_K = nullptr;
    int nf = 0;
    int ct_bytes = 0;
    // lanes
    float *d_S = nullptr;
    uint8_t *d_C = nullptr;
    uint64_t lanes_cap = 0;
    kp_group_dev *d_groups = nullptr;
    uint32_t *d_lanegrp = nullptr;
    float *d_rtrain = nullptr, *d_rtest = nullptr;
    uint64_t *d_nleaves = nullptr;
    uint32_t *d_bad = nullptr;
    uint64_t *d_leaves = nullptr;
    uint64_t small_cap = 0;  // lanes the small buffers above can hold
    uint32_t last_ltot = 0;
    kp_pass_stats stats{};
};

static kp_dev_tables tables_of(const kp_plan *p) {
    kp_dev_tables T;
    T.tabs = p->d_tabs;
    T.lowinfo = p->d_lowinfo;
    T.lorder = p->d_lorder;
    T.loff = p->d_loff;
    T.klofs = p->d_klofs;
    T.kllist = p->d_kllist;
    T.hlist = p->d_hlist;
    T.ldesc = p->d_ldesc;
    T.kl2l = p->d_kl2l;
    T.pw = p->d_pw;
    return T;
}

template <typename T>
static int upload(kp_plan *p, T **dptr, const std::vector<T> &v) {
    size_t bytes = std::max<size_t>(1, v.size()) * sizeof(T);
    KP_HIP(hipMalloc(reinterpret_cast<void **>(dptr), bytes));
    if (!v.empty()) KP_HIP(hipMemcpy(*dptr, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice));
    return KP_OK;
}

static void dfree(void *p) {
    if (p) (void)hipFree(p);
}

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
    int lds = 0;
    if (hipDeviceGetAttribute(&lds, hipDeviceAttributeMaxSharedMemoryPerBlock, device) == hipSuccess && lds > 0)
        c->lds_max = (size_t)lds;
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
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
}

int kp_plan_create(kp_ctx *ctx, const char *gen_pat, uint32_t max_block, kp_plan **out) {
    if (!ctx || !gen_pat || !out) return fail(KP_E_ARG, "null argument");
    KP_HIP(hipSetDevice(ctx->device));
    kp_plan *p = new kp_plan();
    p->ctx = ctx;
    std::string err = kp::build_plan(gen_pat, max_block ? max_block : 4096u, p->hp);
    if (!err.empty()) {
        delete p;
        return fail(KP_E_ARG, err);
    }
    int rc;
    if ((rc = upload(p, &p->d_tabs, p->hp.tabs)) || (rc = upload(p, &p->d_lowinfo, p->hp.lowinfo)) ||
        (rc = upload(p, &p->d_lorder, p->hp.lorder)) || (rc = upload(p, &p->d_loff, p->hp.loff)) ||
        (rc = upload(p, &p->d_klofs, p->hp.klofs)) || (rc = upload(p, &p->d_kllist, p->hp.kllist)) ||
        (rc = upload(p, &p->d_hlist, p->hp.hlist)) || (rc = upload(p, &p->d_ldesc, p->hp.ldesc)) ||
        (rc = upload(p, &p->d_kl2l, p->hp.kl2l)) || (rc = upload(p, &p->d_pw, p->hp.pw))) {
        kp_plan_destroy(p);
        return rc;
    }
    *out = p;
    return KP_OK;
}

void kp_plan_destroy(kp_plan *p) {
    if (!p) return;
    if (p->ctx) (void)hipSetDevice(p->ctx->device);
    void *bufs[] = {p->d_tabs, p->d_lowinfo, p->d_lorder, p->d_loff, p->d_klofs, p->d_kllist, p->d_hlist,
                    p->d_ldesc, p->d_kl2l, p->d_pw,
                    p->d_K, p->d_S, p->d_C, p->d_groups, p->d_lanegrp, p->d_rtrain, p->d_rtest,
                    p->d_nleaves, p->d_bad, p->d_leaves};
    for (void *b : bufs) dfree(b);
    delete p;
}

int kp_plan_get_info(const kp_plan *p, kp_plan_info *o) {
    if (!p || !o) return fail(KP_E_ARG, "null argument");
    const kp::host_plan &h = p->hp;
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
    o->bytes_per_lane = h.g.nblocks * (uint64_t)h.g.Bpad * 5;
    return KP_OK;
}

}  // extern "C"

template <typename CT>
static int run_counts(kp_plan *p, const void *M, const void *U, uint64_t n_kmers, int nf) {
    kp_ctx *c = p->ctx;
    kp_geom g = p->hp.g;
    g.nf = nf;
    size_t in_bytes = n_kmers * (size_t)nf * sizeof(CT);
    CT *dM = nullptr, *dU = nullptr;
    KP_HIP(hipMalloc(&dM, in_bytes));
    KP_HIP(hipMalloc(&dU, in_bytes));
    KP_HIP(hipMemcpyAsync(dM, M, in_bytes, hipMemcpyHostToDevice, c->stream));
    KP_HIP(hipMemcpyAsync(dU, U, in_bytes, hipMemcpyHostToDevice, c->stream));
    size_t kbytes = g.nblocks * (size_t)g.n_kl * nf * 2 * sizeof(CT);
    if (p->d_K && (p->nf != nf || p->ct_bytes != (int)sizeof(CT))) {
        dfree(p->d_K);
        p->d_K = nullptr;
    }
    if (!p->d_K) {
        size_t fr = 0, tot = 0;
        KP_HIP(hipMemGetInfo(&fr, &tot));
        if (kbytes + (64u << 20) > fr) {
            dfree(dM);
            dfree(dU);
            return fail(KP_E_NOMEM, "count tables need " + std::to_string(kbytes) + " bytes");
        }
        KP_HIP(hipMalloc(&p->d_K, kbytes));
    }
    kp_dev_tables T = tables_of(p);
    for (int H = 0; H <= p->hp.hmax; ++H) {
        uint64_t nb = p->hp.hoff[H + 1] - p->hp.hoff[H];
        if (!nb) continue;
        hipLaunchKernelGGL(kp_counts_kernel<CT>, dim3((unsigned)nb), dim3(256), 0, c->stream, g, T, p->hp.hoff[H], H,
                           dM, dU, reinterpret_cast<CT *>(p->d_K));
        KP_HIP(hipGetLastError());
    }
    KP_HIP(hipStreamSynchronize(c->stream));
    dfree(dM);
    dfree(dU);
    p->nf = nf;
    p->ct_bytes = (int)sizeof(CT);
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

}  // extern "C"

static size_t dp_lds_bytes(const kp::host_plan &hp, int nl, size_t ct_bytes) {
    const kp_geom &g = hp.g;
    return (size_t)nl * g.Bpad * 5 + 2 * (size_t)g.Bpad * ct_bytes + (size_t)(g.kh * 7 + 1) * sizeof(kp_hpair) +
           (size_t)g.t * 16 * sizeof(uint64_t) + 16;
}

template <typename CT, int NL>
static int launch_dp(kp_ctx *c, const kp_dp_params &P, unsigned nb, unsigned ngroups, int threads, size_t lds) {
    if (lds > 65536)
        KP_HIP(hipFuncSetAttribute(reinterpret_cast<const void *>(&kp_dp_kernel<CT, NL>),
                                   hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    hipLaunchKernelGGL((kp_dp_kernel<CT, NL>), dim3(nb, ngroups), dim3(threads), lds, c->stream, P);
    KP_HIP(hipGetLastError());
    return KP_OK;
}

template <typename CT>
static int launch_dp_nl(int nl, kp_ctx *c, const kp_dp_params &P, unsigned nb, unsigned ngroups, int threads,
                        size_t lds) {
    switch (nl) {
        case 1: return launch_dp<CT, 1>(c, P, nb, ngroups, threads, lds);
        case 2: return launch_dp<CT, 2>(c, P, nb, ngroups, threads, lds);
        case 3: return launch_dp<CT, 3>(c, P, nb, ngroups, threads, lds);
        case 4: return launch_dp<CT, 4>(c, P, nb, ngroups, threads, lds);
        case 5: return launch_dp<CT, 5>(c, P, nb, ngroups, threads, lds);
        case 6: return launch_dp<CT, 6>(c, P, nb, ngroups, threads, lds);
        case 7: return launch_dp<CT, 7>(c, P, nb, ngroups, threads, lds);
        case 8: return launch_dp<CT, 8>(c, P, nb, ngroups, threads, lds);
    }
    return fail(KP_E_ARG, "lanes per workgroup must be 1..8");
}

static int dp_threads() {
    const char *e = getenv("KP_DP_THREADS");
    int v = e ? atoi(e) : 512;
    return (v == 64 || v == 128 || v == 256 || v == 512 || v == 1024) ? v : 256;
}

static int lanes_per_wg_default() {
    const char *e = getenv("KP_LANES_PER_WG");
    int v = e ? atoi(e) : 3;
    return std::min(std::max(v, 1), KP_GROUP_LANES);
}

template <typename CT>
static int run_pass(kp_plan *p, const kp_group *groups, int n_groups, float *root_train, float *root_test,
                    uint64_t *n_leaves) {
    auto t0 = std::chrono::steady_clock::now();
    kp_ctx *c = p->ctx;
    const kp::host_plan &hp = p->hp;
    kp_geom g = hp.g;
    g.nf = p->nf;
    // split user groups into device groups that fit the LDS budget
    int per_wg = lanes_per_wg_default();
    while (per_wg > 1 && dp_lds_bytes(hp, per_wg, sizeof(CT)) > c->lds_max) --per_wg;
    if (dp_lds_bytes(hp, 1, sizeof(CT)) > c->lds_max) return fail(KP_E_ARG, "block does not fit LDS");
    std::vector<kp_group_dev> dg;
    std::vector<uint32_t> lanegrp;
    uint32_t lane = 0;
    for (int i = 0; i < n_groups; ++i) {
        const kp_group &u = groups[i];
        if (u.n_lanes < 1 || u.n_lanes > KP_GROUP_MAX_LANES) return fail(KP_E_ARG, "group lanes must be 1..8");
        if (u.fold >= p->nf || u.fold < -1) return fail(KP_E_ARG, "fold out of range");
        for (int s = 0; s < u.n_lanes; s += per_wg) {
            kp_group_dev d;
            memset(&d, 0, sizeof(d));
            d.fold = u.fold;
            d.lane0 = (int32_t)lane;
            d.nl = std::min(per_wg, u.n_lanes - s);
            d.alpha = u.alpha;
            d.beta = u.beta;
            for (int j = 0; j < d.nl; ++j) d.pen[j] = u.penalty[s + j];
            for (int j = 0; j < d.nl; ++j) lanegrp.push_back((uint32_t)dg.size());
            lane += (uint32_t)d.nl;
            dg.push_back(d);
        }
    }
    const uint32_t Ltot = lane;
    g.Ltot = Ltot;
    // launch classes: device groups with equal lane counts share one launch per level
    std::stable_sort(dg.begin(), dg.end(), [](const kp_group_dev &a, const kp_group_dev &b) { return a.nl > b.nl; });
    lanegrp.assign(Ltot, 0);
    for (size_t i = 0; i < dg.size(); ++i)
        for (int j = 0; j < dg[i].nl; ++j) lanegrp[dg[i].lane0 + j] = (uint32_t)i;
    // threads per workgroup: every level of the block must fit KP_IPT cells per thread
    int max_level_cells = 0;
    for (int l = 0; l <= hp.lmax; ++l) max_level_cells = std::max(max_level_cells, hp.loff[l + 1] - hp.loff[l]);
    int threads = dp_threads();
    while (threads < KP_DP_MAX_THREADS && threads * KP_IPT < max_level_cells) threads *= 2;
    if (threads * KP_IPT < max_level_cells) return fail(KP_E_ARG, "block level too wide for one workgroup");
    // lane storage
    if (Ltot > p->lanes_cap) {
        dfree(p->d_S);
        dfree(p->d_C);
        p->d_S = nullptr;
        p->d_C = nullptr;
        p->lanes_cap = 0;
        size_t sb = g.nblocks * (size_t)Ltot * g.Bpad * 4, cb = g.nblocks * (size_t)Ltot * g.Bpad;
        size_t fr = 0, tot = 0;
        KP_HIP(hipMemGetInfo(&fr, &tot));
        if (sb + cb + (256u << 20) > fr)
            return fail(KP_E_NOMEM, "lanes need " + std::to_string(sb + cb) + " bytes, free " + std::to_string(fr));
        KP_HIP(hipMalloc(&p->d_S, sb));
        KP_HIP(hipMalloc(&p->d_C, cb));
        KP_HIP(hipMemsetAsync(p->d_S, 0, sb, c->stream));
        p->lanes_cap = Ltot;
    }
    if (Ltot > p->small_cap || dg.size() > p->small_cap) {
        void *bufs[] = {p->d_groups, p->d_lanegrp, p->d_rtrain, p->d_rtest, p->d_nleaves, p->d_bad, p->d_leaves};
        for (void *b : bufs) dfree(b);
        uint64_t cap = std::max<uint64_t>(Ltot, 64);
        KP_HIP(hipMalloc(&p->d_groups, cap * sizeof(kp_group_dev)));
        KP_HIP(hipMalloc(&p->d_lanegrp, cap * sizeof(uint32_t)));
        KP_HIP(hipMalloc(&p->d_rtrain, cap * sizeof(float)));
        KP_HIP(hipMalloc(&p->d_rtest, cap * sizeof(float)));
        KP_HIP(hipMalloc(&p->d_nleaves, cap * sizeof(uint64_t)));
        KP_HIP(hipMalloc(&p->d_bad, cap * sizeof(uint32_t)));
        KP_HIP(hipMalloc(&p->d_leaves, cap * hp.n_kmers * sizeof(uint64_t)));
        p->small_cap = cap;
    }
    KP_HIP(hipMemcpyAsync(p->d_groups, dg.data(), dg.size() * sizeof(kp_group_dev), hipMemcpyHostToDevice, c->stream));
    KP_HIP(hipMemcpyAsync(p->d_lanegrp, lanegrp.data(), lanegrp.size() * sizeof(uint32_t), hipMemcpyHostToDevice,
                          c->stream));

    kp_dp_params P;
    P.g = g;
    P.T = tables_of(p);
    P.K = p->d_K;
    P.S = p->d_S;
    P.C = p->d_C;
    P.groups = p->d_groups;
    P.lmax = hp.lmax;
    P.dbg = getenv("KP_DEBUG_SKIP") ? atoi(getenv("KP_DEBUG_SKIP")) : 0;
    P.remap = getenv("KP_XCD_REMAP") ? atoi(getenv("KP_XCD_REMAP")) : 0;
    KP_HIP(hipEventRecord(c->ev[0], c->stream));
    uint64_t launches = 0;
    for (int H = 0; H <= hp.hmax; ++H) {
        uint64_t nb = hp.hoff[H + 1] - hp.hoff[H];
        if (!nb) continue;
        P.hbase = hp.hoff[H];
        P.H = H;
        for (size_t i = 0; i < dg.size();) {
            size_t j = i;
            while (j < dg.size() && dg[j].nl == dg[i].nl) ++j;
            kp_dp_params Q = P;
            Q.groups = p->d_groups + i;
            int rc = launch_dp_nl<CT>(dg[i].nl, c, Q, (unsigned)nb, (unsigned)(j - i), threads,
                                      dp_lds_bytes(hp, dg[i].nl, sizeof(CT)));
            if (rc) return rc;
            ++launches;
            i = j;
        }
    }
    KP_HIP(hipEventRecord(c->ev[1], c->stream));
    if (!P.dbg) hipLaunchKernelGGL(kp_backtrack_kernel<CT>, dim3(Ltot), dim3(64), 0, c->stream, g, P.T,
                       reinterpret_cast<const CT *>(p->d_K), p->d_S, p->d_C, p->d_groups, p->d_lanegrp, p->d_rtrain,
                       p->d_rtest, p->d_nleaves, p->d_bad, p->d_leaves, (uint64_t)hp.n_kmers);
    KP_HIP(hipGetLastError());
    KP_HIP(hipEventRecord(c->ev[2], c->stream));
    std::vector<uint32_t> bad(Ltot);
    std::vector<float> rtr(Ltot), rte(Ltot);
    std::vector<uint64_t> nlv(Ltot);
    KP_HIP(hipMemcpyAsync(rtr.data(), p->d_rtrain, Ltot * sizeof(float), hipMemcpyDeviceToHost, c->stream));
    KP_HIP(hipMemcpyAsync(rte.data(), p->d_rtest, Ltot * sizeof(float), hipMemcpyDeviceToHost, c->stream));
    KP_HIP(hipMemcpyAsync(nlv.data(), p->d_nleaves, Ltot * sizeof(uint64_t), hipMemcpyDeviceToHost, c->stream));
    KP_HIP(hipMemcpyAsync(bad.data(), p->d_bad, Ltot * sizeof(uint32_t), hipMemcpyDeviceToHost, c->stream));
    KP_HIP(hipStreamSynchronize(c->stream));
    float dp_ms = 0, bt_ms = 0;
    KP_HIP(hipEventElapsedTime(&dp_ms, c->ev[0], c->ev[1]));
    KP_HIP(hipEventElapsedTime(&bt_ms, c->ev[1], c->ev[2]));
    for (uint32_t i = 0; i < Ltot; ++i) {
        if (bad[i] && !P.dbg) return fail(KP_E_PARITY, "argmin tree of lane " + std::to_string(i) + " is broken");
        if (root_train) root_train[i] = rtr[i];
        if (root_test) root_test[i] = rte[i];
        if (n_leaves) n_leaves[i] = nlv[i];
    }
    p->last_ltot = Ltot;
    kp_pass_stats &s = p->stats;
    s.dp_ms = dp_ms;
    s.backtrack_ms = bt_ms;
    s.units = hp.npat * (uint64_t)Ltot;
    s.dp_launches = launches;
    const double sz = (double)sizeof(CT), npat = (double)hp.npat, nk = (double)hp.n_kmers;
    // 16 B per split pair, 8 B per cell write, 6s per aggregated cell, 2s per k-mer
    s.alg_bytes = (double)Ltot * (16.0 * hp.pairs_total + 8.0 * npat + 6.0 * sz * (npat - nk) + 2.0 * sz * nk);
    const double padf = (double)g.Bpad / (double)g.B;
    s.gather_bytes = (double)Ltot * padf * (8.0 * hp.pairs_high + 5.0 * npat);
    s.total_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    return KP_OK;
}

extern "C" {

int kp_pass(kp_plan *p, const kp_group *groups, int n_groups, float *root_train, float *root_test,
            uint64_t *n_leaves) {
    if (!p || !groups || n_groups <= 0) return fail(KP_E_ARG, "bad arguments");
    if (!p->d_K) return fail(KP_E_STATE, "kp_set_counts must come first");
    KP_HIP(hipSetDevice(p->ctx->device));
    if (p->ct_bytes == 4) return run_pass<uint32_t>(p, groups, n_groups, root_train, root_test, n_leaves);
    return run_pass<uint64_t>(p, groups, n_groups, root_train, root_test, n_leaves);
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
    std::vector<float> rowf(g.Bpad);
    std::vector<uint8_t> rowc(g.Bpad);
    for (uint64_t h = 0; h < g.nblocks; ++h) {
        uint64_t off = (h * ltot + lane) * (uint64_t)g.Bpad;
        if (score) {
            KP_HIP(hipMemcpy(rowf.data(), p->d_S + off, g.Bpad * sizeof(float), hipMemcpyDeviceToHost));
            memcpy(score + h * g.B, rowf.data(), g.B * sizeof(float));
        }
        if (code) {
            KP_HIP(hipMemcpy(rowc.data(), p->d_C + off, g.Bpad, hipMemcpyDeviceToHost));
            memcpy(code + h * g.B, rowc.data(), g.B);
        }
    }
    return KP_OK;
}

}  // extern "C"
