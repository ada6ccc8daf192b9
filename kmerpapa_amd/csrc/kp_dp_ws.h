// kp_dp_ws.h -- the sweep for narrow device groups (1 lane) as a persistent,
// wave-specialised kernel; included by kp_hip.hip after kp_dp_kernel.h.
//
// Why: a 1-lane workgroup of kp_dp_kernel runs its phases one after the other -- block
// setup and count tables (dependent global round trips), the gather (HBM-bound), the level
// phase (VALU-bound: the rate, two float64 logs and the split scan for one lane) and the
// store -- and the three workgroups a CU holds overlap them only by chance.  Phase
// ablation of the 1-lane pass (profiles/r06/experiments/ablate_*.txt): NNNNNNNNN 592 ms
// in all, 435 without the gather, 387 without the level phase, 95 with neither; the
// 9-mer 108 / 81 / 65 / 19.  Overlapped perfectly the pass would take about the larger of
// its level and gather parts.
//
// How: each workgroup is persistent over the blocks of one launch (one high level) and
// splits its waves into two roles that work on two consecutive blocks at once:
//   producer waves (the first PW): block j's store-back of block j - 2 (its row buffer),
//     setup (block id, high split pairs, the k-mer-low count rows), separable count tables
//     and gather -- every high split pair's child rows min-reduced into the row buffer,
//     loads as deep as the registers allow;
//   consumer waves (the other CW): block i's level phase, level by level.
// Row buffers and count tables alternate between blocks.  The roles never meet at a
// workgroup barrier: they hand buffers over through LDS counters (FULL: producer waves
// that finished a block; FREE: consumer waves that finished one), and each role
// synchronises its own waves with an LDS counter barrier (the consumer after every level,
// the producer between count-table steps).  Every wait is bounded: past ~0.2 s it sets the
// plan's error word and the workgroup runs to its end without waiting (the pass then fails
// with KP_E_HIP), so a logic error cannot hang the GPU.  Results are the same float32 values
// in the same cells: the per-cell arithmetic is kp_core.h's, the gather's min is
// order-independent.
#pragma once
#include "kp_dp_kernel.h"

#ifndef KP_WS_PW
#define KP_WS_PW 4  // producer waves per workgroup
#endif
#ifndef KP_WS_CW
#define KP_WS_CW 8  // consumer waves per workgroup (the level phase's threads)
#endif
#define KP_WS_THREADS ((KP_WS_PW + KP_WS_CW) * 64)
#ifndef KP_WS_NI
#define KP_WS_NI 2  // producer: gather items per thread at a time
#endif
#ifndef KP_WS_PU
#define KP_WS_PU 2  // producer: split pairs per load step
#endif
#ifndef KP_WS_WAVES
#define KP_WS_WAVES 6  // waves per SIMD: two 12-wave workgroups per CU, <= 80 VGPRs
#endif

// XCD-aware list entry of virtual block v of a launch of nb blocks (kp_dp_kernel's remap
// with gridDim.x = nb): runs of G consecutive list entries per XCD
__device__ inline uint32_t kp_ws_remap(uint32_t v, uint32_t nb, int remap) {
    if (remap > 1) {
        const uint32_t G = (uint32_t)remap, full = nb / (8 * G) * (8 * G);
        if (v < full) {
            const uint32_t x = v & 7u, sl = v >> 3;
            return ((sl / G) * 8 + x) * G + sl % G;
        }
    }
    return v;
}

// one slot's share of the gather: pairs [p0, p1) of the block's high split pairs for every
// item (4 cells of one lane) of the row buffer st; the first share starts from +inf, later
// ones from st; NI items per thread at a time, PU pairs per step
template <int NL, int NI, int PU>
__device__ inline void kp_ws_gather(const kp_dp_params &P, const kp_hpair *hp, int p0, int p1, int nnt, bool first,
                                    bool last, uint32_t lane0, float *st, uint32_t tid, uint32_t nth) {
    const kp_geom &g = P.g;
    const uint32_t Bpad = g.Bpad, nch = Bpad / 4, nitems = (uint32_t)NL * nch;
    const float inf = __builtin_huge_valf();
    for (uint32_t it0 = tid; it0 < nitems; it0 += NI * nth) {
        uint32_t it[NI], o[NI];
        float4 best[NI];
#pragma unroll
        for (int i = 0; i < NI; ++i) {
            it[i] = (it0 + i * nth < nitems) ? it0 + i * nth : it0;
            o[i] = (lane0 + it[i] / nch) * Bpad + 4 * (it[i] % nch);
            if (first) {
                best[i] = make_float4(inf, inf, inf, inf);
            } else {
                const float *sl = st + (size_t)(4 * (it[i] % nch)) * NL + it[i] / nch;
                best[i] = make_float4(sl[0], sl[NL], sl[2 * NL], sl[3 * NL]);
            }
        }
        const int a = p0 < nnt ? p0 : nnt, b = p1 < nnt ? p1 : nnt;  // non-temporal pairs first
        if (a < b) kp_gather_range<NI, PU, true>(P, hp, a, b, o, best);
        const int c = p0 > nnt ? p0 : nnt;
        if (c < p1) kp_gather_range<NI, PU, false>(P, hp, c, p1, o, best);
#pragma unroll
        for (int i = 0; i < NI; ++i) {
            if (i > 0 && it[i] == it0) break;
            const uint32_t ll = it[i] / nch, cc = it[i] % nch;
            if (last && 4 * cc + 4 > g.B) {  // slot B (padding) and past it: +inf
                if (4 * cc + 0 >= g.B) best[i].x = inf;
                if (4 * cc + 1 >= g.B) best[i].y = inf;
                if (4 * cc + 2 >= g.B) best[i].z = inf;
                if (4 * cc + 3 >= g.B) best[i].w = inf;
            }
            float *sl = st + (size_t)(4 * cc) * NL + ll;
            sl[0] = best[i].x;
            sl[NL] = best[i].y;
            sl[2 * NL] = best[i].z;
            sl[3 * NL] = best[i].w;
        }
    }
}

// step s of the separable count tables (kp_core.h kp_build_count_table, one step per slot):
// s = 0 writes T_0 (the block's k-mer-low rows, train = all data - fold) into bufA; step
// s >= 1 expands low position s - 1; the last step writes ptab
template <typename CT>
__device__ inline void kp_ws_count_step(const kp_geom &g, int s, const CT *K, uint64_t krow, int fold,
                                        const uint8_t *lm, CT *bufA, CT *bufB, CT *ptab, uint32_t tid, uint32_t nth,
                                        const kp_cnt &pre) {
    if (s == 0) {
        CT *out0 = (g.t == 1) ? ptab : bufA;
        for (uint32_t kl = tid; kl < g.n_kl; kl += nth) {
            const kp_cnt c = (kl == tid) ? pre : kp_kl_counts<CT>(g, K, krow, kl, fold);
            out0[2 * kl] = (CT)c.mtr;
            out0[2 * kl + 1] = (CT)c.utr;
        }
        return;
    }
    const int e = s - 1;  // expand low position e: T_e (buffer of parity e) -> T_{e+1}
    CT *in = (e & 1) ? bufB : bufA;
    CT *out = (e + 2 == g.t) ? ptab : ((e & 1) ? bufA : bufB);
    uint32_t Rs = 1, rest = 1;
    for (int i = 0; i < e; ++i) Rs *= g.r[i];
    for (int i = e + 1; i < g.t; ++i) rest *= g.n[i];
    const uint32_t rs = g.r[e], ns = g.n[e];
    const uint32_t entries = Rs * rs * rest;
    for (uint32_t q = tid; q < entries; q += nth) {
        const uint32_t D = q % Rs, qq = q / Rs, ds = qq % rs, Nr = qq / rs;
        const uint32_t m = lm[e * 16 + ds];
        CT sm = 0, su = 0;
        for (uint32_t a = 0; a < ns; ++a)
            if (m & (1u << a)) {
                const uint32_t src = D + Rs * (a + ns * Nr);
                sm += in[2 * src];
                su += in[2 * src + 1];
            }
        out[2 * q] = sm;
        out[2 * q + 1] = su;
    }
}

// byte offset BASE of a row buffer at LDS address 0 + BASE (the kernel declares no static LDS)
#define KP_WS_BASE1 16512u  // row buffer 1: 4128 floats in (blocks <= 4096 cells, Bpad <= 4128)

// min over one 4-pair chunk of a cell's split-pair list, one lane, row buffer at LDS BASE
// (kp_core.h kp_chunk_minv's SDWA form: the child's byte offset is one v_mul_u32_u24 of the
// pair word's 16-bit half)
template <uint32_t BASE>
__device__ inline void kp_ws_chunk_min(const uint4 c, float *lmin) {
    const uint32_t e[4] = {c.x, c.y, c.z, c.w};
    float va[4], vb[4];
#pragma unroll
    for (int p = 0; p < 4; ++p) {
        const uint32_t o1 = kp_half_mul<4u, 0>(e[p]), o2 = kp_half_mul<4u, 1>(e[p]);
        va[p] = ((kp_lds_f32 *)(uintptr_t)o1)[BASE / 4u];
        vb[p] = ((kp_lds_f32 *)(uintptr_t)o2)[BASE / 4u];
    }
#pragma unroll
    for (int p = 0; p < 4; ++p) *lmin = fminf(*lmin, va[p] + vb[p]);
}

// one cell of the level phase, one lane (kp_core.h kp_dp_cell_list with NL = W = 1)
template <int PRE, uint32_t BASE>
__device__ inline void kp_ws_cell_list(uint32_t l, uint32_t npairs, const uint4 *pre, const uint4 *lp,
                                       const kp_single_ctx &sc, double alpha, double beta, const double *pen) {
    kp_lds_f32 *row = (kp_lds_f32 *)(uintptr_t)BASE + l;
    float lmin = row[0];
#pragma unroll
    for (int k = 0; k < PRE; ++k)
        if (4u * k < npairs) kp_ws_chunk_min<BASE>(pre[k], &lmin);
    for (uint32_t k = PRE; 4u * k < npairs; ++k) kp_ws_chunk_min<BASE>(lp[k], &lmin);
    kp_cell_store<1>(row, &lmin, sc, pen, alpha, beta, 0);
}

// the consumer's level lam of the block in row buffer BUF (its LDS byte offset is a
// compile-time constant, so the SDWA scan's child offsets fold into the LDS instructions)
template <typename CT, int NL, uint32_t BASE>
__device__ inline void kp_ws_level(const kp_dp_params &P, int lam, const uint4 *cur, const uint8_t *lm,
                                   const CT *ptab, const kp_group_dev *G, const double *pen, double alpha, double beta,
                                   bool exact, uint32_t ctid, int ncons) {
    static_assert(NL == 1, "the wave-specialised sweep holds one lane");
    const kp_geom &g = P.g;
    kp_lds_f32 *st = (kp_lds_f32 *)(uintptr_t)BASE;
    const int beg = P.loffv[lam], cnt = P.loffv[lam + 1] - beg;
    (void)beg;
    (void)G;
    constexpr bool MIX = false;
    if (cnt * KP_PS <= ncons) {
        // the block's narrowest levels: each cell on KP_PS consecutive lanes of one wave
        // (kp_dp_kernel's kPS path): pair chunks r, r + KP_PS, ...; minima met by shuffles
        const int gi = (int)ctid / KP_PS, r = (int)ctid % KP_PS;
        const bool act = gi < cnt;
        float part = __builtin_huge_valf();
        if (act) {
            const uint32_t l = cur[0].x;
            const uint32_t npairs = cur[0].w & 0xFFu;
            const uint4 *lp = P.T.lpairs + (cur[0].w >> 8);
            const uint32_t nch = (npairs + 3u) >> 2;
            for (uint32_t c = (uint32_t)r; c < nch; c += KP_PS) kp_ws_chunk_min<BASE>(lp[c], &part);
#pragma unroll
            for (int m = 1; m < KP_PS; m <<= 1) part = fminf(part, __shfl_xor(part, m, KP_PS));
            if (r == 0) {
                kp_single_ctx sc;
                sc.exact = exact;
                kp_ptab_counts<CT, KP_PTAB_ALL>(g, lm, ptab, l, cur[0].z, &sc.c.mtr, &sc.c.utr);
                sc.kmer = false;
                sc.c.mte = sc.c.ute = 0;
                const double pr = kp_rate(sc.c, alpha, beta);
                sc.logp = kp_dlog<NL, MIX>(pr);
                sc.log1mp = kp_dlog<NL, MIX>(1.0 - pr);
                kp_lds_f32 *row = st + l;
                const double pj = pen[0];
                const float lmin = fminf(row[0], part);
                kp_cell_store<1>(row, &lmin, sc, &pj, alpha, beta, 0);
            }
        }
    } else if (cnt <= ncons) {  // one thread per cell, its whole pair list in flight
        if ((int)ctid < cnt) {
            const uint32_t l = cur[0].x;
            const uint32_t npairs = cur[0].w & 0xFFu;
            const uint4 *lp = P.T.lpairs + (cur[0].w >> 8);
            uint4 pre[KP_NARROW_CHUNKS];
#pragma unroll
            for (int c = 0; c < KP_NARROW_CHUNKS; ++c)
                if (4u * c < npairs) pre[c] = lp[c];
            kp_single_ctx sc;
            sc.exact = exact;
            kp_ptab_counts<CT, KP_PTAB_ALL>(g, lm, ptab, l, cur[0].z, &sc.c.mtr, &sc.c.utr);
            sc.kmer = false;
            sc.c.mte = sc.c.ute = 0;
            const double pr = kp_rate(sc.c, alpha, beta);
            sc.logp = kp_dlog<NL, MIX>(pr);
            sc.log1mp = kp_dlog<NL, MIX>(1.0 - pr);
            kp_ws_cell_list<KP_NARROW_CHUNKS, BASE>(l, npairs, pre, lp, sc, alpha, beta, pen);
        }
    } else {
#pragma unroll
        for (int k = 0; k < KP_IPT; ++k) {
            const int q = (int)ctid + k * ncons;
            if (q < cnt) {
                const uint32_t l = cur[k].x;
                const uint32_t npairs = cur[k].w & 0xFFu;
                const uint4 *lp = P.T.lpairs + (cur[k].w >> 8);
                uint4 pre[KP_PRE_CHUNKS];
#pragma unroll
                for (int c = 0; c < KP_PRE_CHUNKS; ++c)
                    if (4u * c < npairs) pre[c] = lp[c];
                kp_single_ctx sc;
                sc.exact = exact;
                kp_ptab_counts<CT, KP_PTAB_ALL>(g, lm, ptab, l, cur[k].z, &sc.c.mtr, &sc.c.utr);
                sc.kmer = false;
                sc.c.mte = sc.c.ute = 0;
                const double pr = kp_rate(sc.c, alpha, beta);
                sc.logp = kp_dlog<NL, MIX>(pr);
                sc.log1mp = kp_dlog<NL, MIX>(1.0 - pr);
                kp_ws_cell_list<KP_PRE_CHUNKS, BASE>(l, npairs, pre, lp, sc, alpha, beta, pen);
            }
        }
    }
}

// the level-lam descriptors of the consumer thread ctid (kp_dp_kernel's layout: one cell per
// thread on narrow levels, KP_PS threads per cell on the narrowest, else KP_IPT cells per
// thread; threads past the level's cells load its last descriptor and never use it)
__device__ inline void kp_ws_desc(const kp_dp_params &P, int lam, uint32_t ctid, int ncons, uint4 *d) {
    const uint4 *desc = reinterpret_cast<const uint4 *>(P.T.ldesc);
    const int beg = P.loffv[lam], cnt = P.loffv[lam + 1] - beg;
    if (cnt * KP_PS <= ncons) {
        d[0] = desc[beg + min((int)ctid / KP_PS, cnt - 1)];
    } else if (cnt <= ncons) {
        d[0] = desc[beg + min((int)ctid, cnt - 1)];
    } else {
#pragma unroll
        for (int k = 0; k < KP_IPT; ++k) d[k] = desc[beg + min((int)ctid + k * ncons, cnt - 1)];
    }
}

// the launch's parameters, re-read in every block: the persistent loop would otherwise keep
// every kernel argument it touches live in SGPRs across all blocks (they spilled)
// (a constant-address-space pointer: its loads stay scalar; the asm makes the pointer
// opaque each time so that they are not hoisted out of the loop)
typedef const __attribute__((address_space(4))) kp_dp_params kp_dp_params_c;
__device__ inline const kp_dp_params &kp_ws_params(kp_dp_params_c *PP) {
    asm volatile("" : "+s"(PP));
    return *(const kp_dp_params *)PP;
}

// LDS words of the hand-over protocol (monotonic counters, zeroed at kernel start)
struct kp_ws_sync {
    uint32_t full;   // producer waves that finished a block (block j done: full >= (j + 1) * PW)
    uint32_t free_;  // consumer waves that finished a block's levels (block i: free_ >= (i + 1) * CW)
    uint32_t cbar;   // consumer-wave barrier arrivals
    uint32_t pbar;   // producer-wave barrier arrivals
    uint32_t abort;  // a wait timed out: nobody waits any more
    uint32_t pad_[3];
};

#ifndef KP_WS_SPIN_LIMIT
#define KP_WS_SPIN_LIMIT (1u << 21)  // polls (s_sleep 2 each) before a wait gives up: ~0.2 s
#endif

// wait until *ctr >= target (every lane of the wave polls the same LDS word; relaxed polls,
// one acquire).  Bounded: on timeout the workgroup's abort word and the plan's error word
// are set and every later wait returns at once
__device__ inline void kp_ws_wait(uint32_t *ctr, uint32_t target, kp_ws_sync *sy, uint32_t *werr) {
    uint32_t n = 0;
    while (__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < target) {
        if (__hip_atomic_load(&sy->abort, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) break;
        __builtin_amdgcn_s_sleep(2);
        if (++n > KP_WS_SPIN_LIMIT) {
            if (__lane_id() == 0) {
                __hip_atomic_store(&sy->abort, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                if (werr) atomicOr(werr, 1u);
            }
            break;
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

// this wave's LDS (and memory) writes released, then one arrival on ctr
__device__ inline void kp_ws_arrive(uint32_t *ctr) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    if (__lane_id() == 0) __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// barrier of the nw waves of one role: generation gen (1, 2, ...) is complete when nw * gen
// arrivals have been counted
__device__ inline void kp_ws_role_barrier(uint32_t *ctr, uint32_t nw, uint32_t &gen, kp_ws_sync *sy, uint32_t *werr) {
    ++gen;
    kp_ws_arrive(ctr);
    kp_ws_wait(ctr, nw * gen, sy, werr);
}

// one block's row buffer to HBM (non-temporal float4 stores: the rows are read by later
// launches only)
template <int NL>
__device__ inline void kp_ws_store(const kp_dp_params &P, const float *buf, uint64_t h, uint32_t lane0, uint32_t tid,
                                   uint32_t nth) {
    const kp_geom &g = P.g;
    const uint64_t rowstride = (uint64_t)g.Ltot * g.Bpad;
    const uint32_t nch = g.Bpad / 4;
    for (uint32_t item = tid; item < (uint32_t)NL * nch; item += nth) {
        const uint32_t ll = item / nch, c = item % nch;
        const float *sl = buf + (size_t)(4 * c) * NL + ll;
        float4 *dst = reinterpret_cast<float4 *>(P.S + h * rowstride + (uint64_t)(lane0 + ll) * g.Bpad + 4 * c);
        typedef float kp_f4v __attribute__((ext_vector_type(4)));
        const kp_f4v w = {sl[0], sl[NL], sl[2 * NL], sl[3 * NL]};
        __builtin_nontemporal_store(w, reinterpret_cast<kp_f4v *>(dst));
    }
}

// the consumer's levels of one block in row buffer BASE, an LDS counter barrier between
// levels (the last level's writes are released by the FREE arrival instead)
template <typename CT, int NL, uint32_t BASE>
__device__ inline void kp_ws_levels(kp_dp_params_c *PP, int lmax, const uint8_t *lm, const CT *ptab, const double *pen,
                                    double alpha, double beta, bool exact, uint32_t ctid, int ncons, uint4 *cur,
                                    uint32_t &cgen, kp_ws_sync *sy, uint32_t *werr) {
    const kp_dp_params &P = kp_ws_params(PP);
    for (int lam = 0; lam <= lmax; ++lam) {
        uint4 nxt[KP_IPT];
        kp_ws_desc(P, lam < lmax ? lam + 1 : 0, ctid, ncons, nxt);  // the next level's (or block's) cells
        kp_ws_level<CT, NL, BASE>(P, lam, cur, lm, ptab, nullptr, pen, alpha, beta, exact, ctid, ncons);
#pragma unroll
        for (int k = 0; k < KP_IPT; ++k) cur[k] = nxt[k];
        if (lam < lmax) kp_ws_role_barrier(&sy->cbar, KP_WS_CW, cgen, sy, werr);
    }
}

// The persistent wave-specialised sweep of one launch (one high level >= 1, so no k-mer
// cells) for 1-lane device groups (blockIdx.y = the class's device group).  Workgroup w
// takes the launch's virtual blocks w, w + W, ... (W = gridDim.x, a multiple of 8, so a
// workgroup stays on one XCD and the XCD-aware remap of kp_dp_kernel applies unchanged).
// The two roles run separate loops (a wave-uniform branch: each wave is wholly one role).
// LDS: row buffers at 0 and KP_WS_BASE1 | ptab[2] | count scratch A, B | hp | lm | sync
template <typename CT, int NL>
__global__ void __launch_bounds__(KP_WS_THREADS) __attribute__((amdgpu_waves_per_eu(KP_WS_WAVES)))
kp_dp_ws_kernel(const kp_dp_params *Pg, uint32_t nb) {
    static_assert(NL == 1, "the wave-specialised sweep holds one lane");
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    kp_dp_params_c *PP = (kp_dp_params_c *)Pg;  // the launch's parameters in device memory (read-only)
    const kp_dp_params &P0 = kp_ws_params(PP);
    const kp_geom &g0 = P0.g;
    uint32_t *werr = P0.werr;
    const uint32_t tid = threadIdx.x;
    constexpr uint32_t NPROD = KP_WS_PW * 64;
    const int ncons = (int)blockDim.x - (int)NPROD;
    const kp_group_dev *G = P0.groups + blockIdx.y;
    const uint32_t lane0 = (uint32_t)G->lane0;

    const size_t ptab_elems = ((size_t)P0.ptab_entries * 2 + 3) & ~(size_t)3;
    const size_t scr_elems = ((size_t)P0.wscratch_entries * 2 + 3) & ~(size_t)3;
    CT *ptabs = reinterpret_cast<CT *>(smem + 2 * KP_WS_BASE1);
    CT *bufA = ptabs + 2 * ptab_elems;
    CT *bufB = bufA + scr_elems;
    kp_hpair *hp = reinterpret_cast<kp_hpair *>(bufB + scr_elems);
    uint8_t *lm = reinterpret_cast<uint8_t *>(hp + (g0.kh * 7 + 1));
    kp_ws_sync *sy = reinterpret_cast<kp_ws_sync *>(lm + ((g0.t * 16 + 15) & ~15));
    for (uint32_t e = tid; e < (uint32_t)g0.t * 16u; e += blockDim.x) lm[e] = P0.T.lowmask[e];
    if (tid == 0) {
        sy->full = sy->free_ = sy->cbar = sy->pbar = sy->abort = 0;
    }

    const uint32_t W = gridDim.x, w = blockIdx.x;
    const int nblk = w < nb ? (int)((nb - w + W - 1) / W) : 0;
    const int lmax = P0.lmax;
    __syncthreads();  // lm, sync words (the only workgroup barrier)

    if ((uint32_t)__builtin_amdgcn_readfirstlane((int)tid) < NPROD) {
        // ---- producer waves: block j into buffer j & 1, after storing block j - 2 from it ----
        const int fold = G->fold;
        const uint32_t ptid = tid;
        uint32_t pgen = 0;
        uint64_t hj1 = 0, hj2 = 0;  // block ids of blocks j - 1 and j - 2
        for (int j = 0; j < nblk + 2; ++j) {
            const kp_dp_params &P = kp_ws_params(PP);
            const kp_geom &g = P.g;
            const int pb = j & 1;
            float *pst = reinterpret_cast<float *>(smem + (pb ? KP_WS_BASE1 : 0u));
            CT *pptab = ptabs + (size_t)pb * ptab_elems;
            if (j >= 2) {  // block j - 2's levels are done: its rows to HBM, then the buffer is ours
                kp_ws_wait(&sy->free_, (uint32_t)(j - 1) * KP_WS_CW, sy, werr);
                kp_ws_store<NL>(P, pst, hj2, lane0, ptid, NPROD);
            }
            if (j < nblk) {
                // every producer wave is past block j - 1's gather (hp) and count steps (bufA/B)
                // and block j - 2's store (this buffer) before any of them rewrites those
                kp_ws_role_barrier(&sy->pbar, KP_WS_PW, pgen, sy, werr);
                const CT *K = reinterpret_cast<const CT *>(P.K);
                const uint64_t rowstride = (uint64_t)g.Ltot * g.Bpad;
                const uint32_t v = w + (uint32_t)j * W;
                const uint32_t widx = kp_ws_remap(v, nb, P.remap);
                const uint64_t pq = P.hbase + widx;
                const uint32_t kl = ptid < g.n_kl ? ptid : 0u;
                const CT *row = K + (pq * g.n_kl + kl) * 2;
                const CT *fr = row + kp_kslot_elems(g) * (uint64_t)(fold >= 0 ? 1 + fold : 0);
                const CT k0 = row[0], k1 = row[1], k2 = fr[0], k3 = fr[1];
                const uint64_t ph = P.T.hlist[pq];
                const uint64_t hn = P.T.hnp[pq];
                int np = 0, nnt = 0;
                for (int q = 0; q < g.kh; ++q) {
                    const int npi = (int)(hn >> (3 * q)) & 7;
                    np += npi;
                    if ((P.ntmask >> q) & 1u) nnt += npi;
                }
                if (ptid < 64) {  // wave 0: the pairs as child-row offsets, non-temporal ones first
                    const uint32_t p = ptid;
                    const uint64_t e = p < P.T.hps ? P.T.hpd[pq * P.T.hps + p] : 0;
                    const bool valid = (int)p < np;
                    const uint32_t pos = (uint32_t)(e >> 58);
                    const bool ntp = valid && ((P.ntmask >> pos) & 1u);
                    const uint64_t bnt = __ballot(ntp), bv = __ballot(valid);
                    const uint64_t below = (1ull << p) - 1ull;
                    if (valid) {
                        const int slot = ntp ? __popcll(bnt & below) : nnt + __popcll(bv & ~bnt & below);
                        hp[slot].h1 = (ph - (e & 0x1FFFFFFFull)) * rowstride;
                        hp[slot].h2 = (ph - ((e >> 29) & 0x1FFFFFFFull)) * rowstride;
                        hp[slot].code = pos;
                    }
                }
                const uint64_t kte_m = fold >= 0 ? (uint64_t)k2 : 0, kte_u = fold >= 0 ? (uint64_t)k3 : 0;
                const kp_cnt kpre = {(uint64_t)k0 - kte_m, (uint64_t)k1 - kte_u, 0, 0};
                kp_ws_count_step<CT>(g, 0, K, pq, fold, lm, bufA, bufB, pptab, ptid, NPROD, kpre);
                kp_ws_role_barrier(&sy->pbar, KP_WS_PW, pgen, sy, werr);  // hp, T_0
                if (!KP_SKIP(P, 1))  // (timing-ablation builds only: skip the gather)
                    kp_ws_gather<NL, KP_WS_NI, KP_WS_PU>(P, hp, 0, np, nnt, true, true, lane0, pst, ptid, NPROD);
                for (int s = 1; s < g.t; ++s) {
                    kp_ws_count_step<CT>(g, s, K, pq, fold, lm, bufA, bufB, pptab, ptid, NPROD, kp_cnt{});
                    if (s + 1 < g.t) kp_ws_role_barrier(&sy->pbar, KP_WS_PW, pgen, sy, werr);
                }
                kp_ws_arrive(&sy->full);  // block j is in buffer pb (rows, count table, id)
                hj2 = hj1;
                hj1 = ph;
            } else {
                hj2 = hj1;
            }
        }
    } else {
        // ---- consumer waves: block i's levels in buffer i & 1 ----
        const uint32_t ctid = tid - NPROD;
        const double alpha = G->alpha, beta = G->beta;
        double pen[NL];
        pen[0] = G->pen[0];
        const bool exact = P0.exact != 0 || !kp_fast_logs_ok(G->pen, G->nl, alpha, beta);
        uint4 cur[KP_IPT];
        kp_ws_desc(P0, 0, ctid, ncons, cur);
        uint32_t cgen = 0;
        for (int i = 0; i < nblk; ++i) {
            kp_ws_wait(&sy->full, (uint32_t)(i + 1) * KP_WS_PW, sy, werr);
            const CT *cptab = ptabs + (size_t)(i & 1) * ptab_elems;
            if (KP_SKIP(P0, 2)) {  // (timing-ablation builds only: no level phase)
            } else if (i & 1)
                kp_ws_levels<CT, NL, KP_WS_BASE1>(PP, lmax, lm, cptab, pen, alpha, beta, exact, ctid, ncons, cur, cgen,
                                                  sy, werr);
            else
                kp_ws_levels<CT, NL, 0u>(PP, lmax, lm, cptab, pen, alpha, beta, exact, ctid, ncons, cur, cgen, sy,
                                         werr);
            kp_ws_arrive(&sy->free_);  // block i's levels are done (its buffer may be stored and reused)
        }
    }
}
