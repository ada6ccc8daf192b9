// kp_dp_kernel.h -- the lattice-DP sweep kernel (value-only), included by kp_hip.hip.
//
// Kept in its own file so that profiles can be tied to the exact sweep source: the
// kernel tag bench.py records (engine.kernel_tag) hashes kp_core.h, kp_plan.h and this
// file only.  See kp_hip.hip's header for the phases.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "kp_core.h"

#define KP_DP_MAX_THREADS 1024
#define KP_DP_MAX_LEVELS (3 * KP_MAXT)  // low levels of a block (<= 3 per N position)

// LDS-qualified element types: pointers to them are 32-bit and address LDS directly
typedef __attribute__((address_space(3))) float kp_lds_f32;
typedef __attribute__((address_space(3))) uint64_t kp_lds_u64;

struct kp_dev_tables {
    const kp_postab *tabs;
    const uint32_t *lowinfo;
    const int32_t *loff;
    const uint32_t *klofs;
    const uint16_t *kllist;
    const uint32_t *hlist;
    const kp_lowdesc *ldesc;
    const uint64_t *hdig;
    const uint64_t *hnp;
    const uint32_t *kpos;  // block -> its position in the block list = its count row of K
    const uint8_t *lowmask;
    const uint4 *lpairs;  // low split-pair lists in 4-pair chunks (kp_plan.h lpairs)
    // [block list][hps] the block's high split pairs in scan order as kp_hpd_word (child
    // block deltas + position), built once per plan by kp_hpd_kernel; null when a block
    // can have more than 64 pairs (then the pairs come from hdig / tabs)
    const uint64_t *hpd;
    uint32_t hps;
};

struct kp_dp_params {
    kp_geom g;
    kp_dev_tables T;
    const void *K;
    float *S;
    const kp_group_dev *groups;
    uint64_t hbase;
    int H;
    int lmax;
    int32_t loffv[KP_DP_MAX_LEVELS + 2];  // level offsets of the low cells (kernel arguments: scalar loads,
                                          // not vector loads whose waits stalled every level's start)
    uint32_t ptab_entries;     // separable count table entries (kp_plan.h)
    uint32_t pscratch_entries; // largest intermediate table of its build
    uint32_t wscratch_entries; // largest table before the last step (kp_dp_ws.h's build buffers)
    int remap;  // block -> XCD mapping: G > 1 = runs of G list entries per XCD (default 40),
                // 1 = XCD-contiguous (7 % slower), 0 = hardware round-robin
    int lanesplit;  // split a cell's lanes over threads on narrow levels (KP_LANE_SPLIT=0 disables)
    int ntstore;    // 1 = score rows stored non-temporally (default; KP_NT_STORE=0 for plain stores)
    uint32_t ntmask;  // high positions whose child rows are loaded non-temporally (bit i = high position i)
    unsigned long long *stamps;  // diagnostic build only (-DKP_STAMPS): per-phase cycle sums
    uint32_t *werr;              // kp_dp_ws_kernel: set when a hand-over wait timed out (the pass fails)
    int exact;      // 1 = every cell's single term from the C library's logs (KP_EXACT_LOGS=1)
    int dbg;  // -DKP_ABLATION builds only (KP_DEBUG_SKIP, wrong results; always 0 otherwise): 1 = skip gather, 2 = skip level phase,
              // 4 = skip logs, 8 = skip low split scan, 16 = no level barrier
};

#ifdef KP_STAMPS
// diagnostic build: lane 0 of every workgroup sums the shader-clock ticks of each phase
// in LDS and flushes them with one global atomic per slot at the end (never read by the
// kernel; outputs are unchanged)
#define KP_STAMP(slot)                                                                        \
    do {                                                                                      \
        const unsigned long long t_ = __builtin_amdgcn_s_memtime();                           \
        if (threadIdx.x == 0) st_lds[slot] += t_ - st_prev;                                   \
        st_prev = t_;                                                                         \
    } while (0)
#else
#define KP_STAMP(slot) \
    do {               \
    } while (0)
#endif

// phase skipping of the timing-ablation build (-DKP_ABLATION); constant false otherwise
#ifdef KP_ABLATION
#define KP_SKIP(P, bit) (((P).dbg & (bit)) != 0)
#else
#define KP_SKIP(P, bit) false
#endif

#ifndef KP_IPT
#define KP_IPT 2  // low cells per thread per level (host checks level sizes)
#endif
// count-table reads of a cell all in flight at once (kp_ptab_counts ALL): A/B knob, see
// profiles/r03/experiments/count_reads_ab.txt
#ifndef KP_PTAB_ALL
#define KP_PTAB_ALL (NL == 1)
#endif
#ifndef KP_PS
// threads per (cell, lane) on a block's narrowest levels (power of 2, <= 64; 1-lane build only):
// one wave per (cell, lane) on the levels of <= 8 cells -- 1-lane pass 133.0 -> 127.7 ms
// (8: 133.0, 16: 129.4, 32: 132.8, 64: 127.7; profiles/r04/experiments/ps_ab.txt)
#define KP_PS 64
#endif
#ifndef KP_NARROW_CHUNKS
#define KP_NARROW_CHUNKS KP_PRE_CHUNKS  // pair chunks prefetched per cell on lane-split (narrow) levels
#endif

// the fast path's float64 log (within 2 ulp of the C library's: the store guard, kp_core.h
// kp_store_unsafe, sends every result that could depend on it to the C library's restated
// log).  Single-alpha builds of NL lanes with bit NL of KP_FMA_LOG_MASK set take
// kp_fma_log (kp_libm.h: fdlibm's algorithm with the hardware reciprocal and FMAs, ~45
// instructions against ocml's ~80 of double-double arithmetic): pass 1 lane 124.3 -> 111.1
// ms, 4 lanes 317.9 -> 312.3, 5 lanes 380.3 -> 377.0.  The 2- and 3-lane builds (80 VGPRs at
// 6 waves per SIMD) keep the device's own log (ocml): with kp_fma_log their spills grow (3
// lanes 248 -> 284 ms, 2 lanes 179 -> 206; profiles/r04/experiments/fmalog_ab.txt).  The
// mixed-group builds (two rates, four logs per cell) of 4+ lanes take kp_fma_log since the
// split scan's half chunks (KP_CHUNK_SPLIT) freed their registers: 5-lane mixed 123 -> 126
// VGPRs, no VGPR spill, SGPR spills 24 -> 18; pass 397 -> 382 ms, 2 + 2 lanes 353 -> 339
// (profiles/r05/experiments/fmamix_ab.txt; before the half chunks: 404 -> 409).
// -DKP_FAST_LOG: kp_fast_log (fdlibm, IEEE division) in every build (A/B only).
#ifndef KP_FMA_LOG_MASK
#define KP_FMA_LOG_MASK 0x1F2u  // NL = 1, 4, 5, 6, 7, 8
#endif
#ifndef KP_FMA_LOG_MIX
#define KP_FMA_LOG_MIX 1  // the mixed builds too (of the NL in the mask: 4-8 lanes); 0 = ocml there (A/B)
#endif
template <int NL, bool MIX>
__device__ inline double kp_dlog(double x) {
#ifdef KP_FAST_LOG
    return kp_fast_log(x);
#else
    if constexpr ((((KP_FMA_LOG_MASK) >> NL) & 1u) && (!MIX || KP_FMA_LOG_MIX))
        return kp_fma_log(x);
    else
        return log(x);
#endif
}
#define KP_DLOG(x) kp_dlog<NL, MIX>(x)

// v[j] of a small register array for a per-lane j, as a select chain (no memory access)
template <int N>
__device__ inline double kp_pick(const double (&v)[N], uint32_t j) {
    double r = v[0];
#pragma unroll
    for (int i = 1; i < N; ++i) r = (j == (uint32_t)i) ? v[i] : r;
    return r;
}

// a workgroup-uniform 64-bit value (read by every lane from the same LDS word) into SGPRs
__device__ inline uint64_t kp_rfl64(uint64_t v) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)v);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(v >> 32));
    return ((uint64_t)hi << 32) | lo;
}

// float4 min-update with a split candidate a + b (fminf drops NaN candidates like "<")
__device__ inline void kp_min4v(float4 &best, const float4 a, const float4 b) {
    best.x = fminf(best.x, a.x + b.x);
    best.y = fminf(best.y, a.y + b.y);
    best.z = fminf(best.z, a.z + b.z);
    best.w = fminf(best.w, a.w + b.w);
}

// one child-row float4 load; NT = non-temporal (no cache allocation, for rows that will
// not be read again soon)
template <bool NT>
__device__ inline float4 kp_ld4(const float *p) {
    if (NT) {
        typedef float kp_f4v __attribute__((ext_vector_type(4)));
        const kp_f4v v = __builtin_nontemporal_load(reinterpret_cast<const kp_f4v *>(p));
        return make_float4(v.x, v.y, v.z, v.w);
    }
    return *reinterpret_cast<const float4 *>(p);
}

// pairs p0..p1 of the block's high split pairs, NI items per thread, PU pairs per step
template <int NI, int PU, bool NT>
__device__ inline void kp_gather_range(const kp_dp_params &P, const kp_hpair *hp, int p0, int p1,
                                       const uint32_t *o, float4 *best) {
    int p = p0;
    for (; p + PU <= p1; p += PU) {
        const float *r[2 * PU];
#pragma unroll
        for (int q = 0; q < PU; ++q) {
            r[2 * q] = P.S + kp_rfl64(hp[p + q].h1);
            r[2 * q + 1] = P.S + kp_rfl64(hp[p + q].h2);
        }
        float4 v[NI][2 * PU];
#pragma unroll
        for (int q = 0; q < 2 * PU; ++q)
#pragma unroll
            for (int i = 0; i < NI; ++i) v[i][q] = kp_ld4<NT>(r[q] + o[i]);
#pragma unroll
        for (int q = 0; q < PU; ++q)
#pragma unroll
            for (int i = 0; i < NI; ++i) kp_min4v(best[i], v[i][2 * q], v[i][2 * q + 1]);
    }
    for (; p < p1; ++p) {
        const float *ra = P.S + kp_rfl64(hp[p].h1), *rb = P.S + kp_rfl64(hp[p].h2);
#pragma unroll
        for (int i = 0; i < NI; ++i) kp_min4v(best[i], kp_ld4<NT>(ra + o[i]), kp_ld4<NT>(rb + o[i]));
    }
}

// Gather phase of one block: st[cell][lane] = min over the block's high split pairs of
// S[child1] + S[child2], for the NL lanes.  Items are float4 runs (4 cells of one lane);
// each thread takes NI items at a time (NI * 2 * min(np, PU) row loads in flight).  A
// pair's child-row offsets are workgroup-uniform: read into SGPRs, so each load is a
// scalar base plus a 32-bit lane offset.  Pairs 0..nnt-1 (the plan's slowest-varying
// high positions, whose child rows are not re-read while they could still be cached) use
// non-temporal loads.  Slot B (padding) becomes +inf: the cell that padded pair lists
// point at (kp_dp_cell_list).
template <int NL, int NI, int PU = 4>
__device__ inline void kp_gather_items(const kp_dp_params &P, const kp_hpair *hp, int np, int nnt, uint32_t lane0,
                                       float *st) {
    const kp_geom &g = P.g;
    const uint32_t Bpad = g.Bpad, nch = Bpad / 4, nitems = (uint32_t)NL * nch;
    const float inf = __builtin_huge_valf();
    for (uint32_t it0 = threadIdx.x; it0 < nitems; it0 += NI * blockDim.x) {
        uint32_t it[NI], o[NI];
        float4 best[NI];
#pragma unroll
        for (int i = 0; i < NI; ++i) {
            it[i] = (it0 + i * blockDim.x < nitems) ? it0 + i * blockDim.x : it0;
            o[i] = (lane0 + it[i] / nch) * Bpad + 4 * (it[i] % nch);
            best[i] = make_float4(inf, inf, inf, inf);
        }
        if (nnt > 0) kp_gather_range<NI, PU, true>(P, hp, 0, nnt, o, best);
        kp_gather_range<NI, PU, false>(P, hp, nnt, np, o, best);
#pragma unroll
        for (int i = 0; i < NI; ++i) {
            if (i > 0 && it[i] == it0) break;
            const uint32_t ll = it[i] / nch, c = it[i] % nch;
            if (4 * c + 4 > g.B) {
                if (4 * c + 0 >= g.B) best[i].x = inf;
                if (4 * c + 1 >= g.B) best[i].y = inf;
                if (4 * c + 2 >= g.B) best[i].z = inf;
                if (4 * c + 3 >= g.B) best[i].w = inf;
            }
            float *sl = st + (size_t)(4 * c) * NL + ll;
            sl[0] = best[i].x;
            sl[NL] = best[i].y;
            sl[2 * NL] = best[i].z;
            sl[3 * NL] = best[i].w;
        }
    }
}

// Groups of 1-3 lanes (penalties split off their (alpha, fold) group, e.g. by the
// multi-GPU lane split) are latency-bound and their LDS fits 3 workgroups per CU: ask for
// KP_SMALL_WAVES waves per SIMD (6: <= 80 VGPRs, 3 workgroups of 512 threads per CU;
// 1-lane pass 188 -> 157 ms) and gather 2 items per thread instead of 4
#ifndef KP_SMALL_WAVES
#define KP_SMALL_WAVES 6
#endif
#ifndef KP_SMALL_NL
#define KP_SMALL_NL 3  // widest group built for KP_SMALL_WAVES (A/B knob)
#endif
#ifndef KP_ONE_WAVES
#define KP_ONE_WAVES KP_SMALL_WAVES  // the 1-lane build's waves per SIMD (A/B knob)
#endif
// HZ: the build that handles k-mer cells (only high level 0's blocks hold them; their
// xlogy / xlog1py terms call the C library's logs, kp_libm.h); launches of higher levels
// may use the build without that code (kp_hip.hip launch_dp).  MIX: the build for launch
// classes that hold mixed groups (kp_group_dev.nl2 > 0: a second (alpha, beta) set for the
// group's last lanes, a second pair of logs per cell); other classes use MIX = false
template <typename CT, int NL, bool HZ, bool MIX>
__global__ void __launch_bounds__(KP_DP_MAX_THREADS)
__attribute__((amdgpu_waves_per_eu(NL == 1 ? KP_ONE_WAVES : NL <= KP_SMALL_NL ? KP_SMALL_WAVES : 1)))
kp_dp_kernel(kp_dp_params P) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const kp_geom &g = P.g;
#ifdef KP_STAMPS
    unsigned long long st_prev = __builtin_amdgcn_s_memtime();
    const unsigned long long st_real0 = __builtin_amdgcn_s_memrealtime(), st_t0 = st_prev;
#endif
    uint32_t widx = blockIdx.x;
    if (P.remap == 1) {  // XCD-contiguous runs of the level's block list (A/B option)
        const uint32_t nb = gridDim.x, q = nb >> 3, r = nb & 7u, x = blockIdx.x & 7u;
        widx = x * q + (x < r ? x : r) + (blockIdx.x >> 3);
    } else if (P.remap > 1) {  // runs of G = remap consecutive list entries per XCD (A/B option)
        const uint32_t G = (uint32_t)P.remap, full = gridDim.x / (8 * G) * (8 * G);
        if (blockIdx.x < full) {
            const uint32_t x = blockIdx.x & 7u, sl = blockIdx.x >> 3;
            widx = ((sl / G) * 8 + x) * G + sl % G;
        }
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
    // mixed group: lanes js.. take (alpha2, beta2); js = NL when the group is not mixed
    const int js = MIX ? G->nl - G->nl2 : NL;
    const double alpha2 = MIX ? G->alpha2 : alpha, beta2 = MIX ? G->beta2 : beta;
    const bool exact = P.exact != 0 || !kp_fast_logs_ok(G->pen, G->nl, alpha, beta) ||
                       (MIX && js < NL && !kp_fast_logs_ok(G->pen, G->nl, alpha2, beta2));

    // LDS: st[Bpad][NL] f32 (lanes interleaved) | ptab[PE][2] CT | hp[] | lm[t][16]
    //      (count-table scratch aliases st, which the gather fills afterwards; every carve
    //       offset is a multiple of 16 bytes)
    const size_t st_bytes = (size_t)NL * Bpad * 4, scr_bytes = (size_t)P.pscratch_entries * 4 * sizeof(CT);
    unsigned char *lbase = smem;
    float *st = reinterpret_cast<float *>(lbase);
    CT *ptab = reinterpret_cast<CT *>(lbase + (st_bytes > scr_bytes ? st_bytes : ((scr_bytes + 15) & ~(size_t)15)));
    kp_hpair *hp = reinterpret_cast<kp_hpair *>(ptab + (((size_t)P.ptab_entries * 2 + 3) & ~(size_t)3));
    uint8_t *lm = reinterpret_cast<uint8_t *>(hp + (g.kh * 7 + 1));
#ifdef KP_STAMPS
    unsigned long long *st_lds = reinterpret_cast<unsigned long long *>(lm + ((g.t * 16 + 15) & ~15));
    if (threadIdx.x < 32) st_lds[threadIdx.x] = 0;
#endif

    const CT *K = reinterpret_cast<const CT *>(P.K);
    // this thread's k-mer-low count row (the count table's first step), loaded before the
    // high-pair setup below so that the two latencies overlap (unconditional raw loads from
    // valid rows -- a branch would make the compiler wait for them at its join -- and the
    // subtraction after the setup).  K's rows are in block-list order: the address needs
    // no h, so these loads do not wait for the block-list load
    const uint64_t krow = P.hbase + widx;
    CT kraw[4];
    {
        const uint32_t kl = threadIdx.x < g.n_kl ? threadIdx.x : 0u;
        const CT *row = K + (krow * g.n_kl + kl) * 2;
        const CT *fr = row + kp_kslot_elems(g) * (uint64_t)(fold >= 0 ? 1 + fold : 0);
        kraw[0] = row[0];
        kraw[1] = row[1];
        kraw[2] = fr[0];
        kraw[3] = fr[1];
    }
    // the block's high split pairs, scan order (kp_high_pairs): digits and pair counts per
    // high position come packed from the plan (no 64-bit division, no table lookups: the
    // only dependent loads are the pair digits), and wave 0 writes one pair per lane
    const uint64_t hd = P.T.hdig[P.hbase + widx];
    const uint64_t hn = P.T.hnp[P.hbase + widx];
    int np = 0, nnt = 0;
    if (!KP_SKIP(P, 1))
        for (int i = 0; i < g.kh; ++i) {
            const int npi = (int)(hn >> (3 * i)) & 7;
            np += npi;
            if ((P.ntmask >> i) & 1u) nnt += npi;
        }
    const uint64_t rowstride = (uint64_t)g.Ltot * Bpad;
    if (P.T.hpd) {
        // wave 0, lane p = pair p: its child-block deltas come in one load that needs neither
        // h nor the pair counts (the padding words past np are loaded and unused), so the
        // block setup costs one dependent round trip, not two; the non-temporal positions'
        // pairs go first (slot = rank among the pairs of the same kind)
        if (threadIdx.x < 64) {
            const uint32_t p = threadIdx.x;
            const uint64_t e = p < P.T.hps ? P.T.hpd[(P.hbase + widx) * P.T.hps + p] : 0;
            const bool valid = (int)p < np;
            const uint32_t pos = (uint32_t)(e >> 58);
            const bool ntp = valid && ((P.ntmask >> pos) & 1u);
            const uint64_t bnt = __ballot(ntp), bv = __ballot(valid);
            const uint64_t below = (1ull << p) - 1ull;
            if (valid) {
                const int slot = ntp ? __popcll(bnt & below) : nnt + __popcll(bv & ~bnt & below);
                hp[slot].h1 = (h - (e & 0x1FFFFFFFull)) * rowstride;  // child rows as element offsets of lane 0
                hp[slot].h2 = (h - ((e >> 29) & 0x1FFFFFFFull)) * rowstride;
                hp[slot].code = pos;
            }
        }
    } else
    for (int p = (int)threadIdx.x; threadIdx.x < 64 && p < np; p += 64) {  // wave 0
        // pair p in scan order; slot: the non-temporal positions' pairs first (the sweep
        // only takes a min, so pair order does not matter here)
        int rem = p, i = 0, before_nt = 0, before_t = 0;
        uint32_t d = 0;
        for (; i < g.kh; ++i) {
            d = (uint32_t)(hd >> (4 * i)) & 15u;
            const int npi = (int)(hn >> (3 * i)) & 7;
            if (rem < npi) break;
            rem -= npi;
            if ((P.ntmask >> i) & 1u) before_nt += npi; else before_t += npi;
        }
        const int slot = ((P.ntmask >> i) & 1u) ? before_nt + rem : nnt + before_t + rem;
        const kp_postab &T = P.T.tabs[g.t + i];
        hp[slot].h1 = (h - (uint64_t)(d - T.pa[d][rem]) * g.hcg[i]) * rowstride;  // child rows as element
        hp[slot].h2 = (h - (uint64_t)(d - T.pb[d][rem]) * g.hcg[i]) * rowstride;  // offsets of lane 0
        hp[slot].code = (uint32_t)(((g.t + i) << 3) | rem);
    }
    for (uint32_t e = threadIdx.x; e < (uint32_t)g.t * 16u; e += blockDim.x) lm[e] = P.T.lowmask[e];
    __syncthreads();  // lm is read by every thread below

    // ---- separable count tables (train counts of the group fold), kp_core.h ----
    // (kp_kl_counts of the preloaded row: train = all data - fold, CV :22-24)
    const uint64_t kte_m = fold >= 0 ? (uint64_t)kraw[2] : 0, kte_u = fold >= 0 ? (uint64_t)kraw[3] : 0;
    const kp_cnt kpre = {(uint64_t)kraw[0] - kte_m, (uint64_t)kraw[1] - kte_u, kte_m, kte_u};
    kp_build_count_table<CT>(g, K, krow, fold, lm, reinterpret_cast<CT *>(lbase),
                             reinterpret_cast<CT *>(lbase) + (size_t)P.pscratch_entries * 2, ptab, threadIdx.x,
                             blockDim.x, [] { __syncthreads(); }, &kpre);
    __syncthreads();
    KP_STAMP(0);

    // ---- gather: high-position splits, as whole child-block rows (value only) ----
    // four float4 items per thread at a time, two pairs per step: 16 row loads in flight
    // per thread even when the block has few pairs (measured best of 1-4 items x 1-4 pairs)
    kp_gather_items<NL, (NL <= KP_SMALL_NL ? 2 : 4), 2>(P, hp, np, nnt, lane0, st);

    // ---- levels: low cells inside the block, level by level ----
    // one thread per cell: counts and the float64 logs once per cell for all NL lanes;
    // the next level's descriptors are loaded while the current level computes
    const bool high_zero = HZ && P.H == 0;
    const int lmax = KP_SKIP(P, 2) ? -1 : P.lmax;
    const uint4 *desc = reinterpret_cast<const uint4 *>(P.T.ldesc);
    // narrow levels (cells x lanes <= threads, e.g. the block's top levels) split each
    // cell's lanes over NL threads: the same work with a 1/NL-long dependent chain
    const int nthr = (int)blockDim.x;
    // threads per cell of a level: KP_PS * NL on the narrowest levels (the block's top
    // cells: each (cell, lane) split over KP_PS threads by pair chunks, partial minima
    // combined by wave shuffles), NL on narrow ones (one lane per thread), else 1 (KP_IPT
    // cells per thread)
    // (pair split only in the 1-lane build: wider builds spill with it; A/B: 1 lane 136.2 ->
    // 134.2 ms, 3 lanes 248 -> 406, 5 lanes 380 -> 398)
    constexpr bool kPS = NL == 1;
    auto cell_threads = [&](int cells) {
        return !P.lanesplit ? 1 : (kPS && cells * NL * KP_PS <= nthr) ? NL * KP_PS : cells * NL <= nthr ? NL : 1;
    };
    auto lane_split = [&](int cells) { return cell_threads(cells) > 1; };
    // the first level's descriptors, loaded without branches (threads past the level's
    // cells load its last descriptor and never use it) and in flight across the barrier
    uint4 cur[KP_IPT], nxt[KP_IPT];
    {
        const int c = P.loffv[1] - P.loffv[0];
        if (lane_split(c)) {
            cur[0] = desc[P.loffv[0] + min((int)threadIdx.x / cell_threads(c), c - 1)];
        } else {
#pragma unroll
            for (int k = 0; k < KP_IPT; ++k) cur[k] = desc[P.loffv[0] + min((int)threadIdx.x + k * nthr, c - 1)];
        }
    }
    __syncthreads();
    // vmcnt(0) here, before the level loop: otherwise the compiler puts the wait for these
    // loads inside the loop body, where it also catches every level's descriptor prefetch
    __builtin_amdgcn_s_waitcnt(0x0F70);
    KP_STAMP(1);

    for (int lam = 0; lam <= lmax; ++lam) {
        const int beg = P.loffv[lam], cnt = P.loffv[lam + 1] - beg;
        if (lam < lmax) {  // (guarded loads here: the compiler then waits for them only at the level's end)
            const int nbeg = P.loffv[lam + 1], ncnt = P.loffv[lam + 2] - nbeg;
            if (lane_split(ncnt)) {
                const int q = (int)threadIdx.x / cell_threads(ncnt);
                if (q < ncnt) nxt[0] = desc[nbeg + q];
            } else {
#pragma unroll
                for (int k = 0; k < KP_IPT; ++k) {
                    const int q = (int)threadIdx.x + k * nthr;
                    if (q < ncnt) nxt[k] = desc[nbeg + q];
                }
            }
        }
        if (kPS && cell_threads(cnt) == NL * KP_PS) {
          if constexpr (kPS) {
            // each (cell, lane) on KP_PS consecutive lanes of one wave: thread r takes pair
            // chunks r, r + KP_PS, ...; the minima meet by shuffles (min is exact in any
            // order, NaN candidates drop out as in the sequential scan); the group's first
            // thread adds the gathered high minimum and the single-pattern term
            const int gi = (int)threadIdx.x / KP_PS, r = (int)threadIdx.x % KP_PS;
            const int q = gi / NL;
            const uint32_t j = (uint32_t)(gi % NL);
            const bool act = q < cnt && !KP_SKIP(P, 8);
            float part = __builtin_huge_valf();
            if (act) {
                const uint32_t l = cur[0].x;
                const uint32_t npairs = cur[0].w & 0xFFu;
                const uint4 *lp = P.T.lpairs + (cur[0].w >> 8);
                const uint32_t nch = (npairs + 3u) >> 2;
                for (uint32_t c = (uint32_t)r; c < nch; c += KP_PS)
                    kp_chunk_minv<NL, 1, 4, kp_sdwa_on<NL, MIX>()>((kp_lds_f32 *)st, lp[c], j, &part);
#pragma unroll
                for (int m = 1; m < KP_PS; m <<= 1) part = fminf(part, __shfl_xor(part, m, KP_PS));
                if (r == 0) {
                    kp_single_ctx sc;
                    const double aj = (MIX && (int)j >= js) ? alpha2 : alpha, bj = (MIX && (int)j >= js) ? beta2 : beta;
                    sc.exact = exact;
                    kp_ptab_counts<CT, KP_PTAB_ALL>(g, lm, ptab, l, cur[0].z, &sc.c.mtr, &sc.c.utr);
                    sc.kmer = high_zero && lam == 0;
                    sc.c.mte = sc.c.ute = 0;
                    sc.logp = sc.log1mp = 0.0;
                    if (!sc.kmer) {
                        const double pr = kp_rate(sc.c, aj, bj);
                        sc.logp = KP_DLOG(pr);
                        sc.log1mp = KP_DLOG(1.0 - pr);
                    }
                    kp_lds_f32 *row = (kp_lds_f32 *)st + l * NL + j;
                    const double pj = NL <= 2 ? kp_pick(pen, j) : G->pen[j];  // (registers: 2 lanes 185 -> 179 ms; 3-5 lanes slower)
                    if (sc.kmer) {
                        row[0] = kp_kmer_train(sc.c, aj, bj, pj);
                    } else {
                        const float lmin = fminf(row[0], part);
                        kp_cell_store<1>(row, &lmin, sc, &pj, aj, bj, j);
                    }
                }
            }  // (act is uniform over a group's KP_PS lanes: a shuffle only reads active lanes)
          }
        } else if (lane_split(cnt)) {
            const int q = (int)threadIdx.x / NL;
            const uint32_t j = threadIdx.x % NL;
            if (q < cnt && !KP_SKIP(P, 8)) {
                const uint32_t l = cur[0].x;
                const uint32_t info = cur[0].z;
                const uint32_t npairs = cur[0].w & 0xFFu;
                const uint4 *lp = P.T.lpairs + (cur[0].w >> 8);
                // narrow level: every chunk of the cell's list in flight at once (a 3-position
                // block's top cell has 21 pairs = 6 chunks; KP_NARROW_CHUNKS A/B knob)
                uint4 pre[KP_NARROW_CHUNKS];
#pragma unroll
                for (int c = 0; c < KP_NARROW_CHUNKS; ++c)
                    if (4u * c < npairs) pre[c] = lp[c];
                kp_single_ctx sc;
                sc.exact = exact;
                kp_ptab_counts<CT, KP_PTAB_ALL>(g, lm, ptab, l, info, &sc.c.mtr, &sc.c.utr);
                sc.kmer = high_zero && lam == 0;
                sc.c.mte = sc.c.ute = 0;
                sc.logp = sc.log1mp = 0.0;
                // one lane per thread: its own (alpha, beta) set
                const double aj = (MIX && (int)j >= js) ? alpha2 : alpha, bj = (MIX && (int)j >= js) ? beta2 : beta;
                if (!sc.kmer) {
                    const double pr = kp_rate(sc.c, aj, bj);
                    sc.logp = KP_DLOG(pr);
                    sc.log1mp = KP_DLOG(1.0 - pr);
                }
                const double pj = NL <= 2 ? kp_pick(pen, j) : G->pen[j];  // (registers: 2 lanes 185 -> 179 ms; 3-5 lanes slower)
                kp_dp_cell_list<NL, 1, false, KP_NARROW_CHUNKS>(l, npairs, pre, lp, (kp_lds_f32 *)st, sc, aj, bj, &pj, j);
            }
        } else
#pragma unroll
        for (int k = 0; k < KP_IPT; ++k) {
            const int q = (int)threadIdx.x + k * (int)blockDim.x;
            if (q < cnt) {
                const uint32_t l = cur[k].x;
                const uint32_t info = cur[k].z;
                // the cell's split-pair list (plan tables, L2-resident): issued before the
                // logs so the loads overlap them
                const uint32_t npairs = cur[k].w & 0xFFu;
                const uint4 *lp = P.T.lpairs + (cur[k].w >> 8);
                uint4 pre[KP_PRE_CHUNKS];
#pragma unroll
                for (int c = 0; c < KP_PRE_CHUNKS; ++c)
                    if (4u * c < npairs) pre[c] = lp[c];
                // counts: <= 4 table reads (the reference's M_mem/U_mem row of this cell)
                kp_single_ctx sc;
                sc.exact = exact;
                kp_ptab_counts<CT, KP_PTAB_ALL>(g, lm, ptab, l, info, &sc.c.mtr, &sc.c.utr);
                sc.kmer = high_zero && lam == 0;
                sc.c.mte = sc.c.ute = 0;
                sc.logp = sc.log1mp = 0.0;
                if (!sc.kmer && !KP_SKIP(P, 4)) {
                    const double pr = kp_rate(sc.c, alpha, beta);
                    sc.logp = KP_DLOG(pr);
                    sc.log1mp = KP_DLOG(1.0 - pr);
                }
                if (MIX) {  // the second set's logs (group-uniform branch)
                    sc.js = js;
                    sc.a2 = alpha2;
                    sc.b2 = beta2;
                    sc.logp2 = sc.logp;
                    sc.log1mp2 = sc.log1mp;
                    if (js < NL && !sc.kmer) {
                        const double pr2 = kp_rate(sc.c, alpha2, beta2);
                        sc.logp2 = KP_DLOG(pr2);
                        sc.log1mp2 = KP_DLOG(1.0 - pr2);
                    }
                }
                if (!KP_SKIP(P, 8)) {
                    kp_dp_cell_list<NL, NL, MIX>(l, npairs, pre, lp, (kp_lds_f32 *)st, sc, alpha, beta, pen);
                } else {  // timing ablation: no split scan, keep the single term
#pragma unroll
                    for (int j = 0; j < NL; ++j)
                        st[l * NL + j] = (float)kp_single_train(sc.c, sc.logp, sc.log1mp, pen[j]);
                }
            }
        }
        if (!KP_SKIP(P, 16)) __syncthreads();  // (ablation 16: timing without the level barrier)
        KP_STAMP(3 + lam);
#pragma unroll
        for (int k = 0; k < KP_IPT; ++k) cur[k] = nxt[k];
    }

    // ---- store the block's score rows ----
    const uint32_t nch = Bpad / 4;
    for (uint32_t item = threadIdx.x; item < (uint32_t)NL * nch; item += blockDim.x) {
        const uint32_t ll = item / nch, c = item % nch;
        const float *sl = st + (size_t)(4 * c) * NL + ll;
        float4 *dst = reinterpret_cast<float4 *>(P.S + h * rowstride + (uint64_t)(lane0 + ll) * Bpad + 4 * c);
        const float4 v = make_float4(sl[0], sl[NL], sl[2 * NL], sl[3 * NL]);
        if (P.ntstore) {
            typedef float kp_f4v __attribute__((ext_vector_type(4)));
            const kp_f4v w = {v.x, v.y, v.z, v.w};
            __builtin_nontemporal_store(w, reinterpret_cast<kp_f4v *>(dst));
        } else
            *dst = v;
    }
    KP_STAMP(2);
#ifdef KP_STAMPS
    if (threadIdx.x == 0 && P.stamps) {
        for (int q = 0; q < 30; ++q)
            if (st_lds[q]) atomicAdd(P.stamps + q, st_lds[q]);
        atomicAdd(P.stamps + 30, __builtin_amdgcn_s_memtime() - st_t0);
        atomicAdd(P.stamps + 31, __builtin_amdgcn_s_memrealtime() - st_real0);
    }
#endif
}

