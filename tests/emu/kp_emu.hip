// kp_emu.hip -- host-side emulation of the blocked lattice DP (TEST INFRASTRUCTURE).
//
// Runs exactly the per-item functions of kmerpapa_amd/csrc/kp_core.h that the gfx950
// kernels run, serially on the CPU, with the same memory layout, block order and level
// order.  It lets tests/test_emu.py check the block decomposition, the tie combination
// and the argmin backtrack against the oracle without a GPU.  It is never loaded by the
// product package.
#include <stdint.h>
#include <math.h>
#include <string.h>

#include <string>
#include <vector>

#include "../../kmerpapa_amd/csrc/kp_core.h"
#include "../../kmerpapa_amd/csrc/kp_libm.h"
#include "../../kmerpapa_amd/csrc/kp_plan.h"

namespace {
std::string g_err;

void cell_values(int nl, uint32_t l, uint32_t npairs, const uint4 *lp, float *st, const kp_single_ctx &sc, double a,
                 double b, const double *pen) {
    switch (nl) {
        case 1: kp_dp_cell_list<1, 1>(l, npairs, lp, lp, st, sc, a, b, pen); break;
        case 2: kp_dp_cell_list<2, 2>(l, npairs, lp, lp, st, sc, a, b, pen); break;
        case 3: kp_dp_cell_list<3, 3>(l, npairs, lp, lp, st, sc, a, b, pen); break;
        case 4: kp_dp_cell_list<4, 4>(l, npairs, lp, lp, st, sc, a, b, pen); break;
        case 5: kp_dp_cell_list<5, 5>(l, npairs, lp, lp, st, sc, a, b, pen); break;
        case 6: kp_dp_cell_list<6, 6>(l, npairs, lp, lp, st, sc, a, b, pen); break;
        case 7: kp_dp_cell_list<7, 7>(l, npairs, lp, lp, st, sc, a, b, pen); break;
        default: kp_dp_cell_list<8, 8>(l, npairs, lp, lp, st, sc, a, b, pen); break;
    }
}

template <typename CT>
int emu(const char *gp, uint32_t max_block, const CT *M, const CT *U, int nf, const kp_group_dev *groups, int ngroups,
        float *root_train, float *root_test, uint64_t *nleaves, float *dump_score, uint8_t *dump_code,
        uint64_t *leaves) {
    kp::host_plan hp;
    g_err = kp::build_plan(gp, max_block, hp);
    if (!g_err.empty()) return -1;
    kp_geom g = hp.g;
    g.nf = nf;
    uint32_t Ltot = 0;
    for (int i = 0; i < ngroups; ++i) Ltot += (uint32_t)groups[i].nl;
    g.Ltot = Ltot;
    const uint64_t KS = kp_kslots(g), se = kp_kslot_elems(g), per = (uint64_t)g.n_kl * 2;
    std::vector<CT> K(KS * se);
    // counts (kp_counts_kernel): slot-major, slot 0 = all data (sum of the folds), slot 1 + f = fold f
    for (int H = 0; H <= hp.hmax; ++H) {
        for (uint64_t q = hp.hoff[H]; q < hp.hoff[H + 1]; ++q) {
            uint64_t h = hp.hlist[q];
            if (H == 0) {
                uint64_t kbase = 0;
                for (int i = 0; i < g.kh; ++i) kbase += (uint64_t)kp_high_digit(g, h, i) * g.khw[i];
                for (uint64_t kl = 0; kl < g.n_kl; ++kl) {
                    CT am = 0, au = 0;
                    for (int f = 0; f < nf; ++f) {
                        CT *d = K.data() + se * (1 + f) + h * per + 2 * kl;
                        d[0] = M[(kbase + kl) * nf + f];
                        d[1] = U[(kbase + kl) * nf + f];
                        am += d[0];
                        au += d[1];
                    }
                    K[h * per + 2 * kl] = am;
                    K[h * per + 2 * kl + 1] = au;
                }
            } else {
                uint64_t h1 = h, h2 = h;
                for (int i = 0; i < g.kh; ++i) {
                    uint32_t d = kp_high_digit(g, h, i);
                    const kp_postab &T = hp.tabs[g.t + i];
                    if (T.np[d]) {
                        h1 = h - (uint64_t)(d - T.pa[d][0]) * g.hcg[i];
                        h2 = h - (uint64_t)(d - T.pb[d][0]) * g.hcg[i];
                        break;
                    }
                }
                for (uint64_t s = 0; s < KS; ++s)
                    for (uint64_t e = 0; e < per; ++e)
                        K[s * se + h * per + e] = K[s * se + h1 * per + e] + K[s * se + h2 * per + e];
            }
        }
    }
    // the value-only sweep, block by block in the kernel's order and layout
    std::vector<float> S(g.nblocks * (uint64_t)Ltot * g.Bpad, 0.0f);
    std::vector<kp_hpair> hpairs(KP_MAX_HPAIRS);
    std::vector<float> st;
    std::vector<CT> bufA((size_t)hp.pscratch_entries * 2), bufB(bufA.size()), ptab((size_t)hp.ptab_entries * 2);
    for (int H = 0; H <= hp.hmax; ++H) {
        for (uint64_t q = hp.hoff[H]; q < hp.hoff[H + 1]; ++q) {
            uint64_t h = hp.hlist[q];
            int np = kp_high_pairs(g, hp.tabs.data(), h, hpairs.data());
            for (int gi = 0; gi < ngroups; ++gi) {
                const kp_group_dev &G = groups[gi];
                st.assign((size_t)G.nl * g.Bpad, 0.0f);  // interleaved [cell][lane], like the kernel
                kp_build_count_table<CT>(g, K.data(), h, G.fold, hp.lowmask.data(), bufA.data(), bufB.data(),
                                         ptab.data(), 0u, 1u, [] {});
                // gather (values only)
                for (int ll = 0; ll < G.nl; ++ll) {
                    uint32_t lane = (uint32_t)G.lane0 + ll;
                    for (uint32_t l = 0; l < g.Bpad; ++l) {
                        float best = __builtin_huge_valf();
                        for (int p = 0; p < np; ++p)
                            best = fminf(best, S[kp_lane_row(g, hpairs[p].h1, lane) + l] +
                                                   S[kp_lane_row(g, hpairs[p].h2, lane) + l]);
                        st[(size_t)l * G.nl + ll] = l < g.B ? best : __builtin_huge_valf();  // pad slot: +inf
                    }
                }
                // levels (same descriptor table, count table and cell function as kp_dp_kernel)
                for (int lam = 0; lam <= hp.lmax; ++lam) {
                    for (int qq = hp.loff[lam]; qq < hp.loff[lam + 1]; ++qq) {
                        const kp_lowdesc &D = hp.ldesc[qq];
                        kp_single_ctx sc;
                        sc.exact = !kp_fast_logs_ok(G.pen, G.nl, G.alpha, G.beta);
                        kp_ptab_counts<CT>(g, hp.lowmask.data(), ptab.data(), D.l, D.info, &sc.c.mtr, &sc.c.utr);
                        sc.c.mte = sc.c.ute = 0;
                        sc.kmer = (H == 0 && lam == 0);
                        sc.logp = sc.log1mp = 0.0;
                        if (!sc.kmer) {
                            double p = kp_rate(sc.c, G.alpha, G.beta);
                            sc.logp = log(p);
                            sc.log1mp = log(1.0 - p);
                        }
                        const uint4 *lp = reinterpret_cast<const uint4 *>(hp.lpairs.data()) + (D.pl >> 8);
                        cell_values(G.nl, D.l, D.pl & 0xFFu, lp, st.data(), sc, G.alpha, G.beta, G.pen);
                    }
                }
                // store
                for (int ll = 0; ll < G.nl; ++ll) {
                    uint64_t row = kp_lane_row(g, h, (uint32_t)G.lane0 + ll);
                    for (uint32_t l = 0; l < g.Bpad; ++l) S[row + l] = st[(size_t)l * G.nl + ll];
                }
            }
        }
    }
    // backtrack: decisions recomputed from the final scores (kp_cell_decide)
    for (int gi = 0; gi < ngroups; ++gi) {
        const kp_group_dev &G = groups[gi];
        for (int ll = 0; ll < G.nl; ++ll) {
            const uint32_t lane = (uint32_t)G.lane0 + ll;
            const double pen = G.pen[ll];
            auto score = [&](uint64_t y) { return S[kp_lane_row(g, y / g.B, lane) + y % g.B]; };
            uint32_t mism = 0;
            auto decide = [&](uint64_t x, uint64_t dig, kp_cnt *c) {
                *c = kp_cell_counts<CT>(g, hp.klofs.data(), hp.kllist.data(), K.data(), x, G.fold);
                float v;
                const uint32_t code = kp_cell_decide(g, hp.tabs.data(), x, dig, score, *c, G.alpha, G.beta, pen, &v);
                const float sv = score(x);
                if (memcmp(&sv, &v, 4) != 0 && !(sv != sv && v != v)) mism = 1;
                return code;
            };
            auto leaf = [&](uint64_t x, uint64_t dig, const kp_cnt &c) {
                (void)x;
                return kp_leaf_test_term(c, kp_dig_is_kmer(g, dig), G.fold, G.alpha, G.beta);
            };
            root_train[lane] = S[kp_lane_row(g, g.nblocks - 1, lane) + g.B - 1];
            uint64_t n = 0;
            uint32_t bad = 0;
            root_test[lane] = kp_backtrack_dfs(g, hp.tabs.data(), decide, leaf,
                                               leaves ? leaves + lane * hp.n_kmers : nullptr, hp.n_kmers, &n, &bad);
            nleaves[lane] = n;
            if (bad || mism) {
                g_err = bad ? "broken argmin tree" : "recomputed decision does not reproduce the stored score";
                return -5;
            }
            if (dump_code) {
                for (uint64_t x = 0; x < hp.npat; ++x) {
                    kp_cnt c;
                    dump_code[(uint64_t)lane * hp.npat + x] = (uint8_t)decide(x, kp_cell_digits(g, x), &c);
                }
                if (mism) {
                    g_err = "recomputed decision does not reproduce the stored score";
                    return -5;
                }
            }
        }
    }
    if (dump_score) {
        for (uint32_t lane = 0; lane < Ltot; ++lane)
            for (uint64_t h = 0; h < g.nblocks; ++h)
                for (uint32_t l = 0; l < g.B; ++l)
                    dump_score[(uint64_t)lane * hp.npat + h * g.B + l] = S[kp_lane_row(g, h, lane) + l];
    }
    return 0;
}
}  // namespace

extern "C" {
const char *emu_last_error(void) { return g_err.c_str(); }

// the C library restatement of kp_libm.h, host build: which = 0 log, 1 log1p
void emu_libm(const double *x, double *y, uint64_t n, int which) {
    for (uint64_t i = 0; i < n; ++i) y[i] = which ? kp_libm_log1p(x[i]) : kp_libm_log(x[i]);
}

// groups: device-group records (fold, lane0, nl, alpha, beta, pen[8]); M/U [n_kmers][nf]
int emu_run(const char *gp, uint32_t max_block, const void *M, const void *U, int nf, int itype_bytes,
            const kp_group_dev *groups, int ngroups, float *root_train, float *root_test, uint64_t *nleaves,
            float *dump_score, uint8_t *dump_code, uint64_t *leaves) {
    if (itype_bytes == 4)
        return emu<uint32_t>(gp, max_block, (const uint32_t *)M, (const uint32_t *)U, nf, groups, ngroups, root_train,
                             root_test, nleaves, dump_score, dump_code, leaves);
    return emu<uint64_t>(gp, max_block, (const uint64_t *)M, (const uint64_t *)U, nf, groups, ngroups, root_train,
                         root_test, nleaves, dump_score, dump_code, leaves);
}
}
