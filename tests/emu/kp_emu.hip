// kp_emu.hip -- host-side emulation of the blocked lattice DP (TEST INFRASTRUCTURE).
//
// Runs exactly the per-item functions of kmerpapa_amd/csrc/kp_core.h that the gfx950
// kernels run, serially on the CPU, with the same memory layout, block order and level
// order.  It lets tests/test_emu.py check the block decomposition, the tie combination
// and the argmin backtrack against the oracle without a GPU.  It is never loaded by the
// product package.
#include <stdint.h>
#include <string.h>

#include <string>
#include <vector>

#include "../../kmerpapa_amd/csrc/kp_core.h"
#include "../../kmerpapa_amd/csrc/kp_plan.h"

namespace {
std::string g_err;

void cell_lanes(int nl, const kp_geom &g, const uint64_t *tabs, uint32_t l, uint32_t info, float *st,
                const kp_single_ctx &sc, double a, double b, const double *pen, uint32_t *code) {
    switch (nl) {
        case 1: kp_dp_cell_lanes<1>(g, tabs, l, info, st, sc, a, b, pen, code); break;
        case 2: kp_dp_cell_lanes<2>(g, tabs, l, info, st, sc, a, b, pen, code); break;
        case 3: kp_dp_cell_lanes<3>(g, tabs, l, info, st, sc, a, b, pen, code); break;
        case 4: kp_dp_cell_lanes<4>(g, tabs, l, info, st, sc, a, b, pen, code); break;
        case 5: kp_dp_cell_lanes<5>(g, tabs, l, info, st, sc, a, b, pen, code); break;
        case 6: kp_dp_cell_lanes<6>(g, tabs, l, info, st, sc, a, b, pen, code); break;
        case 7: kp_dp_cell_lanes<7>(g, tabs, l, info, st, sc, a, b, pen, code); break;
        default: kp_dp_cell_lanes<8>(g, tabs, l, info, st, sc, a, b, pen, code); break;
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
    const uint64_t per = (uint64_t)g.n_kl * nf * 2;
    std::vector<CT> K(g.nblocks * per);
    // counts (kp_counts_kernel)
    for (int H = 0; H <= hp.hmax; ++H) {
        for (uint64_t q = hp.hoff[H]; q < hp.hoff[H + 1]; ++q) {
            uint64_t h = hp.hlist[q];
            CT *dst = K.data() + h * per;
            if (H == 0) {
                uint64_t kbase = 0;
                for (int i = 0; i < g.kh; ++i) kbase += (uint64_t)kp_high_digit(g, h, i) * g.khw[i];
                for (uint64_t e = 0; e < per / 2; ++e) {
                    uint64_t kl = e / nf, f = e % nf;
                    dst[2 * e] = M[(kbase + kl) * nf + f];
                    dst[2 * e + 1] = U[(kbase + kl) * nf + f];
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
                for (uint64_t e = 0; e < per; ++e) dst[e] = K[h1 * per + e] + K[h2 * per + e];
            }
        }
    }
    std::vector<float> S(g.nblocks * (uint64_t)Ltot * g.Bpad, 0.0f);
    std::vector<uint8_t> C(S.size(), 0);
    std::vector<kp_hpair> hpairs(KP_MAX_HPAIRS);
    std::vector<kp_cnt> kc(g.n_kl);
    std::vector<float> st;
    for (int H = 0; H <= hp.hmax; ++H) {
        for (uint64_t q = hp.hoff[H]; q < hp.hoff[H + 1]; ++q) {
            uint64_t h = hp.hlist[q];
            int np = kp_high_pairs(g, hp.tabs.data(), h, hpairs.data());
            for (int gi = 0; gi < ngroups; ++gi) {
                const kp_group_dev &G = groups[gi];
                st.assign((size_t)G.nl * g.Bpad, 0.0f);  // interleaved [cell][lane], like the kernel
                for (uint32_t kl = 0; kl < g.n_kl; ++kl) kc[kl] = kp_kl_counts<CT>(g, K.data(), h, kl, G.fold);
                // phase 1: gather (value -> st, code -> global C)
                for (int ll = 0; ll < G.nl; ++ll) {
                    uint32_t lane = (uint32_t)G.lane0 + ll;
                    for (uint32_t l = 0; l < g.Bpad; ++l) {
                        float best = __builtin_huge_valf();
                        uint32_t code = KP_NONE;
                        for (int p = 0; p < np; ++p) {
                            float v = S[kp_lane_row(g, hpairs[p].h1, lane) + l] + S[kp_lane_row(g, hpairs[p].h2, lane) + l];
                            if (v < best) { best = v; code = hpairs[p].code; }
                        }
                        st[(size_t)l * G.nl + ll] = best;
                        C[kp_lane_row(g, h, lane) + l] = (uint8_t)code;
                    }
                }
                // phase 2: levels (same descriptor table, count recurrence and cell function as kp_dp_kernel)
                std::vector<CT> cm(g.Bpad, 0), cu(g.Bpad, 0);
                for (uint32_t kl = 0; kl < g.n_kl; ++kl) {
                    cm[hp.kl2l[kl]] = (CT)kc[kl].mtr;
                    cu[hp.kl2l[kl]] = (CT)kc[kl].utr;
                }
                for (int lam = 0; lam <= hp.lmax; ++lam) {
                    for (int qq = hp.loff[lam]; qq < hp.loff[lam + 1]; ++qq) {
                        const kp_lowdesc &D = hp.ldesc[qq];
                        uint32_t l = D.l;
                        CT mt = lam == 0 ? cm[l] : (CT)(cm[D.l1] + cm[D.l2]);
                        CT ut = lam == 0 ? cu[l] : (CT)(cu[D.l1] + cu[D.l2]);
                        cm[l] = mt;
                        cu[l] = ut;
                        kp_single_ctx sc;
                        sc.kmer = (H == 0 && lam == 0);
                        sc.c.mtr = mt;
                        sc.c.utr = ut;
                        sc.c.mte = sc.c.ute = 0;
                        sc.logp = sc.log1mp = 0.0;
                        if (!sc.kmer) {
                            double p = kp_rate(sc.c, G.alpha, G.beta);
                            sc.logp = log(p);
                            sc.log1mp = log(1.0 - p);
                        }
                        uint32_t code[KP_GROUP_LANES];
                        cell_lanes(G.nl, g, hp.pw.data(), l, D.info, st.data(), sc, G.alpha, G.beta, G.pen, code);
                        for (int j = 0; j < G.nl; ++j)
                            if (code[j] != KP_NONE) C[kp_lane_row(g, h, (uint32_t)G.lane0 + j) + l] = (uint8_t)code[j];
                    }
                }
                // phase 3: store
                for (int ll = 0; ll < G.nl; ++ll) {
                    uint64_t row = kp_lane_row(g, h, (uint32_t)G.lane0 + ll);
                    for (uint32_t l = 0; l < g.Bpad; ++l) S[row + l] = st[(size_t)l * G.nl + ll];
                }
            }
        }
    }
    // backtrack
    for (int gi = 0; gi < ngroups; ++gi) {
        const kp_group_dev &G = groups[gi];
        for (int ll = 0; ll < G.nl; ++ll) {
            uint32_t lane = (uint32_t)G.lane0 + ll;
            root_train[lane] = S[kp_lane_row(g, g.nblocks - 1, lane) + g.B - 1];
            uint64_t n = 0;
            uint32_t bad = 0;
            auto leaf = [&](uint64_t x) {
                return kp_leaf_test<CT>(g, hp.tabs.data(), hp.lowinfo.data(), hp.klofs.data(), hp.kllist.data(),
                                        K.data(), x, G.fold, G.alpha, G.beta);
            };
            root_test[lane] = kp_backtrack_lane(g, hp.tabs.data(), C.data(), lane, leaf,
                                                leaves ? leaves + lane * hp.n_kmers : nullptr, hp.n_kmers, &n, &bad);
            nleaves[lane] = n;
            if (bad) {
                g_err = "broken argmin tree";
                return -5;
            }
        }
    }
    if (dump_score || dump_code) {
        for (uint32_t lane = 0; lane < Ltot; ++lane)
            for (uint64_t h = 0; h < g.nblocks; ++h)
                for (uint32_t l = 0; l < g.B; ++l) {
                    uint64_t src = kp_lane_row(g, h, lane) + l, dst = (uint64_t)lane * hp.npat + h * g.B + l;
                    if (dump_score) dump_score[dst] = S[src];
                    if (dump_code) dump_code[dst] = C[src];
                }
    }
    return 0;
}
}  // namespace

extern "C" {
const char *emu_last_error(void) { return g_err.c_str(); }

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
