// kp_plan.h -- host-side construction of the blocked lattice plan.
//
// Input: a general IUPAC pattern (e.g. "NNNNMNNNN").  Output: every table the kernels
// need (kp_core.h).  The IUPAC data restates src/kmerpapa/pattern_utils.py:5-100 of the
// reference (code, perm_code, complements); the digit of a sub-code is its index in
// perm_code[g] and the cell index is mixed radix with position 0 least significant
// (PatternEnumeration, pattern_utils.py:247-266).
#pragma once
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <string>
#include <vector>

#include "kp_core.h"

namespace kp {

static const char *const kIupac = "ACGTRYSWKMBDHVN";
static const char *const kNuc[15] = {"A", "C", "G", "T", "AG", "CT", "GC", "AT", "GT", "AC",
                                     "CGT", "AGT", "ACT", "ACG", "ACGT"};
static const char *const kPerm[15] = {"A", "C", "G", "T", "AGR", "CTY", "GCS", "ATW", "GTK", "ACM",
                                      "CGTSYKB", "AGTRWKD", "ACTMWYH", "ACGMRSV", "ACGTRYSWKMBDHVN"};
// split pairs, two letters per pair, in scan order
static const char *const kSplit[15] = {"", "", "", "", "AG", "CT", "GC", "AT", "GT", "AC",
                                       "CKGYTS", "AKGWTR", "AYCWTM", "ASCRGM", "SWKMRYABCDGHTV"};

inline int iupac_index(char c) {
    if (!c) return -1;
    const char *p = strchr(kIupac, c);
    return p ? (int)(p - kIupac) : -1;
}

struct host_plan {
    std::string gp;
    kp_geom g;
    uint64_t npat = 0;
    int maxlev = 0, hmax = 0, lmax = 0;
    uint64_t n_kmers = 0;
    std::vector<kp_postab> tabs;       // [k]
    std::vector<uint64_t> pw;          // [t][16] pair words of the low positions (kp_pair_word)
    std::vector<uint8_t> lowmask;      // [t][16] nucleotide-index bit mask of each low digit
    uint32_t ptab_entries = 0;         // separable count table: cgl[t-1] low prefixes x n[t-1]
    uint32_t pscratch_entries = 0;     // largest intermediate table of its build
    std::vector<uint32_t> lowinfo;     // [B] packed low digits
    std::vector<uint16_t> lorder;      // [B] low cells sorted by low level
    std::vector<int32_t> loff;         // [lmax + 2]
    std::vector<kp_lowdesc> ldesc;     // [B] low cells in level order
    std::vector<uint32_t> lpairs;      // low split pairs of every cell, in 4-pair chunks (kp_lowdesc.pl)
    uint32_t max_low_pairs = 0;        // most low split pairs of one cell
    std::vector<uint16_t> kl2l;        // [n_kl] k-mer-low index -> low cell
    std::vector<uint32_t> klofs;       // [B + 1]
    std::vector<uint16_t> kllist;      // k-mer-low cells matching each low cell
    std::vector<uint32_t> hlist;       // [nblocks] blocks sorted by high level
    std::vector<uint32_t> kpos;        // [nblocks] block -> its position in hlist (its count row)
    std::vector<uint64_t> hdig;        // [nblocks] their high digits, 4 bits per high position
    std::vector<uint64_t> hnp;         // [nblocks] their split pairs per high position, 3 bits each
    std::vector<uint64_t> hoff;        // [hmax + 2]
    std::vector<int> perm;             // high positions of the block order, fastest first
    int hs = 0;                        // high level sums 0 .. hs - 1
    std::vector<uint32_t> brank;       // [kh][16][hs] rank table of the block order (build_plan)
    bool blocks_on_host = true;        // hlist / kpos / hdig / hnp built here
    uint32_t kh_nuc_weight = 0;
    // algorithmic accounting: split pairs summed over all cells
    double pairs_total = 0.0, pairs_low = 0.0, pairs_high = 0.0;
};

// Build the plan.  max_block bounds the LDS block (cells); returns "" or an error text.
// block_tables = false leaves hlist / kpos / hdig / hnp to the device (kp_blocks_kernel,
// from perm, brank and hoff) unless an experiment block order is set (blocks_on_host).
inline std::string build_plan(const char *gen_pat, uint32_t max_block, host_plan &P, bool block_tables = true) {
    P = host_plan();
    P.gp = gen_pat ? gen_pat : "";
    int k = (int)P.gp.size();
    if (k <= 0 || k > KP_MAXK) return "general pattern length must be 1.." + std::to_string(KP_MAXK);
    kp_geom &g = P.g;
    memset(&g, 0, sizeof(g));
    g.k = k;
    P.tabs.resize(k);
    memset(P.tabs.data(), 0, sizeof(kp_postab) * k);
    uint64_t acc = 1, kacc = 1;
    std::vector<uint64_t> kw(k);
    for (int i = 0; i < k; ++i) {
        int gi = iupac_index(P.gp[i]);
        if (gi < 0) return std::string("not an IUPAC code: ") + P.gp[i];
        const char *perm = kPerm[gi];
        int r = (int)strlen(perm);
        g.r[i] = (uint32_t)r;
        g.n[i] = (uint32_t)strlen(kNuc[gi]);
        g.cgl[i] = acc;
        kw[i] = kacc;
        if (acc > (~0ULL) / (uint64_t)r) return "lattice too large";
        acc *= (uint64_t)r;
        kacc *= g.n[i];
        P.maxlev += (int)g.n[i] - 1;
        for (int d = 0; d < r; ++d) {
            int x = iupac_index(perm[d]);
            P.tabs[i].lev[d] = (uint8_t)(strlen(kNuc[x]) - 1);
            const char *sp = kSplit[x];
            int np = (int)strlen(sp) / 2;
            P.tabs[i].np[d] = (uint8_t)np;
            for (int j = 0; j < np; ++j) {
                P.tabs[i].pa[d][j] = (uint8_t)(strchr(perm, sp[2 * j]) - perm);
                P.tabs[i].pb[d][j] = (uint8_t)(strchr(perm, sp[2 * j + 1]) - perm);
            }
        }
    }
    P.npat = acc;
    P.n_kmers = kacc;
    // low positions: as many as fit the block budget
    int t = 0;
    while (t < k && t < KP_MAXT && g.cgl[t] * g.r[t] <= (uint64_t)max_block) ++t;
    if (t == 0) t = 1;  // a single position always fits (radix <= 15)
    g.t = t;
    g.kh = k - t;
    g.B = (uint32_t)(t < k ? g.cgl[t] : acc);
    {
        // row length of one block lane: >= B + 1 (slot B is the +inf cell of padded pair
        // lists), a multiple of 32 floats so that every lane row starts on a 128-byte cache
        // line (rows [h][lane] are back to back).  At 16 floats (64 B) half the rows of a
        // 5-lane pass started mid-line: 9-mer pass 375 -> 366 ms at 32
        // (profiles/r05/experiments/bpad_align.txt).  KP_BPAD_ALIGN=16/64/.. for experiments.
        const char *e = getenv("KP_BPAD_ALIGN");
        uint32_t al = e ? (uint32_t)atoi(e) : 32u;
        if (al < 16u || (al & (al - 1u))) al = 32u;
        g.Bpad = (g.B + al) & ~(al - 1u);
    }
    g.nblocks = acc / g.B;
    uint32_t nkl = 1;
    for (int i = 0; i < t; ++i) nkl *= g.n[i];
    g.n_kl = nkl;
    for (int i = 0; i < g.kh; ++i) {
        g.hcg[i] = g.cgl[t + i] / g.B;
        g.khw[i] = kw[t + i];
    }
    P.pw.assign((size_t)t * 16, 0);
    for (int i = 0; i < t; ++i)
        for (uint32_t d = 0; d < g.r[i]; ++d) P.pw[i * 16 + d] = kp_pair_word(P.tabs[i], d);
    // nucleotide masks: nucleotide c of general code G has k-mer digit = index of c in code[G]
    P.lowmask.assign((size_t)t * 16, 0);
    for (int i = 0; i < t; ++i) {
        const int gi = iupac_index(P.gp[i]);
        for (uint32_t d = 0; d < g.r[i]; ++d) {
            const char *nucs = kNuc[iupac_index(kPerm[gi][d])];
            uint8_t m = 0;
            for (const char *c = nucs; *c; ++c) m |= (uint8_t)(1u << (strchr(kNuc[gi], *c) - kNuc[gi]));
            P.lowmask[i * 16 + d] = m;
        }
    }
    // separable count tables T_s (kp_dp_kernel): digits of positions < s, nucleotides >= s
    {
        uint64_t R = 1, mx = 1;
        for (int s = 0; s < t; ++s) {
            uint64_t nn = 1;
            for (int i = s; i < t; ++i) nn *= g.n[i];
            mx = std::max<uint64_t>(mx, R * nn);
            if (s < t - 1) R *= g.r[s];
        }
        P.ptab_entries = (uint32_t)(R * g.n[t - 1]);
        P.pscratch_entries = (uint32_t)mx;
    }
    // low cells: digits, levels, order, matching k-mer-low cells
    uint32_t B = g.B;
    if (B > 0xFFFFu) return "block too large for 16-bit cell ids";
    P.lowinfo.resize(B);
    std::vector<int> llev(B);
    int lmax = 0;
    for (int i = 0; i < t; ++i) lmax += (int)g.n[i] - 1;
    P.lmax = lmax;
    P.loff.assign(lmax + 2, 0);
    for (uint32_t l = 0; l < B; ++l) {
        uint32_t q = l, info = 0;
        int s = 0;
        for (int i = 0; i < t; ++i) {
            uint32_t d = q % g.r[i];
            q /= g.r[i];
            info |= d << (4 * i);
            s += P.tabs[i].lev[d];
        }
        P.lowinfo[l] = info;
        llev[l] = s;
        P.loff[s + 1]++;
    }
    for (int s = 0; s <= lmax; ++s) P.loff[s + 1] += P.loff[s];
    P.lorder.resize(B);
    {
        // inside a level any order is valid (cells only read lower levels); cells are
        // sorted by their number of low split pairs, then by split signature, so that the
        // 64 cells of a wave run (nearly) the same number of pair chunks in the level phase
        std::vector<uint32_t> npairs(B);
        std::vector<uint64_t> sigs(B);
        for (uint32_t l = 0; l < B; ++l) {
            uint64_t sig = 0;
            uint32_t np = 0;
            for (int i = 0; i < t; ++i) {
                const uint32_t n = P.tabs[i].np[kp_low_digit(P.lowinfo[l], i)];
                sig = sig * 8 + n;
                np += n;
            }
            sigs[l] = sig;
            npairs[l] = np;
        }
        // KP_LOW_ORDER=1 (experiment): inside a pair-count class, cells with the same digits
        // at every ambiguous low position next to each other, so a wave's split children sit
        // at the same offsets from consecutive-ish cells (fewer LDS bank conflicts)
        const char *lo = getenv("KP_LOW_ORDER");
        const bool bydig = lo && atoi(lo) == 1;
        std::vector<uint32_t> amb(B, 0);  // digits at ambiguous positions, nucleotides zeroed
        for (uint32_t l = 0; l < B; ++l)
            for (int i = 0; i < t; ++i) {
                const uint32_t d = kp_low_digit(P.lowinfo[l], i);
                if (P.tabs[i].np[d]) amb[l] |= d << (4 * i);
            }
        std::vector<uint32_t> idx(B);
        for (uint32_t l = 0; l < B; ++l) idx[l] = l;
        std::sort(idx.begin(), idx.end(), [&](uint32_t a, uint32_t b) {
            if (llev[a] != llev[b]) return llev[a] < llev[b];
            if (npairs[a] != npairs[b]) return npairs[a] < npairs[b];
            if (sigs[a] != sigs[b]) return sigs[a] < sigs[b];
            if (bydig && amb[a] != amb[b]) return amb[a] < amb[b];
            return a < b;
        });
        for (uint32_t q = 0; q < B; ++q) P.lorder[q] = (uint16_t)idx[q];
    }
    // level-ordered descriptors: cell, k-mer-low index, digits, split-pair list
    P.ldesc.resize(B);
    P.kl2l.assign(nkl, 0);
    for (uint32_t q = 0; q < B; ++q) {
        uint32_t l = P.lorder[q];
        kp_lowdesc D;
        memset(&D, 0, sizeof(D));
        D.l = l;
        D.info = P.lowinfo[l];
        if (llev[l] == 0) {
            uint32_t kl = 0, w = 1;
            for (int i = 0; i < t; ++i) {
                kl += kp_low_digit(D.info, i) * w;
                w *= g.n[i];
            }
            D.kl = (uint16_t)kl;
            P.kl2l[kl] = (uint16_t)l;
        }
        // the cell's low split pairs as child-cell pairs (c1 | c2 << 16), position by
        // position in scan order, padded to whole 4-pair chunks with (B, B): slot B of the
        // block holds +inf in every lane, so padding never wins a min
        const uint32_t first = (uint32_t)P.lpairs.size();
        uint32_t np = 0;
        for (int i = 0; i < t; ++i) {
            const uint32_t d = kp_low_digit(D.info, i);
            for (uint32_t p = 0; p < P.tabs[i].np[d]; ++p) {
                const uint32_t c1 = l - (d - P.tabs[i].pa[d][p]) * (uint32_t)g.cgl[i];
                const uint32_t c2 = l - (d - P.tabs[i].pb[d][p]) * (uint32_t)g.cgl[i];
                P.lpairs.push_back(c1 | (c2 << 16));
                ++np;
            }
        }
        while (P.lpairs.size() & 3u) P.lpairs.push_back(B | (B << 16));
        if (np > 255 || (first >> 2) > 0xFFFFFFu) return "too many low split pairs";
        D.pl = ((first >> 2) << 8) | np;
        P.max_low_pairs = std::max(P.max_low_pairs, np);
        P.ldesc[q] = D;
    }
    // nucleotide index sets of every (position, digit): nucleotide c of code x has
    // k-mer digit = index of c in code[g] = perm digit of c (nucleotides come first)
    P.klofs.assign(B + 1, 0);
    for (uint32_t l = 0; l < B; ++l) {
        // enumerate the product of nucleotide sets of the low digits
        std::vector<uint32_t> cur(1, 0);
        uint32_t w = 1;
        for (int i = 0; i < t; ++i) {
            uint32_t d = kp_low_digit(P.lowinfo[l], i);
            int gi = iupac_index(P.gp[i]);
            const char *perm = kPerm[gi];
            const char *nucs = kNuc[iupac_index(perm[d])];
            std::vector<uint32_t> nxt;
            for (uint32_t base : cur)
                for (const char *c = nucs; *c; ++c) nxt.push_back(base + (uint32_t)(strchr(perm, *c) - perm) * w);
            cur.swap(nxt);
            w *= g.n[i];
        }
        for (uint32_t v : cur) P.kllist.push_back((uint16_t)v);
        P.klofs[l + 1] = (uint32_t)P.kllist.size();
    }
    // blocks by high level
    int hmax = 0;
    for (int i = t; i < k; ++i) hmax += (int)g.n[i] - 1;
    P.hmax = hmax;
    P.hoff.assign(hmax + 2, 0);
    if (g.nblocks > 0xFFFFFFFFull) return "too many blocks for 32-bit block ids";
    if (g.kh > 15) return "too many high positions for packed digits";
    // Block order inside a level = the order the sweep kernel runs them in, which sets how
    // often a child row read by several parents is still in L2 / the Infinity Cache.
    // Parents of one child differ in one high position, so the positions that vary fastest
    // get their reuse: those with the most split pairs (largest radix) go first, later
    // positions before earlier ones (measured: random order +25 % time, ascending h
    // (position t fastest) +1 %, this order the best of those tried).
    // KP_BLOCK_PERM="5-4-..." (high positions, fastest first) and KP_BLOCK_ORDER=1
    // (shuffled) / KP_BLOCK_TILE=T override it for experiments.
    std::vector<int> perm;
    if (const char *pe = getenv("KP_BLOCK_PERM")) {  // digits separated by any non-digit
        for (const char *c = pe; *c;) {
            const int v = atoi(c);
            if (v >= 0 && v < g.kh && std::find(perm.begin(), perm.end(), v) == perm.end()) perm.push_back(v);
            while (*c >= '0' && *c <= '9') ++c;
            while (*c && (*c < '0' || *c > '9')) ++c;
        }
    } else {
        for (int i = g.kh - 1; i >= 0; --i) perm.push_back(i);
        std::stable_sort(perm.begin(), perm.end(), [&](int a, int b) { return g.r[g.t + a] > g.r[g.t + b]; });
    }
    for (int i = g.kh - 1; i >= 0; --i)  // complete a partial explicit permutation
        if (std::find(perm.begin(), perm.end(), i) == perm.end()) perm.push_back(i);
    P.perm = perm;
    // Rank tables: the blocks are numbered by a mixed-radix counter, perm[0] fastest; block
    // n goes to hoff[s] + (the number of blocks before n with the same high level s).  With
    // C_j(x) = the digit tuples of positions perm[0..j) whose levels sum to x, that count is
    // the sum over j of brank[j][digit at perm[j]][s - levels of the positions above j],
    // brank[j][d][y] = sum over d' < d of C_j(y - lev(d')) -- a closed form, so the device
    // builds the block list itself (kp_blocks_kernel) and the host never walks the blocks.
    const int HS = hmax + 1;
    P.hs = HS;
    {
        std::vector<uint64_t> C((size_t)(g.kh + 1) * HS, 0);
        C[0] = 1;
        P.brank.assign((size_t)g.kh * 16 * HS, 0);
        for (int j = 0; j < g.kh; ++j) {
            const kp_postab &T = P.tabs[g.t + perm[j]];
            const uint32_t r = g.r[g.t + perm[j]];
            for (uint32_t d = 0; d < r; ++d)
                for (int y = 0; y < HS; ++y) {
                    const uint64_t c = y >= T.lev[d] ? C[(size_t)j * HS + y - T.lev[d]] : 0;
                    if (d + 1 < 16) P.brank[((size_t)j * 16 + d + 1) * HS + y] = P.brank[((size_t)j * 16 + d) * HS + y] + (uint32_t)c;
                    C[(size_t)(j + 1) * HS + y] += c;
                }
        }
        for (int s = 0; s <= hmax; ++s) P.hoff[s + 1] = P.hoff[s] + C[(size_t)g.kh * HS + s];
        if (P.hoff[hmax + 1] != g.nblocks) return "block level counts do not cover every block";
    }
    const char *te = getenv("KP_BLOCK_TILE");
    const uint32_t tile = te ? (uint32_t)atoi(te) : 0u;
    const char *bo = getenv("KP_BLOCK_ORDER");
    const bool shuffled = bo && atoi(bo) == 1;
    P.blocks_on_host = block_tables || tile > 0 || shuffled;
    if (P.blocks_on_host) {
        // high levels of every block: a mixed-radix counter over h (high position 0 fastest)
        // keeps the digits and their level sum, no 64-bit divisions
        std::vector<uint8_t> hl(g.nblocks);
        {
            std::vector<uint32_t> dig(g.kh, 0);
            int s = 0;
            for (uint64_t h = 0; h < g.nblocks; ++h) {
                hl[h] = (uint8_t)s;
                for (int i = 0; i < g.kh; ++i) {
                    const kp_postab &T = P.tabs[g.t + i];
                    s -= T.lev[dig[i]];
                    if (++dig[i] < g.r[g.t + i]) {
                        s += T.lev[dig[i]];
                        break;
                    }
                    dig[i] = 0;
                    s += T.lev[0];
                }
            }
        }
        P.hlist.resize(g.nblocks);
        {
            std::vector<uint64_t> fill(P.hoff.begin(), P.hoff.end() - 1);
            // KP_BLOCK_TILE=T (experiment): tiles of T digits per high position, the digits
            // inside a tile (perm order) varying faster than the tile coordinates
            if (tile > 0) {
                std::vector<uint32_t> tr(g.kh), to(g.kh, 0), ti(g.kh, 0);
                for (int i = 0; i < g.kh; ++i) tr[i] = (g.r[g.t + i] + tile - 1) / tile;
                for (;;) {
                    std::fill(ti.begin(), ti.end(), 0u);
                    for (;;) {
                        bool ok = true;
                        uint64_t h = 0;
                        for (int i = 0; i < g.kh; ++i) {
                            const uint32_t d = to[i] * tile + ti[i];
                            if (d >= g.r[g.t + i]) { ok = false; break; }
                            h += (uint64_t)d * g.hcg[i];
                        }
                        if (ok) P.hlist[fill[hl[h]]++] = (uint32_t)h;
                        int j = 0;
                        for (; j < g.kh; ++j) {
                            const int i = perm[j];
                            if (++ti[i] < tile) break;
                            ti[i] = 0;
                        }
                        if (j == g.kh) break;
                    }
                    int j = 0;
                    for (; j < g.kh; ++j) {
                        const int i = perm[j];
                        if (++to[i] < tr[i]) break;
                        to[i] = 0;
                    }
                    if (j == g.kh) break;
                }
            } else {
                // mixed-radix counter, perm[0] fastest; the packed digits come along
                P.hdig.resize(g.nblocks);
                std::vector<uint32_t> dig(g.kh, 0);
                uint64_t h = 0, w = 0;
                for (uint64_t n = 0; n < g.nblocks; ++n) {
                    const uint64_t q = fill[hl[h]]++;
                    P.hlist[q] = (uint32_t)h;
                    P.hdig[q] = w;
                    for (int j = 0; j < g.kh; ++j) {
                        const int i = perm[j];
                        if (++dig[i] < g.r[g.t + i]) {
                            h += g.hcg[i];
                            w += 1ull << (4 * i);
                            break;
                        }
                        h -= (uint64_t)(dig[i] - 1) * g.hcg[i];
                        w &= ~(15ull << (4 * i));
                        dig[i] = 0;
                    }
                }
            }
            for (int s = 0; s <= hmax; ++s)
                if (fill[s] != P.hoff[s + 1]) return "block order does not cover every block";
            if (shuffled) P.hdig.clear();  // recomputed below for the shuffled list
            if (shuffled)
                for (int s = 0; s <= hmax; ++s) {  // experiment: shuffled (no reuse order)
                    uint32_t *b = P.hlist.data() + P.hoff[s], *e = P.hlist.data() + P.hoff[s + 1];
                    uint64_t x = 0x9E3779B97F4A7C15ull + (uint64_t)s;
                    for (uint32_t *q = e; q - b > 1; --q) {
                        x ^= x << 13; x ^= x >> 7; x ^= x << 17;
                        std::swap(q[-1], b[x % (uint64_t)(q - b)]);
                    }
                }
        }
        if (P.hdig.size() != g.nblocks) {  // experiment orders (tiled, shuffled)
            P.hdig.resize(g.nblocks);
            for (uint64_t q = 0; q < g.nblocks; ++q) {
                uint64_t h = P.hlist[q], w = 0;
                for (int i = 0; i < g.kh; ++i) w |= (uint64_t)kp_high_digit(g, h, i) << (4 * i);
                P.hdig[q] = w;
            }
        }
        P.kpos.resize(g.nblocks);
        for (uint64_t q = 0; q < g.nblocks; ++q) P.kpos[P.hlist[q]] = (uint32_t)q;
        P.hnp.resize(g.nblocks);
        for (uint64_t q = 0; q < g.nblocks; ++q) {
            uint64_t n = 0;
            for (int i = 0; i < g.kh; ++i) n |= (uint64_t)P.tabs[t + i].np[(P.hdig[q] >> (4 * i)) & 15u] << (3 * i);
            P.hnp[q] = n;
        }
    }  // blocks_on_host
    // split pairs per position: sum over digits of np, times the other radices
    for (int i = 0; i < k; ++i) {
        double sum = 0;
        for (uint32_t d = 0; d < g.r[i]; ++d) sum += P.tabs[i].np[d];
        double cnt = sum * (double)(P.npat / g.r[i]);
        P.pairs_total += cnt;
        if (i < t) P.pairs_low += cnt; else P.pairs_high += cnt;
    }
    return "";
}

}  // namespace kp
