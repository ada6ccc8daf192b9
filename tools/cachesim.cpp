// cachesim.cpp -- row-granular cache model of one DP pass of the blocked sweep (tool, not
// product).  Replays the child-row reads and score-row writes of every block of every
// launch, in the order the GPU would run them under a given schedule, through an LRU L2 per
// XCD and one shared LRU Infinity Cache (MALL), and reports L2 misses (what rocprofv3
// FETCH_SIZE counts) and MALL misses (HBM reads).
//
// Concurrency model: workgroups are dealt round-robin to 8 XCDs by dispatch index; each XCD
// runs its blocks in order; the replay interleaves the XCDs block by block (every XCD
// progresses at the same rate).  Reuse among the ~64 workgroups co-resident on an XCD is
// approximated by LRU over the XCD's access sequence.
//
// build: hipcc -O2 -std=c++17 -o tools/cachesim tools/cachesim.cpp   (host code only)
// usage: tools/cachesim GEN_PAT LANES SCHEDULE [param]
//   SCHEDULE: plan      = the plan's block list, runs of `param` (default 8) per XCD
//             square    = fibers over the two fastest high positions kept on one XCD
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <list>
#include <set>
#include <string>
#include <unordered_map>
#include <vector>

#include "../kmerpapa_amd/csrc/kp_plan.h"

struct LRU {
    size_t cap;
    std::list<uint64_t> order;
    std::unordered_map<uint64_t, std::list<uint64_t>::iterator> pos;
    explicit LRU(size_t c) : cap(c) {}
    bool peek(uint64_t key) const { return pos.count(key) > 0; }
    bool touch(uint64_t key) {  // true = hit
        auto it = pos.find(key);
        if (it != pos.end()) {
            order.splice(order.begin(), order, it->second);
            return true;
        }
        order.push_front(key);
        pos[key] = order.begin();
        if (order.size() > cap) {
            pos.erase(order.back());
            order.pop_back();
        }
        return false;
    }
};

int main(int argc, char **argv) {
    if (argc < 4) {
        fprintf(stderr, "usage: %s GEN_PAT LANES SCHEDULE [param] [l2_rows] [mall_rows]\n", argv[0]);
        return 2;
    }
    kp::host_plan P;
    std::string err = kp::build_plan(argv[1], 4096, P);
    if (!err.empty()) {
        fprintf(stderr, "%s\n", err.c_str());
        return 1;
    }
    const int lanes = atoi(argv[2]);
    const std::string sched = argv[3];
    const int param = argc > 4 ? atoi(argv[4]) : 8;
    const kp_geom &g = P.g;
    const double row_bytes = (double)lanes * g.Bpad * 4;
    const size_t l2_rows = argc > 5 ? (size_t)atol(argv[5]) : (size_t)(4.0 * 1048576 / row_bytes);
    const size_t mall_rows = argc > 6 ? (size_t)atol(argv[6]) : (size_t)(256.0 * 1048576 / row_bytes);
    std::vector<LRU> l2(8, LRU(l2_rows));
    // KP_NT_POS="a,b,..." = high positions (0-based among high positions) read non-temporally
    std::set<int> slow_nt;
    if (const char *e = getenv("KP_NT_POS"))
        for (const char *c = e; *c;) {
            slow_nt.insert(atoi(c));
            while (*c >= '0' && *c <= '9') ++c;
            while (*c && (*c < '0' || *c > '9')) ++c;
        }
    LRU mall(mall_rows);
    uint64_t reads = 0, l2miss = 0, mallmiss = 0, writes = 0, distinct = 0;
    for (int H = 0; H <= P.hmax; ++H) {
        const uint64_t b0 = P.hoff[H], nb = P.hoff[H + 1] - b0;
        // dispatch order -> list entry
        std::vector<uint64_t> disp(nb);
        if (sched == "plan") {
            const uint64_t G = (uint64_t)std::max(param, 1), full = nb / (8 * G) * (8 * G);
            for (uint64_t b = 0; b < nb; ++b) {
                uint64_t w = b;
                if (G > 1 && b < full) {
                    const uint64_t x = b & 7u, sl = b >> 3;
                    w = ((sl / G) * 8 + x) * G + sl % G;
                }
                disp[b] = w;
            }
        }
        // per-XCD sequences
        std::vector<std::vector<uint64_t>> xs(8);
        if (sched == "plan") {
            for (uint64_t b = 0; b < nb; ++b) xs[b & 7u].push_back(P.hlist[b0 + disp[b]]);
        } else if (sched == "tile") {
            // tiles = blocks of the launch sharing every high digit except those of the
            // `param` fastest positions of the plan order (positions kh-1, kh-2, ...): a
            // tile's blocks run back to back on one XCD; tiles in list order go to the
            // least-loaded XCD
            const int q = param;
            std::vector<uint64_t> key(nb);
            std::unordered_map<uint64_t, std::vector<uint64_t>> tiles;
            std::vector<uint64_t> korder;
            for (uint64_t e = 0; e < nb; ++e) {
                const uint64_t h = P.hlist[b0 + e];
                uint64_t kk = h;
                for (int j = 0; j < q; ++j) {
                    const int i = g.kh - 1 - j;
                    kk -= (uint64_t)kp_high_digit(g, h, i) * g.hcg[i];
                }
                auto it = tiles.find(kk);
                if (it == tiles.end()) {
                    korder.push_back(kk);
                    tiles[kk] = {h};
                } else
                    it->second.push_back(h);
            }
            std::vector<uint64_t> load(8, 0);
            for (uint64_t kk : korder) {
                int x = 0;
                for (int y = 1; y < 8; ++y)
                    if (load[y] < load[x]) x = y;
                for (uint64_t h : tiles[kk]) xs[x].push_back(h);
                load[x] += tiles[kk].size();
            }
        } else if (sched == "childmajor") {
            // parents emitted child by child: children (blocks of lower level) in list
            // order, each child's not-yet-emitted parents of this launch, dealt in runs of
            // `param` to the XCDs round-robin
            std::vector<uint8_t> done(g.nblocks, 0);
            std::vector<uint8_t> inl(g.nblocks, 0);
            for (uint64_t e = 0; e < nb; ++e) inl[P.hlist[b0 + e]] = 1;
            std::vector<uint64_t> seq;
            seq.reserve(nb);
            const uint64_t c0 = P.hoff[std::max(0, H - 3)], c1 = P.hoff[H];
            // parents of child c along high position i: digits e with a split containing c_i
            for (uint64_t ce = c0; ce < c1; ++ce) {
                const uint64_t c = P.hlist[ce];
                for (int i = 0; i < g.kh; ++i) {
                    const kp_postab &T = P.tabs[g.t + i];
                    const uint32_t a = kp_high_digit(g, c, i);
                    for (uint32_t e = 0; e < g.r[g.t + i]; ++e)
                        for (int j = 0; j < T.np[e]; ++j)
                            if (T.pa[e][j] == a || T.pb[e][j] == a) {
                                const uint64_t h = c + ((uint64_t)e - a) * g.hcg[i];
                                if (inl[h] && !done[h]) {
                                    done[h] = 1;
                                    seq.push_back(h);
                                }
                            }
                }
            }
            for (uint64_t e = 0; e < nb; ++e)
                if (!done[P.hlist[b0 + e]]) seq.push_back(P.hlist[b0 + e]);
            const uint64_t G = (uint64_t)std::max(param, 1);
            for (uint64_t q = 0; q < seq.size(); ++q) xs[(q / G) & 7u].push_back(seq[q]);
        } else if (sched == "morton") {
            // blocks sorted by the bit-interleaved (Z-order) key of their high digits
            // (digit order = KP_DIGIT_ORDER permutation of 0..14 if given)
            std::vector<int> dord(16);
            for (int d = 0; d < 16; ++d) dord[d] = d;
            if (const char *e = getenv("KP_DIGIT_ORDER")) {
                int q = 0;
                for (const char *c = e; *c && q < 15;) {
                    dord[atoi(c)] = q++;
                    while (*c >= '0' && *c <= '9') ++c;
                    while (*c && (*c < '0' || *c > '9')) ++c;
                }
            }
            std::vector<std::pair<uint64_t, uint64_t>> kv(nb);
            for (uint64_t e = 0; e < nb; ++e) {
                const uint64_t h = P.hlist[b0 + e];
                uint64_t key = 0;
                for (int bit = 3; bit >= 0; --bit)
                    for (int i = g.kh - 1; i >= 0; --i) {
                        const uint32_t d = g.r[g.t + i] == 15 ? (uint32_t)dord[kp_high_digit(g, h, i)] : kp_high_digit(g, h, i);
                        key = (key << 1) | ((d >> bit) & 1u);
                    }
                kv[e] = {key, h};
            }
            std::sort(kv.begin(), kv.end());
            const uint64_t G = (uint64_t)std::max(param, 1);
            for (uint64_t q = 0; q < nb; ++q) xs[(q / G) & 7u].push_back(kv[q].second);
        } else if (sched == "chunk3") {
            // plan order (perm fastest-first: kh-1, kh-2, ...), but the third-fastest
            // position is cut into chunks of `param` digits, the chunk coordinate varying
            // just slower than the third position's loop... i.e. key =
            // (slow positions, chunk(p3), p3, p2, p1)
            std::vector<std::pair<std::vector<uint32_t>, uint64_t>> kv(nb);
            const int p1 = g.kh - 1, p2 = g.kh - 2, p3 = g.kh - 3;
            for (uint64_t e = 0; e < nb; ++e) {
                const uint64_t h = P.hlist[b0 + e];
                std::vector<uint32_t> key;
                for (int i = 0; i < g.kh; ++i)
                    if (i != p1 && i != p2 && i != p3) key.push_back(kp_high_digit(g, h, i));
                std::reverse(key.begin(), key.end());  // earlier positions slower? keep plan: M slowest
                const uint32_t d3 = kp_high_digit(g, h, p3);
                key.push_back(d3 / (uint32_t)param);
                key.push_back(d3);
                key.push_back(kp_high_digit(g, h, p2));
                key.push_back(kp_high_digit(g, h, p1));
                kv[e] = {key, h};
            }
            std::stable_sort(kv.begin(), kv.end(), [](const auto &a, const auto &b) { return a.first < b.first; });
            const uint64_t G = 8;
            for (uint64_t q = 0; q < nb; ++q) xs[(q / G) & 7u].push_back(kv[q].second);
        } else if (sched == "keyed") {
            // blocks sorted by a key built from KP_SIM_KEY = comma list, slowest first, of
            // high positions "i" (the digit) or "ci:T" (the digit's chunk, digit / T); then
            // dealt in runs of `param` to the XCDs
            std::vector<std::pair<int, int>> spec;  // (position, chunk size or 0; -1 = snake)
            const char *e = getenv("KP_SIM_KEY");
            for (const char *c = e ? e : ""; *c;) {
                int chunk = 0;
                if (*c == 's') {  // "si": digit order reversed when the slower key is odd
                    chunk = -1;
                    ++c;
                }
                if (*c == 'c') ++c;
                const int pos = atoi(c);
                while (*c >= '0' && *c <= '9') ++c;
                if (*c == ':') {
                    ++c;
                    chunk = atoi(c);
                    while (*c >= '0' && *c <= '9') ++c;
                }
                spec.push_back({pos, chunk});
                while (*c == ',') ++c;
            }
            std::vector<std::pair<uint64_t, uint64_t>> kv(nb);
            for (uint64_t e2 = 0; e2 < nb; ++e2) {
                const uint64_t h = P.hlist[b0 + e2];
                uint64_t key = 0;
                uint64_t par = 0;
                for (auto &sp : spec) {
                    uint32_t d = kp_high_digit(g, h, sp.first);
                    if (sp.second < 0) {
                        if (par & 1u) d = g.r[g.t + sp.first] - 1 - d;
                    } else if (sp.second > 0)
                        d /= (uint32_t)sp.second;
                    key = key * 16 + d;
                    par += d;
                }
                kv[e2] = {key, h};
            }
            std::stable_sort(kv.begin(), kv.end(), [](const auto &a2, const auto &b2) { return a2.first < b2.first; });
            const uint64_t G = (uint64_t)std::max(param, 1);
            for (uint64_t q = 0; q < nb; ++q) xs[(q / G) & 7u].push_back(kv[q].second);
        } else {
            fprintf(stderr, "unknown schedule\n");
            return 2;
        }
        {  // lower bound: distinct children of the launch
            std::unordered_map<uint64_t, int> ch;
            kp_hpair hq[KP_MAX_HPAIRS];
            for (uint64_t e = 0; e < nb; ++e) {
                const int np = kp_high_pairs(g, P.tabs.data(), P.hlist[b0 + e], hq);
                for (int p = 0; p < np; ++p) { ch[hq[p].h1] = 1; ch[hq[p].h2] = 1; }
            }
            distinct += ch.size();
        }
        size_t mx = 0;
        for (auto &v : xs) mx = std::max(mx, v.size());
        kp_hpair hp[KP_MAX_HPAIRS];
        for (size_t s = 0; s < mx; ++s)
            for (int x = 0; x < 8; ++x) {
                if (s >= xs[x].size()) continue;
                const uint64_t h = xs[x][s];
                const int np = kp_high_pairs(g, P.tabs.data(), h, hp);
                for (int p = 0; p < np; ++p) {
                    // high position of the pair (code = position << 3 | pair); its rank in the
                    // plan order: positions kh-1, kh-2, ... are fastest (M last)
                    const int pos = (int)(hp[p].code >> 3) - g.t;
                    const bool nt = slow_nt.count(pos) > 0;
                    for (uint64_t c : {hp[p].h1, hp[p].h2}) {
                        ++reads;
                        if (nt) {  // non-temporal: hits where present, allocates nowhere
                            if (!l2[x].peek(c)) {
                                ++l2miss;
                                if (!mall.peek(c)) ++mallmiss;
                            }
                        } else if (!l2[x].touch(c)) {
                            ++l2miss;
                            if (!mall.touch(c)) ++mallmiss;
                        }
                    }
                }
                ++writes;
                l2[x].touch(h);  // stores keep the line in the XCD's L2 (nt too)
            }
    }
    const double GB = 1e9;
    printf("{\"gen_pat\": \"%s\", \"lanes\": %d, \"schedule\": \"%s\", \"param\": %d, \"row_bytes\": %.0f, "
           "\"l2_rows\": %zu, \"mall_rows\": %zu, \"reads_GB\": %.1f, \"l2_miss_GB\": %.1f, \"mall_miss_GB\": %.1f, "
           "\"writes_GB\": %.1f, \"l2_hit\": %.4f, \"mall_hit_of_l2miss\": %.4f, \"distinct_children_GB\": %.1f}\n",
           argv[1], lanes, sched.c_str(), param, row_bytes, l2_rows, mall_rows, reads * row_bytes / GB,
           l2miss * row_bytes / GB, mallmiss * row_bytes / GB, writes * row_bytes / GB,
           1.0 - (double)l2miss / reads, 1.0 - (double)mallmiss / l2miss, distinct * row_bytes / GB);
    return 0;
}
