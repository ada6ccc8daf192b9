// flowsim.cpp -- timing + cache model of one DP pass under level-synchronous launches or
// a dataflow (ticket-ordered, no launch boundaries) schedule.  Tool, not product: it
// answers whether a sweep that is not level-synchronous would pay.
//
// Machine model (fluid, event driven): 8 XCDs x 32 CUs x 2 workgroup slots (the sweep's
// occupancy).  A block (one LDS block of the plan, all lanes of a pass) runs
//   prologue  P us (block setup + count tables),
//   gather    its high split pairs' child rows, 2 x row bytes per pair, progressing at
//             min(rmax, B / gatherers) bytes/us (B = the chip's effective gather rate),
//   level     the LDS level phase: Lw us alone on its CU, Lw / c2 us while the CU's other
//             slot is in its level phase too (VALU shared),
// then its score row is stored.  Level-synchronous: every launch (one high level) waits
// for the previous one, T_launch us between launches; blocks go to XCDs in runs of R list
// entries (KP_XCD_REMAP).  Dataflow: every XCD walks its own ticket list; a slot takes the
// next ticket, waits until the block's child blocks are complete (flags), then runs it.
// No launch boundaries; the first ticket of a list never waits on a later one (topological
// ticket order), so it cannot deadlock.
//
// Cache model (row granular, as tools/cachesim.cpp): child reads at gather start through
// the XCD's LRU L2 and the shared LRU Infinity Cache (MALL); reads along the plan's three
// slowest high positions are non-temporal (KP_NT_SLOW=3: hit where present, allocate
// nowhere); score-row writes allocate in the L2 and (write-allocate, the guide's residency
// rule counts stored bytes) in the MALL.
//
// build: g++ -O2 -std=c++17 -o tools/flowsim tools/flowsim.cpp
// usage: tools/flowsim GEN_PAT LANES SCHEDULE [key=value ...]
//   SCHEDULE: levels (the product's launches), flow (the same ticket order, no
//   barriers), slab (fast-axis slabs: tickets ordered by (slow-axis level, slow index,
//   fast-axis level, fast index), the plan's `fast` fastest high positions in the slab)
//   keys: P Lw c2 B rmax Tl R fast calib=1 (print per-launch ms)
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <list>
#include <map>
#include <queue>
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
    bool touch(uint64_t key) {
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

static std::map<std::string, double> g_kv;
static double kv(const char *k, double d) {
    auto it = g_kv.find(k);
    return it == g_kv.end() ? d : it->second;
}

int main(int argc, char **argv) {
    if (argc < 4) {
        fprintf(stderr, "usage: %s GEN_PAT LANES SCHEDULE [key=value ...]\n", argv[0]);
        return 2;
    }
    for (int i = 4; i < argc; ++i) {
        const char *eq = strchr(argv[i], '=');
        if (eq) g_kv[std::string(argv[i], eq - argv[i])] = atof(eq + 1);
    }
    kp::host_plan P;
    std::string err = kp::build_plan(argv[1], 4096, P);
    if (!err.empty()) {
        fprintf(stderr, "%s\n", err.c_str());
        return 1;
    }
    const int lanes = atoi(argv[2]);
    const std::string sched = argv[3];
    const kp_geom &g = P.g;
    const uint64_t nb = g.nblocks;
    const double row_bytes = (double)lanes * g.Bpad * 4;
    // model parameters (us, bytes/us); defaults calibrated against the measured 5-lane
    // launch times (see calib)
    const double Pro = kv("P", 8.0), Lw = kv("Lw", 28.0), c2 = kv("c2", 0.667);
    const double B = kv("B", 7.9e6), rmax = kv("rmax", 4.0e4), Tl = kv("Tl", 6.0);
    const uint64_t R = (uint64_t)kv("R", 40);
    const int fast = (int)kv("fast", 3);
    const int calib = (int)kv("calib", 0);
    const bool nt_on = kv("nt", 1) != 0;
    const bool walloc = kv("walloc", 1) != 0;  // score-row writes allocate in the MALL
    // cost=1: a read's fabric cost by where it is served (L2 hit wL2, MALL hit wH, HBM wM; the
    // guide's gather rates: 8.6 TB/s from the Infinity Cache, 6.0 from HBM -> wM/wH = 1.43);
    // B is then in weighted bytes/us
    const bool cost_model = kv("cost", 0) != 0;
    const double wL2 = kv("wL2", 0.25), wH = kv("wH", 1.0), wM = kv("wM", 1.43);
    const size_t l2_rows = (size_t)(4.0 * 1048576 / row_bytes), mall_rows = (size_t)(256.0 * 1048576 / row_bytes);

    // high level of every block, pair count
    std::vector<uint8_t> lev(nb), npairs(nb);
    for (uint64_t h = 0; h < nb; ++h) {
        lev[h] = (uint8_t)kp_high_level(g, P.tabs.data(), h);
        npairs[h] = (uint8_t)kp_high_pair_count(g, P.tabs.data(), h);
    }
    // slow positions (non-temporal reads): the last three of the plan's order
    std::set<int> slow;
    for (size_t j = P.perm.size() >= 3 ? P.perm.size() - 3 : 0; j < P.perm.size(); ++j) slow.insert(P.perm[j]);

    // ticket lists per XCD, and (level-synchronous) the launch boundaries in each list
    std::vector<std::vector<uint32_t>> xl(8);
    std::vector<std::vector<size_t>> xb(8);  // per XCD: list index where launch H starts
    const bool barriers = sched == "levels";
    if (sched == "levels" || sched == "flow") {
        for (int H = 0; H <= P.hmax; ++H) {
            for (int x = 0; x < 8; ++x) xb[x].push_back(xl[x].size());
            const uint64_t b0 = P.hoff[H], n = P.hoff[H + 1] - b0;
            for (uint64_t e = 0; e < n; ++e) xl[(e / R) & 7u].push_back(P.hlist[b0 + e]);
        }
    } else if (sched == "slab") {
        // fast positions = the plan order's first `fast` high positions
        std::vector<int> fpos(P.perm.begin(), P.perm.begin() + std::min<size_t>(fast, P.perm.size()));
        std::vector<std::pair<std::vector<uint64_t>, uint32_t>> kvs(nb);
        for (uint64_t h = 0; h < nb; ++h) {
            uint64_t sl = 0, fl = 0, sidx = 0, fidx = 0;
            for (int q = (int)P.perm.size() - 1; q >= 0; --q) {  // slowest first
                const int i = P.perm[q];
                const uint32_t d = kp_high_digit(g, h, i);
                const bool isf = std::find(fpos.begin(), fpos.end(), i) != fpos.end();
                if (isf) {
                    fl += P.tabs[g.t + i].lev[d];
                    fidx = fidx * 16 + d;
                } else {
                    sl += P.tabs[g.t + i].lev[d];
                    sidx = sidx * 16 + d;
                }
            }
            kvs[h] = {{sl, sidx, fl, fidx}, (uint32_t)h};
        }
        // groups of `G` slabs of one slow level progress together, fast level by fast level
        const uint64_t Gs = (uint64_t)kv("G", 1);
        if (Gs > 1) {
            std::map<std::pair<uint64_t, uint64_t>, uint64_t> rank;
            for (auto &e : kvs) rank[{e.first[0], e.first[1]}] = 0;
            uint64_t r = 0, last = ~0ull;
            for (auto &e : rank) {
                if (e.first.first != last) r = 0, last = e.first.first;
                e.second = r++;
            }
            for (auto &e : kvs) {
                const uint64_t rk = rank[{e.first[0], e.first[1]}];
                e.first = {e.first[0], rk / Gs, e.first[2], e.first[1], e.first[3]};
            }
        }
        std::sort(kvs.begin(), kvs.end());
        for (uint64_t e = 0; e < nb; ++e) xl[(e / R) & 7u].push_back(kvs[e].second);
    } else {
        fprintf(stderr, "unknown schedule\n");
        return 2;
    }

    // ---- simulation ----
    const int NS = 8 * 32 * 2;
    enum { IDLE, WAIT, PRO, GATH, LEVL, DONE };
    struct Slot {
        int st = IDLE;
        uint32_t blk = 0;
        double t_end = 0;   // PRO end time
        double g_fin = 0;   // gather finish on the global progress clock
        double work = 0;    // LEVL remaining work (alone-us)
        double t_mark = 0;  // time of last LEVL rate change
        int ver = 0;
    };
    std::vector<Slot> S(NS);
    std::vector<size_t> next(8, 0), lim(8, 0);
    int H = 0;
    auto set_limits = [&]() {
        for (int x = 0; x < 8; ++x) lim[x] = barriers ? (H + 1 < (int)xb[x].size() + 0 && H + 1 <= P.hmax ? xb[x][H + 1] : xl[x].size()) : xl[x].size();
    };
    if (barriers)
        for (int x = 0; x < 8; ++x) next[x] = xb[x][0];
    set_limits();
    std::vector<uint8_t> done(nb, 0);
    std::vector<uint32_t> pend(NS, 0);
    std::unordered_map<uint32_t, std::vector<int>> waiters;
    std::vector<LRU> l2(8, LRU(l2_rows));
    LRU mall(mall_rows);
    uint64_t reads = 0, l2miss = 0, mallmiss = 0, writes = 0, wmiss = 0;
    double now = 0, G = 0;  // global gather progress clock (bytes per gatherer)
    int ngath = 0;
    std::vector<int> nlev(256, 0);
    double wait_us = 0;
    std::priority_queue<std::pair<double, int>, std::vector<std::pair<double, int>>, std::greater<>> pro_q, gat_q;
    struct LE { double t; int s, ver; bool operator>(const LE &o) const { return t > o.t; } };
    std::priority_queue<LE, std::vector<LE>, std::greater<LE>> lev_q;
    uint64_t completed = 0, level_total = 0, level_done = 0;
    std::vector<double> launch_ms;
    double launch_t0 = 0;
    if (barriers) {
        level_total = P.hoff[1] - P.hoff[0];
    }
    auto rate = [&]() { return ngath ? std::min(rmax, B / ngath) : rmax; };
    auto lrate = [&](int cu) { return nlev[cu] >= 2 ? c2 : 1.0; };
    auto resched_cu = [&](int cu) {
        for (int s = cu * 2; s < cu * 2 + 2; ++s)
            if (S[s].st == LEVL) {
                S[s].ver++;
                lev_q.push({now + S[s].work / lrate(cu), s, S[s].ver});
            }
    };
    auto settle_cu = [&](int cu) {  // account level work done up to now at the current rate
        for (int s = cu * 2; s < cu * 2 + 2; ++s)
            if (S[s].st == LEVL) {
                S[s].work -= (now - S[s].t_mark) * lrate(cu);
                if (S[s].work < 0) S[s].work = 0;
                S[s].t_mark = now;
            }
    };
    kp_hpair hp[KP_MAX_HPAIRS];
    std::function<void(int)> try_take;
    auto start_block = [&](int s) {
        Slot &sl = S[s];
        sl.st = PRO;
        sl.t_end = now + Pro;
        pro_q.push({sl.t_end, s});
    };
    try_take = [&](int s) {
        const int x = (s / 2) % 8;  // CU c = s / 2 sits on XCD c % 8
        Slot &sl = S[s];
        if (next[x] >= lim[x]) {
            sl.st = IDLE;
            return;
        }
        const uint32_t h = xl[x][next[x]++];
        sl.blk = h;
        // children still running?
        uint32_t np = (uint32_t)kp_high_pairs(g, P.tabs.data(), h, hp), cnt = 0;
        for (uint32_t p = 0; p < np; ++p)
            for (uint64_t c : {hp[p].h1, hp[p].h2})
                if (!done[c]) {
                    waiters[(uint32_t)c].push_back(s);
                    ++cnt;
                }
        sl.t_mark = now;
        if (cnt) {
            sl.st = WAIT;
            pend[s] = cnt;
            return;
        }
        start_block(s);
    };
    for (int s = 0; s < NS; ++s) try_take(s);
    while (completed < nb) {
        // next event
        double tp = pro_q.empty() ? 1e300 : pro_q.top().first;
        double tg = gat_q.empty() ? 1e300 : now + (gat_q.top().first - G) / rate();
        while (!lev_q.empty() && (S[lev_q.top().s].st != LEVL || S[lev_q.top().s].ver != lev_q.top().ver)) lev_q.pop();
        double tlv = lev_q.empty() ? 1e300 : lev_q.top().t;
        double t = std::min(tp, std::min(tg, tlv));
        if (t >= 1e299) {
            fprintf(stderr, "deadlock at %llu of %llu blocks\n", (unsigned long long)completed, (unsigned long long)nb);
            return 3;
        }
        // advance clocks
        G += (t - now) * rate();
        now = t;
        if (t == tp) {
            const int s = pro_q.top().second;
            pro_q.pop();
            Slot &sl = S[s];
            const int x = (s / 2) % 8;
            // gather start: replay the child reads
            const uint32_t h = sl.blk;
            const int np = kp_high_pairs(g, P.tabs.data(), h, hp);
            double wsum = 0;  // cache-weighted rows (cost model) or plain rows
            for (int p = 0; p < np; ++p) {
                const int pos = (int)(hp[p].code >> 3) - g.t;
                const bool nt = nt_on && slow.count(pos) > 0;
                for (uint64_t c : {hp[p].h1, hp[p].h2}) {
                    ++reads;
                    int where = 0;  // 0 L2 hit, 1 MALL hit, 2 HBM
                    if (nt) {
                        if (!l2[x].peek(c)) where = mall.peek(c) ? 1 : 2;
                    } else if (!l2[x].touch(c)) {
                        where = mall.touch(c) ? 1 : 2;
                    }
                    if (where >= 1) ++l2miss;
                    if (where == 2) ++mallmiss;
                    wsum += cost_model ? (where == 0 ? wL2 : where == 1 ? wH : wM) : 1.0;
                }
            }
            const double bytes = wsum * row_bytes;
            if (bytes > 0) {
                sl.st = GATH;
                sl.g_fin = G + bytes;
                ++ngath;
                gat_q.push({sl.g_fin, s});
            } else {
                const int cu = s / 2;
                settle_cu(cu);
                sl.st = LEVL;
                sl.work = Lw;
                sl.t_mark = now;
                ++nlev[cu];
                resched_cu(cu);
            }
            continue;
        }
        if (t == tg) {
            const int s = gat_q.top().second;
            gat_q.pop();
            --ngath;
            const int cu = s / 2;
            settle_cu(cu);
            S[s].st = LEVL;
            S[s].work = Lw;
            S[s].t_mark = now;
            ++nlev[cu];
            resched_cu(cu);
            continue;
        }
        // level phase done: block complete
        const int s = lev_q.top().s;
        lev_q.pop();
        const int cu = s / 2, x = cu % 8;
        settle_cu(cu);
        --nlev[cu];
        Slot &sl = S[s];
        sl.st = DONE;
        resched_cu(cu);
        const uint32_t h = sl.blk;
        ++writes;
        l2[x].touch(h);
        if (walloc && !mall.touch(h)) ++wmiss;
        done[h] = 1;
        ++completed;
        // wake waiters
        auto it = waiters.find(h);
        if (it != waiters.end()) {
            std::vector<int> ws;
            ws.swap(it->second);
            waiters.erase(it);
            for (int w : ws)
                if (--pend[w] == 0) {
                    wait_us += now - S[w].t_mark;
                    start_block(w);
                }
        }
        if (barriers) {
            ++level_done;
            if (level_done == level_total) {  // launch complete
                launch_ms.push_back((now - launch_t0) / 1e3);
                ++H;
                if (H <= P.hmax) {
                    now += Tl;
                    launch_t0 = now;
                    level_done = 0;
                    level_total = P.hoff[H + 1] - P.hoff[H];
                    set_limits();
                    for (int q = 0; q < NS; ++q)
                        if (S[q].st == IDLE || S[q].st == DONE) try_take(q);
                }
                continue;
            }
        }
        try_take(s);
        // (level-synchronous: an idle slot stays idle until the next launch)
    }
    const double GB = 1e9;
    printf("{\"gen_pat\": \"%s\", \"lanes\": %d, \"schedule\": \"%s\", \"fast\": %d, \"R\": %llu, "
           "\"P\": %g, \"Lw\": %g, \"c2\": %g, \"B\": %g, \"rmax\": %g, \"Tl\": %g, \"pass_ms\": %.2f, "
           "\"wait_slot_ms\": %.1f, \"reads_GB\": %.1f, \"l2_miss_GB\": %.1f, \"mall_miss_GB\": %.1f, "
           "\"write_GB\": %.1f, \"write_alloc_miss_GB\": %.1f",
           argv[1], lanes, sched.c_str(), fast, (unsigned long long)R, Pro, Lw, c2, B, rmax, Tl, now / 1e3,
           wait_us / 1e3, reads * row_bytes / GB, l2miss * row_bytes / GB, mallmiss * row_bytes / GB,
           writes * row_bytes / GB, wmiss * row_bytes / GB);
    if (calib || barriers) {
        printf(", \"launch_ms\": [");
        for (size_t i = 0; i < launch_ms.size(); ++i) printf("%s%.3f", i ? ", " : "", launch_ms[i]);
        printf("]");
    }
    printf("}\n");
    return 0;
}
