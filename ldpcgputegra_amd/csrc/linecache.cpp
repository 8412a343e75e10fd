// linecache.cpp -- host planner of coop3's LDS line cache.
//
// coop3 keeps V (the int8 LLRs of a workgroup's 16 codewords) in the grouped
// layout Vg[group][row][16 B] and moves the information rows between HBM and
// the workgroup's LDS as whole 128-B lines (8 consecutive rows x 16
// codewords), instead of one scattered 16-B piece per edge and check each way.
// DVB-S2 is what makes lines pay: information bit m of a 360-bit group is
// touched by checks x + m q (ETSI EN 302 307 Annex B, the reference's tables
// code/x86/Constantes/64800x32400.dvb-s2/constantes_sse.h), so the layered
// schedule walks each address of a group through consecutive bits, one bit
// per q = 90 checks (two coop3 windows): one line load serves ~8 uses.
//
// The plan is static (per code, from the coop3 window schedule), periodic
// with the nw windows of one iteration, and self-checked by replaying it:
//   * window u's pre reads its info entries in period u - 1, its post writes
//     them in period u + 1 (coop3_decode's period p: post of window p-1, pre
//     of window p+1);
//   * a residency (a line's accesses, split where two are >= LC_GAP periods
//     apart) is loaded into VGPRs in period tl <= f - 3 (f = first access) by
//     lane group i of slab wave w's set, written into its LDS slot by the same
//     lanes in period tl + LC_PUT, and -- if written to -- written back (slot ->
//     VGPRs -> HBM, whole line) in period tw >= e + 1 (e = last access); the
//     slot is held over [tl + LC_PUT, tw];
//   * a line written back is loaded again >= 3 periods after its store (the
//     kernel's per-period vmcnt waits complete a store by then);
//   * at most S loads and S writebacks per period (S / 8 slab waves x 8 lane
//     groups: one 64-lane global load and one 64-lane global store per wave and
//     period, unused lane groups on the sink line / sink slot);
//   * no load in the last LC_PUT periods of an iteration, so that a segment start
//     has no load in flight: the lines resident at a segment start are filled
//     by its prologue (LcPlan::pro) and the dirty ones left at its end are
//     written back by its epilogue (LcPlan::epi);
//   * slot 0 is the sink (the inactive slots' info entries), HBM line n / 8
//     the sink line (rows n .. n+7: row n is the parity sink as well).
#include <algorithm>
#include <map>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "coop.h"

namespace {

struct Res {
    uint32_t line;
    int f, e;            // first / last access period (f in [0, nw), e >= f, may exceed nw)
    int tl, tw;          // load period, writeback period (tw = e when clean), unrolled around f
    bool dirty, whole;   // written to; resident for the whole iteration
    int fw = 1 << 30;    // first write period (unrolled like e)
    int slot = -1;
    int z = 0;              // XOR swizzle of its rows in the slot (LcPlan)
    int li = -1, wi = -1;   // index of its load / writeback in the period's op list
};

inline int cmod(int a, int m) { return ((a % m) + m) % m; }

// no plan: -1 (LDPC_LC_DEBUG=1 names the planner line that gave up)
int lc_fail(int line)
{
    const char *e = getenv("LDPC_LC_DEBUG");
    if (e && *e == '1') fprintf(stderr, "coop3 line cache plan: none (linecache.cpp:%d)\n", line);
    return -1;
}

}  // namespace

int lc_build_plan(const std::vector<uint32_t> &tab, int recw, int nw, int S, int D0, int n, int k, int max_slots,
                  LcPlan &o)
{
    o = LcPlan{};
    const int X = D0 - 2;
    // line loads / writebacks per period: NLD per lane group (slot) of the slab
    // waves, NLD = ceil(X / 8) (a window's ~S X accesses touch ~S X / 8 new lines)
    const int LC_OPS = S * ((D0 - 2 + 7) / 8);
    if (S % 8 != 0 || S > 64 || nw < 4 * LC_GAP || n % 8 != 0 || k % 8 != 0 || k <= 0 || max_slots < 2 || n / 8 + 1 >= 65536)
        return lc_fail(__LINE__);
    const uint32_t nlines = (uint32_t)(k / 8), sink_line = (uint32_t)(n / 8);
    auto rec_at = [&](int u, int kk) { return &tab[((size_t)u * S + kk) * recw]; };
    // accesses per line: period << 1 | write
    std::vector<std::vector<uint32_t>> acc(nlines);
    for (int u = 0; u < nw; u++)
        for (int kk = 0; kk < S; kk++) {
            const uint32_t *r = rec_at(u, kk);
            if (!(r[D0] & COOP_M_ACT)) continue;
            for (int j = 0; j < X; j++) {
                if (r[j] >= (uint32_t)k) return lc_fail(__LINE__);   // info entries must be information rows
                acc[r[j] / 8].push_back((uint32_t)cmod(u - 1, nw) << 1);
                acc[r[j] / 8].push_back((uint32_t)cmod(u + 1, nw) << 1 | 1u);
            }
            for (int j = X; j < D0; j++)
                if (r[j] < (uint32_t)k) return lc_fail(__LINE__);   // x / o entries: parity rows
        }
    // residencies
    std::vector<Res> rs;
    std::vector<std::vector<int>> res_of(nlines);   // per line, in cyclic order of f
    for (uint32_t L = 0; L < nlines; L++) {
        auto &a = acc[L];
        if (a.empty()) continue;
        std::sort(a.begin(), a.end());
        std::vector<int> per;
        std::vector<char> wr;
        for (uint32_t x : a) {
            const int p = (int)(x >> 1);
            if (per.empty() || per.back() != p) {
                per.push_back(p);
                wr.push_back(0);
            }
            wr.back() |= (char)(x & 1u);
        }
        const int m = (int)per.size();
        std::vector<int> cut;   // i: a cut between access i and i + 1 (cyclic)
        for (int i = 0; i < m; i++) {
            const int gap = i + 1 < m ? per[i + 1] - per[i] : per[0] + nw - per[i];
            if (gap >= LC_GAP) cut.push_back(i);
        }
        if (cut.empty()) {
            Res R{L, per[0], per[0] + nw - 1, 0, 0, false, true};
            for (int i = 0; i < m; i++) R.dirty |= wr[i] != 0;
            res_of[L].push_back((int)rs.size());
            rs.push_back(R);
            continue;
        }
        // start at the access after the last cut so that the residencies come out in cyclic order
        for (size_t c = 0; c < cut.size(); c++) {
            const int s = (cut[c] + 1) % m, t = cut[(c + 1) % cut.size()];
            Res R{L, per[s], per[s], 0, 0, false, false};
            for (int i = s;; i = (i + 1) % m) {
                R.dirty |= wr[i] != 0;
                R.e = per[i] >= R.f ? per[i] : per[i] + nw;
                if (wr[i]) R.fw = std::min(R.fw, R.e);
                if (i == t) break;
            }
            res_of[L].push_back((int)rs.size());
            rs.push_back(R);
        }
        std::sort(res_of[L].begin(), res_of[L].end(), [&](int x, int y) { return rs[x].f < rs[y].f; });
    }
    for (Res &R : rs) {
        R.tl = R.f - LC_LEAD;
        R.tw = R.dirty ? R.e + 1 : R.e;
    }
    // the store of a residency -> the next residency's load of the same line
    // >= 3 periods later (cyclic, the next one may be itself an iteration on)
    auto next_of = [&](int id) -> int {
        const auto &v = res_of[rs[id].line];
        const size_t i = std::find(v.begin(), v.end(), id) - v.begin();
        return v[(i + 1) % v.size()];
    };
    auto prev_of = [&](int id) -> int {
        const auto &v = res_of[rs[id].line];
        const size_t i = std::find(v.begin(), v.end(), id) - v.begin();
        return v[(i + v.size() - 1) % v.size()];
    };
    auto reload_ok = [&](int a, int b) {   // a's store before b's load
        const Res &A = rs[a], &B = rs[b];
        if (A.whole || B.whole || !A.dirty) return true;
        int btl = B.tl;
        while (btl + 0 <= A.tl) btl += nw;   // B's load after A's (unrolled)
        return btl >= A.tw + 3;
    };
    // constraints: no load in the last LC_PUT periods of an iteration; at most
    // LC_OPS loads / writebacks per period (moving loads earlier, writebacks later)
    for (int round = 0;; round++) {
        if (round == 256) return lc_fail(__LINE__);
        bool moved = false;
        std::vector<std::vector<int>> lp(nw), wp(nw);
        for (int i = 0; i < (int)rs.size(); i++) {
            Res &R = rs[i];
            if (R.whole) continue;
            while (cmod(R.tl, nw) >= nw - LC_PUT) {
                R.tl--;
                moved = true;
                if (!reload_ok(prev_of(i), i)) return lc_fail(__LINE__);
            }
            lp[cmod(R.tl, nw)].push_back(i);
            if (R.dirty) wp[cmod(R.tw, nw)].push_back(i);
        }
        for (int p = 0; p < nw; p++) {
            auto life = [&](int x) { return rs[x].tw - rs[x].tl; };
            if ((int)lp[p].size() > LC_OPS) {
                std::stable_sort(lp[p].begin(), lp[p].end(), [&](int x, int y) { return life(x) < life(y); });
                int over = (int)lp[p].size() - LC_OPS;
                for (size_t j = 0; j < lp[p].size() && over > 0; j++) {
                    const int i = lp[p][j];
                    rs[i].tl--;
                    if (!reload_ok(prev_of(i), i)) {
                        rs[i].tl++;
                        continue;
                    }
                    over--;
                    moved = true;
                }
                if (over > 0) return lc_fail(__LINE__);
            }
            if ((int)wp[p].size() > LC_OPS) {
                std::stable_sort(wp[p].begin(), wp[p].end(), [&](int x, int y) { return life(x) < life(y); });
                int over = (int)wp[p].size() - LC_OPS;
                for (size_t j = 0; j < wp[p].size() && over > 0; j++) {
                    const int i = wp[p][j];
                    rs[i].tw++;
                    if (!reload_ok(i, next_of(i))) {
                        rs[i].tw--;
                        continue;
                    }
                    over--;
                    moved = true;
                }
                if (over > 0) return lc_fail(__LINE__);
            }
        }
        if (!moved) break;
    }
    for (int i = 0; i < (int)rs.size(); i++) {
        if (rs[i].whole) continue;
        if (rs[i].tw - (rs[i].tl + LC_PUT) >= nw - 1) return lc_fail(__LINE__);
        if (!reload_ok(prev_of(i), i) || !reload_ok(i, next_of(i))) return lc_fail(__LINE__);
    }
    // slots: circular-arc assignment of the holds [tl + LC_PUT, tw].  Cut at the
    // period p0 with the fewest holds: the holds across p0 get a slot each,
    // the rest go in order of their start to the free slot whose next hold
    // starts soonest after them (best fit)
    std::vector<int> live(nw, 0);
    for (const Res &R : rs)
        if (!R.whole)
            for (int p = R.tl + LC_PUT; p <= R.tw; p++) live[cmod(p, nw)]++;
    // assignment from the cut at p0 with fit rule `rule` (0: the fitting slot
    // whose next hold starts soonest, 1: the one freed last); returns the slots
    // used (sink excluded)
    auto assign = [&](int p0, int rule) -> int {
        std::vector<int> free_from, next_busy;   // per slot 1.. (index + 1), relative to p0
        constexpr int INF = 1 << 30;
        std::vector<int> order;
        for (int i = 0; i < (int)rs.size(); i++) {
            Res &R = rs[i];
            if (R.whole) {
                R.slot = (int)free_from.size() + 1;
                free_from.push_back(INF);
                next_busy.push_back(-1);
                continue;
            }
            const int a = R.tl + LC_PUT, len = R.tw - a;
            if (cmod(p0 - a, nw) <= len) {   // across p0
                R.slot = (int)free_from.size() + 1;
                free_from.push_back(cmod(R.tw - p0, nw) + 1);
                next_busy.push_back(cmod(a - p0, nw));
            } else {
                order.push_back(i);
            }
        }
        std::sort(order.begin(), order.end(), [&](int x, int y) {
            const int ax = cmod(rs[x].tl + LC_PUT - p0, nw), ay = cmod(rs[y].tl + LC_PUT - p0, nw);
            return ax != ay ? ax < ay : x < y;
        });
        for (int i : order) {
            Res &R = rs[i];
            const int ra = cmod(R.tl + LC_PUT - p0, nw), rb = ra + (R.tw - (R.tl + LC_PUT));
            int best = -1;
            for (int c = 0; c < (int)free_from.size(); c++) {
                if (free_from[c] > ra || next_busy[c] <= rb) continue;
                if (rule == 0 ? (best < 0 || next_busy[c] < next_busy[best] ||
                                 (next_busy[c] == next_busy[best] && free_from[c] > free_from[best]))
                              : (best < 0 || free_from[c] > free_from[best] ||
                                 (free_from[c] == free_from[best] && next_busy[c] < next_busy[best])))
                    best = c;
            }
            if (best < 0) {
                best = (int)free_from.size();
                free_from.push_back(0);
                next_busy.push_back(INF);
            }
            free_from[best] = rb + 1;
            R.slot = best + 1;
        }
        return (int)free_from.size();
    };
    // cut candidates: the periods with the fewest holds
    std::vector<int> cand(nw);
    for (int p = 0; p < nw; p++) cand[p] = p;
    std::stable_sort(cand.begin(), cand.end(), [&](int x, int y) { return live[x] < live[y]; });
    const char *ev = getenv("LDPC_LC_CUTS");
    const int ncut = std::min(nw, ev && *ev ? atoi(ev) : 1);
    // slot-by-slot chains: each new slot starts at the unassigned hold that
    // starts first (from p0) and takes, again and again, the unassigned hold
    // that starts soonest after its last one ends and ends before its first
    // one starts again an iteration later -- every slot packed around the
    // circle once (near max-live slots for holds of similar length)
    auto chains = [&](int p0) -> int {
        std::multimap<int, int> free_at;   // start (relative to p0) -> residency
        int nsl = 0;
        for (int i = 0; i < (int)rs.size(); i++) {
            Res &R = rs[i];
            if (R.whole) {
                R.slot = ++nsl;
                continue;
            }
            free_at.emplace(cmod(R.tl + LC_PUT - p0, nw), i);
        }
        while (!free_at.empty()) {
            auto it = free_at.begin();
            const int first = it->first, slot = ++nsl;
            int end = first + (rs[it->second].tw - (rs[it->second].tl + LC_PUT));   // relative to p0, may pass nw
            rs[it->second].slot = slot;
            free_at.erase(it);
            for (;;) {
                // the unassigned hold starting soonest after `end` (on the line
                // unrolled from p0; past nw it wraps to the starts + nw), if it
                // ends before this slot's first hold starts again
                const int want = end + 1;
                bool wrapped = want >= nw;
                auto nx = free_at.lower_bound(wrapped ? want - nw : want);
                if (nx == free_at.end() && !wrapped) {
                    nx = free_at.begin();
                    wrapped = true;
                }
                if (nx == free_at.end()) break;
                const int s_abs = nx->first + (wrapped ? nw : 0);
                const int len = rs[nx->second].tw - (rs[nx->second].tl + LC_PUT);
                if (s_abs + len >= first + nw) break;   // would meet the slot's first hold: slot full
                rs[nx->second].slot = slot;
                end = s_abs + len;
                free_at.erase(nx);
            }
        }
        return nsl;
    };
    // rule 0 first (the r1/2 plan measured in r04/r05); rule 1 only if that
    // does not fit the slots the kernel has
    int best_p0 = cand[0], best_n = 1 << 30, best_rule = 0;
    for (int rule = 0; rule < 2 && best_n + 1 > max_slots; rule++)
        for (int i = 0; i < ncut; i++) {
            const int nsl = assign(cand[i], rule);
            if (ev && *ev) fprintf(stderr, "cut %d rule %d live %d -> %d slots\n", cand[i], rule, live[cand[i]], nsl);
            if (nsl < best_n) {
                best_n = nsl;
                best_p0 = cand[i];
                best_rule = rule;
            }
        }
    int used = assign(best_p0, best_rule);
    if (used + 1 > max_slots) {   // rule 2: packed chains from the same cut
        const int nsl = chains(best_p0);
        const char *dbg = getenv("LDPC_LC_DEBUG");
        if (dbg && *dbg) fprintf(stderr, "coop3 line cache: chains from cut %d -> %d slots (greedy %d)\n", best_p0, nsl, used);
        used = nsl;
    }
    // still too many: empty the least-used slots by moving each of their holds
    // into a gap of another slot (holds are cyclic arcs [tl + LC_PUT, tw]; one
    // slot's arcs must not overlap), fullest targets first, or -- where no gap
    // fits -- into a slot whose only hold in the way moves to a gap elsewhere
    // (one ejection), until no slot can be emptied (the greedy cut above
    // wastes slots near the cut)
    if (used + 1 > max_slots) {
        const int NS1 = used + 1, NWB = (NS1 + 63) / 64;   // slots 1 .. used
        std::vector<int> own((size_t)NS1 * nw, -1);          // residency holding slot t in period p
        std::vector<uint64_t> freeb((size_t)nw * NWB, 0);    // per period: the slots free in it
        std::vector<std::vector<int>> of(NS1);
        for (int p = 0; p < nw; p++)
            for (int t = 1; t < NS1; t++) freeb[(size_t)p * NWB + t / 64] |= 1ull << (t % 64);
        auto span = [&](int i, auto &&f) {   // f(period) over residency i's hold
            const Res &R = rs[i];
            if (R.whole) {
                for (int p = 0; p < nw; p++) f(p);
                return;
            }
            const int a0 = cmod(R.tl + LC_PUT, nw), len = R.tw - (R.tl + LC_PUT);
            for (int q = 0; q <= len; q++) f((a0 + q) % nw);
        };
        auto place = [&](int i, int t) {
            span(i, [&](int p) {
                own[(size_t)t * nw + p] = i;
                freeb[(size_t)p * NWB + t / 64] &= ~(1ull << (t % 64));
            });
            rs[i].slot = t;
            of[t].push_back(i);
        };
        auto unplace = [&](int i) {
            const int t = rs[i].slot;
            span(i, [&](int p) {
                own[(size_t)t * nw + p] = -1;
                freeb[(size_t)p * NWB + t / 64] |= 1ull << (t % 64);
            });
            of[t].erase(std::find(of[t].begin(), of[t].end(), i));
        };
        // the fullest slot free over residency i's whole hold, other than x1 / x2; -1: none
        std::vector<uint64_t> m(NWB);
        auto home = [&](int i, int x1, int x2) -> int {
            std::fill(m.begin(), m.end(), ~0ull);
            span(i, [&](int p) {
                for (int w = 0; w < NWB; w++) m[w] &= freeb[(size_t)p * NWB + w];
            });
            int best = -1;
            for (int w = 0; w < NWB; w++)
                for (uint64_t b = m[w]; b; b &= b - 1) {
                    const int t = w * 64 + __builtin_ctzll(b);
                    if (t == x1 || t == x2 || of[t].empty()) continue;
                    if (best < 0 || of[t].size() > of[best].size()) best = t;
                }
            return best;
        };
        {
            std::vector<int> tmp(rs.size());
            for (int i = 0; i < (int)rs.size(); i++) tmp[i] = rs[i].slot;
            for (int i = 0; i < (int)rs.size(); i++) place(i, tmp[i]);
        }
        for (bool progress = true; progress && used + 1 > max_slots;) {
            progress = false;
            std::vector<int> order;
            for (int s2 = 1; s2 < NS1; s2++)
                if (!of[s2].empty()) order.push_back(s2);
            std::sort(order.begin(), order.end(), [&](int x, int y) { return of[x].size() < of[y].size(); });
            for (int s2 : order) {
                if (of[s2].empty() || used + 1 <= max_slots) continue;
                std::vector<std::pair<int, int>> moves;   // (residency, slot it came from), for the rollback
                bool ok = true;
                const std::vector<int> holds = of[s2];
                for (int i : holds) {
                    int t = home(i, s2, -1);
                    if (t >= 0) {
                        unplace(i);
                        place(i, t);
                        moves.push_back({i, s2});
                        continue;
                    }
                    // one ejection: a slot where a single hold j is in the way and j fits elsewhere
                    bool done = false;
                    for (int t1 = 1; t1 < NS1 && !done; t1++) {
                        if (t1 == s2 || of[t1].empty()) continue;
                        int j = -1;
                        bool single = true;
                        span(i, [&](int p) {
                            const int o2 = own[(size_t)t1 * nw + p];
                            if (o2 >= 0 && o2 != j) {
                                if (j >= 0) single = false;
                                j = o2;
                            }
                        });
                        if (!single || j < 0 || rs[j].whole) continue;
                        const int t2 = home(j, s2, t1);
                        if (t2 < 0) continue;
                        unplace(j);
                        place(j, t2);
                        moves.push_back({j, t1});
                        unplace(i);
                        place(i, t1);
                        moves.push_back({i, s2});
                        done = true;
                    }
                    if (!done) {
                        ok = false;
                        break;
                    }
                }
                if (!ok) {
                    for (auto it = moves.rbegin(); it != moves.rend(); ++it) {
                        unplace(it->first);
                        place(it->first, it->second);
                    }
                    continue;
                }
                used--;
                progress = true;
            }
        }
        // renumber the slots in use densely (1 ..)
        std::vector<int> ren(NS1, 0);
        int n2 = 0;
        for (int s2 = 1; s2 < NS1; s2++)
            if (!of[s2].empty()) ren[s2] = ++n2;
        for (Res &R : rs) R.slot = ren[R.slot];
        used = n2;
    }
    o.slots = used + 1;
    o.residencies = (int)rs.size();
    if (o.slots > max_slots || o.slots > (int)LC_SLOT_MASK + 1) {
        const char *dbg = getenv("LDPC_LC_DEBUG");
        if (dbg && *dbg) {
            int whole = 0;
            for (const Res &R : rs) whole += R.whole;
            fprintf(stderr, "coop3 line cache: %d slots needed, %d available (max live %d + %d whole residencies)\n",
                    o.slots, max_slots, *std::max_element(live.begin(), live.end()), whole);
        }
        return lc_fail(__LINE__);
    }
    // residency holding line L at access period p (cyclic)
    auto res_id_at = [&](uint32_t L, int p) -> int {
        for (int id : res_of[L]) {
            const Res &R = rs[id];
            if (R.whole || cmod(p - R.f, nw) <= R.e - R.f) return id;
        }
        return -1;
    };
    // bank groups: a pre read (ds_read_b32) / post write (ds_write_b16) of info
    // entry j serves slab wave w's slots 8w + 4h .. 8w + 4h + 3 in one 32-lane
    // half h; a piece's bank group is its position in its 128-B slot (slots are
    // 32 dwords = the 32 banks those instructions use), so 4 distinct pieces
    // in one position cost 3 extra cycles.  Access = residency, row (-1: the
    // sink piece of an inactive slot)
    struct Acc {
        int res, row;
    };
    // two lanes per check (first-group degree >= 22, coop3_kernel.h G3::HALF):
    // instruction j of slab wave w serves slots 4w + 2h, 4w + 2h + 1 in 32-lane
    // half h, each with its info entries j (lane half 0) and XH + j (lane half 1)
    const int XH = D0 >= 22 ? ((X + 1) / 2 + 1) / 2 * 2 : 0;
    std::vector<std::vector<Acc>> groups;
    auto acc_of = [&](int u, int kk, int j, std::vector<Acc> &g) -> bool {
        const uint32_t *r = rec_at(u, kk);
        if (!(r[D0] & COOP_M_ACT) || j >= X) {
            g.push_back({-1, 0});
            return true;
        }
        const int id = res_id_at(r[j] / 8, cmod(u - 1, nw));
        if (id < 0) return false;
        g.push_back({id, (int)(r[j] % 8)});
        return true;
    };
    for (int u = 0; u < nw; u++) {
        if (XH > 0) {
            for (int w = 0; w < S / 4; w++)
                for (int hh = 0; hh < 2; hh++)
                    for (int j = 0; j < XH; j++) {
                        std::vector<Acc> g;
                        for (int i = 0; i < 2; i++)
                            if (!acc_of(u, 4 * w + 2 * hh + i, j, g) || !acc_of(u, 4 * w + 2 * hh + i, XH + j, g))
                                return lc_fail(__LINE__);
                        groups.push_back(g);
                    }
            continue;
        }
        for (int w = 0; w < S / 8; w++)
            for (int hh = 0; hh < 2; hh++)
                for (int j = 0; j < X; j++) {
                    std::vector<Acc> g;
                    for (int i = 0; i < 4; i++)
                        if (!acc_of(u, 8 * w + 4 * hh + i, j, g)) return lc_fail(__LINE__);
                    groups.push_back(g);
                }
    }
    auto pos_of = [&](const Acc &a) { return a.res < 0 ? 0 : (a.row ^ rs[a.res].z); };
    // extra LDS cycles of one group: the most distinct pieces in one position, minus 1
    auto extra = [&](const std::vector<Acc> &g) -> int {
        int cnt[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        for (size_t i = 0; i < g.size(); i++) {
            bool dup = false;
            for (size_t k2 = 0; k2 < i; k2++) dup |= g[k2].res == g[i].res && g[k2].row == g[i].row;
            if (!dup) cnt[pos_of(g[i])]++;
        }
        int mx = 0;
        for (int c : cnt) mx = std::max(mx, c);
        return mx - 1;
    };
    auto total = [&]() {
        long t = 0;
        for (const auto &g : groups) t += extra(g);
        return 2 * t;   // the pre read and the post write
    };
    o.bank_extra_plain = total();
    // local search over z: each residency takes the z that minimises the
    // extra cycles of its groups (pairwise same-position count as the
    // smoother objective), a few sweeps (LDPC_LC_SWIZZLE=0: z = 0)
    const char *sz = getenv("LDPC_LC_SWIZZLE");
    if (!(sz && *sz && atoi(sz) == 0)) {
        std::vector<std::vector<int>> gof(rs.size());
        for (int gi = 0; gi < (int)groups.size(); gi++)
            for (const Acc &a : groups[gi])
                if (a.res >= 0 && (gof[a.res].empty() || gof[a.res].back() != gi)) gof[a.res].push_back(gi);
        auto pairs = [&](const std::vector<Acc> &g) -> int {
            int c = 0;
            for (size_t i = 0; i < g.size(); i++)
                for (size_t k2 = 0; k2 < i; k2++)
                    if (!(g[k2].res == g[i].res && g[k2].row == g[i].row) && pos_of(g[k2]) == pos_of(g[i])) c++;
            return c;
        };
        for (int sweep = 0; sweep < 12; sweep++) {
            int changed = 0;
            for (int id = 0; id < (int)rs.size(); id++) {
                if (gof[id].empty()) continue;
                const int z0 = rs[id].z;
                int bz = z0, bc = 1 << 30;
                for (int z = 0; z < 8; z++) {
                    rs[id].z = (z0 + z) & 7;   // ties keep the current z
                    int c = 0;
                    for (int gi : gof[id]) c += 4 * extra(groups[gi]) + pairs(groups[gi]);
                    if (c < bc) {
                        bc = c;
                        bz = rs[id].z;
                    }
                }
                rs[id].z = bz;
                changed += bz != z0;
            }
            if (!changed) break;
        }
    }
    o.bank_extra = total();
    {
        const char *dbg = getenv("LDPC_LC_DEBUG");
        if (dbg && *dbg == '2')
            fprintf(stderr, "coop3 line cache: %d slots, %d residencies; modelled pre/post bank-conflict cycles per "
                            "iteration and workgroup: %ld (z = 0: %ld)\n", o.slots, o.residencies, o.bank_extra,
                    o.bank_extra_plain);
    }
    auto sfield = [&](const Res &R) { return (uint32_t)R.slot | (uint32_t)R.z << LC_SLOT_BITS; };
    // per-period op lists
    std::vector<std::vector<int>> lp(nw), wp(nw);
    for (int i = 0; i < (int)rs.size(); i++) {
        Res &R = rs[i];
        if (R.whole) continue;
        R.li = (int)lp[cmod(R.tl, nw)].size();
        lp[cmod(R.tl, nw)].push_back(i);
        if (R.dirty) {
            R.wi = (int)wp[cmod(R.tw, nw)].size();
            wp[cmod(R.tw, nw)].push_back(i);
        }
    }
    o.ops.assign((size_t)nw * LC_OPS * 2, 0);
    for (size_t i = 0; i < o.ops.size(); i += 2) {
        o.ops[i] = sink_line | sink_line << 16;   // load / writeback line: the sink
        o.ops[i + 1] = 0;                         // ds_write / writeback slot: the sink
    }
    for (const Res &R : rs) {
        if (R.whole) continue;
        uint32_t *ld = &o.ops[((size_t)cmod(R.tl, nw) * LC_OPS + R.li) * 2];
        ld[0] = (ld[0] & 0xFFFF0000u) | R.line;
        uint32_t *dw = &o.ops[((size_t)cmod(R.tl + LC_PUT, nw) * LC_OPS + R.li) * 2];
        dw[1] = (dw[1] & 0xFFFF0000u) | sfield(R);
        if (R.dirty) {
            uint32_t *wb = &o.ops[((size_t)cmod(R.tw, nw) * LC_OPS + R.wi) * 2];
            wb[0] = (wb[0] & 0xFFFFu) | R.line << 16;
            wb[1] = (wb[1] & 0xFFFFu) | sfield(R) << 16;
        }
    }
    auto res_at = [&](uint32_t L, int p) -> const Res * {
        const int id = res_id_at(L, p);
        return id < 0 ? nullptr : &rs[id];
    };
    o.piece.assign((size_t)nw * S * X, 0);
    for (int u = 0; u < nw; u++)
        for (int kk = 0; kk < S; kk++) {
            const uint32_t *r = rec_at(u, kk);
            if (!(r[D0] & COOP_M_ACT)) continue;   // sink slot 0, piece 0
            for (int j = 0; j < X; j++) {
                const Res *R = res_at(r[j] / 8, cmod(u - 1, nw));
                if (!R || R != res_at(r[j] / 8, cmod(u + 1, nw))) return lc_fail(__LINE__);
                o.piece[((size_t)u * S + kk) * X + j] = (uint32_t)R->slot * 128u + ((r[j] % 8) ^ (uint32_t)R->z) * 16u;
            }
        }
    // segment prologue / epilogue: holds across the iteration boundary
    for (const Res &R : rs) {
        const uint32_t w = (uint32_t)R.z << 26 | (uint32_t)R.slot << 16 | R.line;
        if (R.whole) {
            o.pro.push_back(w);
            if (R.dirty) o.epi.push_back(w);
        } else if (R.tl + LC_PUT <= -1 || R.tw >= nw) {
            o.pro.push_back(w);
            // dirty at a segment end: written before it (posts run up to period nw) and not yet written back
            if (R.dirty && R.tw >= nw + 1 && R.fw <= nw) o.epi.push_back(w);
        }
    }
    return lc_check_plan(o, tab, recw, nw, S, D0, n, k, 3);
}

// Replays `iters` iterations of the plan period by period, as the kernel runs
// a period (coop3_decode): the memory wave's slot writes (lines loaded LC_PUT
// periods earlier), then its writebacks (slot -> VGPRs -> HBM) and loads, all
// CONCURRENT with the slab waves' post of window p-1 and pre of window p+1 --
// only the period's closing barrier orders them.  So within one period a slot
// written must hold no line the post / pre touch, its new line must not be
// accessed before the next period, a slot is never both written and written
// back, and a writeback's line is not accessed.  Beyond that: every pre read /
// post write finds its line in the slot the record names, a slot is only
// refilled once its dirty line was written back in an earlier period, a line
// is loaded >= 3 periods after its last store and never while a dirty copy is
// resident, and the dirty lines left at the end are exactly the epilogue's.
int lc_check_plan(const LcPlan &o, const std::vector<uint32_t> &tab, int recw, int nw, int S, int D0, int n, int k,
                  int iters)
{
    const int LC_OPS = S * ((D0 - 2 + 7) / 8);
    const int X = D0 - 2;
    const uint32_t sink_line = (uint32_t)(n / 8);
    const int NSL = o.slots;
    std::vector<int> line_of(NSL, -1), z_of(NSL, 0);
    std::vector<char> dirty(NSL, 0);
    std::vector<long> last_store((size_t)k / 8, -1000000);
    std::vector<int> dirty_copies((size_t)k / 8, 0);
    auto fail = [&](const char *what, long P, int a, int b) {
        fprintf(stderr, "coop3 line cache plan check: %s (period %ld, %d, %d)\n", what, P, a, b);
        return -1;
    };
    for (uint32_t w : o.pro) {
        const int s = (int)((w >> 16) & LC_SLOT_MASK), L = (int)(w & 0xFFFFu);
        if (s <= 0 || s >= NSL || line_of[s] >= 0) return fail("prologue slot", -1, s, L);
        line_of[s] = L;
        z_of[s] = (int)(w >> 26) & 7;
    }
    auto rec_at = [&](int u, int kk) { return &tab[((size_t)u * S + kk) * recw]; };
    std::vector<long> put_at(NSL, -1000000);   // period of the slot's last write by the memory wave
    auto access = [&](int u, bool wr, long P) -> int {   // window u's info entries
        u = cmod(u, nw);
        for (int kk = 0; kk < S; kk++) {
            const uint32_t *r = rec_at(u, kk);
            if (!(r[D0] & COOP_M_ACT)) continue;
            for (int j = 0; j < X; j++) {
                const uint32_t off = o.piece[((size_t)u * S + kk) * X + j];
                const int s = (int)(off / 128);
                if (s <= 0 || s >= NSL || off % 128 != ((r[j] % 8) ^ (uint32_t)z_of[s]) * 16 ||
                    line_of[s] != (int)(r[j] / 8))
                    return fail(wr ? "post finds another line" : "pre finds another line", P, s, (int)r[j]);
                if (put_at[s] == P)
                    return fail(wr ? "post of a line written to its slot this period"
                                   : "pre of a line written to its slot this period", P, s, (int)r[j]);
                if (wr && !dirty[s]) {
                    dirty[s] = 1;
                    dirty_copies[r[j] / 8]++;
                }
            }
        }
        return 0;
    };
    const long G = (long)nw * iters;
    constexpr int NPD = LC_PUT + 1;
    std::vector<uint32_t> pend((size_t)NPD * LC_OPS, sink_line);   // loads of periods P-LC_PUT .. P
    if (access(0, false, -1)) return -1;                           // the pre of window 0 before period 0
    for (long P = 0; P <= G; P++) {
        const int p = (int)(P % nw);
        const uint32_t *ops = &o.ops[(size_t)p * LC_OPS * 2];
        std::vector<char> touched((size_t)k / 8, 0);
        auto touch = [&](int u) {
            u = cmod(u, nw);
            for (int kk = 0; kk < S; kk++) {
                const uint32_t *r = rec_at(u, kk);
                if (r[D0] & COOP_M_ACT)
                    for (int j = 0; j < X; j++) touched[r[j] / 8] = 1;
            }
        };
        if (P >= 1) touch(p - 1);
        if (P + 1 < G) touch(p + 1);
        // LDS slots the post / pre of this period read or write
        std::vector<char> used_slot(NSL, 0);
        auto use = [&](int u) {
            u = cmod(u, nw);
            for (int kk = 0; kk < S; kk++)
                if (rec_at(u, kk)[D0] & COOP_M_ACT)
                    for (int j = 0; j < X; j++) {
                        const uint32_t s = o.piece[((size_t)u * S + kk) * X + j] / 128;
                        if (s < (uint32_t)NSL) used_slot[s] = 1;
                    }
        };
        if (P >= 1) use(p - 1);
        if (P + 1 < G) use(p + 1);
        std::vector<char> wb_slot(NSL, 0);
        for (int i = 0; i < LC_OPS; i++)
            if ((ops[2 * i] >> 16) != sink_line) {
                const int s = (int)((ops[2 * i + 1] >> 16) & LC_SLOT_MASK);
                if (s > 0 && s < NSL) wb_slot[s] = 1;
            }
        // slot writes of the loads of period P - LC_PUT (first in the memory wave's period)
        for (int i = 0; i < LC_OPS; i++) {
            const int s = (int)(ops[2 * i + 1] & LC_SLOT_MASK);
            const uint32_t L = pend[(size_t)((P + 1) % NPD) * LC_OPS + i];   // the load of period P - LC_PUT
            if (s == 0) {
                if (L != sink_line && P >= LC_PUT) return fail("load without a slot", P, s, (int)L);
                continue;
            }
            if (L == sink_line) return fail("slot write without a load", P, s, (int)L);
            if (s >= NSL || dirty[s]) return fail("slot refilled before its writeback", P, s, line_of[s]);
            if (put_at[s] == P) return fail("slot written twice in one period", P, s, (int)L);
            if (wb_slot[s]) return fail("slot written and written back in one period", P, s, (int)L);
            if (used_slot[s]) return fail("slot refilled in a period whose post / pre access it", P, s, line_of[s]);
            line_of[s] = (int)L;
            z_of[s] = (int)((ops[2 * i + 1] & 0xFFFFu) >> LC_SLOT_BITS);
            put_at[s] = P;
        }
        // writebacks (concurrent with the post / pre below)
        for (int i = 0; i < LC_OPS; i++) {
            const uint32_t L = ops[2 * i] >> 16;
            const int s = (int)((ops[2 * i + 1] >> 16) & LC_SLOT_MASK);
            if (L == sink_line) continue;
            if (L >= (uint32_t)k / 8 || s <= 0 || s >= NSL || line_of[s] != (int)L ||
                (int)(ops[2 * i + 1] >> (16 + LC_SLOT_BITS)) != z_of[s])
                return fail("writeback of a line not in its slot (or with another swizzle)", P, s, (int)L);
            if (touched[L]) return fail("writeback in a period accessing the line", P, s, (int)L);
            if (dirty[s]) dirty_copies[L]--;
            dirty[s] = 0;
            last_store[L] = P;
        }
        // post of window p-1, pre of window p+1
        if (P >= 1 && access(p - 1, true, P)) return -1;
        if (P + 1 < G && access(p + 1, false, P)) return -1;
        // loads
        for (int i = 0; i < LC_OPS; i++) {
            const uint32_t L = ops[2 * i] & 0xFFFFu;
            pend[(size_t)(P % NPD) * LC_OPS + i] = L;
            if (L == sink_line) continue;
            if (L >= (uint32_t)k / 8) return fail("load of a bad line", P, i, (int)L);
            if (dirty_copies[L] != 0) return fail("load while a dirty copy is resident", P, i, (int)L);
            if (P - last_store[L] < 3) return fail("load too soon after the line's store", P, i, (int)L);
        }
    }
    // what is left dirty must be the epilogue
    std::vector<uint32_t> left;
    for (int s = 1; s < NSL; s++)
        if (dirty[s]) left.push_back((uint32_t)z_of[s] << 26 | (uint32_t)s << 16 | (uint32_t)line_of[s]);
    std::vector<uint32_t> epi = o.epi;
    std::sort(left.begin(), left.end());
    std::sort(epi.begin(), epi.end());
    if (left != epi) return fail("dirty lines at the end != epilogue", G, (int)left.size(), (int)epi.size());
    return 0;
}
