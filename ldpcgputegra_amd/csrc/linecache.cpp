// linecache.cpp -- host planner of coop3's LDS line cache.
//
// coop3 keeps V (the per-variable LLRs of a workgroup's 16 codewords) in the
// grouped layout V[group][n + 1][16] (DecodeLaunch::vpriv) and, with the line
// cache, moves it between HBM and the workgroup's LDS in whole 128-B lines (8
// consecutive variables x 16 codewords) instead of one scattered 16-B piece
// per edge and check.  DVB-S2 makes this work: information bit m of a 360-bit
// group is touched by checks x + m q (ETSI EN 302 307 Annex B; the reference's
// tables, code/x86/Constantes/64800x32400.dvb-s2/constantes_sse.h), so the
// layered schedule walks each of a group's addresses through consecutive bits,
// one bit per q = 90 checks (two coop3 windows): a line serves 8 consecutive
// uses of each address, and ~600 lines (~75 KB) are live at a time.
//
// The plan is static (per code, from the coop3 window schedule), periodic with
// the nw windows of one iteration, and self-checked by replaying it:
//   * window u's pre reads its records' entries 0..X-1 and D0-1 in period
//     u - 1, its post writes entries 0..X (the tail also D0-1) in period u + 1;
//   * a line instance (its accesses, split where two are >= LC_GAP periods
//     apart) is loaded straight into its cache slot (LDS-DMA) in period f - 2
//     (f = first access; the loading wave waits for it at the end of period
//     f - 1), so the slot is held from period f - 2; if written to, it is
//     written back (slot -> VGPRs -> global) in period e + 1 (e = last
//     access); the slot is free again from the next period;
//   * a line written back is loaded again >= 2 periods after its store (the
//     store and the load come from the same CU, in order);
//   * at most LC_LMAX loads and LC_LMAX writebacks per period (6 slab waves x 8
//     lines); list entry i goes to slab wave i % 6, lane group i / 6;
//   * slot 0 holds the sink line (row n: the inactive slots' reads and
//     writes), never loaded or written back.
#include <algorithm>
#include <cstdint>
#include <vector>

#include "coop.h"

namespace {

struct Inst {
    uint32_t line;
    int f, e;            // first / last access period (e >= f; f in [0, nw), e may exceed nw: wraps)
    bool dirty, whole;   // written to; resident for the whole iteration
    int tl, tw, te;      // load issue, slot write, last period the slot is held (cyclic, unrolled from f)
    int slot = -1;
};

inline int cmod(int a, int m) { return ((a % m) + m) % m; }

}  // namespace

int lc_build_plan(const std::vector<uint32_t> &tab, int recw, int nw, int S, int D0, int tail, int n, int max_slots,
                  LcPlan &o)
{
    o = LcPlan{};
    const int X = D0 - 2;
    if (nw < 2 * LC_GAP || n <= 0 || max_slots < 2) return -1;
    const uint32_t nlines = (uint32_t)(n / 8) + 1;   // + the sink row's line
    const uint32_t sink_line = (uint32_t)(n / 8);
    if (n % 8 != 0 || nlines >= (1u << 16)) return -1;   // the sink row n alone in its line; 16-bit line index
    // accesses per line: (period mod nw) << 1 | write
    std::vector<std::vector<uint32_t>> acc(nlines);
    auto rec_at = [&](int u, int k) { return &tab[((size_t)u * S + k) * recw]; };
    auto add = [&](uint32_t v, int per, bool wr) {
        acc[v / 8].push_back((uint32_t)cmod(per, nw) << 1 | (wr ? 1u : 0u));
    };
    for (int u = 0; u < nw; u++)
        for (int k = 0; k < S; k++) {
            const uint32_t *r = rec_at(u, k);
            if (!(r[D0] & COOP_M_ACT)) continue;
            for (int j = 0; j < X; j++) add(r[j], u - 1, false);
            add(r[D0 - 1], u - 1, false);
            for (int j = 0; j <= X; j++) add(r[j], u + 1, true);
            if (u == tail) add(r[D0 - 1], u + 1, true);
        }
    if (!acc[sink_line].empty()) return -1;
    // instances
    std::vector<Inst> in;
    std::vector<std::vector<std::pair<int, int>>> inst_of(nlines);   // per line: (access period, instance)
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
        if (cut.empty()) {   // resident for the whole iteration
            Inst I{L, per[0], per[0] + nw - 1, false, true, 0, 0, 0};
            for (int i = 0; i < m; i++) I.dirty |= wr[i] != 0;
            const int id = (int)in.size();
            in.push_back(I);
            for (int i = 0; i < m; i++) inst_of[L].push_back({per[i], id});
            continue;
        }
        for (size_t c = 0; c < cut.size(); c++) {
            const int s = (cut[c] + 1) % m;   // first access of the instance
            const int t = cut[(c + 1) % cut.size()];
            Inst I{L, per[s], 0, false, false, 0, 0, 0};
            const int id = (int)in.size();
            for (int i = s;; i = (i + 1) % m) {
                I.dirty |= wr[i] != 0;
                inst_of[L].push_back({per[i], id});
                I.e = per[i] >= I.f ? per[i] : per[i] + nw;
                if (i == t) break;
            }
            in.push_back(I);
        }
    }
    for (Inst &I : in) {
        if (I.whole) continue;
        I.tl = I.f - 2;
        I.tw = I.f - 2;
        I.te = I.dirty ? I.e + 1 : I.e;   // the writeback's slot read is in period e + 1
    }
    // per-period capacity: move loads earlier / writebacks later where a period
    // is over LC_LMAX (keeping the store -> reload distance of the line)
    auto prev_of = [&](int id) -> const Inst * {   // the line's previous instance (cyclic), or null
        const Inst &I = in[id];
        const Inst *best = nullptr;
        int bestd = 1 << 30;
        for (auto &pr : inst_of[I.line]) {
            const Inst &J = in[pr.second];
            if (pr.second == id || J.whole) continue;
            const int d = cmod(I.f - J.f, nw);
            if (d > 0 && d < bestd) {
                bestd = d;
                best = &J;
            }
        }
        return best;
    };
    for (int round = 0; round < 64; round++) {
        std::vector<std::vector<int>> lp(nw), wp(nw);
        for (int i = 0; i < (int)in.size(); i++) {
            if (in[i].whole) continue;
            lp[cmod(in[i].tl, nw)].push_back(i);
            if (in[i].dirty) wp[cmod(in[i].te, nw)].push_back(i);
        }
        bool moved = false, stuck = false;
        for (int p = 0; p < nw; p++) {
            while ((int)lp[p].size() > LC_LMAX) {
                bool ok = false;
                for (size_t j = 0; j < lp[p].size() && !ok; j++) {
                    Inst &I = in[lp[p][j]];
                    const Inst *P = prev_of(lp[p][j]);
                    // store of P at P.te (period e_P + 1) -> this load >= 2 periods later
                    const int pe = P ? (P->dirty ? P->te : P->e) : 0;
                    const int dist = P ? cmod(I.tl - 1 - pe, nw) : nw;
                    if (P && (dist < 2 || cmod(I.tl - 1 - P->tw, nw) < cmod(pe - P->tw, nw))) continue;
                    I.tl--;
                    I.tw--;
                    lp[p].erase(lp[p].begin() + (long)j);
                    ok = moved = true;
                }
                if (!ok) {
                    stuck = true;
                    break;
                }
            }
            while ((int)wp[p].size() > LC_LMAX) {
                bool ok = false;
                for (size_t j = 0; j < wp[p].size() && !ok; j++) {
                    const int id = wp[p][j];
                    Inst &I = in[id];
                    // the next instance of the line must still load >= 2 periods after the store
                    bool safe = true;
                    for (auto &pr : inst_of[I.line]) {
                        const Inst &J = in[pr.second];
                        if (pr.second == id || J.whole) continue;
                        if (prev_of(pr.second) == &I && cmod(J.tl - (I.te + 1), nw) < 2) safe = false;
                    }
                    if (!safe) continue;
                    I.te++;
                    wp[p].erase(wp[p].begin() + (long)j);
                    ok = moved = true;
                }
                if (!ok) {
                    stuck = true;
                    break;
                }
            }
        }
        if (stuck) return -1;
        if (!moved) break;
        if (round == 63) return -1;
    }
    // slot assignment: occupancy bitsets over the nw periods, first fit; the
    // whole-iteration lines first, then by slot-write period
    const int words = (nw + 63) / 64;
    std::vector<uint64_t> occ;   // [slot][words]
    auto span = [&](int a, int b, std::vector<uint64_t> &m) {   // cyclic [a, b], b - a < nw
        m.assign(words, 0);
        for (int p = a; p <= b; p++) {
            const int q = cmod(p, nw);
            m[q >> 6] |= 1ull << (q & 63);
        }
    };
    std::vector<int> order((size_t)in.size());
    for (size_t i = 0; i < in.size(); i++) order[i] = (int)i;
    std::stable_sort(order.begin(), order.end(), [&](int a, int b) {
        if (in[a].whole != in[b].whole) return in[a].whole;
        return cmod(in[a].tw, nw) < cmod(in[b].tw, nw);
    });
    occ.assign((size_t)words, ~0ull);   // slot 0: the sink line
    int nslots = 1;
    std::vector<uint64_t> m;
    for (int id : order) {
        Inst &I = in[id];
        if (I.whole)
            m.assign(words, ~0ull);
        else
            span(I.tw, I.te, m);
        int s = 1;
        for (; s < nslots; s++) {
            bool fit = true;
            for (int w = 0; w < words && fit; w++) fit = (occ[(size_t)s * words + w] & m[w]) == 0;
            if (fit) break;
        }
        if (s == nslots) {
            if (nslots >= max_slots) return -1;
            occ.resize((size_t)(nslots + 1) * words, 0);
            nslots++;
        }
        for (int w = 0; w < words; w++) occ[(size_t)s * words + w] |= m[w];
        I.slot = s;
    }
    // tables
    o.slots = nslots;
    o.rowoff.assign((size_t)nw * S * 8, 0);
    auto inst_at = [&](uint32_t v, int per) -> const Inst * {
        const int p = cmod(per, nw);
        for (auto &pr : inst_of[v / 8])
            if (pr.first == p) return &in[pr.second];
        return nullptr;
    };
    for (int u = 0; u < nw; u++)
        for (int k = 0; k < S; k++) {
            const uint32_t *r = rec_at(u, k);
            uint16_t *ro = &o.rowoff[((size_t)u * S + k) * 8];
            const bool act = (r[D0] & COOP_M_ACT) != 0;
            for (int j = 0; j < D0; j++) {
                if (!act) {
                    ro[j] = (uint16_t)(n % 8);   // slot 0, the sink row
                    continue;
                }
                const bool rd = j < X || j == D0 - 1;
                const Inst *I = inst_at(r[j], rd ? u - 1 : u + 1);
                if (!I) return -1;
                ro[j] = (uint16_t)(I->slot * 8 + (int)(r[j] % 8));
            }
        }
    o.loads.assign((size_t)nw * LC_LMAX, LC_NONE);
    o.wbs.assign((size_t)nw * LC_LMAX, LC_NONE);
    std::vector<int> nl(nw, 0), nb(nw, 0);
    auto code = [](const Inst &I) { return I.line | (uint32_t)I.slot << 16; };
    for (const Inst &I : in) {
        if (I.whole) continue;
        const int p = cmod(I.tl, nw);
        o.loads[(size_t)p * LC_LMAX + nl[p]++] = code(I);
        if (I.dirty) {
            const int q = cmod(I.te, nw);
            o.wbs[(size_t)q * LC_LMAX + nb[q]++] = code(I);
        }
    }
    // prologue: resident during period -1 (slot written at or before it, held
    // past it); epilogue: dirty and resident after the last period (G = 0 mod nw)
    auto covers = [&](const Inst &I, int p) {   // cyclic p in [tw, te]
        return I.whole || cmod(p - I.tw, nw) <= I.te - I.tw;
    };
    for (const Inst &I : in) {
        if (covers(I, -1)) o.pro.push_back(code(I));
        if (I.dirty && (I.whole || (covers(I, 0) && cmod(I.te, nw) != 0))) o.epi.push_back(code(I));
    }
    int mx_l = 0, mx_b = 0;
    for (int p = 0; p < nw; p++) {
        mx_l = std::max(mx_l, nl[p]);
        mx_b = std::max(mx_b, nb[p]);
    }
    o.max_loads = mx_l;
    o.max_wbs = mx_b;
    o.instances = (int)in.size();
    return lc_check_plan(tab, recw, nw, S, D0, tail, n, o);
}

// Replays the plan over three iterations (the kernel's timeline from the
// prologue on) with a model of the cache: every access must find its line in
// the slot the record names, slots are loaded only when free, lines are
// loaded >= 2 periods after their previous writeback, and at the end of every
// iteration the epilogue leaves every dirty line written back.  A load of
// period p may land at any time in periods p and p + 1, so the model puts the
// new line in its slot at the start of period p (an access to the slot's old
// line in period p or later fails).  0 = valid.
int lc_check_plan(const std::vector<uint32_t> &tab, int recw, int nw, int S, int D0, int tail, int n, const LcPlan &o)
{
    const int X = D0 - 2, NS = o.slots;
    const uint32_t sink_line = (uint32_t)(n / 8);
    std::vector<int64_t> holds(NS, -1);        // line held by the slot (-1: free)
    std::vector<char> dirty(NS, 0);
    std::vector<int> last_store((size_t)(n / 8) + 1, -100000);
    holds[0] = sink_line;
    auto line_of = [](uint32_t c) { return c & 0xFFFFu; };
    auto slot_of = [](uint32_t c) { return (int)(c >> 16); };
    for (uint32_t c : o.pro) {
        if (slot_of(c) <= 0 || slot_of(c) >= NS || holds[slot_of(c)] != -1) return -2;
        holds[slot_of(c)] = line_of(c);
    }
    auto rec_at = [&](int u, int k) { return &tab[((size_t)u * S + k) * recw]; };
    auto access = [&](int u, int k, int j, bool wr) -> bool {
        const uint32_t *r = rec_at(cmod(u, nw), k);
        const int row = o.rowoff[((size_t)cmod(u, nw) * S + k) * 8 + j];
        const int s = row / 8;
        if (!(r[D0] & COOP_M_ACT)) return s == 0 && row % 8 == n % 8;
        if (s <= 0 || s >= NS || holds[s] != (int64_t)(r[j] / 8) || row % 8 != (int)(r[j] % 8)) return false;
        if (wr) dirty[s] = 1;
        return true;
    };
    const int G = 3 * nw;
    // period -1: pre of window 0
    for (int k = 0; k < S; k++) {
        for (int j = 0; j < X; j++)
            if (!access(0, k, j, false)) return -3;
        if (!access(0, k, D0 - 1, false)) return -3;
    }
    for (int p = 0; p <= G; p++) {
        const int pm = cmod(p, nw);
        // (I) the loads of period p claim their slots
        for (int i = 0; i < LC_LMAX; i++) {
            const uint32_t c = o.loads[(size_t)pm * LC_LMAX + i];
            if (c == LC_NONE) continue;
            const int s = slot_of(c);
            if (s <= 0 || s >= NS) return -6;
            if (holds[s] != -1 && dirty[s]) return -6;        // would overwrite unsaved data
            if (p - last_store[line_of(c)] < 2) return -8;   // its last writeback too recent
            for (int t = 1; t < NS; t++)                     // a dirty copy still cached: the load is stale
                if (holds[t] == (int64_t)line_of(c) && dirty[t]) return -11;
            holds[s] = line_of(c);
            dirty[s] = 0;
        }
        // (A, D) writebacks: slot read, store (its line must be the one held)
        for (int i = 0; i < LC_LMAX; i++) {
            const uint32_t c = o.wbs[(size_t)pm * LC_LMAX + i];
            if (c == LC_NONE) continue;
            const int s = slot_of(c);
            if (s <= 0 || s >= NS || holds[s] != (int64_t)line_of(c)) return -4;
            last_store[line_of(c)] = p;
            holds[s] = -1;
            dirty[s] = 0;
        }
        // (C) post of window p-1
        if (p >= 1)
            for (int k = 0; k < S; k++) {
                for (int j = 0; j <= X; j++)
                    if (!access(p - 1, k, j, true)) return -5;
                if (cmod(p - 1, nw) == tail && !access(p - 1, k, D0 - 1, true)) return -5;
            }
        // (slots whose instance ended without a writeback, clean, are taken
        // over by the next load into them)
        // (G) pre of window p+1
        if (p + 1 < G)
            for (int k = 0; k < S; k++) {
                for (int j = 0; j < X; j++)
                    if (!access(p + 1, k, j, false)) return -7;
                if (!access(p + 1, k, D0 - 1, false)) return -7;
            }
    }
    // epilogue: every dirty slot must be in the list
    std::vector<char> flushed(NS, 0);
    for (uint32_t c : o.epi) {
        const int s = slot_of(c);
        if (s <= 0 || s >= NS || holds[s] != (int64_t)line_of(c)) return -9;
        flushed[s] = 1;
    }
    for (int s = 1; s < NS; s++)
        if (dirty[s] && !flushed[s]) return -10;
    return 0;
}
