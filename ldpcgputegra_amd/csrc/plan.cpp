// plan.cpp -- static analysis of the layered schedule (host, once per code).
//
// The reference processes checks strictly in table order
// (code/x86/CDecoder/OMS/CDecoder_OMS_fixed_SSE.cpp:172,262,334,...): every
// check sees the V values left by all earlier checks.  To run many checks of
// one codeword in parallel and stay bit-exact we need to know which checks
// touch a variable that an earlier, not-yet-finished check writes:
//
//  * chain links: check i+1 shares exactly one variable with check i (the
//    DVB-S2 parity staircase: check i writes K+i, check i+1 reads it).  The
//    kernel forwards that value in registers, in schedule order.
//  * hazards: any other variable shared by two checks at cyclic schedule
//    distance < min_hazard.  The windowed kernel needs
//    min_hazard >= kMinHazardWindowed (see decode.hip).
#include <algorithm>
#include <unordered_map>

#include "ldpc_internal.h"

static constexpr int kPlanSlots = 16;   // checks per window (lanes per codeword)

// Windows for windowed2.hip: greedy runs of <= S consecutive checks of one
// degree group such that (1) only slot 0 may lack a chain input, (2) inside
// a window only the chain link shares a variable, and (3) no variable read by
// window u (chain input excepted) was written by windows u-P..u-1 of the same
// group (the kernel loads window u's V before those windows store).
int ldpc_plan_windows(const ldpc_code *h, int S, int P, std::vector<ldpc_window> &out)
{
    out.clear();
    if (!h->staircase) return LDPC_OK;
    std::vector<int> writer(h->n, -1);        // last window index writing the variable
    std::vector<int> in_win(h->n, -1);        // window index that touched it (this window)
    int gstart = 0;
    int c = 0;
    while (c < h->m) {
        const int u = (int)out.size();
        const int g = h->check_group[c];
        if (u > 0 && h->check_group[out.back().first] != g) gstart = u;
        int cnt = 0;
        while (c + cnt < h->m && cnt < S) {
            const int ci = c + cnt;
            if (h->check_group[ci] != g) break;
            if (cnt > 0 && h->chain_in[ci] < 0) break;          // chain break: start a new window
            const uint32_t *ev = &h->edge_var[h->check_start[ci]];
            bool ok = true;
            for (int j = 0; j < h->check_deg[ci] && ok; j++) {
                // the chain input arrives in registers from check ci-1 (the
                // previous slot, or the carry of the previous window)
                if (h->chain_in[ci] == j) continue;
                if (in_win[ev[j]] == u) ok = false;               // shared inside the window
                const int lw = writer[ev[j]];
                if (lw >= gstart && lw >= u - P) ok = false;      // written by the read-ahead span
            }
            if (!ok) {
                if (cnt == 0) {   // hazards too short for this read-ahead: no windowed schedule
                    out.clear();
                    return LDPC_OK;
                }
                break;
            }
            for (int j = 0; j < h->check_deg[ci]; j++) in_win[ev[j]] = u;
            cnt++;
        }
        for (int k = 0; k < cnt; k++) {
            const uint32_t *ev = &h->edge_var[h->check_start[c + k]];
            for (int j = 0; j < h->check_deg[c + k]; j++) writer[ev[j]] = u;
        }
        out.push_back({c, cnt});
        c += cnt;
    }
    return LDPC_OK;
}

int ldpc_plan_build(ldpc_code *h)
{
    const int m = h->m;
    h->chain_in.assign(m, -1);
    h->chain_out.assign(m, -1);
    h->windows.clear();
    h->win_slots = 0;

    // --- chain links between cyclically consecutive checks
    bool stair = (m > 1);
    int links = 0;
    for (int i = 0; i < m; i++) {
        const int nx = (i + 1) % m;
        const uint32_t *a = &h->edge_var[h->check_start[i]];
        const uint32_t *b = &h->edge_var[h->check_start[nx]];
        const int da = h->check_deg[i], db = h->check_deg[nx];
        int shared = 0, sa = -1, sb = -1;
        for (int x = 0; x < da; x++)
            for (int y = 0; y < db; y++)
                if (a[x] == b[y]) {
                    shared++;
                    sa = x;
                    sb = y;
                }
        if (shared == 0) continue;
        if (shared > 1 || sa != da - 1 || sb != db - 2) {
            stair = false;
            continue;
        }
        h->chain_out[i] = (int8_t)sa;
        h->chain_in[nx] = (int8_t)sb;
        links++;
    }
    h->staircase = stair && links > 0;
    if (!h->staircase) {
        std::fill(h->chain_in.begin(), h->chain_in.end(), (int8_t)-1);
        std::fill(h->chain_out.begin(), h->chain_out.end(), (int8_t)-1);
    }

    // --- hazard distance (two passes over the cyclic schedule)
    std::vector<int> last(h->n, -1);
    int min_hz = 1 << 30;
    for (int pass = 0; pass < 2; pass++)
        for (int i = 0; i < m; i++) {
            const uint32_t *ev = &h->edge_var[h->check_start[i]];
            for (int j = 0; j < h->check_deg[i]; j++) {
                const uint32_t v = ev[j];
                if (pass == 1 && last[v] >= 0 && last[v] != i) {
                    int d = i - last[v];
                    if (d <= 0) d += m;
                    const bool chain = (h->chain_in[i] == j);   // value arrives via the chain
                    if (!chain) min_hz = std::min(min_hz, d);
                }
                last[v] = i;
            }
        }
    h->min_hazard = (min_hz == (1 << 30)) ? m : min_hz;

    // --- windows: consecutive runs of <= kPlanSlots checks of one degree group
    extern bool windowed_kernel_available();
    if (h->staircase && windowed_kernel_available()) {
        h->win_slots = kPlanSlots;
        int c = 0;
        while (c < m) {
            int g = h->check_group[c], cnt = 0;
            while (c + cnt < m && cnt < kPlanSlots && h->check_group[c + cnt] == g) cnt++;
            h->windows.push_back({c, cnt});
            c += cnt;
        }
        // Verify the windowed kernel's read-ahead (windowed.hip): inside one
        // degree group the V of window u is loaded before windows u-1 and u-2
        // store, and all checks of a window read V before any of them stores.
        // So a variable read by window u (chain-in edges excepted: their value
        // arrives through the chain) must not be written by windows u-2..u.
        // Group boundaries drain the pipeline.
        constexpr int kLookahead = 2;
        std::vector<int> writer_win(h->n, -1);   // last window (this group pass) writing var
        bool ok = true;
        int gstart = 0;
        for (int wi = 0; wi < (int)h->windows.size() && ok; wi++) {
            const ldpc_window &win = h->windows[wi];
            if (wi > 0 && h->check_group[win.first] != h->check_group[h->windows[wi - 1].first]) gstart = wi;
            for (int k = 0; k < win.count && ok; k++) {
                const int ci = win.first + k;
                const uint32_t *ev = &h->edge_var[h->check_start[ci]];
                for (int j = 0; j < h->check_deg[ci]; j++) {
                    if (h->chain_in[ci] == j) continue;
                    const int lw = writer_win[ev[j]];
                    if (lw >= gstart && wi - lw <= kLookahead) ok = false;
                }
            }
            // inside a window only the chain link may share a variable
            std::unordered_map<uint32_t, int> seen;
            for (int k = 0; k < win.count && ok; k++) {
                const int ci = win.first + k;
                const uint32_t *ev = &h->edge_var[h->check_start[ci]];
                for (int j = 0; j < h->check_deg[ci]; j++) {
                    auto it = seen.find(ev[j]);
                    if (it != seen.end() && !(it->second == k - 1 && h->chain_in[ci] == j)) ok = false;
                    seen[ev[j]] = k;
                }
            }
            for (int k = 0; k < win.count; k++) {
                const int ci = win.first + k;
                const uint32_t *ev = &h->edge_var[h->check_start[ci]];
                for (int j = 0; j < h->check_deg[ci]; j++) writer_win[ev[j]] = wi;
            }
        }
        if (!ok) h->windows.clear();
    }
    return LDPC_OK;
}
