// windowed.hip -- layered int8 min-sum for staircase (DVB-S2 IRA) codes.
//
// The reference walks every check of a codeword in schedule order
// (code/x86/CDecoder/OMS/CDecoder_OMS_fixed_SSE.cpp:172-546).  Running one
// codeword per lane (generic.hip) leaves 4096 codewords = 64 waves for 1024
// SIMDs.  This kernel puts S = 16 consecutive checks of a codeword on the 16
// lanes of a DPP row (G = 4 codewords per wave) and splits every check into
//
//   pre   (parallel over the 16 checks): gather V, decode the old compressed
//         message, c_j = V - m_j, min1/min2/sign over all edges except the
//         chain-in edge x;
//   chain (serial, DPP row_shr:1 steps): the only dependency between
//         consecutive checks of a window is the staircase parity variable
//         (check i writes it as its last edge o = D-1, check i+1 reads it as
//         its edge x = D-2); step k turns lane k-1's new value into lane k's
//         new value for o in ~12 VALU ops;
//   post  (parallel): new messages and V for every edge.
//
// Bit-exactness: the value check i writes to o is cst(min_{j != o} a_j) with
// the sign of the other edges -- exactly what the reference's
// (a_o == min1 ? cst(min2) : cst(min1)) selects (ties give min1 == min2).
// V of non-chain variables is read P windows ahead; plan.cpp proves no
// variable read by window u is written by windows u-P..u-1 (min hazard
// distance 51-62 checks for the DVB-S2 tables).
//
// Messages are compressed per check, bit-exactly: cst1 | cst2 << 7 |
// jmin << 14 | sign_j << (19 + j): the message of edge j is
// (j == jmin ? cst1 : cst2) with sign_j -- the reference's CMOV selection
// (CDecoder_OMS_fixed_SSE.cpp:239-244; ties have cst1 == cst2).  4 bytes per
// check (D <= 13) instead of D bytes per check.
//
// Layout: V[N][stride] int8 (codeword fastest), Mc[check][stride] u32.
#include "windowed.h"

#include <algorithm>
#include <vector>

namespace {

constexpr int S = 16;   // checks per window = lanes per DPP row
constexpr int G = 4;    // codewords per wave
// prefetch distance: 2 windows (run_group; plan.cpp verifies the hazards)

// per-slot flags (plan.cpp)
constexpr int F_ACT = 1, F_XIN = 2, F_ODEAD = 4;

struct WinArgs {
    int8_t *V;
    uint32_t *Mc;
    int stride;
    int iters;
    const uint32_t *slotvar;   // per window: [D][S] variable index
    const uint32_t *slotoff;   // [n_windows] offset of the window's block in slotvar
    const uint8_t *flags;      // [n_windows][S]
    const int *win_first;      // [n_windows] first check of the window
    const int *win_cnt;        // [n_windows] checks in the window (<= S)
    int g0_end;                // windows [0, g0_end) are group 0, [g0_end, n_windows) group 1
    int n_windows;
    int param, var_min, msg_max, early;
    int32_t *iters_used;
};

LDPC_DEV int dpp_shr1(int old, int v)
{
    // row_shr:1 -- lane k of each 16-lane row receives lane k-1; lane 0 keeps `old`
    return __builtin_amdgcn_update_dpp(old, v, 0x111, 0xF, 0xF, false);
}

template <int ALGO>
LDPC_DEV int cst_of(int mn, int param, int msg_max)
{
    if constexpr (ALGO == 1)
        return nms_scale(mn, param);
    else
        return min(max(mn - param, 0), msg_max);   // == min(as_i8(subs_u8(mn, off)), msg_max), mn in [0,127]
}

template <int D>
struct Tab {
    uint32_t var[D];
};

template <int D>
struct Buf {
    int v[D];
    uint32_t addr[D];   // byte offset of V[var][b]
    uint32_t m;
};

template <int D>
LDPC_DEV void load_tab(Tab<D> &t, const WinArgs &a, int w, int slot)
{
    const uint32_t *p = a.slotvar + a.slotoff[w] + slot;
#pragma unroll
    for (int j = 0; j < D; j++) t.var[j] = p[j * S];
}

template <int D>
LDPC_DEV void load_buf(Buf<D> &bf, const Tab<D> &t, const WinArgs &a, int w, int slot, int b)
{
    const bool act = a.flags[w * S + slot] & F_ACT;
#pragma unroll
    for (int j = 0; j < D; j++) bf.addr[j] = t.var[j] * (uint32_t)a.stride + (uint32_t)b;
    if (act) {
#pragma unroll
        for (int j = 0; j < D; j++) bf.v[j] = a.V[bf.addr[j]];
        bf.m = a.Mc[(size_t)(a.win_first[w] + slot) * a.stride + b];
    } else {
#pragma unroll
        for (int j = 0; j < D; j++) bf.v[j] = 0;
        bf.m = 0;
    }
}

// One window: pre, chain, post.  `carry` = the row's chain value (new V of
// the previous check's o edge); returns the updated carry.
template <int D, int ALGO, bool LATER>
LDPC_DEV int do_window(const Buf<D> &bf, const WinArgs &a, int w, int slot, int b, int carry, bool live)
{
    constexpr int X = D - 2, O = D - 1;
    // the later-group |min(c, max_msg)| quirk is OMS-only
    constexpr bool LQ = LATER && (ALGO != 1);
    const int cnt = a.win_cnt[w];
    const int fl = a.flags[w * S + slot];
    const bool act = (fl & F_ACT) && live;
    const bool has_x = fl & F_XIN;
    const int vmin = a.var_min, mm = a.msg_max, prm = a.param;

    // ---- decode the old messages
    const uint32_t word = bf.m;
    const int c1o = (int)(word & 127), c2o = (int)((word >> 7) & 127), jmo = (int)((word >> 14) & 31);
    int c[D], av[D], mo[D];
#pragma unroll
    for (int j = 0; j < D; j++) {
        const int r = (jmo == j) ? c1o : c2o;
        mo[j] = ((word >> (19 + j)) & 1) ? -r : r;
    }
    // ---- pre: every edge but x
    int min1 = 127, min2 = 127, jmin = 0, sgn = 0;
    int i1 = 127, s2 = 0;   // over edges other than x and o
#pragma unroll
    for (int j = 0; j < D; j++) {
        if (j == X) continue;
        const int cj = clampi(bf.v[j] - mo[j], vmin, 127);
        const int aj = LQ ? abs(min(cj, mm)) : min(abs(cj), mm);
        c[j] = cj;
        av[j] = aj;
        const int sj = cj < 0;
        sgn ^= sj;
        jmin = (aj < min1) ? j : jmin;
        const int tt = min1;
        min1 = min(aj, min1);
        min2 = min(min2, max(aj, tt));
        if (j != O) {
            i1 = min(i1, aj);
            s2 ^= sj;
        }
    }
    // ---- chain
    const int T = cst_of<ALGO>(i1, prm, mm);
    const int kpar = s2 ^ (D & 1);
    const int mx = mo[X];
    const int vx = bf.v[X];
    const int co = c[O];
    int y = 0;
    for (int k = 0; k < cnt; k++) {
        const int t = dpp_shr1(carry, y);
        const int cx = clampi((has_x ? t : vx) - mx, vmin, 127);
        int r;
        if constexpr (ALGO == 1) {
            const int ax = min(abs(cx), mm);
            r = min(cst_of<ALGO>(ax, prm, mm), T);
        } else {
            // min(cst(a_x), T) with T = cst(I1) <= msg_max; in group 0
            // min(|c|, mm) - off needs no clip at mm because T <= mm - off there
            const int ax = LQ ? abs(min(cx, mm)) : abs(cx);
            r = clampi(ax - prm, 0, T);
        }
        const int neg = (cx < 0) ^ kpar;
        const int yn = clampi(co + (neg ? -r : r), vmin, 127);
        y = (slot == k) ? yn : y;
    }
    // ---- post
    const int t = dpp_shr1(carry, y);
    const int new_carry = __shfl(y, (int)(threadIdx.x & 48) + cnt - 1, 64);
    {
        const int cx = clampi((has_x ? t : vx) - mx, vmin, 127);
        const int ax = LQ ? abs(min(cx, mm)) : min(abs(cx), mm);
        c[X] = cx;
        av[X] = ax;
        jmin = (ax < min1) ? X : jmin;
        const int tt = min1;
        min1 = min(ax, min1);
        min2 = min(min2, max(ax, tt));
        sgn ^= (cx < 0);
    }
    const int cst1 = cst_of<ALGO>(min2, prm, mm), cst2 = cst_of<ALGO>(min1, prm, mm);
    const int par = sgn ^ (D & 1);
    uint32_t nw = (uint32_t)cst1 | ((uint32_t)cst2 << 7) | ((uint32_t)jmin << 14);
    const bool odead = fl & F_ODEAD;
    if (act) {
#pragma unroll
        for (int j = 0; j < D; j++) {
            const int r = (av[j] == min1) ? cst1 : cst2;
            const int neg = par ^ (c[j] < 0);
            nw |= (uint32_t)neg << (19 + j);
            const int vn = clampi(c[j] + (neg ? -r : r), vmin, 127);
            if (j != O || !odead) a.V[bf.addr[j]] = (int8_t)vn;
        }
        a.Mc[(size_t)(a.win_first[w] + slot) * a.stride + b] = nw;
    }
    return new_carry;
}

// Windows [wb, we) of one degree group, software-pipelined: at window t the
// wave issues the table loads of t+3 and the V / message loads of t+2.
template <int D, int ALGO, bool LATER>
LDPC_DEV int run_group(const WinArgs &a, int wb, int we, int slot, int b, int carry, bool live)
{
    Tab<D> T[2];
    Buf<D> B[3];
    if (wb < we) load_tab(T[0], a, wb, slot);
    if (wb + 1 < we) load_tab(T[1], a, wb + 1, slot);
    if (wb < we) load_buf(B[0], T[0], a, wb, slot, b);
    if (wb + 1 < we) load_buf(B[1], T[1], a, wb + 1, slot, b);
    if (wb + 2 < we) load_tab(T[0], a, wb + 2, slot);
    auto step = [&](auto sc, int t) {
        constexpr int s = decltype(sc)::value;
        if (t + 3 < we) load_tab(T[(s + 1) % 2], a, t + 3, slot);
        if (t + 2 < we) load_buf(B[(s + 2) % 3], T[s % 2], a, t + 2, slot, b);
        carry = do_window<D, ALGO, LATER>(B[s % 3], a, t, slot, b, carry, live);
    };
    for (int t = wb; t < we; t += 6) {
        step(std::integral_constant<int, 0>{}, t);
        if (t + 1 < we) step(std::integral_constant<int, 1>{}, t + 1);
        if (t + 2 < we) step(std::integral_constant<int, 2>{}, t + 2);
        if (t + 3 < we) step(std::integral_constant<int, 3>{}, t + 3);
        if (t + 4 < we) step(std::integral_constant<int, 4>{}, t + 4);
        if (t + 5 < we) step(std::integral_constant<int, 5>{}, t + 5);
    }
    return carry;
}

// Syndrome of the row's codeword after a full iteration: each lane checks the
// parity of its checks' hard decisions; OR over windows and the 16 lanes.
template <int D>
LDPC_DEV int syndrome_part(const WinArgs &a, int wb, int we, int slot, int b)
{
    int bad = 0;
    for (int w = wb; w < we; w++) {
        if (!(a.flags[w * S + slot] & F_ACT)) continue;
        const uint32_t *p = a.slotvar + a.slotoff[w] + slot;
        int par = 0;
#pragma unroll
        for (int j = 0; j < D; j++) par ^= (a.V[p[j * S] * (uint32_t)a.stride + b] > 0);
        bad |= par;
    }
    return bad;
}

template <int D0, int ALGO>
__global__ void __launch_bounds__(64) windowed_decode(WinArgs a)
{
    // XCD-aware wave -> codeword mapping: consecutive codeword groups (which
    // share V / Mc cache lines) go to the same XCD (blocks b, b+8, ... share one).
    const int nb = gridDim.x, id = blockIdx.x;
    const int wave = (id % 8) * (nb / 8) + id / 8;
    const int slot = threadIdx.x & 15, row = threadIdx.x >> 4;
    const int b = wave * G + row;
    // chain input of the first check in iteration 0: the initial V of its x
    // variable (afterwards the last check of each iteration provides it)
    int carry = a.V[a.slotvar[a.slotoff[0] + (D0 - 2) * S] * (uint32_t)a.stride + b];
    bool live = true;
    int it = 0;
    while (it < a.iters) {
        carry = run_group<D0, ALGO, false>(a, 0, a.g0_end, slot, b, carry, live);
        carry = run_group<D0 - 1, ALGO, true>(a, a.g0_end, a.n_windows, slot, b, carry, live);
        it++;
        if (a.early) {
            if (live) {
                int bad = syndrome_part<D0>(a, 0, a.g0_end, slot, b) |
                          syndrome_part<D0 - 1>(a, a.g0_end, a.n_windows, slot, b);
                // OR over the 16 lanes of the row
                bad |= __shfl_xor(bad, 1, 64);
                bad |= __shfl_xor(bad, 2, 64);
                bad |= __shfl_xor(bad, 4, 64);
                bad |= __shfl_xor(bad, 8, 64);
                if (!bad) {
                    live = false;
                    if (slot == 0 && a.iters_used) a.iters_used[b] = it;
                }
            }
            if (!__any(live)) break;
        }
    }
    if (live && slot == 0 && a.iters_used) a.iters_used[b] = it;
}

template <int D0>
int launch_d(const WinArgs &a, int algo, int grid, hipStream_t s)
{
    if (algo == 1)
        hipLaunchKernelGGL((windowed_decode<D0, 1>), dim3(grid), dim3(64), 0, s, a);
    else
        hipLaunchKernelGGL((windowed_decode<D0, 0>), dim3(grid), dim3(64), 0, s, a);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

bool degree_ok(int d) { return d == 7 || d == 10; }

}  // namespace

bool windowed_kernel_available() { return true; }

bool windowed_supported(const ldpc_code *h)
{
    return h->staircase && !h->windows.empty() && h->n_groups == 2 && degree_ok(h->group_deg[0]) &&
           h->group_deg[1] == h->group_deg[0] - 1;
}

bool windowed_params_ok(const ldpc_params *p)
{
    // compressed messages hold magnitudes 0..127; abs8(-128) never occurs
    if (p->var_min < -127 || p->var_min > 0 || p->msg_max < 0 || p->msg_max > 127) return false;
    if (p->algo == LDPC_ALGO_NMS) return p->factor >= 0 && p->factor <= 255;
    if (p->algo == LDPC_ALGO_OMS) return p->offset >= 0 && p->offset <= 127;
    return true;
}

int windowed_code_upload(const ldpc_code *h, WindowedCode *w)
{
    *w = WindowedCode{};
    if (!windowed_supported(h)) return LDPC_OK;
    const int nw = (int)h->windows.size();
    std::vector<uint32_t> slotvar, slotoff(nw);
    std::vector<uint8_t> flags((size_t)nw * S, 0);
    std::vector<int> first(nw), cnt(nw);
    int g0_end = nw;
    for (int i = 0; i < nw; i++) {
        const ldpc_window &win = h->windows[i];
        const int d = h->check_deg[win.first];
        if (h->check_group[win.first] != 0 && g0_end == nw) g0_end = i;
        first[i] = win.first;
        cnt[i] = win.count;
        slotoff[i] = (uint32_t)slotvar.size();
        slotvar.resize(slotvar.size() + (size_t)d * S, 0u);
        for (int k = 0; k < win.count; k++) {
            const int c = win.first + k;
            const uint32_t *ev = &h->edge_var[h->check_start[c]];
            for (int j = 0; j < d; j++) slotvar[slotoff[i] + j * S + k] = ev[j];
            uint8_t f = F_ACT;
            if (h->chain_in[c] >= 0) f |= F_XIN;
            // the o edge's V store is dead when the next check (same iteration)
            // consumes it through the chain and then rewrites it
            if (h->chain_out[c] >= 0 && c + 1 < h->m) f |= F_ODEAD;
            flags[(size_t)i * S + k] = f;
        }
        // inactive slots point at variable 0 (loads are skipped anyway)
    }
    // sanity: group 0 windows first, then group 1
    for (int i = 0; i < nw; i++)
        if ((i < g0_end) != (h->check_group[first[i]] == 0))
            return ldpc_set_error(LDPC_EINVAL, "windowed plan: groups out of order");
    w->g0_end = g0_end;
    w->n_windows = nw;
    w->max_deg = h->max_deg;
    w->d0 = h->group_deg[0];
    auto up = [&](void **dst, const void *src, size_t bytes) {
        if (hipMalloc(dst, bytes) != hipSuccess) return false;
        return hipMemcpy(*dst, src, bytes, hipMemcpyHostToDevice) == hipSuccess;
    };
    if (!up((void **)&w->d_slotvar, slotvar.data(), slotvar.size() * 4) ||
        !up((void **)&w->d_slotoff, slotoff.data(), slotoff.size() * 4) ||
        !up((void **)&w->d_flags, flags.data(), flags.size()) || !up((void **)&w->d_first, first.data(), nw * 4) ||
        !up((void **)&w->d_cnt, cnt.data(), nw * 4)) {
        windowed_code_free(w);
        return ldpc_set_error(LDPC_ENOMEM, "windowed tables");
    }
    w->valid = 1;
    return LDPC_OK;
}

void windowed_code_free(WindowedCode *w)
{
    (void)hipFree(w->d_slotvar);
    (void)hipFree(w->d_slotoff);
    (void)hipFree(w->d_flags);
    (void)hipFree(w->d_first);
    (void)hipFree(w->d_cnt);
    *w = WindowedCode{};
}

size_t windowed_msg_bytes(const ldpc_code *h, int stride)
{
    // one compressed word per check: 19 header bits + one sign bit per edge
    return (size_t)h->m * stride * (h->max_deg + 19 < 32 ? 4 : 8);   // windowed2 MsgT
}

int launch_windowed(const DecodeLaunch &L, const WindowedCode &w, hipStream_t s)
{
    if (!w.valid) return -1;
    WinArgs a;
    a.V = (int8_t *)L.V;
    a.Mc = (uint32_t *)L.msg;
    a.stride = L.stride;
    a.iters = L.iters;
    a.slotvar = w.d_slotvar;
    a.slotoff = w.d_slotoff;
    a.flags = w.d_flags;
    a.win_first = w.d_first;
    a.win_cnt = w.d_cnt;
    a.g0_end = w.g0_end;
    a.n_windows = w.n_windows;
    a.param = L.param;
    a.var_min = L.var_min;
    a.msg_max = L.msg_max;
    a.early = L.early;
    a.iters_used = L.iters_used;
    const int grid = L.stride / G;   // stride is a multiple of 64 -> grid % 16 == 0
    switch (w.d0) {
    case 7: return launch_d<7>(a, L.algo, grid, s);
    case 10: return launch_d<10>(a, L.algo, grid, s);
    default: return -1;
    }
}
