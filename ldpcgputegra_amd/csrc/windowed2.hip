// windowed2.hip -- second-generation windowed layered kernel for staircase
// (DVB-S2 IRA) codes, int8 offset-min-sum fast path.
//
// Same decomposition as windowed.hip (pre / serial staircase chain / post per
// window of consecutive checks, bit-exact with
// code/x86/CDecoder/OMS/CDecoder_OMS_fixed_SSE.cpp:172-546), with three
// changes that cut the per-check VALU work:
//
// 1. Sign-normalised ("z-domain") chain.  Check k maps the new value y of the
//    staircase variable it reads to the new value of the one it writes:
//        y_k = co_k + eps_k * dz(y_{k-1} - mx_k),
//        dz(u) = sign(u) * clamp(|u| - offset, 0, T_k) = med3(u - med3(u, -off, off), -T, T)
//    (eps_k = -1 iff the other edges' sign parity is odd, T_k = cst(min over
//    the info edges)).  With rho_k = eps_k rho_{k-1} and z_k = rho_k y_k every
//    step is   u_k = dz(u_{k-1}) + Dprev_k   -- med3, sub, med3, and one
//    DPP add (row_shr:1) that also moves the value to the next lane.
//    Lanes run the recurrence systolically (no per-step select): after s
//    steps lanes 0..s are final.  Chain values stay unclamped; that never
//    changes a dz input that matters because |y - mx| >= 127 - msg_max >
//    T + offset whenever y would have been clamped (needs msg_max <= 63 and
//    var range [-127, 127]; other parameters use windowed.hip).
// 2. S = 32 checks per window and G = 2 codewords per wave (S = 16 / G = 4
//    also built): 2 waves per SIMD at batch 4096, so the SIMD issues every 2
//    cycles instead of every 4.  A 32-lane chain step crosses 16-lane DPP
//    rows with row_bcast:15.
// 3. Cheaper per-edge arithmetic: a = med3(c, -c, msg_max), running min2 =
//    med3(a, min1, min2), sign parity accumulated as XOR of whole words,
//    negation by (r ^ s) + (s & 1).
//
// Read-ahead: V / messages of window t+P are loaded before window t's
// stores.  plan.cpp builds windows so that no variable read by window u
// (chain input excepted) is written by windows u-P..u-1 of the same group,
// and breaks windows where the chain breaks (only slot 0 may lack a chain
// input).  The single check of the later degree group (DVB-S2 check 0) uses
// the exact general step (its |min(c, max_msg)| quirk).
//
// Layout: V[N][stride] int8 (codeword fastest), Mc[check][stride] u32:
// cst1 | cst2 << 7 | jmin << 14 | sign_j << (19 + j).
#include <vector>

#include "windowed.h"

namespace {

constexpr int F_ACT = 1, F_XIN = 2, F_ODEAD = 4;

struct W2Args {
    int8_t *V;
    uint32_t *Mc;
    int stride;
    int iters;
    const uint32_t *slotvar;   // per window [D + 1][S]; group 0 first, then group 1
    int g0_end, n_windows;
    int off, msg_max, early;
    int32_t *iters_used;
};

// ---- lane shifts inside an S-lane row (S = 16: DPP row; S = 32: two rows)
template <int S>
LDPC_DEV int shift1(int old, int v)
{
    if constexpr (S == 32) {
        // rows 1, 3 <- lane 15 of rows 0, 2 ; then lanes 1..15 of every 16-row
        const int t = __builtin_amdgcn_update_dpp(old, v, 0x142, 0xA, 0xF, false);
        return __builtin_amdgcn_update_dpp(t, v, 0x111, 0xF, 0xF, false);
    } else {
        return __builtin_amdgcn_update_dpp(old, v, 0x111, 0xF, 0xF, false);
    }
}

// inclusive XOR scan over the S lanes of a row
template <int S>
LDPC_DEV int xor_scan(int p)
{
    p ^= __builtin_amdgcn_update_dpp(0, p, 0x111, 0xF, 0xF, false);
    p ^= __builtin_amdgcn_update_dpp(0, p, 0x112, 0xF, 0xF, false);
    p ^= __builtin_amdgcn_update_dpp(0, p, 0x114, 0xF, 0xF, false);
    p ^= __builtin_amdgcn_update_dpp(0, p, 0x118, 0xF, 0xF, false);
    if constexpr (S == 32) p ^= __builtin_amdgcn_update_dpp(0, p, 0x142, 0xA, 0xF, false);
    return p;
}

LDPC_DEV int med3(int x, int lo, int hi)
{
    int r;
    asm("v_med3_i32 %0, %1, %2, %3" : "=v"(r) : "v"(x), "v"(lo), "v"(hi));
    return r;
}

// S-1 systolic chain steps: u <- dz(u) + dprev, shifted one lane.
template <int S>
LDPC_DEV int chain_steps(int u, int dprev, int off, int T)
{
    const int noff = -off, nT = -T;
#pragma unroll
    for (int s = 0; s < S - 1; s++) {
        int s1, s2, s3;
        if constexpr (S == 32) {
            asm("v_med3_i32 %1, %0, %5, %6\n\t"
                "v_sub_u32 %2, %0, %1\n\t"
                "v_med3_i32 %3, %2, %7, %8\n\t"
                "s_nop 1\n\t"
                "v_add_u32_dpp %0, %3, %4 row_bcast:15 row_mask:0xa bank_mask:0xf\n\t"
                "v_add_u32_dpp %0, %3, %4 row_shr:1 row_mask:0xf bank_mask:0xf"
                : "+v"(u), "=&v"(s1), "=&v"(s2), "=&v"(s3)
                : "v"(dprev), "v"(noff), "v"(off), "v"(nT), "v"(T));
        } else {
            asm("v_med3_i32 %1, %0, %5, %6\n\t"
                "v_sub_u32 %2, %0, %1\n\t"
                "v_med3_i32 %3, %2, %7, %8\n\t"
                "s_nop 1\n\t"
                "v_add_u32_dpp %0, %3, %4 row_shr:1 row_mask:0xf bank_mask:0xf"
                : "+v"(u), "=&v"(s1), "=&v"(s2), "=&v"(s3)
                : "v"(dprev), "v"(noff), "v"(off), "v"(nT), "v"(T));
        }
    }
    return u;
}

// Per window the table holds [D + 1][S] words: rows 0..D-1 the variable of
// each edge, row D the slot's metadata: check index | flags << 24 |
// (window count - 1) << 27.  Inactive slots point at variable 0 and repeat a
// valid check index, so every lane issues the same loads (no data-dependent
// branch in the read-ahead) and all per-window facts arrive with the table
// loads one window early.  Tables of one degree group are contiguous, so the
// table of window w is at a fixed stride from the group's first table and no
// per-window scalar load (which would force a full vmcnt(0) drain) is needed.
template <int D>
struct Tab {
    uint32_t var[D];
    uint32_t meta;
};

// compressed message word: 19 header bits + one sign bit per edge.  Both
// degree groups of a code must use the same word (the tail check's word sits
// in the same Mc array): D0 = 14 needs 33 bits, so its tail (D = 13) takes 64
// bits as well -- hence u32 only up to D = 12 (the kernel's degrees: 7 / 6,
// 10 / 9 in u32; 14 / 13, 22 / 21, 27 / 26, 30 / 29 in u64)
template <int D>
using MsgT = typename std::conditional<(D + 19 < 32), uint32_t, uint64_t>::type;

template <int D>
struct Buf {
    int v[D];
    uint32_t addr[D];
    uint32_t mc;     // element index of the check's message word
    int fl;          // slot flags
    int cnt;         // active slots of the window
    MsgT<D> m;
};

template <int D, int S>
LDPC_DEV void load_tab(Tab<D> &t, const uint32_t *tab, int i, int slot)
{
    const uint32_t *p = tab + (size_t)i * (D + 1) * S + slot;
#pragma unroll
    for (int j = 0; j < D; j++) t.var[j] = p[j * S];
    t.meta = p[D * S];
}

template <int D, int S>
LDPC_DEV void load_buf(Buf<D> &bf, const Tab<D> &t, const W2Args &a, int b)
{
#pragma unroll
    for (int j = 0; j < D; j++) bf.addr[j] = t.var[j] * (uint32_t)a.stride + (uint32_t)b;
    bf.mc = (t.meta & 0xFFFFFFu) * (uint32_t)a.stride + (uint32_t)b;
    bf.fl = (int)(t.meta >> 24) & 7;
    bf.cnt = (int)(t.meta >> 27) + 1;
#pragma unroll
    for (int j = 0; j < D; j++) bf.v[j] = a.V[bf.addr[j]];
    bf.m = reinterpret_cast<const MsgT<D> *>(a.Mc)[bf.mc];
}

LDPC_DEV int decode_msg(uint32_t word, int j, int c1o, int c2o, int jmo)
{
    const int mag = (jmo == j) ? c1o : c2o;
    const int sm = ((int)(word << (12 - j))) >> 31;   // bit 19 + j, sign-extended
    return (mag ^ sm) - sm;
}

LDPC_DEV int decode_msg(uint64_t word, int j, int c1o, int c2o, int jmo)
{
    const int mag = (jmo == j) ? c1o : c2o;
    const int sm = j < 13 ? ((int)((uint32_t)word << (12 - j))) >> 31
                          : ((int)((uint32_t)(word >> 32) << (44 - j))) >> 31;   // bit 19 + j
    return (mag ^ sm) - sm;
}

// post: new messages and V for all D edges
template <int D>
LDPC_DEV void post_store(const W2Args &a, const Buf<D> &bf, const int (&c)[D], const int (&av)[D], int min1,
                         int sacc, bool act, bool odead, size_t mc_idx, int cst1, int cst2)
{
    using W = MsgT<D>;
    const int P = sacc ^ ((D & 1) ? (int)0x80000000 : 0);
    W nw = (W)cst1 | ((W)cst2 << 7);
    int jmin = 0;
#pragma unroll
    for (int j = 0; j < D; j++) {
        const bool eq = av[j] == min1;
        const int r = eq ? cst1 : cst2;
        jmin = eq ? j : jmin;
        const int t = c[j] ^ P;
        const int sm = t >> 31;
        const int lsb = (int)((uint32_t)t >> 31);
        nw |= (W)lsb << (19 + j);
        const int vn = med3(c[j] + (r ^ sm) + lsb, -127, 127);
        if (act && (j != D - 1 || !odead)) a.V[bf.addr[j]] = (int8_t)vn;
    }
    nw |= (W)jmin << 14;
    if (act) reinterpret_cast<W *>(a.Mc)[mc_idx] = nw;
}

// ---- one window of the first degree group (fast OMS path)
template <int D, int S>
LDPC_DEV int win_fast(const Buf<D> &bf, const W2Args &a, int w, int slot, int b, int carry, bool live)
{
    constexpr int X = D - 2, O = D - 1;
    const int fl = bf.fl;
    const bool act = (fl & F_ACT) && live;
    const int off = a.off, mm = a.msg_max;
    const int cnt = __builtin_amdgcn_readfirstlane(bf.cnt);   // same window in every lane
    const auto word = bf.m;
    const int c1o = (int)(word & 127), c2o = (int)((word >> 7) & 127), jmo = (int)((word >> 14) & 31);
    int c[D], av[D];
    int min1 = 127, min2 = 127, sacc = 0;
#pragma unroll
    for (int j = 0; j < X; j++) {   // info edges
        const int cj = med3(bf.v[j] - decode_msg(word, j, c1o, c2o, jmo), -127, 127);
        const int aj = med3(cj, -cj, mm);
        c[j] = cj;
        av[j] = aj;
        sacc ^= cj;
        min2 = med3(aj, min1, min2);
        min1 = min(aj, min1);
    }
    const int T = max(min1 - off, 0);                    // cst(min over info edges)
    const int kbit = (int)(((uint32_t)sacc >> 31) ^ (D & 1));   // eps = -1 when set
    {
        const int co = med3(bf.v[O] - decode_msg(word, O, c1o, c2o, jmo), -127, 127);
        const int ao = med3(co, -co, mm);
        c[O] = co;
        av[O] = ao;
        sacc ^= co;
        min2 = med3(ao, min1, min2);
        min1 = min(ao, min1);
    }
    const int mx = decode_msg(word, X, c1o, c2o, jmo);
    // rho_k = eps_k * rho_{k-1}, rho_{-1} = +1 (the carry enters as a plain V value)
    const int rbit = xor_scan<S>(kbit);
    const int rho = 1 - 2 * rbit, rho_prev = 1 - 2 * (rbit ^ kbit);
    const int tau = -rho_prev * mx;
    const int C = rho * c[O];
    const int dprev = shift1<S>(0, C) + tau;
    const int y0 = (fl & F_XIN) ? carry : bf.v[X];       // slot 0's chain input
    int u = rho_prev * y0 + tau;                         // only lane 0's value matters
    u = chain_steps<S>(u, dprev, off, T);
    // carry out: y of the window's last check (clamped: a plain V value)
    const int zk = C + med3(u - med3(u, -off, off), -T, T);
    const int ylast = med3(rho * zk, -127, 127);
    const int new_carry = __shfl(ylast, (int)(threadIdx.x & (64 - S)) + cnt - 1, 64);
    // post: the chain input of this check, then all edges
    {
        const int yin = med3(rho_prev * (u - tau), -127, 127);
        const int cx = med3(yin - mx, -127, 127);
        const int ax = med3(cx, -cx, mm);
        c[X] = cx;
        av[X] = ax;
        sacc ^= cx;
        min2 = med3(ax, min1, min2);
        min1 = min(ax, min1);
    }
    const int cst1 = max(min2 - off, 0), cst2 = max(min1 - off, 0);
    post_store<D>(a, bf, c, av, min1, sacc, act, fl & F_ODEAD, bf.mc, cst1, cst2);
    return new_carry;
}

// ---- exact general step (later degree group: |min(c, msg_max)| quirk);
// serial over the window's slots with a per-step commit.
template <int D, int S>
LDPC_DEV int win_exact_later(const Buf<D> &bf, const W2Args &a, int w, int slot, int b, int carry, bool live)
{
    constexpr int X = D - 2, O = D - 1;
    const int fl = bf.fl;
    const bool act = (fl & F_ACT) && live;
    const int off = a.off, mm = a.msg_max;
    const int cnt = __builtin_amdgcn_readfirstlane(bf.cnt);   // same window in every lane
    const auto word = bf.m;
    const int c1o = (int)(word & 127), c2o = (int)((word >> 7) & 127), jmo = (int)((word >> 14) & 31);
    int c[D], av[D];
    int min1 = 127, min2 = 127, sacc = 0;
    auto cst = [&](int v) { return min(max(v - off, 0), mm); };
#pragma unroll
    for (int j = 0; j < D; j++) {
        if (j == X) continue;
        const int cj = med3(bf.v[j] - decode_msg(word, j, c1o, c2o, jmo), -127, 127);
        const int aj = abs(min(cj, mm));
        c[j] = cj;
        av[j] = aj;
        sacc ^= cj;
        min2 = med3(aj, min1, min2);
        min1 = min(aj, min1);
    }
    int i1 = 127, s2 = 0;
#pragma unroll
    for (int j = 0; j < X; j++) {
        i1 = min(i1, av[j]);
        s2 ^= c[j];
    }
    const int T = cst(i1);
    const int kpar = (int)(((uint32_t)s2 >> 31) ^ (D & 1));
    const int mx = decode_msg(word, X, c1o, c2o, jmo);
    const int co = c[O];
    const int vx = bf.v[X];
    const bool has_x = fl & F_XIN;
    int y = 0;
    for (int k = 0; k < cnt; k++) {
        const int t = shift1<S>(carry, y);
        const int cx = med3((has_x ? t : vx) - mx, -127, 127);
        const int r = min(max(abs(min(cx, mm)) - off, 0), T);
        const int neg = (cx < 0) ^ kpar;
        const int yn = med3(co + (neg ? -r : r), -127, 127);
        y = (slot == k) ? yn : y;
    }
    const int t = shift1<S>(carry, y);
    const int new_carry = __shfl(y, (int)(threadIdx.x & (64 - S)) + cnt - 1, 64);
    {
        const int cx = med3((has_x ? t : vx) - mx, -127, 127);
        const int ax = abs(min(cx, mm));
        c[X] = cx;
        av[X] = ax;
        sacc ^= cx;
        min2 = med3(ax, min1, min2);
        min1 = min(ax, min1);
    }
    post_store<D>(a, bf, c, av, min1, sacc, act, fl & F_ODEAD, bf.mc, cst(min2), cst(min1));
    return new_carry;
}

// windows [wb, we) of one degree group, software-pipelined with read-ahead P
template <int D, int S, int P, bool FAST>
LDPC_DEV int run_group(const W2Args &a, const uint32_t *tab, int wb, int we, int slot, int b, int carry, bool live)
{
    Tab<D> T[2];
    Buf<D> B[P + 1];
    // The read-ahead loads are unconditional (past the group's end they
    // re-read its last window, harmlessly): conditional loads make the
    // compiler's wait-count merge pessimistic (a full vmcnt(0) drain before
    // every window).
    const int last = we - 1 - wb;
    // prologue: tables for wb..wb+P, buffers for wb..wb+P-1
#pragma unroll
    for (int i = 0; i < P; i++) {
        load_tab<D, S>(T[i % 2], tab, min(i, last), slot);
        load_buf<D, S>(B[i], T[i % 2], a, b);
    }
    load_tab<D, S>(T[P % 2], tab, min(P, last), slot);
    auto step = [&](auto sc, int i) {
        constexpr int s = decltype(sc)::value;
        load_tab<D, S>(T[(s + P + 1) % 2], tab, min(i + P + 1, last), slot);
        load_buf<D, S>(B[(s + P) % (P + 1)], T[(s + P) % 2], a, b);
        if constexpr (FAST)
            carry = win_fast<D, S>(B[s % (P + 1)], a, wb + i, slot, b, carry, live);
        else
            carry = win_exact_later<D, S>(B[s % (P + 1)], a, wb + i, slot, b, carry, live);
    };
    constexpr int U = (P == 1) ? 2 : 6;   // lcm(2, P + 1)
    const int n = we - wb;
    for (int i = 0; i < n; i += U) {
        step(std::integral_constant<int, 0>{}, i);
        if (i + 1 >= n) break;
        step(std::integral_constant<int, 1>{}, i + 1);
        if constexpr (U == 6) {
            if (i + 2 >= n) break;
            step(std::integral_constant<int, 2>{}, i + 2);
            if (i + 3 >= n) break;
            step(std::integral_constant<int, 3>{}, i + 3);
            if (i + 4 >= n) break;
            step(std::integral_constant<int, 4>{}, i + 4);
            if (i + 5 >= n) break;
            step(std::integral_constant<int, 5>{}, i + 5);
        }
    }
    return carry;
}

// 1 if a check of these windows fails for codeword row `row` (its S lanes
// see the same answer); the row stops at its first failing window -- a live
// codeword almost always fails early, so only converging codewords scan all
template <int D, int S>
LDPC_DEV int syndrome_part(const W2Args &a, const uint32_t *tab, int nwin, int slot, int row, int b)
{
    constexpr unsigned long long RM = (S == 64) ? ~0ull : ((1ull << S) - 1);
    int bad = 0;
    for (int w = 0; w < nwin; w++) {
        const uint32_t *p = tab + (size_t)w * (D + 1) * S + slot;
        int par = 0;
        if ((p[D * S] >> 24) & F_ACT) {
#pragma unroll
            for (int j = 0; j < D; j++) par ^= (a.V[p[j * S] * (uint32_t)a.stride + b] > 0);
        }
        bad |= par;
        if ((__ballot(bad) >> (row * S)) & RM) return 1;
    }
    return 0;
}

template <int D0, int S, int P>
__global__ void __launch_bounds__(64) windowed2_decode(W2Args a)
{
    constexpr int G = 64 / S;
    const int nb = gridDim.x, id = blockIdx.x;
    const int wave = (id % 8) * (nb / 8) + id / 8;   // XCD-aware: neighbours share an XCD
    const int slot = threadIdx.x & (S - 1), row = threadIdx.x / S;
    const int b = wave * G + row;
    const uint32_t *tab0 = a.slotvar, *tab1 = a.slotvar + (size_t)a.g0_end * (D0 + 1) * S;
    int carry = a.V[tab0[(D0 - 2) * S] * (uint32_t)a.stride + b];
    bool live = true;
    int it = 0;
    while (it < a.iters) {
        carry = run_group<D0, S, P, true>(a, tab0, 0, a.g0_end, slot, b, carry, live);
        carry = run_group<D0 - 1, S, 1, false>(a, tab1, a.g0_end, a.n_windows, slot, b, carry, live);
        it++;
        if (a.early) {
            if (live) {
                int bad = syndrome_part<D0, S>(a, tab0, a.g0_end, slot, row, b);
                if (!bad) bad = syndrome_part<D0 - 1, S>(a, tab1, a.n_windows - a.g0_end, slot, row, b);
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

}  // namespace

// ---------------------------------------------------------------- host side

bool windowed2_params_ok(const ldpc_params *p)
{
    return (p->algo == LDPC_ALGO_OMS || p->algo == LDPC_ALGO_MS) && p->var_min == -127 && p->var_max == 127 &&
           p->msg_max >= 0 && p->msg_max <= 63 && (p->algo == LDPC_ALGO_MS || (p->offset >= 0 && p->offset <= 63));
}

int windowed2_upload(const ldpc_code *h, int S, int P, Windowed2Code *w)
{
    *w = Windowed2Code{};
    std::vector<ldpc_window> wins;
    if (!(h->staircase && h->n_groups == 2 && h->group_deg[1] == h->group_deg[0] - 1 &&
          (h->group_deg[0] == 7 || h->group_deg[0] == 10 || h->group_deg[0] == 14 || h->group_deg[0] == 22 ||
           h->group_deg[0] == 27 || h->group_deg[0] == 30)))
        return LDPC_OK;
    extern int ldpc_plan_windows(const ldpc_code *h, int S, int P, std::vector<ldpc_window> &out);
    if (ldpc_plan_windows(h, S, P, wins) != LDPC_OK || wins.empty()) return LDPC_OK;
    const int nw = (int)wins.size();
    if (h->m >= (1 << 24)) return LDPC_OK;   // check index must fit the meta word
    std::vector<uint32_t> slotvar;
    int g0_end = nw;
    for (int i = 0; i < nw; i++) {
        const int c0 = wins[i].first;
        const int d = h->check_deg[c0];
        if (h->check_group[c0] != 0 && g0_end == nw) g0_end = i;
        // the kernel addresses tables by group: group 0 windows, then group 1
        if (h->check_group[c0] != (i < g0_end ? 0 : 1)) return LDPC_OK;
        const size_t base = slotvar.size();
        const uint32_t cbits = (uint32_t)(wins[i].count - 1) << 27;
        slotvar.resize(base + (size_t)(d + 1) * S, 0u);
        for (int k = 0; k < S; k++) {
            // inactive slots: variable 0 and the window's first check (valid,
            // never stored: flags 0)
            slotvar[base + (size_t)d * S + k] = (uint32_t)c0 | cbits;
            if (k >= wins[i].count) continue;
            const int c = c0 + k;
            const uint32_t *ev = &h->edge_var[h->check_start[c]];
            for (int j = 0; j < d; j++) slotvar[base + j * S + k] = ev[j];
            uint32_t f = F_ACT;
            if (h->chain_in[c] >= 0) f |= F_XIN;
            if (h->chain_out[c] >= 0 && c + 1 < h->m) f |= F_ODEAD;
            slotvar[base + (size_t)d * S + k] = (uint32_t)c | (f << 24) | cbits;
        }
    }
    auto up = [&](void **dst, const void *src, size_t bytes) {
        if (hipMalloc(dst, bytes) != hipSuccess) return false;
        return hipMemcpy(*dst, src, bytes, hipMemcpyHostToDevice) == hipSuccess;
    };
    if (!up((void **)&w->d_slotvar, slotvar.data(), slotvar.size() * 4)) {
        windowed2_free(w);
        return ldpc_set_error(LDPC_ENOMEM, "windowed2 tables");
    }
    w->valid = 1;
    w->S = S;
    w->P = P;
    w->d0 = h->group_deg[0];
    w->n_windows = nw;
    w->g0_end = g0_end;
    return LDPC_OK;
}

void windowed2_free(Windowed2Code *w)
{
    (void)hipFree(w->d_slotvar);
    *w = Windowed2Code{};
}

template <int D0, int S, int P>
static int launch3(const W2Args &a, int grid, hipStream_t s, int lds_pad)
{
    hipLaunchKernelGGL((windowed2_decode<D0, S, P>), dim3(grid), dim3(64), (size_t)lds_pad, s, a);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_windowed2(const DecodeLaunch &L, const Windowed2Code &w, hipStream_t s)
{
    if (!w.valid) return -1;
    W2Args a;
    a.V = (int8_t *)L.V;
    a.Mc = (uint32_t *)L.msg;
    a.stride = L.stride;
    a.iters = L.iters;
    a.slotvar = w.d_slotvar;
    a.g0_end = w.g0_end;
    a.n_windows = w.n_windows;
    a.off = L.param;
    a.msg_max = L.msg_max;
    a.early = L.early;
    a.iters_used = L.iters_used;
    const int G = 64 / w.S;
    const int grid = L.stride / G;   // stride % 64 == 0 -> grid % 8 == 0
    if (w.S != 16) return -1;   // S = 32 (one codeword per 32 lanes) was superseded and removed
    if (w.d0 == 7) return launch3<7, 16, 2>(a, grid, s, L.lds_pad);
    if (w.d0 == 10) return launch3<10, 16, 2>(a, grid, s, L.lds_pad);
    if (w.d0 == 14) return launch3<14, 16, 2>(a, grid, s, L.lds_pad);
    if (w.d0 == 22) return launch3<22, 16, 2>(a, grid, s, L.lds_pad);
    if (w.d0 == 27) return launch3<27, 16, 2>(a, grid, s, L.lds_pad);
    if (w.d0 == 30) return launch3<30, 16, 2>(a, grid, s, L.lds_pad);
    return -1;
}
