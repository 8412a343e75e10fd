// coop.hip -- workgroup-cooperative layered int8 offset-min-sum decoder for
// the DVB-S2 staircase codes (the BASELINE.json headline path).
//
// Arithmetic: bit-exact with the reference's CDecoder_OMS_fixed_SSE::decode_8bits
// (code/x86/CDecoder/OMS/CDecoder_OMS_fixed_SSE.cpp:172-546): every check in
// schedule order sees the V values left by all earlier checks.
//
// Layout / decomposition (CDNA4-first, not a translation of the reference's
// per-thread-codeword CUDA kernels):
//
// * A workgroup owns CW = 16 consecutive codewords.  V stays in HBM as
//   V[var][stride] (codeword fastest): one check slot touches 16 contiguous
//   bytes, and the 8 workgroups sharing a 128-B line are placed on one XCD
//   (block -> codeword-group remap) so the line is served by that XCD's L2.
//   Messages are compressed per check (cst1 | cst2 << 7 | jmin << 14 |
//   sign_j << (19 + j)) and laid out Mc[group][check][16]: a wave's 4 slots
//   read 256 contiguous bytes.
// * The schedule is cut into windows of <= S consecutive checks (plan at the
//   bottom).  WS = S / 4 "slab" waves own 4 check slots x 16 codewords each
//   and do all per-edge work in parallel: gather V, decode the old message,
//   min1 / min2 / sign (pre), new messages and V (post).
// * Inside a window the only dependency between checks is the staircase
//   parity variable: check k writes it as its last edge o, check k+1 reads it
//   as its edge x.  Pre reduces each check to six constants and one extra
//   "chain" wave runs the serial recurrence for the 16 codewords (one lane
//   each), 4 VALU per check:
//       Y_k = med3(med3(eps Y + A, co, eps Y + B), co - T, co + T)
//   (= co + eps dz(Y_{k-1} - mx), dz the offset dead zone clipped at T; see
//   pre_fast).  The x-edge inputs Y_{k-1} return to the slab waves through LDS.
// * Period p: the chain wave runs window p; the slab waves post window p-1
//   (phase A), then issue the loads of window p+1+R and pre window p+1
//   (phase B); two workgroup barriers per period.  A value written by window
//   w that window u loaded too early (2 <= u - w <= R + 1; u - w = 1 never
//   shares a variable, by plan) is forwarded through an LDS ring.  Global
//   stores and later loads of one workgroup are ordered by issue order (the
//   gfx950 workgroup-scope memory model needs no vmcnt wait for that).
#include <algorithm>
#include <cstdlib>
#include <type_traits>
#include <vector>

#include "coop.h"

namespace {

constexpr int CW = 16;                          // codewords per workgroup
constexpr uint32_t M_ACT = COOP_M_ACT;
constexpr uint32_t M_FWD = COOP_M_FWD;
constexpr int SRC_SHIFT = COOP_SRC_SHIFT;
constexpr uint32_t CHK_MASK = COOP_CHK_MASK;
constexpr uint32_t FWD_NONE = COOP_FWD_NONE;    // forwarding code: dW << 9 | slot << 3 | edge

template <int D0>
struct Geo {
    static constexpr int X = D0 - 2;                          // info edges of a group-0 check
    static constexpr int NFW = (X + 1) / 2;                   // dwords of u16 forwarding codes
    static constexpr bool WIDE = X > 8;                       // ring-source bits in a record word of their own
    static constexpr int EB = coop_fwd_eb(X);                 // edge bits of a forwarding code
    static constexpr int RECW = (D0 + 1 + NFW + (WIDE ? 1 : 0) + 3) / 4 * 4;   // vars, meta, fwd (, src)
    static_assert(!WIDE || coop_src_word(D0) == D0 + 1 + NFW, "source-bits word");
};

// compressed message word: cst1 | cst2 << 7 | jmin << 14 | sign_j << (19 + j),
// 64 bits when the degree needs them (one width per code: the tail check's
// word sits in the same array)
template <int D0>
using CMsg = typename std::conditional<(D0 + 19 <= 32), uint32_t, uint64_t>::type;

struct CoopArgs {
    int8_t *V;             // V[n + 1][stride]; row n receives masked stores
    void *Mc;              // CMsg<D0> Mc[stride / 16][m][16], then a 512-word sink
    const uint32_t *tab;   // [nw][S][RECW] slot records
    const uint8_t *live;   // [stride] early termination: 0 = codeword frozen (NULL: all live)
    // in-kernel early termination (ET kernels): layered edge list (group 0:
    // checks [0, m0) of degree D0, then degree d1), iterations used
    const uint32_t *ev;
    int32_t *iters_used;
    int iters, batch, m0, d1;
    int stride, G, nw, tail, m, n, off, mm, remap;
};

LDPC_DEV int med3(int x, int y, int z)
{
    int r;
    asm("v_med3_i32 %0, %1, %2, %3" : "=v"(r) : "v"(x), "v"(y), "v"(z));
    return r;
}

LDPC_DEV int mad24(int a, int b, int c)
{
    int r;
    asm("v_mad_i32_i24 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}

LDPC_DEV int clamp127(int x) { return min(max(x, -127), 127); }

// old message of edge j from the compressed word
LDPC_DEV int dec_msg(uint32_t w, int j, int c1, int c2, int jm)
{
    const int mag = (jm == j) ? c1 : c2;
    const int sm = ((int)(w << (12 - j))) >> 31;   // bit 19 + j
    return (mag ^ sm) - sm;
}
LDPC_DEV int dec_msg(uint64_t w, int j, int c1, int c2, int jm)
{
    const int mag = (jm == j) ? c1 : c2;
    const int sm = j < 13 ? ((int)((uint32_t)w << (12 - j))) >> 31
                          : ((int)((uint32_t)(w >> 32) << (44 - j))) >> 31;   // bit 19 + j
    return (mag ^ sm) - sm;
}

template <int D0, int WS, int R>
struct alignas(16) Smem {
    static constexpr int S = 4 * WS, X = Geo<D0>::X, RECW = Geo<D0>::RECW, TQ = R + 4;
    uint32_t tab[TQ][S][RECW];   // slot records of windows p-1 .. p+R+2
    int4 cst0[2][S][CW];         // chain constants (eps, A, B, co)   (pre -> chain)
    int2 cst1[2][S][CW];         //                 (L, H); lane-contiguous: no bank conflicts
    int xin[2][CW][S];           // chain outputs: x-edge input of each slot (chain -> post)
    uint8_t ring[R][S][X][CW];   // forwarded V values of the last R windows
};

template <int D0>
struct Pf {                       // prefetched inputs of one window (raw bytes: the
    uint32_t v[D0 - 1];           // sign extension happens at the use, so no wait
    CMsg<D0> m;                   // is forced right after the load); info, o; message
};

template <int D0>
struct St {                       // one window's state between pre and post
    int c[D0 - 1];                // contributions c_j (info, o); tail: new V values
    int a[D0 - 1];                // |c_j| clipped
    int mx, min1, min2, sacc;     // tail, 32-bit words: sacc = the new message word
    uint32_t twh;                 // tail, 64-bit words: its high half
};

template <int D0, int WS, int R>
struct Slab {
    using SM = Smem<D0, WS, R>;
    static constexpr int S = SM::S, X = SM::X, RECW = SM::RECW, TQ = SM::TQ, NFW = Geo<D0>::NFW;
    static constexpr int EB = Geo<D0>::EB;
    using W = CMsg<D0>;
    SM &sm;
    const CoopArgs &a;
    int k, c;
    uint32_t b, mcbase, vsink, mcsink;
    int bsh;   // bit offset of this codeword's byte in a V dword
    bool live; // early termination: stores of a converged codeword are masked

    // issue the loads of window g (local index u) into pf
    LDPC_DEV void prefetch(int g, int u, Pf<D0> &pf) const
    {
        const uint32_t *r = sm.tab[g % TQ][k];
        uint32_t var[D0];
#pragma unroll
        for (int j = 0; j < D0; j++) var[j] = r[j];
        const uint32_t meta = r[D0];
        const uint32_t st = (uint32_t)a.stride;
        // whole dwords (4 codewords; this lane's byte is extracted in pre):
        // byte loads make the compiler copy the value right after the load
        const uint32_t *V4 = (const uint32_t *)a.V;
#pragma unroll
        for (int j = 0; j < X; j++) pf.v[j] = V4[(var[j] * st + b) >> 2];
        const uint32_t vo = (u == a.tail) ? var[X] : var[D0 - 1];
        pf.v[X] = V4[(vo * st + b) >> 2];
        pf.m = ((const W *)a.Mc)[mcbase + (meta & CHK_MASK) * CW];
    }

    // pre of window g: forwarding, contributions, chain constants
    LDPC_DEV void pre(int g, int u, const Pf<D0> &pf, St<D0> &s) const
    {
        const uint32_t *r = sm.tab[g % TQ][k];
        const uint32_t meta = r[D0];
        int v[D0 - 1];
#pragma unroll
        for (int j = 0; j < D0 - 1; j++) v[j] = __builtin_amdgcn_sbfe(pf.v[j], bsh, 8);
        if (__any((meta & M_FWD) != 0)) {
            uint32_t fw[NFW];
#pragma unroll
            for (int i = 0; i < NFW; i++) fw[i] = r[D0 + 1 + i];
#pragma unroll
            for (int j = 0; j < X; j++) {
                const uint32_t code = (fw[j >> 1] >> ((j & 1) * 16)) & 0xFFFFu;
                const int dw = (int)(code >> (6 + EB));
                if (code != FWD_NONE && g >= dw) {
                    const int q = (g - dw) % R;
                    v[j] = (int8_t)sm.ring[q][(code >> EB) & 63][code & ((1u << EB) - 1)][c];
                }
            }
        }
        const W w = pf.m;
        const int c1 = (int)(w & 127), c2 = (int)((w >> 7) & 127), jm = (int)((w >> 14) & 31);
        const int off = a.off, mm = a.mm;
        int eps, A, B, co, L, H;
        int min1 = 127, min2 = 127, sacc = 0;
        if (u != a.tail) {
            // first degree group: a = min(|c|, msg_max) (OMS_fixed_SSE.cpp:211)
#pragma unroll
            for (int j = 0; j < X; j++) {
                const int cj = clamp127(v[j] - dec_msg(w, j, c1, c2, jm));
                const int aj = med3(cj, -cj, mm);
                s.c[j] = cj;
                s.a[j] = aj;
                sacc ^= cj;
                min2 = med3(aj, min1, min2);
                min1 = min(aj, min1);
            }
            // chain constants of this check: T = cst(min over the info edges),
            // eps = -1 iff the info edges' sign parity (with the odd-degree
            // flip) is odd.  With w = Y_{k-1} - mx:
            //   new V[o] = co + eps * sign(w) * min(max(|w| - off, 0), T)
            //            = med3(med3(eps Y + A, co, eps Y + B), co - T, co + T)
            // A = co - eps (mx + off), B = co - eps (mx - off).  Y may stay
            // unclamped along the chain: a value beyond +-127 gives the same
            // dead-zone output as its clamp because 127 - msg_max >= T + off.
            const int T = max(min1 - off, 0);
            const int kbit = (int)(((uint32_t)sacc >> 31) ^ (uint32_t)(D0 & 1));
            co = clamp127(v[X] - dec_msg(w, D0 - 1, c1, c2, jm));
            const int ao = med3(co, -co, mm);
            s.c[X] = co;
            s.a[X] = ao;
            sacc ^= co;
            min2 = med3(ao, min1, min2);
            min1 = min(ao, min1);
            const int mx = dec_msg(w, X, c1, c2, jm);
            s.mx = mx;
            s.min1 = min1;
            s.min2 = min2;
            s.sacc = sacc;
            eps = 1 - 2 * kbit;
            A = co - eps * (mx + off);
            B = co - eps * (mx - off);
            L = co - T;
            H = co + T;
        } else {
            // the tail check (later degree group: a = |min(c, msg_max)|,
            // OMS_fixed_SSE.cpp:293,314) has no chain input: finish it here
#pragma unroll
            for (int j = 0; j <= X; j++) {
                const int cj = clamp127(v[j] - dec_msg(w, j, c1, c2, jm));
                const int t = min(cj, mm);
                const int aj = max(t, -t);
                s.c[j] = cj;
                s.a[j] = aj;
                sacc ^= cj;
                min2 = med3(aj, min1, min2);
                min1 = min(aj, min1);
            }
            const int cst1 = min(max(min2 - off, 0), mm), cst2 = min(max(min1 - off, 0), mm);
            const int P = sacc ^ (((D0 - 1) & 1) ? (int)0x80000000 : 0);
            W nw = (W)cst1 | ((W)cst2 << 7);
            int jmin = 0;
#pragma unroll
            for (int j = 0; j <= X; j++) {
                const bool eq = s.a[j] == min1;
                const int rr = eq ? cst1 : cst2;
                jmin = eq ? j : jmin;
                const int t = s.c[j] ^ P;
                const int sm = t >> 31;
                const int lsb = (int)((uint32_t)t >> 31);
                nw |= (W)lsb << (19 + j);
                s.c[j] = clamp127(s.c[j] + (rr ^ sm) + lsb);
            }
            nw |= (W)jmin << 14;
            s.sacc = (int)(uint32_t)nw;
            if constexpr (sizeof(W) == 8) s.twh = (uint32_t)(nw >> 32);
            const int y = s.c[X];
            eps = 0;
            A = B = co = L = H = y;
        }
        if (!(meta & M_ACT)) {   // pass-through: Y_k = Y_{k-1}
            eps = 1;
            A = B = co = 0;
            L = -1024;
            H = 1024;
        }
        sm.cst0[g & 1][k][c] = make_int4(eps, A, B, co);
        sm.cst1[g & 1][k][c] = make_int2(L, H);
    }

    // post of window g: new messages and V, stores, LDS ring
    LDPC_DEV void post(int g, int u, const St<D0> &s) const
    {
        const uint32_t *r = sm.tab[g % TQ][k];
        uint32_t var[D0];
#pragma unroll
        for (int j = 0; j < D0; j++) var[j] = r[j];
        const uint32_t meta = r[D0];
        const bool act = (meta & M_ACT) && live;
        const bool tl = (u == a.tail);
        const int xin = sm.xin[g & 1][c][k];
        int vn[D0];
        W nw;
        if (!tl) {
            const int off = a.off, mm = a.mm;
            const int cx = clamp127(clamp127(xin) - s.mx);
            const int ax = med3(cx, -cx, mm);
            const int sacc = s.sacc ^ cx;
            const int min2 = med3(ax, s.min1, s.min2);
            const int min1 = min(ax, s.min1);
            const int cst1 = max(min2 - off, 0), cst2 = max(min1 - off, 0);   // <= msg_max already
            const int P = sacc ^ ((D0 & 1) ? (int)0x80000000 : 0);
            nw = (W)cst1 | ((W)cst2 << 7);
            int jmin = 0;
#pragma unroll
            for (int j = 0; j < D0; j++) {
                const int cj = (j < X) ? s.c[j] : (j == X ? cx : s.c[X]);
                const int aj = (j < X) ? s.a[j] : (j == X ? ax : s.a[X]);
                const bool eq = aj == min1;
                const int rr = eq ? cst1 : cst2;
                jmin = eq ? j : jmin;
                const int t = cj ^ P;
                const int sm = t >> 31;
                const int lsb = (int)((uint32_t)t >> 31);
                nw |= (W)lsb << (19 + j);
                vn[j] = clamp127(cj + (rr ^ sm) + lsb);
            }
            nw |= (W)jmin << 14;
        } else {
#pragma unroll
            for (int j = 0; j <= X; j++) vn[j] = s.c[j];
            vn[D0 - 1] = clamp127(xin);   // V of the last group-0 check's o edge (only the chain had it)
            nw = (W)(uint32_t)s.sacc;
            if constexpr (sizeof(W) == 8) nw |= (W)s.twh << 32;
        }
        // Stores: edges 0..D0-2 (info + x; the tail: info + o).  A group-0 o
        // store is dead (the next check rewrites the variable through its x
        // edge); the last one is written by the tail from the chain.  Masked
        // slots store to the sink row, so every store is issued unconditionally.
        const uint32_t st = (uint32_t)a.stride;
#pragma unroll
        for (int j = 0; j < D0 - 1; j++) a.V[act ? var[j] * st + b : vsink] = (int8_t)vn[j];
        if (tl) a.V[act ? var[D0 - 1] * st + b : vsink] = (int8_t)vn[D0 - 1];
        ((W *)a.Mc)[act ? mcbase + (meta & CHK_MASK) * CW : mcsink] = nw;
        uint32_t srcb;
        if constexpr (Geo<D0>::WIDE)
            srcb = r[coop_src_word(D0)];
        else
            srcb = meta >> SRC_SHIFT;
#pragma unroll
        for (int j = 0; j < X; j++)
            if ((srcb >> j) & 1) sm.ring[g % R][k][j][c] = (uint8_t)vn[j];
    }
};

// chain steps [K0, K1) of window g for the 16 codewords (lanes 0..15).  All
// constants of the range are read first (the LDS latency would otherwise sit
// on the serial chain once per step), then the recurrence runs back to back.
template <int D0, int WS, int R, int K0, int K1>
LDPC_DEV void chain_steps(Smem<D0, WS, R> &sm, int g, int c, int &Y)
{
    constexpr int NK = K1 - K0;
    const int buf = g & 1;
    int4 q0[NK];
    int2 q1[NK];
#pragma unroll
    for (int i = 0; i < NK; i++) {
        q0[i] = sm.cst0[buf][K0 + i][c];
        q1[i] = sm.cst1[buf][K0 + i][c];
    }
    int xv[4];
#pragma unroll
    for (int i = 0; i < NK; i++) {
        const int k = K0 + i;
        xv[k & 3] = Y;
        const int p = mad24(Y, q0[i].x, q0[i].y), q = mad24(Y, q0[i].x, q0[i].z);
        Y = med3(med3(p, q0[i].w, q), q1[i].x, q1[i].y);
        if ((k & 3) == 3) *(int4 *)&sm.xin[buf][c][k - 3] = make_int4(xv[0], xv[1], xv[2], xv[3]);
    }
}

// high bit of byte j set where byte j > 0 (hard decision), SWAR; 16 bytes ->
// 16-bit codeword mask
LDPC_DEV uint32_t pos_bits(uint32_t d)
{
    const uint32_t nz = ((d & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | d;
    return nz & ~d & 0x80808080u;
}
LDPC_DEV uint32_t high_bits16(uint4 x)
{
    auto c4 = [](uint32_t v) { return ((v >> 7) & 1u) | ((v >> 14) & 2u) | ((v >> 21) & 4u) | ((v >> 28) & 8u); };
    return c4(x.x) | c4(x.y) << 4 | c4(x.z) << 8 | c4(x.w) << 12;
}

// ET = true: in-kernel early termination (as coop3_decode<.., ET>): one
// iteration per segment, then the workgroup's syndrome of its live codewords
// (stopping once each has a failing check); converged codewords' stores are
// masked from the next segment on, which freezes their V and messages at the
// iteration they converged (no snapshot needed); the workgroup leaves when
// all 16 have converged
template <int D0, int WS, int R, bool ET = false>
__global__ void __launch_bounds__(64 * (WS + 1)) coop_decode(CoopArgs a)
{
    using SM = Smem<D0, WS, R>;
    constexpr int S = SM::S, X = SM::X, RECW = SM::RECW, TQ = SM::TQ;
    constexpr int U = (R + 1) % 2 ? 2 * (R + 1) : (R + 1);   // lcm(2, R + 1)
    constexpr int SPLIT = (S / 2) & ~3;
    __shared__ SM sm;

    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const int nb = gridDim.x, id = blockIdx.x;
    const int wg = a.remap ? (id & 7) * (nb >> 3) + (id >> 3) : id;   // XCD-aware codeword groups
    const int G = ET ? a.nw : a.G;   // periods per segment (ET: one iteration)
    if (G == 0) return;
    bool live = (!ET && a.live) ? a.live[wg * CW + (lane & 15)] != 0 : true;
    if (!ET && a.live && !__syncthreads_or(live)) return;   // all 16 codewords converged
    // ---- ET state: [0] live codewords, [1] failing codewords (syndrome)
    __shared__ uint32_t et_sh[2];
    constexpr int NT = 64 * (WS + 1);
    const char *etV = (const char *)a.V + (size_t)wg * CW;
    if constexpr (ET) {
        if (threadIdx.x == 0) {
            const int valid = min(CW, max(0, a.batch - wg * CW));
            et_sh[0] = (1u << valid) - 1u;
            et_sh[1] = 0;
        }
        if (threadIdx.x < CW && wg * CW + (int)threadIdx.x < a.batch) a.iters_used[wg * CW + threadIdx.x] = a.iters;
        __syncthreads();
        if (et_sh[0] == 0) return;   // padding columns only
        live = (et_sh[0] >> (lane & 15)) & 1u;
    }
    // after iteration `it` (ET): syndrome and decision, every thread, uniform
    // result (true: decode another iteration)
    auto et_after = [&](int it) -> bool {
        __syncthreads();   // the iteration's stores were issued before the last barrier of the segment
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        const uint32_t lv = et_sh[0];
        constexpr int CPT = D0 > 10 ? 1 : 2;   // checks per thread and round (VGPRs: D0 x 16 B each)
        for (int c0 = 0; c0 < a.m; c0 += NT * CPT * 4) {
            uint4 acc = make_uint4(0, 0, 0, 0);
#pragma unroll
            for (int r = 0; r < 4 * CPT; r++) {
                const int c = c0 + r * NT + (int)threadIdx.x;
                uint4 x = make_uint4(0, 0, 0, 0);
                if (c < a.m0) {
                    const uint32_t *e = a.ev + (size_t)c * D0;
                    uint4 y[D0];
#pragma unroll
                    for (int j = 0; j < D0; j++) y[j] = *(const uint4 *)(etV + (size_t)e[j] * (size_t)a.stride);
#pragma unroll
                    for (int j = 0; j < D0; j++) {
                        x.x ^= pos_bits(y[j].x);
                        x.y ^= pos_bits(y[j].y);
                        x.z ^= pos_bits(y[j].z);
                        x.w ^= pos_bits(y[j].w);
                    }
                } else if (c < a.m) {
                    const uint32_t *e = a.ev + (size_t)a.m0 * D0 + (size_t)(c - a.m0) * a.d1;
                    for (int j = 0; j < a.d1; j++) {
                        const uint4 y = *(const uint4 *)(etV + (size_t)e[j] * (size_t)a.stride);
                        x.x ^= pos_bits(y.x);
                        x.y ^= pos_bits(y.y);
                        x.z ^= pos_bits(y.z);
                        x.w ^= pos_bits(y.w);
                    }
                }
                acc.x |= x.x;
                acc.y |= x.y;
                acc.z |= x.z;
                acc.w |= x.w;
            }
            const uint32_t f = high_bits16(acc) & lv;
            if (f) atomicOr(&et_sh[1], f);
            __syncthreads();
            const uint32_t fail = et_sh[1];
            __syncthreads();
            if ((fail & lv) == lv) break;   // every live codeword has a failing check
        }
        const uint32_t fresh = lv & ~et_sh[1];   // converged after this iteration
        __syncthreads();
        if (threadIdx.x == 0) {
            et_sh[0] = lv & ~fresh;
            et_sh[1] = 0;
        }
        if (threadIdx.x < CW && ((fresh >> threadIdx.x) & 1u)) a.iters_used[wg * CW + threadIdx.x] = it + 1;
        __syncthreads();
        live = (et_sh[0] >> (lane & 15)) & 1u;
        return (lv & ~fresh) != 0 && it + 1 < a.iters;
    };

    if (wave == WS) {
        // ------------------------------------------------------------ chain wave
        constexpr int NCH = S * RECW / 4;   // 16-B chunks per window table
        constexpr int CPL = (NCH + 63) / 64;   // chunks per lane
        const int c = lane & 15;
        static_assert(CPL <= 4, "window table: at most 4 chunks per lane");
        // one window table in flight, CPL 16-B chunks per lane (named
        // registers: an indexed array here ends up in scratch)
        uint4 t0, t1, t2, t3;
        auto load = [&](int u) {
            const uint4 *src = (const uint4 *)(a.tab + (size_t)u * S * RECW);
            t0 = src[min(lane, NCH - 1)];
            if constexpr (CPL > 1) t1 = src[min(lane + 64, NCH - 1)];
            if constexpr (CPL > 2) t2 = src[min(lane + 128, NCH - 1)];
            if constexpr (CPL > 3) t3 = src[min(lane + 192, NCH - 1)];
        };
        auto store = [&](int slot) {
            uint4 *dst = (uint4 *)&sm.tab[slot][0][0];
            if (lane < NCH) dst[lane] = t0;
            if constexpr (CPL > 1)
                if (lane + 64 < NCH) dst[lane + 64] = t1;
            if constexpr (CPL > 2)
                if (lane + 128 < NCH) dst[lane + 128] = t2;
            if constexpr (CPL > 3)
                if (lane + 192 < NCH) dst[lane + 192] = t3;
        };
        const bool cl = lane < CW;   // the chain runs on 16 lanes
        for (int it = 0;; it++) {   // one segment (ET: one iteration per segment)
            for (int q = 0; q <= R + 1; q++) {
                load(q % a.nw);
                store(q);
            }
            int Y = a.V[a.tab[X] * (uint32_t)a.stride + (uint32_t)(wg * CW + c)];   // x input of the first check
            load((R + 2) % a.nw);
            int un = (R + 3) % a.nw;
            __syncthreads();   // prologue: tables in LDS
            __syncthreads();   // pre(0) done: constants of window 0 in LDS
            for (int p = 0; p <= G; p++) {
                if (p < G && cl) chain_steps<D0, WS, R, 0, SPLIT>(sm, p, c, Y);
                store((p + R + 2) % TQ);
                load(un);
                un = (un + 1 == a.nw) ? 0 : un + 1;
                __syncthreads();   // A
                if (p < G && cl) chain_steps<D0, WS, R, SPLIT, S>(sm, p, c, Y);
                __syncthreads();   // B
            }
            if (!ET || !et_after(it)) break;
        }
        return;
    }

    // -------------------------------------------------------------- slab waves
    const int k = 4 * wave + (lane >> 4), c = lane & 15;
    Slab<D0, WS, R> sl{sm, a, k, c, (uint32_t)(wg * CW + c), (uint32_t)(wg * a.m * CW + c),
                       (uint32_t)a.n * (uint32_t)a.stride + (uint32_t)lane,
                       (uint32_t)nb * (uint32_t)a.m * CW + threadIdx.x, (c & 3) * 8, live};
    for (int it = 0;; it++) {   // one segment (ET: one iteration per segment)
        sl.live = live;
        Pf<D0> pf[R + 1];
        St<D0> st[2];
        __syncthreads();   // prologue: tables of windows 0 .. R+1 are in LDS
#pragma unroll
        for (int i = 0; i <= R; i++) sl.prefetch(i, i, pf[i]);   // nw > R + 3
        sl.pre(0, 0, pf[0], st[0]);
        // period 0: chain(0) | nothing to post | loads of R+1, pre(1)
        __syncthreads();   // B of the prologue
        __syncthreads();   // A(0)
        sl.prefetch(R + 1, (R + 1) % a.nw, pf[0]);
        sl.pre(1, 1, pf[1], st[1]);
        __syncthreads();   // B(0)
        int uA = 0, uB = 2 % a.nw, uP = (R + 2) % a.nw;   // windows p-1, p+1, p+1+R (local index)
        auto next = [&](int &u) { u = (u + 1 == a.nw) ? 0 : u + 1; };
        // steady state p = 1 .. G: every memory operation unconditional (loads past
        // the end read valid table rows; their pre only writes unused constants)
        auto step = [&](auto sc, int p) {
            constexpr int s = decltype(sc)::value;
            sl.post(p - 1, uA, st[s % 2]);
            __syncthreads();   // A(p)
            sl.prefetch(p + 1 + R, uP, pf[(s + 1) % (R + 1)]);
            sl.pre(p + 1, uB, pf[(s + 2) % (R + 1)], st[s % 2]);
            __syncthreads();   // B(p)
            next(uA);
            next(uB);
            next(uP);
        };
        // single-exit loop over whole unroll groups (multi-exit loops get
        // restructured and lose the precise wait counts), then the remainder
        const int nfull = G / U;
        int p = 1;
        for (int i = 0; i < nfull; i++, p += U) {
            step(std::integral_constant<int, 0>{}, p);
            step(std::integral_constant<int, 1>{}, p + 1);
            if constexpr (U > 2) {
                step(std::integral_constant<int, 2>{}, p + 2);
                step(std::integral_constant<int, 3>{}, p + 3);
            }
            if constexpr (U > 4) {
                step(std::integral_constant<int, 4>{}, p + 4);
                step(std::integral_constant<int, 5>{}, p + 5);
            }
            if constexpr (U > 6) {
                step(std::integral_constant<int, 6>{}, p + 6);
                step(std::integral_constant<int, 7>{}, p + 7);
            }
            if constexpr (U > 8) {
                step(std::integral_constant<int, 8>{}, p + 8);
                step(std::integral_constant<int, 9>{}, p + 9);
            }
            static_assert(U <= 10, "unroll");
        }
        const int rem = G - nfull * U;
        if (rem > 0) step(std::integral_constant<int, 0>{}, p);
        if (rem > 1) step(std::integral_constant<int, 1>{}, p + 1);
        if constexpr (U > 2) {
            if (rem > 2) step(std::integral_constant<int, 2>{}, p + 2);
            if (rem > 3) step(std::integral_constant<int, 3>{}, p + 3);
        }
        if constexpr (U > 4) {
            if (rem > 4) step(std::integral_constant<int, 4>{}, p + 4);
            if (rem > 5) step(std::integral_constant<int, 5>{}, p + 5);
        }
        if constexpr (U > 6) {
            if (rem > 6) step(std::integral_constant<int, 6>{}, p + 6);
            if (rem > 7) step(std::integral_constant<int, 7>{}, p + 7);
        }
        if constexpr (U > 8) {
            if (rem > 8) step(std::integral_constant<int, 8>{}, p + 8);
        }
        if (!ET || !et_after(it)) break;
    }
}

// ------------------------------------------------------- early termination
// After each iteration (one coop launch): a codeword stops once all its
// parity checks hold on the hard decisions V > 0 (the
// oracle's early_term; not the reference's commented `arret` test,
// CDecoder_OMS_fixed_SSE.cpp:255,551-553, which tests extrinsic sign parity
// per 16-frame call: iterations used are unpinned by the reference).
// Block = 64 consecutive codewords (coalesced V rows) x a chunk of checks;
// the H indices are wave-uniform (scalar loads).
// 1 if any of the 4 consecutive degree-D checks at ev fails
template <int D>
__device__ __forceinline__ int parity4(const int8_t *V, const uint32_t *ev, int stride, int b)
{
    int8_t x[4 * D];
#pragma unroll
    for (int j = 0; j < 4 * D; j++) x[j] = V[(size_t)ev[j] * stride + b];
    int bad = 0;
#pragma unroll
    for (int i = 0; i < 4; i++) {
        int par = 0;
#pragma unroll
        for (int j = 0; j < D; j++) par ^= x[i * D + j] > 0;
        bad |= par;
    }
    return bad;
}

__global__ void __launch_bounds__(64) syndrome_k(const int8_t *V, int stride, int batch, const uint32_t *ev,
                                                 const int *gdeg, const int *gcnt, int ngroups, int m, int chunk,
                                                 const uint8_t *live, uint32_t *bad)
{
    const int b = blockIdx.x * 64 + threadIdx.x;
    if (b >= batch || !live[b]) return;
    if (__hip_atomic_load(&bad[b], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return;   // another chunk failed
    const int c0 = blockIdx.y * chunk, c1 = min(m, c0 + chunk);
    int g = 0, gfirst = 0, e = 0;
    while (g < ngroups && c0 >= gfirst + gcnt[g]) {
        e += gdeg[g] * gcnt[g];
        gfirst += gcnt[g];
        g++;
    }
    int d = gdeg[g];
    e += (c0 - gfirst) * d;
    int gend = gfirst + gcnt[g];
    int badv = 0;
    for (int c = c0; c < c1;) {
        if (c == gend) {
            g++;
            d = gdeg[g];
            gend += gcnt[g];
        }
        // four checks of the coop degrees at a time: all their gathers in flight at once
        if (c + 4 <= min(c1, gend) && (d == 7 || d == 10)) {
            badv = d == 7 ? parity4<7>(V, ev + e, stride, b) : parity4<10>(V, ev + e, stride, b);
            c += 4;
            e += 4 * d;
        } else {
            int par = 0;
            for (int j = 0; j < d; j++) par ^= V[(size_t)ev[e + j] * stride + b] > 0;
            badv = par;
            c++;
            e += d;
        }
        if (badv) break;   // one failing check decides: live codewords stop early
    }
    if (badv) atomicOr(&bad[b], 1u);
}

__global__ void syndrome_finish_k(int batch, uint8_t *live, uint32_t *bad, int32_t *iters_used, int it)
{
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= batch) return;
    if (live[b] && !bad[b]) {
        live[b] = 0;
        iters_used[b] = it;
    }
    bad[b] = 0;
}

__global__ void fill_iters_k(int batch, int32_t *iters_used, int iters)
{
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b < batch) iters_used[b] = iters;
}

// codewords converging after this iteration (live, no failing check): copy
// their V column; block = 64 codewords x a chunk of rows
constexpr int kSnapRows = 128;
// rows [r0, r1) of column b, 16 loads in flight per round (a lone thread's
// strided column copy is latency-bound otherwise)
__device__ __forceinline__ void copy_column(const int8_t *src, int8_t *dst, int stride, int b, int r0, int r1)
{
    int r = r0;
    for (; r + 16 <= r1; r += 16) {
        int8_t x[16];
#pragma unroll
        for (int i = 0; i < 16; i++) x[i] = src[(size_t)(r + i) * stride + b];
#pragma unroll
        for (int i = 0; i < 16; i++) dst[(size_t)(r + i) * stride + b] = x[i];
    }
    for (; r < r1; r++) dst[(size_t)r * stride + b] = src[(size_t)r * stride + b];
}
__global__ void __launch_bounds__(64) snapshot_k(const int8_t *V, int8_t *Vs, int stride, int batch, int rows,
                                                 const uint8_t *live, const uint32_t *bad)
{
    const int b = blockIdx.x * 64 + threadIdx.x;
    if (b >= batch || !live[b] || bad[b]) return;
    copy_column(V, Vs, stride, b, blockIdx.y * kSnapRows, min(rows, (int)(blockIdx.y + 1) * kSnapRows));
}

// after the last iteration: converged codewords take their snapshot back
__global__ void __launch_bounds__(64) merge_snapshot_k(int8_t *V, const int8_t *Vs, int stride, int batch, int rows,
                                                       const uint8_t *live)
{
    const int b = blockIdx.x * 64 + threadIdx.x;
    if (b >= batch || live[b]) return;
    copy_column(Vs, V, stride, b, blockIdx.y * kSnapRows, min(rows, (int)(blockIdx.y + 1) * kSnapRows));
}

// live[] covers the padded stride: padding columns are never live, so a
// workgroup's skip test (any live codeword) does not read stale bytes
__global__ void early_init_k(int batch, int stride, uint8_t *live, uint32_t *bad, int32_t *iters_used, int iters)
{
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= stride) return;
    live[b] = b < batch;
    if (b >= batch) return;
    bad[b] = 0;
    iters_used[b] = iters;
}

}  // namespace

// ------------------------------------------------------------------ host plan

// Windows: runs of <= S consecutive group-0 checks in schedule order such that
// no two checks of a window, and no checks of two consecutive windows
// (cyclically, across the iteration boundary too), share an information
// variable; an empty window is inserted where a check would conflict with the
// previous window.  The tail check (the one check of the second degree group)
// is a window of its own.  Forwarding: every info-edge read whose latest
// writer is 2..R+1 windows earlier (cyclic) reads that writer's LDS ring entry.
int coop_build_plan(const ldpc_code *h, int S, int R, int dist, int recw, CoopPlan &o, bool want_tab)
{
    if (S < 1 || S > 64 || R < 1 || R > 6 || dist < 1 || dist > 2) return -1;   // forwarding code: 6-bit slot
    if (!h->staircase || h->n_groups != 2 || h->group_cnt[1] != 1) return -1;
    const int D0 = h->group_deg[0], X = D0 - 2, M = h->m, T = M - 1;
    if (h->group_deg[1] != D0 - 1 || X < 1 || X > 28 || M < 4 || M >= (1 << 20)) return -1;
    const int EB = coop_fwd_eb(X);
    if (want_tab && X > 8 && recw <= coop_src_word(D0)) return -1;
    auto ev = [&](int c, int j) { return h->edge_var[h->check_start[c] + j]; };
    // staircase: x edge (D0-2) of check c is the o edge (D0-1) of check c-1;
    // the x edge of check 0 is the tail's last edge
    for (int c = 1; c < T; c++)
        if (ev(c, X) != ev(c - 1, D0 - 1)) return -1;
    if (ev(0, X) != ev(T, X)) return -1;
    std::vector<char> par(h->n, 0);
    for (int c = 0; c < T; c++) par[ev(c, X)] = par[ev(c, D0 - 1)] = 1;
    for (int c = 0; c < M; c++)
        for (int j = 0; j < X; j++)
            if (par[ev(c, j)]) return -1;
    std::vector<int> mark(h->n, -(1 << 29));
    auto conflict = [&](int c, int u) {
        for (int j = 0; j < X; j++)
            if (mark[ev(c, j)] >= u - dist) return true;
        return false;
    };
    auto take = [&](int c, int u) {
        for (int j = 0; j < X; j++) mark[ev(c, j)] = u;
    };
    o.first.clear();
    o.count.clear();
    int c = 0;
    while (c < T) {
        const int u = (int)o.first.size();
        if (conflict(c, u)) {   // touched by the previous window: leave a gap
            o.first.push_back(c);
            o.count.push_back(0);
            continue;
        }
        int cnt = 0;
        while (c + cnt < T && cnt < S && !conflict(c + cnt, u)) {
            take(c + cnt, u);
            cnt++;
        }
        o.first.push_back(c);
        o.count.push_back(cnt);
        c += cnt;
    }
    {
        int u = (int)o.first.size();
        if (conflict(T, u)) {
            o.first.push_back(T);
            o.count.push_back(0);
            u++;
        }
        take(T, u);
        o.first.push_back(T);
        o.count.push_back(1);
        o.tail = u;
    }
    // the next iteration's first windows follow the last ones: pad with empty
    // windows until no window within `dist` (cyclically) shares a variable
    for (;;) {
        const int nwin = (int)o.first.size();
        bool bad = false;
        for (int w0 = 0; w0 < dist && w0 < nwin; w0++)
            for (int k = 0; k < o.count[w0]; k++)
                for (int j = 0; j < X; j++) bad |= (mark[ev(o.first[w0] + k, j)] >= nwin + w0 - dist);
        if (!bad) break;
        o.first.push_back(M);
        o.count.push_back(0);
    }
    const int nw = (int)o.first.size();
    if (nw < R + 4) return -1;   // ring / table-ring sizes and parity reuse distance
    // forwarding (two passes over the cyclic schedule)
    std::vector<int> lw(h->n, -1), lk(h->n, 0), lj(h->n, 0);
    std::vector<uint16_t> fwd((size_t)nw * S * X, (uint16_t)FWD_NONE);
    std::vector<uint32_t> src((size_t)nw * S, 0);
    o.n_fwd = 0;
    for (int pass = 0; pass < 2; pass++)
        for (int u = 0; u < nw; u++)
            for (int k = 0; k < o.count[u]; k++) {
                const int cc = o.first[u] + k;
                for (int j = 0; j < X; j++) {
                    const uint32_t v = ev(cc, j);
                    if (pass == 1) {
                        const int gw = lw[v];
                        const int dW = (nw + u) - gw;
                        if (dW <= dist) return -1;   // violates the window rule
                        if (dW > dist && dW <= R + dist) {
                            const int w = gw % nw;
                            fwd[((size_t)u * S + k) * X + j] = (uint16_t)(dW << (6 + EB) | lk[v] << EB | lj[v]);
                            src[(size_t)w * S + lk[v]] |= 1u << lj[v];
                            o.n_fwd++;
                        }
                    }
                    lw[v] = pass * nw + u;
                    lk[v] = k;
                    lj[v] = j;
                }
            }
    if (!want_tab) return 0;
    o.tab.assign((size_t)nw * S * recw, 0u);
    for (int u = 0; u < nw; u++)
        for (int k = 0; k < S; k++) {
            uint32_t *rec = &o.tab[((size_t)u * S + k) * recw];
            for (int i = 0; i < (X + 1) / 2; i++) rec[D0 + 1 + i] = 0xFFFFFFFFu;
            if (k >= o.count[u]) {
                rec[D0] = (uint32_t)std::min(o.first[u], M - 1);   // a valid check, never stored
                continue;
            }
            const int cc = o.first[u] + k;
            for (int j = 0; j < h->check_deg[cc]; j++) rec[j] = ev(cc, j);
            if (u == o.tail) rec[D0 - 1] = ev(T - 1, D0 - 1);   // the last group-0 check's o variable
            bool any = false;
            for (int j = 0; j < X; j++) {
                const uint16_t f = fwd[((size_t)u * S + k) * X + j];
                if (f == FWD_NONE) continue;
                any = true;
                uint32_t &d = rec[D0 + 1 + j / 2];
                d = (j & 1) ? ((d & 0xFFFFu) | ((uint32_t)f << 16)) : ((d & 0xFFFF0000u) | f);
            }
            rec[D0] = (uint32_t)cc | M_ACT | (any ? M_FWD : 0u);
            if (X > 8)
                rec[coop_src_word(D0)] = src[(size_t)u * S + k];
            else
                rec[D0] |= src[(size_t)u * S + k] << SRC_SHIFT;
        }
    return 0;
}

namespace {

constexpr int kWS = 7;   // slab waves: S = 28 checks per window
// prefetch depth (windows): 3, or 2 for degree 22 (R + 1 prefetched windows of
// 21 V dwords per lane would not fit the 256 VGPRs of two waves per SIMD)
constexpr int coop_r(int d0) { return d0 > 16 ? 2 : 3; }

template <int D0>
int launch_d0(const CoopArgs &a, int grid, hipStream_t s, bool et)
{
    constexpr int R = coop_r(D0);
    if (et)
        hipLaunchKernelGGL((coop_decode<D0, kWS, R, true>), dim3(grid), dim3(64 * (kWS + 1)), 0, s, a);
    else
        hipLaunchKernelGGL((coop_decode<D0, kWS, R>), dim3(grid), dim3(64 * (kWS + 1)), 0, s, a);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace

bool coop_params_ok(const ldpc_params *p)
{
    // the unclamped chain needs 127 - msg_max >= T + offset (T <= msg_max - offset)
    return (p->algo == LDPC_ALGO_OMS || p->algo == LDPC_ALGO_MS) && p->var_min == -127 && p->var_max == 127 &&
           p->msg_max >= 0 && p->msg_max <= 63 && (p->algo == LDPC_ALGO_MS || (p->offset >= 0 && p->offset <= 63));
}

int coop_plan_windows(const ldpc_code *h, int S, int R, int dist, std::vector<int> &first, std::vector<int> &count,
                      int *tail, int *n_fwd)
{
    CoopPlan pl;
    if (coop_build_plan(h, S, R, dist, 0, pl, false) != 0) {
        first.clear();
        count.clear();
        return -1;
    }
    first = pl.first;
    count = pl.count;
    if (tail) *tail = pl.tail;
    if (n_fwd) *n_fwd = pl.n_fwd;
    return 0;
}

int coop_upload(const ldpc_code *h, CoopCode *cc)
{
    *cc = CoopCode{};
    if (!h->staircase || h->n_groups != 2) return LDPC_OK;
    const int d0 = h->group_deg[0];
    int recw;
    if (d0 == 7)
        recw = Geo<7>::RECW;
    else if (d0 == 10)
        recw = Geo<10>::RECW;
    else if (d0 == 14)
        recw = Geo<14>::RECW;
    else if (d0 == 22)
        recw = Geo<22>::RECW;
    else
        return LDPC_OK;
    CoopPlan pl;
    if (coop_build_plan(h, 4 * kWS, coop_r(d0), 1, recw, pl, true) != 0) return LDPC_OK;
    if (hipMalloc(&cc->d_tab, pl.tab.size() * 4) != hipSuccess) return ldpc_set_error(LDPC_ENOMEM, "coop tables");
    if (hipMemcpy(cc->d_tab, pl.tab.data(), pl.tab.size() * 4, hipMemcpyHostToDevice) != hipSuccess) {
        coop_free(cc);
        return ldpc_set_error(LDPC_EDEVICE, "coop table upload");
    }
    cc->valid = 1;
    cc->d0 = d0;
    cc->S = 4 * kWS;
    cc->R = coop_r(d0);
    cc->m0 = h->group_cnt[0];
    cc->d1 = h->group_deg[1];
    cc->nw = (int)pl.first.size();
    cc->tail = pl.tail;
    cc->n_fwd = pl.n_fwd;
    return LDPC_OK;
}

void coop_free(CoopCode *cc)
{
    (void)hipFree(cc->d_tab);
    (void)hipFree(cc->d_lc_pro);
    (void)hipFree(cc->d_lc_epi);
    *cc = CoopCode{};
}

static int launch_coop_iters(const DecodeLaunch &L, const CoopCode &cc, int iters, const uint8_t *live,
                             hipStream_t s, bool et = false)
{
    CoopArgs a;
    a.ev = L.d_edge_var;
    a.iters_used = L.iters_used;
    a.iters = iters;
    a.batch = L.batch;
    a.m0 = cc.m0;
    a.d1 = cc.d1;
    a.V = (int8_t *)L.V;
    a.Mc = L.msg;
    a.tab = cc.d_tab;
    a.stride = L.vpitch;   // V row pitch (the grid follows L.stride)
    a.G = cc.nw * iters;
    a.live = live;
    a.nw = cc.nw;
    a.tail = cc.tail;
    a.m = L.m;
    a.n = L.n;
    a.off = L.param;
    a.mm = L.msg_max;
    const int grid = L.stride / CW;
    a.remap = (grid % 8) == 0;
    if (cc.d0 == 7) return launch_d0<7>(a, grid, s, et);
    if (cc.d0 == 10) return launch_d0<10>(a, grid, s, et);
    if (cc.d0 == 14) return launch_d0<14>(a, grid, s, et);
    if (cc.d0 == 22) return launch_d0<22>(a, grid, s, et);
    return -1;
}

int launch_coop(const DecodeLaunch &L, const CoopCode &cc, hipStream_t s)
{
    if (!cc.valid || L.stride % 64) return -1;
    if (!L.early) {
        if (L.iters_used)
            hipLaunchKernelGGL(fill_iters_k, dim3((L.batch + 255) / 256), dim3(256), 0, s, L.batch, L.iters_used,
                               L.iters);
        return launch_coop_iters(L, cc, L.iters, nullptr, s);
    }
    // early termination in the kernel (coop_decode<.., ET>): one launch
    // (LDPC_COOP_ET_KERNEL=0: the per-iteration launches below)
    const char *ek = getenv("LDPC_COOP_ET_KERNEL");
    const bool in_kernel = !(ek && *ek && atoi(ek) == 0);
    if (in_kernel && L.iters_used) {
        if (L.iters == 0) {
            hipLaunchKernelGGL(fill_iters_k, dim3((L.batch + 255) / 256), dim3(256), 0, s, L.batch, L.iters_used, 0);
            return hipGetLastError() == hipSuccess ? 0 : -1;
        }
        return launch_coop_iters(L, cc, L.iters, nullptr, s, true);
    }
    // early termination: one launch per iteration (V, messages and the chain
    // input V[p_0] carry the state), then the syndrome of the live codewords
    if (coop_early_begin(L, s)) return -1;
    for (int it = 0; it < L.iters; it++)
        if (launch_coop_iters(L, cc, 1, L.live, s) || coop_early_after_iter(L, it, s)) return -1;
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int coop_early_begin(const DecodeLaunch &L, hipStream_t s)
{
    if (!L.live || !L.bad || !L.iters_used) return -1;
    const int nb = (L.stride + 255) / 256;
    hipLaunchKernelGGL(early_init_k, dim3(nb), dim3(256), 0, s, L.batch, L.stride, L.live, L.bad, L.iters_used,
                       L.iters);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int coop_early_after_iter(const DecodeLaunch &L, int it, hipStream_t s)
{
    const int nb = (L.batch + 255) / 256;
    // checks per syndrome thread: a codeword that is still failing late in
    // the decode often has few unsatisfied checks, so its threads walk whole
    // chunks; short chunks keep that walk (dependent gather rounds) short
    static const int kChunk = [] {
        const char *e = getenv("LDPC_SYND_CHUNK");
        const int v = (e && *e) ? atoi(e) : 64;
        return v >= 4 && v <= 4096 ? v : 64;
    }();
    // V (and its snapshot Vs) rows are L.vpitch codewords apart (the padded
    // pitch of the coop kernels); live / bad / iters_used are per codeword
    const dim3 sgrid((L.batch + 63) / 64, (L.m + kChunk - 1) / kChunk);
    hipLaunchKernelGGL(syndrome_k, sgrid, dim3(64), 0, s, (const int8_t *)L.V, L.vpitch, L.batch, L.d_edge_var,
                       L.d_group_deg, L.d_group_cnt, L.n_groups, L.m, kChunk, (const uint8_t *)L.live, L.bad);
    if (L.Vs)
        hipLaunchKernelGGL(snapshot_k, dim3((L.batch + 63) / 64, (L.n + kSnapRows - 1) / kSnapRows), dim3(64), 0, s,
                           (const int8_t *)L.V, L.Vs, L.vpitch, L.batch, L.n, (const uint8_t *)L.live,
                           (const uint32_t *)L.bad);
    hipLaunchKernelGGL(syndrome_finish_k, dim3(nb), dim3(256), 0, s, L.batch, L.live, L.bad, L.iters_used, it + 1);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int coop_early_end(const DecodeLaunch &L, hipStream_t s)
{
    if (!L.Vs) return 0;
    hipLaunchKernelGGL(merge_snapshot_k, dim3((L.batch + 63) / 64, (L.n + kSnapRows - 1) / kSnapRows), dim3(64), 0, s,
                       (int8_t *)L.V, (const int8_t *)L.Vs, L.vpitch, L.batch, L.n, (const uint8_t *)L.live);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
