// coop2.hip -- packed-pair variant of the workgroup-cooperative layered int8
// offset-min-sum decoder for the DVB-S2 staircase codes: the BASELINE.json
// headline path (DVB-S2 r1/2, 50 iterations).  Bit-exact with the reference's
// CDecoder_OMS_fixed_SSE::decode_8bits (code/x86/CDecoder/OMS/
// CDecoder_OMS_fixed_SSE.cpp:172-546) like coop.hip, whose window plan
// (coop_build_plan), staircase chain recurrence and period pipeline it
// shares.  What changes is the slab waves' data path.  On MI355X coop.hip is
// bound by instruction issue (about 370 instructions per slab wave and
// period, two slab waves per SIMD, ~3.5k cycles per period at 2.1 TB/s of
// HBM traffic), so this kernel spends fewer instructions per codeword:
//
// * a lane holds TWO codewords, one per 16-bit half of a VGPR, and evaluates
//   the check with gfx950 packed math (v_pk_sub_i16 / v_pk_add_i16 with
//   clamp, v_pk_min_i16, v_pk_max_i16, v_pk_ashrrev_i16) plus v_perm_b32 and
//   v_bfi_b32;
// * an int8 value x sits in a half as R(x) = 256 x + 255 (value in the high
//   byte, low byte all ones) and a message m as C(m) = 256 m.  Then
//   R(x) - C(m) = R(x - m), R(x) + C(m) = R(x + m), and the i16 saturation
//   0x7FFF is R(127): the reference's _mm_subs_epi8 / _mm_adds_epi8 upper
//   clamp for free.  |x| = max(R, 510 - R) stays in R form, and min / max /
//   compares are monotone in R;
// * V moves two bytes at a time (one u16 per pair) through structured buffer
//   loads and stores, address = group base + var * pitch + 2 * pair: no
//   address arithmetic on the VALU;
// * a check's messages for a pair are two dwords
//     MA: bits 2j, 2j+1 (codeword 0) and 16+2j, 17+2j (codeword 1) hold the
//         2-bit code of edge j: bit 0 = message negative, bit 1 = the edge got
//         cst2 (a_j != min1; ties give cst1 == cst2, so this is exact),
//     MB: bytes cst1_0, cst2_0, cst1_1, cst2_1,
//   (4 B per codeword and check, as coop.hip), and an old message is one
//   v_perm_b32 into each codeword's byte table [+cst1, -cst1, +cst2, -cst2];
// * inactive window slots point at a sink V row and a sink message row, so
//   every memory operation is unconditional; the forwarding ring is written
//   for every information edge.
// The workgroup owns 16 codewords: 8 pairs = 8 lanes per slot, 8 slots per
// slab wave, S = 8 WS checks per window.  With WS = 3 every wave has a SIMD of
// its own.  Early termination: one launch per iteration (coop.hip's syndrome
// driver); a converged codeword may share a lane with a live one, so instead
// of masking its stores it keeps iterating and its V column is snapshot when
// it converges and merged back at the end (snapshot_k / merge_snapshot_k).
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <type_traits>
#include <vector>

#include "coop.h"

#include "pk16.h"

namespace {

constexpr int WS_DEFAULT = 3;   // slab waves per role (S = 8 WS checks per window); LDPC_COOP2_WS = 3 | 4
#ifndef LDPC_COOP2_R
#define LDPC_COOP2_R 3
#endif
constexpr int R2 = LDPC_COOP2_R;   // prefetch depth (windows)
constexpr int DIST = 2;    // windows closer than DIST + 1 share no information variable (plan rule)
constexpr int DPER = 3;    // a window table's LDS-DMA is waited for DPER periods after its issue
constexpr int KAHEAD = R2 + 2 + DPER;   // ... which is KAHEAD windows ahead of the chain
constexpr int TQ = 16;     // window-table slots in LDS (>= KAHEAD + 2)
constexpr int RING = 8;    // forwarding ring windows (>= R2 + DIST)
constexpr int NSB = 3;     // pre -> post state buffers (a window's state lives 3 periods)

struct Coop2Args {
    int8_t *V;                     // V[n + 1][pitch]; row n is the sink of inactive slots
    uint8_t *Mc;                   // [pitch / 16][mrows][8 pairs][2] u32; row m is the sink
    const uint32_t *tab;           // [nw][S][RECW] slot records
    unsigned long long *stamps;    // diagnostic build: [grid][waves][4]
    const uint8_t *live;           // early termination: [pitch] 0 = converged (NULL: all live)
    int pitch, G, nw, tail, mrows, n, remap, prio, off;
    int pre_prio, post_prio;       // s_setprio of the pre / post waves (the chain wave: prio ? 2 : 0)
    uint32_t rmm, coff;            // R(msg_max), C(offset) per half
};

template <int D0>
struct Geo {
    static constexpr int X = D0 - 2;
    static constexpr int NFW = (X + 1) / 2;
    static constexpr int RECW = (D0 + 1 + NFW + 3) / 4 * 4;
};

template <int D0, int WS>
struct alignas(16) Smem2 {
    static constexpr int S = 8 * WS, X = Geo<D0>::X, RECW = Geo<D0>::RECW;
    uint32_t tab[TQ][S][RECW];     // slot records, window g in slot g % TQ
    int4 cst0[2][S][CW];           // chain constants (eps, A, B, co)   (pre -> chain)
    int2 cst1[2][S][CW];           //                 (L, H)
    int xin[2][CW][S];             // clamped x input of each slot      (chain -> post)
    uint32_t ring[RING][S][X][NP]; // V pairs (R form) of the last windows, for forwarding
    uint4 st[NSB][WS][4][64];      // one window's St2 per lane          (pre -> post)
};

template <int D0>
struct Pf2 {                       // prefetched raw inputs of one window
    uint32_t v[D0 - 1];            // V dwords (this pair + its neighbour): info edges, then edge D0-1 of the record
    uint32_t ma, mb;
};

template <int D0>
struct St2 {                       // one window between pre and post (R / C pairs): 16 dwords
    uint32_t c[D0 - 1];            // contributions (info, o); tail: new V
    uint32_t a[D0 - 1];            // |c| clipped
    uint32_t mx, min1, min2, sacc; // tail: min1 = MA, min2 = MB
};
static_assert(sizeof(St2<7>) == 64, "pre -> post state is four uint4 per lane");

// one slab wave: lane = (slot k, codeword pair q); the same slots in the pre
// role (prefetch + pre) and in the post role
template <int D0, int WS>
struct Slab2 {
    using SM = Smem2<D0, WS>;
    static constexpr int S = SM::S, X = SM::X, NFW = Geo<D0>::NFW;
    SM &sm;
    const Coop2Args &a;
    i32x4 vr, mr;                  // V rows of this group (stride pitch), message rows (stride 64)
    int k, q, w, lane, tail;
    uint32_t usel;                 // v_perm selector: this pair's two bytes of a V dword -> R pair
    PkK K;

    // whole aligned dwords (two pairs): a u16 load result carried across the
    // loop back-edge gets a zero-extension there, which waits for the load
    LDPC_DEV uint32_t ldv(uint32_t var) const { return sbuf_load_u32(vr, (int)var, 4 * (q >> 1), 0, 0); }
    LDPC_DEV void stv(uint32_t var, uint32_t r) const
    {
        sbuf_store_u16((unsigned short)pack_v(r), vr, (int)var, 2 * q, 0, 0);
    }

    // issue the loads of the window in table slot ts
    LDPC_DEV void prefetch(int ts, Pf2<D0> &pf) const
    {
        const uint32_t *r = sm.tab[ts][k];
        uint32_t var[D0];
#pragma unroll
        for (int j = 0; j < D0; j++) var[j] = r[j];
        const uint32_t meta = r[D0];
#pragma unroll
        for (int j = 0; j < X; j++) pf.v[j] = ldv(var[j]);
        pf.v[X] = ldv(var[D0 - 1]);   // o edge (tail: its last edge, swapped by the upload)
        const i32x2 m = sbuf_load_v2(mr, (int)(meta & COOP_CHK_MASK), 8 * q, 0, 0);
        pf.ma = (uint32_t)m.x;
        pf.mb = (uint32_t)m.y;
    }

    // V pairs written DIST+1 .. R+DIST windows ago replace the loaded ones (rare)
    LDPC_DEV void forward(int ts, int g, uint32_t *v) const
    {
        const uint32_t *r = sm.tab[ts][k];
        uint32_t fw[NFW];
#pragma unroll
        for (int i = 0; i < NFW; i++) fw[i] = r[D0 + 1 + i];
#pragma unroll
        for (int j = 0; j < X; j++) {
            const uint32_t code = (fw[j >> 1] >> ((j & 1) * 16)) & 0xFFFFu;
            const int dw = (int)(code >> 9);
            if (code != COOP_FWD_NONE && g >= dw) v[j] = sm.ring[(g - dw) & (RING - 1)][(code >> 3) & 63][code & 7][q];
        }
    }

    // pre of window g (local index u): chain constants -> cst[g & 1], state -> st[g % NSB]
    LDPC_DEV void pre(int g, int u, const Pf2<D0> &pf) const
    {
        const int ts = g & (TQ - 1), cb = g & 1;
        const uint32_t meta = sm.tab[ts][k][D0];
        uint32_t v[D0 - 1];
#pragma unroll
        for (int j = 0; j < D0 - 1; j++) v[j] = unpack_v(pf.v[j], usel);
        if (__any((meta & COOP_M_FWD) != 0)) forward(ts, g, v);
        const MsgTab t = msg_tab(pf.mb);
        const uint32_t MA = pf.ma, rmm = K.rmm, coff = K.coff, neg127 = K.neg127;
        uint32_t min1 = R127, min2 = R127, sacc = 0;
        St2<D0> s;
        int eps[2], A[2], B[2], co[2], L[2], H[2];
        if (u != tail) {
            // first degree group: a = min(|c|, msg_max) (OMS_fixed_SSE.cpp:211)
            static_for<0, X>([&](auto jc) {
                constexpr int J = decltype(jc)::value;
                const uint32_t c = pk_max(pk_sub_sat(v[J], old_msg<J>(MA, t)), neg127);
                const uint32_t aj = pk_min(abs_r(c, K.c510), rmm);
                s.c[J] = c;
                s.a[J] = aj;
                sacc ^= c;
                min2 = pk_max(min1, pk_min(aj, min2));
                min1 = pk_min(min1, aj);
            });
            // chain constants, as coop.hip: T = cst(min over the info edges),
            // eps = -1 iff the info edges' sign parity (odd-degree flip
            // included) is odd, co = the o-edge contribution, mx = the x-edge
            // old message
            const uint32_t T = pk_max(pk_sub(min1, coff), K.r0);
            const uint32_t kb = sacc ^ ((D0 & 1) ? SIGNS : 0u);
            const uint32_t cor = pk_max(pk_sub_sat(v[X], old_msg<D0 - 1>(MA, t)), neg127);
            const uint32_t ao = pk_min(abs_r(cor, K.c510), rmm);
            s.c[X] = cor;
            s.a[X] = ao;
            s.sacc = sacc ^ cor;
            s.min2 = pk_max(min1, pk_min(ao, min2));
            s.min1 = pk_min(min1, ao);
            const uint32_t mx = old_msg<X>(MA, t);
            s.mx = mx;
#pragma unroll
            for (int h = 0; h < 2; h++) {
                const int th = hi8(T, h), ch = hi8(cor, h), mh = hi8(mx, h);
                eps[h] = 1 - 2 * (int)((kb >> (15 + 16 * h)) & 1u);
                co[h] = ch;
                A[h] = ch - eps[h] * (mh + a.off);
                B[h] = ch - eps[h] * (mh - a.off);
                L[h] = ch - th;
                H[h] = ch + th;
            }
        } else {
            // the tail check (later degree group: a = |min(c, msg_max)|,
            // OMS_fixed_SSE.cpp:293,314) has no chain input: finish it here
            static_for<0, X + 1>([&](auto jc) {
                constexpr int J = decltype(jc)::value;
                const uint32_t c = pk_max(pk_sub_sat(v[J], old_msg<J>(MA, t)), neg127);
                const uint32_t aj = abs_r(pk_min(c, rmm), K.c510);
                s.c[J] = c;
                s.a[J] = aj;
                sacc ^= c;
                min2 = pk_max(min1, pk_min(aj, min2));
                min1 = pk_min(min1, aj);
            });
            const uint32_t k1 = pk_min(pk_max(pk_sub(min2, coff), K.r0), rmm) & HIBYTES;
            const uint32_t k2 = pk_min(pk_max(pk_sub(min1, coff), K.r0), rmm) & HIBYTES;
            const uint32_t P = (sacc ^ (((D0 - 1) & 1) ? SIGNS : 0u)) & SIGNS;
            uint32_t MAn = 0;
            static_for<0, X + 1>([&](auto jc) {
                constexpr int J = decltype(jc)::value;
                s.c[J] = new_msg<J>(s.c[J], s.a[J], min1, k1, k2, P, MAn, neg127);
            });
            s.mx = 0;
            s.sacc = 0;
            s.min1 = MAn;
            s.min2 = perm(k2, k1, 0x07030501u);
#pragma unroll
            for (int h = 0; h < 2; h++) {
                const int y = hi8(s.c[X], h);
                eps[h] = 0;
                A[h] = B[h] = co[h] = L[h] = H[h] = y;
            }
        }
        if (__any(!(meta & COOP_M_ACT))) {   // pass-through slots: Y_k = Y_{k-1}
            if (!(meta & COOP_M_ACT)) {
#pragma unroll
                for (int h = 0; h < 2; h++) {
                    eps[h] = 1;
                    A[h] = B[h] = co[h] = 0;
                    L[h] = -1024;
                    H[h] = 1024;
                }
            }
        }
#pragma unroll
        for (int h = 0; h < 2; h++) {
            sm.cst0[cb][k][2 * q + h] = make_int4(eps[h], A[h], B[h], co[h]);
            sm.cst1[cb][k][2 * q + h] = make_int2(L[h], H[h]);
        }
        const uint4 *sp = (const uint4 *)&s;
#pragma unroll
        for (int i = 0; i < 4; i++) sm.st[(unsigned)g % NSB][w][i][lane] = sp[i];
    }

    // post of window g (local index u): state from st[g % NSB], x inputs from xin[g & 1]
    LDPC_DEV void post(int g, int u) const
    {
        const int ts = g & (TQ - 1), xb = g & 1, rs = g & (RING - 1);
        St2<D0> s;
        uint4 *sp = (uint4 *)&s;
#pragma unroll
        for (int i = 0; i < 4; i++) sp[i] = sm.st[(unsigned)g % NSB][w][i][lane];
        const uint32_t *r = sm.tab[ts][k];
        uint32_t var[D0];
#pragma unroll
        for (int j = 0; j < D0; j++) var[j] = r[j];
        const uint32_t meta = r[D0];
        const uint32_t x0 = (uint32_t)sm.xin[xb][2 * q][k], x1 = (uint32_t)sm.xin[xb][2 * q + 1][k];
        const uint32_t xr = perm(x1, x0, 0x040d000du);   // clamped by the chain -> R pair
        uint32_t MA, MB;
        if (u != tail) {
            const uint32_t cx = pk_max(pk_sub_sat(xr, s.mx), K.neg127);
            const uint32_t ax = pk_min(abs_r(cx, K.c510), K.rmm);
            const uint32_t sacc = s.sacc ^ cx;
            const uint32_t min2 = pk_max(s.min1, pk_min(ax, s.min2)), min1 = pk_min(ax, s.min1);
            const uint32_t k1 = pk_max(pk_sub(min2, K.coff), K.r0) & HIBYTES;   // <= msg_max already
            const uint32_t k2 = pk_max(pk_sub(min1, K.coff), K.r0) & HIBYTES;
            const uint32_t P = (sacc ^ ((D0 & 1) ? SIGNS : 0u)) & SIGNS;
            MA = 0;
            static_for<0, X>([&](auto jc) {
                constexpr int J = decltype(jc)::value;
                const uint32_t vn = new_msg<J>(s.c[J], s.a[J], min1, k1, k2, P, MA, K.neg127);
                stv(var[J], vn);
                sm.ring[rs][k][J][q] = vn;
            });
            stv(var[X], new_msg<X>(cx, ax, min1, k1, k2, P, MA, K.neg127));
            // the o edge: message bits only (the next check rewrites V[o] as its x edge)
            (void)new_msg<D0 - 1>(s.c[X], s.a[X], min1, k1, k2, P, MA, K.neg127);
            MB = perm(k2, k1, 0x07030501u);
        } else {
            static_for<0, X>([&](auto jc) {
                constexpr int J = decltype(jc)::value;
                stv(var[J], s.c[J]);
                sm.ring[rs][k][J][q] = s.c[J];
            });
            stv(var[D0 - 1], s.c[X]);   // the tail's last edge (record entries X, D0-1 swapped)
            stv(var[X], xr);            // V of the last group-0 check's o edge: only the chain had it
            MA = s.min1;
            MB = s.min2;
        }
        i32x2 m;
        m.x = (int)MA;
        m.y = (int)MB;
        sbuf_store_v2(m, mr, (int)(meta & COOP_CHK_MASK), 8 * q, 0, 0);
    }
};

// chain steps [K0, K1) of the window in constant buffer buf for the 16
// codewords (lanes 0..15): the recurrence of coop.hip, one asm block per step
// (clamped x input for post, two mad24, two med3) so that hipcc pads no
// wait states between its four dependent instructions
LDPC_DEV unsigned long long stamp();

template <int D0, int WS, int K0, int K1, bool STAMP = false>
LDPC_DEV void chain_steps2(Smem2<D0, WS> &sm, int buf, int c, int &Y, unsigned long long *sL = nullptr)
{
    constexpr int NK = K1 - K0;
    int4 q0[NK];
    int2 q1[NK];
#pragma unroll
    for (int i = 0; i < NK; i++) {
        q0[i] = sm.cst0[buf][K0 + i][c];
        q1[i] = sm.cst1[buf][K0 + i][c];
    }
    if constexpr (STAMP) {   // diagnostic: the constants' LDS latency apart from the steps
        const unsigned long long t = stamp();
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        *sL += stamp() - t;
    }
    const int lo = -127, hi = 127;
    int xv[4];
#pragma unroll
    for (int i = 0; i < NK; i++) {
        const int k = K0 + i;
        int p, qq;
        asm("v_med3_i32 %1, %0, %8, %9\n\t"
            "v_mad_i32_i24 %2, %0, %4, %5\n\t"
            "v_mad_i32_i24 %3, %0, %4, %6\n\t"
            "v_med3_i32 %2, %2, %7, %3\n\t"
            "v_med3_i32 %0, %2, %10, %11"
            : "+v"(Y), "=&v"(xv[k & 3]), "=&v"(p), "=&v"(qq)
            : "v"(q0[i].x), "v"(q0[i].y), "v"(q0[i].z), "v"(q0[i].w), "v"(lo), "v"(hi), "v"(q1[i].x),
              "v"(q1[i].y));
        if ((k & 3) == 3) *(int4 *)&sm.xin[buf][c][k - 3] = make_int4(xv[0], xv[1], xv[2], xv[3]);
    }
}

LDPC_DEV unsigned long long stamp()
{
    unsigned long long t;
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    __builtin_amdgcn_sched_barrier(0);
    return t;
}

// Waves: 0 .. WS-1 "pre" (loads + pre), WS the chain, WS+1 .. 2 WS "post".
// Workgroup waves go to the SIMDs cyclically, so pre wave i and post wave i
// share a SIMD and the chain has one of its own.  One barrier per period p:
//   chain: steps of window p; LDS-DMA of the table of window p + KAHEAD
//   pre:   loads of window p+1+R, pre of window p+1
//   post:  post of window p-1
// The plan keeps windows within DIST = 2 free of shared information
// variables, so post(p-1) and pre(p+1) need no ordering; values written 3 ..
// R+2 windows before a pre are forwarded through the LDS ring, and every
// other earlier write is ordered before the loads by a barrier.
template <int D0, int WS, bool STAMP>
__global__ void __launch_bounds__(64 * (2 * WS + 1)) coop2_decode(Coop2Args a)
{
    using SM = Smem2<D0, WS>;
    constexpr int S = SM::S, X = SM::X, RECW = SM::RECW, R = R2;
    constexpr int U = R + 1;                  // prefetch buffers repeat
    static_assert(TQ >= KAHEAD + 2 && RING >= R + DIST && NSB >= 3, "ring sizes");
    __shared__ SM sm;

    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const int nb = gridDim.x, id = blockIdx.x;
    const int wg = a.remap ? (id & 7) * (nb >> 3) + (id >> 3) : id;   // XCD-aware codeword groups
    const int G = a.G;
    if (G == 0) return;
    // early termination: a workgroup whose 16 codewords all converged skips
    // the iteration (the others iterate all 16; converged ones were snapshot)
    if (a.live && !__syncthreads_or(threadIdx.x < CW && a.live[wg * CW + threadIdx.x])) return;
    unsigned long long sA = 0, sB = 0, sL = 0, t0 = 0, tx = 0;
    auto write_stamps = [&]() {
        if (STAMP && lane == 0) {
            unsigned long long *o = a.stamps + ((size_t)id * (2 * WS + 1) + wave) * 4;
            o[0] = sA;
            o[1] = sB | sL << 32;
            o[2] = stamp() - t0;
            o[3] = (unsigned long long)G | (unsigned long long)__builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11)) << 32;
        }
    };

    if (wave == WS) {
        // ------------------------------------------------------------ chain wave
        if (a.prio) __builtin_amdgcn_s_setprio(2);
        constexpr int NCH = S * RECW / 4;   // 16-B chunks per window table
        constexpr int CPL = (NCH + 63) / 64;
        static_assert(CPL * DPER <= 63, "table staging");
        const int c = lane & 15;
        // window u's slot records -> LDS slot by LDS-DMA, CPL instructions
        auto stage = [&](int u, int slot) {
            const uint4 *src = (const uint4 *)(a.tab + (size_t)u * S * RECW);
            const uint32_t dst = (uint32_t)(uintptr_t)&sm.tab[slot][0][0];
#pragma unroll
            for (int i = 0; i < CPL; i++)
                if (lane + 64 * i < NCH) dma16(src + 64 * i + lane, dst + 1024 * i);
        };
        for (int w = 0; w < KAHEAD; w++) stage(w % a.nw, w);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        int Y = a.V[(size_t)a.tab[X] * (uint32_t)a.pitch + (uint32_t)(wg * CW + c)];   // x input of check 0
        int un = KAHEAD % a.nw;
        __syncthreads();   // prologue 1: tables of windows 0 .. KAHEAD-1 in LDS
        __syncthreads();   // prologue 2: constants of window 0 in LDS
        const bool cl = lane < CW;
        if (STAMP) t0 = stamp();
        for (int p = 0; p <= G; p++) {
            if (STAMP) tx = stamp();
            if (p < G && cl) {
                if constexpr (S <= 24) {
                    chain_steps2<D0, WS, 0, S, STAMP>(sm, p & 1, c, Y, &sL);
                } else {   // constants of 16 steps at a time (VGPRs)
                    chain_steps2<D0, WS, 0, S / 2, STAMP>(sm, p & 1, c, Y, &sL);
                    chain_steps2<D0, WS, S / 2, S, STAMP>(sm, p & 1, c, Y, &sL);
                }
            }
            if (STAMP) sB += stamp() - tx;
            stage(un, (p + KAHEAD) & (TQ - 1));
            un = (un + 1 == a.nw) ? 0 : un + 1;
            // the tables DMA'd DPER periods ago have landed (the next period's
            // loads read window p+R+2, issued at period p+R+2-KAHEAD = p-DPER)
            asm volatile("s_waitcnt vmcnt(%0)" ::"n"(CPL * DPER) : "memory");
            if (STAMP) sA += stamp() - tx;
            __syncthreads();
        }
        write_stamps();
        return;
    }

    const bool is_pre = wave < WS;
    const int w = is_pre ? wave : wave - WS - 1;
    Slab2<D0, WS> sl{sm,
                     a,
                     buffer_rsrc(a.V + (size_t)wg * CW, (uint32_t)a.pitch, (uint32_t)(a.n + 1)),
                     buffer_rsrc(a.Mc + (size_t)wg * a.mrows * MREC, (uint32_t)MREC, (uint32_t)a.mrows),
                     8 * w + (lane >> 3),
                     lane & 7,
                     w,
                     lane,
                     a.tail,
                     0x010d000du + (uint32_t)(lane & 1) * 0x02000200u,
                     PkK{opaque(RNEG127), opaque(R0), opaque(C510), opaque(a.rmm), opaque(a.coff)}};
    auto next = [&](int &u) { u = (u + 1 == a.nw) ? 0 : u + 1; };
    __syncthreads();   // prologue 1: tables in LDS

    if (is_pre) {
        // ------------------------------------------------------ pre waves
        if (a.pre_prio) __builtin_amdgcn_s_setprio(1);
        Pf2<D0> pf[R + 1];
#pragma unroll
        for (int i = 0; i <= R; i++) sl.prefetch(i, pf[i]);   // nw > R + 3
        sl.pre(0, 0, pf[0]);
        __syncthreads();   // prologue 2
        if (STAMP) t0 = stamp();
        int uB = 1 % a.nw;   // local index of window p+1
        // period p: loads of window p+1+R into pf[(p+R+1) % U], pre of window
        // p+1 from pf[(p+1) % U]
        auto step = [&](auto sc, int p) {
            constexpr int s = decltype(sc)::value;   // p % U
            if (STAMP) tx = stamp();
            sl.prefetch((p + 1 + R) & (TQ - 1), pf[(s + R + 1) % U]);
            sl.pre(p + 1, uB, pf[(s + 1) % U]);
            if (STAMP) sA += stamp() - tx;
            __syncthreads();
            next(uB);
        };
        const int np = G + 1, nfull = np / U;
        int p = 0;
        for (int i = 0; i < nfull; i++, p += U)
            static_for<0, U>([&](auto jc) { step(jc, p + decltype(jc)::value); });
        const int rem = np - nfull * U;
        static_for<0, U - 1>([&](auto jc) {
            if (rem > decltype(jc)::value) step(jc, p + decltype(jc)::value);
        });
    } else {
        // ----------------------------------------------------- post waves
        if (a.post_prio) __builtin_amdgcn_s_setprio(1);
        __syncthreads();   // prologue 2
        if (STAMP) t0 = stamp();
        __syncthreads();   // period 0: nothing to post yet
        int uA = 0;        // local index of window p-1
        for (int p = 1; p <= G; p++) {
            if (STAMP) tx = stamp();
            sl.post(p - 1, uA);
            if (STAMP) sA += stamp() - tx;
            __syncthreads();
            next(uA);
        }
    }
    write_stamps();
}

__global__ void fill_iters2_k(int batch, int32_t *iters_used, int iters)
{
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b < batch) iters_used[b] = iters;
}

int env_int(const char *name, int def)
{
    const char *e = getenv(name);
    return (e && *e) ? atoi(e) : def;
}

// diagnostic build (LDPC_COOP2_STAMP=1): per-period cycles of each wave role
template <int WS>
void report_stamps(const unsigned long long *d, int grid, hipStream_t s)
{
    constexpr int nwaves = 2 * WS + 1;
    std::vector<unsigned long long> h((size_t)grid * nwaves * 4);
    if (hipStreamSynchronize(s) != hipSuccess ||
        hipMemcpy(h.data(), d, h.size() * sizeof(h[0]), hipMemcpyDeviceToHost) != hipSuccess)
        return;
    // role: 0 pre, 1 chain, 2 post; work = cycles between the period's barriers
    double work[3] = {0, 0, 0}, wmax[3] = {0, 0, 0}, total = 0, chain_steps = 0, chain_lds = 0;
    int cnt[3] = {0, 0, 0};
    std::vector<double> per_wave(nwaves, 0.0), per_wave_max(nwaves, 0.0);
    std::vector<int> simd(nwaves, -1);
    for (int b = 0; b < grid; b++)
        for (int w = 0; w < nwaves; w++) {
            const unsigned long long *o = &h[((size_t)b * nwaves + w) * 4];
            const double G = (o[3] & 0xffffffffu) ? (double)(o[3] & 0xffffffffu) : 1.0;
            const int role = w < WS ? 0 : (w == WS ? 1 : 2);
            if (b == 0) simd[w] = (int)((o[3] >> 36) & 3);   // HW_ID SIMD_ID of workgroup 0's waves
            work[role] += o[0] / G;
            wmax[role] = std::max(wmax[role], o[0] / G);
            per_wave[w] += o[0] / G / grid;
            per_wave_max[w] = std::max(per_wave_max[w], o[0] / G);
            if (role == 1) {
                chain_steps += (o[1] & 0xffffffffu) / G;
                chain_lds += (o[1] >> 32) / G;
            }
            cnt[role]++;
            total += o[2] / G;
        }
    fprintf(stderr,
            "coop2 stamps [cycles per period]: total %.0f | pre %.0f (max %.0f) | chain %.0f (max %.0f; steps %.0f, "
            "of which constants wait %.0f) | post %.0f (max %.0f)\n",
            total / (grid * nwaves), work[0] / cnt[0], wmax[0], work[1] / cnt[1], wmax[1], chain_steps / cnt[1],
            chain_lds / cnt[1], work[2] / cnt[2], wmax[2]);
    fprintf(stderr, "coop2 stamps per wave (mean/max):");
    for (int w = 0; w < nwaves; w++) fprintf(stderr, " %d:%.0f/%.0f@simd%d", w, per_wave[w], per_wave_max[w], simd[w]);
    fprintf(stderr, "\n");
}

template <int WS>
int launch_ws(const Coop2Args &a, int grid, bool stamped, hipStream_t s)
{
    constexpr int threads = 64 * (2 * WS + 1);
    if (stamped)
        hipLaunchKernelGGL((coop2_decode<7, WS, true>), dim3(grid), dim3(threads), 0, s, a);
    else
        hipLaunchKernelGGL((coop2_decode<7, WS, false>), dim3(grid), dim3(threads), 0, s, a);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace

bool coop2_params_ok(const ldpc_params *p) { return coop_params_ok(p); }

// the V descriptor's record stride is a 14-bit byte count
bool coop2_stride_ok(int stride) { return stride > 0 && stride % 64 == 0 && stride < (1 << 14); }

size_t coop2_msg_bytes(const ldpc_code *h, int stride) { return (size_t)(h->m + 1) * (size_t)stride * 4; }

int coop2_upload(const ldpc_code *h, CoopCode *cc)
{
    *cc = CoopCode{};
    constexpr int D0 = 7, X = D0 - 2, RECW = Geo<D0>::RECW;
    if (!h->staircase || h->n_groups != 2 || h->group_deg[0] != D0) return LDPC_OK;
    const int ws = env_int("LDPC_COOP2_WS", WS_DEFAULT);
    if (ws != 3 && ws != 4) return ldpc_set_error(LDPC_EINVAL, "LDPC_COOP2_WS must be 3 or 4");
    const int S = 8 * ws;
    CoopPlan pl;
    if (coop_build_plan(h, S, R2, DIST, RECW, pl, true) != 0) return LDPC_OK;
    const int nw = (int)pl.first.size();
    for (int u = 0; u < nw; u++)
        for (int k = 0; k < S; k++) {
            uint32_t *rec = &pl.tab[((size_t)u * S + k) * RECW];
            if (k >= pl.count[u]) {   // inactive slot: sink V row n, sink message row m, no flags
                for (int j = 0; j < D0; j++) rec[j] = (uint32_t)h->n;
                rec[D0] = (uint32_t)h->m;
            } else if (u == pl.tail) {
                std::swap(rec[X], rec[D0 - 1]);   // prefetch always loads record entry D0-1
            }
        }
    if (hipMalloc(&cc->d_tab, pl.tab.size() * 4) != hipSuccess) return ldpc_set_error(LDPC_ENOMEM, "coop2 tables");
    if (hipMemcpy(cc->d_tab, pl.tab.data(), pl.tab.size() * 4, hipMemcpyHostToDevice) != hipSuccess) {
        coop_free(cc);
        return ldpc_set_error(LDPC_EDEVICE, "coop2 table upload");
    }
    cc->valid = 1;
    cc->d0 = D0;
    cc->S = S;
    cc->R = R2;
    cc->nw = nw;
    cc->tail = pl.tail;
    cc->n_fwd = pl.n_fwd;
    return LDPC_OK;
}

static int launch_coop2_iters(const DecodeLaunch &L, const CoopCode &cc, int iters, const uint8_t *live,
                              hipStream_t s);

int launch_coop2(const DecodeLaunch &L, const CoopCode &cc, hipStream_t s)
{
    if (!cc.valid || !coop2_stride_ok(L.stride)) return -1;
    if (L.early) {
        // one launch per iteration as coop.hip; converged codewords keep
        // iterating inside live workgroups, so their V is snapshot when they
        // converge and merged back at the end (L.Vs)
        if (!L.Vs || coop_early_begin(L, s)) return -1;
        for (int it = 0; it < L.iters; it++)
            if (launch_coop2_iters(L, cc, 1, L.live, s) || coop_early_after_iter(L, it, s)) return -1;
        return coop_early_end(L, s);
    }
    if (L.iters_used)
        hipLaunchKernelGGL(fill_iters2_k, dim3((L.batch + 255) / 256), dim3(256), 0, s, L.batch, L.iters_used,
                           L.iters);
    return launch_coop2_iters(L, cc, L.iters, nullptr, s);
}

static int launch_coop2_iters(const DecodeLaunch &L, const CoopCode &cc, int iters, const uint8_t *live,
                              hipStream_t s)
{
    Coop2Args a{};
    a.live = live;
    a.V = (int8_t *)L.V;
    a.Mc = (uint8_t *)L.msg;
    a.tab = cc.d_tab;
    a.pitch = L.stride;
    a.G = cc.nw * iters;
    a.nw = cc.nw;
    a.tail = cc.tail;
    a.mrows = L.m + 1;
    a.n = L.n;
    a.off = L.param;
    a.rmm = (uint32_t)(L.msg_max * 256 + 255) * 0x00010001u;
    a.coff = (uint32_t)(L.param * 256) * 0x00010001u;
    a.prio = env_int("LDPC_COOP2_PRIO", 1);
    a.pre_prio = env_int("LDPC_COOP2_PRE_PRIO", 0);
    a.post_prio = env_int("LDPC_COOP2_POST_PRIO", 0);
    const int grid = L.stride / CW;
    a.remap = (grid % 8) == 0;
    const int ws = cc.S / 8, nwaves = 2 * ws + 1;
    const bool stamped = env_int("LDPC_COOP2_STAMP", 0) != 0;
    if (stamped) {
        const size_t bytes = (size_t)grid * nwaves * 4 * sizeof(unsigned long long);
        if (hipMalloc(&a.stamps, bytes) != hipSuccess) return -1;
        (void)hipMemsetAsync(a.stamps, 0, bytes, s);
    }
    const int rc = ws == 4 ? launch_ws<4>(a, grid, stamped, s) : launch_ws<3>(a, grid, stamped, s);
    if (stamped) {
        if (rc == 0) (ws == 4 ? report_stamps<4>(a.stamps, grid, s) : report_stamps<3>(a.stamps, grid, s));
        (void)hipFree(a.stamps);
    }
    return rc;
}
