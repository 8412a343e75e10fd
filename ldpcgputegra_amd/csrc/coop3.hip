// coop3.hip -- the DVB-S2 staircase-code decoder, third generation: the
// BASELINE.json headline path (DVB-S2 r1/2, 50 iterations, int8 OMS).
// Bit-exact with the reference's CDecoder_OMS_fixed_SSE::decode_8bits
// (code/x86/CDecoder/OMS/CDecoder_OMS_fixed_SSE.cpp:172-546), like coop.hip /
// coop2.hip, whose window plan (coop_build_plan), message format and
// packed-pair arithmetic (pk16.h) it shares.  What changes is the workgroup's
// organisation, built from what bounds coop2 on MI355X:
//
// * slab waves do BOTH halves of a check (pre: gather V + old messages,
//   contributions, min1 / min2 / signs and the chain constants; post: new
//   messages and V) for the same 8 slots, so a window's state stays in VGPRs
//   between its pre (period g-1) and its post (period g+1): no pre -> post
//   LDS round trip (coop2 moved 64 B per lane and period through LDS);
// * the chain (the serial staircase recurrence, one step per check) runs in
//   i16: v_pk_mad_i16 evaluates eps*Y + A and eps*Y + B at once, two
//   v_med3_i16 with op_sel apply the offset dead zone and the [L, H] clamp --
//   3 dependent instructions per check (coop2: 5), constants from ONE
//   ds_read_b128 per step; step outputs are written alternately into the low
//   / high halves of four VGPRs (op_sel dst), so 8 steps' x inputs leave in
//   one ds_write_b128;
// * WS = 6 slab waves (S = 48 checks per window, the plan fills ~45: DVB-S2
//   r1/2 has q = 90) two per SIMD on SIMDs 0-2, the chain wave alone on SIMD
//   3 with the highest priority;
// * a window's checks are permuted over its slots (coop3_upload): the chain
//   still runs them in check order (each record carries its chain step), and
//   every distance-2 forwarding source and reader sits in slab wave 0, so no
//   wave ever waits for another inside a period (one s_barrier per period);
// * vector memory -- the bound on MI355X: each check moves 6 scattered 16-B
//   V row pieces each way per 16 codewords, and the CU's texture path stalls
//   on the scattered stores -- is issued at the start and middle of a
//   period, never at its end: stores one barrier after their post, LDS-DMA
//   gathers R = 2 windows ahead.
//
// Period p (one s_barrier): chain = steps of window p; slab waves = post of
// window p-1, pre of window p+1, stores of window p-2, gathers of window
// p+1+R.  The plan (dist 1) keeps neighbouring windows free of shared
// information variables; values written 2 .. R+3 windows before a pre are
// forwarded through a 4-window LDS stage ring.
//
// The chain recurrence (check i, x edge input Y = V[p_{i-1}]):
//   V[p_i] = clamp(c_o + eps * sign(c_x) * min(max(|c_x| - off, 0), T), +-127)
//   c_x = Y - m_x, c_o = V[p_i] - m_o (old messages), eps = sign parity of the
//   information edges (odd-degree flip included), T = cst(min over them);
// = med3(med3(eps*Y + A, c_o, eps*Y + B), L, H) with A = c_o - eps*m_x - off,
//   B = c_o - eps*m_x + off, L = max(c_o - T, -127), H = min(c_o + T, 127).
// NMS (CDecoder_NMS_fixed_SSE.cpp:188-240: cst = (min * factor) >> 5, no
// offset): the o message is eps * sign(c_x) * min(trunc(|c_x| f / 32), T), so
//   V[p_i] = med3(med3(t >> 5, c_o, (t + 31) >> 5), L, H),  t = eps f Y + A,
// with A = 32 c_o - eps f m_x (floor and ceiling of c_o + eps f c_x / 32 in
// the two halves of one v_pk_mad_i16, the median with c_o truncates toward
// c_o): 4 dependent instructions per check.
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <type_traits>
#include <vector>

#include "coop.h"

#include "pk16.h"

__device__ void sbuf_store_v4(i32x4 v, i32x4 rsrc, int index, int offset, int soffset, int aux)
    __asm("llvm.amdgcn.struct.buffer.store.v4i32");

namespace {

constexpr int D0 = 7, X = D0 - 2;   // first-group check degree, information edges per check
constexpr int NFW = (X + 1) / 2;    // forwarding-code dwords per record
constexpr int RECW = (D0 + 1 + NFW + 3) / 4 * 4;
constexpr int DPER = 3;             // a window table's LDS-DMA is waited for DPER periods after its issue
constexpr int TQ = 16;              // window-table slots in LDS
constexpr int STG_RING = 8192;      // bytes per forwarding-ring slot (power of two: see fwd_code3)

template <int WS, int R>
struct Cfg {
    static constexpr int S = 8 * WS;                   // checks per window
    static constexpr int KAHEAD = R + 2 + DPER;        // tables staged KAHEAD windows ahead of the chain
    static constexpr int NI = R + 1;                   // LDS-DMA input windows in flight per slab wave
    static constexpr int NS = R + 1 < 3 ? 3 : R + 1;   // window states in VGPRs (pre at p-1, post at p+1)
    static constexpr int U = NS;                       // periods unrolled (multiple of NI and NS)
    static constexpr int NR = 4;                       // staged-output windows: window g's entries are read in
                                                       // periods g+1 .. g+R+2 (stores, forwards)
    static constexpr int CHW = WS >= 3 ? 3 : WS;       // the chain wave (waves go to SIMDs 0,2,1,3,0,2,1: wave 3
                                                       // has a SIMD of its own for WS = 3 and WS = 6)
    static constexpr int NB = S / 8;                   // chain blocks of 8 steps
    static_assert(TQ >= KAHEAD + 2, "table ring: a window's records are read until its stores");
    static_assert(NR == 4 && R + 2 <= NR && 8 * (S + 1) * 16 <= STG_RING,
                  "forwarding ring: codes carry (g - dW) mod 4 for dW = 2 .. R+3");
    static_assert(U % NI == 0 && U % NS == 0, "unroll");
};

template <int WS, int R>
struct alignas(16) Smem3 {
    using CF = Cfg<WS, R>;
    static constexpr int S = CF::S, NI = CF::NI, NR = CF::NR;
    uint4 stg[NR][STG_RING / 16];     // new V of a window, [record entry * (S + 1) + slot] x 16 codewords (int8,
                                      // entries padded: the stores' reads of 8 entries are conflict-free): the
                                      // V stores' staging and the forwarding ring (ring slot g % NR, 8 KB apart
                                      // so that a forwarding code + (g << 13) addresses its entry)
    uint32_t tab[TQ][S][RECW];        // slot records, window g in slot g % TQ (LDS-DMA by the chain wave)
    uint4 cst[2][S][2][NP];           // chain constants (K1 = (A, B), K2 = (eps, c_o), K3 = (L, H), 0) per step,
                                      // codeword 2q + h at [h][q]   (pre -> chain)
    uint4 xo[2][S / 8][CW];           // chain inputs Y, 8 steps x i16 per codeword   (chain -> post)
    struct In {                       // one window's inputs of one slab wave, landed by LDS-DMA (lane 8e + slot):
        uint4 a[8][8];                //   [0..5][slot] V rows (info edges, record entry D0-1), [6..7][slot] message
                                      //   0..31 B
        uint4 pad[4];                 //   (rows 6, 7 and b[0], b[1] in different banks)
        uint4 b[2][8];                //   [0..1][slot] message 32..63 B
    } in[WS][NI];                     // (entry-major: the 8 slots of one read are in different banks)
    static constexpr uint32_t IN_B = sizeof(uint4) * (8 * 8 + 4);   // byte offset of In::b
    uint4 mst[WS][8][4];              // new messages of a window per slab wave, [slot] x 64 B
    uint4 et_spare[320];              // early termination: between segments the whole struct holds the
                                      // hard bits of every variable (u16 x 64800 for DVB-S2; one
                                      // workgroup per CU either way)
};

struct Coop3Args {
    int8_t *V;                        // V[n + 1][pitch]; row n is the sink of inactive slots
    uint8_t *Mc;                      // [pitch / 16][mrows][8 pairs][2] u32; row m is the sink
    const uint32_t *tab;              // [nw][S][RECW] slot records
    unsigned long long *stamps;       // diagnostic build: [grid][waves][4]
    const uint8_t *live;              // early termination: [pitch] 0 = converged (NULL: all live)
    int8_t *P;                        // parity rows k + j at P[group][j], j <= m (DecodeLaunch::P)
    // in-kernel early termination (ET kernels): layered edge list (group 0:
    // checks [0, m0) of degree D0, then degree d1), snapshot V [n][pitch],
    // iterations used per codeword
    const uint32_t *ev;
    int8_t *Vs;
    int32_t *iters_used;
    int iters, batch, m0, d1;
    int pitch, G, nw, tail, mrows, n, m, k, x0, remap, prio, slab_prio;
    uint32_t nmsf;                    // NMS factor per half (value form)
    size_t wgoff;                     // bytes between two codeword groups' V (16)
    uint32_t rmm, coff, offp;         // R(msg_max), C(offset), offset per half (value form)
};

struct St3 {                          // one window's state from pre to post (R / C pairs)
    uint32_t c[D0 - 1];               // contributions (info, o); tail: new V
    uint32_t a[D0 - 1];               // |c| (not clipped: min1 / min2 are, where the constants are made)
    uint32_t mn1, mn2, sacc, mx;      // min1 / min2 / sign parity over info + o; x-edge old message
                                      // tail: mn1 = MA, mn2 = MB
    uint32_t xs;                      // the slot's chain step: u16 index of its x input in xo[buf]
    uint32_t v[X];                    // FZ (early termination): the info edges' V as read (R pairs)
};

// record meta (word D0): check | COOP_M_ACT | chain step << STEP_SHIFT.  The
// host permutes a window's checks over its slots (coop3_upload: every
// distance-2 forwarding source and reader in slab wave 0); the chain runs the
// steps in check order, so a slot's constants / x input sit at its step
constexpr int STEP_SHIFT = 22;

LDPC_DEV uint32_t pk_ashr8(uint32_t a) { return us(sv(a) >> (short)8); }
LDPC_DEV uint32_t pk_add(uint32_t a, uint32_t b) { return us(sv(a) + sv(b)); }

constexpr uint32_t V127 = 0x007F007Fu, VNEG127 = 0xFF81FF81u;   // +-127 per half (value form)

LDPC_DEV uint32_t pk_mul_lo(uint32_t a, uint32_t b) { return us(__builtin_bit_cast(s16x2, __builtin_bit_cast(u16x2, a) * __builtin_bit_cast(u16x2, b))); }
// NMS constant of a clipped minimum r (R form, value <= 63) for factor f <= 64
// (value form per half): (v * f) >> 5 as a value / in C form (256 x)
LDPC_DEV uint32_t nms_v(uint32_t r, uint32_t f) { return us(__builtin_bit_cast(s16x2, __builtin_bit_cast(u16x2, pk_mul_lo(pk_ashr8(r), f)) >> (unsigned short)5)); }
LDPC_DEV uint32_t nms_c(uint32_t r, uint32_t f) { return (pk_mul_lo(pk_ashr8(r), f) << 3) & HIBYTES; }   // (<= 4032 << 3: no carry between halves)
LDPC_DEV uint32_t pk_shl5(uint32_t a) { return us(sv(a) << (short)5); }

// what a period reads from LDS, issued together at its start
struct PreIn {
    uint32_t v[D0 - 1];               // raw V dwords (info edges, entry D0-1)
    uint32_t ma, mb;                  // old message record of this pair
    uint4 mf;                         // record words D0 .. D0+3: meta, forwarding codes (read a period early)
    uint32_t fv[X];                   // forwarded V pairs (raw u16) of the info edges with a forwarding code
};
struct StIn {                         // the stores of window p-2
    uint4 vd, md;                     // staged V row piece (16 codewords), message piece
    uint32_t row, chk;                // record entry q of the slot, its meta
};
struct PfIn {                         // the LDS-DMA gathers of window p+1+R
    uint32_t rv, chk2;
};

template <int WS, int R, bool NMS = false>
struct Slab3 {
    using SM = Smem3<WS, R>;
    static constexpr int S = SM::S, NR = SM::NR;
    SM &sm;
    const Coop3Args &a;
    char *vsb;                        // V row store of record entry q: vsb + row * vsm (the parity entries
    uint32_t vsm;                     //   q >= X go to the parity rows' own layout P, see Coop3Args)
    i32x4 mr;                         // message rows in 16-B units
    int k, kl, q, w, lane, tail;      // slot, slot in this wave, codeword pair, wave, lane
    uint32_t usel;                    // v_perm selector: this pair's two bytes of a V dword -> R pair
    uint32_t fsel;                    // ... of a forwarded u16 (0x050d040d, in a VGPR)
    PkK K;
    uint32_t fk;                      // NMS factor per half (value form)
    // per-lane constants of the LDS-DMA gathers (lane (kl, j): j < 6 a V row, j >= 6 a message piece)
    const char *g1base, *g2base;
    uint32_t g1mul, g1mask, recsel;
    uint32_t vrd, mrd;                // byte offsets of this lane's V dword / message pair in an In record
    uint32_t fm = 0;                  // FZ: halves of this pair's converged codewords (early termination):
                                      // their V is rewritten unchanged and the chain passes V[p_i] unchanged
    uint32_t psel = 0x0c0c0705u;      // FZ: perm(new, old, psel) = pack_v of new, or of old where converged

    // ---- reads
    // in.mf = mfc (window g's codes, read in the previous period); mfn <- window g+1's
    LDPC_DEV void read_pre(int g, int ib, PreIn &in, const uint4 &mfc, uint4 &mfn) const
    {
        const char *inb = (const char *)&sm.in[w][ib];
#pragma unroll
        for (int j = 0; j < D0 - 1; j++) in.v[j] = *(const uint32_t *)(inb + vrd + 128 * j);
        const uint2 mm = *(const uint2 *)(inb + mrd);
        in.ma = mm.x;
        in.mb = mm.y;
        in.mf = mfc;
        mfn = read_mf(g + 1);
    }
    LDPC_DEV uint4 read_mf(int g) const { return *(const uint4 *)&sm.tab[g & (TQ - 1)][k][D0]; }
    // forwarded values of window g's info edges: code j (16 bits, fwd_code3)
    // = ((-dW) mod 4) << 13 | stage offset | near << 1 | use; code + (g << 13)
    // carries ring slot (g - dW) mod 4 in bits 13-14.  Unused codes read
    // ring offset 0 (ignored).  Branch-free: 2 VALU + 1 ds_read_u16 per edge.
    LDPC_DEV void fwd_read(int g, PreIn &in) const
    {
        const char *sbase = (const char *)&sm.stg[0][0];
        const uint32_t gs = (uint32_t)__builtin_amdgcn_readfirstlane(g << 13), q2 = 2u * (uint32_t)q;
        const uint32_t fw[3] = {in.mf.y, in.mf.z, in.mf.w};
#pragma unroll
        for (int j = 0; j < X; j++) {
            const uint32_t code = (j & 1) ? fw[j >> 1] >> 16 : fw[j >> 1] & 0xFFFFu;
            in.fv[j] = *(const unsigned short *)(sbase + (((code + gs) & 0x7FF0u) | q2));
        }
    }
    LDPC_DEV void read_st(int g, StIn &in) const
    {
        in.vd = sm.stg[g % NR][q * (S + 1) + k];
        in.md = sm.mst[w][kl][q & 3];
        in.row = sm.tab[g & (TQ - 1)][k][q];
        in.chk = sm.tab[g & (TQ - 1)][k][D0] & COOP_CHK_MASK;
    }
    LDPC_DEV void read_pf(int g, PfIn &in) const
    {
        in.rv = sm.tab[g & (TQ - 1)][8 * w + (lane & 7)][recsel] & g1mask;
        in.chk2 = sm.tab[g & (TQ - 1)][8 * w + (lane & 7)][D0] & COOP_CHK_MASK;
    }
    LDPC_DEV uint32_t read_x(int g, const St3 &s) const   // chain inputs of this slot, codewords 2q, 2q+1 -> R pair
    {
        const unsigned short *xs = (const unsigned short *)&sm.xo[g & 1][0][0] + s.xs + 16 * q;
        const uint32_t x0 = xs[0], x1 = xs[8];
        return perm(x1, x0, 0x040d000du);   // chain values are in [-127, 127]
    }

    // ---- memory operations at the end of a period
    // lane (kl, c): record entry c's 16 codewords (c < 6, the tail 7) and
    // message piece c (c < 4) of its wave's slot kl
    LDPC_DEV void stores(const StIn &in, bool tl) const
    {
        if (q < (tl ? D0 : D0 - 1)) *(uint4 *)(vsb + (size_t)in.row * vsm) = in.vd;
        if (q < 4) sbuf_store_v4(__builtin_bit_cast(i32x4, in.md), mr, (int)(in.chk * 4 + q), 0, 0, 0);
    }
    LDPC_DEV void gathers(const PfIn &in, int ib) const
    {
        static_assert(offsetof(typename SM::In, b) == SM::IN_B, "In layout");
        const uint32_t base = (uint32_t)(uintptr_t)&sm.in[w][ib];
        dma16(g1base + (size_t)in.rv * g1mul, base);
        if (lane < 16) dma16(g2base + (size_t)in.chk2 * MREC, base + SM::IN_B);
    }

    // the first windows of the decode: a code whose source window precedes
    // window 0 (g < dW) is not used
    LDPC_DEV static void mask_early(int g, uint4 &mf)
    {
        uint32_t *fw = &mf.y;
#pragma unroll
        for (int i = 0; i < 3; i++)
#pragma unroll
            for (int h = 0; h < 2; h++) {
                const uint32_t code = (fw[i] >> (16 * h)) & 0xFFFFu;
                const int dw = (int)(((0u - (code >> 13) - 2u) & 3u) + 2u);
                if ((code & 1u) && g < dw) fw[i] &= ~(1u << (16 * h));
            }
    }

    // pre of window g: chain constants -> cst[g & 1], state -> s
    template <bool TL, bool FZ_ = false, int MP = -1>
    LDPC_DEV void pre(int g, const PreIn &in, St3 &s) const
    {
        constexpr bool FZ = FZ_;
        const uint32_t meta = in.mf.x;
        uint32_t v[D0 - 1];
        // V pair of edge j: this pair's two bytes of the loaded V dword, or the
        // forwarded u16 (selector 0x050d040d: bytes 0, 1 of in.fv[j] -> R pair)
        const uint32_t fw[3] = {in.mf.y, in.mf.z, in.mf.w};
#pragma unroll
        for (int j = 0; j < X; j++) {
            const uint32_t m = (uint32_t)__builtin_amdgcn_sbfe((int)fw[j >> 1], 16 * (j & 1), 1);   // 0 / -1
            v[j] = perm(in.fv[j], in.v[j], bfi(m, fsel, usel));
        }
        v[X] = unpack_v(in.v[X], usel);
        const MsgTab t = msg_tab(in.mb);
        const uint32_t MA = in.ma, neg127 = K.neg127, c510 = K.c510;
        uint32_t min1 = R127, min2 = R127, sacc = 0;
        uint32_t A, B, EPS, COV, L, H;
        if constexpr (!TL) {
            // first degree group (OMS_fixed_SSE.cpp:201-218); a = |c| here, the
            // msg_max clip is applied to min1 / min2 (a_j == min1 decides the
            // same edges either way, and min1 == msg_max implies cst1 == cst2)
            static_for<0, X>([&](auto jc) __attribute__((always_inline)) {
                constexpr int J = decltype(jc)::value;
                const uint32_t c = pk_max(pk_sub_sat(v[J], old_msg<J>(MA, t)), neg127);
                const uint32_t aj = abs_r(c, c510);
                s.c[J] = c;
                s.a[J] = aj;
                sacc ^= c;
                min2 = pk_max(min1, pk_min(aj, min2));
                min1 = pk_min(min1, aj);
            });
            if constexpr (MP >= 0) __builtin_amdgcn_s_setprio(MP);   // mid-phase wave priority (fast periods)
            const uint32_t kb = sacc ^ ((D0 & 1) ? SIGNS : 0u);
            const uint32_t cor = pk_max(pk_sub_sat(v[X], old_msg<D0 - 1>(MA, t)), neg127);
            const uint32_t ao = abs_r(cor, c510);
            s.c[X] = cor;
            s.a[X] = ao;
            s.sacc = sacc ^ cor;
            s.mn2 = pk_max(min1, pk_min(ao, min2));
            s.mn1 = pk_min(min1, ao);
            const uint32_t mx = old_msg<X>(MA, t);
            s.mx = mx;
            // chain constants in value form (R >> 8, C >> 8), both codewords at once
            COV = pk_ashr8(cor);
            const uint32_t EM = pk_sra15(kb);   // EM: -1 where eps = -1
            uint32_t TV;                        // cst over the info edges (value form)
            if constexpr (NMS) {
                TV = nms_v(pk_min(min1, K.rmm), fk);
                EPS = pk_sub(fk ^ EM, EM);                                    // eps * f
                const uint32_t efm = pk_mul_lo(pk_ashr8(mx), EPS);            // eps * f * m_x
                A = pk_sub(pk_shl5(COV), efm);                                // 32 c_o - eps f m_x
                B = pk_add(A, 0x001F001Fu);
            } else {
                TV = pk_ashr8(pk_max(pk_sub(pk_min(min1, K.rmm), K.coff), K.r0));
                EPS = EM | 0x00010001u;
                const uint32_t base = pk_sub(COV, pk_sub(pk_ashr8(mx) ^ EM, EM));   // c_o - eps * m_x
                A = pk_sub(base, a.offp);
                B = pk_add(base, a.offp);
            }
            L = pk_max(pk_sub(COV, TV), VNEG127);
            H = pk_min(pk_add(COV, TV), V127);
            if constexpr (FZ) {   // converged codewords: L = H = V[p_i] as read, the step returns it
#pragma unroll
                for (int j = 0; j < X; j++) s.v[j] = v[j];
                const uint32_t VO = pk_ashr8(v[X]);
                L = bfi(fm, VO, L);
                H = bfi(fm, VO, H);
            }
        } else {
            // the tail check (later degree group: a = |min(c, msg_max)|,
            // OMS_fixed_SSE.cpp:293,314) has no chain input: finish it here
            static_for<0, X + 1>([&](auto jc) __attribute__((always_inline)) {
                constexpr int J = decltype(jc)::value;
                const uint32_t c = pk_max(pk_sub_sat(v[J], old_msg<J>(MA, t)), neg127);
                // OMS: a = |min(c, msg_max)| (later group); NMS: min(|c|, msg_max), clipped in min1 / min2
                const uint32_t aj = NMS ? abs_r(c, c510) : abs_r(pk_min(c, K.rmm), c510);
                s.c[J] = c;
                s.a[J] = aj;
                sacc ^= c;
                min2 = pk_max(min1, pk_min(aj, min2));
                min1 = pk_min(min1, aj);
            });
            const uint32_t k1 = NMS ? nms_c(pk_min(min2, K.rmm), fk)
                                    : pk_min(pk_max(pk_sub(min2, K.coff), K.r0), K.rmm) & HIBYTES;
            const uint32_t k2 = NMS ? nms_c(pk_min(min1, K.rmm), fk)
                                    : pk_min(pk_max(pk_sub(min1, K.coff), K.r0), K.rmm) & HIBYTES;
            const uint32_t P = (sacc ^ (((D0 - 1) & 1) ? SIGNS : 0u)) & SIGNS;
            uint32_t MAn = 0;
            static_for<0, X + 1>([&](auto jc) __attribute__((always_inline)) {
                constexpr int J = decltype(jc)::value;
                s.c[J] = new_msg<J>(s.c[J], s.a[J], min1, k1, k2, P, MAn, neg127);
                if constexpr (FZ) s.c[J] = bfi(fm, v[J], s.c[J]);   // converged codewords keep their V
            });
            s.mx = 0;
            s.sacc = 0;
            s.mn1 = MAn;
            s.mn2 = perm(k2, k1, 0x07030501u);
            // the chain passes V[p_0] (the tail's last edge) on: A = B = c_o = L = H = y
            // (NMS: A = 32 y, B = 32 y + 31)
            const uint32_t Y = pk_ashr8(s.c[X]);
            A = B = COV = L = H = Y;
            if constexpr (NMS) {
                A = pk_shl5(Y);
                B = pk_add(A, 0x001F001Fu);
            }
            EPS = 0;
        }
        if (!(meta & COOP_M_ACT)) {   // pass-through slot: Y' = Y (NMS: t = 32 Y + (0, 31))
            A = COV = 0;
            B = NMS ? 0x001F001Fu : 0u;
            EPS = NMS ? 0x00200020u : 0x00010001u;
            L = VNEG127;
            H = V127;
        }
        // per codeword records: (A, B), (eps, c_o), (L, H) as i16 pairs
        uint4 r0, r1;
        r0.x = perm(B, A, 0x05040100u);
        r1.x = perm(B, A, 0x07060302u);
        r0.y = perm(COV, EPS, 0x05040100u);
        r1.y = perm(COV, EPS, 0x07060302u);
        r0.z = perm(H, L, 0x05040100u);
        r1.z = perm(H, L, 0x07060302u);
        r0.w = r1.w = 0;
        const int cb = g & 1;
        const uint32_t step = (meta >> STEP_SHIFT) & 63u;
        s.xs = (step >> 3) * (CW * 8) + (step & 7);
        uint4 *cp = &sm.cst[cb][0][0][q] + step * (2 * NP);
        cp[0] = r0;
        cp[NP] = r1;
    }

    // post of window g (x inputs xr): new V pairs -> stg[g % NR], messages ->
    // mst[w]; they leave in the stores of the same period
    template <bool TL, bool FZ_ = false, int MP = -1>
    LDPC_DEV void post(int g, uint32_t xr, const St3 &s) const
    {
        constexpr bool FZ = FZ_;
        unsigned short *st = (unsigned short *)&sm.stg[g % NR][k];   // [entry][..S slots..][8 pairs] u16
        constexpr int ES = (S + 1) * 8;                                 // u16 between entries
        uint32_t MA, MB;
        if constexpr (!TL) {
            const uint32_t cx = pk_max(pk_sub_sat(xr, s.mx), K.neg127);
            const uint32_t ax = abs_r(cx, K.c510);
            const uint32_t sacc = s.sacc ^ cx;
            const uint32_t min2 = pk_max(s.mn1, pk_min(ax, s.mn2)), min1 = pk_min(ax, s.mn1);
            const uint32_t k1 = NMS ? nms_c(pk_min(min2, K.rmm), fk)
                                    : pk_max(pk_sub(pk_min(min2, K.rmm), K.coff), K.r0) & HIBYTES;
            const uint32_t k2 = NMS ? nms_c(pk_min(min1, K.rmm), fk)
                                    : pk_max(pk_sub(pk_min(min1, K.rmm), K.coff), K.r0) & HIBYTES;
            const uint32_t P = (sacc ^ ((D0 & 1) ? SIGNS : 0u)) & SIGNS;
            MA = 0;
            uint32_t nv[X + 1];
            static_for<0, X>([&](auto jc) __attribute__((always_inline)) {
                constexpr int J = decltype(jc)::value;
                const uint32_t n = new_msg<J>(s.c[J], s.a[J], min1, k1, k2, P, MA, K.neg127);
                nv[J] = FZ ? perm(n, s.v[J], psel) : pack_v(n);   // FZ: pack_v of new / old per codeword
            });
            if constexpr (MP >= 0) __builtin_amdgcn_s_setprio(MP);   // mid-phase wave priority (fast periods)
            // x edge: for converged codewords the chain passed V[p_{i-1}] unchanged
            const uint32_t nx = new_msg<X>(cx, ax, min1, k1, k2, P, MA, K.neg127);
            nv[X] = FZ ? perm(nx, xr, psel) : pack_v(nx);
            // the o edge: message bits only (the next check rewrites V[o] as its x edge)
            (void)new_msg<D0 - 1>(s.c[X], s.a[X], min1, k1, k2, P, MA, K.neg127);
            MB = perm(k2, k1, 0x07030501u);
#pragma unroll
            for (int j = 0; j <= X; j++) st[j * ES + q] = (unsigned short)nv[j];
        } else {
            {
                static_for<0, X>([&](auto jc) __attribute__((always_inline)) {
                    constexpr int J = decltype(jc)::value;
                    st[J * ES + q] = (unsigned short)pack_v(s.c[J]);
                });
                st[X * ES + q] = (unsigned short)pack_v(xr);               // V of the last group-0 check's o edge
                st[(D0 - 1) * ES + q] = (unsigned short)pack_v(s.c[X]);   // the tail's last edge
            }
            MA = s.mn1;
            MB = s.mn2;
        }
        *(uint2 *)((char *)&sm.mst[w][kl][0] + 8 * q) = make_uint2(MA, MB);
    }
};

// one chain step: input = half IH of xin, output = half OH of xout (the other
// half of xout is kept); c = (K1, K2, K3) of the step
#define C3_STEP_SAME(XW, KV)                                                                   \
    asm volatile("v_pk_mad_i16 %1, %0, %3, %2 op_sel:[0,0,0] op_sel_hi:[0,0,1]\n\t"           \
                 "v_med3_i16 %1, %1, %3, %1 op_sel:[0,1,1,0]\n\t"                             \
                 "v_med3_i16 %0, %1, %4, %4 op_sel:[0,0,1,1]"                                 \
                 : "+v"(XW), "=&v"(tmp)                                                       \
                 : "v"((KV).x), "v"((KV).y), "v"((KV).z))
#define C3_STEP_CROSS(XI, XO, KV)                                                              \
    asm volatile("v_pk_mad_i16 %1, %2, %4, %3 op_sel:[1,0,0] op_sel_hi:[1,0,1]\n\t"           \
                 "v_med3_i16 %1, %1, %4, %1 op_sel:[0,1,1,0]\n\t"                             \
                 "v_med3_i16 %0, %1, %5, %5 op_sel:[0,0,1,0]"                                 \
                 : "+v"(XO), "=&v"(tmp)                                                       \
                 : "v"(XI), "v"((KV).x), "v"((KV).y), "v"((KV).z))

// NMS: (t, t + 31) = eps f Y + (A, B); >> 5; median with c_o; clamp [L, H]
#define C3_STEP_SAME_NMS(XW, KV)                                                               \
    asm volatile("v_pk_mad_i16 %1, %0, %3, %2 op_sel:[0,0,0] op_sel_hi:[0,0,1]\n\t"           \
                 "v_pk_ashrrev_i16 %1, 5, %1 op_sel_hi:[0,1]\n\t"                              \
                 "v_med3_i16 %1, %1, %3, %1 op_sel:[0,1,1,0]\n\t"                             \
                 "v_med3_i16 %0, %1, %4, %4 op_sel:[0,0,1,1]"                                 \
                 : "+v"(XW), "=&v"(tmp)                                                       \
                 : "v"((KV).x), "v"((KV).y), "v"((KV).z))
#define C3_STEP_CROSS_NMS(XI, XO, KV)                                                          \
    asm volatile("v_pk_mad_i16 %1, %2, %4, %3 op_sel:[1,0,0] op_sel_hi:[1,0,1]\n\t"           \
                 "v_pk_ashrrev_i16 %1, 5, %1 op_sel_hi:[0,1]\n\t"                              \
                 "v_med3_i16 %1, %1, %4, %1 op_sel:[0,1,1,0]\n\t"                             \
                 "v_med3_i16 %0, %1, %5, %5 op_sel:[0,0,1,0]"                                 \
                 : "+v"(XO), "=&v"(tmp)                                                       \
                 : "v"(XI), "v"((KV).x), "v"((KV).y), "v"((KV).z))

// the chain steps of one window (lanes 0..15 = codewords).  Step k's input
// sits at position k % 8 of w (w[i] low / high half = positions 2i, 2i+1) and
// its output goes to position k+1, so after step 8j+6 positions 0..7 hold the
// inputs of steps 8j .. 8j+7: the x inputs post needs, stored as one uint4.
template <int WS, int R, int B0, int B1, bool NMS = false, typename SMT>
LDPC_DEV void chain_window3(SMT &sm, int buf, int c, uint32_t (&w)[4])
{
    const uint4 *cp = &sm.cst[buf][0][c & 1][c >> 1];
    constexpr int KST = 2 * NP;       // uint4 between steps
    uint4 kq[2][8];
#pragma unroll
    for (int i = 0; i < 8; i++) kq[B0 & 1][i] = cp[(B0 * 8 + i) * KST];
#pragma unroll
    for (int b = B0; b < B1; b++) {
        if (b + 1 < B1) {
#pragma unroll
            for (int i = 0; i < 8; i++) kq[(b + 1) & 1][i] = cp[((b + 1) * 8 + i) * KST];
        }
        uint32_t tmp;
        if constexpr (NMS) {
            C3_STEP_SAME_NMS(w[0], kq[b & 1][0]);
            C3_STEP_CROSS_NMS(w[0], w[1], kq[b & 1][1]);
            C3_STEP_SAME_NMS(w[1], kq[b & 1][2]);
            C3_STEP_CROSS_NMS(w[1], w[2], kq[b & 1][3]);
            C3_STEP_SAME_NMS(w[2], kq[b & 1][4]);
            C3_STEP_CROSS_NMS(w[2], w[3], kq[b & 1][5]);
            C3_STEP_SAME_NMS(w[3], kq[b & 1][6]);
            sm.xo[buf][b][c] = make_uint4(w[0], w[1], w[2], w[3]);
            C3_STEP_CROSS_NMS(w[3], w[0], kq[b & 1][7]);
        } else {
            C3_STEP_SAME(w[0], kq[b & 1][0]);          // pos 0 -> 1
            C3_STEP_CROSS(w[0], w[1], kq[b & 1][1]);   // pos 1 -> 2
            C3_STEP_SAME(w[1], kq[b & 1][2]);          // 2 -> 3
            C3_STEP_CROSS(w[1], w[2], kq[b & 1][3]);   // 3 -> 4
            C3_STEP_SAME(w[2], kq[b & 1][4]);          // 4 -> 5
            C3_STEP_CROSS(w[2], w[3], kq[b & 1][5]);   // 5 -> 6
            C3_STEP_SAME(w[3], kq[b & 1][6]);          // 6 -> 7
            sm.xo[buf][b][c] = make_uint4(w[0], w[1], w[2], w[3]);
            C3_STEP_CROSS(w[3], w[0], kq[b & 1][7]);   // 7 -> 0 (the next block's first input)
        }
    }
}

// diagnostic stamps that do not wait: the compiler waits for s_memtime only
// where the value is used (the end of a period)
LDPC_DEV unsigned long long stampL()
{
    __builtin_amdgcn_sched_barrier(0);
    const unsigned long long t = __builtin_amdgcn_s_memtime();
    __builtin_amdgcn_sched_barrier(0);
    return t;
}

LDPC_DEV unsigned long long stamp3()
{
    unsigned long long t;
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    __builtin_amdgcn_sched_barrier(0);
    return t;
}

// ---- in-kernel early termination helpers (16 codewords = the 16 bytes of a
// V row piece, codeword wg * 16 + j in byte j)
// high bit of byte j set where byte j > 0 (the hard decision)
LDPC_DEV uint32_t pos_bits(uint32_t d)
{
    const uint32_t nz = ((d & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | d;   // high bit: byte != 0
    return nz & ~d & 0x80808080u;
}
LDPC_DEV uint32_t high_bits16(uint4 x)   // byte high bits -> 16-bit codeword mask
{
    auto c4 = [](uint32_t v) { return ((v >> 7) & 1u) | ((v >> 14) & 2u) | ((v >> 21) & 4u) | ((v >> 28) & 8u); };
    return c4(x.x) | c4(x.y) << 4 | c4(x.z) << 8 | c4(x.w) << 12;
}
// Wave CHW: the chain; the others: slab waves (slab index w: slots 8w .. 8w+7).
// ET: in-kernel early termination -- the decode runs one iteration per
// segment (pipeline drained at its end), then the whole workgroup checks the
// syndrome of its live codewords (stopping once each has a failing check),
// snapshots the V of the codewords converging now, and leaves when none is
// live; the snapshots are merged back at the end.  Same result as the
// reference's per-codeword stop (oracle: syndrome after every iteration), with
// one launch instead of one per iteration plus syndrome / snapshot kernels.
template <int WS, int R, bool STAMP, bool ET = false, bool NMS = false>
__global__ void __launch_bounds__(64 * (WS + 1)) coop3_decode(Coop3Args a)
{
    using SM = Smem3<WS, R>;
    using CF = Cfg<WS, R>;
    constexpr int S = CF::S, KAHEAD = CF::KAHEAD, U = CF::U, CHW = CF::CHW, NB = CF::NB;
    __shared__ SM sm;

    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const int nb = gridDim.x, id = blockIdx.x;
    const int wg = a.remap ? (id & 7) * (nb >> 3) + (id >> 3) : id;   // XCD-aware codeword groups
    const int G = ET ? a.nw : a.G;   // periods per segment (ET: one iteration)
    if (G == 0) return;
    if (!ET && a.live && !__syncthreads_or(threadIdx.x < CW && a.live[wg * CW + threadIdx.x])) return;
    // the group's parity rows -> P (consecutive checks' parity values
    // contiguous: a wave's 8 o-edge gathers / x-edge stores touch 1-2 lines,
    // not 8), back into V at the end
    {
        int8_t *vpar = a.V + (size_t)a.k * (size_t)a.pitch + (size_t)wg * a.wgoff;
        int8_t *ppar = a.P + (size_t)wg * (size_t)(a.m + 1) * 16;
#pragma unroll 8
        for (int j = threadIdx.x; j < a.m; j += blockDim.x)
            *(uint4 *)(ppar + 16 * (size_t)j) = *(const uint4 *)(vpar + (size_t)j * (size_t)a.pitch);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
    }
    auto parity_out = [&]() {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        int8_t *vpar = a.V + (size_t)a.k * (size_t)a.pitch + (size_t)wg * a.wgoff;
        const int8_t *ppar = a.P + (size_t)wg * (size_t)(a.m + 1) * 16;
#pragma unroll 8
        for (int j = threadIdx.x; j < a.m; j += blockDim.x)
            *(uint4 *)(vpar + (size_t)j * (size_t)a.pitch) = *(const uint4 *)(ppar + 16 * (size_t)j);
    };
    // ---- ET state: [0] live codewords, [1] failing codewords (syndrome)
    __shared__ uint32_t et_sh[2];
    constexpr int NT = 64 * (WS + 1);
    const char *etV = (const char *)a.V + (size_t)wg * a.wgoff;
    const char *etP = (const char *)a.P + (size_t)wg * (size_t)(a.m + 1) * 16;
    auto et_row = [&](uint32_t v) -> const uint4 * {   // V row piece of variable v (parity rows: in P)
        return ((int)v < a.k) ? (const uint4 *)(etV + (size_t)v * (size_t)a.pitch)
                            : (const uint4 *)(etP + (size_t)(v - (uint32_t)a.k) * 16);
    };
    if constexpr (ET) {
        if (threadIdx.x == 0) {
            const int valid = min(CW, max(0, a.batch - wg * CW));
            et_sh[0] = (1u << valid) - 1u;
            et_sh[1] = 0;
        }
        if (threadIdx.x < CW && wg * CW + (int)threadIdx.x < a.batch) a.iters_used[wg * CW + threadIdx.x] = a.iters;
        __syncthreads();
        if (et_sh[0] == 0) return;   // padding columns only
    }
    // after iteration `it` (ET): syndrome and decision -- every thread,
    // uniform result (true: decode another iteration).  Codewords converged
    // earlier are frozen by the slab waves (Slab3::fm: their V rows are
    // rewritten with the values they had), so no V snapshot is taken.
    // Parity bits of check c over the 16 codewords (byte high bits)
    auto et_check = [&](int c) -> uint4 {
        uint4 x = make_uint4(0, 0, 0, 0);
        if (c < a.m0) {
            const uint32_t *e = a.ev + (size_t)c * D0;
            uint4 y[D0];
#pragma unroll
            for (int j = 0; j < D0; j++) y[j] = *et_row(e[j]);
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
                const uint4 y = *et_row(e[j]);
                x.x ^= pos_bits(y.x);
                x.y ^= pos_bits(y.y);
                x.z ^= pos_bits(y.z);
                x.w ^= pos_bits(y.w);
            }
        }
        return x;
    };
    // a failing check per codeword, kept across iterations (a codeword that
    // does not converge tends to keep failing the same checks): round 0 tests
    // these first
    constexpr int NH = 4;   // hint checks per codeword
    __shared__ uint32_t et_hint[CW * NH];
    if constexpr (ET) {
        if (threadIdx.x < CW * NH) et_hint[threadIdx.x] = (uint32_t)threadIdx.x;
    }
    auto et_note = [&](uint32_t x, int c) {
        for (uint32_t b = x; b; b &= b - 1u) et_hint[__builtin_ctz(b) * NH + (c & (NH - 1))] = (uint32_t)c;
    };
    // exit test of a scan round: true once every live codeword has a failing check
    auto et_round = [&](uint32_t f, uint32_t live) -> bool {
        if (f & live) atomicOr(&et_sh[1], f & live);
        __syncthreads();
        const uint32_t fail = et_sh[1];
        __syncthreads();
        return (fail & live) == live;
    };
    auto et_after = [&](int it) -> bool {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the iteration's stores and table DMAs
        __syncthreads();
        const uint32_t live = et_sh[0];
        // round 0: one check per thread, gathered directly -- threads 0..63
        // the codewords' hint checks, the others checks spread over the code
        // (a codeword still decoding fails many checks: this usually settles
        // every live one)
        {
            const int c = threadIdx.x < CW * NH ? (int)et_hint[threadIdx.x]
                                           : (int)((threadIdx.x + (size_t)it * NT * 5) % (size_t)a.m);
            const uint32_t x = high_bits16(et_check(c)) & live;
            et_note(x, c);
            if (et_round(x, live)) goto et_done;
        }
        {
            // the full syndrome: every variable's hard bits staged in LDS (the
            // pipeline's LDS is idle between segments; the launch checks n
            // fits), then the checks, 8 per thread and round with an exit
            // test after each; loads unconditional (clamped check index) so a
            // round's index loads are in flight together
            uint16_t *hb = reinterpret_cast<uint16_t *>(&sm);
            // (16 unconditional loads in flight per thread: clamped rows)
            auto hbits = [](uint4 y) {
                return (uint16_t)high_bits16(make_uint4(pos_bits(y.x), pos_bits(y.y), pos_bits(y.z), pos_bits(y.w)));
            };
            for (int r0 = 0; r0 < a.k; r0 += NT * 16) {   // information rows: V
                uint4 y[16];
#pragma unroll
                for (int i = 0; i < 16; i++)
                    y[i] = *(const uint4 *)(etV + (size_t)min(r0 + i * NT + (int)threadIdx.x, a.k - 1) * (size_t)a.pitch);
#pragma unroll
                for (int i = 0; i < 16; i++)
                    if (r0 + i * NT + (int)threadIdx.x < a.k) hb[r0 + i * NT + threadIdx.x] = hbits(y[i]);
            }
            for (int r0 = 0; r0 < a.m; r0 += NT * 16) {   // parity rows: P
                uint4 y[16];
#pragma unroll
                for (int i = 0; i < 16; i++)
                    y[i] = *(const uint4 *)(etP + (size_t)min(r0 + i * NT + (int)threadIdx.x, a.m - 1) * 16);
#pragma unroll
                for (int i = 0; i < 16; i++)
                    if (r0 + i * NT + (int)threadIdx.x < a.m) hb[a.k + r0 + i * NT + threadIdx.x] = hbits(y[i]);
            }
            __syncthreads();
            bool done = false;
            for (int c0 = 0; c0 < a.m0 && !done; c0 += NT * 8) {
                uint32_t ev[8][D0];
#pragma unroll
                for (int r = 0; r < 8; r++) {
                    const int cc = min(c0 + r * NT + (int)threadIdx.x, a.m0 - 1);
#pragma unroll
                    for (int j = 0; j < D0; j++) ev[r][j] = a.ev[(size_t)cc * D0 + j];
                }
                uint32_t f = 0;
#pragma unroll
                for (int r = 0; r < 8; r++) {
                    const int c = c0 + r * NT + (int)threadIdx.x;
                    uint32_t x = 0;
#pragma unroll
                    for (int j = 0; j < D0; j++) x ^= hb[ev[r][j]];
                    x = c < a.m0 ? x & live : 0u;
                    f |= x;
                    if (x) et_note(x, c);
                }
                done = et_round(f, live);
            }
            if (!done && a.m > a.m0) {   // the later degree group (DVB-S2: the tail check)
                uint32_t f = 0;
                for (int c = a.m0 + (int)threadIdx.x; c < a.m; c += NT) {
                    const uint32_t *e = a.ev + (size_t)a.m0 * D0 + (size_t)(c - a.m0) * a.d1;
                    uint32_t x = 0;
                    for (int j = 0; j < a.d1; j++) x ^= hb[e[j]];
                    x &= live;
                    f |= x;
                    if (x) et_note(x, c);
                }
                et_round(f, live);
            }
        }
    et_done:
        const uint32_t fresh = live & ~et_sh[1];   // converged after this iteration
        __syncthreads();
        if (threadIdx.x == 0) {
            et_sh[0] = live & ~fresh;
            et_sh[1] = 0;
        }
        if (fresh && threadIdx.x < CW && ((fresh >> threadIdx.x) & 1u)) a.iters_used[wg * CW + threadIdx.x] = it + 1;
        __syncthreads();
        return (live & ~fresh) != 0 && it + 1 < a.iters;
    };
    // stamps (diagnostic build): per wave 8 words: busy, phases 1..3 (slab:
    // vmcnt, first and second half), -, elapsed, -, G
    unsigned long long sA = 0, sP[4] = {0, 0, 0, 0}, sD = 0, t0 = 0, tx = 0;
    auto write_stamps = [&]() {
        if (STAMP && lane == 0) {
            unsigned long long *o = a.stamps + ((size_t)id * (WS + 1) + wave) * 8;
            o[0] = sA;
            for (int i = 0; i < 4; i++) o[1 + i] = sP[i];
            o[5] = stamp3() - t0;
            o[6] = sD;
            o[7] = (unsigned long long)G;
        }
    };

    if (wave == CHW) {
        // ------------------------------------------------------------ chain wave
        if (a.prio) __builtin_amdgcn_s_setprio(3);
        constexpr int TABW = S * RECW;   // words per window table
        constexpr int NCH = TABW / 4;   // 16-B chunks per window table
        constexpr int CPL = (NCH + 63) / 64;
        static_assert(CPL * DPER <= 63, "table staging");
        const int c = lane & 15;
        auto stage = [&](int u, int slot) {
            const uint4 *src = (const uint4 *)(a.tab + (size_t)u * TABW);
            const uint32_t dst = (uint32_t)(uintptr_t)&sm.tab[slot];
#pragma unroll
            for (int i = 0; i < CPL; i++)
                if (lane + 64 * i < NCH) dma16(src + 64 * i + lane, dst + 1024 * i);
        };
        const bool cl = lane < CW;
        for (int it = 0;; it++) {   // one segment (ET: one iteration per segment)
            for (int w = 0; w < KAHEAD; w++) stage(w % a.nw, w);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            uint32_t w4[4] = {0, 0, 0, 0};
            // the chain's first input V[x0] (a parity row: in P during the decode)
            w4[0] = (uint32_t)(int)((const int8_t *)et_row((uint32_t)a.x0))[c] & 0xFFFFu;
            int un = KAHEAD % a.nw;
            __syncthreads();   // prologue 1: tables of windows 0 .. KAHEAD-1 in LDS
            __syncthreads();   // prologue 2: constants of window 0 in LDS
            if (STAMP) t0 = stamp3();
            for (int p = 0; p <= G; p++) {
                if (STAMP) tx = stamp3();
                if (p < G && cl) chain_window3<WS, R, 0, NB, NMS>(sm, p & 1, c, w4);
                if (STAMP) sP[0] += stamp3() - tx;
                stage(un, (p + KAHEAD) & (TQ - 1));
                un = (un + 1 == a.nw) ? 0 : un + 1;
                asm volatile("s_waitcnt vmcnt(%0)" ::"n"(CPL * DPER) : "memory");
                if (STAMP) sA += stamp3() - tx;
                __syncthreads();
            }
            if (!ET || !et_after(it)) break;
        }
        write_stamps();
        parity_out();
        return;
    }

    // ------------------------------------------------------------ slab waves
    const int sw = wave - (wave > CHW ? 1 : 0);   // slab index
    // the second-dispatched half of the slab waves loses VALU arbitration to
    // its SIMD partner; static priority evens them out (MI355X_MICROARCH.md,
    // "Two waves per SIMD", item 4)
    if (a.slab_prio == 1 && wave > CHW) __builtin_amdgcn_s_setprio(1);
    const int kl = lane >> 3, q = lane & 7;
    const char *Vb = (const char *)a.V + (size_t)wg * a.wgoff;
    const char *Mb = (const char *)a.Mc + (size_t)wg * a.mrows * MREC;
    // parity rows k + j of this group at Pb + 16 j: row r at Pb - 16 k + 16 r
    char *Pr = (char *)a.P + ((size_t)wg * (size_t)(a.m + 1) - (size_t)a.k) * 16;
    Slab3<WS, R, NMS> sl{sm,
                    a,
                    q >= X ? Pr : (char *)Vb,
                    q >= X ? 16u : (uint32_t)a.pitch,
                    buffer_rsrc(Mb, 16u, (uint32_t)a.mrows * 4u),
                    8 * sw + kl,
                    kl,
                    q,
                    sw,
                    lane,
                    a.tail,
                    0x010d000du + (uint32_t)(lane & 1) * 0x02000200u,
                    opaque(0x050d040du),
                    PkK{opaque(RNEG127), opaque(R0), opaque(C510), opaque(a.rmm), opaque(a.coff)},
                    opaque(a.nmsf),
                    // DMA lane 8e + slot: entry e < 6 a V row (record entry e, the
                    // o edge's D0-1 for e = X), e >= 6 message piece e - 6
                    kl < X ? Vb : kl == X ? Pr : Mb + (kl - 6) * 16,
                    Mb + (2 + (kl & 1)) * 16,
                    kl < X ? (uint32_t)a.pitch : kl == X ? 16u : (uint32_t)MREC,
                    kl < 6 ? 0xFFFFFFFFu : COOP_CHK_MASK,
                    (uint32_t)(kl < X ? kl : (kl == X ? D0 - 1 : D0)),
                    (uint32_t)(kl * 16 + 4 * (q >> 1)),
                    (uint32_t)(q < 4 ? (6 + (q >> 1)) * 128 + kl * 16 + (q & 1) * 8
                                     : SM::IN_B + ((q >> 1) - 2) * 128 + kl * 16 +
                                           (q & 1) * 8)};
    auto next = [&](int &u) __attribute__((always_inline)) { u = (u + 1 == a.nw) ? 0 : u + 1; };
    constexpr int NI = CF::NI, NS = CF::NS;
    for (int it = 0;; it++) {   // one segment (ET: one iteration per segment)
        __syncthreads();   // prologue 1: tables in LDS
        if constexpr (ET) {   // codewords 2q (low half) and 2q+1 (high half) of this lane: converged?
            const int valid = min(CW, max(0, a.batch - wg * CW));
            const uint32_t conv = (((1u << valid) - 1u) & ~et_sh[0]) >> (2 * q);
            sl.fm = ((conv & 1u) ? 0x0000FFFFu : 0u) | ((conv & 2u) ? 0xFFFF0000u : 0u);
            sl.psel = 0x0c0c0000u | ((conv & 2u) ? 0x0300u : 0x0700u) | ((conv & 1u) ? 0x01u : 0x05u);
        }
        St3 st[NS];
        uint4 mfc;   // records D0 .. D0+3 of the next pre's window
        PfIn pi;
#pragma unroll
        for (int i = 0; i <= R; i++) {   // window i -> in[w][i]   (nw > R + 3)
            sl.read_pf(i, pi);
            sl.gathers(pi, i);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        PreIn in;
        sl.read_pre(0, 0, in, sl.read_mf(0), mfc);
        sl.mask_early(0, in.mf);
        sl.fwd_read(0, in);
        if (a.tail == 0)
            sl.template pre<true, ET>(0, in, st[0]);
        else
            sl.template pre<false, ET>(0, in, st[0]);
        __syncthreads();   // prologue 2
        if (STAMP) t0 = stamp3();
        int uA = a.nw - 1;   // local index of window p-1 (post)
        int uB = 1 % a.nw;   // local index of window p+1 (pre)
        StIn sc;             // the stores of window p-2 (read from the stage at the end of period p-1)
        bool sc_tl = false;  // ... window p-2 is the tail
        // Period p: post of window p-1 (state st[(p-1) % NS], x inputs from the
        // chain's window p-1) -> staged outputs; pre of window p+1 (inputs
        // in[w][(p+1) % NI], -> st[(p+1) % NS]).  Vector memory: the two stores of
        // window p-2 go first, the two LDS-DMA gathers of window p+1+R into
        // in[w][(p+1+R) % NI] follow the first half, so no wave ends a period
        // queueing behind the workgroup's stores (the CU's vector-memory issue is
        // what bounds this kernel at the end of a period).
        // The plan only keeps neighbouring windows free of shared information
        // variables (dist 1): a value window p+1 reads may have been written by
        // the post of window p-1 in this same period.  The host puts every such
        // source and reader in slab wave 0, which posts before its pre and reads
        // those values back from its own stage (LDS keeps a wave's order); the
        // other waves run their pre first, so their x inputs arrive behind it.
        // A value is stored at the start of the second period after its window's
        // chain, so reads 2 .. R+3 windows later are forwarded (plan depth R + 2).
        // The gathers of window p+1 were the last vector memory operations of
        // period p-R, followed by 4 in each later period: in the main loop (every
        // period does everything, no tail window) vmcnt(4(R-1)) covers them.
        constexpr int MP1 = -1, MP2 = -1;   // mid-phase priorities (none: quarter-period levels measured the same)
        const bool fair = a.slab_prio == 2;
        auto period = [&](auto sc_, auto guarded, int p) __attribute__((always_inline)) {
            constexpr int s = decltype(sc_)::value;   // p % U
            constexpr bool GU = decltype(guarded)::value;
            if (STAMP) tx = stampL();
            const bool dpo = p >= 1 && p <= G, dpr = p + 1 < G, dst = p >= 2 && p <= G + 1;
            const bool fast = !GU && uA != a.tail && uB != a.tail && !sc_tl;
            PreIn in;
            PfIn pi;
            St3 &sp = st[(s + NS - 1) % NS], &sn = st[(s + 1) % NS];
            unsigned long long t1 = 0, t2 = 0, t3 = 0;
            if (fast) {
                // every slab wave posts first (window p-1: chain outputs and the
                // state in VGPRs, nothing from memory) and waits for its window
                // p+1 gathers only before its pre, half a period later than at
                // the period start (the stores of this period are 2 more
                // operations in flight): 47.6 -> 46.9 ms
                if (fair) __builtin_amdgcn_s_setprio(1);
                sl.stores(sc, false);
                const uint32_t xr = sl.read_x(p - 1, sp);
                sl.read_pf(p + 1 + R, pi);
                constexpr int VMW = 4 * (R - 1) + 2;
                sl.template post<false, ET, MP1>(p - 1, xr, sp);
                asm volatile("s_waitcnt vmcnt(%0)" ::"n"(VMW) : "memory");
                sl.read_pre(p + 1, (s + 1) % NI, in, mfc, mfc);
                sl.fwd_read(p + 1, in);   // after the stage writes: distance-2 values (wave 0)
                sl.gathers(pi, (s + R + 1) % NI);
                sl.read_st(p - 1, sc);
                if (STAMP) t1 = t2 = stampL();
                if (fair) __builtin_amdgcn_s_setprio(0);
                sl.template pre<false, ET, MP2>(p + 1, in, sn);
                if (STAMP) t3 = stampL();
            } else {
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                if (dst) sl.stores(sc, sc_tl);
                if (dpo) {
                    if (uA == a.tail)
                        sl.template post<true, ET>(p - 1, sl.read_x(p - 1, sp), sp);
                    else
                        sl.template post<false, ET>(p - 1, sl.read_x(p - 1, sp), sp);
                }
                if (STAMP) t1 = t2 = t3 = stampL();
                if (dpo) {
                    sl.read_st(p - 1, sc);
                    sc_tl = uA == a.tail;
                }
                if (dpr) {
                    sl.read_pre(p + 1, (s + 1) % NI, in, mfc, mfc);
                    if (p + 1 < R + 3) sl.mask_early(p + 1, in.mf);
                    sl.fwd_read(p + 1, in);
                    sl.read_pf(p + 1 + R, pi);
                    if (uB == a.tail)
                        sl.template pre<true, ET>(p + 1, in, sn);
                    else
                        sl.template pre<false, ET>(p + 1, in, sn);
                    sl.gathers(pi, (s + R + 1) % NI);
                }
            }
            if (STAMP) {
                const unsigned long long t5 = stampL();
                sA += t5 - tx;
                if (fast) {
                    sP[0] += t1 - tx;
                    sP[1] += t2 - t1;
                    sP[2] += t3 - t2;
                }
            }
            __syncthreads();
            next(uA);
            next(uB);
        };
        using T = std::true_type;
        using F = std::false_type;
        // periods 0 .. U guarded (their pres drop codes whose source window
        // precedes window 0: U + 2 >= R + 3, the largest forwarding distance)
        static_for<0, U + 1>([&](auto jc) __attribute__((always_inline)) {
            if (decltype(jc)::value <= G) period(std::integral_constant<int, decltype(jc)::value % U>{}, T{}, decltype(jc)::value);
        });
        int p = U + 1;
        // periods p .. p+U-1 with p = 1 (mod U): slot index (1 + j) % U
        for (; p + U - 1 <= G - 2; p += U)
            static_for<0, U>([&](auto jc) __attribute__((always_inline)) {
                period(std::integral_constant<int, (1 + decltype(jc)::value) % U>{}, F{}, p + decltype(jc)::value);
            });
        // the rest (at most U + 1 periods: p .. G), guarded
        static_for<0, U + 1>([&](auto jc) __attribute__((always_inline)) {
            if (p + decltype(jc)::value <= G && p + decltype(jc)::value > U)
                period(std::integral_constant<int, (1 + decltype(jc)::value) % U>{}, T{}, p + decltype(jc)::value);
        });
        sl.stores(sc, sc_tl);   // window G-1
        if (!ET || !et_after(it)) break;
    }
    write_stamps();
    parity_out();
}

__global__ void fill_iters3_k(int batch, int32_t *iters_used, int iters)
{
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b < batch) iters_used[b] = iters;
}

int env_int3(const char *name, int def)
{
    const char *e = getenv(name);
    return (e && *e) ? atoi(e) : def;
}

// diagnostic build (LDPC_COOP3_STAMP=1): per-period cycles of each wave
template <int WS>
void report_stamps3(const unsigned long long *d, int grid, hipStream_t s)
{
    constexpr int nwaves = WS + 1, CHW = WS >= 3 ? 3 : WS;
    std::vector<unsigned long long> h((size_t)grid * nwaves * 8);
    if (hipStreamSynchronize(s) != hipSuccess ||
        hipMemcpy(h.data(), d, h.size() * sizeof(h[0]), hipMemcpyDeviceToHost) != hipSuccess)
        return;
    std::vector<double> v((size_t)nwaves * 8, 0.0);
    for (int b = 0; b < grid; b++)
        for (int w = 0; w < nwaves; w++) {
            const unsigned long long *o = &h[((size_t)b * nwaves + w) * 8];
            const double G = o[7] ? (double)o[7] : 1.0;
            for (int i = 0; i < 6; i++) v[w * 8 + i] += o[i] / G / grid;
            v[w * 8 + 6] += ((o[6] >> 16) & 0xffff) / G / grid;
            v[w * 8 + 7] += (o[6] & 0xffff) / G / grid;
        }
    fprintf(stderr, "coop3 stamps [cycles per period]: elapsed %.0f\n", v[5]);
    for (int w = 0; w < nwaves; w++) {
        const double *x = &v[w * 8];
        if (w == CHW)
            fprintf(stderr, "  chain %d: busy %.0f steps %.0f\n", w, x[0], x[1]);
        else
            fprintf(stderr, "  slab %d: busy %.0f | vmcnt %.0f %s %.0f %s %.0f mem %.0f\n", w, x[0], x[1],
                    w == 0 ? "post" : "pre", x[2], w == 0 ? "pre" : "post", x[3], x[0] - x[1] - x[2] - x[3]);
    }
}

template <int WS, int R>
int launch_wsr(const Coop3Args &a, int grid, bool stamped, hipStream_t s)
{
    constexpr int threads = 64 * (WS + 1);
    if (stamped)
        hipLaunchKernelGGL((coop3_decode<WS, R, true>), dim3(grid), dim3(threads), 0, s, a);
    else
        hipLaunchKernelGGL((coop3_decode<WS, R, false>), dim3(grid), dim3(threads), 0, s, a);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace

// forwarding code of a value written dW windows before the reading window,
// by slot `slot`, record entry e (Slab3::fwd_read): ring slot (g - dW) mod 4 is
// ((-dW) mod 4 + g) mod 4, entry offset (e * (S + 1) + slot) * 16 < 8192
static uint32_t fwd_code3(int dW, int slot, int e, int S)
{
    return ((uint32_t)(-dW) & 3u) << 13 | (uint32_t)(e * (S + 1) + slot) * 16u | (dW == 2 ? 2u : 0u) | 1u;
}

// OMS / MS as coop (coop_params_ok); NMS with factor <= 64 (msg_max <= 63: the
// products fit the i16 halves) at the default WS = 6
bool coop3_params_ok(const ldpc_params *p, const CoopCode &cc)
{
    if (p->algo == LDPC_ALGO_NMS)
        return cc.S == 48 && p->var_min == -127 && p->var_max == 127 && p->msg_max >= 0 && p->msg_max <= 63 &&
               p->factor >= 0 && p->factor <= 64;
    return coop_params_ok(p);
}

// V and P are addressed with 64-bit flat addresses: no batch cap
bool coop3_stride_ok(int stride) { return stride > 0 && stride % 64 == 0; }

size_t coop3_msg_bytes(const ldpc_code *h, int stride) { return (size_t)(h->m + 1) * (size_t)stride * 4; }

// host side of coop3's schedule: the window plan with every window's slots
// permuted (distance-2 forwarding sources and readers in slab wave 0) and the
// records rewritten (forwarding codes, chain steps).  1 = no coop3 schedule
// for this code, 0 = ok, < 0 = error (status set)
int coop3_plan_host(const ldpc_code *h, int ws, int r, Coop3Host &o)
{
    o = Coop3Host{};
    if (!h->staircase || h->n_groups != 2 || h->group_deg[0] != D0) return 1;
    if ((ws != 3 && ws != 4 && ws != 6) || r != 2)
        return ldpc_set_error(LDPC_EINVAL, "LDPC_COOP3_WS must be 3 | 4 | 6 and LDPC_COOP3_R 2");
    const int S = 8 * ws;
    CoopPlan &pl = o.pl;
    // dist 1 (distance-2 sources and readers share slab wave 0); a value is
    // stored at the start of the second period after its window's chain, so
    // reads 2 .. r+3 windows later are forwarded from the LDS stage (plan
    // prefetch depth r + 2)
    if (coop_build_plan(h, S, r + 2, 1, RECW, pl, true) != 0) return 1;
    const int nw = (int)pl.first.size();
    auto rec_at = [&](int u, int k) { return &pl.tab[((size_t)u * S + k) * RECW]; };
    auto code_at = [&](const uint32_t *rec, int j) { return (rec[D0 + 1 + j / 2] >> (16 * (j & 1))) & 0xFFFFu; };
    // distance-2 forwarding sources and readers -> slab wave 0 (slots 0..7);
    // the other checks keep their order, the inactive slots come last
    std::vector<char> special((size_t)nw * S, 0);
    for (int u = 0; u < nw; u++)
        for (int k = 0; k < pl.count[u]; k++)
            for (int j = 0; j < X; j++) {
                const uint32_t f = code_at(rec_at(u, k), j);
                if (f == COOP_FWD_NONE || (f >> 9) != 2) continue;
                special[(size_t)u * S + k] = 1;
                special[(size_t)((u + nw - 2) % nw) * S + ((f >> 3) & 63)] = 1;
            }
    std::vector<int> slot_of((size_t)nw * S), check_at((size_t)nw * S);   // plan slot (= chain step) <-> slot
    for (int u = 0; u < nw; u++) {
        int n = 0;
        for (int pass = 0; pass < 3; pass++)
            for (int k = 0; k < S; k++) {
                const bool act = k < pl.count[u], sp = special[(size_t)u * S + k] != 0;
                if ((pass == 0 && sp) || (pass == 1 && act && !sp) || (pass == 2 && !act)) {
                    if (pass == 0 && n >= 8) return 1;   // more than wave 0 holds: no coop3 schedule
                    slot_of[(size_t)u * S + k] = n;
                    check_at[(size_t)u * S + n] = k;
                    n++;
                }
            }
    }
    std::vector<uint32_t> tab(pl.tab.size());
    for (int u = 0; u < nw; u++)
        for (int kn = 0; kn < S; kn++) {
            const int k = check_at[(size_t)u * S + kn];
            const uint32_t *src = rec_at(u, k);
            uint32_t *rec = &tab[((size_t)u * S + kn) * RECW];
            std::copy(src, src + RECW, rec);
            for (int j = 0; j < 2 * NFW; j++) {   // plan codes -> fwd_code3 (the unused last half: 0)
                const uint32_t f = j < X ? code_at(src, j) : COOP_FWD_NONE;
                uint32_t c = 0;
                if (f != COOP_FWD_NONE) {
                    const int dw = (int)(f >> 9), uw = (u + nw - dw) % nw;
                    c = fwd_code3(dw, slot_of[(size_t)uw * S + ((f >> 3) & 63)], (int)(f & 7), S);
                }
                uint32_t &d = rec[D0 + 1 + j / 2];
                d = (d & ~(0xFFFFu << (16 * (j & 1)))) | (c << (16 * (j & 1)));
            }
            if (k >= pl.count[u]) {   // inactive slot: sink V row n, sink message row m, no flags
                for (int j = 0; j < D0; j++) rec[j] = (uint32_t)h->n;
                rec[D0] = (uint32_t)h->m;
            } else {
                rec[D0] &= COOP_CHK_MASK | COOP_M_ACT;
                if (u == pl.tail) std::swap(rec[X], rec[D0 - 1]);   // prefetch always loads record entry D0-1
            }
            rec[D0] |= (uint32_t)k << STEP_SHIFT;
        }
    pl.tab.swap(tab);
    o.S = S;
    o.nw = nw;
    o.recw = RECW;
    o.d0 = D0;
    return 0;
}

int coop3_upload(const ldpc_code *h, CoopCode *cc)
{
    *cc = CoopCode{};
    Coop3Host ho;
    const int ws = env_int3("LDPC_COOP3_WS", 6), r = env_int3("LDPC_COOP3_R", 2);
    const int rc = coop3_plan_host(h, ws, r, ho);
    if (rc != 0) return rc > 0 ? LDPC_OK : rc;
    CoopPlan &pl = ho.pl;
    const int S = ho.S, nw = ho.nw;
    if (hipMalloc(&cc->d_tab, pl.tab.size() * 4) != hipSuccess) return ldpc_set_error(LDPC_ENOMEM, "coop3 tables");
    if (hipMemcpy(cc->d_tab, pl.tab.data(), pl.tab.size() * 4, hipMemcpyHostToDevice) != hipSuccess) {
        coop_free(cc);
        return ldpc_set_error(LDPC_EDEVICE, "coop3 table upload");
    }
    cc->valid = 1;
    cc->d0 = D0;
    cc->S = S;
    cc->R = r;
    cc->nw = nw;
    cc->tail = pl.tail;
    cc->n_fwd = pl.n_fwd;
    cc->x0 = (int)h->edge_var[h->check_start[0] + X];
    cc->m0 = h->group_cnt[0];
    cc->d1 = h->group_deg[1];
    return LDPC_OK;
}

static int launch_coop3_iters(const DecodeLaunch &L, const CoopCode &cc, int iters, const uint8_t *live,
                              hipStream_t s);

// the ET kernel is instantiated for WS = 6 only, and et_after stages the hard
// bits of all n variables (u16 each) in the workgroup's LDS
bool coop3_et_in_kernel(const CoopCode &cc, int n) { return cc.S == 48 && (size_t)n * 2 <= sizeof(Smem3<6, 2>); }

int launch_coop3(const DecodeLaunch &L, const CoopCode &cc, hipStream_t s)
{
    if (!cc.valid || !coop3_stride_ok(L.stride)) return -1;
    if (L.early && coop3_et_in_kernel(cc, L.n)) {
        // in-kernel early termination (one launch, coop3_decode<.., ET>)
        if (!L.iters_used) return -1;
        if (L.iters == 0) {
            hipLaunchKernelGGL(fill_iters3_k, dim3((L.batch + 255) / 256), dim3(256), 0, s, L.batch, L.iters_used, 0);
            return hipGetLastError() == hipSuccess ? 0 : -1;
        }
        return launch_coop3_iters(L, cc, L.iters, nullptr, s);
    }
    if (L.early) {
        // one launch per iteration; converged codewords keep iterating inside
        // live workgroups, so their V is snapshot when they converge and
        // merged back at the end (L.Vs)
        if (!L.Vs || coop_early_begin(L, s)) return -1;
        for (int it = 0; it < L.iters; it++)
            if (launch_coop3_iters(L, cc, 1, L.live, s) || coop_early_after_iter(L, it, s)) return -1;
        return coop_early_end(L, s);
    }
    if (L.iters_used)
        hipLaunchKernelGGL(fill_iters3_k, dim3((L.batch + 255) / 256), dim3(256), 0, s, L.batch, L.iters_used,
                           L.iters);
    return launch_coop3_iters(L, cc, L.iters, nullptr, s);
}

static int launch_coop3_iters(const DecodeLaunch &L, const CoopCode &cc, int iters, const uint8_t *live,
                              hipStream_t s)
{
    Coop3Args a{};
    a.live = live;
    a.V = (int8_t *)L.V;
    a.Mc = (uint8_t *)L.msg;
    a.tab = cc.d_tab;
    // V layout: rows of L.vpitch codewords, a group's 16 B at wg * 16 in each
    a.pitch = L.vpitch;
    a.wgoff = (size_t)CW;
    a.G = cc.nw * iters;
    a.nw = cc.nw;
    a.tail = cc.tail;
    a.mrows = L.m + 1;
    a.n = L.n;
    a.m = L.m;
    a.k = L.n - L.m;
    a.x0 = cc.x0;
    a.P = L.P;
    const bool et = L.early && live == nullptr;   // in-kernel early termination
    a.ev = L.d_edge_var;
    a.Vs = L.Vs;
    a.iters_used = L.iters_used;
    a.iters = iters;
    a.batch = L.batch;
    a.m0 = cc.m0;
    a.d1 = cc.d1;
    a.rmm = (uint32_t)(L.msg_max * 256 + 255) * 0x00010001u;
    const bool nms = L.algo == LDPC_ALGO_NMS;
    a.coff = nms ? 0u : (uint32_t)(L.param * 256) * 0x00010001u;
    a.offp = nms ? 0u : (uint32_t)(L.param & 0xFFFF) * 0x00010001u;
    a.nmsf = nms ? (uint32_t)(L.param & 0xFFFF) * 0x00010001u : 0u;
    a.prio = env_int3("LDPC_COOP3_PRIO", 1);
    a.slab_prio = env_int3("LDPC_COOP3_SLAB_PRIO", 2);   // 0 none, 1 static (second waves), 2 fair by phase
    const int grid = L.stride / CW;
    a.remap = (grid % 8) == 0 && env_int3("LDPC_COOP3_REMAP", 1) != 0;   // XCD-aware codeword groups
    const int ws = cc.S / 8;
    const bool stamped = env_int3("LDPC_COOP3_STAMP", 0) != 0;
    if (stamped) {
        const size_t bytes = (size_t)grid * (ws + 1) * 8 * sizeof(unsigned long long);
        if (hipMalloc(&a.stamps, bytes) != hipSuccess) return -1;
        (void)hipMemsetAsync(a.stamps, 0, bytes, s);
    }
    int rc;
    if (et) {
        if (stamped) (void)hipFree(a.stamps);
        if (L.algo == LDPC_ALGO_NMS)
            hipLaunchKernelGGL((coop3_decode<6, 2, false, true, true>), dim3(grid), dim3(64 * 7), 0, s, a);
        else
            hipLaunchKernelGGL((coop3_decode<6, 2, false, true>), dim3(grid), dim3(64 * 7), 0, s, a);
        return hipGetLastError() == hipSuccess ? 0 : -1;
    }
    if (L.algo == LDPC_ALGO_NMS) {
        if (ws != 6 || stamped) return -1;
        hipLaunchKernelGGL((coop3_decode<6, 2, false, false, true>), dim3(grid), dim3(64 * 7), 0, s, a);
        return hipGetLastError() == hipSuccess ? 0 : -1;
    }
    if (ws == 6)
        rc = launch_wsr<6, 2>(a, grid, stamped, s);
    else if (ws == 4)
        rc = launch_wsr<4, 2>(a, grid, stamped, s);
    else
        rc = launch_wsr<3, 2>(a, grid, stamped, s);
    if (stamped) {
        if (rc == 0)
            (ws == 6   ? report_stamps3<6>(a.stamps, grid, s)
             : ws == 4 ? report_stamps3<4>(a.stamps, grid, s)
                       : report_stamps3<3>(a.stamps, grid, s));
        (void)hipFree(a.stamps);
    }
    return rc;
}
