// coop3_kernel.h -- the DVB-S2 staircase-code decoder, third generation: the
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
//   every check that reads a value written two windows earlier sits in slab
//   wave 0 with the check that wrote it, so no wave ever waits for another
//   inside a period (one s_barrier per period);
// * V lives in the grouped layout Vg[group][row][16 codewords] and the
//   information rows move between HBM and the workgroup's LDS as whole 128-B
//   lines (8 rows x 16 codewords) through a line cache planned on the host
//   (linecache.cpp: each line is loaded 3 periods before its first use and
//   written back after its last, one residency serving ~8 checks) -- whole
//   lines, no scattered 16-B V pieces (on MI355X the CU's texture path stalled
//   on those: 47 ms per launch, 18 % of it on the info-row stores alone,
//   DESIGN.md §8);
// * an eighth wave, the memory wave, shares the chain wave's SIMD and issues
//   every vector-memory operation of the workgroup: per period and slab-wave
//   set of 8 slots one LDS-DMA gather (messages + o-edge parity rows), one
//   64-lane line load, one line writeback and one store (messages + x-edge
//   parity rows).  The slab waves only compute (their share of the memory
//   work cost ~10 % of their VALU-bound period);
// * the pre / post of a check read / write its info rows in the line cache,
//   so a value written by the post of window u-1 .. u-2 is simply there for
//   the pre of window u (the host keeps distance-2 writers and readers in slab
//   wave 0, which posts before its pre).
//
// Period p (one s_barrier): chain = steps of window p; slab waves = post of
// window p-1, pre of window p+1; memory wave = stores of window p-2, gathers
// of window p+1+R, the line cache's writebacks / loads of period p and the
// slot writes of the lines loaded in period p-2.
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
#pragma once
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <type_traits>
#include <vector>

#include "coop.h"

#include "pk16.h"

// raw buffer access: address = resource base + voffset (+ soffset)
__device__ i32x4 rbuf_load_v4(i32x4 rsrc, int voffset, int soffset, int aux) __asm("llvm.amdgcn.raw.buffer.load.v4i32");
__device__ void rbuf_store_v4(i32x4 v, i32x4 rsrc, int voffset, int soffset, int aux)
    __asm("llvm.amdgcn.raw.buffer.store.v4i32");

namespace c3 {

// LDS-DMA through a buffer resource: every active lane copies the 16 B at
// rsrc + voff to lds_dst + 16 * lane (as dma16, not counted by the compiler)
LDPC_DEV void dma16_buf(i32x4 rsrc, uint32_t voff, uint32_t lds_dst)
{
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(voff), "s"(rsrc), "s"(lds_dst)
                 : "memory");
}

constexpr int DPER = 2;             // a window table's LDS-DMA is waited for DPER periods after its issue
constexpr int TQ = 8;               // window-table slots in LDS

// Per first-group check degree D0 (G3): DVB-S2 r1/2 (D0 = 7, 5 information
// edges per check) and r2/3 (D0 = 10, 8), code/gpu_fixed/matrix/64800x21600.
//
// slot record (coop3_upload), X = D0 - 2: words 0 .. X-1 the LDS byte offsets
// (from the line cache) of the info entries' 16-B pieces, W_X / W_O the x / o
// edge parity rows (row - k) in their low halves -- W_X's high half the u16
// index of the slot's chain input in xo[buf] and W_O's the byte offset of its
// chain constants in cst[buf] (from its chain step: the pre needs no
// arithmetic on it) -- W_META = check | COOP_M_ACT | chain step << STEP_SHIFT,
// W_LOP .. W_LOP+3 the period's line ops of lane group (slot & 7) of the
// slot's slab wave (LcPlan::ops) as byte offsets: the line loaded, the line
// written back (from the group's V block), the slot written with the load of
// LC_PUT periods earlier, the slot written back (from the line cache)
//
// Messages of a check, per 16-codeword group (MREC bytes): [8 pairs][MA0,
// MB] u32 (MB: eps cst1 / eps cst2 bytes per codeword; MA0: 2-bit codes of
// edges 0..7, 16 bits per codeword), then for each further 8 edges
// [8 pairs][MAk] (edges 8k .. 8k+7): 4 B (D0 <= 8) up to 10 B (D0 <= 32) per
// codeword and check.
//
// First-group degrees 22, 27, 30 (the shaped r5/6, r8/9, r9/10: 20 to 28
// information edges; HALF) put TWO LANES ON EACH CHECK: lane h of a pair
// reduces info edges [h XH, h XH + XH) (XH = 10 / 14 / 14, even; r8/9's half
// 1 carries 3 sink entries, neutralised as c = R(127)), one DPP quad_perm
// [1,0,3,2] exchange merges min1 / min2 / the sign parity, and the x / o
// edges and the chain constants are computed identically in both lanes.  So
// 4 slab waves (one per SIMD) of 4 slots each cover the S = 16 window -- the
// records, messages and line-op words of larger windows would not leave the
// line cache the ~700 live lines these codes need -- with the window plan at
// distance 2 (windows u and u+2 share no information variable either: at S =
// 16 this costs these codes no window, so no slot permutation is needed).
// Records: words [h XH, h XH + XH) are half h's info offsets (sinks past X);
// messages, MREC = 160: [8 pairs][W0, W1] (half 0), [8 pairs][W2, W3] (half
// 1), [8 pairs][MB]: each half's two words hold code slots 0 .. XH-1 (its
// info edges), 14 (the x edge) and 15 (the o edge / the tail's last edge).
// The memory wave keeps its 8-slot sets (NSET = 2): its gathers (11 pieces
// per slot) and stores (12) take two 64-lane instructions per set, as at
// degree 30 before (r05: 2 slab waves of 8 slots, one lane per check, two
// SIMDs idle beside the chain and memory waves).
template <int D0_>
struct G3 {
    static constexpr int D0 = D0_, X = D0 - 2;                 // check degree, information edges per check
    static constexpr bool HALF = D0 >= 22;                     // two lanes per check (see above)
    static constexpr int XH = HALF ? ((X + 1) / 2 + 1) / 2 * 2 : X;   // info edges per lane
    static constexpr int XR = HALF ? 2 * XH : X;               // info words in a record
    static constexpr int NMA = HALF ? 4 : (D0 + 7) / 8;        // edge-code words per codeword pair
    static constexpr int NW = HALF ? 2 : NMA;                  // edge-code words a lane holds
    static constexpr int MREC = HALF ? 160 : 32 * (NMA + 1);   // message bytes per check and group
    static constexpr int MP = MREC / 16;                       // message pieces (16 B) per check
    static constexpr int NG = MP + 1;                          // pieces gathered per slot (+ the o-edge parity row)
    static constexpr int NGI = (8 * NG + 63) / 64;             // gather instructions per 8-slot set
    static constexpr int NSI = (MP + 2 + 7) / 8;               // store instructions per 8-slot set (MP + 2 pieces)
    static constexpr int W_X = XR, W_O = XR + 1, W_META = XR + 2;
    static constexpr int NLD = (X + 7) / 8;                    // line loads / writebacks per lane group and
                                                               // period (a window touches ~S X / 8 new lines)
    static constexpr int W_LOP = (W_META + 1 + 3) / 4 * 4;     // line-op words (NLD uint4)
    static constexpr int RECW = W_LOP + 4 * NLD;               // slot record words
    static constexpr int NR = (W_META + 1 + 3) / 4;            // uint4 a pre reads of its record
    static constexpr int WS = D0 == 7 ? 6 : (D0 <= 14 || HALF) ? 4 : 2;   // slab waves (r1/2's windows fill 45
                                                               // of 48 slots, r2/3's 30 of 32)
    static constexpr int SPW = HALF ? 4 : 8;                   // slots per slab wave: S = SPW WS checks per window
    static constexpr int S = SPW * WS;
    static constexpr int NSET = S / 8;                         // the memory wave's 8-slot sets
    static constexpr int DIST = (WS == 2 || HALF) ? 2 : 1;     // windows closer than DIST + 1 share no info variable
    static constexpr bool KEEP_AD = XH <= 16 && !HALF;        // info edges' LDS offsets kept from pre to post (HALF: re-read)
    static constexpr int LCS = D0 == 7 ? 752 : D0 == 10 ? 848 : D0 == 14 ? 784 : D0 == 22 ? 944 : 896;
                                                               // line-cache slots (128 B each; slot 0 the sink): what
                                                               // the 160 KB of LDS leave beside the rest
    static_assert(NMA <= 4 && NGI <= 2 && NSI <= 2 && LCS <= 1023, "message pieces / slot field");
    static_assert(!HALF || (XH % 2 == 0 && XH <= 14 && 2 * XH >= X), "HALF: code slots 14, 15 are the x / o edges");
};
#ifndef LDPC_C3_MSLEEP
#define LDPC_C3_MSLEEP 4      // memory wave: s_sleep (x 64 cycles) after its line loads, before its LDS burst
#endif
#ifndef LDPC_C3_STAGGER
#define LDPC_C3_STAGGER 1        // WS = 6: the second-dispatched slab waves (3 .. 5, beside waves 0 .. 2 on the
                                 // same SIMDs) run the pre of window p+1 before the post of window p-1: the two
                                 // waves of a SIMD out of phase (MI355X_MICROARCH.md, "try a stagger")
#endif
#ifndef LDPC_C3_CHAIN_B128
#define LDPC_C3_CHAIN_B128 1     // chain constants read as ds_read_b128 (4 LDS cycles per wave-instruction)
                                 // instead of the b96 the compiler narrows the 12-B records to (8 cycles)
#endif
#ifndef LDPC_C3_XEARLY
#define LDPC_C3_XEARLY 1         // pre-first slab waves read their chain inputs (x) at the period start, with
                                 // the pre's inputs, instead of after the pre (r06d same box: 33.41 vs 33.88 ms;
                                 // the post-first waves 1, 2 issuing their pre's reads beside the x read
                                 // 34.40, the memory wave's gather-index reads before its loads 34.06)
#endif
#ifndef LDPC_C3_HALF_KA
#define LDPC_C3_HALF_KA 1        // HALF, fixed iterations: info offsets kept pre -> post, records read a period ahead
#endif
#ifndef LDPC_C3_PRE_CHUNK_X
#define LDPC_C3_PRE_CHUNK_X 8    // pres of checks with >= this many info edges: stage-major chunks, two min chains
#endif
#ifndef LDPC_C3_POST_CHUNK_X
#define LDPC_C3_POST_CHUNK_X 8   // posts of checks with >= this many info edges run new_v in stage-major chunks
#endif
template <int WS, int R, int SPW = 8>
struct Cfg {
    static constexpr int S = SPW * WS;                 // checks per window
    static constexpr int KAHEAD = R + 2 + DPER;        // tables staged KAHEAD windows ahead of the chain
    static constexpr int NI = R + 1;                   // LDS-DMA input windows in flight per slab wave
    static constexpr int NS = R + 1 < 3 ? 3 : R + 1;   // window states in VGPRs (pre at p-1, post at p+1)
    static constexpr int U = NS;                       // periods unrolled (multiple of NI and NS)
    // the chain wave (waves go to SIMDs 0,2,1,3,0,2,1,3): WS = 6: wave 3, a
    // SIMD of its own beside the memory wave (two slab waves on each other
    // SIMD); WS = 4: wave 4, so that the 4 slab waves have a SIMD each (the
    // chain shares SIMD 0, the memory wave SIMD 2)
    static constexpr int CHW = WS == 4 ? 4 : (WS >= 3 ? 3 : WS);
    static constexpr int NB = S / 8;                   // chain blocks of 8 steps
    static_assert(TQ >= KAHEAD + 2, "table ring: a window's records are read until its stores");
    static_assert(U % NI == 0 && U % NS == 0 && U % 3 == 0, "unroll");
};

template <int D0, int WS, int R>
struct alignas(16) Smem3 {
    using CF = Cfg<WS, R, G3<D0>::SPW>;
    using G = G3<D0>;
    static constexpr int NSET = G::NSET;
    static constexpr int S = CF::S, NI = CF::NI;
    uint4 lc[G::LCS][8];              // line cache: slot = 8 V rows x 16 codewords (LcPlan; slot 0: the sink)
    uint32_t tab[TQ][S][G::RECW];     // slot records, window g in slot g % TQ (LDS-DMA by the chain wave)
    uint4 cst[2][S][2][NP];           // chain constants (K1 = (A, B), K2 = (eps, c_o), K3 = (L, H), 0) per step,
                                      // codeword 2q + h at [h][q]   (pre -> chain)
    uint4 xo[2][S / 8][CW];           // chain inputs Y (chain -> post): [block][codeword][8 steps] (a codeword
                                      // swizzle c ^ (c >> 3) that removed this layout's 2-way bank conflict of
                                      // read_x measured 0.3 % slower, r05g; a [step][codeword] u16 layout, one
                                      // dword per pair, cost the chain 8 ds_write_b16 per 8 steps: +4.8 %, r05n)
    struct In {                       // one window's inputs of one 8-slot set, landed by LDS-DMA (lane 8e + slot):
        uint4 d[G::NG][8];            //   e < MP: message bytes 16e .. 16e+15, e = MP: the o-edge parity row
    } in[NSET][NI];                   //   (NGI = 2: the second gather lands pieces 8 .. MP, 1 KB further)
    uint4 mst[2][NSET][8][G::MP + 2]; // window g's outputs per 8-slot set in mst[g & 1], per slot: its new
                                      // messages (pieces 0..MP-1), the x edge's new V (piece MP) and the
                                      // tail's last edge's (MP + 1), 16 codewords each (posted in period
                                      // g+1, stored by the memory wave in period g+2: lane q its piece q)
};

struct Coop3Args {
    int8_t *V;                        // grouped V: Vg[group][row][16], groups gstride bytes apart; row n (and the
                                      // sink line n / 8) is the sink of inactive slots and unused line ops
    uint8_t *Mc;                      // [pitch / 16][mrows][8 pairs][2] u32; row m is the sink
    const uint32_t *tab;              // [nw][S][G3::RECW] slot records
    const uint32_t *lc_pro, *lc_epi;  // line cache: resident lines at a segment start / written back at its end
    unsigned long long *stamps;       // diagnostic build: [grid][waves][4]
    // in-kernel early termination (ET kernels): layered edge list (group 0:
    // checks [0, m0) of degree D0, then degree d1), iterations used per codeword
    const uint32_t *ev;
    int32_t *iters_used;
    int iters, batch, m0, d1, n_pro, n_epi;
    // ET stages (launch_coop3): iterations done before this launch (added to
    // the iterations recorded), the value recorded for codewords still
    // decoding at its end, and the batch read from device memory (a compacted
    // stage's codeword count) when batch_dev is set
    int iter_base, fill;
    const int *batch_dev;
    int G, nw, tail, mrows, n, m, k, x0, remap, prio, slab_prio, mprio;
    uint32_t nmsf;                    // NMS factor per half (value form)
    size_t gstride;                   // bytes between two codeword groups' V
    uint32_t rmm, coff, offp;         // R(msg_max), C(offset) + 255 (R - coff: C form), offset per half (value form)
};

// LEAN (early termination at degree 14: VGPRs): |c| is not kept from pre to
// post but recomputed there (abs_sat / abs_r of c, 2 VALU per edge)
template <int D0, bool LEAN = false, bool KA = G3<D0>::KEEP_AD>
struct St3 {                          // one window's state from pre to post (R / C pairs)
    static constexpr int X = D0 - 2, XL = G3<D0>::XH, NW = G3<D0>::NW;   // (XL: this lane's info edges)
    uint32_t c[XL + 1];               // contributions (info, o); tail: new V
    uint32_t a[LEAN ? 1 : XL + 1];    // |c| (not clipped: min1 / min2 are, where the constants are made)
    uint32_t mn1, mn2, sacc, mx;      // min1 / min2 / sign parity over info + o; x-edge old message
                                      // tail: mn1 = MA0, mn2 = MB, mat = MA1 ..
    uint32_t mat[NW > 1 ? NW - 1 : 1];
    uint32_t xs;                      // the slot's chain step: u16 index of its x input in xo[buf]
    uint32_t ad[KA ? XL : 1];         // the info edges' pair addresses in the line cache (pre reads, post
                                      // writes; !KEEP_AD: the post re-reads them from the window's records)
    uint32_t v[X > 8 ? 1 : X];        // FZ (early termination): the info edges' V as read (R pairs; X > 8:
                                      // re-read from LDS by the post, Slab3::FZ_REREAD)
};

// record meta (word W_META = D0): check | COOP_M_ACT | chain step <<
// STEP_SHIFT.  The host permutes a window's checks over its slots
// (coop3_upload: every distance-2 writer and reader in slab wave 0); the
// chain runs the steps in check order, so a slot's constants / x input sit at
// its step
constexpr int STEP_SHIFT = 22;
static_assert(G3<7>::W_META == 7 && G3<10>::W_META == 10, "meta word = plan record word D0");

LDPC_DEV uint32_t pk_ashr8(uint32_t a) { return us(sv(a) >> (short)8); }
LDPC_DEV uint32_t pk_add(uint32_t a, uint32_t b) { return us(sv(a) + sv(b)); }

constexpr uint32_t V127 = 0x007F007Fu, VNEG127 = 0xFF81FF81u;   // +-127 per half (value form)

// NMS constant of a clipped minimum r (R form, value <= 63) for factor f <= 64
// (value form per half): (v * f) >> 5 as a value / in C form (256 x)
LDPC_DEV uint32_t nms_v(uint32_t r, uint32_t f) { return us(__builtin_bit_cast(s16x2, __builtin_bit_cast(u16x2, pk_mul_lo(pk_ashr8(r), f)) >> (unsigned short)5)); }
LDPC_DEV uint32_t nms_c(uint32_t r, uint32_t f) { return (pk_mul_lo(pk_ashr8(r), f) << 3) & HIBYTES; }   // (<= 4032 << 3: no carry between halves)
LDPC_DEV uint32_t pk_shl5(uint32_t a) { return us(sv(a) << (short)5); }

// a window's records of one slot as a pre reads them: words 0 .. W_META
template <int D0, bool H = G3<D0>::HALF>
struct Rec {
    uint4 r[G3<D0>::NR];
    LDPC_DEV uint32_t w(int i) const
    {
        const uint4 &q = r[i >> 2];
        return (i & 3) == 0 ? q.x : (i & 3) == 1 ? q.y : (i & 3) == 2 ? q.z : q.w;
    }
};
// HALF: this lane's half of the info offsets (words h XH ..) and W_X, W_O, W_META
template <int D0>
struct Rec<D0, true> {
    using G = G3<D0>;
    uint32_t e[G::XH], wx, wo, meta;
    LDPC_DEV uint32_t w(int i) const { return i == G::W_X ? wx : i == G::W_O ? wo : i == G::W_META ? meta : e[i]; }
};
// what a pre reads from LDS
template <int D0, bool KA = G3<D0>::KEEP_AD>
struct PreIn {
    static constexpr int X = D0 - 2, XL = G3<D0>::XH, NW = G3<D0>::NW;
    uint32_t v[XL + 1];               // raw V dwords (info edges from the line cache, the o edge from In)
    uint32_t ad[KA ? XL : 1];         // the info pairs' byte offsets in the line cache
    uint32_t ma[NW], mb;              // old message record of this pair (MA0 .. MA(NW-1), MB; HALF: this half's)
    uint32_t meta, wx, wo;            // record words W_META, W_X, W_O
};

// old message of edge J: edges 8k .. 8k+7 in MA[k]
template <int J, int NMA>
LDPC_DEV uint32_t old_msg2(const uint32_t (&MA)[NMA], const MsgTab &t, const PkK &K)
{
    return old_msg<J & 7>(MA[J >> 3], t, K.m3, K.c4);
}

template <int D0, int WS, int R, bool NMS = false, bool LEAN = false, bool KA_ = G3<D0>::KEEP_AD>
struct Slab3 {
    using SM = Smem3<D0, WS, R>;
    using G = G3<D0>;
    static constexpr bool KA = KA_;   // info offsets kept from pre to post, the next pre's records read a period ahead
    using St = St3<D0, LEAN, KA>;
    using RecT = Rec<D0>;
    using In = PreIn<D0, KA>;
    static constexpr int S = SM::S, X = G::X, XL = G::XH;   // XL: this lane's info edges (HALF: half of them)
    static constexpr int SX = G::HALF ? 14 : X;           // code slot of the x edge
    static constexpr int SO = G::HALF ? 15 : D0 - 1;      // code slot of the o edge
    static constexpr int SL = G::HALF ? 15 : X;           // the tail check's last edge
    SM &sm;
    const Coop3Args &a;
    int k, kl, q, w, lane, tail;      // slot, slot in its 8-slot set, codeword pair, 8-slot set, lane
    uint32_t usel;                    // v_perm selector: this pair's two bytes of a V dword -> R pair
    PkK K;
    uint32_t fk;                      // NMS factor per half (value form)
    char *Vg;                         // the group's V rows (16 B each; parity row k + j at Pr + 16 j)
    // LDS byte offsets of this lane inside a line-cache piece: the pre's V
    // dword (4 (q >> 1)) and the post's u16 (2 q)
    uint32_t lrd, lwr;
    uint32_t mrd, prd;                // byte offsets in an In record: this lane's message pair / o-edge V dword
    uint32_t m1rd;                    // D0 > 8: byte offset of this lane's MA1 word in an In record
    uint32_t fm = 0;                  // FZ: halves of this pair's converged codewords (early termination):
                                      // their V is rewritten unchanged and the chain passes V[p_i] unchanged
    uint32_t psel = 0x0c0c0705u;      // FZ: perm(new, old, psel) = pack_v of new, or of old where converged
    uint32_t psel_raw = 0x0c0c0705u;  // FZ with X > 8: the same from the old pair's raw u16 (re-read from LDS)
    // FZ: X > 8 keeps no copy of the info edges' old V from pre to post (VGPRs);
    // the post re-reads it from the line cache, where it is unchanged until
    // this post writes it (no other window between this pre and post touches it)
    static constexpr bool FZ_REREAD = X > 8;
    // HALF: this lane's half h of its check, -1 in half 1 (its sink entries
    // past X: c = R(127), no sign, never a minimum), the byte offset of its
    // pair's MB word in an In record
    uint32_t h = 0, hm = 0, mbrd = 0;

    LDPC_DEV const char *lcb() const { return (const char *)&sm.lc[0][0]; }
    LDPC_DEV char *lcw() const { return (char *)&sm.lc[0][0]; }

    // ---- reads
    LDPC_DEV RecT read_rec(int g) const
    {
        RecT o;
        if constexpr (G::HALF) {   // words h XH .. h XH + XH - 1 (8-B aligned: XH even), then W_X, W_O, W_META
            const uint32_t *rw = &sm.tab[g & (TQ - 1)][k][0];
            const uint2 *e2 = (const uint2 *)(rw + XL * h);
#pragma unroll
            for (int i = 0; i < XL / 2; i++) {
                const uint2 d = e2[i];
                o.e[2 * i] = d.x;
                o.e[2 * i + 1] = d.y;
            }
            const uint4 m = *(const uint4 *)(rw + G::W_X);
            o.wx = m.x;
            o.wo = m.y;
            o.meta = m.z;
        } else {
            const uint4 *r = (const uint4 *)&sm.tab[g & (TQ - 1)][k][0];
#pragma unroll
            for (int i = 0; i < G::NR; i++) o.r[i] = r[i];
        }
        return o;
    }
    // pre inputs of the window whose records are rc (its gathers landed in in[w][ib])
    LDPC_DEV void read_pre(int ib, const RecT &rc, In &in) const
    {
        const char *inb = (const char *)&sm.in[w][ib];
        if constexpr (KA) {
#pragma unroll
            for (int j = 0; j < XL; j++) in.ad[j] = rc.w(j) + lwr;
        }
#pragma unroll
        for (int j = 0; j < XL; j++) in.v[j] = *(const uint32_t *)(lcb() + rc.w(j) + lrd);   // the dword holding this lane's pair
        in.v[XL] = *(const uint32_t *)(inb + prd);
        if constexpr (G::HALF) {   // this half's (W0, W1) / (W2, W3) of the pair, and MB
            const uint2 mm = *(const uint2 *)(inb + mrd);
            in.ma[0] = mm.x;
            in.ma[1] = mm.y;
            in.mb = *(const uint32_t *)(inb + mbrd);
        } else {
#ifdef C3X_BANK_MM   // bank-conflict attribution (timing-only builds, results wrong): conflict-free address
            const uint2 mm = *(const uint2 *)(inb + 8 * lane);
#else
            const uint2 mm = *(const uint2 *)(inb + mrd);
#endif
            in.ma[0] = mm.x;
            in.mb = mm.y;
#pragma unroll
            for (int i = 1; i < G::NMA; i++) in.ma[i] = *(const uint32_t *)(inb + m1rd + 256 * (i - 1));   // [8 pairs][MAi]
        }
        in.meta = rc.w(G::W_META);
        in.wx = rc.w(G::W_X);
        in.wo = rc.w(G::W_O);
    }
    // the chain inputs' two LDS loads alone (x_of packs them: a read issued early, used late)
    LDPC_DEV uint2 read_x_raw(int g, const St &s) const
    {
        const unsigned short *xs = (const unsigned short *)&sm.xo[g & 1][0][0] + s.xs + 16 * q;
        return make_uint2(xs[0], xs[8]);
    }
    LDPC_DEV static uint32_t x_of(uint2 x) { return perm(x.y, x.x, 0x040d000du); }
    LDPC_DEV uint32_t read_x(int g, const St &s) const   // chain inputs of this slot, codewords 2q, 2q+1 -> R pair
    {
        const unsigned short *xs = (const unsigned short *)&sm.xo[g & 1][0][0] + s.xs + 16 * q;
#ifdef C3X_BANK_X
        const unsigned short *xz = (const unsigned short *)&sm.xo[g & 1][0][0] + 2 * lane;
        const uint32_t x0 = xz[0], x1 = xz[1];
#else
        const uint32_t x0 = xs[0], x1 = xs[8];
#endif
        return perm(x1, x0, 0x040d000du);   // chain values are in [-127, 127]
    }

    // HALF: min1 / min2 / the sign parity of the other lane of this check
    // (lane ^ 1, DPP quad_perm [1,0,3,2]) merged in: the exact smallest and
    // second smallest of the union of both halves' |c|, ties included
    LDPC_DEV static uint32_t swap1(uint32_t x) { return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0xB1, 0xF, 0xF, true); }
    LDPC_DEV static void merge(uint32_t &min1, uint32_t &min2, uint32_t &sacc)
    {
        const uint32_t m1p = swap1(min1), m2p = swap1(min2), sp = swap1(sacc);
        min2 = pk_min(pk_max(min1, m1p), pk_min(min2, m2p));
        min1 = pk_min(min1, m1p);
        sacc ^= sp;
    }

    // pre of window g: chain constants -> cst[g & 1], state -> s
    template <bool TL, bool FZ_ = false, int MP = -1>
    LDPC_DEV void pre(int g, const In &in, St &s) const
    {
        constexpr bool FZ = FZ_;
        const uint32_t meta = in.meta;
        uint32_t v[XL + 1];
#pragma unroll
        for (int j = 0; j <= XL; j++) v[j] = unpack_v(in.v[j], usel);
        if constexpr (KA) {
#pragma unroll
            for (int j = 0; j < XL; j++) s.ad[j] = in.ad[j];
        }
        // HALF: half 1's entries past X are sinks (r8/9: 25 = 14 + 11 + 3): c = R(127)
        auto sink = [&](auto jc, uint32_t c) __attribute__((always_inline)) -> uint32_t {
            constexpr int J = decltype(jc)::value;
            if constexpr (G::HALF && J < XL && J >= X - XL) return bfi(hm, R127, c);
            else return c;
        };
        const MsgTab t = msg_tab(in.mb);
        const uint32_t neg127 = K.neg127, c510 = K.c510;
        uint32_t min1 = R127, min2 = R127, sacc = 0;
        uint32_t A, B, EPS, COV, L, H;
        if constexpr (!TL) {
            // first degree group (OMS_fixed_SSE.cpp:201-218); a = |c| here, the
            // msg_max clip is applied to min1 / min2 (a_j == min1 decides the
            // same edges either way, and min1 == msg_max implies cst1 == cst2)
            // the info edges' contributions stay unclamped (the saturated
            // 0x8000 below R(-128) included): the post uses only their sign
            // and |c| (abs_sat caps it at R(127) as the reference's clamp does)
            if constexpr (XL < LDPC_C3_PRE_CHUNK_X) {
                static_for<0, XL>([&](auto jc) __attribute__((always_inline)) {
                    constexpr int J = decltype(jc)::value;
                    const uint32_t c = pk_sub_sat(v[J], old_msg2<J>(in.ma, t, K));
                    const uint32_t aj = abs_sat(c, c510);
                    s.c[J] = c;
                    if constexpr (!LEAN) s.a[J] = aj;
                    sacc ^= c;
                    if constexpr (J == 0) {   // a <= R(127): the first edge is min1
                        min1 = aj;
                    } else if constexpr (J == 1) {
                        min2 = pk_max(min1, aj);
                        min1 = pk_min(min1, aj);
                    } else {
                        min2 = pk_max(min1, pk_min(aj, min2));
                        min1 = pk_min(min1, aj);
                    }
                });
            } else {
                // many info edges: contributions in stage-major chunks (as the
                // post's new_v) and min1 / min2 as two interleaved chains (even
                // / odd edges) merged at the end -- the exact smallest and second
                // smallest of the union, ties included
                constexpr int PC = 4;
                uint32_t m1[2] = {R127, R127}, m2[2] = {R127, R127};
                static_for<0, (XL + PC - 1) / PC>([&](auto cc) __attribute__((always_inline)) {
                    constexpr int J0 = decltype(cc)::value * PC, E = XL - J0 < PC ? XL - J0 : PC;
                    uint32_t om[E], aj[E];
                    static_for<0, E>([&](auto ec) __attribute__((always_inline)) {
                        constexpr int e = decltype(ec)::value;
                        om[e] = old_msg2<J0 + e>(in.ma, t, K);
                    });
                    __builtin_amdgcn_sched_barrier(0);
                    static_for<0, E>([&](auto ec) __attribute__((always_inline)) {
                        constexpr int e = decltype(ec)::value;
                        s.c[J0 + e] = sink(std::integral_constant<int, J0 + e>{}, pk_sub_sat(v[J0 + e], om[e]));
                    });
                    __builtin_amdgcn_sched_barrier(0);
                    static_for<0, E>([&](auto ec) __attribute__((always_inline)) {
                        constexpr int e = decltype(ec)::value;
                        aj[e] = abs_sat(s.c[J0 + e], c510);
                        if constexpr (!LEAN) s.a[J0 + e] = aj[e];
                        sacc ^= s.c[J0 + e];
                    });
                    __builtin_amdgcn_sched_barrier(0);
                    static_for<0, E>([&](auto ec) __attribute__((always_inline)) {
                        constexpr int e = decltype(ec)::value, h = (J0 + e) & 1;
                        m2[h] = pk_max(m1[h], pk_min(aj[e], m2[h]));
                        m1[h] = pk_min(m1[h], aj[e]);
                    });
                });
                min1 = pk_min(m1[0], m1[1]);
                min2 = pk_min(pk_max(m1[0], m1[1]), pk_min(m2[0], m2[1]));
            }
            if constexpr (G::HALF) merge(min1, min2, sacc);   // the other half's info edges
            if constexpr (MP >= 0) __builtin_amdgcn_s_setprio(MP);   // mid-phase wave priority (fast periods)
            const uint32_t kb = sacc ^ ((D0 & 1) ? SIGNS : 0u);
            const uint32_t cor = pk_max(pk_sub_sat(v[XL], old_msg2<SO>(in.ma, t, K)), neg127);
            const uint32_t ao = abs_r(cor, c510);
            s.c[XL] = cor;
            if constexpr (!LEAN) s.a[XL] = ao;
            s.sacc = sacc ^ cor;
            s.mn2 = pk_max(min1, pk_min(ao, min2));
            s.mn1 = pk_min(min1, ao);
            const uint32_t mx = old_msg2<SX>(in.ma, t, K);
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
                TV = pk_ashr8(pk_max(pk_sub(pk_min(min1, K.rmm), K.coff), 0u));   // coff = C(off) + 255: C form
                EPS = EM | 0x00010001u;
                const uint32_t base = pk_sub(COV, pk_sub(pk_ashr8(mx) ^ EM, EM));   // c_o - eps * m_x
                A = pk_sub(base, a.offp);
                B = pk_add(base, a.offp);
            }
            L = pk_max(pk_sub(COV, TV), VNEG127);
            H = pk_min(pk_add(COV, TV), V127);
            if constexpr (FZ) {   // converged codewords: L = H = V[p_i] as read, the step returns it
                if constexpr (!FZ_REREAD) {
#pragma unroll
                    for (int j = 0; j < X; j++) s.v[j] = v[j];
                }
                const uint32_t VO = pk_ashr8(v[XL]);
                L = bfi(fm, VO, L);
                H = bfi(fm, VO, H);
            }
        } else {
            // the tail check (later degree group: a = |min(c, msg_max)|,
            // OMS_fixed_SSE.cpp:293,314) has no chain input: finish it here
            uint32_t avl[LEAN ? XL + 1 : 1];   // LEAN: the tail's |c| (used in this pre only), else in s.a
            auto av = [&](int j) __attribute__((always_inline)) -> uint32_t & { return LEAN ? avl[LEAN ? j : 0] : s.a[LEAN ? 0 : j]; };
            // edge J (value index; code slot CS): its contribution into min1 / min2 / sacc
            auto tail_edge = [&](auto jc, auto csc) __attribute__((always_inline)) {
                constexpr int J = decltype(jc)::value, CS = decltype(csc)::value;
                const uint32_t c = sink(jc, pk_max(pk_sub_sat(v[J], old_msg2<CS>(in.ma, t, K)), neg127));
                // OMS: a = |min(c, msg_max)| (later group); NMS: min(|c|, msg_max), clipped in min1 / min2;
                // a sink's a = R(127), never a minimum (|min(R(127), msg_max)| would be msg_max)
                const uint32_t aj = sink(jc, NMS ? abs_r(c, c510) : abs_r(pk_min(c, K.rmm), c510));
                s.c[J] = c;
                av(J) = aj;
                sacc ^= c;
                min2 = pk_max(min1, pk_min(aj, min2));
                min1 = pk_min(min1, aj);
            };
            static_for<0, XL>([&](auto jc) __attribute__((always_inline)) { tail_edge(jc, jc); });
            if constexpr (G::HALF) merge(min1, min2, sacc);   // the other half's info edges
            tail_edge(std::integral_constant<int, XL>{}, std::integral_constant<int, SL>{});   // the last edge
            const uint32_t k1 = NMS ? nms_c(pk_min(min2, K.rmm), fk)
                                    : pk_min(pk_max(pk_sub(min2, K.coff), 0u), K.rmm) & HIBYTES;
            const uint32_t k2 = NMS ? nms_c(pk_min(min1, K.rmm), fk)
                                    : pk_min(pk_max(pk_sub(min1, K.coff), 0u), K.rmm) & HIBYTES;
            uint32_t e1, e2, MAn[G::NW];
#pragma unroll
            for (int i = 0; i < G::NW; i++) MAn[i] = 0;
            signed_csts(k1, k2, sacc ^ (((D0 - 1) & 1) ? SIGNS : 0u), e1, e2);
            auto tail_new = [&](auto jc, auto csc) __attribute__((always_inline)) {
                constexpr int J = decltype(jc)::value, CS = decltype(csc)::value;
                s.c[J] = new_v_later<CS & 7>(s.c[J], av(J), min1, e1, e2, MAn[CS >> 3], neg127);
                if constexpr (FZ) s.c[J] = bfi(fm, v[J], s.c[J]);   // converged codewords keep their V
            };
            static_for<0, XL>([&](auto jc) __attribute__((always_inline)) { tail_new(jc, jc); });
            tail_new(std::integral_constant<int, XL>{}, std::integral_constant<int, SL>{});
            s.mx = 0;
            s.sacc = 0;
            s.mn1 = MAn[0];
#pragma unroll
            for (int i = 1; i < G::NW; i++) s.mat[i - 1] = MAn[i];
            s.mn2 = perm(e2, e1, 0x07030501u);
            // the chain passes V[p_0] (the tail's last edge) on: A = B = c_o = L = H = y
            // (NMS: A = 32 y, B = 32 y + 31)
            const uint32_t Y = pk_ashr8(s.c[XL]);
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
        // per codeword records: (A, B), (eps, c_o), (L, H) as i16 pairs (writing
        // the halves with ds_write_b16 / _d16_hi instead of these 6 v_perm ran
        // 3 % slower: 43.7 vs 42.4 ms)
        const int cb = g & 1;
        s.xs = in.wx >> 16;
        uint4 r0, r1;
        r0.x = perm(B, A, 0x05040100u);
        r1.x = perm(B, A, 0x07060302u);
        r0.y = perm(COV, EPS, 0x05040100u);
        r1.y = perm(COV, EPS, 0x07060302u);
        r0.z = perm(H, L, 0x05040100u);
        r1.z = perm(H, L, 0x07060302u);
        // (12-B ds_write_b96 stores of the three used dwords measured 1.7 %
        // slower than these 16-B ones, r06c)
        r0.w = r1.w = 0;
        uint4 *cp = (uint4 *)((char *)&sm.cst[cb][0][0][q] + (in.wo >> 16));
        if (!G::HALF || h == 0) {   // HALF: both lanes of a check hold the same constants
            cp[0] = r0;
            cp[NP] = r1;
        }
    }

    // post of window g (x inputs xr): new info V pairs -> the line cache (at
    // the addresses its pre read), messages and parity V -> mst[g & 1][w][kl];
    // those leave in the memory wave's store of period g + 2
    template <bool TL, bool FZ_ = false, int MP = -1>
    LDPC_DEV void post(int g, uint32_t xr, const St &s) const
    {
        constexpr bool FZ = FZ_;
        unsigned short *sx = (unsigned short *)&sm.mst[g & 1][w][kl][G::MP] + q,
                       *so = (unsigned short *)&sm.mst[g & 1][w][kl][G::MP + 1] + q;
        auto put = [&](uint32_t ad, uint32_t v) __attribute__((always_inline)) {
            *(unsigned short *)(lcw() + ad) = (unsigned short)v;
        };
        // !KEEP_AD: the info edges' line-cache offsets from the window's records
        // (in the ring until its stores), all read here at once (uint4 reads: one
        // LDS round trip, not one per edge: r05o stamps, degree 30, post 4264 of
        // a 6777-cycle period with one ds_read_b32 per edge)
        RecT rp;
        if constexpr (!KA) rp = read_rec(g);
        auto ad_of = [&](int, const St &st, int j) __attribute__((always_inline)) -> uint32_t {
            if constexpr (KA)
                return st.ad[j];
            else
                return rp.w(j) + lwr;
        };
        // edge J's code into MA[J / 8]
        uint32_t MA[G::NW], MB;
#pragma unroll
        for (int i = 0; i < G::NW; i++) MA[i] = 0;
        const bool lead = !G::HALF || h == 0;   // HALF: the x / tail edges' V and MB are the same in both lanes
        auto nv = [&](auto jc, uint32_t c, uint32_t av, uint32_t min1, uint32_t e1, uint32_t e2)
                      __attribute__((always_inline)) -> uint32_t {
            constexpr int J = decltype(jc)::value;
            return new_v<J & 7>(c, av, min1, e1, e2, MA[J >> 3], K.c510);
        };
        if constexpr (!TL) {
            const uint32_t cx = pk_sub_sat(xr, s.mx);   // unclamped, as the info edges' (new_v)
            const uint32_t ax = abs_sat(cx, K.c510);
            const uint32_t sacc = s.sacc ^ cx;
            const uint32_t min2 = pk_max(s.mn1, pk_min(ax, s.mn2)), min1 = pk_min(ax, s.mn1);
            const uint32_t k1 = NMS ? nms_c(pk_min(min2, K.rmm), fk)
                                    : pk_max(pk_sub(pk_min(min2, K.rmm), K.coff), 0u);   // C(max(min - off, 0))
            const uint32_t k2 = NMS ? nms_c(pk_min(min1, K.rmm), fk)
                                    : pk_max(pk_sub(pk_min(min1, K.rmm), K.coff), 0u);
            uint32_t e1, e2;
            signed_csts(k1, k2, sacc ^ ((D0 & 1) ? SIGNS : 0u), e1, e2);
            auto put_new = [&](auto jc, uint32_t n) __attribute__((always_inline)) {
                constexpr int J = decltype(jc)::value;
                const uint32_t ad = ad_of(g, s, J);
                if constexpr (FZ && FZ_REREAD)
                    put(ad, perm(n, *(const unsigned short *)(lcb() + ad), psel_raw));
                else
                    put(ad, FZ ? perm(n, s.v[FZ_REREAD ? 0 : J], psel) : pack_v(n));   // FZ: pack_v of new / old per codeword
            };
            if constexpr (XL < LDPC_C3_POST_CHUNK_X) {
                static_for<0, XL>([&](auto jc) __attribute__((always_inline)) {
                    constexpr int J = decltype(jc)::value;
                    const uint32_t aJ = LEAN ? abs_sat(s.c[J], K.c510) : s.a[LEAN ? 0 : J];
                    put_new(jc, nv(jc, s.c[J], aJ, min1, e1, e2));
                });
            } else {
                // 8 .. 28 info edges: new_v in chunks of PC edges, stage by stage
                // behind scheduling barriers -- left alone the compiler ran the
                // edges one after another (each a ~14-deep dependent chain: one
                // wave per SIMD exposes every latency; r05o stamps: the post 2.2x
                // the pre at degree 30)
                constexpr int PC = 4;
                static_for<0, (XL + PC - 1) / PC>([&](auto cc) __attribute__((always_inline)) {
                    constexpr int J0 = decltype(cc)::value * PC, E = XL - J0 < PC ? XL - J0 : PC;
                    uint32_t av[E], nq[E], T[E], sc[E];
                    static_for<0, E>([&](auto ec) __attribute__((always_inline)) {
                        constexpr int e = decltype(ec)::value;
                        av[e] = LEAN ? abs_sat(s.c[J0 + e], K.c510) : s.a[LEAN ? 0 : J0 + e];
                    });
                    __builtin_amdgcn_sched_barrier(0);
                    static_for<0, E>([&](auto ec) __attribute__((always_inline)) {
                        constexpr int e = decltype(ec)::value;
                        nq[e] = opaque(pk_sra15(pk_sub(min1, av[e])));   // -1: the edge gets cst2
                        sc[e] = opaque(pk_sra15(s.c[J0 + e]));            // -1: c < 0
                    });
                    __builtin_amdgcn_sched_barrier(0);
                    static_for<0, E>([&](auto ec) __attribute__((always_inline)) {
                        constexpr int e = decltype(ec)::value;
                        T[e] = pk_add_sat(av[e], bfi(nq[e], e2, e1));   // R(|c| + eps cst), capped at R(127)
                    });
                    __builtin_amdgcn_sched_barrier(0);
                    static_for<0, E>([&](auto ec) __attribute__((always_inline)) {
                        constexpr int e = decltype(ec)::value, J = J0 + e;
                        MA[J >> 3] = add_code<J & 7>(MA[J >> 3], sc[e], nq[e]);
                        T[e] = bfi(sc[e], pk_sub(K.c510, T[e]), T[e]);   // new_v's result
                    });
                    __builtin_amdgcn_sched_barrier(0);
                    static_for<0, E>([&](auto ec) __attribute__((always_inline)) {
                        put_new(std::integral_constant<int, J0 + decltype(ec)::value>{}, T[decltype(ec)::value]);
                    });
                });
            }
            if constexpr (MP >= 0) __builtin_amdgcn_s_setprio(MP);   // mid-phase wave priority (fast periods)
            // x edge: for converged codewords the chain passed V[p_{i-1}] unchanged
            const uint32_t nx = nv(std::integral_constant<int, SX>{}, cx, ax, min1, e1, e2);
            if (lead) *sx = (unsigned short)(FZ ? perm(nx, xr, psel) : pack_v(nx));
            // the o edge: its code only (the next check rewrites V[o] as its x edge)
            const uint32_t aO = LEAN ? abs_r(s.c[XL], K.c510) : s.a[LEAN ? 0 : XL];
            msg_code<SO & 7>(s.c[XL], aO, min1, MA[SO >> 3]);
            MB = perm(e2, e1, 0x07030501u);
        } else {
            static_for<0, XL>([&](auto jc) __attribute__((always_inline)) {
                constexpr int J = decltype(jc)::value;
                put(ad_of(g, s, J), pack_v(s.c[J]));
            });
            if (lead) {
                *sx = (unsigned short)pack_v(xr);        // V of the last group-0 check's o edge
                *so = (unsigned short)pack_v(s.c[XL]);   // the tail's last edge
            }
            MA[0] = s.mn1;
            MB = s.mn2;
#pragma unroll
            for (int i = 1; i < G::NW; i++) MA[i] = s.mat[i - 1];
        }
        if constexpr (G::HALF) {   // [8 pairs][W0, W1] (half 0), [8 pairs][W2, W3] (half 1), [8 pairs][MB]
            char *mr = (char *)&sm.mst[g & 1][w][kl][0];
            *(uint2 *)(mr + 64 * h + 8 * q) = make_uint2(MA[0], MA[1]);
            if (lead) *(uint32_t *)(mr + 128 + 4 * q) = MB;
        } else {
#ifdef C3X_BANK_MST
            *(uint2 *)((char *)&sm.mst[g & 1][w][0][0] + 8 * lane) = make_uint2(MA[0], MB);
#else
            *(uint2 *)((char *)&sm.mst[g & 1][w][kl][0] + 8 * q) = make_uint2(MA[0], MB);
#endif
#pragma unroll
            for (int i = 1; i < G::NMA; i++)   // [8 pairs][MAi]: pieces 4 + 2 (i - 1) ..
                *(uint32_t *)((char *)&sm.mst[g & 1][w][kl][4 + 2 * (i - 1)] + 4 * q) = MA[i];
        }
    }
};

// LDPC_C3_CHAIN_B128: the step also names the record's 4th dword (unused), so
// its constants are read by one ds_read_b128
#if LDPC_C3_CHAIN_B128
#define C3_KW(KV) (KV).w
#else
#define C3_KW(KV) 0u
#endif
// one chain step: input = half IH of xin, output = half OH of xout (the other
// half of xout is kept); c = (K1, K2, K3) of the step
#define C3_STEP_SAME(XW, KV)                                                                   \
    asm volatile("v_pk_mad_i16 %1, %0, %3, %2 op_sel:[0,0,0] op_sel_hi:[0,0,1]\n\t"           \
                 "v_med3_i16 %1, %1, %3, %1 op_sel:[0,1,1,0]\n\t"                             \
                 "v_med3_i16 %0, %1, %4, %4 op_sel:[0,0,1,1]"                                 \
                 : "+v"(XW), "=&v"(tmp)                                                       \
                 : "v"((KV).x), "v"((KV).y), "v"((KV).z), "v"(C3_KW(KV)))
#define C3_STEP_CROSS(XI, XO, KV)                                                              \
    asm volatile("v_pk_mad_i16 %1, %2, %4, %3 op_sel:[1,0,0] op_sel_hi:[1,0,1]\n\t"           \
                 "v_med3_i16 %1, %1, %4, %1 op_sel:[0,1,1,0]\n\t"                             \
                 "v_med3_i16 %0, %1, %5, %5 op_sel:[0,0,1,0]"                                 \
                 : "+v"(XO), "=&v"(tmp)                                                       \
                 : "v"(XI), "v"((KV).x), "v"((KV).y), "v"((KV).z), "v"(C3_KW(KV)))

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
// PF2: the constants read two blocks of 8 steps ahead instead of one (degree
// 10 only: r2/3 36.38 -> 35.79 ms same box; r1/2 +0.6 %, degrees 14 .. 30
// within 0.5 %, r06ac / r06ad)
template <int WS, int R, int B0, int B1, bool NMS = false, bool PF2 = false, typename SMT>
LDPC_DEV void chain_window3(SMT &sm, int buf, int c, uint32_t (&w)[4])
{
    const uint4 *cp = &sm.cst[buf][0][c & 1][c >> 1];
    constexpr int KST = 2 * NP;       // uint4 between steps
    if constexpr (PF2) {
        uint4 kq[3][8];
#pragma unroll
        for (int i = 0; i < 8; i++) kq[B0 % 3][i] = cp[(B0 * 8 + i) * KST];
        if (B0 + 1 < B1)
#pragma unroll
            for (int i = 0; i < 8; i++) kq[(B0 + 1) % 3][i] = cp[((B0 + 1) * 8 + i) * KST];
        auto put_x = [&](int b, const uint32_t (&v)[4]) __attribute__((always_inline)) {
            sm.xo[buf][b][c] = make_uint4(v[0], v[1], v[2], v[3]);
        };
#pragma unroll
        for (int b = B0; b < B1; b++) {
            if (b + 2 < B1) {
#pragma unroll
                for (int i = 0; i < 8; i++) kq[(b + 2) % 3][i] = cp[((b + 2) * 8 + i) * KST];
            }
            uint32_t tmp;
            if constexpr (NMS) {
                C3_STEP_SAME_NMS(w[0], kq[b % 3][0]);
                C3_STEP_CROSS_NMS(w[0], w[1], kq[b % 3][1]);
                C3_STEP_SAME_NMS(w[1], kq[b % 3][2]);
                C3_STEP_CROSS_NMS(w[1], w[2], kq[b % 3][3]);
                C3_STEP_SAME_NMS(w[2], kq[b % 3][4]);
                C3_STEP_CROSS_NMS(w[2], w[3], kq[b % 3][5]);
                C3_STEP_SAME_NMS(w[3], kq[b % 3][6]);
                put_x(b, w);
                C3_STEP_CROSS_NMS(w[3], w[0], kq[b % 3][7]);
            } else {
                C3_STEP_SAME(w[0], kq[b % 3][0]);
                C3_STEP_CROSS(w[0], w[1], kq[b % 3][1]);
                C3_STEP_SAME(w[1], kq[b % 3][2]);
                C3_STEP_CROSS(w[1], w[2], kq[b % 3][3]);
                C3_STEP_SAME(w[2], kq[b % 3][4]);
                C3_STEP_CROSS(w[2], w[3], kq[b % 3][5]);
                C3_STEP_SAME(w[3], kq[b % 3][6]);
                put_x(b, w);
                C3_STEP_CROSS(w[3], w[0], kq[b % 3][7]);
            }
        }
    } else {
        uint4 kq[2][8];
        // the x inputs of steps 8b .. 8b+7 (positions 0..7 of w) -> xo
        auto put_x = [&](int b, const uint32_t (&v)[4]) __attribute__((always_inline)) {
            sm.xo[buf][b][c] = make_uint4(v[0], v[1], v[2], v[3]);
        };
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
                put_x(b, w);
                C3_STEP_CROSS_NMS(w[3], w[0], kq[b & 1][7]);
            } else {
                C3_STEP_SAME(w[0], kq[b & 1][0]);          // pos 0 -> 1
                C3_STEP_CROSS(w[0], w[1], kq[b & 1][1]);   // pos 1 -> 2
                C3_STEP_SAME(w[1], kq[b & 1][2]);          // 2 -> 3
                C3_STEP_CROSS(w[1], w[2], kq[b & 1][3]);   // 3 -> 4
                C3_STEP_SAME(w[2], kq[b & 1][4]);          // 4 -> 5
                C3_STEP_CROSS(w[2], w[3], kq[b & 1][5]);   // 5 -> 6
                C3_STEP_SAME(w[3], kq[b & 1][6]);          // 6 -> 7
                put_x(b, w);
                C3_STEP_CROSS(w[3], w[0], kq[b & 1][7]);   // 7 -> 0 (the next block's first input)
            }
        }
    }
}

// LDS byte offset of row i of the line of a prologue / epilogue entry
// (z << 26 | slot << 16 | line): piece i ^ z of its slot (LcPlan swizzle)
LDPC_DEV uint32_t lc_piece(uint32_t pw, uint32_t i)
{
    return ((pw >> 16) & LC_SLOT_MASK) * 128u + ((i ^ (pw >> 26)) & 7u) * 16u;
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
// the hard-bit word of a V row piece (16 codewords): bit j = (V_j > 0)
LDPC_DEV uint32_t row_hbits(uint4 y)
{
    return high_bits16(make_uint4(pos_bits(y.x), pos_bits(y.y), pos_bits(y.z), pos_bits(y.w)));
}
// Wave CHW: the chain; the others: slab waves (slab index w: slots 8w .. 8w+7).
// ET: in-kernel early termination -- the decode runs one iteration per
// segment (pipeline drained and the line cache written back at its end), then
// the whole workgroup checks the syndrome of its live codewords (stopping once
// each has a failing check), records the iterations of the codewords
// converging now and freezes them, and leaves when none is live.  Same result
// as the reference's per-codeword stop (oracle: syndrome after every
// iteration), in one launch.
template <int D0, int WS, int R, bool STAMP, bool ET = false, bool NMS = false>
__global__ void __launch_bounds__(64 * (WS + 2)) coop3_decode(Coop3Args a)
{
    using SM = Smem3<D0, WS, R>;
    using CF = Cfg<WS, R, G3<D0>::SPW>;
    using GG = G3<D0>;
    constexpr int S = CF::S, KAHEAD = CF::KAHEAD, U = CF::U, CHW = CF::CHW, NB = CF::NB;
    __shared__ SM sm;

    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const int nb = gridDim.x, id = blockIdx.x;
    const int wg = a.remap ? (id & 7) * (nb >> 3) + (id >> 3) : id;   // XCD-aware codeword groups
    const int batch = (ET && a.batch_dev) ? *a.batch_dev : a.batch;
    const int G = ET ? a.nw : a.G;   // periods per segment (ET: one iteration)
    if (G == 0) return;
    char *Vg = (char *)a.V + (size_t)wg * a.gstride;
    // ---- ET state: [0] live codewords, [1] failing codewords (syndrome)
    __shared__ uint32_t et_sh[2];
    constexpr int NT = 64 * (WS + 2);
    auto et_row = [&](uint32_t v) -> const uint4 * { return (const uint4 *)(Vg + (size_t)v * 16); };
    if constexpr (ET) {
        if (threadIdx.x == 0) {
            const int valid = min(CW, max(0, batch - wg * CW));
            et_sh[0] = (1u << valid) - 1u;
            et_sh[1] = 0;
        }
        if (threadIdx.x < CW && wg * CW + (int)threadIdx.x < batch) a.iters_used[wg * CW + threadIdx.x] = a.fill;
        __syncthreads();
        if (et_sh[0] == 0) return;   // padding columns only
    }
    // slab waves: sP[3] = segment prologues + epilogues (+ ET syndromes), sD =
    // LDS drain at the period barrier;
    // elapsed from the first segment's start, G x segments periods
    unsigned long long sA = 0, sP[4] = {0, 0, 0, 0}, sD = 0, t0 = 0, tx = 0, tseg = 0;
    // stamps: every wave's barrier arrival per period (double-buffered by
    // period parity); the memory wave sums the per-period LAST arrival (sD)
    // (not degrees 10 / 14 nor ET kernels: their stamped waves would spill)
    constexpr bool ARR = STAMP && !ET && D0 != 10 && D0 != 14;
    __shared__ uint32_t st_arr[ARR ? 16 : 1], st_beg[ARR ? 16 : 1];
    auto begin = [&](int p, unsigned long long t) __attribute__((always_inline)) {
        if (ARR) st_beg[(p & 1) * 8 + wave] = (uint32_t)t;
    };
    auto arrive = [&](int p, unsigned long long t) __attribute__((always_inline)) {
        if (ARR) st_arr[(p & 1) * 8 + wave] = (uint32_t)t;   // every lane (same value): no branch before
                                                               // the barrier (tools/check_vmcnt.py)
    };
    int nseg = 1;
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
    // stamps (chain wave): sP[1] cycles of round 0 (from the entry), sP[2]
    // cycles of full syndromes, sD their count
    auto et_stamp = [&](int k, unsigned long long &t) {
        if (STAMP && wave == CHW) {
            const unsigned long long u = stamp3();
            if (k > 0) sP[k] += u - t;
            t = u;
        }
    };
    auto et_after = [&](int it) -> bool {
        unsigned long long te = 0;
        et_stamp(0, te);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the iteration's stores, writebacks and table DMAs
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
            const bool settled = et_round(x, live);
            et_stamp(1, te);
            if (settled) goto et_done;
        }
        {
            if (STAMP && wave == CHW) sD++;
            // the full syndrome: every variable's hard bits staged in LDS (the
            // pipeline's LDS is idle between segments; the launch checks n
            // fits), then the checks, 8 per thread and round with an exit
            // test after each; loads unconditional (clamped index) so a
            // round's loads are in flight together
            uint16_t *hb = reinterpret_cast<uint16_t *>(&sm);
            // HB rows per thread in flight at once: the staging of 1 MB is
            // latency-bound (16 rounds of 8 took ~124k cycles)
            constexpr int HB = 16;
            for (int r0 = 0; r0 < a.n; r0 += NT * HB) {
                uint4 y[HB];
#pragma unroll
                for (int i = 0; i < HB; i++) y[i] = *et_row((uint32_t)min(r0 + i * NT + (int)threadIdx.x, a.n - 1));
#pragma unroll
                for (int i = 0; i < HB; i++)
                    if (r0 + i * NT + (int)threadIdx.x < a.n) hb[r0 + i * NT + threadIdx.x] = (uint16_t)row_hbits(y[i]);
            }
            __syncthreads();
            bool done = false;
            constexpr int CR = D0 <= 10 ? 8 : D0 <= 16 ? 4 : 2;   // checks per thread and round (edge ids in VGPRs)
            for (int c0 = 0; c0 < a.m0 && !done; c0 += NT * CR) {
                uint32_t ev[CR][D0];
#pragma unroll
                for (int r = 0; r < CR; r++) {
                    const int cc = min(c0 + r * NT + (int)threadIdx.x, a.m0 - 1);
#pragma unroll
                    for (int j = 0; j < D0; j++) ev[r][j] = a.ev[(size_t)cc * D0 + j];
                }
                uint32_t f = 0;
#pragma unroll
                for (int r = 0; r < CR; r++) {
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
            et_stamp(2, te);
        }
    et_done:
        const uint32_t fresh = live & ~et_sh[1];   // converged after this iteration
        __syncthreads();
        if (threadIdx.x == 0) {
            et_sh[0] = live & ~fresh;
            et_sh[1] = 0;
        }
        if (fresh && threadIdx.x < CW && ((fresh >> threadIdx.x) & 1u))
            a.iters_used[wg * CW + threadIdx.x] = a.iter_base + it + 1;
        __syncthreads();
        return (live & ~fresh) != 0 && it + 1 < a.iters;
    };
    // stamps (diagnostic build): per wave 8 words: busy, phases 1..3 (slab:
    // vmcnt, first and second half), -, elapsed, -, G
    auto write_stamps = [&]() {
        if (STAMP && lane == 0) {
            unsigned long long *o = a.stamps + ((size_t)id * (WS + 2) + wave) * 8;
            o[0] = sA;
            for (int i = 0; i < 4; i++) o[1 + i] = sP[i];
            o[5] = stamp3() - t0;
            o[6] = sD;
            o[7] = (unsigned long long)G * (unsigned long long)nseg;
        }
    };

    if (wave == CHW) {
        // ------------------------------------------------------------ chain wave
        // the chain's wave priority (a.prio, coop3_chain_prio): s_setprio
        // takes an immediate
        if (a.prio == 3)
            __builtin_amdgcn_s_setprio(3);
        else if (a.prio == 2)
            __builtin_amdgcn_s_setprio(2);
        else if (a.prio == 1)
            __builtin_amdgcn_s_setprio(1);
        constexpr int TABW = S * GG::RECW;   // words per window table
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
            // the chain's first input V[x0] (a parity row)
            w4[0] = (uint32_t)(int)((const int8_t *)et_row((uint32_t)a.x0))[c] & 0xFFFFu;
            int un = KAHEAD % a.nw;
            __syncthreads();   // prologue 1: tables of windows 0 .. KAHEAD-1 and the resident lines in LDS
            __syncthreads();   // prologue 1b: the memory wave's first gathers landed
            __syncthreads();   // prologue 2: constants of window 0 in LDS
            if (STAMP && it == 0) t0 = stamp3();
            for (int p = 0; p <= G; p++) {
                if (STAMP) {
                    tx = stamp3();
                    begin(p, tx);
                }
                // (skipping a window's trailing pass-through steps -- the plan
                // fills ~44.9 of r1/2's 48 slots -- measured -0.3 % on one box
                // and +0.1 % on another, r06c / r06g: not kept)
                if (p < G && cl) chain_window3<WS, R, 0, NB, NMS, D0 == 10>(sm, p & 1, c, w4);
                if (STAMP) sP[0] += stamp3() - tx;
                stage(un, (p + KAHEAD) & (TQ - 1));
                un = (un + 1 == a.nw) ? 0 : un + 1;
                asm volatile("s_waitcnt vmcnt(%0)" ::"n"(CPL * DPER) : "memory");
                if (STAMP) {
                    const unsigned long long t = stamp3();
                    sA += t - tx;
                    arrive(p, t);
                }
                __syncthreads();
            }
            __syncthreads();   // epilogue: the slab waves' line writebacks read the cache
            if (!ET || !et_after(it)) break;
            nseg++;
        }
        write_stamps();
        return;
    }

    const char *Mb = (const char *)a.Mc + (size_t)wg * a.gstride;   // the group's messages (coop3_group_layout)
    constexpr int NI = CF::NI, NS = CF::NS;
    constexpr int MW = WS + 1;   // the memory wave (shares the chain wave's SIMD)
    const int kl = lane >> 3, q = lane & 7;

    if (wave == MW) {
        constexpr int NST = GG::NSET;   // the 8-slot sets (= WS but for HALF: 4 slab waves of 4 slots)
        // memory wave priority (a.mprio; r1/2 same-box A/B: 2 vs 0 -0.35 %)
        if (a.mprio == 3)
            __builtin_amdgcn_s_setprio(3);
        else if (a.mprio == 2)
            __builtin_amdgcn_s_setprio(2);
        else if (a.mprio == 1)
            __builtin_amdgcn_s_setprio(1);
        // ------------------------------------------------------------ memory wave
        // Every vector-memory operation of the workgroup, per period p for each
        // slab wave's set of 8 slots (w = 0..NST-1), in this order: the line
        // loads of period p (8 lines per set, into VGPRs); the LDS-DMA gathers
        // of window p+1+R (messages + o-edge parity rows); the line writebacks
        // of period p (slot -> VGPRs -> HBM); the stores of window p-2
        // (messages + x-edge parity rows); between them (LDS only) the slot
        // writes of the lines loaded in period p-LC_PUT.  Then vmcnt(36) (see
        // mperiod).  Unused ops go to the sink row / line / slot,
        // so the counts are static; tools/check_vmcnt.py checks the emitted ISA
        // against them at build time.
        char *lcb = (char *)&sm.lc[0][0];
        const uint32_t lq = 16u * (uint32_t)q;
        // every access of the group's block (coop3_group_layout: V rows, then
        // messages) through one buffer resource with 32-bit offsets: one VALU
        // per address (shift-and-add with a per-lane shift and base)
        const i32x4 vr = buffer_rsrc(Vg, 0u, 0xFFFFFFFFu);
        const uint32_t moff = (uint32_t)(Mb - (const char *)Vg), poff = (uint32_t)a.k * 16u;
        // gathers, instruction i: lane (kl, q) = (piece e - 8 i, slot): e < MP message
        // piece e, e = MP the o-edge parity row (Smem3::In; a slot-major order
        // without the pair reads' 2-way bank conflict measured 0.3 % slower, r05g)
        constexpr int MP = GG::MP, NGI = GG::NGI, NSI = GG::NSI;
        constexpr uint32_t MREC = GG::MREC;
        constexpr bool MSHIFT = MREC == 64 || MREC == 128;   // record offsets by a shift, else one mad
        constexpr uint32_t MSH = MREC == 64 ? 6u : 7u;
        uint32_t gshl[NGI], goff[NGI], gmul[NGI], gmask[NGI], gsel[NGI];
#pragma unroll
        for (int i = 0; i < NGI; i++) {
            const int e = kl + 8 * i;
            gshl[i] = e < MP ? MSH : 4u;
            goff[i] = e < MP ? moff + 16u * (uint32_t)e : poff;
            gmul[i] = e < MP ? MREC : 16u;
            gmask[i] = e < MP ? COOP_CHK_MASK : 0xFFFFu;
            gsel[i] = (uint32_t)(e < MP ? GG::W_META : GG::W_O);
        }
        // stores, instruction i: lane (kl, q) of slot 8w + kl, piece c = q + 8 i:
        // c < MP message piece c, c = MP the x-edge parity row, c = MP + 1 the
        // tail's last edge, the rest the sink row
        uint32_t sshl[NSI], soff[NSI], smul[NSI], stw[NSI], stm[NSI], snk[NSI], snk_tl[NSI];
        int qp[NSI];   // lane q's piece of a slot's outputs (c > MP + 1: any, to the sink)
#pragma unroll
        for (int i = 0; i < NSI; i++) {
            const int c = q + 8 * i;
            sshl[i] = c < MP ? MSH : 4u;
            soff[i] = c < MP ? moff + 16u * (uint32_t)c : poff;
            smul[i] = c < MP ? MREC : 16u;
            stw[i] = 4u * (uint32_t)(c < MP ? GG::W_META : c == MP ? GG::W_X : GG::W_O);
            stm[i] = c < MP ? COOP_CHK_MASK : 0xFFFFu;
            snk[i] = c >= MP + 1 ? 0xFFFFFFFFu : 0u;
            snk_tl[i] = c >= MP + 2 ? 0xFFFFFFFFu : 0u;
            qp[i] = c < MP + 1 ? c : MP + 1;
        }
        auto goffs = [&](int i, uint32_t idx) __attribute__((always_inline)) -> uint32_t {
            if constexpr (MSHIFT) return (idx << gshl[i]) + goff[i];
            else return idx * gmul[i] + goff[i];
        };
        auto soffs = [&](int i, uint32_t idx) __attribute__((always_inline)) -> uint32_t {
            if constexpr (MSHIFT) return (idx << sshl[i]) + soff[i];
            else return idx * smul[i] + soff[i];
        };
        // the LDS-DMA of gather instruction i (lanes past piece MP inactive)
        auto dma_in = [&](int i, uint32_t idx, int w, int ib) __attribute__((always_inline)) {
            if (lane + 64 * i < 8 * GG::NG)
                dma16_buf(vr, goffs(i, idx), (uint32_t)(uintptr_t)&sm.in[w][ib] + 1024u * (uint32_t)i);
        };
        auto gather = [&](int w, int g, int ib) __attribute__((always_inline)) {
#pragma unroll
            for (int i = 0; i < NGI; i++) dma_in(i, sm.tab[g & (TQ - 1)][8 * w + (lane & 7)][gsel[i]] & gmask[i], w, ib);
        };
        // the store of window g's slots 8w .. 8w+7: its row / check index, read
        // from window g's records one period before the store (the chain wave
        // restages that table slot in the store's period); tl: the tail window,
        // !live: the sink
        auto store_idx = [&](int i, int w, int g, bool tl, bool live) __attribute__((always_inline)) -> uint32_t {
            const uint32_t rw = *(const uint32_t *)((const char *)&sm.tab[g & (TQ - 1)][8 * w + kl][0] + stw[i]) & stm[i];
            return live ? bfi(tl ? snk_tl[i] : snk[i], (uint32_t)a.m, rw) : (uint32_t)a.m;
        };
        auto store_win = [&](int i, int w, int g, uint32_t idx) __attribute__((always_inline)) {
            rbuf_store_v4(__builtin_bit_cast(i32x4, sm.mst[g & 1][w][kl][qp[i]]), vr, (int)soffs(i, idx), 0, 0);
        };
        for (int it = 0;; it++) {   // one segment (ET: one iteration per segment)
            __syncthreads();   // prologue 1: tables and resident lines in LDS
#pragma unroll
            for (int i = 0; i <= R; i++)   // window i -> in[w][i]   (nw > R + 3)
#pragma unroll
                for (int w = 0; w < NST; w++) gather(w, i, i);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();   // prologue 1b: the first windows' gathers landed
            __syncthreads();   // prologue 2
            if (STAMP && it == 0) t0 = stamp3();
            constexpr int NPD = LC_PUT + 1;
            constexpr int NLD = GG::NLD;
            uint4 pend[NPD][NST][NLD];   // line loads of periods p-LC_PUT .. p (written to their slots LC_PUT periods on)
#pragma unroll
            for (int i = 0; i < NPD; i++)
#pragma unroll
                for (int w = 0; w < NST; w++)
#pragma unroll
                    for (int l = 0; l < NLD; l++) pend[i][w][l] = make_uint4(0, 0, 0, 0);
            int uS = a.nw - 1;   // local index of window p-1 (the next period's stores)
            uint32_t sidx[NST][NSI];   // the stores' indices (window p-2), read in period p-1
            uint4 lop[NST][NLD];  // the line ops of period p (byte offsets, record words W_LOP ..), read in period p-1
#pragma unroll
            for (int w = 0; w < NST; w++) {
#pragma unroll
                for (int i = 0; i < NSI; i++) sidx[w][i] = (uint32_t)a.m;
#pragma unroll
                for (int l = 0; l < NLD; l++) lop[w][l] = *(const uint4 *)&sm.tab[0][8 * w + kl][GG::W_LOP + 4 * l];
            }
            // period p, vector memory in this order: the line loads of period
            // p, the gathers of window p+1+R, the line writebacks of period p,
            // the stores of window p-2 (4 NST ops: 24 at NST = 6); vmcnt(6 NST) =
            // 4 NST + 2 NST at its end completes everything up to the gathers of period p-1
            // (the pre of window p+2 reads them next period) and so the line
            // loads of period p-1 (the slot writes of period p+1 take those of
            // period p+1-LC_PUT = p-1), and a writeback two periods after its
            // issue (its line is loaded again >= 3 periods later,
            // linecache.cpp).  The count holds only while the compiler emits
            // exactly these 4 NST vector-memory instructions per period:
            // tools/check_vmcnt.py (run by __graft_entry__.build) checks the
            // ISA.  The compiler's own waits for the line loads it tracks (it
            // does not see the LDS-DMA gathers) are stricter than needed.
            unsigned long long txp = 0;   // (stamps) the previous period's start
            auto mperiod = [&](auto sc_, int p) __attribute__((always_inline)) {
                constexpr int s = decltype(sc_)::value;   // p % NPD
                if (STAMP) tx = stampL();
                if (ARR) {
                    // period p-1: the last wave's barrier arrival (ready: its
                    // LDS ops done) after the first wave's start -> sD, the
                    // spread of the waves' starts -> sP[2].  Lane w reads wave
                    // w's stamps; min / max over lanes 0..7 by xor shuffles (no
                    // loop or branch); after this period's start stamp, so it
                    // is not timed itself
                    begin(p, tx);
                    const bool wl = (lane & 7) < WS + 2;
                    const uint32_t b0 = st_beg[((p - 1) & 1) * 8 + (lane & 7)];
                    const uint32_t a0 = st_arr[((p - 1) & 1) * 8 + (lane & 7)];
                    int e = wl ? (int)(a0 - (uint32_t)txp) : -(1 << 30);   // relative to this wave's start of p-1
                    int b = wl ? (int)(b0 - (uint32_t)txp) : (1 << 30);
                    int bm = wl ? b : -(1 << 30);
#pragma unroll
                    for (int o = 1; o < 8; o <<= 1) {
                        e = max(e, __shfl_xor(e, o));
                        b = min(b, __shfl_xor(b, o));
                        bm = max(bm, __shfl_xor(bm, o));
                    }
                    const int last = __builtin_amdgcn_readfirstlane(e), first = __builtin_amdgcn_readfirstlane(b),
                              spread = __builtin_amdgcn_readfirstlane(bm) - first;
                    sD += p >= 1 ? (unsigned long long)max(0, last - first) : 0ull;
                    sP[2] += p >= 1 ? (unsigned long long)max(0, spread) : 0ull;
                    txp = tx;
                }
                uint32_t gix[NST][NGI];
                uint4 wbd[NST][NLD], std_[NST][NSI];
                auto loads = [&]() __attribute__((always_inline)) {   // line loads of period p
                    static_for<0, NST>([&](auto wc) __attribute__((always_inline)) {
                        constexpr int w = decltype(wc)::value;
                        static_for<0, NLD>([&](auto lc) __attribute__((always_inline)) {
                            constexpr int l = decltype(lc)::value;
                            pend[s][w][l] = __builtin_bit_cast(uint4, rbuf_load_v4(vr, (int)(lop[w][l].x + lq), 0, 0));
                        });
                    });
                };
                auto read_gix = [&]() __attribute__((always_inline)) {   // gather indices of window p+1+R
                    static_for<0, NST>([&](auto wc) __attribute__((always_inline)) {
                        constexpr int w = decltype(wc)::value;
#pragma unroll
                        for (int i = 0; i < NGI; i++)
                            gix[w][i] = sm.tab[(p + 1 + R) & (TQ - 1)][8 * w + (lane & 7)][gsel[i]] & gmask[i];
                    });
                };
                auto read_out = [&]() __attribute__((always_inline)) {   // writeback and store data
                    static_for<0, NST>([&](auto wc) __attribute__((always_inline)) {
                        constexpr int w = decltype(wc)::value;
#ifdef C3X_BANK_MEM
                        wbd[w][0] = *(const uint4 *)(lcb + 16 * lane);
                        std_[w][0] = *(const uint4 *)((const char *)&sm.mst[(p - 2) & 1][w][0][0] + 16 * (lane & 31));
#else
#pragma unroll
                        for (int l = 0; l < NLD; l++)
                            wbd[w][l] = *(const uint4 *)(lcb + (lop[w][l].w ^ lq));   // row q of the swizzled slot
#pragma unroll
                        for (int i = 0; i < NSI; i++) std_[w][i] = sm.mst[(p - 2) & 1][w][kl][qp[i]];
#endif
                    });
                };
                auto slot_writes = [&]() __attribute__((always_inline)) {   // lines loaded in period p-LC_PUT
                    static_for<0, NST>([&](auto wc) __attribute__((always_inline)) {
                        constexpr int w = decltype(wc)::value;
#pragma unroll
                        for (int l = 0; l < NLD; l++) *(uint4 *)(lcb + (lop[w][l].z ^ lq)) = pend[(s + 1) % NPD][w][l];
                    });
                };
                auto gathers = [&]() __attribute__((always_inline)) {
                    static_for<0, NST>([&](auto wc) __attribute__((always_inline)) {
                        constexpr int w = decltype(wc)::value;
#ifndef C3X_BANK_NODMA
#pragma unroll
                        for (int i = 0; i < NGI; i++) dma_in(i, gix[w][i], w, (p + 1 + R) % NI);
#endif
                    });
                };
                // the line loads first (their addresses are in VGPRs), then a
                // pause, so that the slab waves' chain-input reads of the period
                // start are served before the memory wave's LDS burst (same-box
                // A/B: 35.7 -> 35.3 ms with 4 x 64 cycles; 8 was slower again)
                loads();
                if constexpr (LDPC_C3_MSLEEP > 0) __builtin_amdgcn_s_sleep(LDPC_C3_MSLEEP);
                read_gix();
                read_out();
                gathers();
                slot_writes();
                static_for<0, NST>([&](auto wc) __attribute__((always_inline)) {   // writebacks of period p
                    constexpr int w = decltype(wc)::value;
                    static_for<0, NLD>([&](auto lc) __attribute__((always_inline)) {
                        constexpr int l = decltype(lc)::value;
                        rbuf_store_v4(__builtin_bit_cast(i32x4, wbd[w][l]), vr, (int)(lop[w][l].y + lq), 0, 0);
                    });
                });
                static_for<0, NST>([&](auto wc) __attribute__((always_inline)) {   // stores of window p-2 (sink before period 2)
                    constexpr int w = decltype(wc)::value;
#pragma unroll
                    for (int i = 0; i < NSI; i++)
                        rbuf_store_v4(__builtin_bit_cast(i32x4, std_[w][i]), vr, (int)soffs(i, sidx[w][i]), 0, 0);
                });
                // the indices of window p-1's stores and of the next period's line ops
                static_for<0, NST>([&](auto wc) __attribute__((always_inline)) {
                    constexpr int w = decltype(wc)::value;
#pragma unroll
                    for (int i = 0; i < NSI; i++) sidx[w][i] = store_idx(i, w, p - 1, uS == a.tail, p >= 1);
#pragma unroll
                    for (int l = 0; l < NLD; l++)
                        lop[w][l] = *(const uint4 *)&sm.tab[(p + 1) & (TQ - 1)][8 * w + kl][GG::W_LOP + 4 * l];
                });
                if (STAMP) sP[1] += stampL() - tx;
                // the gathers of p-1: (NLD + NSI) NST ops of p-1 and (2 NLD + NGI + NSI) NST of p after them
                asm volatile("s_waitcnt vmcnt(%0)" ::"n"((3 * NLD + NGI + 2 * NSI) * NST) : "memory");
                if (STAMP) {
                    if (ARR) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // arrival = ready, as the slab waves'
                    const unsigned long long t = stampL();
                    sA += t - tx;
                    arrive(p, t);
                }
                __syncthreads();
                uS = (uS + 1 == a.nw) ? 0 : uS + 1;
            };
            int p = 0;
            for (; p + NPD - 1 <= G; p += NPD)
                static_for<0, NPD>([&](auto jc) __attribute__((always_inline)) {
                    mperiod(std::integral_constant<int, decltype(jc)::value>{}, p + decltype(jc)::value);
                });
            static_for<0, NPD - 1>([&](auto jc) __attribute__((always_inline)) {
                if (p + decltype(jc)::value <= G)
                    mperiod(std::integral_constant<int, decltype(jc)::value>{}, p + decltype(jc)::value);
            });
            // the stores of window G-1 (its post ran in period G)
            static_for<0, NST>([&](auto wc) __attribute__((always_inline)) {
#pragma unroll
                for (int i = 0; i < NSI; i++) store_win(i, decltype(wc)::value, G - 1, sidx[decltype(wc)::value][i]);
            });
            __syncthreads();   // epilogue (the slab waves write the resident dirty lines back)
            if (!ET || !et_after(it)) break;
            nseg++;
        }
        write_stamps();
        return;
    }

    // ------------------------------------------------------------ slab waves
    const int sw = wave - (wave > CHW ? 1 : 0);   // slab index
    constexpr int NSL = 64 * WS;                  // slab threads
    const int st_id = sw * 64 + lane;
    // the second-dispatched half of the slab waves loses VALU arbitration to
    // its SIMD partner; static priority evens them out (MI355X_MICROARCH.md,
    // "Two waves per SIMD", item 4)
    if (a.slab_prio == 1 && wave > CHW) __builtin_amdgcn_s_setprio(1);
    constexpr bool LEAN = (ET && GG::XH > 8) || GG::XH > 16 || GG::HALF;   // HALF: |c| recomputed in the post (VGPRs)
    // HALF: the info offsets kept from pre to post and the next pre's records
    // read a period ahead where the VGPRs allow (not the early-termination
    // kernels: their syndrome code's registers)
    // (same box, r06g: shaped r5/6 37.94 vs 38.55 ms re-reading; r9/10 28.37
    // vs 28.26, so degree 22 only)
    constexpr bool KA = GG::KEEP_AD || (LDPC_C3_HALF_KA && GG::HALF && !ET && GG::XH <= 10);
    // lanes: one lane per check, lane = 8 slot + pair (slot k = 8 sw + kl in
    // set sw); HALF: lane = 16 slot + 2 pair + half (slot k = 4 sw + kls,
    // in set k >> 3 at k & 7)
    const int sk = GG::HALF ? 4 * sw + (lane >> 4) : 8 * sw + kl;   // this lane's slot
    const int sq = GG::HALF ? (lane >> 1) & 7 : q;                  // its codeword pair
    const int skl = sk & 7, sset = sk >> 3;                          // its set and slot in the set
    Slab3<D0, WS, R, NMS, LEAN, KA> sl{sm,
                    a,
                    sk,
                    skl,
                    sq,
                    sset,
                    lane,
                    a.tail,
                    0x010d000du + (uint32_t)(sq & 1) * 0x02000200u,
                    PkK{opaque(RNEG127), opaque(R0), opaque(C510), opaque(a.rmm), opaque(a.coff), opaque(0x03000300u),
                        opaque(0x040c000cu)},
                    opaque(a.nmsf),
                    Vg,
                    (uint32_t)(4 * (sq >> 1)),
                    (uint32_t)(2 * sq),
                    GG::HALF ? (uint32_t)(((4 * (lane & 1) + (sq >> 1)) * 8 + skl) * 16 + (sq & 1) * 8)
                             : (uint32_t)(((sq >> 1) * 8 + skl) * 16 + (sq & 1) * 8),
                    (uint32_t)((8 * GG::MP + skl) * 16 + 4 * (sq >> 1)),
                    (uint32_t)(((4 + (sq >> 2)) * 8 + skl) * 16 + (sq & 3) * 4)};
    if constexpr (GG::HALF) {
        sl.h = (uint32_t)(lane & 1);
        sl.hm = (lane & 1) ? 0xFFFFFFFFu : 0u;
        sl.mbrd = (uint32_t)(((8 + (sq >> 2)) * 8 + skl) * 16 + (sq & 3) * 4);   // record byte 128 + 4 q
    }
    auto next = [&](int &u) __attribute__((always_inline)) { u = (u + 1 == a.nw) ? 0 : u + 1; };
    for (int it = 0;; it++) {   // one segment (ET: one iteration per segment)
        if (STAMP) tseg = stamp3();
        // line cache prologue: the lines resident at a segment start
        // (LcPlan::pro), PB pieces per thread in flight at once (ET runs it
        // every iteration: one HBM round trip per batch, not per piece)
        {
            constexpr int PB = 12;
            for (int i0 = st_id; i0 < 8 * a.n_pro; i0 += PB * NSL) {
                uint32_t pw[PB];
                uint4 d[PB];
#pragma unroll
                for (int j = 0; j < PB; j++) pw[j] = a.lc_pro[min(i0 + j * NSL, 8 * a.n_pro - 1) >> 3];
#pragma unroll
                for (int j = 0; j < PB; j++)
                    d[j] = *(const uint4 *)(Vg + (size_t)(pw[j] & 0xFFFFu) * 128 + (uint32_t)((i0 + j * NSL) & 7) * 16u);
#pragma unroll
                for (int j = 0; j < PB; j++)
                    if (i0 + j * NSL < 8 * a.n_pro)
                        *(uint4 *)((char *)&sm.lc[0][0] + lc_piece(pw[j], (uint32_t)((i0 + j * NSL) & 7))) = d[j];
            }
        }
        __syncthreads();   // prologue 1: tables and resident lines in LDS
        if constexpr (ET) {   // codewords 2q (low half) and 2q+1 (high half) of this lane: converged?
            const int valid = min(CW, max(0, batch - wg * CW));
            const uint32_t conv = (((1u << valid) - 1u) & ~et_sh[0]) >> (2 * sq);
            sl.fm = ((conv & 1u) ? 0x0000FFFFu : 0u) | ((conv & 2u) ? 0xFFFF0000u : 0u);
            sl.psel = 0x0c0c0000u | ((conv & 2u) ? 0x0300u : 0x0700u) | ((conv & 1u) ? 0x01u : 0x05u);
            sl.psel_raw = 0x0c0c0000u | ((conv & 2u) ? 0x0100u : 0x0700u) | ((conv & 1u) ? 0x00u : 0x05u);
        }
        St3<D0, LEAN, KA> st[NS];
        __syncthreads();   // prologue 1b: the memory wave's first gathers landed
        PreIn<D0, KA> in;
        // records of the next pre's window, read a period ahead (!KEEP_AD: read
        // by the pre's period itself -- the VGPRs go to the window states)
        Rec<D0> rcn = sl.read_rec(1 % a.nw);
        sl.read_pre(0, sl.read_rec(0), in);
        if (a.tail == 0)
            sl.template pre<true, ET>(0, in, st[0]);
        else
            sl.template pre<false, ET>(0, in, st[0]);
        __syncthreads();   // prologue 2
        if (STAMP) {
            const unsigned long long t = stamp3();
            if (it == 0) t0 = t;
            sP[3] += t - tseg;
        }
        int uA = a.nw - 1;   // local index of window p-1 (post)
        int uB = 1 % a.nw;   // local index of window p+1 (pre)
        // Period p: post of window p-1 (state st[(p-1) % NS], x inputs from the
        // chain's window p-1, info V into the line cache, parity V and messages
        // staged for the memory wave); pre of window p+1 (inputs from the line
        // cache and in[w][(p+1) % NI], -> st[(p+1) % NS]).  No vector memory:
        // the memory wave moves everything.  The plan only keeps neighbouring
        // windows free of shared information variables (dist 1): a value window
        // p+1 reads may have been written by the post of window p-1 in this same
        // period; the host puts every such writer and reader in slab wave 0,
        // which posts before its pre (LDS keeps a wave's order).
        // mid-phase priorities: none -- four levels over the period (3 at its
        // start, 2 mid-post, 1 at the pre, 0 mid-pre) ran 1.2 % slower than two
        constexpr int MP1 = -1, MP2 = -1, P0 = 1, P1 = 0;
        const bool fair = a.slab_prio == 2;
        // guarded: the first and last periods, and those posting or pre-ing the tail window
        auto period = [&](auto sc_, auto guarded_, int p) __attribute__((always_inline)) {
            constexpr int s = decltype(sc_)::value;   // p % U
            constexpr bool GU = decltype(guarded_)::value;
            if (STAMP) {
                tx = stampL();
                begin(p, tx);
            }
            const bool dpo = p >= 1 && p <= G, dpr = p + 1 < G;
            const bool fast = !GU && uA != a.tail && uB != a.tail;
            PreIn<D0, KA> in;
            St3<D0, LEAN, KA> &sp = st[(s + NS - 1) % NS], &sn = st[(s + 1) % NS];
            unsigned long long t1 = 0, t2 = 0, t3 = 0;
            // pre first only at plan distance 2 (same box, r05u: slab waves 1 ..
            // of the distance-1 kernels pre first -- r2/3 39.48 vs 38.98 ms, r1/2
            // 36.79 vs 35.14: a wave that waits for its chain inputs late keeps
            // the partner SIMD's chain / memory wave waiting on the barrier)
            const bool stag = LDPC_C3_STAGGER && WS == 6 && wave > CHW;
            // (WS = 4 at plan distance 1, r2/3 and the shaped r3/4: slab waves 1
            // .. 3 -- no distance-2 pair -- pre first with the x read early
            // measured 2.4 % slower, r06k)
            const bool prefirst = fast && (GG::DIST == 2 || stag);
            if (prefirst) {
                if (stag && fair) __builtin_amdgcn_s_setprio(P0);
                // plan distance 2 (one slab wave per SIMD): windows p-1 and p+1
                // share no information variable, so the pre of window p+1 runs
                // first and hides the wait for the chain's window p-1 outputs the
                // post needs; at distance 1 the same holds for every slab wave
                // but wave 0 (the plan puts each distance-2 writer / reader pair
                // there, and wave 0 keeps posting first)
                uint2 xe = make_uint2(0, 0);
                if (LDPC_C3_XEARLY) xe = sl.read_x_raw(p - 1, sp);   // x issued first: it lands with the pre's inputs
                sl.read_pre((s + 1) % NI, KA ? rcn : sl.read_rec(p + 1), in);
                if constexpr (KA) rcn = sl.read_rec(p + 2);   // (the next period's pre, either order)
                sl.template pre<false, ET>(p + 1, in, sn);
                if (STAMP) t1 = stampL();
                if (stag && fair) __builtin_amdgcn_s_setprio(P1);
                const uint32_t xr = LDPC_C3_XEARLY ? Slab3<D0, WS, R, NMS, LEAN, KA>::x_of(xe) : sl.read_x(p - 1, sp);
                if (STAMP) {
                    asm volatile("" ::"v"(xr));
                    t2 = stampL();
                }
                sl.template post<false, ET>(p - 1, xr, sp);
                if (STAMP) t3 = stampL();
            } else if (fast) {
                // every slab wave posts first (window p-1: chain outputs and the
                // state in VGPRs), then reads and runs its pre
                if (fair) __builtin_amdgcn_s_setprio(P0);
                {
                    const uint32_t xr = sl.read_x(p - 1, sp);
                    if (STAMP) {   // the chain inputs' arrival (the empty asm makes the wave wait for them)
                        asm volatile("" ::"v"(xr));
                        t2 = stampL();
                    }
                    sl.template post<false, ET, MP1>(p - 1, xr, sp);
                    sl.read_pre((s + 1) % NI, KA ? rcn : sl.read_rec(p + 1), in);
                }
                if constexpr (KA) rcn = sl.read_rec(p + 2);
                if (STAMP) t1 = stampL();
                if (fair) __builtin_amdgcn_s_setprio(P1);
                sl.template pre<false, ET, MP2>(p + 1, in, sn);
                if (STAMP) t3 = stampL();
            } else {
                if (dpo) {
                    const uint32_t xr = sl.read_x(p - 1, sp);
                    if (uA == a.tail)
                        sl.template post<true, ET>(p - 1, xr, sp);
                    else
                        sl.template post<false, ET>(p - 1, xr, sp);
                }
                if (STAMP) t1 = t2 = t3 = stampL();
                if (dpr) sl.read_pre((s + 1) % NI, KA ? rcn : sl.read_rec(p + 1), in);
                if constexpr (KA) rcn = sl.read_rec(p + 2);
                if (dpr) {
                    if (uB == a.tail)
                        sl.template pre<true, ET>(p + 1, in, sn);
                    else
                        sl.template pre<false, ET>(p + 1, in, sn);
                }
            }
            if (STAMP) {
                const unsigned long long t5 = stampL();
                // the wave's own LDS ops still in flight at its barrier (the
                // barrier's lgkmcnt(0)): sD
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                const unsigned long long t6 = stampL();
                sD += t6 - t5;
                sA += t5 - tx;
                arrive(p, t6);   // ready for the barrier: own LDS ops done
                if (prefirst) {   // pre first: x wait after it, post, pre
                    sP[0] += t2 - t1;
                    sP[1] += t3 - t2;
                    sP[2] += t1 - tx;
                } else if (fast) {   // x wait, post (+ the pre's read issue), pre
                    sP[0] += (t2 ? t2 : t1) - tx;
                    sP[1] += t1 - (t2 ? t2 : t1);
                    sP[2] += t3 - t1;
                }
            }
            __syncthreads();
            next(uA);
            next(uB);
        };
        using T = std::true_type;
        using F = std::false_type;
        // periods 0 .. U guarded
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
        // line cache epilogue: the dirty lines still resident (LcPlan::epi)
        if (STAMP) tseg = stamp3();
        __syncthreads();
        {
            constexpr int PB = 8;
            for (int i0 = st_id; i0 < 8 * a.n_epi; i0 += PB * NSL) {
                uint32_t pw[PB];
                uint4 d[PB];
#pragma unroll
                for (int j = 0; j < PB; j++) pw[j] = a.lc_epi[min(i0 + j * NSL, 8 * a.n_epi - 1) >> 3];
#pragma unroll
                for (int j = 0; j < PB; j++)
                    d[j] = *(const uint4 *)((const char *)&sm.lc[0][0] + lc_piece(pw[j], (uint32_t)((i0 + j * NSL) & 7)));
#pragma unroll
                for (int j = 0; j < PB; j++)
                    if (i0 + j * NSL < 8 * a.n_epi) {
                        const uint32_t row = (pw[j] & 0xFFFFu) * 8u + (uint32_t)((i0 + j * NSL) & 7);
                        *(uint4 *)(Vg + (size_t)row * 16u) = d[j];
                    }
            }
        }
        const bool more = ET && et_after(it);
        if (STAMP) sP[3] += stamp3() - tseg;
        if (!more) break;
        nseg++;
    }
    write_stamps();
}

// one decode launch of the D0 kernel (its slab-wave count G3<D0>::WS, R = 2):
// fixed iterations or early termination, OMS / MS or NMS, stamped or not
template <int D0>
int launch_d0(const Coop3Args &a, int grid, bool et, bool nms, bool stamped, hipStream_t s)
{
    constexpr int WS = G3<D0>::WS, R = 2, threads = 64 * (WS + 2);
    if (et && nms)
        hipLaunchKernelGGL((coop3_decode<D0, WS, R, false, true, true>), dim3(grid), dim3(threads), 0, s, a);
    else if (et && stamped)
        hipLaunchKernelGGL((coop3_decode<D0, WS, R, true, true>), dim3(grid), dim3(threads), 0, s, a);
    else if (et)
        hipLaunchKernelGGL((coop3_decode<D0, WS, R, false, true>), dim3(grid), dim3(threads), 0, s, a);
    else if (nms)
        hipLaunchKernelGGL((coop3_decode<D0, WS, R, false, false, true>), dim3(grid), dim3(threads), 0, s, a);
    else if (stamped)
        hipLaunchKernelGGL((coop3_decode<D0, WS, R, true>), dim3(grid), dim3(threads), 0, s, a);
    else
        hipLaunchKernelGGL((coop3_decode<D0, WS, R, false>), dim3(grid), dim3(threads), 0, s, a);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace c3

// the per-degree launchers (coop3_deg.hip, one object per first-group degree)
int coop3_launch_d7(const c3::Coop3Args &a, int grid, bool et, bool nms, bool stamped, hipStream_t s);
int coop3_launch_d10(const c3::Coop3Args &a, int grid, bool et, bool nms, bool stamped, hipStream_t s);
int coop3_launch_d14(const c3::Coop3Args &a, int grid, bool et, bool nms, bool stamped, hipStream_t s);
int coop3_launch_d22(const c3::Coop3Args &a, int grid, bool et, bool nms, bool stamped, hipStream_t s);
int coop3_launch_d27(const c3::Coop3Args &a, int grid, bool et, bool nms, bool stamped, hipStream_t s);
int coop3_launch_d30(const c3::Coop3Args &a, int grid, bool et, bool nms, bool stamped, hipStream_t s);
