// ldsep.hip -- edge-parallel float layered min-sum for short quasi-cyclic
// codes: BASELINE.json configs[1] (802.11n N=648 r1/2, batch 1024, 20
// iterations, float min-sum) and configs[0]'s shape.
//
// Same schedule and arithmetic as the check-serial reference recurrence
// (code/x86/CDecoder/OMS/CDecoder_OMS_fixed_SSE.cpp:172-546, in float as
// SURVEY.md §8(a) defines it, restated by oracle/ldpc_oracle.c
// oracle_decode_f32): layers are maximal runs of consecutive checks sharing
// no variable (lds.hip's plan: one block row of a QC code), so a layer's
// checks commute exactly.  What changes is the mapping:
//
// * one wave = one codeword; a check's edges sit on 8 consecutive lanes (one
//   edge per lane), 8 checks per pass, ceil(width / 8) passes per layer (648:
//   27 checks of degree 7 / 8 -> 4 passes, 48 (layer, pass) slots);
// * each lane keeps its edges' messages in VGPRs for the whole decode (48
//   floats for 648), and the LDS byte offset of its edge's variable per slot
//   (host-built table, loaded once): per layer and pass the only LDS traffic is
//   one V read and one V write per lane;
// * each lane's minimum over the check's OTHER edges and the sign parity of
//   the 8 lanes by a 3-step DPP butterfly (quad_perm xor 1, xor 2,
//   row_half_mirror) on the magnitudes as integers (|c| bit patterns order
//   like the floats) and on the sign bits -- an exclusive-min butterfly (5
//   VALU, r05; min1 / min2 and a select took ~14) whose result equals the
//   reference's (a == min1 ? min2 : min1); each lane's message is its
//   constant with the sign bit of the others' parity xored in (-0.0 exactly
//   as the reference's -r);
// * unused lanes of a check (degree 7 in an 8-lane group) read a sink
//   variable V[N] = -inf: |c| = +inf never wins a minimum, and c < 0 adds one
//   to the sign parity -- exactly the reference's odd-degree flip
//   (sign ^= d & 1, since 8 - d and d have the same parity); the lanes of an
//   empty check slot use a second sink V[N+1] no live check reads.
// Min / max and the xor are order-independent and every per-edge op (sub,
// add, the constant's sub / max or mul) is the oracle's, so the result is
// bit-identical (the float tests keep a 1e-6 tolerance).
#include <algorithm>
#include <cmath>
#include <vector>

#include "kernels.h"
#include "lds.h"

namespace {

constexpr int EP_G = 8;                 // lanes per check
constexpr int EP_CPP = 64 / EP_G;       // checks per pass
constexpr int EP_WAVES = 4;             // codewords (waves) per workgroup

struct EpArgs {
    const float *llr;       // frame-major [batch][N]
    uint8_t *hard;          // frame-major [batch][N], may be null
    float *soft;            // frame-major [batch][N], may be null
    const uint32_t *tab;    // [NL * NP][64]: LDS byte offset of lane's variable in V (sinks N, N+1)
    int n, vstride, batch, iters, nl, algo, early;
    float beta;
    int32_t *iters_used;
    unsigned long long *cnt;   // fused error count (DecodeLaunch::cnt), may be null
    const uint8_t *cnt_ref;
    int cnt_k;
};

// lane permutations inside each group of 8 (every lane written: no old value)
LDPC_DEV uint32_t dpp_xor1(uint32_t x) { return __builtin_amdgcn_mov_dpp((int)x, 0xB1, 0xF, 0xF, true); }
LDPC_DEV uint32_t dpp_xor2(uint32_t x) { return __builtin_amdgcn_mov_dpp((int)x, 0x4E, 0xF, 0xF, true); }
LDPC_DEV uint32_t dpp_hmirror(uint32_t x) { return __builtin_amdgcn_mov_dpp((int)x, 0x141, 0xF, 0xF, true); }

template <int NL, int NP, bool NMS>
__global__ void __launch_bounds__(64 * EP_WAVES) ldsep_decode(EpArgs a)
{
    constexpr int NS = NL * NP;
    constexpr uint32_t SIGN = 0x80000000u;
    extern __shared__ __attribute__((aligned(16))) float ep_smem[];
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const int b = blockIdx.x * EP_WAVES + wave;
    // a wave past the batch skips the decode but stays for the workgroup's
    // error-count reduction (the only workgroup barrier, at the end)
    const bool live_cw = b < a.batch;
    if (!live_cw && !a.cnt) return;
    __shared__ unsigned long long ep_cnt[EP_WAVES][2];
    const uint32_t vbase = (uint32_t)wave * (uint32_t)a.vstride * 4u;
    float *V = ep_smem + (size_t)wave * a.vstride;
    char *L = (char *)ep_smem;
    uint32_t off[NS];   // LDS byte address of this lane's variable per (layer, pass)
    float msg[NS];
#pragma unroll
    for (int s = 0; s < NS; s++) {
        off[s] = a.tab[s * 64 + lane] + vbase;
        msg[s] = 0.0f;   // CDecoder_OMS_fixed_SSE.cpp:129-131
    }
    // LLRs in, -0.0 made +0.0 (x + 0.0f): then no V and no contribution c is
    // ever -0.0 (c = V - msg and V = c + m are -0.0 only from -0.0 operands),
    // so the sign bit of c is exactly the reference's c < 0.  Only the sign of
    // a zero soft value can differ from the reference's, never a comparison.
    const float *src = a.llr + (size_t)b * a.n;
    if (live_cw)
        for (int i = lane; i < a.n; i += 64) V[i] = src[i] + 0.0f;
    if (lane < 2) V[a.n + lane] = -__builtin_huge_valf();
    int it = 0;
    while (live_cw && it < a.iters) {
#pragma unroll
        for (int l = 0; l < NL; l++) {
            float c[NP];
#pragma unroll
            for (int p = 0; p < NP; p++) c[p] = *(const float *)(L + off[l * NP + p]);
#pragma unroll
            for (int p = 0; p < NP; p++) {
                const int s = l * NP + p;
                const float cj = c[p] - msg[s];
                const uint32_t aj = __float_as_uint(cj) & ~SIGN;   // |c| (as an ordered integer)
                const uint32_t sj = __float_as_uint(cj) & SIGN;    // c < 0
                // the minimum over the OTHER 7 lanes of the check (E) by an
                // exclusive-min butterfly: M = the min of this lane's group,
                // E = the min of its group without itself; each stage E =
                // min(E, partner's M), M = min(M, partner's M) (5 VALU, each
                // with its DPP fused).  E is exactly the reference's selection
                // (a_j == min1 ? min2 : min1): min2 is the min without one
                // occurrence of min1
                uint32_t e = dpp_xor1(aj);
                uint32_t mm = min(aj, e);
                e = min(e, dpp_xor2(mm));
                mm = min(mm, dpp_xor2(mm));
                e = min(e, dpp_hmirror(mm));
                uint32_t sg = sj ^ dpp_xor1(sj);
                sg ^= dpp_xor2(sg);
                sg ^= dpp_hmirror(sg);
                // cst of the others' minimum; negative when the parity of the
                // other edges' signs (and the degree flip) is odd
                const float sel = __uint_as_float(e);
                const float r = NMS ? sel * a.beta : fmaxf(sel - a.beta, 0.0f);
                const float m = __uint_as_float(__float_as_uint(r) ^ (sg ^ sj));
                msg[s] = m;
                c[p] = cj + m;
            }
#pragma unroll
            for (int p = 0; p < NP; p++) *(float *)(L + off[l * NP + p]) = c[p];
        }
        it++;
        if (a.early) {   // syndrome of hard(V) over every check (sinks read -inf: never 1)
            uint32_t bad = 0;
#pragma unroll
            for (int s = 0; s < NS; s++) {
                uint32_t h = *(const float *)(L + off[s]) > 0.0f ? 1u : 0u;
                h ^= dpp_xor1(h);
                h ^= dpp_xor2(h);
                h ^= dpp_hmirror(h);
                bad |= h;
            }
            if (__builtin_amdgcn_ballot_w64(bad != 0) == 0) break;
        }
    }
    if (a.iters_used && lane == 0 && live_cw) a.iters_used[b] = it;
    uint8_t *hd = a.hard ? a.hard + (size_t)b * a.n : nullptr;
    float *sd = a.soft ? a.soft + (size_t)b * a.n : nullptr;
    const uint8_t *rf = a.cnt_ref ? a.cnt_ref + (size_t)b * a.n : nullptr;
    int errs = 0;
    for (int i = lane; live_cw && i < a.n; i += 64) {
        const float v = V[i];
        const uint8_t hb = v > 0.0f;   // code/x86/CTools/CTools.cpp:370
        if (hd) hd[i] = hb;
        if (sd) sd[i] = v;
        if (a.cnt && i < a.cnt_k) errs += hb != (rf ? rf[i] : 0);   // CErrorAnalyzer.cpp:123-154
    }
    if (a.cnt) {   // wave = codeword; then the workgroup's 4 codewords: one atomic pair per workgroup
        for (int o = 32; o > 0; o >>= 1) errs += __shfl_xor(errs, o);
        if (lane == 0) {
            ep_cnt[wave][0] = (unsigned long long)errs;
            ep_cnt[wave][1] = errs ? 1ull : 0ull;
        }
        __syncthreads();
        if (threadIdx.x < 2) {
            unsigned long long s = 0;
            for (int w = 0; w < EP_WAVES; w++) s += ep_cnt[w][threadIdx.x];
            if (s) atomicAdd(&a.cnt[threadIdx.x], s);
        }
    }
}

// (NL, NP) shapes compiled: layers x passes of 8 checks
struct EpShape {
    int nl, np;
};
constexpr EpShape kEpShapes[] = {{12, 4}, {11, 6}};   // 648x324 (Z = 27), 576x288 (Z = 24)

}  // namespace

int ldsep_upload(const ldpc_code *h, const std::vector<int4> &layers, LdsCode *lc)
{
    lc->ep_valid = 0;
    if (h->n + 2 > 16384 || layers.empty()) return LDPC_OK;
    int maxw = 0, maxd = 0;
    for (const int4 &L : layers) {
        maxw = std::max(maxw, L.y);
        maxd = std::max(maxd, L.z);
    }
    if (maxd > EP_G) return LDPC_OK;
    const int np = (maxw + EP_CPP - 1) / EP_CPP, nl = (int)layers.size();
    int shape = -1;
    for (int i = 0; i < (int)(sizeof(kEpShapes) / sizeof(kEpShapes[0])); i++)
        if (nl == kEpShapes[i].nl && np <= kEpShapes[i].np && (shape < 0 || kEpShapes[i].np < kEpShapes[shape].np))
            shape = i;
    if (shape < 0) return LDPC_OK;
    const int NP = kEpShapes[shape].np, NL = kEpShapes[shape].nl;
    // [slot][lane] LDS byte offsets: slot (l, p), lane (g, j) = edge j of check 8p + g of layer l
    std::vector<uint32_t> tab((size_t)NL * NP * 64, (uint32_t)(h->n + 1) * 4u);
    for (int l = 0; l < nl; l++) {
        const int4 L = layers[l];
        for (int p = 0; p < NP; p++)
            for (int lane = 0; lane < 64; lane++) {
                const int ck = p * EP_CPP + lane / EP_G, j = lane % EP_G;
                uint32_t v = (uint32_t)(h->n + 1);
                if (ck < L.y) v = j < L.z ? h->edge_var[L.x + ck * L.z + j] : (uint32_t)h->n;
                tab[((size_t)l * NP + p) * 64 + lane] = v * 4u;
            }
    }
    if (hipMalloc(&lc->d_ep_tab, tab.size() * 4) != hipSuccess)
        return ldpc_set_error(LDPC_ENOMEM, "ldsep table");
    if (hipMemcpy(lc->d_ep_tab, tab.data(), tab.size() * 4, hipMemcpyHostToDevice) != hipSuccess)
        return ldpc_set_error(LDPC_EDEVICE, "ldsep table upload");
    lc->ep_nl = nl;
    lc->ep_shape = shape;
    lc->ep_valid = 1;
    return LDPC_OK;
}

bool ldsep_applicable(const ldpc_code *h, const LdsCode &lc, bool is_float)
{
    return is_float && lc.ep_valid && (size_t)EP_WAVES * ((h->n + 2 + 3) / 4 * 4) * 4 <= kLdsMaxBytes;
}

int launch_ldsep(const LdsCode &lc, const ldpc_code *h, const float *llr, uint8_t *hard, float *soft, int batch,
                 int iters, const DecodeLaunch &L, hipStream_t s)
{
    if (!ldsep_applicable(h, lc, true)) return -1;
    EpArgs a{};
    a.llr = llr;
    a.hard = hard;
    a.soft = soft;
    a.tab = lc.d_ep_tab;
    a.n = h->n;
    a.vstride = (h->n + 2 + 3) / 4 * 4;
    a.batch = batch;
    a.iters = iters;
    a.nl = lc.ep_nl;
    a.algo = L.algo;
    a.early = L.early;
    a.beta = L.beta;
    a.iters_used = L.iters_used;
    a.cnt = L.cnt;
    a.cnt_ref = L.cnt_ref;
    a.cnt_k = L.cnt_k;
    const bool nms = L.algo == 1;
    const size_t shm = (size_t)EP_WAVES * a.vstride * 4;
    const dim3 grid((batch + EP_WAVES - 1) / EP_WAVES), block(64 * EP_WAVES);
    switch (lc.ep_shape * 2 + (nms ? 1 : 0)) {
    case 0: hipLaunchKernelGGL((ldsep_decode<12, 4, false>), grid, block, shm, s, a); break;
    case 1: hipLaunchKernelGGL((ldsep_decode<12, 4, true>), grid, block, shm, s, a); break;
    case 2: hipLaunchKernelGGL((ldsep_decode<11, 6, false>), grid, block, shm, s, a); break;
    case 3: hipLaunchKernelGGL((ldsep_decode<11, 6, true>), grid, block, shm, s, a); break;
    default: return -1;
    }
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
