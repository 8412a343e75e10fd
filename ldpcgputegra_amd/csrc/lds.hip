// lds.hip -- LDS-resident layered min-sum decoder for short codes (int8 and
// float): BASELINE.json configs[0..1] (802.11n N=648 r1/2, 20 iterations,
// batch 1024, float min-sum) and the reference's other short tables.
//
// For N and E small enough, a codeword's whole decoder state -- V[N] and the
// per-edge messages msg[E] -- fits in LDS, so a decode reads the LLRs once
// and writes the hard decisions once and every iteration runs out of LDS.
// The layered schedule (the table order, code/x86/CDecoder/OMS/
// CDecoder_OMS_fixed_SSE.cpp:172-546) is split on the host into layers:
// maximal runs of consecutive checks of one degree group that share no
// variable.  Checks inside a layer commute exactly (each one reads and writes
// only its own variables), so a layer's checks run on parallel lanes and the
// result is bit-identical to the check-serial reference.  For a quasi-cyclic
// code a layer is one block row (Z checks: 27 for N=648).
//
// Mapping: one wave = CPW codewords, LPC = 64 / CPW lanes per codeword
// (LPC >= the widest layer when that is <= 32, else 64 and lanes loop).
// LDS per wave: the layer-major edge table (u16, shared by the wave's
// codewords), then V[CPW][N] and msg[CPW][E] in the element type.  Layer
// descriptors are wave-uniform (scalar loads).  Per-check arithmetic is the
// generic kernel's (generic.hip check_i8 / check_f32, same op order).
//
// Roofline: the HBM traffic is N sizeof(T) in + N out per codeword; the
// kernel is bound by LDS latency / VALU issue, not HBM.
#include <algorithm>
#include <vector>

#include "kernels.h"
#include "lds.h"

namespace {

struct LdsArgs {
    const void *llr;          // frame-major [batch][N] (T)
    uint8_t *hard;            // frame-major [batch][N] 0/1, may be null
    void *soft;               // frame-major [batch][N] (T), may be null
    const uint16_t *tab;      // [E] layer-major edge -> variable
    const int4 *layers;       // [nl] (edge base, checks, degree, later-group flag)
    int nl, n, e, batch, iters;
    int lpc_log2;             // lanes per codeword = 1 << lpc_log2
    int algo, param, var_min, msg_max, early;
    float beta;
    int32_t *iters_used;
    int tab_bytes;            // LDS bytes of the table, 16-B aligned
};

template <int D, bool LATER>
LDPC_DEV void lds_check_i8(int8_t *V, int8_t *msg, const uint16_t *tab, int cnt, const LdsArgs &a)
{
    int c[D], av[D], idx[D];
    int sign = 0, min1 = 127, min2 = 127;
#pragma unroll
    for (int j = 0; j < D; j++) {
        idx[j] = tab[j * cnt];
        const int cj = max(sat8((int)V[idx[j]] - (int)msg[j * cnt]), a.var_min);
        const int aj = LATER ? abs8(min(cj, a.msg_max)) : min(abs8(cj), a.msg_max);
        sign ^= cj & 0x80;
        c[j] = cj;
        av[j] = aj;
        const int t = min1;
        min1 = min(aj, min1);
        min2 = min(min2, max(aj, t));
    }
    int cst1, cst2;
    check_constants(a.algo, a.param, a.msg_max, min1, min2, cst1, cst2);
    sign ^= (D & 1) ? 0xC0 : 0x40;
#pragma unroll
    for (int j = 0; j < D; j++) {
        const int r = (av[j] == min1) ? cst1 : cst2;
        const int sig = as_i8(sign ^ (c[j] & 0x80));
        const int m = sig < 0 ? as_i8(-r) : r;
        msg[j * cnt] = (int8_t)m;
        V[idx[j]] = (int8_t)max(sat8(c[j] + m), a.var_min);
    }
}

template <int D>
LDPC_DEV void lds_check_f32(float *V, float *msg, const uint16_t *tab, int cnt, const LdsArgs &a)
{
    float c[D], av[D];
    int idx[D];
    int sign = D & 1;
    float min1 = __builtin_huge_valf(), min2 = __builtin_huge_valf();
#pragma unroll
    for (int j = 0; j < D; j++) {
        idx[j] = tab[j * cnt];
        const float cj = V[idx[j]] - msg[j * cnt];
        const float aj = fabsf(cj);
        sign ^= (cj < 0.0f);
        c[j] = cj;
        av[j] = aj;
        const float t = min1;
        min1 = fminf(aj, min1);
        min2 = fminf(min2, fmaxf(aj, t));
    }
    float cst1, cst2;
    if (a.algo == 1) {
        cst1 = min2 * a.beta;
        cst2 = min1 * a.beta;
    } else {
        cst1 = fmaxf(min2 - a.beta, 0.0f);
        cst2 = fmaxf(min1 - a.beta, 0.0f);
    }
#pragma unroll
    for (int j = 0; j < D; j++) {
        const float r = (av[j] == min1) ? cst1 : cst2;
        const float m = (sign ^ (c[j] < 0.0f)) ? -r : r;
        msg[j * cnt] = m;
        V[idx[j]] = c[j] + m;
    }
}

// Two lanes per check (SPLIT): lane half h takes edges h, h + 2, ...; the
// partial (min1, min2, sign) of the two halves are exchanged with one DPP
// swap of neighbouring lanes and merged: min1 = min(a1, b1), min2 =
// min(a2, b2, max(a1, b1)) is exactly the smallest / second smallest of the
// whole multiset, so the messages are those of the serial loop above.
LDPC_DEV int swap_pair(int x) { return __builtin_amdgcn_mov_dpp(x, 0xB1, 0xF, 0xF, false); }   // quad_perm [1,0,3,2]
LDPC_DEV float swap_pair(float x) { return __int_as_float(swap_pair(__float_as_int(x))); }

template <int D, bool LATER>
LDPC_DEV void lds_check_i8_split(int8_t *V, int8_t *msg, const uint16_t *tab, int cnt, int h, const LdsArgs &a)
{
    constexpr int DH = (D + 1) / 2;
    int c[DH], av[DH], idx[DH];
    int sign = 0, min1 = 127, min2 = 127;
#pragma unroll
    for (int k = 0; k < DH; k++) {
        const int j = 2 * k + h;
        const bool ok = (D % 2 == 0) || k < DH - 1 || h == 0;
        idx[k] = ok ? tab[j * cnt] : 0;
        const int cj = ok ? max(sat8((int)V[idx[k]] - (int)msg[j * cnt]), a.var_min) : 0;
        const int aj = ok ? (LATER ? abs8(min(cj, a.msg_max)) : min(abs8(cj), a.msg_max)) : 127;
        sign ^= cj & 0x80;
        c[k] = cj;
        av[k] = aj;
        const int t = min1;
        min1 = min(aj, min1);
        min2 = min(min2, max(aj, t));
    }
    const int p1 = swap_pair(min1), p2 = swap_pair(min2), ps = swap_pair(sign);
    min2 = min(min(min2, p2), max(min1, p1));
    min1 = min(min1, p1);
    sign ^= ps;
    int cst1, cst2;
    check_constants(a.algo, a.param, a.msg_max, min1, min2, cst1, cst2);
    sign ^= (D & 1) ? 0xC0 : 0x40;
#pragma unroll
    for (int k = 0; k < DH; k++) {
        const int j = 2 * k + h;
        const bool ok = (D % 2 == 0) || k < DH - 1 || h == 0;
        const int r = (av[k] == min1) ? cst1 : cst2;
        const int sig = as_i8(sign ^ (c[k] & 0x80));
        const int m = sig < 0 ? as_i8(-r) : r;
        if (ok) {
            msg[j * cnt] = (int8_t)m;
            V[idx[k]] = (int8_t)max(sat8(c[k] + m), a.var_min);
        }
    }
}

template <int D>
LDPC_DEV void lds_check_f32_split(float *V, float *msg, const uint16_t *tab, int cnt, int h, const LdsArgs &a)
{
    constexpr int DH = (D + 1) / 2;
    float c[DH], av[DH];
    int idx[DH];
    int sign = 0;
    float min1 = __builtin_huge_valf(), min2 = __builtin_huge_valf();
#pragma unroll
    for (int k = 0; k < DH; k++) {
        const int j = 2 * k + h;
        const bool ok = (D % 2 == 0) || k < DH - 1 || h == 0;
        idx[k] = ok ? tab[j * cnt] : 0;
        const float cj = ok ? V[idx[k]] - msg[j * cnt] : 0.0f;
        const float aj = ok ? fabsf(cj) : __builtin_huge_valf();
        sign ^= (cj < 0.0f);
        c[k] = cj;
        av[k] = aj;
        const float t = min1;
        min1 = fminf(aj, min1);
        min2 = fminf(min2, fmaxf(aj, t));
    }
    const float p1 = swap_pair(min1), p2 = swap_pair(min2);
    const int ps = swap_pair(sign);
    min2 = fminf(fminf(min2, p2), fmaxf(min1, p1));
    min1 = fminf(min1, p1);
    sign ^= ps ^ (D & 1);
    float cst1, cst2;
    if (a.algo == 1) {
        cst1 = min2 * a.beta;
        cst2 = min1 * a.beta;
    } else {
        cst1 = fmaxf(min2 - a.beta, 0.0f);
        cst2 = fmaxf(min1 - a.beta, 0.0f);
    }
#pragma unroll
    for (int k = 0; k < DH; k++) {
        const int j = 2 * k + h;
        const bool ok = (D % 2 == 0) || k < DH - 1 || h == 0;
        const float r = (av[k] == min1) ? cst1 : cst2;
        const float m = (sign ^ (c[k] < 0.0f)) ? -r : r;
        if (ok) {
            msg[j * cnt] = m;
            V[idx[k]] = c[k] + m;
        }
    }
}

// the checks li, li + LPC, ... of one layer (lane li of its codeword)
// LATER (int8 only): the later-degree-group rule of a2, a template
// parameter so that the edge loop is straight-line and its LDS loads batch
template <typename T, int D, bool SPLIT, bool LATER>
LDPC_DEV void lds_layer(T *V, T *msg, const uint16_t *tab, int base, int cnt, int li, int lpc, const LdsArgs &a)
{
    if constexpr (SPLIT) {   // lanes 2i, 2i+1: check i (the pair stays together through the loop)
        const int h = li & 1;
        for (int i = li >> 1; i < cnt; i += lpc >> 1) {
            if constexpr (sizeof(T) == 1)
                lds_check_i8_split<D, LATER>((int8_t *)V, (int8_t *)msg + base + i, tab + base + i, cnt, h, a);
            else
                lds_check_f32_split<D>((float *)V, (float *)msg + base + i, tab + base + i, cnt, h, a);
        }
        return;
    }
    for (int i = li; i < cnt; i += lpc) {
        if constexpr (sizeof(T) == 1)
            lds_check_i8<D, LATER>((int8_t *)V, (int8_t *)msg + base + i, tab + base + i, cnt, a);
        else
            lds_check_f32<D>((float *)V, (float *)msg + base + i, tab + base + i, cnt, a);
    }
}

#define LDPC_LDS_DEG_CASES(X) \
    X(2) X(3) X(4) X(5) X(6) X(7) X(8) X(9) X(10) X(11) X(12) X(13) X(14) X(15) X(16) X(17) X(18) X(19) \
    X(20) X(21) X(22) X(23) X(24) X(25) X(26) X(27) X(28) X(29) X(30) X(31) X(32)

template <typename T, bool SPLIT>
__global__ void __launch_bounds__(64) lds_decode(LdsArgs a)
{
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int lane = threadIdx.x;
    const int lpc = 1 << a.lpc_log2, cpw = 64 >> a.lpc_log2;
    const int cl = lane >> a.lpc_log2, li = lane & (lpc - 1);
    const int b = blockIdx.x * cpw + cl;
    const bool active = b < a.batch;
    const int N = a.n, E = a.e;
    uint16_t *tab = (uint16_t *)smem;
    T *Vall = (T *)(smem + a.tab_bytes);
    T *V = Vall + (size_t)cl * N;
    T *msg = Vall + (size_t)cpw * N + (size_t)cl * E;

    // stage the table (whole wave), the LLRs (coalesced, one codeword per
    // lane group) and zero the messages (CDecoder_OMS_fixed_SSE.cpp:129-131)
    {   // 16-B chunks (the device table is padded to tab_bytes), loads batched
        const uint4 *g = (const uint4 *)a.tab;
        uint4 *l = (uint4 *)smem;
#pragma unroll 8
        for (int i = lane; i < a.tab_bytes / 16; i += 64) l[i] = g[i];
    }
    const T *src = (const T *)a.llr + (size_t)b * N;
    if (active) {
        if ((N * sizeof(T)) % 16 == 0) {
            const uint4 *g = (const uint4 *)src;
            uint4 *l = (uint4 *)V;
#pragma unroll 8
            for (int i = li; i < (int)(N * sizeof(T) / 16); i += lpc) l[i] = g[i];
        } else {
#pragma unroll 8
            for (int i = li; i < N; i += lpc) V[i] = src[i];
        }
    } else {
        for (int i = li; i < N; i += lpc) V[i] = (T)0;
    }
#pragma unroll 8
    for (int i = li; i < E; i += lpc) msg[i] = (T)0;
    __syncthreads();

    const unsigned long long gmask = (lpc == 64 ? ~0ull : ((1ull << lpc) - 1)) << (cl * lpc);
    bool live = active;
    int it = 0;
    for (; it < a.iters; it++) {
        if (!__builtin_amdgcn_ballot_w64(live)) break;
        for (int l = 0; l < a.nl; l++) {
            const int4 L = a.layers[l];   // wave-uniform
            if (live) {
                switch (L.z) {
#define X(DD) \
    case DD:                                                                                  \
        if (sizeof(T) == 1 && L.w != 0 && a.algo != 1)                                        \
            lds_layer<T, DD, SPLIT, sizeof(T) == 1>(V, msg, tab, L.x, L.y, li, lpc, a);       \
        else                                                                                  \
            lds_layer<T, DD, SPLIT, false>(V, msg, tab, L.x, L.y, li, lpc, a);                \
        break;
                    LDPC_LDS_DEG_CASES(X)
#undef X
                default: break;
                }
            }
            __syncthreads();   // one wave: orders the layer's LDS writes before the next layer's reads
        }
        if (a.early && live) {
            // syndrome of hard(V) over this lane's checks of every layer
            int bad = 0;
            for (int l = 0; l < a.nl; l++) {
                const int4 L = a.layers[l];
                for (int i = li; i < L.y; i += lpc) {
                    int par = 0;
                    for (int j = 0; j < L.z; j++) par ^= (V[tab[L.x + j * L.y + i]] > (T)0);
                    bad |= par;
                }
            }
            const unsigned long long anybad = __builtin_amdgcn_ballot_w64(bad != 0) & gmask;
            if (!anybad) {
                live = false;
                if (a.iters_used && li == 0) a.iters_used[b] = it + 1;
            }
        }
    }
    if (active && live && a.iters_used && li == 0) a.iters_used[b] = it;
    __syncthreads();
    if (!active) return;
    uint8_t *hd = a.hard ? a.hard + (size_t)b * N : nullptr;
    T *sd = a.soft ? (T *)a.soft + (size_t)b * N : nullptr;
    for (int i = li; i < N; i += lpc) {
        const T v = V[i];
        if (hd) hd[i] = v > (T)0;   // code/x86/CTools/CTools.cpp:370
        if (sd) sd[i] = v;
    }
}

}  // namespace

// layers: maximal runs of consecutive checks of one group sharing no variable
static void lds_plan(const ldpc_code *h, std::vector<int4> &layers, int &maxw)
{
    layers.clear();
    std::vector<int> stamp(h->n, -1);
    maxw = 0;
    for (int i = 0; i < h->m;) {
        const int g = h->check_group[i], d = h->check_deg[i];
        int j = i;
        const int lid = (int)layers.size();
        for (; j < h->m && h->check_group[j] == g; j++) {
            bool clash = false;
            for (int k = 0; k < d && !clash; k++) clash = stamp[h->edge_var[h->check_start[j] + k]] == lid;
            if (clash) break;
            for (int k = 0; k < d; k++) stamp[h->edge_var[h->check_start[j] + k]] = lid;
        }
        layers.push_back(make_int4(h->check_start[i], j - i, d, g > 0 ? 1 : 0));
        maxw = std::max(maxw, j - i);
        i = j;
    }
}

constexpr int kLdsSimds = 256 * 4;   // MI355X: 256 CUs x 4 SIMDs

static int lpc_log2_of(int maxw) { return maxw <= 8 ? 3 : maxw <= 16 ? 4 : maxw <= 32 ? 5 : 6; }

static size_t lds_bytes_of(const ldpc_code *h, int lpc_log2, size_t esz)
{
    return (size_t)(2 * h->e + 15) / 16 * 16 + ((size_t)64 >> lpc_log2) * ((size_t)h->n + (size_t)h->e) * esz;
}

extern "C" int ldpc_code_layer_info(const ldpc_code *h, int *n_layers, int *max_width, int *lds_i8, int *lds_f32)
{
    if (!h) return ldpc_set_error(LDPC_EINVAL, "NULL code");
    std::vector<int4> layers;
    int maxw = 0;
    lds_plan(h, layers, maxw);
    const bool idx16 = h->n <= 65535 && h->e > 0;
    if (n_layers) *n_layers = (int)layers.size();
    if (max_width) *max_width = maxw;
    if (lds_i8) *lds_i8 = idx16 && lds_bytes_of(h, lpc_log2_of(maxw), 1) <= kLdsMaxBytes;
    if (lds_f32) *lds_f32 = idx16 && lds_bytes_of(h, lpc_log2_of(maxw), 4) <= kLdsMaxBytes;
    return LDPC_OK;
}

int lds_upload(const ldpc_code *h, LdsCode *lc)
{
    *lc = LdsCode{};
    if (h->n > 65535 || h->e == 0) return LDPC_OK;
    std::vector<int4> layers;
    int maxw = 0;
    lds_plan(h, layers, maxw);
    // layer-major table: entry base + k * cnt + c = variable of edge k of check c
    std::vector<uint16_t> tab(h->e);
    for (const int4 &L : layers)
        for (int c = 0; c < L.y; c++)
            for (int k = 0; k < L.z; k++) tab[L.x + k * L.y + c] = (uint16_t)h->edge_var[L.x + c * L.z + k];
    const int lpc_log2 = lpc_log2_of(maxw);
    lc->nl = (int)layers.size();
    lc->max_width = maxw;
    lc->lpc_log2 = lpc_log2;
    lc->tab_bytes = (2 * h->e + 15) / 16 * 16;
    tab.resize(lc->tab_bytes / 2, 0);   // padded to whole 16-B chunks
    if (hipMalloc(&lc->d_tab, lc->tab_bytes) != hipSuccess ||
        hipMalloc(&lc->d_layers, sizeof(int4) * layers.size()) != hipSuccess) {
        lds_free(lc);
        return ldpc_set_error(LDPC_ENOMEM, "lds tables");
    }
    if (hipMemcpy(lc->d_tab, tab.data(), lc->tab_bytes, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(lc->d_layers, layers.data(), sizeof(int4) * layers.size(), hipMemcpyHostToDevice) != hipSuccess) {
        lds_free(lc);
        return ldpc_set_error(LDPC_EDEVICE, "lds table upload");
    }
    lc->valid = 1;
    return ldsep_upload(h, layers, lc);
}

void lds_free(LdsCode *lc)
{
    (void)hipFree(lc->d_tab);
    (void)hipFree(lc->d_layers);
    (void)hipFree(lc->d_ep_tab);
    *lc = LdsCode{};
}

size_t lds_bytes(const ldpc_code *h, const LdsCode &lc, bool is_float)
{
    return lds_bytes_of(h, lc.lpc_log2, is_float ? 4 : 1);
}

bool lds_applicable(const ldpc_code *h, const LdsCode &lc, bool is_float)
{
    return lc.valid && lds_bytes(h, lc, is_float) <= kLdsMaxBytes;
}

bool lds_preferred(const ldpc_code *h, const LdsCode &lc, bool is_float)
{
    // enough checks per layer to be worth a wave (QC codes: Z >= 8)
    return lds_applicable(h, lc, is_float) && h->m >= 8 * lc.nl;
}

int launch_lds(const LdsCode &lc, const ldpc_code *h, const void *llr, uint8_t *hard, void *soft, int batch,
               int iters, const DecodeLaunch &L, hipStream_t s)
{
    if (!lds_applicable(h, lc, L.is_float)) return -1;
    LdsArgs a{};
    a.llr = llr;
    a.hard = hard;
    a.soft = soft;
    a.tab = lc.d_tab;
    a.layers = lc.d_layers;
    a.nl = lc.nl;
    a.n = h->n;
    a.e = h->e;
    a.batch = batch;
    a.iters = iters;
    // lanes per codeword: at least the widest layer; more (down to one
    // codeword per wave, two lanes per check) while that still leaves two
    // waves per SIMD of the 256-CU chip -- the kernel is latency-bound, so
    // small batches go faster spread over more waves
    int lg = lc.lpc_log2;
    while (lg < 6 && (batch << lg) / 64 < 2 * kLdsSimds) lg++;
    const bool split = (1 << lg) >= 2 * lc.max_width;
    a.lpc_log2 = lg;
    a.algo = L.algo;
    a.param = L.param;
    a.var_min = L.var_min;
    a.msg_max = L.msg_max;
    a.early = L.early;
    a.beta = L.beta;
    a.iters_used = L.iters_used;
    a.tab_bytes = lc.tab_bytes;
    const int cpw = 64 >> lg;
    const size_t shm = lds_bytes_of(h, lg, L.is_float ? 4 : 1);
    dim3 grid((batch + cpw - 1) / cpw), block(64);
    if (L.is_float)
        hipLaunchKernelGGL((split ? lds_decode<float, true> : lds_decode<float, false>), grid, block, shm, s, a);
    else
        hipLaunchKernelGGL((split ? lds_decode<int8_t, true> : lds_decode<int8_t, false>), grid, block, shm, s, a);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
