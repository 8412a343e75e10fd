// stairf.hip -- float layered min-sum for staircase (DVB-S2 IRA) codes
// (kernel 11, the automatic float choice for them).
//
// The layered float decode of generic.hip (check_f32, which restates
// code/x86/CDecoder/OMS/CDecoder_OMS_fixed_SSE.cpp:122-574 and
// code/x86/CDecoder/NMS/CDecoder_NMS_fixed_SSE.cpp:125-368 in float) walks
// every check of the schedule serially, one HBM round trip per check.  This
// kernel splits each check the way the int8 staircase kernels do:
//
// * a wave holds 64 / S codewords x S consecutive checks (lane = S *
//   codeword + slot, slot = check within the group of S; S = 2, 4, 8 or 16
//   by batch size, stairf_width).  The info edges of the S
//   checks (no two checks closer than the code's hazard distance share an
//   info node) and the o edge (the parity node the next check reads; its V
//   is last iteration's) are independent: each lane reduces its check's info
//   edges and o edge in parallel.
// * the only serial part is the staircase chain: the x edge of check c is the
//   o edge of check c - 1, written by it one check earlier.  S chain steps
//   per group pass the intermediate parity value from slot to slot with one
//   DPP move each (step 0: row_shl:S-1, slot 0 gets slot S-1 of the previous
//   group, the tail check of the previous iteration for check 0; steps 1..:
//   row_shr:1), each step 6 dependent VALU.
// * every exclusive minimum is formed directly (min over the other edges),
//   which is exactly the value the reference's min1 / min2 select gives, so
//   the float results are bit-identical to the serial decode.
// * V stays in HBM (V[node][stride], 64 / S codewords = one piece per node;
//   waves sharing a 128-B line of V are placed on one XCD); messages in the
//   kernel's own layout [wave][group][edge][slot][cw], one 256-B run per
//   instruction.  The loads of group g + P (and the node ids of group g + 2P)
//   are issued while group g is decoded: P groups of HBM latency hidden, legal
//   because the code's hazard distance is >= S P checks.
//
// Design reference: code/gpu_fixed/decoder_oms_v2/cuda/CUDA_OMS_SIMD_v2.cu:28-195
// (per-check contributions shared by the lanes of a check); layout and
// schedule are this kernel's own.
#include <algorithm>
#include <cstdlib>
#include <vector>

#include "stairf.h"

namespace {

struct StairfArgs {
    float *V;
    float *msg;
    const uint32_t *tab;
    int G, T, stride, iters, x0;
    float beta;
    const uint8_t *live;   // early termination: codewords still decoding (stores of the others are off)
};

template <int X, int S>
struct SF {
    static constexpr int W = (X + 3) / 2;   // u32 words of packed u16 node ids per check
    static constexpr int E = X + 2;         // messages per check
    // groups in flight: ring registers 2P * W + P * (2X + 3) stay <= ~180, and
    // S * P <= 48 checks (every DVB-S2 code's hazard distance is >= 51)
    static constexpr int PR = X <= 5 ? 8 : X <= 8 ? 6 : X <= 12 ? 4 : 2;
    static constexpr int P = PR < 48 / S ? PR : 48 / S;
};

constexpr bool x_supported(int X) { return X == 5 || X == 8 || X == 12 || X == 20 || X == 25 || X == 28; }

template <int S>
int p_of(int X)
{
    switch (X) {
    case 5: return SF<5, S>::P;
    case 8: return SF<8, S>::P;
    case 12: return SF<12, S>::P;
    case 20: return SF<20, S>::P;
    case 25: return SF<25, S>::P;
    case 28: return SF<28, S>::P;
    }
    return 0;
}

int p_of_s(int X, int S) { return S == 2 ? p_of<2>(X) : S == 4 ? p_of<4>(X) : S == 8 ? p_of<8>(X) : p_of<16>(X); }
int s_index(int S) { return S == 2 ? 3 : S == 4 ? 0 : S == 8 ? 1 : 2; }

// A: 0 OMS, 1 NMS, 2 OMS with beta = 0 (plain min-sum)
template <int A>
LDPC_DEV float cst(float x, float beta)
{
    // generic.hip check_f32: NMS min * beta, OMS max(min - beta, 0); with
    // beta = 0 that is x itself (x = |c| >= +0: x - 0 = x, max(x, 0) = x)
    if constexpr (A == 1)
        return x * beta;
    else if constexpr (A == 2)
        return x;
    else
        return fmaxf(x - beta, 0.0f);
}

// chain step `step`: slot `step` reads slot step - 1 of its codeword (row_shr:1),
// slot 0 reads slot S - 1 (row_shl:S-1; the previous group's last check)
template <int S>
LDPC_DEV float rot_chain(float t, int step)
{
    // bound_ctrl: lanes whose source is outside the row read 0 (none of them is
    // the step's valid slot), which lets the move fold into the subtract that
    // consumes it (v_sub_f32_dpp): one dependent instruction less per step
    const int v = __float_as_int(t);
    return __int_as_float(step == 0 ? __builtin_amdgcn_update_dpp(0, v, 0x100 + S - 1, 0xF, 0xF, true)
                                    : __builtin_amdgcn_update_dpp(0, v, 0x111, 0xF, 0xF, true));
}

template <int X, int A, int S, bool ET>
__global__ void __launch_bounds__(64) stairf_decode(StairfArgs a)
{
    constexpr int W = SF<X, S>::W, E = SF<X, S>::E, P = SF<X, S>::P, C = 64 / S;
    const int lane = threadIdx.x, slot = lane % S, cwl = lane / S;
    // XCD-aware: the 128 / (4 C) waves whose V pieces share a 128-B line run on one XCD
    const int nb = gridDim.x;
    const int wv = (nb % 8 == 0) ? (int)(blockIdx.x % 8) * (nb / 8) + (int)(blockIdx.x / 8) : (int)blockIdx.x;
    // V: wave base (uniform) + u32 byte offset node * stride * 4 + lane (the
    // host keeps (n + 1) * stride * 4 < 2^32); messages: wave base + group
    // (uniform) + lane + edge * 256 (immediate)
    const uint32_t pitch = (uint32_t)a.stride * 4, lv = (uint32_t)cwl * 4, lm = (uint32_t)(slot * C + cwl) * 4;
    char *Vw = (char *)(a.V + (size_t)wv * C);
    char *Mw = (char *)(a.msg + (size_t)wv * a.G * E * 64);
    const uint32_t *tl = a.tab + slot;
    // early termination: a converged codeword's lanes keep computing (their
    // loads are shared with live codewords' lanes) but store nothing; a wave
    // whose codewords have all converged leaves at once
    const bool alive = !ET || a.live[(size_t)wv * C + cwl];
    if (ET && !__any(alive)) return;
    const int G = a.G;
    const long total = (long)a.iters * G;
    const float INF = __builtin_huge_valf();

    uint32_t id[2 * P][W];
    float vv[P][X + 1];   // info V, o V
    float mm[P][E];       // info messages, x message, o message

    auto node = [&](const uint32_t (&ids)[W], int j) -> uint32_t {
        const uint32_t w = ids[j >> 1];
        return (j & 1) ? (w >> 16) : (w & 0xFFFFu);
    };
    auto load_ids = [&](uint32_t (&ids)[W], int gg) {
#pragma unroll
        for (int i = 0; i < W; i++) ids[i] = tl[((size_t)gg * W + i) * S];
    };
    auto vref = [&](uint32_t nd) -> float & { return *(float *)(Vw + (__umul24(nd, pitch) + lv)); };
    auto load_vm = [&](float (&v)[X + 1], float (&m)[E], const uint32_t (&ids)[W], int gg) {
#pragma unroll
        for (int j = 0; j < X; j++) v[j] = vref(node(ids, j));
        v[X] = vref(node(ids, X + 1));
        const char *mg = Mw + (size_t)gg * E * 256 + lm;
#pragma unroll
        for (int j = 0; j < E; j++) m[j] = *(const float *)(mg + j * 256);
    };

    float t = vref((uint32_t)a.x0);   // check 0's first chain input: its x node's LLR
    auto process = [&](const float (&v)[X + 1], const float (&m)[E], const uint32_t (&ids)[W], int gg) {
        const int c = gg * S + slot;
        const bool hasx = c != a.T;                  // the tail check has no x edge
        const bool sto = c >= a.T - 1;               // o edge not read by the next check (or wraps): store it
        float cv[X], av[X];
        float m1 = INF, m2 = INF;
        bool sI = ((X + 1 + (hasx ? 1 : 0)) & 1) != 0;   // check_f32: sign starts at D & 1
#pragma unroll
        for (int j = 0; j < X; j++) {
            cv[j] = v[j] - m[j];
            av[j] = fabsf(cv[j]);
            sI ^= (cv[j] < 0.0f);
            const float tt = m1;
            m1 = fminf(av[j], m1);
            m2 = fminf(m2, fmaxf(av[j], tt));
        }
        const float co = v[X] - m[X + 1], ao = fabsf(co);
        const bool no = co < 0.0f;
        const float mx = hasx ? m[X] : -INF;         // tail: |c_x| = +inf, sign +
        // the chain: S steps, slot s valid at step s
        float cx = 0.0f;
#pragma unroll
        for (int s = 0; s < S; s++) {
            const float cs = rot_chain<S>(t, s) - mx;
            if (slot == s) cx = cs;
            const float r = cst<A>(fminf(m1, fabsf(cs)), a.beta);
            t = co + ((sI ^ (cs < 0.0f)) ? -r : r);
        }
        const float ax = fabsf(cx);
        const bool nx = cx < 0.0f;
        const float ro = cst<A>(fminf(m1, ax), a.beta);
        const float mo = (sI ^ nx) ? -ro : ro;
        const float rx = cst<A>(fminf(m1, ao), a.beta);
        const float mxn = (sI ^ no) ? -rx : rx;
        const float mxo = fminf(ax, ao);
        const bool sx = sI ^ nx ^ no;
        char *mg = Mw + (size_t)gg * E * 256 + lm;
        if (alive) {
#pragma unroll
            for (int j = 0; j < X; j++) {
                const float r = cst<A>(fminf(av[j] == m1 ? m2 : m1, mxo), a.beta);
                const float mj = (sx ^ (cv[j] < 0.0f)) ? -r : r;
                *(float *)(mg + j * 256) = mj;
                vref(node(ids, j)) = cv[j] + mj;
            }
            *(float *)(mg + X * 256) = mxn;
            *(float *)(mg + (X + 1) * 256) = mo;
            if (hasx) vref(node(ids, X)) = cx + mxn;
            if (sto) vref(node(ids, X + 1)) = co + mo;
        }
    };

    // prologue: ids of groups 0 .. 2P-1, data of groups 0 .. P-1
    int g_p = 0, g_v = P % G, g_i = (2 * P) % G;   // group (mod G) being decoded / loaded / id-loaded
#pragma unroll
    for (int s = 0; s < 2 * P; s++) load_ids(id[s], s % G);
#pragma unroll
    for (int s = 0; s < P; s++) load_vm(vv[s], mm[s], id[s], s % G);
    for (long base = 0; base < total; base += 2 * P) {
#pragma unroll
        for (int s = 0; s < 2 * P; s++) {
            const int k = s % P;
            if (base + s < total) process(vv[k], mm[k], id[s], g_p);
            load_vm(vv[k], mm[k], id[(s + P) % (2 * P)], g_v);
            load_ids(id[s], g_i);
            g_p = g_p + 1 == G ? 0 : g_p + 1;
            g_v = g_v + 1 == G ? 0 : g_v + 1;
            g_i = g_i + 1 == G ? 0 : g_i + 1;
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the prefetches past the end
}

template <int X, int S, bool ET>
int launch_xse(const StairfArgs &a, int blocks, int algo, hipStream_t s)
{
    if (algo == 1)
        hipLaunchKernelGGL((stairf_decode<X, 1, S, ET>), dim3(blocks), dim3(64), 0, s, a);
    else if (algo == 2)
        hipLaunchKernelGGL((stairf_decode<X, 2, S, ET>), dim3(blocks), dim3(64), 0, s, a);
    else
        hipLaunchKernelGGL((stairf_decode<X, 0, S, ET>), dim3(blocks), dim3(64), 0, s, a);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

template <int X, int S>
int launch_xs(const StairfArgs &a, int blocks, int algo, hipStream_t s)
{
    return a.live ? launch_xse<X, S, true>(a, blocks, algo, s) : launch_xse<X, S, false>(a, blocks, algo, s);
}

// early termination (oracle_decode_f32: stop a codeword after the first
// iteration whose hard decisions V > 0 satisfy every check): after each
// one-iteration launch, every check of every live codeword is tested (one
// lane per codeword, a chunk of checks per workgroup, the check's nodes
// wave-uniform), any failing check marks the codeword bad; then live
// codewords without a bad mark stop with that iteration count
__global__ void __launch_bounds__(64) stairf_et_init_k(uint8_t *live, uint32_t *bad, int32_t *iters_used, int batch,
                                                       int stride, int iters)
{
    const int b = blockIdx.x * 64 + threadIdx.x;
    if (b >= stride) return;
    live[b] = b < batch;
    bad[b] = 0;
    if (b < batch) iters_used[b] = iters;
}

__global__ void __launch_bounds__(64) stairf_syndrome_k(const float *V, const uint32_t *ev, const uint8_t *live,
                                                        uint32_t *bad, int m, int d0, int chunk, int stride)
{
    const int b = blockIdx.x * 64 + threadIdx.x;
    const bool on = live[b] != 0;
    if (!__any(on)) return;
    const int c0 = blockIdx.y * chunk, c1 = min(m, c0 + chunk);
    const float *Vb = V + b;
    int fail = 0;
    for (int c = c0; c < c1; c++) {
        const uint32_t *e = ev + (size_t)c * d0;   // layered order: every check d0 edges apart, the tail last
        const int d = c == m - 1 ? d0 - 1 : d0;
        int par = 0;
        for (int j = 0; j < d; j++) par ^= Vb[(size_t)e[j] * stride] > 0.0f;
        fail |= par;
    }
    if (on && fail) bad[b] = 1;
}

__global__ void __launch_bounds__(64) stairf_et_step_k(uint8_t *live, uint32_t *bad, int32_t *iters_used, int batch,
                                                       int it)
{
    const int b = blockIdx.x * 64 + threadIdx.x;
    if (b >= batch) return;
    if (live[b] && !bad[b]) {
        live[b] = 0;
        iters_used[b] = it;
    }
    bad[b] = 0;
}

template <int X>
int launch_x(const StairfArgs &a, int S, int blocks, int algo, hipStream_t s)
{
    return S == 2 ? launch_xs<X, 2>(a, blocks, algo, s)
         : S == 4 ? launch_xs<X, 4>(a, blocks, algo, s)
         : S == 8 ? launch_xs<X, 8>(a, blocks, algo, s)
                  : launch_xs<X, 16>(a, blocks, algo, s);
}

}  // namespace

int stairf_upload(const ldpc_code *h, StairfCode *sc)
{
    *sc = StairfCode{};
    if (!h->staircase || h->n_groups != 2 || h->group_cnt[1] != 1) return LDPC_OK;
    const int D0 = h->group_deg[0], X = D0 - 2, M = h->m, T = M - 1;
    if (h->group_deg[1] != D0 - 1 || !x_supported(X) || M % 4 || M < 32 || h->n > 65536) return LDPC_OK;
    auto ev = [&](int c, int j) { return h->edge_var[h->check_start[c] + j]; };
    // staircase: x edge (slot X) of check c is the o edge (slot X + 1) of
    // check c - 1; check 0's x edge is the tail's parity edge (its slot X)
    for (int c = 1; c < T; c++)
        if (ev(c, X) != ev(c - 1, X + 1)) return LDPC_OK;
    if (ev(0, X) != ev(T, X) || ev(T - 1, X + 1) == ev(T, X)) return LDPC_OK;
    std::vector<char> par(h->n, 0);
    for (int c = 0; c < T; c++) par[ev(c, X)] = par[ev(c, X + 1)] = 1;
    for (int c = 0; c < M; c++)
        for (int j = 0; j < X; j++)
            if (par[ev(c, j)]) return LDPC_OK;
    const int W = (X + 3) / 2;
    for (int S : {2, 4, 8, 16}) {   // one table per group width the code allows
        if (M % S || h->min_hazard < S * p_of_s(X, S)) continue;
        const int G = M / S;
        std::vector<uint32_t> tab((size_t)G * W * S, 0);
        for (int c = 0; c < M; c++) {
            uint32_t ids[32] = {0};
            for (int j = 0; j < X; j++) ids[j] = ev(c, j);
            ids[X] = c < T ? ev(c, X) : 0;                      // tail: no x edge (never stored)
            ids[X + 1] = c < T ? ev(c, X + 1) : ev(T, X);       // tail: its parity edge
            for (int i = 0; i < W; i++)
                tab[((size_t)(c / S) * W + i) * S + c % S] = ids[2 * i] | (ids[2 * i + 1] << 16);
        }
        uint32_t *&d = sc->d_tab[s_index(S)];
        if (hipMalloc(&d, tab.size() * 4) != hipSuccess) {
            d = nullptr;
            stairf_free(sc);
            return ldpc_set_error(LDPC_ENOMEM, "stairf table");
        }
        if (hipMemcpy(d, tab.data(), tab.size() * 4, hipMemcpyHostToDevice) != hipSuccess) {
            stairf_free(sc);
            return ldpc_set_error(LDPC_EDEVICE, "stairf table upload");
        }
    }
    sc->X = X;
    sc->m = M;
    sc->x0 = (int)ev(0, X);
    sc->valid = sc->d_tab[0] || sc->d_tab[1] || sc->d_tab[2] || sc->d_tab[3];
    return LDPC_OK;
}

// group width of a launch: LDPC_STAIRF_S (2 / 4 / 8 / 16) if set and the code has
// that table; else by batch: the widest pieces of V (S = 2: 32 codewords =
// whole 128-B lines) once there are enough waves to fill the chip, narrower
// groups (more waves per codeword) below that.  Measured (DVB-S2 r1/2, 20 it,
// plain min-sum, profiles/r04t_float_long.jsonl), S = 2 / 4 / 8 / 16:
//   batch  1024: 131.4 / 73.3 / 45.9 / 40.2 ms
//   batch  2048: 132.8 / 74.9 / 53.7 / 67.1
//   batch  4096: 137.5 / 80.1 / 117.8 / 179.9
//   batch 16384: 234.3 / 356.1 / 507.2 / 830.3 (S = 2: 4.73 TB/s of HBM traffic)
int stairf_width(const StairfCode &sc, int stride)
{
    const char *e = getenv("LDPC_STAIRF_S");
    const int want = (e && *e) ? atoi(e) : stride >= 8192 ? 2 : stride >= 4096 ? 4 : stride >= 2048 ? 8 : 16;
    for (int S : {want, 8, 4, 16})
        if ((S == 2 || S == 4 || S == 8 || S == 16) && sc.d_tab[s_index(S)]) return S;
    return 0;
}

void stairf_free(StairfCode *sc)
{
    for (uint32_t *d : sc->d_tab)
        if (d) (void)hipFree(d);
    *sc = StairfCode{};
}

bool stairf_stride_ok(const StairfCode &sc, int n, int stride)
{
    return sc.valid && stride % 64 == 0 && ((size_t)n + 1) * stride * 4 < (1ull << 32);
}

size_t stairf_msg_bytes(const StairfCode &sc, int stride)
{
    return (size_t)stride * sc.m * (sc.X + 2) * sizeof(float);
}

int launch_stairf(const DecodeLaunch &L, const StairfCode &sc, hipStream_t s)
{
    if (!stairf_stride_ok(sc, L.n, L.stride) || L.vpitch != L.stride) return -1;
    if (L.early && (!L.live || !L.bad || !L.iters_used || !L.d_edge_var)) return -1;
    const int S = stairf_width(sc, L.stride);
    if (!S) return -1;
    StairfArgs a;
    a.V = (float *)L.V;
    a.msg = (float *)L.msg;
    a.tab = sc.d_tab[s_index(S)];
    a.G = sc.m / S;
    a.T = sc.m - 1;
    a.stride = L.stride;
    a.iters = L.iters;
    a.x0 = sc.x0;
    a.beta = L.beta;
    a.live = nullptr;
    const int algo = L.algo == 1 ? 1 : L.beta == 0.0f ? 2 : 0;
    const int blocks = L.stride / (64 / S);
    auto run = [&]() {
        switch (sc.X) {
        case 5: return launch_x<5>(a, S, blocks, algo, s);
        case 8: return launch_x<8>(a, S, blocks, algo, s);
        case 12: return launch_x<12>(a, S, blocks, algo, s);
        case 20: return launch_x<20>(a, S, blocks, algo, s);
        case 25: return launch_x<25>(a, S, blocks, algo, s);
        case 28: return launch_x<28>(a, S, blocks, algo, s);
        }
        return -1;
    };
    if (!L.early) return L.iters <= 0 ? 0 : run();
    // early termination: one launch per iteration, then the syndrome
    const int cb = L.stride / 64;
    hipLaunchKernelGGL(stairf_et_init_k, dim3(cb), dim3(64), 0, s, L.live, L.bad, L.iters_used, L.batch, L.stride,
                       L.iters);
    if (hipGetLastError() != hipSuccess) return -1;
    const int chunks = std::max(1, std::min(sc.m, 4096 / cb)), chunk = (sc.m + chunks - 1) / chunks;
    a.iters = 1;
    a.live = L.live;
    for (int it = 1; it <= L.iters; it++) {
        if (run()) return -1;
        hipLaunchKernelGGL(stairf_syndrome_k, dim3(cb, (sc.m + chunk - 1) / chunk), dim3(64), 0, s, (const float *)L.V,
                           L.d_edge_var, L.live, L.bad, sc.m, sc.X + 2, chunk, L.stride);
        hipLaunchKernelGGL(stairf_et_step_k, dim3(cb), dim3(64), 0, s, L.live, L.bad, L.iters_used, L.batch, it);
        if (hipGetLastError() != hipSuccess) return -1;
    }
    return 0;
}
