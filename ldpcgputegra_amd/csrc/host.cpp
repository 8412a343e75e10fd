// host.cpp -- the C-ABI's host decoder (ldpc_ctx_create with device = -1):
// the drop-in on a machine without an MI355X (SURVEY.md §8(b) "device = -1";
// code/x86/CDecoder/template/CDecoder.h:28-40 is a host decoder too).
//
// Same layered schedule and int8 / float arithmetic as the GPU kernels and the
// reference (code/x86/CDecoder/OMS/CDecoder_OMS_fixed_SSE.cpp:172-546, NMS
// CDecoder_NMS_fixed_SSE.cpp:125-368), bit-exact for
// int8.  Written for the host's wide vector unit: 32 codewords per AVX2
// register (the reference's SSE decoder does 16), V[N][32] and msg[E][32]
// interleaved per block of 32 codewords (16 where only SSE4.1 is present),
// blocks spread over host threads (the SIMD check loop: host_simd.h, compiled per
// instruction set in host_avx2.cpp / host_sse4.cpp).  A portable loop over the lanes (the same operations, one byte at
// a time) runs where neither is available (LDPC_HOST_PORTABLE forces it).  The float path is scalar per codeword.
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#include "host.h"
#include "host_simd.h"

namespace {

constexpr int HB = 32;   // most codewords per block (one AVX2 register of int8)

// ---- portable lane ops (the reference's SSE semantics, one byte at a time)
inline int sat8(int x) { return x < -128 ? -128 : (x > 127 ? 127 : x); }
inline int abs8(int x) { return x == -128 ? -128 : (x < 0 ? -x : x); }
inline int as_i8(int x) { return (int)(int8_t)(uint8_t)x; }
inline int nms8(int mn, int f)   // packs_epi16((u16(min) * factor) >> 5)
{
    const int s = (int)(int16_t)(uint16_t)(((uint16_t)(uint8_t)mn * (uint16_t)f) >> 5);
    return s > 127 ? 127 : (s < -128 ? -128 : s);
}

// one check over the W lanes of a block, portable
template <bool ET>
void check_portable(int8_t *V, int8_t *msg, const uint32_t *ev, int d, bool later, const I8Params &p,
                    const uint8_t *live, int W)
{
    int c[64][HB], a[64][HB];
    for (int l = 0; l < W; l++) {
        int sign = 0, min1 = 127, min2 = 127;
        for (int j = 0; j < d; j++) {
            const int cj = std::max(sat8(V[(size_t)ev[j] * W + l] - msg[j * W + l]), p.var_min);
            const int aj = (p.algo == LDPC_ALGO_NMS || !later) ? std::min(abs8(cj), p.msg_max)
                                                               : abs8(std::min(cj, p.msg_max));
            sign ^= cj & 0x80;
            c[j][l] = cj;
            a[j][l] = aj;
            const int t = min1;
            min1 = std::min(aj, min1);
            min2 = std::min(min2, std::max(aj, t));
        }
        int cst1, cst2;
        if (p.algo == LDPC_ALGO_NMS) {
            cst1 = nms8(min2, p.param);
            cst2 = nms8(min1, p.param);
        } else {
            cst1 = std::min(as_i8(std::max((min2 & 0xFF) - (p.param & 0xFF), 0)), p.msg_max);
            cst2 = std::min(as_i8(std::max((min1 & 0xFF) - (p.param & 0xFF), 0)), p.msg_max);
        }
        sign ^= (d & 1) ? 0xC0 : 0x40;
        if (ET && !live[l]) continue;
        for (int j = 0; j < d; j++) {
            const int r = a[j][l] == min1 ? cst1 : cst2;
            const int sig = as_i8(sign ^ (c[j][l] & 0x80));   // never 0: bit 6 is set
            const int m = sig < 0 ? as_i8(-r) : r;
            msg[j * W + l] = (int8_t)m;
            V[(size_t)ev[j] * W + l] = (int8_t)std::max(sat8(c[j][l] + m), p.var_min);
        }
    }
}

// lanes whose hard decisions satisfy every check
void syndrome_ok(const ldpc_code *h, const int8_t *V, uint8_t *ok, int W)
{
    uint8_t bad[HB] = {0};
    for (int i = 0; i < h->m; i++) {
        const uint32_t *ev = &h->edge_var[h->check_start[i]];
        uint8_t par[HB] = {0};
        for (int j = 0; j < h->check_deg[i]; j++) {
            const int8_t *v = V + (size_t)ev[j] * W;
            for (int l = 0; l < W; l++) par[l] ^= v[l] > 0;
        }
        for (int l = 0; l < W; l++) bad[l] |= par[l];
    }
    for (int l = 0; l < W; l++) ok[l] = !bad[l];
}

struct Scratch {
    std::vector<int8_t> V, msg;   // V[N + 1][W] (64-B aligned), msg[E][W]
    int8_t *v = nullptr, *m = nullptr;
    void size(const ldpc_code *h, int W)
    {
        V.resize(((size_t)h->n + 2) * W + 64);
        msg.resize((size_t)h->e * W + 64);
        v = (int8_t *)(((uintptr_t)V.data() + 63) & ~(uintptr_t)63);
        m = (int8_t *)(((uintptr_t)msg.data() + 63) & ~(uintptr_t)63);
    }
};

// SIMD path of a block: 32-lane AVX2, 16-lane SSE4.1, or the portable loop
enum class Isa { avx2, sse4, portable };

// one block of up to W codewords (frame-major in / out)
void decode_block_i8(const ldpc_code *h, const int8_t *llr, uint8_t *hard, int nb, int iters, const I8Params &p,
                     Scratch &s, Isa isa, int W)
{
    const int n = h->n;
    s.size(h, W);
    for (int i = 0; i < n; i++)
        for (int l = 0; l < W; l++) s.v[(size_t)i * W + l] = l < nb ? llr[(size_t)l * n + i] : 0;
    std::memset(s.m, 0, (size_t)h->e * W);   // CDecoder_OMS_fixed_SSE.cpp:129-131
    alignas(32) uint8_t live[HB];
    for (int l = 0; l < HB; l++) live[l] = l < nb;
    for (int it = 0; it < iters; it++) {
        if (isa == Isa::avx2)
            host_checks_avx2(h, s.v, s.m, p, live);
        else if (isa == Isa::sse4)
            host_checks_sse4(h, s.v, s.m, p, live);
        else {
            size_t e0 = 0;
            for (int i = 0; i < h->m; i++) {
                const int d = h->check_deg[i];
                const uint32_t *ev = &h->edge_var[h->check_start[i]];
                p.early ? check_portable<true>(s.v, s.m + e0 * W, ev, d, h->check_group[i] > 0, p, live, W)
                        : check_portable<false>(s.v, s.m + e0 * W, ev, d, h->check_group[i] > 0, p, live, W);
                e0 += (size_t)d;
            }
        }
        if (p.early) {   // per codeword: stop after the first iteration whose hard decisions satisfy H
            uint8_t ok[HB];
            syndrome_ok(h, s.v, ok, W);
            bool any = false;
            for (int l = 0; l < W; l++) {
                if (ok[l]) live[l] = 0;
                any |= live[l] != 0;
            }
            if (!any) break;
        }
    }
    for (int l = 0; l < nb; l++)
        for (int i = 0; i < n; i++) hard[(size_t)l * n + i] = s.v[(size_t)i * W + l] > 0;   // CTools.cpp:370
}

// one codeword, float (the same schedule; SURVEY.md §8(a) float variant)
void decode_one_f32(const ldpc_code *h, const float *llr, uint8_t *hard, int iters, int algo, float beta, bool early,
                    std::vector<float> &V, std::vector<float> &msg)
{
    V.assign(llr, llr + h->n);
    msg.assign((size_t)h->e, 0.0f);
    float c[64], a[64];
    for (int it = 0; it < iters; it++) {
        size_t e0 = 0;
        for (int i = 0; i < h->m; i++) {
            const int d = h->check_deg[i];
            const uint32_t *ev = &h->edge_var[h->check_start[i]];
            float *mp = &msg[e0];
            int sign = d & 1;
            float min1 = __builtin_huge_valf(), min2 = min1;
            for (int j = 0; j < d; j++) {
                c[j] = V[ev[j]] - mp[j];
                a[j] = std::fabs(c[j]);
                sign ^= c[j] < 0.0f;
                const float t = min1;
                min1 = std::fmin(a[j], min1);
                min2 = std::fmin(min2, std::fmax(a[j], t));
            }
            const float cst1 = algo == LDPC_ALGO_NMS ? min2 * beta : std::fmax(min2 - beta, 0.0f);
            const float cst2 = algo == LDPC_ALGO_NMS ? min1 * beta : std::fmax(min1 - beta, 0.0f);
            for (int j = 0; j < d; j++) {
                const float r = a[j] == min1 ? cst1 : cst2;
                const float m = (sign ^ (c[j] < 0.0f)) ? -r : r;
                mp[j] = m;
                V[ev[j]] = c[j] + m;
            }
            e0 += (size_t)d;
        }
        if (early) {
            bool ok = true;
            for (int i = 0; i < h->m && ok; i++) {
                int par = 0;
                for (int j = 0; j < h->check_deg[i]; j++) par ^= V[h->edge_var[h->check_start[i] + j]] > 0.0f;
                ok = par == 0;
            }
            if (ok) break;
        }
    }
    for (int i = 0; i < h->n; i++) hard[i] = V[i] > 0.0f;
}

int host_threads_for(int units)
{
    const char *e = getenv("LDPC_HOST_THREADS");
    int t = (e && *e) ? atoi(e) : (int)std::thread::hardware_concurrency();
    return std::max(1, std::min(t, units));
}

// run f(unit) for units 0 .. n-1 on the host threads (each thread its own scratch)
template <typename F>
void parallel_units(int n, F f)
{
    const int t = host_threads_for(n);
    if (t == 1) {
        for (int u = 0; u < n; u++) f(u, 0);
        return;
    }
    std::vector<std::thread> th;
    for (int k = 0; k < t; k++)
        th.emplace_back([&, k]() {
            for (int u = k; u < n; u += t) f(u, k);
        });
    for (auto &x : th) x.join();
}

}  // namespace

bool host_has_avx2() { return __builtin_cpu_supports("avx2"); }

int host_decode_i8(const ldpc_code *h, const int8_t *llr, uint8_t *hard, int batch, int n_iter, const ldpc_params *p)
{
    const I8Params ip{p->algo == LDPC_ALGO_NMS ? LDPC_ALGO_NMS : LDPC_ALGO_OMS,
                      p->algo == LDPC_ALGO_NMS ? p->factor : (p->algo == LDPC_ALGO_MS ? 0 : p->offset), p->var_min,
                      p->msg_max, p->early_term};
    // lanes per block: 32 (AVX2); LDPC_HOST_LANES=16 forces the SSE4.1 width
    // (measured slower even on DVB-S2, whose 32-lane working set is 10.7 MB:
    // 0.39 vs 0.31 ns per edge and codeword on one thread)
    const int forced = getenv("LDPC_HOST_LANES") ? atoi(getenv("LDPC_HOST_LANES")) : 0;
    const bool avx2 = host_has_avx2();
    int W = forced == 16 ? 16 : 32;
    Isa isa = getenv("LDPC_HOST_PORTABLE") ? Isa::portable : W == 32 ? (avx2 ? Isa::avx2 : Isa::sse4) : Isa::sse4;
    if (isa == Isa::sse4) W = 16;
    if (isa == Isa::sse4 && !__builtin_cpu_supports("sse4.1")) isa = Isa::portable;
    const int nblk = (batch + W - 1) / W;
    std::vector<Scratch> sc((size_t)host_threads_for(std::max(nblk, 1)));
    parallel_units(nblk, [&](int b, int k) {
        const int nb = std::min(W, batch - b * W);
        decode_block_i8(h, llr + (size_t)b * W * h->n, hard + (size_t)b * W * h->n, nb, n_iter, ip, sc[k], isa, W);
    });
    return LDPC_OK;
}

int host_decode_f32(const ldpc_code *h, const float *llr, uint8_t *hard, int batch, int n_iter, const ldpc_params *p)
{
    const int algo = p->algo == LDPC_ALGO_NMS ? LDPC_ALGO_NMS : LDPC_ALGO_OMS;
    const float beta = p->algo == LDPC_ALGO_MS ? 0.0f : p->beta;
    const int nt = host_threads_for(std::max(batch, 1));
    std::vector<std::vector<float>> V((size_t)nt), M((size_t)nt);
    parallel_units(batch, [&](int b, int k) {
        decode_one_f32(h, llr + (size_t)b * h->n, hard + (size_t)b * h->n, n_iter, algo, beta, p->early_term != 0,
                       V[k], M[k]);
    });
    return LDPC_OK;
}
