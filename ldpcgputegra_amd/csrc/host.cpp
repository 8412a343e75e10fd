// host.cpp -- the C-ABI's host decoder (ldpc_ctx_create with device = -1):
// the drop-in on a machine without an MI355X (SURVEY.md §8(b) "device = -1";
// code/x86/CDecoder/template/CDecoder.h:28-40 is a host decoder too).
//
// Same layered schedule and int8 / float arithmetic as the GPU kernels and the
// reference (code/x86/CDecoder/OMS/CDecoder_OMS_fixed_SSE.cpp:172-546, NMS
// CDecoder_NMS_fixed_SSE.cpp:125-368), bit-exact for
// int8.  Written for the host's wide vector unit: 32 codewords per AVX2
// register (the reference's SSE decoder does 16), V[N][32] and msg[E][32]
// interleaved per block of 32 codewords, blocks spread over host threads.  A
// portable loop over the 32 lanes (the same operations, one byte at a time)
// runs where AVX2 is absent.  The float path is scalar per codeword.
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#include <immintrin.h>

#include "host.h"

namespace {

constexpr int HB = 32;   // codewords per block (one AVX2 register of int8)

struct I8Params {
    int algo, param, var_min, msg_max, early;
};

// ---- portable lane ops (the reference's SSE semantics, one byte at a time)
inline int sat8(int x) { return x < -128 ? -128 : (x > 127 ? 127 : x); }
inline int abs8(int x) { return x == -128 ? -128 : (x < 0 ? -x : x); }
inline int as_i8(int x) { return (int)(int8_t)(uint8_t)x; }
inline int nms8(int mn, int f)   // packs_epi16((u16(min) * factor) >> 5)
{
    const int s = (int)(int16_t)(uint16_t)(((uint16_t)(uint8_t)mn * (uint16_t)f) >> 5);
    return s > 127 ? 127 : (s < -128 ? -128 : s);
}

// one check over the 32 lanes of a block, portable
template <bool ET>
void check_portable(int8_t *V, int8_t *msg, const uint32_t *ev, int d, bool later, const I8Params &p,
                    const uint8_t *live)
{
    int c[64][HB], a[64][HB];
    for (int l = 0; l < HB; l++) {
        int sign = 0, min1 = 127, min2 = 127;
        for (int j = 0; j < d; j++) {
            const int cj = std::max(sat8(V[(size_t)ev[j] * HB + l] - msg[j * HB + l]), p.var_min);
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
            msg[j * HB + l] = (int8_t)m;
            V[(size_t)ev[j] * HB + l] = (int8_t)std::max(sat8(c[j][l] + m), p.var_min);
        }
    }
}

// NMS constants: (u16(min) * f) >> 5, signed-saturated to int8 (unpack / pack
// stay inside each 128-bit lane, so the byte order is kept)
__attribute__((target("avx2"))) inline __m256i nms_avx2(__m256i mn, __m256i f)
{
    const __m256i z = _mm256_setzero_si256();
    const __m256i lo = _mm256_srli_epi16(_mm256_mullo_epi16(_mm256_unpacklo_epi8(mn, z), f), 5);
    const __m256i hi = _mm256_srli_epi16(_mm256_mullo_epi16(_mm256_unpackhi_epi8(mn, z), f), 5);
    return _mm256_packs_epi16(lo, hi);
}

// the same check on AVX2, 32 lanes per instruction
template <bool ET>
__attribute__((target("avx2"))) void check_avx2(int8_t *V, int8_t *msg, const uint32_t *ev, int d, bool later,
                                                const I8Params &p, const uint8_t *live)
{
    const __m256i vmin = _mm256_set1_epi8((char)p.var_min), mm = _mm256_set1_epi8((char)p.msg_max);
    const __m256i s80 = _mm256_set1_epi8((char)0x80);
    const bool nms = p.algo == LDPC_ALGO_NMS;
    __m256i c[64], a[64];
    __m256i sign = _mm256_setzero_si256(), min1 = _mm256_set1_epi8(127), min2 = min1;
    for (int j = 0; j < d; j++) {
        const __m256i v = _mm256_load_si256((const __m256i *)(V + (size_t)ev[j] * HB));
        const __m256i cj = _mm256_max_epi8(_mm256_subs_epi8(v, _mm256_load_si256((const __m256i *)(msg + j * HB))), vmin);
        const __m256i aj = (nms || !later) ? _mm256_min_epi8(_mm256_abs_epi8(cj), mm)
                                           : _mm256_abs_epi8(_mm256_min_epi8(cj, mm));
        sign = _mm256_xor_si256(sign, _mm256_and_si256(cj, s80));
        c[j] = cj;
        a[j] = aj;
        min2 = _mm256_min_epi8(min2, _mm256_max_epi8(aj, min1));
        min1 = _mm256_min_epi8(min1, aj);
    }
    __m256i cst1, cst2;
    if (nms) {
        const __m256i f = _mm256_set1_epi16((short)p.param);
        cst1 = nms_avx2(min2, f);
        cst2 = nms_avx2(min1, f);
    } else {
        const __m256i off = _mm256_set1_epi8((char)p.param);
        cst1 = _mm256_min_epi8(_mm256_subs_epu8(min2, off), mm);
        cst2 = _mm256_min_epi8(_mm256_subs_epu8(min1, off), mm);
    }
    sign = _mm256_xor_si256(sign, _mm256_set1_epi8((char)((d & 1) ? 0xC0 : 0x40)));
    const __m256i keep = ET ? _mm256_cmpeq_epi8(_mm256_load_si256((const __m256i *)live), _mm256_setzero_si256())
                            : _mm256_setzero_si256();
    for (int j = 0; j < d; j++) {
        const __m256i r = _mm256_blendv_epi8(cst2, cst1, _mm256_cmpeq_epi8(a[j], min1));
        const __m256i m = _mm256_sign_epi8(r, _mm256_xor_si256(sign, _mm256_and_si256(c[j], s80)));
        __m256i nv = _mm256_max_epi8(_mm256_adds_epi8(c[j], m), vmin);
        int8_t *vp = V + (size_t)ev[j] * HB;
        if (ET) nv = _mm256_blendv_epi8(nv, _mm256_load_si256((const __m256i *)vp), keep);   // converged: frozen
        _mm256_store_si256((__m256i *)(msg + j * HB), m);
        _mm256_store_si256((__m256i *)vp, nv);
    }
}

// lanes whose hard decisions satisfy every check
void syndrome_ok(const ldpc_code *h, const int8_t *V, uint8_t *ok)
{
    uint8_t bad[HB] = {0};
    for (int i = 0; i < h->m; i++) {
        const uint32_t *ev = &h->edge_var[h->check_start[i]];
        uint8_t par[HB] = {0};
        for (int j = 0; j < h->check_deg[i]; j++) {
            const int8_t *v = V + (size_t)ev[j] * HB;
            for (int l = 0; l < HB; l++) par[l] ^= v[l] > 0;
        }
        for (int l = 0; l < HB; l++) bad[l] |= par[l];
    }
    for (int l = 0; l < HB; l++) ok[l] = !bad[l];
}

struct Scratch {
    std::vector<int8_t> V, msg;   // V[N + 1][32] (64-B aligned rows), msg[E][32]
    int8_t *v = nullptr, *m = nullptr;
    void size(const ldpc_code *h)
    {
        V.resize(((size_t)h->n + 2) * HB + 64);
        msg.resize((size_t)h->e * HB + 64);
        v = (int8_t *)(((uintptr_t)V.data() + 63) & ~(uintptr_t)63);
        m = (int8_t *)(((uintptr_t)msg.data() + 63) & ~(uintptr_t)63);
    }
};

// one block of up to 32 codewords (frame-major in / out)
void decode_block_i8(const ldpc_code *h, const int8_t *llr, uint8_t *hard, int nb, int iters, const I8Params &p,
                     Scratch &s, bool avx2)
{
    const int n = h->n;
    s.size(h);
    for (int i = 0; i < n; i++)
        for (int l = 0; l < HB; l++) s.v[(size_t)i * HB + l] = l < nb ? llr[(size_t)l * n + i] : 0;
    std::memset(s.m, 0, (size_t)h->e * HB);   // CDecoder_OMS_fixed_SSE.cpp:129-131
    alignas(32) uint8_t live[HB];
    for (int l = 0; l < HB; l++) live[l] = l < nb;
    for (int it = 0; it < iters; it++) {
        size_t e0 = 0;
        for (int i = 0; i < h->m; i++) {
            const int d = h->check_deg[i];
            const bool later = h->check_group[i] > 0;
            const uint32_t *ev = &h->edge_var[h->check_start[i]];
            int8_t *mp = s.m + e0 * HB;
            if (avx2)
                p.early ? check_avx2<true>(s.v, mp, ev, d, later, p, live) : check_avx2<false>(s.v, mp, ev, d, later, p, live);
            else
                p.early ? check_portable<true>(s.v, mp, ev, d, later, p, live)
                        : check_portable<false>(s.v, mp, ev, d, later, p, live);
            e0 += (size_t)d;
        }
        if (p.early) {   // per codeword: stop after the first iteration whose hard decisions satisfy H
            uint8_t ok[HB];
            syndrome_ok(h, s.v, ok);
            bool any = false;
            for (int l = 0; l < HB; l++) {
                if (ok[l]) live[l] = 0;
                any |= live[l] != 0;
            }
            if (!any) break;
        }
    }
    for (int l = 0; l < nb; l++)
        for (int i = 0; i < n; i++) hard[(size_t)l * n + i] = s.v[(size_t)i * HB + l] > 0;   // CTools.cpp:370
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
    const int nblk = (batch + HB - 1) / HB;
    const bool avx2 = host_has_avx2() && getenv("LDPC_HOST_PORTABLE") == nullptr;
    std::vector<Scratch> sc((size_t)host_threads_for(std::max(nblk, 1)));
    parallel_units(nblk, [&](int b, int k) {
        const int nb = std::min(HB, batch - b * HB);
        decode_block_i8(h, llr + (size_t)b * HB * h->n, hard + (size_t)b * HB * h->n, nb, n_iter, ip, sc[k], avx2);
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
