// host_simd.h -- the SIMD check of the host decoder (host.cpp), written once
// over a vector-width trait and compiled per instruction set in its own
// translation unit: host_avx2.cpp (-mavx2: W = 32 lanes) and host_sse4.cpp
// (-msse4.1: W = 16, the reference's width, for hosts without AVX2).  Nothing
// here carries a target attribute: each TU's flags decide the encoding, so the
// SSE4.1 objects hold no VEX instruction (tools/check_host_isa.py checks the
// object at build time).  Everything has internal linkage, so the linker can
// never merge an AVX2-compiled inline copy into the SSE4.1 path.
#pragma once
#include <cstddef>
#include <cstdint>

#include <immintrin.h>

#include "ldpc_internal.h"

struct I8Params {
    int algo, param, var_min, msg_max, early;
};

// one iteration over every check of H, block of W codewords interleaved
// (V[N + 1][W], msg[E][W]); live[l] == 0: lane l converged (frozen)
void host_checks_avx2(const ldpc_code *h, int8_t *V, int8_t *msg, const I8Params &p, const uint8_t *live);
void host_checks_sse4(const ldpc_code *h, int8_t *V, int8_t *msg, const I8Params &p, const uint8_t *live);

#ifdef LDPC_HOST_SIMD_IMPL
namespace {

#ifndef LDPC_HOST_PF
#define LDPC_HOST_PF 2
#endif
constexpr int PF = LDPC_HOST_PF;   // checks ahead whose V rows are prefetched

#if defined(__AVX2__)
struct Simd {
    static constexpr int W = 32;
    using V = __m256i;
    static V ld(const void *p) { return _mm256_load_si256((const V *)p); }
    static void st(void *p, V v) { _mm256_store_si256((V *)p, v); }
    static V set1(int x) { return _mm256_set1_epi8((char)x); }
    static V zero() { return _mm256_setzero_si256(); }
    static V subs(V a, V b) { return _mm256_subs_epi8(a, b); }
    static V adds(V a, V b) { return _mm256_adds_epi8(a, b); }
    static V subs_u(V a, V b) { return _mm256_subs_epu8(a, b); }
    static V max(V a, V b) { return _mm256_max_epi8(a, b); }
    static V min(V a, V b) { return _mm256_min_epi8(a, b); }
    static V abs(V a) { return _mm256_abs_epi8(a); }
    static V xor_(V a, V b) { return _mm256_xor_si256(a, b); }
    static V and_(V a, V b) { return _mm256_and_si256(a, b); }
    static V eq(V a, V b) { return _mm256_cmpeq_epi8(a, b); }
    static V blend(V a, V b, V m) { return _mm256_blendv_epi8(a, b, m); }
    static V sign(V a, V b) { return _mm256_sign_epi8(a, b); }
    // NMS constants: (u16(min) * f) >> 5, signed-saturated to int8 (unpack /
    // pack stay inside each 128-bit lane, so the byte order is kept)
    static V nms(V mn, int f)
    {
        const V z = zero(), ff = _mm256_set1_epi16((short)f);
        const V lo = _mm256_srli_epi16(_mm256_mullo_epi16(_mm256_unpacklo_epi8(mn, z), ff), 5);
        const V hi = _mm256_srli_epi16(_mm256_mullo_epi16(_mm256_unpackhi_epi8(mn, z), ff), 5);
        return _mm256_packs_epi16(lo, hi);
    }
};
#elif defined(__SSE4_1__)
struct Simd {
    static constexpr int W = 16;
    using V = __m128i;
    static V ld(const void *p) { return _mm_load_si128((const V *)p); }
    static void st(void *p, V v) { _mm_store_si128((V *)p, v); }
    static V set1(int x) { return _mm_set1_epi8((char)x); }
    static V zero() { return _mm_setzero_si128(); }
    static V subs(V a, V b) { return _mm_subs_epi8(a, b); }
    static V adds(V a, V b) { return _mm_adds_epi8(a, b); }
    static V subs_u(V a, V b) { return _mm_subs_epu8(a, b); }
    static V max(V a, V b) { return _mm_max_epi8(a, b); }
    static V min(V a, V b) { return _mm_min_epi8(a, b); }
    static V abs(V a) { return _mm_abs_epi8(a); }
    static V xor_(V a, V b) { return _mm_xor_si128(a, b); }
    static V and_(V a, V b) { return _mm_and_si128(a, b); }
    static V eq(V a, V b) { return _mm_cmpeq_epi8(a, b); }
    static V blend(V a, V b, V m) { return _mm_blendv_epi8(a, b, m); }
    static V sign(V a, V b) { return _mm_sign_epi8(a, b); }
    static V nms(V mn, int f)
    {
        const V z = zero(), ff = _mm_set1_epi16((short)f);
        const V lo = _mm_srli_epi16(_mm_mullo_epi16(_mm_unpacklo_epi8(mn, z), ff), 5);
        const V hi = _mm_srli_epi16(_mm_mullo_epi16(_mm_unpackhi_epi8(mn, z), ff), 5);
        return _mm_packs_epi16(lo, hi);
    }
};
#else
#error "host_simd.h: compile with -mavx2 or -msse4.1"
#endif

// one check over the W lanes of a block (OMS_fixed_SSE.cpp:201-254; later
// groups :293-314; NMS_fixed_SSE.cpp:188-240); D > 0: the degree known at
// compile time (the edge loops unrolled, contributions in registers), D = 0:
// runtime degree d.  With a runtime degree the contributions went through the
// stack and DVB-S2 r1/2 took 0.42 ns per edge and codeword on one thread, 0.31
// unrolled.
template <int D, bool ET>
inline void check_simd(int8_t *V, int8_t *msg, const uint32_t *ev, int d, bool later, const I8Params &p,
                       const uint8_t *live)
{
    using S = Simd;
    using Vec = S::V;
    constexpr int W = S::W;
    const int dd = D > 0 ? D : d;
    const Vec vmin = S::set1(p.var_min), mm = S::set1(p.msg_max), s80 = S::set1(0x80);
    const bool nms = p.algo == LDPC_ALGO_NMS;
    Vec c[D > 0 ? D : 64], a[D > 0 ? D : 64];
    Vec sign = S::zero(), min1 = S::set1(127), min2 = min1;
#pragma GCC unroll 32
    for (int j = 0; j < dd; j++) {
        const Vec v = S::ld(V + (size_t)ev[j] * W);
        const Vec cj = S::max(S::subs(v, S::ld(msg + j * W)), vmin);
        const Vec aj = (nms || !later) ? S::min(S::abs(cj), mm) : S::abs(S::min(cj, mm));
        sign = S::xor_(sign, S::and_(cj, s80));
        c[j] = cj;
        a[j] = aj;
        min2 = S::min(min2, S::max(aj, min1));
        min1 = S::min(min1, aj);
    }
    Vec cst1, cst2;
    if (nms) {
        cst1 = S::nms(min2, p.param);
        cst2 = S::nms(min1, p.param);
    } else {
        const Vec off = S::set1(p.param);
        cst1 = S::min(S::subs_u(min2, off), mm);
        cst2 = S::min(S::subs_u(min1, off), mm);
    }
    sign = S::xor_(sign, S::set1((dd & 1) ? 0xC0 : 0x40));
    const Vec keep = ET ? S::eq(S::ld(live), S::zero()) : S::zero();
#pragma GCC unroll 32
    for (int j = 0; j < dd; j++) {
        const Vec r = S::blend(cst2, cst1, S::eq(a[j], min1));
        const Vec m = S::sign(r, S::xor_(sign, S::and_(c[j], s80)));
        Vec nv = S::max(S::adds(c[j], m), vmin);
        int8_t *vp = V + (size_t)ev[j] * W;
        if (ET) nv = S::blend(nv, S::ld(vp), keep);   // converged: frozen
        S::st(msg + j * W, m);
        S::st(vp, nv);
    }
}

template <bool ET>
inline void check_dispatch(int8_t *V, int8_t *msg, const uint32_t *ev, int d, bool later, const I8Params &p,
                           const uint8_t *live)
{
    switch (d) {   // the degrees of the reference's codes (DVB-S2: 7, 10, 14, 22, 27, 30 and the tails)
    case 3: return check_simd<3, ET>(V, msg, ev, d, later, p, live);
    case 6: return check_simd<6, ET>(V, msg, ev, d, later, p, live);
    case 7: return check_simd<7, ET>(V, msg, ev, d, later, p, live);
    case 8: return check_simd<8, ET>(V, msg, ev, d, later, p, live);
    case 10: return check_simd<10, ET>(V, msg, ev, d, later, p, live);
    case 14: return check_simd<14, ET>(V, msg, ev, d, later, p, live);
    case 22: return check_simd<22, ET>(V, msg, ev, d, later, p, live);
    default: return check_simd<0, ET>(V, msg, ev, d, later, p, live);
    }
}

// one layered iteration over every check (the schedule of H's table order)
template <bool ET>
inline void checks_all(const ldpc_code *h, int8_t *V, int8_t *msg, const I8Params &p, const uint8_t *live)
{
    constexpr int W = Simd::W;
    size_t e0 = 0;
    for (int i = 0; i < h->m; i++) {
        const int d = h->check_deg[i];
        const bool later = h->check_group[i] > 0;
        const uint32_t *ev = &h->edge_var[h->check_start[i]];
        if (PF > 0 && i + PF < h->m) {   // the V rows of a check PF ahead (random rows: no HW prefetch)
            const uint32_t *en = &h->edge_var[h->check_start[i + PF]];
            for (int j = 0; j < h->check_deg[i + PF]; j++) __builtin_prefetch(V + (size_t)en[j] * W, 1, 3);
        }
        check_dispatch<ET>(V, msg + e0 * W, ev, d, later, p, live);
        e0 += (size_t)d;
    }
}

}  // namespace
#endif
