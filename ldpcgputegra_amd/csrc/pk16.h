// pk16.h -- packed 16-bit helpers shared by the packed-pair DVB-S2 kernels
// (coop2.hip, coop3.hip): two codewords per lane, one per 16-bit half.
//
// An int8 value x sits in a half as R(x) = 256 x + 255 (value in the high
// byte, low byte all ones) and a message m as C(m) = 256 m.  Then
// R(x) - C(m) = R(x - m), R(x) + C(m) = R(x + m) and the i16 saturation
// 0x7FFF is R(127): the reference's _mm_subs_epi8 / _mm_adds_epi8 upper clamp
// (code/x86/CDecoder/OMS/CDecoder_OMS_fixed_SSE.cpp:201-254) for free.
// |x| = max(R, 510 - R) stays in R form; min / max / compares are monotone.
#pragma once
#include <type_traits>

#include "kernels_common.h"

typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef int i32x2 __attribute__((ext_vector_type(2)));

// structured buffer access, address = base + index * stride + offset
__device__ uint32_t sbuf_load_u32(i32x4 rsrc, int index, int offset, int soffset, int aux)
    __asm("llvm.amdgcn.struct.buffer.load.i32");
__device__ void sbuf_store_u16(unsigned short v, i32x4 rsrc, int index, int offset, int soffset, int aux)
    __asm("llvm.amdgcn.struct.buffer.store.i16");
__device__ i32x2 sbuf_load_v2(i32x4 rsrc, int index, int offset, int soffset, int aux)
    __asm("llvm.amdgcn.struct.buffer.load.v2i32");
__device__ void sbuf_store_v2(i32x2 v, i32x4 rsrc, int index, int offset, int soffset, int aux)
    __asm("llvm.amdgcn.struct.buffer.store.v2i32");

namespace {

constexpr int CW = 16;     // codewords per workgroup
constexpr int NP = 8;      // codeword pairs per workgroup = lanes per slot
constexpr int MREC = 64;   // message bytes per check and workgroup (8 pairs x 8 B)

typedef short s16x2 __attribute__((ext_vector_type(2)));
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));

// descriptor from wave-uniform values (kernel arguments, block index)
LDPC_DEV i32x4 buffer_rsrc(const void *base, uint32_t stride, uint32_t records)
{
    const uint64_t a = (uint64_t)base;
    i32x4 r;
    r.x = __builtin_amdgcn_readfirstlane((int)(uint32_t)a);
    r.y = __builtin_amdgcn_readfirstlane((int)((uint32_t)(a >> 32) | (stride << 16)));
    r.z = __builtin_amdgcn_readfirstlane((int)records);
    r.w = 0x00020000;
    return r;
}

LDPC_DEV s16x2 sv(uint32_t x) { return __builtin_bit_cast(s16x2, x); }
LDPC_DEV uint32_t us(s16x2 x) { return __builtin_bit_cast(uint32_t, x); }
LDPC_DEV uint32_t pk_sub_sat(uint32_t a, uint32_t b) { return us(__builtin_elementwise_sub_sat(sv(a), sv(b))); }
LDPC_DEV uint32_t pk_add_sat(uint32_t a, uint32_t b) { return us(__builtin_elementwise_add_sat(sv(a), sv(b))); }
LDPC_DEV uint32_t pk_max(uint32_t a, uint32_t b) { return us(__builtin_elementwise_max(sv(a), sv(b))); }
LDPC_DEV uint32_t pk_min(uint32_t a, uint32_t b) { return us(__builtin_elementwise_min(sv(a), sv(b))); }
LDPC_DEV uint32_t pk_sub(uint32_t a, uint32_t b) { return us(sv(a) - sv(b)); }
LDPC_DEV uint32_t pk_sra15(uint32_t a) { return us(sv(a) >> (short)15); }
LDPC_DEV uint32_t pk_mul_lo(uint32_t a, uint32_t b)   // v_pk_mul_lo_u16
{
    return us(__builtin_bit_cast(s16x2, __builtin_bit_cast(u16x2, a) * __builtin_bit_cast(u16x2, b)));
}
LDPC_DEV uint32_t bfi(uint32_t m, uint32_t a, uint32_t b) { return (m & a) | (~m & b); }
LDPC_DEV uint32_t perm(uint32_t s0, uint32_t s1, uint32_t sel) { return __builtin_amdgcn_perm(s0, s1, sel); }
// hide a value from the optimiser: keeps sign-splat masks as bit masks (v_bfi_b32)
// instead of per-half compare/select, and constants in VGPRs (no op_sel / literal splits)
LDPC_DEV uint32_t opaque(uint32_t x)
{
    asm volatile("" : "+v"(x));
    return x;
}
LDPC_DEV int hi8(uint32_t x, int h) { return __builtin_amdgcn_sbfe((int)x, 8 + 16 * h, 8); }   // half h's value

constexpr uint32_t RNEG127 = 0x81FF81FFu;   // R(-127) per half
constexpr uint32_t R127 = 0x7FFF7FFFu;      // R(127)
constexpr uint32_t R0 = 0x00FF00FFu;        // R(0)
constexpr uint32_t C510 = 0x01FE01FEu;      // |R(x)| = max(R, 510 - R)
constexpr uint32_t HIBYTES = 0xFF00FF00u;   // R -> C
constexpr uint32_t SIGNS = 0x80008000u;

LDPC_DEV uint32_t unpack_v(uint32_t raw, uint32_t sel) { return perm(raw, raw, sel); }   // V dword -> R pair
LDPC_DEV uint32_t pack_v(uint32_t r) { return perm(r, r, 0x0c0c0301u); }           // R pair -> u16 [b0 b1]
LDPC_DEV uint32_t abs_r(uint32_t r, uint32_t c510) { return pk_max(r, pk_sub(c510, r)); }

// the packed-math constants, held in VGPRs: as SGPR operands hipcc splats
// them with op_sel_hi, and gfx950 then needs a wait state before the result
// is read
struct PkK {
    uint32_t neg127, r0, c510, rmm, coff;   // R(-127), R(0), 510, R(msg_max), C(offset) per half
    uint32_t m3 = 0x03000300u, c4 = 0x040c000cu;   // old_msg's selector mask / constant
};

// byte tables [+cst1, -cst1, +cst2, -cst2] of the two codewords of a pair
struct MsgTab {
    uint32_t t0, t1;
};
LDPC_DEV MsgTab msg_tab(uint32_t MB)
{
    const uint32_t p0 = perm(MB, MB, 0x0c010c00u), p1 = perm(MB, MB, 0x0c030c02u);   // (cst1, cst2) as u16
    return {perm(pk_sub(0u, p0), p0, 0x06020400u), perm(pk_sub(0u, p1), p1, 0x06020400u)};
}

// old message of edge J (C pair): byte 1 = t0[code0], byte 3 = t1[code1].
// m3 / c4: 0x03000300 / 0x040c000c held in VGPRs, so that the mask-and-or is
// one v_bitop3 (gfx9 VOP3 encodes no literal)
template <int J>
LDPC_DEV uint32_t old_msg(uint32_t MA, const MsgTab &t, uint32_t m3 = 0x03000300u, uint32_t c4 = 0x040c000cu)
{
    uint32_t sh;
    if constexpr (J <= 4)
        sh = MA << (8 - 2 * J);
    else
        sh = MA >> (2 * J - 8);
    return perm(t.t1, t.t0, (sh & m3) | c4);
}

// Message record of a check (coop3): MB = eps * cst1, eps * cst2 as signed
// bytes per codeword (eps = -1 where the sign parity of the check's
// contributions, odd-degree flip included, is odd), MA = a 2-bit code per
// edge: bit 0 = the edge's contribution c was negative, bit 1 = the edge got
// cst2 (a > min1).  The message (reference: ((c < 0) ^ par) ? -cst : cst) is
// then (-1)^bit0 * eps * cst, decoded by old_msg through the byte table
// [+eps cst1, -eps cst1, +eps cst2, -eps cst2].

// (a & m) | b as one v_bitop3_b32 (truth table 0xEA); written with | and &
// the compiler builds an and + or3 tree: 1.5 instructions per flag, not 1
#ifndef LDPC_PK_ANDOR
#define LDPC_PK_ANDOR 1   // experiment switch (tools/build_variant.sh): 0 = plain & and |
#endif
LDPC_DEV uint32_t and_or(uint32_t a, uint32_t m, uint32_t b)
{
#if LDPC_PK_ANDOR
    return __builtin_amdgcn_bitop3_b32(a, m, b, 0xEA);
#else
    return (a & m) | b;
#endif
}
// edge J's code (bit 0: c < 0, bit 1: got cst2) into MA, from the two half masks
template <int J>
LDPC_DEV uint32_t add_code(uint32_t MA, uint32_t sc, uint32_t neq)
{
    return and_or(neq, 0x00020002u << (2 * J), and_or(sc, 0x00010001u << (2 * J), MA));
}

// |x| of an R pair, or of a contribution saturated below R(-128) (0x8000):
// the saturating 510 - c caps it at R(127), the reference's |max(c, -127)|
LDPC_DEV uint32_t abs_sat(uint32_t r, uint32_t c510) { return pk_max(r, pk_sub_sat(c510, r)); }

// eps * k (C form) of the check's two constants; par: sign bits = the parity
LDPC_DEV void signed_csts(uint32_t k1, uint32_t k2, uint32_t par, uint32_t &e1, uint32_t &e2)
{
    const uint32_t eps = pk_sra15(par) | 0x00010001u;   // +-1 per half
    e1 = pk_mul_lo(k1, eps);
    e2 = pk_mul_lo(k2, eps);
}

// new V of first-group edge J (R pair), its code into MA.  Sign-magnitude
// form of the reference's max(sat(c + m), -127) (code/x86/CDecoder/OMS/
// CDecoder_OMS_fixed_SSE.cpp:239-254): c + m = sign(c) * (|c| + eps * cst),
// so V' = sign(c) * min(|c| + eps * cst, 127) -- |c| + eps cst >= -cst >= -127
// needs no lower clamp, and c enters only through its sign (a = |c| from
// abs_sat), so c itself need not be clamped at -127
template <int J>
LDPC_DEV uint32_t new_v(uint32_t c, uint32_t a, uint32_t min1, uint32_t e1, uint32_t e2, uint32_t &MA, uint32_t c510)
{
    const uint32_t neq = opaque(pk_sra15(pk_sub(min1, a)));   // -1: a > min1, the edge gets cst2
    const uint32_t T = pk_add_sat(a, bfi(neq, e2, e1));       // R(|c| + eps cst), capped at R(127)
    const uint32_t sc = opaque(pk_sra15(c));                  // -1: c < 0
    MA = add_code<J>(MA, sc, neq);
    return bfi(sc, pk_sub(c510, T), T);
}

// the code of edge J only (an edge whose V the next check rewrites)
template <int J>
LDPC_DEV void msg_code(uint32_t c, uint32_t a, uint32_t min1, uint32_t &MA)
{
    const uint32_t neq = opaque(pk_sra15(pk_sub(min1, a)));
    const uint32_t sc = opaque(pk_sra15(c));
    MA = add_code<J>(MA, sc, neq);
}

// later degree groups (a = |min(c, msg_max)| is not |c|; c clamped at -127):
// V' = max(sat(c + m), -127) with m = (-1)^(c < 0) * (eps * cst), same record
template <int J>
LDPC_DEV uint32_t new_v_later(uint32_t c, uint32_t a, uint32_t min1, uint32_t e1, uint32_t e2, uint32_t &MA,
                              uint32_t neg127)
{
    const uint32_t neq = opaque(pk_sra15(pk_sub(min1, a)));
    const uint32_t sc = pk_sra15(c);
    const uint32_t m = bfi(neq, e2, e1);
    MA |= (sc & (0x00010001u << (2 * J))) | (neq & (0x00020002u << (2 * J)));
    return pk_max(pk_add_sat(c, pk_sub(m ^ sc, sc)), neg127);
}

template <int I, int N, typename F>
LDPC_DEV void static_for(F &&f)
{
    if constexpr (I < N) {
        f(std::integral_constant<int, I>{});
        static_for<I + 1, N>(f);
    }
}

// LDS-DMA: every active lane copies 16 B from gsrc to lds_dst + 16 * lane,
// without passing through VGPRs (the compiler neither counts nor waits for
// it: the chain wave waits with an explicit vmcnt)
LDPC_DEV void dma16(const void *gsrc, uint32_t lds_dst)
{
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(gsrc), "s"(lds_dst)
                 : "memory");
}

}  // namespace
