// kernels_common.h -- device helpers shared by the decode kernels.
//
// Exact int8 semantics of the reference's SSE intrinsics
// (code/x86/CDecoder/OMS/CDecoder_OMS_fixed_SSE.cpp:26-80), evaluated in
// 32-bit VGPRs:
//   sat8      _mm_subs_epi8 / _mm_adds_epi8 (saturate to [-128, 127])
//   abs8      _mm_abs_epi8   (abs8(-128) == -128)
//   subs_u8   _mm_subs_epu8
//   as_i8     reinterpret the low byte as int8 (what the SSE lanes hold)
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define LDPC_DEV __device__ __forceinline__

LDPC_DEV int clampi(int x, int lo, int hi) { return max(lo, min(x, hi)); }
LDPC_DEV int sat8(int x) { return clampi(x, -128, 127); }
LDPC_DEV int abs8(int x) { return x == -128 ? -128 : abs(x); }
LDPC_DEV int as_i8(int x) { return (int)(int8_t)(uint8_t)x; }
LDPC_DEV int subs_u8(int a, int b) { return max((a & 0xFF) - (b & 0xFF), 0); }

// CDecoder_NMS_fixed_SSE.cpp:202-214: packs_epi16((u16(min) * factor) >> 5)
LDPC_DEV int nms_scale(int mn, int factor)
{
    uint32_t prod = ((uint32_t)(mn & 0xFF) * (uint32_t)(factor & 0xFFFF)) & 0xFFFFu;
    int s = (int)(int16_t)(uint16_t)(prod >> 5);
    return clampi(s, -128, 127);
}

// The constants a check sends back (cst1 -> the min1 edge, cst2 -> the rest),
// CDecoder_OMS_fixed_SSE.cpp:229-230 / CDecoder_NMS_fixed_SSE.cpp:202-214.
LDPC_DEV void check_constants(int algo, int param, int msg_max, int min1, int min2, int &cst1, int &cst2)
{
    if (algo == 1) {  // NMS
        cst1 = nms_scale(min2, param);
        cst2 = nms_scale(min1, param);
    } else {          // OMS / MS
        cst1 = min(as_i8(subs_u8(min2, param)), msg_max);
        cst2 = min(as_i8(subs_u8(min1, param)), msg_max);
    }
}

struct AwgnTable {
    uint32_t t[64];   // thresholds, t[63] = sat (ldpc_awgn_i8_table)
};

LDPC_DEV uint64_t splitmix64(uint64_t x)
{
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}
