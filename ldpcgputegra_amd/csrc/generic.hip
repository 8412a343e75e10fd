// generic.hip -- any-H layered min-sum kernels (int8 and float).
//
// One lane = one codeword; every lane walks the checks in schedule order, so
// H indices are wave-uniform (scalar loads) and V/msg accesses are coalesced
// across the wave (layout V[node][stride], msg[edge][stride], codeword
// fastest).  This is the correctness baseline and the fallback for codes the
// windowed kernel (windowed.hip) cannot schedule; it restates
// code/x86/CDecoder/OMS/CDecoder_OMS_fixed_SSE.cpp:122-574 and
// code/x86/CDecoder/NMS/CDecoder_NMS_fixed_SSE.cpp:125-368 per lane.
#include "kernels.h"

namespace {

struct GenArgs {
    void *V;
    void *msg;
    const uint32_t *ev;
    const int *gdeg;
    const int *gcnt;
    int n_groups, m, stride, batch, iters;
    int algo, param, var_min, msg_max, early;
    float beta;
    int32_t *iters_used;
};

template <int D>
LDPC_DEV void check_i8(int8_t *__restrict__ V, int8_t *__restrict__ mp, const uint32_t *__restrict__ ev,
                       size_t stride, int b, bool later_group, const GenArgs &a)
{
    int c[D], av[D];
    int sign = 0, min1 = 127, min2 = 127;   // VECTOR_SET1(vSAT_POS_VAR)
#pragma unroll
    for (int j = 0; j < D; j++) {
        const int v = V[(size_t)ev[j] * stride + b];
        const int m = mp[(size_t)j * stride];
        const int cj = max(sat8(v - m), a.var_min);
        const int aj = later_group ? abs8(min(cj, a.msg_max)) : min(abs8(cj), a.msg_max);
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
        const int sig = as_i8(sign ^ (c[j] & 0x80));          // never 0 (0x40 set)
        const int m = sig < 0 ? as_i8(-r) : r;                  // _mm_sign_epi8
        mp[(size_t)j * stride] = (int8_t)m;
        V[(size_t)ev[j] * stride + b] = (int8_t)max(sat8(c[j] + m), a.var_min);
    }
}

template <int D>
LDPC_DEV void check_f32(float *__restrict__ V, float *__restrict__ mp, const uint32_t *__restrict__ ev,
                        size_t stride, int b, const GenArgs &a)
{
    float c[D], av[D];
    int sign = D & 1;
    float min1 = __builtin_huge_valf(), min2 = __builtin_huge_valf();
#pragma unroll
    for (int j = 0; j < D; j++) {
        const float cj = V[(size_t)ev[j] * stride + b] - mp[(size_t)j * stride];
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
        mp[(size_t)j * stride] = m;
        V[(size_t)ev[j] * stride + b] = c[j] + m;
    }
}

template <typename T>
LDPC_DEV bool syndrome_ok(const T *__restrict__ V, const uint32_t *__restrict__ ev, const int *gdeg,
                          const int *gcnt, int n_groups, size_t stride, int b)
{
    for (int g = 0; g < n_groups; g++) {
        const int d = gdeg[g];
        for (int i = 0; i < gcnt[g]; i++, ev += d) {
            int par = 0;
            for (int j = 0; j < d; j++) par ^= (V[(size_t)ev[j] * stride + b] > (T)0);
            if (par) return false;
        }
    }
    return true;
}

template <int D, typename T>
LDPC_DEV void run_group(T *V, T *msg, const uint32_t *ev, int cnt, size_t stride, int b, bool later,
                        const GenArgs &a)
{
    for (int i = 0; i < cnt; i++) {
        if constexpr (sizeof(T) == 1)
            check_i8<D>((int8_t *)V, (int8_t *)msg + (size_t)i * D * stride, ev + i * D, stride, b, later, a);
        else
            check_f32<D>((float *)V, (float *)msg + (size_t)i * D * stride, ev + i * D, stride, b, a);
    }
}

#define LDPC_DEG_CASES(X) \
    X(2) X(3) X(4) X(5) X(6) X(7) X(8) X(9) X(10) X(11) X(12) X(13) X(14) X(15) X(16) X(17) X(18) X(19) \
    X(20) X(21) X(22) X(23) X(24) X(25) X(26) X(27) X(28) X(29) X(30) X(31) X(32)

template <typename T>
__global__ void __launch_bounds__(64) generic_decode(GenArgs a)
{
    const int b = blockIdx.x * 64 + threadIdx.x;
    if (b >= a.batch) return;
    T *V = (T *)a.V;            // V[node][stride]
    T *msg = (T *)a.msg + b;    // this codeword's column of msg[edge][stride]
    const size_t stride = a.stride;
    int it = 0;
    while (it < a.iters) {
        const uint32_t *ev = a.ev;
        T *mp = msg;
        for (int g = 0; g < a.n_groups; g++) {
            const int d = a.gdeg[g], cnt = a.gcnt[g];
            // later degree groups: vAbs = abs(min(c, max_msg)) (OMS only,
            // CDecoder_OMS_fixed_SSE.cpp:293 vs :211)
            const bool later = (g > 0) && (a.algo != 1);
            switch (d) {
#define X(DD) \
    case DD: run_group<DD, T>(V, mp, ev, cnt, stride, b, later, a); break;
                LDPC_DEG_CASES(X)
#undef X
            default: break;
            }
            ev += (size_t)d * cnt;
            mp += (size_t)d * cnt * stride;
        }
        it++;
        if (a.early && syndrome_ok<T>((T *)a.V, a.ev, a.gdeg, a.gcnt, a.n_groups, stride, b)) break;
    }
    if (a.iters_used) a.iters_used[b] = it;
}

}  // namespace

int launch_generic(const DecodeLaunch &L, hipStream_t s)
{
    GenArgs a;
    a.V = L.V;
    a.msg = L.msg;
    a.ev = L.d_edge_var;
    a.gdeg = L.d_group_deg;
    a.gcnt = L.d_group_cnt;
    a.n_groups = L.n_groups;
    a.m = L.m;
    a.stride = L.stride;
    a.batch = L.batch;
    a.iters = L.iters;
    a.algo = L.algo;
    a.param = L.param;
    a.var_min = L.var_min;
    a.msg_max = L.msg_max;
    a.early = L.early;
    a.beta = L.beta;
    a.iters_used = L.iters_used;
    dim3 grid((L.batch + 63) / 64), block(64);
    if (L.is_float)
        hipLaunchKernelGGL(generic_decode<float>, grid, block, 0, s, a);
    else
        hipLaunchKernelGGL(generic_decode<int8_t>, grid, block, 0, s, a);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
