/*
 * ldpc_oracle.h -- CPU restatement of the reference's layered min-sum decoders.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product (ldpcgputegra_amd/, the
 * C-ABI library, the HIP kernels) links, loads or calls this code.  Only
 * tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use it, and
 * only as the checker / the timed CPU port.
 *
 * Every function restates code/x86 of boiseHPSim/ldpcGpuTegra:
 *   int8 OMS : code/x86/CDecoder/OMS/CDecoder_OMS_fixed_SSE.cpp:122-574
 *   int8 NMS : code/x86/CDecoder/NMS/CDecoder_NMS_fixed_SSE.cpp:125-368
 *   layout   : frame-major in/out, hard = (V > 0)  (code/x86/CTools/CTools.cpp:370)
 * The float decoders have no reference implementation (the reference's
 * CDecoder_fixed_SSE::decode(float*) is a no-op, code/x86/CDecoder/template/
 * CDecoder_fixed_SSE.cpp:35-40); they follow SURVEY.md 8(a) "Float variant".
 *
 * Pinning: tests/test_oracle_golden.py checks the int8 restatement bit-exactly
 * against hard decisions produced by the reference SSE decoder itself,
 * compiled from /root/reference by oracle/Makefile (golden vectors committed
 * under tests/golden/).  The float restatement is parity-unpinned (no
 * reference exists).
 */
#ifndef LDPC_ORACLE_H
#define LDPC_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* A layered H: checks in schedule order, grouped in runs of equal degree
 * (group g holds group_cnt[g] checks of degree group_deg[g]); edge_var lists
 * every check's variables in order.  Mirrors PosNoeudsVariable[] + DEG_k /
 * DEG_k_COMPUTATIONS (code/x86/Constantes/576x288/constantes_sse.h:37-41). */
typedef struct {
    int n, m, e, n_groups;
    const int *group_deg;
    const int *group_cnt;
    const uint32_t *edge_var;
} oracle_code;

enum { ORACLE_OMS = 0, ORACLE_NMS = 1 };

/* int8 layered decode of `batch` frame-major codewords.
 * algo ORACLE_OMS: param = offset (CDecoder_OMS_fixed_SSE::setOffset)
 * algo ORACLE_NMS: param = factor (CDecoder_NMS_fixed_SSE::setFactor, /32)
 * var_min/var_max: setVarRange; msg_max: setMsgRange upper bound.
 * hard: 0/1 per bit; v_out (optional): final int8 V per bit.
 * early_term: stop a codeword once its hard decisions satisfy every check
 * (tested after each full iteration); iters_used (optional) per codeword.
 * Returns 0, or -1 on unsupported parameters (the reference exits). */
int oracle_decode_i8(const oracle_code *h, const int8_t *llr, uint8_t *hard,
                     int8_t *v_out, int batch, int iters, int algo, int param,
                     int var_min, int var_max, int msg_max, int early_term,
                     int32_t *iters_used);

/* float layered min-sum: algo ORACLE_OMS -> r = max(min - beta, 0),
 * ORACLE_NMS -> r = min * beta.  (beta = 0 with OMS is plain min-sum.) */
int oracle_decode_f32(const oracle_code *h, const float *llr, uint8_t *hard,
                      float *v_out, int batch, int iters, int algo, float beta,
                      int early_term, int32_t *iters_used);

/* float -> int8 LLR quantizer, CFastFixConversion::generate
 * (code/x86/CFixPointConversion/CFastFixConversion.cpp:55-65). */
void oracle_quantize(const float *y, int8_t *q, long count, int factor, int sat_neg, int sat_pos);

/* Syndrome weight of hard decisions (number of unsatisfied checks). */
int oracle_syndrome(const oracle_code *h, const uint8_t *hard);

/* Multi-threaded wrapper used only for bench.py's cpu_baseline leg:
 * splits `batch` over `threads` pthreads (one decoder state each). */
int oracle_decode_i8_mt(const oracle_code *h, const int8_t *llr, uint8_t *hard,
                        int batch, int iters, int offset, int threads);

/* The same split for oracle_decode_i8 / oracle_decode_f32 with every output
 * (soft values, early termination, iterations used): tests check whole
 * BASELINE-sized batches with it, and the float cpu_baseline uses all cores. */
int oracle_decode_i8_mt_ex(const oracle_code *h, const int8_t *llr, uint8_t *hard, int8_t *v_out,
                           int batch, int iters, int algo, int param, int early_term,
                           int32_t *iters_used, int threads);
int oracle_decode_f32_mt(const oracle_code *h, const float *llr, uint8_t *hard, float *v_out,
                         int batch, int iters, int algo, float beta, int early_term,
                         int32_t *iters_used, int threads);

#ifdef __cplusplus
}
#endif
#endif
