/*
 * ldpc_oracle.c -- scalar CPU restatement of the reference layered decoders.
 * TEST INFRASTRUCTURE ONLY (see ldpc_oracle.h).  Not part of the product.
 *
 * int8 arithmetic follows the SSE intrinsics of the reference one for one:
 *   _mm_subs_epi8 / _mm_adds_epi8  -> sat8()
 *   _mm_max_epi8(.., min_var)      -> the var_min clamp ("ON DOIT CONSERVER LA
 *                                     SATURATION MIN A CAUSE DE -128",
 *                                     CDecoder_OMS_fixed_SSE.cpp:56-60)
 *   _mm_abs_epi8                   -> abs8()  (abs8(-128) == -128)
 *   _mm_subs_epu8(min, offset)     -> subs_u8()
 *   _mm_sign_epi8(r, sig)          -> sign8()
 */
#include "ldpc_oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

static inline int sat8(int x) { return x < -128 ? -128 : (x > 127 ? 127 : x); }
static inline int abs8(int x) { return x == -128 ? -128 : (x < 0 ? -x : x); }
static inline int imin(int a, int b) { return a < b ? a : b; }
static inline int imax(int a, int b) { return a > b ? a : b; }
static inline int subs_u8(int a, int b)
{
    int r = (a & 0xFF) - (b & 0xFF);
    return r < 0 ? 0 : r;            /* result is 0..255, re-read as int8 below */
}
static inline int as_i8(int x) { return (int)(int8_t)(uint8_t)x; }
static inline int sign8(int r, int sig)
{
    if (sig < 0) return as_i8(-r);
    if (sig == 0) return 0;
    return r;
}

/* NMS scaling: packs_epi16((u16(min) * factor) >> 5)
 * (CDecoder_NMS_fixed_SSE.cpp:202-214). */
static inline int nms_scale(int mn, int factor)
{
    uint16_t prod = (uint16_t)((uint16_t)(uint8_t)mn * (uint16_t)factor);
    int s = (int16_t)(prod >> 5);
    return s > 127 ? 127 : (s < -128 ? -128 : s);
}

/* Early termination (early_term): the build's own definition, SURVEY.md
 * §8(f) row 2 -- PER CODEWORD, on the POSTERIOR hard decisions v > 0, checked
 * AFTER each whole iteration; the codeword's soft output, hard decisions and
 * iterations used freeze there.  This is NOT a restatement of the reference's
 * commented-out `arret` test (CDecoder_OMS_fixed_SSE.cpp:154,167,232-236,255,
 * 551-553), which ORs the sign parity of the EXTRINSIC contributions c_j of
 * every check DURING the iteration (after the odd-degree flip) and would stop
 * the whole 16-frame decode() call at once.  code/x86 runs a fixed iteration
 * count (the test is commented out), so iterations-used parity is pinned by
 * this definition only -- unpinned by the reference; with early_term off the
 * oracle is the reference's recurrence, pinned by the golden vectors. */
static int check_syndrome_ok(const oracle_code *h, const int8_t *v)
{
    const uint32_t *ev = h->edge_var;
    for (int g = 0; g < h->n_groups; g++) {
        int d = h->group_deg[g];
        for (int i = 0; i < h->group_cnt[g]; i++, ev += d) {
            int par = 0;
            for (int j = 0; j < d; j++) par ^= (v[ev[j]] > 0);
            if (par) return 0;
        }
    }
    return 1;
}

/* One codeword, int8.  The per-check body restates
 * CDecoder_OMS_fixed_SSE.cpp:201-254 (first degree group) and :285-327
 * (later groups: vAbs = abs(min(c, max_msg)) instead of min(abs(c), max_msg)).
 * The NMS body restates CDecoder_NMS_fixed_SSE.cpp:188-240 (both groups use
 * min(abs(c), max_msg); constants are normalised, no offset). */
static void decode_one_i8(const oracle_code *h, const int8_t *llr, uint8_t *hard,
                          int8_t *v_out, int iters, int algo, int param, int var_min,
                          int var_max, int msg_max, int early_term, int32_t *iters_used,
                          int8_t *v, int8_t *msg, int *contr, int *absv)
{
    memset(msg, 0, (size_t)h->e);
    for (int i = 0; i < h->n; i++) v[i] = llr[i];
    int it = 0;
    while (it < iters) {
        const uint32_t *ev = h->edge_var;
        int8_t *mp = msg;
        for (int g = 0; g < h->n_groups; g++) {
            const int d = h->group_deg[g];
            const int sfix = (d & 1) ? 0xC0 : 0x40;
            for (int ci = 0; ci < h->group_cnt[g]; ci++, ev += d, mp += d) {
                int sign = 0, min1 = var_max, min2 = var_max;
                for (int j = 0; j < d; j++) {
                    int c = imax(sat8(v[ev[j]] - mp[j]), var_min);
                    int a;
                    if (algo == ORACLE_NMS || g == 0)
                        a = imin(abs8(c), msg_max);
                    else
                        a = abs8(imin(c, msg_max));
                    sign ^= (c & 0x80);
                    contr[j] = c;
                    absv[j] = a;
                    int t = min1;
                    min1 = imin(a, min1);
                    min2 = imin(min2, imax(a, t));
                }
                int cst1, cst2;
                if (algo == ORACLE_NMS) {
                    cst1 = nms_scale(min2, param);
                    cst2 = nms_scale(min1, param);
                } else {
                    cst1 = imin(as_i8(subs_u8(min2, param)), msg_max);
                    cst2 = imin(as_i8(subs_u8(min1, param)), msg_max);
                }
                sign ^= sfix;
                for (int j = 0; j < d; j++) {
                    int r = (absv[j] == min1) ? cst1 : cst2;
                    int sig = as_i8(sign ^ (contr[j] & 0x80));
                    int m = sign8(r, sig);
                    mp[j] = (int8_t)m;
                    v[ev[j]] = (int8_t)imax(sat8(contr[j] + m), var_min);
                }
            }
        }
        it++;
        if (early_term && check_syndrome_ok(h, v)) break;
    }
    if (iters_used) *iters_used = it;
    for (int i = 0; i < h->n; i++) hard[i] = (v[i] > 0);
    if (v_out) memcpy(v_out, v, (size_t)h->n);
}

static int code_ok(const oracle_code *h)
{
    int e = 0, m = 0;
    for (int g = 0; g < h->n_groups; g++) {
        if (h->group_deg[g] <= 0 || h->group_deg[g] > 64) return 0;
        e += h->group_deg[g] * h->group_cnt[g];
        m += h->group_cnt[g];
    }
    return e == h->e && m == h->m;
}

int oracle_decode_i8(const oracle_code *h, const int8_t *llr, uint8_t *hard,
                     int8_t *v_out, int batch, int iters, int algo, int param,
                     int var_min, int var_max, int msg_max, int early_term,
                     int32_t *iters_used)
{
    /* CDecoder_OMS_fixed_SSE::decode exits unless vSAT_POS_VAR == 127 (:116-119) */
    if (var_max != 127 || var_min < -128 || var_min > 0 || msg_max < 0 || msg_max > 127)
        return -1;
    if (!code_ok(h) || batch < 0 || iters < 0) return -1;
    int8_t *v = (int8_t *)malloc((size_t)h->n);
    int8_t *msg = (int8_t *)malloc((size_t)h->e + 1);
    int contr[64], absv[64];
    for (int b = 0; b < batch; b++)
        decode_one_i8(h, llr + (size_t)b * h->n, hard + (size_t)b * h->n,
                      v_out ? v_out + (size_t)b * h->n : NULL, iters, algo, param,
                      var_min, var_max, msg_max, early_term,
                      iters_used ? iters_used + b : NULL, v, msg, contr, absv);
    free(v);
    free(msg);
    return 0;
}

/* ---- float ---------------------------------------------------------- */

static int check_syndrome_ok_f(const oracle_code *h, const float *v)
{
    const uint32_t *ev = h->edge_var;
    for (int g = 0; g < h->n_groups; g++) {
        int d = h->group_deg[g];
        for (int i = 0; i < h->group_cnt[g]; i++, ev += d) {
            int par = 0;
            for (int j = 0; j < d; j++) par ^= (v[ev[j]] > 0.0f);
            if (par) return 0;
        }
    }
    return 1;
}

int oracle_decode_f32(const oracle_code *h, const float *llr, uint8_t *hard,
                      float *v_out, int batch, int iters, int algo, float beta,
                      int early_term, int32_t *iters_used)
{
    if (!code_ok(h) || batch < 0 || iters < 0) return -1;
    float *v = (float *)malloc(sizeof(float) * (size_t)h->n);
    float *msg = (float *)malloc(sizeof(float) * ((size_t)h->e + 1));
    float contr[64], absv[64];
    for (int b = 0; b < batch; b++) {
        const float *in = llr + (size_t)b * h->n;
        memset(msg, 0, sizeof(float) * (size_t)h->e);
        for (int i = 0; i < h->n; i++) v[i] = in[i];
        int it = 0;
        while (it < iters) {
            const uint32_t *ev = h->edge_var;
            float *mp = msg;
            for (int g = 0; g < h->n_groups; g++) {
                const int d = h->group_deg[g];
                const int dpar = d & 1;
                for (int ci = 0; ci < h->group_cnt[g]; ci++, ev += d, mp += d) {
                    int sign = 0;
                    float min1 = INFINITY, min2 = INFINITY;
                    for (int j = 0; j < d; j++) {
                        float c = v[ev[j]] - mp[j];
                        float a = fabsf(c);
                        sign ^= (c < 0.0f);
                        contr[j] = c;
                        absv[j] = a;
                        float t = min1;
                        min1 = fminf(a, min1);
                        min2 = fminf(min2, fmaxf(a, t));
                    }
                    float cst1, cst2;
                    if (algo == ORACLE_NMS) {
                        cst1 = min2 * beta;
                        cst2 = min1 * beta;
                    } else {
                        cst1 = fmaxf(min2 - beta, 0.0f);
                        cst2 = fmaxf(min1 - beta, 0.0f);
                    }
                    sign ^= dpar;
                    for (int j = 0; j < d; j++) {
                        float r = (absv[j] == min1) ? cst1 : cst2;
                        int neg = sign ^ (contr[j] < 0.0f);
                        float m = neg ? -r : r;
                        mp[j] = m;
                        float nv = contr[j] + m;
                        v[ev[j]] = nv;
                    }
                }
            }
            it++;
            if (early_term && check_syndrome_ok_f(h, v)) break;
        }
        if (iters_used) iters_used[b] = it;
        for (int i = 0; i < h->n; i++) hard[(size_t)b * h->n + i] = (v[i] > 0.0f);
        if (v_out) memcpy(v_out + (size_t)b * h->n, v, sizeof(float) * (size_t)h->n);
    }
    free(v);
    free(msg);
    return 0;
}

void oracle_quantize(const float *y, int8_t *q, long count, int factor, int sat_neg, int sat_pos)
{
    for (long i = 0; i < count; i++) {
        int value = (int)((float)factor * y[i]);
        value = (value > sat_neg) ? value : sat_neg;
        value = (value < sat_pos) ? value : sat_pos;
        q[i] = (int8_t)value;
    }
}

int oracle_syndrome(const oracle_code *h, const uint8_t *hard)
{
    const uint32_t *ev = h->edge_var;
    int bad = 0;
    for (int g = 0; g < h->n_groups; g++) {
        int d = h->group_deg[g];
        for (int i = 0; i < h->group_cnt[g]; i++, ev += d) {
            int par = 0;
            for (int j = 0; j < d; j++) par ^= hard[ev[j]] & 1;
            bad += par;
        }
    }
    return bad;
}

typedef struct {
    const oracle_code *h;
    const int8_t *llr;
    uint8_t *hard;
    int8_t *soft;
    int32_t *iters_used;
    const float *fllr;
    float *fsoft;
    int batch, iters, algo, param, early_term, rc;
    float beta;
} mt_job;

static void *mt_worker(void *p)
{
    mt_job *j = (mt_job *)p;
    if (j->fllr)
        j->rc = oracle_decode_f32(j->h, j->fllr, j->hard, j->fsoft, j->batch, j->iters, j->algo, j->beta,
                                  j->early_term, j->iters_used);
    else
        j->rc = oracle_decode_i8(j->h, j->llr, j->hard, j->soft, j->batch, j->iters, j->algo, j->param,
                                 -127, 127, 31, j->early_term, j->iters_used);
    return NULL;
}

/* split `batch` codewords over `threads` pthreads, contiguous ranges */
static int run_mt(mt_job proto, int batch, int threads, int n)
{
    if (threads < 1) threads = 1;
    if (threads > 256) threads = 256;
    pthread_t tid[256];
    mt_job jobs[256];
    int per = (batch + threads - 1) / threads, t = 0;
    for (int s = 0; s < batch; s += per, t++) {
        int cnt = (batch - s < per) ? batch - s : per;
        jobs[t] = proto;
        jobs[t].batch = cnt;
        jobs[t].hard = proto.hard + (size_t)s * n;
        if (proto.llr) jobs[t].llr = proto.llr + (size_t)s * n;
        if (proto.fllr) jobs[t].fllr = proto.fllr + (size_t)s * n;
        if (proto.soft) jobs[t].soft = proto.soft + (size_t)s * n;
        if (proto.fsoft) jobs[t].fsoft = proto.fsoft + (size_t)s * n;
        if (proto.iters_used) jobs[t].iters_used = proto.iters_used + s;
        pthread_create(&tid[t], NULL, mt_worker, &jobs[t]);
    }
    int rc = 0;
    for (int i = 0; i < t; i++) {
        pthread_join(tid[i], NULL);
        rc |= jobs[i].rc;
    }
    return rc;
}

int oracle_decode_i8_mt(const oracle_code *h, const int8_t *llr, uint8_t *hard,
                        int batch, int iters, int offset, int threads)
{
    mt_job j = {h, llr, hard, NULL, NULL, NULL, NULL, batch, iters, ORACLE_OMS, offset, 0, 0, 0.0f};
    return run_mt(j, batch, threads, h->n);
}

int oracle_decode_i8_mt_ex(const oracle_code *h, const int8_t *llr, uint8_t *hard, int8_t *v_out,
                           int batch, int iters, int algo, int param, int early_term,
                           int32_t *iters_used, int threads)
{
    mt_job j = {h, llr, hard, v_out, iters_used, NULL, NULL, batch, iters, algo, param, early_term, 0, 0.0f};
    return run_mt(j, batch, threads, h->n);
}

int oracle_decode_f32_mt(const oracle_code *h, const float *llr, uint8_t *hard, float *v_out,
                         int batch, int iters, int algo, float beta, int early_term,
                         int32_t *iters_used, int threads)
{
    mt_job j = {h, NULL, hard, NULL, iters_used, llr, v_out, batch, iters, algo, 0, early_term, 0, beta};
    return run_mt(j, batch, threads, h->n);
}
