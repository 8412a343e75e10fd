/*
 * ldpc_mi355x.h -- C-ABI of the MI355X layered min-sum LDPC decoder.
 *
 * This is the drop-in boundary for the reference's decode path
 * (boiseHPSim/ldpcGpuTegra).  Plain C types only: no HIP or torch types in any
 * signature (streams are passed as `void *` holding a hipStream_t).  Every
 * function returns an int status (LDPC_OK == 0, negative on error) and never
 * exits the process -- unlike the reference, which prints and calls exit(0)
 * (code/x86/CDecoder/DecoderLibrary.h:37-41, code/gpu_fixed/custom_api/
 * custom_cuda.cu:5-17).
 *
 * Entry point -> reference interface it replaces:
 *   ldpc_code_create / ldpc_code_load / ldpc_code_from_dvbs2_table
 *       -> the compile-time H table PosNoeudsVariable[] + DEG_k macros
 *          (code/x86/Constantes/constantes_sse.h:1-2,
 *           code/x86/Constantes/64800x32400.dvb-s2/constantes_sse.h:6-36)
 *   ldpc_ctx_create(code, device, max_batch)
 *       -> CGPUDecoder(nb_frames, n, k, m) + initialize()
 *          (code/gpu_fixed/decoder_template/CGPUDecoder.h:20-37) and the
 *          decoder constructors that allocate V / msg scratch
 *          (code/x86/CDecoder/template/CDecoder_fixed_SSE.cpp:23-27)
 *   ldpc_params {algo, offset, factor, var/msg range}
 *       -> CreateDecoder(type, arch, format, p_decoder, vMin, vMax, mMin, mMax)
 *          (code/x86/CDecoder/DecoderLibrary.h:44-134), setOffset
 *          (OMS/CDecoder_OMS_fixed_SSE.cpp:104-112), setFactor
 *          (NMS/CDecoder_NMS_fixed_SSE.cpp:107-111), setVarRange/setMsgRange
 *          (template/CDecoder_fixed.h:40-41)
 *   ldpc_decode_i8(ctx, llr, hard, batch, n_iter, params)
 *       -> CDecoder::decode(char var_nodes[], char Rprime_fix[], int iters)
 *          (code/x86/CDecoder/template/CDecoder.h:37), 16 frames per call
 *          there, any batch here; same frame-major layout, same 0/1 output
 *   ldpc_decode_f32(...)
 *       -> CDecoder::decode(float var_nodes[], char Rprime_fix[], int)
 *          (CDecoder.h:38; a no-op for the reference's fixed-point decoders)
 *          and CGPUDecoder::decode(float[], int[], int) (CGPUDecoder.h:31)
 *   ldpc_decode_i8_async / _f32_async
 *       -> CGPU_Decoder_*_SIMD::decode_stream
 *          (code/gpu_fixed/decoder_ms/CGPU_Decoder_MS_SIMD.cu:219-275),
 *          device pointers, caller-owned stream, no hidden sync
 *   ldpc_awgn_*  -> CChanelAWGN_MKL::configure/generate + CFastFixConversion
 *          (code/x86/CChanel/CChanelAWGN_MKL.cpp:95-143,
 *           code/x86/CFixPointConversion/CFastFixConversion.cpp:55-65) and the
 *          on-GPU channel (code/gpu_fixed/awgn_channel/CChanel_AWGN_SIMD.cu:7-30)
 *   ldpc_count_errors_async -> CErrorAnalyzer::generate
 *          (code/x86/CErrorAnalyzer/CErrorAnalyzer.cpp:123-154)
 *
 * Threading: a ldpc_code is immutable and may be shared by any number of
 * contexts/threads.  A ldpc_ctx owns device scratch and is not re-entrant
 * (like the reference decoder objects); use one per host thread / stream.
 */
#ifndef LDPC_MI355X_H
#define LDPC_MI355X_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define LDPC_ABI_VERSION 1

enum {
    LDPC_OK = 0,
    LDPC_EINVAL = -1,      /* bad argument, H table, or saturation ranges */
    LDPC_EUNSUPPORTED = -2,/* valid request the reference would reject (exit) */
    LDPC_EDEVICE = -3,     /* HIP error; see ldpc_last_error() */
    LDPC_ENOMEM = -4,      /* host or device allocation failed */
    LDPC_EIO = -5          /* file not found / malformed table file */
};

enum {
    LDPC_ALGO_OMS = 0,     /* offset min-sum   (CDecoder_OMS_fixed_SSE) */
    LDPC_ALGO_NMS = 1,     /* normalised min-sum (CDecoder_NMS_fixed_SSE) */
    LDPC_ALGO_MS = 2       /* plain min-sum == OMS with offset 0 */
};

typedef struct ldpc_code ldpc_code;
typedef struct ldpc_ctx ldpc_ctx;

typedef struct {
    int algo;        /* LDPC_ALGO_*                                  default OMS */
    int offset;      /* int8 OMS offset (setOffset)                  default 1   */
    int factor;      /* int8 NMS factor, scaled by 1/32 (setFactor)  default 29  */
    float beta;      /* float path: OMS offset or NMS factor         default 0.15*/
    int var_min;     /* setVarRange(min, max)                   default -127,127 */
    int var_max;
    int msg_min;     /* setMsgRange(min, max)                   default -31, 31  */
    int msg_max;
    int early_term;  /* stop a codeword once H*x == 0 (0 = exact n_iter); the
                        DVB-S2 r1/2 kernel decodes batches >= 8192 in stages,
                        compacting the codewords still decoding every few
                        iterations (LDPC_COOP3_ET_K / _STEP / _STAGE_MIN) */
} ldpc_params;

/* ---- errors / version ------------------------------------------------ */
void ldpc_params_default(ldpc_params *p);
const char *ldpc_strerror(int status);
const char *ldpc_last_error(void);          /* thread-local detail of the last error */
int ldpc_abi_version(void);
int ldpc_device_count(int *count);

/* ---- code tables ----------------------------------------------------- */
/* Layered H: checks in schedule order, in n_groups runs of equal degree
 * (group g = group_cnt[g] checks of degree group_deg[g]); edge_var[E] lists
 * each check's variables.  Group 0 vs later groups matters for bit-exactness
 * (reference quirk). */
int ldpc_code_create(int n, int m, int n_groups, const int *group_deg, const int *group_cnt,
                     const uint32_t *edge_var, ldpc_code **out);
/* DVB-S2 IRA code from its Annex-B address table: row r lists row_len[r]
 * parity addresses (concatenated in row_addr).  Layered order as the
 * reference tables: checks 1..M-1 (info vars ascending, K+i-1, K+i), then
 * check 0 (info ascending, K). */
int ldpc_code_from_dvbs2_table(int n, int k_info, int n_rows, const int *row_len,
                               const int *row_addr, ldpc_code **out);
/* Load a ".ldpc" binary table or a DVB-S2 ".txt" address table. */
int ldpc_code_load(const char *path, ldpc_code **out);
int ldpc_code_info(const ldpc_code *h, int *n, int *m, int *e, int *n_groups, int *max_deg);
int ldpc_code_edges(const ldpc_code *h, uint32_t *edge_var, int *group_deg, int *group_cnt);
/* 1 if the layered schedule has the DVB-S2 staircase chain (fast kernel). */
int ldpc_code_plan_info(const ldpc_code *h, int *staircase, int *n_windows, int *min_hazard);
/* Window schedule of the windowed2 kernel for S checks per window and
 * read-ahead P: writes up to max_windows (first check, count) pairs and the
 * total count (0 when the code has no staircase schedule). */
int ldpc_code_window_plan(const ldpc_code *h, int S, int P, int *first, int *count, int max_windows,
                          int *n_windows);
/* Window schedule of the workgroup-cooperative kernel (S checks per window,
 * prefetch depth R windows): (first check, count) per window -- count 0 is
 * an empty window -- the window holding the tail check and the number of
 * info-edge reads per iteration forwarded through LDS.  n_windows = 0 when
 * the code has no such schedule. */
int ldpc_code_coop_plan(const ldpc_code *h, int S, int R, int *first, int *count, int max_windows,
                        int *n_windows, int *tail, int *n_fwd);
/* Same with the window distance rule of the kernel: dist = 1 (coop: consecutive
 * windows share no information variable) or 2 (coop2: nor do windows two
 * apart; reads written dist+1 .. R+dist windows earlier are forwarded). */
int ldpc_code_coop_plan_dist(const ldpc_code *h, int S, int R, int dist, int *first, int *count, int max_windows,
                             int *n_windows, int *tail, int *n_fwd);
/* Line cache of the DVB-S2 r1/2 kernel (kernel 8, coop3): the information
 * rows move between HBM and LDS as 128-B lines (8 rows x 16 codewords) on a
 * static plan checked by replaying it.  slots: LDS line slots the plan uses
 * (0 when the code has no coop3 schedule), max_slots: what the kernel has,
 * residencies: line loads per iteration, prologue / epilogue: lines filled /
 * written back at a segment start / end.  (Introspection for tests; replaces
 * no reference interface.) */
int ldpc_code_coop3_lc_info(const ldpc_code *h, int *slots, int *max_slots, int *residencies, int *prologue,
                            int *epilogue);
/* The line cache's modelled LDS bank conflicts: extra LDS cycles per
 * iteration and workgroup of coop3's pre reads / post writes of the line
 * cache with the planner's per-residency XOR swizzle (swizzled) and with
 * every line unswizzled (plain); 0 / 0 when the code has no coop3 schedule.
 * (Introspection for tests.) */
int ldpc_code_coop3_lc_banks(const ldpc_code *h, long long *swizzled, long long *plain);
/* Layer plan of the LDS-resident kernel (kernel 7): maximal runs of
 * consecutive same-group checks sharing no variable (one block row of a
 * quasi-cyclic code).  lds_i8 / lds_f32: 1 if a codeword's state fits the
 * kernel's LDS budget for that element type. */
int ldpc_code_layer_info(const ldpc_code *h, int *n_layers, int *max_width, int *lds_i8, int *lds_f32);
void ldpc_code_destroy(ldpc_code *h);

/* ---- decoder context --------------------------------------------------- */
/* device >= 0: a GPU context on that HIP device.  device = -1: a host context
 * (no GPU needed): ldpc_decode_i8 / ldpc_decode_f32 /
 * ldpc_quantize_f32_i8 run on the CPU (AVX2 int8 over blocks of 32 codewords
 * on all host threads, LDPC_HOST_THREADS to cap them; the same bit-exact
 * results as the GPU kernels), the device-buffer entry points return
 * LDPC_EUNSUPPORTED and ldpc_ctx_last_kernel reports 10. */
int ldpc_ctx_create(const ldpc_code *h, int device, int max_batch, ldpc_ctx **out);
void ldpc_ctx_destroy(ldpc_ctx *ctx);
int ldpc_ctx_stream(ldpc_ctx *ctx, void **hip_stream);
/* Select kernel family: 0 = auto, 1 = generic (per-edge messages),
 * 2 = windowed layered kernel (compressed messages), 3 = windowed2 (S = 16),
 * 5 = workgroup-cooperative DVB-S2 kernel (coop),
 * 7 = LDS-resident short-code kernel (whole state in LDS; int8 and float),
 * 8 = coop3 (DVB-S2 first-group degree 7: slab waves doing pre + post, i16 chain),
 * 9 = ldsep (float, short QC codes: one wave per codeword, one lane per edge;
 *     the automatic choice for float decodes of the codes it fits),
 * 11 = stairf (float, DVB-S2 staircase codes: S consecutive checks of 64/S
 *     codewords per wave, the staircase chain by DPP; the automatic choice for
 *     float decodes of those codes, early termination by one launch per
 *     iteration + a syndrome pass).
 * 4 and 6 (windowed2 S = 32, coop2) were superseded and are rejected
 * with LDPC_EUNSUPPORTED. */
int ldpc_ctx_set_kernel(ldpc_ctx *ctx, int kernel);
int ldpc_ctx_get_kernel(ldpc_ctx *ctx, int *kernel);
/* Kernel family the last decode actually ran (1 generic, 2 windowed,
 * 3 windowed2 S=16, 5 coop, 7 lds, 8 coop3, 9 ldsep, 10 the host decoder of a
 * device -1 context, 11 stairf; 0 before the first decode). */
int ldpc_ctx_last_kernel(ldpc_ctx *ctx, int *kernel);
/* The fastest kernel of this code that the last automatic selection could
 * not use for the call's parameters (8: coop3, 5: coop -- they take OMS / MS
 * with msg_max <= 63 and var range +-127), 0 when none was skipped. */
int ldpc_ctx_last_skipped(ldpc_ctx *ctx, int *kernel);
/* Early termination of the last decode on coop3 (kernel 8): the iterations of
 * its first stage when it ran staged (batches >= LDPC_COOP3_ET_STAGE_MIN, default
 * 8192 codewords: the codewords still decoding compacted every
 * LDPC_COOP3_ET_STEP iterations), 0 when it ran as one launch. */
int ldpc_ctx_last_et_stage(ldpc_ctx *ctx, int *first_stage_iters);
/* Kernel timing (bench / profiling): when enabled, every decode records HIP
 * events around the decode kernel on the stream it is launched on;
 * ldpc_ctx_kernel_time returns the summed kernel time and launch count since
 * the last reset (it waits for the recorded events). */
int ldpc_ctx_profile(ldpc_ctx *ctx, int enable);
int ldpc_ctx_kernel_time(ldpc_ctx *ctx, double *total_ms, int *launches, int reset);

/* Host buffers, synchronous, frame-major [batch][N]; hard = (V > 0).
 * A large batch (>= 64 MB of LLRs) is decoded in chunks (LDPC_HOST_CHUNKS,
 * default 2, >= 256 codewords each) on the context's copy/decode lanes, so
 * the PCIe copies of one chunk overlap the decode of the other (decode_stream's streams,
 * code/gpu_fixed/decoder_ms/CGPU_Decoder_MS_SIMD.cu:219-275).  With buffers
 * from ldpc_host_alloc the copies are asynchronous DMA. */
int ldpc_decode_i8(ldpc_ctx *ctx, const int8_t *llr, uint8_t *hard, int batch, int n_iter,
                   const ldpc_params *p);
int ldpc_decode_f32(ldpc_ctx *ctx, const float *llr, uint8_t *hard, int batch, int n_iter,
                    const ldpc_params *p);

/* Host buffers, asynchronous: enqueue H2D(llr) -> decode -> D2H(hard) on
 * hip_stream (NULL: the null stream) and return -- the reference's "W streams
 * x F frames in flight" model (paper/ldpcGpuTegra.tex:279-289;
 * CGPU_Decoder_MS_SIMD::decode_stream, code/gpu_fixed/decoder_ms/
 * CGPU_Decoder_MS_SIMD.cu:219-275, without its blocking copies).  llr / hard
 * should be page-locked (ldpc_host_alloc): pageable buffers make the copies
 * synchronous.  The context's device staging and scratch are reused by its
 * next call: each call records an event of the context's own after its D2H
 * copy, and the next call's stream waits for that event before reusing them
 * (so calls on one context may use different streams, but they serialise);
 * two contexts keep two batches in flight (H2D of batch k+1 and D2H of batch
 * k-1 under the decode of batch k).  ldpc_ctx_synchronize (and
 * ldpc_ctx_destroy) wait on that event, never on the caller's stream; hard is
 * valid after it. */
int ldpc_decode_i8_host_async(ldpc_ctx *ctx, void *hip_stream, const int8_t *llr, uint8_t *hard, int batch,
                              int n_iter, const ldpc_params *p);
int ldpc_decode_f32_host_async(ldpc_ctx *ctx, void *hip_stream, const float *llr, uint8_t *hard, int batch,
                               int n_iter, const ldpc_params *p);
int ldpc_ctx_synchronize(ldpc_ctx *ctx);

/* Page-locked host memory for the host-buffer API, replacing the
 * reference's CUDA_MALLOC_HOST (code/gpu_fixed/custom_api/custom_cuda.cu:33). */
int ldpc_host_alloc(void **ptr, size_t bytes);
void ldpc_host_free(void *ptr);

/* Device buffers, asynchronous on `hip_stream`.  NULL means HIP's null
 * stream, i.e. the legacy default stream, ordered with all blocking streams
 * (the reference's decode_stream callers, code/gpu_fixed/test.cpp:347-393, and
 * torch's default stream); the context's own non-blocking stream
 * (ldpc_ctx_stream) is used only when passed explicitly.
 * soft (optional): final V per bit; iters_used (optional): per codeword. */
int ldpc_decode_i8_async(ldpc_ctx *ctx, void *hip_stream, const int8_t *d_llr, uint8_t *d_hard,
                         int8_t *d_soft, int32_t *d_iters_used, int batch, int n_iter,
                         const ldpc_params *p);
int ldpc_decode_f32_async(ldpc_ctx *ctx, void *hip_stream, const float *d_llr, uint8_t *d_hard,
                          float *d_soft, int32_t *d_iters_used, int batch, int n_iter,
                          const ldpc_params *p);
/* Node-major device input: the LLR of bit i of codeword b at d_llr[i * ld + b]
 * (ld >= batch), the interleaved layout the reference's kernels run on
 * (Interleaver_uint8, code/gpu_fixed/transpose/GPU_Transpose_uint8.cu:80-130)
 * and that CGPU_Decoder_MS_SIMD_v2::decode takes from its caller
 * (code/gpu_fixed/decoder_oms_v2/CGPU_Decoder_MS_SIMD_v2.cu:120-251).  Same
 * results as ldpc_decode_i8_async on the transposed input; d_hard / d_soft
 * are frame-major [batch][N], as that decoder returns them. */
int ldpc_decode_i8_nm_async(ldpc_ctx *ctx, void *hip_stream, const int8_t *d_llr, size_t ld, uint8_t *d_hard,
                            int8_t *d_soft, int32_t *d_iters_used, int batch, int n_iter,
                            const ldpc_params *p);

/* ---- mixed-rate batches (BASELINE config 5) ---------------------------- */
/* A batch whose codewords use different codes of equal length N (e.g. the
 * DVB-S2 normal-frame rates).  One decoder context per code; a decode groups
 * the codewords by code id, runs the per-code decodes concurrently on their
 * own streams (forked from / joined back to the caller's stream) and writes
 * hard decisions (and iterations used) back in batch order.  The reference
 * has one compile-time code per binary (code/x86/Constantes/constantes_sse.h). */
typedef struct ldpc_mixed ldpc_mixed;
int ldpc_mixed_create(const ldpc_code *const *codes, int n_codes, int device, int max_batch, ldpc_mixed **out);
void ldpc_mixed_destroy(ldpc_mixed *mx);
/* code_id: HOST array [batch] of indices into `codes`; d_llr/d_hard [batch][N]. */
int ldpc_decode_i8_mixed_async(ldpc_mixed *mx, void *hip_stream, const int8_t *d_llr, uint8_t *d_hard,
                               int32_t *d_iters_used, const int32_t *code_id, int batch, int n_iter,
                               const ldpc_params *p);
/* Kernel family the last mixed decode ran for code `code_index` (numbering of
 * ldpc_ctx_last_kernel; 0 if that code had no codewords in any decode yet). */
int ldpc_mixed_last_kernel(ldpc_mixed *mx, int code_index, int *kernel);
/* ldpc_ctx_last_et_stage of code `code_index`'s context. */
int ldpc_mixed_last_et_stage(ldpc_mixed *mx, int code_index, int *first_stage_iters);
/* Per-code decode-kernel timing (ldpc_ctx_profile / ldpc_ctx_kernel_time of
 * the code's context): the decode launches only, not the gather / scatter. */
int ldpc_mixed_profile(ldpc_mixed *mx, int enable);
int ldpc_mixed_kernel_time(ldpc_mixed *mx, int code_index, double *total_ms, int *launches, int reset);

/* DVB-S2 IRA encoder (codes built from an Annex-B table), as the
 * reference's GenericEncoder::encode (code/x86/CEncoder/GenericEncoder.cpp:38-78):
 * info [batch][K] 0/1 -> codeword [batch][N] = [info, parity]. */
int ldpc_dvbs2_encode(const ldpc_code *h, const uint8_t *info, uint8_t *codeword, int batch);

/* ---- synthetic channel -------------------------------------------------- */
/* sigma = sqrt(10^(-(EbN0 + 10 log10(rate))/10) / 2)  (CChanelAWGN_MKL.cpp:102-105) */
double ldpc_awgn_sigma(double ebn0_db, double rate);
/* the same with the reference's es_n0 option (:97-104): es_n0 != 0 reads
 * snr_db as Es/N0 of a 2-bit (QPSK) symbol, Eb/N0 = Es/N0 - 10 log10(2 rate) */
double ldpc_awgn_sigma_ex(double snr_db, double rate, int es_n0);
/* Threshold table (63 entries) for the integer-exact quantised AWGN generator:
 * q = clamp(trunc(factor*y), -sat, sat), y = -1 + sigma*z (bit 0). */
int ldpc_awgn_i8_table(double sigma, int factor, int sat, uint32_t *table /*[64]*/);
/* General channel of CChanelAWGN_MKL::generate (:127-143): y = +-amp + sigma*z
 * (amp 1 for BPSK, 0.707106781 for QPSK, one bit per real dimension) scaled by
 * norm (1, or 2 / sigma^2 with the reference's normalize option, :114-121),
 * then q = clamp(trunc(factor * y), -sat, sat); the same generators
 * (ldpc_awgn_i8_host / _async) draw from it. */
int ldpc_awgn_i8_table_ex(double sigma, double amp, double norm, int factor, int sat, uint32_t *table /*[64]*/);
/* llr[b][i] for codewords first_cw .. first_cw+batch-1; codeword bits
 * (0/1, [batch][N]) or NULL for the all-zero codeword. */
int ldpc_awgn_i8_host(int n, int batch, uint64_t first_cw, uint64_t seed, const uint32_t *table,
                      const uint8_t *codeword, int8_t *llr);
int ldpc_awgn_i8_async(ldpc_ctx *ctx, void *hip_stream, int8_t *d_llr, int batch,
                       uint64_t first_cw, uint64_t seed, const uint32_t *table,
                       const uint8_t *d_codeword);
/* float -> int8 LLR conversion, replacing CFastFixConversion::generate
 * (code/x86/CFixPointConversion/CFastFixConversion.cpp:55-65) and the GPU
 * converter (code/gpu_fixed/decoder_template/GPU_Scheduled_functions.cu:54-62):
 *   q[i] = clamp((int)((float)factor * y[i]), sat_neg, sat_pos)
 * (int) truncates toward zero; NaN and |product| >= 2^31 give sat_neg, as
 * x86 cvttss2si does.  factor >= 1, -128 <= sat_neg <= sat_pos <= 127
 * (the reference runs factor 8, saturation -31 / +31).
 * _async: device buffers on hip_stream; the plain form: host buffers,
 * synchronous, on the context's stream. */
int ldpc_quantize_f32_i8_async(ldpc_ctx *ctx, void *hip_stream, const float *d_y, int8_t *d_q, long count,
                               int factor, int sat_neg, int sat_pos);
int ldpc_quantize_f32_i8(ldpc_ctx *ctx, const float *y, int8_t *q, long count, int factor, int sat_neg,
                         int sat_pos);
/* Count bit errors over the first k positions of each codeword vs d_ref
 * (NULL = all-zero); d_counts[0] += bit errors, d_counts[1] += frame errors. */
int ldpc_count_errors_async(ldpc_ctx *ctx, void *hip_stream, const uint8_t *d_hard, int batch,
                           int k, const uint8_t *d_ref, unsigned long long *d_counts);
/* Decode and count in one call: ldpc_decode_*_async followed by
 * ldpc_count_errors_async over d_hard (required) -- the reference's
 * decode + CErrorAnalyzer::generate pair (code/x86/main_p.cpp:511-540,
 * CErrorAnalyzer.cpp:123-154).  The edge-parallel float kernel (9) counts in
 * its own epilogue (no second launch); the others launch the count after. */
int ldpc_decode_i8_count_async(ldpc_ctx *ctx, void *hip_stream, const int8_t *d_llr, uint8_t *d_hard,
                               int8_t *d_soft, int32_t *d_iters_used, int batch, int n_iter, const ldpc_params *p,
                               int k, const uint8_t *d_ref, unsigned long long *d_counts);
int ldpc_decode_f32_count_async(ldpc_ctx *ctx, void *hip_stream, const float *d_llr, uint8_t *d_hard,
                                float *d_soft, int32_t *d_iters_used, int batch, int n_iter, const ldpc_params *p,
                                int k, const uint8_t *d_ref, unsigned long long *d_counts);

#ifdef __cplusplus
}
#endif
#endif /* LDPC_MI355X_H */
