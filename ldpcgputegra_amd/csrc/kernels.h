// kernels.h -- launch descriptors shared between the C-ABI (capi.hip) and the
// kernel translation units.
#pragma once
#include "kernels_common.h"

struct DecodeLaunch {
    // state, codeword-fastest layout: V[N][stride], messages per kernel family
    void *V;
    void *msg;
    int stride;          // codeword slots (multiple of 64): the batch padded
    int vpitch;          // V row pitch in codewords (>= stride; coop3 may pad it)
    int batch;
    int iters;
    int is_float;
    // code (device copies)
    const uint32_t *d_edge_var;
    const int *d_group_deg;
    const int *d_group_cnt;
    int n_groups, n, m, e;
    // parameters
    int algo, param, var_min, msg_max, early;
    float beta;
    int32_t *iters_used;
    // early-termination scratch of the coop kernel ([stride] each)
    uint8_t *live;
    uint32_t *bad;
    // coop2 early termination: V snapshot taken when a codeword converges
    // (coop2 keeps iterating converged codewords that share a workgroup with
    // live ones; the snapshot is merged back before the hard decisions)
    int8_t *Vs;
    // coop3: V in the grouped layout Vg[stride / 16][rows][16 codewords],
    // vgroup bytes between groups (0: the row layout V[N][vpitch])
    size_t vgroup;
    // coop3 staged early termination: two more grouped state buffers (each
    // the size of V) and int32 scratch: selection | 2 maps | 2 iteration
    // arrays ([stride] each) | per-stage counts
    void *V2;
    int32_t *et2;
    // dynamic LDS bytes added to the windowed2 launch (mixed batches: keeps its
    // waves off the CUs of a concurrent coop3 decode, see ldpc_ctx_set_lds_pad)
    int lds_pad;
    // fused error count (ldpc_decode_*_count_async; kernels that fuse it, else
    // a count launch after the decode): bits 0 .. cnt_k-1 of each codeword vs
    // cnt_ref (NULL: all-zero), bit errors += cnt[0], frame errors += cnt[1]
    unsigned long long *cnt;
    const uint8_t *cnt_ref;
    int cnt_k;
};

int launch_generic(const DecodeLaunch &L, hipStream_t s);

// frame-major [batch][N] <-> node-major V[N][stride] (+ hard decision x > 0)
int launch_quantize_f32_i8(const float *y, int8_t *q, long count, int factor, int sat_neg, int sat_pos,
                           hipStream_t s);
int launch_interleave_i8(const int8_t *llr, int8_t *V, int n, int batch, int stride, hipStream_t s);
int launch_interleave_f32(const float *llr, float *V, int n, int batch, int stride, hipStream_t s);
int launch_deinterleave_i8(const int8_t *V, uint8_t *hard, int8_t *soft, int n, int batch, int stride,
                           hipStream_t s);
int launch_deinterleave_f32(const float *V, uint8_t *hard, float *soft, int n, int batch, int stride,
                            hipStream_t s);
// frame-major [batch][N] <-> grouped Vg[group][row][16] (group = 16 codewords, groups `gbytes` apart)
int launch_interleave_grp_i8(const int8_t *llr, int8_t *V, int n, int batch, int stride, size_t gbytes,
                             hipStream_t s);
int launch_deinterleave_grp_i8(const int8_t *V, uint8_t *hard, int8_t *soft, int n, int batch, size_t gbytes,
                               hipStream_t s);

// node-major [N][ld] (codeword fastest, the reference's interleaved layout) -> 16-codeword pieces:
// piece (g, i) at dst + g * gstep + i * rstep, g < stride / 16; codewords >= batch zero
int launch_nm_pieces_i8(const int8_t *llr, size_t ld, int n, int batch, int stride, int8_t *dst, size_t gstep,
                        size_t rstep, hipStream_t s);
// zero `width` bytes at base + r * pitch, r < rows (width, pitch multiples of 16)
int launch_zero_rows(void *base, size_t pitch, size_t width, int rows, hipStream_t s);
// rows of `row_bytes` bytes: dst[i] = src[idx[i]] (gather) / dst[idx[i]] = src[i] (scatter)
int launch_gather_rows(const void *src, void *dst, const int32_t *idx, int rows, int row_bytes, hipStream_t s);
int launch_scatter_rows(const void *src, void *dst, const int32_t *idx, int rows, int row_bytes, hipStream_t s);

int launch_awgn_i8(int8_t *llr, int n, int batch, uint64_t first_cw, uint64_t seed, const AwgnTable &t,
                   const uint8_t *codeword, hipStream_t s);
int launch_count_errors(const uint8_t *hard, int n, int batch, int k, const uint8_t *ref,
                        unsigned long long *counts, hipStream_t s);
