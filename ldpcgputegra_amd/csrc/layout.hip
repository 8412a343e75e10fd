// layout.hip -- frame-major <-> node-major transposes, hard decision, the
// synthetic AWGN channel and the error counter.
//
// Reference counterparts: Interleaver_uint8 / InvInterleaver_uint8
// (code/gpu_fixed/transpose/GPU_Transpose_uint8.cu:9-130; the inverse applies
// the hard decision x > 0 as code/x86/CTools/CTools.cpp:370 does), the GPU
// channel (code/gpu_fixed/awgn_channel/CChanel_AWGN_SIMD.cu:7-30) and
// CErrorAnalyzer::generate (code/x86/CErrorAnalyzer/CErrorAnalyzer.cpp:123-154).
//
// Transposes move 64x64 tiles through LDS: global reads are 64 contiguous
// elements per row of the source, writes 64 contiguous codewords per node row.
#include <climits>
#include <algorithm>
#include "kernels.h"

namespace {

template <typename T>
__global__ void __launch_bounds__(256) interleave_k(const T *__restrict__ src, T *__restrict__ dst, int n,
                                                    int batch, int stride)
{
    __shared__ T tile[64][65];
    const int n0 = blockIdx.x * 64, b0 = blockIdx.y * 64;
    const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;   // 64 x 4
#pragma unroll
    for (int r = 0; r < 16; r++) {
        const int b = b0 + ty + 4 * r, i = n0 + tx;
        tile[ty + 4 * r][tx] = (b < batch && i < n) ? src[(size_t)b * n + i] : (T)0;
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < 16; r++) {
        const int i = n0 + ty + 4 * r, b = b0 + tx;
        if (i < n && b < stride) dst[(size_t)i * stride + b] = tile[tx][ty + 4 * r];
    }
}

template <typename T>
__global__ void __launch_bounds__(256) deinterleave_k(const T *__restrict__ V, uint8_t *__restrict__ hard,
                                                      T *__restrict__ soft, int n, int batch, int stride)
{
    __shared__ T tile[64][65];
    const int n0 = blockIdx.x * 64, b0 = blockIdx.y * 64;
    const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
#pragma unroll
    for (int r = 0; r < 16; r++) {
        const int i = n0 + ty + 4 * r, b = b0 + tx;
        tile[ty + 4 * r][tx] = (i < n && b < batch) ? V[(size_t)i * stride + b] : (T)0;
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < 16; r++) {
        const int b = b0 + ty + 4 * r, i = n0 + tx;
        if (b < batch && i < n) {
            const T x = tile[tx][ty + 4 * r];
            if (hard) hard[(size_t)b * n + i] = (x > (T)0) ? 1 : 0;
            if (soft) soft[(size_t)b * n + i] = x;
        }
    }
}

// grouped layout (coop3): Vg[group][row][16 codewords], groups `gbytes` apart.
// A 64x64 tile is 4 groups x 64 rows: one 16-B row piece per thread, so the
// node-major side moves whole contiguous runs of 64 pieces per group.
__global__ void __launch_bounds__(256) interleave_grp_k(const int8_t *__restrict__ src, int8_t *__restrict__ dst,
                                                        int n, int batch, size_t gbytes)
{
    __shared__ int8_t tile[64][65];   // [codeword][node]
    const int n0 = blockIdx.x * 64, b0 = blockIdx.y * 64;
    const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
#pragma unroll
    for (int r = 0; r < 16; r++) {
        const int b = b0 + ty + 4 * r, i = n0 + tx;
        tile[ty + 4 * r][tx] = (b < batch && i < n) ? src[(size_t)b * n + i] : (int8_t)0;
    }
    __syncthreads();
    const int gq = threadIdx.x >> 6, ni = threadIdx.x & 63;   // group of the tile, node
    if (n0 + ni < n) {
        uint32_t w[4];
#pragma unroll
        for (int d = 0; d < 4; d++) {
            w[d] = 0;
#pragma unroll
            for (int j = 0; j < 4; j++) w[d] |= (uint32_t)(uint8_t)tile[16 * gq + 4 * d + j][ni] << (8 * j);
        }
        *(uint4 *)(dst + (size_t)(b0 / 16 + gq) * gbytes + (size_t)(n0 + ni) * 16) = make_uint4(w[0], w[1], w[2], w[3]);
    }
}

// the input transpose with 16-B loads on the frame-major side (n % 16 == 0,
// a 16-B aligned buffer: every DVB-S2 code): one uint4 load per thread
// instead of 16 byte loads (the byte version ran at 1.6 TB/s: 336 vs 135 us
// per 4096 DVB-S2 codewords; the same change on the output side measured
// 122 vs 114 us and was dropped)
__global__ void __launch_bounds__(256) interleave_grp_vec_k(const int8_t *__restrict__ src, int8_t *__restrict__ dst,
                                                            int n, int batch, size_t gbytes)
{
    __shared__ uint4 tile4[64][4];   // [codeword][16-node chunk]: row-contiguous 64 B
    const int n0 = blockIdx.x * 64, b0 = blockIdx.y * 64;
    {
        const int r = threadIdx.x >> 2, c = threadIdx.x & 3, b = b0 + r, i = n0 + 16 * c;
        tile4[r][c] = (b < batch && i < n) ? *(const uint4 *)(src + (size_t)b * n + i) : make_uint4(0, 0, 0, 0);
    }
    __syncthreads();
    const int8_t(*tile)[64] = (const int8_t(*)[64])&tile4[0][0];
    const int gq = threadIdx.x >> 6, ni = threadIdx.x & 63;   // group of the tile, node
    if (n0 + ni < n) {
        uint32_t w[4];
#pragma unroll
        for (int d = 0; d < 4; d++) {
            w[d] = 0;
#pragma unroll
            for (int j = 0; j < 4; j++) w[d] |= (uint32_t)(uint8_t)tile[16 * gq + 4 * d + j][ni] << (8 * j);
        }
        *(uint4 *)(dst + (size_t)(b0 / 16 + gq) * gbytes + (size_t)(n0 + ni) * 16) = make_uint4(w[0], w[1], w[2], w[3]);
    }
}

__global__ void __launch_bounds__(256) deinterleave_grp_k(const int8_t *__restrict__ V, uint8_t *__restrict__ hard,
                                                          int8_t *__restrict__ soft, int n, int batch, size_t gbytes)
{
    __shared__ int8_t tile[64][65];   // [codeword][node]
    const int n0 = blockIdx.x * 64, b0 = blockIdx.y * 64;
    const int gq = threadIdx.x >> 6, ni = threadIdx.x & 63;
    if (n0 + ni < n) {
        const uint4 y = *(const uint4 *)(V + (size_t)(b0 / 16 + gq) * gbytes + (size_t)(n0 + ni) * 16);
        const uint32_t w[4] = {y.x, y.y, y.z, y.w};
#pragma unroll
        for (int d = 0; d < 4; d++)
#pragma unroll
            for (int j = 0; j < 4; j++) tile[16 * gq + 4 * d + j][ni] = (int8_t)(w[d] >> (8 * j));
    }
    __syncthreads();
    const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
#pragma unroll
    for (int r = 0; r < 16; r++) {
        const int b = b0 + ty + 4 * r, i = n0 + tx;
        if (b < batch && i < n) {
            const int8_t x = tile[ty + 4 * r][tx];
            if (hard) hard[(size_t)b * n + i] = x > 0 ? 1 : 0;
            if (soft) soft[(size_t)b * n + i] = x;
        }
    }
}

// node-major input (the reference's interleaved layout, Interleaver_uint8's
// output: LLR of node i, codeword b at src[i * ld + b]) -> the decoder's
// 16-codeword pieces: piece (group g, node i) = codewords 16g..16g+15 of node
// i, stored at dst + g * gstep + i * rstep (grouped layout: gstep = the group
// block, rstep = 16; row layout: gstep = 16, rstep = the row pitch).  No
// transpose: a wave reads 16 nodes x 4 groups (64 contiguous bytes per node)
// and writes 4 runs of 16 contiguous pieces.  Codewords >= batch are zero.
__global__ void __launch_bounds__(256) nm_pieces_k(const int8_t *__restrict__ src, size_t ld, int n, int batch,
                                                   int groups, int8_t *__restrict__ dst, size_t gstep, size_t rstep,
                                                   int vec)
{
    const int g = blockIdx.y * 4 + (threadIdx.x & 3), i = blockIdx.x * 64 + (threadIdx.x >> 2);
    if (g >= groups || i >= n) return;
    const int b0 = 16 * g;
    const int8_t *p = src + (size_t)i * ld + b0;
    uint4 v;
    if (vec && b0 + 16 <= batch) {
        v = *(const uint4 *)p;
    } else {
        uint32_t w[4] = {0, 0, 0, 0};
#pragma unroll
        for (int j = 0; j < 16; j++)
            if (b0 + j < batch) w[j >> 2] |= (uint32_t)(uint8_t)p[j] << (8 * (j & 3));
        v = make_uint4(w[0], w[1], w[2], w[3]);
    }
    *(uint4 *)(dst + (size_t)g * gstep + (size_t)i * rstep) = v;
}

__global__ void __launch_bounds__(256) awgn_i8_k(int8_t *__restrict__ llr, int n, int batch, uint64_t first_cw,
                                                 uint64_t seed, AwgnTable t, const uint8_t *__restrict__ cw)
{
    __shared__ uint32_t th[64];
    if (threadIdx.x < 64) th[threadIdx.x] = t.t[threadIdx.x];
    __syncthreads();
    const int sat = (int)th[63];
    const uint64_t key = seed * 0xD1B54A32D192ED03ull;
    const size_t total = (size_t)n * batch;
    for (size_t e = (size_t)blockIdx.x * 256 + threadIdx.x; e < total; e += (size_t)gridDim.x * 256) {
        const size_t b = e / n, i = e - b * n;
        const uint64_t idx = (first_cw + b) * (uint64_t)n + i;
        const uint32_t u = (uint32_t)(splitmix64(idx ^ key) >> 32);
        int cnt = 0;
        for (int k = 0; k < 2 * sat; k++) cnt += (u >= th[k]);
        int q = cnt - sat;
        if (cw && cw[e]) q = -q;
        llr[e] = (int8_t)q;
    }
}

// one wave per codeword: hard decisions are 0/1 bytes, so the errors of a
// dword are popcount((h ^ r) & 0x01010101); dword loads when the row allows
__global__ void __launch_bounds__(64) count_errors_k(const uint8_t *__restrict__ hard, int n, int k,
                                                     const uint8_t *__restrict__ ref,
                                                     unsigned long long *counts)
{
    const int b = blockIdx.x;
    const uint8_t *h = hard + (size_t)b * n;
    const uint8_t *r = ref ? ref + (size_t)b * n : nullptr;
    int errs = 0;
    if ((n & 15) == 0 && (k & 15) == 0 && ((uintptr_t)hard & 15) == 0 && ((uintptr_t)ref & 15) == 0) {
        // 16-B loads, 4 in flight per lane (DVB-S2 r1/2: k = 32400 = 2025 x 16)
        const uint4 *h16 = (const uint4 *)h, *r16 = (const uint4 *)r;
        const uint4 z = make_uint4(0, 0, 0, 0);
        auto e16 = [](uint4 a, uint4 q) {
            return __builtin_popcount((a.x ^ q.x) & 0x01010101u) + __builtin_popcount((a.y ^ q.y) & 0x01010101u) +
                   __builtin_popcount((a.z ^ q.z) & 0x01010101u) + __builtin_popcount((a.w ^ q.w) & 0x01010101u);
        };
        const int m = k / 16;
#pragma unroll 4
        for (int i = threadIdx.x; i < m; i += 64) errs += e16(h16[i], r16 ? r16[i] : z);
    } else if ((n & 3) == 0 && (k & 3) == 0) {
        const uint32_t *h4 = (const uint32_t *)h, *r4 = (const uint32_t *)r;
        for (int i = threadIdx.x; i < k / 4; i += 64)
            errs += __builtin_popcount((h4[i] ^ (r4 ? r4[i] : 0u)) & 0x01010101u);
    } else {
        for (int i = threadIdx.x; i < k; i += 64) errs += (h[i] != (r ? r[i] : 0));
    }
    for (int off = 32; off > 0; off >>= 1) errs += __shfl_xor(errs, off);
    if (threadIdx.x == 0 && errs) {
        atomicAdd(&counts[0], (unsigned long long)errs);
        atomicAdd(&counts[1], 1ull);
    }
}

// one block per row; 16-B vector copies when the row allows it
__global__ void __launch_bounds__(256) copy_rows_k(const uint8_t *__restrict__ src, uint8_t *__restrict__ dst,
                                                   const int32_t *__restrict__ idx, int row_bytes, int scatter)
{
    const int r = blockIdx.x;
    const size_t so = (size_t)(scatter ? r : idx[r]) * row_bytes;
    const size_t dof = (size_t)(scatter ? idx[r] : r) * row_bytes;
    if ((row_bytes & 15) == 0 && ((uintptr_t)src & 15) == 0 && ((uintptr_t)dst & 15) == 0) {
        const uint4 *s4 = (const uint4 *)(src + so);
        uint4 *d4 = (uint4 *)(dst + dof);
        for (int i = threadIdx.x; i < row_bytes / 16; i += 256) d4[i] = s4[i];
    } else {
        for (int i = threadIdx.x; i < row_bytes; i += 256) dst[dof + i] = src[so + i];
    }
}

// zero `width` bytes (multiple of 16) at base + r * pitch for r < rows: one
// block per row
__global__ void __launch_bounds__(256) zero_rows_k(uint8_t *__restrict__ base, size_t pitch, size_t width)
{
    uint4 *p = (uint4 *)(base + (size_t)blockIdx.x * pitch);
    for (size_t i = threadIdx.x; i < width / 16; i += 256) p[i] = make_uint4(0, 0, 0, 0);
}

inline int ok() { return hipGetLastError() == hipSuccess ? 0 : -1; }

}  // namespace

// float -> int8 LLR, CFastFixConversion::generate
// (code/x86/CFixPointConversion/CFastFixConversion.cpp:55-65): the float
// product truncated toward zero, then clamped.  x86 cvttss2si gives INT_MIN
// for NaN and for |product| >= 2^31: those clamp to sat_neg there, and here.
__global__ void __launch_bounds__(256) quantize_k(const float *__restrict__ y, int8_t *__restrict__ q, long count,
                                                  float factor, int sat_neg, int sat_pos)
{
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < count; i += (long)gridDim.x * blockDim.x) {
        const float v = factor * y[i];
        int value = (fabsf(v) < 2147483648.0f) ? (int)v : INT_MIN;
        value = value > sat_neg ? value : sat_neg;
        value = value < sat_pos ? value : sat_pos;
        q[i] = (int8_t)value;
    }
}

int launch_quantize_f32_i8(const float *y, int8_t *q, long count, int factor, int sat_neg, int sat_pos,
                           hipStream_t s)
{
    if (count <= 0) return 0;
    const long blocks = std::min<long>((count + 255) / 256, 256L * 64);
    hipLaunchKernelGGL(quantize_k, dim3((unsigned)blocks), dim3(256), 0, s, y, q, count, (float)factor, sat_neg,
                       sat_pos);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_interleave_i8(const int8_t *llr, int8_t *V, int n, int batch, int stride, hipStream_t s)
{
    dim3 g((n + 63) / 64, (stride + 63) / 64);
    hipLaunchKernelGGL(interleave_k<int8_t>, g, dim3(256), 0, s, llr, V, n, batch, stride);
    return ok();
}
int launch_interleave_f32(const float *llr, float *V, int n, int batch, int stride, hipStream_t s)
{
    dim3 g((n + 63) / 64, (stride + 63) / 64);
    hipLaunchKernelGGL(interleave_k<float>, g, dim3(256), 0, s, llr, V, n, batch, stride);
    return ok();
}
int launch_deinterleave_i8(const int8_t *V, uint8_t *hard, int8_t *soft, int n, int batch, int stride,
                           hipStream_t s)
{
    dim3 g((n + 63) / 64, (batch + 63) / 64);
    hipLaunchKernelGGL(deinterleave_k<int8_t>, g, dim3(256), 0, s, V, hard, soft, n, batch, stride);
    return ok();
}
int launch_deinterleave_f32(const float *V, uint8_t *hard, float *soft, int n, int batch, int stride,
                            hipStream_t s)
{
    dim3 g((n + 63) / 64, (batch + 63) / 64);
    hipLaunchKernelGGL(deinterleave_k<float>, g, dim3(256), 0, s, V, hard, soft, n, batch, stride);
    return ok();
}
int launch_interleave_grp_i8(const int8_t *llr, int8_t *V, int n, int batch, int stride, size_t gbytes,
                             hipStream_t s)
{
    dim3 g((n + 63) / 64, (stride + 63) / 64);
    if (n % 16 == 0 && (uintptr_t)llr % 16 == 0)
        hipLaunchKernelGGL(interleave_grp_vec_k, g, dim3(256), 0, s, llr, V, n, batch, gbytes);
    else
        hipLaunchKernelGGL(interleave_grp_k, g, dim3(256), 0, s, llr, V, n, batch, gbytes);
    return ok();
}
int launch_deinterleave_grp_i8(const int8_t *V, uint8_t *hard, int8_t *soft, int n, int batch, size_t gbytes,
                               hipStream_t s)
{
    dim3 g((n + 63) / 64, (batch + 63) / 64);
    hipLaunchKernelGGL(deinterleave_grp_k, g, dim3(256), 0, s, V, hard, soft, n, batch, gbytes);
    return ok();
}
int launch_nm_pieces_i8(const int8_t *llr, size_t ld, int n, int batch, int stride, int8_t *dst, size_t gstep,
                        size_t rstep, hipStream_t s)
{
    const int groups = stride / 16;
    const int vec = (ld % 16 == 0) && ((uintptr_t)llr % 16 == 0);
    dim3 g((n + 63) / 64, (groups + 3) / 4);
    hipLaunchKernelGGL(nm_pieces_k, g, dim3(256), 0, s, llr, ld, n, batch, groups, dst, gstep, rstep, vec);
    return ok();
}
int launch_zero_rows(void *base, size_t pitch, size_t width, int rows, hipStream_t s)
{
    if (rows <= 0 || width % 16 != 0 || ((uintptr_t)base & 15) != 0 || pitch % 16 != 0) return -1;
    hipLaunchKernelGGL(zero_rows_k, dim3(rows), dim3(256), 0, s, (uint8_t *)base, pitch, width);
    return ok();
}
int launch_awgn_i8(int8_t *llr, int n, int batch, uint64_t first_cw, uint64_t seed, const AwgnTable &t,
                   const uint8_t *codeword, hipStream_t s)
{
    size_t total = (size_t)n * batch;
    int blocks = (int)std::min<size_t>((total + 255) / 256, 8192);
    if (blocks < 1) blocks = 1;
    hipLaunchKernelGGL(awgn_i8_k, dim3(blocks), dim3(256), 0, s, llr, n, batch, first_cw, seed, t, codeword);
    return ok();
}
int launch_gather_rows(const void *src, void *dst, const int32_t *idx, int rows, int row_bytes, hipStream_t s)
{
    if (rows <= 0) return 0;
    hipLaunchKernelGGL(copy_rows_k, dim3(rows), dim3(256), 0, s, (const uint8_t *)src, (uint8_t *)dst, idx,
                       row_bytes, 0);
    return ok();
}
int launch_scatter_rows(const void *src, void *dst, const int32_t *idx, int rows, int row_bytes, hipStream_t s)
{
    if (rows <= 0) return 0;
    hipLaunchKernelGGL(copy_rows_k, dim3(rows), dim3(256), 0, s, (const uint8_t *)src, (uint8_t *)dst, idx,
                       row_bytes, 1);
    return ok();
}
int launch_count_errors(const uint8_t *hard, int n, int batch, int k, const uint8_t *ref,
                        unsigned long long *counts, hipStream_t s)
{
    if (batch <= 0) return 0;
    hipLaunchKernelGGL(count_errors_k, dim3(batch), dim3(64), 0, s, hard, n, k, ref, counts);
    return ok();
}
