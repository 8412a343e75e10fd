// ubench_barrier.hip -- design input (not part of the library): what one
// workgroup barrier costs coop3's period on gfx950.  A workgroup of NW waves
// (6 or 8, coop3's shapes; one workgroup per CU, the whole chip) runs NREP
// periods of W dependent VALU ops per wave, with and without an s_barrier
// closing each period; the difference per period is the barrier's cost
// (release latency + the waves' re-start), measured without s_memtime stamps
// inside the loop.
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/ubench_barrier tools/ubench_barrier.hip && /tmp/ubench_barrier
#include <hip/hip_runtime.h>

#include <cstdio>

constexpr int NREP = 2048;

__device__ unsigned long long stamp()
{
    unsigned long long t;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    return t;
}

// W dependent v_add_u32 (4 cycles each at wave64) per period; BAR: s_barrier
// after each; LDSW: one ds_write_b32 before the barrier (its lgkmcnt drain)
template <int W, bool BAR, bool LDSW>
__global__ void __launch_bounds__(512) k(unsigned long long *out, int *res, int b)
{
    __shared__ int sink[512];
    int r = threadIdx.x;
    __syncthreads();
    const unsigned long long t0 = stamp();
    for (int i = 0; i < NREP; i++) {
#pragma unroll
        for (int j = 0; j < W; j++) asm volatile("v_add_u32 %0, %0, %1" : "+v"(r) : "v"(b));
        if constexpr (LDSW) sink[threadIdx.x] = r;
        if constexpr (BAR) __syncthreads();
        else asm volatile("" ::: "memory");
    }
    const unsigned long long t1 = stamp();
    if ((threadIdx.x & 63) == 0) out[blockIdx.x * 8 + (threadIdx.x >> 6)] = t1 - t0;
    res[blockIdx.x * blockDim.x + threadIdx.x] = r + sink[threadIdx.x ^ 1];
}

template <int W, bool BAR, bool LDSW>
double run(int nw)
{
    const int grid = 256;
    unsigned long long *d;
    int *r;
    (void)hipMalloc(&d, grid * 8 * sizeof(unsigned long long));
    (void)hipMalloc(&r, grid * 512 * sizeof(int));
    for (int rep = 0; rep < 2; rep++) hipLaunchKernelGGL((k<W, BAR, LDSW>), dim3(grid), dim3(64 * nw), 0, 0, d, r, 1);
    (void)hipDeviceSynchronize();
    unsigned long long h[256 * 8];
    (void)hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    double s = 0;
    for (int g = 0; g < grid; g++) s += (double)h[g * 8];
    (void)hipFree(d);
    (void)hipFree(r);
    return s / grid / NREP;
}

int main()
{
    for (int nw : {6, 8}) {
        const double a0 = run<64, false, false>(nw), b0 = run<64, true, false>(nw), c0 = run<64, true, true>(nw);
        const double a1 = run<256, false, false>(nw), b1 = run<256, true, false>(nw), c1 = run<256, true, true>(nw);
        printf("%d waves: W=64  no barrier %.0f, barrier %.0f (+%.0f), + LDS write %.0f (+%.0f) cycles per period\n", nw, a0,
               b0, b0 - a0, c0, c0 - a0);
        printf("%d waves: W=256 no barrier %.0f, barrier %.0f (+%.0f), + LDS write %.0f (+%.0f) cycles per period\n", nw, a1,
               b1, b1 - a1, c1, c1 - a1);
    }
    return 0;
}
