// chain_probe.hip -- cycles per staircase-chain step (coop2.hip chain wave)
// for one wave alone on a CU: the kernel's 5-instruction step (clamped copy,
// two v_mad_i32_i24, two v_med3_i32) with its constants in VGPRs, 16 or 64
// active lanes.  Design input, not part of the library.  Build + run on the
// GPU box:
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/chain_probe tools/chain_probe.hip && /tmp/chain_probe
#include <hip/hip_runtime.h>

#include <cstdio>

constexpr int NSTEP = 24, NREP = 64;

__device__ unsigned long long stamp()
{
    unsigned long long t;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    return t;
}

template <int KIND>
__global__ void __launch_bounds__(64) probe(unsigned long long *out, int *sink, const int *cst, int lanes)
{
    const int lane = threadIdx.x;
    int q[NSTEP][6];
#pragma unroll
    for (int i = 0; i < NSTEP; i++)
#pragma unroll
        for (int j = 0; j < 6; j++) q[i][j] = cst[(i * 6 + j) * 64 + lane];
    int Y = lane, acc = 0;
    const int lo = -127, hi = 127;
    unsigned long long t0 = 0;
    if (lane < lanes) {
        t0 = stamp();
        for (int r = 0; r < NREP; r++) {
#pragma unroll
            for (int i = 0; i < NSTEP; i++) {
                int x, p, qq;
                if constexpr (KIND == 0) {   // the kernel's step
                    asm volatile("v_med3_i32 %1, %0, %8, %9\n\t"
                                 "v_mad_i32_i24 %2, %0, %4, %5\n\t"
                                 "v_mad_i32_i24 %3, %0, %4, %6\n\t"
                                 "v_med3_i32 %2, %2, %7, %3\n\t"
                                 "v_med3_i32 %0, %2, %10, %11"
                                 : "+v"(Y), "=&v"(x), "=&v"(p), "=&v"(qq)
                                 : "v"(q[i][0]), "v"(q[i][1]), "v"(q[i][2]), "v"(q[i][3]), "v"(lo), "v"(hi),
                                   "v"(q[i][4]), "v"(q[i][5]));
                } else {   // sign-normalised: two v_add_u32 instead of the mads
                    asm volatile("v_med3_i32 %1, %0, %8, %9\n\t"
                                 "v_add_u32 %2, %0, %5\n\t"
                                 "v_add_u32 %3, %0, %6\n\t"
                                 "v_med3_i32 %2, %2, %7, %3\n\t"
                                 "v_med3_i32 %0, %2, %10, %11"
                                 : "+v"(Y), "=&v"(x), "=&v"(p), "=&v"(qq)
                                 : "v"(q[i][0]), "v"(q[i][1]), "v"(q[i][2]), "v"(q[i][3]), "v"(lo), "v"(hi),
                                   "v"(q[i][4]), "v"(q[i][5]));
                }
                acc += x;
            }
        }
    }
    const unsigned long long t1 = stamp();
    if (lane == 0) out[blockIdx.x] = t1 - t0;
    sink[blockIdx.x * blockDim.x + lane] = Y + acc;
}

template <int KIND>
void run(const char *name, int lanes)
{
    unsigned long long *d_out;
    int *d_sink, *d_cst;
    (void)hipMalloc(&d_out, 8 * sizeof(unsigned long long));
    (void)hipMalloc(&d_sink, 64 * 8 * sizeof(int));
    (void)hipMalloc(&d_cst, NSTEP * 6 * 64 * sizeof(int));
    int h_cst[NSTEP * 6 * 64];
    for (int i = 0; i < NSTEP * 6 * 64; i++) h_cst[i] = (i * 37) % 61 - 30;
    (void)hipMemcpy(d_cst, h_cst, sizeof(h_cst), hipMemcpyHostToDevice);
    hipLaunchKernelGGL(probe<KIND>, dim3(1), dim3(64), 0, 0, d_out, d_sink, d_cst, lanes);
    hipLaunchKernelGGL(probe<KIND>, dim3(1), dim3(64), 0, 0, d_out, d_sink, d_cst, lanes);
    unsigned long long h = 0;
    (void)hipMemcpy(&h, d_out, sizeof(h), hipMemcpyDeviceToHost);
    printf("%-40s lanes=%2d  cycles/step = %.2f\n", name, lanes, (double)h / (NREP * NSTEP));
    (void)hipFree(d_out);
    (void)hipFree(d_sink);
    (void)hipFree(d_cst);
}

int main()
{
    for (int lanes : {16, 64}) {
        run<0>("kernel step (med3, 2 mad24, 2 med3)", lanes);
        run<1>("add step (med3, 2 add, 2 med3)", lanes);
    }
    return 0;
}
