// valu_latency.hip -- cycles per VALU instruction on gfx950 for the operations
// of the staircase chain (coop.hip / coop2.hip chain wave) and the slab
// waves' packed math: dependent chains vs independent streams, one wave per
// SIMD (64 threads) and two waves per SIMD (512 threads).  Design input, not
// part of the library.  Build + run on the GPU box:
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/valu_latency tools/valu_latency.hip && /tmp/valu_latency
#include <hip/hip_runtime.h>

#include <cstdio>

#define R4(x) x x x x
#define R16(x) R4(x) R4(x) R4(x) R4(x)

constexpr int kIters = 64;   // x 16 instructions per stream

__device__ unsigned long long stamp()
{
    unsigned long long t;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    return t;
}

template <int KIND>
__global__ void probe(unsigned long long *out, int *sink, int a0)
{
    int y0 = a0 + threadIdx.x, y1 = y0 + 1, y2 = y0 + 2, y3 = y0 + 3, b = 3 + a0, c = 100 + a0;
    const unsigned long long t0 = stamp();
    for (int i = 0; i < kIters; i++) {
        if constexpr (KIND == 0)   // dependent v_med3_i32
            asm volatile(R16("v_med3_i32 %0, %0, %1, %2\n\t") : "+v"(y0) : "v"(b), "v"(c));
        if constexpr (KIND == 1)   // dependent v_mad_i32_i24
            asm volatile(R16("v_mad_i32_i24 %0, %0, %1, %2\n\t") : "+v"(y0) : "v"(b), "v"(c));
        if constexpr (KIND == 2)   // dependent v_pk_max_i16
            asm volatile(R16("v_pk_max_i16 %0, %0, %1\n\t") : "+v"(y0) : "v"(b));
        if constexpr (KIND == 3)   // dependent v_add_u32
            asm volatile(R16("v_add_u32 %0, %0, %1\n\t") : "+v"(y0) : "v"(b));
        if constexpr (KIND == 4)   // 4 independent v_med3_i32 streams
            asm volatile(R4("v_med3_i32 %0, %0, %4, %5\n\tv_med3_i32 %1, %1, %4, %5\n\t"
                            "v_med3_i32 %2, %2, %4, %5\n\tv_med3_i32 %3, %3, %4, %5\n\t")
                         : "+v"(y0), "+v"(y1), "+v"(y2), "+v"(y3)
                         : "v"(b), "v"(c));
        if constexpr (KIND == 5)   // 2 independent streams
            asm volatile(R4("v_med3_i32 %0, %0, %2, %3\n\tv_med3_i32 %1, %1, %2, %3\n\t"
                            "v_med3_i32 %0, %0, %2, %3\n\tv_med3_i32 %1, %1, %2, %3\n\t")
                         : "+v"(y0), "+v"(y1)
                         : "v"(b), "v"(c));
    }
    const unsigned long long t1 = stamp();
    if ((threadIdx.x & 63) == 0) out[blockIdx.x * 16 + (threadIdx.x >> 6)] = t1 - t0;
    sink[blockIdx.x * blockDim.x + threadIdx.x] = y0 + y1 + y2 + y3;
}

template <int KIND>
void run(const char *name, int threads)
{
    unsigned long long *d_out;
    int *d_sink;
    (void)hipMalloc(&d_out, 16 * 16 * sizeof(unsigned long long));
    (void)hipMalloc(&d_sink, 16 * 1024 * sizeof(int));
    (void)hipMemset(d_out, 0, 16 * 16 * sizeof(unsigned long long));
    hipLaunchKernelGGL(probe<KIND>, dim3(1), dim3(threads), 0, 0, d_out, d_sink, 0);   // warm-up
    hipLaunchKernelGGL(probe<KIND>, dim3(1), dim3(threads), 0, 0, d_out, d_sink, 0);
    unsigned long long h[16] = {};
    (void)hipMemcpy(h, d_out, sizeof(h), hipMemcpyDeviceToHost);
    double mean = 0;
    const int waves = threads / 64;
    for (int w = 0; w < waves; w++) mean += (double)h[w];
    mean /= waves;
    printf("%-28s waves=%d  cycles/instruction (per wave) = %.2f\n", name, waves, mean / (kIters * 16.0));
    (void)hipFree(d_out);
    (void)hipFree(d_sink);
}

int main()
{
    for (int t : {64, 512}) {
        run<0>("dependent v_med3_i32", t);
        run<1>("dependent v_mad_i32_i24", t);
        run<2>("dependent v_pk_max_i16", t);
        run<3>("dependent v_add_u32", t);
        run<5>("2 streams v_med3_i32", t);
        run<4>("4 streams v_med3_i32", t);
    }
    return 0;
}
