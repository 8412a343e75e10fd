// ubench_valu.hip -- design input (not part of the library): VALU issue
// throughput on gfx950 of the instructions the coop3 slab waves are made of,
// 8 independent streams per wave, 1 / 2 waves per SIMD (4 / 8 waves per CU).
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/ubench_valu tools/ubench_valu.hip && /tmp/ubench_valu
#include <hip/hip_runtime.h>

#include <cstdio>

constexpr int NREP = 256;

__device__ unsigned long long stamp()
{
    unsigned long long t;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    return t;
}

#define S8(OP) OP(%0) OP(%1) OP(%2) OP(%3) OP(%4) OP(%5) OP(%6) OP(%7)
#define PKSUB(r) "v_pk_sub_i16 " #r ", " #r ", %8\n\t"
#define PKMAX(r) "v_pk_max_i16 " #r ", " #r ", %8\n\t"
#define PKSUBCL(r) "v_pk_sub_i16 " #r ", " #r ", %8 clamp\n\t"
#define PERM(r) "v_perm_b32 " #r ", " #r ", %8, %9\n\t"
#define BITOP3(r) "v_bitop3_b32 " #r ", " #r ", %8, %9 bitop3:0x69\n\t"
#define ANDB(r) "v_and_b32 " #r ", " #r ", %8\n\t"
#define PKASHR(r) "v_pk_ashrrev_i16 " #r ", 15, " #r "\n\t"
#define ADDU(r) "v_add_u32 " #r ", " #r ", %8\n\t"
#define MED3(r) "v_med3_i32 " #r ", " #r ", %8, %9\n\t"
#define ANDOR(r) "v_and_or_b32 " #r ", " #r ", %8, %9\n\t"

template <int KIND>
__global__ void __launch_bounds__(512) k(unsigned long long *out, int *res, int b, int c)
{
    int r0 = threadIdx.x, r1 = r0 + 1, r2 = r0 + 2, r3 = r0 + 3, r4 = r0 + 4, r5 = r0 + 5, r6 = r0 + 6, r7 = r0 + 7;
    __syncthreads();
    const unsigned long long t0 = stamp();
    for (int i = 0; i < NREP; i++) {
#define RUN(M)                                                                                            \
    asm volatile(S8(M) : "+v"(r0), "+v"(r1), "+v"(r2), "+v"(r3), "+v"(r4), "+v"(r5), "+v"(r6), "+v"(r7) \
                 : "v"(b), "v"(c))
        if constexpr (KIND == 0) RUN(ADDU);
        if constexpr (KIND == 1) RUN(PKSUB);
        if constexpr (KIND == 2) RUN(PKSUBCL);
        if constexpr (KIND == 3) RUN(PKMAX);
        if constexpr (KIND == 4) RUN(PERM);
        if constexpr (KIND == 5) RUN(BITOP3);
        if constexpr (KIND == 6) RUN(ANDB);
        if constexpr (KIND == 7) RUN(PKASHR);
        if constexpr (KIND == 8) RUN(MED3);
        if constexpr (KIND == 9) RUN(ANDOR);
    }
    const unsigned long long t1 = stamp();
    if ((threadIdx.x & 63) == 0) out[threadIdx.x >> 6] = t1 - t0;
    res[threadIdx.x] = r0 + r1 + r2 + r3 + r4 + r5 + r6 + r7;
}

template <int KIND>
void run(const char *name)
{
    unsigned long long *d;
    int *r;
    (void)hipMalloc(&d, 8 * sizeof(unsigned long long));
    (void)hipMalloc(&r, 512 * sizeof(int));
    for (int threads : {256, 512}) {
        hipLaunchKernelGGL(k<KIND>, dim3(1), dim3(threads), 0, 0, d, r, 3, 0x05040100);
        hipLaunchKernelGGL(k<KIND>, dim3(1), dim3(threads), 0, 0, d, r, 3, 0x05040100);
        unsigned long long h[8] = {};
        (void)hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
        double m = 0;
        for (int w = 0; w < threads / 64; w++) m += h[w];
        m /= threads / 64;
        printf("%-22s waves/SIMD %d: %.2f cycles per instruction per wave\n", name, threads / 256, m / (NREP * 8.0));
    }
    (void)hipFree(d);
    (void)hipFree(r);
}

int main()
{
    run<0>("v_add_u32");
    run<1>("v_pk_sub_i16");
    run<2>("v_pk_sub_i16 clamp");
    run<3>("v_pk_max_i16");
    run<4>("v_perm_b32");
    run<5>("v_bitop3_b32");
    run<6>("v_and_b32");
    run<7>("v_pk_ashrrev_i16");
    run<8>("v_med3_i32");
    run<9>("v_and_or_b32");
    return 0;
}
