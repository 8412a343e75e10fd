// ubench_chain.hip -- design input for the staircase chain wave (not part of
// the library): cycles per chain step on gfx950 for
//   * dependent single-instruction chains (the step's building blocks),
//   * the r01 5-instruction i32 step (v_med3 copy, 2 x v_mad_i32_i24, 2 x v_med3),
//   * a 3-instruction i16 step: v_pk_mad_i16 (both mads at once, Y broadcast
//     by op_sel_hi) -> v_med3_i16 (dead zone, second operand from the high
//     half by op_sel) -> v_med3_i16 (clamp to [L, H] from one register),
//     with the output written alternately into the low / high half of a
//     register (op_sel dst), so 8 outputs fill a ds_write_b128,
//   * the same with its constants read from LDS (one ds_read_b128 per step,
//     8 steps ahead) and outputs stored to LDS,
// one wave alone on the CU, and beside 1 / 7 filler waves (VALU streams).
// The i16 step is also checked against a host model of the recurrence.
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/ubench_chain tools/ubench_chain.hip && /tmp/ubench_chain
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

constexpr int NSTEP = 32, NREP = 64;

__device__ unsigned long long stamp()
{
    unsigned long long t;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    return t;
}

#define R4(x) x x x x
#define R16(x) R4(x) R4(x) R4(x) R4(x)

// KIND 0..4: dependent chains of one instruction, 16 per loop trip
template <int KIND>
__device__ int single(int y, int b, int c)
{
    for (int i = 0; i < NREP; i++) {
        if constexpr (KIND == 0) asm volatile(R16("v_med3_i32 %0, %0, %1, %2\n\t") : "+v"(y) : "v"(b), "v"(c));
        if constexpr (KIND == 1) asm volatile(R16("v_pk_mad_i16 %0, %0, %1, %2 op_sel_hi:[0,0,1]\n\t") : "+v"(y) : "v"(b), "v"(c));
        if constexpr (KIND == 2) asm volatile(R16("v_med3_i16 %0, %0, %1, %2 op_sel:[0,0,1,0]\n\t") : "+v"(y) : "v"(b), "v"(c));
        if constexpr (KIND == 3) asm volatile(R16("v_pk_add_i16 %0, %0, %1\n\t") : "+v"(y) : "v"(b));
        if constexpr (KIND == 4) asm volatile(R16("v_add_u32 %0, %0, %1\n\t") : "+v"(y) : "v"(b));
        if constexpr (KIND == 5) asm volatile(R16("v_mad_i32_i24 %0, %0, %1, %2\n\t") : "+v"(y) : "v"(b), "v"(c));
        if constexpr (KIND == 6) asm volatile(R16("v_fma_f32 %0, %0, %1, %2\n\t") : "+v"(y) : "v"(b), "v"(c));
        if constexpr (KIND == 7) asm volatile(R16("v_med3_f32 %0, %0, %1, %2\n\t") : "+v"(y) : "v"(b), "v"(c));
        if constexpr (KIND == 8) asm volatile(R16("v_add_f32 %0, %0, %1\n\t") : "+v"(y) : "v"(b));
        if constexpr (KIND == 9) asm volatile(R16("v_max_i16 %0, %0, %1\n\t") : "+v"(y) : "v"(b));
    }
    return y;
}

// constants of one step: k1 = (A, B), k2 = (eps, co), k3 = (L, H) as i16 pairs
struct Cst {
    int k1, k2, k3, pad;
};

// one i16 step; OUT_HI: the output goes to the high half of y (the low half
// is kept), IN_HI: the input is read from the high half of x
#define STEP16(IN_HI, OUT_HI)                                                                     \
    asm volatile("v_pk_mad_i16 %1, %2, %4, %3 op_sel:[" #IN_HI ",0,0] op_sel_hi:[" #IN_HI ",0,1]\n\t" \
                 "v_med3_i16 %1, %1, %4, %1 op_sel:[0,1,1,0]\n\t"                                  \
                 "v_med3_i16 %0, %1, %5, %5 op_sel:[0,0,1," #OUT_HI "]\n\t"                        \
                 : "+v"(yout), "=&v"(t)                                                            \
                 : "v"(yin), "v"(c.k1), "v"(c.k2), "v"(c.k3))

// KIND 10: 5-instruction i32 step (constants in VGPRs)
// KIND 11: 3-instruction i16 step, output to the low half only (constants in VGPRs)
// KIND 12: 3-instruction i16 step, outputs alternating halves (constants in VGPRs)
// KIND 13: as 12, constants from LDS 8 steps ahead, outputs to LDS every 8 steps
template <int KIND>
__global__ void __launch_bounds__(512) chain(unsigned long long *out, int *res, const Cst *cst, int nfill)
{
    __shared__ Cst sc[NSTEP][64];
    __shared__ int4 so[NSTEP / 8][64];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    for (int i = threadIdx.x; i < NSTEP * 64; i += blockDim.x) sc[i / 64][i % 64] = cst[i];
    __syncthreads();
    if (wave > 0) {   // filler: 4 independent VALU streams
        if (wave <= nfill) {
            int a = lane, b = lane + 1, c2 = lane + 2, d = lane + 3, k = res[0];
            for (int i = 0; i < NREP * NSTEP / 4; i++)
                asm volatile(R4("v_add_u32 %0, %0, %4\n\tv_xor_b32 %1, %1, %4\n\tv_add_u32 %2, %2, %4\n\tv_xor_b32 %3, %3, %4\n\t")
                             : "+v"(a), "+v"(b), "+v"(c2), "+v"(d)
                             : "v"(k));
            res[64 + threadIdx.x] = a + b + c2 + d;
        }
        return;
    }
    Cst q[NSTEP];
#pragma unroll
    for (int i = 0; i < NSTEP; i++) q[i] = cst[i * 64 + lane];
    int y = 0;
    unsigned long long t0 = stamp();
    if constexpr (KIND == 10) {
        for (int r = 0; r < NREP; r++)
#pragma unroll
            for (int i = 0; i < NSTEP; i++) {
                int x, p, qq;
                const int eps = (short)(q[i].k2 & 0xffff), co = q[i].k2 >> 16, A = (short)(q[i].k1 & 0xffff),
                          B = q[i].k1 >> 16, L = (short)(q[i].k3 & 0xffff), H = q[i].k3 >> 16;
                asm volatile("v_med3_i32 %1, %0, %8, %9\n\t"
                             "v_mad_i32_i24 %2, %0, %4, %5\n\t"
                             "v_mad_i32_i24 %3, %0, %4, %6\n\t"
                             "v_med3_i32 %2, %2, %7, %3\n\t"
                             "v_med3_i32 %0, %2, %10, %11"
                             : "+v"(y), "=&v"(x), "=&v"(p), "=&v"(qq)
                             : "v"(eps), "v"(A), "v"(B), "v"(co), "v"(-127), "v"(127), "v"(L), "v"(H));
            }
    } else if constexpr (KIND == 11) {
        for (int r = 0; r < NREP; r++)
#pragma unroll
            for (int i = 0; i < NSTEP; i++) {
                int t;
                const Cst c = q[i];
                int &yout = y;
                const int yin = y;
                STEP16(0, 0);
            }
    } else if constexpr (KIND == 12) {
        int w[4] = {0, 0, 0, 0};
        for (int r = 0; r < NREP; r++)
#pragma unroll
            for (int i = 0; i < NSTEP; i++) {
                int t;
                const Cst c = q[i];
                const int s = i & 7;
                const int yin = s == 0 ? w[3] : w[(s - 1) >> 1];
                int &yout = w[s >> 1];
                if (s == 0) STEP16(1, 0);
                else if (s & 1) STEP16(0, 1);
                else STEP16(1, 0);
            }
        y = w[3] >> 16;
    } else if constexpr (KIND == 14 || KIND == 15) {
        // f32 step: a = eps y + A, b = eps y + B (independent), med3(a, co, b), med3(., L, H)
        // KIND 15: the same on lanes 0..15 only (the chain wave's 16 codewords)
        float fq[NSTEP][6];
#pragma unroll
        for (int i = 0; i < NSTEP; i++) {
            fq[i][0] = (float)(short)(q[i].k2 & 0xffff);
            fq[i][1] = (float)(short)(q[i].k1 & 0xffff);
            fq[i][2] = (float)(q[i].k1 >> 16);
            fq[i][3] = (float)(q[i].k2 >> 16);
            fq[i][4] = (float)(short)(q[i].k3 & 0xffff);
            fq[i][5] = (float)(q[i].k3 >> 16);
        }
        float fy = 0.f;
        if (KIND == 14 || lane < 16) {
            for (int r = 0; r < NREP; r++)
#pragma unroll
                for (int i = 0; i < NSTEP; i++) {
                    float ta, tb;
                    asm volatile("v_fma_f32 %1, %0, %3, %4\n\t"
                                 "v_fma_f32 %2, %0, %3, %5\n\t"
                                 "v_med3_f32 %1, %1, %6, %2\n\t"
                                 "v_med3_f32 %0, %1, %7, %8"
                                 : "+v"(fy), "=&v"(ta), "=&v"(tb)
                                 : "v"(fq[i][0]), "v"(fq[i][1]), "v"(fq[i][2]), "v"(fq[i][3]), "v"(fq[i][4]), "v"(fq[i][5]));
                }
        }
        y = (int)fy;
    } else if constexpr (KIND == 16) {   // the i16 step of KIND 12 on lanes 0..15 only
        int w[4] = {0, 0, 0, 0};
        if (lane < 16) {
            for (int r = 0; r < NREP; r++)
#pragma unroll
                for (int i = 0; i < NSTEP; i++) {
                    int t;
                    const Cst c = q[i];
                    const int s = i & 7;
                    const int yin = s == 0 ? w[3] : w[(s - 1) >> 1];
                    int &yout = w[s >> 1];
                    if (s == 0) STEP16(1, 0);
                    else if (s & 1) STEP16(0, 1);
                    else STEP16(1, 0);
                }
        }
        y = w[3] >> 16;
    } else if constexpr (KIND == 17 || KIND == 18 || KIND == 19) {
        // LDS constants, lanes 0..15 only (the real chain wave): 17 as KIND 13
        // (the compiler's 8 ds_read_b128 per block at its start); 18 / 19 one
        // ds_read_b128 inside each step's asm, between the mad and the first
        // med3 (manual lgkmcnt at the block start); 19 on all 64 lanes
        int w[4] = {0, 0, 0, 0};
        if (KIND == 19 || lane < 16) {
            if constexpr (KIND == 17) {
                Cst cb[2][8];
#pragma unroll
                for (int j = 0; j < 8; j++) cb[0][j] = sc[j][lane];
                for (int r = 0; r < NREP; r++) {
#pragma unroll
                    for (int i = 0; i < NSTEP; i++) {
                        int t;
                        const int s = i & 7, blk = i >> 3;
                        if (s == 0) {
#pragma unroll
                            for (int j = 0; j < 8; j++) cb[(blk + 1) & 1][j] = sc[((blk + 1) % (NSTEP / 8)) * 8 + j][lane];
                        }
                        const Cst c = cb[blk & 1][s];
                        const int yin = s == 0 ? w[3] : w[(s - 1) >> 1];
                        int &yout = w[s >> 1];
                        if (s == 0) STEP16(1, 0);
                        else if (s & 1) STEP16(0, 1);
                        else STEP16(1, 0);
                        if (s == 7) so[blk][lane] = make_int4(w[0], w[1], w[2], w[3]);
                    }
                }
            } else {
                typedef int v4i __attribute__((ext_vector_type(4)));
                v4i cb[2][8];
                const uint32_t base = (uint32_t)(uintptr_t)&sc[0][lane];
#pragma unroll
                for (int j = 0; j < 8; j++) cb[0][j] = *(const v4i *)&sc[j][lane];
                for (int r = 0; r < NREP; r++) {
#pragma unroll
                    for (int i = 0; i < NSTEP; i++) {
                        int t;
                        const int s = i & 7, blk = i >> 3;
                        if (s == 0) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                        const v4i cv = cb[blk & 1][s];
                        const int4 c = make_int4(cv[0], cv[1], cv[2], cv[3]);
                        const int yin = s == 0 ? w[3] : w[(s - 1) >> 1];
                        int &yout = w[s >> 1];
                        const uint32_t ra = base + (uint32_t)((((blk + 1) % (NSTEP / 8)) * 8 + s) * 64 * 16);
                        v4i &dst = cb[(blk + 1) & 1][s];
#define STEP16L(IN_HI, OUT_HI)                                                                                \
    asm volatile("v_pk_mad_i16 %1, %3, %5, %4 op_sel:[" #IN_HI ",0,0] op_sel_hi:[" #IN_HI ",0,1]\n\t"         \
                 "ds_read_b128 %2, %7\n\t"                                                                      \
                 "v_med3_i16 %1, %1, %5, %1 op_sel:[0,1,1,0]\n\t"                                             \
                 "v_med3_i16 %0, %1, %6, %6 op_sel:[0,0,1," #OUT_HI "]\n\t"                                   \
                 : "+v"(yout), "=&v"(t), "=&v"(dst)                                                           \
                 : "v"(yin), "v"(c.x), "v"(c.y), "v"(c.z), "v"(ra)                                             \
                 : "memory")
                        if (s == 0) STEP16L(1, 0);
                        else if (s & 1) STEP16L(0, 1);
                        else STEP16L(1, 0);
                        if (s == 7) {
                            const v4i o = {w[0], w[1], w[2], w[3]};
                            const uint32_t oa = (uint32_t)(uintptr_t)&so[blk][lane];
                            asm volatile("ds_write_b128 %0, %1" ::"v"(oa), "v"(o) : "memory");
                        }
                    }
                }
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            }
        }
        y = w[3] >> 16;
    } else if constexpr (KIND == 20) {
        // i32 step without a multiply: a = (y ^ s) + A', b = (y ^ s) + B' (v_xad_u32,
        // s = 0 / -1 for eps = +1 / -1, A' = A - s), med3_i32(a, co, b), med3_i32(., L, H)
        int iq[NSTEP][6];
#pragma unroll
        for (int i = 0; i < NSTEP; i++) {
            const int eps = (short)(q[i].k2 & 0xffff), sgn = eps < 0 ? -1 : 0;
            iq[i][0] = sgn;
            iq[i][1] = (short)(q[i].k1 & 0xffff) - sgn;
            iq[i][2] = (q[i].k1 >> 16) - sgn;
            iq[i][3] = q[i].k2 >> 16;
            iq[i][4] = (short)(q[i].k3 & 0xffff);
            iq[i][5] = q[i].k3 >> 16;
        }
        if (lane < 16) {
            for (int r = 0; r < NREP; r++)
#pragma unroll
                for (int i = 0; i < NSTEP; i++) {
                    int ta, tb;
                    asm volatile("v_xad_u32 %1, %0, %3, %4\n\t"
                                 "v_xad_u32 %2, %0, %3, %5\n\t"
                                 "v_med3_i32 %1, %1, %6, %2\n\t"
                                 "v_med3_i32 %0, %1, %7, %8"
                                 : "+v"(y), "=&v"(ta), "=&v"(tb)
                                 : "v"(iq[i][0]), "v"(iq[i][1]), "v"(iq[i][2]), "v"(iq[i][3]), "v"(iq[i][4]), "v"(iq[i][5]));
                }
        }
    } else if constexpr (KIND == 13) {
        int w[4] = {0, 0, 0, 0};
        Cst cb[2][8];
#pragma unroll
        for (int j = 0; j < 8; j++) cb[0][j] = sc[j][lane];
        for (int r = 0; r < NREP; r++) {
#pragma unroll
            for (int i = 0; i < NSTEP; i++) {
                int t;
                const int s = i & 7, blk = i >> 3;
                if (s == 0) {   // constants of the next 8 steps (cyclic), one block ahead
#pragma unroll
                    for (int j = 0; j < 8; j++) cb[(blk + 1) & 1][j] = sc[((blk + 1) % (NSTEP / 8)) * 8 + j][lane];
                }
                const Cst c = cb[blk & 1][s];
                const int yin = s == 0 ? w[3] : w[(s - 1) >> 1];
                int &yout = w[s >> 1];
                if (s == 0) STEP16(1, 0);
                else if (s & 1) STEP16(0, 1);
                else STEP16(1, 0);
                if (s == 7) so[blk][lane] = make_int4(w[0], w[1], w[2], w[3]);
            }
        }
        y = w[3] >> 16;
    }
    unsigned long long t1 = stamp();
    if (lane == 0) out[blockIdx.x] = t1 - t0;
    res[threadIdx.x] = y;
}

template <int KIND>
__global__ void __launch_bounds__(64) single_k(unsigned long long *out, int *res, int b, int c)
{
    unsigned long long t0 = stamp();
    int y = single<KIND>(threadIdx.x, b, c);
    unsigned long long t1 = stamp();
    if (threadIdx.x == 0) out[0] = t1 - t0;
    res[threadIdx.x] = y;
}

static short h16(int x) { return (short)(x & 0xffff); }

int main()
{
    unsigned long long *d_out;
    int *d_res;
    Cst *d_cst;
    (void)hipMalloc(&d_out, 64 * sizeof(unsigned long long));
    (void)hipMalloc(&d_res, 1024 * sizeof(int));
    (void)hipMalloc(&d_cst, NSTEP * 64 * sizeof(Cst));
    (void)hipMemset(d_res, 0, 1024 * sizeof(int));
    unsigned long long h = 0;
    const char *names[] = {"v_med3_i32", "v_pk_mad_i16 (op_sel_hi)", "v_med3_i16 (op_sel)", "v_pk_add_i16", "v_add_u32",
                           "v_mad_i32_i24", "v_fma_f32", "v_med3_f32", "v_add_f32", "v_max_i16"};
#define SINGLE(K)                                                                                   \
    hipLaunchKernelGGL(single_k<K>, dim3(1), dim3(64), 0, 0, d_out, d_res, 3, 5);                    \
    hipLaunchKernelGGL(single_k<K>, dim3(1), dim3(64), 0, 0, d_out, d_res, 3, 5);                    \
    (void)hipMemcpy(&h, d_out, 8, hipMemcpyDeviceToHost);                                            \
    printf("dependent %-26s %.2f cycles/instruction\n", names[K], (double)h / (NREP * 16.0));
    SINGLE(0) SINGLE(1) SINGLE(2) SINGLE(3) SINGLE(4) SINGLE(5) SINGLE(6) SINGLE(7) SINGLE(8) SINGLE(9)

    // random step constants in the kernel's ranges; eps = +-1, off = 1
    std::vector<Cst> hc(NSTEP * 64);
    srand(7);
    for (auto &c : hc) {
        const int eps = (rand() & 1) ? 1 : -1, co = rand() % 255 - 127, mx = rand() % 63 - 31, T = rand() % 32,
                  off = 1;
        const int A = co - eps * (mx + off), B = co - eps * (mx - off), L = co - T, H = co + T;
        c.k1 = (A & 0xffff) | (B << 16);
        c.k2 = (eps & 0xffff) | (co << 16);
        c.k3 = (L & 0xffff) | (H << 16);
        c.pad = 0;
    }
    (void)hipMemcpy(d_cst, hc.data(), hc.size() * sizeof(Cst), hipMemcpyHostToDevice);
    // host model of NREP * NSTEP steps per lane (i32, as KIND 10)
    std::vector<int> ref(64);
    for (int l = 0; l < 64; l++) {
        int y = 0;
        for (int r = 0; r < NREP; r++)
            for (int i = 0; i < NSTEP; i++) {
                const Cst &c = hc[i * 64 + l];
                const int eps = h16(c.k2), co = c.k2 >> 16, A = h16(c.k1), B = c.k1 >> 16, L = h16(c.k3), H = c.k3 >> 16;
                auto med3 = [](int a, int b, int d) { return std::max(std::min(a, b), std::min(std::max(a, b), d)); };
                y = med3(med3(eps * y + A, co, eps * y + B), L, H);
            }
        ref[l] = y;
    }
    const char *cn[] = {"5-instr i32 step (VGPR constants)", "3-instr i16 step, low half", "3-instr i16 step, alternating halves",
                        "3-instr i16 step, LDS constants + LDS outputs", "f32 step (2 fma + 2 med3)",
                        "f32 step, lanes 0..15", "3-instr i16 step, lanes 0..15", "i16 LDS constants, lanes 0..15",
                        "i16 LDS read inside step, lanes 0..15", "i16 LDS read inside step, 64 lanes",
                        "i32 xad step, lanes 0..15"};
#define CHAIN(K, TH, NF, IDX)                                                                       \
    {                                                                                               \
        hipLaunchKernelGGL(chain<K>, dim3(1), dim3(TH), 0, 0, d_out, d_res, d_cst, NF);             \
        (void)hipMemset(d_res, 0, 64 * sizeof(int));                                                \
        hipLaunchKernelGGL(chain<K>, dim3(1), dim3(TH), 0, 0, d_out, d_res, d_cst, NF);             \
        (void)hipMemcpy(&h, d_out, 8, hipMemcpyDeviceToHost);                                        \
        std::vector<int> got(64);                                                                   \
        (void)hipMemcpy(got.data(), d_res, 64 * 4, hipMemcpyDeviceToHost);                           \
        int bad = 0;                                                                                \
        for (int l = 0; l < ((IDX) >= 5 && (IDX) != 9 ? 16 : 64); l++) bad += (short)got[l] != (short)ref[l];                         \
        printf("%-48s fillers %d: %.2f cycles/step  mismatches %d\n", cn[IDX], NF, (double)h / (NREP * NSTEP), bad); \
    }
    for (int nf : {0, 7}) {
        CHAIN(10, 512, nf, 0)
        CHAIN(11, 512, nf, 1)
        CHAIN(12, 512, nf, 2)
        CHAIN(13, 512, nf, 3)
        CHAIN(14, 512, nf, 4)
        CHAIN(15, 512, nf, 5)
        CHAIN(16, 512, nf, 6)
        CHAIN(17, 512, nf, 7)
        CHAIN(18, 512, nf, 8)
        CHAIN(19, 512, nf, 9)
        CHAIN(20, 512, nf, 10)
    }
    return 0;
}
