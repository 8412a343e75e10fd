// ubench_vmem.hip -- design input (not part of the library): the vector-memory
// floor of coop3's access pattern on MI355X, without its arithmetic.
//
// One 448-thread workgroup per CU (batch 4096 DVB-S2 r1/2 = 256 workgroups of
// 16 codewords), 6 "slab" waves + 1 idle / store wave, one s_barrier per
// period.  Per period and slab wave, as coop3: the 16-B V row
// pieces of 8 checks' 6 rows (5 info + o) are stored (window p-2) and
// gathered by LDS-DMA (window p+3), plus the 64-B message records of the 8
// checks (store: 32 lanes; gathers: 16 + 16 lanes).  The rows are the real
// DVB-S2 r1/2 edge list in layered order (48 consecutive checks per period).
//
// Layouts of the information rows (parity rows: the check-contiguous P layout
// of coop3 in every mode):
//   0  interleaved: V[row][pitch] (pitch 4160 codewords), workgroup wg owns
//      bytes wg*16 .. +15 of every row, XCD-aware block remap (coop3 today)
//   1  private: workgroup wg's rows contiguous, V[wg][row][16]: consecutive
//      bits of a DVB-S2 bit group (touched by checks q = 90 apart) share a
//      128-B line
//   2  ideal lines: every 8 lanes move one whole 128-B line (the traffic shape
//      of an LDS line cache: 6 lines per wave and period)
// Flags: nostore (no V stores), storewave (the 7th wave issues all V stores,
// slab waves only gather), filler = independent VALU ops per slab wave and
// period (coop3's slab waves issue ~296).
//   hipcc --offload-arch=gfx950 -O3 -o tools/ubench_vmem tools/ubench_vmem.hip \
//       -Lldpcgputegra_amd -lldpc_mi355x -Wl,-rpath,'$ORIGIN/../ldpcgputegra_amd'
//   tools/ubench_vmem ldpcgputegra_amd/codes/dvbs2_r1_2.txt
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../include/ldpc_mi355x.h"

constexpr int WS = 6, S = 48, CW = 16, NP = 600;   // slab waves, checks per period, codewords, periods per launch
constexpr int NI = 4;                                 // gathered windows in flight (LDS slots)

struct Args {
    char *V;               // info rows (layout by mode)
    char *P;               // parity rows, [wg][m][16]
    char *M;               // messages [wg][m][64]
    const int *rows;       // [NP][BLK]: [WS][64] row per lane (-1: inactive; lanes q < 6: V rows), [WS][8] check
                           // per slot (mode 2: the 5 info lanes of a slot carry its first info row)
    unsigned long long *out;
    int pitch, k, m, mode;
};

__device__ __forceinline__ void dma16(const void *gsrc, uint32_t lds_dst)
{
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(gsrc), "s"(lds_dst)
                 : "memory");
}

__device__ __forceinline__ char *row_addr(const Args &a, int wg, int r, int lane)
{
    if (r >= a.k) return a.P + ((size_t)wg * (a.m + 1) + (r - a.k)) * 16;
    if (a.mode == 0) return a.V + (size_t)r * a.pitch + (size_t)wg * CW;
    if (a.mode == 1) return a.V + ((size_t)wg * a.k + r) * 16;
    // mode 2: 8 lanes of a slot = one 128-B line (line index from the slot's first row);
    // mode 3: the same confined to 512 lines (64 KB) per workgroup (L2-resident)
    const size_t line = a.mode == 3 ? (size_t)((r >> 3) & 511) : (size_t)(r >> 3);
    return a.V + ((size_t)wg * a.k + line * 8) * 16 + (size_t)(lane & 7) * 16;
}

// index blocks (row per lane of every slab wave, check per slot) are staged
// into an LDS ring by wave WS, 5 periods ahead (coop3 stages its window
// tables by LDS-DMA the same way), so no slab wave waits on an index load
constexpr int BLK = 512, RING = 8;   // ints per period block: [WS][64] rows, then [WS][8] checks

template <int MODE, bool NOSTORE, bool STOREWAVE, int FILLER>
__global__ void __launch_bounds__(64 * (WS + 1)) vmem_k(Args a)
{
    static_assert(FILLER % 8 == 0, "filler");
    static_assert(WS * 64 + WS * 8 <= BLK, "block");
    // V store, message store, 2 gathers per period; the wait at period p
    // (after its stores) covers the gathers of period p-3
    constexpr int VS = (NOSTORE || STOREWAVE) ? 0 : 1, VMW = (VS + 1) + 2 * (VS + 3);
    a.mode = MODE;
    __shared__ uint4 in[WS][NI][80];
    __shared__ int ring[RING][BLK];
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const int nb = gridDim.x, id = blockIdx.x;
    const int wg = MODE == 0 ? (id & 7) * (nb >> 3) + (id >> 3) : id;
    const int kl = lane >> 3, q = lane & 7;
    uint32_t acc = lane, x0 = lane * 3u, x1 = lane * 5u, x2 = lane * 7u, x3 = lane * 11u;
    auto load_block = [&](int t) {   // wave WS: index block t -> ring[t % RING]
        const uint4 *src = (const uint4 *)(a.rows + (size_t)t * BLK);
        const uint4 u0 = src[lane], u1 = src[lane + 64];
        ((uint4 *)ring[t % RING])[lane] = u0;
        ((uint4 *)ring[t % RING])[lane + 64] = u1;
    };
    if (wave == WS)
        for (int t = 0; t < 5; t++) load_block(t);
    __syncthreads();
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    if (wave == WS) {   // index loader; with STOREWAVE also the V stores of window p-2 of every slab wave
        for (int p = 0; p < NP; p++) {
            if (STOREWAVE && !NOSTORE && p >= 2)
                for (int w = 0; w < WS; w++) {
                    const int r = ring[(p - 2) % RING][w * 64 + lane];
                    if (q < 6 && r >= 0) *(uint4 *)row_addr(a, wg, r, lane) = make_uint4(acc, acc + 1, acc + 2, acc + 3);
                }
            if (p + 5 < NP) load_block(p + 5);
            __syncthreads();
        }
    } else {
        const uint32_t base = (uint32_t)(uintptr_t)&in[wave][0][0];
        for (int p = 0; p < NP; p++) {
            // stores of window p-2: V pieces (lanes q < 6) and the message records (q < 4)
            if (p >= 2) {
                const int *blk = ring[(p - 2) % RING];
                const int r = blk[wave * 64 + lane];
                if (VS && q < 6 && r >= 0) *(uint4 *)row_addr(a, wg, r, lane) = make_uint4(acc, x0, x1, x2);
                const int c = blk[WS * 64 + wave * 8 + kl];
                if (q < 4) *(uint4 *)(a.M + ((size_t)wg * (a.m + 1) + c) * 64 + q * 16) = make_uint4(x3, acc, x0, x1);
            }
            // wait for window p's gathers (issued 3 periods ago), consume them
            asm volatile("s_waitcnt vmcnt(%0)" ::"n"(VMW) : "memory");
            const uint4 v = in[wave][p % NI][lane];
            acc += v.x ^ v.w;
#pragma unroll
            for (int i = 0; i < FILLER; i += 8)
                asm volatile("v_add_u32 %0, %0, %4\n\tv_add_u32 %1, %1, %4\n\tv_add_u32 %2, %2, %4\n\tv_add_u32 %3, %3, %4\n\t"
                             "v_xor_b32 %0, %0, %4\n\tv_xor_b32 %1, %1, %4\n\tv_xor_b32 %2, %2, %4\n\tv_xor_b32 %3, %3, %4"
                             : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3)
                             : "v"(acc));
            // gathers of window p+3 into slot (p+3) % NI
            const int pn = p + 3;
            if (pn < NP) {
                const int *blk = ring[pn % RING];
                const int r = blk[wave * 64 + lane];
                const int c = blk[WS * 64 + wave * 8 + kl];
                const char *src = q < 6 ? row_addr(a, wg, r < 0 ? 0 : r, lane)
                                        : a.M + ((size_t)wg * (a.m + 1) + c) * 64 + (q - 6) * 16;
                dma16(src, base + (uint32_t)((pn % NI) * 80 * 16));
                if (lane < 16) {
                    const int c2 = blk[WS * 64 + wave * 8 + (lane & 7)];
                    dma16(a.M + ((size_t)wg * (a.m + 1) + c2) * 64 + (2 + (lane >> 3)) * 16,
                          base + (uint32_t)((pn % NI) * 80 * 16 + 64 * 16));
                }
            }
            __syncthreads();
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (lane == 0) a.out[id * (WS + 1) + wave] = t1 - t0;
    if (acc == 0x12345678u && x0 == 1u && x3 == 2u) a.out[0] = 0;   // keep the arithmetic
}

int main(int argc, char **argv)
{
    const char *path = argc > 1 ? argv[1] : "ldpcgputegra_amd/codes/dvbs2_r1_2.txt";
    ldpc_code *h = nullptr;
    if (ldpc_code_load(path, &h) != LDPC_OK) {
        fprintf(stderr, "cannot load %s: %s\n", path, ldpc_last_error());
        return 1;
    }
    int n, m, e, ng, maxd;
    ldpc_code_info(h, &n, &m, &e, &ng, &maxd);
    std::vector<uint32_t> ev(e);
    std::vector<int> gd(ng), gc(ng);
    ldpc_code_edges(h, ev.data(), gd.data(), gc.data());
    const int k = n - m, D0 = gd[0], T = gc[0];
    // lanes (kl, q): q < 5 info rows, q == 5 the o row (parity), 6 / 7 messages
    std::vector<int> rows((size_t)NP * BLK, -1), rows2((size_t)NP * BLK, -1);
    for (int p = 0; p < NP; p++)
        for (int w = 0; w < WS; w++)
            for (int kl = 0; kl < 8; kl++) {
                const int c = (p * S + w * 8 + kl) % T;
                rows[(size_t)p * BLK + WS * 64 + w * 8 + kl] = rows2[(size_t)p * BLK + WS * 64 + w * 8 + kl] = c;
                for (int q = 0; q < 8; q++) {
                    const size_t i = (size_t)p * BLK + w * 64 + kl * 8 + q;
                    rows[i] = q < 5 ? (int)ev[(size_t)c * D0 + q] : q == 5 ? (int)ev[(size_t)c * D0 + D0 - 1] : -1;
                    rows2[i] = q < 5 ? (int)ev[(size_t)c * D0] : rows[i];
                }
            }
    const int grid = 256, pitch = 4096 + 64;
    Args a{};
    int *d_rows2 = nullptr;
    a.pitch = pitch;
    a.k = k;
    a.m = m;
    size_t vbytes = std::max((size_t)n * pitch, (size_t)grid * k * 16);
    if (hipMalloc(&a.V, vbytes) != hipSuccess || hipMalloc(&a.P, (size_t)grid * (m + 1) * 16) != hipSuccess ||
        hipMalloc(&a.M, (size_t)grid * (m + 1) * 64) != hipSuccess ||
        hipMalloc((void **)&a.rows, rows.size() * 4) != hipSuccess || hipMalloc((void **)&d_rows2, rows2.size() * 4) != hipSuccess ||
        hipMalloc(&a.out, (size_t)grid * (WS + 1) * 8) != hipSuccess) {
        fprintf(stderr, "hipMalloc failed\n");
        return 1;
    }
    hipMemset(a.V, 0, vbytes);
    hipMemcpy((void *)a.rows, rows.data(), rows.size() * 4, hipMemcpyHostToDevice);
    hipMemcpy((void *)d_rows2, rows2.data(), rows2.size() * 4, hipMemcpyHostToDevice);
    const int *d_rows = a.rows;
    struct Cfg {
        const char *name;
        void (*k)(Args);
        int mode;
    } cfgs[] = {
        {"interleaved", vmem_k<0, false, false, 0>, 0},
        {"interleaved nostore", vmem_k<0, true, false, 0>, 0},
        {"interleaved storewave", vmem_k<0, false, true, 0>, 0},
        {"interleaved filler296", vmem_k<0, false, false, 296>, 0},
        {"interleaved storewave f296", vmem_k<0, false, true, 296>, 0},
        {"private", vmem_k<1, false, false, 0>, 1},
        {"private nostore", vmem_k<1, true, false, 0>, 1},
        {"private filler296", vmem_k<1, false, false, 296>, 1},
        {"lines", vmem_k<2, false, false, 0>, 2},
        {"lines filler296", vmem_k<2, false, false, 296>, 2},
        {"filler296 only (nostore)", vmem_k<2, true, false, 296>, 2},
        {"lines64K", vmem_k<3, false, false, 0>, 3},
        {"lines64K nostore", vmem_k<3, true, false, 0>, 3},
        {"lines64K filler296", vmem_k<3, false, false, 296>, 3},
        {"lines64K filler592", vmem_k<3, false, false, 592>, 3},
    };
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    std::vector<unsigned long long> out((size_t)grid * (WS + 1));
    for (const Cfg &c : cfgs) {
        a.rows = c.mode >= 2 ? d_rows2 : d_rows;
        hipLaunchKernelGGL(c.k, dim3(grid), dim3(64 * (WS + 1)), 0, 0, a);   // warm-up
        hipEventRecord(e0, 0);
        const int reps = 3;
        for (int r = 0; r < reps; r++) hipLaunchKernelGGL(c.k, dim3(grid), dim3(64 * (WS + 1)), 0, 0, a);
        hipEventRecord(e1, 0);
        if (hipEventSynchronize(e1) != hipSuccess) {
            fprintf(stderr, "kernel failed: %s\n", hipGetErrorString(hipGetLastError()));
            return 1;
        }
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        hipMemcpy(out.data(), a.out, out.size() * 8, hipMemcpyDeviceToHost);
        double cyc = 0;
        for (int b = 0; b < grid; b++) cyc += out[(size_t)b * (WS + 1)];
        cyc /= grid;
        const double us_per_period = ms * 1e3 / reps / NP;
        printf("%-28s %7.3f us/period  %6.0f cycles/period (wave 0)  -> 50 it x 722 periods = %6.2f ms\n", c.name,
               us_per_period, cyc / NP, us_per_period * 722 * 50 / 1e3);
    }
    ldpc_code_destroy(h);
    return 0;
}
