// ubench_lc.hip -- design input (not part of the library): the period floor of
// a coop3 whose V rows live in an LDS line cache, measured
// with the memory traffic and the instruction mix of that design but without
// its arithmetic.
//
// One 448-thread workgroup per CU (256 workgroups = batch 4096 DVB-S2 r1/2), 6
// slab waves + 1 idle wave, one s_barrier per period.  Per period and slab
// wave (measured plan of the line cache, /tmp-free numbers in DESIGN.md: ~30
// 128-B line loads and ~30 line stores per 45-check window):
//   * line stores: ds_read_b128 of 8 lines (64 lanes x 16 B) from the cache,
//     then global_store_dwordx4 to the workgroup's own V region (coalesced)
//   * line loads: global_load_dwordx4 of 8 lines into VGPRs, written to the
//     cache (ds_write_b128) two periods later
//   * the 64-B message records of the wave's 8 checks: 2 LDS-DMA gathers
//     (window p+3) and one store, as coop3 today
//   * FILLER packed-i16 VALU (v_pk_add_u16: coop3's slab waves issue ~296
//     VALU per period, mostly packed / v_perm at the same issue cost) and
//     NLDS LDS reads of 4 B from scattered cache rows + 8 ds_write_b16
// Lines are spread pseudo-randomly over the workgroup's 1 MB region (an L2
// share far below it: served from the Infinity Cache / HBM, as the cache's
// misses would be).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/ubench_lc tools/ubench_lc.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <type_traits>
#include <vector>

constexpr int WS = 6, NP = 720, CW = 16;
constexpr int LINES = 8100 + 4050;   // info + parity lines of one workgroup (DVB-S2 r1/2, 16 codewords)
constexpr int CACHE = 640;           // cache slots (128 B)
constexpr int M = 32400;

struct Args {
    char *V;    // [wg][LINES][128]
    char *Mc;   // [wg][M + 1][64]
    unsigned long long *out;
};

__device__ __forceinline__ void dma16(const void *gsrc, uint32_t lds_dst)
{
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(gsrc), "s"(lds_dst)
                 : "memory");
}

__device__ __forceinline__ uint32_t hash32(uint32_t x)
{
    x ^= x >> 16;
    x *= 0x7feb352du;
    x ^= x >> 15;
    x *= 0x846ca68bu;
    return x ^ (x >> 16);
}

// FILLER packed VALU + FILLER / 4 cheap bitwise VALU; NLINE lines loaded and
// written back per wave and period (8: 48 per CU, 5: 30 = the plan's mean);
// SEQ: lines swept in order (each loaded once per ~400 periods: HBM), else
// pseudo-random
template <int FILLER, int NLDS, bool STORES, int NLINE = 8, bool SEQ = false>
__global__ void __launch_bounds__(64 * (WS + 1)) lc_k(Args a)
{
    __shared__ uint4 cache[CACHE * 8];
    __shared__ uint4 min_[WS][4][64];   // message DMA landing (4 windows in flight)
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const int wg = blockIdx.x;
    const int l = lane >> 3, q = lane & 7;
    char *Vw = a.V + (size_t)wg * LINES * 128;
    char *Mw = a.Mc + (size_t)wg * (M + 1) * 64;
    uint32_t x0 = lane, x1 = lane * 3u, x2 = lane * 5u, x3 = lane * 7u, acc = 0;
    uint4 ld[2] = {make_uint4(0, 0, 0, 0), make_uint4(0, 0, 0, 0)};   // staged line loads (static indices only)
    __syncthreads();
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    if (wave < WS) {
        const uint32_t mbase = (uint32_t)(uintptr_t)&min_[wave][0][0];
        // one period; S = p % 2 is static (periods unrolled by two) so that the
        // staged line loads stay in named VGPRs the compiler keeps live and
        // waits for (compiler-visible loads: its vmcnt counts only its own
        // operations, which errs on the safe side)
        auto period = [&](auto sc, int p) __attribute__((always_inline)) {
            constexpr int S = decltype(sc)::value;
            const uint32_t key = (uint32_t)(p * WS + wave) * 8u + (uint32_t)l;
            // line stores: 8 lines written back (slots of lines whose last post was period p-1)
            if (STORES && l < NLINE) {
                const int slot = (int)(hash32(key ^ 0x9e3779b9u) % CACHE);
                const uint4 d = cache[slot * 8 + q];
                const int line = SEQ ? (int)(((uint32_t)p * (WS * NLINE) + (uint32_t)(wave * NLINE + l) + 7000u) % LINES)
                                     : (int)(hash32(key ^ 0x85ebca6bu) % LINES);
                *(uint4 *)(Vw + (size_t)line * 128 + q * 16) = d;
            }
            // message store of the wave's 8 checks (window p-2)
            const int chk = (p * 48 + wave * 8 + l) % M;
            if (q < 4) *(uint4 *)(Mw + (size_t)chk * 64 + q * 16) = make_uint4(x0, x1, x2, x3);
            // the message gathers of window p (issued 3 periods ago) have landed:
            // per period [line store], message store, line load, 2 message DMA
            // (a wave with NLINE = 0 issues no line load or store)
            asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NLINE == 0 ? 7 : STORES ? 12 : 9) : "memory");
            // line loads issued two periods ago land in the cache now
            if (l < NLINE) {
                const int slot = (int)(hash32(key ^ 0xc2b2ae35u) % CACHE);
                cache[slot * 8 + q] = ld[S];
            }
            // the window's scattered cache reads / writes (pre + post)
            // (cheap address arithmetic, as the kernel's record offsets are: 2 VALU per access)
            uint32_t r = 0;
            const uint32_t hb = hash32(key);
#pragma unroll
            for (int i = 0; i < NLDS; i++) {
                const uint32_t off = ((hb + (uint32_t)i * 977u) & 4095u) * 16u + 4u * (uint32_t)(q >> 1);
                r += *(const uint32_t *)((const char *)cache + off);
            }
            acc += r + min_[wave][p & 3][lane].x;
#pragma unroll
            for (int i = 0; i < FILLER; i += 4)
                asm volatile("v_pk_add_u16 %0, %0, %4\n\tv_pk_add_u16 %1, %1, %4\n\tv_pk_add_u16 %2, %2, %4\n\tv_pk_add_u16 %3, %3, %4"
                             : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3)
                             : "v"(acc));
#pragma unroll
            for (int i = 0; i < FILLER / 4; i += 4)
                asm volatile("v_xor_b32 %0, %0, %4\n\tv_xor_b32 %1, %1, %4\n\tv_and_b32 %2, %2, %4\n\tv_or_b32 %3, %3, %4"
                             : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3)
                             : "v"(acc));
            if (NLDS) {
#pragma unroll
                for (int i = 0; i < 8; i++) {
                    const uint32_t off = ((hb + (uint32_t)i * 1553u) & 4095u) * 16u + 2u * (uint32_t)q;
                    *(unsigned short *)((char *)cache + off) = (unsigned short)(x0 + i);
                }
            }
            // line loads for period p+2
            if (l < NLINE) {
                const int line = SEQ ? (int)(((uint32_t)p * (WS * NLINE) + (uint32_t)(wave * NLINE + l)) % LINES)
                                     : (int)(hash32(key ^ 0x27d4eb2fu) % LINES);
                ld[S] = *(const uint4 *)(Vw + (size_t)line * 128 + q * 16);
            }
            // message gathers of window p+3
            const int chn = ((p + 3) * 48 + wave * 8 + l) % M;
            dma16(Mw + (size_t)chn * 64 + (q & 3) * 16, mbase + (uint32_t)(((p + 3) & 3) * 64 * 16));
            if (lane < 16) dma16(Mw + (size_t)chn * 64 + 32 + (q & 1) * 16, mbase + (uint32_t)(((p + 3) & 3) * 64 * 16));
            __syncthreads();
        };
        for (int p = 0; p < NP; p += 2) {
            period(std::integral_constant<int, 0>{}, p);
            period(std::integral_constant<int, 1>{}, p + 1);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else {
        for (int p = 0; p < NP; p++) __syncthreads();
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (lane == 0) a.out[wg * (WS + 1) + wave] = t1 - t0;
    if (acc == 0x12345678u && x0 == 1u && x3 == 2u && ld[0].x == 3u) a.out[0] = 0;
}

int main()
{
    const int grid = 256;
    Args a{};
    if (hipMalloc(&a.V, (size_t)grid * LINES * 128) != hipSuccess ||
        hipMalloc(&a.Mc, (size_t)grid * (M + 1) * 64) != hipSuccess ||
        hipMalloc(&a.out, (size_t)grid * (WS + 1) * 8) != hipSuccess) {
        fprintf(stderr, "hipMalloc failed\n");
        return 1;
    }
    (void)hipMemset(a.V, 0, (size_t)grid * LINES * 128);
    struct Cfg {
        const char *name;
        void (*k)(Args);
    } cfgs[] = {
        {"lc mem only (48+48 lines, random)", lc_k<0, 0, true>},
        {"lc mem only (30+30 lines, seq)", lc_k<0, 0, true, 5, true>},
        {"lc 30 seq + 32 LDS", lc_k<0, 32, true, 5, true>},
        {"lc 30 seq + 200 pk + 50 bit VALU", lc_k<200, 0, true, 5, true>},
        {"lc 30 seq + 32 LDS + 200/50 VALU", lc_k<200, 32, true, 5, true>},
        {"lc 30 seq + 32 LDS + 160/40 VALU", lc_k<160, 32, true, 5, true>},
        {"no memory: 32 LDS + 200/50 VALU", lc_k<200, 32, false, 0, true>},
    };
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    std::vector<unsigned long long> out((size_t)grid * (WS + 1));
    for (const Cfg &c : cfgs) {
        hipLaunchKernelGGL(c.k, dim3(grid), dim3(64 * (WS + 1)), 0, 0, a);
        (void)hipEventRecord(e0, 0);
        const int reps = 3;
        for (int r = 0; r < reps; r++) hipLaunchKernelGGL(c.k, dim3(grid), dim3(64 * (WS + 1)), 0, 0, a);
        (void)hipEventRecord(e1, 0);
        if (hipEventSynchronize(e1) != hipSuccess) {
            fprintf(stderr, "kernel failed: %s\n", hipGetErrorString(hipGetLastError()));
            return 1;
        }
        float ms = 0;
        (void)hipEventElapsedTime(&ms, e0, e1);
        (void)hipMemcpy(out.data(), a.out, out.size() * 8, hipMemcpyDeviceToHost);
        double cyc = 0;
        for (int b = 0; b < grid; b++) cyc += out[(size_t)b * (WS + 1)];
        cyc /= grid;
        const double us = ms * 1e3 / reps / NP;
        printf("%-42s %7.3f us/period  %6.0f cycles/period  -> 36100 periods = %6.2f ms\n", c.name, us, cyc / NP,
               us * 36100 / 1e3);
    }
    return 0;
}
