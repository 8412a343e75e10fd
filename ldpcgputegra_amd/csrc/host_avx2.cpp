// host_avx2.cpp -- the host decoder's 32-lane check loop (compiled with -mavx2;
// host.cpp calls it only where the CPU reports AVX2).  See host_simd.h.
#define LDPC_HOST_SIMD_IMPL
#include "host_simd.h"

void host_checks_avx2(const ldpc_code *h, int8_t *V, int8_t *msg, const I8Params &p, const uint8_t *live)
{
    static_assert(Simd::W == 32, "AVX2 translation unit");
    p.early ? checks_all<true>(h, V, msg, p, live) : checks_all<false>(h, V, msg, p, live);
}
