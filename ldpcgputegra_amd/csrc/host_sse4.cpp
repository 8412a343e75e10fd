// host_sse4.cpp -- the host decoder's 16-lane check loop for hosts without
// AVX2 (compiled with -msse4.1 only: no VEX encoding, checked by
// tools/check_host_isa.py).  See host_simd.h.
#define LDPC_HOST_SIMD_IMPL
#include "host_simd.h"

void host_checks_sse4(const ldpc_code *h, int8_t *V, int8_t *msg, const I8Params &p, const uint8_t *live)
{
    static_assert(Simd::W == 16, "SSE4.1 translation unit");
    p.early ? checks_all<true>(h, V, msg, p, live) : checks_all<false>(h, V, msg, p, live);
}
