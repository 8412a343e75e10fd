// host.h -- the host decoder behind the C-ABI's device = -1 contexts (host.cpp).
#pragma once
#include "ldpc_internal.h"

bool host_has_avx2();
// frame-major [batch][N] in, 0/1 hard decisions out; same semantics as the device decoders
int host_decode_i8(const ldpc_code *h, const int8_t *llr, uint8_t *hard, int batch, int n_iter, const ldpc_params *p);
int host_decode_f32(const ldpc_code *h, const float *llr, uint8_t *hard, int batch, int n_iter, const ldpc_params *p);
