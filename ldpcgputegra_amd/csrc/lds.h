// lds.h -- LDS-resident layered decoder for short codes (lds.hip).
#pragma once
#include <vector>

#include "kernels.h"
#include "ldpc_internal.h"

constexpr size_t kLdsMaxBytes = 64 * 1024;   // per wave (one workgroup); 160 KB per CU

struct LdsCode {
    int valid;
    int nl;            // layers per iteration
    int max_width;     // checks in the widest layer
    int lpc_log2;      // lanes per codeword (log2)
    int tab_bytes;     // LDS bytes of the u16 edge table (16-B aligned)
    uint16_t *d_tab;   // [E] layer-major edge -> variable
    int4 *d_layers;    // [nl] (edge base, checks, degree, later-group flag)
    // edge-parallel float kernel (ldsep.hip): compiled shape, layers, per-slot lane table
    int ep_valid = 0, ep_nl = 0, ep_shape = -1;
    uint32_t *d_ep_tab = nullptr;
};

int lds_upload(const ldpc_code *h, LdsCode *lc);
void lds_free(LdsCode *lc);
size_t lds_bytes(const ldpc_code *h, const LdsCode &lc, bool is_float);
bool lds_applicable(const ldpc_code *h, const LdsCode &lc, bool is_float);   // fits in LDS
bool lds_preferred(const ldpc_code *h, const LdsCode &lc, bool is_float);    // auto selection
// edge-parallel float kernel (kernel 9, ldsep.hip): one wave per codeword, one lane per edge
int ldsep_upload(const ldpc_code *h, const std::vector<int4> &layers, LdsCode *lc);
bool ldsep_applicable(const ldpc_code *h, const LdsCode &lc, bool is_float);
int launch_ldsep(const LdsCode &lc, const ldpc_code *h, const float *llr, uint8_t *hard, float *soft, int batch,
                 int iters, const DecodeLaunch &L, hipStream_t s);
// reads frame-major llr, writes frame-major hard / soft directly (no interleave)
int launch_lds(const LdsCode &lc, const ldpc_code *h, const void *llr, uint8_t *hard, void *soft, int batch,
               int iters, const DecodeLaunch &L, hipStream_t s);
