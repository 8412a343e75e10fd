// ldpc_internal.h -- host-side structures shared by the C-ABI translation units.
#pragma once

#include <cstdarg>
#include <cstdint>
#include <string>
#include <vector>

#include "../../include/ldpc_mi355x.h"

// One window of the layered schedule for the windowed kernel (see plan.cpp).
struct ldpc_window {
    int first;   // first check (layered index)
    int count;   // checks in the window (<= kWindowSlots)
};

struct ldpc_code {
    int n = 0, m = 0, e = 0, n_groups = 0, max_deg = 0;
    std::vector<int> group_deg, group_cnt;
    std::vector<uint32_t> edge_var;          // [E] layered order
    // per-check (layered order)
    std::vector<int> check_deg, check_start, check_group;

    // DVB-S2 Annex-B rows when the code was built from a table (encoder)
    int dvbs2_q = 0;
    std::vector<int> dvbs2_row_len, dvbs2_row_addr;

    // ---- schedule plan for the windowed kernel (plan.cpp) ----
    bool staircase = false;       // check i+1 reads the var check i wrote last (DVB-S2 chain)
    int min_hazard = 0;           // min distance between two touches of one non-chain var
    int win_slots = 0;            // window width used by the plan (0 = no plan)
    std::vector<ldpc_window> windows;
    // per check: slot of the chain-in edge (-1: none), chain-out edge (-1: none)
    std::vector<int8_t> chain_in, chain_out;
};

// windowed2 dynamic-LDS pad of a context (capi.hip; mixed batches)
int ldpc_ctx_set_lds_pad(ldpc_ctx *c, int bytes);
// can kernel k (ldpc_ctx_set_kernel numbering) schedule this context's code?
// (no error is recorded either way)
bool ldpc_ctx_has_kernel(const ldpc_ctx *c, int k);

// error reporting (capi.cpp)
int ldpc_set_error(int status, const char *fmt, ...);

// finishes derived fields + plan; returns LDPC_OK or error
int ldpc_code_finalize(ldpc_code *h);
