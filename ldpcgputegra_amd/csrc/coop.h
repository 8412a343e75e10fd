// coop.h -- the workgroup-cooperative DVB-S2 fast path (coop.hip).
#pragma once
#include "kernels.h"
#include "ldpc_internal.h"

struct CoopCode {
    int valid;
    int d0;          // degree of the first group (the tail check has d0 - 1)
    int S, R;        // checks per window, prefetch depth in windows
    int nw;          // windows per iteration (tail and empty windows included)
    int tail;        // window index of the tail check
    int n_fwd;       // forwarded info-edge reads per iteration (plan statistic)
    uint32_t *d_tab; // [nw][S][recw]
};

bool coop_params_ok(const ldpc_params *p);
int coop_upload(const ldpc_code *h, CoopCode *cc);
void coop_free(CoopCode *cc);
int launch_coop(const DecodeLaunch &L, const CoopCode &cc, hipStream_t s);
// host-side plan (tests: ldpc_code_coop_plan)
int coop_plan_windows(const ldpc_code *h, int S, int R, std::vector<int> &first, std::vector<int> &count, int *tail,
                      int *n_fwd);
