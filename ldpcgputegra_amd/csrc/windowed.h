// windowed.h -- the windowed layered kernel (staircase / DVB-S2 fast path).
#pragma once
#include "kernels.h"
#include "ldpc_internal.h"

struct WindowedCode {
    int valid;
    int d0;                 // degree of group 0 (group 1 has d0 - 1)
    int max_deg;
    int n_windows;
    int g0_end;             // first window of group 1
    uint32_t *d_slotvar;    // per window [D][16] variable indices
    uint32_t *d_slotoff;    // [n_windows]
    uint8_t *d_flags;       // [n_windows][16]
    int *d_first;           // [n_windows]
    int *d_cnt;             // [n_windows]
};

// windowed2.hip: z-domain chain, S = 16 (P = 2) or S = 32 (P = 1) checks per window
struct Windowed2Code {
    int valid;
    int S, P, d0;
    int n_windows;
    int g0_end;
    uint32_t *d_slotvar;
};
bool windowed2_params_ok(const ldpc_params *p);
int windowed2_upload(const ldpc_code *h, int S, int P, Windowed2Code *w);
void windowed2_free(Windowed2Code *w);
int launch_windowed2(const DecodeLaunch &L, const Windowed2Code &w, hipStream_t s);

bool windowed_kernel_available();
bool windowed_supported(const ldpc_code *h);
bool windowed_params_ok(const ldpc_params *p);
int windowed_code_upload(const ldpc_code *h, WindowedCode *w);
void windowed_code_free(WindowedCode *w);
size_t windowed_msg_bytes(const ldpc_code *h, int stride);
int launch_windowed(const DecodeLaunch &L, const WindowedCode &w, hipStream_t s);
