// windowed.h -- the windowed layered kernel (staircase / DVB-S2 fast path).
#pragma once
#include "kernels.h"
#include "ldpc_internal.h"

struct WindowedCode {
    int valid;
    int max_deg;
    int words;             // 32-bit words per compressed check message (1 or 2)
    int n_windows;
    int *d_win;            // [n_windows] packed (first | count << 24) ... see windowed.hip
    uint32_t *d_slot;      // per check slot descriptors
};

bool windowed_supported(const ldpc_code *h);
bool windowed_params_ok(const ldpc_params *p);
int windowed_code_upload(const ldpc_code *h, WindowedCode *w);
void windowed_code_free(WindowedCode *w);
size_t windowed_msg_bytes(const ldpc_code *h, int stride);
int launch_windowed(const DecodeLaunch &L, const WindowedCode &w, hipStream_t s);
