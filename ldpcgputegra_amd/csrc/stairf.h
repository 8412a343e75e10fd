// stairf.h -- float layered min-sum for staircase (DVB-S2 IRA) codes, kernel 11.
#pragma once
#include <cstddef>
#include <cstdint>

#include "kernels.h"
#include "ldpc_internal.h"

struct StairfCode {
    bool valid = false;
    int X = 0;               // information edges per check (check degree - 2)
    int m = 0;               // checks
    int x0 = 0;              // node of check 0's chain input (the tail check's parity edge)
    // per group width S = 4, 8, 16, 2 (null: not usable for this code):
    // [M / S][(X + 3) / 2][S] u32: per check X info nodes, x node, o node (u16 pairs)
    uint32_t *d_tab[4] = {nullptr, nullptr, nullptr, nullptr};
};

// plan + device table; leaves sc->valid false (and returns LDPC_OK) when the
// code has no staircase structure the kernel takes
int stairf_upload(const ldpc_code *h, StairfCode *sc);
void stairf_free(StairfCode *sc);
// V offsets are u32 bytes: (n + 1) * stride * 4 < 2^32 (stride <= 16384 for n = 64800)
bool stairf_stride_ok(const StairfCode &sc, int n, int stride);
// message scratch of one decode (the kernel's own layout, zeroed by the caller)
size_t stairf_msg_bytes(const StairfCode &sc, int stride);
int launch_stairf(const DecodeLaunch &L, const StairfCode &sc, hipStream_t s);
