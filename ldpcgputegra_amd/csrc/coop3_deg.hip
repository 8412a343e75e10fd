// coop3_deg.hip -- coop3_decode instantiated for ONE first-group degree
// (C3_DEG, set by the Makefile: one object per degree, compiled in parallel)
#include "coop3_kernel.h"

#ifndef C3_DEG
#error "C3_DEG (first-group degree: 7, 10, 14, 22, 27 or 30) must be defined"
#endif
#define C3_CAT2(a, b) a##b
#define C3_CAT(a, b) C3_CAT2(a, b)

int C3_CAT(coop3_launch_d, C3_DEG)(const c3::Coop3Args &a, int grid, bool et, bool nms, bool stamped, hipStream_t s)
{
    return c3::launch_d0<C3_DEG>(a, grid, et, nms, stamped, s);
}
