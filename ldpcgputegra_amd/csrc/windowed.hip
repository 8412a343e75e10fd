// windowed.hip -- placeholder; the windowed kernel lands in the next step.
#include "windowed.h"

bool windowed_supported(const ldpc_code *) { return false; }
bool windowed_params_ok(const ldpc_params *) { return false; }
int windowed_code_upload(const ldpc_code *, WindowedCode *w)
{
    *w = WindowedCode{};
    return LDPC_OK;
}
void windowed_code_free(WindowedCode *w) { *w = WindowedCode{}; }
size_t windowed_msg_bytes(const ldpc_code *h, int stride) { return (size_t)h->e * stride; }
int launch_windowed(const DecodeLaunch &, const WindowedCode &, hipStream_t) { return -1; }
