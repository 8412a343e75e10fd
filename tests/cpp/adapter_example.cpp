// Reference-shaped caller (as code/x86/main_p.cpp:377-396,485) compiled against
// include/ldpc_mi355x.hpp.  Exit 0 = ok, 3 = no GPU (construction threw
// LDPC_EDEVICE as documented), anything else = failure.
#include <cstdio>
#include <vector>

#include "ldpc_mi355x.hpp"

int main(int argc, char **argv)
{
    using namespace ldpc_mi355x;
    const char *path = argc > 1 ? argv[1] : "ldpcgputegra_amd/codes/576x288.ldpc";
    Code H(path);
    const int N = H.n(), frames = 16;
    param_decoder p;
    CDecoder_fixed *dec = nullptr;
    try {
        dec = CreateDecoder("OMS", "mi355x", "fixed", p, -127, 127, -31, 31, H, frames);
    } catch (const Error &e) {
        std::printf("no device: %s\n", e.what());
        return e.status == LDPC_EDEVICE ? 3 : 1;
    }
    // noiseless all-zero codeword: every LLR -31 -> every decision 0
    std::vector<char> llr((size_t)frames * N, -31), hard((size_t)frames * N, 7);
    dec->decode(llr.data(), hard.data(), 20);
    for (char h : hard)
        if (h != 0) return 2;
    // setOffset twice is an error, as in the reference (exit there, throw here)
    try {
        static_cast<CDecoder_OMS_fixed_MI355X *>(dec)->setOffset(2);
        return 4;
    } catch (const Error &) {
    }
    delete dec;
    std::printf("ok\n");
    return 0;
}
