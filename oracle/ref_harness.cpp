// ref_harness.cpp -- C entry points around the REFERENCE's own SSE decoders.
//
// TEST INFRASTRUCTURE ONLY.  Compiled by oracle/Makefile together with the
// unmodified sources under /root/reference/code/x86 into oracle/_ref/<code>/
// libref.so (one library per code, because the reference selects H at compile
// time through Constantes/constantes_sse.h).  Used to
//   * generate the golden vectors committed under tests/golden/, and
//   * time the reference on the host (bench.py cpu_baseline, kind "reference").
// It drives CDecoder_OMS_fixed_SSE / CDecoder_NMS_fixed_SSE exactly as the
// reference's own driver does (code/x86/CDecoder/DecoderLibrary.h:78-83,
// code/x86/main_p.cpp:485): 16 frame-major codewords per decode() call.
#include <cstdint>
#include <cstring>
#include <thread>
#include <vector>

#include "CDecoder/OMS/CDecoder_OMS_fixed_SSE.h"
#include "CDecoder/NMS/CDecoder_NMS_fixed_SSE.h"

namespace {

CDecoder_fixed_SSE *make(int algo, int param, int vmin, int vmax, int mmin, int mmax)
{
    if (algo == 0) {
        auto *d = new CDecoder_OMS_fixed_SSE();
        d->setOffset(param);
        d->setVarRange(vmin, vmax);
        d->setMsgRange(mmin, mmax);
        return d;
    }
    auto *d = new CDecoder_NMS_fixed_SSE();
    d->setFactor(param);
    d->setVarRange(vmin, vmax);
    d->setMsgRange(mmin, mmax);
    return d;
}

// 16-byte aligned staging (uchar_transpose_sse uses aligned loads)
struct Stage {
    char *in, *out;
    void *raw_in, *raw_out;
    explicit Stage(size_t n)
    {
        raw_in = aligned_alloc(64, (n + 63) / 64 * 64);
        raw_out = aligned_alloc(64, (n + 63) / 64 * 64);
        in = (char *)raw_in;
        out = (char *)raw_out;
    }
    ~Stage() { free(raw_in); free(raw_out); }
};

void run(const int8_t *llr, uint8_t *hard, int nframes, int iters, int algo, int param,
         int vmin, int vmax, int mmin, int mmax)
{
    CDecoder_fixed_SSE *d = make(algo, param, vmin, vmax, mmin, mmax);
    const size_t blk = (size_t)16 * NOEUD;
    Stage st(blk);
    for (int f = 0; f < nframes; f += 16) {
        std::memcpy(st.in, llr + (size_t)f * NOEUD, blk);
        static_cast<CDecoder *>(d)->decode(st.in, st.out, iters);  // char* overload (CDecoder.h:37)
        std::memcpy(hard + (size_t)f * NOEUD, st.out, blk);
    }
    delete d;
}

}  // namespace

extern "C" {

int ref_code_info(int *n, int *m, int *e)
{
    *n = NOEUD;
    *m = _K;
    *e = MESSAGE;
    return 0;
}

// nframes must be a multiple of 16 (the reference decodes 16 frames per call)
int ref_decode(const int8_t *llr, uint8_t *hard, int nframes, int iters, int algo, int param,
               int vmin, int vmax, int mmin, int mmax)
{
    if (nframes % 16) return -1;
    if (vmax != 127) return -1;  // the reference would exit(0)
    run(llr, hard, nframes, iters, algo, param, vmin, vmax, mmin, mmax);
    return 0;
}

// Throughput leg for bench.py: `threads` decoder objects (as main_p.cpp's
// OpenMP sections, :473-576), each decoding its share of 16-frame blocks.
int ref_decode_mt(const int8_t *llr, uint8_t *hard, int nframes, int iters, int offset, int threads)
{
    if (nframes % 16 || threads < 1) return -1;
    int blocks = nframes / 16;
    std::vector<std::thread> pool;
    for (int t = 0; t < threads; t++) {
        int b0 = (int)((long)blocks * t / threads), b1 = (int)((long)blocks * (t + 1) / threads);
        if (b1 <= b0) continue;
        pool.emplace_back([=] {
            run(llr + (size_t)b0 * 16 * NOEUD, hard + (size_t)b0 * 16 * NOEUD, (b1 - b0) * 16, iters,
                0, offset, -127, 127, -31, 31);
        });
    }
    for (auto &th : pool) th.join();
    return 0;
}

}  // extern "C"
