// ldpc_sim.cpp -- native Monte-Carlo BER/FER driver over the C-ABI.
//
// The caller side of the boundary, re-designed from the reference's simulator
// loop (code/x86/main_p.cpp:404-656: SNR sweep, frame-error limit, per-SNR
// report line of code/x86/CTerminal/CTerminal.cpp:78-90, error counting of
// code/x86/CErrorAnalyzer/CErrorAnalyzer.cpp:123-194).  Differences by
// design: the channel runs on the GPU (integer-exact generator), one host
// thread drives each GPU with batches of thousands of codewords, and the
// output is one text line plus one JSON line per SNR.
//
//   ldpc_sim -code dvbs2_r1_2 -min 0.8 -max 1.2 -pas 0.1 -iter 50 -fer 100
//            [-batch 4096] [-frames 1000000] [-OMS 1 | -NMS 29 | -MS]
//            [-encoder] [-et] [-gpus N] [-seed S] [-kernel K]
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include <hip/hip_runtime.h>

#include "../../include/ldpc_mi355x.h"

namespace {

struct Opt {
    std::string code = "dvbs2_r1_2";
    double min = 0.5, max = 3.0, pas = 0.1;
    int iter = 30, fer = 100, batch = 4096, gpus = 1, kernel = 0;
    long frames = 1 << 20;
    bool encoder = false;
    ldpc_params p{};
    uint64_t seed = 1;
};

#define CHECK(x)                                                                              \
    do {                                                                                      \
        int _r = (x);                                                                         \
        if (_r != LDPC_OK) {                                                                  \
            fprintf(stderr, "%s failed: %s (%s)\n", #x, ldpc_strerror(_r), ldpc_last_error()); \
            exit(1);                                                                          \
        }                                                                                     \
    } while (0)

std::string code_path(const std::string &name, const char *argv0)
{
    if (name.find('/') != std::string::npos) return name;
    std::string dir(argv0);
    dir = dir.substr(0, dir.rfind('/') + 1);   // .../ldpcgputegra_amd/bin/
    for (const char *ext : {".ldpc", ".txt"}) {
        std::string p = dir + "../codes/" + name + ext;
        if (FILE *f = fopen(p.c_str(), "rb")) {
            fclose(f);
            return p;
        }
    }
    return name;
}

struct Totals {
    std::atomic<long> frames{0}, fe{0}, be{0};
};

void worker(int dev, const ldpc_code *h, const Opt &o, double sigma, Totals &tot, int n, int k,
            const std::vector<uint8_t> &pool, int pool_n)
{
    ldpc_ctx *ctx;
    CHECK(ldpc_ctx_create(h, dev, o.batch, &ctx));
    if (o.kernel) CHECK(ldpc_ctx_set_kernel(ctx, o.kernel));
    void *stream;
    CHECK(ldpc_ctx_stream(ctx, &stream));
    uint32_t table[64];
    CHECK(ldpc_awgn_i8_table(sigma, 8, 31, table));
    int8_t *d_llr;
    uint8_t *d_hard, *d_cw = nullptr;
    unsigned long long *d_cnt;
    (void)hipSetDevice(dev);
    if (hipMalloc(&d_llr, (size_t)o.batch * n) || hipMalloc(&d_hard, (size_t)o.batch * n) ||
        hipMalloc(&d_cnt, 16)) {
        fprintf(stderr, "hipMalloc failed\n");
        exit(1);
    }
    if (o.encoder) {
        // the codeword pool replicated over the batch (noise differs per codeword)
        std::vector<uint8_t> rep((size_t)o.batch * n);
        for (int b = 0; b < o.batch; b++) memcpy(&rep[(size_t)b * n], &pool[(size_t)(b % pool_n) * n], n);
        if (hipMalloc(&d_cw, rep.size()) || hipMemcpy(d_cw, rep.data(), rep.size(), hipMemcpyHostToDevice)) {
            fprintf(stderr, "codeword upload failed\n");
            exit(1);
        }
    }
    for (long batch_no = dev;; batch_no += o.gpus) {
        if (tot.fe.load() >= o.fer || tot.frames.load() >= o.frames) break;
        const uint64_t first = (uint64_t)batch_no * o.batch;
        (void)hipMemsetAsync(d_cnt, 0, 16, (hipStream_t)stream);
        CHECK(ldpc_awgn_i8_async(ctx, stream, d_llr, o.batch, first, o.seed, table, d_cw));
        CHECK(ldpc_decode_i8_async(ctx, stream, d_llr, d_hard, nullptr, nullptr, o.batch, o.iter, &o.p));
        CHECK(ldpc_count_errors_async(ctx, stream, d_hard, o.batch, k, d_cw, d_cnt));
        unsigned long long c[2];
        if (hipMemcpyAsync(c, d_cnt, 16, hipMemcpyDeviceToHost, (hipStream_t)stream) != hipSuccess ||
            hipStreamSynchronize((hipStream_t)stream) != hipSuccess) {
            fprintf(stderr, "device error: %s\n", hipGetErrorString(hipGetLastError()));
            exit(1);
        }
        tot.be += (long)c[0];
        tot.fe += (long)c[1];
        tot.frames += o.batch;
    }
    (void)hipFree(d_llr);
    (void)hipFree(d_hard);
    (void)hipFree(d_cnt);
    if (d_cw) (void)hipFree(d_cw);
    ldpc_ctx_destroy(ctx);
}

}  // namespace

int main(int argc, char **argv)
{
    Opt o;
    ldpc_params_default(&o.p);
    for (int i = 1; i < argc; i++) {
        std::string a = argv[i];
        auto nxt = [&]() { return (i + 1 < argc) ? argv[++i] : (fprintf(stderr, "missing value\n"), exit(2), ""); };
        if (a == "-code") o.code = nxt();
        else if (a == "-min") o.min = atof(nxt());
        else if (a == "-max") o.max = atof(nxt());
        else if (a == "-pas") o.pas = atof(nxt());
        else if (a == "-iter") o.iter = atoi(nxt());
        else if (a == "-fer") o.fer = atoi(nxt());
        else if (a == "-frames") o.frames = atol(nxt());
        else if (a == "-batch") o.batch = atoi(nxt());
        else if (a == "-gpus") o.gpus = atoi(nxt());
        else if (a == "-kernel") o.kernel = atoi(nxt());
        else if (a == "-seed") o.seed = strtoull(nxt(), nullptr, 10);
        else if (a == "-OMS") { o.p.algo = LDPC_ALGO_OMS; o.p.offset = atoi(nxt()); }
        else if (a == "-NMS") { o.p.algo = LDPC_ALGO_NMS; o.p.factor = atoi(nxt()); }
        else if (a == "-MS") o.p.algo = LDPC_ALGO_MS;
        else if (a == "-encoder") o.encoder = true;
        else if (a == "-et") o.p.early_term = 1;
        else {
            fprintf(stderr, "unknown option %s\n", a.c_str());
            return 2;
        }
    }
    ldpc_code *h;
    CHECK(ldpc_code_load(code_path(o.code, argv[0]).c_str(), &h));
    int n, m, e, ng, md;
    CHECK(ldpc_code_info(h, &n, &m, &e, &ng, &md));
    const int k = n - m;
    int ndev = 0;
    ldpc_device_count(&ndev);
    if (ndev < o.gpus) {
        fprintf(stderr, "need %d GPUs, %d visible\n", o.gpus, ndev);
        return 1;
    }
    std::vector<uint8_t> pool;
    int pool_n = 0;
    if (o.encoder) {
        pool_n = 64;
        std::vector<uint8_t> info((size_t)pool_n * k);
        std::mt19937_64 rng(o.seed);
        for (auto &b : info) b = rng() & 1;
        pool.resize((size_t)pool_n * n);
        CHECK(ldpc_dvbs2_encode(h, info.data(), pool.data(), pool_n));
    }
    printf("(II) code %s N=%d K=%d E=%d | %s | iters %d | batch %d x %d GPU(s)\n", o.code.c_str(), n, k, e,
           o.p.algo == LDPC_ALGO_NMS ? "NMS" : (o.p.algo == LDPC_ALGO_MS ? "MS" : "OMS"), o.iter, o.batch, o.gpus);
    for (double eb = o.min; eb <= o.max + 1e-9; eb += o.pas) {
        const double sigma = ldpc_awgn_sigma(eb, (double)k / n);
        Totals tot;
        auto t0 = std::chrono::steady_clock::now();
        std::vector<std::thread> th;
        for (int d = 0; d < o.gpus; d++)
            th.emplace_back(worker, d, h, std::cref(o), sigma, std::ref(tot), n, k, std::cref(pool), pool_n);
        for (auto &t : th) t.join();
        const double sec = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        const long fr = tot.frames, fe = tot.fe, be = tot.be;
        const double ber = (double)be / fr / k, fer = (double)fe / fr;
        const double mbps = (double)fr * n / sec / 1e6;
        // CTerminal::final_report (code/x86/CTerminal/CTerminal.cpp:78-90) format
        printf("SNR = %.2f | BER =  %2.3e | FER =  %2.3e | BPS =  %2.2f | MATRICES = %10ld| FE = %ld | BE = %ld | "
               "BE/FE = %.1f | RUNTIME = %.2fs\n",
               eb, ber, fer, (double)fr * k / sec / 1e6, fr, fe, be, fe ? (double)be / fe : 0.0, sec);
        printf("{\"ebn0\": %.3f, \"sigma\": %.6f, \"frames\": %ld, \"frame_errors\": %ld, \"bit_errors\": %ld, "
               "\"ber\": %.6e, \"fer\": %.6e, \"coded_mbps\": %.3f}\n",
               eb, sigma, fr, fe, be, ber, fer, mbps);
        fflush(stdout);
    }
    ldpc_code_destroy(h);
    return 0;
}
