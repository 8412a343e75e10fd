// capi.hip -- the C-ABI decoder context and decode entry points
// (include/ldpc_mi355x.h).  Host code only; kernels live in generic.hip,
// windowed.hip and layout.hip.
//
// A context mirrors the reference decoder objects: it owns the device scratch
// (V and messages, allocated up front for max_batch codewords, as
// CDecoder_fixed_SSE's constructor does, code/x86/CDecoder/template/
// CDecoder_fixed_SSE.cpp:23-27, and CGPUDecoder(nb_frames, n, k, m),
// code/gpu_fixed/decoder_template/CGPUDecoder.cpp:14-38) plus its own HIP
// stream -- created once, not per call as the reference's decode_stream does
// (code/gpu_fixed/decoder_ms/CGPU_Decoder_MS_SIMD.cu:223-224).
#include <algorithm>
#include <climits>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <mutex>

#include "kernels.h"
#include "ldpc_internal.h"
#include "windowed.h"
#include "coop.h"
#include "stairf.h"
#include "lds.h"
#include "host.h"

#define HIP_TRY(expr)                                                                          \
    do {                                                                                       \
        hipError_t _e = (expr);                                                                \
        if (_e != hipSuccess)                                                                  \
            return ldpc_set_error(LDPC_EDEVICE, "%s: %s", #expr, hipGetErrorString(_e));       \
    } while (0)

// per-decode device scratch (lazily sized)
struct Scratch {
    void *d_V = nullptr;
    size_t V_bytes = 0;
    void *d_msg = nullptr;
    size_t msg_bytes = 0;
    void *d_early = nullptr;        // coop early termination: live[stride] u8, bad[stride] u32, iters[stride]
    size_t early_bytes = 0;
    void *d_V2 = nullptr;           // coop3 staged early termination: compacted state, map | iterations | count
    size_t V2_bytes = 0;
    void *d_et2 = nullptr;
    size_t et2_bytes = 0;
    void release()
    {
        (void)hipFree(d_V);
        (void)hipFree(d_msg);
        (void)hipFree(d_early);
        (void)hipFree(d_V2);
        (void)hipFree(d_et2);
        *this = Scratch{};
    }
};

struct Lane {
    hipStream_t stream = nullptr;
    Scratch sc;
    void *d_io = nullptr;           // chunk input (LLRs) | output (hard decisions)
    size_t io_bytes = 0;
    hipEvent_t h2d_done = nullptr;  // this lane's input copy finished (the next lane's copy waits on it)
};

struct ldpc_ctx {
    const ldpc_code *code = nullptr;
    int device = 0;
    int max_batch = 0;
    int max_stride = 0;
    int kernel = 0;                 // 0 auto, 1 generic, 2 windowed, 3 windowed2 (S16), 5 coop, 7 lds, 8 coop3,
                                    // 9 ldsep (edge-parallel float)
                                    // (4 and 6, windowed2 S32 and coop2, were superseded and removed)
    int last_kernel = 0;
    int last_et_stage = 0;          // coop3 staged early termination: first-stage iterations (0: one launch)
    int last_skipped = 0;   // the preferred kernel the last decode could not use at its batch size (0: none)
    int lds_pad = 0;        // extra dynamic LDS per windowed2 workgroup (ldpc_ctx_set_lds_pad)
    hipStream_t stream = nullptr;
    // device copy of the code
    uint32_t *d_edge_var = nullptr;
    int *d_group_deg = nullptr, *d_group_cnt = nullptr;
    WindowedCode wcode{};           // windowed-kernel tables (windowed.hip)
    Windowed2Code w16{};            // windowed2.hip tables, S = 16
    CoopCode coop{};                // coop.hip tables (workgroup-cooperative DVB-S2 path)
    CoopCode coop3{};               // coop3.hip tables (pre + post slab waves, i16 chain, D0 = 7)
    LdsCode lds{};                  // lds.hip tables (LDS-resident short-code decoder)
    StairfCode stairf{};            // stairf.hip table (float staircase codes)
    Scratch sc;                     // device-API decodes and the unchunked host path
    void *d_io = nullptr;           // staging for the quantiser's host-buffer API
    size_t io_bytes = 0;
    // host-buffer API pipeline (decode_host): chunk i of a batch runs on lane
    // i % lanes.size(): its own stream, scratch and input / output staging
    std::vector<Lane> lanes;
    // asynchronous host-buffer API: an event of the context's own, recorded
    // after each call's D2H copy (ldpc_ctx_synchronize / destroy wait on it,
    // never on the caller's stream, which may be gone by then; a call on
    // another stream waits on it before reusing d_io and the scratch)
    hipEvent_t host_done = nullptr;
    bool host_pending = false;
    // kernel timing (ldpc_ctx_profile)
    bool profile = false;
    std::vector<std::pair<hipEvent_t, hipEvent_t>> events;
};

static int getenv_int(const char *name, int def)
{
    const char *e = getenv(name);
    return (e && *e) ? atoi(e) : def;
}

static int ensure(void **p, size_t *have, size_t need)
{
    if (*have >= need) return LDPC_OK;
    if (*p) (void)hipFree(*p);
    *p = nullptr;
    *have = 0;
    hipError_t e = hipMalloc(p, need);
    if (e != hipSuccess) {
        *p = nullptr;
        return ldpc_set_error(LDPC_ENOMEM, "hipMalloc(%zu): %s", need, hipGetErrorString(e));
    }
    *have = need;
    return LDPC_OK;
}

extern "C" int ldpc_device_count(int *count)
{
    if (!count) return ldpc_set_error(LDPC_EINVAL, "count is NULL");
    int c = 0;
    hipError_t e = hipGetDeviceCount(&c);
    *count = (e == hipSuccess) ? c : 0;
    return LDPC_OK;
}

// device = -1: a host context (host.cpp) -- host-buffer decodes on the CPU,
// no HIP call at all; the device-pointer entry points reject it
static int host_only(const ldpc_ctx *c)
{
    return ldpc_set_error(LDPC_EUNSUPPORTED, "context %p is a host context (device -1): device buffers need a GPU "
                          "context", (const void *)c);
}

extern "C" int ldpc_ctx_create(const ldpc_code *h, int device, int max_batch, ldpc_ctx **out)
{
    if (!out) return ldpc_set_error(LDPC_EINVAL, "out is NULL");
    *out = nullptr;
    if (!h || max_batch <= 0) return ldpc_set_error(LDPC_EINVAL, "NULL code or max_batch <= 0");
    if (h->max_deg > 32) return ldpc_set_error(LDPC_EUNSUPPORTED, "check degree %d > 32", h->max_deg);
    if (device == -1) {
        auto *c = new ldpc_ctx();
        c->code = h;
        c->device = -1;
        c->max_batch = max_batch;
        c->max_stride = (max_batch + 63) / 64 * 64;
        *out = c;
        return LDPC_OK;
    }
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0)
        return ldpc_set_error(LDPC_EDEVICE, "no HIP device visible");
    if (device < 0 || device >= ndev) return ldpc_set_error(LDPC_EINVAL, "device %d of %d", device, ndev);
    HIP_TRY(hipSetDevice(device));
    auto *c = new ldpc_ctx();
    c->code = h;
    c->device = device;
    c->max_batch = max_batch;
    c->max_stride = (max_batch + 63) / 64 * 64;
    int rc = LDPC_OK;
    auto fail = [&](int r) {
        ldpc_ctx_destroy(c);
        return r;
    };
    if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess)
        return fail(ldpc_set_error(LDPC_EDEVICE, "hipStreamCreate"));
    if (hipMalloc(&c->d_edge_var, 4ull * h->e) != hipSuccess ||
        hipMalloc(&c->d_group_deg, sizeof(int) * h->n_groups) != hipSuccess ||
        hipMalloc(&c->d_group_cnt, sizeof(int) * h->n_groups) != hipSuccess)
        return fail(ldpc_set_error(LDPC_ENOMEM, "code tables"));
    if (hipMemcpy(c->d_edge_var, h->edge_var.data(), 4ull * h->e, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(c->d_group_deg, h->group_deg.data(), sizeof(int) * h->n_groups, hipMemcpyHostToDevice) !=
            hipSuccess ||
        hipMemcpy(c->d_group_cnt, h->group_cnt.data(), sizeof(int) * h->n_groups, hipMemcpyHostToDevice) !=
            hipSuccess)
        return fail(ldpc_set_error(LDPC_EDEVICE, "code table upload"));
    if ((rc = windowed_code_upload(h, &c->wcode)) != LDPC_OK) return fail(rc);
    if ((rc = windowed2_upload(h, 16, 2, &c->w16)) != LDPC_OK) return fail(rc);
    if ((rc = coop_upload(h, &c->coop)) != LDPC_OK) return fail(rc);
    if ((rc = coop3_upload(h, &c->coop3)) != LDPC_OK) return fail(rc);
    if ((rc = lds_upload(h, &c->lds)) != LDPC_OK) return fail(rc);
    if ((rc = stairf_upload(h, &c->stairf)) != LDPC_OK) return fail(rc);
    *out = c;
    return LDPC_OK;
}

extern "C" void ldpc_ctx_destroy(ldpc_ctx *c)
{
    if (!c) return;
    if (c->device < 0) {
        delete c;
        return;
    }
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    if (c->host_pending) (void)hipEventSynchronize(c->host_done);
    if (c->host_done) (void)hipEventDestroy(c->host_done);
    windowed_code_free(&c->wcode);
    windowed2_free(&c->w16);
    coop_free(&c->coop);
    coop_free(&c->coop3);
    lds_free(&c->lds);
    stairf_free(&c->stairf);
    for (auto &pr : c->events) {
        (void)hipEventDestroy(pr.first);
        (void)hipEventDestroy(pr.second);
    }
    (void)hipFree(c->d_edge_var);
    (void)hipFree(c->d_group_deg);
    (void)hipFree(c->d_group_cnt);
    c->sc.release();
    (void)hipFree(c->d_io);
    for (Lane &l : c->lanes) {
        if (l.stream) (void)hipStreamSynchronize(l.stream);
        l.sc.release();
        (void)hipFree(l.d_io);
        if (l.h2d_done) (void)hipEventDestroy(l.h2d_done);
        if (l.stream) (void)hipStreamDestroy(l.stream);
    }
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
}

extern "C" int ldpc_ctx_stream(ldpc_ctx *c, void **s)
{
    if (!c || !s) return ldpc_set_error(LDPC_EINVAL, "NULL ctx/stream");
    *s = (void *)c->stream;
    return LDPC_OK;
}

bool ldpc_ctx_has_kernel(const ldpc_ctx *c, int k)
{
    if (!c || k < 0 || k > 11 || k == 10) return false;
    if (c->device < 0) return k == 0;
    return !((k == 2 && !windowed_supported(c->code)) || (k == 3 && !c->w16.valid) || k == 4 ||
             (k == 5 && !c->coop.valid) || k == 6 || (k == 7 && !c->lds.valid) || (k == 8 && !c->coop3.valid) ||
             (k == 9 && !c->lds.ep_valid) || (k == 11 && !c->stairf.valid));
}

extern "C" int ldpc_ctx_set_kernel(ldpc_ctx *c, int k)
{
    if (!c || k < 0 || k > 11 || k == 10) return ldpc_set_error(LDPC_EINVAL, "kernel must be 0 (auto) .. 9 or 11");
    if (!ldpc_ctx_has_kernel(c, k)) return ldpc_set_error(LDPC_EUNSUPPORTED, "kernel %d cannot schedule this code", k);
    c->kernel = k;
    return LDPC_OK;
}

extern "C" int ldpc_ctx_profile(ldpc_ctx *c, int enable)
{
    if (!c) return ldpc_set_error(LDPC_EINVAL, "NULL ctx");
    c->profile = enable != 0;
    return LDPC_OK;
}

extern "C" int ldpc_ctx_kernel_time(ldpc_ctx *c, double *total_ms, int *launches, int reset)
{
    if (!c) return ldpc_set_error(LDPC_EINVAL, "NULL ctx");
    if (c->device < 0) {   // host context: no kernels
        if (total_ms) *total_ms = 0.0;
        if (launches) *launches = 0;
        return LDPC_OK;
    }
    HIP_TRY(hipSetDevice(c->device));
    double tot = 0.0;
    for (auto &pr : c->events) {
        HIP_TRY(hipEventSynchronize(pr.second));
        float ms = 0.f;
        HIP_TRY(hipEventElapsedTime(&ms, pr.first, pr.second));
        tot += ms;
    }
    if (total_ms) *total_ms = tot;
    if (launches) *launches = (int)c->events.size();
    if (reset) {
        for (auto &pr : c->events) {
            (void)hipEventDestroy(pr.first);
            (void)hipEventDestroy(pr.second);
        }
        c->events.clear();
    }
    return LDPC_OK;
}

// library-internal (mixed.hip): windowed2 workgroups of this context request
// `bytes` of dynamic LDS they do not use, so that none fits beside a coop3
// workgroup (124.5 KB of the CU's 160 KB): a mixed batch's windowed2 waves
// then stay off the CUs running the coop3 decode, whose slab waves are
// VALU-bound and would lose issue slots to them
int ldpc_ctx_set_lds_pad(ldpc_ctx *c, int bytes)
{
    if (!c || bytes < 0 || bytes > 65536) return ldpc_set_error(LDPC_EINVAL, "lds pad");
    c->lds_pad = bytes;
    return LDPC_OK;
}

extern "C" int ldpc_ctx_last_kernel(ldpc_ctx *c, int *k)
{
    if (!c || !k) return ldpc_set_error(LDPC_EINVAL, "NULL");
    *k = c->last_kernel;
    return LDPC_OK;
}

extern "C" int ldpc_ctx_last_skipped(ldpc_ctx *c, int *k)
{
    if (!c || !k) return ldpc_set_error(LDPC_EINVAL, "NULL");
    *k = c->last_skipped;
    return LDPC_OK;
}

extern "C" int ldpc_ctx_last_et_stage(ldpc_ctx *c, int *k)
{
    if (!c || !k) return ldpc_set_error(LDPC_EINVAL, "NULL");
    *k = c->last_et_stage;
    return LDPC_OK;
}

extern "C" int ldpc_ctx_get_kernel(ldpc_ctx *c, int *k)
{
    if (!c || !k) return ldpc_set_error(LDPC_EINVAL, "NULL");
    *k = c->kernel;
    return LDPC_OK;
}

static int check_params(const ldpc_ctx *c, int batch, int n_iter, const ldpc_params *p, bool is_float)
{
    if (batch < 0 || batch > c->max_batch)
        return ldpc_set_error(LDPC_EINVAL, "batch %d outside [0, max_batch=%d]", batch, c->max_batch);
    if (n_iter < 0) return ldpc_set_error(LDPC_EINVAL, "n_iter < 0");
    if (!p) return ldpc_set_error(LDPC_EINVAL, "params NULL");
    if (p->algo < 0 || p->algo > 2) return ldpc_set_error(LDPC_EINVAL, "algo %d", p->algo);
    if (!is_float) {
        // CDecoder_OMS_fixed_SSE::decode / CDecoder_NMS_fixed_SSE::decode exit
        // unless vSAT_POS_VAR == 127 (OMS .cpp:116-119, NMS .cpp:119-122)
        if (p->var_max != 127)
            return ldpc_set_error(LDPC_EUNSUPPORTED, "var_max must be 127 (reference decode_8bits only)");
        if (p->var_min < -128 || p->var_min > 0) return ldpc_set_error(LDPC_EINVAL, "var_min %d", p->var_min);
        if (p->msg_max < 0 || p->msg_max > 127) return ldpc_set_error(LDPC_EINVAL, "msg_max %d", p->msg_max);
        if (p->algo == LDPC_ALGO_OMS && (p->offset < 0 || p->offset > 255))
            return ldpc_set_error(LDPC_EINVAL, "offset %d", p->offset);
    }
    return LDPC_OK;
}

// kernel family for this call: 1 generic, 2 windowed, 3 windowed2 (S=16),
// 5 coop (workgroup-cooperative), 7 lds (LDS-resident short codes, int8 and
// float), 8 coop3 (slab waves doing pre + post, i16 chain).  last_skipped
// records the fastest kernel of this code that the automatic choice could not
// use for these parameters (algorithm, message / variable ranges), 0 if none
static int pick_kernel(ldpc_ctx *c, const ldpc_params *p, bool is_float, int stride)
{
    c->last_skipped = 0;
    const bool ld = lds_applicable(c->code, c->lds, is_float);
    if (c->kernel == 7) return ld ? 7 : -1;
    if (c->kernel == 9) return ldsep_applicable(c->code, c->lds, is_float) ? 9 : -1;
    const bool sf = c->stairf.valid && stairf_stride_ok(c->stairf, c->code->n, stride);
    if (c->kernel == 11) return (is_float && sf) ? 11 : -1;
    if (is_float) {
        if (c->kernel == 0 && ldsep_applicable(c->code, c->lds, true)) return 9;
        if (c->kernel == 0 && sf) return 11;
        return (c->kernel == 0 && lds_preferred(c->code, c->lds, true)) ? 7 : (c->kernel <= 1 ? 1 : -1);
    }
    const bool w1 = windowed_supported(c->code) && windowed_params_ok(p);
    const bool w2 = windowed2_params_ok(p);
    const bool co = c->coop.valid && coop_params_ok(p);
    const bool co3 = c->coop3.valid && coop3_params_ok(p, c->coop3) && coop3_stride_ok(stride) &&
                     (!p->early_term || coop3_et_in_kernel(c->coop3, c->code->n));
    switch (c->kernel) {
    case 1: return 1;
    case 2: return w1 ? 2 : -1;
    case 3: return (w2 && c->w16.valid) ? 3 : -1;
    case 5: return co ? 5 : -1;
    case 8: return co3 ? 8 : -1;
    case 4:
    case 6: return -1;
    default:
        if (co3) return 8;
        if (c->coop3.valid) c->last_skipped = 8;
        if (co) return 5;
        if (c->coop.valid && !c->last_skipped) c->last_skipped = 5;
        if (w2 && c->w16.valid) return 3;
        if (lds_preferred(c->code, c->lds, false)) return 7;
        if (w1) return 2;
        return 1;
    }
}

// alloc_only: size the scratch for this decode and return (decode_host sizes
// every lane before it queues any work: a hipFree mid-pipeline would wait for
// the device)
// error count requested with a decode (ldpc_decode_*_count_async)
struct ErrCount {
    int k;
    const uint8_t *ref;
    unsigned long long *counts;
};

static int decode_device(ldpc_ctx *c, Scratch &sc, hipStream_t s, const void *d_llr, uint8_t *d_hard, void *d_soft,
                         int32_t *d_iters, int batch, int n_iter, const ldpc_params *p, bool is_float,
                         bool alloc_only = false, size_t nm_ld = 0, const ErrCount *ec = nullptr)
{
    int rc = check_params(c, batch, n_iter, p, is_float);
    if (rc != LDPC_OK) return rc;
    if (c->device < 0) return host_only(c);
    if (batch == 0) return LDPC_OK;
    HIP_TRY(hipSetDevice(c->device));
    const ldpc_code *h = c->code;
    const int stride = (batch + 63) / 64 * 64;
    const size_t esz = is_float ? 4 : 1;
    const int kern = pick_kernel(c, p, is_float, stride);
    if (kern < 0)
        return ldpc_set_error(LDPC_EUNSUPPORTED, "kernel %d selected but not applicable to these params", c->kernel);
    c->last_kernel = kern;
    if ((kern == 7 || kern == 9) && alloc_only) return LDPC_OK;
    if (kern == 7 && nm_ld) {   // node-major input: transpose it to frame-major scratch first
        if ((rc = ensure(&sc.d_msg, &sc.msg_bytes, (size_t)h->n * batch)) != LDPC_OK) return rc;
        if (launch_deinterleave_i8((const int8_t *)d_llr, nullptr, (int8_t *)sc.d_msg, h->n, batch, (int)nm_ld, s))
            return ldpc_set_error(LDPC_EDEVICE, "node-major transpose: %s", hipGetErrorString(hipGetLastError()));
        d_llr = sc.d_msg;
    }
    if (kern == 7 || kern == 9) {   // LDS-resident: frame-major in and out, no scratch, no transposes
        DecodeLaunch L{};
        L.batch = batch;
        L.iters = n_iter;
        L.is_float = is_float;
        L.algo = (p->algo == LDPC_ALGO_MS) ? LDPC_ALGO_OMS : p->algo;
        L.param = (p->algo == LDPC_ALGO_NMS) ? p->factor : (p->algo == LDPC_ALGO_MS ? 0 : p->offset);
        L.var_min = p->var_min;
        L.msg_max = p->msg_max;
        L.early = p->early_term;
        L.beta = (p->algo == LDPC_ALGO_MS) ? 0.0f : p->beta;
        L.iters_used = d_iters;
        const bool fuse = ec && kern == 9 && getenv_int("LDPC_FUSED_COUNT", 1) != 0;
        if (fuse) {   // ldsep counts in its epilogue (one wave = one codeword)
            L.cnt = ec->counts;
            L.cnt_ref = ec->ref;
            L.cnt_k = ec->k;
        }
        hipEvent_t ev0 = nullptr, ev1 = nullptr;
        if (c->profile) {
            HIP_TRY(hipEventCreate(&ev0));
            HIP_TRY(hipEventCreate(&ev1));
            HIP_TRY(hipEventRecord(ev0, s));
        }
        const int lr = kern == 9 ? launch_ldsep(c->lds, h, (const float *)d_llr, d_hard, (float *)d_soft, batch,
                                                n_iter, L, s)
                                 : launch_lds(c->lds, h, d_llr, d_hard, d_soft, batch, n_iter, L, s);
        if (c->profile) {
            HIP_TRY(hipEventRecord(ev1, s));
            c->events.emplace_back(ev0, ev1);
        }
        if (lr) return ldpc_set_error(LDPC_EDEVICE, "lds decode launch: %s", hipGetErrorString(hipGetLastError()));
        if (ec && !fuse && launch_count_errors(d_hard, h->n, batch, ec->k, ec->ref, ec->counts, s))
            return ldpc_set_error(LDPC_EDEVICE, "count_errors: %s", hipGetErrorString(hipGetLastError()));
        return LDPC_OK;
    }
    const bool win = kern >= 2 && kern != 11;
    // + a sink row / sink words for the masked stores of the coop kernel
    const size_t msg_zero = (kern == 8    ? 0
                             : kern == 11 ? stairf_msg_bytes(c->stairf, stride)
                             : win        ? windowed_msg_bytes(h, stride)
                                      : (size_t)h->e * stride * esz) +
                            4096;
    // V row pitch (codewords): the coop kernel pads it by LDPC_VPITCH_PAD
    // (default 64; multiple of 64) codewords.  A workgroup touches its 16-B
    // piece of every row and the XCD remap gives each XCD a fixed 512-B window
    // of a row: with a power-of-two pitch (batch 4096) every row's window of an
    // XCD falls on the same few L2 channels.  Measured (DVB-S2 r1/2, 4096 cw,
    // 50 it, the row-layout coop3 of r02): pitch 4096 57.6 ms, 4160 / 4224
    // 49.7 / 49.6 ms, 4352 50.4, 4608 52.7, 5120 57.2.  coop3
    // keeps V grouped per 16 codewords instead (coop3_group_bytes per group).
    const int vpad = kern == 5 ? std::max(0, getenv_int("LDPC_VPITCH_PAD", 64)) / 64 * 64 : 0;
    const int vpitch = stride + vpad;
    size_t vpart = 0, vgroup = 0;   // coop3: per-group blocks of V rows then messages
    if (kern == 8) coop3_group_layout(h, &vpart, &vgroup);
    const size_t v_bytes = kern == 8 ? (size_t)(stride / 16) * vgroup
                                     : ((size_t)h->n + 1) * vpitch * esz;   // row n: the coop kernel's sink row
    if ((rc = ensure(&sc.d_V, &sc.V_bytes, v_bytes)) != LDPC_OK) return rc;
    if (kern != 8 && (rc = ensure(&sc.d_msg, &sc.msg_bytes, msg_zero)) != LDPC_OK) return rc;
    // early termination: live u8 | bad u32 | iterations used i32 (when the caller passed none)
    const bool et_state = (kern == 5 || kern == 8 || kern == 11) && p->early_term;
    if (et_state && (rc = ensure(&sc.d_early, &sc.early_bytes, (size_t)stride * 12)) != LDPC_OK) return rc;
    const bool et_staged = kern == 8 && p->early_term && coop3_et_stage_iters(batch, n_iter) > 0;
    if (!alloc_only) c->last_et_stage = et_staged ? coop3_et_stage_iters(batch, n_iter) : 0;
    if (et_staged && ((rc = ensure(&sc.d_V2, &sc.V2_bytes, 2 * v_bytes)) != LDPC_OK ||
                      (rc = ensure(&sc.d_et2, &sc.et2_bytes, (size_t)stride * 20 + 256)) != LDPC_OK))
        return rc;
    if (alloc_only) return LDPC_OK;
    // messages start at 0 (CDecoder_OMS_fixed_SSE.cpp:129-131); the all-zero
    // compressed word is the all-zero message set as well.
    if (kern == 8) {
        if (launch_zero_rows((char *)sc.d_V + vpart, vgroup, ((size_t)(h->m + 1) * coop3_mrec(h->group_deg[0]) + 15) / 16 * 16,
                             stride / 16, s))
            return ldpc_set_error(LDPC_EDEVICE, "message zeroing: %s", hipGetErrorString(hipGetLastError()));
    } else
        HIP_TRY(hipMemsetAsync(sc.d_msg, 0, msg_zero, s));
    if (nm_ld) {   // node-major input: 16-codeword pieces copied straight into V (no transpose)
        const size_t gstep = kern == 8 ? vgroup : 16, rstep = kern == 8 ? 16 : (size_t)vpitch;
        if (launch_nm_pieces_i8((const int8_t *)d_llr, nm_ld, h->n, batch, kern == 8 ? stride : vpitch, (int8_t *)sc.d_V,
                                gstep, rstep, s))
            return ldpc_set_error(LDPC_EDEVICE, "node-major load: %s", hipGetErrorString(hipGetLastError()));
    } else if (is_float) {
        if (launch_interleave_f32((const float *)d_llr, (float *)sc.d_V, h->n, batch, vpitch, s))
            return ldpc_set_error(LDPC_EDEVICE, "interleave: %s", hipGetErrorString(hipGetLastError()));
    } else if (kern == 8) {
        if (launch_interleave_grp_i8((const int8_t *)d_llr, (int8_t *)sc.d_V, h->n, batch, stride, vgroup, s))
            return ldpc_set_error(LDPC_EDEVICE, "interleave: %s", hipGetErrorString(hipGetLastError()));
    } else {
        if (launch_interleave_i8((const int8_t *)d_llr, (int8_t *)sc.d_V, h->n, batch, vpitch, s))
            return ldpc_set_error(LDPC_EDEVICE, "interleave: %s", hipGetErrorString(hipGetLastError()));
    }
    DecodeLaunch L{};
    L.V = sc.d_V;
    L.msg = kern == 8 ? (void *)((char *)sc.d_V + vpart) : sc.d_msg;
    L.vgroup = vgroup;
    L.stride = stride;
    L.vpitch = vpitch;
    L.batch = batch;
    L.iters = n_iter;
    L.is_float = is_float;
    L.d_edge_var = c->d_edge_var;
    L.d_group_deg = c->d_group_deg;
    L.d_group_cnt = c->d_group_cnt;
    L.n_groups = h->n_groups;
    L.n = h->n;
    L.m = h->m;
    L.e = h->e;
    L.algo = (p->algo == LDPC_ALGO_MS) ? LDPC_ALGO_OMS : p->algo;
    L.param = (p->algo == LDPC_ALGO_NMS) ? p->factor : (p->algo == LDPC_ALGO_MS ? 0 : p->offset);
    L.var_min = p->var_min;
    L.msg_max = p->msg_max;
    L.early = p->early_term;
    L.beta = (p->algo == LDPC_ALGO_MS) ? 0.0f : p->beta;
    L.iters_used = d_iters;
    L.lds_pad = c->lds_pad;
    L.V2 = et_staged ? sc.d_V2 : nullptr;
    L.et2 = et_staged ? (int32_t *)sc.d_et2 : nullptr;
    if (et_state) {
        L.bad = (uint32_t *)sc.d_early;
        if (!L.iters_used) L.iters_used = (int32_t *)((char *)sc.d_early + (size_t)stride * 4);
        L.live = (uint8_t *)sc.d_early + (size_t)stride * 8;
    }
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    if (c->profile) {
        HIP_TRY(hipEventCreate(&ev0));
        HIP_TRY(hipEventCreate(&ev1));
        HIP_TRY(hipEventRecord(ev0, s));
    }
    int lr = kern == 8   ? launch_coop3(L, c->coop3, s)
             : kern == 5 ? launch_coop(L, c->coop, s)
             : kern == 11 ? launch_stairf(L, c->stairf, s)
             : kern == 3 ? launch_windowed2(L, c->w16, s)
             : kern == 2 ? launch_windowed(L, c->wcode, s)
                         : launch_generic(L, s);
    if (c->profile) {
        HIP_TRY(hipEventRecord(ev1, s));
        c->events.emplace_back(ev0, ev1);
    }
    if (lr) {
        const hipError_t e = hipGetLastError();
        return ldpc_set_error(LDPC_EDEVICE, "decode launch (kernel %d): %s", kern,
                              e != hipSuccess ? hipGetErrorString(e) : "launch configuration rejected by the host side");
    }
    if (d_hard || d_soft) {
        int r2 = is_float    ? launch_deinterleave_f32((const float *)sc.d_V, d_hard, (float *)d_soft, h->n, batch,
                                                       vpitch, s)
                 : kern == 8 ? launch_deinterleave_grp_i8((const int8_t *)sc.d_V, d_hard, (int8_t *)d_soft, h->n,
                                                          batch, vgroup, s)
                             : launch_deinterleave_i8((const int8_t *)sc.d_V, d_hard, (int8_t *)d_soft, h->n,
                                                      batch, vpitch, s);
        if (r2) return ldpc_set_error(LDPC_EDEVICE, "deinterleave: %s", hipGetErrorString(hipGetLastError()));
    }
    if (ec && launch_count_errors(d_hard, h->n, batch, ec->k, ec->ref, ec->counts, s))
        return ldpc_set_error(LDPC_EDEVICE, "count_errors: %s", hipGetErrorString(hipGetLastError()));
    return LDPC_OK;
}

extern "C" int ldpc_decode_i8_async(ldpc_ctx *c, void *s, const int8_t *d_llr, uint8_t *d_hard, int8_t *d_soft,
                                    int32_t *d_iters, int batch, int n_iter, const ldpc_params *p)
{
    if (!c || (!d_llr && batch > 0)) return ldpc_set_error(LDPC_EINVAL, "NULL ctx/llr");
    return decode_device(c, c->sc, (hipStream_t)s, d_llr, d_hard, d_soft, d_iters, batch, n_iter, p, false);
}

// Node-major input: LLR of bit i of codeword b at d_llr[i * ld + b] -- the
// layout the reference's decoders run on (Interleaver_uint8's output,
// code/gpu_fixed/transpose/GPU_Transpose_uint8.cu:80-130), which its v2 decoder
// takes straight from the caller (CGPU_Decoder_MS_SIMD_v2::decode,
// code/gpu_fixed/decoder_oms_v2/CGPU_Decoder_MS_SIMD_v2.cu:120-251: copy,
// decode, InvInterleaver_uint8 with the hard decision).  Outputs frame-major,
// as there.
extern "C" int ldpc_decode_i8_nm_async(ldpc_ctx *c, void *s, const int8_t *d_llr, size_t ld, uint8_t *d_hard,
                                       int8_t *d_soft, int32_t *d_iters, int batch, int n_iter, const ldpc_params *p)
{
    if (!c || (!d_llr && batch > 0)) return ldpc_set_error(LDPC_EINVAL, "NULL ctx/llr");
    if (batch > 0 && ld < (size_t)batch)
        return ldpc_set_error(LDPC_EINVAL, "node-major pitch %zu < batch %d", ld, batch);
    return decode_device(c, c->sc, (hipStream_t)s, d_llr, d_hard, d_soft, d_iters, batch, n_iter, p, false, false,
                         batch > 0 ? ld : 0);
}

extern "C" int ldpc_decode_f32_async(ldpc_ctx *c, void *s, const float *d_llr, uint8_t *d_hard, float *d_soft,
                                     int32_t *d_iters, int batch, int n_iter, const ldpc_params *p)
{
    if (!c || (!d_llr && batch > 0)) return ldpc_set_error(LDPC_EINVAL, "NULL ctx/llr");
    return decode_device(c, c->sc, (hipStream_t)s, d_llr, d_hard, d_soft, d_iters, batch, n_iter, p, true);
}

// decode + error count in one call (the reference's decode followed by
// CErrorAnalyzer::generate, code/x86/CErrorAnalyzer/CErrorAnalyzer.cpp:123-154;
// code/x86/main_p.cpp:511-540): fused into the decode kernel's epilogue where
// the kernel writes the hard decisions itself (ldsep), else one count launch
// after the decode (it needs d_hard then)
static int decode_count(ldpc_ctx *c, void *s, const void *d_llr, uint8_t *d_hard, void *d_soft, int32_t *d_iters,
                        int batch, int n_iter, const ldpc_params *p, bool is_float, int k, const uint8_t *d_ref,
                        unsigned long long *d_counts)
{
    if (!c || (!d_llr && batch > 0)) return ldpc_set_error(LDPC_EINVAL, "NULL ctx/llr");
    if (!d_counts || k < 0 || k > c->code->n) return ldpc_set_error(LDPC_EINVAL, "count: NULL counts or k %d", k);
    if (!d_hard) return ldpc_set_error(LDPC_EINVAL, "count: d_hard is required");
    const ErrCount ec{k, d_ref, d_counts};
    return decode_device(c, c->sc, (hipStream_t)s, d_llr, d_hard, d_soft, d_iters, batch, n_iter, p, is_float, false,
                         0, &ec);
}

extern "C" int ldpc_decode_i8_count_async(ldpc_ctx *c, void *s, const int8_t *d_llr, uint8_t *d_hard, int8_t *d_soft,
                                          int32_t *d_iters, int batch, int n_iter, const ldpc_params *p, int k,
                                          const uint8_t *d_ref, unsigned long long *d_counts)
{
    return decode_count(c, s, d_llr, d_hard, d_soft, d_iters, batch, n_iter, p, false, k, d_ref, d_counts);
}

extern "C" int ldpc_decode_f32_count_async(ldpc_ctx *c, void *s, const float *d_llr, uint8_t *d_hard, float *d_soft,
                                           int32_t *d_iters, int batch, int n_iter, const ldpc_params *p, int k,
                                           const uint8_t *d_ref, unsigned long long *d_counts)
{
    return decode_count(c, s, d_llr, d_hard, d_soft, d_iters, batch, n_iter, p, true, k, d_ref, d_counts);
}

// Chunks of the host-buffer path: whole 64-codeword rows, at least 256
// codewords each (16 coop workgroups), LDPC_HOST_CHUNKS of them (default 2
// when the input is large enough for its copy time to matter, >= 64 MB, else
// 1), and no more than the hardware queues left for them.  Concurrent chunk
// decodes need hardware queues of their own: HIP maps streams round-robin onto
// GPU_MAX_HW_QUEUES (default 4) queues per process, and the null stream and
// the context's stream hold two of them, so a third lane would share a queue
// -- and wait for -- the first one's decode (measured: 4 lanes on 2 queues,
// 114 ms per DVB-S2 4096-codeword call vs 68 ms unchunked).
static int host_chunks(int batch, size_t in_bytes)
{
    const int def = in_bytes >= ((size_t)64 << 20) ? 2 : 1;
    const int lanes = std::max(1, getenv_int("GPU_MAX_HW_QUEUES", 4) - 2);
    const int want = std::min(lanes, std::max(1, getenv_int("LDPC_HOST_CHUNKS", def)));
    return std::max(1, std::min(want, batch / 256));
}

// The host-buffer path (CDecoder::decode(char*, char*, int), synchronous).
// The batch is cut into chunks; chunk i runs on lane i (own stream, scratch
// and staging): H2D(i) -> decode(i) -> D2H(i), so the copies of one chunk
// overlap the decodes of the others -- the reference's W streams x F frames
// scheme (paper/ldpcGpuTegra.tex:279-289; its decode_stream,
// code/gpu_fixed/decoder_ms/CGPU_Decoder_MS_SIMD.cu:219-275, runs one stream
// with blocking copies).  A staircase-code decode takes about as long for one
// 16-codeword workgroup as for a whole chip of them (its serial chain is per
// workgroup), so the concurrent chunk decodes cost nothing.  The input copies
// are chained (lane i's waits for lane i-1's): two concurrent copies share
// the link and both finish at the end (measured r03e, pinned, 2 chunks: 4.7
// ms each, side by side), which held every decode back until all the input
// had arrived.  A call therefore takes about H2D(batch) + one decode +
// D2H(one chunk) -- no chunking can do better, since the last chunk cannot
// start before all the input is on the device.  Every lane's
// scratch is sized before any work is queued.  Pinned host buffers
// (ldpc_host_alloc) make the copies asynchronous DMA; pageable ones are
// staged by the HIP runtime (the host thread blocks in the copy, the GPU
// keeps decoding).
static int decode_host(ldpc_ctx *c, const void *llr, uint8_t *hard, int batch, int n_iter, const ldpc_params *p,
                       bool is_float)
{
    if (!c || ((!llr || !hard) && batch > 0)) return ldpc_set_error(LDPC_EINVAL, "NULL ctx/llr/hard");
    int rc = check_params(c, batch, n_iter, p, is_float);
    if (rc != LDPC_OK || batch == 0) return rc;
    if (c->device < 0) {   // host context: the CPU decoder (host.cpp)
        c->last_kernel = 10;
        return is_float ? host_decode_f32(c->code, (const float *)llr, hard, batch, n_iter, p)
                        : host_decode_i8(c->code, (const int8_t *)llr, hard, batch, n_iter, p);
    }
    HIP_TRY(hipSetDevice(c->device));
    const size_t esz = is_float ? 4 : 1;
    const int n = c->code->n, nc_want = host_chunks(batch, (size_t)batch * n * esz);
    // chunk boundaries: equal chunks in units of 1024 codewords where the
    // batch allows (64 coop workgroups: the XCD-aware workgroup remap keeps
    // the 8 workgroups that share a V line on one XCD only when a grid splits
    // evenly into 8 x 8 of them; a chunk with the groups split across XCDs
    // runs ~20 % slower, measured r03h with a 2:1 split of 4096 codewords:
    // 60.2 vs 55.7 ms per call), else 128 (the remap's grid % 8).  The 1024
    // unit is used only while the chunks stay even (the last one at least half
    // of the others): 2049 codewords as 2048 + 1 would leave the big chunk's
    // decode and copy with nothing to overlap
    std::vector<int> b0s(1, 0);
    {
        auto size_for = [&](int unit) { return ((batch + nc_want - 1) / nc_want + unit - 1) / unit * unit; };
        auto even = [&](int cs) {
            const int full = std::min(nc_want, (batch + cs - 1) / cs);
            return full <= 1 || 2 * (batch - (full - 1) * cs) >= cs;
        };
        int cs0 = size_for(128);
        if (batch >= nc_want * 1024 && even(size_for(1024))) cs0 = size_for(1024);
        for (int i = 1; i < nc_want && i * cs0 < batch; i++) b0s.push_back(i * cs0);
        b0s.push_back(batch);
    }
    const int nc = (int)b0s.size() - 1;   // (rounding up can leave fewer chunks)
    int cs = 0;   // largest chunk (the staging size of every lane)
    for (int i = 0; i < nc; i++) cs = std::max(cs, b0s[i + 1] - b0s[i]);
    if ((int)c->lanes.size() < nc) c->lanes.resize(nc);
    auto in_al = [&](int nb) { return ((size_t)nb * n * esz + 255) / 256 * 256; };
    // streams, events and every lane's buffers first (no hipFree between queued work)
    for (int i = 0; i < nc; i++) {
        Lane &l = c->lanes[i];
        const int b0 = b0s[i], nb = b0s[i + 1] - b0;
        if (!l.stream && hipStreamCreateWithFlags(&l.stream, hipStreamNonBlocking) != hipSuccess) {
            l.stream = nullptr;
            return ldpc_set_error(LDPC_EDEVICE, "host path: hipStreamCreate");
        }
        if (!l.h2d_done && hipEventCreateWithFlags(&l.h2d_done, hipEventDisableTiming) != hipSuccess) {
            l.h2d_done = nullptr;
            return ldpc_set_error(LDPC_EDEVICE, "host path: hipEventCreate");
        }
        if ((rc = ensure(&l.d_io, &l.io_bytes, in_al(nb) + (size_t)cs * n)) != LDPC_OK) return rc;
        if ((rc = decode_device(c, l.sc, l.stream, l.d_io, nullptr, nullptr, nullptr, nb, n_iter, p, is_float,
                                true)) != LDPC_OK)
            return rc;
    }
    int used = 0;
    // every queued lane is joined before returning, on success and on error
    auto finish = [&](int r) {
        for (int i = 0; i < used; i++) {
            const hipError_t e = hipStreamSynchronize(c->lanes[i].stream);
            if (e != hipSuccess && r == LDPC_OK) r = ldpc_set_error(LDPC_EDEVICE, "host path: %s", hipGetErrorString(e));
        }
        return r;
    };
    for (int i = 0; i < nc; i++) {
        Lane &l = c->lanes[i];
        const int b0 = b0s[i], nb = b0s[i + 1] - b0;
        char *d_in = (char *)l.d_io, *d_out = d_in + in_al(nb);
        used = i + 1;
        if (i > 0 && hipStreamWaitEvent(l.stream, c->lanes[i - 1].h2d_done, 0) != hipSuccess)
            return finish(ldpc_set_error(LDPC_EDEVICE, "host path: hipStreamWaitEvent"));
        if (hipMemcpyAsync(d_in, (const char *)llr + (size_t)b0 * n * esz, (size_t)nb * n * esz,
                           hipMemcpyHostToDevice, l.stream) != hipSuccess ||
            hipEventRecord(l.h2d_done, l.stream) != hipSuccess)
            return finish(ldpc_set_error(LDPC_EDEVICE, "host path H2D: %s", hipGetErrorString(hipGetLastError())));
        rc = decode_device(c, l.sc, l.stream, d_in, (uint8_t *)d_out, nullptr, nullptr, nb, n_iter, p, is_float);
        if (rc != LDPC_OK) return finish(rc);
    }
    for (int i = 0; i < nc; i++) {
        Lane &l = c->lanes[i];
        const int b0 = b0s[i], nb = b0s[i + 1] - b0;
        if (hipMemcpyAsync(hard + (size_t)b0 * n, (char *)l.d_io + in_al(nb), (size_t)nb * n, hipMemcpyDeviceToHost,
                           l.stream) != hipSuccess)
            return finish(ldpc_set_error(LDPC_EDEVICE, "host path D2H: %s", hipGetErrorString(hipGetLastError())));
    }
    return finish(LDPC_OK);
}

// The asynchronous host-buffer path: one batch, H2D -> decode -> D2H queued on
// the caller's stream through the context's own staging (c->d_io) and scratch
// (c->sc), nothing waited for.  Two contexts on two streams keep two batches in
// flight: the copies of one overlap the decode of the other (the reference's
// W streams x F frames, paper/ldpcGpuTegra.tex:279-289).
static int decode_host_async(ldpc_ctx *c, void *sv, const void *llr, uint8_t *hard, int batch, int n_iter,
                             const ldpc_params *p, bool is_float)
{
    if (!c || ((!llr || !hard) && batch > 0)) return ldpc_set_error(LDPC_EINVAL, "NULL ctx/llr/hard");
    int rc = check_params(c, batch, n_iter, p, is_float);
    if (rc != LDPC_OK || batch == 0) return rc;
    if (c->device < 0) return host_only(c);
    HIP_TRY(hipSetDevice(c->device));
    const hipStream_t s = (hipStream_t)sv;
    const size_t n = (size_t)c->code->n, esz = is_float ? 4 : 1;
    const size_t in_al = ((size_t)batch * n * esz + 255) / 256 * 256;
    // size the staging and the scratch before anything is queued (a hipFree of
    // a buffer the previous call still uses would wait for the device anyway)
    if (!c->host_done) HIP_TRY(hipEventCreateWithFlags(&c->host_done, hipEventDisableTiming));
    // a previous call (possibly on another stream) still using d_io / the scratch:
    // resizing frees them, so wait for it on the host; otherwise order this
    // stream after it on the device
    const bool grow = c->io_bytes < in_al + (size_t)batch * n;
    if (c->host_pending && grow) HIP_TRY(hipEventSynchronize(c->host_done));
    if ((rc = ensure(&c->d_io, &c->io_bytes, in_al + (size_t)batch * n)) != LDPC_OK) return rc;
    if ((rc = decode_device(c, c->sc, s, c->d_io, nullptr, nullptr, nullptr, batch, n_iter, p, is_float, true)) !=
        LDPC_OK)
        return rc;
    if (c->host_pending) HIP_TRY(hipStreamWaitEvent(s, c->host_done, 0));
    char *d_in = (char *)c->d_io, *d_out = d_in + in_al;
    HIP_TRY(hipMemcpyAsync(d_in, llr, (size_t)batch * n * esz, hipMemcpyHostToDevice, s));
    if ((rc = decode_device(c, c->sc, s, d_in, (uint8_t *)d_out, nullptr, nullptr, batch, n_iter, p, is_float)) !=
        LDPC_OK)
        return rc;
    HIP_TRY(hipMemcpyAsync(hard, d_out, (size_t)batch * n, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipEventRecord(c->host_done, s));
    c->host_pending = true;
    return LDPC_OK;
}

extern "C" int ldpc_decode_i8_host_async(ldpc_ctx *c, void *s, const int8_t *llr, uint8_t *hard, int batch,
                                         int n_iter, const ldpc_params *p)
{
    return decode_host_async(c, s, llr, hard, batch, n_iter, p, false);
}

extern "C" int ldpc_decode_f32_host_async(ldpc_ctx *c, void *s, const float *llr, uint8_t *hard, int batch,
                                          int n_iter, const ldpc_params *p)
{
    return decode_host_async(c, s, llr, hard, batch, n_iter, p, true);
}

extern "C" int ldpc_ctx_synchronize(ldpc_ctx *c)
{
    if (!c) return ldpc_set_error(LDPC_EINVAL, "NULL ctx");
    if (!c->host_pending) return LDPC_OK;
    HIP_TRY(hipSetDevice(c->device));
    c->host_pending = false;
    HIP_TRY(hipEventSynchronize(c->host_done));
    return LDPC_OK;
}

extern "C" int ldpc_host_alloc(void **p, size_t bytes)
{
    if (!p) return ldpc_set_error(LDPC_EINVAL, "NULL pointer");
    *p = nullptr;
    if (bytes == 0) return LDPC_OK;
    const hipError_t e = hipHostMalloc(p, bytes, hipHostMallocDefault);
    if (e != hipSuccess) {
        *p = nullptr;
        return ldpc_set_error(LDPC_ENOMEM, "hipHostMalloc(%zu): %s", bytes, hipGetErrorString(e));
    }
    return LDPC_OK;
}

extern "C" void ldpc_host_free(void *p)
{
    if (p) (void)hipHostFree(p);
}

extern "C" int ldpc_decode_i8(ldpc_ctx *c, const int8_t *llr, uint8_t *hard, int batch, int n_iter,
                              const ldpc_params *p)
{
    return decode_host(c, llr, hard, batch, n_iter, p, false);
}

extern "C" int ldpc_decode_f32(ldpc_ctx *c, const float *llr, uint8_t *hard, int batch, int n_iter,
                               const ldpc_params *p)
{
    return decode_host(c, llr, hard, batch, n_iter, p, true);
}

extern "C" int ldpc_awgn_i8_async(ldpc_ctx *c, void *s, int8_t *d_llr, int batch, uint64_t first_cw, uint64_t seed,
                                  const uint32_t *table, const uint8_t *d_codeword)
{
    if (!c || !d_llr || !table || batch < 0) return ldpc_set_error(LDPC_EINVAL, "awgn args");
    if (c->device < 0) return host_only(c);
    if (table[63] < 1 || table[63] > 31) return ldpc_set_error(LDPC_EINVAL, "awgn table sat");
    HIP_TRY(hipSetDevice(c->device));
    AwgnTable t;
    memcpy(t.t, table, sizeof(t.t));
    if (launch_awgn_i8(d_llr, c->code->n, batch, first_cw, seed, t, d_codeword, (hipStream_t)s))
        return ldpc_set_error(LDPC_EDEVICE, "awgn: %s", hipGetErrorString(hipGetLastError()));
    return LDPC_OK;
}

static bool quantize_args_ok(long count, int factor, int sat_neg, int sat_pos)
{
    return count >= 0 && factor >= 1 && sat_neg >= -128 && sat_pos <= 127 && sat_neg <= sat_pos;
}

extern "C" int ldpc_quantize_f32_i8_async(ldpc_ctx *c, void *s, const float *d_y, int8_t *d_q, long count, int factor,
                                          int sat_neg, int sat_pos)
{
    if (!c || (count > 0 && (!d_y || !d_q)) || !quantize_args_ok(count, factor, sat_neg, sat_pos))
        return ldpc_set_error(LDPC_EINVAL, "quantize args");
    if (c->device < 0) return host_only(c);
    HIP_TRY(hipSetDevice(c->device));
    if (launch_quantize_f32_i8(d_y, d_q, count, factor, sat_neg, sat_pos, (hipStream_t)s))
        return ldpc_set_error(LDPC_EDEVICE, "quantize: %s", hipGetErrorString(hipGetLastError()));
    return LDPC_OK;
}

extern "C" int ldpc_quantize_f32_i8(ldpc_ctx *c, const float *y, int8_t *q, long count, int factor, int sat_neg,
                                    int sat_pos)
{
    if (!c || (count > 0 && (!y || !q)) || !quantize_args_ok(count, factor, sat_neg, sat_pos))
        return ldpc_set_error(LDPC_EINVAL, "quantize args");
    if (count == 0) return LDPC_OK;
    if (c->device < 0) {   // host context: CFastFixConversion::generate's rule on the CPU (quantize_k's)
        for (long i = 0; i < count; i++) {
            const float v = (float)factor * y[i];
            int value = (std::fabs(v) < 2147483648.0f) ? (int)v : INT_MIN;
            value = std::min(std::max(value, sat_neg), sat_pos);
            q[i] = (int8_t)value;
        }
        return LDPC_OK;
    }
    HIP_TRY(hipSetDevice(c->device));
    const size_t in_bytes = (size_t)count * sizeof(float), al = (in_bytes + 255) & ~(size_t)255;
    int rc;
    if ((rc = ensure(&c->d_io, &c->io_bytes, al + (size_t)count)) != LDPC_OK) return rc;
    float *d_y = (float *)c->d_io;
    int8_t *d_q = (int8_t *)c->d_io + al;
    const hipStream_t s = c->stream;
    HIP_TRY(hipMemcpyAsync(d_y, y, in_bytes, hipMemcpyHostToDevice, s));
    if (launch_quantize_f32_i8(d_y, d_q, count, factor, sat_neg, sat_pos, s))
        return ldpc_set_error(LDPC_EDEVICE, "quantize: %s", hipGetErrorString(hipGetLastError()));
    HIP_TRY(hipMemcpyAsync(q, d_q, (size_t)count, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    return LDPC_OK;
}

extern "C" int ldpc_count_errors_async(ldpc_ctx *c, void *s, const uint8_t *d_hard, int batch, int k,
                                       const uint8_t *d_ref, unsigned long long *d_counts)
{
    if (!c || !d_hard || !d_counts || batch < 0 || k < 0 || k > c->code->n)
        return ldpc_set_error(LDPC_EINVAL, "count_errors args");
    if (c->device < 0) return host_only(c);
    HIP_TRY(hipSetDevice(c->device));
    if (launch_count_errors(d_hard, c->code->n, batch, k, d_ref, d_counts, (hipStream_t)s))
        return ldpc_set_error(LDPC_EDEVICE, "count_errors: %s", hipGetErrorString(hipGetLastError()));
    return LDPC_OK;
}
