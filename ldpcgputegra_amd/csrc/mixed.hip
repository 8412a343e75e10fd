// mixed.hip -- mixed-rate batches (BASELINE config 5) on top of the per-code
// decoder contexts.  Host code: group codewords by code id, gather each
// group into a contiguous staging batch, decode the groups concurrently on
// their contexts' streams (forked from and joined back to the caller's
// stream with events), scatter hard decisions / iterations back.
#include <algorithm>
#include <cstdlib>
#include <vector>

#include "kernels.h"
#include "ldpc_internal.h"

struct ldpc_mixed {
    int device = 0, n = 0, max_batch = 0;
    std::vector<ldpc_ctx *> ctx;
    std::vector<hipStream_t> stream;
    std::vector<bool> own_stream;     // created here (priority streams), destroyed here
    std::vector<int8_t *> d_in;
    std::vector<uint8_t *> d_out;
    std::vector<int32_t *> d_idx, d_its;
    std::vector<int32_t *> h_idx;     // pinned
    std::vector<hipEvent_t> done;
    std::vector<bool> pending;
    hipEvent_t fork = nullptr;
};

extern "C" void ldpc_mixed_destroy(ldpc_mixed *mx)
{
    if (!mx) return;
    (void)hipSetDevice(mx->device);
    for (size_t c = 0; c < mx->ctx.size(); c++) {
        if (mx->pending[c]) (void)hipEventSynchronize(mx->done[c]);
        (void)hipFree(mx->d_in[c]);
        (void)hipFree(mx->d_out[c]);
        (void)hipFree(mx->d_idx[c]);
        (void)hipFree(mx->d_its[c]);
        if (mx->h_idx[c]) (void)hipHostFree(mx->h_idx[c]);
        if (mx->done[c]) (void)hipEventDestroy(mx->done[c]);
        if (mx->own_stream[c]) (void)hipStreamDestroy(mx->stream[c]);
        ldpc_ctx_destroy(mx->ctx[c]);
    }
    if (mx->fork) (void)hipEventDestroy(mx->fork);
    delete mx;
}

extern "C" int ldpc_mixed_create(const ldpc_code *const *codes, int n_codes, int device, int max_batch,
                                 ldpc_mixed **out)
{
    if (!out) return ldpc_set_error(LDPC_EINVAL, "out is NULL");
    *out = nullptr;
    if (!codes || n_codes <= 0 || max_batch <= 0) return ldpc_set_error(LDPC_EINVAL, "mixed: bad arguments");
    if (device < 0) return ldpc_set_error(LDPC_EUNSUPPORTED, "mixed: device buffers need a GPU (device %d)", device);
    for (int c = 0; c < n_codes; c++)
        if (!codes[c] || codes[c]->n != codes[0]->n)
            return ldpc_set_error(LDPC_EINVAL, "mixed: all codes must be non-NULL with equal N");
    auto *mx = new ldpc_mixed();
    mx->device = device;
    mx->n = codes[0]->n;
    mx->max_batch = max_batch;
    const size_t nc = (size_t)n_codes;
    mx->ctx.assign(nc, nullptr);
    mx->stream.assign(nc, nullptr);
    mx->d_in.assign(nc, nullptr);
    mx->d_out.assign(nc, nullptr);
    mx->d_idx.assign(nc, nullptr);
    mx->d_its.assign(nc, nullptr);
    mx->h_idx.assign(nc, nullptr);
    mx->done.assign(nc, nullptr);
    mx->pending.assign(nc, false);
    mx->own_stream.assign(nc, false);
    // LDPC_MIXED_PRIO=1: the codes with the most checks (longest serial
    // chain per iteration, so the longest latency under early termination)
    // get high-priority streams of their own, so their per-iteration launches
    // are dispatched ahead of the high-rate codes' workgroups; 2 = the reverse
    // order; 0 (default) = the contexts' streams.  configs[4]: 82.9 and
    // 87.3 ms per step with 1, 87.4 with 0 -- within run-to-run spread
    const char *pe = getenv("LDPC_MIXED_PRIO");
    const int prio = (pe && *pe) ? atoi(pe) : 0;
    std::vector<int> ms;
    for (int c = 0; c < n_codes; c++) ms.push_back(codes[c]->m);
    std::sort(ms.begin(), ms.end());
    const int m_hi = ms[ms.size() / 2];
    for (int c = 0; c < n_codes; c++) {
        int rc = ldpc_ctx_create(codes[c], device, max_batch, &mx->ctx[c]);
        if (rc != LDPC_OK) {
            ldpc_mixed_destroy(mx);
            return rc;
        }
        void *s;
        ldpc_ctx_stream(mx->ctx[c], &s);
        mx->stream[c] = (hipStream_t)s;
        if (prio) {
            int least = 0, greatest = 0;
            hipStream_t ps = nullptr;
            if (hipSetDevice(device) != hipSuccess || hipDeviceGetStreamPriorityRange(&least, &greatest) != hipSuccess ||
                hipStreamCreateWithPriority(&ps, hipStreamNonBlocking, (codes[c]->m >= m_hi) == (prio == 1) ? greatest : least) !=
                    hipSuccess) {
                ldpc_mixed_destroy(mx);
                return ldpc_set_error(LDPC_EDEVICE, "mixed: priority stream");
            }
            mx->stream[c] = ps;
            mx->own_stream[c] = true;
        }
        const size_t bytes = (size_t)max_batch * mx->n;
        if (hipMalloc(&mx->d_in[c], bytes) != hipSuccess || hipMalloc(&mx->d_out[c], bytes) != hipSuccess ||
            hipMalloc(&mx->d_idx[c], 4ull * max_batch) != hipSuccess ||
            hipMalloc(&mx->d_its[c], 4ull * max_batch) != hipSuccess ||
            hipHostMalloc(&mx->h_idx[c], 4ull * max_batch, 0) != hipSuccess ||
            hipEventCreateWithFlags(&mx->done[c], hipEventDisableTiming) != hipSuccess) {
            ldpc_mixed_destroy(mx);
            return ldpc_set_error(LDPC_ENOMEM, "mixed: staging buffers");
        }
    }
    // a coop3 decode (one 124.5-KB workgroup per CU, VALU-bound slab waves)
    // runs slower with other rates' windowed2 waves on its CUs: those get an
    // LDS pad that keeps them off (LDPC_MIXED_LDS_PAD bytes, default 40 KB > the
    // 35.5 KB a coop3 workgroup leaves; 0 = off)
    std::vector<bool> c3(nc, false);
    bool any_c3 = false;
    for (int c = 0; c < n_codes; c++) {
        c3[c] = ldpc_ctx_has_kernel(mx->ctx[c], 8);
        any_c3 = any_c3 || c3[c];
    }
    const char *pp = getenv("LDPC_MIXED_LDS_PAD");
    const int pad = (pp && *pp) ? atoi(pp) : 40 * 1024;
    if (any_c3 && pad > 0)
        for (int c = 0; c < n_codes; c++)
            if (!c3[c]) (void)ldpc_ctx_set_lds_pad(mx->ctx[c], pad);
    if (hipEventCreateWithFlags(&mx->fork, hipEventDisableTiming) != hipSuccess) {
        ldpc_mixed_destroy(mx);
        return ldpc_set_error(LDPC_EDEVICE, "mixed: event");
    }
    *out = mx;
    return LDPC_OK;
}

extern "C" int ldpc_decode_i8_mixed_async(ldpc_mixed *mx, void *hip_stream, const int8_t *d_llr, uint8_t *d_hard,
                                          int32_t *d_iters_used, const int32_t *code_id, int batch, int n_iter,
                                          const ldpc_params *p)
{
    if (!mx || batch < 0 || batch > mx->max_batch || (batch > 0 && (!d_llr || !d_hard || !code_id)))
        return ldpc_set_error(LDPC_EINVAL, "mixed decode: bad arguments");
    if (batch == 0) return LDPC_OK;
    const int nc = (int)mx->ctx.size();
    std::vector<int> cnt(nc, 0);
    for (int b = 0; b < batch; b++) {
        if (code_id[b] < 0 || code_id[b] >= nc) return ldpc_set_error(LDPC_EINVAL, "code_id[%d] = %d", b, code_id[b]);
        cnt[code_id[b]]++;
    }
    if (hipSetDevice(mx->device) != hipSuccess) return ldpc_set_error(LDPC_EDEVICE, "hipSetDevice");
    // NULL = HIP's null stream (ordered with the legacy default stream)
    hipStream_t s = (hipStream_t)hip_stream;
    // previous call's index uploads must have finished before we rewrite h_idx
    for (int c = 0; c < nc; c++)
        if (mx->pending[c]) {
            (void)hipEventSynchronize(mx->done[c]);
            mx->pending[c] = false;
        }
    std::vector<int> fill(nc, 0);
    for (int b = 0; b < batch; b++) mx->h_idx[code_id[b]][fill[code_id[b]]++] = b;
    if (hipEventRecord(mx->fork, s) != hipSuccess) return ldpc_set_error(LDPC_EDEVICE, "event record");
    // on a failure after some streams were forked: every forked stream still
    // records its done event (the next call waits for its h_idx upload) and
    // the caller's stream is joined with all of them before returning
    auto join_all = [&](int upto, int rc) {
        for (int c = 0; c <= upto && c < nc; c++) {
            if (!cnt[c] || !mx->pending[c]) continue;
            (void)hipEventRecord(mx->done[c], mx->stream[c]);
            (void)hipStreamWaitEvent(s, mx->done[c], 0);
        }
        return rc;
    };
    for (int c = 0; c < nc; c++) {
        if (!cnt[c]) continue;
        hipStream_t cs = mx->stream[c];
        const int n = mx->n;
        if (hipStreamWaitEvent(cs, mx->fork, 0) != hipSuccess)
            return join_all(c - 1, ldpc_set_error(LDPC_EDEVICE, "mixed: fork"));
        if (hipMemcpyAsync(mx->d_idx[c], mx->h_idx[c], 4ull * cnt[c], hipMemcpyHostToDevice, cs) != hipSuccess)
            return join_all(c - 1, ldpc_set_error(LDPC_EDEVICE, "mixed: index upload"));
        mx->pending[c] = true;   // h_idx[c] is in flight from here on
        if (launch_gather_rows(d_llr, mx->d_in[c], mx->d_idx[c], cnt[c], n, cs))
            return join_all(c, ldpc_set_error(LDPC_EDEVICE, "mixed: gather"));
        int rc = ldpc_decode_i8_async(mx->ctx[c], cs, mx->d_in[c], mx->d_out[c], nullptr,
                                      d_iters_used ? mx->d_its[c] : nullptr, cnt[c], n_iter, p);
        if (rc != LDPC_OK) return join_all(c, rc);
        if (launch_scatter_rows(mx->d_out[c], d_hard, mx->d_idx[c], cnt[c], n, cs) ||
            (d_iters_used && launch_scatter_rows(mx->d_its[c], d_iters_used, mx->d_idx[c], cnt[c], 4, cs)))
            return join_all(c, ldpc_set_error(LDPC_EDEVICE, "mixed: scatter"));
        if (hipEventRecord(mx->done[c], cs) != hipSuccess || hipStreamWaitEvent(s, mx->done[c], 0) != hipSuccess)
            return join_all(c, ldpc_set_error(LDPC_EDEVICE, "mixed: join"));
    }
    return LDPC_OK;
}

extern "C" int ldpc_mixed_last_kernel(ldpc_mixed *mx, int code_index, int *kernel)
{
    if (!mx || !kernel || code_index < 0 || code_index >= (int)mx->ctx.size())
        return ldpc_set_error(LDPC_EINVAL, "mixed last kernel: bad arguments");
    return ldpc_ctx_last_kernel(mx->ctx[code_index], kernel);
}

extern "C" int ldpc_mixed_last_et_stage(ldpc_mixed *mx, int code_index, int *k)
{
    if (!mx || !k || code_index < 0 || code_index >= (int)mx->ctx.size())
        return ldpc_set_error(LDPC_EINVAL, "mixed last et stage: bad arguments");
    return ldpc_ctx_last_et_stage(mx->ctx[code_index], k);
}

extern "C" int ldpc_mixed_profile(ldpc_mixed *mx, int enable)
{
    if (!mx) return ldpc_set_error(LDPC_EINVAL, "mixed profile: NULL");
    for (auto *c : mx->ctx) {
        const int rc = ldpc_ctx_profile(c, enable);
        if (rc != LDPC_OK) return rc;
    }
    return LDPC_OK;
}

extern "C" int ldpc_mixed_kernel_time(ldpc_mixed *mx, int code_index, double *total_ms, int *launches, int reset)
{
    if (!mx || code_index < 0 || code_index >= (int)mx->ctx.size())
        return ldpc_set_error(LDPC_EINVAL, "mixed kernel time: bad arguments");
    return ldpc_ctx_kernel_time(mx->ctx[code_index], total_ms, launches, reset);
}
