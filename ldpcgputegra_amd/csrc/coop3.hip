// coop3.hip -- host side of the coop3 decoder (coop3_kernel.h holds the
// kernel and its description; coop3_deg.hip instantiates it once per
// first-group degree, one object each, so the six degrees compile in
// parallel): the schedule (coop3_plan_host), the line-cache records, the
// uploads, the launches (early termination staged or not) and the staging
// kernels.
#include "coop3_kernel.h"

using namespace c3;

namespace {

__global__ void fill_iters3_k(int batch, int32_t *iters_used, int iters)
{
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b < batch) iters_used[b] = iters;
}

int env_int3(const char *name, int def)
{
    const char *e = getenv(name);
    return (e && *e) ? atoi(e) : def;
}

// diagnostic build (LDPC_COOP3_STAMP=1): per-period cycles of each wave
template <int WS>
void report_stamps3(const unsigned long long *d, int grid, hipStream_t s)
{
    constexpr int nwaves = WS + 2, CHW = Cfg<WS, 2>::CHW;
    std::vector<unsigned long long> h((size_t)grid * nwaves * 8);
    if (hipStreamSynchronize(s) != hipSuccess ||
        hipMemcpy(h.data(), d, h.size() * sizeof(h[0]), hipMemcpyDeviceToHost) != hipSuccess)
        return;
    std::vector<double> v((size_t)nwaves * 8, 0.0);
    for (int b = 0; b < grid; b++)
        for (int w = 0; w < nwaves; w++) {
            const unsigned long long *o = &h[((size_t)b * nwaves + w) * 8];
            const double G = o[7] ? (double)o[7] : 1.0;
            for (int i = 0; i < 6; i++) v[w * 8 + i] += o[i] / G / grid;
            v[w * 8 + 6] += o[6] / G / grid;
            v[w * 8 + 7] += G / grid;
        }
    fprintf(stderr, "coop3 stamps [cycles per period]: elapsed %.0f (%.0f periods per workgroup)\n", v[5], v[7]);
    for (int w = 0; w < nwaves; w++) {
        const double *x = &v[w * 8];
        if (w == CHW)
            fprintf(stderr, "  chain %d: busy %.0f steps %.0f | ET round 0 %.1f, full syndromes %.1f (%.4f per period)\n",
                    w, x[0], x[1], x[2], x[3], x[6]);
        else if (w == WS + 1)
            fprintf(stderr, "  memory %d: busy %.0f | issue %.0f vmcnt %.0f | per period: last wave ready %.0f after the "
                            "first wave's start, starts spread over %.0f\n", w, x[0], x[2], x[0] - x[2], x[6], x[3]);
        else   // fast periods: x-input wait, post, pre; rest = guarded periods' share and the stamps
            fprintf(stderr, "  slab %d: busy %.0f | x wait %.0f post %.0f pre %.0f rest %.0f | LDS drain at the barrier "
                            "%.0f | segment prologue + epilogue (+ ET syndrome) %.1f\n", w, x[0], x[1], x[2], x[3],
                    x[0] - x[1] - x[2] - x[3], x[6], x[4]);
    }
}

int launch_any(int d0, const Coop3Args &a, int grid, bool et, bool nms, bool stamped, hipStream_t s)
{
    switch (d0) {
    case 7: return coop3_launch_d7(a, grid, et, nms, stamped, s);
    case 10: return coop3_launch_d10(a, grid, et, nms, stamped, s);
    case 14: return coop3_launch_d14(a, grid, et, nms, stamped, s);
    case 22: return coop3_launch_d22(a, grid, et, nms, stamped, s);
    case 27: return coop3_launch_d27(a, grid, et, nms, stamped, s);
    case 30: return coop3_launch_d30(a, grid, et, nms, stamped, s);
    default: return -1;
    }
}

// per-degree constants at run time (first-group degrees 7, 10, 14, 22, 27, 30)
template <template <int> class F>
auto g3_at(int d0) -> decltype(F<7>::v)
{
    return d0 == 7 ? F<7>::v : d0 == 10 ? F<10>::v : d0 == 14 ? F<14>::v : d0 == 22 ? F<22>::v : d0 == 27 ? F<27>::v
                                                                                                             : F<30>::v;
}
template <int D> struct RecwOf { static constexpr int v = G3<D>::RECW; };
template <int D> struct WsOf { static constexpr int v = G3<D>::WS; };
template <int D> struct LcsOf { static constexpr int v = G3<D>::LCS; };
template <int D> struct SmemOf { static constexpr size_t v = sizeof(Smem3<D, G3<D>::WS, 2>); };
template <int D> struct DistOf { static constexpr int v = G3<D>::DIST; };
template <int D> struct SOf { static constexpr int v = G3<D>::S; };
template <int D> struct XrOf { static constexpr int v = G3<D>::XR; };
template <int D> struct MrecOf { static constexpr int v = G3<D>::MREC; };
int g3_recw(int d0) { return g3_at<RecwOf>(d0); }
int g3_ws(int d0) { return g3_at<WsOf>(d0); }
size_t g3_smem(int d0) { return g3_at<SmemOf>(d0); }
int g3_dist(int d0) { return g3_at<DistOf>(d0); }
int g3_s(int d0) { return g3_at<SOf>(d0); }
int g3_xr(int d0) { return g3_at<XrOf>(d0); }
bool g3_degree_ok(int d0) { return d0 == 7 || d0 == 10 || d0 == 14 || d0 == 22 || d0 == 27 || d0 == 30; }
static_assert(SmemOf<7>::v + 512 <= 160 * 1024 && SmemOf<10>::v + 512 <= 160 * 1024 && SmemOf<14>::v + 512 <= 160 * 1024 &&
                  SmemOf<22>::v + 512 <= 160 * 1024 && SmemOf<27>::v + 512 <= 160 * 1024 &&
                  SmemOf<30>::v + 512 <= 160 * 1024,
              "LDS: the workgroup's Smem3 plus the ET kernel's static words fit 160 KB");
int g3_lcs(int d0) { return g3_at<LcsOf>(d0); }

// The chain wave's priority (s_setprio level; LDPC_COOP3_PRIO overrides).
// r1/2 (WS = 6): the chain shares its SIMD with the memory wave only and is
// the critical wave: 3.  WS = 4 (every other degree): the chain shares SIMD 0
// with slab wave 0, and at level 3 it took that wave's VALU during its post
// (r06l stamps, r2/3: slab 0 busy 2397 of a 2615-cycle period, slabs 2 / 3
// ~1915).  The chain has slack there; levels 0 / 1 / 2 / 3, same box, ms
// (r06n, profiles/r06n_ab_chain_prio.txt): r1/2 34.76 / 34.77 / 33.16 / 33.18;
// r2/3 37.29 / 36.24 / 37.86 / 37.87; shaped r3/4 29.42 / 29.50 / 31.78 /
// 31.81; shaped r5/6 37.53 / 37.85 / 37.85 / 37.86; r8/9 and r9/10 flat
// (within 0.3 %).  With the memory wave at level 0 (below), levels 0 / 1 / 3
// (r06u, profiles/r06u_ab_chain_prio.txt): r2/3 36.48 / 36.47 / 38.31; r3/4
// 29.39 / 29.42 / 32.15; r5/6 35.48 / 37.00 / 37.00; r8/9 31.17 / 31.20 /
// 31.19; r9/10 27.70 / 27.76 / 27.77 -- level 0 at every WS = 4 degree.
int coop3_chain_prio(int d0) { return g3_ws(d0) == 6 ? 3 : 0; }

// The memory wave's priority (LDPC_COOP3_MPRIO overrides).  r1/2: 2 (r04j:
// 0.35 % over 0; r06t flat).  WS = 4: it shares SIMD 2 with slab wave 1 and
// only issues memory ops and LDS copies -- at level 2 it held that slab wave
// back.  Levels 0 / 1 / 2 / 3, same box, ms (r06t,
// profiles/r06t_ab_mem_prio.txt): r2/3 36.43 / 36.42 / 36.67 / 36.69; shaped
// r3/4 29.47 / 29.69 / 29.75 / 29.74; shaped r5/6 35.47 / 37.82 / 37.82 /
// 37.84; r8/9 31.21 / 31.99 / 31.96 / 31.95; r9/10 27.75 / 28.55 / 28.45 /
// 28.55.
int coop3_mem_prio(int d0) { return g3_ws(d0) == 6 ? 2 : 0; }

}  // namespace

// message bytes per check and 16-codeword group (G3::MREC): 64 for first-group
// degree <= 8, 96 up to 16, 160 for the two-lanes-per-check degrees 22 .. 30
int coop3_mrec(int d0) { return g3_degree_ok(d0) ? g3_at<MrecOf>(d0) : 32 * ((d0 + 7) / 8 + 1); }

// OMS / MS as coop (coop_params_ok); NMS with factor <= 64 (msg_max <= 63: the
// products fit the i16 halves)
bool coop3_params_ok(const ldpc_params *p, const CoopCode &cc)
{
    if (p->algo == LDPC_ALGO_NMS)
        return cc.valid && p->var_min == -127 && p->var_max == 127 && p->msg_max >= 0 && p->msg_max <= 63 &&
               p->factor >= 0 && p->factor <= 64;
    return coop_params_ok(p);
}

// V and P are addressed with 64-bit flat addresses: no batch cap
bool coop3_stride_ok(int stride) { return stride > 0 && stride % 64 == 0; }


// host side of coop3's schedule: the window plan with every window's slots
// permuted (distance-2 forwarding sources and readers in slab wave 0) and the
// records rewritten (forwarding codes, chain steps).  1 = no coop3 schedule
// for this code, 0 = ok, < 0 = error (status set)
int coop3_plan_host(const ldpc_code *h, int ws, int r, Coop3Host &o)
{
    o = Coop3Host{};
    if (!h->staircase || h->n_groups != 2 || !g3_degree_ok(h->group_deg[0])) return 1;
    const int D0 = h->group_deg[0], X = D0 - 2, RECW = g3_recw(D0);
    if (ws != g3_ws(D0) || r != 2)
        return ldpc_set_error(LDPC_EINVAL, "LDPC_COOP3_WS must be %d for first-group degree %d, LDPC_COOP3_R 2",
                              g3_ws(D0), D0);
    const int S = g3_s(D0), dist = g3_dist(D0);
    CoopPlan &pl = o.pl;
    // dist 1: neighbouring windows share no information variable; the plan's
    // forwarding codes mark the reads of values written 2 .. r+3 windows
    // earlier, of which distance 2 (writer's post and reader's pre in the same
    // period) puts writer and reader in slab wave 0.  dist 2 (WS = 2): windows
    // u and u+2 share none either, so no pair needs a slot of its own
    if (coop_build_plan(h, S, r + 2, dist, RECW, pl, true) != 0) return 1;
    const int nw = (int)pl.first.size();
    auto rec_at = [&](int u, int k) { return &pl.tab[((size_t)u * S + k) * RECW]; };
    auto code_at = [&](const uint32_t *rec, int j) { return (rec[D0 + 1 + j / 2] >> (16 * (j & 1))) & 0xFFFFu; };
    // distance-2 writers and readers -> slab wave 0 (slots 0..7);
    // the other checks keep their order, the inactive slots come last
    std::vector<char> special((size_t)nw * S, 0);
    for (int u = 0; u < nw; u++)
        for (int k = 0; k < pl.count[u]; k++)
            for (int j = 0; j < X; j++) {
                const uint32_t f = code_at(rec_at(u, k), j);
                // forwarding code: dW << (6 + EB) | slot << EB | edge (coop.h; EB = 5 above 8 info edges)
                const int EB = coop_fwd_eb(X);
                if (dist != 1 || f == COOP_FWD_NONE || (int)(f >> (6 + EB)) != 2) continue;
                special[(size_t)u * S + k] = 1;
                special[(size_t)((u + nw - 2) % nw) * S + ((f >> EB) & 63)] = 1;
            }
    std::vector<int> check_at((size_t)nw * S);   // slot -> plan slot (= chain step)
    for (int u = 0; u < nw; u++) {
        int n = 0;
        for (int pass = 0; pass < 3; pass++)
            for (int k = 0; k < S; k++) {
                const bool act = k < pl.count[u], sp = special[(size_t)u * S + k] != 0;
                if ((pass == 0 && sp) || (pass == 1 && act && !sp) || (pass == 2 && !act)) {
                    if (pass == 0 && n >= 8) return 1;   // more than wave 0 holds: no coop3 schedule
                    check_at[(size_t)u * S + n] = k;
                    n++;
                }
            }
    }
    std::vector<uint32_t> tab(pl.tab.size());
    for (int u = 0; u < nw; u++)
        for (int kn = 0; kn < S; kn++) {
            const int k = check_at[(size_t)u * S + kn];
            const uint32_t *src = rec_at(u, k);
            uint32_t *rec = &tab[((size_t)u * S + kn) * RECW];
            std::copy(src, src + D0 + 1, rec);   // entries and meta (the forwarding codes are not used)
            if (k >= pl.count[u]) {   // inactive slot: sink V row n, sink message row m, no flags
                for (int j = 0; j < D0; j++) rec[j] = (uint32_t)h->n;
                rec[D0] = (uint32_t)h->m;
            } else {
                rec[D0] &= COOP_CHK_MASK | COOP_M_ACT;
                if (u == pl.tail) std::swap(rec[X], rec[D0 - 1]);   // prefetch always loads record entry D0-1
            }
            rec[D0] |= (uint32_t)k << STEP_SHIFT;
        }
    pl.tab.swap(tab);
    // self-check of what the kernel relies on, from the records themselves:
    // no information variable is shared by a window and its neighbour, and a
    // variable window u reads that window u-2 wrote (the writer's post and the
    // reader's pre run in the same period) has writer and reader in slab wave 0
    // (slots 0..7), which posts before its pre
    {
        std::vector<int> wu(h->n, -1), wk(h->n, -1);   // last writer window / slot per variable (two sweeps)
        for (int pass = 0; pass < 2; pass++)
            for (int u = 0; u < nw; u++)
                for (int k = 0; k < S; k++) {
                    const uint32_t *rec = &pl.tab[((size_t)u * S + k) * RECW];
                    if (!(rec[D0] & COOP_M_ACT)) continue;
                    for (int j = 0; j < X; j++) {
                        const uint32_t v = rec[j];
                        if (pass == 1 && wu[v] >= 0) {
                            const int d = (u - wu[v] + nw) % nw;
                            if ((d >= 1 && d <= dist) || (d == 0 && nw > 1 && wk[v] != k))
                                return ldpc_set_error(LDPC_EINVAL, "coop3 plan: variable %u in windows %d and %d", v,
                                                      wu[v], u);
                            if (d == 2 && (k >= 8 || wk[v] >= 8))
                                return ldpc_set_error(LDPC_EINVAL, "coop3 plan: distance-2 variable %u outside slab "
                                                      "wave 0 (slots %d, %d)", v, wk[v], k);
                        }
                        wu[v] = u;
                        wk[v] = k;
                    }
                }
    }
    o.S = S;
    o.nw = nw;
    o.recw = RECW;
    o.d0 = D0;
    return 0;
}

// slot records as coop3_decode reads them (see RECW): the info entries
// become the LDS offsets of their pieces in the line cache (LcPlan::piece),
// the parity entries rows of the group's parity part, and each record carries
// the line ops of its lane group (LcPlan::ops)
static void coop3_records(const Coop3Host &ho, const LcPlan &lp, int k, std::vector<uint32_t> &out)
{
    const int S = ho.S, nw = ho.nw, D0 = ho.d0, X = D0 - 2, RECW = ho.recw;
    const int XR = g3_xr(D0);   // info words: X, or 2 XH for the two-lanes-per-check degrees (sinks past X: 0)
    const int W_X = XR, W_O = XR + 1, W_META = XR + 2, NLD = (X + 7) / 8, W_LOP = RECW - 4 * NLD;   // G3
    out.assign((size_t)nw * S * RECW, 0);
    for (int u = 0; u < nw; u++)
        for (int kk = 0; kk < S; kk++) {
            const uint32_t *src = &ho.pl.tab[((size_t)u * S + kk) * RECW];
            uint32_t *rec = &out[((size_t)u * S + kk) * RECW];
            for (int j = 0; j < X; j++) rec[j] = lp.piece[((size_t)u * S + kk) * X + j];
            const uint32_t step = (src[D0] >> STEP_SHIFT) & 63u;   // (rows - k <= m < 65536: checked by coop3_plan_lc)
            const uint32_t xi = (step >> 3) * (CW * 8) + (step & 7);   // xo index (u16): [block][codeword][8 steps]
            rec[W_X] = (src[X] - (uint32_t)k) | xi << 16;
            rec[W_O] = (src[D0 - 1] - (uint32_t)k) | (step * 2 * NP * 16) << 16;              // + cst offset
            rec[W_META] = src[D0];
            // lane group kk's line ops (LcPlan::ops, S NLD per period: op sub * S + kk)
            for (int sub = 0; sub < NLD; sub++) {
                const size_t o = (size_t)u * S * NLD + (size_t)sub * S + kk;
                const uint32_t lines = lp.ops[o * 2], slots = lp.ops[o * 2 + 1];
                uint32_t *lw = rec + W_LOP + 4 * sub;
                lw[0] = (lines & 0xFFFFu) * 128u;        // line loaded (byte offset in the group's V block)
                lw[1] = (lines >> 16) * 128u;            // line written back
                // slot byte offsets with the line's swizzle z in bits 4..6: lane q's
                // piece is at (offset ^ 16 q) (LcPlan, coop.h)
                auto slot_off = [](uint32_t f) { return (f & LC_SLOT_MASK) * 128u + (f >> LC_SLOT_BITS) * 16u; };
                lw[2] = slot_off(slots & 0xFFFFu);       // slot written with the load of LC_PUT periods earlier
                lw[3] = slot_off(slots >> 16);           // slot written back
            }
        }
}

int coop3_plan_lc(const ldpc_code *h, Coop3Host &ho, LcPlan &lp)
{
    const int d0 = h->n_groups == 2 ? h->group_deg[0] : 0;
    const int ws = env_int3("LDPC_COOP3_WS", g3_ws(g3_degree_ok(d0) ? d0 : 7)), r = env_int3("LDPC_COOP3_R", 2);
    const int rc = coop3_plan_host(h, ws, r, ho);
    if (rc != 0) return rc;
    const int k = h->n - h->m;
    if (h->m > 0xFFFF) return 1;   // parity rows - k (and the sink row n - k = m) share a record word with 16-bit fields
    if (lc_build_plan(ho.pl.tab, ho.recw, ho.nw, ho.S, ho.d0, h->n, k, g3_lcs(ho.d0), lp) != 0) return 1;
    return 0;
}

int coop3_upload(const ldpc_code *h, CoopCode *cc)
{
    *cc = CoopCode{};
    Coop3Host ho;
    LcPlan lp;
    const int rc = coop3_plan_lc(h, ho, lp);
    if (rc != 0) return rc > 0 ? LDPC_OK : rc;
    std::vector<uint32_t> tab;
    coop3_records(ho, lp, h->n - h->m, tab);
    auto up = [&](uint32_t **d, const std::vector<uint32_t> &v) -> int {
        const size_t bytes = std::max<size_t>(v.size(), 1) * 4;
        if (hipMalloc(d, bytes) != hipSuccess) return ldpc_set_error(LDPC_ENOMEM, "coop3 tables");
        if (!v.empty() && hipMemcpy(*d, v.data(), v.size() * 4, hipMemcpyHostToDevice) != hipSuccess)
            return ldpc_set_error(LDPC_EDEVICE, "coop3 table upload");
        return LDPC_OK;
    };
    int e;
    if ((e = up(&cc->d_tab, tab)) != LDPC_OK || (e = up(&cc->d_lc_pro, lp.pro)) != LDPC_OK ||
        (e = up(&cc->d_lc_epi, lp.epi)) != LDPC_OK) {
        coop_free(cc);
        return e;
    }
    cc->valid = 1;
    cc->d0 = ho.d0;
    cc->S = ho.S;
    cc->R = 2;
    cc->nw = ho.nw;
    cc->tail = ho.pl.tail;
    cc->n_fwd = ho.pl.n_fwd;
    cc->x0 = (int)h->edge_var[h->check_start[0] + ho.d0 - 2];   // check 0's x edge
    cc->m0 = h->group_cnt[0];
    cc->d1 = h->group_deg[1];
    cc->lc_slots = lp.slots;
    cc->n_lc_pro = (int)lp.pro.size();
    cc->n_lc_epi = (int)lp.epi.size();
    return LDPC_OK;
}

// coop3's per-group block: the group's V rows 0 .. n+7 (row n and the line
// n / 8: the sinks) of 16 B, then its messages ((m + 1) checks x MREC B), an
// odd number of 128-B lines in all (groups spread over the L2 channels).  One
// block per group lets the memory wave address all of it with 32-bit buffer
// offsets from one resource
void coop3_group_layout_nm(int n, int m, int mrec, size_t *vpart, size_t *block)
{
    const size_t vlines = ((size_t)n + 8 + 7) / 8, mlines = ((size_t)(m + 1) * mrec + 127) / 128;
    size_t lines = vlines + mlines;
    if (lines % 2 == 0) lines++;
    *vpart = vlines * 128;
    *block = lines * 128;
}
void coop3_group_layout(const ldpc_code *h, size_t *vpart, size_t *block)
{
    coop3_group_layout_nm(h->n, h->m, coop3_mrec(h->n_groups >= 1 ? h->group_deg[0] : 7), vpart, block);
}
size_t coop3_group_bytes(const ldpc_code *h)
{
    size_t v, b;
    coop3_group_layout(h, &v, &b);
    return b;
}

// the workgroup's LDS (the ET kernel stages the hard bits of all n variables,
// u16 each, in it between segments)
bool coop3_et_in_kernel(const CoopCode &cc, int n) { return cc.valid && (size_t)n * 2 <= g3_smem(cc.d0); }

// ---- staged early termination (batches of more than one workgroup per CU):
// after a first launch of K iterations the codewords still decoding are
// compacted into dense 16-codeword groups of a second state buffer (V byte,
// message code and constant halves of each codeword: its slot in the pair
// words), decoded on from there (iterations K+1 ..), and their V moved back.
// A workgroup leaves only when all its 16 codewords have converged, so
// without compaction one slow codeword holds 15 converged ones in its
// workgroup's pipeline until the last iteration.
constexpr int ET_LIVE = -1;   // iters_used of a codeword still decoding after a stage

// the codewords of a stage still decoding (its[j] == ET_LIVE, j < n or
// *n_dev): their stage index -> sel, their batch slot (through prev, the
// stage's own map; none: the identity) -> map, their number -> *count
__global__ void et_select_k(const int32_t *its, int n, const int *n_dev, const int32_t *prev, int32_t *sel,
                            int32_t *map, int *count)
{
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    const int nn = n_dev ? *n_dev : n;
    const bool live = j < nn && its[j] == ET_LIVE;
    const unsigned long long m = __ballot(live);
    int base = 0;
    if ((threadIdx.x & 63) == 0 && m) base = atomicAdd(count, __popcll(m));
    base = __shfl(base, 0, 64);
    if (live) {
        const int k = base + __popcll(m & ((1ull << (threadIdx.x & 63)) - 1ull));
        sel[k] = j;
        map[k] = prev ? prev[j] : j;
    }
}

// dst group g2 (blockIdx.y), rows / checks of the group (x): V bytes and the
// message halves of the codewords map[16 g2 + i] (i < 16; the padding past
// count gets zeros)
__global__ void et_gather_k(const char *Vs, char *Vd, const int32_t *map, const int *count, int vrows, int mrows,
                            size_t gstride, size_t vpart, int mrec, bool half)
{
    const int g2 = blockIdx.y, nlive = *count;
    if (16 * g2 >= nlive) return;
    int src[16];
#pragma unroll
    for (int i = 0; i < 16; i++) src[i] = 16 * g2 + i < nlive ? map[16 * g2 + i] : -1;
    for (int r = blockIdx.x * blockDim.x + threadIdx.x; r < vrows + mrows; r += gridDim.x * blockDim.x) {
        char *d = Vd + (size_t)g2 * gstride;
        if (r < vrows) {   // V row r: byte i = codeword i
            uint32_t w[4] = {0, 0, 0, 0};
#pragma unroll
            for (int i = 0; i < 16; i++)
                if (src[i] >= 0) {
                    const uint8_t v = (uint8_t)Vs[(size_t)(src[i] >> 4) * gstride + (size_t)r * 16 + (src[i] & 15)];
                    w[i >> 2] |= (uint32_t)v << (8 * (i & 3));
                }
            *(uint4 *)(d + (size_t)r * 16) = make_uint4(w[0], w[1], w[2], w[3]);
        } else {   // message record of check c: pair q's (MA0, MB) words, codeword 2q + h in half h of each,
                   // then (mrec > 64) the pairs' MA1, MA2, .. words (8 each); half (two lanes per check,
                   // mrec 160): [8 pairs][W0, W1], [8 pairs][W2, W3], [8 pairs][MB]
            const int c = r - vrows, nw = mrec / 4;   // <= 40 words
            uint32_t w[40];
#pragma unroll
            for (int i = 0; i < 40; i++) w[i] = 0;
#pragma unroll
            for (int i = 0; i < 16; i++)
                if (src[i] >= 0) {
                    const char *rec = Vs + (size_t)(src[i] >> 4) * gstride + vpart + (size_t)c * mrec;
                    const int qs = (src[i] & 15) >> 1, hs = src[i] & 1, qd = i >> 1, hd = i & 1;
                    auto half_of = [&](int byte) { return (uint32_t)((const uint16_t *)(rec + byte))[hs] << (16 * hd); };
                    if (half) {
#pragma unroll
                        for (int k = 0; k < 2; k++) {
                            w[2 * qd + k] |= half_of(8 * qs + 4 * k);
                            w[16 + 2 * qd + k] |= half_of(64 + 8 * qs + 4 * k);
                        }
                        w[32 + qd] |= half_of(128 + 4 * qs);
                        continue;
                    }
                    const uint32_t ma = ((const uint16_t *)(rec + 8 * qs))[hs], mb = ((const uint16_t *)(rec + 8 * qs + 4))[hs];
                    w[2 * qd] |= ma << (16 * hd);
                    w[2 * qd + 1] |= mb << (16 * hd);
#pragma unroll
                    for (int k = 1; k < 4; k++)
                        if (64 + 32 * k <= mrec)
                            w[8 + 8 * k + qd] |= (uint32_t)((const uint16_t *)(rec + 32 + 32 * k + 4 * qs))[hs] << (16 * hd);
                }
            uint4 *o = (uint4 *)(d + vpart + (size_t)c * mrec);
#pragma unroll
            for (int k = 0; k < 10; k++)
                if (4 * k < nw) o[k] = make_uint4(w[4 * k], w[4 * k + 1], w[4 * k + 2], w[4 * k + 3]);
        }
    }
}

// the compacted codewords' V rows and iterations back to their batch slots
__global__ void et_scatter_k(const char *Vs, char *Vd, const int32_t *map, const int *count, const int32_t *its2,
                             int32_t *iters_used, int vrows, size_t gstride)
{
    const int g2 = blockIdx.y, nlive = *count;
    if (16 * g2 >= nlive) return;
    if (blockIdx.x == 0 && threadIdx.x < 16 && 16 * g2 + (int)threadIdx.x < nlive)
        iters_used[map[16 * g2 + threadIdx.x]] = its2[16 * g2 + threadIdx.x];
    int dst[16];
#pragma unroll
    for (int i = 0; i < 16; i++) dst[i] = 16 * g2 + i < nlive ? map[16 * g2 + i] : -1;
    for (int r = blockIdx.x * blockDim.x + threadIdx.x; r < vrows; r += gridDim.x * blockDim.x) {
        const uint4 v = *(const uint4 *)(Vs + (size_t)g2 * gstride + (size_t)r * 16);
        const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int i = 0; i < 16; i++)
            if (dst[i] >= 0)
                Vd[(size_t)(dst[i] >> 4) * gstride + (size_t)r * 16 + (dst[i] & 15)] = (char)(w[i >> 2] >> (8 * (i & 3)));
    }
}

// first-stage iterations of a staged early-termination decode (0: one stage)
int coop3_et_stage_iters(int batch, int iters)
{
    const int k = env_int3("LDPC_COOP3_ET_K", 20), min_batch = env_int3("LDPC_COOP3_ET_STAGE_MIN", 8192);
    return (k > 0 && k < iters && batch >= min_batch) ? k : 0;
}

int launch_coop3(const DecodeLaunch &L, const CoopCode &cc, hipStream_t s)
{
    if (!cc.valid || !coop3_stride_ok(L.stride) || L.vgroup == 0) return -1;
    if (L.iters_used && (!L.early || L.iters == 0)) {
        hipLaunchKernelGGL(fill_iters3_k, dim3((L.batch + 255) / 256), dim3(256), 0, s, L.batch, L.iters_used,
                           L.early ? 0 : L.iters);
        if (hipGetLastError() != hipSuccess) return -1;
    }
    if (L.iters == 0) return 0;
    const bool et = L.early != 0;
    if (et && (!L.iters_used || !coop3_et_in_kernel(cc, L.n))) return -1;
    Coop3Args a{};
    a.V = (int8_t *)L.V;
    a.gstride = L.vgroup;
    a.Mc = (uint8_t *)L.msg;
    a.tab = cc.d_tab;
    a.lc_pro = cc.d_lc_pro;
    a.lc_epi = cc.d_lc_epi;
    a.n_pro = cc.n_lc_pro;
    a.n_epi = cc.n_lc_epi;
    a.G = cc.nw * L.iters;
    a.nw = cc.nw;
    a.tail = cc.tail;
    a.mrows = L.m + 1;
    a.n = L.n;
    a.m = L.m;
    a.k = L.n - L.m;
    a.x0 = cc.x0;
    a.ev = L.d_edge_var;
    a.iters_used = L.iters_used;
    a.iters = L.iters;
    a.batch = L.batch;
    a.iter_base = 0;
    a.fill = L.iters;
    a.batch_dev = nullptr;
    a.m0 = cc.m0;
    a.d1 = cc.d1;
    a.rmm = (uint32_t)(L.msg_max * 256 + 255) * 0x00010001u;
    const bool nms = L.algo == LDPC_ALGO_NMS;
    a.coff = nms ? 0u : (uint32_t)(L.param * 256 + 255) * 0x00010001u;
    a.offp = nms ? 0u : (uint32_t)(L.param & 0xFFFF) * 0x00010001u;
    a.nmsf = nms ? (uint32_t)(L.param & 0xFFFF) * 0x00010001u : 0u;
    a.prio = std::min(3, std::max(0, env_int3("LDPC_COOP3_PRIO", coop3_chain_prio(cc.d0))));
    a.mprio = std::min(3, std::max(0, env_int3("LDPC_COOP3_MPRIO", coop3_mem_prio(cc.d0))));
    a.slab_prio = env_int3("LDPC_COOP3_SLAB_PRIO", 2);   // 0 none, 1 static (second waves), 2 fair by phase
    const int grid = L.stride / CW;
    a.remap = (grid % 8) == 0 && env_int3("LDPC_COOP3_REMAP", 1) != 0;   // XCD-aware codeword groups
    const bool stamped = env_int3("LDPC_COOP3_STAMP", 0) != 0 && !nms;
    if (stamped) {
        const size_t bytes = (size_t)grid * (g3_ws(cc.d0) + 2) * 8 * sizeof(unsigned long long);
        if (hipMalloc(&a.stamps, bytes) != hipSuccess) return -1;
        (void)hipMemsetAsync(a.stamps, 0, bytes, s);
    }
    int rc;
    auto launch_et = [&](const Coop3Args &x) -> int { return launch_any(cc.d0, x, grid, true, nms, stamped, s); };
    const int k1 = et && L.V2 && L.et2 ? coop3_et_stage_iters(L.batch, L.iters) : 0;
    if (et && k1 > 0 && !stamped) {
        // stage 0: K iterations on the whole batch (codewords still decoding
        // record ET_LIVE); then, every ET_STEP iterations, the live codewords
        // are compacted into the other of two dense buffers and decoded on
        // from there; each stage's codewords go back to their batch slots
        // (V rows and iterations) after it
        const int step = std::max(1, env_int3("LDPC_COOP3_ET_STEP", 5));
        size_t vpart = 0, block = 0;
        const int mrec = coop3_mrec(cc.d0);
        coop3_group_layout_nm(L.n, L.m, mrec, &vpart, &block);
        const size_t vbytes = (size_t)grid * L.vgroup;
        char *buf[2] = {(char *)L.V2, (char *)L.V2 + vbytes};
        const int S = L.stride;
        int32_t *sel = L.et2, *map[2] = {L.et2 + S, L.et2 + 2 * S}, *its[2] = {L.et2 + 3 * S, L.et2 + 4 * S};
        int *count = (int *)(L.et2 + 5 * S);   // one counter per stage (<= 64 stages)
        Coop3Args a0 = a;
        a0.iters = k1;
        a0.fill = ET_LIVE;
        if (launch_et(a0)) return -1;
        const char *src = (const char *)L.V;
        const int32_t *src_its = L.iters_used, *src_map = nullptr;
        const int *src_n = nullptr;
        int done = k1;
        // at most 64 stages (one counter each in et2): the 64th takes every
        // iteration left, so the decode always reaches L.iters
        constexpr int MAX_STAGES = 64;
        for (int st = 0; done < L.iters; st++) {
            const int k = st == MAX_STAGES - 1 ? L.iters - done : std::min(step, L.iters - done), b = st & 1;
            const bool last = done + k >= L.iters;
            if (hipMemsetAsync(count + st, 0, sizeof(int), s) != hipSuccess) return -1;
            hipLaunchKernelGGL(et_select_k, dim3((S + 255) / 256), dim3(256), 0, s, src_its, L.batch, src_n, src_map,
                               sel, map[b], count + st);
            hipLaunchKernelGGL(et_gather_k, dim3(64, grid), dim3(256), 0, s, src, buf[b], sel, count + st, L.n + 8,
                               L.m + 1, L.vgroup, vpart, mrec, cc.d0 >= 22);
            if (hipGetLastError() != hipSuccess) return -1;
            // the compacted codewords from iteration `done` on: no XCD remap
            // (the live groups are the first ones), the batch read on the device
            Coop3Args as = a;
            as.V = (int8_t *)buf[b];
            as.Mc = (uint8_t *)buf[b] + vpart;
            as.iters = k;
            as.iter_base = done;
            as.fill = last ? L.iters : ET_LIVE;
            as.batch_dev = count + st;
            as.iters_used = its[b];
            as.remap = false;
            if (launch_et(as)) return -1;
            hipLaunchKernelGGL(et_scatter_k, dim3(64, grid), dim3(256), 0, s, (const char *)buf[b], (char *)L.V, map[b],
                               count + st, its[b], L.iters_used, L.n, L.vgroup);
            if (hipGetLastError() != hipSuccess) return -1;
            src = buf[b];
            src_its = its[b];
            src_map = map[b];
            src_n = count + st;
            done += k;
        }
        return 0;
    }
    rc = launch_any(cc.d0, a, grid, et, nms, stamped, s);
    if (stamped) {
        if (rc == 0)
            (g3_ws(cc.d0) == 6 ? report_stamps3<6> : g3_ws(cc.d0) == 4 ? report_stamps3<4> : report_stamps3<2>)(a.stamps,
                                                                                                            grid, s);
        (void)hipFree(a.stamps);
    }
    return rc;
}

extern "C" int ldpc_code_coop3_lc_banks(const ldpc_code *h, long long *swizzled, long long *plain)
{
    if (!h || !swizzled || !plain) return ldpc_set_error(LDPC_EINVAL, "coop3 lc banks args");
    Coop3Host ho;
    LcPlan lp;
    const int rc = coop3_plan_lc(h, ho, lp);
    if (rc < 0) return rc;
    *swizzled = rc == 0 ? lp.bank_extra : 0;
    *plain = rc == 0 ? lp.bank_extra_plain : 0;
    return LDPC_OK;
}

// line-cache statistics of a code's coop3 schedule (tests, tools)
extern "C" int ldpc_code_coop3_lc_info(const ldpc_code *h, int *slots, int *max_slots, int *residencies,
                                       int *prologue, int *epilogue)
{
    if (!h || !slots) return ldpc_set_error(LDPC_EINVAL, "coop3 lc info args");
    Coop3Host ho;
    LcPlan lp;
    const int rc = coop3_plan_lc(h, ho, lp);
    if (rc < 0) return rc;
    *slots = rc == 0 ? lp.slots : 0;
    if (max_slots) *max_slots = rc == 0 ? g3_lcs(ho.d0) : 0;
    if (residencies) *residencies = rc == 0 ? lp.residencies : 0;
    if (prologue) *prologue = rc == 0 ? (int)lp.pro.size() : 0;
    if (epilogue) *epilogue = rc == 0 ? (int)lp.epi.size() : 0;
    return LDPC_OK;
}
