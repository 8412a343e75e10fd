// code.cpp -- runtime H tables (replaces the reference's compile-time
// PosNoeudsVariable[] headers, code/x86/Constantes/*/constantes_sse.h), table
// loaders, the DVB-S2 Annex-B builder, error reporting and the host side of
// the synthetic channel.
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <sstream>

#include "ldpc_internal.h"
#include "coop.h"

bool windowed_supported(const ldpc_code *h);   // windowed.hip
int ldpc_plan_build(ldpc_code *h);             // plan.cpp

// ---------------------------------------------------------------- errors
static thread_local std::string g_last_error;

int ldpc_set_error(int status, const char *fmt, ...)
{
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_last_error = buf;
    return status;
}

extern "C" const char *ldpc_last_error(void) { return g_last_error.c_str(); }

extern "C" const char *ldpc_strerror(int status)
{
    switch (status) {
    case LDPC_OK: return "ok";
    case LDPC_EINVAL: return "invalid argument";
    case LDPC_EUNSUPPORTED: return "unsupported configuration";
    case LDPC_EDEVICE: return "device (HIP) error";
    case LDPC_ENOMEM: return "out of memory";
    case LDPC_EIO: return "I/O or table format error";
    default: return "unknown error";
    }
}

extern "C" int ldpc_abi_version(void) { return LDPC_ABI_VERSION; }

extern "C" void ldpc_params_default(ldpc_params *p)
{
    if (!p) return;
    // defaults of code/x86/main_p.cpp:90-104,133-141 (offset 1, factor 29,
    // VAR +-127, MSG +-31; float OMS offset 0.15)
    p->algo = LDPC_ALGO_OMS;
    p->offset = 1;
    p->factor = 29;
    p->beta = 0.15f;
    p->var_min = -127;
    p->var_max = 127;
    p->msg_min = -31;
    p->msg_max = 31;
    p->early_term = 0;
}

// ---------------------------------------------------------------- codes
int ldpc_code_finalize(ldpc_code *h)
{
    h->check_deg.clear();
    h->check_start.clear();
    h->check_group.clear();
    h->max_deg = 0;
    int start = 0;
    for (int g = 0; g < h->n_groups; g++) {
        for (int i = 0; i < h->group_cnt[g]; i++) {
            h->check_deg.push_back(h->group_deg[g]);
            h->check_start.push_back(start);
            h->check_group.push_back(g);
            start += h->group_deg[g];
        }
        h->max_deg = std::max(h->max_deg, h->group_deg[g]);
    }
    if (start != h->e || (int)h->check_deg.size() != h->m)
        return ldpc_set_error(LDPC_EINVAL, "group table sums to %d edges / %zu checks, expected %d / %d",
                              start, h->check_deg.size(), h->e, h->m);
    for (int c = 0; c < h->m; c++) {
        const uint32_t *ev = &h->edge_var[h->check_start[c]];
        for (int j = 0; j < h->check_deg[c]; j++)
            for (int k = 0; k < j; k++)
                if (ev[j] == ev[k])
                    return ldpc_set_error(LDPC_EINVAL, "check %d lists variable %u twice", c, ev[j]);
    }
    return ldpc_plan_build(h);
}

extern "C" int ldpc_code_create(int n, int m, int n_groups, const int *group_deg, const int *group_cnt,
                                const uint32_t *edge_var, ldpc_code **out)
{
    if (!out) return ldpc_set_error(LDPC_EINVAL, "out is NULL");
    *out = nullptr;
    if (n <= 0 || m <= 0 || n_groups <= 0 || !group_deg || !group_cnt || !edge_var)
        return ldpc_set_error(LDPC_EINVAL, "bad code dimensions / NULL table");
    long e = 0, mm = 0;
    for (int g = 0; g < n_groups; g++) {
        if (group_deg[g] < 2 || group_deg[g] > 64 || group_cnt[g] <= 0)
            return ldpc_set_error(LDPC_EUNSUPPORTED, "group %d: degree %d count %d (degree must be 2..64)",
                                  g, group_deg[g], group_cnt[g]);
        e += (long)group_deg[g] * group_cnt[g];
        mm += group_cnt[g];
    }
    if (mm != m) return ldpc_set_error(LDPC_EINVAL, "groups hold %ld checks, m = %d", mm, m);
    for (long i = 0; i < e; i++)
        if (edge_var[i] >= (uint32_t)n)
            return ldpc_set_error(LDPC_EINVAL, "edge %ld: variable %u >= n %d", i, edge_var[i], n);
    auto *h = new (std::nothrow) ldpc_code();
    if (!h) return ldpc_set_error(LDPC_ENOMEM, "host alloc");
    h->n = n;
    h->m = m;
    h->e = (int)e;
    h->n_groups = n_groups;
    h->group_deg.assign(group_deg, group_deg + n_groups);
    h->group_cnt.assign(group_cnt, group_cnt + n_groups);
    h->edge_var.assign(edge_var, edge_var + e);
    int rc = ldpc_code_finalize(h);
    if (rc != LDPC_OK) {
        delete h;
        return rc;
    }
    *out = h;
    return LDPC_OK;
}

// DVB-S2 IRA structure: check r (0..M-1) is connected to info bit v = 360*g + k
// when r == (x + k*q) mod M for an address x of row g (ETSI EN 302 307 Annex B;
// encoder form in code/x86/CEncoder/GenericEncoder.cpp:55-69), plus the parity
// staircase.  Layered order of the reference tables: checks 1..M-1, then 0.
extern "C" int ldpc_code_from_dvbs2_table(int n, int k_info, int n_rows, const int *row_len,
                                          const int *row_addr, ldpc_code **out)
{
    if (!out) return ldpc_set_error(LDPC_EINVAL, "out is NULL");
    *out = nullptr;
    const int m = n - k_info;
    if (n <= 0 || k_info <= 0 || m <= 0 || k_info % 360 || m % 360 || n_rows != k_info / 360 || !row_len ||
        !row_addr)
        return ldpc_set_error(LDPC_EINVAL, "DVB-S2 table: n=%d k=%d rows=%d (need k/360 rows, 360 | k, m)", n,
                              k_info, n_rows);
    const int q = m / 360;
    std::vector<std::vector<uint32_t>> info(m);
    const int *a = row_addr;
    for (int g = 0; g < n_rows; g++) {
        for (int t = 0; t < row_len[g]; t++)
            if (a[t] < 0 || a[t] >= m)
                return ldpc_set_error(LDPC_EINVAL, "row %d: address %d out of range", g, a[t]);
        for (int k = 0; k < 360; k++)
            for (int t = 0; t < row_len[g]; t++) info[(a[t] + (long)k * q) % m].push_back(360 * g + k);
        a += row_len[g];
    }
    std::vector<uint32_t> edges;
    std::vector<int> gdeg, gcnt;
    for (int idx = 0; idx < m; idx++) {
        const int r = (idx + 1) % m;   // 1, 2, ..., m-1, 0
        auto &lst = info[r];
        std::sort(lst.begin(), lst.end());
        int d = (int)lst.size();
        edges.insert(edges.end(), lst.begin(), lst.end());
        if (r > 0) {
            edges.push_back(k_info + r - 1);
            edges.push_back(k_info + r);
            d += 2;
        } else {
            edges.push_back(k_info);
            d += 1;
        }
        if (!gdeg.empty() && gdeg.back() == d)
            gcnt.back()++;
        else {
            gdeg.push_back(d);
            gcnt.push_back(1);
        }
    }
    int rc = ldpc_code_create(n, m, (int)gdeg.size(), gdeg.data(), gcnt.data(), edges.data(), out);
    if (rc == LDPC_OK) {
        (*out)->dvbs2_q = q;
        (*out)->dvbs2_row_len.assign(row_len, row_len + n_rows);
        long tot = 0;
        for (int g = 0; g < n_rows; g++) tot += row_len[g];
        (*out)->dvbs2_row_addr.assign(row_addr, row_addr + tot);
    }
    return rc;
}

// DVB-S2 IRA encoder, as the reference's GenericEncoder::encode
// (code/x86/CEncoder/GenericEncoder.cpp:38-78): accumulate the Annex-B
// parity addresses of every set information bit, then the staircase
// p[j] ^= p[j-1].  codeword = [info (K bits), parity (M bits)].
extern "C" int ldpc_dvbs2_encode(const ldpc_code *h, const uint8_t *info, uint8_t *codeword, int batch)
{
    if (!h || (!info && batch > 0) || (!codeword && batch > 0) || batch < 0)
        return ldpc_set_error(LDPC_EINVAL, "encode args");
    if (h->dvbs2_q <= 0) return ldpc_set_error(LDPC_EUNSUPPORTED, "code was not built from a DVB-S2 table");
    const int n = h->n, m = h->m, k = n - m, q = h->dvbs2_q;
    for (int b = 0; b < batch; b++) {
        const uint8_t *in = info + (size_t)b * k;
        uint8_t *cw = codeword + (size_t)b * n;
        uint8_t *p = cw + k;
        memset(p, 0, (size_t)m);
        const int *addr = h->dvbs2_row_addr.data();
        for (size_t g = 0; g < h->dvbs2_row_len.size(); g++) {
            const int len = h->dvbs2_row_len[g];
            for (int kk = 0; kk < 360; kk++) {
                const int v = (int)g * 360 + kk;
                const uint8_t bit = in[v] & 1;
                cw[v] = bit;
                if (bit)
                    for (int t = 0; t < len; t++) p[(addr[t] + (long)kk * q) % m] ^= 1;
            }
            addr += len;
        }
        for (int j = 1; j < m; j++) p[j] ^= p[j - 1];
    }
    return LDPC_OK;
}

static int load_ldpc_binary(const std::string &data, ldpc_code **out)
{
    auto rd32 = [&](size_t off) {
        uint32_t v;
        memcpy(&v, data.data() + off, 4);
        return v;
    };
    if (data.size() < 24 || memcmp(data.data(), "LDPCH001", 8) != 0)
        return ldpc_set_error(LDPC_EIO, "not a LDPCH001 table");
    uint32_t n = rd32(8), m = rd32(12), e = rd32(16), ng = rd32(20);
    if (ng == 0 || ng > 1024 || data.size() != 24 + 8ull * ng + 4ull * e)
        return ldpc_set_error(LDPC_EIO, "truncated LDPCH001 table");
    std::vector<int> gd(ng), gc(ng);
    for (uint32_t g = 0; g < ng; g++) {
        gd[g] = (int)rd32(24 + 8 * g);
        gc[g] = (int)rd32(28 + 8 * g);
    }
    std::vector<uint32_t> ev(e);
    memcpy(ev.data(), data.data() + 24 + 8ull * ng, 4ull * e);
    return ldpc_code_create((int)n, (int)m, (int)ng, gd.data(), gc.data(), ev.data(), out);
}

static int load_dvbs2_text(const std::string &data, ldpc_code **out)
{
    std::istringstream in(data);
    std::string line;
    int n = -1, k = -1;
    std::vector<int> len, addr;
    while (std::getline(in, line)) {
        if (line.empty()) continue;
        if (line[0] == '#') {
            const char *p = strstr(line.c_str(), "N=");
            const char *q = strstr(line.c_str(), "K=");
            if (p && q) {
                n = atoi(p + 2);
                k = atoi(q + 2);
            }
            continue;
        }
        std::istringstream ls(line);
        int v, c = 0;
        while (ls >> v) {
            addr.push_back(v);
            c++;
        }
        if (c) len.push_back(c);
    }
    if (n <= 0 || k <= 0) return ldpc_set_error(LDPC_EIO, "DVB-S2 table without '# N=.. K=..' header");
    return ldpc_code_from_dvbs2_table(n, k, (int)len.size(), len.data(), addr.data(), out);
}

extern "C" int ldpc_code_load(const char *path, ldpc_code **out)
{
    if (!path || !out) return ldpc_set_error(LDPC_EINVAL, "NULL path/out");
    *out = nullptr;
    std::ifstream f(path, std::ios::binary);
    if (!f) return ldpc_set_error(LDPC_EIO, "cannot open %s", path);
    std::string data((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
    if (data.size() >= 8 && memcmp(data.data(), "LDPCH001", 8) == 0) return load_ldpc_binary(data, out);
    return load_dvbs2_text(data, out);
}

extern "C" int ldpc_code_info(const ldpc_code *h, int *n, int *m, int *e, int *n_groups, int *max_deg)
{
    if (!h) return ldpc_set_error(LDPC_EINVAL, "NULL code");
    if (n) *n = h->n;
    if (m) *m = h->m;
    if (e) *e = h->e;
    if (n_groups) *n_groups = h->n_groups;
    if (max_deg) *max_deg = h->max_deg;
    return LDPC_OK;
}

extern "C" int ldpc_code_edges(const ldpc_code *h, uint32_t *edge_var, int *group_deg, int *group_cnt)
{
    if (!h) return ldpc_set_error(LDPC_EINVAL, "NULL code");
    if (edge_var) memcpy(edge_var, h->edge_var.data(), 4ull * h->e);
    if (group_deg) memcpy(group_deg, h->group_deg.data(), sizeof(int) * h->n_groups);
    if (group_cnt) memcpy(group_cnt, h->group_cnt.data(), sizeof(int) * h->n_groups);
    return LDPC_OK;
}

extern "C" int ldpc_code_plan_info(const ldpc_code *h, int *staircase, int *n_windows, int *min_hazard)
{
    if (!h) return ldpc_set_error(LDPC_EINVAL, "NULL code");
    if (staircase) *staircase = h->staircase ? 1 : 0;
    if (n_windows) *n_windows = windowed_supported(h) ? (int)h->windows.size() : 0;
    if (min_hazard) *min_hazard = h->min_hazard;
    return LDPC_OK;
}

int ldpc_plan_windows(const ldpc_code *h, int S, int P, std::vector<ldpc_window> &out);   // plan.cpp

extern "C" int ldpc_code_window_plan(const ldpc_code *h, int S, int P, int *first, int *count, int max_windows,
                                     int *n_windows)
{
    if (!h || S < 1 || S > 64 || P < 0 || !n_windows) return ldpc_set_error(LDPC_EINVAL, "window plan args");
    std::vector<ldpc_window> w;
    int rc = ldpc_plan_windows(h, S, P, w);
    if (rc != LDPC_OK) return rc;
    *n_windows = (int)w.size();
    for (int i = 0; i < (int)w.size() && i < max_windows; i++) {
        if (first) first[i] = w[i].first;
        if (count) count[i] = w[i].count;
    }
    return LDPC_OK;
}

int coop_plan_windows(const ldpc_code *h, int S, int R, int dist, std::vector<int> &first, std::vector<int> &count,
                      int *tail, int *n_fwd);   // coop.hip

extern "C" int ldpc_code_coop_plan(const ldpc_code *h, int S, int R, int *first, int *count, int max_windows,
                                   int *n_windows, int *tail, int *n_fwd)
{
    return ldpc_code_coop_plan_dist(h, S, R, 1, first, count, max_windows, n_windows, tail, n_fwd);
}

extern "C" int ldpc_code_coop_plan_dist(const ldpc_code *h, int S, int R, int dist, int *first, int *count,
                                        int max_windows, int *n_windows, int *tail, int *n_fwd)
{
    if (!h || S < 1 || S > 64 || R < 1 || R > 6 || dist < 1 || dist > 2 || !n_windows)
        return ldpc_set_error(LDPC_EINVAL, "coop plan args");
    std::vector<int> f, c;
    int t = -1, nf = 0;
    *n_windows = 0;
    if (coop_plan_windows(h, S, R, dist, f, c, &t, &nf) != 0) return LDPC_OK;   // no cooperative schedule
    *n_windows = (int)f.size();
    for (int i = 0; i < (int)f.size() && i < max_windows; i++) {
        if (first) first[i] = f[i];
        if (count) count[i] = c[i];
    }
    if (tail) *tail = t;
    if (n_fwd) *n_fwd = nf;
    return LDPC_OK;
}

extern "C" void ldpc_code_destroy(ldpc_code *h) { delete h; }

// ---------------------------------------------------------------- channel
extern "C" double ldpc_awgn_sigma(double ebn0_db, double rate)
{
    // CChanelAWGN_MKL::configure, code/x86/CChanel/CChanelAWGN_MKL.cpp:102-105
    double interm = -0.1 * (ebn0_db + 10.0 * std::log10(rate));
    return std::sqrt(std::pow(10.0, interm) / 2.0);
}

// CChanelAWGN_MKL::configure with its es_n0 option (:97-104): the SNR given in
// Es/N0 (QPSK, 2 bits per symbol) is first turned into Eb/N0
extern "C" double ldpc_awgn_sigma_ex(double snr_db, double rate, int es_n0)
{
    const double ebn0 = es_n0 ? snr_db - 10.0 * std::log10(2.0 * rate) : snr_db;
    return ldpc_awgn_sigma(ebn0, rate);
}

extern "C" int ldpc_awgn_i8_table(double sigma, int factor, int sat, uint32_t *table)
{
    return ldpc_awgn_i8_table_ex(sigma, 1.0, 1.0, factor, sat, table);
}

// P(q <= v) for q = clamp(trunc(factor * norm * y), -sat, sat),
// y = -amp + sigma*z (bit 0; amp 1 BPSK, 0.707106781 QPSK, norm 1 or the
// 2 / sigma^2 normalisation: CChanelAWGN_MKL::generate, :127-143, and
// configure, :114-121).  With f = factor * norm:
// trunc(f*y) <= v  <=>  y < (v+1)/f  (v >= 0)   or   y <= v/f  (v < 0).
extern "C" int ldpc_awgn_i8_table_ex(double sigma, double amp, double norm, int factor, int sat, uint32_t *table)
{
    if (!table || sigma <= 0.0 || factor <= 0 || sat < 1 || sat > 31 || !(amp > 0.0) || !(norm > 0.0))
        return ldpc_set_error(LDPC_EINVAL, "awgn table: sigma>0, amp>0, norm>0, factor>0, 1<=sat<=31");
    const double f = (double)factor * norm;
    // 2*sat+1 levels -sat..sat need 2*sat thresholds; table[63] holds sat.
    for (int k = 0; k < 63; k++) table[k] = 0xFFFFFFFFu;
    table[63] = (uint32_t)sat;
    for (int k = 0; k < 2 * sat; k++) {
        int v = -sat + k;
        double t = (v >= 0) ? (double)(v + 1) / f : (double)v / f;
        double p = 0.5 * std::erfc(-((t + amp) / sigma) / std::sqrt(2.0));
        double u = std::floor(p * 4294967296.0);
        if (u < 0) u = 0;
        if (u > 4294967295.0) u = 4294967295.0;
        table[k] = (uint32_t)u;
    }
    return LDPC_OK;
}

static inline uint64_t splitmix64(uint64_t x)
{
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

// Generator definition (also implemented by the HIP kernel in decode.hip and
// by tests/golden/gen_golden.py): element idx = cw*N + i,
//   u = splitmix64(idx ^ (seed * 0xD1B54A32D192ED03)) >> 32
//   q0 = -sat + #{k < 2*sat : u >= table[k]}  (bit 0 sent as -1; sat = table[63])
//   q  = bit ? -q0 : q0
extern "C" int ldpc_awgn_i8_host(int n, int batch, uint64_t first_cw, uint64_t seed, const uint32_t *table,
                                 const uint8_t *codeword, int8_t *llr)
{
    if (n <= 0 || batch < 0 || !table || !llr) return ldpc_set_error(LDPC_EINVAL, "awgn host args");
    const int sat = (int)table[63];
    if (sat < 1 || sat > 31) return ldpc_set_error(LDPC_EINVAL, "awgn table: bad sat %d", sat);
    const uint64_t key = seed * 0xD1B54A32D192ED03ull;
    for (int b = 0; b < batch; b++)
        for (int i = 0; i < n; i++) {
            uint64_t idx = (first_cw + b) * (uint64_t)n + i;
            uint32_t u = (uint32_t)(splitmix64(idx ^ key) >> 32);
            int cnt = 0;
            for (int k = 0; k < 2 * sat; k++) cnt += (u >= table[k]);
            int q = cnt - sat;
            if (codeword && codeword[(size_t)b * n + i]) q = -q;
            llr[(size_t)b * n + i] = (int8_t)q;
        }
    return LDPC_OK;
}
