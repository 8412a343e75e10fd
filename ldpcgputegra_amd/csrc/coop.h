// coop.h -- the workgroup-cooperative DVB-S2 fast path (coop.hip).
#pragma once
#include "kernels.h"
#include "ldpc_internal.h"

struct CoopCode {
    int valid;
    int d0;          // degree of the first group (the tail check has d0 - 1)
    int S, R;        // checks per window, prefetch depth in windows
    int nw;          // windows per iteration (tail and empty windows included)
    int tail;        // window index of the tail check
    int n_fwd;       // forwarded info-edge reads per iteration (plan statistic)
    int x0;          // coop3: V row of check 0's x edge (the chain's first input)
    int m0, d1;      // coop3: checks of degree d0 (group 0), degree of the later group
    uint32_t *d_tab; // [nw][S][recw]
    // coop3 line cache (LcPlan): slots used, lines resident at a segment start / written back at its end
    int lc_slots, n_lc_pro, n_lc_epi;
    uint32_t *d_lc_pro, *d_lc_epi;
};

bool coop_params_ok(const ldpc_params *p);
int coop_upload(const ldpc_code *h, CoopCode *cc);
void coop_free(CoopCode *cc);
int launch_coop(const DecodeLaunch &L, const CoopCode &cc, hipStream_t s);
// early termination around per-iteration launches (coop with LDPC_COOP_ET_KERNEL=0): init,
// syndrome after iteration `it` (0-based; with L.Vs, snapshot of the codewords
// converging now), and the final merge of the snapshots into V (L.Vs only)
int coop_early_begin(const DecodeLaunch &L, hipStream_t s);
int coop_early_after_iter(const DecodeLaunch &L, int it, hipStream_t s);
int coop_early_end(const DecodeLaunch &L, hipStream_t s);
// host-side plan (tests: ldpc_code_coop_plan)
int coop_plan_windows(const ldpc_code *h, int S, int R, int dist, std::vector<int> &first, std::vector<int> &count,
                      int *tail, int *n_fwd);

// ---- window plan shared by coop.hip and coop3.hip ----
// Slot record [recw] u32: edge variables [D0], meta, forwarding codes (u16 per
// information edge: dW << (6 + EB) | slot << EB | edge, EB = coop_fwd_eb(X);
// 0xFFFF = none); codes with more than 8 information edges (X > 8) carry the
// ring-source bits in the record word after the codes (coop_src_word), not in
// the meta word.
constexpr uint32_t COOP_M_ACT = 1u << 20;            // slot holds a check
constexpr uint32_t COOP_M_FWD = 1u << 21;            // an info edge of the slot reads the LDS ring
constexpr int COOP_SRC_SHIFT = 22;                   // bit 22 + j: info edge j feeds the LDS ring
constexpr uint32_t COOP_CHK_MASK = (1u << 20) - 1;   // check index
constexpr uint32_t COOP_FWD_NONE = 0xFFFFu;
constexpr int coop_fwd_eb(int X) { return X > 8 ? 5 : 3; }          // edge bits of a forwarding code
constexpr int coop_src_word(int D0) { return D0 + 1 + (D0 - 1) / 2; }   // X > 8: the source-bits word

struct CoopPlan {
    std::vector<int> first, count;   // per window: first check, checks (0: empty window)
    int tail = -1, n_fwd = 0;        // window of the tail check; forwarded reads per iteration
    std::vector<uint32_t> tab;       // [nw][S][recw] slot records (want_tab)
};
// S <= 64 checks per window, R <= 6 prefetch windows; windows closer than
// dist + 1 (1: neighbours, 2: also next-but-one) share no information
// variable, reads of values written dist+1 .. R+dist windows earlier are
// forwarded through the LDS ring; -1: no cooperative schedule
int coop_build_plan(const ldpc_code *h, int S, int R, int dist, int recw, CoopPlan &o, bool want_tab);

// ---- coop3.hip: slab waves doing pre + post, i16 chain (first-group degree 7 or 10) ----
bool coop3_params_ok(const ldpc_params *p, const CoopCode &cc);
bool coop3_stride_ok(int stride);
// coop3's per-group block (V rows, then messages): bytes of the V part and of
// the block = the stride between two codeword groups (DecodeLaunch::vgroup)
void coop3_group_layout(const ldpc_code *h, size_t *vpart, size_t *block);
size_t coop3_group_bytes(const ldpc_code *h);
// compressed messages: [stride / 16][m + 1][8 pairs][2] u32 (4 B per codeword and check; row m is the sink)
int coop3_mrec(int d0);   // message bytes per check and 16-codeword group (64: first-group degree <= 8, 96: <= 16)
int coop3_upload(const ldpc_code *h, CoopCode *cc);
// host side of the coop3 schedule (coop3.hip): permuted slot records
struct Coop3Host {
    CoopPlan pl;                 // pl.tab: [nw][S][recw] records as the kernel reads them
    int S = 0, nw = 0, recw = 0, d0 = 0;
};
int coop3_plan_host(const ldpc_code *h, int ws, int r, Coop3Host &o);
struct LcPlan;
// the schedule and its line-cache plan (linecache.cpp): 0 ok, 1 none for this code, < 0 error
int coop3_plan_lc(const ldpc_code *h, Coop3Host &ho, LcPlan &lp);
int launch_coop3(const DecodeLaunch &L, const CoopCode &cc, hipStream_t s);
// first-stage iterations of a staged early-termination decode (0: one launch)
int coop3_et_stage_iters(int batch, int iters);

// ---- linecache.cpp: coop3's LDS line cache (info rows as 128-B lines) ----
constexpr int LC_GAP = 10;    // accesses of a line >= LC_GAP periods apart: separate residencies
constexpr int LC_LEAD = 3;   // a line is loaded (into VGPRs) >= 3 periods before its first access
constexpr int LC_PUT = 2;    // ... and written to its slot 2 periods after its load (coop3: loads first in a
                             // period, vmcnt(36) at its end completes those of the period before)
// A line's 8 rows sit in its slot XOR-swizzled: row i at piece position i ^ z
// (z = 0..7 per residency, chosen by the planner so that the 4 pieces one
// 32-lane half of a pre read / post write touches fall in distinct bank
// groups: the LDS serves a ds_read_b32 / ds_write_b16 half in one cycle only
// if its addresses hit distinct banks, and a piece's bank group is its
// position in the 128-B slot).  Slot fields carry z beside the slot index.
constexpr int LC_SLOT_BITS = 10;                       // slot index < 1024
constexpr uint32_t LC_SLOT_MASK = (1u << LC_SLOT_BITS) - 1;
struct LcPlan {
    int slots = 0;                 // LDS line slots used, the sink (slot 0) included
    int residencies = 0;           // line residencies per iteration
    std::vector<uint32_t> ops;     // [nw][S][2] (S line loads / writebacks per period, one per slab-wave lane
                                   //   group): load line | writeback line << 16,
                                   //   slot written (the load of 2 periods earlier) | writeback slot << 16
                                   //   (each 16-bit slot field: slot | z << LC_SLOT_BITS)
    std::vector<uint32_t> piece;   // [nw][S][D0 - 2]: LDS byte offset (from the cache) of each info entry's piece
    std::vector<uint32_t> pro;     // z << 26 | slot << 16 | line: lines resident at a segment start
    std::vector<uint32_t> epi;     // z << 26 | slot << 16 | line: dirty lines written back at a segment end
    // modelled extra LDS cycles of the pre reads + post writes per iteration
    // and workgroup (bank conflicts, lc_bank_extra), with the planner's
    // swizzle and with z = 0 everywhere
    long bank_extra = 0, bank_extra_plain = 0;
};
// tab: coop3's permuted slot records (Coop3Host::pl.tab); 0 = ok (plan self-checked), -1 = no plan
int lc_build_plan(const std::vector<uint32_t> &tab, int recw, int nw, int S, int D0, int n, int k, int max_slots,
                  LcPlan &o);
int lc_check_plan(const LcPlan &o, const std::vector<uint32_t> &tab, int recw, int nw, int S, int D0, int n, int k,
                  int iters);
// early termination inside the coop3 launch (the only form coop3 has)
bool coop3_et_in_kernel(const CoopCode &cc, int n);
