// kernels.hpp — device-side graph view, batch parameters and kernel launchers.
#pragma once
#include <string>
#include <vector>
#include <hip/hip_runtime.h>

#include <climits>
#include <cstdint>

namespace rgpu {

constexpr int kViews = 64;  // views per batch = wavefront width (lane j <-> view j)

// Uniform label words (kernels.hip): uw[v] = the label every member lane of v holds, or kMixed
// when they differ (the row is then the state).  Bit 31 (kChgFlag) of a uniform word is set when
// the label changed in the superstep that wrote the word; a uniform label is never INT32_MAX, so
// a flagged word never reads as kMixed.
constexpr int32_t kMixed = -1;
constexpr int32_t kChgFlag = INT32_MIN;
// Partitioned mode: the word of a ghost that received no record in the last two steps of the
// buffer's parity — uniform and unchanged (its label is never read: readers fold a neighbour's word
// only when flagged).  Without it such a ghost read as kMixed, and every slot to it cost a second
// dependent load (its change word) in the superstep kernel.
constexpr int32_t kGhostQuiet = 0x7f7f7f7f;
__host__ __device__ inline int32_t uw_label(int32_t w) { return w == kMixed ? kMixed : (w & 0x7fffffff); }
__host__ __device__ inline int32_t uw_word(int32_t u, bool changed) {
  return (u != kMixed && changed) ? (int32_t)((uint32_t)u | 0x80000000u) : u;
}

// One batch of views: hops[K] x windows[W], view bit j = w*KS + k (window-major, KS = hop
// stride of the run, K <= KS hops in this batch, KS*W <= 64).  Window-major order keeps the
// views a vertex belongs to (the long windows) in the low lanes of its label row.
struct BatchParams {
  int K, W, KS;
  int sorted;             // hop[] ascending: K1 advances floors instead of searching per hop
  int iv_max;             // K1 interval form for entities with <= iv_max points in range (< 0: off)
  int64_t hop[kViews];    // view timestamps (RangeAnalysisTask hop times)
  int64_t thr_v[kViews];  // vertex-set window of window index w: min(w_0..w_w)  (shrinkWindow)
  int64_t thr_e[kViews];  // edge window of window index w: w_w (viewAtWithWindow(t, setWindow))
  int64_t jump;           // > 0: hop[k] = hop[0] + k * jump for every k < K (K1's arithmetic hop search)
  // every view's vertex window equals its edge window (descending window lists): then a nodeath
  // slot's window bits imply both endpoints' membership (an EADD is a `+` point of both endpoints,
  // neither of which ever dies), so K2 / the ghost marking skip the neighbour's mask read for it
  int simple_ends;
  // K1 floor carry across a run's hop blocks (§8(f) row 2): 0 off; 1 write each
  // entity's floor index at hop[K-1] into the carry array; 2 also read the previous block's (its
  // last hop <= this block's hop[0]) and advance it instead of searching the history from scratch
  int carry;
};

// Sealed partition resident in HBM.
struct DevGraph {
  int64_t nv = 0, ne = 0, n_in = 0;
  const int64_t *voff = nullptr, *vkey = nullptr;    // vertex histories
  const int64_t *doff = nullptr, *dtime = nullptr;   // vertex death lists
  const uint64_t* dbits = nullptr;                   // bit v: vertex v has a death (null: read doff)
  const uint64_t* esimple = nullptr;                 // bit e: edge e is simple (edge_simple; built with
                                                     // the time-ordered slots; null: test per edge)
  const int32_t* ens = nullptr;                      // the other edges' ids, ascending (K1's SKIP form
  int64_t n_ens = 0;                                 // walks only these; built with esimple)
  const int32_t *esrc = nullptr, *edst = nullptr;    // edges sorted by (src, dst)
  const int64_t *eoff = nullptr, *ekey = nullptr;    // edge own histories
  const int64_t *out_off = nullptr, *in_off = nullptr;
  const int64_t* adj_off = nullptr;                  // out_off + in_off: static slot offset
  const int32_t* in_eid = nullptr;
  int64_t n_own = 0;                                 // ranks [0, n_own) owned (== nv, one partition)
  const int32_t* grank = nullptr;                    // global rank per local rank (null: identity)
  // heavy vertices (static slots > RGPU_HEAVY, power-law hubs): their slots are split into
  // segments of <= kSegSlots static slots, each compacted / gathered / marked by its own wave
  int64_t n_heavy = 0, n_seg = 0;
  const int32_t* hv_of = nullptr;   // [nv] heavy index or -1
  const int32_t* hv_seg = nullptr;  // [n_heavy+1] first segment of each heavy vertex
  const int32_t* seg_v = nullptr;   // [n_seg] vertex rank of the segment
  const int32_t* seg_h = nullptr;   // [n_seg] heavy index of the segment
  const int64_t* seg_lo = nullptr;  // [n_seg] first static slot (absolute, = adj_off[v] + offset)
  const int32_t* seg_n = nullptr;   // [n_seg] static slots in the segment
  // time-ordered static slots (tslots.hip; null: CSR order): per vertex newest last-add first
  const int32_t* ts_e = nullptr;    // [ne + n_in] edge of the slot
  const int32_t* ts_nb = nullptr;   // [ne + n_in] neighbour across it
  const int64_t* ts_t = nullptr;    // [ne + n_in] 4 * the edge's last add time + 2 nodeath + simple (tslots.hip)
  const int32_t* ts_g = nullptr;    // [ne + n_in] grank[ts_nb] (with grank): K2 streams the neighbour's
                                    // label instead of a random grank read per slot
};
// a ts_t word: the edge's last add time; whether neither endpoint ever died (nodeath: the edge's
// window bits then imply both endpoints' membership when the vertex and edge windows agree,
// BatchParams::simple_ends); whether the slot is simple (one add point and nodeath: K2 derives its
// window bits from the time alone)
__host__ __device__ inline int64_t ts_time(int64_t x) { return x >> 2; }
__host__ __device__ inline bool ts_simple(int64_t x) { return x & 1; }
__host__ __device__ inline bool ts_nodeath(int64_t x) { return x & 2; }
// Builds ts_e / ts_nb / ts_t (device arrays of ne + n_in entries) for g; temporaries are
// appended to `temps` (free them after the stream is synchronised).  False: not built (more
// than 2^31 slots), the graph keeps CSR order.
bool build_time_slots(hipStream_t s, const DevGraph& g, int32_t* ts_e, int32_t* ts_nb, int64_t* ts_t,
                      std::vector<void*>& temps);
void build_slot_labels(hipStream_t s, int64_t n, const int32_t* ts_nb, const int32_t* grank, int32_t* ts_g);
constexpr int kSegSlots = 512;
// hub segments per wave and round in the per-superstep hub kernels (k_heavy_gather / k_heavy_mark):
// their prologue loads that many segments' vertex, flag and count at once (lane = segment); the
// value comes from KernOpts.hub_pro (C4, profiles/r05/ab_hubpro_c4.jsonl + ab_occ_c4.jsonl: heavy
// 64.7 ms serial at 1, 49.9 at 8, 48.3 at 16, 47.9 at 32)
constexpr int kHubPro = 32;
constexpr int kHubProPart = 4;  // partitioned contexts and graphs below 2^24 vertices (rgpu_run_view_batch)
// superstep options (k_cc_step_pk, k_heavy_gather, k_cc_slots; RGPU_STEP_OPTS, all by default):
// members holding the final label finished lane-parallel; full folds (one label on every view of
// the member) as a segmented min over the pack (a wave min over a hub segment or a big member's
// chunks, and K2's superstep-1 fold); simple members (every fold full) visited lane-parallel
constexpr int kStepFinLanes = 1, kStepSegMin = 2, kStepSimple = 4;
// (after K2, k_hub_demote) an owned hub keeping at most 64 slots, all in one segment, takes the light path
// for the batch
constexpr int kHubDemote = 8;
// supersteps >= kLongSteps of a long-window batch run the short-window superstep form (launch_cc_step)
constexpr int kLongSteps = 8;
// The kernel options of one run.  rgpu_run_view_batch fills them once per run (the parity tests
// of tests/test_gpu_step_forms.py set RGPU_STEP_OPTS / RGPU_HUB_PRO / RGPU_LONG_STEPS to run every
// superstep form; the defaults are the measured best) and hands them to every launcher, so that a
// run never reads the environment while it launches (loopback partitions are threads of one process).
struct KernOpts {
  int step = kStepFinLanes | kStepSegMin | kStepSimple | kHubDemote;  // superstep options above
  int hub_pro = kHubPro;                                  // hub segments per wave and round, 1..64
  int long_steps = kLongSteps;                            // first superstep of the short form in a long batch
};

// Per-batch state of the heavy-vertex path (one per batch slot).
struct HeavyBuf {
  int32_t* segcnt = nullptr;   // [n_seg] kept slots of the segment (compacted at seg_lo)
  uint64_t* segor = nullptr;   // [n_seg] OR of the segment's kept slot masks
  int32_t* best = nullptr;     // [n_heavy][64] partial minima of the step (INT32_MAX when idle)
  double* pacc = nullptr;      // [n_heavy][64] PageRank pull accumulators (0 when idle)
};

// Small per-batch state cleared by the first kernel of the batch (no memset launches).
struct BatchClear {
  unsigned long long* stats = nullptr;
  int64_t n_stats = 0;
  int32_t* flags = nullptr;
  int64_t n_flags = 0;
  uint8_t* act[3] = {nullptr, nullptr, nullptr};
  int64_t n_act_words = 0;  // uint64 words per act buffer
  uint64_t* cb[3] = {nullptr, nullptr, nullptr};  // changed bits (ChgBits)
  int64_t n_cb_words = 0;
  int32_t* ccount = nullptr;  // changed-vertex counts (kCountShards per step)
  int64_t n_ccount = 0;
};

// Per-step OR of the views (lanes) in which some label changed: words lanechg[step*kLaneShards +
// shard], one non-returning atomicOr per block that saw a change (64 shards: thousands of
// blocks on one word serialise at the memory side; a returning or read-first form made every
// such block wait a round trip at its end, +8 % on the C2 superstep kernel).  The summary
// kernel folds the shards into lanefold[step] so the host copies 128 words per batch.  A view's
// last changing step gives the superstep count the reference's job runs (AnalysisTask.endStep
// :208-225): min(maxSteps, last + 1).
constexpr int kLaneShards = 64;
// changed-vertex counts per superstep, ccount[step * kCountShards + shard] (int32, cleared per
// batch): the dense-step rule of the superstep kernels (kernels.hip dense_rule, RGPU_DENSE)
constexpr int kCountShards = 64;
// Per-view minimum member label of a batch, sharded: mneg[shard][view] = INT32_MAX - min label of the
// shard's members (0: none), atomicMax-ed by K2 and cleared with the batch's counts.  A uniform vertex
// whose label equals that minimum on every member lane holds its final label: no neighbour's label
// is smaller in any of its views, so the superstep kernel and the hub gather skip its gathers.
constexpr int kMinShards = 16;
constexpr int kMinWords = kMinShards * 64;
// dense_div | kDense1: superstep 1 (K2) is dense too (it writes no frontier flags, step 2 visits
// every member; kernels.hip dense_rule).  RGPU_DENSE1 (default on).
constexpr int kDense1 = 1 << 30;
constexpr int kLaneSteps = 128;                          // kMaxSteps (rgpu.cpp)
constexpr int kLaneChgWords = kLaneSteps * kLaneShards;
void launch_lane_fold(hipStream_t s, unsigned long long* lanechg, unsigned long long* lanefold);

// K1.  planar = false: one mask word per entity, view bit w*KS + k.  planar = true (W <=
// kMaxPlanes): one word per window w at out[w*stride + i], bit k = hop of the block.
constexpr int kMaxPlanes = 8;
void launch_batch_clear(hipStream_t s, const BatchClear& clr);
// fc (bp.carry != 0): per-entity floor carry, int32 index relative to the entity's first point (-1 none)
void launch_vertex_mask(hipStream_t s, const DevGraph& g, const BatchParams& bp, uint64_t* vm,
                        int64_t vstride, bool planar, const BatchClear& clr, int32_t* fc = nullptr);
// ecnt (profile runs, else null): alive edges per view (|E_w| of SURVEY §8(d)) added into
// ecnt[(h0 + k) * W + w] for hop k of the block (first hop h0 of the run) and window w
// vm_ends (CC runs, one partition): the vertex masks of the same block (plane stride vstride);
// each edge word is ANDed with both endpoints' words, so that K2 keeps a slot on em alone
void launch_edge_mask(hipStream_t s, const DevGraph& g, const BatchParams& bp, uint64_t* em, bool planar,
                      unsigned long long* ecnt = nullptr, int64_t h0 = 0, const uint64_t* vm_ends = nullptr,
                      int64_t vstride = 0, bool skip_simple = false, int32_t* fc = nullptr);
// tcut: no view of the batch can keep an edge whose last add is older (time-ordered slots)
// ebp (time-ordered slots only; else null): the batch's hops and edge windows, non-planar bit layout
// (view bit w*KS + k): K2 computes the window bits of simple slots inline (kernels.hip simple_bits)
// and reads em only for the others (K1 then runs with skip_simple)
// edges whose bits K2 computes itself (kernels.hip edge_simple), added into *out
void launch_count_simple(hipStream_t s, const DevGraph& g, unsigned long long* out);
// bit e of out ((ne + 63) / 64 words): edge e is simple (edge_simple) — DevGraph.esimple
void launch_edge_simple_bits(hipStream_t s, const DevGraph& g, uint64_t* out);
// the non-simple edges (zero bits of es, e < ne) as an ascending id list: returns the count; out null
// = count only.  Synchronous (one device scan; temporaries freed before it returns)
int64_t build_nonsimple_list(const DevGraph& g, const uint64_t* es, int32_t* out);
void launch_cc_slots(hipStream_t s, const DevGraph& g, int64_t tcut, const uint64_t* vm, const uint64_t* em,
                     int32_t* cnt, int32_t* snbr, uint64_t* smask, uint64_t* vadj, int32_t* lab0,
                     int32_t* lab1, uint64_t* chg1, uint8_t* act2, int32_t* stepflag,
                     int32_t* hostflag, unsigned long long* work, const HeavyBuf& hb,
                     unsigned long long* lanechg, int32_t* uw0 = nullptr, int32_t* uw1 = nullptr,
                     uint64_t* cb1 = nullptr, bool ends = false, int32_t* ccount = nullptr,
                     const BatchParams* ebp = nullptr, int dense_div = 0, int32_t* mneg = nullptr,
                     const uint8_t* gpeer = nullptr, uint8_t* pmask = nullptr, const KernOpts& ko = KernOpts());
// (partitioned: gpeer[g - n_own] = the partition owning ghost g; pmask[v] = the peers owning a ghost
// neighbour of owned v across a kept slot of the batch, every peer for a hub)
// heavy-vertex phases (g.n_seg > 0): K2 segment compaction + superstep-1 partial minima
// (before launch_cc_slots); per superstep, segment gathers (before launch_cc_step) and
// next-frontier marking of the heavy vertices' neighbours (after it; step 1: after slots)
// work (profile runs, else null): the hub kernels' work counters (kernels.hip heavy_work)
void launch_heavy_slots(hipStream_t s, const DevGraph& g, int64_t tcut, const uint64_t* vm, const uint64_t* em,
                        int32_t* snbr, uint64_t* smask, const HeavyBuf& hb, bool ends = false,
                        unsigned long long* work = nullptr, const BatchParams* ebp = nullptr,
                        const KernOpts& ko = KernOpts());
// (kHubDemote) after K2: owned hubs keeping <= 64 slots in one segment take the light path for the batch
void launch_hub_demote(hipStream_t s, const DevGraph& g, const HeavyBuf& hb, int32_t* cnt, int32_t* snbr,
                       uint64_t* smask, const uint64_t* chg1, uint8_t* act2, bool dense1);
void launch_heavy_gather(hipStream_t s, const DevGraph& g, const int32_t* snbr, const uint64_t* smask,
                         const int32_t* lab_cur, const uint64_t* chg_prev, const uint8_t* act_cur,
                         const int32_t* stepflag, int step, const HeavyBuf& hb, const int32_t* uw_cur = nullptr,
                         const uint64_t* cb_prev = nullptr, const int32_t* ccount = nullptr, int dense_div = 0,
                         unsigned long long* work = nullptr, const uint64_t* vm = nullptr,
                         const int32_t* mneg = nullptr, const KernOpts& ko = KernOpts());
// vm/em (partitioned mode): heavy ghosts (ranks >= n_own) have no compacted slots; their kept
// slots are recomputed from the static adjacency (em & vm[nb] & vm[v]) while marking
void launch_heavy_mark(hipStream_t s, const DevGraph& g, const int32_t* snbr, const uint64_t* smask,
                       const uint64_t* chg_now, uint8_t* act_next, const int32_t* stepflag, int step,
                       const HeavyBuf& hb, const uint8_t* act_cur, const uint64_t* vm = nullptr,
                       const uint64_t* em = nullptr, int64_t tcut = INT64_MIN, const int32_t* ccount = nullptr,
                       int dense_div = 0, unsigned long long* work = nullptr, const int32_t* uw_ghost = nullptr,
                       const KernOpts& ko = KernOpts());
// uniform label words (kernels.hip, kMixed): rows of the uniform vertices written into lab
void launch_uw_rows(hipStream_t s, int64_t nv, const uint64_t* vm, const int32_t* uw, int32_t* lab);
// component counts from the uniform words (one partition): counts = zeroed [nv][64] rows, kept
// zero by launch_cc_roots, which also folds iso and writes the summary fields into stats
void launch_cc_count(hipStream_t s, int64_t nv, int nviews, const uint64_t* vm, const uint64_t* vadj,
                     const int32_t* uw, const int32_t* lab, int32_t* counts, unsigned int* iso);
// grank: the label of each rank (null: the rank itself); counts rows are indexed by label, or
// (rows_by_rank, partitioned: labels are ids) by the rank
void launch_cc_roots(hipStream_t s, int64_t nv, int nviews, const uint64_t* vm, const uint64_t* vadj,
                     const int32_t* uw, const int32_t* lab, int32_t* counts, unsigned long long* stats,
                     unsigned int* iso, bool scan_all, const int32_t* grank = nullptr, bool rows_by_rank = false);
// RGPU_CHECK (check.hip): structural checks, violations counted into bad[16]
void launch_check_graph(hipStream_t s, const DevGraph& g, int64_t n_ekey, int64_t n_vkey, unsigned long long* bad);
void launch_check_labels(hipStream_t s, int64_t nv, const uint64_t* vm, const int32_t* uw, const int32_t* lab,
                         unsigned long long* bad, const int32_t* grank = nullptr);
void launch_check_slots(hipStream_t s, int64_t nv, int64_t nv_all, const int64_t* adj_off, const uint64_t* vm, const int32_t* cnt,
                        const int32_t* snbr, const int32_t* uw0, const int32_t* uw1, unsigned long long* bad,
                        const int32_t* grank = nullptr);
// Changed bits (with uniform words and heavy vertices): one bit per local rank, set when the
// vertex's label changed in a step; three bitmaps rotate (step r writes r % 3, the hub gather of
// step r+1 reads it, step r+2 clears it).  The hub gather probes a neighbour's bit (L2-resident:
// 2.5 MB for 20M vertices) before it touches the neighbour's words.  All null: off.
struct ChgBits {
  const uint64_t* prev = nullptr;
  uint64_t* next = nullptr;
  uint64_t* clear = nullptr;
  int64_t words = 0;  // words cleared (every local rank, ghosts included)
};
void launch_cc_step(hipStream_t s, int step, const DevGraph& g, const uint64_t* vm,
                    const int32_t* cnt, const int32_t* snbr, const uint64_t* smask,
                    const int32_t* lab_cur, int32_t* lab_next, const uint64_t* chg_prev,
                    uint64_t* chg_next, const uint8_t* act_cur, uint8_t* act_next,
                    uint8_t* act_clear, int32_t* stepflag, int32_t* hostflag,
                    unsigned long long* work, unsigned long long* lanechg,
                    int32_t* hbest = nullptr, const int32_t* uw_cur = nullptr, int32_t* uw_next = nullptr,
                    const ChgBits& cb = ChgBits(), int32_t* ccount = nullptr, int dense_div = 0,
                    const int32_t* mneg = nullptr, bool long_views = false, const KernOpts& ko = KernOpts());
constexpr int kIsoWords = 64 * 64;  // isolated-member counts [64 shards][64 views]
// DegreeRanking top-20 per view (kernels.hip k_deg_top_merge): key = in-degree << 32 | ~label
constexpr int kTop = 20;
struct DegTop {
  uint64_t* cand_key = nullptr;   // [deg_top_waves(nv)][64][kTop] per-wave candidates
  int32_t* cand_pos = nullptr;
  unsigned long long* key = nullptr;  // [64][kTop] result (0: none)
  int32_t* pos = nullptr;             // its local rank
  int32_t* out = nullptr;             // its out-degree
};
int64_t deg_top_waves(int64_t nv);
// top: also the top-20 by in-degree of every view (null: totals and rows only)
void launch_degree(hipStream_t s, const DevGraph& g, const uint64_t* vm, const uint64_t* em,
                   int32_t* outdeg, int32_t* indeg, unsigned long long* stats, const DegTop* top = nullptr);
void launch_pr_slots(hipStream_t s, const DevGraph& g, const uint64_t* vm, const uint64_t* em,
                     const int32_t* outdeg, int32_t* cnt, int32_t* snbr, uint64_t* smask,
                     double* pr, double* contrib);
// hacc: [n_heavy][64] fp64 accumulators of the heavy vertices (zero between uses), or null
void launch_pr_step(hipStream_t s, const DevGraph& g, const uint64_t* vm, const uint64_t* em,
                    const int32_t* outdeg, const int32_t* cnt, const int32_t* snbr, const uint64_t* smask,
                    const double* contrib_cur, double* contrib_next, double* pr, double* hacc);

// Generic vertex programs (vp.hip; include/rgpu.h rgpu_vertex_program_t): direction 0 out / 1 in /
// 2 all, reduce 0 min / 1 max, init 0 own id / 1 init_value (seed_value at the seed), senders 0 all
// members / 1 the seed; seed_rank = the seed's local rank (-1: none)
struct VpParams {
  int32_t dir = 2, reduce = 0, init = 0, senders = 0;
  int64_t init_value = 0, seed_rank = -1, seed_value = 0, step_add = 0;
  // float programs (rgpu_set_vertex_program_f, ABI 10): VertexMessageFloat summed.  State rows
  // hold the double bit pattern of a float32 value; a sender sends state (/ max(deg, 1) with
  // per_degree: deg = its message targets alive in the view, rows deg[v][64]); a member holding
  // messages takes (float)(f_bias + f_mult * sum) (the sum in double) and sends again
  int32_t fsum = 0, per_degree = 0;
  double f_init = 0, f_seed = 0, f_bias = 0, f_mult = 1;
};
void launch_vp_setup(hipStream_t s, const DevGraph& g, const VpParams& p, const int64_t* vid, const uint64_t* vm,
                     const uint64_t* em, int32_t* cnt, int32_t* snbr, uint64_t* smask, int64_t* st0, uint64_t* chg0,
                     int32_t* deg = nullptr);
void launch_vp_go(hipStream_t s, int32_t* stepflag);
// partitioned vertex programs (rgpu.cpp run_partitioned_vp): boundary records of kVpRec words
constexpr int kVpRec = 65;  // 64 state words + the change word
void launch_vp_xgather(hipStream_t s, int64_t n, const int32_t* xv, const int64_t* st, const uint64_t* chg,
                       int64_t* buf);
void launch_vp_xscatter(hipStream_t s, int64_t n, const int32_t* xv, const int64_t* buf, int64_t* st, uint64_t* chg);
void launch_vp_xgather_deg(hipStream_t s, int64_t n, const int32_t* xv, const int32_t* deg, int32_t* buf);
void launch_vp_xscatter_deg(hipStream_t s, int64_t n, const int32_t* xv, const int32_t* buf, int32_t* deg);
void launch_vp_lanes(hipStream_t s, const unsigned long long* lanechg, int step, unsigned long long* w);
void launch_vp_vote(hipStream_t s, const unsigned long long* w, int step, int32_t* stepflag,
                    unsigned long long* lanechg);
void launch_vp_step(hipStream_t s, int step, const DevGraph& g, const VpParams& p, const uint64_t* vm,
                    const int32_t* cnt, const int32_t* snbr, const uint64_t* smask, const int64_t* st_cur,
                    int64_t* st_next, const uint64_t* chg_prev, uint64_t* chg_next, int32_t* stepflag,
                    int32_t* hostflag, unsigned long long* lanechg, const int32_t* deg = nullptr);

// BinaryDefusion (diffusion.hip): per-lane coin salts of a batch (view j -> (hop, window))
struct DiffSalts {
  uint64_t s[64];
};
// steprow may be null (no per-vertex rows: the run does not retain); stats[view] counts infected
void launch_diff_setup(hipStream_t s, const DevGraph& g, const uint64_t* vm, int64_t seed, uint64_t* inf,
                       uint64_t* front0, uint8_t* act1, uint8_t* steprow, unsigned long long* stats);
void launch_diff_step(hipStream_t s, int step, const DevGraph& g, const int64_t* vid, const uint64_t* vm,
                      const uint64_t* em, uint64_t* inf, const uint64_t* front_in, uint64_t* front_out,
                      const uint8_t* act_cur, uint8_t* act_next, uint8_t* act_clear, uint8_t* steprow,
                      const DiffSalts& salts, int coin, int32_t* stepflag, int32_t* hostflag,
                      unsigned long long* stats);

// ---- vertex-partitioned mode (xchg.hip; host: rgpu.cpp).  Up to kMaxParts partitions.
constexpr int kMaxParts = 8;
static_assert(kMaxParts <= 8, "a peer mask (K2 pmask, one byte per vertex) holds one bit per partition");
// a label record: the new label `val` of boundary entry `e` (index in the sender's list for
// the receiver) in the views `mask`
struct XRec {
  int32_t e;
  int32_t val;
  uint64_t mask;
};
// per-peer layout of a record buffer (by value in kernel arguments)
struct XPeers {
  int np = 1, me = 0;
  int64_t base[kMaxParts] = {};     // first record of peer q's region
  int64_t cap[kMaxParts] = {};      // records that fit in it (send side)
  int64_t pre[kMaxParts + 1] = {};  // receive side: prefix of the records received per peer
  int64_t xoff[kMaxParts + 1] = {}; // first entry of peer q in the send / receive list
};
void launch_xvm_pack(hipStream_t s, int64_t nx, const int32_t* xv, const int32_t* xq, const int64_t* xoff, int planes,
                     const uint64_t* vm, int64_t vstride, uint64_t* out);
void launch_xvm_unpack(hipStream_t s, int64_t nx, const int32_t* xv, const int32_t* xq, const int64_t* xoff,
                       int planes, const uint64_t* in, uint64_t* vm, int64_t vstride);
// The send plan by boundary vertex (build_xsend, from the (peer, vertex) send lists): the owned
// boundary vertices ascending (boundary index b), each owned rank's b (-1: not a boundary vertex),
// and each send entry's b.  Label records name a vertex by b (one broadcast list for every peer).
struct XSend {
  int64_t nb = 0;
  const int32_t* v = nullptr;     // [nb] owned rank of boundary vertex b
  const int32_t* bidx = nullptr;  // [n_own] b of owned rank v, or -1
  const int32_t* eb = nullptr;    // [nx] b of send entry e
};
XSend build_xsend(hipStream_t s, int64_t n_own, int64_t nx, const int32_t* xv, std::vector<void*>& T,
                  std::vector<void*>& L);
// receive tables: ghost rank of (peer q, q's boundary index b) = tab[toff[q] + b], -1 if q's vertex b
// has no ghost here
struct XTab {
  int32_t* tab = nullptr;
  int64_t toff[kMaxParts + 1] = {};
};
// tmp[i]: the sender's boundary index of receive entry i (xr_v[i], from peer xr_q[i])
void launch_xtab_fill(hipStream_t s, int64_t n, const int32_t* xr_v, const int32_t* xr_q, const int32_t* tmp,
                      const XTab& T, unsigned long long* err);
// After superstep `step`: this partition's broadcast label records (xchg.hip: U records into su, at
// most nb; M records into sm, cnt[1] counts past mcap so the host can grow and pack again)
// The pack of a superstep's label records (xchg.hip k_xbc_pack): per 64-owned-rank chunk (one word
// of cb_now, the step's changed bits) a count pass (ccnt[q * nch + c] = U << 32 | M records for
// peer q), a device scan into coff (ccnt[np * nch] must be 0), then the write pass into peer q's
// regions su + q * ucap, sm + q * mcap.  write_only: coff is current (a repack into larger M
// regions).  ccnt / coff hold nch * np + 1 words, scan_tmp xbc_scan_bytes(n_own, np).
size_t xbc_scan_bytes(int64_t n_own, int np);

// counts words (4 per peer): U records, M records (coff / nch: the pack's scan), the halting vote
void launch_xbc_counts(hipStream_t s, int np, int me, const unsigned long long* coff, int64_t nch,
                       const int32_t* stepflag, int64_t* xa);
// the per-view minimum member labels (mneg) folded into 64 words w / w stored back into shard 0
// (partitioned final labels: the host all-reduces w with max in between)
void launch_min_fold(hipStream_t s, const int32_t* mneg, unsigned long long* w);
void launch_min_store(hipStream_t s, const unsigned long long* w, int32_t* mneg);
// component-count records (2 words per peer); scnt reset
void launch_xcounts(hipStream_t s, int np, int me, unsigned long long* scnt, int64_t* xa);
// a received broadcast: U and M receive regions per peer, with the records received (pre), the
// tables, the ghost range and the out-of-plan record counter
struct XBcIn {
  XPeers U, M;
  const unsigned long long* ru = nullptr;
  const XRec* rm = nullptr;
  XTab T;
  int64_t n_own = 0, nv = 0;
  unsigned long long* err = nullptr;
};
// (clr: the ghosts of step r-2's records cleared by the count pass, k_xbc_clear folded in)
void launch_xbc_pack(hipStream_t s, int64_t n_own, int np, const XSend& X, const uint64_t* cb_now,
                     const uint64_t* chg_now, const uint64_t* vadj, const int32_t* lab, const int32_t* uw,
                     const uint8_t* pmask, unsigned long long* su, int64_t ucap, XRec* sm, int64_t mcap,
                     unsigned long long* ccnt, unsigned long long* coff, void* scan_tmp, size_t scan_bytes,
                     bool write_only, const struct XBcIn* clr = nullptr, uint64_t* cchg = nullptr,
                     int32_t* cuw = nullptr);
void launch_xbc_clear(hipStream_t s, const XBcIn& I, uint64_t* chg, int32_t* uw);
// a superstep's received records applied to the ghost words / rows / change words (cb: changed
// bits) and the ghosts' owned neighbours marked in act_next.  tcut / ebp: the batch's slot cut and
// (inline edge bits; null: em for every slot) its edge windows; ccount / dense_div / step: nothing
// is marked when superstep `step` is dense
void launch_xbc_apply(hipStream_t s, const XBcIn& I, int32_t* lab, uint64_t* chg, int32_t* uw, uint64_t* cb,
                      const DevGraph& g, const uint64_t* vm, const uint64_t* em, uint8_t* act_next, int64_t tcut,
                      const BatchParams* ebp, const int32_t* ccount, int dense_div, int step,
                      const int32_t* gcut = nullptr);
// per batch, ghost g: its time-ordered static slots at or after the cut (gcut[g], g >= n_own)
void launch_ghost_cut(hipStream_t s, const DevGraph& g, int64_t tcut, int32_t* gcut);
// owned id -> owned rank: ids ascend with rank; bucket b = id >> shift covers ranks
// [boff[b], boff[b+1]) (about one id per bucket)
// Work units of the record pack and the partitioned counts (xchg.hip): chunks of 64 consecutive owned
// ranks, except the first kSplitChunks chunks, each split kSplitWays ways by mixed member.  (Tried on
// N = 1's k_cc_count / k_cc_roots too: no change there, 6.3 / 4.1 vs 6.7 / 4.2 ms per query.)  Owned
// ranks are in activity order (packer.cpp locality_order), so those chunks hold the partition's
// hubs, which are mostly mixed: one wave walking 64 hub rows in turn was the whole launch (0.8 ms
// of a year batch's count kernel, 0.3-0.4 ms of a record pack pass, profiles/r04).  Unit u < hs *
// kSplitWays: chunk u / kSplitWays, the mixed members whose index among the chunk's mixed members
// is u % kSplitWays (mod kSplitWays), and the uniform ones with sub-unit 0; after that one unit per
// chunk.
constexpr int kSplitChunks = 128, kSplitWays = 16;
__host__ __device__ inline int64_t xbc_units(int64_t n_own) {
  const int64_t nch = (n_own + 63) >> 6, hs = nch < kSplitChunks ? nch : kSplitChunks;
  return nch + hs * (kSplitWays - 1);
}
// unit -> (chunk, sub-unit; -1: the whole chunk)
__device__ __forceinline__ int64_t unit_chunk(int64_t un, int64_t nch, int& sub) {
  const int64_t hs = nch < kSplitChunks ? nch : kSplitChunks;
  if (un < hs * kSplitWays) {
    sub = (int)(un % kSplitWays);
    return un / kSplitWays;
  }
  sub = -1;
  return hs + (un - hs * kSplitWays);
}
// the members (lane mask) a sub-unit takes: every kSplitWays-th, from the sub-th (wave-uniform)
__device__ __forceinline__ uint64_t split_rows(uint64_t m, int sub) {
  if (sub < 0) return m;
  uint64_t r = 0;
  for (int k = 0; m; m &= m - 1, k++)
    if (k % kSplitWays == sub) r |= m & (~m + 1);
  return r;
}
struct OwnIdx {
  const int64_t* vid = nullptr;   // owned ids ascending
  const int32_t* boff = nullptr;  // bucket b = id >> shift: vid[boff[b] .. boff[b + 1])
  const int32_t* pos = nullptr;   // local rank of the k-th owned id (null: k itself)
  int shift = 0;
  int64_t n_own = 0;
  int64_t id_max = -1;            // the largest owned id (the buckets cover [0, id_max])
  unsigned long long* err = nullptr;  // lookups of a label owned here that found no owned vertex:
                                      // a bug upstream, counted and reported by the run (RGPU_EHIP)
};
// bucket shift of an OwnIdx: about one owned id per bucket over the ids' range [0, id_max] (not
// [0, 2^31): ids packed densely below 2^31 would otherwise put dozens of owned ids in a bucket, a
// serial walk of dependent loads per lookup)
inline int own_bucket_shift(int64_t n_own, int64_t id_max) {
  int lg = 0, bits = 0;
  while (((int64_t)1 << lg) < (n_own > 1 ? n_own : 1)) lg++;
  while (bits < 62 && (id_max >> bits) > 0) bits++;
  return bits > lg ? bits - lg : 0;
}
// component counts of the owned members (xchg.hip k_part_count): owned labels counted at their
// count rows (counts[local rank][view]), the others routed to the label owners (remote_only: the
// records again, into a larger buffer, without the local counts); gcnt[q] counts every record for
// peer q.  uw may be null (rows only).
void launch_part_count(hipStream_t s, bool remote_only, const XPeers& P, const OwnIdx& I, int nviews,
                       const uint64_t* vm, const uint64_t* vadj, const int32_t* uw, const int32_t* lab, int32_t* counts,
                       unsigned int* iso, unsigned long long* gcnt, XRec* hsbuf, const int32_t* mneg = nullptr,
                       unsigned int* fin_g = nullptr);
// members carrying the view's global minimum label (mneg) are counted into fin_g (64 shards x 64
// views) instead of records; fold them into w (zeroing the shards), all-reduce w, and the label's
// owner adds w at the label's count row
void launch_min_count_fold(hipStream_t s, unsigned int* fin_g, unsigned long long* w);
void launch_min_count_add(hipStream_t s, const unsigned long long* w, const int32_t* mneg, const OwnIdx& I, int np,
                          int me, int32_t* counts);
// records {label, count, views} received: counted at the owned label's rows
void launch_hist_recv(hipStream_t s, const XPeers& P, const XRec* rbuf, const OwnIdx& I, int32_t* counts);
// PageRank contribution rows of a list (partitioned PageRank): gather into / scatter out of a
// contiguous buffer
void launch_xgather_f64(hipStream_t s, int64_t n, const int32_t* xv, const double* rows, double* buf);
void launch_xscatter_f64(hipStream_t s, int64_t n, const int32_t* xv, const double* buf, double* rows);

// incremental seal (merge.hip): a sealed base graph and a host-packed delta (rgpu_internal.hpp
// Delta), all device pointers
struct MergeIn {
  int64_t nv_old = 0, nv2 = 0, ne_old = 0, nin_old = 0;
  const int32_t *esrc = nullptr, *edst = nullptr, *in_eid = nullptr;  // base
  const int64_t *eoff = nullptr, *ekey = nullptr, *voff = nullptr, *vkey = nullptr, *in_off = nullptr;
  const int32_t *old2new = nullptr, *new2old = nullptr;
  int64_t n_new = 0, nde = 0, ndd = 0, ndv = 0, nni = 0;
  const int64_t* nn_key = nullptr;
  const int32_t *nn_didx = nullptr, *de_base = nullptr;
  const int64_t *dkoff = nullptr, *dkey = nullptr;
  const int32_t* dd_rank = nullptr;
  const int64_t *dd_off = nullptr, *dd_t = nullptr;
  const int32_t* dv_rank = nullptr;
  const int64_t *dv_off = nullptr, *dv_key = nullptr;
  int64_t nvk_old = 0, ndvk = 0;      // base vertex keys, delta vertex keys
  int64_t* coll = nullptr;             // [ndvk + 1] collision flags -> prefix (scratch)
  int64_t* coll_tmp = nullptr;         // scan_tmp_words(ndvk) (scratch)
  const int64_t* ni_key = nullptr;
  const int32_t* ni_idx = nullptr;
};
void launch_edge_find(hipStream_t s, int64_t nq, const int32_t* qs, const int32_t* qd, const int64_t* out_off,
                      const int32_t* edst, int32_t* res);
void launch_merge_edges(hipStream_t s, const MergeIn& m, int32_t* esrc2, int32_t* edst2, int32_t* eo2n,
                        int32_t* mbase, int32_t* mdlt, int32_t* npos);
// off[0, n) counts -> off[0, n] exclusive offsets; tmp: scan_tmp_words(n) int64 words
void launch_scan_counts(hipStream_t s, int64_t n, int64_t* off, int64_t* tmp);
int64_t scan_tmp_words(int64_t n);
void launch_edge_hist(hipStream_t s, bool write, const MergeIn& m, int64_t ne2, const int32_t* mbase,
                      const int32_t* mdlt, const int32_t* esrc2, const int32_t* edst2, int64_t* cnt_off,
                      int64_t* ekey2);
void launch_vertex_hist(hipStream_t s, bool write, const MergeIn& m, int64_t* cnt_off, int64_t* vkey2);
void launch_merge_in(hipStream_t s, const MergeIn& m, const int32_t* eo2n, const int32_t* npos,
                     const int64_t* in_off2, int32_t* in_eid2);

// ---- live-ingest delta packer on the device (gdelta.hip; the host half packer.cpp pack_delta /
// finish_delta builds the same arrays, rgpu_internal.hpp Delta)
struct DevEvent {  // = rgpu::Event (rgpu_internal.hpp): the host's update records, uploaded as they are
  int64_t t, src, dst;
  uint8_t kind, pad[7];
};
struct DeltaDev {
  int64_t nd = 0, nv_old = 0, nv2 = 0;
  int64_t* vid2 = nullptr;                       // merged ids ascending (graph list)
  int32_t *old2new = nullptr, *new2old = nullptr;
  int64_t ndv = 0, ndvk = 0;                     // delta vertex points per rank, collapsed
  int32_t* dv_rank = nullptr;
  int64_t *dv_off = nullptr, *dv_key = nullptr;
  int64_t ndd = 0;                               // delta deaths per rank (times, last delta index)
  int32_t* dd_rank = nullptr;
  int64_t *dd_off = nullptr, *dd_t = nullptr, *dd_last = nullptr;
  int64_t nde = 0;                               // delta edges (distinct (s, d)), their base edge
  int32_t *de_s = nullptr, *de_d = nullptr, *de_base = nullptr;
  int64_t *de_koff = nullptr, *de_key = nullptr; // collapsed, tie-resolved own points
  int64_t n_new = 0, nni = 0;                    // new edges (s << 32 | d), their in-edge records
  int64_t* nn_key = nullptr;
  int32_t* nn_didx = nullptr;
  int64_t* ni_key = nullptr;
  int32_t* ni_idx = nullptr;
  int64_t *out_off = nullptr, *in_off = nullptr, *adj_off = nullptr;  // merged (graph list)
  int64_t *doff = nullptr, *dtime = nullptr;
  uint64_t* dbits = nullptr;
  int64_t n_in = 0, ndt = 0;
  std::vector<int32_t> heavy;                    // ranks with more than heavy_t static slots
  std::vector<int64_t> heavy_a0, heavy_deg;      // their first static slot and slot count
  int64_t n_own2 = 0;                            // owned ranks [0, n_own2) of the merged graph
  std::vector<int64_t> orph_id, orph_t;          // deaths of ids not kept here (partitioned mode)
};
// Partitioned mode (nparts 0: one partition).  Ids are the graph's rank-order keys: the id for
// an owned vertex, 2^31 | id for a ghost.  Orphans: deaths of ids not kept here (device arrays).
struct DeltaPart {
  int part = 0, nparts = 0;
  int64_t n_own_old = 0;
  const int64_t *orph_id = nullptr, *orph_t = nullptr;
  int64_t n_orph = 0;
};
// ev[0, n): the updates since the last seal; vid0: the base ids (device).  Device arrays go to
// T (temporaries) or L (the merged graph).  Returns "" or the first invalid update's message.
std::string gpu_pack_delta(hipStream_t s, const DevEvent* ev, int64_t n, const DevGraph& g0, const int64_t* vid0,
                           const DeltaPart& P, int64_t heavy_t, DeltaDev* out, std::vector<void*>& T,
                           std::vector<void*>& L);
void launch_scatter_i32(hipStream_t s, int64_t n, const int32_t* idx, const int32_t* val, int32_t* out);
// Partition metadata of a merged partitioned graph (keys: its rank-order keys, DeltaPart)
struct PartMeta {
  int32_t* grank = nullptr;                     // [nv] CC label = vertex id
  int32_t *xs_v = nullptr, *xs_q = nullptr, *xr_v = nullptr, *xr_q = nullptr;  // exchange plan
  int64_t *xs_off_d = nullptr, *xr_off_d = nullptr;
  std::vector<int64_t> xs_off, xr_off;
  int64_t nxs = 0, nxr = 0;
  int64_t* own_vid = nullptr;                   // owned ids ascending
  int32_t* own_boff = nullptr;                  // their buckets (id >> shift, own_bucket_shift)
  int shift = 0;
  int64_t id_max = -1;
};
std::string gpu_part_meta(hipStream_t s, const int64_t* keys, int64_t nv, int64_t n_own, const int32_t* esrc,
                          const int32_t* edst, int64_t ne, int nparts, PartMeta* out, std::vector<void*>& T,
                          std::vector<void*>& L);

}  // namespace rgpu
