// rgpu.cpp — C ABI (include/rgpu.h) and the batch scheduler that drives the kernels.
//
// One rgpu_ctx = one Partition Manager's reader (S/core/components/PartitionManager/
// Reader.scala:42-53) bound to one GPU.  rgpu_run_view_batch replaces the whole
// Setup -> NextStep* -> Finish conversation that AnalysisTask (S/core/analysis/Tasks/
// AnalysisTask.scala:162-283) drives through ten ReaderWorkers, for every hop of a Range
// job (RangeAnalysisTask.scala:18-35) and every window of the batch at once.
//
// Scheduling: hops are grouped into batches of K = floor(64/W) hops (64 views).  Two
// batch slots, each with its own HIP stream and buffers, are kept in flight: while the
// host inspects one slot's superstep counters (the halting vote), the other slot's
// kernels keep the GPU busy.  Supersteps are enqueued in chunks; a step whose
// predecessor changed nothing exits at once (device-side halting), so over-enqueueing
// costs only an empty launch.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <climits>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "exchange.hpp"
#include "kernels.hpp"
#include "rgpu_internal.hpp"
#include "xregions.hpp"

using namespace rgpu;

namespace {

struct HipFail {
  std::string msg;
  int code = 0;  // 0: RGPU_EHIP
};
#define HIPCHK(x)                                                                        \
  do {                                                                                   \
    hipError_t e_ = (x);                                                                 \
    if (e_ != hipSuccess) throw HipFail{std::string(#x) + ": " + hipGetErrorString(e_)}; \
  } while (0)

enum KernelId { KID_MASK = 0, KID_SLOTS = 1, KID_STEP = 2, KID_HIST = 3, KID_SUMMARY = 4,
                KID_PR = 5, KID_DEGREE = 6, KID_TAIL = 7, KID_HEAVY = 8, KID_DIFF = 9, KID_VP = 10, KID_EMASK = 11,
                KID_XCHG = 12, KID_XPACK = 13, KID_XUNPACK = 14, KID_XMARK = 15, KID_N = 16 };

constexpr int kMaxSteps = 128;
// stats words: 6 per-view fields + counters row | folded lane words [step] | lane-change shards
// [step][shard] (kernels.hpp).  The host copies the first kStatCopy words of a batch.
constexpr int kFoldOff = 7 * kViews;
constexpr int kLaneOff = kFoldOff + kLaneSteps;
constexpr int kStatCopy = kLaneOff;
constexpr int kStatWords = kLaneOff + kLaneChgWords;
constexpr int kWorkFields = 8;  // kernels.hip add_work
constexpr int kWorkWords = kMaxSteps * 64 * kWorkFields;
constexpr int64_t kPad = 64;  // tail padding of per-vertex / per-slot batch arrays
constexpr int kMaxSlots = 4;  // batches in flight (one HIP stream each; GPU_MAX_HW_QUEUES = 4)
// supersteps per host enqueue: the first chunk of a batch (capped by the step count its window's
// previous batch halted at), then the rest
constexpr int kChunk0 = 12, kChunk = 8;

struct Slot {
  // buffers allocated for this slot (slots are allocated lazily: a run uses min(slots, batches))
  bool a_cc = false, a_deg = false, a_pr = false, h_cc = false, h_pr = false, a_diff = false, a_vp = false;
  int64_t* vst[2] = {nullptr, nullptr};  // vertex program state rows [nv][64] (int64), Jacobi
  int32_t* vdeg = nullptr;                // float programs with per_degree: message targets [nv][64]
  hipStream_t stream = nullptr;
  hipEvent_t ev = nullptr;
  uint64_t *vm = nullptr, *em = nullptr;          // masks of the batch in flight
  bool iem = false;                               // the batch computes simple slots' edge bits inline
  BatchParams ebp{};                              // its hops and edge windows (view bit w*KS + k)
  uint64_t *vm_own = nullptr, *em_own = nullptr;  // this slot's own (hop-major batches)
  int32_t *cnt = nullptr, *snbr = nullptr;
  uint64_t* smask = nullptr;
  int32_t* lab[2] = {nullptr, nullptr};
  int32_t* uw[2] = {nullptr, nullptr};    // uniform label words of lab[0/1] (kernels.hip kMixed)
  uint64_t* cb[3] = {nullptr, nullptr, nullptr};  // changed bits, rotated like act (kernels.hpp ChgBits)
  int32_t* counts = nullptr;              // [nv][64] component counts at the root (zero between batches)
  uint64_t* chg[2] = {nullptr, nullptr};
  int32_t *stepcnt = nullptr, *hist = nullptr;   // stepcnt[r] = 1 iff superstep r changed a label
  int32_t* ccount = nullptr;                      // changed vertices per step (kernels.hpp kCountShards)
  uint8_t* act[3] = {nullptr, nullptr, nullptr};   // CC frontier flags (byte per vertex)
  uint64_t* vadj = nullptr;                         // OR of kept slot masks per vertex
  unsigned long long* work = nullptr;               // [step][64 shards][visited, slots, changed]
  unsigned long long* h_work = nullptr;
  unsigned long long* stats = nullptr;
  int32_t *outdeg = nullptr, *indeg = nullptr;
  DegTop top;                     // DegreeRanking top-20 per view (degree runs)
  unsigned long long* h_top = nullptr;  // pinned copy: [64][kTop] keys | [64][kTop] ranks, out-degrees (int32)
  double *pr = nullptr, *contrib[2] = {nullptr, nullptr};
  int32_t *pcnt = nullptr, *psnbr = nullptr;
  uint64_t* psmask = nullptr;
  int32_t* h_stepcnt = nullptr;   // host-mapped superstep flags, written by the kernels
  int32_t* d_hostflag = nullptr;  // device address of h_stepcnt
  unsigned int* iso = nullptr;    // isolated-member counts [64 shards][64 views] (k_cc_count)
  HeavyBuf hv;                    // heavy-vertex segment state (graphs with hubs)
  // BinaryDefusion (diffusion.hip): infected views, views infected last / this step, step rows
  uint64_t *dinf = nullptr, *dfront[2] = {nullptr, nullptr};
  uint8_t* dstep = nullptr;
  uint8_t* dact[3] = {nullptr, nullptr, nullptr};  // active (message-holding) flags, rotated
  DiffSalts salts;                // coin salt per lane of the batch in flight
  unsigned long long* h_stats = nullptr;
  // state of the batch in flight
  int batch = -1, phase = 0, r_launched = 0, r_final = 0, kb = 0;
  int64_t tcut = INT64_MIN;  // the batch's window cut for time-ordered slots (start_batch)
  bool long_views = false;  // every window of the batch >= long_ratio x its hop span (launch_cc_step)
  uint64_t evseq = 0;  // order in which slot events were recorded (wait on the oldest)
};

struct Retained {  // per batch, RGPU_RUN_RETAIN
  std::vector<uint64_t> vm;
  std::vector<int64_t> v64;   // vertex program: states
  std::vector<int32_t> a, b;  // CC: labels | degree: out, in
  std::vector<double> pr;
  std::vector<uint8_t> st;    // diffusion: infection superstep per (vertex, lane), 0xFF = none
};

// Vertex-partitioned mode (one partition per GPU; kernels: xchg.hip).
// Per batch slot: its own exchange channel, record buffers and counts staging.
struct XSlot {
  Exchange* x = nullptr;                  // this slot's channel (a fork of the ctx's)
  // broadcast label records (xchg.hip k_xbc_pack): one list for every peer
  unsigned long long* su = nullptr;       // U records to send, peer q's at q * su_cap: at most one per
                                          // boundary vertex (sized by the plan: grows only when a live
                                          // merge grows the plan)
  int64_t su_cap = 0, ru_cap = 0;
  XRec* sm = nullptr;                     // M records to send, peer q's at q * smcap (grown on demand)
  int64_t smcap = 0;
  uint8_t* pmask = nullptr;               // [nv] peers that read an owned vertex in the batch (K2)
  int32_t* gcut = nullptr;                // [nv] ghost g: its time-ordered slots at or after the batch's cut
  unsigned long long* ru[2] = {nullptr, nullptr};  // received U records per superstep parity, region q
                                                   // = peer q's boundary count (never grows)
  XRec* rm[2] = {nullptr, nullptr};       // received M records per parity
  int64_t rmcap[kMaxParts] = {};
  int64_t rucnt[2][kMaxParts] = {}, rmcnt[2][kMaxParts] = {};  // records received per parity (their
                                          // ghosts' words are cleared two supersteps later)
  unsigned long long *ccnt = nullptr, *coff = nullptr;  // the pack's per-chunk counts and their scan
  void* scan_tmp = nullptr;               // (xchg.hip launch_xbc_pack; sized with su)
  size_t scan_bytes = 0;
  unsigned long long* err = nullptr;      // received records outside the plan (xchg.hip bc_rec)
  unsigned long long* mfin = nullptr;     // [64] the batch's minimum member labels, all-reduced
  unsigned int* fin_g = nullptr;          // [64 x 64] members carrying them, per shard and view
  int64_t* xab = nullptr;                 // [8P] counts words: sent (xa) | received (xb)
  int64_t* h_xab = nullptr;               // pinned copy
  uint64_t *vms = nullptr, *vmr = nullptr;  // ghost membership words (planes x list)
  int vm_planes = 0;
  unsigned long long* htot = nullptr;     // [kMaxParts] component-count records per peer
  XRec *hsbuf = nullptr, *hrbuf = nullptr;            // component-count records {label, count, views}
  int64_t hscap[kMaxParts] = {}, hrcap[kMaxParts] = {};
  int r = 0;                              // superstep whose counts exchange is in flight
  int64_t hrcnt[kMaxParts] = {};
  double bytes[3] = {};                   // sent by this slot: membership words, records, counts
};
struct Part {
  Exchange* xchg = nullptr;                   // the ctx's channel (rgpu_exchange_init)
  int64_t nxs = 0, nxr = 0;
  std::vector<int64_t> xs_off, xr_off;        // host copies of the plan offsets
  int32_t *xs_v = nullptr, *xs_q = nullptr, *xr_v = nullptr, *xr_q = nullptr;
  int64_t *xs_off_d = nullptr, *xr_off_d = nullptr;
  OwnIdx own;                                 // owned id -> owned rank (label owner counting)
  XSend xsend;                                // the send plan by boundary vertex (record pack)
  XTab tab;                                   // receive tables of the broadcast records
  int64_t nbq[kMaxParts] = {};                // boundary vertices of every partition
  bool tab_ready = false;
  bool no_deaths = false;                     // no partition's graph holds a vertex death (ensure_tab)
  bool all_tslots = false;                    // every partition has time-ordered slots (ensure_tab)
  uint8_t* gpeer = nullptr;                   // [nv - n_own] the partition owning ghost g (getPartition)
  double *sbuf_f = nullptr, *rbuf_f = nullptr;  // PR contribution rows
  bool pr_ready = false;
  XSlot xs[4];                                // per batch slot (kMaxSlots)
  double bytes_sent = 0;
};

// Window-major batches (one window per batch, 64 hops): K1 runs once per 64-hop block for
// every window, into a mask set shared by the block's W batches (on whichever slots run them).
constexpr int kMaskSets = 2;
struct MaskSet {
  uint64_t *vm = nullptr, *em = nullptr;  // plane w: vm[w*(nv+kPad) + v], em[w*ne + e]
  int planes = 0;
  hipEvent_t k1 = nullptr;                // K1 of the current block done
  hipEvent_t done[kMaxPlanes] = {};       // batch (block, w) has stopped reading the set
  int pending = 0;                        // batches of the current block not yet finished
};

struct Timed {
  int kid;
  int slot;
  int batch, step;
  hipEvent_t a, b;
  double bytes;
};

// A merged graph built beside the resident one (seal_delta), waiting to replace it (apply_merged).
struct Merged {
  bool valid = false, dev = true;
  DevGraph g;
  std::vector<void*> L;                   // its device allocations
  int64_t* vid2 = nullptr;                // device packer: its ids
  int64_t ndt = -1, nd = 0, ne_owned = 0, nvk = 0, nek = 0, nv2 = 0;
  PartMeta PM;
  std::vector<int64_t> orph_id, orph_t;   // partitioned: deaths of ids not kept
  std::vector<int64_t> hvid, hdoff, hdtime, hout_off, hin_off;  // host packer: host arrays
};

}  // namespace

struct rgpu_ctx {
  // Locks.  mu: the resident graph and every run / result call (10 ReaderWorkers share a ctx).
  // ingest_mu: the update log (rgpu_ingest, the watermark), so that ingestion goes on while a run
  // holds mu (IngestionWorker keeps applying updates while LiveAnalysisTask runs,
  // IngestionWorker.scala:31-61).  seal_mu: one seal at a time; a live merge builds the merged
  // graph holding only seal_mu (runs on the resident graph go on) and takes mu to swap it in.
  std::mutex mu, ingest_mu, seal_mu;
  int part = 0, nparts = 1, device = 0;
  bool partitioned = false;  // nparts > 1, or RGPU_PARTITIONED=1 (the partitioned path with P = 1)
  std::string err;
  std::vector<Event> events;            // the update log from absolute index ev_base on
  size_t ev_base = 0;                   // updates dropped from the front of the log (sealed, live contexts)
  int64_t newest = -1;
  bool sealed = false;                  // a graph is resident (a seal has succeeded)
  size_t n_sealed = 0;                  // updates [0, n_sealed) (absolute) are in the resident graph
  bool delta_on = true;                 // RGPU_DELTA: merge later updates into it (else re-pack)
  bool delta_host = false;              // RGPU_DELTA=2: the host delta packer (A/B; default the device one)
  int64_t* g_vid = nullptr;             // device delta packer: the resident graph's ids (graph list)
  bool vid_stale = false;               // pk.vid lags g_vid (downloaded when results name ids)
  int64_t n_dtime = -1;                 // device delta packer: death times (pk.dtime is not kept)
  std::vector<int64_t> orph_id, orph_t; // partitioned: deaths of ids not kept here (DeltaPart)
  int vertex_order = RGPU_ORDER_LOCALITY;  // rgpu_set_vertex_order: local rank order of a full seal
  Packed pk;
  DevGraph g;
  Merged pending;                       // a merged graph that replaces g before the next run / seal
  std::vector<void*> graph_allocs;
  // batch-slot and mask-set buffers, sized for cap_* >= the graph (a live-ingest merge that
  // still fits keeps them: reallocating tens of GB per merge would dominate the tick)
  std::vector<void*> slot_allocs;
  int64_t cap_nv = 0, cap_ne = 0, cap_nin = 0;
  int64_t cap_nown = 0;                 // count rows (partitioned: owned ranks only, else every rank)
  Slot slot[kMaxSlots];
  int nslots = 3;                       // batches in flight (2 / 4 measured slower on C4)
  bool prof_lean = false;               // RGPU_PROF_LEAN (work_buf)
  int inject_fail = 0;                  // RGPU_INJECT_FAIL=n (tests): the n-th batch start of a run throws
  bool inject_rec = false;              // RGPU_INJECT_FAIL=rec (tests): corrupt one received label record
  bool inject_cnt = false;              // RGPU_INJECT_FAIL=cnt (tests): one received count record names a
                                        // label routed here that no owned vertex holds
  int dense = -1;                       // RGPU_DENSE: dense-step divisor (kernels.hip dense_rule; -1 by size)
  bool check = false;                   // RGPU_CHECK: structural checks after seal and K2 (check.hip)
  std::string trace_path;               // RGPU_TRACE: per-launch / per-step CSV (profile runs)
  struct StepRec { int batch, step; unsigned long long pv, ps; int changed; unsigned long long pg; };
  std::vector<StepRec> steprec;
  bool wmajor = true;                   // RGPU_WMAJOR: window-major batches when 2 <= W <= kMaxPlanes
  bool hostprof = false;                // RGPU_HOSTPROF: print host-side scheduling times
  int iv_max = 32;                      // RGPU_IVMAX: K1 interval form up to this many points (< 0 off)
  int heavy_t = 2048;                   // static slots above which a vertex is split (hub_threshold)
  int heavy_env = -1;                   // RGPU_HEAVY (0: off), or -1: hub_threshold's rule
  MaskSet mset[kMaskSets];
  int nsets = kMaskSets;                // mask sets in rotation this run (one with one batch slot)
  // K1 floor carry across a run's hop blocks (BatchParams::carry; RGPU_K1_CARRY=0 turns it off):
  // per-entity floor index at the last K1'd block's last hop, that hop, and an event after that
  // K1 (the next block's K1, on another slot's stream, waits for it)
  int32_t *k1c_v = nullptr, *k1c_e = nullptr;
  hipEvent_t k1_ev = nullptr;
  int64_t k1_last = INT64_MIN;          // INT64_MIN: no carry to read
  bool k1_ev_live = false;              // k1_ev recorded this run: a carry K1 (read or write) waits on it
  bool k1_carry = true;
  bool vp_run_fsum = false;             // the last vertex-program run ran a float program
  KernOpts ko;                          // kernel options of the run (RGPU_STEP_OPTS / _HUB_PRO / _LONG_STEPS)
  // RGPU_LONG_RATIO (read per run; default 4, < 0: never): a batch whose every window is at least
  // this many times its hop span runs the long-window superstep form (Slot::long_views)
  int long_ratio = 4;
  int grp_last[kMaxPlanes] = {};        // supersteps of the last batch of each window group
  // last run: views (hop, win) -> batch (hop/K)*G + win/gsize, lane (win%gsize)*K + hop%K
  int algo = -1, K = 0, W = 0, G = 1, gsize = 1;
  size_t n_hops = 0;
  std::vector<rgpu_cc_summary_t> cc;
  int64_t n_simple = -1;                // simple edges (kernels.hip edge_simple; the K1 edge byte model)
  std::vector<int32_t> vlast;           // per view: last superstep in which one of its labels changed
  unsigned long long* d_ecnt = nullptr; // profile runs: alive edges per view (K1 edge masks)
  std::vector<int64_t> deg;  // [view][3]
  struct TopEnt { int64_t id; int32_t out, in; };
  std::vector<TopEnt> degtop;  // [view][kTop] (id -1: none)
  std::vector<int64_t> dcount, dsteps;  // diffusion: infected vertices, supersteps per view
  VpParams vp;                          // rgpu_set_vertex_program
  int64_t vp_seed_id = -1;
  bool vp_set = false;
  std::vector<int64_t> vpsteps;         // vertex program: supersteps per hop (as CC)
  int64_t diff_seed = 31;               // BinaryDefusion.infectedNode (BinaryDefusion.scala:10)
  uint64_t diff_coin_seed = 0;
  int diff_coin = 1;
  int64_t diff_seed_rank = -1;          // of the run in progress
  int64_t* d_vid = nullptr;             // vertex ids on the device (diffusion coins hash ids)
  std::vector<Retained> kept;
  bool retained = false;
  rgpu_stats_t st{};
  // profiling
  bool profile = false;
  std::vector<hipEvent_t> evpool;
  size_t evused = 0;
  uint64_t evcounter = 0;
  std::vector<Timed> timed;
  Part pt;
};

namespace {

// RGPU_POISON=1 (tests): every fresh device buffer starts as 0xa5 bytes, so a read of memory
// no kernel wrote shows up deterministically instead of depending on what the allocator reuses
int g_poison = -1;
template <class T>
T* dalloc(std::vector<void*>& list, size_t n) {
  void* p = nullptr;
  HIPCHK(hipMalloc(&p, sizeof(T) * (n ? n : 1)));
  list.push_back(p);
  if (g_poison < 0) {
    const char* e = std::getenv("RGPU_POISON");
    g_poison = e && std::atoi(e) != 0;
  }
  if (g_poison) {  // (synchronised: the batch streams are non-blocking, a null-stream memset does not order them)
    HIPCHK(hipMemset(p, 0xa5, sizeof(T) * (n ? n : 1)));
    HIPCHK(hipDeviceSynchronize());
  }
  return (T*)p;
}
template <class T>
T* dupload(std::vector<void*>& list, const std::vector<T>& h) {
  T* d = dalloc<T>(list, h.size());
  if (!h.empty()) HIPCHK(hipMemcpy(d, h.data(), sizeof(T) * h.size(), hipMemcpyHostToDevice));
  return d;
}

void release_slots(rgpu_ctx* c);
void free_part_slots(rgpu_ctx* c, bool keep_channels);
void free_graph(rgpu_ctx* c) {
  for (void* p : c->pending.L) (void)hipFree(p);  // (a parked merged graph)
  c->pending = Merged();
  for (void* p : c->graph_allocs) (void)hipFree(p);
  c->graph_allocs.clear();
  c->g_vid = nullptr;
  release_slots(c);
  c->g = DevGraph();
  free_part_slots(c, true);  // the channels (communicators) outlive a re-seal
  {
    Exchange* x = c->pt.xchg;
    XSlot xs[4];
    for (int i = 0; i < 4; i++) xs[i].x = c->pt.xs[i].x;
    c->pt = Part();
    c->pt.xchg = x;
    for (int i = 0; i < 4; i++) c->pt.xs[i].x = xs[i].x;
  }
}

void release_slots(rgpu_ctx* c) {
  for (void* p : c->slot_allocs) (void)hipFree(p);
  c->slot_allocs.clear();
  c->cap_nv = c->cap_ne = c->cap_nin = c->cap_nown = 0;
  c->d_vid = nullptr;
  for (Slot& s : c->slot) {
    if (s.h_stepcnt) (void)hipHostFree(s.h_stepcnt);
    if (s.h_stats) (void)hipHostFree(s.h_stats);
    if (s.h_work) (void)hipHostFree(s.h_work);
    if (s.h_top) (void)hipHostFree(s.h_top);
    if (s.ev) (void)hipEventDestroy(s.ev);
    if (s.stream) (void)hipStreamDestroy(s.stream);
    s = Slot();
  }
  for (MaskSet& m : c->mset) {
    if (m.k1) (void)hipEventDestroy(m.k1);
    for (hipEvent_t e : m.done)
      if (e) (void)hipEventDestroy(e);
    m = MaskSet();
  }
  c->k1c_v = c->k1c_e = nullptr;  // (in slot_allocs)
  if (c->k1_ev) (void)hipEventDestroy(c->k1_ev);
  c->k1_ev = nullptr;
  c->k1_last = INT64_MIN;
}

hipEvent_t take_event(rgpu_ctx* c) {
  if (c->evused == c->evpool.size()) {
    hipEvent_t e;
    HIPCHK(hipEventCreate(&e));
    c->evpool.push_back(e);
  }
  return c->evpool[c->evused++];
}

// Run `fn` (one kernel launch) on slot stream, bracketed by events in profile mode.
// evented = false: the caller brackets a group of launches itself (see launch_chunk).
// RGPU_CHECK: run a check launcher on `st`, wait, and fail with the violation counts
template <class F>
void run_check(hipStream_t st, const char* what, F launch) {
  unsigned long long* bad = nullptr;
  HIPCHK(hipMalloc(&bad, 16 * sizeof(unsigned long long)));
  unsigned long long h[16] = {};
  HIPCHK(hipMemsetAsync(bad, 0, sizeof(h), st));
  launch(bad);
  HIPCHK(hipMemcpyAsync(h, bad, sizeof(h), hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  (void)hipFree(bad);
  std::string msg;
  for (int i = 0; i < 16; i++)
    if (h[i]) msg += " bad[" + std::to_string(i) + "]=" + std::to_string(h[i]);
  if (!msg.empty()) throw HipFail{std::string("RGPU_CHECK ") + what + ":" + msg, RGPU_EHIP};
}


// The work-counter buffer of a profile run.  RGPU_PROF_LEAN=1: none, so the superstep and K2
// kernels run their lean instantiations (the ones timed runs use) under the profile events; a
// counting pass and a lean pass of the same query give bytes and times of the same launches.
unsigned long long* work_buf(const rgpu_ctx* c, const Slot& s) {
  return c->profile && !c->prof_lean ? s.work : nullptr;
}

// dense-step divisor (kernels.hip dense_rule; RGPU_DENSE, 0 = off); K2 is then dense too (kDense1:
// step 2 visited exactly as many vertices as step 1 in all 15 C4 batches).
// Default 4 on graphs of more than 2M vertices (C4: 529 -> 507 ms, `heavy` 103 -> 89 ms; 16:
// 536 ms); off below (C2: 127.5 -> 132.3 ms with it: a small graph's flags are cached anyway).
int dense_div(const rgpu_ctx* c) {
  const int d = c->dense >= 0 ? c->dense : (c->g.nv > ((int64_t)1 << 21) ? 4 : 0);
  return d > 0 ? (d | kDense1) : d;
}

// the batch's per-view minimum member labels (kernels.hpp kMinShards), behind the changed-vertex
// counts; one partition only (a partition's minimum is not the graph's)
// the batch's per-view minimum member labels (kernels.hip final_label), written by K2; partitioned,
// part_min_labels makes them global before superstep 2
int32_t* min_labels(const rgpu_ctx* c, const Slot& s) {
  (void)c;
  return s.ccount ? s.ccount + (size_t)kMaxSteps * kCountShards : nullptr;
}

// changed bits of superstep r (with uniform words; RGPU_CHGBITS=0 turns them off)
ChgBits chg_bits(const rgpu_ctx* c, const Slot& s, int r) {
  ChgBits b;
  if (!s.cb[0]) return b;
  // Written by the superstep kernels, read by the heavy gather only, and only when there are
  // heavy vertices.  The superstep kernel reading them measured slower on C4 (cc_step 263 ->
  // 301 ms serial; the bit probe then the words vs one change word) and on C2; the heavy
  // gather, which walks a hub's whole kept slot list every step, gained (119 -> 103 ms).
  // (partitioned: the record pack reads them too)
  if (c->g.n_seg == 0 && !c->partitioned) return b;
  b.prev = s.cb[(r + 2) % 3];
  b.next = s.cb[r % 3];
  b.clear = s.cb[(r + 1) % 3];
  b.words = (c->g.nv + 63) / 64 + 1;
  return b;
}

template <class F>
void timed_launch(rgpu_ctx* c, int si, int kid, double bytes, F fn, int step = 0, bool evented = true) {
  Slot& s = c->slot[si];
  if (c->profile && evented) {
    hipEvent_t a = take_event(c), b = take_event(c);
    HIPCHK(hipEventRecord(a, s.stream));
    fn();
    HIPCHK(hipEventRecord(b, s.stream));
    c->timed.push_back({kid, si, s.batch, step, a, b, bytes});
  } else {
    fn();
  }
  HIPCHK(hipGetLastError());
  c->st.kernel_launches[kid]++;
  c->st.kernel_bytes[kid] += bytes;
}

void ensure_masks(rgpu_ctx* c, int G, int nuse) {
  auto& L = c->slot_allocs;
  const int64_t nv = c->cap_nv, ne = c->cap_ne;
  if (c->k1_carry && !c->k1c_v) {
    c->k1c_v = dalloc<int32_t>(L, nv);
    c->k1c_e = dalloc<int32_t>(L, ne);
    HIPCHK(hipEventCreateWithFlags(&c->k1_ev, hipEventDisableTiming));
  }
  c->k1_last = INT64_MIN;  // (called once per run, before its first block)
  c->k1_ev_live = false;
  if (G == 1) {
    for (int i = 0; i < nuse; i++) {
      Slot& s = c->slot[i];
      if (!s.vm_own) {
        s.vm_own = dalloc<uint64_t>(L, nv + kPad);
        s.em_own = dalloc<uint64_t>(L, ne);
      }
    }
    return;
  }
  // one batch slot runs the blocks one after another: one mask set serves (a 1B loopback rehearsal of
  // eight partitions on one GPU needs the memory)
  c->nsets = nuse == 1 ? 1 : kMaskSets;
  for (int si = 0; si < c->nsets; si++) {
    MaskSet& m = c->mset[si];
    if (m.planes < G) {  // (a smaller earlier allocation stays in slot_allocs until re-seal)
      m.vm = dalloc<uint64_t>(L, (size_t)G * (nv + kPad));
      m.em = dalloc<uint64_t>(L, (size_t)G * ne);
      m.planes = G;
    }
    if (!m.k1) {
      HIPCHK(hipEventCreateWithFlags(&m.k1, hipEventDisableTiming));
      for (hipEvent_t& e : m.done) HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    }
    m.pending = 0;
  }
}

void ensure_slots(rgpu_ctx* c, int algo, int nuse) {
  const int64_t nrow_need = c->partitioned ? c->pk.n_own : c->g.nv;
  if (c->cap_nv < c->g.nv || c->cap_ne < c->g.ne || c->cap_nin < c->g.n_in || c->cap_nown < nrow_need) {
    release_slots(c);
    c->cap_nv = c->g.nv;
    c->cap_ne = c->g.ne;
    c->cap_nin = c->g.n_in;
    c->cap_nown = nrow_need;
  }
  auto& L = c->slot_allocs;
  auto& LG = c->graph_allocs;  // heavy-vertex buffers: sized by the graph's segments
  const int64_t nv = c->cap_nv, ne = c->cap_ne, nin = c->cap_nin;
  const size_t rows = (size_t)nv * kViews;
  for (int i = 0; i < nuse; i++) {
    Slot& s = c->slot[i];
    if (!s.stream) {
      HIPCHK(hipStreamCreateWithFlags(&s.stream, hipStreamNonBlocking));
      HIPCHK(hipEventCreateWithFlags(&s.ev, hipEventDisableTiming));
      HIPCHK(hipHostMalloc((void**)&s.h_stepcnt, sizeof(int32_t) * kMaxSteps, hipHostMallocMapped));
      HIPCHK(hipHostGetDevicePointer((void**)&s.d_hostflag, s.h_stepcnt, 0));
      HIPCHK(hipHostMalloc((void**)&s.h_stats, sizeof(unsigned long long) * kStatWords));
      HIPCHK(hipHostMalloc((void**)&s.h_work, sizeof(unsigned long long) * kWorkWords));
      s.stepcnt = dalloc<int32_t>(L, kMaxSteps);
      s.ccount = dalloc<int32_t>(L, (size_t)kMaxSteps * kCountShards + kMinWords);  // + the minimum labels (mneg)
      s.stats = dalloc<unsigned long long>(L, kStatWords);
      HIPCHK(hipMemset(s.stats, 0, sizeof(unsigned long long) * kStatWords));
    }
    if (algo == RGPU_ALGO_CC && !s.a_cc) {
      // padded so that the superstep kernel's clamped, unconditional loads stay in bounds
      s.cnt = dalloc<int32_t>(L, nv + kPad);
      s.snbr = dalloc<int32_t>(L, ne + nin + kPad);
      s.smask = dalloc<uint64_t>(L, ne + nin + kPad);
      s.lab[0] = dalloc<int32_t>(L, rows + kPad * kViews);
      s.lab[1] = dalloc<int32_t>(L, rows + kPad * kViews);
      s.uw[0] = dalloc<int32_t>(L, nv + kPad);
      s.uw[1] = dalloc<int32_t>(L, nv + kPad);
      // component counts at the root's row (zero between batches).  Partitioned: a label is counted
      // at its owner, at the label vertex's owned rank (xchg.hip label_row), so only owned rows exist
      // — ghosts are most of a partition's ranks at P = 8 (1B graph: ~15M of ~17M)
      const size_t crows = (size_t)c->cap_nown * kViews + kPad * kViews;
      s.counts = dalloc<int32_t>(L, crows);
      HIPCHK(hipMemset(s.counts, 0, sizeof(int32_t) * crows));
      s.chg[0] = dalloc<uint64_t>(L, nv + kPad);
      s.chg[1] = dalloc<uint64_t>(L, nv + kPad);
      HIPCHK(hipMemset(s.chg[0], 0, sizeof(uint64_t) * (nv + kPad)));
      HIPCHK(hipMemset(s.chg[1], 0, sizeof(uint64_t) * (nv + kPad)));
      HIPCHK(hipMemset(s.snbr, 0, sizeof(int32_t) * (ne + nin + kPad)));
      for (int b = 0; b < 3; b++) s.act[b] = dalloc<uint8_t>(L, (size_t)((nv + 7) / 8 + 1) * 8);
      for (int b = 0; b < 3; b++) s.cb[b] = dalloc<uint64_t>(L, (size_t)((nv + 63) / 64 + 1));
      s.vadj = dalloc<uint64_t>(L, nv);
      s.work = dalloc<unsigned long long>(L, kWorkWords);
      s.iso = dalloc<unsigned int>(L, kIsoWords);  // zero between batches: the summary kernel clears it
      HIPCHK(hipMemset(s.iso, 0, sizeof(unsigned int) * kIsoWords));
    }
    if (algo == RGPU_ALGO_CC && !s.h_cc && c->g.n_seg > 0) {
      s.hv.segcnt = dalloc<int32_t>(LG, c->g.n_seg);
      s.hv.segor = dalloc<uint64_t>(LG, c->g.n_seg);
      s.hv.best = dalloc<int32_t>(LG, (size_t)c->g.n_heavy * kViews);  // INT32_MAX between uses
      HIPCHK(hipMemsetD32((hipDeviceptr_t)s.hv.best, INT32_MAX, (size_t)c->g.n_heavy * kViews));
    }
    if ((algo == RGPU_ALGO_DEGREE || algo == RGPU_ALGO_PR) && !s.a_deg) {
      s.outdeg = dalloc<int32_t>(L, rows);
      s.indeg = dalloc<int32_t>(L, rows);
    }
    if (algo == RGPU_ALGO_DEGREE && !s.top.key) {
      const size_t nc = (size_t)deg_top_waves(nv) * kViews * kTop;
      s.top.cand_key = dalloc<uint64_t>(L, nc);
      s.top.cand_pos = dalloc<int32_t>(L, nc);
      s.top.key = dalloc<unsigned long long>(L, kViews * kTop);
      s.top.pos = dalloc<int32_t>(L, kViews * kTop);
      s.top.out = dalloc<int32_t>(L, kViews * kTop);
      HIPCHK(hipHostMalloc((void**)&s.h_top, sizeof(unsigned long long) * kViews * kTop * 2));
    }
    if (algo == RGPU_ALGO_PR && !s.h_pr && c->g.n_seg > 0) {
      s.hv.pacc = dalloc<double>(LG, (size_t)c->g.n_heavy * kViews);  // zero between uses
      HIPCHK(hipMemset(s.hv.pacc, 0, sizeof(double) * (size_t)c->g.n_heavy * kViews));
    }
    if (algo == RGPU_ALGO_VP && !s.a_vp) {
      if (!s.cnt) s.cnt = dalloc<int32_t>(L, nv + kPad);
      if (!s.snbr) s.snbr = dalloc<int32_t>(L, ne + nin + kPad);
      if (!s.smask) s.smask = dalloc<uint64_t>(L, ne + nin + kPad);
      for (int b = 0; b < 2; b++) {
        if (!s.chg[b]) s.chg[b] = dalloc<uint64_t>(L, nv + kPad);
        s.vst[b] = dalloc<int64_t>(L, rows);
      }
    }
    if (algo == RGPU_ALGO_VP && c->vp.fsum && c->vp.per_degree && !s.vdeg) s.vdeg = dalloc<int32_t>(L, rows);
    if (algo == RGPU_ALGO_DIFFUSION && !s.a_diff) {
      s.dinf = dalloc<uint64_t>(L, nv + kPad);
      s.dfront[0] = dalloc<uint64_t>(L, nv + kPad);
      s.dfront[1] = dalloc<uint64_t>(L, nv + kPad);
      s.dstep = dalloc<uint8_t>(L, rows);
      for (int b = 0; b < 3; b++) s.dact[b] = dalloc<uint8_t>(L, (size_t)((nv + 7) / 8 + 1) * 8);
    }
    if (algo == RGPU_ALGO_PR && !s.a_pr) {
      s.pr = dalloc<double>(L, rows);
      s.contrib[0] = dalloc<double>(L, rows);
      s.contrib[1] = dalloc<double>(L, rows);
      s.pcnt = dalloc<int32_t>(L, nv);
      s.psnbr = dalloc<int32_t>(L, nin + nv);
      s.psmask = dalloc<uint64_t>(L, nin + nv);
    }
  }
  if (c->partitioned && algo == RGPU_ALGO_PR && !c->pt.pr_ready) {
    Part& X = c->pt;
    X.sbuf_f = dalloc<double>(LG, (size_t)std::max<int64_t>(X.nxs, 1) * kViews);
    X.rbuf_f = dalloc<double>(LG, (size_t)std::max<int64_t>(X.nxr, 1) * kViews);
    X.pr_ready = true;
  }
  for (int i = 0; i < nuse; i++) {
    Slot& s = c->slot[i];
    if (algo == RGPU_ALGO_CC) s.a_cc = s.h_cc = true;
    if (algo == RGPU_ALGO_PR) s.h_pr = true;
    if (algo == RGPU_ALGO_DEGREE || algo == RGPU_ALGO_PR) s.a_deg = true;
    if (algo == RGPU_ALGO_PR) s.a_pr = true;
    if (algo == RGPU_ALGO_DIFFUSION) s.a_diff = true;
    if (algo == RGPU_ALGO_VP) s.a_vp = true;
  }
  if ((algo == RGPU_ALGO_DIFFUSION || algo == RGPU_ALGO_VP) && !c->d_vid) c->d_vid = dalloc<int64_t>(L, nv);
}

struct RunCfg {
  int algo, max_steps, pr_iters, flags;
  int K, W;         // hops per batch (64 / gsize), windows of the run
  int G, gsize;     // window groups (batches per hop block), windows per group
  size_t nblk, nb;  // hop blocks, batches
  const int64_t* hops;
  size_t n_hops;
  int64_t thr_v[kViews], thr_e[kViews];
  int64_t wval[kViews];  // the user's window values (-1 = ViewLens): diffusion coin salts
  int chunk0, chunk;
};

// batch slots a run uses: one per batch in flight, never more than the batches it has
int run_slots(const rgpu_ctx* c, const RunCfg& rc) {
  const int n = (rc.flags & RGPU_RUN_SERIAL) ? 1 : c->nslots;
  return (int)std::max<size_t>(1, std::min<size_t>((size_t)n, rc.nb));
}

// diffusion coin salt of a view (include/rgpu.h, rgpu_set_diffusion)
uint64_t hmix64(uint64_t x) {
  x ^= x >> 30;
  x *= 0xbf58476d1ce4e5b9ull;
  x ^= x >> 27;
  x *= 0x94d049bb133111ebull;
  x ^= x >> 31;
  return x;
}
uint64_t diff_salt(uint64_t coin_seed, int64_t t, int64_t w) {
  return hmix64(coin_seed ^ hmix64((uint64_t)t ^ hmix64((uint64_t)w)));
}


// K1 edge masks: per edge its offsets (8), its endpoints (8) and their death bits; an edge the
// SKIP instantiation leaves to K2 (simple: one add point, no endpoint deaths) costs its one
// history point (8) more and nothing else; every other edge its history points, two death-list
// offsets per endpoint (16) and one mask word per plane.
double bytes_emask(const rgpu_ctx* c, int planes, bool skip_simple) {
  const DevGraph& g = c->g;
  const double ne = (double)g.ne, simple = skip_simple ? (double)std::max<int64_t>(c->n_simple, 0) : 0.0;
  const double keys = (double)c->pk.n_ekey;
  if (skip_simple && g.ens) {  // the non-simple list (kernels.hip k_edge_mask): per listed edge its id, its
                               // two offsets, both endpoints, its keys, the death offsets and the plane stores
    const double ns = (double)g.n_ens;
    return 4.0 * ns + 16.0 * ns + 8.0 * ns + 8.0 * (keys - simple) + (16.0 + 8.0 * planes) * ns;
  }
  return 8.0 * (ne + 1) + 8.0 * ne + (skip_simple ? 8.0 * simple : 0.0) + 8.0 * (keys - simple) +
         (16.0 + 8.0 * planes) * (ne - simple);
}

void launch_chunk(rgpu_ctx* c, int si, const RunCfg& rc, int n) {
  Slot& s = c->slot[si];
  const DevGraph& g = c->g;
  int last = std::min(rc.max_steps, s.r_launched + n);
  // profile: ONE event pair around the chunk's back-to-back superstep launches (per-launch
  // pairs add ~3 us of marker latency to a ~12 us kernel; rocprofv3's per-dispatch times
  // agree with the chunk average)
  // With heavy vertices the chunk interleaves k_heavy_gather / k_heavy_mark with the superstep
  // kernel, so each launch gets its own pair instead (a superstep is ~1 ms there, the pair's
  // latency noise), and the superstep kernel's average is its own, as rocprofv3 reports it.
  const bool hv = g.n_seg > 0 && rc.algo == RGPU_ALGO_CC;
  const bool per_launch = c->profile && hv;
  hipEvent_t ea = nullptr, eb = nullptr;
  if (c->profile && !per_launch && last > s.r_launched) {
    ea = take_event(c);
    eb = take_event(c);
    HIPCHK(hipEventRecord(ea, s.stream));
  }
  for (int r = s.r_launched + 1; r <= last; r++) {
    if (rc.algo == RGPU_ALGO_VP) {
      timed_launch(c, si, KID_VP, 0.0, [&] {
        launch_vp_step(s.stream, r, g, c->vp, s.vm, s.cnt, s.snbr, s.smask, s.vst[(r - 1) & 1], s.vst[r & 1],
                       s.chg[(r - 1) & 1], s.chg[r & 1], s.stepcnt, s.d_hostflag,
                       s.stats + kLaneOff, s.vdeg);
      }, r, false);
      continue;
    }
    if (rc.algo == RGPU_ALGO_DIFFUSION) {
      timed_launch(c, si, KID_DIFF, 0.0, [&] {
        launch_diff_step(s.stream, r, g, c->d_vid, s.vm, s.em, s.dinf, s.dfront[(r - 1) & 1], s.dfront[r & 1],
                         s.dact[r % 3], s.dact[(r + 1) % 3], s.dact[(r + 2) % 3],
                         (rc.flags & RGPU_RUN_RETAIN) ? s.dstep : nullptr, s.salts, c->diff_coin, s.stepcnt,
                         s.d_hostflag, s.stats);
      }, r, false);
      continue;
    }
    if (hv)  // heavy vertices: segment minima before the step, neighbour marking after it
      timed_launch(c, si, KID_HEAVY, 0.0, [&] {
        launch_heavy_gather(s.stream, g, s.snbr, s.smask, s.lab[(r - 1) & 1], s.chg[(r - 1) & 1], s.act[r % 3],
                            s.stepcnt, r, s.hv, s.uw[(r - 1) & 1], chg_bits(c, s, r).prev, s.ccount,
                            dense_div(c), work_buf(c, s), s.vm, min_labels(c, s), c->ko);
      }, r, per_launch);
    timed_launch(c, si, KID_STEP, 0.0, [&] {
      launch_cc_step(s.stream, r, g, s.vm, s.cnt, s.snbr, s.smask, s.lab[(r - 1) & 1], s.lab[r & 1],
                     s.chg[(r - 1) & 1], s.chg[r & 1], s.act[r % 3], s.act[(r + 1) % 3],
                     s.act[(r + 2) % 3], s.stepcnt, s.d_hostflag,
                     work_buf(c, s), s.stats + kLaneOff,
                     hv ? s.hv.best : nullptr, s.uw[(r - 1) & 1], s.uw[r & 1],
                     chg_bits(c, s, r), s.ccount, dense_div(c), min_labels(c, s), s.long_views, c->ko);
    }, r, per_launch);
    if (hv)
      timed_launch(c, si, KID_HEAVY, 0.0, [&] {
        launch_heavy_mark(s.stream, g, s.snbr, s.smask, s.chg[r & 1], s.act[(r + 1) % 3], s.stepcnt, r, s.hv,
                          s.act[r % 3], nullptr, nullptr, INT64_MIN, s.ccount, dense_div(c), work_buf(c, s),
                          nullptr, c->ko);
      }, r, per_launch);
  }
  if (ea) {
    HIPCHK(hipEventRecord(eb, s.stream));
    c->timed.push_back({rc.algo == RGPU_ALGO_DIFFUSION ? KID_DIFF : rc.algo == RGPU_ALGO_VP ? KID_VP : KID_STEP, si,
                        s.batch, s.r_launched + 1, ea, eb, 0.0});
  }
  s.r_launched = last;
  if (c->profile && rc.algo == RGPU_ALGO_CC)
    HIPCHK(hipMemcpyAsync(s.h_work, s.work, sizeof(unsigned long long) * kWorkWords,
                          hipMemcpyDeviceToHost, s.stream));
  HIPCHK(hipEventRecord(s.ev, s.stream));
  s.evseq = ++c->evcounter;
  s.phase = 1;
}

// the end of every batch: per-view stats and retained rows to the host, the mask set released
void finish_tail(rgpu_ctx* c, int si, const RunCfg& rc) {
  Slot& s = c->slot[si];
  const DevGraph& g = c->g;
  if (rc.algo == RGPU_ALGO_CC || rc.algo == RGPU_ALGO_VP) launch_lane_fold(s.stream, s.stats + kLaneOff, s.stats + kFoldOff);
  HIPCHK(hipMemcpyAsync(s.h_stats, s.stats, sizeof(unsigned long long) * kStatCopy,
                        hipMemcpyDeviceToHost, s.stream));
  if (c->profile && rc.algo == RGPU_ALGO_CC && s.work)  // the batch's work counters (the partitioned
    HIPCHK(hipMemcpyAsync(s.h_work, s.work, sizeof(unsigned long long) * kWorkWords,  // path copies them here only)
                          hipMemcpyDeviceToHost, s.stream));
  if (rc.algo == RGPU_ALGO_DEGREE) {  // the top-20 lists
    HIPCHK(hipMemcpyAsync(s.h_top, s.top.key, sizeof(unsigned long long) * kViews * kTop, hipMemcpyDeviceToHost,
                          s.stream));
    int32_t* hp = reinterpret_cast<int32_t*>(s.h_top + kViews * kTop);
    HIPCHK(hipMemcpyAsync(hp, s.top.pos, sizeof(int32_t) * kViews * kTop, hipMemcpyDeviceToHost, s.stream));
    HIPCHK(hipMemcpyAsync(hp + kViews * kTop, s.top.out, sizeof(int32_t) * kViews * kTop, hipMemcpyDeviceToHost,
                          s.stream));
  }
  if (rc.flags & RGPU_RUN_RETAIN) {
    Retained& R = c->kept[s.batch];
    const size_t rows = (size_t)g.nv * kViews;
    R.vm.resize(g.nv);
    HIPCHK(hipMemcpyAsync(R.vm.data(), s.vm, sizeof(uint64_t) * g.nv, hipMemcpyDeviceToHost, s.stream));
    if (rc.algo == RGPU_ALGO_CC) {
      R.a.resize(rows);
      HIPCHK(hipMemcpyAsync(R.a.data(), s.lab[s.r_final & 1], sizeof(int32_t) * rows,
                            hipMemcpyDeviceToHost, s.stream));
    } else if (rc.algo == RGPU_ALGO_VP) {
      R.v64.resize(rows);
      HIPCHK(hipMemcpyAsync(R.v64.data(), s.vst[s.r_final & 1], sizeof(int64_t) * rows, hipMemcpyDeviceToHost,
                            s.stream));
    } else if (rc.algo == RGPU_ALGO_DIFFUSION) {
      R.st.resize(rows);
      HIPCHK(hipMemcpyAsync(R.st.data(), s.dstep, rows, hipMemcpyDeviceToHost, s.stream));
    } else if (rc.algo == RGPU_ALGO_DEGREE) {
      R.a.resize(rows);
      R.b.resize(rows);
      HIPCHK(hipMemcpyAsync(R.a.data(), s.outdeg, sizeof(int32_t) * rows, hipMemcpyDeviceToHost, s.stream));
      HIPCHK(hipMemcpyAsync(R.b.data(), s.indeg, sizeof(int32_t) * rows, hipMemcpyDeviceToHost, s.stream));
    } else {
      R.pr.resize(rows);
      HIPCHK(hipMemcpyAsync(R.pr.data(), s.pr, sizeof(double) * rows, hipMemcpyDeviceToHost, s.stream));
    }
  }
  if (rc.G > 1) {  // the batch no longer reads its mask set
    MaskSet& M = c->mset[(s.batch / rc.G) % c->nsets];
    HIPCHK(hipEventRecord(M.done[s.batch % rc.G], s.stream));
    M.pending--;
  }
  HIPCHK(hipEventRecord(s.ev, s.stream));
  s.evseq = ++c->evcounter;
  s.phase = 2;
}

void finish_batch(rgpu_ctx* c, int si, const RunCfg& rc) {
  Slot& s = c->slot[si];
  const DevGraph& g = c->g;
  if (rc.algo == RGPU_ALGO_CC) {
    int32_t* lab = s.lab[s.r_final & 1];
    const int nviews = rc.K * rc.gsize;
    if (c->check)
      run_check(s.stream, "final labels", [&](unsigned long long* bad) {
        launch_check_labels(s.stream, c->partitioned ? c->pk.n_own : g.nv, s.vm, s.uw[s.r_final & 1],
                            lab, bad, g.grank);
      });
    const int32_t* uw = s.uw[s.r_final & 1];
    if (rc.flags & RGPU_RUN_RETAIN) launch_uw_rows(s.stream, g.nv, s.vm, uw, lab);  // full rows to the host
    timed_launch(c, si, KID_HIST, 28.0 * g.nv,
                 [&] { launch_cc_count(s.stream, g.nv, nviews, s.vm, s.vadj, uw, lab, s.counts, s.iso); });
    timed_launch(c, si, KID_SUMMARY, 20.0 * g.nv,
                 [&] { launch_cc_roots(s.stream, g.nv, nviews, s.vm, s.vadj, uw, lab, s.counts, s.stats, s.iso,
                                         s.r_final >= 1 && s.r_final >= rc.max_steps, g.grank); });
  }
  finish_tail(c, si, rc);
}

void part_post_step(rgpu_ctx* c, int si, const RunCfg& rc, int r);
void part_finish_begin(rgpu_ctx* c, int si, const RunCfg& rc);
void part_min_labels(rgpu_ctx* c, int si);
void part_vm_exchange(rgpu_ctx* c, int si, uint64_t* vm, int64_t vstride, int planes, bool free);
bool ghost_vm_free(const rgpu_ctx* c, const RunCfg& rc);

// Batch b = hop block b / G (hops [hb*K, hb*K + K)) x window group b % G.  Hop-major runs
// (G = 1): the batch is the block, all windows in one label row, K1 per batch into the slot's
// own masks.  Window-major runs (G = W): one window per batch; K1 runs once per block, for
// every window, on the stream of the block's first batch, into a shared mask set.
bool can_start(const rgpu_ctx* c, size_t b, const RunCfg& rc) {
  if (rc.G == 1 || b % rc.G != 0) return true;
  return c->mset[(b / rc.G) % c->nsets].pending == 0;  // set still read by an older block
}

// the hops' common step when a block's hops are evenly spaced (K1 then finds hop indices
// arithmetically), else 0
int64_t even_jump(const BatchParams& bp) {
  if (bp.K < 2 || !bp.sorted) return 0;
  const int64_t j = bp.hop[1] - bp.hop[0];
  if (j <= 0 || j > ((int64_t)1 << 40)) return 0;
  for (int k = 2; k < bp.K; k++)
    if (bp.hop[k] - bp.hop[k - 1] != j) return 0;
  return j;
}

void start_batch(rgpu_ctx* c, int si, int b, const RunCfg& rc) {
  Slot& s = c->slot[si];
  const DevGraph& g = c->g;
  if (c->inject_fail > 0 && --c->inject_fail == 0)  // fault injection (tests): after earlier batches ran
    throw HipFail{"RGPU_INJECT_FAIL: injected failure at batch " + std::to_string(b)};
  const size_t hb = (size_t)b / rc.G;
  const int grp = b % rc.G;
  BatchParams bp;
  std::memset(&bp, 0, sizeof(bp));
  const size_t h0 = hb * rc.K;
  bp.K = (int)std::min<size_t>(rc.K, rc.n_hops - h0);
  bp.W = rc.W;
  bp.KS = rc.K;
  bp.sorted = 1;
  bp.iv_max = c->iv_max;
  for (int k = 0; k < bp.K; k++) {
    bp.hop[k] = rc.hops[h0 + k];
    if (k > 0 && bp.hop[k] < bp.hop[k - 1]) bp.sorted = 0;
  }
  bp.jump = even_jump(bp);
  for (int w = 0; w < rc.W; w++) { bp.thr_v[w] = rc.thr_v[w]; bp.thr_e[w] = rc.thr_e[w]; }
  // K2's cut: an edge is kept only where its floor point is an add no older than the window
  // (age <= thr_e), so one whose last add is before min(hop) - max(window of the batch) is
  // dead in every view of the batch
  int64_t tcut = INT64_MIN;
  {
    const int w0 = rc.G == 1 ? 0 : grp * rc.gsize, w1 = rc.G == 1 ? rc.W : w0 + rc.gsize;
    int64_t thr = 0, hmin = INT64_MAX;
    for (int w = w0; w < w1; w++) thr = std::max(thr, rc.thr_e[w]);
    for (int k = 0; k < bp.K; k++) hmin = std::min(hmin, bp.hop[k]);
    if (thr < INT64_MAX / 4 && hmin > INT64_MIN / 4) tcut = hmin - thr;
  }
  s.tcut = tcut;
  {  // long views: the batch's views nearly coincide (the lane-parallel superstep forms pay)
    const int w0 = rc.G == 1 ? 0 : grp * rc.gsize, w1 = rc.G == 1 ? rc.W : w0 + rc.gsize;
    int64_t wmin = INT64_MAX, hmin = INT64_MAX, hmax = INT64_MIN;
    for (int w = w0; w < w1; w++) wmin = std::min(wmin, rc.thr_e[w]);
    for (int k = 0; k < bp.K; k++) {
      hmin = std::min(hmin, bp.hop[k]);
      hmax = std::max(hmax, bp.hop[k]);
    }
    const int64_t span = std::max<int64_t>(hmax - hmin, 1);
    s.long_views = c->long_ratio >= 0 && wmin / span >= c->long_ratio;
  }
  s.batch = b;
  s.kb = bp.K;
  s.r_launched = 0;
  s.r_final = 0;
  std::memset(s.h_stepcnt, 0, sizeof(int32_t) * kMaxSteps);  // slot idle: no kernel writes it
  BatchClear clr;
  clr.stats = s.stats;
  clr.n_stats = kStatCopy;  // the lane shards are zero: cleared by the fold of the slot's previous batch
  clr.flags = s.stepcnt;
  clr.n_flags = kMaxSteps;
  if (rc.algo == RGPU_ALGO_CC || rc.algo == RGPU_ALGO_DIFFUSION) {
    for (int b = 0; b < 3; b++) clr.act[b] = rc.algo == RGPU_ALGO_CC ? s.act[b] : s.dact[b];
    clr.n_act_words = (g.nv + 7) / 8 + 1;
    if (rc.algo == RGPU_ALGO_CC) {
      clr.ccount = s.ccount;
      clr.n_ccount = (int64_t)kMaxSteps * kCountShards + kMinWords;
    }
    const ChgBits cb1 = rc.algo == RGPU_ALGO_CC ? chg_bits(c, s, 1) : ChgBits();
    if (cb1.next) {
      for (int b = 0; b < 3; b++) clr.cb[b] = s.cb[b];
      clr.n_cb_words = cb1.words;
    }
  }
  if (s.work && c->profile)
    HIPCHK(hipMemsetAsync(s.work, 0, sizeof(unsigned long long) * kWorkWords, s.stream));
  // K1 byte models.  Vertex masks: offsets, two floor probes per vertex (the
  // interval form's binary searches; the points between them are not counted: a lower bound) and
  // the plane stores.  Edge masks: see bytes_emask.
  const double bv = 8.0 * (g.nv + 1) + 16.0 * g.nv;
  // partitioned: K1 computes the owned vertices' masks (a ghost's history is its owner's);
  // the ghosts' words arrive from their owners right after
  DevGraph gk = g;
  if (c->partitioned) gk.nv = c->pk.n_own;
  // (K1 folding both endpoints' memberships into the CC edge words measured slower on C4: K1 55 ->
  // 97 ms for K2 122 -> 117 ms; the kernels keep the path, off)
  const bool ends = false;
  // Inline edge bits (kernels.hip simple_bits): CC's K2 computes the window bits of the simple
  // slots (one add point, no endpoint deaths) for the batch's own windows from the time-ordered
  // slot words, so K1 writes edge masks only for the other edges (all of them for the |E_w|
  // counts of an RGPU_RUN_EDGE_COUNTS run).  The partitioned ghost marking (k_xmark) does the same.
  const bool iem = rc.algo == RGPU_ALGO_CC && g.ts_t;
  BatchParams ebp = bp;  // the batch's edge windows, view bit w*KS + k
  if (rc.G > 1) {
    ebp.W = 1;
    ebp.thr_e[0] = rc.thr_e[grp];
  }
  const bool skip_simple = iem && !c->d_ecnt;
  {
    const int w0 = rc.G == 1 ? 0 : grp * rc.gsize, w1 = rc.G == 1 ? rc.W : w0 + rc.gsize;
    ebp.simple_ends = 1;
    for (int w = w0; w < w1; w++) ebp.simple_ends &= rc.thr_v[w] == rc.thr_e[w];
  }
  s.iem = iem;
  s.ebp = ebp;
  // K1 floor carry (BatchParams::carry): read the previous block's floors when its last hop is
  // not after this block's first; write this block's for the next
  const bool k1_runs = rc.G == 1 || grp == 0;
  if (k1_runs && c->k1_carry && c->k1c_v && bp.sorted) {
    bp.carry = c->k1_last != INT64_MIN && c->k1_last <= bp.hop[0] ? 2 : 1;
    // every K1 that writes the carry arrays (carry 1 or 2) is ordered after the previous carry K1
    // of the run, which ran on another slot's stream: a write-only block after a backward hop must
    // not overwrite floors that block is still reading or writing
    if (c->k1_ev_live) HIPCHK(hipStreamWaitEvent(s.stream, c->k1_ev, 0));
    c->k1_last = bp.hop[bp.K - 1];
  } else if (k1_runs) {
    c->k1_last = INT64_MIN;
  }
  int32_t* fcv = bp.carry ? c->k1c_v : nullptr;
  int32_t* fce = bp.carry ? c->k1c_e : nullptr;
  if (rc.G == 1) {
    s.vm = s.vm_own;
    s.em = s.em_own;
    timed_launch(c, si, KID_MASK, bv + 8.0 * g.nv, [&] { launch_vertex_mask(s.stream, gk, bp, s.vm, 0, false, clr, fcv); });
    timed_launch(c, si, KID_EMASK, bytes_emask(c, 1, skip_simple), [&] {
      launch_edge_mask(s.stream, g, bp, s.em, false, c->d_ecnt, (int64_t)h0, ends ? s.vm : nullptr, 0, skip_simple,
                       fce);
    });
    if (bp.carry) {
      HIPCHK(hipEventRecord(c->k1_ev, s.stream));
      c->k1_ev_live = true;
    }
    if (c->partitioned) part_vm_exchange(c, si, s.vm, 0, 1, ghost_vm_free(c, rc));
  } else {
    MaskSet& M = c->mset[hb % c->nsets];
    if (grp == 0) {
      // the set's previous block is finished-enqueued (can_start); wait for it on the device
      for (int w = 0; w < rc.G; w++) HIPCHK(hipStreamWaitEvent(s.stream, M.done[w], 0));
      const BatchClear none;
      timed_launch(c, si, KID_MASK, bv + 8.0 * g.nv * rc.W,
                   [&] { launch_vertex_mask(s.stream, gk, bp, M.vm, g.nv + kPad, true, none, fcv); });
      timed_launch(c, si, KID_EMASK, bytes_emask(c, rc.W, skip_simple), [&] {
        launch_edge_mask(s.stream, g, bp, M.em, true, c->d_ecnt, (int64_t)h0, ends ? M.vm : nullptr, g.nv + kPad,
                         skip_simple, fce);
      });
      if (bp.carry) {
        HIPCHK(hipEventRecord(c->k1_ev, s.stream));
        c->k1_ev_live = true;
      }
      if (c->partitioned) part_vm_exchange(c, si, M.vm, g.nv + kPad, rc.G, ghost_vm_free(c, rc));
      HIPCHK(hipEventRecord(M.k1, s.stream));
      M.pending = rc.G;
    } else {
      HIPCHK(hipStreamWaitEvent(s.stream, M.k1, 0));
    }
    s.vm = M.vm + (size_t)grp * (g.nv + kPad);
    s.em = M.em + (size_t)grp * g.ne;
    launch_batch_clear(s.stream, clr);
    HIPCHK(hipGetLastError());
  }
  if (rc.algo == RGPU_ALGO_VP) {  // setup (superstep 0), only when maxSteps > 1 (AnalysisTask.timeResponse :169)
    launch_vp_setup(s.stream, g, c->vp, c->d_vid, s.vm, s.em, s.cnt, s.snbr, s.smask, s.vst[0], s.chg[0], s.vdeg);
    HIPCHK(hipGetLastError());
    s.r_launched = 0;
    if (rc.max_steps <= 1) {
      s.r_final = 0;
      finish_batch(c, si, rc);
    } else {
      launch_vp_go(s.stream, s.stepcnt);
      const int last = c->grp_last[grp];
      launch_chunk(c, si, rc, last > 0 ? std::max(2, std::min(rc.chunk0, last + 1)) : rc.chunk0);
    }
    return;
  }
  if (rc.algo == RGPU_ALGO_DIFFUSION) {
    // coin salts: lane j = wl*K + k is hop h0 + k, window grp*gsize + wl (include/rgpu.h)
    for (int j = 0; j < kViews; j++) {
      const int k = j % rc.K, wl = j / rc.K;
      const int64_t t = k < bp.K ? bp.hop[k] : 0;
      const int64_t w = wl < rc.gsize ? rc.wval[grp * rc.gsize + wl] : -1;
      s.salts.s[j] = diff_salt(c->diff_coin_seed, t, w);
    }
    // Setup (superstep 0) only when defineMaxSteps > 1 (AnalysisTask.timeResponse :169)
    launch_diff_setup(s.stream, g, s.vm, rc.max_steps > 1 ? c->diff_seed_rank : -1, s.dinf, s.dfront[0],
                      s.dact[1], (rc.flags & RGPU_RUN_RETAIN) ? s.dstep : nullptr, s.stats);
    HIPCHK(hipGetLastError());
    s.r_launched = 0;
    if (rc.max_steps <= 1) {
      s.r_final = 0;
      finish_batch(c, si, rc);
    } else {
      // first chunk sized by the step the group's previous batch halted at (+1 for its halt step)
      const int last = c->grp_last[grp];
      launch_chunk(c, si, rc, last > 0 ? std::max(2, std::min(rc.chunk0, last + 1)) : rc.chunk0);
    }
    return;
  }
  if (rc.algo == RGPU_ALGO_CC) {
    if (c->partitioned && g.nv > c->pk.n_own)  // ghosts: quiet until a record arrives (kGhostQuiet)
      for (int p = 0; p < 2; p++)
        HIPCHK(hipMemsetAsync(s.uw[p] + c->pk.n_own, 0x7f, sizeof(int32_t) * (g.nv - c->pk.n_own), s.stream));
    // bytes: per vertex vm + 4 offsets + label rows 0/1 + cnt/vadj/chg; per static slot index,
    // em, vm[nb]; kept slots written (12 B each, counted in harvest)
    const double b2 = 8.0 * g.nv;  // the view-mask scan; the rest from the work counters (harvest)
    if (g.n_seg > 0)
      timed_launch(c, si, KID_HEAVY, 0.0,
                   [&] {
                     launch_heavy_slots(s.stream, g, tcut, s.vm, s.em, s.snbr, s.smask, s.hv, ends, work_buf(c, s),
                                        iem ? &ebp : nullptr, c->ko);
                   });
    timed_launch(c, si, KID_SLOTS, b2, [&] {  // (partitioned: owned vertices only, gk)
      launch_cc_slots(s.stream, gk, tcut, s.vm, s.em, s.cnt, s.snbr, s.smask, s.vadj, s.lab[0], s.lab[1],
                      s.chg[1], s.act[2], s.stepcnt, s.d_hostflag,
                      work_buf(c, s), s.hv, s.stats + kLaneOff, s.uw[0],
                      s.uw[1], chg_bits(c, s, 1).next, ends, s.ccount, iem ? &ebp : nullptr,
                      dense_div(c), min_labels(c, s), c->partitioned ? c->pt.gpeer : nullptr,
                      c->partitioned ? c->pt.xs[si].pmask : nullptr, c->ko);
    });
    if (c->check)
      run_check(s.stream, "after K2", [&](unsigned long long* bad) {
        launch_check_slots(s.stream, gk.nv, g.nv, g.adj_off, s.vm, s.cnt, s.snbr, s.uw[0],
                           s.uw[1], bad, g.grank);
      });
    if (g.n_seg > 0 && (c->ko.step & kHubDemote)) {  // owned hubs keeping few slots: the light path (§4i)
      const int dd = dense_div(c);
      timed_launch(c, si, KID_HEAVY, 0.0, [&] {
        launch_hub_demote(s.stream, g, s.hv, s.cnt, s.snbr, s.smask, s.chg[1], s.act[2], dd > 0 && (dd & kDense1));
      });
    }
    if (g.n_seg > 0 && !c->partitioned)  // partitioned: after the step's records are in
      timed_launch(c, si, KID_HEAVY, 0.0, [&] {
        launch_heavy_mark(s.stream, g, s.snbr, s.smask, s.chg[1], s.act[2], s.stepcnt, 1, s.hv, nullptr, nullptr,
                          nullptr, INT64_MIN, s.ccount, dense_div(c), work_buf(c, s), nullptr, c->ko);
      });
    s.r_launched = 1;  // superstep 1 ran inside the slot kernel
    if (c->partitioned) {
      s.r_final = 0;
      // the ghosts' slots at or after the batch's cut (the record apply walks only those)
      timed_launch(c, si, KID_XCHG, 0.0, [&] { launch_ghost_cut(s.stream, g, tcut, c->pt.xs[si].gcut); });
      part_min_labels(c, si);  // (also the count pass's minimum-label counts, part_finish_begin)
      if (rc.max_steps <= 1) part_finish_begin(c, si, rc);
      else part_post_step(c, si, rc, 1);
      return;
    }
    if (rc.max_steps <= 1) {  // AnalysisTask.timeResponse :169: no Setup when maxSteps <= 1
      s.r_final = 0;
      finish_batch(c, si, rc);
    } else {
      // first chunk: up to the step the group's previous batch halted at
      const int last = c->grp_last[grp];
      launch_chunk(c, si, rc, last > 0 ? std::max(1, std::min(rc.chunk0, last)) : rc.chunk0);
    }
  } else {
    timed_launch(c, si, KID_DEGREE, g.nv * (8.0 + 32.0 + 512.0) + (double)(g.ne + g.n_in) * 12.0, [&] {
      launch_degree(s.stream, g, s.vm, s.em, s.outdeg, s.indeg, s.stats,
                    rc.algo == RGPU_ALGO_DEGREE ? &s.top : nullptr);
    });
    if (rc.algo == RGPU_ALGO_PR) {
      timed_launch(c, si, KID_SLOTS, g.nv * (8.0 + 24.0 + 256.0 + 1024.0) + (double)(g.n_in) * 24.0, [&] {
        launch_pr_slots(s.stream, g, s.vm, s.em, s.outdeg, s.pcnt, s.psnbr, s.psmask, s.pr, s.contrib[0]);
      });
      for (int it = 0; it < rc.pr_iters; it++) {
        const double bp_bytes = g.nv * (8.0 + 16.0 + 4.0 + 256.0 + 1024.0) + (double)(g.n_in + g.nv) * 12.0;
        timed_launch(c, si, KID_PR, bp_bytes, [&] {
          launch_pr_step(s.stream, g, s.vm, s.em, s.outdeg, s.pcnt, s.psnbr, s.psmask, s.contrib[it & 1],
                         s.contrib[(it + 1) & 1], s.pr, s.hv.pacc);
        });
      }
    }
    finish_batch(c, si, rc);
  }
}

int64_t label_id(const rgpu_ctx* c, int32_t l);

void harvest(rgpu_ctx* c, int si, const RunCfg& rc) {
  Slot& s = c->slot[si];
  const unsigned long long* h = s.h_stats;
  const size_t hb = (size_t)s.batch / rc.G;
  const int grp = s.batch % rc.G;
  int32_t last[kViews] = {};  // per lane: last superstep with a label change (0: none)
  if (rc.algo == RGPU_ALGO_CC || rc.algo == RGPU_ALGO_VP)
    for (int r = 1; r <= s.r_final && r < kMaxSteps; r++)
      for (unsigned long long m = h[kFoldOff + r]; m; m &= m - 1) last[__builtin_ctzll(m)] = r;
  for (int k = 0; k < s.kb; k++)
    for (int wl = 0; wl < rc.gsize; wl++) {
      const int j = wl * rc.K + k;  // view bit: window-major within the batch
      const size_t view = (hb * rc.K + k) * rc.W + (size_t)grp * rc.gsize + wl;
      if (rc.algo == RGPU_ALGO_CC) {
        rgpu_cc_summary_t& o = c->cc[view];
        o.biggest = (int64_t)h[0 * kViews + j];
        o.total = (int64_t)h[1 * kViews + j];
        o.total_without_islands = (int64_t)h[2 * kViews + j];
        o.total_islands = o.total - o.total_without_islands;
        o.clusters_gt2 = (int64_t)h[3 * kViews + j];
        o.sum_all = (int64_t)h[4 * kViews + j];
        o.sum_without_islands = (int64_t)h[5 * kViews + j];
        o.supersteps = s.r_final;  // per hop after the run (finish_supersteps)
        c->vlast[view] = last[j];
      } else if (rc.algo == RGPU_ALGO_DEGREE) {
        for (int f = 0; f < 3; f++) c->deg[view * 3 + f] = (int64_t)h[f * kViews + j];
        const int32_t* hp = reinterpret_cast<const int32_t*>(s.h_top + kViews * kTop);
        for (int i = 0; i < kTop; i++) {
          const unsigned long long key = s.h_top[j * kTop + i];
          rgpu_ctx::TopEnt& e = c->degtop[view * kTop + i];
          if (key == 0) { e = {-1, 0, 0}; continue; }
          e.id = label_id(c, (int32_t)~(uint32_t)(key & 0xffffffffull));
          e.in = (int32_t)(key >> 32);
          e.out = hp[kViews * kTop + j * kTop + i];
        }
      } else if (rc.algo == RGPU_ALGO_DIFFUSION) {
        c->dcount[view] = (int64_t)h[j];
        c->dsteps[view] = s.r_final;
      } else if (rc.algo == RGPU_ALGO_VP) {
        c->vlast[view] = last[j];
      }
    }
  if (rc.algo == RGPU_ALGO_CC) {
    // algorithmic bytes from the profile run's work counters (kernels.hip
    // add_work).  K2 (superstep 1), on top of the 8 B per vertex of the view-mask scan counted
    // at launch: per non-member cnt + vadj cleared (12 B); per member its four offsets, cnt,
    // vadj and change word (52 B); per static slot scanned the time-ordered slot (edge 4,
    // neighbour 4, last-add time 8) and the two random mask words em[e], vm[nbr] (32 B; CSR
    // order: offsets 8 instead of 16); per kept slot nbr + mask written (12 B); uniform words
    // (4 B) and 64-B row lines written.  Supersteps r >= 2: frontier flag read + flag cleared
    // two steps ahead (2 B per vertex); per visited vertex vm,
    // cnt, adj_off, own change and uniform words in, change word out (40 B); per kept slot of
    // a visited vertex nbr + mask (12 B) and the neighbour's uniform word (4 B; without uniform
    // words its change word, 8 B); per slot of a mixed neighbour its change word (8 B); per
    // label lane gathered from a mixed row 4 B; own row lines read and row lines written (64 B
    // each); uniform words written (4 B).
    if (c->profile) {
      auto wsum = [&](int r, int f) {
        unsigned long long t = 0;
        for (int k = 0; k < 64; k++) t += s.h_work[((size_t)r * 64 + k) * kWorkFields + f];
        return t;
      };
      {
        const double mem = (double)wsum(1, 0);
        c->st.kernel_bytes[KID_SLOTS] += 12.0 * ((double)c->g.nv - mem) + 52.0 * mem +
                                         // per static slot: slot words (ts_e 4 + ts_nb 4 + ts_t 8, or the
                                         // CSR's 8), em[e] 8 unless inline (slot_bits: then neither em[e]
                                         // nor ts_e is read for a simple slot), vm[nb] 8
                                         ((c->g.ts_e ? 32.0 : 24.0) - (s.iem ? 12.0 : 0.0)) * (double)wsum(1, 4) +
                                         12.0 * (double)wsum(1, 1) +
                                         4.0 * (double)wsum(1, 7) + 64.0 * (double)wsum(1, 6);
      }
      // hub kernels (kernels.hip heavy_work, the step-0 row): per segment the gather visits, its
      // metadata and the hub's minima row (32 + 256 B); per slot it streams the neighbour (4 B) and
      // its changed bit (1/8 B, L2); per hot slot mask + uniform word (12 B), a mixed one's change
      // word (8 B) and its gathered lanes (4 B each); per slot the mark walks nbr + mask (12 B);
      // per static slot K2's segment pass scans (as K2: 32 B) and per kept slot it writes (12 B)
      c->st.kernel_bytes[KID_HEAVY] += 288.0 * wsum(0, 0) + 4.125 * wsum(0, 1) + 12.0 * wsum(0, 2) +
                                       8.0 * wsum(0, 3) + 4.0 * wsum(0, 4) + 12.0 * wsum(0, 5) +
                                       32.0 * wsum(0, 6) + 12.0 * wsum(0, 7);
      const double per_slot = 16.0;
      for (int r = 2; r <= s.r_final; r++)
        c->st.kernel_bytes[KID_STEP] +=
            2.0 * c->g.nv + 40.0 * (double)wsum(r, 0) + per_slot * (double)wsum(r, 1) +
            8.0 * (double)wsum(r, 4) + 4.0 * (double)wsum(r, 3) + 64.0 * (double)(wsum(r, 5) + wsum(r, 6)) +
            4.0 * (double)wsum(r, 7);
      if (!c->trace_path.empty())
        for (int r = 1; r <= s.r_final; r++)
          c->steprec.push_back({s.batch, r, wsum(r, 0), wsum(r, 1), (int)wsum(r, 2), wsum(r, 3)});
    }
    c->st.supersteps += s.r_final;
    c->grp_last[grp] = s.r_final;
  }
  if (rc.algo == RGPU_ALGO_VP) {
    c->st.supersteps += s.r_final;
    c->grp_last[grp] = s.r_final;
  }
  if (rc.algo == RGPU_ALGO_DIFFUSION) {
    // per executed superstep, the part every step pays: active flag read, flag
    // clear two steps ahead, front word store (9.125 B per vertex).  Active vertices' masks and
    // in-edges come on top and are not counted (a lower bound)
    c->st.kernel_bytes[KID_DIFF] += s.r_final * (9.125 * c->g.nv);
    c->st.supersteps += s.r_final;
    c->grp_last[grp] = s.r_final;
  }
  s.phase = 0;
  s.batch = -1;
}

int run_impl(rgpu_ctx* c, RunCfg& rc) {
  const size_t nb = rc.nb;
  c->st.views += (int64_t)(rc.n_hops * rc.W);
  c->st.batches += (int64_t)nb;
  size_t next = 0;
  const int nslots = run_slots(c, rc);
  using clk = std::chrono::steady_clock;
  double t_block = 0;  // host time blocked on events (RGPU_HOSTPROF)
  const auto t_run = clk::now();
  for (;;) {
    bool busy = false, progressed = false;
    for (int si = 0; si < nslots; si++) {
      Slot& s = c->slot[si];
      if (s.phase == 0) {
        if (next < nb && can_start(c, next, rc)) {
          start_batch(c, si, (int)next++, rc);
          progressed = true;
          busy = true;
        }
        continue;
      }
      busy = true;
      hipError_t q = hipEventQuery(s.ev);
      if (q == hipErrorNotReady) continue;
      HIPCHK(q);
      progressed = true;
      if (s.phase == 1) {
        int r0 = 0;
        for (int r = 1; r <= s.r_launched; r++)
          if (s.h_stepcnt[r] == 0) { r0 = r; break; }
        if (r0) { s.r_final = r0; finish_batch(c, si, rc); }
        else if (s.r_launched >= rc.max_steps) { s.r_final = rc.max_steps; finish_batch(c, si, rc); }
        else launch_chunk(c, si, rc, rc.chunk);
      } else {
        harvest(c, si, rc);
        if (next < nb && can_start(c, next, rc)) start_batch(c, si, (int)next++, rc);
      }
    }
    if (!busy) break;
    if (!progressed) {
      int oldest = -1;
      for (int si = 0; si < nslots; si++)
        if (c->slot[si].phase != 0 && (oldest < 0 || c->slot[si].evseq < c->slot[oldest].evseq)) oldest = si;
      // nothing ready.  Polling (default) reacts to whichever slot finishes first; blocking on
      // the oldest event left the other slots idle behind it (-8 % on the C2 query)
      if (oldest >= 0) __builtin_ia32_pause();
    }
  }
  if (c->hostprof)
    std::fprintf(stderr, "rgpu hostprof: run %.2f ms, blocked on events %.2f ms, launches %lld\n",
                 std::chrono::duration<double, std::milli>(clk::now() - t_run).count(), t_block,
                 (long long)c->evcounter);
  return 0;
}


// ------------------------------------------------------------------ vertex-partitioned runs
// One partition per GPU; kernels in xchg.hip.  A CC batch is the one-GPU
// batch with an exchange after every superstep r (AnalysisTask.syncMessages / endStep,
// AnalysisTask.scala:190-225, with ReaderWorker's vertex-message traffic replaced by records):
//   pack the records of the boundary vertices that changed -> counts all-to-all (records per
//   peer + the partition's halting vote) -> [host] -> clear the ghost change words of step r-2
//   -> grouped send/recv of the records -> ghost rows, ghost change words, next frontier ->
//   superstep r+1 -> ...
// The host reads the counts once per superstep per batch: up to three batches are in flight,
// each on its own stream and exchange channel, and the host serves the slots in a fixed round
// robin so that every partition issues each channel's collectives in the same order.
DevGraph owned_view(const rgpu_ctx* c) {
  DevGraph g = c->g;
  g.nv = c->pk.n_own;  // kernels that compute per-vertex results visit owned ranks only
  return g;
}

// record buffers grow on demand (the counts are known before anything is written into them):
// records of headroom per peer / first-guess records per boundary entry (RGPU_XREC_TINY)
int g_xrec_slack = 1024, g_xrec_init = 2;
template <class T>
void grow_regions(T** buf, int64_t* cap, const int64_t* need, int np, hipStream_t s) {
  bool grow = *buf == nullptr;
  for (int q = 0; q < np; q++) grow |= need[q] > cap[q];
  if (!grow) return;
  HIPCHK(hipStreamSynchronize(s));
  if (*buf) HIPCHK(hipFree(*buf));
  *buf = nullptr;
  int64_t tot = 0;
  for (int q = 0; q < np; q++) {
    cap[q] = std::max(cap[q], need[q] + need[q] / 2 + g_xrec_slack);
    tot += cap[q];
  }
  HIPCHK(hipMalloc((void**)buf, sizeof(T) * (size_t)tot));
}

template <class T>
T* alloc_regions(const int64_t* cap, int np) {
  int64_t tot = 0;
  for (int q = 0; q < np; q++) tot += cap[q];
  T* p = nullptr;
  HIPCHK(hipMalloc((void**)&p, sizeof(T) * (size_t)std::max<int64_t>(tot, 1)));
  return p;
}

XPeers peers_layout(const rgpu_ctx* c, const int64_t* cap, const std::vector<int64_t>& xoff, const int64_t* cnt) {
  XPeers L;
  L.np = c->nparts;
  L.me = c->part;
  int64_t o = 0, p = 0;
  for (int q = 0; q < c->nparts; q++) {
    L.base[q] = o;
    L.cap[q] = cap[q];
    o += cap[q];
    L.pre[q] = p;
    p += cnt ? (q == c->part ? 0 : cnt[q]) : 0;
    L.xoff[q] = xoff[q];
  }
  L.pre[c->nparts] = p;
  L.xoff[c->nparts] = xoff[c->nparts];
  return L;
}

void free_part_slots(rgpu_ctx* c, bool keep_channels) {
  for (XSlot& xs : c->pt.xs) {
    for (void* p : {(void*)xs.su, (void*)xs.sm, (void*)xs.ru[0], (void*)xs.ru[1], (void*)xs.rm[0], (void*)xs.rm[1],
                    (void*)xs.hsbuf, (void*)xs.hrbuf, (void*)xs.ccnt, (void*)xs.coff, xs.scan_tmp, (void*)xs.pmask,
                    (void*)xs.gcut})
      if (p) (void)hipFree(p);
    if (xs.h_xab) (void)hipHostFree(xs.h_xab);
    Exchange* x = xs.x;
    if (!keep_channels) delete x;
    xs = XSlot();
    if (keep_channels) xs.x = x;
  }
}

void drop_alloc(std::vector<void*>& L, void* p);
int sync_vid(rgpu_ctx* c);
// The broadcast records' receive tables (once per sealed graph; collective): every partition's
// boundary count, and for every receive entry the sender's boundary index of its vertex (the
// send plans are aligned: entry e of q's list for us is our receive entry xr_off[q] + e).
void ensure_tab(rgpu_ctx* c) {
  Part& X = c->pt;
  if (X.tab_ready) return;
  const int P = c->nparts, me = c->part;
  hipStream_t st = c->slot[0].stream;
  auto& LG = c->graph_allocs;
  std::vector<void*> T;
  try {
    // every partition's boundary count, whether its graph holds a vertex death, and whether it
    // lacks time-ordered slots (4 nb + 2 no-tslots + deaths): ghost_vm_free must decide the same on
    // every partition, and build_tslots leaves ts_t null on a partition without edges (or past
    // int32 slot words)
    int64_t* d = dalloc<int64_t>(T, 2 * P);
    std::vector<int64_t> h(2 * P, 4 * X.xsend.nb + (c->g.ts_t ? 0 : 2) + (c->st.deaths > 0 ? 1 : 0));
    HIPCHK(hipMemcpy(d, h.data(), sizeof(int64_t) * P, hipMemcpyHostToDevice));
    X.xchg->alltoall_i64(d, d + P, 1, st);
    HIPCHK(hipMemcpyAsync(h.data(), d, sizeof(int64_t) * 2 * P, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    int64_t o = 0;
    X.no_deaths = c->st.deaths == 0;
    X.all_tslots = c->g.ts_t != nullptr;
    for (int q = 0; q < P; q++) {
      if (q != me && (h[P + q] & 1)) X.no_deaths = false;
      if (q != me && (h[P + q] & 2)) X.all_tslots = false;
      X.nbq[q] = q == me ? 0 : h[P + q] >> 2;
      X.tab.toff[q] = o;
      o += X.nbq[q];
    }
    X.tab.toff[P] = o;
    drop_alloc(LG, X.tab.tab);  // (a rebuild after a seal that kept the graph)
    X.tab.tab = dalloc<int32_t>(LG, std::max<int64_t>(o, 1));
    HIPCHK(hipMemsetAsync(X.tab.tab, 0xff, sizeof(int32_t) * std::max<int64_t>(o, 1), st));
    int32_t* tmp = dalloc<int32_t>(T, std::max<int64_t>(X.nxr, 1));
    std::vector<void*> sp(P), rp(P);
    std::vector<size_t> sb(P), rb(P);
    for (int q = 0; q < P; q++) {
      sp[q] = (void*)(X.xsend.eb ? X.xsend.eb + X.xs_off[q] : nullptr);
      rp[q] = tmp + X.xr_off[q];
      sb[q] = q == me ? 0 : sizeof(int32_t) * (size_t)(X.xs_off[q + 1] - X.xs_off[q]);
      rb[q] = q == me ? 0 : sizeof(int32_t) * (size_t)(X.xr_off[q + 1] - X.xr_off[q]);
    }
    X.xchg->sendrecv(sp.data(), sb.data(), rp.data(), rb.data(), st);
    unsigned long long* err = dalloc<unsigned long long>(T, 1);
    HIPCHK(hipMemsetAsync(err, 0, sizeof(unsigned long long), st));
    launch_xtab_fill(st, X.nxr, X.xr_v, X.xr_q, tmp, X.tab, err);
    HIPCHK(hipGetLastError());
    unsigned long long herr = 0;
    HIPCHK(hipMemcpyAsync(&herr, err, sizeof(herr), hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    if (herr) throw HipFail{"exchange plan: " + std::to_string(herr) + " receive entries name no boundary vertex of their sender"};
    // ghost -> owning partition, Utils.getPartition (K2's peer masks: whom an owned vertex's records go to)
    if (sync_vid(c) != RGPU_OK) throw HipFail{"exchange plan: vertex ids"};
    const int64_t ng = c->g.nv - c->pk.n_own;
    std::vector<uint8_t> gp((size_t)std::max<int64_t>(ng, 1), 0);
    for (int64_t k = 0; k < ng; k++) {
      const int64_t id = c->pk.vid[(size_t)(c->pk.n_own + k)];
      gp[(size_t)k] = (uint8_t)(((id < 0 ? -id : id) % (10 * (int64_t)P)) / 10);
    }
    drop_alloc(LG, X.gpeer);
    X.gpeer = dalloc<uint8_t>(LG, gp.size());
    HIPCHK(hipMemcpy(X.gpeer, gp.data(), gp.size(), hipMemcpyHostToDevice));
  } catch (...) {
    for (void* p : T) (void)hipFree(p);
    throw;
  }
  for (void* p : T) (void)hipFree(p);
  X.tab_ready = true;
}

// the M send regions: P of xs.smcap records each (peer q's at q * smcap), at least `need` each
void grow_sm(XSlot& xs, int P, int64_t need, hipStream_t s) {
  if (xs.sm && need <= xs.smcap) return;
  HIPCHK(hipStreamSynchronize(s));
  if (xs.sm) HIPCHK(hipFree(xs.sm));
  xs.sm = nullptr;
  xs.smcap = std::max(xs.smcap, need + need / 2 + g_xrec_slack);
  HIPCHK(hipMalloc((void**)&xs.sm, sizeof(XRec) * (size_t)xs.smcap * P));
}

void ensure_part(rgpu_ctx* c, int nuse, int planes) {
  Part& X = c->pt;
  const int P = c->nparts;
  auto& LG = c->graph_allocs;
  ensure_tab(c);
  if (!X.own.err) X.own.err = dalloc<unsigned long long>(LG, 1);  // (goes with the graph: apply_merged / free_graph)
  HIPCHK(hipMemset(X.own.err, 0, sizeof(unsigned long long)));
  for (int i = 0; i < nuse; i++) {
    XSlot& xs = X.xs[i];
    if (!xs.x) xs.x = X.xchg->fork(i + 1);  // collective: every partition forks the same slots
    if (!xs.err) {
      xs.err = dalloc<unsigned long long>(LG, 1);
      xs.mfin = dalloc<unsigned long long>(LG, 64);
      xs.fin_g = dalloc<unsigned int>(LG, 64 * 64);
      HIPCHK(hipMemset(xs.fin_g, 0, sizeof(unsigned int) * 64 * 64));
      xs.htot = dalloc<unsigned long long>(LG, kMaxParts);
      HIPCHK(hipMemset(xs.htot, 0, sizeof(unsigned long long) * kMaxParts));
      xs.xab = dalloc<int64_t>(LG, 8 * P);
      HIPCHK(hipHostMalloc((void**)&xs.h_xab, sizeof(int64_t) * 8 * P));
    }
    HIPCHK(hipMemset(xs.err, 0, sizeof(unsigned long long)));
    if (xs.vm_planes < planes) {
      xs.vms = dalloc<uint64_t>(LG, (size_t)planes * std::max<int64_t>(X.nxs, 1));
      xs.vmr = dalloc<uint64_t>(LG, (size_t)planes * std::max<int64_t>(X.nxr, 1));
      xs.vm_planes = planes;
    }
    if (xs.su_cap < X.xsend.nb || xs.ru_cap < X.tab.toff[P] || !xs.su) {
      // U records: worst case one per boundary vertex and peer, sent and received (sized by the
      // plan: no growth during a run, no host sizing)
      for (void* p : {(void*)xs.su, (void*)xs.ru[0], (void*)xs.ru[1], (void*)xs.ccnt, (void*)xs.coff, xs.scan_tmp,
                      (void*)xs.pmask, (void*)xs.gcut})
        if (p) HIPCHK(hipFree(p));
      xs.su_cap = std::max<int64_t>(X.xsend.nb, 1);
      xs.ru_cap = std::max<int64_t>(X.tab.toff[P], 1);
      HIPCHK(hipMalloc((void**)&xs.su, sizeof(unsigned long long) * (size_t)xs.su_cap * P));
      for (int p = 0; p < 2; p++) HIPCHK(hipMalloc((void**)&xs.ru[p], sizeof(unsigned long long) * (size_t)xs.ru_cap));
      // the pack's per-(peer, unit) counts and offsets (ccnt[P * units] stays 0)
      const int64_t no = c->pk.n_own;
      const size_t nck = (size_t)(xbc_units(no) * P + 1);
      HIPCHK(hipMalloc((void**)&xs.ccnt, sizeof(unsigned long long) * nck));
      HIPCHK(hipMalloc((void**)&xs.coff, sizeof(unsigned long long) * nck));
      HIPCHK(hipMemset(xs.ccnt, 0, sizeof(unsigned long long) * nck));
      HIPCHK(hipMemset(xs.coff, 0, sizeof(unsigned long long) * nck));
      xs.scan_bytes = std::max<size_t>(xbc_scan_bytes(no, P), 16);
      HIPCHK(hipMalloc(&xs.scan_tmp, xs.scan_bytes));
      HIPCHK(hipMalloc((void**)&xs.pmask, (size_t)std::max<int64_t>(c->g.nv, 1)));
      HIPCHK(hipMalloc((void**)&xs.gcut, sizeof(int32_t) * (size_t)std::max<int64_t>(c->g.nv, 1)));
    }
    if (!xs.sm) {
      // M records: a first guess, grown on demand (both receive parities share one layout, xs.rmcap)
      int64_t nr[kMaxParts] = {};
      grow_sm(xs, P, g_xrec_init * X.xsend.nb / 16, nullptr);
      for (int q = 0; q < P; q++) nr[q] = g_xrec_init * X.nbq[q] / 16;
      grow_regions(&xs.rm[0], xs.rmcap, nr, P, nullptr);
      xs.rm[1] = alloc_regions<XRec>(xs.rmcap, P);
    }
  }
}

// CC runs whose views all have equal vertex and edge windows, on graphs where no partition holds a
// vertex death, read no ghost membership: every slot is nodeath, and its window bits imply both
// endpoints' membership (BatchParams::simple_ends).  The ghost rows are then set to every view
// (readers AND them with bits that imply them) and the exchange is skipped.  The same decision on
// every partition: the windows are the query's, no_deaths and all_tslots are agreed in ensure_tab
// (a partition's own ts_t is not: one without edges has none, and deciding on it alone would send
// that partition into a membership exchange its peers skip).
bool ghost_vm_free(const rgpu_ctx* c, const RunCfg& rc) {
  if (!c->partitioned || rc.algo != RGPU_ALGO_CC || !c->pt.no_deaths || !c->pt.all_tslots) return false;
  for (int w = 0; w < rc.W; w++)
    if (rc.thr_v[w] != rc.thr_e[w]) return false;
  return true;
}

// the boundary vertices' K1 membership words to the peers, theirs into our ghost rows
void part_vm_exchange(rgpu_ctx* c, int si, uint64_t* vm, int64_t vstride, int planes, bool free) {
  Slot& s = c->slot[si];
  Part& X = c->pt;
  XSlot& xs = X.xs[si];
  const int P = c->nparts, me = c->part;
  if (free) {
    const int64_t no = c->pk.n_own, ng = c->g.nv - no;
    for (int p = 0; p < planes && ng > 0; p++)
      HIPCHK(hipMemsetAsync(vm + (size_t)p * vstride + no, 0xff, sizeof(uint64_t) * (size_t)ng, s.stream));
    return;
  }
  timed_launch(c, si, KID_XCHG, 0.0, [&] { launch_xvm_pack(s.stream, X.nxs, X.xs_v, X.xs_q, X.xs_off_d, planes, vm, vstride, xs.vms); });
  HIPCHK(hipGetLastError());
  std::vector<void*> sp(P), rp(P);
  std::vector<size_t> sb(P), rb(P);
  for (int q = 0; q < P; q++) {
    sp[q] = xs.vms + planes * X.xs_off[q];
    rp[q] = xs.vmr + planes * X.xr_off[q];
    sb[q] = q == me ? 0 : sizeof(uint64_t) * planes * (size_t)(X.xs_off[q + 1] - X.xs_off[q]);
    rb[q] = q == me ? 0 : sizeof(uint64_t) * planes * (size_t)(X.xr_off[q + 1] - X.xr_off[q]);
    xs.bytes[0] += (double)sb[q];
  }
  xs.x->sendrecv(sp.data(), sb.data(), rp.data(), rb.data(), s.stream);
  timed_launch(c, si, KID_XCHG, 0.0, [&] { launch_xvm_unpack(s.stream, X.nxr, X.xr_v, X.xr_q, X.xr_off_d, planes, xs.vmr, vm, vstride); });
  HIPCHK(hipGetLastError());
}

// The final-label skip across partitions: K2 left this partition's per-view minimum member labels
// in mneg; the minimum over every partition is the view's (a member holding it in all its views is
// final everywhere).  Collective on the slot's channel, at the same point on every partition.
void part_min_labels(rgpu_ctx* c, int si) {
  Slot& s = c->slot[si];
  XSlot& xs = c->pt.xs[si];
  int32_t* mn = min_labels(c, s);
  if (!mn) return;
  launch_min_fold(s.stream, mn, xs.mfin);
  xs.x->allreduce_u64(xs.mfin, 64, true, s.stream);
  launch_min_store(s.stream, xs.mfin, mn);
  HIPCHK(hipGetLastError());
}

// the label records of superstep r for every peer (U into xs.su, M into xs.sm, peer q's regions),
// from the step's changed bits and K2's peer masks.  write_only: the offsets of the last pack are
// current (a repack into larger M regions)
XBcIn bc_in(const rgpu_ctx* c, const XSlot& xs, int par);
// (clear: the count pass also clears the ghosts that step r-2's records set in parity r & 1 — the
// k_xbc_clear launch folded in; step r-1 has read those words, step r's apply comes after)
void part_pack(rgpu_ctx* c, int si, int r, bool write_only = false) {
  Slot& s = c->slot[si];
  Part& X = c->pt;
  XSlot& xs = X.xs[si];
  const int par = r & 1;
  const XBcIn clr = bc_in(c, xs, par);
  timed_launch(c, si, KID_XPACK, 0.0, [&] {
    launch_xbc_pack(s.stream, c->pk.n_own, c->nparts, X.xsend, chg_bits(c, s, r).next, s.chg[r & 1], s.vadj,
                    s.lab[r & 1], s.uw[r & 1], xs.pmask, xs.su, xs.su_cap, xs.sm, xs.smcap, xs.ccnt, xs.coff,
                    xs.scan_tmp, xs.scan_bytes, write_only, write_only ? nullptr : &clr, s.chg[par], s.uw[par]);
  });
}

// a received broadcast of parity par: regions and record counts (xchg.hip XBcIn)
XBcIn bc_in(const rgpu_ctx* c, const XSlot& xs, int par) {
  XBcIn I;
  const int P = c->nparts;
  I.U.np = I.M.np = P;
  I.U.me = I.M.me = c->part;
  int64_t bu = 0, bm = 0, pu = 0, pm = 0;
  for (int q = 0; q < P; q++) {
    I.U.base[q] = bu;
    I.U.cap[q] = c->pt.nbq[q];
    bu += c->pt.nbq[q];
    I.U.pre[q] = pu;
    pu += xs.rucnt[par][q];
    I.M.base[q] = bm;
    I.M.cap[q] = xs.rmcap[q];
    bm += xs.rmcap[q];
    I.M.pre[q] = pm;
    pm += xs.rmcnt[par][q];
  }
  I.U.pre[P] = pu;
  I.M.pre[P] = pm;
  I.ru = xs.ru[par];
  I.rm = xs.rm[par];
  I.T = c->pt.tab;
  I.n_own = c->pk.n_own;
  I.nv = c->g.nv;
  I.err = xs.err;
  return I;
}

// after superstep r: pack its boundary records and exchange the counts; the host picks the
// slot up in part_after_counts
void part_post_step(rgpu_ctx* c, int si, const RunCfg& rc, int r) {
  Slot& s = c->slot[si];
  Part& X = c->pt;
  XSlot& xs = X.xs[si];
  const int P = c->nparts;
  xs.r = r;
  s.r_launched = r;
  if (r >= rc.max_steps) {  // the cap (AnalysisTask.endStep :214): no superstep reads step r's news
    s.r_final = r;
    part_finish_begin(c, si, rc);
    return;
  }
  part_pack(c, si, r);
  launch_xbc_counts(s.stream, P, c->part, X.xsend.nb > 0 ? xs.coff : nullptr, xbc_units(c->pk.n_own), s.stepcnt + r,
                    xs.xab);
  HIPCHK(hipGetLastError());
  xs.x->alltoall_i64(xs.xab, xs.xab + 4 * P, 4, s.stream);
  HIPCHK(hipMemcpyAsync(xs.h_xab, xs.xab, sizeof(int64_t) * 8 * P, hipMemcpyDeviceToHost, s.stream));
  HIPCHK(hipEventRecord(s.ev, s.stream));
  s.phase = 1;
}

void part_after_counts(rgpu_ctx* c, int si, const RunCfg& rc) {
  Slot& s = c->slot[si];
  Part& X = c->pt;
  XSlot& xs = X.xs[si];
  const DevGraph& g = c->g;
  const int P = c->nparts, me = c->part, r = xs.r;
  // record counts per peer and the vote (xregions.hpp; the region arithmetic is CPU-tested)
  XferPlan xp;
  {
    const std::string e = xfer_counts(P, me, xs.h_xab, xs.h_xab + 4 * P, X.nbq, &xp);
    if (!e.empty()) throw HipFail{e};
  }
  const int64_t* recv_u = xp.recv_u;
  const int64_t* recv_m = xp.recv_m;
  if (xp.max_m > xs.smcap) {  // the counts were exact; the M records did not all fit: pack again, larger
    grow_sm(xs, P, xp.max_m, s.stream);
    part_pack(c, si, r, true);
  }
  if (!xp.any) {  // every partition voted to halt
    s.r_final = r;
    part_finish_begin(c, si, rc);
    return;
  }
  const int par = r & 1;
  // ghosts whose words records of step r-2 set (their records are still in ru / rm [par]): their
  // words go quiet and the M records' change words are cleared, so that this parity holds only
  // step r's news (an M record ORs its views into the change word; hub marking reads a ghost hub's
  // word and change word as this step's).
  // (the ghosts of step r-2's records, in this parity, were cleared by this step's pack: part_pack)
  bool rover = false;
  for (int q = 0; q < P; q++) rover |= recv_m[q] > xs.rmcap[q];
  if (rover) {  // a larger M layout for both parities; the other parity's records of step r-1 are
                // read once more (their clear, two supersteps from now), so they move over
    int64_t old_cap[kMaxParts];
    std::copy(xs.rmcap, xs.rmcap + kMaxParts, old_cap);
    grow_regions(&xs.rm[par], xs.rmcap, recv_m, P, s.stream);  // syncs: the clear above has run
    XRec* nb = alloc_regions<XRec>(xs.rmcap, P);
    int64_t o_old = 0, o_new = 0;
    for (int q = 0; q < P; q++) {
      if (xs.rmcnt[par ^ 1][q])
        HIPCHK(hipMemcpyAsync(nb + o_new, xs.rm[par ^ 1] + o_old, sizeof(XRec) * xs.rmcnt[par ^ 1][q],
                              hipMemcpyDeviceToDevice, s.stream));
      o_old += old_cap[q];
      o_new += xs.rmcap[q];
    }
    HIPCHK(hipStreamSynchronize(s.stream));
    HIPCHK(hipFree(xs.rm[par ^ 1]));
    xs.rm[par ^ 1] = nb;
  }
  std::copy(recv_u, recv_u + kMaxParts, xs.rucnt[par]);
  std::copy(recv_m, recv_m + kMaxParts, xs.rmcnt[par]);
  if (!c->trace_path.empty()) {  // trace: step 1000 + r = the label records received after superstep r (U, M)
    unsigned long long tu = 0, tm = 0;
    for (int q = 0; q < P; q++) tu += recv_u[q], tm += recv_m[q];
    c->steprec.push_back({s.batch, 1000 + r, tu, tm, 0, 0});
  }
  const XBcIn in = bc_in(c, xs, par);
  {
    int64_t rm_alloc = 0;
    for (int q = 0; q < P; q++) rm_alloc += xs.rmcap[q];  // (grow_regions / alloc_regions: sum of the caps)
    const std::string e = xfer_layout(&xp, X.nbq, xs.su_cap, xs.smcap, xs.rmcap, xs.su_cap * P, xs.smcap * P,
                                      xs.ru_cap, rm_alloc);
    if (!e.empty()) throw HipFail{e};
  }
  {  // the broadcast: our U list and M list to every peer, theirs into their regions
    std::vector<void*> sp(P), rp(P);
    std::vector<size_t> sb(P), rb(P);
    for (int q = 0; q < P; q++) {
      sp[q] = xs.su + xp.su_off[q];
      rp[q] = xs.ru[par] + xp.ru_off[q];
      sb[q] = q == me ? 0 : sizeof(unsigned long long) * (size_t)xp.sent_u[q];
      rb[q] = q == me ? 0 : sizeof(unsigned long long) * (size_t)recv_u[q];
      xs.bytes[1] += (double)sb[q];
    }
    xs.x->sendrecv(sp.data(), sb.data(), rp.data(), rb.data(), s.stream);
    for (int q = 0; q < P; q++) {
      sp[q] = xs.sm + xp.sm_off[q];
      rp[q] = xs.rm[par] + xp.rm_off[q];
      sb[q] = q == me ? 0 : sizeof(XRec) * (size_t)xp.sent_m[q];
      rb[q] = q == me ? 0 : sizeof(XRec) * (size_t)recv_m[q];
      xs.bytes[1] += (double)sb[q];
    }
    xs.x->sendrecv(sp.data(), sb.data(), rp.data(), rb.data(), s.stream);
  }
  if (c->inject_rec)  // fault injection (tests): one received U record names no boundary vertex
    for (int q = 0; q < P; q++)
      if (recv_u[q]) {
        HIPCHK(hipMemsetAsync((char*)(xs.ru[par] + in.U.base[q]) + 4, 0xff, 4, s.stream));
        c->inject_rec = false;
        break;
      }
  timed_launch(c, si, KID_XMARK, 0.0, [&] {
    launch_xbc_apply(s.stream, in, s.lab[par], s.chg[par], s.uw[par], chg_bits(c, s, r).next, g, s.vm, s.em,
                     s.act[(r + 1) % 3], s.tcut, s.iem ? &s.ebp : nullptr, s.ccount, dense_div(c), r, xs.gcut);
  });
  // the vote is global: superstep r+1 runs here even if nothing changed here
  HIPCHK(hipMemsetD32Async((hipDeviceptr_t)(s.stepcnt + r), 1, 1, s.stream));
  const bool hv = g.n_seg > 0;
  if (hv)  // neighbours of heavy vertices (owned ones visited in r, ghosts just received) that changed
    timed_launch(c, si, KID_HEAVY, 0.0, [&] {
      launch_heavy_mark(s.stream, g, s.snbr, s.smask, s.chg[par], s.act[(r + 1) % 3], s.stepcnt, r, s.hv,
                        r == 1 ? nullptr : s.act[r % 3], s.vm, s.em, s.tcut, s.ccount, dense_div(c), work_buf(c, s),
                        s.uw[par], c->ko);
    });
  HIPCHK(hipGetLastError());
  // superstep r+1 over the owned vertices
  const int n = r + 1;
  const DevGraph go = owned_view(c);
  if (hv)
    timed_launch(c, si, KID_HEAVY, 0.0, [&] {
      launch_heavy_gather(s.stream, g, s.snbr, s.smask, s.lab[r & 1], s.chg[r & 1], s.act[n % 3], s.stepcnt, n, s.hv,
                          s.uw[r & 1], chg_bits(c, s, n).prev, s.ccount, dense_div(c), work_buf(c, s), s.vm,
                          min_labels(c, s), c->ko);
    });
  timed_launch(c, si, KID_STEP, 0.0, [&] {
    launch_cc_step(s.stream, n, go, s.vm, s.cnt, s.snbr, s.smask, s.lab[r & 1], s.lab[n & 1], s.chg[r & 1],
                   s.chg[n & 1], s.act[n % 3], s.act[(n + 1) % 3], s.act[(n + 2) % 3], s.stepcnt, nullptr,
                   work_buf(c, s), s.stats + kLaneOff, hv ? s.hv.best : nullptr,
                   s.uw[r & 1], s.uw[n & 1], chg_bits(c, s, n), s.ccount,
                   dense_div(c), min_labels(c, s), s.long_views, c->ko);
  }, n);
  part_post_step(c, si, rc, n);
}

// component counts: label -> count of owned members at the label's count row when the label is
// owned here, the others routed to their owner as records (k_part_count); their counts travel,
// the host picks the slot up in part_finish_end
void part_finish_begin(rgpu_ctx* c, int si, const RunCfg& rc) {
  Slot& s = c->slot[si];
  Part& X = c->pt;
  XSlot& xs = X.xs[si];
  const int P = c->nparts;
  const int nviews = rc.K * rc.gsize;
  const int64_t no = c->pk.n_own;
  if (!xs.hsbuf) {  // first guess: 1/16 record per owned vertex and peer (the LDS cache folds most)
    int64_t need[kMaxParts];
    for (int q = 0; q < P; q++) need[q] = no / 16;
    grow_regions(&xs.hsbuf, xs.hscap, need, P, s.stream);
  }
  const int32_t* uw = s.uw[s.r_final & 1];
  if (uw && (rc.flags & RGPU_RUN_RETAIN))  // full rows of the owned vertices for the host
    launch_uw_rows(s.stream, no, s.vm, uw, s.lab[s.r_final & 1]);
  const XPeers L = peers_layout(c, xs.hscap, X.xs_off, nullptr);
  timed_launch(c, si, KID_HIST, 28.0 * no, [&] {
    launch_part_count(s.stream, false, L, X.own, nviews, s.vm, s.vadj, uw, s.lab[s.r_final & 1], s.counts, s.iso,
                      xs.htot, xs.hsbuf, min_labels(c, s), xs.fin_g);
  });
  launch_xcounts(s.stream, P, c->part, xs.htot, xs.xab);
  HIPCHK(hipGetLastError());
  xs.x->alltoall_i64(xs.xab, xs.xab + 2 * P, 2, s.stream);
  HIPCHK(hipMemcpyAsync(xs.h_xab, xs.xab, sizeof(int64_t) * 4 * P, hipMemcpyDeviceToHost, s.stream));
  HIPCHK(hipEventRecord(s.ev, s.stream));
  s.phase = 3;
}

void part_finish_end(rgpu_ctx* c, int si, const RunCfg& rc) {
  Slot& s = c->slot[si];
  Part& X = c->pt;
  XSlot& xs = X.xs[si];
  const int P = c->nparts, me = c->part;
  const int nviews = rc.K * rc.gsize;
  const int64_t no = c->pk.n_own;
  int64_t sent[kMaxParts] = {}, recv[kMaxParts] = {};
  bool over = false;
  for (int q = 0; q < P; q++) {
    sent[q] = q == me ? 0 : xs.h_xab[2 * q];
    recv[q] = q == me ? 0 : xs.h_xab[2 * P + 2 * q];
    over |= sent[q] > xs.hscap[q];
  }
  const int32_t* uw = s.uw[s.r_final & 1];
  if (over) {  // the records again into a larger buffer (the local counts are done); the LDS cache
               // may fold them differently, but the sums per (label, view) are the same
    HIPCHK(hipMemsetAsync(xs.htot, 0, sizeof(unsigned long long) * kMaxParts, s.stream));
    grow_regions(&xs.hsbuf, xs.hscap, sent, P, s.stream);
    const XPeers L = peers_layout(c, xs.hscap, X.xs_off, nullptr);
    launch_part_count(s.stream, true, L, X.own, nviews, s.vm, s.vadj, uw, s.lab[s.r_final & 1], s.counts, s.iso,
                      xs.htot, xs.hsbuf, min_labels(c, s), xs.fin_g);
    HIPCHK(hipMemcpyAsync(xs.h_xab, xs.htot, sizeof(int64_t) * P, hipMemcpyDeviceToHost, s.stream));
    HIPCHK(hipStreamSynchronize(s.stream));
    for (int q = 0; q < P; q++)
      if (q != me && xs.h_xab[q] != sent[q])
        throw HipFail{"component-count records: second pass sent " + std::to_string(xs.h_xab[q]) + " to peer " +
                      std::to_string(q) + ", the counts exchange announced " + std::to_string(sent[q])};
    HIPCHK(hipMemsetAsync(xs.htot, 0, sizeof(unsigned long long) * kMaxParts, s.stream));
  }
  grow_regions(&xs.hrbuf, xs.hrcap, recv, P, s.stream);
  if (!c->trace_path.empty()) {  // trace: step -1 = the batch's count records (pv sent, ps received)
    unsigned long long ts = 0, tr = 0;
    for (int q = 0; q < P; q++) ts += sent[q], tr += recv[q];
    c->steprec.push_back({s.batch, -1, ts, tr, 0, 0});
  }
  {
    const XPeers Ls = peers_layout(c, xs.hscap, X.xs_off, nullptr);
    const XPeers Lr = peers_layout(c, xs.hrcap, X.xr_off, nullptr);
    std::vector<void*> sp(P), rp(P);
    std::vector<size_t> sb(P), rb(P);
    for (int q = 0; q < P; q++) {
      sp[q] = xs.hsbuf + Ls.base[q];
      rp[q] = xs.hrbuf + Lr.base[q];
      sb[q] = sizeof(XRec) * (size_t)sent[q];
      rb[q] = sizeof(XRec) * (size_t)recv[q];
      xs.bytes[2] += (double)sb[q];
    }
    xs.x->sendrecv(sp.data(), sb.data(), rp.data(), rb.data(), s.stream);
  }
  if (c->inject_cnt)  // fault injection (tests): one received count record names a label that getPartition
                      // routes here but no owned vertex holds (above every owned id)
    for (int q = 0; q < P; q++)
      if (recv[q]) {
        const int64_t m = 10 * (int64_t)P;
        const int32_t bad = (int32_t)(((int64_t)INT32_MAX - m) / m * m + 10 * me);
        HIPCHK(hipMemcpyAsync(xs.hrbuf + peers_layout(c, xs.hrcap, X.xr_off, recv).base[q], &bad, sizeof(bad),
                              hipMemcpyHostToDevice, s.stream));
        HIPCHK(hipStreamSynchronize(s.stream));  // (&bad is a stack word)
        c->inject_cnt = false;
        break;
      }
  timed_launch(c, si, KID_XCHG, 0.0, [&] { launch_hist_recv(s.stream, peers_layout(c, xs.hrcap, X.xr_off, recv), xs.hrbuf, X.own, s.counts); });
  // the minimum label's members, counted on every partition (k_part_count): summed, added by its owner
  launch_min_count_fold(s.stream, xs.fin_g, xs.mfin);
  xs.x->allreduce_u64(xs.mfin, 64, false, s.stream);
  launch_min_count_add(s.stream, xs.mfin, min_labels(c, s), X.own, P, me, s.counts);
  HIPCHK(hipGetLastError());
  // roots: every owned member whose label is its own id reads (and zeroes) its count row
  timed_launch(c, si, KID_SUMMARY, 20.0 * no, [&] {
    launch_cc_roots(s.stream, no, nviews, s.vm, s.vadj, uw, s.lab[s.r_final & 1], s.counts, s.stats, s.iso,
                    s.r_final >= 1 && s.r_final >= rc.max_steps, c->g.grank, true);
  });
  // processBatchWindowResults merges the shards: biggest = max, the other fields add up
  xs.x->allreduce_u64(s.stats, kViews, true, s.stream);
  xs.x->allreduce_u64(s.stats + kViews, 5 * kViews, false, s.stream);
  // the batch's ghost change words back to zero (the next batch's ghosts start clean)
  for (int par = 0; par < 2; par++) {
    timed_launch(c, si, KID_XUNPACK, 0.0, [&] { launch_xbc_clear(s.stream, bc_in(c, xs, par), s.chg[par], s.uw[par]); });
    std::fill(xs.rucnt[par], xs.rucnt[par] + kMaxParts, 0);
    std::fill(xs.rmcnt[par], xs.rmcnt[par] + kMaxParts, 0);
  }
  HIPCHK(hipGetLastError());
  finish_tail(c, si, rc);
}

void wait_event(hipEvent_t e) {
  for (;;) {
    const hipError_t q = hipEventQuery(e);
    if (q == hipSuccess) return;
    if (q != hipErrorNotReady) HIPCHK(q);
    __builtin_ia32_pause();
  }
}

int run_partitioned_cc(rgpu_ctx* c, RunCfg& rc) {
  const size_t nb = rc.nb;
  c->st.views += (int64_t)(rc.n_hops * rc.W);
  c->st.batches += (int64_t)nb;
  const int nslots = run_slots(c, rc);
  size_t next = 0;
  for (;;) {  // fixed round robin over the slots (identical collective order on every partition)
    bool busy = false;
    for (int si = 0; si < nslots; si++) {
      Slot& s = c->slot[si];
      if (s.phase == 0) {
        if (next < nb && can_start(c, next, rc)) {
          start_batch(c, si, (int)next++, rc);
          busy = true;
        }
        continue;
      }
      busy = true;
      wait_event(s.ev);
      if (s.phase == 1) part_after_counts(c, si, rc);
      else if (s.phase == 3) part_finish_end(c, si, rc);
      else harvest(c, si, rc);
    }
    if (!busy) break;
  }
  return 0;
}

void pr_exchange(rgpu_ctx* c, double* contrib) {
  Slot& s = c->slot[0];
  Part& X = c->pt;
  Exchange* x = X.xs[0].x;
  const int P = c->nparts, me = c->part;
  launch_xgather_f64(s.stream, X.nxs, X.xs_v, contrib, X.sbuf_f);
  HIPCHK(hipGetLastError());
  std::vector<void*> sp(P), rp(P);
  std::vector<size_t> sb(P), rb(P);
  for (int q = 0; q < P; q++) {
    sp[q] = X.sbuf_f + X.xs_off[q] * kViews;
    rp[q] = X.rbuf_f + X.xr_off[q] * kViews;
    sb[q] = q == me ? 0 : (size_t)(X.xs_off[q + 1] - X.xs_off[q]) * kViews * 8;
    rb[q] = q == me ? 0 : (size_t)(X.xr_off[q + 1] - X.xr_off[q]) * kViews * 8;
    X.bytes_sent += (double)sb[q];
  }
  x->sendrecv(sp.data(), sb.data(), rp.data(), rb.data(), s.stream);
  launch_xscatter_f64(s.stream, X.nxr, X.xr_v, X.rbuf_f, contrib);
  HIPCHK(hipGetLastError());
}

// DegreeBasic / PageRank, one hop-major batch at a time on slot 0
int run_partitioned_dp(rgpu_ctx* c, RunCfg& rc) {
  const size_t nb = rc.nb;  // hop-major (G = 1)
  c->st.views += (int64_t)(rc.n_hops * rc.W);
  c->st.batches += (int64_t)nb;
  Slot& s = c->slot[0];
  const DevGraph go = owned_view(c);
  const DevGraph& g = c->g;
  for (size_t b = 0; b < nb; b++) {
    BatchParams bp;
    std::memset(&bp, 0, sizeof(bp));
    const size_t h0 = b * rc.K;
    bp.K = (int)std::min<size_t>(rc.K, rc.n_hops - h0);
    bp.W = rc.W;
    bp.KS = rc.K;
    bp.sorted = 1;
    bp.iv_max = c->iv_max;
    for (int k = 0; k < bp.K; k++) {
      bp.hop[k] = rc.hops[h0 + k];
      if (k > 0 && bp.hop[k] < bp.hop[k - 1]) bp.sorted = 0;
    }
    bp.jump = even_jump(bp);
    for (int w = 0; w < rc.W; w++) { bp.thr_v[w] = rc.thr_v[w]; bp.thr_e[w] = rc.thr_e[w]; }
    s.batch = (int)b;
    s.kb = bp.K;
    s.r_final = 0;
    BatchClear clr;
    clr.stats = s.stats;
    clr.n_stats = kStatCopy;
    clr.flags = s.stepcnt;
    clr.n_flags = kMaxSteps;
    s.vm = s.vm_own;
    s.em = s.em_own;
    timed_launch(c, 0, KID_MASK, 8.0 * (go.nv + 1) + 16.0 * go.nv + 8.0 * go.nv,
                 [&] { launch_vertex_mask(s.stream, go, bp, s.vm, 0, false, clr); });
    timed_launch(c, 0, KID_EMASK, bytes_emask(c, 1, false),
                 [&] { launch_edge_mask(s.stream, g, bp, s.em, false, c->d_ecnt, (int64_t)h0); });
    part_vm_exchange(c, 0, s.vm, 0, 1, false);
    timed_launch(c, 0, KID_DEGREE, go.nv * (8.0 + 32.0 + 512.0) + (double)(g.ne + g.n_in) * 12.0, [&] {
      launch_degree(s.stream, go, s.vm, s.em, s.outdeg, s.indeg, s.stats, rc.algo == RGPU_ALGO_DEGREE ? &s.top : nullptr);
    });
    if (rc.algo == RGPU_ALGO_PR) {
      timed_launch(c, 0, KID_SLOTS, go.nv * (8.0 + 24.0 + 256.0 + 1024.0) + (double)(g.n_in) * 24.0, [&] {
        launch_pr_slots(s.stream, go, s.vm, s.em, s.outdeg, s.pcnt, s.psnbr, s.psmask, s.pr, s.contrib[0]);
      });
      pr_exchange(c, s.contrib[0]);
      for (int it = 0; it < rc.pr_iters; it++) {
        timed_launch(c, 0, KID_PR, go.nv * (8.0 + 16.0 + 4.0 + 256.0 + 1024.0) + (double)(g.n_in + go.nv) * 12.0, [&] {
          launch_pr_step(s.stream, go, s.vm, s.em, s.outdeg, s.pcnt, s.psnbr, s.psmask, s.contrib[it & 1],
                         s.contrib[(it + 1) & 1], s.pr, s.hv.pacc);
        });
        if (it + 1 < rc.pr_iters) pr_exchange(c, s.contrib[(it + 1) & 1]);
      }
    }
    finish_tail(c, 0, rc);
    HIPCHK(hipStreamSynchronize(s.stream));
    harvest(c, 0, rc);
  }
  return 0;
}

// Generic vertex programs across partitions (VertexVisitor messages cross
// Partition Managers through the mediator, VertexVisitor.scala:99-147), one hop-major batch at a
// time on slot 0.  Setup on every local rank; then, after the setup and after every superstep over
// the owned vertices, each owned boundary vertex's record (its state row and change word) goes to
// the peers that hold it as a ghost — the exchange plan's lists, fixed sizes, so no counts round —
// and the global vote: an all-reduce of the step's per-view change flags, the next superstep
// running everywhere while any partition changed a state (AnalysisTask.endStep :208-225).  A
// per_degree float program's degree rows go to the ghosts once per batch (a ghost's message
// targets live on its owner).
int run_partitioned_vp(rgpu_ctx* c, RunCfg& rc) {
  const size_t nb = rc.nb;  // hop-major (G = 1)
  c->st.views += (int64_t)(rc.n_hops * rc.W);
  c->st.batches += (int64_t)nb;
  Slot& s = c->slot[0];
  const DevGraph go = owned_view(c);
  const DevGraph& g = c->g;
  Part& X = c->pt;
  Exchange* x = X.xs[0].x;
  const int P = c->nparts, me = c->part;
  std::vector<void*> T;
  try {
    int64_t* sbuf = dalloc<int64_t>(T, (size_t)std::max<int64_t>(X.nxs, 1) * kVpRec);
    int64_t* rbuf = dalloc<int64_t>(T, (size_t)std::max<int64_t>(X.nxr, 1) * kVpRec);
    const bool degx = c->vp.fsum && c->vp.per_degree;
    int32_t* sdeg = degx ? dalloc<int32_t>(T, (size_t)std::max<int64_t>(X.nxs, 1) * kViews) : nullptr;
    int32_t* rdeg = degx ? dalloc<int32_t>(T, (size_t)std::max<int64_t>(X.nxr, 1) * kViews) : nullptr;
    unsigned long long* vw = dalloc<unsigned long long>(T, kViews);
    int32_t flag = 0;
    auto sendrecv = [&](void* sb0, void* rb0, size_t bytes_per_entry, int kind) {
      std::vector<void*> sp(P), rp(P);
      std::vector<size_t> sb(P), rb(P);
      for (int q = 0; q < P; q++) {
        sp[q] = (char*)sb0 + bytes_per_entry * X.xs_off[q];
        rp[q] = (char*)rb0 + bytes_per_entry * X.xr_off[q];
        sb[q] = q == me ? 0 : bytes_per_entry * (size_t)(X.xs_off[q + 1] - X.xs_off[q]);
        rb[q] = q == me ? 0 : bytes_per_entry * (size_t)(X.xr_off[q + 1] - X.xr_off[q]);
        X.xs[0].bytes[kind] += (double)sb[q];
      }
      x->sendrecv(sp.data(), sb.data(), rp.data(), rb.data(), s.stream);
    };
    auto records = [&](int par) {  // owned boundary rows of buffer par -> the peers' ghost rows
      timed_launch(c, 0, KID_XCHG, 0.0, [&] { launch_vp_xgather(s.stream, X.nxs, X.xs_v, s.vst[par], s.chg[par], sbuf); });
      sendrecv(sbuf, rbuf, sizeof(int64_t) * kVpRec, 1);
      timed_launch(c, 0, KID_XCHG, 0.0, [&] { launch_vp_xscatter(s.stream, X.nxr, X.xr_v, rbuf, s.vst[par], s.chg[par]); });
    };
    for (size_t b = 0; b < nb; b++) {
      BatchParams bp;
      std::memset(&bp, 0, sizeof(bp));
      const size_t h0 = b * rc.K;
      bp.K = (int)std::min<size_t>(rc.K, rc.n_hops - h0);
      bp.W = rc.W;
      bp.KS = rc.K;
      bp.sorted = 1;
      bp.iv_max = c->iv_max;
      for (int k = 0; k < bp.K; k++) {
        bp.hop[k] = rc.hops[h0 + k];
        if (k > 0 && bp.hop[k] < bp.hop[k - 1]) bp.sorted = 0;
      }
      bp.jump = even_jump(bp);
      for (int w = 0; w < rc.W; w++) { bp.thr_v[w] = rc.thr_v[w]; bp.thr_e[w] = rc.thr_e[w]; }
      s.batch = (int)b;
      s.kb = bp.K;
      s.r_final = 0;
      BatchClear clr;
      clr.stats = s.stats;
      clr.n_stats = kStatCopy;
      clr.flags = s.stepcnt;
      clr.n_flags = kMaxSteps;
      s.vm = s.vm_own;
      s.em = s.em_own;
      timed_launch(c, 0, KID_MASK, 8.0 * (go.nv + 1) + 16.0 * go.nv + 8.0 * go.nv,
                   [&] { launch_vertex_mask(s.stream, go, bp, s.vm, 0, false, clr); });
      timed_launch(c, 0, KID_EMASK, bytes_emask(c, 1, false),
                   [&] { launch_edge_mask(s.stream, g, bp, s.em, false, c->d_ecnt, (int64_t)h0); });
      part_vm_exchange(c, 0, s.vm, 0, 1, false);
      launch_vp_setup(s.stream, g, c->vp, c->d_vid, s.vm, s.em, s.cnt, s.snbr, s.smask, s.vst[0], s.chg[0], s.vdeg);
      HIPCHK(hipGetLastError());
      records(0);  // a ghost's setup state and sender flag are its owner's (a seed owned elsewhere)
      if (degx) {
        launch_vp_xgather_deg(s.stream, X.nxs, X.xs_v, s.vdeg, sdeg);
        sendrecv(sdeg, rdeg, sizeof(int32_t) * kViews, 1);
        launch_vp_xscatter_deg(s.stream, X.nxr, X.xr_v, rdeg, s.vdeg);
      }
      if (rc.max_steps > 1) {
        launch_vp_go(s.stream, s.stepcnt);
        for (int r = 1; r <= rc.max_steps; r++) {
          timed_launch(c, 0, KID_VP, 0.0, [&] {
            launch_vp_step(s.stream, r, go, c->vp, s.vm, s.cnt, s.snbr, s.smask, s.vst[(r - 1) & 1], s.vst[r & 1],
                           s.chg[(r - 1) & 1], s.chg[r & 1], s.stepcnt, nullptr, s.stats + kLaneOff, s.vdeg);
          });
          records(r & 1);
          launch_vp_lanes(s.stream, s.stats + kLaneOff, r, vw);
          x->allreduce_u64(vw, kViews, true, s.stream);
          launch_vp_vote(s.stream, vw, r, s.stepcnt, s.stats + kLaneOff);
          HIPCHK(hipGetLastError());
          HIPCHK(hipMemcpyAsync(&flag, s.stepcnt + r, sizeof(int32_t), hipMemcpyDeviceToHost, s.stream));
          HIPCHK(hipStreamSynchronize(s.stream));
          s.r_final = r;
          if (!flag) break;  // no partition changed a state in superstep r
        }
      }
      c->st.supersteps += s.r_final;
      finish_tail(c, 0, rc);
      HIPCHK(hipStreamSynchronize(s.stream));
      harvest(c, 0, rc);
    }
  } catch (...) {
    (void)hipStreamSynchronize(s.stream);
    for (void* p : T) (void)hipFree(p);
    throw;
  }
  for (void* p : T) (void)hipFree(p);
  return 0;
}

// The reference runs one job per hop for all its windows (BWindowedRangeAnalysisTask); it halts
// at the first superstep in which no label of any window improved, or at maxSteps
// (AnalysisTask.endStep :208-225), so every view of hop h reports min(maxSteps, 1 + the last
// changing step over the hop's windows), or 0 when maxSteps <= 1 (no Setup, :169).  With
// partitions the last changing step is the maximum over them.
void finish_supersteps(rgpu_ctx* c, const RunCfg& rc) {
  const size_t nview = rc.n_hops * rc.W;
  if (c->partitioned && c->nparts > 1) {
    std::vector<unsigned long long> h(nview);
    for (size_t i = 0; i < nview; i++) h[i] = (unsigned long long)c->vlast[i];
    unsigned long long* d = nullptr;
    HIPCHK(hipMalloc(&d, sizeof(unsigned long long) * std::max<size_t>(nview, 1)));
    Slot& s = c->slot[0];
    HIPCHK(hipMemcpyAsync(d, h.data(), sizeof(unsigned long long) * nview, hipMemcpyHostToDevice, s.stream));
    c->pt.xchg->allreduce_u64(d, nview, true, s.stream);
    HIPCHK(hipMemcpyAsync(h.data(), d, sizeof(unsigned long long) * nview, hipMemcpyDeviceToHost, s.stream));
    HIPCHK(hipStreamSynchronize(s.stream));
    (void)hipFree(d);
    for (size_t i = 0; i < nview; i++) c->vlast[i] = (int32_t)h[i];
  }
  for (size_t hop = 0; hop < rc.n_hops; hop++) {
    int32_t r = 0;
    for (int w = 0; w < rc.W; w++) r = std::max(r, c->vlast[hop * rc.W + w]);
    const int64_t steps = rc.max_steps <= 1 ? 0 : std::min<int64_t>(rc.max_steps, (int64_t)r + 1);
    for (int w = 0; w < rc.W; w++) c->cc[hop * rc.W + w].supersteps = steps;
  }
}

int fail(rgpu_ctx* c, int code, const std::string& m);
// After device-packed merges the ids live in HBM (g_vid); the host copy follows when a result
// names vertices.  Returns an RGPU_* code.
int sync_vid(rgpu_ctx* c) {
  if (!c->vid_stale) return RGPU_OK;
  try {
    c->pk.vid.resize((size_t)c->g.nv);
    if (c->g.nv)
      HIPCHK(hipMemcpy(c->pk.vid.data(), c->g_vid, sizeof(int64_t) * c->g.nv, hipMemcpyDeviceToHost));
    if (c->partitioned)  // (rank-order keys: 2^31 | id for a ghost)
      for (int64_t v = c->pk.n_own; v < c->g.nv; v++) c->pk.vid[v] &= ((int64_t)1 << 31) - 1;
  } catch (const HipFail& f) {
    return fail(c, RGPU_EHIP, f.msg);
  } catch (const std::bad_alloc&) {
    return fail(c, RGPU_ENOMEM, "host allocation failed");
  }
  c->vid_stale = false;
  return RGPU_OK;
}

// id of the vertex whose label is l: partitioned, labels are ids; else id ranks
int64_t label_id(const rgpu_ctx* c, int32_t l) {
  if (c->partitioned) return (int64_t)l;
  return c->pk.lid.empty() ? c->pk.vid[l] : c->pk.lid[l];
}

// the k-th owned vertex in ascending id order (result lists are ascending by id)
int64_t own_at(const rgpu_ctx* c, int64_t k) { return c->pk.by_id.empty() ? k : (int64_t)c->pk.by_id[k]; }

// After a failed run (a HIP / RCCL / exchange error or a failed allocation mid-run): the slots may
// hold a batch in any phase, and the per-batch state that only a batch's last kernels bring back
// to zero (count rows, island shards, lane-change shards, hub minima, record counts) may be
// dirty.  Drain the streams and drop every slot and exchange-slot buffer, so that the next run
// allocates them fresh and clean; the run's results are invalid.
void drop_alloc(std::vector<void*>& L, void* p) {
  if (!p) return;
  auto it = std::find(L.begin(), L.end(), p);
  if (it == L.end()) return;
  (void)hipFree(p);
  L.erase(it);
}
void reset_after_failure(rgpu_ctx* c) {
  for (Slot& s : c->slot)
    if (s.stream) (void)hipStreamSynchronize(s.stream);
  (void)hipDeviceSynchronize();
  (void)hipGetLastError();
  auto& LG = c->graph_allocs;
  for (Slot& s : c->slot)
    for (void* p : {(void*)s.hv.segcnt, (void*)s.hv.segor, (void*)s.hv.best, (void*)s.hv.pacc}) drop_alloc(LG, p);
  for (XSlot& xs : c->pt.xs)
    for (void* p : {(void*)xs.err, (void*)xs.mfin, (void*)xs.fin_g, (void*)xs.htot, (void*)xs.xab, (void*)xs.vms, (void*)xs.vmr})
      drop_alloc(LG, p);
  release_slots(c);
  free_part_slots(c, true);
  c->algo = -1;
  c->cc.clear();
  c->vlast.clear();
  c->kept.clear();
  c->retained = false;
  if (c->d_ecnt) { (void)hipFree(c->d_ecnt); c->d_ecnt = nullptr; }
}

int fail(rgpu_ctx* c, int code, const std::string& m) {
  if (c) c->err = m;
  return code;
}

int env_int(const char* k, int d) {
  const char* v = std::getenv(k);
  return v && *v ? std::atoi(v) : d;
}

}  // namespace

// ======================================================================== C ABI
extern "C" {

int rgpu_abi_version(void) { return RGPU_ABI_VERSION; }

int rgpu_open(int partition_id, int num_partitions, int device, rgpu_ctx** out) {
  if (!out) return RGPU_EINVAL;
  *out = nullptr;
  if (num_partitions < 1 || partition_id < 0 || partition_id >= num_partitions || device < 0)
    return RGPU_EINVAL;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || device >= ndev) return RGPU_EHIP;
  rgpu_ctx* c = new (std::nothrow) rgpu_ctx();
  if (!c) return RGPU_ENOMEM;
  c->part = partition_id;
  c->nparts = num_partitions;
  c->device = device;
  c->partitioned = num_partitions > 1 || env_int("RGPU_PARTITIONED", 0) != 0;
  c->check = env_int("RGPU_CHECK", 0) != 0;
  c->wmajor = env_int("RGPU_WMAJOR", 1) != 0;
  c->hostprof = env_int("RGPU_HOSTPROF", 0) != 0;
  c->iv_max = env_int("RGPU_IVMAX", 32);
  // batches in flight (default 3; 2 / 4 measured slower on C4).  RGPU_SLOTS=1 for the
  // 1B loopback rehearsal: eight partitions' slots do not fit one GPU three times over
  c->nslots = std::max(1, std::min(kMaxSlots, env_int("RGPU_SLOTS", 3)));
  c->heavy_env = env_int("RGPU_HEAVY", -1);
  c->heavy_t = c->heavy_env >= 0 ? c->heavy_env : 2048;
  c->delta_on = env_int("RGPU_DELTA", 1) != 0;
  c->delta_host = env_int("RGPU_DELTA", 1) == 2;
  {  // RGPU_XREC_TINY (tests): record buffers start tiny, so that every growth path runs
    const bool tiny = env_int("RGPU_XREC_TINY", 0) != 0;
    g_xrec_slack = tiny ? 1 : 1024;
    g_xrec_init = tiny ? 0 : 2;
  }
  if (const char* tp = std::getenv("RGPU_TRACE"))  // (a partition's trace: path + ".p<partition>")
    c->trace_path = num_partitions > 1 ? std::string(tp) + ".p" + std::to_string(partition_id) : std::string(tp);
  if (hipSetDevice(device) != hipSuccess) { delete c; return RGPU_EHIP; }
  *out = c;
  return RGPU_OK;
}

int rgpu_ingest(rgpu_ctx* c, const int64_t* t, const uint8_t* kind, const int64_t* src,
                const int64_t* dst, size_t n) {
  if (!c) return RGPU_EINVAL;
  std::lock_guard<std::mutex> lk(c->ingest_mu);  // (not mu: ingestion goes on during runs and merges)
  if (n && (!t || !kind || !src)) return fail(c, RGPU_EINVAL, "null input array");
  try {
    const size_t need = c->events.size() + n;  // geometric growth: live ingest appends often
    if (c->events.capacity() < need) c->events.reserve(std::max(need, c->events.capacity() * 2));
    for (size_t i = 0; i < n; i++) {
      if (kind[i] > RGPU_EDEL) return fail(c, RGPU_EINVAL, "unknown update kind");
      if (kind[i] >= RGPU_EADD && !dst) return fail(c, RGPU_EINVAL, "edge update without dst array");
      c->newest = std::max(c->newest, t[i]);
      const int64_t d = kind[i] >= RGPU_EADD ? dst[i] : -1;
      // a partition keeps its own part of the stream (rgpu_internal.hpp: partition_keeps)
      if (!partition_keeps(kind[i], src[i], d, c->part, c->nparts)) continue;
      c->events.push_back({t[i], src[i], d, kind[i]});
    }
  } catch (const std::bad_alloc&) {
    return fail(c, RGPU_ENOMEM, "host allocation failed");
  }
  return RGPU_OK;
}

int rgpu_ingest_rgev(rgpu_ctx* c, const uint8_t* buf, size_t bytes, size_t* consumed) {
  if (!c) return RGPU_EINVAL;
  if (!consumed) return fail(c, RGPU_EINVAL, "null argument");
  size_t n = 0, used = 0;
  if (rgpu_rgev_decode(buf, bytes, nullptr, nullptr, nullptr, nullptr, 0, &n, &used) != RGPU_OK)
    return fail(c, RGPU_EINVAL, rgpu_rgev_last_error());
  *consumed = 0;
  if (n == 0) return RGPU_OK;
  try {
    std::vector<int64_t> t(n), src(n), dst(n);
    std::vector<uint8_t> kind(n);
    if (rgpu_rgev_decode(buf, used, t.data(), kind.data(), src.data(), dst.data(), n, &n, &used) != RGPU_OK)
      return fail(c, RGPU_EINVAL, rgpu_rgev_last_error());
    const int rc = rgpu_ingest(c, t.data(), kind.data(), src.data(), dst.data(), n);
    if (rc == RGPU_OK) *consumed = used;
    return rc;
  } catch (const std::bad_alloc&) {
    return fail(c, RGPU_ENOMEM, "host allocation failed");
  }
}

namespace {

// Heavy vertices (power-law hubs): static slot lists cut into kSegSlots segments.
// hv: the heavy ranks ascending, a0 / deg: their first static slot and slot count
void build_heavy_list(DevGraph& g, std::vector<void*>& L, const std::vector<int32_t>& hv,
                      const std::vector<int64_t>& a0s, const std::vector<int64_t>& degs) {
  if (hv.empty()) return;
  std::vector<int32_t> hv_seg(1, 0), seg_v, seg_h, seg_n, hidx(hv.size());
  std::vector<int64_t> seg_lo;
  for (size_t k = 0; k < hv.size(); k++) {
    const int32_t v = hv[k];
    const int64_t deg = degs[k], a0 = a0s[k];
    const int32_t h = (int32_t)(hv_seg.size() - 1);
    hidx[k] = h;
    for (int64_t o = 0; o < deg; o += kSegSlots) {
      seg_v.push_back((int32_t)v);
      seg_h.push_back(h);
      seg_lo.push_back(a0 + o);
      seg_n.push_back((int32_t)std::min<int64_t>(kSegSlots, deg - o));
    }
    hv_seg.push_back((int32_t)seg_v.size());
  }
  g.n_heavy = (int64_t)hv_seg.size() - 1;
  g.n_seg = (int64_t)seg_v.size();
  {  // hv_of: -1 but at the heavy ranks (a scatter on the device: no O(V) host array)
    int32_t* hv_of = dalloc<int32_t>(L, g.nv);
    std::vector<void*> T;
    try {
      HIPCHK(hipMemsetAsync(hv_of, 0xff, sizeof(int32_t) * g.nv, nullptr));
      const int32_t* d_hv = dupload(T, hv);
      const int32_t* d_h = dupload(T, hidx);
      launch_scatter_i32(nullptr, (int64_t)hv.size(), d_hv, d_h, hv_of);
      HIPCHK(hipStreamSynchronize(nullptr));
    } catch (...) {
      for (void* p : T) (void)hipFree(p);
      throw;
    }
    for (void* p : T) (void)hipFree(p);
    g.hv_of = hv_of;
  }
  g.hv_seg = dupload(L, hv_seg);
  g.seg_v = dupload(L, seg_v);
  g.seg_h = dupload(L, seg_h);
  g.seg_lo = dupload(L, seg_lo);
  g.seg_n = dupload(L, seg_n);
}
// The hub threshold (static slots): RGPU_HEAVY when set; else scaled with the graph's (a partition's:
// its owned) vertices, 2048 at 16M and above, at least 256.  A superstep or K2 launch lasts as long as its slowest wave, and a wave walks a non-hub
// member's slots one chunk after another: with a few owned vertices per wave (8 partitions) that
// tail is the launch.  Measured on the 300M-update prefix at P = 8, slowest partition: 2048 ->
// 118 ms, 512 -> 102, 256 -> 98, 128 -> 99, 64 -> 107 (profiles/r04/part_sim_heavy*.jsonl); the
// 1B graph in one partition: 2048 273 ms, 512 286, 256 296 (hub passes grow).  Round 6: the rule holds
// for a graph that is not partitioned too (it was 2048 whatever the size): the week slice of the 1B
// stream (21M updates, the N > 1 hybrid's replica) answering 21 hops x {w, d, h}: 2048 ->
// 26.3 ms per block, 1024 -> 20.2, 4096 -> 37.6 (profiles/r06/part_sim_replica_ab_1b.jsonl); the
// 1B graph itself (19.9M vertices) keeps 2048.
int hub_threshold(const rgpu_ctx* c, int64_t n_own) {
  if (c->heavy_env >= 0) return c->heavy_env;
  const int64_t t = (int64_t)2048 * n_own / ((int64_t)1 << 24);
  return (int)std::max<int64_t>(256, std::min<int64_t>(2048, t));
}

void build_heavy(rgpu_ctx* c, DevGraph& g, std::vector<void*>& L, const std::vector<int64_t>& out_off,
                 const std::vector<int64_t>& in_off) {
  if (c->heavy_t <= 0) return;
  std::vector<int32_t> hv;
  std::vector<int64_t> a0, deg;
  for (int64_t v = 0; v < g.nv; v++) {
    const int64_t d = (out_off[v + 1] - out_off[v]) + (in_off[v + 1] - in_off[v]);
    if (d <= c->heavy_t) continue;
    hv.push_back((int32_t)v);
    a0.push_back(out_off[v] + in_off[v]);
    deg.push_back(d);
  }
  build_heavy_list(g, L, hv, a0, deg);
}

// K2's time-ordered static slots (tslots.hip), built on the device after the adjacency
void build_tslots(rgpu_ctx* c, DevGraph& g, std::vector<void*>& L) {
  const int64_t n = g.ne + g.n_in;
  if (n <= 0 || n > (int64_t)INT32_MAX) return;  // (int32 slot words)
  int32_t* e = dalloc<int32_t>(L, n);
  int32_t* nb = dalloc<int32_t>(L, n);
  int64_t* t = dalloc<int64_t>(L, n);
  std::vector<void*> T;
  bool ok = false;
  try {
    ok = build_time_slots(nullptr, g, e, nb, t, T);
    HIPCHK(hipDeviceSynchronize());
  } catch (...) {
    for (void* p : T) (void)hipFree(p);
    throw;
  }
  for (void* p : T) (void)hipFree(p);
  if (ok) {
    g.ts_e = e;
    g.ts_nb = nb;
    g.ts_t = t;
    // the simple-edge bitmap (K1's SKIP form reads one word per 64 edges instead of testing each
    // edge's history and endpoints every batch)
    uint64_t* es = dalloc<uint64_t>(L, (g.ne + 63) / 64 + 1);
    launch_edge_simple_bits(nullptr, g, es);
    HIPCHK(hipGetLastError());
    HIPCHK(hipDeviceSynchronize());
    g.esimple = es;
    // and the other edges' ids: K1's SKIP form walks only those (kernels.hip k_edge_mask)
    const int64_t nns = build_nonsimple_list(g, es, nullptr);
    int32_t* ens = dalloc<int32_t>(L, nns + 1);
    g.n_ens = build_nonsimple_list(g, es, ens);
    g.ens = ens;
  }
}

}  // extern "C" (a C++ helper: it returns a struct)

// the send plan by boundary vertex (xchg.hip build_xsend), from the (peer, vertex) lists
static XSend build_send_plan(int64_t n_own, const Part& X, std::vector<void*>& L) {
  std::vector<void*> T;
  XSend xs;
  try {
    xs = build_xsend(nullptr, n_own, X.nxs, X.xs_v, T, L);
  } catch (const std::runtime_error& e) {
    for (void* p : T) (void)hipFree(p);
    throw HipFail{e.what()};
  }
  for (void* p : T) (void)hipFree(p);
  return xs;
}

extern "C" {

// the neighbours' labels (grank) in time-ordered slot order, once grank is known
void build_tslot_labels(DevGraph& g, std::vector<void*>& L) {
  if (!g.ts_nb || !g.grank) return;
  const int64_t n = g.ne + g.n_in;
  int32_t* tg = dalloc<int32_t>(L, n);
  build_slot_labels(nullptr, n, g.ts_nb, g.grank, tg);
  HIPCHK(hipGetLastError());
  HIPCHK(hipDeviceSynchronize());
  g.ts_g = tg;
}

const int64_t* upload_adj(std::vector<void*>& L, const std::vector<int64_t>& out_off,
                          const std::vector<int64_t>& in_off) {
  const int64_t nv = (int64_t)out_off.size() - 1;
  std::vector<int64_t> adj(nv + 1 + 64);  // padded: read unconditionally by the step kernel
  for (int64_t v = 0; v <= nv; v++) adj[v] = out_off[v] + in_off[v];
  for (int64_t v = nv + 1; v < (int64_t)adj.size(); v++) adj[v] = adj[nv];
  return dupload(L, adj);
}

// one bit per vertex: it has a death (K1 skips the death-list offsets of an edge whose
// endpoints have none; DevGraph.dbits)
const uint64_t* upload_death_bits(std::vector<void*>& L, const std::vector<int64_t>& doff) {
  const int64_t nv = doff.empty() ? 0 : (int64_t)doff.size() - 1;
  std::vector<uint64_t> bits((size_t)(nv + 63) / 64 + 1, 0);
  for (int64_t v = 0; v < nv; v++)
    if (doff[v + 1] > doff[v]) bits[v >> 6] |= 1ull << (v & 63);
  return dupload(L, bits);
}

void finish_seal(rgpu_ctx* c, size_t n_end) {
  Packed& P = c->pk;
  {  // simple edges (the K1 edge byte model)
    unsigned long long* d = nullptr;
    HIPCHK(hipMalloc(&d, sizeof(unsigned long long)));
    HIPCHK(hipMemset(d, 0, sizeof(unsigned long long)));
    unsigned long long h = 0;
    launch_count_simple(nullptr, c->g, d);
    const hipError_t e1 = hipGetLastError();
    const hipError_t e2 = hipMemcpy(&h, d, sizeof(h), hipMemcpyDeviceToHost);
    (void)hipFree(d);
    HIPCHK(e1);
    HIPCHK(e2);
    c->n_simple = (int64_t)h;
  }
  c->st.vertices = P.n_own;
  c->st.edges = P.ne;
  c->st.edges_owned = P.ne_owned;
  c->st.vertex_events = P.n_vkey;
  c->st.edge_events = P.n_ekey;
  c->st.deaths = c->n_dtime >= 0 ? c->n_dtime : (int64_t)P.dtime.size();
  c->n_sealed = n_end;
  c->sealed = true;
  if (!c->partitioned) {  // the big arrays live in HBM only (the delta merge keeps them there)
    for (auto* v : {&P.voff, &P.vkey, &P.eoff, &P.ekey}) std::vector<int64_t>().swap(*v);
    for (auto* v : {&P.esrc, &P.edst, &P.in_eid}) std::vector<int32_t>().swap(*v);
  }
}

// Replace the resident graph by a merged one (under mu, between runs).  The last run's results
// named the old graph's ranks: they go.  Batch slots and mask sets stay if they fit (else they are
// reallocated on the next run with 2x headroom for the ticks to come).
// Exception safety: every step that can throw before the commit point (the send plan, which
// allocates) builds into the merged graph's own allocations, so a throw there leaves both the
// resident graph and M intact.  At the commit point M is emptied (a throw after it cannot make a
// later apply_pending re-install freed pointers), and the steps after it only clear slot state:
// if one throws, the slots are released and reallocated by the next run.
void apply_merged(rgpu_ctx* c, Merged& M) {
  XSend xsend;
  if (c->partitioned) {  // (allocates: before the commit point, into M.L)
    Part tmp;
    tmp.nxs = M.PM.nxs;
    tmp.xs_v = M.PM.xs_v;
    xsend = build_send_plan(M.g.n_own, tmp, M.L);
  }
  // ---- commit point: nothing below throws until the slot clears
  Merged T = std::move(M);
  M = Merged();
  Packed& B = c->pk;
  const DevGraph g = T.g;
  const bool dev = T.dev;
  PartMeta& PM = T.PM;
  std::vector<void*> old;
  old.swap(c->graph_allocs);
  c->graph_allocs.swap(T.L);
  c->g = g;
  c->g_vid = T.vid2;
  if (c->partitioned) {  // the old plan's buffers went with the old graph; channels stay
    free_part_slots(c, true);
    Exchange* x = c->pt.xchg;
    XSlot xs[4];
    for (int i = 0; i < 4; i++) xs[i].x = c->pt.xs[i].x;
    c->pt = Part();
    c->pt.xchg = x;
    for (int i = 0; i < 4; i++) c->pt.xs[i].x = xs[i].x;
    Part& X = c->pt;
    X.nxs = PM.nxs;
    X.nxr = PM.nxr;
    X.xs_off = PM.xs_off;
    X.xr_off = PM.xr_off;
    X.xs_v = PM.xs_v;
    X.xs_q = PM.xs_q;
    X.xr_v = PM.xr_v;
    X.xr_q = PM.xr_q;
    X.xs_off_d = PM.xs_off_d;
    X.xr_off_d = PM.xr_off_d;
    X.xsend = xsend;
    X.own.vid = PM.own_vid;
    X.own.pos = nullptr;
    X.own.boff = PM.own_boff;
    X.own.shift = PM.shift;
    X.own.n_own = g.n_own;
    X.own.id_max = PM.id_max;
    c->orph_id.swap(T.orph_id);
    c->orph_t.swap(T.orph_t);
  }
  for (Slot& sl : c->slot) {
    sl.hv = HeavyBuf();
    sl.h_cc = sl.h_pr = false;
  }
  B.nv = T.nv2;
  B.n_own = g.n_own;
  B.ne = g.ne;
  B.ne_owned = T.ne_owned;
  if (dev) {  // the host keeps no offsets; its ids follow on demand (host_vid)
    c->vid_stale = true;
    c->n_dtime = T.ndt;
    for (auto* v : {&B.doff, &B.dtime, &B.out_off, &B.in_off}) std::vector<int64_t>().swap(*v);
  } else {
    B.vid.swap(T.hvid);
    B.doff.swap(T.hdoff);
    B.dtime.swap(T.hdtime);
    B.out_off.swap(T.hout_off);
    B.in_off.swap(T.hin_off);
    c->n_dtime = -1;
  }
  B.n_vkey = T.nvk;
  B.n_ekey = T.nek;
  B.n_in = g.n_in;
  {
    std::lock_guard<std::mutex> il(c->ingest_mu);
    B.newest = c->newest;
  }
  c->st.seal_delta_updates = T.nd;
  c->algo = -1;  // (results of the last run named the old graph)
  c->cc.clear();
  c->vlast.clear();
  c->kept.clear();
  c->retained = false;
  c->pt.tab_ready = false;
  for (void* p : old) (void)hipFree(p);  // (the slots' kernels have finished: runs hold mu)
  // slot state that K2 does not rewrite, for the new graph
  if (g.nv > c->cap_nv || g.ne > c->cap_ne || g.n_in > c->cap_nin ||
      (c->partitioned ? c->pk.n_own : g.nv) > c->cap_nown) {
    release_slots(c);
    c->cap_nv = 2 * g.nv;  // doubling: a growing live graph re-allocates O(log) times
    c->cap_ne = 2 * g.ne;
    c->cap_nin = 2 * g.n_in;
    c->cap_nown = 2 * (c->partitioned ? c->pk.n_own : g.nv);
  } else {
    try {
      for (int i = 0; i < c->nslots; i++) {
        Slot& sl = c->slot[i];
        if (sl.chg[0]) {
          HIPCHK(hipMemset(sl.chg[0], 0, sizeof(uint64_t) * (c->cap_nv + kPad)));
          HIPCHK(hipMemset(sl.chg[1], 0, sizeof(uint64_t) * (c->cap_nv + kPad)));
          HIPCHK(hipMemset(sl.snbr, 0, sizeof(int32_t) * (c->cap_ne + c->cap_nin + kPad)));
        }
      }
    } catch (...) {
      release_slots(c);  // the next run allocates fresh, cleared slots
      throw;
    }
  }
}

// the parked merged graph (if any) replaces the resident one (under mu)
void apply_pending(rgpu_ctx* c) {
  if (!c->pending.valid) return;
  apply_merged(c, c->pending);
  finish_seal(c, c->n_sealed);
}

// A live context (device merges, id order) never re-packs the whole log: once sealed, its updates
// are dropped from the host log (a C4-size base would otherwise keep 32 GB of records and copy them
// whenever the log grows).  Others keep the log for their re-packs.  holding: ingest_mu is held.
void drop_sealed_log(rgpu_ctx* c, bool holding) {
  if (!c->delta_on || c->delta_host || c->pk.relabeled || c->g.nv == 0) return;
  std::unique_lock<std::mutex> il(c->ingest_mu, std::defer_lock);
  if (!holding) il.lock();
  const size_t k = c->n_sealed - c->ev_base;
  if (k == 0) return;
  c->events.erase(c->events.begin(), c->events.begin() + k);
  if (c->events.capacity() > 4 * std::max<size_t>(c->events.size(), 1 << 20)) c->events.shrink_to_fit();
  c->ev_base = c->n_sealed;
}

// Incremental seal: merge the updates ingested since the last seal into the resident graph
// (merge.hip).  The delta arrays come from the device packer (gdelta.hip: the tick's updates
// are uploaded once and never come back) or, RGPU_DELTA=2, from the host packer (packer.cpp
// pack_delta / finish_delta: delta-sized sorts + O(V) offsets on the host).

// Builds the merged graph of the resident one and the updates [n_sealed, n_end) (absolute) into M,
// beside the resident graph: runs on it go on meanwhile (live ingest).  apply_merged swaps it in.
void seal_delta(rgpu_ctx* c, size_t n_end, Merged& M) {
  Packed& B = c->pk;
  const bool dev = !c->delta_host;
  auto tp = std::chrono::steady_clock::now();
  auto phase = [&](const char* what) {  // RGPU_HOSTPROF: host-side phase times
    if (!c->hostprof) return;
    const auto now = std::chrono::steady_clock::now();
    std::fprintf(stderr, "[rgpu seal_delta] %-10s %8.2f ms\n", what,
                 std::chrono::duration<double, std::milli>(now - tp).count());
    tp = now;
  };
  static_assert(sizeof(Event) == sizeof(DevEvent) && offsetof(Event, kind) == offsetof(DevEvent, kind),
                "the device packer reads the host's update records as they are");
  Delta D;      // host packer
  DeltaDev DD;  // device packer
  std::vector<void*> T;  // temporaries
  std::vector<void*> L;  // the merged graph
  hipStream_t s = nullptr;
  try {
    HIPCHK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    const DevGraph& g0 = c->g;
    MergeIn m;
    m.nv_old = g0.nv;
    m.ne_old = g0.ne;
    m.nin_old = g0.n_in;
    m.esrc = g0.esrc;
    m.edst = g0.edst;
    m.in_eid = g0.in_eid;
    m.eoff = g0.eoff;
    m.ekey = g0.ekey;
    m.voff = g0.voff;
    m.vkey = g0.vkey;
    m.in_off = g0.in_off;
    m.nvk_old = B.n_vkey;
    int64_t nv2 = 0, n_in2 = 0;
    if (dev) {
      int64_t* gvid = c->g_vid;
      if (!gvid) {  // the first merge into a full seal: its rank-order keys (DeltaPart)
        std::vector<int64_t> keys(B.vid);
        if (c->partitioned)
          for (int64_t v = B.n_own; v < B.nv; v++) keys[v] |= (int64_t)1 << 31;
        gvid = dalloc<int64_t>(T, g0.nv);
        HIPCHK(hipMemcpy(gvid, keys.data(), sizeof(int64_t) * g0.nv, hipMemcpyHostToDevice));
      }
      const int64_t n = (int64_t)(n_end - c->n_sealed);
      DevEvent* ev = dalloc<DevEvent>(T, n);
      {  // (the log may grow meanwhile: ingestion waits only for this copy)
        std::lock_guard<std::mutex> il(c->ingest_mu);
        HIPCHK(hipMemcpy(ev, c->events.data() + (c->n_sealed - c->ev_base), sizeof(Event) * n, hipMemcpyHostToDevice));
      }
      phase("upload");
      DeltaPart dp;
      if (c->partitioned) {
        dp.part = c->part;
        dp.nparts = c->nparts;
        dp.n_own_old = B.n_own;
        dp.n_orph = (int64_t)c->orph_id.size();
        if (dp.n_orph) {
          dp.orph_id = dupload(T, c->orph_id);
          dp.orph_t = dupload(T, c->orph_t);
        }
      }
      std::string e;
      c->heavy_t = hub_threshold(c, B.n_own);  // (the partition's owned count before the merge)
      try {
        e = gpu_pack_delta(s, ev, n, g0, gvid, dp, c->heavy_t, &DD, T, L);
      } catch (const std::runtime_error& x) {
        throw HipFail{x.what()};
      }
      if (!e.empty()) throw HipFail{e, RGPU_EINVAL};
      phase("pack");
      nv2 = DD.nv2;
      n_in2 = DD.n_in;
      m.old2new = DD.old2new;
      m.new2old = DD.new2old;
      m.n_new = DD.n_new;
      m.nde = DD.nde;
      m.nn_key = DD.nn_key;
      m.nn_didx = DD.nn_didx;
      m.de_base = DD.de_base;
      m.dkoff = DD.de_koff;
      m.dkey = DD.de_key;
      m.ndd = DD.ndd;
      m.dd_rank = DD.dd_rank;
      m.dd_off = DD.dd_off;
      m.dd_t = DD.dd_t;
      m.ndv = DD.ndv;
      m.dv_rank = DD.dv_rank;
      m.dv_off = DD.dv_off;
      m.dv_key = DD.dv_key;
      m.ndvk = DD.ndvk;
      m.nni = DD.nni;
      m.ni_key = DD.ni_key;
      m.ni_idx = DD.ni_idx;
    } else {
      std::string e = pack_delta(c->events, c->n_sealed, B, &D);  // (host packer: ev_base = 0, ingest_mu held)
      phase("pack");
      if (!e.empty()) throw HipFail{e, RGPU_EINVAL};
      const int64_t nde = (int64_t)D.de_s.size();
      std::vector<int32_t> base_eid(nde, -1);
      if (nde) {
        int32_t* qs = dupload(T, D.de_qs);
        int32_t* qd = dupload(T, D.de_qd);
        int32_t* res = dalloc<int32_t>(T, nde);
        launch_edge_find(s, nde, qs, qd, g0.out_off, g0.edst, res);
        HIPCHK(hipMemcpyAsync(base_eid.data(), res, sizeof(int32_t) * nde, hipMemcpyDeviceToHost, s));
        HIPCHK(hipStreamSynchronize(s));
      }
      phase("lookup");
      finish_delta(B, base_eid, &D);
      phase("finish");
      nv2 = D.nv;
      n_in2 = D.in_off[D.nv];
      m.old2new = dupload(T, D.old2new);
      m.new2old = dupload(T, D.new2old);
      m.n_new = (int64_t)D.nn_key.size();
      m.nde = nde;
      m.nn_key = dupload(T, D.nn_key);
      m.nn_didx = dupload(T, D.nn_didx);
      m.de_base = dupload(T, D.de_base);
      m.dkoff = dupload(T, D.de_koff);
      m.dkey = dupload(T, D.de_key);
      m.ndd = (int64_t)D.dd_rank.size();
      m.dd_rank = dupload(T, D.dd_rank);
      m.dd_off = dupload(T, D.dd_off);
      m.dd_t = dupload(T, D.dd_t);
      m.ndv = (int64_t)D.dv_rank.size();
      m.dv_rank = dupload(T, D.dv_rank);
      m.dv_off = dupload(T, D.dv_off);
      m.dv_key = dupload(T, D.dv_key);
      m.ndvk = (int64_t)D.dv_key.size();
      m.nni = (int64_t)D.ni_key.size();
      m.ni_key = dupload(T, D.ni_key);
      m.ni_idx = dupload(T, D.ni_idx);
    }
    m.nv2 = nv2;
    m.coll = dalloc<int64_t>(T, m.ndvk + 1);
    m.coll_tmp = dalloc<int64_t>(T, scan_tmp_words(std::max<int64_t>(m.ndvk, 1)));
    HIPCHK(hipStreamSynchronize(s));
    phase("upload");
    DevGraph g;
    g.nv = nv2;
    g.n_own = dev ? DD.n_own2 : nv2;
    g.ne = g0.ne + m.n_new;
    g.n_in = n_in2;
    int32_t* esrc2 = dalloc<int32_t>(L, g.ne);
    int32_t* edst2 = dalloc<int32_t>(L, g.ne);
    int32_t* eo2n = dalloc<int32_t>(T, g0.ne);
    int32_t* mbase = dalloc<int32_t>(T, g.ne);
    int32_t* mdlt = dalloc<int32_t>(T, g.ne);
    int32_t* npos = dalloc<int32_t>(T, m.n_new);
    phase("alloc e");
    launch_merge_edges(s, m, esrc2, edst2, eo2n, mbase, mdlt, npos);
    HIPCHK(hipStreamSynchronize(s));
    phase("place");
    int64_t* stmp = dalloc<int64_t>(T, scan_tmp_words(std::max(g.ne, g.nv)));
    // edge histories: count, scan, write
    int64_t* eoff2 = dalloc<int64_t>(L, g.ne + 1);
    launch_edge_hist(s, false, m, g.ne, mbase, mdlt, esrc2, edst2, eoff2, nullptr);
    launch_scan_counts(s, g.ne, eoff2, stmp);
    int64_t nek = 0, nvk = 0;
    HIPCHK(hipMemcpyAsync(&nek, eoff2 + g.ne, sizeof(int64_t), hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    phase("e count");
    int64_t* ekey2 = dalloc<int64_t>(L, nek);
    phase("alloc ekey");
    launch_edge_hist(s, true, m, g.ne, mbase, mdlt, esrc2, edst2, eoff2, ekey2);
    // vertex histories
    HIPCHK(hipStreamSynchronize(s));
    phase("e write");
    int64_t* voff2 = dalloc<int64_t>(L, g.nv + 1);
    launch_vertex_hist(s, false, m, voff2, nullptr);
    launch_scan_counts(s, g.nv, voff2, stmp);
    HIPCHK(hipMemcpyAsync(&nvk, voff2 + g.nv, sizeof(int64_t), hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    phase("v count");
    int64_t* vkey2 = dalloc<int64_t>(L, nvk);
    phase("alloc vkey");
    launch_vertex_hist(s, true, m, voff2, vkey2);
    HIPCHK(hipStreamSynchronize(s));
    phase("hist kernels");
    // adjacency offsets, in-edges
    const int64_t* in_off2 = dev ? DD.in_off : dupload(L, D.in_off);
    int32_t* in_eid2 = dalloc<int32_t>(L, g.n_in);
    launch_merge_in(s, m, eo2n, npos, in_off2, in_eid2);
    HIPCHK(hipGetLastError());
    g.esrc = esrc2;
    g.edst = edst2;
    g.eoff = eoff2;
    g.ekey = ekey2;
    g.voff = voff2;
    g.vkey = vkey2;
    g.in_off = in_off2;
    g.in_eid = in_eid2;
    if (dev) {
      g.out_off = DD.out_off;
      g.adj_off = DD.adj_off;
      g.doff = DD.doff;
      g.dtime = DD.dtime;
      g.dbits = DD.dbits;
    } else {
      g.out_off = dupload(L, D.out_off);
      g.adj_off = upload_adj(L, D.out_off, D.in_off);
      g.doff = dupload(L, D.doff);
      g.dtime = dupload(L, D.dtime);
      g.dbits = upload_death_bits(L, D.doff);
    }
    HIPCHK(hipStreamSynchronize(s));
    phase("adjacency");
    if (dev) {
      if (c->heavy_t > 0) build_heavy_list(g, L, DD.heavy, DD.heavy_a0, DD.heavy_deg);
    } else {
      build_heavy(c, g, L, D.out_off, D.in_off);
    }
    HIPCHK(hipStreamSynchronize(s));
    phase("heavy");
    build_tslots(c, g, L);
    phase("time-ordered slots");
    PartMeta PM;
    int64_t ne_owned = g.ne;
    if (c->partitioned) {  // labels = ids, the exchange plan and the owned-id index of the merged graph
      try {
        (void)gpu_part_meta(s, DD.vid2, nv2, g.n_own, esrc2, edst2, g.ne, c->nparts, &PM, T, L);
      } catch (const std::runtime_error& x) {
        throw HipFail{x.what()};
      }
      g.grank = PM.grank;
      build_tslot_labels(g, L);
      HIPCHK(hipMemcpy(&ne_owned, DD.out_off + g.n_own, sizeof(int64_t), hipMemcpyDeviceToHost));  // (owned first)
      phase("partition plan");
    }
    for (void* p : T) (void)hipFree(p);
    T.clear();
    (void)hipStreamDestroy(s);
    s = nullptr;
    // the merged graph, ready to replace the resident one (apply_merged)
    M.g = g;
    M.L.swap(L);
    M.dev = dev;
    M.vid2 = dev ? DD.vid2 : nullptr;
    M.ndt = dev ? DD.ndt : -1;
    M.nd = dev ? DD.nd : D.nd;
    M.PM = std::move(PM);
    M.ne_owned = ne_owned;
    M.nvk = nvk;
    M.nek = nek;
    M.nv2 = nv2;
    if (dev) {
      M.orph_id.swap(DD.orph_id);
      M.orph_t.swap(DD.orph_t);
    } else {
      M.hvid.swap(D.vid);
      M.hdoff.swap(D.doff);
      M.hdtime.swap(D.dtime);
      M.hout_off.swap(D.out_off);
      M.hin_off.swap(D.in_off);
    }
    M.valid = true;
    phase("built");
  } catch (...) {
    if (s) (void)hipStreamSynchronize(s);
    for (void* p : T) (void)hipFree(p);
    for (void* p : L) (void)hipFree(p);
    if (s) (void)hipStreamDestroy(s);
    throw;
  }
}

}  // namespace

int rgpu_seal(rgpu_ctx* c) {
  if (!c) return RGPU_EINVAL;
  std::lock_guard<std::mutex> sl(c->seal_mu);
  const auto t0 = std::chrono::steady_clock::now();
  size_t n_end;
  {
    std::lock_guard<std::mutex> il(c->ingest_mu);
    n_end = c->ev_base + c->events.size();
  }
  std::unique_lock<std::mutex> lk(c->mu, std::defer_lock);
  std::unique_lock<std::mutex> il(c->ingest_mu, std::defer_lock);
  try {
    HIPCHK(hipSetDevice(c->device));
    if (c->n_sealed > 0 && c->n_sealed == n_end) {  // nothing new since the last seal
      lk.lock();
      // partitioned: the broadcast records' receive tables name the peers' boundary lists, which any
      // partition's seal may change — every partition rebuilds them (collectively) at its next run
      c->pt.tab_ready = false;
      c->sealed = true;
      return RGPU_OK;
    }
    // A graph parked by the previous seal goes in first (this one builds on it), and the decision
    // reads the resident graph: both under mu, since a run may be swapping the parked graph in at
    // this moment (apply_pending).  After this point the resident graph (c->g, c->pk's metadata,
    // c->g_vid, the orphan lists) stays as it is until this seal swaps its result in: only a seal
    // parks a graph or re-packs, and seal_mu is held, so seal_delta reads it without mu while runs
    // read it too.  (A locality-ordered base has no monotone rank maps to merge into: it is
    // re-packed; the partitioned merge needs the device packer.)
    bool incremental;
    lk.lock();
    apply_pending(c);
    incremental = c->delta_on && c->n_sealed > 0 && c->g.nv > 0 && !c->pk.relabeled && !(c->partitioned && c->delta_host);
    lk.unlock();
    if (incremental) {
      // live ingest: merge the delta into the resident graph.  The device packer builds it while runs
      // and ingestion go on; the host packer (RGPU_DELTA=2) reads the log, so ingestion waits.
      if (c->delta_host) {
        il.lock();
        n_end = c->ev_base + c->events.size();  // (what the host packer will read)
      }
      Merged M;
      seal_delta(c, n_end, M);
      if (c->check)
        run_check(nullptr, "merged graph", [&](unsigned long long* bad) {
          launch_check_graph(nullptr, M.g, M.nek, M.nvk, bad);
        });
      lk.lock();
      c->st.seal_incremental = 1;
      if (c->algo < 0) {  // no results to keep: swap it in now
        apply_merged(c, M);
        finish_seal(c, n_end);
      } else {  // the last run's results stay readable: the next run (or seal) swaps it in
        c->pending = std::move(M);
        const Merged& P = c->pending;
        c->st.vertices = P.g.n_own;
        c->st.edges = P.g.ne;
        c->st.edges_owned = P.ne_owned;
        c->st.vertex_events = P.nvk;
        c->st.edge_events = P.nek;
        c->st.deaths = P.dev ? P.ndt : (int64_t)P.hdtime.size();
        c->st.seal_delta_updates = P.nd;
        c->n_sealed = n_end;
        c->sealed = true;
      }
      drop_sealed_log(c, il.owns_lock());
      c->st.seal_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
      return RGPU_OK;
    }
    lk.lock();
    il.lock();
    n_end = c->ev_base + c->events.size();  // (the whole log is packed)
    c->pt.tab_ready = false;
    c->sealed = false;
    c->st.seal_incremental = 0;
    c->st.seal_delta_updates = 0;
    if (c->ev_base) return fail(c, RGPU_ESTATE, "the update log before the resident graph was dropped: cannot re-pack");
    std::string e = pack_events(c->events, c->part, c->nparts, &c->pk, c->vertex_order == RGPU_ORDER_LOCALITY);
    if (!e.empty()) return fail(c, RGPU_EINVAL, e);
    free_graph(c);
    c->vid_stale = false;
    c->n_dtime = -1;
    c->orph_id.clear();
    c->orph_t.clear();
    if (c->partitioned && !c->pk.relabeled) {  // deaths of ids not kept here (a later merge may ghost them)
      const Packed& Q = c->pk;
      for (const Event& ev : c->events) {
        if (ev.kind != RGPU_VDEL || partition_of(ev.src, c->nparts) == c->part) continue;
        if (!std::binary_search(Q.vid.begin() + Q.n_own, Q.vid.end(), ev.src)) {
          c->orph_id.push_back(ev.src);
          c->orph_t.push_back(ev.t);
        }
      }
    }
    const Packed& P = c->pk;
    auto& L = c->graph_allocs;
    DevGraph g;
    g.nv = P.nv;
    g.ne = P.ne;
    g.n_in = P.n_in;
    g.voff = dupload(L, P.voff);
    g.vkey = dupload(L, P.vkey);
    g.doff = dupload(L, P.doff);
    g.dtime = dupload(L, P.dtime);
    g.dbits = upload_death_bits(L, P.doff);
    g.esrc = dupload(L, P.esrc);
    g.edst = dupload(L, P.edst);
    g.eoff = dupload(L, P.eoff);
    g.ekey = dupload(L, P.ekey);
    g.out_off = dupload(L, P.out_off);
    g.in_off = dupload(L, P.in_off);
    g.adj_off = upload_adj(L, P.out_off, P.in_off);
    g.in_eid = dupload(L, P.in_eid);
    g.n_own = P.n_own;
    c->heavy_t = hub_threshold(c, P.n_own);
    build_heavy(c, g, L, P.out_off, P.in_off);
    build_tslots(c, g, L);
    if (!c->partitioned && !P.grank.empty()) {  // locality order: labels are id ranks
      g.grank = dupload(L, P.grank);
      build_tslot_labels(g, L);
    }
    if (c->partitioned) {  // CC labels are vertex ids (the label owner routes component counts)
      if (c->nparts > kMaxParts) return fail(c, RGPU_EINVAL, "more than 8 partitions");
      // (also with P = 1, where a relabeled pack's grank holds id ranks)
      g.grank = dupload(L, std::vector<int32_t>(P.vid.begin(), P.vid.end()));
      build_tslot_labels(g, L);
      Part& X = c->pt;
      X.nxs = (int64_t)P.xs_v.size();
      X.nxr = (int64_t)P.xr_v.size();
      X.xs_off = P.xs_off;
      X.xr_off = P.xr_off;
      X.xs_v = dupload(L, P.xs_v);
      X.xs_q = dupload(L, P.xs_q);
      X.xr_v = dupload(L, P.xr_v);
      X.xr_q = dupload(L, P.xr_q);
      X.xs_off_d = dupload(L, P.xs_off);
      X.xr_off_d = dupload(L, P.xr_off);
      X.xsend = build_send_plan(P.n_own, X, L);
      {  // owned ids ascending (index = the count-table row of the label): bucket b = id >> shift,
         // about one id per bucket
        std::vector<int64_t> ids((size_t)P.n_own);
        for (int64_t k = 0; k < P.n_own; k++) ids[k] = P.vid[P.by_id.empty() ? k : P.by_id[k]];
        const int64_t id_max = ids.empty() ? -1 : *std::max_element(ids.begin(), ids.end());
        const int shift = own_bucket_shift(P.n_own, id_max);
        const int64_t nbk = (std::max<int64_t>(id_max, 0) >> shift) + 1;
        std::vector<int32_t> boff(nbk + 1, 0);
        for (int64_t k = 0; k < P.n_own; k++) boff[(ids[k] >> shift) + 1]++;
        for (int64_t b = 0; b < nbk; b++) boff[b + 1] += boff[b];
        X.own.vid = dupload(L, ids);
        X.own.pos = P.by_id.empty() ? nullptr : dupload(L, P.by_id);
        X.own.boff = dupload(L, boff);
        X.own.shift = shift;
        X.own.n_own = P.n_own;
        X.own.id_max = id_max;
      }
    }
    c->g = g;
    HIPCHK(hipDeviceSynchronize());
    const int64_t nek = P.n_ekey, nvk = P.n_vkey;
    finish_seal(c, n_end);
    if (c->check)
      run_check(nullptr, "sealed graph", [&](unsigned long long* bad) {
        launch_check_graph(nullptr, c->g, nek, nvk, bad);
      });
    drop_sealed_log(c, true);
  } catch (const HipFail& f) {
    return fail(c, f.code ? f.code : RGPU_EHIP, f.msg);
  } catch (const std::bad_alloc&) {
    return fail(c, RGPU_ENOMEM, "host allocation failed");
  }
  c->st.seal_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  return RGPU_OK;
}

int rgpu_set_vertex_order(rgpu_ctx* c, int order) {
  if (!c) return RGPU_EINVAL;
  std::lock_guard<std::mutex> lk(c->mu);
  if (order != RGPU_ORDER_LOCALITY && order != RGPU_ORDER_ID) return fail(c, RGPU_EINVAL, "unknown vertex order");
  c->vertex_order = order;
  return RGPU_OK;
}

int rgpu_newest_time(rgpu_ctx* c, int64_t* out) {
  if (!c || !out) return RGPU_EINVAL;
  std::lock_guard<std::mutex> lk(c->ingest_mu);
  *out = c->newest;
  return RGPU_OK;
}

int rgpu_exchange_id(int kind, uint8_t* out) {
  if (!out || (kind != RGPU_XCHG_RCCL && kind != RGPU_XCHG_LOOPBACK && kind != RGPU_XCHG_SHM)) return RGPU_EINVAL;
  return make_exchange_id(kind, out).empty() ? RGPU_OK : RGPU_EHIP;
}

int rgpu_exchange_init(rgpu_ctx* c, const void* id) {
  if (!c || !id) return RGPU_EINVAL;
  std::lock_guard<std::mutex> lk(c->mu);
  if (!c->partitioned) return RGPU_OK;  // one partition: nothing to exchange
  if (c->pt.xchg) return fail(c, RGPU_ESTATE, "exchange already initialised");
  Exchange* x = nullptr;
  std::string e = open_exchange((const uint8_t*)id, c->part, c->nparts, c->device, &x);
  if (!e.empty()) return fail(c, RGPU_EHIP, e);
  c->pt.xchg = x;
  return RGPU_OK;
}

// The partitioned superstep's fixed cost on this context's channel:
// `rounds` repetitions of what a superstep round costs besides its kernels' work, on slot 0's
// channel and a stream of its own — the counts all-to-all (4 words per peer) behind a one-node
// stand-in for the counts kernel, the counts' copy to the host and the host's wait for it (the
// host sizes the record transfers from them), and the two grouped send/recv of the label records
// (8 bytes per peer) — then `rounds` all-reduces of 64 words (the per-batch minimum labels and
// counts).  us[0..3]: round mean / median, all-reduce mean / median, microseconds (3 warm-up
// repetitions each, not counted).  Collective: every partition calls it.
int rgpu_exchange_probe(rgpu_ctx* c, int rounds, double* us) {
  if (!c || !us || rounds <= 0) return RGPU_EINVAL;
  std::lock_guard<std::mutex> lk(c->mu);
  if (!c->partitioned || !c->pt.xchg)
    return fail(c, RGPU_ESTATE, "exchange probe: a partitioned context after rgpu_exchange_init");
  const int P = c->nparts, me = c->part;
  hipStream_t st = nullptr;
  hipEvent_t ev = nullptr;
  int64_t* hx = nullptr;
  std::vector<void*> T;
  try {
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    HIPCHK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    XSlot& xs = c->pt.xs[0];
    if (!xs.x) xs.x = c->pt.xchg->fork(1);  // (the channel slot 0's runs use: collective, as in ensure_part)
    int64_t* xab = dalloc<int64_t>(T, 8 * P);
    unsigned long long* rec = dalloc<unsigned long long>(T, 4 * P);
    unsigned long long* red = dalloc<unsigned long long>(T, 64);
    HIPCHK(hipMemset(rec, 0, sizeof(unsigned long long) * 4 * P));
    HIPCHK(hipMemset(red, 0, sizeof(unsigned long long) * 64));
    HIPCHK(hipHostMalloc((void**)&hx, sizeof(int64_t) * 8 * P));
    std::vector<void*> sp(P), rp(P);
    std::vector<size_t> sb(P), rb(P);
    for (int q = 0; q < P; q++) {
      sp[q] = rec + q;
      rp[q] = rec + 2 * P + q;
      sb[q] = rb[q] = q == me ? 0 : sizeof(unsigned long long);
    }
    using clk = std::chrono::steady_clock;
    std::vector<double> tr, ta;
    auto t_last = clk::now();
    for (int i = 0; i < rounds + 3; i++) {
      HIPCHK(hipMemsetAsync(xab, 0, sizeof(int64_t) * 4 * P, st));  // (stands in for the counts kernel)
      xs.x->alltoall_i64(xab, xab + 4 * P, 4, st);
      HIPCHK(hipMemcpyAsync(hx, xab, sizeof(int64_t) * 8 * P, hipMemcpyDeviceToHost, st));
      HIPCHK(hipEventRecord(ev, st));
      HIPCHK(hipEventSynchronize(ev));  // the host reads the counts
      const auto t = clk::now();
      if (i >= 3) tr.push_back(std::chrono::duration<double, std::micro>(t - t_last).count());
      t_last = t;
      xs.x->sendrecv(sp.data(), sb.data(), rp.data(), rb.data(), st);  // U records
      xs.x->sendrecv(sp.data(), sb.data(), rp.data(), rb.data(), st);  // M records
    }
    HIPCHK(hipStreamSynchronize(st));
    for (int i = 0; i < rounds + 3; i++) {
      const auto t0 = clk::now();
      xs.x->allreduce_u64(red, 64, true, st);
      HIPCHK(hipStreamSynchronize(st));
      if (i >= 3) ta.push_back(std::chrono::duration<double, std::micro>(clk::now() - t0).count());
    }
    auto stat = [](std::vector<double> v, double* o) {
      double sum = 0;
      for (double x : v) sum += x;
      std::sort(v.begin(), v.end());
      o[0] = sum / (double)v.size();
      o[1] = v[v.size() / 2];
    };
    stat(tr, us);
    stat(ta, us + 2);
  } catch (const HipFail& f) {
    exchange_quiesce();
    for (void* p : T) (void)hipFree(p);
    if (hx) (void)hipHostFree(hx);
    if (ev) (void)hipEventDestroy(ev);
    if (st) (void)hipStreamDestroy(st);
    return fail(c, RGPU_EHIP, f.msg);
  } catch (const std::exception& x) {
    exchange_quiesce();
    for (void* p : T) (void)hipFree(p);
    if (hx) (void)hipHostFree(hx);
    if (ev) (void)hipEventDestroy(ev);
    if (st) (void)hipStreamDestroy(st);
    return fail(c, RGPU_EHIP, std::string("exchange probe: ") + x.what());
  }
  for (void* p : T) (void)hipFree(p);
  (void)hipHostFree(hx);
  (void)hipEventDestroy(ev);
  (void)hipStreamDestroy(st);
  return RGPU_OK;
}

int rgpu_run_view_batch(rgpu_ctx* c, int algo, const int64_t* hops, size_t n_hops,
                        const int64_t* windows, size_t n_w, int max_steps, int pr_iters,
                        int flags) {
  if (!c) return RGPU_EINVAL;
  std::lock_guard<std::mutex> lk(c->mu);
  if (!c->sealed) return fail(c, RGPU_ESTATE, "rgpu_run_view_batch before rgpu_seal");
  if (c->partitioned && !c->pt.xchg)
    return fail(c, RGPU_ESTATE, "partitioned context: call rgpu_exchange_init before running");
  if (algo < RGPU_ALGO_CC || algo > RGPU_ALGO_VP) return fail(c, RGPU_EINVAL, "unknown algo");
  if (algo == RGPU_ALGO_DIFFUSION && c->partitioned)
    return fail(c, RGPU_EINVAL, "diffusion runs need one partition");
  if (algo == RGPU_ALGO_VP && !c->vp_set) return fail(c, RGPU_ESTATE, "rgpu_set_vertex_program before a vertex-program run");
  if (!hops || n_hops == 0) return fail(c, RGPU_EINVAL, "no hops");
  if (n_w > (size_t)kViews) return fail(c, RGPU_EINVAL, "more than 64 windows in one batch");
  if (n_w && !windows) return fail(c, RGPU_EINVAL, "null window array");
  if ((algo == RGPU_ALGO_CC || algo == RGPU_ALGO_DIFFUSION || algo == RGPU_ALGO_VP) && max_steps > kMaxSteps - 1)
    return fail(c, RGPU_EINVAL, "max_steps above 127");
  if (algo == RGPU_ALGO_PR && (pr_iters < 0 || pr_iters > 100000))
    return fail(c, RGPU_EINVAL, "bad pr_iters");
  for (size_t i = 0; i < n_hops; i++)
    if (hops[i] < 0 || hops[i] >= ((int64_t)1 << 61)) return fail(c, RGPU_EINVAL, "hop time out of range");
  RunCfg rc;
  rc.algo = algo;
  rc.max_steps = max_steps;
  rc.pr_iters = pr_iters;
  rc.flags = flags;
  rc.W = n_w ? (int)n_w : 1;
  // window-major batches when they pay: each window's views in their own batches (64 hops),
  // so the cheap short windows no longer ride along the long windows' supersteps (not when all
  // views fit one hop-major batch, e.g. a live query of the newest hop)
  const bool wm = c->wmajor && (!c->partitioned || algo == RGPU_ALGO_CC) && rc.W >= 2 && rc.W <= kMaxPlanes &&
                  n_hops * (size_t)rc.W > (size_t)kViews;  // else one hop-major batch holds every view
  rc.G = wm ? rc.W : 1;
  rc.gsize = wm ? 1 : rc.W;
  rc.K = kViews / rc.gsize;
  rc.nblk = (n_hops + rc.K - 1) / rc.K;
  rc.nb = rc.nblk * rc.G;
  rc.hops = hops;
  rc.n_hops = n_hops;
  int64_t run_min = INT64_MAX;
  for (int w = 0; w < rc.W; w++) {
    int64_t wv = n_w ? windows[w] : INT64_MAX;  // ViewLens = no window (aliveAt)
    if (wv < 0) return fail(c, RGPU_EINVAL, "negative window");
    for (int u = 0; u < w; u++)
      if (n_w && windows[u] == wv)
        return fail(c, RGPU_EINVAL,
                    "duplicate window in batch (the reference shares state between them, "
                    "VertexVisitor.scala:81-96; not supported)");
    run_min = std::min(run_min, wv);
    rc.thr_e[w] = wv;
    rc.wval[w] = n_w ? windows[w] : -1;
    rc.thr_v[w] = run_min;  // WindowLens.shrinkWindow keeps the running intersection
  }
  rc.chunk0 = kChunk0;
  rc.chunk = kChunk;
  // knobs re-read per run (profile passes and tests on one sealed graph)
  c->prof_lean = env_int("RGPU_PROF_LEAN", 0) != 0;
  c->inject_fail = env_int("RGPU_INJECT_FAIL", 0);
  {
    const char* e = std::getenv("RGPU_INJECT_FAIL");
    c->inject_rec = e && std::strcmp(e, "rec") == 0;
    c->inject_cnt = e && std::strcmp(e, "cnt") == 0;
  }
  c->dense = env_int("RGPU_DENSE", -1);  // < 0: by graph size (dense_div)
  c->k1_carry = env_int("RGPU_K1_CARRY", 1) != 0;
  c->ko = KernOpts();
  c->ko.step = env_int("RGPU_STEP_OPTS", c->ko.step);
  // (partitioned: 4 segments per wave and round — at P = 8 the hub threshold is low and most segments
  // are active in every superstep, so a wave walking 32 of them in turn was the launch: summed hub
  // kernels 138 -> 101 ms, slowest partition 79.4 -> 74.5 ms, profiles/r06/part_sim_hubpro_p8.jsonl)
  // The same holds for a smaller graph (below 2^24 vertices: a lower hub threshold, shorter windows):
  // the 1B stream's week slice, 21 hops x {w, d, h}, hub kernels 57.3 -> 15.0 ms over eight blocks with 4
  // (22.4 with 8; profiles/r06/part_sim_replica_ab_1b.jsonl); its month slice (8.49M vertices), 168 hops
  // x {m, w, d, h}, 43.5 -> 17.0 ms (part_sim_replica_month_ab_1b.jsonl).  The 1B graph (19.9M) keeps 32.
  c->ko.hub_pro = env_int("RGPU_HUB_PRO", (c->partitioned || c->g.nv < ((int64_t)1 << 24)) ? kHubProPart
                                                                                         : c->ko.hub_pro);
  c->ko.long_steps = env_int("RGPU_LONG_STEPS", c->ko.long_steps);
  c->long_ratio = env_int("RGPU_LONG_RATIO", 4);
  try {
    HIPCHK(hipSetDevice(c->device));
    apply_pending(c);  // a run sees every seal that finished before it started
    {
      const auto ta = std::chrono::steady_clock::now();
      ensure_slots(c, algo, run_slots(c, rc));
      ensure_masks(c, rc.G, run_slots(c, rc));
      if (c->partitioned) ensure_part(c, run_slots(c, rc), rc.G);
      if (c->hostprof) {
        HIPCHK(hipDeviceSynchronize());
        std::fprintf(stderr, "rgpu hostprof: ensure buffers %.2f ms\n",
                     std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - ta).count());
      }
    }
    const size_t nb = rc.nb;
    c->algo = algo;
    c->vp_run_fsum = algo == RGPU_ALGO_VP && c->vp.fsum;  // the retained states' kind (rgpu_vp_result[_f])
    c->K = rc.K;
    c->W = rc.W;
    c->G = rc.G;
    c->gsize = rc.gsize;
    for (int& x : c->grp_last) x = 0;
    c->n_hops = n_hops;
    c->cc.assign(algo == RGPU_ALGO_CC ? n_hops * rc.W : 0, rgpu_cc_summary_t{});
    c->vlast.assign((algo == RGPU_ALGO_CC || algo == RGPU_ALGO_VP) ? n_hops * rc.W : 0, 0);
    c->st.alive_edge_windows = -1;
    if (c->d_ecnt) { (void)hipFree(c->d_ecnt); c->d_ecnt = nullptr; }
    if (flags & RGPU_RUN_EDGE_COUNTS) {
      HIPCHK(hipMalloc(&c->d_ecnt, sizeof(unsigned long long) * n_hops * rc.W));
      HIPCHK(hipMemset(c->d_ecnt, 0, sizeof(unsigned long long) * n_hops * rc.W));
    }
    if (algo == RGPU_ALGO_DEGREE || algo == RGPU_ALGO_DIFFUSION || algo == RGPU_ALGO_VP)
      if (int e = sync_vid(c)) return e;  // (seed ranks and top lists name ids)
    c->deg.assign(algo == RGPU_ALGO_DEGREE ? n_hops * rc.W * 3 : 0, 0);
    c->degtop.assign(algo == RGPU_ALGO_DEGREE ? n_hops * rc.W * kTop : 0, rgpu_ctx::TopEnt{-1, 0, 0});
    c->dcount.assign(algo == RGPU_ALGO_DIFFUSION ? n_hops * rc.W : 0, 0);
    c->dsteps.assign(algo == RGPU_ALGO_DIFFUSION ? n_hops * rc.W : 0, 0);
    if (algo == RGPU_ALGO_DIFFUSION || algo == RGPU_ALGO_VP) {
      // the seed's rank by binary search over the ids in ascending order (-1: not in the graph)
      const auto& vid = c->pk.vid;
      const int64_t seed = algo == RGPU_ALGO_VP ? c->vp_seed_id : c->diff_seed;
      int64_t a = 0, b = c->pk.n_own;
      while (a < b) {
        const int64_t m = (a + b) / 2;
        if (vid[own_at(c, m)] < seed) a = m + 1; else b = m;
      }
      const int64_t rk = (a < c->pk.n_own && vid[own_at(c, a)] == seed) ? own_at(c, a) : -1;
      if (algo == RGPU_ALGO_VP) c->vp.seed_rank = rk; else c->diff_seed_rank = rk;
      if (c->g.nv) HIPCHK(hipMemcpy(c->d_vid, vid.data(), sizeof(int64_t) * c->g.nv, hipMemcpyHostToDevice));
    }
    c->kept.clear();
    c->retained = (flags & RGPU_RUN_RETAIN) != 0;
    if (c->retained) c->kept.resize(nb);
    c->profile = (flags & RGPU_RUN_PROFILE) != 0;
    c->evused = 0;
    c->timed.clear();
    for (int k = 0; k < KID_N; k++) { c->st.kernel_launches[k] = 0; c->st.kernel_ms[k] = 0; c->st.kernel_bytes[k] = 0; }
    c->st.views = c->st.batches = c->st.supersteps = 0;
    // the buffers above were allocated and cleared on the null stream, which does not order
    // the batch slots' non-blocking streams: everything lands before the first batch kernel
    HIPCHK(hipDeviceSynchronize());
    auto t0 = std::chrono::steady_clock::now();
    c->pt.bytes_sent = 0;
    for (XSlot& xs : c->pt.xs) xs.bytes[0] = xs.bytes[1] = xs.bytes[2] = 0;
    if (c->partitioned && algo == RGPU_ALGO_CC) run_partitioned_cc(c, rc);
    else if (c->partitioned && algo == RGPU_ALGO_VP) run_partitioned_vp(c, rc);
    else if (c->partitioned) run_partitioned_dp(c, rc);
    else run_impl(c, rc);
    for (int si = 0; si < kMaxSlots; si++)
      if (c->slot[si].stream) HIPCHK(hipStreamSynchronize(c->slot[si].stream));
    if (algo == RGPU_ALGO_CC) finish_supersteps(c, rc);
    if (algo == RGPU_ALGO_VP) {  // per hop, as CC's: min(maxSteps, 1 + the last changing step of its windows)
      c->vpsteps.assign(n_hops, 0);
      for (size_t hop = 0; hop < n_hops; hop++) {
        int32_t r = 0;
        for (int w = 0; w < rc.W; w++) r = std::max(r, c->vlast[hop * rc.W + w]);
        c->vpsteps[hop] = max_steps <= 1 ? 0 : std::min<int64_t>(max_steps, (int64_t)r + 1);
      }
    }
    for (int k = 0; k < 4; k++) c->st.xchg_bytes_by[k] = 0;
    c->st.xchg_bytes_by[3] = c->pt.bytes_sent;
    for (const XSlot& xs : c->pt.xs)
      for (int k = 0; k < 3; k++) c->st.xchg_bytes_by[k] += xs.bytes[k];
    c->st.xchg_bytes = 0;
    for (int k = 0; k < 4; k++) c->st.xchg_bytes += c->st.xchg_bytes_by[k];
    if (c->d_ecnt) {  // |E_{t,w}| per view (RGPU_RUN_EDGE_COUNTS)
      std::vector<unsigned long long> e(n_hops * rc.W);
      HIPCHK(hipMemcpy(e.data(), c->d_ecnt, sizeof(unsigned long long) * e.size(), hipMemcpyDeviceToHost));
      if (c->partitioned && c->nparts > 1) {
        HIPCHK(hipMemcpy(c->d_ecnt, e.data(), sizeof(unsigned long long) * e.size(), hipMemcpyHostToDevice));
        c->pt.xchg->allreduce_u64(c->d_ecnt, e.size(), false, c->slot[0].stream);
        HIPCHK(hipStreamSynchronize(c->slot[0].stream));
        HIPCHK(hipMemcpy(e.data(), c->d_ecnt, sizeof(unsigned long long) * e.size(), hipMemcpyDeviceToHost));
      }
      c->st.alive_edge_windows = 0;
      for (size_t i = 0; i < e.size(); i++) {
        c->st.alive_edge_windows += (int64_t)e[i];
        if (algo == RGPU_ALGO_CC) c->cc[i].alive_edges = (int64_t)e[i];
      }
      (void)hipFree(c->d_ecnt);
      c->d_ecnt = nullptr;
    } else if (algo == RGPU_ALGO_CC) {
      for (auto& o : c->cc) o.alive_edges = -1;
    }
    auto t1 = std::chrono::steady_clock::now();
    c->st.ms_total = std::chrono::duration<double, std::milli>(t1 - t0).count();
    c->st.launches = 0;
    for (int k = 0; k < KID_N; k++) c->st.launches += c->st.kernel_launches[k];
    FILE* tf = nullptr;
    if (!c->trace_path.empty() && (tf = std::fopen(c->trace_path.c_str(), "w")))
      std::fprintf(tf, "kind,batch,step,kernel,ms,pv,ps,changed,pg\n");
    for (const Timed& tm : c->timed) {
      float ms = 0;
      HIPCHK(hipEventElapsedTime(&ms, tm.a, tm.b));
      c->st.kernel_ms[tm.kid] += ms;
      if (tf) std::fprintf(tf, "L,%d,%d,%d,%.4f,,,,\n", tm.batch, tm.step, tm.kid, ms);
    }
    if (tf) {
      for (const auto& r : c->steprec)
        std::fprintf(tf, "S,%d,%d,,,%llu,%llu,%d,%llu\n", r.batch, r.step, r.pv, r.ps, r.changed, r.pg);
      std::fclose(tf);
    }
    c->steprec.clear();
    // (after the run's last collective, so that every partition has left the exchange)
    if (c->partitioned) {  // received label records outside the exchange plan (xchg.hip bc_rec): a bug upstream
      unsigned long long bad = 0;
      for (const XSlot& xs : c->pt.xs)
        if (xs.err) {
          unsigned long long e = 0;
          HIPCHK(hipMemcpy(&e, xs.err, sizeof(e), hipMemcpyDeviceToHost));
          bad += e;
        }
      if (bad)
        throw HipFail{"exchange: " + std::to_string(bad) + " received label records outside the receive plan"};
      if (c->pt.own.err) {  // component counts of labels routed here that no owned vertex holds (xchg.hip label_row)
        unsigned long long e = 0;
        HIPCHK(hipMemcpy(&e, c->pt.own.err, sizeof(e), hipMemcpyDeviceToHost));
        if (e)
          throw HipFail{"component counts: " + std::to_string(e) + " lookups of a label routed here found no owned vertex"};
      }
    }
  } catch (const HipFail& f) {
    exchange_quiesce();
    reset_after_failure(c);
    return fail(c, RGPU_EHIP, f.msg);
  } catch (const std::bad_alloc&) {
    exchange_quiesce();
    reset_after_failure(c);
    return fail(c, RGPU_ENOMEM, "host allocation failed");
  } catch (const std::exception& x) {  // exchange (RCCL / loopback) failures
    exchange_quiesce();
    reset_after_failure(c);
    return fail(c, RGPU_EHIP, x.what());
  }
  exchange_quiesce();
  return RGPU_OK;
}



static int view_index(rgpu_ctx* c, size_t hop, size_t win, size_t* batch, int* lane) {
  if (hop >= c->n_hops || win >= (size_t)c->W) return fail(c, RGPU_EINVAL, "view index out of range");
  *batch = (hop / c->K) * c->G + win / c->gsize;
  *lane = (int)((win % c->gsize) * c->K + hop % c->K);
  return RGPU_OK;
}

int rgpu_cc_summary(rgpu_ctx* c, size_t hop, size_t win, rgpu_cc_summary_t* out) {
  if (!c || !out) return RGPU_EINVAL;
  std::lock_guard<std::mutex> lk(c->mu);
  if (c->algo != RGPU_ALGO_CC) return fail(c, RGPU_ESTATE, "last run was not CC");
  size_t b;
  int j;
  if (int e = view_index(c, hop, win, &b, &j)) return e;
  *out = c->cc[hop * c->W + win];
  return RGPU_OK;
}

int rgpu_cc_vertex_labels(rgpu_ctx* c, size_t hop, size_t win, int64_t* ids, int64_t* labels,
                          size_t cap, size_t* n) {
  if (!c || !n) return RGPU_EINVAL;
  std::lock_guard<std::mutex> lk(c->mu);
  if (c->algo != RGPU_ALGO_CC || !c->retained) return fail(c, RGPU_ESTATE, "needs a CC run with RGPU_RUN_RETAIN");
  size_t b;
  int j;
  if (int e = view_index(c, hop, win, &b, &j)) return e;
  const Retained& R = c->kept[b];
  if (int e = sync_vid(c)) return e;
  size_t k = 0;
  for (int64_t k_ = 0; k_ < c->pk.n_own; k_++) {
    const int64_t v = own_at(c, k_);
    if (!((R.vm[v] >> j) & 1)) continue;
    if (k < cap) {
      ids[k] = c->pk.vid[v];
      labels[k] = label_id(c, R.a[(size_t)v * kViews + j]);
    }
    k++;
  }
  *n = k;
  return RGPU_OK;
}

int rgpu_cc_result(rgpu_ctx* c, size_t hop, size_t win, int64_t* labels, int32_t* counts,
                   size_t cap, size_t* n) {
  if (!c || !n) return RGPU_EINVAL;
  std::lock_guard<std::mutex> lk(c->mu);
  if (c->algo != RGPU_ALGO_CC || !c->retained) return fail(c, RGPU_ESTATE, "needs a CC run with RGPU_RUN_RETAIN");
  size_t b;
  int j;
  if (int e = view_index(c, hop, win, &b, &j)) return e;
  const Retained& R = c->kept[b];
  if (int e = sync_vid(c)) return e;
  std::vector<int32_t> lab;
  for (int64_t v = 0; v < c->pk.n_own; v++)  // (any order: sorted below)
    if ((R.vm[v] >> j) & 1) lab.push_back(R.a[(size_t)v * kViews + j]);
  std::sort(lab.begin(), lab.end());
  size_t k = 0;
  for (size_t i = 0; i < lab.size();) {
    size_t h = i;
    while (h < lab.size() && lab[h] == lab[i]) h++;
    if (k < cap) { labels[k] = label_id(c, lab[i]); counts[k] = (int32_t)(h - i); }
    k++;
    i = h;
  }
  *n = k;
  return RGPU_OK;
}

int rgpu_degree_vertex(rgpu_ctx* c, size_t hop, size_t win, int64_t* ids, int32_t* outdeg,
                       int32_t* indeg, size_t cap, size_t* n) {
  if (!c || !n) return RGPU_EINVAL;
  std::lock_guard<std::mutex> lk(c->mu);
  if (c->algo != RGPU_ALGO_DEGREE || !c->retained) return fail(c, RGPU_ESTATE, "needs a degree run with RGPU_RUN_RETAIN");
  size_t b;
  int j;
  if (int e = view_index(c, hop, win, &b, &j)) return e;
  const Retained& R = c->kept[b];
  if (int e = sync_vid(c)) return e;
  size_t k = 0;
  for (int64_t k_ = 0; k_ < c->pk.n_own; k_++) {
    const int64_t v = own_at(c, k_);
    if (!((R.vm[v] >> j) & 1)) continue;
    if (k < cap) {
      ids[k] = c->pk.vid[v];
      outdeg[k] = R.a[(size_t)v * kViews + j];
      indeg[k] = R.b[(size_t)v * kViews + j];
    }
    k++;
  }
  *n = k;
  return RGPU_OK;
}

int rgpu_degree_result(rgpu_ctx* c, size_t hop, size_t win, int64_t tot[3], int64_t* top_id,
                       int32_t* top_out, int32_t* top_in) {
  if (!c || !tot) return RGPU_EINVAL;
  std::lock_guard<std::mutex> lk(c->mu);
  if (c->algo != RGPU_ALGO_DEGREE) return fail(c, RGPU_ESTATE, "last run was not degree");
  size_t b;
  int j;
  if (int e = view_index(c, hop, win, &b, &j)) return e;
  for (int f = 0; f < 3; f++) tot[f] = c->deg[(hop * c->W + win) * 3 + f];
  if (top_id && top_out && top_in) {  // the device top-20 (k_deg_top_merge), ties by ascending id
    for (int i = 0; i < kTop; i++) {
      const rgpu_ctx::TopEnt& e = c->degtop[(hop * c->W + win) * kTop + i];
      top_id[i] = e.id;
      top_out[i] = e.id < 0 ? 0 : e.out;
      top_in[i] = e.id < 0 ? 0 : e.in;
    }
  }
  return RGPU_OK;
}

int rgpu_pr_result(rgpu_ctx* c, size_t hop, size_t win, int64_t* ids, double* pr, size_t cap,
                   size_t* n) {
  if (!c || !n) return RGPU_EINVAL;
  std::lock_guard<std::mutex> lk(c->mu);
  if (c->algo != RGPU_ALGO_PR || !c->retained) return fail(c, RGPU_ESTATE, "needs a PR run with RGPU_RUN_RETAIN");
  size_t b;
  int j;
  if (int e = view_index(c, hop, win, &b, &j)) return e;
  const Retained& R = c->kept[b];
  if (int e = sync_vid(c)) return e;
  size_t k = 0;
  for (int64_t k_ = 0; k_ < c->pk.n_own; k_++) {
    const int64_t v = own_at(c, k_);
    if (!((R.vm[v] >> j) & 1)) continue;
    if (k < cap) { ids[k] = c->pk.vid[v]; pr[k] = R.pr[(size_t)v * kViews + j]; }
    k++;
  }
  *n = k;
  return RGPU_OK;
}

int rgpu_set_diffusion(rgpu_ctx* c, int64_t seed_id, uint64_t coin_seed, int coin) {
  if (!c) return RGPU_EINVAL;
  std::lock_guard<std::mutex> lk(c->mu);
  c->diff_seed = seed_id;
  c->diff_coin_seed = coin_seed;
  c->diff_coin = coin ? 1 : 0;
  return RGPU_OK;
}

int rgpu_diffusion_result(rgpu_ctx* c, size_t hop, size_t win, int64_t* infected, int64_t* supersteps) {
  if (!c) return RGPU_EINVAL;
  std::lock_guard<std::mutex> lk(c->mu);
  if (c->algo != RGPU_ALGO_DIFFUSION) return fail(c, RGPU_ESTATE, "last run was not diffusion");
  size_t b;
  int j;
  if (int e = view_index(c, hop, win, &b, &j)) return e;
  if (infected) *infected = c->dcount[hop * c->W + win];
  if (supersteps) *supersteps = c->dsteps[hop * c->W + win];
  return RGPU_OK;
}

int rgpu_diffusion_vertex(rgpu_ctx* c, size_t hop, size_t win, int64_t* ids, int32_t* steps, size_t cap,
                          size_t* n) {
  if (!c || !n) return RGPU_EINVAL;
  std::lock_guard<std::mutex> lk(c->mu);
  if (c->algo != RGPU_ALGO_DIFFUSION || !c->retained)
    return fail(c, RGPU_ESTATE, "needs a diffusion run with RGPU_RUN_RETAIN");
  size_t b;
  int j;
  if (int e = view_index(c, hop, win, &b, &j)) return e;
  const Retained& R = c->kept[b];
  if (int e = sync_vid(c)) return e;
  size_t k = 0;
  for (int64_t k_ = 0; k_ < c->pk.n_own; k_++) {
    const int64_t v = own_at(c, k_);
    const uint8_t r = R.st[(size_t)v * kViews + j];
    if (r == 0xFF) continue;  // returnResults keeps infected vertices only (:43-49)
    if (k < cap) { ids[k] = c->pk.vid[v]; steps[k] = r; }
    k++;
  }
  *n = k;
  return RGPU_OK;
}

int rgpu_set_vertex_program(rgpu_ctx* c, const rgpu_vertex_program_t* p) {
  if (!c || !p) return RGPU_EINVAL;
  std::lock_guard<std::mutex> lk(c->mu);
  if (p->direction < RGPU_VP_OUT || p->direction > RGPU_VP_ALL || p->reduce < RGPU_VP_MIN || p->reduce > RGPU_VP_MAX ||
      p->init < RGPU_VP_INIT_ID || p->init > RGPU_VP_INIT_VALUE || p->senders < RGPU_VP_SEND_ALL ||
      p->senders > RGPU_VP_SEND_SEED)
    return fail(c, RGPU_EINVAL, "bad vertex program");
  c->vp = VpParams();
  c->vp.dir = p->direction;
  c->vp.reduce = p->reduce;
  c->vp.init = p->init;
  c->vp.senders = p->senders;
  c->vp.init_value = p->init_value;
  c->vp.seed_value = p->seed_value;
  c->vp.step_add = p->step_add;
  c->vp_seed_id = p->seed_id;
  c->vp_set = true;
  return RGPU_OK;
}

static int vp_result_rows(rgpu_ctx* c, size_t hop, size_t win, int64_t* ids, int64_t* values, size_t cap, size_t* n);

int rgpu_vp_result(rgpu_ctx* c, size_t hop, size_t win, int64_t* ids, int64_t* values, size_t cap, size_t* n) {
  if (!c || !n) return RGPU_EINVAL;
  std::lock_guard<std::mutex> lk(c->mu);
  if (c->algo != RGPU_ALGO_VP || !c->retained) return fail(c, RGPU_ESTATE, "needs a vertex-program run with RGPU_RUN_RETAIN");
  // the kind of the program the retained run ran (not the one set since): int64 states here
  if (c->vp_run_fsum) return fail(c, RGPU_ESTATE, "the last vertex-program run was a float program (rgpu_vp_result_f)");
  return vp_result_rows(c, hop, win, ids, values, cap, n);
}

// (caller holds mu; the run's program kind checked)
static int vp_result_rows(rgpu_ctx* c, size_t hop, size_t win, int64_t* ids, int64_t* values, size_t cap, size_t* n) {
  size_t b;
  int j;
  if (int e = view_index(c, hop, win, &b, &j)) return e;
  const Retained& R = c->kept[b];
  if (int e = sync_vid(c)) return e;
  size_t k = 0;
  for (int64_t k_ = 0; k_ < c->pk.n_own; k_++) {
    const int64_t v = own_at(c, k_);
    if (!((R.vm[v] >> j) & 1)) continue;
    if (k < cap) { ids[k] = c->pk.vid[v]; values[k] = R.v64[(size_t)v * kViews + j]; }
    k++;
  }
  *n = k;
  return RGPU_OK;
}

int rgpu_set_vertex_program_f(rgpu_ctx* c, const rgpu_vertex_program_f_t* p) {
  if (!c || !p) return RGPU_EINVAL;
  std::lock_guard<std::mutex> lk(c->mu);
  if ((p->direction != RGPU_VP_OUT && p->direction != RGPU_VP_IN) || p->init < RGPU_VP_INIT_ID ||
      p->init > RGPU_VP_INIT_VALUE || p->senders < RGPU_VP_SEND_ALL || p->senders > RGPU_VP_SEND_SEED ||
      (p->per_degree != 0 && p->per_degree != 1))
    return fail(c, RGPU_EINVAL, "bad float vertex program (direction OUT or IN)");
  c->vp = VpParams();
  c->vp.dir = p->direction;
  c->vp.init = p->init;
  c->vp.senders = p->senders;
  c->vp.fsum = 1;
  c->vp.per_degree = p->per_degree;
  c->vp.f_init = p->init_value;
  c->vp.f_seed = p->seed_value;
  c->vp.f_bias = p->bias;
  c->vp.f_mult = p->mult;
  c->vp_seed_id = p->seed_id;
  c->vp_set = true;
  return RGPU_OK;
}

int rgpu_vp_result_f(rgpu_ctx* c, size_t hop, size_t win, int64_t* ids, double* values, size_t cap, size_t* n) {
  if (!c || !n) return RGPU_EINVAL;
  std::lock_guard<std::mutex> lk(c->mu);
  if (c->algo != RGPU_ALGO_VP || !c->retained) return fail(c, RGPU_ESTATE, "needs a vertex-program run with RGPU_RUN_RETAIN");
  if (!c->vp_run_fsum) return fail(c, RGPU_ESTATE, "the last vertex-program run was not a float program");
  static_assert(sizeof(double) == sizeof(int64_t), "state rows hold double bits");
  return vp_result_rows(c, hop, win, ids, reinterpret_cast<int64_t*>(values), cap, n);
}

int rgpu_vp_supersteps(rgpu_ctx* c, size_t hop, int64_t* supersteps) {
  if (!c || !supersteps) return RGPU_EINVAL;
  std::lock_guard<std::mutex> lk(c->mu);
  if (c->algo != RGPU_ALGO_VP) return fail(c, RGPU_ESTATE, "last run was not a vertex program");
  if (hop >= c->vpsteps.size()) return fail(c, RGPU_EINVAL, "hop index out of range");
  *supersteps = c->vpsteps[hop];
  return RGPU_OK;
}

int rgpu_stats(rgpu_ctx* c, rgpu_stats_t* out) {
  if (!c || !out) return RGPU_EINVAL;
  std::lock_guard<std::mutex> lk(c->mu);
  *out = c->st;
  return RGPU_OK;
}

const char* rgpu_last_error(rgpu_ctx* c) { return c ? c->err.c_str() : "null context"; }

void rgpu_close(rgpu_ctx* c) {
  if (!c) return;
  {
    std::lock_guard<std::mutex> sl(c->seal_mu);
    std::lock_guard<std::mutex> lk(c->mu);
    (void)hipSetDevice(c->device);
    for (Slot& s : c->slot)
      if (s.stream) (void)hipStreamSynchronize(s.stream);
    free_graph(c);
    free_part_slots(c, false);
    delete c->pt.xchg;
    c->pt.xchg = nullptr;
    for (hipEvent_t e : c->evpool) (void)hipEventDestroy(e);
  }
  delete c;
}

}  // extern "C"
