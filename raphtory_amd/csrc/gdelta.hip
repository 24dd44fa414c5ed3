// gdelta.hip — the live-ingest delta packer on the device.
//
// The same arrays as the host half (packer.cpp pack_delta + finish_delta, which stays as the
// RGPU_DELTA=2 A/B path and the CPU tests' subject), built in HBM from the raw updates by stable
// radix sorts, scans and position formulas, so that a 10M-update tick never leaves the device
// after its upload.  The reference appends each update to its entity's TreeMap as it arrives
// (EntityStorage.scala:73-453, Entity.scala:25-57: at equal times the later put wins); the
// arrays below are what pack_events would build from base + delta, which tests/test_gpu_live.py
// checks against the oracle and against the host half.
//
//   ids      every (update, endpoint) slot sorted by id; distinct ids, the ones not in the base,
//            and both rank maps by position formulas (base id a lands at a + #(new ids below it),
//            new id j at j + #(base ids below it))
//   order    updates by (time, stream index): the identity for a time-ordered tick (the usual
//            live case), else one stable 61-bit radix sort; every later sort is stable, so each
//            entity's points come out by (time, index)
//   vpoints  (rank, endpoint) records sorted by rank, collapsed per (rank, time): last put wins
//   deaths   VertexDelete records by rank: distinct times with the last delta index
//   epoints  edge updates sorted by (src, dst) = src * nv + dst; groups = delta edges
//   keys     per delta edge its collapsed points with the endpoint-death tie resolved (count,
//            scan, write), new edges and their in-edge records (sorted by (dst, src))
//   offsets  merged out / in offsets (base counts + new edges, one scan each), adjacency
//            offsets, merged death lists and death bits, and the heavy-vertex candidates
// Irregular integer work: HBM- and sort-bound, a few passes over the tick's 32-B updates.
#include <hip/hip_runtime.h>

#include <hipcub/device/device_radix_sort.hpp>
#include <hipcub/device/device_scan.hpp>
#include <hipcub/device/device_select.hpp>

#include <algorithm>
#include <climits>
#include <cstdint>
#include <stdexcept>
#include <string>

#include "../../include/rgpu.h"
#include "kernels.hpp"

namespace rgpu {
namespace {

constexpr int kB = 256;
constexpr int64_t kMaxT = (int64_t)1 << 61;

inline unsigned gridn(int64_t n) {
  int64_t b = (n + kB - 1) / kB;
  if (b > 65536) b = 65536;
  return (unsigned)(b < 1 ? 1 : b);
}
#define GLOOP(i, n) for (int64_t i = blockIdx.x * (int64_t)kB + threadIdx.x; i < (n); i += (int64_t)gridDim.x * kB)

inline void chk(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string("gpu_pack_delta ") + what + ": " + hipGetErrorString(e));
}
#define GCHK(x) chk((x), #x)

int bits_for(uint64_t x) {  // bits to hold values up to x
  int b = 1;
  while (b < 64 && (x >> b)) b++;
  return b;
}

// device allocations (T: temporaries, L: the merged graph) and one grow-only temp buffer for
// the hipcub passes (stream-ordered, so one buffer serves them all)
struct Mem {
  std::vector<void*>& T;
  std::vector<void*>& L;
  void* tmp = nullptr;
  size_t tmp_bytes = 0;
  template <class X>
  X* alloc(int64_t n, bool graph = false) {
    void* p = nullptr;
    GCHK(hipMalloc(&p, sizeof(X) * (size_t)std::max<int64_t>(n, 1)));
    (graph ? L : T).push_back(p);
    return (X*)p;
  }
  void* temp(size_t b) {
    if (b > tmp_bytes) {
      tmp_bytes = b + b / 4 + 256;
      tmp = alloc<char>((int64_t)tmp_bytes);
    }
    return tmp;
  }
};

template <class K, class V>
void sort_pairs(Mem& M, hipStream_t s, const K* kin, K* kout, const V* vin, V* vout, int64_t n, int end_bit) {
  if (n <= 0) return;
  size_t b = 0;
  GCHK(hipcub::DeviceRadixSort::SortPairs(nullptr, b, kin, kout, vin, vout, (int)n, 0, end_bit, s));
  void* t = M.temp(b);
  GCHK(hipcub::DeviceRadixSort::SortPairs(t, b, kin, kout, vin, vout, (int)n, 0, end_bit, s));
}
// exclusive sum of n items into out[0, n)
template <class I, class O>
void excl_sum(Mem& M, hipStream_t s, const I* in, O* out, int64_t n) {
  if (n <= 0) return;
  size_t b = 0;
  GCHK(hipcub::DeviceScan::ExclusiveSum(nullptr, b, in, out, (int)n, s));
  void* t = M.temp(b);
  GCHK(hipcub::DeviceScan::ExclusiveSum(t, b, in, out, (int)n, s));
}
template <class X>
X fetch(hipStream_t s, const X* p) {
  X x{};
  GCHK(hipMemcpyAsync(&x, p, sizeof(X), hipMemcpyDeviceToHost, s));
  GCHK(hipStreamSynchronize(s));
  return x;
}

// first index in a[0, n) with a[i] >= x
template <class A, class X>
__device__ __forceinline__ int64_t lower(const A* __restrict__ a, int64_t n, X x) {
  int64_t lo = 0, hi = n;
  while (lo < hi) {
    const int64_t m = (lo + hi) >> 1;
    if (a[m] < x) lo = m + 1;
    else hi = m;
  }
  return lo;
}

// ---- validation, order flag, kind counts: err = min over invalid updates of (index << 2 | code)
// with the host packer's check order (kind, time, source, destination); cnt[0] = out-of-order
// pairs seen, cnt[1] = VertexDeletes, cnt[2] = edge updates
__global__ __launch_bounds__(kB) void k_validate(int64_t n, const DevEvent* __restrict__ ev,
                                                 unsigned long long* __restrict__ err,
                                                 unsigned long long* __restrict__ cnt) {
  unsigned long long un = 0, del = 0, edg = 0;
  GLOOP(i, n) {
    const DevEvent e = ev[i];
    int code = 0;
    if (e.kind > RGPU_EDEL) code = 1;
    else if (e.t < 0 || e.t >= kMaxT) code = 2;
    else if (e.src < 0 || e.src > INT32_MAX) code = 3;
    else if (e.kind >= RGPU_EADD && (e.dst < 0 || e.dst > INT32_MAX)) code = 3;
    if (code) atomicMin(err, ((unsigned long long)i << 2) | (unsigned long long)code);
    un += i > 0 && e.t < ev[i - 1].t;
    del += e.kind == RGPU_VDEL;
    edg += e.kind >= RGPU_EADD && e.kind <= RGPU_EDEL;
  }
  for (int o = 32; o > 0; o >>= 1) {
    un += __shfl_xor(un, o);
    del += __shfl_xor(del, o);
    edg += __shfl_xor(edg, o);
  }
  if ((threadIdx.x & 63) == 0) {
    if (un) atomicAdd(&cnt[0], un);
    if (del) atomicAdd(&cnt[1], del);
    if (edg) atomicAdd(&cnt[2], edg);
  }
}

// ---- ids
constexpr uint32_t kNoId = 0x80000000u;  // above every id (ids are < 2^31)
__global__ __launch_bounds__(kB) void k_id_slots(int64_t n, const DevEvent* __restrict__ ev, uint32_t* __restrict__ key,
                                                 uint32_t* __restrict__ val) {
  GLOOP(i, n) {
    const DevEvent e = ev[i];
    key[2 * i] = (uint32_t)e.src;
    val[2 * i] = (uint32_t)(2 * i);
    key[2 * i + 1] = e.kind >= RGPU_EADD ? (uint32_t)e.dst : kNoId;
    val[2 * i + 1] = (uint32_t)(2 * i + 1);
  }
}
// head[p] = slot p starts a run of equal ids (head[m] = 0: the scan's total lands at m)
__global__ __launch_bounds__(kB) void k_heads(int64_t m, const uint32_t* __restrict__ key, int32_t* __restrict__ head) {
  GLOOP(p, m + 1) head[p] = p < m && key[p] != kNoId && (p == 0 || key[p] != key[p - 1]);
}
__global__ __launch_bounds__(kB) void k_ids(int64_t m, const uint32_t* __restrict__ key, const int32_t* __restrict__ head,
                                            const int32_t* __restrict__ pos, int64_t* __restrict__ ids) {
  GLOOP(p, m) if (head[p]) ids[pos[p]] = key[p];
}
// ---- partition roles (partitioned mode: pack_events' owned / ghost / not kept).  Owner of an id:
// Utils.getPartition (rgpu_internal.hpp partition_of); nparts = 0: one partition, all owned.
// Rank order = ascending key, key = id for owned vertices and kGhost | id for ghosts (owned by
// id, then ghosts by id), so both rank maps stay monotone and the position formulas hold.
constexpr int64_t kGhost = (int64_t)1 << 31;
__device__ __forceinline__ bool owned_id(int64_t id, int part, int nparts) {
  return nparts <= 0 || (int)((id % (10 * (int64_t)nparts)) / 10) == part;
}
// a non-owned endpoint of an edge update whose other endpoint is owned is kept as a ghost
__global__ __launch_bounds__(kB) void k_ghost_need(int64_t m, const uint32_t* __restrict__ key,
                                                   const uint32_t* __restrict__ val, const int32_t* __restrict__ head,
                                                   const int32_t* __restrict__ pos, const DevEvent* __restrict__ ev,
                                                   int part, int nparts, uint8_t* __restrict__ need) {
  GLOOP(p, m) {
    if (key[p] == kNoId) continue;
    const uint32_t slot = val[p];
    const DevEvent e = ev[slot >> 1];
    if (e.kind < RGPU_EADD || e.src == e.dst) continue;
    const int64_t me = (slot & 1) ? e.dst : e.src, other = (slot & 1) ? e.src : e.dst;
    if (!owned_id(me, part, nparts) && owned_id(other, part, nparts)) need[pos[p] + head[p] - 1] = 1;
  }
}
// per distinct delta id: its rank-order key (-1: not kept here) and whether it is new
__global__ __launch_bounds__(kB) void k_roles(int64_t nid, const int64_t* __restrict__ ids,
                                              const int64_t* __restrict__ vid0, int64_t nv_old, int part, int nparts,
                                              const uint8_t* __restrict__ need, int64_t* __restrict__ keyk,
                                              uint8_t* __restrict__ isnew) {
  GLOOP(k, nid) {
    const int64_t id = ids[k];
    const bool own = owned_id(id, part, nparts);
    const int64_t key = own ? id : (kGhost | id);
    const int64_t j = lower(vid0, nv_old, key);
    const bool inbase = j < nv_old && vid0[j] == key;
    const bool keep = own || inbase || (need && need[k]);
    keyk[k] = keep ? key : -1;
    isnew[k] = keep && !inbase;
  }
}
__global__ __launch_bounds__(kB) void k_count_below(int64_t n, const int64_t* __restrict__ a, int64_t x,
                                                    int64_t* __restrict__ out) {
  if (blockIdx.x == 0 && threadIdx.x == 0) *out = lower(a, n, x);
}
__global__ __launch_bounds__(kB) void k_place_old(int64_t nv_old, const int64_t* __restrict__ vid0,
                                                  const int64_t* __restrict__ nid, int64_t nnew, int64_t* __restrict__ vid2,
                                                  int32_t* __restrict__ old2new, int32_t* __restrict__ new2old) {
  GLOOP(a, nv_old) {
    const int64_t r = a + lower(nid, nnew, vid0[a]);
    vid2[r] = vid0[a];
    old2new[a] = (int32_t)r;
    new2old[r] = (int32_t)a;
  }
}
__global__ __launch_bounds__(kB) void k_place_new(int64_t nnew, const int64_t* __restrict__ nid,
                                                  const int64_t* __restrict__ vid0, int64_t nv_old,
                                                  int64_t* __restrict__ vid2, int32_t* __restrict__ new2old) {
  GLOOP(j, nnew) {
    const int64_t r = j + lower(vid0, nv_old, nid[j]);
    vid2[r] = nid[j];
    new2old[r] = -1;
  }
}
// every sorted slot p: its update's endpoint rank (the id's merged rank, a search in vid2 once
// per distinct id through the run head)
__global__ __launch_bounds__(kB) void k_idrank(int64_t nid, const int64_t* __restrict__ keyk, const int64_t* __restrict__ vid2,
                                               int64_t nv2, int32_t* __restrict__ idrank) {
  GLOOP(k, nid) idrank[k] = keyk[k] >= 0 ? (int32_t)lower(vid2, nv2, keyk[k]) : -1;
}
__global__ __launch_bounds__(kB) void k_ranks(int64_t m, const uint32_t* __restrict__ key, const uint32_t* __restrict__ val,
                                              const int32_t* __restrict__ head, const int32_t* __restrict__ pos,
                                              const int32_t* __restrict__ idrank, int32_t* __restrict__ rs,
                                              int32_t* __restrict__ rd) {
  GLOOP(p, m) {
    if (key[p] == kNoId) continue;
    const int32_t r = idrank[pos[p] + head[p] - 1];  // pos = exclusive sum of heads: the run's index
    const uint32_t slot = val[p];
    (slot & 1 ? rd : rs)[slot >> 1] = r;
  }
}

// ---- order: q -> update index (ord null: identity)
__global__ __launch_bounds__(kB) void k_time_keys(int64_t n, const DevEvent* __restrict__ ev, uint64_t* __restrict__ tk,
                                                  uint32_t* __restrict__ iv) {
  GLOOP(i, n) {
    tk[i] = (uint64_t)ev[i].t;
    iv[i] = (uint32_t)i;
  }
}
__device__ __forceinline__ int64_t ord_at(const uint32_t* __restrict__ ord, int64_t q) { return ord ? (int64_t)ord[q] : q; }

// ---- vertex points: record 2q = the update's source (not for EdgeDelete), 2q+1 = its
// destination (EdgeAdd, not a self-loop); value = 2i + endpoint
// (owned ranks only: a ghost's history lives on its owner)
__global__ __launch_bounds__(kB) void k_vrec(int64_t n, const DevEvent* __restrict__ ev, const uint32_t* __restrict__ ord,
                                             const int32_t* __restrict__ rs, const int32_t* __restrict__ rd, int64_t n_own,
                                             uint32_t sent, uint32_t* __restrict__ key, uint32_t* __restrict__ val) {
  GLOOP(q, n) {
    const int64_t i = ord_at(ord, q);
    const uint8_t kd = ev[i].kind;
    const int32_t a = rs[i], b = rd[i];
    key[2 * q] = (kd != RGPU_EDEL && a >= 0 && a < n_own) ? (uint32_t)a : sent;
    val[2 * q] = (uint32_t)(2 * i);
    key[2 * q + 1] = (kd == RGPU_EADD && b != a && b >= 0 && b < n_own) ? (uint32_t)b : sent;
    val[2 * q + 1] = (uint32_t)(2 * i + 1);
  }
}
// kept = the last record of its (rank, time) run; start = first record of its rank.  Index m:
// zeros (the scans' totals).  shift: value -> update index
__global__ __launch_bounds__(kB) void k_run_flags(int64_t m, const uint32_t* __restrict__ key,
                                                  const uint32_t* __restrict__ val, int shift, uint32_t sent,
                                                  const DevEvent* __restrict__ ev, int32_t* __restrict__ kept,
                                                  int32_t* __restrict__ start) {
  GLOOP(p, m + 1) {
    int32_t k = 0, st = 0;
    if (p < m && key[p] != sent) {
      st = p == 0 || key[p - 1] != key[p];
      k = !(p + 1 < m && key[p + 1] == key[p] && ev[val[p + 1] >> shift].t == ev[val[p] >> shift].t);
    }
    kept[p] = k;
    start[p] = st;
  }
}
__global__ __launch_bounds__(kB) void k_vfill(int64_t m, const uint32_t* __restrict__ key, const uint32_t* __restrict__ val,
                                              const DevEvent* __restrict__ ev, const int32_t* __restrict__ kept,
                                              const int32_t* __restrict__ start, const int64_t* __restrict__ kpos,
                                              const int64_t* __restrict__ spos, int32_t* __restrict__ dv_rank,
                                              int64_t* __restrict__ dv_off, int64_t* __restrict__ dv_key) {
  GLOOP(p, m) {
    if (start[p]) {
      dv_rank[spos[p]] = (int32_t)key[p];
      dv_off[spos[p]] = kpos[p];
    }
    if (kept[p]) {
      const uint32_t v = val[p];
      const DevEvent& e = ev[v >> 1];
      const int64_t f = (v & 1) ? 1 : (e.kind == RGPU_VDEL ? 0 : 1);
      dv_key[kpos[p]] = e.t * 2 + f;
    }
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) dv_off[spos[m]] = kpos[m];
}

// ---- deaths: the tick's VertexDeletes in (time, index) order, after the orphans (deaths of ids
// that were not kept here when they arrived: partitioned mode keeps every VertexDelete, and an id
// that later turns ghost needs its earlier deaths, which count as base deaths: last index 0)
__global__ __launch_bounds__(kB) void k_del_flags(int64_t n, const DevEvent* __restrict__ ev,
                                                  const uint32_t* __restrict__ ord, int32_t* __restrict__ f) {
  GLOOP(q, n + 1) f[q] = q < n && ev[ord_at(ord, q)].kind == RGPU_VDEL;
}
__global__ __launch_bounds__(kB) void k_del_list(int64_t n, const uint32_t* __restrict__ ord, const int32_t* __restrict__ f,
                                                 const int64_t* __restrict__ pos, uint32_t* __restrict__ delq) {
  GLOOP(q, n) if (f[q]) delq[pos[q]] = (uint32_t)ord_at(ord, q);
}
__global__ __launch_bounds__(kB) void k_orph_rec(int64_t no, const int64_t* __restrict__ oid, const int64_t* __restrict__ ot,
                                                 const int64_t* __restrict__ vid2, int64_t nv2, uint32_t sent,
                                                 uint64_t* __restrict__ rt, uint32_t* __restrict__ rrank,
                                                 int64_t* __restrict__ rlast, int64_t* __restrict__ rid,
                                                 uint32_t* __restrict__ perm) {
  GLOOP(k, no) {
    const int64_t key = kGhost | oid[k];  // (an owned id is always kept: orphans are never owned)
    const int64_t j = lower(vid2, nv2, key);
    rrank[k] = j < nv2 && vid2[j] == key ? (uint32_t)j : sent;
    rt[k] = (uint64_t)ot[k];
    rlast[k] = 0;
    rid[k] = oid[k];
    perm[k] = (uint32_t)k;
  }
}
__global__ __launch_bounds__(kB) void k_del_rec(int64_t nd, int64_t no, const uint32_t* __restrict__ delq,
                                                const DevEvent* __restrict__ ev, const int32_t* __restrict__ rs, uint32_t sent,
                                                uint64_t* __restrict__ rt, uint32_t* __restrict__ rrank,
                                                int64_t* __restrict__ rlast, int64_t* __restrict__ rid,
                                                uint32_t* __restrict__ perm) {
  GLOOP(j, nd) {
    const uint32_t i = delq[j];
    rrank[no + j] = rs[i] >= 0 ? (uint32_t)rs[i] : sent;
    rt[no + j] = (uint64_t)ev[i].t;
    rlast[no + j] = (int64_t)i + 1;
    rid[no + j] = ev[i].src;
    perm[no + j] = (uint32_t)(no + j);
  }
}
__global__ __launch_bounds__(kB) void k_gather_u32(int64_t n, const uint32_t* __restrict__ perm,
                                                   const uint32_t* __restrict__ a, uint32_t* __restrict__ out) {
  GLOOP(k, n) out[k] = a[perm[k]];
}
// records sorted by (rank, time, last): kept = last of its (rank, time) run; start = first of its rank
__global__ __launch_bounds__(kB) void k_drun_flags(int64_t R, const uint32_t* __restrict__ rk, const uint32_t* __restrict__ perm,
                                                   const uint64_t* __restrict__ rt, uint32_t sent,
                                                   int32_t* __restrict__ kept, int32_t* __restrict__ start) {
  GLOOP(p, R + 1) {
    int32_t k = 0, st = 0;
    if (p < R && rk[p] != sent) {
      st = p == 0 || rk[p - 1] != rk[p];
      k = !(p + 1 < R && rk[p + 1] == rk[p] && rt[perm[p + 1]] == rt[perm[p]]);
    }
    kept[p] = k;
    start[p] = st;
  }
}
__global__ __launch_bounds__(kB) void k_dfill(int64_t R, const uint32_t* __restrict__ rk, const uint32_t* __restrict__ perm,
                                              const uint64_t* __restrict__ rt, const int64_t* __restrict__ rlast,
                                              const int32_t* __restrict__ kept, const int32_t* __restrict__ start,
                                              const int64_t* __restrict__ kpos, const int64_t* __restrict__ spos,
                                              int32_t* __restrict__ dd_rank, int64_t* __restrict__ dd_off,
                                              int64_t* __restrict__ dd_t, int64_t* __restrict__ dd_last) {
  GLOOP(p, R) {
    if (start[p]) {
      dd_rank[spos[p]] = (int32_t)rk[p];
      dd_off[spos[p]] = kpos[p];
    }
    if (kept[p]) {
      dd_t[kpos[p]] = (int64_t)rt[perm[p]];
      dd_last[kpos[p]] = rlast[perm[p]];
    }
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) dd_off[spos[R]] = kpos[R];
}

// ---- edge points: key = src * nv2 + dst for edge updates (sentinel nv2^2); value = i
// (kept iff both endpoints are kept and one is owned; cnt = the kept records)
__global__ __launch_bounds__(kB) void k_erec(int64_t n, const DevEvent* __restrict__ ev, const uint32_t* __restrict__ ord,
                                             const int32_t* __restrict__ rs, const int32_t* __restrict__ rd, uint64_t nv2,
                                             int64_t n_own, uint64_t* __restrict__ key, uint32_t* __restrict__ val,
                                             unsigned long long* __restrict__ cnt) {
  unsigned long long c = 0;
  GLOOP(q, n) {
    const int64_t i = ord_at(ord, q);
    const int32_t a = rs[i], b = rd[i];
    const bool kept = ev[i].kind >= RGPU_EADD && a >= 0 && b >= 0 && (a < n_own || b < n_own);
    key[q] = kept ? (uint64_t)a * nv2 + (uint64_t)b : nv2 * nv2;
    val[q] = (uint32_t)i;
    c += kept;
  }
  for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o);
  if ((threadIdx.x & 63) == 0 && c) atomicAdd(cnt, c);
}
__global__ __launch_bounds__(kB) void k_egroups(int64_t m, const uint64_t* __restrict__ key, int32_t* __restrict__ start) {
  GLOOP(p, m + 1) start[p] = p < m && (p == 0 || key[p] != key[p - 1]);
}
__global__ __launch_bounds__(kB) void k_efill(int64_t nr, const uint64_t* __restrict__ key, const uint32_t* __restrict__ val,
                                              const int32_t* __restrict__ start, const int32_t* __restrict__ gpos,
                                              const int32_t* __restrict__ rs, const int32_t* __restrict__ rd,
                                              const int32_t* __restrict__ new2old, int32_t* __restrict__ de_s,
                                              int32_t* __restrict__ de_d, int32_t* __restrict__ de_qs,
                                              int32_t* __restrict__ de_qd, int64_t* __restrict__ de_poff, int64_t nde) {
  GLOOP(p, nr) {
    if (!start[p]) continue;
    const int32_t g = gpos[p];
    const uint32_t i = val[p];
    const int32_t s = rs[i], d = rd[i];
    de_s[g] = s;
    de_d[g] = d;
    de_qs[g] = new2old[s];
    de_qd[g] = new2old[d];
    de_poff[g] = p;
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) de_poff[nde] = nr;
}

// death of rank v at exactly t: the last delta index, 0 for a base death, -1 for none
struct Deaths {
  int64_t ndd;
  const int32_t* dd_rank;
  const int64_t *dd_off, *dd_t, *dd_last;
  const int32_t* new2old;
  const int64_t *doff, *dtime;
  __device__ int64_t at(int32_t v, int64_t t) const {
    if (ndd) {
      const int64_t j = lower(dd_rank, ndd, v);
      if (j < ndd && dd_rank[j] == v) {
        const int64_t a = dd_off[j], nb = dd_off[j + 1] - a;
        const int64_t f = lower(dd_t + a, nb, t);
        if (f < nb && dd_t[a + f] == t) return dd_last[a + f];
      }
    }
    const int32_t u = new2old[v];
    if (u >= 0 && doff) {
      const int64_t a = doff[u], nb = doff[u + 1] - a;
      if (nb) {
        const int64_t f = lower(dtime + a, nb, t);
        if (f < nb && dtime[a + f] == t) return 0;
      }
    }
    return -1;
  }
};

// own points of delta edge g: equal times collapse (last put wins), then the tie with an
// endpoint death at the same time as pack_events resolves it (x2 positions; a base edge was
// created at 0).  WRITE = false: count only
template <bool WRITE>
__global__ __launch_bounds__(kB) void k_emit(int64_t nde, const int64_t* __restrict__ poff,
                                             const uint32_t* __restrict__ pval, const DevEvent* __restrict__ ev,
                                             const int32_t* __restrict__ de_s, const int32_t* __restrict__ de_d,
                                             const int32_t* __restrict__ de_base, Deaths D, int64_t* __restrict__ koff,
                                             int64_t* __restrict__ key) {
  GLOOP(g, nde) {
    const int64_t p0 = poff[g], p1 = poff[g + 1];
    if (!WRITE) {
      int64_t m = 0;
      for (int64_t k = p0; k < p1; k++) m += !(k + 1 < p1 && ev[pval[k + 1]].t == ev[pval[k]].t);
      koff[g] = m;
      continue;
    }
    int64_t cr = 0;  // creation put: the edge's first delta update
    if (de_base[g] < 0) {
      cr = INT64_MAX;
      for (int64_t k = p0; k < p1; k++) cr = min(cr, (int64_t)pval[k] + 1);
    }
    const int32_t s = de_s[g], d = de_d[g];
    int64_t o = koff[g];
    for (int64_t k = p0; k < p1; k++) {
      const DevEvent& e = ev[pval[k]];
      if (k + 1 < p1 && ev[pval[k + 1]].t == e.t) continue;
      int64_t flag = e.kind == RGPU_EADD;
      int64_t pd = D.at(s, e.t);
      if (d != s) pd = max(pd, D.at(d, e.t));
      if (pd >= 0) {
        const int64_t pd2 = pd < cr ? 2 * cr + 1 : 2 * pd;
        if (pd2 > 2 * ((int64_t)pval[k] + 1)) flag = 0;
      }
      key[o++] = e.t * 2 + flag;
    }
  }
}

// new edges (no base edge) and their in-edge records (self-loops never enter incomingEdges)
__global__ __launch_bounds__(kB) void k_new_flags(int64_t nde, const int32_t* __restrict__ de_base,
                                                  const int32_t* __restrict__ de_s, const int32_t* __restrict__ de_d,
                                                  int32_t* __restrict__ fn, int32_t* __restrict__ fi) {
  GLOOP(g, nde + 1) {
    const bool nw = g < nde && de_base[g] < 0;
    fn[g] = nw;
    fi[g] = nw && de_s[g] != de_d[g];
  }
}
__global__ __launch_bounds__(kB) void k_new_fill(int64_t nde, const int32_t* __restrict__ de_base,
                                                 const int32_t* __restrict__ de_s, const int32_t* __restrict__ de_d,
                                                 const int32_t* __restrict__ pn, const int32_t* __restrict__ pi, uint64_t nv2,
                                                 int64_t* __restrict__ nn_key, int32_t* __restrict__ nn_didx,
                                                 uint64_t* __restrict__ ik, int32_t* __restrict__ iv) {
  GLOOP(g, nde) {
    if (de_base[g] >= 0) continue;
    const int32_t s = de_s[g], d = de_d[g], a = pn[g];
    nn_key[a] = ((int64_t)s << 32) | (uint32_t)d;
    nn_didx[a] = (int32_t)g;
    if (s != d) {
      ik[pi[g]] = (uint64_t)d * nv2 + (uint64_t)s;
      iv[pi[g]] = a;
    }
  }
}
__global__ __launch_bounds__(kB) void k_ni_decode(int64_t nni, const uint64_t* __restrict__ ik, uint64_t nv2,
                                                  int64_t* __restrict__ ni_key) {
  GLOOP(k, nni) ni_key[k] = ((int64_t)(ik[k] / nv2) << 32) | (int64_t)(ik[k] % nv2);
}

// ---- merged offsets: base counts, + new edges (atomics: the runs are short), one scan each
__global__ __launch_bounds__(kB) void k_base_counts(int64_t nv2, const int32_t* __restrict__ new2old,
                                                    const int64_t* __restrict__ out_off, const int64_t* __restrict__ in_off,
                                                    int64_t* __restrict__ co, int64_t* __restrict__ ci) {
  GLOOP(v, nv2 + 1) {
    const int32_t u = v < nv2 ? new2old[v] : -1;
    co[v] = u >= 0 ? out_off[u + 1] - out_off[u] : 0;
    ci[v] = u >= 0 ? in_off[u + 1] - in_off[u] : 0;
  }
}
__global__ __launch_bounds__(kB) void k_new_counts(int64_t n, const int64_t* __restrict__ key, int64_t* __restrict__ c) {
  GLOOP(k, n) atomicAdd((unsigned long long*)&c[key[k] >> 32], 1ull);
}
__global__ __launch_bounds__(kB) void k_adj(int64_t nv2, const int64_t* __restrict__ out_off,
                                            const int64_t* __restrict__ in_off, int64_t* __restrict__ adj) {
  GLOOP(v, nv2 + 65) adj[v] = v <= nv2 ? out_off[v] + in_off[v] : out_off[nv2] + in_off[nv2];
}

// merged death lists: per rank the sorted union of its base and delta times
template <bool WRITE>
__global__ __launch_bounds__(kB) void k_deaths(int64_t nv2, Deaths D, const int64_t* __restrict__ doff2,
                                               int64_t* __restrict__ cnt, int64_t* __restrict__ dtime2) {
  GLOOP(v, nv2) {
    const int32_t u = D.new2old[v];
    const int64_t* b0 = nullptr;
    int64_t nb = 0;
    if (u >= 0 && D.doff) {
      b0 = D.dtime + D.doff[u];
      nb = D.doff[u + 1] - D.doff[u];
    }
    const int64_t* c0 = nullptr;
    int64_t nc = 0;
    if (D.ndd) {
      const int64_t j = lower(D.dd_rank, D.ndd, (int32_t)v);
      if (j < D.ndd && D.dd_rank[j] == (int32_t)v) {
        c0 = D.dd_t + D.dd_off[j];
        nc = D.dd_off[j + 1] - D.dd_off[j];
      }
    }
    int64_t i = 0, j = 0, o = WRITE ? doff2[v] : 0;
    while (i < nb || j < nc) {
      int64_t t;
      if (j == nc || (i < nb && b0[i] < c0[j])) t = b0[i++];
      else if (i == nb || c0[j] < b0[i]) t = c0[j++];
      else { t = b0[i++]; j++; }
      if (WRITE) dtime2[o] = t;
      o++;
    }
    if (!WRITE) cnt[v] = o;
  }
}
__global__ __launch_bounds__(kB) void k_dbits(int64_t nw, int64_t nv2, const int64_t* __restrict__ doff2,
                                              uint64_t* __restrict__ bits) {
  GLOOP(w, nw) {
    uint64_t b = 0;
    for (int k = 0; k < 64; k++) {
      const int64_t v = w * 64 + k;
      if (v < nv2 && doff2[v + 1] > doff2[v]) b |= 1ull << k;
    }
    bits[w] = b;
  }
}
__global__ __launch_bounds__(kB) void k_heavy_flags(int64_t nv2, const int64_t* __restrict__ adj, int64_t t,
                                                    int32_t* __restrict__ f) {
  GLOOP(v, nv2 + 1) f[v] = v < nv2 && adj[v + 1] - adj[v] > t;
}
__global__ __launch_bounds__(kB) void k_heavy_list(int64_t nv2, const int32_t* __restrict__ f,
                                                   const int32_t* __restrict__ pos, int32_t* __restrict__ hv) {
  GLOOP(v, nv2) if (f[v]) hv[pos[v]] = (int32_t)v;
}
__global__ __launch_bounds__(kB) void k_gather_adj(int64_t n, const int32_t* __restrict__ hv,
                                                   const int64_t* __restrict__ adj, int64_t* __restrict__ a0,
                                                   int64_t* __restrict__ deg) {
  GLOOP(k, n) {
    a0[k] = adj[hv[k]];
    deg[k] = adj[hv[k] + 1] - adj[hv[k]];
  }
}
__global__ __launch_bounds__(kB) void k_scatter_i32(int64_t n, const int32_t* __restrict__ idx,
                                                    const int32_t* __restrict__ val, int32_t* __restrict__ out) {
  GLOOP(k, n) out[idx[k]] = val[k];
}

// ---- partition metadata of a merged partitioned graph (what pack_events + rgpu_seal build on
// the host for a full seal): labels = ids, the exchange plan, the owned-id index
__global__ __launch_bounds__(kB) void k_grank(int64_t nv, const int64_t* __restrict__ keys, int32_t* __restrict__ grank) {
  GLOOP(v, nv) grank[v] = (int32_t)(keys[v] & (kGhost - 1));
}
// an edge between owned v and ghost g (owner q): v goes on the send list to q, g on the receive
// list from q (ranks ascend with ids within a role, so (q, rank) order is pack_events' (q, id))
__global__ __launch_bounds__(kB) void k_cut_pairs(int64_t ne, const int32_t* __restrict__ esrc,
                                                  const int32_t* __restrict__ edst, const int64_t* __restrict__ keys,
                                                  int64_t n_own, int nparts, uint64_t* __restrict__ sk,
                                                  uint64_t* __restrict__ rk) {
  const uint64_t sent = (uint64_t)nparts << 32;
  GLOOP(e, ne) {
    const int32_t a = esrc[e], b = edst[e];
    if ((a < n_own) == (b < n_own)) {
      sk[e] = rk[e] = sent;
      continue;
    }
    const int32_t own = a < n_own ? a : b, gh = a < n_own ? b : a;
    const int64_t id = keys[gh] & (kGhost - 1);
    const uint64_t q = (uint64_t)((id % (10 * (int64_t)nparts)) / 10);
    sk[e] = (q << 32) | (uint32_t)own;
    rk[e] = (q << 32) | (uint32_t)gh;
  }
}
__global__ __launch_bounds__(kB) void k_uniq_flags(int64_t n, const uint64_t* __restrict__ k, uint64_t sent,
                                                   int32_t* __restrict__ f) {
  GLOOP(p, n + 1) f[p] = p < n && k[p] != sent && (p == 0 || k[p] != k[p - 1]);
}
__global__ __launch_bounds__(kB) void k_uniq_fill(int64_t n, const uint64_t* __restrict__ k, const int32_t* __restrict__ f,
                                                  const int32_t* __restrict__ pos, int32_t* __restrict__ v,
                                                  int32_t* __restrict__ q) {
  GLOOP(p, n) if (f[p]) {
    v[pos[p]] = (int32_t)(k[p] & 0xffffffffu);
    q[pos[p]] = (int32_t)(k[p] >> 32);
  }
}
__global__ __launch_bounds__(kB) void k_q_offsets(int64_t n, const int32_t* __restrict__ q, int nparts,
                                                  int64_t* __restrict__ off) {
  GLOOP(p, nparts + 1) off[p] = lower(q, n, (int32_t)p);
}
__global__ __launch_bounds__(kB) void k_bucket_counts(int64_t n, const int64_t* __restrict__ ids, int shift,
                                                      int32_t* __restrict__ cnt) {
  GLOOP(k, n) atomicAdd(&cnt[ids[k] >> shift], 1);
}

}  // namespace

void launch_scatter_i32(hipStream_t s, int64_t n, const int32_t* idx, const int32_t* val, int32_t* out) {
  if (n > 0) k_scatter_i32<<<gridn(n), kB, 0, s>>>(n, idx, val, out);
}

std::string gpu_pack_delta(hipStream_t s, const DevEvent* ev, int64_t n, const DevGraph& g0, const int64_t* vid0,
                           const DeltaPart& P, int64_t heavy_t, DeltaDev* out, std::vector<void*>& T,
                           std::vector<void*>& L) {
  Mem M{T, L};
  DeltaDev& D = *out;
  D = DeltaDev();
  D.nd = n;
  D.nv_old = g0.nv;
  if (n <= 0 || n >= ((int64_t)1 << 31)) return n <= 0 ? "" : "more than 2^31 updates in one seal";
  const int64_t nv_old = g0.nv;
  // ---- validation and flags
  unsigned long long* flags = M.alloc<unsigned long long>(4);
  GCHK(hipMemsetAsync(flags, 0, 4 * sizeof(unsigned long long), s));
  GCHK(hipMemsetAsync(flags, 0xff, sizeof(unsigned long long), s));
  k_validate<<<gridn(n), kB, 0, s>>>(n, ev, flags, flags + 1);
  unsigned long long h[4];
  GCHK(hipMemcpyAsync(h, flags, sizeof(h), hipMemcpyDeviceToHost, s));
  GCHK(hipStreamSynchronize(s));
  if (h[0] != ~0ull) {
    static const char* msg[4] = {"", "unknown update kind", "time out of range [0, 2^61)",
                                 "vertex id out of range [0, 2^31)"};
    return msg[h[0] & 3];
  }
  const bool mono = h[1] == 0;
  const int64_t n_vdel = (int64_t)h[2], n_eupd = (int64_t)h[3];
  // ---- ids
  const int64_t m = 2 * n;
  uint32_t* k0 = M.alloc<uint32_t>(m);
  uint32_t* v0 = M.alloc<uint32_t>(m);
  uint32_t* k1 = M.alloc<uint32_t>(m);
  uint32_t* v1 = M.alloc<uint32_t>(m);
  k_id_slots<<<gridn(n), kB, 0, s>>>(n, ev, k0, v0);
  sort_pairs(M, s, k0, k1, v0, v1, m, 32);
  int32_t* head = M.alloc<int32_t>(m + 1);
  int32_t* hpos = M.alloc<int32_t>(m + 1);
  k_heads<<<gridn(m + 1), kB, 0, s>>>(m, k1, head);
  excl_sum(M, s, head, hpos, m + 1);
  const int64_t nid = fetch(s, hpos + m);
  int64_t* ids = M.alloc<int64_t>(nid);
  k_ids<<<gridn(m), kB, 0, s>>>(m, k1, head, hpos, ids);
  // roles and rank-order keys; the new keys ascending
  uint8_t* need = nullptr;
  if (P.nparts > 0) {
    need = M.alloc<uint8_t>(nid);
    GCHK(hipMemsetAsync(need, 0, nid, s));
    k_ghost_need<<<gridn(m), kB, 0, s>>>(m, k1, v1, head, hpos, ev, P.part, P.nparts, need);
  }
  int64_t* keyk = M.alloc<int64_t>(nid);
  uint8_t* isnew = M.alloc<uint8_t>(nid);
  k_roles<<<gridn(nid), kB, 0, s>>>(nid, ids, vid0, nv_old, P.part, P.nparts, need, keyk, isnew);
  int64_t* nidv = M.alloc<int64_t>(nid);
  int* nsel = M.alloc<int>(1);
  {
    size_t b = 0;
    GCHK(hipcub::DeviceSelect::Flagged(nullptr, b, keyk, isnew, nidv, nsel, (int)nid, s));
    void* t = M.temp(b);
    GCHK(hipcub::DeviceSelect::Flagged(t, b, keyk, isnew, nidv, nsel, (int)nid, s));
  }
  const int64_t nnew = fetch(s, nsel);
  if (P.nparts > 0 && nnew > 1) {  // owned keys, then ghost keys: ascending again
    uint64_t* sorted = (uint64_t*)M.alloc<int64_t>(nnew);
    size_t b = 0;
    GCHK(hipcub::DeviceRadixSort::SortKeys(nullptr, b, (const uint64_t*)nidv, sorted, (int)nnew, 0, 32, s));
    void* t = M.temp(b);
    GCHK(hipcub::DeviceRadixSort::SortKeys(t, b, (const uint64_t*)nidv, sorted, (int)nnew, 0, 32, s));
    nidv = (int64_t*)sorted;
  }
  int64_t n_own2 = nv_old + nnew;
  if (P.nparts > 0) {
    int64_t* below = M.alloc<int64_t>(1);
    k_count_below<<<1, 64, 0, s>>>(nnew, nidv, kGhost, below);
    n_own2 = P.n_own_old + fetch(s, below);
  }
  D.n_own2 = n_own2;
  const int64_t nv2 = nv_old + nnew;
  if (nv2 > (int64_t)INT32_MAX - 1) return "more than 2^31 - 1 vertices";
  D.nv2 = nv2;
  D.vid2 = M.alloc<int64_t>(nv2, true);
  D.old2new = M.alloc<int32_t>(nv_old);
  D.new2old = M.alloc<int32_t>(nv2);
  if (nv_old) k_place_old<<<gridn(nv_old), kB, 0, s>>>(nv_old, vid0, nidv, nnew, D.vid2, D.old2new, D.new2old);
  if (nnew) k_place_new<<<gridn(nnew), kB, 0, s>>>(nnew, nidv, vid0, nv_old, D.vid2, D.new2old);
  int32_t* idrank = M.alloc<int32_t>(nid);
  k_idrank<<<gridn(nid), kB, 0, s>>>(nid, keyk, D.vid2, nv2, idrank);
  int32_t* rs = M.alloc<int32_t>(n);
  int32_t* rd = M.alloc<int32_t>(n);
  GCHK(hipMemsetAsync(rd, 0xff, sizeof(int32_t) * n, s));
  k_ranks<<<gridn(m), kB, 0, s>>>(m, k1, v1, head, hpos, idrank, rs, rd);
  // ---- order by (time, index) unless the tick is time-ordered already
  uint32_t* ord = nullptr;
  if (!mono) {
    uint64_t* tk0 = M.alloc<uint64_t>(n);
    uint64_t* tk1 = M.alloc<uint64_t>(n);
    uint32_t* iv0 = M.alloc<uint32_t>(n);
    ord = M.alloc<uint32_t>(n);
    k_time_keys<<<gridn(n), kB, 0, s>>>(n, ev, tk0, iv0);
    sort_pairs(M, s, tk0, tk1, iv0, ord, n, 61);
  }
  const uint32_t vsent = (uint32_t)nv2;
  const int vbits = bits_for((uint64_t)nv2);
  int32_t* kept = M.alloc<int32_t>(m + 1);
  int32_t* start = M.alloc<int32_t>(m + 1);
  int64_t* kpos = M.alloc<int64_t>(m + 1);
  int64_t* spos = M.alloc<int64_t>(m + 1);
  // ---- vertex points
  k_vrec<<<gridn(n), kB, 0, s>>>(n, ev, ord, rs, rd, n_own2, vsent, k0, v0);
  sort_pairs(M, s, k0, k1, v0, v1, m, vbits);
  k_run_flags<<<gridn(m + 1), kB, 0, s>>>(m, k1, v1, 1, vsent, ev, kept, start);
  excl_sum(M, s, kept, kpos, m + 1);
  excl_sum(M, s, start, spos, m + 1);
  {
    int64_t t2[2];
    GCHK(hipMemcpyAsync(&t2[0], kpos + m, sizeof(int64_t), hipMemcpyDeviceToHost, s));
    GCHK(hipMemcpyAsync(&t2[1], spos + m, sizeof(int64_t), hipMemcpyDeviceToHost, s));
    GCHK(hipStreamSynchronize(s));
    D.ndvk = t2[0];
    D.ndv = t2[1];
  }
  D.dv_rank = M.alloc<int32_t>(D.ndv);
  D.dv_off = M.alloc<int64_t>(D.ndv + 1);
  D.dv_key = M.alloc<int64_t>(D.ndvk);
  k_vfill<<<gridn(m), kB, 0, s>>>(m, k1, v1, ev, kept, start, kpos, spos, D.dv_rank, D.dv_off, D.dv_key);
  // ---- deaths (VertexDelete is rare: compacted first; skipped when there are none)
  if (n_vdel || P.n_orph) {
    int64_t* dpos = kpos;  // (reused)
    uint32_t* delq = k0;
    if (n_vdel) {
      k_del_flags<<<gridn(n + 1), kB, 0, s>>>(n, ev, ord, kept);
      excl_sum(M, s, kept, dpos, n + 1);
      k_del_list<<<gridn(n), kB, 0, s>>>(n, ord, kept, dpos, delq);
    }
    const int64_t no = P.n_orph, R = no + n_vdel;
    uint64_t* rt = M.alloc<uint64_t>(R);
    uint64_t* rt1 = M.alloc<uint64_t>(R);
    uint32_t* rrank = M.alloc<uint32_t>(R);
    uint32_t* rk1 = M.alloc<uint32_t>(R);
    uint32_t* rk2 = M.alloc<uint32_t>(R);
    int64_t* rlast = M.alloc<int64_t>(R);
    int64_t* rid = M.alloc<int64_t>(R);
    uint32_t* perm0 = M.alloc<uint32_t>(R);
    uint32_t* perm1 = M.alloc<uint32_t>(R);
    uint32_t* perm2 = M.alloc<uint32_t>(R);
    if (no) k_orph_rec<<<gridn(no), kB, 0, s>>>(no, P.orph_id, P.orph_t, D.vid2, nv2, vsent, rt, rrank, rlast, rid, perm0);
    if (n_vdel) k_del_rec<<<gridn(n_vdel), kB, 0, s>>>(n_vdel, no, delq, ev, rs, vsent, rt, rrank, rlast, rid, perm0);
    // (time, record order), then rank: both stable
    sort_pairs(M, s, rt, rt1, perm0, perm1, R, 61);
    k_gather_u32<<<gridn(R), kB, 0, s>>>(R, perm1, rrank, rk1);
    sort_pairs(M, s, rk1, rk2, perm1, perm2, R, bits_for((uint64_t)nv2));
    int32_t* dk = M.alloc<int32_t>(R + 1);
    int32_t* dst = M.alloc<int32_t>(R + 1);
    int64_t* dkp = M.alloc<int64_t>(R + 1);
    int64_t* dsp = M.alloc<int64_t>(R + 1);
    k_drun_flags<<<gridn(R + 1), kB, 0, s>>>(R, rk2, perm2, rt, vsent, dk, dst);
    excl_sum(M, s, dk, dkp, R + 1);
    excl_sum(M, s, dst, dsp, R + 1);
    int64_t t2[2];
    GCHK(hipMemcpyAsync(&t2[0], dkp + R, sizeof(int64_t), hipMemcpyDeviceToHost, s));
    GCHK(hipMemcpyAsync(&t2[1], dsp + R, sizeof(int64_t), hipMemcpyDeviceToHost, s));
    // deaths of ids still not kept here: the orphans of the next seal (host list)
    std::vector<uint32_t> hr(R);
    std::vector<int64_t> hid(R), ht(R);
    if (P.nparts > 0) {
      GCHK(hipMemcpyAsync(hr.data(), rrank, sizeof(uint32_t) * R, hipMemcpyDeviceToHost, s));
      GCHK(hipMemcpyAsync(hid.data(), rid, sizeof(int64_t) * R, hipMemcpyDeviceToHost, s));
      GCHK(hipMemcpyAsync(ht.data(), rt, sizeof(int64_t) * R, hipMemcpyDeviceToHost, s));
    }
    GCHK(hipStreamSynchronize(s));
    if (P.nparts > 0)
      for (int64_t k = 0; k < R; k++)
        if (hr[k] == vsent) {
          D.orph_id.push_back(hid[k]);
          D.orph_t.push_back(ht[k]);
        }
    D.ndd = t2[1];
    D.dd_rank = M.alloc<int32_t>(D.ndd);
    D.dd_off = M.alloc<int64_t>(D.ndd + 1);
    D.dd_t = M.alloc<int64_t>(t2[0]);
    D.dd_last = M.alloc<int64_t>(t2[0]);
    k_dfill<<<gridn(R), kB, 0, s>>>(R, rk2, perm2, rt, rlast, dk, dst, dkp, dsp, D.dd_rank, D.dd_off, D.dd_t,
                                    D.dd_last);
  }
  // ---- edge points grouped by (src, dst)
  if (n_eupd) {
    uint64_t* ek0 = M.alloc<uint64_t>(n);
    uint64_t* ek1 = M.alloc<uint64_t>(n);
    uint32_t* pval = M.alloc<uint32_t>(n);
    const uint64_t nvu = (uint64_t)nv2;
    unsigned long long* ecnt = (unsigned long long*)M.alloc<int64_t>(1);
    GCHK(hipMemsetAsync(ecnt, 0, sizeof(unsigned long long), s));
    k_erec<<<gridn(n), kB, 0, s>>>(n, ev, ord, rs, rd, nvu, n_own2, ek0, v0, ecnt);
    sort_pairs(M, s, ek0, ek1, v0, pval, n, bits_for(nvu * nvu));
    const int64_t nr = (int64_t)fetch(s, ecnt);  // the kept records come first
    int32_t* gpos = hpos;       // (reused: m + 1 >= nr + 1)
    k_egroups<<<gridn(nr + 1), kB, 0, s>>>(nr, ek1, start);
    excl_sum(M, s, start, gpos, nr + 1);
    const int64_t nde = fetch(s, gpos + nr);
    D.nde = nde;
    D.de_s = M.alloc<int32_t>(nde);
    D.de_d = M.alloc<int32_t>(nde);
    int32_t* de_qs = M.alloc<int32_t>(nde);
    int32_t* de_qd = M.alloc<int32_t>(nde);
    int64_t* de_poff = M.alloc<int64_t>(nde + 1);
    k_efill<<<gridn(nr), kB, 0, s>>>(nr, ek1, pval, start, gpos, rs, rd, D.new2old, D.de_s, D.de_d, de_qs, de_qd,
                                     de_poff, nde);
    D.de_base = M.alloc<int32_t>(nde);
    launch_edge_find(s, nde, de_qs, de_qd, g0.out_off, g0.edst, D.de_base);
    Deaths dz{D.ndd, D.dd_rank, D.dd_off, D.dd_t, D.dd_last, D.new2old, g0.doff, g0.dtime};
    D.de_koff = M.alloc<int64_t>(nde + 1);
    int64_t* kc = M.alloc<int64_t>(nde + 1);
    GCHK(hipMemsetAsync(kc + nde, 0, sizeof(int64_t), s));
    k_emit<false><<<gridn(nde), kB, 0, s>>>(nde, de_poff, pval, ev, D.de_s, D.de_d, D.de_base, dz, kc, nullptr);
    excl_sum(M, s, kc, D.de_koff, nde + 1);
    const int64_t ndek = fetch(s, D.de_koff + nde);
    D.de_key = M.alloc<int64_t>(ndek);
    k_emit<true><<<gridn(nde), kB, 0, s>>>(nde, de_poff, pval, ev, D.de_s, D.de_d, D.de_base, dz, D.de_koff, D.de_key);
    // new edges and their in-edge records
    int32_t* fn = kept;
    int32_t* fi = start;
    int32_t* pn = M.alloc<int32_t>(nde + 1);
    int32_t* pi = M.alloc<int32_t>(nde + 1);
    k_new_flags<<<gridn(nde + 1), kB, 0, s>>>(nde, D.de_base, D.de_s, D.de_d, fn, fi);
    excl_sum(M, s, fn, pn, nde + 1);
    excl_sum(M, s, fi, pi, nde + 1);
    {
      int32_t t2[2];
      GCHK(hipMemcpyAsync(&t2[0], pn + nde, sizeof(int32_t), hipMemcpyDeviceToHost, s));
      GCHK(hipMemcpyAsync(&t2[1], pi + nde, sizeof(int32_t), hipMemcpyDeviceToHost, s));
      GCHK(hipStreamSynchronize(s));
      D.n_new = t2[0];
      D.nni = t2[1];
    }
    D.nn_key = M.alloc<int64_t>(D.n_new);
    D.nn_didx = M.alloc<int32_t>(D.n_new);
    uint64_t* ik0 = ek0;  // (reused)
    uint64_t* ik1 = M.alloc<uint64_t>(D.nni);
    int32_t* iv0 = (int32_t*)v0;
    D.ni_idx = M.alloc<int32_t>(D.nni);
    k_new_fill<<<gridn(nde), kB, 0, s>>>(nde, D.de_base, D.de_s, D.de_d, pn, pi, nvu, D.nn_key, D.nn_didx, ik0, iv0);
    sort_pairs(M, s, ik0, ik1, iv0, D.ni_idx, D.nni, bits_for(nvu * nvu));
    D.ni_key = M.alloc<int64_t>(D.nni);
    if (D.nni) k_ni_decode<<<gridn(D.nni), kB, 0, s>>>(D.nni, ik1, nvu, D.ni_key);
  }
  // ---- merged offsets
  int64_t* co = M.alloc<int64_t>(nv2 + 1);
  int64_t* ci = M.alloc<int64_t>(nv2 + 1);
  k_base_counts<<<gridn(nv2 + 1), kB, 0, s>>>(nv2, D.new2old, g0.out_off, g0.in_off, co, ci);
  if (D.n_new) k_new_counts<<<gridn(D.n_new), kB, 0, s>>>(D.n_new, D.nn_key, co);
  if (D.nni) k_new_counts<<<gridn(D.nni), kB, 0, s>>>(D.nni, D.ni_key, ci);
  D.out_off = M.alloc<int64_t>(nv2 + 1, true);
  D.in_off = M.alloc<int64_t>(nv2 + 1, true);
  excl_sum(M, s, co, D.out_off, nv2 + 1);
  excl_sum(M, s, ci, D.in_off, nv2 + 1);
  D.adj_off = M.alloc<int64_t>(nv2 + 65, true);
  k_adj<<<gridn(nv2 + 65), kB, 0, s>>>(nv2, D.out_off, D.in_off, D.adj_off);
  D.n_in = fetch(s, D.in_off + nv2);
  // ---- merged deaths
  Deaths dz{D.ndd, D.dd_rank, D.dd_off, D.dd_t, D.dd_last, D.new2old, g0.doff, g0.dtime};
  int64_t* dc = co;  // (reused)
  GCHK(hipMemsetAsync(dc + nv2, 0, sizeof(int64_t), s));
  k_deaths<false><<<gridn(nv2), kB, 0, s>>>(nv2, dz, nullptr, dc, nullptr);
  D.doff = M.alloc<int64_t>(nv2 + 1, true);
  excl_sum(M, s, dc, D.doff, nv2 + 1);
  D.ndt = fetch(s, D.doff + nv2);
  D.dtime = M.alloc<int64_t>(D.ndt, true);
  if (D.ndt) k_deaths<true><<<gridn(nv2), kB, 0, s>>>(nv2, dz, D.doff, nullptr, D.dtime);
  const int64_t nw = (nv2 + 63) / 64 + 1;
  D.dbits = M.alloc<uint64_t>(nw, true);
  k_dbits<<<gridn(nw), kB, 0, s>>>(nw, nv2, D.doff, D.dbits);
  // ---- heavy-vertex candidates (static slots above heavy_t): ranks and their slot ranges
  if (heavy_t > 0 && nv2) {
    int32_t* hf = M.alloc<int32_t>(nv2 + 1);
    int32_t* hp = M.alloc<int32_t>(nv2 + 1);
    k_heavy_flags<<<gridn(nv2 + 1), kB, 0, s>>>(nv2, D.adj_off, heavy_t, hf);
    excl_sum(M, s, hf, hp, nv2 + 1);
    const int64_t nh = fetch(s, hp + nv2);
    int32_t* hv = M.alloc<int32_t>(nh);
    if (nh) k_heavy_list<<<gridn(nv2), kB, 0, s>>>(nv2, hf, hp, hv);
    D.heavy.resize(nh);
    D.heavy_a0.resize(nh);
    D.heavy_deg.resize(nh);
    if (nh) {
      int64_t* ha = M.alloc<int64_t>(2 * nh);
      k_gather_adj<<<gridn(nh), kB, 0, s>>>(nh, hv, D.adj_off, ha, ha + nh);
      GCHK(hipMemcpyAsync(D.heavy.data(), hv, sizeof(int32_t) * nh, hipMemcpyDeviceToHost, s));
      GCHK(hipMemcpyAsync(D.heavy_a0.data(), ha, sizeof(int64_t) * nh, hipMemcpyDeviceToHost, s));
      GCHK(hipMemcpyAsync(D.heavy_deg.data(), ha + nh, sizeof(int64_t) * nh, hipMemcpyDeviceToHost, s));
      GCHK(hipStreamSynchronize(s));
    }
  }
  GCHK(hipGetLastError());
  GCHK(hipStreamSynchronize(s));
  return "";
}

namespace {
// (q, rank) pairs -> distinct, ascending; per-q offsets (device and host)
void plan_list(Mem& M, hipStream_t s, uint64_t* k0, uint64_t* k1, int64_t ne, int nparts, int32_t** v, int32_t** q,
               int64_t** off_d, std::vector<int64_t>& off, int64_t* n_out) {
  const uint64_t sent = (uint64_t)nparts << 32;
  if (ne > 0) {
    size_t b = 0;
    const int eb = 32 + bits_for((uint64_t)nparts);
    GCHK(hipcub::DeviceRadixSort::SortKeys(nullptr, b, k0, k1, (int)ne, 0, eb, s));
    void* t = M.temp(b);
    GCHK(hipcub::DeviceRadixSort::SortKeys(t, b, k0, k1, (int)ne, 0, eb, s));
  }
  int32_t* f = M.alloc<int32_t>(ne + 1);
  int32_t* pos = M.alloc<int32_t>(ne + 1);
  k_uniq_flags<<<gridn(ne + 1), kB, 0, s>>>(ne, k1, sent, f);
  excl_sum(M, s, f, pos, ne + 1);
  const int64_t n = fetch(s, pos + ne);
  *v = M.alloc<int32_t>(n, true);
  *q = M.alloc<int32_t>(n, true);
  if (ne) k_uniq_fill<<<gridn(ne), kB, 0, s>>>(ne, k1, f, pos, *v, *q);
  *off_d = M.alloc<int64_t>(nparts + 1, true);
  k_q_offsets<<<1, kB, 0, s>>>(n, *q, nparts, *off_d);
  off.resize(nparts + 1);
  GCHK(hipMemcpyAsync(off.data(), *off_d, sizeof(int64_t) * (nparts + 1), hipMemcpyDeviceToHost, s));
  GCHK(hipStreamSynchronize(s));
  *n_out = n;
}
}  // namespace

std::string gpu_part_meta(hipStream_t s, const int64_t* keys, int64_t nv, int64_t n_own, const int32_t* esrc,
                          const int32_t* edst, int64_t ne, int nparts, PartMeta* out, std::vector<void*>& T,
                          std::vector<void*>& L) {
  Mem M{T, L};
  PartMeta& X = *out;
  X = PartMeta();
  X.grank = M.alloc<int32_t>(nv, true);
  if (nv) k_grank<<<gridn(nv), kB, 0, s>>>(nv, keys, X.grank);
  uint64_t* sk = M.alloc<uint64_t>(ne);
  uint64_t* rk = M.alloc<uint64_t>(ne);
  uint64_t* k1 = M.alloc<uint64_t>(ne);
  if (ne) k_cut_pairs<<<gridn(ne), kB, 0, s>>>(ne, esrc, edst, keys, n_own, nparts, sk, rk);
  plan_list(M, s, sk, k1, ne, nparts, &X.xs_v, &X.xs_q, &X.xs_off_d, X.xs_off, &X.nxs);
  plan_list(M, s, rk, k1, ne, nparts, &X.xr_v, &X.xr_q, &X.xr_off_d, X.xr_off, &X.nxr);
  // owned ids ascending (the owned keys are the ids), bucketed by id >> shift (about one id per
  // bucket; rgpu_seal's full-seal index)
  X.own_vid = M.alloc<int64_t>(n_own, true);
  if (n_own) GCHK(hipMemcpyAsync(X.own_vid, keys, sizeof(int64_t) * n_own, hipMemcpyDeviceToDevice, s));
  X.id_max = -1;
  if (n_own) {
    GCHK(hipMemcpyAsync(&X.id_max, keys + n_own - 1, sizeof(int64_t), hipMemcpyDeviceToHost, s));
    GCHK(hipStreamSynchronize(s));
  }
  X.shift = own_bucket_shift(n_own, X.id_max);
  const int64_t nbk = (std::max<int64_t>(X.id_max, 0) >> X.shift) + 1;
  int32_t* cnt = M.alloc<int32_t>(nbk + 1);
  GCHK(hipMemsetAsync(cnt, 0, sizeof(int32_t) * (nbk + 1), s));
  if (n_own) k_bucket_counts<<<gridn(n_own), kB, 0, s>>>(n_own, X.own_vid, X.shift, cnt);
  X.own_boff = M.alloc<int32_t>(nbk + 1, true);
  excl_sum(M, s, cnt, X.own_boff, nbk + 1);
  GCHK(hipGetLastError());
  GCHK(hipStreamSynchronize(s));
  return "";
}

}  // namespace rgpu
