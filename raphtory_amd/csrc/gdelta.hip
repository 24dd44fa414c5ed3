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
__global__ __launch_bounds__(kB) void k_isnew(int64_t nid, const int64_t* __restrict__ ids, const int64_t* __restrict__ vid0,
                                              int64_t nv_old, uint8_t* __restrict__ isnew) {
  GLOOP(k, nid) {
    const int64_t j = lower(vid0, nv_old, ids[k]);
    isnew[k] = !(j < nv_old && vid0[j] == ids[k]);
  }
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
__global__ __launch_bounds__(kB) void k_idrank(int64_t nid, const int64_t* __restrict__ ids, const int64_t* __restrict__ vid2,
                                               int64_t nv2, int32_t* __restrict__ idrank) {
  GLOOP(k, nid) idrank[k] = (int32_t)lower(vid2, nv2, ids[k]);
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
__global__ __launch_bounds__(kB) void k_vrec(int64_t n, const DevEvent* __restrict__ ev, const uint32_t* __restrict__ ord,
                                             const int32_t* __restrict__ rs, const int32_t* __restrict__ rd, uint32_t sent,
                                             uint32_t* __restrict__ key, uint32_t* __restrict__ val) {
  GLOOP(q, n) {
    const int64_t i = ord_at(ord, q);
    const uint8_t kd = ev[i].kind;
    key[2 * q] = kd != RGPU_EDEL ? (uint32_t)rs[i] : sent;
    val[2 * q] = (uint32_t)(2 * i);
    key[2 * q + 1] = (kd == RGPU_EADD && rd[i] != rs[i]) ? (uint32_t)rd[i] : sent;
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

// ---- deaths: record q = the update's source if it is a VertexDelete; value = i
__global__ __launch_bounds__(kB) void k_drec(int64_t n, const DevEvent* __restrict__ ev, const uint32_t* __restrict__ ord,
                                             const int32_t* __restrict__ rs, uint32_t sent, uint32_t* __restrict__ key,
                                             uint32_t* __restrict__ val) {
  GLOOP(q, n) {
    const int64_t i = ord_at(ord, q);
    key[q] = ev[i].kind == RGPU_VDEL ? (uint32_t)rs[i] : sent;
    val[q] = (uint32_t)i;
  }
}
__global__ __launch_bounds__(kB) void k_dfill(int64_t m, const uint32_t* __restrict__ key, const uint32_t* __restrict__ val,
                                              const DevEvent* __restrict__ ev, const int32_t* __restrict__ kept,
                                              const int32_t* __restrict__ start, const int64_t* __restrict__ kpos,
                                              const int64_t* __restrict__ spos, int32_t* __restrict__ dd_rank,
                                              int64_t* __restrict__ dd_off, int64_t* __restrict__ dd_t,
                                              int64_t* __restrict__ dd_last) {
  GLOOP(p, m) {
    if (start[p]) {
      dd_rank[spos[p]] = (int32_t)key[p];
      dd_off[spos[p]] = kpos[p];
    }
    if (kept[p]) {
      dd_t[kpos[p]] = ev[val[p]].t;
      dd_last[kpos[p]] = (int64_t)val[p] + 1;
    }
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) dd_off[spos[m]] = kpos[m];
}

// ---- edge points: key = src * nv2 + dst for edge updates (sentinel nv2^2); value = i
__global__ __launch_bounds__(kB) void k_erec(int64_t n, const DevEvent* __restrict__ ev, const uint32_t* __restrict__ ord,
                                             const int32_t* __restrict__ rs, const int32_t* __restrict__ rd, uint64_t nv2,
                                             uint64_t* __restrict__ key, uint32_t* __restrict__ val) {
  GLOOP(q, n) {
    const int64_t i = ord_at(ord, q);
    key[q] = ev[i].kind >= RGPU_EADD ? (uint64_t)rs[i] * nv2 + (uint64_t)rd[i] : nv2 * nv2;
    val[q] = (uint32_t)i;
  }
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

}  // namespace

void launch_scatter_i32(hipStream_t s, int64_t n, const int32_t* idx, const int32_t* val, int32_t* out) {
  if (n > 0) k_scatter_i32<<<gridn(n), kB, 0, s>>>(n, idx, val, out);
}

std::string gpu_pack_delta(hipStream_t s, const DevEvent* ev, int64_t n, const DevGraph& g0, const int64_t* vid0,
                           int64_t heavy_t, DeltaDev* out, std::vector<void*>& T, std::vector<void*>& L) {
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
  uint8_t* isnew = M.alloc<uint8_t>(nid);
  k_isnew<<<gridn(nid), kB, 0, s>>>(nid, ids, vid0, nv_old, isnew);
  int64_t* nidv = M.alloc<int64_t>(nid);
  int* nsel = M.alloc<int>(1);
  {
    size_t b = 0;
    GCHK(hipcub::DeviceSelect::Flagged(nullptr, b, ids, isnew, nidv, nsel, (int)nid, s));
    void* t = M.temp(b);
    GCHK(hipcub::DeviceSelect::Flagged(t, b, ids, isnew, nidv, nsel, (int)nid, s));
  }
  const int64_t nnew = fetch(s, nsel);
  const int64_t nv2 = nv_old + nnew;
  if (nv2 > (int64_t)INT32_MAX - 1) return "more than 2^31 - 1 vertices";
  D.nv2 = nv2;
  D.vid2 = M.alloc<int64_t>(nv2, true);
  D.old2new = M.alloc<int32_t>(nv_old);
  D.new2old = M.alloc<int32_t>(nv2);
  if (nv_old) k_place_old<<<gridn(nv_old), kB, 0, s>>>(nv_old, vid0, nidv, nnew, D.vid2, D.old2new, D.new2old);
  if (nnew) k_place_new<<<gridn(nnew), kB, 0, s>>>(nnew, nidv, vid0, nv_old, D.vid2, D.new2old);
  int32_t* idrank = M.alloc<int32_t>(nid);
  k_idrank<<<gridn(nid), kB, 0, s>>>(nid, ids, D.vid2, nv2, idrank);
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
  k_vrec<<<gridn(n), kB, 0, s>>>(n, ev, ord, rs, rd, vsent, k0, v0);
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
  // ---- deaths (VertexDelete is rare: skipped when the tick has none)
  if (n_vdel) {
    k_drec<<<gridn(n), kB, 0, s>>>(n, ev, ord, rs, vsent, k0, v0);
    sort_pairs(M, s, k0, k1, v0, v1, n, vbits);
    k_run_flags<<<gridn(n + 1), kB, 0, s>>>(n, k1, v1, 0, vsent, ev, kept, start);
    excl_sum(M, s, kept, kpos, n + 1);
    excl_sum(M, s, start, spos, n + 1);
    int64_t t2[2];
    GCHK(hipMemcpyAsync(&t2[0], kpos + n, sizeof(int64_t), hipMemcpyDeviceToHost, s));
    GCHK(hipMemcpyAsync(&t2[1], spos + n, sizeof(int64_t), hipMemcpyDeviceToHost, s));
    GCHK(hipStreamSynchronize(s));
    D.ndd = t2[1];
    D.dd_rank = M.alloc<int32_t>(D.ndd);
    D.dd_off = M.alloc<int64_t>(D.ndd + 1);
    D.dd_t = M.alloc<int64_t>(t2[0]);
    D.dd_last = M.alloc<int64_t>(t2[0]);
    k_dfill<<<gridn(n), kB, 0, s>>>(n, k1, v1, ev, kept, start, kpos, spos, D.dd_rank, D.dd_off, D.dd_t, D.dd_last);
  }
  // ---- edge points grouped by (src, dst)
  if (n_eupd) {
    uint64_t* ek0 = M.alloc<uint64_t>(n);
    uint64_t* ek1 = M.alloc<uint64_t>(n);
    uint32_t* pval = M.alloc<uint32_t>(n);
    const uint64_t nvu = (uint64_t)nv2;
    k_erec<<<gridn(n), kB, 0, s>>>(n, ev, ord, rs, rd, nvu, ek0, v0);
    sort_pairs(M, s, ek0, ek1, v0, pval, n, bits_for(nvu * nvu));
    const int64_t nr = n_eupd;  // the valid records come first
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

}  // namespace rgpu
