// Time-ordered static slots (built once per seal, on the device).
//
// K2 (k_cc_slots / k_heavy_slots) keeps slot (v, e) of a batch iff em[e] & vm[nb] & vm[v] != 0,
// and an edge can only be alive in view (t, w) if its floor point at t is an add no older than
// the window (EntityStorage alive-at-with-window: Entity.scala:173-201), i.e. if its LAST add
// time is >= t - w.  With every vertex's static slots ordered by the edge's last add time,
// newest first, a batch whose views all start after `cut` (min over its views of t - w) only
// walks each member's prefix of slots with last add >= cut: a day or hour window near the
// newest hops touches the recent edges, not the vertex's whole history.
//
//   ts_e[p]  edge of static slot p       (p in [adj_off[v], adj_off[v+1]), newest first)
//   ts_nb[p] the neighbour across it
//   ts_t[p]  4 * (the edge's last add time) + 2 nodeath + simple   (INT64_MIN: never added;
//            ts_time / ts_nodeath / ts_simple in kernels.hpp)
//
// nodeath = neither endpoint ever died; simple = nodeath and the edge's history is one add point:
// its aliveness in any view (t, w) is then tf <= t <= tf + w with tf = ts_time, so K2 computes the
// slot's window bits from the word it already streams (kernels.hip slot_bits) instead of reading
// em[e].  A nodeath slot's bits imply both endpoints' membership (BatchParams::simple_ends).
//
// The order only changes which kept slot lands where inside the vertex's kept range: CC is a
// minimum over the kept slots, so results are unchanged.
#include "kernels.hpp"

#include <hipcub/device/device_segmented_sort.hpp>

namespace rgpu {

namespace {

__global__ __launch_bounds__(256) void k_slot_keys(int64_t nv, const int64_t* __restrict__ out_off,
                                                   const int64_t* __restrict__ in_off,
                                                   const int32_t* __restrict__ in_eid,
                                                   const int64_t* __restrict__ eoff,
                                                   const int64_t* __restrict__ ekey, const int32_t* __restrict__ esrc,
                                                   const int32_t* __restrict__ edst, const int64_t* __restrict__ doff,
                                                   const uint64_t* __restrict__ dbits, int64_t* __restrict__ key,
                                                   int32_t* __restrict__ val) {
  // one wave per vertex, lanes over its slots (out-edges then in-edges, CSR order)
  const int lane = threadIdx.x & 63;
  const int64_t wave = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t v = wave; v < nv; v += nwaves) {
    const int64_t o0 = out_off[v], o1 = out_off[v + 1], i0 = in_off[v], i1 = in_off[v + 1];
    const int64_t nout = o1 - o0, ntot = nout + (i1 - i0), base = o0 + i0;
    for (int64_t j = lane; j < ntot; j += 64) {
      const int32_t e = j < nout ? (int32_t)(o0 + j) : in_eid[i0 + (j - nout)];
      int64_t t = INT64_MIN;  // last add point: histories are sorted, key = 2 * time + alive
      const int64_t h0 = eoff[e], h1 = eoff[e + 1];
      for (int64_t i = h1 - 1; i >= h0; i--)
        if (ekey[i] & 1) { t = ekey[i] >> 1; break; }
      const int32_t a = esrc[e], b = edst[e];
      const bool da = dbits ? ((dbits[a >> 6] >> (a & 63)) & 1) : doff[a + 1] > doff[a];
      const bool db = dbits ? ((dbits[b >> 6] >> (b & 63)) & 1) : doff[b + 1] > doff[b];
      const bool nodeath = !da && !db && t != INT64_MIN;
      const bool simple = nodeath && h1 - h0 == 1;
      key[base + j] = t == INT64_MIN ? INT64_MIN : 4 * t + (nodeath ? 2 : 0) + (simple ? 1 : 0);
      val[base + j] = e;
    }
  }
}

__global__ __launch_bounds__(256) void k_slot_nbrs(int64_t nv, const int64_t* __restrict__ adj_off,
                                                   const int32_t* __restrict__ esrc,
                                                   const int32_t* __restrict__ edst,
                                                   const int32_t* __restrict__ ts_e, int32_t* __restrict__ ts_nb) {
  const int lane = threadIdx.x & 63;
  const int64_t wave = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t v = wave; v < nv; v += nwaves) {
    for (int64_t p = adj_off[v] + lane; p < adj_off[v + 1]; p += 64) {
      const int32_t e = ts_e[p], s = esrc[e];
      ts_nb[p] = s == (int32_t)v ? edst[e] : s;  // out-slot (or self-loop): the destination
    }
  }
}

__global__ __launch_bounds__(256) void k_slot_labels(int64_t n, const int32_t* __restrict__ ts_nb,
                                                     const int32_t* __restrict__ grank, int32_t* __restrict__ ts_g) {
  for (int64_t p = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; p < n; p += (int64_t)gridDim.x * blockDim.x)
    ts_g[p] = grank[ts_nb[p]];
}

unsigned grid_waves(int64_t n) {
  const int64_t g = (n + 3) / 4;
  return (unsigned)std::max<int64_t>(1, std::min<int64_t>(g, 16384));
}

}  // namespace

bool build_time_slots(hipStream_t s, const DevGraph& g, int32_t* ts_e, int32_t* ts_nb, int64_t* ts_t,
                      std::vector<void*>& temps) {
  const int64_t n = g.ne + g.n_in;
  if (n <= 0 || n > (int64_t)INT32_MAX) return false;  // (the segmented sort counts items in int)
  auto tmp = [&](size_t bytes) {
    void* p = nullptr;
    if (hipMalloc(&p, bytes) != hipSuccess) throw std::bad_alloc();
    temps.push_back(p);
    return p;
  };
  int64_t* key = static_cast<int64_t*>(tmp(sizeof(int64_t) * n));
  int32_t* val = static_cast<int32_t*>(tmp(sizeof(int32_t) * n));
  k_slot_keys<<<grid_waves(g.nv), 256, 0, s>>>(g.nv, g.out_off, g.in_off, g.in_eid, g.eoff, g.ekey, g.esrc, g.edst,
                                               g.doff, g.dbits, key, val);
  size_t bytes = 0;
  if (hipcub::DeviceSegmentedSort::SortPairsDescending(nullptr, bytes, key, ts_t, val, ts_e, (int)n, (int)g.nv,
                                                       g.adj_off, g.adj_off + 1, s) != hipSuccess)
    return false;
  void* work = tmp(std::max<size_t>(bytes, 16));
  if (hipcub::DeviceSegmentedSort::SortPairsDescending(work, bytes, key, ts_t, val, ts_e, (int)n, (int)g.nv,
                                                       g.adj_off, g.adj_off + 1, s) != hipSuccess)
    return false;
  k_slot_nbrs<<<grid_waves(g.nv), 256, 0, s>>>(g.nv, g.adj_off, g.esrc, g.edst, ts_e, ts_nb);
  return hipGetLastError() == hipSuccess;
}

void build_slot_labels(hipStream_t s, int64_t n, const int32_t* ts_nb, const int32_t* grank, int32_t* ts_g) {
  k_slot_labels<<<(unsigned)std::min<int64_t>((n + 255) / 256, 65536), 256, 0, s>>>(n, ts_nb, grank, ts_g);
}

}  // namespace rgpu
