// window_bits.hpp — a batch's hop table in LDS and the window bits of one history point (K1, and
// the inline edge bits of K2 / the partitioned ghost marking).  Device code only; included by the
// .hip translation units that need it.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "kernels.hpp"

namespace rgpu {

// ---- interval form (hops ascending).  floor(t) = the last point with time <= t (key >> 1),
// so point i is the floor exactly for the hops with time(i) <= t_k < time(i+1): one interval
// of hop indices per point.  Walking the few points between the block's first and last hop
// (one floor search, then a linear walk) replaces a floor search per hop; per alive point the
// window test is another interval, t_k <= time(i) + w.  Edges also end an interval at the
// first endpoint death after time(i) (a death in (time(i), t] kills: killList /
// vertexRemoval).  Entities with more than bp.iv_max points in the block's range (power-law
// hubs) keep the per-hop form.
struct HopLDS {
  int64_t hop[kViews];
  int64_t thr[kViews];
  int K, W, KS;
  int64_t jump;  // > 0: hop[k] = hop[0] + k * jump (a Range job's hops; hop_lb is arithmetic)
  double inv;    // 1 / jump
};
__device__ __forceinline__ void hop_lds_init(HopLDS& L, const BatchParams& bp, const int64_t* thr) {
  if (threadIdx.x < kViews) {
    L.hop[threadIdx.x] = bp.hop[threadIdx.x];
    L.thr[threadIdx.x] = thr[threadIdx.x];
  }
  if (threadIdx.x == 0) {
    L.K = bp.K; L.W = bp.W; L.KS = bp.KS;
    L.jump = bp.jump;
    L.inv = bp.jump > 0 ? 1.0 / (double)bp.jump : 0.0;
  }
  __syncthreads();
}
// first hop index with hop >= x (K if none).  Evenly spaced hops (every Range job's hops but a
// clamped last one): ceil((x - hop0) / jump) from a double product, corrected by one integer
// compare each way (exact: |x - hop0| < 2^53) — no dependent LDS probes.
__device__ __forceinline__ int hop_lb(const HopLDS& L, int64_t x) {
  if (L.jump > 0) {
    const int64_t d = x - L.hop[0];
    if (d <= 0) return 0;
    if (x > L.hop[L.K - 1]) return L.K;
    int64_t k = (int64_t)((double)d * L.inv);
    if (k * L.jump < d) k++;
    if (k > 0 && (k - 1) * L.jump >= d) k--;
    return (int)k;
  }
  int a = 0, b = L.K;
  while (a < b) {
    const int m = (a + b) >> 1;
    if (L.hop[m] < x) a = m + 1; else b = m;
  }
  return a;
}
__device__ __forceinline__ uint64_t range_bits(int a, int b) {  // bits [a, b)
  if (b <= a) return 0;
  return (b - a >= 64 ? ~0ull : ((1ull << (b - a)) - 1)) << a;
}
// bits of alive point time tf whose floor interval is hop indices [a, b)
template <bool PLANAR>
__device__ __forceinline__ void interval_bits(uint64_t (&m)[PLANAR ? kMaxPlanes : 1], const HopLDS& L,
                                              int64_t tf, int a, int b) {
  if (a >= b) return;
  const int64_t tlast = L.hop[b - 1];
  if constexpr (PLANAR) {
#pragma unroll
    for (int w = 0; w < kMaxPlanes; w++)
      if (w < L.W) {
        const int u = L.thr[w] >= tlast - tf ? b : min(b, hop_lb(L, tf + L.thr[w] + 1));
        m[w] |= range_bits(a, u);
      }
  } else {
    for (int w = 0; w < L.W; w++) {
      const int u = L.thr[w] >= tlast - tf ? b : min(b, hop_lb(L, tf + L.thr[w] + 1));
      m[0] |= range_bits(a, u) << (w * L.KS);
    }
  }
}
// the per-hop form's window bits from the LDS copy
template <bool PLANAR>
__device__ __forceinline__ void hop_bits(uint64_t (&m)[PLANAR ? kMaxPlanes : 1], const HopLDS& L,
                                         int64_t age, int k) {
  if constexpr (PLANAR) {
#pragma unroll
    for (int w = 0; w < kMaxPlanes; w++)
      if (w < L.W && age <= L.thr[w]) m[w] |= 1ull << k;
  } else {
    for (int w = 0; w < L.W; w++)
      if (age <= L.thr[w]) m[0] |= 1ull << (w * L.KS + k);
  }
}


// Inline edge bits (K2 of a CC batch): the window bits of a simple static slot (tslots.hip: the
// edge's history is one add point at tf and neither endpoint ever died) for the batch's own views,
// computed where K2 streams the slot's time word instead of loaded from K1's em[e], a random 8-B
// load per static slot and the bulk of K2's traffic.  Such an edge is alive in view (t, w) iff
// tf <= t <= tf + w.  Any other slot reads em[e], which K1 then writes for the other edges only
// (k_edge_mask SKIP).  (Running K1's whole edge_bits inline for them instead took K2 from 77 to 123
// VGPRs.)
// first hop index with hop >= x, by a binary search of the LDS table (few registers: K2 runs this
// per static slot, and the arithmetic form of hop_lb cost it a wave of occupancy)
__device__ __forceinline__ int hop_lb_search(const HopLDS& L, int64_t x) {
  int lo = 0, n = L.K;
  while (n > 0) {
    const int h = n >> 1;
    if (L.hop[lo + h] < x) {
      lo += h + 1;
      n -= h + 1;
    } else {
      n = h;
    }
  }
  return lo;
}
__device__ __forceinline__ uint64_t simple_bits(const HopLDS& L, int sorted, int64_t tf) {
  uint64_t m[1] = {0};
  if (sorted) {  // hops [first >= tf, first > tf + w) of each window
    // (a point before the block's first hop — most slots of a long window — needs no search)
    const int a = tf <= L.hop[0] ? 0 : hop_lb_search(L, tf);
    const int64_t tlast = L.hop[L.K - 1];
    for (int w = 0; w < L.W; w++) {  // (a window reaching past the last hop: no search, no overflow)
      const int u = L.thr[w] >= tlast - tf ? L.K : hop_lb_search(L, tf + L.thr[w] + 1);
      m[0] |= range_bits(a, u) << (w * L.KS);
    }
  } else {
    for (int k = 0; k < L.K; k++)
      if (L.hop[k] >= tf) hop_bits<false>(m, L, L.hop[k] - tf, k);
  }
  return m[0];
}
}  // namespace rgpu
