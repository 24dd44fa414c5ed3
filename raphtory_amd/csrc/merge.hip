// merge.hip — incremental seal (live ingest), device half.
//
// A sealed partition stays resident in HBM; a delta of later updates (packed on the host
// into small sorted lists, packer.cpp pack_delta / finish_delta) is merged into it in place
// of a full re-pack.  The reference appends every update to its entity's TreeMap as it
// arrives (EntityStorage.scala:73-453, Entity.scala:25-57); the merged arrays here equal
// what pack_events would build from base + delta, which the parity tests check.
//
// Every merged array is written by a position formula (no sort on the device):
//  * ranks: old -> new is monotone (new ids are inserted in order), so base edges keep their
//    (src, dst) order; a base edge e lands at e + #(new edges with a smaller key), a new edge
//    i at i + #(base edges with a smaller key) (binary searches);
//  * histories: per entity, base points and delta points are merged by time; at equal time
//    the delta point wins (later put).  Edge histories (short) merge one entity per thread;
//    vertex histories (power-law: hubs hold millions of points) place every point by itself.  A base edge point at the time of a DELTA endpoint
//    death becomes a removal (the kill is the later put, EntityStorage.scala:189-228);
//  * in-edges: per destination, base in-edges and new in-edges interleave by source rank.
// Irregular integer work; HBM-bound.  Bytes per merged entity are its old + new arrays.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "kernels.hpp"

namespace rgpu {
namespace {

constexpr int kB = 256;

inline int grid_for(int64_t n) {
  int64_t b = (n + kB - 1) / kB;
  if (b > 65536) b = 65536;
  return (int)(b < 1 ? 1 : b);
}

// first index in a[0, n) with a[i] >= x
__device__ __forceinline__ int64_t lower64(const int64_t* __restrict__ a, int64_t n, int64_t x) {
  int64_t lo = 0, hi = n;
  while (lo < hi) {
    const int64_t m = (lo + hi) >> 1;
    if (a[m] < x) lo = m + 1;
    else hi = m;
  }
  return lo;
}

__device__ __forceinline__ int64_t base_key(int64_t e, const int32_t* __restrict__ esrc,
                                            const int32_t* __restrict__ edst,
                                            const int32_t* __restrict__ old2new) {
  return ((int64_t)old2new[esrc[e]] << 32) | (uint32_t)old2new[edst[e]];
}

// delta death of rank v at exactly time t
__device__ __forceinline__ bool delta_death(int32_t v, int64_t t, int64_t ndd, const int32_t* __restrict__ dd_rank,
                                            const int64_t* __restrict__ dd_off, const int64_t* __restrict__ dd_t) {
  int64_t lo = 0, hi = ndd;
  while (lo < hi) {
    const int64_t m = (lo + hi) >> 1;
    if (dd_rank[m] < v) lo = m + 1;
    else hi = m;
  }
  if (lo == ndd || dd_rank[lo] != v) return false;
  const int64_t a = dd_off[lo], n = dd_off[lo + 1] - a;
  const int64_t j = lower64(dd_t + a, n, t);
  return j < n && dd_t[a + j] == t;
}

__global__ __launch_bounds__(kB) void k_edge_find(int64_t nq, const int32_t* __restrict__ qs,
                                                  const int32_t* __restrict__ qd,
                                                  const int64_t* __restrict__ out_off,
                                                  const int32_t* __restrict__ edst, int32_t* __restrict__ res) {
  for (int64_t i = blockIdx.x * (int64_t)kB + threadIdx.x; i < nq; i += (int64_t)gridDim.x * kB) {
    const int32_t s = qs[i], d = qd[i];
    int32_t r = -1;
    if (s >= 0 && d >= 0) {
      int64_t lo = out_off[s], hi = out_off[s + 1];
      while (lo < hi) {
        const int64_t m = (lo + hi) >> 1;
        if (edst[m] < d) lo = m + 1;
        else hi = m;
      }
      if (lo < out_off[s + 1] && edst[lo] == d) r = (int32_t)lo;
    }
    res[i] = r;
  }
}

__global__ __launch_bounds__(kB) void k_place_base_edges(int64_t ne_old, const int32_t* __restrict__ esrc,
                                                         const int32_t* __restrict__ edst,
                                                         const int32_t* __restrict__ old2new,
                                                         int64_t n_new, const int64_t* __restrict__ nn_key,
                                                         int32_t* __restrict__ esrc2, int32_t* __restrict__ edst2,
                                                         int32_t* __restrict__ eo2n, int32_t* __restrict__ mbase) {
  for (int64_t e = blockIdx.x * (int64_t)kB + threadIdx.x; e < ne_old; e += (int64_t)gridDim.x * kB) {
    const int64_t k = base_key(e, esrc, edst, old2new);
    const int64_t pos = e + lower64(nn_key, n_new, k);
    esrc2[pos] = (int32_t)(k >> 32);
    edst2[pos] = (int32_t)(k & 0xffffffff);
    eo2n[e] = (int32_t)pos;
    mbase[pos] = (int32_t)e;
  }
}

__global__ __launch_bounds__(kB) void k_place_new_edges(int64_t n_new, const int64_t* __restrict__ nn_key,
                                                        const int32_t* __restrict__ nn_didx, int64_t ne_old,
                                                        const int32_t* __restrict__ esrc,
                                                        const int32_t* __restrict__ edst,
                                                        const int32_t* __restrict__ old2new,
                                                        int32_t* __restrict__ esrc2, int32_t* __restrict__ edst2,
                                                        int32_t* __restrict__ mbase, int32_t* __restrict__ mdlt,
                                                        int32_t* __restrict__ npos) {
  for (int64_t i = blockIdx.x * (int64_t)kB + threadIdx.x; i < n_new; i += (int64_t)gridDim.x * kB) {
    const int64_t k = nn_key[i];
    int64_t lo = 0, hi = ne_old;  // base edges with a smaller (remapped) key
    while (lo < hi) {
      const int64_t m = (lo + hi) >> 1;
      if (base_key(m, esrc, edst, old2new) < k) lo = m + 1;
      else hi = m;
    }
    const int64_t pos = i + lo;
    esrc2[pos] = (int32_t)(k >> 32);
    edst2[pos] = (int32_t)(k & 0xffffffff);
    mbase[pos] = -1;
    mdlt[pos] = nn_didx[i];
    npos[i] = (int32_t)pos;
  }
}

__global__ __launch_bounds__(kB) void k_link_delta_edges(int64_t nde, const int32_t* __restrict__ de_base,
                                                         const int32_t* __restrict__ eo2n,
                                                         int32_t* __restrict__ mdlt) {
  for (int64_t i = blockIdx.x * (int64_t)kB + threadIdx.x; i < nde; i += (int64_t)gridDim.x * kB)
    if (de_base[i] >= 0) mdlt[eo2n[de_base[i]]] = (int32_t)i;
}

// Merge of one entity's base keys a[0,na) and delta keys b[0,nb) (both by time, distinct
// times), delta winning at equal time.  WRITE = false: count only.
template <bool WRITE, class Fix>
__device__ __forceinline__ int64_t merge_keys(const int64_t* __restrict__ a, int64_t na,
                                              const int64_t* __restrict__ b, int64_t nb,
                                              int64_t* __restrict__ out, Fix fix) {
  int64_t i = 0, j = 0, o = 0;
  while (i < na || j < nb) {
    int64_t k;
    if (j == nb || (i < na && (a[i] >> 1) < (b[j] >> 1))) {
      k = fix(a[i++]);
    } else {
      if (i < na && (a[i] >> 1) == (b[j] >> 1)) i++;
      k = b[j++];
    }
    if (WRITE) out[o] = k;
    o++;
  }
  return o;
}

template <bool WRITE>
__global__ __launch_bounds__(kB) void k_edge_hist(int64_t ne2, const int32_t* __restrict__ mbase,
                                                  const int32_t* __restrict__ mdlt,
                                                  const int64_t* __restrict__ eoff, const int64_t* __restrict__ ekey,
                                                  const int64_t* __restrict__ dkoff, const int64_t* __restrict__ dkey,
                                                  const int32_t* __restrict__ esrc2, const int32_t* __restrict__ edst2,
                                                  int64_t ndd, const int32_t* __restrict__ dd_rank,
                                                  const int64_t* __restrict__ dd_off, const int64_t* __restrict__ dd_t,
                                                  int64_t* __restrict__ cnt_off, int64_t* __restrict__ ekey2) {
  for (int64_t e = blockIdx.x * (int64_t)kB + threadIdx.x; e < ne2; e += (int64_t)gridDim.x * kB) {
    const int32_t ob = mbase[e], od = mdlt[e];
    const int64_t a0 = ob >= 0 ? eoff[ob] : 0, na = ob >= 0 ? eoff[ob + 1] - a0 : 0;
    const int64_t b0 = od >= 0 ? dkoff[od] : 0, nb = od >= 0 ? dkoff[od + 1] - b0 : 0;
    const int32_t s = esrc2[e], d = edst2[e];
    auto fix = [&](int64_t k) -> int64_t {
      if (ndd && (k & 1) &&
          (delta_death(s, k >> 1, ndd, dd_rank, dd_off, dd_t) || delta_death(d, k >> 1, ndd, dd_rank, dd_off, dd_t)))
        return k & ~(int64_t)1;
      return k;
    };
    if (WRITE) merge_keys<true>(ekey + a0, na, dkey + b0, nb, ekey2 + cnt_off[e], fix);
    else cnt_off[e] = merge_keys<false>(ekey + a0, na, dkey + b0, nb, nullptr, fix);
  }
}

// ---- vertex histories by position formula (power-law safe: no per-entity serial merge, whose
// cost per wave is the longest history among its 64 lanes — a hub's millions of points).
// Base and delta lists of one vertex are both time-sorted with distinct times; a delta point
// replaces a base point at the same time.  coll[j] = 1 iff delta key j has such a twin; after
// an exclusive scan, coll[j] counts the colliding delta keys before j.
//   count(v)          = na + nb - collisions(v)
//   pos(base a_i)     = voff2[v] + i + #(delta times < t_i) - #(colliding delta keys among those)
//   pos(delta b_j)    = voff2[v] + j + #(base times < t_j) - #(colliding delta keys before j)
// (the base keys dropped before a point are exactly the colliding delta keys before it).
__device__ __forceinline__ int64_t seg_of(const int64_t* __restrict__ off, int64_t nseg, int64_t j) {
  int64_t lo = 0, hi = nseg + 1;  // first index with off > j, minus one
  while (lo < hi) {
    const int64_t m = (lo + hi) >> 1;
    if (off[m] <= j) lo = m + 1;
    else hi = m;
  }
  return lo - 1;
}
__device__ __forceinline__ int64_t find_rank(const int32_t* __restrict__ a, int64_t n, int32_t v) {
  int64_t lo = 0, hi = n;
  while (lo < hi) {
    const int64_t m = (lo + hi) >> 1;
    if (a[m] < v) lo = m + 1;
    else hi = m;
  }
  return lo < n && a[lo] == v ? lo : -1;
}

__global__ __launch_bounds__(kB) void k_dv_collide(int64_t ndvk, int64_t ndv, const int32_t* __restrict__ dv_rank,
                                                   const int64_t* __restrict__ dv_off, const int64_t* __restrict__ dv_key,
                                                   const int32_t* __restrict__ new2old, const int64_t* __restrict__ voff,
                                                   const int64_t* __restrict__ vkey, int64_t* __restrict__ coll) {
  for (int64_t j = blockIdx.x * (int64_t)kB + threadIdx.x; j < ndvk; j += (int64_t)gridDim.x * kB) {
    const int32_t u = new2old[dv_rank[seg_of(dv_off, ndv, j)]];
    int64_t c = 0;
    if (u >= 0) {
      const int64_t a0 = voff[u], na = voff[u + 1] - a0, T = dv_key[j] >> 1;
      const int64_t i = lower64(vkey + a0, na, 2 * T);
      c = i < na && (vkey[a0 + i] >> 1) == T;
    }
    coll[j] = c;
  }
}

__global__ __launch_bounds__(kB) void k_vertex_count(int64_t nv2, const int32_t* __restrict__ new2old,
                                                     const int64_t* __restrict__ voff, int64_t ndv,
                                                     const int32_t* __restrict__ dv_rank, const int64_t* __restrict__ dv_off,
                                                     const int64_t* __restrict__ coll, int64_t* __restrict__ cnt) {
  for (int64_t v = blockIdx.x * (int64_t)kB + threadIdx.x; v < nv2; v += (int64_t)gridDim.x * kB) {
    const int32_t u = new2old[v];
    int64_t c = u >= 0 ? voff[u + 1] - voff[u] : 0;
    const int64_t sg = find_rank(dv_rank, ndv, (int32_t)v);
    if (sg >= 0) c += (dv_off[sg + 1] - dv_off[sg]) - (coll[dv_off[sg + 1]] - coll[dv_off[sg]]);
    cnt[v] = c;
  }
}

__global__ __launch_bounds__(kB) void k_vertex_write_base(int64_t nvk_old, int64_t nv_old, const int64_t* __restrict__ voff,
                                                          const int64_t* __restrict__ vkey, const int32_t* __restrict__ old2new,
                                                          int64_t ndv, const int32_t* __restrict__ dv_rank,
                                                          const int64_t* __restrict__ dv_off, const int64_t* __restrict__ dv_key,
                                                          const int64_t* __restrict__ coll, const int64_t* __restrict__ voff2,
                                                          int64_t* __restrict__ vkey2) {
  for (int64_t i = blockIdx.x * (int64_t)kB + threadIdx.x; i < nvk_old; i += (int64_t)gridDim.x * kB) {
    const int64_t u = seg_of(voff, nv_old, i);
    const int32_t v = old2new[u];
    const int64_t key = vkey[i], T = key >> 1;
    int64_t blt = 0, clt = 0;
    const int64_t sg = find_rank(dv_rank, ndv, v);
    if (sg >= 0) {
      const int64_t b0 = dv_off[sg], nb = dv_off[sg + 1] - b0;
      blt = lower64(dv_key + b0, nb, 2 * T);
      if (blt < nb && (dv_key[b0 + blt] >> 1) == T) continue;  // replaced by the delta point
      clt = coll[b0 + blt] - coll[b0];
    }
    vkey2[voff2[v] + (i - voff[u]) + blt - clt] = key;
  }
}

__global__ __launch_bounds__(kB) void k_vertex_write_delta(int64_t ndvk, int64_t ndv, const int32_t* __restrict__ dv_rank,
                                                           const int64_t* __restrict__ dv_off, const int64_t* __restrict__ dv_key,
                                                           const int32_t* __restrict__ new2old, const int64_t* __restrict__ voff,
                                                           const int64_t* __restrict__ vkey, const int64_t* __restrict__ coll,
                                                           const int64_t* __restrict__ voff2, int64_t* __restrict__ vkey2) {
  for (int64_t j = blockIdx.x * (int64_t)kB + threadIdx.x; j < ndvk; j += (int64_t)gridDim.x * kB) {
    const int64_t sg = seg_of(dv_off, ndv, j);
    const int32_t v = dv_rank[sg];
    const int32_t u = new2old[v];
    const int64_t b0 = dv_off[sg], key = dv_key[j];
    const int64_t alt = u >= 0 ? lower64(vkey + voff[u], voff[u + 1] - voff[u], 2 * (key >> 1)) : 0;
    vkey2[voff2[v] + (j - b0) + alt - (coll[j] - coll[b0])] = key;
  }
}

// base in-edge slot j of old vertex u -> merged slot of new vertex old2new[u]
__global__ __launch_bounds__(kB) void k_in_base(int64_t nin_old, int64_t nv_old, const int64_t* __restrict__ in_off,
                                                const int32_t* __restrict__ in_eid, const int32_t* __restrict__ esrc,
                                                const int32_t* __restrict__ old2new, const int32_t* __restrict__ eo2n,
                                                const int64_t* __restrict__ in_off2, int64_t nni,
                                                const int64_t* __restrict__ ni_key, int32_t* __restrict__ in_eid2) {
  for (int64_t j = blockIdx.x * (int64_t)kB + threadIdx.x; j < nin_old; j += (int64_t)gridDim.x * kB) {
    int64_t lo = 0, hi = nv_old + 1;  // last u with in_off[u] <= j
    while (lo < hi) {
      const int64_t m = (lo + hi) >> 1;
      if (in_off[m] <= j) lo = m + 1;
      else hi = m;
    }
    const int64_t u = lo - 1;
    const int32_t e = in_eid[j];
    const int64_t v = old2new[u], s = old2new[esrc[e]];
    const int64_t before = lower64(ni_key, nni, (v << 32) | s) - lower64(ni_key, nni, v << 32);
    in_eid2[in_off2[v] + (j - in_off[u]) + before] = eo2n[e];
  }
}

__global__ __launch_bounds__(kB) void k_in_new(int64_t nni, const int64_t* __restrict__ ni_key,
                                               const int32_t* __restrict__ ni_idx, const int32_t* __restrict__ npos,
                                               const int32_t* __restrict__ new2old, const int64_t* __restrict__ in_off,
                                               const int32_t* __restrict__ in_eid, const int32_t* __restrict__ esrc,
                                               const int32_t* __restrict__ old2new, const int64_t* __restrict__ in_off2,
                                               int32_t* __restrict__ in_eid2) {
  for (int64_t k = blockIdx.x * (int64_t)kB + threadIdx.x; k < nni; k += (int64_t)gridDim.x * kB) {
    const int64_t key = ni_key[k];
    const int64_t v = key >> 32;
    const int32_t s = (int32_t)(key & 0xffffffff);
    const int64_t idx = k - lower64(ni_key, nni, v << 32);
    const int32_t u = new2old[v];
    int64_t before = 0;
    if (u >= 0) {  // base in-edges of v with a smaller source
      int64_t lo = in_off[u], hi = in_off[u + 1];
      while (lo < hi) {
        const int64_t m = (lo + hi) >> 1;
        if (old2new[esrc[in_eid[m]]] < s) lo = m + 1;
        else hi = m;
      }
      before = lo - in_off[u];
    }
    in_eid2[in_off2[v] + idx + before] = npos[ni_idx[k]];
  }
}

// exclusive prefix sum in place over off[0, n] where off[i] holds a count for i < n:
// one pass per 1,024-element tile (block scan), tile sums scanned by a single block, fix-up.
constexpr int kScanTile = 1024;
__global__ __launch_bounds__(kB) void k_scan_tiles(int64_t n, int64_t* __restrict__ a, int64_t* __restrict__ tsum) {
  __shared__ int64_t s[kScanTile];
  const int64_t t0 = (int64_t)blockIdx.x * kScanTile;
  for (int i = threadIdx.x; i < kScanTile; i += kB) s[i] = t0 + i < n ? a[t0 + i] : 0;
  __syncthreads();
  for (int off = 1; off < kScanTile; off <<= 1) {  // Hillis-Steele on 4 elements per thread
    int64_t v[4];
    for (int q = 0; q < 4; q++) {
      const int i = threadIdx.x + q * kB;
      v[q] = i >= off ? s[i - off] : 0;
    }
    __syncthreads();
    for (int q = 0; q < 4; q++) s[threadIdx.x + q * kB] += v[q];
    __syncthreads();
  }
  for (int i = threadIdx.x; i < kScanTile; i += kB)
    if (t0 + i < n) a[t0 + i] = i ? s[i - 1] : 0;  // exclusive within the tile
  if (threadIdx.x == 0) tsum[blockIdx.x] = s[kScanTile - 1];
}
__global__ __launch_bounds__(1024) void k_scan_sums(int64_t nt, int64_t* __restrict__ tsum, int64_t* __restrict__ total) {
  // one block: serial chunks of 1,024 with a block scan each
  __shared__ int64_t s[1024];
  int64_t carry = 0;
  for (int64_t c = 0; c < nt; c += 1024) {
    const int64_t i = c + threadIdx.x;
    s[threadIdx.x] = i < nt ? tsum[i] : 0;
    __syncthreads();
    for (int off = 1; off < 1024; off <<= 1) {
      const int64_t v = threadIdx.x >= off ? s[threadIdx.x - off] : 0;
      __syncthreads();
      s[threadIdx.x] += v;
      __syncthreads();
    }
    if (i < nt) tsum[i] = carry + (threadIdx.x ? s[threadIdx.x - 1] : 0);
    carry += s[1023];
    __syncthreads();
  }
  if (threadIdx.x == 0) *total = carry;
}
__global__ __launch_bounds__(kB) void k_scan_fix(int64_t n, int64_t* __restrict__ a, const int64_t* __restrict__ tsum,
                                                 const int64_t* __restrict__ total) {
  for (int64_t i = blockIdx.x * (int64_t)kB + threadIdx.x; i <= n; i += (int64_t)gridDim.x * kB)
    a[i] = i < n ? a[i] + tsum[i / kScanTile] : *total;
}

}  // namespace

void launch_edge_find(hipStream_t s, int64_t nq, const int32_t* qs, const int32_t* qd, const int64_t* out_off,
                      const int32_t* edst, int32_t* res) {
  if (nq) k_edge_find<<<grid_for(nq), kB, 0, s>>>(nq, qs, qd, out_off, edst, res);
}

void launch_merge_edges(hipStream_t s, const MergeIn& m, int32_t* esrc2, int32_t* edst2, int32_t* eo2n,
                        int32_t* mbase, int32_t* mdlt, int32_t* npos) {
  (void)hipMemsetAsync(mdlt, 0xff, sizeof(int32_t) * (m.ne_old + m.n_new), s);
  if (m.ne_old)
    k_place_base_edges<<<grid_for(m.ne_old), kB, 0, s>>>(m.ne_old, m.esrc, m.edst, m.old2new, m.n_new, m.nn_key,
                                                         esrc2, edst2, eo2n, mbase);
  if (m.n_new)
    k_place_new_edges<<<grid_for(m.n_new), kB, 0, s>>>(m.n_new, m.nn_key, m.nn_didx, m.ne_old, m.esrc, m.edst,
                                                       m.old2new, esrc2, edst2, mbase, mdlt, npos);
  if (m.nde) k_link_delta_edges<<<grid_for(m.nde), kB, 0, s>>>(m.nde, m.de_base, eo2n, mdlt);
}

void launch_scan_counts(hipStream_t s, int64_t n, int64_t* off, int64_t* tmp) {
  const int64_t nt = (n + kScanTile - 1) / kScanTile;
  int64_t* tsum = tmp;
  int64_t* total = tmp + (nt ? nt : 1);
  if (nt) {
    k_scan_tiles<<<(unsigned)nt, kB, 0, s>>>(n, off, tsum);
    k_scan_sums<<<1, 1024, 0, s>>>(nt, tsum, total);
  } else {
    (void)hipMemsetAsync(total, 0, sizeof(int64_t), s);
  }
  k_scan_fix<<<grid_for(n + 1), kB, 0, s>>>(n, off, tsum, total);
}
int64_t scan_tmp_words(int64_t n) { return (n + kScanTile - 1) / kScanTile + 2; }

void launch_edge_hist(hipStream_t s, bool write, const MergeIn& m, int64_t ne2, const int32_t* mbase,
                      const int32_t* mdlt, const int32_t* esrc2, const int32_t* edst2, int64_t* cnt_off,
                      int64_t* ekey2) {
  if (!ne2) return;
  if (write)
    k_edge_hist<true><<<grid_for(ne2), kB, 0, s>>>(ne2, mbase, mdlt, m.eoff, m.ekey, m.dkoff, m.dkey, esrc2, edst2,
                                                   m.ndd, m.dd_rank, m.dd_off, m.dd_t, cnt_off, ekey2);
  else
    k_edge_hist<false><<<grid_for(ne2), kB, 0, s>>>(ne2, mbase, mdlt, m.eoff, m.ekey, m.dkoff, m.dkey, esrc2, edst2,
                                                    m.ndd, m.dd_rank, m.dd_off, m.dd_t, cnt_off, ekey2);
}

void launch_vertex_hist(hipStream_t s, bool write, const MergeIn& m, int64_t* cnt_off, int64_t* vkey2) {
  if (!m.nv2) return;
  if (!write) {  // collision flags -> exclusive prefix (m.coll[0, ndvk]), then per-vertex counts
    if (m.ndvk) {
      k_dv_collide<<<grid_for(m.ndvk), kB, 0, s>>>(m.ndvk, m.ndv, m.dv_rank, m.dv_off, m.dv_key, m.new2old, m.voff,
                                                  m.vkey, m.coll);
      launch_scan_counts(s, m.ndvk, m.coll, m.coll_tmp);
    }
    k_vertex_count<<<grid_for(m.nv2), kB, 0, s>>>(m.nv2, m.new2old, m.voff, m.ndv, m.dv_rank, m.dv_off, m.coll,
                                                 cnt_off);
    return;
  }
  if (m.nvk_old)
    k_vertex_write_base<<<grid_for(m.nvk_old), kB, 0, s>>>(m.nvk_old, m.nv_old, m.voff, m.vkey, m.old2new, m.ndv,
                                                           m.dv_rank, m.dv_off, m.dv_key, m.coll, cnt_off, vkey2);
  if (m.ndvk)
    k_vertex_write_delta<<<grid_for(m.ndvk), kB, 0, s>>>(m.ndvk, m.ndv, m.dv_rank, m.dv_off, m.dv_key, m.new2old,
                                                         m.voff, m.vkey, m.coll, cnt_off, vkey2);
}

void launch_merge_in(hipStream_t s, const MergeIn& m, const int32_t* eo2n, const int32_t* npos,
                     const int64_t* in_off2, int32_t* in_eid2) {
  if (m.nin_old)
    k_in_base<<<grid_for(m.nin_old), kB, 0, s>>>(m.nin_old, m.nv_old, m.in_off, m.in_eid, m.esrc, m.old2new, eo2n,
                                                 in_off2, m.nni, m.ni_key, in_eid2);
  if (m.nni)
    k_in_new<<<grid_for(m.nni), kB, 0, s>>>(m.nni, m.ni_key, m.ni_idx, npos, m.new2old, m.in_off, m.in_eid, m.esrc,
                                            m.old2new, in_off2, in_eid2);
}

}  // namespace rgpu
