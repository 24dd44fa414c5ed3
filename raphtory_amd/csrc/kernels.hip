// kernels.hip — gfx950 kernels of the windowed temporal-analysis path.
//
// Layout: a *batch* holds up to 64 views (hop k, window w) -> bit / lane j = k*W + w.
// Every per-vertex quantity of a batch is a 64-lane row (one wavefront lane per view), so
// one pass over the adjacency serves every view of every hop in the batch.
//
//   k_vertex_mask  K1  Entity.aliveAtWithWindow for every vertex x hop x window, with the
//                      batched running-min window (WindowLens.shrinkWindow, WindowLens.scala:59-65)
//   k_edge_mask    K1  the same for edges: own history + endpoint death lists (killList)
//   k_cc_slots     K2  per-view adjacency filter (Vertex.viewAtWithWindow, Vertex.scala:70-74)
//                      compacted into a batch CSR with a 64-bit view mask per slot
//   k_cc_step      K3  one CC superstep for all views (ConnectedComponents.analyse :19-35)
//   k_cc_count/roots K5 label->count at the root's row + processBatchWindowResults summary (:137-145)
//   k_degree       DegreeBasic.returnResults (DegreeBasic.scala:16-28)
//   k_pr_slots/k_pr_step  PageRank spec
#include <hip/hip_runtime.h>

#include <type_traits>

#include <climits>
#include <cstdint>
#include <cstring>
#include <cstdlib>

#include <algorithm>
#include <stdexcept>

#include <hipcub/device/device_scan.hpp>

#include "kernels.hpp"
#include "window_bits.hpp"

namespace rgpu {

__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }
__device__ __forceinline__ uint64_t readlane64(uint64_t x, int l) {
  uint32_t lo = __builtin_amdgcn_readlane((uint32_t)x, l);
  uint32_t hi = __builtin_amdgcn_readlane((uint32_t)(x >> 32), l);
  return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ uint64_t lanemask_lt() {
  int l = lane_id();
  return l == 0 ? 0ull : (~0ull >> (64 - l));
}

// ---------------------------------------------------------------- label-row access
// A label row is 64 lanes x 4 B = 256 B (four 64-B lines).  Rows are read and written
// through a per-row buffer descriptor (the row base is wave-uniform): a lane that must not
// touch memory gets an out-of-range offset, so it reads 0 / writes nothing with no memory
// traffic and no exec-masked branch (a branchy predicated load makes hipcc wait vmcnt(0)
// before the other path writes the same register).  Stores cover whole 64-B lines of the
// lanes that matter, never partial lines (a partial-line store costs a fill).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t row_rsrc(const int32_t* row) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)row, (short)0, 256, 0x00020000);
}
__device__ __forceinline__ int32_t row_load(const int32_t* row, bool on, int lane) {
  return (int32_t)__builtin_amdgcn_raw_buffer_load_b32(row_rsrc(row), on ? lane * 4 : 0x7fffffff, 0, 0);
}
__device__ __forceinline__ void row_store(int32_t* row, int32_t x, bool on, int lane) {
  __builtin_amdgcn_raw_buffer_store_b32(x, row_rsrc(row), on ? lane * 4 : 0x7fffffff, 0, 0);
}
// lanes of the 64-B lines (16 lanes each) that hold at least one view of mask m
__device__ __forceinline__ bool line_has(uint64_t m, int lane) { return ((m >> (lane & 48)) & 0xffffull) != 0; }

// Uniform label words (uw, one int32 per vertex and label buffer): when every member lane of
// a vertex's row holds the same label x the row is kept as uw[v] = x alone (kMixed: the row in
// the label buffer is the state).  A gather from a uniform neighbour costs its 4-B word, not
// its 256-B row, and a uniform vertex neither reads nor writes its own row.  In a batch of
// near-identical views (64 hourly hops of a year window) almost every row is uniform.  The
// state of a vertex in a buffer is the pair (uw, row); every writer writes uw, and the row
// only when mixed, so the "both buffers agree unless changed in the last two steps" rule of
// the label rows carries over unchanged.  Rows are materialised (k_uw_rows) before anything
// outside the superstep loop reads them.
// kMixed, kChgFlag, uw_label, uw_word: kernels.hpp.  A uniform word also carries bit 31
// (kChgFlag) when the vertex's label changed in the step that wrote it, so a neighbour reads one
// random 4-B word per slot (label and "changed" together) instead of its 8-B change word and then
// the word.  Only mixed neighbours (kMixed) need their change word and row.  A flag left over from
// an older step (a vertex not visited since) only makes a reader fold an unchanged label, which
// changes nothing: L_r(v) = min over the ball of radius r, and the neighbour's current label was
// already folded into v's when the neighbour last changed.

// fold the labels x (per lane = slot, wave-uniform loop over the lanes of `bal`) into best
// (lane = view) on the views a of each slot
__device__ __forceinline__ int32_t fold_uniform(uint64_t bal, uint64_t a, int32_t x, int32_t best, int lane) {
  while (bal) {
    const int L = __builtin_ctzll(bal);
    bal &= bal - 1;
    const int32_t q = __builtin_amdgcn_readlane(x, L);
    if ((readlane64(a, L) >> lane) & 1) best = min(best, q);
  }
  return best;
}

// uw of a freshly computed row (lane = view, member lanes mv): x if uniform, else kMixed.  The
// label INT32_MAX is kept as a row (its flagged form would read as kMixed).
__device__ __forceinline__ uint64_t shfl_xor64(uint64_t x, int d) {
  const uint32_t lo = __shfl_xor((uint32_t)x, d), hi = __shfl_xor((uint32_t)(x >> 32), d);
  return ((uint64_t)hi << 32) | lo;
}
// fold_uniform by distinct label, smallest first: the smallest label among the remaining lanes is
// final on every view its lanes cover (no remaining lane can lower those views), and lanes whose
// views are all covered drop out.  A hub's changed neighbours in a converging view carry few
// distinct labels, so this is a few rounds (two wave reductions each) instead of one round per
// lane; the last few lanes go lane by lane (folding a larger label into a covered view is a no-op).
__device__ __forceinline__ int32_t fold_uniform_by_label(uint64_t bal, uint64_t a, int32_t x, int32_t best, int lane) {
  bal &= __ballot(a != 0);
  uint64_t done = 0;
  while (__popcll(bal) > 8) {
    int32_t y = ((bal >> lane) & 1) ? x : INT32_MAX;
    for (int o = 32; o > 0; o >>= 1) y = min(y, __shfl_xor(y, o));
    const uint64_t sel = __ballot(((bal >> lane) & 1) && x == y);
    uint64_t cov = ((sel >> lane) & 1) ? a : 0ull;
    for (int o = 32; o > 0; o >>= 1) cov |= shfl_xor64(cov, o);
    cov &= ~done;
    if ((cov >> lane) & 1) best = min(best, y);
    done |= cov;
    bal &= ~sel & __ballot((a & ~done) != 0);
  }
  return fold_uniform(bal, a, x, best, lane);
}
__device__ __forceinline__ int32_t row_uniform(int32_t best, uint64_t mv, int lane) {
  const int32_t x0 = __builtin_amdgcn_readlane(best, __builtin_ctzll(mv));
  return (x0 == INT32_MAX || __ballot(((mv >> lane) & 1) && best != x0)) ? kMixed : x0;
}

// floor(t) of a sorted key list (key = time*2 + alive): index of the last key <= 2t+1, or -1.
__device__ __forceinline__ int64_t floor_idx(const int64_t* key, int64_t lo, int64_t hi, int64_t t) {
  const int64_t probe = 2 * t + 1;
  int64_t a = lo, b = hi;
  while (a < b) {
    int64_t m = (a + b) >> 1;
    if (key[m] <= probe) a = m + 1; else b = m;
  }
  return a - 1 >= lo ? a - 1 : -1;
}
// last death time <= t in a sorted list, or -1
__device__ __forceinline__ int64_t last_death(const int64_t* dt, int64_t lo, int64_t hi, int64_t t) {
  int64_t a = lo, b = hi;
  while (a < b) {
    int64_t m = (a + b) >> 1;
    if (dt[m] <= t) a = m + 1; else b = m;
  }
  return a > lo ? dt[a - 1] : -1;
}

// ---------------------------------------------------------------- K1: window masks
// Advance a floor index to hop time t (hops of a batch ascend when bp.sorted): step forward
// while the next key is <= 2t+1; after 8 steps fall back to a binary search of the rest.
__device__ __forceinline__ int64_t floor_advance(const int64_t* key, int64_t f, int64_t lo, int64_t hi,
                                                 int64_t t) {
  const int64_t probe = 2 * t + 1;
  int64_t g = f < lo ? lo : f + 1;  // first candidate after the current floor
  for (int s = 0; s < 8; s++) {
    if (g >= hi || key[g] > probe) return g - 1 >= lo ? g - 1 : -1;
    g++;
  }
  return floor_idx(key, g, hi, t) >= 0 ? floor_idx(key, g, hi, t) : g - 1;
}
// first index in [p, hi) whose death time is > t (binary search)
__device__ __forceinline__ int64_t first_after(const int64_t* dt, int64_t p, int64_t hi, int64_t t) {
  int64_t a = p, b = hi;
  while (a < b) {
    const int64_t m = (a + b) >> 1;
    if (dt[m] <= t) a = m + 1; else b = m;
  }
  return a;
}
// A batch's small state (stats words, superstep flags, frontier flags) is cleared by its
// first kernel: the vertex-mask kernel when the batch has its own masks, else k_batch_clear.
__device__ __forceinline__ void batch_clear(const BatchClear& clr) {
  const int64_t tid = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  const int64_t nth = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = tid; i < clr.n_stats; i += nth) clr.stats[i] = 0;
  for (int64_t i = tid; i < clr.n_flags; i += nth) clr.flags[i] = 0;
  for (int b = 0; b < 3; b++)
    if (clr.act[b])
      for (int64_t i = tid; i < clr.n_act_words; i += nth) reinterpret_cast<uint64_t*>(clr.act[b])[i] = 0;
  for (int b = 0; b < 3; b++)
    if (clr.cb[b])
      for (int64_t i = tid; i < clr.n_cb_words; i += nth) clr.cb[b][i] = 0;
  for (int64_t i = tid; i < clr.n_ccount; i += nth) clr.ccount[i] = 0;
}
__global__ __launch_bounds__(256) void k_batch_clear(BatchClear clr) { batch_clear(clr); }

// Window bits of an entity.  PLANAR = false: one word, bit w*KS + k (all windows of the batch
// in one label row).  PLANAR = true: one word per window (plane w, bit k), W <= kMaxPlanes —
// the masks of one hop block for every window-major batch that will use it.
template <bool PLANAR>
__device__ __forceinline__ void store_bits(const uint64_t (&m)[PLANAR ? kMaxPlanes : 1], const BatchParams& bp,
                                           uint64_t* out, int64_t stride, int64_t i) {
  if constexpr (PLANAR) {
#pragma unroll
    for (int w = 0; w < kMaxPlanes; w++)
      if (w < bp.W) out[w * stride + i] = m[w];
  } else {
    out[i] = m[0];
  }
}

// (the hop table and the interval / per-hop window bits: window_bits.hpp)

// The floors at a sorted block's first and last hop.  carry == 2: the entity's floor at the run's
// previous block's last hop (fc[i], relative to lo; that hop <= hop[0]) is advanced instead of
// searched — a history rarely has a point between two adjacent blocks, so this is one compare in
// place of a binary search (§8(f) row 2, RangeAnalysisTask.restart's hop after hop).  The floor
// at the last hop is advanced from the first's either way (few points fall inside a block).
__device__ __forceinline__ void block_floors(const int64_t* __restrict__ key, int64_t lo, int64_t hi,
                                             const BatchParams& bp, const HopLDS& L, const int32_t* __restrict__ fc,
                                             int64_t i, int64_t& f0, int64_t& f1) {
  if (bp.carry == 2) {
    const int32_t c = fc[i];
    f0 = floor_advance(key, c < 0 ? -1 : lo + c, lo, hi, L.hop[0]);
  } else {
    f0 = floor_idx(key, lo, hi, L.hop[0]);
  }
  f1 = bp.carry ? floor_advance(key, f0, lo, hi, L.hop[L.K - 1]) : floor_idx(key, lo, hi, L.hop[L.K - 1]);
}
__device__ __forceinline__ void store_carry(int32_t* __restrict__ fc, const BatchParams& bp, int64_t i, int64_t f1,
                                            int64_t lo) {
  if (bp.carry) fc[i] = f1 < 0 ? -1 : (int32_t)(f1 - lo);
}

// An entity with more than bp.iv_max points between a sorted block's first and last hop (a
// power-law hub: a vertex has a point per EADD touching it, thousands per hour) took the per-hop
// form in its own thread: 64 dependent floor advances, each up to 8 steps and a binary search —
// ~1,800 dependent loads, so that thread alone set the launch's length (a K1 launch over a 2.2M-
// vertex partition lasted 0.5 ms).  The wave now takes such entities one at a time, lane = hop: each
// lane searches its own hop's floor in [f0, f1] (the block's first and last floors bound every hop's),
// all in flight together, and the window bits are ballots (lane k is bit k of a plane).
// (f0 < 0: no point at or before the first hop; the points from lo on count)
__device__ __forceinline__ int64_t block_points(int64_t lo, int64_t f0, int64_t f1) { return f1 - (f0 < 0 ? lo - 1 : f0); }
// floor of lane k's hop within [a, f1] (f1 = the floor at the block's last hop), or -1
__device__ __forceinline__ int64_t floor_in(const int64_t* __restrict__ key, int64_t a, int64_t f1, int64_t t) {
  const int64_t probe = 2 * t + 1;
  int64_t lo = a, hi = f1 + 1;
  while (lo < hi) {
    const int64_t m = (lo + hi) >> 1;
    if (key[m] <= probe) lo = m + 1; else hi = m;
  }
  return lo - 1 >= a ? lo - 1 : -1;
}
// lane = hop: the window planes of one entity from each lane's (alive, age), as ballots
template <bool PLANAR>
__device__ __forceinline__ void lane_hop_bits(uint64_t (&m)[PLANAR ? kMaxPlanes : 1], const HopLDS& L, bool alive,
                                              int64_t age) {
  if constexpr (PLANAR) {
#pragma unroll
    for (int w = 0; w < kMaxPlanes; w++) m[w] = w < L.W ? __ballot(alive && age <= L.thr[w]) : 0ull;
  } else {
    m[0] = 0;
    for (int w = 0; w < L.W; w++) m[0] |= __ballot(alive && age <= L.thr[w]) << (w * L.KS);
  }
}

template <bool PLANAR>
__global__ __launch_bounds__(256) void k_vertex_mask(int64_t nv, const int64_t* __restrict__ voff,
                                                     const int64_t* __restrict__ vkey, BatchParams bp,
                                                     uint64_t* __restrict__ vm, int64_t vstride,
                                                     BatchClear clr, int32_t* __restrict__ fc) {
  __shared__ HopLDS L;
  hop_lds_init(L, bp, bp.thr_v);
  batch_clear(clr);
  const int K = L.K;
  const int lane = lane_id();
  // wave-uniform loop (lane = vertex): the wave's hubs are then done together, lane = hop
  for (int64_t v0 = blockIdx.x * (int64_t)blockDim.x + (threadIdx.x & ~63); v0 < nv;
       v0 += (int64_t)gridDim.x * blockDim.x) {
    const int64_t v = v0 + lane;
    bool hub = false;
    int64_t lo = 0, f0 = -1, f1 = -1;
    if (v < nv) {
      lo = voff[v];
      const int64_t hi = voff[v + 1];
      uint64_t m[PLANAR ? kMaxPlanes : 1] = {};
      if (bp.sorted) {
        block_floors(vkey, lo, hi, bp, L, fc, v, f0, f1);
        store_carry(fc, bp, v, f1, lo);
        if (bp.iv_max >= 0 && block_points(lo, f0, f1) <= bp.iv_max) {  // f1 < 0: dead at every hop
          for (int64_t i = f0 < 0 ? lo : f0; i <= f1; i++) {
            const int64_t key = vkey[i];
            if (!(key & 1)) continue;  // a deletion: dead over its interval
            const int64_t tf = key >> 1;
            const int b = i + 1 < hi ? hop_lb(L, vkey[i + 1] >> 1) : K;
            interval_bits<PLANAR>(m, L, tf, hop_lb(L, tf), b);
          }
          store_bits<PLANAR>(m, bp, vm, vstride, v);
        } else {
          hub = true;
        }
      } else {  // hops not ascending: the per-hop search in this thread
        for (int k = 0; k < K; k++) {
          const int64_t t = L.hop[k];
          const int64_t f = floor_idx(vkey, lo, hi, t);
          if (f < 0) continue;
          const int64_t key = vkey[f];
          if (!(key & 1)) continue;  // floor is a deletion
          hop_bits<PLANAR>(m, L, t - (key >> 1), k);
        }
        store_bits<PLANAR>(m, bp, vm, vstride, v);
      }
    }
    for (uint64_t hb = __ballot(hub); hb; hb &= hb - 1) {
      const int H = __builtin_ctzll(hb);
      const int64_t loH = (int64_t)readlane64((uint64_t)lo, H), f0H = (int64_t)readlane64((uint64_t)f0, H);
      const int64_t f1H = (int64_t)readlane64((uint64_t)f1, H);
      bool alive = false;
      int64_t age = 0;
      if (lane < K && f1H >= 0) {
        const int64_t t = L.hop[lane];
        const int64_t f = floor_in(vkey, f0H < 0 ? loH : f0H, f1H, t);
        if (f >= 0) {
          const int64_t key = vkey[f];
          alive = (key & 1) != 0;
          age = t - (key >> 1);
        }
      }
      uint64_t m[PLANAR ? kMaxPlanes : 1];
      lane_hop_bits<PLANAR>(m, L, alive, age);
      if (lane == H) store_bits<PLANAR>(m, bp, vm, vstride, v);
    }
  }
}

// Window bits of edge e (own history + endpoint death lists), interval or per-hop form.  A sorted
// block's edge with more than bp.iv_max points in the block is not done here: the function returns
// true with its floors (f0, f1) and death-list ranges, and the wave does it lane = hop (edge_hub_bits).
struct EdgeHub {
  int64_t lo = 0, f0 = -1, f1 = -1, s0 = 0, s1 = 0, d0 = 0, d1 = 0;
};
template <bool PLANAR>
__device__ __forceinline__ bool edge_bits(uint64_t (&m)[PLANAR ? kMaxPlanes : 1], const HopLDS& L,
                                          const BatchParams& bp, int64_t e, const int32_t* __restrict__ esrc,
                                          const int32_t* __restrict__ edst, const int64_t* __restrict__ eoff,
                                          const int64_t* __restrict__ ekey, const int64_t* __restrict__ doff,
                                          const int64_t* __restrict__ dtime, const uint64_t* __restrict__ dbits,
                                          int32_t* __restrict__ fc, EdgeHub& hb) {
  const int K = L.K;
  const int64_t lo = eoff[e], hi = eoff[e + 1];
  const int32_t s = esrc[e], d = edst[e];
  // endpoints without deaths (an L2-resident bit each) skip their death-list offsets: an empty
  // list [0, 0) reads as "no death" everywhere below
  const bool ds = !dbits || ((dbits[s >> 6] >> (s & 63)) & 1), dd = !dbits || ((dbits[d >> 6] >> (d & 63)) & 1);
  const int64_t s0 = ds ? doff[s] : 0, s1 = ds ? doff[s + 1] : 0, d0 = dd ? doff[d] : 0, d1 = dd ? doff[d + 1] : 0;
  if (bp.sorted) {
    int64_t f0, f1;
    block_floors(ekey, lo, hi, bp, L, fc, e, f0, f1);
    store_carry(fc, bp, e, f1, lo);
    if (bp.iv_max >= 0 && block_points(lo, f0, f1) <= bp.iv_max) {
      for (int64_t i = f0 < 0 ? lo : f0; i <= f1; i++) {
        const int64_t key = ekey[i];
        if (!(key & 1)) continue;
        const int64_t tf = key >> 1;
        int b = i + 1 < hi ? hop_lb(L, ekey[i + 1] >> 1) : K;
        // first endpoint death after tf ends the interval
        const int64_t ps = first_after(dtime, s0, s1, tf), pd = first_after(dtime, d0, d1, tf);
        const int64_t dn = min(ps < s1 ? dtime[ps] : INT64_MAX, pd < d1 ? dtime[pd] : INT64_MAX);
        if (dn != INT64_MAX) b = min(b, hop_lb(L, dn));
        interval_bits<PLANAR>(m, L, tf, hop_lb(L, tf), b);
      }
      return false;
    }
    hb.lo = lo; hb.f0 = f0; hb.f1 = f1; hb.s0 = s0; hb.s1 = s1; hb.d0 = d0; hb.d1 = d1;
    return true;
  }
  for (int k = 0; k < K; k++) {  // hops not ascending: the per-hop search in this thread
    const int64_t t = L.hop[k];
    const int64_t f = floor_idx(ekey, lo, hi, t);
    if (f < 0) continue;
    const int64_t key = ekey[f];
    if (!(key & 1)) continue;
    const int64_t ft = key >> 1;
    // an endpoint death in (ft, t] is a later kill point (killList / vertexRemoval)
    const int64_t lds = s1 > s0 ? last_death(dtime, s0, s1, t) : -1;
    const int64_t ldd = d1 > d0 ? last_death(dtime, d0, d1, t) : -1;
    if (lds > ft || ldd > ft) continue;
    hop_bits<PLANAR>(m, L, t - ft, k);
  }
  return false;
}
// lane = hop: the window bits of a hub edge (edge_bits returned true), every lane's floor and
// endpoint death searches in flight together; call from the whole wave
template <bool PLANAR>
__device__ __forceinline__ void edge_hub_bits(uint64_t (&m)[PLANAR ? kMaxPlanes : 1], const HopLDS& L,
                                              const EdgeHub& h, const int64_t* __restrict__ ekey,
                                              const int64_t* __restrict__ dtime, int lane) {
  bool alive = false;
  int64_t age = 0;
  if (lane < L.K && h.f1 >= 0) {
    const int64_t t = L.hop[lane];
    const int64_t f = floor_in(ekey, h.f0 < 0 ? h.lo : h.f0, h.f1, t);
    if (f >= 0) {
      const int64_t key = ekey[f];
      const int64_t ft = key >> 1;
      const int64_t lds = h.s1 > h.s0 ? last_death(dtime, h.s0, h.s1, t) : -1;
      const int64_t ldd = h.d1 > h.d0 ? last_death(dtime, h.d0, h.d1, t) : -1;
      alive = (key & 1) && !(lds > ft || ldd > ft);
      age = t - ft;
    }
  }
  lane_hop_bits<PLANAR>(m, L, alive, age);
}

// an edge whose bits K2 computes itself (the same test as tslots.hip k_slot_keys)
__device__ __forceinline__ bool edge_simple(int64_t lo, int64_t hi, const int64_t* __restrict__ ekey, int32_t s,
                                            int32_t d, const int64_t* __restrict__ doff,
                                            const uint64_t* __restrict__ dbits) {
  if (hi - lo != 1 || !(ekey[lo] & 1)) return false;
  const bool ds = dbits ? ((dbits[s >> 6] >> (s & 63)) & 1) : doff[s + 1] > doff[s];
  const bool dd = dbits ? ((dbits[d >> 6] >> (d & 63)) & 1) : doff[d + 1] > doff[d];
  return !ds && !dd;
}

// simple edges (edge_simple) of a graph: the edge-mask kernel's SKIP byte model (rgpu.cpp bytes_emask)
__global__ __launch_bounds__(256) void k_count_simple(int64_t ne, const int32_t* __restrict__ esrc,
                                                      const int32_t* __restrict__ edst,
                                                      const int64_t* __restrict__ eoff,
                                                      const int64_t* __restrict__ ekey,
                                                      const int64_t* __restrict__ doff,
                                                      const uint64_t* __restrict__ dbits,
                                                      unsigned long long* __restrict__ out) {
  unsigned long long k = 0;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < ne; e += (int64_t)gridDim.x * blockDim.x)
    k += edge_simple(eoff[e], eoff[e + 1], ekey, esrc[e], edst[e], doff, dbits);
  for (int o = 32; o > 0; o >>= 1) k += __shfl_xor(k, o);
  if ((threadIdx.x & 63) == 0 && k) atomicAdd(out, k);
}
void launch_count_simple(hipStream_t s, const DevGraph& g, unsigned long long* out) {
  if (g.ne > 0)
    k_count_simple<<<1024, 256, 0, s>>>(g.ne, g.esrc, g.edst, g.eoff, g.ekey, g.doff, g.dbits, out);
}
// lane = edge, one bitmap word per wave (64 consecutive edges)
__global__ __launch_bounds__(256) void k_edge_simple_bits(int64_t ne, const int32_t* __restrict__ esrc,
                                                          const int32_t* __restrict__ edst,
                                                          const int64_t* __restrict__ eoff,
                                                          const int64_t* __restrict__ ekey,
                                                          const int64_t* __restrict__ doff,
                                                          const uint64_t* __restrict__ dbits,
                                                          uint64_t* __restrict__ out) {
  const int lane = lane_id();
  for (int64_t e0 = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) & ~63ll; e0 < ne;
       e0 += (int64_t)gridDim.x * blockDim.x) {
    const int64_t e = e0 + lane;
    const uint64_t w = __ballot(e < ne && edge_simple(eoff[e], eoff[e + 1], ekey, esrc[e], edst[e], doff, dbits));
    if (lane == 0) out[e0 >> 6] = w;
  }
}
void launch_edge_simple_bits(hipStream_t s, const DevGraph& g, uint64_t* out) {
  if (g.ne > 0)
    k_edge_simple_bits<<<(unsigned)std::min<int64_t>((g.ne + 255) / 256, 16384), 256, 0, s>>>(
        g.ne, g.esrc, g.edst, g.eoff, g.ekey, g.doff, g.dbits, out);
}

// the non-simple edge list (DevGraph.ens): per 64-edge word its count, scanned, then each written
__global__ __launch_bounds__(256) void k_ns_count(int64_t ne, const uint64_t* __restrict__ es, int32_t* __restrict__ cnt) {
  const int64_t nw = (ne + 63) >> 6;
  for (int64_t w = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; w < nw; w += (int64_t)gridDim.x * blockDim.x) {
    const int64_t left = ne - w * 64;
    const uint64_t valid = left >= 64 ? ~0ull : ((1ull << left) - 1);
    cnt[w] = __popcll(~es[w] & valid);
  }
}
__global__ __launch_bounds__(256) void k_ns_write(int64_t ne, const uint64_t* __restrict__ es, const int64_t* __restrict__ off,
                                                  int32_t* __restrict__ out) {
  const int64_t nw = (ne + 63) >> 6;
  for (int64_t w = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; w < nw; w += (int64_t)gridDim.x * blockDim.x) {
    const int64_t left = ne - w * 64;
    uint64_t m = ~es[w] & (left >= 64 ? ~0ull : ((1ull << left) - 1));
    int64_t o = off[w];
    for (; m; m &= m - 1) out[o++] = (int32_t)(w * 64 + __builtin_ctzll(m));
  }
}
int64_t build_nonsimple_list(const DevGraph& g, const uint64_t* es, int32_t* out) {
  const int64_t nw = (g.ne + 63) / 64;
  if (nw == 0) return 0;
  int32_t* cnt = nullptr;
  int64_t* off = nullptr;
  void* tmp = nullptr;
  size_t tb = 0;
  int64_t total = 0;
  auto chk = [](hipError_t e) { if (e != hipSuccess) throw std::runtime_error(hipGetErrorString(e)); };
  try {
    chk(hipMalloc((void**)&cnt, sizeof(int32_t) * nw));
    chk(hipMalloc((void**)&off, sizeof(int64_t) * (nw + 1)));
    const unsigned grid = (unsigned)std::min<int64_t>((nw + 255) / 256, 16384);
    k_ns_count<<<grid, 256>>>(g.ne, es, cnt);
    chk(hipGetLastError());
    chk(hipcub::DeviceScan::ExclusiveSum(nullptr, tb, cnt, off, (int)nw));
    chk(hipMalloc(&tmp, tb));
    chk(hipcub::DeviceScan::ExclusiveSum(tmp, tb, cnt, off, (int)nw));  // (the total: last offset + count)
    int64_t last_off = 0;
    int32_t last_cnt = 0;
    chk(hipMemcpy(&last_off, off + nw - 1, sizeof(int64_t), hipMemcpyDeviceToHost));
    chk(hipMemcpy(&last_cnt, cnt + nw - 1, sizeof(int32_t), hipMemcpyDeviceToHost));
    total = last_off + last_cnt;
    if (out && total > 0) {
      k_ns_write<<<grid, 256>>>(g.ne, es, off, out);
      chk(hipGetLastError());
    }
    chk(hipDeviceSynchronize());
  } catch (...) {
    (void)hipFree(cnt);
    (void)hipFree(off);
    (void)hipFree(tmp);
    throw;
  }
  (void)hipFree(cnt);
  (void)hipFree(off);
  (void)hipFree(tmp);
  return total;
}

// The loop runs wave-uniform (lane = edge within a 64-edge group) so that profile runs can
// count alive edges per view: the wave's 64 mask words are bit-transposed (lane j <- view j)
// and popcounted; the block sums them in LDS, one atomicAdd per (plane, view) per block.
__device__ __forceinline__ uint64_t transpose64(uint64_t x, int lane);
// SKIP: simple edges (edge_simple) are left unwritten: every reader computes their bits itself.  With
// the non-simple edge list (ens) the lanes walk only those edges: on C4 ~15 % of the edges are not
// simple and spread evenly, so almost every 64-edge group held one and the bitmap skip left most lanes
// idle (edge masks 2.77 ms per launch over 290M edges)
template <bool PLANAR, bool COUNT, bool SKIP>
__global__ __launch_bounds__(256) void k_edge_mask(int64_t ne, const int32_t* __restrict__ esrc,
                                                   const int32_t* __restrict__ edst,
                                                   const int64_t* __restrict__ eoff,
                                                   const int64_t* __restrict__ ekey,
                                                   const int64_t* __restrict__ doff,
                                                   const int64_t* __restrict__ dtime, BatchParams bp,
                                                   uint64_t* __restrict__ em, int64_t estride,
                                                   unsigned long long* __restrict__ ecnt, int64_t h0,
                                                   int64_t own_lim, const uint64_t* __restrict__ vm_ends,
                                                   int64_t vstride, const uint64_t* __restrict__ dbits,
                                                   int32_t* __restrict__ fc, const uint64_t* __restrict__ esimple,
                                                   const int32_t* __restrict__ ens, int64_t n_ens) {
  __shared__ HopLDS L;
  __shared__ unsigned int cnt_s[PLANAR ? kMaxPlanes : 1][64];
  hop_lds_init(L, bp, bp.thr_e);
  constexpr int NP = PLANAR ? kMaxPlanes : 1;
  if (COUNT)
    for (int i = threadIdx.x; i < NP * 64; i += blockDim.x) (&cnt_s[0][0])[i] = 0;
  const int lane = lane_id();
  uint32_t acc[COUNT ? NP : 1] = {};
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const bool list = SKIP && ens != nullptr;
  const int64_t nitems = list ? n_ens : ne;
  for (int64_t e0 = blockIdx.x * (int64_t)blockDim.x + (threadIdx.x & ~63); e0 < nitems; e0 += stride) {
    const int64_t ii = e0 + lane;
    const int64_t e = list ? (ii < n_ens ? (int64_t)ens[ii] : ne) : ii;
    uint64_t m[NP] = {};
    uint64_t mo[NP];  // the edge's own aliveness (the |E_w| counts)
    bool skip = e >= ne;
    if (list) {
      // (every listed edge is non-simple)
    } else if (SKIP && esimple) {  // the group's simple bits (a wave of simple edges costs one 8-B load)
      const uint64_t sw = esimple[e0 >> 6];
      if (sw == ~0ull) continue;
      skip = skip || ((sw >> lane) & 1);
    } else if (SKIP && !skip && edge_simple(eoff[e], eoff[e + 1], ekey, esrc[e], edst[e], doff, dbits)) {
      skip = true;
    }
    EdgeHub hb;
    const bool hub = !skip && edge_bits<PLANAR>(m, L, bp, e, esrc, edst, eoff, ekey, doff, dtime, dbits, fc, hb);
    for (uint64_t hw = __ballot(hub); hw; hw &= hw - 1) {  // hub edges: the whole wave, lane = hop
      const int H = __builtin_ctzll(hw);
      EdgeHub h;
      h.lo = (int64_t)readlane64((uint64_t)hb.lo, H);
      h.f0 = (int64_t)readlane64((uint64_t)hb.f0, H);
      h.f1 = (int64_t)readlane64((uint64_t)hb.f1, H);
      h.s0 = (int64_t)readlane64((uint64_t)hb.s0, H);
      h.s1 = (int64_t)readlane64((uint64_t)hb.s1, H);
      h.d0 = (int64_t)readlane64((uint64_t)hb.d0, H);
      h.d1 = (int64_t)readlane64((uint64_t)hb.d1, H);
      uint64_t mh[NP];
      edge_hub_bits<PLANAR>(mh, L, h, ekey, dtime, lane);
      if (lane == H)
#pragma unroll
        for (int w = 0; w < NP; w++) m[w] = mh[w];
    }
    if (!skip) {
#pragma unroll
      for (int w = 0; w < NP; w++) mo[w] = m[w];
      if (vm_ends) {  // CC: both endpoints' memberships folded in (K2 then skips vm[nb])
        const int32_t s = esrc[e], d = edst[e];
#pragma unroll
        for (int w = 0; w < NP; w++)
          if (!PLANAR || w < L.W) m[w] &= vm_ends[w * vstride + s] & vm_ends[w * vstride + d];
      }
      store_bits<PLANAR>(m, bp, em, estride, e);
    } else {
#pragma unroll
      for (int w = 0; w < NP; w++) mo[w] = 0;
    }
    if constexpr (COUNT) {  // an edge counts once over the partitions: where its source is owned
      const bool mine = e < ne && esrc[e] < own_lim;
#pragma unroll
      for (int w = 0; w < NP; w++)
        if (!PLANAR || w < L.W) acc[w] += __popcll(transpose64(mine ? mo[w] : 0ull, lane));
    }
  }
  if constexpr (COUNT) {
    __syncthreads();  // cnt_s cleared
#pragma unroll
    for (int w = 0; w < NP; w++)
      if (acc[w]) atomicAdd(&cnt_s[w][lane], acc[w]);
    __syncthreads();
    for (int i = threadIdx.x; i < NP * 64; i += blockDim.x) {  // (plane | window, bit) -> view
      const unsigned int x = (&cnt_s[0][0])[i];
      const int w = PLANAR ? i >> 6 : (i & 63) / L.KS, k = PLANAR ? i & 63 : (i & 63) % L.KS;
      if (x && k < L.K && w < L.W) atomicAdd(&ecnt[(h0 + k) * L.W + w], (unsigned long long)x);
    }
  }
}

// Block-wide OR of the views that changed in a step (per-wave values), then one sharded
// atomicOr (kernels.hpp, lanechg).  Call from every thread of the block; `slot` is LDS.
// `lanes` is wave-uniform (a ballot or an OR of ballots); callers that OR straight into the LDS
// word pass 0.
__device__ __forceinline__ void publish_lanes(uint64_t lanes, unsigned long long* slot,
                                              unsigned long long* lanechg, int step) {
  if ((threadIdx.x & 63) == 0 && lanes) atomicOr(slot, (unsigned long long)lanes);
  __syncthreads();
  if (threadIdx.x == 0 && *slot && lanechg)  // result unused: the wave does not wait for it
    atomicOr(&lanechg[step * kLaneShards + (blockIdx.x & (kLaneShards - 1))], *slot);
}

// lanefold[r] = OR of the shards of step r (one wave per step), and the shards cleared for the
// slot's next batch
__global__ __launch_bounds__(256) void k_lane_fold(unsigned long long* __restrict__ lanechg,
                                                   unsigned long long* __restrict__ lanefold) {
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6), lane = lane_id();
  if (r >= kLaneSteps) return;
  unsigned long long x = lanechg[r * kLaneShards + lane];
  if (x) lanechg[r * kLaneShards + lane] = 0;
  for (int o = 32; o > 0; o >>= 1) x |= __shfl_xor(x, o);
  if (lane == 0) lanefold[r] = x;
}
void launch_lane_fold(hipStream_t s, unsigned long long* lanechg, unsigned long long* lanefold) {
  k_lane_fold<<<kLaneSteps / 4, 256, 0, s>>>(lanechg, lanefold);
}

// Per-step work counters, sharded 64 ways so that blocks never pile up on one address (a
// same-address atomic is serialised at the memory side, ~10 ns each: 3k blocks x 3 counters
// on one word cost more than a sparse superstep).  Layout work[(step*64 + shard)*4 + f],
// f = visited vertices, visited slots, changed vertices, gathered labels.  Only written when
// work != nullptr (profile / trace runs).  The halting vote is a plain flag store instead.
// Profile-run work counters, [step][shard][kWorkFields] (rgpu.cpp turns them into bytes):
//   supersteps: 0 visited vertices, 1 their kept slots, 2 changed vertices, 3 label lanes
//   gathered from mixed rows, 4 slots whose (mixed) neighbour's change word was read, 5 own-row 64-B
//   lines read, 6 row lines written, 7 uniform words written;
//   superstep 1 (K2): 0 members, 1 kept slots, 2 changed, 4 static slots scanned, 6, 7 as above.
__device__ __forceinline__ void add_work(unsigned long long* work, int step, const unsigned long long (&f)[8]) {
  if (!work) return;
  unsigned long long* w = work + ((size_t)step * 64 + (blockIdx.x & 63)) * 8;
#pragma unroll
  for (int i = 0; i < 8; i++)
    if (f[i]) atomicAdd(&w[i], f[i]);
}
__device__ __forceinline__ void add_work(unsigned long long* work, int step, unsigned long long a,
                                         unsigned long long b, unsigned long long c,
                                         unsigned long long d = 0) {
  const unsigned long long f[8] = {a, b, c, d, 0, 0, 0, 0};
  add_work(work, step, f);
}
// 64-B lines of a label row holding the lanes of m
__device__ __forceinline__ unsigned row_lines(uint64_t m) {
  return (unsigned)((m & 0xffffull) != 0) + ((m >> 16 & 0xffffull) != 0) + ((m >> 32 & 0xffffull) != 0) +
         ((m >> 48) != 0);
}
// superstep work of one wave (g per lane, the rest wave-uniform)
// DenseRule: superstep r is dense when r >= 2 and step r-1 changed at least nv / div vertices
// (ccount[(r-1)*64 + shard]: changed vertices per step, 64 shards, summed here by each wave;
// every block of a launch computes the same answer from counts the previous launch finished).
// div <= 0: never.  Step 1 (K2) is always dense when the rule is on: with every member sending
// its own id, every member with a kept slot to a smaller label changes and every member next to a
// change is flagged, so step 2 visits the members anyway (C4 trace: step 2 visited as many vertices
// as step 1 in all 15 batches), and K2's random 1-B flag stores per kept slot buy nothing.
__device__ __forceinline__ bool dense_rule(const int32_t* __restrict__ ccount, int r, int64_t nv, int div) {
  if (div <= 0 || !ccount || r < 1) return false;
  if (r == 1) return (div & kDense1) != 0;
  div &= kDense1 - 1;
  int64_t x = ccount[(r - 1) * kCountShards + (threadIdx.x & 63)];
  for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o);
  return x * div >= nv;
}


// Group-cyclic dealing of n items over the waves of a grid-stride loop: items go in groups of G
// consecutive ones (G a power of two, gmax at most, about n / nwaves when that is smaller), group
// g to wave g mod nwaves; in round r lane l takes item l mod G of the wave's group r * 64/G + l / G.
// G consecutive items keep the lanes' first loads in whole cache lines (G = 16 view masks or 32
// chunk flag words = one 128-B line), and dealing the groups cyclically spreads a run of busy items
// (the locality order puts the hubs first) over many waves.  Small graphs get small groups, so
// that every wave has work.
__device__ __forceinline__ int deal_group(int64_t n, int64_t nwaves, int gmax) {
  const int64_t s = (n + nwaves - 1) / nwaves;
  int G = 1;
  while (G < s && G < gmax) G <<= 1;
  return G;
}
__device__ __forceinline__ int64_t dealt_item(int64_t wave, int64_t nwaves, int64_t r, int G, int l) {
  return (wave + (r * (64 / G) + l / G) * nwaves) * G + (l & (G - 1));
}

struct StepWork {
  unsigned long long v = 0, s = 0, g = 0, a = 0, lr = 0, lw = 0, uw = 0;
};
// The work counters of a launch without a work buffer: every update compiles away (the counters
// otherwise hold 14 VGPRs through the superstep kernel)
struct NoCount {
  __device__ NoCount& operator+=(unsigned long long) { return *this; }
};
struct NoWork {
  NoCount v, s, g, a, lr, lw, uw;
};

// ---------------------------------------------------------------- K2: batch CSR (+ superstep 1)
// One wave per vertex.  Static slots of rank v = its out-edges then its in-edges
// (adjacency offset out_off[v] + in_off[v]).  Slot kept iff its view mask
//   em[e] & vm[nbr] & vm[v]  != 0
// i.e. the edge is alive in the view's own window AND both endpoints are in the view's
// (running-min) vertex set — messages to vertices outside the lens are never read
// (WindowLens.getVerticesWithMessages, WindowLens.scala:41-50).  Self-loops only
// message the vertex itself and never change a label: dropped.
//
// Setup (ConnectedComponents.setup :10-17) sends every member's own id, so superstep 1 needs
// no gather: label_1(v) = min(own rank, ranks of kept neighbours) per view.  This kernel
// writes label_0 (= rank) and label_1 rows, the step-1 change words, the step-2 frontier
// bitmap and stepcnt[1]; vadj[v] = OR of v's kept slot masks (v isolated in view j iff bit j
// is clear).

// A kept slot's view bits before the own mask: the edge's window bits (inline for simple slots)
// and the neighbour's membership.  With ebp.simple_ends the nodeath slots skip the neighbour's
// mask: their bits already imply it (BatchParams::simple_ends).
__device__ __forceinline__ uint64_t slot_bits(const HopLDS& L, const BatchParams& ebp, int64_t tsw,
                                              const uint64_t* __restrict__ em, int64_t e,
                                              const uint64_t* __restrict__ vm, int32_t nb) {
  const uint64_t b = ts_simple(tsw) ? simple_bits(L, ebp.sorted, ts_time(tsw)) : em[e];
  return (ebp.simple_ends && ts_nodeath(tsw)) ? b : b & vm[nb];
}

// PROF = false: the work counters compile away (launch_cc_slots: work == null).  IEM: inline edge
// bits (slot_bits; time-ordered slots required), em unused
template <bool PROF, bool IEM, bool PART, int WPE = 1>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WPE))) void k_cc_slots(int64_t nv, int64_t n_own,
                                                  const int64_t* __restrict__ out_off,
                                                  const int64_t* __restrict__ in_off,
                                                  const int32_t* __restrict__ in_eid,
                                                  const int32_t* __restrict__ esrc,
                                                  const int32_t* __restrict__ edst,
                                                  const int32_t* __restrict__ grank,
                                                  const uint64_t* __restrict__ vm,
                                                  const uint64_t* __restrict__ em,
                                                  int32_t* __restrict__ cnt, int32_t* __restrict__ snbr,
                                                  uint64_t* __restrict__ smask,
                                                  uint64_t* __restrict__ vadj,
                                                  int32_t* __restrict__ lab0, int32_t* __restrict__ lab1,
                                                  uint64_t* __restrict__ chg1, uint8_t* __restrict__ act2,
                                                  int32_t* __restrict__ stepflag,
                                                  int32_t* __restrict__ hostflag,
                                                  unsigned long long* __restrict__ work,
                                                  const int32_t* __restrict__ hv_of,
                                                  const int32_t* __restrict__ hv_seg,
                                                  const int32_t* __restrict__ segcnt,
                                                  const uint64_t* __restrict__ segor,
                                                  int32_t* __restrict__ hbest,
                                                  unsigned long long* __restrict__ lanechg,
                                                  const int32_t* __restrict__ ts_e,
                                                  const int32_t* __restrict__ ts_nb,
                                                  const int64_t* __restrict__ ts_t, int64_t tcut,
                                                  int32_t* __restrict__ uw0, int32_t* __restrict__ uw1,
                                                  uint64_t* __restrict__ cb1, int ends,
                                                  int32_t* __restrict__ ccount, int gmax, BatchParams ebp,
                                                  int dense1, const int32_t* __restrict__ ts_g,
                                                  int32_t* __restrict__ mneg, const uint8_t* __restrict__ gpeer,
                                                  uint8_t* __restrict__ pmask, int kopts) {
  __shared__ unsigned long long red[4];
  int32_t wmin = INT32_MAX;  // lane = view: the minimum label of this wave's owned members
  __shared__ HopLDS L;
  if (threadIdx.x < 4) red[threadIdx.x] = 0;
  if constexpr (IEM) hop_lds_init(L, ebp, ebp.thr_e);  // (its barrier also publishes red)
  __syncthreads();
  const int lane = lane_id();
  const int64_t wave = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  using Ctr = std::conditional_t<PROF, unsigned long long, NoCount>;
  Ctr members{}, alive{}, scanned{}, lw{}, uwn{};
  unsigned long long changed = 0;
  uint64_t lanes = 0;  // views with a step-1 change in this wave
  // Vertices are dealt in groups of up to gmax (deal_group; RGPU_DEAL_SLOTS): per round the lanes
  // read 64 vertices' view masks, clear the non-members' count / mask words, and the wave then
  // walks the members one by one.
  const int G = deal_group(nv, nwaves, gmax);
  for (int64_t r = 0; (wave + r * (64 / G) * nwaves) * G < nv; r++) {
   const int64_t vlane = dealt_item(wave, nwaves, r, G, lane);
   const uint64_t mvl = vlane < nv ? vm[vlane] : 0;
   if (vlane < nv && mvl == 0) { cnt[vlane] = 0; vadj[vlane] = 0; }
   // The round's members' offsets, hub flags and (time-ordered) newest slot times, loaded by
   // their lanes at once: the member walk below starts each vertex at its slot loads instead of
   // two dependent trips (offsets, then the cut check) per member.
   int64_t o0l = 0, i0l = 0, tfl = INT64_MAX;
   int32_t noutl = 0, ntotl = 0;
   bool hvl = false;
   if (mvl) {
     o0l = out_off[vlane];
     i0l = in_off[vlane];
     noutl = (int32_t)(out_off[vlane + 1] - o0l);
     ntotl = noutl + (int32_t)(in_off[vlane + 1] - i0l);
     hvl = hv_of && hv_of[vlane] >= 0;
     if (ts_t && ntotl > 0) tfl = ts_time(ts_t[o0l + i0l]);
   }
   const uint64_t heavyl = __ballot(hvl);
   uint64_t todo = __ballot(mvl != 0);
   if (ts_e && ts_t) {
     // Light members (at most 64 static slots, not hubs) are packed into 64-lane passes: lane =
     // slot over the concatenated slot lists of consecutive members, so one round of loads serves
     // every member of the pack instead of one dependent trip per member.  A member whose newest
     // slot predates the cut takes no lanes.
     const int32_t neff = (tfl < tcut) ? 0 : ntotl;
     const int32_t mel = mvl ? (grank ? grank[vlane] : (int32_t)vlane) : 0;
     uint64_t light = todo & ~heavyl & __ballot(ntotl <= 64);
     todo &= ~light;
     // (software-pipelining the packs — the next pack's slot words loaded before this pack's bits,
     // stores and member loop — measured 2.5 % faster than the same build without it, but its
     // registers doubled the spills of the 6-wave hold and that build's K2 was ~10 % slower than
     // without the code: profiles/r06/ab_k2_pipe_c4_rejected.jsonl)
     while (light) {
      uint64_t pack = 0;
      int sum = 0, myL = 0, myj = 0;
      while (light) {
        const int Lp = __builtin_ctzll(light);
        const int n = __builtin_amdgcn_readlane(neff, Lp);
        if (pack && sum + n > 64) break;
        if (lane >= sum && lane < sum + n) { myL = Lp; myj = lane - sum; }
        pack |= 1ull << Lp;
        sum += n;
        light &= light - 1;
      }
      // every lane of the pack: its member, slot and kept views
      const bool on = lane < sum;
      const int64_t vmy = dealt_item(wave, nwaves, r, G, myL);
      const int64_t bmy = (int64_t)__shfl(o0l + i0l, myL);
      const uint64_t mvmy = ((uint64_t)(uint32_t)__shfl((int)(mvl >> 32), myL) << 32) | (uint32_t)__shfl((int)mvl, myL);
      uint64_t m = 0;
      int32_t nb = 0, lb = 0;
      if (on) {
        const int64_t p = bmy + myj;
        const int64_t tsw = ts_t[p];
        nb = ts_nb[p];
        const int32_t e = (IEM && ts_simple(tsw)) ? 0 : ts_e[p];  // (a simple slot's bits need no edge index)
        if (nb != (int32_t)vmy && ts_time(tsw) >= tcut) {
          if constexpr (IEM) {
            m = slot_bits(L, ebp, tsw, em, e, vm, nb) & mvmy;
          } else {
            m = em[e] & (ends ? mvmy : vm[nb]) & mvmy;
          }
        }
        lb = ts_g ? ts_g[p] : (grank ? grank[nb] : nb);
      }
      // partitioned: the peer owning a ghost neighbour across a kept slot (pmask, k_xbc_pack)
      uint32_t pbit = 0u;
      if constexpr (PART) pbit = (m && nb >= (int32_t)n_own) ? (1u << gpeer[nb - n_own]) : 0u;
      const uint64_t bal = __ballot(m != 0);
      if (m) {  // compacted at the member's static offset, in lane order within the member
        const uint64_t below = lanemask_lt() & ~((1ull << (lane - myj)) - 1);
        const int64_t pos = bmy + __popcll(bal & below);
        snbr[pos] = nb;
        smask[pos] = m;
      }
      // Full kept slots (kept on every view of their member: the usual slot of a long window) fold
      // the same label into all of the member's views: a segmented min over the pack (lane = slot,
      // spans of consecutive lanes), read from the span's last lane; the member loop below folds
      // only the other kept slots one by one (as k_cc_step_pk).  Partitioned: the peer bits OR-ed
      // the same way.
      const bool fullk = (kopts & kStepSegMin) && m != 0 && m == mvmy;
      const uint64_t fullb = __ballot(fullk);
      int32_t fmin = fullk ? lb : INT32_MAX;
      if (fullb) {
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
          const int32_t y = __shfl_up(fmin, d);
          if (myj >= d) fmin = min(fmin, y);
        }
      }
      if constexpr (PART) {
        if (__ballot(pbit != 0)) {
#pragma unroll
          for (int d = 1; d < 64; d <<= 1) {
            const uint32_t y = (uint32_t)__shfl_up((int)pbit, d);
            if (myj >= d) pbit |= y;
          }
        }
      }
      // per member of the pack: superstep 1 (lane = view) and its words
      int pre = 0;
      for (uint64_t pk = pack; pk; pk &= pk - 1) {
        const int Lp = __builtin_ctzll(pk);
        const int n = __builtin_amdgcn_readlane(neff, Lp);
        const uint64_t span = n == 0 ? 0ull : ((n >= 64 ? ~0ull : ((1ull << n) - 1)) << pre);
        pre += n;
        const int64_t v = dealt_item(wave, nwaves, r, G, Lp);
        const uint64_t mv = readlane64(mvl, Lp);
        const bool own = v < n_own;
        const int32_t me = __builtin_amdgcn_readlane(mel, Lp);
        if (uw0) {
          if (lane == 0) uw0[v] = me == INT32_MAX ? kMixed : me;
          if (me == INT32_MAX) row_store(lab0 + v * 64, me, line_has(mv, lane), lane);
        } else {
          row_store(lab0 + v * 64, me, line_has(mv, lane), lane);
        }
        if (own && ((mv >> lane) & 1)) wmin = min(wmin, me);
        const uint64_t kept = bal & span;
        const int32_t count = __popcll(kept);
        scanned += (unsigned long long)n;
        int32_t best = me;
        uint64_t any = 0;
        uint32_t pm = 0;
        if (own) {
          const int32_t fL = n == 0 ? INT32_MAX : __builtin_amdgcn_readlane(fmin, pre - 1);
          if (fL != INT32_MAX) {  // (a full slot: labels are never INT32_MAX)
            any = mv;
            if (((mv >> lane) & 1) && fL < best) best = fL;
          }
          if constexpr (PART) pm = n == 0 ? 0u : (uint32_t)__builtin_amdgcn_readlane((int)pbit, pre - 1);
          for (uint64_t b = kept & ~fullb; b; b &= b - 1) {
            const int K = __builtin_ctzll(b);
            const int32_t q = __builtin_amdgcn_readlane(lb, K);
            const uint64_t mK = readlane64(m, K);
            any |= mK;
            if (((mK >> lane) & 1) && q < best) best = q;
          }
        }
        if constexpr (PART)
          if (lane == 0) pmask[v] = (uint8_t)pm;
        if (uw1) {
          const int32_t u = row_uniform(best, mv, lane);
          const bool ch1 = __ballot(best < me) != 0;
          if (lane == 0) uw1[v] = uw_word(u, ch1);
          if (u == kMixed) row_store(lab1 + v * 64, best, line_has(mv, lane), lane);
          uwn += 2;
          if (u == kMixed) lw += row_lines(mv);
        } else {
          row_store(lab1 + v * 64, best, line_has(mv, lane), lane);
          lw += 2 * row_lines(mv);
        }
        const uint64_t ch = __ballot(best < me);
        if (lane == 0) {
          cnt[v] = count;
          vadj[v] = any;
          chg1[v] = ch;
          if (ch && cb1) atomicOr((unsigned long long*)&cb1[v >> 6], 1ull << (v & 63));
        }
        if (!own) continue;
        lanes |= ch;
        if (ch) changed++;
        if (ch && !dense1) {  // (a dense step 1: step 2 visits every member, dense_rule)
          if (lane == 0) act2[v] = 1;
          if (((span >> lane) & 1) && (m & ch)) act2[nb] = 1;
        }
        members += 1;
        alive += (unsigned long long)count;
      }
     }
   }
   while (todo) {
    const int Lm = __builtin_ctzll(todo);
    const int64_t v = dealt_item(wave, nwaves, r, G, Lm);
    const uint64_t mv = readlane64(mvl, Lm);
    todo &= todo - 1;
    const int64_t o0 = (int64_t)readlane64((uint64_t)o0l, Lm), i0 = (int64_t)readlane64((uint64_t)i0l, Lm);
    const int64_t tfirst = (int64_t)readlane64((uint64_t)tfl, Lm);
    if ((heavyl >> Lm) & 1) {
      // heavy vertex: its segments were compacted by k_heavy_slots, which also left the
      // superstep-1 minima of its neighbours' labels in hbest; neighbours of a change are
      // marked by k_heavy_mark.  A heavy ghost (partitioned mode) only needs its kept count and
      // mask OR here: its labels come from its owner.
      const bool own = v < n_own;
      const int32_t h = hv_of[v], me = grank ? grank[v] : (int32_t)v;
      if (own && ((mv >> lane) & 1)) wmin = min(wmin, me);
      const int32_t x = hbest[(int64_t)h * 64 + lane];
      hbest[(int64_t)h * 64 + lane] = INT32_MAX;
      const int32_t best = own ? min(me, x) : me;
      if (own) {
        if (uw0) {  // label_0 = own rank on every member lane: uniform
          const int32_t u = row_uniform(best, mv, lane);
          const bool ch1 = __ballot(best < me) != 0;  // (a ballot of the whole wave, outside lane 0's branch)
          if (lane == 0) { uw0[v] = me == INT32_MAX ? kMixed : me; uw1[v] = uw_word(u, ch1); }
          if (me == INT32_MAX) row_store(lab0 + v * 64, me, line_has(mv, lane), lane);
          if (u == kMixed) row_store(lab1 + v * 64, best, line_has(mv, lane), lane);
        } else {
          row_store(lab0 + v * 64, me, line_has(mv, lane), lane);
          row_store(lab1 + v * 64, best, line_has(mv, lane), lane);
        }
      }
      uint64_t any = 0;
      unsigned long long kept = 0;
      for (int32_t k = hv_seg[h] + lane; k < hv_seg[h + 1]; k += 64) {
        any |= segor[k];
        kept += (unsigned long long)segcnt[k];
      }
      for (int o = 32; o > 0; o >>= 1) {
        any |= __shfl_xor(any, o);
        kept += __shfl_xor(kept, o);
      }
      const uint64_t ch = __ballot(best < me);
      if (lane == 0) {
        if constexpr (PART) pmask[v] = 0xff;  // (a hub: every peer)
        cnt[v] = 0;
        vadj[v] = any;
        chg1[v] = ch;
        if (ch && !dense1) act2[v] = 1;
        if (ch && cb1) atomicOr((unsigned long long*)&cb1[v >> 6], 1ull << (v & 63));
      }
      if (!own) continue;
      changed += ch != 0;
      lanes |= ch;
      members += 1;
      alive += kept;
      continue;
    }
    // label = global rank (== local rank with one partition).  A ghost (v >= n_own) only
    // gets its slots (to its owned neighbours) and label_0 rows here: its label_1 row comes
    // from its owner in the step-1 exchange.
    const bool own = v < n_own;
    const int32_t me = grank ? grank[v] : (int32_t)v;
    if (own && ((mv >> lane) & 1)) wmin = min(wmin, me);
    if (uw0) {
      if (lane == 0) uw0[v] = me == INT32_MAX ? kMixed : me;
      if (me == INT32_MAX) row_store(lab0 + v * 64, me, line_has(mv, lane), lane);
    } else {
      row_store(lab0 + v * 64, me, line_has(mv, lane), lane);
    }
    const int64_t nout = __builtin_amdgcn_readlane(noutl, Lm), ntot = __builtin_amdgcn_readlane(ntotl, Lm),
                  base = o0 + i0;
    int32_t count = 0, best = me;
    uint64_t any = 0;
    uint32_t pm = 0;      // partitioned: peers owning a ghost neighbour across a kept slot
    uint64_t m_keep = 0;  // ntot <= 64: this lane's slot stays in registers for the marking below
    int32_t nb_keep = 0;
    for (int64_t c = 0; c < ntot; c += 64) {
      const int64_t j = c + lane;
      // newest first: the rest are dead in every view (chunk 0: the hoisted time)
      if (ts_t && (c == 0 ? tfirst : ts_time(ts_t[base + c])) < tcut) break;
      scanned += ntot - c < 64 ? ntot - c : 64;
      uint64_t m = 0;
      int32_t nb = 0, lb = 0;
      if (j < ntot) {
        int64_t e;
        const int64_t tsw = ts_t ? ts_t[base + j] : 0;
        if (ts_e) {
          e = (IEM && ts_simple(tsw)) ? 0 : ts_e[base + j];  // (a simple slot's bits need no edge index)
          nb = ts_nb[base + j];
        } else if (j < nout) {
          e = o0 + j;
          nb = edst[e];
        } else {
          e = in_eid[i0 + (j - nout)];
          nb = esrc[e];
        }
        if (nb != (int32_t)v && (!ts_t || ts_time(tsw) >= tcut)) {
          if constexpr (IEM) {
            m = slot_bits(L, ebp, tsw, em, e, vm, nb) & mv;
          } else {
            m = em[e] & (ends ? mv : vm[nb]) & mv;
          }
        }
        lb = ts_g ? ts_g[base + j] : (grank ? grank[nb] : nb);
      }
      uint32_t pbit = 0u;
      if constexpr (PART) pbit = (m && nb >= (int32_t)n_own) ? (1u << gpeer[nb - n_own]) : 0u;
      uint64_t bal = __ballot(m != 0);
      if (m) {
        const int64_t pos = base + count + __popcll(bal & lanemask_lt());
        snbr[pos] = nb;
        smask[pos] = m;
      }
      count += __popcll(bal);
      m_keep = m;
      nb_keep = nb;
      if (!own) continue;
      while (bal) {  // superstep 1: neighbours' labels are their own ranks
        const int L = __builtin_ctzll(bal);
        bal &= bal - 1;
        const int32_t q = __builtin_amdgcn_readlane(lb, L);
        const uint64_t mL = readlane64(m, L);
        if constexpr (PART) pm |= (uint32_t)__builtin_amdgcn_readlane((int)pbit, L);
        any |= mL;
        if (((mL >> lane) & 1) && q < best) best = q;
      }
    }
    if (uw1) {
      const int32_t u = row_uniform(best, mv, lane);
      const bool ch1 = __ballot(best < me) != 0;  // (a ballot of the whole wave, outside lane 0's branch)
      if (lane == 0) uw1[v] = uw_word(u, ch1);
      if (u == kMixed) row_store(lab1 + v * 64, best, line_has(mv, lane), lane);
      uwn += 2;
      if (u == kMixed) lw += row_lines(mv);
    } else {
      row_store(lab1 + v * 64, best, line_has(mv, lane), lane);
      lw += 2 * row_lines(mv);
    }
    const uint64_t ch = __ballot(best < me);
    if (lane == 0) {
      cnt[v] = count;
      vadj[v] = any;
      chg1[v] = ch;
      if constexpr (PART) pmask[v] = (uint8_t)pm;
      if (ch && cb1) atomicOr((unsigned long long*)&cb1[v >> 6], 1ull << (v & 63));
    }
    if (!own) continue;
    lanes |= ch;
    if (ch) {
      changed++;
    }
    if (ch && !dense1) {  // (a dense step 1: step 2 visits every member, dense_rule)
      if (lane == 0) act2[v] = 1;
      if (ntot <= 64) {  // one slot chunk: mark from registers, no re-read of the stored slots
        if (m_keep & ch) act2[nb_keep] = 1;
      } else {
        for (int32_t c = 0; c < count; c += 64) {
          const int32_t j = c + lane;
          if (j < count && (smask[base + j] & ch)) act2[snbr[base + j]] = 1;
        }
      }
    }
    members += 1;
    alive += (unsigned long long)count;
   }
  }
  if (lane == 0) {
    if constexpr (PROF) {
      if (members) atomicAdd(&red[0], members);
      if (alive) atomicAdd(&red[1], alive);
    }
    if (changed) atomicAdd(&red[2], changed);
  }
  if (mneg && wmin != INT32_MAX) atomicMax(&mneg[(blockIdx.x & (kMinShards - 1)) * 64 + lane], INT32_MAX - wmin);
  publish_lanes(lanes, &red[3], lanechg, 1);  // (its barrier also publishes red[0..2])
  if (threadIdx.x == 0) {
    if (red[2] && ccount) atomicAdd(&ccount[1 * kCountShards + (blockIdx.x & (kCountShards - 1))], (int32_t)red[2]);
    if (red[2] && stepflag[1] == 0) {
      stepflag[1] = 1;
      if (hostflag) hostflag[1] = 1;
    }
    add_work(work, 1, red[0], red[1], red[2]);
  }
  if constexpr (PROF) {
    if (work && lane == 0) {  // (uniform per wave)
      const unsigned long long f[8] = {0, 0, 0, 0, scanned, 0, lw, uwn};
      add_work(work, 1, f);
    }
  }
}

// ---------------------------------------------------------------- K3: CC superstep
// Jacobi min-label step for every view of the batch at once: a vertex takes the min of
// its own label and the labels of neighbours whose label improved in the previous step
// (only those sent messages: ConnectedComponents.analyse :19-35, VertexMutliQueue parity
// queues).  step 1 consumes the setup messages (every member "changed").  A step with no
// improvement anywhere ends the job (AnalysisTask.endStep :208-225): later launches exit.
//
// Frontier: step r only visits vertices set in the bitmap act_cur, which step r-1 filled
// with every vertex that changed (so both label buffers catch up) and every neighbour that
// shares a view with the change.  Bitmaps rotate over three buffers; each step zeroes the
// one it will not touch (read two steps ago, written next step).

// Gather the label rows of the neighbours flagged in `act` (lane = slot) and fold them into
// `best` (lane = view); four row loads in flight per round, each touching only the lanes
// (views) in which that neighbour changed (row_load).
// One always-cached 64-B line: lanes whose value will be discarded read it instead of their
// (cold) line of a label row, so a gather only pulls the lines of the views it needs — no
// branch, no descriptor.  Only read, never written.
__device__ int32_t g_dummy_line[16];

template <bool BUF>
__device__ __forceinline__ int32_t row_get(const int32_t* row, bool on, int lane) {
  if (BUF) return row_load(row, on, lane);
  return *(on ? row + lane : g_dummy_line + (lane & 15));  // off lanes: caller's select discards
}

template <bool BUF>
__device__ __forceinline__ int32_t gather_min(uint64_t act, int32_t nb, int32_t best,
                                              const int32_t* __restrict__ lab_cur, int lane) {
  uint64_t bal = __ballot(act != 0);
  while (bal) {
    const int L0 = __builtin_ctzll(bal);
    bal &= bal - 1;
    const int L1 = bal ? __builtin_ctzll(bal) : L0;
    bal &= bal - 1;
    const int L2 = bal ? __builtin_ctzll(bal) : L0;
    bal &= bal - 1;
    const int L3 = bal ? __builtin_ctzll(bal) : L0;
    bal &= bal - 1;
    const int32_t q0 = __builtin_amdgcn_readlane(nb, L0), q1 = __builtin_amdgcn_readlane(nb, L1);
    const int32_t q2 = __builtin_amdgcn_readlane(nb, L2), q3 = __builtin_amdgcn_readlane(nb, L3);
    const bool o0 = (readlane64(act, L0) >> lane) & 1, o1 = (readlane64(act, L1) >> lane) & 1;
    const bool o2 = (readlane64(act, L2) >> lane) & 1, o3 = (readlane64(act, L3) >> lane) & 1;
    const int32_t x0 = row_get<BUF>(lab_cur + (int64_t)q0 * 64, o0, lane);
    const int32_t x1 = row_get<BUF>(lab_cur + (int64_t)q1 * 64, o1, lane);
    const int32_t x2 = row_get<BUF>(lab_cur + (int64_t)q2 * 64, o2, lane);
    const int32_t x3 = row_get<BUF>(lab_cur + (int64_t)q3 * 64, o3, lane);
    const int32_t y0 = o0 ? x0 : INT32_MAX, y1 = o1 ? x1 : INT32_MAX;
    const int32_t y2 = o2 ? x2 : INT32_MAX, y3 = o3 ? x3 : INT32_MAX;
    best = min(best, min(min(y0, y1), min(y2, y3)));
  }
  return best;
}

// lane j: the batch's minimum member label in view j (mneg, kernels.hpp), or INT32_MIN when unknown
__device__ __forceinline__ int32_t final_label(const int32_t* __restrict__ mneg, int lane) {
  if (!mneg) return INT32_MIN;
  int32_t x = 0;
#pragma unroll
  for (int sh = 0; sh < kMinShards; sh++) x = max(x, mneg[sh * 64 + lane]);
  return x ? INT32_MAX - x : INT32_MIN;
}
// wave-uniform call with every lane active (lane j holds view j's mfin): a uniform word u holds the
// final label on every member lane of mv.  A lane whose view has no member in the batch (mfin
// INT32_MIN) is not a member lane of any vertex, so it never votes against.
__device__ __forceinline__ bool holds_final(int32_t u, uint64_t mv, int32_t mfin, int lane) {
  return u != kMixed && __ballot(((mv >> lane) & 1) && (u & 0x7fffffff) != mfin) == 0;
}

// Next-frontier flag of v on the lanes with `want`: a plain byte store (idempotent, no RMW).
__device__ __forceinline__ void mark(bool want, int32_t v, uint8_t* act_next) {
  if (want) act_next[v] = 1;
}

// Per lane: the views whose final label (mfin, lane = view: final_label) equals this lane's label
// x.  The loop runs once per distinct final label of the batch (one for a long window: its views
// share their smallest member), so a wave tests 64 members at once instead of one per ballot.
// Call it with every lane of the wave active (its loop takes one view's label per round from
// the ballot of all lanes; the view itself is always retired, so the loop ends regardless).
__device__ __forceinline__ uint64_t views_with_final(int32_t x, int32_t mfin) {
  uint64_t eq = 0;
  for (uint64_t rest = ~0ull; rest;) {
    const int L = __builtin_ctzll(rest);
    const int32_t d = __builtin_amdgcn_readlane(mfin, L);
    const uint64_t m = __ballot(mfin == d) | (1ull << L);
    rest &= ~m;
    if (x == d) eq |= m;
  }
  return eq;
}

// One CH-vertex chunk of a superstep.  Vertex i (< CH) of the chunk is readlane(vl, i) and
// is taken iff bit i of `bits` is set; every lane holds a valid (padded) vertex for the
// unconditional loads.  The chunk runs loads-first: metadata + own change words + own label
// rows, slot rows, neighbour change words, then every label gather of the chunk, and only
// then the stores (rows, change words, next-frontier flags).  On CDNA stores and atomics
// count in vmcnt, so interleaving them with the next vertex's loads would serialise the
// chunk.  All loads are unconditional from padded buffers (see gather_min).  A visited
// vertex rewrites its row only if it changed now or in the previous step (the only cases
// where the two label buffers differ).  uw_cur / uw_next: uniform label words (null: rows only).
template <int CH, bool BUF, class WK>
__device__ __forceinline__ void cc_chunk(int64_t vl, uint32_t bits, const int64_t* __restrict__ adj_off,
                                         const uint64_t* __restrict__ vm, const int32_t* __restrict__ cnt,
                                         const int32_t* __restrict__ snbr,
                                         const uint64_t* __restrict__ smask,
                                         const int32_t* __restrict__ lab_cur, int32_t* __restrict__ lab_next,
                                         const uint64_t* __restrict__ chg_prev,
                                         uint64_t* __restrict__ chg_next, uint8_t* __restrict__ act_next,
                                         int lane, int32_t& changed,
                                         unsigned long long* __restrict__ lds_lanes,
                                         WK& wk, const int32_t* __restrict__ hv_of = nullptr,
                                         int32_t* __restrict__ hbest = nullptr,
                                         const int32_t* __restrict__ uw_cur = nullptr,
                                         int32_t* __restrict__ uw_next = nullptr,
                                         uint64_t* __restrict__ cb_next = nullptr, bool skip_marks = false,
                                         int32_t mfin = INT32_MIN, bool use_fin = false, bool segmin = false) {
  {
    // stage 1: metadata (lane i -> vertex i of the chunk), own change words, own label rows
    const bool okl = lane < CH && ((bits >> lane) & 1);
    const uint64_t mv_l = okl ? vm[vl] : 0;
    int32_t n_l = okl ? cnt[vl] : 0;  // 0 for a heavy vertex (its slots are in segments)
    const int32_t hh_l = (okl && hv_of) ? hv_of[vl] : -1;
    const int64_t b_l = adj_off[vl];
    const uint64_t cp_l = chg_prev[vl];
    const int32_t u_l = uw_cur ? uw_cur[vl] : kMixed;
    // the vertex's word in the buffer this step writes: a flag left there by a change two steps
    // ago is cleared below when the vertex does not rewrite the word (else every reader of the
    // next step would fold this vertex again)
    const int32_t un_l = uw_next ? uw_next[vl] : kMixed;
    int64_t vv[CH];
    int32_t cur[CH];
    if (use_fin) {  // (wave-uniform) a vertex that holds the final label gathers nothing
#pragma unroll
      for (int i = 0; i < CH; i++) {
        const bool fin = holds_final(__builtin_amdgcn_readlane(u_l, i), readlane64(mv_l, i), mfin, lane);
        if (fin && lane == i) n_l = 0;
      }
    }
#pragma unroll
    for (int i = 0; i < CH; i++) {
      vv[i] = (int64_t)readlane64((uint64_t)vl, i);
      const int32_t u = __builtin_amdgcn_readlane(u_l, i);
      if (u != kMixed) {
        cur[i] = u & 0x7fffffff;  // wave-uniform: no row load
      } else {
        cur[i] = row_get<BUF>(lab_cur + vv[i] * 64, (readlane64(mv_l, i) >> lane) & 1, lane);
        wk.lr += row_lines(readlane64(mv_l, i));
      }
    }
    // stage 2: first 64 kept slots of each vertex (clamped loads, masked by select)
    int32_t nb[CH];
    uint64_t sm[CH];
#pragma unroll
    for (int i = 0; i < CH; i++) {
      const int32_t n = __builtin_amdgcn_readlane(n_l, i);
      const int64_t base = (int64_t)readlane64((uint64_t)b_l, i);
      const int64_t idx = base + (lane < n ? lane : 0);
      const int32_t q = snbr[idx];
      const uint64_t m = smask[idx];
      nb[i] = lane < n ? q : 0;
      sm[i] = lane < n ? m : 0;
    }
    // stage 3: with uniform words, every slot's neighbour word (label + changed flag: one random
    // 4-B load; vertex 0's word for idle lanes, masked by sm = 0), then the change words of the
    // mixed neighbours only (a wave-uniform branch: most chunks have none).  A uniform neighbour
    // that changed is folded on every kept view of the slot (exact: kernels.hpp uw_word).
    // Without uniform words: every neighbour's change word.
    uint64_t act[CH];
    int32_t un[CH];
    if (uw_cur) {
      int32_t w[CH];
#pragma unroll
      for (int i = 0; i < CH; i++) w[i] = uw_cur[nb[i]];  // (unconditional: skipping the loads of slotless
                                                         // vertices with a branch measured 367 vs 347 ms on C4)
      uint64_t mixed = 0;
#pragma unroll
      for (int i = 0; i < CH; i++) {
        act[i] = (w[i] != kMixed && w[i] < 0) ? sm[i] : 0;
        un[i] = w[i] == kMixed ? kMixed : (w[i] & 0x7fffffff);
        mixed |= __ballot(w[i] == kMixed && sm[i] != 0);
      }
      if (mixed) {
        uint64_t cw[CH];
#pragma unroll
        for (int i = 0; i < CH; i++) cw[i] = chg_prev[(w[i] == kMixed && sm[i] != 0) ? nb[i] : 0];
#pragma unroll
        for (int i = 0; i < CH; i++) {
          if (w[i] == kMixed) act[i] = sm[i] & cw[i];
          wk.a += __popcll(__ballot(w[i] == kMixed && sm[i] != 0));  // change words read
        }
      }
    } else {
#pragma unroll
      for (int i = 0; i < CH; i++) {
        act[i] = sm[i] & chg_prev[nb[i]];
        un[i] = kMixed;
      }
    }
#pragma unroll
    for (int i = 0; i < CH; i++) wk.g += un[i] == kMixed ? __popcll(act[i]) : 0;  // lanes gathered from rows (per lane)
    // own rows are only meaningful on member lanes
#pragma unroll
    for (int i = 0; i < CH; i++) cur[i] = ((readlane64(mv_l, i) >> lane) & 1) ? cur[i] : INT32_MAX;
    // stage 4a: all gathers of the chunk (loads only): rows of the mixed neighbours, then the
    // uniform ones' words
    int32_t best[CH];
    uint64_t actr[CH];
#pragma unroll
    for (int i = 0; i < CH; i++) {
      best[i] = cur[i];
      actr[i] = un[i] == kMixed ? act[i] : 0;
    }
#pragma unroll
    for (int i = 0; i < CH; i++) best[i] = gather_min<BUF>(actr[i], nb[i], best[i], lab_cur, lane);
    // full slots (a changed uniform neighbour folded on every view of the vertex): a wave min
    // (lane = slot) over all its chunks, applied once below, instead of a fold lane by lane
    int32_t fmv[CH];
#pragma unroll
    for (int i = 0; i < CH; i++) fmv[i] = INT32_MAX;
    if (uw_cur) {
#pragma unroll
      for (int i = 0; i < CH; i++) {
        const uint64_t mvi = readlane64(mv_l, i);
        const bool full = segmin && un[i] != kMixed && act[i] != 0 && (act[i] & mvi) == mvi;
        if (full) fmv[i] = un[i];
        best[i] = fold_uniform(__ballot(un[i] != kMixed && act[i] != 0 && !full), act[i], un[i], best[i], lane);
      }
    }
#pragma unroll
    for (int i = 0; i < CH; i++) {
      const int32_t n = __builtin_amdgcn_readlane(n_l, i);
      if (n > 64) {  // vertices with more than 64 kept slots (a two-block unrolled round measured
                     // slower on C4: cc_step 263 -> 275 ms serial)
        const int64_t base = (int64_t)readlane64((uint64_t)b_l, i);
        for (int32_t c2 = 64; c2 < n; c2 += 64) {
          const int32_t j = c2 + lane;
          const int64_t idx = base + (j < n ? j : c2);
          const int32_t q = snbr[idx];
          const uint64_t m2 = j < n ? smask[idx] : 0;
          uint64_t a2;
          int32_t u2 = kMixed;
          if (uw_cur) {  // as stage 3
            const int32_t w2 = uw_cur[q];
            a2 = (w2 != kMixed && w2 < 0) ? m2 : 0;
            u2 = w2 == kMixed ? kMixed : (w2 & 0x7fffffff);
            const bool mx = w2 == kMixed && m2 != 0;
            if (__ballot(mx)) {
              const uint64_t c2 = chg_prev[mx ? q : 0];
              if (mx) a2 = m2 & c2;
              wk.a += __popcll(__ballot(mx));
            }
          } else {
            a2 = m2 & chg_prev[q];
          }
          wk.g += u2 == kMixed ? __popcll(a2) : 0;
          best[i] = gather_min<BUF>(u2 == kMixed ? a2 : 0, q, best[i], lab_cur, lane);
          if (uw_cur) {
            const uint64_t mvi = readlane64(mv_l, i);
            const bool full = segmin && u2 != kMixed && a2 != 0 && (a2 & mvi) == mvi;
            if (full) fmv[i] = min(fmv[i], u2);
            best[i] = fold_uniform(__ballot(u2 != kMixed && a2 != 0 && !full), a2, u2, best[i], lane);
          }
        }
      }
    }
    if (segmin) {
#pragma unroll
      for (int i = 0; i < CH; i++) {
        int32_t f = fmv[i];
        for (int o = 32; o > 0; o >>= 1) f = min(f, __shfl_xor(f, o));
        if ((readlane64(mv_l, i) >> lane) & 1) best[i] = min(best[i], f);
      }
    }
    // heavy vertices: the step's minima over their segments (k_heavy_gather); reset for the
    // next step.  Their neighbours are marked by k_heavy_mark.
    if (hv_of) {
#pragma unroll
      for (int i = 0; i < CH; i++) {
        const int32_t h = __builtin_amdgcn_readlane(hh_l, i);
        if (h >= 0) {
          const int32_t x = hbest[(int64_t)h * 64 + lane];
          hbest[(int64_t)h * 64 + lane] = INT32_MAX;
          best[i] = min(best[i], ((readlane64(mv_l, i) >> lane) & 1) ? x : INT32_MAX);
        }
      }
    }
    // stage 4b: publish
    uint64_t cbits = 0;  // (lane 0) changed bits of the chunk: CH consecutive ranks, one bitmap word
#pragma unroll
    for (int i = 0; i < CH; i++) {
      const uint64_t mv = readlane64(mv_l, i);
      if (mv == 0) continue;
      const int64_t v = vv[i];
      const int32_t n = __builtin_amdgcn_readlane(n_l, i);
      wk.v += 1;
      wk.s += (unsigned long long)n;
      const uint64_t ch = __ballot(best[i] < cur[i]);
      if (ch || readlane64(cp_l, i)) {
        const int32_t u = uw_next ? row_uniform(best[i], mv, lane) : kMixed;
        if (uw_next && lane == 0) uw_next[v] = uw_word(u, ch != 0);
        if (uw_next) wk.uw += 1;
        if (u == kMixed) {
          if (BUF) row_store(lab_next + v * 64, best[i], line_has(mv, lane), lane);
          else lab_next[v * 64 + lane] = best[i];
          wk.lw += BUF ? row_lines(mv) : 4;
        }
      } else if (uw_next) {
        const int32_t un = __builtin_amdgcn_readlane(un_l, i);
        if (un != kMixed && un < 0 && lane == 0) uw_next[v] = un & 0x7fffffff;  // stale flag
      }
      if (lane == 0) chg_next[v] = ch;
      if (ch) {
        cbits |= 1ull << (v & 63);
        if (lane == 0) atomicOr(lds_lanes, (unsigned long long)ch);  // LDS: views changed this step
        changed++;
        if (skip_marks) continue;  // dense step: the next step visits every member
        mark(lane == 0, (int32_t)v, act_next);
        mark((sm[i] & ch) != 0, nb[i], act_next);
        if (n > 64) {
          const int64_t base = (int64_t)readlane64((uint64_t)b_l, i);
          for (int32_t c2 = 64; c2 < n; c2 += 64) {
            const int32_t j = c2 + lane;
            const int64_t idx = base + (j < n ? j : c2);
            const int32_t q = snbr[idx];
            mark(j < n && (smask[idx] & ch) != 0, q, act_next);
          }
        }
      }
    }
    if (cb_next && cbits && lane == 0) atomicOr((unsigned long long*)&cb_next[vv[0] >> 6], (unsigned long long)cbits);
  }
}

// Rows of the uniform vertices written out (lane = view, member lines only): after the last
// superstep, for the readers outside the loop (component counts, retained labels).
__global__ __launch_bounds__(256) void k_uw_rows(int64_t nv, const uint64_t* __restrict__ vm,
                                                 const int32_t* __restrict__ uw, int32_t* __restrict__ lab) {
  const int lane = lane_id();
  const int64_t wave = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t b0 = wave * 64; b0 < nv; b0 += nwaves * 64) {
    const int64_t vl = b0 + lane;
    const uint64_t mvl = vl < nv ? vm[vl] : 0;
    const int32_t ul = vl < nv ? uw[vl] : kMixed;
    for (uint64_t todo = __ballot(mvl != 0 && ul != kMixed); todo; todo &= todo - 1) {
      const int L = __builtin_ctzll(todo);
      row_store(lab + (b0 + L) * 64, __builtin_amdgcn_readlane(ul, L) & 0x7fffffff, line_has(readlane64(mvl, L), lane),
                lane);
    }
  }
}

// Superstep kernel (full grid; the packed form).  Step r visits the vertices flagged in act_cur
// (bytes, plain idempotent stores by step r-1) and clears act_clear (read two steps ago, written
// next step).  A wave takes 64 vertices per round (lane = vertex, dealt in
// groups of consecutive ranks): their frontier flags and then the flagged members' metadata (view
// mask, kept-slot count and offset, change word, uniform words, hub index) in one coalesced load
// each.  The kept slots of the members with at most 64 of them are packed into 64-lane passes
// (lane = slot over the concatenated slot lists, as K2 packs its light members): one round of slot
// loads and one of neighbour words per pass serves every member in it, instead of one dependent
// chain per 2-vertex chunk.  The fold then runs per member (lane = view) from registers: uniform
// neighbours' words, and the label rows of mixed neighbours (gather_min).  Every member's new
// uniform word, change word and own frontier flag are stored lane-parallel at the end of the round.
// Members with more than 64 kept slots take the chunk path (cc_chunk) one at a time, before the
// packs (so its registers do not add to the round's).
// (the lean form is held to 6 waves per SIMD, <= 80 VGPRs: at 5 waves the kernel measured 13 %
// slower on C4, profiles/r05/ab_occ_c4.jsonl)
template <bool BUF, bool PROF, bool LONG, int WPE = (PROF || !LONG) ? 1 : 6>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WPE))) void k_cc_step_pk(int step, int64_t nv, const int64_t* __restrict__ adj_off,
                                                    const uint64_t* __restrict__ vm, const int32_t* __restrict__ cnt,
                                                    const int32_t* __restrict__ snbr, const uint64_t* __restrict__ smask,
                                                    const int32_t* __restrict__ lab_cur, int32_t* __restrict__ lab_next,
                                                    const uint64_t* __restrict__ chg_prev, uint64_t* __restrict__ chg_next,
                                                    const uint8_t* __restrict__ act_cur, uint8_t* __restrict__ act_next,
                                                    uint8_t* __restrict__ act_clear, int32_t* __restrict__ stepflag,
                                                    int32_t* __restrict__ hostflag, unsigned long long* __restrict__ work,
                                                    const int32_t* __restrict__ hv_of, int32_t* __restrict__ hbest,
                                                    unsigned long long* __restrict__ lanechg,
                                                    const int32_t* __restrict__ uw_cur, int32_t* __restrict__ uw_next,
                                                    uint64_t* __restrict__ cb_next, uint64_t* __restrict__ cb_clear,
                                                    int64_t cb_words, int32_t* __restrict__ ccount, int dense_div, int gmax,
                                                    const int32_t* __restrict__ mneg, int opts_in) {
  if (stepflag[step - 1] == 0) return;
  // LONG (a batch of long windows, launch_cc_step): the lane-parallel forms (RGPU_STEP_OPTS) are
  // compiled in; the short-window form is the round-4 kernel (its registers stay at 77, no spills)
  const int opts = LONG ? opts_in : 0;
  const int lane = lane_id();
  const bool use_fin = mneg != nullptr && uw_cur != nullptr;
  const int32_t mfin = final_label(mneg, lane);
  const bool skip_marks = dense_rule(ccount, step, nv, dense_div);
  const bool visit_all = dense_rule(ccount, step - 1, nv, dense_div);
  __shared__ int32_t red;
  __shared__ unsigned long long wred[8];  // [0..6] work fields (StepWork), [7] changed views (LDS OR)
  if (threadIdx.x < 8) wred[threadIdx.x] = 0;
  if (threadIdx.x == 0) red = 0;
  // act_clear (the flags step r+2 will write) was last written by step r-2 — by the superstep, the hub
  // mark and the partitioned record apply, all of which write nothing in a dense step (dense_rule) —
  // and cleared by step r-3 before that (step 2: by the batch's first kernel).  So the nv-byte sweep
  // runs only after a step that wrote flags (every launch swept it, 20 MB on C4)
  const bool clear_act = step >= 3 && !dense_rule(ccount, step - 2, nv, dense_div);
  const int64_t nwords = clear_act ? (nv + 7) >> 3 : 0;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < nwords; i += (int64_t)gridDim.x * blockDim.x)
    reinterpret_cast<uint64_t*>(act_clear)[i] = 0;
  if (cb_clear)
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < cb_words; i += (int64_t)gridDim.x * blockDim.x)
      cb_clear[i] = 0;
  __syncthreads();
  const int64_t wave = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  int32_t changed = 0;
  uint64_t lanes_or = 0;
  std::conditional_t<PROF, StepWork, NoWork> wk;
  const int G = deal_group(nv, nwaves, gmax);
  for (int64_t r = 0; (wave + r * (64 / G) * nwaves) * G < nv; r++) {
    const int64_t vl = dealt_item(wave, nwaves, r, G, lane);
    const bool inb = vl < nv;
    uint64_t mv = 0;
    bool flag = false;
    if (inb) {
      if (visit_all) {
        mv = vm[vl];
        flag = mv != 0;
      } else {
        flag = act_cur[vl] != 0;
      }
    }
    uint64_t todo = __ballot(flag);
    if (!todo) continue;
    // the flagged members' metadata in one trip: kept-slot count (0 for a hub: its slots are in
    // segments), view mask, slot offset, change word, uniform words, hub index
    int32_t n = 0, u = kMixed, un = kMixed, hh = -1;
    int64_t base = 0;
    uint64_t cp = 0;
    if (flag) {
      n = cnt[vl];
      if (!visit_all) mv = vm[vl];
      base = adj_off[vl];
      cp = chg_prev[vl];
      if (uw_cur) u = uw_cur[vl];
      if (uw_next) un = uw_next[vl];
      if (hv_of) hh = hv_of[vl];
    }
    flag = flag && mv != 0;  // (a flagged non-member has nothing to do)
    if (use_fin && uw_next && (opts & kStepFinLanes)) {
      // A member that holds its views' final label (uniform, and equal to every member view's
      // final label: views_with_final, lane-parallel) gathers nothing and cannot change.  The
      // non-hubs among them are finished here, lane = member, as the member loop below would
      // finish them: the word rewritten (without the changed flag) if it changed in step r-1 —
      // both label buffers then differ — else a stale changed flag cleared; no change word.
      // (Hubs keep their slot-less visit below: it resets their minima row.)
      const uint64_t eqf = views_with_final(u & 0x7fffffff, mfin);  // (every lane: see its note)
      const bool fin = flag && u != kMixed && hh < 0 && (mv & ~eqf) == 0;
      const uint64_t fz = __ballot(fin);
      if (fz) {
        if (fin) {
          if (cp) uw_next[vl] = u & 0x7fffffff;
          else if (un != kMixed && un < 0) uw_next[vl] = un & 0x7fffffff;
          chg_next[vl] = 0;
        }
        wk.v += __popcll(fz);
        flag = flag && !fin;
      }
    }
    // members with more than 64 kept slots: the chunk path, one vertex at a time
    for (uint64_t big = __ballot(flag && n > 64); big; big &= big - 1) {
      const int L = __builtin_ctzll(big);
      cc_chunk<2, BUF>((int64_t)readlane64((uint64_t)vl, L), 1u, adj_off, vm, cnt, snbr, smask, lab_cur, lab_next,
                       chg_prev, chg_next, act_next, lane, changed, &wred[7], wk, hv_of, hbest, uw_cur, uw_next, cb_next,
                       skip_marks, mfin, use_fin, (opts & kStepSegMin) != 0);
    }
    bool mine = flag && n <= 64;  // this lane's member is handled below
    todo = __ballot(mine);
    if (!todo) continue;
    if (use_fin && !(uw_next && (opts & kStepFinLanes))) {  // (the members' own test, one at a time)
      for (uint64_t t = todo; t; t &= t - 1) {
        const int L = __builtin_ctzll(t);
        const bool fin = holds_final(__builtin_amdgcn_readlane(u, L), readlane64(mv, L), mfin, lane);
        if (fin && lane == L) n = 0;
      }
    }
    // results of the round, lane = member
    uint64_t my_ch = 0;
    int32_t my_w = 0;
    bool has_w = false;
    uint64_t pend = todo;
    // (software-pipelining the packs — the next pack's slot loads issued behind this pack's gather —
    // measured 1.5 % faster than the same build without it, but its registers spilled 32 B more and
    // the build with it was 5 % slower than without the code: profiles/r06/ab_step_pipe_c4_rejected.jsonl)
    while (pend) {
      // the next pack: members in lane order while their slots fit 64 lanes
      uint64_t pack = 0;
      int sum = 0, myL = 0, myj = 0;
      while (pend) {
        const int Lp = __builtin_ctzll(pend);
        const int k = __builtin_amdgcn_readlane(n, Lp);
        if (pack && sum + k > 64) break;
        if (lane >= sum && lane < sum + k) { myL = Lp; myj = lane - sum; }
        pack |= 1ull << Lp;
        sum += k;
        pend &= pend - 1;
      }
      const bool on = lane < sum;
      // lane = slot: the slot, then the neighbour's word (vertex 0's for idle lanes: masked by sm = 0)
      const int64_t bmy = (int64_t)(((uint64_t)(uint32_t)__shfl((int)((uint64_t)base >> 32), myL) << 32) |
                                    (uint32_t)__shfl((int)base, myL));
      const int64_t idx = on ? bmy + myj : 0;
      const int32_t q = snbr[idx];
      const uint64_t m = smask[idx];
      const int32_t nbp = on ? q : 0;
      const uint64_t smp = on ? m : 0;
      // (probing the neighbour's changed bit before its word measured slower twice: DESIGN.md §4c, §4h)
      const uint64_t sma = smp;
      uint64_t act = 0;
      int32_t unp = kMixed;
      if (uw_cur) {
        const int32_t w = uw_cur[nbp];
        act = (w != kMixed && w < 0) ? sma : 0;
        unp = w == kMixed ? kMixed : (w & 0x7fffffff);
        const bool mx = w == kMixed && sma != 0;
        const uint64_t mixed = __ballot(mx);
        if (mixed) {
          const uint64_t cw = chg_prev[mx ? nbp : 0];
          if (mx) act = sma & cw;
          wk.a += __popcll(mixed);
        }
      } else {
        act = sma & chg_prev[nbp];
      }
      wk.g += unp == kMixed ? __popcll(act) : 0;
      // Full slots: a changed uniform neighbour whose fold covers every view of its member (the
      // usual slot of a long window) adds the same label to all of them, so the pack folds those
      // at once, lane = slot: a min over each member's span of lanes (a segmented scan, 6 shuffle
      // rounds), read by the member below from its span's last lane.  The other uniform slots
      // fold view by view (fold_uniform_by_label), the mixed ones from their rows (gather_min).
      bool full = false;
      int32_t fmin = INT32_MAX;
      if (uw_cur && (opts & kStepSegMin)) {
        const uint64_t mvs = ((uint64_t)(uint32_t)__shfl((int)(mv >> 32), myL) << 32) | (uint32_t)__shfl((int)mv, myL);
        full = on && unp != kMixed && act != 0 && (act & mvs) == mvs;
        fmin = full ? unp : INT32_MAX;
        if (__ballot(full)) {
#pragma unroll
          for (int d = 1; d < 64; d <<= 1) {
            const int32_t y = __shfl_up(fmin, d);
            if (myj >= d) fmin = min(fmin, y);
          }
        }
      }
      uint64_t markp = 0;  // lane = slot: its neighbour joins the next frontier
      // lane = member of the pack: the first slot lane of its span (exclusive prefix of the counts)
      const bool inpk = (pack >> lane) & 1;
      const int32_t kin = inpk ? n : 0;
      int32_t prem = kin;
      if (LONG) {
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
          const int32_t y = __shfl_up(prem, d);
          if (lane >= d) prem += y;
        }
      }
      prem -= kin;
      // Simple members (lane = member): uniform, no hub, and every fold in their span full.  Their
      // new label is min(own, span minimum) on all their views, so their whole visit is lane-
      // parallel: the span's minimum and its "any other fold" flag are read from the span's last
      // lane, then the word, change word, changed views and the neighbours' frontier marks follow
      // exactly as the member loop below writes them for any member.
      uint64_t simple = 0;
      if (uw_cur && uw_next && (opts & kStepSegMin) && (opts & kStepSimple)) {
        int32_t bad = (on && act != 0 && !full) ? 1 : 0;  // a fold that is not full
        if (__ballot(bad)) {
#pragma unroll
          for (int d = 1; d < 64; d <<= 1) {
            const int32_t y = __shfl_up(bad, d);
            if (myj >= d) bad |= y;
          }
        }
        const int lastl = kin > 0 ? prem + kin - 1 : 0;
        const int32_t fm = __shfl(fmin, lastl), bd = __shfl(bad, lastl);
        const bool sl = inpk && u != kMixed && hh < 0 && (kin == 0 || bd == 0);
        simple = __ballot(sl);
        if (simple) {
          uint64_t sch = 0;
          if (sl) {
            const int32_t X = u & 0x7fffffff;
            const int32_t nbl = kin > 0 ? min(X, fm) : X;
            if (nbl < X) {
              sch = mv;
              my_w = uw_word(nbl, true);
              has_w = true;
            } else if (cp) {  // both label buffers differ: rewrite the word
              my_w = X;
              has_w = true;
            } else if (un != kMixed && un < 0) {  // stale flag
              my_w = un & 0x7fffffff;
              has_w = true;
            }
            my_ch = sch;
          }
          const uint64_t chb = __ballot(sch != 0);
          if (chb) {
            changed += __popcll(chb);
            uint64_t o = sch;
            for (int d = 32; d > 0; d >>= 1) o |= shfl_xor64(o, d);
            lanes_or |= o;
            const uint64_t chm = ((uint64_t)(uint32_t)__shfl((int)(sch >> 32), myL) << 32) |
                                 (uint32_t)__shfl((int)sch, myL);
            if (on && (smp & chm)) markp = 1;
          }
          wk.v += __popcll(simple);
          if constexpr (PROF) {
            unsigned long long ks = sl ? (unsigned long long)kin : 0ull;
            for (int d = 32; d > 0; d >>= 1) ks += __shfl_xor(ks, d);
            wk.s += ks;
            wk.uw += __popcll(__ballot(sl && (sch != 0 || cp != 0)));
          }
        }
      }
      int pre_run = 0;  // (the short-window form: the running prefix, every pack member in order)
      for (uint64_t pk = pack & ~simple; pk; pk &= pk - 1) {
        const int L = __builtin_ctzll(pk);
        const int k = __builtin_amdgcn_readlane(n, L);
        const int pre = LONG ? __builtin_amdgcn_readlane(prem, L) : pre_run;
        pre_run += k;
        const uint64_t span = k == 0 ? 0ull : ((k >= 64 ? ~0ull : ((1ull << k) - 1)) << pre);
        const int32_t fL = k == 0 ? INT32_MAX : __builtin_amdgcn_readlane(fmin, pre + k - 1);
        const uint64_t mvL = readlane64(mv, L);
        const int64_t v = (int64_t)readlane64((uint64_t)vl, L);
        const int32_t uL = __builtin_amdgcn_readlane(u, L);
        const bool mem = (mvL >> lane) & 1;
        int32_t cur;
        if (uL != kMixed) {
          cur = uL & 0x7fffffff;
        } else {
          cur = row_get<BUF>(lab_cur + v * 64, mem, lane);
          wk.lr += row_lines(mvL);
        }
        cur = mem ? cur : INT32_MAX;
        const bool inspan = (span >> lane) & 1;
        int32_t best = gather_min<BUF>(inspan && unp == kMixed ? act : 0, nbp, cur, lab_cur, lane);
        if (uw_cur) {
          if (mem) best = min(best, fL);
          best = fold_uniform_by_label(__ballot(inspan && unp != kMixed && act != 0 && !full), act, unp, best, lane);
        }
        const int32_t hL = __builtin_amdgcn_readlane(hh, L);
        if (hL >= 0) {  // a hub: the step's minima over its segments (k_heavy_gather), reset for the next step
          const int32_t x = hbest[(int64_t)hL * 64 + lane];
          hbest[(int64_t)hL * 64 + lane] = INT32_MAX;
          best = min(best, mem ? x : INT32_MAX);
        }
        wk.v += 1;
        wk.s += (unsigned long long)k;
        const uint64_t ch = __ballot(best < cur);
        if (ch || readlane64(cp, L)) {  // both label buffers differ: rewrite the word (and row)
          const int32_t uu = uw_next ? row_uniform(best, mvL, lane) : kMixed;
          if (lane == L) { my_w = uw_word(uu, ch != 0); has_w = uw_next != nullptr; }
          if (uw_next) wk.uw += 1;
          if (uu == kMixed) {
            if (BUF) row_store(lab_next + v * 64, best, line_has(mvL, lane), lane);
            else lab_next[v * 64 + lane] = best;
            wk.lw += BUF ? row_lines(mvL) : 4;
          }
        } else if (uw_next) {
          const int32_t unL = __builtin_amdgcn_readlane(un, L);
          if (unL != kMixed && unL < 0 && lane == L) { my_w = unL & 0x7fffffff; has_w = true; }  // stale flag
        }
        if (lane == L) my_ch = ch;
        if (ch) {
          lanes_or |= ch;
          changed++;
          if (inspan && (smp & ch)) markp = 1;
        }
      }
      if (!skip_marks && markp) act_next[nbp] = 1;
    }
    // the round's members, lane-parallel: words, change words, own frontier flags, changed bits
    if (mine) {
      if (has_w) uw_next[vl] = my_w;
      chg_next[vl] = my_ch;
      if (my_ch && !skip_marks) act_next[vl] = 1;
    }
    if (cb_next) {  // a dealt group is G consecutive, G-aligned ranks: one bitmap word, one atomic per group
      const uint64_t cbm = __ballot(mine && my_ch != 0);
      const int gl = lane & ~(G - 1);
      const uint64_t sub = (cbm >> gl) & (G >= 64 ? ~0ull : ((1ull << G) - 1));
      if (lane == gl && sub) atomicOr((unsigned long long*)&cb_next[vl >> 6], (unsigned long long)(sub << (vl & 63)));
    }
  }
  if (lanes_or && lane == 0) atomicOr(&wred[7], (unsigned long long)lanes_or);
  if constexpr (PROF)
    for (int o = 32; o > 0; o >>= 1) wk.g += __shfl_xor(wk.g, o);
  if (lane == 0) {
    if (changed) atomicAdd(&red, changed);
    if constexpr (PROF) {
      const unsigned long long f[7] = {wk.v, wk.s, 0, wk.g, wk.a, wk.lr, wk.lw};
#pragma unroll
      for (int i = 0; i < 7; i++)
        if (f[i]) atomicAdd(&wred[i], f[i]);
      if (wk.uw) atomicAdd(&wred[2], wk.uw);
    }
  }
  publish_lanes(0, &wred[7], lanechg, step);
  if (threadIdx.x == 0) {
    if (red && ccount) atomicAdd(&ccount[step * kCountShards + (blockIdx.x & (kCountShards - 1))], red);
    if (red && stepflag[step] == 0) {
      stepflag[step] = 1;
      if (hostflag) hostflag[step] = 1;
    }
    const unsigned long long f[8] = {wred[0], wred[1], (unsigned long long)red, wred[3], wred[4], wred[5], wred[6],
                                     wred[2]};
    add_work(work, step, f);
  }
}

// ---------------------------------------------------------------- heavy vertices
// Profile runs: the hub kernels' work, for their byte model (rgpu.cpp harvest), in the work
// buffer's step-0 row (supersteps start at 1): [shard][f], f = 0 segments visited by the gather,
// 1 slots it streamed, 2 hot slots (changed neighbour), 3 hot slots of mixed neighbours, 4 label
// lanes gathered from rows, 5 slots walked by the mark, 6 static slots scanned by K2's segment
// pass, 7 slots it kept.  One atomic per wave and field.
__device__ __forceinline__ void heavy_work(unsigned long long* work, int f, unsigned long long x) {
  if (work && x && (threadIdx.x & 63) == 0) atomicAdd(&work[(blockIdx.x & 63) * 8 + f], x);
}
// A power-law hub has 1e5-1e6 slots: as one wave's serial loop it would be the whole
// superstep.  Its static slots are cut into segments of <= kSegSlots, one wave each.  A
// segment's wave loads 64 slots at a time (lane = slot) and then folds the kept / changed ones
// with lane = view, as a normal vertex does (gather_min: the changed neighbours' label rows,
// four coalesced row loads in flight); the segment's minima go to the hub's row in hbest with
// one coalesced atomicMin.  (A lane = slot fold needs a 64-entry array per lane, which the
// compiler demotes to scratch memory: measured 2x slower on C4.)

// K2 for heavy vertices: compact each segment's kept slots (kept iff em[e] & vm[nb] & vm[v])
// at its static position, record its count and mask OR, and fold the superstep-1 minima
// (neighbours' ranks, ConnectedComponents.setup sends own ids) into hbest.
template <bool IEM>
__global__ __launch_bounds__(256) void k_heavy_slots(int64_t nseg, const int32_t* __restrict__ seg_v,
                                                     const int32_t* __restrict__ seg_h,
                                                     const int64_t* __restrict__ seg_lo,
                                                     const int32_t* __restrict__ seg_n,
                                                     const int64_t* __restrict__ out_off,
                                                     const int64_t* __restrict__ in_off,
                                                     const int64_t* __restrict__ adj_off,
                                                     const int32_t* __restrict__ in_eid,
                                                     const int32_t* __restrict__ esrc,
                                                     const int32_t* __restrict__ edst,
                                                     const uint64_t* __restrict__ vm,
                                                     const uint64_t* __restrict__ em,
                                                     int32_t* __restrict__ snbr, uint64_t* __restrict__ smask,
                                                     int32_t* __restrict__ segcnt, uint64_t* __restrict__ segor,
                                                     int32_t* __restrict__ hbest, const int32_t* __restrict__ grank,
                                                     int64_t n_own, const int32_t* __restrict__ ts_e,
                                                     const int32_t* __restrict__ ts_nb,
                                                     const int64_t* __restrict__ ts_t, int64_t tcut, int ends,
                                                     unsigned long long* __restrict__ work, BatchParams ebp,
                                                     const int32_t* __restrict__ ts_g, int kopts) {
  __shared__ HopLDS L;
  if constexpr (IEM) hop_lds_init(L, ebp, ebp.thr_e);
  const int lane = lane_id();
  const int64_t wave = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  unsigned long long w_scan = 0, w_kept = 0;
  for (int64_t sg = wave; sg < nseg; sg += nwaves) {
    const int32_t v = seg_v[sg];
    const int64_t lo0 = seg_lo[sg];
    // a heavy ghost (partitioned) is compacted too: k_heavy_mark walks its kept slots when its
    // owner's records say it changed.  With time-ordered slots a segment whose newest edge
    // predates the batch's cut keeps none.
    const uint64_t mv = !(ts_t && ts_time(ts_t[lo0]) < tcut) ? vm[v] : 0;
    if (mv == 0) {
      if (lane == 0) { segcnt[sg] = 0; segor[sg] = 0; }
      continue;
    }
    const int64_t lo = seg_lo[sg], rel0 = lo - adj_off[v], o0 = out_off[v], i0 = in_off[v];
    const int64_t nout = out_off[v + 1] - o0;
    const int32_t ns = seg_n[sg];
    int32_t best = INT32_MAX;  // lane = view
    int32_t fmin = INT32_MAX;  // lane = slot: the full slots' minimum label
    const bool segmin = (kopts & kStepSegMin) != 0;
    int32_t count = 0;
    uint64_t any = 0;
    for (int32_t c = 0; c < ns; c += 64) {
      const int32_t jj = c + lane;
      if (ts_t && ts_time(ts_t[lo + c]) < tcut) break;
      w_scan += ns - c < 64 ? ns - c : 64;
      uint64_t m = 0;
      int32_t nb = 0;
      if (jj < ns) {
        const int64_t rel = rel0 + jj;
        int64_t e;
        const int64_t tsw = ts_t ? ts_t[lo + jj] : 0;
        if (ts_e) {
          e = (IEM && ts_simple(tsw)) ? 0 : ts_e[lo + jj];  // (as K2)
          nb = ts_nb[lo + jj];
        } else if (rel < nout) {
          e = o0 + rel;
          nb = edst[e];
        } else {
          e = in_eid[i0 + (rel - nout)];
          nb = esrc[e];
        }
        if (nb != v && (!ts_t || ts_time(tsw) >= tcut)) {
          if constexpr (IEM) {
            m = slot_bits(L, ebp, tsw, em, e, vm, nb) & mv;
          } else {
            m = em[e] & (ends ? mv : vm[nb]) & mv;
          }
        }
      }
      const uint64_t bal = __ballot(m != 0);
      if (m) {
        const int64_t pos = lo + count + __popcll(bal & lanemask_lt());
        snbr[pos] = nb;
        smask[pos] = m;
      }
      count += __popcll(bal);
      any |= m;
      const int32_t lb = (grank && m) ? (ts_g ? ts_g[lo + jj] : grank[nb]) : nb;  // setup sends the neighbour's label (id)
      // full slots (kept on every view of the hub): their labels' wave min, folded once below
      const bool fullk = segmin && m != 0 && m == mv;
      if (fullk) fmin = min(fmin, lb);
      for (uint64_t b = bal & ~__ballot(fullk); b; b &= b - 1) {  // lane = view from here: the other kept slots one by one
        const int L = __builtin_ctzll(b);
        const int32_t q = __builtin_amdgcn_readlane(lb, L);
        if ((readlane64(m, L) >> lane) & 1) best = min(best, q);
      }
    }
    if (segmin) {
      for (int o = 32; o > 0; o >>= 1) fmin = min(fmin, __shfl_xor(fmin, o));
      if ((mv >> lane) & 1) best = min(best, fmin);
    }
    for (int o = 32; o > 0; o >>= 1) any |= __shfl_xor(any, o);
    if (lane == 0) { segcnt[sg] = count; segor[sg] = any; }
    w_kept += (unsigned long long)count;
    if (best != INT32_MAX && v < n_own) atomicMin(&hbest[(int64_t)seg_h[sg] * 64 + lane], best);  // (a ghost's
                                                                                             // labels are its owner's)
  }
  heavy_work(work, 6, w_scan);
  heavy_work(work, 7, w_kept);
}

// Hub demotion (kHubDemote; after K2, before the step-1 hub mark): an owned hub whose kept slots in
// this batch fit one pass (<= 64) and sit in one segment (the slots are time-ordered, so usually the
// first) takes the light path for the batch: its kept slots move to its static offset, cnt = their
// count, its segment reports 0 — the hub gather and mark skip it, the superstep packs it with the
// other members and marks its neighbours itself (its `hbest` row stays INT32_MAX: nothing gathers into
// it).  K2 flagged no neighbour of a hub (k_heavy_mark did that after step 1), so a demoted hub that
// changed in step 1 flags its own here when step 1 was not dense.  In short windows most hubs keep a
// few slots, and a hub segment costs a dependent chain per superstep (P = 8 hour batches: ~170 us of
// hub kernels a superstep).  One wave per hub; a separate kernel so that K2's registers stay as they are.
__global__ __launch_bounds__(256) void k_hub_demote(int64_t n_heavy, int64_t n_own, const int32_t* __restrict__ hv_seg,
                                                    const int32_t* __restrict__ seg_v,
                                                    const int64_t* __restrict__ seg_lo,
                                                    const int64_t* __restrict__ adj_off,
                                                    int32_t* __restrict__ segcnt, int32_t* __restrict__ cnt,
                                                    int32_t* __restrict__ snbr, uint64_t* __restrict__ smask,
                                                    const uint64_t* __restrict__ chg1, uint8_t* __restrict__ act2,
                                                    int dense1) {
  const int lane = lane_id();
  const int64_t wave = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t h = wave; h < n_heavy; h += nwaves) {
    const int32_t s0 = hv_seg[h], s1 = hv_seg[h + 1];
    const int32_t v = seg_v[s0];
    if (v >= n_own) continue;  // (a ghost hub's marks come from k_heavy_mark)
    int32_t kept = 0, nzc = 0, nzk = -1;
    for (int32_t k = s0 + lane; k < s1; k += 64) {
      const int32_t c = segcnt[k];
      kept += c;
      if (c > 0) { nzc++; nzk = k; }
    }
    for (int o = 32; o > 0; o >>= 1) {
      kept += __shfl_xor(kept, o);
      nzc += __shfl_xor(nzc, o);
      nzk = max(nzk, __shfl_xor(nzk, o));
    }
    if (kept == 0 || kept > 64 || nzc != 1) continue;
    const int64_t from = seg_lo[nzk], to = adj_off[v];
    const bool in = lane < kept;
    const int32_t q = in ? snbr[from + lane] : 0;
    const uint64_t m = in ? smask[from + lane] : 0;
    if (in && from != to) {
      snbr[to + lane] = q;
      smask[to + lane] = m;
    }
    const uint64_t ch = dense1 ? 0ull : chg1[v];
    if (in && (m & ch)) act2[q] = 1;
    if (lane == 0) {
      cnt[v] = kept;
      segcnt[nzk] = 0;
    }
  }
}

// Superstep r, before the full-grid kernel: minimum over each segment of a flagged heavy
// vertex of the labels of its neighbours that changed in r-1 (views where they did).
template <int WPE>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WPE))) void k_heavy_gather(int step, int64_t nseg, const int32_t* __restrict__ seg_v,
                                                      const int32_t* __restrict__ seg_h,
                                                      const int64_t* __restrict__ seg_lo,
                                                      const int32_t* __restrict__ segcnt,
                                                      const int32_t* __restrict__ snbr,
                                                      const uint64_t* __restrict__ smask,
                                                      const int32_t* __restrict__ lab_cur,
                                                      const uint64_t* __restrict__ chg_prev,
                                                      const uint8_t* __restrict__ act_cur,
                                                      const int32_t* __restrict__ stepflag,
                                                      int32_t* __restrict__ hbest, int64_t n_own,
                                                      const int32_t* __restrict__ uw_cur,
                                                      const uint64_t* __restrict__ cb_prev,
                                                      const int32_t* __restrict__ ccount, int dense_div, int64_t nv_all,
                                                      unsigned long long* __restrict__ work,
                                                      const uint64_t* __restrict__ vm,
                                                      const int32_t* __restrict__ mneg, int pro, int pro_opts) {
  if (stepflag[step - 1] == 0) return;
  const bool use_fin = vm && uw_cur && mneg;
  const int32_t mfin = use_fin ? final_label(mneg, threadIdx.x & 63) : INT32_MIN;
  const bool visit_all = dense_rule(ccount, step - 1, nv_all, dense_div);  // step-1 wrote no flags
  const int lane = lane_id();
  const int64_t wave = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  unsigned long long w_seg = 0, w_slots = 0, w_hot = 0, w_mixed = 0, w_lanes = 0;
  // pro (kHubPro) segments per wave and round, strided over the waves as one segment per wave was: their
  // vertex, flag and kept count load lane-parallel (lane l < pro: segment wave + (r + l)·nwaves),
  // so a late step's idle segments cost one round of loads per pro of them instead of a
  // dependent chain each (the launch is pro times smaller, launch_heavy_gather)
  for (int64_t r0 = 0; wave + r0 * nwaves < nseg; r0 += pro) {
    const int64_t sl = wave + (r0 + lane) * nwaves;
    const bool in = lane < pro && sl < nseg;
    const int32_t vl = in ? seg_v[sl] : 0;
    const int32_t nl = in ? segcnt[sl] : 0;
    // ghosts are not visited (their owner computes them)
    const bool on = in && vl < n_own && nl > 0 && (visit_all || act_cur[vl] != 0);
    // (the final-label test's word and the hub's view mask, loaded with the segments')
    const int32_t ul = (use_fin && on) ? uw_cur[vl] : kMixed;
    const uint64_t ml = on ? vm[vl] : 0;
    for (uint64_t todo = __ballot(on); todo; todo &= todo - 1) {
      const int L = __builtin_ctzll(todo);
      const int64_t sg = wave + (r0 + L) * nwaves;
      const int32_t n = __builtin_amdgcn_readlane(nl, L);
      // its label is final (wave-uniform)
      if (use_fin && holds_final(__builtin_amdgcn_readlane(ul, L), readlane64(ml, L), mfin, lane)) continue;
      if (work) { w_seg++; w_slots += (unsigned long long)n; }
      const int64_t base = seg_lo[sg];
      int32_t best = INT32_MAX;  // lane = view
      if (cb_prev && uw_cur && n <= kSegSlots) {
        // Loads first over the segment's (at most 8) chunks: neighbours, their changed-bit words,
        // then the hot slots' masks and words, then the folds — three dependent trips per segment
        // instead of three per chunk.
        constexpr int NC = kSegSlots / 64;
        int32_t q[NC];
        uint64_t cbw[NC], m[NC];
        int32_t u[NC];
  #pragma unroll
        for (int k = 0; k < NC; k++) q[k] = k * 64 < n ? snbr[base + (k * 64 + lane < n ? k * 64 + lane : k * 64)] : 0;
  #pragma unroll
        for (int k = 0; k < NC; k++) cbw[k] = k * 64 < n ? cb_prev[q[k] >> 6] : 0;
  #pragma unroll
        for (int k = 0; k < NC; k++) {
          const bool hot = k * 64 + lane < n && ((cbw[k] >> (q[k] & 63)) & 1);
          m[k] = hot ? smask[base + k * 64 + lane] : 0;
          u[k] = hot ? uw_label(uw_cur[q[k]]) : kMixed;
        }
        // full slots (a changed uniform neighbour folded on every view of the hub): one wave min
        // over the segment (lane = slot) instead of a fold per distinct label (as k_cc_step_pk)
        const uint64_t mvv = readlane64(ml, L);
        const bool segmin = (pro_opts & kStepSegMin) != 0;
        int32_t fm = INT32_MAX;
  #pragma unroll
        for (int k = 0; k < NC; k++) {
          if (k * 64 >= n) break;
          const uint64_t a = (m[k] && u[k] == kMixed) ? (m[k] & chg_prev[q[k]]) : m[k];
          if (work) {
            w_hot += __popcll(__ballot(a != 0));
            w_mixed += __popcll(__ballot(a != 0 && u[k] == kMixed));
            unsigned long long g = u[k] == kMixed ? (unsigned long long)__popcll(a) : 0ull;
            for (int o = 32; o > 0; o >>= 1) g += __shfl_xor(g, o);
            w_lanes += g;
          }
          const bool fullk = segmin && u[k] != kMixed && a != 0 && (a & mvv) == mvv;
          if (fullk) fm = min(fm, u[k]);
          best = gather_min<false>(u[k] == kMixed ? a : 0, q[k], best, lab_cur, lane);
          best = fold_uniform_by_label(__ballot(u[k] != kMixed && !fullk), a, u[k], best, lane);
        }
        if (segmin) {
          for (int o = 32; o > 0; o >>= 1) fm = min(fm, __shfl_xor(fm, o));
          if ((mvv >> lane) & 1) best = min(best, fm);
        }
        if (best != INT32_MAX) atomicMin(&hbest[(int64_t)seg_h[sg] * 64 + lane], best);
        continue;
      }
      for (int32_t c = 0; c < n; c += 64) {
        const int32_t jj = c + lane;
        const int64_t idx = base + (jj < n ? jj : c);
        const int32_t q = snbr[idx];
        uint64_t a;
        int32_t u;
        if (cb_prev) {  // changed bits: uniform changed neighbours on every kept view (exact);
                        // the slot's mask word is read only for a changed neighbour (the walk streams
                        // the hub's slot list: 4 B instead of 12 B per unchanged neighbour)
          const bool hot = jj < n && ((cb_prev[q >> 6] >> (q & 63)) & 1);
          const uint64_t m = hot ? smask[idx] : 0;
          u = hot ? uw_label(uw_cur[q]) : kMixed;
          a = hot ? (u == kMixed ? m & chg_prev[q] : m) : 0;
        } else {
          a = jj < n ? (smask[idx] & chg_prev[q]) : 0;
          u = (uw_cur && a) ? uw_label(uw_cur[q]) : kMixed;
        }
        // lane = view: the changed mixed rows (4 in flight), then the uniform neighbours' words
        if (work) {
          w_hot += __popcll(__ballot(a != 0));
          w_mixed += __popcll(__ballot(a != 0 && u == kMixed));
          unsigned long long g = u == kMixed ? (unsigned long long)__popcll(a) : 0ull;
          for (int o = 32; o > 0; o >>= 1) g += __shfl_xor(g, o);
          w_lanes += g;
        }
        best = gather_min<false>(u == kMixed ? a : 0, q, best, lab_cur, lane);
        if (uw_cur) best = fold_uniform_by_label(__ballot(u != kMixed), a, u, best, lane);
      }
      if (best != INT32_MAX) atomicMin(&hbest[(int64_t)seg_h[sg] * 64 + lane], best);
    }
  }
  heavy_work(work, 0, w_seg);
  heavy_work(work, 1, w_slots);
  heavy_work(work, 2, w_hot);
  heavy_work(work, 3, w_mixed);
  heavy_work(work, 4, w_lanes);
}

// Superstep r, after the full-grid kernel: the neighbours of every heavy vertex that changed
// in r (and was visited: its change word is current) sharing a changed view join the next
// frontier.  act_cur = nullptr: every member was visited (superstep 1).
__global__ __launch_bounds__(256) void k_heavy_mark(int step, int64_t nseg, const int32_t* __restrict__ seg_v,
                                                    const int64_t* __restrict__ seg_lo,
                                                    const int32_t* __restrict__ segcnt,
                                                    const int32_t* __restrict__ snbr,
                                                    const uint64_t* __restrict__ smask,
                                                    const uint64_t* __restrict__ chg_now,
                                                    const uint8_t* __restrict__ act_cur,
                                                    uint8_t* __restrict__ act_next,
                                                    const int32_t* __restrict__ stepflag, int64_t n_own,
                                                    const int32_t* __restrict__ seg_n,
                                                    const int64_t* __restrict__ out_off,
                                                    const int64_t* __restrict__ in_off,
                                                    const int64_t* __restrict__ adj_off,
                                                    const int32_t* __restrict__ in_eid,
                                                    const int32_t* __restrict__ esrc,
                                                    const int32_t* __restrict__ edst,
                                                    const uint64_t* __restrict__ vm,
                                                    const uint64_t* __restrict__ em,
                                                    const int32_t* __restrict__ ts_e,
                                                    const int32_t* __restrict__ ts_nb,
                                                    const int64_t* __restrict__ ts_t, int64_t tcut,
                                                    const int32_t* __restrict__ ccount, int dense_div, int64_t nv_all,
                                                    unsigned long long* __restrict__ work,
                                                    const int32_t* __restrict__ uw_ghost, int pro) {
  if (stepflag[step] == 0) return;
  if (dense_rule(ccount, step, nv_all, dense_div)) return;  // dense step: the next one visits every member
  if (dense_rule(ccount, step - 1, nv_all, dense_div)) act_cur = nullptr;  // this step visited every member
  const int lane = lane_id();
  const int64_t wave = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  unsigned long long w_walk = 0;
  for (int64_t r0 = 0; wave + r0 * nwaves < nseg; r0 += pro) {  // (the gather's rounds)
    const int64_t sl = wave + (r0 + lane) * nwaves;
    const bool in = lane < pro && sl < nseg;
    const int32_t vl = in ? seg_v[sl] : 0;
    // a ghost's word is current (set by its records)
    bool on = in && !(act_cur && vl < n_own && !act_cur[vl]);
    // a ghost hub's U record sets its uniform word (changed: every view) and no change word
    const int32_t wg = (on && uw_ghost && vl >= n_own) ? uw_ghost[vl] : kMixed;
    const uint64_t chl = on ? ((wg != kMixed && wg < 0) ? ~0ull : chg_now[vl]) : 0ull;
    const int32_t nl = (on && chl) ? segcnt[sl] : 0;
    on = on && chl != 0 && nl > 0;
    for (uint64_t todo = __ballot(on); todo; todo &= todo - 1) {
      const int L = __builtin_ctzll(todo);
      const int64_t sg = wave + (r0 + L) * nwaves;
      const uint64_t ch = readlane64(chl, L);
      const int32_t n = __builtin_amdgcn_readlane(nl, L);
      const int64_t base = seg_lo[sg];
      w_walk += (unsigned long long)n;
      for (int32_t c = 0; c < n; c += 64) {
        const int32_t jj = c + lane;
        if (jj < n && (smask[base + jj] & ch)) act_next[snbr[base + jj]] = 1;
      }
    }
  }
  heavy_work(work, 5, w_walk);
}

// ---------------------------------------------------------------- K5: CC reductions
// Fold the isolated-member shards of view j into the summary (islands: count 1 each) and
// clear them for the next batch.  Called by block (0, j) of a summary kernel.
__device__ __forceinline__ void fold_iso(unsigned int* __restrict__ iso_g, int j,
                                         unsigned long long* __restrict__ stats) {
  if (threadIdx.x >= 64) return;
  unsigned long long k = iso_g[threadIdx.x * 64 + j];
  if (k) iso_g[threadIdx.x * 64 + j] = 0;
  for (int o = 32; o > 0; o >>= 1) k += __shfl_xor(k, o);
  if (threadIdx.x == 0 && k) {
    atomicMax(&stats[0 * 64 + j], 1ull);
    atomicAdd(&stats[1 * 64 + j], k);
    atomicAdd(&stats[4 * 64 + j], k);
  }
}

// ---- component counts from the uniform label words (one partition, kernels.hip kMixed).
// k_cc_count: counts[label][view] (rows of 64, the root's row) += members carrying the label,
// lane = vertex, 64 vertices per wave round.  Uniform members with the same (label, views) are
// one row-wide atomicAdd per group; the wave keeps its most recent group in registers across
// rounds (a giant component costs one atomic per wave, not per 64 vertices).  Mixed members
// add their row's labels lane = view.  Every add goes through a 64-row LDS cache of count rows
// (claimed first come, keyed by label): a giant component's root row takes one global atomic
// per block and view instead of one per member group (month/week batches, where members'
// view sets differ, measured 16-94 ms per batch without it on C4).  Isolated members (no kept
// slot in the view) are islands: counted per view into iso[shard][view] (64 shards).
// k_cc_roots: every root (a member whose label in the view is its own rank and that has a kept
// slot there) reads its count row, folds it into the processBatchWindowResults fields per view
// (ConnectedComponents.scala:137-145) and zeroes it again, so the count rows stay zero between
// batches without a memset; block 0 also folds the island shards.  A batch cut off by maxSteps
// before it converged has labels whose own label is smaller (label of a vertex within
// maxSteps hops): scan_all then reads the count row of every non-isolated member.
__global__ __launch_bounds__(256) void k_cc_count(int64_t nv, uint64_t vmask, const uint64_t* __restrict__ vm,
                                                  const uint64_t* __restrict__ vadj,
                                                  const int32_t* __restrict__ uw,
                                                  const int32_t* __restrict__ lab,
                                                  int32_t* __restrict__ counts, unsigned int* __restrict__ iso_g) {
  constexpr int kRows = 64;
  __shared__ unsigned int iso[64];
  __shared__ int32_t ckey[kRows];
  __shared__ unsigned int crow[kRows][64];
  if (threadIdx.x < 64) iso[threadIdx.x] = 0;
  if (threadIdx.x < kRows) ckey[threadIdx.x] = -1;
  for (int i = threadIdx.x; i < kRows * 64; i += blockDim.x) (&crow[0][0])[i] = 0;
  __syncthreads();
  auto add = [&](int32_t x, int j, unsigned int c) {  // counts[x][j] += c
    const int h0 = (int)(((uint32_t)x * 2654435761u) >> 26);
    for (int p = 0; p < 4; p++) {  // four probes, then the global row
      const int h = (h0 + p) & (kRows - 1);
      int32_t k = ckey[h];
      if (k == -1) {
        k = atomicCAS(&ckey[h], -1, x);
        if (k == -1) k = x;
      }
      if (k == x) {
        atomicAdd(&crow[h][j], c);
        return;
      }
    }
    atomicAdd(&counts[(int64_t)x * 64 + j], (int32_t)c);
  };
  const int lane = lane_id();
  const int64_t wave = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  unsigned int iso_acc = 0;              // lane = view
  int32_t sx = -1;                       // the wave's pending group: label, views, members
  uint64_t sm = 0;
  int32_t sc = 0;
  for (int64_t b0 = wave * 64; b0 < nv; b0 += nwaves * 64) {
    const int64_t v = b0 + lane;
    const uint64_t mv = v < nv ? vm[v] & vmask : 0;
    const uint64_t ad = v < nv ? vadj[v] : 0;
    const int32_t x = v < nv ? uw_label(uw[v]) : kMixed;
    iso_acc += (unsigned)__popcll(transpose64(mv & ~ad, lane));
    const uint64_t m = mv & ad;
    uint64_t todo = __ballot(m != 0 && x != kMixed);
    while (todo) {
      const int L = __builtin_ctzll(todo);
      const int32_t xL = __builtin_amdgcn_readlane(x, L);
      const uint64_t mL = readlane64(m, L);
      const uint64_t same = __ballot(((todo >> lane) & 1) && x == xL && m == mL);
      todo &= ~same;
      if (xL == sx && mL == sm) {
        sc += __popcll(same);
      } else {
        if (sc && ((sm >> lane) & 1)) add(sx, lane, (unsigned)sc);
        sx = xL;
        sm = mL;
        sc = __popcll(same);
      }
    }
    for (uint64_t mixed = __ballot(m != 0 && x == kMixed); mixed; mixed &= mixed - 1) {
      const int L = __builtin_ctzll(mixed);
      const uint64_t mL = readlane64(m, L);
      if ((mL >> lane) & 1) add(lab[(b0 + L) * 64 + lane], lane, 1u);
    }
  }
  if (sc && ((sm >> lane) & 1)) add(sx, lane, (unsigned)sc);
  if (iso_acc) atomicAdd(&iso[lane], iso_acc);
  __syncthreads();
  for (int i = threadIdx.x; i < kRows * 64; i += blockDim.x) {
    const unsigned int c = (&crow[0][0])[i];
    if (c) atomicAdd(&counts[(int64_t)ckey[i >> 6] * 64 + (i & 63)], (int32_t)c);
  }
  if (threadIdx.x < 64 && iso[threadIdx.x])
    atomicAdd(&iso_g[(blockIdx.x & 63) * 64 + threadIdx.x], iso[threadIdx.x]);
}

__global__ __launch_bounds__(256) void k_cc_roots(int64_t nv, uint64_t vmask, const uint64_t* __restrict__ vm,
                                                  const uint64_t* __restrict__ vadj,
                                                  const int32_t* __restrict__ uw,
                                                  const int32_t* __restrict__ lab, int32_t* __restrict__ counts,
                                                  unsigned long long* __restrict__ stats,
                                                  unsigned int* __restrict__ iso_g, int scan_all,
                                                  const int32_t* __restrict__ grank, int rows_by_rank) {
  __shared__ unsigned long long red[6][64];
  for (int i = threadIdx.x; i < 6 * 64; i += blockDim.x) (&red[0][0])[i] = 0;
  __syncthreads();
  if (blockIdx.x == 0 && threadIdx.x < 64) {  // islands: count 1 each
    const int j = threadIdx.x;
    unsigned long long k = 0;
    for (int sh = 0; sh < 64; sh++) {
      const unsigned int x = iso_g[sh * 64 + j];
      if (x) { k += x; iso_g[sh * 64 + j] = 0; }
    }
    if (k) {
      atomicMax(&stats[0 * 64 + j], 1ull);
      atomicAdd(&stats[1 * 64 + j], k);
      atomicAdd(&stats[4 * 64 + j], k);
    }
  }
  const int lane = lane_id();
  const int64_t wave = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  unsigned long long big = 0, tot = 0, nis = 0, gt2 = 0, sum = 0, snis = 0;  // lane = view
  for (int64_t b0 = wave * 64; b0 < nv; b0 += nwaves * 64) {
    const int64_t v = b0 + lane;
    const uint64_t m = v < nv ? vm[v] & vmask & vadj[v] : 0;
    const int32_t x = (v < nv && uw) ? uw_label(uw[v]) : kMixed;
    const int32_t me = v < nv ? (grank ? grank[v] : (int32_t)v) : -2;  // the vertex's own label
    for (uint64_t cand = __ballot(m != 0 && (scan_all || x == me || x == kMixed)); cand; cand &= cand - 1) {
      const int L = __builtin_ctzll(cand);
      const int32_t meL = __builtin_amdgcn_readlane(me, L);
      const int64_t r = rows_by_rank ? b0 + L : (int64_t)meL;  // its count row
      const uint64_t mL = readlane64(m, L);
      const bool in = (mL >> lane) & 1;
      const bool root = scan_all || __builtin_amdgcn_readlane(x, L) != kMixed ? in
                                                                            : (in && lab[(b0 + L) * 64 + lane] == meL);
      const int32_t c = root ? counts[r * 64 + lane] : 0;
      if (c) {
        counts[r * 64 + lane] = 0;
        const unsigned long long uc = (unsigned long long)c;
        big = uc > big ? uc : big;
        tot += 1;
        nis += c > 1;
        gt2 += c > 2;
        sum += uc;
        snis += c > 1 ? uc : 0;
      }
    }
  }
  if (tot) {
    atomicMax(&red[0][lane], big);
    atomicAdd(&red[1][lane], tot);
    atomicAdd(&red[2][lane], nis);
    atomicAdd(&red[3][lane], gt2);
    atomicAdd(&red[4][lane], sum);
    atomicAdd(&red[5][lane], snis);
  }
  __syncthreads();
  if (threadIdx.x < 64) {
    const int j = threadIdx.x;
    if (red[1][j]) {
      atomicMax(&stats[0 * 64 + j], red[0][j]);
      atomicAdd(&stats[1 * 64 + j], red[1][j]);
      atomicAdd(&stats[2 * 64 + j], red[2][j]);
      atomicAdd(&stats[3 * 64 + j], red[3][j]);
      atomicAdd(&stats[4 * 64 + j], red[4][j]);
      atomicAdd(&stats[5 * 64 + j], red[5][j]);
    }
  }
}

// ---------------------------------------------------------------- degree
// DegreeBasic.returnResults (DegreeBasic.scala:16-28) for every view: out = alive
// out-edges incl. a self-loop, in = alive in-edges (a self-loop never enters
// incomingEdges, EntityStorage.scala:257), edges filtered by their own history only
// (Vertex.viewAtWithWindow).  Per-vertex rows are written to outdeg/indeg; per-view
// totals (V, sum out, sum in) into stats[f*64 + view].
// 64x64 bit-matrix transpose across the wave: lane r holds row r (bit c = column c) and gets
// column r back (bit s = row s).  Six butterfly levels of 64-bit shuffles.
__device__ __forceinline__ uint64_t transpose64(uint64_t x, int lane) {
  const uint64_t M[6] = {0x00000000FFFFFFFFull, 0x0000FFFF0000FFFFull, 0x00FF00FF00FF00FFull,
                         0x0F0F0F0F0F0F0F0Full, 0x3333333333333333ull, 0x5555555555555555ull};
#pragma unroll
  for (int k = 0; k < 6; k++) {
    const int d = 32 >> k;
    const uint64_t y = shfl_xor64(x, d);
    x = (lane & d) ? ((x & ~M[k]) | ((y & ~M[k]) >> d)) : ((x & M[k]) | ((y & M[k]) << d));
  }
  return x;
}

// DegreeRanking / DegreeBasic top-20 (DegreeRanking.scala:14-26, DegreeBasic.scala:16-28): per view
// the 20 members with the largest in-degree, ties by ascending id (the reference's ParTrieMap order
// is unordered).  A candidate is key = in-degree << 32 | ~label (labels are order-preserving with
// ids), so a larger key wins; 0 = none.  TOP: k_degree keeps every lane's (view's) best 20 in
// registers over the vertices its wave scans and writes them out ([wave][view][kTop], sorted);
// k_deg_top_merge (one block per view) merges the waves' lists and the heavy vertices (their
// in-degrees are completed by k_heavy_degree after k_degree).
template <int N>
__device__ __forceinline__ void top_insert(uint64_t (&tk)[N], int32_t (&tp)[N], uint64_t x, int32_t xp) {
  if (x <= tk[N - 1]) return;
#pragma unroll
  for (int i = 0; i < N; i++)
    if (x > tk[i]) {
      const uint64_t a = tk[i];
      const int32_t b = tp[i];
      tk[i] = x;
      tp[i] = xp;
      x = a;
      xp = b;
    }
}

template <bool TOP>
__global__ __launch_bounds__(256) void k_degree(int64_t nv, const int64_t* __restrict__ out_off,
                                                const int64_t* __restrict__ in_off,
                                                const int32_t* __restrict__ in_eid,
                                                const uint64_t* __restrict__ vm,
                                                const uint64_t* __restrict__ em,
                                                int32_t* __restrict__ outdeg,
                                                int32_t* __restrict__ indeg,
                                                unsigned long long* __restrict__ stats,
                                                const int32_t* __restrict__ hv_of,
                                                const int32_t* __restrict__ grank,
                                                uint64_t* __restrict__ cand_key, int32_t* __restrict__ cand_pos) {
  uint64_t tk[TOP ? kTop : 1];
  int32_t tp[TOP ? kTop : 1];
#pragma unroll
  for (int i = 0; i < (TOP ? kTop : 1); i++) { tk[i] = 0; tp[i] = -1; }
  __shared__ unsigned long long red[3][64];
  for (int i = threadIdx.x; i < 3 * 64; i += blockDim.x) (&red[0][0])[i] = 0;
  __syncthreads();
  const int lane = lane_id();
  const int64_t wave = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  unsigned long long tv = 0, to = 0, ti = 0;
  for (int64_t v = wave; v < nv; v += nwaves) {
    const uint64_t mv = vm[v];
    int32_t od = 0, id = 0;
    if (mv) {
      const int64_t o0 = out_off[v], o1 = out_off[v + 1], i0 = in_off[v], i1 = in_off[v + 1];
      const bool heavy = hv_of && hv_of[v] >= 0;  // counted by k_heavy_degree (rows start at 0)
      for (int dir = 0; dir < 2 && !heavy; dir++) {
        const int64_t n = dir ? i1 - i0 : o1 - o0;
        int32_t acc = 0;
        for (int64_t c = 0; c < n; c += 64) {  // lane = edge -> transpose -> lane = view
          const int64_t j = c + lane;
          uint64_t m = 0;
          if (j < n) m = em[dir ? in_eid[i0 + j] : o0 + j];
          acc += __popcll(transpose64(m, lane));
        }
        if (dir) id = acc; else od = acc;
      }
      const int in_view = (int)((mv >> lane) & 1);
      od = in_view ? od : 0;
      id = in_view ? id : 0;
      tv += in_view;
      to += od;
      ti += id;
      if constexpr (TOP) {
        if (in_view && !(hv_of && hv_of[v] >= 0)) {  // (heavy vertices: k_deg_top_merge)
          const uint32_t lb = grank ? (uint32_t)grank[v] : (uint32_t)v;
          top_insert(tk, tp, ((uint64_t)(uint32_t)id << 32) | (uint32_t)~lb, (int32_t)v);
        }
      }
    }
    outdeg[v * 64 + lane] = od;
    indeg[v * 64 + lane] = id;
  }
  if constexpr (TOP) {
#pragma unroll
    for (int i = 0; i < kTop; i++) {
      cand_key[(wave * 64 + lane) * kTop + i] = tk[i];
      cand_pos[(wave * 64 + lane) * kTop + i] = tp[i];
    }
  }
  atomicAdd(&red[0][lane], tv);
  atomicAdd(&red[1][lane], to);
  atomicAdd(&red[2][lane], ti);
  __syncthreads();
  if (threadIdx.x < 64)
    for (int f = 0; f < 3; f++)
      if (red[f][threadIdx.x]) atomicAdd(&stats[f * 64 + threadIdx.x], red[f][threadIdx.x]);
}

// Degree of heavy vertices: per segment, alive out- / in-slots counted per view (lane = slot ->
// bit transpose -> lane = view), added to the hub's rows and the view totals.
__global__ __launch_bounds__(256) void k_heavy_degree(int64_t nseg, const int32_t* __restrict__ seg_v,
                                                      const int64_t* __restrict__ seg_lo,
                                                      const int32_t* __restrict__ seg_n,
                                                      const int64_t* __restrict__ out_off,
                                                      const int64_t* __restrict__ in_off,
                                                      const int64_t* __restrict__ adj_off,
                                                      const int32_t* __restrict__ in_eid,
                                                      const uint64_t* __restrict__ vm,
                                                      const uint64_t* __restrict__ em,
                                                      int32_t* __restrict__ outdeg, int32_t* __restrict__ indeg,
                                                      unsigned long long* __restrict__ stats, int64_t n_own) {
  const int lane = lane_id();
  const int64_t wave = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t sg = wave; sg < nseg; sg += nwaves) {
    const int32_t v = seg_v[sg];
    if (v >= n_own) continue;  // a heavy ghost: its owner counts it
    const uint64_t mv = vm[v];
    if (mv == 0) continue;
    const int64_t rel0 = seg_lo[sg] - adj_off[v], o0 = out_off[v], i0 = in_off[v];
    const int64_t nout = out_off[v + 1] - o0;
    const int32_t ns = seg_n[sg];
    int32_t co = 0, ci = 0;
    for (int32_t c = 0; c < ns; c += 64) {
      const int32_t jj = c + lane;
      uint64_t mo = 0, mi = 0;
      if (jj < ns) {
        const int64_t rel = rel0 + jj;
        if (rel < nout) mo = em[o0 + rel];
        else mi = em[in_eid[i0 + (rel - nout)]];
      }
      co += __popcll(transpose64(mo, lane));
      ci += __popcll(transpose64(mi, lane));
    }
    const bool in_view = (mv >> lane) & 1;
    if (in_view && co) {
      atomicAdd(&outdeg[(int64_t)v * 64 + lane], co);
      atomicAdd(&stats[1 * 64 + lane], (unsigned long long)co);
    }
    if (in_view && ci) {
      atomicAdd(&indeg[(int64_t)v * 64 + lane], ci);
      atomicAdd(&stats[2 * 64 + lane], (unsigned long long)ci);
    }
  }
}

// One block per view: the waves' candidate lists and the heavy vertices -> the view's top 20
// (key, local rank, out-degree); keys of 0 pad a short list.
__global__ __launch_bounds__(256) void k_deg_top_merge(int64_t ncand_waves, const uint64_t* __restrict__ cand_key,
                                                       const int32_t* __restrict__ cand_pos, int64_t n_heavy,
                                                       const int32_t* __restrict__ hv_seg,
                                                       const int32_t* __restrict__ seg_v, int64_t n_own,
                                                       const uint64_t* __restrict__ vm,
                                                       const int32_t* __restrict__ indeg,
                                                       const int32_t* __restrict__ outdeg,
                                                       const int32_t* __restrict__ grank,
                                                       unsigned long long* __restrict__ top_key,
                                                       int32_t* __restrict__ top_pos, int32_t* __restrict__ top_out) {
  const int j = blockIdx.x;
  uint64_t tk[kTop];
  int32_t tp[kTop];
#pragma unroll
  for (int i = 0; i < kTop; i++) { tk[i] = 0; tp[i] = -1; }
  for (int64_t w = threadIdx.x; w < ncand_waves; w += blockDim.x) {
    const int64_t b = (w * 64 + j) * kTop;
    for (int i = 0; i < kTop; i++) {
      const uint64_t x = cand_key[b + i];
      if (x <= tk[kTop - 1]) break;  // each list is sorted, descending
      top_insert(tk, tp, x, cand_pos[b + i]);
    }
  }
  for (int64_t h = threadIdx.x; h < n_heavy; h += blockDim.x) {
    const int32_t v = seg_v[hv_seg[h]];
    if (v >= n_own || !((vm[v] >> j) & 1)) continue;  // (a heavy ghost is its owner's)
    const uint32_t lb = grank ? (uint32_t)grank[v] : (uint32_t)v;
    top_insert(tk, tp, ((uint64_t)(uint32_t)indeg[(int64_t)v * 64 + j] << 32) | (uint32_t)~lb, v);
  }
  // 20 rounds of a block-wide maximum over the threads' heads (keys are distinct)
  __shared__ unsigned long long wbest[4];
  __shared__ unsigned long long best;
  const int lane = lane_id(), wid = threadIdx.x >> 6;
  for (int r = 0; r < kTop; r++) {
    unsigned long long x = tk[0];
    for (int o = 32; o > 0; o >>= 1) {
      const unsigned long long y = shfl_xor64(x, o);
      x = y > x ? y : x;
    }
    if (lane == 0) wbest[wid] = x;
    __syncthreads();
    if (threadIdx.x == 0) {
      unsigned long long m = wbest[0];
      for (int k = 1; k < (int)(blockDim.x >> 6); k++) m = wbest[k] > m ? wbest[k] : m;
      best = m;
    }
    __syncthreads();
    const unsigned long long m = best;
    if (m != 0 && tk[0] == m) {  // the winner pops its head
      top_key[j * kTop + r] = m;
      top_pos[j * kTop + r] = tp[0];
      top_out[j * kTop + r] = outdeg[(int64_t)tp[0] * 64 + j];
#pragma unroll
      for (int i = 0; i < kTop - 1; i++) { tk[i] = tk[i + 1]; tp[i] = tp[i + 1]; }
      tk[kTop - 1] = 0;
      tp[kTop - 1] = -1;
    } else if (m == 0 && threadIdx.x == 0) {
      top_key[j * kTop + r] = 0;
      top_pos[j * kTop + r] = -1;
      top_out[j * kTop + r] = 0;
    }
    __syncthreads();
  }
}

// PageRank pull for heavy vertices: per segment, the alive in-slots' contributions (views in
// em[e] & vm[src] & vm[v]) summed per view, four neighbour rows in flight, then added to the
// hub's fp64 accumulator row (k_pr_step adds it and resets it).  fp64 atomics make the sum
// order vary between runs: within the spec's L1 <= 1e-6 (App. A.5), not bit-stable.
__global__ __launch_bounds__(256) void k_heavy_pr(int64_t nseg, const int32_t* __restrict__ seg_v,
                                                  const int32_t* __restrict__ seg_h,
                                                  const int64_t* __restrict__ seg_lo,
                                                  const int32_t* __restrict__ seg_n,
                                                  const int64_t* __restrict__ out_off,
                                                  const int64_t* __restrict__ in_off,
                                                  const int64_t* __restrict__ adj_off,
                                                  const int32_t* __restrict__ in_eid,
                                                  const int32_t* __restrict__ esrc,
                                                  const uint64_t* __restrict__ vm,
                                                  const uint64_t* __restrict__ em,
                                                  const double* __restrict__ contrib_cur,
                                                  double* __restrict__ hacc, int64_t n_own) {
  const int lane = lane_id();
  const int64_t wave = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t sg = wave; sg < nseg; sg += nwaves) {
    const int32_t v = seg_v[sg];
    if (v >= n_own) continue;  // a heavy ghost: its owner pulls it
    const uint64_t mv = vm[v];
    if (mv == 0) continue;
    const int64_t rel0 = seg_lo[sg] - adj_off[v], i0 = in_off[v];
    const int64_t nout = out_off[v + 1] - out_off[v];
    const int32_t ns = seg_n[sg];
    if (rel0 + ns <= nout) continue;  // out-slots only
    double acc = 0.0;
    for (int32_t c = 0; c < ns; c += 64) {
      const int64_t rel = rel0 + c + lane;
      uint64_t m = 0;
      int32_t nb = 0;
      if (c + lane < ns && rel >= nout) {
        const int32_t e = in_eid[i0 + (rel - nout)];
        nb = esrc[e];
        m = em[e] & vm[nb] & mv;
      }
      uint64_t bal = __ballot(m != 0);
      while (bal) {
        int L[4];
#pragma unroll
        for (int u = 0; u < 4; u++) {
          L[u] = bal ? __builtin_ctzll(bal) : -1;
          if (bal) bal &= bal - 1;
        }
        double x[4];
#pragma unroll
        for (int u = 0; u < 4; u++) {
          const int Lu = L[u] < 0 ? L[0] : L[u];
          const int32_t q = __builtin_amdgcn_readlane(nb, Lu);
          const bool on = L[u] >= 0 && ((readlane64(m, Lu) >> lane) & 1);
          x[u] = on ? contrib_cur[(int64_t)q * 64 + lane] : 0.0;
        }
        acc += (x[0] + x[1]) + (x[2] + x[3]);
      }
    }
    if (acc != 0.0) atomicAdd(&hacc[(int64_t)seg_h[sg] * 64 + lane], acc);
  }
}

// ---------------------------------------------------------------- PageRank (App. A.5)
// Pull slots of rank v = its in-edges plus its self-loop (messageAllOutgoingNeighbors
// reaches the vertex itself); kept iff em[e] & vm[src] & vm[v] != 0.  Static capacity
// in-degree + 1 at offset in_off[v] + v.  Initialises PR0 = 1 and contrib = 1/max(od,1).
__global__ __launch_bounds__(256) void k_pr_slots(int64_t nv, const int64_t* __restrict__ out_off,
                                                  const int64_t* __restrict__ in_off,
                                                  const int32_t* __restrict__ in_eid,
                                                  const int32_t* __restrict__ esrc,
                                                  const int32_t* __restrict__ edst,
                                                  const uint64_t* __restrict__ vm,
                                                  const uint64_t* __restrict__ em,
                                                  const int32_t* __restrict__ outdeg,
                                                  int32_t* __restrict__ cnt, int32_t* __restrict__ snbr,
                                                  uint64_t* __restrict__ smask,
                                                  double* __restrict__ pr,
                                                  double* __restrict__ contrib,
                                                  const int32_t* __restrict__ hv_of) {
  const int lane = lane_id();
  const int64_t wave = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t v = wave; v < nv; v += nwaves) {
    const int32_t od = outdeg[v * 64 + lane];
    pr[v * 64 + lane] = 1.0;  // defaultPR, PageRank.scala:14
    contrib[v * 64 + lane] = 1.0 / (double)(od > 1 ? od : 1);
    const uint64_t mv = vm[v];
    if (mv == 0) {
      if (lane == 0) cnt[v] = 0;
      continue;
    }
    const int64_t i0 = in_off[v], i1 = in_off[v + 1], base = i0 + v;
    // a heavy vertex's in-slots are pulled per segment by k_heavy_pr: only its self-loop here
    const int64_t nin = (hv_of && hv_of[v] >= 0) ? 0 : i1 - i0;
    int32_t count = 0;
    for (int64_t c = 0; c < nin; c += 64) {
      const int64_t j = c + lane;
      uint64_t m = 0;
      int32_t nb = 0;
      if (j < nin) {
        const int32_t e = in_eid[i0 + j];
        nb = esrc[e];
        m = em[e] & vm[nb] & mv;
      }
      const uint64_t bal = __ballot(m != 0);
      if (m) {
        const int64_t pos = base + count + __popcll(bal & lanemask_lt());
        snbr[pos] = nb;
        smask[pos] = m;
      }
      count += __popcll(bal);
    }
    // self-loop: out-edges of v are sorted by dst
    int64_t a = out_off[v], b = out_off[v + 1];
    while (a < b) {
      const int64_t mid = (a + b) >> 1;
      if (edst[mid] < (int32_t)v) a = mid + 1; else b = mid;
    }
    if (lane == 0) {
      if (a < out_off[v + 1] && edst[a] == (int32_t)v) {
        const uint64_t m = em[a] & mv;
        if (m) {
          snbr[base + count] = (int32_t)v;
          smask[base + count] = m;
          count++;
        }
      }
      cnt[v] = count;
    }
  }
}

__global__ __launch_bounds__(256) void k_pr_step(int64_t nv, const int64_t* __restrict__ in_off,
                                                 const uint64_t* __restrict__ vm,
                                                 const int32_t* __restrict__ outdeg,
                                                 const int32_t* __restrict__ cnt,
                                                 const int32_t* __restrict__ snbr,
                                                 const uint64_t* __restrict__ smask,
                                                 const double* __restrict__ contrib_cur,
                                                 double* __restrict__ contrib_next,
                                                 double* __restrict__ pr,
                                                 const int32_t* __restrict__ hv_of,
                                                 double* __restrict__ hacc) {
  const int lane = lane_id();
  const int64_t wave = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t v = wave; v < nv; v += nwaves) {
    const uint64_t mv = vm[v];
    if (mv == 0) continue;
    const int32_t n = cnt[v];
    const int64_t base = in_off[v] + v;
    double acc = 0.0;
    for (int32_t c = 0; c < n; c += 64) {
      const int32_t j = c + lane;
      uint64_t m = 0;
      int32_t nb = 0;
      if (j < n) { nb = snbr[base + j]; m = smask[base + j]; }
      uint64_t bal = __ballot(m != 0);
      while (bal) {  // four neighbour rows in flight
        int L[4];
#pragma unroll
        for (int u = 0; u < 4; u++) {
          L[u] = bal ? __builtin_ctzll(bal) : -1;
          if (bal) bal &= bal - 1;
        }
        double x[4];
#pragma unroll
        for (int u = 0; u < 4; u++) {
          const int Lu = L[u] < 0 ? L[0] : L[u];
          const int32_t q = __builtin_amdgcn_readlane(nb, Lu);
          const bool on = L[u] >= 0 && ((readlane64(m, Lu) >> lane) & 1);
          x[u] = on ? contrib_cur[(int64_t)q * 64 + lane] : 0.0;
        }
        acc += (x[0] + x[1]) + (x[2] + x[3]);
      }
    }
    if (hv_of) {
      const int32_t h = hv_of[v];
      if (h >= 0) {
        acc += hacc[(int64_t)h * 64 + lane];
        hacc[(int64_t)h * 64 + lane] = 0.0;
      }
    }
    if ((mv >> lane) & 1) {
      const double p = 0.15 + 0.85 * acc;  // dumplingFactor 0.85, PageRank.scala:11
      const int32_t od = outdeg[v * 64 + lane];
      pr[v * 64 + lane] = p;
      contrib_next[v * 64 + lane] = p / (double)(od > 1 ? od : 1);
    }
  }
}

// ---------------------------------------------------------------- partitioned PageRank
// fp64 rows (PageRank contributions) of a whole list: gather into / scatter out of a
// contiguous buffer, one wave per entry
__global__ __launch_bounds__(256) void k_xgather_f64(int64_t n, const int32_t* __restrict__ xv,
                                                     const double* __restrict__ rows,
                                                     double* __restrict__ buf) {
  const int lane = lane_id();
  const int64_t wave = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t k = wave; k < n; k += nwaves) buf[k * 64 + lane] = rows[(int64_t)xv[k] * 64 + lane];
}
__global__ __launch_bounds__(256) void k_xscatter_f64(int64_t n, const int32_t* __restrict__ xv,
                                                      const double* __restrict__ buf,
                                                      double* __restrict__ rows) {
  const int lane = lane_id();
  const int64_t wave = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t k = wave; k < n; k += nwaves) rows[(int64_t)xv[k] * 64 + lane] = buf[k * 64 + lane];
}

// ---------------------------------------------------------------- launchers
// Launch constants (measured on MI355X).
// deal_group maxima of K2 / the superstep kernel (C4 A/B, profiles/r03/c4_ab_deal.log: K2 16 ~ 64 < 1,
// superstep 4 << 64)
constexpr int kDealSlots = 16;
// supersteps >= kLateStep have small frontiers: at most kLateGrid blocks, the GPU left to the other batches
constexpr int kLateStep = 14, kLateGrid = 1024;

static unsigned grid_for(int64_t items, int per_block, unsigned cap = 8192) {
  int64_t g = (items + per_block - 1) / per_block;
  if (g < 1) g = 1;
  return (unsigned)(g > cap ? cap : g);
}

void launch_batch_clear(hipStream_t s, const BatchClear& clr) {
  k_batch_clear<<<16, 256, 0, s>>>(clr);
}
void launch_vertex_mask(hipStream_t s, const DevGraph& g, const BatchParams& bp, uint64_t* vm,
                        int64_t vstride, bool planar, const BatchClear& clr, int32_t* fc) {
  BatchParams b = bp;
  if (!fc || !bp.sorted) b.carry = 0;
  if (planar) k_vertex_mask<true><<<grid_for(g.nv, 256), 256, 0, s>>>(g.nv, g.voff, g.vkey, b, vm, vstride, clr, fc);
  else k_vertex_mask<false><<<grid_for(g.nv, 256), 256, 0, s>>>(g.nv, g.voff, g.vkey, b, vm, vstride, clr, fc);
}
void launch_edge_mask(hipStream_t s, const DevGraph& g, const BatchParams& bp, uint64_t* em, bool planar,
                      unsigned long long* ecnt, int64_t h0, const uint64_t* vm_ends, int64_t vstride,
                      bool skip_simple, int32_t* fc) {
  BatchParams b = bp;
  if (!fc || !bp.sorted) b.carry = 0;
#define RGPU_EM_ARGS g.ne, g.esrc, g.edst, g.eoff, g.ekey, g.doff, g.dtime, b, em, g.ne, ecnt, h0, g.n_own, vm_ends, \
    vstride, g.dbits, fc, esimple, ens, g.n_ens
  const uint64_t* esimple = g.esimple;
  const int32_t* ens = (skip_simple && g.ens) ? g.ens : nullptr;
  if (skip_simple && g.ens && g.n_ens == 0) return;  // every edge simple: nothing to write
  const unsigned grid = grid_for(ens ? g.n_ens : g.ne, 256);
  if (planar && ecnt) k_edge_mask<true, true, false><<<grid, 256, 0, s>>>(RGPU_EM_ARGS);
  else if (planar && skip_simple) k_edge_mask<true, false, true><<<grid, 256, 0, s>>>(RGPU_EM_ARGS);
  else if (planar) k_edge_mask<true, false, false><<<grid, 256, 0, s>>>(RGPU_EM_ARGS);
  else if (ecnt) k_edge_mask<false, true, false><<<grid, 256, 0, s>>>(RGPU_EM_ARGS);
  else if (skip_simple) k_edge_mask<false, false, true><<<grid, 256, 0, s>>>(RGPU_EM_ARGS);
  else k_edge_mask<false, false, false><<<grid, 256, 0, s>>>(RGPU_EM_ARGS);
#undef RGPU_EM_ARGS
}
void launch_cc_slots(hipStream_t s, const DevGraph& g, int64_t tcut, const uint64_t* vm, const uint64_t* em,
                     int32_t* cnt, int32_t* snbr, uint64_t* smask, uint64_t* vadj, int32_t* lab0,
                     int32_t* lab1, uint64_t* chg1, uint8_t* act2, int32_t* stepflag,
                     int32_t* hostflag, unsigned long long* work, const HeavyBuf& hb,
                     unsigned long long* lanechg, int32_t* uw0, int32_t* uw1, uint64_t* cb1, bool ends,
                     int32_t* ccount, const BatchParams* ebp, int dense_div, int32_t* mneg,
                     const uint8_t* gpeer, uint8_t* pmask, const KernOpts& ko) {
  const bool hv = g.n_seg > 0;
  const bool iem = ebp != nullptr && g.ts_t != nullptr;
  // (partitioned: the peer masks; gpeer and pmask both set)
  auto* kern = (gpeer && pmask)
                   ? (work ? (iem ? k_cc_slots<true, true, true> : k_cc_slots<true, false, true>)
                           : (iem ? k_cc_slots<false, true, true> : k_cc_slots<false, false, true>))
                   : (work ? (iem ? k_cc_slots<true, true, false> : k_cc_slots<true, false, false>)
                           : (iem ? k_cc_slots<false, true, false> : k_cc_slots<false, false, false>));
  // the lean one-partition form held to 6 waves per SIMD (<= 80 VGPRs): C4 cc_slots 54.7 -> 53.4 ms
  // serial at 7 waves before the full-slot fold, 50.8 (7) -> 49.2 ms (6) with it
  // (profiles/r05/ab_occ_c4.jsonl, ab_k2_c4.jsonl)
  if (!work && iem && !(gpeer && pmask)) kern = k_cc_slots<false, true, false, 6>;
  // (a lane-parallel K2 for long windows measured no gain: DESIGN.md §4h)
  if (!work && iem && gpeer && pmask) kern = k_cc_slots<false, true, true, 6>;  // (86 VGPRs unheld)
  BatchParams bp0;
  if (!iem) std::memset(&bp0, 0, sizeof(bp0));
  kern<<<grid_for(g.nv, 4), 256, 0, s>>>(g.nv, g.n_own, g.out_off, g.in_off, g.in_eid, g.esrc,
                                                g.edst, g.grank, vm, em, cnt, snbr, smask, vadj, lab0, lab1, chg1, act2,
                                                stepflag, hostflag, work, hv ? g.hv_of : nullptr, g.hv_seg,
                                                hb.segcnt, hb.segor, hb.best, lanechg, g.ts_e, g.ts_nb, g.ts_t, tcut,
                                                uw0, uw1, cb1, ends ? 1 : 0, ccount, kDealSlots, iem ? *ebp : bp0,
                                                dense_div > 0 && (dense_div & kDense1) && ccount ? 1 : 0,
                                                g.ts_g, mneg, gpeer, pmask, ko.step);
}
void launch_uw_rows(hipStream_t s, int64_t nv, const uint64_t* vm, const int32_t* uw, int32_t* lab) {
  k_uw_rows<<<grid_for(nv, 256), 256, 0, s>>>(nv, vm, uw, lab);
}
void launch_cc_count(hipStream_t s, int64_t nv, int nviews, const uint64_t* vm, const uint64_t* vadj,
                     const int32_t* uw, const int32_t* lab, int32_t* counts, unsigned int* iso) {
  const uint64_t vmask = nviews >= 64 ? ~0ull : ((1ull << nviews) - 1);
  k_cc_count<<<grid_for(nv, 256, 4096), 256, 0, s>>>(nv, vmask, vm, vadj, uw, lab, counts, iso);
}
void launch_cc_roots(hipStream_t s, int64_t nv, int nviews, const uint64_t* vm, const uint64_t* vadj,
                     const int32_t* uw, const int32_t* lab, int32_t* counts, unsigned long long* stats,
                     unsigned int* iso, bool scan_all, const int32_t* grank, bool rows_by_rank) {
  const uint64_t vmask = nviews >= 64 ? ~0ull : ((1ull << nviews) - 1);
  k_cc_roots<<<grid_for(nv, 256, 4096), 256, 0, s>>>(nv, vmask, vm, vadj, uw, lab, counts, stats, iso,
                                                     scan_all ? 1 : 0, grank, rows_by_rank ? 1 : 0);
}
void launch_cc_step(hipStream_t s, int step, const DevGraph& g, const uint64_t* vm,
                    const int32_t* cnt, const int32_t* snbr, const uint64_t* smask,
                    const int32_t* lab_cur, int32_t* lab_next, const uint64_t* chg_prev,
                    uint64_t* chg_next, const uint8_t* act_cur, uint8_t* act_next,
                    uint8_t* act_clear, int32_t* stepflag, int32_t* hostflag,
                    unsigned long long* work, unsigned long long* lanechg, int32_t* hbest, const int32_t* uw_cur, int32_t* uw_next,
                    const ChgBits& cb, int32_t* ccount, int dense_div, const int32_t* mneg, bool long_views,
                    const KernOpts& ko) {
  // late supersteps have small frontiers: a smaller grid leaves the GPU to the other batches.
  // A small graph's dense supersteps are latency-bound and share the GPU with the other batch
  // slots too: a 1,024-block cap measured 4 % faster on C2 (100k vertices) and 2 % slower on a
  // 4.7M-vertex C4-shaped graph, hence the size rule.
  const unsigned full = g.nv <= ((int64_t)1 << 21) ? 1024u : 4096u;
  const unsigned cap = step >= kLateStep ? (full < (unsigned)kLateGrid ? full : (unsigned)kLateGrid) : full;
  const int32_t* hv_of = hbest ? g.hv_of : nullptr;
  // work != null (profile runs): the counting instantiation; the timed runs use the lean one.
  // Same-box A/B against the 2-vertex-chunk kernel it replaced (profiles/r04/ab_packed_step.jsonl):
  // C4 serial cc_step 207.6 -> 155.1 ms, query 343 -> 286 ms.
#define RGPU_PK_ARGS step, g.nv, g.adj_off, vm, cnt, snbr, smask, lab_cur, lab_next, chg_prev, chg_next, \
    act_cur, act_next, act_clear, stepflag, hostflag, work, hv_of, hbest, lanechg, uw_cur, uw_next, \
    cb.next, cb.clear, cb.words, ccount, dense_div, kDealSlots, uw_cur ? mneg : nullptr, opts
  const int opts = ko.step;
  const unsigned gridp = grid_for(g.nv, 256, cap);
  // The long-window form (lane-parallel members, full folds) pays in the busy early supersteps; it
  // spills a few registers, and a kernel with scratch launches its waves more slowly, which the
  // late, sparse supersteps (mostly idle waves) feel: from kLongSteps on, the short form runs.
  const bool lf = long_views && step < ko.long_steps;
  if (work) {
    if (lf) k_cc_step_pk<false, true, true><<<gridp, 256, 0, s>>>(RGPU_PK_ARGS);
    else k_cc_step_pk<false, true, false><<<gridp, 256, 0, s>>>(RGPU_PK_ARGS);
  } else if (lf) {
    k_cc_step_pk<false, false, true><<<gridp, 256, 0, s>>>(RGPU_PK_ARGS);
  } else {
    k_cc_step_pk<false, false, false><<<gridp, 256, 0, s>>>(RGPU_PK_ARGS);
  }
#undef RGPU_PK_ARGS
}
void launch_heavy_slots(hipStream_t s, const DevGraph& g, int64_t tcut, const uint64_t* vm, const uint64_t* em,
                        int32_t* snbr, uint64_t* smask, const HeavyBuf& hb, bool ends, unsigned long long* work,
                        const BatchParams* ebp, const KernOpts& ko) {
  if (g.n_seg <= 0) return;
  const bool iem = ebp != nullptr && g.ts_t != nullptr;
  BatchParams bp0;
  if (!iem) std::memset(&bp0, 0, sizeof(bp0));
  (iem ? k_heavy_slots<true> : k_heavy_slots<false>)<<<grid_for(g.n_seg, 4, 16384), 256, 0, s>>>(
      g.n_seg, g.seg_v, g.seg_h, g.seg_lo, g.seg_n, g.out_off, g.in_off, g.adj_off, g.in_eid, g.esrc, g.edst, vm, em,
      snbr, smask, hb.segcnt, hb.segor, hb.best, g.grank, g.n_own, g.ts_e, g.ts_nb, g.ts_t, tcut, ends ? 1 : 0, work,
      iem ? *ebp : bp0, g.ts_g, ko.step);
}
// segments per wave and round of the hub kernels' prologue (kernels.hpp kHubPro, KernOpts.hub_pro)
static int hub_pro(const KernOpts& ko) { return ko.hub_pro < 1 ? 1 : (ko.hub_pro > 64 ? 64 : ko.hub_pro); }
void launch_hub_demote(hipStream_t s, const DevGraph& g, const HeavyBuf& hb, int32_t* cnt, int32_t* snbr,
                       uint64_t* smask, const uint64_t* chg1, uint8_t* act2, bool dense1) {
  if (g.n_heavy <= 0) return;
  k_hub_demote<<<grid_for(g.n_heavy, 4, 16384), 256, 0, s>>>(g.n_heavy, g.n_own, g.hv_seg, g.seg_v, g.seg_lo, g.adj_off,
                                                             hb.segcnt, cnt, snbr, smask, chg1, act2, dense1 ? 1 : 0);
}
void launch_heavy_gather(hipStream_t s, const DevGraph& g, const int32_t* snbr, const uint64_t* smask,
                         const int32_t* lab_cur, const uint64_t* chg_prev, const uint8_t* act_cur,
                         const int32_t* stepflag, int step, const HeavyBuf& hb, const int32_t* uw_cur,
                         const uint64_t* cb_prev, const int32_t* ccount, int dense_div, unsigned long long* work,
                         const uint64_t* vm, const int32_t* mneg, const KernOpts& ko) {
  if (g.n_seg <= 0) return;
  // held to 6 waves per SIMD (<= 80 VGPRs; unconstrained it takes 103, 4 waves): C4 heavy 48.6 ->
  // 47.7 ms serial (profiles/r05/ab_occ_c4.jsonl)
  const int pro = hub_pro(ko);
  k_heavy_gather<6><<<grid_for(g.n_seg, 4 * pro, 16384), 256, 0, s>>>(step, g.n_seg, g.seg_v, g.seg_h, g.seg_lo, hb.segcnt,
                                                             snbr, smask, lab_cur, chg_prev, act_cur, stepflag,
                                                             hb.best, g.n_own, uw_cur, cb_prev, ccount, dense_div,
                                                             g.n_own, work, vm, mneg, pro, ko.step);
}
void launch_heavy_mark(hipStream_t s, const DevGraph& g, const int32_t* snbr, const uint64_t* smask,
                       const uint64_t* chg_now, uint8_t* act_next, const int32_t* stepflag, int step,
                       const HeavyBuf& hb, const uint8_t* act_cur, const uint64_t* vm, const uint64_t* em,
                       int64_t tcut, const int32_t* ccount, int dense_div, unsigned long long* work,
                       const int32_t* uw_ghost, const KernOpts& ko) {
  if (g.n_seg <= 0) return;
  k_heavy_mark<<<grid_for(g.n_seg, 4 * hub_pro(ko), 16384), 256, 0, s>>>(step, g.n_seg, g.seg_v, g.seg_lo, hb.segcnt, snbr, smask,
                                                           chg_now, act_cur, act_next, stepflag, g.n_own, g.seg_n,
                                                           g.out_off, g.in_off, g.adj_off, g.in_eid, g.esrc, g.edst,
                                                           vm, em, g.ts_e, g.ts_nb, g.ts_t, tcut, ccount, dense_div,
                                                           g.n_own, work, uw_ghost, hub_pro(ko));
}
int64_t deg_top_waves(int64_t nv) { return (int64_t)grid_for(nv, 4, 2048) * 4; }
void launch_degree(hipStream_t s, const DevGraph& g, const uint64_t* vm, const uint64_t* em,
                   int32_t* outdeg, int32_t* indeg, unsigned long long* stats, const DegTop* top) {
  const unsigned grid = grid_for(g.nv, 4, 2048);
  const int32_t* hv = g.n_seg > 0 ? g.hv_of : nullptr;
  if (top)
    k_degree<true><<<grid, 256, 0, s>>>(g.nv, g.out_off, g.in_off, g.in_eid, vm, em, outdeg, indeg, stats, hv,
                                        g.grank, top->cand_key, top->cand_pos);
  else
    k_degree<false><<<grid, 256, 0, s>>>(g.nv, g.out_off, g.in_off, g.in_eid, vm, em, outdeg, indeg, stats, hv,
                                         nullptr, nullptr, nullptr);
  if (g.n_seg > 0)
    k_heavy_degree<<<grid_for(g.n_seg, 4, 16384), 256, 0, s>>>(g.n_seg, g.seg_v, g.seg_lo, g.seg_n, g.out_off,
                                                               g.in_off, g.adj_off, g.in_eid, vm, em, outdeg, indeg,
                                                               stats, g.nv);
  if (top)
    k_deg_top_merge<<<kViews, 256, 0, s>>>((int64_t)grid * 4, top->cand_key, top->cand_pos, g.n_seg > 0 ? g.n_heavy : 0,
                                           g.hv_seg, g.seg_v, g.nv, vm, indeg, outdeg, g.grank, top->key, top->pos,
                                           top->out);
}
void launch_pr_slots(hipStream_t s, const DevGraph& g, const uint64_t* vm, const uint64_t* em,
                     const int32_t* outdeg, int32_t* cnt, int32_t* snbr, uint64_t* smask,
                     double* pr, double* contrib) {
  k_pr_slots<<<grid_for(g.nv, 4), 256, 0, s>>>(g.nv, g.out_off, g.in_off, g.in_eid, g.esrc, g.edst,
                                                vm, em, outdeg, cnt, snbr, smask, pr, contrib,
                                                g.n_seg > 0 ? g.hv_of : nullptr);
}
void launch_pr_step(hipStream_t s, const DevGraph& g, const uint64_t* vm, const uint64_t* em,
                    const int32_t* outdeg, const int32_t* cnt, const int32_t* snbr, const uint64_t* smask,
                    const double* contrib_cur, double* contrib_next, double* pr, double* hacc) {
  if (g.n_seg > 0 && hacc)
    k_heavy_pr<<<grid_for(g.n_seg, 4, 16384), 256, 0, s>>>(g.n_seg, g.seg_v, g.seg_h, g.seg_lo, g.seg_n, g.out_off,
                                                           g.in_off, g.adj_off, g.in_eid, g.esrc, vm, em, contrib_cur,
                                                           hacc, g.nv);
  k_pr_step<<<grid_for(g.nv, 4), 256, 0, s>>>(g.nv, g.in_off, vm, outdeg, cnt, snbr, smask,
                                               contrib_cur, contrib_next, pr,
                                               g.n_seg > 0 && hacc ? g.hv_of : nullptr, hacc);
}

void launch_xgather_f64(hipStream_t s, int64_t n, const int32_t* xv, const double* rows, double* buf) {
  if (n > 0) k_xgather_f64<<<grid_for(n, 4, 4096), 256, 0, s>>>(n, xv, rows, buf);
}
void launch_xscatter_f64(hipStream_t s, int64_t n, const int32_t* xv, const double* buf, double* rows) {
  if (n > 0) k_xscatter_f64<<<grid_for(n, 4, 4096), 256, 0, s>>>(n, xv, buf, rows);
}

}  // namespace rgpu
