// xchg.hip — device side of the vertex-partitioned mode (host: rgpu.cpp).
//
// A partition keeps its owned vertices and ghost copies of their remote neighbours (the
// reference's SplitEdge copies, EntityStorage.scala:303-305).  Three exchanges:
//
//   ghost membership   once per hop block: the owners' K1 vertex-mask words of the boundary
//                      vertices (a ghost's own history is not on this partition).  Fixed sizes.
//   label records      once per superstep: the ReaderWorker's VertexMessage traffic
//                      (VertexVisitor.messageAllNeighbours, VertexVisitor.scala:112-147) as
//                      records {entry, label, views}: one per distinct new label of a changed
//                      boundary vertex, restricted to the views in which it has a kept
//                      neighbour — a window-major batch (64 hops of one window) mostly changes
//                      every lane to the same label, so a record is 16 B instead of a 256-B row.
//   component counts   once per batch: (label, view, count) to the label's owner, which counts
//                      at the label vertex (ConnectedComponents.returnResults :37-42 merged by
//                      processBatchWindowResults :137).
#include <hip/hip_runtime.h>

#include <climits>
#include <cstdint>
#include <cstring>

#include <hipcub/device/device_scan.hpp>

#include <stdexcept>
#include <vector>

#include "kernels.hpp"
#include "window_bits.hpp"

namespace rgpu {

namespace {

__device__ __forceinline__ int lane_of() { return threadIdx.x & 63; }
__device__ __forceinline__ uint64_t rl64(uint64_t x, int l) {
  const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)x, l);
  const uint32_t hi = __builtin_amdgcn_readlane((uint32_t)(x >> 32), l);
  return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ uint64_t lanemask_below(int lane) { return lane ? (~0ull >> (64 - lane)) : 0ull; }
__device__ __forceinline__ int owner_of(int64_t id, int np) { return (int)(((id < 0 ? -id : id) % (10 * (int64_t)np)) / 10); }
// record index i of a receive layout -> peer
__device__ __forceinline__ int peer_of(const XPeers& P, int64_t i) {
  int q = 0;
  while (q + 1 < P.np && i >= P.pre[q + 1]) q++;
  return q;
}
// rank of owned vertex `id`, or -1 (bucket index: about one probe)
__device__ __forceinline__ int64_t owned_rank(const OwnIdx& I, int64_t id) {
  const int64_t b = id >> I.shift;
  for (int64_t i = I.boff[b], e = I.boff[b + 1]; i < e; i++)
    if (I.vid[i] == id) return i;
  return -1;
}

// kernels.hip dense_rule(ccount, r - 1): superstep r ran with every member visited (its flags
// were not written by a dense step r - 1)
__device__ __forceinline__ bool dense_after(const int32_t* __restrict__ ccount, int r, int64_t nv, int div) {
  if (div <= 0 || !ccount || r < 2) return false;
  if (r == 2) return (div & kDense1) != 0;  // step 1 (K2) dense (kernels.hpp kDense1)
  div &= kDense1 - 1;
  int64_t x = ccount[(r - 2) * kCountShards + (threadIdx.x & 63)];
  for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o);
  return x * div >= nv;
}

}  // namespace

// ------------------------------------------------------------------ ghost membership
// Send layout: peer q's words are [plane][entry] at planes * xoff[q] (receive layout mirrors it).
__global__ __launch_bounds__(256) void k_xvm_pack(int64_t nx, const int32_t* __restrict__ xv,
                                                  const int32_t* __restrict__ xq,
                                                  const int64_t* __restrict__ xoff, int planes,
                                                  const uint64_t* __restrict__ vm, int64_t vstride,
                                                  uint64_t* __restrict__ out) {
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < nx; e += (int64_t)gridDim.x * blockDim.x) {
    const int q = xq[e];
    const int64_t n = xoff[q + 1] - xoff[q], base = planes * xoff[q] + (e - xoff[q]);
    const int32_t v = xv[e];
    for (int p = 0; p < planes; p++) out[base + p * n] = vm[p * vstride + v];
  }
}
__global__ __launch_bounds__(256) void k_xvm_unpack(int64_t nx, const int32_t* __restrict__ xv,
                                                    const int32_t* __restrict__ xq,
                                                    const int64_t* __restrict__ xoff, int planes,
                                                    const uint64_t* __restrict__ in, uint64_t* __restrict__ vm,
                                                    int64_t vstride) {
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < nx; e += (int64_t)gridDim.x * blockDim.x) {
    const int q = xq[e];
    const int64_t n = xoff[q + 1] - xoff[q], base = planes * xoff[q] + (e - xoff[q]);
    const int32_t g = xv[e];
    for (int p = 0; p < planes; p++) vm[p * vstride + g] = in[base + p * n];
  }
}

// ------------------------------------------------------------------ label records
// Boundary entry e (owned vertex xv[e], peer xq[e]) is sent when the vertex was visited in the
// step (act; null = every member, superstep 1) and changed in a view where it has a kept
// neighbour (vadj, the OR of its kept slot masks).  Per distinct new label one record with the
// views holding it.  A wave takes 64 entries: it counts the records per peer (lane q), reserves
// them with one atomicAdd per (wave, peer), then writes them; scnt counts past the capacity
// too, so the host sees an overflow and repeats the pack into a larger buffer.
// A wave takes a run of kPackRun chunks of 64 boundary vertices: it counts its records per peer over
// the whole run, reserves them with one atomicAdd per peer, then writes them.  (Runs of 16 chunks,
// to cut the reservations on the 8 counters, measured 4.7x slower at P = 8: the pack is bound by
// each chunk's chain of dependent loads, and fewer, longer waves hide less of it.)
constexpr int kPackRun = 1;
__device__ __forceinline__ void pack_chunk(bool write, const XPeers& P, const XSend& X, int64_t c,
                                           const uint8_t* __restrict__ act, const uint64_t* __restrict__ chg_now,
                                           const uint64_t* __restrict__ vadj, const int32_t* __restrict__ lab,
                                           const int32_t* __restrict__ uw, XRec* __restrict__ sbuf,
                                           unsigned long long& cq, unsigned long long& off, int lane) {
  // lane = boundary vertex (ascending owned rank): its words are read once for all its peers
  const int64_t b = c * 64 + lane;
  const bool ok = b < X.nb;
  const int32_t v = ok ? X.v[b] : 0;
  const uint32_t pm = ok ? X.pm[b] : 0u;
  uint64_t m = 0;
  if (ok && (act == nullptr || act[v])) m = chg_now[v] & vadj[v];
  if (!__ballot(m != 0)) return;
  // A uniform sender (its word is its row) has one label: one record per peer, written by its own
  // lane.  Only mixed senders walk their distinct labels one by one (lane = view).
  const int32_t u = (m != 0 && uw) ? uw_label(uw[v]) : kMixed;
  const bool uni = m != 0 && u != kMixed;
  const uint64_t mixed = __ballot(m != 0 && !uni);
  for (int p = 0; p < P.np; p++) {  // uniform records, in lane order per peer
    const uint64_t bp = __ballot(uni && ((pm >> p) & 1));
    if (!bp) continue;
    if (write) {
      const unsigned long long base = __builtin_amdgcn_readlane((uint32_t)off, p) |
                                      ((unsigned long long)__builtin_amdgcn_readlane((uint32_t)(off >> 32), p) << 32);
      if ((bp >> lane) & 1) {
        const unsigned long long pos = base + __popcll(bp & lanemask_below(lane));
        if (pos < (unsigned long long)P.cap[p]) {
          XRec r;
          r.e = X.e[b * kMaxParts + p];
          r.val = (int32_t)((uint32_t)u | 0x80000000u);  // sign bit: sender uniform
          r.mask = m;
          sbuf[P.base[p] + pos] = r;
        }
      }
      if (lane == p) off += (unsigned long long)__popcll(bp);
    } else if (lane == p) {
      cq += (unsigned long long)__popcll(bp);
    }
  }
  for (uint64_t bb = mixed; bb; bb &= bb - 1) {  // mixed senders: per distinct label, per peer
    const int L = __builtin_ctzll(bb);
    const int32_t vL = __builtin_amdgcn_readlane(v, L);
    const uint32_t pmL = __builtin_amdgcn_readlane(pm, L);
    const int64_t bL = c * 64 + L;
    uint64_t mm = rl64(m, L);
    const int32_t x = lab[(int64_t)vL * 64 + lane];
    while (mm) {
      const int32_t val = __builtin_amdgcn_readlane(x, __builtin_ctzll(mm));
      const uint64_t same = __ballot(((mm >> lane) & 1) && x == val);
      if (write) {
        for (uint32_t pp = pmL; pp; pp &= pp - 1) {
          const int p = __builtin_ctz(pp);
          const unsigned long long pos = __builtin_amdgcn_readlane((uint32_t)off, p) |
                                         ((unsigned long long)__builtin_amdgcn_readlane((uint32_t)(off >> 32), p) << 32);
          if (lane == 0 && pos < (unsigned long long)P.cap[p]) {
            XRec r;
            r.e = X.e[bL * kMaxParts + p];
            r.val = val;
            r.mask = same;
            sbuf[P.base[p] + pos] = r;
          }
          if (lane == p) off++;
        }
      } else if (lane < 32 && ((pmL >> lane) & 1)) {
        cq++;
      }
      mm &= ~same;
    }
  }
}
__global__ __launch_bounds__(256) void k_xpack_rec(XPeers P, XSend X, const uint8_t* __restrict__ act,
                                                   const uint64_t* __restrict__ chg_now,
                                                   const uint64_t* __restrict__ vadj,
                                                   const int32_t* __restrict__ lab,
                                                   const int32_t* __restrict__ uw, XRec* __restrict__ sbuf,
                                                   unsigned long long* __restrict__ scnt,
                                                   const int32_t* __restrict__ ccount, int dense_div, int step,
                                                   int64_t n_own) {
  const int lane = lane_of();
  if (dense_after(ccount, step, n_own, dense_div)) act = nullptr;  // the step visited every member
  const int64_t wave = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  const int64_t nchunks = (X.nb + 63) / 64;
  for (int64_t c0 = wave * kPackRun; c0 < nchunks; c0 += nwaves * kPackRun) {
    const int64_t c1 = c0 + kPackRun < nchunks ? c0 + kPackRun : nchunks;
    unsigned long long cq = 0, off = 0;  // lane p: this run's records for peer p, then its next position
    for (int64_t c = c0; c < c1; c++) pack_chunk(false, P, X, c, act, chg_now, vadj, lab, uw, sbuf, cq, off, lane);
    if (!__ballot(cq != 0)) continue;
    if (lane < P.np && cq) off = atomicAdd(&scnt[lane], cq);
    for (int64_t c = c0; c < c1; c++) pack_chunk(true, P, X, c, act, chg_now, vadj, lab, uw, sbuf, cq, off, lane);
  }
}

// ------------------------------------------------------------------ send index (per boundary vertex)
__global__ __launch_bounds__(256) void k_xsend_flag(int64_t nx, const int32_t* __restrict__ xv,
                                                    int32_t* __restrict__ flag) {
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < nx; e += (int64_t)gridDim.x * blockDim.x)
    flag[xv[e]] = 1;  // (idempotent plain stores)
}
__global__ __launch_bounds__(256) void k_xsend_list(int64_t n_own, const int32_t* __restrict__ flag,
                                                    const int32_t* __restrict__ pos, int32_t* __restrict__ xb) {
  for (int64_t v = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; v < n_own; v += (int64_t)gridDim.x * blockDim.x)
    if (flag[v]) xb[pos[v]] = (int32_t)v;
}
__global__ __launch_bounds__(256) void k_xsend_entries(int64_t nx, const int32_t* __restrict__ xv,
                                                       const int32_t* __restrict__ xq, const int64_t* __restrict__ xoff,
                                                       const int32_t* __restrict__ pos, int32_t* __restrict__ xe,
                                                       uint32_t* __restrict__ pm) {
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < nx; e += (int64_t)gridDim.x * blockDim.x) {
    const int q = xq[e];
    const int64_t b = pos[xv[e]];
    xe[b * kMaxParts + q] = (int32_t)(e - xoff[q]);
    atomicOr(&pm[b], 1u << q);
  }
}

// counts exchange words: [2q] = records for q (0 for self), [2q+1] = this partition changed a
// label in the step (the halting vote, AnalysisTask.endStep :208-225); the counters are reset
// for the next pack
__global__ void k_xcounts(int np, int me, unsigned long long* __restrict__ scnt, const int32_t* __restrict__ stepflag,
                          int64_t* __restrict__ xa) {
  const int q = threadIdx.x;
  if (q >= np) return;
  xa[2 * q] = q == me ? 0 : (int64_t)scnt[q];
  xa[2 * q + 1] = stepflag ? (stepflag[0] != 0) : 0;
  scnt[q] = 0;
}

// ghosts whose change word a record set two supersteps ago: clear it in that parity's words, and
// set their uniform word back to kGhostQuiet (uw non-null)
__global__ __launch_bounds__(256) void k_xclear(XPeers P, const XRec* __restrict__ rbuf,
                                                const int32_t* __restrict__ xrv, uint64_t* __restrict__ chg,
                                                int32_t* __restrict__ uw) {
  const int64_t n = P.pre[P.np];
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int q = peer_of(P, i);
    const int32_t g = xrv[P.xoff[q] + rbuf[P.base[q] + i - P.pre[q]].e];
    chg[g] = 0;
    if (uw) uw[g] = kGhostQuiet;
  }
}

// Records into ghost rows: the record's label in its views, and its views into the ghost's
// change word (a ghost's records arrive together; the OR collects them).  A record whose sender's
// row is uniform (sign bit of val; it is then the ghost's only record of the step) sets the
// ghost's uniform word instead of its row, lane = record: readers only gather a ghost in the views
// its change word holds, which are the record's.  Other records mark the ghost mixed (kernels.hip
// kMixed), one per wave iteration with lane = view.  (Four records per wave, 16 lanes each, with
// two atomics per record, made the unpack the largest partitioned kernel.)
__global__ __launch_bounds__(256) void k_xunpack_rec(XPeers P, const XRec* __restrict__ rbuf,
                                                     const int32_t* __restrict__ xrv, int32_t* __restrict__ lab,
                                                     uint64_t* __restrict__ chg, int32_t* __restrict__ uw,
                                                     uint64_t* __restrict__ cb) {
  const int64_t n = P.pre[P.np];
  const int lane = lane_of();
  const int64_t wave = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t i0 = wave * 64; i0 < n; i0 += nwaves * 64) {
    // lane = record: a uniform record is its ghost's only record of the step, so its word and
    // change word are plain stores; mixed records (rows, OR-ed change words) one by one below
    const int64_t i = i0 + lane;
    const bool ok = i < n;
    XRec r{0, 0, 0};
    int32_t g = 0;
    if (ok) {
      const int q = peer_of(P, i);
      r = rbuf[P.base[q] + i - P.pre[q]];
      g = xrv[P.xoff[q] + r.e];
    }
    const bool uni = ok && uw && r.val < 0;
    if (uni) {
      uw[g] = uw_word(r.val & 0x7fffffff, true);  // the ghost changed in this step (kChgFlag)
      chg[g] = r.mask;
      if (cb) atomicOr((unsigned long long*)&cb[g >> 6], 1ull << (g & 63));  // (ChgBits)
    }
    for (uint64_t b = __ballot(ok && !uni); b; b &= b - 1) {
      const int L = __builtin_ctzll(b);
      const int32_t gL = __builtin_amdgcn_readlane(g, L);
      const int32_t val = __builtin_amdgcn_readlane(r.val, L) & 0x7fffffff;
      const uint64_t mL = rl64(r.mask, L);
      if ((mL >> lane) & 1) lab[(int64_t)gL * 64 + lane] = val;
      if (lane == 0) {
        if (uw) uw[gL] = kMixed;
        atomicOr((unsigned long long*)&chg[gL], (unsigned long long)mL);
        if (cb) atomicOr((unsigned long long*)&cb[gL >> 6], 1ull << (gL & 63));
      }
    }
  }
}

// After the unpack: the first record of every ghost marks the ghost's owned neighbours that
// share a changed view (the next frontier, as a local change would).  Ghosts keep no compacted
// slots (K2 runs over the owned vertices only): the kept views of a static slot, bits & vm[nb] &
// vm[g], are recomputed here for the ghosts that changed, over the time-ordered slots up to the
// batch's cut (bits: K2's inline edge bits for a simple slot, else em[e]; without time-ordered
// slots the CSR order and em).  Nothing to mark when superstep r is dense (the next one visits
// every member).  Heavy ghosts: k_heavy_mark.
template <bool TS>
__global__ __launch_bounds__(256) void k_xmark(XPeers P, const XRec* __restrict__ rbuf,
                                               const int32_t* __restrict__ xrv, const uint64_t* __restrict__ chg,
                                               const int64_t* __restrict__ out_off,
                                               const int64_t* __restrict__ in_off,
                                               const int32_t* __restrict__ in_eid,
                                               const int32_t* __restrict__ esrc, const int32_t* __restrict__ edst,
                                               const uint64_t* __restrict__ vm, const uint64_t* __restrict__ em,
                                               const int32_t* __restrict__ hv_of, uint8_t* __restrict__ act_next,
                                               const int64_t* __restrict__ adj_off, const int32_t* __restrict__ ts_e,
                                               const int32_t* __restrict__ ts_nb, const int64_t* __restrict__ ts_t,
                                               int64_t tcut, BatchParams ebp, int iem,
                                               const int32_t* __restrict__ ccount, int dense_div, int step,
                                               int64_t n_own, int64_t nv_all) {
  if (dense_after(ccount, step + 1, n_own, dense_div)) return;  // step r dense: r+1 visits every member
  __shared__ HopLDS L;
  if (TS && iem) hop_lds_init(L, ebp, ebp.thr_e);
  const int64_t n = P.pre[P.np];
  const int lane = lane_of();
  const int64_t wave = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t i = wave; i < n; i += nwaves) {
    const int q = peer_of(P, i);
    const int64_t k = i - P.pre[q];
    const int32_t e0 = rbuf[P.base[q] + k].e;
    if (k > 0 && rbuf[P.base[q] + k - 1].e == e0) continue;  // not the ghost's first record
    // (bounds guards: a record outside the plan is a bug upstream — the parity tests see its
    // missing marks — and must not become a fault that takes the device down)
    if (e0 < 0 || e0 >= P.xoff[q + 1] - P.xoff[q]) continue;
    const int32_t g = xrv[P.xoff[q] + e0];
    if (g < 0 || g >= nv_all) continue;
    if (hv_of && hv_of[g] >= 0) continue;
    const uint64_t ch = chg[g] & vm[g];
    if (TS) {
      const int64_t a = adj_off[g], ntot = adj_off[g + 1] - a;
      for (int64_t c = 0; c < ntot; c += 64) {
        if (ts_time(ts_t[a + c]) < tcut) break;  // newest first: the rest are dead in every view
        const int64_t j = c + lane;
        if (j >= ntot) continue;
        const int64_t tsw = ts_t[a + j];
        if (ts_time(tsw) < tcut) continue;
        const int32_t nb = ts_nb[a + j];
        if (nb == g) continue;
        const uint64_t bits = (iem && ts_simple(tsw)) ? simple_bits(L, ebp.sorted, ts_time(tsw)) : em[ts_e[a + j]];
        if (bits & vm[nb] & ch) act_next[nb] = 1;
      }
      continue;
    }
    const int64_t o0 = out_off[g], i0 = in_off[g];
    const int64_t nout = out_off[g + 1] - o0, ntot = nout + (in_off[g + 1] - i0);
    for (int64_t c = 0; c < ntot; c += 64) {
      const int64_t j = c + lane;
      if (j >= ntot) continue;
      int64_t e;
      int32_t nb;
      if (j < nout) { e = o0 + j; nb = edst[e]; }
      else { e = in_eid[i0 + (j - nout)]; nb = esrc[e]; }
      if (nb != g && (em[e] & vm[nb] & ch)) act_next[nb] = 1;
    }
  }
}

// ------------------------------------------------------------------ component counts
// Label -> count of the partition's owned members (ConnectedComponents.returnResults :37-42)
// Component counts, partitioned (ConnectedComponents.returnResults :37-42 merged by
// processBatchWindowResults :137): as kernels.hip k_cc_count, from the owned members' uniform
// words (a group of uniform members with the same (label, views) is one row-wide add) or rows
// (mixed members, lane = view), through a 64-row LDS cache keyed by label.  A label owned here is
// counted at its count row (the label vertex's local rank, through OwnIdx); any other label
// becomes records (label | view << 31 | count << 37) for its owner — the cache turns the giant
// component of a block into one record per view.  Records are reserved per (wave | block, peer)
// with one atomicAdd; gcnt[q] counts every record for peer q (past the capacity too, so the host
// sees an overflow and runs the REMOTE_ONLY pass again into a larger buffer).  Members with no
// kept slot in a view are islands (iso[shard][view]).
__device__ __forceinline__ uint64_t shfl_xor64(uint64_t x, int d) {
  const uint32_t lo = __shfl_xor((uint32_t)x, d), hi = __shfl_xor((uint32_t)(x >> 32), d);
  return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ uint64_t transpose64(uint64_t x, int lane) {  // (kernels.hip)
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
// count row (local rank) of owned label x
__device__ __forceinline__ int64_t label_row(const OwnIdx& I, int32_t x) {
  const int64_t k = owned_rank(I, x);
  return k < 0 ? -1 : (I.pos ? (int64_t)I.pos[k] : k);
}
__device__ __forceinline__ unsigned long long count_rec(int32_t x, int j, unsigned c) {
  return (unsigned long long)(uint32_t)x | ((unsigned long long)j << 31) | ((unsigned long long)c << 37);
}
// A wave's outgoing count records are staged in LDS, kStage per peer, and reserved in the send
// buffer with one atomicAdd per flush: one global atomic per (group of records, peer) serialised
// on the 8 gcnt words (~10 ns each at the memory side, DESIGN.md §4 lesson 1) and made the
// partitioned count pass ~20x the one-partition one.  The flush order is fixed per wave, so a
// REMOTE_ONLY re-run emits the same records per peer (in another order at most).
constexpr int kStage = 64;
struct CountStage {
  unsigned long long (*rec)[kStage];  // [peer][kStage], wave-private LDS
  int n;                              // lane q: records staged for peer q (a register, not LDS: the
                                      // lanes read it right after another lane's update)
};
// wave-uniform: reserve peer q's staged records in the send buffer and write them out
__device__ __forceinline__ void stage_flush(CountStage& st, int q, const XPeers& P,
                                            unsigned long long* __restrict__ gcnt,
                                            unsigned long long* __restrict__ hsbuf, int lane) {
  const int n = __builtin_amdgcn_readlane(st.n, q);
  if (n == 0) return;
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");  // the other lanes' LDS record stores
  unsigned long long base = 0;
  if (lane == 0) base = atomicAdd(&gcnt[q], (unsigned long long)n);
  base = ((unsigned long long)__builtin_amdgcn_readlane((uint32_t)(base >> 32), 0) << 32) |
         __builtin_amdgcn_readlane((uint32_t)base, 0);
  if (lane < n && base + lane < (unsigned long long)P.cap[q]) hsbuf[P.base[q] + (int64_t)(base + lane)] = st.rec[q][lane];
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");  // read before the slots are reused
  if (lane == q) st.n = 0;
}
// wave-wide: the lanes with `on` send (x, j, c) (remote labels, staged) or add it (owned labels)
template <bool REMOTE_ONLY>
__device__ __forceinline__ void count_direct(bool on, int32_t x, int j, unsigned c, const XPeers& P, const OwnIdx& I,
                                             int32_t* __restrict__ counts, unsigned long long* __restrict__ gcnt,
                                             unsigned long long* __restrict__ hsbuf, int lane, CountStage& st) {
  const int q = on ? owner_of(x, P.np) : -1;
  if (!REMOTE_ONLY && q == P.me) {
    const int64_t r = label_row(I, x);  // always found: a label is a member's id
    if (r >= 0) atomicAdd(&counts[r * 64 + j], (int32_t)c);
  }
  for (uint64_t todo = __ballot(q >= 0 && q != P.me); todo;) {
    const int qL = __builtin_amdgcn_readlane(q, __builtin_ctzll(todo));
    const uint64_t mine = __ballot(q == qL);
    todo &= ~mine;
    const int n = __popcll(mine);
    if (__builtin_amdgcn_readlane(st.n, qL) + n > kStage) stage_flush(st, qL, P, gcnt, hsbuf, lane);
    const int c0 = __builtin_amdgcn_readlane(st.n, qL);
    if (q == qL) st.rec[qL][c0 + __popcll(mine & (lane ? (~0ull >> (64 - lane)) : 0ull))] = count_rec(x, j, c);
    if (lane == qL) st.n = c0 + n;
  }
}
template <bool REMOTE_ONLY>
__global__ __launch_bounds__(256) void k_part_count(XPeers P, OwnIdx I, uint64_t vmask, const uint64_t* __restrict__ vm,
                                                    const uint64_t* __restrict__ vadj, const int32_t* __restrict__ uw,
                                                    const int32_t* __restrict__ lab, int32_t* __restrict__ counts,
                                                    unsigned int* __restrict__ iso_g,
                                                    unsigned long long* __restrict__ gcnt,
                                                    unsigned long long* __restrict__ hsbuf) {
  // The cache is private to a wave (16 rows each): a wave's operations run in a fixed order, so
  // the records it emits are the same on every run — the REMOTE_ONLY pass after a send-buffer
  // overflow must emit exactly the records the counts exchange announced.
  constexpr int kRows = 16;
  __shared__ unsigned int iso[64];
  __shared__ int32_t ckey_s[4][kRows];
  __shared__ unsigned int crow_s[4][kRows][64];
  __shared__ unsigned long long srec_s[4][kMaxParts][kStage];
  const int lane = lane_of(), wib = threadIdx.x >> 6;
  int32_t* ckey = ckey_s[wib];
  unsigned int (*crow)[64] = crow_s[wib];
  CountStage st{srec_s[wib], 0};
  if (threadIdx.x < 64) iso[threadIdx.x] = 0;
  if (lane < kRows) ckey[lane] = -1;
  for (int h = 0; h < kRows; h++) crow[h][lane] = 0;
  __syncthreads();
  auto cached = [&](int32_t x, int j, unsigned c) -> bool {  // per lane
    const int h0 = (int)(((uint32_t)x * 2654435761u) >> 28);
    for (int p = 0; p < 4; p++) {
      const int h = (h0 + p) & (kRows - 1);
      int32_t k = ckey[h];
      if (k == -1) {
        k = atomicCAS(&ckey[h], -1, x);
        if (k == -1) k = x;
      }
      if (k == x) {
        atomicAdd(&crow[h][j], c);
        return true;
      }
    }
    return false;
  };
  const int64_t n_own = I.n_own;
  const int64_t wave = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  unsigned int iso_acc = 0;  // lane = view
  for (int64_t b0 = wave * 64; b0 < n_own; b0 += nwaves * 64) {
    const int64_t v = b0 + lane;
    const uint64_t mv = v < n_own ? vm[v] & vmask : 0;
    const uint64_t ad = v < n_own ? vadj[v] : 0;
    const int32_t x = (v < n_own && uw) ? uw_label(uw[v]) : kMixed;
    if (!REMOTE_ONLY) iso_acc += (unsigned)__popcll(transpose64(mv & ~ad, lane));
    const uint64_t m = mv & ad;
    uint64_t todo = __ballot(m != 0 && x != kMixed);
    while (todo) {  // uniform members, grouped by (label, views): lane = view
      const int L = __builtin_ctzll(todo);
      const int32_t xL = __builtin_amdgcn_readlane(x, L);
      const uint64_t mL = rl64(m, L);
      const uint64_t same = __ballot(((todo >> lane) & 1) && x == xL && m == mL);
      todo &= ~same;
      const bool on = (mL >> lane) & 1;
      const unsigned c = (unsigned)__popcll(same);
      const bool hit = on && cached(xL, lane, c);
      count_direct<REMOTE_ONLY>(on && !hit, xL, lane, c, P, I, counts, gcnt, hsbuf, lane, st);
    }
    for (uint64_t mixed = __ballot(m != 0 && x == kMixed); mixed; mixed &= mixed - 1) {  // rows
      const int L = __builtin_ctzll(mixed);
      const uint64_t mL = rl64(m, L);
      const bool on = (mL >> lane) & 1;
      const int32_t l = on ? lab[(b0 + L) * 64 + lane] : 0;
      const bool hit = on && cached(l, lane, 1u);
      count_direct<REMOTE_ONLY>(on && !hit, l, lane, 1u, P, I, counts, gcnt, hsbuf, lane, st);
    }
  }
  for (int h = 0; h < kRows; h++) {  // the wave's cache: owned labels at their rows, the rest as records
    const int32_t k = ckey[h];
    if (k == -1) continue;
    const unsigned int c = crow[h][lane];
    count_direct<REMOTE_ONLY>(c != 0, k, lane, c, P, I, counts, gcnt, hsbuf, lane, st);
  }
  for (int q = 0; q < P.np; q++) stage_flush(st, q, P, gcnt, hsbuf, lane);
  if (!REMOTE_ONLY && iso_acc) atomicAdd(&iso[lane], iso_acc);
  __syncthreads();
  if (!REMOTE_ONLY && threadIdx.x < 64 && iso[threadIdx.x])
    atomicAdd(&iso_g[(blockIdx.x & 63) * 64 + threadIdx.x], iso[threadIdx.x]);
}

// records received from the other partitions: count at the owned label vertex's row
__global__ __launch_bounds__(256) void k_hist_recv(XPeers P, const unsigned long long* __restrict__ rbuf, OwnIdx I,
                                                   int32_t* __restrict__ counts) {
  const int64_t n = P.pre[P.np];
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int q = peer_of(P, i);
    const unsigned long long r = rbuf[P.base[q] + i - P.pre[q]];
    const int32_t L = (int32_t)(r & 0x7fffffffull);
    const int j = (int)((r >> 31) & 63);
    const int32_t c = (int32_t)(r >> 37);
    const int64_t row = label_row(I, L);
    if (row >= 0) atomicAdd(&counts[row * 64 + j], c);
  }
}

// ------------------------------------------------------------------ launchers
static unsigned xgrid(int64_t items, int per_block, unsigned cap = 8192) {
  int64_t g = (items + per_block - 1) / per_block;
  if (g < 1) g = 1;
  return (unsigned)(g > cap ? cap : g);
}
void launch_xvm_pack(hipStream_t s, int64_t nx, const int32_t* xv, const int32_t* xq, const int64_t* xoff, int planes,
                     const uint64_t* vm, int64_t vstride, uint64_t* out) {
  if (nx > 0) k_xvm_pack<<<xgrid(nx, 256), 256, 0, s>>>(nx, xv, xq, xoff, planes, vm, vstride, out);
}
void launch_xvm_unpack(hipStream_t s, int64_t nx, const int32_t* xv, const int32_t* xq, const int64_t* xoff,
                       int planes, const uint64_t* in, uint64_t* vm, int64_t vstride) {
  if (nx > 0) k_xvm_unpack<<<xgrid(nx, 256), 256, 0, s>>>(nx, xv, xq, xoff, planes, in, vm, vstride);
}
void launch_xpack_rec(hipStream_t s, const XPeers& P, const XSend& X, const uint8_t* act, const uint64_t* chg_now,
                      const uint64_t* vadj, const int32_t* lab, const int32_t* uw, XRec* sbuf, unsigned long long* scnt,
                      const int32_t* ccount, int dense_div, int step, int64_t n_own) {
  if (X.nb > 0)
    k_xpack_rec<<<xgrid(X.nb, 4 * 64 * kPackRun, 4096), 256, 0, s>>>(P, X, act, chg_now, vadj, lab, uw, sbuf, scnt, ccount,
                                                           dense_div, step, n_own);
}
XSend build_xsend(hipStream_t s, int64_t n_own, int64_t nx, const int32_t* xv, const int32_t* xq, const int64_t* xoff,
                  std::vector<void*>& T, std::vector<void*>& L) {
  auto alloc = [&](std::vector<void*>& list, size_t bytes) {
    void* p = nullptr;
    if (hipMalloc(&p, std::max<size_t>(bytes, 16)) != hipSuccess) throw std::runtime_error("build_xsend: hipMalloc");
    list.push_back(p);
    return p;
  };
  XSend X;
  if (nx <= 0 || n_own <= 0) return X;
  int32_t* flag = (int32_t*)alloc(T, sizeof(int32_t) * (n_own + 1));
  int32_t* pos = (int32_t*)alloc(T, sizeof(int32_t) * (n_own + 1));
  if (hipMemsetAsync(flag, 0, sizeof(int32_t) * (n_own + 1), s) != hipSuccess) throw std::runtime_error("build_xsend");
  k_xsend_flag<<<xgrid(nx, 256), 256, 0, s>>>(nx, xv, flag);
  size_t tb = 0;
  (void)hipcub::DeviceScan::ExclusiveSum(nullptr, tb, flag, pos, (int)(n_own + 1), s);
  void* tmp = alloc(T, tb);
  if (hipcub::DeviceScan::ExclusiveSum(tmp, tb, flag, pos, (int)(n_own + 1), s) != hipSuccess)
    throw std::runtime_error("build_xsend: scan");
  int32_t nb = 0;
  if (hipMemcpyAsync(&nb, pos + n_own, sizeof(int32_t), hipMemcpyDeviceToHost, s) != hipSuccess ||
      hipStreamSynchronize(s) != hipSuccess)
    throw std::runtime_error("build_xsend: count");
  X.nb = nb;
  int32_t* xb = (int32_t*)alloc(L, sizeof(int32_t) * nb);
  int32_t* xe = (int32_t*)alloc(L, sizeof(int32_t) * nb * kMaxParts);
  uint32_t* pm = (uint32_t*)alloc(L, sizeof(uint32_t) * nb);
  if (hipMemsetAsync(pm, 0, sizeof(uint32_t) * nb, s) != hipSuccess) throw std::runtime_error("build_xsend");
  k_xsend_list<<<xgrid(n_own, 256), 256, 0, s>>>(n_own, flag, pos, xb);
  k_xsend_entries<<<xgrid(nx, 256), 256, 0, s>>>(nx, xv, xq, xoff, pos, xe, pm);
  if (hipGetLastError() != hipSuccess || hipStreamSynchronize(s) != hipSuccess)
    throw std::runtime_error("build_xsend: kernels");
  X.v = xb;
  X.e = xe;
  X.pm = pm;
  return X;
}
void launch_xcounts(hipStream_t s, int np, int me, unsigned long long* scnt, const int32_t* stepflag, int64_t* xa) {
  k_xcounts<<<1, 64, 0, s>>>(np, me, scnt, stepflag, xa);
}
void launch_xclear(hipStream_t s, const XPeers& P, const XRec* rbuf, const int32_t* xrv, uint64_t* chg, int32_t* uw) {
  if (P.pre[P.np] > 0) k_xclear<<<xgrid(P.pre[P.np], 256), 256, 0, s>>>(P, rbuf, xrv, chg, uw);
}
void launch_xunpack_rec(hipStream_t s, const XPeers& P, const XRec* rbuf, const int32_t* xrv, int32_t* lab,
                        uint64_t* chg, int32_t* uw, uint64_t* cb) {
  if (P.pre[P.np] > 0) k_xunpack_rec<<<xgrid(P.pre[P.np], 256), 256, 0, s>>>(P, rbuf, xrv, lab, chg, uw, cb);
}
void launch_xmark(hipStream_t s, const XPeers& P, const XRec* rbuf, const int32_t* xrv, const uint64_t* chg,
                  const DevGraph& g, const uint64_t* vm, const uint64_t* em, uint8_t* act_next, int64_t tcut,
                  const BatchParams* ebp, const int32_t* ccount, int dense_div, int step) {
  if (P.pre[P.np] <= 0) return;
  BatchParams bp0;
  if (!ebp) std::memset(&bp0, 0, sizeof(bp0));
  auto* kern = g.ts_t ? k_xmark<true> : k_xmark<false>;
  kern<<<xgrid(P.pre[P.np], 4), 256, 0, s>>>(P, rbuf, xrv, chg, g.out_off, g.in_off, g.in_eid, g.esrc, g.edst, vm, em,
                                             g.n_seg > 0 ? g.hv_of : nullptr, act_next, g.adj_off, g.ts_e, g.ts_nb,
                                             g.ts_t, tcut, ebp ? *ebp : bp0, ebp ? 1 : 0, ccount, dense_div, step,
                                             g.n_own, g.nv);
}
void launch_part_count(hipStream_t s, bool remote_only, const XPeers& P, const OwnIdx& I, int nviews,
                       const uint64_t* vm, const uint64_t* vadj, const int32_t* uw, const int32_t* lab, int32_t* counts,
                       unsigned int* iso, unsigned long long* gcnt, unsigned long long* hsbuf) {
  const uint64_t vmask = nviews >= 64 ? ~0ull : ((1ull << nviews) - 1);
  const unsigned grid = xgrid(I.n_own, 256, 2048);
  if (remote_only)
    k_part_count<true><<<grid, 256, 0, s>>>(P, I, vmask, vm, vadj, uw, lab, counts, iso, gcnt, hsbuf);
  else
    k_part_count<false><<<grid, 256, 0, s>>>(P, I, vmask, vm, vadj, uw, lab, counts, iso, gcnt, hsbuf);
}
void launch_hist_recv(hipStream_t s, const XPeers& P, const unsigned long long* rbuf, const OwnIdx& I, int32_t* counts) {
  if (P.pre[P.np] > 0) k_hist_recv<<<xgrid(P.pre[P.np], 256), 256, 0, s>>>(P, rbuf, I, counts);
}

}  // namespace rgpu
