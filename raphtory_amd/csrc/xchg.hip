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
  if (id < 0 || id > I.id_max) return -1;  // (the buckets cover [0, id_max])
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

// ------------------------------------------------------------------ label records (broadcast)
// After superstep r every partition broadcasts ONE list of records for its changed boundary
// vertices to all peers (the ReaderWorker's VertexMessage traffic, VertexVisitor.messageAllNeighbours
// :112-120, sent once per vertex instead of once per (vertex, peer)).  A boundary vertex is named by
// its index b in the sender's boundary list (ascending owned rank); a receiver maps (peer q, b) to
// its ghost rank through tab[toff[q] + b] (-1: q's vertex is no ghost here, the record is skipped).
//   U record (8 B): b << 32 | label — a uniform sender (kernels.hpp kMixed) that changed in any
//                   view where it has a kept neighbour: the ghost takes the label as its uniform
//                   word with the changed flag, exactly as a local uniform vertex's word reads
//                   (readers fold a changed uniform neighbour on every kept view of the slot; in
//                   the views where it did not change the label is its current one, so the fold
//                   changes nothing there).
//   M record (16 B, XRec): {b, label, views} per distinct new label of a mixed sender.
// A sender's U records need at most nb slots (one per boundary vertex): U buffers are sized for the
// worst case at plan time and never grow; M records (mixed senders: rare) grow on demand.
// The pack runs in two passes over units (kernels.hpp xbc_units: chunks of 64 consecutive owned
// ranks, the hub chunks split by mixed member; lane = vertex; one word of the step's changed bits
// per chunk, so an unchanged chunk costs one scalar load): the count pass writes each (peer,
// unit)'s U and M record counts (ccnt[q * units + u] = U << 32 | M), a device
// scan turns them into offsets, and the write pass puts the records in peer q's region (U at
// q * ucap, M at q * mcap).  A changed boundary vertex is sent only to the peers in pmask: those
// owning a ghost neighbour across one of its kept slots in the batch (K2) — no other partition's
// vertex reads it in this batch (kept slots are symmetric: both sides compute em & vm & vm).  No
// shared counter: one atomic per wave on a single address serialised at the memory side
// (DESIGN.md §4 lesson 1).  A mixed sender's distinct labels are found on its row (lane = view);
// rows of up to kRowsInFlight senders are loaded before any is folded.
constexpr int kRowsInFlight = 4;
__device__ __forceinline__ int distinct_labels(int32_t x, uint64_t mm, int lane) {
  int k = 0;
  while (mm) {
    const int32_t val = __builtin_amdgcn_readlane(x, __builtin_ctzll(mm));
    mm &= ~__ballot(((mm >> lane) & 1) && x == val);
    k++;
  }
  return k;
}
__device__ __forceinline__ int64_t bc_total(const XBcIn& I);
__device__ __forceinline__ int32_t bc_rec(const XBcIn& I, int64_t i, int32_t& b, int32_t& val, uint64_t& mask, bool& isu,
                                          bool& first, int64_t* mj, int64_t* mend);
template <bool WRITE>
__global__ __launch_bounds__(256) void k_xbc_pack(int64_t n_own, int np, const int32_t* __restrict__ bidx,
                                                  const uint64_t* __restrict__ cb_now,
                                                  const uint64_t* __restrict__ chg_now,
                                                  const uint64_t* __restrict__ vadj, const int32_t* __restrict__ lab,
                                                  const int32_t* __restrict__ uw, const uint8_t* __restrict__ pmask,
                                                  unsigned long long* __restrict__ su, int64_t ucap,
                                                  XRec* __restrict__ sm, int64_t mcap,
                                                  unsigned long long* __restrict__ ccnt,
                                                  const unsigned long long* __restrict__ coff, XBcIn CI, int do_clear,
                                                  uint64_t* __restrict__ cchg, int32_t* __restrict__ cuw) {
  // (the count pass also clears the ghosts that step r-2's records set: k_xbc_clear folded in, one
  // launch less per superstep — the pack runs after step r-1 read those words, before step r's apply)
  if (!WRITE && do_clear) {
    const int64_t nc = bc_total(CI);
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < nc; i += (int64_t)gridDim.x * blockDim.x) {
      int32_t b, val;
      uint64_t mask;
      bool isu, first;
      const int32_t g = bc_rec(CI, i, b, val, mask, isu, first, nullptr, nullptr);
      if (g < 0) continue;
      if (!isu) cchg[g] = 0;
      cuw[g] = kGhostQuiet;
    }
  }
  const int lane = lane_of();
  const int64_t wave = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  const int64_t nch = (n_own + 63) >> 6, nun = xbc_units(n_own);
  for (int64_t un = wave; un < nun; un += nwaves) {
    int sub;
    const int64_t c = unit_chunk(un, nch, sub);
    const uint64_t w = cb_now[c];  // (wave-uniform: a scalar load)
    if (w == 0) {
      if (!WRITE && lane < np) ccnt[(int64_t)lane * nun + un] = 0;
      continue;
    }
    const int64_t v = c * 64 + lane;
    const bool ch = ((w >> lane) & 1) && v < n_own;
    const int32_t b = ch ? bidx[v] : -1;
    const uint64_t m = b >= 0 ? chg_now[v] & vadj[v] : 0;
    const uint32_t pm = m ? pmask[v] : 0u;
    const int32_t u = pm ? uw_label(uw[v]) : kMixed;
    const bool full = pm != 0 && u != kMixed && sub <= 0;  // a uniform sender: one U record per peer in pm
    const uint64_t mixed0 = split_rows(__ballot(pm != 0 && u == kMixed), sub);
    if constexpr (!WRITE) {
      unsigned long long nm = 0;  // lane q: M records for peer q
      for (uint64_t mixed = mixed0; mixed;) {
        int Ls[kRowsInFlight];
        int32_t x[kRowsInFlight];
        int k = 0;
        for (; k < kRowsInFlight && mixed; k++, mixed &= mixed - 1) Ls[k] = __builtin_ctzll(mixed);
        for (int i = 0; i < k; i++) x[i] = lab[(c * 64 + Ls[i]) * 64 + lane];
        for (int i = 0; i < k; i++) {
          const int d = distinct_labels(x[i], rl64(m, Ls[i]), lane);
          const uint32_t pL = (uint32_t)__builtin_amdgcn_readlane((int)pm, Ls[i]);
          if (lane < np && ((pL >> lane) & 1)) nm += (unsigned long long)d;
        }
      }
      unsigned long long nu = 0;
      for (int q = 0; q < np; q++) {
        const unsigned long long cq = (unsigned long long)__popcll(__ballot(full && ((pm >> q) & 1)));
        if (lane == q) nu = cq;
      }
      if (lane < np) ccnt[(int64_t)lane * nun + un] = (nu << 32) | nm;
    } else {
      unsigned long long uo = 0, mo = 0;  // lane q: peer q's offsets in its regions
      if (lane < np) {
        const unsigned long long o = coff[(int64_t)lane * nun + un], o0 = coff[(int64_t)lane * nun];
        uo = (o >> 32) - (o0 >> 32);
        mo = (o & 0xffffffffull) - (o0 & 0xffffffffull);
      }
      for (int q = 0; q < np; q++) {
        const bool mine = full && ((pm >> q) & 1);
        const uint64_t bu = __ballot(mine);
        if (!bu) continue;
        const unsigned long long base = (unsigned long long)__builtin_amdgcn_readlane((int)(uint32_t)uo, q);
        if (mine)
          su[(int64_t)q * ucap + (int64_t)(base + __popcll(bu & lanemask_below(lane)))] =
              ((unsigned long long)(uint32_t)b << 32) | (uint32_t)u;
      }
      for (uint64_t mixed = mixed0; mixed;) {
        int Ls[kRowsInFlight];
        int32_t x[kRowsInFlight];
        int k = 0;
        for (; k < kRowsInFlight && mixed; k++, mixed &= mixed - 1) Ls[k] = __builtin_ctzll(mixed);
        for (int i = 0; i < k; i++) x[i] = lab[(c * 64 + Ls[i]) * 64 + lane];
        for (int i = 0; i < k; i++) {
          const uint64_t mL = rl64(m, Ls[i]);
          const int32_t bL = __builtin_amdgcn_readlane(b, Ls[i]);
          const uint32_t pL = (uint32_t)__builtin_amdgcn_readlane((int)pm, Ls[i]);
          for (uint64_t mm = mL; mm;) {
            const int32_t val = __builtin_amdgcn_readlane(x[i], __builtin_ctzll(mm));
            const uint64_t same = __ballot(((mm >> lane) & 1) && x[i] == val);
            mm &= ~same;
            // lane q < np writes peer q's copy
            if (lane < np && ((pL >> lane) & 1)) {
              if (mo < (unsigned long long)mcap) sm[(int64_t)lane * mcap + (int64_t)mo] = XRec{bL, val, same};
              mo++;
            }
          }
        }
      }
    }
  }
}

// ------------------------------------------------------------------ send index (per boundary vertex)
__global__ __launch_bounds__(256) void k_xsend_flag(int64_t nx, const int32_t* __restrict__ xv,
                                                    int32_t* __restrict__ flag) {
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < nx; e += (int64_t)gridDim.x * blockDim.x)
    flag[xv[e]] = 1;  // (idempotent plain stores)
}
__global__ __launch_bounds__(256) void k_xsend_list(int64_t n_own, const int32_t* __restrict__ flag,
                                                    const int32_t* __restrict__ pos, int32_t* __restrict__ xb,
                                                    int32_t* __restrict__ bidx) {
  for (int64_t v = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; v < n_own; v += (int64_t)gridDim.x * blockDim.x) {
    const bool f = flag[v] != 0;
    if (f) xb[pos[v]] = (int32_t)v;
    bidx[v] = f ? pos[v] : -1;
  }
}
__global__ __launch_bounds__(256) void k_xsend_entries(int64_t nx, const int32_t* __restrict__ xv,
                                                       const int32_t* __restrict__ pos, int32_t* __restrict__ eb) {
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < nx; e += (int64_t)gridDim.x * blockDim.x)
    eb[e] = pos[xv[e]];
}
// receive tables: peer q's boundary index of receive entry i (tmp) -> the ghost rank it names
__global__ __launch_bounds__(256) void k_xtab_fill(int64_t n, const int32_t* __restrict__ xr_v,
                                                   const int32_t* __restrict__ xr_q, const int32_t* __restrict__ tmp,
                                                   XTab T, unsigned long long* __restrict__ err) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int q = xr_q[i];
    const int32_t b = tmp[i];
    if (b < 0 || (int64_t)b >= T.toff[q + 1] - T.toff[q]) {
      atomicAdd(err, 1ull);
      continue;
    }
    T.tab[T.toff[q] + b] = xr_v[i];
  }
}

// counts exchange words, 4 per peer: [4q] U records for q, [4q+1] M records for q (0 for self),
// [4q+2] this partition changed a label in the step (the halting vote, AnalysisTask.endStep
// :208-225), [4q+3] 0.  coff = the pack's scanned per-(peer, chunk) offsets (null: no records).
__global__ void k_xbc_counts(int np, int me, const unsigned long long* __restrict__ coff, int64_t nun,
                             const int32_t* __restrict__ stepflag, int64_t* __restrict__ xa) {
  const int q = threadIdx.x;
  if (q < np) {
    unsigned long long t = 0;
    if (coff && q != me) t = coff[(int64_t)(q + 1) * nun] - coff[(int64_t)q * nun];
    xa[4 * q] = (int64_t)(t >> 32);
    xa[4 * q + 1] = (int64_t)(t & 0xffffffffull);
    xa[4 * q + 2] = stepflag ? (stepflag[0] != 0) : 0;
    xa[4 * q + 3] = 0;
  }
}
// component-count records (one region per peer): [2q] = records for q, [2q+1] = 0
__global__ void k_xcounts(int np, int me, unsigned long long* __restrict__ scnt, int64_t* __restrict__ xa) {
  const int q = threadIdx.x;
  if (q >= np) return;
  xa[2 * q] = q == me ? 0 : (int64_t)scnt[q];
  xa[2 * q + 1] = 0;
  scnt[q] = 0;
}

// M records received in a superstep from which the record apply goes per ghost (k_xbc_apply phase 1)
constexpr int64_t kMGhostMin = 32768;
// lanes (views) of the 64-B lines of a row (16 lanes each) that hold at least one view of m
__device__ __forceinline__ bool line_of(uint64_t m, int lane) { return ((m >> (lane & 48)) & 0xffffull) != 0; }

// record i of a received broadcast (U records of every peer, then M records of every peer, XBcIn)
// -> the ghost it names (-1: none here; out-of-plan records are counted into err and skipped — a
// bug upstream, reported by the run instead of faulting the device)
__device__ __forceinline__ int64_t bc_total(const XBcIn& I) { return I.U.pre[I.U.np] + I.M.pre[I.M.np]; }
// (b, label, views, is_u) of record i and the ghost it names; for an M record also its index in rm
// and the end of its sender's region (mj, mend; -1 for a U record)
__device__ __forceinline__ int32_t bc_rec(const XBcIn& I, int64_t i, int32_t& b, int32_t& val, uint64_t& mask, bool& isu,
                                          bool& first, int64_t* mj, int64_t* mend) {
  const int64_t nu = I.U.pre[I.U.np];
  int q;
  first = true;
  if (i < nu) {
    q = peer_of(I.U, i);
    const unsigned long long r = I.ru[I.U.base[q] + i - I.U.pre[q]];
    b = (int32_t)(r >> 32);
    val = (int32_t)(uint32_t)r;
    mask = ~0ull;
    isu = true;
    if (mj) *mj = *mend = -1;
  } else {
    const int64_t k = i - nu;
    q = peer_of(I.M, k);
    const int64_t j = I.M.base[q] + k - I.M.pre[q];
    const XRec r = I.rm[j];
    b = r.e;
    val = r.val;
    mask = r.mask;
    isu = false;
    first = k == I.M.pre[q] || I.rm[j - 1].e != b;  // a mixed sender's records are consecutive
    if (mj) {
      *mj = j;
      *mend = I.M.base[q] + (I.M.pre[q + 1] - I.M.pre[q]);
    }
  }
  if (b < 0 || (int64_t)b >= I.T.toff[q + 1] - I.T.toff[q]) {
    atomicAdd(I.err, 1ull);
    return -1;
  }
  const int32_t g = I.T.tab[I.T.toff[q] + b];
  if (g >= 0 && (g < I.n_own || g >= I.nv)) {
    atomicAdd(I.err, 1ull);
    return -1;
  }
  return g;
}

// ghosts whose words records of two supersteps ago set: uniform word back to kGhostQuiet, and for
// an M record the change word cleared in that parity (a U record writes no change word)
__global__ __launch_bounds__(256) void k_xbc_clear(XBcIn I, uint64_t* __restrict__ chg, int32_t* __restrict__ uw) {
  const int64_t n = bc_total(I);
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    int32_t b, val;
    uint64_t mask;
    bool isu, first;
    const int32_t g = bc_rec(I, i, b, val, mask, isu, first, nullptr, nullptr);
    if (g < 0) continue;
    if (!isu) chg[g] = 0;
    uw[g] = kGhostQuiet;
  }
}

// A superstep's received records applied and their ghosts' neighbours marked, in one pass (lane =
// record).  Apply: a U record's ghost takes the label as its uniform word with the changed flag (a
// plain store: a ghost has one sender and a U sender sends one record; no change word — readers of
// a changed uniform word fold it on every kept view of the slot, and hub marking reads the word);
// M records mark the ghost mixed (kMixed), write the label into the row lanes of their views and OR
// the views into its change word (one per wave iteration, lane = view).  Mark: every changed ghost
// (a U record, or the first M record of its sender with the union of the sender's masks) flags its
// owned neighbours that share a changed view (the next frontier, as a local change would).  Ghosts
// keep no compacted slots (K2 runs over the owned vertices only): the kept views of a static slot,
// bits & vm[nb] & vm[g], are recomputed over the time-ordered slots up to the batch's cut (bits:
// K2's inline edge bits for a simple slot, else em[e]; without time-ordered slots the CSR order and
// em).  A ghost holds only its edges to this partition's vertices (a few slots), so the wave packs
// its records' ghosts' slot lists into 64-lane passes (lane = slot), as K2 packs its light members;
// ghosts with more than 64 static slots walk theirs one at a time.  Nothing to mark when superstep
// r is dense (the next one visits every member).  Heavy ghosts: k_heavy_mark.
template <bool TS>
__device__ __forceinline__ void mark_slot(int64_t p, int32_t g, uint64_t ch, const int64_t* __restrict__ ts_t,
                                          const int32_t* __restrict__ ts_nb, const int32_t* __restrict__ ts_e,
                                          int64_t tcut, const HopLDS& L, const BatchParams& ebp, int iem,
                                          const uint64_t* __restrict__ vm, const uint64_t* __restrict__ em,
                                          uint8_t* __restrict__ act_next) {
  const int64_t tsw = ts_t[p];
  if (ts_time(tsw) < tcut) return;
  const int32_t nb = ts_nb[p];
  if (nb == g) return;
  // (a nodeath slot with ebp.simple_ends: its bits imply nb's membership, BatchParams::simple_ends)
  const uint64_t bits = (iem && ts_simple(tsw)) ? simple_bits(L, ebp.sorted, ts_time(tsw)) : em[ts_e[p]];
  if (bits & ch & ((iem && ebp.simple_ends && ts_nodeath(tsw)) ? ~0ull : vm[nb])) act_next[nb] = 1;
}
// Per batch: the number of each ghost's time-ordered static slots at or after the batch's cut (the
// slots are newest first, so the ones older than the cut are a suffix, dead in every view of the
// batch).  A ghost's records then walk only that prefix: in a short window most ghosts with more than
// 64 static slots keep a few, so they pack into the lane = slot passes with the others instead of
// taking the wave one at a time (P = 8, hour batches: ~280 us per record apply before).
__global__ __launch_bounds__(256) void k_ghost_cut(int64_t n_own, int64_t nv, const int64_t* __restrict__ adj_off,
                                                   const int64_t* __restrict__ ts_t, int64_t tcut,
                                                   int32_t* __restrict__ gcut) {
  for (int64_t g = n_own + blockIdx.x * (int64_t)blockDim.x + threadIdx.x; g < nv; g += (int64_t)gridDim.x * blockDim.x) {
    const int64_t lo = adj_off[g];
    int64_t a = lo, b = adj_off[g + 1];
    while (a < b) {  // first slot older than the cut
      const int64_t m = (a + b) >> 1;
      if (ts_time(ts_t[m]) >= tcut) a = m + 1; else b = m;
    }
    gcut[g] = (int32_t)(a - lo);
  }
}

template <bool TS>
__global__ __launch_bounds__(256) void k_xbc_apply(XBcIn I, int32_t* __restrict__ lab, uint64_t* __restrict__ chg,
                                                   int32_t* __restrict__ uw, uint64_t* __restrict__ cb,
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
                                                   const int32_t* __restrict__ gcut, int phase) {
  // phase 0: the U records (apply + mark); phase 1 (a second launch, only when M records arrived): the
  // M records, one ghost at a time per wave.  A ghost has one owner, so one sender, whose records for
  // it are consecutive and at most 64 (one per distinct label of its views): the wave loads them lane
  // = record, forms the ghost's new row lane = view and stores it in whole 64-B lines over the old
  // row, sets its words once (no atomics on its change word), and its marking uses the union of the
  // views.  Before, every M record wrote its row lanes as single 4-B stores (each a partial-line fill)
  // and ORed its views with atomics, and the marking lane walked the sender's further records one
  // dependent load at a time: ~300 us per apply in the P = 8 hour batches (297k M records a step).
  const bool do_mark = !dense_after(ccount, step + 1, I.n_own, dense_div);  // step r dense: r+1 visits every member
  __shared__ HopLDS L;
  if (TS && iem) hop_lds_init(L, ebp, ebp.thr_e);
  // phase 0 walks the U records, phase 1 the M records (bc_rec: U records first, then M); phase 2 (few
  // M records: the per-ghost loop would serialise a wave's ghosts) walks all of them per lane
  const int64_t nu = I.U.pre[I.U.np];
  const int64_t i0 = phase == 1 ? nu : 0, n = phase == 0 ? nu : phase == 1 ? I.M.pre[I.M.np] : nu + I.M.pre[I.M.np];
  const int lane = lane_of();
  const int64_t wave = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  // records -> lanes: groups of 8 consecutive records (one 64-B line of U records), a wave's 8
  // groups 1/8 of the records apart.  A sender's records are in its rank order, so its hubs come
  // first, and their ghosts here are the ones with the most slots to walk: consecutive records in a
  // wave put up to 64 of those walks on one wave (one at a time, ~4 us each: the launch), spread
  // records put a few on each.
  const int64_t ncw = (n + 63) >> 6;  // chunk-waves
  for (int64_t cw = wave; cw < ncw; cw += nwaves) {
    const int64_t i = (((int64_t)(lane >> 3) * ncw + cw) << 3) + (lane & 7);
    int32_t b = 0, val = 0, g = -1;
    uint64_t mask = 0;
    bool isu = false, first = false;
    int64_t mj = -1, mend = -1;
    if (i < n) g = bc_rec(I, i0 + i, b, val, mask, isu, first, &mj, &mend);
    uint64_t chv = 0;  // phase 1, a ghost's first M record: the views its records changed
    if (phase != 1) {  // (wave-uniform) U records
      if (g >= 0 && isu) {
        uw[g] = uw_word(val, true);
        if (cb) atomicOr((unsigned long long*)&cb[g >> 6], 1ull << (g & 63));  // (ChgBits)
      }
    }
    if (phase == 2) {  // M records per lane: row lanes as single stores, views ORed with atomics
      const bool mrec = g >= 0 && !isu;
      const bool wide = mrec && __popcll(mask) > 8;
      if (mrec) {
        uw[g] = kMixed;
        atomicOr((unsigned long long*)&chg[g], (unsigned long long)mask);
        if (cb) atomicOr((unsigned long long*)&cb[g >> 6], 1ull << (g & 63));
        if (!wide)
          for (uint64_t mm = mask; mm; mm &= mm - 1) lab[(int64_t)g * 64 + __builtin_ctzll(mm)] = val;
      }
      for (uint64_t bb = __ballot(wide); bb; bb &= bb - 1) {
        const int L = __builtin_ctzll(bb);
        const int32_t gL = __builtin_amdgcn_readlane(g, L);
        const int32_t vL = __builtin_amdgcn_readlane(val, L);
        const uint64_t mL = rl64(mask, L);
        if ((mL >> lane) & 1) lab[(int64_t)gL * 64 + lane] = vL;
      }
      if (g >= 0 && !isu && first) {  // the marking lane: the union of its sender's records
        chv = mask;
        for (int64_t j = mj + 1; j < mend && I.rm[j].e == b; j++) chv |= I.rm[j].mask;
      }
    }
    if (phase == 1) {  // M records: per ghost (its sender's run of records), lane = record, then lane = view
      for (uint64_t t = __ballot(g >= 0 && !isu && first); t; t &= t - 1) {
        const int L = __builtin_ctzll(t);
        const int32_t gL = __builtin_amdgcn_readlane(g, L), bL = __builtin_amdgcn_readlane(b, L);
        const int64_t j0 = (int64_t)rl64((uint64_t)mj, L), je = (int64_t)rl64((uint64_t)mend, L);
        const int64_t jj = j0 + lane;
        XRec rr{-1, 0, 0};
        if (jj < je) rr = I.rm[jj];
        const uint64_t run = __ballot(jj < je && rr.e == bL);  // (a prefix: the sender's records are consecutive)
        const uint64_t sel = run == ~0ull ? ~0ull : ((1ull << __builtin_ctzll(~run)) - 1);
        int32_t nv_ = 0;
        uint64_t uni = 0;
        for (uint64_t rs = sel; rs; rs &= rs - 1) {
          const int R = __builtin_ctzll(rs);
          const uint64_t mR = rl64(rr.mask, R);
          uni |= mR;
          if ((mR >> lane) & 1) nv_ = __builtin_amdgcn_readlane(rr.val, R);
        }
        int32_t* row = lab + (int64_t)gL * 64;
        const int32_t old = row[lane];
        if (line_of(uni, lane)) row[lane] = ((uni >> lane) & 1) ? nv_ : old;
        if (lane == 0) {
          uw[gL] = kMixed;
          chg[gL] = uni;  // (the parity's clear left it 0: this step's views only)
          if (cb) atomicOr((unsigned long long*)&cb[gL >> 6], 1ull << (gL & 63));
        }
        if (lane == L) chv = uni;
      }
    }
    if (!do_mark) continue;
    // mark: lane = record, its ghost when it is the ghost's first record and the ghost is no hub (U
    // records in phase 0, M records in phase 1)
    const bool go = g >= 0 && first && (phase == 2 || isu == (phase == 0)) && !(hv_of && hv_of[g] >= 0);
    uint64_t ch = 0;
    int64_t a = 0;
    int32_t k = 0;
    if (go) {
      const uint64_t views = isu ? mask : chv;  // U: every view; M: the union of its records
      ch = views & vm[g];
      if (TS) {
        a = adj_off[g];
        k = gcut ? gcut[g] : (int32_t)(adj_off[g + 1] - a);  // (the slots at or after the cut, k_ghost_cut)
      } else {
        a = out_off[g];
        k = (int32_t)((out_off[g + 1] - a) + (in_off[g + 1] - in_off[g]));
      }
      if (ch == 0) k = 0;
    }
    if (!TS) {  // CSR order (no time-ordered slots): one ghost at a time, lane = slot
      for (uint64_t t = __ballot(k > 0); t; t &= t - 1) {
        const int Lg = __builtin_ctzll(t);
        const int32_t gL = __builtin_amdgcn_readlane(g, Lg);
        const uint64_t chL = rl64(ch, Lg);
        const int64_t o0 = out_off[gL], i0e = in_off[gL];
        const int64_t nout = out_off[gL + 1] - o0, ntot = nout + (in_off[gL + 1] - i0e);
        for (int64_t c = 0; c < ntot; c += 64) {
          const int64_t j = c + lane;
          if (j >= ntot) continue;
          int64_t e;
          int32_t nb;
          if (j < nout) { e = o0 + j; nb = edst[e]; }
          else { e = in_eid[i0e + (j - nout)]; nb = esrc[e]; }
          if (nb != gL && (em[e] & vm[nb] & chL)) act_next[nb] = 1;
        }
      }
      continue;
    }
    // ghosts with more than 64 static slots: one at a time (newest first: stop at the cut)
    for (uint64_t t = __ballot(k > 64); t; t &= t - 1) {
      const int Lg = __builtin_ctzll(t);
      const int32_t gL = __builtin_amdgcn_readlane(g, Lg);
      const uint64_t chL = rl64(ch, Lg);
      const int64_t aL = (int64_t)rl64((uint64_t)a, Lg);
      const int32_t kL = __builtin_amdgcn_readlane(k, Lg);
      for (int32_t c = 0; c < kL; c += 64) {
        if (ts_time(ts_t[aL + c]) < tcut) break;
        if (c + lane < kL) mark_slot<TS>(aL + c + lane, gL, chL, ts_t, ts_nb, ts_e, tcut, L, ebp, iem, vm, em, act_next);
      }
    }
    // the others packed, lane = slot
    uint64_t pend = __ballot(k > 0 && k <= 64);
    while (pend) {
      int sum = 0, myL = 0, myj = 0;
      while (pend) {
        const int Lp = __builtin_ctzll(pend);
        const int kk = __builtin_amdgcn_readlane(k, Lp);
        if (sum && sum + kk > 64) break;
        if (lane >= sum && lane < sum + kk) { myL = Lp; myj = lane - sum; }
        sum += kk;
        pend &= pend - 1;
      }
      const int64_t aL = (int64_t)(((uint64_t)(uint32_t)__shfl((int)((uint64_t)a >> 32), myL) << 32) |
                                   (uint32_t)__shfl((int)a, myL));
      const uint64_t chL = ((uint64_t)(uint32_t)__shfl((int)(ch >> 32), myL) << 32) | (uint32_t)__shfl((int)ch, myL);
      const int32_t gL = __shfl(g, myL);
      if (lane < sum) mark_slot<TS>(aL + myj, gL, chL, ts_t, ts_nb, ts_e, tcut, L, ebp, iem, vm, em, act_next);
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
// count row (local rank) of label x, which getPartition places here.  A label is a member's id, so
// the lookup always finds it; a miss (id out of the buckets' range, or absent) is counted into
// I.err, and the run fails after its last collective instead of dropping the count.
__device__ __forceinline__ int64_t label_row(const OwnIdx& I, int32_t x) {
  const int64_t k = owned_rank(I, x);
  if (k < 0) {
    if (I.err) atomicAdd(I.err, 1ull);
    return -1;
  }
  return I.pos ? (int64_t)I.pos[k] : k;
}
// Count records are XRec {label, count, views}: `count` members carry `label` in every view of
// `views`.  A uniform member group (the same label over the same views, kernels.hip k_cc_count)
// whose label is remote is ONE record for all its views instead of one 8-B record per view, so a
// small component that lives through many hops of a long window costs one record per group.
// A wave's outgoing records are staged in LDS, kStage per peer, and reserved in the send buffer
// with one atomicAdd per flush: one global atomic per (group of records, peer) serialised on the
// gcnt words (~10 ns each at the memory side, DESIGN.md §4 lesson 1).  The flush order is fixed per
// wave, so a REMOTE_ONLY re-run emits the same records per peer (in another order at most).
constexpr int kStage = 32;
struct CountStage {
  XRec (*rec)[kStage];  // [peer][kStage], wave-private LDS
  int n;                // lane q: records staged for peer q (a register, not LDS: the lanes read it
                        // right after another lane's update)
};
// wave-uniform: reserve peer q's staged records in the send buffer and write them out
__device__ __forceinline__ void stage_flush(CountStage& st, int q, const XPeers& P,
                                            unsigned long long* __restrict__ gcnt, XRec* __restrict__ hsbuf,
                                            int lane) {
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
// wave-uniform (x, views, c): added at the count row when x is owned here, else one staged record.
// row: x's count row when the caller looked it up already (the lanes' lookups run in parallel
// before the serial group loops: a lookup is two dependent global loads), else -2
template <bool REMOTE_ONLY>
__device__ __forceinline__ void emit_count(int32_t x, uint64_t views, unsigned c, const XPeers& P, const OwnIdx& I,
                                           int32_t* __restrict__ counts, unsigned long long* __restrict__ gcnt,
                                           XRec* __restrict__ hsbuf, int lane, CountStage& st, int64_t row = -2) {
  if (views == 0 || c == 0) return;
  const int q = owner_of(x, P.np);
  if (q == P.me) {
    if (!REMOTE_ONLY) {
      const int64_t r = row != -2 ? row : label_row(I, x);  // (a miss is counted into I.err)
      if (r >= 0 && ((views >> lane) & 1)) atomicAdd(&counts[r * 64 + lane], (int32_t)c);
    }
    return;
  }
  if (__builtin_amdgcn_readlane(st.n, q) + 1 > kStage) stage_flush(st, q, P, gcnt, hsbuf, lane);
  const int c0 = __builtin_amdgcn_readlane(st.n, q);
  if (lane == 0) st.rec[q][c0] = XRec{x, (int32_t)c, views};
  if (lane == q) st.n = c0 + 1;
}
// per lane (lane = view) label l with count c on the lanes of `on`: grouped by (label, count); the
// lanes look their owned labels' rows up first, in parallel
template <bool REMOTE_ONLY>
__device__ __forceinline__ void emit_lanes(bool on, int32_t l, unsigned c, const XPeers& P, const OwnIdx& I,
                                           int32_t* __restrict__ counts, unsigned long long* __restrict__ gcnt,
                                           XRec* __restrict__ hsbuf, int lane, CountStage& st) {
  const int64_t rl = (!REMOTE_ONLY && on && owner_of(l, P.np) == P.me) ? label_row(I, l) : -1;
  for (uint64_t rest = __ballot(on); rest;) {
    const int L = __builtin_ctzll(rest);
    const int32_t xL = __builtin_amdgcn_readlane(l, L);
    const unsigned cL = (unsigned)__builtin_amdgcn_readlane((int)c, L);
    const uint64_t same = __ballot(((rest >> lane) & 1) && l == xL && c == cL);
    rest &= ~same;
    emit_count<REMOTE_ONLY>(xL, same, cL, P, I, counts, gcnt, hsbuf, lane, st, (int64_t)rl64((uint64_t)rl, L));
  }
}
template <bool REMOTE_ONLY>
__global__ __launch_bounds__(256) void k_part_count(XPeers P, OwnIdx I, uint64_t vmask, const uint64_t* __restrict__ vm,
                                                    const uint64_t* __restrict__ vadj, const int32_t* __restrict__ uw,
                                                    const int32_t* __restrict__ lab, int32_t* __restrict__ counts,
                                                    unsigned int* __restrict__ iso_g,
                                                    unsigned long long* __restrict__ gcnt, XRec* __restrict__ hsbuf,
                                                    const int32_t* __restrict__ mneg, unsigned int* __restrict__ fin_g) {
  // The cache is private to a wave (16 rows each): a wave's operations run in a fixed order, so
  // the records it emits are the same on every run — the REMOTE_ONLY pass after a send-buffer
  // overflow must emit exactly the records the counts exchange announced.
  constexpr int kRows = 16;
  __shared__ unsigned int iso[64];
  __shared__ unsigned int fin[64];
  __shared__ int32_t ckey_s[4][kRows];
  __shared__ unsigned int crow_s[4][kRows][64];
  __shared__ XRec srec_s[4][kMaxParts][kStage];
  const int lane = lane_of(), wib = threadIdx.x >> 6;
  int32_t* ckey = ckey_s[wib];
  unsigned int (*crow)[64] = crow_s[wib];
  CountStage st{srec_s[wib], 0};
  if (threadIdx.x < 64) iso[threadIdx.x] = 0, fin[threadIdx.x] = 0;
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
  // The view's global minimum member label (part_min_labels) is very likely its giant component,
  // whose members sit on every partition: they are counted here per view (fin_acc) and summed over
  // the partitions by an all-reduce (launch_min_count) instead of records that all converge on one
  // count row of one partition.
  int32_t mfin = INT32_MIN;
  if (mneg) {
    int32_t x = 0;
    for (int sh = 0; sh < kMinShards; sh++) x = max(x, mneg[sh * 64 + lane]);
    mfin = x ? INT32_MAX - x : INT32_MIN;
  }
  unsigned int fin_acc = 0;
  // units (kernels.hpp xbc_units): a hub chunk's mixed members are split over kSplitWays waves
  const int64_t nch = (n_own + 63) >> 6, nun = xbc_units(n_own);
  for (int64_t un = wave; un < nun; un += nwaves) {
    int sub;
    const int64_t b0 = unit_chunk(un, nch, sub) * 64;
    const int64_t v = b0 + lane;
    const uint64_t mv = v < n_own ? vm[v] & vmask : 0;
    const uint64_t ad = v < n_own ? vadj[v] : 0;
    const int32_t x = (v < n_own && uw) ? uw_label(uw[v]) : kMixed;
    if (!REMOTE_ONLY && sub <= 0) iso_acc += (unsigned)__popcll(transpose64(mv & ~ad, lane));
    const uint64_t m = mv & ad;
    uint64_t todo = __ballot(m != 0 && x != kMixed && sub <= 0);
    // the lanes' owned labels' count rows, looked up in parallel before the group loop
    const int64_t rx = (!REMOTE_ONLY && sub <= 0 && m != 0 && x != kMixed && owner_of(x, P.np) == P.me)
                           ? label_row(I, x)
                           : -1;
    while (todo) {  // uniform members, grouped by (label, views): lane = view
      const int L = __builtin_ctzll(todo);
      const int32_t xL = __builtin_amdgcn_readlane(x, L);
      const uint64_t mL = rl64(m, L);
      const uint64_t same = __ballot(((todo >> lane) & 1) && x == xL && m == mL);
      todo &= ~same;
      const bool fl = ((mL >> lane) & 1) && xL == mfin;
      const bool on = ((mL >> lane) & 1) && !fl;
      const unsigned c = (unsigned)__popcll(same);
      if (fl) fin_acc += c;
      const bool hit = on && cached(xL, lane, c);
      emit_count<REMOTE_ONLY>(xL, __ballot(on && !hit), c, P, I, counts, gcnt, hsbuf, lane, st,
                              (int64_t)rl64((uint64_t)rx, L));
    }
    for (uint64_t mixed = split_rows(__ballot(m != 0 && x == kMixed), sub); mixed; mixed &= mixed - 1) {  // rows
      const int L = __builtin_ctzll(mixed);
      const uint64_t mL = rl64(m, L);
      const bool mem = (mL >> lane) & 1;
      const int32_t l = mem ? lab[(b0 + L) * 64 + lane] : 0;
      const bool fl = mem && l == mfin;
      const bool on = mem && !fl;
      if (fl) fin_acc += 1u;
      const bool hit = on && cached(l, lane, 1u);
      emit_lanes<REMOTE_ONLY>(on && !hit, l, 1u, P, I, counts, gcnt, hsbuf, lane, st);
    }
  }
  // the wave's cache: owned labels at their rows (looked up in parallel, lane h), the rest as records
  const int32_t kl = lane < kRows ? ckey[lane] : -1;
  const int64_t rk = (!REMOTE_ONLY && kl != -1 && owner_of(kl, P.np) == P.me) ? label_row(I, kl) : -1;
  for (int h = 0; h < kRows; h++) {
    const int32_t k = ckey[h];
    if (k == -1) continue;
    const unsigned int c = crow[h][lane];
    if (owner_of(k, P.np) == P.me) {
      const int64_t r = (int64_t)rl64((uint64_t)rk, h);
      if (!REMOTE_ONLY && r >= 0 && c) atomicAdd(&counts[r * 64 + lane], (int32_t)c);
      continue;
    }
    emit_lanes<REMOTE_ONLY>(c != 0, k, c, P, I, counts, gcnt, hsbuf, lane, st);
  }
  for (int q = 0; q < P.np; q++) stage_flush(st, q, P, gcnt, hsbuf, lane);
  if (!REMOTE_ONLY && iso_acc) atomicAdd(&iso[lane], iso_acc);
  if (!REMOTE_ONLY && fin_acc) atomicAdd(&fin[lane], fin_acc);
  __syncthreads();
  if (!REMOTE_ONLY && threadIdx.x < 64 && iso[threadIdx.x])
    atomicAdd(&iso_g[(blockIdx.x & 63) * 64 + threadIdx.x], iso[threadIdx.x]);
  if (!REMOTE_ONLY && fin_g && threadIdx.x < 64 && fin[threadIdx.x])
    atomicAdd(&fin_g[(blockIdx.x & 63) * 64 + threadIdx.x], fin[threadIdx.x]);
}

// records received from the other partitions: counted at the owned label vertex's row (lane =
// record for the lookups, then lane = view per record).  A label whose members sit on every
// partition (a big component that is not its views' minimum label, k_part_count fin_acc) arrives
// as records from every wave of every sender, all for one count row: a wave folds its records'
// counts in a private LDS cache keyed by row first (16 rows), so a hot row costs one global atomic
// per (wave, view) instead of one per record and view (the per-address atomics serialise at the
// memory side: 2-5 ms per batch on the owner before, profiles/r04/part_sim_p8_hist_trace.txt).
// One chunk of 64 records per wave: the lookups are dependent loads, and chunks walked in turn by
// one wave serialise them.
__global__ __launch_bounds__(256) void k_hist_recv(XPeers P, const XRec* __restrict__ rbuf, OwnIdx I,
                                                   int32_t* __restrict__ counts) {
  constexpr int kRows = 16;
  __shared__ int32_t ckey_s[4][kRows];
  __shared__ int32_t crow_s[4][kRows][64];
  const int lane = lane_of(), wib = threadIdx.x >> 6;
  int32_t* ckey = ckey_s[wib];
  if (lane < kRows) ckey[lane] = -1;
  for (int h = 0; h < kRows; h++) crow_s[wib][h][lane] = 0;
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  // per lane: view j of count row `row` takes c (cached when the row has or gets a cache row; the
  // rows are indexed through the __shared__ array itself, so that the add stays an LDS atomic — a
  // flat one waits for the wave's outstanding global atomics)
  auto add = [&](int32_t row, int j, int32_t c) {
    const int h0 = (int)(((uint32_t)row * 2654435761u) >> 28);
    for (int p = 0; p < 4; p++) {
      const int h = (h0 + p) & (kRows - 1);
      int32_t k = ckey[h];
      if (k == -1) {
        k = atomicCAS(&ckey[h], -1, row);
        if (k == -1) k = row;
      }
      if (k == row) {
        atomicAdd(&crow_s[wib][h][j], c);
        return;
      }
    }
    atomicAdd(&counts[(int64_t)row * 64 + j], c);
  };
  const int64_t n = P.pre[P.np];
  const int64_t wave = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t i0 = wave * 64; i0 < n; i0 += nwaves * 64) {
    const int64_t i = i0 + lane;
    int32_t row = -1;
    XRec r{0, 0, 0};
    if (i < n) {
      const int q = peer_of(P, i);
      r = rbuf[P.base[q] + i - P.pre[q]];
      row = (int32_t)label_row(I, r.e);  // (< n_own < 2^31)
    }
    // a record with few views: its lane adds them; many views: the wave adds its row (lane = view)
    const bool wide = row >= 0 && __popcll(r.mask) > 8;
    for (uint64_t m = (row >= 0 && !wide) ? r.mask : 0ull; m; m &= m - 1) add(row, __builtin_ctzll(m), r.val);
    for (uint64_t t = __ballot(wide); t; t &= t - 1) {
      const int L = __builtin_ctzll(t);
      const int32_t rowL = __builtin_amdgcn_readlane(row, L);
      const uint64_t mL = rl64(r.mask, L);
      const int32_t cL = __builtin_amdgcn_readlane(r.val, L);
      if ((mL >> lane) & 1) add(rowL, lane, cL);
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  for (int h = 0; h < kRows; h++) {
    const int32_t k = ckey[h];
    const int32_t c = crow_s[wib][h][lane];
    if (k != -1 && c) atomicAdd(&counts[(int64_t)k * 64 + lane], c);
  }
}

// ------------------------------------------------------------------ final labels across partitions
// The batch's per-view minimum member label (kernels.hip final_label: INT32_MAX - label in kMinShards
// shards, 0 = no member) over every partition: the shards folded into 64 words here, all-reduced
// (max) by the host, stored back into shard 0 (the others hold local values, never larger).
__global__ void k_min_fold(const int32_t* __restrict__ mneg, unsigned long long* __restrict__ w) {
  const int j = threadIdx.x;
  if (j >= 64) return;
  int32_t x = 0;
  for (int sh = 0; sh < kMinShards; sh++) x = max(x, mneg[sh * 64 + j]);
  w[j] = (unsigned long long)(uint32_t)x;
}
__global__ void k_min_store(const unsigned long long* __restrict__ w, int32_t* __restrict__ mneg) {
  const int j = threadIdx.x;
  if (j < 64) mneg[j] = (int32_t)w[j];
}

// The minimum-label counts (k_part_count fin_g, 64 shards x 64 views): folded into w (and the
// shards zeroed for the next batch); after the all-reduce (sum) over the partitions the label's
// owner adds them at the label's count row
__global__ void k_min_count_fold(unsigned int* __restrict__ fin_g, unsigned long long* __restrict__ w) {
  const int j = threadIdx.x;
  if (j >= 64) return;
  unsigned long long t = 0;
  for (int sh = 0; sh < 64; sh++) {
    t += fin_g[sh * 64 + j];
    fin_g[sh * 64 + j] = 0;
  }
  w[j] = t;
}
__global__ void k_min_count_add(const unsigned long long* __restrict__ w, const int32_t* __restrict__ mneg, OwnIdx I,
                                int np, int me, int32_t* __restrict__ counts) {
  const int j = threadIdx.x;
  if (j >= 64 || w[j] == 0) return;
  int32_t x = 0;
  for (int sh = 0; sh < kMinShards; sh++) x = max(x, mneg[sh * 64 + j]);
  if (!x) return;
  const int32_t l = INT32_MAX - x;
  if (owner_of(l, np) != me) return;
  const int64_t r = label_row(I, l);
  if (r >= 0) counts[r * 64 + j] += (int32_t)w[j];  // (one thread per view: no race)
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
size_t xbc_scan_bytes(int64_t n_own, int np) {
  const int n = (int)(xbc_units(n_own) * np + 1);
  size_t tb = 0;
  (void)hipcub::DeviceScan::ExclusiveSum(nullptr, tb, (unsigned long long*)nullptr, (unsigned long long*)nullptr, n);
  return tb;
}
void launch_xbc_pack(hipStream_t s, int64_t n_own, int np, const XSend& X, const uint64_t* cb_now,
                     const uint64_t* chg_now, const uint64_t* vadj, const int32_t* lab, const int32_t* uw,
                     const uint8_t* pmask, unsigned long long* su, int64_t ucap, XRec* sm, int64_t mcap,
                     unsigned long long* ccnt, unsigned long long* coff, void* scan_tmp, size_t scan_bytes,
                     bool write_only, const XBcIn* clr, uint64_t* cchg, int32_t* cuw) {
  if (X.nb <= 0 || n_own <= 0) {
    if (clr) launch_xbc_clear(s, *clr, cchg, cuw);
    return;
  }
  const int64_t nun = xbc_units(n_own);
  const unsigned grid = xgrid(nun, 4, 4096);
  XBcIn none;
  std::memset(&none, 0, sizeof(none));
  if (!write_only) {
    k_xbc_pack<false><<<grid, 256, 0, s>>>(n_own, np, X.bidx, cb_now, chg_now, vadj, lab, uw, pmask, su, ucap, sm, mcap,
                                           ccnt, coff, clr ? *clr : none, clr ? 1 : 0, cchg, cuw);
    // ccnt[np * nun] stays 0: coff[q * nun] .. coff[(q + 1) * nun] = peer q's records
    if (hipcub::DeviceScan::ExclusiveSum(scan_tmp, scan_bytes, ccnt, coff, (int)(nun * np + 1), s) != hipSuccess)
      throw std::runtime_error("xbc pack: scan");
  }
  k_xbc_pack<true><<<grid, 256, 0, s>>>(n_own, np, X.bidx, cb_now, chg_now, vadj, lab, uw, pmask, su, ucap, sm, mcap,
                                        ccnt, coff, none, 0, nullptr, nullptr);
}
XSend build_xsend(hipStream_t s, int64_t n_own, int64_t nx, const int32_t* xv, std::vector<void*>& T,
                  std::vector<void*>& L) {
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
  int32_t* bidx = (int32_t*)alloc(L, sizeof(int32_t) * n_own);
  int32_t* eb = (int32_t*)alloc(L, sizeof(int32_t) * nx);
  k_xsend_list<<<xgrid(n_own, 256), 256, 0, s>>>(n_own, flag, pos, xb, bidx);
  k_xsend_entries<<<xgrid(nx, 256), 256, 0, s>>>(nx, xv, pos, eb);
  if (hipGetLastError() != hipSuccess || hipStreamSynchronize(s) != hipSuccess)
    throw std::runtime_error("build_xsend: kernels");
  X.v = xb;
  X.bidx = bidx;
  X.eb = eb;
  return X;
}
void launch_xtab_fill(hipStream_t s, int64_t n, const int32_t* xr_v, const int32_t* xr_q, const int32_t* tmp,
                      const XTab& T, unsigned long long* err) {
  if (n > 0) k_xtab_fill<<<xgrid(n, 256), 256, 0, s>>>(n, xr_v, xr_q, tmp, T, err);
}
void launch_xbc_counts(hipStream_t s, int np, int me, const unsigned long long* coff, int64_t nch,
                       const int32_t* stepflag, int64_t* xa) {
  k_xbc_counts<<<1, 64, 0, s>>>(np, me, coff, nch, stepflag, xa);
}
void launch_min_fold(hipStream_t s, const int32_t* mneg, unsigned long long* w) { k_min_fold<<<1, 64, 0, s>>>(mneg, w); }
void launch_min_store(hipStream_t s, const unsigned long long* w, int32_t* mneg) { k_min_store<<<1, 64, 0, s>>>(w, mneg); }
void launch_xcounts(hipStream_t s, int np, int me, unsigned long long* scnt, int64_t* xa) {
  k_xcounts<<<1, 64, 0, s>>>(np, me, scnt, xa);
}
void launch_xbc_clear(hipStream_t s, const XBcIn& I, uint64_t* chg, int32_t* uw) {
  const int64_t n = I.U.pre[I.U.np] + I.M.pre[I.M.np];
  if (n > 0) k_xbc_clear<<<xgrid(n, 256), 256, 0, s>>>(I, chg, uw);
}
void launch_xbc_apply(hipStream_t s, const XBcIn& I, int32_t* lab, uint64_t* chg, int32_t* uw, uint64_t* cb,
                      const DevGraph& g, const uint64_t* vm, const uint64_t* em, uint8_t* act_next, int64_t tcut,
                      const BatchParams* ebp, const int32_t* ccount, int dense_div, int step, const int32_t* gcut) {
  const int64_t n = I.U.pre[I.U.np] + I.M.pre[I.M.np];
  if (n <= 0) return;
  BatchParams bp0;
  if (!ebp) std::memset(&bp0, 0, sizeof(bp0));
  auto* kern = g.ts_t ? k_xbc_apply<true> : k_xbc_apply<false>;
  // many M records (short windows' early supersteps): U records, then M records per ghost; else one
  // pass over every record (the per-ghost loop serialises a wave's ghosts: late supersteps with a few
  // thousand M records took ~100 us that way, profiles/r06/part_sim_*_mrow*)
  // (per ghost pays where a mixed sender has many labels — short windows, M records ~5x the U records —
  // and loses where it has two or three: month views' M records are 0.2-0.5x the U records, and a
  // wave then walks dozens of ghosts in turn)
  const bool split = I.M.pre[I.M.np] >= kMGhostMin && I.M.pre[I.M.np] > 2 * I.U.pre[I.U.np];
  for (int phase = split ? 0 : 2; phase < (split ? 2 : 3); phase++) {
    const int64_t np = phase == 0 ? I.U.pre[I.U.np] : phase == 1 ? I.M.pre[I.M.np] : n;
    if (np > 0)
    kern<<<xgrid(np, 256), 256, 0, s>>>(I, lab, chg, uw, cb, g.out_off, g.in_off, g.in_eid, g.esrc, g.edst, vm, em,
                                     g.n_seg > 0 ? g.hv_of : nullptr, act_next, g.adj_off, g.ts_e, g.ts_nb, g.ts_t, tcut,
                                     ebp ? *ebp : bp0, ebp ? 1 : 0, ccount, dense_div, step, g.ts_t ? gcut : nullptr,
                                     phase);
  }
}
void launch_ghost_cut(hipStream_t s, const DevGraph& g, int64_t tcut, int32_t* gcut) {
  if (g.ts_t && g.nv > g.n_own)
    k_ghost_cut<<<xgrid(g.nv - g.n_own, 256), 256, 0, s>>>(g.n_own, g.nv, g.adj_off, g.ts_t, tcut, gcut);
}
void launch_part_count(hipStream_t s, bool remote_only, const XPeers& P, const OwnIdx& I, int nviews,
                       const uint64_t* vm, const uint64_t* vadj, const int32_t* uw, const int32_t* lab, int32_t* counts,
                       unsigned int* iso, unsigned long long* gcnt, XRec* hsbuf, const int32_t* mneg,
                       unsigned int* fin_g) {
  const uint64_t vmask = nviews >= 64 ? ~0ull : ((1ull << nviews) - 1);
  // 16 chunks of 64 members per wave: a wave flushes its label cache once, as records, so fewer
  // waves emit fewer records (one per cached label and count group) and flush less (grid 2048 ->
  // 512 at 2.2M members: 7.3 -> 5.0 ms per partition and query, profiles/r04/ab_part_count_grid.jsonl).
  // (Round 6: 2 chunks per wave for short windows, whose members are mostly mixed, doubled the hour
  // batches' count time at P = 8 — 324 -> 708 us, more flushes — profiles/r06/part_sim_p8_300m_count_grid_rejected.jsonl)
  const unsigned grid = xgrid(xbc_units(I.n_own), 4 * 16, 2048);
  if (remote_only)
    k_part_count<true><<<grid, 256, 0, s>>>(P, I, vmask, vm, vadj, uw, lab, counts, iso, gcnt, hsbuf, mneg, fin_g);
  else
    k_part_count<false><<<grid, 256, 0, s>>>(P, I, vmask, vm, vadj, uw, lab, counts, iso, gcnt, hsbuf, mneg, fin_g);
}
void launch_min_count_fold(hipStream_t s, unsigned int* fin_g, unsigned long long* w) {
  k_min_count_fold<<<1, 64, 0, s>>>(fin_g, w);
}
void launch_min_count_add(hipStream_t s, const unsigned long long* w, const int32_t* mneg, const OwnIdx& I, int np,
                          int me, int32_t* counts) {
  k_min_count_add<<<1, 64, 0, s>>>(w, mneg, I, np, me, counts);
}
void launch_hist_recv(hipStream_t s, const XPeers& P, const XRec* rbuf, const OwnIdx& I, int32_t* counts) {
  if (P.pre[P.np] > 0) k_hist_recv<<<xgrid(P.pre[P.np], 256), 256, 0, s>>>(P, rbuf, I, counts);
}

}  // namespace rgpu
