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

#include "kernels.hpp"

namespace rgpu {

namespace {

__device__ __forceinline__ int lane_of() { return threadIdx.x & 63; }
__device__ __forceinline__ uint64_t rl64(uint64_t x, int l) {
  const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)x, l);
  const uint32_t hi = __builtin_amdgcn_readlane((uint32_t)(x >> 32), l);
  return ((uint64_t)hi << 32) | lo;
}
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
  if (div <= 0 || !ccount || r < 3) return false;
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
__global__ __launch_bounds__(256) void k_xpack_rec(XPeers P, int64_t nx, const int32_t* __restrict__ xv,
                                                   const int32_t* __restrict__ xq, const uint8_t* __restrict__ act,
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
  for (int64_t c = wave; c * 64 < nx; c += nwaves) {
    const int64_t e = c * 64 + lane;
    const bool ok = e < nx;
    const int32_t v = ok ? xv[e] : 0;
    const int q = ok ? xq[e] : 0;
    uint64_t m = 0;
    if (ok && (act == nullptr || act[v])) m = chg_now[v] & vadj[v];
    const uint64_t todo = __ballot(m != 0);
    if (!todo) continue;
    unsigned long long cq = 0;  // lane p: records of this wave for peer p
    for (uint64_t b = todo; b; b &= b - 1) {
      const int L = __builtin_ctzll(b);
      const int32_t vL = __builtin_amdgcn_readlane(v, L);
      const int qL = __builtin_amdgcn_readlane(q, L);
      uint64_t mm = rl64(m, L);
      const int32_t uL = uw ? uw[vL] : -1;  // a uniform row is its word (kernels.hip kMixed = -1)
      const int32_t x = uL != -1 ? uL : lab[(int64_t)vL * 64 + lane];
      int n = 0;
      while (mm) {
        const int32_t val = __builtin_amdgcn_readlane(x, __builtin_ctzll(mm));
        mm &= ~__ballot(((mm >> lane) & 1) && x == val);
        n++;
      }
      if (lane == qL) cq += (unsigned long long)n;
    }
    unsigned long long off = 0;
    if (lane < P.np && cq) off = atomicAdd(&scnt[lane], cq);
    for (uint64_t b = todo; b; b &= b - 1) {
      const int L = __builtin_ctzll(b);
      const int32_t vL = __builtin_amdgcn_readlane(v, L);
      const int qL = __builtin_amdgcn_readlane(q, L);
      const int32_t eL = (int32_t)(c * 64 + L - P.xoff[qL]);
      uint64_t mm = rl64(m, L);
      const int32_t uL = uw ? uw[vL] : -1;
      const int32_t x = uL != -1 ? uL : lab[(int64_t)vL * 64 + lane];
      while (mm) {
        const int32_t val = __builtin_amdgcn_readlane(x, __builtin_ctzll(mm));
        const uint64_t same = __ballot(((mm >> lane) & 1) && x == val);
        const unsigned long long pos = __builtin_amdgcn_readlane((uint32_t)off, qL) |
                                       ((unsigned long long)__builtin_amdgcn_readlane((uint32_t)(off >> 32), qL) << 32);
        if (lane == 0 && pos < (unsigned long long)P.cap[qL]) {
          XRec r;
          r.e = eL;
          r.val = uL != -1 ? (int32_t)((uint32_t)val | 0x80000000u) : val;  // sign bit: sender uniform
          r.mask = same;
          sbuf[P.base[qL] + pos] = r;
        }
        if (lane == qL) off++;
        mm &= ~same;
      }
    }
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

// ghosts whose change word a record set two supersteps ago: clear it in that parity's words
__global__ __launch_bounds__(256) void k_xclear(XPeers P, const XRec* __restrict__ rbuf,
                                                const int32_t* __restrict__ xrv, uint64_t* __restrict__ chg) {
  const int64_t n = P.pre[P.np];
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int q = peer_of(P, i);
    chg[xrv[P.xoff[q] + rbuf[P.base[q] + i - P.pre[q]].e]] = 0;
  }
}

// Records into ghost rows: the record's label in its views, and its views into the ghost's
// change word (a ghost's records arrive together; the OR collects them).  A wave takes four
// records, 16 lanes each covering the 64 views in 4 passes.  A record whose sender's row is
// uniform (sign bit of val; it is then the ghost's only record of the step) sets the ghost's
// uniform word instead of its row: readers only gather a ghost in the views its change word
// holds, which are the record's.  Other records mark the ghost mixed (kernels.hip kMixed).
__global__ __launch_bounds__(256) void k_xunpack_rec(XPeers P, const XRec* __restrict__ rbuf,
                                                     const int32_t* __restrict__ xrv, int32_t* __restrict__ lab,
                                                     uint64_t* __restrict__ chg, int32_t* __restrict__ uw,
                                                     uint64_t* __restrict__ cb) {
  const int64_t n = P.pre[P.np];
  const int lane = lane_of(), sub = lane >> 4, l16 = lane & 15;
  const int64_t wave = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t i0 = wave * 4; i0 < n; i0 += nwaves * 4) {
    const int64_t i = i0 + sub;
    if (i >= n) continue;
    const int q = peer_of(P, i);
    const XRec r = rbuf[P.base[q] + i - P.pre[q]];
    const int32_t g = xrv[P.xoff[q] + r.e];
    const bool uni = r.val < 0;
    const int32_t val = r.val & 0x7fffffff;
    if (!uni || !uw) {
#pragma unroll
      for (int k = 0; k < 4; k++) {
        const int j = k * 16 + l16;
        if ((r.mask >> j) & 1) lab[(int64_t)g * 64 + j] = val;
      }
    }
    if (l16 == 0) {
      if (uw) uw[g] = uni ? val : -1;
      atomicOr((unsigned long long*)&chg[g], (unsigned long long)r.mask);
      if (cb) atomicOr((unsigned long long*)&cb[g >> 6], 1ull << (g & 63));  // the ghost changed (ChgBits)
    }
  }
}

// After the unpack: the first record of every ghost marks the ghost's owned neighbours that
// share a changed view (the next frontier, as a local change would).  Ghosts keep no compacted
// slots (K2 runs over the owned vertices only): the kept views of a static slot, em[e] & vm[nb] &
// vm[g], are recomputed here for the ghosts that changed.  Heavy ghosts: k_heavy_mark.
__global__ __launch_bounds__(256) void k_xmark(XPeers P, const XRec* __restrict__ rbuf,
                                               const int32_t* __restrict__ xrv, const uint64_t* __restrict__ chg,
                                               const int64_t* __restrict__ out_off,
                                               const int64_t* __restrict__ in_off,
                                               const int32_t* __restrict__ in_eid,
                                               const int32_t* __restrict__ esrc, const int32_t* __restrict__ edst,
                                               const uint64_t* __restrict__ vm, const uint64_t* __restrict__ em,
                                               const int32_t* __restrict__ hv_of, uint8_t* __restrict__ act_next) {
  const int64_t n = P.pre[P.np];
  const int lane = lane_of();
  const int64_t wave = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t i = wave; i < n; i += nwaves) {
    const int q = peer_of(P, i);
    const int64_t k = i - P.pre[q];
    const int32_t e0 = rbuf[P.base[q] + k].e;
    if (k > 0 && rbuf[P.base[q] + k - 1].e == e0) continue;  // not the ghost's first record
    const int32_t g = xrv[P.xoff[q] + e0];
    if (hv_of && hv_of[g] >= 0) continue;
    const uint64_t ch = chg[g] & vm[g];
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
// routed to the label's owner: as k_cc_hist, a block stages 64 vertices' label rows and its
// eight waves dedup each view's labels (after `rounds` labels, one entry per lane).  Counts of
// labels owned here go straight into hist[view][owned rank]; the others become records
// (label | view << 31 | count << 37), staged per peer in LDS and flushed after every chunk with
// one atomicAdd per (block, peer).  Members with no kept slot are islands, counted in iso.
constexpr int kStage = 256;  // staged records per peer and chunk (more: written directly)
template <bool REMOTE_ONLY>
__global__ __launch_bounds__(512) void k_hist_route(XPeers P, OwnIdx I, int nviews,
                                                    const uint64_t* __restrict__ vm,
                                                    const uint64_t* __restrict__ vadj,
                                                    const int32_t* __restrict__ lab, int32_t* __restrict__ hist,
                                                    unsigned int* __restrict__ iso_g, int rounds,
                                                    unsigned long long* __restrict__ gcnt,
                                                    unsigned long long* __restrict__ hsbuf) {
  __shared__ int32_t tile[64][65];
  __shared__ unsigned int iso[64];
  __shared__ unsigned long long stage[kMaxParts][kStage];
  __shared__ unsigned int pc[kMaxParts];
  __shared__ unsigned long long fb[kMaxParts];
  const int64_t n_own = I.n_own;
  const int lane = lane_of(), wib = threadIdx.x >> 6;
  if (threadIdx.x < 64) iso[threadIdx.x] = 0;
  if (threadIdx.x < kMaxParts) pc[threadIdx.x] = 0;
  const uint64_t vmask = (nviews >= 64 ? ~0ull : ((1ull << nviews) - 1)) & (0x0101010101010101ull << wib);
  __syncthreads();
  auto emit = [&](int32_t L, int j, unsigned int c, bool on) {  // per lane
    if (!on) return;
    const int q = owner_of(L, P.np);
    if (q == P.me) {
      if (!REMOTE_ONLY) {
        const int64_t rk = owned_rank(I, L);  // always found: a label is a member's id
        if (rk >= 0) atomicAdd(&hist[(int64_t)j * n_own + rk], (int32_t)c);
      }
      return;
    }
    const unsigned long long rec = (unsigned long long)L | ((unsigned long long)j << 31) | ((unsigned long long)c << 37);
    const unsigned int k = atomicAdd(&pc[q], 1u);
    if (k < kStage) {
      stage[q][k] = rec;
    } else {  // a chunk with more records for q than the stage holds: straight out
      const unsigned long long pos = atomicAdd(&gcnt[q], 1ull);
      if (pos < (unsigned long long)P.cap[q]) hsbuf[P.base[q] + (int64_t)pos] = rec;
    }
  };
  for (int64_t c = blockIdx.x; c * 64 < n_own; c += gridDim.x) {
    const int64_t v0 = c * 64;
    const int nvc = (int)(n_own - v0 < 64 ? n_own - v0 : 64);
    {
      int32_t r[8];
#pragma unroll
      for (int k = 0; k < 8; k++) {
        const int i = wib * 8 + k;
        r[k] = i < nvc ? lab[(v0 + i) * 64 + lane] : 0;
      }
#pragma unroll
      for (int k = 0; k < 8; k++) tile[wib * 8 + k][lane] = r[k];
    }
    const uint64_t mvl = lane < nvc ? vm[v0 + lane] : 0;
    const uint64_t adl = lane < nvc ? vadj[v0 + lane] : 0;
    uint64_t any = mvl;
    for (int o = 32; o > 0; o >>= 1) any |= __shfl_xor(any, o);
    any = rl64(any, 0) & vmask;
    __syncthreads();
    while (any) {
      const int j = __builtin_ctzll(any);
      any &= any - 1;
      const bool in_view = (mvl >> j) & 1;
      const bool member = in_view && ((adl >> j) & 1);
      if (!REMOTE_ONLY) {
        const uint64_t isolated = __ballot(in_view && !member);
        if (lane == 0 && isolated) iso[j] += (unsigned)__popcll(isolated);
      }
      const int32_t l = tile[lane][j];
      uint64_t todo = __ballot(member);
      for (int it = 0; todo; it++) {
        if (it == rounds) {
          emit(l, j, 1u, (todo >> lane) & 1);
          break;
        }
        const int leader = __builtin_ctzll(todo);
        const int32_t L = __builtin_amdgcn_readlane(l, leader);
        const uint64_t same = __ballot(member && l == L);
        emit(L, j, (unsigned)__popcll(same), lane == leader);
        todo &= ~same;
      }
    }
    __syncthreads();  // the chunk's records are staged (and the tile is free)
    if (threadIdx.x < P.np) {
      const unsigned int n = pc[threadIdx.x] < kStage ? pc[threadIdx.x] : kStage;
      fb[threadIdx.x] = n ? atomicAdd(&gcnt[threadIdx.x], (unsigned long long)n) : 0ull;
    }
    __syncthreads();
    for (int q = 0; q < P.np; q++) {
      const unsigned int n = pc[q] < kStage ? pc[q] : kStage;
      for (unsigned int i = threadIdx.x; i < n; i += blockDim.x) {
        const unsigned long long pos = fb[q] + i;
        if (pos < (unsigned long long)P.cap[q]) hsbuf[P.base[q] + (int64_t)pos] = stage[q][i];
      }
    }
    __syncthreads();
    if (threadIdx.x < kMaxParts) pc[threadIdx.x] = 0;
    __syncthreads();
  }
  if (!REMOTE_ONLY && threadIdx.x < 64 && iso[threadIdx.x])
    atomicAdd(&iso_g[(blockIdx.x & 63) * 64 + threadIdx.x], iso[threadIdx.x]);
}

// records received from the other partitions: count at the owned label vertex
__global__ __launch_bounds__(256) void k_hist_recv(XPeers P, const unsigned long long* __restrict__ rbuf, OwnIdx I,
                                                   int32_t* __restrict__ hist) {
  const int64_t n = P.pre[P.np];
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int q = peer_of(P, i);
    const unsigned long long r = rbuf[P.base[q] + i - P.pre[q]];
    const int64_t L = (int64_t)(r & 0x7fffffffull);
    const int j = (int)((r >> 31) & 63);
    const int32_t c = (int32_t)(r >> 37);
    const int64_t rk = owned_rank(I, L);
    if (rk >= 0) atomicAdd(&hist[(int64_t)j * I.n_own + rk], c);
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
void launch_xpack_rec(hipStream_t s, const XPeers& P, int64_t nx, const int32_t* xv, const int32_t* xq,
                      const uint8_t* act, const uint64_t* chg_now, const uint64_t* vadj, const int32_t* lab,
                      const int32_t* uw, XRec* sbuf, unsigned long long* scnt, const int32_t* ccount, int dense_div,
                      int step, int64_t n_own) {
  if (nx > 0)
    k_xpack_rec<<<xgrid(nx, 4 * 64, 4096), 256, 0, s>>>(P, nx, xv, xq, act, chg_now, vadj, lab, uw, sbuf, scnt,
                                                         ccount, dense_div, step, n_own);
}
void launch_xcounts(hipStream_t s, int np, int me, unsigned long long* scnt, const int32_t* stepflag, int64_t* xa) {
  k_xcounts<<<1, 64, 0, s>>>(np, me, scnt, stepflag, xa);
}
void launch_xclear(hipStream_t s, const XPeers& P, const XRec* rbuf, const int32_t* xrv, uint64_t* chg) {
  if (P.pre[P.np] > 0) k_xclear<<<xgrid(P.pre[P.np], 256), 256, 0, s>>>(P, rbuf, xrv, chg);
}
void launch_xunpack_rec(hipStream_t s, const XPeers& P, const XRec* rbuf, const int32_t* xrv, int32_t* lab,
                        uint64_t* chg, int32_t* uw, uint64_t* cb) {
  if (P.pre[P.np] > 0) k_xunpack_rec<<<xgrid(P.pre[P.np], 16), 256, 0, s>>>(P, rbuf, xrv, lab, chg, uw, cb);
}
void launch_xmark(hipStream_t s, const XPeers& P, const XRec* rbuf, const int32_t* xrv, const uint64_t* chg,
                  const DevGraph& g, const uint64_t* vm, const uint64_t* em, uint8_t* act_next) {
  if (P.pre[P.np] > 0)
    k_xmark<<<xgrid(P.pre[P.np], 4), 256, 0, s>>>(P, rbuf, xrv, chg, g.out_off, g.in_off, g.in_eid, g.esrc, g.edst,
                                                   vm, em, g.n_seg > 0 ? g.hv_of : nullptr, act_next);
}
void launch_hist_route(hipStream_t s, bool remote_only, const XPeers& P, const OwnIdx& I, int nviews,
                       const uint64_t* vm, const uint64_t* vadj, const int32_t* lab, int32_t* hist, unsigned int* iso,
                       unsigned long long* gcnt, unsigned long long* hsbuf) {
  const unsigned grid = xgrid(I.n_own, 64, 8192);
  if (remote_only)
    k_hist_route<true><<<grid, 512, 0, s>>>(P, I, nviews, vm, vadj, lab, hist, iso, g_hist_rounds, gcnt, hsbuf);
  else
    k_hist_route<false><<<grid, 512, 0, s>>>(P, I, nviews, vm, vadj, lab, hist, iso, g_hist_rounds, gcnt, hsbuf);
}
void launch_hist_recv(hipStream_t s, const XPeers& P, const unsigned long long* rbuf, const OwnIdx& I, int32_t* hist) {
  if (P.pre[P.np] > 0) k_hist_recv<<<xgrid(P.pre[P.np], 256), 256, 0, s>>>(P, rbuf, I, hist);
}

}  // namespace rgpu
