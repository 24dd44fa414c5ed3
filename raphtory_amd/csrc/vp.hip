// vp.hip — generic vertex programs on the GPU (rgpu_set_vertex_program, include/rgpu.h; SURVEY.md
// §8(f) row 4): the VertexVisitor messaging surface (messageAllOutgoingNeighbors /
// messageAllIngoingNeighbors / messageAllNeighbours, getOrSetCompValue / setCompValue,
// voteToHalt; VertexVisitor.scala:81-166) for an Analyser whose analyse() folds its message queue
// with min or max.  Semantics: oracle.h orc_vertex_program.  Lane = view, as in CC: one pass over
// the batch's pull slots serves its 64 views.
//
//   k_vp_slots  per member, the neighbours whose messages it receives — the senders that name it
//               in the program's direction — kept iff em[e] & vm[sender] & vm[v], compacted at the
//               vertex's static slot offset (out + in edges; every direction fits)
//   k_vp_init   setup (superstep 0): the members' state rows (int64) and the senders' change words
//   k_vp_step   superstep r: per member, the fold (min / max) of sender state + step_add over the
//               kept slots whose sender changed in r-1 (those sent it a message); a member whose
//               state the fold changes keeps it and sends next step, the others vote to halt
//   float programs (ABI 10, VertexMessageFloat summed — the message shape of the reference's float
//   analyser, examples/random/depricated/PageRank.scala:20-37, with its commented-out queue loop
//   done):
//   k_vp_deg    per member and view, its message targets alive in the view (the divisor of
//               per_degree programs: getOutgoingNeighbors.size for OUT)
//   k_vp_step_f superstep r: per member, the sum (double) of the senders' float messages, state =
//               (float)(bias + mult * sum) when a message arrived (it sends again), else unchanged
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
__device__ __forceinline__ uint64_t lanes_below(int lane) { return lane ? (~0ull >> (64 - lane)) : 0ull; }
__device__ __forceinline__ int64_t sat_add(int64_t a, int64_t b) {
  if (b > 0 && a > INT64_MAX - b) return INT64_MAX;
  if (b < 0 && a < INT64_MIN - b) return INT64_MIN;
  return a + b;
}

// pull slots of v: for direction OUT the in-edges' sources and a self-loop; IN: the out-edges'
// targets but v itself (a self-loop never enters incomingEdges, EntityStorage.scala:257); ALL: both
__global__ __launch_bounds__(256) void k_vp_slots(int64_t nv, int dir, const int64_t* __restrict__ out_off,
                                                  const int64_t* __restrict__ in_off,
                                                  const int64_t* __restrict__ adj_off,
                                                  const int32_t* __restrict__ in_eid,
                                                  const int32_t* __restrict__ esrc,
                                                  const int32_t* __restrict__ edst,
                                                  const uint64_t* __restrict__ vm, const uint64_t* __restrict__ em,
                                                  int32_t* __restrict__ cnt, int32_t* __restrict__ snbr,
                                                  uint64_t* __restrict__ smask) {
  const int lane = lane_of();
  const int64_t wave = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t v = wave; v < nv; v += nwaves) {
    const uint64_t mv = vm[v];
    if (mv == 0) {
      if (lane == 0) cnt[v] = 0;
      continue;
    }
    const int64_t o0 = out_off[v], nout = out_off[v + 1] - o0, i0 = in_off[v], nin = in_off[v + 1] - i0;
    const int64_t base = adj_off[v];
    int32_t count = 0;
    for (int part = 0; part < 2; part++) {  // 0: in-edges (senders of OUT / ALL), 1: out-edges
      if (part == 0 && dir == 1) continue;
      if (part == 1 && dir == 0) {
        // OUT: only a self-loop of the out-edges sends to v (out-edges are sorted by target)
        int64_t a = o0, b = o0 + nout;
        while (a < b) {
          const int64_t m = (a + b) >> 1;
          if (edst[m] < (int32_t)v) a = m + 1; else b = m;
        }
        if (lane == 0 && a < o0 + nout && edst[a] == (int32_t)v) {
          const uint64_t m = em[a] & mv;
          if (m) {
            snbr[base + count] = (int32_t)v;
            smask[base + count] = m;
          }
          count += m != 0;
        }
        count = __builtin_amdgcn_readlane(count, 0);
        continue;
      }
      const int64_t n = part == 0 ? nin : nout;
      for (int64_t c = 0; c < n; c += 64) {
        const int64_t j = c + lane;
        uint64_t m = 0;
        int32_t nb = 0;
        if (j < n) {
          const int32_t e = part == 0 ? in_eid[i0 + j] : (int32_t)(o0 + j);
          nb = part == 0 ? esrc[e] : edst[e];
          if (!(part == 1 && dir == 1 && nb == (int32_t)v)) m = em[e] & vm[nb] & mv;
        }
        const uint64_t bal = __ballot(m != 0);
        if (m) {
          const int64_t pos = base + count + __popcll(bal & lanes_below(lane));
          snbr[pos] = nb;
          smask[pos] = m;
        }
        count += __popcll(bal);
      }
    }
    if (lane == 0) cnt[v] = count;
  }
}

__device__ __forceinline__ int64_t f_bits(double x) { return __double_as_longlong(x); }
__device__ __forceinline__ double f_val(int64_t b) { return __longlong_as_double(b); }

__global__ __launch_bounds__(256) void k_vp_init(int64_t nv, VpParams p, const int32_t* __restrict__ grank,
                                                 const int64_t* __restrict__ vid, const uint64_t* __restrict__ vm,
                                                 int64_t* __restrict__ st, uint64_t* __restrict__ chg) {
  const int lane = lane_of();
  const int64_t wave = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t v = wave; v < nv; v += nwaves) {
    const uint64_t mv = vm[v];
    const int64_t x = p.fsum ? f_bits((double)(float)(p.init == 0 ? (double)vid[v] : (v == p.seed_rank ? p.f_seed : p.f_init)))
                             : (p.init == 0 ? vid[v] : (v == p.seed_rank ? p.seed_value : p.init_value));
    st[v * 64 + lane] = x;
    if (lane == 0) chg[v] = (p.senders == 0 || v == p.seed_rank) ? mv : 0ull;  // the setup's senders
  }
}
// superstep 1 always runs after a setup (its halting vote counts the message holders)
__global__ void k_vp_go(int32_t* __restrict__ stepflag) { stepflag[0] = 1; }

template <int RED>
__global__ __launch_bounds__(256) void k_vp_step(int step, int64_t nv, int64_t step_add, const int64_t* __restrict__ adj_off,
                                                 const uint64_t* __restrict__ vm, const int32_t* __restrict__ cnt,
                                                 const int32_t* __restrict__ snbr, const uint64_t* __restrict__ smask,
                                                 const int64_t* __restrict__ st_cur, int64_t* __restrict__ st_next,
                                                 const uint64_t* __restrict__ chg_prev, uint64_t* __restrict__ chg_next,
                                                 int32_t* __restrict__ stepflag, int32_t* __restrict__ hostflag,
                                                 unsigned long long* __restrict__ lanechg) {
  if (stepflag[step - 1] == 0) return;  // the job halted (AnalysisTask.endStep)
  __shared__ unsigned long long lanes_s;
  if (threadIdx.x == 0) lanes_s = 0;
  __syncthreads();
  const int lane = lane_of();
  const int64_t wave = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  const int64_t ident = RED == 0 ? INT64_MAX : INT64_MIN;
  uint64_t lanes = 0;
  for (int64_t v = wave; v < nv; v += nwaves) {
    const uint64_t mv = vm[v];
    if (mv == 0) continue;
    const int32_t n = cnt[v];
    const int64_t base = adj_off[v];
    const int64_t cur = st_cur[v * 64 + lane];
    int64_t m = ident;
    bool got = false;  // lane = view: a message arrived (moreMessages)
    for (int32_t c = 0; c < n; c += 64) {
      const int32_t j = c + lane;
      int32_t nb = 0;
      uint64_t a = 0;
      if (j < n) {
        nb = snbr[base + j];
        a = smask[base + j] & chg_prev[nb];
      }
      for (uint64_t bal = __ballot(a != 0); bal; bal &= bal - 1) {
        const int L = __builtin_ctzll(bal);
        const int32_t q = __builtin_amdgcn_readlane(nb, L);
        if ((rl64(a, L) >> lane) & 1) {
          const int64_t x = sat_add(st_cur[(int64_t)q * 64 + lane], step_add);
          m = RED == 0 ? (x < m ? x : m) : (x > m ? x : m);
          got = true;
        }
      }
    }
    const bool member = (mv >> lane) & 1;
    const int64_t nx = (member && got) ? (RED == 0 ? (m < cur ? m : cur) : (m > cur ? m : cur)) : cur;
    const uint64_t ch = __ballot(member && nx != cur);
    st_next[v * 64 + lane] = nx;
    if (lane == 0) chg_next[v] = ch;
    lanes |= ch;
  }
  if (lane == 0 && lanes) atomicOr(&lanes_s, (unsigned long long)lanes);
  __syncthreads();
  if (threadIdx.x == 0 && lanes_s) {
    atomicOr(&lanechg[step * kLaneShards + (blockIdx.x & (kLaneShards - 1))], lanes_s);
    if (stepflag[step] == 0) {
      stepflag[step] = 1;
      if (hostflag) hostflag[step] = 1;
    }
  }
}

// message targets of member v alive in each view (lane = view): OUT its out-edges (a self-loop
// included, outgoingProcessing), IN its in-edges (a self-loop never enters incomingEdges)
__global__ __launch_bounds__(256) void k_vp_deg(int64_t nv, int dir, const int64_t* __restrict__ out_off,
                                                const int64_t* __restrict__ in_off, const int32_t* __restrict__ in_eid,
                                                const int32_t* __restrict__ esrc, const uint64_t* __restrict__ vm,
                                                const uint64_t* __restrict__ em, int32_t* __restrict__ deg) {
  const int lane = lane_of();
  const int64_t wave = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t v = wave; v < nv; v += nwaves) {
    const uint64_t mv = vm[v];
    int32_t d = 0;
    if (mv) {
      const int64_t a0 = dir == 0 ? out_off[v] : in_off[v], n = (dir == 0 ? out_off[v + 1] : in_off[v + 1]) - a0;
      for (int64_t c = 0; c < n; c++) {  // (a few edges per vertex: the wave walks them, lane = view)
        const int32_t e = dir == 0 ? (int32_t)(a0 + c) : in_eid[a0 + c];
        if (dir == 1 && esrc[e] == (int32_t)v) continue;
        d += (int32_t)((em[e] & mv) >> lane) & 1;
      }
    }
    deg[v * 64 + lane] = d;
  }
}

// float programs: superstep r (see k_vp_step); the messages of a sender q are (float)(state_q /
// max(deg_q, 1)) with per_degree, else its state; summed in double in slot order
__global__ __launch_bounds__(256) void k_vp_step_f(int step, int64_t nv, VpParams p, const int64_t* __restrict__ adj_off,
                                                   const uint64_t* __restrict__ vm, const int32_t* __restrict__ cnt,
                                                   const int32_t* __restrict__ snbr, const uint64_t* __restrict__ smask,
                                                   const int64_t* __restrict__ st_cur, int64_t* __restrict__ st_next,
                                                   const uint64_t* __restrict__ chg_prev, uint64_t* __restrict__ chg_next,
                                                   int32_t* __restrict__ stepflag, int32_t* __restrict__ hostflag,
                                                   unsigned long long* __restrict__ lanechg,
                                                   const int32_t* __restrict__ deg) {
  if (stepflag[step - 1] == 0) return;
  __shared__ unsigned long long lanes_s;
  if (threadIdx.x == 0) lanes_s = 0;
  __syncthreads();
  const int lane = lane_of();
  const int64_t wave = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  uint64_t lanes = 0;
  for (int64_t v = wave; v < nv; v += nwaves) {
    const uint64_t mv = vm[v];
    if (mv == 0) continue;
    const int32_t n = cnt[v];
    const int64_t base = adj_off[v];
    const int64_t cur = st_cur[v * 64 + lane];
    double sum = 0.0;
    bool got = false;
    for (int32_t c = 0; c < n; c += 64) {
      const int32_t j = c + lane;
      int32_t nb = 0;
      uint64_t a = 0;
      if (j < n) {
        nb = snbr[base + j];
        a = smask[base + j] & chg_prev[nb];
      }
      for (uint64_t bal = __ballot(a != 0); bal; bal &= bal - 1) {  // slot order
        const int L = __builtin_ctzll(bal);
        const int32_t q = __builtin_amdgcn_readlane(nb, L);
        if ((rl64(a, L) >> lane) & 1) {
          double x = f_val(st_cur[(int64_t)q * 64 + lane]);
          if (p.per_degree) {
            const int32_t dq = deg[(int64_t)q * 64 + lane];
            x = (double)(float)(x / (double)(dq > 1 ? dq : 1));
          }
          sum += x;
          got = true;
        }
      }
    }
    const bool member = (mv >> lane) & 1;
    const bool upd = member && got;
    const int64_t nx = upd ? f_bits((double)(float)(p.f_bias + p.f_mult * sum)) : cur;
    const uint64_t ch = __ballot(upd);  // a member that received messages sends again
    st_next[v * 64 + lane] = nx;
    if (lane == 0) chg_next[v] = ch;
    lanes |= ch;
  }
  if (lane == 0 && lanes) atomicOr(&lanes_s, (unsigned long long)lanes);
  __syncthreads();
  if (threadIdx.x == 0 && lanes_s) {
    atomicOr(&lanechg[step * kLaneShards + (blockIdx.x & (kLaneShards - 1))], lanes_s);
    if (stepflag[step] == 0) {
      stepflag[step] = 1;
      if (hostflag) hostflag[step] = 1;
    }
  }
}

// Partitioned vertex programs: a boundary vertex's record for a peer = its 64 state words and its
// change word (kVpRec words; one wave per entry, lane = view), gathered in the plan's send order
// and scattered into the receiver's ghost rows (xv: send / receive entries -> local ranks)
__global__ __launch_bounds__(256) void k_vp_xgather(int64_t n, const int32_t* __restrict__ xv,
                                                    const int64_t* __restrict__ st, const uint64_t* __restrict__ chg,
                                                    int64_t* __restrict__ buf) {
  const int lane = lane_of();
  const int64_t wave = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t k = wave; k < n; k += nwaves) {
    const int64_t v = xv[k];
    buf[k * kVpRec + lane] = st[v * 64 + lane];
    if (lane == 0) buf[k * kVpRec + 64] = (int64_t)chg[v];
  }
}
__global__ __launch_bounds__(256) void k_vp_xscatter(int64_t n, const int32_t* __restrict__ xv,
                                                     const int64_t* __restrict__ buf, int64_t* __restrict__ st,
                                                     uint64_t* __restrict__ chg) {
  const int lane = lane_of();
  const int64_t wave = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t k = wave; k < n; k += nwaves) {
    const int64_t v = xv[k];
    st[v * 64 + lane] = buf[k * kVpRec + lane];
    if (lane == 0) chg[v] = (uint64_t)buf[k * kVpRec + 64];
  }
}
// the degree rows of per_degree float programs (a ghost's targets live on its owner), once per batch
__global__ __launch_bounds__(256) void k_vp_xgather_deg(int64_t n, const int32_t* __restrict__ xv,
                                                        const int32_t* __restrict__ deg, int32_t* __restrict__ buf) {
  const int lane = lane_of();
  const int64_t wave = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t k = wave; k < n; k += nwaves) buf[k * 64 + lane] = deg[(int64_t)xv[k] * 64 + lane];
}
__global__ __launch_bounds__(256) void k_vp_xscatter_deg(int64_t n, const int32_t* __restrict__ xv,
                                                         const int32_t* __restrict__ buf, int32_t* __restrict__ deg) {
  const int lane = lane_of();
  const int64_t wave = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t k = wave; k < n; k += nwaves) deg[(int64_t)xv[k] * 64 + lane] = buf[k * 64 + lane];
}
// the step's views with a change, folded from the lane shards (the global vote is their all-reduce)
__global__ void k_vp_lanes(const unsigned long long* __restrict__ lanechg, int step, unsigned long long* __restrict__ w) {
  const int j = threadIdx.x;
  if (j >= 64) return;
  unsigned long long x = 0;
  for (int sh = 0; sh < kLaneShards; sh++) x |= lanechg[step * kLaneShards + sh];
  w[j] = (x >> j) & 1;
}
// after the all-reduce (max) of the per-view change flags: the step's flag, as if this partition
// had changed a state itself (the next superstep runs on every partition while any changed)
__global__ void k_vp_vote(const unsigned long long* __restrict__ w, int step, int32_t* __restrict__ stepflag,
                          unsigned long long* __restrict__ lanechg) {
  const int j = threadIdx.x;
  if (j >= 64) return;
  const bool any = __ballot(w[j] != 0) != 0;
  if (j == 0) {
    stepflag[step] = any ? 1 : 0;
    unsigned long long m = 0;
    for (int k = 0; k < 64; k++) m |= (w[k] ? 1ull : 0ull) << k;
    lanechg[step * kLaneShards] |= m;  // (the views' last changing step: global, as the reference's job)
  }
}

unsigned vgrid(int64_t items, int per_block, unsigned cap) {
  int64_t g = (items + per_block - 1) / per_block;
  if (g < 1) g = 1;
  return (unsigned)(g > cap ? cap : g);
}

}  // namespace

void launch_vp_setup(hipStream_t s, const DevGraph& g, const VpParams& p, const int64_t* vid, const uint64_t* vm,
                     const uint64_t* em, int32_t* cnt, int32_t* snbr, uint64_t* smask, int64_t* st0, uint64_t* chg0,
                     int32_t* deg) {
  const unsigned grid = vgrid(g.nv, 4, 8192);
  k_vp_slots<<<grid, 256, 0, s>>>(g.nv, p.dir, g.out_off, g.in_off, g.adj_off, g.in_eid, g.esrc, g.edst, vm, em, cnt,
                                  snbr, smask);
  k_vp_init<<<grid, 256, 0, s>>>(g.nv, p, g.grank, vid, vm, st0, chg0);
  if (p.fsum && p.per_degree && deg)
    k_vp_deg<<<grid, 256, 0, s>>>(g.nv, p.dir, g.out_off, g.in_off, g.in_eid, g.esrc, vm, em, deg);
}
void launch_vp_go(hipStream_t s, int32_t* stepflag) { k_vp_go<<<1, 1, 0, s>>>(stepflag); }

void launch_vp_step(hipStream_t s, int step, const DevGraph& g, const VpParams& p, const uint64_t* vm,
                    const int32_t* cnt, const int32_t* snbr, const uint64_t* smask, const int64_t* st_cur,
                    int64_t* st_next, const uint64_t* chg_prev, uint64_t* chg_next, int32_t* stepflag,
                    int32_t* hostflag, unsigned long long* lanechg, const int32_t* deg) {
  const unsigned grid = vgrid(g.nv, 4, 8192);
  if (p.fsum)
    k_vp_step_f<<<grid, 256, 0, s>>>(step, g.nv, p, g.adj_off, vm, cnt, snbr, smask, st_cur, st_next, chg_prev, chg_next,
                                     stepflag, hostflag, lanechg, deg);
  else if (p.reduce == 0)
    k_vp_step<0><<<grid, 256, 0, s>>>(step, g.nv, p.step_add, g.adj_off, vm, cnt, snbr, smask, st_cur, st_next,
                                      chg_prev, chg_next, stepflag, hostflag, lanechg);
  else
    k_vp_step<1><<<grid, 256, 0, s>>>(step, g.nv, p.step_add, g.adj_off, vm, cnt, snbr, smask, st_cur, st_next,
                                      chg_prev, chg_next, stepflag, hostflag, lanechg);
}

}  // namespace rgpu

namespace rgpu {
void launch_vp_xgather(hipStream_t s, int64_t n, const int32_t* xv, const int64_t* st, const uint64_t* chg,
                       int64_t* buf) {
  if (n > 0) k_vp_xgather<<<vgrid(n, 4, 4096), 256, 0, s>>>(n, xv, st, chg, buf);
}
void launch_vp_xscatter(hipStream_t s, int64_t n, const int32_t* xv, const int64_t* buf, int64_t* st, uint64_t* chg) {
  if (n > 0) k_vp_xscatter<<<vgrid(n, 4, 4096), 256, 0, s>>>(n, xv, buf, st, chg);
}
void launch_vp_xgather_deg(hipStream_t s, int64_t n, const int32_t* xv, const int32_t* deg, int32_t* buf) {
  if (n > 0) k_vp_xgather_deg<<<vgrid(n, 4, 4096), 256, 0, s>>>(n, xv, deg, buf);
}
void launch_vp_xscatter_deg(hipStream_t s, int64_t n, const int32_t* xv, const int32_t* buf, int32_t* deg) {
  if (n > 0) k_vp_xscatter_deg<<<vgrid(n, 4, 4096), 256, 0, s>>>(n, xv, buf, deg);
}
void launch_vp_lanes(hipStream_t s, const unsigned long long* lanechg, int step, unsigned long long* w) {
  k_vp_lanes<<<1, 64, 0, s>>>(lanechg, step, w);
}
void launch_vp_vote(hipStream_t s, const unsigned long long* w, int step, int32_t* stepflag,
                    unsigned long long* lanechg) {
  k_vp_vote<<<1, 64, 0, s>>>(w, step, stepflag, lanechg);
}
}  // namespace rgpu
