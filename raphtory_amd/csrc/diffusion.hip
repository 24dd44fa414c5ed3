// BinaryDefusion on the GPU: generic VertexVisitor messaging for an
// infection analyser, S/core/analysis/Algorithms/BinaryDefusion.scala:9-51.
//
//   setup (superstep 0, only when defineMaxSteps > 1, AnalysisTask.scala:169): the seed
//     vertex (infectedNode, :10), if it is in the view, records infected = 0 (:15) and
//     messages each out-neighbour on a coin flip (:16-18);
//   superstep r: every view member holding messages (WindowLens.getVerticesWithMessages)
//     clears its queue; if already infected it votes to halt (:27-28), else it records
//     infected = r (:30) and messages each out-neighbour on a coin flip (:31-33);
//   halt when every message holder voted (no new infection) or after step 100 (:51).
//
// Random.nextBoolean() is unseeded in the reference, so no run of it is reproducible.  Here
// the coin is a fixed hash of (coin seed, hop time, window, sender id, receiver id, send
// step), specified in include/rgpu.h, and the oracle (oracle/oracle.c:orc_diffusion) uses
// the same coin, so GPU and oracle runs are bit-comparable.  coin = 0 sends every message:
// the deterministic taint (reachability by superstep) form of the same analyser.
//
// Layout: lane = view (64 per batch), as in CC.  Per vertex: inf (u64, infected views),
// front[2] (u64, views infected in the previous / this step), and a u8 row of 64 infection
// steps (0xFF = not infected).  One wave per vertex pulls over its in-edges (in_off /
// in_eid), 64 in-edges per load round: a message from u reaches v in view j iff u was infected in j at step r-1, the
// edge is alive in j (K1 edge mask: own history + endpoint deaths) and the coin is heads;
// v takes it iff v is a member of j and not yet infected there.  Bound: one pass over the
// in-CSR per superstep (HBM / Infinity-Cache gathers), no MFMA.
#include "kernels.hpp"

namespace rgpu {

__device__ __forceinline__ uint64_t dmix64(uint64_t x) {
  x ^= x >> 30;
  x *= 0xbf58476d1ce4e5b9ull;
  x ^= x >> 27;
  x *= 0x94d049bb133111ebull;
  x ^= x >> 31;
  return x;
}

// include/rgpu.h: coin(u, v, r, salt) = top bit of mix(salt ^ mix(u*phi ^ mix(v + r)))
__device__ __forceinline__ bool diff_coin(uint64_t salt, int64_t u, int64_t v, int r) {
  const uint64_t a = dmix64((uint64_t)v + (uint64_t)(int64_t)r);
  const uint64_t b = dmix64(((uint64_t)u * 0x9E3779B97F4A7C15ull) ^ a);
  return (dmix64(salt ^ b) >> 63) != 0;
}

// superstep 0: clear the batch state; the seed (rank `seed`, < 0 if absent) is infected in
// every view it belongs to, at step 0, and its out-neighbours are flagged active for step 1
// (act1 was cleared by the batch's first kernel).  Rows are written as u64 words (8 views).
__global__ __launch_bounds__(256) void k_diff_setup(int64_t nv, const uint64_t* __restrict__ vm, int64_t seed,
                                                    const int64_t* __restrict__ out_off,
                                                    const int32_t* __restrict__ edst,
                                                    uint64_t* __restrict__ inf, uint64_t* __restrict__ front0,
                                                    uint8_t* __restrict__ act1,
                                                    uint64_t* __restrict__ steprow,
                                                    unsigned long long* __restrict__ stats) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int64_t i0 = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  for (int64_t v = i0; v < nv; v += stride) {
    const uint64_t m = v == seed ? vm[v] : 0;
    inf[v] = m;
    front0[v] = m;
    if (m)
      for (uint64_t b = m; b; b &= b - 1) atomicAdd(&stats[__builtin_ctzll(b)], 1ull);  // infected counts
  }
  // the seed's out-neighbours, spread over the whole grid (a hub seed has millions)
  if (seed >= 0 && vm[seed])
    for (int64_t k = out_off[seed] + i0; k < out_off[seed + 1]; k += stride) act1[edst[k]] = 1;
  if (!steprow) return;  // rows only when the run retains per-vertex results
  for (int64_t i = i0; i < nv * 8; i += stride) {
    uint64_t w = ~0ull;
    if (i / 8 == seed) {
      const uint64_t m = vm[seed] >> ((i & 7) * 8);
      for (int b = 0; b < 8; b++)
        if ((m >> b) & 1) w &= ~(0xffull << (8 * b));  // infected = superStep 0 (:15)
    }
    steprow[i] = w;
  }
}

// Superstep `step`.  Only vertices flagged active (an in-neighbour was newly infected at
// step-1, flagged by that step) can receive a message.  A wave takes 64 vertices (lane =
// vertex: flags, masks, front stores coalesced), then for each active candidate pulls its
// in-edges 64 at a time (lane = in-edge) and flips the coins of the edges carrying a
// message (lane = view).  A newly infected vertex flags its out-neighbours for step+1.
// Flag buffers rotate over three steps: read act_cur, write act_next, clear act_clear.
__global__ __launch_bounds__(256) void k_diff_step(int step, int64_t nv, const int64_t* __restrict__ in_off,
                                                   const int32_t* __restrict__ in_eid,
                                                   const int32_t* __restrict__ esrc,
                                                   const int64_t* __restrict__ out_off,
                                                   const int32_t* __restrict__ edst,
                                                   const int64_t* __restrict__ vid,
                                                   const uint64_t* __restrict__ vm,
                                                   const uint64_t* __restrict__ em,
                                                   uint64_t* __restrict__ inf,
                                                   const uint64_t* __restrict__ front_in,
                                                   uint64_t* __restrict__ front_out,
                                                   const uint8_t* __restrict__ act_cur,
                                                   uint8_t* __restrict__ act_next,
                                                   uint8_t* __restrict__ act_clear,
                                                   uint8_t* __restrict__ steprow, DiffSalts salts, int coin,
                                                   int32_t* __restrict__ stepflag,
                                                   int32_t* __restrict__ hostflag,
                                                   unsigned long long* __restrict__ stats) {
  if (step >= 2 && stepflag[step - 1] == 0) return;  // halted: nobody was infected at step-1
  __shared__ int32_t red;
  __shared__ unsigned int acc[64];  // newly infected per view, this block
  if (threadIdx.x == 0) red = 0;
  if (threadIdx.x < 64) acc[threadIdx.x] = 0;
  const int64_t nwords = (nv + 7) >> 3;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < nwords;
       i += (int64_t)gridDim.x * blockDim.x)
    reinterpret_cast<uint64_t*>(act_clear)[i] = 0;
  __syncthreads();
  unsigned int mycnt = 0;  // lane j: vertices this wave infected in view j
  const int lane = threadIdx.x & 63;
  const uint64_t salt = salts.s[lane];
  const int64_t wave = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  int32_t changed = 0;
  for (int64_t c = wave; c * 64 < nv; c += nwaves) {
    const int64_t v = c * 64 + lane;
    const bool in = v < nv;
    const bool a = in && act_cur[v] != 0;
    const uint64_t infl = a ? inf[v] : 0;
    const uint64_t cand_l = a ? (vm[v] & ~infl) : 0;  // members not yet infected
    uint64_t newly_l = 0;
    uint64_t todo = __ballot(cand_l != 0);
    while (todo) {
      const int l = __builtin_ctzll(todo);
      todo &= todo - 1;
      const int64_t vv = c * 64 + l;
      const uint64_t cand = __shfl(cand_l, l);
      const int64_t k0 = in_off[vv], k1 = in_off[vv + 1];
      const int64_t myid = vid[vv];
      bool hit = false;
      for (int64_t base = k0; base < k1; base += 64) {
        const int64_t k = base + lane;
        uint64_t f = 0;
        int32_t u = 0;
        if (k < k1) {
          const int32_t e = in_eid[k];
          u = esrc[e];
          f = front_in[u] & em[e] & cand;
        }
        uint64_t msg = __ballot(f != 0);
        while (msg) {
          const int m = __builtin_ctzll(msg);
          msg &= msg - 1;
          const uint64_t fm = __shfl(f, m);
          const int32_t um = __shfl(u, m);
          if (!hit && ((fm >> lane) & 1)) hit = coin ? diff_coin(salt, vid[um], myid, step - 1) : true;
        }
        if ((__ballot(hit) & cand) == cand) break;  // every candidate view already infected
      }
      const uint64_t newly = __ballot(hit) & cand;
      if (newly) {
        if (lane == l) newly_l = newly;
        if ((newly >> lane) & 1) {
          if (steprow) steprow[vv * 64 + lane] = (uint8_t)step;
          mycnt++;
        }
        for (int64_t k = out_off[vv] + lane; k < out_off[vv + 1]; k += 64) act_next[edst[k]] = 1;
      }
    }
    if (in) {
      front_out[v] = newly_l;
      if (newly_l) inf[v] = infl | newly_l;
    }
    changed |= newly_l != 0;
  }
  if (changed) red = 1;
  if (mycnt) atomicAdd(&acc[lane], mycnt);
  __syncthreads();
  if (threadIdx.x == 0 && red && stepflag[step] == 0) {
    stepflag[step] = 1;
    if (hostflag) hostflag[step] = 1;
  }
  if (red && threadIdx.x < 64 && acc[threadIdx.x])
    atomicAdd(&stats[threadIdx.x], (unsigned long long)acc[threadIdx.x]);
}

static unsigned dgrid(int64_t items, int per_block, unsigned cap) {
  int64_t g = (items + per_block - 1) / per_block;
  if (g < 1) g = 1;
  return (unsigned)(g > cap ? cap : g);
}

void launch_diff_setup(hipStream_t s, const DevGraph& g, const uint64_t* vm, int64_t seed, uint64_t* inf,
                       uint64_t* front0, uint8_t* act1, uint8_t* steprow, unsigned long long* stats) {
  k_diff_setup<<<dgrid(steprow ? g.nv * 8 : g.nv, 256, 4096), 256, 0, s>>>(
      g.nv, vm, seed, g.out_off, g.edst, inf, front0, act1, reinterpret_cast<uint64_t*>(steprow), stats);
}

void launch_diff_step(hipStream_t s, int step, const DevGraph& g, const int64_t* vid, const uint64_t* vm,
                      const uint64_t* em, uint64_t* inf, const uint64_t* front_in, uint64_t* front_out,
                      const uint8_t* act_cur, uint8_t* act_next, uint8_t* act_clear, uint8_t* steprow,
                      const DiffSalts& salts, int coin, int32_t* stepflag, int32_t* hostflag,
                      unsigned long long* stats) {
  k_diff_step<<<dgrid(g.nv, 256, 1024), 256, 0, s>>>(step, g.nv, g.in_off, g.in_eid, g.esrc, g.out_off, g.edst,
                                                      vid, vm, em, inf, front_in, front_out, act_cur, act_next,
                                                      act_clear, steprow, salts, coin, stepflag, hostflag, stats);
}

}  // namespace rgpu
