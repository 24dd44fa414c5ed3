// RGPU_CHECK=1 (debugging): structural checks of the resident graph after a seal and of K2's
// output after the slot kernel.  Every read is in bounds by construction (no index taken from
// the data under test is dereferenced), so a corrupt array is reported as a count, never as a
// memory fault.  Counters (bad[i]):
//   0 edge endpoint out of [0, V)        1 out_off not monotone / out_off[V] != E
//   2 in_off not monotone / in_off[V] != E_in                 3 in_eid out of [0, E)
//   4 eoff not monotone / eoff[E] != N_ep                      5 voff not monotone / voff[V] != N_vp
//   6 ts_e out of [0, E)                 7 ts_nb out of [0, V)   9 adj_off != out_off + in_off
//   10 member's kept count above its static degree             11 kept neighbour out of [0, V)
//   12 member's uniform word neither kMixed nor in [0, V)      13 uw0 != own rank
//   14 final uniform label out of [0, V)                       15 final mixed row label out of [0, V)
#include "kernels.hpp"

namespace rgpu {

namespace {

__device__ __forceinline__ void bump(unsigned long long* bad, int i) { atomicAdd(&bad[i], 1ull); }

__global__ __launch_bounds__(256) void k_check_graph(DevGraph g, int64_t n_ekey, int64_t n_vkey,
                                                     unsigned long long* bad) {
  const int64_t tid = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  const int64_t nth = (int64_t)gridDim.x * blockDim.x;
  for (int64_t e = tid; e < g.ne; e += nth) {
    if (g.esrc[e] < 0 || g.esrc[e] >= g.nv || g.edst[e] < 0 || g.edst[e] >= g.nv) bump(bad, 0);
    if (g.eoff[e] > g.eoff[e + 1]) bump(bad, 4);
  }
  for (int64_t v = tid; v < g.nv; v += nth) {
    if (g.out_off[v] > g.out_off[v + 1]) bump(bad, 1);
    if (g.in_off[v] > g.in_off[v + 1]) bump(bad, 2);
    if (g.voff[v] > g.voff[v + 1]) bump(bad, 5);
    if (g.adj_off[v] != g.out_off[v] + g.in_off[v]) bump(bad, 9);
  }
  if (tid == 0) {
    if (g.out_off[g.nv] != g.ne) bump(bad, 1);
    if (g.in_off[g.nv] != g.n_in) bump(bad, 2);
    if (n_ekey >= 0 && g.eoff[g.ne] != n_ekey) bump(bad, 4);
    if (n_vkey >= 0 && g.voff[g.nv] != n_vkey) bump(bad, 5);
    if (g.adj_off[g.nv] != g.ne + g.n_in) bump(bad, 9);
  }
  for (int64_t i = tid; i < g.n_in; i += nth)
    if (g.in_eid[i] < 0 || g.in_eid[i] >= g.ne) bump(bad, 3);
  if (g.ts_e)
    for (int64_t p = tid; p < g.ne + g.n_in; p += nth) {
      if (g.ts_e[p] < 0 || g.ts_e[p] >= g.ne) bump(bad, 6);
      if (g.ts_nb[p] < 0 || g.ts_nb[p] >= g.nv) bump(bad, 7);
    }
}

// nv: the vertices whose slots are checked (partitioned: the owned ones); nv_all: every local rank (a
// kept slot of an owned vertex may name a ghost)
__global__ __launch_bounds__(256) void k_check_slots(int64_t nv, int64_t nv_all, const int64_t* __restrict__ adj_off,
                                                     const uint64_t* __restrict__ vm, const int32_t* __restrict__ cnt,
                                                     const int32_t* __restrict__ snbr, const int32_t* __restrict__ uw0,
                                                     const int32_t* __restrict__ uw1, const int32_t* __restrict__ grank,
                                                     unsigned long long* bad) {
  const int64_t tid = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  const int64_t nth = (int64_t)gridDim.x * blockDim.x;
  for (int64_t v = tid; v < nv; v += nth) {
    if (!vm[v]) continue;
    const int64_t deg = adj_off[v + 1] - adj_off[v];
    const int64_t n = cnt[v];
    if (n < 0 || n > deg) {
      bump(bad, 10);
      continue;
    }
    for (int64_t k = 0; k < n; k++) {
      const int32_t q = snbr[adj_off[v] + k];
      if (q < 0 || q >= nv_all) bump(bad, 11);
    }
    if (uw0) {
      const int32_t me = grank ? grank[v] : (int32_t)v;
      if (uw0[v] != (me == INT32_MAX ? -1 : me)) bump(bad, 13);
      const int32_t u1 = uw_label(uw1[v]);
      if (u1 != -1 && (u1 < 0 || (!grank && u1 >= nv))) bump(bad, 12);
    }
  }
}

__global__ __launch_bounds__(256) void k_check_labels(int64_t nv, const uint64_t* __restrict__ vm,
                                                      const int32_t* __restrict__ uw, const int32_t* __restrict__ lab,
                                                      const int32_t* __restrict__ grank, unsigned long long* bad) {
  const int64_t tid = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  const int64_t nth = (int64_t)gridDim.x * blockDim.x;
  for (int64_t v = tid; v < nv; v += nth) {
    const uint64_t m = vm[v];
    if (!m) continue;
    const int32_t x = uw ? uw_label(uw[v]) : -1;
    if (x != -1) {
      if (x < 0 || (!grank && x >= nv)) bump(bad, 14);
      continue;
    }
    for (int j = 0; j < 64; j++)
      if ((m >> j) & 1) {
        const int32_t l = lab[v * 64 + j];
        if (l < 0 || (!grank && l >= nv)) bump(bad, 15);
      }
  }
}

}  // namespace

void launch_check_labels(hipStream_t s, int64_t nv, const uint64_t* vm, const int32_t* uw, const int32_t* lab,
                         unsigned long long* bad, const int32_t* grank) {
  k_check_labels<<<1024, 256, 0, s>>>(nv, vm, uw, lab, grank, bad);
}
void launch_check_graph(hipStream_t s, const DevGraph& g, int64_t n_ekey, int64_t n_vkey, unsigned long long* bad) {
  k_check_graph<<<1024, 256, 0, s>>>(g, n_ekey, n_vkey, bad);
}
void launch_check_slots(hipStream_t s, int64_t nv, int64_t nv_all, const int64_t* adj_off, const uint64_t* vm,
                        const int32_t* cnt, const int32_t* snbr, const int32_t* uw0, const int32_t* uw1,
                        unsigned long long* bad, const int32_t* grank) {
  k_check_slots<<<1024, 256, 0, s>>>(nv, nv_all, adj_off, vm, cnt, snbr, uw0, uw1, grank, bad);
}

}  // namespace rgpu
