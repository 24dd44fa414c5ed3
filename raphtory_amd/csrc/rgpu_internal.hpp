// rgpu_internal.hpp — shared declarations of librgpu (host packer + HIP kernels + C ABI).
#pragma once
#include <cstdint>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/rgpu.h"

namespace rgpu {

// Packed, sealed graph of one partition.  All arrays are SoA.
// History keys are  key = t*2 + alive  so that one int64 compare orders (time, flag)
// and `key <= 2*t+1` finds floor(t) (Entity.closestTime, Entity.scala:173-183).
struct Packed {
  int64_t nv = 0, ne = 0;
  std::vector<int64_t> vid;          // [nv] vertex ids, ascending; rank = index
  std::vector<int64_t> voff, vkey;   // vertex histories: [nv+1], [voff[nv]]
  std::vector<int64_t> doff, dtime;  // vertex death times (VertexDelete), ascending, distinct
  std::vector<int32_t> esrc, edst;   // [ne] edge endpoints (ranks), sorted by (src, dst)
  std::vector<int64_t> eoff, ekey;   // edge own histories, ties vs endpoint deaths pre-resolved
  std::vector<int64_t> out_off;      // [nv+1] out-edges of rank v are edges [out_off[v], out_off[v+1])
  std::vector<int64_t> in_off;       // [nv+1] in-edges (no self-loops), ordered by (dst, src)
  std::vector<int32_t> in_eid;       // [in_off[nv]] edge ids of in-edges
  int64_t newest = -1;
  int64_t n_vkey = 0, n_ekey = 0, n_in = 0;  // sizes (the big arrays are dropped after upload)
  int64_t ne_owned = 0;              // edges whose source is owned here (their sum over the
                                     // partitions is the graph's edge entities)
  // ---- vertex partitioning (num_partitions > 1); identity when P = 1
  int part = 0, nparts = 1;
  int64_t n_own = 0;                 // ranks [0, n_own) are owned here, [n_own, nv) are ghosts
  // ---- local rank order (pack_events `locality`): ranks are ids ascending, or (relabeled) a
  // locality order: vertices by activity, most active first
  bool relabeled = false;
  std::vector<int64_t> lid;          // P = 1 relabeled: id of label l (labels are id ranks)
  std::vector<int32_t> by_id;        // relabeled: owned local ranks in ascending id order
  std::vector<int32_t> grank;        // [nv] CC label of each local rank: its vertex id (P > 1) or
                                     // its id rank (P = 1 relabeled); empty: the rank itself
  std::vector<uint8_t> lowner;       // [nv] owning partition of each local rank (P > 1)
  // exchange plan: per peer q, owned ranks that are ghosts on q (xs) and ghosts owned by q
  // (xr), both ascending by id, so q's xr list for this partition equals this xs list for q
  std::vector<int64_t> xs_off, xr_off;  // [P+1]
  std::vector<int32_t> xs_v, xr_v, xs_q, xr_q;
};

// Utils.getPartition (S/core/utils/Utils.scala:32-33): (|id| mod 10P) div 10
inline int partition_of(int64_t id, int nparts) {
  const int64_t a = id < 0 ? -id : id;
  return (int)((a % (10 * (int64_t)nparts)) / 10);
}

// What a partition keeps of the update stream (partitioned mode, rgpu_ingest): every update of
// an owned vertex, every edge update with an owned endpoint (the reference routes an edge to
// its source's PM and copies it to the destination's as a SplitEdge, EntityStorage.scala:
// 237-314), and every VertexDelete (an endpoint death kills the edges of any partition,
// killList / RemoteReturnDeaths, raphtoryMessages.scala:62,65).  So a rank holds O(stream/P)
// updates whether it is handed the whole stream or only this part of it.
inline bool partition_keeps(uint8_t kind, int64_t src, int64_t dst, int part, int nparts) {
  if (nparts <= 1 || kind == RGPU_VDEL) return true;
  if (partition_of(src, nparts) == part) return true;
  return kind >= RGPU_EADD && partition_of(dst, nparts) == part;
}

struct Event {
  int64_t t;
  int64_t src, dst;
  uint8_t kind;
};

// Host packer (packer.cpp).  Returns empty string or an error message.
// locality = true: local ranks in locality order (Packed.relabeled); false: ids ascending
std::string pack_events(const std::vector<Event>& ev, int partition, int num_partitions,
                        Packed* out, bool locality = false);
// locality order of n vertices from their activity: position -> index in [0, n)
std::vector<int32_t> locality_order(const std::vector<int32_t>& act, int nt);

// Incremental seal (live ingest), host half.  Updates ev[first, n)
// arrive after a sealed one-partition base; every one of them comes later in stream order
// than every base update, so at equal times a delta put wins (TreeMap put-overwrite,
// Entity.scala:25).  Only delta-sized work and O(V) offset arrays stay on the host; the big
// history / edge / in-edge arrays are merged in HBM (merge.hip).  Ranks below are in the
// merged rank space unless named old.
struct Delta {
  int64_t nv_old = 0, nv = 0, nd = 0;  // nd = delta updates
  std::vector<int64_t> vid;             // merged ids (rank = index)
  std::vector<int32_t> old2new, new2old;
  // delta vertex points per rank, collapsed (last put wins), ranks ascending
  std::vector<int32_t> dv_rank;
  std::vector<int64_t> dv_off, dv_key;
  // delta deaths (VertexDelete): distinct times per rank, with the last delta index (1-based)
  std::vector<int32_t> dd_rank;
  std::vector<int64_t> dd_off, dd_t, dd_last;
  // delta edges: distinct (s, d), ascending; old ranks (-1: endpoint is new) for the base lookup
  std::vector<int32_t> de_s, de_d, de_qs, de_qd;
  std::vector<int64_t> de_poff, de_pt, de_pidx;  // raw points per edge, by (t, idx); idx 1-based
  std::vector<uint8_t> de_pflag;
  // after the base lookup (finish_delta)
  std::vector<int32_t> de_base;          // base edge id or -1 (new edge)
  std::vector<int64_t> de_koff, de_key;  // collapsed, tie-resolved own points
  std::vector<int64_t> nn_key;           // new edges: (s << 32) | d ascending
  std::vector<int32_t> nn_didx;          // their delta edge index
  std::vector<int64_t> ni_key;           // new non-loop edges by (d << 32) | s ascending
  std::vector<int32_t> ni_idx;           // their index in nn_*
  std::vector<int64_t> out_off, in_off, doff, dtime;  // merged
};
std::string pack_delta(const std::vector<Event>& ev, size_t first, const Packed& base, Delta* out);
void finish_delta(const Packed& base, const std::vector<int32_t>& base_eid, Delta* d);

}  // namespace rgpu
