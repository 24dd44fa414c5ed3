// packer.cpp — host-side sort + merge + pack of an update stream into SoA histories.
//
// The reference builds histories incrementally, one actor message at a time, in
// EntityStorage (S/core/storage/EntityStorage.scala:73-453, S = mainproject/cluster/src/
// main/scala/com/raphtory/).  Only the final (quiescent) history matters to the analysis
// path, so here the whole stream is sorted once and the same final state is derived:
//
//  vertex v:  + at every VertexAdd(v) (:73-87) and every EdgeAdd touching v as src or dst
//             (:240, :259); - at every VertexDelete(v) (:148-157).  EdgeDelete only creates
//             empty placeholders (:89-97) — an entity with no points.
//  edge u->v: + at EdgeAdd(u,v) (:250, revive :269); - at EdgeDelete(u,v) (:341, :366);
//             and - at EVERY VertexDelete of u or v, whenever it happened: new edges copy
//             the endpoints' removeList (killList, Edge.scala:36-44; :262, :277-278) and
//             existing edges are killed (:189-228).
//  equal keys collapse, last put wins (TreeMap, Entity.scala:25).
//
// Endpoint deaths are NOT copied into every edge (a hub with many deaths would multiply
// its degree by its death count).  They stay in per-vertex death lists, and the window
// kernel applies them.  The one place that needs stream order — an own
// edge point and an endpoint death at the same time — is resolved here, per point, as the
// reference's put order resolves it: a death that happened before the edge existed is
// applied right after the edge's creation (killList at creation), later deaths at their
// own stream position.
//
// Parallel layout (std::thread, RGPU_THREADS, default min(16, cores)): ids are sorted by
// chunk sort + pairwise merges; every record is then scattered by entity rank (counting
// sort, one atomic cursor per rank) and each entity's small segment is sorted on its own.
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <atomic>
#include <cstdlib>
#include <cstring>
#include <thread>

#include "rgpu_internal.hpp"

namespace rgpu {
namespace {

struct VPoint {
  int64_t t, idx;
  uint8_t flag;
};
struct EPoint {
  int32_t d;
  uint8_t flag;
  int64_t t, idx;
};
struct Death {
  int64_t t, idx;
};

int num_threads() {
  const char* e = std::getenv("RGPU_THREADS");
  int t = e && *e ? std::atoi(e) : 0;
  if (t <= 0) {
    t = (int)std::thread::hardware_concurrency();
    if (t > 16) t = 16;  // a GPU box's CPU share
  }
  return t < 1 ? 1 : t;
}

// run f(lo, hi, tid) over [0, n) in T contiguous chunks
template <class F>
void parallel_for(size_t n, int T, F f) {
  if (T <= 1 || n < 4096) {
    f((size_t)0, n, 0);
    return;
  }
  std::vector<std::thread> th;
  for (int k = 0; k < T; k++) {
    const size_t lo = n * k / T, hi = n * (k + 1) / T;
    th.emplace_back([=, &f] { f(lo, hi, k); });
  }
  for (auto& x : th) x.join();
}

template <class T, class C>
void parallel_sort(std::vector<T>& v, int nt, C cmp) {
  const size_t n = v.size();
  if (nt <= 1 || n < (1u << 16)) {
    std::sort(v.begin(), v.end(), cmp);
    return;
  }
  int parts = 1;
  while (parts * 2 <= nt) parts *= 2;
  std::vector<size_t> cut(parts + 1);
  for (int k = 0; k <= parts; k++) cut[k] = n * k / parts;
  {
    std::vector<std::thread> th;
    for (int k = 0; k < parts; k++)
      th.emplace_back([&, k] { std::sort(v.begin() + cut[k], v.begin() + cut[k + 1], cmp); });
    for (auto& x : th) x.join();
  }
  std::vector<T> buf(n);
  std::vector<T>* src = &v;
  std::vector<T>* dst = &buf;
  for (int w = 1; w < parts; w *= 2) {
    std::vector<std::thread> th;
    for (int k = 0; k < parts; k += 2 * w)
      th.emplace_back([&, k] {
        const size_t a = cut[k], m = cut[k + w], b = cut[std::min(k + 2 * w, parts)];
        std::merge(src->begin() + a, src->begin() + m, src->begin() + m, src->begin() + b,
                   dst->begin() + a, cmp);
      });
    for (auto& x : th) x.join();
    std::swap(src, dst);
  }
  if (src != &v) v.swap(*src);
}

// counting-sort scatter: key(i) in [0, nkeys) -> records grouped by key, offsets in off[nkeys+1]
template <class R, class KeyF, class MakeF>
void group_by_key(size_t n, int64_t nkeys, int nt, KeyF key, MakeF make, std::vector<int64_t>& off,
                  std::vector<R>& out) {
  off.assign(nkeys + 1, 0);
  std::vector<std::atomic<int64_t>> cnt(nkeys + 1);
  for (auto& c : cnt) c.store(0, std::memory_order_relaxed);
  parallel_for(n, nt, [&](size_t lo, size_t hi, int) {
    for (size_t i = lo; i < hi; i++) {
      const int64_t k = key(i);
      if (k >= 0) cnt[k + 1].fetch_add(1, std::memory_order_relaxed);
    }
  });
  for (int64_t k = 0; k < nkeys; k++) off[k + 1] = off[k] + cnt[k + 1].load(std::memory_order_relaxed);
  for (int64_t k = 0; k <= nkeys; k++) cnt[k].store(off[k], std::memory_order_relaxed);
  out.resize(off[nkeys]);
  parallel_for(n, nt, [&](size_t lo, size_t hi, int) {
    for (size_t i = lo; i < hi; i++) {
      const int64_t k = key(i);
      if (k >= 0) out[cnt[k].fetch_add(1, std::memory_order_relaxed)] = make(i);
    }
  });
}

// per-segment sorts, load-balanced by segment start (segments are small; hubs get a thread)
template <class R, class C>
void sort_segments(std::vector<R>& recs, const std::vector<int64_t>& off, int nt, C cmp) {
  const int64_t nseg = (int64_t)off.size() - 1;
  std::atomic<int64_t> next(0);
  auto work = [&] {
    for (;;) {
      const int64_t s0 = next.fetch_add(1024);
      if (s0 >= nseg) return;
      const int64_t s1 = std::min(nseg, s0 + 1024);
      for (int64_t s = s0; s < s1; s++)
        if (off[s + 1] - off[s] > 1) std::sort(recs.begin() + off[s], recs.begin() + off[s + 1], cmp);
    }
  };
  std::vector<std::thread> th;
  for (int k = 0; k < nt; k++) th.emplace_back(work);
  for (auto& x : th) x.join();
}

// Stable parallel LSD radix sort of (key, val) pairs on key bits [0, bits): <= 12-bit digits,
// per-thread digit histograms, each thread scattering its own contiguous input range in order.
template <class V>
void radix_sort_pairs(std::vector<uint64_t>& key, std::vector<V>& val, int bits, int nt) {
  const size_t n = key.size();
  if (n < 2 || bits <= 0) return;
  const int passes = (bits + 11) / 12;                // digits of at most 12 bits, as few passes as
  const int kD = (bits + passes - 1) / passes;         // possible (24-bit ranks: 2 x 12, 31-bit ids: 3 x 11)
  const size_t kNB = (size_t)1 << kD;
  const int T = n < (1u << 16) ? 1 : nt;
  std::vector<uint64_t> k2(n);
  std::vector<V> v2(n);
  std::vector<size_t> hist((size_t)T * kNB);
  auto run = [&](auto f) {
    if (T == 1) {
      f(0);
      return;
    }
    std::vector<std::thread> th;
    for (int q = 0; q < T; q++) th.emplace_back([&, q] { f(q); });
    for (auto& x : th) x.join();
  };
  for (int sh = 0; sh < bits; sh += kD) {
    std::fill(hist.begin(), hist.end(), 0);
    run([&](int q) {
      size_t* h = hist.data() + (size_t)q * kNB;
      for (size_t i = n * q / T, e = n * (q + 1) / T; i < e; i++) h[(key[i] >> sh) & (kNB - 1)]++;
    });
    size_t run_off = 0;
    for (size_t d = 0; d < kNB; d++)
      for (int q = 0; q < T; q++) {
        const size_t c = hist[(size_t)q * kNB + d];
        hist[(size_t)q * kNB + d] = run_off;
        run_off += c;
      }
    run([&](int q) {
      size_t* h = hist.data() + (size_t)q * kNB;
      for (size_t i = n * q / T, e = n * (q + 1) / T; i < e; i++) {
        const size_t o = h[(key[i] >> sh) & (kNB - 1)]++;
        k2[o] = key[i];
        v2[o] = val[i];
      }
    });
    key.swap(k2);
    val.swap(v2);
  }
}

// Parallel build of (key, val) pairs in stream order: emit(i, out) writes the 0..M pairs of
// item i (M = max_per) into out and returns how many; chunks are concatenated in order.
template <class Emit>
void build_pairs(size_t n, int nt, int max_per, std::vector<uint64_t>& key, std::vector<uint64_t>& val, Emit emit) {
  const int T = n < 4096 ? 1 : nt;
  std::vector<size_t> cnt(T + 1, 0);
  parallel_for(n, nt, [&](size_t lo, size_t hi, int q) {
    uint64_t k[4], v[4];
    size_t c = 0;
    for (size_t i = lo; i < hi; i++) c += emit(i, k, v);
    cnt[q + 1] = c;
  });
  for (int q = 0; q < T; q++) cnt[q + 1] += cnt[q];
  key.resize(cnt[T]);
  val.resize(cnt[T]);
  parallel_for(n, nt, [&](size_t lo, size_t hi, int q) {
    uint64_t k[4], v[4];
    size_t o = cnt[q];
    for (size_t i = lo; i < hi; i++) {
      const int m = emit(i, k, v);
      for (int j = 0; j < m; j++) {
        key[o] = k[j];
        val[o++] = v[j];
      }
    }
  });
  (void)max_per;
}

inline int bits_for(uint64_t maxv) {
  int b = 1;
  while (b < 64 && (maxv >> b)) b++;
  return b;
}

}  // namespace

// Locality order.  The superstep and K2 gather one random word per slot from the
// neighbour (uniform / change word, view mask); on a power-law graph most slots point at a few
// hubs.  Ranking vertices by activity (updates naming them, a proxy for degree), most active
// first, packs the hubs' words into few cache lines, so the hot set stays L2-resident.  The
// superstep kernel and K2 deal chunks / vertices to the waves cyclically, so the busy low ranks
// spread over every wave (kernels.hip).
std::vector<int32_t> locality_order(const std::vector<int32_t>& act, int nt) {
  const int64_t n = (int64_t)act.size();
  std::vector<uint64_t> key(n);
  parallel_for((size_t)n, nt, [&](size_t lo, size_t hi, int) {
    for (size_t i = lo; i < hi; i++) key[i] = ((uint64_t)(uint32_t)(INT32_MAX - act[i]) << 32) | (uint64_t)i;
  });
  parallel_sort(key, nt, std::less<uint64_t>());  // activity descending, index ascending
  std::vector<int32_t> ord(n);
  parallel_for((size_t)n, nt, [&](size_t lo, size_t hi, int) {
    for (size_t i = lo; i < hi; i++) ord[i] = (int32_t)(key[i] & 0xffffffffu);
  });
  return ord;
}

std::string pack_events(const std::vector<Event>& ev, int partition, int num_partitions,
                        Packed* out, bool locality) {
  if (num_partitions < 1 || partition < 0 || partition >= num_partitions) return "bad partition";
  const int nt = num_threads();
  const size_t n = ev.size();
  const int64_t kMaxT = (int64_t)1 << 61;
  for (const Event& e : ev) {
    if (e.kind > RGPU_EDEL) return "unknown update kind";
    if (e.t < 0 || e.t >= kMaxT) return "time out of range [0, 2^61)";
    if (e.src < 0 || e.src > INT32_MAX) return "vertex id out of range [0, 2^31)";
    if (e.kind >= RGPU_EADD && (e.dst < 0 || e.dst > INT32_MAX)) return "vertex id out of range [0, 2^31)";
  }
  Packed& P = *out;
  P = Packed();
  P.part = partition;
  P.nparts = num_partitions;
  // ---- vertex ids: sorted, distinct; global rank = position
  std::vector<int64_t> ids;
  ids.reserve(n * 2);
  int64_t newest = -1;
  for (const Event& e : ev) {
    ids.push_back(e.src);
    if (e.kind >= RGPU_EADD) ids.push_back(e.dst);
    newest = std::max(newest, e.t);
  }
  parallel_sort(ids, nt, std::less<int64_t>());
  ids.erase(std::unique(ids.begin(), ids.end()), ids.end());
  P.newest = newest;
  std::vector<int32_t> rs(n), rd(n, -1);
  parallel_for(n, nt, [&](size_t lo, size_t hi, int) {
    for (size_t i = lo; i < hi; i++) {
      rs[i] = (int32_t)(std::lower_bound(ids.begin(), ids.end(), ev[i].src) - ids.begin());
      if (ev[i].kind >= RGPU_EADD)
        rd[i] = (int32_t)(std::lower_bound(ids.begin(), ids.end(), ev[i].dst) - ids.begin());
    }
  });
  // activity of every id (updates naming it): the locality order's ranking
  std::vector<int32_t> act;
  if (locality) {
    std::vector<std::atomic<int32_t>> a(ids.size());
    parallel_for(ids.size(), nt, [&](size_t lo, size_t hi, int) {
      for (size_t g = lo; g < hi; g++) a[g].store(0, std::memory_order_relaxed);
    });
    parallel_for(n, nt, [&](size_t lo, size_t hi, int) {
      for (size_t i = lo; i < hi; i++) {
        a[rs[i]].fetch_add(1, std::memory_order_relaxed);
        if (rd[i] >= 0 && rd[i] != rs[i]) a[rd[i]].fetch_add(1, std::memory_order_relaxed);
      }
    });
    act.resize(ids.size());
    for (size_t g = 0; g < ids.size(); g++) act[g] = a[g].load(std::memory_order_relaxed);
  }
  P.relabeled = locality;
  if (num_partitions == 1 && !locality) {
    P.nv = P.n_own = (int64_t)ids.size();
    P.vid = std::move(ids);
  } else if (num_partitions == 1) {
    // labels stay id ranks (order-preserving); local rank = position in the locality order
    const int64_t nv = (int64_t)ids.size();
    const std::vector<int32_t> ord = locality_order(act, nt);
    std::vector<int32_t> pos(nv);
    P.nv = P.n_own = nv;
    P.vid.resize(nv);
    P.grank.resize(nv);
    parallel_for((size_t)nv, nt, [&](size_t lo, size_t hi, int) {
      for (size_t k = lo; k < hi; k++) {
        pos[ord[k]] = (int32_t)k;
        P.vid[k] = ids[ord[k]];
        P.grank[k] = ord[k];
      }
    });
    P.by_id = pos;
    P.lid = std::move(ids);
    parallel_for(n, nt, [&](size_t lo, size_t hi, int) {
      for (size_t i = lo; i < hi; i++) {
        rs[i] = pos[rs[i]];
        if (rd[i] >= 0) rd[i] = pos[rd[i]];
      }
    });
  } else {
    // Partition view (the reference's PM keeps its own vertices plus SplitEdge copies,
    // EntityStorage.scala:303-305): owned vertices, ghosts = other endpoints of edges that
    // touch an owned vertex.  The partition keeps (rgpu_ingest) every update of its own
    // vertices, every edge update with an owned endpoint and every VertexDelete, so owned
    // histories, kept edges' histories and every endpoint's deaths (killList) are complete;
    // a ghost's vertex history is not (its membership comes from its owner, per hop block).
    // Local rank order: owned by id, then ghosts by id; CC labels are vertex ids.
    const int64_t ng = (int64_t)ids.size();
    std::vector<std::atomic<uint8_t>> role(ng);  // 0 owned, 1 ghost, 2 not kept
    parallel_for((size_t)ng, nt, [&](size_t lo, size_t hi, int) {
      for (size_t g = lo; g < hi; g++)
        role[g].store(partition_of(ids[g], num_partitions) == partition ? 0 : 2, std::memory_order_relaxed);
    });
    parallel_for(n, nt, [&](size_t lo, size_t hi, int) {
      for (size_t i = lo; i < hi; i++) {
        if (ev[i].kind < RGPU_EADD || rs[i] == rd[i]) continue;
        const bool so = role[rs[i]].load(std::memory_order_relaxed) == 0;
        const bool dn = role[rd[i]].load(std::memory_order_relaxed) == 0;
        if (so && !dn) role[rd[i]].store(1, std::memory_order_relaxed);
        if (dn && !so) role[rs[i]].store(1, std::memory_order_relaxed);
      }
    });
    std::vector<int32_t> g2l(ng, -1);
    for (int r = 0; r < 2; r++) {
      std::vector<int32_t> gs;  // global ranks of this role, ids ascending
      for (int64_t g = 0; g < ng; g++)
        if (role[g].load(std::memory_order_relaxed) == r) gs.push_back((int32_t)g);
      if (locality) {  // owned and ghost ranks each in their own locality order
        std::vector<int32_t> a(gs.size());
        for (size_t k = 0; k < gs.size(); k++) a[k] = act[gs[k]];
        const std::vector<int32_t> ord = locality_order(a, nt);
        std::vector<int32_t> o2(gs.size());
        for (size_t k = 0; k < gs.size(); k++) o2[k] = gs[ord[k]];
        if (r == 0) {  // owned local ranks in id order
          P.by_id.resize(gs.size());
          for (size_t k = 0; k < gs.size(); k++) P.by_id[ord[k]] = (int32_t)(P.vid.size() + k);
        }
        gs.swap(o2);
      }
      for (int32_t g : gs) {
        g2l[g] = (int32_t)P.vid.size();
        P.vid.push_back(ids[g]);
        P.grank.push_back((int32_t)ids[g]);  // label = id (ids < 2^31): order-preserving, global
        P.lowner.push_back((uint8_t)partition_of(ids[g], num_partitions));
        if (r == 0) P.n_own++;
      }
    }
    P.nv = (int64_t)P.vid.size();
    parallel_for(n, nt, [&](size_t lo, size_t hi, int) {
      for (size_t i = lo; i < hi; i++) {
        rs[i] = g2l[rs[i]];
        if (rd[i] >= 0) rd[i] = g2l[rd[i]];
      }
    });
  }
  const int64_t n_own = P.n_own;
  // an edge is kept iff both endpoints are kept and one of them is owned
  auto edge_kept = [&](size_t i) {
    return rs[i] >= 0 && rd[i] >= 0 && (rs[i] < n_own || rd[i] < n_own);
  };

  // ---- vertex histories: records grouped by rank (src of every update; dst of EdgeAdd unless
  // a self-loop), each segment sorted by (t, idx), equal t collapsed (last put wins)
  {
    // a record slot per (event, end): 2i = src side, 2i+1 = dst side
    auto vkey_of = [&](size_t j) -> int64_t {  // owned ranks only: a ghost's history is partial here
      const size_t i = j >> 1;
      const Event& e = ev[i];
      if (!(j & 1)) return e.kind == RGPU_EDEL || rs[i] < 0 || rs[i] >= n_own ? -1 : rs[i];
      return (e.kind == RGPU_EADD && rd[i] != rs[i] && rd[i] >= 0 && rd[i] < n_own) ? rd[i] : -1;
    };
    auto vmake = [&](size_t j) {
      const size_t i = j >> 1;
      return VPoint{ev[i].t, (int64_t)i, (uint8_t)(ev[i].kind == RGPU_VDEL ? 0 : 1)};
    };
    std::vector<int64_t> off;
    std::vector<VPoint> vp;
    group_by_key<VPoint>(2 * n, P.nv, nt, vkey_of, vmake, off, vp);
    sort_segments(vp, off, nt, [](const VPoint& a, const VPoint& b) {
      return a.t != b.t ? a.t < b.t : a.idx < b.idx;
    });
    // collapse: count distinct times per rank, then fill
    P.voff.assign(P.nv + 1, 0);
    parallel_for((size_t)P.nv, nt, [&](size_t lo, size_t hi, int) {
      for (size_t r = lo; r < hi; r++) {
        int64_t c = 0;
        for (int64_t k = off[r]; k < off[r + 1]; k++)
          if (k + 1 == off[r + 1] || vp[k + 1].t != vp[k].t) c++;
        P.voff[r + 1] = c;
      }
    });
    for (int64_t v = 0; v < P.nv; v++) P.voff[v + 1] += P.voff[v];
    P.vkey.resize(P.voff[P.nv]);
    parallel_for((size_t)P.nv, nt, [&](size_t lo, size_t hi, int) {
      for (size_t r = lo; r < hi; r++) {
        int64_t o = P.voff[r];
        for (int64_t k = off[r]; k < off[r + 1]; k++)
          if (k + 1 == off[r + 1] || vp[k + 1].t != vp[k].t) P.vkey[o++] = vp[k].t * 2 + vp[k].flag;
      }
    });
  }

  // ---- death lists: distinct VDEL times per rank, with the last stream index at each time
  std::vector<int64_t> dlast;
  {
    auto dkey = [&](size_t i) -> int64_t { return ev[i].kind == RGPU_VDEL && rs[i] >= 0 ? rs[i] : -1; };
    auto dmake = [&](size_t i) { return Death{ev[i].t, (int64_t)i}; };
    std::vector<int64_t> off;
    std::vector<Death> dd;
    group_by_key<Death>(n, P.nv, nt, dkey, dmake, off, dd);
    sort_segments(dd, off, nt, [](const Death& a, const Death& b) {
      return a.t != b.t ? a.t < b.t : a.idx < b.idx;
    });
    P.doff.assign(P.nv + 1, 0);
    for (int64_t r = 0; r < P.nv; r++) {
      int64_t c = 0;
      for (int64_t k = off[r]; k < off[r + 1]; k++)
        if (k + 1 == off[r + 1] || dd[k + 1].t != dd[k].t) {
          P.dtime.push_back(dd[k].t);
          dlast.push_back(dd[k].idx);
          c++;
        }
      P.doff[r + 1] = P.doff[r] + c;
    }
  }
  auto death_at = [&](int32_t r, int64_t t) -> int64_t {  // -1 if no death at exactly t
    auto b = P.dtime.begin() + P.doff[r], e = P.dtime.begin() + P.doff[r + 1];
    auto it = std::lower_bound(b, e, t);
    return (it != e && *it == t) ? dlast[it - P.dtime.begin()] : -1;
  };

  // ---- edge own histories: grouped by src rank, each src segment sorted by (dst, t, idx)
  {
    auto ekey = [&](size_t i) -> int64_t { return ev[i].kind >= RGPU_EADD && edge_kept(i) ? rs[i] : -1; };
    auto emake = [&](size_t i) {
      return EPoint{rd[i], (uint8_t)(ev[i].kind == RGPU_EADD ? 1 : 0), ev[i].t, (int64_t)i};
    };
    std::vector<int64_t> off;
    std::vector<EPoint> ep;
    group_by_key<EPoint>(n, P.nv, nt, ekey, emake, off, ep);
    sort_segments(ep, off, nt, [](const EPoint& a, const EPoint& b) {
      if (a.d != b.d) return a.d < b.d;
      if (a.t != b.t) return a.t < b.t;
      return a.idx < b.idx;
    });
    // per src: number of edges and of collapsed points (parallel), then fill
    std::vector<int64_t> ne_of(P.nv + 1, 0), np_of(P.nv + 1, 0);
    parallel_for((size_t)P.nv, nt, [&](size_t lo, size_t hi, int) {
      for (size_t r = lo; r < hi; r++) {
        int64_t ce = 0, cp = 0;
        for (int64_t k = off[r]; k < off[r + 1]; k++) {
          const bool last_of_edge = k + 1 == off[r + 1] || ep[k + 1].d != ep[k].d;
          if (last_of_edge) ce++;
          if (last_of_edge || ep[k + 1].t != ep[k].t) cp++;
        }
        ne_of[r + 1] = ce;
        np_of[r + 1] = cp;
      }
    });
    for (int64_t r = 0; r < P.nv; r++) { ne_of[r + 1] += ne_of[r]; np_of[r + 1] += np_of[r]; }
    P.ne = ne_of[P.nv];
    P.esrc.resize(P.ne);
    P.edst.resize(P.ne);
    P.eoff.assign(P.ne + 1, 0);
    P.ekey.resize(np_of[P.nv]);
    parallel_for((size_t)P.nv, nt, [&](size_t lo, size_t hi, int) {
      for (size_t r = lo; r < hi; r++) {
        int64_t e = ne_of[r], p = np_of[r];
        for (int64_t g = off[r]; g < off[r + 1];) {
          int64_t h = g, created = ep[g].idx;  // stream index of the edge's first update
          while (h < off[r + 1] && ep[h].d == ep[g].d) { created = std::min(created, ep[h].idx); h++; }
          for (int64_t k = g; k < h; k++) {
            if (k + 1 < h && ep[k + 1].t == ep[k].t) continue;  // collapse: last put wins
            uint8_t flag = ep[k].flag;
            // tie with an endpoint death at the same time: compare put positions (x2 so that
            // "right after creation" = 2*created+1 sits between two stream indices)
            int64_t pd = death_at((int32_t)r, ep[k].t);
            if (ep[k].d != (int32_t)r) pd = std::max(pd, death_at(ep[k].d, ep[k].t));
            if (pd >= 0) {
              const int64_t pd2 = pd < created ? 2 * created + 1 : 2 * pd;
              if (pd2 > 2 * ep[k].idx) flag = 0;
            }
            P.ekey[p++] = ep[k].t * 2 + flag;
          }
          P.esrc[e] = (int32_t)r;
          P.edst[e] = ep[g].d;
          P.eoff[e + 1] = p;
          e++;
          g = h;
        }
      }
    });
  }

  // ---- adjacency: out-edges by src (edge order), in-edges by (dst, src), self-loops
  // never enter incomingEdges (EntityStorage.scala:257)
  P.out_off.assign(P.nv + 1, 0);
  P.in_off.assign(P.nv + 1, 0);
  for (int64_t e = 0; e < P.ne; e++) {
    P.out_off[P.esrc[e] + 1]++;
    if (P.esrc[e] != P.edst[e]) P.in_off[P.edst[e] + 1]++;
  }
  for (int64_t v = 0; v < P.nv; v++) {
    P.out_off[v + 1] += P.out_off[v];
    P.in_off[v + 1] += P.in_off[v];
  }
  P.in_eid.assign(P.in_off[P.nv], 0);
  std::vector<int64_t> fill(P.in_off.begin(), P.in_off.end() - 1);
  for (int64_t e = 0; e < P.ne; e++)
    if (P.esrc[e] != P.edst[e]) P.in_eid[fill[P.edst[e]]++] = (int32_t)e;

  // ---- exchange plan (P > 1): an edge between owned v and ghost g (owner q) puts v on the
  // send list to q and g on the receive list from q; q derives the same pair from the same
  // edge, and both sides order by id, so entry i of our list for q is entry i of q's list
  const int np = num_partitions;
  std::vector<std::vector<int32_t>> S(np), R(np);
  if (np > 1)
    for (int64_t e = 0; e < P.ne; e++) {
      const int32_t a = P.esrc[e], b = P.edst[e];
      if ((a < n_own) == (b < n_own)) continue;
      const int32_t own = a < n_own ? a : b, gh = a < n_own ? b : a;
      const int q = partition_of(P.vid[gh], np);
      S[q].push_back(own);
      R[q].push_back(gh);
    }
  P.xs_off.assign(np + 1, 0);
  P.xr_off.assign(np + 1, 0);
  for (int q = 0; q < np; q++) {
    for (auto* L : {&S[q], &R[q]}) {  // by id (local ranks need not follow ids)
      std::sort(L->begin(), L->end(), [&](int32_t x, int32_t y) { return P.vid[x] < P.vid[y]; });
      L->erase(std::unique(L->begin(), L->end()), L->end());
    }
    P.xs_v.insert(P.xs_v.end(), S[q].begin(), S[q].end());
    P.xs_q.insert(P.xs_q.end(), S[q].size(), q);
    P.xr_v.insert(P.xr_v.end(), R[q].begin(), R[q].end());
    P.xr_q.insert(P.xr_q.end(), R[q].size(), q);
    P.xs_off[q + 1] = (int64_t)P.xs_v.size();
    P.xr_off[q + 1] = (int64_t)P.xr_v.size();
  }
  P.n_vkey = (int64_t)P.vkey.size();
  P.n_ekey = (int64_t)P.ekey.size();
  P.n_in = P.in_off[P.nv];
  P.ne_owned = 0;
  for (int64_t e = 0; e < P.ne; e++) P.ne_owned += P.esrc[e] < n_own;
  return "";
}

// ---------------------------------------------------------------------------------------
// Incremental seal, host half (rgpu_internal.hpp: Delta).  Delta indices are 1-based so
// that 0 can stand for "somewhere in the base": every base put precedes every delta put.
// RGPU_HOSTPROF=1: host phase times of the delta packer on stderr
struct PhaseTimer {
  const char* tag;
  bool on = std::getenv("RGPU_HOSTPROF") && std::atoi(std::getenv("RGPU_HOSTPROF")) != 0;
  std::chrono::steady_clock::time_point t = std::chrono::steady_clock::now();
  void operator()(const char* what) {
    if (!on) return;
    const auto n = std::chrono::steady_clock::now();
    std::fprintf(stderr, "[rgpu %s] %-12s %8.2f ms\n", tag, what, std::chrono::duration<double, std::milli>(n - t).count());
    t = n;
  }
};

std::string pack_delta(const std::vector<Event>& ev, size_t first, const Packed& B, Delta* out) {
  const int nt = num_threads();
  PhaseTimer ph{"pack_delta"};
  const size_t n = ev.size() - first;
  const int64_t kMaxT = (int64_t)1 << 61;
  for (size_t i = first; i < ev.size(); i++) {
    const Event& e = ev[i];
    if (e.kind > RGPU_EDEL) return "unknown update kind";
    if (e.t < 0 || e.t >= kMaxT) return "time out of range [0, 2^61)";
    if (e.src < 0 || e.src > INT32_MAX) return "vertex id out of range [0, 2^31)";
    if (e.kind >= RGPU_EADD && (e.dst < 0 || e.dst > INT32_MAX)) return "vertex id out of range [0, 2^31)";
  }
  ph("validate");
  Delta& D = *out;
  D = Delta();
  D.nd = (int64_t)n;
  D.nv_old = B.nv;
  // ---- ids: new ids merged into the base order; both rank maps are monotone.  Every id slot
  // (2i = src of update i, 2i+1 = its dst) is radix-sorted by id, so the ranks are scattered
  // back from the sorted order with no per-update search.
  std::vector<uint64_t> sk;
  std::vector<uint64_t> sv;
  {
    std::vector<size_t> cnt(nt + 1, 0);
    parallel_for(n, nt, [&](size_t lo, size_t hi, int q) {
      size_t c = 0;
      for (size_t i = lo; i < hi; i++) c += ev[first + i].kind >= RGPU_EADD ? 2 : 1;
      cnt[q + 1] = c;
    });
    const int used = n < 4096 ? 1 : nt;
    for (int q = 0; q < used; q++) cnt[q + 1] += cnt[q];
    sk.resize(cnt[used]);
    sv.resize(cnt[used]);
    parallel_for(n, nt, [&](size_t lo, size_t hi, int q) {
      size_t o = cnt[q];
      for (size_t i = lo; i < hi; i++) {
        const Event& e = ev[first + i];
        sk[o] = (uint64_t)e.src;
        sv[o++] = 2 * (uint64_t)i;
        if (e.kind >= RGPU_EADD) {
          sk[o] = (uint64_t)e.dst;
          sv[o++] = 2 * (uint64_t)i + 1;
        }
      }
    });
  }
  ph("ids build");
  radix_sort_pairs(sk, sv, 31, nt);
  ph("i radix");
  std::vector<int64_t> ids;  // distinct delta ids, ascending
  std::vector<uint32_t> uidx(sk.size());  // sorted slot -> index in ids
  for (size_t p = 0; p < sk.size(); p++) {
    if (p == 0 || sk[p] != sk[p - 1]) ids.push_back((int64_t)sk[p]);
    uidx[p] = (uint32_t)(ids.size() - 1);
  }
  ph("ids sort");
  // ids not in the base (parallel searches), then both rank maps by position formulas: base
  // id a lands at a + #(new ids below it), new id j at j + #(base ids below it)
  std::vector<uint8_t> isnew(ids.size());
  parallel_for(ids.size(), nt, [&](size_t lo, size_t hi, int) {
    for (size_t k = lo; k < hi; k++) isnew[k] = !std::binary_search(B.vid.begin(), B.vid.end(), ids[k]);
  });
  std::vector<int64_t> nid;
  for (size_t k = 0; k < ids.size(); k++)
    if (isnew[k]) nid.push_back(ids[k]);
  D.nv = B.nv + (int64_t)nid.size();
  D.vid.resize(D.nv);
  D.old2new.resize(B.nv);
  D.new2old.assign(D.nv, -1);
  parallel_for((size_t)B.nv, nt, [&](size_t lo, size_t hi, int) {
    if (lo >= hi) return;
    size_t b = std::lower_bound(nid.begin(), nid.end(), B.vid[lo]) - nid.begin();
    for (size_t a = lo; a < hi; a++) {
      while (b < nid.size() && nid[b] < B.vid[a]) b++;
      const size_t r = a + b;
      D.vid[r] = B.vid[a];
      D.old2new[a] = (int32_t)r;
      D.new2old[r] = (int32_t)a;
    }
  });
  parallel_for(nid.size(), nt, [&](size_t lo, size_t hi, int) {
    for (size_t j = lo; j < hi; j++)
      D.vid[j + (std::lower_bound(B.vid.begin(), B.vid.end(), nid[j]) - B.vid.begin())] = nid[j];
  });
  ph("id merge");
  // merged rank of every delta id (ids ascending, so one walk), then each update's ranks by
  // a search in the delta's own id list (much smaller than the graph's)
  std::vector<int32_t> idrank(ids.size());
  parallel_for(ids.size(), nt, [&](size_t lo, size_t hi, int) {
    if (lo >= hi) return;
    size_t r = std::lower_bound(D.vid.begin(), D.vid.end(), ids[lo]) - D.vid.begin();
    for (size_t k = lo; k < hi; k++) {
      while (D.vid[r] < ids[k]) r++;
      idrank[k] = (int32_t)r;
    }
  });
  std::vector<int32_t> rs(n), rd(n, -1);
  parallel_for(sk.size(), nt, [&](size_t lo, size_t hi, int) {
    for (size_t p = lo; p < hi; p++) {
      if (p + 16 < hi) __builtin_prefetch(&(sv[p + 16] & 1 ? rd : rs)[sv[p + 16] >> 1], 1);
      const uint64_t slot = sv[p];
      (slot & 1 ? rd : rs)[slot >> 1] = idrank[uidx[p]];
    }
  });
  std::vector<uint64_t>().swap(sk);
  std::vector<uint64_t>().swap(sv);
  std::vector<uint32_t>().swap(uidx);
  // times non-decreasing in stream order (the usual live case): a stable sort by entity then
  // already leaves each entity's points in (t, idx) order
  bool mono = true;
  for (size_t i = 1; i < n && mono; i++) mono = ev[first + i].t >= ev[first + i - 1].t;
  ph("ranks");
  // ---- vertex points (same records as pack_events), collapsed per (rank, t): last put wins
  {
    struct R { int32_t v; uint8_t f; int64_t t, idx; };
    std::vector<R> r;
    if (mono) {  // radix by rank over (update, endpoint) records built in stream order
      std::vector<uint64_t> key, val;
      build_pairs(n, nt, 2, key, val, [&](size_t i, uint64_t* k, uint64_t* v) {
        const uint8_t kd = ev[first + i].kind;
        int m = 0;
        if (kd != RGPU_EDEL) { k[m] = (uint64_t)rs[i]; v[m++] = 2 * (uint64_t)i; }
        if (kd == RGPU_EADD && rd[i] != rs[i]) { k[m] = (uint64_t)rd[i]; v[m++] = 2 * (uint64_t)i + 1; }
        return m;
      });
  ph("v build");
      radix_sort_pairs(key, val, bits_for((uint64_t)D.nv), nt);
  ph("v radix");
      r.resize(key.size());
      parallel_for(key.size(), nt, [&](size_t lo, size_t hi, int) {
        for (size_t p = lo; p < hi; p++) {
          if (p + 16 < hi) __builtin_prefetch(&ev[first + (val[p + 16] >> 1)]);  // random gathers: keep 16 in flight
          const size_t i = val[p] >> 1;
          const Event& e = ev[first + i];
          const uint8_t f = (val[p] & 1) ? 1 : (uint8_t)(e.kind == RGPU_VDEL ? 0 : 1);
          r[p] = {(int32_t)key[p], f, e.t, (int64_t)i + 1};
        }
      });
    } else {
      r.reserve(2 * n);
      for (size_t i = 0; i < n; i++) {
        const Event& e = ev[first + i];
        if (e.kind != RGPU_EDEL) r.push_back({rs[i], (uint8_t)(e.kind == RGPU_VDEL ? 0 : 1), e.t, (int64_t)i + 1});
        if (e.kind == RGPU_EADD && rd[i] != rs[i]) r.push_back({rd[i], 1, e.t, (int64_t)i + 1});
      }
      parallel_sort(r, nt, [](const R& a, const R& b) {
        if (a.v != b.v) return a.v < b.v;
        return a.t != b.t ? a.t < b.t : a.idx < b.idx;
      });
    }
    ph("v fill");
    // collapse equal (rank, t) to the last put; one group per rank run (the last record of a
    // run is always kept).  Parallel: per-chunk counts of kept records and run starts, then fill.
    const size_t nr = r.size();
    auto kept = [&](size_t k) { return !(k + 1 < nr && r[k + 1].v == r[k].v && r[k + 1].t == r[k].t); };
    auto start = [&](size_t k) { return k == 0 || r[k - 1].v != r[k].v; };
    const int T = nr < 4096 ? 1 : nt;
    std::vector<size_t> ck(T + 1, 0), cg(T + 1, 0);
    parallel_for(nr, nt, [&](size_t lo, size_t hi, int q) {  // (local sums: no false sharing)
      size_t a = 0, g = 0;
      for (size_t k = lo; k < hi; k++) {
        a += kept(k);
        g += start(k);
      }
      ck[q + 1] = a;
      cg[q + 1] = g;
    });
    for (int q = 0; q < T; q++) {
      ck[q + 1] += ck[q];
      cg[q + 1] += cg[q];
    }
    D.dv_key.resize(ck[T]);
    D.dv_rank.resize(cg[T]);
    D.dv_off.resize(cg[T] + 1);
    parallel_for(nr, nt, [&](size_t lo, size_t hi, int q) {
      size_t a = ck[q], g = cg[q];
      for (size_t k = lo; k < hi; k++) {
        if (start(k)) {
          D.dv_rank[g] = r[k].v;
          D.dv_off[g++] = (int64_t)a;
        }
        if (kept(k)) D.dv_key[a++] = r[k].t * 2 + r[k].f;
      }
    });
    D.dv_off[cg[T]] = (int64_t)ck[T];
    if (nr == 0) D.dv_off.assign(1, 0);
  }
  ph("vpoints");
  // ---- delta deaths: distinct times per rank with the last delta index at each time
  {
    struct R { int32_t v; int64_t t, idx; };
    std::vector<R> r;
    for (size_t i = 0; i < n; i++)
      if (ev[first + i].kind == RGPU_VDEL) r.push_back({rs[i], ev[first + i].t, (int64_t)i + 1});
    std::sort(r.begin(), r.end(), [](const R& a, const R& b) {
      if (a.v != b.v) return a.v < b.v;
      return a.t != b.t ? a.t < b.t : a.idx < b.idx;
    });
    D.dd_off.push_back(0);
    for (size_t k = 0; k < r.size(); k++) {
      if (k + 1 < r.size() && r[k + 1].v == r[k].v && r[k + 1].t == r[k].t) continue;
      if (D.dd_rank.empty() || D.dd_rank.back() != r[k].v) {
        if (!D.dd_rank.empty()) D.dd_off.push_back((int64_t)D.dd_t.size());
        D.dd_rank.push_back(r[k].v);
      }
      D.dd_t.push_back(r[k].t);
      D.dd_last.push_back(r[k].idx);
    }
    if (!D.dd_rank.empty()) D.dd_off.push_back((int64_t)D.dd_t.size());
  }
  ph("deaths");
  // ---- delta edge points grouped by (s, d), each edge's points by (t, idx)
  {
    struct R { int32_t s, d; uint8_t f; int64_t t, idx; };
    std::vector<R> r;
    if (mono) {  // radix by (s, d) = s * nv + d over the edge updates in stream order
      std::vector<uint64_t> key, val;
      build_pairs(n, nt, 1, key, val, [&](size_t i, uint64_t* k, uint64_t* v) {
        if (ev[first + i].kind < RGPU_EADD) return 0;
        k[0] = (uint64_t)rs[i] * (uint64_t)D.nv + (uint64_t)rd[i];
        v[0] = i;
        return 1;
      });
  ph("e build");
      radix_sort_pairs(key, val, bits_for((uint64_t)D.nv * (uint64_t)D.nv), nt);
  ph("e radix");
      r.resize(key.size());
      parallel_for(key.size(), nt, [&](size_t lo, size_t hi, int) {
        for (size_t p = lo; p < hi; p++) {
          if (p + 16 < hi) __builtin_prefetch(&ev[first + val[p + 16]]);
          const size_t i = val[p];
          const Event& e = ev[first + i];
          r[p] = {rs[i], rd[i], (uint8_t)(e.kind == RGPU_EADD ? 1 : 0), e.t, (int64_t)i + 1};
        }
      });
    } else {
      for (size_t i = 0; i < n; i++) {
        const Event& e = ev[first + i];
        if (e.kind >= RGPU_EADD) r.push_back({rs[i], rd[i], (uint8_t)(e.kind == RGPU_EADD ? 1 : 0), e.t, (int64_t)i + 1});
      }
      parallel_sort(r, nt, [](const R& a, const R& b) {
        if (a.s != b.s) return a.s < b.s;
        if (a.d != b.d) return a.d < b.d;
        return a.t != b.t ? a.t < b.t : a.idx < b.idx;
      });
    }
    ph("e fill");
    // one group per distinct (s, d); every point is kept.  Parallel counts of group starts, fill.
    const size_t nr = r.size();
    auto start = [&](size_t k) { return k == 0 || r[k].s != r[k - 1].s || r[k].d != r[k - 1].d; };
    const int T = nr < 4096 ? 1 : nt;
    std::vector<size_t> cg(T + 1, 0);
    parallel_for(nr, nt, [&](size_t lo, size_t hi, int q) {
      size_t g = 0;
      for (size_t k = lo; k < hi; k++) g += start(k);
      cg[q + 1] = g;
    });
    for (int q = 0; q < T; q++) cg[q + 1] += cg[q];
    const size_t ng = cg[T];
    D.de_s.resize(ng);
    D.de_d.resize(ng);
    D.de_qs.resize(ng);
    D.de_qd.resize(ng);
    D.de_poff.resize(ng + 1);
    D.de_pt.resize(nr);
    D.de_pidx.resize(nr);
    D.de_pflag.resize(nr);
    parallel_for(nr, nt, [&](size_t lo, size_t hi, int q) {
      size_t g = cg[q];
      for (size_t k = lo; k < hi; k++) {
        if (start(k)) {
          D.de_s[g] = r[k].s;
          D.de_d[g] = r[k].d;
          D.de_qs[g] = D.new2old[r[k].s];
          D.de_qd[g] = D.new2old[r[k].d];
          D.de_poff[g++] = (int64_t)k;
        }
        D.de_pt[k] = r[k].t;
        D.de_pidx[k] = r[k].idx;
        D.de_pflag[k] = r[k].f;
      }
    });
    D.de_poff[ng] = (int64_t)nr;
    if (nr == 0) D.de_poff.assign(1, 0);
  }
  ph("epoints");
  return "";
}

void finish_delta(const Packed& B, const std::vector<int32_t>& base_eid, Delta* out) {
  Delta& D = *out;
  PhaseTimer ph{"finish_delta"};
  const int64_t nde = (int64_t)D.de_s.size();
  D.de_base = base_eid;
  // death at exactly t: the last delta index, 0 for a base death, -1 for none
  auto death_at = [&](int32_t v, int64_t t) -> int64_t {
    auto it = std::lower_bound(D.dd_rank.begin(), D.dd_rank.end(), v);
    if (it != D.dd_rank.end() && *it == v) {
      const size_t j = it - D.dd_rank.begin();
      auto b = D.dd_t.begin() + D.dd_off[j], e = D.dd_t.begin() + D.dd_off[j + 1];
      auto f = std::lower_bound(b, e, t);
      if (f != e && *f == t) return D.dd_last[f - D.dd_t.begin()];
    }
    const int32_t u = D.new2old[v];
    if (u >= 0) {
      auto b = B.dtime.begin() + B.doff[u], e = B.dtime.begin() + B.doff[u + 1];
      if (std::binary_search(b, e, t)) return 0;
    }
    return -1;
  };
  // own points: collapse equal t (last put wins), then the tie with an endpoint death at the
  // same t exactly as pack_events resolves it (x2 positions; a base edge was created at 0)
  // per edge: emit(i, out) writes its keys (out = nullptr: count only); counts, scan, fill
  auto emit = [&](int64_t i, int64_t* out) -> int64_t {
    const int64_t p0 = D.de_poff[i], p1 = D.de_poff[i + 1];
    int64_t cr = 0;  // creation put: the edge's first delta update (points are in time order)
    if (base_eid[i] < 0) {
      cr = D.de_pidx[p0];
      for (int64_t k = p0; k < p1; k++) cr = std::min(cr, D.de_pidx[k]);
    }
    int64_t m = 0;
    for (int64_t k = p0; k < p1; k++) {
      if (k + 1 < p1 && D.de_pt[k + 1] == D.de_pt[k]) continue;
      if (out) {
        uint8_t flag = D.de_pflag[k];
        int64_t pd = death_at(D.de_s[i], D.de_pt[k]);
        if (D.de_d[i] != D.de_s[i]) pd = std::max(pd, death_at(D.de_d[i], D.de_pt[k]));
        if (pd >= 0) {
          const int64_t pd2 = pd < cr ? 2 * cr + 1 : 2 * pd;
          if (pd2 > 2 * D.de_pidx[k]) flag = 0;
        }
        out[m] = D.de_pt[k] * 2 + flag;
      }
      m++;
    }
    return m;
  };
  const int nt0 = num_threads();
  D.de_koff.assign(nde + 1, 0);
  parallel_for((size_t)nde, nt0, [&](size_t lo, size_t hi, int) {
    for (size_t i = lo; i < hi; i++) D.de_koff[i + 1] = emit((int64_t)i, nullptr);
  });
  for (int64_t i = 0; i < nde; i++) D.de_koff[i + 1] += D.de_koff[i];
  D.de_key.resize(D.de_koff[nde]);
  parallel_for((size_t)nde, nt0, [&](size_t lo, size_t hi, int) {
    for (size_t i = lo; i < hi; i++) emit((int64_t)i, D.de_key.data() + D.de_koff[i]);
  });
  ph("own keys");
  // new edges, and their in-edge records (self-loops never enter incomingEdges)
  {  // in delta-edge order, i.e. (s, d) ascending: per-chunk counts, then a parallel fill
    const int T = nde < 4096 ? 1 : nt0;
    std::vector<size_t> cn(T + 1, 0), ci(T + 1, 0);
    parallel_for((size_t)nde, nt0, [&](size_t lo, size_t hi, int q) {  // (local sums)
      size_t a = 0, b = 0;
      for (size_t i = lo; i < hi; i++)
        if (base_eid[i] < 0) {
          a++;
          b += D.de_s[i] != D.de_d[i];
        }
      cn[q + 1] = a;
      ci[q + 1] = b;
    });
    for (int q = 0; q < T; q++) {
      cn[q + 1] += cn[q];
      ci[q + 1] += ci[q];
    }
    D.nn_key.resize(cn[T]);
    D.nn_didx.resize(cn[T]);
    D.ni_key.resize(ci[T]);
    D.ni_idx.resize(ci[T]);
    parallel_for((size_t)nde, nt0, [&](size_t lo, size_t hi, int q) {
      size_t a = cn[q], b = ci[q];
      for (size_t i = lo; i < hi; i++) {
        if (base_eid[i] >= 0) continue;
        const int32_t s = D.de_s[i], d = D.de_d[i];
        D.nn_key[a] = ((int64_t)s << 32) | d;
        D.nn_didx[a] = (int32_t)i;
        if (s != d) {
          D.ni_key[b] = ((int64_t)d << 32) | s;
          D.ni_idx[b++] = (int32_t)a;
        }
        a++;
      }
    });
  }
  const int nt = num_threads();
  {  // by (d, s) = d * nv + s (keys are distinct, so stability does not matter here)
    const uint64_t nv = (uint64_t)D.nv;
    std::vector<uint64_t> key(D.ni_key.size()), val(D.ni_key.size());
    parallel_for(key.size(), nt, [&](size_t lo, size_t hi, int) {
      for (size_t k = lo; k < hi; k++) {
        key[k] = (uint64_t)(D.ni_key[k] >> 32) * nv + (uint64_t)(D.ni_key[k] & 0xffffffff);
        val[k] = (uint64_t)D.ni_idx[k];
      }
    });
    radix_sort_pairs(key, val, bits_for(nv * nv), nt);
    parallel_for(key.size(), nt, [&](size_t lo, size_t hi, int) {
      for (size_t k = lo; k < hi; k++) {
        D.ni_key[k] = ((int64_t)(key[k] / nv) << 32) | (int64_t)(key[k] % nv);
        D.ni_idx[k] = (int32_t)val[k];
      }
    });
  }
  ph("new edges");
  // merged offsets and death lists (O(V) host work)
  D.out_off.assign(D.nv + 1, 0);
  D.in_off.assign(D.nv + 1, 0);
  parallel_for((size_t)D.nv, nt, [&](size_t lo, size_t hi, int) {  // counts, then one prefix pass
    if (lo >= hi) return;
    // new out-edges of v: its run in nn_key ((s, d) ascending); new in-edges: its run in ni_key
    size_t po = std::lower_bound(D.nn_key.begin(), D.nn_key.end(), (int64_t)lo << 32) - D.nn_key.begin();
    size_t pi = std::lower_bound(D.ni_key.begin(), D.ni_key.end(), (int64_t)lo << 32) - D.ni_key.begin();
    for (size_t v = lo; v < hi; v++) {
      const int32_t u = D.new2old[v];
      int64_t oc = 0, ic = 0;
      for (; po < D.nn_key.size() && (size_t)(D.nn_key[po] >> 32) == v; po++) oc++;
      for (; pi < D.ni_key.size() && (size_t)(D.ni_key[pi] >> 32) == v; pi++) ic++;
      if (u >= 0) {
        oc += B.out_off[u + 1] - B.out_off[u];
        ic += B.in_off[u + 1] - B.in_off[u];
      }
      D.out_off[v + 1] = oc;
      D.in_off[v + 1] = ic;
    }
  });
  {  // two-level parallel prefix: chunk totals, then each chunk adds its offset
    const int T = D.nv < 4096 ? 1 : nt;
    std::vector<int64_t> to(T + 1, 0), ti(T + 1, 0);
    parallel_for((size_t)D.nv, nt, [&](size_t lo, size_t hi, int q) {
      int64_t a = 0, b = 0;
      for (size_t v = lo; v < hi; v++) {
        a += D.out_off[v + 1];
        b += D.in_off[v + 1];
        D.out_off[v + 1] = a;
        D.in_off[v + 1] = b;
      }
      to[q + 1] = a;
      ti[q + 1] = b;
    });
    for (int q = 0; q < T; q++) {
      to[q + 1] += to[q];
      ti[q + 1] += ti[q];
    }
    parallel_for((size_t)D.nv, nt, [&](size_t lo, size_t hi, int q) {
      for (size_t v = lo; v < hi; v++) {
        D.out_off[v + 1] += to[q];
        D.in_off[v + 1] += ti[q];
      }
    });
  }
  ph("offsets");
  D.doff.assign(D.nv + 1, 0);
  D.dtime.clear();
  D.dtime.reserve(B.dtime.size() + D.dd_t.size());
  size_t jd = 0;
  for (int64_t v = 0; v < D.nv && !(B.dtime.empty() && D.dd_t.empty()); v++) {
    const int32_t u = D.new2old[v];
    const int64_t* b0 = u >= 0 ? B.dtime.data() + B.doff[u] : nullptr;
    const int64_t* b1 = u >= 0 ? B.dtime.data() + B.doff[u + 1] : nullptr;
    const int64_t *c0 = nullptr, *c1 = nullptr;
    if (jd < D.dd_rank.size() && D.dd_rank[jd] == v) {
      c0 = D.dd_t.data() + D.dd_off[jd];
      c1 = D.dd_t.data() + D.dd_off[jd + 1];
      jd++;
    }
    while (b0 != b1 || c0 != c1) {  // sorted union of distinct times
      int64_t t;
      if (c0 == c1 || (b0 != b1 && *b0 < *c0)) t = *b0++;
      else if (b0 == b1 || *c0 < *b0) t = *c0++;
      else { t = *b0++; c0++; }
      D.dtime.push_back(t);
    }
    D.doff[v + 1] = (int64_t)D.dtime.size();
  }
  ph("deaths");
}

}  // namespace rgpu
