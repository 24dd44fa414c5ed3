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
#include <algorithm>
#include <cstring>

#include "rgpu_internal.hpp"

namespace rgpu {
namespace {

struct VPoint {
  int32_t r;
  uint8_t flag;
  int64_t t, idx;
};
struct EPoint {
  int32_t s, d;
  uint8_t flag;
  int64_t t, idx;
};
struct Death {
  int32_t r;
  int64_t t, idx;
};

}  // namespace

std::string pack_events(const std::vector<Event>& ev, int partition, int num_partitions,
                        Packed* out) {
  if (num_partitions != 1 || partition != 0)
    return "vertex-partitioned contexts (num_partitions > 1) are not in this build; "
           "run one replica context per GPU";
  const int64_t kMaxT = (int64_t)1 << 61;
  std::vector<int64_t> ids;
  ids.reserve(ev.size() * 2);
  int64_t newest = -1;
  for (const Event& e : ev) {
    if (e.kind > RGPU_EDEL) return "unknown update kind";
    if (e.t < 0 || e.t >= kMaxT) return "time out of range [0, 2^61)";
    if (e.src < 0 || e.src > INT32_MAX) return "vertex id out of range [0, 2^31)";
    ids.push_back(e.src);
    if (e.kind >= RGPU_EADD) {
      if (e.dst < 0 || e.dst > INT32_MAX) return "vertex id out of range [0, 2^31)";
      ids.push_back(e.dst);
    }
    newest = std::max(newest, e.t);
  }
  std::sort(ids.begin(), ids.end());
  ids.erase(std::unique(ids.begin(), ids.end()), ids.end());
  Packed& P = *out;
  P = Packed();
  P.newest = newest;
  P.nv = (int64_t)ids.size();
  P.vid = ids;
  auto rank = [&](int64_t id) {
    return (int32_t)(std::lower_bound(ids.begin(), ids.end(), id) - ids.begin());
  };

  std::vector<VPoint> vp;
  std::vector<EPoint> ep;
  std::vector<Death> dd;
  vp.reserve(ev.size() * 2);
  ep.reserve(ev.size());
  for (size_t i = 0; i < ev.size(); i++) {
    const Event& e = ev[i];
    int64_t idx = (int64_t)i;
    int32_t rs = rank(e.src);
    switch (e.kind) {
      case RGPU_VADD: vp.push_back({rs, 1, e.t, idx}); break;
      case RGPU_VDEL:
        vp.push_back({rs, 0, e.t, idx});
        dd.push_back({rs, e.t, idx});
        break;
      case RGPU_EADD: {
        int32_t rd = rank(e.dst);
        vp.push_back({rs, 1, e.t, idx});
        if (rd != rs) vp.push_back({rd, 1, e.t, idx});
        ep.push_back({rs, rd, 1, e.t, idx});
        break;
      }
      case RGPU_EDEL: ep.push_back({rs, rank(e.dst), 0, e.t, idx}); break;
    }
  }

  // ---- vertex histories: sort (rank, t, idx), collapse equal t (last put wins)
  std::sort(vp.begin(), vp.end(), [](const VPoint& a, const VPoint& b) {
    if (a.r != b.r) return a.r < b.r;
    if (a.t != b.t) return a.t < b.t;
    return a.idx < b.idx;
  });
  P.voff.assign(P.nv + 1, 0);
  P.vkey.reserve(vp.size());
  for (size_t i = 0; i < vp.size(); i++) {
    if (i + 1 < vp.size() && vp[i + 1].r == vp[i].r && vp[i + 1].t == vp[i].t) continue;
    P.vkey.push_back(vp[i].t * 2 + vp[i].flag);
    P.voff[vp[i].r + 1]++;
  }
  for (int64_t v = 0; v < P.nv; v++) P.voff[v + 1] += P.voff[v];

  // ---- death lists: distinct times, with the last stream index at each time
  std::sort(dd.begin(), dd.end(), [](const Death& a, const Death& b) {
    if (a.r != b.r) return a.r < b.r;
    if (a.t != b.t) return a.t < b.t;
    return a.idx < b.idx;
  });
  P.doff.assign(P.nv + 1, 0);
  std::vector<int64_t> dlast;  // max stream index of a death at dtime[i]
  for (size_t i = 0; i < dd.size(); i++) {
    if (i + 1 < dd.size() && dd[i + 1].r == dd[i].r && dd[i + 1].t == dd[i].t) continue;
    P.dtime.push_back(dd[i].t);
    dlast.push_back(dd[i].idx);
    P.doff[dd[i].r + 1]++;
  }
  for (int64_t v = 0; v < P.nv; v++) P.doff[v + 1] += P.doff[v];
  auto death_at = [&](int32_t r, int64_t t) -> int64_t {  // -1 if no death at exactly t
    auto b = P.dtime.begin() + P.doff[r], e = P.dtime.begin() + P.doff[r + 1];
    auto it = std::lower_bound(b, e, t);
    return (it != e && *it == t) ? dlast[it - P.dtime.begin()] : -1;
  };

  // ---- edge own histories
  std::sort(ep.begin(), ep.end(), [](const EPoint& a, const EPoint& b) {
    if (a.s != b.s) return a.s < b.s;
    if (a.d != b.d) return a.d < b.d;
    if (a.t != b.t) return a.t < b.t;
    return a.idx < b.idx;
  });
  P.eoff.push_back(0);
  for (size_t g = 0; g < ep.size();) {
    size_t h = g;
    int64_t created = ep[g].idx;  // stream index of the edge's first update
    while (h < ep.size() && ep[h].s == ep[g].s && ep[h].d == ep[g].d) {
      created = std::min(created, ep[h].idx);
      h++;
    }
    for (size_t i = g; i < h; i++) {
      if (i + 1 < h && ep[i + 1].t == ep[i].t) continue;  // collapse: last put wins
      uint8_t flag = ep[i].flag;
      // tie with an endpoint death at the same time: compare put positions (x2 so that
      // "right after creation" = 2*created+1 sits between two stream indices)
      int64_t pd = death_at(ep[i].s, ep[i].t);
      if (ep[i].d != ep[i].s) pd = std::max(pd, death_at(ep[i].d, ep[i].t));
      if (pd >= 0) {
        int64_t pd2 = pd < created ? 2 * created + 1 : 2 * pd;
        if (pd2 > 2 * ep[i].idx) flag = 0;
      }
      P.ekey.push_back(ep[i].t * 2 + flag);
    }
    P.esrc.push_back(ep[g].s);
    P.edst.push_back(ep[g].d);
    P.eoff.push_back((int64_t)P.ekey.size());
    g = h;
  }
  P.ne = (int64_t)P.esrc.size();

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
  return "";
}

}  // namespace rgpu
