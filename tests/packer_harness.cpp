// TEST INFRASTRUCTURE: CPU harness around the product's host packer (raphtory_amd/csrc/
// packer.cpp, compiled here with g++).  ph_alive restates the window-mask kernels' liveness
// rule (kernels.hip: k_vertex_mask / k_edge_mask) on the packed arrays so that the packer
// can be checked against the oracle's literal EntityStorage replay without a GPU.
#include <algorithm>
#include <cstdint>
#include <vector>

#include "rgpu_internal.hpp"

using rgpu::Event;
using rgpu::Packed;

// local vertex order of the next packs (pack_events `locality`: 1 = RGPU_ORDER_LOCALITY)
static bool g_locality = false;
extern "C" void ph_set_locality(int on) { g_locality = on != 0; }

extern "C" void* ph_pack(const int64_t* t, const uint8_t* kind, const int64_t* src, const int64_t* dst,
                         size_t n) {
  std::vector<Event> ev(n);
  for (size_t i = 0; i < n; i++) ev[i] = {t[i], src[i], kind[i] >= 2 ? dst[i] : -1, kind[i]};
  Packed* p = new Packed();
  if (!rgpu::pack_events(ev, 0, 1, p, g_locality).empty()) { delete p; return nullptr; }
  return p;
}
// partition view (num_partitions > 1): same stream, one partition's pack
extern "C" void* ph_pack_part(const int64_t* t, const uint8_t* kind, const int64_t* src, const int64_t* dst,
                              size_t n, int part, int nparts) {
  std::vector<Event> ev;  // what rgpu_ingest keeps for this partition
  for (size_t i = 0; i < n; i++)
    if (rgpu::partition_keeps(kind[i], src[i], kind[i] >= 2 ? dst[i] : -1, part, nparts))
      ev.push_back({t[i], src[i], kind[i] >= 2 ? dst[i] : -1, kind[i]});
  Packed* p = new Packed();
  if (!rgpu::pack_events(ev, part, nparts, p, g_locality).empty()) { delete p; return nullptr; }
  return p;
}
// what: 0 local vertex ids [nv], 1 CC label per local rank [nv] (P > 1), 2 send list ids of
// peer q, 3 receive list ids of peer q, 4 edge src ids, 5 edge dst ids, 6 owner partition per
// local rank (P > 1); returns the count
extern "C" int64_t ph_list(void* h, int what, int q, int64_t* out) {
  const Packed* p = (const Packed*)h;
  std::vector<int64_t> v;
  if (what == 0) v.assign(p->vid.begin(), p->vid.end());
  if (what == 1) v.assign(p->grank.begin(), p->grank.end());
  if (what == 2) for (int64_t i = p->xs_off[q]; i < p->xs_off[q + 1]; i++) v.push_back(p->vid[p->xs_v[i]]);
  if (what == 3) for (int64_t i = p->xr_off[q]; i < p->xr_off[q + 1]; i++) v.push_back(p->vid[p->xr_v[i]]);
  if (what == 4) for (int64_t e = 0; e < p->ne; e++) v.push_back(p->vid[p->esrc[e]]);
  if (what == 5) for (int64_t e = 0; e < p->ne; e++) v.push_back(p->vid[p->edst[e]]);
  if (what == 6) v.assign(p->lowner.begin(), p->lowner.end());
  if (what == 7)  // owned ids in the order of by_id (ascending ids when it is right)
    for (int64_t k = 0; k < p->n_own; k++) v.push_back(p->vid[p->by_id.empty() ? k : p->by_id[k]]);
  if (what == 8)  // the id of every local rank's label (P = 1 relabeled: lid[grank]; P > 1: grank)
    for (int64_t r = 0; r < p->nv; r++)
      v.push_back(p->grank.empty() ? p->vid[r] : p->nparts > 1 ? p->grank[r] : p->lid[p->grank[r]]);
  if (what == 9)  // per edge: its history keys, with the edge's (src id, dst id) first
    for (int64_t e = 0; e < p->ne; e++) {
      v.push_back(p->vid[p->esrc[e]]);
      v.push_back(p->vid[p->edst[e]]);
      v.push_back(p->eoff[e + 1] - p->eoff[e]);
      for (int64_t k = p->eoff[e]; k < p->eoff[e + 1]; k++) v.push_back(p->ekey[k]);
    }
  if (what == 10)  // per local rank: id, vertex history size + keys, death count + times
    for (int64_t r = 0; r < p->nv; r++) {
      v.push_back(p->vid[r]);
      v.push_back(p->voff[r + 1] - p->voff[r]);
      for (int64_t k = p->voff[r]; k < p->voff[r + 1]; k++) v.push_back(p->vkey[k]);
      v.push_back(p->doff[r + 1] - p->doff[r]);
      for (int64_t k = p->doff[r]; k < p->doff[r + 1]; k++) v.push_back(p->dtime[k]);
    }
  if (what == 11) {  // structural checks of any order: 0 = fine, else the first failed check
    int bad = 0;
    for (int64_t e = 0; e + 1 < p->ne && !bad; e++)
      if (p->esrc[e] > p->esrc[e + 1] || (p->esrc[e] == p->esrc[e + 1] && p->edst[e] >= p->edst[e + 1])) bad = 1;
    for (int64_t v2 = 0; v2 < p->nv && !bad; v2++)
      for (int64_t k = p->in_off[v2]; k < p->in_off[v2 + 1]; k++) {
        const int32_t e = p->in_eid[k];
        if (p->edst[e] != v2 || (k > p->in_off[v2] && p->esrc[p->in_eid[k - 1]] >= p->esrc[e])) bad = 2;
      }
    for (int64_t k = 0; k + 1 < (int64_t)p->by_id.size() && !bad; k++)
      if (p->vid[p->by_id[k]] >= p->vid[p->by_id[k + 1]]) bad = 3;
    if (p->relabeled && p->nparts == 1 && !bad)
      for (int64_t r = 0; r < p->nv; r++)
        if (p->lid[p->grank[r]] != p->vid[r] || p->by_id[p->grank[r]] != r) { bad = 4; break; }
    v.push_back(bad);
  }
  if (out) std::copy(v.begin(), v.end(), out);
  return (int64_t)v.size();
}
extern "C" void ph_free(void* h) { delete (Packed*)h; }
extern "C" int64_t ph_num(void* h, int what) {
  const Packed* p = (const Packed*)h;
  return what == 0 ? p->nv : what == 1 ? p->ne : what == 2 ? (int64_t)p->vkey.size()
       : what == 3 ? (int64_t)p->ekey.size() : p->n_own;
}

static int64_t floor_key(const std::vector<int64_t>& key, int64_t lo, int64_t hi, int64_t t) {
  auto it = std::upper_bound(key.begin() + lo, key.begin() + hi, 2 * t + 1);
  return it == key.begin() + lo ? -1 : *(it - 1);
}
static int64_t last_death(const Packed* p, int32_t r, int64_t t) {
  auto b = p->dtime.begin() + p->doff[r], e = p->dtime.begin() + p->doff[r + 1];
  auto it = std::upper_bound(b, e, t);
  return it == b ? -1 : *(it - 1);
}
// window < 0 => ViewLens (no window)
extern "C" int ph_alive(void* h, int is_edge, int64_t src, int64_t dst, int64_t t, int64_t window) {
  const Packed* p = (const Packed*)h;
  auto rank = [&](int64_t id) -> int64_t {  // local order is (owned, ghost) by id: search both runs
    if (p->relabeled) {  // locality order: a scan (test sizes)
      for (int64_t r = 0; r < p->nv; r++)
        if (p->vid[r] == id) return r;
      return -1;
    }
    for (auto [lo, hi] : {std::pair<int64_t, int64_t>{0, p->n_own}, {p->n_own, p->nv}}) {
      auto it = std::lower_bound(p->vid.begin() + lo, p->vid.begin() + hi, id);
      if (it != p->vid.begin() + hi && *it == id) return it - p->vid.begin();
    }
    return -1;
  };
  const int64_t rs = rank(src);
  if (rs < 0) return 0;
  const int64_t w = window < 0 ? INT64_MAX : window;
  if (!is_edge) {
    const int64_t k = floor_key(p->vkey, p->voff[rs], p->voff[rs + 1], t);
    return k >= 0 && (k & 1) && t - (k >> 1) <= w;
  }
  const int64_t rd = rank(dst);
  if (rd < 0) return 0;
  int64_t e = -1;
  for (int64_t x = p->out_off[rs]; x < p->out_off[rs + 1]; x++)
    if (p->edst[x] == rd) e = x;
  if (e < 0) return 0;
  const int64_t k = floor_key(p->ekey, p->eoff[e], p->eoff[e + 1], t);
  if (k < 0 || !(k & 1)) return 0;
  const int64_t ft = k >> 1;
  if (last_death(p, (int32_t)rs, t) > ft || last_death(p, (int32_t)rd, t) > ft) return 0;
  return t - ft <= w;
}

// Live-ingest host half (packer.cpp pack_delta / finish_delta) against a one-shot pack of the
// same stream: base = updates [0, cut), delta = [cut, n).  The base-edge lookup that the device
// does (k_edge_find) is done here by binary search.  Checks the merged ids, rank maps, adjacency
// offsets, death lists, the merged edge set, and every vertex history merged as merge.hip's
// position formulas define it (base and delta by time, the delta point winning a tie).
// Returns 0, or the number of the first failed check.
extern "C" int ph_delta_check(const int64_t* t, const uint8_t* kind, const int64_t* src, const int64_t* dst,
                              size_t n, size_t cut) {
  std::vector<Event> ev(n);
  for (size_t i = 0; i < n; i++) ev[i] = {t[i], src[i], kind[i] >= 2 ? dst[i] : -1, kind[i]};
  std::vector<Event> head(ev.begin(), ev.begin() + cut);
  Packed B, F;
  if (!rgpu::pack_events(head, 0, 1, &B).empty() || !rgpu::pack_events(ev, 0, 1, &F).empty()) return 1;
  rgpu::Delta D;
  if (!rgpu::pack_delta(ev, cut, B, &D).empty()) return 2;
  std::vector<int32_t> base_eid(D.de_s.size(), -1);
  for (size_t i = 0; i < D.de_s.size(); i++) {
    const int32_t qs = D.de_qs[i], qd = D.de_qd[i];
    if (qs < 0 || qd < 0) continue;
    auto lo = B.edst.begin() + B.out_off[qs], hi = B.edst.begin() + B.out_off[qs + 1];
    auto it = std::lower_bound(lo, hi, qd);
    if (it != hi && *it == qd) base_eid[i] = (int32_t)(it - B.edst.begin());
  }
  rgpu::finish_delta(B, base_eid, &D);
  if (D.nv != F.nv || D.vid != F.vid) return 3;
  for (int64_t a = 0; a < B.nv; a++)
    if (D.vid[D.old2new[a]] != B.vid[a] || D.new2old[D.old2new[a]] != a) return 4;
  if (D.out_off != F.out_off || D.in_off != F.in_off) return 5;
  if (D.doff != F.doff || D.dtime != F.dtime) return 6;
  // merged edge set: base edges (remapped) + new edges == the one-shot pack's edges
  std::vector<int64_t> keys;
  for (int64_t e = 0; e < B.ne; e++)
    keys.push_back(((int64_t)D.old2new[B.esrc[e]] << 32) | D.old2new[B.edst[e]]);
  for (int64_t k : D.nn_key) keys.push_back(k);
  std::sort(keys.begin(), keys.end());
  if ((int64_t)keys.size() != F.ne) return 7;
  for (int64_t e = 0; e < F.ne; e++)
    if (keys[e] != (((int64_t)F.esrc[e] << 32) | F.edst[e])) return 8;
  // vertex histories
  for (int64_t v = 0; v < D.nv; v++) {
    std::vector<int64_t> a, b, m;
    const int32_t u = D.new2old[v];
    if (u >= 0) a.assign(B.vkey.begin() + B.voff[u], B.vkey.begin() + B.voff[u + 1]);
    auto it = std::lower_bound(D.dv_rank.begin(), D.dv_rank.end(), (int32_t)v);
    if (it != D.dv_rank.end() && *it == v) {
      const size_t g = it - D.dv_rank.begin();
      b.assign(D.dv_key.begin() + D.dv_off[g], D.dv_key.begin() + D.dv_off[g + 1]);
    }
    size_t i = 0, j = 0;
    while (i < a.size() || j < b.size()) {
      if (j == b.size() || (i < a.size() && (a[i] >> 1) < (b[j] >> 1))) m.push_back(a[i++]);
      else {
        if (i < a.size() && (a[i] >> 1) == (b[j] >> 1)) i++;
        m.push_back(b[j++]);
      }
    }
    if (!std::equal(m.begin(), m.end(), F.vkey.begin() + F.voff[v]) || (int64_t)m.size() != F.voff[v + 1] - F.voff[v])
      return 9;
  }
  return 0;
}
