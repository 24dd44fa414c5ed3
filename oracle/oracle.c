/*
 * oracle.c — TEST INFRASTRUCTURE ONLY (see oracle.h for the rules and parity status).
 *
 * A plain-C restatement of the reference's hot path, organised like the Scala it
 * follows so each step can be checked line by line:
 *
 *   S/ = /root/reference/mainproject/cluster/src/main/scala/com/raphtory/
 *
 *   history map ........ S/core/model/graphentities/Entity.scala:25-57 (TreeMap put-overwrite,
 *                        revive/kill, checkOldestNewest), Edge.scala:36-44 (killList)
 *   ingest ............. S/core/storage/EntityStorage.scala:73-97 (vertexAdd, placeholder),
 *                        :148-232 (vertexRemoval), :237-290 (edgeAdd), :327-383 (edgeRemoval)
 *   liveness ........... Entity.scala:173-201 (closestTime linear scan, aliveAt, aliveAtWithWindow)
 *   view filter ........ GraphLenses/WindowLens.scala:23-68, ViewLens.scala:20-54,
 *                        Vertex.scala:64-74 (viewAt / viewAtWithWindow)
 *   BSP driver ......... PartitionManager/Workers/ReaderWorker.scala:159-257 (setup/nextStep/
 *                        returnResults with shrinkWindow), Tasks/AnalysisTask.scala:162-283
 *   messaging .......... entityVisitors/VertexVisitor.scala:81-120, VertexMutliQueue.scala:11-38
 *   CC ................. Algorithms/ConnectedComponents.scala:10-42,160
 *   degree ............. Algorithms/DegreeBasic.scala:16-28
 *   PageRank ........... SURVEY.md App. A.5 (constants from examples/random/depricated/PageRank.scala:11-45)
 *
 * The whole stream is applied to ONE storage (a single Partition Manager whose 10
 * workers share Edge objects through local actor messages), in stream order, with
 * remote/other-worker messages delivered immediately (the quiescent state).
 */
#include "oracle.h"

#include <limits.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------ TreeMap */
/* mutable.TreeMap[Long,Boolean] with put-overwrite (Entity.scala:25).  Kept
 * ascending; HistoryOrdering's descending order never changes a lookup result. */
typedef struct {
  int64_t* k;
  uint8_t* v;
  int64_t* s; /* lazy-edge build only: stream index of the last put per key (NULL otherwise) */
  int n, cap;
} TMap;

static int tm_put_seq(TMap* m, int64_t k, uint8_t v, int64_t seq, int keep_seq) {
  int lo = 0, hi = m->n;
  if (m->n > 0 && m->k[m->n - 1] < k) {
    lo = hi = m->n; /* append fast path: streams are mostly time ordered */
  } else {
    while (lo < hi) {
      int mid = (lo + hi) >> 1;
      if (m->k[mid] < k) lo = mid + 1; else hi = mid;
    }
    if (lo < m->n && m->k[lo] == k) { /* last put wins */
      m->v[lo] = v;
      if (m->s) m->s[lo] = seq;
      return 0;
    }
  }
  if (m->n == m->cap) {
    int nc = m->cap ? m->cap * 2 : 4;
    int64_t* nk = (int64_t*)realloc(m->k, sizeof(int64_t) * nc);
    if (!nk) return -1;
    m->k = nk;
    uint8_t* nv = (uint8_t*)realloc(m->v, nc);
    if (!nv) return -1;
    m->v = nv;
    if (keep_seq || m->s) {
      int64_t* ns = (int64_t*)realloc(m->s, sizeof(int64_t) * nc);
      if (!ns) return -1;
      m->s = ns;
    }
    m->cap = nc;
  }
  memmove(m->k + lo + 1, m->k + lo, sizeof(int64_t) * (m->n - lo));
  memmove(m->v + lo + 1, m->v + lo, (size_t)(m->n - lo));
  if (m->s) memmove(m->s + lo + 1, m->s + lo, sizeof(int64_t) * (m->n - lo));
  m->k[lo] = k; m->v[lo] = v;
  if (m->s) m->s[lo] = seq;
  m->n++;
  return 0;
}
static int tm_put(TMap* m, int64_t k, uint8_t v) { return tm_put_seq(m, k, v, 0, 0); }
static void tm_free(TMap* m) {
  free(m->k); free(m->v); free(m->s);
  m->k = NULL; m->v = NULL; m->s = NULL; m->n = m->cap = 0;
}

/* ----------------------------------------------------------------- entities */
typedef struct {
  TMap hist;   /* previousState */
  TMap rem;    /* removeList */
  int64_t oldest, newest;
} Entity;

typedef struct { int* a; int n, cap; } IVec;
static int iv_push(IVec* v, int x) {
  if (v->n == v->cap) {
    int nc = v->cap ? v->cap * 2 : 4;
    int* na = (int*)realloc(v->a, sizeof(int) * nc);
    if (!na) return -1;
    v->a = na; v->cap = nc;
  }
  v->a[v->n++] = x;
  return 0;
}

/* Lazy-edge build (orc_build_ex(..., ORC_LAZY_EDGES)): an edge keeps only its OWN puts, each
 * with the stream index of its last put; the endpoint-death puts that the literal replay copies
 * into it (killList at creation, Edge.scala:36-44, EntityStorage.scala:262,277-278) or writes
 * into it later (vertexRemoval's kill loops, :189-228) are read from the endpoints' removeLists
 * when the edge is evaluated.  c = stream index of the edge's creation; si/di = endpoint
 * vertex indices. */
typedef struct { Entity e; int64_t src, dst; int32_t si, di; int64_t c; } Edge;
/* dl_t/dl_s: the vertex's VertexDelete log in stream order (lazy build); dsuf[i] = min dl_t[i..] */
typedef struct { Entity e; int64_t id; IVec out, in; int64_t *dl_t, *dl_s, *dsuf; int dn, dcap; } Vertex;

/* Entity constructor (Entity.scala:18-36): previousState = {creationTime -> isInitialValue},
 * removeList = {creationTime -> false} iff !isInitialValue.  seq/keep: lazy-build bookkeeping. */
static void ent_init(Entity* e, int64_t t, int initial, int64_t seq, int keep) {
  memset(e, 0, sizeof(*e));
  tm_put_seq(&e->hist, t, (uint8_t)(initial ? 1 : 0), seq, keep);
  if (!initial) tm_put_seq(&e->rem, t, 0, seq, keep);
  e->oldest = e->newest = t;
}
static void ent_check(Entity* e, int64_t t) { /* checkOldestNewest, Entity.scala:52-57 */
  if (t > e->newest) e->newest = t;
  if (e->oldest > t) e->oldest = t;
}
static void ent_revive(Entity* e, int64_t t, int64_t seq, int keep) { /* :41-44 */
  ent_check(e, t);
  tm_put_seq(&e->hist, t, 1, seq, keep);
}
static void ent_kill(Entity* e, int64_t t, int64_t seq, int keep) { /* :46-50 */
  ent_check(e, t);
  tm_put_seq(&e->rem, t, 0, seq, keep);
  tm_put_seq(&e->hist, t, 0, seq, keep);
}
static void edge_killlist(Entity* e, const TMap* vk) { /* Edge.killList, Edge.scala:36-44 (no checkOldestNewest) */
  for (int i = 0; i < vk->n; i++) { tm_put(&e->rem, vk->k[i], 0); tm_put(&e->hist, vk->k[i], 0); }
}

/* closestTime, Entity.scala:173-183: full linear scan, closest starts at -1. */
static void closest_time(const Entity* e, int64_t time, int64_t* ct, int* val) {
  int64_t c = -1; int v = 0;
  for (int i = 0; i < e->hist.n; i++) {
    int64_t k = e->hist.k[i];
    if (k <= time && (time - k) < (time - c)) { c = k; v = e->hist.v[i]; }
  }
  *ct = c; *val = v;
}
/* aliveAt (:185-191) for window < 0, aliveAtWithWindow (:193-201) otherwise. */
static int ent_alive(const Entity* e, int64_t time, int64_t window) {
  if (time < e->oldest) return 0;
  int64_t c; int v;
  closest_time(e, time, &c, &v);
  if (window < 0) return v;
  return (time - c <= window) ? v : 0;
}

/* ---------------------------------------------------------------- hash map */
typedef struct { uint64_t* keys; int32_t* vals; size_t cap, n; } HMap;
static uint64_t mix64(uint64_t x) {
  x ^= x >> 33; x *= 0xff51afd7ed558ccdULL; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ULL; x ^= x >> 33;
  return x;
}
static int hm_init(HMap* h, size_t cap) {
  h->cap = 16; while (h->cap < cap * 2) h->cap <<= 1;
  h->keys = (uint64_t*)malloc(sizeof(uint64_t) * h->cap);
  h->vals = (int32_t*)malloc(sizeof(int32_t) * h->cap);
  if (!h->keys || !h->vals) return -1;
  for (size_t i = 0; i < h->cap; i++) h->vals[i] = -1;
  h->n = 0;
  return 0;
}
static int32_t hm_get(const HMap* h, uint64_t k) {
  size_t i = mix64(k) & (h->cap - 1);
  while (h->vals[i] >= 0) { if (h->keys[i] == k) return h->vals[i]; i = (i + 1) & (h->cap - 1); }
  return -1;
}
static int hm_put(HMap* h, uint64_t k, int32_t v);
static int hm_grow(HMap* h) {
  HMap n2;
  if (hm_init(&n2, h->cap) != 0) return -1; /* doubles */
  for (size_t i = 0; i < h->cap; i++) if (h->vals[i] >= 0) hm_put(&n2, h->keys[i], h->vals[i]);
  free(h->keys); free(h->vals); *h = n2;
  return 0;
}
static int hm_put(HMap* h, uint64_t k, int32_t v) {
  if ((h->n + 1) * 2 > h->cap && hm_grow(h) != 0) return -1;
  size_t i = mix64(k) & (h->cap - 1);
  while (h->vals[i] >= 0) { if (h->keys[i] == k) { h->vals[i] = v; return 0; } i = (i + 1) & (h->cap - 1); }
  h->keys[i] = k; h->vals[i] = v; h->n++;
  return 0;
}

/* ----------------------------------------------------------------- storage */
struct orc_graph {
  Vertex* vs; size_t nv, capv;
  Edge* es; size_t ne, cape;
  HMap vmap, emap;
  int32_t* order; /* vertex indices sorted by id (ParTrieMap iteration order is irrelevant) */
  int lazy;       /* ORC_LAZY_EDGES: endpoint deaths read at evaluation, not copied (see Edge) */
  int64_t seq;    /* stream index of the update being applied */
};

static uint64_t ekey(int64_t s, int64_t d) { return ((uint64_t)s << 32) | (uint64_t)d; }

static int new_vertex(orc_graph* g, int64_t t, int64_t id, int initial) {
  if (g->nv == g->capv) {
    size_t nc = g->capv ? g->capv * 2 : 1024;
    Vertex* nvs = (Vertex*)realloc(g->vs, sizeof(Vertex) * nc);
    if (!nvs) return -1;
    g->vs = nvs; g->capv = nc;
  }
  Vertex* v = &g->vs[g->nv];
  memset(v, 0, sizeof(*v));
  ent_init(&v->e, t, initial, g->seq, g->lazy);
  v->id = id;
  if (hm_put(&g->vmap, (uint64_t)id, (int32_t)g->nv) != 0) return -1;
  return (int)g->nv++;
}
static int new_edge(orc_graph* g, int64_t t, int64_t s, int64_t d, int initial, int si) {
  if (g->ne == g->cape) {
    size_t nc = g->cape ? g->cape * 2 : 1024;
    Edge* nes = (Edge*)realloc(g->es, sizeof(Edge) * nc);
    if (!nes) return -1;
    g->es = nes; g->cape = nc;
  }
  Edge* e = &g->es[g->ne];
  memset(e, 0, sizeof(*e));
  ent_init(&e->e, t, initial, g->seq, g->lazy);
  e->src = s; e->dst = d;
  e->si = e->di = si;
  e->c = g->seq;
  if (hm_put(&g->emap, ekey(s, d), (int32_t)g->ne) != 0) return -1;
  return (int)g->ne++;
}

/* EntityStorage.vertexAdd, :73-87 */
static int vertex_add(orc_graph* g, int64_t t, int64_t id) {
  int32_t vi = hm_get(&g->vmap, (uint64_t)id);
  if (vi >= 0) { ent_revive(&g->vs[vi].e, t, g->seq, g->lazy); return vi; }
  return new_vertex(g, t, id, 1);
}
/* EntityStorage.getVertexOrPlaceholder, :89-97 (new vertex, then wipe()) */
static int vertex_or_placeholder(orc_graph* g, int64_t t, int64_t id) {
  int32_t vi = hm_get(&g->vmap, (uint64_t)id);
  if (vi >= 0) return vi;
  vi = new_vertex(g, t, id, 1);
  if (vi >= 0) g->vs[vi].e.hist.n = 0; /* Entity.wipe, Entity.scala:158 (oldestPoint untouched) */
  return vi;
}
/* EntityStorage.vertexRemoval, :148-232 */
static int vertex_removal(orc_graph* g, int64_t t, int64_t id) {
  int32_t vi = hm_get(&g->vmap, (uint64_t)id);
  if (vi >= 0) ent_kill(&g->vs[vi].e, t, g->seq, g->lazy);
  else if ((vi = new_vertex(g, t, id, 0)) < 0) return -1; /* placeholder created dead, :153-156 */
  Vertex* v = &g->vs[vi];
  if (g->lazy) { /* the kill loops below, deferred: log the death (time, stream index) */
    if (v->dn == v->dcap) {
      int nc = v->dcap ? v->dcap * 2 : 4;
      int64_t* nt = (int64_t*)realloc(v->dl_t, sizeof(int64_t) * nc);
      if (!nt) return -1;
      v->dl_t = nt;
      int64_t* ns = (int64_t*)realloc(v->dl_s, sizeof(int64_t) * nc);
      if (!ns) return -1;
      v->dl_s = ns;
      v->dcap = nc;
    }
    v->dl_t[v->dn] = t;
    v->dl_s[v->dn] = g->seq;
    v->dn++;
    return 0;
  }
  for (int i = 0; i < v->in.n; i++) ent_kill(&g->es[v->in.a[i]].e, t, g->seq, 0);   /* :189-213 */
  for (int i = 0; i < v->out.n; i++) ent_kill(&g->es[v->out.a[i]].e, t, g->seq, 0); /* :214-228 */
  return 0;
}
/* EntityStorage.edgeAdd, :237-290 (local && sameWorker order; other-worker and remote
 * paths deliver the same puts, :99-116, :292-314, :447-453). */
static int edge_add(orc_graph* g, int64_t t, int64_t s, int64_t d) {
  int si = vertex_add(g, t, s);
  if (si < 0) return -1;
  int32_t ei = hm_get(&g->emap, ekey(s, d));
  int present = ei >= 0;
  if (!present) {
    if ((ei = new_edge(g, t, s, d, 1, si)) < 0) return -1;
    if (iv_push(&g->vs[si].out, ei) != 0) return -1; /* srcVertex.addOutgoingEdge, :255 */
  }
  if (s != d) { /* :257-263 */
    int di = vertex_add(g, t, d);
    if (di < 0) return -1;
    if (!present) {
      g->es[ei].di = di;
      if (iv_push(&g->vs[di].in, ei) != 0) return -1;
      if (!g->lazy) edge_killlist(&g->es[ei].e, &g->vs[di].e.rem);
    }
  }
  if (present) ent_revive(&g->es[ei].e, t, g->seq, g->lazy);                /* :268-269 */
  else if (!g->lazy) edge_killlist(&g->es[ei].e, &g->vs[si].e.rem);         /* :276-278 */
  return 0;
}
/* EntityStorage.edgeRemoval, :327-383 */
static int edge_removal(orc_graph* g, int64_t t, int64_t s, int64_t d) {
  int si = vertex_or_placeholder(g, t, s);
  if (si < 0) return -1;
  int32_t ei = hm_get(&g->emap, ekey(s, d));
  int present = ei >= 0;
  if (!present) {
    if ((ei = new_edge(g, t, s, d, 0, si)) < 0) return -1;   /* initialValue = false, :341 */
    if (iv_push(&g->vs[si].out, ei) != 0) return -1;
  }
  if (s != d) {
    int di = vertex_or_placeholder(g, t, d);
    if (di < 0) return -1;
    if (!present) {
      g->es[ei].di = di;
      if (iv_push(&g->vs[di].in, ei) != 0) return -1;
      if (!g->lazy) edge_killlist(&g->es[ei].e, &g->vs[di].e.rem);
    }
  }
  if (present) ent_kill(&g->es[ei].e, t, g->seq, g->lazy);                  /* :365-366 */
  else if (!g->lazy) edge_killlist(&g->es[ei].e, &g->vs[si].e.rem);         /* :373-375 */
  return 0;
}

/* ---- lazy edges: the merged history, read on demand ----
 * A put's effective order: own puts at 2*seq; an endpoint death logged after the edge's
 * creation (vertexRemoval's kill loop) at 2*seq; one logged before it (copied by killList right
 * after the creation put, Edge.scala:36-44) at 2*c+1.  At equal keys the later put wins, as in
 * the TreeMap.  A death's key in removeList carries its LAST stream index (tm_put_seq). */
static int64_t death_order(const Edge* e, int64_t seq) { return seq > e->c ? 2 * seq : 2 * e->c + 1; }

/* largest removeList key <= t of vertex x (-1 if none), with its last stream index */
static int64_t death_floor(const Vertex* x, int64_t t, int64_t* seq) {
  const TMap* r = &x->e.rem;
  int lo = 0, hi = r->n;
  while (lo < hi) {
    int mid = (lo + hi) >> 1;
    if (r->k[mid] <= t) lo = mid + 1; else hi = mid;
  }
  if (lo == 0) return -1;
  *seq = r->s[lo - 1];
  return r->k[lo - 1];
}

/* closestTime (Entity.scala:173-183) over the merged history of a lazy edge: the own points by
 * the reference's linear scan, the endpoints' deaths by binary search, ties by put order. */
static void lazy_closest(const orc_graph* g, const Edge* e, int64_t time, int64_t* ct, int* val) {
  int64_t c = -1, ord = -1;
  int v = 0;
  const TMap* h = &e->e.hist;
  for (int i = 0; i < h->n; i++) {
    int64_t k = h->k[i];
    if (k <= time && (time - k) < (time - c)) { c = k; v = h->v[i]; ord = 2 * h->s[i]; }
  }
  for (int x = 0; x < 2; x++) {
    if (x == 1 && e->di == e->si) break; /* self-loop: one endpoint */
    int64_t sq = 0;
    int64_t kd = death_floor(&g->vs[x ? e->di : e->si], time, &sq);
    if (kd < 0) continue;
    int64_t od = death_order(e, sq);
    if (kd > c || (kd == c && od > ord)) { c = kd; v = 0; ord = od; }
  }
  *ct = c; *val = v;
}

/* after the replay: suffix minima of the death logs, and each lazy edge's oldestPoint, which
 * the deferred kills would have lowered (ent_kill -> checkOldestNewest; killList does not) */
static int lazy_finish(orc_graph* g) {
  for (size_t i = 0; i < g->nv; i++) {
    Vertex* x = &g->vs[i];
    if (!x->dn) continue;
    x->dsuf = (int64_t*)malloc(sizeof(int64_t) * x->dn);
    if (!x->dsuf) return -1;
    int64_t m = INT64_MAX;
    for (int k = x->dn - 1; k >= 0; k--) { m = x->dl_t[k] < m ? x->dl_t[k] : m; x->dsuf[k] = m; }
  }
  for (size_t i = 0; i < g->ne; i++) {
    Edge* e = &g->es[i];
    for (int x = 0; x < 2; x++) {
      if (x == 1 && e->di == e->si) break;
      const Vertex* v = &g->vs[x ? e->di : e->si];
      int lo = 0, hi = v->dn; /* first death logged after the creation */
      while (lo < hi) {
        int mid = (lo + hi) >> 1;
        if (v->dl_s[mid] <= e->c) lo = mid + 1; else hi = mid;
      }
      if (lo < v->dn && v->dsuf[lo] < e->e.oldest) e->e.oldest = v->dsuf[lo];
    }
  }
  return 0;
}

static int edge_alive(const orc_graph* g, const Edge* e, int64_t time, int64_t window) {
  if (!g->lazy) return ent_alive(&e->e, time, window);
  if (time < e->e.oldest) return 0;
  int64_t c; int v;
  lazy_closest(g, e, time, &c, &v);
  if (window < 0) return v;
  return (time - c <= window) ? v : 0;
}

static const orc_graph* g_sort_ctx;
static int cmp_vid(const void* a, const void* b) {
  int64_t x = g_sort_ctx->vs[*(const int32_t*)a].id, y = g_sort_ctx->vs[*(const int32_t*)b].id;
  return (x > y) - (x < y);
}

orc_graph* orc_build(const int64_t* t, const uint8_t* kind, const int64_t* src,
                     const int64_t* dst, size_t n) {
  return orc_build_ex(t, kind, src, dst, n, 0);
}

orc_graph* orc_build_ex(const int64_t* t, const uint8_t* kind, const int64_t* src,
                        const int64_t* dst, size_t n, int flags) {
  orc_graph* g = (orc_graph*)calloc(1, sizeof(orc_graph));
  if (!g) return NULL;
  g->lazy = (flags & ORC_LAZY_EDGES) != 0;
  if (hm_init(&g->vmap, 1024) || hm_init(&g->emap, 1024)) { orc_free(g); return NULL; }
  for (size_t i = 0; i < n; i++) {
    g->seq = (int64_t)i;
    /* keys >= 0, ids in [0, 2^31) (message targets are .toInt, VertexVisitor.scala:117) */
    if (t[i] < 0 || src[i] < 0 || src[i] > INT32_MAX) { orc_free(g); return NULL; }
    if ((kind[i] == ORC_EADD || kind[i] == ORC_EDEL) && (dst[i] < 0 || dst[i] > INT32_MAX)) { orc_free(g); return NULL; }
    int rc;
    switch (kind[i]) {
      case ORC_VADD: rc = vertex_add(g, t[i], src[i]) < 0 ? -1 : 0; break;
      case ORC_VDEL: rc = vertex_removal(g, t[i], src[i]); break;
      case ORC_EADD: rc = edge_add(g, t[i], src[i], dst[i]); break;
      case ORC_EDEL: rc = edge_removal(g, t[i], src[i], dst[i]); break;
      default: rc = -1;
    }
    if (rc != 0) { orc_free(g); return NULL; }
  }
  if (g->lazy && lazy_finish(g) != 0) { orc_free(g); return NULL; }
  g->order = (int32_t*)malloc(sizeof(int32_t) * (g->nv ? g->nv : 1));
  if (!g->order) { orc_free(g); return NULL; }
  for (size_t i = 0; i < g->nv; i++) g->order[i] = (int32_t)i;
  g_sort_ctx = g;
  qsort(g->order, g->nv, sizeof(int32_t), cmp_vid);
  return g;
}

void orc_free(orc_graph* g) {
  if (!g) return;
  for (size_t i = 0; i < g->nv; i++) {
    tm_free(&g->vs[i].e.hist); tm_free(&g->vs[i].e.rem);
    free(g->vs[i].out.a); free(g->vs[i].in.a);
    free(g->vs[i].dl_t); free(g->vs[i].dl_s); free(g->vs[i].dsuf);
  }
  for (size_t i = 0; i < g->ne; i++) { tm_free(&g->es[i].e.hist); tm_free(&g->es[i].e.rem); }
  free(g->vs); free(g->es); free(g->order);
  free(g->vmap.keys); free(g->vmap.vals); free(g->emap.keys); free(g->emap.vals);
  free(g);
}

size_t orc_num_vertices(const orc_graph* g) { return g->nv; }
size_t orc_num_edges(const orc_graph* g) { return g->ne; }

static const Vertex* find_vertex(const orc_graph* g, int64_t s) {
  if (s < 0 || s > INT32_MAX) return NULL;
  int32_t vi = hm_get(&g->vmap, (uint64_t)s);
  return vi >= 0 ? &g->vs[vi] : NULL;
}
static const Edge* find_edge(const orc_graph* g, int64_t s, int64_t d) {
  if (s < 0 || s > INT32_MAX || d < 0 || d > INT32_MAX) return NULL;
  int32_t ei = hm_get(&g->emap, ekey(s, d));
  return ei >= 0 ? &g->es[ei] : NULL;
}

static int cmp_i64(const void* a, const void* b) {
  int64_t x = *(const int64_t*)a, y = *(const int64_t*)b;
  return (x > y) - (x < y);
}

long orc_history(const orc_graph* g, int is_edge, int64_t src, int64_t dst,
                 int64_t* times, uint8_t* flags, size_t cap) {
  const Entity* e;
  if (is_edge) {
    const Edge* x = find_edge(g, src, dst);
    if (!x) return -1;
    if (g->lazy) { /* merged history: every own key and endpoint death key, winner by put order */
      size_t nk = (size_t)x->e.hist.n + (size_t)g->vs[x->si].e.rem.n +
                  (x->di != x->si ? (size_t)g->vs[x->di].e.rem.n : 0);
      int64_t* ks = (int64_t*)malloc(sizeof(int64_t) * (nk ? nk : 1));
      if (!ks) return -1;
      size_t m = 0;
      for (int i = 0; i < x->e.hist.n; i++) ks[m++] = x->e.hist.k[i];
      for (int i = 0; i < g->vs[x->si].e.rem.n; i++) ks[m++] = g->vs[x->si].e.rem.k[i];
      if (x->di != x->si)
        for (int i = 0; i < g->vs[x->di].e.rem.n; i++) ks[m++] = g->vs[x->di].e.rem.k[i];
      qsort(ks, m, sizeof(int64_t), cmp_i64);
      long n = 0;
      for (size_t i = 0; i < m; i++) {
        if (i && ks[i] == ks[i - 1]) continue;
        int64_t c; int v;
        lazy_closest(g, x, ks[i], &c, &v);
        if ((size_t)n < cap) { times[n] = ks[i]; flags[n] = (uint8_t)v; }
        n++;
      }
      free(ks);
      return n;
    }
    e = &x->e;
  } else {
    const Vertex* v = find_vertex(g, src);
    if (!v) return -1;
    e = &v->e;
  }
  for (int i = 0; i < e->hist.n && (size_t)i < cap; i++) { times[i] = e->hist.k[i]; flags[i] = e->hist.v[i]; }
  return e->hist.n;
}

int orc_alive(const orc_graph* g, int is_edge, int64_t src, int64_t dst, int64_t t, int64_t window) {
  if (is_edge) {
    const Edge* e = find_edge(g, src, dst);
    return e ? edge_alive(g, e, t, window) : 0;
  }
  const Vertex* v = find_vertex(g, src);
  return v ? ent_alive(&v->e, t, window) : 0;
}

/* ------------------------------------------------------------ lens helpers */
/* Window list of the job: nw == 0 => ViewLens (aliveAt, window -1), ReaderWorker.scala:324-352. */
typedef struct {
  int nwin;
  int64_t w[64];
  int canon[64]; /* comp keys / job ids are name+t+w (VertexVisitor.scala:81-96, WindowLens.scala:52):
                    equal window values share state */
} WinSet;

static int winset_init(WinSet* ws, const int64_t* windows, int nw) {
  if (nw < 0 || nw > 64) return -1;
  ws->nwin = nw ? nw : 1;
  for (int i = 0; i < ws->nwin; i++) {
    ws->w[i] = nw ? windows[i] : -1;
    if (nw && windows[i] < 0) return -1;
    ws->canon[i] = i;
    for (int j = 0; j < i; j++) if (ws->w[j] == ws->w[i]) { ws->canon[i] = ws->canon[j]; break; }
  }
  return 0;
}

/* Lens key sets: new WindowLens(t, w0) filters every vertex (WindowLens.scala:23-24), then
 * shrinkWindow(w_i) filters the running key set (WindowLens.scala:59-65).  mem[i*nv + v]. */
static void build_keysets(const orc_graph* g, int64_t t, const WinSet* ws, uint8_t* mem) {
  size_t nv = g->nv;
  for (size_t v = 0; v < nv; v++) mem[v] = (uint8_t)ent_alive(&g->vs[v].e, t, ws->w[0]);
  for (int i = 1; i < ws->nwin; i++)
    for (size_t v = 0; v < nv; v++)
      mem[(size_t)i * nv + v] = mem[(size_t)(i - 1) * nv + v] && ent_alive(&g->vs[v].e, t, ws->w[i]);
}

/* messageAllNeighbours: keys(outgoingProcessing) ∪ keys(incomingProcessing) after
 * viewAtWithWindow(t, setWindow) (VertexVisitor.scala:119-120, Vertex.scala:70-74).
 * Writes distinct neighbour vertex indices into nb; uses mark[] (all zero on entry/exit). */
static int neighbours(const orc_graph* g, int vi, int64_t t, int64_t w, int* nb, uint8_t* mark) {
  const Vertex* v = &g->vs[vi];
  int n = 0;
  for (int i = 0; i < v->out.n; i++) {
    const Edge* e = &g->es[v->out.a[i]];
    if (!edge_alive(g, e, t, w)) continue;
    int x = hm_get(&g->vmap, (uint64_t)e->dst);
    if (!mark[x]) { mark[x] = 1; nb[n++] = x; }
  }
  for (int i = 0; i < v->in.n; i++) {
    const Edge* e = &g->es[v->in.a[i]];
    if (!edge_alive(g, e, t, w)) continue;
    int x = hm_get(&g->vmap, (uint64_t)e->src);
    if (!mark[x]) { mark[x] = 1; nb[n++] = x; }
  }
  for (int i = 0; i < n; i++) mark[nb[i]] = 0;
  return n;
}

/* ------------------------------------------------------------------- CC */
int orc_cc(const orc_graph* g, int64_t t, const int64_t* windows, int nw, int max_steps,
           int mode, int64_t* ids, int64_t* labels, size_t cap, size_t* n_out, int* steps) {
  WinSet ws;
  if (winset_init(&ws, windows, nw) != 0) return -1;
  size_t nv = g->nv;
  int nwin = ws.nwin;
  size_t nvs = nv ? nv : 1;
  uint8_t* mem = (uint8_t*)calloc((size_t)nwin * nvs, 1);
  uint8_t* lset = (uint8_t*)calloc((size_t)nwin * nvs, 1);      /* computationValues contains */
  int64_t* lbl = (int64_t*)malloc(sizeof(int64_t) * nwin * nvs);
  int64_t* qmin = (int64_t*)malloc(sizeof(int64_t) * 2 * nwin * nvs); /* VertexMutliQueue even/odd */
  uint32_t* qcnt = (uint32_t*)calloc((size_t)2 * nwin * nvs, sizeof(uint32_t));
  int* nb = (int*)malloc(sizeof(int) * nvs);
  int* list = (int*)malloc(sizeof(int) * nvs);
  uint8_t* mark = (uint8_t*)calloc(nvs, 1);
  /* mode 1 cache: filtered neighbour lists per (window, vertex) */
  int** nbc = NULL; int* nbn = NULL;
  int rc = -1;
  if (!mem || !lset || !lbl || !qmin || !qcnt || !nb || !list || !mark) goto done;
  *steps = 0;

  build_keysets(g, t, &ws, mem);
  if (mode == 1) {
    nbc = (int**)calloc((size_t)nwin * nvs, sizeof(int*));
    nbn = (int*)calloc((size_t)nwin * nvs, sizeof(int));
    if (!nbc || !nbn) goto done;
    for (int i = 0; i < nwin; i++)
      for (size_t v = 0; v < nv; v++) {
        if (!mem[(size_t)i * nv + v]) continue;
        int k = neighbours(g, (int)v, t, ws.w[i], nb, mark);
        nbn[(size_t)i * nv + v] = k;
        nbc[(size_t)i * nv + v] = (int*)malloc(sizeof(int) * (k ? k : 1));
        if (!nbc[(size_t)i * nv + v]) goto done;
        memcpy(nbc[(size_t)i * nv + v], nb, sizeof(int) * k);
      }
  }

#define NEIGH(i, v, outp, outn)                                                  \
  do {                                                                           \
    if (mode == 1) { outp = nbc[(size_t)(i) * nv + (v)]; outn = nbn[(size_t)(i) * nv + (v)]; } \
    else { outn = neighbours(g, (v), t, ws.w[i], nb, mark); outp = nb; }         \
  } while (0)
#define SEND(i, step, lab, v)                                                   \
  do {                                                                           \
    const int* np_; int nn_;                                                     \
    NEIGH(i, v, np_, nn_);                                                       \
    size_t qb_ = ((size_t)((step) + 1) % 2 * nwin + ws.canon[i]) * nv;           \
    for (int q_ = 0; q_ < nn_; q_++) {                                           \
      size_t x_ = qb_ + np_[q_];                                                 \
      if (qcnt[x_] == 0 || (lab) < qmin[x_]) qmin[x_] = (lab);                   \
      qcnt[x_]++;                                                                \
    }                                                                            \
  } while (0)

  if (max_steps > 1) { /* AnalysisTask.timeResponse :169 — Setup only when maxSteps > 1 */
    /* ReaderWorker.setup :173-186 — ConnectedComponents.setup :10-17 per window */
    for (int i = 0; i < nwin; i++) {
      int c = ws.canon[i];
      for (size_t v = 0; v < nv; v++) {
        if (!mem[(size_t)i * nv + v]) continue;
        size_t li = (size_t)c * nv + v;
        if (!lset[li]) { lset[li] = 1; lbl[li] = g->vs[v].id; } /* getOrSetCompValue("cclabel", id) */
        int64_t toSend = lbl[li];
        SEND(i, 0, toSend, (int)v);
      }
    }
    for (int s = 1;; s++) {
      /* ReaderWorker.nextStep :190-219 — a NEW WindowLens per superstep */
      if (mode == 0) build_keysets(g, t, &ws, mem);
      long totalKeys = 0, votes = 0;
      for (int i = 0; i < nwin; i++) {
        int c = ws.canon[i];
        size_t qb = ((size_t)(s % 2) * nwin + c) * nv;
        /* getVerticesWithMessages, WindowLens.scala:41-50 */
        int nl = 0;
        for (size_t v = 0; v < nv; v++)
          if (mem[(size_t)i * nv + v] && qcnt[qb + v] > 0) list[nl++] = (int)v;
        totalKeys += nl;
        /* ConnectedComponents.analyse :19-35 */
        for (int a = 0; a < nl; a++) {
          int v = list[a];
          int64_t label = qmin[qb + v];
          qcnt[qb + v] = 0; /* clearQueue */
          size_t li = (size_t)c * nv + v;
          if (!lset[li]) { lset[li] = 1; lbl[li] = label; }
          int64_t cur = lbl[li];
          if (label < cur) { lbl[li] = label; SEND(i, s, label, v); }
          else votes++;
        }
      }
      *steps = s;
      /* AnalysisTask.endStep :208-225, WindowLens.checkVotes WindowLens.scala:67-68 */
      if (s == max_steps || totalKeys == votes) break;
    }
  }
  /* ReaderWorker.returnResults :232-257 — ConnectedComponents.returnResults :37-42 */
  if (mode == 0) build_keysets(g, t, &ws, mem);
  for (int i = 0; i < nwin; i++) {
    int c = ws.canon[i];
    size_t k = 0;
    for (size_t r = 0; r < nv; r++) {
      int v = g->order[r];
      if (!mem[(size_t)i * nv + v]) continue;
      if (k >= cap) goto done;
      size_t li = (size_t)c * nv + v;
      ids[(size_t)i * cap + k] = g->vs[v].id;
      labels[(size_t)i * cap + k] = lset[li] ? lbl[li] : g->vs[v].id;
      k++;
    }
    n_out[i] = k;
  }
  rc = 0;
#undef SEND
#undef NEIGH
done:
  if (nbc) { for (size_t i = 0; i < (size_t)nwin * nvs; i++) free(nbc[i]); free(nbc); }
  free(nbn);
  free(mem); free(lset); free(lbl); free(qmin); free(qcnt); free(nb); free(list); free(mark);
  return rc;
}

/* ---------------------------------------------------------------- degree */
static void vertex_degree(const orc_graph* g, int v, int64_t t, int64_t w, int32_t* od, int32_t* id) {
  const Vertex* x = &g->vs[v];
  int32_t o = 0, in = 0;
  for (int i = 0; i < x->out.n; i++) o += edge_alive(g, &g->es[x->out.a[i]], t, w);
  for (int i = 0; i < x->in.n; i++) in += edge_alive(g, &g->es[x->in.a[i]], t, w);
  *od = o; *id = in;
}

int orc_degree(const orc_graph* g, int64_t t, const int64_t* windows, int nw,
               int64_t* ids, int32_t* outdeg, int32_t* indeg, size_t cap, size_t* n_out) {
  WinSet ws;
  if (winset_init(&ws, windows, nw) != 0) return -1;
  size_t nv = g->nv;
  uint8_t* mem = (uint8_t*)calloc((size_t)ws.nwin * (nv ? nv : 1), 1);
  if (!mem) return -1;
  build_keysets(g, t, &ws, mem);
  for (int i = 0; i < ws.nwin; i++) {
    size_t k = 0;
    for (size_t r = 0; r < nv; r++) {
      int v = g->order[r];
      if (!mem[(size_t)i * nv + v]) continue;
      if (k >= cap) { free(mem); return -1; }
      size_t o = (size_t)i * cap + k;
      ids[o] = g->vs[v].id;
      vertex_degree(g, v, t, ws.w[i], &outdeg[o], &indeg[o]);
      k++;
    }
    n_out[i] = k;
  }
  free(mem);
  return 0;
}

/* -------------------------------------------------------------- pagerank */
int orc_pagerank(const orc_graph* g, int64_t t, const int64_t* windows, int nw, int iters,
                 int64_t* ids, double* pr, size_t cap, size_t* n_out) {
  WinSet ws;
  if (winset_init(&ws, windows, nw) != 0) return -1;
  size_t nv = g->nv, nvs = nv ? nv : 1;
  uint8_t* mem = (uint8_t*)calloc((size_t)ws.nwin * nvs, 1);
  double* cur = (double*)malloc(sizeof(double) * nvs);
  double* nxt = (double*)malloc(sizeof(double) * nvs);
  int32_t* od = (int32_t*)malloc(sizeof(int32_t) * nvs);
  /* per window: alive out-edges of members whose dst is a member, as CSR (the messages
   * messageAllOutgoingNeighbors would send and a member would read), built once per view */
  size_t* off = (size_t*)malloc(sizeof(size_t) * (nvs + 1));
  int* adj = NULL;
  size_t adj_cap = 0;
  int rc = -1;
  if (!mem || !cur || !nxt || !od || !off) goto done;
  build_keysets(g, t, &ws, mem);
  for (int i = 0; i < ws.nwin; i++) {
    const uint8_t* m = mem + (size_t)i * nv;
    size_t ne_w = 0;
    off[0] = 0;
    for (size_t u = 0; u < nv; u++) {
      cur[u] = 1.0; /* defaultPR, PageRank.scala:14 */
      od[u] = 0;
      if (m[u]) {
        const Vertex* x = &g->vs[u];
        for (int k = 0; k < x->out.n; k++) {
          const Edge* e = &g->es[x->out.a[k]];
          if (!edge_alive(g, e, t, ws.w[i])) continue;
          od[u]++; /* out-degree counts every alive out-edge (DegreeBasic), member dst or not */
          int d = hm_get(&g->vmap, (uint64_t)e->dst);
          if (!m[d]) continue;
          if (ne_w == adj_cap) {
            size_t nc = adj_cap ? 2 * adj_cap : 1024;
            int* na = (int*)realloc(adj, sizeof(int) * nc);
            if (!na) goto done;
            adj = na; adj_cap = nc;
          }
          adj[ne_w++] = d;
        }
      }
      off[u + 1] = ne_w;
    }
    for (int it = 0; it < iters; it++) {
      for (size_t v = 0; v < nv; v++) nxt[v] = 0.0;
      for (size_t u = 0; u < nv; u++) {
        if (!m[u]) continue;
        double c = cur[u] / (double)(od[u] > 1 ? od[u] : 1); /* max(outdeg,1), PageRank.scala:35 */
        for (size_t k = off[u]; k < off[u + 1]; k++) nxt[adj[k]] += c;
      }
      for (size_t v = 0; v < nv; v++) cur[v] = m[v] ? 0.15 + 0.85 * nxt[v] : 1.0; /* d = 0.85, :11 */
    }
    size_t k = 0;
    for (size_t r = 0; r < nv; r++) {
      int v = g->order[r];
      if (!m[v]) continue;
      if (k >= cap) goto done;
      ids[(size_t)i * cap + k] = g->vs[v].id;
      pr[(size_t)i * cap + k] = cur[v];
      k++;
    }
    n_out[i] = k;
  }
  rc = 0;
done:
  free(mem); free(cur); free(nxt); free(od); free(off); free(adj);
  return rc;
}

/* ------------------------------------------------------------ diffusion */
/* BinaryDefusion.scala:9-51 run through the reference's BSP: Setup (superstep 0, only when
 * maxSteps > 1, AnalysisTask.scala:169), then per superstep s the vertices with messages
 * (getVerticesWithMessages, WindowLens.scala:41-50) clear their queue; an infected one
 * votes to halt (:27-28), a new one records infected = s and messages every out-neighbour
 * (outgoingProcessing after viewAtWithWindow, VertexVisitor.scala:32) on a coin flip (:31-33);
 * halt at s == maxSteps or when every message holder voted (AnalysisTask.endStep :208-225).
 * The coin replaces the unseeded Random.nextBoolean() by the hash specified in
 * include/rgpu.h (rgpu_set_diffusion); coin == 0 sends every message. */
static uint64_t dmix(uint64_t x) {
  x ^= x >> 30; x *= 0xbf58476d1ce4e5b9ull; x ^= x >> 27; x *= 0x94d049bb133111ebull; x ^= x >> 31;
  return x;
}
static int dcoin(uint64_t salt, int64_t u, int64_t v, int r) {
  uint64_t a = dmix((uint64_t)v + (uint64_t)(int64_t)r);
  uint64_t b = dmix(((uint64_t)u * 0x9E3779B97F4A7C15ull) ^ a);
  return (int)(dmix(salt ^ b) >> 63);
}

int orc_diffusion(const orc_graph* g, int64_t t, const int64_t* windows, int nw, int max_steps,
                  int64_t seed_id, uint64_t coin_seed, int coin, int64_t* ids, int32_t* step_out,
                  size_t cap, size_t* n_out, int* steps) {
  WinSet ws;
  if (winset_init(&ws, windows, nw) != 0) return -1;
  size_t nv = g->nv, nvs = nv ? nv : 1;
  int nwin = ws.nwin;
  uint8_t* mem = (uint8_t*)calloc((size_t)nwin * nvs, 1);
  int32_t* inf = (int32_t*)malloc(sizeof(int32_t) * nwin * nvs);  /* compValue "infected", -1 = none */
  uint32_t* q = (uint32_t*)calloc((size_t)2 * nwin * nvs, sizeof(uint32_t)); /* queue sizes, parity */
  int* list = (int*)malloc(sizeof(int) * nvs);
  uint64_t salt[64];
  int rc = -1;
  if (!mem || !inf || !q || !list) goto done;
  for (size_t i = 0; i < (size_t)nwin * nvs; i++) inf[i] = -1;
  for (int i = 0; i < nwin; i++) salt[i] = dmix(coin_seed ^ dmix((uint64_t)t ^ dmix((uint64_t)ws.w[i])));
  build_keysets(g, t, &ws, mem);
  *steps = 0;
  /* messageNeighbour to every out-neighbour of v whose edge is alive in the view */
#define DSEND(i, s, v)                                                                   \
  do {                                                                                   \
    const Vertex* x_ = &g->vs[(v)];                                                      \
    size_t qb_ = ((size_t)(((s) + 1) % 2) * nwin + ws.canon[i]) * nv;                    \
    for (int k_ = 0; k_ < x_->out.n; k_++) {                                             \
      const Edge* e_ = &g->es[x_->out.a[k_]];                                            \
      if (!edge_alive(g, e_, t, ws.w[i])) continue;                                       \
      int d_ = hm_get(&g->vmap, (uint64_t)e_->dst);                                      \
      if (!coin || dcoin(salt[i], x_->id, e_->dst, (s))) q[qb_ + d_]++;                  \
    }                                                                                    \
  } while (0)
  if (max_steps > 1) {
    int32_t sv = hm_get(&g->vmap, (uint64_t)seed_id);
    for (int i = 0; i < nwin; i++) { /* setup :11-21 */
      if (seed_id < 0 || seed_id >= ((int64_t)1 << 31) || sv < 0 || !mem[(size_t)i * nv + sv]) continue;
      size_t li = (size_t)ws.canon[i] * nv + sv;
      if (inf[li] < 0) inf[li] = 0;  /* getOrSetCompValue("infected", superStep = 0) */
      DSEND(i, 0, sv);
    }
    for (int s = 1;; s++) {
      long totalKeys = 0, votes = 0;
      for (int i = 0; i < nwin; i++) {
        int c = ws.canon[i];
        size_t qb = ((size_t)(s % 2) * nwin + c) * nv;
        int nl = 0;
        for (size_t v = 0; v < nv; v++)
          if (mem[(size_t)i * nv + v] && q[qb + v] > 0) list[nl++] = (int)v;
        totalKeys += nl;
        for (int a = 0; a < nl; a++) { /* analyse :23-36 */
          int v = list[a];
          q[qb + v] = 0; /* clearQueue */
          size_t li = (size_t)c * nv + v;
          if (inf[li] >= 0) { votes++; continue; }
          inf[li] = s;
          DSEND(i, s, v);
        }
      }
      *steps = s;
      if (s == max_steps || totalKeys == votes) break;
    }
  }
#undef DSEND
  for (int i = 0; i < nwin; i++) { /* returnResults :38-49, ascending id */
    size_t k = 0;
    for (size_t r = 0; r < nv; r++) {
      int v = g->order[r];
      if (!mem[(size_t)i * nv + v]) continue;
      int32_t x = inf[(size_t)ws.canon[i] * nv + v];
      if (x < 0) continue;
      if (k >= cap) goto done;
      ids[(size_t)i * cap + k] = g->vs[v].id;
      step_out[(size_t)i * cap + k] = x;
      k++;
    }
    n_out[i] = k;
  }
  rc = 0;
done:
  free(mem); free(inf); free(q); free(list);
  return rc;
}

/* ------------------------------------------------------- vertex program */
static int64_t vp_add(int64_t a, int64_t b) { /* saturating a + b */
  if (b > 0 && a > INT64_MAX - b) return INT64_MAX;
  if (b < 0 && a < INT64_MIN - b) return INT64_MIN;
  return a + b;
}
/* keys(outgoingProcessing) (dir 0), keys(incomingProcessing) (1) or their union (2) after
 * viewAtWithWindow (Vertex.scala:70-74); a self-loop is an outgoing key only
 * (EntityStorage.scala:257) */
static int vp_neighbours(const orc_graph* g, int vi, int64_t t, int64_t w, int dir, int* nb, uint8_t* mark) {
  const Vertex* v = &g->vs[vi];
  int n = 0;
  if (dir != 1)
    for (int i = 0; i < v->out.n; i++) {
      const Edge* e = &g->es[v->out.a[i]];
      if (!edge_alive(g, e, t, w)) continue;
      int x = hm_get(&g->vmap, (uint64_t)e->dst);
      if (!mark[x]) { mark[x] = 1; nb[n++] = x; }
    }
  if (dir != 0)
    for (int i = 0; i < v->in.n; i++) {
      const Edge* e = &g->es[v->in.a[i]];
      if (!edge_alive(g, e, t, w)) continue;
      int x = hm_get(&g->vmap, (uint64_t)e->src);
      if (!mark[x]) { mark[x] = 1; nb[n++] = x; }
    }
  for (int i = 0; i < n; i++) mark[nb[i]] = 0;
  return n;
}

int orc_vertex_program(const orc_graph* g, int64_t t, const int64_t* windows, int nw, int max_steps,
                       int dir, int reduce, int init, int senders, int64_t init_value, int64_t seed_id,
                       int64_t seed_value, int64_t step_add, int64_t* ids, int64_t* values, size_t cap,
                       size_t* n_out, int* steps) {
  WinSet ws;
  if (winset_init(&ws, windows, nw) != 0 || dir < 0 || dir > 2 || reduce < 0 || reduce > 1) return -1;
  size_t nv = g->nv, nvs = nv ? nv : 1;
  int nwin = ws.nwin;
  uint8_t* mem = (uint8_t*)calloc((size_t)nwin * nvs, 1);
  uint8_t* sset = (uint8_t*)calloc((size_t)nwin * nvs, 1);       /* computationValues contains */
  int64_t* st = (int64_t*)malloc(sizeof(int64_t) * nwin * nvs);
  int64_t* qv = (int64_t*)malloc(sizeof(int64_t) * 2 * nwin * nvs); /* queue fold, even/odd parity */
  uint32_t* qc = (uint32_t*)calloc((size_t)2 * nwin * nvs, sizeof(uint32_t));
  int* nb = (int*)malloc(sizeof(int) * nvs);
  int* list = (int*)malloc(sizeof(int) * nvs);
  uint8_t* mark = (uint8_t*)calloc(nvs, 1);
  int rc = -1;
  int32_t sv = (seed_id >= 0 && seed_id < ((int64_t)1 << 31)) ? hm_get(&g->vmap, (uint64_t)seed_id) : -1;
  if (!mem || !sset || !st || !qv || !qc || !nb || !list || !mark) goto done;
  *steps = 0;
  build_keysets(g, t, &ws, mem);
#define VSEND(i, s, val, v)                                                        \
  do {                                                                             \
    int nn_ = vp_neighbours(g, (v), t, ws.w[i], dir, nb, mark);                    \
    size_t qb_ = ((size_t)(((s) + 1) % 2) * nwin + ws.canon[i]) * nv;              \
    for (int q_ = 0; q_ < nn_; q_++) {                                             \
      size_t x_ = qb_ + nb[q_];                                                    \
      if (qc[x_] == 0 || (reduce == 0 ? (val) < qv[x_] : (val) > qv[x_])) qv[x_] = (val); \
      qc[x_]++;                                                                    \
    }                                                                              \
  } while (0)
  if (max_steps > 1) { /* AnalysisTask.timeResponse :169 */
    for (int i = 0; i < nwin; i++) {
      int c = ws.canon[i];
      for (size_t v = 0; v < nv; v++) {
        if (!mem[(size_t)i * nv + v]) continue;
        size_t li = (size_t)c * nv + v;
        if (!sset[li]) { /* getOrSetCompValue */
          sset[li] = 1;
          st[li] = init == 0 ? g->vs[v].id : ((int32_t)v == sv ? seed_value : init_value);
        }
        if (senders == 0 || (int32_t)v == sv) VSEND(i, 0, vp_add(st[li], step_add), (int)v);
      }
    }
    for (int s = 1;; s++) {
      long totalKeys = 0, votes = 0;
      for (int i = 0; i < nwin; i++) {
        int c = ws.canon[i];
        size_t qb = ((size_t)(s % 2) * nwin + c) * nv;
        int nl = 0;
        for (size_t v = 0; v < nv; v++) /* getVerticesWithMessages, WindowLens.scala:41-50 */
          if (mem[(size_t)i * nv + v] && qc[qb + v] > 0) list[nl++] = (int)v;
        totalKeys += nl;
        for (int a = 0; a < nl; a++) {
          int v = list[a];
          int64_t m = qv[qb + v];
          qc[qb + v] = 0; /* clearQueue */
          size_t li = (size_t)c * nv + v;
          int64_t cur = st[li];
          int64_t nx = reduce == 0 ? (m < cur ? m : cur) : (m > cur ? m : cur);
          if (nx != cur) { st[li] = nx; VSEND(i, s, vp_add(nx, step_add), v); }
          else votes++;
        }
      }
      *steps = s;
      if (s == max_steps || totalKeys == votes) break;
    }
  }
#undef VSEND
  for (int i = 0; i < nwin; i++) {
    int c = ws.canon[i];
    size_t k = 0;
    for (size_t r = 0; r < nv; r++) {
      int v = g->order[r];
      if (!mem[(size_t)i * nv + v]) continue;
      if (k >= cap) goto done;
      size_t li = (size_t)c * nv + v;
      ids[(size_t)i * cap + k] = g->vs[v].id;
      values[(size_t)i * cap + k] = sset[li] ? st[li] : (init == 0 ? g->vs[v].id : ((int32_t)v == sv ? seed_value : init_value));
      k++;
    }
    n_out[i] = k;
  }
  rc = 0;
done:
  free(mem); free(sset); free(st); free(qv); free(qc); free(nb); free(list); free(mark);
  return rc;
}

/* Float vertex programs (include/rgpu.h rgpu_vertex_program_f_t): VertexMessageFloat messages
 * (raphtoryMessages.scala:117, VertexVisitor.scala:137-147) summed.  The reference's BSP as
 * orc_vertex_program: Setup sends, then every member holding messages takes (float)(bias + mult *
 * sum) and sends again (no vote to halt); the job halts when no member held a message, or at
 * maxSteps.  A message is the sender's state, or with per_degree (float)(state / max(deg, 1)), deg
 * = its message targets alive in the view (vp_neighbours: distinct, members or not).  The queue sums
 * in double in arrival order (the reference sums Floats in nondeterministic arrival order). */
int orc_vertex_program_f(const orc_graph* g, int64_t t, const int64_t* windows, int nw, int max_steps, int dir,
                         int init, int senders, int per_degree, int64_t seed_id, double init_value, double seed_value,
                         double bias, double mult, int64_t* ids, double* values, size_t cap, size_t* n_out,
                         int* steps) {
  WinSet ws;
  if (winset_init(&ws, windows, nw) != 0 || dir < 0 || dir > 2) return -1;
  size_t nv = g->nv, nvs = nv ? nv : 1;
  int nwin = ws.nwin;
  uint8_t* mem = (uint8_t*)calloc((size_t)nwin * nvs, 1);
  uint8_t* sset = (uint8_t*)calloc((size_t)nwin * nvs, 1);
  double* st = (double*)malloc(sizeof(double) * nwin * nvs);
  double* qs = (double*)calloc((size_t)2 * nwin * nvs, sizeof(double)); /* queue sums, even/odd parity */
  uint32_t* qc = (uint32_t*)calloc((size_t)2 * nwin * nvs, sizeof(uint32_t));
  int* nb = (int*)malloc(sizeof(int) * nvs);
  int* list = (int*)malloc(sizeof(int) * nvs);
  uint8_t* mark = (uint8_t*)calloc(nvs, 1);
  int rc = -1;
  int32_t sv = (seed_id >= 0 && seed_id < ((int64_t)1 << 31)) ? hm_get(&g->vmap, (uint64_t)seed_id) : -1;
  if (!mem || !sset || !st || !qs || !qc || !nb || !list || !mark) goto done;
  *steps = 0;
  build_keysets(g, t, &ws, mem);
#define FSEND(i, s, val, v)                                                        \
  do {                                                                             \
    int nn_ = vp_neighbours(g, (v), t, ws.w[i], dir, nb, mark);                    \
    const double x_ = per_degree ? (double)(float)((val) / (double)(nn_ > 1 ? nn_ : 1)) : (val); \
    size_t qb_ = ((size_t)(((s) + 1) % 2) * nwin + ws.canon[i]) * nv;              \
    for (int q_ = 0; q_ < nn_; q_++) {                                             \
      qs[qb_ + nb[q_]] += x_;                                                      \
      qc[qb_ + nb[q_]]++;                                                          \
    }                                                                              \
  } while (0)
  if (max_steps > 1) { /* AnalysisTask.timeResponse :169 */
    for (int i = 0; i < nwin; i++) {
      int c = ws.canon[i];
      for (size_t v = 0; v < nv; v++) {
        if (!mem[(size_t)i * nv + v]) continue;
        size_t li = (size_t)c * nv + v;
        if (!sset[li]) {
          sset[li] = 1;
          st[li] = (double)(float)(init == 0 ? (double)g->vs[v].id : ((int32_t)v == sv ? seed_value : init_value));
        }
        if (senders == 0 || (int32_t)v == sv) FSEND(i, 0, st[li], (int)v);
      }
    }
    for (int s = 1;; s++) {
      long totalKeys = 0;
      for (int i = 0; i < nwin; i++) {
        int c = ws.canon[i];
        size_t qb = ((size_t)(s % 2) * nwin + c) * nv;
        int nl = 0;
        for (size_t v = 0; v < nv; v++)
          if (mem[(size_t)i * nv + v] && qc[qb + v] > 0) list[nl++] = (int)v;
        totalKeys += nl;
        for (int a = 0; a < nl; a++) { /* every message holder updates and sends (it never votes) */
          int v = list[a];
          size_t li = (size_t)c * nv + v;
          st[li] = (double)(float)(bias + mult * qs[qb + v]);
          qs[qb + v] = 0.0;
          qc[qb + v] = 0;
          FSEND(i, s, st[li], v);
        }
        for (size_t v = 0; v < nv; v++) { qs[qb + v] = 0.0; qc[qb + v] = 0; } /* non-members' drops */
      }
      *steps = s;
      if (s == max_steps || totalKeys == 0) break;
    }
  }
#undef FSEND
  for (int i = 0; i < nwin; i++) {
    int c = ws.canon[i];
    size_t k = 0;
    for (size_t r = 0; r < nv; r++) {
      int v = g->order[r];
      if (!mem[(size_t)i * nv + v]) continue;
      if (k >= cap) goto done;
      size_t li = (size_t)c * nv + v;
      ids[(size_t)i * cap + k] = g->vs[v].id;
      values[(size_t)i * cap + k] = sset[li] ? st[li]
                                             : (double)(float)(init == 0 ? (double)g->vs[v].id
                                                                         : ((int32_t)v == sv ? seed_value : init_value));
      k++;
    }
    n_out[i] = k;
  }
  rc = 0;
done:
  free(mem); free(sset); free(st); free(qs); free(qc); free(nb); free(list); free(mark);
  return rc;
}

/* ============================================================ add-only streams (C4 / GAB)
 * A memory-compact restatement for streams of VertexAdds and EdgeAdds only, in time order
 * (GabUserGraphRouter.scala:31-33 emits nothing else).  Every history point is then an add, and
 * Entity.aliveAtWithWindow (Entity.scala:193-201) — floor(t) is an add and t - floor(t) <= w —
 * holds iff the entity has a point in [t - w, t] (the floor is the newest point <= t).  A vertex
 * has a point at its VertexAdds and at every EdgeAdd touching it (EntityStorage.scala:240,259);
 * an edge (s,d) at its EdgeAdds.  So the view (t, w) is read off the time-sorted stream itself:
 * its members are the endpoints of the updates with time in [t - w_v, t] (w_v = min(w_0..w_i),
 * WindowLens.shrinkWindow), its edges the EdgeAdds in [t - w_i, t] (WindowLens.scala:54-65) — no
 * per-entity TreeMap, so a year of the 1B-update C4 stream fits in memory.
 * ConnectedComponents (ConnectedComponents.scala:10-35) runs as the Jacobi form of its BSP:
 * label_r(v) = min(label_{r-1}(v), label_{r-1}(u) for u in N(v)) over members and edges with both
 * ends members (a message to a non-member is never processed, WindowLens.scala:41-50).  A vertex
 * whose neighbour did not change in r-1 already received that label, so this is the message form
 * of orc_cc exactly.  The hop's supersteps: a window's labels change in steps 1..D_w exactly (the
 * vertex at distance k from its component minimum changes at step k), so the BSP, which halts
 * when no window improved (AnalysisTask.scala:208-225), runs min(maxSteps, 1 + max_w D_w) steps.
 * Checked against orc_cc on random add-only streams and the C4 prefix goldens
 * (tests/test_oracle_addonly.py). */
struct orc_addonly {
  const int64_t* t;      /* the caller's time column (kept alive by the caller) */
  size_t n;
  int32_t *s, *d;        /* dense ranks of src / dst (d = -1 for a VertexAdd) */
  int64_t* ids;          /* rank -> id, ascending */
  size_t nv;
};


orc_addonly* orc_addonly_build(const int64_t* t, const uint8_t* kind, const int64_t* src, const int64_t* dst,
                               size_t n) {
  orc_addonly* a = (orc_addonly*)calloc(1, sizeof(orc_addonly));
  if (!a) return NULL;
  a->t = t;
  a->n = n;
  a->s = (int32_t*)malloc(sizeof(int32_t) * (n ? n : 1));
  a->d = (int32_t*)malloc(sizeof(int32_t) * (n ? n : 1));
  HMap m;
  memset(&m, 0, sizeof(m));
  int64_t* tmp = NULL;
  size_t k = 0;
  if (!a->s || !a->d || hm_init(&m, 1 << 20) != 0) goto fail;
  for (size_t i = 0; i < n; i++) { /* validation, then the distinct ids in first-seen order */
    if ((kind[i] != ORC_VADD && kind[i] != ORC_EADD) || t[i] < 0 || (i && t[i] < t[i - 1])) goto fail;
    for (int e = 0; e < (kind[i] == ORC_EADD ? 2 : 1); e++) {
      const int64_t id = e ? dst[i] : src[i];
      if (id < 0 || id >= ((int64_t)1 << 31)) goto fail;
      if (hm_get(&m, (uint64_t)id) < 0) {
        if (hm_put(&m, (uint64_t)id, (int32_t)k) != 0) goto fail;
        k++;
      }
    }
  }
  a->nv = k;
  a->ids = (int64_t*)malloc(sizeof(int64_t) * (k ? k : 1));
  tmp = (int64_t*)malloc(sizeof(int64_t) * (k ? k : 1));
  if (!a->ids || !tmp) goto fail;
  for (size_t i = 0; i < m.cap; i++)
    if (m.vals[i] >= 0) a->ids[m.vals[i]] = (int64_t)m.keys[i];
  memcpy(tmp, a->ids, sizeof(int64_t) * k);
  qsort(tmp, k, sizeof(int64_t), cmp_i64);  /* ranks in id order: min label = min rank */
  for (size_t r = 0; r < k; r++) hm_put(&m, (uint64_t)tmp[r], (int32_t)r);
  memcpy(a->ids, tmp, sizeof(int64_t) * k);
  for (size_t i = 0; i < n; i++) {
    a->s[i] = hm_get(&m, (uint64_t)src[i]);
    a->d[i] = kind[i] == ORC_EADD ? hm_get(&m, (uint64_t)dst[i]) : -1;
  }
  free(tmp);
  free(m.keys);
  free(m.vals);
  return a;
fail:
  free(tmp);
  free(m.keys);
  free(m.vals);
  orc_addonly_free(a);
  return NULL;
}

void orc_addonly_free(orc_addonly* a) {
  if (!a) return;
  free(a->s);
  free(a->d);
  free(a->ids);
  free(a);
}

size_t orc_addonly_num_vertices(const orc_addonly* a) { return a->nv; }

static size_t first_ge(const int64_t* t, size_t n, int64_t x) { /* first index with t >= x */
  size_t lo = 0, hi = n;
  while (lo < hi) {
    size_t mid = (lo + hi) / 2;
    if (t[mid] >= x) hi = mid; else lo = mid + 1;
  }
  return lo;
}

/* one window: members (mem), labels after min(max_steps, D + 1) Jacobi steps; returns D, the
 * last step in which a label changed (capped runs: max_steps), or -1 on allocation failure */
static int addonly_window(const orc_addonly* a, int64_t tq, int64_t wv, int64_t we, int max_steps, uint8_t* mem,
                          int32_t* lab) {
  const size_t nv = a->nv, hi = first_ge(a->t, a->n, tq == INT64_MAX ? tq : tq + 1);
  const size_t lv = wv < 0 ? 0 : first_ge(a->t, hi, tq - wv < 0 ? 0 : tq - wv);
  const size_t le = we < 0 ? 0 : first_ge(a->t, hi, tq - we < 0 ? 0 : tq - we);
  memset(mem, 0, nv);
  for (size_t i = lv; i < hi; i++) {
    mem[a->s[i]] = 1;
    if (a->d[i] >= 0) mem[a->d[i]] = 1;
  }
  for (size_t v = 0; v < nv; v++) lab[v] = (int32_t)v;
  if (max_steps <= 1) return 0;
  size_t* off = (size_t*)calloc(nv + 1, sizeof(size_t));
  int32_t* nxt = (int32_t*)malloc(sizeof(int32_t) * (nv ? nv : 1));
  uint8_t* chg = (uint8_t*)malloc(nv ? nv : 1);
  uint8_t* chn = (uint8_t*)malloc(nv ? nv : 1);
  int32_t* adj = NULL;
  int D = -1;
  if (!off || !nxt || !chg || !chn) goto out;
  for (size_t i = le; i < hi; i++) {
    const int32_t s = a->s[i], d = a->d[i];
    if (d < 0 || !mem[s] || !mem[d]) continue;
    off[s + 1]++;
    off[d + 1]++;
  }
  for (size_t v = 0; v < nv; v++) off[v + 1] += off[v];
  adj = (int32_t*)malloc(sizeof(int32_t) * (off[nv] ? off[nv] : 1));
  if (!adj) goto out;
  {
    size_t* fill = (size_t*)malloc(sizeof(size_t) * (nv ? nv : 1));
    if (!fill) goto out;
    memcpy(fill, off, sizeof(size_t) * nv);
    for (size_t i = le; i < hi; i++) {
      const int32_t s = a->s[i], d = a->d[i];
      if (d < 0 || !mem[s] || !mem[d]) continue;
      adj[fill[s]++] = d;
      adj[fill[d]++] = s;
    }
    free(fill);
  }
  /* Setup (superstep 0): every member sends its own id; supersteps 1..: the changed ones send */
  for (size_t v = 0; v < nv; v++) chg[v] = mem[v];
  D = 0;
  for (int r = 1;; r++) {
    memcpy(nxt, lab, sizeof(int32_t) * nv);
    for (size_t u = 0; u < nv; u++) {
      if (!chg[u]) continue;
      const int32_t x = lab[u];
      for (size_t k = off[u]; k < off[u + 1]; k++)
        if (x < nxt[adj[k]]) nxt[adj[k]] = x;
    }
    int any = 0;
    for (size_t v = 0; v < nv; v++) {
      chn[v] = nxt[v] < lab[v];
      any |= chn[v];
    }
    memcpy(lab, nxt, sizeof(int32_t) * nv);
    { uint8_t* x = chg; chg = chn; chn = x; }
    if (any) D = r;
    if (!any || r == max_steps) break;
  }
out:
  free(off); free(nxt); free(chg); free(chn); free(adj);
  return D;
}

int orc_addonly_cc(const orc_addonly* a, int64_t t, const int64_t* windows, int nw, int max_steps, int64_t* ids,
                   int64_t* labels, size_t cap, size_t* n_out, int* steps) {
  if (nw < 0 || nw > 64) return -1;
  const size_t nv = a->nv, nvs = nv ? nv : 1;
  uint8_t* mem = (uint8_t*)malloc(nvs);
  int32_t* lab = (int32_t*)malloc(sizeof(int32_t) * nvs);
  int rc = -1, dmax = 0;
  if (!mem || !lab) goto done;
  int64_t run_min = INT64_MAX;
  for (int i = 0; i < (nw ? nw : 1); i++) {
    const int64_t we = nw ? windows[i] : -1;
    if (nw && we < 0) goto done;
    if (nw && we < run_min) run_min = we;
    const int D = addonly_window(a, t, nw ? run_min : -1, we, max_steps, mem, lab);
    if (D < 0) goto done;
    if (D > dmax) dmax = D;
    size_t k = 0;
    for (size_t v = 0; v < nv; v++) {
      if (!mem[v]) continue;
      if (k >= cap) goto done;
      ids[(size_t)i * cap + k] = a->ids[v];
      labels[(size_t)i * cap + k] = a->ids[lab[v]];
      k++;
    }
    n_out[i] = k;
  }
  *steps = max_steps <= 1 ? 0 : (dmax + 1 < max_steps ? dmax + 1 : max_steps);
  rc = 0;
done:
  free(mem);
  free(lab);
  return rc;
}
