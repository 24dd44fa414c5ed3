/*
 * oracle.h — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of Raphtory's windowed temporal-analysis path, written from the
 * reference Scala source (Haaroon/raphtory @ v0).  It is the *checker* for the HIP
 * path: only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load it.  The product library (raphtory_amd/) never links or calls it.
 *
 * Parity status: the reference is Scala/Akka and cannot be built or run in this
 * image (no JDK / scalac / sbt, no dependency cache) and it ships no tests, golden
 * vectors or reproducible sample outputs.  This oracle is therefore pinned only by
 * hand-derived known-answer tests that cite the Scala lines they follow
 * (tests/test_oracle_kat.py, tests/golden/kat_*.json) — "parity unpinned" against
 * reference-run outputs.
 *
 * Event kinds follow GraphUpdate (raphtoryMessages.scala:38-55).
 */
#ifndef RAPHTORY_ORACLE_H
#define RAPHTORY_ORACLE_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum { ORC_VADD = 0, ORC_VDEL = 1, ORC_EADD = 2, ORC_EDEL = 3 };

typedef struct orc_graph orc_graph;

/* Replays the stream, in order, through a restatement of EntityStorage
 * (EntityStorage.scala:73-453) for one Partition Manager.  Returns NULL on bad input. */
orc_graph* orc_build(const int64_t* t, const uint8_t* kind, const int64_t* src,
                     const int64_t* dst, size_t n);

/* Same replay with flags.  ORC_LAZY_EDGES: an edge stores only its own puts; the endpoint
 * deaths that the literal replay copies into every edge (Edge.killList at creation,
 * vertexRemoval's kill loops — O(degree x deaths) for a hub that dies often) are read from the
 * endpoints' removeLists when the edge is evaluated, with the TreeMap's last-put-wins order
 * kept by stream index.  Every query answers identically (tests/test_oracle_scale.py checks
 * the two builds against each other); this one fits power-law streams of 10^8 updates. */
#define ORC_LAZY_EDGES 1
orc_graph* orc_build_ex(const int64_t* t, const uint8_t* kind, const int64_t* src,
                        const int64_t* dst, size_t n, int flags);
void orc_free(orc_graph* g);

size_t orc_num_vertices(const orc_graph* g);
size_t orc_num_edges(const orc_graph* g);

/* History of one entity as the reference leaves it (Entity.previousState,
 * Entity.scala:25), ascending by time.  Returns number of points (may exceed cap),
 * or -1 if the entity does not exist.  Edge = (src,dst); vertex: dst ignored. */
long orc_history(const orc_graph* g, int is_edge, int64_t src, int64_t dst,
                 int64_t* times, uint8_t* flags, size_t cap);

/* Entity.aliveAtWithWindow (Entity.scala:193-201); window < 0 => Entity.aliveAt (:185-191). */
int orc_alive(const orc_graph* g, int is_edge, int64_t src, int64_t dst, int64_t t, int64_t window);

/* ConnectedComponents over one view at time t with the batched window list
 * `windows[nw]` (nw == 0 => ViewLens).  mode 0 = reference structure (lens rebuilt
 * every superstep by linear closestTime scans, adjacency re-filtered on every
 * getVertex); mode 1 = same semantics with per-view caching.
 * Outputs, per window i: n_out[i] vertices written to ids/labels at offset
 * i*cap (ascending id).  *steps = supersteps executed (AnalysisTask.endStep).
 * Returns 0 or -1 (cap too small / bad args). */
int orc_cc(const orc_graph* g, int64_t t, const int64_t* windows, int nw, int max_steps,
           int mode, int64_t* ids, int64_t* labels, size_t cap, size_t* n_out, int* steps);

/* DegreeBasic.returnResults (DegreeBasic.scala:16-28) per window, per vertex. */
int orc_degree(const orc_graph* g, int64_t t, const int64_t* windows, int nw,
               int64_t* ids, int32_t* outdeg, int32_t* indeg, size_t cap, size_t* n_out);

/* PageRank, SURVEY.md App. A.5 spec (the reference PageRank.scala is broken):
 * PR0 = 1, PR' = 0.15 + 0.85 * sum_{u->v} PR(u)/max(outdeg(u),1), fp64, iters rounds. */
/* BinaryDefusion (reference BSP structure, hash coin of include/rgpu.h): per window the
 * infected vertices (ascending id) with their infection superstep. */
int orc_diffusion(const orc_graph* g, int64_t t, const int64_t* windows, int nw, int max_steps,
                  int64_t seed_id, uint64_t coin_seed, int coin, int64_t* ids, int32_t* step_out,
                  size_t cap, size_t* n_out, int* steps);
/* Generic vertex program (VertexVisitor messaging, VertexVisitor.scala:81-166) through the
 * reference's BSP structure (as orc_cc): Setup (superstep 0, only when maxSteps > 1) sets every
 * member's state to init (getOrSetCompValue) and the senders (every member, or only the seed)
 * message their neighbours in direction dir (0 = messageAllOutgoingNeighbors, 1 =
 * messageAllIngoingNeighbors, 2 = messageAllNeighbours) the value state + step_add (saturating);
 * superstep s: a member holding messages folds them with reduce (0 = min, 1 = max); if the fold
 * of its state and that changes the state it keeps it and messages again, else it votes to halt;
 * halt when every message holder voted, or at s == maxSteps.  init: 0 = own id, 1 = init_value
 * (seed_value at the seed).  senders: 0 = all members, 1 = the seed.  Per window: every member's
 * state (ascending id). */
int orc_vertex_program(const orc_graph* g, int64_t t, const int64_t* windows, int nw, int max_steps,
                       int dir, int reduce, int init, int senders, int64_t init_value, int64_t seed_id,
                       int64_t seed_value, int64_t step_add, int64_t* ids, int64_t* values, size_t cap,
                       size_t* n_out, int* steps);
int orc_pagerank(const orc_graph* g, int64_t t, const int64_t* windows, int nw, int iters,
                 int64_t* ids, double* pr, size_t cap, size_t* n_out);
/* Float vertex program (include/rgpu.h rgpu_vertex_program_f_t): VertexMessageFloat summed; per
 * window every member's float state (as a double), ascending id. */
int orc_vertex_program_f(const orc_graph* g, int64_t t, const int64_t* windows, int nw, int max_steps, int dir,
                         int init, int senders, int per_degree, int64_t seed_id, double init_value, double seed_value,
                         double bias, double mult, int64_t* ids, double* values, size_t cap, size_t* n_out,
                         int* steps);

/* Add-only streams (VertexAdds and EdgeAdds in time order — the GAB / C4 shape): a
 * memory-compact restatement that reads each view off the time-sorted stream (oracle.c, "add-only
 * streams", for why that is exact) instead of replaying it into per-entity TreeMaps.  The caller
 * keeps t alive while the object lives.  NULL on another kind, a time out of order, or a bad id.
 * orc_addonly_cc: orc_cc's output contract (per window the members in ascending id and their
 * labels; the hop's superstep count). */
typedef struct orc_addonly orc_addonly;
orc_addonly* orc_addonly_build(const int64_t* t, const uint8_t* kind, const int64_t* src, const int64_t* dst,
                               size_t n);
void orc_addonly_free(orc_addonly* a);
size_t orc_addonly_num_vertices(const orc_addonly* a);
int orc_addonly_cc(const orc_addonly* a, int64_t t, const int64_t* windows, int nw, int max_steps, int64_t* ids,
                   int64_t* labels, size_t cap, size_t* n_out, int* steps);

#ifdef __cplusplus
}
#endif
#endif
