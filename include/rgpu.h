/*
 * rgpu.h — C ABI of librgpu.so, the MI355X-native windowed temporal-analysis library.
 *
 * This is the drop-in boundary that replaces the per-partition analysis hot path of
 * Raphtory (Haaroon/raphtory @ v0).  Citations use
 *   S/ = mainproject/cluster/src/main/scala/com/raphtory/
 * A JNI shim binds these entry points from a GpuReaderWorker that
 * takes the place of S/core/components/PartitionManager/Workers/ReaderWorker.scala.
 *
 * Conventions
 *   - return 0 on success, a negative RGPU_E* code on failure; rgpu_last_error() says why.
 *     Nothing throws or aborts across this boundary.
 *   - caller-owned host arrays are copied during the call and never retained.
 *   - device memory (and, later, communicators) are owned by the rgpu_ctx.
 *   - result buffers are caller-allocated with (cap, *n); if *n > cap, call again.
 *   - calls on one ctx are serialised by an internal mutex (10 ReaderWorker actors run
 *     concurrently on reader-dispatcher, application.conf:246-264), with two exceptions for live
 *     ingest (ABI 9): rgpu_ingest takes only the update log's lock, so it never waits for a run;
 *     rgpu_seal takes a seal lock (one seal at a time) and holds the run mutex only briefly, so a
 *     seal may run concurrently with rgpu_run_view_batch and the result calls (see rgpu_seal).
 *   - times are int64 milliseconds >= 0; vertex ids are int64 in [0, 2^31)
 *     (message targets are truncated with .toInt, VertexVisitor.scala:117-122).
 */
#ifndef RGPU_H
#define RGPU_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RGPU_ABI_VERSION 10

/* error codes */
#define RGPU_OK 0
#define RGPU_EINVAL (-1)   /* bad argument (ids out of range, windows, hop index ...) */
#define RGPU_ESTATE (-2)   /* call not valid in this state (e.g. run before seal) */
#define RGPU_EHIP (-3)     /* HIP runtime failure */
#define RGPU_ENOMEM (-4)   /* host or device allocation failed */
#define RGPU_ENOTSUP (-5)  /* feature not available in this build */

/* GraphUpdate kinds, S/core/model/communication/raphtoryMessages.scala:38-55 */
#define RGPU_VADD 0        /* VertexAdd        -> EntityStorage.vertexAdd      :73-87  */
#define RGPU_VDEL 1        /* VertexDelete     -> EntityStorage.vertexRemoval  :148-232 */
#define RGPU_EADD 2        /* EdgeAdd          -> EntityStorage.edgeAdd        :237-290 */
#define RGPU_EDEL 3        /* EdgeDelete       -> EntityStorage.edgeRemoval    :327-383 */

/* analysers recognised on the GPU (AnalyserPresentCheck by class name, Reader.scala:68-85) */
#define RGPU_ALGO_CC 0     /* S/core/analysis/Algorithms/ConnectedComponents.scala */
#define RGPU_ALGO_DEGREE 1 /* S/core/analysis/Algorithms/DegreeBasic.scala (and DegreeRanking) */
#define RGPU_ALGO_PR 2     /* PageRank per SURVEY.md App. A.5 (reference PageRank.scala is broken) */
#define RGPU_ALGO_DIFFUSION 3 /* S/core/analysis/Algorithms/BinaryDefusion.scala (ABI 5) */
#define RGPU_ALGO_VP 4     /* a generic vertex program, rgpu_set_vertex_program (ABI 7) */

/* rgpu_run_view_batch flags */
#define RGPU_RUN_RETAIN 1   /* keep per-vertex results of every view (for *_vertex_* queries) */
#define RGPU_RUN_PROFILE 2  /* time every kernel launch with HIP events (rgpu_stats) */
#define RGPU_RUN_SERIAL 4   /* one batch in flight (clean per-kernel event times) */
#define RGPU_RUN_EDGE_COUNTS 8  /* count |E_{t,w}| per view (rgpu_cc_summary_t.alive_edges) (ABI 6) */

typedef struct rgpu_ctx rgpu_ctx;

/* ConnectedComponents.processBatchWindowResults summary of one view,
 * ConnectedComponents.scala:137-145 (computed over the label->count map). */
typedef struct {
  int64_t biggest;               /* max component size ("biggest")                 */
  int64_t total;                 /* number of labels ("total")                     */
  int64_t total_without_islands; /* labels with count > 1                          */
  int64_t total_islands;         /* total - total_without_islands                  */
  int64_t clusters_gt2;          /* labels with count > 2 ("clustersGT2")          */
  int64_t sum_all;               /* sum of counts = |view vertices| (proportion)   */
  int64_t sum_without_islands;   /* sum of counts > 1 (proportionWithoutIslands)   */
  int64_t supersteps;            /* supersteps the reference's job for this hop runs: min(maxSteps,
                                    1 + last superstep in which a label of any of the hop's windows
                                    changed); 0 when maxSteps <= 1 (no Setup, AnalysisTask.scala:169)
                                    (ABI 6; before: the step count of the batch holding the view) */
  int64_t alive_edges;           /* |E_{t,w}|: edges alive in the view's window; filled by
                                    RGPU_RUN_EDGE_COUNTS runs, else -1 (ABI 6) */
} rgpu_cc_summary_t;

typedef struct {
  int64_t vertices, edges;       /* packed entity counts of this partition */
  int64_t vertex_events, edge_events, deaths;
  int64_t views, batches, supersteps, launches;
  double ms_total;               /* wall ms inside the last rgpu_run_view_batch */
  /* per-kernel event timing (RGPU_RUN_PROFILE): 0=window_mask 1=slots 2=cc_step 3=cc_hist
   * 4=cc_summary 5=pr_step 6=degree 7=cc_tail (late supersteps, one workgroup)
   * 8=heavy (hub segment kernels) 9=diffusion step 10=vertex-program step
   * 11=edge_mask (K1's edge masks; 0 = its vertex masks) 12=xchg (partitioned mode: ghost membership
   * words and received counts) 13=xchg_pack (label records) 14=xchg_unpack (records into ghost words /
   * rows, the clear two steps later) 15=xchg_mark (owned neighbours of changed ghosts) (ABI 8) */
  int64_t kernel_launches[16];  /* (12 before ABI 8) */
  double kernel_ms[16];
  double kernel_bytes[16];       /* algorithmic bytes summed over launches */
  /* last rgpu_seal: wall ms, 1 if it merged a delta into the resident graph (live ingest),
   * and the number of updates that delta held (ABI 3) */
  double seal_ms;
  int64_t seal_incremental, seal_delta_updates;
  /* last run, RGPU_RUN_EDGE_COUNTS: sum over its views of |E_{t,w}| (else -1) (ABI 6) */
  int64_t alive_edge_windows;
  /* edge entities whose source vertex this partition owns: summed over the partitions, the
     graph's edge entities (`edges` counts every edge kept here, SplitEdge copies included) */
  int64_t edges_owned;
  /* last run, partitioned mode: bytes this partition sent to its peers, in all and by kind
     [0] ghost membership words [1] label records [2] component counts [3] PageRank rows */
  double xchg_bytes;
  double xchg_bytes_by[4];
} rgpu_stats_t;

int rgpu_abi_version(void);

/* One context per Partition Manager / GPU (Reader.scala:42-53 spawns one reader per PM). */
int rgpu_open(int partition_id, int num_partitions, int device, rgpu_ctx** out);

/* Append updates (any order).  Replaces the Router -> IngestionWorker -> EntityStorage
 * path for the analysis hot path; the final histories follow EntityStorage.scala:73-453. */
int rgpu_ingest(rgpu_ctx* ctx, const int64_t* t, const uint8_t* kind, const int64_t* src,
                const int64_t* dst, size_t n);

/* Binary GraphUpdate log ("RGEV") — the Router-side packer and the
 * partition-side decoder, replacing one Tracked*GraphUpdate actor message per update
 * (RouterWorker.sendGraphUpdate, S/core/components/Router/RouterWorker.scala:88-116; update
 * case classes raphtoryMessages.scala:38-55).  A log is a sequence of self-checking blocks
 * (little-endian):
 *    0 u32 magic 0x56454752 ("RGEV")   4 u16 version = 1   6 u16 flags = 0
 *    8 u32 n, 1..RGPU_RGEV_MAX_BLOCK  12 u32 checksum      16 i64 t_base (min time in block)
 *   24 u32 dt[n] (t - t_base) | u8 kind[n] zero-padded to a multiple of 4 | i32 src[n] | i32 dst[n]
 * checksum = lo32(a) ^ hi32(a) ^ lo32(b) ^ hi32(b) of a Fletcher-64 over the payload's u32
 * words (a += w; b += a, both mod 2^64).  Stream order is kept (ties resolve by it); vertex
 * updates carry dst = -1; 13 bytes per update + 24 per block.
 * rgpu_rgev_encode: pass out = NULL for the size (*written); blocks hold at most `block`
 *   updates (0 = RGPU_RGEV_MAX_BLOCK) and end early where the time span would pass 2^32 - 1.
 * rgpu_rgev_decode: expands every WHOLE block in buf (a trailing partial block is left:
 *   *consumed says how far it read, so a socket reader keeps the rest for the next call);
 *   pass t = NULL for the count (*n).  Any malformed block fails the call, nothing written.
 * rgpu_ingest_rgev: decode + rgpu_ingest in one call (same validation, same order).
 * The codec calls need no GPU and no ctx; their errors are in rgpu_rgev_last_error(). */
#define RGPU_RGEV_MAX_BLOCK (1u << 20)
int rgpu_rgev_encode(const int64_t* t, const uint8_t* kind, const int64_t* src, const int64_t* dst,
                     size_t n, size_t block, uint8_t* out, size_t cap, size_t* written);
int rgpu_rgev_decode(const uint8_t* buf, size_t bytes, int64_t* t, uint8_t* kind, int64_t* src,
                     int64_t* dst, size_t cap, size_t* n, size_t* consumed);
const char* rgpu_rgev_last_error(void);
int rgpu_ingest_rgev(rgpu_ctx* ctx, const uint8_t* buf, size_t bytes, size_t* consumed);

/* Sort + merge + pack the ingested stream into SoA histories and copy them to HBM.
 * Live ingest (IngestionWorker.scala:31-256 keeps appending while LiveAnalysisTask.scala:13-107
 * re-runs): after the first seal, rgpu_ingest + rgpu_seal again merges only the new updates
 * into the HBM-resident graph (merge.hip; one partition in RGPU_ORDER_ID order, RGPU_DELTA=0
 * forces a full re-pack).
 * The new updates count as later in stream order than every sealed one.
 * Concurrency (ABI 9, IngestionWorker keeps applying updates while LiveAnalysisTask runs):
 *   - rgpu_ingest may be called while a run or a seal is in progress; a seal packs the updates
 *     ingested before it started.  An ingest does not unseal the context: a run after an ingest
 *     without a seal analyses the resident graph (the updates since the last seal wait for the
 *     next one).
 *   - a delta seal builds the merged graph beside the resident one while runs go on.  If the last
 *     run's results are still readable (a run has happened on the resident graph), the merged graph
 *     is PARKED: rgpu_cc_*, rgpu_degree_*, rgpu_pr_* keep answering for the run they came from, and
 *     the next rgpu_run_view_batch (or rgpu_seal) swaps the parked graph in first.  rgpu_stats'
 *     entity counts (vertices, edges, *_events, deaths, seal_*) describe the newest sealed graph,
 *     i.e. the parked one while one is parked.
 *   - a full re-pack (first seal, RGPU_DELTA=0, a locality-ordered base) holds the run mutex
 *     throughout. */
int rgpu_seal(rgpu_ctx* ctx);

/* Local vertex order of the next full seal (ABI 7).  Results and labels do not depend on it.
 *   RGPU_ORDER_LOCALITY (default): vertices ranked by activity, hubs clustered in cache-line
 *     groups spread over the rank range: the superstep gathers hit L2 more often.
 *     A later rgpu_seal on such a context re-packs the whole stream.
 *   RGPU_ORDER_ID: ids ascending.  Needed by live ingest: a later rgpu_seal then merges only the
 *     new updates into the resident graph (IngestionWorker / LiveAnalysisTask contexts). */
#define RGPU_ORDER_LOCALITY 0
#define RGPU_ORDER_ID 1
int rgpu_set_vertex_order(rgpu_ctx* ctx, int order);

/* Newest ingested time: the watermark ReaderWorker.processTimeCheckRequest compares
 * against (ReaderWorker.scala:259-274). */
int rgpu_newest_time(rgpu_ctx* ctx, int64_t* out);

/* Multi-GPU vertex-partitioned mode.  A context opened with
 * num_partitions = P > 1 owns the vertices with Utils.getPartition(id, P) == partition_id
 * (S/core/utils/Utils.scala:32-33) plus ghost copies of their remote neighbours, as a
 * Partition Manager keeps SplitEdge copies (EntityStorage.scala:303-305).  Every partition
 * must be handed the WHOLE update stream (rgpu_ingest); each keeps what it needs.
 *
 * rgpu_exchange_id: make the id blob (RGPU_XCHG_ID_BYTES) once, on one rank, and hand it to
 *   every partition (RGPU_XCHG_RCCL: an ncclUniqueId — one process per GPU;
 *   RGPU_XCHG_LOOPBACK: partitions living in one process, e.g. to test on one GPU;
 *   RGPU_XCHG_SHM (ABI 9): one process per partition on one host, collectives staged through
 *   POSIX shared memory — processes sharing a GPU, or a host without an RCCL transport).
 * rgpu_exchange_init: join the group (collective over the P partitions; before the first
 *   run).  A no-op when num_partitions == 1.
 * A partitioned run is collective too: every partition calls rgpu_run_view_batch with the
 * same arguments.  Results: rgpu_cc_summary is the merged (all-partition) summary on every
 * partition; rgpu_cc_result / *_vertex_* / rgpu_pr_result / rgpu_degree_result cover this
 * partition's own vertices (the per-shard returnResults the caller merges). */
#define RGPU_XCHG_ID_BYTES 128
#define RGPU_XCHG_RCCL 0
#define RGPU_XCHG_LOOPBACK 1
#define RGPU_XCHG_SHM 2
int rgpu_exchange_id(int kind, uint8_t* out /* RGPU_XCHG_ID_BYTES */);
int rgpu_exchange_init(rgpu_ctx* ctx, const void* id /* RGPU_XCHG_ID_BYTES */);
/* rgpu_exchange_probe (ABI 10): the partitioned superstep's fixed cost on this context's channel,
 * measured — `rounds` repetitions of a round's collectives and host round trip besides its kernels
 * (the counts all-to-all, the counts' copy to the host and the host's wait, the two grouped
 * send/recv of the label records; AnalysisTask's per-superstep barrier, AnalysisTask.scala:208-225)
 * and of a 64-word all-reduce.  us[4] = round mean, round median, all-reduce mean, all-reduce median,
 * in microseconds.  Collective: every partition calls it with the same rounds. */
int rgpu_exchange_probe(rgpu_ctx* ctx, int rounds, double* us /* [4] */);

/* Run one analyser over every (hop, window) view: hops[n_hops] are the Range hop
 * timestamps (RangeAnalysisTask.restart, RangeAnalysisTask.scala:18-35), windows[n_w]
 * the user's batched window list in the user's order (n_w == 0 => ViewLens, no
 * window).  Replaces the Setup / NextStep* / Finish rounds that AnalysisTask drives
 * through ReaderWorker (AnalysisTask.scala:162-283, ReaderWorker.scala:159-257).
 * max_steps: Analyser.defineMaxSteps (CC = 100).  pr_iters: PageRank iterations. */
int rgpu_run_view_batch(rgpu_ctx* ctx, int algo, const int64_t* hops, size_t n_hops,
                        const int64_t* windows, size_t n_w, int max_steps, int pr_iters,
                        int flags);

/* CC summary of view (hop, win) of the last run (ConnectedComponents.scala:137-145). */
int rgpu_cc_summary(rgpu_ctx* ctx, size_t hop, size_t win, rgpu_cc_summary_t* out);

/* CC label -> count map of view (hop, win): ConnectedComponents.returnResults
 * (ConnectedComponents.scala:37-42) merged over the partition.  Needs RGPU_RUN_RETAIN. */
int rgpu_cc_result(rgpu_ctx* ctx, size_t hop, size_t win, int64_t* labels, int32_t* counts,
                   size_t cap, size_t* n);

/* Per-vertex CC labels of view (hop, win), ascending id.  Needs RGPU_RUN_RETAIN. */
int rgpu_cc_vertex_labels(rgpu_ctx* ctx, size_t hop, size_t win, int64_t* ids, int64_t* labels,
                          size_t cap, size_t* n);

/* DegreeBasic.returnResults (DegreeBasic.scala:16-28): tot = {totalV, totalOut, totalIn};
 * top-20 by in-degree (ties by ascending id), computed on the device in every degree run
 * (no RGPU_RUN_RETAIN needed); slots past the view's vertex count hold id -1 and zero degrees.
 * top_id/top_out/top_in may all be NULL to skip the list. */
int rgpu_degree_result(rgpu_ctx* ctx, size_t hop, size_t win, int64_t tot[3], int64_t* top_id,
                       int32_t* top_out, int32_t* top_in);

/* Per-vertex degrees of view (hop, win), ascending id.  Needs RGPU_RUN_RETAIN. */
int rgpu_degree_vertex(rgpu_ctx* ctx, size_t hop, size_t win, int64_t* ids, int32_t* outdeg,
                       int32_t* indeg, size_t cap, size_t* n);

/* PageRank of view (hop, win), ascending id.  Needs RGPU_RUN_RETAIN. */
int rgpu_pr_result(rgpu_ctx* ctx, size_t hop, size_t win, int64_t* ids, double* pr, size_t cap,
                   size_t* n);

/* BinaryDefusion (BinaryDefusion.scala:9-51; VertexVisitor messaging, VertexVisitor.scala:99-135)
 * parameters for later RGPU_ALGO_DIFFUSION runs: seed_id = infectedNode (:10, default 31).
 * The reference flips Random.nextBoolean() per message (:17,:32), unseeded and so not
 * reproducible; here the flip is a fixed hash (coin = 1, the default; coin = 0 sends every
 * message, the deterministic taint/reachability form).  With mix = the splitmix64 finaliser
 * (x ^= x>>30; x *= 0xbf58476d1ce4e5b9; x ^= x>>27; x *= 0x94d049bb133111eb; x ^= x>>31), u64
 * wrap-around arithmetic and w = the view's window (-1 for a ViewLens):
 *   salt(t, w)         = mix(coin_seed ^ mix((u64)t ^ mix((u64)w)))
 *   heads(u, v, r, t, w) = top bit of mix(salt(t, w) ^ mix((u64)u * 0x9E3779B97F4A7C15 ^ mix((u64)v + r)))
 * for a message from vertex id u to vertex id v sent at superstep r (setup = 0).
 * Diffusion runs need one partition (num_partitions == 1) and max_steps <= 127. */
int rgpu_set_diffusion(rgpu_ctx* ctx, int64_t seed_id, uint64_t coin_seed, int coin);

/* Diffusion result of view (hop, win): infected vertices and the supersteps its batch ran. */
int rgpu_diffusion_result(rgpu_ctx* ctx, size_t hop, size_t win, int64_t* infected, int64_t* supersteps);

/* BinaryDefusion.returnResults (:38-49): (id, infected superstep) of every infected vertex of
 * the view, ascending id.  Needs RGPU_RUN_RETAIN. */
int rgpu_diffusion_vertex(rgpu_ctx* ctx, size_t hop, size_t win, int64_t* ids, int32_t* steps,
                          size_t cap, size_t* n);

/* Generic VertexVisitor messaging (ABI 7; VertexVisitor.scala:81-166): a
 * user Analyser whose analyse() folds its message queue with min or max runs on the GPU as a
 * vertex program, with the reference's BSP structure (AnalysisTask / ReaderWorker):
 *   setup (superstep 0, only when maxSteps > 1): every view member sets its state
 *     (getOrSetCompValue) to its own id (RGPU_VP_INIT_ID) or init_value (seed_value at the vertex
 *     seed_id; RGPU_VP_INIT_VALUE); the senders — every member, or only the seed — message their
 *     neighbours in `direction` (messageAllOutgoingNeighbors / messageAllIngoingNeighbors /
 *     messageAllNeighbours, over edges alive in the view) the value state + step_add (saturating);
 *   superstep r >= 1: a member holding messages folds them and its state with `reduce`; if that
 *     changes its state it keeps it and messages again, else it votes to halt;
 *   the job halts at the first superstep in which no state changed in any window of the hop, or
 *     at maxSteps.
 * CC = {ALL, MIN, INIT_ID, SEND_ALL, step_add 0}; hop distance from a seed over out-edges = {OUT,
 * MIN, INIT_VALUE init_value INT64_MAX seed_value 0, SEND_SEED, step_add 1}.  max_steps <= 127.
 * Partitioned contexts (ABI 10) run it too: after setup and every superstep each partition sends
 * its peers the states of its changed boundary vertices (the messages that cross partitions, as
 * the mediator carries VertexMessage between PMs), and the halt vote is global (an all-reduce).
 * Oracle: oracle.h orc_vertex_program. */
#define RGPU_VP_OUT 0
#define RGPU_VP_IN 1
#define RGPU_VP_ALL 2
#define RGPU_VP_MIN 0
#define RGPU_VP_MAX 1
#define RGPU_VP_INIT_ID 0
#define RGPU_VP_INIT_VALUE 1
#define RGPU_VP_SEND_ALL 0
#define RGPU_VP_SEND_SEED 1
typedef struct {
  int32_t direction, reduce, init, senders;
  int64_t init_value, seed_id, seed_value, step_add;
} rgpu_vertex_program_t;
int rgpu_set_vertex_program(rgpu_ctx* ctx, const rgpu_vertex_program_t* program);
/* every member's final state of view (hop, win), ascending id (needs RGPU_RUN_RETAIN) */
int rgpu_vp_result(rgpu_ctx* ctx, size_t hop, size_t win, int64_t* ids, int64_t* values, size_t cap, size_t* n);
/* supersteps the reference's job for that hop runs (as rgpu_cc_summary_t.supersteps) */
int rgpu_vp_supersteps(rgpu_ctx* ctx, size_t hop, int64_t* supersteps);

/* Float vertex programs (ABI 10): VertexMessageFloat (raphtoryMessages.scala:117; messageNeighbour /
 * messageAllOutgoingNeighbors(Float) / messageAllIngoingNeighbors(Float), VertexVisitor.scala:
 * 137-147) folded by summation — the message shape of the reference's float analyser
 * (examples/random/depricated/PageRank.scala:20-37, whose queue loop is commented out there).
 *   setup (superstep 0, maxSteps > 1): every member's state = (float) its id (RGPU_VP_INIT_ID) or
 *     init_value (seed_value at seed_id); the senders (every member, or the seed) message their
 *     neighbours in `direction` (OUT or IN) the value state, or with per_degree (float)(state /
 *     max(deg, 1)) — deg = its message targets over edges alive in the view (getOutgoingNeighbors.size
 *     for OUT, self-loop included; in-edges without the self-loop for IN);
 *   superstep r >= 1: a member holding messages sets state = (float)(bias + mult * sum), the sum in
 *     double precision, and messages again (it never votes to halt); the others keep their state;
 *   the job halts when no member received a message in some superstep, or at maxSteps.
 * Floats are IEEE binary32 values carried as doubles.  The reference sums its Float queue in
 * message-arrival order (nondeterministic across actors), so parity is stated within float32
 * rounding: per member |gpu - oracle| <= 1e-6 * max(1, |oracle|) (oracle.h orc_vertex_program_f).
 * RGPU_ALGO_VP runs it, on one partition or partitioned (as above; with per_degree the ghosts'
 * out/in degrees in the view are exchanged once per batch); rgpu_vp_result_f reads the states
 * (rgpu_vp_result returns their double bit patterns). */
typedef struct {
  int32_t direction, init, senders, per_degree;
  int64_t seed_id;
  double init_value, seed_value, bias, mult;
} rgpu_vertex_program_f_t;
int rgpu_set_vertex_program_f(rgpu_ctx* ctx, const rgpu_vertex_program_f_t* program);
int rgpu_vp_result_f(rgpu_ctx* ctx, size_t hop, size_t win, int64_t* ids, double* values, size_t cap, size_t* n);

int rgpu_stats(rgpu_ctx* ctx, rgpu_stats_t* out);
const char* rgpu_last_error(rgpu_ctx* ctx);
void rgpu_close(rgpu_ctx* ctx);

#ifdef __cplusplus
}
#endif
#endif
