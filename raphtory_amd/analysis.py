"""Host-side mirror of Raphtory's analysis plugin surface for the GPU path.

S/ = mainproject/cluster/src/main/scala/com/raphtory/ in the reference.

* ``Analyser`` subclasses keep the reference names and result shapes:
  ``ConnectedComponents`` (S/core/analysis/Algorithms/ConnectedComponents.scala),
  ``DegreeBasic`` (Algorithms/DegreeBasic.scala), ``PageRank`` (SURVEY.md App. A.5 spec; the
  reference examples/random/depricated/PageRank.scala is broken).  ``returnResults`` gives the
  merged per-partition result (label->count map / degree tuple) and the ``process*Results``
  methods format the reference's output lines.
* ``*AnalysisTask`` classes mirror S/core/analysis/Tasks/** : the job kinds spawned by
  AnalysisManager (AnalysisManager.scala:133-167) for windowType "false"/"true"/"batched".
  Where the reference runs Setup/NextStep*/Finish per hop through ten ReaderWorkers, one
  ``TemporalGraph.run`` call evaluates every hop x window on the GPU.
"""
from __future__ import annotations

import json
import threading
import time
from typing import Dict, List, Optional, Sequence

import numpy as np

from .graph import TemporalGraph
from .jfloat import double_to_string, float_to_string
from .synth import range_hops


# ---------------------------------------------------------------- JVM number printing
def java_float_str(x, double: bool = False) -> str:
    """Float.toString / Double.toString as the reference's JDK 12 prints them: the FloatingDecimal
    digit generation restated in jfloat.py (not always the shortest round-trip string)."""
    return double_to_string(float(x)) if double else float_to_string(float(np.float32(x)))


# ---------------------------------------------------------------- analysers
class Analyser:
    """S/core/analysis/API/Analyser.scala:30-63"""
    algo = ""

    def __init__(self, args: Sequence[str] = ()):
        self.args = list(args)
        self.lines: List[str] = []

    def defineMaxSteps(self) -> int:  # noqa: N802 (reference names)
        raise NotImplementedError

    def returnResults(self, graph: TemporalGraph, hop: int, win: int):  # noqa: N802
        raise NotImplementedError

    def processResults(self, results, timestamp, viewCompleteTime):  # noqa: N802
        raise NotImplementedError

    def processViewResults(self, results, timestamp, viewCompleteTime):  # noqa: N802
        self.processResults(results, timestamp, viewCompleteTime)

    def processWindowResults(self, results, timestamp, windowSize, viewCompleteTime):  # noqa: N802
        self.processResults(results, timestamp, viewCompleteTime)

    def processBatchWindowResults(self, results, timestamp, windowSet, viewCompleteTime):  # noqa: N802
        self.processResults(results, timestamp, viewCompleteTime)


def cc_fields(grouped: Dict[int, int]) -> Optional[dict]:
    """ConnectedComponents.processBatchWindowResults summary (ConnectedComponents.scala:137-145);
    None for an empty view (maxBy throws UnsupportedOperationException -> "No activity")."""
    if not grouped:
        return None
    counts = np.fromiter(grouped.values(), np.int64)
    non_isl = counts[counts > 1]
    biggest = int(counts.max())
    return {
        "biggest": biggest,
        "total": int(counts.size),
        "totalWithoutIslands": int(non_isl.size),
        "totalIslands": int(counts.size - non_isl.size),
        "proportion": np.float32(biggest) / np.float32(int(counts.sum())),
        "proportionWithoutIslands": (np.float32(biggest) / np.float32(int(non_isl.sum()))
                                     if non_isl.size else np.float32(np.inf)),
        "clustersGT2": int((counts > 2).sum()),
    }


def cc_fields_from_summary(s) -> Optional[dict]:
    """Same fields from the GPU-side summary (rgpu_cc_summary_t), no label map needed."""
    if s.total == 0:
        return None
    return {
        "biggest": int(s.biggest),
        "total": int(s.total),
        "totalWithoutIslands": int(s.total_without_islands),
        "totalIslands": int(s.total_islands),
        "proportion": np.float32(s.biggest) / np.float32(s.sum_all),
        "proportionWithoutIslands": (np.float32(s.biggest) / np.float32(s.sum_without_islands)
                                     if s.sum_without_islands else np.float32(np.inf)),
        "clustersGT2": int(s.clusters_gt2),
    }


class ConnectedComponents(Analyser):
    """S/core/analysis/Algorithms/ConnectedComponents.scala:8-162"""
    algo = "cc"

    def defineMaxSteps(self) -> int:  # :160
        return 100

    def returnResults(self, graph, hop, win):  # :37-42 (merged over the partition)
        return graph.cc_result(hop, win)

    @staticmethod
    def _line(timestamp, window, f, view_ms) -> str:
        head = f'{{"time":{timestamp},' + (f'"windowsize":{window},' if window is not None else "")
        return (head + f'"biggest":{f["biggest"]},"total":{f["total"]},'
                f'"totalWithoutIslands":{f["totalWithoutIslands"]},"totalIslands":{f["totalIslands"]},'
                f'"proportion":{java_float_str(f["proportion"])},'
                f'"proportionWithoutIslands":{java_float_str(f["proportionWithoutIslands"])},'
                f'"clustersGT2":{f["clustersGT2"]},"viewTime":{view_ms},"concatTime":0}},')

    def _emit(self, fields, timestamp, window, view_ms):
        if fields is None:
            where = f"view at {timestamp}" + (f" with window {window}" if window is not None else "")
            self.lines.append(f"No activity for  {where}")  # :65/:89/:119/:154
        else:
            self.lines.append(self._line(timestamp, window, fields, view_ms))

    def processResults(self, results, timestamp, viewCompleteTime):  # :44-67
        merged: Dict[int, int] = {}
        for part in results:
            for k, v in part.items():
                merged[k] = merged.get(k, 0) + v
        self._emit(cc_fields(merged), timestamp, None, viewCompleteTime)

    def processWindowResults(self, results, timestamp, windowSize, viewCompleteTime):  # :93-122
        merged: Dict[int, int] = {}
        for part in results:
            for k, v in part.items():
                merged[k] = merged.get(k, 0) + v
        self._emit(cc_fields(merged), timestamp, windowSize, viewCompleteTime)

    def processBatchWindowResults(self, results, timestamp, windowSet, viewCompleteTime):  # :124-158
        for i, window in enumerate(results):
            merged: Dict[int, int] = {}
            for part in window:
                for k, v in part.items():
                    merged[k] = merged.get(k, 0) + v
            self._emit(cc_fields(merged), timestamp, windowSet[i], viewCompleteTime)


class DegreeBasic(Analyser):
    """S/core/analysis/Algorithms/DegreeBasic.scala:8-79"""
    algo = "degree"

    def defineMaxSteps(self) -> int:  # :30
        return 1

    def returnResults(self, graph, hop, win):  # :16-28 -> (totalV, totalOut, totalIn, top20)
        return graph.degree_result(hop, win)

    @staticmethod
    def _degree(results):
        tv = sum(r[0] for r in results)
        te = sum(r[2] for r in results)
        deg = (te / tv) if tv else float("nan")  # Int/Int as Double: 0.0/0.0 = NaN
        return tv, te, deg

    def processResults(self, results, timestamp, viewCompleteTime):  # :32-46
        tv, te, deg = self._degree(results)
        self.lines.append(f"{timestamp},{tv},{te},{java_float_str(deg, double=True)}")

    def processWindowResults(self, results, timestamp, windowSize, viewCompleteTime):  # :48-66
        tv, te, deg = self._degree(results)
        self.lines.append(f"{timestamp},{windowSize},{tv},{te},{java_float_str(deg, double=True)}")

    def processBatchWindowResults(self, results, timestamp, windowSet, viewCompleteTime):  # :68-78
        for i, window in enumerate(results):
            self.processWindowResults(window, timestamp, windowSet[i], viewCompleteTime)


class DegreeRanking(Analyser):
    """S/core/analysis/Algorithms/DegreeRanking.scala:8-124.  Per shard (totalV, totalOut, totalIn,
    top 20 by in-degree); the lines merge the shards' top lists and keep the best 20 by in-degree
    ("bestusers").  The top list is computed on the GPU for every view (k_deg_top_merge); ties go
    by ascending id (the reference's order under ties is ParTrieMap's, unordered)."""
    algo = "degree"

    def defineMaxSteps(self) -> int:  # :30
        return 1

    def returnResults(self, graph, hop, win):  # :14-26
        return graph.degree_result(hop, win)

    @staticmethod
    def _body(results) -> str:
        tv = sum(r[0] for r in results)
        te = sum(r[2] for r in results)
        deg = (te / tv) if tv else float("nan")  # Int.toDouble / Int.toDouble: 0.0/0.0 = NaN
        top = sorted((u for r in results for u in r[3]), key=lambda u: (-u[2], u[0]))[:20]  # sortBy(_._3) desc
        best = "[" + ",".join(f'{{"id":{i},"indegree":{d_in},"outdegree":{d_out}}}' for i, d_out, d_in in top) + "]"
        return f'"vertices":{tv},"edges":{te},"degree":{java_float_str(deg, double=True)},"bestusers":{best}'

    def processResults(self, results, timestamp, viewCompleteTime):  # :32-55
        self.lines.append(f'{{"time":{timestamp},{self._body(results)},"viewTime":{viewCompleteTime},"concatTime":0}},')

    def processViewResults(self, results, timestamp, viewCompleteTime):  # :57-80
        self.processResults(results, timestamp, viewCompleteTime)

    def processWindowResults(self, results, timestamp, windowSize, viewCompleteTime):  # :82-111
        self.lines.append(f'{{"time":{timestamp},"windowsize":{windowSize},{self._body(results)},'
                          f'"viewTime":{viewCompleteTime},"concatTime":0}},')

    def processBatchWindowResults(self, results, timestamp, windowSet, viewCompleteTime):  # :113-123
        for i, window in enumerate(results):
            self.processWindowResults(window, timestamp, windowSet[i], viewCompleteTime)


class PageRank(Analyser):
    """PageRank as specified in SURVEY.md App. A.5 (constants of
    examples/random/depricated/PageRank.scala:11-45; 20 iterations per BASELINE config C3)."""
    algo = "pagerank"

    def __init__(self, args: Sequence[str] = (), iterations: int = 20):
        super().__init__(args)
        self.iterations = iterations

    def defineMaxSteps(self) -> int:
        return self.iterations

    def returnResults(self, graph, hop, win):
        ids, pr = graph.pr_result(hop, win)
        return dict(zip(ids.tolist(), pr.tolist()))

    def processResults(self, results, timestamp, viewCompleteTime):
        merged: Dict[int, float] = {}
        for part in results:
            merged.update(part)
        top = sorted(merged.items(), key=lambda kv: (-kv[1], kv[0]))[:5]
        self.lines.append(json.dumps({"time": timestamp, "top5": top, "vertices": len(merged)}))


class BinaryDefusion(Analyser):
    """S/core/analysis/Algorithms/BinaryDefusion.scala:9-60 on the GPU (raphtory_amd/csrc/diffusion.hip).

    The reference's per-message ``Random.nextBoolean()`` (:17, :32) is unseeded; here it is the
    hash coin of ``include/rgpu.h`` (``coin_seed``), or no coin at all (``coin=False``: every
    message is sent, the taint/reachability form).  ``processResults`` is ``???`` in the
    reference (:53); views print the infected (id, superstep) list and its size (:55-59)."""
    algo = "diffusion"

    def __init__(self, args: Sequence[str] = (), infected_node: int = 31, coin_seed: int = 0, coin: bool = True):
        super().__init__(args)
        self.infectedNode = infected_node  # :10
        self.coin_seed = coin_seed
        self.coin = coin

    def defineMaxSteps(self) -> int:  # :51
        return 100

    def prepare(self, graph) -> None:
        graph.set_diffusion(self.infectedNode, self.coin_seed, self.coin)

    def returnResults(self, graph, hop, win):  # :38-49
        ids, steps = graph.diffusion_vertex(hop, win)
        return list(zip(ids.tolist(), steps.tolist()))

    def processViewResults(self, results, timestamp, viewCompleteTime):  # :55-59
        end = sorted(x for part in results for x in part)
        self.lines.append(json.dumps({"time": timestamp, "infected": end, "size": len(end)}))

    def processResults(self, results, timestamp, viewCompleteTime):
        # deliberate extension: the reference's is ``???`` (:53, NotImplementedError), so a
        # non-batched Range job of it throws there; here it prints the view line instead
        self.processViewResults(results, timestamp, viewCompleteTime)

    def processBatchWindowResults(self, results, timestamp, windowSet, viewCompleteTime):
        for w, per_window in zip(windowSet, results):
            end = sorted(x for part in per_window for x in part)
            self.lines.append(json.dumps({"time": timestamp, "windowsize": w, "infected": end, "size": len(end)}))


class VertexProgram(Analyser):
    """A user Analyser written against the VertexVisitor messaging surface (VertexVisitor.scala:
    81-166) whose analyse() folds its message queue with min or max — run on the GPU as a vertex
    program (include/rgpu.h rgpu_set_vertex_program, raphtory_amd/csrc/vp.hip):

        setup():   setCompValue(key, init); if sender: messageAll<direction>(state + step_add)
        analyse(): m = fold(messageQueue); if fold(state, m) != state: setCompValue(key, that);
                   messageAll<direction>(that + step_add) else voteToHalt()

    ``returnResults`` gives {id: state} for the view's members; the lines list the members whose
    state differs from ``init_value`` (or every member for init="id")."""
    algo = "vp"

    def __init__(self, args: Sequence[str] = (), direction: str = "all", reduce: str = "min", init: str = "id",
                 senders: str = "all", init_value: int = 0, seed_id: int = -1, seed_value: int = 0,
                 step_add: int = 0, max_steps: int = 100):
        super().__init__(args)
        self.program = dict(direction=direction, reduce=reduce, init=init, senders=senders, init_value=init_value,
                            seed_id=seed_id, seed_value=seed_value, step_add=step_add)
        self.max_steps = max_steps

    def defineMaxSteps(self) -> int:  # noqa: N802
        return self.max_steps

    def prepare(self, graph) -> None:
        graph.set_vertex_program(**self.program)

    def returnResults(self, graph, hop, win):  # noqa: N802
        ids, vals = graph.vp_result(hop, win)
        return dict(zip(ids.tolist(), vals.tolist()))

    def _line(self, results, timestamp, window=None) -> str:
        merged: Dict[int, int] = {}
        for part in results:
            merged.update(part)
        keep = merged if self.program["init"] == "id" else \
            {k: v for k, v in merged.items() if v != self.program["init_value"]}
        d = {"time": timestamp}
        if window is not None:
            d["windowsize"] = window
        d.update({"vertices": len(merged), "reached": len(keep), "states": sorted(keep.items())})
        return json.dumps(d)

    def processResults(self, results, timestamp, viewCompleteTime):  # noqa: N802
        self.lines.append(self._line(results, timestamp))

    def processWindowResults(self, results, timestamp, windowSize, viewCompleteTime):  # noqa: N802
        self.lines.append(self._line(results, timestamp, windowSize))

    def processBatchWindowResults(self, results, timestamp, windowSet, viewCompleteTime):  # noqa: N802
        for i, window in enumerate(results):
            self.lines.append(self._line(window, timestamp, windowSet[i]))


class HopDistance(VertexProgram):
    """Out-edge hop distance from a seed vertex (a taint / reachability analyser, as the
    reference's example BinaryDefusion spreads from infectedNode, without its coin)."""

    def __init__(self, args: Sequence[str] = (), seed_id: int = 31, direction: str = "out", max_steps: int = 100):
        super().__init__(args, direction=direction, reduce="min", init="value", senders="seed",
                         init_value=2**63 - 1, seed_id=seed_id, seed_value=0, step_add=1, max_steps=max_steps)


class FloatVertexProgram(Analyser):
    """A user Analyser that sends Float messages (VertexMessageFloat, VertexVisitor.scala:137-147)
    and sums its queue — run on the GPU as a float vertex program (include/rgpu.h
    rgpu_set_vertex_program_f):

        setup():   setCompValue(key, init); if sender: messageAll<direction>(state [/ degree])
        analyse(): if moreMessages: state = bias + mult * sum(queue); setCompValue(key, state);
                   messageAll<direction>(state [/ degree])

    ``returnResults`` gives {id: state}; the lines print the top five states per view as the
    reference's float analyser's processResults does (examples/random/depricated/PageRank.scala:
    45-50), with Float.toString."""
    algo = "vp"

    def __init__(self, args: Sequence[str] = (), direction: str = "out", init: str = "id", senders: str = "all",
                 per_degree: bool = False, seed_id: int = -1, init_value: float = 0.0, seed_value: float = 0.0,
                 bias: float = 0.0, mult: float = 1.0, max_steps: int = 100):
        super().__init__(args)
        self.program = dict(direction=direction, init=init, senders=senders, per_degree=per_degree, seed_id=seed_id,
                            init_value=init_value, seed_value=seed_value, bias=bias, mult=mult)
        self.max_steps = max_steps

    def defineMaxSteps(self) -> int:  # noqa: N802
        return self.max_steps

    def prepare(self, graph) -> None:
        graph.set_vertex_program_f(**self.program)

    def returnResults(self, graph, hop, win):  # noqa: N802
        ids, vals = graph.vp_result_f(hop, win)
        return dict(zip(ids.tolist(), vals.tolist()))

    def _line(self, results, timestamp, window=None) -> str:
        merged: Dict[int, float] = {}
        for part in results:
            merged.update(part)
        top = sorted(merged.items(), key=lambda kv: (-kv[1], kv[0]))[:5]
        d = "{" + f'"time":{timestamp},' + (f'"windowsize":{window},' if window is not None else "")
        return d + '"top5":[' + ",".join(f"[{k},{java_float_str(v)}]" for k, v in top) + "]}"

    def processResults(self, results, timestamp, viewCompleteTime):  # noqa: N802
        self.lines.append(self._line(results, timestamp))

    def processWindowResults(self, results, timestamp, windowSize, viewCompleteTime):  # noqa: N802
        self.lines.append(self._line(results, timestamp, windowSize))

    def processBatchWindowResults(self, results, timestamp, windowSet, viewCompleteTime):  # noqa: N802
        for i, window in enumerate(results):
            self.lines.append(self._line(window, timestamp, windowSet[i]))


class FloatPageRank(FloatVertexProgram):
    """The PageRank its fields declare (examples/random/depricated/PageRank.scala:11-14: defaultPR 1f,
    dumplingFactor 0.85f, defineMaxSteps 10) as a float vertex program: a sender sends PR / its
    out-degree in the view, a receiver takes 0.15 + 0.85 * sum.  The reference's own analyse() is a
    stub (its queue loop is commented out, so every PR becomes 0 / outdegree), which this does not
    reproduce; the fp64 PageRank of SURVEY App. A.5 is RGPU_ALGO_PR."""

    def __init__(self, args: Sequence[str] = (), max_steps: int = 10):
        super().__init__(args, direction="out", init="value", per_degree=True, init_value=1.0, bias=0.15, mult=0.85,
                         max_steps=max_steps)


# ---------------------------------------------------------------- tasks
class TimeNotIngested(RuntimeError):
    """TimeCheck failed (ReaderWorker.processTimeCheckRequest :259-274); the reference retries in 10 s."""


class AnalysisTask:
    """S/core/analysis/Tasks/AnalysisTask.scala — here one GPU call per job."""

    def __init__(self, graphs: Sequence[TemporalGraph], analyser: Analyser, retain_results: bool = True):
        self.graphs = list(graphs)
        self.analyser = analyser
        self.retain = retain_results
        self.view_ms = 0.0

    # overridden by the subclasses
    def hops(self) -> np.ndarray:
        raise NotImplementedError

    def windowSet(self) -> List[int]:  # noqa: N802
        return []

    def windowSize(self) -> int:  # noqa: N802
        return -1

    def _windows(self) -> List[int]:
        ws = self.windowSet()
        if ws:
            return list(ws)
        return [self.windowSize()] if self.windowSize() != -1 else []

    def time_check(self, hops: np.ndarray) -> None:
        newest = min(g.newest_time() for g in self.graphs)
        if hops.size and int(hops.max()) > newest:
            raise TimeNotIngested(f"{int(hops.max())} is yet to be ingested, currently at {newest}")

    def run(self) -> List[str]:
        hops = self.hops()
        self.time_check(hops)
        windows = self._windows()
        a = self.analyser
        max_steps = a.defineMaxSteps()
        t0 = time.perf_counter()
        _run_all(self.graphs, a, hops, windows, max_steps, self.retain)
        self.view_ms = (time.perf_counter() - t0) * 1e3 / max(1, len(hops))
        vt = int(round(self.view_ms))
        for h, t in enumerate(hops.tolist()):
            if self.windowSet():
                # BWindowed*AnalysisTask.result: [worker][window] -> [window][worker]
                results = [[g_res for g_res in (a.returnResults(g, h, w) for g in self.graphs)]
                           for w in range(len(windows))]
                a.processBatchWindowResults(results, t, windows, vt)
            elif windows:
                a.processWindowResults([a.returnResults(g, h, 0) for g in self.graphs], t, windows[0], vt)
            else:
                a.processViewResults([a.returnResults(g, h, 0) for g in self.graphs], t, vt)
        return a.lines


class ViewAnalysisTask(AnalysisTask):
    def __init__(self, graphs, analyser, timestamp: int, **kw):
        super().__init__(graphs, analyser, **kw)
        self.timestamp = timestamp

    def hops(self):
        return np.asarray([self.timestamp], np.int64)


class WindowedViewAnalysisTask(ViewAnalysisTask):
    def __init__(self, graphs, analyser, timestamp: int, window: int, **kw):
        super().__init__(graphs, analyser, timestamp, **kw)
        self.window = window

    def windowSize(self):  # noqa: N802
        return self.window


class BWindowedViewAnalysisTask(ViewAnalysisTask):
    def __init__(self, graphs, analyser, timestamp: int, windows: Sequence[int], **kw):
        super().__init__(graphs, analyser, timestamp, **kw)
        self.windows = list(windows)

    def windowSet(self):  # noqa: N802
        return self.windows


class RangeAnalysisTask(AnalysisTask):
    """RangeTasks/RangeAnalysisTask.scala:12-39 (restart :18-35)"""

    def __init__(self, graphs, analyser, start: int, end: int, jump: int, **kw):
        super().__init__(graphs, analyser, **kw)
        self.start, self.end, self.jump = start, end, jump

    def hops(self):
        return range_hops(self.start, self.end, self.jump)


class WindowedRangeAnalysisTask(RangeAnalysisTask):
    def __init__(self, graphs, analyser, start, end, jump, window: int, **kw):
        super().__init__(graphs, analyser, start, end, jump, **kw)
        self.window = window

    def windowSize(self):  # noqa: N802
        return self.window


class BWindowedRangeAnalysisTask(RangeAnalysisTask):
    def __init__(self, graphs, analyser, start, end, jump, windows: Sequence[int], **kw):
        super().__init__(graphs, analyser, start, end, jump, **kw)
        self.windows = list(windows)

    def windowSet(self):  # noqa: N802
        return self.windows


def _run_all(graphs, a, hops, windows, max_steps, retain) -> None:
    """One job on every partition.  Runs are collective in partitioned mode (the partitions
    exchange per superstep), so with several partitions in this process each runs on its own
    thread, as the reference's Readers run concurrently."""
    def one(g):
        if hasattr(a, "prepare"):
            a.prepare(g)
        g.run(a.algo, hops, windows, max_steps=max_steps if a.algo in ("cc", "diffusion", "vp") else 100,
              pr_iters=max_steps if a.algo == "pagerank" else 0, retain=retain)
    if len(graphs) == 1:
        one(graphs[0])
        return
    errs = []

    def body(g):
        try:
            one(g)
        except BaseException as e:  # noqa: BLE001 - re-raised below
            errs.append(e)
    th = [threading.Thread(target=body, args=(g,)) for g in graphs]
    for t in th:
        t.start()
    for t in th:
        t.join()
    if errs:
        raise errs[0]


# ---------------------------------------------------------------- live tasks
class LiveAnalysisTask(AnalysisTask):
    """S/core/analysis/Tasks/LiveTasks/LiveAnalysisTask.scala:13-107.  One ``tick()`` is one job of
    the repeating live task: its time check (TimeCheck to every partition, ReaderWorker.
    processTimeCheckRequest :259-274: ok iff timestamp <= the partition's newest time) and, when
    every partition is ok, the view at ``timestamp()`` — ``liveTime`` = the minimum newest time
    over the partitions (setLiveTime :20-27).  The first job runs at that minimum; then
    (``restart`` :33-48, ``restartTime`` :29-31):
      * event time: the next timestamp is liveTime + repeatTime, where liveTime is the minimum
        taken at the previous successful check — the job waits until every partition has
        ingested that far;
      * processing time: after repeatTime ms the job runs at the then-current minimum.
    A failed check returns None (the reference re-checks after 1 s, :96-100).  The job runs an
    un-windowed view and prints processResults lines (AnalysisTask.processResults :82)."""

    def __init__(self, graphs, analyser, repeat_time: int, event_time: bool, **kw):
        super().__init__(graphs, analyser, **kw)
        self.repeat_time = int(repeat_time)
        self.event_time = bool(event_time)
        self.current_timestamp = 1  # :15
        self.live_time = 0
        self.first_time = True
        self.last_job_time = None   # the timestamp of the last job that ran
        self._pending = False       # a restart happened: the next tick checks the new timestamp

    def timestamp(self) -> int:
        return self.current_timestamp

    def hops(self):
        return np.asarray([self.current_timestamp], np.int64)

    def _set_live_time(self, newest: List[int]) -> None:  # :20-27
        self.live_time = min(newest)
        if not self.event_time or self.first_time:
            self.first_time = False
            self.current_timestamp = self.live_time

    def restart(self) -> None:  # :33-48
        if self.repeat_time > 0:
            self.current_timestamp = (self.live_time + self.repeat_time) if self.event_time else self.live_time
            self._pending = True

    def tick(self) -> Optional[List[str]]:
        """One live job: None if some partition has not ingested timestamp() yet, else the lines
        the job printed (then the task restarts for the next job, if repeatTime > 0)."""
        if not self.first_time and not self._pending:
            return []  # repeatTime <= 0: the task ran once and stopped
        newest = [g.newest_time() for g in self.graphs]
        if any(self.current_timestamp > n for n in newest):  # TimeResponse(ok = false)
            return None
        self._set_live_time(newest)
        self._pending = False
        a = self.analyser
        n0 = len(a.lines)
        ts = self.current_timestamp
        max_steps = a.defineMaxSteps()
        t0 = time.perf_counter()
        _run_all(self.graphs, a, [ts], [], max_steps, self.retain)
        self.last_job_time = ts
        vt = int(round((time.perf_counter() - t0) * 1e3))
        a.processResults([a.returnResults(g, 0, 0) for g in self.graphs], ts, vt)
        self.restart()
        return a.lines[n0:]

    def run(self) -> List[str]:
        out = self.tick()
        if out is None:
            raise TimeNotIngested(f"{self.current_timestamp} is yet to be ingested")
        return out


class WindowedLiveAnalysisTask(LiveAnalysisTask):
    """LiveTasks/WindowedLiveAnalysisTask.scala:7-10: takes a window but never overrides
    windowSize(), so the job runs un-windowed (reproduced)."""

    def __init__(self, graphs, analyser, repeat_time, event_time, window: int, **kw):
        super().__init__(graphs, analyser, repeat_time, event_time, **kw)
        self.window = window  # unused, as in the reference


class BWindowedLiveAnalysisTask(LiveAnalysisTask):
    """LiveTasks/BWindowedLiveAnalysisTask.scala:9-26: takes a window set but never overrides
    windowSet(); its result() inversion is never called (processResults reads the raw results,
    AnalysisTask.scala:82), so the job is the un-windowed one."""

    def __init__(self, graphs, analyser, repeat_time, event_time, windows: Sequence[int], **kw):
        super().__init__(graphs, analyser, repeat_time, event_time, **kw)
        self.windows = list(windows)  # unused, as in the reference
