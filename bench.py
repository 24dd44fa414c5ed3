#!/usr/bin/env python3
"""Benchmark: temporal edge-windows processed/sec for a batched-window CC Range query, 1-8 GPUs.

Headline workload (BASELINE.json configs[3], "C4"; the north star's 1B-event query):
  the seeded GAB-shaped add-only stream (VADD s, VADD d, EADD s->d at one t,
  GabUserGraphRouter.scala:31-33), 20M users, 333,333,334 interactions = 1,000,000,002 updates
  from 2016-08-10 to 2018-05-31; Range query over the last 168 hours, hopping 1 h, batched
  windows {year, month, week, day, hour}, ConnectedComponents (100-superstep cap).

  edge-windows = N_E x |windows| x |hops|   (N_E = directed edge entities)

One "step" = one complete Range query (every hop x window: window filter, CSR compaction, CC
supersteps, component-size reductions).  The packed graph is resident in HBM before timing.

N = 1: one partition (the one-GPU path).  N > 1 (python -m torch.distributed.run
--nproc-per-node N bench.py --gpus N): vertex-partitioned, partition = rank =
Utils.getPartition(id, N) (Utils.scala:32-33); each rank generates only the updates its
partition keeps (O(stream/N) host memory) and the library exchanges boundary label records
over RCCL every superstep.  The query is the same at every N ("scaling":
"strong"); timing = barrier + synchronize on both sides, max over ranks.

--config c2 is the BASELINE configs[1] query (C2, 100k vertices / 1M updates, 8,041 hourly
hops); at N = 1 the headline line carries it as a secondary object.  c3 / c5 / diffusion are
secondary lines.
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=3)
    p.add_argument("--warmup", type=int, default=1)
    p.add_argument("--cpu-seconds", type=float, default=12.0, help="bounded CPU-baseline sample")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-profile-pass", action="store_true")
    p.add_argument("--profile-only", action="store_true",
                   help="only the serial HIP-event profile passes (the command rocprofv3 is run on, so "
                        "that its per-kernel averages match the roofline figures)")
    p.add_argument("--lean-pass-only", action="store_true",
                   help="with --profile-only: the lean profile pass alone (no counting pass), so that a "
                        "rocprofv3 kernel trace holds exactly the launches bench.py times")
    p.add_argument("--config", default="c4", choices=["c2", "c3", "c4", "c5", "diffusion"],
                   help="c4 = the headline (north-star) query at every N; c2 = BASELINE configs[1]; "
                        "diffusion = BinaryDefusion over the C2 query (secondary)")
    p.add_argument("--no-secondary", action="store_true", help="N = 1: skip the C2 secondary object")
    p.add_argument("--partitioned", action="store_true",
                   help="N = 1: run the partitioned path with one partition (a one-rank RCCL channel): the "
                        "exchange protocol's fixed costs without peers")
    p.add_argument("--no-edge-counts", action="store_true", help="skip the SURVEY §8(d) byte-model pass")
    p.add_argument("--diff-seed", type=int, default=31,
                   help="diffusion infectedNode (BinaryDefusion.scala:10); -1 = the vertex with most EADDs as source")
    p.add_argument("--c5-users", type=int, default=20_000_000)
    p.add_argument("--c5-base", type=int, default=33_333_334, help="sealed base interactions (x3 updates)")
    p.add_argument("--c5-tick", type=int, default=3_333_334, help="interactions streamed per hour tick (x3 updates)")
    p.add_argument("--c5-ticks", type=int, default=6)
    p.add_argument("--c5-loopback", type=int, default=0,
                   help="C5 rehearsal on this many loopback partitions of one GPU, every kernel timed")
    p.add_argument("--c3-vertices", type=int, default=10_000_000)
    p.add_argument("--c3-events", type=int, default=100_000_000)
    p.add_argument("--c4-users", type=int, default=20_000_000)
    p.add_argument("--c4-interactions", type=int, default=333_333_334, help="x3 updates (1B at the default)")
    p.add_argument("--c4-hops", type=int, default=168)
    p.add_argument("--exchange", default="rccl", choices=["rccl", "shm"],
                   help="N > 1, C4 / C5: the label-record channel.  shm = the library's shared-memory group of "
                        "processes on one host, rank r on GPU r mod the visible GPUs: a rehearsal of the N > 1 "
                        "bench path on a one-GPU box (never a scaling number)")
    p.add_argument("--hybrid", default="auto",
                   help="C4: these windows (letters of 'ymwdh') are answered on a replica of the stream's time slice "
                        "[hop0 - the longest of them, end] (exact on the add-only C4 stream: a view (t, w) reads only "
                        "the updates in [t - w, t]), the others on the graph.  N > 1: hop-sharded, rank r runs its "
                        "contiguous block of the hops on its replica, the partitions answer the other windows.  "
                        "auto = 'mwdh' at N = 1, 'wdh' at N > 1 (measured, DESIGN.md §7); '' = off")
    p.add_argument("--hybrid-serial", action="store_true",
                   help="N = 1: run the graph's and the replica's parts one after the other (default: on two threads)")
    p.add_argument("--vertex-order", default="locality", choices=["locality", "id"],
                   help="local vertex order of the sealed graph (rgpu_set_vertex_order; A/B runs)")
    return p.parse_args()


def dist_env():
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    return rank, world, local


def pmc_traffic(kernel, config="C2"):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 PMC passes of `config`
    (tools/gpu_profile.sh -> profiles/latest_pmc[_c4].json), or None."""
    path = os.path.join(ROOT, "profiles", "latest_pmc.json" if config == "C2" else f"latest_pmc_{config.lower()}.json")
    try:
        with open(path) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None, None
    if kernel not in d.get("FETCH_SIZE", {}).get("kernel", ""):
        return None, None
    return (round(d["traffic_bytes_per_launch"]["value"]),
            os.path.relpath(path, ROOT) + " [" + d["FETCH_SIZE"]["kernel"] + "]: "
            + d["traffic_bytes_per_launch"]["formula"])


AGG_KERNELS = ("window_mask", "edge_mask", "cc_slots", "heavy", "cc_step")


def aggregate_roofline(kraw, config):
    """The north star's figure (BASELINE.json: "≥50% of MI355X HBM bandwidth on the window-filter+CC
    kernels"): K1 (vertex + edge window masks), K2 (cc_slots), the hub kernels (K2's segment pass,
    the per-superstep gather and mark) and K3 (the superstep kernel), pooled — the sum of their
    DESIGN.md §4 algorithmic bytes (counting pass) over the sum of their serial lean-pass ms.  Beside
    each group: the HBM traffic the committed rocprofv3 PMC passes of the same command counted
    (profiles/latest_pmc[_c4].json "by_group", per launch x this pass's launches) and its ratio to
    the model."""
    path = os.path.join(ROOT, "profiles", "latest_pmc.json" if config == "C2" else f"latest_pmc_{config.lower()}.json")
    try:
        with open(path) as f:
            pmc = json.load(f).get("by_group", {})
    except (OSError, ValueError):
        pmc = {}
    per, tb, tms, ttr, covered = {}, 0.0, 0.0, 0.0, True
    for k in AGG_KERNELS:
        d = kraw.get(k)
        if not d or not d["launches"]:
            continue
        e = {"launches": d["launches"], "ms": round(d["ms"], 3), "algorithmic_bytes": d["bytes"],
             "achieved_GBps": round(d["bytes"] / max(d["ms"], 1e-9) / 1e6, 1),
             "frac": round(d["bytes"] / max(d["ms"], 1e-9) / 1e6 / HBM_PEAK_GBS, 4)}
        p = pmc.get(k)
        if p:
            tr = p["traffic_bytes_per_launch"] * d["launches"]
            e["traffic_bytes"] = round(tr)
            e["pmc_dispatches"] = p["dispatches"]
            if d["bytes"] > 0:
                e["traffic_over_algorithmic"] = round(tr / d["bytes"], 2)
            ttr += tr
        else:
            covered = False
        per[k] = e
        tb += d["bytes"]
        tms += d["ms"]
    gbs = tb / max(tms, 1e-9) / 1e6
    return {"kernels": "+".join(per), "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(gbs / HBM_PEAK_GBS, 4), "ms": round(tms, 3), "algorithmic_bytes": tb,
            "traffic": round(ttr) if covered and per else None,
            "traffic_over_algorithmic": round(ttr / tb, 2) if covered and tb > 0 else None,
            "traffic_source": os.path.relpath(path, ROOT) + " by_group" if pmc else None,
            "by_kernel": per}


def cpu_info():
    """(threads the host gives this job, nproc, CPU model): the GPU box shares its cores, and
    says how many through OMP_NUM_THREADS (os.cpu_count() shows the whole machine)."""
    aff = len(os.sched_getaffinity(0))
    want = int(os.environ.get("OMP_NUM_THREADS") or 0) or aff
    model = "?"
    try:
        with open("/proc/cpuinfo") as f:
            model = next((l.split(":", 1)[1].strip() for l in f if l.startswith("model name")), "?")
    except OSError:
        pass
    return max(1, min(want, aff)), os.cpu_count(), model


def cpu_baseline(stream, hops, windows, budget_s, n_edges, what, lazy=False):
    """The CPU oracle on the host's cores (ctypes releases the GIL: one view job per thread), over
    hops drawn uniformly from the whole range: mode 0 = the reference's algorithmic structure
    ("refsim": the lens rebuilt by linear closestTime scans every superstep, adjacency re-filtered
    on every visit, queue messages; the reported value), mode 1 = the same semantics with
    per-view caching (a fairer CPU bound, reported beside it)."""
    from concurrent.futures import ThreadPoolExecutor
    from oracle import Oracle
    threads, nproc, model = cpu_info()
    t0 = time.perf_counter()
    o = Oracle.from_stream(stream, lazy=lazy)
    build_s = time.perf_counter() - t0
    order = np.random.default_rng(0).permutation(len(hops))  # uniform over the range
    out = {}
    for mode, budget in ((0, budget_s), (1, budget_s / 2)):
        done, t0 = 0, time.perf_counter()
        with ThreadPoolExecutor(threads) as ex:
            while done < len(order) and time.perf_counter() - t0 < budget:
                batch = order[done:done + threads]
                list(ex.map(lambda h: o.cc(int(hops[h]), windows, max_steps=100, mode=mode), batch))
                done += len(batch)
        dt = time.perf_counter() - t0
        out[mode] = (n_edges * len(windows) * done / dt, done, dt)
    o.close()
    v0, d0, t0_ = out[0]
    v1, d1, t1_ = out[1]
    return {
        "value": v0,
        "unit": "edge-windows/s",
        "cores": threads,
        "kind": "port",
        "nproc": nproc,
        "cpu_model": model,
        "sample": f"{what}: {d0} of {len(hops)} hops (uniform random over the range) x {len(windows)} windows, "
                  f"oracle refsim mode (reference algorithmic structure), {t0_:.1f} s on {threads} threads "
                  f"(oracle build {build_s:.1f} s, not timed); restatement, not the JVM",
        "fast_oracle": {"value": v1, "unit": "edge-windows/s", "cores": threads,
                        "sample": f"{d1} hops, oracle mode 1 (cached adjacency), {t1_:.1f} s"},
    }


def cpu_same_config(inter, users, hops, budget_s, n_edges):
    """The CPU oracle on the headline's own stream and views: the month, week, day
    and hour views of the real 1B-update query (4 of its 5 windows), at hops drawn uniformly from its
    168, replayed from the time slice [hop0 - month, hop167] of the stream (exact: on an add-only
    stream a view (t, w) depends only on the updates in [t - w, t], tools/make_c4_sliced_goldens.py,
    tests/test_c4_slice.py).  The four windows run as one batched-window job per hop, as the
    reference's ReaderWorker runs a batch (ReaderWorker.scala:159-257); their vertex sets are the
    running minimum of [y,m,w,d,h] at those positions, i.e. each window itself.  The year window
    (564M updates of slice) does not fit the literal replay.  The slice holds only the entities
    active in the last ~37 days, where the reference's lens scans every vertex of its shard each
    superstep (ReaderWorker.scala:171,202), so this CPU time is a lower bound on the reference
    structure's.  One month view costs ~130 s of refsim on one core, so at least one hop per thread
    runs whatever the budget.  Value = edge entities of the whole graph x 4 windows x hops done /
    time, the metric's own definition."""
    from concurrent.futures import ThreadPoolExecutor
    from oracle import Oracle
    from raphtory_amd.synth import DAY, HOUR, MONTH, WEEK, Stream, gen_gab_range
    from tools.make_c4_sliced_goldens import first_at
    threads, _, _ = cpu_info()
    wins, wnames = [MONTH, WEEK, DAY, HOUR], "month, week, day, hour (4 of the query's 5)"
    t0 = time.perf_counter()
    first = first_at(int(hops[0]) - MONTH, inter, inter)
    parts = [gen_gab_range(4, users, inter, f, min(10_000_000, inter - f)) for f in range(first, inter, 10_000_000)]
    sl = Stream(*(np.concatenate([getattr(p, k) for p in parts]) for k in ("t", "kind", "src", "dst")))
    del parts
    log(f"same-config CPU baseline: slice of {len(sl)} updates; building the oracle")
    o = Oracle.from_stream(sl, lazy=True)
    n_slice = len(sl)
    del sl
    build_s = time.perf_counter() - t0
    log(f"same-config CPU baseline: oracle built in {build_s:.0f} s; refsim over {threads} hops at a time")
    order = np.random.default_rng(0).permutation(len(hops))
    done, t1 = 0, time.perf_counter()
    with ThreadPoolExecutor(threads) as ex:
        while done < len(order) and time.perf_counter() - t1 < budget_s:
            batch = order[done:done + threads]
            list(ex.map(lambda h: o.cc(int(hops[h]), wins, max_steps=100, mode=0), batch))
            done += len(batch)
    dt = time.perf_counter() - t1
    o.close()
    log(f"same-config CPU baseline: {done} hops in {dt:.0f} s")
    return {"value": n_edges * len(wins) * done / dt, "unit": "edge-windows/s", "cores": threads, "kind": "port",
            "windows": wnames,
            "sample": f"the 1B headline's own month, week, day and hour views (one batched job per hop): {done} of "
                      f"{len(hops)} hops (uniform random), oracle refsim mode, {dt:.1f} s on {threads} threads, "
                      f"replayed from the time slice [hop0 - month, hop167] ({n_slice} updates; slice + oracle build "
                      f"{build_s:.1f} s, not timed); a lower bound on the reference structure's time (its lens scans "
                      "every shard vertex).  (No cached-oracle pass here: its month views cost ~40 s more; the "
                      "1/100-scale line carries one.)"}


def setup_latency(g, hops, windows, n=40):
    """The per-Setup drop-in path (GpuReaderWorker): one rgpu_run_view_batch
    per hop (1 hop x |windows|, RGPU_RUN_RETAIN) followed by rgpu_cc_result per window (the
    label -> count map ConnectedComponents.returnResults ships, ConnectedComponents.scala:37-42),
    over n hops drawn uniformly from the range; and the summary-only form (rgpu_cc_summary,
    no retained rows).  Wall ms per Setup = one hop's whole batched-window job."""
    import torch
    pick = np.sort(np.random.default_rng(1).choice(len(hops), size=min(n, len(hops)), replace=False))
    out = {}
    for form in ("cc_result", "summary"):
        ts = []
        for h in pick:
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            g.run("cc", [int(hops[h])], windows, retain=form == "cc_result")
            if form == "cc_result":
                for w in range(len(windows)):
                    g.cc_result(0, w)
            else:
                for w in range(len(windows)):
                    g.cc_summary(0, w)
            ts.append((time.perf_counter() - t0) * 1e3)
        ts = np.array(ts)
        out[form] = {"ms_per_setup_mean": round(float(ts.mean()), 3), "ms_per_setup_median": round(float(np.median(ts)), 3),
                     "ms_per_view_mean": round(float(ts.mean()) / len(windows), 3), "setups": int(len(ts))}
    out["note"] = (f"{len(pick)} hops uniform over the range, one call per hop x {len(windows)} windows "
                   "(RangeAnalysisTask restarting per hop); the batched headline answers every hop in one call")
    return out


def run_c3(a, rank, world, local):
    """BASELINE configs[2] (C3): power-law stream, 10M vertices / 100M updates over two years;
    Range over the last 60 days, daily hops, windows [month, week, day]; PageRank (20
    iterations) + DegreeBasic.  A secondary line, not the headline metric."""
    import torch
    from raphtory_amd import TemporalGraph
    from raphtory_amd.synth import DAY, MONTH, T0_README, WEEK, YEAR, gen_powerlaw, range_hops
    t0 = time.perf_counter()
    nv, ne = (a.c3_vertices, a.c3_events)
    s = gen_powerlaw(3, nv, ne, t0=T0_README, t1=T0_README + 2 * YEAR)
    gen_s = time.perf_counter() - t0
    g = TemporalGraph(device=local)
    g.ingest_stream(s)
    t0 = time.perf_counter()
    g.seal()
    seal_s = time.perf_counter() - t0
    end = T0_README + 2 * YEAR
    hops = range_hops(end - 60 * DAY, end, DAY)
    windows = [MONTH, WEEK, DAY]
    st = g.stats()
    out = {"config": "C3", "vertices": st["vertices"], "edge_entities": st["edges"],
           "vertex_events": st["vertex_events"], "edge_events": st["edge_events"], "deaths": st["deaths"],
           "gen_s": round(gen_s, 2), "seal_s": round(seal_s, 2), "hops": len(hops), "windows": len(windows)}
    for algo in ("pagerank", "degree"):
        g.run(algo, hops, windows, pr_iters=20)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            g.run(algo, hops, windows, pr_iters=20)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) * 1e3 / a.steps
        out[algo] = {"ms": round(ms, 2), "edge_windows_per_s": st["edges"] * len(windows) * len(hops) / (ms / 1e3)}
        g.run(algo, hops, windows, pr_iters=20, profile=True, serial=True)
        out[algo]["kernels"] = {k: {"launches": v["launches"], "ms": round(v["ms"], 3),
                                    "GBps": round(v["bytes"] / max(v["ms"], 1e-9) / 1e6, 1)}
                                for k, v in g.stats()["kernels"].items() if v["launches"]}
    tot = [g.degree_result(h, w)[:3] for h in (0, len(hops) - 1) for w in range(3)]
    out["degree_totals_first_last_hop"] = tot
    g.close()
    print(json.dumps(out))


def run_diffusion(a, rank, world, local):
    """Secondary line: BinaryDefusion (BinaryDefusion.scala) over the C2
    query (8,041 hourly hops x {y,m,w,d,h}, infectedNode 31), hash coin and taint (no coin)."""
    import torch
    from raphtory_amd import TemporalGraph
    from raphtory_amd.synth import BATCH_WINDOWS, DAY, HOUR, T0_README, gen_uniform, range_hops
    stream = gen_uniform(1, 100_000, 1_000_000)
    hops = range_hops(T0_README + 30 * DAY, T0_README + 365 * DAY, HOUR)
    seed = a.diff_seed
    if seed < 0:
        import numpy as np
        ids, cnt = np.unique(stream.src[stream.kind == 2], return_counts=True)
        seed = int(ids[np.argmax(cnt)])
    g = TemporalGraph(device=local)
    g.ingest_stream(stream)
    g.seal()
    st = g.stats()
    out = {"config": "C2 query, BinaryDefusion", "infectedNode": seed, "vertices": st["vertices"],
           "edge_entities": st["edges"], "hops": len(hops), "windows": len(BATCH_WINDOWS)}
    for name, coin in (("coin", True), ("taint", False)):
        g.set_diffusion(seed, 0, coin)
        g.run("diffusion", hops, BATCH_WINDOWS)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            g.run("diffusion", hops, BATCH_WINDOWS)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) * 1e3 / a.steps
        r = {"ms": round(ms, 2), "edge_windows_per_s": st["edges"] * len(BATCH_WINDOWS) * len(hops) / (ms / 1e3)}
        sizes = [g.diffusion_result(h, w)[0] for h in (0, len(hops) // 2, len(hops) - 1) for w in range(5)]
        r["infected_first_mid_last_hop"] = sizes
        g.run("diffusion", hops, BATCH_WINDOWS, profile=True, serial=True)
        r["supersteps"] = g.stats()["supersteps"]
        r["kernels"] = {k: {"launches": v["launches"], "ms": round(v["ms"], 3),
                            "GBps": round(v["bytes"] / max(v["ms"], 1e-9) / 1e6, 1)}
                        for k, v in g.stats()["kernels"].items() if v["launches"]}
        out[name] = r
    g.close()
    print(json.dumps(out))


_PHASE = ["start"]


def log(msg):
    _PHASE[0] = msg[:120]
    print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def heartbeat(every_s=50.0):
    """A progress line on stderr every `every_s` seconds (the CPU baselines run minutes without
    output; a watchdog that takes a silent job for hung must see it alive)."""
    import threading

    def beat():
        while True:
            time.sleep(every_s)
            print(f"[bench {time.strftime('%H:%M:%S')}] alive, last phase: {_PHASE[0]}", file=sys.stderr, flush=True)

    threading.Thread(target=beat, daemon=True).start()


def kernel_table(stats):
    """Per kernel group: launches, serial ms, and GB/s of the DESIGN.md §4 byte model (None where
    the group has no byte model: the hub kernels)."""
    return {k: {"launches": v["launches"], "ms": round(v["ms"], 3),
                "avg_us": round(v["ms"] * 1e3 / v["launches"], 2),
                "GBps": round(v["bytes"] / max(v["ms"], 1e-9) / 1e6, 1) if v["bytes"] > 0 else None}
            for k, v in stats["kernels"].items() if v["launches"]}


def profile_passes(g, hops, windows, lean_only=False):
    """Two serial profiled passes of the same query: a counting pass (the kernels' work counters ->
    DESIGN.md §4 bytes per kernel) and a lean pass (RGPU_PROF_LEAN=1: the same launches on the
    instantiations the timed runs use, under HIP events -> ms).  Returns {kernel: {launches, ms,
    bytes}} with bytes from the first and launches / ms from the second.  lean_only: the lean pass
    alone (the command a rocprofv3 kernel trace runs, so that its per-kernel sums are this pass's)."""
    counted = {}
    if not lean_only:
        g.run("cc", hops, windows, profile=True, serial=True)
        counted = g.stats()["kernels"]
    os.environ["RGPU_PROF_LEAN"] = "1"
    try:
        g.run("cc", hops, windows, profile=True, serial=True)
    finally:
        os.environ.pop("RGPU_PROF_LEAN", None)
    lean = g.stats()["kernels"]
    return {k: {"launches": v["launches"], "ms": v["ms"], "bytes": counted.get(k, {}).get("bytes", 0.0),
                "ms_counting_pass": counted.get(k, {}).get("ms", 0.0)} for k, v in lean.items()}


def survey_bytes(summ, n_hops, windows, nv, ne, n_ev, ks, launches_step):
    """SURVEY.md §8(d) algorithmic bytes of the query from the per-view counts the library
    reports (|E_{t,w}| = alive_edges, R = the hop's superstep count):
      K1  B1 = sum over hop blocks [8 N_ev + 8 (N_ent + 1) + K N_ent]
      K2  B2 = sum over hops [N_E + sum_w (8|E_w| + 4 d |E_w| + 4 (V + 1))],  d = 2
      K3  B3 = sum over views and executed supersteps [4 (V + 1) + 8 d |E_w| + 8 V + V / 4]
    Superstep 1 runs inside the K2 kernel here, so the superstep kernel's share is supersteps
    2..R."""
    W = len(windows)
    alive = summ[..., 8].astype(np.float64)
    R = summ[..., 7].astype(np.float64)
    n_ent = nv + ne
    blocks = [min(64, n_hops - h) for h in range(0, n_hops, 64)]
    b1 = sum(8.0 * n_ev + 8.0 * (n_ent + 1) + k * n_ent for k in blocks)
    b2 = n_hops * ne + 16.0 * alive.sum() + n_hops * W * 4.0 * (nv + 1)
    unit = 4.0 * (nv + 1) + 16.0 * alive + 8.0 * nv + nv / 4.0
    b3 = float((R * unit).sum())
    b3_step = float((np.maximum(R - 1, 0) * unit).sum())
    t = sum(ks.get(k, {}).get("ms", 0.0) for k in ("window_mask", "cc_slots", "cc_step", "heavy", "cc_tail"))
    t_step = ks.get("cc_step", {}).get("ms", 0.0)
    return {"B1": b1, "B2": b2, "B3": b3, "alive_edge_windows": float(alive.sum()),
            "supersteps_per_view_mean": float(R.mean()),
            "K1_K2_K3_ms": t, "achieved_GBps": (b1 + b2 + b3) / max(t, 1e-9) / 1e6,
            "cc_step": {"B3_steps_2_to_R": b3_step, "launches": launches_step,
                        "bytes_per_launch": b3_step / max(1, launches_step),
                        "achieved_GBps": b3_step / max(t_step, 1e-9) / 1e6}}


def run_c4(a, rank, world, local):
    """The headline line: BASELINE configs[3] (C4), the 1B-update GAB-shaped stream, batched
    windows {y,m,w,d,h} over the last 168 hourly hops, CC, on N = world GPUs (one partition per
    GPU when N > 1)."""
    import torch
    from raphtory_amd import TemporalGraph
    from raphtory_amd.partitioned import combine_window_groups, hop_blocks
    from raphtory_amd.synth import BATCH_WINDOWS, HOUR, gab_first_at, gen_gab_range, range_hops
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("gloo")  # control plane; the data path is the library's RCCL
    if dist is not None:
        from raphtory_amd.partitioned import open_rccl_partition
        g = open_rccl_partition(local, dist, kind=a.exchange)
    elif a.partitioned:
        os.environ["RGPU_PARTITIONED"] = "1"
        g = TemporalGraph(device=local)
        g.exchange_init(TemporalGraph.exchange_id())
    else:
        g = TemporalGraph(device=local)
    if a.vertex_order != "locality":
        g.set_vertex_order(a.vertex_order)
    users, inter = a.c4_users, a.c4_interactions
    t0 = time.perf_counter()
    chunk = 20_000_000
    n_kept = 0
    for first in range(0, inter, chunk):  # this rank's updates only: O(stream / N) host memory
        s = gen_gab_range(4, users, inter, first, chunk, rank, world)
        g.ingest_stream(s)
        n_kept += len(s)
        del s
    end = int(gen_gab_range(4, users, inter, inter - 1, 1).t[-1])
    gen_s = time.perf_counter() - t0
    log(f"rank {rank}: C4 stream generated + ingested in {gen_s:.1f} s ({n_kept} of {3 * inter} updates kept)")
    t0 = time.perf_counter()
    g.seal()
    seal_s = time.perf_counter() - t0
    st = g.stats()

    def total(x):
        if dist is None:
            return int(x)
        t = torch.tensor([int(x)], dtype=torch.int64)
        dist.all_reduce(t)
        return int(t.item())

    n_edges = total(st["edges_owned"])
    n_vert = total(st["vertices"])
    log(f"rank {rank}: sealed in {seal_s:.1f} s: {st['vertices']} owned vertices, {st['edges']} edges here; "
        f"graph {n_vert} vertices, {n_edges} edge entities")
    hops = range_hops(end - (a.c4_hops - 1) * HOUR, end, HOUR)
    windows = BATCH_WINDOWS
    # N > 1 (--hybrid): the short windows hop-sharded on a time-slice replica, the others partitioned
    if a.hybrid == "auto":
        a.hybrid = "wdh" if world > 1 else "mwdh"
    short_i = [i for i, c in enumerate("ymwdh") if c in a.hybrid]
    long_w = [w for i, w in enumerate(windows) if i not in short_i]
    short_w = [windows[i] for i in short_i]
    blocks = hop_blocks(len(hops), world)
    gs = None
    if short_i:
        t1 = time.perf_counter()
        f0 = gab_first_at(4, users, inter, int(hops[0]) - max(short_w))
        gs = TemporalGraph(device=local)
        for first in range(f0, inter, chunk):
            gs.ingest_stream(gen_gab_range(4, users, inter, first, min(chunk, inter - first)))
        gs.seal()
        log(f"rank {rank}: windows {a.hybrid} hop-sharded: slice replica of {3 * (inter - f0)} updates, hops "
            f"[{blocks[rank][0]}, {blocks[rank][1]}), built in {time.perf_counter() - t1:.1f} s")
    my_hops = hops[blocks[rank][0]:blocks[rank][1]]

    def query():
        if gs is not None and len(my_hops) and dist is None and not a.hybrid_serial:
            # N = 1: the two runs on two host threads (the library call drops the GIL), so that each run's
            # sparse late supersteps overlap the other's work on the GPU
            err = []

            def short():
                try:
                    gs.run("cc", my_hops, short_w)
                except BaseException as e:  # noqa: BLE001  (re-raised below)
                    err.append(e)
            th = threading.Thread(target=short)
            th.start()
            try:
                g.run("cc", hops, long_w)
            finally:
                th.join()
            if err:
                raise err[0]
            return
        g.run("cc", hops, long_w)  # collective over the partitions
        if gs is not None and len(my_hops):
            gs.run("cc", my_hops, short_w)  # this rank's block, no exchange

    def summaries():
        sl = g.cc_summaries()
        if gs is None:
            return sl
        got = [None] * world
        if dist is None:
            got = [gs.cc_summaries()]
        else:
            dist.all_gather_object(got, gs.cc_summaries() if len(my_hops) else None)
        return combine_window_groups(len(windows), [i for i in range(len(windows)) if i not in short_i], sl, short_i,
                                     [(lo, hi, x) for (lo, hi), x in zip(blocks, got)])

    def barrier():
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()

    if a.profile_only:
        a.steps, a.warmup, a.no_cpu_baseline = 1, 0, True
    if a.lean_pass_only:  # a rocprofv3 trace of this command holds the serial lean pass alone
        a.no_edge_counts = True
    for _ in range(a.warmup):
        query()
    barrier()
    t0 = time.perf_counter()
    for _ in range(0 if a.profile_only else a.steps):
        query()
    barrier()
    elapsed = time.perf_counter() - t0
    if dist is not None:
        from raphtory_amd.replicas import max_over_ranks
        elapsed = max_over_ranks(elapsed, dist)
    ms_per_step = elapsed * 1e3 / max(1, a.steps)
    value = n_edges * len(windows) * len(hops) / (ms_per_step / 1e3)
    if a.profile_only:
        ms_per_step = value = None
    log(f"rank {rank}: query {ms_per_step} ms")
    summ = None if a.profile_only or gs is not None else g.cc_summaries()  # (profile-only: after the profile pass)
    if gs is not None and not a.profile_only:
        summ = summaries()  # (collective) before the profile passes overwrite the partitions' results
    roofline, ks, s8d = None, {}, None
    if not a.no_profile_pass:
        log("profile passes")
        kraw = profile_passes(g, hops, long_w, lean_only=a.lean_pass_only)  # collective at N > 1
        if gs is not None and len(my_hops):  # the replica's share of the query, pooled per kernel
            for k, v in profile_passes(gs, my_hops, short_w, lean_only=a.lean_pass_only).items():
                d = kraw.setdefault(k, {"launches": 0, "ms": 0.0, "bytes": 0.0, "ms_counting_pass": 0.0})
                for f in ("launches", "ms", "bytes", "ms_counting_pass"):
                    d[f] += v[f]
        ks = kernel_table({"kernels": kraw})
        if summ is None:
            summ = summaries()
        d = kraw["cc_step"]
        gbs = d["bytes"] / (d["ms"] / 1e3) / 1e9
        traffic, tsrc = pmc_traffic("k_cc_step_pk", config="C4")
        roofline = {"bound": "hbm", "kernel": "cc_step (k_cc_step_pk)", "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS,
                    "unit": "GB/s", "frac": round(gbs / HBM_PEAK_GBS, 4), "traffic": traffic, "traffic_source": tsrc,
                    "avg_launch_us": round(d["ms"] * 1e3 / d["launches"], 2),
                    "algorithmic_bytes_per_launch": d["bytes"] / d["launches"],
                    "avg_launch_us_counting_pass": round(d["ms_counting_pass"] * 1e3 / d["launches"], 2),
                    "bytes_model": "DESIGN.md §4 (bytes the superstep must touch per visited vertex / slot / "
                                   "gathered label, counted by the kernel in a counting pass); time = the same "
                                   "launches of the lean instantiation the timed query runs (RGPU_PROF_LEAN)"}
        if traffic:  # the memory system's real rate and its waste (the progress signal beside frac)
            roofline["traffic_rate_GBps"] = round(traffic / (d["ms"] / d["launches"] / 1e3) / 1e9, 1)
            if d["bytes"] > 0:  # (--lean-pass-only runs no counting pass: no algorithmic bytes)
                roofline["traffic_over_algorithmic"] = round(traffic / (d["bytes"] / d["launches"]), 2)
        if not a.lean_pass_only:
            roofline["aggregate"] = aggregate_roofline(kraw, "C4")
        if not a.no_edge_counts and world == 1:
            g.run("cc", hops, windows, edge_counts=True)
            summ = g.cc_summaries()  # (every window on the graph here)
            s8d = survey_bytes(summ, len(hops), windows, st["vertices"], st["edges"],
                               st["vertex_events"] + st["edge_events"] + st["deaths"], ks, d["launches"])
            roofline["survey_8d"] = {"achieved": round(s8d["cc_step"]["achieved_GBps"], 1),
                                     "frac": round(s8d["cc_step"]["achieved_GBps"] / HBM_PEAK_GBS, 4),
                                     "bytes_per_launch": s8d["cc_step"]["bytes_per_launch"],
                                     "note": "SURVEY §8(d) B3 over supersteps 2..R of every view (one CSR pass "
                                             "per view per superstep) / the same launches' time"}
    cpu = None
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        log("CPU baseline (1/100-scale stream)")
        from raphtory_amd.synth import gen_gab
        sm = gen_gab(4, users // 100, inter // 100)  # the same query on the 1/100-scale stream
        sm_end = int(sm.t[-1])
        sm_hops = range_hops(sm_end - (a.c4_hops - 1) * HOUR, sm_end, HOUR)
        gs = TemporalGraph(device=local)
        gs.ingest_stream(sm)
        gs.seal()
        sm_edges = gs.stats()["edges"]
        gs.close()
        cpu = cpu_baseline(sm, sm_hops, windows, a.cpu_seconds, sm_edges,
                           f"C4 query on the 1/100-scale GAB stream ({len(sm)} updates, {users // 100} users, "
                           f"{sm_edges} edge entities, same span)", lazy=True)
        if inter == 333_333_334 and len(hops) == 168:  # the headline query itself
            cpu["same_config"] = cpu_same_config(inter, users, hops, a.cpu_seconds, n_edges)
    secondary = None
    if rank == 0 and world == 1 and not a.no_secondary and not a.profile_only:
        log("C2 secondary line")
        secondary = run_c2(a, 0, 1, local, quiet=True)
    if rank == 0:
        out = {
            "metric": "temporal edge-windows processed/sec for batched-window CC range query",
            "value": round(value, 1) if value is not None else None,
            "unit": "edge-windows/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(ms_per_step, 3) if ms_per_step is not None else None,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "int32",
            "data": "synthetic (seeded GAB-shaped add-only stream, SURVEY.md App. B gen_gab)",
            "config": {"workload": "C4: 1B-update GAB-shaped stream (20M users, 333,333,334 interactions), "
                                   "168 hourly hops x 5 batched windows {y,m,w,d,h}, ConnectedComponents",
                       "updates": 3 * inter, "vertices": n_vert, "edge_entities": n_edges, "hops": int(len(hops)),
                       "windows": len(windows),
                       "parallelism": ("one GPU, partitioned path (P = 1)" if a.partitioned else
                                       f"one GPU; windows {a.hybrid} on a time-slice replica" if short_i else "one GPU")
                                      if world == 1 else
                                      f"vertex-partitioned x{world} (Utils.getPartition), "
                                      + ("RCCL label records" if a.exchange == "rccl" else
                                         "shared-memory label records on one host (rehearsal, not a scaling number)")
                                      + (f"; windows {a.hybrid} hop-sharded over the ranks on a time-slice replica"
                                         if short_i else ""),
                       "gen_ingest_s": round(gen_s, 1), "seal_s": round(seal_s, 1),
                       "supersteps_per_view_mean": round(float(summ[..., 7].mean()), 2),
                       "alive_edge_windows": s8d["alive_edge_windows"] if s8d else None,
                       "alive_edge_windows_frac": (s8d["alive_edge_windows"] / (n_edges * len(windows) * len(hops)))
                                                  if s8d else None},
            "roofline": roofline,
            "survey_8d_bytes": s8d,
            "cpu_baseline": cpu,
            "kernels": ks,
            "check": {"views": int(summ.shape[0] * summ.shape[1]), "sum_biggest": int(summ[..., 0].sum()),
                      "sum_total": int(summ[..., 1].sum()), "sum_members": int(summ[..., 5].sum()),
                      "sum_supersteps": int(summ[..., 7].sum())},
            "secondary": secondary,
        }
        print(json.dumps(out), flush=True)
    g.close()
    if gs is not None:
        gs.close()
    if dist is not None:
        dist.destroy_process_group()


def run_c5(a, rank, world, local):
    """BASELINE configs[4] (C5): live analysis under ingest.  A GAB-shaped base (default 100M
    updates, 20M users) is sealed once; then every hour tick the Router's next 10M updates (one
    hour of stream time past the newest point) are ingested and merged into the HBM-resident
    graph by the incremental seal (gdelta.hip + merge.hip), and CC (batched windows {y,m,w,d,h})
    and PageRank (20 iterations, hour window) run on the newest hour at the live time (the minimum
    newest time over the partitions), as LiveAnalysisTask does (LiveAnalysisTask.scala:13-107).
    Ingestion does not wait for the analysis: while tick i's CC + PR run, a second host thread
    ingests tick i+1 and merges it (the library builds the merged graph beside the resident one and
    swaps it in between runs), as the reference's IngestionWorker keeps applying updates while
    LiveAnalysisTask runs (IngestionWorker.scala:31-61).  N > 1: one vertex partition per GPU
    (RCCL), each rank ingesting and merging its own part of every tick.  Reported: sustained
    updates/s over the whole loop, tick 0 included (first ingest to last analysis), and per tick the
    analysis and the ingest + merge that overlapped it.  Generating the updates (the Router's side)
    is outside the timed region.  --c5-loopback P: the same loop (no overlap) on P loopback
    partitions of one GPU with every kernel timed per partition (RGPU_LOOPBACK_ISOLATE) — a
    rehearsal of the partitioned tick.  Secondary line."""
    if a.c5_loopback > 1:
        return run_c5_loopback(a)
    import threading
    import torch
    from raphtory_amd import TemporalGraph
    from raphtory_amd.synth import BATCH_WINDOWS, HOUR, gen_gab_range
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("gloo")  # control plane; the data path is the library's RCCL
        from raphtory_amd.partitioned import open_rccl_partition
        g = open_rccl_partition(local, dist, vertex_order="id", kind=a.exchange)  # live: later seals merge
    elif a.partitioned:
        os.environ["RGPU_PARTITIONED"] = "1"
        g = TemporalGraph(device=local, vertex_order="id")
        g.exchange_init(TemporalGraph.exchange_id())
    else:
        g = TemporalGraph(device=local, vertex_order="id")

    def reduce(x, op):
        if dist is None:
            return x
        t = torch.tensor([x], dtype=torch.float64)
        dist.all_reduce(t, op=op)
        return t.item()

    def barrier():
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()

    MIN, MAX = (dist.ReduceOp.MIN, dist.ReduceOp.MAX) if dist is not None else (None, None)
    s = gen_gab_range(4, a.c5_users, a.c5_base, 0, a.c5_base, rank, world)
    n_base = 3 * a.c5_base
    g.ingest_stream(s)
    del s
    barrier()
    t0 = time.perf_counter()
    g.seal()
    base_seal_s = reduce(time.perf_counter() - t0, MAX)
    now = int(reduce(g.newest_time(), MAX))
    log(f"rank {rank}: C5 base: {n_base} updates ({g.stats()['vertices']} owned vertices here) sealed in "
        f"{base_seal_s:.1f} s")
    ticks = []  # the Router's next ticks, generated before the clock starts
    for i in range(a.c5_ticks):
        ticks.append(gen_gab_range(100 + i, a.c5_users, a.c5_tick, 0, a.c5_tick, rank, world, t0=now + 1,
                                   t1=now + HOUR, id_key=4))
        now += HOUR
    upd_ticks = 3 * a.c5_tick  # (updates of the whole stream per tick; a rank keeps its part)
    recs = [dict() for _ in ticks]
    err = []

    def ingest_merge(i):
        try:
            t = time.perf_counter()
            g.ingest_stream(ticks[i])
            t1 = time.perf_counter()
            g.seal()
            t2 = time.perf_counter()
            recs[i].update(ingest_ms=(t1 - t) * 1e3, merge_ms=(t2 - t1) * 1e3, merge_done=t2)
        except BaseException as e:  # noqa: BLE001 - re-raised in the main thread
            err.append(e)

    barrier()
    t_start = time.perf_counter()
    ingest_merge(0)  # tick 0: nothing to overlap with yet
    for i in range(len(ticks)):
        if err:
            raise err[0]
        assert g.stats()["seal_incremental"] == 1
        live = int(reduce(g.newest_time(), MIN))  # LiveAnalysisTask.setLiveTime (tick i is sealed)
        th = threading.Thread(target=ingest_merge, args=(i + 1,)) if i + 1 < len(ticks) else None
        ta = time.perf_counter()
        if th is not None:
            th.start()  # tick i+1 streams in while tick i is analysed
        g.run("cc", [live], BATCH_WINDOWS)
        tb = time.perf_counter()
        g.run("pagerank", [live], [HOUR], pr_iters=20)
        torch.cuda.synchronize()
        tc = time.perf_counter()
        if th is not None:
            th.join()
        td = time.perf_counter()
        recs[i].update(cc_ms=(tb - ta) * 1e3, pr_ms=(tc - tb) * 1e3, tick_ms=(td - ta) * 1e3)
    barrier()
    wall = reduce(time.perf_counter() - t_start, MAX)
    if err:
        raise err[0]
    st = g.stats()
    for r in recs:
        for k in ("ingest_ms", "merge_ms", "cc_ms", "pr_ms", "tick_ms"):
            r[k] = reduce(r[k], MAX)
        r.pop("merge_done", None)
    if rank == 0:
        for i, r in enumerate(recs):
            log(f"tick {i}: " + " ".join(f"{k}={v:.1f}" for k, v in r.items()))
    up = upd_ticks * len(ticks)
    n_v = int(reduce(st["vertices"], dist.ReduceOp.SUM) if dist is not None else st["vertices"])
    n_e = int(reduce(st["edges_owned"], dist.ReduceOp.SUM) if dist is not None else st["edges"])
    out = {"metric": "live updates/s sustained (ingest + merge + CC {y,m,w,d,h} + PageRank per tick)",
           "value": up / wall if wall else None, "unit": "updates/s", "higher_is_better": True,
           "config": "C5", "n_gpus": world, "base_updates": n_base, "base_seal_s": round(base_seal_s, 1),
           "ticks": len(ticks), "updates_per_tick": upd_ticks,
           "live_updates_per_s": up / wall if wall else None, "wall_s": round(wall, 3),
           "sustained_note": "every tick included (tick 0's ingest + merge too), first ingest to last analysis",
           "mean_ms": {k: round(sum(r[k] for r in recs) / len(recs), 1)
                       for k in ("ingest_ms", "merge_ms", "cc_ms", "pr_ms", "tick_ms")},
           "ticks_ms": [{k: round(v, 1) for k, v in r.items()} for r in recs],
           "final_vertices": n_v, "final_edges": n_e,
           "parallelism": (f"vertex-partitioned x{world}, RCCL" if world > 1 else
                           "one GPU, partitioned path (P = 1)" if a.partitioned else "one GPU"),
           "overlap": "tick i+1's ingest + merge (host thread, merge stream) overlap tick i's CC + PR",
           "delta_packer": "host (RGPU_DELTA=2)" if os.environ.get("RGPU_DELTA") == "2" else "device (gdelta.hip)",
           "analysis": "CC over {y,m,w,d,h} + PageRank(20, hour) at the live time, every tick"}
    if rank == 0:
        print(json.dumps(out), flush=True)
    g.close()
    if dist is not None:
        dist.destroy_process_group()


def run_c5_loopback(a):
    """The C5 tick on P loopback partitions of one GPU (the partitioned live merge + CC + PR at P
    ranks), one partition's GPU work at a time (RGPU_LOOPBACK_ISOLATE=1), every kernel timed: per
    tick and partition the merge's wall time and the analyses' serial kernel ms.  The slowest
    partition per tick is what P GPUs would each do."""
    os.environ["RGPU_LOOPBACK_ISOLATE"] = "1"
    from raphtory_amd.partitioned import LoopbackPartitions
    from raphtory_amd.synth import BATCH_WINDOWS, HOUR, gen_gab_range
    P = a.c5_loopback
    lp = LoopbackPartitions(P, vertex_order="id")
    for p, g in enumerate(lp.parts):
        g.ingest_stream(gen_gab_range(4, a.c5_users, a.c5_base, 0, a.c5_base, p, P))
    lp.seal()
    now = max(g.newest_time() for g in lp.parts)
    recs = []
    for i in range(a.c5_ticks):
        d = [gen_gab_range(100 + i, a.c5_users, a.c5_tick, 0, a.c5_tick, p, P, t0=now + 1, t1=now + HOUR, id_key=4)
             for p in range(P)]
        now += HOUR
        merge = [0.0] * P
        for p, g in enumerate(lp.parts):  # one partition at a time: its own merge time
            t = time.perf_counter()
            g.ingest_stream(d[p])
            g.seal()
            merge[p] = (time.perf_counter() - t) * 1e3
        live = min(g.newest_time() for g in lp.parts)
        lp.run("cc", [live], BATCH_WINDOWS, profile=True, serial=True)
        cc = [sum(v["ms"] for v in g.stats()["kernels"].values()) for g in lp.parts]
        lp.run("pagerank", [live], [HOUR], pr_iters=20, profile=True, serial=True)
        pr = [sum(v["ms"] for v in g.stats()["kernels"].values()) for g in lp.parts]
        tot = [m + x + y for m, x, y in zip(merge, cc, pr)]
        recs.append({"merge_ms": [round(x, 1) for x in merge], "cc_kernel_ms": [round(x, 1) for x in cc],
                     "pr_kernel_ms": [round(x, 1) for x in pr], "slowest_partition_ms": round(max(tot), 1)})
        log(f"loopback tick {i}: slowest partition {max(tot):.1f} ms (merge {max(merge):.1f}, cc {max(cc):.1f}, "
            f"pr {max(pr):.1f})")
    upd = 3 * a.c5_tick
    slow = sum(r["slowest_partition_ms"] for r in recs) / len(recs)
    out = {"config": "C5", "rehearsal": f"{P} loopback partitions on one GPU, one at a time (RGPU_LOOPBACK_ISOLATE)",
           "base_updates": 3 * a.c5_base, "ticks": len(recs), "updates_per_tick": upd,
           "slowest_partition_tick_ms_mean": round(slow, 1),
           "modelled_updates_per_s_at_P_gpus": upd / (slow / 1e3),
           "model": "per tick the slowest partition's merge wall + CC + PR serial kernel ms (no overlap, no "
                    "exchange transfer time)", "ticks_ms": recs}
    print(json.dumps(out), flush=True)
    lp.close()


def run_c2(a, rank, world, local, quiet=False):
    """BASELINE configs[1] (C2): the RandomSpout-shaped 1M-update stream, 8,041 hourly hops x
    {y,m,w,d,h}, CC.  N > 1: replicas (every rank holds the 30 MB graph and runs the grid offset
    by r*jump/N: "weak").  quiet: return the line as the headline's secondary object."""
    import torch
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    from raphtory_amd import TemporalGraph
    from raphtory_amd.replicas import max_over_ranks, replica_hops
    from raphtory_amd.synth import BATCH_WINDOWS, DAY, HOUR, T0_README, gen_uniform, range_hops

    stream = gen_uniform(1, 100_000, 1_000_000)
    jump = HOUR
    base = range_hops(T0_README + 30 * DAY, T0_README + 365 * DAY, jump)
    hops = replica_hops(base, jump, rank, world)  # replica r runs the grid offset by r*jump/N
    windows = BATCH_WINDOWS

    g = TemporalGraph(device=local)
    g.ingest_stream(stream)
    t_seal = time.perf_counter()
    g.seal()
    seal_s = time.perf_counter() - t_seal
    st = g.stats()
    n_edges = st["edges"]

    def barrier():
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()

    steps, warmup = (max(a.steps, 5), max(a.warmup, 2)) if quiet else (a.steps, a.warmup)
    profile_only = a.profile_only and not quiet
    for _ in range(0 if profile_only else warmup):
        g.run("cc", hops, windows)
    barrier()
    t0 = time.perf_counter()
    for _ in range(0 if profile_only else steps):
        g.run("cc", hops, windows)
    barrier()
    elapsed = time.perf_counter() - t0
    elapsed = max_over_ranks(elapsed, dist, device="cuda")
    ms_per_step = elapsed * 1e3 / steps
    units = n_edges * len(windows) * len(hops) * world
    value = units / (ms_per_step / 1e3)
    if profile_only:  # no timed steps: report the kernel profile only
        ms_per_step = value = None

    # per-kernel timing (HIP events on the library's streams) over one more pass
    roofline = None
    kstats = {}
    s8d = None
    lean_only = a.lean_pass_only and not quiet
    if not a.no_profile_pass:
        kraw = profile_passes(g, hops, windows, lean_only=lean_only)
        kstats = kernel_table({"kernels": kraw})
        d = kraw["cc_step"]
        gbs = d["bytes"] / (d["ms"] / 1e3) / 1e9
        traffic, tsrc = pmc_traffic("k_cc_step_pk")
        roofline = {"bound": "hbm", "kernel": "cc_step (k_cc_step_pk)", "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS,
                    "unit": "GB/s", "frac": round(gbs / HBM_PEAK_GBS, 4), "traffic": traffic,
                    "traffic_source": tsrc, "avg_launch_us": round(d["ms"] * 1e3 / d["launches"], 2),
                    "algorithmic_bytes_per_launch": d["bytes"] / d["launches"]}
        if traffic:
            roofline["traffic_rate_GBps"] = round(traffic / (d["ms"] / d["launches"] / 1e3) / 1e9, 1)
            if d["bytes"] > 0:
                roofline["traffic_over_algorithmic"] = round(traffic / (d["bytes"] / d["launches"]), 2)
        if not lean_only:
            roofline["aggregate"] = aggregate_roofline(kraw, "C2")
        if not a.no_edge_counts and not lean_only:
            g.run("cc", hops, windows, edge_counts=True)
            s8d = survey_bytes(g.cc_summaries(), len(hops), windows, st["vertices"], st["edges"],
                               st["vertex_events"] + st["edge_events"] + st["deaths"], kstats, d["launches"])
            roofline["survey_8d"] = {"achieved": round(s8d["cc_step"]["achieved_GBps"], 1),
                                     "frac": round(s8d["cc_step"]["achieved_GBps"] / HBM_PEAK_GBS, 4),
                                     "bytes_per_launch": s8d["cc_step"]["bytes_per_launch"]}

    summ = g.cc_summaries()
    drop_in = setup_latency(g, hops, windows) if rank == 0 and not profile_only else None
    cpu = None
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        cpu = cpu_baseline(stream, hops, windows, a.cpu_seconds, n_edges,
                           "the same C2 stream and query")

    out = None
    if rank == 0:
        out = {
            "metric": "temporal edge-windows processed/sec for batched-window CC range query",
            "value": round(value, 1) if value is not None else None,
            "unit": "edge-windows/s",
            "n_gpus": world,
            "steps": steps,
            "warmup": warmup,
            "ms_per_step": round(ms_per_step, 3) if ms_per_step is not None else None,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "int32",
            "data": "synthetic (seeded RandomSpout-shaped stream, SURVEY.md App. B)",
            "config": {"workload": "C2: 100k vertices, 1M updates, 8041 hourly hops x 5 batched windows "
                                   "{y,m,w,d,h}, ConnectedComponents",
                       "edge_entities": n_edges, "hops_per_gpu": int(len(hops)), "windows": len(windows),
                       "parallelism": f"replicas x{world} (hop grid sharded, no exchange)",
                       "seal_s": round(seal_s, 3),
                       "supersteps_per_view_mean": round(float(summ[..., 7].mean()), 2),
                       "alive_edge_windows": s8d["alive_edge_windows"] if s8d else None,
                       "alive_edge_windows_frac": (s8d["alive_edge_windows"] / (n_edges * len(windows) * len(hops)))
                                                  if s8d else None},
            "roofline": roofline,
            "survey_8d_bytes": s8d,
            "cpu_baseline": cpu,
            "kernels": kstats,
            "drop_in_per_setup": drop_in,
            "check": {"views": int(summ.shape[0] * summ.shape[1]),
                      "sum_biggest": int(summ[..., 0].sum()), "sum_total": int(summ[..., 1].sum())},
        }
        if not quiet:
            print(json.dumps(out))
    g.close()
    if dist is not None:
        dist.destroy_process_group()
    return out


def main():
    a = parse()
    heartbeat()
    rank, world, local = dist_env()
    import torch
    if a.exchange == "shm":  # one-host rehearsal: ranks share the visible GPUs (device_count: no HIP init)
        local %= max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    run = {"c2": run_c2, "c3": run_c3, "c4": run_c4, "c5": run_c5, "diffusion": run_diffusion}[a.config]
    run(a, rank, world, local)


if __name__ == "__main__":
    main()
