#!/usr/bin/env python3
"""Benchmark: temporal edge-windows processed/sec for a batched-window CC Range query.

Workload (BASELINE.json configs[1], "C2"): seeded RandomSpout-shaped stream, 100k vertices,
1M updates (30/40/10/20 % VADD/EADD/VDEL/EDEL) over one year; Range query from T0+30d to
T0+365d hopping 1 h (8,041 hops) with batched windows {year, month, week, day, hour}, CC
(ConnectedComponents, 100-superstep cap) on one MI355X.

  edge-windows = N_E x |windows| x |hops|   (N_E = directed edge entities)

One "step" = one complete Range query (every hop x window: window filter, CSR compaction, CC
supersteps, component-size reductions).  The packed graph is resident in HBM before timing.

Multi-GPU (python -m torch.distributed.run --nproc-per-node N bench.py --gpus N): replicas —
every rank holds the whole graph and runs its own share of a finer hop grid (rank r's hops
are offset by r*jump/N), so per-GPU work is fixed and there is no data-path collective
("scaling": "weak").  Timing: barrier + synchronize on both sides, max over ranks.
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
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
                   help="only the serial HIP-event profile pass (the command rocprofv3 is run on, so "
                        "that its per-kernel averages match the roofline figures)")
    p.add_argument("--config", default="c2", choices=["c2", "c3", "c4", "c5", "diffusion"],
                   help="c2 = the headline metric; diffusion = BinaryDefusion over the C2 query (secondary)")
    p.add_argument("--diff-seed", type=int, default=31,
                   help="diffusion infectedNode (BinaryDefusion.scala:10); -1 = the vertex with most EADDs as source")
    p.add_argument("--c5-users", type=int, default=20_000_000)
    p.add_argument("--c5-base", type=int, default=33_333_334, help="sealed base interactions (x3 updates)")
    p.add_argument("--c5-tick", type=int, default=3_333_334, help="interactions streamed per hour tick (x3 updates)")
    p.add_argument("--c5-ticks", type=int, default=6)
    p.add_argument("--c3-vertices", type=int, default=10_000_000)
    p.add_argument("--c3-events", type=int, default=100_000_000)
    p.add_argument("--c4-users", type=int, default=20_000_000)
    p.add_argument("--c4-interactions", type=int, default=333_333_334, help="x3 updates (1B at the default)")
    p.add_argument("--c4-hops", type=int, default=168)
    return p.parse_args()


def dist_env():
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    return rank, world, local


def pmc_traffic(kernel):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 PMC passes
    (tools/gpu_profile.sh -> profiles/latest_pmc.json), or None."""
    path = os.path.join(ROOT, "profiles", "latest_pmc.json")
    try:
        with open(path) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None, None
    if kernel not in d.get("FETCH_SIZE", {}).get("kernel", ""):
        return None, None
    return round(d["traffic_bytes_per_launch"]["value"]), "profiles/latest_pmc.json: " + d["traffic_bytes_per_launch"]["formula"]


def cpu_baseline(stream, hops, windows, budget_s, n_edges):
    """The oracle in reference structure (mode 0: lens rebuilt by linear closestTime scans every
    superstep, adjacency re-filtered on every visit), single thread, on a bounded prefix of
    the same hop list."""
    from oracle import Oracle
    o = Oracle.from_stream(stream)
    done, t0 = 0, time.perf_counter()
    for t in hops.tolist():
        o.cc(int(t), windows, max_steps=100, mode=0)
        done += 1
        if time.perf_counter() - t0 > budget_s:
            break
    dt = time.perf_counter() - t0
    return {
        "value": n_edges * len(windows) * done / dt,
        "unit": "edge-windows/s",
        "cores": 1,
        "kind": "port",
        "sample": f"first {done} of {len(hops)} hops x {len(windows)} windows of the same C2 query, "
                  f"oracle refsim mode (reference algorithmic structure), {dt:.1f} s, 1 thread",
    }


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


def log(msg):
    print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def run_c4(a, rank, world, local):
    """BASELINE configs[3] (C4): GAB-shaped add-only stream — (VADD s, VADD d, EADD s->d) triples
    at one t (GabUserGraphRouter.scala:31-33) — 20M users, 333M interactions = 1B updates,
    2016-08-10 -> 2018-05-31; batched windows {y,m,w,d,h}, hourly hops, the last 168 hops; CC.
    N = 1: one graph.  N > 1: vertex-partitioned (Utils.getPartition), one partition per GPU,
    boundary label rows exchanged over RCCL every superstep; every rank
    generates the same seeded stream and keeps what its partition needs.  Secondary line."""
    import torch
    from raphtory_amd import TemporalGraph
    from raphtory_amd.synth import BATCH_WINDOWS, HOUR, gen_gab, range_hops
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("gloo")  # control plane; the data path is the library's RCCL
    t0 = time.perf_counter()
    s = gen_gab(4, a.c4_users, a.c4_interactions)
    gen_s = time.perf_counter() - t0
    log(f"C4 stream: {len(s)} updates generated in {gen_s:.1f} s")
    if dist is not None:
        from raphtory_amd.partitioned import open_rccl_partition
        g = open_rccl_partition(local, dist)
    else:
        g = TemporalGraph(device=local)
    g.ingest_stream(s)
    end = int(s.t[-1])
    n_up = len(s)
    del s
    t0 = time.perf_counter()
    g.seal()
    seal_s = time.perf_counter() - t0
    st = g.stats()
    log(f"sealed in {seal_s:.1f} s: {st['vertices']} vertices, {st['edges']} edge entities")
    hops = range_hops(end - (a.c4_hops - 1) * HOUR, end, HOUR)
    windows = BATCH_WINDOWS
    g.run("cc", hops, windows)  # warm-up
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        g.run("cc", hops, windows)
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    ms = (time.perf_counter() - t0) * 1e3 / a.steps
    if dist is not None:
        from raphtory_amd.replicas import max_over_ranks
        ms = max_over_ranks(ms, dist)
    log(f"query {ms:.1f} ms")
    g.run("cc", hops, windows, profile=True, serial=True)
    ks = {k: v for k, v in g.stats()["kernels"].items() if v["launches"]}
    summ = g.cc_summaries()
    out = {"config": "C4", "n_gpus": world, "updates": n_up, "vertices": st["vertices"], "edge_entities": st["edges"],
           "vertex_events": st["vertex_events"], "edge_events": st["edge_events"], "gen_s": round(gen_s, 1),
           "seal_s": round(seal_s, 1), "hops": len(hops), "windows": len(windows), "ms_per_query": round(ms, 2),
           "edge_windows_per_s": st["edges"] * len(windows) * len(hops) / (ms / 1e3) if world == 1 else None,
           "supersteps_per_batch_mean": round(g.stats()["supersteps"] / max(1, g.stats()["batches"]), 2),
           "kernels": {k: {"launches": v["launches"], "ms": round(v["ms"], 3), "avg_us": round(v["ms"] * 1e3 / v["launches"], 2),
                           "GBps": round(v["bytes"] / max(v["ms"], 1e-9) / 1e6, 1)} for k, v in ks.items()},
           "check": {"sum_biggest": int(summ[..., 0].sum()), "sum_total": int(summ[..., 1].sum()),
                     "sum_members": int(summ[..., 5].sum())}}
    if rank == 0:
        print(json.dumps(out), flush=True)
    g.close()
    if dist is not None:
        dist.destroy_process_group()


def run_c5(a, rank, world, local):
    """BASELINE configs[4] (C5), one GPU: live analysis under ingest.  A GAB-shaped base
    (default 100M updates, 20M users) is sealed once; then every hour tick the Router's next
    10M updates (one hour of stream time past the newest point) are ingested and merged into
    the HBM-resident graph by the incremental seal (merge.hip), and CC (batched windows
    {y,m,w,d,h}) and PageRank (20 iterations, hour window) are re-run on the newest hour, as
    LiveAnalysisTask does (LiveAnalysisTask.scala:13-107).  Reported: sustained updates/s over
    the whole loop (ingest + merge + both analyses), the merge alone, and per-tick latencies.
    Generating the updates (the Router's side) is outside the timed region.  Secondary line."""
    import torch
    from raphtory_amd import TemporalGraph
    from raphtory_amd.synth import BATCH_WINDOWS, HOUR, gen_gab
    s = gen_gab(4, a.c5_users, a.c5_base)
    g = TemporalGraph(device=local)
    g.ingest_stream(s)
    t0 = time.perf_counter()
    g.seal()
    base_seal_s = time.perf_counter() - t0
    now = int(s.t[-1])
    n_base = len(s)
    del s
    log(f"C5 base: {n_base} updates sealed in {base_seal_s:.1f} s")
    ticks = []
    for i in range(a.c5_ticks + 1):  # tick 0 is warm-up
        d = gen_gab(100 + i, a.c5_users, a.c5_tick, t0=now + 1, t1=now + HOUR, id_key=4)
        now = int(d.t[-1])
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        g.ingest_stream(d)
        t1 = time.perf_counter()
        g.seal()
        t2 = time.perf_counter()
        g.run("cc", [now], BATCH_WINDOWS)
        t3 = time.perf_counter()
        g.run("pagerank", [now], [HOUR], pr_iters=20)
        torch.cuda.synchronize()
        t4 = time.perf_counter()
        st = g.stats()
        assert st["seal_incremental"] == 1
        ticks.append({"updates": len(d), "ingest_ms": (t1 - t0) * 1e3, "merge_ms": (t2 - t1) * 1e3,
                      "cc_ms": (t3 - t2) * 1e3, "pr_ms": (t4 - t3) * 1e3, "total_ms": (t4 - t0) * 1e3,
                      "vertices": st["vertices"], "edges": st["edges"]})
        log(f"tick {i}: " + " ".join(f"{k}={v:.1f}" if isinstance(v, float) else f"{k}={v}"
                                     for k, v in ticks[-1].items()))
    tt = ticks[1:]
    up = sum(t["updates"] for t in tt)
    wall = sum(t["total_ms"] for t in tt) / 1e3
    merge = sum(t["ingest_ms"] + t["merge_ms"] for t in tt) / 1e3
    out = {"config": "C5", "n_gpus": 1, "base_updates": n_base, "base_seal_s": round(base_seal_s, 1),
           "ticks": len(tt), "updates_per_tick": tt[0]["updates"] if tt else 0,
           "live_updates_per_s": up / wall if wall else None,
           "ingest_merge_updates_per_s": up / merge if merge else None,
           "mean_ms": {k: round(sum(t[k] for t in tt) / len(tt), 1)
                       for k in ("ingest_ms", "merge_ms", "cc_ms", "pr_ms", "total_ms")},
           "final_vertices": tt[-1]["vertices"] if tt else None, "final_edges": tt[-1]["edges"] if tt else None,
           "analysis": "CC over {y,m,w,d,h} + PageRank(20, hour) on the newest hour, every tick"}
    print(json.dumps(out), flush=True)
    g.close()


def main():
    a = parse()
    if a.config == "c4":
        rank, world, local = dist_env()
        import torch
        torch.cuda.set_device(local)
        return run_c4(a, rank, world, local)
    if a.config == "c5":
        rank, world, local = dist_env()
        import torch
        torch.cuda.set_device(local)
        return run_c5(a, rank, world, local)
    if a.config == "diffusion":
        rank, world, local = dist_env()
        import torch
        torch.cuda.set_device(local)
        return run_diffusion(a, rank, world, local)
    if a.config == "c3":
        rank, world, local = dist_env()
        import torch
        torch.cuda.set_device(local)
        return run_c3(a, rank, world, local)
    rank, world, local = dist_env()
    import torch
    torch.cuda.set_device(local)
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

    if a.profile_only:
        a.steps, a.warmup, a.no_cpu_baseline = 1, 0, True
    for _ in range(a.warmup):
        g.run("cc", hops, windows)
    barrier()
    t0 = time.perf_counter()
    for _ in range(0 if a.profile_only else a.steps):
        g.run("cc", hops, windows)
    barrier()
    elapsed = time.perf_counter() - t0
    elapsed = max_over_ranks(elapsed, dist, device="cuda")
    ms_per_step = elapsed * 1e3 / a.steps
    units = n_edges * len(windows) * len(hops) * world
    value = units / (ms_per_step / 1e3)
    if a.profile_only:  # no timed steps: report the kernel profile only
        ms_per_step = value = None

    # per-kernel timing (HIP events on the library's streams) over one more pass
    roofline = None
    kstats = {}
    if not a.no_profile_pass:
        g.run("cc", hops, windows, profile=True, serial=True)
        ks = g.stats()["kernels"]
        kstats = {k: v for k, v in ks.items() if v["launches"]}
        dom = max(kstats, key=lambda k: kstats[k]["ms"])
        d = kstats[dom]
        gbs = d["bytes"] / (d["ms"] / 1e3) / 1e9
        traffic, tsrc = pmc_traffic(dom)
        roofline = {"bound": "hbm", "kernel": dom, "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS,
                    "unit": "GB/s", "frac": round(gbs / HBM_PEAK_GBS, 4), "traffic": traffic,
                    "traffic_source": tsrc,
                    "avg_launch_us": round(d["ms"] * 1e3 / d["launches"], 2),
                    "algorithmic_bytes_per_launch": d["bytes"] / d["launches"]}

    summ = g.cc_summaries()
    cpu = None
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        cpu = cpu_baseline(stream, hops, windows, a.cpu_seconds, n_edges)

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
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "int32",
            "data": "synthetic (seeded RandomSpout-shaped stream, SURVEY.md App. B)",
            "config": {"workload": "C2: 100k vertices, 1M updates, 8041 hourly hops x 5 batched windows "
                                   "{y,m,w,d,h}, ConnectedComponents",
                       "edge_entities": n_edges, "hops_per_gpu": int(len(hops)), "windows": len(windows),
                       "parallelism": f"replicas x{world} (hop grid sharded, no exchange)",
                       "seal_s": round(seal_s, 3),
                       "supersteps_per_batch_mean": round(g.stats()["supersteps"] / max(1, g.stats()["batches"]), 2),
                       "alive_edge_windows_frac": None},
            "roofline": roofline,
            "cpu_baseline": cpu,
            "kernels": {k: {"launches": v["launches"], "ms": round(v["ms"], 3),
                            "GBps": round(v["bytes"] / max(v["ms"], 1e-9) / 1e6, 1)} for k, v in kstats.items()},
            "check": {"views": int(summ.shape[0] * summ.shape[1]),
                      "sum_biggest": int(summ[..., 0].sum()), "sum_total": int(summ[..., 1].sum())},
        }
        print(json.dumps(out))
    g.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
