"""One-GPU rehearsal of the vertex-partitioned C4 query: P partitions in one
process over the loopback exchange (LoopbackPartitions), P = 1..8, on a C4-shaped prefix of the
1B stream.  RGPU_LOOPBACK_ISOLATE=1 makes the partitions' GPU work between collectives run one
partition at a time, so the serial profile pass's kernel times are each partition's own: their
maximum is the compute one of P GPUs would do, their sum the partitioning's total work.  Also:
the bytes the partitions send each other per query (by kind) and the summaries' check sums
(identical at every P).  Prints one JSON line per P.

Round 5 (the model must carry the exchange's fixed per-superstep costs): before the
partitions, a P = 1 partitioned context on a real RCCL channel measures one superstep round's
fixed cost (rgpu_exchange_probe: counts all-to-all, the counts' copy to the host and the host's
wait, two grouped send/recv) and a 64-word all-reduce.  Each partition's model then adds, beside
its kernel ms and the xGMI bandwidth term, rounds x that round cost + batches x 2 all-reduces,
serialised (no overlap with the other batch slots: an upper bound on what they cost; the kernel
ms alone is the lower bound).  RCCL at P = 8 adds peer latency that one rank does not have; the
line reports the ratio at the measured cost and with an extra 25 / 50 us per round."""
import argparse
import hashlib
import json
import os
import sys
import time

import numpy as np

os.environ.setdefault("RGPU_LOOPBACK_ISOLATE", "1")

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from raphtory_amd import TemporalGraph  # noqa: E402
from raphtory_amd.partitioned import LoopbackPartitions, combine_window_groups, hop_blocks  # noqa: E402
from raphtory_amd.synth import BATCH_WINDOWS, HOUR, gen_gab_range, range_hops  # noqa: E402


class _Env:
    """library knobs set for a block of calls ('K=V[,K=V]'): rgpu_open and each run read them"""

    def __init__(self, spec: str):
        self.kv = dict(x.split("=", 1) for x in spec.split(",") if x.strip())

    def __enter__(self):
        self.old = {k: os.environ.get(k) for k in self.kv}
        os.environ.update(self.kv)

    def __exit__(self, *exc):
        for k, v in self.old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def open_replica(s, cut, env=""):
    """the --hybrid time-slice replica: the updates with t >= cut, one graph"""
    keep = s.t >= cut
    with _Env(env):
        replica = TemporalGraph()  # (rgpu_open reads the knobs)
    replica.ingest_stream(type(s)(s.t[keep], s.kind[keep], s.src[keep], s.dst[keep]))
    replica.seal()
    return replica, int(keep.sum())


def profile_blocks(replica, hops, sw, P, rounds, env=""):
    """rank r's block of the hops (hop_blocks), short windows, on the replica: serial kernel ms per
    block (best of `rounds` profile passes), kernel ms by group summed, and (lo, hi, summaries)"""
    blk_ms, blk_ks, got = [], {}, []
    with _Env(env):
        for lo, hi in hop_blocks(len(hops), P):
            blk = hops[lo:hi]
            replica.run("cc", blk, sw)
            bm, bk = None, None
            for _ in range(max(1, rounds)):
                replica.run("cc", blk, sw, profile=True, serial=True)
                kk = {k: v["ms"] for k, v in replica.stats()["kernels"].items() if v["launches"]}
                if bm is None or sum(kk.values()) < bm:
                    bm, bk = sum(kk.values()), kk
            blk_ms.append(round(bm, 1))
            for k, v in bk.items():
                blk_ks[k] = blk_ks.get(k, 0.0) + v
            got.append((lo, hi, replica.cc_summaries()))
    return blk_ms, blk_ks, got


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--users", type=int, default=20_000_000)
    ap.add_argument("--interactions", type=int, default=33_333_334, help="prefix of the 1B stream (x3 updates)")
    ap.add_argument("--parts", default="1,2,4,8")
    ap.add_argument("--trace", default="", help="directory: per-superstep trace CSVs (RGPU_TRACE) of the profile pass")
    ap.add_argument("--profile-rounds", type=int, default=2,
                    help="profile passes; the one with the smallest slowest-partition time is reported")
    ap.add_argument("--probe-rounds", type=int, default=500, help="rgpu_exchange_probe rounds (0: skip)")
    ap.add_argument("--ab", default="",
                    help="per-run knob settings to profile on the same sealed partitions after the main pass, "
                         "';'-separated, each 'K=V[,K=V]' (read per run by the library): one extra JSON line each")
    ap.add_argument("--hybrid", default="",
                    help="P > 1: these windows (letters of 'ymwdh', e.g. 'dh') run hop-sharded instead of partitioned: "
                         "rank r answers them for its block of the hops on a replica of the stream's time slice "
                         "[hop0 - the longest of them, end] (exact: a view (t, w) reads only updates in (t - w, t]); "
                         "the partitions run the other windows.  Per rank: its partition's kernel ms + its block's")
    ap.add_argument("--replica-env", default="",
                    help="--hybrid: 'K=V[,K=V]' library knobs set while the slice replica opens (A/B of its options)")
    ap.add_argument("--replica-ab", default="",
                    help="--hybrid: replica knob settings to compare (';'-separated 'K=V[,K=V]'): per P a fresh "
                         "replica per setting, its blocks profiled, one JSON line each")
    ap.add_argument("--replica-only", action="store_true",
                    help="--hybrid: profile only the replica's blocks per P (no partitions): quick replica A/B")
    a = ap.parse_args()
    probe = None
    if a.probe_rounds > 0:  # one RCCL rank: the fixed cost of a round without peer latency
        os.environ["RGPU_PARTITIONED"] = "1"
        gp = TemporalGraph()
        del os.environ["RGPU_PARTITIONED"]
        gp.exchange_init(TemporalGraph.exchange_id(kind="rccl"))
        probe = gp.exchange_probe(a.probe_rounds)
        gp.close()
        print(json.dumps({"exchange_probe_rccl_p1": probe}), flush=True)
    inter_full = 333_333_334
    s = gen_gab_range(4, a.users, inter_full, 0, a.interactions)
    end = int(s.t[-1])
    hops = range_hops(end - 167 * HOUR, end, HOUR)
    short_i = [i for i, c in enumerate("ymwdh") if c in a.hybrid]
    long_i = [i for i in range(len(BATCH_WINDOWS)) if i not in short_i]
    replica, replica_n = None, 0  # the time-slice replica (--hybrid), built at the first P > 1
    sw = [BATCH_WINDOWS[i] for i in short_i]
    cut = int(hops[0]) - max(sw) if short_i else 0
    if short_i and a.replica_only:
        for P in [int(x) for x in a.parts.split(",")]:
            for setting in [a.replica_env] + [x for x in a.replica_ab.split(";") if x.strip()]:
                rep, n = open_replica(s, cut, setting)
                blk_ms, blk_ks, _ = profile_blocks(rep, hops, sw, P, a.profile_rounds, setting)
                nv = rep.stats()["vertices"]
                rep.close()
                print(json.dumps({"P": P, "replica_only": "".join("ymwdh"[i] for i in short_i), "replica_env": setting,
                                  "replica_updates": n, "replica_vertices": nv, "replica_block_kernel_ms": blk_ms,
                                  "replica_block_kernel_ms_max": max(blk_ms),
                                  "replica_kernel_ms_sum_by_kernel": {k: round(v, 1) for k, v in blk_ks.items()}}),
                      flush=True)
        return
    for P in [int(x) for x in a.parts.split(",")]:
        t0 = time.time()
        if a.trace:  # read when a context opens; a partition's file gets ".p<partition>"
            os.makedirs(a.trace, exist_ok=True)
            os.environ["RGPU_TRACE"] = os.path.join(a.trace, f"trace_P{P}.csv")
        print(f"P={P}: packing", file=sys.stderr, flush=True)
        if P == 1:
            g = TemporalGraph()
            g.ingest_stream(s)
            g.seal()
            parts = [g]
            run = lambda **kw: g.run("cc", hops, BATCH_WINDOWS, **kw)  # noqa: E731
        else:
            lp = LoopbackPartitions(P)
            lp.ingest_stream(s)
            lp.seal()
            parts = lp.parts
            pw = [BATCH_WINDOWS[i] for i in long_i] if short_i else BATCH_WINDOWS
            run = lambda **kw: lp.run("cc", hops, pw, **kw)  # noqa: E731
            if short_i and replica is None:
                replica, replica_n = open_replica(s, cut, a.replica_env)
                print(f"hybrid: slice replica of {replica_n} updates (t >= hop0 - {max(sw)} ms)", file=sys.stderr,
                      flush=True)
        print(f"P={P}: sealed in {time.time() - t0:.0f} s", file=sys.stderr, flush=True)
        run()
        print(f"P={P}: warm run done", file=sys.stderr, flush=True)
        best = None
        for _ in range(max(1, a.profile_rounds)):
            t_prof = time.time()
            run(profile=True, serial=True)
            t_prof = time.time() - t_prof
            per = []
            ks = {}
            for g in parts:
                mine = 0.0
                for k, v in g.stats()["kernels"].items():
                    if v["launches"]:
                        ks[k] = ks.get(k, 0.0) + v["ms"]
                        mine += v["ms"]
                per.append(round(mine, 1))
            p0 = {k: [v["launches"], round(v["ms"], 2)] for k, v in parts[0].stats()["kernels"].items() if v["launches"]}
            if best is None or max(per) < max(best[0]):
                best = (per, ks, p0, t_prof)
        per, ks, p0, t_prof = best
        hyb = None
        summ = parts[0].cc_summaries()
        if short_i and P > 1:
            # rank r's block of the hops, short windows, on the slice replica: profile each block (best of
            # the profile rounds) and assemble the whole query's summaries for the check
            blk_ms, blk_ks, got = profile_blocks(replica, hops, sw, P, a.profile_rounds, a.replica_env)
            long_summ = summ
            summ = combine_window_groups(len(BATCH_WINDOWS), long_i, summ, short_i, got)
            for setting in [x for x in a.replica_ab.split(";") if x.strip()]:  # same partitions, other replicas
                rep, _ = open_replica(s, cut, setting)
                bms, bks, bgot = profile_blocks(rep, hops, sw, P, a.profile_rounds, setting)
                rep.close()
                same = np.array_equal(combine_window_groups(len(BATCH_WINDOWS), long_i, long_summ, short_i, bgot), summ)
                print(json.dumps({"P": P, "replica_ab": setting, "replica_block_kernel_ms": bms,
                                  "slowest_rank_ms": max(x + y for x, y in zip(per, bms)), "summaries_equal": bool(same),
                                  "replica_kernel_ms_sum_by_kernel": {k: round(v, 1) for k, v in bks.items()}}),
                      flush=True)
            hyb = {"windows_replicated": "".join("ymwdh"[i] for i in short_i), "replica_env": a.replica_env,
                   "replica_updates": replica_n,
                   "partition_kernel_ms": per, "replica_block_kernel_ms": blk_ms,
                   "replica_kernel_ms_sum_by_kernel": {k: round(v, 1) for k, v in blk_ks.items()}}
            per = [round(x + y, 1) for x, y in zip(per, blk_ms)]
            for k, v in blk_ks.items():
                ks[k] = ks.get(k, 0.0) + v
        by = {}
        for g in parts:
            for k, v in g.stats()["xchg_bytes_by"].items():
                by[k] = by.get(k, 0.0) + v / 1e6
        # modelled exchange time per partition: the bytes it sends, spread over its P-1 xGMI links
        # (point-to-point, ~153 GB/s each per the MI355X platform figures in the task brief) — a
        # bandwidth term only; the number of exchange rounds (one per superstep per batch, plus one
        # membership and one counts round per batch) is reported beside it
        link = 153e9
        xms = [(g.stats()["xchg_bytes"] / max(1, P - 1)) / link * 1e3 if P > 1 else 0.0 for g in parts]
        tot = [round(k + x, 1) for k, x in zip(per, xms)]
        st0 = parts[0].stats()
        rounds = st0["supersteps"] + 2 * st0["batches"]
        fixed = {}
        if probe is not None and P > 1:
            for extra in (0, 25, 50):
                f_ms = (rounds * (probe["round_us_median"] + extra) + 2 * st0["batches"] * probe["allreduce_us_median"]) / 1e3
                fixed[f"+{extra}us_per_round"] = round(f_ms, 1)
        out = {"P": P, "kernel_ms_per_partition": per, "kernel_ms_max": max(per), "kernel_ms_total": round(sum(per), 1),
               "kernel_ms_sum_by_kernel": {k: round(v, 1) for k, v in ks.items()},
               "partition0_kernels": p0, "profile_rounds": a.profile_rounds,
               # algorithmic bytes (the counting pass's work counters) summed over the
               # partitions: more bytes than at P = 1 = more work, not slower work
               "kernel_GB_sum_by_kernel": {k: round(sum(g.stats()["kernels"][k].get("bytes", 0.0) for g in parts) / 1e9, 2)
                                           for k in ks},
               "xchg_MB_per_query": {k: round(v, 1) for k, v in by.items()},
               "xchg_model_ms_per_partition": [round(x, 2) for x in xms], "xchg_link_GBps": link / 1e9,
               "xchg_rounds_per_partition": rounds,
               "kernel_plus_xchg_ms_max": max(tot),
               # the fixed per-round cost serialised on top (rgpu_exchange_probe, RCCL, one rank), per
               # partition; the model = kernel ms + bandwidth term + this
               "fixed_round_ms": fixed,
               "model_ms_max_with_fixed": {k: round(max(tot) + v, 1) for k, v in fixed.items()},
               # the serial profiled run's wall time over P: one partition's share of everything the
               # timers above leave out too (exchange pack / unpack / mark kernels, host turns)
               "serial_wall_ms_per_partition": round(t_prof * 1e3 / P, 1),
               "vertices_here": [g.stats()["vertices"] for g in parts], "edges_here": [g.stats()["edges"] for g in parts],
               "check": [int(summ[..., 0].sum()), int(summ[..., 1].sum()), int(summ[..., 5].sum())],
               # every view's summary fields (biggest .. supersteps), hashed: equal at every P
               "summaries_sha256": hashlib.sha256(np.ascontiguousarray(summ[..., :8]).tobytes()).hexdigest()[:16]}
        if hyb:
            out["hybrid"] = hyb
        print(json.dumps(out), flush=True)
        if short_i and P == 1:  # the hybrid on one GPU: long windows on the graph + every hop on the replica
            if replica is None:
                replica, replica_n = open_replica(s, cut, a.replica_env)
            lw = [BATCH_WINDOWS[i] for i in long_i]
            g.run("cc", hops, lw)
            g.run("cc", hops, lw, profile=True, serial=True)
            lks = {k: v["ms"] for k, v in g.stats()["kernels"].items() if v["launches"]}
            bms, bks, bgot = profile_blocks(replica, hops, sw, 1, a.profile_rounds, a.replica_env)
            same = np.array_equal(combine_window_groups(len(BATCH_WINDOWS), long_i, g.cc_summaries(), short_i, bgot), summ)
            print(json.dumps({"P": 1, "hybrid_p1": "".join("ymwdh"[i] for i in short_i),
                              "kernel_ms": round(sum(lks.values()) + bms[0], 1), "graph_kernel_ms": round(sum(lks.values()), 1),
                              "replica_kernel_ms": bms[0], "summaries_equal": bool(same),
                              "graph_kernel_ms_by_kernel": {k: round(v, 1) for k, v in lks.items()},
                              "replica_kernel_ms_by_kernel": {k: round(v, 1) for k, v in bks.items()}}), flush=True)
        for setting in [x for x in a.ab.split(";") if x.strip()]:  # same-process A/B on these partitions
            kv = dict(x.split("=", 1) for x in setting.split(","))
            old = {k: os.environ.get(k) for k in kv}
            os.environ.update(kv)
            try:
                run(profile=True, serial=True)
            finally:
                for k, v in old.items():
                    if v is None:
                        os.environ.pop(k, None)
                    else:
                        os.environ[k] = v
            per, ks = [], {}
            for g in parts:
                mine = 0.0
                for k, v in g.stats()["kernels"].items():
                    if v["launches"]:
                        ks[k] = ks.get(k, 0.0) + v["ms"]
                        mine += v["ms"]
                per.append(round(mine, 1))
            summ = parts[0].cc_summaries()
            print(json.dumps({"P": P, "ab": setting, "kernel_ms_per_partition": per, "kernel_ms_max": max(per),
                              "kernel_ms_total": round(sum(per), 1),
                              "kernel_ms_sum_by_kernel": {k: round(v, 1) for k, v in ks.items()},
                              "check": [int(summ[..., 0].sum()), int(summ[..., 1].sum()), int(summ[..., 5].sum())]}),
                  flush=True)
        for g in parts:
            g.close()
    if replica is not None:
        replica.close()


if __name__ == "__main__":
    main()
