"""Summarise rocprofv3 PMC passes (FETCH_SIZE and WRITE_SIZE, one counter per pass, no tracing) of
the serial lean profile pass, per kernel group of the bench's roofline.

usage: python tools/pmc_summary.py <fetch_dir> <write_dir> <out.json>

Groups (rgpu_stats kernel groups): cc_step = k_cc_step_pk, cc_slots = k_cc_slots,
heavy = k_heavy_slots / k_heavy_gather / k_heavy_mark, window_mask = k_vertex_mask, edge_mask =
k_edge_mask, cc_hist = k_cc_count, cc_summary = k_cc_roots.  Only the lean instantiations (the
PROF template flag false: what the timed query launches) are pooled, as for the dominant kernel.
Traffic per launch = 2 * FETCH_SIZE * 1024 + WRITE_SIZE * 1024 (MI355X_MICROARCH.md HBM section:
gfx950 FETCH_SIZE counts half of a wide read; narrow 4/8-B gathers are uncalibrated; Infinity-Cache
hits are counted).  The top level keeps the dominant kernel's record in the format bench.py's
pmc_traffic reads; "by_group" holds every group."""
import csv
import glob
import json
import sys

GROUPS = {
    "cc_step": ("k_cc_step_pk",),
    "cc_slots": ("k_cc_slots",),
    "heavy": ("k_heavy_slots", "k_heavy_gather", "k_heavy_mark"),
    "window_mask": ("k_vertex_mask",),
    "edge_mask": ("k_edge_mask",),
    "cc_hist": ("k_cc_count",),
    "cc_summary": ("k_cc_roots",),
}
FORMULA = ("2*FETCH_SIZE*1024 + WRITE_SIZE*1024 (MI355X_MICROARCH.md HBM section: gfx950 FETCH_SIZE counts "
           "half of a wide read; narrow 4/8-B gathers are uncalibrated; Infinity-Cache hits are counted)")


def base_name(kname):
    return kname.split("(")[0].replace("void ", "").strip()


def lean(name):
    """the PROF template flag (second argument of k_cc_step_pk, first of k_cc_slots / k_heavy_*
    have none): false = the lean instantiation the timed run launches"""
    if "k_cc_step_pk" in name:
        a = name[name.find("<") + 1:name.rfind(">")].split(",")
        return len(a) < 2 or a[1].strip() == "false"
    if "k_cc_slots" in name:
        a = name[name.find("<") + 1:name.rfind(">")].split(",")
        return a[0].strip() == "false"
    return True


def group_of(name):
    for g, pats in GROUPS.items():
        if any(p in name for p in pats):
            return g
    return None


def read(d, ctr):
    rows = {}
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if r.get("Counter_Name") != ctr:
                continue
            n = base_name(r.get("Kernel_Name", ""))
            vals = rows.setdefault(n, [])
            vals.append(float(r["Counter_Value"]))
    return rows


def summarise(fetch_dir, write_dir):
    fe, wr = read(fetch_dir, "FETCH_SIZE"), read(write_dir, "WRITE_SIZE")
    by = {}
    for g in GROUPS:
        names = sorted(n for n in fe if group_of(n) == g and lean(n))
        if not names:
            continue
        fv = [x for n in names for x in fe[n]]
        wv = [x for n in names for x in wr.get(n, [])]
        if not wv:
            continue
        by[g] = {"kernels": names, "dispatches": len(fv),
                 "fetch_kb_total": sum(fv), "write_kb_total": sum(wv),
                 "traffic_bytes_total": 2 * sum(fv) * 1024 + sum(wv) * 1024,
                 "traffic_bytes_per_launch": (2 * sum(fv) * 1024 + sum(wv) * 1024) / len(fv),
                 "per_kernel": {n: len(fe[n]) for n in names}}
    out = {"by_group": by, "formula": FORMULA}
    if "cc_step" in by:  # the dominant kernel, in the format bench.py pmc_traffic reads
        d = by["cc_step"]
        kern = " + ".join(d["kernels"])
        out["FETCH_SIZE"] = {"kernel": kern, "dispatches": d["dispatches"],
                             "mean_kb_per_dispatch": d["fetch_kb_total"] / d["dispatches"], "total_kb": d["fetch_kb_total"]}
        out["WRITE_SIZE"] = {"kernel": kern, "dispatches": d["dispatches"],
                             "mean_kb_per_dispatch": d["write_kb_total"] / d["dispatches"], "total_kb": d["write_kb_total"]}
        out["traffic_bytes_per_launch"] = {"formula": FORMULA, "value": d["traffic_bytes_per_launch"]}
    return out


if __name__ == "__main__":
    res = summarise(sys.argv[1], sys.argv[2])
    json.dump(res, open(sys.argv[3], "w"), indent=1)
    print(json.dumps({g: (v["dispatches"], round(v["traffic_bytes_per_launch"] / 1e6, 2)) for g, v in res["by_group"].items()}))
