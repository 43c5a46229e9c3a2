#!/usr/bin/env python3
"""Summarise tools/pmc.sh: HBM bytes = (2 * FETCH_SIZE + WRITE_SIZE) KiB
(gfx950, checked by tools/microbench/pmc_calib.hip) per launch of the headline
kernel, per batch of the propagation hops and per-call passes, per heartbeat
round (the last round of bench.py's heartbeat leg).  Each section carries the workload
it measured, in bench.py's keys (bench.pmc_bytes compares them).
usage: pmc_bytes.py <dir> <headline config key, e.g. n=1000000,T=8,d=6,E=11999954> [summary to merge into]
(a section whose runs are absent is taken from the merged summary)"""
import collections
import csv
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def dispatches(path):
    """-> [(dispatch id, kernel, value)] in dispatch order (values summed per dispatch)."""
    v = collections.OrderedDict()
    for r in csv.DictReader(open(path)):
        k = (int(r["Dispatch_Id"]), r["Kernel_Name"])
        v[k] = v.get(k, 0.0) + float(r["Counter_Value"])
    return sorted(((d, n, x) for (d, n), x in v.items()))


def load(d, name):
    f = dispatches(f"{d}/{name}/FETCH_SIZE/pmc_counter_collection.csv")
    w = dispatches(f"{d}/{name}/WRITE_SIZE/pmc_counter_collection.csv")
    assert [n for _, n, _ in f] == [n for _, n, _ in w], name  # the same dispatch sequence in both passes
    return [(n, 2 * a * 1024, b * 1024) for (_, n, a), (_, _, b) in zip(f, w)]


def short(n):
    return n.split("(")[0].replace("void ", "").replace("gsx::", "")


def main():
    d = sys.argv[1]
    out = {"bytes": "2 x FETCH_SIZE + WRITE_SIZE (KiB x 1024), gfx950"}
    if len(sys.argv) > 3:
        out.update(json.load(open(sys.argv[3])))
    has = lambda name: os.path.isdir(f"{d}/{name}")  # noqa: E731
    if has("calib"):
        section_calib(d, out)
    if has("head"):
        section_head(d, out)
    for name in ("p1024", "p64"):
        if has(name):
            section_prop(d, out, name)
    if has("hb"):
        section_hb(d, out)
    print(json.dumps(out, indent=1))


def section_calib(d, out):
    cal = load(d, "calib")
    out["calibration"] = {short(n): {"read": r / 2**30, "write": w / 2**30} for n, r, w in cal}


def section_head(d, out):
    head = [x for x in load(d, "head") if short(x[0]) == "k_refresh_score<8, true>"]
    out["k_refresh_score<8, true>"] = {
        "workload": {"config": sys.argv[2]},
        "launches": len(head),
        "read_bytes_per_launch": sum(x[1] for x in head) / len(head),
        "write_bytes_per_launch": sum(x[2] for x in head) / len(head),
        "hbm_bytes_per_launch": sum(x[1] + x[2] for x in head) / len(head),
    }


def section_prop(d, out, name, batches=3):
    import bench

    rows = load(d, name)
    marks = [i for i, x in enumerate(rows) if short(x[0]) == "k_prop_hops_export"]
    if marks:  # prop_profile.py --warmup: the batches after the marker (steady state)
        rows = rows[marks[-1] + 1:]
    hop = [x for x in rows if short(x[0]).startswith("k_prop_hop")]
    call = [x for x in rows if short(x[0]).startswith(("k_prop", "k_mc_summary")) and x not in hop]
    per = collections.defaultdict(float)
    for n, r, w in call:
        per[short(n)] += (r + w) / batches
    out[name] = {
        "workload": bench.prop_workload(1_000_000, 1024 if name == "p1024" else 64),
        "batches": batches,
        "hop_launches": len(hop),
        "hop_bytes_per_batch": sum(r + w for _, r, w in hop) / batches,
        "hop_read_bytes_per_batch": sum(r for _, r, _ in hop) / batches,
        "hop_write_bytes_per_batch": sum(w for _, _, w in hop) / batches,
        "per_call_pass_bytes_per_batch": sum(per.values()),
        "per_call_passes": dict(sorted(per.items(), key=lambda kv: -kv[1])),
    }


def section_hb(d, out):
    import bench

    rows = load(d, "hb")
    rounds, cur = [], None
    for n, r, w in rows:
        s = short(n)
        if s in ("k_gx_promises", "k_hb_clear_backoff") or (s == "k_hb_scan" and (cur is None or "k_hb_scan" in cur)):
            cur = collections.OrderedDict()
            rounds.append(cur)
        if s.startswith("k_prop"):
            cur = None
            continue
        if cur is not None:
            cur[s] = cur.get(s, 0.0) + r + w
    last = rounds[-1]
    out["heartbeat_last_round"] = {"workload": bench.hb_workload(1_000_000, 8, 256, True),
                                   "hbm_bytes": sum(last.values()),
                                   "kernels": dict(sorted(last.items(), key=lambda kv: -kv[1]))}


if __name__ == "__main__":
    main()
