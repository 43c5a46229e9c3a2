#!/usr/bin/env python3
"""Per heartbeat round (a round starts at each k_hb_scan dispatch), the time of
every kernel between it and the next round's scan, grouped by kernel name,
largest first; propagation kernels (k_prop_*) between rounds are left out.

    python tools/kt_rounds.py kt_kernel_trace.csv [top] [kernel ...]

Kernels named after `top` also get their dispatch durations listed in order
(e.g. k_gxf_pull_g k_gxf_mark: the forwarding's per-hop times)."""
import csv
import re
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
top = int(sys.argv[2]) if len(sys.argv) > 2 else 14
each = sys.argv[3:]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))


def short(n):
    n = re.sub(r"\(.*", "", n)
    n = n.replace("void ", "").replace("gsx::", "")
    return n


rounds, cur = [], None
for r in rows:
    name = short(r["Kernel_Name"])
    if name == "k_hb_scan":
        cur = {"t0": int(r["Start_Timestamp"]), "k": defaultdict(float), "n": defaultdict(int), "end": 0,
               "each": defaultdict(list)}
        rounds.append(cur)
    if cur is None or name.startswith("k_prop_") or name.startswith("k_mc_summary"):
        if cur is not None and name.startswith("k_prop_"):
            cur = None  # a propagation: the round is over
        continue
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000
    cur["k"][name] += d
    cur["n"][name] += 1
    if any(name.startswith(x) for x in each):
        cur["each"][name].append(d)
    cur["end"] = int(r["End_Timestamp"])
for i, R in enumerate(rounds):
    tot = sum(R["k"].values())
    span = (R["end"] - R["t0"]) / 1000
    print(f"round {i}: kernels {tot:.0f} us, span {span:.0f} us")
    for k, v in sorted(R["k"].items(), key=lambda x: -x[1])[:top]:
        print(f"   {k:40s} {v:9.1f} us  x{R['n'][k]}")
    for k, ds in R["each"].items():
        print(f"   {k}: " + " ".join(f"{d:.0f}" for d in ds))
