#!/usr/bin/env python3
"""Per kernel: dispatches, time, L2 hits / misses (hit rate) and L2 read
requests to the fabric (TCC_EA0_RDREQ: Infinity Cache or HBM) from one
rocprofv3 --pmc pass (tools/pmc_hit.sh).

    python tools/pmc_hit.py pmc_counter_collection.csv pmc_kernel_trace.csv
"""
import collections
import csv
import sys


def short(n):
    return n.split("(")[0].replace("void ", "").replace("gsx::", "")


def main():
    cc, kt = sys.argv[1:3]
    dur = {int(r["Dispatch_Id"]): int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in csv.DictReader(open(kt))}
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    seen = collections.defaultdict(set)
    for r in csv.DictReader(open(cc)):
        k, d = short(r["Kernel_Name"]), int(r["Dispatch_Id"])
        per[k][r["Counter_Name"]] += float(r["Counter_Value"])
        seen[k].add(d)
    rows = []
    for k, c in per.items():
        t = sum(dur.get(d, 0) for d in seen[k])
        hit, miss, rd = c.get("TCC_HIT_sum", 0), c.get("TCC_MISS_sum", 0), c.get("TCC_EA0_RDREQ_sum", 0)
        rows.append((t, k, len(seen[k]), hit, miss, rd))
    print(f"{'kernel':44s} {'n':>4s} {'ms':>8s} {'L2 hit':>7s} {'misses':>10s} {'EA rdreq':>10s}")
    for t, k, n, hit, miss, rd in sorted(rows, reverse=True)[:16]:
        hr = hit / (hit + miss) if hit + miss else 0.0
        print(f"{k[:44]:44s} {n:4d} {t / 1e6:8.3f} {hr:7.3f} {miss:10.3e} {rd:10.3e}")


if __name__ == "__main__":
    main()
