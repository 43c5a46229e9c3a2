#!/usr/bin/env python3
"""Kernel stats split by launch shape: a rocprofv3 kt_kernel_trace.csv ->
one row per (kernel, grid size, workgroup size), so kernels launched on
different workloads in one run (e.g. k_refresh_score on the cfg3 engine and
on the single-observer engine) get separate averages.

usage: kt_split.py kt_kernel_trace.csv [out.csv]  (stdout without out.csv)
"""
import csv
import statistics
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    groups = {}
    for r in rows:
        key = (r["Kernel_Name"], int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"]),
               int(r["Workgroup_Size_X"]) * int(r["Workgroup_Size_Y"]) * int(r["Workgroup_Size_Z"]))
        groups.setdefault(key, []).append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    out = open(sys.argv[2], "w", newline="") if len(sys.argv) > 2 else sys.stdout
    w = csv.writer(out, quoting=csv.QUOTE_NONNUMERIC)
    w.writerow(["Name", "Grid", "Workgroup", "Calls", "TotalDurationNs", "AverageNs", "MinNs", "MaxNs", "StdDev"])
    for (name, grid, wg), d in sorted(groups.items(), key=lambda kv: -sum(kv[1])):
        w.writerow([name, grid, wg, len(d), sum(d), sum(d) / len(d), min(d), max(d),
                    statistics.pstdev(d) if len(d) > 1 else 0.0])


if __name__ == "__main__":
    main()
