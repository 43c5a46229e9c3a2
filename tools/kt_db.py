#!/usr/bin/env python3
"""Kernel summary of a rocprofv3 --kernel-trace database (rocpd sqlite):
per kernel calls, total / average microseconds, share.  Optional --seq NAME...
prints the dispatch sequence of the kernels whose names contain NAME.

    python tools/kt_db.py gpurun_out/X/prof/run_results.db [--top 20] [--seq hop_fast1 pack_front]
"""
import argparse
import sqlite3

ap = argparse.ArgumentParser()
ap.add_argument("db")
ap.add_argument("--top", type=int, default=20)
ap.add_argument("--seq", nargs="*")
ap.add_argument("--csv", help="write the summary as CSV here")
a = ap.parse_args()
c = sqlite3.connect(a.db)
rows = list(c.execute("select name, total_calls, total_duration, average, percentage from top_kernels"))
if a.csv:
    with open(a.csv, "w") as f:
        f.write("Name,Calls,TotalDurationNs,AverageNs,Percentage\n")
        for n, k, t, av, p in rows:
            f.write(f"\"{n}\",{k},{t * 1000:.0f},{av * 1000:.0f},{p:.4f}\n")
for n, k, t, av, p in rows[: a.top]:
    print(f"{n[:90]:90s} {k:6d} {t / 1e3:10.3f} ms {av:9.1f} us {p:5.1f}%")
if a.seq:
    for n, s, e in c.execute("select name, start, end from kernels order by start"):
        if any(x in n for x in a.seq):
            print(f"{n[:60]:60s} {(e - s) / 1e3:9.1f} us")
