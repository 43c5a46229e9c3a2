#!/usr/bin/env python3
"""Per-dispatch HBM bytes of one kernel from two rocprofv3 --pmc passes
(FETCH_SIZE and WRITE_SIZE, tools/pmc.sh's layout and gfx950 correction:
bytes = 2 * FETCH_SIZE KiB + WRITE_SIZE KiB) beside the dispatch's duration
(the pass's own kernel trace).  Lists the K longest dispatches whose name
contains PATTERN, and the pattern's totals.

    python tools/pmc_disp.py DIR NAME PATTERN [K]
"""
import csv
import sys

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from pmc_bytes import dispatches  # noqa: E402


def durations(path):
    return {int(r["Dispatch_Id"]): int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in csv.DictReader(open(path))}


def main():
    d, name, pat = sys.argv[1:4]
    k = int(sys.argv[4]) if len(sys.argv) > 4 else 12
    f = dispatches(f"{d}/{name}/FETCH_SIZE/pmc_counter_collection.csv")
    w = {i: x for i, _, x in dispatches(f"{d}/{name}/WRITE_SIZE/pmc_counter_collection.csv")}
    t = durations(f"{d}/{name}/FETCH_SIZE/pmc_kernel_trace.csv")
    rows = [(t.get(i, 0), n, 2 * a * 1024, w.get(i, 0) * 1024) for i, n, a in f if pat in n]
    tot = [sum(r[j] for r in rows) for j in (0, 2, 3)]
    print(f"{pat}: {len(rows)} dispatches, {tot[0] / 1e3:.1f} us, read {tot[1] / 1e9:.3f} GB, write {tot[2] / 1e9:.3f} GB")
    for ns, n, rd, wr in sorted(rows, reverse=True)[:k]:
        gbs = (rd + wr) / ns if ns else 0
        print(f"   {ns / 1e3:8.1f} us  read {rd / 1e6:8.1f} MB  write {wr / 1e6:7.1f} MB  {gbs:6.0f} GB/s  {n[:60]}")


if __name__ == "__main__":
    main()
