#!/usr/bin/env python3
"""Host side of one heartbeat: the HIP API calls and kernels inside each
round's wall-clock window (tools/hb_micro.py prints `window TICK T0 T1` on the
profiler's clock, CLOCK_BOOTTIME).  Per round: wall, kernel busy time, the
API calls by name (count, total us) and the longest host gaps between kernels.

    python tools/hb_api.py hb_micro.log KT_DIR/kt_hip_api_trace.csv KT_DIR/kt_kernel_trace.csv
"""
import collections
import csv
import sys


def rows(path):
    with open(path) as f:
        return list(csv.DictReader(f))


def main():
    log, api_p, kt_p = sys.argv[1:4]
    wins = []
    for ln in open(log):
        if ln.startswith("window "):
            _, tick, a, b = ln.split()
            wins.append((int(tick), int(a), int(b)))
    api = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Function"]) for r in rows(api_p)]
    kt = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows(kt_p)]
    for tick, a, b in wins:
        calls = collections.defaultdict(lambda: [0, 0])
        for s, e, fn in api:
            if a <= s < b:
                calls[fn][0] += 1
                calls[fn][1] += e - s
        ks = sorted((s, e, n) for s, e, n in kt if a <= s < b)
        busy = sum(e - s for s, e, _ in ks)
        print(f"tick {tick}: wall {(b - a) / 1e3:.1f} us, {len(ks)} kernels busy {busy / 1e3:.1f} us, "
              f"first kernel at +{(ks[0][0] - a) / 1e3 if ks else 0:.1f} us, last ends {(b - ks[-1][1]) / 1e3 if ks else 0:.1f} us "
              "before the window")
        for fn, (c, t) in sorted(calls.items(), key=lambda x: -x[1][1])[:14]:
            print(f"   {fn:40s} x{c:4d} {t / 1e3:9.1f} us")
        gaps = sorted(((ks[i + 1][0] - ks[i][1], ks[i][2][:40], ks[i + 1][2][:40]) for i in range(len(ks) - 1)),
                      reverse=True)[:8]
        for g, x, y in gaps:
            print(f"   gap {g / 1e3:7.1f} us  {x} -> {y}")


if __name__ == "__main__":
    main()
