#!/usr/bin/env python3
"""Per-round heartbeat kernel breakdown from a rocprofv3 kernel trace
(kt_kernel_trace.csv): every round runs k_hb_scan ... k_hb_answer."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
cur, out = None, []
for r in rows:
    n = r["Kernel_Name"].split("(")[0].replace("gsx::", "").replace("void ", "")
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    if n == "k_hb_scan" or n == "k_hb_clear_backoff":
        cur = cur if (cur is not None and n == "k_hb_scan" and cur and cur[-1][0] == "k_hb_clear_backoff") else []
    if cur is not None:
        cur.append((n, d))
        if n == "k_hb_answer":
            out.append(cur)
            cur = None
for i, r in enumerate(out):
    agg = {}
    for n, d in r:
        agg[n] = agg.get(n, 0) + d
    print(i, " ".join(f"{k}={v:.0f}" for k, v in agg.items()), "total=%.0f us" % sum(agg.values()))
