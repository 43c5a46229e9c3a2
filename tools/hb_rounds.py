#!/usr/bin/env python3
"""Per-round heartbeat kernel breakdown from a rocprofv3 kernel trace
(kt_kernel_trace.csv): a round runs from one k_hb_scan (or the
k_hb_clear_backoff before it) to the last heartbeat-side kernel before the
next propagation."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
HB = ("k_hb", "k_mask_and", "k_refresh_score<", "__amd_rocclr_fill", "k_mc_summary")
out, cur = [], None
for r in rows:
    n = r["Kernel_Name"].split("(")[0].replace("gsx::", "").replace("void ", "")
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    if n in ("k_hb_scan", "k_hb_clear_backoff") and not (cur and cur[-1][0] == "k_hb_clear_backoff"):
        cur = []
        out.append(cur)
    if cur is None:
        continue
    if n.startswith(HB) and not n.startswith("k_refresh_score<8, true>"):
        cur.append((n, d))
    elif n.startswith("k_prop"):
        cur = None
for i, r in enumerate(out):
    agg = {}
    for n, d in r:
        agg[n] = agg.get(n, 0) + d
    print(i, " ".join(f"{k}={v:.0f}" for k, v in agg.items()), "total=%.0f us" % sum(agg.values()))
