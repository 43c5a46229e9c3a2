#!/usr/bin/env python3
"""Per-kernel totals from a rocprofv3 kernel-trace database (rocpd sqlite:
rocprofv3 --kernel-trace without --output-format csv).
usage: kt_db.py <results.db> [top]"""
import collections
import sqlite3
import sys

c = sqlite3.connect(sys.argv[1])
top = int(sys.argv[2]) if len(sys.argv) > 2 else 30
ks = {r[0]: r[1] for r in c.execute("select id, kernel_name from rocpd_info_kernel_symbol")}
agg = collections.defaultdict(lambda: [0, 0.0])
for k, s, e in c.execute("select kernel_id, start, end from rocpd_kernel_dispatch order by start"):
    n = ks[k].split("(")[0].replace("void ", "").replace("gsx::", "")
    if n.startswith("_Z"):
        import subprocess
        n = subprocess.run(["c++filt", n.replace(".kd", "")], capture_output=True, text=True).stdout.strip().split("(")[0].replace("gsx::", "")
    agg[n][0] += 1
    agg[n][1] += (e - s) / 1e6
tot = sum(v[1] for v in agg.values())
print(f"{'ms':>10} {'calls':>6} {'us/call':>9}  kernel   (total {tot:.3f} ms)")
for n, (cnt, ms) in sorted(agg.items(), key=lambda x: -x[1][1])[:top]:
    print(f"{ms:10.3f} {cnt:6d} {1e3 * ms / cnt:9.1f}  {n}")
