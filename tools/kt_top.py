#!/usr/bin/env python3
"""Top kernels of a rocprofv3 kernel_stats.csv: name, calls, average and total time."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 14
for x in rows[:n]:
    print(f"{x['Name'][:72]:74s} {x['Calls']:>5s} avg {float(x['AverageNs']) / 1e3:9.1f} us  "
          f"total {float(x['TotalDurationNs']) / 1e6:8.2f} ms")
