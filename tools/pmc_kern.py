#!/usr/bin/env python3
"""Per dispatch of the kernels whose name matches REGEX: duration and every
counter of one rocprofv3 --pmc pass (summed over the counter's dimensions).

    python tools/pmc_kern.py pmc_counter_collection.csv pmc_kernel_trace.csv REGEX
"""
import collections
import csv
import re
import sys


def main():
    cc, kt, rx = sys.argv[1], sys.argv[2], re.compile(sys.argv[3])
    dur = {int(r["Dispatch_Id"]): int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in csv.DictReader(open(kt))}
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    name = {}
    for r in csv.DictReader(open(cc)):
        if not rx.search(r["Kernel_Name"]):
            continue
        d = int(r["Dispatch_Id"])
        per[d][r["Counter_Name"]] += float(r["Counter_Value"])
        name[d] = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("gsx::", "")
    for d in sorted(per):
        c = per[d]
        print(f"{d:6d} {name[d]:28s} {dur.get(d, 0) / 1e3:8.1f} us  " +
              "  ".join(f"{k}={v:.4g}" for k, v in sorted(c.items())))


if __name__ == "__main__":
    main()
