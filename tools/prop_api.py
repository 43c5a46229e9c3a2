#!/usr/bin/env python3
"""One propagation call's host/device sequence from a rocprofv3
--hip-runtime-trace --kernel-trace run of tools/prop_profile.py: every HIP API
call (name, host us) and every kernel / fill / copy (device us) between the
last two k_prop_clear launches, in start order.

    python tools/prop_api.py KT_DIR/kt_hip_api_trace.csv KT_DIR/kt_kernel_trace.csv [KT_DIR/kt_memory_copy_trace.csv]
"""
import csv
import sys


def rows(path):
    with open(path) as f:
        return list(csv.DictReader(f))


def main():
    api = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "api " + r["Function"]) for r in rows(sys.argv[1])]
    kt = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "gpu " + r["Kernel_Name"].split("(")[0][:60])
          for r in rows(sys.argv[2])]
    clears = sorted(s for s, _, n in kt if "k_prop_clear" in n)
    if len(clears) < 2:
        print("fewer than two calls in the trace")
        return
    a, b = clears[-2], clears[-1]
    # the API calls that led to the window's first kernel start before it: take them from the previous clear's launch
    launches = sorted(s for s, _, n in api if "LaunchKernel" in n)
    ev = sorted([x for x in kt if a <= x[0] < b] + [x for x in api if a - 2_000_000 <= x[0] < b])
    t0 = ev[0][0]
    for s, e, n in ev:
        print(f"{(s - t0) / 1e3:10.1f} us  {(e - s) / 1e3:8.1f} us  {n}")


if __name__ == "__main__":
    main()
