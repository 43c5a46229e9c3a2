#!/usr/bin/env python3
"""Per-launch HBM traffic of k_refresh_score from the rocprofv3 PMC passes.

FETCH_SIZE/WRITE_SIZE are in KiB.  tools/microbench/pmc_calib.hip streams a
known 1 GiB with 1-, 8- and 16-byte lanes: on gfx950 FETCH_SIZE read exactly
half of it for every width and WRITE_SIZE exactly all of it (MI355X_MICROARCH.md
§HBM), so bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024.
usage: pmc_summary.py <dir with fetch/write csv> <config key> <out json>
"""
import collections
import csv
import json
import sys


def avg(path, kernel_prefix):
    v = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        v[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    ks = [k for k in v if k.startswith(kernel_prefix)]
    assert len(ks) == 1, ks
    return sum(v[ks[0]]) / len(v[ks[0]]), len(v[ks[0]]), ks[0]


def calib(path, kernel):
    v = [float(r["Counter_Value"]) for r in csv.DictReader(open(path)) if r["Kernel_Name"].startswith(kernel)]
    return sum(v) / len(v) * 1024 / 2**30


def main():
    d, key, out = sys.argv[1], sys.argv[2], sys.argv[3]
    k = "void gsx::k_refresh_score<8, true>"
    f, nf, name = avg(f"{d}/fetch_size_counter_collection.csv", k)
    w, nw, _ = avg(f"{d}/write_size_counter_collection.csv", k)
    cal = {
        "fetch_fraction_8B_lanes": calib(f"{d}/calib_fetch_size.csv", "void k_read<double>"),
        "fetch_fraction_16B_lanes": calib(f"{d}/calib_fetch_size.csv", "void k_read<HIP_vector_type"),
        "fetch_fraction_1B_lanes": calib(f"{d}/calib_fetch_size.csv", "k_read_u8"),
        "write_fraction_8B_lanes": calib(f"{d}/calib_write_size.csv", "void k_write<double>"),
    }
    res = {
        "config": key,
        "kernel": name,
        "launches": [nf, nw],
        "fetch_size_kib": f,
        "write_size_kib": w,
        "calibration": cal,
        "read_bytes_per_launch": 2 * f * 1024,
        "write_bytes_per_launch": w * 1024,
        "hbm_bytes_per_launch": (2 * f + w) * 1024,
    }
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
