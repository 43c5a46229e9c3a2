"""Per-dispatch PMC table for one kernel across the passes of tools/prop_pmc.sh."""
import collections, csv, glob, sys
base, kern = sys.argv[1], sys.argv[2]
agg = collections.defaultdict(dict)
for f in sorted(glob.glob(f"{base}/p*/pmc_counter_collection.csv")):
    per = collections.defaultdict(dict)
    for r in csv.DictReader(open(f)):
        if kern not in r['Kernel_Name']:
            continue
        per[int(r['Dispatch_Id'])][r['Counter_Name']] = per[int(r['Dispatch_Id'])].get(r['Counter_Name'], 0) + float(r['Counter_Value'])
    for k, (i, v) in enumerate(sorted(per.items())):
        agg[k].update(v)
for k in sorted(agg):
    print(k, {n: f"{x:.3g}" for n, x in agg[k].items()})
