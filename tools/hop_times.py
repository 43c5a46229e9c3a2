"""Per-hop k_prop_hop times (us) of the last propagation batch in a rocprofv3
kernel trace: the plain and SRC launches of a hop are summed."""
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r['Dispatch_Id']))
hops = [r for r in rows if 'k_prop_hop' in r['Kernel_Name']]
d = lambda r: (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1000
per = 2 if any('true>' in r['Kernel_Name'] and r['Kernel_Name'].count('true') + r['Kernel_Name'].count('false') >= 2 and 'true>(' in r['Kernel_Name'] for r in hops) else 1
last = hops[-24 * per:]
t = [sum(d(r) for r in last[i:i + per]) for i in range(0, len(last), per)]
print(len(hops), [round(x) for x in t], round(sum(t) / 1000, 3), 'ms (hop kernels of the last batch)')
tail = rows[-60:]
print({r['Kernel_Name'].split('(')[0][-22:]: round(d(r)) for r in tail if 'hop' not in r['Kernel_Name'] and 'rocclr' not in r['Kernel_Name']})
