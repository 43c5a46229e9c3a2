import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
hops = [r for r in rows if 'k_prop_hop' in r['Kernel_Name']]
d = lambda r: (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1000
print(len(hops), [round(d(r)) for r in hops[-24:]], round(sum(d(r) for r in hops[-24:]) / 1000, 3), 'ms')
last = rows[-40:]
print({r['Kernel_Name'].split('(')[0][-22:]: round(d(r)) for r in last if 'hop' not in r['Kernel_Name'] and 'rocclr' not in r['Kernel_Name']})
