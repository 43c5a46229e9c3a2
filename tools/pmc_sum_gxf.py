"""Sums the PMC passes of tools/gxf_pmc.sh over the heavy (>150 us) dispatches."""
import csv,collections,sys
base=sys.argv[1]
d=collections.defaultdict(dict)
for i in range(1,5):
    for r in csv.DictReader(open(f'{base}/p{i}/pmc_counter_collection.csv')):
        k=(i,int(r['Dispatch_Id']))
        d[k][r['Counter_Name']]=d[k].get(r['Counter_Name'],0)+float(r['Counter_Value'])
        d[k]['dur']=(int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1e3
tot=collections.Counter()
for k,v in d.items():
    if v['dur']>150:
        for a,b in v.items(): tot[a]+=b
        tot['n%d'%k[0]]+=1
print({a:round(b) for a,b in tot.items()})
