"""Per-round forwarding-pull hop durations (>100 us) and gx kernel totals from a
rocprofv3 kernel trace CSV (tools/gxf_ab.sh, tools/hbx_prof.sh)."""
import csv, sys
rows=list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r:int(r['Start_Timestamp']))
tot={}
cur=[]
for r in rows:
    n=r['Kernel_Name'].split('(')[0].replace('void gsx::','').replace('gsx::','')
    d=(int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1e3
    if 'k_gx_setprep' in n and cur:
        print(' '.join(cur)); cur=[]
    if 'gx' in n:
        tot[n]=tot.get(n,0)+d
        if 'pull' in n and d>100: cur.append(f"{d:.0f}")
print(' '.join(cur))
for k,v in sorted(tot.items(),key=lambda x:-x[1]): print(f"{k:30s} {v/1e3:8.2f} ms")
