#!/usr/bin/env python3
"""Idle time between consecutive kernels in a rocprofv3 kernel-trace CSV (--kernel-trace --output-format csv):
per kernel, the median and mean gap before it and its median duration; then N consecutive launches from the middle
of the run.  Usage: python tools/trace_gaps.py run_kernel_trace.csv [N].  (DESIGN.md §5 host flow.)"""
import csv,collections,sys
rows=list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r:int(r['Start_Timestamp']))
short=lambda n: n.split('(')[0].replace('void ','').replace('gwo::','')[:34]
g=collections.defaultdict(list); d=collections.defaultdict(list); prev=None
for r in rows:
    s,e=int(r['Start_Timestamp']),int(r['End_Timestamp'])
    if prev: g[short(r['Kernel_Name'])].append(s-prev)
    d[short(r['Kernel_Name'])].append(e-s); prev=e
for k,v in g.items():
    v.sort(); dd=sorted(d[k]); print('  %-36s n %5d median gap %7.2f  mean gap %7.2f  median dur %7.2f'%(k,len(v),v[len(v)//2]/1000,sum(v)/len(v)/1000,dd[len(dd)//2]/1000))
mid=len(rows)//2; prev=None
for r in rows[mid:mid+int(sys.argv[2]) if len(sys.argv)>2 else mid+10]:
    s,e=int(r['Start_Timestamp']),int(r['End_Timestamp'])
    print(f"{short(r['Kernel_Name']):30s} gap {(s-prev)/1000 if prev else 0:6.2f} dur {(e-s)/1000:6.2f}"); prev=e
