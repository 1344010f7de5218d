"""Per-bucket timeline of the kb tree loop from a rocprofv3 --kernel-trace CSV (the last tree
of the run): for each bucket the apply chain's span on the main stream and its kernels
(refresh, spine, zipper, union, label), beside the next bucket's map on the side stream.
  python scripts/kb_timeline.py gpurun_out/tr/r26/run_kernel_trace.csv
"""
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r['Start_Timestamp']))
picks = [i for i, r in enumerate(rows) if 'k_kb_pick' in r['Kernel_Name']]
# the last tree: picks after the last k_iota preceding the final pick run
last_iota = max(i for i, r in enumerate(rows) if 'k_iota' in r['Kernel_Name'] and i < picks[-1])
rows = rows[last_iota:]
t0 = int(rows[0]['Start_Timestamp'])
def T(r, k): return (int(r[k]) - t0) / 1e6
buckets = []
cur = None
maps = []
for r in rows:
    n = r['Kernel_Name']
    if 'k_kb_map' in n: maps.append((T(r,'Start_Timestamp'), T(r,'End_Timestamp'))); continue
    for key in ('pick','gb_sum','refresh','spine','zip','union','label'):
        if 'k_kb_' + key in n or 'k_' + key in n:
            if key == 'pick':
                cur = {'start': T(r,'Start_Timestamp')}; buckets.append(cur)
            if cur is not None:
                cur[key] = cur.get(key, 0) + T(r,'End_Timestamp') - T(r,'Start_Timestamp')
                cur['end'] = T(r,'End_Timestamp')
print(f"{'b':>3} {'start':>8} {'span':>6} {'map':>6} {'refr':>6} {'spine':>6} {'zip':>6} {'union':>6} {'label':>6}")
tot = {}
for i, b in enumerate(buckets):
    mp = maps[i+1] if i + 1 < len(maps) else (0,0)
    span = b['end'] - b['start']
    print(f"{i:3d} {b['start']:8.3f} {span:6.3f} {mp[1]-mp[0]:6.3f} {b.get('refresh',0):6.3f} {b.get('spine',0):6.3f} {b.get('zip',0):6.3f} {b.get('union',0):6.3f} {b.get('label',0):6.3f}")
    for k in ('refresh','spine','zip','union','label','pick','gb_sum'): tot[k] = tot.get(k,0) + b.get(k,0)
print('total', {k: round(v,3) for k,v in tot.items()}, 'maps', round(sum(e-s for s,e in maps),3))
print('tree', round(buckets[-1]['end'] - maps[0][0], 3))
