"""Per-bucket kb kernel times of the last step in a rocprofv3 kernel trace."""
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r['Start_Timestamp']))
idx = [i for i, r in enumerate(rows) if 'k_kb_bounds' in r['Kernel_Name']][-1]
buckets, cur = [], {}
for r in rows[idx + 1:]:
    n = re.sub(r'\(.*', '', r['Kernel_Name']).replace('sheep::', '').replace('void ', '').split('<')[0]
    d = (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3
    cur[n] = cur.get(n, 0) + d
    if n == 'k_kb_label':
        buckets.append(cur)
        cur = {}
step = int(sys.argv[2]) if len(sys.argv) > 2 else 6
for i, b in enumerate(buckets):
    if i % step == 0 or i > len(buckets) - 4:
        print(i, {k[5:]: round(v, 1) for k, v in b.items() if k.startswith('k_kb')})
