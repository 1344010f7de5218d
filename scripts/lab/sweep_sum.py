"""Per-config means of an ab_env.sh sweep (default against SHEEP_KB_BIRTH=1): step and tree ms,
and the worst difference.  python scripts/lab/sweep_sum.py gpurun_out/r06x/ab.jsonl"""
import json, collections, sys
d=collections.defaultdict(lambda: collections.defaultdict(list))
for l in open(sys.argv[1]):
    r=json.loads(l); a=r['args'].replace(' --no-cpu-baseline','').split(' --steps')[0] or 'rmat26'
    d[a][r['env'] or 'default'].append((r['ms'], r['phases'].get('tree_insert',-1)))
worst=-9
for a in d:
    e=d[a]; b=e.get('default',[]); n=e.get('SHEEP_KB_BIRTH=1',[])
    if not b or not n: continue
    mb=sum(x[0] for x in b)/len(b); mn=sum(x[0] for x in n)/len(n)
    tb=sum(x[1] for x in b)/len(b); tn=sum(x[1] for x in n)/len(n)
    worst=max(worst, mn-mb)
    print(f"{a:32s} default {mb:7.3f} (tree {tb:6.3f})  birth {mn:7.3f} (tree {tn:6.3f})  diff {mn-mb:+.3f}")
print("worst diff", round(worst,3))
