import json,glob,collections,sys,statistics
tag=sys.argv[1]
d=collections.defaultdict(list)
for f in sorted(glob.glob(f'gpurun_out/{tag}/*.json')):
    n=f.split('/')[-1][:-5]; cfg,nm,i=n.rsplit('_',2)
    try: b=json.loads(open(f).read().strip().splitlines()[-1])
    except Exception as e: print(f,e); continue
    d[(cfg,nm)].append((b['value']/1e6, b['step_kernel_ms']*1e3))
for k in sorted(d): print(k, [round(v,1) for v,_ in d[k]], 'median', round(statistics.median([v for v,_ in d[k]]),1), [round(u,2) for _,u in d[k]])
