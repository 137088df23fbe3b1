"""Pairwise summary of an interleaved A/B (scripts/box_r5_head_ab.sh, box_e2e_pair_ab.sh): per config,
the median CPU per event and events/s of each arm, and in how many pairs the new arm used less CPU.
Usage: python scripts/ab_pairs.py gpurun_out/<out>/ab.jsonl"""
import json,statistics as st,sys
from collections import defaultdict
rows=[json.loads(l) for l in open(sys.argv[1])]
by=defaultdict(lambda: defaultdict(list))
for r in rows:
    eps=r.get('eps', r.get('events_per_sec')); cpu=r.get('cpu_us', r.get('cpu_us_per_event'))
    by[r['cfg']][(r['pair'],r['arm'])].append((eps,cpu))
for cfg,d in by.items():
    pairs=sorted({p for p,_ in d})
    wins=0; n=0; out=[]
    for p in pairs:
        if (p,'new') in d and (p,'old') in d:
            a=st.median(x[1] for x in d[(p,'new')]); b=st.median(x[1] for x in d[(p,'old')])
            out.append('%.3f/%.3f'%(a,b)); wins+= a<b; n+=1
    allnew=[x[1] for p in pairs for x in d.get((p,'new'),[])]; allold=[x[1] for p in pairs for x in d.get((p,'old'),[])]
    en=[x[0] for p in pairs for x in d.get((p,'new'),[])]; eo=[x[0] for p in pairs for x in d.get((p,'old'),[])]
    print(cfg, 'cpu new/old median %.3f / %.3f'%(st.median(allnew),st.median(allold)), 'eps %.0f / %.0f'%(st.median(en),st.median(eo)), 'new wins %d of %d pairs'%(wins,n))
    print('  ', ' '.join(out))
