#!/usr/bin/env python3
"""Ghost-set sizes of the partitioned programs: for the bench graph split N ways
(equal ranges), per rank the distinct remote sources of its PageRank in-lists and the distinct
remote neighbours of its bothE lists, next to the values an all-gather moves.
usage: python scripts/ghost_sets.py <scale> <N>   (host only; numpy)"""
import sys, numpy as np, time, json
sys.path.insert(0, __import__('os').path.join(__import__('os').path.dirname(__import__('os').path.abspath(__file__)), '..'))
from titan_amd import rmat_edges
scale=int(sys.argv[1]); W=int(sys.argv[2])
t=time.time()
src,dst,_=rmat_edges(scale,16,threads=8)
n=1<<scale; nl=n//W
deg = np.bincount(src,minlength=n)+np.bincount(dst,minlength=n)
active = deg>0
act_per_rank=[int(active[r*nl:(r+1)*nl].sum()) for r in range(W)]
span=max(act_per_rank)  # roughly: the layout puts active rows first
own_s = src//nl; own_d = dst//nl
res={"scale":scale,"W":W,"n":n,"m":int(len(src)),"active":int(active.sum()),"span":span}
pr=[]; bfs=[]
for r in range(W):
    # PageRank pull over inE: rows = dst owned by r, sources = src
    sel=(own_d==r)&(own_s!=r)
    pr.append(int(len(np.unique(src[sel]))))
    # bothE pull (MS-BFS dense): rows owned by r, neighbours both ways
    a=src[(own_d==r)&(own_s!=r)]; b=dst[(own_s==r)&(own_d!=r)]
    bfs.append(int(len(np.unique(np.concatenate([a,b])))))
res["pr_ghosts_per_rank"]=pr; res["bothE_ghosts_per_rank"]=bfs
res["allgather_values_per_rank"]=(W-1)*span
print(json.dumps(res)); print('time',time.time()-t, file=sys.stderr)
