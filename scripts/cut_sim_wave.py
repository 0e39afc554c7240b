"""The same as scripts/cut_sim.py with cuts served only by idle lanes of the chain's own wave (the wave slot,
diagnostic timeline column 15): no cross-wave hand-over.
    python scripts/cut_sim_wave.py ROWS.npz GARBAGE MAXCUTS"""
import numpy as np, sys, heapq
from collections import defaultdict
rows = np.load(sys.argv[1])["rows"].astype(np.int64)
garb = float(sys.argv[2]) if len(sys.argv)>2 else 6.0
maxcuts = int(sys.argv[3]) if len(sys.argv)>3 else 1
t0 = rows[:,4].min(); start=(rows[:,4]-t0)/1e5; end=(rows[:,5]-t0)/1e5
wave = rows[:,3]; recs = rows[:,6]; hw = rows[:,15]
lane = (wave==0) & (hw!=0)
t_q = start[lane].max()
per = defaultdict(list)
for i in np.where(lane)[0]: per[hw[i]].append(i)
base=[]; cut=[]
for h, items in per.items():
    items=np.array(items)
    e=end[items]; r=(end[items]-start[items])/np.maximum(recs[items],1)
    base.append(e.max())
    pieces=[[e[k], r[k], 0] for k in range(len(items)) if e[k]>t_q]   # [end, ms/sample, cuts]
    done_before = max([v for v in e if v<=t_q], default=0.0)
    idle = [t_q]*max(0,64-len(pieces))
    # event loop
    while True:
        # next free lane: earliest of idle times and piece ends
        cand_piece = min(range(len(pieces)), key=lambda q: pieces[q][0]) if pieces else None
        tf = min(idle) if idle else None
        if cand_piece is not None and (tf is None or pieces[cand_piece][0] < tf):
            tf = pieces[cand_piece][0]; pieces.pop(cand_piece)
        elif tf is not None:
            idle.remove(tf)
        else: break
        if not pieces: break
        j = max(range(len(pieces)), key=lambda q: pieces[q][0])
        en, rr, nc = pieces[j]
        left = en - tf
        if nc >= maxcuts or left <= 2*garb*rr + 0.2: 
            # no worthwhile cut for the longest piece: stop
            break
        half = left/2
        pieces[j] = [tf+half, rr, nc+1]
        pieces.append([tf+half+garb*rr, rr, nc+1])
    cut.append(max(done_before, max([p[0] for p in pieces], default=0.0)))
print(sys.argv[1], "garbage", garb, "cuts/piece", maxcuts, "| launch end base", round(max(base),1), "-> with intra-wave cuts", round(max(cut),1),
      "| wave end p50/p90/p99 base", np.percentile(base,[50,90,99]).round(1), "cut", np.percentile(cut,[50,90,99]).round(1))
