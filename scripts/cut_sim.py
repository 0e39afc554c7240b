"""What run-time cuts of slow chains could give, from a launch's item rows (r06 estimate): once
the work items are all handed out (or from a gate time), every lane that runs free takes half of the remaining
stream of the chain that would end last (a cut: the new piece pays `garbage` samples before it lands on the
true chain, at the original chain's measured per-sample rate), up to `maxcuts` cuts per chain.
    python scripts/cut_sim.py ROWS.npz GARBAGE MAXCUTS [GATE_MS]"""
import numpy as np, sys, heapq
rows = np.load(sys.argv[1])["rows"].astype(np.int64)
garb = float(sys.argv[2]); maxcuts=int(sys.argv[3]); tgate=float(sys.argv[4]) if len(sys.argv)>4 else None
t0 = rows[:,4].min(); start=(rows[:,4]-t0)/1e5; end=(rows[:,5]-t0)/1e5
wave = rows[:,3]; recs = rows[:,6]
lane = (wave==0)
t_q = start[lane].max() if tgate is None else tgate
rate=(end-start)/np.maximum(recs,1)
# pieces alive at t_q
alive = np.where(lane & (end > t_q) & (start <= t_q))[0]
done_before = end[~np.isin(np.arange(len(rows)), alive)].max()
# max-heap of pieces by end; min-heap of free lanes by time
pieces = [(-end[i], rate[i], 0) for i in alive]
heapq.heapify(pieces)
nlanes = 327680
free = [t_q]*(nlanes-len(alive))
# lanes also free when pieces end: approximate by pushing each alive piece's end as a future free time
ends = sorted(end[alive])
import bisect
fi = 0
freeh = free; heapq.heapify(freeh)
for e in ends: heapq.heappush(freeh, e)
cuts=0
while pieces and freeh:
    tf = heapq.heappop(freeh)
    ne, rr, nc = pieces[0]; en = -ne
    if tf >= en: continue
    left = en - tf
    if nc >= maxcuts or left <= 2*garb*rr + 0.1:
        # longest can't be cut further: nothing better for any lane
        break
    heapq.heappop(pieces)
    half = left/2
    heapq.heappush(pieces, (-(tf+half), rr, nc+1))
    heapq.heappush(pieces, (-(tf+half+garb*rr), rr, nc+1))
    heapq.heappush(freeh, tf+half+garb*rr)  # the cutting lane frees when its piece ends
    cuts+=1
final = max(done_before, -pieces[0][0] if pieces else 0)
print(sys.argv[1], f"gate {t_q:.1f} garbage {garb} maxcuts {maxcuts}: end {end.max():.1f} -> {final:.1f} ms ({cuts} cuts)")
