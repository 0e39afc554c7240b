"""Offline analysis of chain-launch item rows (scripts/chain_probe.py with CHAIN_ROWS=1): how far the
planner's stream-length estimate is from each pixel's true stream length, and what that does to the
last segments.
    python scripts/tail_analysis.py gpurun_out/chain_rows_8_7_plan.npz gpurun_out/chain_rows_8_7_exact.npz
The "exact" rows come from the plan whose pre-pass ran at full spp with no smoothing (RT_LPT_SPP=spp,
RT_COST_BUDGET=0, RT_CHAIN_SMOOTH=0): their pre-pass draw count is the pixel's true stream length.
Row columns (rt_hip.h: rt_scene_chain_diag): 0 pixel, 1 segment, 2 K, 3 whole-wave, 4/5 start/end
ticks, 6 records, 7 flags, 8/9 link t:c, 10 seg_len, 11 pre-pass draws, 12 pre-pass cost."""
import sys

import numpy as np

plan = np.load(sys.argv[1])["rows"].astype(np.int64)
exact = np.load(sys.argv[2])["rows"].astype(np.int64)
spp = int(sys.argv[3]) if len(sys.argv) > 3 else 1000
lpt = int(sys.argv[4]) if len(sys.argv) > 4 else 16

npx = int(max(plan[:, 0].max(), exact[:, 0].max())) + 1
true = np.zeros(npx)
true[exact[:, 0]] = exact[:, 11]          # the exact run: pre-pass at full spp = the stream length
pre = np.zeros(npx)
pre[plan[:, 0]] = plan[:, 11]             # the plan run's 16-spp pre-pass draws (extrapolated past the budget)
cost = np.zeros(npx)
cost[plan[:, 0]] = plan[:, 12]
tcost = np.zeros(npx)
tcost[exact[:, 0]] = exact[:, 12]

first = plan[(plan[:, 1] == 0)]
K = np.ones(npx, np.int64)
seg_len = np.zeros(npx)
K[first[:, 0]] = first[:, 2]
seg_len[first[:, 0]] = first[:, 10]
split = K > 1
est = seg_len * K
r = true[split] / np.maximum(est[split], 1)
print(f"pixels {npx}, split {split.sum()}; true / planned stream p1/p10/p50/p90/p99/p99.9: "
      f"{np.percentile(r, [1, 10, 50, 90, 99, 99.9]).round(3)}")
for lo, hi in ((2, 3), (3, 5), (5, 8), (8, 16), (16, 65)):
    k = split & (K >= lo) & (K < hi)
    if k.any():
        rr = true[k] / est[k]
        over = (true[k] - (K[k] - 1) * seg_len[k]) / seg_len[k]  # last segment's share, in segment lengths
        print(f"  K {lo:2d}-{hi - 1:2d}: {k.sum():6d} px  true/est p10/p50/p90/p99 {np.percentile(rr, [10, 50, 90, 99]).round(3)}"
              f"  last segment / seg_len p50/p90/p99/max {np.percentile(over, [50, 90, 99, 100]).round(2)}")

# the row neighbourhood estimators the planner could use (the share's rows are contiguous in the rows)
W = 1200
rows = npx // W
d16 = pre.reshape(rows, W) * lpt / spp  # back to the 16-spp draw counts (approximately, past the budget)
tr = true.reshape(rows, W)
def box(a, h):
    c = np.cumsum(np.pad(a, ((0, 0), (h + 1, h)), mode="edge"), axis=1)
    return (c[:, 2 * h + 1:] - c[:, :-2 * h - 1]) / (2 * h + 1)


for name, e in (("own", d16), ("+-1", box(d16, 1)), ("+-2", box(d16, 2)), ("+-4", box(d16, 4)), ("+-8", box(d16, 8)),
                ("max(own,+-4)", np.maximum(d16, box(d16, 4)))):
    q = (tr / np.maximum(e * spp / lpt, 1)).reshape(-1)[split]
    print(f"  estimator {name:13s} true/est p1/p10/p50/p90/p99: {np.percentile(q, [1, 10, 50, 90, 99]).round(3)}  "
          f"mean |log| {np.mean(np.abs(np.log(np.maximum(q, 1e-3)))):.4f}")

# the padded plan offline: K' = ceil(K pad) segments of seg_len for K >= k0
for pad in (1.0, 1.1, 1.2, 1.3, 1.5):
    for k0 in (4, 8):
        Kp = np.where(split & (K >= k0), np.minimum(np.ceil(K * pad), 32), K)
        reach = Kp * seg_len
        inside = true <= reach
        last = np.where(inside, true - np.floor(np.maximum(true - 1, 0) / np.maximum(seg_len, 1)) * seg_len,
                        true - (Kp - 1) * seg_len) / np.maximum(seg_len, 1)
        surplus = np.where(split, np.maximum(0, Kp - np.ceil(true / np.maximum(seg_len, 1))), 0)
        print(f"  pad {pad:.1f} K>={k0}: last real segment / seg_len p90/p99/p99.9/max "
              f"{np.percentile(last[split], [90, 99, 99.9, 100]).round(2)}  surplus segments {int(surplus.sum())} "
              f"(+{surplus.sum() / max(1, K[split].sum()) * 100:.1f} % of the split pixels' segments)")
