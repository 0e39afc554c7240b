"""Bounds of a chain launch from its item rows (scripts/chain_probe.py with CHAIN_ROWS=1; columns as in
rt_hip.h rt_scene_chain_diag): what the launch would take if its lanes were never idle, at the per-sample
latencies the rows measured.
    python scripts/tail_bound.py ROWS.npz LANES [PREPASS_MS]
LANES: lane slots of the launch's grid (waves resident x 64; e.g. 262144 for 4 waves per SIMD on 256 CUs).
Prints:
  * capacity bound  = total lane-busy time / lanes   (every lane busy until the end: the packing limit);
  * critical path   = the longest chain any pixel could be cut into under the planner's segment cap
                      (kmax_lane) at its own measured latency, + the coupling overhead (5 garbage samples)
    -- the launch can end no earlier than the larger of the two;
  * the measured end, and how the lanes were used over time (in flight every 5 ms)."""
import sys

import numpy as np

rows = np.load(sys.argv[1])["rows"].astype(np.int64)
lanes = int(sys.argv[2])
prepass = float(sys.argv[3]) if len(sys.argv) > 3 else 0.0
spp, kmax, garbage = 1000, 32, 5

t0 = rows[:, 4].min()
start = (rows[:, 4] - t0) / 1e5  # wall_clock64 ticks, 100 MHz -> ms
end = (rows[:, 5] - t0) / 1e5
width = np.where(rows[:, 3] >= 1, 64, 1)  # whole-wave items hold 64 lane slots
busy = ((end - start) * width).sum()
cap = busy / lanes
# per pixel: ms per sample on a lane (its lane items, before any migration)
lane_items = (rows[:, 3] == 0) & (rows[:, 13] == 0) & (rows[:, 6] > 0)
lat = np.zeros(int(rows[:, 0].max()) + 1)
np.maximum.at(lat, rows[lane_items, 0], (end - start)[lane_items] / rows[lane_items, 6])
crit = (lat * (spp / kmax + garbage)).max()
pe = np.zeros_like(lat)
np.maximum.at(pe, rows[:, 0], end)
print(f"{sys.argv[1]}: items {len(rows)}, pixels {int((pe > 0).sum())}, lane slots {lanes}")
print(f"  measured end {end.max():.1f} ms (+ {prepass:.1f} ms pre-pass / plan / fold)")
print(f"  capacity bound {cap:.1f} ms = {busy / 1e3:.0f} lane-s busy / {lanes} lanes; critical path {crit:.1f} ms "
      f"(slowest pixel {lat.max() * 1e3:.0f} us per sample x ({spp}/{kmax} + {garbage}))")
print(f"  packing efficiency (capacity bound / measured end) {cap / end.max():.2f}")
print(f"  pixel completion p50/p90/p99/p99.9/max {np.percentile(pe[pe > 0], [50, 90, 99, 99.9, 100]).round(1)} ms")
ts = np.arange(0.0, end.max() + 5.0, 5.0)
inflight = [int(width[(start <= t) & (end > t)].sum()) for t in ts]
print("  lane slots in use every 5 ms: " + " ".join(f"{t:.0f}:{100 * v / lanes:.0f}%" for t, v in zip(ts, inflight)))
