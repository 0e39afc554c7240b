"""Where a chain launch's tail comes from, from its item rows (scripts/chain_probe.py with CHAIN_ROWS=1;
columns as in rt_hip.h rt_scene_chain_diag) -- VERDICT r05 item 1.
    python scripts/tail_attrib.py ROWS.npz LANES [SPP]

1. The floor.  Capacity bound = lane-busy time / lane slots (no lane ever idle).  Per pixel, the fastest
   its samples could run: on lanes, cut into at most kmax segments at its own measured per-sample lane
   latency (+5 garbage samples per cut), or on whole waves at the helpers' measured ray latency (6.9 k
   clocks = 2.9 us per ray) x its rays per sample x spp / kmax_wave (whole-wave items hold
   at most 8 segments) -- the smaller of the two.  The launch can end no earlier than
   max(capacity bound, the largest per-pixel floor).
2. The tail.  From the moment the lane slots stop being all busy (t_full) to the end, the idle slot area;
   and how much of the launch's end each class of late item explains: every item is given the duration
   it would have had at its planned share (spp / K records + 5 garbage samples, at its own per-sample
   latency), one class at a time, and the launch's end recomputed:
     overrun last   last segments that wrote > 1.25x their share (the stream-length estimate's error);
     late coupling  non-last segments that wrote > 1.25x their share (they coupled late: a parity trap of
                    theirs or their successor's garbage prefix);
     whole pixels   unsplit items (K = 1) -- the planner kept them whole;
   "end if all" removes all three."""
import sys

import numpy as np

rows = np.load(sys.argv[1])["rows"].astype(np.int64)
lanes = int(sys.argv[2])
spp = int(sys.argv[3]) if len(sys.argv) > 3 else 1000
kmax, kmax_wave, garbage = 32, 8, 5
clk_ray_us = 6.9e3 / 2.4e3  # helper whole-wave ray, DESIGN.md §4.2 (dfa8efbf)

t0 = rows[:, 4].min()
start = (rows[:, 4] - t0) / 1e5
end = (rows[:, 5] - t0) / 1e5
dur = end - start
pix, seg, K, wave, recs = rows[:, 0], rows[:, 1], rows[:, 2], rows[:, 3], rows[:, 6]
mig = rows[:, 13] > 0
width = np.where(wave >= 1, 64, 1)
busy = (dur * width).sum()
cap = busy / lanes
T = end.max()

# per pixel: measured lane latency per sample (lane items before migration), and rays per sample
npx = int(pix.max()) + 1
lane_items = (wave == 0) & ~mig & (recs > 0)
lat = np.zeros(npx)
np.maximum.at(lat, pix[lane_items], dur[lane_items] / recs[lane_items])
draws = np.zeros(npx)
draws[pix] = rows[:, 11]
rays = np.maximum(1.0, (draws / 64.0 - 2.0) / 2.0 + 1.0)  # pre-pass draws per sample (64 spp): 2 jitter + ~2 per bounce
floor_lane = lat * (spp / kmax + garbage)
floor_wave = rays * clk_ray_us * 1e-3 * (spp / kmax_wave + garbage) * 1.5  # (+50 %: shading and protocol, §4.2)
floor_px = np.where(lat > 0, np.minimum(floor_lane, floor_wave), 0.0)
print(f"{sys.argv[1]}: items {len(rows)}, lane slots {lanes}, measured end {T:.1f} ms")
print(f"  capacity bound {cap:.1f} ms; per-pixel floor max {floor_px.max():.1f} ms "
      f"(lane-only floor max {floor_lane.max():.1f} ms); floor = {max(cap, floor_px.max()):.1f} ms, "
      f"packing {cap / T:.2f}")

# the tail: idle slot area after the slots stop being all busy
ts = np.arange(0.0, T + 0.25, 0.25)
inflight = np.array([width[(start <= t) & (end > t)].sum() for t in ts])
full = ts[inflight >= 0.98 * lanes]
t_full = full.max() if len(full) else 0.0
idle = ((lanes - inflight[ts >= t_full]) * 0.25).sum() / 1e3  # lane-s
print(f"  all slots busy until {t_full:.1f} ms; idle slot area after it {idle:.1f} lane-s "
      f"= {idle * 1e3 / lanes:.1f} ms of the whole grid")

share = np.where(K > 1, spp / np.maximum(K, 1), spp).astype(float)
ratio = recs / share
per = np.where(recs > 0, dur / np.maximum(recs, 1), 0.0)
planned = per * (share + garbage)
last = (K > 1) & (seg == K - 1)
classes = {
    "overrun last": last & (ratio > 1.25) & (wave == 0),
    "late coupling": (K > 1) & ~last & (ratio > 1.25) & (wave == 0),
    "whole pixels": (K == 1) & (wave == 0),
}


def end_with(mask):
    e = end.copy()
    m = mask & (planned < dur)
    e[m] = start[m] + planned[m]
    return e.max()


late = end > t_full
print(f"  items ending after t_full: {int(late.sum())}; by class (items, of them after t_full, lane-s after t_full, "
      f"launch end if that class ran to plan):")
for name, m in classes.items():
    area = (np.clip(end[m], t_full, None) - np.clip(start[m], t_full, None)).clip(0).sum() / 1e3
    print(f"    {name:14s} {int(m.sum()):7d} {int((m & late).sum()):6d}  {area:7.2f} lane-s   end {end_with(m):5.1f} ms")
allm = np.zeros_like(late)
for m in classes.values():
    allm |= m
print(f"    {'end if all':14s} {'':7s} {'':6s}  {'':7s}          end {end_with(allm):5.1f} ms")
# the last 20 pixels to complete: class of their latest item
pe = np.zeros(npx)
np.maximum.at(pe, pix, end)
order = np.argsort(-pe)[:20]
print("  last pixels: pixel end_ms K latest-item(seg, records/share, start, migrated) own-cost lat_us/sample floor_ms")
for p in order:
    it = np.where(pix == p)[0]
    j = it[np.argmax(end[it])]
    mt = (rows[j, 13] - t0) / 1e5 if mig[j] else float("nan")
    print(f"    {p:7d} {pe[p]:5.1f} {K[j]:3d} ({seg[j]:2d}, {ratio[j]:4.2f}, {start[j]:4.1f}, {mt:4.1f}) "
          f"{rows[j, 12]:6d} {lat[p] * 1e3:6.1f} {floor_px[p]:5.1f}")
