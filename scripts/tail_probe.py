"""Where the frame's time goes, per work item: start/end of every pixel of one rank's share of the
headline frame (RT_PX_TIME=1 diagnostic), against its pre-pass cost and its mode (whole wave or lane).
    python scripts/tail_probe.py WORLD RANK [SPP]     (RT_* knobs from the environment)
Prints the last-finishing items, the per-mode finish-time profile and the clocks per pre-pass step."""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "ray-tracing-c_amd"))
os.environ["RT_PX_TIME"] = "1"
import torch  # noqa: E402  (initialised before rtc: see rtc._init_torch_runtime_first)
import rtc  # noqa: E402

world, rank = int(sys.argv[1]), int(sys.argv[2])
spp = int(sys.argv[3]) if len(sys.argv) > 3 else 1000
L = rtc.lib()
L.rt_scene_px_time.argtypes = [ctypes.c_void_p] * 5 + [ctypes.c_int64]
sc = rtc.Scene.preset(1, 1200, spp, 50)
row0, stride, n_rows = rtc.rows_of(sc.height, rank, world)
ds = rtc.DeviceScene(sc, 0)
buf = torch.empty((n_rows, sc.width, 3), dtype=torch.uint8, device="cuda")
st = torch.cuda.current_stream()
for _ in range(2):
    ds.render_rows_async(row0, stride, n_rows, buf.data_ptr(), st.cuda_stream)
    torch.cuda.synchronize()
n = n_rows * sc.width
times = np.zeros(2 * n, dtype=np.uint32)
cost = np.zeros(n, dtype=np.uint32)
order = np.zeros(n, dtype=np.int32)
ncoop = np.zeros(1, dtype=np.uint32)
assert L.rt_scene_px_time(ds._h, times.ctypes.data, cost.ctypes.data, order.ctypes.data, ncoop.ctypes.data, n) == 0
t0, t1 = times[0::2].astype(np.int64), times[1::2].astype(np.int64)
base = t0.min()
start, end = (t0 - base) / 1e5, (t1 - base) / 1e5  # ms (wall_clock64 runs at 100 MHz)
coop = np.zeros(n, dtype=bool)
coop[order[: int(ncoop[0])]] = True
lpt_spp = int(os.environ.get("RT_LPT_SPP", "8"))
steps = cost.astype(np.float64) * spp / lpt_spp  # estimated frame steps per item
dur = end - start
print(f"world={world} rank={rank} items={n} whole-wave={int(coop.sum())} kernel_ms={ds.last_launch_ms():.1f} "
      f"frame_end_ms={end.max():.1f}")
for name, m in (("lane", ~coop), ("wave", coop)):
    if not m.any():
        continue
    clk = dur[m] * 2.4e6 / np.maximum(steps[m], 1)  # ~2.4 GHz shader clock per estimated step
    print(f"  {name}: items {int(m.sum())}, end p50/p90/p99/max {np.percentile(end[m], [50, 90, 99, 100]).round(1)} ms, "
          f"start max {start[m].max():.1f} ms, clocks/step p50/p90 {np.percentile(clk, [50, 90]).round(0)}")
nc = int(ncoop[0])
if nc:
    head = order[: min(nc, 8)]
    print("  whole-wave order head (item, pre-pass steps/sample, start ms, end ms):",
          [(int(k), round(float(cost[k]) / lpt_spp), round(float(start[k]), 1), round(float(end[k]), 1)) for k in head])
    print(f"  whole-wave start min {start[coop].min():.1f} ms; heaviest whole-wave item at order position "
          f"{int(np.argmax(cost[order[:nc]]))}")
last = np.argsort(-end)[:12]
print("  last to finish: (item, mode, pre-pass steps/sample, start ms, end ms)")
for k in last:
    print(f"    {k:7d} {'wave' if coop[k] else 'lane'} {cost[k] / lpt_spp:8.0f} {start[k]:7.1f} {end[k]:7.1f}")
ds.close()
