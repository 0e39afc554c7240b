"""Timeline of one chain launch (RT_PX_TIME=1 diagnostic of the diagnostic build librtc_amd_diag.so):
every work item's start / end, by kind (unsplit lane pixel, lane segment, whole-wave segment), and the
items that finish last.
    python scripts/chain_probe.py WORLD RANK [SPP]       (RT_* knobs from the environment)"""
import os
import sys
import time

os.environ["RT_PX_TIME"] = "1"
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "ray-tracing-c_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import rtc  # noqa: E402

world, rank = int(sys.argv[1]), int(sys.argv[2])
spp = int(sys.argv[3]) if len(sys.argv) > 3 else 1000
with rtc.use_diag():
    sc = rtc.Scene.preset(1, 1200, spp, 50)
    ds = rtc.DeviceScene(sc, 0)
row0, stride, n = rtc.rows_of(sc.height, rank, world)
buf = torch.empty((n, sc.width, 3), dtype=torch.uint8, device="cuda")
st = torch.cuda.current_stream()
for _ in range(2):
    t0 = time.perf_counter()
    ds.render_rows_async(row0, stride, n, buf.data_ptr(), st.cuda_stream)
    torch.cuda.synchronize()
    t = time.perf_counter() - t0
rows = ds.chain_diag(n * sc.width * 64)
m = len(rows)
r = rows.astype(np.int64)
t0 = r[:, 4].min()
start = (r[:, 4] - t0) / 1e5  # wall_clock64: 100 MHz -> ms
end = (r[:, 5] - t0) / 1e5
print(f"build={ds._L.rt_build_id().decode()} (diag) box={rtc.box_identity(0)}", flush=True)
print(f"world={world} rank={rank} ms={t * 1e3:.1f} kernel_ms={ds.last_launch_ms():.1f} items={m} "
      f"last_end={end.max():.1f} ms", flush=True)
kinds = {"unsplit lane": (r[:, 2] == 1) & (r[:, 3] == 0), "unsplit wave": (r[:, 2] == 1) & (r[:, 3] == 1),
         "segment lane": (r[:, 2] > 1) & (r[:, 3] == 0), "segment wave": (r[:, 2] > 1) & (r[:, 3] == 1)}
for name, k in kinds.items():
    if k.any():
        d = end[k] - start[k]
        print(f"  {name:13s} items {k.sum():7d}  end p50/p90/p99/max {np.percentile(end[k], [50, 90, 99, 100]).round(1)} ms"
              f"  start max {start[k].max():.1f}  duration p50/p99/max {np.percentile(d, [50, 99, 100]).round(1)}"
              f"  records p50/max {np.percentile(r[k, 6], [50, 100])}", flush=True)
# coupling: per split pixel, samples computed (head samples + every record) against spp
sp = (r[:, 2] > 1) & (r[:, 3] < 2)  # planned segments
if sp.any():
    pix = r[sp, 0]
    tot = np.bincount(pix, weights=r[sp, 6])
    Kp = np.zeros_like(tot); Kp[pix] = r[sp, 2]
    has = Kp > 0
    infl = tot[has] / spp
    print(f"  split pixels {has.sum()}: samples/spp p50/p90/p99/max {np.percentile(infl, [50, 90, 99, 100]).round(3)}", flush=True)
    mid = sp & (r[:, 1] + 1 < r[:, 2])
    nc = mid & ((r[:, 7] & 1) == 0)
    print(f"  non-last segments {mid.sum()}: not coupled {nc.sum()}  (records p50/max of those "
          f"{np.percentile(r[nc, 6], [50, 100]) if nc.any() else '-'})", flush=True)
    cpl = sp & ((r[:, 7] & 1) == 1) & (r[:, 8] > 0)
    print(f"  link record (successor's garbage samples) p50/p90/p99/max {np.percentile(r[cpl, 9], [50, 90, 99, 100])}", flush=True)
    lastseg = sp & (r[:, 1] + 1 == r[:, 2])
    ratio = r[lastseg, 6] / (spp / r[lastseg, 2])
    print(f"  last segments: records / (spp/K) p50/p90/p99/max {np.percentile(ratio, [50, 90, 99, 100]).round(2)}", flush=True)
# items in flight over time (lanes: 64 per wave of the grid); whole-wave items count 64
ts = np.arange(0.0, end.max() + 5.0, 5.0)
w = np.where(r[:, 3] >= 1, 64, 1)
inflight = [int(w[(start <= t) & (end > t)].sum()) for t in ts]
print("  lane-equivalents in flight every 5 ms: " + " ".join(f"{t:.0f}:{v // 1000}k" for t, v in zip(ts, inflight)), flush=True)
last = np.argsort(-end)[:16]
mig = np.where(r[:, 13] > 0, (r[:, 13] - t0) / 1e5, np.nan)
print(f"  migrated to helper waves: {int(np.isfinite(mig).sum())} items, at p50/p90/max "
      f"{np.nanpercentile(mig, [50, 90, 100]).round(1) if np.isfinite(mig).any() else '-'} ms", flush=True)
print("  last to finish: (item, pixel, seg/K, wave, start ms, end ms, migrated ms, records, flags, link t:c, seg_len, pre-pass draws)")
for q in last:
    print(f"    {q:7d} {r[q, 0]:7d} {r[q, 1]}/{r[q, 2]} {r[q, 3]} {start[q]:7.1f} {end[q]:7.1f} {mig[q]:7.1f} {r[q, 6]:5d} {r[q, 7]} "
          f"{r[q, 8]}:{r[q, 9]} {r[q, 10]} {r[q, 11]}")
if os.environ.get("CHAIN_ROWS"):  # the item rows for offline analysis (uint32, compressed)
    np.savez_compressed(os.path.join(os.environ.get("GRAFT_REPO_ROOT", "."), "gpurun_out", f"chain_rows_{world}_{rank}{os.environ.get('CHAIN_TAG', '')}.npz"),
                        rows=rows)
ds.close()
