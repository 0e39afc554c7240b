"""Where a slow headline launch loses its time: LAUNCHES back-to-back chain launches of the
headline frame on the diagnostic build with item timelines (RT_PX_TIME=1); every launch's kernel ms, and
for the slowest and the median launch the lane slots in use over time, the migration counts and the items
that end last.  The rows of both are saved (gpurun_out/slow_rows_<world>_<rank>_{slow,median}.npz) for tail_bound.py.
    python scripts/slow_launch_probe.py [LAUNCHES] [SPP] [WORLD RANK]   (a rank's share: rows j % WORLD == RANK)"""
import os
import sys

os.environ["RT_PX_TIME"] = "1"
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "ray-tracing-c_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import rtc  # noqa: E402

launches = int(sys.argv[1]) if len(sys.argv) > 1 else 12
spp = int(sys.argv[2]) if len(sys.argv) > 2 else 1000
world, rank = (int(sys.argv[3]), int(sys.argv[4])) if len(sys.argv) > 4 else (1, 0)
with rtc.use_diag():
    sc = rtc.Scene.preset(1, 1200, spp, 50)
    ds = rtc.DeviceScene(sc, 0)
row0, stride, nrows = rtc.rows_of(sc.height, rank, world)
buf = torch.empty((nrows, sc.width, 3), dtype=torch.uint8, device="cuda")
st = torch.cuda.current_stream()
print(f"build={ds._L.rt_build_id().decode()} (diag) box={rtc.box_identity(0)} world={world} rank={rank}", flush=True)
kept = []  # (kernel ms, launch, rows): 52 MB of rows per launch
for k in range(launches):
    ds.render_rows_async(row0, stride, nrows, buf.data_ptr(), st.cuda_stream)
    torch.cuda.synchronize()
    ds.check()
    ms = ds.last_launch_ms()
    kept.append((ms, k, ds.chain_diag(sc.width * nrows * 64)))
    print(f"launch {k}: kernel_ms={ms:.1f}", flush=True)
kept.sort(key=lambda e: -e[0])
out = os.path.join(os.environ.get("GRAFT_REPO_ROOT", "."), "gpurun_out")


def describe(tag, ms, k, rows):
    r = rows.astype(np.int64)
    t0 = r[:, 4].min()
    start, end = (r[:, 4] - t0) / 1e5, (r[:, 5] - t0) / 1e5
    mig = np.where(r[:, 13] > 0, (r[:, 13] - t0) / 1e5, np.nan)
    np.savez_compressed(os.path.join(out, f"slow_rows_{world}_{rank}_{tag}.npz"), rows=rows)
    w = np.where(r[:, 3] >= 1, 64, 1)
    ts = np.arange(round(0.6 * end.max() / 5.0) * 5.0, end.max() + 5.0, 5.0)
    inflight = [int(w[(start <= t) & (end > t)].sum()) for t in ts]
    print(f"{tag} launch {k}: kernel_ms={ms:.1f} last item end {end.max():.1f} ms; migrated "
          f"{int(np.isfinite(mig).sum())} at p50/p90/max {np.nanpercentile(mig, [50, 90, 100]).round(1)} ms", flush=True)
    print(f"  lane slots in use from {ts[0]:.0f} ms, every 5 ms: " + " ".join(f"{t:.0f}:{v // 1000}k" for t, v in zip(ts, inflight)))
    unsplit = r[:, 2] == 1
    print(f"  unsplit items {int(unsplit.sum())}: start max {start[unsplit].max():.1f}, duration p50/p99/max "
          f"{np.percentile((end - start)[unsplit], [50, 99, 100]).round(1)} ms")
    print("  last to finish: (pixel, seg/K, start ms, end ms, migrated ms, records)")
    for q in np.argsort(-end)[:8]:
        print(f"    {r[q, 0]:7d} {r[q, 1] & 0xffff}/{r[q, 2]} {start[q]:7.1f} {end[q]:7.1f} {mig[q]:7.1f} {r[q, 6]:5d}")


describe("slow", *kept[0])
describe("median", *kept[len(kept) // 2])
