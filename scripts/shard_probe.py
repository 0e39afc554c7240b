"""Time each rank's share of the headline frame on one GPU (rows j % world == rank), as bench.py's
N-GPU run would give it; with the RT_* variant knobs in the environment.
    python scripts/shard_probe.py WORLDS [RANKS|all] [SPP]      e.g.  2,4,8 all 1000
The N-GPU frame time is the max over ranks; "scale" is (1-GPU frame time) / (that max)."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "ray-tracing-c_amd"))
import torch  # noqa: E402  (initialised before rtc: see rtc._init_torch_runtime_first)
import rtc  # noqa: E402

worlds = [int(w) for w in sys.argv[1].split(",")]
ranks_arg = sys.argv[2] if len(sys.argv) > 2 else "0"
spp = int(sys.argv[3]) if len(sys.argv) > 3 else 1000
# RTC_DIAG=1: the diagnostic build (librtc_amd_diag.so), which reads the A/B switches (RT_CHAIN_PAD ...)
with rtc.use_diag(os.environ.get("RTC_DIAG") == "1"):
    sc = rtc.Scene.preset(1, 1200, spp, 50)
    ds = rtc.DeviceScene(sc, 0)
st = torch.cuda.current_stream()


REPS = int(os.environ.get("SHARD_REPS", "3"))


def time_rows(row0, stride, n, reps=REPS):
    """Best wall / kernel time of `reps` launches after a warm-up; every rep is printed (rng)."""
    global last, walls, kerns
    buf = torch.empty((n, sc.width, 3), dtype=torch.uint8, device="cuda")
    ds.render_rows_async(row0, stride, n, buf.data_ptr(), st.cuda_stream)  # warm-up
    torch.cuda.synchronize()
    walls, kerns = [], []
    for _ in range(reps):
        t0 = time.perf_counter()
        ds.render_rows_async(row0, stride, n, buf.data_ptr(), st.cuda_stream)
        torch.cuda.synchronize()
        walls.append(time.perf_counter() - t0)
        ds.check()  # every work item finished
        kerns.append(ds.last_launch_ms())
    last = buf.cpu().numpy()
    return min(walls), min(kerns)


def rng():
    return f"(reps ms {'/'.join(f'{w * 1e3:.1f}' for w in walls)}; kernel {'/'.join(f'{k:.1f}' for k in kerns)})"


print(f"build={ds._L.rt_build_id().decode()} box={rtc.box_identity(0)} "
      f"env={ {k: v for k, v in os.environ.items() if k.startswith('RT_') or k == 'RTC_DIAG'} }", flush=True)
t1, k1 = time_rows(0, 1, sc.height)
full = last
print(f"world=1 ms={t1 * 1e3:.1f} kernel_ms={k1:.1f} Msamples/s={sc.width * sc.height * spp / t1 / 1e6:.0f} {rng()}", flush=True)
for world in worlds:
    ranks = range(world) if ranks_arg == "all" else [int(r) for r in ranks_arg.split(",")]
    worst = 0.0
    for rank in ranks:
        row0, stride, n = rtc.rows_of(sc.height, rank, world)
        t, k = time_rows(row0, stride, n)
        worst = max(worst, t)
        same = bool((last == full[row0::stride][:n]).all())  # rows identical to the 1-GPU frame
        print(f"  world={world} rank={rank} rows={n} ms={t * 1e3:.1f} kernel_ms={k:.1f} identical={same} {rng()}", flush=True)
    print(f"world={world} max_ms={worst * 1e3:.1f} frame_Msamples/s={sc.width * sc.height * spp / worst / 1e6:.0f} "
          f"scale={t1 / worst:.2f}x", flush=True)
ds.close()
