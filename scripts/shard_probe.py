"""Time one rank's share of the headline frame on one GPU (rows j % world == rank), as bench.py's
N-GPU run would give it; with the RT_* variant knobs in the environment.
    python scripts/shard_probe.py WORLD [RANK] [SPP]"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "ray-tracing-c_amd"))
import torch  # noqa: E402  (initialised before rtc: see rtc._init_torch_runtime_first)
import rtc  # noqa: E402

world = int(sys.argv[1])
rank = int(sys.argv[2]) if len(sys.argv) > 2 else 0
spp = int(sys.argv[3]) if len(sys.argv) > 3 else 1000
sc = rtc.Scene.preset(1, 1200, spp, 50)
row0, stride, n = rtc.rows_of(sc.height, rank, world)
ds = rtc.DeviceScene(sc, 0)
buf = torch.empty((n, sc.width, 3), dtype=torch.uint8, device="cuda")
st = torch.cuda.current_stream()
ds.render_rows_async(row0, stride, n, buf.data_ptr(), st.cuda_stream)  # warm-up
torch.cuda.synchronize()
times = []
for _ in range(2):
    t0 = time.perf_counter()
    ds.render_rows_async(row0, stride, n, buf.data_ptr(), st.cuda_stream)
    torch.cuda.synchronize()
    times.append(time.perf_counter() - t0)
t = min(times)
print(f"world={world} rank={rank} rows={n} ms={t * 1e3:.1f} kernel_ms={ds.last_launch_ms():.1f} "
      f"frame_Msamples/s_if_all_ranks_equal={sc.width * sc.height * spp / t / 1e6:.0f}", flush=True)
ds.close()
