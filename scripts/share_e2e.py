"""End to end of one rank's share through the drop-in path, beside its step time.

    python scripts/share_e2e.py [SHARES]      e.g.  8:7,2:1,1:0   (n_shares:share, default that)

For each share, on one GPU:
  cold   rt_render_share with RT_SCENE_CACHE=0: what every Camera_render did until r06 -- host pack,
         upload, allocations (the record arena), the launch (pre-pass, plan, record fill, chain kernel,
         fold), D2H of the rows, completion check; the scene is freed again;
  first  the same with the cache on, from an empty cache (a process's first Camera_render);
  warm   repeated calls with the cache on (every later Camera_render of the same world);
  step   the share's launch on a persistent DeviceScene, synchronised (shard_probe.py's number).
Every rendered share is compared with the same rows of the one-GPU frame (identical=...)."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "ray-tracing-c_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402  (initialised before rtc: rtc._init_torch_runtime_first)
import rtc  # noqa: E402

shares = [tuple(int(x) for x in s.split(":")) for s in (sys.argv[1] if len(sys.argv) > 1 else "8:7,2:1,1:0").split(",")]
spp = int(os.environ.get("E2E_SPP", "1000"))
reps = int(os.environ.get("E2E_REPS", "3"))
sc = rtc.Scene.preset(1, 1200, spp, 50)
print(f"build={rtc.build_id()} box={rtc.box_identity(0)} spp={spp}", flush=True)

full = rtc.render(sc, n_gpus=1)  # the one-GPU frame (also warms the code objects)
rtc.release_cache()


def fmt(p):
    return f"total {p['total']:.1f} (setup {p['setup']:.1f} run {p['run']:.1f} d2h {p['d2h']:.1f})"


ds = rtc.DeviceScene(sc, 0)
st = torch.cuda.current_stream()
for G, g in shares:
    row0, stride, n = rtc.rows_of(sc.height, g, G)
    out = np.zeros_like(full)
    res = {}
    os.environ["RT_SCENE_CACHE"] = "0"
    cold = []
    for _ in range(2):
        t0 = time.perf_counter()
        rtc.render_share(sc, g, G, 0, out)
        cold.append(((time.perf_counter() - t0) * 1e3, rtc.last_share_ms(g)))
    os.environ["RT_SCENE_CACHE"] = "1"
    rtc.release_cache()
    t0 = time.perf_counter()
    rtc.render_share(sc, g, G, 0, out)
    first = ((time.perf_counter() - t0) * 1e3, rtc.last_share_ms(g))
    warm = []
    for _ in range(reps):
        t0 = time.perf_counter()
        rtc.render_share(sc, g, G, 0, out)
        warm.append(((time.perf_counter() - t0) * 1e3, rtc.last_share_ms(g)))
    same = bool((out[row0::stride][:n] == full[row0::stride][:n]).all())
    rtc.release_cache()
    # the persistent scene's step, as shard_probe.py times it
    buf = torch.empty((n, sc.width, 3), dtype=torch.uint8, device="cuda")
    ds.render_rows_async(row0, stride, n, buf.data_ptr(), st.cuda_stream)
    torch.cuda.synchronize()
    steps = []
    for _ in range(reps):
        t0 = time.perf_counter()
        ds.render_rows_async(row0, stride, n, buf.data_ptr(), st.cuda_stream)
        torch.cuda.synchronize()
        steps.append((time.perf_counter() - t0) * 1e3)
    ds.check()
    step_same = bool((buf.cpu().numpy() == full[row0::stride][:n]).all())
    best_warm = min(w[0] for w in warm)
    print(f"share {g}/{G} rows={n} identical={same and step_same}\n"
          f"  step  ms {min(steps):.1f} (reps {'/'.join(f'{s:.1f}' for s in steps)})\n"
          f"  cold  ms {'/'.join(f'{c[0]:.1f}' for c in cold)}: {fmt(cold[-1][1])}\n"
          f"  first ms {first[0]:.1f}: {fmt(first[1])}\n"
          f"  warm  ms {best_warm:.1f} (reps {'/'.join(f'{w[0]:.1f}' for w in warm)}): {fmt(warm[-1][1])}\n"
          f"  warm - step {best_warm - min(steps):+.2f} ms, cold - step {min(c[0] for c in cold) - min(steps):+.2f} ms",
          flush=True)
ds.close()
