"""Frame time of one preset scene on one GPU under several RT_* settings (one process, one library:
RTC_LIB picks the build), with the image checked identical across settings.
    python scripts/scene_time.py SCENE WIDTH SPP "ENV;ENV;..." [REPS]
ENV is comma-separated K=V pairs ("" = defaults), e.g.  7 1000 256 ";RT_GEN_RARE=1;RT_GEN_RARE=16"
The library reads its RT_* configuration when a scene is uploaded, so each setting gets a fresh
upload of the same scene.  The A/B switches are read by the diagnostic build only (librtc_amd_diag.so,
used here unless RTC_LIB names another build)."""
import hashlib
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "ray-tracing-c_amd"))
import torch  # noqa: E402  (initialised before rtc: see rtc._init_torch_runtime_first)
import rtc  # noqa: E402

scene, width, spp = (int(x) for x in sys.argv[1:4])
settings = sys.argv[4].split(";") if len(sys.argv) > 4 else [""]
reps = int(sys.argv[5]) if len(sys.argv) > 5 else 2
diag = rtc.use_diag(not os.environ.get("RTC_LIB"))
with diag:
    sc = rtc.Scene.preset(scene, width, spp, 50, substitute_earth=True)
st = torch.cuda.current_stream()
buf = torch.empty((sc.height, sc.width, 3), dtype=torch.uint8, device="cuda")
base = {k: os.environ.get(k) for s in settings for k in (kv.split("=")[0] for kv in s.split(",") if kv)}
ref_sha = None
for s in settings:
    for k, v in base.items():  # back to the process environment, then this setting
        if v is None:
            os.environ.pop(k, None)
        else:
            os.environ[k] = v
    for kv in (x for x in s.split(",") if x):
        k, v = kv.split("=", 1)
        os.environ[k] = v
    with diag:
        ds = rtc.DeviceScene(sc, 0)
    ds.render_rows_async(0, 1, sc.height, buf.data_ptr(), st.cuda_stream)  # warm-up
    torch.cuda.synchronize()
    best, kbest = 1e30, 1e30
    for _ in range(reps):
        t0 = time.perf_counter()
        ds.render_rows_async(0, 1, sc.height, buf.data_ptr(), st.cuda_stream)
        torch.cuda.synchronize()
        best = min(best, time.perf_counter() - t0)
        kbest = min(kbest, ds.last_launch_ms())
    sha = hashlib.sha256(buf.cpu().numpy().tobytes()).hexdigest()
    ref_sha = ref_sha or sha
    print(f"scene={scene} {sc.width}x{sc.height}x{spp} [{s or 'default'}] ms={best * 1e3:.1f} kernel_ms={kbest:.1f} "
          f"Msamples/s={sc.width * sc.height * spp / best / 1e6:.1f} sha={sha[:12]} same={sha == ref_sha}", flush=True)
    ds.close()
