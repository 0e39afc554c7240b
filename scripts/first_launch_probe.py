"""Where the slow first launch comes from: the headline frame's chain kernel, launch by launch,
on a first device scene, then on a second one uploaded afterwards (fresh HBM allocations, the kernel code
already loaded), then again on the first.
    python scripts/first_launch_probe.py [SPP] [LAUNCHES]
Prints each launch's kernel ms (rt_scene_last_launch_ms) and wall ms."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "ray-tracing-c_amd"))
import torch  # noqa: E402  (initialised before rtc: see rtc._init_torch_runtime_first)
import rtc  # noqa: E402

spp = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
launches = int(sys.argv[2]) if len(sys.argv) > 2 else 3
sc = rtc.Scene.preset(1, 1200, spp, 50)
st = torch.cuda.current_stream()
buf = torch.empty((sc.height, sc.width, 3), dtype=torch.uint8, device="cuda")
print(f"build={rtc.build_id()} box={rtc.box_identity(0)}", flush=True)


def run(ds, tag):
    for k in range(launches):
        t0 = time.perf_counter()
        ds.render_rows_async(0, 1, sc.height, buf.data_ptr(), st.cuda_stream)
        torch.cuda.synchronize()
        ds.check()
        print(f"{tag} launch {k}: kernel_ms={ds.last_launch_ms():.1f} wall_ms={1e3 * (time.perf_counter() - t0):.1f}",
              flush=True)


a = rtc.DeviceScene(sc, 0)
run(a, "scene A (first in the process)")
b = rtc.DeviceScene(sc, 0)
run(b, "scene B (uploaded second: fresh allocations)")
run(a, "scene A again")
b.close()
a.close()
