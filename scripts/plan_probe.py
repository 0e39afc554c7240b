"""The chain plan of one launch per share (diagnostic build, RT_DEBUG=1: the library prints the plan --
items, split pixels, records reserved against the arena's capacity -- and the launch's phase times).
    python scripts/plan_probe.py [SHARES]      e.g.  1:0,2:1,8:7   (n_shares:share)"""
import os
import sys

os.environ["RT_DEBUG"] = "1"
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "ray-tracing-c_amd"))
import torch  # noqa: E402
import rtc  # noqa: E402

shares = [tuple(int(x) for x in s.split(":")) for s in (sys.argv[1] if len(sys.argv) > 1 else "1:0,2:1,8:7").split(",")]
with rtc.use_diag():
    sc = rtc.Scene.preset(1, 1200, 1000, 50)
    ds = rtc.DeviceScene(sc, 0)
st = torch.cuda.current_stream()
for G, g in shares:
    row0, stride, n = rtc.rows_of(sc.height, g, G)
    buf = torch.empty((n, sc.width, 3), dtype=torch.uint8, device="cuda")
    print(f"== share {g}/{G}: {n} rows, {n * sc.width} pixels", file=sys.stderr, flush=True)
    ds.render_rows_async(row0, stride, n, buf.data_ptr(), st.cuda_stream)
    torch.cuda.synchronize()
    ds.check()
ds.close()
