"""Repeated cold calls of one share through the drop-in path (RT_SCENE_CACHE=0: every call uploads, allocates and
frees its device scene), each call's phases printed -- to catch the occasional multi-second cold call of
DESIGN.md §5.3.  RTC_DIAG=1: the diagnostic build (reads RT_CHAIN_MB, the record arena's budget in MiB).
    python scripts/cold_probe.py SHARES REPS      e.g.  2:1,1:0 6"""
import os
import sys
import time

os.environ["RT_SCENE_CACHE"] = "0"
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "ray-tracing-c_amd"))
import numpy as np  # noqa: E402
import rtc  # noqa: E402

shares = [tuple(int(x) for x in s.split(":")) for s in sys.argv[1].split(",")]
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 6
with rtc.use_diag(os.environ.get("RTC_DIAG") == "1"):
    sc = rtc.Scene.preset(1, 1200, 1000, 50)
    print(f"build={rtc.build_id()} env={ {k: v for k, v in os.environ.items() if k.startswith('RT_')} }", flush=True)
    out = np.zeros((sc.height, sc.width, 3), np.uint8)
    for G, g in shares:
        for r in range(reps):
            t0 = time.perf_counter()
            rtc.render_share(sc, g, G, 0, out)
            ms = (time.perf_counter() - t0) * 1e3
            p = rtc.last_share_ms(g)
            print(f"share {g}/{G} call {r}: {ms:8.1f} ms (setup {p['setup']:.1f} run {p['run']:.1f} d2h {p['d2h']:.1f})", flush=True)
