"""Book-1 kernel counters (RT_BOOK1_STATS=1 diagnostic build) on the headline scene at reduced spp.
BATCHES=32,48 SPP=100 python scripts/stats_probe.py"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "ray-tracing-c_amd"))
os.environ["RT_BOOK1_STATS"] = "1"
import torch  # noqa: E402  (initialised before rtc: see rtc._init_torch_runtime_first)
import rtc  # noqa: E402

L = rtc.lib()
L.rt_book1_stats.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
N = 29
for batch in os.environ.get("BATCHES", "48").split(","):
    os.environ["RT_SHADE_BATCH"] = batch.split(":")[0]
    if ":" in batch:
        os.environ["RT_SPHERE_BATCH"] = batch.split(":")[1]
    sc = rtc.Scene.preset(1, int(os.environ.get("WIDTH", "1200")), int(os.environ.get("SPP", "100")), 50)
    ds = rtc.DeviceScene(sc, 0)
    buf = torch.empty((sc.height, sc.width, 3), dtype=torch.uint8, device="cuda")
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    ds.render_rows_async(0, 1, sc.height, buf.data_ptr(), torch.cuda.current_stream().cuda_stream)
    e1.record()
    torch.cuda.synchronize()
    kernel_ms = e0.elapsed_time(e1)
    n_waves = torch.cuda.get_device_properties(0).multi_processor_count * 4 * 4  # 4 blocks x 4 waves / CU (approx.)
    st = (ctypes.c_ulonglong * N)()
    assert L.rt_book1_stats(ds._h, st, N) == 0
    st = [float(v) for v in st]
    cyc = st[8] + st[9]
    print(f"batch={batch} rays={st[4]:.3e} nodes/ray={st[5]/st[4]:.2f} steps/ray={st[1]/st[4]:.2f} "
          f"eff_trav={st[1]/st[0]:.3f} eff_shade={st[3]/max(st[2],1):.3f} "
          f"wave_trav_iters={st[10]:.3e} wave_shade_iters={st[11]:.3e} "
          f"clk/trav_iter={st[8]/max(st[10],1):.0f} clk/shade_iter={st[9]/max(st[11],1):.0f} "
          f"trav_share={st[8]/max(cyc,1):.3f} box_phases={st[12]:.3e} sphere_phases={st[13]:.3e} "
          f"lanes/box_phase={st[5]/max(st[12],1):.1f} lanes/sphere_phase={st[6]/max(st[13],1):.1f} "
          f"[v5: sphere fast={st[12]:.3e} slow={st[13]:.3e} wave_sphere_regions={st[14]:.3e} "
          f"wave_fallbacks={st[15]:.3e} wave_steps={st[10]*4:.3e}] "
          f"kernel_ms={kernel_ms:.1f} clock64_per_wave={st[16]/n_waves:.3e} => clock64 MHz~{st[16]/n_waves/kernel_ms/1e3:.0f} "
          f"wall_ticks_per_wave={st[17]/n_waves:.3e} span_wall_ticks={st[19]-st[18]:.4e} => wall MHz~{(st[19]-st[18])/kernel_ms/1e3:.1f} "
          f"concurrency~{st[17]/max(st[19]-st[18],1):.0f} waves last_start_at={(st[20]-st[18])/(st[19]-st[18]):.3f} "
          f"counter_dry_at={(st[21]-st[18])/(st[19]-st[18]):.3f} (fractions of the span) box_hits/ray={st[22]/st[4]:.2f} coop_traces={st[23]:.3e} windows/coop={st[25]/max(st[23],1):.1f} scan/coop={st[26]/max(st[23],1):.1f} clk/window={st[27]/max(st[25],1):.0f} walk_clk/window={st[28]/max(st[25],1):.0f}", flush=True)
    if os.environ.get("PIXEL_COST"):
        import numpy as np
        L.rt_book1_pixel_cost.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64]
        pc = np.zeros((sc.height * sc.width, 2), np.uint32)
        assert L.rt_book1_pixel_cost(ds._h, pc.ctypes.data, sc.height * sc.width) == 0
        np.save(os.environ["PIXEL_COST"], pc)
        steps, ticks = pc[:, 0].astype(np.float64), pc[:, 1].astype(np.float64)
        q = lambda a: " ".join(f"{v:.3g}" for v in np.percentile(a, [0, 50, 90, 99, 99.9, 100]))
        print(f"pixel steps pct[0,50,90,99,99.9,100]={q(steps)} mean={steps.mean():.3g}; "
              f"pixel ms pct={q(ticks / 1e5)} mean={ticks.mean() / 1e5:.3g}; kernel_ms={kernel_ms:.1f}", flush=True)
    ds.close()
