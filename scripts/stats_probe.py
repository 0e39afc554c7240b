import os, sys, ctypes, time
sys.path.insert(0, 'ray-tracing-c_amd')
os.environ['RT_BOOK1_STATS'] = '1'
import torch, rtc
L = rtc.lib(); L.rt_book1_stats.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
for batch in os.environ.get('BATCHES', '48').split(','):
    os.environ['RT_SHADE_BATCH'] = batch
    sc = rtc.Scene.preset(1, 1200, int(os.environ.get('SPP', '100')), 50)
    ds = rtc.DeviceScene(sc, 0)
    buf = torch.empty((sc.height, sc.width, 3), dtype=torch.uint8, device='cuda')
    ds.render_rows_async(0, 1, sc.height, buf.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    st = (ctypes.c_ulonglong * 8)()
    assert L.rt_book1_stats(ds._h, st) == 0
    st = list(st)
    print(f"batch={batch} trav_iters={st[0]:.3e} useful_steps={st[1]:.3e} eff_trav={st[1]/st[0]:.3f} "
          f"shade_iters={st[2]:.3e} shading_lanes={st[3]:.3e} eff_shade={st[3]/max(st[2],1):.3f} rays={st[4]:.3e} "
          f"nodes/ray={st[5]/st[4]:.2f} leafsteps/ray={st[6]/st[4]:.2f} steps/ray={st[1]/st[4]:.2f}", flush=True)
    ds.close()
