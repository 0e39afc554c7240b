"""Counters of the general kernel's batched loop (build with -DRT_DIAG -DRT_GEN_STATS, RT_DEBUG=1), summarised.
    scripts/ab_variant.sh gstats "-DRT_DIAG -DRT_GEN_STATS"
    RTC_LIB=ab/gstats.so RT_DEBUG=1 python scripts/gen_stats_probe.py [SCENE] [WIDTH] [SPP]
Prints the library's "[rtc] gen stats:" line (stderr) and the derived shares: cycles by loop phase,
lanes per trace / shade iteration, entry kinds per traversal step, materials and textures shaded."""
import os
import re
import subprocess
import sys
import tempfile

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "ray-tracing-c_amd"))

if len(sys.argv) > 1 and sys.argv[1] == "--child":
    import time

    import torch  # noqa: F401  (initialised before rtc: see rtc._init_torch_runtime_first)
    import rtc

    scene, width, spp = (int(x) for x in sys.argv[2:5])
    sc = rtc.Scene.preset(scene, width, spp, 50, substitute_earth=True)
    t0 = time.perf_counter()
    rtc.render(sc, 1)
    print(f"frame_ms={1e3 * (time.perf_counter() - t0):.1f} {sc.width}x{sc.height}x{spp}", flush=True)
    sys.exit(0)

scene, width, spp = (sys.argv[1:4] + ["7", "1000", "64"][len(sys.argv[1:4]):])
with tempfile.TemporaryFile("w+") as err:
    r = subprocess.run([sys.executable, __file__, "--child", scene, width, spp], stderr=err, stdout=subprocess.PIPE, text=True,
                       env={**os.environ, "RT_DEBUG": "1"}, timeout=600)
    err.seek(0)
    log = err.read()
if r.returncode:
    print(log[-3000:])
    sys.exit(r.returncode)
line = [x for x in log.splitlines() if "gen stats:" in x][-1]
q = {k: int(v) for k, v in re.findall(r"(\w+)=(\d+)", line)}
print(line)
cyc = q["cyc_iter_refill"] + q["cyc_iter_trace"] + q["cyc_iter_shade"]
pc = lambda v: f"{100.0 * v / max(cyc, 1):.1f}%"
print(f"cycles: trace iters {pc(q['cyc_iter_trace'])} shade iters {pc(q['cyc_iter_shade'])} "
      f"refill-only {pc(q['cyc_iter_refill'])}")
print(f"  in shade: record {pc(q['cyc_record'])} emit {pc(q['cyc_emit'])} scatter {pc(q['cyc_scatter'])} "
      f"scatter(perlin passes) {pc(q['cyc_scatter_perlin'])} lights {pc(q['cyc_lights'])} fold {pc(q['cyc_fold'])} "
      f"camera {pc(q.get('cyc_camera', 0))} first-bounce begin {pc(q.get('cyc_begin', 0))} "
      f"loop top (shade iters) {pc(q.get('cyc_top', 0))} whole bounce {pc(q.get('cyc_bounce', 0))} "
      f"pixel write {pc(q.get('cyc_write', 0))}")
ti, si = max(q["trace_iters"], 1), max(q["shade_iters"], 1)
if "cyc_common" in q:
    print(f"  in trace: classify {pc(q['cyc_classify'])} common {pc(q['cyc_common'])} rare {pc(q['cyc_rare'])}; "
          f"steps running rare actions {q['rare_steps']} ({100.0 * q['rare_steps'] / max(q['trace_iters'], 1):.2f} per iteration)")
print(f"trace iters {q['trace_iters']} lanes/iter {q['trace_lanes'] / ti:.1f} cyc/iter {q['cyc_iter_trace'] / ti:.0f}; "
      f"shade iters {q['shade_iters']} lanes/iter {q['shade_lanes'] / si:.1f} cyc/iter {q['cyc_iter_shade'] / si:.0f}")
ks = ["kind_box", "kind_sphere", "kind_quad", "kind_xform", "kind_medium", "kind_other"]
tot = max(sum(q[k] for k in ks), 1)
print("entry kinds (lane-steps, first step of each trace iteration): " +
      " ".join(f"{k[5:]} {100.0 * q[k] / tot:.1f}%" for k in ks) + f"; kinds per step {q['step_kinds'] / ti:.2f}")
ms = ["mat_lam", "mat_metal", "mat_diel", "mat_iso", "mat_end", "miss"]
tm = max(sum(q[k] for k in ms), 1)
print("shaded lanes: " + " ".join(f"{k} {100.0 * q[k] / tm:.1f}%" for k in ms))
tx = ["tex_solid", "tex_checker", "tex_image", "tex_perlin"]
print("textures (lanes): " + " ".join(f"{k[4:]} {q[k]}" for k in tx) +
      f"; shade passes with a perlin lane {100.0 * q['pass_perlin'] / si:.1f}%")
if "paths" in q:  # path records (rt_general.h: RT_GEN_REPLAY): how paths end, what outgrows the register stacks
    P = max(q["paths"], 1)
    print(f"paths with records {q['paths']}: zero tail {100.0 * q['path_zero'] / P:.1f}%; outgrew the register stacks "
          f"{100.0 * q['path_trunc'] / P:.2f}% (of those zero tail {100.0 * q['path_trunc_zero'] / max(q['path_trunc'], 1):.1f}%); "
          f"entries beyond the registers {q['spill_st']} ({100.0 * q['spill_st_zero'] / max(q['spill_st'], 1):.1f}% on "
          f"zero-tail paths); weights == 2.0f {100.0 * q['w2'] / max(q['weighted'], 1):.1f}% of weighted records; "
          f"folds skipped {100.0 * q['fold_skips'] / P:.1f}%")
print([x for x in r.stdout.splitlines() if x.startswith("frame_ms")][-1])
