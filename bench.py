#!/usr/bin/env python3
"""bench.py — Msamples/s of the MI355X render path on the reference's headline benchmark.

Workload (BASELINE.json configs[2]): the Book-1 final scene (reference CLI scene 1, src/main.c:32-85),
1200x675, 1000 samples per pixel, max depth 50 — exactly `./main 1 1200 1000 _` of the reference.
A "step" is one full frame: every pixel's 1000-sample path loop over that GPU's rows -- the launch
rt_render_rows_async makes (cost pre-pass, device-side plan, chain kernel, fold).  The scene arrays
are resident in HBM before timing starts; the frame stays in HBM.  At N=1, after timing, rank 0 also
times the drop-in boundary end to end (rt_render: flatten-free upload, launch, D2H into a host
buffer, i.e. what Camera_render does after rt_flatten) and reports it as "end_to_end" -- never as
"value".

Multi-GPU (python -m torch.distributed.run --nproc-per-node N bench.py --gpus N): one process per
GPU, rows j % N == rank, no collective on the data path; the frame is fixed, so this
is strong scaling.  Timing: barrier + synchronize on both sides of K steps, max over ranks.

After timing (outside the timed region) the ranks' rows are gathered and the frame's sha256 is
compared with the reference render's (tests/golden/manifest.json) when that config has a golden.

rank 0 at N=1 first times the reference's own CPU build (oracle/_ref/ref_render_fast: upstream
`-std=c11 -Ofast -fopenmp`) on a bounded sample of the same workload, before the GPU is touched.
"""
import argparse
import hashlib
import json
import os
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "ray-tracing-c_amd"))

METRIC = "Msamples/s (pixels×spp) Book-1 final 1200×675×1000spp; max-abs pixel diff"
# FP32 operations per sample (instrumented reference event counts x per-event op counts)
OPS_PER_SAMPLE = {0: 0.48e3, 1: 2.82e3, 7: 6.0e3}
PEAK_FP32_TFLOPS = 157.3      # MI355X_MICROARCH.md: peak FP32 vector (= f32 MFMA) rate, FMA = 2 flops
# the realistic ceiling for this code: non-FMA, non-packed VALU issue -- 256 CUs x 4 SIMDs
# x 32 lanes per cycle (a wave64 VALU op issues over 2 cycles, MI355X_MICROARCH.md) x 2.4 GHz
ISSUE_TOPS = 256 * 4 * 32 * 2.4e9 / 1e12
# committed rocprofv3 PMC summaries, one per configuration (scripts/gpu_profile.sh -> scripts/pmc_summary.py):
# profiles/<round>/pmc_<config key>.json, stamped with the build id of the library they measured
PMC_DIR = os.path.join(ROOT, "profiles", "r06")


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--scene", type=int, default=1)
    ap.add_argument("--width", type=int, default=1200)
    ap.add_argument("--spp", type=int, default=1000)
    ap.add_argument("--depth", type=int, default=50)
    ap.add_argument("--cpu-spp", type=int, default=100, help="spp of the bounded CPU-baseline sample")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-parity", action="store_true")
    return ap.parse_args()


def cpu_baseline(args):
    """Reference CPU build (upstream flags) on a bounded sample: same scene and size, fewer spp."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle  # test infrastructure: used only as the measured CPU baseline here

    # the reference's OpenMP team default is every hardware thread (src/raytracing.c:91); here that is
    # every CPU this process may run on, capped by the cgroup CPU quota when one is set (the GPU box
    # grants 16 CPUs of a 128-core host: 256 threads under a 16-CPU quota measured 20x slower)
    affinity = len(os.sched_getaffinity(0))
    quota = _cgroup_cpus()
    threads = min(affinity, max(1, int(quota + 0.5))) if quota else affinity
    kind, exe = "reference", pyoracle.REF_FAST
    if not os.path.exists(exe):
        return None
    with tempfile.TemporaryDirectory() as td:
        t0 = time.perf_counter()
        w, h = pyoracle.ref_render(args.scene, args.width, args.cpu_spp, args.depth, os.path.join(td, "o.rgb"),
                                   fast=True, threads=threads, timeout=600)
        dt = time.perf_counter() - t0
    return {"value": round(w * h * args.cpu_spp / dt / 1e6, 3), "unit": "Msamples/s", "cores": threads,
            "threads": threads, "affinity_cpus": affinity, "cgroup_cpu_quota": quota, "kind": kind,
            "sample": (f"scene {args.scene} {w}x{h} at {args.cpu_spp} spp (of {args.spp}), depth {args.depth}: the "
                       f"reference sources built with its Makefile flags -std=c11 -Ofast -fopenmp "
                       f"(oracle/_ref/ref_render_fast), {threads} OpenMP threads = the {affinity} affine CPUs "
                       f"capped by the cgroup quota ({quota} CPUs), wall {dt:.2f} s"),
            "host_cpu": _cpu_model()}


def _cgroup_cpus():
    """CPUs the cgroup v2 / v1 quota allows (None: unlimited or unknown)."""
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        return None if q == "max" else round(int(q) / int(per), 2)
    except (OSError, ValueError):
        pass
    try:
        q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
        per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
        return None if q <= 0 else round(q / per, 2)
    except (OSError, ValueError):
        return None


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def _spread(step_list, kern_list):
    """Per-step spread of the timed steps (HIP events on the launch stream; the slowest rank per step at
    N > 1): min / p50 / max of the step and of its frame kernel, and every step's kernel ms, so that a
    slow launch inside the timed steps shows in the line."""
    def q(v):
        v = sorted(v)
        return {"min": round(v[0], 3), "p50": round(v[len(v) // 2], 3), "max": round(v[-1], 3),
                "max_over_min": round(v[-1] / v[0], 4) if v[0] > 0 else None} if v else None
    return {"step_ms": q(step_list), "kernel_ms": q(kern_list),
            "kernel_ms_per_step": [round(x, 3) for x in kern_list]}


def golden_for(args):
    try:
        man = json.load(open(os.path.join(ROOT, "tests", "golden", "manifest.json")))
    except OSError:
        return None, None
    for name, e in man.get("renders", {}).items():
        if (e["scene"], e["width"], e["spp"], e["depth"]) == (args.scene, args.width, args.spp, args.depth):
            return name, e
    return None, None


def pmc_for(config_key, kernel_name, build_id):
    """The committed rocprofv3 PMC summary of this kernel at this configuration (per-frame HBM bytes and
    VALU figures), as (path, entry, status): status "ok" only when the summary was taken with this
    very library (same rt_build_id); "stale" when it measured another build; "none" when absent."""
    path = os.path.join(PMC_DIR, f"pmc_{config_key}.json")
    try:
        t = json.load(open(path))
    except (OSError, ValueError):
        return None, None, "none"
    rel = os.path.relpath(path, ROOT)
    if t.get("build_id") != build_id:
        return rel, None, "stale"
    for name, e in t.get("kernels", {}).items():
        if name.split("(")[0].replace("void ", "").replace(" ", "") == kernel_name.replace(" ", ""):
            return rel, e, "ok"
    return rel, None, "none"


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and world > 1:
        print(f"warning: WORLD_SIZE={world} but --gpus {args.gpus}", file=sys.stderr)

    base = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        base = cpu_baseline(args)  # before anything initialises the GPU

    import torch
    import torch.distributed as dist

    import rtc

    # RT_BENCH_SHARE_DEVICE=1: rehearsal of the N-rank launch on a box with fewer GPUs -- rank r uses
    # GPU r % count and the (CPU) gloo backend, since RCCL refuses two ranks on one device.  The
    # timings are then contended and meaningless; the partition, gather and parity are the point.
    share = os.environ.get("RT_BENCH_SHARE_DEVICE", "0") == "1"
    if share:
        local = local % max(1, torch.cuda.device_count())
    coll_dev = "cpu" if share else f"cuda:{local}"
    torch.cuda.set_device(local)
    if world > 1:
        if share:
            dist.init_process_group(backend="gloo")
        else:
            dist.init_process_group(backend="nccl", device_id=torch.device("cuda", local))

    # (scenes 3 and 7: the documented substitute earth picture, DESIGN.md §7 -- the reference repo ships none)
    sc = rtc.Scene.preset(args.scene, args.width, args.spp, args.depth, substitute_earth=True)
    W, H, spp = sc.width, sc.height, sc.spp
    row0, stride, n_rows = rtc.rows_of(H, rank, world)
    ds = rtc.DeviceScene(sc, local)
    buf = torch.zeros((max(n_rows, 1), W, 3), dtype=torch.uint8, device=f"cuda:{local}")
    stream = torch.cuda.current_stream(local)

    def step():
        if n_rows > 0:
            ds.render_rows_async(row0, stride, n_rows, buf.data_ptr(), stream.cuda_stream)

    def barrier():
        if world > 1:
            dist.barrier()

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    kernel_name = ds.kernel_name  # (after a launch: the instantiation this rank's share actually runs)

    starts = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps)]
    ends = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps)]
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(args.steps):
        starts[k].record(stream)
        step()
        ends[k].record(stream)
    torch.cuda.synchronize()
    barrier()
    elapsed = time.perf_counter() - t0
    ds.check()  # every work item of every timed launch finished (raises otherwise: no number for a partial frame)
    step_list = [s.elapsed_time(e) for s, e in zip(starts, ends)]
    step_ms = sum(step_list) / max(args.steps, 1)
    # the frame kernel alone (HIP events the library records around it on the same stream; the
    # step also holds the longest-first cost pre-pass and its sort): per timed step, and the last one
    kern_list = ds.launch_history(args.steps) if n_rows > 0 else []
    kernel_source = "history"  # (the library's launch ring: 64 launches, brackets only on chain / lane launches)
    if len(kern_list) != args.steps or min(kern_list, default=-1.0) <= 0:
        kern_list = list(step_list)
        kernel_source = "step_events"  # (kernel_ms then holds the pre-pass, plan and fold too)
    kernel_ms = kern_list[-1] if kern_list else step_ms

    if world > 1:
        t = torch.tensor([elapsed, kernel_ms] + step_list + kern_list, dtype=torch.float64, device=coll_dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        v = t.tolist()
        elapsed, kernel_ms_max = v[0], v[1]
        step_list, kern_list = v[2:2 + args.steps], v[2 + args.steps:]  # per step: the slowest rank
    else:
        kernel_ms_max = kernel_ms

    # ---- parity (outside the timed region): gather rows, compare the frame with the reference
    parity = None
    if not args.no_parity:
        rows = buf[:n_rows]
        if world > 1:
            m = (H + world - 1) // world
            pad = torch.zeros((m, W, 3), dtype=torch.uint8, device=coll_dev)
            pad[:n_rows] = rows.to(coll_dev)
            parts = [torch.empty_like(pad) for _ in range(world)]
            dist.all_gather(parts, pad)
        else:
            parts = [rows]
        if rank == 0:
            frame = rtc.assemble_frame([p.cpu().numpy() for p in parts], H, world)
            sha = hashlib.sha256(frame.tobytes()).hexdigest()
            name, g = golden_for(args)
            parity = {"frame_sha256": sha, "golden": name,
                      "pixel_identical_to_reference": (sha == g["sha256"]) if g else None,
                      "max_abs_pixel_diff": None}
            if g and sha == g["sha256"]:
                parity["max_abs_pixel_diff"] = 0
            elif g and g.get("file"):  # a full reference image: the actual difference
                import gzip

                import numpy as np
                with gzip.open(os.path.join(ROOT, "tests", "golden", g["file"]), "rb") as f:
                    ref = np.frombuffer(f.read(), np.uint8).reshape(g["height"], g["width"], 3)
                parity["max_abs_pixel_diff"] = int(np.abs(frame.astype(np.int16) - ref.astype(np.int16)).max())
            elif g:  # sha and 32x32 crops only: the largest difference inside the differing crops is unknown
                bad = [c for c, h in g.get("crops", {}).items()
                       if hashlib.sha256(frame[int(c.split(",")[1]):int(c.split(",")[1]) + 32,
                                               int(c.split(",")[0]):int(c.split(",")[0]) + 32].tobytes()).hexdigest() != h]
                parity["crops_differing"] = bad

    # the drop-in boundary end to end (after timing, every rank): rt_render_share = the host pack, scene
    # upload and allocations, launch, D2H of this rank's rows into a host frame and the completion check --
    # what Camera_render runs after rt_flatten (src/raytracing.c:86-135 as a whole, timed by the reference's
    # main.c:334-338) for this rank's share.  "first": from an empty device-scene cache (a process's first
    # call); "warm": the same call again, the cached scene reused.  Max over ranks.
    e2e = None
    if not args.no_parity:
        import numpy as np

        host = np.zeros((H, W, 3), np.uint8)
        rtc.release_cache()
        barrier()
        t0 = time.perf_counter()
        rtc.render_share(sc, rank, world, local, host)
        t_first = time.perf_counter() - t0
        ph_first = rtc.last_share_ms(rank)
        t_warm = []
        for _ in range(2):
            barrier()
            t0 = time.perf_counter()
            rtc.render_share(sc, rank, world, local, host)
            t_warm.append(time.perf_counter() - t0)
        ph_warm = rtc.last_share_ms(rank)
        rtc.release_cache()
        same = bool((host[row0::stride][:n_rows] == buf[:n_rows].cpu().numpy()).all())
        v = [t_first, min(t_warm), ph_first["setup"], ph_warm["setup"], 0.0 if same else 1.0]
        if world > 1:
            t = torch.tensor(v, dtype=torch.float64, device=coll_dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            v = t.tolist()
        e2e = {"value": round(W * H * spp / v[1] / 1e6, 3), "unit": "Msamples/s", "ms": round(v[1] * 1e3, 3),
               "first_ms": round(v[0] * 1e3, 3), "setup_ms_first": round(v[2], 3), "setup_ms_warm": round(v[3], 3),
               "rows_identical_to_timed_step": v[4] == 0.0,
               "what": "rt_render_share per rank (Camera_render after rt_flatten, this rank's rows): host pack, upload, "
                       "allocations, launch, D2H into a host frame, completion check; value/ms: the warm call (cached "
                       "device scene, best of 2), first_ms: from an empty cache; max over ranks"}

    if rank == 0:
        frame_samples = W * H * spp
        value = frame_samples * args.steps / elapsed / 1e6
        ops = OPS_PER_SAMPLE.get(args.scene)
        launch_samples = n_rows * W * spp
        # over the step's kernels: the cost pre-pass renders each pixel's first samples and the frame kernel
        # goes on from them, so the samples of a launch are shared by both -- the step's HIP
        # events (pre-pass, plan, frame kernel, fold) are the time of the whole launch's work
        achieved = (launch_samples * ops / (step_ms / 1e3) / 1e12) if ops else None
        workload = (f"Book-1 final scene (reference CLI scene 1) {W}x{H}, {spp} spp, depth {args.depth}"
                    if args.scene == 1 else f"reference scene {args.scene} {W}x{H}, {spp} spp, depth {args.depth}")
        config_key = f"s{args.scene}_{W}x{H}_{spp}spp_d{args.depth}_n{world}"
        build_id = rtc.build_id()
        pmc_src, pmc, pmc_status = pmc_for(config_key, kernel_name, build_id)
        headline = args.scene == 1 and (W, H, spp, args.depth) == (1200, 675, 1000, 50)
        line = {
            "metric": METRIC if headline else f"Msamples/s (pixels×spp) scene {args.scene} {W}×{H}×{spp}spp; max-abs pixel diff",
            "value": round(value, 3),
            "unit": "Msamples/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": round(value / base["value"], 2) if base else None,
            "vs_baseline_source": ("cpu_baseline below: the reference's own -Ofast OpenMP build on this box's host "
                                   "cores, same scene and size" if base else "no same-box CPU baseline in this run"),
            "dtype": "f32",
            "data": "synthetic: the reference's procedural scene (pcg32 seed 19,29) and per-pixel pcg32 streams",
            "config": {"workload": workload, "scene": args.scene, "width": W, "height": H, "spp": spp,
                       "max_depth": args.depth, "partition": f"rows j % {world}", "rows_on_rank0": n_rows},
            "roofline": {"bound": "valu", "achieved": round(achieved, 4) if achieved else None,
                         "peak": PEAK_FP32_TFLOPS, "unit": "TFLOP/s",
                         "frac": round(achieved / PEAK_FP32_TFLOPS, 5) if achieved else None,
                         "issue_ceiling": ISSUE_TOPS,
                         "frac_of_issue_ceiling": round(achieved / ISSUE_TOPS, 5) if achieved else None,
                         "traffic": (round(pmc["fetch_bytes"] + pmc["write_bytes"])
                                     if pmc and "fetch_bytes" in pmc and "write_bytes" in pmc else None),
                         "pmc": ({k: round(pmc[k], 4) for k in ("valu_busy", "lanes_active", "valu_insts_per_sample",
                                                                "lds_bank_conflict_frac", "kernel_ms_per_frame",
                                                                "kernel_ms_per_timed_frame")
                                  if k in pmc} if pmc else pmc_status if pmc_status == "stale" else None),
                         "pmc_source": pmc_src if pmc else None,
                         "build_id": build_id,
                         "kernel": kernel_name, "kernel_ms_avg": round(kernel_ms, 3),
                         "step_ms_avg": round(step_ms, 3),
                         "kernel_ms_max_over_ranks": round(kernel_ms_max, 3),
                         "algorithmic_work": f"{ops:.0f} FP32 ops/sample (SURVEY §8d) x {launch_samples} samples/launch"
                         if ops else None,
                         "achieved_basis": "samples per launch x ops / step_ms_avg (HIP events around the step: cost "
                                           "pre-pass, plan, frame kernel, fold -- the pre-pass renders the pixels' "
                                           "first samples, the frame kernel the rest)",
                         "note": "VALU-bound branchy FP32 + u64 integer work, no MFMA, scene in LDS (HBM roof does "
                                 "not apply). peak = dense f32 rate (FMA = 2); issue_ceiling = non-FMA non-packed "
                                 "VALU lane-ops/s (256 CU x 4 SIMD x 32 lanes x 2.4 GHz), the realistic ceiling for "
                                 "bit-exact code (no contraction). achieved counts algorithmic FP32 ops only; traffic "
                                 "= FETCH_SIZE x 2 + WRITE_SIZE bytes per frame from the committed PMC pass of "
                                 "this build (build_id); pmc 'stale' = the committed pass measured another build"},
            "spread": dict(_spread(step_list, kern_list), kernel_source=kernel_source),
            "cpu_baseline": base,
            "end_to_end": e2e,
            "parity": parity,
            "box": rtc.box_identity(local),
        }
        if share:
            line["rehearsal"] = "RT_BENCH_SHARE_DEVICE: ranks share GPUs over gloo; timings contended, not a result"
        print(json.dumps(line), flush=True)

    ds.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
