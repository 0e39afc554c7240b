"""Probe: does torch's bundled HIP runtime still initialise after librtc_amd.so's (/opt/rocm) one?
python scripts/probe_runtime_order.py {ours_first|torch_first|ours_count_only}"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "ray-tracing-c_amd"))
import numpy as np

mode = sys.argv[1]
if mode == "torch_first":
    import torch
    torch.cuda.init()
import rtc

print("rt_device_count", rtc.device_count())
if mode != "ours_count_only":
    print("diag", rtc.diag_libm(2, np.array([0.5, 2.0], np.float32)))
import torch

torch.cuda.init()
print(mode, "torch ok", torch.cuda.device_count(), torch.zeros(4, device="cuda").sum().item())
