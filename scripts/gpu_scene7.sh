#!/bin/bash
# Config 5 (scene 7, 1000x1000, 1000 spp, depth 50) on one GPU: bench line with the CPU baseline
# (reference -Ofast build at 10 spp) and a rocprofv3 kernel-stats profile of one frame.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-s7}
timeout -k 10 400 python bench.py --scene 7 --width 1000 --spp 1000 --steps 2 --warmup 1 --cpu-spp 10 \
    > gpurun_out/${TAG}_bench.log 2>&1 || { tail -20 gpurun_out/${TAG}_bench.log; exit 1; }
grep '^{' gpurun_out/${TAG}_bench.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o run -- \
    python bench.py --scene 7 --width 1000 --spp 1000 --steps 1 --warmup 0 --no-cpu-baseline --no-parity \
    > gpurun_out/${TAG}_rocprof.log 2>&1 || { tail -20 gpurun_out/${TAG}_rocprof.log; exit 1; }
cat gpurun_out/${TAG}_prof/run_kernel_stats.csv
