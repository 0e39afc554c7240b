#!/bin/bash
# General-kernel iteration: GPU parity (render + API worlds), then scene timings: the base build
# (ab/base.so) against the tree under the settings in SETS, then the counters (ab/gstats.so).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
SCENE=${SCENE:-7}; W=${W:-1000}; SPP=${SPP:-256}
timeout -k 10 420 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_render_gpu.py tests/test_api_worlds.py > gpurun_out/t.log 2>&1
rc=$?; tail -3 gpurun_out/t.log; [ $rc -ne 0 ] && exit $rc
RTC_LIB=$PWD/ab/base.so timeout -k 10 300 python -u scripts/scene_time.py $SCENE $W $SPP "" > gpurun_out/ab_base.log 2>&1 \
  || { tail -5 gpurun_out/ab_base.log; exit 1; }
cat gpurun_out/ab_base.log
timeout -k 10 600 python -u scripts/scene_time.py $SCENE $W $SPP "${SETS:-}" > gpurun_out/ab_tree.log 2>&1 \
  || { tail -5 gpurun_out/ab_tree.log; exit 1; }
cat gpurun_out/ab_tree.log
if [ -f ab/gstats.so ]; then
  RTC_LIB=$PWD/ab/gstats.so timeout -k 10 200 python -u scripts/gen_stats_probe.py $SCENE $W 64 > gpurun_out/gs.log 2>&1 \
    || { tail -5 gpurun_out/gs.log; exit 1; }
  tail -7 gpurun_out/gs.log
fi
