#!/bin/bash
# Quick A/B on one GPU: the default bench (parity-checked headline frame) and the GPU tests.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-ab}
timeout -k 10 300 python bench.py --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/${TAG}_bench.log 2>&1; rc=$?
grep '^{' gpurun_out/${TAG}_bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('value', d['value'], 'kernel_ms', d['roofline']['kernel_ms_avg'], 'parity', d['parity'])" || tail -5 gpurun_out/${TAG}_bench.log
[ $rc -ne 0 ] && exit $rc
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 600 python -u -m pytest tests -x -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1; rc=$?
  tail -3 gpurun_out/${TAG}_pytest.log
  [ $rc -ne 0 ] && exit $rc
fi
if [ -n "${SHARD:-}" ]; then
  timeout -k 10 400 python -u scripts/shard_probe.py $SHARD > gpurun_out/${TAG}_shard.log 2>&1; rc=$?
  grep "^world" gpurun_out/${TAG}_shard.log
fi
exit $rc
