#!/bin/bash
# GPU pass used during development: parity tests, the default bench, a rocprofv3 kernel-trace profile.
# Every GPU step has its own time limit; a crash/timeout/abort ends the script (no retries).
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${TAG:-dev}
step() {  # step <name> <timeout> <cmd...>: test failures (rc 1) are reported, anything worse stops here
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "gpurun_out/${TAG}_${name}.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n 25 "gpurun_out/${TAG}_${name}.log"
  if [ $rc -gt 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
[ "${SKIP_TESTS:-0}" = 1 ] || step pytest_gpu 900 python -m pytest tests -q -m gpu -p no:cacheprovider
[ "${SKIP_BENCH:-0}" = 1 ] || step bench 600 python bench.py ${BENCH_ARGS:-}
if [ "${PROFILE:-1}" = 1 ]; then
  export TMPDIR=/tmp
  step rocprof 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o run -- \
      python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-parity
  find gpurun_out/${TAG}_prof -name '*kernel_stats.csv' -exec cat {} \;
fi
