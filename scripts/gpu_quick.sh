#!/bin/bash
# Development GPU pass: the -m gpu tests (one process, per-test time limit), then the default bench and
# the per-rank shard probe.  Every GPU step has its own time limit; anything worse than a test
# failure ends the script (no retries).
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${TAG:-dev}
step() {
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "gpurun_out/${TAG}_${name}.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n ${TAIL:-25} "gpurun_out/${TAG}_${name}.log"
  if [ $rc -gt 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
export TMPDIR=/tmp
[ "${SKIP_TESTS:-0}" = 1 ] || step pytest_gpu 900 python -u -m pytest tests -x -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"}
[ "${SKIP_BENCH:-0}" = 1 ] || step bench 600 python bench.py --no-cpu-baseline ${BENCH_ARGS:-}
[ "${SKIP_SHARD:-0}" = 1 ] || step shard 900 python -u scripts/shard_probe.py ${WORLDS:-2,4,8} ${RANKS:-all} 1000
