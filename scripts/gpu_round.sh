#!/bin/bash
# Round-end style GPU pass: parity tests, smoke, the default bench (N=1), a rocprofv3 kernel-trace
# profile of the bench, and the per-rank shard probe for N=2/4/8 (rows j % N, each share on one GPU).
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${TAG:-dev}
step() {
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "gpurun_out/${TAG}_${name}.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n 12 "gpurun_out/${TAG}_${name}.log"
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
export TMPDIR=/tmp
[ "${SKIP_TESTS:-0}" = 1 ] || step pytest_gpu 600 python -u -m pytest tests -x -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread
[ "${SKIP_TESTS:-0}" = 1 ] || step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench 600 python bench.py ${BENCH_ARGS:-}
step rocprof 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o run -- \
    python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-parity
find gpurun_out/${TAG}_prof -name '*kernel_stats.csv' -exec cat {} \;
[ "${SKIP_SHARD:-0}" = 1 ] || step shard 900 python -u scripts/shard_probe.py 2,4,8 all 1000
