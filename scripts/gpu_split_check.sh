#!/bin/bash
# Split-render check on one GPU: its parity tests, then the N=8 per-rank share timing (rank 0 and 1)
# under a few planner settings (RT_SPLIT_* from the list in SWEEP, ';'-separated env assignments).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_render_gpu.py -x -v -p no:cacheprovider --timeout 120 --timeout-method thread -k "split or SPLIT" > gpurun_out/sp_pytest.log 2>&1; rc=$?
tail -8 gpurun_out/sp_pytest.log
[ $rc -ne 0 ] && exit $rc
IFS=';' read -ra CFG <<< "${SWEEP:-RT_SPLIT=2}"
n=0
for c in "${CFG[@]}"; do
  echo "== $c"
  env $c RT_DEBUG=${DBG:-0} timeout -k 10 200 python -u scripts/shard_probe.py ${WORLDS:-8} ${RANKS:-0,1} 1000 > gpurun_out/sp_shard_$n.log 2>&1; rc=$?
  grep -v "lpt\|book1 v9" gpurun_out/sp_shard_$n.log | tail -${TAILN:-14}
  [ $rc -ne 0 ] && exit $rc
  n=$((n+1))
done
exit 0
