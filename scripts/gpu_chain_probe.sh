#!/bin/bash
# Chain-render timelines (scripts/chain_probe.py) for a list of WORLD:RANK pairs; one time limit each.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${TAG:-dev}
for wr in ${PAIRS:-8:4 2:1 1:0}; do
  w=${wr%%:*}; r=${wr##*:}
  timeout -k 10 300 python -u scripts/chain_probe.py $w $r ${SPP:-1000} > gpurun_out/${TAG}_chain_${w}_${r}.log 2>&1
  rc=$?
  echo "== chain $w $r rc=$rc"; cat gpurun_out/${TAG}_chain_${w}_${r}.log | grep -v amdgpu.ids
  [ $rc -ne 0 ] && exit $rc
done
exit 0
