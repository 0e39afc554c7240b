#!/bin/bash
# shard_probe.py (per-rank shares of the headline frame on one GPU) once per environment setting
# (';'-separated list in SWEEP); prints the per-world max lines.  One time limit per setting.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
IFS=';' read -ra CFG <<< "${SWEEP:-RT_DEBUG=0}"
i=0
for c in "${CFG[@]}"; do
  i=$((i+1))
  env $c timeout -k 10 300 python -u scripts/shard_probe.py ${WORLDS:-2,4,8} ${RANKS:-all} ${SPP:-1000} > gpurun_out/${TAG:-dev}_sweep_$i.log 2>&1
  rc=$?
  echo "== [$c] rc=$rc"; grep -E "^world|identical=False|Error|error" gpurun_out/${TAG:-dev}_sweep_$i.log
  [ $rc -ne 0 ] && exit $rc
done
exit 0
