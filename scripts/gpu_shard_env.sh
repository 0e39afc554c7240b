#!/bin/bash
# Same-box sweep of RT_* settings on the per-rank shard probe (scripts/shard_probe.py): one probe run
# per ';'-separated setting in SWEEP, each under its own time limit; a failing run ends the script.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
IFS=';' read -ra CFG <<< "${SWEEP:-RT_DEBUG=0}"
i=0
for c in "${CFG[@]}"; do
  env $c timeout -k 10 300 python -u scripts/shard_probe.py ${WORLDS:-2,4,8} ${RANKS:-all} ${SPP:-1000} > gpurun_out/${TAG:-se}_$i.log 2>&1
  rc=$?
  echo "== [$c] rc=$rc"; grep -E "^world|identical=False|Error|error" gpurun_out/${TAG:-se}_$i.log
  [ $rc -ne 0 ] && exit $rc
  i=$((i+1))
done
exit 0
