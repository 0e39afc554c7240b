#!/bin/bash
# Same-box sweep of the product library's scheduling knobs over the rank shares (run on the GPU box):
#   bash scripts/knob_sweep.sh WORLDS "ENV1" "ENV2" ...     e.g.  2,8 "" "RT_MIG_IDLE=50" ""
# Each variant: scripts/shard_probe.py WORLDS all 1000 with that environment, output in
# gpurun_out/sweep_<i>.txt; the summary lines (max rank ms per world) are printed per variant.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
worlds=$1; shift
i=0
for v in "$@"; do
  env $v timeout -k 10 300 python3 -u scripts/shard_probe.py "$worlds" all 1000 > gpurun_out/sweep_$i.txt 2>&1
  rc=$?
  echo "[$i] '$v' rc=$rc $(grep -E '^world' gpurun_out/sweep_$i.txt | sed -E 's/ frame_Msamples.s=[0-9]+//' | tr '\n' ' ')"
  [ $rc -ne 0 ] && exit $rc
  i=$((i + 1))
done
exit 0
