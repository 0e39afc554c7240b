#!/bin/bash
# Same-box A/B of library builds: shard_probe.py under each build in LIBS (';'-separated paths,
# "tree" = the in-tree library), alternating, ROUNDS times.  One time limit per run.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
IFS=';' read -ra L <<< "${LIBS:-tree}"
for r in $(seq 1 ${ROUNDS:-2}); do
  for lib in "${L[@]}"; do
    if [ "$lib" = tree ]; then unset RTC_LIB; else export RTC_LIB=$GRAFT_REPO_ROOT/$lib; fi
    timeout -k 10 300 python -u scripts/shard_probe.py ${WORLDS:-8} ${RANKS:-all} ${SPP:-1000} > gpurun_out/ab.log 2>&1
    rc=$?
    echo "== [$lib] round $r rc=$rc"; grep -E "^world|identical=False|Error" gpurun_out/ab.log
    [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
