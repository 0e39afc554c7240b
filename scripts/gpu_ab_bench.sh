#!/bin/bash
# Same-box A/B of library builds on one bench configuration: bench.py under each build in LIBS
# (';'-separated, "tree" = the in-tree library), alternating, ROUNDS times; one time limit per run.
#   LIBS="ab/base.so;tree" BENCH_ARGS="--scene 7 --width 1000 --steps 1 --warmup 1" bash scripts/gpu_ab_bench.sh
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
IFS=';' read -ra L <<< "${LIBS:-tree}"
for r in $(seq 1 ${ROUNDS:-2}); do
  for lib in "${L[@]}"; do
    if [ "$lib" = tree ]; then unset RTC_LIB; else export RTC_LIB=$GRAFT_REPO_ROOT/$lib; fi
    timeout -k 10 300 python bench.py --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/abb.log 2>&1
    rc=$?
    echo "== [$lib] round $r rc=$rc $(grep '^{' gpurun_out/abb.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('value', d['value'], 'kernel_ms', d['roofline']['kernel_ms_avg'], 'identical', (d.get('parity') or {}).get('pixel_identical_to_reference'))" 2>&1)"
    [ $rc -ne 0 ] && { tail -5 gpurun_out/abb.log; exit $rc; }
  done
done
exit 0
