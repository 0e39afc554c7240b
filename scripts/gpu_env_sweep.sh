#!/bin/bash
# One bench line per environment setting (';'-separated list in SWEEP), BENCH_ARGS shared.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
IFS=';' read -ra CFG <<< "${SWEEP:-RT_DEBUG=0}"
for c in "${CFG[@]}"; do
  env $c timeout -k 10 300 python bench.py --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/sweep.log 2>&1 || { tail -5 gpurun_out/sweep.log; exit 1; }
  echo "$c => $(grep '^{' gpurun_out/sweep.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'])")"
done
