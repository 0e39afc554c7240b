#!/bin/bash
# A/B sweep of kernel variants on the default bench workload (one process per variant).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
TAG=${TAG:-dev}
for spec in "${@}"; do
  name=$(echo "$spec" | tr ' =' '_-')
  timeout -k 10 300 env $spec python bench.py --steps 2 --warmup 1 --no-cpu-baseline ${SWEEP_ARGS:-} > gpurun_out/${TAG}_sweep_${name}.json 2> gpurun_out/${TAG}_sweep_${name}.err
  rc=$?
  echo "== $spec rc=$rc $(python3 -c "import json,sys; d=json.load(open('gpurun_out/${TAG}_sweep_${name}.json')); print(d['value'], d['ms_per_step'], (d.get('parity') or {}).get('pixel_identical_to_reference'))" 2>/dev/null)"
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/${TAG}_sweep_${name}.err; exit $rc; fi
done
