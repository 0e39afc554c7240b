#!/bin/bash
# Custom PMC passes (one rocprofv3 run each, kernel-trace only) over one bench frame:
#   TAG=... BENCH_ARGS="--scene 7 --width 600 --spp 64" PASSES="A B C;D E" bash scripts/gpu_pmc_passes.sh
# PASSES: ';'-separated groups of counters (each group within the per-block limits).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-pp}
ARGS="--steps 1 --warmup 0 --no-cpu-baseline --no-parity ${BENCH_ARGS:-}"
IFS=';' read -ra P <<< "$PASSES"
dirs=""
for i in "${!P[@]}"; do
  timeout -s KILL 120 rocprofv3 --pmc ${P[$i]} --output-format csv -d gpurun_out/${TAG}_p$i -o run -- python3 bench.py $ARGS \
      > gpurun_out/${TAG}_p$i.log 2>&1
  rc=$?; echo "== pass $i (${P[$i]}) rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/${TAG}_p$i.log; exit $rc; fi
  dirs="$dirs gpurun_out/${TAG}_p$i"
done
python3 scripts/pmc_summary.py gpurun_out/${TAG}_summary.json --build-id "${BID:-unknown}" --config "${KEY:-custom}" --samples-per-frame "${SAMPLES:-1}" $dirs
