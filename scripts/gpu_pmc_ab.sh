#!/bin/bash
# A/B of instruction counters across kernel variants: one rocprofv3 --pmc pass (kernel-trace only) per
# variant spec, e.g.  scripts/gpu_pmc_ab.sh "RT_BOOK1_V=5" "RT_BOOK1_V=6"
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-dev}
COUNTERS=${COUNTERS:-SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_BUSY_CYCLES}
for spec in "$@"; do
  name=$(echo "$spec" | tr ' =' '_-')
  out=gpurun_out/${TAG}_pmcab_${name}
  # the variant's environment is exported here: rocprofv3 must exec python directly (no env/bash hop)
  ( export $spec; timeout -k 10 300 rocprofv3 --pmc $COUNTERS --output-format csv -d $out -o run -- \
      python bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-parity > $out.log 2>&1 )
  rc=$?
  echo "== $spec rc=$rc"
  if [ $rc -ne 0 ]; then tail -20 $out.log; exit $rc; fi
  python3 scripts/pmc_summary.py $out
done
