#!/bin/bash
# The two SQ counter passes of gpu_pmc.sh only (instruction mix, lane utilisation, waits).
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
TAG=${TAG:-dev}
ARGS=${PMC_BENCH_ARGS:---steps 1 --warmup 0 --no-cpu-baseline --no-parity}
pass() {
  local name=$1; shift
  timeout -k 10 300 rocprofv3 --pmc "$@" --output-format csv -d gpurun_out/${TAG}_pmc_${name} -o run -- \
      python bench.py $ARGS > gpurun_out/${TAG}_pmc_${name}.log 2>&1
  local rc=$?
  echo "== pmc $name rc=$rc"
  if [ $rc -ne 0 ]; then tail -20 gpurun_out/${TAG}_pmc_${name}.log; exit $rc; fi
}
pass sq1 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES
pass sq2 SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE
