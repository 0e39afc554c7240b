#!/bin/bash
# Round profile of the headline configuration: the default bench line (N=1, CPU baseline), a
# rocprofv3 kernel-trace/stats pass of the bench, the PMC passes (counters in separate passes,
# kernel-trace only) summarised per kernel, and the per-rank shard probe (N=2/4/8 shares on one GPU).
# Every GPU step has its own time limit; a failing step ends the script.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r02}
step() {
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "gpurun_out/${TAG}_${name}.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n ${TAIL:-4} "gpurun_out/${TAG}_${name}.log" | cut -c1-400
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
[ "${SKIP_BENCH:-0}" = 1 ] || step bench 600 python bench.py
step stats 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o run -- \
    python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-parity
ARGS="--steps 1 --warmup 0 --no-cpu-baseline --no-parity"
step pmc_sq1 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
    --output-format csv -d gpurun_out/${TAG}_pmc_sq1 -o run -- python3 bench.py $ARGS
step pmc_sq2 300 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE \
    --output-format csv -d gpurun_out/${TAG}_pmc_sq2 -o run -- python3 bench.py $ARGS
step pmc_fetch 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/${TAG}_pmc_fetch -o run -- python3 bench.py $ARGS
step pmc_write 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/${TAG}_pmc_write -o run -- python3 bench.py $ARGS
python3 scripts/pmc_summary.py gpurun_out/${TAG}_pmc_chain.json ${PMC_SAMPLES:-810000000} \
    gpurun_out/${TAG}_pmc_sq1 gpurun_out/${TAG}_pmc_sq2 gpurun_out/${TAG}_pmc_fetch gpurun_out/${TAG}_pmc_write
find gpurun_out/${TAG}_prof -name '*kernel_stats.csv' -exec cp {} gpurun_out/${TAG}_kernel_stats.csv \;
head -6 gpurun_out/${TAG}_kernel_stats.csv | cut -c1-200
[ "${SKIP_SHARD:-0}" = 1 ] || step shard 900 python -u scripts/shard_probe.py 2,4,8 all 1000
