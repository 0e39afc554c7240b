#!/bin/bash
# PMC passes (separate runs, kernel-trace only) over one bench frame of an arbitrary config:
#   TAG=... SAMPLES=<samples per frame> BENCH_ARGS="--scene 7 --width 400 --spp 64" bash scripts/gpu_pmc_cfg.sh
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-pmc}
ARGS="--steps 1 --warmup 0 --no-cpu-baseline --no-parity ${BENCH_ARGS:-}"
pass() {
  local name=$1; shift
  timeout -k 10 300 rocprofv3 --pmc "$@" --output-format csv -d gpurun_out/${TAG}_${name} -o run -- python3 bench.py $ARGS \
      > gpurun_out/${TAG}_${name}.log 2>&1
  local rc=$?
  echo "== pmc $name rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/${TAG}_${name}.log; exit $rc; fi
}
pass sq1 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES
pass sq2 SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE
pass fetch FETCH_SIZE
pass write WRITE_SIZE
python3 scripts/pmc_summary.py gpurun_out/${TAG}_summary.json ${SAMPLES:-1} gpurun_out/${TAG}_sq1 gpurun_out/${TAG}_sq2 \
    gpurun_out/${TAG}_fetch gpurun_out/${TAG}_write
