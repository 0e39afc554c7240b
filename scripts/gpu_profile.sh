#!/bin/bash
# Profile of one bench configuration with the library in this tree (run on the GPU box):
#   TAG=r03a CFG="--scene 1 --width 1200 --spp 1000" bash scripts/gpu_profile.sh
# 1. [SKIP_BENCH=1 skips] the bench line of the configuration (N=1, CPU baseline);
# 2. rocprofv3 --kernel-trace --stats over bench.py (--steps 2 --warmup 1: 3 frames);
# 3. five rocprofv3 --pmc passes (counters in separate runs, kernel-trace only), 1 frame each;
# 4. scripts/pmc_summary.py -> gpurun_out/${TAG}_pmc_<config key>.json, per frame, stamped with the
#    library's rt_build_id (copy it to profiles/<round>/ for bench.py to attach).
# Every GPU step has its own time limit; a failing step ends the script.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-prof}
CFG=${CFG:-}
step() {
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "gpurun_out/${TAG}_${name}.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n ${TAIL:-3} "gpurun_out/${TAG}_${name}.log" | cut -c1-600
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
read -r KEY SAMPLES BID < <(python3 - $CFG <<'PY'
import sys, argparse
sys.path.insert(0, "ray-tracing-c_amd")
ap = argparse.ArgumentParser(); ap.add_argument("--scene", type=int, default=1); ap.add_argument("--width", type=int, default=1200)
ap.add_argument("--spp", type=int, default=1000); ap.add_argument("--depth", type=int, default=50)
a, _ = ap.parse_known_args()
import rtc
s = rtc.Scene.preset(a.scene, a.width, 1, 1, substitute_earth=True)
print(f"s{a.scene}_{s.width}x{s.height}_{a.spp}spp_d{a.depth}_n1", s.width * s.height * a.spp, rtc.build_id())
PY
)
BOX=$(python3 -c "import sys, json; sys.path.insert(0, 'ray-tracing-c_amd'); import rtc; print(json.dumps(rtc.box_identity()))")
echo "config $KEY samples/frame $SAMPLES build $BID box $BOX"
[ "${SKIP_BENCH:-0}" = 1 ] || step bench 900 python3 bench.py $CFG
step stats 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_stats -o run -- \
    python3 bench.py $CFG --steps 2 --warmup 1 --no-cpu-baseline --no-parity
A="$CFG --steps 1 --warmup 1 --no-cpu-baseline --no-parity"  # (2 frames: the first pays one-time costs)
step pmc_sq1 600 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
    --output-format csv -d gpurun_out/${TAG}_pmc_sq1 -o run -- python3 bench.py $A
step pmc_sq2 600 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE \
    --output-format csv -d gpurun_out/${TAG}_pmc_sq2 -o run -- python3 bench.py $A
step pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/${TAG}_pmc_fetch -o run -- python3 bench.py $A
step pmc_write 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/${TAG}_pmc_write -o run -- python3 bench.py $A
# the L2's atomics and its memory-side requests (the chain protocol's cross-XCD words; box-to-box comparison)
# (not fatal: the summary is written without it if this pass fails)
ATOM=""
timeout -k 10 -s KILL 600 rocprofv3 --pmc TCC_ATOMIC_sum TCC_EA0_ATOMIC_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum \
    --output-format csv -d gpurun_out/${TAG}_pmc_atom -o run -- python3 bench.py $A > gpurun_out/${TAG}_pmc_atom.log 2>&1 \
  && ATOM=gpurun_out/${TAG}_pmc_atom
echo "== pmc_atom ${ATOM:-failed}"
python3 scripts/pmc_summary.py gpurun_out/${TAG}_pmc_${KEY}.json --build-id "$BID" --config "$KEY" --samples-per-frame "$SAMPLES" --box "$BOX" \
    --stats gpurun_out/${TAG}_stats --stats-frames 3 --stats-warmup 1 --pmc-frames 2 \
    gpurun_out/${TAG}_pmc_sq1 gpurun_out/${TAG}_pmc_sq2 gpurun_out/${TAG}_pmc_fetch gpurun_out/${TAG}_pmc_write $ATOM
find gpurun_out/${TAG}_stats -name '*kernel_stats.csv' -exec cp {} gpurun_out/${TAG}_kernel_stats_${KEY}.csv \;
