#!/bin/bash
# The closing measurements of the tree's library, on one GPU box (each GPU step has its own
# time limit; a failing step ends the script):
#   PART=s1   headline: scripts/gpu_profile.sh (bench line, kernel stats, PMC), the shard probe
#             N = 1-8 (all ranks), one share end to end per N = 8 / 2 / 1 (scripts/share_e2e.py), the rank-7 chain timeline (diagnostic build), the full -m gpu log
#   PART=s7   config 5: scripts/gpu_profile.sh for scene 7
#   PART=pmc  the headline's PMC passes again (a second box, for the box-to-box comparison)
# Outputs under gpurun_out/ with TAG r06 (copy to profiles/r06/ with the build id in the name).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
step() {
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "gpurun_out/r06_${name}.txt" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; grep -v amdgpu.ids "gpurun_out/r06_${name}.txt" | tail -n ${TAIL:-12} | cut -c1-400
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
case "${PART:-s1}" in
  s1)
    TAG=r06 CFG="--scene 1 --width 1200 --spp 1000 --steps 20 --warmup 5" bash scripts/gpu_profile.sh || exit $?
    step gpu_tests 900 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 300 --timeout-method thread
    step shard_probe 600 python -u scripts/shard_probe.py 2,3,4,5,6,7,8 all 1000
    step share_e2e 600 python -u scripts/share_e2e.py 8:7,2:1,1:0
    CHAIN_ROWS=1 step chain_8_7 300 python -u scripts/chain_probe.py 8 7 1000
    CHAIN_ROWS=1 step chain_2_1 300 python -u scripts/chain_probe.py 2 1 1000
    ;;
  s7)
    TAG=r06s7 CFG="--scene 7 --width 1000 --spp 1000 --steps 3 --warmup 1" bash scripts/gpu_profile.sh || exit $?
    ;;
  pmc)
    SKIP_BENCH=1 TAG=r06b CFG="--scene 1 --width 1200 --spp 1000" bash scripts/gpu_profile.sh || exit $?
    ;;
esac
exit 0
