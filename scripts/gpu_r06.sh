#!/bin/bash
# One GPU pass of round-6 work (each step has its own time limit; a failing step ends the script):
#   TESTS=1      pytest -m gpu (all parity tests)
#   BENCH=1      the default bench line (N=1, parity-checked)
#   AB="ab/r03.so;tree;diag:RT_LEAF_MIN=16"  same-box A/B of library builds / diag settings, ROUNDS rounds
#   AB7="..."    the same on config 5 (scene 7)
#                (entries: a path, "tree" = the product library, "env:<VAR=V ...>" = it under those
#                variables, "diag:<VAR=V ...>" = the diagnostic build under them); BENCH_ARGS for other
#                configurations
#   S7=1         the config-5 bench line (scene 7)
#   SHARD=1      the per-rank shard probe (WORLDS, default 2,4,8)
#   PAIRS="8:7 1:0"  chain timelines (diagnostic build), rows saved; EXACT=1 also with the exact plan
#   E2E="8:7,2:1,1:0"  one share end to end through rt_render_share (cold / first / warm) beside its step
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r6}
step() {
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "gpurun_out/${TAG}_${name}.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; grep -v amdgpu.ids "gpurun_out/${TAG}_${name}.log" | tail -n ${TAIL:-25} | cut -c1-400
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
summ() { grep '^{' "$1" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; sp=d.get('spread') or {}; print('value', d['value'], 'kernel_ms', r['kernel_ms_avg'], 'kernel_spread', (sp.get('kernel_ms') or {}), 'parity', (d.get('parity') or {}).get('pixel_identical_to_reference'), 'build', r['build_id'])"; }
[ "${TESTS:-0}" = 1 ] && step pytest 900 python -u -m pytest tests -x -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread
[ "${BENCH:-0}" = 1 ] && step bench 300 python bench.py --no-cpu-baseline
ab() {  # ab "<entries>" "<bench args>"
  IFS=';' read -ra E <<< "$1"
  for r in $(seq 1 ${ROUNDS:-2}); do
    for e in "${E[@]}"; do
      vars=""; lib=""
      case "$e" in
        tree) lib="" ;;
        diag:*) lib=ray-tracing-c_amd/librtc_amd_diag.so; vars="${e#diag:}" ;;
        env:*) lib=""; vars="${e#env:}" ;;  # the product library under documented parameters
        *) lib="$e" ;;
      esac
      if [ -n "$lib" ]; then export RTC_LIB=$GRAFT_REPO_ROOT/$lib; else unset RTC_LIB; fi
      np="--no-parity"; [ "${PARITY:-0}" = 1 ] && np=""  # PARITY=1: every A/B line checks its frame
      env $vars timeout -k 10 300 python bench.py --no-cpu-baseline $np $2 > gpurun_out/${TAG}_ab.log 2>&1
      rc=$?
      echo "== [$e] round $r rc=$rc $(summ gpurun_out/${TAG}_ab.log 2>&1)"
      [ $rc -ne 0 ] && { tail -5 gpurun_out/${TAG}_ab.log; exit $rc; }
    done
  done
  unset RTC_LIB
}
[ -n "${AB:-}" ] && ab "$AB" "${BENCH_ARGS:-}"
# AB7: the same for config 5 (scene 7, 1000x1000x1000 spp, one frame)
[ -n "${AB7:-}" ] && ab "$AB7" "--scene 7 --width 1000 --steps 1 --warmup 1"
# LOOPSTATS="loopstats loopstats_pair": loop-stats builds (ab/<name>.so, -DRT_DIAG -DRT_LOOP_STATS): phase split
for ls in ${LOOPSTATS:-}; do
  RTC_LIB=$GRAFT_REPO_ROOT/ab/$ls.so RT_DEBUG=1 timeout -k 10 300 python bench.py --steps 1 --warmup 0 \
      --no-cpu-baseline --no-parity > gpurun_out/${TAG}_$ls.log 2>&1
  rc=$?; echo "== $ls rc=$rc"; grep "\[rtc\] \(loop\|chain launch ms\)" gpurun_out/${TAG}_$ls.log
  [ $rc -ne 0 ] && { tail -5 gpurun_out/${TAG}_$ls.log; exit $rc; }
done
# GSTATS="7 1000 64": general-kernel counters (ab/gstats.so, -DRT_DIAG -DRT_GEN_STATS) at scene / width / spp
if [ -n "${GSTATS:-}" ]; then
  RTC_LIB=$GRAFT_REPO_ROOT/ab/gstats.so step gstats 300 python -u scripts/gen_stats_probe.py $GSTATS
fi
[ "${S7:-0}" = 1 ] && step s7_bench 300 python bench.py --no-cpu-baseline --scene 7 --width 1000 --steps 1 --warmup 1
[ -n "${E2E:-}" ] && step e2e 600 python -u scripts/share_e2e.py "$E2E"
[ "${SHARD:-0}" = 1 ] && step shard 400 python -u scripts/shard_probe.py ${WORLDS:-2,4,8} all 1000
# SHARD_ENVS="RT_CHAIN_PAD=1.2;...": the shard probe on the diagnostic build under each setting
if [ -n "${SHARD_ENVS:-}" ]; then
  IFS=';' read -ra SE <<< "$SHARD_ENVS"
  for r in $(seq 1 ${ROUNDS:-2}); do
    for e in "${SE[@]}"; do
      env RTC_DIAG=1 $e timeout -k 10 400 python -u scripts/shard_probe.py ${WORLDS:-2,4,8} all 1000 > gpurun_out/${TAG}_shard_env.log 2>&1
      rc=$?
      echo "== shard [$e] round $r rc=$rc"; grep -E "^world|identical=False|Error" gpurun_out/${TAG}_shard_env.log
      [ $rc -ne 0 ] && { tail -5 gpurun_out/${TAG}_shard_env.log; exit $rc; }
    done
  done
fi
for wr in ${PAIRS:-}; do
  w=${wr%%:*}; r=${wr##*:}
  CHAIN_ROWS=1 CHAIN_TAG=_plan step chain_${w}_${r} 300 python -u scripts/chain_probe.py $w $r 1000
  if [ "${EXACT:-0}" = 1 ]; then
    CHAIN_ROWS=1 CHAIN_TAG=_exact RT_LPT_SPP=1000 RT_COST_BUDGET=0 RT_CHAIN_SMOOTH=0 \
      step chain_${w}_${r}_exact 300 python -u scripts/chain_probe.py $w $r 1000
  fi
done
exit 0
