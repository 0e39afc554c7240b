cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pt.log 2>&1; tail -3 gpurun_out/pt.log
echo "== auto"; RT_DEBUG=1 timeout -k 10 300 python scripts/shard_probe.py 2,4,8 0 1000 2>&1 | grep -E "world|rtc. lpt" | uniq
echo "== group N=1,2"; RT_MODE=group timeout -k 10 300 python scripts/shard_probe.py 2 0 1000 2>&1 | grep "world="
echo "== tail 8"; timeout -k 10 120 python scripts/tail_probe.py 8 2 1000 2>&1 | grep -v amdgpu.ids | head -8
