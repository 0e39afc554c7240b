cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for m in 1900,2714,180 2500,2714,180 1900,2714,250 2800,2714,220; do
  echo "== lane $m"; RT_MODEL_LANE=$m timeout -k 10 300 python scripts/shard_probe.py 2 0 1000 2>&1 | grep -E "world=1|world=2 max"
done
for m in 850,850,180 1100,700,180 850,850,250 1100,620,250 1300,700,220; do
  echo "== group $m"; RT_MODEL_GROUP=$m timeout -k 10 300 python scripts/shard_probe.py 4,8 0 1000 2>&1 | grep -E "max"
done
