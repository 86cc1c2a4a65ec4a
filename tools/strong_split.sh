#!/bin/bash
# Strong-scaling projection on ONE GPU: the per-GPU shard of a fixed-N plan timed alone
# (bench.py --candidates n), for the headline cheetah N=4096 (BASELINE configs[2]) and walker
# N=16384 (configs[3]). One JSON line per shard size into gpurun_out/strong_split.jsonl.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OUT=gpurun_out/strong_split.jsonl
: > $OUT
for spec in "3 4096" "3 2048" "3 1024" "3 512" "4 16384" "4 8192" "4 4096" "4 2048"; do
  set -- $spec
  timeout -k 10 300 python bench.py --config $1 --candidates $2 --steps ${STEPS:-30} --warmup 5 --no-cpu-baseline \
      --no-variants --no-strong --no-train > gpurun_out/ss.log 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/ss.log; exit $rc; fi
  tail -1 gpurun_out/ss.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps(dict(config=$1, candidates=$2, ms_per_plan=d['ms_per_step'], rollout_ms=d['roofline']['avg_launch_ms'], frac=d['roofline']['frac'])))" >> $OUT
  tail -1 $OUT
done
