#!/bin/bash
# Strong-scaling projection on ONE GPU: the per-GPU shard of a fixed-N plan timed alone
# (bench.py --candidates n), for the headline cheetah N=4096 (BASELINE configs[2]), walker N=16384
# (configs[3]) and the humanoid E=5 ensemble N=32768 H=50 (configs[4]). One JSON line per shard size
# into gpurun_out/strong_split.jsonl. Usage: bash tools/strong_split.sh [config ...] (default: 3 4 5)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OUT=gpurun_out/strong_split.jsonl
: > $OUT
CFGS="${*:-3 4 5}"
for c in $CFGS; do
  case $c in
    3) specs="4096 2048 1024 512"; steps=${STEPS:-30};;
    4) specs="16384 8192 4096 2048"; steps=${STEPS:-30};;
    5) specs="32768 16384 8192 4096"; steps=${STEPS5:-8};;
    *) echo "unknown config $c"; exit 2;;
  esac
  for n in $specs; do
    timeout -k 10 300 python bench.py --config $c --candidates $n --steps $steps --warmup 2 --no-cpu-baseline \
        --no-variants --no-strong --no-train > gpurun_out/ss.log 2>&1
    rc=$?
    if [ $rc -ne 0 ]; then tail -5 gpurun_out/ss.log; exit $rc; fi
    tail -1 gpurun_out/ss.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps(dict(config=$c, candidates=$n, ms_per_plan=d['ms_per_step'], plan_gpu_ms=d['plan_gpu_ms'], rollout_ms=d['roofline']['avg_launch_ms'], frac=d['roofline']['frac'])))" >> $OUT
    tail -1 $OUT
  done
done
python3 - "$OUT" <<'EOF'
import json, sys
rows = [json.loads(l) for l in open(sys.argv[1])]
full = {}
for r in rows:
    full.setdefault(r["config"], r["ms_per_plan"])   # the first row of a config is its full N (1 GPU)
for r in rows:
    base = [x for x in rows if x["config"] == r["config"]][0]
    r["gpus"] = base["candidates"] // r["candidates"]
    r["projected_speedup"] = round(full[r["config"]] / r["ms_per_plan"], 3)
with open(sys.argv[1], "w") as f:
    for r in rows:
        f.write(json.dumps(r) + "\n")
for r in rows:
    print(f"config {r['config']} N/{r['gpus']}={r['candidates']}: {r['ms_per_plan']:.3f} ms/plan, "
          f"rollout {r['rollout_ms']:.3f} ms (frac {r['frac']:.3f}), projected {r['projected_speedup']:.2f}x")
EOF
