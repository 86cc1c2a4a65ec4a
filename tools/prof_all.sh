#!/bin/bash
# rocprofv3 kernel traces of bench.py for every BASELINE config (and the walker 8-GPU shard), one
# profiler run each, summarised by tools/plan_timeline.py into gpurun_out/prof_all/<label>.json.
#   tools/prof_all.sh [label ...]      labels: c2 c3 c4 c4s2048 c4s4096 c5 c6 (default: all)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/prof_all
mkdir -p $OUT
declare -A ARGS=([c2]="--config 2" [c3]="--config 3" [c4]="--config 4" [c4s2048]="--config 4 --candidates 2048"
                 [c4s4096]="--config 4 --candidates 4096" [c5]="--config 5" [c6]="--config 6")
LABELS="${*:-c2 c3 c4 c4s2048 c5 c6}"
STEPS=${STEPS:-20}
for l in $LABELS; do
  rm -rf $OUT/$l
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$l -o run -- \
      python3 bench.py --steps $STEPS --warmup 3 --no-cpu-baseline --no-variants --no-train --no-strong ${ARGS[$l]} \
      > $OUT/$l.log 2>&1
  rc=$?; echo "$l rocprof rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 $OUT/$l.log; exit $rc; fi
  python3 tools/plan_timeline.py $OUT/$l $OUT/$l.log $STEPS $OUT/$l.json > /dev/null || exit 1
  cp "$(find $OUT/$l -name '*kernel_stats.csv' | head -1)" $OUT/${l}_kernel_stats.csv
done
