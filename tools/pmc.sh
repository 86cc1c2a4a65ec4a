#!/bin/bash
# PMC counter passes for the rollout kernel (each pass its own rocprofv3 run; no tracing domains).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
CMD="python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-variants --no-train ${BENCH_ARGS:-}"
rm -rf gpurun_out/pmc && mkdir -p gpurun_out/pmc
i=0
for set in "${@}"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-include-regex "${KREGEX:-rollout_kernel}" --pmc $set --output-format csv \
      -d gpurun_out/pmc/p$i -o p$i -- $CMD > gpurun_out/pmc/p$i.log 2>&1
  rc=$?; echo "pass $i ($set) rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/pmc/p$i.log; exit $rc; fi
done
