#!/bin/bash
# One GPU-box session: parity tests, smoke, bench, rocprofv3 kernel-trace summary.
# Every GPU step has its own time limit; a crash/fault/timeout (rc other than 0/1) ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
STEP="${1:-all}"

fatal() { case "$1" in 0|1) return 1;; *) return 0;; esac; }

if [ "$STEP" = all ] || [ "$STEP" = test ]; then
  timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider -x ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -40 gpurun_out/pytest_gpu.log
  if fatal $rc; then exit $rc; fi
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
  rc=$?; echo "smoke rc=$rc"; tail -5 gpurun_out/smoke.log
  if fatal $rc; then exit $rc; fi
fi
if [ "$STEP" = all ] || [ "$STEP" = bench ]; then
  timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1
  rc=$?; echo "bench rc=$rc"; tail -5 gpurun_out/bench.log
  if fatal $rc; then exit $rc; fi
fi
if [ "$STEP" = all ] || [ "$STEP" = prof ]; then
  rm -rf gpurun_out/prof
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- \
      python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-variants --no-train --no-strong ${PROF_ARGS:-} > gpurun_out/prof.log 2>&1
  rc=$?; echo "rocprof rc=$rc"; tail -3 gpurun_out/prof.log
  find gpurun_out/prof -name "*stats*" | head
  python3 tools/prof_summary.py gpurun_out/prof gpurun_out/prof.log 20 gpurun_out/prof/rollout_summary.json
fi
