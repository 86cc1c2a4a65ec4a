#!/bin/bash
# Bench every variant library mujoco-mbrl_amd/mbrl_amd/libv*.so (built by hand with -D flags) against
# the default build, config 3, on one GPU. Prints: lib ms/plan rollout-ms frac.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for f in mujoco-mbrl_amd/mbrl_amd/libmbrl_cem.so mujoco-mbrl_amd/mbrl_amd/libv*.so; do
  v=$(basename $f .so)
  MBRL_AMD_LIB=$PWD/$f timeout -k 10 120 python bench.py --steps 10 --warmup 2 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/var_$v.log 2>&1 || exit 1
  echo "$v $(python -c "import json,sys; d=json.loads(open('gpurun_out/var_$v.log').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['roofline']['avg_launch_ms'], d['roofline']['frac'])")"
done
