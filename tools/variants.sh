#!/bin/bash
# Bench every variant library mujoco-mbrl_amd/mbrl_amd/libv*.so (built by hand with -D flags) against
# the default build on one GPU (config ${CONFIG:-3}); ${ROUNDS:-2} alternating rounds, each line:
# lib round ms/plan rollout-ms frac.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
libs="mujoco-mbrl_amd/mbrl_amd/libmbrl_cem.so $(ls mujoco-mbrl_amd/mbrl_amd/libv*.so 2>/dev/null)"
for round in $(seq 1 ${ROUNDS:-2}); do
  for f in $libs; do
    v=$(basename $f .so)
    MBRL_AMD_LIB=$PWD/$f timeout -k 10 120 python bench.py --config ${CONFIG:-3} --steps ${STEPS:-20} --warmup 2 \
        --no-cpu-baseline > gpurun_out/var_$v.log 2>&1 || exit 1
    echo "$v $round $(python -c "import json,sys; d=json.loads(open('gpurun_out/var_$v.log').read().strip().splitlines()[-1]); print(round(d['ms_per_step'],4), round(d['roofline']['avg_launch_ms'],4), round(d['roofline']['frac'],4))")"
  done
done
