#!/bin/bash
# HBM traffic of the rollout kernel for every BASELINE config: two rocprofv3 PMC passes each
# (FETCH_SIZE, WRITE_SIZE: separate runs, no tracing domains), summarised by tools/traffic.py into
# profiles/<tag>_<label>_rollout_pmc.csv and profiles/rollout_traffic.json[config name] (bench.py's
# roofline.traffic).   tools/pmc_all.sh <round tag> [label ...]   labels: c2 c3 c4 c5 c6
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG="$1"; shift
declare -A NAME=([c2]=cartpole-swingup-cem [c3]=cheetah-run-cem [c4]=walker-walk-cem [c5]=humanoid-stand-cem-ens5
                 [c6]=cheetah-run-reward-cem)
for l in ${*:-c2 c3 c4 c5 c6}; do
  KREGEX="rollout_(m8_)?kernel" BENCH_ARGS="--config ${l#c} --no-strong" bash tools/pmc.sh FETCH_SIZE WRITE_SIZE || exit $?
  python3 tools/traffic.py "${NAME[$l]}" "${TAG}_$l" || exit 1
done
