# r06: HBM traffic per rollout launch (FETCH_SIZE, WRITE_SIZE: one rocprofv3 --pmc pass each) for every
# config's dominant rollout kernel, summarised into gpurun_out/r06pmc (copied to profiles/r06/pmc/)
set -o pipefail
export PROFILE_DIR=gpurun_out/r06pmc
mkdir -p $PROFILE_DIR
declare -A NAME=([c2]=cartpole-swingup-cem [c3]=cheetah-run-cem [c4]=walker-walk-cem [c5]=humanoid-stand-cem-ens5
                 [c6]=cheetah-run-reward-cem [c4s2048]=walker-walk-cem-shard2048)
declare -A ARGS=([c2]="--config 2" [c3]="--config 3" [c4]="--config 4" [c5]="--config 5" [c6]="--config 6"
                 [c4s2048]="--config 4 --candidates 2048")
declare -A REGEX=([c2]="rollout_m8_kernel" [c3]="rollout_kernel" [c4]="rollout_kernel" [c5]="rollout_kernel"
                  [c6]="rollout_kernel" [c4s2048]="rollout_kernel")
for l in ${*:-c3 c4 c4s2048 c2 c5 c6}; do
  KREGEX="${REGEX[$l]}" BENCH_ARGS="${ARGS[$l]} --no-strong" bash tools/pmc.sh FETCH_SIZE WRITE_SIZE || exit $?
  for i in 1 2; do mkdir -p $PROFILE_DIR/raw_$l/p$i; cp gpurun_out/pmc/p$i/*counter_collection.csv $PROFILE_DIR/raw_$l/p$i/ || exit 1; done
  python3 tools/traffic.py "${NAME[$l]}" "r06_$l" || exit 1
done
