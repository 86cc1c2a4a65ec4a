set -u
cd $GRAFT_REPO_ROOT
for v in libmbrl_cem libv2 libv3 libv4; do
  MBRL_AMD_LIB=$PWD/mujoco-mbrl_amd/mbrl_amd/$v.so timeout -k 10 120 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/var_$v.log 2>&1 || exit 1
  echo "$v $(python -c "import json,sys; d=json.loads(open('gpurun_out/var_$v.log').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['roofline']['avg_launch_ms'], d['roofline']['frac'])")"
done
