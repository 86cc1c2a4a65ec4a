# r06: the trajectory kernel's prologue with batched weight loads -- A/B against the previous library
# (duration against the horizon under rocprofv3), trajectory tests
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06o
rm -rf $O; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu -k "traj or trajectory or states" > $O/t.log 2>&1 || { echo TESTS FAILED; tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
cd /tmp
for v in base new; do
  if [ $v = base ]; then export MBRL_AMD_LIB=/root/repo/mujoco-mbrl_amd/mbrl_amd/libmbrl_cem_base.so; else unset MBRL_AMD_LIB; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /root/repo/$O/traj_$v -o run -- python3 /root/repo/tools/traj_bench.py > /root/repo/$O/traj_$v.log 2>&1 || exit 1
  python3 /root/repo/tools/traj_bench.py --parse /root/repo/$O/traj_$v > /root/repo/$O/traj_$v.json || exit 1
  rm -rf /root/repo/$O/traj_$v
done
