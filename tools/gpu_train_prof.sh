# rocprofv3 kernel trace of the training bench (fused default and the five-launch layout)
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf gpurun_out/trainprof
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/trainprof -o run -- python3 tools/train_bench.py 512 10 > gpurun_out/train_bench.txt 2>&1
rc=$?; echo "prof rc=$rc"; tail -1 gpurun_out/train_bench.txt
[ $rc -eq 0 ] || exit $rc
find gpurun_out/trainprof -name "*kernel_stats.csv" | head -3
