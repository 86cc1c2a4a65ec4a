# r06: kernel trace of one rank's plan (walker G=8, timing emulation), and the default bench line
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/prof_rank
rm -rf $OUT; mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/c4g8 -o run -- \
    python3 tools/rank_split.py --configs 4 --gpus 8 --plans 30 --t1-ms 19.58 > $OUT/c4g8.log 2>&1 || { tail -5 $OUT/c4g8.log; exit 1; }
python3 tools/plan_timeline.py $OUT/c4g8 $OUT/c4g8.log 30 $OUT/c4g8.json > /dev/null || exit 1
cp "$(find $OUT/c4g8 -name '*kernel_stats.csv' | head -1)" $OUT/c4g8_kernel_stats.csv
timeout -k 10 400 python bench.py --no-cpu-baseline > gpurun_out/bench_b.log 2>&1 || { tail -5 gpurun_out/bench_b.log; exit 1; }
tail -1 gpurun_out/bench_b.log
