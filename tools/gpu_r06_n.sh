# r06 final evidence: rocprofv3 kernel traces of bench.py for every BASELINE config, one rank's plan of
# walker over 8 GPUs under the profiler, the per-rank-faithful rows (event-free timing), the bench line
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06n
rm -rf $O gpurun_out/prof_all; mkdir -p $O
STEPS=20 bash tools/prof_all.sh c2 c3 c4 c5 c6 > $O/prof_all.log 2>&1 || { tail -5 $O/prof_all.log; exit 1; }
mkdir -p $O/prof_rank
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_rank/c4g8 -o run -- \
    python3 tools/rank_split.py --configs 4 --gpus 8 --plans 30 --t1-ms 19.44 > $O/prof_rank/c4g8.log 2>&1 || { tail -5 $O/prof_rank/c4g8.log; exit 1; }
python3 tools/plan_timeline.py $O/prof_rank/c4g8 $O/prof_rank/c4g8.log 30 $O/prof_rank/c4g8.json > /dev/null || exit 1
cp "$(find $O/prof_rank/c4g8 -name '*kernel_stats.csv' | head -1)" $O/prof_rank/c4g8_kernel_stats.csv
rm -rf $O/prof_rank/c4g8
timeout -k 10 400 python tools/rank_split.py --mode strong --configs 4 --gpus 2 4 8 --out $O/strong.jsonl > $O/rs.log 2>&1 || exit 1
timeout -k 10 300 python tools/rank_split.py --mode strong --configs 5 --gpus 8 --plans 60 --out $O/strong.jsonl >> $O/rs.log 2>&1 || exit 1
timeout -k 10 300 python tools/rank_split.py --mode weak --configs 3 --gpus 2 4 8 --out $O/weak.jsonl >> $O/rs.log 2>&1 || exit 1
timeout -k 10 500 python bench.py > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 1; }
tail -1 $O/bench.log > $O/bench.json
