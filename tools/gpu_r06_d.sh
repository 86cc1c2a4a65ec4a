# r06: per-rank-faithful strong rows (c4, c3, c5), weak rows (c3), kernel trace of one rank's plan, the
# default bench line -- written under gpurun_out/r06/
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06
mkdir -p $O
rm -f $O/strong_split.jsonl $O/weak_split.jsonl
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_fused_update.py tests/test_gpu_sharded_emul.py -k "select or fused or split or timing or peer or pair or full_size" > $O/t_select.log 2>&1 || { echo TESTS FAILED; tail -30 $O/t_select.log; exit 1; }
tail -1 $O/t_select.log
timeout -k 10 120 python tools/select_bench.py > $O/select_bench.json 2>&1 || exit 1
timeout -k 10 400 python tools/rank_split.py --mode strong --configs 4 3 --gpus 2 4 8 --out $O/strong_split.jsonl > $O/strong.log 2>&1 || { tail -5 $O/strong.log; exit 1; }
timeout -k 10 400 python tools/rank_split.py --mode strong --configs 5 --gpus 2 4 8 --plans 60 --out $O/strong_split.jsonl >> $O/strong.log 2>&1 || { tail -5 $O/strong.log; exit 1; }
timeout -k 10 300 python tools/rank_split.py --mode weak --configs 3 --gpus 2 4 8 --out $O/weak_split.jsonl > $O/weak.log 2>&1 || { tail -5 $O/weak.log; exit 1; }
rm -rf $O/prof_rank; mkdir -p $O/prof_rank
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_rank/c4g8 -o run -- \
    python3 tools/rank_split.py --configs 4 --gpus 8 --plans 30 --t1-ms 19.58 > $O/prof_rank/c4g8.log 2>&1 || { tail -5 $O/prof_rank/c4g8.log; exit 1; }
python3 tools/plan_timeline.py $O/prof_rank/c4g8 $O/prof_rank/c4g8.log 30 $O/prof_rank/c4g8.json > /dev/null || exit 1
cp "$(find $O/prof_rank/c4g8 -name '*kernel_stats.csv' | head -1)" $O/prof_rank/c4g8_kernel_stats.csv
timeout -k 10 500 python bench.py > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 1; }
tail -1 $O/bench.log > $O/bench.json
