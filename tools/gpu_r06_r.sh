# r06: the 12-wave column-split pair kernel (two compute waves per SIMD) -- pair tests for both kernels,
# then walker's rank plan at G = 8 with each (A/B), plus the sharded-plan tests with the 12-wave kernel
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06r
rm -rf $O; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_pair.py > $O/t_pair.log 2>&1 || { echo PAIR TESTS FAILED; grep -E "FAILED|Error|assert" $O/t_pair.log | head -20; tail -5 $O/t_pair.log; exit 1; }
tail -1 $O/t_pair.log
timeout -k 10 300 python tools/rank_split.py --mode strong --configs 4 --gpus 8 --t1-ms 19.4 --option pair_waves=8 --out $O/ab.jsonl > $O/ab.log 2>&1 || exit 1
timeout -k 10 300 python tools/rank_split.py --mode strong --configs 4 --gpus 8 --t1-ms 19.4 --option pair_waves=12 --out $O/ab.jsonl >> $O/ab.log 2>&1 || exit 1
timeout -k 10 300 python tools/rank_split.py --mode strong --configs 4 --gpus 8 --t1-ms 19.4 --option pair_waves=8 --out $O/ab.jsonl >> $O/ab.log 2>&1 || exit 1
timeout -k 10 300 python tools/rank_split.py --mode strong --configs 4 --gpus 8 --t1-ms 19.4 --option pair_waves=12 --out $O/ab.jsonl >> $O/ab.log 2>&1 || exit 1
