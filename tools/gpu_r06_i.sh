# r06: ballots from the compare, whole-wave-valid passes -- tests, select / update timing and stamps
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06i
rm -rf $O; mkdir -p $O
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_fused_update.py tests/test_gpu_sharded_emul.py tests/test_gpu_m8.py tests/test_gpu_fuzz.py -k "select or fused or split or timing or peer or pair or full_size or fuzz or m8" > $O/t.log 2>&1 || { echo TESTS FAILED; tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
timeout -k 10 120 python tools/select_bench.py > $O/select_bench.json 2>&1 || exit 1
for n in 4096 16384 32768; do timeout -k 10 120 python tools/select_stamps.py $n 130 250 >> $O/select_stamps.txt 2>&1 || exit 1; done
timeout -k 10 120 python tools/update_bench.py --stamps > $O/update_bench.jsonl 2>&1 || exit 1
timeout -k 10 180 python tools/split_stamps.py 4 8 > $O/split_stamps.jsonl 2>&1 || exit 1
timeout -k 10 300 python tools/rank_split.py --mode strong --configs 4 --gpus 8 --out $O/strong_c4g8.jsonl > $O/rs.log 2>&1 || exit 1
