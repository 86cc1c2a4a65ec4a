# r06: chunk sums over -0.0-padded chunks without per-element predicates -- tests, split-update stamps, update timing
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06t
rm -rf $O; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_fused_update.py tests/test_gpu_sharded_emul.py tests/test_gpu_plan_batch.py tests/test_gpu_pair.py > $O/t.log 2>&1 || { echo TESTS FAILED; tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
timeout -k 10 180 python tools/split_stamps.py 4 8 > $O/split_auto.jsonl 2>&1 || exit 1
timeout -k 10 120 python tools/update_bench.py --stamps > $O/update_bench.jsonl 2>&1 || exit 1
