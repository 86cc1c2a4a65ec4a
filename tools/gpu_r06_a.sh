# r06: sharded-plan, selection and training checks, selection timing, per-rank projection
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_fused_update.py tests/test_gpu_sharded_emul.py tests/test_gpu_multi_rccl.py tests/test_gpu_recognition_cache.py tests/test_gpu_train_native.py "tests/test_gpu_parity.py" -k "select or sharded or rccl or staged or fused or update or goal or cached or train" > gpurun_out/t1.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/t1.log; exit 1; }
tail -3 gpurun_out/t1.log
timeout -k 10 120 python tools/select_bench.py > gpurun_out/select_bench.json 2>&1 || exit 1
cat gpurun_out/select_bench.json
for n in 4096 16384 32768; do timeout -k 10 120 python tools/select_stamps.py $n 130 250 >> gpurun_out/select_stamps.txt 2>&1 || exit 1; timeout -k 10 120 python tools/select_stamps.py $n >> gpurun_out/select_stamps.txt 2>&1 || exit 1; done
timeout -k 10 500 python tools/rank_split.py --configs 4 3 --gpus 8 4 2 --out gpurun_out/rank_split.jsonl > gpurun_out/rs.log 2>&1
