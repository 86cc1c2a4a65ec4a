set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_train_native.py tests/test_gpu_train_adam.py tests/test_train.py -m gpu > gpurun_out/train_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -15 gpurun_out/train_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/train_split_ab.py 512 200 50 > gpurun_out/train_split_ab.jsonl 2>&1
rc=$?; echo "ab rc=$rc"; cat gpurun_out/train_split_ab.jsonl
