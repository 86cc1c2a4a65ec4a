set -u
mkdir -p gpurun_out
timeout -k 10 120 python -u tools/train_stamps.py 512 0 > gpurun_out/train_stamps_fused.txt 2>&1
rc=$?; echo "stamps rc=$rc"; cat gpurun_out/train_stamps_fused.txt | grep -v amdgpu.ids
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u tools/train_stamps.py 512 1 > gpurun_out/train_stamps_split.txt 2>&1
rc=$?; echo "stamps rc=$rc"; cat gpurun_out/train_stamps_split.txt | grep -v amdgpu.ids
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/train_split_ab.py 512 > gpurun_out/train_split_ab.jsonl 2>&1
rc=$?; echo "ab rc=$rc"; cat gpurun_out/train_split_ab.jsonl | grep -v amdgpu.ids
