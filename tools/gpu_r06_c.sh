# r06: selection rewrite + split update: checks and timing (select / update benches and stamps), walker
# rank projection with the split update on and off
set -o pipefail
mkdir -p gpurun_out
rm -f gpurun_out/select_stamps.txt gpurun_out/upd.log gpurun_out/rank_split2.jsonl
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_fused_update.py tests/test_gpu_sharded_emul.py tests/test_gpu_parity.py tests/test_gpu_m8.py -k "select or sharded or fused or update or golden or full or plan or m8" > gpurun_out/t2.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/t2.log; exit 1; }
tail -2 gpurun_out/t2.log
timeout -k 10 120 python tools/select_bench.py > gpurun_out/select_bench.json 2>&1 || exit 1
for n in 4096 16384 32768; do timeout -k 10 120 python tools/select_stamps.py $n 130 250 >> gpurun_out/select_stamps.txt 2>&1 || exit 1; done
timeout -k 10 120 python tools/update_bench.py > gpurun_out/upd.log 2>&1 || exit 1
timeout -k 10 120 python tools/update_bench.py --stamps >> gpurun_out/upd.log 2>&1 || exit 1
for sp in 1 0; do timeout -k 10 300 python tools/rank_split.py --configs 4 --gpus 8 --t1-ms 19.58 --option update_split=$sp --out gpurun_out/rank_split2.jsonl > gpurun_out/rs2_$sp.log 2>&1 || exit 1; done
