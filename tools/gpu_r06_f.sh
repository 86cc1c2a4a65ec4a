# r06: selection after reverting the wave-0 bucket search (tests + timing), then the PMC traffic passes
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06f
rm -rf $O; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_fused_update.py -k "select or fused or split" > $O/t.log 2>&1 || { echo TESTS FAILED; tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
timeout -k 10 120 python tools/select_bench.py > $O/select_bench.json 2>&1 || exit 1
bash tools/gpu_r06_pmc.sh > $O/pmc.log 2>&1 || { tail -20 $O/pmc.log; exit 1; }
tail -8 $O/pmc.log
