# r06 final (bitmap compaction from 8 keys per lane): the full GPU suite, smoke, select / update timing, the rank rows and the bench line
# projection and the bench line on the final tree
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06v
rm -rf $O; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gputest.txt 2>&1 || { echo TESTS FAILED; tail -30 $O/gputest.txt; exit 1; }
tail -1 $O/gputest.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { tail -5 $O/smoke.txt; exit 1; }
timeout -k 10 120 python tools/select_bench.py > $O/select_bench.json 2>&1 || exit 1
timeout -k 10 120 python tools/update_bench.py > $O/update_bench.jsonl 2>&1 || exit 1
timeout -k 10 400 python tools/rank_split.py --mode strong --configs 4 --gpus 2 4 8 --out $O/strong.jsonl > $O/rs.log 2>&1 || exit 1
timeout -k 10 300 python tools/rank_split.py --mode weak --configs 3 --gpus 2 4 8 --out $O/weak.jsonl >> $O/rs.log 2>&1 || exit 1
timeout -k 10 500 python bench.py > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 1; }
tail -1 $O/bench.log > $O/bench.json
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /root/repo/$O/prof -o run -- python3 /root/repo/bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-variants --no-train --no-strong > /root/repo/$O/prof.log 2>&1 || exit 1
