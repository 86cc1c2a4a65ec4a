# r06: where the split update's time goes at a walker rank -- per-workgroup stamps, workgroups per row A/B
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06j
rm -rf $O; mkdir -p $O
timeout -k 10 180 python tools/split_stamps.py 4 8 > $O/split_auto.jsonl 2>&1 || exit 1
for S in 4 2 16; do MBRL_DIAG_SPLIT_S=$S timeout -k 10 180 python tools/split_stamps.py 4 8 > $O/split_s$S.jsonl 2>&1 || exit 1; done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /root/repo/$O/prof -o rs -- python3 /root/repo/tools/rank_split.py --mode strong --configs 4 --gpus 8 --plans 20 --t1-ms 19.55 > /root/repo/$O/rs_prof.log 2>&1 || exit 1
