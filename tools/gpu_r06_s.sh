# r06: soak of the plans' cross-workgroup paths on the final library (pairs, cooperative trajectory) --
# whole plans with this round's selection and refit, each compared bit for bit with the first
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06s
rm -rf $O; mkdir -p $O
timeout -k 10 400 python -u tools/soak.py 90 cem > $O/soak.txt 2>&1 || { tail -20 $O/soak.txt; exit 1; }
tail -3 $O/soak.txt
