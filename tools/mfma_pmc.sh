#!/bin/bash
# MFMA utilisation counters of each config's dominant rollout kernel: one
# rocprofv3 --pmc pass per config (SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F32
# GRBM_GUI_ACTIVE; no tracing domains), summarised by tools/mfma_util.py.
#   tools/mfma_pmc.sh <out dir> [label ...]   labels: c2 c3 c4 c4s2048 c5 c6
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT="$1"; shift
mkdir -p "$OUT"
declare -A ARGS=([c2]="--config 2" [c3]="--config 3" [c4]="--config 4" [c4s2048]="--config 4 --candidates 2048"
                 [c5]="--config 5" [c6]="--config 6")
for l in ${*:-c2 c3 c4 c4s2048 c5 c6}; do
  rm -rf "$OUT/$l"
  timeout -k 10 240 rocprofv3 --kernel-include-regex "rollout_(m8_)?kernel" \
      --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F32 GRBM_GUI_ACTIVE \
      --output-format csv -d "$OUT/$l" -o run -- \
      python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-variants --no-train --no-strong ${ARGS[$l]} > "$OUT/$l.log" 2>&1
  rc=$?; echo "$l pmc rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 "$OUT/$l.log"; exit $rc; fi
done
