#!/bin/bash
# A/B of two builds of the extension on one box: alternate runs of bench.py's rollout timing.
#   bash tools/ab.sh <lib A> <lib B> [bench args...]
set -u
A="$1"; B="$2"; shift 2
for i in 1 2 3; do
  for lib in "$A" "$B"; do
    MBRL_AMD_LIB="$lib" timeout -k 10 120 python bench.py --no-cpu-baseline --no-variants --no-train --steps 30 "$@" 2>/dev/null | tail -1 | \
      python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$(basename $lib)', round(d['ms_per_step'],4), round(d['roofline']['avg_launch_ms'],4), round(d['roofline']['frac'],4))" || exit 1
  done
done
