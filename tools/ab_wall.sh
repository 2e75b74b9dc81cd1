#!/bin/bash
# Developer A/B of the whole timed env-step (bench.py's ms_per_step: every kernel of the
# step, not only gm_step_kernel) for alternating builds.  usage: bash tools/ab_wall.sh <tag> <libA> <libB> [...]
set -e -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
for r in 1 2 3; do
  for L in "$@"; do
    echo "== $L" >> $OUT/ab.txt
    GM_LIB=$L timeout -k 10 150 python bench.py --steps 20 --no-cpu --no-parity --no-policy --no-c2 2>/dev/null | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['roofline']['kernel_avg_ms'])" >> $OUT/ab.txt
  done
done
echo done > $OUT/DONE
