#!/bin/bash
# Developer A/B of the chunked env-step: the same library under different dispatch settings,
# alternating, on the bench's steady-state C3 workload (tools/quick_bench_n.py; the
# final-state digest must agree across settings).  Each setting is K[:margin[:yields[:cmargin]]]
# -- GM_CHUNK_SUBSTEPS (0 = one-shot kernel), GM_CHUNK_MARGIN (%), GM_CHUNK_YIELDS,
# GM_CHUNK_CMARGIN (%, -1 = no yielding to yielded envs).
# usage: bash tools/chunk_ab.sh <tag> <setting>...
set -e -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
for r in 1 2; do
  for S in "$@"; do
    IFS=: read K M Y CM <<< "$S"
    echo -n "setting=$S " >> $OUT/ab.txt
    GM_CHUNK_SUBSTEPS=$K GM_CHUNK_MARGIN=${M:-50} GM_CHUNK_YIELDS=${Y:-20} GM_CHUNK_CMARGIN=${CM:-50} \
      timeout -k 10 120 python tools/quick_bench_n.py 8 4096 10 2>/dev/null >> $OUT/ab.txt
  done
done
echo done > $OUT/DONE
