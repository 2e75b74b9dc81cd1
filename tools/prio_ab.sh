#!/bin/bash
# A/B of the chunked queue's issue priority (GM_CHUNK_PRIO) on the rollout launch's tail
# (tools/tail_timeline.py, 3 launches per run), alternating, then the bench lines.
# usage: bash tools/prio_ab.sh <tag> [rounds]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-prio}; mkdir -p $OUT
N=${2:-2}
for i in $(seq 1 $N); do
  for p in 0 1; do
    echo "== GM_CHUNK_PRIO=$p round $i"
    GM_CHUNK_PRIO=$p timeout -k 10 300 python -u $R/tools/tail_timeline.py 4096 10 > $OUT/tail_p${p}_$i.txt 2>&1 || { tail -5 $OUT/tail_p${p}_$i.txt; exit 1; }
    grep "^n=" $OUT/tail_p${p}_$i.txt | cut -c1-200
  done
done
