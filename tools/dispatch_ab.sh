#!/bin/bash
# Alternating A/B/... of chunked-dispatch settings on the C3 rollout launch's tail
# (tools/tail_timeline.py: 3 launches per run; launch ms, busy, work-end percentiles).
# usage: bash tools/dispatch_ab.sh <tag> <rounds> "<env settings 1>" "<env settings 2>" ...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-dab}; mkdir -p $OUT; shift
N=$1; shift
for i in $(seq 1 $N); do
  j=0
  for e in "$@"; do
    j=$((j+1))
    echo "== [$e] round $i"
    timeout -k 10 300 env $e python -u $R/tools/tail_timeline.py 4096 10 > $OUT/v${j}_$i.txt 2>&1 || { tail -5 $OUT/v${j}_$i.txt; exit 1; }
    grep "^n=" $OUT/v${j}_$i.txt | sed -e 's/ yields.*work ends (ms) p1\/10\/25\/50\/75\/90\/99\/100/ ends/' | cut -c1-150
  done
done
