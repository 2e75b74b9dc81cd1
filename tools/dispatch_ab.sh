#!/bin/bash
# A/B of dispatch settings on the C3 rollout launch (tools/tail_timeline.py), alternating
# usage: bash tools/dispatch_ab.sh <tag> "<env A>" "<env B>" [rounds]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-ab}; mkdir -p $OUT
A=$2; B=$3; N=${4:-2}
for i in $(seq 1 $N); do
  timeout -k 10 200 env $A python -u $R/tools/tail_timeline.py 4096 10 > $OUT/a$i.txt 2>&1 || { tail -5 $OUT/a$i.txt; exit 1; }
  timeout -k 10 200 env $B python -u $R/tools/tail_timeline.py 4096 10 > $OUT/b$i.txt 2>&1 || { tail -5 $OUT/b$i.txt; exit 1; }
done
for f in $OUT/a*.txt $OUT/b*.txt; do echo "== $f"; grep "n=" $f | sed 's/|.*//'; done
