#!/bin/bash
# one tail_timeline run (3 launches) per dispatch setting, settings as arguments ("VAR=x VAR2=y" or "-")
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-sweep}; shift; mkdir -p $OUT
i=0
for s in "$@"; do
  i=$((i+1))
  e=$s; [ "$e" = "-" ] && e=""
  timeout -k 10 200 env $e python -u $R/tools/tail_timeline.py 4096 10 > $OUT/s$i.txt 2>&1 || { tail -5 $OUT/s$i.txt; exit 1; }
  echo "== $s"; grep "n=" $OUT/s$i.txt | sed 's/ poll.*fresh-empty/ fresh-empty/; s/|.*//'
done
