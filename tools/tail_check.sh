#!/bin/bash
# tail shape of rollout launches (tools/tail_timeline.py) at a few batch sizes
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-tail}; mkdir -p $OUT
timeout -k 10 200 python -u $R/tools/tail_timeline.py 4096 10 > $OUT/t4096.txt 2>&1 || { tail -5 $OUT/t4096.txt; exit 1; }
timeout -k 10 200 python -u $R/tools/tail_timeline.py 8192 10 > $OUT/t8192.txt 2>&1 || { tail -5 $OUT/t8192.txt; exit 1; }
timeout -k 10 200 python -u $R/tools/tail_timeline.py 4096 5 > $OUT/t4096r5.txt 2>&1 || { tail -5 $OUT/t4096r5.txt; exit 1; }
grep "n=" $OUT/*.txt
