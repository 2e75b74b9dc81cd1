#!/bin/bash
# Developer A/B timing on one box: alternate two builds of libgm (GM_LIB) in separate
# processes.  usage: bash tools/ab_time.sh <libA> <libB> <tag>
set -e -o pipefail
OUT=gpurun_out/$3
mkdir -p $OUT
for r in 1 2 3; do
  for L in $1 $2; do
    echo "== $L round $r" >> $OUT/ab.txt
    GM_LIB=$L timeout -k 10 120 python tools/quick_time.py 4096 >> $OUT/ab.txt 2>&1
  done
done
echo done > $OUT/DONE
