#!/bin/bash
# Developer A/B on one box: alternate builds of libgm (GM_LIB) on the bench's steady-state
# C3 workload (tools/quick_bench_n.py: mean kernel ms + final-state digest, which must
# agree for a bit-identical change).  usage: [AB_C2=1] [AB_ROUNDS=3] bash tools/ab_bench.sh <tag> <libA> <libB> [...]
# (AB_C2=1 adds the C2 workload: 256 envs, one cylinder)
set -e -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
for r in $(seq ${AB_ROUNDS:-3}); do
  for L in "$@"; do
    GM_LIB=$L timeout -k 10 120 python tools/quick_bench_n.py 8 4096 10 >> $OUT/ab.txt 2>&1
    if [ -n "$AB_C2" ]; then
      GM_LIB=$L timeout -k 10 120 python tools/quick_bench_n.py 8 256 20 cylinder >> $OUT/ab.txt 2>&1
    fi
  done
done
echo done > $OUT/DONE
