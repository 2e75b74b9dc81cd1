#!/bin/bash
# Developer probe on the GPU box: per-phase cycles at 1, 2 and 2+ waves per SIMD (1024,
# 2048, 4096 envs) -- a phase whose cycles do not grow with the wave count is latency
# bound, one that doubles is issue bound.  usage: bash tools/occupancy_probe.sh <tag> [lib]
set -e -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
[ -n "$2" ] && export GM_LIB=$2
for n in 1024 2048 4096; do
  timeout -k 10 200 python tools/phase_profile.py $n > $OUT/phase_$n.txt 2>&1
done
echo done > $OUT/DONE
