#!/bin/bash
# HBM write / fetch bytes of the step kernel with and without the chunked dispatch
# (GM_CHUNK_SUBSTEPS=0: one-shot kernel, no yields), each counter its own rocprofv3 pass
# over 3 timed bench steps.  usage (on the GPU box): bash tools/write_traffic.sh <tag>
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
B="python3 $R/bench.py --steps 3 --warmup 1 --no-cpu --no-parity --no-policy --no-c2 --no-random --no-scripted --no-c1"
for mode in chunked oneshot; do
  for ctr in WRITE_SIZE FETCH_SIZE; do
    if [ $mode = oneshot ]; then export GM_CHUNK_SUBSTEPS=0; else unset GM_CHUNK_SUBSTEPS; fi
    timeout -s KILL 300 rocprofv3 --pmc $ctr --output-format csv -d $OUT/${mode}_$ctr -o run -- $B > $OUT/${mode}_$ctr.log 2>&1
    echo "pass $mode $ctr ok"
  done
done
unset GM_CHUNK_SUBSTEPS
echo done > $OUT/DONE
