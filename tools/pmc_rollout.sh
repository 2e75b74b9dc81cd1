#!/bin/bash
# HBM traffic of the headline's gm_rollout launches: rocprofv3 --pmc FETCH_SIZE and
# WRITE_SIZE, each in its own pass, over the bench headline alone (--steps 10 --warmup 10:
# two 10-env-step rollout launches after the per-step pre-roll).  Summarised on the CPU
# side by tools/pmc_rollout_summary.py.  usage (on the GPU box): bash tools/pmc_rollout.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for ctr in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 180 rocprofv3 --pmc $ctr --output-format csv -d $OUT/$ctr -o run -- python3 $R/bench.py --steps 10 --warmup 10 --no-cpu --no-parity --no-policy --no-c2 --no-random --no-scripted --no-c1 > $OUT/$ctr.log 2>&1 || { echo "pass $ctr failed"; tail -5 $OUT/$ctr.log; exit 1; }
  echo "pass $ctr ok"
done
echo done > $OUT/DONE
