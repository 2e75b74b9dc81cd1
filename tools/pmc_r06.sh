#!/bin/bash
# Round-6 counter passes over the bench headline alone (bench.py --steps 10 --warmup 10, the
# 10-env-step gm_rollout launches of the C3 benchmark mix): HBM traffic (FETCH_SIZE, WRITE_SIZE)
# and the SQ issue / wait / instruction-mix groups, each counter group its own rocprofv3 run.
# Summaries on the CPU side: tools/pmc_rollout_summary.py (traffic), tools/pmc_sq_rollout_summary.py
# (SQ).  usage (on the GPU box): bash tools/pmc_r06.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
HL="python3 $R/bench.py --steps 10 --warmup 10 --no-cpu --no-parity --no-policy --no-c2 --no-random --no-scripted --no-c1"
pass() { local name=$1; shift; timeout -s KILL 240 rocprofv3 --pmc "$@" --output-format csv -d $OUT/$name -o run -- $HL > $OUT/$name.log 2>&1 || { echo "pass $name failed"; tail -5 $OUT/$name.log; exit 1; }; echo "pass $name ok"; }
pass FETCH_SIZE FETCH_SIZE
pass WRITE_SIZE WRITE_SIZE
pass sq1 SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES
pass sq2 SQ_INSTS_SALU SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_THREAD_CYCLES_VALU
echo done > $OUT/DONE
