#!/bin/bash
# Round-5 SQ passes (issue / waits / VALU and SALU mix), each counter group its own run:
# C3 (4096 envs, one-wave kernel) and C2 (256 envs, one cylinder: DUO workgroups), over
# tools/pmc_grasp.py's steady-state grasp workload.  usage (GPU box): bash tools/pmc_r05.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
pass() { local name=$1; shift; local prog=$1; shift; timeout -s KILL 240 rocprofv3 --pmc "$@" --output-format csv -d $OUT/$name -o run -- $prog > $OUT/$name.log 2>&1 || { echo "pass $name failed"; tail -5 $OUT/$name.log; exit 1; }; echo "pass $name ok"; }
C3="python3 $R/tools/pmc_grasp.py 4096 3"
C2="python3 $R/tools/pmc_grasp.py 256 3 cylinder"
for w in c3 c2; do
  P=$C3; [ $w = c2 ] && P=$C2
  pass ${w}_sq1 "$P" SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES
  pass ${w}_sq2 "$P" SQ_INSTS_SALU SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_THREAD_CYCLES_VALU
done
echo done > $OUT/DONE
