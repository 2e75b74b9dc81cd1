#!/bin/bash
# Developer A/B of two libgm builds on one box: alternating kernel-time rounds
# (tools/ab_bench.sh: C3 and, with AB_C2=1, C2, state digests for bit-identity) and then
# one SQ counter pass per build over the C3 grasp workload (tools/pmc_grasp.py), each pass its
# own rocprofv3 run.  usage (GPU box): [AB_C2=1] [AB_ROUNDS=3] bash tools/ab_pmc.sh <tag> <libA> <libB>
set -e -o pipefail
TAG=$1
R=${GRAFT_REPO_ROOT:-$(pwd)}
A=$(realpath $2); B=$(realpath $3)
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
bash $R/tools/ab_bench.sh $TAG $A $B
cat $OUT/ab.txt
cd /tmp && export TMPDIR=/tmp
for v in A B; do
  L=$A; [ $v = B ] && L=$B
  GM_LIB=$L timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_THREAD_CYCLES_VALU --output-format csv -d $OUT/sq2_$v -o run -- python3 $R/tools/pmc_grasp.py 4096 3 > $OUT/sq2_$v.log 2>&1 || { echo "pass sq2_$v failed"; tail -5 $OUT/sq2_$v.log; exit 1; }
  GM_LIB=$L timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES --output-format csv -d $OUT/sq1_$v -o run -- python3 $R/tools/pmc_grasp.py 4096 3 > $OUT/sq1_$v.log 2>&1 || { echo "pass sq1_$v failed"; tail -5 $OUT/sq1_$v.log; exit 1; }
  echo "pmc $v ok"
done
echo done > $OUT/DONE
