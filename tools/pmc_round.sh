#!/bin/bash
# PMC passes on the current kernel (each counter group its own run): SQ instruction /
# wait counters on tools/pmc_step.py, FETCH_SIZE and WRITE_SIZE on short bench runs.
# usage (on the GPU box): bash tools/pmc_round.sh <tag>
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES --output-format csv -d $OUT/sq1 -o run -- python3 $R/tools/pmc_step.py 4096 > $OUT/sq1.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_THREAD_CYCLES_VALU --output-format csv -d $OUT/sq2 -o run -- python3 $R/tools/pmc_step.py 4096 > $OUT/sq2.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu --no-parity --no-policy --no-c2 > $OUT/fetch.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu --no-parity --no-policy --no-c2 > $OUT/write.log 2>&1
echo done > $OUT/DONE
