#!/bin/bash
# Round-4 PMC passes on the C3 steady-state workload (tools/pmc_grasp.py), each counter
# group its own run: SQ issue / wait / instruction mix, memory-instruction levels, the
# instruction cache, vector L1; FETCH_SIZE and WRITE_SIZE on short bench runs.
# usage (on the GPU box): bash tools/pmc_r04.sh <tag>
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$1
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
P="python3 $R/tools/pmc_grasp.py 4096 3"
pass() { local name=$1; shift; timeout -s KILL 240 rocprofv3 --pmc "$@" --output-format csv -d $OUT/$name -o run -- $P > $OUT/$name.log 2>&1; echo "pass $name ok"; }
pass sq1 SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES
pass sq2 SQ_INSTS_SALU SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_THREAD_CYCLES_VALU
pass sq3 SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INST_LEVEL_VMEM SQ_INST_LEVEL_LDS SQ_INST_LEVEL_SMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INSTS_BRANCH
pass sqc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQC_DCACHE_HITS SQC_DCACHE_MISSES SQ_IFETCH_LEVEL SQ_BUSY_CYCLES SQ_WAVES
pass tcp TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu --no-parity --no-policy --no-c2 --no-random --no-scripted --no-c1 > $OUT/fetch.log 2>&1; echo "pass fetch ok"
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu --no-parity --no-policy --no-c2 --no-random --no-scripted --no-c1 > $OUT/write.log 2>&1; echo "pass write ok"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu --no-parity --no-policy --no-c2 --no-random --no-scripted --no-c1 > $OUT/trace.log 2>&1; echo "kernel trace ok"
echo done > $OUT/DONE
