#!/bin/bash
# Round-end measurement on one box: the bench line, then rocprofv3 kernel stats, the two
# HBM PMC passes, the SQ counters and the phase / dispatch-tail probes, all under
# gpurun_out/<tag>/ (tools/collect_profiles.py copies them into profiles/).
# usage: bash tools/profile_final.sh <tag>
set -e -o pipefail
TAG=${1:-final}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu --no-parity --no-policy --no-c2 > $OUT/stats.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu --no-parity --no-policy --no-c2 > $OUT/pmc_fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu --no-parity --no-policy --no-c2 > $OUT/pmc_write.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES --output-format csv -d $OUT/pmc_sq -o run -- python3 tools/pmc_step.py 4096 > $OUT/pmc_sq.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_THREAD_CYCLES_VALU --output-format csv -d $OUT/pmc_lanes -o run -- python3 tools/pmc_step.py 4096 > $OUT/pmc_lanes.log 2>&1
timeout -k 10 200 python tools/phase_profile.py 4096 > $OUT/phase_profile.txt 2>&1
timeout -k 10 200 python tools/tail_bench.py > $OUT/tail_bench.txt 2>&1
echo done > $OUT/DONE
