#!/bin/bash
# rocprofv3 kernel stats and the two HBM PMC passes (FETCH_SIZE, WRITE_SIZE run
# separately) over short bench runs, under gpurun_out/<tag>/.  usage: bash tools/profile_pmc.sh <tag>
set -e -o pipefail
TAG=${1:-prof}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu --no-parity --no-policy --no-c2 > $OUT/stats.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu --no-parity --no-policy --no-c2 > $OUT/pmc_fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu --no-parity --no-policy --no-c2 > $OUT/pmc_write.log 2>&1
echo done > $OUT/DONE
