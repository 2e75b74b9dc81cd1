#!/bin/bash
# tail shape of rollout launches (tools/tail_timeline.py) at a few batch sizes
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-tail}; mkdir -p $OUT
timeout -k 10 200 python -u $R/tools/tail_timeline.py 4096 10 > $OUT/t4096.txt 2>&1 || { tail -5 $OUT/t4096.txt; exit 1; }
timeout -k 10 200 python -u $R/tools/tail_timeline.py 8192 10 > $OUT/t8192.txt 2>&1 || { tail -5 $OUT/t8192.txt; exit 1; }
timeout -k 10 300 env GM_DUO=1 python -u $R/bench.py --no-cpu --no-parity --no-policy --no-random --no-c2 --no-c1 > $OUT/bench_duo4096.json 2> $OUT/bench_duo4096.err || { echo "bench duo 4096 failed"; tail -20 $OUT/bench_duo4096.err; exit 1; }
grep "n=" $OUT/t*.txt
cut -c1-300 $OUT/bench_duo4096.json
