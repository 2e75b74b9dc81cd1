#!/bin/bash
# DUO vs one-wave: the DUO parity tests, then the bench's C1 / C2 lines with DUO forced off
# and at the default, then the C3 rollout tail probe.  usage: bash tools/duo_check.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-duo}; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest $R/tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|assert" $OUT/tests.log | head -30; tail -5 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 300 env GM_DUO=0 python -u $R/bench.py --no-cpu --no-parity --no-policy --no-random > $OUT/bench_one.json 2> $OUT/bench_one.err || { echo "bench one failed"; tail -20 $OUT/bench_one.err; exit 1; }
timeout -k 10 300 python -u $R/bench.py --no-cpu --no-parity --no-policy --no-random > $OUT/bench_duo.json 2> $OUT/bench_duo.err || { echo "bench duo failed"; tail -20 $OUT/bench_duo.err; exit 1; }
timeout -k 10 200 python -u $R/tools/tail_timeline.py 4096 10 > $OUT/t4096.txt 2>&1 || { tail -5 $OUT/t4096.txt; exit 1; }
timeout -k 10 200 python -u $R/tools/tail_timeline.py 8192 10 > $OUT/t8192.txt 2>&1 || { tail -5 $OUT/t8192.txt; exit 1; }
grep "n=" $OUT/t*.txt
echo ok
