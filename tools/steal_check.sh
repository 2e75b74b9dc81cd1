#!/bin/bash
# cross-XCD resumption: the dispatch bit-identity tests, then the C3 rollout tail with and without it
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-steal}; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest $R/tests/test_chunked_dispatch.py $R/tests/test_rollout.py $R/tests/test_duo.py -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|assert" $OUT/tests.log | head -30; tail -5 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 200 python -u $R/tools/tail_timeline.py 4096 10 > $OUT/t_steal.txt 2>&1 || { tail -5 $OUT/t_steal.txt; exit 1; }
timeout -k 10 200 env GM_CHUNK_STEAL=0 python -u $R/tools/tail_timeline.py 4096 10 > $OUT/t_nosteal.txt 2>&1 || { tail -5 $OUT/t_nosteal.txt; exit 1; }
timeout -k 10 200 python -u $R/tools/tail_timeline.py 4096 10 > $OUT/t_steal2.txt 2>&1 || { tail -5 $OUT/t_steal2.txt; exit 1; }
grep -h "n=" $OUT/t_*.txt
