#!/bin/bash
# One GPU call of round evidence: the -m gpu suite, smoke(), the default bench line, and the
# rocprofv3 kernel trace (--stats) of the headline alone (no side lines), all under their own
# time limits.  usage (on the GPU box): bash tools/round_evidence.sh <tag>
set -o pipefail
tag=${1:?tag}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$tag
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest $R/tests -m gpu -v --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error" $OUT/tests.log | head -20; tail -5 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 600 python -u $R/bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -20 $OUT/bench.err; exit 1; }
cut -c1-400 $OUT/bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 $R/bench.py --steps 20 --warmup 10 --no-cpu --no-parity --no-c2 --no-policy --no-random --no-scripted --no-c1 > $OUT/prof.log 2>&1 || { echo "rocprof failed"; tail -20 $OUT/prof.log; exit 1; }
echo "evidence ok"
