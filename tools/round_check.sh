#!/bin/bash
# One GPU call: the -m gpu suite, smoke(), the default bench line, then the per-phase
# profile on the bench's grasp workload.  usage: bash tools/round_check.sh <tag> [skip-tests]
set -o pipefail
TAG=${1:-check}
OUT=gpurun_out/$TAG
mkdir -p $OUT
if [ "${2:-}" != "skip-tests" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error" $OUT/tests.log | head -20; tail -5 $OUT/tests.log; exit 1; }
  tail -2 $OUT/tests.log
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $OUT/smoke.log; exit 1; }
  tail -1 $OUT/smoke.log
fi
timeout -k 10 600 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -20 $OUT/bench.err; exit 1; }
cut -c1-400 $OUT/bench.json
timeout -k 10 300 python -u tools/phase_profile_grasp.py 4096 > $OUT/phase_grasp.txt 2>&1 || { echo "phase profile failed"; tail -5 $OUT/phase_grasp.txt; exit 1; }
cat $OUT/phase_grasp.txt
