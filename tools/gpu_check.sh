#!/bin/bash
# One GPU call: -m gpu tests, then a bench line, then a rocprofv3 kernel-trace summary.
# usage: bash tools/gpu_check.sh <tag> [pytest-args...]
set -o pipefail
tag=${1:-run}; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 1000 python -u -m pytest $R/tests -m gpu -v --timeout 300 --timeout-method thread "$@" > $R/gpurun_out/${tag}_tests.log 2>&1 || { echo "tests failed"; tail -30 $R/gpurun_out/${tag}_tests.log; exit 1; }
  tail -3 $R/gpurun_out/${tag}_tests.log
fi
timeout -k 10 600 python -u $R/bench.py --steps 20 --warmup 3 > $R/gpurun_out/${tag}_bench.json 2> $R/gpurun_out/${tag}_bench.err || { echo "bench failed"; tail -20 $R/gpurun_out/${tag}_bench.err; exit 1; }
cut -c1-600 $R/gpurun_out/${tag}_bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${tag}_prof -o run -- python3 $R/bench.py --steps 20 --warmup 3 --no-cpu --no-parity --no-c2 --no-policy > $R/gpurun_out/${tag}_prof.log 2>&1 || { echo "rocprof failed"; tail -20 $R/gpurun_out/${tag}_prof.log; exit 1; }
find $R/gpurun_out/${tag}_prof -name "*kernel_stats.csv" | head -3
