#!/bin/bash
# after a kernel change: the whole -m gpu suite, the C3 phase profile and the bench lines
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-kc}; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest $R/tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|assert" $OUT/tests.log | head -30; tail -5 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 300 python -u $R/tools/phase_profile_grasp.py > $OUT/phase.txt 2>&1 || { tail -5 $OUT/phase.txt; exit 1; }
grep -E "per substep|newton_solve|n:factor|integrate|n:H_ass|collision" $OUT/phase.txt
timeout -k 10 300 python -u $R/tools/phase_profile_grasp.py 256 cylinder > $OUT/phase_c2.txt 2>&1 || { tail -5 $OUT/phase_c2.txt; exit 1; }
grep -E "per substep|collision|newton_solve" $OUT/phase_c2.txt
timeout -k 10 300 python -u $R/bench.py --no-cpu --no-parity --no-policy --no-random > $OUT/bench.json 2> $OUT/bench.err || { tail -5 $OUT/bench.err; exit 1; }
python3 -c "import json; d=json.loads(open('$OUT/bench.json').read().strip().split(chr(10))[-1]); print('C3', d['ms_per_step'], 'per-step', d['per_step_api']['ms_per_step'], 'C2', d['c2_single_cylinder_256']['ms_per_step'], 'C1', d['c1_single_env_200_steps']['device']['ms_per_step'])"
