#!/bin/bash
# The DUO helper forming the first Newton point's contact composites (newton_composites /
# duo_comp): the DUO / parity / rollout tests on the tree's libgm.so, then alternating A/B of
# lib/ab_A.so and lib/ab_B.so on C1, C2 (tools/duo_rows_ab.sh) and C3 (tools/ab_bench.sh).
# usage: bash tools/duo_comp_ab.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-duocomp}; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest $R/tests/test_duo.py $R/tests/test_grasp_parity.py $R/tests/test_facade_mjenv.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|assert" $OUT/tests.log | head -30; tail -5 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
LIBS="A B" bash $R/tools/duo_rows_ab.sh ${1:-duocomp}_small 3 || exit 1
AB_ROUNDS=2 bash $R/tools/ab_bench.sh ${1:-duocomp}_c3 $R/gripper-mujoco_amd/lib/ab_A.so $R/gripper-mujoco_amd/lib/ab_B.so && grep -v amdgpu $R/gpurun_out/${1:-duocomp}_c3/ab.txt | cut -c1-150
