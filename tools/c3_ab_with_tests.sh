#!/bin/bash
# The -m gpu suite on the tree's libgm.so, then tools/ab_bench.sh's C3 A/B of lib/ab_A.so and
# lib/ab_B.so (tools/build_ab.sh makes them).  usage: bash tools/c3_ab_with_tests.sh
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/r06i
timeout -k 10 900 python -u -m pytest $R/tests -m gpu -x -q --timeout 300 --timeout-method thread > $R/gpurun_out/r06i/tests.log 2>&1 || { grep -E "FAILED|Error" $R/gpurun_out/r06i/tests.log | head; tail -3 $R/gpurun_out/r06i/tests.log; exit 1; }
tail -1 $R/gpurun_out/r06i/tests.log
AB_ROUNDS=3 bash $R/tools/ab_bench.sh c3ab $R/gripper-mujoco_amd/lib/ab_A.so $R/gripper-mujoco_amd/lib/ab_B.so && grep -v amdgpu $R/gpurun_out/c3ab/ab.txt | cut -c1-170
