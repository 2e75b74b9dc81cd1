#!/bin/bash
# The DUO helper forming the constraint setup's contact rows (contact_rows / duo_rows): the
# DUO and parity tests on the working tree's libgm.so, then alternating A/B of
# lib/ab_A.so (before) and lib/ab_B.so (after) on C2 (tools/quick_bench_n.py, 256 envs,
# one cylinder: mean kernel ms + final-state digest) and C1 (tools/c1_probe.py).
# usage: [LIBS="A B"] bash tools/duo_rows_ab.sh <tag> [rounds]   (lib/ab_<X>.so for X in LIBS)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-duorows}; mkdir -p $OUT
N=${2:-3}
timeout -k 10 600 python -u -m pytest $R/tests/test_duo.py $R/tests/test_grasp_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|assert" $OUT/tests.log | head -30; tail -5 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for i in $(seq 1 $N); do
  for v in ${LIBS:-A B}; do
    L=$R/gripper-mujoco_amd/lib/ab_$v.so
    GM_LIB=$L timeout -k 10 120 python -u $R/tools/quick_bench_n.py 8 256 20 cylinder > $OUT/c2_$v$i.txt 2>&1 || { tail -5 $OUT/c2_$v$i.txt; exit 1; }
    GM_LIB=$L timeout -k 10 120 python -u $R/tools/c1_probe.py > $OUT/c1_$v$i.txt 2>&1 || { tail -5 $OUT/c1_$v$i.txt; exit 1; }
    echo "$v$i C2: $(grep -v amdgpu $OUT/c2_$v$i.txt | tail -1 | cut -c1-150)"
    echo "$v$i C1: $(grep -v amdgpu $OUT/c1_$v$i.txt | tail -1 | cut -c1-150)"
  done
done
