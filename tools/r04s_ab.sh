#!/bin/bash
# A/B: A (committed, 2 waves per SIMD register budget) vs OW (the one-wave-per-SIMD instance for batches of at most 4 envs per CU) on C2 and 1024 envs
set -o pipefail
mkdir -p gpurun_out/r04s_ab
for r in 1 2 3; do
  for L in gripper-mujoco_amd/lib/ab_A.so gripper-mujoco_amd/lib/ab_OW.so; do
    GM_LIB=$L timeout -k 10 120 python tools/quick_bench_n.py 8 256 20 cylinder >> gpurun_out/r04s_ab/ab.txt 2>&1 || exit 1
    GM_LIB=$L timeout -k 10 120 python tools/quick_bench_n.py 8 1024 10 >> gpurun_out/r04s_ab/ab.txt 2>&1 || exit 1
  done
done
grep -v amdgpu.ids gpurun_out/r04s_ab/ab.txt
