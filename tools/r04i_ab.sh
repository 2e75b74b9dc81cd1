#!/bin/bash
# A/B: K0 (committed) vs N (operands loaded on every lane and selected); setup split profile
set -o pipefail
bash tools/ab_bench.sh r04i_ab gripper-mujoco_amd/lib/ab_K0.so gripper-mujoco_amd/lib/ab_N.so || exit 1
grep -v amdgpu.ids gpurun_out/r04i_ab/ab.txt
GM_LIB=gripper-mujoco_amd/lib/prof_setup.so timeout -k 10 300 python tools/phase_profile_grasp.py 4096 > gpurun_out/r04i_ab/split_setup.txt 2>&1 && grep -v amdgpu.ids gpurun_out/r04i_ab/split_setup.txt
