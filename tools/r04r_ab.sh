#!/bin/bash
# A/B: A (committed) vs B (MPR instance with the cylinder-box support types fixed), C3 + C2
set -o pipefail
AB_C2=$AB_C2 bash tools/ab_bench.sh r04r_ab gripper-mujoco_amd/lib/ab_A.so gripper-mujoco_amd/lib/ab_B.so || exit 1
grep -v amdgpu.ids gpurun_out/r04r_ab/ab.txt
