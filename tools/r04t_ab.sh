#!/bin/bash
# A/B: A (committed) vs M (the cylinder-box MPR's three stages as one straight-line loop), C3 + C2
set -o pipefail
AB_C2=1 bash tools/ab_bench.sh r04t_ab gripper-mujoco_amd/lib/ab_A.so gripper-mujoco_amd/lib/ab_M.so || exit 1
grep -v amdgpu.ids gpurun_out/r04t_ab/ab.txt
