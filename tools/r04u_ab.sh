#!/bin/bash
# A/B: A (committed) vs MC (the device scheduler's max-memory-clause strategy), C3 + C2
set -o pipefail
AB_C2=1 bash tools/ab_bench.sh r04u_ab gripper-mujoco_amd/lib/ab_A.so gripper-mujoco_amd/lib/ab_MC.so || exit 1
grep -v amdgpu.ids gpurun_out/r04u_ab/ab.txt
