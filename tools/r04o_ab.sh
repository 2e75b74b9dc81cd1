#!/bin/bash
# A/B: Z (committed), BB (box-box pass-1 hits kept in the LDS union for pass 2), SC (BB + border transfers loaded in batches)
set -o pipefail
bash tools/ab_bench.sh r04o_ab gripper-mujoco_amd/lib/ab_Z.so gripper-mujoco_amd/lib/ab_BB.so gripper-mujoco_amd/lib/ab_SC.so || exit 1
grep -v amdgpu.ids gpurun_out/r04o_ab/ab.txt
