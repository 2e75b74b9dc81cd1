#!/bin/bash
# A/B: SC (committed) vs BS (box-box separating axes evaluated branch-free, then tested)
set -o pipefail
bash tools/ab_bench.sh r04q_ab gripper-mujoco_amd/lib/ab_SC.so gripper-mujoco_amd/lib/ab_BS.so || exit 1
grep -v amdgpu.ids gpurun_out/r04q_ab/ab.txt
