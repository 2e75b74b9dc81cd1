#!/bin/bash
# A/B: R (committed); W (select operands pinned, H rows and border / palm composites loaded
# in batches); Z (W + the object's motion-subspace rows batched in H assembly, border rows and
# body_vel, the palm rows); K2 (Z + phase C constants fetched with phase A)
set -o pipefail
bash tools/ab_bench.sh r04m_ab gripper-mujoco_amd/lib/ab_R.so gripper-mujoco_amd/lib/ab_W.so gripper-mujoco_amd/lib/ab_Z.so gripper-mujoco_amd/lib/ab_K2.so || exit 1
grep -v amdgpu.ids gpurun_out/r04m_ab/ab.txt
