#!/bin/bash
# A/B: C (committed), D (kinematics C on scan lanes), E (D + per-phase opaque lane ids)
set -o pipefail
bash tools/ab_bench.sh r04f_ab gripper-mujoco_amd/lib/ab_C.so gripper-mujoco_amd/lib/ab_D.so gripper-mujoco_amd/lib/ab_E.so || exit 1
grep -v amdgpu.ids gpurun_out/r04f_ab/ab.txt
