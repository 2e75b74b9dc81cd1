#!/bin/bash
# A/B: E (committed), I (update_all inlined, deferred pivot scaling, one contact loop),
# J2 (I with alias analysis in codegen), K0 (I + branch-free H-row loads, H assembly cdof by
# row_newbcast), K (K0 + chain mass rows / forces formed in crb_rne)
set -o pipefail
bash tools/ab_bench.sh r04g_ab gripper-mujoco_amd/lib/ab_E.so gripper-mujoco_amd/lib/ab_I.so gripper-mujoco_amd/lib/ab_J2.so gripper-mujoco_amd/lib/ab_K0.so gripper-mujoco_amd/lib/ab_K.so || exit 1
grep -v amdgpu.ids gpurun_out/r04g_ab/ab.txt
