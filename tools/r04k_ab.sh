#!/bin/bash
# A/B: N; R (lock rows in crb first block, base composite one lane per value, no per-phase clock branches);
# Q (R with the wave-scope fence only); S (R + contact impedance / D in the collision epilogue)
# substep_loop without the per-phase clock branches), Q (R with the wave-scope fence only)
set -o pipefail
bash tools/ab_bench.sh r04k_ab gripper-mujoco_amd/lib/ab_N.so gripper-mujoco_amd/lib/ab_R.so gripper-mujoco_amd/lib/ab_Q.so gripper-mujoco_amd/lib/ab_S.so || exit 1
grep -v amdgpu.ids gpurun_out/r04k_ab/ab.txt
