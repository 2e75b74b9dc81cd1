#!/bin/bash
# A/B: N (operands loaded and selected) vs O (N + lock rows inside crb_rne's first block)
set -o pipefail
bash tools/ab_bench.sh r04j_ab gripper-mujoco_amd/lib/ab_N.so gripper-mujoco_amd/lib/ab_O.so || exit 1
grep -v amdgpu.ids gpurun_out/r04j_ab/ab.txt
