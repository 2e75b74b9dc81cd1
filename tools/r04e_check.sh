#!/bin/bash
# round-4 checkpoint: A/B of the current variants, the GPU suite + bench + phase profile,
# the narrowphase split profile and the counter list for the PMC passes
set -o pipefail
mkdir -p gpurun_out/r04e
bash tools/ab_bench.sh r04e_ab gripper-mujoco_amd/lib/ab_C.so gripper-mujoco_amd/lib/ab_D.so || exit 1
grep -v amdgpu.ids gpurun_out/r04e_ab/ab.txt
GM_LIB=gripper-mujoco_amd/lib/prof_narrow.so timeout -k 10 300 python tools/phase_profile_grasp.py 4096 > gpurun_out/r04e/split_narrow.txt 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/r04e/split_narrow.txt
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 120 rocprofv3 -L > $GRAFT_REPO_ROOT/gpurun_out/r04e/counters.txt 2>&1); echo listed
bash tools/round_check.sh r04e
timeout -k 10 300 python -u tools/phase_profile_grasp.py 256 cylinder > gpurun_out/r04e/phase_c2.txt 2>&1 && grep -v amdgpu.ids gpurun_out/r04e/phase_c2.txt
GM_LIB=gripper-mujoco_amd/lib/prof_narrow.so timeout -k 10 300 python tools/phase_profile_grasp.py 256 cylinder > gpurun_out/r04e/split_narrow_c2.txt 2>&1 && grep -v amdgpu.ids gpurun_out/r04e/split_narrow_c2.txt
