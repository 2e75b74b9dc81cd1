#!/bin/bash
# Developer probe: the grasp-workload phase profile with the collision and the constraint
# setup split into sub-phases (GM_PHASE_SPLIT_COLL / _SETUP builds).  usage: bash tools/split_profiles.sh <tag>
set -e -o pipefail
OUT=gpurun_out/$1; mkdir -p $OUT
GM_LIB=gripper-mujoco_amd/lib/prof_coll.so timeout -k 10 300 python tools/phase_profile_grasp.py 4096 > $OUT/split_coll.txt 2>&1
GM_LIB=gripper-mujoco_amd/lib/prof_setup.so timeout -k 10 300 python tools/phase_profile_grasp.py 4096 > $OUT/split_setup.txt 2>&1
grep -v amdgpu.ids $OUT/split_coll.txt | head -12
grep -v amdgpu.ids $OUT/split_setup.txt | head -18
