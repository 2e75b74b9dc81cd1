#!/bin/bash
# narrowphase and collision splits on the current kernel (C3, C2)
set -o pipefail
mkdir -p gpurun_out/r04p
GM_LIB=gripper-mujoco_amd/lib/prof_narrow.so timeout -k 10 300 python tools/phase_profile_grasp.py 4096 > gpurun_out/r04p/narrow_c3.txt 2>&1 || exit 1
GM_LIB=gripper-mujoco_amd/lib/prof_coll.so timeout -k 10 300 python tools/phase_profile_grasp.py 4096 > gpurun_out/r04p/coll_c3.txt 2>&1 || exit 1
GM_LIB=gripper-mujoco_amd/lib/prof_narrow.so timeout -k 10 300 python tools/phase_profile_grasp.py 256 cylinder > gpurun_out/r04p/narrow_c2.txt 2>&1 || exit 1
for f in narrow_c3 coll_c3 narrow_c2; do echo "== $f"; grep -E "collision|k:A|k:B|crb:ch|warm|n:solve" gpurun_out/r04p/$f.txt; done
