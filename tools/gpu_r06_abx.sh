set -o pipefail
AB_ROUNDS=3 bash tools/ab_bench.sh abx gripper-mujoco_amd/lib/libgm.so gripper-mujoco_amd/lib/ab_B.so && cat gpurun_out/abx/ab.txt | grep "kernel ms" && timeout -k 10 900 bash tools/pmc_r06.sh pmc06a
