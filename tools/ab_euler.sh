set -e -o pipefail
OUT=gpurun_out/ab_euler; mkdir -p $OUT
for r in 1 2 3; do
  for L in gripper-mujoco_amd/lib/ab_A.so gripper-mujoco_amd/lib/ab_B.so; do
    GM_LIB=$L timeout -k 10 120 python tools/quick_bench_n.py 8 4096 10 >> $OUT/ab.txt 2>&1
  done
  GM_MJ=0 GM_LIB=gripper-mujoco_amd/lib/ab_B.so timeout -k 10 120 python tools/quick_bench_n.py 8 4096 10 >> $OUT/ab.txt 2>&1
done
cat $OUT/ab.txt | grep -v amdgpu.ids
