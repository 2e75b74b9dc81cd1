#!/bin/bash
# round-4 checkpoint on the committed kernel: GPU suite, smoke, bench, phase profiles
# (C3 grasp at 2 waves/SIMD, at 1 wave/SIMD with 1024 envs, C2), then the PMC passes
set -o pipefail
bash tools/round_check.sh r04h || exit 1
timeout -k 10 300 python -u tools/phase_profile_grasp.py 1024 > gpurun_out/r04h/phase_1wave.txt 2>&1 || exit 1
timeout -k 10 300 python -u tools/phase_profile_grasp.py 256 cylinder > gpurun_out/r04h/phase_c2.txt 2>&1 || exit 1
bash tools/pmc_r04.sh r04h_pmc
