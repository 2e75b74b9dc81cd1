#!/bin/bash
# Round-4 final evidence on the committed kernel (one GPU call): the -m gpu suite, smoke,
# the default bench line, the phase profiles (C3 at 2 and 1 waves per SIMD, C2), then the
# PMC passes and the kernel trace of tools/pmc_r04.sh.
set -o pipefail
bash tools/round_check.sh r04_final || exit 1
timeout -k 10 300 python -u tools/phase_profile_grasp.py 1024 > gpurun_out/r04_final/phase_1wave.txt 2>&1 || exit 1
timeout -k 10 300 python -u tools/phase_profile_grasp.py 256 cylinder > gpurun_out/r04_final/phase_c2.txt 2>&1 || exit 1
bash tools/pmc_r04.sh r04_final_pmc
