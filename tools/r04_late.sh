#!/bin/bash
# Late round-4 evidence on the committed kernel (cylinder-box MPR instance): the -m gpu
# suite, smoke, the bench line, the phase profiles (C3 at 2 / 1 waves per SIMD, C2), the
# PMC passes and the kernel trace.  Same steps as tools/r04_final.sh, own output tag.
set -o pipefail
bash tools/round_check.sh r04_late || exit 1
timeout -k 10 300 python -u tools/phase_profile_grasp.py 1024 > gpurun_out/r04_late/phase_1wave.txt 2>&1 || exit 1
timeout -k 10 300 python -u tools/phase_profile_grasp.py 256 cylinder > gpurun_out/r04_late/phase_c2.txt 2>&1 || exit 1
bash tools/pmc_r04.sh r04_late_pmc
