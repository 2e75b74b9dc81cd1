#!/bin/bash
# Round evidence on the committed kernel in one GPU call: the -m gpu suite, smoke and the
# bench line (tools/round_check.sh), the phase profiles (C3 at 2 and 1 waves per SIMD, C2),
# then the PMC passes and the kernel trace (tools/pmc_r04.sh).  usage: bash tools/evidence.sh <tag>
# (A/B comparisons of alternative builds: tools/ab_bench.sh <tag> <libA> <libB> ...)
set -o pipefail
tag=${1:?tag}
bash tools/round_check.sh $tag || exit 1
timeout -k 10 300 python -u tools/phase_profile_grasp.py 1024 > gpurun_out/$tag/phase_1wave.txt 2>&1 || exit 1
timeout -k 10 300 python -u tools/phase_profile_grasp.py 256 cylinder > gpurun_out/$tag/phase_c2.txt 2>&1 || exit 1
bash tools/pmc_r04.sh ${tag}_pmc
