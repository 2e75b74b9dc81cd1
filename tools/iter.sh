#!/bin/bash
# Developer loop on the GPU box: parity tests, then the phase profile and a timing probe.
# usage: bash tools/iter.sh <tag>
set -e -o pipefail
TAG=${1:-iter}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
timeout -k 10 200 python tools/phase_profile.py 4096 > $OUT/phase.txt 2>&1
timeout -k 10 200 python tools/tail_probe.py 4096 2048 > $OUT/tail.txt 2>&1
echo done > $OUT/DONE
