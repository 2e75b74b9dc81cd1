#!/bin/bash
# alternating A/B of an env setting on the bench's C3 lines (headline, per-step API, C5)
# usage: bash tools/bench_ab.sh <tag> "<env A>" "<env B>" [rounds]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-bab}; mkdir -p $OUT
A=$2; B=$3; N=${4:-2}
for i in $(seq 1 $N); do
  for v in a b; do
    e=$A; [ $v = b ] && e=$B; [ "$e" = "-" ] && e=""
    timeout -k 10 300 env $e python -u $R/bench.py --no-cpu --no-parity --no-c2 --no-c1 --no-random > $OUT/$v$i.json 2> $OUT/$v$i.err || { tail -5 $OUT/$v$i.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open('$OUT/$v$i.json').read().strip().split(chr(10))[-1]); print('$v$i', '$e', 'C3', d['ms_per_step'], 'per-step', d['per_step_api']['ms_per_step'], d['per_step_api']['step_kernel_ms'], 'C5', d['c5_device_policy_rollout']['ms_per_step'], 'scripted', (d.get('c3_scripted_mix_only') or {}).get('ms_per_step'))"
  done
done
