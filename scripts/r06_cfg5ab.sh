#!/bin/bash
# config-5 bench lines per environment spec, two rounds: scripts/r06_cfg5ab.sh OUT ENV...
set -o pipefail
O=gpurun_out/${1:?out}; mkdir -p $O; export TMPDIR=/tmp
shift
for r in 1 2; do
  for e in "$@"; do
    tag=$(echo "$e" | tr ',=/.' '____' | tail -c 48)
    envs=$( [ "$e" = "-" ] && echo "" || echo "$e" | tr ',' ' ')
    env $envs timeout -k 10 400 python -u bench.py --config 5 --no-cpu-baseline --steps 10 --warmup 2 > $O/b_${r}_${tag}.log 2>&1 || { tail -20 $O/b_${r}_${tag}.log; exit 1; }
    echo "$e: $(tail -1 $O/b_${r}_${tag}.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"], 4))')"
  done
done
