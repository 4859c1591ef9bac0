#!/bin/bash
# GPU tests matching TESTEXPR, then config-3 bench lines per environment spec, two rounds:
#   scripts/r06_cfg3ab.sh OUT TESTEXPR ENV...
set -o pipefail
O=gpurun_out/${1:?out}; mkdir -p $O; export TMPDIR=/tmp
T=$2; shift 2
if [ "$T" != "-" ]; then
  timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$T" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
  tail -1 $O/tests.log
fi
for r in 1 2; do
  for e in "$@"; do
    tag=$(echo "$e" | tr ',=/.' '____' | tail -c 48)
    envs=$( [ "$e" = "-" ] && echo "" || echo "$e" | tr ',' ' ')
    env $envs timeout -k 10 300 python -u bench.py --config 3 --no-cpu-baseline > $O/b_${r}_${tag}.log 2>&1 || { tail -20 $O/b_${r}_${tag}.log; exit 1; }
    echo "$e: $(tail -1 $O/b_${r}_${tag}.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"], 4))')"
  done
done
