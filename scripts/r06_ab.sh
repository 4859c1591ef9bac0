#!/bin/bash
# scripts/r06_ab.sh OUT TESTEXPR ENVA ENVB: the GPU tests matching TESTEXPR (if not "-"), then
# four default bench lines (no CPU baseline) alternating environment A / B (A/B/A/B, one box)
set -o pipefail
O=gpurun_out/${1:?out}; mkdir -p $O; export TMPDIR=/tmp
if [ "$2" != "-" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "$2" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
  tail -1 $O/tests.log
fi
for r in 1 2; do
  for e in "$3" "$4"; do
    env $e timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/b_${r}_$(echo $e | tr ' =' '__').log 2>&1 || { tail -20 $O/b_*.log; exit 1; }
    echo "$e: $(tail -1 $O/b_${r}_$(echo $e | tr ' =' '__').log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["roofline"]["frac"] if d.get("roofline") else "")')"
  done
done
