#!/bin/bash
# round-3 evaluation call: GPU suite, 20-step bench line, kernel trace of the bench
# usage: scripts/r03_eval.sh OUTDIR [pytest -k expr]
set -o pipefail
O=gpurun_out/${1:?out}; mkdir -p "$O"; export TMPDIR=/tmp
K=${2:+-k "$2"}
echo "== tests $(date +%T)"
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu $K > "$O/tests.log" 2>&1 \
    || { tail -40 "$O/tests.log"; exit 1; }
tail -2 "$O/tests.log"
echo "== bench $(date +%T)"
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > "$O/bench20.log" 2>&1 \
    || { tail -20 "$O/bench20.log"; exit 1; }
tail -1 "$O/bench20.log" | cut -c1-300
echo "== kt $(date +%T)"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -f csv -d "$O/kt" -o bench -- \
    python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > "$O/kt.log" 2>&1 || exit 1
f=$(find "$O/kt" -name "*kernel_stats.csv" | head -1); cp "$f" "$O/kernel_stats.csv"
cut -d, -f1-4 "$f" | head -14
