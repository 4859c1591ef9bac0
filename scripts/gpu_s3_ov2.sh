#!/bin/bash
set -o pipefail
O=gpurun_out/s3
mkdir -p $O
export TMPDIR=/tmp
for e in 0 1; do
RMT_OVERLAP_EARLY=$e timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/bench_ov_e$e.log 2>&1 || exit $?
echo "early=$e"; grep -o '"ms_per_step": [0-9.]*' $O/bench_ov_e$e.log; grep -o '"phase_ms_per_step.*' $O/bench_ov_e$e.log
done
