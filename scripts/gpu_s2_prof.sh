#!/bin/bash
# kernel trace + stats of the N=4096 bench (kernel-level breakdown)
set -o pipefail
O=gpurun_out/s2
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -T -f csv -d $O/kt -o bench -- python3 bench.py --n 4096 --steps 5 --warmup 2 --no-cpu-baseline > $O/bench_kt.log 2>&1
rc=$?; echo "rocprof exit $rc"; f=$(find $O/kt -name "*kernel_stats.csv" | head -1); head -30 "$f" | cut -d, -f1-4
exit $rc
