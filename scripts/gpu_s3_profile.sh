#!/bin/bash
# round-1 session-3 evidence: default bench line (with the CPU baseline), kernel trace + stats
set -o pipefail
O=gpurun_out/s3p
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u bench.py > $O/bench_default.log 2>&1 || exit $?
tail -1 $O/bench_default.log | cut -c1-200
timeout -k 10 400 rocprofv3 --kernel-trace --stats -T -f csv -d $O/kt -o bench -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > $O/bench_kt.log 2>&1 || exit $?
f=$(find $O/kt -name "*kernel_stats.csv" | head -1); cp "$f" $O/kernel_stats_n4096.csv; cut -d, -f1-4 "$f" | head -16
timeout -k 10 400 rocprofv3 --kernel-trace --stats -T -f csv -d $O/mkt -o mac -- python3 tools/mac_bench.py 8192 3 > $O/mac_kt.log 2>&1 || exit $?
f=$(find $O/mkt -name "*kernel_stats.csv" | head -1); cp "$f" $O/kernel_stats_mac_n8192.csv; cut -d, -f1-4 "$f" | head -12
