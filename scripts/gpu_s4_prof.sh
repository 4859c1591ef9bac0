#!/bin/bash
# bench line at N=4096 + kernel stats (config 4) and the MAC single-GPU step (config 5)
set -o pipefail
O=gpurun_out/s4p
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/bench_n4096.log 2>&1 || exit $?
tail -1 $O/bench_n4096.log | cut -c1-300
timeout -k 10 400 rocprofv3 --kernel-trace --stats -T -f csv -d $O/kt -o bench -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > $O/bench_kt.log 2>&1 || exit $?
f=$(find $O/kt -name "*kernel_stats.csv" | head -1); cp "$f" $O/kernel_stats_n4096.csv; cut -d, -f1-4 "$f" | head -24
timeout -k 10 300 python -u tools/mac_bench.py 8192 5 > $O/mac.json 2>&1 || exit $?
tail -1 $O/mac.json
