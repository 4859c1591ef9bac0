#!/bin/bash
# session 5: full GPU suite, default bench line (with CPU baseline), kernel stats of the bench,
# MAC line -- on the tree after the SL block skip and the output writers
set -o pipefail
O=gpurun_out/${1:-s5f}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 500 python -u bench.py > $O/bench_default.log 2>&1 || exit $?
tail -1 $O/bench_default.log | cut -c1-250
timeout -k 10 400 rocprofv3 --kernel-trace --stats -T -f csv -d $O/kt -o bench -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > $O/bench_kt.log 2>&1 || exit $?
f=$(find $O/kt -name "*kernel_stats.csv" | head -1); cp "$f" $O/kernel_stats_n4096.csv; cut -d, -f1-4 "$f" | head -14
timeout -k 10 300 python -u tools/mac_bench.py 8192 5 > $O/mac.json 2>&1 || exit $?
tail -1 $O/mac.json
