#!/bin/bash
set -o pipefail
O=gpurun_out/r06/base; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/benchq.log 2>&1 || exit 1
tail -1 $O/benchq.log | cut -c1-300
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -T -f csv -d $O/kt4 -o kt -- python3 bench.py --no-cpu-baseline --steps 20 --warmup 5 > $O/kt4.log 2>&1 || exit 1
t=$(find $O/kt4 -name "*kernel_trace.csv" | head -1)
python3 tools/step_window.py "$t" 12 > $O/step_window_n4096.txt && tail -1 $O/step_window_n4096.txt
f=$(find $O/kt4 -name "*kernel_stats.csv" | head -1); cp "$f" $O/kt_stats_cfg4.csv
rm -rf $O/kt4
