#!/bin/bash
# Kernel stats of a short N=4096 bench for two libraries, and a config-5 kernel trace:
#   scripts/r05_kt2.sh OUT LIB_B
set -o pipefail
O=gpurun_out/${1:?out}; mkdir -p "$O"; export TMPDIR=/tmp
B="python3 bench.py --no-cpu-baseline --steps 10 --warmup 3"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -f csv -d "$O/ka" -o a -- $B > "$O/ka.log" 2>&1 || exit 1
RMT_LIB=$2 timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -f csv -d "$O/kb" -o b -- $B > "$O/kb.log" 2>&1 || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -T -f csv -d "$O/k5" -o c5 -- python3 bench.py --config 5 --no-cpu-baseline --steps 3 --warmup 1 > "$O/k5.log" 2>&1 || exit 1
for d in ka kb k5; do f=$(find "$O/$d" -name "*kernel_stats.csv" | head -1); echo "== $d"; cut -d, -f1-4 "$f" | head -14; done
