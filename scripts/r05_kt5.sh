#!/bin/bash
# Config-5 kernel trace (3 steps) and one steady step's kernel summary:  scripts/r05_kt5.sh OUT
set -o pipefail
O=gpurun_out/${1:?out}; mkdir -p "$O"; export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -T -f csv -d "$O/k5" -o c5 -- python3 bench.py --config 5 --no-cpu-baseline --steps 3 --warmup 1 > "$O/k5.log" 2>&1 || exit 1
t=$(find "$O/k5" -name "*kernel_trace.csv" | head -1)
python3 tools/step_window.py "$t" 2 k_mac_centres_m2 > "$O/step5.txt" && tail -1 "$O/step5.txt"
awk '{print $4, $5}' "$O/step5.txt" | awk '{a[$2]+=$1; n[$2]++} END {for (k in a) printf "%8.1f %3d %s\n", a[k], n[k], k}' | sort -rn | head -25
