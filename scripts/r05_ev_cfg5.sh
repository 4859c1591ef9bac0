#!/bin/bash
# Config-5 evidence at the benched commit: kernel trace + stats (step window) and the
# FETCH_SIZE / WRITE_SIZE passes (one counter group per run):  scripts/r05_ev_cfg5.sh OUT
set -o pipefail
O=gpurun_out/${1:?out}; mkdir -p "$O"; export TMPDIR=/tmp
run() {  # name timeout args...
    local n=$1 t=$2; shift 2
    echo "== $n $(date +%T)"
    timeout -s KILL "$t" rocprofv3 "$@" > "$O/$n.log" 2>&1 || { tail -5 "$O/$n.log"; exit 1; }
}
B5="python3 bench.py --config 5 --no-cpu-baseline"
run kt5 300 --kernel-trace --stats -T -f csv -d "$O/kt5" -o kt -- $B5 --steps 4 --warmup 1
run f5 200 --pmc FETCH_SIZE --kernel-trace -T -f csv -d "$O/f5" -o f -- $B5 --steps 3 --warmup 1
run w5 200 --pmc WRITE_SIZE --kernel-trace -T -f csv -d "$O/w5" -o w -- $B5 --steps 3 --warmup 1
rev=$(cat .git_rev 2>/dev/null || echo unknown)
python3 tools/pmc_traffic.py "$O/f5" "$O/w5" "$O/pmc_traffic_cfg5_n8192.json" "$rev" k_mac_centres_m2,k_m2_bound | head -8
f=$(find "$O/kt5" -name "*kernel_stats.csv" | head -1); cp "$f" "$O/kt_stats_cfg5.csv"
t=$(find "$O/kt5" -name "*kernel_trace.csv" | head -1)
python3 tools/step_window.py "$t" 1 k_m2_bound > "$O/step_window_cfg5.txt" && tail -1 "$O/step_window_cfg5.txt"
echo done
