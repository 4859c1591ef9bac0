#!/bin/bash
# Round-6 evidence at the benched commit (one counter group per rocprofv3 run, MI355X_MICROARCH.md
# HBM section):  scripts/r06_evidence.sh OUT [4|53]
#   config 4: kernel trace + stats (step window), FETCH_SIZE / WRITE_SIZE passes, the fp64
#   VALU pass of k_mom_stage, an SQ pass of the chain kernel; configs 5 and 3: kernel trace and
#   FETCH / WRITE passes.  Summaries are written by the tools/ scripts into OUT.
set -o pipefail
O=gpurun_out/${1:?out}; mkdir -p "$O"; export TMPDIR=/tmp
PART=${2:-4}
rev=$(cat .git_rev 2>/dev/null || echo unknown)
B4="python3 bench.py --no-cpu-baseline"
run() {  # name timeout args...
    local n=$1 t=$2; shift 2
    echo "== $n $(date +%T)"
    timeout -s KILL "$t" rocprofv3 "$@" > "$O/$n.log" 2>&1 || { tail -5 "$O/$n.log"; exit 1; }
}
if [ "$PART" = 4 ]; then
run kt4 300 --kernel-trace --stats -T -f csv -d "$O/kt4" -o kt -- $B4 --steps 20 --warmup 5
run f4 150 --pmc FETCH_SIZE --kernel-trace -T -f csv -d "$O/f4" -o f -- $B4 --steps 6 --warmup 1
run w4 150 --pmc WRITE_SIZE --kernel-trace -T -f csv -d "$O/w4" -o w -- $B4 --steps 6 --warmup 1
timeout -k 10 60 tools/ubench_f64 > "$O/ubench_f64.log" 2>&1 || exit 1
run v4 240 --pmc SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 \
    SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES \
    --kernel-include-regex "k_mom_stage" --kernel-trace -T -f csv -d "$O/f64" -o f64 -- $B4 --steps 6 --warmup 1
run c4 150 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS \
    SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_INSTS_BRANCH --kernel-include-regex "k_ex_chain" \
    --kernel-trace -T -f csv -d "$O/c4" -o c -- $B4 --steps 3 --warmup 1
python3 tools/pmc_traffic.py "$O/f4" "$O/w4" "$O/pmc_traffic_n4096.json" "$rev" | head -8
python3 tools/f64_roof.py "$O" "$O/f64_roof_n4096.json" "$rev" | tail -2
f=$(find "$O/kt4" -name "*kernel_stats.csv" | head -1); cp "$f" "$O/kt_stats_cfg4.csv"
t=$(find "$O/kt4" -name "*kernel_trace.csv" | head -1)
python3 tools/step_window.py "$t" 12 > "$O/step_window_n4096.txt" && tail -1 "$O/step_window_n4096.txt"
else
B5="python3 bench.py --config 5 --no-cpu-baseline"
run kt5 300 --kernel-trace --stats -T -f csv -d "$O/kt5" -o kt -- $B5 --steps 4 --warmup 1
run f5 200 --pmc FETCH_SIZE --kernel-trace -T -f csv -d "$O/f5" -o f -- $B5 --steps 3 --warmup 1
run w5 200 --pmc WRITE_SIZE --kernel-trace -T -f csv -d "$O/w5" -o w -- $B5 --steps 3 --warmup 1
B3="python3 bench.py --config 3 --no-cpu-baseline"
run kt3 300 --kernel-trace --stats -T -f csv -d "$O/kt3" -o kt -- $B3 --steps 6 --warmup 1
run f3 200 --pmc FETCH_SIZE --kernel-trace -T -f csv -d "$O/f3" -o f -- $B3 --steps 4 --warmup 1
run w3 200 --pmc WRITE_SIZE --kernel-trace -T -f csv -d "$O/w3" -o w -- $B3 --steps 4 --warmup 1
python3 tools/pmc_traffic.py "$O/f5" "$O/w5" "$O/pmc_traffic_cfg5_n8192.json" "$rev" k_mac_centres_m2,k_m2_bound | head -3
python3 tools/pmc_traffic.py "$O/f3" "$O/w3" "$O/pmc_traffic_cfg3_n1024.json" "$rev" | head -3
for c in 5 3; do
    f=$(find "$O/kt$c" -name "*kernel_stats.csv" | head -1); cp "$f" "$O/kt_stats_cfg$c.csv"
done
t=$(find "$O/kt5" -name "*kernel_trace.csv" | head -1)
python3 tools/step_window.py "$t" 1 k_m2_bound > "$O/step_window_cfg5.txt" && tail -1 "$O/step_window_cfg5.txt"
fi
echo done
