#!/bin/bash
# Kernel trace (stats + one steady step window) and counter passes of a short N=4096 bench:
#   scripts/r05_prof.sh OUT [RMT_LIB]
# pass a: SQ issue / wait counters; pass f: FETCH_SIZE; pass w: WRITE_SIZE (one group each,
# separate runs, MI355X_MICROARCH.md HBM section); tools/pmc_summary.py joins them per kernel.
set -o pipefail
O=gpurun_out/${1:?out}; mkdir -p "$O"; export TMPDIR=/tmp
[ -n "$2" ] && export RMT_LIB=$2
B="python3 bench.py --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -f csv -d "$O/kt" -o bench -- $B --steps 20 --warmup 5 \
    > "$O/kt.log" 2>&1 || { tail -5 "$O/kt.log"; exit 1; }
f=$(find "$O/kt" -name "*kernel_stats.csv" | head -1); cp "$f" "$O/kt_stats.csv"
t=$(find "$O/kt" -name "*kernel_trace.csv" | head -1)
python3 tools/step_window.py "$t" 12 > "$O/step_window.txt" && tail -1 "$O/step_window.txt"
tail -1 "$O/kt.log" | cut -c1-200
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU \
    SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_INSTS_SALU --kernel-trace -T -f csv -d "$O/pa" -o a \
    -- $B --steps 3 --warmup 1 > "$O/pa.log" 2>&1 || { tail -5 "$O/pa.log"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -T -f csv -d "$O/pf" -o f \
    -- $B --steps 3 --warmup 1 > "$O/pf.log" 2>&1 || { tail -5 "$O/pf.log"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace -T -f csv -d "$O/pw" -o w \
    -- $B --steps 3 --warmup 1 > "$O/pw.log" 2>&1 || { tail -5 "$O/pw.log"; exit 1; }
python3 tools/pmc_summary.py "$O" > "$O/pmc_summary.txt" && head -40 "$O/pmc_summary.txt"
