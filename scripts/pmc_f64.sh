# fp64 VALU roof of k_mom_stage: the measured FMA peak (tools/ubench_f64), then one SQ counter
# pass (8 SQ counters, k_mom_stage only) of a short bench -> tools/f64_roof.py
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:?out dir}
mkdir -p "$O"
timeout -k 10 60 tools/ubench_f64 > "$O/ubench_f64.log" 2>&1 || exit 1
cat "$O/ubench_f64.log"
timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 \
    SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES \
    --kernel-include-regex "k_mom_stage" --kernel-trace -T -f csv -d "$O/f64" -o f64 -- \
    python3 bench.py --steps 6 --warmup 1 --no-cpu-baseline > "$O/pmc_f64.log" 2>&1 || exit 1
echo "f64 pass done"
