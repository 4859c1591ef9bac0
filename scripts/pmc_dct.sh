# SQ counters of k_dct1 / k_transpose on the standalone DCT-I solve (tools/dct_bench.py 4096)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:?out dir}
mkdir -p "$O"
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS \
    SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_VALU \
    --kernel-include-regex "k_dct1|k_transpose" --kernel-trace -T -f csv -d "$O/dct" -o dct -- \
    python3 tools/dct_bench.py 4096 3 > "$O/pmc_dct.log" 2>&1 || { tail -20 "$O/pmc_dct.log"; exit 1; }
grep -E "dct solve|max" "$O/pmc_dct.log"
