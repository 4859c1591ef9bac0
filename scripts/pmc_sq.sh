set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_INST_LDS SQ_BUSY_CYCLES --kernel-include-regex "k_mom_stage|k_sim_sl|k_dct1" -T -f csv -d gpurun_out/pmc1/a -o a -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/pmc1/a.log 2>&1
echo rc=$?
