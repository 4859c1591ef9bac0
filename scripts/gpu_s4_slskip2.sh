#!/bin/bash
set -o pipefail
O=gpurun_out/s4k2
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_mac.py tests/test_gpu_mac_slab.py tests/test_distributed.py -m gpu > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats -T -f csv -d $O/kt -o b -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > $O/kt.log 2>&1 || exit $?
tail -1 $O/kt.log | cut -c1-200
f=$(find $O/kt -name "*kernel_stats.csv" | head -1); grep -E "k_sim_sl|k_ex_chain" "$f" | cut -d, -f1-4
timeout -k 10 300 python -u tools/mac_bench.py 8192 5 > $O/mac.json 2>&1 || exit $?
tail -1 $O/mac.json | cut -c1-80
