#!/bin/bash
# record arena: fixed per-fit slots vs the shared bump cursor (k_ex_geom time), parity
set -o pipefail
O=gpurun_out/s4a
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -m gpu > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for mode in bump slots; do
  RMT_EX_ARENA=$mode timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/bench_$mode.log 2>&1 || exit $?
  echo $mode $(tail -1 $O/bench_$mode.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'])")
  RMT_EX_ARENA=$mode timeout -k 10 400 rocprofv3 --kernel-trace --stats -T -f csv -d $O/kt_$mode -o b -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > $O/kt_$mode.log 2>&1 || exit $?
  f=$(find $O/kt_$mode -name "*kernel_stats.csv" | head -1); grep -E "k_ex_geom|k_ex_chain|k_ex_fix" "$f" | cut -d, -f1-4
done
