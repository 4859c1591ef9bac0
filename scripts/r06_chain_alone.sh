#!/bin/bash
# chain duration with and without the second stream beside it (RMT_TEST_DELAY_SIDE pushes the
# side work past the chain's end)
set -o pipefail
O=gpurun_out/r06/chain_alone; mkdir -p $O; export TMPDIR=/tmp
for d in 0 700; do
  RMT_TEST_DELAY_SIDE=$d timeout -s KILL 300 rocprofv3 --kernel-trace --stats -T -f csv -d $O/kt_$d -o kt -- python3 bench.py --no-cpu-baseline --steps 20 --warmup 5 > $O/kt_$d.log 2>&1 || exit 1
  f=$(find $O/kt_$d -name "*kernel_stats.csv" | head -1); cp "$f" $O/kt_stats_delay$d.csv
  grep -h "k_ex_chain\|k_mom_stage\|k_dct1" $O/kt_stats_delay$d.csv | cut -d, -f1-8
  rm -rf $O/kt_$d
done
