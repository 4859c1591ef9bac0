#!/bin/bash
# chain variants: per-phase clocks and the per-fit trace (critical-path analysis on the host)
set -o pipefail
O=gpurun_out/${1:?out}; shift
mkdir -p $O
for v in "$@"; do
  RMT_CH_VARIANT=$v RMT_EX_PROFILE=1 RMT_EX_TRACE=$O/trace_v$v.bin timeout -k 10 200 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline > $O/v$v.log 2>&1 || { tail -5 $O/v$v.log; exit 1; }
  echo "v$v $(grep chain-prof $O/v$v.log | tail -1)"
done
