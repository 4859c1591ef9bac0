#!/bin/bash
# extrapolation v3 (K bit planes, prefetch of final window cells): parity, profile, bench
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -x -q -k "extrapolation or soft_disc or momentum or lid or taylor" > gpurun_out/pytest_ex_h.log 2>&1
rc=$?; echo "pytest exit $rc" >> gpurun_out/pytest_ex_h.log
[ $rc -eq 0 ] || exit $rc
RMT_EX_PROFILE=1 timeout -k 10 300 python bench.py --n 4096 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/exprof_h.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --n 4096 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench4096_h.log 2>&1
echo "done $?"
