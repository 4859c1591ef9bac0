#!/bin/bash
set -o pipefail
O=gpurun_out/s3
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread > $O/pytest_gpu3.log 2>&1
rc=$?; tail -4 $O/pytest_gpu3.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/bench_ov.log 2>&1 || exit $?
tail -1 $O/bench_ov.log | cut -c1-420
RMT_NO_OVERLAP=1 timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/bench_noov.log 2>&1 || exit $?
tail -1 $O/bench_noov.log | cut -c1-420
