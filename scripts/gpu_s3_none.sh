#!/bin/bash
set -o pipefail
O=gpurun_out/s3
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread > $O/pytest_gpu2.log 2>&1
rc=$?; tail -5 $O/pytest_gpu2.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/mac_bench.py 8192 3 > $O/mac_8192b.log 2>&1
rc=$?; tail -2 $O/mac_8192b.log; exit $rc
