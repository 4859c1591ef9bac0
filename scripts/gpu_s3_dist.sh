#!/bin/bash
# slab-decomposed step: new distributed tests, then the full GPU suite
set -o pipefail
O=gpurun_out/s3
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_distributed.py -x -v -m gpu --timeout 300 --timeout-method thread > $O/pytest_dist.log 2>&1
rc=$?; tail -30 $O/pytest_dist.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 500 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -15 $O/pytest_gpu.log; exit $rc
