#!/bin/bash
set -o pipefail
O=gpurun_out/s4v
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_varrho.py -m gpu > $O/tests.log 2>&1
rc=$?
tail -40 $O/tests.log
exit $rc
