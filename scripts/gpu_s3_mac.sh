#!/bin/bash
set -o pipefail
O=gpurun_out/s3
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_mac.py -v -m gpu --timeout 120 --timeout-method thread > $O/pytest_mac.log 2>&1
rc=$?; grep -E "PASS|FAIL|Error|assert|Mismatch|Max abs" $O/pytest_mac.log | head -60; exit $rc
