#!/bin/bash
set -o pipefail
O=gpurun_out/s3
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_schemes.py -v -m gpu --timeout 120 --timeout-method thread > $O/pytest_schemes.log 2>&1
rc=$?; grep -E "PASS|FAIL|Error|assert|Mismatch|Max abs|rror" $O/pytest_schemes.log | head -40; exit $rc
