#!/bin/bash
# Session 2: LDS FFT DCT-I -- parity (sizes, projection pieces, whole loops), then bench.
set -o pipefail
O=gpurun_out/s2
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -k "dct or projection" > $O/pytest_dct.log 2>&1
rc=$?; echo "pytest dct exit $rc"; grep -E "PASS|FAIL|Error|assert" $O/pytest_dct.log | tail -14; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest gpu exit $rc"; tail -2 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --n 4096 --steps 5 --warmup 2 --no-cpu-baseline > $O/bench_n4096.log 2>&1
rc=$?; echo "bench exit $rc"; grep -o '"ms_per_step[^,]*\|"phase_ms_per_step.*' $O/bench_n4096.log
exit $rc
