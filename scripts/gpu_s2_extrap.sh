#!/bin/bash
# Session 2: extrapolation chain path -- parity first (each step has its own limit, the
# chain stops at the first failure), then the per-phase chain profile and a short bench.
set -o pipefail
O=gpurun_out/s2
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -k "extrapolation" > $O/pytest_extrap.log 2>&1
rc=$?; echo "pytest extrap exit $rc"; tail -3 $O/pytest_extrap.log; [ $rc -eq 0 ] || exit $rc
RMT_EX_PROFILE=1 timeout -k 10 200 python tools/chain_prof.py disc4096 > $O/chain_prof.log 2>&1
rc=$?; grep chain-prof $O/chain_prof.log | tail -1; [ $rc -eq 0 ] || exit $rc
if [ "$1" == "full" ]; then
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest gpu exit $rc"; tail -2 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --n 4096 --steps 5 --warmup 2 --no-cpu-baseline > $O/bench_n4096.log 2>&1
rc=$?; echo "bench exit $rc"; tail -1 $O/bench_n4096.log | cut -c1-300; grep -o '"phase_ms_per_step.*' $O/bench_n4096.log
fi
exit $rc
