#!/bin/bash
# GPU pass for the multi-wave extrapolation sweep: extrapolation parity first (bitwise vs the
# oracle, incl. 4096^2), then the rest of the parity suite, smoke, the N=4096 bench and the
# Ghia full runs.  Each GPU step under its own timeout; stop at the first failure.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -x -q -k "extrapolation" > gpurun_out/pytest_ex_f.log 2>&1
rc=$?; echo "pytest exit $rc" >> gpurun_out/pytest_ex_f.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -m pytest tests -m gpu -x -q -k "not extrapolation and not ghia" > gpurun_out/pytest_gpu_f.log 2>&1
rc=$?; echo "pytest exit $rc" >> gpurun_out/pytest_gpu_f.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_f.log 2>&1 || exit $?
timeout -k 10 600 python bench.py --n 4096 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench4096_f.log 2>&1 || exit $?
timeout -k 10 900 python -m pytest tests -m gpu -x -q -k "ghia" > gpurun_out/pytest_ghia_f.log 2>&1
rc=$?; echo "pytest exit $rc" >> gpurun_out/pytest_ghia_f.log
echo "done $rc"
