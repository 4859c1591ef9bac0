#!/bin/bash
# GPU pass with the per-cell momentum kernels: parity tests in ONE process (stop at the
# first failure), then smoke and short benches.  Each GPU step under its own timeout.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
AMD_SERIALIZE_KERNEL=3 RMT_DEBUG_SYNC=1 timeout -k 10 900 python -m pytest tests -m gpu -x -q -k "not ghia" > gpurun_out/pytest_gpu_e.log 2>&1
rc=$?; echo "pytest exit $rc" >> gpurun_out/pytest_gpu_e.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_e.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --n 1024 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench1024_e.log 2>&1 || exit $?
timeout -k 10 600 python bench.py --n 4096 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench4096_e.log 2>&1
echo "done $?"
