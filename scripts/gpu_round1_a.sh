#!/bin/bash
# First GPU pass: parity tests (without the long Ghia runs), smoke, short bench, profile.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
rocm-smi --showproductname > gpurun_out/gpu_info.txt 2>&1; nproc >> gpurun_out/gpu_info.txt; lscpu | grep "Model name" >> gpurun_out/gpu_info.txt
timeout -k 10 600 python -m pytest tests -m gpu -x -q -k "not ghia" > gpurun_out/pytest_gpu.log 2>&1
echo "pytest exit $?" >> gpurun_out/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 300 python bench.py --n 1024 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench1024.log 2>&1 && \
timeout -k 10 400 python bench.py --n 4096 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench4096.log 2>&1
echo "done $?"
