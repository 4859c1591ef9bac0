#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
AMD_SERIALIZE_KERNEL=3 RMT_DEBUG_SYNC=1 timeout -k 10 600 python -m pytest tests -m gpu -q -x -k "not ghia" > gpurun_out/pytest_gpu_c.log 2>&1
echo "pytest exit $?" >> gpurun_out/pytest_gpu_c.log
