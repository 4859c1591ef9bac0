#!/bin/bash
# MAC slab decomposition: parity tests on one GPU (virtual slabs + 2 processes over gloo)
set -o pipefail
mkdir -p gpurun_out/s4
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread \
  tests/test_gpu_mac_slab.py tests/test_gpu_mac.py tests/test_distributed.py -m gpu \
  > gpurun_out/s4/macslab_tests.log 2>&1
rc=$?
tail -30 gpurun_out/s4/macslab_tests.log
exit $rc
