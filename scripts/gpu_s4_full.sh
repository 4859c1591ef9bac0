#!/bin/bash
# full GPU suite, then the MAC slab bench (N=8192, G=8 virtual slabs)
set -o pipefail
mkdir -p gpurun_out/s4
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu \
  > gpurun_out/s4/full_tests.log 2>&1
rc=$?
tail -15 gpurun_out/s4/full_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/mac_slab_bench.py 8192 8 3 > gpurun_out/s4/macslab_g8b.json 2> gpurun_out/s4/macslab_g8b.err
rc=$?
cat gpurun_out/s4/macslab_g8b.json
exit $rc
