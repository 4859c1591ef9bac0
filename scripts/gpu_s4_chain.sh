#!/bin/bash
# chain variants: inline late products (bit 8) vs the tv round trip; parity with variant 11
set -o pipefail
O=gpurun_out/s4c
mkdir -p $O
export TMPDIR=/tmp
RMT_CH_VARIANT=11 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "extrap or step or trace" > $O/tests11.log 2>&1 || { tail -30 $O/tests11.log; exit 1; }
tail -2 $O/tests11.log
timeout -k 10 400 python -u tools/chain_time.py 3 8 9 11 > $O/chain.log 2>&1 || { tail -20 $O/chain.log; exit 1; }
grep variant $O/chain.log
