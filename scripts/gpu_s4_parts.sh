#!/bin/bash
# two-part chain: parity (extrapolation + fused steps) with RMT_CH_PARTS=2, then chain time 1 vs 2 parts
set -o pipefail
O=gpurun_out/s4p2
mkdir -p $O
RMT_CH_PARTS=4 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -m gpu > $O/tests2.log 2>&1 || { tail -30 $O/tests2.log; exit 1; }
tail -2 $O/tests2.log
for p in 3 4; do
  RMT_CH_PARTS=$p timeout -k 10 200 python -u tools/chain_time.py 3 > $O/chain_p$p.log 2>&1 || { tail -5 $O/chain_p$p.log; exit 1; }
  echo parts=$p $(grep variant $O/chain_p$p.log)
done
true
true
