#!/bin/bash
# chain: 12 waves (current), 12 waves with half-chunk fold, 16 waves (spills) -- chain time
set -o pipefail
O=gpurun_out/s4c
mkdir -p $O
cp pyrmt_amd/librmt.so /tmp/librmt_base.so
for v in base w12h w16; do
  if [ $v != base ]; then cp pyrmt_amd/librmt_$v.so pyrmt_amd/librmt.so; fi
  echo $v
  timeout -k 10 300 python -u tools/chain_time.py 3 > $O/chain_$v.log 2>&1 || { tail -5 $O/chain_$v.log; cp /tmp/librmt_base.so pyrmt_amd/librmt.so; exit 1; }
  grep variant $O/chain_$v.log
done
cp /tmp/librmt_base.so pyrmt_amd/librmt.so
