#!/bin/bash
set -o pipefail
O=gpurun_out/s4c
mkdir -p $O
RMT_EX_PROFILE=1 timeout -k 10 300 python -u tools/chain_time.py 3 > $O/chainprof.log 2>&1 || { tail -20 $O/chainprof.log; exit 1; }
grep -E "chain-prof|variant" $O/chainprof.log | tail -4
