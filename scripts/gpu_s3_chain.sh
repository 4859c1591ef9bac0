#!/bin/bash
set -o pipefail
O=gpurun_out/s3
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u tools/chain_time.py "$@" > $O/chain_time.log 2>&1
rc=$?; grep variant $O/chain_time.log; tail -3 $O/chain_time.log; exit $rc
