#!/bin/bash
set -o pipefail
O=gpurun_out/s3
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 python -u tools/mac_bench.py 1024 5 > $O/mac_1024.log 2>&1 || exit $?
tail -1 $O/mac_1024.log
timeout -k 10 400 python -u tools/mac_bench.py 8192 3 > $O/mac_8192.log 2>&1
rc=$?; tail -3 $O/mac_8192.log; exit $rc
