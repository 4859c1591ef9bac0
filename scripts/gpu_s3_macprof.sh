#!/bin/bash
set -o pipefail
O=gpurun_out/s3
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -T -f csv -d $O/mackt -o mac -- python3 tools/mac_bench.py 8192 3 > $O/mac_kt.log 2>&1
rc=$?; f=$(find $O/mackt -name "*kernel_stats.csv" | head -1); cut -d, -f1-4 "$f" | head -25; exit $rc
