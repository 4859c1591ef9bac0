#!/bin/bash
# Round-1 evidence pass: full GPU parity suite, rocprofv3 kernel trace + stats of the N=4096
# bench, PMC HBM-traffic passes (FETCH_SIZE and WRITE_SIZE in separate passes, kernel trace
# only), the 8-byte-access calibration of those counters, then the default bench line
# (with the CPU baseline).  Each GPU step has its own time limit; the chain stops at the
# first failure.
set -o pipefail
R=$PWD
O=$R/gpurun_out/r01
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1200 python -m pytest tests -m gpu -x -q > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest exit $rc" >> $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats -T -f csv -d $O/kt -o bench -- python3 bench.py --n 4096 --steps 5 --warmup 2 --no-cpu-baseline > $O/bench_kt.log 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace -T -f csv -d $O/pmc_fetch -o bench -- python3 bench.py --n 4096 --steps 2 --warmup 1 --no-cpu-baseline > $O/bench_fetch.log 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace -T -f csv -d $O/pmc_write -o bench -- python3 bench.py --n 4096 --steps 2 --warmup 1 --no-cpu-baseline > $O/bench_write.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -T -f csv -d $O/cal_fetch -o cal -- python3 tools/calib_traffic.py > $O/cal_fetch.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -T -f csv -d $O/cal_write -o cal -- python3 tools/calib_traffic.py > $O/cal_write.log 2>&1 || exit $?
timeout -k 10 600 python3 bench.py > $O/bench_default.log 2>&1
echo "done $?"
