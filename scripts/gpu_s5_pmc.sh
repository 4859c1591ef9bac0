#!/bin/bash
# session 5: GPU suite, default bench line, kernel stats, then FETCH_SIZE / WRITE_SIZE passes
# (one counter group per run) of a short bench for the per-launch HBM traffic
set -o pipefail
O=gpurun_out/${1:-s5i}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 500 python -u bench.py > $O/bench_default.log 2>&1 || exit $?
tail -1 $O/bench_default.log | cut -c1-250
timeout -k 10 400 rocprofv3 --kernel-trace --stats -T -f csv -d $O/kt -o bench -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > $O/bench_kt.log 2>&1 || exit $?
f=$(find $O/kt -name "*kernel_stats.csv" | head -1); cp "$f" $O/kernel_stats_n4096.csv; cut -d, -f1-4 "$f" | head -8
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -T -f csv -d $O/pf -o fetch -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > $O/pmc_fetch.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -T -f csv -d $O/pw -o write -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > $O/pmc_write.log 2>&1 || exit $?
ls -R $O/pf $O/pw | head -20
