#!/bin/bash
# One parameterised GPU-box script (run through gpurun from the repo root):
#   scripts/gpu.sh OUT STEP [STEP ...]
# Steps run in order, each under its own time limit; the first failure ends the call.
#   tests          full `pytest -m gpu` suite
#   tests:EXPR     only tests matching the -k expression EXPR
#   configs        tests/test_gpu_configs.py with -s (prints the achieved parity bars)
#   bench          default bench line (N=4096, with the CPU baselines)
#   benchq         bench line without the CPU baselines
#   kt             rocprofv3 --kernel-trace --stats of a short bench (kernel_stats.csv)
#   pmc            FETCH_SIZE and WRITE_SIZE passes of a short bench (one counter group each)
#   chainprof      per-phase clocks of the extrapolation chain (RMT_EX_PROFILE=1)
#   mac            tools/mac_bench.py at N=8192
#   py:SCRIPT      python -u SCRIPT (a tools/ probe)
set -o pipefail
O=gpurun_out/${1:?out dir}
shift
mkdir -p "$O"
export TMPDIR=/tmp
PYT="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
for s in "$@"; do
    echo "== $s $(date +%T)"
    case "$s" in
        tests) timeout -k 10 1000 $PYT tests -m gpu > "$O/tests.log" 2>&1 \
                   || { tail -40 "$O/tests.log"; exit 1; }
               tail -2 "$O/tests.log" ;;
        tests:*) timeout -k 10 600 $PYT tests -m gpu -k "${s#tests:}" -s > "$O/tests_k.log" 2>&1 \
                   || { tail -40 "$O/tests_k.log"; exit 1; }
               grep -E "^\[|passed|failed" "$O/tests_k.log" | tail -20 ;;
        configs) timeout -k 10 900 $PYT tests/test_gpu_configs.py -s > "$O/configs.log" 2>&1 \
                   || { tail -40 "$O/configs.log"; exit 1; }
               grep -E "^\[|energy|passed|failed" "$O/configs.log" ;;
        bench) timeout -k 10 600 python -u bench.py > "$O/bench.log" 2>&1 || { tail -20 "$O/bench.log"; exit 1; }
               tail -1 "$O/bench.log" | cut -c1-400 ;;
        benchq) timeout -k 10 300 python -u bench.py --no-cpu-baseline > "$O/benchq.log" 2>&1 \
                   || { tail -20 "$O/benchq.log"; exit 1; }
               tail -1 "$O/benchq.log" | cut -c1-400 ;;
        kt) timeout -k 10 400 rocprofv3 --kernel-trace --stats -T -f csv -d "$O/kt" -o bench -- \
                python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > "$O/kt.log" 2>&1 || exit 1
            f=$(find "$O/kt" -name "*kernel_stats.csv" | head -1); cp "$f" "$O/kernel_stats.csv"
            cut -d, -f1-4 "$f" | head -16 ;;
        pmc) timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -T -f csv -d "$O/pf" -o fetch -- \
                 python3 bench.py --steps 6 --warmup 1 --no-cpu-baseline > "$O/pmc_fetch.log" 2>&1 || exit 1
             timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -T -f csv -d "$O/pw" -o write -- \
                 python3 bench.py --steps 6 --warmup 1 --no-cpu-baseline > "$O/pmc_write.log" 2>&1 || exit 1
             echo "pmc done" ;;
        chainprof) RMT_EX_PROFILE=1 timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 \
                       --no-cpu-baseline > "$O/chainprof.log" 2>&1 || { tail -20 "$O/chainprof.log"; exit 1; }
                   grep -E "chain-prof" "$O/chainprof.log" | tail -4 ;;
        mac) timeout -k 10 300 python -u tools/mac_bench.py 8192 5 > "$O/mac.log" 2>&1 || exit 1
             tail -1 "$O/mac.log" | cut -c1-300 ;;
        py:*) timeout -k 10 600 python -u ${s#py:} > "$O/$(basename ${s#py:} .py).log" 2>&1 \
                  || { tail -30 "$O/$(basename ${s#py:} .py).log"; exit 1; }
              tail -15 "$O/$(basename ${s#py:} .py).log" ;;
        *) echo "unknown step $s"; exit 2 ;;
    esac
done
