#!/bin/bash
# round-3 GPU steps: scripts/r03_run.sh OUT STEP [STEP ...]; each step under its own limit,
# the first failure ends the call.
#   suite          pytest -m gpu without the parallel-extrapolation tests
#   par            tests/test_gpu_extrap_par.py
#   t:EXPR         pytest -m gpu -k EXPR
#   bench          20-step bench line (no CPU baseline)
#   bench100       three 100-step bench lines (ms/step each)
#   smoke          __graft_entry__.smoke()
#   benchfull      the default bench line (the driver's command: CPU baselines included)
#   benchpar       the same with RMT_EXTRAP_PARALLEL=1
#   kt / ktpar     rocprofv3 kernel trace + stats of the 20-step bench (exact / parallel)
#   env:K=V        export K=V for the following steps
#   out:SUB        write the following steps' logs under OUT/SUB
set -o pipefail
BASE=gpurun_out/${1:?out}; O=$BASE; shift; mkdir -p "$O"; export TMPDIR=/tmp
PYT="python -u -m pytest -v --timeout 240 --timeout-method thread"
for s in "$@"; do
    echo "== $s $(date +%T)"
    case "$s" in
        suite) timeout -k 10 900 $PYT tests -m gpu --ignore=tests/test_gpu_extrap_par.py -x > "$O/suite.log" 2>&1 \
                   || { grep -E "FAIL|Error|error" "$O/suite.log" | head -20; tail -30 "$O/suite.log"; exit 1; }
               tail -2 "$O/suite.log" ;;
        par) timeout -k 10 900 $PYT -s tests/test_gpu_extrap_par.py > "$O/par.log" 2>&1 \
                   || { grep -E "^\[|FAIL|Error" "$O/par.log" | head -30; tail -30 "$O/par.log"; exit 1; }
             grep -E "^\[|passed|failed" "$O/par.log" | tail -20 ;;
        t:*) timeout -k 10 900 $PYT -s tests -m gpu -k "${s#t:}" > "$O/t.log" 2>&1 \
                   || { tail -40 "$O/t.log"; exit 1; }
             grep -E "^\[|passed|failed" "$O/t.log" | tail -20 ;;
        bench) timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > "$O/bench.log" 2>&1 \
                   || { tail -20 "$O/bench.log"; exit 1; }
               tail -1 "$O/bench.log" | cut -c1-400 ;;
        smoke) timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 \
                   || { tail -20 "$O/smoke.log"; exit 1; }
               tail -1 "$O/smoke.log" ;;
        benchfull) timeout -k 10 900 python -u bench.py > "$O/benchfull.log" 2>&1 \
                   || { tail -20 "$O/benchfull.log"; exit 1; }
               tail -1 "$O/benchfull.log" | cut -c1-300 ;;
        bench100) for k in 1 2 3; do
                      timeout -k 10 300 python -u bench.py --steps 100 --warmup 10 --no-cpu-baseline > "$O/bench100_$k.log" 2>&1 \
                          || { tail -20 "$O/bench100_$k.log"; exit 1; }
                      tail -1 "$O/bench100_$k.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('bench100', round(d['ms_per_step'], 4))"
                  done ;;
        benchpar) RMT_EXTRAP_PARALLEL=1 timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > "$O/benchpar.log" 2>&1 \
                   || { tail -20 "$O/benchpar.log"; exit 1; }
               tail -1 "$O/benchpar.log" | cut -c1-400 ;;
        kt|ktpar) [ "$s" = ktpar ] && export RMT_EXTRAP_PARALLEL=1
            timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -f csv -d "$O/$s" -o bench -- \
                python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > "$O/$s.log" 2>&1 || exit 1
            unset RMT_EXTRAP_PARALLEL
            f=$(find "$O/$s" -name "*kernel_stats.csv" | head -1); cp "$f" "$O/${s}_stats.csv"
            cut -d, -f1-4 "$f" | head -16 ;;
        pmc|pmcpar)   # counter passes (one group each) over a short bench, stage / SL / DCT / px kernels
            [ "$s" = pmcpar ] && export RMT_EXTRAP_PARALLEL=1
            RX="k_mom_stage|k_mom_rows|k_sim_sl|k_dct1|k_px_|k_divergence_rc|k_project_correct|k_mom_prep|k_transpose"
            timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
                SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_INST_LDS SQ_BUSY_CYCLES --kernel-include-regex "$RX" \
                --kernel-trace -T -f csv -d "$O/${s}_sq" -o sq -- python3 bench.py --steps 2 --warmup 1 \
                --no-cpu-baseline > "$O/${s}_sq.log" 2>&1 || exit 1
            timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$RX" --kernel-trace -T -f csv \
                -d "$O/${s}_fetch" -o fetch -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline \
                > "$O/${s}_fetch.log" 2>&1 || exit 1
            timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU_FMA_F64 \
                --kernel-include-regex "$RX" --kernel-trace -T -f csv \
                -d "$O/${s}_write" -o write -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline \
                > "$O/${s}_write.log" 2>&1 || exit 1
            unset RMT_EXTRAP_PARALLEL
            echo "pmc passes done" ;;
        pmcchain)   # issue counters of the chain kernel (two passes)
            timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS \
                SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS \
                --kernel-include-regex "k_ex_chain" --kernel-trace -T -f csv -d "$O/pmcchain1" -o c1 -- \
                python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > "$O/pmcchain1.log" 2>&1 || exit 1
            timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_ANY \
                SQ_ACTIVE_INST_ANY SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA SQ_LDS_BANK_CONFLICT \
                --kernel-include-regex "k_ex_chain" --kernel-trace -T -f csv -d "$O/pmcchain2" -o c2 -- \
                python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > "$O/pmcchain2.log" 2>&1 || exit 1
            for f in $(find "$O/pmcchain1" "$O/pmcchain2" -name "*counter_collection.csv"); do cp "$f" "$O/$(basename $(dirname $f))_$(basename $f)"; done
            echo "pmcchain done" ;;
        trace)   # per-fit chain trace (the profiled build at 12 waves: at 16 its counters spill)
            RMT_LIB=pyrmt_amd/librmt_w12.so RMT_EX_PROFILE=1 RMT_EX_TRACE=$O/trace.bin timeout -k 10 200 \
                python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline > "$O/trace.log" 2>&1 || { tail -5 "$O/trace.log"; exit 1; }
            grep chain-prof "$O/trace.log" | tail -1
            python3 tools/chain_trace.py "$O/trace.bin" > "$O/trace.txt" && head -5 "$O/trace.txt" ;;
        trace16)   # the same trace with the default 16-wave build (its profiled kernel fits
                   # 128 VGPRs since round 4)
            RMT_EX_PROFILE=1 RMT_EX_TRACE=$O/trace16.bin timeout -k 10 200 \
                python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline > "$O/trace16.log" 2>&1 || { tail -5 "$O/trace16.log"; exit 1; }
            grep chain-prof "$O/trace16.log" | tail -1
            python3 tools/chain_trace.py "$O/trace16.bin" > "$O/trace16.txt" && head -5 "$O/trace16.txt" ;;
        cfg:*)   # one BASELINE config's bench line (CPU baseline included) and its kernel stats
            c=${s#cfg:}
            timeout -k 10 600 python -u bench.py --config $c --steps 10 --warmup 2 > "$O/cfg$c.log" 2>&1 \
                || { tail -20 "$O/cfg$c.log"; exit 1; }
            tail -1 "$O/cfg$c.log" | cut -c1-500
            timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -f csv -d "$O/kt_cfg$c" -o bench -- \
                python3 bench.py --config $c --steps 10 --warmup 2 --no-cpu-baseline > "$O/kt_cfg$c.log" 2>&1 || exit 1
            f=$(find "$O/kt_cfg$c" -name "*kernel_stats.csv" | head -1); cp "$f" "$O/kt_cfg${c}_stats.csv"
            cut -d, -f1-4 "$f" | head -12 ;;
        local)   # LocalComm phase times of the slab step, G = 1, 2, 4, 8, exact and parallel mode
            for m in 0 1; do for g in 1 2 4 8; do
                RMT_EXTRAP_PARALLEL=$m timeout -k 10 300 python -u tools/dist_local_bench.py 4096 $g 5 \
                    > "$O/local_m${m}_G$g.json" 2> "$O/local_m${m}_G$g.err" || { tail -5 "$O/local_m${m}_G$g.err"; exit 1; }
                cut -c1-160 "$O/local_m${m}_G$g.json"
            done; done ;;
        out:*) O=$BASE/${s#out:}; mkdir -p "$O" ;;
        env:*) export "${s#env:}"; echo "exported ${s#env:}" ;;
        *) echo "unknown step $s"; exit 2 ;;
    esac
done
