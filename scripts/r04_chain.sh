#!/bin/bash
# round 4: a chain variant's parity (extrapolation + config tests), A/B bench lines against
# the default, and per-fit traces (tools/chain_trace.py); W16=1 adds the CH_W=16 build
#   scripts/r04_chain.sh OUT VARIANT
set -o pipefail
O=gpurun_out/${1:?out}; V=${2:?variant}
mkdir -p "$O"
RMT_CH_VARIANT=$V timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
    tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -k "extrap or config4_fused or config2" > "$O/tests_v$V.log" 2>&1 \
    || { tail -30 "$O/tests_v$V.log"; exit 1; }
tail -2 "$O/tests_v$V.log"
W=pyrmt_amd/librmt_w16.so
if [ -n "$W16" ]; then
  RMT_LIB=$W RMT_CH_VARIANT=$V timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
      tests/test_gpu_parity.py -m gpu -k "extrap" > "$O/tests_w16_v$V.log" 2>&1 \
      || { tail -30 "$O/tests_w16_v$V.log"; exit 1; }
  tail -1 "$O/tests_w16_v$V.log"
fi
bash scripts/ab_env.sh "${1}" "" "RMT_CH_VARIANT=$V" ${W16:+"RMT_LIB=$W RMT_CH_VARIANT=$V"} || exit 1
bash scripts/chain_ab.sh "${1}" $V || exit 1
python3 tools/chain_trace.py $O/trace_v$V.bin > $O/trace_v$V.txt && head -5 $O/trace_v$V.txt
if [ -n "$W16" ]; then
  RMT_LIB=$W RMT_CH_VARIANT=$V RMT_EX_PROFILE=1 RMT_EX_TRACE=$O/trace_w16.bin timeout -k 10 200 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline > $O/w16.log 2>&1 || { tail -5 $O/w16.log; exit 1; }
  grep chain-prof $O/w16.log | tail -1
  python3 tools/chain_trace.py $O/trace_w16.bin > $O/trace_w16.txt && head -5 $O/trace_w16.txt
fi
