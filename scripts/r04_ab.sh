#!/bin/bash
# A/B bench lines (20 steps, no CPU baseline) for environment variants; then, optionally,
# a per-fit trace of one variant.   scripts/r04_ab.sh OUT "ENV..." ["ENV..." ...]
set -o pipefail
O=gpurun_out/${1:?out}; shift
bash scripts/ab_env.sh "${O#gpurun_out/}" "$@" || exit 1
if [ -n "$TRACE_ENV" ]; then
  env $TRACE_ENV RMT_EX_PROFILE=1 RMT_EX_TRACE=$O/trace.bin timeout -k 10 200 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline > $O/trace.log 2>&1 || { tail -5 $O/trace.log; exit 1; }
  grep chain-prof $O/trace.log | tail -1
  python3 tools/chain_trace.py $O/trace.bin 4096 ${TRACE_PARTS:-2} > $O/trace.txt && head -5 $O/trace.txt
fi
