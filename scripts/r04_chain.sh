#!/bin/bash
# round 4: a chain variant's parity (extrapolation + config tests), A/B bench lines against
# the default, and per-fit traces of both (tools/chain_trace.py)
#   scripts/r04_chain.sh OUT VARIANT
set -o pipefail
O=gpurun_out/${1:?out}; V=${2:?variant}
mkdir -p "$O"
RMT_CH_VARIANT=$V timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
    tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -k "extrap or config4 or config2" > "$O/tests_v$V.log" 2>&1 \
    || { tail -30 "$O/tests_v$V.log"; exit 1; }
tail -2 "$O/tests_v$V.log"
bash scripts/ab_env.sh "${1}" "" "RMT_CH_VARIANT=$V" || exit 1
bash scripts/chain_ab.sh "${1}" 3 $V || exit 1
for v in 3 $V; do python3 tools/chain_trace.py $O/trace_v$v.bin > $O/trace_v$v.txt && head -5 $O/trace_v$v.txt; done
