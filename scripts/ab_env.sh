#!/bin/bash
# A/B bench lines under environment variants (run through gpurun from the repo root):
#   scripts/ab_env.sh OUT "VAR=a VAR2=b" "VAR=c" ...     (an empty string = defaults)
set -o pipefail
O=gpurun_out/${1:?out dir}; shift
mkdir -p "$O"
k=0
for v in "$@"; do
    k=$((k + 1))
    echo "== [$v]"
    env $v timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 20 > "$O/ab_$k.log" 2>&1 \
        || { tail -20 "$O/ab_$k.log"; exit 1; }
    tail -1 "$O/ab_$k.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['ms_per_step'],3), d.get('phase_ms_per_step',{}).get('extrap_sweep_kernel'))"
done
