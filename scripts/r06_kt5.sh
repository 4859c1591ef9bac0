#!/bin/bash
# config-5 kernel stats per environment spec: scripts/r06_kt5.sh OUT REGEX ENV...
set -o pipefail
O=gpurun_out/${1:?out}; mkdir -p $O; export TMPDIR=/tmp
RX=$2; shift 2
for e in "$@"; do
  tag=$(echo "$e" | tr ',=/.' '____' | tail -c 48)
  envs=$( [ "$e" = "-" ] && echo "" || echo "$e" | tr ',' ' ')
  env $envs timeout -s KILL 300 rocprofv3 --kernel-trace --stats -T -f csv -d $O/kt_$tag -o kt -- python3 bench.py --config 5 --no-cpu-baseline --steps 4 --warmup 1 > $O/kt_$tag.log 2>&1 || exit 1
  f=$(find $O/kt_$tag -name "*kernel_stats.csv" | head -1); cp "$f" $O/stats_$tag.csv; rm -rf $O/kt_$tag
  echo "== $e $(tail -1 $O/kt_$tag.log | python3 -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])')"; grep -E "$RX" $O/stats_$tag.csv | cut -d, -f1-4
done
