#!/bin/bash
# kernel stats of a short bench per environment spec: scripts/r06_kt_ab.sh OUT REGEX ENV...
set -o pipefail
O=gpurun_out/${1:?out}; mkdir -p $O; export TMPDIR=/tmp
RX=$2; shift 2
for e in "$@"; do
  tag=$(echo "$e" | tr ',=/.' '____' | tail -c 48)
  envs=$( [ "$e" = "-" ] && echo "" || echo "$e" | tr ',' ' ')
  env $envs timeout -s KILL 300 rocprofv3 --kernel-trace --stats -T -f csv -d $O/kt_$tag -o kt -- python3 bench.py --no-cpu-baseline --steps 20 --warmup 5 > $O/kt_$tag.log 2>&1 || exit 1
  f=$(find $O/kt_$tag -name "*kernel_stats.csv" | head -1); cp "$f" $O/stats_$tag.csv; rm -rf $O/kt_$tag
  echo "== $e"; grep -E "$RX" $O/stats_$tag.csv | cut -d, -f1-7
done
