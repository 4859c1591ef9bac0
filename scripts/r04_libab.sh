#!/bin/bash
# Same-call A/B of two library builds: fused-step hashes, kernel-trace stats of the 20-step
# bench, then interleaved 20-step bench lines.   scripts/r04_libab.sh OUT LIB_A LIB_B [REGEX]
set -o pipefail
O=gpurun_out/${1:?out}; A=${2:?lib a}; B=${3:?lib b}; RX=${4:-k_dct1|k_project_correct|k_transpose}
mkdir -p "$O"; export TMPDIR=/tmp
for L in "$A" "$B"; do
    t=$(basename "$L" .so)
    RMT_LIB=$L timeout -k 10 300 python -u tools/fused_sha.py 4096 3 > "$O/sha_$t.txt" 2>&1 || { tail -5 "$O/sha_$t.txt"; exit 1; }
    tail -1 "$O/sha_$t.txt"
    RMT_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -f csv -d "$O/kt_$t" -o bench -- \
        python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > "$O/kt_$t.log" 2>&1 || { tail -5 "$O/kt_$t.log"; exit 1; }
    f=$(find "$O/kt_$t" -name "*kernel_stats.csv" | head -1); cp "$f" "$O/kt_${t}_stats.csv"
    grep -E "$RX" "$f" | cut -d, -f1-5 || true
done
bash scripts/ab_env.sh "${O#gpurun_out/}" "RMT_LIB=$A" "RMT_LIB=$B" "RMT_LIB=$A" "RMT_LIB=$B"
