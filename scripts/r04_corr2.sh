# Round-4 A/B of the two-cell correction kernel (RMT_CORRECT2; measured no faster and
# reverted -- kept as the record of profiles/r04/correct2/, not runnable at HEAD)
set -o pipefail
O=gpurun_out/r04/corr2; mkdir -p $O; export TMPDIR=/tmp
RMT_CORRECT2=0 timeout -k 10 300 python -u tools/fused_sha.py 4096 3 > $O/sha_one.txt 2>&1 || { tail -5 $O/sha_one.txt; exit 1; }
timeout -k 10 300 python -u tools/fused_sha.py 4096 3 > $O/sha_two.txt 2>&1 || { tail -5 $O/sha_two.txt; exit 1; }
tail -1 $O/sha_one.txt; tail -1 $O/sha_two.txt
for v in 0 1; do
RMT_CORRECT2=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -f csv -d $O/kt$v -o bench -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/kt$v.log 2>&1 || { tail -5 $O/kt$v.log; exit 1; }
f=$(find $O/kt$v -name "*kernel_stats.csv" | head -1); grep -E "k_project_correct" $f | cut -d, -f1-5 || true
done
bash scripts/ab_env.sh r04/corr2 "RMT_CORRECT2=0" "RMT_CORRECT2=1" "RMT_CORRECT2=0" "RMT_CORRECT2=1"
