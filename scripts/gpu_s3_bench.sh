#!/bin/bash
set -o pipefail
O=gpurun_out/s3
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/bench_n4096.log 2>&1 || exit $?
tail -1 $O/bench_n4096.log
timeout -k 10 200 python -u tools/dist_local_bench.py 4096 1 5 > $O/local_g1.log 2>&1 || exit $?
tail -1 $O/local_g1.log
timeout -k 10 200 python -u tools/dist_local_bench.py 4096 4 3 > $O/local_g4.log 2>&1 || exit $?
tail -1 $O/local_g4.log
RMT_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 --grid 1024 > $O/bench_gloo2.log 2>&1 || exit $?
tail -1 $O/bench_gloo2.log
