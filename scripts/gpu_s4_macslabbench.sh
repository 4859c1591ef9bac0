#!/bin/bash
# MAC slab step at N=8192: G=1 and G=8 virtual slabs (per-phase split), kernel stats at G=8
set -o pipefail
mkdir -p gpurun_out/s4
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 240 python -u tools/mac_slab_bench.py 8192 1 3 > gpurun_out/s4/macslab_g1.json 2> gpurun_out/s4/macslab_g1.err &&
timeout -k 10 300 python -u tools/mac_slab_bench.py 8192 8 3 > gpurun_out/s4/macslab_g8.json 2> gpurun_out/s4/macslab_g8.err &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/s4/prof_g8 -o run -- python3 tools/mac_slab_bench.py 8192 8 3 > gpurun_out/s4/prof_g8.log 2>&1
rc=$?
cat gpurun_out/s4/macslab_g1.json gpurun_out/s4/macslab_g8.json
exit $rc
