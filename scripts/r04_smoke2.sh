#!/bin/bash
mkdir -p gpurun_out/s1
for L in "" "RMT_LIB=pyrmt_amd/librmt_w12.so"; do
  echo "== [$L]"
  env $L timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s1/smoke.log 2>&1; echo rc=$?; tail -3 gpurun_out/s1/smoke.log | cut -c1-200
done
