#!/bin/bash
# Checked (bounds-reporting) build of librmt + standalone momentum driver; then the
# momentum tests alone on the normal build.  Each GPU step under its own timeout.
set -o pipefail
mkdir -p gpurun_out/chk
export TMPDIR=/tmp
cd pyrmt_amd/csrc
for f in ops momentum extrap poisson sim; do
  /opt/rocm/bin/hipcc -O1 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -DRMT_CHECKED -c $f.hip -o ../../gpurun_out/chk/$f.o || exit 1
done
cd ../..
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared gpurun_out/chk/*.o -L/opt/rocm/lib -lrocfft -o gpurun_out/chk/librmt_checked.so || exit 1
/opt/rocm/bin/hipcc --offload-arch=gfx950 -std=c++17 -Wno-unused-value -c tools/mom_check.cpp -o gpurun_out/chk/mom_check.o && /opt/rocm/bin/hipcc --offload-arch=gfx950 gpurun_out/chk/mom_check.o -L$PWD/gpurun_out/chk -lrmt_checked -Wl,-rpath,$PWD/gpurun_out/chk -o gpurun_out/chk/mom_check || exit 1
AMD_SERIALIZE_KERNEL=3 timeout -k 10 120 gpurun_out/chk/mom_check 129 > gpurun_out/mom_check.log 2>&1
rc=$?
echo "mom_check exit $rc" >> gpurun_out/mom_check.log
rm -f gpurun_out/chk/*.o
[ $rc -eq 0 ] || exit $rc
grep -q RMT_CHECKED gpurun_out/mom_check.log && exit 3
AMD_SERIALIZE_KERNEL=3 RMT_DEBUG_SYNC=1 timeout -k 10 300 python -m pytest tests -m gpu -q -k "momentum or projection or timestep or weno or error" > gpurun_out/pytest_gpu_d.log 2>&1
echo "pytest exit $?" >> gpurun_out/pytest_gpu_d.log
