#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -q -k "not ghia and not soft_disc and not taylor and not lid_cavity" > gpurun_out/pytest_gpu_b.log 2>&1
echo "pytest exit $?" >> gpurun_out/pytest_gpu_b.log
timeout -k 10 300 python -X faulthandler -c "
import sys; sys.path.insert(0,'.')
import numpy as np, torch, pyrmt_amd as R
print('dct test', flush=True)
N=65; X,Y,dx,dy = R.create_grid(N,N,1.0,1.0)
eig = R._precompute_poisson_eigenvalues(N,N,dx,dy)
p = R._solve_poisson_dct(np.cos(np.pi*X)*np.cos(np.pi*Y), eig); print('dct ok', float(np.abs(p).max()), flush=True)
from pyrmt_amd.simulation import soft_disc_in_lid_driven
print('create sim', flush=True)
sim = soft_disc_in_lid_driven(65); print('created', flush=True)
sim.step(1); print('stepped', flush=True)
print(sim.diagnostics(), flush=True)
" > gpurun_out/debug_b.log 2>&1
echo "debug exit $?" >> gpurun_out/debug_b.log
