"""DCT-I Poisson solve alone at N x N (for counter / timing runs).
    python tools/dct_bench.py [N] [reps]"""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
import pyrmt_amd as P
N = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
dx = 1.0 / (N - 1)
eig = P._precompute_poisson_eigenvalues(N, N, dx, dx)
rhs = torch.randn(N, N, dtype=torch.float64, device="cuda")
for _ in range(2):
    P._solve_poisson_dct(rhs, eig)
torch.cuda.synchronize()
t = time.perf_counter()
for _ in range(reps):
    P._solve_poisson_dct(rhs, eig)
torch.cuda.synchronize()
print(f"dct solve N={N}: {(time.perf_counter() - t) / reps * 1e3:.3f} ms")
