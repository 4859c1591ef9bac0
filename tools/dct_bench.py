"""DCT-I Poisson solve alone at N x N (for counter / timing runs), checked against scipy's
dctn / idctn (the reference's functions.py:1107-1119 calls).
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
rhs = torch.randn(N, N, dtype=torch.float64, device="cuda", generator=torch.Generator("cuda").manual_seed(1))
for _ in range(2):
    p = P._solve_poisson_dct(rhs, eig)
torch.cuda.synchronize()
t = time.perf_counter()
for _ in range(reps):
    P._solve_poisson_dct(rhs, eig)
torch.cuda.synchronize()
print(f"dct solve N={N}: {(time.perf_counter() - t) / reps * 1e3:.3f} ms")
from scipy.fft import dctn, idctn
r = rhs.cpu().numpy()
e = eig.cpu().numpy() if torch.is_tensor(eig) else np.asarray(eig)
want = idctn(dctn(r, type=1) / e, type=1)
want -= want.mean()
got = p.cpu().numpy()
print(f"max |p - scipy| / max |p| = {np.abs(got - want).max() / np.abs(want).max():.3g}")
