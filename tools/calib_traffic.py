"""PMC calibration for FETCH_SIZE / WRITE_SIZE with librmt's own access width (8-B fp64 per
lane): rmt_smoothed_heaviside reads one N^2 fp64 plane and writes one, exactly once.
Run under `rocprofv3 --pmc FETCH_SIZE --kernel-trace` (and WRITE_SIZE in its own pass);
expected per dispatch: 8*N^2 bytes read, 8*N^2 bytes written (N = 4096: 134.2 MB)."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import pyrmt_amd as P

N = 4096
phi = torch.linspace(-1, 1, N * N, device="cuda", dtype=torch.float64).reshape(N, N)
for _ in range(5):
    H = P.smoothed_heaviside(phi, 2.0 / (N - 1))
torch.cuda.synchronize()
print("calibration dispatches done; bytes per plane", 8 * N * N)
