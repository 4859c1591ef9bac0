import sys, numpy as np
sys.path.insert(0, '.')
from pyrmt_amd.simulation import soft_disc_in_lid_driven
sim = soft_disc_in_lid_driven(4096)
sim.step(3)
phi = sim.get("phi")
N = 4096; dx = 1.0 / (N - 1); thr = 2 * dx
ok = phi > thr
seg = ok.reshape(N, 64, 64).all(axis=2)
# halo columns
left = np.ones((N, 64), bool); right = np.ones((N, 64), bool)
for t in range(64):
    lo = 64 * t - 2; hi = 64 * t + 66
    if lo >= 0: left[:, t] = ok[:, lo] & ok[:, lo + 1]
    if hi <= N: right[:, t] = ok[:, hi - 2] & ok[:, hi - 1]
f = seg & left & right
print("non-fluid segments:", 1 - f.mean(), "phi<=0 frac", (phi <= 0).mean(), "nan", np.isnan(phi).sum())
print("phi sample far:", phi[10, 10], phi[100, 4000], "min/max", np.nanmin(phi), np.nanmax(phi))
