"""Config 5 loop body (mac_multi_disc_lid.py, 3 discs, seed 3) on one GPU: ms per step.
    python tools/mac_bench.py [N] [steps]"""
import json
import os
import sys
import time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from pyrmt_amd.mac import MacMultiDisc
from pyrmt_amd import functions as F

N = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
K = int(sys.argv[2]) if len(sys.argv) > 2 else 5
t0 = time.perf_counter()
sim = MacMultiDisc(N, n_discs=3, seed=3)
init = time.perf_counter() - t0
sim.step(1)
torch.cuda.synchronize()
t = time.perf_counter()
sim.step(K)
torch.cuda.synchronize()
ms = (time.perf_counter() - t) / K * 1e3
d = sim.diagnostics()
print(json.dumps({"N": N, "ms_per_step": ms, "init_s": init, "cell_updates_per_s": N * N / ms * 1e3,
                  "ex_path": F.extrapolation_last_path(N, N), "minJ": float(d["minJ"][-1]),
                  "maxJ": float(d["maxJ"][-1]), "cx": d["cx"][-1].tolist()}))
