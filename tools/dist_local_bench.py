"""Time the slab-decomposed step with G virtual slabs on one GPU (LocalComm) next to the
fused step: the orchestration overhead and the per-phase split.
    python tools/dist_local_bench.py [N] [G] [steps]"""
import json
import os
import sys
import time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from pyrmt_amd import distributed as D

N = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
G = int(sys.argv[2]) if len(sys.argv) > 2 else 1
K = int(sys.argv[3]) if len(sys.argv) > 3 else 5
sim = D.soft_disc_in_lid_driven(N, D.LocalComm(G))
sim.step(2)
torch.cuda.synchronize()
t = time.perf_counter()
sim.step(K)
torch.cuda.synchronize()
ms_plain = (time.perf_counter() - t) / K * 1e3
sim.set_profiling(True)
torch.cuda.synchronize()
t = time.perf_counter()
sim.step(K)
torch.cuda.synchronize()
ms = (time.perf_counter() - t) / K * 1e3
print(json.dumps({"N": N, "G": G, "ms_per_step": ms_plain, "ms_per_step_profiled": ms,
                  "phases": {k: v[0] / K for k, v in sim.phase_times().items()}}))
