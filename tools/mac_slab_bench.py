"""Time the config-5 MAC step decomposed into G virtual slabs on one GPU (LocalComm):
per-phase split summed over the slabs.  With G slabs on G GPUs the row-split phases take
about 1/G of these sums each, the extrapolation (replicated) its per-slab share.
    python tools/mac_slab_bench.py [N] [G] [steps]"""
import json
import os
import sys
import time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from pyrmt_amd import distributed as D

N = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
G = int(sys.argv[2]) if len(sys.argv) > 2 else 8
K = int(sys.argv[3]) if len(sys.argv) > 3 else 3
t0 = time.perf_counter()
sim = D.mac_multi_disc_lid(N, D.LocalComm(G))
init = time.perf_counter() - t0
sim.step(1)
sim.set_profiling(True)
torch.cuda.synchronize()
t = time.perf_counter()
sim.step(K)
torch.cuda.synchronize()
ms = (time.perf_counter() - t) / K * 1e3
d = sim.diagnostics()
print(json.dumps({"N": N, "G": G, "ms_per_step": ms, "init_s": init,
                  "phases_ms": {k: v[0] / K for k, v in sim.phase_times().items()},
                  "fitted": int(d["fitted"][-1]), "minJ": float(d["minJ"][-1])}))
