"""sha256 of the fused config-4 fields after K steps (diagnosis: compare two libraries).
    RMT_LIB=... python tools/fused_sha.py [N] [K]"""
import hashlib
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from pyrmt_amd.simulation import soft_disc_in_lid_driven

N = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
K = int(sys.argv[2]) if len(sys.argv) > 2 else 2
sim = soft_disc_in_lid_driven(N)
for k in range(K):
    sim.step(1)
    print(k + 1, {f: hashlib.sha256(np.ascontiguousarray(sim.get(f)).tobytes()).hexdigest()[:12]
                  for f in ("u", "v", "p", "X1", "X2")}, flush=True)
