"""Hashes of the config-5 fields after a few MAC steps (A/B of library builds via RMT_LIB):
   python tools/mac_sha.py N STEPS"""
import hashlib
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from pyrmt_amd.mac import MacMultiDisc  # noqa: E402


def sha(a):
    return hashlib.sha1(np.ascontiguousarray(a).tobytes()).hexdigest()[:12]


N, K = int(sys.argv[1]), int(sys.argv[2])
sim = MacMultiDisc(N, n_discs=3, seed=3)
sim.step(K)
h = {n: sha(sim.get(n)) for n in ("u", "v", "p")}
h.update({f"X1_{k}": sha(sim.get("X1", k)) for k in range(3)})
print(K, h)
