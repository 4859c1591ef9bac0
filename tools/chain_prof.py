"""Per-phase clock breakdown of k_ex_chain on the bench-size disc (RMT_EX_PROFILE=1).
    RMT_EX_PROFILE=1 python tools/chain_prof.py [case]"""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import pyrmt_amd as P
from test_gpu_parity import _extrap_case
name = sys.argv[1] if len(sys.argv) > 1 else "disc4096"
X1, X2, phi, dx, dy, layers = _extrap_case(name)
for _ in range(3):
    P.extrapolate_reference_map(X1, X2, phi, dx, dy, layers)
print("path", P.extrapolation_last_path(*phi.shape))
