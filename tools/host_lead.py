"""Host enqueue time vs device time of rmt_sim_step : is the host ahead of the GPU?
   python tools/host_lead.py [steps] [N]"""
import sys, time
import torch
sys.path.insert(0, ".")
from pyrmt_amd.simulation import soft_disc_in_lid_driven

K = int(sys.argv[1]) if len(sys.argv) > 1 else 20
N = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
s = soft_disc_in_lid_driven(N)
s.step(5)
torch.cuda.synchronize()
for rep in range(3):
    t0 = time.perf_counter()
    s.step(K)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"steps {K}: host returns after {1e3 * (t1 - t0):.2f} ms, device done after "
          f"{1e3 * (t2 - t0):.2f} ms ({1e3 * (t2 - t0) / K:.4f} ms/step)", flush=True)
