"""Worker for tests/test_distributed.py (GPU): the slab-decomposed step over
torch.distributed, every rank on cuda:0 (gloo) or its own GPU (nccl), against the fused
single-domain step on rank 0.   args: N steps backend [mac]"""
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    N, K, backend = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3]
    dist.init_process_group(backend)
    rank = dist.get_rank()
    torch.cuda.set_device(0 if backend == "gloo" else int(os.environ.get("LOCAL_RANK", 0)))
    from pyrmt_amd import distributed as D
    if len(sys.argv) > 4 and sys.argv[4] == "mac":
        return mac(N, K, rank, D)
    sim = D.soft_disc_in_lid_driven(N, D.TorchComm())
    sim.step(K)
    fields = {f: sim.gather(f) for f in ("u", "v", "X1", "X2")}
    d = sim.diagnostics()
    if rank == 0:
        from pyrmt_amd.simulation import soft_disc_in_lid_driven
        ref = soft_disc_in_lid_driven(N)
        ref.step(K)
        r = ref.diagnostics()
        np.testing.assert_array_equal(d["dt"], r["dt"])
        np.testing.assert_allclose(d["cx"], r["cx"], rtol=1e-12)
        np.testing.assert_allclose(d["cy"], r["cy"], rtol=1e-12)
        for f, v in fields.items():
            np.testing.assert_allclose(v, ref.get(f), rtol=0, atol=1e-10, err_msg=f)
        print("dist_step ok", dist.get_world_size())
    dist.barrier()
    dist.destroy_process_group()


def mac(N, K, rank, D):
    """config 5: MacDistributedSim over TorchComm against MacMultiDisc"""
    sim = D.mac_multi_disc_lid(N, D.TorchComm())
    sim.step(K)
    names = ["u", "v", "p"] + [f"{a}:{k}" for k in range(sim.K) for a in ("X1", "X2", "phi")]
    fields = {f: sim.gather(f) for f in names}
    d = sim.diagnostics()
    if rank == 0:
        from pyrmt_amd.mac import MacMultiDisc
        ref = MacMultiDisc(N)
        ref.step(K)
        r = ref.diagnostics()
        np.testing.assert_array_equal(d["minJ"], r["minJ"])
        np.testing.assert_allclose(d["cx"], r["cx"], rtol=1e-12)
        for f, v in fields.items():
            base, _, k = f.partition(":")
            np.testing.assert_allclose(v, ref.get(base, int(k or 0)), rtol=0, atol=1e-10,
                                       err_msg=f)
        print("dist_step ok", dist.get_world_size())
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
