"""Worker for tests/test_distributed.py (CPU, gloo): every TorchComm collective against
LocalComm run over all G ranks' data in this process.  Launched with
python -m torch.distributed.run --nproc-per-node G ... tests/workers/dist_comm.py"""
import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from pyrmt_amd.distributed import LocalComm, TorchComm, even_splits   # noqa: E402

HALO, N, NX = 12, 70, 9


class FakeSlab:
    """The fields of one slab as CPU tensors (what Slab.view returns on the GPU)."""

    def __init__(self, rank, G, splits, seed):
        self.rank, self.G, self.splits = rank, G, splits
        self.r0, self.r1 = splits[rank], splits[rank + 1]
        self.lo, self.hi = max(0, self.r0 - HALO), min(N, self.r1 + HALO)
        g = torch.Generator().manual_seed(seed * 100 + rank)
        nl = self.hi - self.lo
        self.v = {
            "u": torch.randn(nl, NX, generator=g, dtype=torch.float64),
            "pc": torch.randn(nl, NX, generator=g, dtype=torch.float64),
            "bits": torch.randint(0, 1 << 40, (N, 3), generator=g),
            "scal": torch.randn(16, generator=g, dtype=torch.float64),
            "rim": torch.randn(50, 3, generator=g, dtype=torch.float64),
            "A": torch.randn(200, generator=g, dtype=torch.float64),
            "B": torch.zeros(200, dtype=torch.float64),
            # a MAC v-face plane: rows lo .. hi, owned rows [r0, r1 + 1)
            "vf": torch.randn(nl + 1, NX, generator=g, dtype=torch.float64),
        }
        gv = torch.Generator().manual_seed(seed)
        self.truth = torch.randn(N + 1, NX, generator=gv, dtype=torch.float64)
        self.v["vf"][self.r0 - self.lo:self.r1 + 1 - self.lo] = self.truth[self.r0:self.r1 + 1]

    def view(self, name):
        return self.v[name]

    def top_extra(self, name):
        return 1 if name == "vf" else 0


def main():
    dist.init_process_group("gloo")
    G, rank = dist.get_world_size(), dist.get_rank()
    splits = even_splits(N, G, HALO)
    mine = FakeSlab(rank, G, splits, 1)
    allr = [FakeSlab(k, G, splits, 1) for k in range(G)]
    tc, lc = TorchComm(), LocalComm(G)
    # halo exchange
    tc.halo([mine], ("u",), HALO)
    lc.halo(allr, ("u",), HALO)
    assert torch.equal(mine.view("u"), allr[rank].view("u")), "halo"
    tc.halo([mine], ("pc",), 2)
    lc.halo(allr, ("pc",), 2)
    assert torch.equal(mine.view("pc"), allr[rank].view("pc")), "halo 2 rows"
    # face plane with one extra top row: every resident row equals the global plane
    tc.halo([mine], ("vf",), HALO)
    lc.halo(allr, ("vf",), HALO)
    assert torch.equal(mine.view("vf"), allr[rank].view("vf")), "halo faces"
    assert torch.equal(mine.view("vf"), mine.truth[mine.lo:mine.hi + 1]), "halo faces truth"
    # known-bit rows
    tc.allgather_rows([mine], "bits")
    lc.allgather_rows(allr, "bits")
    assert torch.equal(mine.view("bits"), allr[rank].view("bits")), "allgather_rows"
    # scalars
    (a,) = tc.allgather([mine.view("scal")])
    b = lc.allgather([s.view("scal") for s in allr])[rank]
    assert torch.equal(a, b), "allgather"
    # padded rim entries
    counts = [7 + 5 * k for k in range(G)]
    (a,), cap = tc.allgather_padded([mine.view("rim")], counts, 3)
    bl, cap2 = lc.allgather_padded([s.view("rim") for s in allr], counts, 3)
    assert cap == cap2
    for k in range(G):
        n = counts[k] * 3
        assert torch.equal(a[k, :n], bl[rank][k, :n]), "allgather_padded"
    # uneven all_to_all (split sizes as the DCT transposes make them)
    snd = [[3 + k + m for m in range(G)] for k in range(G)]
    rcv = [[snd[k][m] for k in range(G)] for m in range(G)]
    tc.all_to_all([mine.view("A")], [mine.view("B")], [snd[rank]], [rcv[rank]])
    lc.all_to_all([s.view("A") for s in allr], [s.view("B") for s in allr], snd, rcv)
    n = sum(rcv[rank])
    assert torch.equal(mine.view("B")[:n], allr[rank].view("B")[:n]), "all_to_all"
    dist.barrier()
    if rank == 0:
        print("dist_comm ok", G)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
