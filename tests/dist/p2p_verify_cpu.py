"""torchrun worker (CPU, gloo): the CPU FakeComm twin of the fused-exchange verification
(mlapi_amd/parallel/p2p.py): the same rank-tagged synthetic gradient through the communicator's
all-reduce must equal the exact sum bit for bit; a corrupted all-reduce must be caught; the replica
hash check and the rank-0 re-sync work on CPU tensors. Writes OK_<rank> under $OUT."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
from mlapi_amd.parallel.comm import all_reduce_sum_, broadcast_, init_distributed, shutdown  # noqa: E402
from mlapi_amd.parallel.p2p import check_allreduce, replicas_agree  # noqa: E402

info = init_distributed(use_gpu=False)
r, w = info.rank, info.world


def via_comm(local):
    t = torch.from_numpy(np.ascontiguousarray(local)).clone()
    all_reduce_sum_(t, info)
    return t.numpy()


def corrupted(local):
    out = via_comm(local)
    if r == 1:
        out[5] += 1.0  # one wrong word on one rank
    return out


for width in (4, 260, 4096):
    assert check_allreduce(via_comm, r, w, width) == 0, width
assert check_allreduce(corrupted, r, w, 260) == (3 if r == 1 else 0)
p = torch.arange(12, dtype=torch.float32) * 0.5
assert replicas_agree(p, info)
q = p.clone()
if r == 1:
    q[3] += 1e-6
assert not replicas_agree(q, info)
broadcast_(q, info, 0)
assert replicas_agree(q, info) and torch.equal(q, p)
open(os.path.join(os.environ["OUT"], f"OK_{r}"), "w").write("ok")
shutdown(info)
