"""torchrun worker: the framework communicator's collectives (FakeComm on CPU, NativeComm on GPU).

Writes OK_<rank> under $OUT when every check passed."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
from mlapi_amd.models.linear import LinearModel  # noqa: E402
from mlapi_amd.parallel.comm import (all_gather_floats, all_reduce_max, all_reduce_sum_, barrier,  # noqa: E402
                                     broadcast_model, init_distributed, shutdown)
from mlapi_amd.parallel.rccl import default_store, exchange_unique_id  # noqa: E402

info = init_distributed()
c = info.comm
assert c is not None, "MLAPI_COMM must select a framework communicator"
dev = c.device
r, w = info.rank, info.world

t = torch.full((1000,), float(r + 1), device=dev)
c.all_reduce_(t)
assert torch.all(t == w * (w + 1) / 2)
m = torch.tensor([float(r)], device=dev)
c.all_reduce_(m, "max")
assert m.item() == w - 1
b = torch.full((17,), float(r), dtype=torch.float64, device=dev)
c.broadcast_(b, src=w - 1)
assert torch.all(b == w - 1)
g = c.all_gather(torch.tensor([r, 10 * r], dtype=torch.int32, device=dev))
assert g.cpu().tolist() == [[i, 10 * i] for i in range(w)]
rs = c.reduce_scatter(torch.arange(4 * w, dtype=torch.float32, device=dev))
assert rs.cpu().tolist() == [float(w * (4 * r + j)) for j in range(4)]
bf = torch.full((64,), 0.5, dtype=torch.bfloat16, device=dev)
c.all_reduce_(bf)
assert torch.all(bf.float() == 0.5 * w)
c.barrier()
# module-level helpers route through the communicator
assert all_reduce_max(float(r), info) == w - 1
assert all_gather_floats([r, 2.0], info).tolist() == [[i, 2.0] for i in range(w)]
s = torch.ones(5, device=dev)
all_reduce_sum_(s, info)
assert torch.all(s == w)
mdl = LinearModel.random(8, 3, seed=1, labels=["x", "y", "z"]) if r == 0 else None
mdl = broadcast_model(mdl, info)
assert list(mdl.classes) == ["x", "y", "z"] and mdl.W.shape == (3, 8)
barrier(info)
if w > 1:  # host-channel bootstrap used by NativeComm
    uid = exchange_unique_id(default_store(), r, lambda: bytes(range(128)), generation=99)
    assert uid == bytes(range(128))
open(os.path.join(os.environ["OUT"], f"OK_{r}"), "w").write(c.kind)
shutdown(info)
