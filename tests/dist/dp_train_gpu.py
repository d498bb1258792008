"""torchrun worker (GPU): data-parallel SGD whose gradient all-reduce runs on the GPU through the
one-shot P2P kernel (MLAPI_COMM=p2p), binary and multiclass, plus the C1 model broadcast.
Writes <name>_<world>_<rank>.npy and bcast_<world>_<rank>.json under $OUT."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
from mlapi_amd.models.linear import LinearModel  # noqa: E402
from mlapi_amd.parallel.comm import broadcast_model, init_distributed, shutdown  # noqa: E402
from mlapi_amd.train.sgd import BinarySGDTrainer, synthetic_binary  # noqa: E402
from mlapi_amd.train.softmax_sgd import SoftmaxSGDTrainer, synthetic_multiclass  # noqa: E402

info = init_distributed(use_gpu=True, comm="p2p")
assert info.backend == "p2p+gloo"
dev, out, r, w = info.device, os.environ["OUT"], info.rank, info.world
m = LinearModel.random(6, 5, seed=7, labels=["a", "b", "c", "d", "e"]) if r == 0 else None
m = broadcast_model(m, info)
B = 2048
per = B // w
X, y = synthetic_binary(8192, 256, seed=5, dtype=torch.bfloat16)
X, y = X.to(dev), y.to(dev)
tr = BinarySGDTrainer(256, info=info, lr=0.5, l2=1e-3, momentum=0.9, device=dev)
for s in range(20):
    lo = s * B % 8192
    sl = slice(lo + r * per, lo + (r + 1) * per)
    tr.step(X[sl], y[sl])
np.save(f"{out}/params_{w}_{r}.npy", tr.params.cpu().numpy())
Xm, ym = synthetic_multiclass(8192, 256, 16, seed=3, noise=0.3)
mc = SoftmaxSGDTrainer(256, 16, info=info, lr=0.5, l2=1e-3, momentum=0.9, device=dev)
Xma = mc.prepare(Xm.to(dev))
ym = ym.to(dev)
for s in range(15):
    lo = s * B % 8192
    sl = slice(lo + r * per, lo + (r + 1) * per)
    mc.step(Xma[sl], ym[sl])
np.save(f"{out}/mc_params_{w}_{r}.npy", mc.params.cpu().numpy())
info.comm.wait()  # raises if a P2P call timed out
json.dump({"W": m.W.tolist(), "classes": list(m.classes), "acc": tr.last_accuracy(),
           "p2p_calls": 0 if info.comm.p2p is None else info.comm.p2p._p.epoch},
          open(f"{out}/bcast_{w}_{r}.json", "w"))
shutdown(info)
