"""torchrun worker (GPU): data-parallel SGD, binary and multiclass, plus the C1 model broadcast.
MLAPI_DP_FUSED=1 (default): the all-reduce runs inside the gradient's final reduction kernel
(csrc/dist/p2p_device.h); MLAPI_DP_FUSED=0: the unfused path (gradient, one-shot P2P all-reduce
kernel, update). Writes <name>_<world>_<rank><tag>.npy and bcast_<world>_<rank><tag>.json under
$OUT (tag = "" fused, "_unfused" otherwise)."""
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
fused = os.environ.get("MLAPI_DP_FUSED", "1") != "0"
tag = ("" if fused else "_unfused") + ("_two" if os.environ.get("MLAPI_DP_TWO_SHOT") == "1" else "")
m = LinearModel.random(6, 5, seed=7, labels=["a", "b", "c", "d", "e"]) if r == 0 else None
m = broadcast_model(m, info)
B = 2048
per = B // w
X, y = synthetic_binary(8192, 256, seed=5, dtype=torch.bfloat16)
X, y = X.to(dev), y.to(dev)
tr = BinarySGDTrainer(256, info=info, lr=0.5, l2=1e-3, momentum=0.9, device=dev)
# one replica: the local step (no exchange object); N > 1: the in-kernel exchange unless unfused
assert tr.dp_exchange == ("local" if w == 1 else ("fused-p2p" if fused else "rccl")), tr.dp_exchange
assert w == 1 or info.__dict__.get("p2p_selftest") == ("ok" if fused else None), info.__dict__.get("p2p_selftest")
for s in range(20):
    lo = s * B % 8192
    sl = slice(lo + r * per, lo + (r + 1) * per)
    tr.step(X[sl], y[sl])
np.save(f"{out}/params_{w}_{r}{tag}.npy", tr.params.cpu().numpy())
Xm, ym = synthetic_multiclass(8192, 256, 16, seed=3, noise=0.3)
mc = SoftmaxSGDTrainer(256, 16, info=info, lr=0.5, l2=1e-3, momentum=0.9, device=dev)
Xma = mc.prepare(Xm.to(dev))
ym = ym.to(dev)
for s in range(15):
    lo = s * B % 8192
    sl = slice(lo + r * per, lo + (r + 1) * per)
    mc.step(Xma[sl], ym[sl])
assert mc.dp_exchange == tr.dp_exchange
np.save(f"{out}/mc_params_{w}_{r}{tag}.npy", mc.params.cpu().numpy())
info.comm.wait()  # raises if a P2P call timed out
tr.check()
mc.check()
json.dump({"W": m.W.tolist(), "classes": list(m.classes), "acc": tr.last_accuracy(),
           "p2p_calls": 0 if info.comm.p2p is None else info.comm.p2p._p.epoch},
          open(f"{out}/bcast_{w}_{r}{tag}.json", "w"))
shutdown(info)
