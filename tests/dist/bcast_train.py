"""torchrun worker: C1 broadcast + DP SGD determinism on gloo (CPU). Writes rank results to $OUT."""
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

info = init_distributed(use_gpu=False)
out = os.environ["OUT"]
m = LinearModel.random(6, 5, seed=7, labels=["a", "b", "c", "d", "e"]) if info.rank == 0 else None
m = broadcast_model(m, info)
X, y = synthetic_binary(4096, 32, seed=5, dtype=torch.float32)
B = 512
per = B // info.world
tr = BinarySGDTrainer(32, info=info, lr=0.5, l2=1e-3, momentum=0.9)
for s in range(20):
    lo = s * B % 4096
    xs, ys = X[lo + info.rank * per: lo + (info.rank + 1) * per], y[lo + info.rank * per: lo + (info.rank + 1) * per]
    tr.step(xs, ys)
np.save(f"{out}/params_{info.world}_{info.rank}.npy", tr.params.numpy())
# multiclass DP: [dW_aug | loss | correct] all-reduce + identical updates
Xm, ym = synthetic_multiclass(2048, 32, 5, seed=3, noise=0.3)
mc = SoftmaxSGDTrainer(32, 5, info=info, lr=0.5, l2=1e-3, momentum=0.9, device=torch.device("cpu"))
Xma = mc.prepare(Xm)
for s in range(15):
    lo = s * B % 2048
    sl = slice(lo + info.rank * per, lo + (info.rank + 1) * per)
    mc.step(Xma[sl], ym[sl])
np.save(f"{out}/mc_params_{info.world}_{info.rank}.npy", mc.params.numpy())
json.dump({"W": m.W.tolist(), "b": m.b.tolist(), "classes": list(m.classes), "kind": int(m.kind),
           "loss": tr.last_loss(), "acc": tr.last_accuracy()}, open(f"{out}/bcast_{info.world}_{info.rank}.json", "w"))
shutdown(info)
