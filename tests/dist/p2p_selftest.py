"""torchrun worker (GPU, 2 ranks on one device, MLAPI_COMM=p2p): the fused DP exchange proves itself
before first use (mlapi_amd/parallel/p2p.py verify_exchange) and by the replica hash every
MLAPI_DP_VERIFY_EVERY steps. Faults: MLAPI_P2P_SELFTEST_CORRUPT=<rank> (a wrong IPC pattern word),
MLAPI_P2P_VERIFY_FAULT=<rank> (one block's flag never published: a stale flag for the peer),
CORRUPT_AT_STEP=<n> (rank 1's parameters nudged after step n: the periodic check must catch it).
Every failure must make every rank fall back from the fused in-kernel exchange to the unfused
all-reduce path and still train bitwise-identical replicas."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
from mlapi_amd.parallel.comm import init_distributed, shutdown  # noqa: E402
from mlapi_amd.train.softmax_sgd import SoftmaxSGDTrainer, synthetic_multiclass  # noqa: E402

info = init_distributed(use_gpu=True, comm="p2p")
dev, out, r, w = info.device, os.environ["OUT"], info.rank, info.world
corrupt_at = int(os.environ.get("CORRUPT_AT_STEP", "-1"))
Xm, ym = synthetic_multiclass(4096, 256, 16, seed=3, noise=0.3)
mc = SoftmaxSGDTrainer(256, 16, info=info, lr=0.5, l2=1e-3, device=dev)
first = mc.dp_exchange
Xma = mc.prepare(Xm.to(dev))
ym = ym.to(dev)
per = 1024 // w
for s in range(6):
    lo = s * 1024 % 4096
    sl = slice(lo + r * per, lo + (r + 1) * per)
    mc.step(Xma[sl], ym[sl])
    if s + 1 == corrupt_at and r == 1:
        mc.params[0, 0] += 1e-3  # a replica that silently diverged
        mc._refresh_shadow()
mc.check()
np.save(f"{out}/st_params_{r}.npy", mc.params.cpu().numpy())
json.dump({"p2p_selftest": info.__dict__.get("p2p_selftest"), "p2p_verify": info.__dict__.get("p2p_verify"),
           "dp_exchange_first": first, "dp_exchange": mc.dp_exchange},
          open(f"{out}/selftest_{r}.json", "w"))
shutdown(info)
