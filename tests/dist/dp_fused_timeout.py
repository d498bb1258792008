"""torchrun worker (GPU, 2 ranks): rank 1 skips a fused DP training step; rank 0's in-kernel
exchange must time out (bounded spin), leave its parameters untouched and report the failure."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
from mlapi_amd.parallel.comm import barrier, init_distributed, shutdown  # noqa: E402
from mlapi_amd.train.sgd import BinarySGDTrainer, synthetic_binary  # noqa: E402

info = init_distributed(use_gpu=True, comm="p2p")
dev, out = info.device, os.environ["OUT"]
X, y = synthetic_binary(1024, 256, seed=5, dtype=torch.bfloat16)
X, y = X.to(dev), y.to(dev)
tr = BinarySGDTrainer(256, info=info, lr=0.5, device=dev)
assert tr.dp_exchange == "fused-p2p"
tr.dp_timeout_ms = 300
barrier(info)
if info.rank == 0:
    before = tr.params.clone()
    t0 = time.time()
    tr.step(X, y)
    raised = False
    try:
        tr.check()
    except RuntimeError:
        raised = True
    # the sticky status is host-mapped: the next step stops at once (no silent divergence)
    next_raised = False
    try:
        tr.step(X, y)
    except RuntimeError:
        next_raised = True
    torch.cuda.synchronize()
    res = {"raised": raised, "params_unchanged": bool(torch.equal(before, tr.params)), "elapsed_s": time.time() - t0,
           "next_step_raised": next_raised}
    json.dump(res, open(f"{out}/timeout_{info.rank}.json", "w"))
barrier(info)
shutdown(info)
