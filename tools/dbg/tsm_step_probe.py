"""Where the 1000-class training step's time goes beyond its kernels: the bench's eager step
(SoftmaxSGDTrainer.step, fused update) timed with device events, one shard and two alternating,
against the same step captured in a HIP graph and the bare gradient call."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
from mlapi_amd.parallel.comm import init_distributed  # noqa: E402
from mlapi_amd.train.softmax_sgd import SoftmaxSGDTrainer, synthetic_multiclass  # noqa: E402

info = init_distributed()
F, K, B = 256, 1000, 65536
X, y = synthetic_multiclass(B * 2, F, K, seed=99, device=info.device)
tr = SoftmaxSGDTrainer(F, K, info=info, lr=0.5, l2=1e-5, device=info.device)
Xa = tr.prepare(X)
shards = [(Xa[:B], y[:B]), (Xa[B:], y[B:])]


def timed(fn, n=200):
    for _ in range(20):
        fn(0)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record()
    for s in range(n):
        fn(s)
    e1.record()
    host = (time.perf_counter() - t0) * 1e6 / n
    torch.cuda.synchronize()
    return round(e0.elapsed_time(e1) * 1e3 / n, 2), round(host, 2)


res = {}
res["eager_two_shards"] = timed(lambda s: tr.step(*shards[s % 2]))
res["eager_one_shard"] = timed(lambda s: tr.step(*shards[0]))
tr.capture(*shards[0])
res["graph_one_shard"] = timed(lambda s: tr.step(*shards[0]))
print(json.dumps({k: {"device_us": v[0], "host_us": v[1]} for k, v in res.items()}), flush=True)
