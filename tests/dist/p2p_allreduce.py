"""torchrun worker (GPU): the one-shot P2P all-reduce across ranks sharing the box's GPU(s).

Every result must equal the rank-ordered float32 sum bit for bit (bfloat16: fp32 sum, one RNE
rounding); more than two epochs exercise the double-buffered halves; the last call is made by rank 0
alone and must time out (status 1) instead of hanging. Writes P2P_<rank>.json under $OUT."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
from mlapi_amd.parallel.comm import barrier, init_distributed, shutdown  # noqa: E402
from mlapi_amd.parallel.p2p import P2PAllReduce  # noqa: E402

info = init_distributed(use_gpu=True, comm="fake")  # gloo control plane; data plane = P2P kernel
r, w, dev = info.rank, info.world, info.device
p2p = P2PAllReduce(r, w, dev, max_bytes=1 << 20)


def inputs(n, dtype, seed):
    return [torch.randn(n, generator=torch.Generator().manual_seed(seed * 131 + k)).to(dtype) for k in range(w)]


checks = 0
for call, (n, dtype) in enumerate([(1000, torch.float32), (4096, torch.bfloat16), (3, torch.float32),
                                   (262144, torch.float32), (77, torch.bfloat16), (524288, torch.bfloat16),
                                   (1001, torch.float32)]):
    xs = inputs(n, dtype, call)
    t = xs[r].to(dev)
    p2p.all_reduce_(t)
    acc = xs[0].float()
    for k in range(1, w):
        acc = acc + xs[k].float()  # rank order, float32 (as the kernel)
    want = acc.to(dtype)
    got = t.cpu()
    assert torch.equal(got, want), (call, n, dtype, (got.float() - want.float()).abs().max().item())
    checks += 1
assert p2p.status() == 0
# latency of back-to-back 256 KiB float32 calls (ranks sharing one GPU: a functional number only)
t = torch.ones(65536, device=dev)
barrier(info)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(50):
    p2p.all_reduce_(t)
torch.cuda.synchronize()
us = (time.perf_counter() - t0) / 50 * 1e6
assert torch.all(t == float(w) ** 50 if w > 1 else t == 1.0)
assert p2p.status() == 0
barrier(info)
timed_out = None
if r == 0 and w > 1:  # a peer that never arrives: bounded wait, sticky status, no hang
    p2p.all_reduce_(torch.ones(16, device=dev), timeout_ms=300)
    timed_out = p2p.status()
barrier(info)
json.dump({"checks": checks, "epoch": p2p._p.epoch, "us_per_call_256k": us, "timed_out": timed_out},
          open(os.path.join(os.environ["OUT"], f"P2P_{r}.json"), "w"))
shutdown(info)
