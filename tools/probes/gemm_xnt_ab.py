"""A/B of gemm_softmax32's X loads (plain, the default since round 6, vs the nontemporal hint,
forced kernel 9) at B = 262,144, K = 1000, F = 256 bf16: CUDA-event time per launch, interleaved."""
import sys

import torch

sys.path.insert(0, ".")
from mlapi_amd._native import C  # noqa: E402
from mlapi_amd.ops import linear as ops  # noqa: E402

dev = torch.device("cuda", 0)
B, F, K = 262144, 256, 1000
X = torch.randn(B, F, device=dev).to(torch.bfloat16)
W = (torch.randn(K, F, device=dev) / 16).to(torch.bfloat16)
b = torch.randn(K, device=dev) * 0.1
out = (torch.empty(B, dtype=torch.int32, device=dev), torch.empty(B, device=dev))
res = {}
# default: plain vs nontemporal X; argv "all": also the W look-ahead (1 / 3 k-steps) and s_setprio variants
VARIANTS = [("plain", 0), ("nontemporal", 9)]
if "all" in sys.argv[1:]:
    VARIANTS += [("ahead1", 6), ("ahead3", 7), ("setprio", 8)]
for rnd in range(4):
    for name, kern in VARIANTS:
        C().gemm_softmax_force_plan(0, 0, kern)
        op = ops.GemmSoftmax(B, K, F, dev)
        for _ in range(10):
            op(X, W, b, out=out)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(50):
            op(X, W, b, out=out)
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / 50
        res.setdefault(name, []).append(us)
        print(f"r{rnd} {name:12s} {us:7.2f} us  {2 * B * K * F / us / 1e6:6.1f} TF/s", flush=True)
C().gemm_softmax_force_plan(0, 0, 0)
for k, v in res.items():
    print(k, "median %.2f us" % sorted(v)[len(v) // 2])
