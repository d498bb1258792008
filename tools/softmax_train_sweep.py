"""Time the fused multiclass gradient (row stats + softmax_grad_dw.hip + slab sums) over forced
plans (class tiles per wave, cross-tile pipeline, row-group counts) and feature widths; every
plan's dW is checked against the automatic plan's."""
import json
import sys

import torch

sys.path.insert(0, ".")
from mlapi_amd._native import C  # noqa: E402
from mlapi_amd.ops import linear as ops  # noqa: E402


def timeit(fn, n=20):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / n


dev = torch.device("cuda", 0)
B, K = 65536, 1000
res = {}
stf = torch.zeros(2, device=dev)
for F in (128, 256, 512):
    Fa = ops.softmax_train_faug(F)
    X = ops.augment_features(torch.randn(B, F, device=dev), Fa)
    W = (torch.randn(K, F, device=dev) / 16).to(torch.bfloat16)
    bias = torch.zeros(K, device=dev)
    y = torch.randint(0, K, (B,), device=dev, dtype=torch.int32)
    out = torch.empty(K, Fa, device=dev)
    fb = ops.SoftmaxTrainBuffers(B, K, F, dev)
    res[f"F{F}_auto_us"] = timeit(lambda: ops.softmax_train_grad(X, W, bias, y, 2, bufs=fb, dW_out=out, stats_out=stf))
    ref = out.clone()
    plans = (1, 2) if F < 512 else (1,)
    for nc in plans:
        for groups in (0, 16, 32, 64):
            C().softmax_grad_dw_force_plan(groups, nc)
            pb = ops.SoftmaxTrainBuffers(B, K, F, dev)  # the workspace layout depends on the forced plan
            res[f"F{F}_nc{nc}_groups{groups}_us"] = timeit(
                lambda: ops.softmax_train_grad(X, W, bias, y, 2, bufs=pb, dW_out=out, stats_out=stf))
            res[f"F{F}_nc{nc}_groups{groups}_maxdiff"] = (out - ref).abs().max().item()
    C().softmax_grad_dw_force_plan(0, 0)
    res[f"F{F}_tflops_auto"] = 4 * B * K * Fa / res[f"F{F}_auto_us"] / 1e6  # rowstats + logits + dW
for k, v in res.items():
    print(f"{k:36s} {v:10.3f}")
json.dump(res, open("gpurun_out/softmax_train_sweep.json", "w"), indent=1)
