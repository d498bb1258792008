"""Sweep gemm_softmax plans (rows-per-wave tiles x class splits) on one GPU, interleaved rounds in
one process (cdna_hip_programming.md 5.4 rule 24). Prints median us per call for each plan."""
import itertools
import json
import sys

import torch

sys.path.insert(0, ".")
from mlapi_amd._native import C  # noqa: E402
from mlapi_amd.ops import linear as ops  # noqa: E402

dev = torch.device("cuda", 0)
F, K = 256, 1000
res = {}
for B in (1024, 8192, 262144):
    X = torch.randn(B, F, device=dev).to(torch.bfloat16)
    W = (torch.randn(K, F, device=dev) / 16).to(torch.bfloat16)
    b = torch.randn(K, device=dev) * 0.1
    Z = X.float() @ W.float().T + b
    ref_idx = torch.argmax(Z, 1).to(torch.int32)
    plans = [(0, 0)] + list(itertools.product((1, 2), (1, 2, 4, 8, 16)))
    times = {p: [] for p in plans}
    ops_ = {}
    for p in plans:
        C().gemm_softmax_force_plan(*p)
        ops_[p] = ops.GemmSoftmax(B, K, F, dev)
        idx, _ = ops_[p](X, W, b)
        torch.cuda.synchronize()
        agree = (idx == ref_idx).float().mean().item()
        assert agree > 0.99, (B, p, agree)
    for rnd in range(5):
        for p in plans:
            C().gemm_softmax_force_plan(*p)
            op = ops_[p]
            out = (torch.empty(B, dtype=torch.int32, device=dev), torch.empty(B, device=dev))
            for _ in range(5):
                op(X, W, b, out=out)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            n = 50 if B <= 8192 else 10
            e0.record()
            for _ in range(n):
                op(X, W, b, out=out)
            e1.record()
            torch.cuda.synchronize()
            times[p].append(e0.elapsed_time(e1) * 1e3 / n)
    C().gemm_softmax_force_plan(0, 0)
    for p in plans:
        t = sorted(times[p])[len(times[p]) // 2]
        res[f"B{B}_nt{p[0]}_s{p[1]}"] = t
        tf = 2 * B * F * K / t / 1e6
        print(f"B={B:7d} plan nt={p[0]} splits={p[1]:2d}: {t:9.2f} us  {tf:7.1f} TF/s", flush=True)
json.dump(res, open("gpurun_out/gemm_plan_sweep.json", "w"), indent=1)
