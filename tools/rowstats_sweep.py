"""The 1000-class training step (row stats + fused G/dW + slab sums) timed over forced plans of its
row-stats pass (gemm_softmax MODE 2: kernel, rows per wave, class splits) crossed with the fused
gradient's row-group count; every plan's dW is checked against the automatic plan's.
    python3 tools/rowstats_sweep.py            -> one JSON line per plan (median of 5 x 20 calls)"""
import json
import os
import sys

import torch

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
from mlapi_amd._native import C  # noqa: E402
from mlapi_amd.ops import linear as ops  # noqa: E402

dev = torch.device("cuda", 0)
B, K, F = 65536, 1000, 256
Fa = ops.softmax_train_faug(F)
X = ops.augment_features(torch.randn(B, F, device=dev), Fa)
W = (torch.randn(K, F, device=dev) / 16).to(torch.bfloat16)
bias = torch.zeros(K, device=dev)
y = torch.randint(0, K, (B,), device=dev, dtype=torch.int32)
stf = torch.zeros(2, device=dev)


def timed(fn, n=20, rounds=5):
    for _ in range(3):
        fn()
    out = []
    for _ in range(rounds):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(n):
            fn()
        e1.record()
        torch.cuda.synchronize()
        out.append(e0.elapsed_time(e1) * 1e3 / n)
    return sorted(out)[len(out) // 2]


# (nt, splits, kernel) of the row-stats pass x fused-gradient row groups (0 = automatic)
GEMM = [(0, 0, 0), (0, 1, 3), (0, 2, 3), (0, 4, 3), (2, 1, 1), (2, 2, 1), (2, 4, 1)]
GROUPS = [0, 16, 32, 64]
if os.environ.get("SWEEP_GEMM"):
    GEMM = [tuple(int(v) for v in t.split(",")) for t in os.environ["SWEEP_GEMM"].split()]
if os.environ.get("SWEEP_GROUPS"):
    GROUPS = [int(v) for v in os.environ["SWEEP_GROUPS"].split()]
ref = None
for gp in GEMM:
    for rg in GROUPS:
        C().gemm_softmax_force_plan(*gp)
        C().softmax_grad_dw_force_plan(rg, 0)
        fb = ops.SoftmaxTrainBuffers(B, K, F, dev)  # the workspace layout depends on both plans
        out = torch.empty(K, Fa, device=dev)
        fn = lambda: ops.softmax_train_grad(X, W, bias, y, 2, bufs=fb, dW_out=out, stats_out=stf)  # noqa: E731
        us = timed(fn)
        if ref is None:
            ref = out.clone()
        err = ((out - ref).abs().max() / ref.abs().max()).item()
        print(json.dumps({"gemm_plan": gp, "row_groups": rg, "us": round(us, 2), "max_rel_dw_err": err}), flush=True)
C().gemm_softmax_force_plan(0, 0, 0)
C().softmax_grad_dw_force_plan(0, 0)
