"""Sweep gemm_softmax plans on one GPU, interleaved rounds in one process (cdna_hip_programming.md
5.4 rule 24): the tiles kernel's (rows-per-wave tiles x class splits) plans and the row-group
kernel. Prints median us per call for each plan
(graph replay = GPU time; eager = through the Python op)."""
import itertools
import json
import os
import sys

import torch

sys.path.insert(0, ".")
from mlapi_amd._native import C  # noqa: E402
from mlapi_amd.ops import linear as ops  # noqa: E402

dev = torch.device("cuda", 0)
F, K = int(os.environ.get("SWEEP_F", 256)), int(os.environ.get("SWEEP_K", 1000))
res = {}
for B in tuple(int(a) for a in sys.argv[1:]) or (1, 64, 256, 1024, 2048, 4096, 8192, 262144):
    X = torch.randn(B, F, device=dev).to(torch.bfloat16)
    W = (torch.randn(K, F, device=dev) / 16).to(torch.bfloat16)
    b = torch.randn(K, device=dev) * 0.1
    Z = X.float() @ W.float().T + b
    ref_idx = torch.argmax(Z, 1).to(torch.int32)
    plans = [(0, 0, 0), (0, 0, 2)]
    if F <= 512:
        plans += [(nt, sp, 1) for nt, sp in itertools.product((1, 2), (2, 4, 8, 16, 32))]
    if F in (64, 128, 256):
        plans += [(0, sp, 3) for sp in (0, 2, 4, 8)]
    if os.environ.get("SWEEP_PLANS"):  # e.g. "0,0,3 0,0,8": (nt, splits, kernel) triples only
        plans = [tuple(int(v) for v in t.split(",")) for t in os.environ["SWEEP_PLANS"].split()]
    times = {p: [] for p in plans}
    ops_ = {}
    for p in plans:
        C().gemm_softmax_force_plan(*p)
        ops_[p] = ops.GemmSoftmax(B, K, F, dev)
        idx, _ = ops_[p](X, W, b)
        torch.cuda.synchronize()
        agree = (idx == ref_idx).float().mean().item()
        assert agree > 0.99, (B, p, agree)
    # GPU time per call: 20 launches captured in one HIP graph, replayed (no Python dispatch in
    # the timed region); the eager figure adds the per-call host overhead of ops.GemmSoftmax.
    graphs = {}
    for p in plans:
        C().gemm_softmax_force_plan(*p)
        op = ops_[p]
        out = (torch.empty(B, dtype=torch.int32, device=dev), torch.empty(B, device=dev))
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            op(X, W, b, out=out)
        torch.cuda.current_stream().wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(20):
                op(X, W, b, out=out)
        graphs[p] = (g, op, out)
    eager = {p: [] for p in plans}
    for rnd in range(5):
        for p in plans:
            g, op, out = graphs[p]
            g.replay()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            reps = 5 if B <= 8192 else 1
            e0.record()
            for _ in range(reps):
                g.replay()
            e1.record()
            torch.cuda.synchronize()
            times[p].append(e0.elapsed_time(e1) * 1e3 / (20 * reps))
            C().gemm_softmax_force_plan(*p)
            n = 50 if B <= 8192 else 10
            e0.record()
            for _ in range(n):
                op(X, W, b, out=out)
            e1.record()
            torch.cuda.synchronize()
            eager[p].append(e0.elapsed_time(e1) * 1e3 / n)
    C().gemm_softmax_force_plan(0, 0, 0)
    for p in plans:
        t = sorted(times[p])[len(times[p]) // 2]
        te = sorted(eager[p])[len(eager[p]) // 2]
        res[f"B{B}_nt{p[0]}_s{p[1]}_k{p[2]}"] = {"graph_us": t, "eager_us": te}
        tf = 2 * B * F * K / t / 1e6
        name = {0: "auto", 1: "tiles", 2: "rows", 3: "t32"}.get(p[2], f"k{p[2]}")
        print(f"B={B:7d} {name:5s} nt={p[0]} splits={p[1]:2d}: {t:9.2f} us graph {te:9.2f} us eager  {tf:7.1f} TF/s", flush=True)
json.dump(res, open("gpurun_out/gemm_plan_sweep.json", "w"), indent=1)
