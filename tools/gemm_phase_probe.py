"""Where a gemm_softmax wave spends its time: every wave of one launch writes 4 s_memtime stamps
(entry, first W chunk + X landed, class loop done, row state reduced) and, in the 32x32 kernel, the
cycles its class loop waited at the per-chunk DMA wait + barrier; this prints per-phase
cycle statistics per kernel plan. Run on the GPU box:

    python tools/gemm_phase_probe.py [B ...]          (default 1024 262144)
"""
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from mlapi_amd._native import C  # noqa: E402
from mlapi_amd.ops import linear as ops  # noqa: E402

dev = torch.device("cuda", 0)
F, K = 256, 1000
PLANS = {"auto": (0, 0, 0), "t16_nt2": (2, 0, 1), "t32": (0, 0, 3), "t32_noepi": (0, 0, 5), "t32_ahead1": (0, 0, 6), "t32_ahead3": (0, 0, 7), "t32_xnt": (0, 0, 9)}
for B in tuple(int(a) for a in sys.argv[1:]) or (1024, 262144):
    X = torch.randn(B, F, device=dev).to(torch.bfloat16)
    W = (torch.randn(K, F, device=dev) / 16).to(torch.bfloat16)
    b = torch.randn(K, device=dev) * 0.1
    stamps = torch.zeros(8 * (B // 16 + 64) * 16, dtype=torch.int64, device=dev)
    for name, plan in PLANS.items():
        C().gemm_softmax_force_plan(*plan)
        op = ops.GemmSoftmax(B, K, F, dev)
        out = (torch.empty(B, dtype=torch.int32, device=dev), torch.empty(B, device=dev))
        for _ in range(5):
            op(X, W, b, out=out)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            op(X, W, b, out=out)
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / 10
        stamps.zero_()
        C().gemm_softmax_set_stamps(stamps.data_ptr())
        op(X, W, b, out=out)
        torch.cuda.synchronize()
        C().gemm_softmax_set_stamps(0)
        t8 = stamps.view(-1, 8).cpu().numpy()
        t8 = t8[t8[:, 0] != 0].astype(np.float64)
        t, wait = t8[:, :4], t8[:, 4]
        d = np.diff(t, axis=1)
        life = t[:, 3] - t[:, 0]
        q = lambda a: f"{np.median(a):9.0f} {np.percentile(a, 90):9.0f}"  # noqa: E731
        print(f"B={B:7d} {name:8s} {us:8.2f} us/launch  waves {len(t):6d} | median/p90 cycles: "
              f"prologue {q(d[:, 0])} | loop {q(d[:, 1])} (wait+barrier {q(wait)}) | reduce {q(d[:, 2])} | "
              f"life {q(life)}", flush=True)
    C().gemm_softmax_force_plan(0, 0, 0)
