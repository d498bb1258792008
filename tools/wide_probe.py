"""Phase timing of the f64-accumulating wide predict (csrc/kernels/linear_wide.h): the kernel is
launched repeatedly at serving batch sizes with the measurement probe set to stop after the MFMA
loop (1), before the class merge (2) or not at all (0); run under
  rocprofv3 --kernel-trace --stats --output-format csv -d <dir> -o prof -- python3 tools/wide_probe.py
and read the per-probe durations from the trace in launch order (each phase runs `iters` launches,
in the order below, separated by a 2 ms idle gap)."""
import sys
import time

import numpy as np
import torch

sys.path.insert(0, __import__("os").environ.get("GRAFT_REPO_ROOT", "."))
from mlapi_amd._native import C  # noqa: E402
from mlapi_amd.models.linear import Kind, LinearModel  # noqa: E402
from mlapi_amd.ops.linear import LinearWide  # noqa: E402

F = int(sys.argv[1]) if len(sys.argv) > 1 else 256
K = int(sys.argv[2]) if len(sys.argv) > 2 else 1000
iters = 200
m = LinearModel.random(F, K, seed=1)
for td in (torch.float32, torch.float64):
    op = LinearWide(32, F, K, td, "cuda")
    W = torch.tensor(m.W, device="cuda").to(td)
    b = torch.tensor(m.b, device="cuda")
    for B in (8, 24):
        X = torch.randn(B, F, device="cuda", dtype=torch.float64).to(td)
        for probe in (1, 2, 0):
            C().linear_wide_set_probe(probe)
            for _ in range(iters):
                op(X, W, b, int(Kind.MULTINOMIAL))
            torch.cuda.synchronize()
            time.sleep(0.002)
            print(f"phase dtype={td} B={B} probe={probe}", flush=True)
C().linear_wide_set_probe(0)
# reference: the f32-accumulating class-split kernel (linear_split.h) on the same shapes
from mlapi_amd.ops.linear import LinearSplit  # noqa: E402

sp = LinearSplit(32, K, "cuda")
Wf = torch.tensor(m.W, device="cuda", dtype=torch.float32)
bf = torch.tensor(m.b, device="cuda", dtype=torch.float32)
for B in (8, 24):
    Xf = torch.randn(B, F, device="cuda")
    for _ in range(iters):
        sp(Xf, Wf, bf)
    torch.cuda.synchronize()
    time.sleep(0.002)
    print(f"phase split f32 B={B}", flush=True)
