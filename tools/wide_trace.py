"""In-kernel timeline of the f64-accumulating wide predict (csrc/kernels/linear_wide.h) at serving
batch sizes: every block stamps the 100 MHz wall clock at entry, after its MFMA loop and after
publishing its row states; the merging block also stamps its poll begin / end and the rows
written (linear_wide_set_trace). Prints the median over `iters` launches of each stamp relative to
the first block's entry, in µs:
  python3 tools/wide_trace.py [F] [K] [iters]
(pair with tools/wide_probe.py under rocprofv3 for the launch overhead around the in-kernel span)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
from mlapi_amd._native import C  # noqa: E402
from mlapi_amd.models.linear import Kind, LinearModel  # noqa: E402
from mlapi_amd.ops.linear import LinearWide  # noqa: E402

F = int(sys.argv[1]) if len(sys.argv) > 1 else 256
K = int(sys.argv[2]) if len(sys.argv) > 2 else 1000
iters = int(sys.argv[3]) if len(sys.argv) > 3 else 200
m = LinearModel.random(F, K, seed=1)
c = C()
for td in (torch.float64, torch.float32):
    op = LinearWide(32, F, K, td, "cuda")
    W = torch.tensor(m.W, device="cuda").to(td)
    b = torch.tensor(m.b, device="cuda")
    for B in (1, 8, 24):
        ncb = (K + 15) // 16
        tr = torch.zeros(ncb * 64 * 8, dtype=torch.int64, device="cuda")  # generous: nfs x ncb blocks
        X = torch.randn(B, F, device="cuda", dtype=torch.float64).to(td)
        c.linear_wide_set_trace(tr.data_ptr())
        rows = []
        for it in range(iters + 20):
            tr.zero_()
            op(X, W, b, int(Kind.MULTINOMIAL))
            torch.cuda.synchronize()
            if it < 20:
                continue
            t = tr.view(-1, 8).cpu().numpy()
            t = t[t[:, 0] != 0]
            base = t[:, 0].min()
            mg = t[t[:, 5] != 0]  # the merging block(s)
            rows.append([
                (t[:, 0].max() - base),             # last block entry
                (np.median(t[:, 1]) - base),        # median block MFMA done
                (t[:, 1].max() - base),             # last block MFMA done
                (t[:, 2].max() - base),             # last state published
                (mg[:, 3].max() - base) if len(mg) else 0,  # merger poll begin
                (mg[:, 4].max() - base) if len(mg) else 0,  # merger poll end
                (mg[:, 5].max() - base) if len(mg) else 0,  # rows written
                (np.median(t[:, 0]) - base),        # median block entry
                np.median(t[:, 1] - t[:, 0]),       # median per-block MFMA phase
                np.max(t[:, 1] - t[:, 0]),          # longest per-block MFMA phase
                np.median(t[:, 2] - t[:, 1]),       # median per-block epilogue
                np.median(t[:, 7] - t[:, 0]),       # median entry -> kernel arguments arrived
                np.median(t[:, 6] - t[:, 0]),       # median entry -> first operands landed
            ])
        c.linear_wide_set_trace(0)
        r = np.median(np.array(rows, dtype=np.float64), axis=0) / 100.0  # 100 MHz ticks -> us
        print(f"dtype={str(td)[6:]} F={F} K={K} B={B} blocks={len(t)}: last entry {r[0]:.2f}  mfma med {r[1]:.2f} "
              f"last {r[2]:.2f}  states {r[3]:.2f}  poll begin {r[4]:.2f} end {r[5]:.2f}  rows {r[6]:.2f} us"
              f" | entry med {r[7]:.2f}  per-block mfma med {r[8]:.2f} max {r[9]:.2f}  epilogue med {r[10]:.2f}"
              f"  kernargs +{r[11]:.2f} operands +{r[12]:.2f}",
              flush=True)
