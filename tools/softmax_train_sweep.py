"""Time the multiclass training step's pieces (K=1000, F=256, B=65536): MFMA row-stat/grad
launches at NT 1/2 and the dW GEMM as one hipBLASLt mm vs a batched split-B bmm + sum (the
"gemm" dW path), and the fused G + dW kernel (softmax_grad_dw.hip) over forced row-group counts."""
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
B, F, K = 65536, 256, 1000
Fa = ops.softmax_train_faug(F)
X = ops.augment_features(torch.randn(B, F, device=dev), Fa)
W = (torch.randn(K, F, device=dev) / 16).to(torch.bfloat16)
bias = torch.zeros(K, device=dev)
y = torch.randint(0, K, (B,), device=dev, dtype=torch.int32)
res = {}
for nt in (1, 2):
    C().gemm_softmax_force_plan(nt, 0)
    bufs = ops.SoftmaxTrainBuffers(B, K, F, dev, dw_path="gemm")
    st = torch.zeros(2, device=dev)
    t = timeit(lambda: C().softmax_train_grad(X.data_ptr(), Fa, W.data_ptr(), bias.data_ptr(), y.data_ptr(), B, F, K, 2,
                                              bufs.G.data_ptr(), bufs.ldg, st.data_ptr(), bufs.ws.data_ptr(),
                                              bufs.ws.numel(), torch.cuda.current_stream().cuda_stream))
    res[f"grad_launches_nt{nt}_us"] = t
C().gemm_softmax_force_plan(0, 0)
G = bufs.G[:B, :K]
out = torch.empty(K, Fa, device=dev)
res["dW_mm_us"] = timeit(lambda: torch.mm(G.t(), X, out_dtype=torch.float32, out=out))
ref = out.clone()
for S in (2, 4, 8, 16, 32, 64):
    Gs = bufs.G[:B].view(S, B // S, bufs.ldg)[:, :, :K]
    Xs = X.view(S, B // S, Fa)
    part = torch.empty(S, K, Fa, device=dev)

    def f():
        torch.bmm(Gs.transpose(1, 2), Xs, out_dtype=torch.float32, out=part)
        torch.sum(part, dim=0, out=out)

    res[f"dW_bmm_S{S}_us"] = timeit(f)
    res[f"dW_bmm_S{S}_maxdiff"] = (out - ref).abs().max().item()
# fused path: rowstats + G/dW kernel + slab sums, whole call
stf = torch.zeros(2, device=dev)
for nc, pipe in ((1, 0), (2, 1), (2, 2)):
    for groups in (0, 16, 32, 64):
        C().softmax_grad_dw_force_plan(groups, nc, pipe)
        fb = ops.SoftmaxTrainBuffers(B, K, F, dev, dw_path="fused")
        res[f"fused_nc{nc}_pipe{pipe}_groups{groups}_us"] = timeit(
            lambda: ops.softmax_train_grad(X, W, bias, y, 2, bufs=fb, dW_out=out, stats_out=stf))
        res[f"fused_nc{nc}_pipe{pipe}_groups{groups}_maxdiff"] = (out - ref).abs().max().item()
C().softmax_grad_dw_force_plan(0, 0, 0)
gb = ops.SoftmaxTrainBuffers(B, K, F, dev, dw_path="gemm")
res["gemm_path_total_us"] = timeit(lambda: ops.softmax_train_grad(X, W, bias, y, 2, bufs=gb, dW_out=out, stats_out=stf))
res["dW_ref_absmax"] = ref.abs().max().item()
for k, v in res.items():
    print(f"{k:28s} {v:10.3f}")
json.dump(res, open("gpurun_out/softmax_train_sweep.json", "w"), indent=1)
