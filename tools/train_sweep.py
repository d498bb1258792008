"""Sweep the gradient kernel's grid cap (bytes in flight vs slabs to reduce), interleaved rounds."""
import json
import sys

import torch

sys.path.insert(0, ".")
from mlapi_amd._native import C  # noqa: E402

dev = torch.device("cuda", 0)
F = 256
res = {}
for B in (65536, 262144, 1 << 20):
    X = torch.randn(B, F, device=dev).to(torch.bfloat16)
    y = (torch.rand(B, device=dev) > 0.5).float()
    params = torch.zeros(F + 1, device=dev)
    grad = torch.empty(F + 3, device=dev)
    ws = torch.empty((8192 + 64) * (F + 3) * 4, dtype=torch.uint8, device=dev)
    caps = (256, 512, 1024, 2048, 4096)
    times = {c: [] for c in caps}
    s = torch.cuda.current_stream().cuda_stream
    for rnd in range(5):
        for cap in caps:
            C().train_binary_set_max_blocks(cap)
            for _ in range(3):
                C().train_binary_step(2, X.data_ptr(), y.data_ptr(), params.data_ptr(), 0, B, F, grad.data_ptr(),
                                      ws.data_ptr(), ws.numel(), 0.1, 1.0 / B, 0.0, 0.0, s)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(20):
                C().train_binary_step(2, X.data_ptr(), y.data_ptr(), params.data_ptr(), 0, B, F, grad.data_ptr(),
                                      ws.data_ptr(), ws.numel(), 0.1, 1.0 / B, 0.0, 0.0, s)
            e1.record()
            torch.cuda.synchronize()
            times[cap].append(e0.elapsed_time(e1) * 1e3 / 20)
    C().train_binary_set_max_blocks(0)
    for cap in caps:
        t = sorted(times[cap])[2]
        res[f"B{B}_cap{cap}"] = t
        print(f"B={B:8d} cap={cap:5d}: {t:8.2f} us/step  {B * F * 2 / t / 1e6:7.2f} TB/s  {B / t:8.1f} M samples/s",
              flush=True)
json.dump(res, open("gpurun_out/train_sweep.json", "w"), indent=1)
