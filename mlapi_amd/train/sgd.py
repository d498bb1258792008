"""Data-parallel mini-batch SGD for logistic regression (BASELINE config 5).

Re-imagines the reference's offline ``LogisticRegression().fit`` (`Logistic Regression.ipynb:33-34`)
as a DP training loop. Per step and rank, TWO launches at any world size (one GPU per rank, ranks
on one host - the MI355X node):

  1. the gradient kernel (one HBM pass over the rank's shard: forward, sigmoid, BCE, and the
     dW = sum g_i x_i reduction - all fused) writes per-block slabs of
     [gW (F) | gb | loss_sum | n_correct];
  2. the slab-reduction kernel sums them, exchanges each block's column sums with the same block
     of every rank through IPC-mapped buffers over xGMI (C2 + C3, csrc/dist/p2p_device.h: one
     hop, peers summed in rank order) and applies w -= lr * (g / N_global + l2 * w) (intercept
     unpenalized, like sklearn's L2) in the same kernel.

World = 1 runs the same two kernels (the exchange with itself), so the N = 1 and N > 1 benches
time the same code. Ranks on several hosts (or ``MLAPI_DP_FUSED=0``) use the unfused path: the
gradient, an RCCL all-reduce of the fused buffer, then ``sgd_update``.

Every rank applies the identical update to identical parameters, so replicas stay bitwise equal
(checked by tests) without ever broadcasting parameters after initialisation.

The objective matches sklearn's (mean log-loss + l2/2 ||w||^2 with l2 = 1 / (C * N)).
"""
from __future__ import annotations

from typing import Optional, Tuple

import torch

from mlapi_amd.parallel.comm import DistInfo, all_reduce_sum_


def synthetic_binary(n: int, F: int, *, seed: int = 0, device=None, dtype=torch.bfloat16, noise: float = 0.5):
    """Linearly separable-ish synthetic tabular data with a fixed planted weight vector."""
    g = torch.Generator(device="cpu").manual_seed(seed)
    w_true = torch.randn(F, generator=torch.Generator().manual_seed(42)) / F ** 0.5
    X = torch.randn(n, F, generator=g)
    z = X @ w_true + noise * torch.randn(n, generator=g)
    y = (z > 0).float()
    return X.to(dtype).to(device), y.to(device)


class BinarySGDTrainer:
    """Binary LR trainer on one GPU per rank (fp32 master weights, bf16/f32 data)."""

    def __init__(self, n_features: int, *, info: Optional[DistInfo] = None, lr: float = 0.1, l2: float = 0.0,
                 momentum: float = 0.0, device=None):
        from mlapi_amd._native import C

        self.F = n_features
        self.info = info or DistInfo(device=device)
        self.device = device if device is not None else self.info.device
        self.on_gpu = self.device is not None and torch.device(self.device).type == "cuda"
        if self.device is None:
            self.device = torch.device("cpu")  # explicit CPU path (gloo tests / GPU-less hosts)
        self.lr, self.l2, self.momentum = lr, l2, momentum
        # params = [w (F) | b]; grad buffer = [gw | gb | loss | correct]
        self.params = torch.zeros(n_features + 1, dtype=torch.float32, device=self.device)
        self.grad = torch.zeros(n_features + 3, dtype=torch.float32, device=self.device)
        self.mom = torch.zeros_like(self.params) if momentum else None
        self._ws = None
        self._C = C()
        self._dp = None
        if self.on_gpu:
            from mlapi_amd.parallel.p2p import dp_exchange

            self._dp = dp_exchange(self.info, (n_features + 3) * 4)
        self.dp_timeout_ms = 60_000
        from mlapi_amd.parallel.p2p import verify_every

        self.verify_every = verify_every()  # fused steps between replica checks (MLAPI_DP_VERIFY_EVERY)
        self.steps = 0
        self._stats = torch.zeros(2, dtype=torch.float64)
        self._n_seen = 0

    @property
    def w(self) -> torch.Tensor:
        return self.params[: self.F]

    @property
    def b(self) -> torch.Tensor:
        return self.params[self.F:]

    def _workspace(self, B: int) -> torch.Tensor:
        need = self._C.train_binary_workspace(B, self.F)
        if self._ws is None or self._ws.numel() < need:
            self._ws = torch.empty(need, dtype=torch.uint8, device=self.device)
        return self._ws

    def _grad_cpu(self, X: torch.Tensor, y: torch.Tensor) -> None:
        """Same sums as the fused kernel, in float32 PyTorch (CPU path)."""
        Xf = X.float()
        z = Xf @ self.w + self.b
        g = torch.sigmoid(z) - y
        self.grad[: self.F] = Xf.T @ g
        self.grad[self.F] = g.sum()
        self.grad[self.F + 1] = (torch.clamp(z, min=0) - z * y + torch.log1p(torch.exp(-z.abs()))).sum()
        self.grad[self.F + 2] = ((z > 0) == (y > 0.5)).sum()

    @property
    def dp_exchange(self) -> str:
        """How this trainer's step reduces over ranks: ``fused-p2p`` (in-kernel, 2 launches),
        ``local`` (one replica without an exchange), ``rccl`` (unfused), ``cpu``."""
        if not self.on_gpu:
            return "cpu"
        if self._dp is not None:
            return "fused-p2p"
        return "local" if self.info.world == 1 else "rccl"

    def _fused_step(self, X: torch.Tensor, y: torch.Tensor) -> None:
        # gradient + reduce (+ in-kernel DP exchange) + update: 2 launches at any world size
        from mlapi_amd.ops.linear import _DT, _check, _stream

        _check(X, y)
        B = X.shape[0]
        ws = self._workspace(B)
        self._C.train_binary_step(_DT[X.dtype], X.data_ptr(), y.data_ptr(), self.params.data_ptr(),
                                  0 if self.mom is None else self.mom.data_ptr(), B, self.F,
                                  self.grad.data_ptr(), ws.data_ptr(), ws.numel(), float(self.lr),
                                  1.0 / (B * self.info.world), float(self.l2), float(self.momentum), _stream(),
                                  p2p=None if self._dp is None else self._dp.native, timeout_ms=self.dp_timeout_ms)

    def check(self) -> None:
        """Raise if a fused DP exchange timed out waiting for a peer (synchronises the device)."""
        if self._dp is not None:
            self._dp.check()

    def verify_replicas(self) -> bool:
        """Collective: every replica's parameter hash must match (the fused exchange keeps replicas
        bitwise identical). On a mismatch the trainer leaves the fused exchange for the RCCL
        all-reduce for good, re-syncs every replica to rank 0's parameters and records
        ``info.p2p_verify = "failed:param-hash"``. True if they agreed."""
        from mlapi_amd.parallel.p2p import replicas_agree

        if replicas_agree(self.params, self.info):
            return True
        import logging

        from mlapi_amd.parallel.comm import broadcast_

        logging.getLogger("mlapi_amd.train").warning(
            "DP replicas diverged at step %d (parameter hashes differ): fused exchange off, replicas re-synced "
            "from rank 0", self.steps)
        self._dp = None
        self.info.__dict__["p2p_verify"] = "failed:param-hash"
        broadcast_(self.params, self.info, 0)
        if self.mom is not None:
            broadcast_(self.mom, self.info, 0)
        return False

    def capture(self, X: torch.Tensor, y: torch.Tensor) -> None:
        """Capture the one-replica step for (X, y) in a HIP graph; later ``step(X, y)`` calls with
        these exact tensors replay it (one host call for the whole step - small batches are
        launch-bound). Single replica only (the all-reduce stays outside graphs)."""
        if not self.on_gpu or self.info.world != 1:
            raise RuntimeError("graph capture: single-GPU replica only (DP steps exchange per call)")
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        saved = (self.params.clone(), None if self.mom is None else self.mom.clone())
        with torch.cuda.stream(s):  # warm-up: allocates the workspace outside the capture
            self._fused_step(X, y)
        torch.cuda.current_stream().wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            self._fused_step(X, y)
        self.params.copy_(saved[0])
        if self.mom is not None:
            self.mom.copy_(saved[1])
        self._graph = (g, X, y)

    def step(self, X: torch.Tensor, y: torch.Tensor) -> None:
        B = X.shape[0]
        if self.on_gpu and self._dp is not None and self.info.world > 1:
            self._fused_step(X, y)
            self._dp.check_now()  # a missed exchange stops the loop (no silent divergence)
            self.steps += 1
            self._n_seen = B * self.info.world
            if self.verify_every > 0 and self.steps % self.verify_every == 0:
                self.verify_replicas()
            return
        if self.on_gpu and self.info.world == 1:
            g = getattr(self, "_graph", None)
            if g is not None and g[1] is X and g[2] is y:
                g[0].replay()
            else:
                self._fused_step(X, y)
            self.steps += 1
            self._n_seen = B
            return
        if self.on_gpu:
            from mlapi_amd.ops.linear import sgd_update, train_binary_grad

            train_binary_grad(X, y, self.w, self.b, ws=self._workspace(B), out=self.grad)
        else:
            self._grad_cpu(X, y)
        all_reduce_sum_(self.grad, self.info)
        n_global = B * self.info.world
        if self.on_gpu:
            sgd_update(self.params, self.grad, self.F, self.lr, 1.0 / n_global, self.l2, self.momentum, self.mom)
        else:
            d = self.grad[: self.F + 1] / n_global
            d[: self.F] += self.l2 * self.params[: self.F]
            if self.mom is not None:
                self.mom.mul_(self.momentum).add_(d)
                d = self.mom
            self.params.sub_(self.lr * d)
        self.steps += 1
        self._n_seen = n_global

    def last_loss(self) -> float:
        """Mean loss of the last step's global batch (reads back the fused buffer)."""
        self.check()
        g = self.grad.detach().cpu()
        return float(g[self.F + 1]) / max(1, self._n_seen)

    def last_accuracy(self) -> float:
        self.check()
        g = self.grad.detach().cpu()
        return float(g[self.F + 2]) / max(1, self._n_seen)

    def state_dict(self) -> dict:
        self.check()
        return {"params": self.params.detach().cpu(), "mom": None if self.mom is None else self.mom.detach().cpu(),
                "steps": self.steps}

    def load_state_dict(self, sd: dict) -> None:
        self.params.copy_(sd["params"].to(self.device))
        if self.mom is not None and sd.get("mom") is not None:
            self.mom.copy_(sd["mom"].to(self.device))
        self.steps = int(sd["steps"])

    def to_model(self, classes=(0, 1)):
        import numpy as np

        from mlapi_amd.models.linear import Kind, LinearModel

        p = self.params.detach().cpu().double().numpy()
        return LinearModel(p[None, : self.F], p[self.F:], np.asarray(classes), Kind.BINARY,
                           meta={"solver": "sgd", "n_iter_": [self.steps]})

    def evaluate(self, X: torch.Tensor, y: torch.Tensor) -> Tuple[float, float]:
        """(mean loss, accuracy) on (X, y) without updating."""
        saved = self.grad.clone()
        if self.on_gpu:
            from mlapi_amd.ops.linear import train_binary_grad

            train_binary_grad(X, y, self.w, self.b, ws=self._workspace(X.shape[0]), out=self.grad)
        else:
            self._grad_cpu(X, y)
        o = self.grad.cpu().clone()
        self.grad.copy_(saved)
        return float(o[self.F + 1]) / X.shape[0], float(o[self.F + 2]) / X.shape[0]
