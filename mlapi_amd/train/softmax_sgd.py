"""Data-parallel mini-batch SGD for multiclass (softmax / one-vs-rest) logistic regression.

The reference fits its 3-class Iris model once with sklearn's full-batch L-BFGS
(`Logistic Regression.ipynb:33-34`); :mod:`mlapi_amd.train.lbfgs` reproduces that fit.
This module is the scale-out counterpart (BASELINE config 5 with K classes): per step and rank

  1. ``softmax_train_grad``: a row-stats MFMA launch (logsumexp / argmax per row), then one fused
     MFMA kernel that forms G = P - Y in registers and accumulates dW_aug = G^T X_aug from the same
     LDS tile of X (G never reaches HBM), with the loss / correct sums. X_aug carries a ones column
     (X_aug = [X | 0.. | 1 | 0 x 7]), so dW_aug also holds the intercept gradient. The kernel
     trains at Fk = 128 / 256 / 512 features; narrower models are zero-padded to Fk (padded
     weights get zero gradients and stay 0), so no width needs a vendor GEMM;
  2. the final slab sum of that kernel's partials exchanges [dW_aug | loss_sum | n_correct] with
     every rank in-kernel (C2 + C3 over IPC-mapped buffers on xGMI, csrc/dist/p2p_device.h; each
     block pairs with the same block of every rank, ranks summed in rank order) and applies
     W_aug = [W | b] -= lr * (g / N_global + l2 * W) (intercept unpenalized), writing the bf16 W and
     f32 b the next forward reads in the same pass.
  That is 3 launches per step at any world size; world = 1 runs the same kernels. Ranks on several
  hosts (or ``MLAPI_DP_FUSED=0``) fall back to an RCCL all-reduce of the fused buffer followed by
  ``sgd_update_2d``.

fp32 master weights; every rank applies the identical update, so replicas stay bitwise equal.
One replica (world == 1) can capture the whole step in a HIP graph (:meth:`capture`).
"""
from __future__ import annotations

from typing import Optional, Tuple

import numpy as np
import torch

from mlapi_amd.models.linear import Kind
from mlapi_amd.parallel.comm import DistInfo, all_reduce_sum_


def synthetic_multiclass(n: int, F: int, K: int, *, seed: int = 0, device=None, noise: float = 1.0):
    """Gaussian features, labels = argmax of a planted linear model + Gumbel-ish noise."""
    g = torch.Generator(device="cpu").manual_seed(seed)
    W_true = torch.randn(K, F, generator=torch.Generator().manual_seed(43)) * (2.0 / F ** 0.5)
    X = torch.randn(n, F, generator=g)
    z = X @ W_true.T + noise * torch.randn(n, K, generator=g)
    y = torch.argmax(z, dim=1).to(torch.int32)
    return X.to(device), y.to(device)


def _kernel_width(F: int) -> int:
    from mlapi_amd.ops.linear import softmax_kernel_width

    return softmax_kernel_width(F)


class SoftmaxSGDTrainer:
    """Multiclass LR trainer, one GPU per rank (or the explicit CPU path used by gloo tests)."""

    def __init__(self, n_features: int, n_classes: int, *, kind: int = Kind.MULTINOMIAL,
                 info: Optional[DistInfo] = None, lr: float = 0.1, l2: float = 0.0, momentum: float = 0.0,
                 device=None):
        if kind not in (Kind.MULTINOMIAL, Kind.OVR):
            raise ValueError("SoftmaxSGDTrainer: kind must be MULTINOMIAL or OVR (binary: BinarySGDTrainer)")
        if n_classes < 2:
            raise ValueError("need at least 2 classes")
        self.F, self.K, self.kind = int(n_features), int(n_classes), int(kind)
        self.Fk = _kernel_width(self.F)  # trained width (zero-padded features beyond F)
        self.F_aug = self.Fk + 8
        self.info = info or DistInfo(device=device)
        self.device = device if device is not None else self.info.device
        if self.device is None:
            self.device = torch.device("cpu")
        self.on_gpu = torch.device(self.device).type == "cuda"
        self.lr, self.l2, self.momentum = lr, l2, momentum
        self.params = torch.zeros(self.K, self.F_aug, dtype=torch.float32, device=self.device)
        # what the MFMA forward reads: bf16 W [K, Fk] and f32 intercepts (refreshed by every update)
        self.shadow_w = torch.zeros(self.K, self.Fk, dtype=torch.bfloat16, device=self.device) if self.on_gpu else None
        self.shadow_b = torch.zeros(self.K, dtype=torch.float32, device=self.device) if self.on_gpu else None
        n = self.K * self.F_aug
        self.grad = torch.zeros(n + 2, dtype=torch.float32, device=self.device)  # [dW_aug | loss | correct]
        self.mom = torch.zeros_like(self.params) if momentum else None
        self._bufs = {}  # batch size -> SoftmaxTrainBuffers (a ragged last batch keeps its own)
        self._graph = None
        self._dp = None
        if self.on_gpu:
            from mlapi_amd.parallel.p2p import dp_exchange

            # gradient slice + stats, then (two-shot exchange) the published [grad | params | momenta]
            self._dp = dp_exchange(self.info, (4 * n + 16) * 4, width=n)
        self.dp_timeout_ms = 60_000
        from mlapi_amd.parallel.p2p import verify_every

        self.verify_every = verify_every()  # fused steps between replica checks (MLAPI_DP_VERIFY_EVERY)
        self.steps = 0
        self._n_seen = 0

    # ---------------------------------------------------------------------------------- data
    def prepare(self, X: torch.Tensor) -> torch.Tensor:
        """Augmented features [X | 1 | 0...] (bf16 on GPU, f32 on CPU); build once per dataset."""
        from mlapi_amd.ops.linear import augment_features

        Xa = augment_features(X.to(self.device), self.F_aug)
        return Xa if self.on_gpu else Xa.float()

    @property
    def W(self) -> torch.Tensor:
        return self.params[:, : self.F]

    @property
    def b(self) -> torch.Tensor:
        return self.params[:, self.Fk]

    def _dW(self) -> torch.Tensor:
        return self.grad[: self.K * self.F_aug].view(self.K, self.F_aug)

    def set_params(self, W: torch.Tensor, b: torch.Tensor) -> None:
        self.params.zero_()
        self.params[:, : self.F] = W.to(self.params)
        self.params[:, self.Fk] = b.reshape(-1).to(self.params)
        self._refresh_shadow()

    def _refresh_shadow(self) -> None:
        if self.shadow_w is not None:
            self.shadow_w.copy_(self.params[:, : self.Fk])
            self.shadow_b.copy_(self.params[:, self.Fk])

    # ---------------------------------------------------------------------------------- step
    @property
    def dp_exchange(self) -> str:
        if not self.on_gpu:
            return "cpu"
        if self._dp is not None:
            return "fused-p2p"
        return "local" if self.info.world == 1 else "rccl"

    def check(self) -> None:
        """Raise if a fused DP exchange timed out waiting for a peer (synchronises the device)."""
        if self._dp is not None:
            self._dp.check()

    def verify_replicas(self) -> bool:
        """Collective: every replica's parameter hash must match (the fused exchange keeps replicas
        bitwise identical). On a mismatch the trainer leaves the fused exchange for the RCCL
        all-reduce for good, re-syncs every replica to rank 0's parameters (and its bf16 / f32
        shadows) and records ``info.p2p_verify = "failed:param-hash"``. True if they agreed."""
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
        self._refresh_shadow()
        return False

    def _local_grad(self, Xa: torch.Tensor, y: torch.Tensor, fused_update_n: int = 0, dp=None) -> None:
        """Gradient sums into self.grad; with ``fused_update_n`` the SGD update for that global
        batch size runs inside the gradient's final slab sum, after the in-kernel DP exchange when
        ``dp`` is given (then self.grad holds the global sums)."""
        if self.on_gpu:
            from mlapi_amd.ops.linear import SoftmaxTrainBuffers, softmax_train_grad

            B = Xa.shape[0]
            if B not in self._bufs:
                self._bufs[B] = SoftmaxTrainBuffers(B, self.K, self.Fk, Xa.device)
            upd = None
            if fused_update_n:
                upd = dict(params=self.params, lr=self.lr, inv_n=1.0 / fused_update_n, l2=self.l2,
                           momentum=self.momentum, mom_buf=self.mom, shadow_w=self.shadow_w, shadow_b=self.shadow_b)
            softmax_train_grad(Xa, self.shadow_w, self.shadow_b, y, self.kind, bufs=self._bufs[B], dW_out=self._dW(),
                               stats_out=self.grad[self.K * self.F_aug:], update=upd, p2p=dp,
                               timeout_ms=self.dp_timeout_ms)
        else:
            from mlapi_amd.ops.reference import softmax_train_ref

            _, dW, loss, correct = softmax_train_ref(Xa, y, self.params, self.kind)
            self._dW().copy_(dW)
            self.grad[-2] = loss
            self.grad[-1] = correct

    def _update(self, n_global: int) -> None:
        if self.on_gpu:
            from mlapi_amd.ops.linear import sgd_update_2d

            sgd_update_2d(self.params, self.grad, self.Fk, self.lr, 1.0 / n_global, self.l2, self.momentum, self.mom,
                          self.shadow_w, self.shadow_b)
        else:
            d = self._dW() / n_global
            d[:, : self.Fk] += self.l2 * self.params[:, : self.Fk]
            if self.mom is not None:
                self.mom.mul_(self.momentum).add_(d)
                d = self.mom
            self.params.sub_(self.lr * d)

    def step(self, Xa: torch.Tensor, y: torch.Tensor) -> None:
        """One SGD step on this rank's shard (Xa from :meth:`prepare`, y int32 class indices)."""
        if self._graph is not None and self._graph[1] is Xa and self._graph[2] is y:
            self._graph[0].replay()
        elif self.on_gpu and (self._dp is not None or self.info.world == 1):
            self._local_grad(Xa, y, fused_update_n=Xa.shape[0] * self.info.world, dp=self._dp)
            if self._dp is not None:
                self._dp.check_now()  # a missed exchange stops the loop (no silent divergence)
                if self.verify_every > 0 and (self.steps + 1) % self.verify_every == 0:
                    self.verify_replicas()
        else:
            self._local_grad(Xa, y)
            all_reduce_sum_(self.grad, self.info)
            self._update(Xa.shape[0] * self.info.world)
        self.steps += 1
        self._n_seen = Xa.shape[0] * self.info.world

    def capture(self, Xa: torch.Tensor, y: torch.Tensor) -> None:
        """Capture one whole step (row stats + fused gradient + slab sums + update) in a HIP graph.

        Later ``step(Xa, y)`` calls with these exact tensors replay it: one launch from the host.
        Single replica only (the all-reduce stays outside graphs)."""
        if not self.on_gpu or self.info.world != 1:
            raise RuntimeError("graph capture: single-GPU replica only")
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        saved = (self.params.clone(), None if self.mom is None else self.mom.clone())
        with torch.cuda.stream(s):  # warm-up: allocates the buffers
            for _ in range(2):
                self._local_grad(Xa, y, fused_update_n=Xa.shape[0], dp=self._dp)
        torch.cuda.current_stream().wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            self._local_grad(Xa, y, fused_update_n=Xa.shape[0], dp=self._dp)
        self.params.copy_(saved[0])
        self._refresh_shadow()
        if self.mom is not None:
            self.mom.copy_(saved[1])
        self._graph = (g, Xa, y)

    # ---------------------------------------------------------------------------------- stats
    def last_loss(self) -> float:
        self.check()
        return float(self.grad[-2].item()) / max(1, self._n_seen)

    def last_accuracy(self) -> float:
        self.check()
        return float(self.grad[-1].item()) / max(1, self._n_seen)

    def evaluate(self, Xa: torch.Tensor, y: torch.Tensor) -> Tuple[float, float]:
        saved = self.grad.clone()
        self._local_grad(Xa, y)
        o = self.grad[-2:].cpu().clone()
        self.grad.copy_(saved)
        return float(o[0]) / Xa.shape[0], float(o[1]) / Xa.shape[0]

    def state_dict(self) -> dict:
        self.check()
        return {"params": self.params.detach().cpu(), "mom": None if self.mom is None else self.mom.detach().cpu(),
                "steps": self.steps}

    def load_state_dict(self, sd: dict) -> None:
        self.params.copy_(sd["params"].to(self.device))
        self._refresh_shadow()
        if self.mom is not None and sd.get("mom") is not None:
            self.mom.copy_(sd["mom"].to(self.device))
        self.steps = int(sd["steps"])

    def to_model(self, classes=None):
        from mlapi_amd.models.linear import LinearModel

        p = self.params.detach().cpu().double().numpy()
        classes = np.arange(self.K) if classes is None else np.asarray(classes)
        return LinearModel(p[:, : self.F].copy(), p[:, self.Fk].copy(), classes, Kind(self.kind),
                           meta={"solver": "sgd", "n_iter_": [self.steps]})
