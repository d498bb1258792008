"""Model parallelism for very wide linear models (SURVEY 2.5 "TP (tensor / class-sharded)" and 5.7
"wide F": the analogue of sequence/context parallelism for a model without a sequence axis).

Data parallelism (one full replica per GPU, :mod:`mlapi_amd.parallel.dp_serve`) is the default and
is what the Iris-scale reference needs: a 1000 x 256 bf16 W is 500 KiB. These two layouts are for
models whose W does not fit - or should not be replicated - e.g. extreme classification (K in the
millions) or very wide sparse-feature models (F in the hundreds of thousands):

* :class:`ClassShardedLinear` (TP over K): rank r owns classes [k0_r, k1_r). Each rank runs the MFMA
  GEMM + online-softmax epilogue on its shard (gemm_softmax MODE 4) and publishes 16 B per row -
  {max logit, sum-exp relative to it, shard-local argmax}; ONE all-gather (N x B x 16 B over xGMI)
  and a merge kernel in rank order give the exact (label, p_max) of the full model. The B x K logits
  never leave the GPU that computed them.
* :class:`FeatureShardedLinear` (split-F): rank r owns features [f0_r, f1_r) of W and receives only
  those columns of X (vertically partitioned data). Each rank computes partial logits
  X_r W_r^T (gemm_softmax MODE 1), ONE all-reduce (B x K f32) sums them, and the logits epilogue
  kernel adds the bias and applies sklearn's epilogue for the model kind.

Both reproduce :meth:`LinearModel.predict_max` (the reference's ``predict`` +
``predict_proba().max()``, `main.py:21-22`) up to bf16 GEMM rounding. Without a GPU (gloo tests),
the same collectives run over float32 PyTorch math.
"""
from __future__ import annotations

from typing import List, Optional, Tuple

import numpy as np
import torch

from mlapi_amd.models.linear import Kind, LinearModel
from mlapi_amd.parallel.comm import DistInfo, _coll_device, all_reduce_sum_

_MULTICLASS = (Kind.MULTINOMIAL, Kind.OVR)
_PIECE_F = 512  # widest exact-width gemm_softmax instantiation


def shard_bounds(n: int, world: int) -> List[Tuple[int, int]]:
    """Contiguous near-equal [lo, hi) ranges of ``n`` items over ``world`` ranks (rank order)."""
    base, extra = divmod(n, world)
    out, lo = [], 0
    for r in range(world):
        hi = lo + base + (1 if r < extra else 0)
        out.append((lo, hi))
        lo = hi
    return out


def _all_gather(t: torch.Tensor, info: DistInfo) -> torch.Tensor:
    """[world, *t.shape] on t's device (the collective runs on the comm's device)."""
    if info.world == 1:
        return t.unsqueeze(0)
    dev = _coll_device(info)
    src = t.to(dev).contiguous()
    if info.comm is not None:
        out = info.comm.all_gather(src)
    else:
        import torch.distributed as dist

        parts = [torch.empty_like(src) for _ in range(info.world)]
        dist.all_gather(parts, src)
        out = torch.stack(parts)
    return out.to(t.device)


# ------------------------------------------------------------------------ reference math (CPU path)
def rowstate_ref(Z: torch.Tensor, kind: int) -> torch.Tensor:
    """[B, K] logits -> [B, 4] {max, sum-exp rel. max (OvR: sum sigmoid), argmax, 0} in float32."""
    m, bi = Z.max(dim=1)  # torch.max returns the first maximal index
    s = torch.sigmoid(Z).sum(1) if kind == Kind.OVR else torch.exp(Z - m[:, None]).sum(1)
    return torch.stack([m, s, bi.to(Z.dtype), torch.zeros_like(m)], 1).float()


def merge_rowstates_ref(parts: torch.Tensor, offsets: List[int], kind: int) -> Tuple[torch.Tensor, torch.Tensor]:
    """[N, B, 4] shard states (rank order) -> (int32 label, float32 p_max)."""
    m = parts[..., 0].double()
    s = parts[..., 1].double()
    bi = parts[..., 2].long() + torch.as_tensor(offsets, dtype=torch.long, device=parts.device)[:, None]
    M, first = m.max(dim=0)  # first shard holding the max = lowest class index
    idx = bi.gather(0, first[None]).squeeze(0).to(torch.int32)
    if kind == Kind.OVR:
        p = torch.sigmoid(M) / s.sum(0)
    else:
        p = 1.0 / (s * torch.exp(m - M[None])).sum(0)
    return idx, p.float()


def logits_epilogue_ref(Z: torch.Tensor, b: torch.Tensor, kind: int) -> Tuple[torch.Tensor, torch.Tensor]:
    z = Z.double() + b.double()
    if kind in (Kind.BINARY, Kind.BINARY_SOFTMAX):
        z = z[:, 0]
        scale = 1.0 if kind == Kind.BINARY else 2.0
        return (z > 0).to(torch.int32), torch.sigmoid(scale * z.abs()).float()
    idx = z.argmax(1).to(torch.int32)
    if kind == Kind.OVR:
        sg = torch.sigmoid(z)
        return idx, (sg.max(1).values / sg.sum(1)).float()
    return idx, torch.softmax(z, 1).max(1).values.float()


def _on_gpu(device) -> bool:
    return device is not None and torch.device(device).type == "cuda"


# --------------------------------------------------------------------------------- class sharding
class ClassShardedLinear:
    """Rank ``info.rank``'s slice of a multiclass model's classes; ``predict`` is collective."""

    def __init__(self, model: LinearModel, info: DistInfo, device=None):
        if model.kind not in _MULTICLASS:
            raise ValueError("class sharding needs a multiclass (multinomial / OvR) model")
        self.info = info
        self.kind = int(model.kind)
        self.K, self.F = model.n_outputs, model.n_features
        self.bounds = shard_bounds(self.K, info.world)
        if min(hi - lo for lo, hi in self.bounds) < 1:
            raise ValueError(f"{self.K} classes cannot be split over {info.world} ranks")
        self.k0, self.k1 = self.bounds[info.rank]
        self.device = device if device is not None else (info.device or torch.device("cpu"))
        W = torch.as_tensor(model.W[self.k0:self.k1], dtype=torch.float32)
        b = torch.as_tensor(model.b[self.k0:self.k1], dtype=torch.float32)
        if _on_gpu(self.device):
            from mlapi_amd.ops.linear import _pad_cols

            self.W = _pad_cols(W.to(self.device).to(torch.bfloat16))  # exact-width MFMA instantiations
            self.b = b.to(self.device).contiguous()
            self._ws = None
        else:
            self.W, self.b = W, b
        self.classes = model.classes

    def local_rowstate(self, X: torch.Tensor) -> torch.Tensor:
        """[B, 4] float32 online-softmax state of this rank's classes (shard-local argmax)."""
        if not _on_gpu(self.device):
            return rowstate_ref(X.float() @ self.W.T + self.b, self.kind)
        from mlapi_amd._native import C
        from mlapi_amd.ops.linear import _check, _pad_cols, _stream

        Xb = X.to(self.device, torch.bfloat16)
        if Xb.shape[1] != self.W.shape[1]:
            Xb = _pad_cols(Xb)
        Xb = Xb.contiguous()
        B, Fp = Xb.shape
        K = self.W.shape[0]
        need = max(16, C().gemm_softmax_workspace(B, K, Fp))
        if self._ws is None or self._ws.numel() < need:
            self._ws = torch.zeros(need, dtype=torch.uint8, device=self.device)  # counters re-arm in-kernel
        out = torch.empty(B, 4, dtype=torch.float32, device=self.device)
        _check(Xb, self.W, self.b)
        C().gemm_rowstate(Xb.data_ptr(), self.W.data_ptr(), self.b.data_ptr(), B, Fp, K, self.kind, out.data_ptr(),
                          self._ws.data_ptr(), self._ws.numel(), _stream())
        return out

    def merge(self, parts: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
        """[N, B, 4] gathered states -> (global label index, p_max)."""
        offsets = [lo for lo, _ in self.bounds]
        if not _on_gpu(parts.device):
            return merge_rowstates_ref(parts, offsets, self.kind)
        from mlapi_amd._native import C
        from mlapi_amd.ops.linear import _stream

        parts = parts.contiguous()
        N, B = parts.shape[0], parts.shape[1]
        idx = torch.empty(B, dtype=torch.int32, device=parts.device)
        p = torch.empty(B, dtype=torch.float32, device=parts.device)
        C().merge_rowstates(parts.data_ptr(), N, B, offsets, self.kind, idx.data_ptr(), p.data_ptr(), _stream())
        return idx, p

    def predict(self, X: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
        """Collective: every rank passes the same X [B, F]; every rank gets (label index, p_max)."""
        return self.merge(_all_gather(self.local_rowstate(X), self.info))


# ------------------------------------------------------------------------------- feature sharding
class FeatureShardedLinear:
    """Rank ``info.rank``'s slice of the feature columns; ``predict`` is collective."""

    def __init__(self, model: LinearModel, info: DistInfo, device=None):
        self.info = info
        self.kind = int(model.kind)
        self.K, self.F = model.n_outputs, model.n_features
        self.bounds = shard_bounds(self.F, info.world)
        self.f0, self.f1 = self.bounds[info.rank]
        if self.f1 <= self.f0:
            raise ValueError(f"{self.F} features cannot be split over {info.world} ranks")
        self.device = device if device is not None else (info.device or torch.device("cpu"))
        W = torch.as_tensor(model.W[:, self.f0:self.f1], dtype=torch.float32)
        b = torch.as_tensor(model.b, dtype=torch.float32)
        if _on_gpu(self.device):
            from mlapi_amd.ops.linear import _pad_cols

            # A rank's slice wider than one MFMA tile row (512) is split-F inside the GPU too:
            # 512-column pieces, padded once here to the exact-width kernel instantiations.
            Wb = W.to(self.device).to(torch.bfloat16)
            self.pieces = [(c, min(c + _PIECE_F, Wb.shape[1])) for c in range(0, Wb.shape[1], _PIECE_F)]
            self.W = [_pad_cols(Wb[:, c0:c1]) for c0, c1 in self.pieces]
            self.zero_b = torch.zeros(self.K, dtype=torch.float32, device=self.device)
        else:
            self.W = W
        self.b = b.to(self.device)
        self.classes = model.classes

    def local_logits(self, X_local: torch.Tensor) -> torch.Tensor:
        """Partial logits [B, K] f32 of this rank's feature slice (no bias)."""
        if X_local.shape[1] != self.f1 - self.f0:
            raise ValueError(f"rank {self.info.rank} expects features [{self.f0}, {self.f1}) of X")
        if not _on_gpu(self.device):
            return X_local.float() @ self.W.T
        from mlapi_amd.ops.linear import _pad_cols, gemm_logits

        Xb = X_local.to(self.device, torch.bfloat16)
        Z = None
        for (c0, c1), Wp in zip(self.pieces, self.W):
            Xp = Xb[:, c0:c1]
            Xp = _pad_cols(Xp) if Xp.shape[1] != Wp.shape[1] else Xp.contiguous()
            Zp = gemm_logits(Xp, Wp, self.zero_b)
            Z = Zp if Z is None else Z.add_(Zp)
        return Z

    def finish(self, Z: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
        """Summed logits [B, K] -> (label index, p_max) with the model's epilogue."""
        if not _on_gpu(Z.device):
            return logits_epilogue_ref(Z, self.b, self.kind)
        from mlapi_amd._native import C
        from mlapi_amd.ops.linear import _stream

        Z = Z.contiguous()
        B = Z.shape[0]
        idx = torch.empty(B, dtype=torch.int32, device=Z.device)
        p = torch.empty(B, dtype=torch.float32, device=Z.device)
        C().logits_epilogue(Z.data_ptr(), self.b.data_ptr(), B, self.K, self.kind, idx.data_ptr(), p.data_ptr(),
                            _stream())
        return idx, p

    def predict(self, X_local: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
        """Collective: rank r passes X[:, f0_r:f1_r]; every rank gets (label index, p_max)."""
        Z = self.local_logits(X_local)
        dev = _coll_device(self.info)
        Zc = Z if Z.device == dev else Z.to(dev)
        all_reduce_sum_(Zc, self.info)
        return self.finish(Zc.to(Z.device))


def labels(classes: np.ndarray, idx: torch.Tensor) -> np.ndarray:
    return np.asarray(classes)[idx.cpu().numpy()]
