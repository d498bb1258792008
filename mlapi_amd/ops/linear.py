"""torch-facing wrappers of the HIP kernels (csrc/kernels/*.hip).

Every op takes device tensors and launches on ``torch.cuda.current_stream()``; there is no
silent CPU / PyTorch fallback: a CPU tensor or a missing extension raises. Pure-PyTorch oracles
for tests live in :mod:`mlapi_amd.ops.reference`.

Dispatch for ``predict`` (the reference's ``predict`` + ``predict_proba().max()``,
`main.py:21-22`):
  * f64 / f32 inputs with small F, K  -> ``linear_small`` (fused, one row per lane);
  * binary (K == 1) bf16 / f32        -> ``gemv_binary`` (HBM-streaming GEMV + sigmoid);
  * multiclass bf16                   -> ``gemm_softmax`` (MFMA + online softmax/argmax; any F:
                                         the row-group kernel loops wide F in 256-feature slices).
"""
from __future__ import annotations

import os
from typing import Tuple

import torch

from mlapi_amd._native import C
from mlapi_amd.models.linear import Kind

_DT = {torch.float64: 0, torch.float32: 1, torch.bfloat16: 2}


def _stream() -> int:
    return torch.cuda.current_stream().cuda_stream


def _check(*ts: torch.Tensor) -> None:
    for t in ts:
        if not isinstance(t, torch.Tensor) or not t.is_cuda:
            raise ValueError("mlapi_amd.ops: inputs must be GPU tensors (no CPU fallback)")
        if not t.is_contiguous():
            raise ValueError("mlapi_amd.ops: inputs must be contiguous")


def linear_small(X: torch.Tensor, W: torch.Tensor, b: torch.Tensor, kind: int) -> Tuple[torch.Tensor, torch.Tensor]:
    """Fused z = X W^T + b -> (int32 label index, p_max) in X's dtype (f64 or f32)."""
    _check(X, W, b)
    if X.dtype not in (torch.float64, torch.float32) or W.dtype != X.dtype or b.dtype != X.dtype:
        raise TypeError("linear_small: X, W, b must share dtype f64 or f32")
    B, F = X.shape
    K = W.shape[0]
    if W.shape[1] != F or b.numel() != K:
        raise ValueError("linear_small: shape mismatch")
    idx = torch.empty(B, dtype=torch.int32, device=X.device)
    p = torch.empty(B, dtype=X.dtype, device=X.device)
    C().linear_small(_DT[X.dtype], X.data_ptr(), F, W.data_ptr(), b.data_ptr(), B, F, K, int(kind), idx.data_ptr(),
                     p.data_ptr(), _stream())
    return idx, p


def gemv_binary(X: torch.Tensor, w: torch.Tensor, bias: float, kind: int = Kind.BINARY, out=None):
    """Binary LR over a large batch: (int32 z>0, f32 sigmoid(|z|)). X: [B, F] bf16/f32.
    ``out=(idx, p)`` writes into preallocated outputs (graph-capture safe)."""
    _check(X, w)
    if X.dtype not in (torch.bfloat16, torch.float32) or w.dtype != X.dtype:
        raise TypeError("gemv_binary: X and w must share dtype bf16 or f32")
    B, F = X.shape
    if w.numel() != F:
        raise ValueError("gemv_binary: w must have F entries")
    if out is None:
        out = (torch.empty(B, dtype=torch.int32, device=X.device), torch.empty(B, dtype=torch.float32, device=X.device))
    idx, p = out
    C().gemv_binary(_DT[X.dtype], X.data_ptr(), w.data_ptr(), float(bias), B, F, int(kind), idx.data_ptr(),
                    p.data_ptr(), _stream())
    return idx, p


def gemm_width(F: int) -> int:
    """Feature width the multiclass kernels run at: a power of two >= 32 up to 256, else a multiple
    of 256 (wider models loop F in 256-feature slices inside one launch; zero columns add nothing)."""
    F = int(F)
    if F <= 256:
        return max(32, 1 << (F - 1).bit_length())
    return (F + 255) // 256 * 256


def _pad_cols(t: torch.Tensor) -> torch.Tensor:
    F = t.shape[1]
    Fp = gemm_width(F)
    return t.contiguous() if Fp == F else torch.nn.functional.pad(t, (0, Fp - F)).contiguous()


class GemmSoftmax:
    """Multiclass predict with a cached workspace (capture-safe launches after construction)."""

    def __init__(self, max_batch: int, n_classes: int, n_features: int, device):
        self.max_batch, self.K, self.F = max_batch, n_classes, n_features
        nbytes = C().gemm_softmax_workspace(max_batch, n_classes, n_features)
        # zero-initialised once: the in-kernel split merge publishes tagged state granules here and
        # the merging block clears the tags it consumed, so graph replays (one baked tag) stay exact.
        self.ws = torch.zeros(max(nbytes, 16), dtype=torch.uint8, device=device)

    def __call__(self, X, W, b, kind: int = Kind.MULTINOMIAL, out=None):
        _check(X, W, b)
        if X.dtype != torch.bfloat16 or W.dtype != torch.bfloat16 or b.dtype != torch.float32:
            raise TypeError("gemm_softmax: X, W bf16 and b f32")
        B, F = X.shape
        K = W.shape[0]
        if W.shape[1] != F or b.numel() != K:
            raise ValueError("gemm_softmax: W must be [K, F] and b [K]")
        if gemm_width(F) != F:  # kernels are instantiated for exact widths: zero-pad the rest
            X, W = _pad_cols(X), _pad_cols(W)
            F = X.shape[1]
        need = C().gemm_softmax_workspace(B, K, F)
        if need > self.ws.numel():
            self.ws = torch.zeros(need, dtype=torch.uint8, device=X.device)
        if out is None:
            out = (torch.empty(B, dtype=torch.int32, device=X.device), torch.empty(B, dtype=torch.float32, device=X.device))
        idx, p = out
        C().gemm_softmax(X.data_ptr(), W.data_ptr(), b.data_ptr(), B, F, K, int(kind), idx.data_ptr(), p.data_ptr(),
                         self.ws.data_ptr(), self.ws.numel(), _stream())
        return idx, p

    def xcd_errors(self) -> int:
        """Bit mask of XCDs whose merging block read a partial written on another XCD (or never saw
        one) during an XCD-local split merge (gemm_softmax.hip, granule_merge); 0 while every merge
        stayed in one L2."""
        o = C().gemm_softmax_xcd_err_offset()
        if self.ws.numel() < o + 4:
            return 0  # no split plan has run: nothing was checked
        return int(self.ws[o:o + 4].view(torch.int32).item())


class LinearSplit:
    """Class-split multiclass predict (csrc/kernels/linear_split.h): small batches (one launch,
    one cross-block merge round trip) and f32 models via v_mfma_f32_16x16x4_f32. X, W share dtype
    bf16 or f32; F a power of two (bf16 32..512, f32 16..512; narrower models are zero-padded)."""

    def __init__(self, max_batch: int, n_classes: int, device):
        self.max_batch, self.K = max_batch, n_classes
        self.ws = torch.zeros(C().linear_split_workspace(max_batch, n_classes), dtype=torch.uint8, device=device)

    def __call__(self, X, W, b, kind: int = Kind.MULTINOMIAL, out=None):
        _check(X, W, b)
        if X.dtype not in (torch.bfloat16, torch.float32) or W.dtype != X.dtype or b.dtype != torch.float32:
            raise TypeError("linear_split: X, W bf16 or f32 (same dtype), b f32")
        B, F = X.shape
        K = W.shape[0]
        if W.shape[1] != F or b.numel() != K or K != self.K:
            raise ValueError("linear_split: W must be [K, F] and b [K]")
        if not C().linear_split_supported(_DT[X.dtype], F):
            Fp = max(16 if X.dtype == torch.float32 else 32, 1 << (F - 1).bit_length())
            X = torch.nn.functional.pad(X, (0, Fp - F)).contiguous()
            W = torch.nn.functional.pad(W, (0, Fp - F)).contiguous()
            F = Fp
        need = C().linear_split_workspace(B, K)
        if need > self.ws.numel():
            self.ws = torch.zeros(need, dtype=torch.uint8, device=X.device)
        if out is None:
            out = (torch.empty(B, dtype=torch.int32, device=X.device), torch.empty(B, dtype=torch.float32, device=X.device))
        idx, p = out
        C().linear_split(_DT[X.dtype], X.data_ptr(), F, W.data_ptr(), b.data_ptr(), B, F, K, int(kind), idx.data_ptr(),
                         p.data_ptr(), self.ws.data_ptr(), self.ws.numel(), _stream())
        return idx, p

    def xcd_errors(self) -> int:
        """Bit mask of XCDs whose merging block read a partial written on another XCD (XCD-local
        merge); 0 while the splits of every row group met in one XCD's L2."""
        o = C().linear_split_xcd_err_offset()
        return int(self.ws[o:o + 4].view(torch.int32).item())


def linear_split(X, W, b, kind: int = Kind.MULTINOMIAL):
    return LinearSplit(X.shape[0], W.shape[0], X.device)(X, W, b, kind)


class LinearWide:
    """Wide-model predict with float64 accumulation on the matrix cores
    (csrc/kernels/linear_wide.h, v_mfma_f64_16x16x4_f64): X, W stored as f64 or f32 (same
    dtype), b f64; any F (zero-padded here to the plan's width), any K, every kind (binary kinds:
    W is [1, F]). Returns (int32 label index, f64 p_max). A row whose in-kernel class merge gave up
    waiting (1 s: a class block never ran - not expected, the launch's blocks are dispatched in
    order) comes back as index WIDE_TIMEOUT_IDX (-3) and p NaN; :meth:`failed` counts them (it
    synchronises). HIP-graph capture is safe: the merging block clears the tags of the granules it
    consumed, so replays (one epoch baked into the graph) never see the previous replay's states."""

    WIDE_TIMEOUT_IDX = -3

    @staticmethod
    def failed(idx: torch.Tensor) -> int:
        return int((idx < 0).sum().item())

    def __init__(self, max_batch: int, n_features: int, n_classes: int, dtype: torch.dtype, device):
        self.dt = _DT[dtype]
        self.plan = C().linear_wide_plan(self.dt, n_features, n_classes)
        self.ws = torch.zeros(max(256, C().linear_wide_workspace(max_batch, self.dt, n_features, n_classes)),
                              dtype=torch.uint8, device=device)

    def __call__(self, X, W, b, kind: int = Kind.MULTINOMIAL, out=None):
        _check(X, W, b)
        if X.dtype not in (torch.float64, torch.float32) or W.dtype != X.dtype or b.dtype != torch.float64:
            raise TypeError("linear_wide: X, W f64 or f32 (same dtype), b f64")
        B, F = X.shape
        K = W.shape[0]
        if W.shape[1] != F or b.numel() != K:
            raise ValueError("linear_wide: W must be [K, F] and b [K]")
        ld = self.plan["ldx"]
        if ld != F:
            X = torch.nn.functional.pad(X, (0, ld - F)).contiguous()
            W = torch.nn.functional.pad(W, (0, ld - F)).contiguous()
        need = C().linear_wide_workspace(B, self.dt, F, K)
        if need > self.ws.numel():
            self.ws = torch.zeros(need, dtype=torch.uint8, device=X.device)
        if out is None:
            out = (torch.empty(B, dtype=torch.int32, device=X.device), torch.empty(B, dtype=torch.float64, device=X.device))
        idx, p = out
        C().linear_wide(self.dt, X.data_ptr(), ld, W.data_ptr(), b.data_ptr(), B, F, K, int(kind), idx.data_ptr(),
                        p.data_ptr(), self.ws.data_ptr(), self.ws.numel(), _stream())
        return idx, p


def linear_wide(X, W, b, kind: int = Kind.MULTINOMIAL):
    return LinearWide(X.shape[0], X.shape[1], W.shape[0], X.dtype, X.device)(X, W, b, kind)


def gemm_softmax(X, W, b, kind: int = Kind.MULTINOMIAL):
    return GemmSoftmax(X.shape[0], W.shape[0], X.shape[1], X.device)(X, W, b, kind)


def gemm_logits(X, W, b) -> torch.Tensor:
    _check(X, W, b)
    if gemm_width(X.shape[1]) != X.shape[1]:
        X, W = _pad_cols(X), _pad_cols(W)
    B, F = X.shape
    K = W.shape[0]
    Z = torch.empty(B, K, dtype=torch.float32, device=X.device)
    C().gemm_logits(X.data_ptr(), W.data_ptr(), b.data_ptr(), B, F, K, Z.data_ptr(), _stream())
    return Z


def predict(X: torch.Tensor, W: torch.Tensor, b: torch.Tensor, kind: int):
    """Dispatching predict: returns (int32 index, p_max)."""
    K, F = W.shape
    if X.dtype in (torch.float64,) or (X.dtype == torch.float32 and F <= 32 and K <= 16):
        return linear_small(X, W.to(X.dtype).contiguous(), b.to(X.dtype).contiguous(), kind)
    if K == 1:
        return gemv_binary(X, W.reshape(-1).to(X.dtype).contiguous(), float(b.reshape(-1)[0]), kind)
    return gemm_softmax(X.to(torch.bfloat16).contiguous(), W.to(torch.bfloat16).contiguous(),
                        b.to(torch.float32).contiguous(), kind)


# ------------------------------------------------------------------------------------------ train
def train_binary_grad(X: torch.Tensor, y: torch.Tensor, w: torch.Tensor, b: torch.Tensor, ws: torch.Tensor = None,
                      out: torch.Tensor = None) -> torch.Tensor:
    """Sums over the batch: out = [dL/dw (F) | dL/db | loss_sum | n_correct] (f32)."""
    _check(X, y, w, b)
    B, F = X.shape
    if ws is None:
        ws = torch.empty(C().train_binary_workspace(B, F), dtype=torch.uint8, device=X.device)
    if out is None:
        out = torch.empty(F + 3, dtype=torch.float32, device=X.device)
    C().train_binary_grad(_DT[X.dtype], X.data_ptr(), y.data_ptr(), w.data_ptr(), b.data_ptr(), B, F, out.data_ptr(),
                          ws.data_ptr(), ws.numel(), _stream())
    return out


def train_small_grad(X: torch.Tensor, y: torch.Tensor, W: torch.Tensor, b: torch.Tensor, kind: int,
                     ws: torch.Tensor = None, out: torch.Tensor = None) -> torch.Tensor:
    """out = [dL/dW (K*F row-major) | dL/db (K) | loss_sum | n_correct] in X's dtype (f64/f32)."""
    _check(X, y, W, b)
    B, F = X.shape
    K = W.shape[0]
    if ws is None:
        ws = torch.empty(C().train_small_workspace(B, F, K), dtype=torch.uint8, device=X.device)
    if out is None:
        out = torch.empty(K * F + K + 2, dtype=X.dtype, device=X.device)
    C().train_small_grad(_DT[X.dtype], X.data_ptr(), y.data_ptr(), W.data_ptr(), b.data_ptr(), B, F, K, int(kind),
                         out.data_ptr(), ws.data_ptr(), ws.numel(), _stream())
    return out


def sgd_update(params: torch.Tensor, grad: torch.Tensor, n_penalized: int, lr: float, inv_n: float, l2: float,
               momentum: float = 0.0, mom_buf: torch.Tensor = None) -> None:
    _check(params, grad)
    C().sgd_update(params.data_ptr(), grad.data_ptr(), 0 if mom_buf is None else mom_buf.data_ptr(), params.numel(),
                   n_penalized, float(lr), float(inv_n), float(l2), float(momentum), _stream())


def cast(src: torch.Tensor, dtype: torch.dtype) -> torch.Tensor:
    _check(src)
    dst = torch.empty(src.shape, dtype=dtype, device=src.device)
    C().cast(_DT[src.dtype], src.data_ptr(), _DT[dtype], dst.data_ptr(), src.numel(), _stream())
    return dst


# ------------------------------------------------------------------- multiclass training (MFMA)
SOFTMAX_TRAIN_WIDTHS = (128, 256, 512)


def softmax_kernel_width(F: int) -> int:
    """Feature width the multiclass training kernels run at: F rounded up to 128 / 256 / 512 (the
    fused gradient kernel), or to a multiple of 256 above 512 (softmax_grad_wide.hip).

    Narrower models are zero-padded: padded columns of X are 0, so their weights get a zero
    gradient (and a zero L2 / momentum term) and stay exactly 0 - the trained model is the same."""
    for w in SOFTMAX_TRAIN_WIDTHS:
        if int(F) <= w:
            return w
    return (int(F) + 255) // 256 * 256


def softmax_train_faug(F: int) -> int:
    """Width F_aug = Fk + 8 of the augmented features [X | 0.. | 1 | 0 x 7] (and of W_aug = [W | 0.. | b | 0]),
    with Fk = :func:`softmax_kernel_width` (F)."""
    return softmax_kernel_width(F) + 8


def xaug_row_stride(F_aug: int) -> int:
    """Row stride (elements) of an augmented feature matrix: padded to a multiple of 64 bf16 = 128
    bytes, so every row starts on a cache line. Unpadded (F_aug = Fk + 8) a row starts 16 bytes
    further into its line each time, and the kernels' row segments straddle one line more
    (the F = 1024 G^T X launch: 197.5 -> 182.8 us padded; MLAPI_XAUG_PAD=0: unpadded)."""
    if os.environ.get("MLAPI_XAUG_PAD", "1") != "0":
        return (F_aug + 63) // 64 * 64
    return F_aug


def augment_features(X: torch.Tensor, F_aug: int) -> torch.Tensor:
    """[X | 0.. | 1 | 0...] in bf16, shape [B, F_aug], the ones column at F_aug - 8 (done once per
    dataset, not per step), as a row-padded view (:func:`xaug_row_stride`)."""
    B, F = X.shape
    ld = xaug_row_stride(F_aug)
    out = torch.zeros(B, ld, dtype=torch.bfloat16, device=X.device)[:, :F_aug]
    out[:, :F] = X
    out[:, F_aug - 8] = 1.0
    return out


def augment_weights(W: torch.Tensor, b: torch.Tensor, F_aug: int) -> torch.Tensor:
    """[W | 0.. | b | 0...] in f32, shape [K, F_aug], the intercept at column F_aug - 8."""
    K, F = W.shape
    out = torch.zeros(K, F_aug, dtype=torch.float32, device=W.device)
    out[:, :F] = W
    out[:, F_aug - 8] = b.reshape(-1)
    return out


class SoftmaxTrainBuffers:
    """Persistent per-batch-size workspace of the fused multiclass gradient."""

    def __init__(self, B: int, K: int, F: int, device):
        self.B, self.K, self.F = B, K, F
        self.wide = C().softmax_grad_wide_supported(F)
        if not (self.wide or C().softmax_grad_dw_supported(F)):
            raise ValueError(f"training kernel width must be one of {SOFTMAX_TRAIN_WIDTHS} or a multiple of 256 "
                             f"above 512 (got {F})")
        self.stats = torch.zeros(2, dtype=torch.float32, device=device)
        nbytes = (C().softmax_grad_wide_workspace(B, K, F) if self.wide else C().softmax_grad_dw_workspace(B, K, F))
        self.ws = torch.zeros(nbytes, dtype=torch.uint8, device=device)


def softmax_train_grad(X_aug: torch.Tensor, W: torch.Tensor, b: torch.Tensor, y: torch.Tensor, kind: int,
                       bufs: SoftmaxTrainBuffers = None, dW_out: torch.Tensor = None,
                       stats_out: torch.Tensor = None, update: dict = None, p2p=None, timeout_ms: int = 60000):
    """Sums over the batch of the multiclass objective's gradient, intercept included.

    X_aug: [B, Fk + 8] bf16 from :func:`augment_features`; W: [K, Fk] bf16 (Fk in 128/256/512;
    zero-pad narrower models); b: [K] f32; y: int32. Returns (dW_aug f32 [K, Fk + 8] with the
    intercept gradient in column Fk, stats f32 [loss_sum, n_correct]). Two HIP launches and no
    vendor GEMM: a row-stats pass (logsumexp / argmax per row, gemm_softmax.hip MODE 2), then
    softmax_grad_dw.hip, which forms G = P - Y in registers and accumulates dW_aug = G^T X_aug from
    the same LDS tile (G never reaches HBM), followed by its deterministic slab sums.

    ``update``: the SGD step :func:`sgd_update_2d` would apply next, fused into the final slab sum -
    keys params [K, Fk + 8] f32, lr, inv_n (1 / global batch), l2, and optionally momentum, mom_buf,
    shadow_w, shadow_b. ``p2p`` (a :class:`mlapi_amd.parallel.p2p.P2PAllReduce`): the data-parallel
    all-reduce of [dW_aug | loss | correct] runs inside that final slab sum too (p2p_device.h), so
    a DP step stays 3 launches at any world size.
    """
    _check(W, b, y)
    if not isinstance(X_aug, torch.Tensor) or not X_aug.is_cuda:
        raise ValueError("mlapi_amd.ops: inputs must be GPU tensors (no CPU fallback)")
    if X_aug.dtype != torch.bfloat16 or W.dtype != torch.bfloat16 or b.dtype != torch.float32 \
            or y.dtype != torch.int32:
        raise TypeError("softmax_train_grad: X_aug, W bf16, b f32 and y int32")
    B, F_aug = X_aug.shape
    K, F = W.shape
    # rows may be padded (augment_features): unit column stride, row stride a multiple of 8
    # elements (16-byte aligned rows)
    ldx = X_aug.stride(0) if B > 0 else F_aug
    if X_aug.stride(1) != 1 or ldx < F_aug or ldx % 8 != 0:
        raise ValueError("mlapi_amd.ops: X_aug rows must be contiguous with a row stride >= F_aug, a "
                         "multiple of 8")
    if (F not in SOFTMAX_TRAIN_WIDTHS and not C().softmax_grad_wide_supported(F)) or F_aug != F + 8 \
            or b.numel() != K or y.numel() != B:
        raise ValueError("softmax_train_grad: shape mismatch (W must be [K, Fk], Fk in 128/256/512 or a multiple "
                         "of 256 above 512, X_aug [B, Fk + 8])")
    if bufs is None or bufs.B != B or bufs.K != K or bufs.F != F:
        bufs = SoftmaxTrainBuffers(B, K, F, X_aug.device)
    stats = bufs.stats if stats_out is None else stats_out
    if dW_out is None:
        dW_out = torch.empty(K, F_aug, dtype=torch.float32, device=X_aug.device)
    if not dW_out.is_contiguous() or dW_out.shape != (K, F_aug) or dW_out.dtype != torch.float32:
        raise ValueError("softmax_train_grad: dW_out must be a contiguous f32 [K, Fk + 8] tensor")
    upd = {}
    if update is not None:
        p = update["params"]
        if not p.is_contiguous() or p.shape != (K, F_aug) or p.dtype != torch.float32:
            raise ValueError("softmax_train_grad: update params must be a contiguous f32 [K, Fk + 8] tensor")
        ptr = lambda t: 0 if t is None else t.data_ptr()  # noqa: E731
        upd = dict(params=p.data_ptr(), mom=ptr(update.get("mom_buf")), shadow_w=ptr(update.get("shadow_w")),
                   shadow_b=ptr(update.get("shadow_b")), pen_cols=F, lr=float(update["lr"]),
                   inv_n=float(update["inv_n"]), l2=float(update.get("l2", 0.0)),
                   momentum=float(update.get("momentum", 0.0)))
    launch = C().softmax_grad_wide if bufs.wide else C().softmax_grad_dw  # F > 512: softmax_grad_wide.hip
    launch(X_aug.data_ptr(), ldx, W.data_ptr(), b.data_ptr(), y.data_ptr(), B, F, K, int(kind),
           dW_out.data_ptr(), stats.data_ptr(), bufs.ws.data_ptr(), bufs.ws.numel(), _stream(), **upd,
           p2p=None if p2p is None else p2p.native, timeout_ms=int(timeout_ms))
    return dW_out, stats


def sgd_update_2d(params: torch.Tensor, grad: torch.Tensor, pen_cols: int, lr: float, inv_n: float, l2: float,
                  momentum: float = 0.0, mom_buf: torch.Tensor = None, shadow_w: torch.Tensor = None,
                  shadow_b: torch.Tensor = None) -> None:
    """params [rows, cols] f32 -= lr * (grad / N + l2 * params[:, :pen_cols]); refreshes the bf16
    weight copy shadow_w [rows, pen_cols] and the f32 bias copy shadow_b (column pen_cols)."""
    _check(params, grad)
    rows, cols = params.shape
    C().sgd_update_2d(params.data_ptr(), grad.data_ptr(), 0 if mom_buf is None else mom_buf.data_ptr(), rows, cols,
                      int(pen_cols), float(lr), float(inv_n), float(l2), float(momentum),
                      0 if shadow_w is None else shadow_w.data_ptr(), 0 if shadow_b is None else shadow_b.data_ptr(),
                      _stream())
