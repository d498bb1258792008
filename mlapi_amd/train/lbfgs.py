"""Full-batch L-BFGS fit that reproduces sklearn's ``LogisticRegression().fit`` (solver 'lbfgs').

The reference's training step is ``LogisticRegression().fit(X_train, y_train)``
(`Logistic Regression.ipynb:33-34`): scipy L-BFGS-B on
    mean_i loss_i + (1 / (2 C N)) ||W||^2          (intercept unpenalized)
with loss = half-multinomial (K > 2) or half-binomial (K = 2), options maxiter=max_iter,
maxls=50, gtol=tol, ftol=64 eps, parameters laid out (K, F+1) in Fortran order (sklearn
_logistic.py). We run the same optimizer on the same objective; only the loss+gradient
evaluation differs: it is the fused fp64 HIP kernel ``train_small_grad`` on a GPU (X stays
resident on the device), or the identical float64 math in numpy on a CPU.
"""
from __future__ import annotations

from typing import Callable, Optional, Tuple

import numpy as np

from mlapi_amd.models.linear import Kind, LinearModel


def _numpy_grad(X: np.ndarray, yi: np.ndarray, kind: Kind) -> Callable:
    def fn(W: np.ndarray, b: np.ndarray) -> Tuple[np.ndarray, np.ndarray, float]:
        z = X @ W.T + b
        if kind == Kind.BINARY:
            zz = z[:, 0]
            y = yi.astype(np.float64)
            g = (1.0 / (1.0 + np.exp(-zz)) - y)[:, None]
            loss = np.sum(np.maximum(zz, 0) - zz * y + np.log1p(np.exp(-np.abs(zz))))
        else:
            m = z.max(axis=1, keepdims=True)
            e = np.exp(z - m)
            s = e.sum(axis=1, keepdims=True)
            g = e / s
            g[np.arange(len(yi)), yi] -= 1.0
            loss = np.sum(m[:, 0] + np.log(s[:, 0]) - z[np.arange(len(yi)), yi])
        return g.T @ X, g.sum(axis=0), float(loss)

    return fn


def _gpu_grad(X: np.ndarray, yi: np.ndarray, kind: Kind, device) -> Callable:
    import torch

    from mlapi_amd._native import C
    from mlapi_amd.ops.linear import train_small_grad

    Xd = torch.as_tensor(X, dtype=torch.float64, device=device).contiguous()
    yd = torch.as_tensor(yi, dtype=torch.int32, device=device)
    N, F = X.shape
    K = 1 if kind == Kind.BINARY else int(yi.max()) + 1
    ws = torch.empty(C().train_small_workspace(N, F, K), dtype=torch.uint8, device=device)
    out = torch.empty(K * F + K + 2, dtype=torch.float64, device=device)
    Wd = torch.empty(K, F, dtype=torch.float64, device=device)
    bd = torch.empty(K, dtype=torch.float64, device=device)

    def fn(W: np.ndarray, b: np.ndarray):
        Wd.copy_(torch.from_numpy(np.ascontiguousarray(W)))
        bd.copy_(torch.from_numpy(np.ascontiguousarray(b)))
        train_small_grad(Xd, yd, Wd, bd, int(kind), ws=ws, out=out)
        o = out.cpu().numpy()
        return o[: K * F].reshape(K, F), o[K * F: K * F + K], float(o[K * F + K])

    return fn


def _minimize(grad_fn: Callable, rows: int, F: int, N: int, C: float, max_iter: int, tol: float):
    from scipy import optimize

    l2 = 1.0 / (C * N)

    def fun(w):
        Wf = w.reshape((rows, F + 1), order="F")
        W, b = Wf[:, :F], Wf[:, F]
        gW, gb, loss = grad_fn(W, b)
        f = loss / N + 0.5 * l2 * float(np.sum(W * W))
        g = np.empty((rows, F + 1))
        g[:, :F] = gW / N + l2 * W
        g[:, F] = gb / N
        return f, g.ravel(order="F")

    w0 = np.zeros((rows, F + 1), order="F").ravel(order="F")
    res = optimize.minimize(fun, w0, method="L-BFGS-B", jac=True,
                            options={"maxiter": max_iter, "maxls": 50, "gtol": tol,
                                     "ftol": 64 * np.finfo(float).eps})
    Wf = res.x.reshape((rows, F + 1), order="F")
    return Wf[:, :F].copy(), Wf[:, F].copy(), int(res.nit), res


def fit_logistic_lbfgs(X, y, *, C: float = 1.0, max_iter: int = 100, tol: float = 1e-4, multi_class: str = "auto",
                       device=None) -> LinearModel:
    """Fit like sklearn ``LogisticRegression(C, max_iter, tol, solver='lbfgs')`` and return a LinearModel.

    ``device``: a torch device (GPU kernel path) or None (numpy float64 path).
    """
    X = np.asarray(X, dtype=np.float64)
    y = np.asarray(y)
    if not np.isfinite(X).all():
        raise ValueError("Input X contains NaN or infinity.")
    classes = np.unique(y)
    if classes.dtype.kind == "U":
        classes = classes.astype(object)
    yi = np.searchsorted(np.asarray(classes).astype(y.dtype) if classes.dtype == object else classes, y)
    N, F = X.shape
    K = len(classes)
    if K < 2:
        raise ValueError("needs samples of at least 2 classes")

    def grad_for(kind, labels):
        return _gpu_grad(X, labels, kind, device) if device is not None else _numpy_grad(X, labels, kind)

    meta = {"solver": "lbfgs", "C": C, "multi_class": multi_class}
    if K == 2:
        W, b, nit, _ = _minimize(grad_for(Kind.BINARY, yi), 1, F, N, C, max_iter, tol)
        meta["n_iter_"] = [nit]
        return LinearModel(W, b, classes, Kind.BINARY, meta)
    if multi_class == "ovr":
        Ws, bs, its = [], [], []
        for k in range(K):
            W, b, nit, _ = _minimize(grad_for(Kind.BINARY, (yi == k).astype(np.int64)), 1, F, N, C, max_iter, tol)
            Ws.append(W[0])
            bs.append(b[0])
            its.append(nit)
        meta["n_iter_"] = its
        return LinearModel(np.stack(Ws), np.array(bs), classes, Kind.OVR, meta)
    W, b, nit, _ = _minimize(grad_for(Kind.MULTINOMIAL, yi), K, F, N, C, max_iter, tol)
    meta["n_iter_"] = [nit]
    return LinearModel(W, b, classes, Kind.MULTINOMIAL, meta)
