"""Plain-PyTorch fp32/fp64 reference implementations of every HIP kernel (test oracles)."""
from __future__ import annotations

import torch

from mlapi_amd.models.linear import Kind


def predict_ref(X: torch.Tensor, W: torch.Tensor, b: torch.Tensor, kind: int, dtype=torch.float64):
    X, W, b = X.to(dtype), W.to(dtype), b.to(dtype)
    z = X @ W.T + b
    if kind in (Kind.BINARY, Kind.BINARY_SOFTMAX):
        z = z[:, 0]
        a = z.abs() * (2.0 if kind == Kind.BINARY_SOFTMAX else 1.0)
        return (z > 0).to(torch.int32), torch.sigmoid(a)
    idx = torch.argmax(z, dim=1).to(torch.int32)  # first max (torch.argmax is first-occurrence)
    if kind == Kind.MULTINOMIAL:
        return idx, torch.softmax(z, dim=1).max(dim=1).values
    s = torch.sigmoid(z)
    return idx, (s / s.sum(dim=1, keepdim=True)).max(dim=1).values


def logits_ref(X, W, b, dtype=torch.float32):
    return X.to(dtype) @ W.to(dtype).T + b.to(dtype)


def train_binary_ref(X, y, w, b):
    X = X.to(torch.float64)
    z = X @ w.to(torch.float64) + b.to(torch.float64)
    y = y.to(torch.float64)
    g = torch.sigmoid(z) - y
    loss = (torch.clamp(z, min=0) - z * y + torch.log1p(torch.exp(-z.abs()))).sum()
    correct = ((z > 0) == (y > 0.5)).sum()
    return torch.cat([X.T @ g, g.sum().reshape(1), loss.reshape(1), correct.to(torch.float64).reshape(1)])


def train_small_ref(X, y, W, b, kind: int):
    X, W, b = X.to(torch.float64), W.to(torch.float64), b.to(torch.float64)
    y = y.long()
    z = X @ W.T + b
    K = W.shape[0]
    if kind in (Kind.BINARY, Kind.BINARY_SOFTMAX):
        sc = 2.0 if kind == Kind.BINARY_SOFTMAX else 1.0
        zz = sc * z[:, 0]
        yy = y.to(torch.float64)
        g = (sc * (torch.sigmoid(zz) - yy))[:, None]
        loss = (torch.clamp(zz, min=0) - zz * yy + torch.log1p(torch.exp(-zz.abs()))).sum()
        correct = ((z[:, 0] > 0) == (y == 1)).sum()
    elif kind == Kind.MULTINOMIAL:
        p = torch.softmax(z, dim=1)
        Y = torch.nn.functional.one_hot(y, K).to(torch.float64)
        g = p - Y
        loss = (torch.logsumexp(z, dim=1) - z.gather(1, y[:, None])[:, 0]).sum()
        correct = (torch.argmax(z, dim=1) == y).sum()
    else:
        Y = torch.nn.functional.one_hot(y, K).to(torch.float64)
        g = torch.sigmoid(z) - Y
        loss = (torch.clamp(z, min=0) - z * Y + torch.log1p(torch.exp(-z.abs()))).sum()
        correct = (torch.argmax(z, dim=1) == y).sum()
    return torch.cat([(g.T @ X).reshape(-1), g.sum(0), loss.reshape(1), correct.to(torch.float64).reshape(1)])


def softmax_train_ref(X_aug, y, W_aug, kind: int, dtype=torch.float32):
    """Oracle of ops.linear.softmax_train_grad: (G [B, K], dW_aug [K, F_aug], loss_sum, n_correct).

    Also the CPU path of the multiclass SGD trainer (dtype float32)."""
    X, W = X_aug.to(dtype), W_aug.to(dtype)
    y = y.long()
    z = X @ W.T
    K = W.shape[0]
    Y = torch.nn.functional.one_hot(y, K).to(dtype)
    if kind == Kind.MULTINOMIAL:
        G = torch.softmax(z, dim=1) - Y
        loss = (torch.logsumexp(z, dim=1) - z.gather(1, y[:, None])[:, 0]).sum()
    else:
        G = torch.sigmoid(z) - Y
        loss = (torch.clamp(z, min=0) - z * Y + torch.log1p(torch.exp(-z.abs()))).sum()
    correct = (torch.argmax(z, dim=1) == y).sum().to(dtype)
    return G, G.T @ X, loss, correct
