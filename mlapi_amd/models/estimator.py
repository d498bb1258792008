"""sklearn-compatible ``LogisticRegression`` estimator running on the framework's kernels.

Drop-in for the reference notebook (`Logistic Regression.ipynb:33-42`)::

    from mlapi_amd.models import LogisticRegression
    clf = LogisticRegression().fit(X_train, y_train)      # L-BFGS, same objective as sklearn
    clf.score(X_test, y_test)                             # 0.9666666666666667 on the Iris split
    clf.save("LRClassifier.pkl")                          # the reference's checkpoint format

Fitting evaluates the loss/gradient with the fp64 ``train_small_grad`` HIP kernel when a GPU is
selected (``device='cuda'`` / ``'auto'`` with a GPU visible) and with float64 numpy otherwise.
Prediction uses the fused ``linear_small`` (fp64) kernel on the GPU, or the float64 oracle.
``solver='sgd'`` trains with the mini-batch SGD kernels instead: the fused binary step for two
classes, the fused MFMA softmax / one-vs-rest gradient kernel (G and dW = G^T X in one kernel, no
vendor GEMM) for more.
"""
from __future__ import annotations

from typing import Optional

import numpy as np

from mlapi_amd.models.linear import Kind, LinearModel


class NotFittedError(ValueError, AttributeError):
    pass


class LogisticRegression:
    def __init__(self, C: float = 1.0, max_iter: int = 100, tol: float = 1e-4, multi_class: str = "auto",
                 solver: str = "lbfgs", device: str = "auto", lr: float = 0.5, batch_size: int = 4096,
                 epochs: int = 20, random_state: Optional[int] = 0):
        self.C, self.max_iter, self.tol, self.multi_class = C, max_iter, tol, multi_class
        self.solver, self.device = solver, device
        self.lr, self.batch_size, self.epochs, self.random_state = lr, batch_size, epochs, random_state
        self.model_: Optional[LinearModel] = None

    # ------------------------------------------------------------------ sklearn-style attributes
    def _m(self) -> LinearModel:
        if self.model_ is None:
            raise NotFittedError("This LogisticRegression instance is not fitted yet.")
        return self.model_

    @property
    def coef_(self) -> np.ndarray:
        return self._m().W

    @property
    def intercept_(self) -> np.ndarray:
        return self._m().b

    @property
    def classes_(self) -> np.ndarray:
        return self._m().classes

    @property
    def n_iter_(self) -> np.ndarray:
        return np.asarray(self._m().meta.get("n_iter_", [0]), dtype=np.int32)

    @property
    def n_features_in_(self) -> int:
        return self._m().n_features

    # ------------------------------------------------------------------ device selection
    def _torch_device(self):
        d = str(self.device).lower()
        if d == "cpu":
            return None
        try:
            import torch

            from mlapi_amd._native import available

            if not (torch.cuda.is_available() and available()):
                if d != "auto":
                    raise RuntimeError(f"device={self.device!r} requested but no GPU / native extension")
                return None
            return torch.device("cuda", 0) if d in ("auto", "cuda", "gpu") else torch.device(d)
        except ImportError:  # pragma: no cover
            return None

    # ------------------------------------------------------------------ fit
    def fit(self, X, y) -> "LogisticRegression":
        dev = self._torch_device()
        if self.solver == "lbfgs":
            from mlapi_amd.train.lbfgs import fit_logistic_lbfgs

            self.model_ = fit_logistic_lbfgs(X, y, C=self.C, max_iter=self.max_iter, tol=self.tol,
                                             multi_class=self.multi_class, device=dev)
        elif self.solver == "sgd":
            self.model_ = self._fit_sgd(X, y, dev)
        else:
            raise ValueError(f"unknown solver {self.solver!r} (lbfgs | sgd)")
        return self

    def _fit_sgd(self, X, y, dev) -> LinearModel:
        import torch

        from mlapi_amd.train.sgd import BinarySGDTrainer

        X = np.asarray(X, dtype=np.float64)
        y = np.asarray(y)
        classes = np.unique(y)
        if len(classes) < 2:
            raise ValueError("need at least 2 classes")
        n, F = X.shape
        if len(classes) > 2:
            return self._fit_sgd_multiclass(X, y, classes, dev)
        yb = (y == classes[1]).astype(np.float32)
        Xt = torch.as_tensor(X, dtype=torch.float32, device=dev)
        yt = torch.as_tensor(yb, device=dev)
        tr = BinarySGDTrainer(F, lr=self.lr, l2=1.0 / (self.C * n), momentum=0.9, device=dev)
        rng = np.random.default_rng(self.random_state)
        for _ in range(self.epochs):
            perm = torch.as_tensor(rng.permutation(n), device=dev)
            for s in range(0, n, self.batch_size):
                idx = perm[s:s + self.batch_size]
                tr.step(Xt[idx].contiguous(), yt[idx].contiguous())
        m = tr.to_model(classes=classes)
        m.meta["n_iter_"] = [tr.steps]
        return m

    def _fit_sgd_multiclass(self, X: np.ndarray, y: np.ndarray, classes: np.ndarray, dev) -> LinearModel:
        import torch

        from mlapi_amd.train.softmax_sgd import SoftmaxSGDTrainer

        n, F = X.shape
        yi = torch.as_tensor(np.searchsorted(classes, y).astype(np.int32), device=dev)
        kind = Kind.OVR if self.multi_class == "ovr" else Kind.MULTINOMIAL
        # the trainer zero-pads F to its kernel width; padded weights get zero gradients and stay 0
        tr = SoftmaxSGDTrainer(F, len(classes), kind=kind, lr=self.lr, l2=1.0 / (self.C * n), momentum=0.9,
                               device=dev)
        Xa = tr.prepare(torch.as_tensor(np.asarray(X, dtype=np.float32), device=dev))
        rng = np.random.default_rng(self.random_state)
        for _ in range(self.epochs):
            perm = torch.as_tensor(rng.permutation(n), device=dev)
            for s in range(0, n, self.batch_size):
                idx = perm[s:s + self.batch_size]
                tr.step(Xa[idx].contiguous(), yi[idx].contiguous())
        m = tr.to_model(classes=classes)
        m.meta.update(solver="sgd", n_iter_=[tr.steps])
        return m

    # ------------------------------------------------------------------ predict
    def decision_function(self, X) -> np.ndarray:
        return self._m().decision_function(X)

    def predict_proba(self, X) -> np.ndarray:
        return self._m().predict_proba(X)

    def predict_max(self, X):
        """(label index, max probability) per row — the /predict computation, on the GPU if selected."""
        m = self._m()
        dev = self._torch_device()
        X = LinearModel._check(X)
        if dev is None or m.n_features > 32 or m.n_outputs > 16:
            return m.predict_max(X)
        import torch

        from mlapi_amd.ops.linear import linear_small

        idx, p = linear_small(torch.as_tensor(X, device=dev), torch.as_tensor(m.W, device=dev),
                              torch.as_tensor(m.b, device=dev), int(m.kind))
        return idx.cpu().numpy().astype(np.int64), p.cpu().numpy()

    def predict(self, X) -> np.ndarray:
        return self._m().classes[self.predict_max(X)[0]]

    def score(self, X, y) -> float:
        return float(np.mean(self.predict(X) == np.asarray(y)))

    # ------------------------------------------------------------------ persistence
    def save(self, path: str, format: str = "sklearn") -> None:
        """'sklearn': the reference's pickle format (LRClassifier.pkl); 'native': safetensors."""
        if format == "sklearn":
            from mlapi_amd.ckpt.sklearn_pickle import export_sklearn_pickle

            export_sklearn_pickle(self._m(), path, hparams={"C": self.C, "max_iter": self.max_iter, "tol": self.tol})
        elif format == "native":
            from mlapi_amd.ckpt.native import save_native

            save_native(path, self._m())
        else:
            raise ValueError(format)

    @classmethod
    def load(cls, path: str, **kw) -> "LogisticRegression":
        from mlapi_amd.ckpt.native import load_model

        est = cls(**kw)
        est.model_ = load_model(path)
        return est

    def get_params(self, deep: bool = True) -> dict:
        return {k: getattr(self, k) for k in ("C", "max_iter", "tol", "multi_class", "solver", "device", "lr",
                                              "batch_size", "epochs", "random_state")}

    def __repr__(self) -> str:
        return f"LogisticRegression(solver={self.solver!r}, C={self.C}, device={self.device!r})"


__all__ = ["LogisticRegression", "NotFittedError", "Kind"]
