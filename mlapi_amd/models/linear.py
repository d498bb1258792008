"""Linear-model IR and the float64 CPU oracle (sklearn predict semantics).

The reference serves ``loaded_model.predict(data_in)`` and ``predict_proba(data_in).max()``
(`main.py:21-22`). Both reduce to ``z = X @ coef_.T + intercept_`` followed by an epilogue whose
form depends on the estimator (all verified against sklearn 1.7.2):

* ``BINARY``          (coef_ 1xF, OvR/auto):      label = classes_[z > 0], p_max = sigmoid(|z|)
* ``BINARY_SOFTMAX``  (coef_ 1xF, multinomial):   softmax([-z, z]) -> p_max = sigmoid(2|z|)
* ``MULTINOMIAL``     (K > 2, lbfgs/auto):        label = classes_[argmax z] (first max wins),
                                                   p_max = 1 / sum_k exp(z_k - z_max)
* ``OVR``             (K > 2, 'ovr'/liblinear):   p_k = sigmoid(z_k) / sum_j sigmoid(z_j)

The same enum values are shared with the HIP kernels (``csrc/include/mlapi/kinds.h``).
This module is the numerical oracle that every kernel test compares against.
"""
from __future__ import annotations

import enum
import json
from dataclasses import dataclass, field
from typing import Any, Dict, Optional, Sequence, Tuple

import numpy as np

__all__ = ["Kind", "LinearModel"]


class Kind(enum.IntEnum):
    BINARY = 0
    BINARY_SOFTMAX = 1
    MULTINOMIAL = 2
    OVR = 3


def _is_ovr(multi_class: Optional[str], solver: Optional[str], n_classes: int) -> bool:
    # sklearn 1.7 LogisticRegression.predict_proba; 0.24 behaves identically for these values.
    mc = multi_class if multi_class is not None else "auto"
    if mc in ("ovr", "warn"):
        return True
    if mc in ("auto", "deprecated"):
        return n_classes <= 2 or solver == "liblinear"
    return False  # 'multinomial'


@dataclass
class LinearModel:
    """A fitted linear classifier: ``W`` (K x F float64), ``b`` (K), ``classes`` (K or 2)."""

    W: np.ndarray
    b: np.ndarray
    classes: np.ndarray
    kind: Kind
    meta: Dict[str, Any] = field(default_factory=dict)

    def __post_init__(self) -> None:
        self.W = np.ascontiguousarray(np.asarray(self.W, dtype=np.float64))
        if self.W.ndim != 2:
            raise ValueError("W must be 2-D (K x F)")
        self.b = np.ascontiguousarray(np.asarray(self.b, dtype=np.float64).reshape(-1))
        if self.b.shape[0] != self.W.shape[0]:
            raise ValueError(f"intercept has {self.b.shape[0]} entries, W has {self.W.shape[0]} rows")
        self.classes = np.asarray(self.classes)
        self.kind = Kind(self.kind)
        binary = self.kind in (Kind.BINARY, Kind.BINARY_SOFTMAX)
        if binary and (self.W.shape[0] != 1 or len(self.classes) != 2):
            raise ValueError("binary model needs W of shape 1xF and 2 classes")
        if not binary and self.W.shape[0] != len(self.classes):
            raise ValueError("multiclass model needs one W row per class")

    # ---------------------------------------------------------------- shape helpers
    @property
    def n_features(self) -> int:
        return int(self.W.shape[1])

    @property
    def n_outputs(self) -> int:
        """Rows of W (1 for binary)."""
        return int(self.W.shape[0])

    @property
    def n_classes(self) -> int:
        return int(len(self.classes))

    # ---------------------------------------------------------------- construction
    @classmethod
    def from_sklearn_state(cls, state: Dict[str, Any], estimator: str = "LogisticRegression") -> "LinearModel":
        try:
            coef = np.asarray(state["coef_"], dtype=np.float64)
            intercept = np.asarray(state.get("intercept_", np.zeros(coef.shape[0])), dtype=np.float64)
            classes = np.asarray(state["classes_"])
        except KeyError as e:
            raise ValueError(f"checkpoint is not a fitted estimator (missing {e.args[0]})") from None
        if coef.ndim == 1:
            coef = coef[None, :]
        intercept = np.broadcast_to(intercept.reshape(-1), (coef.shape[0],)).copy()
        k = len(classes)
        if estimator == "SGDClassifier":
            if state.get("loss") not in ("log", "log_loss"):
                raise ValueError("only SGDClassifier(loss='log_loss') has predict_proba")
            ovr = True
        else:
            ovr = _is_ovr(state.get("multi_class"), state.get("solver"), k)
        if coef.shape[0] == 1:
            if k != 2:
                raise ValueError("1-row coef_ requires exactly 2 classes")
            kind = Kind.BINARY if ovr else Kind.BINARY_SOFTMAX
        else:
            kind = Kind.OVR if ovr else Kind.MULTINOMIAL
        meta = {key: state[key] for key in ("solver", "multi_class", "C", "_sklearn_version", "n_iter_")
                if key in state}
        meta["estimator"] = estimator
        return cls(coef, intercept, classes, kind, meta)

    def to_sklearn_state(self) -> Dict[str, Any]:
        return {
            "n_features_in_": self.n_features,
            "classes_": np.array(list(self.classes), dtype=self.classes.dtype),
            "n_iter_": np.asarray(self.meta.get("n_iter_", np.array([0])), dtype=np.int32).reshape(-1),
            "coef_": self.W.copy(),
            "intercept_": self.b.copy(),
        }

    def sklearn_multi_class(self) -> str:
        return "ovr" if self.kind in (Kind.BINARY, Kind.OVR) and self.n_outputs > 1 else (
            "multinomial" if self.kind == Kind.BINARY_SOFTMAX else "auto")

    # ---------------------------------------------------------------- oracle math (float64)
    def decision_function(self, X) -> np.ndarray:
        X = self._check(X)
        z = X @ self.W.T + self.b
        return z[:, 0] if self.n_outputs == 1 else z

    def predict_proba(self, X) -> np.ndarray:
        z = self.decision_function(X)
        with np.errstate(over="ignore", invalid="ignore"):
            if self.kind == Kind.BINARY:
                p1 = 1.0 / (1.0 + np.exp(-z))
                return np.stack([1.0 - p1, p1], axis=1)
            if self.kind == Kind.BINARY_SOFTMAX:
                z = np.stack([-z, z], axis=1)
            if self.kind in (Kind.BINARY_SOFTMAX, Kind.MULTINOMIAL):
                z = z - z.max(axis=1, keepdims=True)
                e = np.exp(z)
                return e / e.sum(axis=1, keepdims=True)
            s = 1.0 / (1.0 + np.exp(-z))  # OVR
            return s / s.sum(axis=1, keepdims=True)

    def predict_index(self, X) -> np.ndarray:
        z = self.decision_function(X)
        if self.n_outputs == 1:
            return (z > 0).astype(np.int64)
        return np.argmax(z, axis=1)

    def predict(self, X) -> np.ndarray:
        return self.classes[self.predict_index(X)]

    def predict_max(self, X) -> Tuple[np.ndarray, np.ndarray]:
        """(label index, max class probability) per row — what `/predict` returns."""
        return self.predict_index(X), self.predict_proba(X).max(axis=1)

    def score(self, X, y) -> float:
        return float(np.mean(self.predict(X) == np.asarray(y)))

    @staticmethod
    def _check(X) -> np.ndarray:
        """sklearn ``check_array``: float64, 2-D, finite (NaN/inf -> ValueError -> HTTP 500)."""
        X = np.asarray(X, dtype=np.float64)
        if X.ndim == 1:
            X = X[None, :]
        if not np.isfinite(X).all():
            raise ValueError("Input X contains NaN or infinity.")
        return X

    # ---------------------------------------------------------------- label rendering
    def label_json(self) -> list:
        """JSON encoding of each class label, as the reference's response would render it.

        str labels -> JSON strings (byte-identical to FastAPI's json.dumps). Integer labels made
        the reference return HTTP 500 (numpy.int64 is not JSON-encodable); we
        intentionally render them as JSON numbers instead.
        """
        out = []
        for c in self.classes.tolist():
            if isinstance(c, bool):
                out.append("true" if c else "false")
            elif isinstance(c, (int, float, str)):
                out.append(json.dumps(c, ensure_ascii=False, allow_nan=False))
            else:
                out.append(json.dumps(str(c), ensure_ascii=False))
        return out

    def label_python(self, idx: int):
        c = self.classes[int(idx)]
        return c.item() if hasattr(c, "item") else c

    # ---------------------------------------------------------------- misc
    @classmethod
    def random(cls, n_features: int, n_classes: int, *, seed: int = 0, kind: Optional[Kind] = None,
               scale: float = 1.0, labels: Optional[Sequence] = None) -> "LinearModel":
        """Random-init model of a given architecture (synthetic benchmarks / tests)."""
        rng = np.random.default_rng(seed)
        k_rows = 1 if n_classes == 2 else n_classes
        if kind is None:
            kind = Kind.BINARY if n_classes == 2 else Kind.MULTINOMIAL
        W = rng.standard_normal((k_rows, n_features)) * scale / np.sqrt(n_features)
        b = rng.standard_normal(k_rows) * 0.1
        classes = np.asarray(labels) if labels is not None else np.arange(n_classes)
        return cls(W, b, classes, kind)
