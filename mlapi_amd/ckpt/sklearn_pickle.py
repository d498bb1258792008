"""Restricted loader / exporter for the reference's checkpoint format.

The reference writes its model with ``pickle.dump(classifier, open('LRClassifier.pkl','wb'))``
(`Logistic Regression.ipynb:37`) and reads it back with an unrestricted ``pickle.load`` on every
request (`main.py:19`). An unrestricted unpickle of an arbitrary file is arbitrary code execution,
so this module implements the same file format with an allow-list: only the globals that a fitted
``sklearn.linear_model.LogisticRegression`` pickle references are resolvable:

* ``sklearn.linear_model._logistic.LogisticRegression`` (sklearn >= 0.22) and the older
  ``sklearn.linear_model.logistic.LogisticRegression`` -> :class:`PickledEstimator` (a plain
  state holder: sklearn itself is never imported, so the serving path does not need it);
* ``numpy.core.multiarray._reconstruct`` / ``numpy._core.multiarray._reconstruct`` (numpy 1.x and
  2.x spellings), ``numpy.ndarray``, ``numpy.dtype`` and ``numpy[._]core.multiarray.scalar``;
* ``copyreg._reconstructor`` + ``builtins.object`` (protocol 0/1 pickles) for allow-listed classes.

Anything else raises :class:`UnsafeCheckpointError`.

The exporter writes the same format back (``export_sklearn_pickle``) without importing sklearn,
so a model trained by :mod:`mlapi_amd.train` can be served by the *unmodified* reference app.
"""
from __future__ import annotations

import copyreg
import io
import os
import pickle
from typing import Any, BinaryIO, Dict, Union

import numpy as np

__all__ = [
    "UnsafeCheckpointError",
    "PickledEstimator",
    "SafeUnpickler",
    "safe_loads",
    "load_sklearn_pickle",
    "export_sklearn_pickle",
    "ESTIMATOR_GLOBALS",
]


class UnsafeCheckpointError(pickle.UnpicklingError):
    """A checkpoint referenced a global outside the allow-list (or is not an estimator)."""


# (module, qualname) of every estimator class we accept -> canonical estimator name.
ESTIMATOR_GLOBALS: Dict[tuple, str] = {
    ("sklearn.linear_model._logistic", "LogisticRegression"): "LogisticRegression",
    ("sklearn.linear_model.logistic", "LogisticRegression"): "LogisticRegression",
    # SGDClassifier(loss='log_loss'/'log') is also a linear logistic model; served identically.
    ("sklearn.linear_model._stochastic_gradient", "SGDClassifier"): "SGDClassifier",
    ("sklearn.linear_model.stochastic_gradient", "SGDClassifier"): "SGDClassifier",
}


class PickledEstimator:
    """State holder standing in for a pickled sklearn estimator.

    ``pickle`` creates it with ``cls.__new__`` (NEWOBJ) and fills it through ``__setstate__``
    (BUILD) with the estimator's ``__getstate__`` dict, exactly like the real class would be.
    """

    estimator_name = "LogisticRegression"

    def __setstate__(self, state: Dict[str, Any]) -> None:
        if not isinstance(state, dict):
            raise UnsafeCheckpointError("estimator state is not a dict")
        self.__dict__.update(state)

    def __repr__(self) -> str:  # pragma: no cover - debugging aid
        keys = ",".join(sorted(self.__dict__))
        return f"PickledEstimator<{self.estimator_name}>({keys})"


def _make_estimator_class(name: str) -> type:
    return type(f"Pickled{name}", (PickledEstimator,), {"estimator_name": name})


_ESTIMATOR_CLASSES = {n: _make_estimator_class(n) for n in set(ESTIMATOR_GLOBALS.values())}


def _np_reconstruct():
    try:
        from numpy._core.multiarray import _reconstruct  # numpy >= 2
    except ImportError:  # pragma: no cover - numpy 1.x
        from numpy.core.multiarray import _reconstruct
    return _reconstruct


def _np_scalar():
    try:
        from numpy._core.multiarray import scalar  # numpy >= 2
    except ImportError:  # pragma: no cover
        from numpy.core.multiarray import scalar
    return scalar


def _safe_reconstructor(cls, base, state):
    """``copyreg._reconstructor`` restricted to allow-listed estimator classes."""
    if not (isinstance(cls, type) and issubclass(cls, PickledEstimator)) or base is not object:
        raise UnsafeCheckpointError("copyreg._reconstructor on a non allow-listed class")
    return copyreg._reconstructor(cls, base, state)


def _safe_codecs_encode(obj, encoding="utf-8"):
    """Protocol-2 pickles store numpy array bytes as ``_codecs.encode(str, 'latin1')``."""
    if not isinstance(obj, str) or encoding not in ("latin1", "latin-1", "utf-8", "utf8"):
        raise UnsafeCheckpointError("_codecs.encode with unexpected arguments")
    return obj.encode(encoding)


class _InertLoss:
    """Stand-in for sklearn's Cython loss objects inside SGDClassifier pickles (inert data)."""

    def __init__(self, *args, **kwargs):
        self.args = args

    def __setstate__(self, state):
        pass


def _safe_frombuffer(buf, dtype, shape, order):
    dtype = np.dtype(dtype)
    if dtype.hasobject:
        raise UnsafeCheckpointError("object arrays cannot come from a raw buffer")
    arr = np.frombuffer(buf, dtype=dtype)
    return arr.reshape(shape, order=order).copy()


class SafeUnpickler(pickle.Unpickler):
    """``pickle.Unpickler`` whose ``find_class`` only resolves the allow-list above."""

    def find_class(self, module: str, name: str):  # noqa: D401 - pickle API
        key = (module, name)
        if key in ESTIMATOR_GLOBALS:
            return _ESTIMATOR_CLASSES[ESTIMATOR_GLOBALS[key]]
        if module in ("numpy.core.multiarray", "numpy._core.multiarray"):
            if name == "_reconstruct":
                return _np_reconstruct()
            if name == "scalar":
                return _np_scalar()
        if (module in ("_loss", "sklearn._loss._loss", "sklearn.linear_model._sgd_fast",
                       "sklearn.linear_model.sgd_fast") and name.isidentifier()):
            return _InertLoss  # SGDClassifier's Cython loss object: never used for predict
        if module in ("numpy.core.numeric", "numpy._core.numeric") and name == "_frombuffer":
            return _safe_frombuffer  # pickle protocol 5 arrays
        if module == "numpy" and name == "ndarray":
            return np.ndarray
        if module == "numpy" and name == "dtype":
            return np.dtype
        if module in ("copyreg", "copy_reg") and name == "_reconstructor":  # copy_reg: py2 name (proto 0/1)
            return _safe_reconstructor
        if module in ("builtins", "__builtin__") and name == "object":
            return object
        if module == "_codecs" and name == "encode":
            return _safe_codecs_encode
        raise UnsafeCheckpointError(f"global '{module}.{name}' is not allowed in a checkpoint")


def safe_loads(data: bytes) -> Any:
    return SafeUnpickler(io.BytesIO(data)).load()


def load_sklearn_pickle(src: Union[str, os.PathLike, bytes, BinaryIO]):
    """Load a pickled sklearn logistic model and return a :class:`mlapi_amd.models.LinearModel`."""
    from mlapi_amd.models.linear import LinearModel

    if isinstance(src, (bytes, bytearray)):
        obj = safe_loads(bytes(src))
    elif hasattr(src, "read"):
        obj = SafeUnpickler(src).load()
    else:
        with open(src, "rb") as f:
            obj = SafeUnpickler(f).load()
    if not isinstance(obj, PickledEstimator):
        raise UnsafeCheckpointError(f"checkpoint does not hold an estimator (got {type(obj).__name__})")
    return LinearModel.from_sklearn_state(obj.__dict__, estimator=obj.estimator_name)


# --------------------------------------------------------------------------------------------
# Export: write a pickle that unpickles into sklearn's LogisticRegression, without sklearn.
# --------------------------------------------------------------------------------------------

_DEFAULT_HPARAMS = {  # sklearn 0.24.1 LogisticRegression() defaults (requirements.txt:11)
    "penalty": "l2",
    "dual": False,
    "tol": 1e-4,
    "C": 1.0,
    "fit_intercept": True,
    "intercept_scaling": 1,
    "class_weight": None,
    "random_state": None,
    "solver": "lbfgs",
    "max_iter": 100,
    "multi_class": "auto",
    "verbose": 0,
    "warm_start": False,
    "n_jobs": None,
    "l1_ratio": None,
}


def export_sklearn_pickle(model, dst: Union[str, os.PathLike, None] = None, *,
                          numpy_compat: str = "1.x", sklearn_version: str = "0.24.1",
                          hparams: Dict[str, Any] | None = None) -> bytes:
    """Serialize ``model`` (a LinearModel) as a ``LogisticRegression`` pickle.

    ``numpy_compat='1.x'`` spells the array reconstructor ``numpy.core.multiarray`` so that the
    reference-era stack (numpy 1.20, `requirements.txt:5`) can read it; numpy 2 still resolves
    that spelling. The object is written as ``GLOBAL; EMPTY_TUPLE; NEWOBJ; <state>; BUILD`` which
    is exactly what ``pickle.dump`` of the real estimator produces.
    """
    state = dict(_DEFAULT_HPARAMS)
    if hparams:
        state.update(hparams)
    state.update(model.to_sklearn_state())
    state["_sklearn_version"] = sklearn_version
    if "multi_class" not in (hparams or {}):
        state["multi_class"] = model.sklearn_multi_class()

    inner = pickle.dumps(state, protocol=3)  # protocol 3: raw bytes opcodes (readable by Python >= 3.0)
    assert inner[:2] == b"\x80\x03" and inner[-1:] == b"."
    body = inner[2:-1]
    if numpy_compat == "1.x":
        body = body.replace(b"cnumpy._core.multiarray\n", b"cnumpy.core.multiarray\n")
    out = (b"\x80\x03"
           + b"csklearn.linear_model._logistic\nLogisticRegression\n"
           + b")\x81"  # EMPTY_TUPLE, NEWOBJ
           + body
           + b"b.")  # BUILD, STOP
    if dst is not None:
        tmp = f"{os.fspath(dst)}.tmp.{os.getpid()}"
        with open(tmp, "wb") as f:
            f.write(out)
        os.replace(tmp, dst)  # atomic: a live-reloading server never sees a torn file
    return out
