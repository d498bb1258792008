"""Native checkpoint format (safetensors container) with full training state for resume.

The reference's only checkpoint is a one-shot pickle of the estimator
(`Logistic Regression.ipynb:37`); ``warm_start=False`` means training can never resume. Our native
format stores, in one safetensors file (no code execution on load, mmap-able):

* tensors: ``W`` (K x F f64), ``b`` (K f64), optional optimizer state (``opt.*``) and the RNG
  state (``rng.state`` uint64 words);
* metadata (str -> str JSON): ``kind``, ``classes``, ``step``, ``epoch``, ``data_cursor``,
  ``config`` and free-form ``extra``.

Writes are atomic (tmp + ``os.replace``) so a live-reloading server never reads a torn file.
"""
from __future__ import annotations

import json
import os
from dataclasses import dataclass, field
from typing import Any, Dict, Optional

import numpy as np

from mlapi_amd.models.linear import Kind, LinearModel

FORMAT = "mlapi_amd.linear.v1"

__all__ = ["TrainState", "save_native", "load_native", "load_model", "FORMAT"]


@dataclass
class TrainState:
    step: int = 0
    epoch: int = 0
    data_cursor: int = 0
    opt: Dict[str, np.ndarray] = field(default_factory=dict)
    rng_state: Optional[np.ndarray] = None
    config: Dict[str, Any] = field(default_factory=dict)
    extra: Dict[str, Any] = field(default_factory=dict)


def _classes_to_json(classes: np.ndarray) -> str:
    vals = classes.tolist()
    return json.dumps({"dtype": classes.dtype.str if classes.dtype != object else "object", "values": vals})


def _classes_from_json(s: str) -> np.ndarray:
    d = json.loads(s)
    if d["dtype"] == "object":
        return np.array(d["values"], dtype=object)
    return np.array(d["values"], dtype=np.dtype(d["dtype"]))


def save_native(path: str | os.PathLike, model: LinearModel, state: Optional[TrainState] = None) -> None:
    from safetensors.numpy import save_file

    tensors = {"W": np.ascontiguousarray(model.W), "b": np.ascontiguousarray(model.b)}
    meta = {
        "format": FORMAT,
        "kind": model.kind.name,
        "classes": _classes_to_json(model.classes),
        "meta": json.dumps({k: (v.tolist() if isinstance(v, np.ndarray) else v) for k, v in model.meta.items()}),
    }
    if state is not None:
        for k, v in state.opt.items():
            tensors[f"opt.{k}"] = np.ascontiguousarray(v)
        if state.rng_state is not None:
            tensors["rng.state"] = np.ascontiguousarray(state.rng_state)
        meta.update(step=str(state.step), epoch=str(state.epoch), data_cursor=str(state.data_cursor),
                    config=json.dumps(state.config), extra=json.dumps(state.extra))
    tmp = f"{os.fspath(path)}.tmp.{os.getpid()}"
    save_file(tensors, tmp, metadata=meta)
    os.replace(tmp, path)


def load_native(path: str | os.PathLike):
    """Return ``(LinearModel, TrainState | None)``."""
    from safetensors import safe_open

    with safe_open(os.fspath(path), framework="np") as f:
        meta = f.metadata() or {}
        if meta.get("format") != FORMAT:
            raise ValueError(f"{path}: not a {FORMAT} checkpoint")
        names = list(f.keys())
        tensors = {k: f.get_tensor(k) for k in names}
    model = LinearModel(tensors["W"], tensors["b"], _classes_from_json(meta["classes"]), Kind[meta["kind"]],
                        json.loads(meta.get("meta", "{}")))
    state = None
    if "step" in meta:
        state = TrainState(step=int(meta["step"]), epoch=int(meta["epoch"]), data_cursor=int(meta["data_cursor"]),
                           opt={k[4:]: v for k, v in tensors.items() if k.startswith("opt.")},
                           rng_state=tensors.get("rng.state"), config=json.loads(meta.get("config", "{}")),
                           extra=json.loads(meta.get("extra", "{}")))
    return model, state


def load_model(path: str | os.PathLike) -> LinearModel:
    """Load either format: safetensors (native) or the reference's sklearn pickle."""
    with open(path, "rb") as f:
        head = f.read(9)
    # safetensors: u64 little-endian header length, then the JSON header ('{'); anything else is
    # treated as a pickle (restricted loader).
    if len(head) == 9 and head[8:9] == b"{" and int.from_bytes(head[:8], "little") < (1 << 30):
        return load_native(path)[0]
    from mlapi_amd.ckpt.sklearn_pickle import load_sklearn_pickle

    return load_sklearn_pickle(path)
