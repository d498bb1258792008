"""Checkpoint formats: the reference's sklearn pickle (restricted) and the native safetensors format."""
from mlapi_amd.ckpt.sklearn_pickle import (PickledEstimator, SafeUnpickler, UnsafeCheckpointError,
                                          export_sklearn_pickle, load_sklearn_pickle, safe_loads)
from mlapi_amd.ckpt.native import TrainState, load_model, load_native, save_native

__all__ = ["PickledEstimator", "SafeUnpickler", "UnsafeCheckpointError", "export_sklearn_pickle",
           "load_sklearn_pickle", "safe_loads", "TrainState", "load_model", "load_native", "save_native"]
