"""P2P all-reduce front end on CPU: argument checks and the NativeComm opt-in switch (the kernel
itself runs in tests/test_comm_gpu.py::test_p2p_allreduce_multiprocess)."""
import pytest
import torch

from mlapi_amd.parallel.p2p import P2PAllReduce, from_env


def test_p2p_needs_gpu_device():
    with pytest.raises(ValueError):
        P2PAllReduce(0, 1, torch.device("cpu"))
    with pytest.raises(ValueError):
        P2PAllReduce(0, 1, None)


def test_p2p_from_env_is_opt_in(monkeypatch):
    monkeypatch.delenv("MLAPI_P2P_BYTES", raising=False)
    assert from_env(0, 8, torch.device("cuda", 0)) is None  # default: RCCL for every collective
    monkeypatch.setenv("MLAPI_P2P_BYTES", "1048576")
    assert from_env(0, 1, torch.device("cuda", 0)) is None  # nothing to reduce at world 1
