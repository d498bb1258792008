"""T3 for the sharded-model kernels (csrc/kernels/shard.hip + gemm_softmax MODE 4) on one GPU.

The N ranks of a class- or feature-sharded model are emulated in one process: each shard runs
its own native GEMM, the all-gather / all-reduce is a torch.stack / sum on the device, and the
native merge / epilogue kernel must reproduce the unsharded float64 oracle (LinearModel)."""
import numpy as np
import pytest
import torch

from mlapi_amd.models.linear import Kind, LinearModel
from mlapi_amd.parallel.comm import DistInfo
from mlapi_amd.parallel.tensor_parallel import ClassShardedLinear, FeatureShardedLinear

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


def _bf16_exact(m: LinearModel, X: np.ndarray):
    """Round W and X to bf16 so the float64 oracle sees the kernel's operands."""
    r = lambda a: torch.from_numpy(a).to(torch.bfloat16).double().numpy()
    return LinearModel(r(m.W), m.b, m.classes, m.kind), r(X)


def _clear_rows(m: LinearModel, X: np.ndarray) -> np.ndarray:
    z = m.decision_function(X)
    if z.ndim == 1:
        return np.abs(z) > 1e-3
    top2 = np.sort(z, axis=1)[:, -2:]
    return top2[:, 1] - top2[:, 0] > 1e-3


@pytest.mark.parametrize("world", [1, 3, 8])
@pytest.mark.parametrize("B,F,K", [(1024, 256, 1000), (77, 64, 37), (5000, 128, 200), (20000, 256, 1000)])
@pytest.mark.parametrize("kind", [Kind.MULTINOMIAL, Kind.OVR])
def test_class_sharded_merge(world, B, F, K, kind):
    m, X = _bf16_exact(LinearModel.random(F, K, seed=K + world, kind=kind), np.random.default_rng(3).standard_normal((B, F)))
    shards = [ClassShardedLinear(m, DistInfo(rank=r, world=world, device=DEV), device=DEV) for r in range(world)]
    Xd = torch.from_numpy(X).to(DEV)
    parts = torch.stack([s.local_rowstate(Xd) for s in shards])  # the all-gather
    idx, p = shards[0].merge(parts)
    torch.cuda.synchronize()
    want_idx, want_p = m.predict_max(X)
    clear = _clear_rows(m, X)
    assert np.array_equal(idx.cpu().numpy()[clear], want_idx[clear])
    np.testing.assert_allclose(p.cpu().numpy(), want_p, rtol=2e-4, atol=2e-5)


def test_class_sharded_ties_resolve_to_lowest_class():
    K, F, world = 130, 32, 4
    W = np.zeros((K, F))
    b = np.zeros(K)
    b[[5, 77, 129]] = 1.0  # tie across three shards
    m = LinearModel(W, b, np.arange(K), Kind.MULTINOMIAL)
    shards = [ClassShardedLinear(m, DistInfo(rank=r, world=world, device=DEV), device=DEV) for r in range(world)]
    Xd = torch.ones(256, F, device=DEV)
    idx, p = shards[0].merge(torch.stack([s.local_rowstate(Xd) for s in shards]))
    assert (idx == 5).all()
    torch.testing.assert_close(p.double().cpu(), torch.full((256,), float(torch.softmax(torch.tensor(b), 0).max()),
                                                             dtype=torch.float64), rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("world,F", [(1, 512), (2, 512), (5, 512), (2, 1500)])  # 1500/2: two pieces per rank
@pytest.mark.parametrize("K,kind", [(1000, Kind.MULTINOMIAL), (19, Kind.OVR), (1, Kind.BINARY),
                                    (1, Kind.BINARY_SOFTMAX)])
def test_feature_sharded_epilogue(world, F, K, kind):
    B = 700
    ncls = 2 if K == 1 else K
    m, X = _bf16_exact(LinearModel.random(F, ncls, seed=world, kind=kind), np.random.default_rng(4).standard_normal((B, F)))
    shards = [FeatureShardedLinear(m, DistInfo(rank=r, world=world, device=DEV), device=DEV) for r in range(world)]
    Xd = torch.from_numpy(X).to(DEV)
    Z = sum(s.local_logits(Xd[:, s.f0:s.f1]) for s in shards)  # the all-reduce
    idx, p = shards[0].finish(Z)
    torch.cuda.synchronize()
    want_idx, want_p = m.predict_max(X)
    clear = _clear_rows(m, X)
    assert np.array_equal(idx.cpu().numpy()[clear], want_idx[clear])
    np.testing.assert_allclose(p.cpu().numpy(), want_p, rtol=2e-4, atol=2e-5)
