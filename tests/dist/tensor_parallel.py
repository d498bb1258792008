"""torchrun worker: class-sharded (TP over K) and feature-sharded (split-F) prediction over the
framework's collectives must reproduce the unsharded float64 oracle (LinearModel.predict_max).

Writes TP_OK_<rank> under $OUT when every check passed."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
from mlapi_amd.models.linear import Kind, LinearModel  # noqa: E402
from mlapi_amd.parallel.comm import init_distributed, shutdown  # noqa: E402
from mlapi_amd.parallel.tensor_parallel import ClassShardedLinear, FeatureShardedLinear  # noqa: E402

info = init_distributed(use_gpu=False)
rng = np.random.default_rng(7)  # same stream on every rank: identical model and data
B, F = 67, 37
for K, kind in ((13, Kind.MULTINOMIAL), (11, Kind.OVR), (2, Kind.BINARY), (2, Kind.BINARY_SOFTMAX)):
    m = LinearModel.random(F, K, seed=K, kind=kind)
    X = rng.standard_normal((B, F))
    want_idx, want_p = m.predict_max(X)
    Xt = torch.from_numpy(X)
    if kind in (Kind.MULTINOMIAL, Kind.OVR):
        tp = ClassShardedLinear(m, info)
        assert (tp.k0, tp.k1) == tp.bounds[info.rank]
        idx, p = tp.predict(Xt)
        assert np.array_equal(idx.numpy(), want_idx), (kind, idx, want_idx)
        np.testing.assert_allclose(p.numpy(), want_p, rtol=1e-5)
        # a tie across shard boundaries resolves to the lowest class index (numpy argmax)
        m2 = LinearModel(np.zeros((K, F)), np.zeros(K), np.arange(K), kind)
        idx, p = ClassShardedLinear(m2, info).predict(Xt[:5])
        assert idx.tolist() == [0] * 5, idx
        np.testing.assert_allclose(p.numpy(), 1.0 / K, rtol=1e-6)
    fs = FeatureShardedLinear(m, info)
    idx, p = fs.predict(Xt[:, fs.f0:fs.f1])
    assert np.array_equal(idx.numpy(), want_idx), (kind, idx, want_idx)
    np.testing.assert_allclose(p.numpy(), want_p, rtol=1e-5)
    if info.world > 1:
        try:
            fs.predict(Xt)  # full X on a feature-sharded rank is a usage error
        except ValueError:
            pass
        else:
            raise AssertionError("FeatureShardedLinear must reject the full feature matrix")
try:
    ClassShardedLinear(LinearModel.random(F, 2, seed=1), info)
except ValueError:
    pass
else:
    raise AssertionError("binary models cannot be class-sharded")
open(os.path.join(os.environ["OUT"], f"TP_OK_{info.rank}"), "w").write(str(info.world))
shutdown(info)
